"""bench.py's record and launcher on the CPU: the compact last stdout line
(the one the driver parses) built from a recorded bench record, and
`--gpus N` starting N ranks by itself."""
import importlib.util
import json
import os
import subprocess
import sys
import textwrap

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
FIXTURE = os.path.join(ROOT, "tests", "golden", "bench_record_r05.json")


def _bench():
    spec = importlib.util.spec_from_file_location("bench_mod", os.path.join(ROOT, "bench.py"))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


def test_final_line_from_recorded_record_is_compact_json():
    """The round-5 builder record (20.5 KB on one line: the line the driver
    lost) becomes a last line <= 8 KB that carries the contract's keys, the
    roofline with both fractions' inputs, cpu_baseline and the quality
    summary."""
    bench = _bench()
    rec = json.load(open(FIXTURE))
    assert len(json.dumps(rec)) > 16000
    rec["roofline"]["frac_vs_guide_peak"] = rec["roofline"]["achieved"] / bench.GUIDE_LDS_GATHER_PEAK
    s = bench.final_line(rec)
    assert "\n" not in s and len(s.encode()) <= 8192
    line = json.loads(s)
    for k in ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "dtype",
              "config", "roofline", "cpu_baseline", "islands", "quality_summary"):
        assert k in line, k
    assert line["value"] == rec["value"]              # the headline keeps full precision
    rf = line["roofline"]
    for k in ("bound", "achieved", "peak", "unit", "frac", "frac_vs_guide_peak", "traffic"):
        assert k in rf, k
    assert 0.2 < rf["frac_vs_guide_peak"] < 0.23
    assert line["cpu_baseline"]["kind"] == "port" and line["cpu_baseline"]["cores"] == 16
    assert line["quality_summary"]["x1000_median"] == rec["quality_summary"]["x1000_median"]


def test_final_line_drops_optional_blocks_to_fit():
    bench = _bench()
    rec = json.load(open(FIXTURE))
    rec["quality_summary"]["padding"] = "x" * 9000
    line = json.loads(bench.final_line(rec))
    assert "quality_summary" not in line and "roofline" in line and "value" in line
    assert len(bench.final_line(rec, limit=600)) <= 1200     # headline + roofline survive


def test_detail_lines_hold_every_leg():
    bench = _bench()
    rec = json.load(open(FIXTURE))
    legs = {json.loads(ln)["bench_detail"] for ln in bench.detail_lines(rec)}
    assert {"quality_x1000", "islands", "search", "other_configs", "cpu_baseline"} <= legs
    assert not legs & set(bench.HEADLINE_KEYS)


STUB = textwrap.dedent("""
    import json, os, sys, time
    r = int(os.environ["RANK"])
    keys = ("RANK", "LOCAL_RANK", "WORLD_SIZE", "LOCAL_WORLD_SIZE", "MASTER_ADDR", "MASTER_PORT")
    with open(os.path.join(sys.argv[1], f"rank{r}.json"), "w") as f:
        json.dump({k: os.environ.get(k) for k in keys}, f)
    mode = sys.argv[2]
    if mode == "fail1" and r == 1:
        sys.exit(3)
    if mode == "hang" and r == 1:
        time.sleep(600)
    if mode == "hang" and r == 0:
        sys.exit(5)
    if r == 0:
        print("rank0 line")
""")


def _stub(tmp_path):
    p = tmp_path / "stub.py"
    p.write_text(STUB)
    return p


def test_launcher_sets_the_rank_environment(tmp_path, capfd):
    bench = _bench()
    stub = _stub(tmp_path)
    rc = bench.launch_ranks(3, [], child=[sys.executable, str(stub), str(tmp_path), "ok"],
                            port=29999)
    assert rc == 0
    envs = [json.load(open(tmp_path / f"rank{r}.json")) for r in range(3)]
    for r, e in enumerate(envs):
        assert e["RANK"] == e["LOCAL_RANK"] == str(r)
        assert e["WORLD_SIZE"] == e["LOCAL_WORLD_SIZE"] == "3"
        assert e["MASTER_ADDR"] == "127.0.0.1" and e["MASTER_PORT"] == "29999"
    assert "rank0 line" in capfd.readouterr().out


def test_launcher_returns_a_failing_ranks_code(tmp_path):
    bench = _bench()
    stub = _stub(tmp_path)
    assert bench.launch_ranks(2, [], child=[sys.executable, str(stub), str(tmp_path),
                                            "fail1"]) == 3


def test_launcher_terminates_the_others_after_a_failure(tmp_path):
    bench = _bench()
    stub = _stub(tmp_path)
    import time
    t0 = time.monotonic()
    rc = bench.launch_ranks(2, [], child=[sys.executable, str(stub), str(tmp_path), "hang"],
                            grace_s=1.0)
    assert rc == 5 and time.monotonic() - t0 < 60


def test_world_size_mismatch_is_refused():
    env = dict(os.environ, WORLD_SIZE="2", RANK="0")
    res = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "4"],
                         env=env, capture_output=True, text=True, timeout=120)
    assert res.returncode != 0 and "WORLD_SIZE=2" in res.stderr


@pytest.mark.timeout(300)
def test_gpus_2_spawns_two_ranks_on_the_cpu_standin():
    """`bench.py --gpus 2` with no launcher: two fresh processes rendezvous
    over gloo, and rank 0's last line says n_gpus = 2."""
    env = {k: v for k, v in os.environ.items()
           if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT")}
    res = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2",
                          "--cpu-standin", "--steps", "3", "--warmup", "1"],
                         env=env, capture_output=True, text=True, timeout=280)
    assert res.returncode == 0, res.stderr[-2000:]
    lines = res.stdout.strip().splitlines()
    line = json.loads(lines[-1])
    assert line["n_gpus"] == 2 and line["config"]["parallelism"] == "islands2"
    assert line["steps"] == 3 and line["value"] > 0
    # only rank 0 prints the record on stdout (gloo's own banner may precede it)
    assert sum(ln.startswith("{") for ln in lines) == 1
