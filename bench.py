#!/usr/bin/env python3
"""Headline benchmark: candidate route evaluations per second.

Workload (BASELINE.json configs[1]): CVRP, 100 customers, 8 vehicles,
uniform capacity, random Euclidean integer durations, on one MI355X.  One
"step" is one pass of the scoring hot path (``vrpms_eval``) over a batch of
C candidate giant tours (uint8, 100 B each) that is already resident in HBM
and larger than the 256 MiB Infinity Cache, so every step streams it from
HBM.  Multi-GPU: every rank scores its own batch (independent islands, no
collective in the data path) -> weak scaling; the driver launches one
process per GPU via torch.distributed.run.

Reported beside the value:
  roofline      the dominant kernel (eval_cvrp_words2, word-interleaved
                tours: the layout the GA / ACO kernels emit) timed with HIP
                events on the stream it runs on.  It is LDS-gather bound, so
                achieved = evals/s x G (G = n + K gathers per eval, SURVEY.md
                §8d) against the measured random ds_read_b64 rate R_gather;
                hbm_roofline = algorithmic HBM bytes (C x (100 B tour + 8 B
                key)) / mean launch time against 8 TB/s.  rows_layout times
                the same batch in the API's row-major layout (eval_cvrp_rows2).
  search        GA / ACO / BF throughput on cfg 2 (the endpoints' algorithms).
  cfg1_main_py  BASELINE cfg 1: main.py's calls through the drop-in.
  cpu_baseline  the C restatement of the spec (oracle/oracle_c.c, OpenMP)
                on a bounded sample of the same workload, rank 0 only.
"""
from __future__ import annotations

import argparse
import collections
import json
import math
import os
import sys
import time
import traceback

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

_T0 = time.perf_counter()


def progress(msg):
    """A progress line on stderr (stdout carries only the JSON line): a long
    run keeps showing it is alive."""
    print(f"[bench {time.perf_counter() - _T0:7.1f} s] {msg}", file=sys.stderr, flush=True)


METRIC = "candidate route evals/sec (1/2/4/8 GPU) + best-cost gap at fixed wall time"
# TD-200 equal-time cells (sa_td_kernel): chains, moves per step, migrated elites, final
# temperature per typical edge (tools/td_quality_scan.py)
TD_SHAPE = (1024, 64, 128, 0.004)
HBM_PEAK_GBS = 8000.0          # MI355X_MICROARCH.md chip table (spec)
# the guide's conflict-free ds_read_b64 rate (MI355X_MICROARCH.md §LDS: 256 B/clk/CU x
# 256 CUs x 2.4 GHz), in 8-byte gathers per second
GUIDE_LDS_GATHER_PEAK = 256 * 256 * 2.4e9 / 8
# the driver keeps a bounded tail of stdout: the LAST line (the one it parses) stays
# under this many bytes; every detailed leg is printed on an earlier stdout line
FINAL_LINE_MAX = 8192
HEADLINE_KEYS = ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step",
                 "higher_is_better", "scaling", "vs_baseline", "dtype", "data", "config")


def parse(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--candidates", type=int, default=16 * 1024 * 1024)
    ap.add_argument("--seed", type=int, default=0)
    ap.add_argument("--cpu-seconds", type=float, default=10.0,
                    help="target CPU work for the cpu_baseline sample")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-other-configs", action="store_true")
    ap.add_argument("--island-epochs", type=int, default=60,
                    help="cfg 4 island-SA leg (all ranks, RCCL elite all-gather); 0 disables")
    ap.add_argument("--island-steps", type=int, default=500,
                    help="SA steps per island epoch (60 x 500 ~ 1.1 s of wall time)")
    ap.add_argument("--quality-seconds", type=float, default=5.0,
                    help="wall time per side for the best-cost gap (0 disables)")
    ap.add_argument("--x1000-quality-seconds", type=float, default=10.0,
                    help="wall time per side for the cfg-4 X-1000 best-cost gaps (seeds 0-2, "
                         "the host leg at 32 and at 64 moves per step, the better kept, seed 0's "
                         "host leg repeated for the run-to-run spread; 0 disables)")
    ap.add_argument("--x1000-seeds", type=int, nargs="+", default=[0, 1, 2])
    ap.add_argument("--x1000-long-seconds", type=float, default=0.0,
                    help="opt-in: one longer X-1000 cell (seed 0) at this wall time per side "
                         "(e.g. 60); the host at the move count that won most of the 10-s "
                         "cells (ties: the smaller), one run; 0 (default) disables -- at 60 s "
                         "it costs ~120 s of the default run's time budget")
    ap.add_argument("--td-quality-seconds", type=float, default=10.0,
                    help="wall time per side for the cfg-3 TD-200 x 24 best-cost gaps: the "
                         "uniform fleet (seed 0) and the reference's normal request -- three "
                         "capacity classes, staggered start times (seeds --het-seeds); 0 disables")
    ap.add_argument("--het-seeds", type=int, nargs="+", default=[0, 1, 2])
    ap.add_argument("--cpu-standin", action="store_true",
                    help="launcher / rendezvous rehearsal without a GPU: each rank times a "
                         "numpy TSP tour-cost pass over gloo and rank 0 prints the final line "
                         "(not a measurement; tests/test_bench_cpu.py)")
    ap.add_argument("--host-repeats", type=int, default=2,
                    help="extra runs of seed 0's better host leg in every equal-time cell "
                         "family (X-1000, TD-200, heterogeneous TD-200): the host's run-to-run "
                         "spread over 1 + this many runs")
    return ap.parse_args(argv)


def launch_ranks(n, argv, child=None, port=None, poll_s=0.2, grace_s=30.0):
    """`bench.py --gpus N` without a launcher: start N fresh child processes,
    one per GPU, with the torch.distributed.run environment (RANK, LOCAL_RANK,
    WORLD_SIZE, LOCAL_WORLD_SIZE, MASTER_ADDR=127.0.0.1, MASTER_PORT), and wait
    for all of them.  The caller has not touched the GPU (nothing here imports
    torch), so no process that initialised HIP is replaced: the children are
    new programs.  Rank 0's stdout is this process's stdout (it prints the
    one JSON line); the other ranks' stdout goes to stderr.  When a rank exits
    non-zero the others get `grace_s` to finish, then are terminated; the
    return value is the first non-zero exit status (0 when every rank
    succeeded).  `child` replaces the command (tests: a stub program)."""
    import socket
    import subprocess
    if port is None:
        with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
            s.bind(("127.0.0.1", 0))
            port = s.getsockname()[1]
    cmd = list(child) if child else [sys.executable, os.path.abspath(__file__)] + list(argv)
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n),
                   LOCAL_WORLD_SIZE=str(n), GROUP_RANK="0", MASTER_ADDR="127.0.0.1",
                   MASTER_PORT=str(port))
        procs.append(subprocess.Popen(cmd, env=env, stdout=None if r == 0 else sys.stderr))
    first_bad, deadline = 0, None
    while True:
        codes = [p.poll() for p in procs]
        for c in codes:
            if c not in (None, 0) and not first_bad:
                first_bad = c
                deadline = time.monotonic() + grace_s
        if all(c is not None for c in codes):
            break
        if deadline is not None and time.monotonic() > deadline:
            for p in procs:
                if p.poll() is None:
                    p.terminate()
            for p in procs:
                try:
                    p.wait(10)
                except subprocess.TimeoutExpired:
                    p.kill()
                    p.wait()
            break
        time.sleep(poll_s)
    if first_bad:
        print(f"[bench] a rank failed (exit {first_bad}); ranks' exit codes: "
              f"{[p.returncode for p in procs]}", file=sys.stderr, flush=True)
    return first_bad


def _sig(x, digits=6):
    """Floats to `digits` significant digits (compact final line)."""
    if isinstance(x, float):
        return float(f"{x:.{digits}g}")
    if isinstance(x, dict):
        return {k: _sig(v, digits) for k, v in x.items()}
    if isinstance(x, list):
        return [_sig(v, digits) for v in x]
    return x


def _pick(d, keys):
    if not isinstance(d, dict):
        return None
    if "error" in d:
        return {"error": str(d["error"])[-200:]}
    return {k: d[k] for k in keys if k in d}


def final_line(out, limit=FINAL_LINE_MAX):
    """The bench's LAST stdout line: the headline keys of the contract, the
    roofline (measured-ceiling frac and the guide-peak frac side by side),
    and compact cpu_baseline / islands / search / other-config /
    quality_summary blocks -- the details are earlier stdout lines
    ({"bench_detail": leg, ...}).  Optional blocks are dropped, least
    important first, until the line fits in `limit` bytes; the headline and
    the roofline are never dropped."""
    line = {k: out[k] for k in HEADLINE_KEYS if k in out}
    rf = out.get("roofline") or {}
    line["roofline"] = _pick(rf, ("bound", "achieved", "peak", "unit", "frac",
                                  "frac_vs_guide_peak", "guide_peak", "traffic", "traffic_unit",
                                  "kernel", "kernel_ms", "G_per_eval", "peak_source"))
    if out.get("hbm_roofline"):
        line["hbm_roofline"] = _pick(out["hbm_roofline"], ("achieved", "peak", "unit", "frac"))
    if "rows_vs_words_identical" in out:
        line["rows_vs_words_identical"] = out["rows_vs_words_identical"]
    cb = out.get("cpu_baseline")
    if cb:
        c = _pick(cb, ("value", "unit", "cores", "kind", "sample", "cpu_model",
                       "parity_on_sample"))
        if isinstance(cb.get("python_port"), dict):
            c["python_port_evals_per_s"] = cb["python_port"].get("value")
        line["cpu_baseline"] = c
    isl = out.get("islands")
    if isl:
        line["islands"] = _pick(isl, ("ranks", "rccl_ranks", "chains_per_gpu", "epochs",
                                      "chain_steps_per_s", "move_evals_per_s", "exchanges",
                                      "exchange_ms_mean", "exchange_share_of_wall", "best",
                                      "exchange_path"))
    optional = []
    se = out.get("search")
    if isinstance(se, dict):
        s = {}
        if "error" in se:
            s["error"] = str(se["error"])[-200:]
        ga = se.get("ga") or {}
        if ga.get("fused"):
            f = ga["fused"]
            s["ga"] = {"child_evals_per_s": f.get("child_evals_per_s"),
                       "us_per_generation": 1e6 / f["generations_per_s"]
                       if f.get("generations_per_s") else None,
                       "frac_vs_measured": f.get("lds_gather_frac_whole_generation"),
                       "speedup_fused": ga.get("speedup_fused")}
        aco = se.get("aco") or {}
        if aco:
            s["aco"] = {"ant_tours_per_s": aco.get("ant_tours_per_s"),
                        "iterations_per_s": aco.get("iterations_per_s"),
                        "roofline": _pick(aco.get("roofline"), ("achieved", "peak", "unit",
                                                                "frac", "frac_vs_guide_peak"))}
        bf = se.get("bf") or {}
        if bf:
            s["bf_evals_per_s"] = {k: v.get("evals_per_s") for k, v in bf.items()
                                   if isinstance(v, dict)}
        optional.append(("search", s))
    oc = out.get("other_configs")
    if isinstance(oc, dict):
        o = {}
        if "error" in oc:
            o["error"] = str(oc["error"])[-200:]
        for k in ("cfg3_tdvrp200_h24", "cfg4_x1000"):
            if isinstance(oc.get(k), dict) and "evals_per_s" in oc[k]:
                o[k] = {"evals_per_s": oc[k]["evals_per_s"],
                        "l2_frac": (oc[k].get("l2_roofline") or {}).get("frac")}
        c5 = oc.get("cfg5_tsp50_x10k")
        if isinstance(c5, dict) and "requests_per_s" in c5:
            o["cfg5_kernel"] = {"requests_per_s": c5["requests_per_s"],
                                "frac": (c5.get("roofline") or {}).get("frac")}
        for k, keys in (("cfg5_http", ("requests_per_s", "ok", "answer_mismatches",
                                       "banner_equal", "error_bytes_equal")),
                        ("cfg5_api", ("requests_per_s", "ok", "duration_mismatches")),
                        ("cfg5_api_one_process", ("requests_per_s", "ok"))):
            if isinstance(oc.get(k), dict):
                o[k] = _pick(oc[k], keys)
        optional.append(("other_configs", o))
    c1 = out.get("cfg1_main_py")
    if isinstance(c1, dict):
        optional.append(("cfg1_main_py", _pick(c1, ("calculate_duration_calls_per_s",))
                         | {"solve_vrp_problem_calls_per_s":
                            (c1.get("solve_vrp_problem") or {}).get("calls_per_s")}))
    if out.get("quality_summary"):
        optional.append(("quality_summary", out["quality_summary"]))
    # most important last, so the drop order below is least important first
    order = ("cfg1_main_py", "other_configs", "search", "quality_summary")
    optional.sort(key=lambda kv: order.index(kv[0]))
    for k, v in optional:
        line[k] = v
    line["detail"] = "earlier stdout lines {\"bench_detail\": <leg>, \"data\": {...}}"
    line = _sig(line)
    line["value"] = out.get("value")          # full precision for the headline number
    s = json.dumps(line, separators=(",", ":"))
    for k, _ in optional:
        if len(s.encode()) <= limit:
            break
        line.pop(k, None)
        s = json.dumps(line, separators=(",", ":"))
    for k in ("hbm_roofline", "islands", "cpu_baseline"):
        if len(s.encode()) <= limit:
            break
        line.pop(k, None)
        s = json.dumps(line, separators=(",", ":"))
    return s


def detail_lines(out):
    """One stdout line per detailed leg (everything final_line shortens)."""
    for k, v in out.items():
        if k in HEADLINE_KEYS:
            continue
        yield json.dumps({"bench_detail": k, "data": v}, separators=(",", ":"))


def make_batch(ctx, C, n, seed, dtype=None):
    """C Philox Fisher-Yates permutations of 1..n (vrpms_random_tours, the
    library's start-tour kernel; SURVEY.md §8d "candidate perms are
    Philox-seeded") as uint8 rows, generated on the device."""
    import torch
    return ctx.random_tours(C, n, seed, stream_id=0xBE7C, dtype=dtype or torch.uint8)


def cpu_model() -> str:
    """The host CPU model (lscpu's "Model name", from /proc/cpuinfo)."""
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    import platform
    return platform.processor() or "unknown"


def host_cores():
    """(threads, record) for the host legs: every CPU this process may run
    on (sched_getaffinity), capped by the cgroup's CPU quota (cpu.max: a
    quota of q CPUs' time makes more than ceil(q) busy threads time-slice)
    and by OMP_NUM_THREADS when the box sets it; the record says which bound
    applied."""
    aff = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else os.cpu_count()
    quota = None
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            q, period = f.read().split()[:2]
            if q != "max":
                quota = int(q) / int(period)
    except (OSError, ValueError):
        pass
    omp = int(os.environ.get("OMP_NUM_THREADS", "0") or 0)
    threads = aff
    bound = "sched_getaffinity"
    if quota is not None and math.ceil(quota) < threads:
        threads, bound = int(math.ceil(quota)), "cgroup cpu.max quota"
    if omp and omp < threads:
        threads, bound = omp, "OMP_NUM_THREADS"
    return max(1, threads), {"threads": max(1, threads), "bound_by": bound,
                             "sched_getaffinity": aff, "cgroup_cpu_quota": quota,
                             "OMP_NUM_THREADS": omp or None, "os_cpu_count": os.cpu_count()}


def cpu_baseline(inst, perms_dev, seconds):
    """Time the C oracle (OpenMP, all threads it is given) on a bounded
    sample of the same tours; returns the cpu_baseline object."""
    import numpy as np
    from oracle import coracle
    coracle.build()
    threads, cores = host_cores()
    S = int(min(perms_dev.shape[0], 4 << 20))
    sample = perms_dev[:S].cpu().numpy()
    passes, dt, ref = 0, 0.0, None
    while dt < seconds and passes < 64:        # repeat passes until ~`seconds` of CPU work
        t0 = time.perf_counter()
        ref = coracle.eval_batch(inst.durations, sample, inst.demand, inst.capacities,
                                 inst.start_times, 1, 0, threads=threads)
        dt += time.perf_counter() - t0
        passes += 1
    # the pure-Python restatement in the reference's own stdlib style (SURVEY
    # §8d comparator (i)), one core, a small slice of the same tours
    from oracle import spec
    py_n, t0 = 0, time.perf_counter()
    while time.perf_counter() - t0 < min(2.0, seconds) and py_n < S:
        spec.eval_cvrp(inst.durations, sample[py_n], inst.demand, inst.capacities,
                       inst.start_times)
        py_n += 1
    py_dt = time.perf_counter() - t0
    return {"value": S * passes / dt, "unit": "evals/s", "cores": threads, "kind": "port",
            "cpu_model": cpu_model(), "host_cpus_visible": os.cpu_count(), "host_cores": cores,
            "sample": f"{passes} pass(es) over the first {S} of the same CVRP-100 tours, C "
                      f"restatement oracle/oracle_c.c (OpenMP, {threads} threads), "
                      f"{dt:.2f} s",
            "python_port": {"value": py_n / py_dt, "unit": "evals/s", "cores": 1,
                            "sample": f"first {py_n} of the same tours through oracle/spec.py "
                                      f"eval_cvrp (pure Python, the reference's language), "
                                      f"{py_dt:.2f} s"}}, ref, S


class _TimedCooling:
    """Geometric cooling from t0 to t_end spread over a WALL-TIME budget: after
    every epoch the remaining ratio t_cur/t_end is re-spread over the steps the
    measured rate says still fit, so both legs end cold exactly when their
    time runs out (a step-count schedule calibrated up front finishes early
    or late by whatever the calibration missed)."""

    def __init__(self, seconds, t0, t_end, epochs=40):
        self.seconds, self.t_end, self.epochs = seconds, t_end, epochs
        self.inv_t = np.float32(1.0 / t0)
        self.t_start = time.perf_counter()

    def elapsed(self):
        return time.perf_counter() - self.t_start

    def plan(self, steps_done, min_steps=50):
        """(steps for the next epoch, inv_alpha for it), or (0, None) when the
        budget is spent.  The first epoch is a short rate probe."""
        el = self.elapsed()
        left = self.seconds - el
        if left <= 0:
            return 0, None
        if steps_done == 0:
            remaining = None
            steps = min_steps
        else:
            rate = steps_done / el
            remaining = max(min_steps, int(rate * left))
            steps = min(remaining, max(min_steps, int(rate * self.seconds / self.epochs)))
        t_cur = 1.0 / float(self.inv_t)
        if remaining is None or t_cur <= self.t_end:
            inv_a = np.float32(1.0)
        else:
            inv_a = np.float32((t_cur / self.t_end) ** (1.0 / remaining))
        return steps, inv_a

    def advance(self, steps, inv_a):
        for _ in range(steps):          # the kernels' float32 recurrence
            self.inv_t = np.float32(self.inv_t * inv_a)


def quality(ctx, inst, seconds, world, rank, dist, with_cpu, chains=4096, label="cvrp100_k8 seed 0",
            gpu_seed=None, n_sep=None, window=0, window_types=0, start="random", moves=64,
            cpu_moves=64, gpu=True, mig_every=1, mig_E=None, epochs=40, t0_frac=0.5,
            tend_frac=0.002, cpu_tend_frac=None, cpu_t0_frac=None):
    """Best-cost gap at fixed wall time (the metric's second half): the same SA
    (Philox streams, 64 sampled moves per step, geometric cooling from
    t0_frac to tend_frac x the typical edge spread over the wall-time budget
    by _TimedCooling, `epochs` epochs) on the GPU -- `chains` chains, every
    `mig_every` epochs the mig_E best-so-far tours replace the mig_E worst
    current ones (across ranks when N > 1) -- and on the host cores
    (the same migration scaled to its chains; cpu_tend_frac: its own final
    temperature) (oracle/oracle_c.c oracle_sa_run_resync, one chain per OpenMP thread,
    each candidate priced by walking only the span the move can change and
    jumping over unchanged routes -- the same trajectories as the full walk).  Both legs run until
    `seconds` of wall time are spent.  Both legs search giant tours with
    n_sep A10 route separators (default K - 1, the front-end's VRP SA), so
    the moves place route boundaries too; `window` > 0 samples A11 windowed
    moves of the A12 types `window_types`, and `start` places the separators
    of the start tours ("random", "greedy": the greedy split's route
    boundaries, "pack": first-fit routes -- large instances).  `moves` is the
    GPU leg's move sample per step (64 W on W wavefronts per chain, at about
    the per-step latency of one), `cpu_moves` the host leg's.  gap = (gpu - cpu) / cpu on the
    objective key's primary term (durationSum) with unvisited == 0."""
    import torch
    from vrpms_amd import islands, runners
    n = inst.n
    n_sep = inst.K - 1 if n_sep is None else n_sep
    # a quarter of the chains restart from the elites every epoch (at most the
    # 1024 vrpms_pool_elites selects at once)
    mig_E = min(max(1, chains // 4), 1024) if mig_E is None else mig_E
    dev = ctx.dev
    edge = runners.typical_edge(inst.durations)
    t0, t_end = t0_frac * edge, tend_frac * edge
    out = {"T_s": seconds, "algorithm": "sa", "instance": label, "cooling": "wall-time geometric",
           "t0_per_edge": {"gpu": t0_frac, "cpu": cpu_t0_frac or t0_frac},
           "t_end_per_edge": {"gpu": tend_frac, "cpu": cpu_tend_frac or tend_frac},
           "separators": n_sep, "window": window, "window_types": window_types, "start": start}
    if gpu:
        warm = runners.SARunner(ctx, n, chains=chains, total_steps=1000, durations=inst.durations,
                                n_sep=n_sep, window=window, window_types=window_types, start=start,
                                moves=moves)
        warm.epoch(20)                       # first launch: code object load, LDS setup
        torch.cuda.synchronize(dev)
        del warm
        seed = (1000 + rank) if gpu_seed is None else gpu_seed
        r = runners.SARunner(ctx, n, chains=chains, seed=seed, total_steps=1000,
                             durations=inst.durations, t0=t0, t_end=t_end, n_sep=n_sep,
                             window=window, window_types=window_types, start=start, moves=moves)
        if world > 1:
            dist.barrier()
        cool = _TimedCooling(seconds, t0, t_end, epochs=epochs)
        e = 0
        while True:
            steps, inv_a = cool.plan(r.step)
            if steps == 0:
                break
            r.inv_alpha = inv_a
            r.epoch(steps)
            cool.advance(steps, inv_a)
            e += 1
            if e % mig_every == 0:
                if world > 1:
                    islands.exchange(r, mig_E)
                else:
                    r.inject(*r.elites(mig_E))
            torch.cuda.synchronize(dev)
        gpu_wall = cool.elapsed()
        key, tour = r.best()
        if world > 1:
            key, tour = islands.global_best(r)
        # the search's own key for its best tour against a fresh exact score
        # of that tour (the library's scoring kernel, parity-tested)
        rescored = _rescore(ctx, tour)
        out["gpu"] = {"chains_per_gpu": chains, "moves_per_step": moves, "steps_per_chain": r.step,
                      "migration": {"every_epochs": mig_every, "elites": mig_E},
                      "epochs": e, "wall_s": gpu_wall, "unvisited": key >> 56,
                      "duration_sum": (key >> 28) & (2**28 - 1),
                      "rescored_equal": rescored == key}
    if with_cpu:
        from oracle import coracle
        threads, cores = host_cores()
        if n_sep and start == "greedy":
            t0_ = ctx.insert_separators(ctx.random_tours(threads, n, 7), n_sep)
        elif n_sep and start == "pack":
            t0_ = ctx.pack_separators(ctx.random_tours(threads, n, 7), n_sep)
        else:
            t0_ = ctx.random_tours(threads, n, 7, n_sep=n_sep)
        cur = np.asarray(t0_.cpu().numpy()).view(np.uint16)
        cur = cur.copy()
        best = cur.copy()
        bk = np.full(threads, 2**64 - 1, dtype=np.uint64)
        # the host leg's final temperature (its own best schedule, if given)
        t_end_h = t_end if cpu_tend_frac is None else cpu_tend_frac * edge
        t0_h = t0 if cpu_t0_frac is None else cpu_t0_frac * edge
        cool = _TimedCooling(seconds, t0_h, t_end_h, epochs=epochs)
        # the GPU leg's migration scaled to the host's chains: every mig_every
        # epochs the same fraction of chains restarts from the best-so-far
        # tours (the E best by key replace the E worst current tours)
        e_host = max(1, int(round(threads * mig_E / chains))) if mig_every else 0
        step = e = 0
        while True:
            steps, inv_a = cool.plan(step)
            if steps == 0:
                break
            ck = coracle.sa_run(inst.durations, cur, best, bk, steps, float(cool.inv_t),
                                float(inv_a), 1, step, inst.demand, inst.capacities,
                                inst.start_times, threads=threads, window=window,
                                window_types=window_types, resync=True, moves=cpu_moves)
            cool.advance(steps, inv_a)
            step += steps
            e += 1
            if e_host and e % mig_every == 0 and threads > 1:
                top = np.argsort(bk, kind="stable")[:e_host]
                worst = np.argsort(np.asarray(ck, dtype=np.uint64), kind="stable")[::-1][:e_host]
                cur[worst] = best[top]
        cpu_wall = cool.elapsed()
        ck = int(bk.min())
        cpu_rescored = _rescore(ctx, best[int(np.argmin(bk))].tolist())
        out["cpu"] = {"chains": threads, "cores": threads, "host_cores": cores,
                      "moves_per_step": cpu_moves,
                      "migration": {"every_epochs": mig_every, "elites": e_host},
                      "steps_per_chain": step,
                      "wall_s": cpu_wall, "unvisited": ck >> 56,
                      "duration_sum": (ck >> 28) & (2**28 - 1),
                      "rescored_equal": cpu_rescored == ck,
                      "kind": "port (oracle/oracle_c.c oracle_sa_run_resync: "
                              "candidates priced by walking only what the move changes)"}
        if gpu:
            g, c = out["gpu"], out["cpu"]
            ok = g["unvisited"] == 0 and c["unvisited"] == 0 and c["duration_sum"]
            out["gap"] = (g["duration_sum"] - c["duration_sum"]) / c["duration_sum"] if ok else None
            out["gap_sign"] = "negative = GPU better"
    return out


def algo_quality(ctx, inst, seconds, seed=0, polish_steps=100, polish_top=4,
                 aco_shape=(64, 64, 5)):
    """The GA and ACO endpoints' best cost at the same wall time as the SA
    quality leg (cfg 2, api/vrp/{ga,aco}/index.py): each runs on the GPU for
    `seconds` of wall time -- GA 256 islands x 256 (randomPermutationCount),
    20 fused generations per epoch; ACO 64 colonies x 64 ants, 5 iterations
    per epoch, best-so-far deposit every 5th -- with elite migration every 5
    epochs (inject(elites(16)), as the SA leg).  Both are memetic: after each
    epoch the GA's `polish_top` best members of every island and ACO's colony
    bests take `polish_steps` SA steps (runners.Polish, the SA endpoint's
    moves), cooled from 0.05 to 0.002 x the mean edge over the wall-time
    budget (_TimedCooling).  Their giant tours carry no separators: the A3
    greedy split places the routes."""
    import torch
    from vrpms_amd import runners
    out = {}
    edge = runners.typical_edge(inst.durations)
    for name in ("ga", "aco"):
        pol = runners.Polish(polish_steps, inst.durations, seed=seed + 17) if polish_steps else None
        if name == "ga":
            r = runners.GARunner(ctx, inst.n, islands=256, pop=256, seed=seed, gens_per_epoch=20,
                                 polish=pol, polish_top=polish_top)
            unit, per = "generations", 20
        else:
            r = runners.ACORunner(ctx, inst.n, colonies=aco_shape[0], ants=aco_shape[1],
                                  seed=seed, iters_per_epoch=aco_shape[2], bsf_period=5,
                                  polish=pol)
            unit, per = "iterations", aco_shape[2]
        r.epoch()                              # first launch: code object load
        torch.cuda.synchronize(ctx.dev)
        cool = _TimedCooling(seconds, 0.05 * edge, 0.002 * edge)
        e = done = 0
        while True:
            _, inv_a = cool.plan(done, min_steps=polish_steps or 1)
            if inv_a is None:
                break
            if pol is not None:
                pol.inv_t, pol.inv_alpha = cool.inv_t, inv_a
            r.epoch()
            if pol is not None:
                cool.advance(polish_steps, inv_a)
                done += polish_steps
            else:
                done += 1
            e += 1
            if e % 5 == 0:
                r.inject(*r.elites(16))
            torch.cuda.synchronize(ctx.dev)
        wall = cool.elapsed()
        key, _ = r.best()
        out[name] = {unit: (e + 1) * per, "epochs": e, "wall_s": wall,
                     "memetic": {"polish_steps_per_epoch": polish_steps,
                                 "polished": f"top {polish_top} per island" if name == "ga"
                                 else "colony bests"} if pol is not None else None,
                     "unvisited": key >> 56, "duration_sum": (key >> 28) & (2**28 - 1)}
        del r
    return out


def _host_best(ctx, inst, seconds, dist, kw, moves_list):
    """The host leg at each move count; (best leg, all legs) by durationSum."""
    legs = [quality(ctx, inst, seconds, 1, 0, dist, with_cpu=True, cpu_moves=m, gpu=False,
                    **kw)["cpu"] for m in moves_list]
    ok = [c for c in legs if c["unvisited"] == 0]
    best = min(ok, key=lambda c: c["duration_sum"]) if ok else legs[0]
    return best, legs


def _gap(g, c):
    if g["unvisited"] == 0 and c["unvisited"] == 0 and c["duration_sum"]:
        return (g["duration_sum"] - c["duration_sum"]) / c["duration_sum"]
    return None


def _rescore(ctx, tour):
    """Exact key of one tour (a list of tokens) by the library's scoring
    kernel, as an unsigned int."""
    import torch
    t = torch.tensor([list(tour)], dtype=torch.int16, device=ctx.dev)
    return int(ctx.eval(t)[0]) & (2**64 - 1)


def equal_time_cells(ctx, seconds, dist, with_cpu, instance="x1000", seeds=(0, 1, 2),
                     cpu_moves=(32, 64), repeat_host=True, host_repeats=2):
    """The metric's second half, several seeds: per seed the GPU
    leg (x1000: sa_seg_kernel; tdvrp200: sa_route_kernel -- 256 chains x 128
    moves per step, W = 2 wavefronts per chain) against the host port
    (oracle_sa_run_resync, one chain per host thread) at each of `cpu_moves`
    moves per step, the better host result kept.  `repeat_host` runs seed
    0's better host leg a second time: the host's run-to-run spread (its
    wall-time cooling follows the measured step rate, so two runs of one seed
    differ) is reported beside the gaps, and a gap counts as a GPU win only
    when it is below minus that spread."""
    import statistics

    from vrpms_amd import synth
    from vrpms_amd.core import CVRP
    make = {"x1000": lambda sd: synth.x_style(1000, seed=sd),
            "tdvrp200": lambda sd: synth.td_cvrp(200, 16, seed=sd),
            "tdvrp200_het": lambda sd: synth.td_cvrp_het(200, 16, seed=sd)}[instance]
    # GPU shapes from tools/migration_scan.py (10 s, seeds 0-2): X-1000 at 1024
    # chains x 128 moves (W = 2: two wavefronts per SIMD, sa_seg_kernel's OCC = 2
    # variant), a migration every epoch of 80 with the 256 best replacing the
    # 256 worst; TD-200 at 256 x
    # 128 (its shapes were within run-to-run noise of each other).  Final
    # temperatures from tools/sched_scan.py (10 s, seeds 0-1, both legs at six
    # schedules): each leg at the one that scored best for it on average --
    # X-1000: (t0, t_end) = (0.5, 0.004) x the typical edge for the GPU, (0.5,
    # 0.002) for the host; TD-200: (0.5, 0.004) and (1.0, 0.002).  Round 6
    # (tools/migration_scan.py, seeds 0-2, profiles/round6_x1000_shape_scan_*):
    # the GPU's X-1000 t_end 0.004 -> 0.003 (82,844 / 78,514 / 78,392 against
    # 83,156 / 78,730 / 78,291; 512 x 128, 512 x 256, 256 x 256 and 1,024 x 256
    # were worse on the mean)
    # TD-200 (uniform and heterogeneous fleets) on sa_td_kernel, round 5: shape
    # and final temperature from tools/td_quality_scan.py
    kw = dict(chains=1024, moves=128, window=32, window_types=2, start="pack", epochs=80,
              mig_E=256, tend_frac=0.003, cpu_tend_frac=0.002) if instance == "x1000" else \
        dict(chains=TD_SHAPE[0], moves=TD_SHAPE[1], window=32, window_types=2, start="pack",
             mig_E=TD_SHAPE[2], tend_frac=TD_SHAPE[3], cpu_t0_frac=1.0, cpu_tend_frac=0.002)
    cells = []
    spread = None
    for sd in seeds:
        progress(f"{instance} seed {sd}")
        x = make(sd)
        ctx.set_instance(CVRP, x.durations, x.demand, x.capacities, x.start_times)
        q = quality(ctx, x, seconds, 1, 0, dist, with_cpu=False, label=f"{instance} seed {sd}",
                    **kw)
        cell = {"seed": sd, "gpu": q["gpu"]}
        if with_cpu:
            progress(f"{instance} seed {sd}: host legs")
            best, legs = _host_best(ctx, x, seconds, dist, kw, cpu_moves)
            cell["cpu"] = best
            cell["cpu_legs"] = [{"moves_per_step": c["moves_per_step"],
                                 "duration_sum": c["duration_sum"], "unvisited": c["unvisited"],
                                 "steps_per_chain": c["steps_per_chain"]} for c in legs]
            cell["gap"] = _gap(q["gpu"], best)
            if repeat_host and spread is None:
                runs = [best["duration_sum"]]
                for _ in range(max(1, host_repeats)):
                    runs.append(quality(ctx, x, seconds, 1, 0, dist, with_cpu=True, gpu=False,
                                        cpu_moves=best["moves_per_step"], **kw)["cpu"]
                                ["duration_sum"])
                spread = {"seed": sd, "moves_per_step": best["moves_per_step"], "runs": runs,
                          "min": min(runs), "max": max(runs),
                          "rel": (max(runs) - min(runs)) / min(runs)}
        cells.append(cell)
    out = {"instance": instance, "T_s": seconds, "seeds": list(seeds),
           "fleet": {"capacities": [int(c) for c in make(seeds[0]).capacities],
                     "start_times": [int(t) for t in make(seeds[0]).start_times]}
           if instance == "tdvrp200_het" else "uniform",
           "gpu_kernel": "sa_seg_kernel" if instance == "x1000" else "sa_td_kernel",
           "gpu_shape": f"{kw['chains']} chains x {kw['moves']} moves per step "
                        f"(W = {kw['moves'] // 64})",
           "host": f"oracle_sa_run_resync, better of {list(cpu_moves)} moves per step",
           "window": 32, "window_types": 2, "start": "pack", "cells": cells,
           "gap_sign": "negative = GPU better"}
    gaps = [c["gap"] for c in cells if c.get("gap") is not None]
    if gaps:
        out["gap_median"] = statistics.median(gaps)
        out["gpu_better"] = f"{sum(g < 0 for g in gaps)} / {len(gaps)}"
    if spread is not None:
        out["host_run_to_run"] = spread
        if gaps:
            out["median_beyond_spread"] = out["gap_median"] < -spread["rel"]
    return out


def quality_summary(out):
    """Every equal-time cell as [gpu, host, gap %] (durationSum, gap negative
    = GPU better), the medians and the host's run-to-run spread."""
    def r(x, nd=2):
        return None if x is None else round(100.0 * x, nd)
    s = {}
    q = out.get("quality") or {}
    if "gpu" in q and "cpu" in q:
        s["cfg2_sa"] = [q["gpu"]["duration_sum"], q["cpu"]["duration_sum"], r(q.get("gap"))]
        for name, v in (q.get("by_algorithm") or {}).items():
            s[f"cfg2_{name}"] = [v.get("duration_sum"), q["cpu"]["duration_sum"],
                                 r(v.get("gap_vs_host_sa"))]
    for key, tag in (("quality_x1000", "x1000"), ("quality_x1000_long", "x1000_long"),
                     ("quality_tdvrp200", "td200"), ("quality_tdvrp200_het", "td200het")):
        c = out.get(key) or {}
        for cell in c.get("cells", []):
            if "cpu" in cell:
                s[f"{tag}_s{cell['seed']}"] = [cell["gpu"]["duration_sum"],
                                               cell["cpu"]["duration_sum"], r(cell.get("gap"))]
        if "gap_median" in c:
            s[f"{tag}_median"] = r(c["gap_median"])
            s[f"{tag}_gpu_better"] = c.get("gpu_better")
        sp = c.get("host_run_to_run")
        if sp:
            s[f"{tag}_host_spread"] = {"runs": sp["runs"], "min": sp["min"], "max": sp["max"],
                                       "rel_pct": r(sp["rel"])}
            s[f"{tag}_median_beyond_spread"] = c.get("median_beyond_spread")
        if "error" in c:
            s[f"{tag}_error"] = c["error"][-200:]
    s["units"] = "[gpu, host, gap %] durationSum at equal wall time; gap < 0 = GPU better"
    return s


def other_configs(ctx, torch, dev, seed=0, r_lds=None):
    """Secondary lines for the other BASELINE.json configs (not the headline)."""
    from vrpms_amd import synth
    from vrpms_amd.core import CVRP
    out = {}
    # measured L2-gather ceiling (random 2-byte loads over a uint16 table the
    # size of each matrix; vrpms_probe_l2_gather) -- the staged kernels' roofline
    r_td = ctx.probe_l2_gather(slots=24 * 201 * 201)
    r_x = ctx.probe_l2_gather(slots=1001 * 1001)

    def kernel_time(fn, reps=5):
        fn()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        torch.cuda.synchronize(dev)
        e0.record()
        for _ in range(reps):
            fn()
        e1.record()
        torch.cuda.synchronize(dev)
        return e0.elapsed_time(e1) * 1e-3 / reps

    # cfg 3: time-dependent VRP-200 x 24 h (4.0 MB int32 / 1.9 MB u16: L2-resident gathers)
    td = synth.td_cvrp(200, 16, seed=seed)
    ctx.set_instance(CVRP, td.durations, td.demand, td.capacities, td.start_times)
    C = 1 << 21
    perms = make_batch(ctx, C, td.n, seed + 11)
    keys = torch.empty(C, dtype=torch.int64, device=dev)
    t = kernel_time(lambda: ctx.eval(perms, out=keys))
    out["cfg3_tdvrp200_h24"] = {"kernel": "eval_staged<u16 L2, H=24, u8 tours>",
                                "evals_per_s": C / t, "candidates": C,
                                "gathers_per_eval": td.n + td.K, "l2_gathers_per_eval": td.n,
                                "l2_roofline": {"r_gather_measured": r_td, "unit": "gathers/s",
                                                "frac": C / t * td.n / r_td}}
    # cfg 4: X-style CVRP-1000 (uint16 tours, 2.0 MB u16 matrix: L2-resident)
    x = synth.x_style(1000, seed=seed)
    ctx.set_instance(CVRP, x.durations, x.demand, x.capacities, x.start_times)
    C = 1 << 18
    p16 = make_batch(ctx, C, x.n, seed + 13, dtype=torch.int16)
    keys = torch.empty(C, dtype=torch.int64, device=dev)
    t = kernel_time(lambda: ctx.eval(p16, out=keys))
    out["cfg4_x1000"] = {"kernel": "eval_staged<u16 L2, H=1, u16 tours>", "evals_per_s": C / t,
                         "candidates": C, "vehicles": x.K, "gathers_per_eval": x.n + x.K,
                         "l2_gathers_per_eval": x.n,
                         "l2_roofline": {"r_gather_measured": r_x, "unit": "gathers/s",
                                         "frac": C / t * x.n / r_x}}
    # cfg 5: throughput mode, 10k concurrent TSP-50 requests, one workgroup per request
    R, steps = 10000, 1000
    rng = np.random.default_rng(seed)
    mats = torch.tensor(np.stack([synth.random_symmetric(50, rng) for _ in range(R)]),
                        dtype=torch.int32, device=dev)
    t = kernel_time(lambda: ctx.tsp_batch_sa(mats, steps, 1 / 80.0, 1 / 0.995, 1), reps=3)
    mev = R * 4 * steps * 64 / t
    out["cfg5_tsp50_x10k"] = {"kernel": "tsp_batch_sa_kernel (1 WG / request, 4 chains)",
                              "requests_per_s": R / t, "batch_latency_ms": t * 1e3,
                              "sa_steps_per_chain": steps,
                              "move_evals_per_s": mev,
                              # each move: an O(1) symmetric delta of 8 matrix gathers from the
                              # request's LDS-staged matrix (tsp_move_delta_sym), priced against
                              # the measured random LDS-gather rate
                              "roofline": {"bound": "lds_gather", "gathers_per_move": 8,
                                           "achieved": mev * 8, "peak": r_lds, "unit": "gathers/s",
                                           "frac": mev * 8 / r_lds if r_lds else None}}
    del mats
    try:
        out["cfg5_http"] = cfg5_http_leg(R=R, steps=steps)
    except Exception:
        out["cfg5_http"] = {"error": traceback.format_exc(limit=3)}
    try:
        out["cfg5_api"] = cfg5_api_pool_leg(R=R, steps=steps)
    except Exception:
        out["cfg5_api"] = {"error": traceback.format_exc(limit=3)}
    try:
        out["cfg5_api_one_process"] = cfg5_api_leg(torch, dev, R=R, steps=steps, seed=seed)
    except Exception:
        out["cfg5_api_one_process"] = {"error": traceback.format_exc(limit=3)}
    return out


def cfg5_api_pool_leg(R=10000, steps=1000):
    """Config 5 at the API across processes (vrpms_amd.frontends.FrontEndPool):
    front-end worker processes parse / ingest / answer the R /api/tsp/sa
    requests and feed one GPU-owner process through shared memory.  This
    process has initialised the GPU, so the pool runs as a child program
    (forked workers must come from a process that has not); its own clock
    brackets the R requests, and it checks a sample of the answers'
    durations against their tours (A4)."""
    import subprocess
    threads, cores = host_cores()
    workers = max(2, threads - 2)        # the parent and the GPU owner keep a core each
    cmd = [sys.executable, "-m", "vrpms_amd.frontends", "bench", "--requests", str(R),
           "--workers", str(workers), "--steps", str(steps)]
    res = subprocess.run(cmd, cwd=ROOT, capture_output=True, text=True, timeout=600)
    if res.returncode != 0:
        return {"error": f"exit {res.returncode}", "stderr": res.stderr[-2000:]}
    out = json.loads(res.stdout.strip().splitlines()[-1])
    out["host_cores"] = cores
    return out


def cfg5_http_leg(R=10000, steps=1000, connections=1024):
    """Config 5 over real sockets (BASELINE cfg 5: 10k concurrent TSP-50
    requests): FrontEndPool workers listen on one port (SO_REUSEPORT) and a
    load generator in separate client processes holds `connections`
    keep-alive connections sending R POST /api/tsp/sa; requests/s at the
    client.  Runs as a child program (this process has initialised the GPU)."""
    import subprocess
    threads, cores = host_cores()
    clients = max(1, min(4, threads // 4))
    workers = max(2, threads - clients - 1)   # the GPU owner keeps a core (the pool's parent sleeps)
    cmd = [sys.executable, "-m", "vrpms_amd.frontends", "bench-http", "--requests", str(R),
           "--workers", str(workers), "--steps", str(steps), "--clients", str(clients),
           "--connections", str(connections)]
    res = subprocess.run(cmd, cwd=ROOT, capture_output=True, text=True, timeout=600)
    if res.returncode != 0:
        return {"error": f"exit {res.returncode}", "stderr": res.stderr[-2000:]}
    out = json.loads(res.stdout.strip().splitlines()[-1])
    out["host_cores"] = cores
    return out


def cfg5_api_leg(torch, dev, R=10000, steps=1000, workers=256, seed=0, N=50):
    """Config 5 at the API in ONE process (the GIL-bound contrast to
    cfg5_api_pool_leg): R concurrent /api/tsp/sa requests (the reference's
    request body, api/tsp/sa/index.py:40-44; each its own random symmetric
    50-node matrix served as the DB's JSON nested lists) posted in-process
    to service.App from a `workers`-thread pool; TspBatcher coalesces them
    into tsp_batch_sa launches (one workgroup per request).  End-to-end
    requests/s counts JSON parsing, parameter checks, the matrix ingest and
    compaction, batching, the launch and the response dict, beside the
    kernel-only line above."""
    import json as _json
    from concurrent.futures import ThreadPoolExecutor

    from vrpms_amd import service, synth
    rng = np.random.default_rng(seed + 5)
    store = service.MemoryStore({0: [{"id": i} for i in range(N)]},
                                {i: synth.random_symmetric(N, rng).tolist() for i in range(R)})
    bodies = [_json.dumps({"solutionName": "n", "solutionDescription": "d", "locationsKey": 0,
                           "durationsKey": i, "customers": list(range(1, N)), "startNode": 0,
                           "startTime": 0}).encode() for i in range(R)]
    app = service.App(store, batch_tsp=True, batch_window_s=0.002, batch_steps=steps)
    post = lambda b: app.post("tsp", "sa", b)  # noqa: E731
    with ThreadPoolExecutor(workers) as ex:
        list(ex.map(post, bodies[:512]))          # warm: code objects, context, pools
        launches0, req0 = app.batcher.launches, app.batcher.requests
        t0 = time.perf_counter()
        res = list(ex.map(post, bodies))
        dt = time.perf_counter() - t0
    ok = sum(1 for st, _ in res if st == 200)
    launches = app.batcher.launches - launches0
    # host-only cost of one request's parse / ingest / compaction (no GPU)
    t1 = time.perf_counter()
    for b in bodies[:500]:
        errs = []
        params, _ = service.parse("tsp", "sa", _json.loads(b), errs)
        d = store.session(None).get_durations_by_id(params["durations_key"], errs)
        app._batched_tsp(params, d)
    host_us = (time.perf_counter() - t1) / 500 * 1e6
    return {"workload": f"{R} POST /api/tsp/sa, TSP-{N} each, in-process App + TspBatcher",
            "threads": workers, "batch_window_ms": 2.0, "sa_steps_per_chain": steps,
            "requests_per_s": R / dt, "wall_s": dt, "ok": ok, "launches": launches,
            "requests_per_launch": (app.batcher.requests - req0) / max(launches, 1),
            "host_parse_ingest_us_per_request": host_us,
            "note": "one Python process: JSON + nested-list matrix ingest (~0.3 ms per request) "
                    "under the GIL bounds the API path, not the kernel"}


def island_leg(ctx, torch, dev, world, rank, dist, epochs=40, steps=500, chains=1024, E=8,
               every=5, seed=0, window=32):
    """BASELINE.json cfg 4 as a search, not a scoring pass: X-style CVRP-1000
    (u16 matrix L2-resident), `chains` SA chains per GPU, a fixed number of
    epochs with an elite exchange every `every` epochs through the library's
    own communicator: vrpms_island_exchange = device top-E, one RCCL
    ncclAllGather of every rank's E best (tour + key) over xGMI, device merge
    and injection (islands.init_comm creates it from the torch.distributed
    group at N > 1; at N = 1 a world-1 communicator, so the same RCCL call
    runs).  If the communicator cannot be created on every rank, every rank
    falls back to torch.distributed's all-gather around the same library
    pack / merge / inject and says so.  Tours carry K - 1 A10 separators
    from first-fit ("pack") starts and the moves are A11-windowed 2-opt,
    priced in O(1) by sa_seg_kernel (prefix sums over the positions, no
    walk), so the throughput is reported as exact move pricings per second
    -- not comparable with the headline's streamed full-tour evals.  Every
    rank runs the same control flow (islands.run_fixed), and a pre-flight
    all-reduce makes all ranks skip together if any rank failed to set up.
    ~1 s of wall time by default, so the exchange share means something."""
    from vrpms_amd import islands, runners, synth
    from vrpms_amd.core import CVRP
    ok, err, r = 1, None, None
    try:
        x = synth.x_style(1000, seed=seed)
        ctx.set_instance(CVRP, x.durations, x.demand, x.capacities, x.start_times)
        # the front-end's large-instance SA: K - 1 separators packed first-fit,
        # A11 windowed 2-opt priced route-locally
        r = runners.SARunner(ctx, x.n, chains=chains, seed=500 + rank,
                             total_steps=epochs * steps, steps_per_epoch=steps,
                             durations=x.durations, n_sep=x.K - 1, window=window,
                             window_types=2, start="pack")
        r.epoch(2)                          # code object load, instance staging
        torch.cuda.synchronize(dev)
    except Exception:
        ok, err = 0, traceback.format_exc(limit=3)
    if world > 1:
        f = torch.tensor([ok], dtype=torch.int32, device=dev)
        dist.all_reduce(f, op=dist.ReduceOp.MIN)
        ok = int(f.item())
    if not ok:
        return {"error": err or "another rank failed to set up"}
    comm_err = None
    try:
        if world > 1:
            islands.init_comm(ctx, timeout_s=120)   # raises on every rank or on none
        else:
            ctx.island_init(ctx.island_unique_id(), 0, 1)
        path = "vrpms_island_exchange (library RCCL ncclAllGather" + \
               (" over xGMI)" if world > 1 else ", world-1 communicator)")
    except Exception:
        comm_err = traceback.format_exc(limit=2)
        path = "library pack/merge/inject around torch.distributed all_gather (fallback)"
    # untimed warm epoch + exchange: sort/gather kernels load, communicators form
    islands.run_fixed(r, 1, 1, E)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    step0 = r.step
    t0 = time.perf_counter()
    n_ex, t_ex = islands.run_fixed(r, epochs, every, E,
                                   sync=lambda: torch.cuda.synchronize(dev))
    torch.cuda.synchronize(dev)
    wall = time.perf_counter() - t0
    chain_steps = r.step - step0
    key, tour = r.best()
    if world > 1:
        t = torch.tensor([wall, t_ex], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        wall, t_ex = float(t[0]), float(t[1])
        key, _ = islands.global_best(r)
    moves = world * chains * chain_steps * 64
    out = {"workload": "cfg4 X-style CVRP-1000, island SA", "ranks": world,
           # the library communicator's own count (0: the torch fallback ran)
           "rccl_ranks": ctx.island_world(),
           "exchange_path": "fallback" if comm_err else "library rccl",
           "vehicles": x.K,
           "separators": x.K - 1, "window": window,
           "kernel": "sa_seg_kernel (every move priced in O(1) from prefix sums over the "
                     "positions; static symmetric matrix, one capacity)",
           "chains_per_gpu": chains, "epochs": epochs, "steps_per_epoch": steps,
           "moves_per_step": 64, "exchange_every": every, "elites": E,
           "exchange": path, "wall_s": wall,
           "move_evals_per_s": moves / wall,
           "move_evals_unit": "exact move pricings (each the moved tour's full key, priced "
                              "from prefix sums without walking it; not comparable with the "
                              "headline's streamed full-tour evals)",
           "chain_steps_per_s": chain_steps / wall,
           "exchanges": n_ex, "exchange_ms_mean": t_ex / max(n_ex, 1) * 1e3,
           "exchange_share_of_wall": t_ex / wall,
           "best": {"unvisited": key >> 56, "duration_sum": (key >> 28) & (2**28 - 1)}}
    if comm_err:
        out["comm_error"] = comm_err
    return out


def search_lines(ctx, torch, dev, r_gather, seed=0):
    """Throughput of the GA / ACO / BF endpoints' algorithms on BASELINE cfg 2
    (CVRP-100, K = 8) -- the slots api/vrp/{ga,aco,bf}/index.py fill.  GA and
    ACO score their children / ants with eval_cvrp_words2 (the headline
    kernel) inside vrpms_ga_generation / vrpms_aco_iteration; evals/s counts
    full tour evaluations, the LDS-gather fraction prices them at G = n + K
    gathers against the measured R_gather (the whole generation's time, so
    breeding / construction and selection are inside it)."""
    from vrpms_amd import runners, synth
    from vrpms_amd.core import CVRP
    inst = synth.cvrp(100, 8, seed=seed)
    ctx.set_instance(CVRP, inst.durations, inst.demand, inst.capacities, inst.start_times)
    G = inst.n + inst.K
    out = {}

    def timed(fn, reps):
        fn()
        torch.cuda.synchronize(dev)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        t0 = time.perf_counter()
        e0.record()
        for _ in range(reps):
            fn()
        e1.record()
        torch.cuda.synchronize(dev)
        return (time.perf_counter() - t0) / reps, e0.elapsed_time(e1) * 1e-3 / reps

    # GA: 256 islands x 256 (randomPermutationCount) -- one island per CU --
    # 20 generations per call, fused (one workgroup per island for the whole
    # call) and, for comparison, the three-launch path on the same islands
    islands_, pop = 256, 256
    ga_out = {}
    for mode, gens, reps in ((0, 20, 5), (2, 5, 3)):
        ctx.set_ga_fused(mode)
        ga = runners.GARunner(ctx, inst.n, islands=islands_, pop=pop, seed=seed,
                              gens_per_epoch=gens)
        wall, dev_s = timed(ga.epoch, reps)
        children = islands_ * pop * gens
        ga_out["fused" if mode == 0 else "three_kernel"] = {
            "generations_per_call": gens, "generations_per_s": gens / dev_s,
            "child_evals_per_s": children / dev_s, "wall_generations_per_s": gens / wall,
            "lds_gather_frac_whole_generation": children / dev_s * G / r_gather}
        best = ga.best()[0]
        del ga
    ctx.set_ga_fused(0)
    out["ga"] = {"workload": "cfg2 CVRP-100, island GA", "islands": islands_, "pop": pop,
                 "kernel": "ga_fused_kernel (breed + score + select per island in LDS)",
                 **ga_out, "speedup_fused": ga_out["fused"]["child_evals_per_s"]
                 / ga_out["three_kernel"]["child_evals_per_s"],
                 "best": {"duration_sum": (best >> 28) & (2**28 - 1), "unvisited": best >> 56}}
    # ACO: 64 colonies x 64 ants (one wavefront per ant), 5 iterations per epoch
    colonies, ants, iters = 64, 64, 5
    aco = runners.ACORunner(ctx, inst.n, colonies=colonies, ants=ants, seed=seed,
                            iters_per_epoch=iters)
    wall, dev_s = timed(aco.epoch, 3)
    # roofline: the roulette reads the weight (tau >> 8) * eta of every free
    # node at every ant step -- n - s of them at step s, n (n + 1) / 2 per
    # ant -- one 8-byte LDS gather each (aco_construct_lds_kernel), against
    # the LDS-gather peaks; timed over the whole iteration (construct +
    # eval_cvrp_words2 scoring + the fused update), so a lower bound for the
    # construct kernel alone (its own time: rocprofv3 stats in profiles/)
    reads = inst.n * (inst.n + 1) // 2
    rd_s = colonies * ants * iters * reads / dev_s
    out["aco"] = {"workload": "cfg2 CVRP-100, integer max-min ACO", "colonies": colonies,
                  "ants": ants, "scoring_kernel": "eval_cvrp_words2",
                  "construct_kernel": "aco_construct_lds_kernel (colony weights staged in LDS)",
                  "iterations_per_s": iters / dev_s, "ant_tours_per_s": colonies * ants * iters / dev_s,
                  "wall_iterations_per_s": iters / wall,
                  "roofline": {"bound": "lds_gather", "weight_reads_per_ant": reads,
                               "achieved": rd_s, "peak": r_gather, "unit": "gathers/s",
                               "frac": rd_s / r_gather if r_gather else None,
                               "frac_vs_guide_peak": rd_s / GUIDE_LDS_GATHER_PEAK,
                               "timed": "whole iteration (construct + scoring + update)"},
                  "best": {"duration_sum": (aco.best()[0] >> 28) & (2**28 - 1)}}
    del aco
    # BF: exhaustive lexicographic ranks on CVRP-n sub-instances (K = 3)
    bf = {}
    for n in (10, 11, 12):
        sub = synth.cvrp(n, 3, seed=seed)
        ctx.set_instance(CVRP, sub.durations, sub.demand, sub.capacities, sub.start_times)
        total = math.factorial(n)
        t0 = time.perf_counter()
        ctx.bf_run(n, 0, total)
        dt = time.perf_counter() - t0
        bf[f"n{n}"] = {"permutations": total, "seconds": dt, "evals_per_s": total / dt}
    out["bf"] = {"workload": "CVRP-n, K = 3, all n! giant tours", **bf}
    return out


def cfg1_leg():
    """BASELINE cfg 1: main.py's two calls (reference main.py:5-6) through the
    drop-in front-end -- calculate_duration("A", "B") (no matrix loaded: the
    reference's stub behaviour) and solve_vrp_problem() (no arguments: the
    15-node instance, solved on the GPU) -- plus a TSP-20 solve per
    algorithm.  The reference stub itself measured 144,054 / 1,541,860
    calls/s on the survey container; it computes no cost."""
    from vrpms_amd import solver, synth
    out = {}
    t0, n = time.perf_counter(), 0
    while time.perf_counter() - t0 < 0.5:
        solver.calculate_duration("A", "B")
        n += 1
    out["calculate_duration_calls_per_s"] = n / (time.perf_counter() - t0)
    solver.solve_vrp_problem(seed=1)                  # warm: code objects, context
    t0, n = time.perf_counter(), 0
    while time.perf_counter() - t0 < 2.0 or n < 3:
        r = solver.solve_vrp_problem(seed=n)
        n += 1
    out["solve_vrp_problem"] = {"calls_per_s": n / (time.perf_counter() - t0),
                                "total_time_last": r["total_time"], "tour_len": len(r["tour"])}
    t = synth.tsp20(0)
    algos = {}
    for algo in ("bf", "ga", "sa", "aco"):
        kw = {"time_limit": None}
        if algo == "bf":
            D = t.durations[0][:12, :12]               # 11 customers: exhaustive
            cust = list(range(1, 12))
        else:
            D, cust = t.durations[0], list(range(1, 20))
        solver.solve_tsp(algo, D, cust, 0, 0, seed=0, **kw)
        t0 = time.perf_counter()
        res = solver.solve_tsp(algo, D, cust, 0, 0, seed=0, **kw)
        algos[algo] = {"seconds": time.perf_counter() - t0, "duration": res["duration"],
                       "customers": len(cust)}
    out["solve_tsp_tsp20"] = algos
    return out


def pmc_traffic(kernel, grid):
    """HBM bytes per launch from the committed PMC pass of this same command
    (profiles/pmc_traffic.json, written by tools/summarize_profiles.py from
    FETCH_SIZE x 2 + WRITE_SIZE), or None when it does not match."""
    p = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    try:
        rec = json.load(open(p))
    except (OSError, ValueError):
        return None
    if kernel in rec.get("kernel", "") and rec.get("grid") == grid:
        return rec["bytes_per_launch"]
    return None


def standin_main(args):
    """The bench's multi-rank control flow on the CPU (gloo): rendezvous from
    the launcher's environment, W untimed steps, K steps bracketed by
    barriers, the max over ranks, rank 0's final line.  A step is a numpy
    TSP tour-cost pass (random 50-node matrix, 4096 random tours) -- a
    rehearsal of the plumbing, not a measurement."""
    import torch.distributed as dist
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    if world > 1:
        dist.init_process_group("gloo", rank=rank, world_size=world)
    rng = np.random.default_rng(args.seed + rank)
    n, C = 50, 4096
    D = rng.integers(1, 100, size=(n, n)).astype(np.int64)
    tours = np.argsort(rng.random((C, n)), axis=1)

    def step():
        return int(D[tours, np.roll(tours, -1, axis=1)].sum())

    for _ in range(args.warmup):
        step()
    if world > 1:
        dist.barrier()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    if world > 1:
        dist.barrier()
    wall = time.perf_counter() - t0
    if world > 1:
        import torch
        t = torch.tensor([wall], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        wall = float(t.item())
    if rank == 0:
        out = {"metric": METRIC, "value": C * args.steps * world / wall, "unit": "evals/s",
               "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
               "ms_per_step": wall * 1e3 / args.steps, "higher_is_better": True,
               "scaling": "weak", "vs_baseline": None, "dtype": "int64",
               "data": "CPU stand-in (launcher rehearsal, not a measurement)",
               "config": {"workload": "cpu_standin_tsp50", "per_rank_batch": C,
                          "parallelism": f"islands{world}"},
               "roofline": {"bound": "none", "achieved": None, "peak": None, "unit": None,
                            "frac": None, "traffic": None}}
        print(final_line(out), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()
    return 0


def main():
    args = parse()
    env_world = os.environ.get("WORLD_SIZE")
    if env_world is None and args.gpus > 1:
        # no launcher: start one fresh process per GPU before anything here
        # touches the GPU (this process never imports torch)
        sys.exit(launch_ranks(args.gpus, sys.argv[1:]))
    if env_world is not None and int(env_world) != args.gpus:
        sys.exit(f"bench.py: WORLD_SIZE={env_world} but --gpus {args.gpus}; "
                 "launch with --nproc-per-node equal to --gpus")
    if args.cpu_standin:
        return standin_main(args)
    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)

    from vrpms_amd import synth
    from vrpms_amd.core import CVRP, Context
    inst = synth.cvrp(100, 8, seed=args.seed)
    ctx = Context(local)
    ctx.set_instance(CVRP, inst.durations, inst.demand, inst.capacities, inst.start_times)
    C, n = args.candidates, inst.n
    perms = make_batch(ctx, C, n, args.seed * 1000 + rank)
    words = ctx.to_words(perms, n)           # word-interleaved layout, resident in HBM
    keys = torch.empty(C, dtype=torch.int64, device=dev)
    keys_rows = torch.empty(C, dtype=torch.int64, device=dev)
    assert ctx.eval_path(perms) == 0, "expected the packed-LDS row kernel"
    stream = torch.cuda.current_stream(dev)

    def timed(fn, steps, warmup, sync_ranks):
        """W untimed steps, then K steps bracketed by barrier + synchronize;
        returns (max-over-ranks wall seconds, mean kernel ms from HIP events
        recorded on the stream the kernels run on)."""
        for _ in range(warmup):
            fn()
        ev0 = torch.cuda.Event(enable_timing=True)
        ev1 = torch.cuda.Event(enable_timing=True)
        torch.cuda.synchronize(dev)
        if sync_ranks:
            dist.barrier()
        torch.cuda.synchronize(dev)
        t0 = time.perf_counter()
        ev0.record(stream)
        for _ in range(steps):
            fn()
        ev1.record(stream)
        torch.cuda.synchronize(dev)
        if sync_ranks:
            dist.barrier()
        torch.cuda.synchronize(dev)
        wall = time.perf_counter() - t0
        if sync_ranks:
            t = torch.tensor([wall], dtype=torch.float64, device=dev)
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            wall = float(t.item())
        return wall, ev0.elapsed_time(ev1) / steps

    progress("headline: eval_cvrp_words2")
    wall, kernel_ms = timed(lambda: ctx.eval_words(words, n, out=keys), args.steps, args.warmup,
                            world > 1)
    value = C * args.steps * world / wall
    rows_wall, rows_ms = timed(lambda: ctx.eval(perms, out=keys_rows), max(3, args.steps // 4),
                               1, False)
    r_gather = ctx.probe_lds_gather(slots=inst.N * inst.N) if rank == 0 else None
    qual = None
    # The quality comparison is an N=1 side measurement: at N>1 the headline
    # stays a collective-free weak-scaling line (island exchange is covered by
    # the gloo tests, tests/test_islands_cpu.py).
    if args.quality_seconds > 0 and world == 1:
        try:
            progress("cfg-2 equal-time SA / GA / ACO")
            qual = quality(ctx, inst, args.quality_seconds, world, rank, dist,
                           with_cpu=(rank == 0 and not args.no_cpu_baseline))
            by = algo_quality(ctx, inst, args.quality_seconds)
            base = qual.get("cpu", qual.get("gpu"))
            for v in by.values():
                if base and v["unvisited"] == 0 and base["unvisited"] == 0:
                    v["gap_vs_host_sa"] = (v["duration_sum"] - base["duration_sum"]) \
                        / base["duration_sum"]
            qual["by_algorithm"] = by
        except Exception:
            qual = {"error": traceback.format_exc(limit=3)}

    xq = tdq = None
    if args.x1000_quality_seconds > 0 and world == 1:
        try:
            progress("X-1000 equal-time cells")
            xq = equal_time_cells(ctx, args.x1000_quality_seconds, dist,
                                  with_cpu=(rank == 0 and not args.no_cpu_baseline),
                                  seeds=tuple(args.x1000_seeds), host_repeats=args.host_repeats)
        except Exception:
            xq = {"error": traceback.format_exc(limit=3)}
    xlong = None
    if args.x1000_long_seconds > 0 and world == 1 and xq is not None and xq.get("cells"):
        try:
            progress("X-1000 long cell")
            won = collections.Counter(c["cpu"]["moves_per_step"] for c in xq["cells"]
                                      if c.get("cpu"))
            hm = min(won, key=lambda m: (-won[m], m)) if won else 32
            xlong = equal_time_cells(ctx, args.x1000_long_seconds, dist,
                                     with_cpu=(rank == 0 and not args.no_cpu_baseline),
                                     seeds=(0,), cpu_moves=(hm,), repeat_host=False)
            xlong["host_rule"] = ("the host move count that won most of the 10-s X-1000 cells "
                                  "(ties: the smaller), one run")
        except Exception:
            xlong = {"error": traceback.format_exc(limit=3)}
    hetq = None
    if args.td_quality_seconds > 0 and world == 1:
        try:
            progress("TD-200 equal-time cells")
            tdq = equal_time_cells(ctx, args.td_quality_seconds, dist,
                                   with_cpu=(rank == 0 and not args.no_cpu_baseline),
                                   instance="tdvrp200", seeds=(0,),
                                   host_repeats=args.host_repeats)
        except Exception:
            tdq = {"error": traceback.format_exc(limit=3)}
        try:
            progress("heterogeneous TD-200 equal-time cells")
            hetq = equal_time_cells(ctx, args.td_quality_seconds, dist,
                                    with_cpu=(rank == 0 and not args.no_cpu_baseline),
                                    instance="tdvrp200_het", seeds=tuple(args.het_seeds),
                                    host_repeats=args.host_repeats)
        except Exception:
            hetq = {"error": traceback.format_exc(limit=3)}

    isl = None
    if args.island_epochs > 0:
        # after every other device use of the matrix instance: it loads its own
        progress("island leg")
        isl = island_leg(ctx, torch, dev, world, rank, dist, epochs=args.island_epochs,
                         steps=args.island_steps)

    if rank == 0:
        cus = torch.cuda.get_device_properties(dev).multi_processor_count
        nbytes = 4 * ((n + 3) // 4)
        bytes_per_launch = C * (nbytes + 8)
        achieved = bytes_per_launch / (kernel_ms * 1e-3) / 1e9
        # north-star roofline: random LDS gathers, G = n + K per eval
        # (the K route-closure legs ride in the same packed
        # entries, so the kernel issues n ds_read_b64 per eval), against
        # R_gather measured by vrpms_probe_lds_gather on this device
        evals_s = C / (kernel_ms * 1e-3)
        G = n + inst.K
        out = {
            "metric": METRIC,
            "value": value,
            "unit": "evals/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": wall * 1e3 / args.steps,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "int32",
            "data": "synthetic (seeded CVRP-100 instance, Philox random giant tours from "
                    "vrpms_random_tours)",
            "config": {"workload": "cvrp100_k8_full_tour_eval", "customers": n, "vehicles": 8,
                       "candidates_per_step": C, "tour_dtype": "u8",
                       "tour_layout": "words [n/4][C] u32 (the layout GA/ACO emit)",
                       "per_rank_batch": C, "parallelism": f"islands{world}"},
            "roofline": {"bound": "lds_gather", "achieved": evals_s * G, "peak": r_gather,
                         "unit": "gathers/s", "frac": evals_s * G / r_gather,
                         "frac_vs_guide_peak": evals_s * G / GUIDE_LDS_GATHER_PEAK,
                         "guide_peak": GUIDE_LDS_GATHER_PEAK,
                         "peak_source": "measured random ds_read_b64 ceiling "
                                        "(vrpms_probe_lds_gather, 1024-lane WGs, 2/CU); the "
                                        "guide's conflict-free ds_read_b64 rate is ~19.7 T/s",
                         "G_per_eval": G, "issued_per_eval": n,
                         "frac_issued": evals_s * n / r_gather,
                         # launch_words2's auto grid: two tours per lane, one
                         # 1024-lane workgroup per CU
                         "traffic": pmc_traffic("eval_cvrp_words2",
                                                min((C + 2047) // 2048, cus) * 1024),
                         "traffic_unit": "HBM bytes/launch (PMC, profiles/pmc_traffic.json)",
                         "kernel": "eval_cvrp_words2", "kernel_ms": kernel_ms},
            "hbm_roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS,
                             "unit": "GB/s", "frac": achieved / HBM_PEAK_GBS,
                             "bytes_per_launch": bytes_per_launch},
            "rows_layout": {"kernel": "eval_cvrp_rows2", "evals_per_s": C / (rows_ms * 1e-3),
                            "kernel_ms": rows_ms,
                            "lds_gather_frac": C / (rows_ms * 1e-3) * G / r_gather},
        }
        import numpy as np
        same = bool(torch.equal(keys, keys_rows))
        out["rows_vs_words_identical"] = same
        if qual is not None:
            out["quality"] = qual
        if xq is not None:
            out["quality_x1000"] = xq
        if xlong is not None:
            out["quality_x1000_long"] = xlong
        if tdq is not None:
            out["quality_tdvrp200"] = tdq
        if hetq is not None:
            out["quality_tdvrp200_het"] = hetq
        if isl is not None:
            out["islands"] = isl
        if world == 1 and not args.no_cpu_baseline:
            progress("cpu baseline")
            cb, ref, S = cpu_baseline(inst, perms, args.cpu_seconds)
            got = keys[:S].cpu().numpy().view(np.uint64)
            cb["parity_on_sample"] = bool((got == ref[0]).all())
            out["cpu_baseline"] = cb
        if world == 1 and not args.no_other_configs:
            del perms, words
            try:   # secondary lines must never cost the headline line
                progress("other configs (cfg 3-5, API legs)")
                out["other_configs"] = other_configs(ctx, torch, dev, r_lds=r_gather)
            except Exception:
                out["other_configs"] = {"error": traceback.format_exc(limit=3)}
            try:
                progress("search lines")
                out["search"] = search_lines(ctx, torch, dev, r_gather)
            except Exception:
                out["search"] = {"error": traceback.format_exc(limit=3)}
            try:
                out["cfg1_main_py"] = cfg1_leg()
            except Exception:
                out["cfg1_main_py"] = {"error": traceback.format_exc(limit=3)}
        out["quality_summary"] = quality_summary(out)
        # details first, one leg per line; the LAST line is the compact record
        # the driver parses (<= FINAL_LINE_MAX bytes)
        for ln in detail_lines(out):
            print(ln, flush=True)
        print(final_line(out), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()
    ctx.close()


if __name__ == "__main__":
    main()
