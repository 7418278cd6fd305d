"""HTTP host (vrpms_amd/service.py) against the reference's wire contract.

Every byte the reference's handlers emit without running an algorithm --
GET banners, the VRP GA preflight, missing-parameter and missing-record
error lists, the zero-result responses and the save payload -- is pinned by
tests/golden/reference_fixtures.json (captured from the reference's own
handler classes).  The solver is injected here (the zero result the
reference's TODO slot returns); tests/test_service_gpu.py runs the real one.
"""
import io
import json
import os
import threading
import urllib.error
import urllib.request

import pytest

from vrpms_amd import service

FX = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "reference_fixtures.json")))
WIRE = FX["wire"]
ENDPOINTS = sorted(WIRE)

FULL = {
    "vrp": {"solutionName": "n", "solutionDescription": "d", "locationsKey": 1,
            "durationsKey": 2, "capacities": [5, 5], "startTimes": [0, 30],
            "ignoredCustomers": [], "completedCustomers": [], "multiThreaded": False,
            "randomPermutationCount": 10, "iterationCount": 5},
    "tsp": {"solutionName": "n", "solutionDescription": "d", "locationsKey": 1,
            "durationsKey": 2, "customers": [1, 2, 3], "startNode": 0, "startTime": 0},
}
MATRIX = [[0, 5, 6, 7], [5, 0, 8, 9], [6, 8, 0, 4], [7, 9, 4, 0]]


def store():
    return service.MemoryStore({1: [{"id": i} for i in range(4)]}, {2: MATRIX},
                               {"jwt": "tester@example.com"})


def zero_solve(problem, algorithm, params, knobs, locations, durations):
    """The reference's TODO-slot result."""
    if problem == "tsp":
        return {"duration": 0, "vehicle": []}
    return {"durationMax": 0, "durationSum": 0, "vehicles": []}


def call(handler_cls, method, body=None, raw=None):
    """Drive one request through a handler class without a socket (the same
    harness tests/golden/gen_reference_fixtures.py used on the reference)."""
    h = handler_cls.__new__(handler_cls)
    data = raw if raw is not None else (json.dumps(body).encode() if body is not None else b"")
    h.rfile = io.BytesIO(data)
    h.wfile = io.BytesIO()
    h.headers = {"Content-Length": str(len(data))}
    h.request_version = "HTTP/1.0"
    h.requestline = f"{method} / HTTP/1.0"
    h.command = method
    h.client_address = ("127.0.0.1", 0)
    getattr(h, "do_" + method)()
    text = h.wfile.getvalue().decode()
    head, _, payload = text.partition("\r\n\r\n")
    lines = head.split("\r\n")
    headers = [ln for ln in lines[1:] if not ln.startswith(("Date:", "Server:"))]
    return {"status_line": lines[0], "headers": headers, "body": payload}


def handler(ep, app=None):
    problem, algorithm = ep.split("/")
    return service.endpoint_handler(app or service.App(store(), solve=zero_solve),
                                    problem, algorithm)


@pytest.mark.parametrize("ep", ENDPOINTS)
def test_get_banner_and_preflight(ep):
    h = handler(ep)
    assert call(h, "GET") == WIRE[ep]["GET"]
    if "OPTIONS" in WIRE[ep]:
        assert call(h, "OPTIONS") == WIRE[ep]["OPTIONS"]
    else:
        assert not hasattr(h, "do_OPTIONS")


@pytest.mark.parametrize("ep", ENDPOINTS)
def test_post_errors_and_zero_results(ep):
    h = handler(ep)
    body = FULL[ep.split("/")[0]]
    assert call(h, "POST", {}) == WIRE[ep]["POST_empty"]
    assert call(h, "POST", {**body, "durationsKey": 99}) == WIRE[ep]["POST_missing_db"]
    assert call(h, "POST", body) == WIRE[ep]["POST_full"]


@pytest.mark.parametrize("ep", ENDPOINTS)
def test_post_auth_saves_the_reference_payload(ep):
    st = store()
    h = handler(ep, service.App(st, solve=zero_solve))
    problem = ep.split("/")[0]
    body = {**FULL[problem], "auth": "jwt"}
    if problem == "vrp":
        body["ignoredCustomers"] = [2]
    assert call(h, "POST", body) == WIRE[ep]["POST_auth"]
    assert [{"table": "solutions", "data": row} for row in st.solutions] == \
        WIRE[ep]["POST_auth_insert"]


@pytest.mark.parametrize("problem", ["vrp", "tsp"])
def test_save_with_unknown_token_is_not_permitted(problem):
    st = store()
    h = handler(f"{problem}/sa", service.App(st, solve=zero_solve))
    r = call(h, "POST", {**FULL[problem], "auth": "expired"})
    assert r["status_line"] == "HTTP/1.0 400 Bad Request"
    err = json.loads(r["body"])["errors"]
    assert err[0]["what"] == "Not permitted" and st.solutions == []


def test_missing_locations_and_durations_both_reported():
    r = call(handler("vrp/ga"), "POST", {**FULL["vrp"], "locationsKey": 7, "durationsKey": 8})
    errs = json.loads(r["body"])["errors"]
    assert [e["reason"].split(".")[0] for e in errs] == [
        "No location set found with given id 7", "No duration matrix found with given id 8"]


def test_invalid_json_and_non_object_bodies():
    h = handler("tsp/ga")
    for raw in (b"{not json", b"[1, 2]"):
        r = call(h, "POST", raw=raw)
        assert r["status_line"] == "HTTP/1.0 400 Bad Request"
        assert json.loads(r["body"])["errors"][0]["what"] == "Invalid request"


def test_solver_errors_become_400():
    def boom(*a):
        raise ValueError("3 locations but a 4-node duration matrix")
    r = call(handler("vrp/bf", service.App(store(), solve=boom)), "POST", FULL["vrp"])
    assert r["status_line"] == "HTTP/1.0 400 Bad Request"
    assert json.loads(r["body"])["errors"] == [
        {"what": "Solver error", "reason": "3 locations but a 4-node duration matrix"}]


def test_gpu_solver_without_gpu_fails_loudly():
    import torch
    if torch.cuda.is_available():
        pytest.skip("GPU present: covered by tests/test_service_gpu.py")
    r = call(handler("tsp/sa", service.App(store())), "POST", FULL["tsp"])
    assert r["status_line"] == "HTTP/1.0 400 Bad Request"
    err = json.loads(r["body"])["errors"][0]
    assert err["what"] == "Solver error" and "GPU" in err["reason"]


def test_parse_matches_reference_parsers():
    names = {("vrp", None): "parse_common_vrp_parameters", ("vrp", "ga"): "parse_vrp_ga_parameters",
             ("vrp", "sa"): "parse_vrp_sa_parameters", ("vrp", "aco"): "parse_vrp_aco_parameters",
             ("tsp", None): "parse_common_tsp_parameters", ("tsp", "ga"): "parse_tsp_ga_parameters",
             ("tsp", "sa"): "parse_tsp_sa_parameters", ("tsp", "aco"): "parse_tsp_aco_parameters"}
    for (problem, algo), name in names.items():
        for label, case in FX["parse"][name].items():
            body = {"empty": {}, "vrp_full": FULL["vrp"], "tsp_full": FULL["tsp"],
                    "falsy": {k: 0 for k in FULL["vrp"]}}[label]
            errors = []
            common, knobs = service.parse(problem, algo or "bf", dict(body), errors)
            got = common if algo is None else knobs
            want_err = case["errors"] if algo is None else case["errors"]
            assert got == case["params"], (name, label)
            if algo is None:
                assert errors[:len(want_err)] == want_err, (name, label)


def test_memory_store_json_roundtrip(tmp_path):
    p = tmp_path / "db.json"
    p.write_text(json.dumps({"locations": {"1": [{"id": 0}]}, "durations": {"2": [[0]]},
                             "users": {"t": "a@b"}}))
    st = service.MemoryStore.from_json(str(p))
    s = st.session("t")
    errs = []
    assert s.get_locations_by_id(1, errs) == [{"id": 0}]
    assert s.get_durations_by_id("2", errs) == [[0]]
    assert s.get_durations_by_id([1], errs) is None and len(errs) == 1


def test_router_over_http():
    srv = service.serve(service.App(store(), solve=zero_solve), "127.0.0.1", 0)
    port = srv.server_address[1]
    th = threading.Thread(target=srv.serve_forever, daemon=True)
    th.start()
    opener = urllib.request.build_opener(urllib.request.ProxyHandler({}))
    base = f"http://127.0.0.1:{port}"
    try:
        assert opener.open(base + "/api").read() == b"Hello!"
        assert opener.open(base + "/api/vrp/aco").read() == \
            WIRE["vrp/aco"]["GET"]["body"].encode()
        req = urllib.request.Request(base + "/api/tsp/ga", data=json.dumps(FULL["tsp"]).encode(),
                                     headers={"Content-Type": "application/json"})
        assert json.loads(opener.open(req).read()) == json.loads(WIRE["tsp/ga"]["POST_full"]["body"])
        with pytest.raises(urllib.error.HTTPError) as e:
            opener.open(base + "/api/nope")
        assert e.value.code == 404
    finally:
        srv.shutdown()
        srv.server_close()


def test_tsp_batcher_coalesces_and_groups_by_node_count():
    """Throughput mode: concurrent /api/tsp/sa requests share launches
    (grouped by node count); each gets its own tour back.  The launch is
    injected (the identity tour); the GPU one is in test_service_gpu.py."""
    calls = []

    def fake_launch(N, cis):
        calls.append((N, len(cis)))
        return [list(range(1, N)) for _ in cis]

    st = service.MemoryStore({1: [{"id": i} for i in range(6)]},
                             {2: [[abs(i - j) * 3 for j in range(6)] for i in range(6)]})
    app = service.App(st, solve=zero_solve, batch_tsp=True, batch_window_s=0.05,
                      batch_launch=fake_launch)
    bodies = [{**FULL["tsp"], "customers": [1, 2, 3]}] * 6 + \
             [{**FULL["tsp"], "customers": [1, 2, 3, 4, 5]}] * 4
    out = [None] * len(bodies)

    def go(i):
        out[i] = app.post("tsp", "sa", json.dumps(bodies[i]).encode())

    ths = [threading.Thread(target=go, args=(i,)) for i in range(len(bodies))]
    for t in ths:
        t.start()
    for t in ths:
        t.join()
    assert sorted(calls) == [(4, 6), (6, 4)] and app.batcher.launches == 2
    for (status, body), b in zip(out, bodies):
        assert status == 200
        k = len(b["customers"])
        assert body["message"]["vehicle"] == [0] + list(range(1, k + 1)) + [0]
        assert body["message"]["duration"] == 3 * k + 3 * k     # out and back along a line
    # other algorithms never ride the batcher
    status, body = app.post("tsp", "ga", json.dumps(bodies[0]).encode())
    assert status == 200 and app.batcher.launches == 2


def test_remote_front_end_over_http(monkeypatch):
    """A host without a GPU (VRPMS_REMOTE set) sends solve_tsp / solve_vrp /
    solve_vrp_problem to the GPU box's HTTP host (POST /solve/...) with the
    instance inline; here the box's solver slot is a stand-in that records
    the compact request, so the wire path is checked on CPU."""
    import threading

    from vrpms_amd import remote, solver

    seen = []

    def fake_solve(problem, algorithm, params, knobs, locations, durations):
        assert knobs.get("device") == 0      # the app's one device
        knobs = {k: v for k, v in knobs.items() if k != "device"}
        seen.append((problem, algorithm, params, knobs, locations, durations))
        if problem == "tsp":
            return {"duration": 24, "vehicle": [0, 1, 2, 3, 0]}
        return {"durationMax": 21, "durationSum": 21,
                "vehicles": [{"tour": [0, 1, 3, 0], "duration": 21}, {"tour": [0, 0], "duration": 0}]}

    srv = service.serve(service.App(store(), solve=fake_solve), "127.0.0.1", 0)
    th = threading.Thread(target=srv.serve_forever, daemon=True)
    th.start()
    try:
        monkeypatch.setenv("VRPMS_REMOTE", f"http://127.0.0.1:{srv.server_address[1]}")
        r = solver.solve_tsp("sa", MATRIX, [1, 2, 3], 0, 0)
        assert r == {"duration": 24, "vehicle": [0, 1, 2, 3, 0]}
        assert seen[-1][:3] == ("tsp", "sa", {"customers": [1, 2, 3], "start_node": 0,
                                              "start_time": 0})
        assert seen[-1][5] == MATRIX
        locs = [{"id": i} for i in range(4)]
        v = solver.solve_vrp("ga", MATRIX, locs, [5, 5], [0, 30], [2], [],
                             random_permutation_count=10, iteration_count=5)
        assert v["durationSum"] == 21
        assert seen[-1][3] == {"random_permutationCount": 10, "iteration_count": 5, "seed": 0,
                               "objective": "sum", "inline": {}}
        assert seen[-1][2]["ignored_customers"] == [2]
        # objective, seed and time limit travel with the instance
        solver.solve_vrp("sa", MATRIX, locs, [5, 5], [0, 30], [], [], seed=3, objective="max",
                         time_limit=2.5)
        assert seen[-1][3] == {"random_permutationCount": None, "iteration_count": None,
                               "seed": 3, "time_limit": 2.5, "objective": "max", "inline": {}}
        solver.solve_tsp("sa", MATRIX, [1, 2, 3], 0, 0, seed=5)
        assert seen[-1][3] == {"seed": 5, "inline": {}}
        # the search knobs a local call takes travel too (the same
        # call is accepted with or without a local GPU)
        solver.solve_vrp("sa", MATRIX, locs, [5, 5], [0, 30], [], [], chains=64, window=8)
        assert seen[-1][3]["inline"] == {"chains": 64, "window": 8}
        solver.solve_tsp("ga", MATRIX, [1, 2, 3], 0, 0, pop=32, islands=2)
        assert seen[-1][3]["inline"] == {"pop": 32, "islands": 2}
        # an argument no solver takes is refused, not dropped
        with pytest.raises(ValueError, match="unknown"):
            solver.solve_vrp("sa", MATRIX, locs, [5, 5], [0, 30], [], [], chainz=64)
        st, body = service.App(store(), solve=fake_solve).solve_inline(
            "tsp", "sa", json.dumps({"durations": MATRIX, "customers": [1], "startNode": 0,
                                     "startTime": 0, "knobs": {"bogus": 1}}).encode())
        assert st == 400 and "unknown knob" in body["errors"][0]["reason"]
        p = solver.solve_vrp_problem(MATRIX, locs, [5, 5], [0, 30], [2], [])
        assert p["tour"] == [0, 1, 3, 0] and p["total_time"] == 21 and p["unvisited"] == []
        with pytest.raises(ValueError, match="Invalid request"):
            remote._post(f"http://127.0.0.1:{srv.server_address[1]}", "tsp", "tabu", {},
                                10)
    finally:
        srv.shutdown()
        srv.server_close()


def test_multi_device_scheduling_and_batcher_round_robin():
    """App(devices=[0, 1]): small requests take a free device each, a large
    SA request takes both (the island model), and TspBatcher launches go to
    the devices round-robin (replicas only); stand-ins record where they ran."""
    import threading
    import time

    seen = []
    gate = threading.Event()

    def fake_solve(problem, algorithm, params, knobs, locations, durations):
        seen.append((algorithm, knobs.get("device"), knobs.get("devices")))
        if algorithm == "ga":
            gate.wait(5)      # hold the first device while the next request arrives
        return {"duration": 1, "vehicle": [0, 1, 0]}

    launched = []

    def fake_launch(N, cis, device):
        launched.append((device, len(cis)))
        return [list(range(1, N)) for _ in cis]

    app = service.App(store(), devices=[0, 1], solve=fake_solve, island_min_n=3,
                      batch_tsp=True, batch_window_s=0.001, batch_launch=fake_launch)
    body = json.dumps(FULL["tsp"]).encode()
    th = threading.Thread(target=app.post, args=("tsp", "ga", body))
    th.start()
    time.sleep(0.2)
    app.post("tsp", "aco", body)               # device 0 is busy: device 1
    gate.set()
    th.join()
    assert seen[0] == ("ga", 0, None) and seen[1] == ("aco", 1, None)
    big = dict(FULL["tsp"], customers=[1, 2, 3, 1])   # 4 > island_min_n customers
    app.post("tsp", "bf", json.dumps(big).encode())    # brute force: one device
    app.post("tsp", "ga", json.dumps(big).encode())    # both: islands
    assert seen[2][2] is None and seen[3][2] == [0, 1]
    # the batcher alternates devices launch by launch
    for _ in range(4):
        st, b = app.post("tsp", "sa", body)
        assert st == 200
    assert [d for d, _ in launched] == [0, 1, 0, 1]
    assert app.batcher.per_device == {0: 2, 1: 2}


def test_repeated_device_list_does_not_deadlock():
    """devices=[0, 0] (one GPU standing in for two, as the GPU island test
    does): a large request takes the island path and returns instead of
    blocking on the second acquire of device 0's lock."""
    seen = []

    def fake_solve(problem, algorithm, params, knobs, locations, durations):
        seen.append(knobs.get("devices"))
        return {"duration": 1, "vehicle": [0, 1, 0]}

    app = service.App(store(), devices=[0, 0], solve=fake_solve, island_min_n=2)
    big = dict(FULL["tsp"], customers=[1, 2, 3])
    out = {}
    th = threading.Thread(target=lambda: out.setdefault("r", app.post("tsp", "ga",
                                                                      json.dumps(big).encode())))
    th.start()
    th.join(10)
    assert not th.is_alive(), "island request deadlocked on a repeated device"
    assert out["r"][0] == 200 and seen == [[0, 0]]
    assert all(not lk.locked() for lk in app.locks.values())


@pytest.mark.parametrize("mt,want", [(True, [0, 1]), (False, None), ("false", None),
                                     ("0", None), (0, None), ("TRUE", [0, 1]), (1, [0, 1]),
                                     # not a boolean: the size rule (3 customers: one device)
                                     ("maybe", None), ([1], None)])
def test_multithreaded_selects_island_model(mt, want):
    """VRP GA's multiThreaded (api/parameters.py:20): true runs the island
    model over every device, false one device -- whatever the request size
    (island_min_n is far above this 3-customer request)."""
    seen = []

    def fake_solve(problem, algorithm, params, knobs, locations, durations):
        seen.append(knobs.get("devices"))
        return {"durationMax": 0, "durationSum": 0, "vehicles": []}

    app = service.App(store(), devices=[0, 1], solve=fake_solve, island_min_n=1000)
    st, _ = app.post("vrp", "ga", json.dumps(dict(FULL["vrp"], multiThreaded=mt)).encode())
    assert st == 200 and seen == [want]


def test_bench_quality_summary_collects_every_cell():
    """bench.quality_summary: [gpu, host, gap %] per cell, medians and the
    host spread, from a bench record (CPU: a synthetic record)."""
    import importlib.util
    spec_ = importlib.util.spec_from_file_location(
        "bench_mod", os.path.join(os.path.dirname(os.path.dirname(__file__)), "bench.py"))
    bench = importlib.util.module_from_spec(spec_)
    spec_.loader.exec_module(bench)
    cell = lambda sd, g, c: {"seed": sd, "gpu": {"duration_sum": g}, "cpu": {"duration_sum": c},  # noqa: E731
                             "gap": (g - c) / c}
    out = {"quality": {"gpu": {"duration_sum": 100}, "cpu": {"duration_sum": 101}, "gap": -1 / 101,
                       "by_algorithm": {"ga": {"duration_sum": 102, "gap_vs_host_sa": 1 / 101}}},
           "quality_x1000": {"cells": [cell(0, 99, 100), cell(1, 98, 100)], "gap_median": -0.015,
                             "gpu_better": "2 / 2",
                             "host_run_to_run": {"runs": [100, 101, 100], "min": 100, "max": 101,
                                                 "rel": 0.01},
                             "median_beyond_spread": True},
           "quality_x1000_long": {"cells": [cell(0, 97, 100)], "gap_median": -0.03,
                                  "gpu_better": "1 / 1"},
           "quality_tdvrp200_het": {"cells": [cell(0, 95, 100)], "gap_median": -0.05}}
    s = bench.quality_summary(out)
    assert s["x1000_long_s0"] == [97, 100, -3.0] and s["x1000_long_gpu_better"] == "1 / 1"
    assert s["cfg2_sa"] == [100, 101, -0.99] and s["cfg2_ga"][2] == 0.99
    assert s["x1000_s0"] == [99, 100, -1.0] and s["x1000_median"] == -1.5
    assert s["x1000_host_spread"]["min"] == 100 and s["x1000_median_beyond_spread"] is True
    assert s["td200het_s0"] == [95, 100, -5.0]
    assert list(out) != [] and "units" in s


@pytest.mark.parametrize("knob,value", [("islands", 10**6), ("ants", 10**7), ("chains", 2**30),
                                        ("pop", 1), ("steps", 0), ("window", -1),
                                        ("window_types", 8), ("chains", True), ("pop", [4])])
def test_inline_knobs_out_of_range_are_400(knob, value):
    """/solve knobs from the network are range-checked (a 400,
    never an allocation); in-range values pass through as ints."""
    seen = []

    def fake_solve(problem, algorithm, params, knobs, locations, durations):
        seen.append(knobs.get("inline"))
        return {"duration": 1, "vehicle": [0, 1, 0]}

    app = service.App(store(), solve=fake_solve)
    body = {"durations": MATRIX, "customers": [1], "startNode": 0, "startTime": 0}
    st, res = app.solve_inline("tsp", "sa", json.dumps(dict(body, knobs={knob: value})).encode())
    assert st == 400 and knob in res["errors"][0]["reason"] and not seen
    st, _ = app.solve_inline("tsp", "sa", json.dumps(dict(body, knobs={knob: 7})).encode())
    assert st == 200 and seen == [{knob: 7}]
