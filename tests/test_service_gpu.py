"""HTTP host with the GPU solver in the slot: the 8 endpoints answer the
reference's request bodies with real solutions, and saves carry them."""
import json
import os

import pytest

from vrpms_amd import service

from test_service_cpu import FULL, WIRE, call, store

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("algo", ["bf", "ga", "sa", "aco"])
def test_tsp_endpoints_solve(algo):
    st = store()
    h = service.endpoint_handler(service.App(st), "tsp", algo)
    r = call(h, "POST", {**FULL["tsp"], "auth": "jwt"})
    assert r["status_line"] == "HTTP/1.0 200 OK"
    assert r["headers"] == WIRE[f"tsp/{algo}"]["POST_full"]["headers"]
    msg = json.loads(r["body"])["message"]
    # 4-node instance, start 0, customers 1..3: both optimal cycles cost 24
    assert msg["duration"] == 24
    assert msg["vehicle"][0] == msg["vehicle"][-1] == 0
    assert sorted(msg["vehicle"][1:-1]) == [1, 2, 3]
    (row,) = st.solutions
    assert row["duration"] == 24 and row["vehicle"] == msg["vehicle"]
    assert row["owner"] == "tester@example.com"


@pytest.mark.parametrize("algo", ["bf", "ga", "sa", "aco"])
def test_vrp_endpoints_solve(algo):
    st = store()
    h = service.endpoint_handler(service.App(st), "vrp", algo)
    body = {**FULL["vrp"], "auth": "jwt", "ignoredCustomers": [2]}
    r = call(h, "POST", body)
    assert r["status_line"] == "HTTP/1.0 200 OK"
    msg = json.loads(r["body"])["message"]
    assert len(msg["vehicles"]) == 2
    served = sorted(c for v in msg["vehicles"] for c in v["tour"][1:-1])
    assert served == [1, 3]                       # customer 2 ignored
    for v in msg["vehicles"]:
        assert v["tour"][0] == v["tour"][-1] == 0
    assert msg["durationSum"] == sum(v["duration"] for v in msg["vehicles"])
    assert msg["durationMax"] == max(v["duration"] for v in msg["vehicles"])
    # one vehicle serving 1 and 3 from t = 0: 5 + 9 + 7 = 21 is the optimum
    assert msg["durationSum"] == 21
    (row,) = st.solutions
    assert row["locations"] == [{"id": 0}, {"id": 1}, {"id": 3}]
    assert row["vehicles"] == msg["vehicles"] and row["durationSum"] == 21


def test_tsp_batcher_on_gpu():
    """Concurrent /api/tsp/sa requests ride shared tsp_batch_sa launches and
    each gets an optimal tour of the 4-node instance."""
    import threading
    app = service.App(store(), batch_tsp=True, batch_window_s=0.05, batch_steps=200)
    body = json.dumps(FULL["tsp"]).encode()
    out = [None] * 24

    def go(i):
        out[i] = app.post("tsp", "sa", body)

    ths = [threading.Thread(target=go, args=(i,)) for i in range(len(out))]
    for t in ths:
        t.start()
    for t in ths:
        t.join()
    assert 1 <= app.batcher.launches < len(out)
    for status, resp in out:
        assert status == 200
        msg = resp["message"]
        assert msg["duration"] == 24 and sorted(msg["vehicle"][1:-1]) == [1, 2, 3]


@pytest.mark.gpu
def test_frontend_pool_cfg5_api_on_gpu():
    """cfg 5 at the API across processes (vrpms_amd.frontends): forked
    front-end workers + a GPU-owner process running vrpms_tsp_batch_sa.  The
    pool runs as a child program (this test process may already hold the
    GPU); every answer is a 200 and a sample's durations equal their tours'
    closed-tour costs."""
    import json
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    res = subprocess.run([sys.executable, "-m", "vrpms_amd.frontends", "bench", "--requests",
                          "3000", "--workers", "4", "--steps", "300"], cwd=root,
                         capture_output=True, text=True, timeout=240)
    assert res.returncode == 0, res.stderr[-2000:]
    out = json.loads(res.stdout.strip().splitlines()[-1])
    assert out["ok"] == 3000 and out["duration_mismatches"] == 0 and out["duration_checked"] > 0
