"""FrontEndPool (vrpms_amd/frontends.py, cfg 5 at the API across processes)
on the CPU: forked front-end workers feed two stand-in GPU owners ("fake
devices") through the shared-memory arena, round-robin; the answers follow
App.post's contract (api/tsp/sa/index.py) request for request."""
import json
import multiprocessing as mp

import numpy as np
import pytest

from vrpms_amd import frontends, service, synth


def _store(R, N, seed=0):
    rng = np.random.default_rng(seed)
    return service.MemoryStore({0: [{"id": i} for i in range(N)]},
                               {i: synth.random_symmetric(N, rng).tolist() for i in range(R)},
                               {"tok": "a@b.c"})


def _body(i, N, **kw):
    b = {"solutionName": "n", "solutionDescription": "d", "locationsKey": 0, "durationsKey": i,
         "customers": list(range(1, N)), "startNode": 0, "startTime": 0}
    b.update(kw)
    return json.dumps(b).encode()


def _stand_in(counts):
    """Launch factory: the identity tour of each request, its exact
    duration; counts[dev] += requests launched on dev."""
    def factory(dev):
        def launch(N, host):
            with counts.get_lock():
                counts[dev] += host.shape[0]
            R = host.shape[0]
            tours = np.tile(np.arange(1, N, dtype=np.int16), (R, 1))
            path = np.arange(N + 1) % N
            durs = host[:, path[:-1], path[1:]].sum(axis=1).astype(np.int64)
            return tours, durs
        return launch
    return factory


def _fake_app(store):
    def factory(dev):
        def solve(problem, algorithm, params, knobs, locations, durations):
            D = np.asarray(durations)
            n = D.shape[0]
            return {"duration": int(sum(D[i, (i + 1) % n] for i in range(n))),
                    "vehicle": list(range(n)) + [0]}
        return service.App(store, device=dev, solve=solve)
    return factory


def test_pool_round_robin_two_devices_matches_app_contract():
    N, R = 12, 240
    store = _store(R, N)
    counts = mp.get_context("fork").Array("l", 2)
    bodies = [_body(i, N) for i in range(R)]
    bodies[5] = b"{not json"
    bodies[6] = json.dumps({"durationsKey": 1}).encode()           # missing parameters
    bodies[7] = _body(10**6, N)                                    # no such matrix
    bodies[8] = _body(8, N, auth="tok")                            # saved
    bodies[9] = _body(9, N, auth="bad")                            # not permitted
    bodies[10] = _body(10, N, customers=[1, 2, 99])                # outside the matrix
    ref_app = _fake_app(store)(0)
    with frontends.FrontEndPool(store, workers=3, devices=(0, 1), slots_per_worker=32, nmax=16,
                                chunk=16, launch_factory=_stand_in(counts),
                                app_factory=_fake_app(store)) as pool:
        res = pool.post_many("tsp", "sa", bodies)
        # the same requests as the served bytes: the handler's JSON of each body
        raw = pool.post_many("tsp", "sa", bodies[:40], raw=True)
        # another endpoint: not batchable, the owners' App.post
        ga = pool.post_many("tsp", "ga", [_body(3, N)])
    assert len(res) == R
    for i, (st, b) in enumerate(raw):
        assert isinstance(b, bytes) and (st, json.loads(b)) == res[i]
    for i in (5, 6, 7, 9, 10):
        st, body = res[i]
        want = ref_app.post("tsp", "sa", bodies[i]) if i != 10 else None
        assert st == 400 and not body["success"]
        if want is not None:
            assert (st, body) == want, i
    assert "outside" in res[10][1]["errors"][0]["reason"]
    path = list(range(1, N)) + [0]
    for i, (st, body) in enumerate(res):
        if i in (5, 6, 7, 9, 10):
            continue
        assert st == 200, (i, body)
        D = np.asarray(store.durations[i])
        assert body["message"]["vehicle"] == [0] + path
        assert body["message"]["duration"] == int(D[[0] + path[:-1], path].sum())
    # both fake devices launched, the batches split between them
    c = list(counts)
    # 9 is solved, then refused a save; the raw pass solved 40 - 4 again
    assert c[0] > 0 and c[1] > 0 and c[0] + c[1] == R - 4 + 36
    # the auth request's solution reached the parent's store (once per pass)
    assert len(store.solutions) == 2 and store.solutions[0]["owner"] == "a@b.c"
    assert store.solutions[0]["duration"] == res[8][1]["message"]["duration"]
    st, body = ga[0]
    assert st == 200 and body["message"]["vehicle"][0] == 0


def test_pool_rejects_empty_configuration():
    with pytest.raises(ValueError):
        frontends.FrontEndPool(_store(1, 5), workers=0)


def test_pool_raises_when_an_owner_dies():
    """A GPU owner that exits leaves its batches unanswered: post_many raises
    (it does not wait forever) and close() tears the pool down."""
    import os

    def factory(dev):
        def launch(N, host):
            os._exit(3)
        return launch
    N = 8
    store = _store(4, N)
    pool = frontends.FrontEndPool(store, workers=1, devices=(0,), slots_per_worker=8, nmax=16,
                                  chunk=4, launch_factory=factory, app_factory=_fake_app(store))
    try:
        with pytest.raises(RuntimeError, match="exited"):
            pool.post_many("tsp", "sa", [_body(i, N) for i in range(4)])
    finally:
        pool.close()


def test_http_pool_over_sockets_matches_the_handler_contract():
    """listen mode: the workers serve HTTP on one port (SO_REUSEPORT); a
    load-generator process pair holds 64 keep-alive connections and sends
    every request; the answers, the GET banners, the VRP GA preflight, an
    error body, a saved solution and an unbatched endpoint all follow the
    reference handler's contract (service.endpoint_handler)."""
    import http.client
    N, R = 12, 300
    store = _store(R, N)
    counts = mp.get_context("fork").Array("l", 1)
    path = list(range(1, N)) + [0]
    with frontends.FrontEndPool(store, workers=3, devices=(0,), slots_per_worker=64, nmax=16,
                                chunk=16, launch_factory=_stand_in(counts),
                                app_factory=_fake_app(store), listen=("127.0.0.1", 0)) as pool:
        out = frontends.loadgen("127.0.0.1", pool.port, R, N, connections=64, procs=2, sample=R)
        c = http.client.HTTPConnection("127.0.0.1", pool.port, timeout=30)
        c.request("GET", "/api/vrp/ga")
        r = c.getresponse()
        banner = (r.status, r.read())
        c.request("GET", "/api")
        r = c.getresponse()
        hello = (r.status, r.read())
        c.request("OPTIONS", "/api/vrp/ga")
        r = c.getresponse()
        pre = (r.status, r.getheader("Access-Control-Allow-Origin"), r.read())
        c.request("POST", "/api/tsp/sa", body=json.dumps({"durationsKey": 1}))
        r = c.getresponse()
        err = (r.status, r.read())
        c.request("POST", "/api/tsp/sa", body=_body(8, N, auth="tok"))
        r = c.getresponse()
        saved = (r.status, json.loads(r.read()))
        c.request("POST", "/api/tsp/ga", body=_body(3, N))   # unbatched: an owner's App.post
        r = c.getresponse()
        ga = (r.status, json.loads(r.read()))
        c.request("GET", "/nowhere")
        r = c.getresponse()
        missing = r.status
        r.read()
        c.close()
    assert out["requests"] == R and out["ok"] == R and out["errors"] == 0
    assert len(out["sample"]) == R
    for i, (st, text) in out["sample"].items():
        body = json.loads(text)
        D = np.asarray(store.durations[i])
        assert st == 200 and body["message"]["vehicle"] == [0] + path
        assert body["message"]["duration"] == int(D[[0] + path[:-1], path].sum())
        assert text == json.dumps(body)          # the handler's encoding of that result
    assert banner == (200, b"Hi, this is the VRP Genetic Algorithm endpoint")
    assert hello == (200, b"Hello!") and missing == 404
    assert pre[0] == 200 and pre[1] == "*"
    want = _fake_app(store)(0).post("tsp", "sa", json.dumps({"durationsKey": 1}).encode())
    assert err == (400, json.dumps(want[1]).encode())
    assert saved[0] == 200 and len(store.solutions) == 1
    assert store.solutions[0]["duration"] == saved[1]["message"]["duration"]
    assert ga[0] == 200 and ga[1]["message"]["vehicle"][0] == 0
    assert counts[0] == R + 1


def test_pool_unbatched_post_does_not_block_batches():
    """A slow unbatched request (another endpoint) runs on the owner's post
    thread: batched TSP SA answers keep arriving meanwhile."""
    import http.client
    import threading
    import time
    N = 10
    store = _store(64, N)
    counts = mp.get_context("fork").Array("l", 1)

    def slow_app(st):
        def factory(dev):
            def solve(problem, algorithm, params, knobs, locations, durations):
                time.sleep(6.0)
                return {"duration": 0, "vehicle": [0, 0]}
            return service.App(st, device=dev, solve=solve)
        return factory

    with frontends.FrontEndPool(store, workers=2, devices=(0,), slots_per_worker=64, nmax=16,
                                chunk=8, launch_factory=_stand_in(counts),
                                app_factory=slow_app(store), listen=("127.0.0.1", 0)) as pool:
        slow = {}

        def post_slow():
            c = http.client.HTTPConnection("127.0.0.1", pool.port, timeout=30)
            c.request("POST", "/api/tsp/ga", body=_body(1, N))
            r = c.getresponse()
            slow["r"] = (r.status, r.read(), time.perf_counter())
            c.close()

        th = threading.Thread(target=post_slow)
        th.start()
        time.sleep(0.3)
        out = frontends.loadgen("127.0.0.1", pool.port, 64, N, connections=8, procs=1, sample=0)
        t_done = time.perf_counter()
        th.join()
    assert out["ok"] == 64
    assert t_done < slow["r"][2], "batched answers waited for the slow request"
    assert slow["r"][0] == 200


def test_pool_refuses_calls_after_a_death():
    """post_many after a failure raises at once (the pool is marked broken)."""
    import os

    def factory(dev):
        def launch(N, host):
            os._exit(3)
        return launch
    N = 8
    store = _store(4, N)
    pool = frontends.FrontEndPool(store, workers=1, devices=(0,), slots_per_worker=8, nmax=16,
                                  chunk=4, launch_factory=factory, app_factory=_fake_app(store))
    try:
        with pytest.raises(RuntimeError, match="exited"):
            pool.post_many("tsp", "sa", [_body(i, N) for i in range(4)])
        with pytest.raises(RuntimeError, match="broken"):
            pool.post_many("tsp", "sa", [_body(0, N)])
    finally:
        pool.close()


def _raw_http(port, data, timeout=10):
    """Send raw bytes, return everything the server writes before closing."""
    import socket
    s = socket.create_connection(("127.0.0.1", port), timeout=timeout)
    s.sendall(data)
    out = b""
    try:
        while True:
            b = s.recv(65536)
            if not b:
                break
            out += b
    except socket.timeout:
        pass
    s.close()
    return out


def test_http_pool_bounds_content_length_and_serves_solve():
    """a negative or unparsable Content-Length is a 400 and an
    oversized one a 413, each closing the connection; two pipelined requests
    on one connection are both answered, in order; POST /solve/<p>/<a> (the
    remote front-end's route) reaches an owner's App.solve_inline."""
    N = 10
    store = _store(8, N)
    counts = mp.get_context("fork").Array("l", 1)
    with frontends.FrontEndPool(store, workers=1, devices=(0,), slots_per_worker=64, nmax=16,
                                chunk=8, launch_factory=_stand_in(counts),
                                app_factory=_fake_app(store), listen=("127.0.0.1", 0)) as pool:
        neg = _raw_http(pool.port, b"POST /api/tsp/sa HTTP/1.1\r\nContent-Length: -5\r\n\r\n")
        bad = _raw_http(pool.port, b"POST /api/tsp/sa HTTP/1.1\r\nContent-Length: x\r\n\r\n")
        big = _raw_http(pool.port, b"POST /api/tsp/sa HTTP/1.1\r\nContent-Length: %d\r\n\r\n"
                        % (frontends.MAX_BODY + 1))
        b1, b2 = _body(1, N), _body(2, N)
        piped = _raw_http(pool.port, b"POST /api/tsp/sa HTTP/1.1\r\nContent-Length: %d\r\n\r\n"
                          % len(b1) + b1 + b"POST /api/tsp/sa HTTP/1.1\r\nConnection: close\r\n"
                          b"Content-Length: %d\r\n\r\n" % len(b2) + b2, timeout=30)
        D = synth.random_symmetric(N, np.random.default_rng(3)).tolist()
        inline = json.dumps({"durations": D, "customers": list(range(1, N)), "startNode": 0,
                             "startTime": 0}).encode()
        solve = _raw_http(pool.port, b"POST /solve/tsp/sa HTTP/1.1\r\nConnection: close\r\n"
                          b"Content-Length: %d\r\n\r\n" % len(inline) + inline, timeout=30)
    assert neg.startswith(b"HTTP/1.1 400") and b"Connection: close" in neg
    assert bad.startswith(b"HTTP/1.1 400")
    assert big.startswith(b"HTTP/1.1 413")
    assert piped.count(b"HTTP/1.1 200") == 2
    bodies = [json.loads(x.split(b"\r\n\r\n", 1)[1]) for x in piped.split(b"HTTP/1.1 ")[1:]]
    for i, body in zip((1, 2), bodies):
        Di = np.asarray(store.durations[i])
        path = list(range(1, N)) + [0]
        assert body["message"]["duration"] == int(Di[[0] + path[:-1], path].sum())
    assert solve.startswith(b"HTTP/1.1 200"), solve[:300]
    want = _fake_app(store)(0).solve_inline("tsp", "sa", inline)
    assert json.loads(solve.split(b"\r\n\r\n", 1)[1]) == want[1]
