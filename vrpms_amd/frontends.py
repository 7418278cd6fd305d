"""Throughput mode at the API (BASELINE.json cfg 5: many concurrent
/api/tsp/sa requests, api/tsp/sa/index.py:40-44) across processes.

One Python process cannot serve cfg 5: the per-request JSON parse, the DB
matrix ingest (a nested list of N^2 JSON integers -> int32) and the response
build all hold the GIL, so one process saturates near 5 k requests/s while
the kernel could answer ~1 M/s.  FrontEndPool splits the work:

  * W front-end WORKER processes (forked before any GPU call; they never
    touch the GPU) run the reference's request contract -- parse, parameter
    checks (api/parameters.py), DB fetch, compaction, save, response -- and
    write each batchable request's compact int32 matrix into a slot of a
    shared-memory arena;
  * one GPU-OWNER process per device (forked before any GPU call, it then
    opens its device) takes slot lists from its queue, coalesces them for a
    short window, stages each node count's matrices straight from the arena
    into one int32 buffer, runs vrpms_tsp_batch_sa (one workgroup per
    request), and writes the tours and durations back into the slots;
  * the workers hand their batches to the owners round-robin (SURVEY.md §8e
    cfg 5: replicas only, no collective), wait for the slots, and answer
    with the response bytes the HTTP handler would write (encoding is part
    of serving, so it runs in parallel in the workers);
  * an owner launches asynchronously (pinned staging, rotating streams) and
    keeps up to two batches on the device while it collects the next; a
    pool whose worker or owner process died raises instead of waiting.

Requests that are not batchable (other endpoints, hour-indexed matrices,
node counts outside the arena) go to an owner's full App.post (the unbatched
GPU path), so every endpoint keeps its contract.  Saved solutions travel
back with the answers and are appended to the parent's store, so a
MemoryStore ends up as it would in one process.

The arena, the queues and the owners are created by the parent before any
of them touches the GPU (`fork`); a process that has already initialised the
GPU (e.g. bench.py) starts this module as a child program instead
(`python -m vrpms_amd.frontends bench ...`).
"""
from __future__ import annotations

import argparse
import json
import multiprocessing as mp
import os
import queue
import sys
import threading
import time

import numpy as np

_STOP = None


class Arena:
    """Shared slots: an int32 [nmax][nmax] matrix and its node count per
    slot, the answer (tour int16 [nmax], duration int64, status int32)."""

    def __init__(self, slots: int, nmax: int):
        from multiprocessing import shared_memory
        self.slots, self.nmax = slots, nmax
        mb = slots * nmax * nmax * 4
        tb = slots * nmax * 2
        self._shm = shared_memory.SharedMemory(create=True, size=mb + tb + slots * 16)
        buf = self._shm.buf
        self.mats = np.ndarray((slots, nmax, nmax), dtype=np.int32, buffer=buf, offset=0)
        self.tours = np.ndarray((slots, nmax), dtype=np.int16, buffer=buf, offset=mb)
        self.dur = np.ndarray((slots,), dtype=np.int64, buffer=buf, offset=mb + tb)
        self.N = np.ndarray((slots,), dtype=np.int32, buffer=buf, offset=mb + tb + slots * 8)
        self.status = np.ndarray((slots,), dtype=np.int32, buffer=buf,
                                 offset=mb + tb + slots * 12)

    def close(self, unlink: bool):
        self.mats = self.tours = self.dur = self.N = self.status = None
        try:
            self._shm.close()
            if unlink:
                self._shm.unlink()
        except (FileNotFoundError, BufferError):
            pass


def gpu_launch(device: int, steps: int, seed: int, streams: int = 3):
    """The owner's default launch: (N, int32 [R][N][N]) -> a finish() that
    returns (tours int16 [R][N-1], durations int64 [R]) once
    vrpms_tsp_batch_sa on `device` has run.  The launch is asynchronous: the
    matrices go up from a pinned buffer and the answers come back into
    pinned buffers on one of `streams` streams (round-robin), so the owner
    stages and launches the next batch while this one runs, and a small
    batch (fewer workgroups than the chip holds) runs beside the previous
    one.  The temperature schedule is scaled to the batch's mean edge (as
    service.TspBatcher)."""
    state = {"k": 0}

    def launch(N, host):
        import torch
        from . import solver
        if "ctx" not in state:
            state["ctx"] = solver.context(device)
            state["streams"] = [torch.cuda.Stream(device=device) for _ in range(streams)]
        ctx = state["ctx"]
        stream = state["streams"][state["k"] % streams]
        state["k"] += 1
        R = host.shape[0]
        nz = host[host > 0]
        edge = float(nz.mean()) if nz.size else 1.0
        inv_t0 = 1.0 / (0.5 * edge)
        inv_alpha = (0.5 / 0.002) ** (1.0 / max(1, steps))
        pin = torch.from_numpy(host).pin_memory()
        tours_h = torch.empty((R, max(N - 1, 1)), dtype=torch.int16, pin_memory=True)
        keys_h = torch.empty(R, dtype=torch.int64, pin_memory=True)
        with torch.cuda.stream(stream):
            mats = pin.to(ctx.dev, non_blocking=True)
            tours, keys = ctx.tsp_batch_sa(mats, steps, inv_t0, inv_alpha, seed)
            tours_h.copy_(tours, non_blocking=True)
            keys_h.copy_(keys, non_blocking=True)
            done = torch.cuda.Event()
            done.record(stream)
        keep = [pin, mats, tours, keys]   # alive until the stream is done with them

        def finish():
            done.synchronize()
            keep.clear()
            t = tours_h.numpy()
            k = keys_h.numpy().view(np.uint64)
            clamp = (1 << 28) - 1
            durs = ((k >> np.uint64(28)) & np.uint64(clamp)).astype(np.int64)
            # a clamped key (2^28 - 1) is summed on the host from the tour
            for x in np.flatnonzero(durs == clamp):
                path = [0] + [int(c) for c in t[x]] + [0]
                durs[x] = int(sum(int(host[x, a, b]) for a, b in zip(path, path[1:])))
            return t, durs
        return finish
    return launch


def _owner_main(dev, arena, submit_q, done_qs, stats_q, make_launch, make_app, window_s,
                max_batch, max_inflight=2):
    """GPU owner of one device: coalesce the workers' slot lists, one launch
    per node count, answers into the arena, then each worker's done queue.
    A launch may return its answers at once or a finish() (asynchronous
    launches): up to `max_inflight` batches are then on the device while the
    next one is collected and staged."""
    from collections import deque
    launch = make_launch(dev)
    app = None
    st = {"device": dev, "batches": 0, "requests": 0, "stage_s": 0.0, "launch_s": 0.0,
          "wait_s": 0.0, "collect_s": 0.0, "max_batch": 0}
    pending = deque()          # (messages, [(group slots, N, answers or finish)])
    stopping = False

    def complete():
        msgs, groups = pending.popleft()
        for grp, N, res in groups:
            try:
                t0 = time.perf_counter()
                tours, durs = res() if callable(res) else res
                st["wait_s"] += time.perf_counter() - t0
                arena.tours[grp, :N - 1] = tours[:, :N - 1]
                arena.dur[grp] = durs
                arena.status[grp] = 0
            except Exception as e:  # noqa: BLE001 -- every waiter of the group sees it
                arena.status[grp] = 1
                sys.stderr.write(f"owner {dev}: launch failed: {e}\n")
        for m in msgs:
            done_qs[m[1]].put(("slots", m[3]))

    while not (stopping and not pending):
        batch = []
        n_slots = 0
        tc = time.perf_counter()
        if not stopping:
            if not pending:              # idle: wait for work, then a short window for company
                msg = submit_q.get()
                batch.append(msg)
                deadline = time.perf_counter() + window_s
            else:                        # busy: take what is queued, no window
                deadline = None
            while True:
                try:
                    if deadline is None:
                        m = submit_q.get_nowait()
                    else:
                        left = deadline - time.perf_counter()
                        if left <= 0:
                            break
                        m = submit_q.get(timeout=left)
                except queue.Empty:
                    break
                batch.append(m)
                if m is not _STOP and m[0] == "slots":
                    n_slots += len(m[2])
                    if n_slots >= max_batch:
                        break
            if batch and batch[0] is _STOP or any(m is _STOP for m in batch):
                stopping = True
                batch = [m for m in batch if m is not _STOP]
        st["collect_s"] += time.perf_counter() - tc
        slot_msgs = [m for m in batch if m[0] == "slots"]
        if slot_msgs:
            sl = np.asarray([x for m in slot_msgs for x in m[2]], dtype=np.int64)
            Ns = arena.N[sl]
            st["batches"] += 1
            st["requests"] += len(sl)
            st["max_batch"] = max(st["max_batch"], len(sl))
            groups = []
            for N in np.unique(Ns):
                grp = sl[Ns == N]
                t1 = time.perf_counter()
                host = np.ascontiguousarray(arena.mats[grp, :N, :N])
                t2 = time.perf_counter()
                try:
                    res = launch(int(N), host)
                except Exception as e:  # noqa: BLE001
                    sys.stderr.write(f"owner {dev}: launch failed: {e}\n")

                    def res(e=e):
                        raise e
                st["stage_s"] += t2 - t1
                st["launch_s"] += time.perf_counter() - t2
                groups.append((grp, int(N), res))
            pending.append((slot_msgs, groups))
        for m in batch:
            if m[0] == "post":           # ("post", worker, token, problem, algorithm, body)
                _, w, token, problem, algorithm, body = m
                if app is None:
                    app = make_app(dev)
                before = len(app.store.solutions)
                status, resp = app.post(problem, algorithm, body)
                rows = list(app.store.solutions[before:])
                del app.store.solutions[before:]
                done_qs[w].put(("post", token, status, resp, rows))
        # answer the oldest batch when the device holds enough, or nothing new came
        while pending and (len(pending) > max_inflight or not slot_msgs or stopping):
            complete()
            if slot_msgs and not stopping:
                break
    stats_q.put(("owner", st))


def _worker_main(w, arena, lo, hi, req_q, resp_q, submit_qs, done_q, store, batchable_nmax,
                 stats_q, inflight=3):
    """Front-end worker: the request contract on the CPU, batchable TSP SA
    requests through the arena and an owner (round-robin over owners).  Up
    to `inflight` jobs at a time: the next chunk is parsed while the owner
    runs the previous one."""
    from . import service, solver
    rr = w % len(submit_qs)
    free = list(range(lo, hi))
    jobs = {}          # token -> job state
    st = {"worker": w, "jobs": 0, "requests": 0, "parse_s": 0.0, "answer_s": 0.0, "idle_s": 0.0}
    stop = False
    token = 0

    def start(job):
        nonlocal rr, token
        t0 = time.perf_counter()
        job_id, problem, algorithm, bodies = job
        out = [None] * len(bodies)
        pending = []   # (index, slot, compact instance, params, locations, db)
        posts = {}
        before = len(store.solutions)
        for i, raw in enumerate(bodies):
            if (problem, algorithm) != ("tsp", "sa"):
                posts[i] = raw
                continue
            text = raw.decode("utf-8") if raw else ""
            try:
                content = json.loads(text) if text else {}
            except ValueError as e:
                out[i] = (400, {"success": False,
                                "errors": [{"what": "Invalid request", "reason": str(e)}]})
                continue
            if not isinstance(content, dict):
                out[i] = (400, {"success": False, "errors": [
                    {"what": "Invalid request", "reason": "the body must be a JSON object"}]})
                continue
            errors = []
            params, _ = service.parse(problem, algorithm, content, errors)
            if errors:
                out[i] = (400, {"success": False, "errors": errors})
                continue
            db = store.session(params["auth"])
            locations = db.get_locations_by_id(params["locations_key"], errors)
            durations = db.get_durations_by_id(params["durations_key"], errors)
            if errors:
                out[i] = (400, {"success": False, "errors": errors})
                continue
            try:
                ci = solver.compact_tsp(durations, params["customers"], params["start_node"],
                                        params["start_time"] or 0)
            except Exception as e:  # noqa: BLE001 -- the unbatched path's error contract
                out[i] = (400, {"success": False,
                                "errors": [{"what": "Solver error", "reason": str(e)}]})
                continue
            if not (service.TspBatcher.accepts(ci) and ci.N <= batchable_nmax) or not free:
                posts[i] = raw
                continue
            s = free.pop()
            N = ci.N
            arena.mats[s, :N, :N] = ci.durations[0]
            arena.N[s] = N
            pending.append((i, s, ci, params, locations, db))
        token += 1
        waiting = (1 if pending else 0) + len(posts)
        jobs[token] = {"id": job_id, "out": out, "pending": pending, "waiting": waiting,
                       "rows": list(store.solutions[before:])}
        del store.solutions[before:]
        if pending:
            submit_qs[rr].put(("slots", w, [p[1] for p in pending], token))
            rr = (rr + 1) % len(submit_qs)
        for i, raw in posts.items():   # the unbatched path on an owner
            submit_qs[rr].put(("post", w, (token, i), problem, algorithm, raw))
            rr = (rr + 1) % len(submit_qs)
        st["jobs"] += 1
        st["requests"] += len(bodies)
        st["parse_s"] += time.perf_counter() - t0
        if waiting == 0:
            finish(token)

    def finish(tk):
        t0 = time.perf_counter()
        j = jobs.pop(tk)
        out = j["out"]
        before = len(store.solutions)
        for i, s, ci, params, locations, db in j["pending"]:
            if arena.status[s] != 0:
                out[i] = (400, {"success": False, "errors": [
                    {"what": "Solver error", "reason": "batched launch failed"}]})
            else:
                N = ci.N
                path = [0] + arena.tours[s, :N - 1].tolist() + [0]
                result = {"duration": int(arena.dur[s]), "vehicle": [ci.nodes[c] for c in path]}
                errors = []
                if params["auth"]:
                    data = {"name": params["name"], "description": params["description"],
                            "duration": result["duration"], "locations": locations,
                            "vehicle": result["vehicle"]}
                    db.save_solution("tsp", data, errors)
                out[i] = (400, {"success": False, "errors": errors}) if errors else \
                    (200, {"success": True, "message": result})
            free.append(s)
        rows = j["rows"] + list(store.solutions[before:])
        del store.solutions[before:]
        # the response bytes as the HTTP handler writes them (service.py
        # do_POST): encoding is part of serving, so it runs here, in parallel
        enc = [(st, json.dumps(body).encode("utf-8")) for st, body in out]
        resp_q.put((j["id"], enc, rows))
        st["answer_s"] += time.perf_counter() - t0

    while not (stop and not jobs):
        if not stop and len(jobs) < inflight:
            try:
                job = req_q.get() if not jobs else req_q.get_nowait()
            except queue.Empty:
                pass            # jobs in flight, none waiting: wait for an answer below
            else:
                if job is _STOP:
                    stop = True
                else:
                    start(job)
                continue
        if not jobs:
            continue
        t0 = time.perf_counter()
        m = done_q.get()
        st["idle_s"] += time.perf_counter() - t0
        if m[0] == "slots":
            tk = m[1]
            jobs[tk]["waiting"] -= 1
        else:                                   # ("post", (token, index), status, resp, rows)
            _, (tk, i), status, resp, saved = m
            jobs[tk]["out"][i] = (status, resp)
            jobs[tk]["rows"] += saved
            jobs[tk]["waiting"] -= 1
        if jobs[tk]["waiting"] == 0:
            finish(tk)
    stats_q.put(("worker", st))


def _default_app(store, seed, steps):
    def make_app(dev):
        from . import service
        return service.App(store, device=dev, seed=seed)
    return make_app


class FrontEndPool:
    """W front-end worker processes + one GPU-owner process per device (see
    the module docstring).  post_many() answers a list of request bodies for
    one endpoint with the (status, response dict) pairs App.post would give."""

    INFLIGHT = 3   # jobs a worker keeps in flight

    def __init__(self, store, workers: int = 16, devices=(0,), steps: int = 1000, seed: int = 0,
                 window_s: float = 0.002, slots_per_worker: int = 1024, nmax: int = 64,
                 chunk: int = 64, max_batch: int = 16384, launch_factory=None, app_factory=None):
        self.store = store
        self.workers, self.devices, self.chunk = int(workers), list(devices), int(chunk)
        if not self.devices or self.workers < 1:
            raise ValueError("FrontEndPool needs at least one worker and one device")
        ctx = mp.get_context("fork")
        # every job a worker has in flight needs its slots (else its requests
        # take the unbatched path)
        slots_per_worker = max(int(slots_per_worker), self.INFLIGHT * self.chunk)
        self.arena = Arena(self.workers * slots_per_worker, nmax)
        self._resp_q = ctx.Queue()
        self._req_qs = [ctx.Queue() for _ in range(self.workers)]
        self._done_qs = [ctx.Queue() for _ in range(self.workers)]
        self._submit_qs = [ctx.Queue() for _ in self.devices]
        self._stats_q = ctx.Queue()
        self.stats = []
        make_launch = launch_factory or (lambda dev: gpu_launch(dev, steps, seed))
        make_app = app_factory or _default_app(store, seed, steps)
        self._procs = []
        for d, dev in enumerate(self.devices):
            p = ctx.Process(target=_owner_main, daemon=True, name=f"vrpms-owner{dev}",
                            args=(dev, self.arena, self._submit_qs[d], self._done_qs,
                                  self._stats_q, make_launch, make_app, window_s, max_batch))
            p.start()
            self._procs.append(p)
        for w in range(self.workers):
            p = ctx.Process(target=_worker_main, daemon=True, name=f"vrpms-front{w}",
                            args=(w, self.arena, w * slots_per_worker, (w + 1) * slots_per_worker,
                                  self._req_qs[w], self._resp_q, self._submit_qs,
                                  self._done_qs[w], store, nmax, self._stats_q, self.INFLIGHT))
            p.start()
            self._procs.append(p)
        self._next_job = 0
        self._lock = threading.Lock()

    def post_many(self, problem: str, algorithm: str, bodies, raw: bool = False):
        """(status, body) per request, in order; chunks go to the workers
        round-robin and are answered as they complete.  The workers send each
        response as the HTTP handler's JSON bytes; raw=True returns those
        bytes, else the decoded dicts (App.post's contract)."""
        with self._lock:
            bodies = list(bodies)
            jobs = {}
            for k, start in enumerate(range(0, len(bodies), self.chunk)):
                jid = self._next_job
                self._next_job += 1
                jobs[jid] = start
                self._req_qs[k % self.workers].put(
                    (jid, problem, algorithm, bodies[start:start + self.chunk]))
            out = [None] * len(bodies)
            for _ in range(len(jobs)):
                while True:   # a worker or owner that died leaves its jobs unanswered: raise
                    try:
                        jid, res, rows = self._resp_q.get(timeout=5.0)
                        break
                    except queue.Empty:
                        dead = [p.name for p in self._procs if not p.is_alive()]
                        if dead:
                            raise RuntimeError(f"FrontEndPool: process(es) {dead} exited; "
                                               f"{len(jobs)} job(s) of this call unanswered")
                s = jobs[jid]
                out[s:s + len(res)] = res if raw else [(st, json.loads(b)) for st, b in res]
                if rows:
                    self.store.solutions.extend(rows)
            return out

    def close(self):
        if any(not p.is_alive() for p in self._procs):   # a process died: no orderly drain
            for p in self._procs:
                if p.is_alive():
                    p.terminate()
                p.join(timeout=10)
            self.arena.close(unlink=True)
            return
        for q in self._req_qs:
            q.put(_STOP)
        for _ in range(self.workers):           # workers drain before the owners stop
            try:
                self.stats.append(self._stats_q.get(timeout=30))
            except queue.Empty:
                break
        for q in self._submit_qs:
            q.put(_STOP)
        for _ in self.devices:
            try:
                self.stats.append(self._stats_q.get(timeout=30))
            except queue.Empty:
                break
        for p in self._procs:
            p.join(timeout=10)
            if p.is_alive():
                p.terminate()
        self.arena.close(unlink=True)

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()


# ---------------------------------------------------------------------------
# cfg 5 at the API, as a child program (bench.py has already initialised the
# GPU, so it starts this module instead of forking itself)
# ---------------------------------------------------------------------------
def bench_api(R: int = 10000, N: int = 50, workers: int = 16, steps: int = 1000, seed: int = 0,
              window_ms: float = 2.0, check: int = 200):
    from . import service, synth
    rng = np.random.default_rng(seed + 5)
    store = service.MemoryStore({0: [{"id": i} for i in range(N)]},
                                {i: synth.random_symmetric(N, rng).tolist() for i in range(R)})
    bodies = [json.dumps({"solutionName": "n", "solutionDescription": "d", "locationsKey": 0,
                          "durationsKey": i, "customers": list(range(1, N)), "startNode": 0,
                          "startTime": 0}).encode() for i in range(R)]
    with FrontEndPool(store, workers=workers, steps=steps, seed=seed,
                      window_s=window_ms * 1e-3) as pool:
        pool.post_many("tsp", "sa", bodies[:2 * workers * pool.chunk])   # warm: GPU context
        t0 = time.perf_counter()
        res = pool.post_many("tsp", "sa", bodies, raw=True)   # the response bytes, as served
        dt = time.perf_counter() - t0
    ok = sum(1 for st, _ in res if st == 200)
    owners = [x for kind, x in pool.stats if kind == "owner"]
    wk = [x for kind, x in pool.stats if kind == "worker"]
    agg = {k: sum(x[k] for x in wk) for k in ("parse_s", "answer_s", "idle_s", "requests")}
    # each sampled answer's duration is its closed tour's cost (A4: a static
    # matrix, start time 0 -- the sum of the tour's edges) and its tour visits
    # every customer once
    bad = 0
    idx = np.random.default_rng(1).choice(R, size=min(check, R), replace=False)
    for i in idx:
        st, body = res[i][0], json.loads(res[i][1])
        D = np.asarray(store.durations[int(i)])
        v = body["message"]["vehicle"] if st == 200 else None
        if v is None or sorted(v[1:-1]) != list(range(1, N)) or v[0] != 0 or v[-1] != 0 or \
                int(D[v[:-1], v[1:]].sum()) != body["message"]["duration"]:
            bad += 1
    return {"workload": f"{R} POST /api/tsp/sa, TSP-{N} each, {workers} front-end processes "
                        f"+ 1 GPU-owner process (vrpms_amd.frontends.FrontEndPool)",
            "requests_per_s": R / dt, "wall_s": dt, "ok": ok, "workers": workers,
            "batch_window_ms": window_ms, "sa_steps_per_chain": steps,
            "duration_checked": int(len(idx)), "duration_mismatches": bad,
            "owners": owners,
            "workers_total": {k: round(v, 4) if isinstance(v, float) else v
                              for k, v in agg.items()},
            "note": "owner/worker times include the warm-up batch"}


def main(argv=None):
    ap = argparse.ArgumentParser(description="cfg-5 API throughput through FrontEndPool")
    ap.add_argument("cmd", choices=["bench"])
    ap.add_argument("--requests", type=int, default=10000)
    ap.add_argument("--workers", type=int, default=16)
    ap.add_argument("--steps", type=int, default=1000)
    ap.add_argument("--window-ms", type=float, default=2.0)
    args = ap.parse_args(argv)
    out = bench_api(R=args.requests, workers=args.workers, steps=args.steps,
                    window_ms=args.window_ms)
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    main()
