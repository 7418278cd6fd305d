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
import asyncio
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
    app = {"app": None}
    st = {"device": dev, "batches": 0, "requests": 0, "stage_s": 0.0, "launch_s": 0.0,
          "wait_s": 0.0, "collect_s": 0.0, "max_batch": 0}
    pending = deque()          # (messages, [(group slots, N, answers or finish)])
    stopping = False
    # unbatched requests (other endpoints, unbatchable TSP SA) run App.post on
    # a thread of their own: one can take seconds, and the loop below must
    # keep collecting and answering batches meanwhile
    post_q = queue.Queue()

    def poster():
        while True:
            m = post_q.get()
            if m is _STOP:
                return
            _, w, token, problem, algorithm, body = m
            if app["app"] is None:
                app["app"] = make_app(dev)
            a = app["app"]
            before = len(a.store.solutions)
            if problem.startswith("solve:"):    # POST /solve/<problem>/<algo> (vrpms_amd.remote)
                status, resp = a.solve_inline(problem[6:], algorithm, body)
            else:
                status, resp = a.post(problem, algorithm, body)
            rows = list(a.store.solutions[before:])
            del a.store.solutions[before:]
            done_qs[w].put(("post", token, status, resp, rows))

    post_th = threading.Thread(target=poster, daemon=True)
    post_th.start()

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
                post_q.put(m)
        # answer the oldest batch when the device holds enough, or nothing new came
        while pending and (len(pending) > max_inflight or not slot_msgs or stopping):
            complete()
            if slot_msgs and not stopping:
                break
    post_q.put(_STOP)
    post_th.join()
    stats_q.put(("owner", st))


class _FrontEnd:
    """One worker's request machinery: the request contract on the CPU,
    batchable TSP SA requests through the arena and an owner (round-robin
    over owners), everything else as an unbatched post on an owner.  A job is
    a list of request bodies for one endpoint; `deliver(job_id, responses,
    saved_rows)` receives its answers, each as (status, the response bytes
    the HTTP handler writes)."""

    def __init__(self, w, arena, lo, hi, submit_qs, store, batchable_nmax, deliver):
        self.w, self.arena, self.submit_qs, self.store = w, arena, submit_qs, store
        self.nmax, self.deliver = batchable_nmax, deliver
        self.rr = w % len(submit_qs)
        self.free = list(range(lo, hi))
        self.jobs = {}          # token -> job state
        self.token = 0
        self.st = {"worker": w, "jobs": 0, "requests": 0, "parse_s": 0.0, "answer_s": 0.0,
                   "idle_s": 0.0}

    def start(self, job):
        from . import service, solver
        t0 = time.perf_counter()
        job_id, problem, algorithm, bodies = job
        store, arena = self.store, self.arena
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
            if not (service.TspBatcher.accepts(ci) and ci.N <= self.nmax) or not self.free:
                posts[i] = raw
                continue
            s = self.free.pop()
            N = ci.N
            arena.mats[s, :N, :N] = ci.durations[0]
            arena.N[s] = N
            pending.append((i, s, ci, params, locations, db))
        self.token += 1
        token = self.token
        waiting = (1 if pending else 0) + len(posts)
        self.jobs[token] = {"id": job_id, "out": out, "pending": pending, "waiting": waiting,
                            "rows": list(store.solutions[before:])}
        del store.solutions[before:]
        nq = len(self.submit_qs)
        if pending:
            self.submit_qs[self.rr].put(("slots", self.w, [p[1] for p in pending], token))
            self.rr = (self.rr + 1) % nq
        for i, raw in posts.items():   # the unbatched path on an owner
            self.submit_qs[self.rr].put(("post", self.w, (token, i), problem, algorithm, raw))
            self.rr = (self.rr + 1) % nq
        self.st["jobs"] += 1
        self.st["requests"] += len(bodies)
        self.st["parse_s"] += time.perf_counter() - t0
        if waiting == 0:
            self.finish(token)

    def finish(self, tk):
        t0 = time.perf_counter()
        store, arena = self.store, self.arena
        j = self.jobs.pop(tk)
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
            self.free.append(s)
        rows = j["rows"] + list(store.solutions[before:])
        del store.solutions[before:]
        # the response bytes as the HTTP handler writes them (service.py
        # do_POST): encoding is part of serving, so it runs here, in parallel
        enc = [(st, json.dumps(body).encode("utf-8")) for st, body in out]
        self.st["answer_s"] += time.perf_counter() - t0
        self.deliver(j["id"], enc, rows)

    def on_done(self, m):
        """An owner's answer: a batch of slots, or one unbatched post."""
        if m[0] == "slots":
            tk = m[1]
            self.jobs[tk]["waiting"] -= 1
        else:                                   # ("post", (token, index), status, resp, rows)
            _, (tk, i), status, resp, saved = m
            self.jobs[tk]["out"][i] = (status, resp)
            self.jobs[tk]["rows"] += saved
            self.jobs[tk]["waiting"] -= 1
        if self.jobs[tk]["waiting"] == 0:
            self.finish(tk)


def _worker_main(w, arena, lo, hi, req_q, resp_q, submit_qs, done_q, store, batchable_nmax,
                 stats_q, inflight=3):
    """Front-end worker driven by FrontEndPool.post_many: up to `inflight`
    jobs at a time, so the next chunk is parsed while the owner runs the
    previous one."""
    fe = _FrontEnd(w, arena, lo, hi, submit_qs, store, batchable_nmax,
                   lambda jid, enc, rows: resp_q.put((jid, enc, rows)))
    stop = False
    while not (stop and not fe.jobs):
        if not stop and len(fe.jobs) < inflight:
            try:
                job = req_q.get() if not fe.jobs else req_q.get_nowait()
            except queue.Empty:
                pass            # jobs in flight, none waiting: wait for an answer below
            else:
                if job is _STOP:
                    stop = True
                else:
                    fe.start(job)
                continue
        if not fe.jobs:
            continue
        t0 = time.perf_counter()
        m = done_q.get()
        fe.st["idle_s"] += time.perf_counter() - t0
        fe.on_done(m)
    stats_q.put(("worker", fe.st))


# ---------------------------------------------------------------------------
# HTTP front: every worker listens on the same port (SO_REUSEPORT, the kernel
# spreads the connections) and serves the reference's routes itself
# ---------------------------------------------------------------------------
_REASON = {200: "OK", 400: "Bad Request", 404: "Not Found", 413: "Payload Too Large",
           431: "Request Header Fields Too Large", 501: "Not Implemented"}
MAX_BODY = 64 << 20        # bytes of one request body (an inline /solve matrix fits)
MAX_HEAD = 64 << 10        # bytes of one request's header section


def _listen_socket(host: str, port: int):
    import socket
    sk = socket.socket(socket.AF_INET, socket.SOCK_STREAM)
    sk.setsockopt(socket.SOL_SOCKET, socket.SO_REUSEADDR, 1)
    sk.setsockopt(socket.SOL_SOCKET, socket.SO_REUSEPORT, 1)
    sk.bind((host, port))
    return sk


class _HttpConn(asyncio.Protocol):
    """asyncio protocol of one client connection: HTTP/1.1 keep-alive (or
    HTTP/1.0, closed after the response), one request at a time in order."""

    def __init__(self, server):
        self.server = server
        self.tr = None
        self.buf = bytearray()
        self.busy = False
        self.version = "HTTP/1.1"

    def connection_made(self, tr):
        self.tr = tr
        self.loop = asyncio.get_running_loop()

    def connection_lost(self, exc):
        self.tr = None

    def eof_received(self):
        return False

    def data_received(self, data):
        self.buf += data
        self._next()

    def pause_writing(self):
        pass

    def resume_writing(self):
        pass

    def _next(self):
        if self.busy or self.tr is None:
            return
        i = self.buf.find(b"\r\n\r\n")
        if i < 0:
            if len(self.buf) > MAX_HEAD:
                self._refuse(431)
            return
        lines = bytes(self.buf[:i]).decode("latin-1").split("\r\n")
        try:
            method, path, version = lines[0].split(" ", 2)
        except ValueError:
            self.tr.close()
            return
        hdrs = {}
        for ln in lines[1:]:
            k, _, v = ln.partition(":")
            hdrs[k.strip().lower()] = v.strip()
        # Content-Length is the client's claim: not a number or negative is a
        # 400, beyond MAX_BODY a 413, and the connection closes either way
        # (its byte stream can no longer be framed)
        try:
            n = int(hdrs.get("content-length", 0) or 0)
        except ValueError:
            n = -1
        if n < 0 or n > MAX_BODY:
            self._refuse(400 if n < 0 else 413)
            return
        if len(self.buf) < i + 4 + n:
            return
        body = bytes(self.buf[i + 4:i + 4 + n])
        del self.buf[:i + 4 + n]
        conn = hdrs.get("connection", "").lower()
        self.version = "HTTP/1.0" if version == "HTTP/1.0" else "HTTP/1.1"
        close = conn == "close" or (version == "HTTP/1.0" and conn != "keep-alive")
        self.busy = True
        self.server.handle(self, method, path, body, close)

    def _refuse(self, status):
        self.busy = True          # nothing more is parsed from this connection
        self.buf.clear()
        if self.tr is not None:
            self.tr.write((f"{self.version} {status} {_REASON[status]}\r\nContent-Length: 0"
                           "\r\nConnection: close\r\n\r\n").encode("latin-1"))
            self.tr.close()
            self.tr = None

    def respond(self, status, body: bytes, ctype="application/json", close=False, extra=()):
        if self.tr is None:
            return
        head = [f"{self.version} {status} {_REASON.get(status, 'OK')}"]
        if ctype:
            head.append(f"Content-type: {ctype}")
        head.extend(extra)
        head.append(f"Content-Length: {len(body)}")
        if close:
            head.append("Connection: close")
        self.tr.write(("\r\n".join(head) + "\r\n\r\n").encode("latin-1") + body)
        self.busy = False
        if close:
            self.tr.close()
            self.tr = None
        else:
            # the next pipelined request is parsed from the event loop, not
            # from inside this call: respond() can run inside a flush() that
            # is still walking its pending lists
            self.loop.call_soon(self._next)


def _http_worker_main(w, arena, lo, hi, host, port, submit_qs, done_q, store, batchable_nmax,
                      stats_q, saved_q, ready_q, stop_ev, chunk, window_s):
    """A front-end worker serving HTTP on (host, port) itself: the
    reference's routes (api/index.py, api/{tsp,vrp}/{bf,ga,sa,aco}/index.py)
    with the handlers' bytes; POSTs of one endpoint are gathered for up to
    `window_s` or `chunk` requests into one job (batchable TSP SA requests
    ride the arena and an owner's launch), and each is answered on its own
    connection as the job completes."""
    import asyncio
    from . import service
    loop = asyncio.new_event_loop()
    asyncio.set_event_loop(loop)
    conns = {}                 # job id -> [(conn, close)]
    pending = {}               # (problem, algorithm) -> [(body, conn, close)]
    timer = {"h": None}
    nj = {"id": 0}
    banners = {f"/api/{p}/{a}": f"Hi, this is the {p.upper()} {t} endpoint".encode("utf-8")
               for p in ("tsp", "vrp") for a, t in service.TITLES.items()}
    st_http = {"connections": 0}

    def deliver(jid, enc, rows):
        for (conn, close), (status, body) in zip(conns.pop(jid), enc):
            conn.respond(status, body, close=close)
        if rows:
            saved_q.put(rows)
        loop.call_soon(flush)   # slots came free (not re-entrantly: start() may finish a job)

    fe = _FrontEnd(w, arena, lo, hi, submit_qs, store, batchable_nmax, deliver)

    def flush(force=False):
        timer["h"] = None
        for key in list(pending):
            items = pending.get(key)
            if items is None:
                continue
            while items:
                take = items[:chunk]
                if len(take) < chunk and not force:
                    break
                if key == ("tsp", "sa") and len(fe.free) < len(take):
                    return          # wait for slots (a job's finish calls flush again)
                del items[:len(take)]
                jid = nj["id"]
                nj["id"] += 1
                conns[jid] = [(c, cl) for _, c, cl in take]
                fe.start((jid, key[0], key[1], [b for b, _, _ in take]))
            if not items:
                pending.pop(key, None)
        if pending and timer["h"] is None:
            timer["h"] = loop.call_later(window_s, flush, True)

    class Server:
        @staticmethod
        def handle(conn, method, path, body, close):
            path = path.split("?", 1)[0].rstrip("/")
            if method == "GET":
                if path == "/api":
                    conn.respond(200, b"Hello!", "text/plain", close)
                elif path in banners:
                    conn.respond(200, banners[path], "text/plain", close)
                else:
                    conn.respond(404, b"", None, close)
                return
            if method == "OPTIONS" and path == "/api/vrp/ga":   # the handler's preflight
                conn.respond(200, b"", None, close,
                             ("Access-Control-Allow-Origin: *", "Access-Control-Allow-Methods: *",
                              "Access-Control-Allow-Headers: *", "Access-Control-Allow-Headers: *"))
                return
            parts = path.split("/")
            if method == "POST" and len(parts) == 4 and parts[1] == "solve" and \
                    parts[2] in ("tsp", "vrp") and parts[3] in service.TITLES:
                # the remote front-end's inline route (vrpms_amd.remote), run by
                # an owner's App.solve_inline
                key = ("solve:" + parts[2], parts[3])
            elif method != "POST" or path not in banners:
                conn.respond(404 if path not in banners else 501, b"", None, close)
                return
            else:
                key = (parts[2], parts[3])
            pending.setdefault(key, []).append((body, conn, close))
            if len(pending[key]) >= chunk:
                flush()
            elif timer["h"] is None:
                timer["h"] = loop.call_later(window_s, flush, True)

    def protocol():
        st_http["connections"] += 1
        return _HttpConn(Server)

    def on_done(m):
        fe.on_done(m)

    def reader():               # the owners' answers, into the event loop
        while True:
            m = done_q.get()
            if m is _STOP:
                return
            loop.call_soon_threadsafe(on_done, m)

    th = threading.Thread(target=reader, daemon=True)
    th.start()
    sk = _listen_socket(host, port)
    srv = loop.run_until_complete(loop.create_server(protocol, sock=sk, backlog=4096))
    ready_q.put(w)

    async def watch():
        while not stop_ev.is_set():
            await asyncio.sleep(0.05)
        srv.close()
        flush(True)
        for _ in range(400):    # drain the jobs in flight (at most ~20 s)
            if not fe.jobs and not pending:
                break
            await asyncio.sleep(0.05)

    loop.run_until_complete(watch())
    fe.st.update(st_http)
    stats_q.put(("worker", fe.st))


def _default_app(store, seed, steps, max_seconds=None):
    def make_app(dev):
        from . import service
        return service.App(store, device=dev, seed=seed, max_seconds=max_seconds)
    return make_app


class FrontEndPool:
    """W front-end worker processes + one GPU-owner process per device (see
    the module docstring).  post_many() answers a list of request bodies for
    one endpoint with the (status, response dict) pairs App.post would give.
    With `listen=(host, port)` the workers serve HTTP themselves instead,
    every one on the same port (SO_REUSEPORT; port 0 picks a free one,
    `self.port`), and serve_forever() keeps the parent's store up to date."""

    INFLIGHT = 3   # jobs a worker keeps in flight

    def __init__(self, store, workers: int = 16, devices=(0,), steps: int = 1000, seed: int = 0,
                 window_s: float = 0.002, slots_per_worker: int = 1024, nmax: int = 64,
                 chunk: int = 64, max_batch: int = 16384, launch_factory=None, app_factory=None,
                 listen=None):
        self.store = store
        self.workers, self.devices, self.chunk = int(workers), list(devices), int(chunk)
        if not self.devices or self.workers < 1:
            raise ValueError("FrontEndPool needs at least one worker and one device")
        if "torch" in sys.modules:   # forked owners would inherit an initialised HIP runtime
            import torch
            if torch.cuda.is_initialized():
                raise RuntimeError("FrontEndPool forks its processes: create it before any GPU "
                                   "call, or start it as a child program "
                                   "(python -m vrpms_amd.frontends / vrpms_amd.service --workers)")
        self._broken = None
        self.listen = listen
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
        self._stop_ev = ctx.Event()
        self._saved_q = ctx.Queue()
        reserve = None
        if listen is not None:
            # hold the port (SO_REUSEPORT, not listening) until every worker listens on it
            reserve = _listen_socket(listen[0], int(listen[1]))
            self.port = reserve.getsockname()[1]
            ready_q = ctx.Queue()
        for w in range(self.workers):
            lo, hi = w * slots_per_worker, (w + 1) * slots_per_worker
            if listen is None:
                p = ctx.Process(target=_worker_main, daemon=True, name=f"vrpms-front{w}",
                                args=(w, self.arena, lo, hi, self._req_qs[w], self._resp_q,
                                      self._submit_qs, self._done_qs[w], store, nmax,
                                      self._stats_q, self.INFLIGHT))
            else:
                p = ctx.Process(target=_http_worker_main, daemon=True, name=f"vrpms-http{w}",
                                args=(w, self.arena, lo, hi, listen[0], self.port,
                                      self._submit_qs, self._done_qs[w], store, nmax,
                                      self._stats_q, self._saved_q, ready_q, self._stop_ev,
                                      self.chunk, window_s))
            p.start()
            self._procs.append(p)
        if reserve is not None:
            try:
                for _ in range(self.workers):
                    ready_q.get(timeout=60)
            except queue.Empty:
                self.close()
                raise RuntimeError("FrontEndPool: a worker did not start listening")
            finally:
                reserve.close()
        self._next_job = 0
        self._lock = threading.Lock()

    def _check_alive(self):
        dead = [p.name for p in self._procs if not p.is_alive()]
        if dead:
            self._broken = f"process(es) {dead} exited"
        return dead

    def serve_forever(self, poll_s: float = 0.2, until=None):
        """(listen mode) Keep the parent's store up to date with the saved
        solutions the workers report, until `until()` is true or a process
        dies (raises)."""
        while until is None or not until():
            try:
                rows = self._saved_q.get(timeout=poll_s)
                self.store.solutions.extend(rows)
            except queue.Empty:
                pass
            if self._check_alive():
                raise RuntimeError(f"FrontEndPool: {self._broken}")

    def post_many(self, problem: str, algorithm: str, bodies, raw: bool = False):
        """(status, body) per request, in order; chunks go to the workers
        round-robin and are answered as they complete.  The workers send each
        response as the HTTP handler's JSON bytes; raw=True returns those
        bytes, else the decoded dicts (App.post's contract)."""
        if self.listen is not None:
            raise RuntimeError("FrontEndPool: an HTTP pool is driven through its socket")
        if self._broken:
            raise RuntimeError(f"FrontEndPool is broken ({self._broken}); close() it")
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
                while True:   # (answers of another call's jobs are dropped)   # a worker or owner that died leaves its jobs unanswered: raise
                    try:
                        jid, res, rows = self._resp_q.get(timeout=5.0)
                        if jid in jobs:
                            break
                    except queue.Empty:
                        dead = self._check_alive()
                        if dead:
                            raise RuntimeError(f"FrontEndPool: process(es) {dead} exited; "
                                               f"{len(jobs)} job(s) of this call unanswered")
                s = jobs.pop(jid)
                out[s:s + len(res)] = res if raw else [(st, json.loads(b)) for st, b in res]
                if rows:
                    self.store.solutions.extend(rows)
            return out

    def close(self):
        if self.listen is not None and not self._check_alive():
            self._stop_ev.set()                 # workers stop listening and drain their jobs
            for _ in range(self.workers):
                try:
                    self.stats.append(self._stats_q.get(timeout=30))
                except queue.Empty:
                    break
            while True:
                try:
                    self.store.solutions.extend(self._saved_q.get_nowait())
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
            return
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


# ---------------------------------------------------------------------------
# cfg 5 over real sockets: a load generator in processes of its own
# ---------------------------------------------------------------------------
_REQ_PARTS = {}


def _tsp_request(i: int, N: int, host: str = "127.0.0.1") -> bytes:
    """POST /api/tsp/sa with the reference's body (api/tsp/sa/index.py:16-63)
    on matrix i, HTTP/1.1 keep-alive.  The body's bytes around durationsKey
    are encoded once per (N, host): the load generator should not spend its
    cores re-encoding the same JSON."""
    parts = _REQ_PARTS.get((N, host))
    if parts is None:
        mark = -7310
        body = json.dumps({"solutionName": "n", "solutionDescription": "d", "locationsKey": 0,
                           "durationsKey": mark, "customers": list(range(1, N)), "startNode": 0,
                           "startTime": 0}).encode()
        pre, post = body.split(str(mark).encode())
        head = (f"POST /api/tsp/sa HTTP/1.1\r\nHost: {host}\r\nContent-Type: application/json"
                f"\r\nContent-Length: ").encode("latin-1")
        parts = _REQ_PARTS[(N, host)] = (head, pre, post)
    head, pre, post = parts
    key = str(i).encode()
    return b"".join((head, str(len(pre) + len(key) + len(post)).encode(), b"\r\n\r\n", pre, key,
                     post))


def _loadgen_proc(host, port, idx, N, conns, start_at, sample, out_q):
    """One client process: `conns` keep-alive connections take requests
    (indices `idx`) from one shared iterator, each sending its next request
    when the previous answer has fully arrived; all connections are open
    before `start_at` (time.monotonic), when the clock starts."""
    loop = asyncio.new_event_loop()
    asyncio.set_event_loop(loop)
    it = iter(idx)
    res = {"n": 0, "ok": 0, "sample": {}, "errors": 0}
    left = {"conns": conns}
    done = loop.create_future()

    class Client(asyncio.Protocol):
        def __init__(self):
            self.tr, self.buf, self.cur = None, bytearray(), None

        def connection_made(self, tr):
            self.tr = tr

        def connection_lost(self, exc):
            if self.cur is not None:
                res["errors"] += 1
                self.cur = None
                self._finish()

        def _finish(self):
            left["conns"] -= 1
            if left["conns"] == 0 and not done.done():
                done.set_result(time.monotonic())

        def send(self):
            self.cur = next(it, None)
            if self.cur is None:
                self.tr.close()
                self._finish()
                return
            self.tr.write(_tsp_request(self.cur, N))

        def data_received(self, data):
            self.buf += data
            i = self.buf.find(b"\r\n\r\n")
            if i < 0:
                return
            head = bytes(self.buf[:i])
            c = head.lower().find(b"\r\ncontent-length:")
            n = int(head[c + 17:head.find(b"\r\n", c + 2) if head.find(b"\r\n", c + 2) > 0
                         else len(head)]) if c >= 0 else 0
            if len(self.buf) < i + 4 + n:
                return
            status = int(head[9:12])
            body = bytes(self.buf[i + 4:i + 4 + n])
            del self.buf[:i + 4 + n]
            res["n"] += 1
            res["ok"] += status == 200
            if self.cur in sample:
                res["sample"][self.cur] = (status, body.decode("utf-8"))
            self.send()

    async def run():
        clients = []
        for _ in range(conns):
            _, c = await loop.create_connection(Client, host, port)
            clients.append(c)
        await asyncio.sleep(max(0.0, start_at - time.monotonic()))
        t0 = time.monotonic()
        for c in clients:
            c.send()
        t1 = await done
        return t0, t1

    t0, t1 = loop.run_until_complete(run())
    res.update(t0=t0, t1=t1)
    out_q.put(res)


def loadgen(host, port, R, N, connections=1024, procs=4, sample=200, seed=1):
    """R requests over `connections` concurrent keep-alive connections from
    `procs` client processes -> requests/s at the client (first send to last
    answer), answers counted, and a sample of (status, response body)."""
    ctx = mp.get_context("fork")
    q = ctx.Queue()
    pick = set(np.random.default_rng(seed).choice(R, size=min(sample, R), replace=False).tolist())
    start_at = time.monotonic() + 2.0 + connections / 2000.0
    per = [list(range(k, R, procs)) for k in range(procs)]
    cps = [connections // procs + (1 if k < connections % procs else 0) for k in range(procs)]
    ps = [ctx.Process(target=_loadgen_proc, args=(host, port, per[k], N, cps[k], start_at,
                                                  pick & set(per[k]), q)) for k in range(procs)]
    for p in ps:
        p.start()
    outs = [q.get(timeout=600) for _ in ps]
    for p in ps:
        p.join(timeout=10)
    t0 = min(o["t0"] for o in outs)
    t1 = max(o["t1"] for o in outs)
    samp = {}
    for o in outs:
        samp.update(o["sample"])
    return {"requests": sum(o["n"] for o in outs), "ok": sum(o["ok"] for o in outs),
            "errors": sum(o["errors"] for o in outs), "wall_s": t1 - t0,
            "requests_per_s": sum(o["n"] for o in outs) / (t1 - t0), "connections": connections,
            "client_processes": procs, "sample": samp}


def bench_http(R: int = 10000, N: int = 50, workers: int = 12, steps: int = 1000, seed: int = 0,
               window_ms: float = 2.0, connections: int = 1024, clients: int = 4,
               check: int = 200):
    """BASELINE cfg 5 through sockets: a FrontEndPool whose workers listen on
    one port (SO_REUSEPORT) and `clients` load-generator processes holding
    `connections` concurrent connections that send R POST /api/tsp/sa.
    requests/s is measured at the client.  A sample of the answers is
    checked: a 200 answer whose tour visits every customer once, whose
    duration is its closed tour's cost (A4), and whose body bytes are the
    handler's encoding of that result (service.endpoint_handler do_POST:
    json.dumps); and the GET banner / a 400 answer through the same socket
    equal the reference handler's bytes."""
    from . import service, synth
    rng = np.random.default_rng(seed + 5)
    store = service.MemoryStore({0: [{"id": i} for i in range(N)]},
                                {i: synth.random_symmetric(N, rng).tolist() for i in range(R)})
    with FrontEndPool(store, workers=workers, steps=steps, seed=seed, window_s=window_ms * 1e-3,
                      listen=("127.0.0.1", 0)) as pool:
        port = pool.port
        warm = loadgen("127.0.0.1", port, min(R, 2 * workers * pool.chunk), N,
                       connections=min(connections, 256), procs=clients, sample=0)
        out = loadgen("127.0.0.1", port, R, N, connections=connections, procs=clients,
                      sample=check)
        import urllib.request
        with urllib.request.urlopen(f"http://127.0.0.1:{port}/api/tsp/sa", timeout=30) as r:
            banner = r.read()
        req = urllib.request.Request(f"http://127.0.0.1:{port}/api/tsp/sa", data=b"{}",
                                     method="POST")
        try:
            urllib.request.urlopen(req, timeout=30)
            err_body = None
        except urllib.error.HTTPError as e:
            err_body = e.read()
    bad = 0
    for i, (st, text) in out.pop("sample").items():
        body = json.loads(text)
        D = np.asarray(store.durations[int(i)])
        v = body["message"]["vehicle"] if st == 200 else None
        if v is None or sorted(v[1:-1]) != list(range(1, N)) or v[0] != 0 or v[-1] != 0 or \
                int(D[v[:-1], v[1:]].sum()) != body["message"]["duration"] or \
                json.dumps(body) != text:
            bad += 1
    want_err = json.dumps(service.App(store, solve=lambda *a: None).post("tsp", "sa", b"{}")[1])
    owners = [x for kind, x in pool.stats if kind == "owner"]
    out.update({"workload": f"{R} POST /api/tsp/sa (TSP-{N}) over {connections} concurrent "
                           f"keep-alive connections from {clients} client processes; {workers} "
                           f"front-end processes listening on one port (SO_REUSEPORT) + 1 "
                           f"GPU-owner process (vrpms_amd.frontends)",
                "workers": workers, "batch_window_ms": window_ms, "sa_steps_per_chain": steps,
                "warmup_requests_per_s": warm["requests_per_s"],
                "duration_checked": check, "answer_mismatches": bad,
                "banner_equal": banner == b"Hi, this is the TSP Simulated Annealing endpoint",
                "error_bytes_equal": err_body is not None and err_body.decode() == want_err,
                "owners": owners})
    return out


def main(argv=None):
    ap = argparse.ArgumentParser(description="cfg-5 API throughput through FrontEndPool")
    ap.add_argument("cmd", choices=["bench", "bench-http"])
    ap.add_argument("--requests", type=int, default=10000)
    ap.add_argument("--workers", type=int, default=16)
    ap.add_argument("--steps", type=int, default=1000)
    ap.add_argument("--window-ms", type=float, default=2.0)
    ap.add_argument("--connections", type=int, default=1024)
    ap.add_argument("--clients", type=int, default=4)
    args = ap.parse_args(argv)
    if args.cmd == "bench":
        out = bench_api(R=args.requests, workers=args.workers, steps=args.steps,
                        window_ms=args.window_ms)
    else:
        out = bench_http(R=args.requests, workers=args.workers, steps=args.steps,
                         window_ms=args.window_ms, connections=args.connections,
                         clients=args.clients)
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    main()
