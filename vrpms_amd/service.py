"""GPU-box HTTP host for the eight solver endpoints.

The reference serves each algorithm as a Vercel function
(api/{tsp,vrp}/{bf,ga,sa,aco}/index.py): parse the body, fetch the location
set and duration matrix from Supabase, run the algorithm (the
`# TODO: Run algorithm` slot), optionally save the solution, respond.  This
module keeps that request/response contract byte for byte -- banners,
preflight headers, error lists, status lines, the save payload -- and fills
the slot with the GPU solver (vrpms_amd.solver).  One process owns one GPU
context per served device; requests are served by a threading HTTP server,
one at a time per device (App.devices; large requests as an island model
across all of them).  Throughput mode across processes: vrpms_amd.frontends.

Storage is pluggable: anything with the three calls of the reference's
Database classes (api/database.py) works.  `MemoryStore` (JSON-backed, the
default and the one the tests use) returns the reference's exact error
messages; a Supabase adapter is sketched in INTEGRATION.md §6.

  python -m vrpms_amd.service --port 8000 --data instances.json

Deliberate differences: a body that is not JSON gets a 400 with
{'what': 'Invalid request'} (the reference's handler raises and drops the
connection), and a solver exception becomes a 400 {'what': 'Solver error'}.
"""
from __future__ import annotations

import argparse
import json
import sys
import threading
import time
from http.server import BaseHTTPRequestHandler, ThreadingHTTPServer

TITLES = {"bf": "Brute Force", "ga": "Genetic Algorithm", "sa": "Simulated Annealing",
          "aco": "Ant Colony Optimization"}

# (body key, params key) in the order the reference checks them
# (api/parameters.py:4-15 and 34-44); 'auth' is the only optional one
_COMMON = {
    "vrp": [("solutionName", "name"), ("auth", "auth"), ("solutionDescription", "description"),
            ("locationsKey", "locations_key"), ("durationsKey", "durations_key"),
            ("capacities", "capacities"), ("startTimes", "start_times"),
            ("ignoredCustomers", "ignored_customers"),
            ("completedCustomers", "completed_customers")],
    "tsp": [("solutionName", "name"), ("auth", "auth"), ("solutionDescription", "description"),
            ("locationsKey", "locations_key"), ("durationsKey", "durations_key"),
            ("customers", "customers"), ("startNode", "start_node"), ("startTime", "start_time")],
}
# search knobs of solver.solve_tsp / solve_vrp that the /solve route accepts
# in its "knobs" object (vrpms_amd.remote forwards them): name -> type
INLINE_KNOBS = {"steps": int, "separators": int, "window": int, "chains": int,
                "window_types": int, "pop": int, "islands": int, "colonies": int, "ants": int}
# their accepted ranges (inclusive): a value from the network outside them is a
# 400, never an allocation (islands = 10**6 or chains = 2**30 would
# exhaust device memory while the request holds every device lock)
KNOB_RANGES = {"steps": (1, 10**8), "separators": (0, 4096), "window": (0, 65535),
               "chains": (1, 1 << 16), "window_types": (0, 7), "pop": (2, 4096),
               "islands": (1, 4096), "colonies": (1, 4096), "ants": (1, 4096)}


def check_knob(name, value):
    """INLINE_KNOBS[name](value), range-checked by KNOB_RANGES (ValueError)."""
    if isinstance(value, bool) or not isinstance(value, (int, float, str)):
        raise ValueError(f"knob {name} must be an integer")
    v = INLINE_KNOBS[name](value)
    lo, hi = KNOB_RANGES[name]
    if not lo <= v <= hi:
        raise ValueError(f"knob {name}={v} outside [{lo}, {hi}]")
    return v


def multi_threaded(value):
    """The VRP GA `multiThreaded` value (api/parameters.py:20 passes the raw
    JSON through): a JSON boolean as is; the strings "true"/"1" and "false"/
    "0" (any case) and the numbers 1 / 0 as those booleans; anything else is
    None -- the size rule decides (bool("false") was True)."""
    if isinstance(value, bool):
        return value
    if isinstance(value, (int, float)) and value in (0, 1):
        return bool(value)
    if isinstance(value, str) and value.strip().lower() in ("true", "1", "false", "0"):
        return value.strip().lower() in ("true", "1")
    return None
# algorithm knobs (api/parameters.py:18-23; every other algorithm takes none)
_KNOBS = {("vrp", "ga"): [("multiThreaded", "multi_threaded"),
                          ("randomPermutationCount", "random_permutationCount"),
                          ("iterationCount", "iteration_count")]}


def get_parameter(name, content, errors, optional=False):
    """api/helpers.py:5-8."""
    if name not in content and not optional:
        errors += [{"what": "Missing parameter", "reason": f"'{name}' was not provided"}]
    return content.get(name)


def parse(problem: str, algorithm: str, content: dict, errors: list):
    """(common params, algorithm params) exactly as parse_common_*_parameters
    and parse_*_<algo>_parameters build them."""
    common = {key: get_parameter(name, content, errors, optional=(name == "auth"))
              for name, key in _COMMON[problem]}
    knobs = {key: get_parameter(name, content, errors)
             for name, key in _KNOBS.get((problem, algorithm), [])}
    return common, knobs


def remove_unused_locations(locations, ignored_customers, completed_customers):
    """api/helpers.py:11-13."""
    disregard = ignored_customers + completed_customers
    return [loc for loc in locations if loc["id"] not in disregard]


# ---------------------------------------------------------------------------
# storage
# ---------------------------------------------------------------------------
_NOT_FOUND = ("Make sure you are accessing public data or data owned by you. "
              "Check if your authentication token has expired.")
_NOT_PERMITTED = {
    "vrp": ("An authentication token is required to save solutions to database. "
            "Please provide 'auth' with a valid JWT token in the request body. "
            "If you have already provided a token, it has very likely expired."),
    "tsp": ("An authentication token is required to save solutions to database."
            " Please provide 'auth' with a valid JWT token in the request body"),
}


class MemoryStore:
    """In-process stand-in for the Supabase tables the handlers use:
    `locations` {id: [location, ...]}, `durations` {id: matrix},
    `users` {token: email}; saved rows are appended to `solutions`."""

    def __init__(self, locations=None, durations=None, users=None):
        self.locations = dict(locations or {})
        self.durations = dict(durations or {})
        self.users = dict(users or {})
        self.solutions = []
        self._lock = threading.Lock()

    @classmethod
    def from_json(cls, path):
        """{"locations": {"1": [...]}, "durations": {"2": [[...]]}, "users": {...}};
        ids are matched as strings or ints."""
        with open(path) as f:
            raw = json.load(f)
        return cls(raw.get("locations"), raw.get("durations"), raw.get("users"))

    def session(self, auth):
        return _Session(self, auth)

    def _get(self, table, key):
        for k in (key, str(key)):
            try:
                if k in table:
                    return table[k]
            except TypeError:       # unhashable id from the request body
                return None
        return None


class _Session:
    """The per-request Database object of api/database.py."""

    def __init__(self, store: MemoryStore, auth):
        self.store = store
        self.email = store.users.get(auth) if isinstance(auth, str) else None

    def get_locations_by_id(self, key, errors):
        rows = self.store._get(self.store.locations, key)
        if rows is None:
            errors += [{"what": "Database read error",
                        "reason": f"No location set found with given id {key}. " + _NOT_FOUND}]
        return rows

    def get_durations_by_id(self, key, errors):
        m = self.store._get(self.store.durations, key)
        if m is None:
            errors += [{"what": "Database read error",
                        "reason": f"No duration matrix found with given id {key}. " + _NOT_FOUND}]
        return m

    def save_solution(self, problem, data: dict, errors):
        """DatabaseVRP/DatabaseTSP.save_solution: owner from the token."""
        if not self.email:
            errors += [{"what": "Not permitted", "reason": _NOT_PERMITTED[problem]}]
            return
        row = {"name": data["name"], "description": data["description"], "owner": self.email}
        row.update({k: v for k, v in data.items() if k not in ("name", "description")})
        with self.store._lock:
            self.store.solutions.append(row)


# ---------------------------------------------------------------------------
# throughput mode: concurrent small TSP requests share one launch
# ---------------------------------------------------------------------------
class TspBatcher:
    """Coalesces concurrent /api/tsp/sa requests on static matrices into one
    `tsp_batch_sa` launch per node count (one workgroup per request, config
    5 of BASELINE.json).  A request waits at most `window_s` for company.
    Requests in one launch share its seed and temperature schedule (scaled
    to the batch's mean edge), so a batched answer depends on the batch it
    rode in; the unbatched path is deterministic per request.  With several
    devices the launches go to them round-robin (SURVEY.md §8e cfg 5:
    replicas only), one launch thread per device, so they run together."""

    MIN_N, MAX_N = 4, 190        # compact nodes; N*N int32 must fit the LDS

    def __init__(self, app, window_s: float = 0.005, steps: int = 2000, max_batch: int = 16384,
                 launch=None):
        self.app = app
        self.window_s = window_s
        self.steps = steps
        self.max_batch = max_batch
        self.launches = 0
        self.requests = 0
        self._launch = launch or self._gpu_launch
        self._q = []
        self._cv = threading.Condition()
        self.devices = list(getattr(app, "devices", None) or [getattr(app, "device", 0)])
        self.per_device = {d: 0 for d in self.devices}
        self._rr = 0
        self._pool = None
        if len(self.devices) > 1:
            from concurrent.futures import ThreadPoolExecutor
            self._pool = ThreadPoolExecutor(len(self.devices), thread_name_prefix="tsp-launch")
        threading.Thread(target=self._loop, daemon=True, name="tsp-batcher").start()

    @classmethod
    def accepts(cls, ci) -> bool:
        """Static matrices of MIN_N..MAX_N nodes that also pass the A9 int32
        guard vrpms_set_instance applies on the unbatched path
        ((N + K + 1) * max_duration < 2^31, K = 1, start time 0 here because
        a static tour's duration does not depend on it); anything else takes
        the unbatched path, so both paths share one error contract."""
        if ci.durations.shape[0] != 1 or not cls.MIN_N <= ci.N <= cls.MAX_N:
            return False
        mx = int(ci.durations.max()) if ci.durations.size else 0
        return (ci.N + 2) * mx < 2**31

    def solve(self, ci) -> dict:
        """Blocks until the request's launch finished -> the TSP slot dict."""
        job = {"ci": ci, "done": threading.Event()}
        with self._cv:
            self._q.append(job)
            self._cv.notify()
        job["done"].wait()
        if "error" in job:
            raise job["error"]
        path = [0] + list(job["tour"]) + [0]
        duration = job.get("duration")
        if duration is None:  # a launch that returns tours only (tests' stand-in launches)
            D = ci.durations[0]
            duration = int(sum(int(D[a][b]) for a, b in zip(path, path[1:])))
        return {"duration": duration, "vehicle": [ci.nodes[c] for c in path]}

    def _loop(self):
        while True:
            with self._cv:
                while not self._q:
                    self._cv.wait()
            time.sleep(self.window_s)          # let concurrent requests join
            with self._cv:
                batch, self._q = self._q[:self.max_batch], self._q[self.max_batch:]
            groups = {}
            for job in batch:
                groups.setdefault(job["ci"].N, []).append(job)
            for N, jobs in groups.items():
                dev = self.devices[self._rr % len(self.devices)]
                self._rr += 1
                if self._pool is None:
                    self._run(N, jobs, dev)
                else:
                    self._pool.submit(self._run, N, jobs, dev)

    def _run(self, N, jobs, dev):
        try:
            if len(self.devices) > 1:
                res = self._launch(N, [j["ci"] for j in jobs], dev)
            else:
                res = self._launch(N, [j["ci"] for j in jobs])
            tours, durs = res if isinstance(res, tuple) else (res, None)
            with self._cv:
                self.launches += 1
                self.requests += len(jobs)
                self.per_device[dev] += len(jobs)
            for x, (j, t) in enumerate(zip(jobs, tours)):
                j["tour"] = t
                if durs is not None and durs[x] is not None:
                    j["duration"] = durs[x]
        except Exception as e:         # every waiter of the group sees it
            for j in jobs:
                j["error"] = e
        for j in jobs:
            j["done"].set()

    def _gpu_launch(self, N, cis, device=None):
        """-> (tours, durations) on `device` (default: the app's first): the
        durations are the kernel's keys' primary term (A8: a TSP key is
        duration << 28), exact below the 2^28 - 1 clamp; a clamped one is
        summed on the host."""
        import numpy as np
        import torch
        from . import solver
        # one int32 staging buffer (no per-request stack of int64 copies);
        # the mean edge over the batch from the same buffer
        host = np.empty((len(cis), N, N), dtype=np.int32)
        for x, ci in enumerate(cis):
            host[x] = ci.durations[0]
        nz = host[host > 0]
        edge = float(nz.mean()) if nz.size else 1.0
        inv_t0 = 1.0 / (0.5 * edge)
        inv_alpha = (0.5 / 0.002) ** (1.0 / max(1, self.steps))
        dev = self.devices[0] if device is None else device
        with self.app.locks[dev]:
            ctx = solver.context(dev)
            mats = torch.from_numpy(host).to(ctx.dev)
            tours, keys = ctx.tsp_batch_sa(mats, self.steps, inv_t0, inv_alpha, self.app.seed)
            tours, keys = tours.cpu().tolist(), keys.cpu().tolist()
        clamp = (1 << 28) - 1
        durs = [None if (k >> 28) & clamp == clamp else (k >> 28) & clamp for k in keys]
        return tours, durs


# ---------------------------------------------------------------------------
# the endpoint logic
# ---------------------------------------------------------------------------
class App:
    """Parse -> fetch -> solve -> save -> respond for one endpoint call.
    `solve` is injectable (tests); by default it is the GPU solver.

    `devices` (default [device]): the GPUs this process serves.  Each has
    its own context and lock; a request takes the first free device (one
    request per device at a time), and a large SA / GA / ACO request (more
    than `island_min_n` customers) with two or more devices takes them all
    and runs as an island model across them (solver.search_islands).  The
    VRP GA endpoint's `multiThreaded` (api/parameters.py:20, the reference's
    only parallelism knob) decides that for its request instead: true runs
    the island model over every device, false one device.  A device listed
    twice (one GPU standing in for two) is locked once."""

    def __init__(self, store, device: int = 0, seed: int = 0, max_seconds: float | None = None,
                 solve=None, batch_tsp: bool = False, batch_window_s: float = 0.005,
                 batch_steps: int = 2000, batch_launch=None, devices=None,
                 island_min_n: int = 150):
        self.store = store
        self.devices = list(devices) if devices else [device]
        self.device = self.devices[0]
        self.seed = seed
        self.max_seconds = max_seconds
        self.island_min_n = island_min_n
        self.locks = {d: threading.Lock() for d in self.devices}
        self.gpu_lock = self.locks[self.device]
        self._rr = 0
        self._rr_lock = threading.Lock()
        self._solve = solve or self._gpu_solve
        self.batcher = TspBatcher(self, batch_window_s, batch_steps, launch=batch_launch) \
            if batch_tsp else None

    def _scheduled(self, problem, algorithm, params, knobs, locations, durations):
        """Run the solve on a device: all of them (in order, as an island
        model) for a large SA / GA / ACO request when there are several, else
        the first free one (round-robin start), waiting for one if all are
        busy."""
        n = len(params.get("customers") or []) if problem == "tsp" else \
            max(0, len(locations or []) - 1)
        knobs = dict(knobs)
        mt = multi_threaded(knobs.get("multi_threaded"))
        islands = n > self.island_min_n if mt is None else mt
        if len(self.devices) > 1 and algorithm != "bf" and islands:
            held = sorted(set(self.devices))   # each lock once, in one global order
            for d in held:
                self.locks[d].acquire()
            try:
                knobs["devices"] = list(self.devices)
                return self._solve(problem, algorithm, params, knobs, locations, durations)
            finally:
                for d in reversed(held):
                    self.locks[d].release()
        with self._rr_lock:
            start = self._rr
            self._rr = (self._rr + 1) % len(self.devices)
        order = self.devices[start:] + self.devices[:start]
        dev = next((d for d in order if self.locks[d].acquire(blocking=False)), None)
        if dev is None:
            dev = order[0]
            self.locks[dev].acquire()
        try:
            knobs["device"] = dev
            return self._solve(problem, algorithm, params, knobs, locations, durations)
        finally:
            self.locks[dev].release()

    def _batched_tsp(self, params, durations):
        """The compact instance when this request rides the batcher, else None."""
        if self.batcher is None:
            return None
        from . import solver
        ci = solver.compact_tsp(durations, params["customers"], params["start_node"],
                                params["start_time"] or 0)
        return ci if TspBatcher.accepts(ci) else None

    def _gpu_solve(self, problem, algorithm, params, knobs, locations, durations):
        """knobs may carry "seed", "time_limit" and "objective" (the /solve
        route's options, vrpms_amd.remote); the endpoints use the app's."""
        from . import solver
        seed = int(knobs.get("seed", self.seed))
        tl = knobs.get("time_limit", self.max_seconds)
        devs = knobs.get("devices") or [knobs.get("device", self.device)]
        dv = dict(device=devs[0], devices=devs if len(devs) > 1 else None)
        extra = dict(knobs.get("inline") or {})
        if problem == "tsp":
            return solver.solve_tsp(algorithm, durations, params["customers"],
                                    params["start_node"], params["start_time"] or 0,
                                    seed=seed, time_limit=tl, **dv, **extra)
        if knobs.get("random_permutationCount"):
            extra["random_permutation_count"] = int(knobs["random_permutationCount"])
        if knobs.get("iteration_count"):
            extra["iteration_count"] = int(knobs["iteration_count"])
        return solver.solve_vrp(algorithm, durations, locations, params["capacities"],
                                params["start_times"], params["ignored_customers"],
                                params["completed_customers"], seed=seed,
                                objective=knobs.get("objective", "sum"),
                                time_limit=tl, **dv, **extra)

    def post(self, problem: str, algorithm: str, raw: bytes):
        """-> (status, response dict) for a POST body."""
        text = raw.decode("utf-8") if raw else ""
        try:
            content = json.loads(text) if text else dict()
        except ValueError as e:
            return 400, {"success": False,
                         "errors": [{"what": "Invalid request", "reason": str(e)}]}
        if not isinstance(content, dict):
            return 400, {"success": False, "errors": [
                {"what": "Invalid request", "reason": "the body must be a JSON object"}]}
        errors = []
        params, knobs = parse(problem, algorithm, content, errors)
        if errors:
            return 400, {"success": False, "errors": errors}
        db = self.store.session(params["auth"])
        locations = db.get_locations_by_id(params["locations_key"], errors)
        durations = db.get_durations_by_id(params["durations_key"], errors)
        if errors:
            return 400, {"success": False, "errors": errors}
        try:
            ci = self._batched_tsp(params, durations) if (problem, algorithm) == ("tsp", "sa") \
                else None
            if ci is not None:
                result = self.batcher.solve(ci)
            else:
                result = self._scheduled(problem, algorithm, params, knobs, locations, durations)
        except Exception as e:   # bad instance shape, GPU unavailable, ...
            return 400, {"success": False,
                         "errors": [{"what": "Solver error", "reason": str(e)}]}
        if params["auth"]:
            if problem == "vrp":
                data = {"name": params["name"], "description": params["description"],
                        "durationMax": result["durationMax"], "durationSum": result["durationSum"],
                        "locations": remove_unused_locations(locations, params["ignored_customers"],
                                                             params["completed_customers"]),
                        "vehicles": result["vehicles"]}
            else:
                data = {"name": params["name"], "description": params["description"],
                        "duration": result["duration"], "locations": locations,
                        "vehicle": result["vehicle"]}
            db.save_solution(problem, data, errors)
        if errors:
            return 400, {"success": False, "errors": errors}
        return 200, {"success": True, "message": result}


    def solve_inline(self, problem: str, algorithm: str, raw: bytes):
        """POST /solve/{tsp,vrp}/<algo>: the instance inline (no DB) -- what a
        host without a GPU sends to the GPU box (vrpms_amd.remote).  Body: the
        solve_tsp / solve_vrp arguments in the request's camelCase names
        ("durations" is the DB's `matrix` payload); response as the
        handlers': {"success": true, "message": result} or a 400 error list."""
        try:
            content = json.loads(raw.decode("utf-8")) if raw else {}
            if not isinstance(content, dict):
                raise ValueError("the body must be a JSON object")
        except ValueError as e:
            return 400, {"success": False,
                         "errors": [{"what": "Invalid request", "reason": str(e)}]}
        if problem not in ("tsp", "vrp") or algorithm not in TITLES:
            return 400, {"success": False, "errors": [
                {"what": "Invalid request", "reason": f"no solver /solve/{problem}/{algorithm}"}]}
        names = (["durations", "customers", "startNode", "startTime"] if problem == "tsp" else
                 ["durations", "locations", "capacities", "startTimes", "ignoredCustomers",
                  "completedCustomers"])
        errors = []
        vals = {name: get_parameter(name, content, errors) for name in names}
        if errors:
            return 400, {"success": False, "errors": errors}
        if problem == "tsp":
            params = {"customers": vals["customers"], "start_node": vals["startNode"],
                      "start_time": vals["startTime"]}
            knobs, locations = {}, None
        else:
            params = {"capacities": vals["capacities"], "start_times": vals["startTimes"],
                      "ignored_customers": vals["ignoredCustomers"] or [],
                      "completed_customers": vals["completedCustomers"] or []}
            knobs = {"random_permutationCount": content.get("randomPermutationCount"),
                     "iteration_count": content.get("iterationCount")}
            locations = vals["locations"]
        # the remote front-end's options (vrpms_amd.remote): seed, time limit
        # (capped by the box's own), objective
        try:
            if "seed" in content:
                knobs["seed"] = int(content["seed"])
            if content.get("timeLimit") is not None:
                tl = float(content["timeLimit"])
                knobs["time_limit"] = tl if self.max_seconds is None else min(tl, self.max_seconds)
            if problem == "vrp" and "objective" in content:
                if content["objective"] not in ("sum", "max"):
                    raise ValueError("objective must be 'sum' or 'max'")
                knobs["objective"] = content["objective"]
            inline = content.get("knobs") or {}
            if not isinstance(inline, dict):
                raise ValueError("knobs must be a JSON object")
            bad = sorted(k for k in inline if k not in INLINE_KNOBS)
            if bad:
                raise ValueError(f"unknown knob(s) {bad}; known: {sorted(INLINE_KNOBS)}")
            knobs["inline"] = {k: check_knob(k, v) for k, v in inline.items()}
        except (TypeError, ValueError) as e:
            return 400, {"success": False,
                         "errors": [{"what": "Invalid request", "reason": str(e)}]}
        try:
            result = self._scheduled(problem, algorithm, params, knobs, locations,
                                     vals["durations"])
        except Exception as e:
            return 400, {"success": False,
                         "errors": [{"what": "Solver error", "reason": str(e)}]}
        return 200, {"success": True, "message": result}


def endpoint_handler(app: App, problem: str, algorithm: str):
    """A BaseHTTPRequestHandler class for one endpoint, with the reference's
    GET banner, POST contract and (VRP GA only) preflight response."""
    banner = f"Hi, this is the {problem.upper()} {TITLES[algorithm]} endpoint"

    class Handler(BaseHTTPRequestHandler):
        def log_message(self, *a):
            pass

        def do_GET(self):
            self.send_response(200)
            self.send_header("Content-type", "text/plain")
            self.end_headers()
            self.wfile.write(banner.encode("utf-8"))

        def do_POST(self):
            n = int(self.headers.get("Content-Length", 0))
            status, body = app.post(problem, algorithm, self.rfile.read(n))
            self.send_response(status)
            self.send_header("Content-type", "application/json")
            self.end_headers()
            self.wfile.write(json.dumps(body).encode("utf-8"))

    if (problem, algorithm) == ("vrp", "ga"):
        def do_OPTIONS(self):   # api/vrp/ga/index.py: the header is sent twice there too
            self.send_response(200, "ok")
            self.send_header("Access-Control-Allow-Origin", "*")
            self.send_header("Access-Control-Allow-Methods", "*")
            self.send_header("Access-Control-Allow-Headers", "*")
            self.send_header("Access-Control-Allow-Headers", "*")
            self.end_headers()
        Handler.do_OPTIONS = do_OPTIONS
    return Handler


def router(app: App):
    """One server for every route: /api (api/index.py) and
    /api/{tsp,vrp}/{bf,ga,sa,aco}."""
    routes = {f"/api/{p}/{a}": endpoint_handler(app, p, a)
              for p in ("tsp", "vrp") for a in TITLES}

    class Router(BaseHTTPRequestHandler):
        def log_message(self, *a):
            pass

        def _dispatch(self, method):
            path = self.path.split("?", 1)[0].rstrip("/")
            if path == "/api" and method == "GET":
                self.send_response(200)
                self.send_header("Content-type", "text/plain")
                self.end_headers()
                self.wfile.write(b"Hello!")
                return
            if path.startswith("/solve/") and method == "POST":   # vrpms_amd.remote
                _, _, problem, algorithm = (path.split("/") + ["", ""])[:4]
                n = int(self.headers.get("Content-Length", 0))
                status, body = app.solve_inline(problem, algorithm, self.rfile.read(n))
                self.send_response(status)
                self.send_header("Content-type", "application/json")
                self.end_headers()
                self.wfile.write(json.dumps(body).encode("utf-8"))
                return
            cls = routes.get(path)
            fn = getattr(cls, "do_" + method, None) if cls else None
            if fn is None:
                self.send_error(404 if cls is None else 501)
                return
            fn(self)

        def do_GET(self):
            self._dispatch("GET")

        def do_POST(self):
            self._dispatch("POST")

        def do_OPTIONS(self):
            self._dispatch("OPTIONS")

    return Router


def serve(app: App, host: str = "127.0.0.1", port: int = 8000) -> ThreadingHTTPServer:
    return ThreadingHTTPServer((host, port), router(app))


def main(argv=None):
    ap = argparse.ArgumentParser(description=__doc__.split("\n")[0])
    ap.add_argument("--host", default="127.0.0.1")
    ap.add_argument("--port", type=int, default=8000)
    ap.add_argument("--data", help="MemoryStore JSON (locations / durations / users)")
    ap.add_argument("--device", type=int, default=0)
    ap.add_argument("--devices", default=None,
                    help="comma-separated GPUs to serve (default: --device); large SA / GA / ACO "
                         "requests run as an island model across them")
    ap.add_argument("--seed", type=int, default=0)
    ap.add_argument("--max-seconds", type=float, default=None,
                    help="wall-time cap per solve (default: the algorithm's own budget)")
    ap.add_argument("--batch-tsp", action="store_true",
                    help="coalesce concurrent /api/tsp/sa requests into one launch")
    ap.add_argument("--batch-window-ms", type=float, default=5.0)
    ap.add_argument("--batch-steps", type=int, default=2000)
    ap.add_argument("--workers", type=int, default=0,
                    help="throughput mode (BASELINE cfg 5): W front-end processes listen on "
                         "--port together (SO_REUSEPORT) and feed one GPU-owner process per "
                         "device (vrpms_amd.frontends.FrontEndPool); /api/tsp/sa requests are "
                         "batched into tsp_batch_sa launches")
    args = ap.parse_args(argv)
    store = MemoryStore.from_json(args.data) if args.data else MemoryStore()
    devices = [int(x) for x in args.devices.split(",")] if args.devices else None
    if devices:   # a GPU listed twice would only queue behind itself
        devices = list(dict.fromkeys(devices))
    if args.workers > 0:
        from .frontends import FrontEndPool, _default_app
        if devices and len(devices) > 1:
            # each GPU owner holds one device: large requests run on one
            print("vrpms_amd service: --workers serves every device through its own owner "
                  "process; requests are not run as an island model across --devices",
                  file=sys.stderr, flush=True)
        # --batch-tsp is implied (the owners batch /api/tsp/sa); --max-seconds
        # caps every unbatched solve in the owners' App
        pool = FrontEndPool(store, workers=args.workers, devices=devices or [args.device],
                            steps=args.batch_steps, seed=args.seed,
                            window_s=args.batch_window_ms * 1e-3, listen=(args.host, args.port),
                            app_factory=_default_app(store, args.seed, args.batch_steps,
                                                     args.max_seconds))
        print(f"vrpms_amd service ({args.workers} front-end processes) on "
              f"http://{args.host}:{pool.port}/api", flush=True)
        try:
            pool.serve_forever()
        except KeyboardInterrupt:
            pass
        finally:
            pool.close()
        return
    app = App(store, device=args.device, seed=args.seed, max_seconds=args.max_seconds,
              batch_tsp=args.batch_tsp, batch_window_s=args.batch_window_ms * 1e-3,
              batch_steps=args.batch_steps, devices=devices)
    srv = serve(app, args.host, args.port)
    print(f"vrpms_amd service on http://{args.host}:{args.port}/api", flush=True)
    try:
        srv.serve_forever()
    except KeyboardInterrupt:
        pass
    srv.server_close()


if __name__ == "__main__":
    main()
