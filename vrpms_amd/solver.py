"""Drop-in solver front-end for the vrpms HTTP handlers.

Keeps the reference's entry points and result schema:
  calculate_duration(source, target, time_of_day=0)   src/solver.py:7-15
  solve_vrp_problem(**instance)                       src/solver.py:18-27
and adds the two calls the eight handler TODO slots make:
  solve_tsp(algorithm, durations, customers, start_node, start_time, ...)
      -> {'duration': int, 'vehicle': [node, ...]}     api/tsp/ga/index.py:40-44
  solve_vrp(algorithm, durations, locations, capacities, start_times,
            ignored_customers, completed_customers, ...)
      -> {'durationMax': int, 'durationSum': int,
          'vehicles': [{'tour': [0, ..., 0], 'duration': int}, ...]}
                                                       api/vrp/ga/index.py:48-53
`algorithm` is the endpoint name: 'bf', 'ga', 'sa' or 'aco'.  All search
and scoring runs in the gfx950 kernels (vrpms_amd.core); this module only
builds the compact instance and maps results
back to matrix indices.  Node ids in results are matrix row indices
(A1), the depot / start node closing every tour as in src/solver.py:24.
"""
from __future__ import annotations

import datetime
import random
import threading
import time
from dataclasses import dataclass

import numpy as np

from . import runners
from .core import CVRP, OBJ_MAX, OBJ_SUM, TSP, Context

ALGORITHMS = ("bf", "ga", "sa", "aco")
# exhaustive search over n! giant tours: 13! = 6.2 G tours is ~0.1 s at the
# measured ~64 G evals/s of bf_kernel on one MI355X (bench "search.bf") on a
# static matrix; an hour-indexed one prices every edge at its departure
# hour (several times slower), so it keeps 11 (39.9 M tours).
# vrpms_bf_run itself accepts n <= 15 (nibble-packed tours)
BF_MAX_CUSTOMERS = 13
BF_MAX_CUSTOMERS_TD = 11
# SA on tours of more than SA_WINDOW_MIN_N customers samples A11 windowed
# moves (second position within SA_WINDOW of the first)
SA_WINDOW, SA_WINDOW_MIN_N = 32, 150


@dataclass
class CompactInstance:
    problem: int
    durations: np.ndarray      # int64 [H][N][N] over compact nodes
    nodes: list                # compact index -> original matrix index
    demand: np.ndarray | None
    capacities: np.ndarray | None
    start_times: np.ndarray

    @property
    def N(self):
        return len(self.nodes)

    @property
    def n(self):
        return self.N - 1


def _matrix(durations) -> np.ndarray:
    """A2/A3: the DB `matrix` payload (api/database.py:45) as int64 [H][N][N]."""
    D = np.asarray(durations)
    if D.dtype == object:
        raise ValueError("duration matrix must be rectangular")
    if D.ndim == 2:
        D = D[None]
    if D.ndim != 3 or D.shape[1] != D.shape[2] or D.shape[1] == 0:
        raise ValueError("duration matrix must be [N][N] or [24][N][N]")
    if D.shape[0] not in (1, 24):
        raise ValueError("hour-indexed duration matrix must have 24 slices")
    if np.issubdtype(D.dtype, np.integer):       # the DB's JSON integers: one check
        if D.size and D.min() < 0:
            raise ValueError("durations must be non-negative integers (minutes)")
        return D.astype(np.int64, copy=False)
    if not np.issubdtype(D.dtype, np.number) or not np.all(np.isfinite(D)):
        raise ValueError("durations must be numbers")
    if np.any(D != np.floor(D)) or np.any(D < 0):
        raise ValueError("durations must be non-negative integers (minutes)")
    return D.astype(np.int64)


def compact_tsp(durations, customers, start_node, start_time=0) -> CompactInstance:
    """A4: node 0 = startNode, then the distinct customers in request order."""
    D = _matrix(durations)
    N = D.shape[1]
    start = int(start_node)
    if not 0 <= start < N:
        raise ValueError(f"startNode {start} outside the {N}-node matrix")
    nodes = [start]
    seen = {start}
    for c in customers or []:
        c = int(c)
        if not 0 <= c < N:
            raise ValueError(f"customer {c} outside the {N}-node matrix")
        if c not in seen:
            seen.add(c)
            nodes.append(c)
    # every node in matrix order (the common request): no copy
    sub = D if nodes == list(range(N)) else D[:, nodes][:, :, nodes]
    return CompactInstance(TSP, sub, nodes, None, None, np.array([int(start_time or 0)]))


def active_customers(locations, ignored_customers, completed_customers):
    """Rows i >= 1 whose location id is not ignored/completed: the solver's
    view of remove_unused_locations (api/helpers.py:11-13); the depot (row 0,
    A1) always stays."""
    disregard = list(ignored_customers or []) + list(completed_customers or [])
    return [i for i, loc in enumerate(locations) if i > 0 and loc.get("id") not in disregard]


def compact_vrp(durations, locations, capacities, start_times, ignored_customers=(),
                completed_customers=()) -> CompactInstance:
    """A1/A5: depot = node 0, customers = active locations; demand defaults to 1."""
    D = _matrix(durations)
    N = D.shape[1]
    locations = list(locations or [])
    if len(locations) != N:
        raise ValueError(f"{len(locations)} locations but a {N}-node duration matrix")
    caps = [int(c) for c in (capacities if capacities is not None else [])]
    starts = [int(s) for s in (start_times if start_times is not None else [])]
    if not caps:
        raise ValueError("at least one vehicle capacity is required")
    if len(starts) != len(caps):
        raise ValueError("capacities and startTimes must have the same length")
    if min(caps) < 0 or min(starts) < 0:
        raise ValueError("capacities and start times must be non-negative")
    nodes = [0] + active_customers(locations, ignored_customers, completed_customers)
    dem = np.array([0] + [int(locations[i].get("demand", 1)) for i in nodes[1:]], dtype=np.int64)
    if dem.min() < 0:
        raise ValueError("demands must be non-negative")
    sub = D[:, nodes][:, :, nodes]
    return CompactInstance(CVRP, sub, nodes, dem, np.array(caps), np.array(starts))


# ---------------------------------------------------------------------------
# device context (one per process; the handlers call in sequentially)
# ---------------------------------------------------------------------------
_CTX: dict = {}
_CTX_LOCK = threading.Lock()


def context(device: int = 0) -> Context:
    """The process-wide context on `device`, one per device (created once;
    the check and the creation are one critical section, so concurrent first
    calls from the request threads and the batcher share a single vrpms_ctx
    per device)."""
    with _CTX_LOCK:
        ctx = _CTX.get(device)
        if ctx is None:
            ctx = _CTX[device] = Context(device)
        return ctx


def load(ctx: Context, ci: CompactInstance, objective: int = OBJ_SUM):
    if ci.problem == TSP:
        ctx.set_instance(TSP, ci.durations, start_times=ci.start_times, objective=objective)
    else:
        ctx.set_instance(CVRP, ci.durations, ci.demand, ci.capacities, ci.start_times,
                         objective=objective)


def _runner(ctx: Context, ci: CompactInstance, algorithm: str, seed: int, knobs: dict):
    """(runner, epochs) for SA / GA / ACO on the loaded instance."""
    n = ci.n
    iters = knobs.get("iteration_count")
    if algorithm == "sa":
        steps = int(iters or knobs.get("steps", 4000))
        # VRP: K - 1 route separators (A10) let the moves place route
        # boundaries instead of leaving them to the greedy split alone
        n_sep = int(knobs.get("separators", len(ci.capacities) - 1 if ci.problem == CVRP else 0))
        # large tours: A11/A12 windowed 2-opt, swap / relocate anywhere
        # (priced in O(1) / route-locally); separators start where first-fit
        # routes end (a feasible start on a tight fleet, where random
        # separator positions would leave customers unserved)
        window = int(knobs.get("window", SA_WINDOW if n > SA_WINDOW_MIN_N else 0))
        r = runners.SARunner(ctx, n, chains=int(knobs.get("chains", 1024)), seed=seed,
                             total_steps=steps, durations=ci.durations, n_sep=n_sep,
                             window=window, window_types=int(knobs.get("window_types", 2)),
                             start="pack" if n_sep > 0 else "random")
        return r, max(1, steps // r.steps_per_epoch)
    if algorithm == "ga":
        pop = int(knobs.get("random_permutation_count") or knobs.get("pop", 256))
        gens = int(iters or 400)
        r = runners.GARunner(ctx, n, islands=int(knobs.get("islands", 8)), pop=max(2, min(pop, 4096)),
                             seed=seed)
        return r, max(1, gens // r.gens_per_epoch)
    if algorithm == "aco":
        its = int(iters or 100)
        r = runners.ACORunner(ctx, n, colonies=int(knobs.get("colonies", 4)),
                              ants=int(knobs.get("ants", 64)), seed=seed)
        return r, max(1, its // r.iters_per_epoch)
    raise ValueError(f"unknown algorithm {algorithm!r}; expected one of {ALGORITHMS}")


def search_islands(ci: CompactInstance, algorithm: str, devices, seed: int = 0,
                   time_limit: float | None = None, objective: int = OBJ_SUM, **knobs):
    """The island model inside one process: one SA / GA / ACO
    island per device (seed + 1000 d), the same epochs enqueued on every
    device, the E best migrating every 5 epochs device to device
    (islands.exchange_local).  -> (key, compact giant tour) of the best
    island."""
    import torch
    from . import islands
    if ci.n <= 1 or algorithm == "bf":
        raise ValueError("search_islands: SA / GA / ACO on two or more customers")
    rs, epochs = [], 1
    for d, dev in enumerate(devices):
        ctx = context(dev)
        load(ctx, ci, objective)
        r, epochs = _runner(ctx, ci, algorithm, seed + 1000 * d, knobs)
        rs.append(r)

    def sync():
        for dev in devices:
            torch.cuda.synchronize(dev)
    key, tour = islands.run_local(rs, epochs, exchange_every=5, E=min(8, rs[0].src()[1].numel()),
                                  time_limit=time_limit, sync=sync if time_limit else None)
    return key, [int(x) for x in tour.cpu().tolist()]


def search(ctx: Context, ci: CompactInstance, algorithm: str, seed: int = 0,
           time_limit: float | None = None, **knobs):
    """Run one algorithm on the loaded instance -> (key, compact giant tour)."""
    n = ci.n
    if n == 0:
        return None, []
    if n == 1:
        return None, [1]
    if algorithm == "bf":
        cap = BF_MAX_CUSTOMERS if ci.durations.shape[0] == 1 else BF_MAX_CUSTOMERS_TD
        if n > cap:
            raise ValueError(f"brute force supports at most {cap} customers "
                             f"({n} given)")
        return runners.brute_force(ctx, n)
    r, epochs = _runner(ctx, ci, algorithm, seed, knobs)
    t0 = time.perf_counter()
    e = 0
    while True:
        r.epoch()
        e += 1
        if time_limit is not None:
            if time.perf_counter() - t0 >= time_limit:
                break
        elif e >= epochs:
            break
    key, tour = r.best()
    return key, [int(x) for x in tour.cpu().tolist()]


def _decode(ctx: Context, tour):
    import torch
    t = torch.tensor(tour, dtype=torch.int16, device=ctx.dev)
    return ctx.decode(t, len(tour))


def _remote():
    """VRPMS_REMOTE set and no local GPU: the GPU box's URL (vrpms_amd.remote)."""
    from . import remote
    if remote.url() is None:
        return None
    import torch
    return None if torch.cuda.is_available() else remote


def _searched(ci, algorithm, seed, time_limit, device, devices, objective, knobs):
    """(context holding the instance, compact tour): one device, or the
    island model across `devices` (two or more) for SA / GA / ACO."""
    if devices is not None and len(devices) > 1 and algorithm != "bf" and ci.n > 1:
        _, tour = search_islands(ci, algorithm, list(devices), seed=seed, time_limit=time_limit,
                                 objective=objective, **knobs)
        return context(devices[0]), tour
    ctx = context(device)
    load(ctx, ci, objective)
    _, tour = search(ctx, ci, algorithm, seed=seed, time_limit=time_limit, **knobs)
    return ctx, tour


def solve_tsp(algorithm: str, durations, customers, start_node, start_time=0, *, seed: int = 0,
              time_limit: float | None = None, device: int = 0, devices=None, **knobs) -> dict:
    """Result dict of the TSP TODO slot (api/tsp/ga/index.py:40-44).
    `devices` (two or more): SA / GA / ACO as an island model across them."""
    rem = _remote()
    if rem is not None:
        return rem.solve_tsp(algorithm, durations, customers, start_node, start_time, seed=seed,
                             time_limit=time_limit, **knobs)
    ci = compact_tsp(durations, customers, start_node, start_time)
    ctx, tour = _searched(ci, algorithm, seed, time_limit, device, devices, OBJ_SUM, knobs)
    _, dur = _decode(ctx, tour)
    vehicle = [ci.nodes[0]] + [ci.nodes[c] for c in tour] + [ci.nodes[0]]
    return {"duration": int(dur[0]), "vehicle": vehicle}


def solve_vrp(algorithm: str, durations, locations, capacities, start_times,
              ignored_customers=(), completed_customers=(), *, seed: int = 0,
              objective: str = "sum", time_limit: float | None = None, device: int = 0,
              devices=None, with_unvisited: bool = False, **knobs) -> dict:
    """Result dict of the VRP TODO slot (api/vrp/ga/index.py:48-53); A7 shapes.
    `devices` (two or more): SA / GA / ACO as an island model across them."""
    rem = _remote()
    if rem is not None:
        out = rem.solve_vrp(algorithm, durations, locations, capacities, start_times,
                            ignored_customers, completed_customers, seed=seed,
                            objective=objective, time_limit=time_limit, **knobs)
        if with_unvisited:   # the served customers' complement (the remote answers the slot dict)
            served = {c for v in out["vehicles"] for c in v["tour"][1:-1]}
            nodes = [0] + active_customers(list(locations or []), ignored_customers,
                                           completed_customers)
            out["unvisited"] = [c for c in nodes[1:] if c not in served]
        return out
    ci = compact_vrp(durations, locations, capacities, start_times, ignored_customers,
                     completed_customers)
    ctx, tour = _searched(ci, algorithm, seed, time_limit, device, devices,
                          OBJ_MAX if objective == "max" else OBJ_SUM, knobs)
    K = len(ci.capacities)
    routes = [[] for _ in range(K)]
    unvisited = []
    if tour:
        veh, durs = _decode(ctx, tour)
        for c, v in zip(tour, veh):
            if v == -2:                # A10 separator: a route boundary, not a customer
                continue
            (routes[v] if v >= 0 else unvisited).append(ci.nodes[c])
    else:
        durs = [0] * K
    vehicles = [{"tour": [ci.nodes[0]] + r + [ci.nodes[0]], "duration": int(d)}
                for r, d in zip(routes, durs)]
    out = {"durationMax": int(max(durs) if durs else 0), "durationSum": int(sum(durs)),
           "vehicles": vehicles}
    if with_unvisited:
        out["unvisited"] = unvisited
    return out


# ---------------------------------------------------------------------------
# reference entry points (src/solver.py)
# ---------------------------------------------------------------------------
_LOOKUP = None


def set_duration_matrix(durations, location_ids=None):
    """Back calculate_duration with a loaded matrix."""
    global _LOOKUP
    D = _matrix(durations)
    ids = list(location_ids) if location_ids is not None else list(range(D.shape[1]))
    _LOOKUP = (D, {v: i for i, v in enumerate(ids)})


def calculate_duration(source, target, time_of_day: int = 0):
    """src/solver.py:7-15 signature and return dict.  With a matrix loaded
    (set_duration_matrix) this is the A3 lookup D[(t // 60) % H][s][t];
    without one it keeps the reference's stub behaviour (randint(3, 320))."""
    if _LOOKUP is None:
        duration = random.randint(3, 320)
    else:
        D, index = _LOOKUP
        h = (int(time_of_day) // 60) % D.shape[0]
        duration = int(D[h, index[source], index[target]])
    return {"source": source, "target": target, "duration": duration, "units": "minutes"}


def get_current_date():
    """src/utilities/helper.py:4-6."""
    return datetime.date.today().strftime("%d-%m-%Y")


def solve_vrp_problem(durations=None, locations=None, capacities=None, start_times=None,
                      ignored_customers=(), completed_customers=(), algorithm: str = "sa",
                      seed: int | None = None, **knobs):
    """src/solver.py:18-27 return shape: {'tour','total_time','unvisited','date'}.

    With no instance (the reference's no-argument call from main.py) a
    random symmetric 15-node matrix (randint(3, 320), src/solver.py:12) is
    solved as a single-vehicle tour over customers 1..14 (src/solver.py:22-24).
    `tour` concatenates the vehicle routes; `total_time` is durationSum."""
    if durations is None:
        rng = random.Random(seed)
        N = 15
        D = np.zeros((N, N), dtype=np.int64)
        for i in range(N):
            for j in range(i + 1, N):
                D[i, j] = D[j, i] = rng.randint(3, 320)
        durations = D
        locations = [{"id": i} for i in range(N)]
        capacities = [N]
        start_times = [0]
    res = solve_vrp(algorithm, durations, locations, capacities, start_times, ignored_customers,
                    completed_customers, seed=seed or 0, with_unvisited=True, **knobs)
    depot = res["vehicles"][0]["tour"][0] if res["vehicles"] else 0
    tour = [depot]
    for v in res["vehicles"]:
        if len(v["tour"]) > 2:
            tour += v["tour"][1:]          # route customers, back to the depot
    if len(tour) == 1:
        tour.append(depot)
    return {"tour": tour, "total_time": res["durationSum"], "unvisited": res["unvisited"],
            "date": get_current_date()}


__all__ = ["ALGORITHMS", "calculate_duration", "solve_vrp_problem", "solve_tsp", "solve_vrp",
           "compact_tsp", "compact_vrp", "active_customers", "set_duration_matrix",
           "get_current_date"]
