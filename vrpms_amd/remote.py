"""The drop-in on a host without a GPU (the reference's Vercel functions,
main.py on a laptop): the front-end calls are sent to the GPU box's HTTP
host (vrpms_amd.service, POST /solve/{tsp,vrp}/<algo>) with the instance
inline, and answered by the same gfx950 kernels there.  Nothing is computed
locally -- there is no CPU solver.

Enabled by VRPMS_REMOTE=http://gpu-box:8000 (vrpms_amd.solver delegates
when that is set and no local GPU is visible), or called directly."""
from __future__ import annotations

import json
import os
import urllib.error
import urllib.request

import numpy as np


def url() -> str | None:
    return os.environ.get("VRPMS_REMOTE") or None


def _post(base: str, problem: str, algorithm: str, body: dict, timeout: float) -> dict:
    def plain(x):
        if isinstance(x, np.ndarray):
            return x.tolist()
        if isinstance(x, (np.integer,)):
            return int(x)
        raise TypeError(f"not JSON serializable: {type(x)}")
    data = json.dumps(body, default=plain).encode("utf-8")
    req = urllib.request.Request(f"{base.rstrip('/')}/solve/{problem}/{algorithm}", data=data,
                                 headers={"Content-Type": "application/json"}, method="POST")
    try:
        with urllib.request.urlopen(req, timeout=timeout) as resp:
            out = json.loads(resp.read().decode("utf-8"))
    except urllib.error.HTTPError as e:
        out = json.loads(e.read().decode("utf-8"))
    if not out.get("success"):
        reasons = "; ".join(f"{x.get('what')}: {x.get('reason')}" for x in out.get("errors", []))
        raise ValueError(reasons or "remote solve failed")
    return out["message"]


# knobs with a request name of their own (api/parameters.py:21-22); every
# other search knob of solver.solve_tsp / solve_vrp (chains, pop, islands, ...)
# travels in "knobs" and the GPU box's /solve route applies the same set
# (service.INLINE_KNOBS), so a call behaves the same with or without a local GPU
_FORWARDED = {"random_permutation_count": "randomPermutationCount",
              "iteration_count": "iterationCount"}


def _options(body: dict, seed, time_limit, knobs: dict, objective=None):
    from .service import INLINE_KNOBS
    extra = sorted(k for k in knobs if k not in _FORWARDED and k not in INLINE_KNOBS)
    if extra:
        raise ValueError(f"remote solve: unknown argument(s) {extra} "
                         f"(known: seed, time_limit, objective, "
                         f"{sorted(set(_FORWARDED) | set(INLINE_KNOBS))})")
    for k, name in _FORWARDED.items():
        if knobs.get(k):
            body[name] = int(knobs[k])
    more = {k: knobs[k] for k in INLINE_KNOBS if knobs.get(k) is not None}
    if more:
        body["knobs"] = more
    body["seed"] = int(seed)
    if time_limit is not None:
        body["timeLimit"] = float(time_limit)
    if objective is not None:
        body["objective"] = str(objective)
    return body


def solve_tsp(algorithm, durations, customers, start_node, start_time=0, *, base=None,
              timeout: float = 600.0, seed: int = 0, time_limit=None, **knobs):
    """solver.solve_tsp on the GPU box -> {'duration', 'vehicle'}."""
    body = {"durations": durations, "customers": list(customers or []),
            "startNode": start_node, "startTime": start_time}
    return _post(base or url(), "tsp", algorithm, _options(body, seed, time_limit, knobs), timeout)


def solve_vrp(algorithm, durations, locations, capacities, start_times, ignored_customers=(),
              completed_customers=(), *, base=None, timeout: float = 600.0, seed: int = 0,
              objective: str = "sum", time_limit=None, **knobs):
    """solver.solve_vrp on the GPU box -> {'durationMax', 'durationSum', 'vehicles'}."""
    body = {"durations": durations, "locations": list(locations or []),
            "capacities": list(capacities), "startTimes": list(start_times),
            "ignoredCustomers": list(ignored_customers or []),
            "completedCustomers": list(completed_customers or [])}
    return _post(base or url(), "vrp", algorithm,
                 _options(body, seed, time_limit, knobs, objective), timeout)
