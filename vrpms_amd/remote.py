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


def solve_tsp(algorithm, durations, customers, start_node, start_time=0, *, base=None,
              timeout: float = 600.0, **_):
    """solver.solve_tsp on the GPU box -> {'duration', 'vehicle'}."""
    return _post(base or url(), "tsp", algorithm,
                 {"durations": durations, "customers": list(customers or []),
                  "startNode": start_node, "startTime": start_time}, timeout)


def solve_vrp(algorithm, durations, locations, capacities, start_times, ignored_customers=(),
              completed_customers=(), *, base=None, timeout: float = 600.0, **knobs):
    """solver.solve_vrp on the GPU box -> {'durationMax', 'durationSum', 'vehicles'}."""
    body = {"durations": durations, "locations": list(locations or []),
            "capacities": list(capacities), "startTimes": list(start_times),
            "ignoredCustomers": list(ignored_customers or []),
            "completedCustomers": list(completed_customers or [])}
    if knobs.get("random_permutation_count"):
        body["randomPermutationCount"] = int(knobs["random_permutation_count"])
    if knobs.get("iteration_count"):
        body["iterationCount"] = int(knobs["iteration_count"])
    return _post(base or url(), "vrp", algorithm, body, timeout)
