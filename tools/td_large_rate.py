#!/usr/bin/env python3
"""Which SA kernel should take hour-indexed requests too large for
sa_td_kernel's LDS rows: steps per second per chain of
sa_route_kernel with per-vehicle capacities / start times (option 3,
RouteHK) against sa_kernel's full L2 walks (option 2) on TD-n x 24 with
three capacity classes (1.3 / 1.0 / 0.8) and staggered starts -- the
reference's normal VRP request (api/vrp/sa/index.py:40-45, capacities /
startTimes api/parameters.py:11-12) -- plus what the automatic dispatch
(option 0) picks; trajectories checked equal across the kernels.
usage: td_large_rate.py [chains] [steps] [n ...]"""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import numpy as np  # noqa: E402
import torch  # noqa: E402

from vrpms_amd import runners, synth  # noqa: E402
from vrpms_amd.core import CVRP, Context  # noqa: E402

argv = sys.argv[1:]
chains = int(argv[0]) if len(argv) > 0 else 256
steps = int(argv[1]) if len(argv) > 1 else 60
sizes = [int(x) for x in argv[2:]] or [400, 600, 800, 1000]
# FLEET=uniform: one capacity, one start time (sa_route_kernel's exchangeable
# fleet, RouteK) instead of the heterogeneous one
uniform = os.environ.get("FLEET") == "uniform"
ctx = Context(0)
rows = []
for n in sizes:
    K = max(8, n // 20)
    x = synth.td_cvrp(n, K, seed=0)
    base = int(x.capacities[0])
    fr = (1.3, 1.0, 0.8)
    caps = np.array([max(int(base * fr[k * 3 // K]), int(x.demand.max())) for k in range(K)])
    starts = np.arange(K, dtype=np.int64) * 37 % 240 + 420
    if uniform:
        caps, starts = x.capacities, x.start_times
    ctx.set_instance(CVRP, x.durations, x.demand, caps, starts)
    out, rates = {}, {}
    for mode in (0, 3, 2):
        ctx.set_sa_route(mode)
        try:
            r = runners.SARunner(ctx, x.n, chains=chains, total_steps=steps + 4,
                                 durations=x.durations, n_sep=K - 1, window=32, window_types=2,
                                 start="pack", moves=64)
            r.epoch(4)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            r.epoch(steps)
            torch.cuda.synchronize()
            dt = time.perf_counter() - t0
        finally:
            ctx.set_sa_route(0)
        out[mode] = (r.cur.cpu(), r.cur_key.cpu())
        rates[mode] = steps / dt
        print(f"TD-{n} x 24 {'uniform' if uniform else 'het'} K={K}: option {mode}: {steps / dt:,.1f} steps/s per chain",
              flush=True)
    same = all(torch.equal(out[0][0], out[m][0]) and torch.equal(out[0][1], out[m][1])
               for m in out)
    row = {"n": n, "K": K, "fleet": "uniform" if uniform else "het", "chains": chains, "steps": steps, "auto": rates[0],
           "route": rates[3], "sa_kernel": rates[2], "route_over_sa": rates[3] / rates[2],
           "same_trajectories": same}
    rows.append(row)
    print(json.dumps(row), flush=True)
ctx.close()
print(json.dumps({"td_large_rate": rows}))
