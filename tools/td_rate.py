#!/usr/bin/env python3
"""SA steps per second per chain on the hour-indexed TD-200 x 24 (the
reference's normal VRP request shape: time_of_day, src/solver.py:7;
per-vehicle capacities / start times, api/parameters.py:11-12) for every SA
kernel that takes it: sa_td_kernel (option 4, LDS hour rows), sa_route_kernel
(option 3, route-local walks) and sa_kernel (option 2, L2 full walks), on a
heterogeneous fleet (three capacity classes 1.3 / 1.0 / 0.8, staggered
starts) and a uniform one; same trajectories checked across kernels.
usage: td_rate.py [chains] [steps] [moves]"""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import numpy as np  # noqa: E402
import torch  # noqa: E402

from vrpms_amd import runners, synth  # noqa: E402
from vrpms_amd.core import CVRP, Context  # noqa: E402

argv = [a for a in sys.argv[1:] if not a.startswith("--")]
chains = int(argv[0]) if len(argv) > 0 else 256
steps = int(argv[1]) if len(argv) > 1 else 400
moves = int(argv[2]) if len(argv) > 2 else 64
ctx = Context(0)
for fleet in ("het", "uniform"):
    x = synth.td_cvrp(200, 16, seed=0)
    K, base = len(x.capacities), int(x.capacities[0])
    caps, starts = x.capacities, x.start_times
    if fleet == "het":
        fr = (1.3, 1.0, 0.8)
        caps = np.array([max(int(base * fr[k * 3 // K]), int(x.demand.max())) for k in range(K)])
        starts = np.arange(K, dtype=np.int64) * 37 % 240 + 420
    ctx.set_instance(CVRP, x.durations, x.demand, caps, starts)
    out = {}
    for mode, label in ((4, "sa_td_kernel (LDS hour rows)"), (3, "sa_route_kernel"),
                        (2, "sa_kernel (L2 walks)")):
        if mode == 2 and moves > 64:
            continue
        ctx.set_sa_route(mode)
        try:
            r = runners.SARunner(ctx, x.n, chains=chains, total_steps=steps + 10,
                                 durations=x.durations, n_sep=K - 1, window=16, window_types=2,
                                 start="pack", moves=moves)
            r.epoch(10)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            r.epoch(steps)
            torch.cuda.synchronize()
            dt = time.perf_counter() - t0
        finally:
            ctx.set_sa_route(0)
        out[mode] = (r.cur.cpu(), r.cur_key.cpu())
        out[f"rate{mode}"] = steps / dt
        print(f"{fleet}: {label}: {steps / dt:,.0f} steps/s per chain ({chains} chains x {moves} "
              f"moves), best {r.best()[0] >> 28 & (2**28 - 1)} (unvisited {r.best()[0] >> 56})",
              flush=True)
    same = all(torch.equal(out[4][0], out[m][0]) and torch.equal(out[4][1], out[m][1])
               for m in out if isinstance(m, int))
    ref = out.get("rate2") or out.get("rate3")
    print(f"{fleet}: same trajectories: {same}; sa_td / sa_kernel "
          f"{out['rate4'] / out['rate2'] if 'rate2' in out else float('nan'):.2f}x, "
          f"sa_td / sa_route {out['rate4'] / out['rate3']:.2f}x", flush=True)
ctx.close()
