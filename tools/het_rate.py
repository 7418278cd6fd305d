#!/usr/bin/env python3
"""Heterogeneous-fleet SA on cfg 4's size: X-1000 with three capacity classes
(1.4 / 1.1 / 0.9 x the uniform capacity, in vehicle order) and staggered
start times, K - 1 first-fit separators, windowed 2-opt + swap / relocate
anywhere.  Steps per second per chain of sa_seg_kernel's heterogeneous
variant against the full re-evaluation kernel it replaces (sa_kernel,
ctx.set_sa_route(2)), and whether both follow the same trajectories.
usage: het_rate.py [chains] [steps]"""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import numpy as np  # noqa: E402
import torch  # noqa: E402

from vrpms_amd import runners, synth  # noqa: E402
from vrpms_amd.core import CVRP, Context  # noqa: E402

chains = int(sys.argv[1]) if len(sys.argv) > 1 else 256
steps = int(sys.argv[2]) if len(sys.argv) > 2 else 400
x = synth.x_style(1000, seed=0)
K, base = len(x.capacities), int(x.capacities[0])
caps = np.array([max(int(base * (1.4, 1.1, 0.9)[k * 3 // K]), int(x.demand.max())) for k in range(K)])
starts = np.arange(K, dtype=np.int64) * 37 % 240
ctx = Context(0)
ctx.set_instance(CVRP, x.durations, x.demand, caps, starts)
out = {}
for mode, label in ((0, "sa_seg_kernel (heterogeneous)"), (2, "sa_kernel (full re-evaluation)")):
    ctx.set_sa_route(mode)
    r = runners.SARunner(ctx, x.n, chains=chains, total_steps=steps + 10, durations=x.durations,
                         n_sep=K - 1, window=32, window_types=2, start="pack", moves=64)
    r.epoch(10)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    r.epoch(steps)
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    out[mode] = (r.cur.cpu(), r.cur_key.cpu())
    print(f"{label}: {steps / dt:,.0f} steps/s per chain ({chains} chains x 64 moves), "
          f"best {r.best()[0] >> 28 & (2**28 - 1)} (unvisited {r.best()[0] >> 56})", flush=True)
print("same trajectories:", torch.equal(out[0][0], out[2][0]) and torch.equal(out[0][1], out[2][1]))
ctx.set_sa_route(0)
