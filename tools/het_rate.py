#!/usr/bin/env python3
"""Heterogeneous-fleet SA on cfg 4's size: X-1000 with three capacity classes
(1.4 / 1.1 / 0.9 x the uniform capacity, in vehicle order) and staggered
start times, K - 1 first-fit separators, windowed 2-opt + swap / relocate
anywhere.  Steps per second per chain of sa_seg_kernel's heterogeneous
variant against the full re-evaluation kernel it replaces (sa_kernel,
ctx.set_sa_route(2)), and whether both follow the same trajectories.
With --td: the reference's normal VRP request shape instead -- the
hour-indexed TD-200 x 24 (time_of_day, src/solver.py:7) with three capacity
classes (1.3 / 1.0 / 0.8) and staggered start times: sa_route_kernel's
heterogeneous variant (walks re-synchronise on the same vehicle) against
sa_kernel.
usage: het_rate.py [chains] [steps] [--td]"""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import numpy as np  # noqa: E402
import torch  # noqa: E402

from vrpms_amd import runners, synth  # noqa: E402
from vrpms_amd.core import CVRP, Context  # noqa: E402

TD = "--td" in sys.argv
argv = [a for a in sys.argv[1:] if not a.startswith("--")]
chains = int(argv[0]) if len(argv) > 0 else 256
steps = int(argv[1]) if len(argv) > 1 else 400
x = synth.td_cvrp(200, 16, seed=0) if TD else synth.x_style(1000, seed=0)
K, base = len(x.capacities), int(x.capacities[0])
fr = (1.3, 1.0, 0.8) if TD else (1.4, 1.1, 0.9)
caps = np.array([max(int(base * fr[k * 3 // K]), int(x.demand.max())) for k in range(K)])
starts = np.arange(K, dtype=np.int64) * 37 % 240 + (420 if TD else 0)
window = 16 if TD else 32
if os.environ.get("VRPMS_LIB"):  # an A/B build (e.g. build_ab/het8/libvrpms.so)
    from vrpms_amd import _lib
    _lib.load(os.environ["VRPMS_LIB"])
ctx = Context(0)
ctx.set_instance(CVRP, x.durations, x.demand, caps, starts)
out = {}
fast = "sa_route_kernel (heterogeneous, same-vehicle resync)" if TD else \
    "sa_seg_kernel (heterogeneous)"
for mode, label in ((0, fast), (2, "sa_kernel (full re-evaluation)")):
    ctx.set_sa_route(mode)
    r = runners.SARunner(ctx, x.n, chains=chains, total_steps=steps + 10, durations=x.durations,
                         n_sep=K - 1, window=window, window_types=2, start="pack", moves=64)
    r.epoch(10)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    r.epoch(steps)
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    out[mode] = (r.cur.cpu(), r.cur_key.cpu())
    out[f"rate{mode}"] = steps / dt
    print(f"{label}: {steps / dt:,.0f} steps/s per chain ({chains} chains x 64 moves), "
          f"best {r.best()[0] >> 28 & (2**28 - 1)} (unvisited {r.best()[0] >> 56})", flush=True)
print("same trajectories:", torch.equal(out[0][0], out[2][0]) and torch.equal(out[0][1], out[2][1]),
      f"speed-up {out['rate0'] / out['rate2']:.2f}x")
ctx.set_sa_route(0)
