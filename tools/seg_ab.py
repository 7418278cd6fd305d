#!/usr/bin/env python3
"""Steps per second per chain of the SA pricing kernels on cfg 4 (X-1000,
K - 1 separators, first-fit starts, windowed 2-opt + swap / relocate
anywhere): sa_seg_kernel (O(1) segment pricing, VRPMS_OPT_SA_ROUTE 0) vs
sa_route_kernel (route-local walks, 3), same chains and Philox streams, so
the same trajectories (checked).  usage: seg_ab.py [chains] [moves] [steps]"""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from vrpms_amd import runners, synth  # noqa: E402
from vrpms_amd.core import CVRP, Context  # noqa: E402

chains = int(sys.argv[1]) if len(sys.argv) > 1 else 256
moves = int(sys.argv[2]) if len(sys.argv) > 2 else 128
steps = int(sys.argv[3]) if len(sys.argv) > 3 else 2000
ctx = Context(0)
x = synth.x_style(1000, seed=0)
ctx.set_instance(CVRP, x.durations, x.demand, x.capacities, x.start_times)
res = {}
for mode in (0, 3):
    ctx.set_sa_route(mode)
    r = runners.SARunner(ctx, x.n, chains=chains, total_steps=steps, durations=x.durations,
                         n_sep=x.K - 1, window=32, window_types=2, start="pack", moves=moves)
    r.epoch(20)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    r.epoch(steps)
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    k, _ = r.best()
    res[mode] = (r.cur.cpu(), r.cur_key.cpu(), k)
    print(f"mode {mode} ({'seg' if mode == 0 else 'route walks'}): chains {chains} moves {moves}: "
          f"{steps / dt:,.0f} steps/s per chain, best {k >> 28 & (2**28 - 1)}", flush=True)
ctx.set_sa_route(0)
same = torch.equal(res[0][0], res[3][0]) and torch.equal(res[0][1], res[3][1])
print("identical trajectories:", same)
