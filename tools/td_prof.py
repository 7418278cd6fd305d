#!/usr/bin/env python3
"""One sa_td_kernel launch shape for profiling (rocprofv3 --kernel-trace /
--pmc): heterogeneous TD-200 x 24 (three capacity classes, staggered starts),
first-fit starts, windowed 2-opt + swap / relocate anywhere.
usage: td_prof.py [chains] [steps] [moves] [mode]   (mode 4 = sa_td_kernel,
2 = sa_kernel, 3 = sa_route_kernel)"""
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
steps = int(argv[1]) if len(argv) > 1 else 400
moves = int(argv[2]) if len(argv) > 2 else 64
mode = int(argv[3]) if len(argv) > 3 else 4
x = synth.td_cvrp(200, 16, seed=0)
K, base = len(x.capacities), int(x.capacities[0])
fr = (1.3, 1.0, 0.8)
caps = np.array([max(int(base * fr[k * 3 // K]), int(x.demand.max())) for k in range(K)])
starts = np.arange(K, dtype=np.int64) * 37 % 240 + 420
ctx = Context(0)
ctx.set_instance(CVRP, x.durations, x.demand, caps, starts)
ctx.set_sa_route(mode)
r = runners.SARunner(ctx, x.n, chains=chains, total_steps=2 * steps + 10, durations=x.durations,
                     n_sep=K - 1, window=16, window_types=2, start="pack", moves=moves)
r.epoch(10)
torch.cuda.synchronize()
for rep in range(2):
    t0 = time.perf_counter()
    r.epoch(steps)
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    print(f"mode {mode}: {steps / dt:,.0f} steps/s per chain ({chains} x {moves}), "
          f"best {r.best()[0] >> 28 & (2**28 - 1)}", flush=True)
ctx.set_sa_route(0)
ctx.close()
