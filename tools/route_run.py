#!/usr/bin/env python3
"""sa_route_kernel alone on its cfg-4 workload (X-1000, 2048 chains, K - 1
separators, first-fit start, windowed 2-opt), a few launches -- a short
target for rocprofv3 --pmc / --stats passes.  usage: route_run.py [launches]"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from vrpms_amd import runners, synth  # noqa: E402
from vrpms_amd.core import CVRP, Context  # noqa: E402

reps = int(sys.argv[1]) if len(sys.argv) > 1 else 3
ctx = Context(0)
x = synth.x_style(1000, seed=0)
ctx.set_instance(CVRP, x.durations, x.demand, x.capacities, x.start_times)
r = runners.SARunner(ctx, x.n, chains=2048, total_steps=300 * reps, durations=x.durations,
                     n_sep=x.K - 1, window=32, window_types=2, start="pack")
for _ in range(reps):
    r.epoch(300)
torch.cuda.synchronize()
print("done", r.best()[0] >> 28 & (2 ** 28 - 1))
