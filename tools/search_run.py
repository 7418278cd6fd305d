#!/usr/bin/env python3
"""Run only the search kernels on their bench workloads, a few launches each
-- a short target for rocprofv3 --pmc passes:
  cfg 5: tsp_batch_sa_kernel, 10,000 TSP-50 requests x 1000 SA steps
  cfg 2: sa_packed_kernel, 4096 SA chains on CVRP-100 K = 8, 400-step epochs
usage: search_run.py [reps]"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import numpy as np  # noqa: E402
import torch  # noqa: E402

from vrpms_amd import runners, synth  # noqa: E402
from vrpms_amd.core import CVRP, Context  # noqa: E402

reps = int(sys.argv[1]) if len(sys.argv) > 1 else 3
ctx = Context(0)
rng = np.random.default_rng(0)
mats = torch.tensor(np.stack([synth.random_symmetric(50, rng) for _ in range(10000)]),
                    dtype=torch.int32, device=ctx.dev)
for _ in range(reps):
    ctx.tsp_batch_sa(mats, 1000, 1 / 80.0, 1 / 0.995, 1)
torch.cuda.synchronize()
del mats

inst = synth.cvrp(100, 8, seed=0)
ctx.set_instance(CVRP, inst.durations, inst.demand, inst.capacities, inst.start_times)
r = runners.SARunner(ctx, inst.n, chains=4096, total_steps=400 * reps, durations=inst.durations)
for _ in range(reps):
    r.epoch(400)
torch.cuda.synchronize()
print("done", r.best()[0])
