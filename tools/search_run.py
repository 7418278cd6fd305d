#!/usr/bin/env python3
"""Run only the search kernels on their bench workloads, a few launches each
-- a short target for rocprofv3 --pmc / --stats passes:
  cfg 5: tsp_batch_sa_kernel, 10,000 TSP-50 requests x 1000 SA steps
  cfg 2: sa_packed_kernel, 4096 SA chains on CVRP-100 K = 8, 400-step epochs
  cfg 2: ga_fused_kernel, 256 islands x 256, 20 generations per call
  cfg 2: aco_construct_kernel, 64 colonies x 64 ants, 5 iterations per epoch
         (one construct launch per iteration: n = 100 ant steps)
  cfg 4: sa_seg_kernel, 1024 SA chains x 128 moves on X-1000 with K - 1
         separators (first-fit start, windowed 2-opt), 100-step epochs
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
ga = runners.GARunner(ctx, inst.n, islands=256, pop=256, seed=1, gens_per_epoch=20)
for _ in range(reps):
    ga.epoch()
aco = runners.ACORunner(ctx, inst.n, colonies=64, ants=64, seed=1, iters_per_epoch=5)
for _ in range(reps):
    aco.epoch()
torch.cuda.synchronize()
x = synth.x_style(1000, seed=0)
ctx.set_instance(CVRP, x.durations, x.demand, x.capacities, x.start_times)
rx = runners.SARunner(ctx, x.n, chains=1024, total_steps=100 * reps, durations=x.durations,
                      n_sep=x.K - 1, window=32, window_types=2, start="pack", moves=128)
for _ in range(reps):
    rx.epoch(100)
torch.cuda.synchronize()
print("done", r.best()[0], ga.best()[0], aco.best()[0], rx.best()[0])
