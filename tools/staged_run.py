#!/usr/bin/env python3
"""Run only the L2-tier scoring kernel (eval_staged) on BASELINE.json cfg 3
(TD-VRP-200 x 24 h, u8 tours, C = 2 Mi) and cfg 4 (X-style CVRP-1000, u16
tours, C = 256 Ki), `reps` launches each -- a short target for rocprofv3
--pmc passes (L2 hit rate: TCC_HIT / TCC_MISS; HBM: FETCH_SIZE).
usage: staged_run.py [reps]"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

import bench  # noqa: E402
from vrpms_amd import synth  # noqa: E402
from vrpms_amd.core import CVRP, Context  # noqa: E402

reps = int(sys.argv[1]) if len(sys.argv) > 1 else 3
ctx = Context(0)
dev = ctx.dev

td = synth.td_cvrp(200, 16, seed=0)
ctx.set_instance(CVRP, td.durations, td.demand, td.capacities, td.start_times)
C = 1 << 21
perms = bench.make_batch(ctx, C, td.n, 11)
keys = torch.empty(C, dtype=torch.int64, device=dev)
for _ in range(reps):
    ctx.eval(perms, out=keys)
torch.cuda.synchronize()
del perms

x = synth.x_style(1000, seed=0)
ctx.set_instance(CVRP, x.durations, x.demand, x.capacities, x.start_times)
C = 1 << 18
g = torch.Generator(device=dev)
g.manual_seed(13)
p16 = torch.empty((C, x.n), dtype=torch.int16, device=dev)
for s in range(0, C, 1 << 15):
    r = torch.rand((min(C, s + (1 << 15)) - s, x.n), generator=g, device=dev)
    p16[s:s + r.shape[0]] = (r.argsort(dim=1) + 1).to(torch.int16)
keys = torch.empty(C, dtype=torch.int64, device=dev)
for _ in range(reps):
    ctx.eval(p16, out=keys)
torch.cuda.synchronize()
print("done", int(keys[0]))
