#!/usr/bin/env python3
"""Run only the headline kernel (vrpms_eval_words on CVRP-100, K = 8,
C = 16 Mi) `reps` times -- a short target for rocprofv3 --pmc passes.
usage: words_run.py [gen(0|1)] [ilp(0|1|2)] [reps]"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

import bench  # noqa: E402
from vrpms_amd import synth  # noqa: E402
from vrpms_amd.core import CVRP, Context  # noqa: E402

gen = int(sys.argv[1]) if len(sys.argv) > 1 else 0
ilp = int(sys.argv[2]) if len(sys.argv) > 2 else 0
reps = int(sys.argv[3]) if len(sys.argv) > 3 else 5
ctx = Context(0)
inst = synth.cvrp(100, 8, seed=0)
ctx.set_instance(CVRP, inst.durations, inst.demand, inst.capacities, inst.start_times)
C = 16 << 20
perms = bench.make_batch(ctx, C, inst.n, 0)
words = ctx.to_words(perms, inst.n)
del perms
ctx.set_words_kernel(gen)
ctx.set_words_ilp(ilp)
keys = torch.empty(C, dtype=torch.int64, device=ctx.dev)
for _ in range(reps):
    ctx.eval_words(words, inst.n, out=keys)
torch.cuda.synchronize()
print("done", int(keys[0]))
