#!/usr/bin/env python3
"""sa_seg_kernel alone on cfg 4 (X-1000, K - 1 separators, first-fit
starts, windowed 2-opt + swap / relocate anywhere) -- a short target for
rocprofv3 --pmc / --stats passes.  usage: seg_run.py [chains] [moves] [steps]   (SEG_LIB=<path>: another libvrpms.so;
SEG_HET=1: three capacity classes)"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from vrpms_amd import _lib, runners, synth  # noqa: E402
from vrpms_amd.core import CVRP, Context  # noqa: E402

chains = int(sys.argv[1]) if len(sys.argv) > 1 else 256
moves = int(sys.argv[2]) if len(sys.argv) > 2 else 128
steps = int(sys.argv[3]) if len(sys.argv) > 3 else 1000
if os.environ.get("SEG_LIB"):  # an A/B build of the library
    _lib.load(os.environ["SEG_LIB"])
ctx = Context(0)
x = synth.x_style(1000, seed=0)
caps = x.capacities
if os.environ.get("SEG_HET"):  # three capacity classes (the heterogeneous variant)
    import numpy as np
    K, base = len(caps), int(caps[0])
    fr = (1.4, 1.1, 0.9)
    caps = np.array([max(int(base * fr[k * 3 // K]), int(x.demand.max())) for k in range(K)])
ctx.set_instance(CVRP, x.durations, x.demand, caps, x.start_times)
r = runners.SARunner(ctx, x.n, chains=chains, total_steps=2 * steps, durations=x.durations,
                     n_sep=x.K - 1, window=32, window_types=2, start="pack", moves=moves)
r.epoch(steps)
r.epoch(steps)
torch.cuda.synchronize()
print("done", r.best()[0] >> 28 & (2 ** 28 - 1))
