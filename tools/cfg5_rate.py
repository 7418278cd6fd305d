#!/usr/bin/env python3
"""cfg-5 kernel rate: 10k TSP-50 requests x 4 chains x 1000 SA steps in one
vrpms_tsp_batch_sa launch (tsp_batch_sa_kernel), best of 3, and the C
restatement's answer on a few requests (parity spot check)."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from vrpms_amd import synth  # noqa: E402
from vrpms_amd.core import Context  # noqa: E402

R = int(sys.argv[1]) if len(sys.argv) > 1 and sys.argv[1].isdigit() else 10000
steps = 1000
if "--lib" in sys.argv:  # an A/B build (tools/ab_build.py) instead of the tree's
    from vrpms_amd import _lib
    _lib.load(sys.argv[sys.argv.index("--lib") + 1])
ctx = Context(0)
rng = np.random.default_rng(0)
mats = np.stack([synth.random_symmetric(50, rng) for _ in range(R)])
M = torch.tensor(mats, dtype=torch.int32, device=ctx.dev)
ctx.tsp_batch_sa(M[:64], 10, 1 / 80.0, 1 / 0.995, 1)
torch.cuda.synchronize()
best = 1e9
for _ in range(3):
    t0 = time.perf_counter()
    tours, keys = ctx.tsp_batch_sa(M, steps, 1 / 80.0, 1 / 0.995, 1)
    torch.cuda.synchronize()
    best = min(best, time.perf_counter() - t0)
print(f"cfg5 kernel: {R / best:,.0f} requests/s ({best * 1e3:.2f} ms for {R} x 4 chains x {steps} "
      f"steps)", flush=True)
if "--check" in sys.argv:
    from oracle import coracle
    coracle.build()
    rt, rk = coracle.tsp_batch_sa(mats[:64], steps, 1 / 80.0, 1 / 0.995, 1)
    t2, k2 = ctx.tsp_batch_sa(M[:64], steps, 1 / 80.0, 1 / 0.995, 1)
    ok = (t2.cpu().numpy().view(np.uint16) == rt).all() and \
        [int(x) & (2**64 - 1) for x in k2.cpu().tolist()] == [int(x) for x in rk]
    print("parity vs C on 64 requests:", bool(ok), flush=True)
ctx.close()
