#!/usr/bin/env python3
"""sa_seg_kernel with W wavefronts per chain (VRPMS_OPT_SEG_WAVES) on cfg 4
(X-1000, K - 1 separators, first-fit starts, windowed 2-opt + swap /
relocate anywhere): steps per second per chain and moves priced per second
for W = 1, 2, 4 at each (chains, moves), and a check that every W follows
the same trajectories.  usage: seg_waves.py [steps] [chains:moves ...]"""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from vrpms_amd import runners, synth  # noqa: E402
from vrpms_amd.core import CVRP, Context  # noqa: E402

steps = int(sys.argv[1]) if len(sys.argv) > 1 else 2000
cfgs = [tuple(int(v) for v in c.split(":")) for c in sys.argv[2:]] or [(256, 128), (1024, 256),
                                                                       (2048, 128)]
ctx = Context(0)
x = synth.x_style(1000, seed=0)
ctx.set_instance(CVRP, x.durations, x.demand, x.capacities, x.start_times)
ctx.set_sa_route(0)
for chains, moves in cfgs:
    ref = None
    for w in (1, 2, 4):
        if moves // 64 % w:
            continue
        ctx.set_seg_waves(w)
        r = runners.SARunner(ctx, x.n, chains=chains, total_steps=steps, durations=x.durations,
                             n_sep=x.K - 1, window=32, window_types=2, start="pack", moves=moves)
        r.epoch(20)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        r.epoch(steps)
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
        k, _ = r.best()
        out = (r.cur.cpu(), r.cur_key.cpu())
        same = ref is None or (torch.equal(out[0], ref[0]) and torch.equal(out[1], ref[1]))
        ref = ref or out
        print(f"chains {chains} moves {moves} W {w}: {steps / dt:,.0f} steps/s per chain, "
              f"{chains * moves * steps / dt / 1e9:.2f} G moves/s, best {k >> 28 & (2**28 - 1)}, "
              f"same trajectories as W=1: {same}", flush=True)
ctx.set_seg_waves(0)
