#!/usr/bin/env python3
"""sa_route_kernel step rate on X-1000 (first-fit start, K - 1 separators,
windowed 2-opt + swap / relocate anywhere) against the move sample per step
(W = moves / 64 wavefronts per chain) and the workgroups per CU (the
resident set: 1 workgroup per CU = 256 multi-wave chains or 1024 one-wave
chains).  usage: route_moves_probe.py [steps]"""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from vrpms_amd import runners, synth  # noqa: E402
from vrpms_amd.core import CVRP, Context  # noqa: E402

steps = int(sys.argv[1]) if len(sys.argv) > 1 else 300
ctx = Context(0)
x = synth.x_style(1000, seed=0)
ctx.set_instance(CVRP, x.durations, x.demand, x.capacities, x.start_times)
edge = runners.typical_edge(x.durations)
CONFIGS = [(64, 2, 2048), (64, 1, 1024), (128, 1, 256), (256, 1, 256), (256, 2, 512),
           (512, 1, 256)]
for moves, per_cu, chains in CONFIGS:
    ctx.set_route_wg_per_cu(per_cu)
    for T in (0.5, 0.01):
        r = runners.SARunner(ctx, x.n, chains=chains, total_steps=10 ** 6, durations=x.durations,
                             n_sep=x.K - 1, window=32, window_types=2, start="pack",
                             t0=T * edge, t_end=T * edge * 0.999, moves=moves)
        r.epoch(4)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        r.epoch(steps)
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
        print(json.dumps({"moves": moves, "wg_per_cu": per_cu, "chains": chains, "T_over_edge": T,
                          "steps_per_s_per_chain": round(steps / dt), "ms": round(dt * 1e3, 1),
                          "move_evals_per_s": round(steps * moves * chains / dt),
                          "best": r.best()[0] >> 28 & (2 ** 28 - 1)}), flush=True)
