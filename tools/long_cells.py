#!/usr/bin/env python3
"""The bench's equal-wall-time X-1000 cells at a longer budget (default 60 s):
per seed the GPU leg and the host leg at 32 and 64 moves per step (the better
kept), the same shapes and schedules as bench.equal_time_cells; one line per
leg as it finishes (so a long run keeps printing).
usage: long_cells.py [seconds] [seed ...]"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
from vrpms_amd import synth  # noqa: E402
from vrpms_amd.core import CVRP, Context  # noqa: E402

T = float(sys.argv[1]) if len(sys.argv) > 1 else 60.0
seeds = [int(s) for s in sys.argv[2:]] or [0, 1, 2]
kw = dict(chains=1024, moves=128, window=32, window_types=2, start="pack", epochs=80,
          mig_E=256, tend_frac=0.004, cpu_tend_frac=0.002)
ctx = Context(0)
for sd in seeds:
    x = synth.x_style(1000, seed=sd)
    ctx.set_instance(CVRP, x.durations, x.demand, x.capacities, x.start_times)
    g = bench.quality(ctx, x, T, 1, 0, None, with_cpu=False, **kw)["gpu"]
    print(json.dumps({"seed": sd, "T": T, "leg": "gpu", "duration_sum": g["duration_sum"],
                      "unvisited": g["unvisited"], "steps": g["steps_per_chain"],
                      "rescored_equal": g["rescored_equal"]}), flush=True)
    for m in (32, 64):
        c = bench.quality(ctx, x, T, 1, 0, None, with_cpu=True, gpu=False, cpu_moves=m, **kw)["cpu"]
        print(json.dumps({"seed": sd, "T": T, "leg": f"cpu{m}", "duration_sum": c["duration_sum"],
                          "unvisited": c["unvisited"], "steps": c["steps_per_chain"],
                          "rescored_equal": c["rescored_equal"]}), flush=True)
