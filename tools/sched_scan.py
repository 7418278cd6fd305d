#!/usr/bin/env python3
"""Cooling-schedule scan on X-1000 (cfg 4) at T seconds: for each (t0, t_end)
as fractions of the typical edge, the GPU leg (bench.quality: 512 chains x
128 moves, migration every epoch, 80 epochs) and the host leg (16 threads,
32 moves per step), the same schedule on both.
usage: sched_scan.py T seed t0:tend [t0:tend ...]"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
from vrpms_amd import synth  # noqa: E402
from vrpms_amd.core import CVRP, Context  # noqa: E402

T, seed = float(sys.argv[1]), int(sys.argv[2])
ctx = Context(0)
# INSTANCE=td: cfg 3's TD-200 x 24 (sa_route_kernel, 256 chains, 40 epochs)
td = os.environ.get("INSTANCE") == "td"
x = synth.td_cvrp(200, 16, seed=seed) if td else synth.x_style(1000, seed=seed)
ctx.set_instance(CVRP, x.durations, x.demand, x.capacities, x.start_times)
for spec in sys.argv[3:]:
    a, b = (float(v) for v in spec.split(":"))
    shape = dict(chains=256, mig_E=128, epochs=40) if td else dict(chains=512, mig_E=128, epochs=80)
    q = bench.quality(ctx, x, T, 1, 0, None, with_cpu=True, moves=128, window=32, window_types=2,
                      start="pack", mig_every=1, cpu_moves=32, t0_frac=a, tend_frac=b, **shape)
    print(json.dumps({"t0": a, "t_end": b, "gpu": q["gpu"]["duration_sum"],
                      "gpu_ok": q["gpu"]["rescored_equal"], "cpu": q["cpu"]["duration_sum"],
                      "cpu_ok": q["cpu"]["rescored_equal"], "gap": q.get("gap")}), flush=True)
