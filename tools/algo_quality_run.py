#!/usr/bin/env python3
"""cfg 2 (CVRP-100, K = 8) best cost at equal wall time: GPU SA and host SA
(bench.quality), then the GA and ACO endpoints' memetic runs
(bench.algo_quality) for the same seconds.
usage: algo_quality_run.py [seconds] [polish_steps] [polish_top] [seed]
(ACO_SHAPE=colonies:ants:iterations_per_epoch, default 64:64:5; ONLY=aco|ga)"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402
from vrpms_amd import synth  # noqa: E402
from vrpms_amd.core import CVRP, Context  # noqa: E402

T = float(sys.argv[1]) if len(sys.argv) > 1 else 5.0
ps = int(sys.argv[2]) if len(sys.argv) > 2 else 50
top = int(sys.argv[3]) if len(sys.argv) > 3 else 4
seed = int(sys.argv[4]) if len(sys.argv) > 4 else 0
ctx = Context(0)
inst = synth.cvrp(100, 8, seed=seed)
ctx.set_instance(CVRP, inst.durations, inst.demand, inst.capacities, inst.start_times)
q = bench.quality(ctx, inst, T, 1, 0, None, with_cpu=True)
print(json.dumps({"sa_gpu": q["gpu"]["duration_sum"], "sa_host": q["cpu"]["duration_sum"],
                  "gap": q.get("gap")}), flush=True)
shape = tuple(int(x) for x in os.environ.get("ACO_SHAPE", "64:64:5").split(":"))
by = bench.algo_quality(ctx, inst, T, seed=seed, polish_steps=ps, polish_top=top,
                        aco_shape=shape)
for k, v in by.items():
    v["gap_vs_host_sa"] = (v["duration_sum"] - q["cpu"]["duration_sum"]) / q["cpu"]["duration_sum"]
print(json.dumps(by), flush=True)
