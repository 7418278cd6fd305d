#!/usr/bin/env python3
"""GPU-only equal-time scan on the hour-indexed TD-200 x 24 (sa_td_kernel):
best durationSum after T seconds per (chains, moves, t_end) shape, seeds
given, heterogeneous fleet (synth.td_cvrp_het) or uniform (synth.td_cvrp).
usage: td_quality_scan.py [--het] [--T 10] [--seeds 0 1] [--cpu]"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

import bench  # noqa: E402
from vrpms_amd import synth  # noqa: E402
from vrpms_amd.core import CVRP, Context  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--het", action="store_true")
ap.add_argument("--x1000", action="store_true", help="X-1000 (sa_seg_kernel) instead of TD-200")
ap.add_argument("--T", type=float, default=10.0)
ap.add_argument("--seeds", type=int, nargs="+", default=[0])
ap.add_argument("--cpu", action="store_true")
ap.add_argument("--shapes", default="256x128,512x64,1024x64,512x128,1024x128")
ap.add_argument("--tend", type=float, nargs="+", default=[0.004])
ap.add_argument("--lib", default=None, help="an A/B build (tools/ab_build.py) instead of the tree's")
args = ap.parse_args()
if args.lib:
    from vrpms_amd import _lib
    _lib.load(args.lib)
ctx = Context(0)
for sd in args.seeds:
    x = synth.x_style(1000, seed=sd) if args.x1000 else (
        synth.td_cvrp_het(200, 16, seed=sd) if args.het else synth.td_cvrp(200, 16, seed=sd))
    ctx.set_instance(CVRP, x.durations, x.demand, x.capacities, x.start_times)
    for shape in args.shapes.split(","):
        chains, moves = (int(v) for v in shape.split("x"))
        for te in args.tend:
            q = bench.quality(ctx, x, args.T, 1, 0, torch.distributed, with_cpu=False,
                              chains=chains, moves=moves, window=32, window_types=2,
                              start="pack", mig_E=max(1, chains // 4 if args.x1000 else chains // 8),
                              tend_frac=te, epochs=80 if args.x1000 else 40)
            g = q["gpu"]
            print(json.dumps({"seed": sd, "het": args.het, "chains": chains, "moves": moves,
                              "t_end": te, "duration_sum": g["duration_sum"],
                              "unvisited": g["unvisited"], "steps": g["steps_per_chain"],
                              "rescored_equal": g["rescored_equal"]}), flush=True)
    if args.cpu:
        for m in (32, 64):
            q = bench.quality(ctx, x, args.T, 1, 0, torch.distributed, with_cpu=True, gpu=False,
                              chains=256, moves=128, window=32, window_types=2, start="pack",
                              mig_E=32, cpu_moves=m, cpu_t0_frac=1.0, cpu_tend_frac=0.002)
            c = q["cpu"]
            print(json.dumps({"seed": sd, "het": args.het, "host_moves": m,
                              "duration_sum": c["duration_sum"], "unvisited": c["unvisited"],
                              "steps": c["steps_per_chain"], "threads": c["chains"]}), flush=True)
ctx.close()
