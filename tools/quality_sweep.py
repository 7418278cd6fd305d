#!/usr/bin/env python3
"""Best-cost gap at equal wall time, swept over T and instance seeds
(T in {1, 10, 60} s, median over seeds 0..4).

Each (seed, T) cell runs bench.quality(): the GPU SA leg (4096 chains, elite
migration) and the C/OpenMP SA leg on the host cores, each for T seconds of
wall time with the cooling schedule spread over that time.  Writes
gpurun_out/quality_sweep.json and prints one line per cell as it finishes.

usage: python tools/quality_sweep.py [--T 1 10 60] [--seeds 0 1 2 3 4]
"""
from __future__ import annotations

import argparse
import json
import os
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--T", type=float, nargs="+", default=[1.0, 10.0, 60.0])
    ap.add_argument("--seeds", type=int, nargs="+", default=[0, 1, 2, 3, 4])
    ap.add_argument("--chains", type=int, default=None,
                    help="GPU chains (default 4096 for cvrp100; 2048 otherwise, the route-local "
                         "kernel's resident count: 2 workgroups x 4 chains per CU)")
    ap.add_argument("--types", type=int, default=None,
                    help="A12 window move types (bit 0 swap, 1 2-opt, 2 relocate; "
                         "default 2 = windowed 2-opt only when windowed)")
    ap.add_argument("--start", default=None, choices=["random", "greedy", "pack"],
                    help="separator placement of the start tours (default: random for "
                         "cvrp100, pack otherwise)")
    ap.add_argument("--window", type=int, default=None,
                    help="A11 move window (default: 0 for cvrp100, 32 otherwise)")
    ap.add_argument("--instance", default="cvrp100",
                    choices=["cvrp100", "cvrp200", "x1000", "tdvrp200"],
                    help="cfg 2 CVRP-100 K=8, CVRP-200 K=16, cfg 4 X-style CVRP-1000, or cfg 3 "
                         "time-dependent VRP-200 x 24 hourly matrices (K=16, start 480)")
    ap.add_argument("--sep", type=int, default=None,
                    help="A10 route separators per tour (default K - 1; 0 = plain giant tours)")
    ap.add_argument("--moves", type=int, default=64,
                    help="GPU moves per step (64 W: W wavefronts per chain)")
    ap.add_argument("--cpu-moves", type=int, nargs="+", default=[64],
                    help="host moves per step; several values: each cell reports the host's best")
    ap.add_argument("--wg-per-cu", type=int, default=0,
                    help="sa_route_kernel workgroups per CU (0 = auto)")
    ap.add_argument("--no-cpu", action="store_true", help="GPU legs only (parameter scans)")
    ap.add_argument("--out", default=os.path.join(ROOT, "gpurun_out", "quality_sweep.json"))
    args = ap.parse_args()

    import torch
    import bench
    from vrpms_amd import synth
    from vrpms_amd.core import CVRP, Context

    torch.cuda.set_device(0)
    ctx = Context(0)
    ctx.set_route_wg_per_cu(args.wg_per_cu)
    cells = []
    summary = {}
    os.makedirs(os.path.dirname(args.out), exist_ok=True)
    t_start = time.time()
    make = {"cvrp100": lambda s: synth.cvrp(100, 8, seed=s),
            "cvrp200": lambda s: synth.cvrp(200, 16, seed=s),
            "x1000": lambda s: synth.x_style(1000, seed=s),
            "tdvrp200": lambda s: synth.td_cvrp(200, 16, seed=s)}[args.instance]
    for seed in args.seeds:
        inst = make(seed)
        ctx.set_instance(CVRP, inst.durations, inst.demand, inst.capacities, inst.start_times)
        for T in args.T:
            window = args.window if args.window is not None else (
                0 if args.instance == "cvrp100" else 32)
            chains = args.chains or (4096 if args.instance == "cvrp100" else 2048) * 64 // args.moves
            q = bench.quality(ctx, inst, T, 1, 0, None, with_cpu=not args.no_cpu, chains=chains,
                              moves=args.moves, cpu_moves=args.cpu_moves[0],
                              label=f"{args.instance} seed {seed}", n_sep=args.sep,
                              window=window,
                              window_types=args.types if args.types is not None else 2,
                              start=args.start or ("random" if args.instance == "cvrp100"
                                                   else "pack"))
            if args.no_cpu:
                print(json.dumps({"seed": seed, "T_s": T, "moves": args.moves, "chains": chains,
                                  "gpu": q["gpu"]["duration_sum"],
                                  "steps_per_chain": q["gpu"]["steps_per_chain"]}), flush=True)
                continue
            print(json.dumps({"progress": f"seed {seed} T {T}: gpu {q['gpu']['duration_sum']} "
                                          f"cpu(m={args.cpu_moves[0]}) {q['cpu']['duration_sum']}"}),
                  flush=True)
            for cm in args.cpu_moves[1:]:   # the host leg at its best sample size
                q2 = bench.quality(ctx, inst, T, 1, 0, None, with_cpu=True, chains=chains,
                                   moves=args.moves, cpu_moves=cm, gpu=False,
                                   label=f"{args.instance} seed {seed}", n_sep=args.sep,
                                   window=window,
                                   window_types=args.types if args.types is not None else 2,
                                   start=args.start or ("random" if args.instance == "cvrp100"
                                                        else "pack"))
                q.setdefault("cpu_alternatives", []).append(q2["cpu"])
                if q2["cpu"]["unvisited"] == 0 and q2["cpu"]["duration_sum"] < q["cpu"]["duration_sum"]:
                    q["cpu_alternatives"][-1] = q["cpu"]
                    q["cpu"] = q2["cpu"]
                    q["gap"] = (q["gpu"]["duration_sum"] - q["cpu"]["duration_sum"]) / q["cpu"]["duration_sum"]
            q["seed"] = seed
            cells.append(q)
            print(json.dumps({"seed": seed, "T_s": T, "gpu": q["gpu"]["duration_sum"],
                              "cpu": q["cpu"]["duration_sum"], "cpu_moves": q["cpu"]["moves_per_step"],
                              "gap": q["gap"],
                              "gpu_wall": round(q["gpu"]["wall_s"], 3),
                              "cpu_wall": round(q["cpu"]["wall_s"], 3),
                              "elapsed": round(time.time() - t_start, 1)}), flush=True)
            summary = {}
            for t in args.T:
                gaps = [c["gap"] for c in cells if c["T_s"] == t and c["gap"] is not None]
                if gaps:
                    summary[str(t)] = {"median_gap": statistics.median(gaps), "n": len(gaps),
                                       "min_gap": min(gaps), "max_gap": max(gaps),
                                       "gpu_better": sum(g < 0 for g in gaps)}
            with open(args.out, "w") as f:
                json.dump({"metric": "best-cost gap at equal wall time, (gpu - cpu) / cpu "
                                     "on durationSum, negative = GPU better",
                           "workload": f"{args.instance} (vrpms_amd.synth), SA on both sides",
                           "separators": cells[0]["separators"],
                           "window": cells[0]["window"], "window_types": cells[0]["window_types"],
                           "start": cells[0]["start"],
                           "cpu_cores": cells[0]["cpu"]["cores"],
                           "summary": summary, "cells": cells}, f, indent=1)
    if cells:
        print(json.dumps({"summary": summary}), flush=True)


if __name__ == "__main__":
    main()
