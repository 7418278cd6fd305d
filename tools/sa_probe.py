#!/usr/bin/env python3
"""Probe SA / GA / ACO throughput on CVRP-100 (sizing for bench.py's
fixed-wall-time quality comparison).  Prints one JSON line per setting."""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from vrpms_amd import runners, synth  # noqa: E402
from vrpms_amd.core import CVRP, TSP, Context  # noqa: E402


def main():
    inst = synth.cvrp(100, 8, seed=0)
    ctx = Context(0)
    ctx.set_instance(CVRP, inst.durations, inst.demand, inst.capacities, inst.start_times)
    def sa(label, c, n, chains, durations):
        r = runners.SARunner(c, n, chains=chains, total_steps=400, steps_per_epoch=200,
                             durations=durations)
        r.epoch(20)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        r.epoch(200)
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
        k, _ = r.best()
        print(json.dumps({"algo": "sa", "instance": label, "chains": chains,
                          "steps_per_s": 200 / dt, "evals_per_s": chains * 64 * 200 / dt,
                          "best": (k >> 28) & (2**28 - 1)}), flush=True)

    for chains in (256, 1024, 4096, 16384):
        sa("cvrp100", ctx, inst.n, chains, inst.durations)
    ctx.set_split_mode(2)  # generic split kernel, for comparison
    sa("cvrp100 (generic split)", ctx, inst.n, 4096, inst.durations)
    ctx.set_split_mode(0)
    tsp = synth.tsp50(0)
    tctx = Context(0)
    tctx.set_instance(TSP, tsp.durations, start_times=tsp.start_times)
    for chains in (1024, 4096):
        sa("tsp50 (O(1) deltas)", tctx, tsp.n, chains, tsp.durations)
    for islands, pop in ((8, 256), (64, 256), (256, 256)):
        g = runners.GARunner(ctx, inst.n, islands=islands, pop=pop)
        g.epoch(2)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        g.epoch(20)
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
        print(json.dumps({"algo": "ga", "islands": islands, "pop": pop, "gens_per_s": 20 / dt,
                          "children_per_s": islands * pop * 20 / dt}), flush=True)
    for colonies, ants in ((4, 64), (32, 64)):
        a = runners.ACORunner(ctx, inst.n, colonies=colonies, ants=ants)
        a.epoch(1)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        a.epoch(5)
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
        print(json.dumps({"algo": "aco", "colonies": colonies, "ants": ants,
                          "iters_per_s": 5 / dt, "tours_per_s": colonies * ants * 5 / dt}),
              flush=True)


if __name__ == "__main__":
    main()
