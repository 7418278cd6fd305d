#!/usr/bin/env python3
"""sa_route_kernel step rate on X-1000 (first-fit start, K - 1 separators):
SA steps per chain per second against the chain count, the temperature
(hot: most steps accept and rebuild the route stats; cold: few do) and the
A12 window types.  usage: route_probe.py [steps] [--schedule]"""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import numpy as np  # noqa: E402
import torch  # noqa: E402

from vrpms_amd import runners, synth  # noqa: E402
from vrpms_amd.core import CVRP, Context  # noqa: E402

steps = int(sys.argv[1]) if len(sys.argv) > 1 and sys.argv[1].isdigit() else 400
ctx = Context(0)
x = synth.x_style(1000, seed=0)
ctx.set_instance(CVRP, x.durations, x.demand, x.capacities, x.start_times)
edge = runners.typical_edge(x.durations)


def rate(chains, t, types, window=32, route=0):
    ctx.set_sa_route(route)
    r = runners.SARunner(ctx, x.n, chains=chains, total_steps=10 ** 6, durations=x.durations,
                         n_sep=x.K - 1, window=window, window_types=types, start="pack",
                         t0=t * edge, t_end=t * edge * 0.999)
    r.epoch(4)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    r.epoch(steps)
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    ctx.set_sa_route(0)
    return {"chains": chains, "T_over_edge": t, "types": types, "window": window, "route": route,
            "steps_per_s_per_chain": round(steps / dt), "ms": round(dt * 1e3, 1),
            "best": r.best()[0] >> 28 & (2 ** 28 - 1)}


for chains in (() if "--schedule" in sys.argv else (256, 1024, 2048, 4096)):
    for t in (0.5, 0.01):
        print(json.dumps(rate(chains, t, 2)), flush=True)
if "--schedule" not in sys.argv:
    print(json.dumps(rate(1024, 0.5, 7)), flush=True)
    print(json.dumps(rate(1024, 0.01, 7)), flush=True)
    print(json.dumps(rate(1024, 0.5, 2, route=2)), flush=True)

# the quality leg's schedule (bench.quality): per-epoch step rate and how
# many current tours leave customers unserved (their moves re-walk in full)
if "--schedule" in sys.argv:
    import bench
    r = runners.SARunner(ctx, x.n, chains=2048, seed=1000, total_steps=1000,
                         durations=x.durations, t0=0.5 * edge, t_end=0.002 * edge,
                         n_sep=x.K - 1, window=32, window_types=2, start="pack")
    cool = bench._TimedCooling(6.0, 0.5 * edge, 0.002 * edge)
    e = 0
    while True:
        steps, inv_a = cool.plan(r.step)
        if steps == 0:
            break
        r.inv_alpha = inv_a
        t0 = time.perf_counter()
        r.epoch(steps)
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
        cool.advance(steps, inv_a)
        e += 1
        ck = r.cur_key.cpu()
        unv = int(((ck >> 56) & 0xFF).gt(0).sum())
        print(json.dumps({"epoch": e, "steps": steps, "ms": round(dt * 1e3, 1),
                          "steps_per_s": round(steps / dt), "chains_unserved": unv,
                          "best": r.best()[0] >> 28 & (2 ** 28 - 1),
                          "elapsed": round(cool.elapsed(), 2)}), flush=True)
        if e % 5 == 0:
            r.inject(*r.elites(16))
    # the same (good) tours at a fixed temperature: cold, then hot
    for tt in (0.002, 0.05, 0.5):
        r.inv_t = np.float32(1.0 / (tt * edge))
        r.inv_alpha = np.float32(1.0)
        t0 = time.perf_counter()
        r.epoch(300)
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
        print(json.dumps({"fixed_T_over_edge": tt, "steps_per_s": round(300 / dt),
                          "best": r.best()[0] >> 28 & (2 ** 28 - 1)}), flush=True)
    if "--save" in sys.argv:
        np.save("gpurun_out/route_good_tours.npy", r.cur[:512].cpu().numpy())
        start = runners.SARunner(ctx, x.n, chains=512, seed=1000, durations=x.durations,
                                 n_sep=x.K - 1, window=32, window_types=2, start="pack")
        np.save("gpurun_out/route_start_tours.npy", start.cur.cpu().numpy())
