#!/usr/bin/env python3
"""Where sa_route_kernel's time goes (search.hip built with
-DVRPMS_ROUTE_PROF into build_ab/routeprof/libvrpms.so): per SA step the
pricing and accept time (wall_clock64 ticks of lane 0, 100 MHz), accept
rate, walked tokens (wave max and lane mean), lanes re-evaluated in full and
tokens re-walked per accepted move -- on X-1000 first-fit start tours and
again after the quality leg's cooling schedule has improved them.

usage: tools/route_prof.py build   (CPU: compile the variant)
       tools/route_prof.py         (GPU)"""
import ctypes
import json
import os
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
VARIANT = os.environ.get("ROUTE_PROF_VARIANT", "")  # e.g. NOGATHER (A/B: no L2 gathers)
LIB = os.path.join(ROOT, "build_ab", "routeprof" + VARIANT.lower(), "libvrpms.so")


def build():
    from vrpms_amd import build as b
    os.makedirs(os.path.dirname(LIB), exist_ok=True)
    extra = [f"-DVRPMS_ROUTE_{VARIANT}"] if VARIANT else []
    cmd = [b.HIPCC, *b.FLAGS, "-shared", "-DVRPMS_ROUTE_PROF", *extra, "-o", LIB, *b.sources(),
           "-L/opt/rocm/lib", "-lrccl"]
    subprocess.run(cmd, check=True)


def run():
    import numpy as np
    import torch

    import bench
    from vrpms_amd import _lib, runners, synth
    from vrpms_amd.core import CVRP, Context
    lib = _lib.load(LIB)
    lib.vrpms_debug_route_prof.restype = ctypes.c_int
    lib.vrpms_debug_route_prof.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_int]
    ctx = Context(0)
    x = synth.x_style(1000, seed=0)
    ctx.set_instance(CVRP, x.durations, x.demand, x.capacities, x.start_times)
    edge = runners.typical_edge(x.durations)
    chains = 2048
    buf = (ctypes.c_ulonglong * (12 * 8192))()

    def report(tag, r, steps, T):
        lib.vrpms_debug_route_prof(buf, 12 * 8192, 1)
        r.inv_t = np.float32(1.0 / (T * edge))
        r.inv_alpha = np.float32(1.0)
        t0 = time.perf_counter()
        r.epoch(steps)
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
        lib.vrpms_debug_route_prof(buf, 12 * 8192, 1)
        a = np.array(buf[:12 * chains], dtype=np.float64).reshape(chains, 12).sum(0)
        st = a[2]
        print(json.dumps({
            "tours": tag, "T_over_edge": T, "steps_per_s_per_chain": round(steps / dt),
            "us_pricing_per_step": round(a[0] / st / 100.0, 2),
            "us_accept_per_step": round(a[1] / st / 100.0, 2),
            "accept_rate": round(a[3] / st, 3),
            "walk_tokens_wave_max": round(a[4] / st, 1),
            "walk_tokens_lane_mean": round(a[5] / st / 64, 1),
            "full_lanes_per_step": round(a[6] / st, 2),
            "full_builds_per_accept": round(a[7] / max(a[3], 1), 4),
            "us_walk_wave_max": round(a[8] / st / 100.0, 2),
            "blocks_wave_max": round(a[9] / st, 2),
            "us_prologue_mean": round(a[10] / chains / 100.0, 1),
            "ms_chain_kernel_mean": round(a[11] / chains / 1e5, 2),
            "ms_launch_wall": round(dt * 1e3, 2),
            "best": r.best()[0] >> 28 & (2 ** 28 - 1)}), flush=True)

    r = runners.SARunner(ctx, x.n, chains=chains, seed=1000, total_steps=1000,
                         durations=x.durations, t0=0.5 * edge, t_end=0.002 * edge,
                         n_sep=x.K - 1, window=32, window_types=2, start="pack")
    r.epoch(2)
    torch.cuda.synchronize()
    report("first-fit start", r, 300, 0.5)
    cool = bench._TimedCooling(6.0, 0.5 * edge, 0.002 * edge)
    r.inv_t = np.float32(1.0 / (0.5 * edge))
    done = 0
    while True:
        steps, inv_a = cool.plan(done)
        if steps == 0:
            break
        r.inv_alpha = inv_a
        r.epoch(steps)
        cool.advance(steps, inv_a)
        done += steps
        torch.cuda.synchronize()
    for T in (0.002, 0.05, 0.5):
        report("after 6 s of cooling", r, 300, T)


if __name__ == "__main__":
    build() if sys.argv[1:] == ["build"] else run()
