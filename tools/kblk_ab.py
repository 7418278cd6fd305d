#!/usr/bin/env python3
"""A/B of sa_route_kernel's walk block size (kBlk): each variant is search.hip
built with -DVRPMS_KBLK=<k> into build_ab/kblk<k>/libvrpms.so; one process per
variant times SA steps per chain on X-1000 first-fit tours after a short
cooling (1024 chains, windowed 2-opt, K - 1 separators) and prints the best
key, which must not depend on kBlk (trajectories are block-size independent).

usage: tools/kblk_ab.py build 4 8 12     (CPU)
       tools/kblk_ab.py run 4 8 12       (GPU)"""
import json
import os
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def lib(k):
    return os.path.join(ROOT, "build_ab", f"kblk{k}", "libvrpms.so")


def build(k):
    from vrpms_amd import build as b
    os.makedirs(os.path.dirname(lib(k)), exist_ok=True)
    subprocess.run([b.HIPCC, *b.FLAGS, "-shared", f"-DVRPMS_KBLK={k}", "-o", lib(k), *b.sources(),
                    "-L/opt/rocm/lib", "-lrccl"], check=True)


def one(k):
    import numpy as np
    import torch
    from vrpms_amd import _lib, runners, synth
    from vrpms_amd.core import CVRP, Context
    _lib.load(lib(k))
    ctx = Context(0)
    x = synth.x_style(1000, seed=0)
    ctx.set_instance(CVRP, x.durations, x.demand, x.capacities, x.start_times)
    edge = runners.typical_edge(x.durations)
    r = runners.SARunner(ctx, x.n, chains=1024, seed=1000, total_steps=100000, durations=x.durations,
                         t0=0.5 * edge, t_end=0.002 * edge, n_sep=x.K - 1, window=32, window_types=2,
                         start="pack")
    r.inv_alpha = np.float32(1.0)
    r.epoch(20)
    torch.cuda.synchronize()
    out = {"kblk": k}
    for T in (0.5, 0.02):
        r.inv_t = np.float32(1.0 / (T * edge))
        t0 = time.perf_counter()
        r.epoch(2000)
        torch.cuda.synchronize()
        out[f"steps_per_s_T{T}"] = round(2000 / (time.perf_counter() - t0))
    out["best"] = int(r.best()[0])
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    mode, ks = sys.argv[1], [int(v) for v in sys.argv[2:]]
    if mode == "build":
        for k in ks:
            build(k)
    elif mode == "one":
        one(ks[0])
    else:
        for k in ks:
            subprocess.run([sys.executable, __file__, "one", str(k)], check=True, timeout=300)
