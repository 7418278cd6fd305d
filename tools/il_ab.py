#!/usr/bin/env python3
"""A/B of library builds that differ only in compile-time schedule knobs
(e.g. -DVRPMS_IL_VALU=<n>, eval_words.hip): each build_ab/<tag>/libvrpms.so
is timed in its own process on the headline workload (eval_cvrp_words2,
CVRP-100, K = 8, C = 16 Mi) and its keys' checksum compared with the
in-tree library's.
usage: il_ab.py            (parent: every build_ab/*/libvrpms.so + in-tree)
       il_ab.py <lib.so>   (child: one library)"""
import glob
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def child(path):
    from vrpms_amd import _lib
    _lib.load.__defaults__ = (path,)
    import torch

    import bench
    from vrpms_amd import synth
    from vrpms_amd.core import CVRP, Context
    ctx = Context(0)
    inst = synth.cvrp(100, 8, seed=0)
    ctx.set_instance(CVRP, inst.durations, inst.demand, inst.capacities, inst.start_times)
    C = 16 << 20
    words = ctx.to_words(bench.make_batch(ctx, C, inst.n, 0), inst.n)
    keys = torch.empty(C, dtype=torch.int64, device=ctx.dev)
    for _ in range(3):
        ctx.eval_words(words, inst.n, out=keys)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    e0.record()
    for _ in range(30):
        ctx.eval_words(words, inst.n, out=keys)
    e1.record()
    torch.cuda.synchronize()
    t = e0.elapsed_time(e1) * 1e-3 / 30
    print(json.dumps({"lib": path, "ms": t * 1e3, "evals_per_s": C / t,
                      "checksum": int(keys.sum())}), flush=True)


def main():
    if len(sys.argv) > 1:
        return child(sys.argv[1])
    libs = sorted(glob.glob(os.path.join(ROOT, "build_ab", "*", "libvrpms.so")))
    libs.append(os.path.join(ROOT, "vrpms_amd", "libvrpms.so"))
    for rep in range(2):
        for p in libs:
            r = subprocess.run([sys.executable, __file__, p], capture_output=True, text=True,
                               timeout=240)
            print(r.stdout.strip() or r.stderr[-500:], flush=True)
            if r.returncode != 0:
                sys.exit(r.returncode)


if __name__ == "__main__":
    main()
