#!/usr/bin/env python3
"""Phase timing of the fused GA island kernel (ga_fused.hip built with
-DVRPMS_GA_PROF into build_ab/gaprof/libvrpms.so): cycles per generation in
breed / score / sort / survivor bookkeeping, from wall_clock64 (100 MHz
constant clock on gfx950) stamps of thread 0 between workgroup barriers.

usage: tools/ga_prof.py build   (CPU: compile the variant)
       tools/ga_prof.py         (GPU: run CVRP-100, 256 islands x 256)"""
import ctypes
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
# GA_PROF_TAG=x: build_ab/gaprof_x (A/B); GA_PROF_SRC=<file>: that ga_fused.hip
# instead of the tree's (e.g. an older revision written out by git show)
TAG = os.environ.get("GA_PROF_TAG", "")
LIB = os.path.join(ROOT, os.environ.get("AB_DIR", "build_ab"), "gaprof" + (f"_{TAG}" if TAG else ""), "libvrpms.so")


def build():
    from vrpms_amd import build as b
    os.makedirs(os.path.dirname(LIB), exist_ok=True)
    srcs = b.sources()
    alt = os.environ.get("GA_PROF_SRC")
    if alt:
        srcs = [alt if os.path.basename(x) == "ga_fused.hip" else x for x in srcs]
    cmd = [b.HIPCC, *b.FLAGS, "-shared", "-DVRPMS_GA_PROF", f"-I{b.CSRC}", "-o", LIB, *srcs,
           "-L/opt/rocm/lib", "-lrccl"]
    subprocess.run(cmd, check=True)


def run():
    import numpy as np
    import torch

    from vrpms_amd import _lib, runners, synth
    from vrpms_amd.core import CVRP, Context
    lib = _lib.load(LIB)
    lib.vrpms_debug_ga_prof.restype = ctypes.c_int
    lib.vrpms_debug_ga_prof.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_int]
    ctx = Context(0)
    inst = synth.cvrp(100, 8, seed=0)
    ctx.set_instance(CVRP, inst.durations, inst.demand, inst.capacities, inst.start_times)
    for islands, pop, pmut in ((256, 256, 0.2), (256, 256, 0.0), (256, 128, 0.2)):
        ga = runners.GARunner(ctx, inst.n, islands=islands, pop=pop, seed=1, gens_per_epoch=20,
                              pmut=pmut)
        ga.epoch()
        torch.cuda.synchronize()
        buf = (ctypes.c_ulonglong * (6 * 4096))()
        lib.vrpms_debug_ga_prof(buf, 6 * 4096, 1)
        ga.epoch()
        torch.cuda.synchronize()
        lib.vrpms_debug_ga_prof(buf, 6 * 4096, 1)
        a = np.array(buf[:4 * islands], dtype=np.float64).reshape(islands, 4) / 20
        redo = np.array(buf[4 * 4096:4 * 4096 + islands], dtype=np.float64) / 20
        # selection up to the run-sort barrier (sorted-parents generations)
        sort_a = np.array(buf[5 * 4096:5 * 4096 + islands], dtype=np.uint64).astype(np.float64) / 20
        # whole calls (prologue + 20 generations + epilogue) by HIP events
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(5):
            ga.epoch()
        e1.record()
        torch.cuda.synchronize()
        call_us = e0.elapsed_time(e1) * 1e3 / 5
        names = ["breed", "score", "sort", "survivors"]
        print(json.dumps({"islands": islands, "pop": pop, "pmut": pmut,
                          "ticks_per_generation": dict(zip(names, a.mean(0).round(1).tolist())),
                          "us_per_generation": round(a.mean(0).sum() / 100.0, 2),
                          "sort_to_run_barrier": round(float(sort_a.mean()), 1),
                          "call_us_per_generation": round(call_us / 20, 2),
                          "exact_rewalks_per_generation": {"mean": round(redo.mean(), 2),
                                                           "islands_with_any": int((redo > 0).sum())}}),
              flush=True)
        del ga


if __name__ == "__main__":
    build() if sys.argv[1:] == ["build"] else run()
