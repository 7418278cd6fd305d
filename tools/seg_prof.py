#!/usr/bin/env python3
"""Where sa_seg_kernel's time goes (built with -DVRPMS_SEG_PROF into
build_ab/segprof/libvrpms.so): per SA step the pricing and accept (table
rebuild) time (wall_clock64 ticks of lane 0, 100 MHz), the accept rate and
the cross-wavefront exchange (W > 1, SEG_WAVES=W -> VRPMS_OPT_SEG_WAVES) -- on X-1000 first-fit start tours at a hot
and a cold fixed temperature.

usage: tools/seg_prof.py build   (CPU: compile the variant; SEG_PROF_HET=1: three
                                 capacity classes)
       tools/seg_prof.py [chains] [moves]   (GPU)"""
import ctypes
import os
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
VARIANT = os.environ.get("SEG_PROF_VARIANT", "")  # e.g. NOCUT (A/B: no capacity cuts)
# abl/ travels to the GPU box (build_ab/ is in .gpurunignore)
LIB = os.path.join(ROOT, "abl", "segprof" + VARIANT.lower(), "libvrpms.so")


def build():
    from vrpms_amd import build as b
    os.makedirs(os.path.dirname(LIB), exist_ok=True)
    extra = [f"-DVRPMS_SEG_{VARIANT}"] if VARIANT else []
    cmd = [b.HIPCC, *b.FLAGS, "-shared", "-DVRPMS_SEG_PROF", *extra, "-o", LIB, *b.sources(),
           "-L/opt/rocm/lib", "-lrccl"]
    subprocess.run(cmd, check=True)


def run(chains, moves):
    import numpy as np
    import torch

    from vrpms_amd import _lib, runners, synth
    from vrpms_amd.core import CVRP, Context
    lib = _lib.load(LIB)
    lib.vrpms_debug_seg_prof.restype = ctypes.c_int
    lib.vrpms_debug_seg_prof.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_int]
    ctx = Context(0)
    ctx.set_seg_waves(int(os.environ.get("SEG_WAVES", "0")))
    x = synth.x_style(1000, seed=0)
    caps = x.capacities
    if os.environ.get("SEG_PROF_HET"):  # three capacity classes (tools/het_rate.py)
        K, base = len(caps), int(caps[0])
        caps = np.array([max(int(base * (1.4, 1.1, 0.9)[k * 3 // K]), int(x.demand.max()))
                         for k in range(K)])
    ctx.set_instance(CVRP, x.durations, x.demand, caps, x.start_times)
    edge = runners.typical_edge(x.durations)
    NP = 22
    buf = (ctypes.c_ulonglong * (NP * 8192))()
    r = runners.SARunner(ctx, x.n, chains=chains, total_steps=1000, durations=x.durations,
                         n_sep=x.K - 1, window=32, window_types=2, start="pack", moves=moves)
    for tag, T, steps in (("hot T=0.5e", 0.5, 1000), ("warm T=0.05e", 0.05, 2000),
                          ("cold T=0.005e", 0.005, 3000), ("cold T=0.005e", 0.005, 3000)):
        lib.vrpms_debug_seg_prof(buf, NP * 8192, 1)
        r.inv_t = np.float32(1.0 / (T * edge))
        r.inv_alpha = np.float32(1.0)
        t0 = time.perf_counter()
        r.epoch(steps)
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
        lib.vrpms_debug_seg_prof(buf, NP * 8192, 1)
        a = np.array(buf[:NP * chains], dtype=np.float64).reshape(chains, NP).sum(0)
        st = a[2]
        mv = st * max(1, moves // 64 // int(os.environ.get("SEG_WAVES", "1"))) / 10
        print(f"{tag}: {steps / dt:,.0f} steps/s/chain | per step: pricing {a[0] / st * 10:.0f} ns, "
              f"rebuild {a[1] / max(a[7], 1) * 10:.0f} ns x {a[7] / st:.3f}/step "
              f"(positions {a[8] / max(a[7], 1) * 10:.0f}, segments {a[9] / max(a[7], 1) * 10:.0f}, "
              f"routes {a[10] / max(a[7], 1) * 10:.0f}, sparse {a[11] / max(a[7], 1) * 10:.0f}), "
              f"pricing parts per move (draw {a[12] / mv:.0f}, r1 {a[13] / mv:.0f}, r2 {a[14] / mv:.0f}, "
              f"r3 {a[15] / mv:.0f}, compose {a[16] / mv:.0f}, full {a[17] / mv:.0f}), "
              f"accept rate {a[3] / st:.3f}, cuts per step wave-max {a[18] / st:.2f} "
              f"(lanes {a[19] / st:.1f} of 64), search steps wave-max {a[20] / st:.1f}, "
              f"over-budget lanes {a[21] / st:.1f}, "
              f"exchange {a[4] / st * 10:.0f} ns, setup {a[5] / chains * 10 / 1e3:.1f} us, "
              f"kernel {a[6] / chains * 10 / 1e3:.1f} us/chain | best "
              f"{r.best()[0] >> 28 & (2**28 - 1)}", flush=True)


if __name__ == "__main__":
    if len(sys.argv) > 1 and sys.argv[1] == "build":
        build()
    else:
        run(int(sys.argv[1]) if len(sys.argv) > 1 else 256,
            int(sys.argv[2]) if len(sys.argv) > 2 else 128)
