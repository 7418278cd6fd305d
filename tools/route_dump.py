#!/usr/bin/env python3
"""Debug: sa_route_kernel's route tables (built with -DVRPMS_ROUTE_DUMP into
build_ab/routedump/libvrpms.so) after k SA steps, against the tables rebuilt
from scratch (oracle/route_model.Tables) for the tour the kernel returns, on
the uniform-fleet TD-200 first-fit start (seed 21) where the kernel first
left the C restatement at step 3 (tools/route_td_diag.py).
usage: tools/route_dump.py build | tools/route_dump.py [seed]"""
import ctypes
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
LIB = os.path.join(ROOT, "build_ab", "routedump", "libvrpms.so")


def build():
    from vrpms_amd import build as b
    os.makedirs(os.path.dirname(LIB), exist_ok=True)
    cmd = [b.HIPCC, *b.FLAGS, "-shared", "-DVRPMS_ROUTE_DUMP", "-o", LIB, *b.sources(),
           "-L/opt/rocm/lib", "-lrccl"]
    subprocess.run(cmd, check=True)


def run():
    import numpy as np
    import torch

    from oracle import coracle, route_model as rmod, spec
    from vrpms_amd import _lib, core, synth
    lib = _lib.load(LIB)
    lib.vrpms_debug_route_dump.restype = ctypes.c_int
    lib.vrpms_debug_route_dump.argtypes = [ctypes.c_void_p, ctypes.c_int]
    ctx = core.Context(0)   # _lib.load caches the debug library loaded above
    assert ctx.lib is lib
    seed = int(sys.argv[1]) if len(sys.argv) > 1 else 21
    inst = synth.td_cvrp(200, 16, seed=seed)
    ctx.set_instance(core.CVRP, inst.durations, inst.demand, inst.capacities, inst.start_times)
    S, C = inst.K - 1, 8
    P0 = synth.random_perms(C, inst.n, seed=9, dtype=np.uint16)
    P = np.array([spec.pack_separators(p, S, inst.demand, inst.capacities) for p in P0])
    P = P.astype(np.int16)
    dem = [int(x) for x in inst.demand]
    RM = (2 * inst.K + 2 + 1 + 7) & ~7
    n = inst.n + S
    for k in range(1, 8):
        cur = torch.from_numpy(P).to(ctx.dev)
        best = cur.clone()
        ck = torch.empty(C, dtype=torch.int64, device=ctx.dev)
        bk = torch.full((C,), -1, dtype=torch.int64, device=ctx.dev)
        ctx.sa_run(cur, ck, best, bk, steps=k, inv_t0=1 / 200.0, inv_alpha=1 / 0.99, seed=21,
                   step0=7, window=16, window_types=2)
        torch.cuda.synchronize()
        buf = np.zeros(4096 * 64, dtype=np.int32)
        assert lib.vrpms_debug_route_dump(buf.ctypes.data, buf.size) == 0
        tours = cur.cpu().numpy().view(np.uint16)
        for c in range(C):
            d = buf[4096 * c:]
            R, ok = int(d[0]), int(d[1])
            dur = d[2:2 + RM]
            rs = d[2 + RM:2 + 2 * RM]
            dsp = d[2 + 2 * RM:2 + 3 * RM]
            rid = d[2 + 3 * RM:2 + 3 * RM + n]
            A = [int(x) for x in tours[c]]
            T = rmod.Tables(inst.durations, A, dem, inst.capacities, inst.start_times)
            bad = []
            if R != T.R:
                bad.append(f"R {R} vs {T.R}")
            else:
                for r in range(R):
                    if dur[r] != T.dur[r]:
                        bad.append(f"dur[{r}] {dur[r]} vs {T.dur[r]}")
                    if rs[r] != T.rs[r]:
                        bad.append(f"rs[{r}] {rs[r]} vs {T.rs[r]}")
                for r in range(R + 1):
                    if dsp[r] != T.dsp[r]:
                        bad.append(f"dsp[{r}] {dsp[r]} vs {T.dsp[r]}")
                for q in range(n):
                    if rid[q] != T.rid[q]:
                        bad.append(f"rid[{q}] {rid[q]} vs {T.rid[q]}")
                        break
            if bad:
                print(f"steps {k} chain {c} (route_ok {ok}): {bad[:8]}", flush=True)
        print(f"steps {k} checked", flush=True)


if __name__ == "__main__":
    build() if sys.argv[1:2] == ["build"] else run()
