#!/usr/bin/env python3
"""Diagnostic: the first SA step at which sa_route_kernel (mode 0),
sa_kernel (mode 2) leave the C restatement on the uniform-fleet TD-200
(seed 21, first-fit start), and at that step which of the 64 candidate
moves the device and C each took and their exact keys (spec.eval_cvrp)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))

import numpy as np  # noqa: E402

import test_separators_gpu as t  # noqa: E402
from oracle import coracle, route_model as rmod, spec  # noqa: E402
from vrpms_amd import synth  # noqa: E402
from vrpms_amd.core import Context  # noqa: E402

ctx = Context(0)
seed = int(sys.argv[1]) if len(sys.argv) > 1 else 21
inst = synth.td_cvrp(200, 16, seed=seed)
t.load(ctx, inst)
S, C, W, TY, IT = inst.K - 1, 8, 16, 2, 1 / 200.0
P0 = synth.random_perms(C, inst.n, seed=9, dtype=np.uint16)
P = np.array([spec.pack_separators(p, S, inst.demand, inst.capacities) for p in P0]).astype(np.int16)
key = spec.seed_key(21)
dem = [int(x) for x in inst.demand]


def c_run(k):
    ccur, cbest = P.view(np.uint16).copy(), P.view(np.uint16).copy()
    cbk = np.full(C, 2**64 - 1, dtype=np.uint64)
    cck = coracle.sa_run(inst.durations, ccur, cbest, cbk, k, IT, 1 / 0.99, 21, 7, inst.demand,
                         inst.capacities, inst.start_times, window=W, window_types=TY)
    return ccur, [int(x) for x in cck]


for mode in (0, 2):
    ctx.set_sa_route(mode)
    firsts = {}
    for k in range(1, 41):
        got = t._run_sa(ctx, P, k, IT, 1 / 0.99, 21, 7, W, TY)
        ccur, cck = c_run(k)
        for c in range(C):
            if c in firsts:
                continue
            if not (got[0][c].view(np.uint16) == ccur[c]).all() or got[1][c] != cck[c]:
                firsts[c] = k
                prev, _ = c_run(k - 1)
                A = [int(x) for x in prev[c]]
                n = len(A)
                step = 7 + k - 1
                T = rmod.Tables(inst.durations, A, dem, inst.capacities, inst.start_times)
                g_tour = [int(x) for x in got[0][c].view(np.uint16)]
                c_tour = [int(x) for x in ccur[c]]
                g_lane = c_lane = None
                rows = []
                for lane in range(64):
                    r = spec.philox4x32_10((step & 0xffffffff, step >> 32, c, lane), key)
                    m = spec.decode_move_window(r[0], r[1], r[2], n, W, TY)
                    mv = rmod._moved(A, m)
                    ref = spec.eval_cvrp(inst.durations, mv, inst.demand, inst.capacities,
                                         inst.start_times, 0)
                    rows.append((ref["key"], lane, m, rmod.price(T, m, inst.K, 0)))
                    if mv == g_tour and g_lane is None:
                        g_lane = lane
                    if mv == c_tour and c_lane is None:
                        c_lane = lane
                rows.sort()
                true_g = spec.eval_cvrp(inst.durations, g_tour, inst.demand, inst.capacities,
                                        inst.start_times, 0)["key"]
                print(f"mode {mode} chain {c} first divergence at step {k}: gpu ck {hex(got[1][c])} "
                      f"(true {hex(true_g)}), C ck {hex(cck[c])}; gpu lane {g_lane}, C lane {c_lane}; "
                      f"best 3 by exact key: {[(hex(x[0]), x[1], x[2], x[3] == x[0] or x[3]) for x in rows[:3]]}; "
                      f"stayed: gpu {g_tour == A}, C {c_tour == A}", flush=True)
    print(f"mode {mode}: first divergence per chain {firsts}", flush=True)
ctx.set_sa_route(0)
