#!/usr/bin/env python3
"""Determinism / parity probe of sa_route_kernel on hour-indexed TD-200:
the same SA call twice on the device (must be identical) and against the C
restatement, for a heterogeneous fleet and for the uniform fleet of the
same instance, at a few step counts."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))

import dataclasses  # noqa: E402

import numpy as np  # noqa: E402

import test_separators_gpu as t  # noqa: E402
from oracle import coracle, spec  # noqa: E402
from vrpms_amd import synth  # noqa: E402
from vrpms_amd.core import Context  # noqa: E402

ctx = Context(0)
base = synth.td_cvrp(200, 16, seed=21)
insts = {"het": t._starts(t._classes(base, (1.3, 1.0, 0.8))),
         "caps_only": t._classes(base, (1.3, 1.0, 0.8)),
         "starts_only": t._starts(base),
         "uniform": base}
for name, inst in insts.items():
    t.load(ctx, inst)
    S = inst.K - 1
    P0 = synth.random_perms(8, inst.n, seed=9, dtype=np.uint16)
    P = np.array([spec.pack_separators(p, S, inst.demand, inst.capacities) for p in P0])
    P = P.astype(np.int16)
    for steps in (20, 40, 60, 120):
        a = t._run_sa(ctx, P, steps, 1 / 200.0, 1 / 0.99, 21, 7, 16, 2)
        b = t._run_sa(ctx, P, steps, 1 / 200.0, 1 / 0.99, 21, 7, 16, 2)
        same = (a[0] == b[0]).all() and a[1] == b[1]
        ccur, cbest = P.view(np.uint16).copy(), P.view(np.uint16).copy()
        cbk = np.full(8, 2**64 - 1, dtype=np.uint64)
        cck = coracle.sa_run(inst.durations, ccur, cbest, cbk, steps, 1 / 200.0, 1 / 0.99, 21, 7,
                             inst.demand, inst.capacities, inst.start_times, window=16,
                             window_types=2)
        ok = (a[0].view(np.uint16) == ccur).all() and a[1] == [int(x) for x in cck]
        bad = [c for c in range(8) if a[1][c] != int(cck[c])]
        print(f"{name} steps {steps}: deterministic {same}, equals C {ok}, chains off {bad}",
              flush=True)
