#!/usr/bin/env python3
"""Diagnostic: first step at which sa_route_kernel (mode 0/3) or sa_kernel
(mode 2) leaves the C restatement's trajectory on heterogeneous-fleet cases
(one chain at a time, growing step counts)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests"))

import numpy as np  # noqa: E402
import torch  # noqa: E402

import test_separators_gpu as t  # noqa: E402
from oracle import coracle, spec  # noqa: E402
from vrpms_amd import synth  # noqa: E402
from vrpms_amd.core import Context  # noqa: E402

ctx = Context(0)
cases = {c[0]: c for c in t.ROUTE_CASES}
for name in sys.argv[1:] or ["td200_het_classes_starts", "x1000_asym_het_starts",
                             "td200_het_shuffled_hot", "cvrp150_asym_het_random"]:
    _, maker, start, chains, steps, inv_t0, window, types = cases[name]
    inst = maker()
    t.load(ctx, inst)
    S = inst.K - 1
    if start == "random":
        P = t.sep_tours(chains, inst.n, S, seed=9, dtype=np.uint16)
    else:
        P0 = synth.random_perms(chains, inst.n, seed=9, dtype=np.uint16)
        P = np.array([spec.pack_separators(p, S, inst.demand, inst.capacities) for p in P0])
    P = P.astype(np.int16)
    for mode in (0, 2):
        ctx.set_sa_route(mode)
        first = None
        for k in sorted(set([1, 2, 4, 8, 16, 24, 32, 40, 48, 52, 56, 58, 59, steps])):
            if k > steps:
                break
            got = t._run_sa(ctx, P, k, inv_t0, 1 / 0.99, 21, 7, window, types)
            ccur, cbest = P.view(np.uint16).copy(), P.view(np.uint16).copy()
            cbk = np.full(chains, 2**64 - 1, dtype=np.uint64)
            cck = coracle.sa_run(inst.durations, ccur, cbest, cbk, k, inv_t0, 1 / 0.99, 21, 7,
                                 inst.demand, inst.capacities, inst.start_times, window=window,
                                 window_types=types)
            bad = [c for c in range(chains) if not (got[0][c].view(np.uint16) == ccur[c]).all()
                   or got[1][c] != int(cck[c])]
            if bad:
                c = bad[0]
                first = (k, bad, hex(got[1][c]), hex(int(cck[c])))
                break
        print(name, "mode", mode, "first divergence (steps, chains, gpu key, C key):", first,
              flush=True)
    ctx.set_sa_route(0)
