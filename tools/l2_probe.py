#!/usr/bin/env python3
"""Staged-kernel probe: cfg 3 (TD-VRP-200 x 24 h) and cfg 4 (X-1000) scoring
rates per kernel variant, against the measured L2-gather ceiling.  Checks a
sample of every variant's keys against the C oracle.  One JSON line each."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import numpy as np  # noqa: E402
import torch  # noqa: E402

from oracle import coracle  # noqa: E402
from vrpms_amd import synth  # noqa: E402
from vrpms_amd.core import CVRP, Context  # noqa: E402


def timed(fn, reps=5):
    fn()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) * 1e-3 / reps


def perms(C, n, dt, seed):
    g = torch.Generator(device="cuda")
    g.manual_seed(seed)
    out = torch.empty((C, n), dtype=dt, device="cuda")
    for s in range(0, C, 1 << 16):
        r = torch.rand((min(C, s + (1 << 16)) - s, n), generator=g, device="cuda")
        out[s:s + r.shape[0]] = (r.argsort(dim=1) + 1).to(dt)
    return out


def main():
    ctx = Context(0)
    r_l2 = {s: ctx.probe_l2_gather(slots=s) for s in (24 * 201 * 201, 1001 * 1001)}
    print(json.dumps({"probe": "l2_gather", "gathers_per_s": r_l2}), flush=True)
    for name, inst, C, dt in (("cfg3_tdvrp200", synth.td_cvrp(200, 16, seed=0), 1 << 21, torch.uint8),
                              ("cfg4_x1000", synth.x_style(1000, seed=0), 1 << 18, torch.int16)):
        ctx.set_instance(CVRP, inst.durations, inst.demand, inst.capacities, inst.start_times)
        P = perms(C, inst.n, dt, 5)
        keys = torch.empty(C, dtype=torch.int64, device="cuda")
        S = 2048
        host = P[:S].cpu().numpy()
        host = host.view(np.uint16) if dt == torch.int16 else host
        ref = coracle.eval_batch(inst.durations, host, inst.demand, inst.capacities,
                                 inst.start_times)[0]
        for m in (0, 1, 2):
            ctx.set_staged_m(m)
            t = timed(lambda: ctx.eval(P, out=keys))
            ok = bool((keys[:S].cpu().numpy().view(np.uint64) == ref).all())
            G = inst.n + inst.K
            slots = inst.H * inst.N * inst.N
            rate = C / t
            print(json.dumps({"config": name, "staged_m": m, "evals_per_s": rate, "ms": t * 1e3,
                              "gathers_per_eval": inst.n, "G": G,
                              "frac_l2": rate * inst.n / r_l2.get(slots, r_l2[24 * 201 * 201]),
                              "parity": ok}), flush=True)
        ctx.set_staged_m(0)


if __name__ == "__main__":
    main()
