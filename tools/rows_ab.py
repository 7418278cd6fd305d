#!/usr/bin/env python3
"""A/B of the API-layout scoring kernels (row-major uint8 tours, the
vrpms_eval layout) on the bench workload (CVRP-100, K = 8, C = 16 Mi):
eval_cvrp_rows2 (LDS-staged tiles) in each (chunk words, candidates per
lane) configuration, with eval_cvrp_words2 on the transposed batch as the
reference point.  Prints kernel time, evals/s, the
LDS-gather fraction (G = n + K against the measured R_gather) and whether
every variant agrees bit for bit (and with the C oracle on a sample)."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import numpy as np  # noqa: E402
import torch  # noqa: E402

import bench  # noqa: E402
from oracle import coracle  # noqa: E402
from vrpms_amd import synth  # noqa: E402
from vrpms_amd.core import CVRP, Context  # noqa: E402


def timed(fn, reps=20):
    for _ in range(3):
        fn()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) * 1e-3 / reps


def main():
    C = int(sys.argv[1]) if len(sys.argv) > 1 else 16 << 20
    ctx = Context(0)
    r_gather = None
    for seed, (n, K, ld) in enumerate([(100, 8, 100), (100, 8, 104), (97, 7, 100), (110, 9, 112)]):
        inst = synth.cvrp(n, K, seed=seed)
        ctx.set_instance(CVRP, inst.durations, inst.demand, inst.capacities, inst.start_times)
        if r_gather is None:
            r_gather = ctx.probe_lds_gather(slots=inst.N * inst.N)
        perms = bench.make_batch(ctx, C - seed, inst.n, seed)
        if ld != inst.n:
            p2 = torch.zeros((perms.shape[0], ld), dtype=torch.uint8, device=ctx.dev)
            p2[:, :inst.n] = perms
            perms = p2
        out, keys = {}, {}
        G = inst.n + inst.K
        for name, cfg in (("rows2_auto", 0), ("rows2_cw8_ilp2", 1), ("rows2_cw16_ilp1", 2),
                          ("rows2_cw4_ilp2", 3), ("rows2_cw8_ilp1", 4)):
            ctx.set_rows_config(cfg)
            k = torch.empty(perms.shape[0], dtype=torch.int64, device=ctx.dev)
            t = timed(lambda: ctx.eval(perms, n=inst.n, out=k))
            out[name] = {"ms": t * 1e3, "evals_per_s": perms.shape[0] / t,
                         "lds_gather_frac": perms.shape[0] / t * G / r_gather}
            keys[name] = k
        ctx.set_rows_config(0)
        words = ctx.to_words(perms, inst.n)
        k = torch.empty(perms.shape[0], dtype=torch.int64, device=ctx.dev)
        t = timed(lambda: ctx.eval_words(words, inst.n, out=k))
        out["words2"] = {"ms": t * 1e3, "evals_per_s": perms.shape[0] / t,
                         "lds_gather_frac": perms.shape[0] / t * G / r_gather}
        keys["words2"] = k
        S = 1 << 16
        ref = coracle.eval_batch(inst.durations, perms[-S:].cpu().numpy(), inst.demand,
                                 inst.capacities, inst.start_times, n=inst.n)[0]
        out["identical"] = all(bool(torch.equal(keys["words2"], v)) for v in keys.values())
        out["oracle_tail_sample_ok"] = all(
            bool((v[-S:].cpu().numpy().view(np.uint64) == ref).all()) for v in keys.values())
        out["n"], out["K"], out["ld"], out["C"] = n, K, ld, int(perms.shape[0])
        out["r_gather"] = r_gather
        print(json.dumps(out), flush=True)
        del perms, words, keys


if __name__ == "__main__":
    main()
