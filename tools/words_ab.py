#!/usr/bin/env python3
"""A/B of the LDS-packed scoring kernels on the bench workload (CVRP-100,
K = 8, C = 16 Mi tours): eval_cvrp_words2 with one or two candidates per
lane and one or two words of gathers in flight on the word-interleaved
layout, and eval_cvrp_packed vs eval_cvrp_rows2 on the API's row-major
layout (tools/rows_ab.py sweeps rows2's configurations).  (Round 1 also
timed the first-generation eval_cvrp_words, since removed.)
Prints kernel time, evals/s and whether every variant agrees bit for bit
(and with the C oracle on a sample)."""
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
    for seed, (n, K) in enumerate([(100, 8), (100, 8), (97, 7), (110, 9), (101, 9)]):
        inst = synth.cvrp(n, K, seed=seed)
        ctx.set_instance(CVRP, inst.durations, inst.demand, inst.capacities, inst.start_times)
        perms = bench.make_batch(ctx, C, inst.n, seed)
        words = ctx.to_words(perms, inst.n)
        out = {}
        keys = {}
        for name, gen, ilp, la in (("words2_i1", 0, 1, 1), ("words2_i2", 0, 2, 1),
                                   ("words2_i1_la2", 0, 1, 2), ("words2_i2_la2", 0, 2, 2)):
            ctx.set_words_kernel(gen)
            ctx.set_words_ilp(ilp)
            ctx.set_words_lookahead(la)
            k = torch.empty(C, dtype=torch.int64, device=ctx.dev)
            t = timed(lambda: ctx.eval_words(words, inst.n, out=k))
            out[name] = {"ms": t * 1e3, "evals_per_s": C / t}
            keys[name] = k
        for name, gen in (("rows_packed", 1), ("rows2", 0)):
            ctx.set_words_kernel(gen)
            k = torch.empty(C, dtype=torch.int64, device=ctx.dev)
            t = timed(lambda: ctx.eval(perms, n=inst.n, out=k))
            out[name] = {"ms": t * 1e3, "evals_per_s": C / t}
            keys[name] = k
        ctx.set_words_kernel(0)
        ctx.set_words_ilp(0)
        ctx.set_words_lookahead(0)
        S = 1 << 16
        ref = coracle.eval_batch(inst.durations, perms[:S].cpu().numpy(), inst.demand,
                                 inst.capacities, inst.start_times)[0]
        out["identical"] = all(bool(torch.equal(keys["words2_i2"], v)) for v in keys.values())
        out["oracle_sample_ok"] = all(bool((v[:S].cpu().numpy().view(np.uint64) == ref).all())
                                      for v in keys.values())
        out["n"], out["K"] = n, K
        print(json.dumps(out), flush=True)
        del perms, words, keys


if __name__ == "__main__":
    main()
