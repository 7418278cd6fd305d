#!/usr/bin/env python3
"""A/B of the headline kernel's fit test (eval_cvrp_words2 on the bench
workload, CVRP-100, K = 8, C = 16 Mi tours): the add's carry (split mode 0,
every demand >= 1) against the compare of the sum's sign (split mode 3).
Prints kernel time and evals/s per form, whether the keys agree bit for bit
and agree with the C oracle on a sample; then the same on an instance with
zero-demand customers (the carry form is not used there: mode 0 == 3)."""
import dataclasses
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
from words_ab import timed  # noqa: E402


def run(ctx, inst, C, seed):
    ctx.set_instance(CVRP, inst.durations, inst.demand, inst.capacities, inst.start_times)
    perms = bench.make_batch(ctx, C, inst.n, seed)
    words = ctx.to_words(perms, inst.n)
    out, keys = {}, {}
    for rep in range(2):
        for mode in (0, 3):
            ctx.set_split_mode(mode)
            k = torch.empty(C, dtype=torch.int64, device=ctx.dev)
            t = timed(lambda: ctx.eval_words(words, inst.n, out=k))
            out[f"mode{mode}_r{rep}"] = {"ms": round(t * 1e3, 4), "G_evals_per_s": round(C / t / 1e9, 3)}
            keys[mode] = k
    ctx.set_split_mode(0)
    same = bool(torch.equal(keys[0], keys[3]))
    idx = np.random.default_rng(seed).choice(C, 4096, replace=False)
    P = perms[torch.as_tensor(idx, device=ctx.dev)].cpu().numpy().astype(np.uint16)[:, :inst.n]
    ref = coracle.eval_batch(inst.durations, P, inst.demand, inst.capacities, inst.start_times)[0]
    oracle_ok = bool((keys[0].cpu().numpy()[idx].view(np.uint64) == ref).all())
    return {"times": out, "carry_equals_compare": same, "equals_oracle_sample": oracle_ok}


def main():
    C = int(sys.argv[1]) if len(sys.argv) > 1 else 16 << 20
    ctx = Context(0)
    inst = synth.cvrp(100, 8, seed=0)
    print(json.dumps({"cvrp100_k8": run(ctx, inst, C, 0)}), flush=True)
    z = synth.cvrp(100, 8, seed=3)
    dem = z.demand.copy()
    dem[1::7] = 0  # zero-demand customers: the carry form is refused
    z = dataclasses.replace(z, demand=dem)
    print(json.dumps({"cvrp100_zero_demands": run(ctx, z, 1 << 20, 3)}), flush=True)


if __name__ == "__main__":
    main()
