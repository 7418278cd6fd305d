"""A CPU stand-in for ``vrpms_amd.core.Context`` -- TEST INFRASTRUCTURE ONLY.

It implements the subset of the Context API the search runners and the
island model call (random_tours, eval, sa_run, ga_generation, argmin, the
pool / island-message operations) with the oracle restatements
(oracle/coracle.py, oracle/search.py, oracle/pool.py) on CPU torch tensors,
so the real ``vrpms_amd.runners`` classes and ``vrpms_amd.islands`` can be
driven through a multi-rank gloo group in the CPU test suite.  The product
path never imports it (vrpms_amd fails loudly without its HIP library).
"""
from __future__ import annotations

import numpy as np

from . import coracle, pool, search, spec

M64 = (1 << 64) - 1


def _u64(t):
    return [int(x) & M64 for x in t.reshape(-1).tolist()]


def _i64(vals):
    import torch
    return torch.tensor([v - (1 << 64) if v >= (1 << 63) else v for v in vals], dtype=torch.int64)


class StandInContext:
    def __init__(self, inst, objective: int = 0):
        import torch
        self.dev = torch.device("cpu")
        self.inst = inst
        self.N = inst.N
        self.objective = objective
        self.problem = 0 if inst.problem == "tsp" else 1
        self.score = search.Scorer(inst.durations, inst.demand, inst.capacities, inst.start_times,
                                   inst.problem, objective)

    # -- runners --------------------------------------------------------------
    def random_tours(self, count, n, seed, stream_id=0, ld=None, dtype=None, n_sep=0):
        import torch
        rows = [pool.philox_tour(n, seed, r, stream_id, n_sep) for r in range(count)]
        return torch.tensor(np.array(rows, dtype=np.int64).reshape(count, n + n_sep),
                            dtype=torch.int16)

    def eval(self, perms, n=None, with_parts=False, out=None):
        P = perms.numpy().astype(np.uint16)
        k = coracle.eval_batch(self.inst.durations, P, self.inst.demand, self.inst.capacities,
                               self.inst.start_times, self.problem, self.objective)[0]
        return _i64([int(x) for x in k])

    def sa_run(self, cur, cur_key, best, best_key, steps, inv_t0, inv_alpha, seed, step0,
               window=0, window_types=0, moves=64):
        c = cur.numpy().view(np.uint16).copy()
        b = best.numpy().view(np.uint16).copy()
        bk = np.array(_u64(best_key), dtype=np.uint64)
        ck = coracle.sa_run(self.inst.durations, c, b, bk, steps, inv_t0, inv_alpha, seed, step0,
                            self.inst.demand, self.inst.capacities, self.inst.start_times,
                            self.problem, self.objective, window=window,
                            window_types=window_types, resync=True, moves=moves)
        cur.copy_(_as_i16(c))
        best.copy_(_as_i16(b))
        cur_key.copy_(_i64([int(x) for x in ck]))
        best_key.copy_(_i64([int(x) for x in bk]))

    def ga_generation(self, pop, keys, generations, pmut, seed, gen0):
        islands, P, n = pop.shape
        pm = min(int(round(float(pmut) * 2**32)), 2**32 - 1)
        rp = [[list(r) for r in pop[i].tolist()] for i in range(islands)]
        rk = [_u64(keys[i]) for i in range(islands)]
        for g in range(generations):
            rp, rk = search.ga_generation(self.score, rp, rk, seed, gen0 + g, pm)
        import torch
        pop.copy_(torch.tensor(rp, dtype=torch.int16))
        keys.copy_(_i64([k for ks in rk for k in ks]).view(islands, P))

    def insert_separators(self, tours, n_sep):
        import torch
        rows = [spec.insert_separators(t, n_sep, self.inst.demand, self.inst.capacities)
                for t in tours.tolist()]
        return torch.tensor(rows, dtype=torch.int16)

    def pack_separators(self, tours, n_sep):
        import torch
        rows = [spec.pack_separators(t, n_sep, self.inst.demand, self.inst.capacities)
                for t in tours.tolist()]
        return torch.tensor(rows, dtype=torch.int16)

    def argmin(self, keys):
        vals = _u64(keys)
        i = min(range(len(vals)), key=lambda j: (vals[j], j))
        return vals[i], i

    # -- pools and island messages ----------------------------------------------
    def island_world(self) -> int:
        return 0

    def pool_elites(self, tours, keys, E):
        t, k = pool.pool_elites(tours.reshape(-1, tours.shape[-1]).tolist(), _u64(keys), E)
        import torch
        return torch.tensor(t, dtype=torch.int16), _i64(k)

    def pool_inject(self, tours, keys, mode, mig_tours, mig_keys, groups=1):
        import torch
        n = tours.shape[-1]
        t, k = pool.pool_inject(tours.reshape(-1, n).tolist(), _u64(keys), mode,
                                mig_tours.tolist(), _u64(mig_keys), groups)
        tours.copy_(torch.tensor(t, dtype=torch.int16).view(tours.shape))
        keys.copy_(_i64(k).view(keys.shape))

    def island_msg_bytes(self, E, n):
        return pool.msg_bytes(E, n)

    def island_pack(self, tours, keys, E):
        import torch
        n = tours.shape[-1]
        b = pool.island_pack(tours.reshape(-1, n).tolist(), _u64(keys), E, n)
        return torch.frombuffer(bytearray(b), dtype=torch.uint8)

    def island_merge(self, msgs, world, E, n):
        import torch
        t, k = pool.island_merge(bytes(msgs.numpy().tobytes()), world, E, n)
        return torch.tensor(t, dtype=torch.int16).view(E, n), _i64(k)

    def island_exchange(self, src, dst, mode, E, groups=1):
        msg = self.island_pack(*src, E)
        t, k = self.island_merge(msg, 1, E, src[0].shape[-1])
        self.pool_inject(*dst, mode, t, k, groups)


def _as_i16(a):
    import torch
    return torch.from_numpy(a.view(np.int16).copy())


__all__ = ["StandInContext", "spec"]
