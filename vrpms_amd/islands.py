"""Island model across GPUs: one process per GPU, each runs
independent SA chains / GA populations / ant colonies; every few epochs the
E best tours of every rank are all-gathered (torch.distributed: "nccl" is
RCCL over xGMI on the MI355X node, "gloo" in the CPU tests) and each rank
injects the global E best into its own search.  The payload is tiny
(E x (2n + 8) bytes per rank), so the exchange is latency-bound and runs
only every `exchange_every` epochs.  Brute force shards lexicographic rank
ranges instead and reduces the (key, rank) minimum.

The merge order is deterministic: global elites are ranked by
(key, source rank, position), identical on every rank.
"""
from __future__ import annotations

import math


def _torch():
    import torch
    return torch


def _u64_order(keys):
    """int64 tensor holding uint64 keys -> int64 values with the same order."""
    torch = _torch()
    return keys ^ torch.tensor(-(2**63), dtype=keys.dtype, device=keys.device)


def gather_elites(tours, keys, group=None):
    """All-gather (tours [E][n], keys [E]) from every rank, concatenated in rank order."""
    import torch.distributed as dist
    torch = _torch()
    world = dist.get_world_size(group)
    t32 = tours.to(torch.int32).contiguous()          # gloo has no int16 collectives
    tl = [t32.new_empty(t32.shape) for _ in range(world)]
    kl = [keys.new_empty(keys.shape) for _ in range(world)]
    dist.all_gather(tl, t32, group=group)
    dist.all_gather(kl, keys.contiguous(), group=group)
    return torch.cat(tl).to(tours.dtype), torch.cat(kl)


def select_global(tours, keys, E: int):
    """The E best of the gathered elites by (key, gathered position)."""
    torch = _torch()
    order = torch.argsort(_u64_order(keys), stable=True)[:E]
    return tours[order], keys[order]


def exchange(runner, E: int, group=None):
    """One migration epoch: gather every rank's E elites, inject the global E best."""
    tours, keys = runner.elites(E)
    gt, gk = gather_elites(tours, keys, group)
    bt, bk = select_global(gt, gk, E)
    runner.inject(bt, bk)
    return bk


def run_islands(runner, epochs: int, exchange_every: int = 5, E: int = 8, group=None):
    """Advance `runner` for `epochs`, migrating every `exchange_every` epochs."""
    import torch.distributed as dist
    dist_on = dist.is_available() and dist.is_initialized()
    for e in range(1, epochs + 1):
        runner.epoch()
        if dist_on and dist.get_world_size(group) > 1 and e % exchange_every == 0:
            exchange(runner, E, group)
    return runner.best()


def run_fixed(runner, epochs: int, exchange_every: int = 5, E: int = 8, group=None, sync=None):
    """`epochs` island epochs with a migration every `exchange_every` epochs,
    on a FIXED count: every rank runs the identical control flow (no
    wall-clock exit), so every rank enters every collective.  With one rank
    the migration is local (the E best re-injected into the worst chains).
    `sync` (e.g. torch.cuda.synchronize) brackets each exchange so its time
    is measured apart.  Returns (exchanges, exchange_seconds)."""
    import time

    import torch.distributed as dist
    multi = dist.is_available() and dist.is_initialized() and dist.get_world_size(group) > 1
    n_ex, t_ex = 0, 0.0
    for e in range(1, epochs + 1):
        runner.epoch()
        if e % exchange_every == 0:
            if sync:
                sync()
            t0 = time.perf_counter()
            if multi:
                exchange(runner, E, group)
            else:
                runner.inject(*runner.elites(E))
            if sync:
                sync()
            t_ex += time.perf_counter() - t0
            n_ex += 1
    return n_ex, t_ex


def global_best(key: int, tour, n: int, group=None, device=None):
    """Reduce the per-rank best (key, tour) to the global best on every rank."""
    import torch.distributed as dist
    torch = _torch()
    t = torch.as_tensor(list(tour), dtype=torch.int16, device=device).reshape(1, n)
    k = torch.tensor([key - (1 << 64) if key >= (1 << 63) else key], dtype=torch.int64,
                     device=device)
    gt, gk = gather_elites(t, k, group)
    bt, bk = select_global(gt, gk, 1)
    return int(bk[0]) & (2**64 - 1), bt[0].tolist()


def bf_rank_range(n: int, rank: int, world: int):
    """Contiguous share [lo, hi) of the n! lexicographic ranks for one rank."""
    total = math.factorial(n)
    return total * rank // world, total * (rank + 1) // world


def bf_distributed(bf_fn, n: int, group=None, device=None):
    """bf_fn(lo, hi) -> (key, rank) on this rank's share; returns the global
    (key, rank) minimum (ties -> smallest rank)."""
    import torch.distributed as dist
    torch = _torch()
    world, me = dist.get_world_size(group), dist.get_rank(group)
    lo, hi = bf_rank_range(n, me, world)
    k, r = bf_fn(lo, hi)
    to_i64 = lambda v: v - (1 << 64) if v >= (1 << 63) else v  # noqa: E731
    pair = torch.tensor([[to_i64(k), to_i64(r)]], dtype=torch.int64, device=device)
    parts = [torch.empty_like(pair) for _ in range(world)]
    dist.all_gather(parts, pair, group=group)
    best = min((int(p[0, 0]) & (2**64 - 1), int(p[0, 1]) & (2**64 - 1)) for p in parts)
    return best
