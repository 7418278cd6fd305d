"""Island model across GPUs: one process per GPU, each runs
independent SA chains / GA populations / ant colonies; every few epochs the
E best tours of every rank are all-gathered and every rank injects the same
global E best into its own search.

The exchange is the library's (include/vrpms.h):
  * ``vrpms_island_exchange`` -- pack the E elites (device top-E), one RCCL
    ``ncclAllGather`` of the messages over xGMI, merge by (key, rank,
    position) on the device, inject; used once ``init_comm`` has given the
    context its communicator;
  * without a communicator but with a multi-rank torch.distributed group
    (e.g. "gloo"), the same library pack / merge / inject run around a
    torch.distributed all-gather of the message bytes (the fallback
    communicator);
  * with one rank, the exchange is local (pack -> merge -> inject).
The payload is tiny (E x (2n + 8) bytes per rank), so the exchange is
latency-bound and runs only every `exchange_every` epochs.  Brute force
shards lexicographic rank ranges instead and reduces the (key, rank) minimum.
"""
from __future__ import annotations

import math


def _torch():
    import torch
    return torch


def _dist_world(group=None) -> int:
    import torch.distributed as dist
    if not (dist.is_available() and dist.is_initialized()):
        return 1
    return dist.get_world_size(group)


def _agree(flag: int, group=None, device=None) -> int:
    """MIN of `flag` over the group (1 on every rank only if 1 on all)."""
    import torch.distributed as dist
    torch = _torch()
    if dist.get_backend(group) == "nccl":
        device = device if device is not None else torch.device("cuda",
                                                                torch.cuda.current_device())
    else:
        device = "cpu"
    f = torch.tensor([int(flag)], dtype=torch.int32, device=device)
    dist.all_reduce(f, op=dist.ReduceOp.MIN, group=group)
    return int(f.item())


def init_comm(ctx, group=None, timeout_s: int | None = None) -> int:
    """Give `ctx` an RCCL communicator spanning the torch.distributed group:
    rank 0 draws the unique id (vrpms_island_unique_id), the group
    broadcasts it, every rank calls vrpms_island_init (non-blocking creation
    with a deadline, so a rank that never joins is an error, not a hang).
    The ranks then agree over the torch group: the communicator is used only
    when every rank has one (ctx.island_comm_group is set on all ranks or on
    none), otherwise every rank raises.  Returns the world."""
    import torch.distributed as dist
    world, rank = dist.get_world_size(group), dist.get_rank(group)
    if timeout_s is not None:
        ctx.set_island_timeout(timeout_s)
    err = None
    # rank 0 always reaches the broadcast: a failed unique id travels as None
    # (every rank then skips island_init), so no rank is left waiting in a
    # collective the others never enter before the agreement below
    uid = None
    if rank == 0:
        try:
            uid = ctx.island_unique_id()
        except Exception as e:  # noqa: BLE001 -- reported after the agreement
            err = e
    obj = [uid]
    dist.broadcast_object_list(obj, src=0, group=group)
    ok = 0
    if obj[0] is None:
        err = err or RuntimeError("rank 0 could not create the RCCL unique id")
    else:
        try:
            ctx.island_init(obj[0], rank, world)
            ok = int(ctx.island_world() == world)
        except Exception as e:  # noqa: BLE001 -- reported after the agreement
            ok, err = 0, e
    if not _agree(ok, group, getattr(ctx, "dev", None)):
        ctx.island_comm_group = None
        raise RuntimeError(f"vrpms_island_init failed on at least one rank "
                           f"(this rank: {err or 'ok'})")
    ctx.island_comm_group = (group, world)
    return world


def all_gather_bytes(msg, group=None):
    """The fallback communicator: all-gather one uint8 message per rank
    through torch.distributed, concatenated in rank order (CPU tensors for
    gloo, device tensors for nccl)."""
    import torch.distributed as dist
    torch = _torch()
    world = dist.get_world_size(group)
    send = msg if dist.get_backend(group) == "nccl" else msg.cpu()
    parts = [torch.empty_like(send) for _ in range(world)]
    dist.all_gather(parts, send.contiguous(), group=group)
    return torch.cat(parts)


def exchange(runner, E: int, group=None):
    """One migration epoch: every rank's E elites of runner.src() are
    gathered, the global E best by (key, rank, position) are injected into
    runner.dst() by runner.inject_mode.  Returns nothing (device state)."""
    ctx = runner.ctx
    world = _dist_world(group)
    # the library's communicator only when init_comm agreed on it across the
    # ranks for this group: every rank takes the same path
    if world == 1 or getattr(ctx, "island_comm_group", None) == (group, world):
        ctx.island_exchange(runner.src(), runner.dst(), runner.inject_mode, E, runner.groups)
        return
    msg = ctx.island_pack(*runner.src(), E)
    msgs = all_gather_bytes(msg, group)
    tours, keys = ctx.island_merge(msgs, world, E, runner.n)
    ctx.pool_inject(*runner.dst(), runner.inject_mode, tours, keys, runner.groups)


def exchange_local(runners, E: int):
    """One migration among islands held by ONE process on several devices
    (the service's multi-GPU path): each runner's E elites are
    packed on its device, every message is copied device to device (xGMI
    peer copies), and each device merges the same gathered messages and
    injects the global E best -- the all-gather exchange without a
    communicator.  Messages go in runner order, so every island receives the
    same migrants as vrpms_island_exchange would give ranks in that order."""
    torch = _torch()
    msgs = [r.ctx.island_pack(*r.src(), E) for r in runners]
    world = len(runners)
    for r in runners:
        allm = torch.cat([m.to(r.ctx.dev) for m in msgs])
        tours, keys = r.ctx.island_merge(allm, world, E, r.n)
        r.ctx.pool_inject(*r.dst(), r.inject_mode, tours, keys, r.groups)


def run_local(runners, epochs: int, exchange_every: int = 5, E: int = 8, time_limit=None,
              sync=None):
    """Islands on several devices of one process: every epoch is enqueued on
    each device in turn (the launches are asynchronous, so the devices run
    together), a migration every `exchange_every` epochs.  Stops after
    `epochs`, or when `time_limit` seconds have passed (checked after each
    epoch, as the single-device search does).  Returns the global best
    (key, tour) by (key, island)."""
    import time
    t0 = time.perf_counter()
    for e in range(1, epochs + 1):
        for r in runners:
            r.epoch()
        if e % exchange_every == 0 and len(runners) > 1:
            exchange_local(runners, E)
        if sync is not None:
            sync()
        if time_limit is not None and time.perf_counter() - t0 >= time_limit:
            break
    best = None
    for r in runners:
        k, t = r.best()
        if best is None or k < best[0]:
            best = (k, t)
    return best


def run_islands(runner, epochs: int, exchange_every: int = 5, E: int = 8, group=None):
    """Advance `runner` for `epochs`, migrating every `exchange_every` epochs."""
    for e in range(1, epochs + 1):
        runner.epoch()
        if _dist_world(group) > 1 and e % exchange_every == 0:
            exchange(runner, E, group)
    return runner.best()


def run_fixed(runner, epochs: int, exchange_every: int = 5, E: int = 8, group=None, sync=None):
    """`epochs` island epochs with a migration every `exchange_every` epochs,
    on a FIXED count: every rank runs the identical control flow (no
    wall-clock exit), so every rank enters every collective.  With one rank
    the migration is local (the E best re-injected).  `sync` (e.g.
    torch.cuda.synchronize) brackets each exchange so its time is measured
    apart.  Returns (exchanges, exchange_seconds)."""
    import time
    n_ex, t_ex = 0, 0.0
    for e in range(1, epochs + 1):
        runner.epoch()
        if e % exchange_every == 0:
            if sync:
                sync()
            t0 = time.perf_counter()
            exchange(runner, E, group)
            if sync:
                sync()
            t_ex += time.perf_counter() - t0
            n_ex += 1
    return n_ex, t_ex


def global_best(runner, group=None):
    """The best (key, tour) over every rank's runner.src(), identical on
    every rank: a one-elite pack / all-gather / merge."""
    ctx = runner.ctx
    world = _dist_world(group)
    msg = ctx.island_pack(*runner.src(), 1)
    msgs = msg if world == 1 else all_gather_bytes(msg, group)
    tours, keys = ctx.island_merge(msgs, world, 1, runner.n)
    return int(keys[0]) & (2**64 - 1), [int(x) for x in tours[0].cpu().tolist()]


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
