"""The RCCL side of vrpms_island_exchange on the one-GPU box: a world-1
communicator (ncclGetUniqueId -> ncclCommInitRank -> ncclAllGather) must
give the same migrants as the local exchange.  Multi-rank RCCL runs only on
the 8-GPU node (bench.py island leg); its merge / inject semantics at
world > 1 are covered by tests/test_pool_gpu.py (fabricated messages) and
tests/test_islands_cpu.py (gloo)."""
import numpy as np
import pytest

from oracle import pool as opool

pytestmark = pytest.mark.gpu


def test_rccl_world1_exchange_equals_local():
    import torch

    from vrpms_amd.core import Context
    rng = np.random.default_rng(3)
    n, E, count = 30, 5, 128
    src_t = rng.integers(1, 31, size=(count, n))
    src_k = rng.integers(0, 2**60, size=count).tolist()
    dst_t = rng.integers(1, 31, size=(count, n))
    dst_k = rng.integers(0, 2**60, size=count).tolist()
    with Context(0) as ctx:
        ctx.island_init(ctx.island_unique_id(), 0, 1)
        assert ctx.island_world() == 1
        dev = ctx.dev
        s = (torch.tensor(src_t, dtype=torch.int16, device=dev),
             torch.tensor(src_k, dtype=torch.int64, device=dev))
        d = (torch.tensor(dst_t, dtype=torch.int16, device=dev),
             torch.tensor(dst_k, dtype=torch.int64, device=dev))
        ctx.island_exchange(s, d, opool.INJECT_WORST, E)
        torch.cuda.synchronize(dev)
        got_t, got_k = d[0].cpu().tolist(), d[1].cpu().tolist()
    msg = opool.island_pack(src_t.tolist(), src_k, E, n)
    mt, mk = opool.island_merge(msg, 1, E, n)
    rt, rk = opool.pool_inject(dst_t.tolist(), dst_k, opool.INJECT_WORST, mt, mk)
    assert got_k == rk and got_t == rt


def test_rccl_init_times_out_when_a_rank_never_joins():
    """vrpms_island_init creates the communicator non-blocking with a
    deadline: rank 0 of a world-2 communicator whose rank 1 never arrives
    gets VRPMS_ETIMEOUT (and no communicator) instead of hanging."""
    import time

    from vrpms_amd import _lib
    from vrpms_amd.core import Context, VrpmsError
    with Context(0) as ctx:
        ctx.set_island_timeout(3)
        t0 = time.perf_counter()
        with pytest.raises(VrpmsError) as ei:
            ctx.island_init(ctx.island_unique_id(), 0, 2)
        assert ei.value.code == _lib.VRPMS_ETIMEOUT
        assert time.perf_counter() - t0 < 60
        assert ctx.island_world() == 0
        # a later world-1 communicator still forms on the same context
        ctx.island_init(ctx.island_unique_id(), 0, 1)
        assert ctx.island_world() == 1


def test_init_comm_agrees_and_runner_exchange_uses_library_rccl():
    """islands.init_comm over a world-1 torch.distributed group: the ranks
    agree on the communicator, and islands.exchange of a real SARunner then
    runs vrpms_island_exchange (library RCCL) -- same migrants as the local
    pack / merge / inject replay (oracle/pool.py)."""
    import os
    import socket

    import torch
    import torch.distributed as dist

    from oracle import pool as opool
    from vrpms_amd import islands, runners, synth
    from vrpms_amd.core import CVRP, Context
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=0, world_size=1)
    try:
        with Context(0) as ctx:
            inst = synth.cvrp(30, 3, seed=2)
            ctx.set_instance(CVRP, inst.durations, inst.demand, inst.capacities, inst.start_times)
            assert islands.init_comm(ctx, timeout_s=60) == 1
            assert ctx.island_comm_group == (None, 1) and ctx.island_world() == 1
            r = runners.SARunner(ctx, inst.n, chains=16, seed=3, total_steps=40,
                                 steps_per_epoch=20, durations=inst.durations)
            r.epoch()
            torch.cuda.synchronize(ctx.dev)
            src = [x.cpu() for x in r.src()]
            dst = [x.cpu() for x in r.dst()]
            islands.exchange(r, 4)
            torch.cuda.synchronize(ctx.dev)
            got_t, got_k = r.dst()[0].cpu().tolist(), r.dst()[1].cpu().tolist()
    finally:
        dist.destroy_process_group()
    M = (1 << 64) - 1
    n = inst.n
    msg = opool.island_pack(src[0].tolist(), [int(k) & M for k in src[1].tolist()], 4, n)
    mt, mk = opool.island_merge(msg, 1, 4, n)
    rt, rk = opool.pool_inject(dst[0].tolist(), [int(k) & M for k in dst[1].tolist()],
                               opool.INJECT_WORST, mt, mk)
    assert got_t == rt
    assert [int(k) & M for k in got_k] == rk
