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
