"""GPU parity of the population / island kernels (csrc/pool.hip) against
oracle/pool.py: Philox start tours, elite selection, the three injection
modes, island messages byte for byte, the multi-rank merge and the local
exchange; ACO's device-side colony-best tracking."""
import numpy as np
import pytest

from oracle import pool as opool
from oracle import search
from vrpms_amd import synth

pytestmark = pytest.mark.gpu
M64 = (1 << 64) - 1


def torch_():
    import torch
    return torch


def u64(t):
    return [int(x) & M64 for x in t.reshape(-1).cpu().tolist()]


def i64(vals):
    torch = torch_()
    return torch.tensor([v - (1 << 64) if v >= (1 << 63) else v for v in vals], dtype=torch.int64)


@pytest.mark.parametrize("n,ld,dt", [(1, 1, "i16"), (2, 4, "u8"), (13, 16, "u8"), (100, 100, "u8"),
                                     (100, 100, "i16"), (1000, 1000, "i16")])
def test_random_tours_match_oracle(ctx, n, ld, dt):
    torch = torch_()
    dtype = torch.uint8 if dt == "u8" else torch.int16
    T = ctx.random_tours(77, n, seed=2**40 + 5, stream_id=3, ld=ld, dtype=dtype).cpu().numpy()
    T = T.astype(np.int64) & (0xFF if dt == "u8" else 0xFFFF)
    for r in (0, 1, 38, 76):
        assert T[r, :n].tolist() == opool.philox_tour(n, 2**40 + 5, r, 3)
        assert (T[r, n:] == 0).all()
    assert all(sorted(row[:n]) == list(range(1, n + 1)) for row in T.tolist())


def _keys(rng, count, dup=True):
    k = rng.integers(0, 2**62, size=count, dtype=np.int64).astype(np.uint64)
    if dup:
        k[rng.integers(0, count, size=count // 3)] = k[0]      # ties resolved by index
        k[rng.integers(0, count, size=5)] = np.uint64(M64)
    return [int(x) for x in k]


@pytest.mark.parametrize("count,E", [(7, 7), (300, 16), (5000, 32), (70000, 8)])
def test_pool_elites_match_oracle(ctx, count, E):
    torch = torch_()
    rng = np.random.default_rng(count)
    n = 5
    keys = _keys(rng, count)
    tours = rng.integers(1, 6, size=(count, n))
    t, k = ctx.pool_elites(torch.tensor(tours, dtype=torch.int16, device=ctx.dev),
                           i64(keys).to(ctx.dev), E)
    rt, rk = opool.pool_elites(tours.tolist(), keys, E)
    assert u64(k) == rk and t.cpu().tolist() == rt


@pytest.mark.parametrize("mode", [opool.INJECT_WORST, opool.INJECT_SORTED, opool.INJECT_BETTER])
def test_pool_inject_matches_oracle(ctx, mode):
    torch = torch_()
    rng = np.random.default_rng(mode)
    groups, P, n, E = 4, 50, 9, 11
    count = groups * P
    keys = _keys(rng, count)
    if mode == opool.INJECT_SORTED:   # GA islands are kept sorted by (key, index)
        keys = [k for g in range(groups) for k in sorted(keys[g * P:(g + 1) * P])]
    tours = rng.integers(1, 10, size=(count, n))
    mk = sorted(_keys(rng, E, dup=False))
    mt = rng.integers(1, 10, size=(E, n))
    dt = torch.tensor(tours, dtype=torch.int16, device=ctx.dev)
    dk = i64(keys).to(ctx.dev)
    ctx.pool_inject(dt, dk, mode, torch.tensor(mt, dtype=torch.int16, device=ctx.dev),
                    i64(mk).to(ctx.dev), groups)
    rt, rk = opool.pool_inject(tours.tolist(), keys, mode, mt.tolist(), mk, groups)
    assert u64(dk) == rk and dt.cpu().tolist() == rt


def test_island_pack_bytes_and_merge_match_oracle(ctx):
    torch = torch_()
    rng = np.random.default_rng(11)
    world, count, n, E = 5, 400, 37, 12
    pools = [(rng.integers(1, 38, size=(count, n)), _keys(rng, count)) for _ in range(world)]
    msgs = []
    for tours, keys in pools:
        m = ctx.island_pack(torch.tensor(tours, dtype=torch.int16, device=ctx.dev),
                            i64(keys).to(ctx.dev), E)
        got = bytes(m.cpu().numpy().tobytes())
        assert got == opool.island_pack(tours.tolist(), keys, E, n)
        msgs.append(m)
    assert ctx.island_msg_bytes(E, n) == opool.msg_bytes(E, n)
    t, k = ctx.island_merge(torch.cat(msgs), world, E, n)
    rt, rk = opool.island_merge(b"".join(bytes(m.cpu().numpy().tobytes()) for m in msgs), world,
                                E, n)
    assert u64(k) == rk and t.cpu().tolist() == rt


def test_local_exchange_equals_oracle(ctx):
    torch = torch_()
    rng = np.random.default_rng(5)
    n, E = 20, 6
    src_t = rng.integers(1, 21, size=(64, n))
    src_k = _keys(rng, 64)
    dst_t = rng.integers(1, 21, size=(64, n))
    dst_k = _keys(rng, 64)
    s = (torch.tensor(src_t, dtype=torch.int16, device=ctx.dev), i64(src_k).to(ctx.dev))
    d = (torch.tensor(dst_t, dtype=torch.int16, device=ctx.dev), i64(dst_k).to(ctx.dev))
    assert ctx.island_world() == 0
    ctx.island_exchange(s, d, opool.INJECT_WORST, E)
    msg = opool.island_pack(src_t.tolist(), src_k, E, n)
    mt, mk = opool.island_merge(msg, 1, E, n)
    rt, rk = opool.pool_inject(dst_t.tolist(), dst_k, opool.INJECT_WORST, mt, mk)
    assert u64(d[1]) == rk and d[0].cpu().tolist() == rt


def test_aco_colony_best_tracking_on_device(ctx):
    from vrpms_amd.core import CVRP
    torch = torch_()
    inst = synth.cvrp(12, 3, seed=1, slack=0.95)
    ctx.set_instance(CVRP, inst.durations, inst.demand, inst.capacities, inst.start_times)
    colonies, ants = 3, 8
    tau, eta = ctx.aco_init(colonies, 1 << 20)
    bt = torch.zeros((colonies, inst.n), dtype=torch.int16, device=ctx.dev)
    bk = torch.full((colonies,), -1, dtype=torch.int64, device=ctx.dev)
    ref_k = [M64] * colonies
    ref_t = [[0] * inst.n for _ in range(colonies)]
    for it in range(4):
        tours, keys, ib = ctx.aco_iteration(tau, eta, ants, seed=9, it=it, best_tours=bt,
                                            best_keys=bk)
        T = tours.cpu().tolist()
        for c, (k, a) in enumerate(ib.cpu().tolist()):
            k &= M64
            if k < ref_k[c]:
                ref_k[c], ref_t[c] = k, T[c][a]
    assert u64(bk) == ref_k and bt.cpu().tolist() == ref_t
    sc = search.Scorer(inst.durations, inst.demand, inst.capacities, inst.start_times, "cvrp")
    assert all(sc(t) == k for t, k in zip(ref_t, ref_k))
