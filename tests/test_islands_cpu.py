"""world_size-2 gloo tests of the island model (the N > 1 path) on CPU.

The real runners of vrpms_amd.runners (SARunner, GARunner) are driven
through vrpms_amd.islands with oracle.standin.StandInContext in place of the
GPU context: the same exchange code path as on the MI355X node with the
fallback communicator (library-format messages all-gathered by
torch.distributed), every pool operation restated by oracle/pool.py.  The
expected migrants are recomputed from every rank's pre-exchange state.
"""
import math
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from oracle import pool as opool
from oracle.standin import StandInContext
from vrpms_amd import islands, runners, synth

M64 = (1 << 64) - 1


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _u64(t):
    return [int(x) & M64 for x in t.reshape(-1).tolist()]


def _inst():
    return synth.cvrp(12, 3, seed=5, slack=1.0)


def _snap(tours, keys):
    return tours.reshape(-1, tours.shape[-1]).tolist(), _u64(keys)


def _worker(rank, world, port, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        inst = _inst()
        ctx = StandInContext(inst)
        res = {}
        # SA chains: elites from the bests, migrants restart the worst chains
        r = runners.SARunner(ctx, inst.n, chains=6, seed=40 + rank, total_steps=60,
                             steps_per_epoch=10, durations=inst.durations)
        r.epoch()
        res["sa_src"], res["sa_dst"] = _snap(*r.src()), _snap(*r.dst())
        islands.exchange(r, E=3)
        res["sa_after"] = _snap(*r.dst())
        # GA islands: migrants take the worst slots, islands stay sorted
        g = runners.GARunner(ctx, inst.n, islands=2, pop=6, seed=70 + rank, gens_per_epoch=2)
        g.epoch()
        res["ga_src"] = _snap(*g.src())
        islands.exchange(g, E=3)
        res["ga_after"] = _snap(*g.dst())
        # the global best is identical on every rank
        res["gb"] = islands.global_best(r)

        # brute-force split: bf over [lo, hi) of 5! with key = (x * 7919) % 113
        def bf_fn(lo, hi):
            return min(((x * 7919) % 113, x) for x in range(lo, hi))
        res["bf"] = islands.bf_distributed(bf_fn, 5)
        # a fixed epoch count: every rank enters the same collectives
        r2 = runners.SARunner(ctx, inst.n, chains=4, seed=90 + rank, total_steps=40,
                              steps_per_epoch=5, durations=inst.durations)
        res["fixed"] = islands.run_fixed(r2, epochs=8, exchange_every=4, E=2)[0]
        res["fixed_best"] = islands.global_best(r2)
        q.put((rank, res))
    finally:
        dist.destroy_process_group()


def _expected(srcs, dsts, E, n, mode, groups=1):
    """oracle/pool.py: pack every rank's src, merge, inject into each dst."""
    msgs = b"".join(opool.island_pack(t, k, E, n) for t, k in srcs)
    mt, mk = opool.island_merge(msgs, len(srcs), E, n)
    return [opool.pool_inject(t, k, mode, mt, mk, groups) for t, k in dsts], mk


def test_island_exchange_world2_real_runners():
    mpc = mp.get_context("spawn")
    q = mpc.Queue()
    port = _free_port()
    procs = [mpc.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    out = dict(q.get(timeout=300) for _ in procs)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    n = _inst().n
    # SA: WORST injection of the global 3 best of both ranks' bests
    want, mk = _expected([out[r]["sa_src"] for r in (0, 1)], [out[r]["sa_dst"] for r in (0, 1)],
                         3, n, opool.INJECT_WORST)
    for r in (0, 1):
        assert [list(x) for x in out[r]["sa_after"][0]] == want[r][0]
        assert out[r]["sa_after"][1] == want[r][1]
    assert mk == sorted(mk)
    # GA: SORTED injection, both islands re-sorted
    want, _ = _expected([out[r]["ga_src"] for r in (0, 1)], [out[r]["ga_src"] for r in (0, 1)],
                        3, n, opool.INJECT_SORTED, groups=2)
    for r in (0, 1):
        assert [list(x) for x in out[r]["ga_after"][0]] == want[r][0]
        assert out[r]["ga_after"][1] == want[r][1]
        ks = out[r]["ga_after"][1]
        assert ks[:6] == sorted(ks[:6]) and ks[6:] == sorted(ks[6:])
    assert out[0]["gb"] == out[1]["gb"]
    assert out[0]["gb"][0] == min(min(out[r]["sa_after"][1] + out[r]["sa_src"][1]) for r in (0, 1))
    want_bf = min(((x * 7919) % 113, x) for x in range(math.factorial(5)))
    assert out[0]["bf"] == out[1]["bf"] == want_bf
    assert out[0]["fixed"] == out[1]["fixed"] == 2
    assert out[0]["fixed_best"] == out[1]["fixed_best"]


@pytest.mark.parametrize("n,world", [(5, 2), (7, 3), (10, 8)])
def test_bf_rank_ranges_partition(n, world):
    spans = [islands.bf_rank_range(n, r, world) for r in range(world)]
    assert spans[0][0] == 0 and spans[-1][1] == math.factorial(n)
    assert all(a[1] == b[0] for a, b in zip(spans, spans[1:]))


def test_merge_orders_as_uint64_then_rank_then_position():
    n, E = 2, 3
    a = opool.island_pack([[1, 2], [2, 1], [1, 2]], [5, M64, 3], E, n)   # M64 sorts last
    b = opool.island_pack([[2, 1], [1, 2], [2, 1]], [3, 7, 9], E, n)
    t, k = opool.island_merge(a + b, 2, E, n)
    assert k == [3, 3, 5]
    assert t == [[1, 2], [2, 1], [1, 2]]      # rank 0's 3 before rank 1's 3


def test_pool_inject_modes():
    tours = [[1, 2], [2, 1], [1, 2], [2, 1]]
    keys = [9, 4, 9, 1]
    t, k = opool.pool_inject(tours, keys, opool.INJECT_WORST, [[7, 7], [8, 8]], [2, 3])
    assert k == [2, 4, 3, 1]                  # the two 9s (lowest index first) replaced
    t, k = opool.pool_inject(tours, keys, opool.INJECT_BETTER, [[7, 7], [8, 8]], [2, 5])
    assert k == [2, 4, 9, 1] and t[0] == [7, 7]
    t, k = opool.pool_inject(tours, [1, 4, 2, 6], opool.INJECT_SORTED, [[7, 7], [8, 8]], [0, 3],
                             groups=2)
    assert k == [0, 1, 2, 3] and t[0] == [7, 7] and t[3] == [8, 8]


def test_run_fixed_single_rank_injects_locally():
    inst = _inst()
    ctx = StandInContext(inst)
    r = runners.SARunner(ctx, inst.n, chains=4, seed=3, total_steps=20, steps_per_epoch=5,
                         durations=inst.durations)
    n_ex, _ = islands.run_fixed(r, epochs=4, exchange_every=2, E=2)
    assert n_ex == 2 and r.step == 20
    keys = _u64(r.cur_key)
    assert all(k < M64 for k in keys)


def test_philox_tours_are_permutations():
    rows = [opool.philox_tour(13, 99, r, 2) for r in range(20)]
    assert all(sorted(t) == list(range(1, 14)) for t in rows)
    assert len({tuple(t) for t in rows}) == 20
    assert opool.philox_tour(1, 5, 0) == [1] and opool.philox_tour(0, 5, 0) == []
    assert np.all(np.array(opool.philox_tour(13, 99, 4, 2)) == np.array(rows[4]))


class _CommStandIn(StandInContext):
    """Stand-in with a library communicator that fails on `bad_rank`."""

    def __init__(self, inst, rank, bad_rank):
        super().__init__(inst)
        self.rank, self.bad_rank, self._world = rank, bad_rank, 0
        self.island_comm_group = None

    def set_island_timeout(self, s):
        self.timeout = s

    def island_unique_id(self):
        if self.bad_rank == "uid":
            raise RuntimeError("simulated ncclGetUniqueId failure")
        return bytes(128)

    def island_init(self, uid, rank, world):
        self.init_called = True
        if rank == self.bad_rank:
            raise RuntimeError("simulated ncclCommInitRank failure")
        self._world = world

    def island_world(self):
        return self._world


def _agree_worker(rank, world, port, bad_rank, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        ctx = _CommStandIn(_inst(), rank, bad_rank)
        try:
            islands.init_comm(ctx, timeout_s=5)
            q.put((rank, ("ok", ctx.island_comm_group, ctx.timeout)))
        except RuntimeError as e:
            q.put((rank, ("raised", ctx.island_comm_group, str(e),
                          getattr(ctx, "init_called", False))))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("bad_rank", [-1, 1, "uid"])
def test_init_comm_ranks_agree_on_the_exchange_path(bad_rank):
    """init_comm sets the communicator on every rank or on none: when one
    rank's vrpms_island_init fails, every rank raises (no rank is left to
    call ncclAllGather while another calls torch's all-gather).  "uid": rank
    0 cannot create the unique id -- it still enters the broadcast (with
    None), no rank calls island_init, every rank raises."""
    mpc = mp.get_context("spawn")
    q = mpc.Queue()
    port = _free_port()
    procs = [mpc.Process(target=_agree_worker, args=(r, 2, port, bad_rank, q)) for r in range(2)]
    for p in procs:
        p.start()
    out = dict(q.get(timeout=300) for _ in procs)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    if bad_rank == "uid":
        assert out[0][0] == out[1][0] == "raised"
        assert out[0][1] is None and out[1][1] is None
        assert "ncclGetUniqueId" in out[0][2] and "unique id" in out[1][2]
        assert not out[0][3] and not out[1][3]
    elif bad_rank < 0:
        assert out[0] == out[1] == ("ok", (None, 2), 5)
    else:
        assert out[0][0] == out[1][0] == "raised"
        assert out[0][1] is None and out[1][1] is None
        assert "simulated" in out[1][2]
