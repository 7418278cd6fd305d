"""world_size-2 gloo tests of the island exchange and the brute-force rank
split (the N > 1 path), on CPU tensors with stand-in runners."""
import math
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from vrpms_amd import islands


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


class FakeRunner:
    """Keys are sums of the tour (so different ranks hold different elites)."""

    def __init__(self, rank, n=6, members=5):
        g = torch.Generator().manual_seed(100 + rank)
        self.n = n
        self.tours = torch.stack([torch.randperm(n, generator=g) + 1 for _ in range(members)]).to(torch.int16)
        self.keys = (torch.arange(members, dtype=torch.int64) * 10 + rank * 3 + 1)
        self.injected = None

    def elites(self, E):
        order = torch.argsort(self.keys, stable=True)[:E]
        return self.tours[order].clone(), self.keys[order].clone()

    def inject(self, tours, keys):
        self.injected = (tours.clone(), keys.clone())

    def epoch(self):
        pass

    def best(self):
        i = int(torch.argmin(self.keys))
        return int(self.keys[i]), self.tours[i]


def _worker(rank, world, port, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        r = FakeRunner(rank)
        bk = islands.exchange(r, E=3)
        res = {"keys": bk.tolist(), "inj": r.injected[1].tolist(),
               "tours": r.injected[0].tolist()}
        # brute-force split: bf over [lo, hi) of 5! with key = (rank * 7919) % 113
        def bf_fn(lo, hi):
            return min(((x * 7919) % 113, x) for x in range(lo, hi))
        res["bf"] = islands.bf_distributed(bf_fn, 5)
        k, t = islands.global_best(int(r.keys.min()) + 1000 * rank, r.tours[0].tolist(), r.n)
        res["gb"] = (k, t)
        q.put((rank, res))
    finally:
        dist.destroy_process_group()


def test_exchange_and_bf_split_world2():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    out = dict(q.get(timeout=120) for _ in procs)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    # rank 0 keys 1, 11, 21 ... ; rank 1 keys 4, 14, 24 -> global best three: 1, 4, 11
    assert out[0]["keys"] == [1, 4, 11] == out[1]["keys"]
    assert out[0]["tours"] == out[1]["tours"]          # identical merge on every rank
    want = min(((x * 7919) % 113, x) for x in range(math.factorial(5)))
    assert out[0]["bf"] == out[1]["bf"] == want
    assert out[0]["gb"] == out[1]["gb"] and out[0]["gb"][0] == 1


@pytest.mark.parametrize("n,world", [(5, 2), (7, 3), (10, 8)])
def test_bf_rank_ranges_partition(n, world):
    spans = [islands.bf_rank_range(n, r, world) for r in range(world)]
    assert spans[0][0] == 0 and spans[-1][1] == math.factorial(n)
    assert all(a[1] == b[0] for a, b in zip(spans, spans[1:]))


def test_select_global_orders_as_uint64():
    keys = torch.tensor([5, -1, 3, 3], dtype=torch.int64)   # -1 is UINT64_MAX
    tours = torch.arange(8, dtype=torch.int16).reshape(4, 2)
    t, k = islands.select_global(tours, keys, 3)
    assert k.tolist() == [3, 3, 5]
    assert t[:, 0].tolist() == [4, 6, 0]


class CountingRunner(FakeRunner):
    """Epochs lower one member's key, so migrations carry changing elites."""

    def __init__(self, rank):
        super().__init__(rank)
        self.epochs = 0
        self.log = []

    def epoch(self):
        self.epochs += 1
        self.keys[self.epochs % self.keys.shape[0]] -= 1

    def inject(self, tours, keys):
        super().inject(tours, keys)
        self.log.append(keys.tolist())


def _fixed_worker(rank, world, port, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        r = CountingRunner(rank)
        n_ex, t_ex = islands.run_fixed(r, epochs=12, exchange_every=4, E=2)
        q.put((rank, {"n_ex": n_ex, "epochs": r.epochs, "log": r.log, "t_ex": t_ex}))
    finally:
        dist.destroy_process_group()


def test_run_fixed_world2_same_collectives_and_merges():
    """The bench's island leg (cfg 4) at N > 1: a fixed epoch count, so every
    rank enters the same number of all-gathers and injects identical elites."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_fixed_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    out = dict(q.get(timeout=120) for _ in procs)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert out[0]["n_ex"] == out[1]["n_ex"] == 3
    assert out[0]["epochs"] == out[1]["epochs"] == 12
    assert out[0]["log"] == out[1]["log"] and len(out[0]["log"]) == 3
    assert all(k == sorted(k) for k in out[0]["log"])


def test_run_fixed_single_rank_injects_locally():
    r = CountingRunner(0)
    n_ex, _ = islands.run_fixed(r, epochs=10, exchange_every=5, E=2)
    assert n_ex == 2 and len(r.log) == 2 and r.epochs == 10
