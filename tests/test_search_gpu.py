"""GPU parity of the search kernels against the CPU replay (oracle/search.py).

Small instances: the whole trajectory must match exactly (tours, keys,
best-so-far, pheromone matrices), because every random choice is a Philox
word both sides compute and every cost is integer.  Larger instances: the
invariants (tours stay permutations, reported keys == vrpms_eval of the
reported tours, search improves on its start).
"""
import math

import numpy as np
import pytest

from oracle import search, spec
from vrpms_amd import synth

pytestmark = pytest.mark.gpu


def torch_():
    import torch
    return torch


def load(ctx, inst, objective=0):
    from vrpms_amd.core import CVRP, TSP
    if inst.problem == "tsp":
        ctx.set_instance(TSP, inst.durations, start_times=inst.start_times, objective=objective)
    else:
        ctx.set_instance(CVRP, inst.durations, inst.demand, inst.capacities, inst.start_times,
                         objective=objective)


def scorer(inst, objective=0):
    return search.Scorer(inst.durations, inst.demand, inst.capacities, inst.start_times,
                         inst.problem, objective)


def u64(t):
    return [int(x) for x in t.cpu().numpy().view(np.uint64).reshape(-1)]


SMALL = [
    ("cvrp", lambda: synth.cvrp(12, 3, seed=1, slack=0.95)),
    ("tsp", lambda: synth.Instance("tsp11", synth.tsp20(2).durations[:, :11, :11], None, None,
                                   np.array([0]), "tsp")),
    ("td", lambda: synth.td_cvrp(10, 2, seed=4)),
    ("tsp_asym", lambda: synth.Instance(
        "tsp10a", np.array([np.where(np.eye(10, dtype=bool), 0, np.random.default_rng(8).integers(
            3, 320, size=(10, 10)))]), None, None, np.array([0]), "tsp")),
]


@pytest.mark.parametrize("name,maker", SMALL, ids=[s[0] for s in SMALL])
def test_sa_trajectory_matches_oracle(ctx, name, maker):
    torch = torch_()
    inst = maker()
    load(ctx, inst)
    chains, n = 3, inst.n
    P = synth.random_perms(chains, n, seed=7).astype(np.int16)
    cur = torch.from_numpy(P).to(ctx.dev)
    best = cur.clone()
    ck = torch.empty(chains, dtype=torch.int64, device=ctx.dev)
    bk = torch.full((chains,), -1, dtype=torch.int64, device=ctx.dev)   # UINT64_MAX
    seed, inv_t0, inv_alpha = 12345, 1.0 / 200.0, 1.0 / 0.97
    ctx.sa_run(cur, ck, best, bk, steps=20, inv_t0=inv_t0, inv_alpha=inv_alpha, seed=seed, step0=0)
    ref = search.sa_run(scorer(inst), P.tolist(), P.tolist(), [2**64 - 1] * chains, seed, 0, 20,
                        inv_t0, inv_alpha)
    assert cur.cpu().numpy().tolist() == ref[0]
    assert u64(ck) == ref[1]
    assert best.cpu().numpy().tolist() == ref[2]
    assert u64(bk) == ref[3]
    # a second call continues the same streams (step0 = 20)
    inv_t1 = np.float32(inv_t0)
    for _ in range(20):
        inv_t1 = np.float32(inv_t1 * np.float32(inv_alpha))
    ctx.sa_run(cur, ck, best, bk, steps=10, inv_t0=float(inv_t1), inv_alpha=inv_alpha, seed=seed,
               step0=20)
    ref2 = search.sa_run(scorer(inst), ref[0], ref[2], ref[3], seed, 20, 10, float(inv_t1),
                         inv_alpha)
    assert cur.cpu().numpy().tolist() == ref2[0]
    assert u64(bk) == ref2[3]


@pytest.mark.parametrize("split_mode", [0, 2], ids=["branchfree", "branchy"])
@pytest.mark.parametrize("n_cust", [1, 2, 3, 5, 8, 13])
def test_sa_split_paths_match_oracle(ctx, split_mode, n_cust):
    """CVRP SA through the packed branch-free kernel (mode 0) and the generic
    split (mode 2): identical trajectories, ragged and tiny tours included,
    tight capacity so some candidates leave customers unvisited."""
    torch = torch_()
    inst = synth.cvrp(n_cust, 2, seed=n_cust, slack=0.8)
    load(ctx, inst)
    ctx.set_split_mode(split_mode)
    try:
        chains = 5
        P = synth.random_perms(chains, n_cust, seed=n_cust).astype(np.int16)
        cur = torch.from_numpy(P).to(ctx.dev)
        best = cur.clone()
        ck = torch.empty(chains, dtype=torch.int64, device=ctx.dev)
        bk = torch.full((chains,), -1, dtype=torch.int64, device=ctx.dev)
        ctx.sa_run(cur, ck, best, bk, steps=12, inv_t0=1 / 40.0, inv_alpha=1 / 0.97, seed=77,
                   step0=5)
        ref = search.sa_run(scorer(inst), P.tolist(), P.tolist(), [2**64 - 1] * chains, 77, 5,
                            12, 1 / 40.0, 1 / 0.97)
    finally:
        ctx.set_split_mode(0)
    assert cur.cpu().numpy().tolist() == ref[0]
    assert u64(ck) == ref[1]
    assert best.cpu().numpy().tolist() == ref[2]
    assert u64(bk) == ref[3]


def test_sa_cvrp100_matches_c_restatement(ctx, coracle):
    """Full-size parity: 32 chains x 150 steps of the GPU SA on CVRP-100 vs the
    C/OpenMP restatement driven by the same Philox streams."""
    torch = torch_()
    inst = synth.cvrp(100, 8, seed=0)
    load(ctx, inst)
    chains, n = 32, inst.n
    P = synth.random_perms(chains, n, seed=21).astype(np.int16)
    cur = torch.from_numpy(P).to(ctx.dev)
    best = cur.clone()
    ck = torch.empty(chains, dtype=torch.int64, device=ctx.dev)
    bk = torch.full((chains,), -1, dtype=torch.int64, device=ctx.dev)
    ctx.sa_run(cur, ck, best, bk, steps=150, inv_t0=1 / 80.0, inv_alpha=1 / 0.995, seed=5,
               step0=3)
    ccur, cbest = P.view(np.uint16).copy(), P.view(np.uint16).copy()
    cbk = np.full(chains, 2**64 - 1, dtype=np.uint64)
    cck = coracle.sa_run(inst.durations, ccur, cbest, cbk, 150, 1 / 80.0, 1 / 0.995, 5, 3,
                         inst.demand, inst.capacities, inst.start_times)
    assert (cur.cpu().numpy().view(np.uint16) == ccur).all()
    assert u64(ck) == [int(x) for x in cck]
    assert u64(bk) == [int(x) for x in cbk]
    assert (best.cpu().numpy().view(np.uint16) == cbest).all()


L2_CASES = [
    # BASELINE cfg 3: 24 x 201^2 u16 = 1.94 MB (L2 tier, hour-indexed clock)
    ("tdvrp200_h24", lambda: synth.td_cvrp(200, 16, seed=0)),
    # BASELINE cfg 4: X-style CVRP-1000, 1001^2 u16 = 2.0 MB (L2 tier)
    ("x1000", lambda: synth.x_style(1000, seed=0)),
]


@pytest.mark.parametrize("name,maker", L2_CASES, ids=[c[0] for c in L2_CASES])
def test_sa_l2_tier_matches_c_restatement(ctx, coracle, name, maker):
    """sa_kernel with the matrix L2-resident (mat_lds = 0) at the sizes
    configs 3 and 4 run: 16 chains x 30 steps, tours and keys bit-equal to
    the C restatement driven by the same Philox streams."""
    torch = torch_()
    inst = maker()
    load(ctx, inst)
    chains, n = 16, inst.n
    P = synth.random_perms(chains, n, seed=31, dtype=np.uint16).astype(np.int16)
    cur = torch.from_numpy(P).to(ctx.dev)
    best = cur.clone()
    ck = torch.empty(chains, dtype=torch.int64, device=ctx.dev)
    bk = torch.full((chains,), -1, dtype=torch.int64, device=ctx.dev)
    ctx.sa_run(cur, ck, best, bk, steps=30, inv_t0=1 / 100.0, inv_alpha=1 / 0.99, seed=17,
               step0=40)
    ccur, cbest = P.view(np.uint16).copy(), P.view(np.uint16).copy()
    cbk = np.full(chains, 2**64 - 1, dtype=np.uint64)
    cck = coracle.sa_run(inst.durations, ccur, cbest, cbk, 30, 1 / 100.0, 1 / 0.99, 17, 40,
                         inst.demand, inst.capacities, inst.start_times)
    assert (cur.cpu().numpy().view(np.uint16) == ccur).all()
    assert u64(ck) == [int(x) for x in cck]
    assert u64(bk) == [int(x) for x in cbk]
    assert (best.cpu().numpy().view(np.uint16) == cbest).all()


def test_sa_l2_tier_small_td_matches_python_oracle(ctx):
    """A small hour-indexed instance whose matrix (24 x 61^2 u16 = 179 KB)
    still exceeds the 64 KB LDS budget: the L2 branch against the pure-Python
    replay."""
    torch = torch_()
    inst = synth.td_cvrp(60, 5, seed=12)
    load(ctx, inst)
    chains, n = 3, inst.n
    P = synth.random_perms(chains, n, seed=4).astype(np.int16)
    cur = torch.from_numpy(P).to(ctx.dev)
    best = cur.clone()
    ck = torch.empty(chains, dtype=torch.int64, device=ctx.dev)
    bk = torch.full((chains,), -1, dtype=torch.int64, device=ctx.dev)
    ctx.sa_run(cur, ck, best, bk, steps=8, inv_t0=1 / 90.0, inv_alpha=1 / 0.98, seed=3, step0=0)
    ref = search.sa_run(scorer(inst), P.tolist(), P.tolist(), [2**64 - 1] * chains, 3, 0, 8,
                        1 / 90.0, 1 / 0.98)
    assert cur.cpu().numpy().tolist() == ref[0]
    assert u64(ck) == ref[1]
    assert best.cpu().numpy().tolist() == ref[2]
    assert u64(bk) == ref[3]


def test_ga_cvrp100_matches_oracle(ctx):
    """GA at the cfg-2 size (4 islands x 64, 5 generations): every
    population and key equal to the Python replay."""
    torch = torch_()
    inst = synth.cvrp(100, 8, seed=0)
    load(ctx, inst)
    islands, pop, n = 4, 64, inst.n
    P = synth.random_perms(islands * pop, n, seed=13).astype(np.int16)
    dpop = torch.from_numpy(P.reshape(islands, pop, n).copy()).to(ctx.dev)
    keys = ctx.eval(dpop.view(islands * pop, n)).view(islands, pop)
    sc = scorer(inst)
    rpop = [[list(r) for r in P.reshape(islands, pop, n)[i]] for i in range(islands)]
    rkeys = [[sc(t) for t in rpop[i]] for i in range(islands)]
    seed, pmut = 2024, 0.25
    pm = min(int(round(pmut * 2**32)), 2**32 - 1)
    for g in range(5):
        rpop, rkeys = search.ga_generation(sc, rpop, rkeys, seed, 10 + g, pm)
    ctx.ga_generation(dpop, keys, generations=5, pmut=pmut, seed=seed, gen0=10)
    assert dpop.cpu().numpy().tolist() == rpop
    assert u64(keys) == [k for ks in rkeys for k in ks]


def test_tsp_batch_tsp50_matches_c_restatement(ctx, coracle):
    """Config-5 kernel at its real size (N = 50) on 128 requests x 300 steps:
    best tours and keys equal the C restatement (full re-evaluation)."""
    torch = torch_()
    rng = np.random.default_rng(50)
    R = 128
    mats = np.stack([synth.random_symmetric(50, rng) for _ in range(R)])
    M = torch.tensor(mats, dtype=torch.int32, device=ctx.dev)
    tours, keys = ctx.tsp_batch_sa(M, steps=300, inv_t0=1 / 80.0, inv_alpha=1 / 0.99, seed=8)
    rt, rk = coracle.tsp_batch_sa(mats, 300, 1 / 80.0, 1 / 0.99, 8)
    assert (tours.cpu().numpy().view(np.uint16) == rt).all()
    assert u64(keys) == [int(k) for k in rk]


@pytest.mark.parametrize("N", [64, 65, 90])
def test_tsp_batch_long_tours_match_c_restatement(ctx, coracle, N):
    """Tours of n = N - 1 >= 63 customers: an accepted move at n < 64 keeps the
    moved tour in registers (one position per lane), longer tours take the
    loop over positions -- both sides of that boundary equal the C
    restatement on 16 requests x 200 steps."""
    torch = torch_()
    rng = np.random.default_rng(N)
    mats = np.stack([synth.random_symmetric(N, rng) for _ in range(16)])
    M = torch.tensor(mats, dtype=torch.int32, device=ctx.dev)
    tours, keys = ctx.tsp_batch_sa(M, steps=200, inv_t0=1 / 80.0, inv_alpha=1 / 0.99, seed=3)
    rt, rk = coracle.tsp_batch_sa(mats, 200, 1 / 80.0, 1 / 0.99, 3)
    assert (tours.cpu().numpy().view(np.uint16) == rt).all()
    assert u64(keys) == [int(k) for k in rk]


@pytest.mark.parametrize("kind", ["symmetric", "asymmetric", "large"])
def test_tsp_batch_matches_oracle(ctx, kind):
    """Config-5 throughput kernel: O(1)-delta SA == full-evaluation replay.
    "large": entries >= 2^26 / N take the 64-bit (key, lane) argmin instead
    of the one-dword (duration << 6 | lane) one."""
    torch = torch_()
    rng = np.random.default_rng(4)
    mats = []
    for r in range(3):
        if kind == "symmetric":
            mats.append(synth.random_symmetric(9, rng))
        else:
            hi = 320 if kind == "asymmetric" else 12_000_000
            m = rng.integers(3 if hi == 320 else 8_000_000, hi, size=(9, 9))
            np.fill_diagonal(m, 0)
            mats.append(m)
    M = torch.tensor(np.array(mats), dtype=torch.int32, device=ctx.dev)
    tours, keys = ctx.tsp_batch_sa(M, steps=25, inv_t0=1 / 60.0, inv_alpha=1 / 0.97, seed=31)
    rt, rk = search.tsp_batch_sa(mats, 25, 1 / 60.0, 1 / 0.97, 31)
    assert tours.cpu().numpy().tolist() == rt
    assert u64(keys) == rk


def test_tsp_batch_tsp50_invariants(ctx):
    torch = torch_()
    rng = np.random.default_rng(0)
    R = 300
    mats = np.stack([synth.random_symmetric(50, rng) for _ in range(R)])
    M = torch.tensor(mats, dtype=torch.int32, device=ctx.dev)
    tours, keys = ctx.tsp_batch_sa(M, steps=400, inv_t0=1 / 80.0, inv_alpha=1 / 0.99, seed=2)
    T = tours.cpu().numpy()
    K = u64(keys)
    for r in range(0, R, 37):
        assert sorted(T[r]) == list(range(1, 50))
        assert K[r] == spec.tsp_key(spec.eval_tsp(mats[r], T[r]))
    rand = np.mean([spec.eval_tsp(mats[r], rng.permutation(np.arange(1, 50))) for r in range(20)])
    assert np.mean([k >> 28 for k in K]) < 0.5 * rand


def test_sa_large_invariants(ctx):
    torch = torch_()
    inst = synth.cvrp(100, 8, seed=0)
    load(ctx, inst)
    chains, n = 64, inst.n
    P = synth.random_perms(chains, n, seed=3).astype(np.int16)
    cur = torch.from_numpy(P).to(ctx.dev)
    best = cur.clone()
    ck = torch.empty(chains, dtype=torch.int64, device=ctx.dev)
    bk = torch.full((chains,), -1, dtype=torch.int64, device=ctx.dev)
    start = ctx.eval(cur, with_parts=False)
    ctx.sa_run(cur, ck, best, bk, steps=300, inv_t0=1 / 50.0, inv_alpha=1 / 0.99, seed=1, step0=0)
    B = best.cpu().numpy()
    assert all(sorted(r) == list(range(1, n + 1)) for r in B)
    assert u64(ctx.eval(best)) == u64(bk)
    assert u64(ctx.eval(cur)) == u64(ck)
    assert np.mean(u64(bk)) < 0.6 * np.mean(u64(start))


@pytest.mark.parametrize("name,maker", SMALL[:2], ids=[s[0] for s in SMALL[:2]])
def test_ga_generations_match_oracle(ctx, name, maker):
    torch = torch_()
    inst = maker()
    load(ctx, inst)
    islands, pop, n = 2, 16, inst.n
    P = synth.random_perms(islands * pop, n, seed=5).astype(np.int16)
    dpop = torch.from_numpy(P.reshape(islands, pop, n).copy()).to(ctx.dev)
    keys = ctx.eval(dpop.view(islands * pop, n)).view(islands, pop)
    sc = scorer(inst)
    rpop = [[list(r) for r in P.reshape(islands, pop, n)[i]] for i in range(islands)]
    rkeys = [[sc(t) for t in rpop[i]] for i in range(islands)]
    assert u64(keys) == [k for ks in rkeys for k in ks]
    seed, pmut = 99, 0.3
    pm = min(int(round(pmut * 2**32)), 2**32 - 1)
    for g in range(3):
        rpop, rkeys = search.ga_generation(sc, rpop, rkeys, seed, g, pm)
    ctx.ga_generation(dpop, keys, generations=3, pmut=pmut, seed=seed, gen0=0)
    assert dpop.cpu().numpy().tolist() == rpop
    assert u64(keys) == [k for ks in rkeys for k in ks]


def test_ga_large_invariants(ctx):
    torch = torch_()
    inst = synth.cvrp(100, 8, seed=0)
    load(ctx, inst)
    islands, pop, n = 4, 128, inst.n
    P = synth.random_perms(islands * pop, n, seed=8).astype(np.int16)
    dpop = torch.from_numpy(P.reshape(islands, pop, n).copy()).to(ctx.dev)
    keys = ctx.eval(dpop.view(-1, n)).view(islands, pop)
    k0 = min(u64(keys))
    ctx.ga_generation(dpop, keys, generations=30, pmut=0.2, seed=3, gen0=0)
    flat = dpop.view(-1, n)
    assert all(sorted(r) == list(range(1, n + 1)) for r in flat.cpu().numpy())
    assert u64(ctx.eval(flat)) == u64(keys)
    assert min(u64(keys)) < k0
    ks = np.array(u64(keys), dtype=np.uint64).reshape(islands, pop)
    assert (np.diff(ks.astype(np.float64), axis=1) >= 0).all()     # survivors sorted


@pytest.mark.parametrize("name,maker", SMALL[:2], ids=[s[0] for s in SMALL[:2]])
def test_aco_iterations_match_oracle(ctx, name, maker):
    inst = maker()
    load(ctx, inst)
    colonies, ants, tau0 = 2, 8, 1 << 20
    tau, eta = ctx.aco_init(colonies, tau0)
    ref_eta = search.aco_eta(inst.durations[0])
    assert (eta.cpu().numpy().astype(np.int64) & 0xFFFFFFFF).tolist() == ref_eta.tolist()
    rtau = [np.full((inst.N, inst.N), tau0, dtype=np.int64) for _ in range(colonies)]
    sc = scorer(inst)
    for it in range(3):
        tours, keys, ib = ctx.aco_iteration(tau, eta, ants, seed=7, it=it, evap_shift=3,
                                            tau_min=1 << 10, tau_max=1 << 30)
        rt, rk, rib = search.aco_iteration(sc, rtau, ref_eta, ants, inst.n, 7, it, 3, 1 << 10,
                                           1 << 30)
        assert tours.cpu().numpy().tolist() == rt
        assert u64(keys) == [k for ks in rk for k in ks]
        assert [(a & (2**64 - 1), b) for a, b in ib.cpu().tolist()] == rib
        got_tau = tau.cpu().numpy().astype(np.int64) & 0xFFFFFFFF
        assert all((got_tau[c] == rtau[c]).all() for c in range(colonies))


ACO_SIZES = [
    # register path, 1 / 2 / 4 chunks of 64 nodes per lane (words layout for CVRP), and the
    # LDS path past 256 nodes
    ("tsp60", lambda: synth.Instance("tsp60", synth.random_symmetric(60, np.random.default_rng(3))[None],
                                     None, None, np.array([0]), "tsp")),
    ("cvrp100", lambda: synth.cvrp(100, 8, seed=0)),
    ("cvrp150", lambda: synth.cvrp(150, 12, seed=2)),
    ("cvrp300", lambda: synth.cvrp(300, 24, seed=5)),
]


@pytest.mark.parametrize("name,maker", ACO_SIZES, ids=[s[0] for s in ACO_SIZES])
def test_aco_iterations_match_oracle_at_size(ctx, name, maker):
    inst = maker()
    load(ctx, inst)
    colonies, ants, tau0 = 2, 8, 1 << 20
    tau, eta = ctx.aco_init(colonies, tau0)
    ref_eta = search.aco_eta(inst.durations[0])
    rtau = [np.full((inst.N, inst.N), tau0, dtype=np.int64) for _ in range(colonies)]
    sc = scorer(inst)
    for it in range(2):
        tours, keys, ib = ctx.aco_iteration(tau, eta, ants, seed=11, it=it, evap_shift=3,
                                            tau_min=1 << 10, tau_max=1 << 30)
        rt, rk, rib = search.aco_iteration(sc, rtau, ref_eta, ants, inst.n, 11, it, 3, 1 << 10,
                                           1 << 30)
        assert tours.cpu().numpy().tolist() == rt
        assert u64(keys) == [k for ks in rk for k in ks]
        assert [(a & (2**64 - 1), b) for a, b in ib.cpu().tolist()] == rib
        got_tau = tau.cpu().numpy().astype(np.int64) & 0xFFFFFFFF
        assert all((got_tau[c] == rtau[c]).all() for c in range(colonies))


ACO_STAGED = [
    # (name, instance, colonies, ants): ants not a multiple of the 16-ant
    # workgroup (16 + 16 + 8), one ant per colony, the largest N whose
    # weights fit the LDS (140 x 140 x 8 B + 16 tour buffers; rows padded to
    # an even stride), the TSP layout
    ("cvrp100_40ants", lambda: synth.cvrp(100, 8, seed=0), 3, 40),
    ("cvrp60_1ant", lambda: synth.cvrp(60, 5, seed=4), 5, 1),
    ("cvrp139_17ants", lambda: synth.cvrp(139, 10, seed=6), 2, 17),
    ("cvrp140_past_lds", lambda: synth.cvrp(140, 10, seed=6), 2, 17),   # N = 141: the L2 path
    ("tsp40_64ants", lambda: synth.Instance("tsp40", synth.random_symmetric(
        40, np.random.default_rng(8))[None], None, None, np.array([0]), "tsp"), 2, 64),
]


@pytest.mark.parametrize("name,maker,colonies,ants", ACO_STAGED, ids=[s[0] for s in ACO_STAGED])
def test_aco_lds_staged_construct_matches_l2_path_and_oracle(ctx, name, maker, colonies, ants):
    """Round 6: the LDS-staged construction (VRPMS_OPT_ACO_CONSTRUCT auto)
    gives the same tours, keys, iteration bests and tau as the L2 path
    (option 2) and as oracle/search.py."""
    inst = maker()
    load(ctx, inst)
    tau0 = 1 << 20
    runs = []
    for mode in (0, 2):
        ctx.set_aco_construct(mode)
        try:
            tau, eta = ctx.aco_init(colonies, tau0)
            out = []
            for it in range(2):
                tours, keys, ib = ctx.aco_iteration(tau, eta, ants, seed=13, it=it, evap_shift=3,
                                                    tau_min=1 << 10, tau_max=1 << 30)
                out.append((tours.cpu().numpy().tolist(), u64(keys), ib.cpu().tolist(),
                            (tau.cpu().numpy().astype(np.int64) & 0xFFFFFFFF).tolist()))
            runs.append(out)
        finally:
            ctx.set_aco_construct(0)
    assert runs[0] == runs[1]
    ref_eta = search.aco_eta(inst.durations[0])
    rtau = [np.full((inst.N, inst.N), tau0, dtype=np.int64) for _ in range(colonies)]
    sc = scorer(inst)
    for it in range(2):
        rt, rk, rib = search.aco_iteration(sc, rtau, ref_eta, ants, inst.n, 13, it, 3, 1 << 10,
                                           1 << 30)
        assert runs[0][it][0] == rt
        assert runs[0][it][1] == [k for ks in rk for k in ks]


@pytest.mark.parametrize("name,maker", SMALL, ids=[s[0] for s in SMALL])
def test_bf_matches_oracle(ctx, name, maker):
    inst = maker()
    load(ctx, inst)
    n = 7
    sub = synth.Instance(inst.name, inst.durations[:, : n + 1, : n + 1],
                         None if inst.demand is None else inst.demand[: n + 1],
                         inst.capacities, inst.start_times, inst.problem)
    load(ctx, sub)
    best = ctx.bf_run(n, 0, math.factorial(n))
    assert best == search.bf(scorer(sub), n)
    # disjoint rank ranges (the multi-GPU split) reduce to the same optimum
    parts = [ctx.bf_run(n, a, b) for a, b in [(0, 1000), (1000, 3333), (3333, 5040)]]
    assert min(parts) == best
    # the reported rank decodes to a tour with the reported key
    tour = search.unrank(best[1], n)
    assert scorer(sub)(tour) == best[0]


@pytest.mark.parametrize("problem", ["cvrp", "tsp"])
def test_bf_n11_matches_c_restatement(ctx, coracle, problem):
    """The largest brute force the C restatement finishes in about a second
    (11! = 39.9 M tours): the full range and a ragged sub-range."""
    import math
    from vrpms_amd.core import CVRP, TSP
    if problem == "cvrp":
        inst = synth.cvrp(11, 3, seed=0)
        ctx.set_instance(CVRP, inst.durations, inst.demand, inst.capacities, inst.start_times)
        kw = dict(demand=inst.demand, capacities=inst.capacities, start_times=inst.start_times)
    else:
        D = synth.tsp20(5).durations[:, :12, :12]
        inst = synth.Instance("t11", D, None, None, np.array([0]), "tsp")
        ctx.set_instance(TSP, inst.durations, start_times=inst.start_times)
        kw = dict(start_times=inst.start_times, problem=0)
    full = math.factorial(11)
    assert ctx.bf_run(11, 0, full) == coracle.bf(inst.durations, 11, 0, full, **kw)
    assert ctx.bf_run(11, 12345, 9876543) == coracle.bf(inst.durations, 11, 12345, 9876543, **kw)


def test_bf_n10_optimum_le_every_sampled_tour(ctx, coracle):
    inst = synth.cvrp(10, 3, seed=9)
    load(ctx, inst)
    k, r = ctx.bf_run(10, 0, math.factorial(10))
    P = synth.random_perms(20000, 10, seed=1)
    keys = coracle.eval_batch(inst.durations, P, inst.demand, inst.capacities, inst.start_times)[0]
    assert k <= int(keys.min())
    assert scorer(inst)(search.unrank(r, 10)) == k


GA_FUSED_CASES = [
    # (n, K, slack, islands, pop, gens, pmut): ragged tours, tight fleets
    # (exact re-walks), odd population sizes, the cfg-2 size, and a large
    # island of a small instance
    (100, 8, 1.1, 3, 64, 6, 0.3),
    (97, 7, 1.03, 2, 50, 5, 0.5),
    (30, 3, 0.8, 5, 33, 7, 0.9),
    (1, 1, 1.0, 2, 4, 3, 0.5),
    (2, 2, 1.0, 2, 6, 4, 0.5),
    (19, 2, 1.0, 2, 1000, 3, 0.2),
    # three 64-position slots per lane (the span bitmask's widest case that
    # fits the packed matrix in LDS)
    (130, 10, 1.05, 2, 32, 4, 0.5),
]


@pytest.mark.parametrize("n,K,slack,islands,pop,gens,pmut", GA_FUSED_CASES)
def test_ga_fused_equals_three_kernel_path(ctx, n, K, slack, islands, pop, gens, pmut):
    """The fused one-workgroup-per-island GA (ga_fused.hip) and the
    breed / score / select launches produce identical populations and keys."""
    torch = torch_()
    inst = synth.cvrp(n, K, seed=n + pop, slack=slack)
    load(ctx, inst)
    P = synth.random_perms(islands * pop, n, seed=pop).astype(np.int16)
    out = []
    for mode in (0, 2):
        ctx.set_ga_fused(mode)
        try:
            dpop = torch.from_numpy(P.reshape(islands, pop, n).copy()).to(ctx.dev)
            keys = ctx.eval(dpop.view(islands * pop, n)).view(islands, pop)
            ctx.ga_generation(dpop, keys, generations=gens, pmut=pmut, seed=7 + n, gen0=3)
            out.append((dpop.cpu().numpy(), u64(keys)))
        finally:
            ctx.set_ga_fused(0)
    assert (out[0][0] == out[1][0]).all()
    assert out[0][1] == out[1][1]
    flat = out[0][0].reshape(-1, n)
    assert all(sorted(r) == list(range(1, n + 1)) for r in flat[:: max(1, len(flat) // 50)])


def test_ga_fused_small_matches_python_oracle(ctx):
    """Fused kernel vs the pure-Python GA replay, several generations."""
    torch = torch_()
    inst = synth.cvrp(13, 3, seed=2, slack=0.9)
    load(ctx, inst)
    islands, pop, n = 3, 10, inst.n
    P = synth.random_perms(islands * pop, n, seed=4).astype(np.int16)
    dpop = torch.from_numpy(P.reshape(islands, pop, n).copy()).to(ctx.dev)
    keys = ctx.eval(dpop.view(-1, n)).view(islands, pop)
    sc = scorer(inst)
    rpop = [[list(r) for r in P.reshape(islands, pop, n)[i]] for i in range(islands)]
    rkeys = [[sc(t) for t in rpop[i]] for i in range(islands)]
    pm = min(int(round(0.6 * 2**32)), 2**32 - 1)
    for g in range(6):
        rpop, rkeys = search.ga_generation(sc, rpop, rkeys, 55, g, pm)
    ctx.ga_generation(dpop, keys, generations=6, pmut=0.6, seed=55, gen0=0)
    assert dpop.cpu().numpy().tolist() == rpop
    assert u64(keys) == [k for ks in rkeys for k in ks]


# --- round 3: the product shapes the front-end and the bench actually run ---

def test_ga_fused_pop256_cfg2_equals_three_kernel_and_oracle(ctx):
    """The front-end default population (randomPermutationCount -> 256,
    solver.py) at CVRP-100 is the largest island the fused kernel keeps in
    LDS: 4 islands x 3 generations fused == three-launch, and the first 2
    generations == the Python replay (oracle/search.py ga_generation).
    Reference slot: api/vrp/ga/index.py:48-53."""
    torch = torch_()
    inst = synth.cvrp(100, 8, seed=0)
    load(ctx, inst)
    islands, pop, n = 4, 256, inst.n
    P = synth.random_perms(islands * pop, n, seed=256).astype(np.int16)
    seed, pmut = 4242, 0.2
    out = []
    for mode, gens in ((0, 3), (2, 3), (0, 2)):
        ctx.set_ga_fused(mode)
        try:
            dpop = torch.from_numpy(P.reshape(islands, pop, n).copy()).to(ctx.dev)
            keys = ctx.eval(dpop.view(islands * pop, n)).view(islands, pop)
            ctx.ga_generation(dpop, keys, generations=gens, pmut=pmut, seed=seed, gen0=1)
            out.append((dpop.cpu().numpy(), u64(keys)))
        finally:
            ctx.set_ga_fused(0)
    assert (out[0][0] == out[1][0]).all()
    assert out[0][1] == out[1][1]
    sc = scorer(inst)
    rpop = [[list(r) for r in P.reshape(islands, pop, n)[i]] for i in range(islands)]
    rkeys = [[sc(t) for t in rpop[i]] for i in range(islands)]
    pm = min(int(round(pmut * 2**32)), 2**32 - 1)
    for g in range(2):
        rpop, rkeys = search.ga_generation(sc, rpop, rkeys, seed, 1 + g, pm)
    assert out[2][0].tolist() == rpop
    assert out[2][1] == [k for ks in rkeys for k in ks]


@pytest.mark.parametrize("how", ["zero_demands", "split_mode_3"])
def test_ga_fused_without_carry_form_matches_three_kernel_and_oracle(ctx, how):
    """The fused GA's scoring walk takes the carry form of the split step only
    when every demand is >= 1 (ga_fused.hip, template CY): an instance with
    zero-demand customers, and VRPMS_OPT_SPLIT_MODE = 3 on an ordinary one,
    run the other instantiation -- same populations and keys as the
    three-launch path and the Python replay (oracle/search.py)."""
    torch = torch_()
    inst = synth.cvrp(60, 5, seed=21, slack=1.05)
    if how == "zero_demands":
        dem = inst.demand.copy()
        dem[1::7] = 0
        inst = synth.Instance(inst.name, inst.durations, dem, inst.capacities, inst.start_times,
                              inst.problem, inst.meta)
    load(ctx, inst)
    if how == "split_mode_3":
        ctx.set_split_mode(3)
    try:
        islands, pop, n, gens, seed, pmut = 3, 48, inst.n, 3, 99, 0.4
        P = synth.random_perms(islands * pop, n, seed=5).astype(np.int16)
        out = []
        for mode in (0, 2):
            ctx.set_ga_fused(mode)
            try:
                dpop = torch.from_numpy(P.reshape(islands, pop, n).copy()).to(ctx.dev)
                keys = ctx.eval(dpop.view(islands * pop, n)).view(islands, pop)
                ctx.ga_generation(dpop, keys, generations=gens, pmut=pmut, seed=seed, gen0=0)
                out.append((dpop.cpu().numpy(), u64(keys)))
            finally:
                ctx.set_ga_fused(0)
        assert (out[0][0] == out[1][0]).all()
        assert out[0][1] == out[1][1]
        sc = scorer(inst)
        rpop = [[list(r) for r in P.reshape(islands, pop, n)[i]] for i in range(islands)]
        rkeys = [[sc(t) for t in rpop[i]] for i in range(islands)]
        pm = min(int(round(pmut * 2**32)), 2**32 - 1)
        for g in range(gens):
            rpop, rkeys = search.ga_generation(sc, rpop, rkeys, seed, g, pm)
        assert out[0][0].tolist() == rpop
        assert out[0][1] == [k for ks in rkeys for k in ks]
    finally:
        ctx.set_split_mode(0)


@pytest.mark.parametrize("problem", ["cvrp", "tsp"])
def test_bf_n13_rank_windows_match_c_restatement(ctx, coracle, problem):
    """The front-end cap (13 customers, 13! = 6.2 G > 2^32 ranks): a window
    straddling rank 2^32 (64-bit unranking) and the first 10^6 ranks equal
    the C brute force.  Reference slots: api/{tsp,vrp}/bf/index.py:39-44."""
    from vrpms_amd.core import CVRP, TSP
    if problem == "cvrp":
        inst = synth.cvrp(13, 3, seed=13)
        ctx.set_instance(CVRP, inst.durations, inst.demand, inst.capacities, inst.start_times)
        kw = dict(demand=inst.demand, capacities=inst.capacities, start_times=inst.start_times)
    else:
        D = synth.tsp20(13).durations[:, :14, :14]
        inst = synth.Instance("t13", D, None, None, np.array([0]), "tsp")
        ctx.set_instance(TSP, inst.durations, start_times=inst.start_times)
        kw = dict(start_times=inst.start_times, problem=0)
    n = 13
    for lo, hi in ((2**32 - 5000, 2**32 + 5000), (0, 10**6), (math.factorial(13) - 7777,
                                                               math.factorial(13))):
        got = ctx.bf_run(n, lo, hi)
        ref = coracle.bf(inst.durations, n, lo, hi, **kw)
        assert got == ref, (lo, hi)
        assert lo <= got[1] < hi
        assert scorer(inst)(search.unrank(got[1], n)) == got[0]


@pytest.mark.parametrize("lo,hi", [(65_536, 1_000_000), (70_000, 4_000_000)],
                         ids=["i32_stage_dword_argmin", "i32_stage_u64_argmin"])
def test_tsp_batch_tsp50_int32_staging_matches_c_restatement(ctx, coracle, lo, hi):
    """cfg 5 at N = 50 with entries >= 65,536: the matrix cannot be staged as
    uint16, so the int32 LDS staging runs; the second range also pushes the
    tour sum past 2^26 (64-bit (key, lane) argmin).  64 requests x 200 steps
    vs the C restatement.  Reference slot: api/tsp/sa/index.py:40-44."""
    torch = torch_()
    rng = np.random.default_rng(lo)
    R, N = 64, 50
    mats = []
    for _ in range(R):
        m = rng.integers(lo, hi, size=(N, N))
        m = np.triu(m, 1)
        m = m + m.T
        mats.append(m)
    mats = np.stack(mats)
    assert mats.max() * N < 2**28
    M = torch.tensor(mats, dtype=torch.int32, device=ctx.dev)
    tours, keys = ctx.tsp_batch_sa(M, steps=200, inv_t0=1 / (0.3 * lo), inv_alpha=1 / 0.99,
                                   seed=77)
    rt, rk = coracle.tsp_batch_sa(mats, 200, 1 / (0.3 * lo), 1 / 0.99, 77)
    assert (tours.cpu().numpy().view(np.uint16) == rt).all()
    assert u64(keys) == [int(k) for k in rk]


@pytest.mark.parametrize("name,maker", [ACO_SIZES[1], ACO_SIZES[3]], ids=["cvrp100", "cvrp300"])
def test_aco_best_so_far_deposit_matches_oracle(ctx, name, maker):
    """Max-min global-best deposits (bsf_period): every 2nd iteration the
    colony's best-so-far -- here seeded with a migrant-like tour that beats
    the first ants -- deposits instead of the iteration best; tau, tours,
    keys and the best-so-far equal the oracle on the fused (N <= 256) and
    the multi-launch (N > 256) update paths."""
    torch = torch_()
    inst = maker()
    load(ctx, inst)
    colonies, ants, tau0, n = 2, 8, 1 << 20, inst.n
    tau, eta = ctx.aco_init(colonies, tau0)
    ref_eta = search.aco_eta(inst.durations[0])
    rtau = [np.full((inst.N, inst.N), tau0, dtype=np.int64) for _ in range(colonies)]
    sc = scorer(inst)
    # colony 0 starts from a good injected tour (a greedy nearest-neighbour order), colony 1 empty
    D0 = inst.durations[0]
    cur, left, nn = 0, set(range(1, n + 1)), []
    while left:
        cur = min(left, key=lambda c: (D0[cur, c], c))
        nn.append(cur)
        left.remove(cur)
    rbest = [[list(nn), [0] * n], [sc(nn), 2**64 - 1]]
    bt = torch.tensor([nn, [0] * n], dtype=torch.int16, device=ctx.dev)
    bk = torch.tensor([sc(nn) - (1 << 64) if sc(nn) >= 1 << 63 else sc(nn), -1], dtype=torch.int64,
                      device=ctx.dev)
    for it in range(4):
        tours, keys, ib = ctx.aco_iteration(tau, eta, ants, seed=5, it=it, evap_shift=3,
                                            tau_min=1 << 10, tau_max=1 << 30, best_tours=bt,
                                            best_keys=bk, bsf_period=2)
        rt, rk, rib = search.aco_iteration(sc, rtau, ref_eta, ants, n, 5, it, 3, 1 << 10, 1 << 30,
                                           best=rbest, bsf_period=2)
        assert tours.cpu().numpy().tolist() == rt
        assert u64(keys) == [k for ks in rk for k in ks]
        assert [(a & (2**64 - 1), b) for a, b in ib.cpu().tolist()] == rib
        got_tau = tau.cpu().numpy().astype(np.int64) & 0xFFFFFFFF
        assert all((got_tau[c] == rtau[c]).all() for c in range(colonies)), it
        assert bt.cpu().numpy().tolist() == rbest[0] and u64(bk) == rbest[1]


@pytest.mark.parametrize("algo", ["ga", "aco"])
def test_memetic_polish_matches_c_restatement(ctx, coracle, algo):
    """The memetic step of the GA / ACO endpoints (runners.Polish): after an
    epoch, the GA's top-T members of every island / ACO's colony bests are
    the C restatement's SA best-so-far from the un-polished epoch's rows
    (same Philox stream, temperature and step counter); every other GA slot
    is the plain generation's."""
    from vrpms_amd import runners
    inst = synth.cvrp(60, 5, seed=21, slack=1.2)
    load(ctx, inst)
    pol = runners.Polish(25, inst.durations, seed=9)
    inv_t, inv_a, pseed = float(pol.inv_t), float(pol.inv_alpha), pol.seed
    if algo == "ga":
        T = 3
        r = runners.GARunner(ctx, inst.n, islands=4, pop=32, seed=5, gens_per_epoch=3,
                             polish=pol, polish_top=T)
        plain = runners.GARunner(ctx, inst.n, islands=4, pop=32, seed=5, gens_per_epoch=3)
        r.epoch()
        plain.epoch()
        rows = plain.tours[:, :T, :].reshape(-1, inst.n).cpu().numpy().view(np.uint16).copy()
        keys = u64(plain.keys[:, :T].reshape(-1))
        got_t = r.tours[:, :T, :].reshape(-1, inst.n).cpu().numpy().view(np.uint16)
        got_k = u64(r.keys[:, :T].reshape(-1))
        assert torch_().equal(r.tours[:, T:], plain.tours[:, T:])
        assert torch_().equal(r.keys[:, T:], plain.keys[:, T:])
    else:
        r = runners.ACORunner(ctx, inst.n, colonies=3, ants=16, seed=5, iters_per_epoch=2,
                              polish=pol)
        plain = runners.ACORunner(ctx, inst.n, colonies=3, ants=16, seed=5, iters_per_epoch=2)
        r.epoch()
        plain.epoch()
        rows = plain.best_t.cpu().numpy().view(np.uint16).copy()
        keys = u64(plain.best_key)
        got_t = r.best_t.cpu().numpy().view(np.uint16)
        got_k = u64(r.best_key)
    cur, best = rows.copy(), rows.copy()
    bk = np.array(keys, dtype=np.uint64)
    coracle.sa_run(inst.durations, cur, best, bk, 25, inv_t, inv_a, pseed, 0, inst.demand,
                   inst.capacities, inst.start_times)
    assert (got_t == best).all()
    assert got_k == [int(x) for x in bk]
    assert all(g <= k for g, k in zip(got_k, keys))
    assert any(g < k for g, k in zip(got_k, keys))      # the polish improved something
