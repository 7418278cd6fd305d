"""A10 route separators (token 0 inside a CVRP giant tour) on every scoring
path, the decode and the SA kernels, against the C / Python oracle."""
import numpy as np
import pytest

from oracle import search, spec
from oracle import pool as opool
from vrpms_amd import synth

pytestmark = pytest.mark.gpu


def torch_():
    import torch
    return torch


def u64(t):
    return [int(x) & (2**64 - 1) for x in t.reshape(-1).cpu().tolist()]


def sep_tours(C, n, S, seed, ld=None, dtype=np.uint8):
    """C random orders of customers 1..n plus S separators (zeros)."""
    rng = np.random.default_rng(seed)
    L = n + S
    ld = L if ld is None else ld
    out = np.zeros((C, ld), dtype=dtype)
    base = np.concatenate([np.arange(1, n + 1), np.zeros(S, dtype=np.int64)])
    out[:, :L] = rng.permuted(np.tile(base, (C, 1)), axis=1).astype(dtype)
    return out


def load(ctx, inst, objective=0):
    from vrpms_amd.core import CVRP
    ctx.set_instance(CVRP, inst.durations, inst.demand, inst.capacities, inst.start_times,
                     objective=objective)


def check(ctx, coracle, inst, P, L, objective=0):
    torch = torch_()
    dP = torch.from_numpy(P).to(ctx.dev)
    keys, sums, maxs, unv = ctx.eval(dP, n=L, with_parts=True)
    ref = coracle.eval_batch(inst.durations, P, inst.demand, inst.capacities, inst.start_times,
                             1, objective, n=L)
    got = keys.cpu().numpy().view(np.uint64)
    np.testing.assert_array_equal(got, ref[0])
    np.testing.assert_array_equal(sums.cpu().numpy(), ref[1])
    np.testing.assert_array_equal(maxs.cpu().numpy(), ref[2])
    np.testing.assert_array_equal(unv.cpu().numpy(), ref[3])
    for i in range(0, P.shape[0], max(1, P.shape[0] // 5)):
        r = spec.eval_cvrp(inst.durations, P[i, :L], inst.demand, inst.capacities,
                           inst.start_times, objective)
        assert int(got[i]) == r["key"]
    return got


@pytest.mark.parametrize("slack,S", [(1.1, 7), (0.9, 3), (1.3, 12)])
def test_fast_split_kernels_with_separators(ctx, coracle, slack, S):
    """rows2 (every configuration), words2 and eval_cvrp_packed MODE 1/2 on
    CVRP-100 tours with S separators; tight fleets exhaust (exact re-walk)."""
    from vrpms_amd.core import VrpmsError  # noqa: F401
    inst = synth.cvrp(100, 8, seed=S, slack=slack)
    load(ctx, inst)
    L = inst.n + S
    ld = (L + 3) // 4 * 4
    P = sep_tours(6007, inst.n, S, seed=S, ld=ld)
    try:
        ref = check(ctx, coracle, inst, P, L)
        for cfg in range(1, 6):
            ctx.set_rows_config(cfg)
            np.testing.assert_array_equal(check(ctx, coracle, inst, P, L), ref)
        ctx.set_rows_config(0)
        ctx.set_words_kernel(1)          # eval_cvrp_packed, prefix-ret (MODE 1)
        np.testing.assert_array_equal(check(ctx, coracle, inst, P, L), ref)
        ctx.set_split_mode(2)            # eval_cvrp_packed, branchy (MODE 2)
        np.testing.assert_array_equal(check(ctx, coracle, inst, P, L), ref)
    finally:
        ctx.set_rows_config(0)
        ctx.set_words_kernel(0)
        ctx.set_split_mode(0)
    torch = torch_()
    words = ctx.to_words(torch.from_numpy(P).to(ctx.dev), L)
    k = ctx.eval_words(words, L)
    np.testing.assert_array_equal(k.cpu().numpy().view(np.uint64), ref)


def test_heterogeneous_fleet_and_generic_paths(ctx, coracle):
    """MODE 0 (heterogeneous capacities, packed) and the L2 / generic paths
    (uint16 tours, N = 150; hour-indexed TD-60) with separators."""
    inst = synth.cvrp(40, 5, seed=3, slack=1.0)
    inst.capacities = np.array([30, 60, 45, 80, 50])
    load(ctx, inst)
    P = sep_tours(3001, inst.n, 4, seed=1, ld=44)
    check(ctx, coracle, inst, P, inst.n + 4)
    big = synth.cvrp(150, 12, seed=4)
    load(ctx, big)
    P = sep_tours(2003, big.n, 11, seed=2, dtype=np.uint16).astype(np.int16)
    check(ctx, coracle, big, P, big.n + 11)
    td = synth.td_cvrp(60, 5, seed=5)
    load(ctx, td)
    P = sep_tours(2001, td.n, 4, seed=3, ld=64)
    check(ctx, coracle, td, P, td.n + 4)


def test_decode_marks_separators(ctx):
    torch = torch_()
    inst = synth.cvrp(20, 4, seed=6, slack=1.2)
    load(ctx, inst)
    P = sep_tours(5, inst.n, 3, seed=9)
    for row in P:
        veh, dur = ctx.decode(torch.from_numpy(row.astype(np.int16)).to(ctx.dev), len(row))
        r = spec.eval_cvrp(inst.durations, row, inst.demand, inst.capacities, inst.start_times)
        assert veh == r["vehicle_of"] and dur == r["durations"]


@pytest.mark.parametrize("kind", ["packed", "generic_td"])
def test_sa_with_separators_matches_oracle(ctx, coracle, kind):
    """SA trajectories over separator tours: sa_packed_kernel (cfg-2 style)
    against the C restatement, sa_kernel on an hour-indexed instance against
    the Python replay."""
    torch = torch_()
    if kind == "packed":
        inst, S, chains, steps = synth.cvrp(60, 6, seed=7, slack=1.05), 5, 16, 60
    else:
        inst, S, chains, steps = synth.td_cvrp(12, 3, seed=8), 2, 3, 10
    load(ctx, inst)
    L = inst.n + S
    P = sep_tours(chains, inst.n, S, seed=4, dtype=np.uint16).astype(np.int16)
    cur = torch.from_numpy(P).to(ctx.dev)
    best = cur.clone()
    ck = torch.empty(chains, dtype=torch.int64, device=ctx.dev)
    bk = torch.full((chains,), -1, dtype=torch.int64, device=ctx.dev)
    ctx.sa_run(cur, ck, best, bk, steps=steps, inv_t0=1 / 60.0, inv_alpha=1 / 0.99, seed=3,
               step0=11)
    if kind == "packed":
        ccur, cbest = P.view(np.uint16).copy(), P.view(np.uint16).copy()
        cbk = np.full(chains, 2**64 - 1, dtype=np.uint64)
        cck = coracle.sa_run(inst.durations, ccur, cbest, cbk, steps, 1 / 60.0, 1 / 0.99, 3, 11,
                             inst.demand, inst.capacities, inst.start_times)
        assert (cur.cpu().numpy().view(np.uint16) == ccur).all()
        assert u64(ck) == [int(x) for x in cck] and u64(bk) == [int(x) for x in cbk]
    else:
        sc = search.Scorer(inst.durations, inst.demand, inst.capacities, inst.start_times)
        ref = search.sa_run(sc, P.tolist(), P.tolist(), [2**64 - 1] * chains, 3, 11, steps,
                            1 / 60.0, 1 / 0.99)
        assert cur.cpu().numpy().tolist() == ref[0] and u64(bk) == ref[3]
    assert all(sorted(r) == [0] * S + list(range(1, inst.n + 1)) for r in cur.cpu().tolist())


def test_random_tours_with_separators(ctx):
    T = ctx.random_tours(50, 30, seed=4, stream_id=1, n_sep=5).cpu().tolist()
    for r in (0, 17, 49):
        assert T[r] == opool.philox_tour(30, 4, r, 1, 5)
    assert all(sorted(t) == [0] * 5 + list(range(1, 31)) for t in T)


def _run_sa(ctx, P, steps, inv_t0, inv_alpha, seed, step0, window, types=0):
    torch = torch_()
    cur = torch.from_numpy(P).to(ctx.dev)
    best = cur.clone()
    ck = torch.empty(P.shape[0], dtype=torch.int64, device=ctx.dev)
    bk = torch.full((P.shape[0],), -1, dtype=torch.int64, device=ctx.dev)
    ctx.sa_run(cur, ck, best, bk, steps=steps, inv_t0=inv_t0, inv_alpha=inv_alpha, seed=seed,
               step0=step0, window=window, window_types=types)
    return cur.cpu().numpy(), u64(ck), best.cpu().numpy(), u64(bk)


def _asym(inst, seed, scale=1):
    """inst with an asymmetric static matrix (the route kernel's reverse-edge
    cache); scale > 1 pushes entries past 65535 (int32 matrix)."""
    import dataclasses
    rng = np.random.default_rng(seed)
    D = inst.durations[0] * scale + rng.integers(0, 40, size=inst.durations.shape[1:])
    np.fill_diagonal(D, 0)
    return dataclasses.replace(inst, durations=D[None])


ROUTE_CASES = [
    # cfg 4: X-1000, K - 1 separators where the greedy split closes routes
    ("x1000_greedy", lambda: synth.x_style(1000, seed=1), "greedy", 16, 40, 1 / 300.0, 32, 0),
    # cfg 4 as the front-end runs it: first-fit routes (a feasible start), windowed 2-opt,
    # swap / relocate anywhere (two-zone pricing)
    ("x1000_pack_2opt", lambda: synth.x_style(1000, seed=2), "pack", 16, 60, 1 / 300.0, 32, 2),
    # many accepted moves (hot): the route tables are updated around every accepted zone
    ("x1000_pack_long_hot", lambda: synth.x_style(1000, seed=4), "pack", 8, 400, 1 / 2000.0, 32,
     2),
    ("x1000_pack_all_windowed", lambda: synth.x_style(1000, seed=5), "pack", 8, 150, 1 / 300.0,
     24, 0),
    # cfg 3: hour-indexed TD-200 (one start time), random separators: an infeasible start,
    # so moves that leave customers unserved are re-evaluated in full
    ("td200_random", lambda: synth.td_cvrp(200, 16, seed=2), "random", 8, 30, 1 / 200.0, 16, 0),
    ("td200_random_2opt", lambda: synth.td_cvrp(200, 16, seed=4), "random", 8, 30, 1 / 200.0, 16,
     2),
    # first-fit start (trailing separators): an accepted move whose second
    # zone walks to the tour end closes an empty last route there -- its
    # start is the zone's end (the table update once left it stale)
    ("td200_pack_uniform", lambda: synth.td_cvrp(200, 16, seed=21), "pack", 8, 60, 1 / 200.0, 16,
     2),
    # hot chains: the unserved-move shortcut is off (invT < 2^-20)
    ("cvrp150_hot", lambda: synth.cvrp(150, 12, seed=3), "greedy", 8, 30, 1e-7, 8, 0),
    ("cvrp150_pack_hot", lambda: synth.cvrp(150, 12, seed=5, slack=1.02), "pack", 8, 40, 1e-7, 6,
     2),
    # no separators at all: one segment, re-synchronising walks cascade over many
    # routes (more than a lane records: the accepted zones are re-walked)
    ("cvrp200_no_seps", lambda: synth.cvrp(200, 16, seed=7, slack=1.3), "nosep", 8, 80,
     1 / 50.0, 12, 2),
    # many separators per route (S > K - 1 is never route-local; S < K - 1 is)
    ("cvrp120_few_seps", lambda: synth.cvrp(120, 10, seed=6), "pack_few", 8, 40, 1 / 100.0, 5, 2),
    # asymmetric static matrices: reversed adjacencies read the reverse-edge cache
    ("x1000_asym_u16", lambda: _asym(synth.x_style(1000, seed=3), 1), "pack", 8, 120, 1 / 300.0,
     32, 0),
    ("cvrp300_asym_i32", lambda: _asym(synth.cvrp(300, 24, seed=8), 2, scale=60), "pack", 8, 120,
     1 / 18000.0, 24, 0),
    # fleets of different vehicles (api/parameters.py:11-12): three capacity
    # classes and staggered start times on the hour-indexed TD-200 x 24 (the
    # reference's normal VRP request), shuffled classes hot, and static
    # asymmetric matrices (the segment kernel needs a symmetric one): walks
    # re-synchronise on the same vehicle only
    ("td200_het_classes_starts", lambda: _starts(_classes(synth.td_cvrp(200, 16, seed=21),
                                                          (1.3, 1.0, 0.8))), "pack", 8, 60,
     1 / 200.0, 16, 2),
    ("td200_het_shuffled_hot", lambda: _classes(synth.td_cvrp(200, 16, seed=22), (1.2, 0.9),
                                                shuffle=True), "pack", 8, 40, 1e-7, 16, 0),
    ("x1000_asym_het_starts", lambda: _starts(_classes(_asym(synth.x_style(1000, seed=23), 1),
                                                       (1.4, 1.1, 0.9))), "pack", 8, 120,
     1 / 300.0, 32, 2),
    ("cvrp150_asym_het_random", lambda: _classes(_asym(synth.cvrp(150, 12, seed=24, slack=1.3), 2),
                                                 (1.3, 0.8), shuffle=True), "random", 8, 60,
     1 / 100.0, 8, 0),
]


@pytest.mark.parametrize("name,maker,start,chains,steps,inv_t0,window,types", ROUTE_CASES,
                         ids=[c[0] for c in ROUTE_CASES])
def test_route_local_sa_matches_c_restatement(ctx, coracle, name, maker, start, chains, steps,
                                              inv_t0, window, types):
    """sa_route_kernel (windowed moves priced route-locally) against the C
    restatement's full re-evaluation, and against sa_kernel on the device."""
    inst = maker()
    load(ctx, inst)
    S = {"pack_few": inst.K - 4, "nosep": 0}.get(start, inst.K - 1)
    if start == "nosep":
        P = synth.random_perms(chains, inst.n, seed=9, dtype=np.uint16)
    elif start != "random":
        P0 = synth.random_perms(chains, inst.n, seed=9, dtype=np.uint16)
        f = spec.insert_separators if start == "greedy" else spec.pack_separators
        P = np.array([f(p, S, inst.demand, inst.capacities) for p in P0])
        torch = torch_()
        g = ctx.insert_separators if start == "greedy" else ctx.pack_separators
        dev = g(torch.from_numpy(P0.astype(np.int16)).to(ctx.dev), S)
        assert dev.cpu().numpy().tolist() == P.tolist()
    else:
        P = sep_tours(chains, inst.n, S, seed=9, dtype=np.uint16)
    P = P.astype(np.int16)
    got = _run_sa(ctx, P, steps, inv_t0, 1 / 0.99, 21, 7, window, types)
    ccur, cbest = P.view(np.uint16).copy(), P.view(np.uint16).copy()
    cbk = np.full(chains, 2**64 - 1, dtype=np.uint64)
    cck = coracle.sa_run(inst.durations, ccur, cbest, cbk, steps, inv_t0, 1 / 0.99, 21, 7,
                         inst.demand, inst.capacities, inst.start_times, window=window,
                         window_types=types)
    assert (got[0].view(np.uint16) == ccur).all()
    assert got[1] == [int(x) for x in cck] and got[3] == [int(x) for x in cbk]
    assert (got[2].view(np.uint16) == cbest).all()
    # the same chains through the route-local walks (3) and full re-evaluation (2)
    for mode in (3, 2):
        ctx.set_sa_route(mode)
        try:
            other = _run_sa(ctx, P, steps, inv_t0, 1 / 0.99, 21, 7, window, types)
        finally:
            ctx.set_sa_route(0)
        assert (other[0] == got[0]).all() and other[1] == got[1] and other[3] == got[3]


MULTIWAVE_CASES = [
    # (case, moves): W = moves / 64 wavefronts per chain price 64 W moves per step
    ("x1000_pack_2opt", 512),
    ("x1000_pack_long_hot", 256),
    ("td200_random", 256),
    ("cvrp150_hot", 128),
    ("cvrp200_no_seps", 192),
    ("x1000_asym_u16", 512),
    ("td200_het_classes_starts", 256),
    ("x1000_asym_het_starts", 128),
]


@pytest.mark.parametrize("name,moves", MULTIWAVE_CASES, ids=[f"{c}-m{m}" for c, m in MULTIWAVE_CASES])
def test_route_local_multiwave_matches_c_restatement(ctx, coracle, name, moves):
    """W wavefronts per chain (64 W moves per step, move index lane + 64 w,
    (key, index) minimum across wavefronts) against the C restatement with
    the same `moves`, full re-walk and route-resync pricing alike."""
    case = {c[0]: c for c in ROUTE_CASES}[name]
    _, maker, start, chains, steps, inv_t0, window, types = case
    inst = maker()
    load(ctx, inst)
    S = {"pack_few": inst.K - 4, "nosep": 0}.get(start, inst.K - 1)
    if start == "nosep":
        P = synth.random_perms(chains, inst.n, seed=9, dtype=np.uint16)
    elif start != "random":
        P0 = synth.random_perms(chains, inst.n, seed=9, dtype=np.uint16)
        f = spec.insert_separators if start == "greedy" else spec.pack_separators
        P = np.array([f(p, S, inst.demand, inst.capacities) for p in P0])
    else:
        P = sep_tours(chains, inst.n, S, seed=9, dtype=np.uint16)
    P = P.astype(np.int16)
    torch = torch_()
    cur = torch.from_numpy(P).to(ctx.dev)
    best = cur.clone()
    ck = torch.empty(chains, dtype=torch.int64, device=ctx.dev)
    bk = torch.full((chains,), -1, dtype=torch.int64, device=ctx.dev)
    ctx.sa_run(cur, ck, best, bk, steps=steps, inv_t0=inv_t0, inv_alpha=1 / 0.99, seed=21,
               step0=7, window=window, window_types=types, moves=moves)
    for resync in (False, True):
        ccur, cbest = P.view(np.uint16).copy(), P.view(np.uint16).copy()
        cbk = np.full(chains, 2**64 - 1, dtype=np.uint64)
        cck = coracle.sa_run(inst.durations, ccur, cbest, cbk, steps, inv_t0, 1 / 0.99, 21, 7,
                             inst.demand, inst.capacities, inst.start_times, window=window,
                             window_types=types, resync=resync, moves=moves)
        assert (cur.cpu().numpy().view(np.uint16) == ccur).all()
        assert u64(ck) == [int(x) for x in cck] and u64(bk) == [int(x) for x in cbk]
        assert (best.cpu().numpy().view(np.uint16) == cbest).all()


def test_sa_moves_validation(ctx):
    inst = synth.cvrp(30, 4, seed=1)
    load(ctx, inst)
    torch = torch_()
    P = torch.from_numpy(synth.random_perms(4, inst.n, seed=1, dtype=np.uint16).astype(np.int16))
    cur = P.to(ctx.dev)
    ck = torch.empty(4, dtype=torch.int64, device=ctx.dev)
    bk = torch.full((4,), -1, dtype=torch.int64, device=ctx.dev)
    with pytest.raises(RuntimeError):   # not a multiple of 64
        ctx.sa_run(cur, ck, cur.clone(), bk, 2, 0.01, 1.0, 1, 0, window=4, moves=100)
    with pytest.raises(RuntimeError):   # more than 8 wavefronts
        ctx.sa_run(cur, ck, cur.clone(), bk, 2, 0.01, 1.0, 1, 0, window=4, moves=576)
    asym = _asym(synth.cvrp(30, 4, seed=1), 3)   # static asymmetric: no segment pricing
    load(ctx, asym)
    with pytest.raises(RuntimeError):   # window 0: not the route-local kernel
        ctx.sa_run(cur, ck, cur.clone(), bk, 2, 0.01, 1.0, 1, 0, window=0, moves=128)
    td = synth.td_cvrp(30, 4, seed=1)    # hour-indexed: the hour-row kernel takes any window
    load(ctx, td)
    ctx.sa_run(cur, ck, cur.clone(), bk, 2, 0.01, 1.0, 1, 0, window=0, moves=128)
    with pytest.raises(RuntimeError):   # and at most 4 wavefronts (then the route kernel,
        ctx.sa_run(cur, ck, cur.clone(), bk, 2, 0.01, 1.0, 1, 0, window=0, moves=320)  # window 0)


def test_route_local_sa_small_matches_python_oracle(ctx):
    inst = synth.cvrp(24, 4, seed=11, slack=1.15)
    load(ctx, inst)
    P = sep_tours(3, inst.n, 3, seed=2, dtype=np.uint16).astype(np.int16)
    got = _run_sa(ctx, P, 15, 1 / 80.0, 1 / 0.98, 4, 0, 3)
    sc = search.Scorer(inst.durations, inst.demand, inst.capacities, inst.start_times)
    ref = search.sa_run(sc, P.tolist(), P.tolist(), [2**64 - 1] * 3, 4, 0, 15, 1 / 80.0,
                        1 / 0.98, window=3)
    assert got[0].tolist() == ref[0] and got[1] == ref[1]
    assert got[2].tolist() == ref[2] and got[3] == ref[3]


def test_route_local_sa_two_zone_small_matches_python_oracle(ctx):
    """Windowed 2-opt with swap / relocate anywhere (A12), separators moved
    across routes, against the Python replay."""
    inst = synth.cvrp(40, 6, seed=12, slack=1.1)
    load(ctx, inst)
    P = sep_tours(3, inst.n, 5, seed=3, dtype=np.uint16).astype(np.int16)
    got = _run_sa(ctx, P, 25, 1 / 60.0, 1 / 0.98, 5, 3, 4, 2)
    sc = search.Scorer(inst.durations, inst.demand, inst.capacities, inst.start_times)
    ref = search.sa_run(sc, P.tolist(), P.tolist(), [2**64 - 1] * 3, 5, 3, 25, 1 / 60.0,
                        1 / 0.98, window=4, window_types=2)
    assert got[0].tolist() == ref[0] and got[1] == ref[1]
    assert got[2].tolist() == ref[2] and got[3] == ref[3]


def test_pack_separators_matches_spec(ctx):
    """First-fit start tours (vrpms_pack_separators) == oracle/spec.py, and
    they serve every customer on the cfg-4 fleet."""
    torch = torch_()
    x = synth.x_style(1000, seed=3)
    load(ctx, x)
    P0 = synth.random_perms(64, x.n, seed=5, dtype=np.uint16)
    dev = ctx.pack_separators(torch.from_numpy(P0.astype(np.int16)).to(ctx.dev), x.K - 1)
    got = dev.cpu().numpy().view(np.uint16)
    for r in (0, 31, 63):
        assert got[r].tolist() == spec.pack_separators(P0[r], x.K - 1, x.demand, x.capacities)
    keys, sums, maxs, unv = ctx.eval(dev, n=x.n + x.K - 1, with_parts=True)
    assert int(unv.max()) == 0
    het = synth.cvrp(50, 6, seed=2, slack=1.05)
    het.capacities = np.array([40, 90, 60, 70, 55, 80])
    load(ctx, het)
    P0 = synth.random_perms(17, het.n, seed=1, dtype=np.uint16)
    for S in (2, 5, 9):
        dev = ctx.pack_separators(torch.from_numpy(P0.astype(np.int16)).to(ctx.dev), S)
        want = [spec.pack_separators(p, S, het.demand, het.capacities) for p in P0]
        assert dev.cpu().numpy().tolist() == want


SEG_CASES = [
    # (case, instance, start, chains, steps, inv_t0, window, types, moves): the
    # segment-priced kernel on the fleets / move mixes the walk kernel cannot take
    ("x1000_full_range_m256", lambda: synth.x_style(1000, seed=6), "pack", 8, 120, 1 / 300.0, 0,
     0, 256),
    ("x1000_staggered_starts", lambda: _starts(synth.x_style(1000, seed=7)), "pack", 8, 150,
     1 / 300.0, 32, 2, 64),
    ("cvrp300_hot_m128", lambda: synth.cvrp(300, 24, seed=9, slack=1.05), "random", 8, 60, 1e-7, 0,
     0, 128),
    ("cvrp1200_long_tours", lambda: synth.cvrp(1200, 60, seed=10), "pack", 4, 60, 1 / 300.0, 32, 2,
     64),
    # heterogeneous fleets (per-vehicle capacities): the variant that tracks each
    # route's vehicle -- capacity classes in vehicle order with staggered starts,
    # shuffled per-vehicle capacities, and a hot infeasible start whose segments
    # split into several routes (the split's fixed-point pass, tail re-evaluation)
    ("x1000_three_classes_starts", lambda: _starts(_classes(synth.x_style(1000, seed=11),
                                                            (1.25, 1.0, 0.8))), "pack", 8, 150,
     1 / 300.0, 32, 2, 128),
    ("x1000_shuffled_caps_full_range", lambda: _classes(synth.x_style(1000, seed=12),
                                                        (1.3, 1.0, 0.85, 1.1), shuffle=True),
     "pack", 8, 100, 1 / 300.0, 0, 0, 64),
    ("cvrp300_het_hot_random", lambda: _classes(synth.cvrp(300, 24, seed=13, slack=1.2),
                                                (1.5, 1.0, 0.7)), "random", 8, 80, 1e-7, 0, 0, 128),
    ("cvrp300_het_warm_m256", lambda: _classes(synth.cvrp(300, 24, seed=14, slack=1.3),
                                               (1.2, 0.9), shuffle=True), "pack", 8, 200,
     1 / 60.0, 24, 2, 256),
    # four wavefronts x two moves per lane, and an int32 matrix (entries past 65535)
    ("x1000_het_m512", lambda: _classes(synth.x_style(1000, seed=15), (1.4, 1.1, 0.9)), "pack",
     4, 80, 1 / 300.0, 32, 2, 512),
    ("cvrp300_het_i32", lambda: _scaled(_classes(synth.cvrp(300, 24, seed=16, slack=1.3),
                                                 (1.3, 1.0, 0.8)), 90), "pack", 8, 120,
     1 / 27000.0, 24, 2, 128),
    # cold chains on full first-fit routes: overflowing runs stop at the cut budget
    # (K - 1 separators: no cut affordable; K - 4: up to three routes may split)
    ("x1000_cold_cut_budget", lambda: synth.x_style(1000, seed=17), "pack", 8, 300, 1.0, 32, 2,
     128),
    ("cvrp300_few_seps_cold", lambda: synth.cvrp(300, 24, seed=18), "pack_few", 8, 300, 0.5, 24,
     2, 128),
    # round 6: the incremental split (only the segments a move touches are
    # split again, the routes after them shifted) over a long warm run, where
    # most steps accept and route counts change -- and a windowless one, whose
    # swaps / relocates span 64 segments or more (the full pass)
    ("x1000_warm_incremental", lambda: synth.x_style(1000, seed=20), "pack", 8, 600, 1 / 30.0,
     32, 2, 128),
    ("cvrp600_warm_windowless", lambda: synth.cvrp(600, 40, seed=21), "pack", 8, 300, 1 / 60.0,
     0, 0, 64),
    # total demand past 2^31 with the capacity: the u32 prefix demands cannot hold
    # it, so the launcher hands the chains to the full re-evaluation kernels
    ("cvrp150_huge_demand", lambda: _huge_demand(synth.cvrp(150, 12, seed=19)), "pack", 4, 40,
     1 / 300.0, 0, 0, 64),
]


def _huge_demand(inst):
    """inst with demands x 1e7 (total ~2^33) and capacities to match."""
    import dataclasses
    k = 10_000_000
    return dataclasses.replace(inst, demand=inst.demand * k, capacities=inst.capacities * k)


def _scaled(inst, k):
    """inst with its (symmetric) durations times k: entries past 65535 put the
    matrix in int32."""
    import dataclasses
    return dataclasses.replace(inst, durations=inst.durations * k)


def _classes(inst, fracs, shuffle=False):
    """inst with per-vehicle capacities: len(fracs) classes of base * frac in
    vehicle order (shuffled: in a random order), each at least the largest
    demand."""
    import dataclasses
    K = len(inst.capacities)
    base = int(inst.capacities[0])
    caps = np.array([max(int(base * fracs[k * len(fracs) // K]), int(inst.demand.max()))
                     for k in range(K)], dtype=np.int64)
    if shuffle:
        np.random.default_rng(K).shuffle(caps)
    return dataclasses.replace(inst, capacities=caps)


def _starts(inst):
    import dataclasses
    st = np.arange(inst.K, dtype=np.int64) * 37 % 240
    return dataclasses.replace(inst, start_times=st)


@pytest.mark.parametrize("name,maker,start,chains,steps,inv_t0,window,types,moves", SEG_CASES,
                         ids=[c[0] for c in SEG_CASES])
def test_segment_sa_matches_c_restatement(ctx, coracle, name, maker, start, chains, steps, inv_t0,
                                          window, types, moves):
    """sa_seg_kernel (O(1) segment pricing) on full-range moves, several
    moves per lane, staggered vehicle start times (static matrix: a route's
    duration does not depend on its start) and tours longer than 1,100
    tokens, against the C restatement (full walks and segment pricing)."""
    inst = maker()
    load(ctx, inst)
    S = inst.K - 4 if start == "pack_few" else inst.K - 1
    if start in ("pack", "pack_few"):
        P0 = synth.random_perms(chains, inst.n, seed=9, dtype=np.uint16)
        P = np.array([spec.pack_separators(p, S, inst.demand, inst.capacities) for p in P0])
    else:
        P = sep_tours(chains, inst.n, S, seed=9, dtype=np.uint16)
    P = P.astype(np.int16)
    torch = torch_()
    cur = torch.from_numpy(P).to(ctx.dev)
    best = cur.clone()
    ck = torch.empty(chains, dtype=torch.int64, device=ctx.dev)
    bk = torch.full((chains,), -1, dtype=torch.int64, device=ctx.dev)
    ctx.sa_run(cur, ck, best, bk, steps=steps, inv_t0=inv_t0, inv_alpha=1 / 0.99, seed=33,
               step0=5, window=window, window_types=types, moves=moves)
    for resync in (False, True):
        ccur, cbest = P.view(np.uint16).copy(), P.view(np.uint16).copy()
        cbk = np.full(chains, 2**64 - 1, dtype=np.uint64)
        cck = coracle.sa_run(inst.durations, ccur, cbest, cbk, steps, inv_t0, 1 / 0.99, 33, 5,
                             inst.demand, inst.capacities, inst.start_times, window=window,
                             window_types=types, resync=resync, moves=moves)
        assert (cur.cpu().numpy().view(np.uint16) == ccur).all()
        assert u64(ck) == [int(x) for x in cck] and u64(bk) == [int(x) for x in cbk]
        assert (best.cpu().numpy().view(np.uint16) == cbest).all()


@pytest.mark.parametrize("het,moves", [(False, 128), (True, 64)])
def test_segment_sa_two_wavefronts_per_simd_same_trajectories(ctx, het, moves):
    """A launch with more wavefronts than the chip has SIMDs runs
    sa_seg_kernel's OCC = 2 variant (registers capped for two wavefronts per
    SIMD).  Chain c draws the same Philox streams in any launch, so the first
    chains of a 1,280-chain launch must follow exactly the trajectories of
    an 8-chain launch (the OCC = 1 variant, checked against the C
    restatement above)."""
    torch = torch_()
    inst = synth.x_style(1000, seed=3)
    if het:
        inst = _classes(inst, (1.4, 1.1, 0.9))
    load(ctx, inst)
    S = inst.K - 1
    big = 1280
    P0 = synth.random_perms(big, inst.n, seed=9, dtype=np.uint16)
    P = np.array([spec.pack_separators(p, S, inst.demand, inst.capacities) for p in P0])
    P = P.astype(np.int16)
    out = []
    for chains in (8, big):
        cur = torch.from_numpy(P[:chains].copy()).to(ctx.dev)
        best = cur.clone()
        ck = torch.empty(chains, dtype=torch.int64, device=ctx.dev)
        bk = torch.full((chains,), -1, dtype=torch.int64, device=ctx.dev)
        ctx.sa_run(cur, ck, best, bk, steps=60, inv_t0=1 / 300.0, inv_alpha=1 / 0.99, seed=33,
                   step0=5, window=32, window_types=2, moves=moves)
        out.append((cur.cpu().numpy()[:8], u64(ck)[:8], best.cpu().numpy()[:8], u64(bk)[:8]))
    a, b = out
    assert (a[0] == b[0]).all() and a[1] == b[1] and (a[2] == b[2]).all() and a[3] == b[3]
