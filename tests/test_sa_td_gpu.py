"""sa_td_kernel: SA on hour-indexed matrices (A3 time_of_day, src/solver.py:7)
whose walks read every duration from 24-hour edge rows cached per tour
position in LDS -- the reference's normal VRP request (per-vehicle
capacities and start times, api/parameters.py:11-12; endpoint
api/vrp/sa/index.py:40-45).  Every case runs the kernel forced (option 4)
against the C restatement's full re-evaluation (same Philox streams) and
against sa_kernel (option 2) on the device: tours, current keys, best tours
and best keys bit-equal."""
import dataclasses

import numpy as np
import pytest

from oracle import spec
from vrpms_amd import synth

pytestmark = pytest.mark.gpu


def torch_():
    import torch
    return torch


def u64(t):
    return [int(x) & (2**64 - 1) for x in t.reshape(-1).cpu().tolist()]


def _classes(inst, fracs, shuffle=False):
    K = len(inst.capacities)
    base = int(inst.capacities[0])
    caps = np.array([max(int(base * fracs[k * len(fracs) // K]), int(inst.demand.max()))
                     for k in range(K)], dtype=np.int64)
    if shuffle:
        np.random.default_rng(K).shuffle(caps)
    return dataclasses.replace(inst, capacities=caps)


def _tight(inst, fracs, shuffle=False):
    """Capacity classes whose smallest vehicle is below the largest demand
    (half of it): some customers fit only some vehicles, so sa_td_kernel
    takes its non-FAST walk (the per-token capacity branch, max_dem >
    min_cap) -- ADVICE r5."""
    K = len(inst.capacities)
    base = int(inst.capacities[0])
    small = max(1, int(inst.demand.max()) // 2)
    caps = np.array([max(int(base * fracs[k * len(fracs) // K]), int(inst.demand.max()))
                     for k in range(K)], dtype=np.int64)
    caps[K // 2::3] = small
    if shuffle:
        np.random.default_rng(K + 1).shuffle(caps)
    out = dataclasses.replace(inst, capacities=caps)
    assert int(out.capacities.min()) < int(out.demand.max())
    return out


def _starts(inst, base=420):
    st = np.arange(inst.K, dtype=np.int64) * 37 % 240 + base
    return dataclasses.replace(inst, start_times=st)


def _asym_td(inst, seed):
    """every hour slice perturbed asymmetrically (reverse rows R[q])."""
    rng = np.random.default_rng(seed)
    D = inst.durations + rng.integers(0, 30, size=inst.durations.shape)
    for h in range(D.shape[0]):
        np.fill_diagonal(D[h], 0)
    return dataclasses.replace(inst, durations=D)


def _tsp_td(n, seed):
    td = synth.td_cvrp(n, 2, seed=seed)
    return synth.Instance(f"tsptd{n}", td.durations, None, None, np.array([470]), "tsp")


def sep_tours(C, n, S, seed):
    rng = np.random.default_rng(seed)
    base = np.concatenate([np.arange(1, n + 1), np.zeros(S, dtype=np.int64)])
    return rng.permuted(np.tile(base, (C, 1)), axis=1).astype(np.uint16)


def load(ctx, inst):
    from vrpms_amd.core import CVRP, TSP
    if inst.problem == "tsp":
        ctx.set_instance(TSP, inst.durations, start_times=inst.start_times)
    else:
        ctx.set_instance(CVRP, inst.durations, inst.demand, inst.capacities, inst.start_times)


def starts(ctx, inst, kind, chains, seed=9):
    if inst.problem == "tsp":
        return synth.random_perms(chains, inst.n, seed=seed, dtype=np.uint16)
    S = inst.K - 1
    if kind == "random":
        return sep_tours(chains, inst.n, S, seed)
    P0 = synth.random_perms(chains, inst.n, seed=seed, dtype=np.uint16)
    if kind == "nosep":
        return P0
    return np.array([spec.pack_separators(p, S, inst.demand, inst.capacities) for p in P0],
                    dtype=np.uint16)


def run(ctx, P, steps, inv_t0, inv_alpha, seed, step0, window, types, moves, mode):
    torch = torch_()
    cur = torch.from_numpy(P.astype(np.int16)).to(ctx.dev)
    best = cur.clone()
    ck = torch.empty(P.shape[0], dtype=torch.int64, device=ctx.dev)
    bk = torch.full((P.shape[0],), -1, dtype=torch.int64, device=ctx.dev)
    ctx.set_sa_route(mode)
    try:
        ctx.sa_run(cur, ck, best, bk, steps=steps, inv_t0=inv_t0, inv_alpha=inv_alpha, seed=seed,
                   step0=step0, window=window, window_types=types, moves=moves)
    finally:
        ctx.set_sa_route(0)
    return cur.cpu().numpy().view(np.uint16), u64(ck), best.cpu().numpy().view(np.uint16), u64(bk)


TD_CASES = [
    # (case, instance, start, chains, steps, inv_t0, window, types, moves)
    # the reference's normal request: three capacity classes, staggered starts
    ("td200_het_classes_starts", lambda: _starts(_classes(synth.td_cvrp(200, 16, seed=21),
                                                          (1.3, 1.0, 0.8))), "pack", 8, 80,
     1 / 200.0, 16, 2, 64),
    # uniform fleet, one start time, first-fit start
    ("td200_uniform_pack", lambda: synth.td_cvrp(200, 16, seed=22), "pack", 8, 80, 1 / 200.0, 0,
     0, 64),
    # infeasible random separators: unserved customers, vehicles exhausted
    ("td200_random_seps", lambda: synth.td_cvrp(200, 16, seed=23), "random", 8, 60, 1 / 200.0,
     16, 0, 64),
    # hot (accept nearly every step: the row caches are rewritten every step)
    ("td200_het_shuffled_hot", lambda: _classes(synth.td_cvrp(200, 16, seed=24), (1.2, 0.9),
                                                shuffle=True), "pack", 8, 80, 1e-7, 0, 0, 64),
    # asymmetric in every hour: reversed adjacencies read the reverse rows
    ("td150_asym_het", lambda: _starts(_classes(_asym_td(synth.td_cvrp(150, 12, seed=25), 3),
                                                (1.3, 0.9))), "pack", 8, 80, 1e-7, 0, 0, 64),
    ("td120_asym_random", lambda: _asym_td(synth.td_cvrp(120, 10, seed=26), 4), "random", 8, 60,
     1 / 150.0, 0, 0, 64),
    # W = 2 / 4 wavefronts per chain (move index lane + 64 w)
    ("td200_het_m128", lambda: _starts(_classes(synth.td_cvrp(200, 16, seed=27),
                                                (1.3, 1.0, 0.8))), "pack", 4, 60, 1 / 200.0, 16, 2,
     128),
    ("td150_asym_m256_hot", lambda: _asym_td(synth.td_cvrp(150, 12, seed=28), 5), "pack", 4, 50,
     1e-7, 0, 0, 256),
    # no separators at all (the greedy split places every route)
    ("td100_nosep", lambda: synth.td_cvrp(100, 8, seed=29), "nosep", 8, 60, 1 / 100.0, 0, 0, 64),
    # hour-indexed TSP (startTime, api/parameters.py:12)
    ("tsp_td120", lambda: _tsp_td(120, 30), "perm", 8, 80, 1 / 300.0, 0, 0, 64),
    ("tsp_td61_m192", lambda: _tsp_td(61, 31), "perm", 4, 60, 1e-7, 0, 0, 192),
    # tiny tours (2 and 3 tokens, every move touches the ends)
    ("td2", lambda: synth.td_cvrp(2, 1, seed=32), "nosep", 4, 20, 1 / 50.0, 0, 0, 64),
    ("td3_seps", lambda: synth.td_cvrp(3, 2, seed=33), "random", 4, 20, 1 / 50.0, 0, 0, 64),
    # round 6: a vehicle class smaller than the largest demand --
    # the non-FAST variant (per-token capacity branch) -- packed and random
    # separators, staggered starts, asymmetric hours, W = 2
    ("td200_tight_pack_starts", lambda: _starts(_tight(synth.td_cvrp(200, 16, seed=41),
                                                       (1.3, 1.0))), "pack", 8, 80, 1 / 200.0,
     16, 2, 64),
    ("td200_tight_random_seps", lambda: _tight(synth.td_cvrp(200, 16, seed=42), (1.2, 1.0),
                                               shuffle=True), "random", 8, 60, 1 / 200.0, 0, 0,
     64),
    ("td150_tight_asym_hot", lambda: _starts(_tight(_asym_td(synth.td_cvrp(150, 12, seed=43), 6),
                                                    (1.3, 0.9))), "pack", 8, 60, 1e-7, 0, 0, 64),
    ("td200_tight_m128", lambda: _starts(_tight(synth.td_cvrp(200, 16, seed=44), (1.3, 1.0),
                                                shuffle=True)), "random", 4, 60, 1 / 200.0, 16,
     2, 128),
]


@pytest.mark.parametrize("name,maker,start,chains,steps,inv_t0,window,types,moves", TD_CASES,
                         ids=[c[0] for c in TD_CASES])
def test_td_rows_sa_matches_c_restatement(ctx, coracle, name, maker, start, chains, steps, inv_t0,
                                          window, types, moves):
    inst = maker()
    load(ctx, inst)
    P = starts(ctx, inst, start, chains)
    got = run(ctx, P, steps, inv_t0, 1 / 0.99, 21, 7, window, types, moves, 4)
    ccur, cbest = P.copy(), P.copy()
    cbk = np.full(chains, 2**64 - 1, dtype=np.uint64)
    cck = coracle.sa_run(inst.durations, ccur, cbest, cbk, steps, inv_t0, 1 / 0.99, 21, 7,
                         inst.demand, inst.capacities, inst.start_times,
                         problem=0 if inst.problem == "tsp" else 1, window=window,
                         window_types=types, moves=moves)
    assert (got[0] == ccur).all()
    assert got[1] == [int(x) for x in cck] and got[3] == [int(x) for x in cbk]
    assert (got[2] == cbest).all()
    # the automatic dispatch takes the same kernel; sa_kernel (one wavefront
    # per chain) follows the same trajectories
    auto = run(ctx, P, steps, inv_t0, 1 / 0.99, 21, 7, window, types, moves, 0)
    assert (auto[0] == got[0]).all() and auto[1] == got[1] and auto[3] == got[3]
    if moves == 64:
        full = run(ctx, P, steps, inv_t0, 1 / 0.99, 21, 7, window, types, moves, 2)
        assert (full[0] == got[0]).all() and full[1] == got[1] and full[3] == got[3]


def test_td_rows_sa_launch_shape_independent(ctx):
    """1,024 chains (four chains per workgroup sharing the depot legs) and
    1 chain: the first chain's trajectory is the same."""
    inst = _starts(_classes(synth.td_cvrp(200, 16, seed=34), (1.3, 1.0, 0.8)))
    load(ctx, inst)
    P = starts(ctx, inst, "pack", 1024)
    big = run(ctx, P, 40, 1 / 200.0, 1 / 0.99, 5, 0, 16, 2, 64, 4)
    small = run(ctx, P[:8].copy(), 40, 1 / 200.0, 1 / 0.99, 5, 0, 16, 2, 64, 4)
    assert (big[0][:8] == small[0]).all() and big[1][:8] == small[1] and big[3][:8] == small[3]


def test_td_rows_sa_forced_rejects_static(ctx):
    """Option 4 on a static matrix is an error, not a silent fallback."""
    inst = synth.cvrp(30, 4, seed=1)
    load(ctx, inst)
    P = synth.random_perms(4, inst.n, seed=1, dtype=np.uint16)
    with pytest.raises(RuntimeError):
        run(ctx, P, 2, 0.01, 1.0, 1, 0, 0, 0, 64, 4)


def test_td_rows_sa_large_instance_falls_back(ctx, coracle):
    """TD-1000 x 24: the depot-leg rows alone (96 KB) and one chain's rows do
    not fit the LDS -- option 4 is refused, the automatic dispatch takes the
    full-walk L2 kernel, and the trajectory still equals the C restatement."""
    inst = synth.td_cvrp(1000, 50, seed=35)
    load(ctx, inst)
    P = starts(ctx, inst, "pack", 2)
    with pytest.raises(RuntimeError):
        run(ctx, P, 3, 1 / 200.0, 1 / 0.99, 5, 0, 32, 2, 64, 4)
    got = run(ctx, P, 3, 1 / 200.0, 1 / 0.99, 5, 0, 32, 2, 64, 0)
    ccur, cbest = P.copy(), P.copy()
    cbk = np.full(2, 2**64 - 1, dtype=np.uint64)
    cck = coracle.sa_run(inst.durations, ccur, cbest, cbk, 3, 1 / 200.0, 1 / 0.99, 5, 0,
                         inst.demand, inst.capacities, inst.start_times, window=32,
                         window_types=2)
    assert (got[0] == ccur).all() and got[1] == [int(x) for x in cck]


def test_td_rows_sa_mid_size_fits(ctx, coracle):
    """TD-600 x 24 (n + separators ~ 640 tokens): still one chain per
    workgroup in the LDS, trajectory equal to the C restatement."""
    inst = _starts(_classes(synth.td_cvrp(600, 40, seed=36), (1.2, 1.0)))
    load(ctx, inst)
    P = starts(ctx, inst, "pack", 4)
    got = run(ctx, P, 20, 1 / 200.0, 1 / 0.99, 5, 0, 32, 2, 64, 4)
    ccur, cbest = P.copy(), P.copy()
    cbk = np.full(4, 2**64 - 1, dtype=np.uint64)
    cck = coracle.sa_run(inst.durations, ccur, cbest, cbk, 20, 1 / 200.0, 1 / 0.99, 5, 0,
                         inst.demand, inst.capacities, inst.start_times, window=32,
                         window_types=2)
    assert (got[0] == ccur).all() and got[1] == [int(x) for x in cck]
    assert got[3] == [int(x) for x in cbk]
