"""oracle_sa_run_resync (the quality leg's CPU baseline) against the full-walk
oracle_sa_run: same streams and moves, so cur / best tours and keys must be
equal bit for bit on every instance shape the quality sweep and the front-end
use (X-1000 windowed, CVRP-100 with random separators, TD-200, full-range
moves, a tight fleet that exhausts, a non-uniform fleet that falls back)."""
import numpy as np
import pytest

from oracle import coracle, pool, spec
from vrpms_amd import synth


def _starts(inst, chains, n_sep, start, seed):
    rows = []
    for c in range(chains):
        if start == "pack":
            p = pool.philox_tour(inst.n, seed, c)
            rows.append(spec.pack_separators(p, n_sep, inst.demand, inst.capacities))
        else:
            rows.append(pool.philox_tour(inst.n, seed, c, n_sep=n_sep))
    return np.array(rows, dtype=np.uint16)


def _both(inst, P, steps, inv_t0, inv_a, seed, window=0, types=0, step0=0):
    out = []
    for resync in (False, True):
        cur, best = P.copy(), P.copy()
        bk = np.full(P.shape[0], 2**64 - 1, dtype=np.uint64)
        ck = coracle.sa_run(inst.durations, cur, best, bk, steps, inv_t0, inv_a, seed, step0,
                            inst.demand, inst.capacities, inst.start_times, threads=4,
                            window=window, window_types=types, resync=resync)
        out.append((cur, best, bk, ck))
    for a, b in zip(*out):
        assert np.array_equal(a, b)
    return out[1]


@pytest.mark.parametrize("types", [2, 0])
def test_resync_x1000_windowed(types):
    inst = synth.x_style(1000, seed=1)
    P = _starts(inst, 4, inst.K - 1, "pack", 3)
    edge = float(np.asarray(inst.durations)[np.asarray(inst.durations) > 0].mean())
    cur, _, bk, _ = _both(inst, P, 300, 1 / (0.5 * edge), 1 / 0.995, 9, window=32, types=types)
    assert (bk >> np.uint64(56) == 0).all()


def test_resync_cvrp100_random_separators_full_range():
    inst = synth.cvrp(100, 8, seed=2)
    P = _starts(inst, 6, inst.K - 1, "random", 5)
    _both(inst, P, 400, 1 / 150.0, 1 / 0.99, 4)


def test_resync_td200_windowed():
    inst = synth.td_cvrp(200, 16, seed=0)
    P = _starts(inst, 4, inst.K - 1, "pack", 1)
    _both(inst, P, 200, 1 / 120.0, 1 / 0.99, 7, window=16, types=0, step0=13)


def test_resync_tight_fleet_and_plain_giant_tours():
    # slack 1.0: the fleet is barely enough, walks meet the K-th vehicle
    inst = synth.cvrp(60, 6, seed=3, slack=1.0)
    P = _starts(inst, 6, 0, "random", 2)
    _both(inst, P, 300, 1 / 60.0, 1 / 0.99, 11)
    P = _starts(inst, 6, inst.K - 1, "random", 2)
    _both(inst, P, 300, 1 / 60.0, 1 / 0.99, 12)


def test_resync_nonuniform_fleet_falls_back():
    inst = synth.cvrp(40, 4, seed=4)
    caps = np.asarray(inst.capacities).copy()
    caps[1] += 7
    inst = inst._replace(capacities=caps) if hasattr(inst, "_replace") else inst
    if hasattr(inst, "_replace"):
        P = _starts(inst, 3, inst.K - 1, "random", 6)
        _both(inst, P, 100, 1 / 60.0, 1 / 0.99, 3)


@pytest.mark.parametrize("n_sep_off", [1, 4])
def test_resync_cold_cut_budget(n_sep_off):
    """Cold chains on first-fit routes: most moved pieces overflow a full
    route; segment pricing stops an overflowing run once the composed
    segments' cuts exceed what the fleet count allows (K - 1 - S + T minus the
    other segments' cuts).  n_sep_off 1: K - 1 separators, no cut is ever
    affordable; 4: K - 4 separators, up to three routes may split."""
    inst = synth.x_style(1000, seed=3)
    P = _starts(inst, 4, inst.K - n_sep_off, "pack", 8)
    edge = float(np.asarray(inst.durations)[np.asarray(inst.durations) > 0].mean())
    _both(inst, P, 300, 1 / (0.005 * edge), 1.0, 17, window=32, types=2)
    small = synth.cvrp(120, 10, seed=6)
    P = _starts(small, 6, small.K - n_sep_off, "pack", 2)
    _both(small, P, 400, 1 / 5.0, 1.0, 19)


def _het(inst, fracs, starts=True):
    import dataclasses
    K = len(inst.capacities)
    base = int(inst.capacities[0])
    caps = np.array([max(int(base * fracs[k * len(fracs) // K]), int(inst.demand.max()))
                     for k in range(K)], dtype=np.int64)
    st = (np.arange(K, dtype=np.int64) * 37 % 240 + 420) if starts else inst.start_times
    return dataclasses.replace(inst, capacities=caps, start_times=st)


@pytest.mark.parametrize("hot", [False, True])
def test_resync_heterogeneous_td(hot):
    """Hour-indexed TD-200 x 24 with staggered start times and three capacity
    classes (the reference's request shape, api/parameters.py:11-12): the walk
    re-synchronises only on the same vehicle; same trajectories as the full
    walk."""
    inst = _het(synth.td_cvrp(200, 16, seed=3), (1.3, 1.0, 0.8))
    P = _starts(inst, 4, inst.K - 1, "pack", 2)
    _both(inst, P, 200, 1 / (1e6 if hot else 60.0), 1 / 0.99, 5, window=16, types=2)


def test_resync_heterogeneous_static_full_range():
    inst = _het(synth.cvrp(150, 12, seed=4, slack=1.2), (1.4, 0.9), starts=False)
    P = _starts(inst, 4, inst.K - 1, "random", 3)
    _both(inst, P, 300, 1 / 80.0, 1 / 0.99, 6)
