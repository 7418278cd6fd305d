"""CPU tests of the spec oracle itself (pins it before it checks anything)."""
import itertools

import numpy as np
import pytest

from oracle import spec
from vrpms_amd import synth


# Random123 v1.09 kat_vectors, philox4x32 R=10 (the three published rows).
PHILOX_KAT = [
    ((0, 0, 0, 0), (0, 0), (0x6627E8D5, 0xE169C58D, 0xBC57AC4C, 0x9B00DBD8)),
    ((0xFFFFFFFF,) * 4, (0xFFFFFFFF,) * 2, (0x408F276D, 0x41C83B0E, 0xA20BC7C6, 0x6D5451FD)),
    ((0x243F6A88, 0x85A308D3, 0x13198A2E, 0x03707344), (0xA4093822, 0x299F31D0),
     (0xD16CFE09, 0x94FDCCEB, 0x5001E420, 0x24126EA1)),
]


@pytest.mark.parametrize("ctr,key,out", PHILOX_KAT)
def test_philox_known_answers(ctr, key, out):
    assert spec.philox4x32_10(ctr, key) == out


def test_key_packing_orders_lexicographically():
    assert spec.pack_key(0, 5, 7) < spec.pack_key(0, 6, 0)
    assert spec.pack_key(0, 2**28 + 5, 0) == spec.pack_key(0, 2**28 - 1, 0)  # clamp
    assert spec.pack_key(1, 0, 0) > spec.pack_key(0, 2**28 - 1, 2**28 - 1)
    assert spec.unpack_key(spec.pack_key(3, 11, 13)) == (3, 11, 13)
    assert spec.pack_key(300, 0, 0) >> 56 == 255


def test_tsp_hand_example():
    D = np.array([[0, 1, 10], [2, 0, 3], [20, 4, 0]])
    # 0 -> 1 -> 2 -> 0 = 1 + 3 + 20
    assert spec.eval_tsp(D, [1, 2]) == 24
    assert spec.eval_tsp(D, [2, 1]) == 10 + 4 + 2
    assert spec.eval_tsp(D, []) == 0


def test_td_hour_boundaries():
    # two slices: hour 0 costs 10, hour 1 costs 100 (H=2 cycles every 2h)
    D = np.zeros((2, 3, 3), dtype=np.int64)
    D[0] += 10
    D[1] += 100
    # start 45: 0->1 at t=45 (h0) +10 -> 55; 1->2 at 55 (h0) +10 -> 65; 2->0 at 65 (h1) +100
    assert spec.eval_tsp(D, [1, 2], start_time=45) == 120
    # start 60: +100 (h1) -> 160 (h0) +10 -> 170 (h0) +10 -> 180
    assert spec.eval_tsp(D, [1, 2], start_time=60) == 120
    # start 100: 100 (h1), 200 (h1), 300 (h1): three 100-minute legs
    assert spec.eval_tsp(D, [1, 2], start_time=100) == 300
    assert spec.hour_index(60 * 24 + 5, 24) == 0


def test_cvrp_hand_example_split_and_unvisited():
    N = 5
    D = np.arange(N * N).reshape(N, N) % 7 + 1
    np.fill_diagonal(D, 0)
    dem = [0, 2, 2, 3, 5]
    cap = [4, 4]
    st = [0, 10]
    r = spec.eval_cvrp(D, [1, 2, 3, 4], dem, cap, st)
    # v0: 1,2 (load 4); 3 does not fit -> close; v1: 3 (3); 4 (5) does not fit v1 -> close,
    # no vehicle left -> 4 unvisited
    assert r["routes"] == [[1, 2], [3]]
    assert r["vehicle_of"] == [0, 0, 1, -1]
    assert r["unvisited"] == 1
    d0 = D[0, 1] + D[1, 2] + D[2, 0]
    d1 = D[0, 3] + D[3, 0]
    assert r["durations"] == [d0, d1]
    assert r["sum"] == d0 + d1 and r["max"] == max(d0, d1)
    assert r["key"] == spec.pack_key(1, d0 + d1, max(d0, d1))


def test_cvrp_separators_close_routes():
    """A10: token 0 closes the current route and opens the next vehicle; an
    empty route has duration 0; after the K-th vehicle separators are ignored
    and never counted unvisited."""
    N = 5
    D = np.arange(N * N).reshape(N, N) % 7 + 1
    np.fill_diagonal(D, 0)
    dem = [0, 1, 1, 1, 1]
    r = spec.eval_cvrp(D, [1, 0, 2, 3, 0, 4], dem, [10, 10, 10], [0, 0, 0])
    assert r["routes"] == [[1], [2, 3], [4]]
    assert r["vehicle_of"] == [0, -2, 1, 1, -2, 2] and r["unvisited"] == 0
    assert r["durations"] == [D[0, 1] + D[1, 0], D[0, 2] + D[2, 3] + D[3, 0], D[0, 4] + D[4, 0]]
    # leading / doubled separators burn empty vehicles; later customers unvisited
    r = spec.eval_cvrp(D, [0, 1, 0, 0, 2, 3, 4], dem, [10, 10, 10], [0, 0, 0])
    assert r["routes"] == [[], [1], []] and r["unvisited"] == 3
    assert r["vehicle_of"] == [-2, 1, -2, -2, -1, -1, -1] and r["durations"][0] == 0
    # a separator after the fleet is exhausted changes nothing
    a = spec.eval_cvrp(D, [1, 2, 3, 0, 4], dem, [1, 1], [0, 0])
    b = spec.eval_cvrp(D, [1, 2, 3, 4], dem, [1, 1], [0, 0])
    assert (a["key"], a["unvisited"]) == (b["key"], b["unvisited"]) == (a["key"], 2)


def test_c_restatement_matches_python_spec_with_separators(coracle):
    for slack, S in [(0.9, 4), (1.2, 3), (1.5, 2)]:
        inst = synth.cvrp(15, 4, seed=2, slack=slack)
        rng = np.random.default_rng(S)
        P = np.array([rng.permutation(np.concatenate([np.arange(1, 16), np.zeros(S, dtype=int)]))
                      for _ in range(400)]).astype(np.uint8)
        for obj in (0, 1):
            ref = spec.eval_cvrp_batch(inst.durations, P, inst.demand, inst.capacities,
                                       inst.start_times, obj)
            got = coracle.eval_batch(inst.durations, P, inst.demand, inst.capacities,
                                     inst.start_times, 1, obj)
            for x, y in zip(ref, got):
                assert (np.asarray(x).astype(np.int64) == np.asarray(y).astype(np.int64)).all()
        for i in range(0, 400, 37):
            r = spec.eval_cvrp(inst.durations, P[i], inst.demand, inst.capacities,
                               inst.start_times, 1)   # ref: the last (objective 1) pass
            assert r["key"] == int(ref[0][i])


def test_cvrp_oversized_customer_skips_empty_vehicles():
    D = np.ones((4, 4), dtype=np.int64)
    np.fill_diagonal(D, 0)
    r = spec.eval_cvrp(D, [3, 1, 2], [0, 1, 1, 8], [5, 10, 5], [0, 0, 0])
    # 3 (d=8) skips vehicle 0 (empty, unused), rides vehicle 1; 1, 2 fit vehicle 1 too
    assert r["routes"] == [[], [3, 1, 2], []]
    assert r["durations"] == [0, 4, 0]
    assert r["unvisited"] == 0


def test_cvrp_time_dependent_start_times():
    D = np.zeros((24, 3, 3), dtype=np.int64)
    for h in range(24):
        D[h] = h + 1
        np.fill_diagonal(D[h], 0)
    r = spec.eval_cvrp(D, [1, 2], [0, 1, 1], [1, 1], [60, 600])
    # v0 leaves 60 (h1: +2) -> 62, back +2 = 4; v1 leaves 600 (h10: +11) ->611, back +11 = 22
    assert r["durations"] == [4, 22]


def test_scalar_batch_and_objective_agree():
    inst = synth.cvrp(25, 3, seed=3, slack=0.9)   # tight: unvisited customers appear
    P = synth.random_perms(200, inst.n, seed=1)
    for obj in (spec.OBJ_SUM, spec.OBJ_MAX):
        keys, s, m, u = spec.eval_cvrp_batch(inst.durations, P, inst.demand, inst.capacities,
                                             inst.start_times, obj)
        assert u.max() > 0
        for i in range(0, 200, 7):
            r = spec.eval_cvrp(inst.durations, P[i], inst.demand, inst.capacities,
                               inst.start_times, obj)
            assert (r["key"], r["sum"], r["max"], r["unvisited"]) == (keys[i], s[i], m[i], u[i])


def test_c_restatement_matches_python_spec(coracle):
    cases = [synth.tsp20(2), synth.cvrp(40, 4, seed=4, slack=0.95), synth.td_cvrp(30, 3, seed=5)]
    for inst in cases:
        P = synth.random_perms(300, inst.n, seed=9)
        if inst.problem == "tsp":
            d = spec.eval_tsp_batch(inst.durations, P, int(inst.start_times[0]))
            k, s, m, u = coracle.eval_batch(inst.durations, P, start_times=inst.start_times,
                                            problem=0)
            assert (s == d).all() and (m == d).all() and (u == 0).all()
            assert [int(x) for x in k] == [spec.tsp_key(int(x)) for x in d]
        else:
            for obj in (0, 1):
                ref = spec.eval_cvrp_batch(inst.durations, P, inst.demand, inst.capacities,
                                           inst.start_times, obj)
                got = coracle.eval_batch(inst.durations, P, inst.demand, inst.capacities,
                                         inst.start_times, 1, obj)
                for a, b in zip(ref, got):
                    assert (np.asarray(a).astype(np.int64) == np.asarray(b).astype(np.int64)).all()


@pytest.mark.parametrize("kind", ["cvrp", "td", "tsp"])
def test_c_sa_matches_python_replay(coracle, kind):
    from oracle import search
    inst = {"cvrp": synth.cvrp(11, 3, seed=2, slack=0.9), "td": synth.td_cvrp(9, 2, seed=3),
            "tsp": synth.tsp20(4)}[kind]
    if kind == "tsp":
        inst = synth.Instance("t9", inst.durations[:, :10, :10], None, None, np.array([0]), "tsp")
    P = synth.random_perms(2, inst.n, seed=11).astype(np.uint16)
    cur, best = P.copy(), P.copy()
    bk = np.full(2, 2**64 - 1, dtype=np.uint64)
    ck = coracle.sa_run(inst.durations, cur, best, bk, 15, 1 / 150.0, 1 / 0.95, 77, 5,
                        inst.demand, inst.capacities, inst.start_times,
                        problem=0 if kind == "tsp" else 1)
    sc = search.Scorer(inst.durations, inst.demand, inst.capacities, inst.start_times,
                       inst.problem)
    ref = search.sa_run(sc, P.tolist(), P.tolist(), [2**64 - 1] * 2, 77, 5, 15, 1 / 150.0,
                        1 / 0.95)
    assert cur.tolist() == ref[0] and [int(x) for x in ck] == ref[1]
    assert best.tolist() == ref[2] and [int(x) for x in bk] == ref[3]


def test_c_sa_windowed_with_separators_matches_python_replay(coracle):
    """A11 windowed moves on A10 separator tours: C == Python replay."""
    from oracle import search
    inst = synth.cvrp(30, 4, seed=6, slack=1.1)
    rng = np.random.default_rng(2)
    P = np.array([rng.permutation(np.concatenate([np.arange(1, 31), np.zeros(3, dtype=int)]))
                  for _ in range(2)]).astype(np.uint16)
    cur, best = P.copy(), P.copy()
    bk = np.full(2, 2**64 - 1, dtype=np.uint64)
    ck = coracle.sa_run(inst.durations, cur, best, bk, 12, 1 / 90.0, 1 / 0.97, 5, 2,
                        inst.demand, inst.capacities, inst.start_times, window=4)
    sc = search.Scorer(inst.durations, inst.demand, inst.capacities, inst.start_times)
    ref = search.sa_run(sc, P.tolist(), P.tolist(), [2**64 - 1] * 2, 5, 2, 12, 1 / 90.0,
                        1 / 0.97, window=4)
    assert cur.tolist() == ref[0] and [int(x) for x in ck] == ref[1]
    assert best.tolist() == ref[2] and [int(x) for x in bk] == ref[3]


def test_windowed_moves_stay_in_window():
    rng = np.random.default_rng(1)
    for _ in range(2000):
        n, W = int(rng.integers(12, 60)), int(rng.integers(1, 5))
        r = [int(x) for x in rng.integers(0, 2**32, size=3, dtype=np.uint64)]
        t, i, j = spec.decode_move_window(*r, n, W)
        assert i != j and 0 <= i < n and 0 <= j < n and abs(i - j) <= W
    assert spec.decode_move_window(5, 6, 7, 9, 4) == spec.decode_move(5, 6, 7, 9)


def test_insert_separators_keeps_the_greedy_cost():
    inst = synth.cvrp(40, 6, seed=3, slack=1.2)
    P = synth.random_perms(30, 40, seed=5)
    for p in P:
        t = spec.insert_separators(p, 5, inst.demand, inst.capacities)
        assert sorted(t) == [0] * 5 + list(range(1, 41))
        a = spec.eval_cvrp(inst.durations, p, inst.demand, inst.capacities, inst.start_times)
        b = spec.eval_cvrp(inst.durations, t, inst.demand, inst.capacities, inst.start_times)
        if a["unvisited"] == 0:
            assert (a["sum"], a["max"]) == (b["sum"], b["max"])


def test_pack_separators_first_fit():
    """First-fit start: every customer once, exactly n_sep separators, each
    route within its capacity whenever first fit finds room, routes in
    input order; X-1000's fleet (K = LB + 2) packs where next fit fails."""
    inst = synth.cvrp(40, 6, seed=3, slack=1.05)
    for p in synth.random_perms(20, 40, seed=6):
        t = spec.pack_separators(p, 5, inst.demand, inst.capacities)
        assert sorted(t) == [0] * 5 + list(range(1, 41))
        routes, cur = [], []
        for c in t + [0]:
            if c == 0:
                routes.append(cur)
                cur = []
            else:
                cur.append(c)
        assert len(routes) == 6
        pos = {int(c): i for i, c in enumerate(p)}
        for r in routes:
            assert [pos[c] for c in r] == sorted(pos[c] for c in r)
        loads = [sum(int(inst.demand[c]) for c in r) for r in routes]
        assert all(x <= int(inst.capacities[0]) for x in loads[:-1])
    x = synth.x_style(1000, seed=0)
    p = synth.random_perms(1, 1000, seed=1, dtype=np.uint16)[0]
    packed = spec.eval_cvrp(x.durations, spec.pack_separators(p, x.K - 1, x.demand, x.capacities),
                            x.demand, x.capacities, x.start_times)
    greedy = spec.eval_cvrp(x.durations, spec.insert_separators(p, x.K - 1, x.demand,
                                                                x.capacities),
                            x.demand, x.capacities, x.start_times)
    assert packed["unvisited"] == 0 and greedy["unvisited"] > 0


def test_window_types_limit_the_window():
    """A12: only the move types in the mask are windowed."""
    rng = np.random.default_rng(4)
    n, W = 200, 5
    seen = set()
    for _ in range(3000):
        r = [int(v) for v in rng.integers(0, 2**32, size=3)]
        t, i, j = spec.decode_move_window(*r, n, W, 2)
        seen.add(t)
        if t == 1:
            assert 1 <= abs(i - j) <= W
        else:
            assert (t, i, j) == spec.decode_move(*r, n)
        assert spec.decode_move_window(*r, n, W, 0) == spec.decode_move_window(*r, n, W, 7)
    assert seen == {0, 1, 2}


def test_c_sa_window_types_matches_python_replay(coracle):
    """A12 (windowed 2-opt only) on separator tours: C == Python replay."""
    from oracle import search
    inst = synth.cvrp(36, 5, seed=8, slack=1.1)
    rng = np.random.default_rng(3)
    P = np.array([rng.permutation(np.concatenate([np.arange(1, 37), np.zeros(4, dtype=int)]))
                  for _ in range(2)]).astype(np.uint16)
    cur, best = P.copy(), P.copy()
    bk = np.full(2, 2**64 - 1, dtype=np.uint64)
    ck = coracle.sa_run(inst.durations, cur, best, bk, 15, 1 / 90.0, 1 / 0.97, 9, 4,
                        inst.demand, inst.capacities, inst.start_times, window=3, window_types=2)
    sc = search.Scorer(inst.durations, inst.demand, inst.capacities, inst.start_times)
    ref = search.sa_run(sc, P.tolist(), P.tolist(), [2**64 - 1] * 2, 9, 4, 15, 1 / 90.0,
                        1 / 0.97, window=3, window_types=2)
    assert cur.tolist() == ref[0] and [int(x) for x in ck] == ref[1]
    assert best.tolist() == ref[2] and [int(x) for x in bk] == ref[3]


@pytest.mark.parametrize("kind", ["symmetric", "asymmetric"])
def test_c_tsp_batch_matches_python_replay(coracle, kind):
    """The C restatement of vrpms_tsp_batch_sa (used for the TSP-50 GPU
    parity test, where the pure-Python replay is too slow) == search.py."""
    from oracle import search
    rng = np.random.default_rng(6)
    mats = []
    for _ in range(3):
        if kind == "symmetric":
            mats.append(synth.random_symmetric(8, rng))
        else:
            m = rng.integers(3, 320, size=(8, 8))
            np.fill_diagonal(m, 0)
            mats.append(m)
    tours, keys = coracle.tsp_batch_sa(mats, 20, 1 / 60.0, 1 / 0.97, 31)
    rt, rk = search.tsp_batch_sa(mats, 20, 1 / 60.0, 1 / 0.97, 31)
    assert tours.tolist() == rt and [int(k) for k in keys] == rk


@pytest.mark.parametrize("kind", ["cvrp", "tsp"])
def test_c_bf_matches_python_replay(coracle, kind):
    from oracle import search
    if kind == "cvrp":
        inst = synth.cvrp(7, 3, seed=8, slack=0.9)
        kw = dict(demand=inst.demand, capacities=inst.capacities, start_times=inst.start_times)
    else:
        inst = synth.Instance("t7", synth.tsp20(1).durations[:, :8, :8], None, None,
                              np.array([0]), "tsp")
        kw = dict(start_times=inst.start_times, problem=0)
    sc = search.Scorer(inst.durations, inst.demand, inst.capacities, inst.start_times,
                       inst.problem)
    assert coracle.bf(inst.durations, 7, **kw) == search.bf(sc, 7)
    assert coracle.bf(inst.durations, 7, 33, 4000, **kw) == search.bf(sc, 7, 33, 4000)


def test_accept_threshold_tracks_exp():
    from oracle import search
    for dp in [1, 5, 37, 400, 2000]:
        for invT in [1e-3, 0.01, 0.05, 0.2]:
            want = int(2**24 * np.exp(-dp * np.float32(invT)))
            got = search.accept_threshold(dp, np.float32(invT))
            assert abs(got - want) <= 64 + want * 4e-6
    assert search.accept_threshold(0, 1.0) == 2**24
    assert search.accept_threshold(10**6, 1.0) == 0


def test_brute_force_small_tsp_matches_itertools():
    inst = synth.tsp20(7)
    D = inst.durations[0][:7, :7]
    best = min(spec.eval_tsp(D, p) for p in itertools.permutations(range(1, 7)))
    P = np.array(list(itertools.permutations(range(1, 7))), dtype=np.uint8)
    assert spec.eval_tsp_batch(D, P).min() == best


def test_moves_mapping_is_consistent():
    rng = np.random.default_rng(0)
    for _ in range(500):
        n = int(rng.integers(2, 12))
        p = list(range(n))
        r = [int(x) for x in rng.integers(0, 2**32, size=3, dtype=np.uint64)]
        t, i, j = spec.decode_move(*r, n)
        assert i != j and 0 <= i < n and 0 <= j < n
        q = spec.apply_move(p, t, i, j)
        assert sorted(q) == p
        assert [p[spec.moved_index(x, t, i, j)] for x in range(n)] == q


def test_overflow_guard():
    D = np.full((3, 3), 2**29)
    assert not spec.fits_int32(D, 2, 1, [0])
    assert spec.fits_int32(np.full((3, 3), 1000), 2, 1, [0])
