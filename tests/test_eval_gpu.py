"""GPU parity of batched scoring (vrpms_eval) against the spec oracle.

Bar: bit-exact keys, durationSum, durationMax and unvisited counts on the
same tours, for every kernel path (packed-LDS CVRP, staged TSP, generic
LDS/L2 tiers, H = 24 time-dependent) and the edge cases the spec defines.
"""
import numpy as np
import pytest

from oracle import spec
from vrpms_amd import synth

pytestmark = pytest.mark.gpu


def _torch():
    import torch
    return torch


def upload(ctx, P):
    torch = _torch()
    t = torch.from_numpy(P.view(np.int16) if P.dtype == np.uint16 else P)
    return t.to(ctx.dev)


def load(ctx, inst, objective=0):
    from vrpms_amd.core import CVRP, TSP
    if inst.problem == "tsp":
        ctx.set_instance(TSP, inst.durations, start_times=inst.start_times, objective=objective)
    else:
        ctx.set_instance(CVRP, inst.durations, inst.demand, inst.capacities, inst.start_times,
                         objective=objective)


def check_batch(ctx, coracle, inst, P, n=None, objective=0, expect_path=None):
    load(ctx, inst, objective)
    dP = upload(ctx, P)
    if expect_path is not None:
        assert ctx.eval_path(dP) == expect_path
    keys, sums, maxs, unv = ctx.eval(dP, n=n, with_parts=True)
    ref = coracle.eval_batch(inst.durations, P, inst.demand, inst.capacities, inst.start_times,
                             problem=0 if inst.problem == "tsp" else 1, objective=objective, n=n)
    got_k = keys.cpu().numpy().view(np.uint64)
    np.testing.assert_array_equal(got_k, ref[0])
    np.testing.assert_array_equal(sums.cpu().numpy(), ref[1])
    np.testing.assert_array_equal(maxs.cpu().numpy(), ref[2])
    np.testing.assert_array_equal(unv.cpu().numpy(), ref[3])
    # and a few rows straight against the pure-Python spec
    for i in range(0, P.shape[0], max(1, P.shape[0] // 7)):
        row = P[i, : (P.shape[1] if n is None else n)]
        if inst.problem == "tsp":
            assert got_k[i] == spec.tsp_key(spec.eval_tsp(inst.durations, row,
                                                          int(inst.start_times[0])))
        else:
            r = spec.eval_cvrp(inst.durations, row, inst.demand, inst.capacities,
                               inst.start_times, objective)
            assert got_k[i] == r["key"]
    return got_k


# 0: auto (the words kernel tests fits by the add's carry when every demand
# is >= 1), 2: the branchy split, 3: the words kernel's sign-compare form
@pytest.fixture(params=[0, 2, 3], ids=["prefix_ret", "branchy", "prefix_ret_compare"])
def split_mode(request, ctx):
    ctx.set_split_mode(request.param)
    yield request.param
    ctx.set_split_mode(0)


@pytest.mark.parametrize("objective", [0, 1])
def test_cvrp100_packed_path(ctx, coracle, objective, split_mode):
    inst = synth.cvrp(100, 8, seed=0)
    P = synth.random_perms(20000 + 37, inst.n, seed=1)          # ragged last tile
    check_batch(ctx, coracle, inst, P, objective=objective, expect_path=0)


def test_cvrp_tight_capacity_unvisited(ctx, coracle, split_mode):
    inst = synth.cvrp(100, 8, seed=2, slack=0.85)
    P = synth.random_perms(5000, inst.n, seed=3)
    k = check_batch(ctx, coracle, inst, P, expect_path=0)
    assert (k >> np.uint64(56)).max() > 0


def test_cvrp_single_vehicle_and_oversized_first(ctx, coracle, split_mode):
    inst = synth.cvrp(30, 1, seed=5, slack=0.5)            # K = 1: exhausts early
    P = synth.random_perms(3000, inst.n, seed=6, ld=32)
    check_batch(ctx, coracle, inst, P, n=inst.n, expect_path=0)
    inst = synth.cvrp(30, 4, seed=7)
    inst.demand[3] = int(inst.capacities[0]) + 1           # fits no vehicle at all
    P = synth.random_perms(3000, inst.n, seed=8, ld=32)
    P[:50, 0] = 3                                           # ... and sometimes comes first
    P[:50, 1:inst.n] = np.array([x for x in range(1, inst.n + 1) if x != 3], dtype=np.uint8)
    check_batch(ctx, coracle, inst, P, n=inst.n, expect_path=0)


def test_cvrp_asymmetric_matrix_prefix_ret(ctx, coracle, split_mode):
    # asymmetric durations: dur(a,b) + ret(b) - ret(a) goes negative often
    rng = np.random.default_rng(3)
    N = 70
    D = rng.integers(0, 3000, size=(N, N))
    np.fill_diagonal(D, 0)
    D[:, 0] = rng.integers(2000, 3000, size=N)              # expensive returns
    D[0, 0] = 0
    dem = np.concatenate([[0], rng.integers(1, 30, N - 1)])
    inst = synth.Instance("asym", D[None], dem, np.full(6, 200), np.zeros(6, dtype=np.int64),
                          "cvrp")
    P = synth.random_perms(6000, inst.n, seed=4, ld=72)
    check_batch(ctx, coracle, inst, P, n=inst.n, expect_path=0)


@pytest.fixture
def words_gen(ctx):
    """Reset the LDS-packed kernel generation after a test forces one."""
    yield ctx
    ctx.set_words_kernel(0)
    ctx.set_rows_config(0)
    ctx.set_words_ilp(0)
    ctx.set_words_lookahead(0)


# eval_cvrp_rows2 (row-major tiles staged through LDS) in every (CW, ILP)
# configuration that fits, against eval_cvrp_packed and the oracle: N <= 101
# (all five fit), N = 111 (the ILP-2 CW-8 tile no longer fits), ragged
# tiles, short tours, and N = 121 where no tile fits next to the matrix
# (falls back to eval_cvrp_packed).
@pytest.mark.parametrize("n,K,ld,C", [(100, 8, 100, 20037), (97, 7, 100, 5000), (30, 3, 32, 4099),
                                      (5, 2, 8, 3000), (110, 9, 112, 5000), (120, 10, 120, 6000)])
def test_rows2_matches_packed_and_oracle(words_gen, coracle, n, K, ld, C):
    from vrpms_amd.core import VrpmsError
    ctx = words_gen
    inst = synth.cvrp(n, K, seed=n)
    P = synth.random_perms(C, inst.n, seed=K, ld=ld)
    ctx.set_words_kernel(1)         # eval_cvrp_packed
    ref = check_batch(ctx, coracle, inst, P, n=inst.n, objective=n % 2, expect_path=0)
    ctx.set_words_kernel(0)
    for cfg in range(6):            # auto, then every forced (CW, ILP)
        ctx.set_rows_config(cfg)
        try:
            got = check_batch(ctx, coracle, inst, P, n=inst.n, objective=n % 2, expect_path=0)
        except VrpmsError as e:     # a forced tile that does not fit is refused, never wrong
            assert cfg > 0 and "does not fit" in str(e)
            continue
        np.testing.assert_array_equal(got, ref)


@pytest.mark.parametrize("ilp,la", [(2, 1), (2, 2)])
def test_words2_ilp_variants(words_gen, coracle, ilp, la):
    ctx = words_gen
    ctx.set_words_ilp(ilp)
    ctx.set_words_lookahead(la)
    inst = synth.cvrp(100, 8, seed=11)
    check_words(ctx, coracle, inst, synth.random_perms(4097, inst.n, seed=ilp), inst.n)


def check_words(ctx, coracle, inst, P, n, objective=0):
    """Same tours through the word-interleaved layout (vrpms_eval_words)."""
    load(ctx, inst, objective)
    words = ctx.to_words(upload(ctx, P), n=n)
    keys, sums, maxs, unv = ctx.eval_words(words, n, with_parts=True)
    ref = coracle.eval_batch(inst.durations, P, inst.demand, inst.capacities, inst.start_times,
                             problem=1, objective=objective, n=n)
    np.testing.assert_array_equal(keys.cpu().numpy().view(np.uint64), ref[0])
    np.testing.assert_array_equal(sums.cpu().numpy(), ref[1])
    np.testing.assert_array_equal(maxs.cpu().numpy(), ref[2])
    np.testing.assert_array_equal(unv.cpu().numpy(), ref[3])


@pytest.mark.parametrize("C", [1, 1023, 70001])
def test_words_layout_cvrp100(ctx, coracle, C):
    inst = synth.cvrp(100, 8, seed=0)
    check_words(ctx, coracle, inst, synth.random_perms(C, inst.n, seed=C), inst.n)


@pytest.mark.parametrize("n,K,slack", [(29, 1, 0.5), (37, 4, 0.9), (5, 2, 1.0), (64, 8, 0.8),
                                       (100, 8, 1.03), (100, 8, 1.05), (101, 8, 1.0)])
def test_words_layout_ragged_and_tight(ctx, coracle, n, K, slack, split_mode):
    inst = synth.cvrp(n, K, seed=n, slack=slack)
    P = synth.random_perms(20000, inst.n, seed=1)
    check_words(ctx, coracle, inst, P, inst.n, objective=n % 2)


def test_words_layout_zero_demands_asymmetric(ctx, coracle, split_mode):
    """Zero-demand customers on an asymmetric matrix: an edge term
    dur(a,b) + ret(b) - ret(a) below 0 with no demand above it would carry
    on a fit, so the carry form is not used (FastSplit::carry); keys still
    equal the oracle's, with and without zero demands."""
    rng = np.random.default_rng(12)
    N = 90
    D = rng.integers(0, 3000, size=(N, N))
    np.fill_diagonal(D, 0)
    D[:, 0] = rng.integers(2000, 3000, size=N)
    D[0, 0] = 0
    dem = np.concatenate([[0], rng.integers(1, 30, N - 1)])
    for zeros in (False, True):
        d = dem.copy()
        if zeros:
            d[1::5] = 0
        inst = synth.Instance("asym0", D[None], d, np.full(7, 180), np.zeros(7, dtype=np.int64),
                              "cvrp")
        check_words(ctx, coracle, inst, synth.random_perms(12000, inst.n, seed=5), inst.n)


def test_words_layout_oversize_and_fallbacks(ctx, coracle):
    inst = synth.cvrp(40, 4, seed=7)
    inst.demand[3] = int(inst.capacities[0]) + 1            # OVS variant of the fast kernel
    check_words(ctx, coracle, inst, synth.random_perms(9000, inst.n, seed=2), inst.n)
    het = synth.cvrp(60, 6, seed=4)
    het.capacities = np.array([40, 5, 90, 30, 7, 60])        # generic fallback, words access
    check_words(ctx, coracle, het, synth.random_perms(5000, het.n, seed=3), het.n)
    td = synth.td_cvrp(30, 3, seed=3)                        # H = 24 through words
    check_words(ctx, coracle, td, synth.random_perms(5000, td.n, seed=4), td.n)


def test_cvrp_heterogeneous_fleet_and_oversized_demand(ctx, coracle):
    inst = synth.cvrp(60, 6, seed=4)
    inst.capacities = np.array([40, 5, 90, 30, 7, 60])
    inst.demand[5] = 80                        # only vehicle 2 can ever carry it
    inst.start_times = np.array([0, 5, 10, 0, 3, 9])
    P = synth.random_perms(4096, inst.n, seed=5)
    check_batch(ctx, coracle, inst, P, expect_path=0)


def test_cvrp_generic_path_unaligned_ld(ctx, coracle):
    inst = synth.cvrp(50, 5, seed=6)
    P = synth.random_perms(3000, inst.n, seed=7, ld=inst.n + 1)    # ld % 4 != 0
    check_batch(ctx, coracle, inst, P, n=inst.n, expect_path=2)


def test_cvrp_uint16_tours(ctx, coracle):
    inst = synth.cvrp(100, 8, seed=8)
    P = synth.random_perms(3000, inst.n, seed=9, dtype=np.uint16)
    check_batch(ctx, coracle, inst, P, expect_path=2)


def test_tdvrp200_l2_tier(ctx, coracle):
    inst = synth.td_cvrp(200, 16, seed=0)
    P = synth.random_perms(8192, inst.n, seed=2)
    check_batch(ctx, coracle, inst, P, expect_path=2)


def test_tdvrp_small_lds_tier(ctx, coracle):
    inst = synth.td_cvrp(20, 3, seed=3)       # 24 x 21 x 21 x 2 B fits the LDS tier
    P = synth.random_perms(4000, inst.n, seed=4)
    check_batch(ctx, coracle, inst, P, expect_path=2)


def test_max_uint8_instance(ctx, coracle):
    """N = 256, the largest instance uint8 tours can name (255 customers):
    row-major and word-interleaved layouts, ragged batch."""
    inst = synth.cvrp(255, 20, seed=9)
    P = synth.random_perms(3001, inst.n, seed=2)
    check_batch(ctx, coracle, inst, P, expect_path=2)
    check_words(ctx, coracle, inst, P, inst.n)


def test_x1000_l2_tier(ctx, coracle):
    inst = synth.x_style(1000, seed=0)
    P = synth.random_perms(2048, inst.n, seed=1, dtype=np.uint16)
    check_batch(ctx, coracle, inst, P, expect_path=2)


@pytest.mark.parametrize("maker", [synth.tsp20, synth.tsp50])
def test_tsp_staged_path(ctx, coracle, maker):
    inst = maker(3)
    ld = (inst.n + 3) // 4 * 4
    P = synth.random_perms(10000 + 5, inst.n, seed=5, ld=ld)
    check_batch(ctx, coracle, inst, P, n=inst.n, expect_path=1)


def test_tsp_time_dependent(ctx, coracle):
    base = synth.td_cvrp(30, 2, seed=1)
    inst = synth.Instance("tdtsp", base.durations, None, None, np.array([415]), "tsp")
    P = synth.random_perms(3000, inst.n, seed=6)
    check_batch(ctx, coracle, inst, P, expect_path=2)


def test_large_matrix_int32_values(ctx, coracle):
    rng = np.random.default_rng(0)
    N = 40
    D = rng.integers(60000, 900000, size=(N, N))         # > 65535: int32 matrix path
    np.fill_diagonal(D, 0)
    inst = synth.Instance("big", D[None], np.concatenate([[0], rng.integers(1, 9, N - 1)]),
                          np.array([60, 60, 60, 60]), np.zeros(4, dtype=np.int64), "cvrp")
    P = synth.random_perms(2000, inst.n, seed=1)
    check_batch(ctx, coracle, inst, P)


def test_empty_batch_and_zero_length_tours(ctx, coracle):
    torch = _torch()
    inst = synth.cvrp(10, 2, seed=1)
    load(ctx, inst)
    empty = torch.zeros((0, 12), dtype=torch.uint8, device=ctx.dev)
    assert ctx.eval(empty).numel() == 0
    P = np.zeros((5, 4), dtype=np.uint8)
    k = ctx.eval(upload(ctx, P), n=0).cpu().numpy().view(np.uint64)
    assert (k == 0).all()


def test_decode_matches_spec_routes(ctx):
    for inst in (synth.cvrp(100, 8, seed=3, slack=0.9), synth.td_cvrp(40, 4, seed=2)):
        load(ctx, inst)
        P = synth.random_perms(4, inst.n, seed=11)
        for row in P:
            veh, dur = ctx.decode(upload(ctx, row[None]))
            r = spec.eval_cvrp(inst.durations, row, inst.demand, inst.capacities,
                               inst.start_times)
            assert veh == r["vehicle_of"]
            assert dur == r["durations"]


def test_argmin(ctx):
    torch = _torch()
    rng = np.random.default_rng(0)
    keys = rng.integers(0, 2**62, size=100003, dtype=np.int64)
    keys[[777, 5000, 99999]] = 3
    best, idx = ctx.argmin(torch.from_numpy(keys).to(ctx.dev))
    assert (best, idx) == (3, 777)


def test_errors_are_raised(ctx):
    from vrpms_amd.core import CVRP, VrpmsError
    D = np.ones((5, 5), dtype=np.int64)
    D[1, 2] = -1
    with pytest.raises(VrpmsError, match="negative duration"):
        ctx.set_instance(CVRP, D, [0, 1, 1, 1, 1], [3], [0])
    with pytest.raises(VrpmsError, match="A9"):
        ctx.set_instance(CVRP, np.full((5, 5), 2**29), [0, 1, 1, 1, 1], [3], [0])


# The headline kernels walk the split without the fleet-exhaustion test and
# re-walk exactly the lanes whose vehicle counter met the fleet limit
# (eval_words.hip split_step_fast / redo_exact): waves where some lanes
# exhaust and others do not, on every ILP / look-ahead variant and on the
# row-major kernel, against the oracle.
@pytest.mark.parametrize("ilp,la", [(2, 1), (2, 2)])
@pytest.mark.parametrize("slack", [1.03, 0.9])
def test_words2_mixed_exhaustion(words_gen, coracle, ilp, la, slack):
    ctx = words_gen
    ctx.set_words_ilp(ilp)
    ctx.set_words_lookahead(la)
    inst = synth.cvrp(100, 8, seed=12, slack=slack)
    check_words(ctx, coracle, inst, synth.random_perms(8191, inst.n, seed=ilp + 2 * la), inst.n,
                objective=la - 1)


@pytest.mark.parametrize("n,ld,slack", [(100, 100, 1.03), (97, 100, 0.95), (30, 32, 0.7)])
def test_rows2_mixed_exhaustion(words_gen, coracle, n, ld, slack):
    ctx = words_gen
    inst = synth.cvrp(n, 8 if n > 50 else 3, seed=n + 1, slack=slack)
    P = synth.random_perms(6001, inst.n, seed=3, ld=ld)
    for cfg in range(6):
        ctx.set_rows_config(cfg)
        check_batch(ctx, coracle, inst, P, n=inst.n, expect_path=0)
