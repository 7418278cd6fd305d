"""CPU replay of the search kernels -- TEST INFRASTRUCTURE ONLY.

The reference exposes SA / GA / ACO / BF endpoints (api/{tsp,vrp}/{sa,ga,
aco,bf}/index.py) whose algorithm slot is `# TODO: Run algorithm`
(e.g. api/vrp/sa/index.py:40-45, api/vrp/ga/index.py:48-53); the knobs it
declares are the GA's (api/parameters.py:18-23).  The build therefore
defines the algorithms (SURVEY.md §8a'); this module restates them
step-for-step from the same Philox streams so the GPU trajectories are
checked exactly (parity unpinned by the reference; pinned to this spec).

Every tour is scored with oracle.spec (eval_tsp / eval_cvrp), i.e. the same
semantics the scoring kernels are checked against.
"""
from __future__ import annotations

import itertools

import numpy as np

from . import spec

M32 = 0xFFFFFFFF


class Scorer:
    """Key of a compact tour for an instance (TSP or CVRP)."""

    def __init__(self, durations, demand=None, capacities=None, start_times=(0,),
                 problem: str = "cvrp", objective: int = 0):
        self.D = spec.as_3d(durations)
        self.demand, self.capacities = demand, capacities
        self.start_times = [int(x) for x in start_times]
        self.problem, self.objective = problem, objective

    def __call__(self, tour) -> int:
        if self.problem == "tsp":
            return spec.tsp_key(spec.eval_tsp(self.D, tour, self.start_times[0]))
        return spec.eval_cvrp(self.D, tour, self.demand, self.capacities, self.start_times,
                              self.objective)["key"]


# ---------------------------------------------------------------------------
# SA acceptance: floor(2^24 * exp(-dp * invT)) with float32 steps identical
# to tour.hpp accept_threshold (no FMA; hex constants are the same floats).
# ---------------------------------------------------------------------------
_F = np.float32
_LOG2E = _F(float.fromhex("0x1.715476p+0"))
_LN2 = _F(float.fromhex("0x1.62e43p-1"))
_C720 = _F(float.fromhex("0x1.6c16c2p-10"))
_C120 = _F(float.fromhex("0x1.111112p-7"))
_C24 = _F(float.fromhex("0x1.555556p-5"))
_C6 = _F(float.fromhex("0x1.555556p-3"))


def accept_threshold(dp: int, invT) -> int:
    if dp == 0:
        return 1 << 24
    x = _F(_F(dp) * _F(invT))
    y = _F(x * _LOG2E)
    if not (y < _F(24.0)):
        return 0
    kf = _F(np.floor(y))
    f = _F(y - kf)
    g = _F(f * _LN2)
    p = _C720
    p = _F(p * g)
    p = _F(_C120 - p)
    p = _F(p * g)
    p = _F(_C24 - p)
    p = _F(p * g)
    p = _F(_C6 - p)
    p = _F(p * g)
    p = _F(_F(0.5) - p)
    p = _F(p * g)
    p = _F(_F(1.0) - p)
    p = _F(p * g)
    p = _F(_F(1.0) - p)
    k = int(kf)
    return int(_F(p * _F(1 << (24 - k))))


def sa_run(score: Scorer, cur_tours, best_tours, best_keys, seed: int, step0: int, steps: int,
           inv_t0: float, inv_alpha: float, window: int = 0, window_types: int = 0):
    """vrpms_sa_run: one chain per tour; returns (cur, cur_keys, best, best_keys).
    `window` > 0 samples A11 windowed moves (spec.decode_move_window) of the
    A12 types `window_types` (0 = all)."""
    key = spec.seed_key(seed)
    cur_out, ck_out, best_out, bk_out = [], [], [], []
    for c, cur in enumerate(cur_tours):
        cur = [int(x) for x in cur]
        n = len(cur)
        ck = score(cur)
        bk, best = int(best_keys[c]), [int(x) for x in best_tours[c]]
        if ck < bk:
            bk, best = ck, cur[:]
        invT = _F(inv_t0)
        if n >= 2:
            for s in range(steps):
                step = step0 + s
                cands = []
                for lane in range(64):
                    r = spec.philox4x32_10((step & M32, step >> 32, c, lane), key)
                    m = spec.decode_move_window(r[0], r[1], r[2], n, window, window_types)
                    cands.append((score(spec.apply_move(cur, *m)), lane, m, r[3]))
                kk, lane, m, r3 = min(cands, key=lambda t: (t[0], t[1]))
                acc = kk <= ck
                if not acc:
                    dp = min((kk >> 28) - (ck >> 28), M32)
                    acc = (r3 >> 8) < accept_threshold(dp, invT)
                if acc:
                    cur = spec.apply_move(cur, *m)
                    ck = kk
                    if ck < bk:
                        bk, best = ck, cur[:]
                invT = _F(invT * _F(inv_alpha))
        cur_out.append(cur)
        ck_out.append(ck)
        best_out.append(best)
        bk_out.append(bk)
    return cur_out, ck_out, best_out, bk_out


def tsp_batch_sa(mats, steps: int, inv_t0: float, inv_alpha: float, seed: int):
    """vrpms_tsp_batch_sa: per request 4 chains (Philox Fisher-Yates starts,
    counters (0xffffffff, 0xffffffff, 4r + w, i)); A13: one Philox block per
    lane with counters (s >> 2, 0, 4r + w, lane) serves four SA steps -- step
    s decodes its move from word s & 3 (spec.decode_move1) -- and the chain's
    acceptance draw of step s is word s & 3 of the block with counters
    (s >> 2, 1, 4r + w, 0), one per chain; best (key, wave).  Costs by full re-evaluation -- the device prices moves by O(1)
    deltas, so equality checks the deltas."""
    key = spec.seed_key(seed)
    out_t, out_k = [], []
    for r, D in enumerate(mats):
        D = np.asarray(D)
        n = D.shape[0] - 1
        score = Scorer(D, problem="tsp")
        best = None
        for w in range(4):
            cid = 4 * r + w
            t = list(range(1, n + 1))
            for i in range(n - 1, 0, -1):
                x = spec.philox4x32_10((M32, M32, cid, i), key)
                j = x[0] % (i + 1)
                t[i], t[j] = t[j], t[i]
            ck = score(t)
            bk, bt = ck, t[:]
            invT = _F(inv_t0)
            if n >= 2:
                for s in range(steps):
                    cands = []
                    for lane in range(64):
                        rr = spec.philox4x32_10((s >> 2, 0, cid, lane), key)
                        m = spec.decode_move1(rr[s & 3], n)
                        cands.append((score(spec.apply_move(t, *m)), lane, m))
                    kk, lane, m = min(cands, key=lambda c: (c[0], c[1]))
                    r3 = spec.philox4x32_10((s >> 2, 1, cid, 0), key)[s & 3]
                    acc = kk <= ck
                    if not acc:
                        dp = min((kk >> 28) - (ck >> 28), M32)
                        acc = (r3 >> 8) < accept_threshold(dp, invT)
                    if acc:
                        t = spec.apply_move(t, *m)
                        ck = kk
                        if ck < bk:
                            bk, bt = ck, t[:]
                    invT = _F(invT * _F(inv_alpha))
            if best is None or bk < best[0]:
                best = (bk, bt)
        out_k.append(best[0])
        out_t.append(best[1])
    return out_t, out_k


# ---------------------------------------------------------------------------
# GA: tournament(2) x 2, OX1, Philox-gated mutation, (mu + lambda) survivors
# ---------------------------------------------------------------------------
def _tourney(keys, pop, r0, r1):
    x, y = r0 % pop, r1 % pop
    return y if (keys[y] < keys[x] or (keys[y] == keys[x] and y < x)) else x


def ox1(A, B, lo, hi):
    n = len(A)
    out = [None] * n
    out[lo:hi + 1] = A[lo:hi + 1]
    used = set(A[lo:hi + 1])
    rest = n - (hi - lo + 1)
    filled = 0
    for q in range(n):
        g = B[(hi + 1 + q) % n]
        if g not in used:
            if filled < rest:
                out[(hi + 1 + filled) % n] = g
            filled += 1
    return out


def ga_generation(score: Scorer, pops, keys, seed: int, gen: int, pmut: int):
    """vrpms_ga_generation for one generation; pops[island][i] tours."""
    skey = spec.seed_key(seed)
    new_pops, new_keys = [], []
    for island, (P, K) in enumerate(zip(pops, keys)):
        pop = len(P)
        children = []
        for child in range(pop):
            cid = island * pop + child
            r = spec.philox4x32_10((gen & M32, gen >> 32, cid, 0), skey)
            r2 = spec.philox4x32_10((gen & M32, gen >> 32, cid, 1), skey)
            pa, pb = _tourney(K, pop, r[0], r[1]), _tourney(K, pop, r[2], r[3])
            A, B = list(P[pa]), list(P[pb])
            n = len(A)
            if n < 2:
                children.append(A)
                continue
            lo, hi = r2[0] % n, r2[1] % n
            if lo > hi:
                lo, hi = hi, lo
            out = ox1(A, B, lo, hi)
            if r2[2] < pmut:
                m = spec.decode_move(r2[3], r[0] ^ r2[0], r[1] ^ r2[1], n)
                out = spec.apply_move(out, *m)
            children.append(out)
        ck = [score(t) for t in children]
        merged = sorted([(int(K[i]), i) for i in range(pop)] + [(ck[i], pop + i) for i in range(pop)])
        sel = merged[:pop]
        new_pops.append([list(P[i]) if i < pop else children[i - pop] for _, i in sel])
        new_keys.append([k for k, _ in sel])
    return new_pops, new_keys


# ---------------------------------------------------------------------------
# Integer ACO
# ---------------------------------------------------------------------------
def aco_eta(D0) -> np.ndarray:
    d1 = 1 + np.asarray(D0, dtype=np.int64)
    return ((1 << 24) // (d1 * d1)).astype(np.int64)


def aco_iteration(score: Scorer, tau, eta, ants: int, n: int, seed: int, it: int,
                  evap_shift: int, tau_min: int, tau_max: int, best=None, bsf_period: int = 0):
    """tau: list (per colony) of int64 [N][N] arrays, updated in place.
    Returns (tours[colony][ant], keys[colony][ant], iter_best[(key, ant)]).

    best: optional (tours[colony], keys[colony]) best-so-far, updated in
    place when the iteration best is strictly better.  bsf_period > 0: on
    iterations with (it + 1) % bsf_period == 0 the colony's best-so-far
    (after that update) deposits instead of the iteration best (max-min ant
    system's global-best update; migrants injected into the best-so-far
    then shape the pheromone).  Anchor: api/vrp/aco/index.py:40-45."""
    skey = spec.seed_key(seed)
    N = eta.shape[0]
    all_tours, all_keys, ib = [], [], []
    for colony, T in enumerate(tau):
        tours = []
        for ant in range(ants):
            vis = np.zeros(N, dtype=bool)
            vis[0] = True
            cur, tour = 0, []
            for s in range(n):
                r = spec.philox4x32_10((it & M32, it >> 32, colony * ants + ant, s), skey)
                w = np.where(vis, 0, (T[cur] >> 8) * eta[cur])
                tot = int(w.sum())
                if tot == 0:
                    pick = int(np.flatnonzero(~vis)[0])
                else:
                    rr = ((r[1] << 32) | r[0]) % tot
                    cs = np.cumsum(w)
                    pick = int(np.flatnonzero((w > 0) & (cs > rr))[0])
                tour.append(pick)
                vis[pick] = True
                cur = pick
            tours.append(tour)
        keys = [score(t) for t in tours]
        b = min(range(ants), key=lambda a: (keys[a], a))
        ib.append((keys[b], b))
        dkey, t = keys[b], tours[b]
        if best is not None:
            if keys[b] < best[1][colony]:
                best[0][colony] = list(tours[b])
                best[1][colony] = keys[b]
            if bsf_period > 0 and (it + 1) % bsf_period == 0:
                dkey, t = best[1][colony], best[0][colony]
        T[:] = np.minimum(tau_max, np.maximum(tau_min, T - (T >> evap_shift)))
        primary = (dkey >> 28) & ((1 << 28) - 1)
        dep = (1 << 30) // (1 + primary)
        for q in range(n + 1):
            fr = 0 if q == 0 else t[q - 1]
            to = 0 if q == n else t[q]
            T[fr, to] = (int(T[fr, to]) + dep) & M32
        all_tours.append(tours)
        all_keys.append(keys)
    return all_tours, all_keys, ib


# ---------------------------------------------------------------------------
# Brute force over lexicographic ranks
# ---------------------------------------------------------------------------
def bf(score: Scorer, n: int, r0: int = 0, r1: int | None = None):
    best = (2**64 - 1, 2**64 - 1)
    for rank, p in enumerate(itertools.permutations(range(1, n + 1))):
        if rank < r0:
            continue
        if r1 is not None and rank >= r1:
            break
        k = score(p)
        if (k, rank) < best:
            best = (k, rank)
    return best


def unrank(rank: int, n: int):
    """Lexicographic rank -> permutation of 1..n."""
    avail = list(range(1, n + 1))
    out = []
    for i in range(n):
        f = 1
        for x in range(2, n - i):
            f *= x
        d, rank = divmod(rank, f)
        out.append(avail.pop(d))
    return out
