"""Spec oracle for the vrpms solver hot path -- TEST INFRASTRUCTURE ONLY.

This module is the CPU restatement that the HIP library is checked against.
Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s
``cpu_baseline`` leg may import it; the product path (``vrpms_amd``) never
does, and fails loudly when its HIP library is missing.

What the reference pins and what it does not
--------------------------------------------
The reference snapshot (metehkaya/vrpms) ships no cost function: every
algorithm endpoint stops at ``# TODO: Run algorithm``
(``api/vrp/ga/index.py:48-53``, ``api/tsp/ga/index.py:40-44`` and the six
siblings) and ``src/solver.py:7-27`` is a random stub.  Cost arithmetic is
therefore **parity unpinned by the reference**; this file freezes the
build-defined semantic spec of SURVEY.md Appendix A (A1-A9), each function
citing the reference line that motivates it.  What *is* pinned by the
reference (parameter schema, ``remove_unused_locations``, entry-point return
shapes) is captured as golden fixtures under ``tests/golden/`` by
``tests/golden/gen_reference_fixtures.py``.  Philox4x32-10 is pinned by the
published Random123 known-answer vectors (``tests/test_oracle.py``).

Everything here is integer arithmetic on Python ints / int64 numpy arrays
(no overflow possible at the sizes the host guard admits, A9).
"""
from __future__ import annotations

import numpy as np

# ----------------------------------------------------------------------------
# A8: objective key
# ----------------------------------------------------------------------------
KEY_FIELD_BITS = 28
KEY_CLAMP = (1 << KEY_FIELD_BITS) - 1
UNV_CLAMP = 255
OBJ_SUM = 0   # primary = durationSum, secondary = durationMax
OBJ_MAX = 1   # primary = durationMax, secondary = durationSum


def pack_key(unvisited: int, primary: int, secondary: int) -> int:
    """A8: ``unv<<56 | min(P,2^28-1)<<28 | min(S,2^28-1)``; smaller is better.

    Anchor: SURVEY.md Appendix A8 (north-star DPP min-reduction); the fields
    come from ``src/solver.py:27`` (``total_time``, ``unvisited``).
    """
    return (min(int(unvisited), UNV_CLAMP) << 56) | (min(int(primary), KEY_CLAMP) << 28) \
        | min(int(secondary), KEY_CLAMP)


def pack_key_np(unv, primary, secondary):
    u = np.minimum(unv.astype(np.uint64), np.uint64(UNV_CLAMP))
    p = np.minimum(primary.astype(np.uint64), np.uint64(KEY_CLAMP))
    s = np.minimum(secondary.astype(np.uint64), np.uint64(KEY_CLAMP))
    return (u << np.uint64(56)) | (p << np.uint64(28)) | s


def unpack_key(key: int):
    key = int(key)
    return key >> 56, (key >> 28) & KEY_CLAMP, key & KEY_CLAMP


# ----------------------------------------------------------------------------
# A3: time-dependent edge lookup
# ----------------------------------------------------------------------------
def hour_index(t: int, H: int) -> int:
    """A3: slice used for an edge departing at minute t: ``(t // 60) % H``.

    H = 1 is the static matrix, H = 24 the hour-indexed one.  Anchor:
    ``src/solver.py:7`` (``time_of_day`` argument of ``calculate_duration``).
    """
    return (t // 60) % H


def as_3d(D) -> np.ndarray:
    """A3: ``[N][N]`` (static) or ``[H][N][N]`` (hour-indexed) -> int64 [H][N][N]."""
    a = np.asarray(D, dtype=np.int64)
    if a.ndim == 2:
        a = a[None]
    if a.ndim != 3 or a.shape[1] != a.shape[2]:
        raise ValueError("duration matrix must be [N][N] or [H][N][N]")
    return a


# ----------------------------------------------------------------------------
# A4: TSP closed tour
# ----------------------------------------------------------------------------
def eval_tsp(D, perm, start_time: int = 0) -> int:
    """A4: duration of the closed tour ``0 -> perm... -> 0`` starting at
    ``start_time``; node 0 is the (compacted) ``startNode``.

    Anchors: ``api/parameters.py:41-43`` (customers/startNode/startTime),
    ``src/solver.py:24`` (closed tour), result key ``duration`` at
    ``api/tsp/ga/index.py:41-44``.
    """
    D = as_3d(D)
    H = D.shape[0]
    t = int(start_time)
    prev = 0
    for c in perm:
        c = int(c)
        t += int(D[hour_index(t, H), prev, c])
        prev = c
    t += int(D[hour_index(t, H), prev, 0])
    return t - int(start_time)


def eval_tsp_batch(D, perms, start_time: int = 0) -> np.ndarray:
    """Vectorised A4 over candidates (rows of ``perms``)."""
    D = as_3d(D)
    H = D.shape[0]
    perms = np.asarray(perms, dtype=np.int64)
    C, n = perms.shape
    t = np.full(C, int(start_time), dtype=np.int64)
    prev = np.zeros(C, dtype=np.int64)
    for i in range(n):
        c = perms[:, i]
        t = t + D[(t // 60) % H, prev, c]
        prev = c
    t = t + D[(t // 60) % H, prev, 0]
    return t - int(start_time)


def tsp_key(duration: int) -> int:
    """A8 for TSP: primary = duration, no secondary, never unvisited."""
    return pack_key(0, duration, 0)


# ----------------------------------------------------------------------------
# A5-A7: CVRP greedy split of a giant tour
# ----------------------------------------------------------------------------
def eval_cvrp(D, perm, demand, capacities, start_times, objective: int = OBJ_SUM):
    """A6/A7 greedy capacity split, returning the full decoded solution.

    Walk the giant tour; customer c joins vehicle k while
    ``load + demand[c] <= cap[k]``.  Otherwise vehicle k returns to the depot
    (an empty vehicle is simply skipped: tour [0,0], duration 0) and k+1
    opens at ``start_times[k+1]``; c is retried on it.  Customers reached
    after all K vehicles are closed are unvisited.  Route duration = arrival
    back at depot - start_times[k] (A7).

    A10 (route separators): the token 0 (the depot) may appear in the tour
    any number of times; it closes vehicle k's route (an empty route has
    duration 0) and opens vehicle k+1, exactly like a customer that does
    not fit, but is not itself a customer: once all K vehicles are closed
    later separators change nothing and are never counted as unvisited.

    Anchors: ``api/parameters.py:11-12`` (capacities, startTimes),
    ``src/solver.py:27`` (``unvisited``), result keys at
    ``api/vrp/ga/index.py:49-53``, vehicles payload at
    ``api/database.py:73-76``; A10: ``src/solver.py:24`` (the depot 0 inside
    the returned ``tour`` list marks route boundaries).
    Returns dict(sum, max, unvisited, key, routes, durations, vehicle_of)
    where ``vehicle_of[i]`` is the vehicle of tour position i, -1 when the
    customer is unvisited, -2 for a separator.
    """
    D = as_3d(D)
    H = D.shape[0]
    dem = [int(x) for x in demand]
    cap = [int(x) for x in capacities]
    st = [int(x) for x in start_times]
    K = len(cap)
    routes = [[] for _ in range(K)]
    durs = [0] * K
    vehicle_of = []
    k, load, prev = 0, 0, 0
    t = st[0] if K else 0
    unv = 0

    def close(k, t, prev):
        if prev != 0:
            t += int(D[hour_index(t, H), prev, 0])
            durs[k] = t - st[k]

    for c in perm:
        c = int(c)
        if c == 0:                      # A10: separator
            vehicle_of.append(-2)
            if k < K:
                close(k, t, prev)
                k += 1
                if k < K:
                    load, t, prev = 0, st[k], 0
            continue
        while k < K and load + dem[c] > cap[k]:
            close(k, t, prev)
            k += 1
            if k < K:
                load, t, prev = 0, st[k], 0
        if k >= K:
            unv += 1
            vehicle_of.append(-1)
            continue
        t += int(D[hour_index(t, H), prev, c])
        load += dem[c]
        prev = c
        routes[k].append(c)
        vehicle_of.append(k)
    if k < K:
        close(k, t, prev)
    dsum = sum(durs)
    dmax = max(durs) if durs else 0
    if objective == OBJ_SUM:
        key = pack_key(unv, dsum, dmax)
    else:
        key = pack_key(unv, dmax, dsum)
    return dict(sum=dsum, max=dmax, unvisited=unv, key=key,
                routes=routes, durations=durs, vehicle_of=vehicle_of)


def eval_cvrp_batch(D, perms, demand, capacities, start_times, objective: int = OBJ_SUM):
    """Vectorised A6/A7 (+ A10 separators) over candidates; returns (keys
    u64, sums, maxs, unv)."""
    D = as_3d(D)
    H = D.shape[0]
    perms = np.asarray(perms, dtype=np.int64)
    dem = np.asarray(demand, dtype=np.int64)
    cap = np.asarray(capacities, dtype=np.int64)
    st = np.asarray(start_times, dtype=np.int64)
    K = cap.shape[0]
    C, n = perms.shape
    k = np.zeros(C, dtype=np.int64)
    load = np.zeros(C, dtype=np.int64)
    prev = np.zeros(C, dtype=np.int64)
    t = np.full(C, st[0] if K else 0, dtype=np.int64)
    unv = np.zeros(C, dtype=np.int64)
    dsum = np.zeros(C, dtype=np.int64)
    dmax = np.zeros(C, dtype=np.int64)

    def close(mask):
        nonlocal dsum, dmax
        has = mask & (prev != 0)
        kk = np.minimum(k, K - 1)
        tc = t + D[(t // 60) % H, prev, 0]
        rd = np.where(has, tc - st[kk], 0)
        dsum = dsum + rd
        dmax = np.maximum(dmax, rd)

    def advance(act):
        nonlocal k, load, t, prev
        k = np.where(act, k + 1, k)
        kk = np.minimum(k, K - 1)
        load = np.where(act, 0, load)
        t = np.where(act, st[kk], t)
        prev = np.where(act, 0, prev)

    for i in range(n):
        c = perms[:, i]
        sep = c == 0
        act = sep & (k < K)                     # A10: separators close the route
        close(act)
        advance(act)
        while True:
            act = ~sep & (k < K) & (load + dem[c] > cap[np.minimum(k, K - 1)])
            if not act.any():
                break
            close(act)
            advance(act)
        ok = ~sep & (k < K)
        unv = unv + (~sep & ~ok)
        step = D[(t // 60) % H, prev, c]
        t = np.where(ok, t + step, t)
        load = np.where(ok, load + dem[c], load)
        prev = np.where(ok, c, prev)
    close(k < K)
    if objective == OBJ_SUM:
        keys = pack_key_np(unv, dsum, dmax)
    else:
        keys = pack_key_np(unv, dmax, dsum)
    return keys, dsum, dmax, unv


# ----------------------------------------------------------------------------
# A9: host overflow guard
# ----------------------------------------------------------------------------
def fits_int32(D, n: int, K: int, start_times) -> bool:
    """A9: every device clock/accumulator stays below 2^31."""
    D = as_3d(D)
    mx = int(D.max()) if D.size else 0
    s = max([int(x) for x in start_times] + [0])
    return s + (n + K + 1) * mx < (1 << 31)


# ----------------------------------------------------------------------------
# Philox4x32-10 (Salmon et al., SC'11; Random123 v1.09 constants)
# ----------------------------------------------------------------------------
PHILOX_M0 = 0xD2511F53
PHILOX_M1 = 0xCD9E8D57
PHILOX_W0 = 0x9E3779B9
PHILOX_W1 = 0xBB67AE85
MASK32 = 0xFFFFFFFF


def philox4x32_10(ctr, key):
    """Counter-based RNG; pinned by the Random123 KAT vectors in the tests."""
    c0, c1, c2, c3 = (int(x) & MASK32 for x in ctr)
    k0, k1 = (int(x) & MASK32 for x in key)
    for r in range(10):
        if r:
            k0 = (k0 + PHILOX_W0) & MASK32
            k1 = (k1 + PHILOX_W1) & MASK32
        p0 = PHILOX_M0 * c0
        p1 = PHILOX_M1 * c2
        c0, c1, c2, c3 = (((p1 >> 32) ^ c1 ^ k0) & MASK32, p1 & MASK32,
                          ((p0 >> 32) ^ c3 ^ k1) & MASK32, p0 & MASK32)
    return c0, c1, c2, c3


def seed_key(seed: int):
    """64-bit seed -> Philox key words."""
    seed = int(seed) & ((1 << 64) - 1)
    return seed & MASK32, seed >> 32


# ----------------------------------------------------------------------------
# Neighbourhood moves on a giant tour (positions 0..n-1)
# ----------------------------------------------------------------------------
MOVE_SWAP = 0
MOVE_2OPT = 1
MOVE_RELOCATE = 2


def decode_move(r0: int, r1: int, r2: int, n: int):
    """Philox words -> (type, i, j), i != j; swap/2-opt canonicalised i < j."""
    typ = r0 % 3
    i = r1 % n
    j = r2 % (n - 1)
    if j >= i:
        j += 1
    if typ != MOVE_RELOCATE and i > j:
        i, j = j, i
    return typ, i, j


def decode_move1(x: int, n: int):
    """A13: one Philox word -> (type, i, j), the throughput kernel's move
    (vrpms_tsp_batch_sa: four SA steps per lane's Philox block, the
    acceptance draws from one block per chain, oracle/search.py).  The word is split
    by successive fixed-point multiplications: type = hi(3x), i = hi(n * f1)
    with f1 = lo(3x), j' = hi((n - 1) * f2) with f2 = lo(n * f1); j = j' + 1
    when j' >= i; swap / 2-opt canonicalised i < j."""
    x = int(x) & MASK32
    p = 3 * x
    typ, f1 = p >> 32, p & MASK32
    p = n * f1
    i, f2 = p >> 32, p & MASK32
    j = ((n - 1) * f2) >> 32
    if j >= i:
        j += 1
    if typ != MOVE_RELOCATE and i > j:
        i, j = j, i
    return typ, i, j


def decode_move_window(r0: int, r1: int, r2: int, n: int, window: int, types: int = 0):
    """A11: a move whose second position lies within `window` of the first
    (the neighbourhood SA samples on large tours).  window <= 0 or
    2 * window + 1 >= n: decode_move.  Else i = r1 % n, o = r2 % (2 window),
    d = o - window (o < window) or o - window + 1, j = i + d, reflected to
    i - d when outside [0, n); swap / 2-opt canonicalised i < j.

    A12: `types` (bit t for move type t; 0 = all) limits the window to some
    move types; a move of another type is drawn by decode_move.  Windowed
    2-opt with unrestricted swap / relocate keeps reversals short (they are
    priced by walking the reversed span) while customers still move
    anywhere in the tour."""
    types = types or 7
    if window <= 0 or 2 * window + 1 >= n or not (types >> (r0 % 3)) & 1:
        return decode_move(r0, r1, r2, n)
    typ = r0 % 3
    i = r1 % n
    o = r2 % (2 * window)
    d = o - window if o < window else o - window + 1
    j = i + d
    if j < 0 or j >= n:
        j = i - d
    if typ != MOVE_RELOCATE and i > j:
        i, j = j, i
    return typ, i, j


def insert_separators(perm, n_sep: int, demand, capacities):
    """The giant tour `perm` (customers only) with A10 separators at the
    route boundaries the greedy split (A6) places: a 0 goes where a customer
    does not fit and opens the next route (at most n_sep of them); the
    separators left over are appended.  Same cost as `perm` when the
    greedy split never runs out of vehicles; used for feasible SA starts."""
    dem = [int(x) for x in demand]
    cap = [int(x) for x in capacities]
    K = len(cap)
    out, load, used = [], 0, 0
    for c in perm:
        c = int(c)
        if used < n_sep and load > 0 and load + dem[c] > cap[min(used, K - 1)]:
            out.append(0)
            used += 1
            load = 0
        load += dem[c]
        out.append(c)
    return out + [0] * (n_sep - used)


def pack_separators(perm, n_sep: int, demand, capacities):
    """First-fit start: the customers of `perm`, in that order, each go to
    the first of n_sep + 1 routes with room for them (route b holds up to
    cap[min(b, K - 1)]; a customer that fits nowhere joins the last route),
    and the tour lists route 0, a separator, route 1, ... route n_sep, every
    route in `perm` order.  Exactly n_sep separators.  Unlike
    insert_separators (next fit) it packs a fleet with little spare capacity
    into K routes, so SA starts feasible where the greedy split of a random
    order runs out of vehicles."""
    dem = [int(x) for x in demand]
    cap = [int(x) for x in capacities]
    K = len(cap)
    B = n_sep + 1
    load = [0] * B
    bins = [[] for _ in range(B)]
    for c in perm:
        c = int(c)
        d = dem[c]
        b = next((b for b in range(B) if load[b] + d <= cap[min(b, K - 1)]), B - 1)
        load[b] += d
        bins[b].append(c)
    out = []
    for b in range(B):
        if b:
            out.append(0)
        out += bins[b]
    return out


def apply_move(perm, typ: int, i: int, j: int):
    """Return a new list with the move applied.

    swap(i<j): exchange; 2-opt(i<j): reverse p[i..j]; relocate(i,j): pop
    position i and insert it so that it lands at position j.
    """
    p = list(perm)
    if typ == MOVE_SWAP:
        p[i], p[j] = p[j], p[i]
    elif typ == MOVE_2OPT:
        p[i:j + 1] = p[i:j + 1][::-1]
    else:
        x = p.pop(i)
        p.insert(j, x)
    return p


def moved_index(q: int, typ: int, i: int, j: int) -> int:
    """Position in the ORIGINAL perm read at position q of the moved perm."""
    if typ == MOVE_SWAP:
        return j if q == i else (i if q == j else q)
    if typ == MOVE_2OPT:
        return i + j - q if i <= q <= j else q
    if i < j:
        if q < i or q > j:
            return q
        return i if q == j else q + 1
    if q < j or q > i:
        return q
    return i if q == j else q - 1
