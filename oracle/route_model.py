"""Pure-Python model of sa_route_kernel's move pricing (route tables,
re-synchronising walks, two zones, composed key) -- TEST INFRASTRUCTURE.

It mirrors the kernel step for step so the composition rules can be
checked against oracle/spec.py eval_cvrp on many random moves on the CPU
(tests/test_route_model.py); the device kernel is then checked against the
C restatement on the GPU.  Exchangeable fleet only: one capacity, one start
time, every demand fits an empty vehicle.
"""
from __future__ import annotations

import numpy as np

from . import spec


class Tables:
    """Greedy-split routes of tour A with unlimited vehicles: rs (first
    position), dur, cus (holds a customer), rid (route of each position).

    D: [N][N] static or [H][N][N] hour-indexed (A3).  cap / st0: one value
    (an exchangeable fleet) or one per vehicle (api/parameters.py:11-12);
    route r runs on vehicle min(r, K - 1) -- past the fleet the routes serve
    no one and the fleet count (X below) rejects the tour."""

    def __init__(self, D, A, dem, cap, st0):
        D = np.asarray(D)
        self.D = D if D.ndim == 3 else D[None]
        self.H = self.D.shape[0]
        self.dem = dem
        self.caps = [int(c) for c in np.atleast_1d(cap)]
        self.sts = [int(t) for t in np.atleast_1d(st0)]
        K = max(len(self.caps), len(self.sts))
        self.caps += [self.caps[-1]] * (K - len(self.caps))
        self.sts += [self.sts[-1]] * (K - len(self.sts))
        self.uniform = len(set(self.caps)) == 1 and len(set(self.sts)) == 1
        self.A = list(A)
        n = len(A)
        rs, dur, cus, rid = [0], [], [], [0] * n
        w = Walk(self, 0)
        for q, c in enumerate(A):
            if c == 0:
                rid[q] = len(dur)
                cu = w.prev != 0
                dur.append(w.close())
                cus.append(cu)
                rs.append(q + 1)
                continue
            if w.load + dem[c] > w.cap:
                cu = w.prev != 0
                dur.append(w.close())
                cus.append(cu)
                rs.append(q)
            w.add(c)
            rid[q] = len(dur)
        cu = w.prev != 0
        dur.append(w.close())
        cus.append(cu)
        self.R = len(dur)
        rs[self.R:] = [n]
        self.rs, self.dur, self.cus, self.rid = rs, dur, cus, rid
        self.dsp = [0]
        for d in dur:
            self.dsp.append(self.dsp[-1] + d)
        self.pmx = [0]
        for d in dur:
            self.pmx.append(max(self.pmx[-1], d))
        self.smx = [0] * (self.R + 1)
        for r in range(self.R - 1, -1, -1):
            self.smx[r] = max(self.smx[r + 1], dur[r])
        self.lnea = [0] * (self.R + 1)
        for r in range(self.R - 1, -1, -1):
            self.lnea[r] = int(self.lnea[r + 1] or cus[r])
        self.lnb = [-1]
        for r in range(self.R):
            self.lnb.append(r if cus[r] else self.lnb[-1])

    def cap_of(self, v):
        return self.caps[min(v, len(self.caps) - 1)]

    def st_of(self, v):
        return self.sts[min(v, len(self.sts) - 1)]

    def edge(self, t, a, b):
        return int(self.D[(t // 60) % self.H, a, b])


class Walk:
    """The greedy split from a route start on vehicle v (its capacity and
    start time)."""

    def __init__(self, T, v=0):
        self.T = T
        self.v = v
        self.load, self.t, self.prev = 0, T.st_of(v), 0
        self.cap = T.cap_of(v)
        self.cnt = self.ds = self.dm = 0
        self.xs = -1

    def close(self):
        rd = 0
        if self.prev:
            self.t += self.T.edge(self.t, self.prev, 0)
            rd = self.t - self.T.st_of(self.v)
            self.ds += rd
            self.dm = max(self.dm, rd)
        self.cnt += 1
        self.v += 1
        self.load, self.t, self.prev = 0, self.T.st_of(self.v), 0
        self.cap = self.T.cap_of(self.v)
        return rd

    def closes(self, c):
        return c == 0 or self.load + self.T.dem[c] > self.cap

    def in_step(self, c, r=None):
        """Back in step with the current tour at a position where its route r
        starts: the walk is at a route start too (fresh, or c does not fit);
        on a fleet of different vehicles also on route r's vehicle."""
        nofit = c != 0 and self.load + self.T.dem[c] > self.cap
        if not (self.prev == 0 or nofit):
            return False
        if self.T.uniform or r is None:
            return True
        return (self.v + 1 if self.prev != 0 else self.v) == r

    def add(self, c):
        self.t += self.T.edge(self.t, self.prev, c)
        self.load += self.T.dem[c]
        self.prev = c
        self.xs = self.cnt


def price(T: Tables, m, K: int, objective: int = 0):
    """Composed key of tour T.A moved by m = (typ, i, j), or None when the
    moved tour leaves a customer unserved (the kernel then re-evaluates in
    full or uses the largest key).  A fleet of different vehicles
    re-synchronises only on the same vehicle (Walk.in_step), so every zone
    that re-synchronises keeps its route count (d1 = d2 = 0) and one that
    does not is walked to the end of the tour."""
    typ, i, j = m
    A, n = T.A, len(T.A)
    mv = _moved(A, m)
    lo, hi = min(i, j), max(i, j)
    dl, bq0 = 0, lo + 1
    if typ == spec.MOVE_RELOCATE and i < j:
        dl, bq0 = -1, lo
    elif typ == spec.MOVE_RELOCATE:
        dl = 1
    # a changed token also decides whether the route before it closes there,
    # so each zone starts at the route holding the position before its first
    # change (a relocate to i < j inserts after A[hi], which stays put)
    r1s = T.rid[lo - 1] if lo > 0 else 0
    P1 = T.rs[r1s]
    r2s = T.rid[hi] if (typ == spec.MOVE_RELOCATE and i < j) or typ == spec.MOVE_2OPT \
        else T.rid[hi - 1]
    Z2 = T.rs[r2s] + dl
    two = typ != spec.MOVE_2OPT and Z2 > bq0
    phase = 1 if two else 3
    w, w1 = Walk(T, r1s), Walk(T, r1s)
    r1e, r2e = 0, T.R
    q = P1
    while q < n:
        c = mv[q]
        if phase == 1 and q >= bq0:
            qo = q - dl
            if T.rs[T.rid[qo]] == qo and w.in_step(c, T.rid[qo]):
                if w.prev:
                    w.close()
                w1, r1e = w, T.rid[qo]
                w = Walk(T, r2s + w1.cnt - (r1e - r1s))
                phase = 2
                q = Z2
                continue
            if q == Z2:
                phase = 3
        if phase >= 2 and q > hi:
            if T.rs[T.rid[q]] == q and w.in_step(c, T.rid[q]):
                if w.prev:
                    w.close()
                r2e = T.rid[q]
                break
        if w.closes(c):
            w.close()
        if c:
            w.add(c)
        q += 1
    if q >= n:
        w.close()
    if phase != 2:
        w1, w = w, Walk(T, T.R)
        r1e = r2s = r2e
    d1 = w1.cnt - (r1e - r1s)
    d2 = w.cnt - (r2e - r2s)
    if T.lnea[r2e]:
        X = T.lnb[T.R] + d1 + d2
    elif w.xs >= 0:
        X = r2s + d1 + w.xs
    elif T.lnb[r2s] >= r1e:
        X = T.lnb[r2s] + d1
    elif w1.xs >= 0:
        X = r1s + w1.xs
    else:
        X = T.lnb[r1s]
    if X >= K:
        return None
    dsum = T.dsp[T.R] - (T.dsp[r1e] - T.dsp[r1s]) - (T.dsp[r2e] - T.dsp[r2s]) + w1.ds + w.ds
    mid = max(T.dur[r1e:r2s], default=0)
    dmax = max(T.pmx[r1s], T.smx[r2e], w1.dm, w.dm, mid)
    if objective == spec.OBJ_SUM:
        return spec.pack_key(0, dsum, dmax)
    return spec.pack_key(0, dmax, dsum)


def _moved(A, m):
    typ, i, j = m
    return [A[spec.moved_index(q, typ, i, j)] for q in range(len(A))]


# ---------------------------------------------------------------------------
# Segment pricing (sa_seg_kernel, oracle_c.c seg_key): static symmetric
# matrix, every demand fits an empty vehicle, any tour.  The greedy split
# with unlimited vehicles is the concatenation, over the separator-delimited
# segments, of each segment's own greedy split, started on the vehicle its
# first route is given (every separator closes a route, an empty one lasting
# 0).  A route's duration is a sum of consecutive edges of the tour (a
# separator standing for the depot), so with prefix sums over the positions
# any run of a moved tour that reads the current tour contiguously (forward,
# or reversed on a symmetric matrix) is priced in O(1), and a capacity cut
# inside a run is found by a binary search on the prefix demands.  The fleet
# limit is one count: with R routes (empty segments included) and T
# separators after the last customer, the split serves everyone iff R - T <=
# K (R - 1 - T closures precede the last customer).  Start times do not
# enter a static route's duration.
#
# Heterogeneous fleets (per-vehicle capacities, route r on vehicle r): a
# move that changes the number of routes before a stretch of the current
# tour hands that stretch's routes to other vehicles (r -> r + delta).
# Route r keeps its split on vehicle r + delta iff need[r] <= cap(r + delta)
# <= allow[r] (need = its load; allow = load + the demand of the customer
# that did not fit - 1 when a capacity cut closed it, else unbounded), so
# whole segments are still priced from the tables when that holds for all
# their routes, and walked otherwise.  The unchanged tail after the move is
# priced from the tables up to its first route that fails, whose segment is
# walked on its new vehicles; delta then changes by that segment's change of
# route count and the tail continues (FULL: |delta| > SHIFT, re-evaluate).
# ---------------------------------------------------------------------------
INF = 1 << 62
FULL = "full"
SHIFT = 6        # the kernel's shift tables: |delta| <= 6 (kSegShift)


class SegTables:
    """Tables of tour A (capacity `cap`: one int for the whole fleet, or one
    per vehicle; every demand <= the smallest).

    e(p), p in [0, n]: edge into position p from the token before it (A[-1] =
    A[n] = 0), 0 between two depots.  PE[q] = sum e(p < q) (q <= n + 1);
    PD[q] = demand of A[0..q-1]; SC[q] = separators in A[0..q-1]; SP[k] =
    position of separator k (spx(-1) = -1, spx(S) = n); PC[q] / NC[q]: last /
    first customer position <= q / >= q (-1 / n: none).  Routes (unlimited
    vehicles, route r on vehicle min(r, K - 1)): RB[s] = first route of
    segment s (RB[S + 1] = R), dur[r], need[r], allow[r]; T = separators
    after the last customer."""

    def __init__(self, D, A, dem, cap):
        self.D, self.dem = D, dem
        self.caps = [int(cap)] if isinstance(cap, (int, np.integer)) else [int(c) for c in cap]
        self.A = list(A)
        n = self.n = len(A)
        ext = [0] + self.A + [0]
        e = [0 if ext[p] == 0 and ext[p + 1] == 0 else int(D[ext[p], ext[p + 1]])
             for p in range(n + 1)]
        self.PE = [0]
        for x in e:
            self.PE.append(self.PE[-1] + x)
        self.PD, self.SC = [0], [0]
        for c in self.A:
            self.PD.append(self.PD[-1] + (dem[c] if c else 0))
            self.SC.append(self.SC[-1] + (c == 0))
        self.SP = [q for q, c in enumerate(self.A) if c == 0]
        self.S = len(self.SP)
        self.PC, last = [], -1
        for q, c in enumerate(self.A):
            last = q if c else last
            self.PC.append(last)
        self.NC, nxt = [n] * (n + 1), n
        for q in range(n - 1, -1, -1):
            nxt = q if self.A[q] else nxt
            self.NC[q] = nxt
        self.dur, self.RB, self.need, self.allow = [], [], [], []
        for s in range(self.S + 1):
            self.RB.append(len(self.dur))
            acc = Acc(v=len(self.dur))
            run(self, acc, self.spx(s - 1) + 1, self.spx(s) - 1, False)
            close_route(self, acc)
            self.dur += acc.routes
            self.need += acc.needs
            self.allow += acc.allows
        self.R = len(self.dur)
        self.RB.append(self.R)
        self.T = n - 1 - self.PC[n - 1] if n else 0
        self.dsp = [0]
        for d in self.dur:
            self.dsp.append(self.dsp[-1] + d)
        self.pmx = [0]
        for d in self.dur:
            self.pmx.append(max(self.pmx[-1], d))
        self.smx = [0] * (self.R + 1)
        for r in range(self.R - 1, -1, -1):
            self.smx[r] = max(self.smx[r + 1], self.dur[r])

    def spx(self, k):
        return -1 if k < 0 else (self.n if k >= self.S else self.SP[k])

    def d0(self, a, b):
        return 0 if a == 0 and b == 0 else int(self.D[a, b])

    def cap_of(self, v):
        return self.caps[min(v, len(self.caps) - 1)]

    def keeps(self, r0, r1, delta):
        """Routes r0..r1-1 split the same on vehicles r + delta."""
        return all(self.route_keeps(r, delta) for r in range(r0, r1))

    def route_keeps(self, r, delta):
        return r + delta >= 0 and self.need[r] <= self.cap_of(r + delta) <= self.allow[r]

    def seg_of_route(self, r):
        """The segment holding route r (last s with RB[s] <= r)."""
        return max(s for s in range(self.S + 1) if self.RB[s] <= r)

    def one_class(self, v0, v1):
        """Vehicles v0..v1 all have the same capacity (v1 < v0: none)."""
        return all(self.cap_of(v) == self.cap_of(v0) for v in range(v0, v1 + 1))


class Acc:
    """The open route of a pricing walk (on vehicle v) and what the walk has
    closed."""

    def __init__(self, dur=0, load=0, prev=0, v=0):
        self.dur, self.load, self.prev, self.v = dur, load, prev, v
        self.routes, self.needs, self.allows = [], [], []


def close_route(T, acc, nxt_dem=None):
    """Close the open route; nxt_dem = the demand of the customer that did
    not fit (a capacity cut), None for a separator or the tour's end."""
    acc.routes.append(acc.dur + T.d0(acc.prev, 0))
    acc.needs.append(acc.load)
    acc.allows.append(INF if nxt_dem is None else acc.load + nxt_dem - 1)
    acc.dur = acc.load = acc.prev = 0
    acc.v += 1


def run(T, acc, a, b, rev):
    """Customers A[a..b] (no separator among them) joined to the open route
    in the moved order (reversed: A[b] first), cutting the route wherever
    the greedy split's next customer does not fit its vehicle."""
    PE, PD, A = T.PE, T.PD, T.A
    while a <= b:
        room = T.cap_of(acc.v) - acc.load
        if PD[b + 1] - PD[a] <= room:
            acc.dur += T.d0(acc.prev, A[b] if rev else A[a]) + PE[b + 1] - PE[a + 1]
            acc.load += PD[b + 1] - PD[a]
            acc.prev = A[a] if rev else A[b]
            return
        if not rev:
            # last q in [a - 1, b] with PD[q + 1] - PD[a] <= room
            lo_, hi_ = a - 1, b
            while lo_ < hi_:
                mid = (lo_ + hi_ + 1) // 2
                if PD[mid + 1] - PD[a] <= room:
                    lo_ = mid
                else:
                    hi_ = mid - 1
            q = lo_
            if q >= a:
                acc.dur += T.d0(acc.prev, A[a]) + PE[q + 1] - PE[a + 1]
                acc.load += PD[q + 1] - PD[a]
                acc.prev = A[q]
            close_route(T, acc, PD[q + 2] - PD[q + 1])
            a = q + 1
        else:
            # first x in [a, b + 1] with PD[b + 1] - PD[x] <= room
            lo_, hi_ = a, b + 1
            while lo_ < hi_:
                mid = (lo_ + hi_) // 2
                if PD[b + 1] - PD[mid] <= room:
                    hi_ = mid
                else:
                    lo_ = mid + 1
            x = lo_
            if x <= b:
                acc.dur += T.d0(acc.prev, A[b]) + PE[b + 1] - PE[x + 1]
                acc.load += PD[b + 1] - PD[x]
                acc.prev = A[x]
            close_route(T, acc, PD[x] - PD[x - 1])
            b = x - 1


def price_seg(T: SegTables, m, K: int, objective: int = 0):
    """Key of T.A moved by m; None when the moved tour leaves a customer
    unserved (R - T > K); FULL when (heterogeneous fleet) the tail after the
    changed segments moves by more than SHIFT vehicles."""
    typ, i, j = m
    A, SC = T.A, T.SC
    n = T.n
    lo, hi = min(i, j), max(i, j)
    s0 = SC[lo]                         # first changed segment
    st = T.spx(s0 - 1) + 1              # its first position
    en = T.spx(SC[hi + 1])              # separator closing the last changed one (n: the end)
    if typ == spec.MOVE_2OPT:
        mid = [(i, j, True)]
    elif typ == spec.MOVE_SWAP:
        mid = [(j, j, False), (i + 1, j - 1, False), (i, i, False)]
    elif i < j:
        mid = [(i + 1, j, False), (i, i, False)]
    else:
        mid = [(i, i, False), (j, i - 1, False)]
    acc = Acc(v=T.RB[s0])
    inner = {"sum": 0, "max": 0, "cnt": 0}
    tr = {"seps": 0, "cust": False}      # separators since the last customer of the region

    def sep():
        close_route(T, acc)
        tr["seps"] += 1

    def crun(a, b, rev):
        if a <= b:
            run(T, acc, a, b, rev)
            tr["seps"], tr["cust"] = 0, True

    def piece(a, b, rev):
        if a > b:
            return
        if SC[b + 1] == SC[a]:
            crun(a, b, rev)
            return
        smin, smax = T.spx(SC[a]), T.spx(SC[b + 1] - 1)
        if rev:
            crun(smax + 1, b, True)
        else:
            crun(a, smin - 1, False)
        sep()
        if smin < smax:                  # whole segments of A between the piece's separators
            g0, g1 = SC[smin] + 1, SC[smax]
            r0, r1 = T.RB[g0], T.RB[g1 + 1]
            v = acc.v                    # the vehicle their first route gets now
            if rev:
                # a reversed segment of several routes splits differently, and
                # reversed single-route segments keep their splits when one
                # capacity class serves them before and after
                # (the moved order hands them to the vehicles in reverse)
                tabled = r1 - r0 == g1 - g0 + 1 and T.one_class(r0, r1 - 1) and \
                    T.one_class(v, v + r1 - r0 - 1) and T.cap_of(v) == T.cap_of(r0)
            else:
                tabled = v == r0 or T.keeps(r0, r1, v - r0)
            if not tabled:               # walk them
                gs = range(g1, g0 - 1, -1) if rev else range(g0, g1 + 1)
                for g in gs:
                    crun(T.spx(g - 1) + 1, T.spx(g) - 1, rev)
                    sep()
            else:
                inner["sum"] += T.dsp[r1] - T.dsp[r0]
                inner["max"] = max([inner["max"]] + T.dur[r0:r1])
                inner["cnt"] += r1 - r0
                acc.v += r1 - r0
                if rev:
                    c = T.NC[smin]       # the interior's last customer in the moved order
                    if c < smax:
                        tr["seps"], tr["cust"] = SC[c] - SC[smin], True
                    else:
                        tr["seps"] += SC[smax] - SC[smin]
                else:
                    c = T.PC[smax]
                    if c > smin:
                        tr["seps"], tr["cust"] = SC[smax + 1] - SC[c + 1], True
                    else:
                        tr["seps"] += SC[smax] - SC[smin]
        if rev:
            crun(a, smin - 1, True)
        else:
            crun(smax + 1, b, False)

    crun(st, lo - 1, False)
    for a, b, rev in mid:
        piece(a, b, rev)
    if en < n:
        piece(hi + 1, en, False)
    else:
        crun(hi + 1, n - 1, False)
        close_route(T, acc)
    g_last = SC[en] if en < n else T.S   # last segment of the region
    ra, rz = T.RB[s0], T.RB[g_last + 1]  # current routes the region replaces
    # the tail: routes rz.. of the current tour on vehicles shifted by delta
    tail = []                            # its route durations in the moved tour
    r, delta = rz, acc.v - rz            # (r: always the first route of a segment)
    while r < T.R:
        if delta < -SHIFT or delta > SHIFT:
            return FULL
        if delta == 0:
            tail += T.dur[r:]
            break
        rb = r
        while rb < T.R and T.route_keeps(rb, delta):
            rb += 1
        if rb == T.R:
            tail += T.dur[r:]
            break
        g = T.seg_of_route(rb)           # walk the segment holding the first that fails
        tail += T.dur[r:T.RB[g]]
        w = Acc(v=T.RB[g] + delta)
        run(T, w, T.spx(g - 1) + 1, T.spx(g) - 1, False)
        close_route(T, w)
        tail += w.routes
        delta += len(w.routes) - (T.RB[g + 1] - T.RB[g])
        r = T.RB[g + 1]
    R = ra + len(acc.routes) + inner["cnt"] + len(tail)
    if en < n and T.PC[n - 1] > en:     # the tail after the region keeps the last customer
        Tb = T.T
    elif tr["cust"]:
        Tb = tr["seps"] + (n - 1 - en if en < n else 0)
    else:
        Tb = T.T
    if R - Tb > K:
        return None
    dsum = T.dsp[ra] + sum(acc.routes) + inner["sum"] + sum(tail)
    dmax = max([T.pmx[ra], inner["max"]] + acc.routes + tail)
    if objective == spec.OBJ_SUM:
        return spec.pack_key(0, dsum, dmax)
    return spec.pack_key(0, dmax, dsum)
