"""Pure-Python model of sa_route_kernel's move pricing (route tables,
re-synchronising walks, two zones, composed key) -- TEST INFRASTRUCTURE.

It mirrors the kernel step for step so the composition rules can be
checked against oracle/spec.py eval_cvrp on many random moves on the CPU
(tests/test_route_model.py); the device kernel is then checked against the
C restatement on the GPU.  Exchangeable fleet only: one capacity, one start
time, every demand fits an empty vehicle.
"""
from __future__ import annotations

from . import spec


class Tables:
    """Greedy-split routes of tour A with unlimited vehicles: rs (first
    position), dur, cus (holds a customer), rid (route of each position)."""

    def __init__(self, D, A, dem, cap, st0):
        self.D, self.dem, self.cap, self.st0 = D, dem, cap, st0
        self.A = list(A)
        n = len(A)
        rs, dur, cus, rid = [0], [], [], [0] * n
        w = Walk(self)
        for q, c in enumerate(A):
            if c == 0:
                rid[q] = len(dur)
                cu = w.prev != 0
                dur.append(w.close())
                cus.append(cu)
                rs.append(q + 1)
                continue
            if w.load + dem[c] > cap:
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


class Walk:
    def __init__(self, T):
        self.T = T
        self.load, self.t, self.prev = 0, T.st0, 0
        self.cnt = self.ds = self.dm = 0
        self.xs = -1

    def close(self):
        rd = 0
        if self.prev:
            self.t += int(self.T.D[self.prev, 0])
            rd = self.t - self.T.st0
            self.ds += rd
            self.dm = max(self.dm, rd)
        self.cnt += 1
        self.load, self.t, self.prev = 0, self.T.st0, 0
        return rd

    def closes(self, c):
        return c == 0 or self.load + self.T.dem[c] > self.T.cap

    def in_step(self, c):
        return self.prev == 0 or (c != 0 and self.load + self.T.dem[c] > self.T.cap)

    def add(self, c):
        self.t += int(self.T.D[self.prev, c])
        self.load += self.T.dem[c]
        self.prev = c
        self.xs = self.cnt


def price(T: Tables, m, K: int, objective: int = 0):
    """Composed key of tour T.A moved by m = (typ, i, j), or None when the
    moved tour leaves a customer unserved (the kernel then re-evaluates in
    full or uses the largest key)."""
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
    w, w1 = Walk(T), Walk(T)
    r1e, r2e = 0, T.R
    q = P1
    while q < n:
        c = mv[q]
        if phase == 1 and q >= bq0:
            qo = q - dl
            if T.rs[T.rid[qo]] == qo and w.in_step(c):
                if w.prev:
                    w.close()
                w1, r1e = w, T.rid[qo]
                w = Walk(T)
                phase = 2
                q = Z2
                continue
            if q == Z2:
                phase = 3
        if phase >= 2 and q > hi:
            if T.rs[T.rid[q]] == q and w.in_step(c):
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
        w1, w = w, Walk(T)
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
# "Clean" tours: O(1) move pricing (sa_route_kernel's fast mode, and
# oracle_c.c resync_clean).  A tour is clean when its greedy split closes
# routes only at A10 separators: every separator-delimited segment fits one
# vehicle and there are at most K - 1 separators.  Then on a static
# symmetric matrix every route's duration is a sum of consecutive edges of
# the tour (the separator standing for the depot), so prefix sums over the
# positions price any route of a moved tour that is a few contiguous pieces
# of the current one (forward or reversed) in O(1), whatever the move's span.
# ---------------------------------------------------------------------------
class CleanTables:
    """Position prefix tables of tour A (uniform capacity `cap`).

    e(p), p in [0, n]: edge into position p from the token before it (A[-1] =
    A[n] = 0, the depot), 0 between two depots (an empty route lasts 0).
    PE[q] = sum e(p < q) (q <= n + 1); PD[q] = demand of A[0..q-1];
    SC[q] = separators in A[0..q-1]; SP[k] = position of separator k,
    SPx(-1) = -1, SPx(S) = n.  Route r = segment SPx(r-1)+1 .. SPx(r)-1."""

    def __init__(self, D, A, dem, cap):
        self.D, self.dem, self.cap = D, dem, cap
        self.A = list(A)
        n = self.n = len(A)
        ext = [0] + self.A + [0]
        self.e = [0 if ext[p] == 0 and ext[p + 1] == 0 else int(D[ext[p], ext[p + 1]])
                  for p in range(n + 1)]
        self.PE = [0]
        for x in self.e:
            self.PE.append(self.PE[-1] + x)
        self.PD = [0]
        self.SC = [0]
        for c in self.A:
            self.PD.append(self.PD[-1] + (dem[c] if c else 0))
            self.SC.append(self.SC[-1] + (c == 0))
        self.SP = [q for q, c in enumerate(self.A) if c == 0]
        self.S = len(self.SP)
        R = self.S + 1
        self.dur = [self.PE[self.spx(r) + 1] - self.PE[self.spx(r - 1) + 1] for r in range(R)]
        self.load = [self.PD[self.spx(r)] - self.PD[self.spx(r - 1) + 1] for r in range(R)]
        self.dsp = [0]
        for d in self.dur:
            self.dsp.append(self.dsp[-1] + d)
        self.pmx = [0]
        for d in self.dur:
            self.pmx.append(max(self.pmx[-1], d))
        self.smx = [0] * (R + 1)
        for r in range(R - 1, -1, -1):
            self.smx[r] = max(self.smx[r + 1], self.dur[r])

    def spx(self, k):
        return -1 if k < 0 else (self.n if k >= self.S else self.SP[k])

    def clean(self, K):
        return self.S <= K - 1 and all(x <= self.cap for x in self.load)

    def d0(self, a, b):
        return 0 if a == 0 and b == 0 else int(self.D[a, b])


def price_clean(T: CleanTables, m, objective: int = 0):
    """Key of T.A moved by m on a clean tour and a static symmetric matrix,
    or None when a route of the moved tour exceeds the capacity (the kernel
    then gives the largest key when that provably leaves a customer
    unserved, else prices the move by a walk)."""
    typ, i, j = m
    A, PE, PD, SC = T.A, T.PE, T.PD, T.SC
    n = T.n
    lo, hi = min(i, j), max(i, j)
    ra = SC[lo]                      # first changed route (B's routes before it are A's)
    st = T.spx(ra - 1) + 1           # its first position
    en = T.spx(SC[hi + 1])           # first separator at or after hi + 1 (n: none)
    # pieces of the moved tour between lo and hi, A positions (a, b, reversed)
    if typ == spec.MOVE_2OPT:
        mid = [(i, j, True)]
    elif typ == spec.MOVE_SWAP:
        mid = [(j, j, False), (i + 1, j - 1, False), (i, i, False)]
    elif i < j:
        mid = [(i + 1, j, False), (i, i, False)]
    else:
        mid = [(i, i, False), (j, i - 1, False)]
    st_ = {"load": PD[lo] - PD[st], "dur": PE[lo] - PE[st], "prev": A[lo - 1] if st < lo else 0}
    routes = []          # (dur, load) of the changed routes, in order
    inner = [0, 0]       # sum and max of the whole current-tour routes inside pieces

    def close():
        routes.append((st_["dur"], st_["load"]))

    def piece(a, b, rev):
        if a > b:
            return
        F, L = (A[b], A[a]) if rev else (A[a], A[b])
        ns = SC[b + 1] - SC[a]
        if ns == 0:
            st_["dur"] += T.d0(st_["prev"], F) + PE[b + 1] - PE[a + 1]
            st_["load"] += PD[b + 1] - PD[a]
            st_["prev"] = L
            return
        smin, smax = T.spx(SC[a]), T.spx(SC[b + 1] - 1)
        sf, sl = (smax, smin) if rev else (smin, smax)
        # the part before the first separator (in the moved order) ends the open route
        if not rev and sf > a:
            st_["dur"] += T.d0(st_["prev"], A[a]) + PE[sf + 1] - PE[a + 1]
            st_["load"] += PD[sf] - PD[a]
        elif rev and sf < b:
            st_["dur"] += T.d0(st_["prev"], A[b]) + PE[b + 1] - PE[sf + 1]
            st_["load"] += PD[b + 1] - PD[sf + 1]
        else:
            st_["dur"] += T.d0(st_["prev"], 0)
        close()
        # whole routes between the piece's first and last separator
        r0, r1 = SC[smin] + 1, SC[smax]
        if r0 <= r1:
            inner[0] += T.dsp[r1 + 1] - T.dsp[r0]
            inner[1] = max(inner[1], max(T.dur[r0:r1 + 1]))
        # the part after the last separator opens the next route
        if not rev:
            if sl < b:
                st_.update(dur=PE[b + 1] - PE[sl + 1], load=PD[b + 1] - PD[sl + 1], prev=A[b])
            else:
                st_.update(dur=0, load=0, prev=0)
        else:
            if sl > a:
                st_.update(dur=PE[sl + 1] - PE[a + 1], load=PD[sl] - PD[a], prev=A[a])
            else:
                st_.update(dur=0, load=0, prev=0)

    for a, b, rev in mid:
        piece(a, b, rev)
    if en < n:
        piece(hi + 1, en, False)         # closes the last changed route at A's separator en
    else:
        piece(hi + 1, n - 1, False)
        st_["dur"] += T.d0(st_["prev"], 0)
        close()
    if any(ld > T.cap for _, ld in routes):
        return None
    after = SC[en] + 1
    dsum = T.dsp[ra] + sum(d for d, _ in routes) + inner[0] + T.dsp[T.S + 1] - T.dsp[after]
    dmax = max([T.pmx[ra], T.smx[after], inner[1]] + [d for d, _ in routes])
    if objective == spec.OBJ_SUM:
        return spec.pack_key(0, dsum, dmax)
    return spec.pack_key(0, dmax, dsum)
