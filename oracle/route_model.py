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
