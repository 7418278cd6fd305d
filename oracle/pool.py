"""CPU restatement of the population / island-model operations of
libvrpms (``vrpms_amd/csrc/pool.hip``, declared in ``include/vrpms.h``) --
TEST INFRASTRUCTURE ONLY.

The reference has no island model (no collectives anywhere);
the exchange semantics are build-defined (all-gather of each
rank's E elites, deterministic merge, re-injection), so this module is the
spec the device kernels and the multi-rank CPU tests are checked against.
Keys are A8 uint64 values held as Python ints; tours are lists / numpy rows.
"""
from __future__ import annotations

import numpy as np

from . import spec

INJECT_WORST, INJECT_SORTED, INJECT_BETTER = 0, 1, 2


def philox_tour(n: int, seed: int, row: int, stream_id: int = 0, n_sep: int = 0):
    """vrpms_random_tours row `row`: Fisher-Yates over the tokens 1..n+n_sep,
    i = n+n_sep-1 .. 1, j = w % (i + 1), w = word (i & 3) of philox((i >> 2,
    0xfffffffe, row, stream_id), seed); tokens above n become 0 (A10)."""
    key = spec.seed_key(seed)
    L = n + n_sep
    t = list(range(1, L + 1))
    w = None
    for i in range(L - 1, 0, -1):
        if (i & 3) == 3 or i == L - 1:
            w = spec.philox4x32_10((i >> 2, 0xFFFFFFFE, row, stream_id), key)
        j = w[i & 3] % (i + 1)
        t[i], t[j] = t[j], t[i]
    return [0 if v > n else v for v in t]


def elites_order(keys, E: int):
    """Indices of the E best rows by (key, index)."""
    return sorted(range(len(keys)), key=lambda i: (int(keys[i]), i))[:E]


def worst_order(keys, E: int):
    """Indices of the E worst rows by (key desc, index asc)."""
    return sorted(range(len(keys)), key=lambda i: (-int(keys[i]), i))[:E]


def pool_elites(tours, keys, E: int):
    idx = elites_order(keys, E)
    return [list(tours[i]) for i in idx], [int(keys[i]) for i in idx]


def pool_inject(tours, keys, mode: int, mig_tours, mig_keys, groups: int = 1):
    """Returns new (tours, keys) lists after injecting the migrants."""
    tours = [list(t) for t in tours]
    keys = [int(k) for k in keys]
    E = len(mig_keys)
    if mode == INJECT_WORST:
        for e, r in enumerate(worst_order(keys, E)):
            tours[r], keys[r] = list(mig_tours[e]), int(mig_keys[e])
    elif mode == INJECT_BETTER:
        for e in range(min(E, len(keys))):
            if int(mig_keys[e]) < keys[e]:
                tours[e], keys[e] = list(mig_tours[e]), int(mig_keys[e])
    else:
        P = len(keys) // groups
        for g in range(groups):
            gt, gk = tours[g * P:(g + 1) * P], keys[g * P:(g + 1) * P]
            for e in range(g, E, groups):
                slot = P - 1 - e // groups
                if slot < 0:
                    break
                gt[slot], gk[slot] = list(mig_tours[e]), int(mig_keys[e])
            order = sorted(range(P), key=lambda i: (gk[i], i))
            tours[g * P:(g + 1) * P] = [gt[i] for i in order]
            keys[g * P:(g + 1) * P] = [gk[i] for i in order]
    return tours, keys


def msg_bytes(E: int, n: int) -> int:
    return (E * 8 + E * n * 2 + 15) & ~15


def island_pack(tours, keys, E: int, n: int) -> bytes:
    """[E keys u64 LE][E x n tours u16 LE], zero padded to 16 bytes."""
    t, k = pool_elites(tours, keys, E)
    buf = np.zeros(msg_bytes(E, n), dtype=np.uint8)
    buf[:8 * E] = np.asarray(k, dtype=np.uint64).view(np.uint8)
    buf[8 * E:8 * E + 2 * E * n] = np.asarray(t, dtype=np.uint16).reshape(-1).view(np.uint8)
    return bytes(buf)


def island_merge(msgs: bytes, world: int, E: int, n: int):
    """The E best of `world` messages (back to back, rank order) by
    (key, rank, position)."""
    mb = msg_bytes(E, n)
    cands = []
    for r in range(world):
        m = np.frombuffer(msgs[r * mb:(r + 1) * mb], dtype=np.uint8)
        ks = m[:8 * E].view(np.uint64)
        ts = m[8 * E:8 * E + 2 * E * n].view(np.uint16).reshape(E, n)
        for e in range(E):
            cands.append((int(ks[e]), r * E + e, ts[e].tolist()))
    cands.sort(key=lambda c: (c[0], c[1]))
    best = cands[:E]
    return [c[2] for c in best], [c[0] for c in best]
