"""Synthetic instances for the five BASELINE.json configs.

There is no network and no instance data in the reference (its matrices
live in a remote Supabase table, ``api/database.py:38-48``), so every
benchmark and parity case uses these seeded generators.  All matrices are
integer minutes (A2); rounding is round-half-up, ``floor(x + 0.5)``.
"""
from __future__ import annotations

import math
from dataclasses import dataclass, field

import numpy as np


@dataclass
class Instance:
    name: str
    durations: np.ndarray          # int64 [H][N][N]
    demand: np.ndarray | None      # int64 [N] (demand[0] = 0), None for TSP
    capacities: np.ndarray | None  # int64 [K]
    start_times: np.ndarray        # int64 [K] (TSP: [startTime])
    problem: str                   # "tsp" | "cvrp"
    meta: dict = field(default_factory=dict)

    @property
    def N(self):
        return int(self.durations.shape[1])

    @property
    def n(self):
        return self.N - 1

    @property
    def H(self):
        return int(self.durations.shape[0])

    @property
    def K(self):
        return int(self.start_times.shape[0])


def _round(x):
    return np.floor(np.asarray(x, dtype=np.float64) + 0.5).astype(np.int64)


def euclid_matrix(xy: np.ndarray) -> np.ndarray:
    d = np.sqrt(((xy[:, None, :] - xy[None, :, :]) ** 2).sum(-1))
    return _round(d)


def random_symmetric(N: int, rng, lo: int = 3, hi: int = 320) -> np.ndarray:
    """Cfg 1/5: symmetric ``randint(lo, hi)`` with zero diagonal (range from
    the stub ``calculate_duration`` at src/solver.py:12)."""
    a = rng.integers(lo, hi + 1, size=(N, N), dtype=np.int64)
    a = np.triu(a, 1)
    a = a + a.T
    return a


def tsp20(seed: int = 0) -> Instance:
    rng = np.random.default_rng(seed)
    D = random_symmetric(20, rng)
    return Instance("tsp20", D[None], None, None, np.array([0]), "tsp")


def tsp50(seed: int = 0) -> Instance:
    rng = np.random.default_rng(seed)
    D = random_symmetric(50, rng)
    return Instance("tsp50", D[None], None, None, np.array([0]), "tsp")


def cvrp(n: int = 100, K: int = 8, seed: int = 0, dmax: int = 10, slack: float = 1.1,
         name: str | None = None) -> Instance:
    """Cfg 2: depot + n customers, coords uniform int [0,1000]^2, demand
    1..dmax, K vehicles of uniform capacity ceil(slack * sum(d) / K)."""
    rng = np.random.default_rng(seed)
    xy = rng.integers(0, 1001, size=(n + 1, 2)).astype(np.float64)
    D = euclid_matrix(xy)
    dem = np.concatenate([[0], rng.integers(1, dmax + 1, size=n)]).astype(np.int64)
    cap = int(math.ceil(slack * dem.sum() / K))
    return Instance(name or f"cvrp{n}", D[None], dem, np.full(K, cap, dtype=np.int64),
                    np.zeros(K, dtype=np.int64), "cvrp", {"xy": xy})


HOUR_FACTOR = np.array([1.0] * 24)
for _h, _f in {6: 1.2, 7: 1.5, 8: 1.8, 9: 1.5, 10: 1.2, 15: 1.2, 16: 1.5, 17: 1.8,
               18: 1.5, 19: 1.2}.items():
    HOUR_FACTOR[_h] = _f


def td_cvrp(n: int = 200, K: int = 16, seed: int = 0, start: int = 480) -> Instance:
    """Cfg 3: 24 hourly matrices D_h = round(euclid * f_h), f_h in [1.0, 1.8]
    peaking at 08:00 and 17:00; every vehicle leaves at ``start`` (08:00)."""
    rng = np.random.default_rng(seed)
    xy = rng.integers(0, 1001, size=(n + 1, 2)).astype(np.float64)
    base = np.sqrt(((xy[:, None, :] - xy[None, :, :]) ** 2).sum(-1))
    D = np.stack([_round(base * HOUR_FACTOR[h]) for h in range(24)])
    dem = np.concatenate([[0], rng.integers(1, 11, size=n)]).astype(np.int64)
    cap = int(math.ceil(1.1 * dem.sum() / K))
    return Instance(f"tdvrp{n}", D, dem, np.full(K, cap, dtype=np.int64),
                    np.full(K, start, dtype=np.int64), "cvrp", {"xy": xy})


def td_cvrp_het(n: int = 200, K: int = 16, seed: int = 0, fracs=(1.3, 1.0, 0.8),
                start: int = 420) -> Instance:
    """The reference's normal VRP request on cfg 3's matrix: td_cvrp's 24
    hourly matrices with per-vehicle capacities (len(fracs) classes of
    frac x the uniform capacity, in vehicle order, each at least the largest
    demand; api/parameters.py:11) and staggered start times start + 37 k mod
    240 (api/parameters.py:12)."""
    x = td_cvrp(n, K, seed)
    base = int(x.capacities[0])
    caps = np.array([max(int(base * fracs[k * len(fracs) // K]), int(x.demand.max()))
                     for k in range(K)], dtype=np.int64)
    starts = np.arange(K, dtype=np.int64) * 37 % 240 + start
    return Instance(f"tdvrp{n}_het", x.durations, x.demand, caps, starts, "cvrp", x.meta)


def x_style(n: int = 1000, seed: int = 0, r: float = 12.0) -> Instance:
    """Cfg 4: Uchoa et al. (2017) X-style generator -- central depot,
    random-clustered customer positions, unitary-to-large demands, route
    size r (average customers per route) giving Q = ceil(r * sum(d) / n)."""
    rng = np.random.default_rng(seed)
    depot = np.array([[500.0, 500.0]])
    n_rand = n // 2
    n_clu = n - n_rand
    seeds = rng.uniform(0, 1000, size=(max(3, n // 100), 2))
    pts = [rng.uniform(0, 1000, size=(n_rand, 2))]
    clu = []
    while len(clu) < n_clu:
        s = seeds[rng.integers(0, len(seeds))]
        p = rng.uniform(0, 1000, size=2)
        if rng.random() < math.exp(-np.linalg.norm(p - s) / 40.0):
            clu.append(p)
    pts.append(np.array(clu))
    xy = np.floor(np.concatenate([depot] + pts))
    D = euclid_matrix(xy)
    dem = np.concatenate([[0], rng.integers(1, 101, size=n)]).astype(np.int64)
    cap = int(math.ceil(r * dem.sum() / n))
    K = int(math.ceil(dem.sum() / cap)) + 2
    return Instance(f"x{n}", D[None], dem, np.full(K, cap, dtype=np.int64),
                    np.zeros(K, dtype=np.int64), "cvrp", {"xy": xy})


CONFIGS = {
    "tsp20": tsp20,
    "cvrp100": lambda seed=0: cvrp(100, 8, seed),
    "tdvrp200": lambda seed=0: td_cvrp(200, 16, seed),
    "x1000": lambda seed=0: x_style(1000, seed),
    "tsp50": tsp50,
}


def random_perms(C: int, n: int, seed: int = 0, ld: int | None = None, dtype=np.uint8) -> np.ndarray:
    """C random permutations of customers 1..n, rows padded to ``ld``."""
    rng = np.random.default_rng(seed)
    ld = n if ld is None else ld
    out = np.zeros((C, ld), dtype=dtype)
    out[:, :n] = (rng.permuted(np.tile(np.arange(1, n + 1, dtype=np.int64), (C, 1)), axis=1)
                  ).astype(dtype)
    return out
