"""Epoch-driven search runners over the HIP kernels.

Each runner owns its device state (tours, keys) as torch tensors, advances
it with one C-ABI call per epoch, and exposes the operations the island
model and the front-end need:

  epoch()            advance the search (GPU kernels only)
  best()             (key, tour) of the best solution seen (device argmin)
  elites(E) / inject(tours, keys)   migration hooks (islands.py), both
                     library kernels (vrpms_pool_elites / vrpms_pool_inject)
  src() / dst() / inject_mode / groups   the pools vrpms_island_exchange
                     reads the elites from and injects the migrants into

torch only owns buffers here: start tours come from the library's Philox
Fisher-Yates kernel, elite selection / injection / ACO best tracking from
its pool kernels.

Defaults follow the reference's knobs where it has any
(api/parameters.py:18-23: randomPermutationCount -> population,
iterationCount -> generations); SA/ACO/BF endpoints declare no knobs
(api/parameters.py:26-31, 47-56), so their defaults are build-defined.
"""
from __future__ import annotations

import math

import numpy as np

from ._lib import INJECT_BETTER, INJECT_SORTED, INJECT_WORST
from .core import Context


def _torch():
    import torch
    return torch


def random_tours(ctx: Context, count: int, n: int, seed: int, stream_id: int = 0):
    """count Philox Fisher-Yates permutations of 1..n as int16 rows
    (vrpms_random_tours, oracle/pool.py philox_tour)."""
    return ctx.random_tours(count, n, seed, stream_id)


def typical_edge(durations) -> float:
    D = np.asarray(durations, dtype=np.float64)
    nz = D[D > 0]
    return float(nz.mean()) if nz.size else 1.0


class _Base:
    inject_mode = INJECT_WORST
    groups = 1

    def best(self):
        tours, keys = self.src()
        k, i = self.ctx.argmin(keys.reshape(-1))
        return k, tours.reshape(-1, self.n)[i]

    def elites(self, E: int):
        """The E best (tour, key) rows of src() by (key, index)."""
        return self.ctx.pool_elites(*self.src(), E)

    def inject(self, tours, keys):
        """Migrants into dst() by inject_mode (vrpms_pool_inject)."""
        self.ctx.pool_inject(*self.dst(), self.inject_mode, tours, keys, self.groups)


class SARunner(_Base):
    """Independent SA chains (one wavefront each), geometric cooling from
    t0 to t_end over `total_steps` steps.  `n_sep` A10 route separators
    (CVRP) ride in every tour, so the moves also place route boundaries;
    tours then hold n + n_sep tokens (self.n).  `window` > 0 samples A11
    windowed moves of the A12 types `window_types` (0 = all; priced
    route-locally on an exchangeable fleet; `moves` = 64 W samples per step
    on W wavefronts per chain).  `start` places the separators:
    "random" (Philox tokens), "greedy" (where the greedy split of a random
    order closes routes) or "pack" (first-fit routes of a random order, a
    feasible start when the fleet has little spare capacity)."""

    def __init__(self, ctx: Context, n: int, chains: int = 1024, seed: int = 0,
                 total_steps: int = 2000, steps_per_epoch: int = 250, t0: float | None = None,
                 t_end: float | None = None, durations=None, n_sep: int = 0, window: int = 0,
                 window_types: int = 0, start: str = "random", moves: int = 64):
        torch = _torch()
        self.ctx, self.n, self.seed = ctx, n + n_sep, seed
        self.n_sep, self.window, self.window_types = n_sep, window, window_types
        self.moves = moves
        self.chains = chains
        edge = typical_edge(durations) if durations is not None else 100.0
        t0 = t0 if t0 is not None else 0.5 * edge
        t_end = t_end if t_end is not None else 0.002 * edge
        self.inv_alpha = np.float32((t0 / t_end) ** (1.0 / max(total_steps, 1)))
        self.inv_t = np.float32(1.0 / t0)
        self.steps_per_epoch = steps_per_epoch
        self.step = 0
        if n_sep and start == "greedy":   # separators where the greedy split closes routes
            self.cur = ctx.insert_separators(ctx.random_tours(chains, n, seed), n_sep)
        elif n_sep and start == "pack":   # first-fit routes
            self.cur = ctx.pack_separators(ctx.random_tours(chains, n, seed), n_sep)
        else:
            self.cur = ctx.random_tours(chains, n, seed, n_sep=n_sep)
        self.best_t = self.cur.clone()
        self.cur_key = torch.empty(chains, dtype=torch.int64, device=ctx.dev)
        self.best_key = torch.full((chains,), -1, dtype=torch.int64, device=ctx.dev)

    def epoch(self, steps: int | None = None):
        s = self.steps_per_epoch if steps is None else steps
        self.ctx.sa_run(self.cur, self.cur_key, self.best_t, self.best_key, s, float(self.inv_t),
                        float(self.inv_alpha), self.seed, self.step, window=self.window,
                        window_types=self.window_types, moves=self.moves)
        for _ in range(s):      # same float32 recurrence as the kernel
            self.inv_t = np.float32(self.inv_t * self.inv_alpha)
        self.step += s

    # elites come from the best-so-far; migrants restart the worst chains
    def src(self):
        return self.best_t, self.best_key

    def dst(self):
        return self.cur, self.cur_key


class Polish:
    """The memetic step of the GA / ACO endpoints (api/vrp/{ga,aco}/index.py):
    `steps` SA steps (vrpms_sa_run: the same moves, Philox streams and
    acceptance as the SA endpoint) on some rows of a pool, whose best-so-far
    tours and keys then replace those rows.  The temperature cools
    geometrically from t0 to t_end over `total_steps` polish steps (or by
    whatever inv_t / inv_alpha the caller sets, e.g. a wall-time schedule);
    the Philox stream is the pool's seed ^ 0x9E3779B9 with the step counter
    running across calls."""

    def __init__(self, steps: int, durations=None, t0: float | None = None,
                 t_end: float | None = None, total_steps: int = 20000, seed: int = 0):
        edge = typical_edge(durations) if durations is not None else 100.0
        t0 = t0 if t0 is not None else 0.05 * edge
        t_end = t_end if t_end is not None else 0.002 * edge
        self.steps = int(steps)
        self.inv_t = np.float32(1.0 / t0)
        self.inv_alpha = np.float32((t0 / t_end) ** (1.0 / max(total_steps, 1)))
        self.seed = (int(seed) ^ 0x9E3779B9) & (2**64 - 1)
        self.step = 0

    def run(self, ctx: Context, rows, keys):
        """SA from each row of `rows` (int16 [R][n], contiguous); returns the
        chains' best (tours, keys) -- never worse than the rows' own keys."""
        torch = _torch()
        cur = rows.clone()
        best = rows.clone()
        ck = torch.empty(rows.shape[0], dtype=torch.int64, device=rows.device)
        bk = keys.clone()
        ctx.sa_run(cur, ck, best, bk, self.steps, float(self.inv_t), float(self.inv_alpha),
                   self.seed, self.step)
        for _ in range(self.steps):       # the kernel's float32 recurrence
            self.inv_t = np.float32(self.inv_t * self.inv_alpha)
        self.step += self.steps
        return best, bk


class GARunner(_Base):
    """Island GA: `islands` populations of `pop` members, each kept sorted by
    (key, index); migrants take the worst slots of the islands round robin.
    `polish` (a Polish): after each epoch's generations the `polish_top`
    best members of every island are improved by SA (memetic GA) and put
    back in their slots (the next generation re-sorts the islands)."""

    inject_mode = INJECT_SORTED

    def __init__(self, ctx: Context, n: int, islands: int = 8, pop: int = 256, seed: int = 0,
                 pmut: float = 0.2, gens_per_epoch: int = 20, polish: Polish | None = None,
                 polish_top: int = 4):
        self.ctx, self.n, self.seed = ctx, n, seed
        self.islands, self.pop, self.pmut = islands, pop, pmut
        self.gens_per_epoch = gens_per_epoch
        self.gen = 0
        self.groups = islands
        self.polish, self.polish_top = polish, max(1, min(polish_top, pop))
        self.tours = random_tours(ctx, islands * pop, n, seed).view(islands, pop, n).contiguous()
        self.keys = ctx.eval(self.tours.view(-1, n)).view(islands, pop)

    def epoch(self, gens: int | None = None):
        g = self.gens_per_epoch if gens is None else gens
        self.ctx.ga_generation(self.tours, self.keys, g, self.pmut, self.seed, self.gen)
        self.gen += g
        if self.polish is not None and self.n >= 2:
            T = self.polish_top
            rows = self.tours[:, :T, :].reshape(-1, self.n).contiguous()
            keys = self.keys[:, :T].reshape(-1).contiguous()
            best, bk = self.polish.run(self.ctx, rows, keys)
            self.tours[:, :T, :] = best.view(self.islands, T, self.n)
            self.keys[:, :T] = bk.view(self.islands, T)

    def src(self):
        return self.tours, self.keys

    def dst(self):
        return self.tours, self.keys


class ACORunner(_Base):
    """Integer max-min ant colonies (one pheromone matrix per colony); each
    colony's best-so-far is tracked on the device and deposits on every
    `bsf_period`-th iteration (the iteration best on the others), so a
    migrant injected into a colony's best-so-far shapes its pheromone."""

    inject_mode = INJECT_BETTER

    def __init__(self, ctx: Context, n: int, colonies: int = 4, ants: int = 64, seed: int = 0,
                 iters_per_epoch: int = 5, evap_shift: int = 3, bsf_period: int = 5,
                 polish: Polish | None = None):
        torch = _torch()
        if n != ctx.N - 1:
            raise ValueError("ACO builds complete giant tours: n must be N - 1")
        self.ctx, self.n, self.seed = ctx, n, seed
        self.colonies, self.ants = colonies, ants
        self.iters_per_epoch, self.evap_shift = iters_per_epoch, evap_shift
        self.bsf_period = bsf_period
        self.tau_max, self.tau_min = 1 << 30, 1 << 12
        self.tau, self.eta = ctx.aco_init(colonies, 1 << 24)
        self.it = 0
        self.best_key = torch.full((colonies,), -1, dtype=torch.int64, device=ctx.dev)
        self.best_t = torch.zeros((colonies, n), dtype=torch.int16, device=ctx.dev)
        self.polish = polish

    def epoch(self, iters: int | None = None):
        """`polish` (a Polish): after the epoch's iterations every colony's
        best-so-far is improved by SA (ACO with local search), so the next
        best-so-far deposit lays pheromone on the improved tour."""
        for _ in range(self.iters_per_epoch if iters is None else iters):
            self.ctx.aco_iteration(self.tau, self.eta, self.ants, self.seed, self.it,
                                   self.evap_shift, self.tau_min, self.tau_max,
                                   best_tours=self.best_t, best_keys=self.best_key,
                                   bsf_period=self.bsf_period)
            self.it += 1
        if self.polish is not None and self.n >= 2:
            best, bk = self.polish.run(self.ctx, self.best_t.contiguous(), self.best_key)
            self.best_t.copy_(best)
            self.best_key.copy_(bk)

    # migrant e replaces colony e's best-so-far when better
    def src(self):
        return self.best_t, self.best_key

    def dst(self):
        return self.best_t, self.best_key


def brute_force(ctx: Context, n: int, rank_begin: int = 0, rank_end: int | None = None):
    """Exact optimum over lexicographic ranks [begin, end) -> (key, tour)."""
    if rank_end is None:
        rank_end = math.factorial(n)
    key, rank = ctx.bf_run(n, rank_begin, rank_end)
    return key, unrank(rank, n) if rank != 2**64 - 1 else None


def unrank(rank: int, n: int):
    """Lexicographic rank -> permutation of 1..n (host-side index arithmetic)."""
    avail = list(range(1, n + 1))
    out = []
    for i in range(n):
        f = math.factorial(n - 1 - i)
        d, rank = divmod(rank, f)
        out.append(avail.pop(d))
    return out
