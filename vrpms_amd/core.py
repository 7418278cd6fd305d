"""Device context: owns one ``vrpms_ctx`` and moves instances/tours through the
C-ABI.  PyTorch-ROCm tensors are used only as device-buffer owners and for
the current HIP stream; all arithmetic happens in libvrpms's kernels.
"""
from __future__ import annotations

import ctypes

import numpy as np

from . import _lib
from ._lib import (CVRP, INJECT_BETTER, INJECT_SORTED, INJECT_WORST, OBJ_MAX,  # noqa: F401
                   OBJ_SUM, TSP, VrpmsError, check)


def _torch():
    import torch
    return torch


def require_gpu():
    torch = _torch()
    if not torch.cuda.is_available():
        raise RuntimeError("vrpms_amd needs a ROCm GPU: torch.cuda.is_available() is False "
                           "(there is no CPU fallback by design)")
    return torch


def perm_dtype_bytes(t) -> int:
    torch = _torch()
    if t.dtype == torch.uint8:
        return 1
    if t.dtype in (torch.int16, getattr(torch, "uint16", torch.int16)):
        return 2
    raise TypeError(f"tours must be uint8 or (u)int16, got {t.dtype}")


def tour_dtype(N: int):
    """Narrowest tour element for an N-node instance (uint8 for N <= 256)."""
    torch = _torch()
    return torch.uint8 if N <= 256 else torch.int16


class Context:
    """One solver context on one GPU (``vrpms_ctx_create``)."""

    def __init__(self, device: int = 0):
        torch = require_gpu()
        self.lib = _lib.load()
        self.device = int(device)
        self.dev = torch.device("cuda", self.device)
        ptr = ctypes.c_void_p()
        check(self.lib.vrpms_ctx_create(self.device, ctypes.byref(ptr)))
        self._ctx = ptr
        self.problem = None
        self.N = self.H = self.K = 0
        self.objective = OBJ_SUM
        # (group, world) once islands.init_comm agreed on a communicator
        self.island_comm_group = None

    # -- lifetime -----------------------------------------------------------
    def close(self):
        if getattr(self, "_ctx", None):
            self.lib.vrpms_ctx_destroy(self._ctx)
            self._ctx = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    @property
    def handle(self):
        return self._ctx

    def stream(self):
        return ctypes.c_void_p(_torch().cuda.current_stream(self.dev).cuda_stream)

    # -- instance -----------------------------------------------------------
    def set_instance(self, problem: int, durations, demand=None, capacities=None,
                     start_times=(0,), objective: int = OBJ_SUM):
        """``durations``: int [N][N] or [H][N][N] (compact node indices)."""
        torch = _torch()
        D = np.asarray(durations)
        if D.ndim == 2:
            D = D[None]
        if D.ndim != 3 or D.shape[1] != D.shape[2]:
            raise ValueError("durations must be [N][N] or [H][N][N]")
        if D.size and (D.min() < np.iinfo(np.int32).min or D.max() > np.iinfo(np.int32).max):
            raise VrpmsError(_lib.VRPMS_ERANGE, "durations do not fit int32")
        H, N = int(D.shape[0]), int(D.shape[1])
        st = np.asarray(start_times, dtype=np.int64).reshape(-1)
        K = int(st.shape[0])
        d_dur = torch.as_tensor(np.ascontiguousarray(D, dtype=np.int32), device=self.dev)
        d_st = torch.as_tensor(st.astype(np.int32), device=self.dev)
        d_dem = d_cap = None
        if problem == CVRP:
            d_dem = torch.as_tensor(np.asarray(demand, dtype=np.int32).reshape(-1), device=self.dev)
            d_cap = torch.as_tensor(np.asarray(capacities, dtype=np.int32).reshape(-1), device=self.dev)
            if d_dem.numel() != N:
                raise ValueError(f"demand has {d_dem.numel()} entries, matrix has {N} nodes")
            if d_cap.numel() != K:
                raise ValueError("capacities and start_times must have the same length")
        check(self.lib.vrpms_set_instance(
            self._ctx, int(problem), d_dur.data_ptr(), H, N,
            d_dem.data_ptr() if d_dem is not None else None,
            d_cap.data_ptr() if d_cap is not None else None,
            d_st.data_ptr(), K, int(objective), self.stream()))
        self.problem, self.N, self.H, self.K, self.objective = problem, N, H, K, objective

    # -- scoring ------------------------------------------------------------
    def eval(self, perms, n: int | None = None, with_parts: bool = False, out=None):
        """Score a [C][ld] tour tensor on the device.  Returns keys (uint64
        stored as int64) or (keys, sums, maxs, unvisited) with ``with_parts``."""
        torch = _torch()
        if perms.device != self.dev or perms.dim() != 2:
            raise ValueError(f"tours must be a 2-D tensor on {self.dev}")
        if not perms.is_contiguous():
            raise ValueError("tours must be contiguous")
        C, ld = perms.shape
        n = ld if n is None else int(n)
        pb = perm_dtype_bytes(perms)
        keys = out if out is not None else torch.empty(C, dtype=torch.int64, device=self.dev)
        sums = maxs = unv = None
        if with_parts:
            sums = torch.empty(C, dtype=torch.int32, device=self.dev)
            maxs = torch.empty(C, dtype=torch.int32, device=self.dev)
            unv = torch.empty(C, dtype=torch.int32, device=self.dev)
        ptr = lambda t: t.data_ptr() if t is not None else None  # noqa: E731
        check(self.lib.vrpms_eval(self._ctx, perms.data_ptr(), pb, C, n, ld, keys.data_ptr(),
                                  ptr(sums), ptr(maxs), ptr(unv), self.stream()))
        return (keys, sums, maxs, unv) if with_parts else keys

    def to_words(self, perms, n: int | None = None):
        """uint8 [C][ld] rows -> int32 [ceil(n/4)][C] word-interleaved layout."""
        torch = _torch()
        C, ld = perms.shape
        n = ld if n is None else int(n)
        words = torch.empty(((n + 3) // 4, C), dtype=torch.int32, device=self.dev)
        check(self.lib.vrpms_rows_to_words(self._ctx, perms.data_ptr(), C, n, ld,
                                           words.data_ptr(), self.stream()))
        return words

    def eval_words(self, words, n: int, with_parts: bool = False, out=None):
        """Score tours in the word-interleaved layout (see vrpms_eval_words)."""
        torch = _torch()
        if words.device != self.dev or words.dim() != 2 or not words.is_contiguous():
            raise ValueError("words must be a contiguous 2-D tensor on the context device")
        if words.shape[0] != (int(n) + 3) // 4:
            raise ValueError("words must have ceil(n/4) rows")
        C = words.shape[1]
        keys = out if out is not None else torch.empty(C, dtype=torch.int64, device=self.dev)
        parts = [torch.empty(C, dtype=torch.int32, device=self.dev) for _ in range(3)] \
            if with_parts else [None, None, None]
        ptr = lambda t: t.data_ptr() if t is not None else None  # noqa: E731
        check(self.lib.vrpms_eval_words(self._ctx, words.data_ptr(), C, int(n), keys.data_ptr(),
                                        *[ptr(p) for p in parts], self.stream()))
        return (keys, *parts) if with_parts else keys

    def set_split_mode(self, mode: int):
        """0 = auto (branch-free prefix-ret split when it fits), 2 = branchy."""
        check(self.lib.vrpms_set_option(self._ctx, _lib.OPT_SPLIT_MODE, int(mode)))

    def set_words_kernel(self, gen: int):
        """Path 0 of vrpms_eval: 0 = auto (eval_cvrp_rows2), 1 = eval_cvrp_packed."""
        check(self.lib.vrpms_set_option(self._ctx, _lib.OPT_WORDS_KERNEL, int(gen)))

    def set_sa_route(self, mode: int):
        """0 = auto (O(1) segment pricing on static symmetric instances,
        hour-row walks on hour-indexed ones, else route-local walks for
        windowed SA), 2 = full re-evaluation (sa_kernel), 3 = force the
        route-local walks, 4 = force the hour-row walks (sa_td_kernel)."""
        check(self.lib.vrpms_set_option(self._ctx, _lib.OPT_SA_ROUTE, int(mode)))

    def set_route_wg_per_cu(self, wg: int):
        """sa_route_kernel workgroups per CU: 0 = auto (1 for multi-wavefront
        chains), 1 or 2 force."""
        check(self.lib.vrpms_set_option(self._ctx, _lib.OPT_ROUTE_WG_PER_CU, int(wg)))

    def set_seg_waves(self, w: int):
        """sa_seg_kernel wavefronts per chain: 0 = auto, 1..4 force (A/B)."""
        check(self.lib.vrpms_set_option(self._ctx, _lib.OPT_SEG_WAVES, int(w)))

    def set_aco_construct(self, mode: int):
        """0 = auto (LDS-staged colony weights when they fit), 2 = the L2 path (A/B)."""
        check(self.lib.vrpms_set_option(self._ctx, _lib.OPT_ACO_CONSTRUCT, int(mode)))

    def set_ga_fused(self, mode: int):
        """0 = auto (fused one-workgroup-per-island GA when it fits), 2 = three kernels."""
        check(self.lib.vrpms_set_option(self._ctx, _lib.OPT_GA_FUSED, int(mode)))

    def set_rows_config(self, cfg: int):
        """eval_cvrp_rows2 (CW, ILP): 0 = auto, 1 = (8, 2), 2 = (16, 1),
        3 = (4, 2), 4 = (8, 1), 5 = (4, 1)."""
        check(self.lib.vrpms_set_option(self._ctx, _lib.OPT_ROWS_CONFIG, int(cfg)))

    def set_words_ilp(self, ilp: int):
        """Candidates per lane in eval_cvrp_words2: 0 = auto, 1 or 2 force."""
        check(self.lib.vrpms_set_option(self._ctx, _lib.OPT_WORDS_ILP, int(ilp)))

    def set_words_lookahead(self, la: int):
        """Words of gathers eval_cvrp_words2 keeps in flight: 0 = auto, 1 or 2."""
        check(self.lib.vrpms_set_option(self._ctx, _lib.OPT_WORDS_LOOKAHEAD, int(la)))

    def set_staged_m(self, m: int):
        """Candidates per lane in eval_staged: 0 = auto, 1 or 2 force."""
        check(self.lib.vrpms_set_option(self._ctx, _lib.OPT_STAGED_M, int(m)))

    def eval_path(self, perms) -> int:
        return self.lib.vrpms_eval_path(self._ctx, perm_dtype_bytes(perms), perms.shape[-1],
                                        perms.data_ptr())

    def decode(self, perm, n: int | None = None):
        """Vehicle of each tour position and per-vehicle durations (host lists)."""
        torch = _torch()
        perm = perm.reshape(-1).contiguous()
        n = perm.numel() if n is None else int(n)
        veh = torch.empty(max(n, 1), dtype=torch.int32, device=self.dev)
        dur = torch.empty(self.K, dtype=torch.int32, device=self.dev)
        check(self.lib.vrpms_decode(self._ctx, perm.data_ptr(), perm_dtype_bytes(perm), n,
                                    veh.data_ptr(), dur.data_ptr(), self.stream()))
        return veh[:n].cpu().tolist(), dur.cpu().tolist()

    def argmin(self, keys):
        """(min key, first index) over a key tensor, reduced on the device."""
        torch = _torch()
        out = torch.empty(2, dtype=torch.int64, device=self.dev)
        check(self.lib.vrpms_argmin(self._ctx, keys.data_ptr(), keys.numel(), out.data_ptr(),
                                    self.stream()))
        k, i = out.cpu().tolist()
        return k & ((1 << 64) - 1), i


    # -- search kernels (state lives in caller-owned device tensors) ----------
    def sa_run(self, cur, cur_key, best, best_key, steps: int, inv_t0: float, inv_alpha: float,
               seed: int, step0: int, window: int = 0, window_types: int = 0, moves: int = 64):
        """Advance every chain (rows of the int16 [chains][n] tensor ``cur``);
        window > 0 samples A11 windowed moves of the A12 types
        ``window_types`` (bit t for move type t, 0 = all); ``moves`` per step
        (64 W: W wavefronts per chain)."""
        chains, n = cur.shape
        p = _lib.SaParams(chains, int(steps), float(inv_t0), float(inv_alpha),
                          int(seed) & (2**64 - 1), int(step0), int(window), int(window_types),
                          int(moves))
        check(self.lib.vrpms_sa_run(self._ctx, ctypes.byref(p), cur.data_ptr(),
                                    cur_key.data_ptr(), best.data_ptr(), best_key.data_ptr(), n,
                                    self.stream()))

    def ga_generation(self, pop, keys, generations: int, pmut: float, seed: int, gen0: int):
        """pop int16 [islands][P][n], keys int64 [islands][P] (must score pop)."""
        islands, P, n = pop.shape
        pm = min(int(round(float(pmut) * 2**32)), 2**32 - 1)
        p = _lib.GaParams(islands, P, int(generations), pm, int(seed) & (2**64 - 1), int(gen0))
        check(self.lib.vrpms_ga_generation(self._ctx, ctypes.byref(p), pop.data_ptr(),
                                           keys.data_ptr(), n, self.stream()))

    def aco_init(self, colonies: int, tau0: int):
        torch = _torch()
        tau = torch.empty((colonies, self.N, self.N), dtype=torch.int32, device=self.dev)
        eta = torch.empty((self.N, self.N), dtype=torch.int32, device=self.dev)
        check(self.lib.vrpms_aco_init(self._ctx, colonies, int(tau0), tau.data_ptr(),
                                      eta.data_ptr(), self.stream()))
        return tau, eta

    def aco_iteration(self, tau, eta, ants: int, seed: int, it: int, evap_shift: int = 3,
                      tau_min: int = 1 << 10, tau_max: int = 1 << 30, best_tours=None,
                      best_keys=None, bsf_period: int = 0):
        """One ACO iteration -> (tours, keys, iteration-best (key, ant) per
        colony); `best_tours`/`best_keys` (per colony) are updated in place
        on the device when given; with `bsf_period` > 0 the best-so-far
        deposits on every bsf_period-th iteration."""
        torch = _torch()
        colonies = tau.shape[0]
        n = self.N - 1
        tours = torch.empty((colonies, ants, n), dtype=torch.int16, device=self.dev)
        keys = torch.empty((colonies, ants), dtype=torch.int64, device=self.dev)
        ib = torch.empty((colonies, 2), dtype=torch.int64, device=self.dev)
        p = _lib.AcoParams(colonies, ants, evap_shift, tau_min, tau_max,
                           int(seed) & (2**64 - 1), int(it), int(bsf_period))
        ptr = lambda t: t.data_ptr() if t is not None else None  # noqa: E731
        check(self.lib.vrpms_aco_iteration(self._ctx, ctypes.byref(p), tau.data_ptr(),
                                           eta.data_ptr(), tours.data_ptr(), keys.data_ptr(),
                                           ib.data_ptr(), ptr(best_tours), ptr(best_keys), n,
                                           self.stream()))
        return tours, keys, ib

    def bf_run(self, n: int, rank_begin: int, rank_end: int):
        """(min key, smallest lexicographic rank) over ranks [begin, end)."""
        torch = _torch()
        out = torch.empty(2, dtype=torch.int64, device=self.dev)
        check(self.lib.vrpms_bf_run(self._ctx, int(n), int(rank_begin), int(rank_end),
                                    out.data_ptr(), self.stream()))
        k, r = out.cpu().tolist()
        return k & (2**64 - 1), r & (2**64 - 1)


    def tsp_batch_sa(self, mats, steps: int, inv_t0: float, inv_alpha: float, seed: int):
        """One workgroup per request: mats int32 [R][N][N] on the device ->
        (best tours int16 [R][N-1], best keys int64 [R])."""
        torch = _torch()
        R, N, _ = mats.shape
        tours = torch.empty((R, max(N - 1, 1)), dtype=torch.int16, device=self.dev)
        keys = torch.empty(R, dtype=torch.int64, device=self.dev)
        p = _lib.SaParams(4 * R, int(steps), float(inv_t0), float(inv_alpha),
                          int(seed) & (2**64 - 1), 0, 0)
        check(self.lib.vrpms_tsp_batch_sa(self._ctx, mats.data_ptr(), R, N, ctypes.byref(p),
                                          tours.data_ptr(), keys.data_ptr(), self.stream()))
        return tours, keys

    # -- populations and the island model (pool.hip) ---------------------------
    def random_tours(self, count: int, n: int, seed: int, stream_id: int = 0, ld: int | None = None,
                     dtype=None, n_sep: int = 0):
        """Philox Fisher-Yates permutations of 1..n plus `n_sep` route
        separators (token 0, A10) -- vrpms_random_tours -- as int16 (default)
        or uint8 rows of `ld` elements."""
        torch = _torch()
        dtype = torch.int16 if dtype is None else dtype
        ld = n + n_sep if ld is None else int(ld)
        out = torch.zeros((int(count), ld), dtype=dtype, device=self.dev)
        check(self.lib.vrpms_random_tours(self._ctx, int(count), int(n), int(n_sep), ld,
                                          perm_dtype_bytes(out), int(seed) & (2**64 - 1),
                                          int(stream_id) & 0xFFFFFFFF, out.data_ptr(),
                                          self.stream()))
        return out

    def insert_separators(self, tours, n_sep: int):
        """int16 [count][n] customer tours -> [count][n + n_sep] with A10
        separators at the greedy split's route boundaries (vrpms_insert_separators)."""
        torch = _torch()
        count, n = tours.shape
        out = torch.empty((count, n + int(n_sep)), dtype=torch.int16, device=self.dev)
        check(self.lib.vrpms_insert_separators(self._ctx, tours.contiguous().data_ptr(), count, n,
                                               int(n_sep), out.data_ptr(), self.stream()))
        return out

    def pack_separators(self, tours, n_sep: int):
        """int16 [count][n] customer tours -> [count][n + n_sep]: first-fit
        routes in input order, one separator between consecutive routes
        (vrpms_pack_separators)."""
        torch = _torch()
        count, n = tours.shape
        out = torch.empty((count, n + int(n_sep)), dtype=torch.int16, device=self.dev)
        check(self.lib.vrpms_pack_separators(self._ctx, tours.contiguous().data_ptr(), count, n,
                                             int(n_sep), out.data_ptr(), self.stream()))
        return out

    @staticmethod
    def pool(tours, keys, groups: int = 1):
        """vrpms_pool over an int16 [count][n] (or [g][p][n]) tour tensor and its keys."""
        count = keys.numel()
        n = tours.shape[-1]
        if tours.numel() != count * n or not tours.is_contiguous() or not keys.is_contiguous():
            raise ValueError("pool: tours must be a contiguous [count][n] tensor matching keys")
        return _lib.Pool(tours.data_ptr(), keys.data_ptr(), count, n, int(groups))

    def pool_elites(self, tours, keys, E: int):
        """The E best rows by (key, index) -> (tours [E][n], keys [E])."""
        torch = _torch()
        n = tours.shape[-1]
        t = torch.empty((E, n), dtype=torch.int16, device=self.dev)
        k = torch.empty(E, dtype=torch.int64, device=self.dev)
        p = self.pool(tours, keys)
        check(self.lib.vrpms_pool_elites(self._ctx, ctypes.byref(p), int(E), t.data_ptr(),
                                         k.data_ptr(), self.stream()))
        return t, k

    def pool_inject(self, tours, keys, mode: int, mig_tours, mig_keys, groups: int = 1):
        p = self.pool(tours, keys, groups)
        mt = mig_tours.to(_torch().int16).contiguous()
        mk = mig_keys.contiguous()
        check(self.lib.vrpms_pool_inject(self._ctx, ctypes.byref(p), int(mode), mt.data_ptr(),
                                         mk.data_ptr(), int(mk.numel()), self.stream()))

    def island_msg_bytes(self, E: int, n: int) -> int:
        return int(self.lib.vrpms_island_msg_bytes(int(E), int(n)))

    def island_pack(self, tours, keys, E: int):
        """The E elites as one island message (uint8 device tensor)."""
        torch = _torch()
        n = tours.shape[-1]
        msg = torch.empty(self.island_msg_bytes(E, n), dtype=torch.uint8, device=self.dev)
        p = self.pool(tours, keys)
        check(self.lib.vrpms_island_pack(self._ctx, ctypes.byref(p), int(E), msg.data_ptr(),
                                         self.stream()))
        return msg

    def island_merge(self, msgs, world: int, E: int, n: int):
        """The E best of `world` gathered messages -> (tours [E][n], keys [E])."""
        torch = _torch()
        msgs = msgs.to(self.dev).contiguous()
        t = torch.empty((E, n), dtype=torch.int16, device=self.dev)
        k = torch.empty(E, dtype=torch.int64, device=self.dev)
        check(self.lib.vrpms_island_merge(self._ctx, msgs.data_ptr(), int(world), int(E), int(n),
                                          t.data_ptr(), k.data_ptr(), self.stream()))
        return t, k

    def island_unique_id(self) -> bytes:
        buf = ctypes.create_string_buffer(128)
        check(self.lib.vrpms_island_unique_id(buf))
        return buf.raw

    def island_init(self, unique_id: bytes, rank: int, world: int):
        buf = ctypes.create_string_buffer(bytes(unique_id), 128)
        check(self.lib.vrpms_island_init(self._ctx, buf, int(rank), int(world)))

    def island_world(self) -> int:
        return int(self.lib.vrpms_island_world(self._ctx))

    def set_island_timeout(self, seconds: int):
        """Deadline of vrpms_island_init (VRPMS_OPT_ISLAND_TIMEOUT_S)."""
        check(self.lib.vrpms_set_option(self._ctx, _lib.OPT_ISLAND_TIMEOUT_S, int(seconds)))

    def island_exchange(self, src, dst, mode: int, E: int, groups: int = 1):
        """vrpms_island_exchange: src/dst are (tours, keys) pairs."""
        ps = self.pool(*src)
        pd = self.pool(*dst, groups=groups)
        check(self.lib.vrpms_island_exchange(self._ctx, ctypes.byref(ps), ctypes.byref(pd),
                                             int(mode), int(E), self.stream()))

    def probe_lds_gather(self, slots: int = 101 * 101, iters: int = 4096, blocks: int | None = None,
                         reps: int = 5):
        """Measured random ds_read_b64 gather rate (gathers/s), best of `reps`."""
        torch = _torch()
        blocks = blocks or 2 * 256
        table = torch.randint(0, 2**62, (slots,), dtype=torch.int64, device=self.dev)
        sink = torch.zeros(1, dtype=torch.int64, device=self.dev)
        best = 0.0
        for _ in range(reps + 1):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            check(self.lib.vrpms_probe_lds_gather(self._ctx, table.data_ptr(), slots, iters,
                                                  blocks, sink.data_ptr(), self.stream()))
            e1.record()
            torch.cuda.synchronize(self.dev)
            best = max(best, blocks * 1024 * 4 * iters / (e0.elapsed_time(e1) * 1e-3))
        return best

    def probe_l2_gather(self, slots: int = 24 * 201 * 201, iters: int = 256,
                        blocks: int | None = None, reps: int = 5):
        """Measured random 2-byte global-load gather rate (gathers/s) over an
        L2-resident uint16 table of `slots` entries, best of `reps`."""
        torch = _torch()
        blocks = blocks or 8 * 256 * 4
        table = torch.randint(0, 2**15, (slots,), dtype=torch.int16, device=self.dev)
        sink = torch.zeros(1, dtype=torch.int64, device=self.dev)
        best = 0.0
        for _ in range(reps + 1):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            check(self.lib.vrpms_probe_l2_gather(self._ctx, table.data_ptr(), slots, iters,
                                                 blocks, sink.data_ptr(), self.stream()))
            e1.record()
            torch.cuda.synchronize(self.dev)
            best = max(best, blocks * 256 * 8 * iters / (e0.elapsed_time(e1) * 1e-3))
        return best


def keys_to_u64(keys) -> np.ndarray:
    """int64 tensor of A8 keys -> numpy uint64 (bit-identical view)."""
    return keys.cpu().numpy().view(np.uint64)
