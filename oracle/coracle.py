"""ctypes wrapper of liboracle.so (the C restatement) -- TEST INFRASTRUCTURE."""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB = os.path.join(HERE, "liboracle.so")
_lib = None


def build(force: bool = False) -> str:
    src = os.path.join(HERE, "oracle_c.c")
    if force or not os.path.exists(LIB) or os.path.getmtime(LIB) < os.path.getmtime(src):
        subprocess.run(["make", "-s", "-B" if force else "-s", "-C", HERE], check=True)
    return LIB


def load():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB):
            build()
        lib = ctypes.CDLL(LIB)
        vp, i32, i64 = ctypes.c_void_p, ctypes.c_int32, ctypes.c_int64
        lib.oracle_eval_batch.restype = ctypes.c_int
        lib.oracle_eval_batch.argtypes = [i32, vp, i32, i32, vp, vp, vp, i32, i32, vp, vp, i64,
                                          i32, i64, vp, vp, vp, vp, i32]
        lib.oracle_max_threads.restype = ctypes.c_int
        f32, u64 = ctypes.c_float, ctypes.c_uint64
        lib.oracle_sa_run.restype = ctypes.c_int
        lib.oracle_sa_run.argtypes = [i32, vp, i32, i32, vp, vp, vp, i32, i32, vp, vp, vp, vp, i32,
                                      i32, i32, f32, f32, u64, u64, i32, ctypes.c_uint32, i32, i32]
        lib.oracle_sa_run_resync.restype = ctypes.c_int
        lib.oracle_sa_run_resync.argtypes = lib.oracle_sa_run.argtypes
        lib.oracle_bf.restype = ctypes.c_int
        lib.oracle_bf.argtypes = [i32, vp, i32, i32, vp, vp, vp, i32, i32, i32, u64, u64, vp, i32]
        lib.oracle_tsp_batch_sa.restype = ctypes.c_int
        lib.oracle_tsp_batch_sa.argtypes = [vp, i32, i32, i32, f32, f32, u64, vp, vp, i32]
        _lib = lib
    return _lib


def _p(a):
    return None if a is None else a.ctypes.data_as(ctypes.c_void_p)


def eval_batch(durations, perms, demand=None, capacities=None, start_times=(0,),
               problem: int = 1, objective: int = 0, n: int | None = None, threads: int = 0):
    """Returns (keys u64, sums, maxs, unv) numpy arrays."""
    lib = load()
    D = np.asarray(durations, dtype=np.int32)
    if D.ndim == 2:
        D = D[None]
    D = np.ascontiguousarray(D)
    H, N = D.shape[0], D.shape[1]
    perms = np.ascontiguousarray(perms)
    C, ld = perms.shape
    n = ld if n is None else n
    st = np.ascontiguousarray(np.asarray(start_times, dtype=np.int32).reshape(-1))
    K = st.shape[0]
    dem = None if demand is None else np.ascontiguousarray(np.asarray(demand, dtype=np.int32))
    cap = None if capacities is None else np.ascontiguousarray(np.asarray(capacities, dtype=np.int32))
    p8 = perms if perms.dtype == np.uint8 else None
    p16 = perms.astype(np.uint16, copy=False) if p8 is None else None
    keys = np.empty(C, dtype=np.uint64)
    sums = np.empty(C, dtype=np.int32)
    maxs = np.empty(C, dtype=np.int32)
    unv = np.empty(C, dtype=np.int32)
    lib.oracle_eval_batch(problem, _p(D), H, N, _p(dem), _p(cap), _p(st), K, objective, _p(p8),
                          _p(p16), C, n, ld, _p(keys), _p(sums), _p(maxs), _p(unv), threads)
    return keys, sums, maxs, unv


def sa_run(durations, cur, best, best_key, steps, inv_t0, inv_alpha, seed, step0,
           demand=None, capacities=None, start_times=(0,), problem: int = 1, objective: int = 0,
           threads: int = 0, window: int = 0, window_types: int = 0, resync: bool = False,
           moves: int = 64):
    """C/OpenMP SA (same streams as vrpms_sa_run); cur/best uint16 [chains][n]
    and best_key uint64 [chains] are updated in place; returns cur_key.
    resync=True prices candidates by oracle_sa_run_resync (walks only what
    the move can change; same keys, same trajectories)."""
    lib = load()
    D = np.ascontiguousarray(np.asarray(durations, dtype=np.int32).reshape(
        (-1,) + np.asarray(durations).shape[-2:]))
    H, N = D.shape[0], D.shape[1]
    st = np.ascontiguousarray(np.asarray(start_times, dtype=np.int32).reshape(-1))
    dem = None if demand is None else np.ascontiguousarray(np.asarray(demand, dtype=np.int32))
    cap = None if capacities is None else np.ascontiguousarray(np.asarray(capacities, dtype=np.int32))
    assert cur.dtype == np.uint16 and best.dtype == np.uint16 and best_key.dtype == np.uint64
    chains, n = cur.shape
    cur_key = np.empty(chains, dtype=np.uint64)
    fn = lib.oracle_sa_run_resync if resync else lib.oracle_sa_run
    fn(problem, _p(D), H, N, _p(dem), _p(cap), _p(st), st.shape[0], objective,
       _p(cur), _p(cur_key), _p(best), _p(best_key), chains, n, int(steps),
       float(inv_t0), float(inv_alpha), int(seed) & (2**64 - 1), int(step0),
       int(window), int(window_types), threads, int(moves))
    return cur_key


def tsp_batch_sa(mats, steps, inv_t0, inv_alpha, seed, threads: int = 0):
    """C/OpenMP restatement of vrpms_tsp_batch_sa (N <= 257): mats int [R][N][N]
    -> (tours uint16 [R][N-1], keys uint64 [R])."""
    lib = load()
    M = np.ascontiguousarray(np.asarray(mats, dtype=np.int32))
    R, N = M.shape[0], M.shape[1]
    assert 2 <= N <= 257
    tours = np.zeros((R, max(N - 1, 1)), dtype=np.uint16)
    keys = np.zeros(R, dtype=np.uint64)
    lib.oracle_tsp_batch_sa(_p(M), R, N, int(steps), float(inv_t0), float(inv_alpha),
                            int(seed) & (2**64 - 1), _p(tours), _p(keys), threads)
    return tours, keys


def bf(durations, n, r0=0, r1=None, demand=None, capacities=None, start_times=(0,),
       problem: int = 1, objective: int = 0, threads: int = 0):
    """C/OpenMP brute force over lexicographic ranks [r0, r1) -> (key, rank)."""
    import math
    lib = load()
    D = np.ascontiguousarray(np.asarray(durations, dtype=np.int32).reshape(
        (-1,) + np.asarray(durations).shape[-2:]))
    st = np.ascontiguousarray(np.asarray(start_times, dtype=np.int32).reshape(-1))
    dem = None if demand is None else np.ascontiguousarray(np.asarray(demand, dtype=np.int32))
    cap = None if capacities is None else np.ascontiguousarray(np.asarray(capacities, dtype=np.int32))
    r1 = math.factorial(n) if r1 is None else r1
    out = np.zeros(2, dtype=np.uint64)
    lib.oracle_bf(problem, _p(D), D.shape[0], D.shape[1], _p(dem), _p(cap), _p(st), st.shape[0],
                  objective, n, int(r0), int(r1), _p(out), threads)
    return int(out[0]), int(out[1])


def max_threads() -> int:
    return load().oracle_max_threads()
