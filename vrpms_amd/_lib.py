"""ctypes binding of ``include/vrpms.h`` (the C-ABI of libvrpms.so).

There is deliberately no CPU fallback: if the HIP library is missing or no
GPU is visible, every compute entry point raises.  ``torch`` is imported
before the library is opened so that libvrpms's ``NEEDED libamdhip64.so.7``
binds to the HIP runtime torch already loaded (same SONAME), giving one HIP
runtime per process and letting torch streams/tensors cross the boundary.
"""
from __future__ import annotations

import ctypes
import os
import threading

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "libvrpms.so")

VRPMS_OK = 0
VRPMS_EINVAL = -1
VRPMS_EHIP = -2
VRPMS_ERANGE = -3
VRPMS_ESTATE = -4
VRPMS_ENOMEM = -5
VRPMS_ETIMEOUT = -6

TSP = 0
CVRP = 1
OPT_SPLIT_MODE = 1
OPT_STAGED_M = 2
OPT_WORDS_KERNEL = 3
OPT_WORDS_ILP = 4
OPT_WORDS_LOOKAHEAD = 5
OPT_ROWS_CONFIG = 6
OPT_GA_FUSED = 7
OPT_SA_ROUTE = 8
OPT_ROUTE_WG_PER_CU = 9
OPT_ISLAND_TIMEOUT_S = 10
OPT_SEG_WAVES = 11
OPT_ACO_CONSTRUCT = 12
OBJ_SUM = 0
OBJ_MAX = 1
INJECT_WORST = 0
INJECT_SORTED = 1
INJECT_BETTER = 2

_c = ctypes
_vp = _c.c_void_p
_i32 = _c.c_int32
_i64 = _c.c_int64
_u64 = _c.c_uint64

class SaParams(ctypes.Structure):
    _fields_ = [("chains", _i32), ("steps", _i32), ("inv_t0", ctypes.c_float),
                ("inv_alpha", ctypes.c_float), ("seed", _u64), ("step0", _u64),
                ("window", _i32), ("window_types", _c.c_uint32), ("moves", _i32)]


class GaParams(ctypes.Structure):
    _fields_ = [("islands", _i32), ("pop", _i32), ("generations", _i32),
                ("pmut", ctypes.c_uint32), ("seed", _u64), ("gen0", _u64)]


class AcoParams(ctypes.Structure):
    _fields_ = [("colonies", _i32), ("ants", _i32), ("evap_shift", _i32),
                ("tau_min", ctypes.c_uint32), ("tau_max", ctypes.c_uint32), ("seed", _u64),
                ("iter", _u64), ("bsf_period", ctypes.c_uint32)]


class Pool(ctypes.Structure):
    _fields_ = [("tours", ctypes.c_void_p), ("keys", ctypes.c_void_p), ("count", _i32),
                ("n", _i32), ("groups", _i32)]


# name -> (restype, argtypes); mirrors include/vrpms.h one-for-one.
SIGNATURES = {
    "vrpms_version": (_c.c_int, []),
    "vrpms_last_error": (_c.c_char_p, []),
    "vrpms_ctx_create": (_c.c_int, [_c.c_int, _c.POINTER(_vp)]),
    "vrpms_ctx_destroy": (_c.c_int, [_vp]),
    "vrpms_set_instance": (_c.c_int, [_vp, _i32, _vp, _i32, _i32, _vp, _vp, _vp, _i32, _i32, _vp]),
    "vrpms_eval": (_c.c_int, [_vp, _vp, _i32, _i64, _i32, _i64, _vp, _vp, _vp, _vp, _vp]),
    "vrpms_eval_path": (_c.c_int, [_vp, _i32, _i64, _vp]),
    "vrpms_eval_words": (_c.c_int, [_vp, _vp, _i64, _i32, _vp, _vp, _vp, _vp, _vp]),
    "vrpms_rows_to_words": (_c.c_int, [_vp, _vp, _i64, _i32, _i64, _vp, _vp]),
    "vrpms_set_option": (_c.c_int, [_vp, _i32, _i32]),
    "vrpms_decode": (_c.c_int, [_vp, _vp, _i32, _i32, _vp, _vp, _vp]),
    "vrpms_argmin": (_c.c_int, [_vp, _vp, _i64, _vp, _vp]),
    "vrpms_sa_run": (_c.c_int, [_vp, _c.POINTER(SaParams), _vp, _vp, _vp, _vp, _i32, _vp]),
    "vrpms_ga_generation": (_c.c_int, [_vp, _c.POINTER(GaParams), _vp, _vp, _i32, _vp]),
    "vrpms_aco_init": (_c.c_int, [_vp, _i32, _c.c_uint32, _vp, _vp, _vp]),
    "vrpms_aco_iteration": (_c.c_int, [_vp, _c.POINTER(AcoParams), _vp, _vp, _vp, _vp, _vp,
                                       _vp, _vp, _i32, _vp]),
    "vrpms_bf_run": (_c.c_int, [_vp, _i32, _u64, _u64, _vp, _vp]),
    "vrpms_probe_lds_gather": (_c.c_int, [_vp, _vp, _i32, _i32, _i32, _vp, _vp]),
    "vrpms_probe_l2_gather": (_c.c_int, [_vp, _vp, _i32, _i32, _i32, _vp, _vp]),
    "vrpms_tsp_batch_sa": (_c.c_int, [_vp, _vp, _i32, _i32, _c.POINTER(SaParams), _vp, _vp,
                                      _vp]),
    "vrpms_random_tours": (_c.c_int, [_vp, _i64, _i32, _i32, _i64, _i32, _u64, _c.c_uint32, _vp,
                                      _vp]),
    "vrpms_insert_separators": (_c.c_int, [_vp, _vp, _i64, _i32, _i32, _vp, _vp]),
    "vrpms_pack_separators": (_c.c_int, [_vp, _vp, _i64, _i32, _i32, _vp, _vp]),
    "vrpms_pool_elites": (_c.c_int, [_vp, _c.POINTER(Pool), _i32, _vp, _vp, _vp]),
    "vrpms_pool_inject": (_c.c_int, [_vp, _c.POINTER(Pool), _i32, _vp, _vp, _i32, _vp]),
    "vrpms_island_msg_bytes": (_i64, [_i32, _i32]),
    "vrpms_island_pack": (_c.c_int, [_vp, _c.POINTER(Pool), _i32, _vp, _vp]),
    "vrpms_island_merge": (_c.c_int, [_vp, _vp, _i32, _i32, _i32, _vp, _vp, _vp]),
    "vrpms_island_unique_id": (_c.c_int, [_vp]),
    "vrpms_island_init": (_c.c_int, [_vp, _vp, _i32, _i32]),
    "vrpms_island_world": (_c.c_int, [_vp]),
    "vrpms_island_exchange": (_c.c_int, [_vp, _c.POINTER(Pool), _c.POINTER(Pool), _i32, _i32,
                                         _vp]),
}


class VrpmsError(RuntimeError):
    """A libvrpms call returned a negative status."""

    def __init__(self, code: int, message: str):
        super().__init__(f"[vrpms {code}] {message}")
        self.code = code


_lock = threading.Lock()
_lib = None


def load(path: str = LIB_PATH):
    """Open libvrpms.so (once) and declare every symbol of include/vrpms.h."""
    global _lib
    with _lock:
        if _lib is not None:
            return _lib
        import torch  # noqa: F401  -- binds libamdhip64.so.7 before our NEEDED entry
        if not os.path.exists(path):
            raise ImportError(
                f"libvrpms.so not found at {path}; build it with "
                "`python -m vrpms_amd.build` (hipcc --offload-arch=gfx950)")
        lib = ctypes.CDLL(path)
        for name, (res, args) in SIGNATURES.items():
            fn = getattr(lib, name)
            fn.restype = res
            fn.argtypes = args
        _lib = lib
        return lib


def check(code: int) -> None:
    if code != VRPMS_OK:
        msg = _lib.vrpms_last_error()
        raise VrpmsError(code, msg.decode() if msg else "unknown error")
