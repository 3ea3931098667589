"""ctypes binding of the C-ABI in include/admm_tomo.h (libadmm_tomo.so, built in-tree).

There is no CPU fallback: if the shared library is missing or fails to load,
importing the operator or solver raises ``AdmmLibraryError``.
"""
from __future__ import annotations

import ctypes as C
import os
import threading

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_NAME = "libadmm_tomo.so"
LIB_PATH = os.path.join(_HERE, LIB_NAME)

ADMM_DTYPE_F32 = 0
ADMM_DTYPE_F64 = 1
ADMM_TV_ISO = 0
ADMM_TV_ANISO = 1
ADMM_FUSE_MIDPOINT = 0
ADMM_FUSE_WEIGHTED = 1
ADMM_BATCH_KEEP_X = 1  # admm_batch.flags: x_ext local rows written only by admm_node_update
ABI_VERSION = 9
ADMM_MASK_KNN = 0
ADMM_MASK_MST = 1
ADMM_MASK_CHAIN = 2
ADMM_Q_ARITHMETIC = 0
ADMM_Q_HARMONIC = 1
MASK_MAX_NODES = 64
NODE_STATS = 6  # mse_sino, |g|^2, TV, quad, img, split-Bregman stationarity residual^2
EDGE_STATS = 3  # |x_a-z|^2, |x_b-z|^2, |dz|^2


class AdmmLibraryError(RuntimeError):
    pass


class AdmmError(RuntimeError):
    pass


class Geom(C.Structure):
    _fields_ = [
        ("N", C.c_int32),
        ("n_angles", C.c_int32),
        ("n_det", C.c_int32),
        ("reserved", C.c_int32),
        ("angle_min", C.c_double),
        ("angle_max", C.c_double),
        ("det_min", C.c_double),
        ("det_max", C.c_double),
    ]


class Batch(C.Structure):
    _fields_ = [
        ("V", C.c_int32),
        ("n_xext", C.c_int32),
        ("n_edges", C.c_int32),
        ("tv_iters", C.c_int32),
        ("cg_iters", C.c_int32),
        ("tv_kind", C.c_int32),
        ("rho", C.c_double),
        ("lam", C.c_double),
        ("mu", C.c_double),
        ("x_ext", C.c_void_p),
        ("d", C.c_void_p),
        ("e", C.c_void_p),
        ("atb", C.c_void_p),
        ("dsum", C.c_void_p),
        ("b", C.c_void_p),
        ("phantom", C.c_void_p),
        ("y", C.c_void_p),
        ("z", C.c_void_p),
        ("q", C.c_void_p),
        ("edge_a", C.c_void_p),
        ("edge_b", C.c_void_p),
        ("inc_off", C.c_void_p),
        ("inc_edge", C.c_void_p),
        ("inc_qslot", C.c_void_p),
        ("inc_sign", C.c_void_p),
        ("node_stats", C.c_void_p),
        ("edge_stats", C.c_void_p),
        ("fusion", C.c_int32),
        ("flags", C.c_int32),
        ("y_b", C.c_void_p),
        ("w", C.c_void_p),
        ("x_prev", C.c_void_p),
    ]


# (name, argtypes) of every symbol declared in include/admm_tomo.h
SYMBOLS = {
    "admm_abi_version": [],
    "admm_last_error": [],
    "admm_ctx_create": [C.POINTER(C.c_void_p), C.POINTER(Geom), C.c_int, C.c_int, C.c_int],
    "admm_ctx_create_matrix": [C.POINTER(C.c_void_p), C.c_int, C.c_int, C.c_longlong, C.c_void_p, C.c_void_p,
                               C.c_void_p, C.c_int, C.c_int, C.c_int],
    "admm_ctx_destroy": [C.c_void_p],
    "admm_project_fwd": [C.c_void_p, C.c_void_p, C.c_void_p, C.c_int, C.c_void_p],
    "admm_project_adj": [C.c_void_p, C.c_void_p, C.c_void_p, C.c_int, C.c_void_p],
    "admm_column_norms_sq": [C.c_void_p, C.c_void_p, C.c_void_p],
    "admm_tv_grad": [C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, C.c_int, C.c_void_p],
    "admm_tv_div": [C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, C.c_int, C.c_void_p],
    "admm_batch_bind": [C.c_void_p, C.POINTER(Batch)],
    "admm_batch_atb": [C.c_void_p, C.c_void_p, C.c_void_p],
    "admm_node_update": [C.c_void_p, C.c_void_p],
    "admm_node_update_rounds": [C.c_void_p, C.c_int, C.c_void_p],
    "admm_consensus": [C.c_void_p, C.c_void_p],
    "admm_time_forward": [C.c_void_p, C.c_int, C.c_int, C.c_void_p, C.POINTER(C.c_double)],
    "admm_batch_info": [C.c_void_p, C.POINTER(C.c_int), C.POINTER(C.c_int)],
    "admm_time_back": [C.c_void_p, C.c_void_p, C.POINTER(C.c_double)],
    "admm_consensus_range": [C.c_void_p, C.c_int, C.c_int, C.c_int, C.c_void_p],
    "admm_fwd_plan_info": [C.c_void_p, C.c_int, C.POINTER(C.c_int), C.POINTER(C.c_int),
                           C.POINTER(C.c_double), C.POINTER(C.c_int)],
    "admm_pixel_masks": [C.c_void_p, C.c_int, C.c_int64, C.c_int, C.c_int, C.c_int, C.c_void_p,
                         C.c_void_p, C.c_void_p],
    "admm_chain_orders": [C.POINTER(C.c_uint64), C.c_int, C.c_uint32, C.c_int, C.c_int64, C.c_void_p,
                          C.POINTER(C.c_uint64)],
}

_lock = threading.Lock()
_lib = None


def load(path: str | None = None):
    """Load libadmm_tomo.so (raises AdmmLibraryError if absent)."""
    global _lib
    with _lock:
        if _lib is not None and path is None:
            return _lib
        p = path or os.environ.get("ADMM_TOMO_LIB") or LIB_PATH
        if not os.path.exists(p):
            raise AdmmLibraryError(
                f"{p} not found: build the HIP extension first "
                "(python -c 'import __graft_entry__ as g; g.build()')")
        try:
            lib = C.CDLL(p, mode=C.RTLD_GLOBAL)
        except OSError as exc:  # pragma: no cover - depends on the box
            raise AdmmLibraryError(f"cannot load {p}: {exc}") from exc
        for name, args in SYMBOLS.items():
            fn = getattr(lib, name)
            fn.argtypes = args
            fn.restype = C.c_char_p if name == "admm_last_error" else C.c_int
        if lib.admm_abi_version() != ABI_VERSION:
            raise AdmmLibraryError("ABI version mismatch")
        if path is None:
            _lib = lib
        return lib


def check(rc: int, what: str) -> None:
    if rc != 0:
        msg = load().admm_last_error().decode(errors="replace")
        raise AdmmError(f"{what} failed (rc={rc}): {msg}")
