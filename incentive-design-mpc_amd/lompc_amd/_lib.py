"""ctypes binding of the C-ABI in ``include/lompc_amd.h``.

The shared library ``liblompc_amd.so`` is built in-tree (``lompc_amd.build``)
from ``csrc/lompc_kernels.hip`` with ``hipcc --offload-arch=gfx950``.  There is
no CPU fallback: if the library is missing or no HIP device is visible, every
entry point raises ``RuntimeError``.
"""
from __future__ import annotations

import ctypes
import os
import threading

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, "liblompc_amd.so")
# diagnostics only (scripts/ sweeps of compile-time variants): another in-tree build of the same C-ABI
if os.environ.get("LOMPC_LIB"):
    LIB_PATH = os.path.join(_HERE, os.path.basename(os.environ["LOMPC_LIB"]))

# status codes (include/lompc_amd.h)
LOMPC_OK = 0
LOMPC_ERR_INVALID_ARG = 1
LOMPC_ERR_NOT_CONVERGED = 2
LOMPC_ERR_HIP = 3
LOMPC_ERR_UNSUPPORTED = 4

LOMPC_EV_SMALL = 0
LOMPC_EV_LARGE = 1
LOMPC_MODE_PATH = 0
LOMPC_MODE_DIRECT = 1
LOMPC_PLAN_MAX_CTX = 4
LOMPC_PLAN_K_PATH = 0
LOMPC_PLAN_K_EVAL = 1
LOMPC_PLAN_K_FINAL = 2
LOMPC_PLAN_KERNELS = 3
LOMPC_PLAN_WARM_START = 1
LOMPC_PLAN_DIAG_REPAIR = 2
LOMPC_PLAN_CLOSE_IN_EVAL = 8
LOMPC_PLAN_SORTED_GAMMA = 16
LOMPC_PLAN_CLOSE_IN_FINALIZE = 32
LOMPC_PLAN_CELLS_SHIFT = 20
LOMPC_STEPS_PER_KERNEL = 1
LOMPC_STEPS_SPAN_EVENTS = 2


def LOMPC_PLAN_CELLS(g: int) -> int:
    """flags | LOMPC_PLAN_CELLS(g): g gamma cells per set (include/lompc_amd.h)."""
    return int(g) << LOMPC_PLAN_CELLS_SHIFT


LOMPC_QP_OK = 0
LOMPC_QP_REPAIRED = 1
LOMPC_QP_FAILED = 2
LOMPC_QP_INVALID = 3

LOMPC_STAT_COUNT = 0
LOMPC_STAT_SUM_W0 = 1
LOMPC_STAT_SUM_PRICE0 = 2
LOMPC_STAT_MAX_ERR = 3
LOMPC_STAT_SUM_COST = 4
LOMPC_STAT_N_REPAIRED = 5
LOMPC_STAT_N_FAILED = 6
LOMPC_STAT_N_INVALID = 7
LOMPC_SET_STATS = 8
LOMPC_MAX_N = 64

# (name, restype, argtypes) — must match include/lompc_amd.h exactly.
_P = ctypes.c_void_p
_D = ctypes.c_double
_I = ctypes.c_int
_L = ctypes.c_int64
SIGNATURES = [
    ("lompc_create", _I, [_I, _D, _D, _D, _D, _I, _I, ctypes.POINTER(_P)]),
    ("lompc_destroy", _I, [_P]),
    ("lompc_set_mode", _I, [_P, _I]),
    ("lompc_set_params", _I, [_P, _L, _P, _P, _P, _P, _P]),
    ("lompc_solve_batch", _I, [_P, _L, _P, _P, _P, _P, _P, _P, _P, _P, _P]),
    ("lompc_run", _I, [_P, _L, _P, _P, _P, _P, _L, _P, _P, _P, _P, _P, _P, _P, _P, _P]),
    ("lompc_solve_host", _I, [_P, _P, _D, _D, _P, _P]),
    ("lompc_last_status", _I, [_P, _P, _P, _P, _P]),
    ("lompc_profile_enable", _I, [_P, _I]),
    ("lompc_profile_read", _I, [_P, _P, _P, _I]),
    ("lompc_get_info", _I, [_P, _P, _P]),
    ("lompc_status_string", ctypes.c_char_p, [_I]),
    ("lompc_last_error", ctypes.c_char_p, [_P]),
    ("lompc_abi_version", _I, []),
    ("lompc_price_step", _I, [_I, _I, _D, _D, _D, _D, _D, _P, _P, _P, _P, _P, _P]),
    ("lompc_price_regularize", _I, [_I, _I, _D, _D, _P, _P, _P, _P]),
    ("lompc_lp_separable", _I, [_I, _I, _P, _P, _P, _P]),
    ("lompc_lp_solve", _I, [_I, _I, _P, _P, _P, _P, _P]),
    ("lompc_bimpc_solve", _I, [_I, _I, _I] + [_D] * 10 + [_P] * 6 + [_D] + [_P] * 6),
    ("lompc_plan_create", _I, [_I, _P, _P, _L, _P, _P, _P, _I, _P, ctypes.POINTER(_P)]),
    ("lompc_plan_run", _I, [_P, _P, _P, _P, _P, _P, _P, _P, _P, _P]),
    ("lompc_plan_run_steps", _I, [_P, _P, _L, _P, _L, _I, _I, _P, _P, _P, _P, _P, _P, _L, _L, _L, _I, _P]),
    ("lompc_plan_run_chain", _I, [_P, _P, _P, _P, _D, _I, _P, _P, _P, _P, _P, _P, _P, _P]),
    ("lompc_levels_layout", _I, [_P, _L, _P, _I, _P, _P, _P, _P, ctypes.POINTER(ctypes.c_size_t), _P]),
    ("lompc_levels_gamma", _I, [_P, _L, _P, _I, _D, _I, _P, _P, _P]),
    ("lompc_levels_stats", _I, [_P, _L, _P, _I, _P, _P, ctypes.POINTER(ctypes.c_size_t), _P]),
    ("lompc_plan_status", _I, [_P, _P, _P, _P, _P]),
    ("lompc_plan_get_info", _I, [_P, _P, _P, _P, _P, _P]),
    ("lompc_plan_update", _I, [_P, _L, _P, _P, _P, _P]),
    ("lompc_plan_reserve", _I, [_P, _L]),
    ("lompc_price_loop", _I, [_P, _P, _P, _P, _P, _P, _P, _P, _P, _P]),
    ("lompc_price_chain", _I, [_I, _P, _P, _P, _P]),
    ("lompc_plan_profile_enable", _I, [_P, _I]),
    ("lompc_plan_profile_read", _I, [_P, _I, _P, _P, _I]),
    ("lompc_plan_last_error", ctypes.c_char_p, [_P]),
    ("lompc_plan_destroy", _I, [_P]),
    ("lompc_comm_get_unique_id", _I, [_P]),
    ("lompc_comm_create", _I, [_P, _I, _I, _I, ctypes.POINTER(_P)]),
    ("lompc_comm_destroy", _I, [_P]),
    ("lompc_plan_set_comm", _I, [_P, _P]),
    ("lompc_combine_records", _I, [_P, _I, _L, _I, _P, _P, _I, _P]),
]
LOMPC_COMM_ID_BYTES = 128
# lompc_price_loop_args.prof entries
LOMPC_LOOP_PROF_ITERS = 0
LOMPC_LOOP_PROF_WALL = 1
LOMPC_LOOP_PROF_ISSUE = 2
LOMPC_LOOP_PROF_WAIT = 3
LOMPC_LOOP_PROF_GPU = 4
LOMPC_LOOP_PROF_STEP = 5
LOMPC_LOOP_PROF_HOST = 6
LOMPC_LOOP_PROF = 8
LOMPC_LOOP_AHEAD = 2
LOMPC_BIMPC_WEIGHTED = 0
LOMPC_BIMPC_UNWEIGHTED = 1
LOMPC_BIMPC_EXP_UNWEIGHTED = 2
LOMPC_BIMPC_INFO = 5
ABI_VERSION = 5


class PriceLoopArgs(ctypes.Structure):
    """include/lompc_amd.h lompc_price_loop_args."""
    _fields_ = [("N", ctypes.c_int), ("r", ctypes.c_int), ("max_iter", ctypes.c_int), ("tol_avg", ctypes.c_int),
                ("theta", ctypes.c_double), ("w_max", ctypes.c_double), ("m", ctypes.c_double),
                ("kappa", ctypes.c_double), ("eps_reg", ctypes.c_double), ("tol", ctypes.c_double),
                ("n_evs", ctypes.c_double), ("lmbd_r", ctypes.c_double),
                ("A_bar", ctypes.c_void_p), ("w_ref", ctypes.c_void_p), ("dev_in", ctypes.c_void_p),
                ("host_in", ctypes.c_void_p), ("dev_sw", ctypes.c_void_p), ("dev_st", ctypes.c_void_p),
                ("host_sw", ctypes.c_void_p), ("host_st", ctypes.c_void_p), ("prof", ctypes.c_void_p),
                ("device_loop", ctypes.c_int)]

class PriceChainPart(ctypes.Structure):
    """include/lompc_amd.h lompc_price_chain_part."""
    _fields_ = [("plan", ctypes.c_void_p), ("n_evs", ctypes.c_double), ("tol", ctypes.c_double),
                ("w_ref", ctypes.c_void_p), ("dev_sw", ctypes.c_void_p), ("dev_st", ctypes.c_void_p),
                ("lmbd", ctypes.c_void_p), ("w_k", ctypes.c_void_p), ("dec_actual", ctypes.c_void_p),
                ("dec_pred", ctypes.c_void_p), ("iterations", ctypes.c_int), ("calls", ctypes.c_int),
                ("rc", ctypes.c_int), ("pad", ctypes.c_int), ("price_before_reg", ctypes.c_double),
                ("price_after_reg", ctypes.c_double)]


_lock = threading.Lock()
_lib = None


def load(path: str | None = None) -> ctypes.CDLL:
    """Load (once) and type the C-ABI library. Raises RuntimeError if absent."""
    global _lib
    with _lock:
        if _lib is not None and path is None:
            return _lib
        p = path or LIB_PATH
        if not os.path.exists(p):
            raise RuntimeError(
                f"lompc_amd: HIP extension not built ({p} missing); run "
                "`python -c 'import __graft_entry__ as g; g.build()'` — there is no CPU fallback")
        lib = ctypes.CDLL(p)
        for name, res, args in SIGNATURES:
            fn = getattr(lib, name)
            fn.restype = res
            fn.argtypes = args
        if lib.lompc_abi_version() != ABI_VERSION:
            raise RuntimeError("lompc_amd: ABI version mismatch; rebuild the extension")
        if path is None:
            _lib = lib
        return lib


def status_text(lib, ctx, rc: int, plan=None) -> str:
    msg = lib.lompc_plan_last_error(plan) if plan else (lib.lompc_last_error(ctx) if ctx else b"")
    base = lib.lompc_status_string(rc).decode()
    return f"{base}: {msg.decode()}" if msg else base
