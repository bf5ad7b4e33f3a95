"""ctypes loader for the C oracle (oracle/_build/liboracle_lompc.so).

TEST INFRASTRUCTURE ONLY — used by tests/ and bench.py's cpu_baseline leg.
"""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
SO = os.path.join(HERE, "_build", "liboracle_lompc.so")


SO_PATH = os.path.join(HERE, "_build", "libpath_cpu.so")


def build() -> str:
    srcs = [os.path.join(HERE, f) for f in ("lompc_oracle.c", "path_cpu.cpp", "Makefile")]
    t = max(os.path.getmtime(f) for f in srcs)
    if any(not os.path.exists(x) or os.path.getmtime(x) < t for x in (SO, SO_PATH)):
        subprocess.run(["make", "-s", "-C", HERE], check=True)
    return SO


_lib = None


def load():
    global _lib
    if _lib is None:
        if not os.path.exists(SO):
            build()
        lib = ctypes.CDLL(SO)
        P, D, I, L = ctypes.c_void_p, ctypes.c_double, ctypes.c_int, ctypes.c_int64
        lib.oracle_lompc_solve.restype = I
        lib.oracle_lompc_solve.argtypes = [I, I, D, D, D, D, P, D, D, P, P, P]
        lib.oracle_lompc_solve_batch.restype = L
        lib.oracle_lompc_solve_batch.argtypes = [I, I, D, D, D, D, P, D, L, P, P, P, I]
        lib.oracle_lompc_solve_batch_warm.restype = L
        lib.oracle_lompc_solve_batch_warm.argtypes = [I, I, D, D, D, D, P, D, L, P, P, P, I]
        lib.oracle_lompc_solve_batch_state.restype = L
        lib.oracle_lompc_solve_batch_state.argtypes = [I, I, D, D, D, D, P, D, L, P, P, P, P, P, I]
        lib.oracle_max_threads.restype = I
        _lib = lib
    return _lib


def solve_batch_state(N, consts, lmbd, lmbd_r, gamma, state, nthreads=0):
    """solve_batch with a per-EV working set kept between calls: ``state`` is a dict owned by the
    caller (empty at first); the same optima, each solve started from the EV's previous working set."""
    lib = load()
    lm = np.ascontiguousarray(np.asarray(lmbd, dtype=np.float64))
    g = np.ascontiguousarray(np.asarray(gamma, dtype=np.float64))
    B = g.shape[0]
    if state.get("ws") is None or state["ws"].shape != (B, N):
        state["ws"] = np.zeros((B, N), dtype=np.uint8)
        state["fresh"] = ctypes.c_int(1)
    w = np.empty((B, N))
    nf = lib.oracle_lompc_solve_batch_state(int(N), int(consts.ev_type == "small"), consts.delta, consts.theta,
                                            consts.y_max, consts.w_max, lm.ctypes.data, float(lmbd_r), B,
                                            g.ctypes.data, w.ctypes.data, None, state["ws"].ctypes.data,
                                            ctypes.byref(state["fresh"]), int(nthreads))
    return w, int(nf)


def solve_batch(N, consts, lmbd, lmbd_r, gamma, nthreads=0, warm=False):
    """(B,) gammas against one parameter set -> (w (B,N), cost (B,), nfail).  warm: each thread's
    solves start from its previous solve's working set (oracle_lompc_solve_batch_warm; fast for
    sorted gamma, same optimum)."""
    lib = load()
    fn = lib.oracle_lompc_solve_batch_warm if warm else lib.oracle_lompc_solve_batch
    lm = np.ascontiguousarray(np.asarray(lmbd, dtype=np.float64))
    g = np.ascontiguousarray(np.asarray(gamma, dtype=np.float64))
    B = g.shape[0]
    w = np.empty((B, N))
    cost = np.empty(B)
    nf = fn(int(N), int(consts.ev_type == "small"), consts.delta, consts.theta,
                                      consts.y_max, consts.w_max, lm.ctypes.data, float(lmbd_r), B,
                                      g.ctypes.data, w.ctypes.data, cost.ctypes.data, int(nthreads))
    return w, cost, int(nf)


def max_threads() -> int:
    return int(load().oracle_max_threads())


_plib = None


def load_path():
    global _plib
    if _plib is None:
        if not os.path.exists(SO_PATH):
            build()
        lib = ctypes.CDLL(SO_PATH)
        P, I, L = ctypes.c_void_p, ctypes.c_int, ctypes.c_int64
        lib.path_cpu_run.restype = I
        lib.path_cpu_run.argtypes = [I, I, P, P, P, P, P, L, P, P, I, P, P, P, P, I, P]
        lib.path_cpu_max_threads.restype = I
        _plib = lib
    return _plib


def path_run(N, consts, sets_per_ctx, lmbd, lmbd_r, gamma, set_off, w_ref=None, cells=0, nthreads=0, want_w=True,
             want_cost=True, out=None):
    """The path engine's algorithm on the host (oracle/path_cpu.cpp): B QPs grouped by set (the sets of
    consts[0] first), lmbd (S, 3N), lmbd_r (S,), gamma (B,), set_off (S+1,).  Returns a dict of w (B, N),
    cost (B,), set_sum_w (S, N), set_stats (S, 8) and info (pieces, certified cells, EVs solved
    individually, EVs failed).  ``out``: a previous call's dict, whose buffers are rewritten (a fresh
    50 MB w per call spends its time in first-touch page faults, which serialise the threads)."""
    lib = load_path()
    cs = np.ascontiguousarray(np.array([[c.delta, c.theta, c.y_max, c.w_max, 1.0 if c.ev_type == "small" else 0.0]
                                        for c in consts], dtype=np.float64))
    spc = np.ascontiguousarray(np.asarray(sets_per_ctx, dtype=np.int64))
    lm = np.ascontiguousarray(np.asarray(lmbd, dtype=np.float64))
    lr = np.ascontiguousarray(np.asarray(lmbd_r, dtype=np.float64))
    g = np.ascontiguousarray(np.asarray(gamma, dtype=np.float64))
    off = np.ascontiguousarray(np.asarray(set_off, dtype=np.int64))
    wr = None if w_ref is None else np.ascontiguousarray(np.asarray(w_ref, dtype=np.float64))
    S, B = off.shape[0] - 1, g.shape[0]
    if out is None or out["set_sum_w"].shape != (S, N) or (want_w and (out["w"] is None or out["w"].shape != (B, N))):
        out = {"w": np.empty((B, N)) if want_w else None, "cost": np.empty(B) if want_cost else None,
               "set_sum_w": np.empty((S, N)), "set_stats": np.empty((S, 8))}
    info = np.zeros(4, dtype=np.int64)
    ptr = lambda a: None if a is None else a.ctypes.data
    rc = lib.path_cpu_run(int(N), len(consts), cs.ctypes.data, spc.ctypes.data, lm.ctypes.data, lr.ctypes.data,
                          ptr(wr), B, g.ctypes.data, off.ctypes.data, int(cells), ptr(out["w"]), ptr(out["cost"]),
                          out["set_sum_w"].ctypes.data, out["set_stats"].ctypes.data, int(nthreads), info.ctypes.data)
    if rc:
        raise ValueError(f"path_cpu_run: {rc}")
    out["info"] = info
    return out
