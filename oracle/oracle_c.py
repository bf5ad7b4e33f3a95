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


def build() -> str:
    src = os.path.join(HERE, "lompc_oracle.c")
    if not os.path.exists(SO) or os.path.getmtime(SO) < os.path.getmtime(src):
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
        lib.oracle_max_threads.restype = I
        _lib = lib
    return _lib


def solve_batch(N, consts, lmbd, lmbd_r, gamma, nthreads=0):
    """(B,) gammas against one parameter set -> (w (B,N), cost (B,), nfail)."""
    lib = load()
    lm = np.ascontiguousarray(np.asarray(lmbd, dtype=np.float64))
    g = np.ascontiguousarray(np.asarray(gamma, dtype=np.float64))
    B = g.shape[0]
    w = np.empty((B, N))
    cost = np.empty(B)
    nf = lib.oracle_lompc_solve_batch(int(N), int(consts.ev_type == "small"), consts.delta, consts.theta,
                                      consts.y_max, consts.w_max, lm.ctypes.data, float(lmbd_r), B,
                                      g.ctypes.data, w.ctypes.data, cost.ctypes.data, int(nthreads))
    return w, cost, int(nf)


def max_threads() -> int:
    return int(load().oracle_max_threads())
