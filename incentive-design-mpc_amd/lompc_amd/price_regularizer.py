"""CVXPY-free ``PriceRegularizer`` (chargingstation/price_regularizer.py:9-85).

The reference solves  min c'x  s.t.  A x = b, x >= 0  with CVXPY's default LP
solver (price_regularizer.py:45,83).  Its only caller passes A = Dphi(w)',
b = Dphi(w)' lmbd, c = phi(w) (price_solver.py:248-255), and every column of
Dphi(w)' has one nonzero (lompc.py:179-187), so the LP separates into one-row
LPs solved in closed form by ``lompc_lp_separable`` in the C-ABI library; any other
LP (the reference's class accepts every A, b, c) goes to ``lompc_lp_solve``, a dense
two-phase simplex.  Same constructor (N, r) and method signature as the reference.
"""
from __future__ import annotations

import numpy as np

from . import _lib


class PriceRegularizerError(Exception):
    """The LP is infeasible or unbounded (the reference would raise SolverError or return
    None from CVXPY)."""


class PriceRegularizer:
    """
    Solves the LP:
    min  c.T @ x,
    s.t. A @ x == b,
         x >= 0.
    When c = phi(w), A = D phi(w).T, and b = D phi(w).T @ lmbd,
    where w = w*(lmbd), the LP minimizes total price without
    affecting the incentive controllability property.
    """

    def __init__(self, N: int, r: int) -> None:
        assert (N >= 0) and (r >= 0)  # price_regularizer.py:26
        self.N = N
        self.r = r
        self._lib = _lib.load()

    def solve_price_regularization(self, A: np.ndarray, b: np.ndarray, c: np.ndarray) -> np.ndarray:
        """price_regularizer.py:68-85: A (N, r), b (N,), c (r,) -> x_opt (r,)."""
        A = np.ascontiguousarray(np.asarray(A, dtype=np.float64))
        b = np.ascontiguousarray(np.asarray(b, dtype=np.float64))
        c = np.ascontiguousarray(np.asarray(c, dtype=np.float64))
        if A.shape != (self.N, self.r) or b.shape != (self.N,) or c.shape != (self.r,):
            raise ValueError("Invalid dimensions for Parameter value.")
        x = np.empty(self.r)
        rc = self._lib.lompc_lp_separable(self.N, self.r, A.ctypes.data, b.ctypes.data, c.ctypes.data,
                                          x.ctypes.data)
        if rc == _lib.LOMPC_ERR_UNSUPPORTED:  # not column-separable: the general LP
            rc = self._lib.lompc_lp_solve(self.N, self.r, A.ctypes.data, b.ctypes.data, c.ctypes.data,
                                          x.ctypes.data, None)
            if rc == _lib.LOMPC_ERR_UNSUPPORTED:
                raise PriceRegularizerError("LP unbounded")
        if rc != _lib.LOMPC_OK:
            raise PriceRegularizerError("LP infeasible: " + _lib.status_text(self._lib, None, rc))
        return x
