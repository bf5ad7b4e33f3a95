"""Helpers of the batched price iteration (``chargingstation/price_solver.py``).

The reference's per-EV loops (``PriceSolver._get_w_err``, price_solver.py:196-214, and
``PriceSolver.get_w0_price0``, :272-285) are methods of ``lompc_amd.PriceSolver`` here, each one
batched engine call.  This module keeps the stateless pieces: ``solve_sets`` (every
(EV type, partition) parameter set of a time step in one launch), ``set_errors`` (the
price_solver.py:210-214 formulas over fused reductions) and ``structured_abar`` (:191-192).
"""
from __future__ import annotations

import numpy as np

from . import _lib
from .lompc import LoMPC


def structured_abar(A: np.ndarray, delta: float, lmbd_r: float) -> np.ndarray:
    """A_bar = A'A + (lmbd_r/delta) I (price_solver.py:191-192)."""
    kappa = lmbd_r / delta
    return A.T @ A + kappa * np.eye(A.shape[0])


def solve_sets(lompc: LoMPC, lmbd_sets, lmbd_r_sets, gamma, set_offsets, w_ref_sets=None,
               **kw) -> dict:
    """Throughput form: S parameter sets (e.g. all partitions of one EV type)
    and their EVs (set-contiguous) in one launch.  Returns solve_batch's dict."""
    lompc.set_params(lmbd_sets, lmbd_r_sets, w_ref=w_ref_sets)
    return lompc.solve_batch(gamma, set_offsets, **kw)


def set_errors(A_bar: np.ndarray, w_ref_sets: np.ndarray, set_sum_w: np.ndarray, set_stats: np.ndarray):
    """Per-set (w_err_max, w0_err, w_avg_err) from the fused reductions, as
    price_solver.py:210-214 computes them from the loop's accumulators."""
    n = set_stats[:, _lib.LOMPC_STAT_COUNT]
    w_avg = set_sum_w / n[:, None]
    dv = w_avg - w_ref_sets
    w_avg_err = np.sqrt(np.einsum("si,ij,sj->s", dv, A_bar, dv))
    w0_err = np.abs(dv[:, 0])
    return set_stats[:, _lib.LOMPC_STAT_MAX_ERR].copy(), w0_err, w_avg_err
