"""Batched counterparts of the per-EV loops in ``chargingstation/price_solver.py``.

The reference solves one LoMPC per EV in Python loops:

* ``PriceSolver._get_w_err``   (price_solver.py:196-214, loop :203-209)
* ``PriceSolver.get_w0_price0`` (price_solver.py:272-285, loop :280-283)

``PriceSolverLoops`` keeps those method names, arguments and return values,
and replaces each loop with ONE ``LoMPC.solve_batch`` call whose reductions
(sum of w, max A_bar error, sum of price0) are fused into the kernels.  The
small host-side helpers (``set_charge_levels``, ``get_robustness_bounds``,
``_get_w_inner_product_metric``) are restated verbatim so the object can stand
in for the reference's ``PriceSolver`` in those calls.  The price-QP step and
the regularizer LP (price_solver.py:216-270) are not part of the hot path and
are not provided here.

``solve_sets`` is the throughput form: every (EV type, partition) parameter set
of a time step in one launch.
"""
from __future__ import annotations

import numpy as np

from . import _lib
from .lompc import LoMPC, LoMPCConstants
from .settings import PRICE_SOLVER_EPS_REG, PRICE_SOLVER_EPS_TOL


def _torch():
    import torch

    return torch


def structured_abar(A: np.ndarray, delta: float, lmbd_r: float) -> np.ndarray:
    """A_bar = A'A + (lmbd_r/delta) I (price_solver.py:191-192)."""
    kappa = lmbd_r / delta
    return A.T @ A + kappa * np.eye(A.shape[0])


class PriceSolverLoops:
    """The LoMPC-facing part of ``PriceSolver`` (price_solver.py:16-285)."""

    def __init__(self, N: int, consts: LoMPCConstants, price_type: str, device: int | None = None,
                 mode: str | None = None) -> None:
        assert (price_type == "linear") or (price_type == "linear-convex")  # :24
        self.lompc = LoMPC(N, consts, device=device, mode=mode)
        # price_solver.py:42-64
        self.nEVs = None
        self.N = N
        self.r = 2 * self.N if price_type == "linear" else 3 * self.N
        self.consts = consts
        self.price_type = price_type
        self.y0 = None
        self.y0_rng = None
        self.gamma_sc = None
        self.prev_prices = np.zeros((self.r,))
        self.A = self.lompc.get_input_mat()
        self.eps_reg = PRICE_SOLVER_EPS_REG
        self.eps_tol = PRICE_SOLVER_EPS_TOL
        self.m = self.lompc.get_sc_modulus()
        self._out = {}

    # ------------------------------------------------ price_solver.py helpers
    def set_charge_levels(self, y0: np.ndarray) -> None:
        """price_solver.py:66-77."""
        assert all(y0 >= 0) and all(y0 <= self.consts.y_max)
        assert len(y0.shape) == 1
        self.nEVs = len(y0)
        self.y0 = y0
        self.y0_rng = (np.max(self.y0) - np.min(self.y0)) / 2  # = \bar{\Gamma}
        self.gamma_sc = self.consts.y_max - (np.max(self.y0) + np.min(self.y0)) / 2
        self.gamma_sm = self.consts.y_max - np.mean(self.y0)

    def get_gamma_sc(self) -> float:
        return self.gamma_sc

    def get_gamma_sm(self) -> float:
        return self.gamma_sm

    def get_robustness_bounds(self, lmbd_r: float) -> tuple[float, float]:
        """price_solver.py:182-186."""
        kappa = lmbd_r / self.consts.delta + 1e-5
        w_err_bound = np.sqrt(self.N) * self.y0_rng + self.eps_tol
        w0_err_bound = w_err_bound * np.min((1, 1 / np.sqrt(kappa)))
        return w_err_bound, w0_err_bound

    def _get_w_inner_product_metric(self, lmbd_r: float) -> tuple[np.ndarray, np.ndarray]:
        """price_solver.py:188-194."""
        kappa = lmbd_r / self.consts.delta
        A_bar = self.A.T @ self.A + kappa * np.eye(self.N)
        A_bar_inv = np.linalg.inv(A_bar)
        return A_bar, A_bar_inv

    # ------------------------------------------------------- batched loops
    def _gamma(self):
        torch = _torch()
        y0 = torch.as_tensor(np.asarray(self.y0, dtype=np.float64), device=f"cuda:{self.lompc.device}")
        return self.consts.y_max - y0

    def _get_w_err(self, lmbd: np.ndarray, lmbd_r: float, w_ref: np.ndarray,
                   A_bar: np.ndarray) -> tuple[float, float, float]:
        """price_solver.py:196-214 with the per-EV loop as one batched solve.

        Returns (w_err_max, w0_err, w_avg_err)."""
        N = self.N
        if not np.allclose(A_bar, structured_abar(self.A, self.consts.delta, lmbd_r), rtol=1e-12, atol=1e-12):
            raise ValueError("A_bar must be A'A + (lmbd_r/delta) I (price_solver.py:191-192)")
        w_ref = np.asarray(w_ref, dtype=np.float64)
        self.lompc.set_params(np.asarray(lmbd, dtype=np.float64)[None, :], [lmbd_r], w_ref=w_ref[None, :])
        res = self.lompc.solve_batch(self._gamma(), np.array([0, self.nEVs], dtype=np.int64), want_w=False,
                                     want_cost=False, want_set=True, out=self._out)
        sum_w = res["set_sum_w"][0].cpu().numpy()
        stats = res["set_stats"][0].cpu().numpy()
        w_err_max = float(stats[_lib.LOMPC_STAT_MAX_ERR])
        w_avg = sum_w / self.nEVs
        w_avg_err = np.sqrt((w_avg - w_ref) @ A_bar @ (w_avg - w_ref))
        w0_err = np.abs(w_avg[0] - w_ref[0])
        return w_err_max, w0_err, w_avg_err

    def get_w0_price0(self, lmbd: np.ndarray, lmbd_r: float) -> tuple[np.ndarray, float]:
        """price_solver.py:272-285 with the per-EV loop as one batched solve."""
        lmbd_ = np.zeros((3 * self.N))
        lmbd_[: self.r] = lmbd
        self.lompc.set_params(lmbd_[None, :], [lmbd_r])
        res = self.lompc.solve_batch(self._gamma(), np.array([0, self.nEVs], dtype=np.int64), want_w=False,
                                     want_cost=False, want_w0=True, want_set=True, out=self._out)
        w0 = res["w0"].cpu().numpy().copy()
        stats = res["set_stats"][0].cpu().numpy()
        price0 = float(stats[_lib.LOMPC_STAT_SUM_PRICE0]) / self.nEVs
        return w0, price0


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
