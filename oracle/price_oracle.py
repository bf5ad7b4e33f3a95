"""CPU ORACLE for the price iteration around the LoMPC hot path — TEST INFRASTRUCTURE ONLY.

Only ``tests/`` may import this module, and only as the *checker*.

Restates, in dense numpy exactly as the reference builds them (citations are
``chargingstation/<file>:<line>`` in AkshayThiru/incentive-design-mpc @ 2025-10-17):

* ``PriceSolver._price_gradient_descent_step`` price_solver.py:216-246 with its
  CVXPY problem (:257-270): P = Dphi A_bar^-1 Dphi'/(2m) + eps I built with
  ``np.linalg.inv`` / ``np.linalg.cholesky`` like the reference, then
  min ||P_chol x||^2 + q'x, x >= 0 solved as a non-negative least-squares
  problem by ``scipy.optimize.nnls`` (Lawson-Hanson) — an algorithm independent
  of the engine's Woodbury active set.
* ``PriceRegularizer.solve_price_regularization`` price_regularizer.py:68-85 with
  ``scipy.optimize.linprog`` (HiGHS) — the reference uses CVXPY's default LP
  solver (version-dependent, price_regularizer.py:45,83).
* ``PriceSolver.compute_optimal_prices`` price_solver.py:79-174 (the loop, with the
  oracle LoMPC of lompc_oracle.py / oracle_c.py for the per-EV solves).

PARITY UNPINNED by reference artifacts (cvxpy/clarabel absent, no golden data in
the reference); pinned instead by KKT certificates of the
unique optimum of the strictly convex price QP (eps_reg > 0) and by the LP's
optimal value (the LP optimum is not unique when w_j = 0: DESIGN.md).
"""
from __future__ import annotations

import numpy as np

import lompc_oracle as O

EPS_REG = O.PRICE_SOLVER_EPS_REG
MAX_ITERS = 1000  # settings.py:14


def phi(N, theta, w_max, w):
    """lompc.py:172-177."""
    q_s = 3 * theta / (4 * w_max)
    return np.hstack((theta * w, theta * (w_max - w), q_s * (w * w)))


def Dphi(N, theta, w_max, w):
    """lompc.py:179-187."""
    q_s = 3 * theta / (4 * w_max)
    return np.block([[theta * np.eye(N)], [-theta * np.eye(N)], [2 * q_s * np.diag(w)]])


def price_qp_data(N, r, theta, w_max, m, A_bar_inv, w_ref, w, lmbd, eps_reg=EPS_REG):
    """price_solver.py:229-236: (P, q, dual_cost) exactly as the reference forms them."""
    phi_ref = phi(N, theta, w_max, w_ref)[:r]
    ph = phi(N, theta, w_max, w)[:r]
    D = Dphi(N, theta, w_max, w)[:r, :]
    P = 1 / (2 * m) * D @ A_bar_inv @ D.T + eps_reg * np.eye(r)
    q = -2 * P @ lmbd - (ph - phi_ref)
    dual_cost = lmbd @ P @ lmbd + q @ lmbd
    return P, q, dual_cost


def price_step(N, r, theta, w_max, m, A_bar_inv, w_ref, w, lmbd, eps_reg=EPS_REG):
    """price_solver.py:216-246 -> (lmbd_next, dual_cost_decrease).

    min x'Px + q'x = ||L'x + c||^2 - ||c||^2 with P = LL', c = L^-1 q / 2."""
    from scipy.optimize import nnls

    P, q, dual_cost = price_qp_data(N, r, theta, w_max, m, A_bar_inv, w_ref, w, lmbd, eps_reg)
    L = np.linalg.cholesky(P)
    c = np.linalg.solve(L, q) / 2
    x, _ = nnls(L.T, -c, maxiter=50 * r)
    cost_new = x @ P @ x + q @ x
    return x, dual_cost - cost_new


def price_qp_kkt(P, q, x):
    """Max KKT violation of min x'Px + q'x, x >= 0 (gradient mu = 2Px + q)."""
    mu = 2 * P @ x + q
    res = max(0.0, -float(np.min(x)))
    res = max(res, float(np.max(np.where(x > 0, np.abs(mu), np.maximum(0.0, -mu)))))
    return res


def lp_highs(A, b, c):
    """price_regularizer.py:68-85 with HiGHS: (x, optimal value)."""
    from scipy.optimize import linprog

    res = linprog(c, A_eq=A, b_eq=b, bounds=[(0, None)] * len(c), method="highs")
    assert res.status == 0, res.message
    return res.x, float(res.fun)


def regularize(N, r, theta, w_max, w, lmbd):
    """price_solver.py:248-255 via lp_highs."""
    D = Dphi(N, theta, w_max, w)[:r, :]
    return lp_highs(D.T, D.T @ lmbd, phi(N, theta, w_max, w)[:r])


def lp_vertex_rule(A, b, c):
    """The documented tie rule for the degenerate regularizer LP: row by
    row, the cheapest column (cost per unit of |b_j|) whose coefficient has b_j's
    sign, lowest index on ties.  Only meaningful for column-separable A; its optimal
    VALUE is checked against HiGHS (lp_highs) in the tests."""
    A = np.asarray(A, dtype=np.float64)
    x = np.zeros(A.shape[1])
    for j in range(A.shape[0]):
        if b[j] == 0:
            continue
        cols = [i for i in range(A.shape[1]) if A[j, i] != 0 and (A[j, i] > 0) == (b[j] > 0)]
        ratios = [c[i] / abs(A[j, i]) for i in cols]
        i = cols[int(np.argmin(ratios))]
        x[i] = b[j] / A[j, i]
    return x


class OraclePriceSolver:
    """price_solver.py:16-285 on the CPU oracle (small populations only)."""

    def __init__(self, N, consts, price_type, lp=None):
        assert price_type in ("linear", "linear-convex")
        self.lompc = O.OracleLoMPC(N, consts)
        self.N = N
        self.r = 2 * N if price_type == "linear" else 3 * N
        self.consts = consts
        self.prev_prices = np.zeros(self.r)
        self.A = self.lompc.get_input_mat()
        self.m = self.lompc.get_sc_modulus()
        self.lp = lp  # optional LP solver override (A, b, c) -> x
        # oracle_c's warm-started batch (same optima): True = each solve from the previous EV's working
        # set (fast on sorted gamma); "state" = each EV from its own working set of the previous call
        # (fast along a price loop, whose iterations move the prices a little)
        self.warm = False
        self._ws = {}

    def set_charge_levels(self, y0):
        self.nEVs, self.y0_rng, self.gamma_sc, self.gamma_sm = O.set_charge_levels(y0, self.consts.y_max)
        self.y0 = np.asarray(y0, dtype=np.float64)
        self._ws = {}

    def _batch(self, lmbd, lmbd_r):
        import oracle_c

        g = self.consts.y_max - self.y0
        if self.warm == "state":
            w, nf = oracle_c.solve_batch_state(self.N, self.consts, lmbd, lmbd_r, g, self._ws)
        else:
            w, _, nf = oracle_c.solve_batch(self.N, self.consts, lmbd, lmbd_r, g, warm=self.warm)
        assert nf == 0
        return w

    def _get_w_err(self, lmbd, lmbd_r, w_ref, A_bar, want_max=True):
        """price_solver.py:196-214 (vectorised over the oracle batch; want_max=False: w_err_max is not
        computed — the loop tests the average error, settings.py PRICE_SOLVER_TOL_TYPE "avg")."""
        W = self._batch(lmbd, lmbd_r)
        w_err_max = float("nan")
        if want_max:
            dv = W - w_ref
            w_err_max = float(np.max(np.sqrt(np.einsum("bi,bi->b", dv @ A_bar, dv))))
        w_avg = W.sum(axis=0) / self.nEVs
        w_avg_err = np.sqrt((w_avg - w_ref) @ A_bar @ (w_avg - w_ref))
        return w_err_max, np.abs(w_avg[0] - w_ref[0]), w_avg_err

    def compute_optimal_prices(self, w_ref, lmbd_r):
        """price_solver.py:79-174 (PRINT_LEVEL 0; the same array aliasing as the reference)."""
        N, r = self.N, self.r
        th, wm = self.consts.theta, self.consts.w_max
        tol, _ = O.get_robustness_bounds(N, self.consts.delta, self.y0_rng, lmbd_r)
        A_bar, A_bar_inv = O.w_inner_product_metric(self.A, self.consts.delta, lmbd_r)
        lmbd_k, lmbd_k_new = np.zeros(3 * N), np.zeros(3 * N)
        lmbd_k[:r] = self.prev_prices
        phi_w_ref = phi(N, th, wm, w_ref)
        w_k, dual_cost = self.lompc.solve_lompc(lmbd_k, lmbd_r, self.gamma_sc)
        ac, pred = [], []
        for it in range(MAX_ITERS):
            _, _, w_avg_err = self._get_w_err(lmbd_k, lmbd_r, w_ref, A_bar, want_max=False)
            if w_avg_err <= tol:
                break
            lmbd_k_new[:r], dec = price_step(N, r, th, wm, self.m, A_bar_inv, w_ref, w_k, lmbd_k[:r])
            w_k, dual_cost_new = self.lompc.solve_lompc(lmbd_k_new, lmbd_r, self.gamma_sc)
            ac.append(dual_cost_new - dual_cost + (lmbd_k - lmbd_k_new) @ phi_w_ref)
            pred.append(dec)
            dual_cost = dual_cost_new
            lmbd_k = lmbd_k_new
        price_pre = phi(N, th, wm, w_k) @ lmbd_k
        D = Dphi(N, th, wm, w_k)[:r, :]
        c = phi(N, th, wm, w_k)[:r]
        lp = self.lp or lp_vertex_rule
        lmbd_k[:r] = lp(D.T, D.T @ lmbd_k[:r], c)
        price_new = phi(N, th, wm, w_k) @ lmbd_k
        self.prev_prices = lmbd_k[:r]
        stats = {"iter": it, "price_before_reg": price_pre, "price_after_reg": price_new,
                 "dual_cost_decrease_actual": np.array(ac), "dual_cost_decrease_predicted": np.array(pred)}
        return lmbd_k, stats

    def get_w0_price0(self, lmbd, lmbd_r):
        return O.get_w0_price0(self.lompc, self.y0, lmbd, self.r, lmbd_r)

    def get_w0_price0_batch(self, lmbd, lmbd_r):
        """get_w0_price0 (price_solver.py:272-285, lompc.py:164-170) over the C oracle batch: the same
        per-EV optima and price0 formula as lompc_oracle.get_w0_price0, vectorised (large batches)."""
        N, c = self.N, self.consts
        lm = np.zeros(3 * N)
        lm[: self.r] = lmbd
        W = self._batch(lm, lmbd_r)
        w0 = W[:, 0].copy()
        q_scale = 3 * c.theta / (4 * c.w_max)
        price0 = (c.theta * (w0 * lm[0] + (c.w_max - w0) * lm[N]) + q_scale * w0 ** 2 * lm[2 * N]
                  + c.theta ** 2 * w0 ** 2 * lmbd_r)
        return w0, float(price0.sum()) / len(w0)
