"""CPU ORACLE for the closed-loop BiMPC step (charging_station.py) — TEST INFRASTRUCTURE ONLY.

Only ``tests/`` may import this module, and only as the checker.  A numpy restatement
of ``ChargingStation`` (charging_station.py:42-433, PRINT_LEVEL 0) whose
components are the other oracles: ``price_oracle.OraclePriceSolver`` (C-oracle LoMPC
per EV, dense scipy price QP, LP vertex rule) and ``bimpc_oracle.BiMPCLiteral``'s dense
interior point on the literal BiMPC problem.  Same legacy ``np.random`` draws in the
same order as the reference (:95-100, :339-341, :348-350).
"""
from __future__ import annotations

import numpy as np

import bimpc_oracle as BO
import lompc_oracle as O
import price_oracle as PO

MIN_INITIAL_SOC, MAX_INITIAL_SOC, MIN_FULL_CHARGE_FRACTION = 0.3, 0.5, 0.95  # settings.py:27-31


class OracleStation:
    def __init__(self, N_bi, N_lo, M_2, P, demand, bi, cs, cl, price_type, Tf):
        """bi: dict(delta, c_g, u_g_max, u_b_max, x_max, cost_type, exp_rate); cs/cl: OracleConstants."""
        self.N_bi, self.N_lo, self.M_2, self.P, self.demand, self.bi = N_bi, N_lo, M_2, P, demand, bi
        self.cs, self.cl, self.Tf = cs, cl, Tf
        self.r = 2 * N_lo if price_type == "linear" else 3 * N_lo
        self.ps_s = PO.OraclePriceSolver(N_lo, cs, price_type)
        self.ps_l = PO.OraclePriceSolver(N_lo, cl, price_type)
        self.y0_s_rng = np.linspace(MIN_INITIAL_SOC, cs.y_max, P + 1)
        self.y0_l_rng = np.linspace(MIN_INITIAL_SOC, cl.y_max, P + 1)
        self.B = (cs.theta + cl.theta) * M_2
        lo, hi = MIN_INITIAL_SOC, MAX_INITIAL_SOC
        self.y_s = lo + (hi - lo) * np.random.random((M_2,))
        self.y_l = lo + (hi - lo) * np.random.random((M_2,))
        self.x, self.t, self.ncharged_s, self.ncharged_l = 0, 0, 0, 0
        self.idx_s = np.zeros(M_2, dtype=int)
        self.idx_l = np.zeros(M_2, dtype=int)
        self._update_indices()
        self.logs = {k: np.zeros((P, Tf)) for k in ("w_s", "w_l", "w_hat_s", "w_hat_l", "beta_s", "beta_l",
                                                       "gamma_sm", "gamma_lm", "avg_price_s", "avg_price_l",
                                                       "price_red_s", "price_red_l")}
        self.logs.update({k: np.zeros((P, Tf), dtype=int) for k in ("niter_s", "niter_l", "Mp_s", "Mp_l")})
        self.logs.update(u_g=np.zeros(Tf), x=np.zeros(Tf))

    def _update_indices(self):
        for p in range(self.P):
            self.idx_s[(self.y_s >= self.y0_s_rng[p]) & (self.y_s <= self.y0_s_rng[p + 1])] = p
            self.idx_l[(self.y_l >= self.y0_l_rng[p]) & (self.y_l <= self.y0_l_rng[p + 1])] = p

    def step(self):
        P, t = self.P, self.t
        # _get_bimpc_solution (:187-266)
        Mp_s, Mp_l = np.zeros(P, dtype=int), np.zeros(P, dtype=int)
        beta_s, beta_l, g_s, g_l = np.zeros(P), np.zeros(P), np.zeros(P), np.zeros(P)
        for p in range(P):
            for y, idx, ps, Mp, beta, g in ((self.y_s, self.idx_s, self.ps_s, Mp_s, beta_s, g_s),
                                            (self.y_l, self.idx_l, self.ps_l, Mp_l, beta_l, g_l)):
                m = idx == p
                Mp[p] = m.sum()
                if Mp[p] > 0:
                    ps.set_charge_levels(y[m])
                    _, beta[p] = O.get_robustness_bounds(ps.N, ps.consts.delta, ps.y0_rng, 0)
                    g[p] = ps.gamma_sm
        demand = self.demand[t: t + self.N_bi] / self.B
        lit = BO.BiMPCLiteral(self.N_bi, P, self.bi, self.cs.theta, self.cl.theta, self.cs.w_max, self.cl.w_max,
                              dict(Mp_s=Mp_s / self.B, Mp_l=Mp_l / self.B, beta_s=beta_s, beta_l=beta_l,
                                   gamma_sm=g_s, gamma_lm=g_l, x0=self.x, demand=demand))
        z, _, _ = lit.solve_ipm()
        w_hat_s, w_hat_l, u_g = lit.split(z)
        # _get_optimal_prices (:268-308)
        prices = {"s": np.zeros((P, self.r)), "l": np.zeros((P, self.r))}
        for p in range(P):
            for k, y, idx, ps, w_hat in (("s", self.y_s, self.idx_s, self.ps_s, w_hat_s),
                                         ("l", self.y_l, self.idx_l, self.ps_l, w_hat_l)):
                y0p = y[idx == p]
                if len(y0p) > 0:
                    ps.set_charge_levels(y0p)
                    lm, st = ps.compute_optimal_prices(w_hat[p, : self.N_lo], 0)
                    prices[k][p] = lm[: self.r]
                    self.logs["niter_" + k][p, t] = st["iter"]
                    self.logs["price_red_" + k][p, t] = st["price_after_reg"] - st["price_before_reg"]
                else:
                    self.logs["niter_" + k][p, t] = -1
                    self.logs["price_red_" + k][p, t] = np.nan
        # _get_w0_price0 (:310-329)
        w0 = {"s": np.zeros(self.M_2), "l": np.zeros(self.M_2)}
        for p in range(P):
            for k, y, idx, ps in (("s", self.y_s, self.idx_s, self.ps_s), ("l", self.y_l, self.idx_l, self.ps_l)):
                m = idx == p
                if m.sum() > 0:
                    ps.set_charge_levels(y[m])
                    w0[k][m], self.logs["avg_price_" + k][p, t] = ps.get_w0_price0(prices[k][p], 0)
                    self.logs["w_" + k][p, t] = np.mean(w0[k][m])
        self.logs["w_hat_s"][:, t], self.logs["w_hat_l"][:, t], self.logs["u_g"][t] = w_hat_s[:, 0], w_hat_l[:, 0], u_g[0]
        for k, v in (("beta_s", beta_s), ("beta_l", beta_l), ("gamma_sm", g_s), ("gamma_lm", g_l), ("Mp_s", Mp_s),
                     ("Mp_l", Mp_l)):
            self.logs[k][:, t] = v
        self.logs["x"][t] = self.x  # _update_logs runs before _update_state (:181-183)
        # _update_state (:331-370), ADD_RESIDUAL_CHARGE_TO_BATTERY = False
        lo, hi = MIN_INITIAL_SOC, MAX_INITIAL_SOC
        self.y_s += w0["s"]
        ms = self.y_s > MIN_FULL_CHARGE_FRACTION * self.cs.y_max
        self.y_s[ms] = lo + (hi - lo) * np.random.random((ms.sum(),))
        self.ncharged_s += ms.sum()
        self.y_l += w0["l"]
        ml = self.y_l > MIN_FULL_CHARGE_FRACTION * self.cl.y_max
        self.y_l[ml] = lo + (hi - lo) * np.random.random((ml.sum(),))
        self.ncharged_l += ml.sum()
        self._update_indices()
        u0_b = u_g[0] + (-self.cs.theta * np.sum(w0["s"]) - self.cl.theta * np.sum(w0["l"]) - self.demand[t]) / self.B
        self.x += u0_b
        self.t += 1
