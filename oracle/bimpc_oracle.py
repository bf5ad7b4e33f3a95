"""CPU ORACLE for the BiMPC planner (bimpc.py) — TEST INFRASTRUCTURE ONLY.

Only ``tests/`` may import this module, and only as the checker.

``BiMPCLiteral`` restates bimpc.py:182-265 term by term as torch (CPU, fp64)
expressions in the reference's own variables (w_hat_s, w_hat_l, u_g as P x N /
N arrays, Mp @ W products, A = tril(1)).  Autograd of those literal expressions
gives the objective gradient and the Jacobian of every constraint, independent
of the structured formulas in csrc/lompc_bimpc.cpp.  ``kkt`` certifies a point and
its multipliers (stationarity, primal feasibility, complementarity, dual
feasibility); the problem is strictly convex, so a certified point is THE optimum
Clarabel is asked for.  ``solve_slsqp`` is an independent cross-check for small
instances (scipy SLSQP on the same literal problem).

PARITY UNPINNED by reference artifacts (cvxpy/clarabel absent; the reference's
test_bimpc.py only plots).
"""
from __future__ import annotations

import numpy as np


class BiMPCLiteral:
    def __init__(self, N, P, bi, theta_s, theta_l, w_max_s, w_max_l, params):
        self.N, self.P = N, P
        self.bi = bi  # dict: delta, c_g, u_g_max, u_b_max, x_max, cost_type (0/1/2), exp_rate
        self.theta_s, self.theta_l = theta_s, theta_l
        self.w_max_s, self.w_max_l = w_max_s, w_max_l
        self.p = params  # dict of numpy arrays: Mp_s, Mp_l, beta_s, beta_l, gamma_sm, gamma_lm, x0, demand
        self.n = (2 * P + 1) * N

    def split(self, z):
        N, P = self.N, self.P
        return z[: P * N].reshape(P, N), z[P * N: 2 * P * N].reshape(P, N), z[2 * P * N:]

    def objective_t(self, z):
        """bimpc.py:220-265 (torch)."""
        import torch

        N, P = self.N, self.P
        bi, p = self.bi, self.p
        Ws, Wl, ug = self.split(z)
        A = torch.tril(torch.ones(N, N, dtype=torch.float64))
        Mp_s, Mp_l = torch.as_tensor(p["Mp_s"]), torch.as_tensor(p["Mp_l"])
        gs, gl = torch.as_tensor(p["gamma_sm"]), torch.as_tensor(p["gamma_lm"])
        cost = bi["c_g"] * torch.sum(torch.clamp(ug, min=0.0) ** 1.7)  # cv.power(u_g, 1.7), :221
        ch = 0.0
        if bi["cost_type"] == 0:  # :233-242
            for k in range(P):
                ch = ch + self.theta_s ** 2 * torch.sum((A @ Ws[k] * Mp_s[k] - Mp_s[k] * gs[k]) ** 2)
                ch = ch + self.theta_l ** 2 * torch.sum((A @ Wl[k] * Mp_l[k] - Mp_l[k] * gl[k]) ** 2)
        elif bi["cost_type"] == 1:  # :244-253
            for k in range(P):
                ch = ch + torch.sum((A @ Ws[k] - gs[k]) ** 2) + torch.sum((A @ Wl[k] - gl[k]) ** 2)
        else:  # :255-265
            ew = torch.as_tensor(np.power(bi["exp_rate"], np.arange(-N + 1, 1, 1, dtype=np.float64)))
            for k in range(P):
                ch = ch + ew @ (A @ Ws[k] - gs[k]) ** 2 + ew @ (A @ Wl[k] - gl[k]) ** 2
        return cost + bi["delta"] * ch

    def constraints_t(self, z):
        """All constraints as g(z) <= 0, in the engine's dual order:
        [lower bounds (n) | upper bounds (n) | :201 (N) | :203 (N) | :216 (N) | :218 (N)]."""
        import torch

        N = self.N
        bi, p = self.bi, self.p
        Ws, Wl, ug = self.split(z)
        A = torch.tril(torch.ones(N, N, dtype=torch.float64))
        Mp_s, Mp_l = torch.as_tensor(p["Mp_s"]), torch.as_tensor(p["Mp_l"])
        dem = torch.as_tensor(p["demand"])
        ub = torch.cat([torch.full((self.P * N,), self.w_max_s, dtype=torch.float64),
                        torch.full((self.P * N,), self.w_max_l, dtype=torch.float64),
                        torch.full((N,), bi["u_g_max"], dtype=torch.float64)])
        u_b_hat = ug - dem - self.theta_s * Mp_s @ Ws - self.theta_l * Mp_l @ Wl  # :189-194
        e1 = torch.zeros(N, dtype=torch.float64)
        e1[0] = 1
        d_err = self.theta_s * float(p["Mp_s"] @ p["beta_s"]) + self.theta_l * float(p["Mp_l"] @ p["beta_l"])
        x_hat = A @ u_b_hat + p["x0"] * torch.ones(N, dtype=torch.float64)  # :206-211
        return torch.cat([
            -z, z - ub,
            -(u_b_hat - d_err * e1) - bi["u_b_max"],   # :201
            (u_b_hat + d_err * e1) - bi["u_b_max"],    # :203
            -(x_hat - d_err),                          # :216
            (x_hat + d_err) - bi["x_max"],             # :218
        ])

    def pack(self, Ws, Wl, ug):
        return np.concatenate([np.asarray(Ws).ravel(), np.asarray(Wl).ravel(), np.asarray(ug)])

    def kkt(self, z, lam):
        """(stationarity, primal infeasibility, complementarity, dual infeasibility), each
        relative to the gradient / constraint scale."""
        import torch

        zt = torch.tensor(z, dtype=torch.float64, requires_grad=True)
        f = self.objective_t(zt)
        (g,) = torch.autograd.grad(f, zt)
        J = torch.autograd.functional.jacobian(self.constraints_t, torch.tensor(z, dtype=torch.float64))
        c = self.constraints_t(torch.tensor(z, dtype=torch.float64)).numpy()
        g, J = g.numpy(), J.numpy()
        lam = np.asarray(lam)
        stat = np.max(np.abs(g + J.T @ lam)) / (1.0 + np.max(np.abs(g)))
        infeas = max(0.0, float(np.max(c)))
        comp = float(np.max(np.abs(lam * c))) / (1.0 + abs(float(f.detach())))
        dual_inf = max(0.0, -float(np.min(lam)))
        return stat, infeas, comp, dual_inf

    def objective(self, z):
        import torch

        return float(self.objective_t(torch.tensor(z, dtype=torch.float64)))

    def dense_data(self):
        """(G, h, Hq) from autograd of the literal expressions: constraints G z <= h, and the
        (constant) Hessian of the quadratic charging part."""
        import torch

        n = self.n
        z0 = torch.zeros(n, dtype=torch.float64)
        G = torch.autograd.functional.jacobian(self.constraints_t, z0).numpy()
        h = -self.constraints_t(z0).numpy()
        c_g = self.bi["c_g"]
        self.bi["c_g"] = 0.0
        try:  # quadratic part: its Hessian is constant; evaluate inside the boxes (u > 0)
            Hq = torch.autograd.functional.hessian(self.objective_t, torch.as_tensor(0.5 * h[n:2 * n])).numpy()
        finally:
            self.bi["c_g"] = c_g
        return G, h, Hq

    def solve_ipm(self, tol=1e-11, max_iter=200, trace=None):
        """Dense primal-dual interior point (Mehrotra) on the literal problem — the oracle's
        own BiMPC solver (dense KKT, numpy).  Returns (z, lam, iterations)."""
        import torch

        n, N = self.n, self.N
        G, h, Hq = self.dense_data()
        m = len(h)
        c_g = self.bi["c_g"]
        ub = h[n:2 * n]
        z = 0.5 * ub
        s = h - G @ z
        gz = self._grad(z)
        mu0 = 1.0 + 0.1 * np.max(np.abs(gz)) * np.max(ub)
        s[2 * n:] = np.maximum(s[2 * n:], 0.1 * (1 + np.max(np.abs(h[2 * n:]))))
        lam = mu0 / s
        it = 0
        best = (np.inf, z, lam)
        for it in range(max_iter):
            g = self._grad(z)
            rd = g + G.T @ lam
            rp = G @ z + s - h
            mu = s @ lam / m
            fz = self.objective(z)
            merit = max(np.max(np.abs(rp)) / (1 + np.max(np.abs(h))), np.max(np.abs(rd)) / (1 + np.max(np.abs(g))),
                        s @ lam / (1 + abs(fz)))
            if not np.isfinite(merit):
                break
            if merit < best[0]:
                best = (merit, z.copy(), lam.copy())
            if (np.max(np.abs(rp)) <= 1e-10 * (1 + np.max(np.abs(h))) and np.max(np.abs(rd)) <= tol * (1 + np.max(np.abs(g)))
                    and s @ lam <= tol * (1 + abs(fz))):
                break
            H = Hq.copy()
            u = z[2 * self.P * N:]
            H[2 * self.P * N:, 2 * self.P * N:] += np.diag(1.19 * c_g * u ** -0.3)
            Mx = H + G.T @ (G * (lam / s)[:, None])
            Mx[np.diag_indices(n)] += 1e-15 * (1.0 + np.max(np.abs(Hq)))

            def direction(rc):
                rhs = -rd - G.T @ ((rc + lam * rp) / s)
                dz = np.linalg.solve(Mx, rhs)
                ds = -rp - G @ dz
                dl = (rc - lam * ds) / s
                return dz, ds, dl

            def alpha(ds, dl):
                a = 1.0
                for v, dv in ((s, ds), (lam, dl)):
                    neg = dv < 0
                    if np.any(neg):
                        a = min(a, float(np.min(-v[neg] / dv[neg])))
                return a

            try:
                dz_a, ds_a, dl_a = direction(-s * lam)
            except np.linalg.LinAlgError:
                break
            aa = alpha(ds_a, dl_a)
            mu_aff = (s + aa * ds_a) @ (lam + aa * dl_a) / m
            sigma = min(1.0, mu_aff / mu) ** 3
            dz, ds, dl = direction(sigma * mu - s * lam - ds_a * dl_a)
            a = min(1.0, 0.99 * alpha(ds, dl))
            z, s, lam = z + a * dz, s + a * ds, lam + a * dl
            if trace is not None:
                trace.append((z.copy(), a, sigma))
        if trace is None:  # best iterate (numerically flat directions can stall the last steps)
            z, lam = best[1], best[2]
            zp = self.polish(z, lam, G, h, Hq)
            if zp is not None:
                z, lam = zp
        return z, lam, it

    def polish(self, z, lam, G, h, Hq):
        """Dense active-set polish: rows whose multiplier exceeds their slack become equalities;
        Newton on the equality-constrained KKT system (dense solve); accepted only if primal
        feasible with non-negative multipliers.  Returns (z, lam) or None."""
        n, N = self.n, self.N
        c_g = self.bi["c_g"]
        s = h - G @ z
        act = np.where(lam > s)[0]
        for _outer in range(10):  # active-set corrections: add violated rows, drop wrong-sign ones
            zp = z.copy()
            for _ in range(6):
                Ga = G[act]
                for _ in range(20):
                    g = self._grad(zp)
                    H = Hq.copy()
                    u = zp[2 * self.P * N:]
                    if np.any(u <= 0):
                        return None
                    H[2 * self.P * N:, 2 * self.P * N:] += np.diag(1.19 * c_g * u ** -0.3)
                    K = np.block([[H, Ga.T], [Ga, np.zeros((len(act), len(act)))]])
                    rhs = np.concatenate([-g, h[act] - Ga @ zp])
                    try:
                        sol = np.linalg.solve(K, rhs)
                    except np.linalg.LinAlgError:
                        sol = np.linalg.lstsq(K, rhs, rcond=1e-14)[0]
                    dz, nu = sol[:n], sol[n:]
                    zp = zp + dz
                    if np.max(np.abs(dz)) <= 1e-15:
                        break
                viol = np.setdiff1d(np.where(G @ zp - h > 1e-12 * (1 + np.abs(h)))[0], act)
                if len(viol) == 0:
                    break
                act = np.union1d(act, viol)
            if np.any(G @ zp - h > 1e-12 * (1 + np.abs(h))):
                return None
            g = self._grad(zp)
            neg = nu < -1e-9 * (1 + np.max(np.abs(g)))
            if not np.any(neg):
                break
            act = act[~neg]
        else:
            return None
        lam_p = np.zeros(len(h))
        lam_p[act] = np.maximum(nu, 0.0)
        if np.max(np.abs(g + G.T @ lam_p)) > 1e-8 * (1 + np.max(np.abs(g))):
            return None
        return zp, lam_p

    def _grad(self, z):
        import torch

        zt = torch.tensor(z, dtype=torch.float64, requires_grad=True)
        (g,) = torch.autograd.grad(self.objective_t(zt), zt)
        return g.numpy()

    def solve_slsqp(self, z0=None):
        """Independent cross-check (small instances): scipy SLSQP on the literal problem."""
        import torch
        from scipy.optimize import minimize

        n = self.n
        lo = np.zeros(n)
        hi = -self.constraints_t(torch.zeros(n, dtype=torch.float64)).numpy()[n:2 * n]
        zt0 = torch.zeros(n, dtype=torch.float64)
        Jg = torch.autograd.functional.jacobian(self.constraints_t, zt0).numpy()[2 * n:]
        cg = self.constraints_t(zt0).numpy()[2 * n:]

        def fun(z):
            zt = torch.tensor(z, dtype=torch.float64, requires_grad=True)
            f = self.objective_t(zt)
            (g,) = torch.autograd.grad(f, zt)
            return float(f), g.numpy()

        x0 = 0.5 * hi if z0 is None else z0
        res = minimize(fun, x0, jac=True, method="SLSQP", bounds=list(zip(lo, hi)),
                       constraints=[{"type": "ineq", "fun": lambda z: -(Jg @ z + cg), "jac": lambda z: -Jg}],
                       options={"ftol": 1e-15, "maxiter": 2000})
        return res.x, res
