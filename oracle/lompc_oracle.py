"""CPU ORACLE for the LoMPC hot path — TEST INFRASTRUCTURE ONLY.

Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline``
leg may import this module, and only as the *checker*.  The product path
(``incentive-design-mpc_amd/``) never imports it and has no CPU fallback.

What it restates (all citations are ``chargingstation/<file>:<line>`` in the
reference, AkshayThiru/incentive-design-mpc @ 2025-10-17):

* ``LoMPC._set_constants``            lompc.py:59-71  (q_scale, A = tril(1), m)
* ``LoMPC`` cost/constraint builders  lompc.py:92-135 (box, degradation,
  charging cost, prices)  -> dense standard form (H, g, c0) + a separable
  convex piecewise-linear term for large EVs.
* ``LoMPC.solve_lompc``               lompc.py:137-156 -> the unique optimum of
  that strictly convex program (the reference asks Clarabel for it; Clarabel
  is un-vendored Rust, absent here, so the oracle computes the same
  mathematical object exactly with a *dense* primal active-set method and
  certifies it by its KKT residual, optionally in mpmath at 50 digits).
* ``LoMPC.get_price0 / phi / Dphi``   lompc.py:164-187
* ``PriceSolver.set_charge_levels``   price_solver.py:66-77
* ``PriceSolver.get_robustness_bounds`` price_solver.py:182-186
* ``PriceSolver._get_w_inner_product_metric`` price_solver.py:188-194
* ``PriceSolver._get_w_err``          price_solver.py:196-214
* ``PriceSolver.get_w0_price0``       price_solver.py:272-285

PARITY UNPINNED by reference artifacts: the reference ships no golden data and
its tests have no assertions; cvxpy/clarabel are not
importable in this container (ModuleNotFoundError, not a permission denial),
so no reference output can be produced here.  The oracle is instead pinned by (1) exact optimality certificates (KKT residual <= 1e-30 relative
in 50-digit arithmetic, ``refine_mp``), (2) known-answer cases
(lambda = 0, gamma = 0 => w = 0), and (3) the reference's own test
invariants (test_lompc.py:54-55, 83-86).

This file deliberately uses the *dense* formulation (explicit N x N Hessian,
``numpy.linalg.solve``) so it shares no algorithmic shortcut with the HIP
kernels (which use an O(N) Riccati recursion).
"""
from __future__ import annotations

import math
from dataclasses import dataclass

import numpy as np

# settings.py:7-9
MIN_MAX_BAT_SOC = 0.75
MAX_MAX_BAT_SOC = 0.9
MAX_BAT_CHARGE_RATE = 0.25
# settings.py:18-19
PRICE_SOLVER_EPS_REG = 0.01
PRICE_SOLVER_EPS_TOL = 0.01

# Large-EV piecewise-linear degradation, lompc.py:108-114:
#   max(0*u, u - 0.125, 1.5u - 0.375, 2u - 0.75),  u = w / w_max
PWL_KNOTS_REL = (0.0, 0.125, 0.5, 0.75, 1.0)
PWL_SLOPES_REL = (0.0, 1.0, 1.5, 2.0)


@dataclass
class OracleConstants:
    """Mirror of ``LoMPCConstants`` (lompc.py:12-26)."""

    delta: float
    theta: float
    y_max: float
    w_max: float
    ev_type: str


def small_consts() -> OracleConstants:
    # real_time_price_control.py:27-31 / test_lompc.py:15-19
    return OracleConstants(0.05, 10.0, 0.9, 0.25, "small")


def large_consts() -> OracleConstants:
    # real_time_price_control.py:33-37 / test_lompc.py:20-24
    return OracleConstants(0.025, 50.0, 0.9, 0.15, "large")


class OracleLoMPC:
    """Dense CPU restatement of ``LoMPC`` (lompc.py:29-187)."""

    def __init__(self, N: int, consts: OracleConstants) -> None:
        # lompc.py:36-38
        assert (consts.y_max >= MIN_MAX_BAT_SOC) and (consts.y_max <= MAX_MAX_BAT_SOC)
        assert (consts.w_max >= 0) and (consts.w_max <= MAX_BAT_CHARGE_RATE)
        assert (consts.ev_type == "small") or (consts.ev_type == "large")
        # lompc.py:59-71
        self.N = int(N)
        self.delta = float(consts.delta)
        self.theta = float(consts.theta)
        self.y_max = float(consts.y_max)
        self.w_max = float(consts.w_max)
        self.ev_type = consts.ev_type
        self.q_scale = 3 * self.theta / (4 * self.w_max)
        self.A = np.tril(np.ones((self.N, self.N)))
        self.m = 2 * self.delta * self.theta ** 2
        # Generalised "knots" of the separable term: box [0, w_max] plus, for
        # large EVs, the kinks of the degradation PWL (lompc.py:108-114).
        if self.ev_type == "small":
            self.knots = np.array([0.0, self.w_max])
            self.slopes = np.array([0.0])
        else:
            self.knots = self.w_max * np.array(PWL_KNOTS_REL)
            scale = (self.theta * self.w_max) ** 2 / self.w_max
            self.slopes = scale * np.array(PWL_SLOPES_REL)

    # ------------------------------------------------------------------ data
    def qp_data(self, lmbd, lmbd_r, gamma):
        """Dense standard form: 0.5 w'Hw + g'w + c0 (+ large-EV PWL).

        Term by term from lompc.py:101-135:
          small degradation  theta^2 ||w/0.9||^2               (:105)
          charging cost      delta theta^2 (||Aw||^2 - 2 gamma 1'Aw)  (:117-122)
          linear prices      theta (l1'w + l2'(w_max - w))      (:126-129)
          quadratic prices   q_scale l3' w^2                    (:131)
          robustness price   lmbd_r theta^2 ||w||^2             (:133)
        """
        N, th, de = self.N, self.theta, self.delta
        lmbd = np.asarray(lmbd, dtype=np.float64)
        l1, l2, l3 = lmbd[:N], lmbd[N:2 * N], lmbd[2 * N:3 * N]
        A = self.A
        H = 2 * de * th ** 2 * (A.T @ A)
        H = H + 2 * lmbd_r * th ** 2 * np.eye(N)
        H = H + 2 * self.q_scale * np.diag(l3)
        if self.ev_type == "small":
            H = H + 2 * th ** 2 / (0.9 ** 2) * np.eye(N)
        g = th * (l1 - l2) - 2 * de * th ** 2 * gamma * (A.T @ np.ones(N))
        c0 = th * self.w_max * np.sum(l2)
        return H, g, c0

    def objective(self, w, lmbd, lmbd_r, gamma) -> float:
        """Literal evaluation of ``self.cost`` (lompc.py:95-135), as
        ``self.cost.value`` does at lompc.py:155."""
        N, th = self.N, self.theta
        w = np.asarray(w, dtype=np.float64)
        lmbd = np.asarray(lmbd, dtype=np.float64)
        cost = 0.0
        if self.ev_type == "small":
            cost += th ** 2 * np.sum((w / 0.9) ** 2)
        else:
            w_rel = w / self.w_max
            pwl = np.sum(np.maximum.reduce([0.0 * w_rel, w_rel - 0.125,
                                            1.5 * w_rel - 0.375, 2 * w_rel - 0.75]))
            cost += (th * self.w_max) ** 2 * pwl
        y = self.A @ w
        cost += self.delta * th ** 2 * (np.sum(y ** 2) - 2 * gamma * np.sum(y))
        l_price = th * (lmbd[:N] @ w + lmbd[N:2 * N] @ (self.w_max - w))
        q_price = self.q_scale * lmbd[2 * N:] @ (w ** 2)
        r_price = lmbd_r * th ** 2 * np.sum(w ** 2)
        cost += l_price + q_price + r_price
        return float(cost)

    # ---------------------------------------------------------------- solver
    def _subproblem(self, H, g, st):
        """Exact minimiser for a working set (dense solve)."""
        free = (st % 2) == 1
        fixed = ~free
        w = np.zeros(self.N)
        w[fixed] = self.knots[st[fixed] // 2]
        if free.any():
            lin = g[free] + self.slopes[(st[free] - 1) // 2]
            rhs = -(lin + H[np.ix_(free, fixed)] @ w[fixed])
            w[free] = np.linalg.solve(H[np.ix_(free, free)], rhs)
        return w

    def solve_state(self, lmbd, lmbd_r, gamma, max_iter=10000):
        """Dense primal active-set method (Nocedal & Wright Alg. 16.3, with
        the PWL kinks as extra 'knots').  Returns (w, state)."""
        self._check(lmbd, lmbd_r, gamma)
        H, g, _ = self.qp_data(lmbd, lmbd_r, gamma)
        N = self.N
        nk = len(self.knots)
        st = np.zeros(N, dtype=np.int64)  # all fixed at knot 0 (w = 0, feasible)
        w = np.zeros(N)
        scale = 1.0 + np.max(np.abs(g)) + np.max(np.abs(H)) * self.w_max * N
        if len(self.slopes):
            scale += np.max(np.abs(self.slopes))
        tol = 1e-12 * scale
        for _ in range(max_iter):
            w_hat = self._subproblem(H, g, st)
            p = w_hat - w
            alpha, blk, blk_knot = 1.0, -1, -1
            for j in range(N):
                if st[j] % 2 == 0:
                    continue
                k = (st[j] - 1) // 2
                if p[j] > 0:
                    a = (self.knots[k + 1] - w[j]) / p[j]
                    kn = k + 1
                elif p[j] < 0:
                    a = (self.knots[k] - w[j]) / p[j]
                    kn = k
                else:
                    continue
                if a < alpha:
                    alpha, blk, blk_knot = a, j, kn
            if blk < 0:
                w = w_hat
                r = H @ w + g
                best, bj, bdir = tol, -1, 0
                for j in range(N):
                    if st[j] % 2 == 1:
                        continue
                    k = st[j] // 2
                    if k < nk - 1:
                        v = -r[j] - self.slopes[k]
                        if v > best:
                            best, bj, bdir = v, j, +1
                    if k > 0:
                        v = r[j] + self.slopes[k - 1]
                        if v > best:
                            best, bj, bdir = v, j, -1
                if bj < 0:
                    return w, st
                st[bj] = st[bj] + bdir  # knot k -> segment k (up) / k-1 (down)
            else:
                alpha = max(alpha, 0.0)
                w = w + alpha * p
                st[blk] = 2 * blk_knot
                w[blk] = self.knots[blk_knot]
        raise RuntimeError("oracle active-set did not terminate")

    def solve_lompc(self, lmbd, lmbd_r, gamma):
        """Restates lompc.py:137-156: returns (w*, cost(w*)) with the full
        objective including c0."""
        w, _ = self.solve_state(lmbd, lmbd_r, gamma)
        return w, self.objective(w, lmbd, lmbd_r, gamma)

    def _check(self, lmbd, lmbd_r, gamma):
        # lompc.py:87 assert; nonneg Parameters lompc.py:78-82
        assert gamma <= self.y_max
        if gamma < 0 or lmbd_r < 0 or np.any(np.asarray(lmbd) < 0):
            raise ValueError("Parameter value must be nonnegative.")
        assert np.asarray(lmbd).shape == (3 * self.N,)

    # ----------------------------------------------------------- certificate
    def kkt_residual(self, w, lmbd, lmbd_r, gamma, knot_tol=1e-12):
        """Relative KKT residual of ``w``: distance of -(Hw+g)_j from the
        subdifferential of the separable term (incl. box normal cone) at w_j,
        plus primal infeasibility.  0 at the exact optimum."""
        H, g, _ = self.qp_data(lmbd, lmbd_r, gamma)
        r = H @ w + g
        scale = 1.0 + np.max(np.abs(g)) + np.max(np.abs(H)) * self.w_max * self.N
        res = 0.0
        for j in range(self.N):
            res = max(res, _coord_residual(w[j], -r[j], self.knots, self.slopes,
                                           knot_tol * self.w_max))
        infeas = max(0.0, -np.min(w), np.max(w) - self.w_max)
        return res / scale, infeas

    # ----------------------------------------------------------- lompc.py API
    def get_sc_modulus(self):
        return self.m

    def get_input_mat(self):
        return self.A

    def get_price0(self, w, lmbd, lmbd_r):
        # lompc.py:164-170
        return (self.theta * (w[0] * lmbd[0] + (self.w_max - w[0]) * lmbd[self.N])
                + self.q_scale * w[0] ** 2 * lmbd[2 * self.N]
                + self.theta ** 2 * w[0] ** 2 * lmbd_r)

    def phi(self, w):
        # lompc.py:172-177
        assert w.shape == (self.N,)
        return np.hstack((self.theta * w, self.theta * (self.w_max - w), self.q_scale * (w * w)))

    def Dphi(self, w):
        # lompc.py:179-187
        assert w.shape == (self.N,)
        return np.block([[self.theta * np.eye(self.N)], [-self.theta * np.eye(self.N)],
                         [2 * self.q_scale * np.diag(w)]])


def _coord_residual(wj, neg_rj, knots, slopes, ktol):
    """Distance of neg_rj from the subdifferential interval at wj."""
    m = len(slopes)
    for k in range(m + 1):
        if abs(wj - knots[k]) <= ktol:
            lo = -math.inf if k == 0 else slopes[k - 1]
            hi = math.inf if k == m else slopes[k]
            if neg_rj < lo:
                return lo - neg_rj
            if neg_rj > hi:
                return neg_rj - hi
            return 0.0
    for k in range(m):
        if knots[k] < wj < knots[k + 1]:
            return abs(neg_rj - slopes[k])
    return math.inf  # outside the box


# --------------------------------------------------------------------------
# 50-digit certificate / refinement
# --------------------------------------------------------------------------
def refine_mp(lompc: OracleLoMPC, st, lmbd, lmbd_r, gamma, dps=50):
    """Solve the working set ``st`` exactly at ``dps`` digits from the fp64
    inputs and certify optimality there.  Returns (w_mp as fp64 array,
    relative KKT residual at dps digits, min strict-interior slack)."""
    import mpmath as mp

    mp.mp.dps = dps
    N = lompc.N
    th, de = mp.mpf(lompc.theta), mp.mpf(lompc.delta)
    wmax = mp.mpf(lompc.w_max)
    lm = [mp.mpf(float(x)) for x in np.asarray(lmbd)]
    lr, ga = mp.mpf(float(lmbd_r)), mp.mpf(float(gamma))
    qs = 3 * th / (4 * wmax)
    # H = 2 de th^2 A'A + diag(...)   (A'A)_{jk} = N - max(j,k)
    H = mp.matrix(N, N)
    for j in range(N):
        for k in range(N):
            H[j, k] = 2 * de * th ** 2 * (N - max(j, k))
        H[j, j] += 2 * lr * th ** 2 + 2 * qs * lm[2 * N + j]
        if lompc.ev_type == "small":
            H[j, j] += 2 * th ** 2 / (mp.mpf(0.9) ** 2)
    g = [th * (lm[j] - lm[N + j]) - 2 * de * th ** 2 * ga * (N - j) for j in range(N)]
    if lompc.ev_type == "small":
        knots = [mp.mpf(0), wmax]
        slopes = [mp.mpf(0)]
    else:
        knots = [wmax * mp.mpf(x) for x in PWL_KNOTS_REL]
        sc = (th * wmax) ** 2 / wmax
        slopes = [sc * mp.mpf(x) for x in PWL_SLOPES_REL]
    st = np.asarray(st)
    free = [j for j in range(N) if st[j] % 2 == 1]
    fixed = [j for j in range(N) if st[j] % 2 == 0]
    w = [mp.mpf(0)] * N
    for j in fixed:
        w[j] = knots[int(st[j]) // 2]
    if free:
        nf = len(free)
        Hff = mp.matrix(nf, nf)
        rhs = mp.matrix(nf, 1)
        for a, j in enumerate(free):
            s = g[j] + slopes[(int(st[j]) - 1) // 2]
            for k in fixed:
                s += H[j, k] * w[k]
            rhs[a] = -s
            for b, k in enumerate(free):
                Hff[a, b] = H[j, k]
        x = mp.lu_solve(Hff, rhs)
        for a, j in enumerate(free):
            w[j] = x[a]
    r = [sum(H[j, k] * w[k] for k in range(N)) + g[j] for j in range(N)]
    scale = 1 + max(abs(x) for x in g) + 2 * de * th ** 2 * N * wmax * N
    res = mp.mpf(0)
    slack = mp.inf
    m = len(slopes)
    for j in range(N):
        if st[j] % 2 == 1:
            k = (int(st[j]) - 1) // 2
            res = max(res, abs(-r[j] - slopes[k]))
            slack = min(slack, (w[j] - knots[k]) / wmax, (knots[k + 1] - w[j]) / wmax)
        else:
            k = int(st[j]) // 2
            lo = None if k == 0 else slopes[k - 1]
            hi = None if k == m else slopes[k]
            v = -r[j]
            if lo is not None:
                res = max(res, lo - v)
                slack = min(slack, (v - lo) / scale)
            if hi is not None:
                res = max(res, v - hi)
                slack = min(slack, (hi - v) / scale)
    w64 = np.array([float(x) for x in w])
    return w64, float(res / scale), float(slack)


# --------------------------------------------------------------------------
# PriceSolver reductions (price_solver.py)
# --------------------------------------------------------------------------
def set_charge_levels(y0, y_max):
    """price_solver.py:66-77 -> (nEVs, y0_rng, gamma_sc, gamma_sm)."""
    y0 = np.asarray(y0, dtype=np.float64)
    assert all(y0 >= 0) and all(y0 <= y_max)
    assert len(y0.shape) == 1
    y0_rng = (np.max(y0) - np.min(y0)) / 2
    gamma_sc = y_max - (np.max(y0) + np.min(y0)) / 2
    gamma_sm = y_max - np.mean(y0)
    return len(y0), y0_rng, gamma_sc, gamma_sm


def get_robustness_bounds(N, delta, y0_rng, lmbd_r, eps_tol=PRICE_SOLVER_EPS_TOL):
    """price_solver.py:182-186."""
    kappa = lmbd_r / delta + 1e-5
    w_err_bound = np.sqrt(N) * y0_rng + eps_tol
    w0_err_bound = w_err_bound * np.min((1, 1 / np.sqrt(kappa)))
    return w_err_bound, w0_err_bound


def w_inner_product_metric(A, delta, lmbd_r):
    """price_solver.py:188-194."""
    kappa = lmbd_r / delta
    A_bar = A.T @ A + kappa * np.eye(A.shape[0])
    return A_bar, np.linalg.inv(A_bar)


def get_w_err(lompc: OracleLoMPC, y0, lmbd, lmbd_r, w_ref, A_bar):
    """price_solver.py:196-214 (sequential per-EV loop)."""
    N = lompc.N
    n = len(y0)
    w_avg = np.zeros(N)
    w_err_max = 0
    gamma = lompc.y_max - np.asarray(y0)
    for i in range(n):
        w_i, _ = lompc.solve_lompc(lmbd, lmbd_r, gamma[i])
        w_avg += w_i
        w_err_i = np.sqrt((w_i - w_ref) @ A_bar @ (w_i - w_ref))
        if w_err_i > w_err_max:
            w_err_max = w_err_i
    w_avg = w_avg / n
    w_avg_err = np.sqrt((w_avg - w_ref) @ A_bar @ (w_avg - w_ref))
    w0_err = np.abs(w_avg[0] - w_ref[0])
    return w_err_max, w0_err, w_avg_err


def get_w0_price0(lompc: OracleLoMPC, y0, lmbd, r, lmbd_r):
    """price_solver.py:272-285."""
    N = lompc.N
    lmbd_ = np.zeros(3 * N)
    lmbd_[:r] = lmbd
    n = len(y0)
    w0 = np.zeros(n)
    price0 = 0
    gamma = lompc.y_max - np.asarray(y0)
    for i in range(n):
        w_i, _ = lompc.solve_lompc(lmbd_, lmbd_r, gamma[i])
        w0[i] = w_i[0]
        price0 += lompc.get_price0(w_i, lmbd_, lmbd_r)
    return w0, price0 / n
