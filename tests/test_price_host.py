"""CPU tests of the host-side price iteration solvers in the C-ABI library
(no device needed): the price-gradient QP (price_solver.py:216-246) against the
dense numpy/scipy restatement (oracle/price_oracle.py), its KKT certificate, and
the regularizer LP (price_regularizer.py:68-85) against HiGHS, plus the reference
test's own invariants (test_price_regularizer.py:13-14)."""
import ctypes

import numpy as np
import pytest

import lompc_oracle as O
import price_oracle as PO
from lompc_amd import _lib
from lompc_amd.price_regularizer import PriceRegularizer, PriceRegularizerError


def c_price_step(N, r, c, m, kappa, w_ref, w, lmbd, eps=PO.EPS_REG):
    lib = _lib.load()
    out = np.empty(r)
    dec = ctypes.c_double()
    it = ctypes.c_int()
    rc = lib.lompc_price_step(N, r, c.theta, c.w_max, m, kappa, eps, np.ascontiguousarray(w_ref).ctypes.data,
                              np.ascontiguousarray(w).ctypes.data, np.ascontiguousarray(lmbd).ctypes.data,
                              out.ctypes.data, ctypes.byref(dec), ctypes.byref(it))
    assert rc == 0, rc
    return out, dec.value, it.value


def cases(n):
    rng = np.random.default_rng(123)
    for k in range(n):
        ev = "small" if k % 2 == 0 else "large"
        c = O.small_consts() if ev == "small" else O.large_consts()
        N = (12, 24, 48)[k % 3]
        price = ("linear-convex", "linear")[(k // 3) % 2]
        r = 3 * N if price == "linear-convex" else 2 * N
        lmbd_r = 0.0 if k % 4 < 2 else 3 * N * c.delta * rng.random()
        w = c.w_max * rng.random(N)
        w[rng.random(N) < 0.3] = 0.0          # optimal w sits on its bounds often
        w[rng.random(N) < 0.1] = c.w_max
        w_ref = c.w_max * rng.random(N)
        lmbd = c.theta * rng.random(r) * (rng.random(r) < 0.6)
        yield ev, c, N, r, lmbd_r, w, w_ref, lmbd


@pytest.mark.parametrize("case", list(cases(24)), ids=lambda c: f"{c[0]}-N{c[2]}-r{c[3]}")
def test_price_step_matches_dense_oracle(case):
    ev, c, N, r, lmbd_r, w, w_ref, lmbd = case
    m = 2 * c.delta * c.theta ** 2
    kappa = lmbd_r / c.delta
    A = np.tril(np.ones((N, N)))
    _, A_bar_inv = O.w_inner_product_metric(A, c.delta, lmbd_r)
    x, dec, _ = c_price_step(N, r, c, m, kappa, w_ref, w, lmbd)
    xo, deco = PO.price_step(N, r, c.theta, c.w_max, m, A_bar_inv, w_ref, w, lmbd)
    P, q, _ = PO.price_qp_data(N, r, c.theta, c.w_max, m, A_bar_inv, w_ref, w, lmbd)
    scale = 1.0 + np.max(np.abs(q))
    # the engine's answer is a KKT point of the reference's own (dense) problem
    assert PO.price_qp_kkt(P, q, x) <= 1e-9 * scale
    # unique optimum (P > 0): both solvers agree
    np.testing.assert_allclose(x, xo, rtol=0, atol=1e-8 * (1 + np.max(np.abs(xo))))
    assert abs(dec - deco) <= 1e-8 * max(1.0, abs(deco))
    assert dec >= -1e-9 * max(1.0, abs(deco))  # a descent step never increases the majorizer


def test_price_step_fixed_point():
    """At the minimiser the step returns its input and zero decrease."""
    c = O.large_consts()
    N, r = 12, 36
    rng = np.random.default_rng(4)
    w = c.w_max * rng.random(N)
    w_ref = c.w_max * rng.random(N)
    m = 2 * c.delta * c.theta ** 2
    x1, _, _ = c_price_step(N, r, c, m, 0.0, w_ref, w, np.zeros(r))
    # q depends on lmbd only through -2P lmbd, so the minimiser for lmbd = x1 is x1 + argmin at 0 ...
    # but for w == w_ref, phi - phi_ref = 0 and the step keeps any lmbd >= 0 fixed
    lm = c.theta * rng.random(r)
    x2, dec2, _ = c_price_step(N, r, c, m, 0.0, w, w, lm)
    np.testing.assert_allclose(x2, lm, rtol=0, atol=1e-10)
    assert abs(dec2) <= 1e-9
    assert np.all(x1 >= 0)


def test_price_step_rejects_bad_args():
    lib = _lib.load()
    z = np.zeros(36)
    assert lib.lompc_price_step(12, 30, 10.0, 0.25, 10.0, 0.0, 0.01, z.ctypes.data, z.ctypes.data, z.ctypes.data,
                                z.ctypes.data, None, None) == _lib.LOMPC_ERR_INVALID_ARG
    assert lib.lompc_price_step(12, 36, 10.0, 0.25, 10.0, -1.0, 0.01, z.ctypes.data, z.ctypes.data,
                                z.ctypes.data, z.ctypes.data, None, None) == _lib.LOMPC_ERR_INVALID_ARG


@pytest.mark.parametrize("price", ["linear-convex", "linear"])
@pytest.mark.parametrize("ev", ["small", "large"])
def test_regularizer_matches_highs_value(ev, price):
    """price_solver.py:248-255: same optimal value as HiGHS, feasible, and the same
    vertex wherever the LP optimum is unique (w_j > 0)."""
    rng = np.random.default_rng(9 + (ev == "large") + 2 * (price == "linear"))
    c = O.small_consts() if ev == "small" else O.large_consts()
    for N in (12, 24, 48):
        r = 3 * N if price == "linear-convex" else 2 * N
        reg = PriceRegularizer(N, r)
        for _ in range(5):
            w = c.w_max * rng.random(N)
            w[rng.random(N) < 0.25] = 0.0
            lmbd = c.theta * rng.random(r) * (rng.random(r) < 0.7)
            D = PO.Dphi(N, c.theta, c.w_max, w)[:r, :]
            ph = PO.phi(N, c.theta, c.w_max, w)[:r]
            b = D.T @ lmbd
            x = reg.solve_price_regularization(D.T, b, ph)
            xh, val = PO.lp_highs(D.T, b, ph)
            assert np.all(x >= 0)
            np.testing.assert_allclose(D.T @ x, b, rtol=1e-12, atol=1e-10)
            assert abs(ph @ x - val) <= 1e-9 * max(1.0, abs(val))
            assert ph @ x <= ph @ lmbd + 1e-9  # never raises the total price (price_regularizer.py:10-18)
            uniq = np.tile(w > 0, r // N)
            np.testing.assert_allclose(x[uniq], xh[uniq], rtol=1e-9, atol=1e-9)
            np.testing.assert_array_equal(x, PO.lp_vertex_rule(D.T, b, ph))


def test_regularizer_reference_invariants():
    """test_price_regularizer.py:13-24: A = [I, -I], c = 1 -> A x = b and x[:N] . x[N:] = 0."""
    N, r = 12, 24
    rng = np.random.default_rng(0)
    A = np.block([np.eye(N), -np.eye(N)])
    c = np.ones(r)
    reg = PriceRegularizer(N, r)
    for _ in range(1000):
        b = 200 * (rng.random(N) - 0.5)
        x = reg.solve_price_regularization(A, b, c)
        assert np.linalg.norm(A @ x - b) <= 1e-12
        assert x[:N] @ x[N:] == 0.0


def test_regularizer_general_lp_matches_highs():
    """The reference's PriceRegularizer accepts any LP (price_regularizer.py:62-85): dense,
    non-separable instances go to lompc_lp_solve (two-phase simplex) — same optimal value as
    scipy's HiGHS, feasible, non-negative."""
    from scipy.optimize import linprog

    rng = np.random.default_rng(11)
    for trial in range(40):
        m, n = int(rng.integers(2, 20)), int(rng.integers(20, 60))
        A = rng.standard_normal((m, n))
        x0 = rng.random(n) * (rng.random(n) < 0.5)  # a feasible point: b = A x0, x0 >= 0
        b = A @ x0
        c = rng.random(n) + 0.1  # positive costs: bounded
        if trial % 4 == 0:
            A[-1] = A[0]  # a redundant row
            b[-1] = b[0]
        reg = PriceRegularizer(m, n)
        x = reg.solve_price_regularization(A, b, c)
        ref = linprog(c, A_eq=A, b_eq=b, bounds=(0, None), method="highs")
        assert ref.status == 0
        assert np.all(x >= 0.0)
        np.testing.assert_allclose(A @ x, b, rtol=0, atol=1e-9 * (1 + np.abs(b).max()))
        assert abs(c @ x - ref.fun) <= 1e-9 * (1 + abs(ref.fun)), (trial, c @ x, ref.fun)


def test_regularizer_general_lp_infeasible_and_unbounded():
    reg = PriceRegularizer(2, 3)
    A = np.array([[1.0, 1.0, 0.0], [1.0, 1.0, 0.0]])
    with pytest.raises(PriceRegularizerError):  # x1 + x2 = 1 and = 2
        reg.solve_price_regularization(A, np.array([1.0, 2.0]), np.ones(3))
    A = np.array([[1.0, -1.0, 0.0], [0.0, 0.0, 1.0]])
    with pytest.raises(PriceRegularizerError):  # x1 - x2 = 1 with cost -x1: unbounded
        reg.solve_price_regularization(A, np.array([1.0, 1.0]), np.array([-1.0, 0.0, 1.0]))


def test_regularizer_rejects_bad_shapes():
    reg = PriceRegularizer(2, 3)
    x = reg.solve_price_regularization(np.ones((2, 3)), np.ones(2), np.ones(3))  # general LP now
    np.testing.assert_allclose(np.ones((2, 3)) @ x, np.ones(2))
    with pytest.raises(ValueError):
        reg.solve_price_regularization(np.ones((3, 3)), np.ones(2), np.ones(3))


@pytest.mark.parametrize("price", ["linear-convex", "linear"])
@pytest.mark.parametrize("ev", ["small", "large"])
def test_price_regularize_matches_regularizer(ev, price):
    """lompc_price_regularize (the regularisation step of price_solver.py:142-147 with :248-255, shared
    by the price chain and PriceSolver's per-partition loop): lmbd[:r] the regularizer LP's solution
    for A = Dphi(w)', b = A lmbd, c = phi(w) (the same vertex as PriceRegularizer), lmbd[r:] untouched,
    and phi(w)' lmbd before / after within rounding of the numpy products."""
    rng = np.random.default_rng(31 + (ev == "large") + 2 * (price == "linear"))
    c = O.small_consts() if ev == "small" else O.large_consts()
    lib = _lib.load()
    for N in (12, 24, 48):
        r = 3 * N if price == "linear-convex" else 2 * N
        reg = PriceRegularizer(N, r)
        for _ in range(5):
            w = c.w_max * rng.random(N)
            w[rng.random(N) < 0.25] = 0.0
            lm = np.zeros(3 * N)
            lm[:r] = c.theta * rng.random(r) * (rng.random(r) < 0.7)
            ph = PO.phi(N, c.theta, c.w_max, w)
            D = PO.Dphi(N, c.theta, c.w_max, w)[:r, :]
            x = reg.solve_price_regularization(D.T, D.T @ lm[:r], ph[:r])
            out = lm.copy()
            pre, post = ctypes.c_double(0.0), ctypes.c_double(0.0)
            assert lib.lompc_price_regularize(N, r, float(c.theta), float(c.w_max), w.ctypes.data, out.ctypes.data,
                                              ctypes.byref(pre), ctypes.byref(post)) == _lib.LOMPC_OK
            np.testing.assert_array_equal(out[:r], x)
            np.testing.assert_array_equal(out[r:], lm[r:])
            assert abs(pre.value - ph @ lm) <= 1e-12 * max(1.0, abs(ph @ lm))
            assert abs(post.value - ph @ out) <= 1e-12 * max(1.0, abs(ph @ out))
    w = np.zeros(12)
    assert lib.lompc_price_regularize(12, 30, 1.0, 1.0, w.ctypes.data, np.zeros(36).ctypes.data,
                                      ctypes.byref(ctypes.c_double()), ctypes.byref(ctypes.c_double())) \
        == _lib.LOMPC_ERR_INVALID_ARG


@pytest.mark.parametrize("edge", ["below_zero", "above_w_max"])
def test_price_regularize_w_a_rounding_error_outside_the_box(edge):
    """The loop's final w_k is an unclamped piece aggregate: a coordinate can sit a rounding error
    outside [0, w_max] (w_t = -1e-17 or w_max + 1e-15), which makes one cost entry of phi(w) slightly
    negative.  lompc_price_regularize then takes the general LP (lompc_lp_solve) as
    PriceRegularizer.solve_price_regularization does, instead of failing: same x as the regularizer,
    A x = b, and the optimal value of HiGHS."""
    c = O.large_consts()
    lib = _lib.load()
    rng = np.random.default_rng(77 + (edge == "above_w_max"))
    for N, r in ((12, 36), (48, 144), (24, 48)):
        reg = PriceRegularizer(N, r)
        w = c.w_max * rng.random(N)
        w[3] = -1e-17 if edge == "below_zero" else c.w_max + 1e-15
        lm = np.zeros(3 * N)
        lm[:r] = c.theta * rng.random(r)
        ph = PO.phi(N, c.theta, c.w_max, w)
        assert np.min(ph[:r]) < 0  # (the case: a cost entry below zero)
        D = PO.Dphi(N, c.theta, c.w_max, w)[:r, :]
        x = reg.solve_price_regularization(D.T, D.T @ lm[:r], ph[:r])
        out = lm.copy()
        pre, post = ctypes.c_double(0.0), ctypes.c_double(0.0)
        assert lib.lompc_price_regularize(N, r, float(c.theta), float(c.w_max), w.ctypes.data, out.ctypes.data,
                                          ctypes.byref(pre), ctypes.byref(post)) == _lib.LOMPC_OK
        np.testing.assert_array_equal(out[:r], x)
        assert np.all(out[:r] >= 0)
        np.testing.assert_allclose(D.T @ out[:r], D.T @ lm[:r], rtol=1e-9, atol=1e-9 * c.theta)
        _, best = PO.lp_highs(D.T, D.T @ lm[:r], ph[:r])
        assert abs(ph[:r] @ out[:r] - best) <= 1e-9 * max(1.0, abs(best))
        assert abs(post.value - ph @ out) <= 1e-12 * max(1.0, abs(ph @ out))
