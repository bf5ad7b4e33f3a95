"""CPU tests: the oracle against the committed 50-digit golden vectors and the
reference's own test invariants (chargingstation/test/test_lompc.py)."""
import numpy as np
import pytest

import lompc_oracle as O
import oracle_c
from conftest import oracle_consts

TOL_W = 1e-12  # fp64 oracle vs 50-digit optimum (absolute, w in [0, 0.25])


def test_golden_manifest(golden):
    assert len(golden) == 36
    kinds = {(c["ev_type"], c["N"], c["price"]) for c in golden}
    assert len(kinds) == 18


def test_python_oracle_matches_golden(golden):
    for case in golden[::3]:
        o = O.OracleLoMPC(case["N"], oracle_consts(case))
        for i, g in enumerate(case["gamma"][:6]):
            w, cost = o.solve_lompc(case["lmbd"], case["lmbd_r"], g)
            np.testing.assert_allclose(w, case["w"][i], rtol=0, atol=TOL_W)
            assert abs(cost - case["cost"][i]) <= 1e-10 * max(1.0, abs(case["cost"][i]))


def test_c_oracle_matches_golden(golden):
    for case in golden:
        w, cost, nfail = oracle_c.solve_batch(case["N"], oracle_consts(case), case["lmbd"], case["lmbd_r"],
                                              case["gamma"], nthreads=2)
        assert nfail == 0
        np.testing.assert_allclose(w, case["w"], rtol=0, atol=TOL_W)
        np.testing.assert_allclose(cost, case["cost"], rtol=1e-10, atol=1e-10)


def test_golden_kkt_certificates(golden):
    """Every stored optimum satisfies the KKT conditions in fp64 too."""
    for case in golden:
        o = O.OracleLoMPC(case["N"], oracle_consts(case))
        for i, g in enumerate(case["gamma"]):
            res, infeas = o.kkt_residual(case["w"][i], case["lmbd"], case["lmbd_r"], g, knot_tol=1e-10)
            assert res <= 1e-13 and infeas == 0.0


def test_mp_refinement_certifies_fresh_solve():
    o = O.OracleLoMPC(24, O.large_consts())
    rng = np.random.default_rng(5)
    lmbd = 50 * rng.random(72)
    w, st = o.solve_state(lmbd, 0.7, 0.45)
    wmp, res, _ = O.refine_mp(o, st, lmbd, 0.7, 0.45)
    assert res < 1e-30
    np.testing.assert_allclose(w, wmp, atol=1e-14)


def test_known_answer_zero_price_zero_gamma():
    """lambda = 0, gamma = 0 => w = 0 and cost = 0 (g = 0, H > 0)."""
    for c in (O.small_consts(), O.large_consts()):
        o = O.OracleLoMPC(12, c)
        w, cost = o.solve_lompc(np.zeros(36), 0.0, 0.0)
        assert np.all(w == 0.0) and cost == 0.0


def test_unpriced_response_charges_towards_gamma():
    """test_lompc.py:43-58: with lambda = 0 and gamma = y_max the cumulative
    charge approaches gamma (up to w_max per step)."""
    c = O.small_consts()
    o = O.OracleLoMPC(12, c)
    w, _ = o.solve_lompc(np.zeros(36), 0.0, c.y_max)
    y = np.cumsum(w)
    assert np.all(np.diff(y) >= -1e-15)
    assert y[-1] <= c.y_max + 1e-12 and y[-1] > 0.5 * c.y_max


def test_robustness_bound_invariant():
    """test_lompc.py:61-98: ||w_avg - w_ref||_{A_bar} <= sqrt(N) Gamma_bar."""
    rng = np.random.default_rng(3)
    N = 12
    c = O.small_consts()
    o = O.OracleLoMPC(N, c)
    lmbd = c.theta * rng.random(3 * N)
    kappa = (3 * N) * rng.random() + 1e-5
    lmbd_r = c.delta * kappa
    A_bar = o.A.T @ o.A + kappa * np.eye(N)
    for gmax in (0.9, 0.5, 0.1):
        gam = gmax * rng.random(10)
        w_avg = np.mean([o.solve_lompc(lmbd, lmbd_r, g)[0] for g in gam], axis=0)
        w_ref, _ = o.solve_lompc(lmbd, lmbd_r, (gam.max() + gam.min()) / 2)
        err = np.sqrt((w_avg - w_ref) @ A_bar @ (w_avg - w_ref))
        assert err <= np.sqrt(N) * gmax / 2 + 1e-12


def test_reductions_restate_price_solver(golden):
    """price_solver.py:196-214 / 272-285 restated: recompute from the golden w."""
    for case in golden[:12]:
        o = O.OracleLoMPC(case["N"], oracle_consts(case))
        A_bar, _ = O.w_inner_product_metric(o.A, case["delta"], case["lmbd_r"])
        W = case["w"]
        dv = W - case["w_ref"]
        errs = np.sqrt(np.einsum("bi,ij,bj->b", dv, A_bar, dv))
        assert abs(errs.max() - case["w_err_max"]) <= 1e-10
        w_avg = W.mean(axis=0)
        assert abs(np.sqrt((w_avg - case["w_ref"]) @ A_bar @ (w_avg - case["w_ref"])) - case["w_avg_err"]) <= 1e-10
        np.testing.assert_allclose(W[:, 0], case["w0"], atol=1e-12)


def test_oracle_input_checks():
    o = O.OracleLoMPC(12, O.small_consts())
    with pytest.raises(AssertionError):
        o.solve_lompc(np.zeros(36), 0.0, 0.95)
    with pytest.raises(ValueError):
        o.solve_lompc(-np.ones(36), 0.0, 0.5)
    with pytest.raises(AssertionError):
        O.OracleLoMPC(12, O.OracleConstants(0.05, 10, 0.95, 0.25, "small"))


def test_c_oracle_warm_batch_equals_cold_batch():
    """oracle_c.solve_batch(warm=True) (each solve started from the previous solve's working set)
    returns the same optima as the cold batch (the same final equality-constrained solve)."""
    import oracle_c

    rng = np.random.default_rng(4)
    for c, N in ((O.small_consts(), 48), (O.large_consts(), 48), (O.large_consts(), 12)):
        lm = c.theta * rng.random(3 * N)
        g = np.sort(c.y_max - (0.3 + 0.2 * rng.random(3000)))
        for gg in (g, rng.permutation(g)):
            w, cost, nf = oracle_c.solve_batch(N, c, lm, 0.0, gg)
            w2, cost2, nf2 = oracle_c.solve_batch(N, c, lm, 0.0, gg, warm=True)
            assert nf == nf2 == 0
            np.testing.assert_allclose(w2, w, rtol=0, atol=1e-12)
            np.testing.assert_allclose(cost2, cost, rtol=1e-12, atol=1e-12)
