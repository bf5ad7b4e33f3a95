"""CPU tests of the CVXPY-free BiMPC planner (bimpc.py) — the interior-point solver
in the C-ABI library, certified against the literal torch restatement of
bimpc.py:182-265 (oracle/bimpc_oracle.py): stationarity with the returned
multipliers, feasibility, complementarity; cross-checked against the oracle's own
dense interior point and scipy SLSQP.  Instances follow the reference's
test_bimpc.py:24-77 (random simplex EV distributions, gamma ~ 0.6 U[0,1],
early-peak demand) and the example's constants (real_time_price_control.py:42-52).

Tolerances: KKT measures relative to the gradient / objective scale; 1e-7 where the
problem is well conditioned, 1e-5 (Clarabel's reduced "almost solved" level) for the
EXP_UNWEIGHTED weights 5^(t-N+1) at N = 24, whose early steps carry ~1e-16 weight.
"""
import numpy as np
import pytest

import bimpc_oracle as BO
from lompc_amd.bimpc import BiMPC, BiMPCChargingCostType, BiMPCConstants, BiMPCParameters
from lompc_amd.demand_data import medium_term_demand_forecast
from lompc_amd.lompc import LoMPCConstants, SolverError

CS = LoMPCConstants(0.05, 10, 0.9, 0.25, "small")
CL = LoMPCConstants(0.025, 50, 0.9, 0.15, "large")


def simplex(rng, n):
    v = rng.random(n) + 1e-6  # test_bimpc.py:39-41
    return v / np.sum(v)


def instance(N, P, seed, cost_type=2, u_g_max=1.5, x_max=1.5, u_b_max=0.3, beta_scale=None, M=500, x0=0.0):
    """test_bimpc.py:44-77 (random_Mp, random_gamma, early_peak_demand).  beta defaults to the
    reference's sqrt(N) 0.3 / P, capped at 0.1 so that the first-step storage bounds stay
    feasible for small P (d_e = (theta_s M_s + theta_l M_l) beta / B = beta here)."""
    if beta_scale is None:
        beta_scale = min(0.3, 0.1 * P / np.sqrt(N))
    rng = np.random.default_rng(seed)
    B = CS.theta * M + CL.theta * M
    Mp_s = M * simplex(rng, P) / B
    Mp_l = M * simplex(rng, P) / B
    beta = np.sqrt(N) * beta_scale / P * np.ones(P)
    gs = 0.6 * rng.random(P)
    gl = 0.6 * rng.random(P)
    demand = medium_term_demand_forecast(24 + N, 1 / 4, interpolate=False) / B
    demand = demand[17:17 + N]
    params = BiMPCParameters(Mp_s, Mp_l, beta, beta.copy(), gs, gl, x0, demand)
    bi = BiMPCConstants(1e3, 1, u_g_max, u_b_max, x_max, BiMPCChargingCostType(cost_type), 5)
    lit = BO.BiMPCLiteral(N, P, dict(delta=1e3, c_g=1, u_g_max=u_g_max, u_b_max=u_b_max, x_max=x_max,
                                     cost_type=cost_type, exp_rate=5),
                          CS.theta, CL.theta, CS.w_max, CL.w_max,
                          dict(Mp_s=Mp_s, Mp_l=Mp_l, beta_s=beta, beta_l=beta, gamma_sm=gs, gamma_lm=gl, x0=x0,
                               demand=demand))
    return bi, params, lit


def solve(N, P, bi, params):
    b = BiMPC(N, P, bi, CS, CL)
    ws, wl, ug = b.solve_bimpc(params)
    return b, ws, wl, ug


@pytest.mark.parametrize("N,P,ct,tol", [(24, 12, 2, 1e-5), (16, 12, 2, 1e-7), (24, 12, 1, 1e-7), (12, 4, 0, 1e-7),
                                        (12, 4, 1, 1e-7), (48, 12, 2, 1e-5), (48, 12, 1, 1e-7)])
def test_kkt_certificate(N, P, ct, tol):
    bi, params, lit = instance(N, P, seed=N * 10 + ct, cost_type=ct)
    b, ws, wl, ug = solve(N, P, bi, params)
    assert ws.shape == (P, N) and wl.shape == (P, N) and ug.shape == (N,)
    stat, infeas, comp, dual_inf = lit.kkt(lit.pack(ws, wl, ug), b.last_duals)
    assert stat <= tol and comp <= tol and dual_inf == 0.0
    assert infeas <= 1e-9


def test_example_constants_config1():
    """real_time_price_control.py:42-52: u_g_max 1, u_b_max 0.3, x_max 0.3, EXP rate 5, N_bi 16."""
    bi, params, lit = instance(16, 12, seed=3, cost_type=2, u_g_max=1.0, x_max=0.3)
    b, ws, wl, ug = solve(16, 12, bi, params)
    stat, infeas, comp, dual_inf = lit.kkt(lit.pack(ws, wl, ug), b.last_duals)
    assert stat <= 1e-7 and comp <= 1e-7 and infeas <= 1e-9 and dual_inf == 0.0
    assert np.all(ws >= 0) and np.all(ws <= CS.w_max) and np.all(wl <= CL.w_max) and np.all(ug <= 1.0)


@pytest.mark.parametrize("ct", [0, 1, 2])
def test_matches_dense_oracle_ipm(ct):
    """Same optimum as the oracle's dense interior point on the literal problem (unique:
    strictly convex).  Compared on the objective and on the well-determined quantities
    the rest of the loop consumes: u_g and the partition targets A w_hat (last step)."""
    N, P = 12, 4
    bi, params, lit = instance(N, P, seed=100 + ct, cost_type=ct)
    b, ws, wl, ug = solve(N, P, bi, params)
    zo, lam, _ = lit.solve_ipm()
    z = lit.pack(ws, wl, ug)
    fo, f = lit.objective(zo), lit.objective(z)
    assert abs(f - fo) <= 1e-8 * max(1.0, abs(fo))
    np.testing.assert_allclose(ug, zo[-N:], atol=1e-5)
    wso, wlo, _ = lit.split(zo)
    np.testing.assert_allclose(ws.sum(1), wso.sum(1), atol=1e-5)
    np.testing.assert_allclose(wl.sum(1), wlo.sum(1), atol=1e-5)


def test_slsqp_cross_check():
    """An independent local solver (scipy SLSQP on the literal problem) never finds a
    feasible point better than the engine's optimum."""
    N, P = 8, 2
    bi, params, lit = instance(N, P, seed=7, cost_type=1, beta_scale=0.05)
    b, ws, wl, ug = solve(N, P, bi, params)
    zs, res = lit.solve_slsqp()
    import torch

    assert float(np.max(lit.constraints_t(torch.tensor(zs)).numpy())) <= 1e-8  # SLSQP point feasible
    z = lit.pack(ws, wl, ug)
    fs = lit.objective(zs)
    assert lit.objective(z) <= fs + 1e-9 * max(1.0, abs(fs))


def test_infeasible_storage_bounds_raise():
    """N = 8, P = 3 with the test_bimpc.py robustness bounds: the first-step battery
    constraints (bimpc.py:201-218) cannot all hold -> SolverError (Clarabel: infeasible)."""
    bi, params, _ = instance(8, 3, seed=0, cost_type=0, beta_scale=0.3)
    with pytest.raises(SolverError):
        solve(8, 3, bi, params)


def test_reference_input_checks():
    bi, params, _ = instance(8, 2, seed=0)
    with pytest.raises(AssertionError):  # bimpc.py:84
        BiMPC(8, 2, BiMPCConstants(1e3, 1, 1, 0.3, 0.3, BiMPCChargingCostType.EXP_UNWEIGHTED, 0.5), CS, CL)
    b = BiMPC(8, 2, bi, CS, CL)
    with pytest.raises(AssertionError):  # bimpc.py:278
        b.solve_bimpc(BiMPCParameters(np.ones(3), np.ones(2), np.ones(2), np.ones(2), np.ones(2), np.ones(2), 0,
                                      np.ones(8)))
    bad = BiMPCParameters(params.Mp_s, params.Mp_l, params.beta_s, params.beta_l, -params.gamma_sm,
                          params.gamma_lm, 0.0, params.demand)
    with pytest.raises(ValueError):  # nonneg cvx.Parameter (bimpc.py:152)
        b.solve_bimpc(bad)
    assert np.array_equal(b.get_bat_input_mat(), np.tril(np.ones((8, 8))))


def test_demand_forecast_restates_reference():
    """demand_data.py:21-37 on the shipped forecast rows: hour 1 = 73822, hour 24 = 76068,
    half-hour values are the mean of neighbouring hours (wrapping), decimated when not
    interpolated, tiled to the horizon, scaled."""
    d = medium_term_demand_forecast(66, 1 / 4, interpolate=False)
    assert d.shape == (66,)
    assert d[0] == pytest.approx((73822 + 76068) / 2 / 4)
    assert d[1] == pytest.approx((70492 + 73822) / 2 / 4)
    np.testing.assert_array_equal(d[:24], d[24:48])
    di = medium_term_demand_forecast(24, 1.0, interpolate=True)
    assert di.shape == (48,) and di[1] == 73822 and di[47] == 76068
