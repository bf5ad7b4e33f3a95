"""GPU tests of the CVXPY-free PriceSolver (price_solver.py:16-285) on the batched
engine against the CPU oracle loop (oracle/price_oracle.py: C-oracle LoMPC per EV,
dense scipy price QP, the documented LP vertex rule).  The sweep is the reference's
own convergence test (chargingstation/test/test_price_solver.py:38-106): single EV x
{small, large} x {linear, linear-convex}; 100 EVs; N in {12, 24}; lmbd_r in
{0, N, 2N, 3N}; initial-SoC spread 1/3 or 1/36 of y_max.

Tolerance: the iteration count must match exactly; prices within 1e-6 * theta
(absolute), the north star's 1e-6 relative; stats entries within 1e-6 relative.
"""
import zlib

import numpy as np
import pytest

import lompc_oracle as O
import price_oracle as PO
from lompc_amd import LoMPCConstants, settings
from lompc_amd.price_solver import PriceSolver

pytestmark = pytest.mark.gpu


def consts(ev):
    c = O.small_consts() if ev == "small" else O.large_consts()
    return c, LoMPCConstants(c.delta, c.theta, c.y_max, c.w_max, c.ev_type)


SWEEP = (
    [("single", 1, 12, ev, pt, 0.0, 1 / 3.0) for ev in ("small", "large") for pt in ("linear", "linear-convex")]
    + [("multi", 100, 12, ev, "linear-convex", 0.0, 1 / 36.0) for ev in ("small", "large")]
    + [("horizon", 10, N, ev, "linear-convex", 0.0, 1 / 36.0) for ev in ("small", "large") for N in (12, 24)]
    + [("robust", 10, 12, ev, "linear-convex", lr, 1 / 36.0) for ev in ("small", "large") for lr in (12, 24, 36)]
)


def compare(lm, st, lmo, sto, theta):
    assert st["iter"] == sto["iter"]
    np.testing.assert_allclose(lm, lmo, rtol=0, atol=1e-6 * theta)
    for k in ("price_before_reg", "price_after_reg"):
        assert abs(st[k] - sto[k]) <= 1e-6 * max(1.0, abs(sto[k])), k
    for k in ("dual_cost_decrease_actual", "dual_cost_decrease_predicted"):
        assert st[k].shape == sto[k].shape, k
        np.testing.assert_allclose(st[k], sto[k], rtol=1e-6, atol=1e-6 * np.max(np.abs(sto[k]), initial=1.0))


@pytest.mark.parametrize("loop", ["device", "host", "python"])
@pytest.mark.parametrize("case", SWEEP, ids=lambda c: f"{c[0]}-{c[3]}-{c[4]}-N{c[2]}-lr{c[5]}")
def test_compute_optimal_prices_matches_oracle(gpu, case, loop, monkeypatch):
    """All three loops: the device-resident loop (lompc_price_loop, device_loop = 1: convergence test
    and price QP on the GPU, the default), the host C++ loop (device_loop = 0) and the Python
    restatement (used with PRINT_LEVEL >= 2 and on gloo-sharded ranks)."""
    name, nev, N, ev, price_type, lmbd_r, spread = case
    monkeypatch.setattr(settings, "PRINT_LEVEL", 0)
    c, lc = consts(ev)
    rng = np.random.default_rng(zlib.crc32(repr(case).encode()))
    ps = PriceSolver(N, lc, price_type, device=0)
    ps.native_loop = loop != "python"
    ps.device_loop = loop == "device"
    po = PO.OraclePriceSolver(N, c, price_type)
    for call in range(2):  # the second call starts from prev_prices (price_solver.py:104, :166)
        y0 = spread * c.y_max * rng.random(nev)  # test_price_solver.py:32
        w_ref = c.w_max * rng.random(N)          # test_price_solver.py:34
        ps.set_charge_levels(y0)
        po.set_charge_levels(y0)
        lm, st = ps.compute_optimal_prices(w_ref, lmbd_r)
        lmo, sto = po.compute_optimal_prices(w_ref, lmbd_r)
        compare(lm, st, lmo, sto, c.theta)
        assert np.all(st["dual_cost_decrease_predicted"] >= -1e-9)
        np.testing.assert_array_equal(ps.prev_prices, lm[: ps.r])
        # get_w0_price0 (price_solver.py:272-285)
        w0, p0 = ps.get_w0_price0(lm[: ps.r], lmbd_r)
        w0o, p0o = po.get_w0_price0(lmo[: po.r], lmbd_r)
        np.testing.assert_allclose(w0, w0o, rtol=0, atol=1e-6 * c.w_max)
        assert abs(p0 - p0o) <= 1e-6 * max(1.0, abs(p0o))


def test_get_w_err_and_print_level_path(gpu, capsys, monkeypatch):
    """_get_w_err standalone (price_solver.py:196-214) and the PRINT_LEVEL >= 1 extra
    batch (:150-164) that prints the w0 error line."""
    monkeypatch.setattr(settings, "PRINT_LEVEL", 1)
    c, lc = consts("large")
    N = 12
    rng = np.random.default_rng(7)
    ps = PriceSolver(N, lc, "linear-convex", device=0)
    y0 = 0.3 + 0.05 * rng.random(37)
    ps.set_charge_levels(y0)
    w_ref = c.w_max * rng.random(N)
    lmbd = c.theta * rng.random(3 * N)
    A_bar, _ = ps._get_w_inner_product_metric(0.0)
    got = ps._get_w_err(lmbd, 0.0, w_ref, A_bar)
    o = O.OracleLoMPC(N, c)
    exp = O.get_w_err(o, y0, lmbd, 0.0, w_ref, A_bar)
    np.testing.assert_allclose(got, exp, rtol=1e-9, atol=1e-10)
    ps.compute_optimal_prices(w_ref, 0.0)
    assert "w0-error" in capsys.readouterr().out


def test_dual_cost_guarantee_large_evs(gpu, monkeypatch):
    """plots.py:115-178: 100 large EVs, lmbd_r = 0 — the predicted (guaranteed) decrease is
    non-negative every iteration and the first actual decrease is at least the guarantee."""
    monkeypatch.setattr(settings, "PRINT_LEVEL", 0)
    c, lc = consts("large")
    N = 12
    rng = np.random.default_rng(11)
    ps = PriceSolver(N, lc, "linear-convex", device=0)
    ps.set_charge_levels(0.3 + 1 / 24 * c.y_max * rng.random(100))
    _, st = ps.compute_optimal_prices(c.w_max * rng.random(N), 0.0)
    pred, act = st["dual_cost_decrease_predicted"], st["dual_cost_decrease_actual"]
    assert len(pred) == st["iter"] and np.all(pred >= -1e-9)
    if len(act):
        assert act[0] >= pred[0] - 1e-6 * max(1.0, abs(pred[0]))


@pytest.mark.parametrize("ev,price_type", [("small", "linear"), ("large", "linear-convex")])
@pytest.mark.parametrize("N", [12, 24, 48])
def test_device_loop_matches_host_loop(gpu, monkeypatch, ev, price_type, N):
    """The device-resident loop against the host C++ loop over consecutive calls (warm prices,
    several partitions' worth of EVs): the same iteration counts, prices within 1e-9 theta, dual
    cost decreases within 1e-8 relative (the price QP on one wave vs the host's sequential
    tridiagonal solves: same method, different rounding), and the loop's engine calls counted
    once (no call of the enqueued-ahead tail reaches the results)."""
    monkeypatch.setattr(settings, "PRINT_LEVEL", 0)
    c, lc = consts(ev)
    rng = np.random.default_rng(100 + N + (ev == "large"))
    sols = {}
    for mode in ("device", "host"):
        ps = PriceSolver(N, lc, price_type, device=0)
        ps.device_loop = mode == "device"
        sols[mode] = ps
    for call in range(4):
        y0 = 0.3 + (0.02 + 0.02 * call) * c.y_max * rng.random(3000 + 500 * call)
        w_ref = c.w_max * (0.2 + 0.6 * rng.random(N))
        lr = 0.0 if call < 2 else 3.0 * N * c.delta * rng.random()
        res = {}
        for mode, ps in sols.items():
            ps.set_charge_levels(y0)
            n0 = ps.n_batched_calls
            lm, st = ps.compute_optimal_prices(w_ref, lr)
            res[mode] = (lm.copy(), st, ps.n_batched_calls - n0)
        (ld, sd, nd), (lh, sh, nh) = res["device"], res["host"]
        assert sd["iter"] == sh["iter"] and nd == nh == sd["iter"] + 1
        np.testing.assert_allclose(ld, lh, rtol=0, atol=1e-9 * c.theta)
        for k in ("dual_cost_decrease_actual", "dual_cost_decrease_predicted"):
            np.testing.assert_allclose(sd[k], sh[k], rtol=1e-8, atol=1e-8 * np.max(np.abs(sh[k]), initial=1.0), err_msg=k)
        for k in ("price_before_reg", "price_after_reg"):
            assert abs(sd[k] - sh[k]) <= 1e-9 * max(1.0, abs(sh[k])), k


@pytest.mark.parametrize("N", [12, 48])
def test_device_loop_is_one_launch(gpu, monkeypatch, N):
    """Over a gamma-sorted loop plan the device loop runs the WHOLE loop as ONE persistent launch
    (k_loop_run2: per call path, aggregation and loop step, every wave running the same step after a
    counter barrier;
    timed as k_path): no k_eval / k_agg launch, and the same iterations and prices as the host loop
    (which runs k_path + k_agg + the host step per iteration)."""

    monkeypatch.setattr(settings, "PRINT_LEVEL", 0)
    c, lc = consts("large")
    rng = np.random.default_rng(5 + N)
    y0 = 0.3 + 0.05 * c.y_max * rng.random(20000)
    w_ref = c.w_max * (0.2 + 0.6 * rng.random(N))
    res = {}
    for mode in ("device", "host"):
        ps = PriceSolver(N, lc, "linear-convex", device=0)
        ps.device_loop = mode == "device"
        ps.set_charge_levels(y0)
        plan = ps._plan
        plan.profile(enable=("k_path", "k_eval"))
        for k in ("k_path", "k_eval"):
            plan.profile(read=True, reset=True, kernel=k)
        lm, st = ps.compute_optimal_prices(w_ref, 0.0)
        n = {k: plan.profile(read=True, kernel=k)[1] for k in ("k_path", "k_eval")}
        plan.profile(enable=False)
        res[mode] = (lm.copy(), st, n)
    (ld, sd, nd), (lh, sh, nh) = res["device"], res["host"]
    assert sd["iter"] == sh["iter"]
    assert nd["k_eval"] == 0, nd
    assert nd["k_path"] == 1, nd  # (k_loop_iter per call would be iter + 1 .. iter + 1 + LOMPC_LOOP_AHEAD)
    assert sd["iter"] >= 3  # (a loop of several calls in the one launch)
    assert nh["k_eval"] == nh["k_path"] == sh["iter"] + 1, nh
    np.testing.assert_allclose(ld, lh, rtol=0, atol=1e-9 * c.theta)
