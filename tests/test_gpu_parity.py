"""GPU parity tests: the HIP engine (through the C-ABI via lompc_amd) against
the 50-digit golden vectors and the CPU oracle, plus size-independent
properties at BASELINE.json's full sizes.

Tolerance (fp64, written here as the north star asks): every w within
|dw| <= 1e-9 absolute (w in [0, 0.25]) and every cost within 1e-9 relative of
the certified optimum — three orders tighter than the 1e-6 the north star
states for trajectories.
"""
import numpy as np
import pytest
import torch

import lompc_oracle as O
import oracle_c
from conftest import oracle_consts
from lompc_amd import LoMPC, LoMPCConstants, SolverError, _lib
from lompc_amd.price_solver import PriceSolver

pytestmark = pytest.mark.gpu

TOL_W = 1e-9
TOL_C = 1e-9


def mk(case_or_consts, N, mode="path"):
    c = case_or_consts
    if isinstance(c, dict):
        consts = LoMPCConstants(c["delta"], c["theta"], c["y_max"], c["w_max"], c["ev_type"])
    else:
        consts = LoMPCConstants(c.delta, c.theta, c.y_max, c.w_max, c.ev_type)
    return LoMPC(N, consts, device=0, mode=mode)


def check_cost(cost, ref):
    assert np.all(np.abs(cost - ref) <= TOL_C * np.maximum(1.0, np.abs(ref))), np.max(np.abs(cost - ref))


@pytest.mark.parametrize("mode", ["path", "direct"])
def test_golden_single_set(gpu, golden, mode):
    for case in golden:
        lompc = mk(case, case["N"], mode)
        lompc.set_params(case["lmbd"], [case["lmbd_r"]], w_ref=case["w_ref"])
        res = lompc.solve_batch(case["gamma"], want_w0=True, want_status=True)
        w = res["w"].cpu().numpy()
        np.testing.assert_allclose(w, case["w"], rtol=0, atol=TOL_W, err_msg=f"case {case['id']}")
        check_cost(res["cost"].cpu().numpy(), case["cost"])
        st = res["status"].cpu().numpy()
        assert np.all((st == _lib.LOMPC_QP_OK) | (st == _lib.LOMPC_QP_REPAIRED))
        stats = res["set_stats"][0].cpu().numpy()
        assert stats[_lib.LOMPC_STAT_COUNT] == len(case["gamma"])
        assert abs(stats[_lib.LOMPC_STAT_MAX_ERR] - case["w_err_max"]) <= 1e-9
        np.testing.assert_allclose(res["set_sum_w"][0].cpu().numpy(), case["w"].sum(0), atol=1e-12)
        np.testing.assert_allclose(res["w0"].cpu().numpy(), case["w"][:, 0], atol=TOL_W)


def test_golden_multi_set_batch(gpu, golden):
    """All cases of one (EV type, N) as S parameter sets in ONE launch."""
    groups = {}
    for c in golden:
        groups.setdefault((c["ev_type"], c["N"]), []).append(c)
    for (ev, N), cases in groups.items():
        lompc = mk(cases[0], N)
        lm = np.stack([c["lmbd"] for c in cases])
        lr = np.array([c["lmbd_r"] for c in cases])
        wr = np.stack([c["w_ref"] for c in cases])
        g = np.concatenate([c["gamma"] for c in cases])
        off = np.concatenate([[0], np.cumsum([len(c["gamma"]) for c in cases])]).astype(np.int64)
        lompc.set_params(lm, lr, w_ref=wr)
        res = lompc.solve_batch(g, off)
        w = res["w"].cpu().numpy()
        np.testing.assert_allclose(w, np.concatenate([c["w"] for c in cases]), rtol=0, atol=TOL_W)
        stats = res["set_stats"].cpu().numpy()
        for s, c in enumerate(cases):
            assert abs(stats[s, _lib.LOMPC_STAT_MAX_ERR] - c["w_err_max"]) <= 1e-9
            p0 = np.mean([O.OracleLoMPC(N, oracle_consts(c)).get_price0(c["w"][i], c["lmbd"], c["lmbd_r"])
                          for i in range(len(c["gamma"]))])
            assert abs(stats[s, _lib.LOMPC_STAT_SUM_PRICE0] / len(c["gamma"]) - p0) <= 1e-9 * max(1, abs(p0))


def test_solve_lompc_single_matches_golden(gpu, golden):
    for case in golden[::2]:
        lompc = mk(case, case["N"])
        for i in (0, 1, 5):
            w, cost = lompc.solve_lompc(case["lmbd"], case["lmbd_r"], case["gamma"][i])
            assert isinstance(w, np.ndarray) and w.shape == (case["N"],)
            np.testing.assert_allclose(w, case["w"][i], atol=TOL_W)
            assert abs(cost - case["cost"][i]) <= TOL_C * max(1.0, abs(case["cost"][i]))


@pytest.mark.parametrize("mode", ["path", "direct"])
def test_price_solver_loops_match_reference_semantics(gpu, golden, mode):
    """PriceSolver._get_w_err / get_w0_price0 (price_solver.py:196-214, 272-285), both engine modes."""
    for case in golden[::5]:
        c = case
        consts = LoMPCConstants(c["delta"], c["theta"], c["y_max"], c["w_max"], c["ev_type"])
        price_type = "linear" if c["price"] == "linear" else "linear-convex"
        ps = PriceSolver(c["N"], consts, price_type, device=0, mode=mode)
        y0 = c["y_max"] - c["gamma"]
        ps.set_charge_levels(y0)
        A_bar, _ = ps._get_w_inner_product_metric(c["lmbd_r"])
        emax, w0e, avge = ps._get_w_err(c["lmbd"], c["lmbd_r"], c["w_ref"], A_bar)
        assert abs(emax - c["w_err_max"]) <= 1e-9
        assert abs(w0e - c["w0_err"]) <= 1e-9
        assert abs(avge - c["w_avg_err"]) <= 1e-9
        w0, price0 = ps.get_w0_price0(c["lmbd"][: ps.r], c["lmbd_r"])
        np.testing.assert_allclose(w0, c["w0"], atol=TOL_W)
        assert abs(price0 - c["price0"]) <= 1e-9 * max(1.0, abs(c["price0"]))


@pytest.mark.parametrize("ev", ["small", "large"])
@pytest.mark.parametrize("N", [1, 5, 12, 13, 16, 24, 32, 48, 64])
def test_random_batch_vs_c_oracle(gpu, ev, N):
    """Random sets and EVs (test_lompc.py:34-36 distributions) against the C oracle."""
    rng = np.random.default_rng(1000 + N + (ev == "large"))
    c = O.small_consts() if ev == "small" else O.large_consts()
    S, per = 3, 300 if N <= 24 else 120
    lm = c.theta * rng.random((S, 3 * N))
    lr = np.array([0.0, 3 * N * c.delta * rng.random(), 3 * N * c.delta * rng.random()])
    g = c.y_max * rng.random(S * per)
    off = np.arange(S + 1, dtype=np.int64) * per
    lompc = mk(c, N)
    lompc.set_params(lm, lr)
    res = lompc.solve_batch(g, off, want_status=True)
    w = res["w"].cpu().numpy()
    cost = res["cost"].cpu().numpy()
    for s in range(S):
        wo, co, nf = oracle_c.solve_batch(N, c, lm[s], lr[s], g[s * per:(s + 1) * per])
        assert nf == 0
        np.testing.assert_allclose(w[s * per:(s + 1) * per], wo, atol=TOL_W)
        check_cost(cost[s * per:(s + 1) * per], co)


def test_path_and_direct_agree(gpu):
    rng = np.random.default_rng(7)
    c = O.large_consts()
    N, S, per = 24, 4, 2000
    lm = c.theta * rng.random((S, 3 * N))
    lr = np.zeros(S)
    g = c.y_max * rng.random(S * per)
    off = np.arange(S + 1, dtype=np.int64) * per
    outs = []
    for mode in ("path", "direct"):
        lompc = mk(c, N, mode)
        lompc.set_params(lm, lr, gamma_ref=np.full(S, 0.5))
        outs.append(lompc.solve_batch(g, off)["w"].cpu().numpy())
    np.testing.assert_allclose(outs[0], outs[1], atol=1e-10)


def test_edge_cases(gpu):
    c = O.small_consts()
    N = 24
    lompc = mk(c, N)
    # lambda = 0, gamma = 0  =>  w = 0, cost = 0 (known answer)
    lompc.set_params(np.zeros((1, 3 * N)), [0.0])
    res = lompc.solve_batch(np.array([0.0, 0.0]))
    assert np.all(res["w"].cpu().numpy() == 0.0) and np.all(res["cost"].cpu().numpy() == 0.0)
    # empty parameter sets and ragged sets
    rng = np.random.default_rng(11)
    lm = c.theta * rng.random((4, 3 * N))
    lompc.set_params(lm, np.zeros(4))
    off = np.array([0, 0, 3, 3, 260], dtype=np.int64)
    g = c.y_max * rng.random(260)
    g[0], g[1] = 0.0, c.y_max
    res = lompc.solve_batch(g, off)
    st = res["set_stats"].cpu().numpy()
    assert st[0, _lib.LOMPC_STAT_COUNT] == 0 and st[2, _lib.LOMPC_STAT_COUNT] == 0
    assert np.all(res["set_sum_w"].cpu().numpy()[[0, 2]] == 0.0)
    w = res["w"].cpu().numpy()
    for s, (a, b) in enumerate(zip(off[:-1], off[1:])):
        if b > a:
            wo, _, _ = oracle_c.solve_batch(N, c, lm[s], 0.0, g[a:b])
            np.testing.assert_allclose(w[a:b], wo, atol=TOL_W)
    # empty batch
    lompc.set_params(lm[:1], [0.0])
    res = lompc.solve_batch(np.zeros(0))
    assert res["w"].shape == (0, N)
    # invalid inputs map to the reference's exception types
    with pytest.raises(AssertionError):
        lompc.solve_batch(np.array([c.y_max + 0.01]))
    with pytest.raises(ValueError):
        lompc.solve_batch(np.array([-0.1]))
    with pytest.raises(ValueError):
        lompc.set_params(-np.ones((1, 3 * N)), [0.0])
    with pytest.raises(AssertionError):
        lompc.solve_lompc(np.zeros(3 * N), 0.0, c.y_max + 1e-3)
    with pytest.raises(ValueError):
        lompc.solve_lompc(np.zeros(3 * N), -1.0, 0.5)


def test_full_size_config3_properties(gpu):
    """BASELINE config 3 (262 144 EVs, N = 24, S = 24 sets): every QP certified,
    a random subsample equals the oracle, reductions equal sums of the outputs,
    and the result is bitwise reproducible."""
    rng = np.random.default_rng(2)
    N, S, B = 24, 24, 262144
    per = B // S
    off = np.array([min(B, s * per) if s < S else B for s in range(S + 1)], dtype=np.int64)
    y0 = 0.3 + 0.2 * rng.random(B)
    for ev, c in (("small", O.small_consts()), ("large", O.large_consts())):
        lompc = mk(c, N)
        lm = c.theta * rng.random((S, 3 * N))
        lr = np.zeros(S)
        wr = c.w_max * rng.random((S, N))
        g = torch.as_tensor(c.y_max - y0, device="cuda:0")
        lompc.set_params(lm, lr, w_ref=wr)
        r1 = lompc.solve_batch(g, off, want_status=True)
        rep, fail, inv = lompc.check_last()
        assert fail == 0 and inv == 0
        w1 = r1["w"].clone()
        sw1 = r1["set_sum_w"].clone()
        r2 = lompc.solve_batch(g, off)
        assert torch.equal(w1, r2["w"]) and torch.equal(sw1, r2["set_sum_w"])
        wn = w1.cpu().numpy()
        gn = c.y_max - y0
        for s in range(0, S, 6):
            idx = rng.choice(np.arange(off[s], off[s + 1]), 64, replace=False)
            wo, _, _ = oracle_c.solve_batch(N, c, lm[s], 0.0, gn[idx])
            np.testing.assert_allclose(wn[idx], wo, atol=TOL_W)
        ref_sum = np.add.reduceat(wn, off[:-1], axis=0)
        np.testing.assert_allclose(sw1.cpu().numpy(), ref_sum, rtol=1e-12, atol=1e-9)


def test_not_converged_maps_to_solver_error_type():
    assert issubclass(SolverError, Exception)
