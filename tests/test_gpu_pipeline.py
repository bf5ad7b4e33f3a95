"""GPU tests of the PATH pipeline behind lompc_run / BatchPlan (K1 path cells ->
K2 per-EV blocks with in-place repairs -> K3 per-set reductions): one call per
price iteration, parameter epochs across runs, ragged / empty / very large sets.

Tolerances as in test_gpu_parity.py (|dw| <= 1e-9, cost 1e-9 relative);
reductions equal the sums of the per-EV outputs to 1e-11 relative (sums of up to 3e5 terms).
"""
import numpy as np
import pytest
import torch

import lompc_oracle as O
import oracle_c
from lompc_amd import BatchPlan, LoMPC, LoMPCConstants, _lib

pytestmark = pytest.mark.gpu

TOL_W = 1e-9


def mk(c, N, mode="path"):
    return LoMPC(N, LoMPCConstants(c.delta, c.theta, c.y_max, c.w_max, c.ev_type), device=0, mode=mode)


def check_reductions(out, off, N):
    w = out["w"].cpu().numpy()
    st = out["set_stats"].cpu().numpy()
    sw = out["set_sum_w"].cpu().numpy()
    cost = out["cost"].cpu().numpy()
    for s in range(len(off) - 1):
        a, b = off[s], off[s + 1]
        assert st[s, _lib.LOMPC_STAT_COUNT] == b - a
        ref = w[a:b].sum(0) if b > a else np.zeros(N)
        np.testing.assert_allclose(sw[s], ref, rtol=1e-11, atol=1e-9)
        np.testing.assert_allclose(st[s, _lib.LOMPC_STAT_SUM_W0], ref[0], rtol=1e-11, atol=1e-9)
        np.testing.assert_allclose(st[s, _lib.LOMPC_STAT_SUM_COST], cost[a:b].sum(), rtol=1e-11, atol=1e-9)
        assert st[s, _lib.LOMPC_STAT_N_FAILED] == 0 and st[s, _lib.LOMPC_STAT_N_INVALID] == 0


@pytest.mark.parametrize("ev", ["small", "large"])
def test_run_matches_two_calls_and_oracle(gpu, ev):
    """Ragged sets: empty, one full block, one partial block, ~4.7k blocks."""
    rng = np.random.default_rng(31 + (ev == "large"))
    c = O.small_consts() if ev == "small" else O.large_consts()
    N = 24
    sizes = [0, 64, 37, 300000, 5000, 0]
    off = np.concatenate([[0], np.cumsum(sizes)]).astype(np.int64)
    S, B = len(sizes), int(off[-1])
    g = torch.as_tensor(c.y_max * rng.random(B), device="cuda:0")
    lm = torch.as_tensor(c.theta * rng.random((S, 3 * N)), device="cuda:0")
    lr = torch.as_tensor(3 * N * c.delta * rng.random(S), device="cuda:0")
    wr = torch.as_tensor(c.w_max * rng.random((S, N)), device="cuda:0")
    lompc = mk(c, N)
    # window=False: the full-range path, bitwise comparable with set_params + solve_batch
    plan = BatchPlan(lompc, g, off, w_ref=wr, want_w=True, want_cost=True, want_w0=True, want_status=True,
                     window=False)
    out = plan.run(lm, lr)
    torch.cuda.synchronize()
    rep, fail, inv = lompc.check_last()
    assert fail == 0 and inv == 0
    w1 = out["w"].clone()
    st1 = out["set_stats"].clone()
    # the same batch through set_params + solve_batch (two launches)
    lompc.set_params(lm, lr, w_ref=wr)
    r2 = lompc.solve_batch(g, off, want_status=True)
    assert torch.equal(w1, r2["w"]) and torch.equal(st1, r2["set_stats"])
    check_reductions(out, off, N)
    st = out["status"].cpu().numpy()
    assert np.all((st == _lib.LOMPC_QP_OK) | (st == _lib.LOMPC_QP_REPAIRED))
    np.testing.assert_array_equal(out["w0"].cpu().numpy(), w1[:, 0].cpu().numpy())
    # subsample of every non-empty set against the C oracle
    wn, gn, lmn, lrn = w1.cpu().numpy(), g.cpu().numpy(), lm.cpu().numpy(), lr.cpu().numpy()
    cn = out["cost"].cpu().numpy()
    for s in range(S):
        if off[s + 1] == off[s]:
            continue
        idx = rng.choice(np.arange(off[s], off[s + 1]), min(64, off[s + 1] - off[s]), replace=False)
        wo, co, nf = oracle_c.solve_batch(N, c, lmn[s], lrn[s], gn[idx])
        assert nf == 0
        np.testing.assert_allclose(wn[idx], wo, atol=TOL_W)
        np.testing.assert_allclose(cn[idx], co, rtol=1e-9, atol=1e-9)


def test_epochs_across_runs(gpu):
    """Alternating price vectors through one plan: each run sees only its own table."""
    rng = np.random.default_rng(5)
    c = O.large_consts()
    N, S, per = 24, 12, 4096
    off = np.arange(S + 1, dtype=np.int64) * per
    g = torch.as_tensor(c.y_max * rng.random(S * per), device="cuda:0")
    lms = [torch.as_tensor(c.theta * rng.random((S, 3 * N)), device="cuda:0") for _ in range(2)]
    lr = torch.zeros(S, dtype=torch.float64, device="cuda:0")
    lompc = mk(c, N)
    plan = BatchPlan(lompc, g, off)
    res = []
    for k in (0, 1, 0, 1, 1, 0):
        res.append(plan.run(lms[k], lr)["w"].clone())
    torch.cuda.synchronize()
    assert torch.equal(res[0], res[2]) and torch.equal(res[0], res[5])
    assert torch.equal(res[1], res[3]) and torch.equal(res[1], res[4])
    assert not torch.equal(res[0], res[1])
    lompc.set_params(lms[1], lr)
    assert torch.equal(lompc.solve_batch(g, off)["w"], res[1])


@pytest.mark.parametrize("ev", ["small", "large"])
@pytest.mark.parametrize("N", [12, 24])
def test_in_place_repair_path(gpu, ev, N):
    """PATH_REPAIR publishes empty cells: every EV takes the in-place wave re-solve."""
    rng = np.random.default_rng(77 + N + (ev == "large"))
    c = O.small_consts() if ev == "small" else O.large_consts()
    sizes = [150, 0, 64, 9]
    off = np.concatenate([[0], np.cumsum(sizes)]).astype(np.int64)
    S, B = len(sizes), int(off[-1])
    gn = c.y_max * rng.random(B)
    gn[:2] = [0.0, c.y_max]
    lmn = c.theta * rng.random((S, 3 * N))
    lrn = np.array([0.0, 1.0, 3 * N * c.delta * rng.random(), 0.5])
    lompc = mk(c, N, mode="path_repair")
    plan = BatchPlan(lompc, torch.as_tensor(gn, device="cuda:0"), off, want_status=True)
    out = plan.run(torch.as_tensor(lmn, device="cuda:0"), torch.as_tensor(lrn, device="cuda:0"))
    torch.cuda.synchronize()
    st = out["status"].cpu().numpy()
    assert np.all(st == _lib.LOMPC_QP_REPAIRED)
    stats = out["set_stats"].cpu().numpy()
    np.testing.assert_array_equal(stats[:, _lib.LOMPC_STAT_N_REPAIRED], sizes)
    check_reductions(out, off, N)
    w, cost = out["w"].cpu().numpy(), out["cost"].cpu().numpy()
    for s in range(S):
        a, b = off[s], off[s + 1]
        if b > a:
            wo, co, nf = oracle_c.solve_batch(N, c, lmn[s], lrn[s], gn[a:b])
            assert nf == 0
            np.testing.assert_allclose(w[a:b], wo, atol=TOL_W)
            np.testing.assert_allclose(cost[a:b], co, rtol=1e-9, atol=1e-9)


@pytest.mark.parametrize("ev", ["small", "large"])
@pytest.mark.parametrize("N", [24, 48])
def test_gamma_window_matches_full_path(gpu, ev, N):
    """lompc_set_gamma_window: paths over each set's own gamma range (BatchPlan default) give
    the full-range answers; gamma moved outside the measured window afterwards is re-solved
    (status REPAIRED) and still matches the oracle."""
    rng = np.random.default_rng(77 + N + (ev == "large"))
    c = O.small_consts() if ev == "small" else O.large_consts()
    sizes = [4000, 1, 0, 2500, 640]
    off = np.concatenate([[0], np.cumsum(sizes)]).astype(np.int64)
    S, B = len(sizes), int(off[-1])
    # partitions by SoC: narrow gamma ranges per set (charging_station.py:111-116), one single-EV set
    lo = np.array([0.05, 0.4, 0.0, 0.6, 0.3]) * c.y_max
    gn = np.concatenate([lo[s] + 0.08 * c.y_max * rng.random(sizes[s]) for s in range(S)])
    g = torch.as_tensor(gn, device="cuda:0")
    lm = torch.as_tensor(c.theta * rng.random((S, 3 * N)), device="cuda:0")
    lr = torch.as_tensor(3 * N * c.delta * rng.random(S), device="cuda:0")
    wr = torch.as_tensor(c.w_max * rng.random((S, N)), device="cuda:0")
    lompc = mk(c, N)
    kw = dict(w_ref=wr, want_w=True, want_cost=True, want_status=True)
    full = BatchPlan(lompc, g, off, window=False, **kw)
    o_full = {k: (v.clone() if v is not None else None) for k, v in full.run(lm, lr).items()}
    win = BatchPlan(lompc, g, off, **kw)
    assert win.window is not None
    o_win = win.run(lm, lr)
    torch.cuda.synchronize()
    rep, fail, inv = lompc.check_last()
    assert fail == 0 and inv == 0 and rep == 0
    np.testing.assert_allclose(o_win["w"].cpu().numpy(), o_full["w"].cpu().numpy(), rtol=0, atol=1e-12)
    np.testing.assert_allclose(o_win["cost"].cpu().numpy(), o_full["cost"].cpu().numpy(), rtol=1e-12, atol=1e-12)
    np.testing.assert_allclose(o_win["set_sum_w"].cpu().numpy(), o_full["set_sum_w"].cpu().numpy(), rtol=1e-11,
                               atol=1e-10)
    check_reductions(o_win, off, N)
    # gamma changed in place outside the plan's window: repaired, still exact
    g[off[0]:off[0] + 10] = torch.as_tensor(0.95 * c.y_max * np.ones(10), device="cuda:0")
    o2 = win.run(lm, lr)
    torch.cuda.synchronize()
    rep, fail, inv = lompc.check_last()
    assert fail == 0 and inv == 0 and rep >= 10
    st = o2["status"].cpu().numpy()
    assert np.all(st[:10] == _lib.LOMPC_QP_REPAIRED)
    o = O.OracleLoMPC(N, c)
    w2 = o2["w"].cpu().numpy()
    for i in range(10):
        wo, _ = o.solve_lompc(lm[0].cpu().numpy(), float(lr[0]), 0.95 * c.y_max)
        assert np.max(np.abs(w2[i] - wo)) <= TOL_W
