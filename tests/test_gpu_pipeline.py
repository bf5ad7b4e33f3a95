"""GPU tests of the PATH engine behind lompc_plan_* / BatchPlan (plan: per-set gamma window and
cells, the evaluation block map; run: k_path over (set, cell) waves -> certified path pieces,
k_eval over the EVs in caller order with the set's pieces in LDS, k_reduce): one call per price
iteration, repeated runs, several EV types in one plan, ragged / empty / very large sets,
invalid and moved gamma, warm starts, cell counts, the individual-repair path.

Tolerances as in test_gpu_parity.py (|dw| <= 1e-9, cost 1e-9 relative); reductions equal the
sums of the per-EV outputs to 1e-11 relative (sums of up to 3e5 terms).
"""
import os

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


def oracle_check(out, g, lm, lr, off, c, N, rng, k=64):
    wn, gn, lmn, lrn = out["w"].cpu().numpy(), g.cpu().numpy(), lm.cpu().numpy(), lr.cpu().numpy()
    cn = out["cost"].cpu().numpy()
    for s in range(len(off) - 1):
        if off[s + 1] == off[s]:
            continue
        idx = rng.choice(np.arange(off[s], off[s + 1]), min(k, off[s + 1] - off[s]), replace=False)
        wo, co, nf = oracle_c.solve_batch(N, c, lmn[s], lrn[s], gn[idx])
        assert nf == 0
        np.testing.assert_allclose(wn[idx], wo, atol=TOL_W)
        np.testing.assert_allclose(cn[idx], co, rtol=1e-9, atol=1e-9)


@pytest.mark.parametrize("ev", ["small", "large"])
def test_plan_matches_solve_batch_and_oracle(gpu, ev):
    """Ragged sets: empty, one full block, one partial block, 300k EVs."""
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
    plan = BatchPlan(lompc, g, off, w_ref=wr, want_w=True, want_cost=True, want_w0=True, want_status=True)
    out = plan.run(lm, lr)
    rep, fail, inv = plan.check()
    assert fail == 0 and inv == 0
    w1 = out["w"].clone()
    st1 = out["set_stats"].clone()
    # the same batch through set_params + solve_batch (the context's transient plan): bitwise
    lompc.set_params(lm, lr, w_ref=wr)
    r2 = lompc.solve_batch(g, off, want_status=True)
    assert torch.equal(w1, r2["w"]) and torch.equal(st1, r2["set_stats"])
    check_reductions(out, off, N)
    st = out["status"].cpu().numpy()
    assert np.all((st == _lib.LOMPC_QP_OK) | (st == _lib.LOMPC_QP_REPAIRED))
    np.testing.assert_array_equal(out["w0"].cpu().numpy(), w1[:, 0].cpu().numpy())
    oracle_check(out, g, lm, lr, off, c, N, rng)


def test_repeated_runs(gpu):
    """Alternating price vectors through one plan: every run depends only on its own prices."""
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
def test_individual_repair_path(gpu, ev, N):
    """LOMPC_PLAN_DIAG_REPAIR: no path pieces, every EV takes the whole-wave certified re-solve."""
    rng = np.random.default_rng(77 + N + (ev == "large"))
    c = O.small_consts() if ev == "small" else O.large_consts()
    sizes = [150, 0, 64, 9]
    off = np.concatenate([[0], np.cumsum(sizes)]).astype(np.int64)
    S, B = len(sizes), int(off[-1])
    gn = c.y_max * rng.random(B)
    gn[:2] = [0.0, c.y_max]
    lmn = c.theta * rng.random((S, 3 * N))
    lrn = np.array([0.0, 1.0, 3 * N * c.delta * rng.random(), 0.5])
    lompc = mk(c, N)
    plan = BatchPlan(lompc, torch.as_tensor(gn, device="cuda:0"), off, want_status=True, diag_repair=True)
    out = plan.run(torch.as_tensor(lmn, device="cuda:0"), torch.as_tensor(lrn, device="cuda:0"))
    rep, fail, inv = plan.check()
    assert rep == B and fail == 0 and inv == 0
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


@pytest.mark.parametrize("N", [24, 48])
def test_two_ev_types_in_one_plan(gpu, N):
    """Both EV types' sets stacked in one plan (one fused launch) give the per-type plans'
    answers bit for bit (same cell count), and match the oracle."""
    rng = np.random.default_rng(900 + N)
    cs = [O.small_consts(), O.large_consts()]
    P = 3
    sizes = [[700, 1, 2000], [1500, 0, 333]]
    lms, offs, gs, wrs = [], [], [], []
    for c, sz in zip(cs, sizes):
        offs.append(np.concatenate([[0], np.cumsum(sz)]).astype(np.int64))
        gs.append(torch.as_tensor(c.y_max - (0.3 + 0.2 * rng.random(sum(sz))), device="cuda:0"))
        lms.append(torch.as_tensor(c.theta * rng.random((P, 3 * N)), device="cuda:0"))
        wrs.append(torch.as_tensor(c.w_max * rng.random((P, N)), device="cuda:0"))
    lr = torch.zeros(2 * P, dtype=torch.float64, device="cuda:0")
    lompcs = [mk(c, N) for c in cs]
    off = np.concatenate([offs[0], offs[0][-1] + offs[1][1:]])
    both = BatchPlan(lompcs, torch.cat(gs), off, sets_per_ctx=[P, P], w_ref=torch.cat(wrs), want_status=True)
    ob = both.run(torch.cat(lms), lr)
    assert both.check()[1:] == (0, 0)
    B0 = int(offs[0][-1])
    for k in range(2):
        one = BatchPlan(lompcs[k], gs[k], offs[k], w_ref=wrs[k])
        assert one.cells == both.cells
        o1 = one.run(lms[k], lr[:P])
        torch.cuda.synchronize()
        sl = slice(0, B0) if k == 0 else slice(B0, None)
        assert torch.equal(o1["w"], ob["w"][sl]) and torch.equal(o1["cost"], ob["cost"][sl])
        assert torch.equal(o1["set_stats"], ob["set_stats"][k * P:(k + 1) * P])
        oracle_check(o1, gs[k], lms[k], lr[:P], offs[k], cs[k], N, rng, k=40)
    check_reductions(ob, off, N)


@pytest.mark.parametrize("ev", ["small", "large"])
def test_invalid_gamma_and_moved_gamma(gpu, ev):
    """gamma outside [0, y_max] or NaN: status INVALID, NaN outputs, counted per set, the rest
    exact; gamma moved in place after plan creation outside the set's window: re-solved
    individually (status REPAIRED) and exact."""
    rng = np.random.default_rng(12 + (ev == "large"))
    c = O.small_consts() if ev == "small" else O.large_consts()
    N = 24
    off = np.array([0, 500, 800], dtype=np.int64)
    gn = 0.3 + 0.2 * c.y_max * rng.random(800)
    bad = [3, 17, 501, 799]
    gn[bad] = [-0.1, np.nan, c.y_max + 1e-9, 5.0]
    g = torch.as_tensor(gn, device="cuda:0")
    lm = torch.as_tensor(c.theta * rng.random((2, 3 * N)), device="cuda:0")
    lr = torch.zeros(2, dtype=torch.float64, device="cuda:0")
    lompc = mk(c, N)
    plan = BatchPlan(lompc, g, off, want_status=True, want_w0=True, validate=False)
    out = plan.run(lm, lr)
    with pytest.raises(AssertionError):
        plan.check()
    st = out["status"].cpu().numpy()
    assert np.all(st[bad] == _lib.LOMPC_QP_INVALID)
    good = np.setdiff1d(np.arange(800), bad)
    assert np.all(st[good] == _lib.LOMPC_QP_OK)
    w = out["w"].cpu().numpy()
    assert np.all(np.isnan(w[bad])) and np.all(np.isnan(out["cost"].cpu().numpy()[bad]))
    stats = out["set_stats"].cpu().numpy()
    np.testing.assert_array_equal(stats[:, _lib.LOMPC_STAT_N_INVALID], [2, 2])
    np.testing.assert_allclose(stats[:, _lib.LOMPC_STAT_SUM_W0], [w[good[good < 500], 0].sum(),
                                                                 w[good[good >= 500], 0].sum()], rtol=1e-11)
    for s, idx in ((0, good[good < 500][:50]), (1, good[good >= 500][:50])):
        wo, _, nf = oracle_c.solve_batch(N, c, lm[s].cpu().numpy(), 0.0, gn[idx])
        np.testing.assert_allclose(w[idx], wo, atol=TOL_W)
    # move 10 valid EVs of set 0 far outside its window (and fix the invalid ones)
    g2 = gn.copy()
    g2[bad] = 0.5 * c.y_max
    g2[:10] = 0.02 * c.y_max
    g.copy_(torch.as_tensor(g2, device="cuda:0"))
    out2 = plan.run(lm, lr)
    rep, fail, inv = plan.check()
    assert fail == 0 and inv == 0 and rep >= 10
    st2 = out2["status"].cpu().numpy()
    assert np.all(st2[:10] == _lib.LOMPC_QP_REPAIRED)
    w2 = out2["w"].cpu().numpy()
    for s, idx in ((0, np.arange(0, 60)), (1, np.arange(500, 560))):
        wo, _, nf = oracle_c.solve_batch(N, c, lm[s].cpu().numpy(), 0.0, g2[idx])
        np.testing.assert_allclose(w2[idx], wo, atol=TOL_W)


@pytest.mark.parametrize("ev", ["small", "large"])
@pytest.mark.parametrize("N", [24, 48])
def test_warm_start_and_cell_counts(gpu, ev, N):
    """The answer does not depend on how the path is computed: warm-started cells (from the
    previous run's working sets), 16 / 64 / 512 cells and clustered gamma per set (station
    partitions by SoC) all give the same outputs to 1e-12 and match the oracle."""
    rng = np.random.default_rng(40 + N + (ev == "large"))
    c = O.small_consts() if ev == "small" else O.large_consts()
    sizes = [4000, 1, 0, 2500, 640]
    off = np.concatenate([[0], np.cumsum(sizes)]).astype(np.int64)
    S = len(sizes)
    lo = np.array([0.05, 0.4, 0.0, 0.6, 0.3]) * c.y_max
    gn = np.concatenate([lo[s] + 0.08 * c.y_max * rng.random(sizes[s]) for s in range(S)])
    g = torch.as_tensor(gn, device="cuda:0")
    lms = [torch.as_tensor(c.theta * rng.random((S, 3 * N)), device="cuda:0") for _ in range(3)]
    lr = torch.as_tensor(3 * N * c.delta * rng.random(S), device="cuda:0")
    wr = torch.as_tensor(c.w_max * rng.random((S, N)), device="cuda:0")
    lompc = mk(c, N)
    kw = dict(w_ref=wr, want_w=True, want_cost=True, want_status=True)
    cold = BatchPlan(lompc, g, off, **kw)
    warm = BatchPlan(lompc, g, off, warm_start=True, **kw)
    for k in range(3):
        oc = {n: v.clone() for n, v in cold.run(lms[k], lr).items() if v is not None}
        ow = warm.run(lms[k], lr)
        assert cold.check()[1:] == (0, 0) and warm.check()[1:] == (0, 0)
        np.testing.assert_allclose(ow["w"].cpu().numpy(), oc["w"].cpu().numpy(), rtol=0, atol=1e-12)
        np.testing.assert_allclose(ow["cost"].cpu().numpy(), oc["cost"].cpu().numpy(), rtol=1e-12, atol=1e-12)
        check_reductions(ow, off, N)
    oracle_check(oc, g, lms[2], lr, off, c, N, rng)
    for G in (1, 16, 512):
        p = BatchPlan(lompc, g, off, cells=G, **kw)
        assert p.cells == G
        o = p.run(lms[2], lr)
        assert p.check()[1:] == (0, 0)
        np.testing.assert_allclose(o["w"].cpu().numpy(), oc["w"].cpu().numpy(), rtol=0, atol=1e-12)
        np.testing.assert_allclose(o["set_sum_w"].cpu().numpy(), oc["set_sum_w"].cpu().numpy(), rtol=1e-11,
                                   atol=1e-10)


def test_status_tallies_every_run(gpu):
    """plan.check() sees a failure in ANY run since the previous check (sticky device tallies),
    not only the last run's: an invalid gamma in the middle one of three runs, and a negative price in
    the middle step of one run_steps call, both fail the check after the last run (the bench's
    correctness gate over its timed steps)."""
    rng = np.random.default_rng(8)
    c = O.large_consts()
    N, S, per = 24, 4, 3000
    off = np.arange(S + 1, dtype=np.int64) * per
    gn = c.y_max - (0.3 + 0.2 * rng.random(S * per))
    g = torch.as_tensor(gn, device="cuda:0")
    lm = torch.as_tensor(c.theta * rng.random((3, S, 3 * N)), device="cuda:0")
    lr = torch.zeros((3, S), dtype=torch.float64, device="cuda:0")
    lompc = mk(c, N)
    for want_w in (True, False):
        plan = BatchPlan(lompc, g, off, want_w=want_w, validate=False)
        plan.run(lm[0], lr[0])
        assert plan.check() == (0, 0, 0)
        g[per + 7] = -1.0  # run 2 of 3 sees one invalid EV
        plan.run(lm[0], lr[0])
        g[per + 7] = float(gn[per + 7])
        plan.run(lm[1], lr[1])
        with pytest.raises(AssertionError):
            plan.check()
        assert plan.check() == (0, 0, 0)  # read and zeroed: the next window is clean
        bad = lm.clone()
        bad[1, 2, 5] = -1.0  # a negative lambda_1 in the middle step of a run_steps call (H stays SPD)
        plan.run_steps(bad, lr, 3, bad[0].numel(), lr[0].numel())
        with pytest.raises(ValueError):
            plan.check()
        plan.run_steps(lm, lr, 3, lm[0].numel(), lr[0].numel())
        assert plan.check() == (0, 0, 0)


@pytest.mark.parametrize("ev", ["small", "large"])
def test_close_mode_sums_at_box_bounds(gpu, ev):
    """Runs without w close their sets inside k_eval from per-piece aggregates (n_p a + Gamma_p b,
    unclamped); runs with w sum the clamped rows.  With EVs at and next to the box bounds
    (gamma = 0: nothing left to charge; gamma = y_max: empty battery) the two agree to 1e-11 and
    match the per-EV oracle sums."""
    rng = np.random.default_rng(70 + (ev == "large"))
    c = O.small_consts() if ev == "small" else O.large_consts()
    N, per = 24, 2000
    gn = np.concatenate([np.zeros(300), np.full(300, c.y_max), 1e-9 * rng.random(300),
                         c.y_max - 1e-9 * rng.random(300), c.y_max * rng.random(per - 1200)])
    gn = np.concatenate([gn, c.y_max * rng.random(per)])
    off = np.array([0, per, 2 * per], dtype=np.int64)
    g = torch.as_tensor(gn, device="cuda:0")
    lm = torch.as_tensor(c.theta * rng.random((2, 3 * N)), device="cuda:0")
    lm[1, :N] = 0.0  # set 1: no charging price, the upper bound active
    lr = torch.as_tensor([0.0, 0.2], dtype=torch.float64, device="cuda:0")
    wr = torch.as_tensor(c.w_max * rng.random((2, N)), device="cuda:0")
    lompc = mk(c, N)
    full = BatchPlan(lompc, g, off, w_ref=wr, want_w=True, want_cost=True)
    red = BatchPlan(lompc, g, off, w_ref=wr, want_w=False, want_cost=True)
    of = full.run(lm, lr)
    orr = red.run(lm, lr)
    assert full.check()[1:] == (0, 0) and red.check()[1:] == (0, 0)
    np.testing.assert_allclose(orr["set_sum_w"].cpu().numpy(), of["set_sum_w"].cpu().numpy(), rtol=1e-11, atol=1e-11)
    np.testing.assert_allclose(orr["set_stats"].cpu().numpy(), of["set_stats"].cpu().numpy(), rtol=1e-11, atol=1e-11)
    lmn, lrn = lm.cpu().numpy(), lr.cpu().numpy()
    sw = orr["set_sum_w"].cpu().numpy()
    for s in range(2):
        wo, _, nf = oracle_c.solve_batch(N, c, lmn[s], lrn[s], gn[off[s]:off[s + 1]])
        assert nf == 0
        np.testing.assert_allclose(sw[s], wo.sum(0), rtol=1e-10, atol=1e-9)


@pytest.mark.parametrize("diag_repair", [False, True])
def test_close_in_eval_matches_k_finalize(gpu, diag_repair):
    """LOMPC_PLAN_CLOSE_IN_EVAL closes each set inside k_eval (its last-arriving workgroup reduces
    the set's records and re-solves the listed EVs); default plans run the same closing as the
    k_finalize launch.  Per-EV outputs are bitwise equal, the set reductions equal up to the
    summation order (8 vs 4 waves).  Empty sets (closed by the extra workgroup), sets of one EV,
    every EV re-solved (diag_repair), and repeated runs (the arrival counters reset)."""
    N, P = 24, 5
    rng = np.random.default_rng(33)
    cs = [O.small_consts(), O.large_consts()]
    lompcs = [LoMPC(N, LoMPCConstants(c.delta, c.theta, c.y_max, c.w_max, c.ev_type), device=0) for c in cs]
    sizes = [[700, 0, 333, 1, 0], [0, 512, 1, 0, 900]] if diag_repair else [[9000, 0, 4321, 1, 0], [0, 7000, 1, 0, 12000]]
    off = np.concatenate([[0], np.cumsum(np.concatenate(sizes))]).astype(np.int64)
    B = int(off[-1])
    ctx_of = np.repeat(np.arange(2 * P) // P, np.diff(off))
    g = torch.as_tensor(np.array([cs[k].y_max for k in ctx_of]) - (0.3 + 0.2 * rng.random(B)), device="cuda:0")
    wr = torch.as_tensor(np.concatenate([c.w_max * rng.random((P, N)) for c in cs]), device="cuda:0")
    lms = [torch.as_tensor(np.concatenate([c.theta * rng.random((P, 3 * N)) for c in cs]), device="cuda:0")
           for _ in range(3)]
    lr = torch.as_tensor(np.concatenate([[0.0, 0.1, 0.0, 0.2, 0.0]] * 2), device="cuda:0")
    outs = []
    for close in (True, False):
        plan = BatchPlan(lompcs, g, off, sets_per_ctx=[P, P], w_ref=wr, want_status=True, want_w0=True,
                         diag_repair=diag_repair, close_in_eval=close)
        res = []
        for lm in lms:
            out = plan.run(lm, lr)
            rep, fail, inv = plan.check()
            assert fail == 0 and inv == 0
            if diag_repair:
                assert rep == B
            res.append({k: v.clone() for k, v in out.items() if v is not None})
        outs.append(res)
    for a, b in zip(*outs):
        for k in a:
            if k in ("set_sum_w", "set_stats"):
                np.testing.assert_allclose(a[k].cpu().numpy(), b[k].cpu().numpy(), rtol=1e-12, atol=1e-12, err_msg=k)
            else:
                assert torch.equal(a[k], b[k]), k
        st = a["set_stats"].cpu().numpy()
        np.testing.assert_array_equal(st[:, 0], np.diff(off))  # LOMPC_STAT_COUNT, empty sets included


def test_reductions_only_runs_close_in_eval(gpu):
    """Runs without w output (a price loop's) close their sets inside k_eval by default; the
    same plan with close_in_finalize (k_finalize launch) gives the same costs bitwise and the same
    set reductions up to the summation order (an empty set and a set of one EV included)."""
    N, P = 48, 3
    rng = np.random.default_rng(5)
    c = O.large_consts()
    lo = LoMPC(N, LoMPCConstants(c.delta, c.theta, c.y_max, c.w_max, c.ev_type), device=0)
    off = np.array([0, 5000, 5000, 5001], dtype=np.int64)
    g = torch.as_tensor(c.y_max - (0.3 + 0.2 * rng.random(5001)), device="cuda:0")
    wr = torch.as_tensor(c.w_max * rng.random((P, N)), device="cuda:0")
    lm = torch.as_tensor(c.theta * rng.random((P, 3 * N)), device="cuda:0")
    lr = torch.as_tensor([0.0, 0.3, 0.1], dtype=torch.float64, device="cuda:0")
    outs = []
    for fin in (False, True):
        plan = BatchPlan(lo, g, off, w_ref=wr, want_w=False, want_cost=True, warm_start=True, close_in_finalize=fin)
        assert plan.launches_per_run() == (3 if fin else 2)
        res = []
        for _ in range(3):
            out = plan.run(lm, lr)
            assert plan.check()[1:] == (0, 0)
            res.append({k: v.clone() for k, v in out.items() if v is not None})
        outs.append(res)
    for a, b in zip(*outs):
        assert torch.equal(a["cost"], b["cost"])
        for k in ("set_sum_w", "set_stats"):
            np.testing.assert_allclose(a[k].cpu().numpy(), b[k].cpu().numpy(), rtol=1e-12, atol=1e-12, err_msg=k)


def same_sets(a, b, staged, what):
    """Set reductions of run_steps vs single runs: bitwise, or — in the wide form's staged evaluation
    (k_evals_st: seven row waves, so the rows' sums group differently) — to 1e-12 relative."""
    if not staged:
        assert torch.equal(a, b), what
        return
    an, bn = a.cpu().numpy(), b.cpu().numpy()
    np.testing.assert_allclose(an, bn, rtol=1e-12, atol=1e-12 * max(1.0, float(np.abs(bn).max())), err_msg=str(what))


@pytest.mark.parametrize("K", [2, 3, 7, 70])
@pytest.mark.parametrize("want_w", [True, False])
def test_run_steps_matches_single_runs(gpu, want_w, K):
    """lompc_plan_run_steps (K runs in one C-ABI call, the benchmark's timed steps) with per-run set
    outputs: EVERY run's set reductions equal those of an independent lompc_plan_run at the same
    prices bit for bit (the wide form's staged evaluation: to 1e-12, its row sums grouped by seven
    row waves), and the oracle's per-EV sums to 1e-9; the per-EV outputs equal the last run's bit for
    bit.  Both issue forms (stepped k_step and LOMPC_STEPS_PER_KERNEL, the same parts one launch
    each) give the same bits; HIP events sit on the sampled runs only; runs without w (their
    evaluation sums rows it does not store) take the stepped form too.  A plan whose cells do not
    fill whole path workgroups (6 cells) takes the launch-per-kernel form: the same equalities.
    K = 70 > 64: the wide form's paths in two launches and its table ring wrapped; the span events
    then cover the first path group's steady launches."""
    N, P, E = 24, 4, 3
    rng = np.random.default_rng(9)
    cs = [O.small_consts(), O.large_consts()]
    lompcs = [LoMPC(N, LoMPCConstants(c.delta, c.theta, c.y_max, c.w_max, c.ev_type), device=0) for c in cs]
    M = [6000, 5000]
    off1 = [np.array([(m * p) // P for p in range(P + 1)], dtype=np.int64) for m in M]
    off = np.concatenate([off1[0], M[0] + off1[1][1:]])
    gn = np.concatenate([c.y_max - (0.3 + 0.2 * rng.random(m)) for c, m in zip(cs, M)])
    g = torch.as_tensor(gn, device="cuda:0")
    lm = torch.as_tensor(np.stack([np.concatenate([c.theta * rng.random((P, 3 * N)) for c in cs]) for _ in range(K)]),
                         device="cuda:0")
    lr = torch.as_tensor(0.05 * rng.random((K, 2 * P)), device="cuda:0")
    for cells in (None, 6):
        # (single runs without w close in k_finalize here, summing rows as run_steps' evaluation does;
        # by default they close inside k_eval from piece aggregates, equal only to ~1e-12)
        kw = dict(sets_per_ctx=[P, P], want_status=True, want_w=want_w, cells=cells, close_in_finalize=True)
        ref = BatchPlan(lompcs, g, off, **kw)
        runs = []
        for k in range(K):
            runs.append({n: v.clone() for n, v in ref.run(lm[k], lr[k]).items() if v is not None})
        assert ref.check()[1:] == (0, 0)
        plan = BatchPlan(lompcs, g, off, **kw)
        plan.profile(enable=("k_eval",))
        plan.profile(read=True, reset=True)
        out = plan.run_steps(lm, lr, K, lm[0].numel(), lr[0].numel(), profile_every=E, per_run_sets=True)
        assert plan.check()[1:] == (0, 0)
        for key in ("w", "cost", "status"):
            if out.get(key) is not None:
                assert torch.equal(out[key], runs[-1][key]), key
        # (runs without w: the wide form's evaluation sums per-piece aggregates, n_p a_p + Gamma_p b_p
        # unclamped, where the single runs sum the clamped rows — equal to 1e-12, as the staged form)
        staged = plan.info()["evals_staged"] or (not want_w and cells is None)
        for k in range(K):
            for key in ("set_sum_w", "set_stats"):
                same_sets(out[key][k], runs[k][key], staged, (cells, k, key))
        ms, n = plan.profile(read=True)
        if cells is None:
            assert plan.info()["steps_group"] == 1  # (shared per-EV outputs: one run per launch)
            assert n >= (K - 1 + E - 1) // E and ms > 0.0
        # the same runs, one kernel per launch (without w: the batched kernels one run per group, whose
        # evaluation sums the certified pieces as the wide form's does): the same bits
        seq = BatchPlan(lompcs, g, off, **kw)
        out_s = seq.run_steps(lm, lr, K, lm[0].numel(), lr[0].numel(), per_run_sets=True, per_kernel=True)
        assert seq.check()[1:] == (0, 0)
        for key in ("w", "cost", "status", "set_sum_w", "set_stats"):
            if out.get(key) is not None:
                assert torch.equal(out[key], out_s[key]), key
        # every output per run (per-EV outputs at a per-run stride, every closing writes its run's
        # re-solved rows): every run's outputs those of its single run; the span events count the
        # steady-state launches
        for split in (False, True):
            pr = BatchPlan(lompcs, g, off, **kw)
            pr.profile(enable=("k_eval",))
            pr.profile(read=True, reset=True)
            o = pr.run_steps(lm, lr, K, lm[0].numel(), lr[0].numel(), per_run=True, per_kernel=split, span_events=True)
            assert pr.check()[1:] == (0, 0)
            if cells is None:
                assert pr.info()["steps_group"] == 1
                ms, n = pr.profile(read=True)
                # (batched: one pair around the first group's k_evals, read as its runs; split: the steady launches)
                # (the staged evaluation's split form: groups of one run, the pair around the first)
                one = pr.info()["evals_staged"] or not want_w  # (split: groups of one run, the pair around the first)
                exp = (1 if one else min(K, 64) - 1) if split else min(K, 64)
                assert n == exp and (ms > 0.0) == (n > 0)
            for k in range(K):
                for key in ("w", "cost", "status", "set_sum_w", "set_stats"):
                    if o.get(key) is not None:
                        if key in ("set_sum_w", "set_stats"):
                            same_sets(o[key][k], runs[k][key], pr.info()["evals_staged"] or not want_w,
                                      (cells, split, k, key))
                        else:
                            assert torch.equal(o[key][k], runs[k][key]), (cells, split, k, key)
    if K != 7 or not want_w:
        return
    # every run vs the oracle: per-set sums of the per-EV optima
    sw, st = out["set_sum_w"].cpu().numpy(), out["set_stats"].cpu().numpy()
    for k in range(K):
        for s in range(2 * P):
            a, b = off[s], off[s + 1]
            wo, co, nf = oracle_c.solve_batch(N, cs[s // P], lm[k, s].cpu().numpy(), float(lr[k, s]), gn[a:b])
            assert nf == 0
            np.testing.assert_allclose(sw[k, s], wo.sum(0), rtol=1e-10, atol=1e-9)
            assert abs(st[k, s, _lib.LOMPC_STAT_SUM_COST] - co.sum()) <= 1e-9 * max(1.0, abs(co.sum()))
            assert st[k, s, _lib.LOMPC_STAT_COUNT] == b - a


@pytest.mark.parametrize("N", [24, 48])
def test_run_steps_repairs_match_single_runs(gpu, N):
    """run_steps closes run k inside run k + 1's path launch (k_path_fin, one wave per set); its
    individual re-solves start from run k's cell-start working sets, which run k + 1's path must
    not overwrite (the two halves alternate).  With EVs moved outside the plan's gamma windows
    after its creation (re-solved individually from the edge cells' working sets) and
    warm-started paths, K runs through run_steps equal K single runs bit for bit, and the oracle."""
    rng = np.random.default_rng(60 + N)
    c = O.large_consts()
    sizes = [3000, 0, 1, 2570]
    off = np.concatenate([[0], np.cumsum(sizes)]).astype(np.int64)
    S, K, B = len(sizes), 3, int(off[-1])
    gn = c.y_max - (0.3 + 0.2 * rng.random(B))
    g = torch.as_tensor(gn, device="cuda:0")
    lm = torch.as_tensor(c.theta * rng.random((K, S, 3 * N)), device="cuda:0")
    lr = torch.as_tensor(0.05 * rng.random((K, S)), device="cuda:0")
    wr = torch.as_tensor(c.w_max * rng.random((S, N)), device="cuda:0")
    lompc = mk(c, N)
    kw = dict(w_ref=wr, want_w=True, want_cost=True, want_status=True, warm_start=True)
    ref = BatchPlan(lompc, g, off, **kw)
    plan = BatchPlan(lompc, g, off, **kw)
    moved = rng.choice(B, B // 10, replace=False)  # outside every window: below / above it
    gm = gn.copy()
    gm[moved] = np.where(rng.random(moved.size) < 0.5, 0.02 * rng.random(moved.size) * c.y_max,
                         c.y_max * (1.0 - 0.02 * rng.random(moved.size)))
    g.copy_(torch.as_tensor(gm))
    outs = []
    for k in range(K):
        outs.append({n: v.clone() for n, v in ref.run(lm[k], lr[k]).items() if v is not None})
    rep, fail, inv = ref.check()
    assert rep >= K * (moved.size - 2) and fail == 0 and inv == 0
    out = plan.run_steps(lm, lr, K, lm[0].numel(), lr[0].numel())
    assert plan.check() == (rep, 0, 0)
    for key in ("w", "cost", "status", "set_sum_w", "set_stats"):
        assert torch.equal(out[key], outs[-1][key]), key
    oracle_check(outs[-1], g, lm[-1], lr[-1], off, c, N, rng)


@pytest.mark.parametrize("N", [24, 48])
@pytest.mark.parametrize("diag_repair", [False, True])
def test_sorted_gamma_aggregation(gpu, N, diag_repair):
    """LOMPC_PLAN_SORTED_GAMMA: reductions-only runs aggregate each certified piece's EVs from
    prefix sums over the gamma-sorted set (k_agg) instead of evaluating every EV.  The set sums,
    costs, price0 sums, max A_bar errors and counts equal the full per-EV evaluation's (k_finalize
    over the w rows) to 1e-11 and the oracle's per-EV sums to 1e-9; sets: empty, one EV, one
    wave, clustered (duplicate gammas), 300 000 EVs, gammas at the box bounds, and invalid
    gammas after the valid ones (counted, AssertionError).  diag_repair: no certified pieces, every
    EV takes the individual re-solve path of k_agg.  An unsorted set reports all its EVs failed."""
    rng = np.random.default_rng(500 + N + diag_repair)
    cs = [O.small_consts(), O.large_consts()]
    lompcs = [mk(c, N) for c in cs]
    small = diag_repair  # the re-solve path: keep it short
    sizes = [[0, 1, 64, 3000], [2000, 0, 1500, 7]] if small else [[0, 1, 64, 300000], [20000, 0, 1500, 7]]
    parts = []
    for k, c in enumerate(cs):
        for j, m in enumerate(sizes[k]):
            g = c.y_max * rng.random(m)
            if m == 1500:
                g = np.repeat(c.y_max * rng.random(50), 30)  # clustered, duplicates
            if m >= 2000:
                g[:5] = 0.0
                g[5:10] = c.y_max
            parts.append(np.sort(g))
    off = np.concatenate([[0], np.cumsum([len(x) for x in parts])]).astype(np.int64)
    P = len(sizes[0])
    gn = np.concatenate(parts)
    g = torch.as_tensor(gn, device="cuda:0")
    lm = torch.as_tensor(np.concatenate([c.theta * rng.random((P, 3 * N)) for c in cs]), device="cuda:0")
    lr = torch.as_tensor(np.concatenate([[0.0, 0.3, 0.0, 0.1]] * 2), device="cuda:0")
    wr = torch.as_tensor(np.concatenate([c.w_max * rng.random((P, N)) for c in cs]), device="cuda:0")
    kw = dict(sets_per_ctx=[P, P], w_ref=wr, diag_repair=diag_repair)
    agg = BatchPlan(lompcs, g, off, want_w=False, want_cost=False, sorted_gamma=True, **kw)
    full = BatchPlan(lompcs, g, off, want_w=True, want_cost=True, **kw)
    assert agg.launches_per_run() == 2
    oa = {k: v.clone() for k, v in agg.run(lm, lr).items() if v is not None}
    of = full.run(lm, lr)
    ra, fa, ia = agg.check()
    rf, ff, i_f = full.check()
    assert (fa, ia) == (0, 0) and (ff, i_f) == (0, 0) and ra == rf
    if diag_repair:
        assert ra == len(gn)
    np.testing.assert_allclose(oa["set_sum_w"].cpu().numpy(), of["set_sum_w"].cpu().numpy(), rtol=1e-11, atol=1e-9)
    sa, sf = oa["set_stats"].cpu().numpy(), of["set_stats"].cpu().numpy()
    np.testing.assert_array_equal(sa[:, _lib.LOMPC_STAT_COUNT], np.diff(off))
    np.testing.assert_allclose(sa, sf, rtol=1e-11, atol=1e-9)
    w, cost = of["w"].cpu().numpy(), of["cost"].cpu().numpy()
    for s in range(2 * P):
        a, b = off[s], off[s + 1]
        if b == a:
            continue
        c = cs[s // P]
        wo, co, nf = oracle_c.solve_batch(N, c, lm[s].cpu().numpy(), float(lr[s]), gn[a:b])
        assert nf == 0
        np.testing.assert_allclose(oa["set_sum_w"][s].cpu().numpy(), wo.sum(0), rtol=1e-10, atol=1e-9)
        assert abs(sa[s, _lib.LOMPC_STAT_SUM_COST] - co.sum()) <= 1e-10 * max(1.0, abs(co.sum()))
    # repeated runs at other prices through the same prefix sums
    lm2 = lm.flip(1).contiguous()
    oa2 = agg.run(lm2, lr)
    of2 = full.run(lm2, lr)
    assert agg.check()[1:] == (0, 0) and full.check()[1:] == (0, 0)
    np.testing.assert_allclose(oa2["set_stats"].cpu().numpy(), of2["set_stats"].cpu().numpy(), rtol=1e-11, atol=1e-9)
    if small:
        return
    # invalid gammas after the valid ones: counted; an unsorted set: every EV failed
    g2 = gn.copy()
    e = off[P + 1]  # end of the second type's first set
    g2[e - 3:e] = [np.nan, -1.0, 7.0]
    bad = BatchPlan(lompcs, torch.as_tensor(g2, device="cuda:0"), off, want_w=False, want_cost=False,
                    sorted_gamma=True, validate=False, **kw)
    ob = bad.run(lm, lr)
    with pytest.raises(AssertionError):
        bad.check()
    assert ob["set_stats"].cpu().numpy()[P, _lib.LOMPC_STAT_N_INVALID] == 3
    g3 = gn.copy()
    g3[off[3] + 10], g3[off[3] + 11] = g3[off[3] + 11], g3[off[3] + 10] + 1e-3
    uns = BatchPlan(lompcs, torch.as_tensor(g3, device="cuda:0"), off, want_w=False, want_cost=False,
                    sorted_gamma=True, **kw)
    ou = uns.run(lm, lr)
    with pytest.raises(Exception):
        uns.check()
    assert ou["set_stats"].cpu().numpy()[3, _lib.LOMPC_STAT_N_FAILED] == off[4] - off[3]


@pytest.mark.parametrize("reserve", [0, 200000])
def test_plan_update_matches_fresh_plan(gpu, reserve):
    """lompc_plan_update re-targets one plan at batches of changing size (the station's partition
    plans: EVs move between partitions) — growing and shrinking, with and without the
    lompc_plan_reserve size hint — and every run equals, bitwise, a plan freshly created for that
    batch (sorted sets without per-EV output, the loop plans' kind; and a plan with w rows)."""
    rng = np.random.default_rng(33)
    N = 24
    c = O.large_consts()
    lompc = mk(c, N)
    for kw in (dict(want_w=False, want_cost=False, sorted_gamma=True), dict(want_w=True, want_cost=True)):
        plan = None
        for m in (1000, 50000, 300, 120000, 7, 90000):
            g = np.sort(c.y_max * rng.random(m))
            off = np.array([0, m // 3, m], dtype=np.int64)
            gt = torch.as_tensor(g, device="cuda:0")
            lm = torch.as_tensor(c.theta * rng.random((2, 3 * N)), device="cuda:0")
            lr = torch.as_tensor([0.1, 0.0], device="cuda:0")
            if plan is None:
                plan = BatchPlan(lompc, gt, off, **kw)
                if reserve:
                    plan.reserve(reserve)
            else:
                plan.update(gt, off)
            o1 = {k: v.clone() for k, v in plan.run(lm, lr).items() if v is not None}
            assert plan.check()[1:] == (0, 0)
            fresh = BatchPlan(lompc, gt, off, **kw)
            o2 = fresh.run(lm, lr)
            assert fresh.check()[1:] == (0, 0)
            for k, v in o2.items():
                if v is not None:
                    assert torch.equal(o1[k], v), (m, k)


def test_run_steps_sorted_wide(gpu):
    """run_steps over gamma-sorted sets without per-EV output (the reductions contract on the
    station's sorted partitions): per group of up to 64 runs ONE k_paths and ONE k_aggs launch (one
    workgroup per (run, set), k_agg's per-piece aggregation on the run's ring slot).  Every run's set
    sums and stats equal, bitwise, the sequential form (LOMPC_STEPS_PER_KERNEL: k_path + k_agg per run)
    and single runs; 70 runs take two groups (the ring wraps); shared outputs hold the last run's; the
    sums match the oracle's per-EV sums (rtol 1e-10, atol 1e-9, test_sorted_gamma_aggregation's bar);
    empty, one-EV, clustered and box-bound sets."""
    rng = np.random.default_rng(71)
    N, K = 24, 70
    cs = [O.small_consts(), O.large_consts()]
    lompcs = [mk(c, N) for c in cs]
    sizes = [[0, 1, 64, 30000], [20000, 0, 1500, 7]]
    parts = []
    for k, c in enumerate(cs):
        for m in sizes[k]:
            g = c.y_max * rng.random(m)
            if m == 1500:
                g = np.repeat(c.y_max * rng.random(50), 30)
            if m >= 20000:
                g[:5] = 0.0
                g[5:10] = c.y_max
            parts.append(np.sort(g))
    off = np.concatenate([[0], np.cumsum([len(x) for x in parts])]).astype(np.int64)
    P = len(sizes[0])
    gn = np.concatenate(parts)
    g = torch.as_tensor(gn, device="cuda:0")
    lm = torch.as_tensor(np.stack([np.concatenate([c.theta * rng.random((P, 3 * N)) for c in cs]) for _ in range(K)]),
                         device="cuda:0")
    lr = torch.as_tensor(0.2 * rng.random((K, 2 * P)), device="cuda:0")
    wr = torch.as_tensor(np.concatenate([c.w_max * rng.random((P, N)) for c in cs]), device="cuda:0")
    agg = BatchPlan(lompcs, g, off, sets_per_ctx=[P, P], w_ref=wr, want_w=False, want_cost=False, sorted_gamma=True)
    st = (lm[0].numel(), lr[0].numel())
    ow = {k: v.clone() for k, v in agg.run_steps(lm, lr, K, *st, per_run_sets=True).items() if v is not None}
    rw, fw, iw = agg.check()
    assert (fw, iw) == (0, 0)
    osq = agg.run_steps(lm, lr, K, *st, per_run_sets=True, per_kernel=True)
    assert agg.check() == (rw, 0, 0)
    for key in ("set_sum_w", "set_stats"):
        assert torch.equal(ow[key], osq[key]), key
    for k in (0, 1, 63, 64, K - 1):
        o1 = agg.run(lm[k], lr[k])
        assert torch.equal(o1["set_sum_w"], ow["set_sum_w"][k]) and torch.equal(o1["set_stats"], ow["set_stats"][k]), k
    agg.check()
    osh = agg.run_steps(lm, lr, K, *st)  # shared outputs: the last run's
    assert agg.check()[1:] == (0, 0)
    assert torch.equal(osh["set_sum_w"], ow["set_sum_w"][-1]) and torch.equal(osh["set_stats"], ow["set_stats"][-1])
    sa = ow["set_stats"].cpu().numpy()
    np.testing.assert_array_equal(sa[:, :, _lib.LOMPC_STAT_COUNT], np.broadcast_to(np.diff(off), (K, 2 * P)))
    for k in (0, 64, K - 1):
        for s in range(2 * P):
            a, b = off[s], off[s + 1]
            if b == a:
                continue
            c = cs[s // P]
            wo, co, nf = oracle_c.solve_batch(N, c, lm[k, s].cpu().numpy(), float(lr[k, s]), gn[a:b])
            assert nf == 0
            np.testing.assert_allclose(ow["set_sum_w"][k, s].cpu().numpy(), wo.sum(0), rtol=1e-10, atol=1e-9)
            assert abs(sa[k, s, _lib.LOMPC_STAT_SUM_COST] - co.sum()) <= 1e-10 * max(1.0, abs(co.sum()))


def test_sort_sets_plan_on_unsorted_batch(gpu):
    """BatchPlan(sort_sets=True) over an UNSORTED batch (the reductions contract: only per-set sums
    leave, so the order inside a set is free): the plan snapshots gamma with each set sorted on the
    device and runs as a sorted_gamma plan — its run_steps (k_paths + k_aggs) equal, bitwise, a
    sorted_gamma plan over the host-sorted batch, and the oracle's per-EV sums (rtol 1e-10, atol 1e-9);
    NaN / out-of-range gammas sort after the valid ones and are counted invalid; a plan asking for
    per-EV outputs is refused."""
    rng = np.random.default_rng(12)
    N, K, P = 24, 5, 3
    cs = [O.small_consts(), O.large_consts()]
    lompcs = [mk(c, N) for c in cs]
    sizes = [[5000, 1, 0], [20000, 64, 333]]
    parts = [c.y_max * rng.random(m) for c, ms in zip(cs, sizes) for m in ms]
    off = np.concatenate([[0], np.cumsum([len(x) for x in parts])]).astype(np.int64)
    gn = np.concatenate(parts)
    lm = torch.as_tensor(np.stack([np.concatenate([c.theta * rng.random((P, 3 * N)) for c in cs]) for _ in range(K)]),
                         device="cuda:0")
    lr = torch.as_tensor(0.1 * rng.random((K, 2 * P)), device="cuda:0")
    kw = dict(sets_per_ctx=[P, P], want_w=False, want_cost=False)
    st = (lm[0].numel(), lr[0].numel())
    a = BatchPlan(lompcs, torch.as_tensor(gn, device="cuda:0"), off, sort_sets=True, **kw)
    gs = np.concatenate([np.sort(gn[off[s]:off[s + 1]]) for s in range(2 * P)])
    b = BatchPlan(lompcs, torch.as_tensor(gs, device="cuda:0"), off, sorted_gamma=True, **kw)
    oa = {k: v.clone() for k, v in a.run_steps(lm, lr, K, *st, per_run_sets=True).items() if v is not None}
    ob = b.run_steps(lm, lr, K, *st, per_run_sets=True)
    assert a.check()[1:] == (0, 0) and b.check()[1:] == (0, 0)
    for key in ("set_sum_w", "set_stats"):
        assert torch.equal(oa[key], ob[key]), key
    for s in range(2 * P):
        if off[s + 1] == off[s]:
            continue
        wo, co, nf = oracle_c.solve_batch(N, cs[s // P], lm[K - 1, s].cpu().numpy(), float(lr[K - 1, s]), gn[off[s]:off[s + 1]])
        assert nf == 0
        np.testing.assert_allclose(oa["set_sum_w"][K - 1, s].cpu().numpy(), wo.sum(0), rtol=1e-10, atol=1e-9)
    g2 = gn.copy()
    g2[[3, 40, 4000]] = [np.nan, 2.0 * cs[0].y_max, np.nan]
    c = BatchPlan(lompcs, torch.as_tensor(g2, device="cuda:0"), off, sort_sets=True, validate=False, **kw)
    oc = c.run(lm[0], lr[0])
    with pytest.raises(AssertionError):
        c.check()
    assert oc["set_stats"].cpu().numpy()[0, _lib.LOMPC_STAT_N_INVALID] == 3
    with pytest.raises(ValueError):
        BatchPlan(lompcs, torch.as_tensor(gn, device="cuda:0"), off, sets_per_ctx=[P, P], sort_sets=True)


@pytest.mark.parametrize("ev", ["small", "large"])
def test_run_steps_piece_sums_match_oracle(gpu, ev):
    """The reductions-only contract (price_solver.py:196-214: only the per-set sums of w, the max
    A_bar error and the counts leave) through the wide run_steps: its evaluation sums each certified
    piece's EVs from their count and fixed-point gamma sum (n_p a_p + Gamma_p b_p, unclamped) instead of
    evaluating N rows per EV.  Every run's sums equal the oracle's per-EV sums (to the unclamped
    aggregates' documented tolerance, DESIGN §10: rtol 1e-10, atol 1e-9), with EVs at and next to the
    box bounds, a set of one EV and an empty set; the max error and the counts as the rows form."""
    rng = np.random.default_rng(90 + (ev == "large"))
    c = O.small_consts() if ev == "small" else O.large_consts()
    N, K = 24, 5
    parts = [np.concatenate([np.zeros(200), np.full(200, c.y_max), 1e-9 * rng.random(200),
                             c.y_max - 1e-9 * rng.random(200), c.y_max * rng.random(3000)]),
             c.y_max * rng.random(1), np.zeros(0), c.y_max - (0.3 + 0.2 * rng.random(9000))]
    gn = np.concatenate(parts)
    off = np.concatenate([[0], np.cumsum([len(x) for x in parts])]).astype(np.int64)
    S = len(parts)
    g = torch.as_tensor(gn, device="cuda:0")
    lm = torch.as_tensor(c.theta * rng.random((K, S, 3 * N)), device="cuda:0")
    lm[:, 0, :N] = 0.0  # (set 0: no charging price, the upper bound active)
    lr = torch.as_tensor(0.1 * rng.random((K, S)), device="cuda:0")
    wr = torch.as_tensor(c.w_max * rng.random((S, N)), device="cuda:0")
    lompc = mk(c, N)
    red = BatchPlan(lompc, g, off, w_ref=wr, want_w=False, want_cost=False, cells=4)
    rows = BatchPlan(lompc, g, off, w_ref=wr, want_w=True, want_cost=False, cells=4)
    o = red.run_steps(lm, lr, K, lm[0].numel(), lr[0].numel(), per_run_sets=True)
    orow = rows.run_steps(lm, lr, K, lm[0].numel(), lr[0].numel(), per_run_sets=True)
    assert red.check()[1:] == (0, 0) and rows.check()[1:] == (0, 0)
    sw, st = o["set_sum_w"].cpu().numpy(), o["set_stats"].cpu().numpy()
    stw = orow["set_stats"].cpu().numpy()
    np.testing.assert_allclose(sw, orow["set_sum_w"].cpu().numpy(), rtol=1e-11, atol=1e-11)
    np.testing.assert_array_equal(st[:, :, _lib.LOMPC_STAT_MAX_ERR], stw[:, :, _lib.LOMPC_STAT_MAX_ERR])
    np.testing.assert_array_equal(st[:, :, _lib.LOMPC_STAT_COUNT], stw[:, :, _lib.LOMPC_STAT_COUNT])
    lmn, lrn = lm.cpu().numpy(), lr.cpu().numpy()
    for k in range(K):
        for s in range(S):
            a, b = off[s], off[s + 1]
            assert st[k, s, _lib.LOMPC_STAT_COUNT] == b - a
            if b == a:
                assert np.all(sw[k, s] == 0.0)
                continue
            wo, _, nf = oracle_c.solve_batch(N, c, lmn[k, s], float(lrn[k, s]), gn[a:b])
            assert nf == 0
            np.testing.assert_allclose(sw[k, s], wo.sum(0), rtol=1e-10, atol=1e-9, err_msg=f"run {k} set {s}")
