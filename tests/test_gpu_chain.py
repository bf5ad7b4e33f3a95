"""GPU tests of lompc_plan_run_chain: K DEPENDENT runs, run k's prices computed on the device from
run k-1's set reductions (the call pattern of the reference's price loop, price_solver.py:111-140,
which no independent batching can follow).

* the prices of every run follow the documented rule from the previous run's reductions (host
  restatement of the projected dual-gradient step; phi of lompc.py:172-177), to rounding;
* every run's set reductions equal an independent wide run_steps over the recorded prices bit for
  bit (the same optima, the same closing order), and the oracle's per-EV sums to 1e-9;
* a warm-started plan (the price loops' form) gives the same reductions to 1e-12.
"""
import numpy as np
import pytest
import torch

import lompc_oracle as O
import oracle_c
from lompc_amd import BatchPlan, LoMPC, LoMPCConstants, _lib

pytestmark = pytest.mark.gpu


def phi(c, w):
    q_s = 3 * c.theta / (4 * c.w_max)
    return np.concatenate([c.theta * w, c.theta * (c.w_max - w), q_s * w * w], axis=-1)


def setup(rng, N=24, P=4, M=(6000, 5000)):
    cs = [O.small_consts(), O.large_consts()]
    lompcs = [LoMPC(N, LoMPCConstants(c.delta, c.theta, c.y_max, c.w_max, c.ev_type), device=0) for c in cs]
    off1 = [np.array([(m * p) // P for p in range(P + 1)], dtype=np.int64) for m in M]
    off = np.concatenate([off1[0], M[0] + off1[1][1:]])
    gn = np.concatenate([c.y_max - (0.3 + 0.2 * rng.random(m)) for c, m in zip(cs, M)])
    lm0 = np.concatenate([c.theta * rng.random((P, 3 * N)) for c in cs])
    wt = np.concatenate([c.w_max * (0.2 + 0.6 * rng.random((P, N))) for c in cs])
    return cs, lompcs, off, gn, lm0, wt


@pytest.mark.parametrize("want_w", [True, False])
def test_run_chain_follows_its_rule_and_matches_independent_runs(gpu, want_w):
    N, P, K, step = 24, 4, 6, 0.5
    rng = np.random.default_rng(21)
    cs, lompcs, off, gn, lm0, wt = setup(rng, N, P)
    g = torch.as_tensor(gn, device="cuda:0")
    lr = torch.as_tensor(0.05 * rng.random(2 * P), device="cuda:0")
    kw = dict(sets_per_ctx=[P, P], want_w=want_w, want_cost=True, close_in_finalize=True)
    plan = BatchPlan(lompcs, g, off, w_ref=torch.as_tensor(wt, device="cuda:0"), **kw)
    out = plan.run_chain(lm0, lr, wt, step, K)
    assert plan.check()[1:] == (0, 0)
    lm = out["lmbd"].cpu().numpy()
    sw, st = out["set_sum_w"].cpu().numpy(), out["set_stats"].cpu().numpy()
    np.testing.assert_array_equal(lm[0], lm0)
    # (1) the rule, restated on the host from run k-1's reductions
    for k in range(1, K):
        for s in range(2 * P):
            c = cs[s // P]
            wb = sw[k - 1, s] / st[k - 1, s, _lib.LOMPC_STAT_COUNT]
            exp = np.maximum(0.0, lm[k - 1, s] + step * (phi(c, wb) - phi(c, wt[s])))
            np.testing.assert_allclose(lm[k, s], exp, rtol=1e-14, atol=1e-14 * c.theta)
        assert not np.array_equal(lm[k], lm[k - 1])  # the prices move
    # (2) every run = an independent wide run_steps at the recorded prices: per-EV outputs bit for bit,
    # set reductions bit for bit (or, through the staged evaluation k_evals_st, whose row sums group by
    # seven row waves, to 1e-12; without w rows the wide form's sums come from the certified pieces'
    # counts and fixed-point gamma sums, unclamped — to the piece aggregates' tolerance, rtol 1e-10,
    # atol 1e-9, as test_gpu_pipeline.py::test_run_steps_piece_sums_match_oracle)
    ref = BatchPlan(lompcs, g, off, w_ref=torch.as_tensor(wt, device="cuda:0"), **kw)
    o = ref.run_steps(out["lmbd"], lr, K, 2 * P * 3 * N, 0, per_run_sets=True)
    assert ref.check()[1:] == (0, 0)
    staged = ref.info()["evals_staged"]
    for k in range(K):
        for key in ("set_sum_w", "set_stats"):
            if staged:
                a_, b_ = o[key][k].cpu().numpy(), out[key][k].cpu().numpy()
                np.testing.assert_allclose(a_, b_, rtol=1e-12, atol=1e-12 * max(1.0, float(np.abs(b_).max())))
            elif not want_w:
                a_, b_ = o[key][k].cpu().numpy(), out[key][k].cpu().numpy()
                np.testing.assert_allclose(a_, b_, rtol=1e-10, atol=1e-9)
            else:
                assert torch.equal(o[key][k], out[key][k]), (k, key)
    for key in ("w", "cost"):
        if o.get(key) is not None:
            assert torch.equal(o[key], out[key]), key
    # (3) the oracle's per-EV sums at the first and last run
    for k in (0, K - 1):
        for s in range(2 * P):
            a, b = off[s], off[s + 1]
            wo, co, nf = oracle_c.solve_batch(N, cs[s // P], lm[k, s], float(lr[s]), gn[a:b])
            assert nf == 0
            np.testing.assert_allclose(sw[k, s], wo.sum(0), rtol=1e-10, atol=1e-9)
            assert abs(st[k, s, _lib.LOMPC_STAT_SUM_COST] - co.sum()) <= 1e-9 * max(1.0, abs(co.sum()))


def test_run_chain_warm_plan_and_errors(gpu):
    """A warm-started plan (each cell's start solve from the previous run's working set: the price
    loops' plans) follows the same chain to 1e-12; bad arguments raise."""
    N, P, K, step = 48, 3, 5, 0.3
    rng = np.random.default_rng(22)
    cs, lompcs, off, gn, lm0, wt = setup(rng, N, P, M=(4000, 3000))
    g = torch.as_tensor(gn, device="cuda:0")
    lr = torch.zeros(2 * P, dtype=torch.float64, device="cuda:0")
    outs = []
    for warm in (False, True):
        plan = BatchPlan(lompcs, g, off, sets_per_ctx=[P, P], want_w=True, want_cost=True, warm_start=warm)
        o = plan.run_chain(lm0, lr, wt, step, K)
        assert plan.check()[1:] == (0, 0)
        outs.append({k: o[k].cpu().numpy() for k in ("lmbd", "set_sum_w", "set_stats", "w")})
    a, b = outs
    for k in ("lmbd", "set_sum_w", "w"):
        np.testing.assert_allclose(b[k], a[k], rtol=1e-12, atol=1e-12, err_msg=k)
    np.testing.assert_array_equal(b["set_stats"][:, :, 0], a["set_stats"][:, :, 0])
    with pytest.raises(ValueError):
        plan.run_chain(lm0, lr, wt, -1.0, K)
    nos = BatchPlan(lompcs, g, off, sets_per_ctx=[P, P], want_set=False)
    with pytest.raises(ValueError):
        nos.run_chain(lm0, lr, wt, step, K)
