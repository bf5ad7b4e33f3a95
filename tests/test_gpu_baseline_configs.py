"""GPU parity at BASELINE.json's batch configurations, every EV checked against the C oracle
(oracle/lompc_oracle.c: dense primal active set, an independent restatement of
lompc.py:92-156; the reference's own timing harness draws test_lompc.py:34-36).

* config 2: 4 096 EVs, horizon 24, half small / half large, 12 partitions per type,
  lmbd ~ theta U[0,1]^{3N}, lmbd_r in {0, 3 N delta U[0,1]}, seeds {0, 1, 2};
* config 3: 262 144 EVs, horizon 24 (the bench's workload): one two-type plan, all EVs;
* config 4's workload on one GPU: 2 097 152 EVs, horizon 24, all EVs, plus the 8-way EV
  sharding of BASELINE config 4 (8 shard plans, per-rank reductions combined in rank order as
  lompc_amd.dist.combine_set_results does) against the unsharded reductions.

Tolerances: |dw| <= 1e-9 absolute, cost 1e-9 relative (1e-9 absolute floor); reductions equal
the sums of the per-EV outputs to 1e-11 relative.
"""
import numpy as np
import pytest
import torch

import lompc_oracle as O
import oracle_c
from lompc_amd import BatchPlan, LoMPC, LoMPCConstants, _lib
from lompc_amd.dist import shard_sets

pytestmark = pytest.mark.gpu

TOL_W = 1e-9
CS = [O.small_consts(), O.large_consts()]


def mk(c, N):
    return LoMPC(N, LoMPCConstants(c.delta, c.theta, c.y_max, c.w_max, c.ev_type), device=0)


def station_batch(B, N, P, rng, lr_random=False):
    """Half small / half large EVs, P partitions per type (2P sets, small first): gamma = y_max - y0,
    y0 ~ U[0.3, 0.5] (settings.py:27-28), lmbd ~ theta U[0,1]^{3N} (test_lompc.py:34),
    lmbd_r = 0 (charging_station.py:162) or 3 N delta U[0,1] (test_lompc.py:35)."""
    M = [B // 2, B - B // 2]
    off1 = [np.array([(m * p) // P for p in range(P + 1)], dtype=np.int64) for m in M]
    off = np.concatenate([off1[0], M[0] + off1[1][1:]])
    g = np.concatenate([c.y_max - (0.3 + 0.2 * rng.random(m)) for c, m in zip(CS, M)])
    lm = np.concatenate([c.theta * rng.random((P, 3 * N)) for c in CS])
    lr = np.concatenate([3 * N * c.delta * rng.random(P) if lr_random else np.zeros(P) for c in CS])
    wr = np.concatenate([c.w_max * rng.random((P, N)) for c in CS])
    return off, g, lm, lr, wr


def check_all(out, off, g, lm, lr, N, P):
    w = out["w"].cpu().numpy()
    cost = out["cost"].cpu().numpy()
    sw = out["set_sum_w"].cpu().numpy()
    st = out["set_stats"].cpu().numpy()
    for s in range(2 * P):
        a, b = off[s], off[s + 1]
        c = CS[s // P]
        wo, co, nf = oracle_c.solve_batch(N, c, lm[s], lr[s], g[a:b])
        assert nf == 0
        dw = np.max(np.abs(w[a:b] - wo)) if b > a else 0.0
        assert dw <= TOL_W, (s, dw)
        np.testing.assert_allclose(cost[a:b], co, rtol=1e-9, atol=1e-9)
        np.testing.assert_allclose(sw[s], w[a:b].sum(0), rtol=1e-11, atol=1e-9)
        np.testing.assert_allclose(st[s, _lib.LOMPC_STAT_SUM_COST], cost[a:b].sum(), rtol=1e-11, atol=1e-9)
        assert st[s, _lib.LOMPC_STAT_COUNT] == b - a
        assert st[s, _lib.LOMPC_STAT_N_FAILED] == 0 and st[s, _lib.LOMPC_STAT_N_INVALID] == 0


def run_plan(off, g, lm, lr, wr, N, P, **kw):
    lompcs = [mk(c, N) for c in CS]
    gt = torch.as_tensor(g, device="cuda:0")
    plan = BatchPlan(lompcs, gt, off, sets_per_ctx=[P, P], w_ref=torch.as_tensor(wr, device="cuda:0"), **kw)
    out = plan.run(torch.as_tensor(lm, device="cuda:0"), torch.as_tensor(lr, device="cuda:0"))
    rep, fail, inv = plan.check()
    assert fail == 0 and inv == 0
    return plan, out


@pytest.mark.parametrize("seed", [0, 1, 2])
@pytest.mark.parametrize("lr_random", [False, True], ids=["lr0", "lrU"])
def test_config2_all_evs(gpu, seed, lr_random):
    N, P, B = 24, 12, 4096
    rng = np.random.default_rng(seed)
    off, g, lm, lr, wr = station_batch(B, N, P, rng, lr_random)
    _, out = run_plan(off, g, lm, lr, wr, N, P)
    check_all(out, off, g, lm, lr, N, P)


def test_config3_all_evs(gpu):
    N, P, B = 24, 12, 262144
    rng = np.random.default_rng(3)
    off, g, lm, lr, wr = station_batch(B, N, P, rng)
    plan, out = run_plan(off, g, lm, lr, wr, N, P, want_status=True)
    check_all(out, off, g, lm, lr, N, P)
    assert np.all(out["status"].cpu().numpy() <= _lib.LOMPC_QP_REPAIRED)
    w1 = out["w"].clone()
    sw1 = out["set_sum_w"].clone()
    plan.run(torch.as_tensor(lm, device="cuda:0"), torch.as_tensor(lr, device="cuda:0"))
    torch.cuda.synchronize()
    assert torch.equal(w1, out["w"]) and torch.equal(sw1, out["set_sum_w"])  # bitwise reproducible


def test_config4_workload_and_sharding(gpu):
    N, P, B = 24, 12, 2097152
    rng = np.random.default_rng(4)
    off, g, lm, lr, wr = station_batch(B, N, P, rng)
    plan, out = run_plan(off, g, lm, lr, wr, N, P)
    check_all(out, off, g, lm, lr, N, P)
    sw_full = out["set_sum_w"].cpu().numpy()
    st_full = out["set_stats"].cpu().numpy()
    w_full = out["w"]
    del plan, out
    # BASELINE config 4: the EV batch sharded 8 ways (dist.shard_sets: every set's EVs split
    # contiguously over the ranks), each shard its own plan; the per-rank reductions combined in
    # rank order (sums, max of the A_bar error) as combine_set_results does after its all-gather
    world = 8
    sw_tot, st_tot = None, None
    for rank in range(world):
        idx, loc = shard_sets(off, rank, world)
        _, o = run_plan(loc, g[idx], lm, lr, wr, N, P)
        dw = (o["w"] - w_full[torch.as_tensor(idx, device="cuda:0")]).abs().max().item()
        assert dw <= 1e-12, dw  # the shard's own gamma windows and cells: the same optimum
        sw, st = o["set_sum_w"].cpu().numpy(), o["set_stats"].cpu().numpy()
        if sw_tot is None:
            sw_tot, st_tot = sw.copy(), st.copy()
        else:
            sw_tot += sw
            mx = np.maximum(st_tot[:, _lib.LOMPC_STAT_MAX_ERR], st[:, _lib.LOMPC_STAT_MAX_ERR])
            st_tot += st
            st_tot[:, _lib.LOMPC_STAT_MAX_ERR] = mx
    np.testing.assert_allclose(sw_tot, sw_full, rtol=1e-11, atol=1e-9)
    np.testing.assert_allclose(st_tot, st_full, rtol=1e-11, atol=1e-9)
