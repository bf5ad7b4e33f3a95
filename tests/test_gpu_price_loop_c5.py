"""Open-loop parity of the station's device price loop at config-5 partition size.

Config 5 (BASELINE.json) runs 2 097 152 EVs at horizon 48, 12 partitions per EV type: about
87 000 EVs per (type, partition) price loop (charging_station.py:268-308).  Here, per EV type,
three consecutive partitions of 87 381 EVs (= 2^20 / 12), charge levels uniform over the
station's partition ranges (np.linspace(MIN_INITIAL_SOC, y_max, P + 1), charging_station.py:
85-90), laid out as the station lays them out (descending charge level, each partition's plan
staged ahead, stage_partition / use_partition), run through ``PriceSolver.compute_optimal_prices``
in its default form — the device-resident loop, one ``k_loop_iter`` launch per price iteration —
with prev_prices chaining the partitions (price_solver.py:104, :166).  The checker is the CPU
oracle loop (oracle/price_oracle.py: the C oracle's dense active set per EV, warm-started along the
sorted batch, a dense scipy NNLS price QP, the documented LP vertex rule).  w_ref = 0.8 w_max U[0,1]^N
takes the loop through 5-30 iterations per partition (measured with the oracle).

Tolerance: identical iteration counts; prices within 1e-6 theta (absolute); price before / after
regularisation within 1e-6 relative; get_w0_price0 (price_solver.py:272-285): w0 within 1e-6 and
the mean price0 within 1e-6 relative.
"""
import numpy as np
import pytest
import torch

import lompc_oracle as O
import price_oracle as PO
from lompc_amd import LoMPCConstants, settings
from lompc_amd.price_solver import PriceSolver
from lompc_amd.settings import MIN_INITIAL_SOC

pytestmark = pytest.mark.gpu

N = 48
NEV = 87381  # one partition of config 5's 1 048 576 EVs per type
PARTS = 3


def consts(ev):
    c = O.small_consts() if ev == "small" else O.large_consts()
    return c, LoMPCConstants(c.delta, c.theta, c.y_max, c.w_max, c.ev_type)


@pytest.mark.parametrize("ev", ["small", "large"])
def test_device_price_loop_matches_oracle_at_config5_partitions(gpu, monkeypatch, ev):
    monkeypatch.setattr(settings, "PRINT_LEVEL", 0)
    c, lc = consts(ev)
    rng = np.random.default_rng(500 + (ev == "large"))
    ps = PriceSolver(N, lc, "linear-convex", device=0)
    assert ps.device_loop and ps.native_loop  # the default: k_loop_iter, one launch per iteration
    po = PO.OraclePriceSolver(N, c, "linear-convex")
    po.warm = True
    edges = np.linspace(MIN_INITIAL_SOC, c.y_max, 13)
    levels = []
    for p in range(PARTS):  # staged ahead, as ChargingStation._stage_partitions does
        y0 = np.sort(edges[p] + (edges[p + 1] - edges[p]) * rng.random(NEV))[::-1].copy()
        yd = torch.as_tensor(y0, device="cuda:0")
        ps.stage_partition(p, yd, NEV, float(y0.max()), float(y0.min()), float(y0.sum()), descending=True)
        levels.append((y0, yd))
    iters = []
    for p, (y0, _) in enumerate(levels):
        w_ref = 0.8 * c.w_max * rng.random(N)
        ps.use_partition(p)
        po.set_charge_levels(y0)
        n0 = ps.n_batched_calls
        lm, st = ps.compute_optimal_prices(w_ref, 0.0)
        lmo, sto = po.compute_optimal_prices(w_ref, 0.0)
        assert st["iter"] == sto["iter"], (p, st["iter"], sto["iter"])
        assert ps.n_batched_calls - n0 == st["iter"] + 1
        np.testing.assert_allclose(lm, lmo, rtol=0, atol=1e-6 * c.theta, err_msg=f"partition {p}")
        for k in ("price_before_reg", "price_after_reg"):
            assert abs(st[k] - sto[k]) <= 1e-6 * max(1.0, abs(sto[k])), (p, k, st[k], sto[k])
        for k in ("dual_cost_decrease_actual", "dual_cost_decrease_predicted"):
            assert st[k].shape == sto[k].shape, k
            np.testing.assert_allclose(st[k], sto[k], rtol=1e-6, atol=1e-6 * np.max(np.abs(sto[k]), initial=1.0))
        np.testing.assert_array_equal(ps.prev_prices, lm[: ps.r])  # the chain into partition p + 1
        w0, p0 = ps.get_w0_price0(lm[: ps.r], 0.0)
        w0o, p0o = po.get_w0_price0_batch(lmo[: po.r], 0.0)
        np.testing.assert_allclose(w0, w0o, rtol=0, atol=1e-6)
        assert abs(p0 - p0o) <= 1e-6 * max(1.0, abs(p0o)), (p, p0, p0o)
        iters.append(st["iter"])
    assert sum(iters) >= 10, iters  # tens of iterations through k_loop_iter, not a trivial loop


@pytest.mark.parametrize("ev", ["small", "large"])
def test_price_chain_equals_partition_loops(gpu, monkeypatch, ev):
    """lompc_price_chain (one native call for a type's partitions, ChargingStation's default) gives the
    per-partition loops' results bit for bit: iteration counts, dual cost decreases, prices and the
    prices before / after regularisation (both regularise through lompc_price_regularize,
    price_solver.py:142-147), prev_prices chained the same way; a partition without EVs is skipped."""
    monkeypatch.setattr(settings, "PRINT_LEVEL", 0)
    c, lc = consts(ev)
    rng = np.random.default_rng(600 + (ev == "large"))
    edges = np.linspace(MIN_INITIAL_SOC, c.y_max, 13)
    sol = {}
    for mode in ("loops", "chain"):
        ps = PriceSolver(N, lc, "linear-convex", device=0)
        sol[mode] = ps
    parts = [0, 1, 3]  # (partition 2 has no EVs)
    w_refs = 0.8 * c.w_max * rng.random((4, N))
    for p in parts:
        y0 = np.sort(edges[p] + (edges[p + 1] - edges[p]) * rng.random(6000))[::-1].copy()
        yd = torch.as_tensor(y0, device="cuda:0")
        for ps in sol.values():
            ps.stage_partition(p, yd, len(y0), float(y0.max()), float(y0.min()), float(y0.sum()), descending=True)
    res_loops = []
    for p in parts:
        ps = sol["loops"]
        ps.use_partition(p)
        lm, st = ps.compute_optimal_prices(w_refs[p], 0.0)
        res_loops.append((lm.copy(), st))
    ps = sol["chain"]
    assert ps.chain_ok(parts)
    res_chain = ps.compute_optimal_prices_chain(parts, w_refs[parts], 0.0)
    assert sol["chain"].n_batched_calls == sol["loops"].n_batched_calls
    for (la, sa), (lb, sb) in zip(res_loops, res_chain):
        assert sa["iter"] == sb["iter"]
        np.testing.assert_array_equal(lb, la)  # (both regularise with lompc_price_regularize)
        for k in ("price_before_reg", "price_after_reg"):
            assert sa[k] == sb[k], k
        for k in ("dual_cost_decrease_actual", "dual_cost_decrease_predicted"):
            np.testing.assert_array_equal(sb[k], sa[k])
    np.testing.assert_array_equal(sol["chain"].prev_prices, sol["loops"].prev_prices)
