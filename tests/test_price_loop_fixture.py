"""CPU checks of the long-regime price-loop fixture (tests/golden/price_loop_long.npz, made by
tests/golden/make_price_loop_cases.py): its expected outputs are the CPU oracle loop's
(oracle/price_oracle.py) on its inputs.  Re-deriving all 999 capped iterations takes over a minute,
so this re-runs the first iterations of both long loops and both followers in full, bit for bit."""
import json
import os

import numpy as np
import pytest

import lompc_oracle as O
import price_oracle as PO

HERE = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
N = 48


@pytest.fixture(scope="module")
def cases():
    with open(os.path.join(HERE, "price_loop_long.json")) as f:
        meta = json.load(f)["cases"]
    return meta, np.load(os.path.join(HERE, "price_loop_long.npz"), allow_pickle=False)


def loop(c, y0, w_ref, prev, lr):
    po = PO.OraclePriceSolver(N, c, "linear-convex")
    po.warm = "state"
    po.set_charge_levels(y0)
    po.prev_prices = np.array(prev, copy=True)
    return po.compute_optimal_prices(w_ref, lr)


@pytest.mark.parametrize("cls", ["capped", "mid"])
def test_fixture_is_the_oracle_loop(monkeypatch, cases, cls):
    meta, arr = cases
    m = meta[cls]
    g = lambda k: arr[f"{cls}_{k}"]
    c = O.large_consts() if m["kind"] == "Large" else O.small_consts()
    assert m["iter"] >= (999 if cls == "capped" else 150)
    # (a capped loop takes a step at every one of its 1000 passes, the last at iter = 999)
    n_dec = m["iter"] + (cls == "capped")
    assert len(g("dec_actual")) == n_dec and len(g("dec_pred")) == n_dec
    # the inputs: descending charge levels inside the type's [MIN_INITIAL_SOC, y_max]
    for y in (g("y0"), g("next_y0")):
        assert np.all(np.diff(y) <= 0) and y[-1] >= 0.3 - 1e-12 and y[0] <= c.y_max
    K = 6
    monkeypatch.setattr(PO, "MAX_ITERS", K)
    _, st = loop(c, g("y0"), g("w_ref"), g("prev_prices"), m["lmbd_r"])
    assert st["iter"] == K - 1
    np.testing.assert_array_equal(st["dual_cost_decrease_actual"], g("dec_actual")[:K])
    np.testing.assert_array_equal(st["dual_cost_decrease_predicted"], g("dec_pred")[:K])
    monkeypatch.setattr(PO, "MAX_ITERS", 1000)
    # the follower from the long loop's final prices: the whole loop
    lm2, st2 = loop(c, g("next_y0"), g("next_w_ref"), g("prices")[:3 * N], m["lmbd_r"])
    assert st2["iter"] == m["next_iter"]
    np.testing.assert_array_equal(lm2, g("next_prices"))
    assert st2["price_after_reg"] == m["next_price_after_reg"]
