"""Oracle parity of the station's device price loop in the LONG regime (hundreds of iterations, and the
reference's cap of MAX_PRICE_SOLVER_ITERATIONS = 1000), on loops taken from bench.py's own config-5
trajectory (tests/golden/make_price_loop_cases.py: inputs dumped by scripts/dump_price_cases.py from
the station at seed 0, expected outputs from the CPU oracle loop, oracle/price_oracle.py).

* capped: large EVs, partition 5 of step 19 — 15 731 EVs, the loop runs to the cap (999): w_hat is out
  of the partition's reach, and the loop drives one convex-price component to ~3.9e5 theta;
* mid:    small EVs, partition 4 of step 7 — 61 475 EVs, 208 iterations.

Each is followed by the next partition of its type's chain (4 096 of its EVs), whose loop starts from
the long loop's final prices (prev_prices, price_solver.py:104, :166; charging_station.py:275-307).
Both partitions run through ``PriceSolver.compute_optimal_prices_chain`` — the station's default path:
the device loop (one ``k_loop_iter`` launch per price iteration) then ``lompc_price_regularize``,
the next partition from those prices, in one native call.

Tolerance (what is asserted):
* iteration counts identical (both partitions);
* prices per component within 1e-6 * max(theta, |lambda_i|) — the north star's 1e-6 relative; the
  mid loop also within 1e-6 theta absolute.  (In the capped loop the prices reach 3.9e5 theta: one
  fp64 ulp of such a price is 6e-11 theta, and 1000 dependent price steps, each an exact QP solve
  whose rounding order differs between a wave-parallel PDAS and Lawson-Hanson NNLS, amplify it to
  1.5e-2 theta = 1.0e-7 relative — measured — so an absolute 1e-6 theta bound cannot hold there);
* prices before / after regularisation within 1e-6 relative;
* every dual cost decrease (actual and predicted, all 999) within 1e-6 relative (atol 1e-6 of the
  largest);
* the chain: prev_prices after the long loop equal its returned prices bit for bit, and the follower
  (started from them) matches the oracle's follower (started from the oracle's);
* get_w0_price0 (price_solver.py:272-285) at the oracle's final prices of the capped loop: w0 of
  every EV within 1e-6, the mean price0 within 1e-6 relative.
"""
import json
import os

import numpy as np
import pytest
import torch

import lompc_oracle as O
from lompc_amd import LoMPCConstants, settings
from lompc_amd.price_solver import PriceSolver

pytestmark = pytest.mark.gpu

HERE = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
N = 48


@pytest.fixture(scope="module")
def cases():
    with open(os.path.join(HERE, "price_loop_long.json")) as f:
        meta = json.load(f)["cases"]
    arr = np.load(os.path.join(HERE, "price_loop_long.npz"), allow_pickle=False)
    return meta, arr


def stats(y):
    return len(y), float(y.max()), float(y.min()), float(y.sum())


@pytest.mark.parametrize("cls", ["capped", "mid"])
def test_long_price_loop_matches_oracle(gpu, monkeypatch, cases, cls):
    monkeypatch.setattr(settings, "PRINT_LEVEL", 0)
    meta, arr = cases
    m = meta[cls]
    g = lambda k: arr[f"{cls}_{k}"]
    c = O.large_consts() if m["kind"] == "Large" else O.small_consts()
    lc = LoMPCConstants(c.delta, c.theta, c.y_max, c.w_max, c.ev_type)
    ps = PriceSolver(N, lc, "linear-convex", device=0)
    assert ps.device_loop and ps.native_loop
    y0, ny = g("y0"), g("next_y0")
    assert np.all(np.diff(y0) <= 0) and np.all(np.diff(ny) <= 0)  # (descending, as the station lays them out)
    n, ymax, ymin, ysum = g("pstats")
    assert int(n) == len(y0) and ymax == y0.max() and ymin == y0.min()
    ps.stage_partition(0, torch.as_tensor(y0, device="cuda:0"), int(n), ymax, ymin, ysum, descending=True)
    ps.stage_partition(1, torch.as_tensor(ny, device="cuda:0"), *stats(ny), descending=True)
    ps.prev_prices = np.array(g("prev_prices"), copy=True)
    lr = m["lmbd_r"]
    assert ps.chain_ok([0, 1])
    (lm, st), (lm2, st2) = ps.compute_optimal_prices_chain([0, 1], np.stack([g("w_ref"), g("next_w_ref")]), lr)
    # iteration counts (999 = the cap for the capped loop, as on the bench's trajectory)
    assert st["iter"] == m["iter"], (st["iter"], m["iter"])
    assert st["iter"] == m["iter_gpu_trajectory"]
    assert st2["iter"] == m["next_iter"], (st2["iter"], m["next_iter"])
    th = c.theta
    for got, want, what in ((lm, g("prices"), "prices"), (lm2, g("next_prices"), "next partition's prices")):
        err = np.abs(got - want) / np.maximum(th, np.abs(want))
        assert err.max() <= 1e-6, (what, float(err.max()), int(np.argmax(err)))
    if cls == "mid":
        np.testing.assert_allclose(lm, g("prices"), rtol=0, atol=1e-6 * th)
    for s, pre in ((st, ""), (st2, "next_")):
        for k in ("price_before_reg", "price_after_reg"):
            want = m[pre + k]
            assert abs(s[k] - want) <= 1e-6 * max(1.0, abs(want)), (pre + k, s[k], want)
    for s, pre in ((st, ""), (st2, "next_")):
        for k, gk in (("dual_cost_decrease_actual", "dec_actual"), ("dual_cost_decrease_predicted", "dec_pred")):
            want = g(pre + gk)
            assert s[k].shape == want.shape, (pre + k, s[k].shape, want.shape)
            if want.size:
                np.testing.assert_allclose(s[k], want, rtol=1e-6, atol=1e-6 * np.max(np.abs(want)), err_msg=pre + k)
    # the chain: the follower started from the long loop's prices; the solver ends on the follower's
    np.testing.assert_array_equal(ps.prev_prices, lm2[: ps.r])
    if cls == "capped":
        ps.use_partition(0)
        w0, p0 = ps.get_w0_price0(g("prices")[: ps.r], lr)
        np.testing.assert_allclose(w0, g("w0"), rtol=0, atol=1e-6)
        assert abs(p0 - m["price0_mean"]) <= 1e-6 * max(1.0, abs(m["price0_mean"])), (p0, m["price0_mean"])
