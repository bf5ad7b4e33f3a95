"""Diagnostic: the device price loop's time per iteration on the long-regime fixtures
(tests/golden/price_loop_long.npz: a capped 999-iteration loop of 15 731 large EVs and a 208-iteration
loop of 61 475 small EVs, N = 48), wall time of compute_optimal_prices_chain / iterations, best of R
repetitions.  Library: LOMPC_LIB (a variant build of scripts/build_variant.py) or the product.

    python scripts/loop_timing.py [reps]
"""
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "incentive-design-mpc_amd"), os.path.join(ROOT, "oracle")]
import lompc_oracle as O  # noqa: E402
from lompc_amd import LoMPCConstants, settings  # noqa: E402
from lompc_amd.price_solver import PriceSolver  # noqa: E402

settings.PRINT_LEVEL = 0
R = int(sys.argv[1]) if len(sys.argv) > 1 else 5
HERE = os.path.join(ROOT, "tests", "golden")
meta = json.load(open(os.path.join(HERE, "price_loop_long.json")))["cases"]
arr = np.load(os.path.join(HERE, "price_loop_long.npz"), allow_pickle=False)
for cls in ("capped", "mid"):
    m = meta[cls]
    g = lambda k: arr[f"{cls}_{k}"]
    c = O.large_consts() if m["kind"] == "Large" else O.small_consts()
    ps = PriceSolver(48, LoMPCConstants(c.delta, c.theta, c.y_max, c.w_max, c.ev_type), "linear-convex", device=0)
    if os.environ.get("LT_CELLS"):  # (the loop plans' path cells per set instead of the engine's choice)
        ps.loop_cells = int(os.environ["LT_CELLS"])
    y0 = g("y0")
    n, ymax, ymin, ysum = g("pstats")
    best = None
    for r in range(R + 1):
        ps._staged = {}
        ps._plan = None
        ps.stage_partition(0, torch.as_tensor(y0, device="cuda:0"), int(n), ymax, ymin, ysum, descending=True)
        ps.prev_prices = np.array(g("prev_prices"), copy=True)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        (lm, st), = ps.compute_optimal_prices_chain([0], np.stack([g("w_ref")]), m["lmbd_r"])
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
        if r > 0:
            best = dt if best is None else min(best, dt)
    it = st["iter"]
    print(f"{cls}: cells {ps._staged[0]['_plan'].info()['cells']}, {len(y0)} EVs, {it} iterations: best {best * 1e3:.2f} ms = {best / (it + 1) * 1e6:.2f} us per iteration",
          flush=True)
