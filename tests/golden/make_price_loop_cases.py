"""Golden price-loop cases in the LONG regime, from the bench's own config-5 station trajectory.

    python scripts/dump_price_cases.py            (on the GPU box: writes gpurun_out/price_cases/)
    python tests/golden/make_price_loop_cases.py  (here: writes tests/golden/price_loop_long.npz)

Inputs: two (EV type, partition) price loops that bench.py's config-5 station (seed 0, 2 097 152
EVs, N = 48, 12 partitions per type, linear-convex prices) runs at length — one that reaches the
reference's cap MAX_PRICE_SOLVER_ITERATIONS = 1000 (settings.py:14, price_solver.py:111-140), one of
150-500 iterations — each with the partition that follows it in the type's chain (its prev_prices
are the loop's final prices, price_solver.py:166, charging_station.py:275-307).  Stored per case:
the partition's charge levels (descending, as the station lays them out), w_hat, prev_prices,
lmbd_r; the follower's levels subsampled to NEXT_EVS evenly spaced EVs (its first and last kept,
so its robustness tolerance is unchanged).

Expected outputs: the CPU ORACLE loop (oracle/price_oracle.py: the C oracle's dense active set per
EV, scipy NNLS for the price QP, the documented LP vertex rule) run on those inputs here — iteration
counts, prices, the prices before / after regularisation, the dual cost decreases, the follower's
loop, and get_w0_price0 (price_solver.py:272-285) at the capped loop's final prices.  These are
checker outputs (no reference code ran: cvxpy is absent); the trajectory inputs
come from the GPU run, the expected outputs only from the oracle.
"""
from __future__ import annotations

import json
import os
import sys
import time

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(ROOT, "oracle"))

import lompc_oracle as O  # noqa: E402
import price_oracle as PO  # noqa: E402

SRC = os.path.join(ROOT, "gpurun_out", "price_cases")
CASES = {"capped": "capped_Large_t19_p5", "mid": "mid_Small_t7_p4"}
NEXT_EVS = 4096
N = 48


def oracle_loop(c, y0, w_ref, prev, lmbd_r):
    po = PO.OraclePriceSolver(N, c, "linear-convex")
    po.warm = "state"
    po.set_charge_levels(y0)
    po.prev_prices = np.array(prev, copy=True)
    lm, st = po.compute_optimal_prices(w_ref, lmbd_r)
    return po, lm, st


def main():
    out, meta = {}, {}
    for cls, name in CASES.items():
        d = np.load(os.path.join(SRC, name + ".npz"))
        nx = np.load(os.path.join(SRC, name + "_next.npz"))
        kind = str(d["kind"])
        c = O.large_consts() if kind == "Large" else O.small_consts()
        lr = float(d["lmbd_r"])
        ny = nx["y0"]
        sel = np.unique(np.round(np.linspace(0, len(ny) - 1, NEXT_EVS)).astype(np.int64))
        ny = np.ascontiguousarray(ny[sel])
        t0 = time.perf_counter()
        po, lm, st = oracle_loop(c, d["y0"], d["w_ref"], d["prev_prices"], lr)
        po2, lm2, st2 = oracle_loop(c, ny, nx["w_ref"], lm[: po.r], lr)
        w0, p0 = po.get_w0_price0_batch(lm[: po.r], lr)
        dt = time.perf_counter() - t0
        p = f"{cls}_"
        out.update({p + "y0": d["y0"], p + "w_ref": d["w_ref"], p + "prev_prices": d["prev_prices"],
                    p + "pstats": d["pstats"], p + "next_y0": ny, p + "next_w_ref": nx["w_ref"],
                    p + "prices": lm, p + "dec_actual": st["dual_cost_decrease_actual"],
                    p + "dec_pred": st["dual_cost_decrease_predicted"], p + "next_prices": lm2,
                    p + "next_dec_actual": st2["dual_cost_decrease_actual"],
                    p + "next_dec_pred": st2["dual_cost_decrease_predicted"], p + "w0": w0})
        meta[cls] = {"source": name, "kind": kind, "lmbd_r": lr, "n_evs": int(len(d["y0"])),
                     "next_n_evs": int(len(ny)), "next_n_evs_station": int(len(nx["y0"])),
                     "iter": int(st["iter"]), "iter_gpu_trajectory": int(d["iter"]),
                     "price_before_reg": float(st["price_before_reg"]), "price_after_reg": float(st["price_after_reg"]),
                     "next_iter": int(st2["iter"]), "next_price_before_reg": float(st2["price_before_reg"]),
                     "next_price_after_reg": float(st2["price_after_reg"]), "price0_mean": float(p0),
                     "max_price_over_theta": float(np.abs(lm).max() / c.theta), "oracle_seconds": round(dt, 1)}
        print(cls, meta[cls], flush=True)
    np.savez(os.path.join(HERE, "price_loop_long.npz"), **out)
    with open(os.path.join(HERE, "price_loop_long.json"), "w") as f:
        json.dump({"doc": __doc__.split("\n\n")[2].replace("\n", " "), "cases": meta}, f, indent=1)


if __name__ == "__main__":
    main()
