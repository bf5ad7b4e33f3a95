"""Dump price-loop problems from the bench's config-5 station trajectory (diagnostic / fixture maker).

Runs the station exactly as bench.py's station leg does (seed 0, config 5: 2 097 152 EVs, N = 48,
12 partitions per type, u_b_max = x_max = 0.5) and records, for every (step, type, partition) price
loop, the loop's inputs — the partition's charge levels (descending), w_hat (the BiMPC's w_ref),
prev_prices (the chain's start), lmbd_r — and its outcome (iterations, prices).  Levels are kept
only for loops in the long regime (``--min-iter``), the first ``--keep`` of each class (capped at the
reference's MAX_PRICE_SOLVER_ITERATIONS, or 150-500 iterations).

    python scripts/dump_price_cases.py --steps 23 --out gpurun_out/price_cases
"""
import argparse
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "incentive-design-mpc_amd")]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=23)
    ap.add_argument("--evs", type=int, default=2097152)
    ap.add_argument("--seed", type=int, default=0)
    ap.add_argument("--keep", type=int, default=3)
    ap.add_argument("--out", default=os.path.join(ROOT, "gpurun_out", "price_cases"))
    args = ap.parse_args()
    import torch

    from lompc_amd import settings
    from lompc_amd.charging_station import ChargingStation
    from lompc_amd.example import DEMAND_SCALE, NUM_EVS_PER_EV_TYPE, station_consts

    settings.PRINT_LEVEL = 0
    N, P = 48, 12
    M_2 = args.evs // 2
    consts = station_consts(args.steps + 4, M_2, n_lo=N, n_bi=N, partitions=P, price_type="linear-convex",
                            demand_scale=DEMAND_SCALE * M_2 / NUM_EVS_PER_EV_TYPE, u_b_max=0.5, x_max=0.5)
    np.random.seed(args.seed)
    st = ChargingStation(consts, device=0)
    os.makedirs(args.out, exist_ok=True)
    meta = []
    kept = {"capped": 0, "mid": 0}

    def hook(kind, solver):
        orig = solver.compute_optimal_prices_chain

        def chain(parts, w_refs, lmbd_r):
            prev0 = np.array(solver.prev_prices, copy=True)
            res = orig(parts, w_refs, lmbd_r)
            torch.cuda.synchronize()
            _, ys, seg = st._layout[kind]
            prev = prev0
            follow = None  # a kept loop's successor in the chain (its prev_prices = the kept loop's prices)
            for k, p in enumerate(parts):
                lm, stats = res[k]
                it = int(stats["iter"])
                cls = "capped" if it >= settings.MAX_PRICE_SOLVER_ITERATIONS - 1 else ("mid" if 150 <= it <= 500 else None)
                rec = {"t": st.t, "kind": kind, "p": p, "iter": it, "n": seg[p][1] - seg[p][0]}
                save = None
                if follow is not None:
                    save, follow = follow + "_next.npz", None
                elif cls and kept[cls] < args.keep:
                    kept[cls] += 1
                    follow = f"{cls}_{kind}_t{st.t}_p{p}"
                    save = follow + ".npz"
                if save:
                    a, b = seg[p]
                    name = save
                    np.savez(os.path.join(args.out, name), y0=ys[a:b].cpu().numpy(), w_ref=np.asarray(w_refs[k]),
                             prev_prices=prev, lmbd_r=float(lmbd_r), iter=it, prices=lm, kind=kind,
                             pstats=np.asarray(st._pstats[0 if kind == "Small" else 1][p]),
                             price_before_reg=stats["price_before_reg"], price_after_reg=stats["price_after_reg"],
                             dec_actual=stats["dual_cost_decrease_actual"],
                             dec_pred=stats["dual_cost_decrease_predicted"])
                    rec["file"] = name
                meta.append(rec)
                prev = np.array(lm[: solver.r], copy=True)
            return res

        solver.compute_optimal_prices_chain = chain

    hook("Small", st.price_solver_s)
    hook("Large", st.price_solver_l)
    for k in range(args.steps):
        st._step()
        print(f"step {k}: " + " ".join(f"{m['kind'][0]}{m['p']}:{m['iter']}" for m in meta if m["t"] == k), flush=True)
    import json

    with open(os.path.join(args.out, "meta.json"), "w") as f:
        json.dump(meta, f)
    print("kept", kept)


if __name__ == "__main__":
    main()
