"""Generate the committed golden vectors for the LoMPC hot path.

    python tests/golden/make_golden.py      (writes tests/golden/lompc_golden.npz + .json)

Every vector comes from the CPU oracle (oracle/lompc_oracle.py, a dense
restatement of chargingstation/lompc.py:59-156) and is CERTIFIED in 50-digit
arithmetic: the oracle's working set is re-solved in mpmath and its KKT
residual must be <= 1e-30 (relative).  The stored w is that 50-digit optimum
rounded to fp64.  The reference itself cannot run here (cvxpy/clarabel absent,
SURVEY.md section 8(c)) and ships no golden data, so this is the pinning
evidence for parity.  Inputs follow the reference's own test generators:
lambda ~ theta U[0,1]^{3N}, lmbd_r ~ 3N delta U[0,1] (test_lompc.py:34-36),
gamma ~ y_max U[0,1], plus the edge cases gamma in {0, y_max}, lambda = 0
(test_lompc.py:48) and the "linear" price type (lambda_3 = 0,
price_solver.py:103-104).
"""
from __future__ import annotations

import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(ROOT, "oracle"))

import lompc_oracle as O  # noqa: E402

SEED = 20251017
NEV = 16


def cases():
    rng = np.random.default_rng(SEED)
    out = []
    for ev in ("small", "large"):
        for N in (12, 24, 48):
            for price in ("linear-convex", "linear", "zero"):
                for lr_kind in ("zero", "random"):
                    c = O.small_consts() if ev == "small" else O.large_consts()
                    lmbd = c.theta * rng.random(3 * N)
                    if price == "linear":
                        lmbd[2 * N:] = 0.0
                    if price == "zero":
                        lmbd[:] = 0.0
                    lmbd_r = 0.0 if lr_kind == "zero" else (3 * N) * c.delta * rng.random()
                    gamma = c.y_max * rng.random(NEV)
                    gamma[0] = 0.0
                    gamma[1] = c.y_max
                    w_ref = c.w_max * rng.random(N)  # test_price_solver.py:148
                    out.append(dict(ev=ev, N=N, price=price, lr_kind=lr_kind, consts=c, lmbd=lmbd,
                                    lmbd_r=lmbd_r, gamma=gamma, w_ref=w_ref))
    return out


def main():
    arrays = {}
    meta = []
    worst_kkt = 0.0
    worst_dw = 0.0
    for k, cs in enumerate(cases()):
        c = cs["consts"]
        o = O.OracleLoMPC(cs["N"], c)
        W = np.zeros((NEV, cs["N"]))
        C = np.zeros(NEV)
        ST = np.zeros((NEV, cs["N"]), dtype=np.int8)
        for i, g in enumerate(cs["gamma"]):
            w64, st = o.solve_state(cs["lmbd"], cs["lmbd_r"], g)
            wmp, res, slack = O.refine_mp(o, st, cs["lmbd"], cs["lmbd_r"], g)
            assert res <= 1e-30, (k, i, res)
            worst_kkt = max(worst_kkt, res)
            worst_dw = max(worst_dw, float(np.max(np.abs(wmp - w64))))
            W[i] = wmp
            C[i] = o.objective(wmp, cs["lmbd"], cs["lmbd_r"], g)
            ST[i] = st
        y0 = c.y_max - cs["gamma"]
        A_bar, _ = O.w_inner_product_metric(o.A, c.delta, cs["lmbd_r"])
        err_max, w0_err, avg_err = O.get_w_err(o, y0, cs["lmbd"], cs["lmbd_r"], cs["w_ref"], A_bar)
        r = 2 * cs["N"] if cs["price"] == "linear" else 3 * cs["N"]
        w0, price0 = O.get_w0_price0(o, y0, cs["lmbd"][:r], r, cs["lmbd_r"])
        p = f"c{k}_"
        arrays[p + "lmbd"] = cs["lmbd"]
        arrays[p + "gamma"] = cs["gamma"]
        arrays[p + "w_ref"] = cs["w_ref"]
        arrays[p + "w"] = W
        arrays[p + "cost"] = C
        arrays[p + "state"] = ST
        arrays[p + "w0"] = w0
        meta.append(dict(id=k, ev_type=cs["ev"], N=cs["N"], price=cs["price"], lmbd_r=cs["lmbd_r"],
                         delta=c.delta, theta=c.theta, y_max=c.y_max, w_max=c.w_max, r=r,
                         w_err_max=float(err_max), w0_err=float(w0_err), w_avg_err=float(avg_err),
                         price0=float(price0)))
        print(f"case {k:2d} {cs['ev']:5s} N={cs['N']:2d} {cs['price']:13s} lr={cs['lr_kind']:6s} ok", flush=True)
    np.savez_compressed(os.path.join(HERE, "lompc_golden.npz"), **arrays)
    with open(os.path.join(HERE, "lompc_golden.json"), "w") as f:
        json.dump(dict(seed=SEED, nev=NEV, generator="tests/golden/make_golden.py",
                       certificate="50-digit KKT residual <= 1e-30 (oracle.refine_mp)",
                       worst_kkt_rel=worst_kkt, worst_fp64_vs_mp=worst_dw, cases=meta), f, indent=1)
    print("worst KKT (50 digits):", worst_kkt, " worst |w64 - w_mp|:", worst_dw)


if __name__ == "__main__":
    main()
