"""Diagnostic: A/B of a station option inside ONE process at config 5 (bench.py's station leg):
alternating blocks of steps with ChargingStation.<attr> True / False, per-step host phase marks
(last_step_ms; no extra synchronisation).  The price phase depends on the trajectory, so compare the
fixed phases (bimpc = interior point + what staging it leaves exposed, w0_price0, state).

    python scripts/station_ab.py [attr] [--blocks 4] [--steps 6]
"""
import argparse
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "incentive-design-mpc_amd"))
ap = argparse.ArgumentParser()
ap.add_argument("attr", nargs="?", default="gamma_layout")
ap.add_argument("--blocks", type=int, default=4)
ap.add_argument("--steps", type=int, default=6)
args = ap.parse_args()

import torch  # noqa: E402

from lompc_amd import settings  # noqa: E402
from lompc_amd.charging_station import ChargingStation  # noqa: E402
from lompc_amd.example import DEMAND_SCALE, NUM_EVS_PER_EV_TYPE, station_consts  # noqa: E402

settings.PRINT_LEVEL = 0
M_2, N, P = 1048576, 48, 12
consts = station_consts(8 * args.blocks * args.steps + 8, M_2, n_lo=N, n_bi=N, partitions=P,
                        price_type="linear-convex", demand_scale=DEMAND_SCALE * M_2 / NUM_EVS_PER_EV_TYPE,
                        u_b_max=0.5, x_max=0.5)
np.random.seed(0)
st = ChargingStation(consts, device=0)
for _ in range(3):
    st._step()
res = {True: [], False: []}
for blk in range(2 * args.blocks):
    val = blk % 2 == 0
    setattr(st, args.attr, val)
    for _ in range(args.steps):
        st._step()
        res[val].append(dict(st.last_step_ms))
    print(f"block {blk} ({args.attr}={val}) done", flush=True)
for val, rows in res.items():
    keys = rows[0].keys()
    print(f"{args.attr}={val}: " + "  ".join(f"{k} {np.median([r[k] for r in rows]):6.3f}" for k in keys) + " ms (median)")
