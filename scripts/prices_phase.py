"""Diagnostic: where the station's price phase goes beyond its slower chain, at config 5 (bench.py's
station leg): per step the phase's wall time, each type's native chain call (start / end relative to
the phase's start, on its thread), and the rest.

    python scripts/prices_phase.py [--steps 12]
"""
import argparse
import os
import sys
import threading
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "incentive-design-mpc_amd"))
ap = argparse.ArgumentParser()
ap.add_argument("--steps", type=int, default=12)
args = ap.parse_args()

import torch  # noqa: E402

from lompc_amd import settings  # noqa: E402
from lompc_amd.charging_station import ChargingStation  # noqa: E402
from lompc_amd.example import DEMAND_SCALE, NUM_EVS_PER_EV_TYPE, station_consts  # noqa: E402

settings.PRINT_LEVEL = 0
M_2, N, P = 1048576, 48, 12
consts = station_consts(args.steps + 8, M_2, n_lo=N, n_bi=N, partitions=P, price_type="linear-convex",
                        demand_scale=DEMAND_SCALE * M_2 / NUM_EVS_PER_EV_TYPE, u_b_max=0.5, x_max=0.5)
np.random.seed(0)
st = ChargingStation(consts, device=0)
ev = []
t_phase = [0.0]


def wrap(solver, kind):
    f = solver.compute_optimal_prices_chain

    def w(*a, **k):
        t0 = time.perf_counter()
        r = f(*a, **k)
        t1 = time.perf_counter()
        ev.append((kind, threading.current_thread().name, (t0 - t_phase[0]) * 1e3, (t1 - t_phase[0]) * 1e3))
        return r
    solver.compute_optimal_prices_chain = w


wrap(st.price_solver_s, "Small")
wrap(st.price_solver_l, "Large")
g = st._get_optimal_prices
rows = []


def gp(*a, **k):
    t_phase[0] = time.perf_counter()
    ev.clear()
    r = g(*a, **k)
    rows.append(((time.perf_counter() - t_phase[0]) * 1e3, list(ev)))
    return r


st._get_optimal_prices = gp
for _ in range(3):
    st._step()
rows.clear()
for _ in range(args.steps):
    st._step()
for tot, e in rows:
    print(f"phase {tot:7.3f} ms: " + "  ".join(f"{k}@{th[:10]} {a:6.3f}..{b:6.3f}" for k, th, a, b in e))
