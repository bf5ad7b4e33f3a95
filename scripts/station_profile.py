"""Diagnostic: where the time of one closed-loop ChargingStation step goes (bench.py's
BiMPC steps/sec leg, config-5 shape).  Prints per-phase wall times and a cProfile
summary of the timed steps."""
import cProfile
import os
import pstats
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "incentive-design-mpc_amd"))
from lompc_amd import settings  # noqa: E402
from lompc_amd.charging_station import ChargingStation  # noqa: E402
from lompc_amd.example import DEMAND_SCALE, NUM_EVS_PER_EV_TYPE, station_consts  # noqa: E402

N = int(os.environ.get("N", "48"))
M_2 = int(os.environ.get("M2", "131072"))
settings.PRINT_LEVEL = 0
torch.cuda.set_device(0)
consts = station_consts(4, M_2, n_lo=N, n_bi=N, demand_scale=DEMAND_SCALE * M_2 / NUM_EVS_PER_EV_TYPE,
                        u_b_max=0.5, x_max=0.5)
np.random.seed(0)
st = ChargingStation(consts, device=0)
phases = {}
for name in ("_get_bimpc_solution", "_get_optimal_prices", "_get_w0_price0", "_update_state", "_update_logs"):
    f = getattr(st, name)

    def wrap(*a, _f=f, _n=name, **k):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        r = _f(*a, **k)
        torch.cuda.synchronize()
        phases[_n] = phases.get(_n, 0.0) + time.perf_counter() - t0
        return r

    setattr(st, name, wrap)
for obj, name, label in ((st.bimpc, "solve_bimpc", "  bimpc.solve_bimpc"),
                         (st.price_solver_s, "_iterate", "  price._iterate (s)"),
                         (st.price_solver_l, "_iterate", "  price._iterate (l)"),
                         (st.price_solver_s, "_price_gradient_descent_step", "  price step (s)"),
                         (st.price_solver_l, "_price_gradient_descent_step", "  price step (l)"),
                         (st.price_solver_s, "set_charge_levels", "  set_charge_levels (s)"),
                         (st.price_solver_l, "set_charge_levels", "  set_charge_levels (l)")):
    f = getattr(obj, name)

    def wrap2(*a, _f=f, _n=label, **k):
        t0 = time.perf_counter()
        r = _f(*a, **k)
        phases[_n] = phases.get(_n, 0.0) + time.perf_counter() - t0
        return r

    setattr(obj, name, wrap2)
orig_step = st.price_solver_s._price_gradient_descent_step
st._step()
phases.clear()
pr = cProfile.Profile()
t0 = time.perf_counter()
pr.enable()
for _ in range(2):
    st._step()
pr.disable()
dt = (time.perf_counter() - t0) / 2
print(f"step {dt * 1e3:.1f} ms")
for k, v in phases.items():
    print(f"  {k:22s} {v / 2 * 1e3:8.2f} ms")
it = st.logs["statistics"]
print("bimpc last info:", st.bimpc.last_info)
print("price iterations per (type, partition):", it["niter_s"][:, 1:3].tolist(), it["niter_l"][:, 1:3].tolist())
pstats.Stats(pr).sort_stats("tottime").print_stats(25)
