"""Diagnostic: run the closed loop (tests/test_gpu_station.py config) and dump the logs."""
import os, sys, json
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "incentive-design-mpc_amd"), os.path.join(ROOT, "tests")]
from lompc_amd import settings
settings.PRINT_LEVEL = int(os.environ.get("PL", "0"))
from lompc_amd.bimpc import BiMPCChargingCostType, BiMPCConstants
from lompc_amd.charging_station import ChargingStationConstants
from lompc_amd.demand_data import medium_term_demand_forecast
from lompc_amd.lompc import LoMPCConstants


def consts(M_2, Tf=3, N_LO=12, N_BI=16, P=12):  # tests/test_gpu_station.py
    cs = LoMPCConstants(0.05, 10, 0.9, 0.25, "small")
    cl = LoMPCConstants(0.025, 50, 0.9, 0.15, "large")
    bi = BiMPCConstants(1e3, 1, 1, 0.3, 0.3, BiMPCChargingCostType.UNWEIGHTED, 5)
    demand = medium_term_demand_forecast(Tf + N_BI + 1, 1 / 4 * M_2 / 500, interpolate=False)
    return ChargingStationConstants(Tf, N_BI, N_LO, M_2, P, demand, bi, cs, cl, "linear-convex")
from lompc_amd.charging_station import ChargingStation
np.random.seed(1)
cs = ChargingStation(consts(60), device=0)
logs = cs.simulate()
flat = {}
for sec in ("inputs", "bounds", "prices", "statistics", "states"):
    for k, v in logs[sec].items():
        flat[k] = np.asarray(v)
np.savez(os.path.join(ROOT, "gpurun_out", "station_logs.npz"), **flat)
print("done")
