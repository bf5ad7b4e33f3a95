"""Config 1 (BASELINE.json): the paper experiment of
chargingstation/example/real_time_price_control.py on the engine, without CVXPY.

The reference's driver builds its constants (real_time_price_control.py:11-78), runs
``ChargingStation(consts).simulate()`` and pickles the logs (:81-93).  Here the same
experiment runs on the CVXPY-free stack: the batched LoMPC engine for every per-EV solve,
the host price / regularizer / BiMPC solvers of the C-ABI library for the rest.

    python -m lompc_amd.example [--hours 49] [--evs 500] [--price-type linear-convex]
                                [--seed 0] [--out logs.npz]

The reference seeds nothing (charging_station.py:95-100 uses the legacy global
``np.random`` stream); ``--seed`` seeds that stream so a run is repeatable.  Logs are
written with ``numpy.savez`` (no pickle).
"""
from __future__ import annotations

import argparse
import time

import numpy as np

from . import settings
from .bimpc import BiMPCChargingCostType, BiMPCConstants
from .charging_station import ChargingStation, ChargingStationConstants
from .demand_data import medium_term_demand_forecast
from .lompc import LoMPCConstants

# real_time_price_control.py:11-23
SIMULATION_LENGTH = 49
HORIZON_LOMPC = 12
HORIZON_BIMPC = 16
NUM_EVS_PER_EV_TYPE = 500
NUM_PARTITIONS = 12
PRICE_TYPE = "linear-convex"
DEMAND_SCALE = 1 / 4


def lompc_consts() -> tuple[LoMPCConstants, LoMPCConstants]:
    """real_time_price_control.py:26-39."""
    return (LoMPCConstants(0.05, 10, 0.9, 0.25, "small"), LoMPCConstants(0.025, 50, 0.9, 0.15, "large"))


def bimpc_consts(cost_type: BiMPCChargingCostType = BiMPCChargingCostType.EXP_UNWEIGHTED, u_b_max: float = 0.3,
                 x_max: float = 0.3) -> BiMPCConstants:
    """real_time_price_control.py:42-52 (normalized)."""
    return BiMPCConstants(1e3, 1, 1, u_b_max, x_max, cost_type, 5)


def station_consts(hours: int = SIMULATION_LENGTH, evs: int = NUM_EVS_PER_EV_TYPE, n_lo: int = HORIZON_LOMPC,
                   n_bi: int = HORIZON_BIMPC, partitions: int = NUM_PARTITIONS, price_type: str = PRICE_TYPE,
                   demand_scale: float = DEMAND_SCALE,
                   cost_type: BiMPCChargingCostType = BiMPCChargingCostType.EXP_UNWEIGHTED,
                   u_b_max: float = 0.3, x_max: float = 0.3) -> ChargingStationConstants:
    """real_time_price_control.py:55-78.  ``demand_scale`` multiplies the forecast; for EV
    populations other than 500 per type pass DEMAND_SCALE * evs / 500 so the normalized demand
    (charging_station.py:92, :214) stays that of the example.

    Storage feasibility: the BiMPC keeps d_e = sum_p theta Mp beta_p / B away from the storage
    bounds (bimpc.py:195-218) with beta_p = sqrt(N_lo) Gamma_p + eps_tol (price_solver.py:182-186).
    From an empty battery (x0 = 0) the first step needs d_e <= u_b_max - d_e, i.e.
    u_b_max >= 2 d_e: with the example's u_b_max = 0.3 and partitions of SoC width 0.05 this
    holds up to N_lo ~ 20 (beta = 0.097 at N_lo = 12, 0.183 at N_lo = 48)."""
    cs, cl = lompc_consts()
    demand = medium_term_demand_forecast(hours + n_bi + 1, demand_scale, interpolate=False)
    return ChargingStationConstants(hours, n_bi, n_lo, evs, partitions, demand,
                                    bimpc_consts(cost_type, u_b_max, x_max), cs, cl, price_type)


def flatten_logs(logs: dict) -> dict:
    """The logs dict (charging_station.py:118-149) as flat arrays for numpy.savez."""
    out = {}
    for sec in ("inputs", "states", "bounds", "statistics", "prices"):
        for k, v in logs[sec].items():
            out[f"{sec}/{k}"] = np.asarray(v)
    return out


def main(argv=None) -> dict:
    ap = argparse.ArgumentParser(description=__doc__.splitlines()[0])
    ap.add_argument("--hours", type=int, default=SIMULATION_LENGTH)
    ap.add_argument("--evs", type=int, default=NUM_EVS_PER_EV_TYPE)
    ap.add_argument("--price-type", default=PRICE_TYPE, choices=["linear", "linear-convex"])
    ap.add_argument("--seed", type=int, default=0)
    ap.add_argument("--print-level", type=int, default=0)
    ap.add_argument("--out", default=None)
    args = ap.parse_args(argv)
    settings.PRINT_LEVEL = args.print_level
    consts = station_consts(args.hours, args.evs, price_type=args.price_type,
                            demand_scale=DEMAND_SCALE * args.evs / NUM_EVS_PER_EV_TYPE)
    np.random.seed(args.seed)
    t0 = time.perf_counter()
    cs = ChargingStation(consts)
    logs = cs.simulate()
    dt = time.perf_counter() - t0
    it = np.concatenate([logs["statistics"]["niter_s"].ravel(), logs["statistics"]["niter_l"].ravel()])
    print(f"{args.hours} steps in {dt:.2f} s ({args.hours / dt:.2f} steps/s); price iterations per "
          f"(type, partition, step): mean {np.mean(it[it >= 0]):.1f}; EVs charged: "
          f"{cs.ncharged_s} small, {cs.ncharged_l} large")
    if args.out:
        np.savez(args.out, **flatten_logs(logs))
    return logs


if __name__ == "__main__":
    main()
