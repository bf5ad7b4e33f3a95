"""The ``chargingstation`` drop-in package exports the reference's public names
(chargingstation/{lompc,settings,demand_data,price_regularizer,price_solver,bimpc,
charging_station}.py) so the reference's example imports resolve to the engine
(INTEGRATION.md §1).  CPU only: imports and constants, no solves."""
import importlib

import pytest

# public names per reference module (class / function / constant definitions)
REFERENCE_NAMES = {
    "lompc": ["LoMPC", "LoMPCConstants"],  # lompc.py:12,29
    "settings": ["PRINT_LEVEL", "MIN_MAX_BAT_SOC", "MAX_MAX_BAT_SOC", "MAX_BAT_CHARGE_RATE", "LOMPC_SOLVER",
                 "MAX_PRICE_SOLVER_ITERATIONS", "PRICE_SOLVER_TOL_TYPE", "PRICE_SOLVER_EPS_REG",
                 "PRICE_SOLVER_EPS_TOL", "PRICE_SOLVER_SOLVER", "BIMPC_SOLVER", "MIN_INITIAL_SOC",
                 "MAX_INITIAL_SOC", "MIN_FULL_CHARGE_FRACTION", "ADD_RESIDUAL_CHARGE_TO_BATTERY"],  # settings.py:4-33
    "demand_data": ["medium_term_demand_forecast"],  # demand_data.py:21
    "price_regularizer": ["PriceRegularizer"],  # price_regularizer.py:9
    "price_solver": ["PriceSolver"],  # price_solver.py:16
    "bimpc": ["BiMPC", "BiMPCChargingCostType", "BiMPCConstants", "BiMPCParameters"],  # bimpc.py:12-62
    "charging_station": ["ChargingStation", "ChargingStationConstants"],  # charging_station.py:16,42
}


@pytest.mark.parametrize("mod", sorted(REFERENCE_NAMES))
def test_dropin_exports(mod):
    m = importlib.import_module(f"chargingstation.{mod}")
    missing = [n for n in REFERENCE_NAMES[mod] if not hasattr(m, n)]
    assert not missing, (mod, missing)


def test_dropin_is_engine():
    import chargingstation.bimpc as cb
    import chargingstation.charging_station as cs
    import chargingstation.lompc as cl
    import chargingstation.price_solver as cp
    import lompc_amd

    assert cl.LoMPC is lompc_amd.LoMPC
    assert cp.PriceSolver.__module__ == "lompc_amd.price_solver"
    assert cb.BiMPC.__module__ == "lompc_amd.bimpc"
    assert cs.ChargingStation.__module__ == "lompc_amd.charging_station"


def test_settings_values():
    import chargingstation.settings as s

    # settings.py:7-9, 27-28: the values the station's constraints and initial draws use
    assert (s.MIN_MAX_BAT_SOC, s.MAX_MAX_BAT_SOC, s.MAX_BAT_CHARGE_RATE) == (0.75, 0.9, 0.25)
    assert (s.MIN_INITIAL_SOC, s.MAX_INITIAL_SOC) == (0.3, 0.5)
