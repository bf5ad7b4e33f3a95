"""Constants of the hot path, mirrored from chargingstation/settings.py.

The reference module imports ``cvxpy`` at line 1 (``from cvxpy import
CLARABEL``); this mirror carries only the numbers the LoMPC path uses, with the
same names, so host code reads like the reference.
"""

PRINT_LEVEL = 1  # settings.py:4

# LoMPC settings (settings.py:7-9)
MIN_MAX_BAT_SOC = 0.75
MAX_MAX_BAT_SOC = 0.9
MAX_BAT_CHARGE_RATE = 0.25

# LOMPC_SOLVER = CLARABEL (settings.py:11) -> the HIP engine; the mode below is
# the engine's own algorithm choice (LOMPC_MODE_PATH / LOMPC_MODE_DIRECT).
LOMPC_SOLVER = "lompc_amd"
LOMPC_MODE = "path"

# PriceSolver settings (settings.py:14-19)
MAX_PRICE_SOLVER_ITERATIONS = 1000
PRICE_SOLVER_TOL_TYPE = "avg"
PRICE_SOLVER_EPS_REG = 0.01
PRICE_SOLVER_EPS_TOL = 0.01

# ChargingStation settings (settings.py:27-33)
MIN_INITIAL_SOC = 0.3
MAX_INITIAL_SOC = 0.5
MIN_FULL_CHARGE_FRACTION = 0.95
ADD_RESIDUAL_CHARGE_TO_BATTERY = False
