"""Drop-in module for ``chargingstation/settings.py`` (settings.py:1-33): the same names,
read from ``lompc_amd.settings``.  The solver names the reference hands to CVXPY
(``LOMPC_SOLVER``, ``PRICE_SOLVER_SOLVER``, ``BIMPC_SOLVER``) name the engine's own solvers
here.  Mutating a value must go through ``lompc_amd.settings`` (the modules read it there)."""
from lompc_amd.settings import *  # noqa: F401,F403
from lompc_amd.settings import LOMPC_SOLVER  # noqa: F401

PRICE_SOLVER_SOLVER = "lompc_price_step"  # settings.py:21 (CVXPY QP -> exact host QP)
BIMPC_SOLVER = "lompc_bimpc_solve"        # settings.py:24 (Clarabel -> host interior point)
