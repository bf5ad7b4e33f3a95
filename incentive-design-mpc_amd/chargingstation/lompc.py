"""Drop-in module for ``chargingstation/lompc.py``.

Put ``incentive-design-mpc_amd/`` ahead of the reference checkout on
PYTHONPATH: ``chargingstation`` is a namespace package in the reference (no
``__init__.py``), so ``from chargingstation.lompc import LoMPC`` then resolves
here.  The sibling modules (settings, demand_data, price_regularizer,
price_solver, bimpc, charging_station) are drop-ins too, so the reference's
example runs without CVXPY; delete a sibling to take that module from the
reference instead.  See INTEGRATION.md.
"""
from lompc_amd.lompc import LoMPC, LoMPCConstants, SolverError  # noqa: F401
