"""Drop-in module for ``chargingstation/lompc.py``.

Put ``incentive-design-mpc_amd/`` ahead of the reference checkout on
PYTHONPATH: ``chargingstation`` is a namespace package in the reference (no
``__init__.py``), so ``from chargingstation.lompc import LoMPC`` then resolves
here while ``chargingstation.price_solver`` etc. still come from the
reference.  See INTEGRATION.md.
"""
from lompc_amd.lompc import LoMPC, LoMPCConstants, SolverError  # noqa: F401
