"""lompc_amd — MI355X-native batched LoMPC QP engine (drop-in for lompc.py's CVXPY path).

Import path: add ``incentive-design-mpc_amd/`` to ``sys.path`` (the reference is
also used via PYTHONPATH, README.md:25-28).
"""
from .lompc import BatchPlan, LoMPC, LoMPCConstants, SolverError  # noqa: F401
from .price_ops import solve_sets, set_errors  # noqa: F401

__all__ = ["BatchPlan", "LoMPC", "LoMPCConstants", "SolverError", "solve_sets", "set_errors"]
