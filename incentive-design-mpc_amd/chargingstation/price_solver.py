"""Drop-in module for ``chargingstation/price_solver.py`` (class PriceSolver,
price_solver.py:16-285), CVXPY-free: batched LoMPC engine + exact host price QP."""
from lompc_amd.price_solver import PriceSolver  # noqa: F401
