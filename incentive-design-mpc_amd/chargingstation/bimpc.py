"""Drop-in module for ``chargingstation/bimpc.py`` (bimpc.py:12-295), CVXPY-free: the
BiMPC conic program is solved by the host interior point lompc_bimpc_solve."""
from lompc_amd.bimpc import BiMPC, BiMPCChargingCostType, BiMPCConstants, BiMPCParameters  # noqa: F401
