"""Drop-in module for ``chargingstation/demand_data.py`` (demand_data.py:21-37)."""
from lompc_amd.demand_data import medium_term_demand_forecast  # noqa: F401
