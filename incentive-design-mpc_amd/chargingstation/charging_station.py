"""Drop-in module for ``chargingstation/charging_station.py`` (charging_station.py:16-433):
the closed-loop station on the batched engine (device-resident EV state)."""
from lompc_amd.charging_station import ChargingStation, ChargingStationConstants  # noqa: F401
