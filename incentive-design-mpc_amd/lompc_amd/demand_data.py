"""External demand forecast (chargingstation/demand_data.py:21-37) without matplotlib.

The 24 "MediumTermLoadForecast" rows the reference reads from
``data/Real-Time Total Load.csv`` (``data[30:54]``, demand_data.py:26) ship as
``data/medium_term_load_forecast.json`` (the reference's own input data, copied
as numbers with its provenance recorded in the file).
"""
from __future__ import annotations

import json
import os

import numpy as np

_DATA = os.path.join(os.path.dirname(os.path.abspath(__file__)), "data", "medium_term_load_forecast.json")


def _get_forecast_24() -> np.ndarray:
    with open(_DATA) as f:
        rows = json.load(f)["rows"]
    return np.asarray(rows, dtype=float)  # (24, 2): Hour_End, Load_Forecast


def medium_term_demand_forecast(hours: int, scale: float, interpolate: bool = False) -> np.ndarray:
    """demand_data.py:21-37."""
    # Mid-hour forecasts every hour, starting at 00:00.
    forecast_24 = _get_forecast_24()
    # Interpolated demand forecasts every 30 mins, starting from 00:00.
    forecast_48 = np.zeros((48,))
    forecast_48[1::2] = forecast_24[:, 1]
    forecast_48[0::2] = (forecast_24[:, 1] + forecast_24[:, 1].take(range(-1, 23), mode="wrap")) / 2
    forecast_48_ = forecast_48.tolist()
    demand = forecast_48_ * (hours // 24) + forecast_48_[: 2 * (hours % 24)]
    if not interpolate:
        demand = demand[0::2]
    return scale * np.array(demand)
