"""Drop-in module for ``chargingstation/price_regularizer.py`` (class PriceRegularizer,
price_regularizer.py:9-85), CVXPY-free: closed-form separable LP (lompc_lp_separable)."""
from lompc_amd.price_regularizer import PriceRegularizer, PriceRegularizerError  # noqa: F401
