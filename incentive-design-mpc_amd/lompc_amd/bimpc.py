"""CVXPY-free ``BiMPC`` (chargingstation/bimpc.py:12-295).

Same enum, dataclasses, constructor checks, attributes and ``solve_bimpc``
signature as the reference.  The conic problem the reference builds with CVXPY
and solves with Clarabel (bimpc.py:87-114, :182-292) is solved by
``lompc_bimpc_solve`` in the C-ABI library: a primal-dual interior-point method
on the same smooth, strictly convex program (see csrc/lompc_bimpc.cpp).
"""
from __future__ import annotations

import ctypes
from dataclasses import dataclass
from enum import Enum

import time

import numpy as np

from . import _lib
from .lompc import LoMPCConstants, SolverError


class BiMPCChargingCostType(Enum):
    WEIGHTED = 0
    UNWEIGHTED = 1
    EXP_UNWEIGHTED = 2


@dataclass
class BiMPCConstants:
    """
    delta:              Relative weight of charging cost.
    c_g:                Electricity generation cost coefficient.
    u_g_max:            Maximum electricity generation per timestep.
    u_b_max:            Maximum charge/discharge rate of the storage battery.
    x_max:              Battery storage capacity.
    charging_cost_type: Enum of type BiMPCChargingCostType.
    exp_rate:           Rate of expoenential growth for EXP_UNWEIGHTED charging cost.
    """

    delta: float
    c_g: float
    u_g_max: float
    u_b_max: float
    x_max: float
    charging_cost_type: BiMPCChargingCostType
    exp_rate: float = 1  # Use np.Inf if only the cost at the final timestep is needed.


@dataclass
class BiMPCParameters:
    """
    Mp_s:       Number of small EVs in each partition.
    Mp_l:       Number of large EVs in each partition.
    beta_s:     Robustness bounds, for each partition of small EVs.
    beta_l:     Robustness bounds, for each partition of large EVs.
    gamma_sm:   Average fraction of battery capacity to be charged, for each partition of small EVs.
    gamma_lm:   Average fraction of battery capacity to be charged, for each partition of large EVs.
    x0:         Current charge of the storage battery.
    demand:     External electricity demand forecast for the control horizon.
    """

    Mp_s: np.ndarray
    Mp_l: np.ndarray
    beta_s: np.ndarray
    beta_l: np.ndarray
    gamma_sm: np.ndarray
    gamma_lm: np.ndarray
    x0: float
    demand: np.ndarray


def _c(a) -> np.ndarray:
    return np.ascontiguousarray(np.asarray(a, dtype=np.float64))


class BiMPC:
    def __init__(self, N: int, P: int, consts_bi: BiMPCConstants, consts_s: LoMPCConstants,
                 consts_l: LoMPCConstants) -> None:
        """
        Inputs:
            N:                  Horizon length.
            P:                  Number of partitions per EV type.
            consts_bi:          BiMPC constants.
            consts_s:           LoMPC constants for small EVs.
            consts_l:           LoMPC constants for large EVs.
        """
        # bimpc.py:79-84
        assert consts_bi.delta >= 0
        assert consts_bi.c_g >= 0
        assert consts_bi.u_g_max >= 0
        assert consts_bi.u_b_max >= 0
        assert consts_bi.x_max >= 0
        assert consts_bi.exp_rate >= 1
        self._set_constants(N, P, consts_bi, consts_s, consts_l)
        self._lib = _lib.load()
        self.last_info = None
        self.last_duals = None

    def _set_constants(self, N, P, consts_bi, consts_s, consts_l) -> None:
        # bimpc.py:116-140
        self.N = N
        self.P = P
        self.delta = consts_bi.delta
        self.c_g = consts_bi.c_g
        self.u_g_max = consts_bi.u_g_max
        self.u_b_max = consts_bi.u_b_max
        self.x_max = consts_bi.x_max
        self.exp_rate = consts_bi.exp_rate * 1.0
        self.charging_cost_type = consts_bi.charging_cost_type
        self.theta_s = consts_s.theta
        self.theta_l = consts_l.theta
        self.w_max_s = consts_s.w_max
        self.w_max_l = consts_l.w_max
        # BiMPC input matrix, x = A u_b + x0 1.
        self.A = np.tril(np.ones((self.N, self.N)))

    def solve_bimpc(self, params: BiMPCParameters) -> tuple[np.ndarray, np.ndarray, np.ndarray]:
        """
        Inputs:
            params: BiMPC problem parameters.
        Outputs:
            w_hat_s_opt:    Team-optimal electricity output for small EVs.
            w_hat_l_opt:    Team-optimal electricity output for large EVs.
            u_g_opt:        Team-optimal electricity generation.
        """
        # bimpc.py:278-283
        assert (params.Mp_s.shape == (self.P,)) and (params.Mp_l.shape == (self.P,))
        assert (params.beta_s.shape == (self.P,)) and (params.beta_l.shape == (self.P,))
        assert (params.gamma_sm.shape == (self.P,)) and (params.gamma_lm.shape == (self.P,))
        assert params.demand.shape == (self.N,)
        # cvxpy nonneg Parameters (bimpc.py:149-167)
        for name in ("Mp_s", "Mp_l", "gamma_sm", "gamma_lm", "demand"):
            if np.any(np.asarray(getattr(params, name)) < 0):
                raise ValueError("Parameter value must be nonnegative.")
        if params.Mp_s @ params.beta_s < 0 or params.Mp_l @ params.beta_l < 0:
            raise ValueError("Parameter value must be nonnegative.")
        N, P = self.N, self.P
        w_s = np.empty((P, N))
        w_l = np.empty((P, N))
        u_g = np.empty(N)
        n = (2 * P + 1) * N
        duals = np.empty(2 * n + 4 * N)
        info = np.zeros(_lib.LOMPC_BIMPC_INFO)  # info[0] = 0: default iteration cap
        arrs = [_c(params.Mp_s), _c(params.Mp_l), _c(params.beta_s), _c(params.beta_l), _c(params.gamma_sm),
                _c(params.gamma_lm)]
        dem = _c(params.demand)
        t0 = time.perf_counter()
        rc = self._lib.lompc_bimpc_solve(
            N, P, int(self.charging_cost_type.value), float(self.delta), float(self.c_g), float(self.u_g_max),
            float(self.u_b_max), float(self.x_max), float(self.exp_rate), float(self.theta_s), float(self.theta_l),
            float(self.w_max_s), float(self.w_max_l), *[a.ctypes.data for a in arrs], float(params.x0),
            dem.ctypes.data, w_s.ctypes.data, w_l.ctypes.data, u_g.ctypes.data, duals.ctypes.data,
            info.ctypes.data)
        self.last_info = dict(iterations=int(info[0]), objective=info[1], primal_residual=info[2],
                              dual_residual=info[3], complementarity=info[4],
                              solve_ms=(time.perf_counter() - t0) * 1e3)
        self.last_duals = duals
        if rc == _lib.LOMPC_ERR_NOT_CONVERGED:
            raise SolverError("BiMPC interior point did not converge (infeasible storage bounds?)")
        if rc != _lib.LOMPC_OK:
            raise ValueError(_lib.status_text(self._lib, None, rc))
        return w_s, w_l, u_g

    def get_bat_input_mat(self) -> np.ndarray:
        return self.A
