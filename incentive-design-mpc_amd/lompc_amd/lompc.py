"""Drop-in ``LoMPC`` for the reference's CVXPY/Clarabel path.

Mirrors ``chargingstation/lompc.py`` (AkshayThiru/incentive-design-mpc):
same ``LoMPCConstants`` dataclass (lompc.py:12-26), same constructor checks
(lompc.py:36-38), same attributes (``N, delta, theta, y_max, w_max, ev_type,
q_scale, A, m`` — lompc.py:59-71) and the same methods ``solve_lompc``,
``get_sc_modulus``, ``get_input_mat``, ``get_price0``, ``phi``, ``Dphi``
(lompc.py:137-187).  ``solve_lompc`` returns a fresh ``(N,)`` ndarray and the
optimal cost including its constant, exactly what ``self.w.value`` /
``self.cost.value`` give at lompc.py:154-156.

Added for the batched hot path: ``set_params`` (S parameter sets at once) and
``solve_batch`` (B QPs in one device call with fused per-set reductions).

All numerics run in the HIP extension (``liblompc_amd.so``); this module only
moves buffers and maps status codes to the reference's exception types:
AssertionError (gamma > y_max, lompc.py:87), ValueError (negative
parameters: cvxpy nonneg Parameters, lompc.py:78-82) and ``SolverError``
(cvxpy.error.SolverError).
"""
from __future__ import annotations

import ctypes
from dataclasses import dataclass

import numpy as np

from . import _lib
from .settings import MAX_BAT_CHARGE_RATE, MAX_MAX_BAT_SOC, MIN_MAX_BAT_SOC, LOMPC_MODE


class SolverError(Exception):
    """Counterpart of ``cvxpy.error.SolverError``: no certified optimum."""


@dataclass
class LoMPCConstants:
    """
    delta:      Relative weight of charging cost.
    theta:      Battery capacity [kWh].
    y_max:      Maximum allowed state of charge (SoC) as a fraction of capacity.
    w_max:      Maximum fraction of charge replenished per time step (normalized charging rate).
    ev_type:    EV type, either "small" or "large".
    """

    delta: float
    theta: float
    y_max: float
    w_max: float
    ev_type: str


def _torch():
    import torch

    return torch


def _ptr(t) -> int | None:
    return None if t is None else t.data_ptr()


class LoMPC:
    def __init__(self, N: int, consts: LoMPCConstants, device: int | None = None,
                 mode: str | None = None) -> None:
        """
        Inputs:
            N:      LoMPC horizon length.
            consts: LoMPC constants.
            device: HIP device index (default: torch's current device).
            mode:   "path" (default) or "direct" — engine algorithm, see DESIGN.md.
        """
        # lompc.py:36-38
        assert (consts.y_max >= MIN_MAX_BAT_SOC) and (consts.y_max <= MAX_MAX_BAT_SOC)
        assert (consts.w_max >= 0) and (consts.w_max <= MAX_BAT_CHARGE_RATE)
        assert (consts.ev_type == "small") or (consts.ev_type == "large")
        self._ctx = None
        self._set_constants(N, consts)
        torch = _torch()
        self._lib = _lib.load()
        if not torch.cuda.is_available():
            raise RuntimeError("lompc_amd: no HIP device visible (the engine has no CPU path)")
        self.device = torch.cuda.current_device() if device is None else int(device)
        ctx = ctypes.c_void_p()
        ev = _lib.LOMPC_EV_SMALL if self.ev_type == "small" else _lib.LOMPC_EV_LARGE
        rc = self._lib.lompc_create(int(N), float(self.delta), float(self.theta), float(self.y_max),
                                    float(self.w_max), ev, self.device, ctypes.byref(ctx))
        if rc == _lib.LOMPC_ERR_UNSUPPORTED:
            raise ValueError(f"lompc_amd supports horizons N <= {_lib.LOMPC_MAX_N}")
        if rc == _lib.LOMPC_ERR_INVALID_ARG:
            raise AssertionError("invalid LoMPC constants (delta > 0, theta > 0 required)")
        if rc != _lib.LOMPC_OK:
            raise RuntimeError("lompc_create failed: " + _lib.status_text(self._lib, None, rc))
        self._ctx = ctx
        self._keep = ()
        self.S = 0
        self.set_mode(mode or LOMPC_MODE)

    def __del__(self):
        if getattr(self, "_ctx", None) is not None:
            try:
                self._lib.lompc_destroy(self._ctx)
            except Exception:
                pass
            self._ctx = None

    # ------------------------------------------------------------ lompc.py
    def _set_constants(self, N: int, consts: LoMPCConstants) -> None:
        # lompc.py:59-71
        self.N = N
        self.delta = consts.delta
        self.theta = consts.theta
        self.y_max = consts.y_max
        self.w_max = consts.w_max
        self.ev_type = consts.ev_type
        # Scaling factor for the quadratic electricity cost.
        self.q_scale = 3 * self.theta / (4 * self.w_max)
        # LoMPC input matrix, y = A w.
        self.A = np.tril(np.ones((self.N, self.N)))
        # Strong convexity modulus.
        self.m = 2 * self.delta * self.theta ** 2

    def _check_rc(self, rc: int) -> None:
        if rc == _lib.LOMPC_OK:
            return
        text = _lib.status_text(self._lib, self._ctx, rc)
        if rc == _lib.LOMPC_ERR_INVALID_ARG:
            raise ValueError(text)
        if rc == _lib.LOMPC_ERR_NOT_CONVERGED:
            raise SolverError(text)
        raise RuntimeError(text)

    def _validate_params(self, lmbd, lmbd_r, gamma) -> None:
        # lompc.py:87 and cvxpy's nonneg Parameter checks (lompc.py:78-82)
        assert gamma <= self.y_max
        lmbd = np.asarray(lmbd, dtype=np.float64)
        if lmbd.shape != (3 * self.N,):
            raise ValueError(f"Invalid dimensions {lmbd.shape} for Parameter value.")
        if gamma < 0 or lmbd_r < 0 or np.any(lmbd < 0):
            raise ValueError("Parameter value must be nonnegative.")

    def solve_lompc(self, lmbd: np.ndarray, lmbd_r: float, gamma: float) -> tuple[np.ndarray, float]:
        """
        Inputs:
            lmbd:   Unit price (incentive) vector.
            lmbd_r: Robustness price parameter.
            gamma:  Fraction of battery capacity remaining to be charged.
        Outputs:
            w_opt:      Optimal w vector.
            cost_opt:   Optimal cost.
        """
        self._validate_params(lmbd, lmbd_r, gamma)
        lm = np.ascontiguousarray(np.asarray(lmbd, dtype=np.float64))
        w = np.empty(self.N, dtype=np.float64)
        cost = ctypes.c_double(0.0)
        rc = self._lib.lompc_solve_host(self._ctx, lm.ctypes.data, float(lmbd_r), float(gamma),
                                        w.ctypes.data, ctypes.addressof(cost))
        self._check_rc(rc)
        self.S = 0  # the single-QP call reloads the context's parameter sets
        return w, float(cost.value)

    def get_sc_modulus(self) -> float:
        return self.m

    def get_input_mat(self) -> np.ndarray:
        return self.A

    def get_price0(self, w: np.ndarray, lmbd: np.ndarray, lmbd_r: float) -> float:
        # lompc.py:164-170
        price0 = (
            self.theta * (w[0] * lmbd[0] + (self.w_max - w[0]) * lmbd[self.N])
            + self.q_scale * w[0] ** 2 * lmbd[2 * self.N]
            + self.theta ** 2 * w[0] ** 2 * lmbd_r
        )
        return price0

    def phi(self, w: np.ndarray) -> np.ndarray:
        # lompc.py:172-177
        assert w.shape == (self.N,)
        return np.hstack((self.theta * w, self.theta * (self.w_max - w), self.q_scale * (w * w)))

    def Dphi(self, w: np.ndarray) -> np.ndarray:
        # lompc.py:179-187
        assert w.shape == (self.N,)
        return np.block([[self.theta * np.eye(self.N)], [-self.theta * np.eye(self.N)],
                         [2 * self.q_scale * np.diag(w)]])

    # ------------------------------------------------------------ batch API
    def set_mode(self, mode: str) -> None:
        m = {"path": _lib.LOMPC_MODE_PATH, "direct": _lib.LOMPC_MODE_DIRECT}[mode]
        self._check_rc(self._lib.lompc_set_mode(self._ctx, m))
        self.mode = mode

    def _dev(self, x, dtype=None):
        torch = _torch()
        dtype = dtype or torch.float64
        if isinstance(x, torch.Tensor):
            t = x.to(device=f"cuda:{self.device}", dtype=dtype)
        else:
            t = torch.as_tensor(np.asarray(x), dtype=dtype, device=f"cuda:{self.device}")
        return t.contiguous()

    def _stream(self) -> int:
        return _torch().cuda.current_stream(self.device).cuda_stream

    def set_params(self, lmbd, lmbd_r, w_ref=None, gamma_ref=None, validate: bool = True) -> None:
        """Load S parameter sets (one per (EV type, partition) price vector).

        lmbd: (S, 3N) or (3N,); lmbd_r: (S,) or scalar; w_ref: (S, N) or (N,)
        (needed for the A_bar error reduction); gamma_ref: (S,) central gamma
        (DIRECT mode warm start).  Device tensors are used in place.
        """
        torch = _torch()
        lm = self._dev(lmbd)
        if lm.dim() == 1:
            lm = lm.unsqueeze(0)
        S = lm.shape[0]
        if lm.shape[1] != 3 * self.N:
            raise ValueError(f"lmbd must have 3N = {3 * self.N} columns")
        lr = self._dev(lmbd_r).reshape(-1)
        if lr.numel() == 1 and S > 1:
            lr = lr.expand(S).contiguous()
        if lr.numel() != S:
            raise ValueError("lmbd_r must have one entry per parameter set")
        wr = None
        if w_ref is not None:
            wr = self._dev(w_ref).reshape(S, self.N)
        gr = None
        if gamma_ref is not None:
            gr = self._dev(gamma_ref).reshape(S)
        if validate:
            bad = torch.logical_not(lm >= 0).any() | torch.logical_not(lr >= 0).any()
            if bool(bad):
                raise ValueError("Parameter value must be nonnegative.")
        rc = self._lib.lompc_set_params(self._ctx, S, _ptr(lm), _ptr(lr), _ptr(wr), _ptr(gr), self._stream())
        self._check_rc(rc)
        self._keep = (lm, lr, wr, gr)
        self.S = S

    def solve_batch(self, gamma, set_offsets=None, *, want_w: bool = True, want_cost: bool = True,
                    want_w0: bool = False, want_status: bool = False, want_set: bool = True,
                    out: dict | None = None, check: bool = True) -> dict:
        """Solve B QPs against the loaded parameter sets.

        gamma: (B,) gamma_i = y_max - y0_i (device tensor or array-like).
        set_offsets: host int64 (S+1,) — EVs of set s are
            [set_offsets[s], set_offsets[s+1]); default: all EVs in set 0 (S must be 1).
        Returns a dict of device tensors: "w" (B, N), "cost" (B,), "w0" (B,),
        "status" (B,) int8, "set_sum_w" (S, N), "set_stats" (S, 8).
        ``check`` synchronises and raises on invalid input / uncertified QPs.
        """
        torch = _torch()
        if self.S < 1:
            raise RuntimeError("solve_batch: call set_params first")
        g = self._dev(gamma).reshape(-1)
        B = g.numel()
        if set_offsets is None:
            if self.S != 1:
                raise ValueError("set_offsets required when more than one parameter set is loaded")
            set_offsets = np.array([0, B], dtype=np.int64)
        off = np.ascontiguousarray(np.asarray(set_offsets, dtype=np.int64))
        if off.shape != (self.S + 1,):
            raise ValueError(f"set_offsets must have S+1 = {self.S + 1} entries")
        if check:
            # lompc.py:87 (assert gamma <= y_max); nonneg Parameter (lompc.py:82)
            if bool((g > self.y_max).any()):
                raise AssertionError("gamma <= y_max required")
            if bool(torch.logical_not(g >= 0).any()):
                raise ValueError("Parameter value must be nonnegative.")
        dev = f"cuda:{self.device}"
        res = {} if out is None else out

        def buf(name, shape, dtype=torch.float64, want=True):
            if not want:
                return None
            t = res.get(name)
            if t is None or tuple(t.shape) != tuple(shape) or t.dtype != dtype:
                t = torch.empty(shape, dtype=dtype, device=dev)
                res[name] = t
            return t

        w = buf("w", (B, self.N), want=want_w)
        cost = buf("cost", (B,), want=want_cost)
        w0 = buf("w0", (B,), want=want_w0)
        status = buf("status", (B,), torch.int8, want=want_status)
        ssw = buf("set_sum_w", (self.S, self.N), want=want_set)
        sst = buf("set_stats", (self.S, _lib.LOMPC_SET_STATS), want=want_set)
        rc = self._lib.lompc_solve_batch(self._ctx, B, _ptr(g), off.ctypes.data, _ptr(w), _ptr(cost),
                                         _ptr(w0), _ptr(status), _ptr(ssw), _ptr(sst), self._stream())
        self._check_rc(rc)
        res["_gamma"] = g
        if check:
            self.check_last()
        return res

    def check_last(self) -> tuple[int, int, int]:
        """Synchronise and raise on uncertified QPs; returns (repaired, failed, invalid)."""
        rep, fail, inv = ctypes.c_int64(0), ctypes.c_int64(0), ctypes.c_int64(0)
        rc = self._lib.lompc_last_status(self._ctx, self._stream(), ctypes.byref(rep), ctypes.byref(fail),
                                         ctypes.byref(inv))
        self._check_rc(rc)
        if inv.value:
            raise AssertionError(f"{inv.value} EVs with gamma outside [0, y_max]")
        if fail.value:  # a context has no plan: its own error text, if it set one
            why = self._lib.lompc_last_error(self._ctx).decode(errors="replace") or \
                "LoMPC QPs without a certified optimum"
            raise SolverError(f"{fail.value} EVs failed: {why}")
        return rep.value, fail.value, inv.value

    def profile(self, enable: bool | None = None, read: bool = False, reset: bool = False):
        """Kernel-time profiling of the per-EV evaluation kernel (HIP events)."""
        if enable is not None:
            self._check_rc(self._lib.lompc_profile_enable(self._ctx, int(bool(enable))))
        if read:
            ms, n = ctypes.c_double(0.0), ctypes.c_int64(0)
            self._check_rc(self._lib.lompc_profile_read(self._ctx, ctypes.byref(ms), ctypes.byref(n),
                                                        int(bool(reset))))
            return ms.value, n.value
        return None


class BatchPlan:
    """A fixed EV batch solved at new prices every price iteration: one C-ABI call per run.

    Wraps ``lompc_plan_create`` / ``lompc_plan_run`` (include/lompc_amd.h).  ``lompc`` is one
    ``LoMPC`` or a list of them (EV types of the same horizon and device); their parameter
    sets are stacked in list order (``sets_per_ctx`` gives how many each owns) and every
    ``run`` is ONE fused launch over all of them plus the per-set reduction.
    At construction the batch is validated, each set's gamma window is measured on the device
    (a plan is built per price loop / time step, where gamma_i = y_max - y0_i is fixed,
    price_solver.py:66-77; gamma is read at every run, and values moved outside the window
    later are still solved exactly, by the individual re-solve) and the outputs are allocated.
    ``run(lmbd, lmbd_r)`` then issues one ``lompc_plan_run`` with cached pointers; lmbd:
    contiguous fp64 device tensor (S, 3N), lmbd_r (S,) on the same device (or raw device
    pointers).  No synchronisation; ``check()`` synchronises and raises on failures of ANY run
    since the previous check (sticky device tallies).
    w_ref (S, N) is read at every run (update it in place).  ``warm_start``: every gamma
    cell's exact solve starts from the working set the previous run ended with.  ``diag_repair``
    (diagnostics): no solution path, every EV is re-solved individually.  ``close_in_eval``: the
    per-set reductions and re-solves inside k_eval (each set's last-arriving workgroup) instead of
    the k_finalize launch (measured slower with w rows: DESIGN.md §10).  ``sorted_gamma``: every
    set's gamma is ascending and stays unmodified until the next ``update`` — runs without per-EV
    outputs then aggregate per certified piece from prefix sums (k_agg, O(pieces) per run; a set
    found unsorted reports all its EVs failed).  ``sort_sets``: for plans without per-EV outputs
    (the price loop's reductions contract, price_solver.py:196-214: only per-set sums leave, so the
    EVs' order within a set does not matter) — the plan takes a SNAPSHOT of gamma at construction /
    ``update``, each set sorted ascending on the device (two stable sorts: by gamma, then by set), and
    runs as ``sorted_gamma`` over it; later in-place changes of the caller's gamma are not seen.
    ``close_in_finalize``: runs without w output close
    their sets in the k_finalize launch as well (A/B of the close mode).  ``cells``: gamma cells per
    set instead of the plan's choice (the answer does not depend on it).  ``set_comm(comm)``: a
    sharded batch — every run combines the set reductions of all ranks on the device (RCCL).
    DIRECT-mode contexts fall back to ``lompc_run`` (one context only).
    """

    def __init__(self, lompc, gamma, set_offsets, *, sets_per_ctx=None, w_ref=None, gamma_ref=None, want_w=True,
                 want_cost=True, want_w0=False, want_status=False, want_set=True, stream=None, validate=True,
                 warm_start=False, diag_repair=False, close_in_eval=False, sorted_gamma=False,
                 close_in_finalize=False, cells=None, sort_sets=False):
        torch = _torch()
        lompcs = list(lompc) if isinstance(lompc, (list, tuple)) else [lompc]
        self.lompcs = lompcs
        self.lompc = lompcs[0]
        lo = self.lompc
        N = lo.N
        if any(x.N != N or x.device != lo.device for x in lompcs):
            raise ValueError("BatchPlan: every LoMPC must have the same horizon and device")
        if len(lompcs) > _lib.LOMPC_PLAN_MAX_CTX:
            raise ValueError(f"BatchPlan: at most {_lib.LOMPC_PLAN_MAX_CTX} contexts")
        S = np.asarray(set_offsets).shape[0] - 1
        if sets_per_ctx is None:
            if len(lompcs) != 1:
                raise ValueError("sets_per_ctx required with several contexts")
            sets_per_ctx = [S]
        self.sets_per_ctx = np.ascontiguousarray(np.asarray(sets_per_ctx, dtype=np.int64))
        if self.sets_per_ctx.shape != (len(lompcs),) or int(self.sets_per_ctx.sum()) != S:
            raise ValueError("sets_per_ctx must give one count per context, summing to S")
        self.N = N
        self._want = dict(w=want_w, cost=want_cost, w0=want_w0, status=want_status, set=want_set)
        self.sort_sets = bool(sort_sets)
        if self.sort_sets and (want_w or want_cost or want_w0 or want_status):
            raise ValueError("sort_sets: plans without per-EV outputs only (the EVs are reordered)")
        sorted_gamma = sorted_gamma or self.sort_sets
        self._stream = (stream if stream is not None else torch.cuda.current_stream(lo.device)).cuda_stream
        self._lib = lo._lib
        self._plan = None
        self._broken = None
        self.comm = None
        self.direct = any(x.mode == "direct" for x in lompcs)
        if self.direct and len(lompcs) != 1:
            raise ValueError("DIRECT mode plans hold one context")
        self.gamma_ref = None if gamma_ref is None else lo._dev(gamma_ref).reshape(S)
        self._layout(gamma, set_offsets, w_ref, validate)
        if self.direct:
            return
        ctxs = (ctypes.c_void_p * len(lompcs))(*[x._ctx.value for x in lompcs])
        plan = ctypes.c_void_p()
        flags = ((_lib.LOMPC_PLAN_WARM_START if warm_start else 0) | (_lib.LOMPC_PLAN_DIAG_REPAIR if diag_repair else 0)
                 | (_lib.LOMPC_PLAN_CLOSE_IN_EVAL if close_in_eval else 0)
                 | (_lib.LOMPC_PLAN_SORTED_GAMMA if sorted_gamma else 0)
                 | (_lib.LOMPC_PLAN_CLOSE_IN_FINALIZE if close_in_finalize else 0)
                 | (_lib.LOMPC_PLAN_CELLS(cells) if cells else 0))
        self._flags = flags
        rc = self._lib.lompc_plan_create(len(lompcs), ctypes.cast(ctxs, ctypes.c_void_p), self.sets_per_ctx.ctypes.data,
                                         self.B, _ptr(self.gamma), self.off.ctypes.data, _ptr(self.w_ref), flags,
                                         self._stream, ctypes.byref(plan))
        if rc != _lib.LOMPC_OK:
            lo._check_rc(rc)
        self._plan = plan
        self.cells = self.info()["cells"]

    def _layout(self, gamma, set_offsets, w_ref, validate) -> None:
        """Validate and take a batch (gamma, set_offsets, w_ref); (re)allocate the outputs when
        the batch size changed."""
        torch = _torch()
        lo, N = self.lompc, self.N
        gamma = lo._dev(gamma).reshape(-1)
        B = gamma.numel()
        off = np.ascontiguousarray(np.asarray(set_offsets, dtype=np.int64))
        S = off.shape[0] - 1
        if S < 1 or off[0] != 0 or off[-1] != B or np.any(np.diff(off) < 0):
            raise ValueError("set_offsets must be non-decreasing from 0 to B")
        if S != int(self.sets_per_ctx.sum()):
            raise ValueError("the number of parameter sets is fixed for a plan")
        if validate:  # (callers that already checked 0 <= gamma <= y_max skip two host syncs)
            ym = np.repeat([x.y_max for x in self.lompcs], self.sets_per_ctx)
            ymax_ev = torch.as_tensor(np.repeat(ym, np.diff(off)), device=gamma.device)
            if bool((gamma > ymax_ev).any()):
                raise AssertionError("gamma <= y_max required")
            if bool(torch.logical_not(gamma >= 0).any()):
                raise ValueError("Parameter value must be nonnegative.")
        if getattr(self, "sort_sets", False) and B > 0:
            # each set's gamma ascending (NaN after the values: torch's sort order), by two stable
            # sorts — by gamma, then by set — on the device, once per batch
            g = gamma.to(torch.float64)
            o1 = torch.sort(g, stable=True).indices
            sid = torch.repeat_interleave(torch.arange(S, device=g.device),
                                          torch.as_tensor(np.diff(off), device=g.device))
            o2 = torch.sort(sid[o1], stable=True).indices
            gamma = g[o1[o2]].contiguous()
        self.gamma, self.off = gamma, off
        self.w_ref = None if w_ref is None else lo._dev(w_ref).reshape(S, N)
        wt = self._want
        per_ev = wt["w"] or wt["cost"] or wt["w0"] or wt["status"]
        # (re)allocate what the new shape changes: per-EV outputs with B, set outputs with S (a price loop's
        # plan, re-targeted at a partition of another size every step, has only set outputs)
        if getattr(self, "S", None) != S or (per_ev and getattr(self, "B", None) != B):
            dev = f"cuda:{lo.device}"
            e = lambda shape, dt=torch.float64: torch.empty(shape, dtype=dt, device=dev)
            self.out = {
                "w": e((B, N)) if wt["w"] else None,
                "cost": e((B,)) if wt["cost"] else None,
                "w0": e((B,)) if wt["w0"] else None,
                "status": e((B,), torch.int8) if wt["status"] else None,
                "set_sum_w": e((S, N)) if wt["set"] else None,
                "set_stats": e((S, _lib.LOMPC_SET_STATS)) if wt["set"] else None,
            }
            self._outs = [_ptr(self.out[k]) for k in ("w", "cost", "w0", "status", "set_sum_w", "set_stats")]
        self.S, self.B = S, B
        if self.direct:
            self._args = [_ptr(self.w_ref), _ptr(self.gamma_ref), B, _ptr(self.gamma), self.off.ctypes.data] + \
                self._outs + [self._stream]

    def launches_per_run(self) -> int:
        """Kernel launches of one run: k_path + k_eval + k_finalize; two when the sets close inside
        k_eval (runs without w output unless close_in_finalize, LOMPC_PLAN_CLOSE_IN_EVAL); a
        communicator adds the all-gather and the combine kernel."""
        if self.direct:
            return 2
        if self._flags & _lib.LOMPC_PLAN_SORTED_GAMMA and not any(self._want[k] for k in ("w", "cost", "w0", "status")):
            return 2 + (2 if self.comm is not None else 0)  # k_path + k_agg
        close = bool(self._flags & _lib.LOMPC_PLAN_CLOSE_IN_EVAL) or (
            not self._want["w"] and not self._flags & _lib.LOMPC_PLAN_CLOSE_IN_FINALIZE)
        return (2 if close else 3) + (2 if self.comm is not None else 0)

    def set_comm(self, comm) -> "BatchPlan":
        """Attach (None: detach) a ``dist.RcclComm``: every later run combines the set reductions of
        all ranks on the device (lompc_plan_set_comm) — collective: every rank runs the same
        sequence of runs."""
        if self.direct:
            raise ValueError("set_comm: PATH-mode plans only")
        self._check_rc(self._lib.lompc_plan_set_comm(self._plan, None if comm is None else comm.handle))
        self.comm = comm
        return self

    def info(self) -> dict:
        """Batch size, parameter sets, gamma cells per set, k_eval workgroups of the plan, the runs per
        stepped run_steps launch (1 once the stepped form has run, else 0) and whether run_steps' wide
        form evaluates through k_evals_st (the stager wave: set reductions grouped by seven row waves)."""
        if self.direct:
            return {"B": self.B, "sets": self.S, "cells": 0, "workgroups": 0, "steps_group": 0, "evals_staged": False}
        B, S, cells, wg, grp = ctypes.c_int64(0), ctypes.c_int64(0), ctypes.c_int(0), ctypes.c_int(0), ctypes.c_int(0)
        self._check_rc(self._lib.lompc_plan_get_info(self._plan, ctypes.byref(B), ctypes.byref(S), ctypes.byref(cells),
                                                     ctypes.byref(wg), ctypes.byref(grp)))
        return {"B": B.value, "sets": S.value, "cells": cells.value, "workgroups": wg.value,
                "steps_group": min(grp.value, 1), "evals_staged": grp.value == 2}

    def update(self, gamma, set_offsets, w_ref=None, validate=True) -> "BatchPlan":
        """Re-target the plan at a new batch with the same contexts and set counts (e.g. the
        next partition of a price loop): device buffers, events and pinned staging are reused,
        the outputs are reallocated only when the batch size changes.  If the device-side update
        fails the plan is unusable (every later run raises): the C plan may still point at the
        previous buffers, which stay referenced."""
        old = (self.gamma, self.w_ref, getattr(self, "out", None))
        self._layout(gamma, set_offsets, w_ref, validate)
        if not self.direct:
            rc = self._lib.lompc_plan_update(self._plan, self.B, _ptr(self.gamma), self.off.ctypes.data,
                                             _ptr(self.w_ref), self._stream)
            if rc != _lib.LOMPC_OK:
                self._broken = (old, _lib.status_text(self._lib, None, rc, plan=self._plan))
                self._check_rc(rc)
        return self

    def reserve(self, max_B: int) -> "BatchPlan":
        """Size hint (lompc_plan_reserve): every workspace that must grow is sized for batches of
        up to max_B EVs at once.  The plan's current batch is re-prepared here, so the workspaces
        are allocated now (at plan creation) rather than inside a later ``update``."""
        if not self.direct:
            self._check_rc(self._lib.lompc_plan_reserve(self._plan, int(max_B)))
            self.update(self.gamma, self.off, self.w_ref, validate=False)
        return self

    def _usable(self) -> None:
        if getattr(self, "_broken", None):
            raise RuntimeError(f"BatchPlan unusable after a failed update: {self._broken[1]}")
        if self.comm is not None and self.comm.handle is None:  # (dist.release_comms destroyed it)
            raise RuntimeError("BatchPlan: its communicator was closed; attach another (set_comm) or None")

    def __del__(self):
        if getattr(self, "_plan", None) is not None:
            try:
                self._lib.lompc_plan_destroy(self._plan)
            except Exception:
                pass
            self._plan = None

    def _check_rc(self, rc: int) -> None:
        if rc == _lib.LOMPC_OK:
            return
        text = _lib.status_text(self._lib, None, rc, plan=self._plan)
        if rc == _lib.LOMPC_ERR_INVALID_ARG:
            raise ValueError(text)
        if rc == _lib.LOMPC_ERR_NOT_CONVERGED:
            raise SolverError(text)
        raise RuntimeError(text)

    def run(self, lmbd, lmbd_r) -> dict:
        """lmbd / lmbd_r: device tensors, or raw device pointers (int)."""
        pl = lmbd if isinstance(lmbd, int) else lmbd.data_ptr()
        pr = lmbd_r if isinstance(lmbd_r, int) else lmbd_r.data_ptr()
        self._usable()
        if self.direct:
            lo = self.lompc
            rc = lo._lib.lompc_run(lo._ctx, self.S, pl, pr, *self._args)
            if rc:
                lo._check_rc(rc)
            lo.S = self.S
            return self.out
        rc = self._lib.lompc_plan_run(self._plan, pl, pr, *self._outs, self._stream)
        if rc:
            self._check_rc(rc)
        return self.out

    def run_steps(self, lmbd, lmbd_r, n_runs: int, lmbd_stride: int, lmbd_r_stride: int = 0,
                  profile_every: int = 0, per_run_sets: bool = False, per_run: bool = False, out=None,
                  per_kernel: bool = False, span_events: bool = False) -> dict:
        """n_runs consecutive independent runs in ONE C-ABI call (lompc_plan_run_steps): run k at the
        prices lmbd + k lmbd_stride, lmbd_r + k lmbd_r_stride (device pointers or tensors, strides in
        doubles); profile_every > 0: only every E-th stepped launch carries the enabled HIP events.

        Outputs: by default every run writes the plan's ``out`` buffers (the last run's remain).
        per_run_sets: every run's set reductions kept — ``set_sum_w`` / ``set_stats`` of the returned
        dict are (n_runs, S, N) / (n_runs, S, 8); per_run: every output kept per run (w (n_runs, B, N),
        cost / w0 / status (n_runs, B), sets as above).  out: a dict of preallocated per-run tensors for any of those keys (the others as the
        flags say).  per_kernel: LOMPC_STEPS_PER_KERNEL (the same runs, one part per launch, bit for
        bit the same outputs); span_events: one event pair over the stepped launches
        (LOMPC_STEPS_SPAN_EVENTS)."""
        call, res = self.steps_call(lmbd, lmbd_r, n_runs, lmbd_stride, lmbd_r_stride, profile_every=profile_every,
                                    per_run_sets=per_run_sets, per_run=per_run, out=out, per_kernel=per_kernel,
                                    span_events=span_events)
        call()
        return res

    def steps_call(self, lmbd, lmbd_r, n_runs: int, lmbd_stride: int, lmbd_r_stride: int = 0,
                   profile_every: int = 0, per_run_sets: bool = False, per_run: bool = False, out=None,
                   per_kernel: bool = False, span_events: bool = False):
        """run_steps prepared: (call, outputs) — ``call()`` issues the same lompc_plan_run_steps with
        every argument already converted (no Python work between the caller's clock and the C-ABI
        entry beyond one ctypes call); it may be called again for the same runs into the same
        outputs."""
        if self.direct:
            raise ValueError("run_steps: PATH-mode plans only")
        self._usable()
        torch = _torch()
        K = int(n_runs)
        pl = lmbd if isinstance(lmbd, int) else lmbd.data_ptr()
        pr = lmbd_r if isinstance(lmbd_r, int) else lmbd_r.data_ptr()
        keys = ("w", "cost", "w0", "status", "set_sum_w", "set_stats")
        shapes = {"w": (K, self.B, self.N), "cost": (K, self.B), "w0": (K, self.B), "status": (K, self.B),
                  "set_sum_w": (K, self.S, self.N), "set_stats": (K, self.S, _lib.LOMPC_SET_STATS)}
        given = dict(out or {})
        res = dict(self.out)
        for k in keys:
            if self.out[k] is None:
                if given.get(k) is not None:
                    raise ValueError(f"run_steps: the plan has no {k} output")
                continue
            if k in given or per_run or (per_run_sets and k in ("set_sum_w", "set_stats")):
                t = given.get(k)
                if t is None:
                    t = torch.empty(shapes[k], dtype=self.out[k].dtype, device=self.out[k].device)
                elif tuple(t.shape) != shapes[k] or t.dtype != self.out[k].dtype or not t.is_contiguous() \
                        or t.device != self.out[k].device:
                    raise ValueError(f"run_steps: out[{k!r}] must be a contiguous {self.out[k].dtype} tensor {shapes[k]}")
                res[k] = t
        per_ev = [k for k in ("w", "cost", "w0", "status") if res[k] is not None]
        strided = [res[k].dim() == self.out[k].dim() + 1 for k in per_ev]
        if any(strided) and not all(strided):
            raise ValueError("run_steps: the per-EV outputs are either all per run or all shared")
        ev_stride = self.B if per_ev and strided[0] else 0
        sw_stride = self.S * self.N if res["set_sum_w"] is not None and res["set_sum_w"].dim() == 3 else 0
        st_stride = self.S * _lib.LOMPC_SET_STATS if res["set_stats"] is not None and res["set_stats"].dim() == 3 else 0
        if (res["set_sum_w"] is None) != (res["set_stats"] is None) or (sw_stride == 0) != (st_stride == 0):
            raise ValueError("run_steps: set_sum_w and set_stats are both per run or both shared")
        flags = (_lib.LOMPC_STEPS_PER_KERNEL if per_kernel else 0) | (_lib.LOMPC_STEPS_SPAN_EVENTS if span_events else 0)
        ptrs = [_ptr(res[k]) for k in keys]
        fn = self._lib.lompc_plan_run_steps
        args = (self._plan, pl, int(lmbd_stride), pr, int(lmbd_r_stride), K, int(profile_every), *ptrs, sw_stride,
                st_stride, ev_stride, flags, self._stream)
        check = self._check_rc

        def call():
            rc = fn(*args)
            if rc:
                check(rc)

        return call, res

    def run_chain(self, lmbd0, lmbd_r, w_target, step: float, n_runs: int, out=None) -> dict:
        """n_runs DEPENDENT runs in one C-ABI call (lompc_plan_run_chain): run 0 at lmbd0 (S, 3N), run
        k >= 1 at prices computed on the device from run k-1's set reductions by a projected
        dual-gradient step ``max(0, lmbd + step (phi(sum_w / count) - phi(w_target)))`` — the
        dependence of the reference's price iterations (price_solver.py:111-140).  Returns the plan's
        ``out`` with ``lmbd`` (n_runs, S, 3N), ``set_sum_w`` (n_runs, S, N) and ``set_stats``
        (n_runs, S, 8) per run (``out``: preallocated tensors for any of those three); the per-EV
        outputs are the plan's buffers, holding the last run's."""
        if self.direct:
            raise ValueError("run_chain: PATH-mode plans only")
        if self.out["set_sum_w"] is None:
            raise ValueError("run_chain: the plan needs its set outputs (want_set=True)")
        self._usable()
        torch = _torch()
        K, S, N = int(n_runs), self.S, self.N
        dev = self.out["set_sum_w"].device
        shapes = {"lmbd": (K, S, 3 * N), "set_sum_w": (K, S, N), "set_stats": (K, S, _lib.LOMPC_SET_STATS)}
        res = dict(self.out)
        for k, shp in shapes.items():
            t = (out or {}).get(k)
            if t is None:
                t = torch.empty(shp, dtype=torch.float64, device=dev)
            elif tuple(t.shape) != shp or t.dtype != torch.float64 or not t.is_contiguous() or t.device != dev:
                raise ValueError(f"run_chain: out[{k!r}] must be a contiguous float64 tensor {shp} on {dev}")
            res[k] = t
        lo = self.lompc
        l0, lr, wt = lo._dev(lmbd0).reshape(S, 3 * N), lo._dev(lmbd_r).reshape(S), lo._dev(w_target).reshape(S, N)
        rc = self._lib.lompc_plan_run_chain(self._plan, _ptr(l0), _ptr(lr), _ptr(wt), float(step), K, _ptr(res["lmbd"]),
                                            *self._outs[:4], _ptr(res["set_sum_w"]), _ptr(res["set_stats"]),
                                            self._stream)
        if rc:
            self._check_rc(rc)
        res["_keep"] = (l0, lr, wt)  # (alive until the caller's stream has used them)
        return res

    def check(self) -> tuple[int, int, int]:
        """Synchronise the plan's stream; raise on uncertified QPs; returns (repaired, failed, invalid)."""
        if self.direct:
            torch = _torch()
            with torch.cuda.stream(torch.cuda.ExternalStream(self._stream)):
                return self.lompc.check_last()
        rep, fail, inv = ctypes.c_int64(0), ctypes.c_int64(0), ctypes.c_int64(0)
        rc = self._lib.lompc_plan_status(self._plan, self._stream, ctypes.byref(rep), ctypes.byref(fail),
                                         ctypes.byref(inv))
        self._check_rc(rc)
        if inv.value:
            raise AssertionError(f"{inv.value} EVs with gamma outside [0, y_max]")
        if fail.value:  # (the plan's text names an unsorted set of a sorted_gamma plan)
            why = self._lib.lompc_plan_last_error(self._plan).decode(errors="replace") or \
                "LoMPC QPs without a certified optimum"
            raise SolverError(f"{fail.value} EVs failed: {why}")
        return rep.value, fail.value, inv.value

    KERNELS = ("k_path", "k_eval", "k_finalize")

    def profile(self, enable=None, read: bool = False, reset: bool = False, kernel: str = "k_eval"):
        """HIP-event timing of the plan's kernels (DIRECT: k_direct only).

        enable: True (k_eval), False, or a collection of kernel names from KERNELS;
        read: (total ms, launches) of ``kernel`` since the last reset."""
        if self.direct:
            return self.lompc.profile(enable=enable, read=read, reset=reset)
        if enable is not None:
            if enable is True:
                enable = ("k_eval",)
            mask = 0 if enable is False else sum(1 << self.KERNELS.index(k) for k in enable)
            self._check_rc(self._lib.lompc_plan_profile_enable(self._plan, mask))
        if read:
            ms, n = ctypes.c_double(0.0), ctypes.c_int64(0)
            self._check_rc(self._lib.lompc_plan_profile_read(self._plan, self.KERNELS.index(kernel), ctypes.byref(ms),
                                                             ctypes.byref(n), int(bool(reset))))
            return ms.value, n.value
        return None
