"""CVXPY-free ``PriceSolver`` on the batched engine (chargingstation/price_solver.py:16-285).

Same constructor, attributes and methods as the reference.  What runs where:

* every LoMPC solve of a price iteration — the per-EV loop of ``_get_w_err``
  (price_solver.py:203-209) AND the central solve at gamma_sc (:106, :132) — is
  ONE ``lompc_run`` call: parameter set 0 holds this rank's EVs (fused sum of w,
  max A_bar error), set 1 holds the single central QP (its w and cost come back
  as set 1's sum of w and sum of cost);
* the price-gradient step (:216-246) is ``lompc_price_step`` (exact non-negative
  QP on the host, no CVXPY/Clarabel), the regularizer LP (:248-255) is
  ``PriceRegularizer`` (closed-form separable LP);
* ``get_w0_price0`` (:272-285) is one batched solve with fused price0 sums.

The loop keeps the reference's numpy arrays and their aliasing
(``lmbd_k = lmbd_k_new`` at :140 makes the two names one array, so from the
second iteration on the price term of ``dual_cost_decrease_actual`` at :136 is
zero) so ``solver_stats`` match the reference's entry by entry.

Sharded mode (``group`` given): ``set_charge_levels`` receives this rank's EVs;
the batch statistics (min / max / mean / count, price_solver.py:73-77) are combined with
torch.distributed.  On RCCL the plans carry the extension's own communicator
(``dist.device_comm``): every engine call combines the fused reductions of all ranks on the
device, so the whole price loop stays ONE C-ABI call (``lompc_price_loop``) exactly as on a
single rank, and every rank takes the same price steps on bitwise identical inputs.  On gloo
(the CPU tests) the Python loop combines them with ``dist.combine_set_results``.
DIRECT-mode plans also take the Python loop.
"""
from __future__ import annotations

import ctypes
import functools
import time

import numpy as np

from . import _lib
from . import settings as _settings
from .lompc import BatchPlan, LoMPC, LoMPCConstants, SolverError
from .price_regularizer import PriceRegularizer, PriceRegularizerError
from .settings import PRICE_SOLVER_EPS_REG, PRICE_SOLVER_EPS_TOL


def _torch():
    import torch

    return torch


def _solver_stream(fn):
    """Run a PriceSolver method on the solver's own stream, ordered after the caller's stream
    (its inputs) and before it (its outputs), so two solvers' loops can run side by side."""

    @functools.wraps(fn)
    def wrapped(self, *args, **kwargs):
        torch = _torch()
        caller = torch.cuda.current_stream(self.lompc.device)
        if caller == self._stream:
            return fn(self, *args, **kwargs)
        self._stream.wait_stream(caller)
        try:
            with torch.cuda.stream(self._stream):
                return fn(self, *args, **kwargs)
        finally:
            caller.wait_stream(self._stream)

    return wrapped


class PriceSolver:
    def __init__(self, N: int, consts: LoMPCConstants, price_type: str, device: int | None = None,
                 mode: str | None = None, group=None) -> None:
        """
        Inputs:
            N:          Horizon length.
            consts:     LoMPC constants.
            price_type: "linear" or "linear-convex".
            device:     HIP device (default: torch's current device).
            mode:       LoMPC engine mode ("path" default).
            group:      torch.distributed process group when the EVs are sharded over ranks.
        """
        assert (price_type == "linear") or (price_type == "linear-convex")  # price_solver.py:24
        self.lompc = LoMPC(N, consts, device=device, mode=mode)
        self._set_constants(N, consts, price_type)
        self.price_reg = PriceRegularizer(self.N, self.r)
        self.group = group
        self._lib = _lib.load()
        torch = _torch()
        dev = f"cuda:{self.lompc.device}"
        self._dev = dev
        # per-iteration inputs [lmbd (2, 3N) | lmbd_r (2) | w_ref (2, N)]: staged in pinned host
        # memory and moved by ONE async copy per engine call
        n_in = 6 * N + 2 + 2 * N
        self._in = torch.zeros(n_in, dtype=torch.float64, device=dev)
        self._h_in = torch.zeros(n_in, dtype=torch.float64).pin_memory()
        self._h_in_np = self._h_in.numpy()
        self._lm2 = self._in[: 6 * N].view(2, 3 * N)
        self._lr2 = self._in[6 * N: 6 * N + 2]
        self._wr2 = self._in[6 * N + 2:].view(2, N)
        self._h_sw = torch.zeros((2, N), dtype=torch.float64).pin_memory()
        self._h_st = torch.zeros((2, _lib.LOMPC_SET_STATS), dtype=torch.float64).pin_memory()
        self._plan = None
        # path cells per set of the loop plans (None: the engine's choice).  6: the device loop's
        # iteration is a chain through the slowest of its S x G waves and their records — fewer, longer
        # cells measured faster (scripts/loop_timing.py on the long-regime fixtures, us per iteration:
        # 4 cells 13.64 / 15.60, 6: 13.66 / 15.10, 8: 13.86 / 15.25, 16: 14.43 / 15.49, 32: 16.06 / 17.37)
        self.loop_cells = 6
        self.reserve_evs = 0  # > 0: the loop plans' workspaces sized for this many EVs (BatchPlan.reserve)
        self._plan_w0 = None
        self._w0_live = False
        self._staged = {}  # partition -> its loop plan and levels (stage_partition / use_partition)
        self._A_bar = None
        self._A_bar_inv = None
        self._kappa = None
        self.native_loop = True  # the price loop in C++ (lompc_price_loop) whenever the plan allows it
        self.profile_loops = False  # accumulate the native loop's per-part times in loop_prof
        # the convergence test and the price QP on the GPU after every engine call, no host round trip
        # per iteration (lompc_loop.hip); False: the host form (one copy + sync per iteration)
        self.device_loop = True
        if self.group is not None:
            import torch.distributed as dist

            # several ranks: the host-synchronous C++ loop (one engine call, its collective and a sync
            # per iteration, nothing enqueued ahead) until the device loop's ahead-enqueued collectives
            # have run on RCCL at world >= 2 (only world-1 RCCL runs on the one-GPU test box)
            if dist.get_world_size(self.group) > 1:
                self.device_loop = False
        self.loop_prof = np.zeros(_lib.LOMPC_LOOP_PROF)
        self.loop_host_ms = {"native_loop": 0.0, "finish_prices": 0.0}
        # the solver's own stream: its loop can run beside the other EV type's (charging_station)
        self._stream = torch.cuda.Stream(device=self.lompc.device)
        self.n_batched_calls = 0

    # ------------------------------------------------------------ price_solver.py
    def _set_constants(self, N: int, consts: LoMPCConstants, price_type: str) -> None:
        # price_solver.py:42-64
        self.nEVs = None
        self.N = N
        if price_type == "linear":
            self.r = 2 * self.N
        else:
            self.r = 3 * self.N
        self.consts = consts
        self.price_type = price_type
        self.y0 = None
        self.y0_rng = None
        self.gamma_sc = None
        self.prev_prices = np.zeros((self.r,))
        self.A = self.lompc.get_input_mat()
        self.eps_reg = PRICE_SOLVER_EPS_REG
        self.eps_tol = PRICE_SOLVER_EPS_TOL
        self.m = self.lompc.get_sc_modulus()

    def _rank(self) -> int:
        if self.group is None:
            return 0
        import torch.distributed as dist

        return dist.get_rank(self.group)


    @_solver_stream
    def set_charge_levels(self, y0) -> None:
        """price_solver.py:66-77.  y0: (nEVs,) ndarray or device tensor (this rank's shard
        in sharded mode)."""
        torch = _torch()
        if isinstance(y0, torch.Tensor):
            y0d = y0.to(device=self._dev, dtype=torch.float64).reshape(-1)
            assert y0d.dim() == 1
            if self.group is None:
                n = int(y0d.numel())
                if n == 0:
                    raise ValueError("zero-size array to reduction operation maximum which has no identity")
                stats = torch.stack([y0d.max(), y0d.min(), y0d.sum()]).cpu().numpy()  # one host sync
                assert stats[1] >= 0 and stats[0] <= self.consts.y_max  # 0 <= y0 <= y_max (NaN fails)
                self.nEVs = n
                y_hi, y_lo, y_mean = stats[0], stats[1], stats[2] / n
            else:
                y_hi, y_lo, y_mean = self._global_levels(y0d)
            self.y0 = y0d
            gamma = self.consts.y_max - y0d
        else:
            y0 = np.asarray(y0, dtype=np.float64)
            assert all(y0 >= 0) and all(y0 <= self.consts.y_max)
            assert len(y0.shape) == 1
            if self.group is None:
                self.nEVs = len(y0)
                y_hi, y_lo, y_mean = np.max(y0), np.min(y0), np.mean(y0)
            else:
                y_hi, y_lo, y_mean = self._global_levels(torch.as_tensor(y0, device=self._dev))
            self.y0 = y0
            gamma = torch.as_tensor(self.consts.y_max - y0, device=self._dev)
        self._y_hi, self._y_lo = float(y_hi), float(y_lo)
        self.y0_rng = (y_hi - y_lo) / 2  # = \bar{\Gamma}
        self.gamma_sc = self.consts.y_max - (y_hi + y_lo) / 2
        self.gamma_sm = self.consts.y_max - y_mean
        self._build_plans(gamma)


    @_solver_stream
    def set_charge_levels_stats(self, y0d, n: int, y_hi: float, y_lo: float, y_sum: float,
                                descending: bool = False, gamma_view=None) -> None:
        """set_charge_levels for a device slice of charge levels whose (global) count / max /
        min / sum the caller already has (ChargingStation computes every partition's in one pass
        per step, charging_station.py:187-266): no host sync, no collective.  ``descending``: y0d
        is already in descending order (gamma ascending), so the loop plan needs no sort.
        ``gamma_view``: the plan's batch prebuilt by the caller (_build_plans' ``prebuilt``)."""
        if not (n > 0 and 0.0 <= y_lo <= y_hi <= self.consts.y_max):
            raise AssertionError("0 <= y0 <= y_max required (price_solver.py:71)")
        self.y0 = y0d
        self.nEVs = int(n)
        self._y_hi, self._y_lo = float(y_hi), float(y_lo)
        self.y0_rng = (y_hi - y_lo) / 2  # = \bar{\Gamma}
        self.gamma_sc = self.consts.y_max - (y_hi + y_lo) / 2
        self.gamma_sm = self.consts.y_max - y_sum / n
        if gamma_view is not None:
            self._build_plans(None, presorted=True, prebuilt=gamma_view)
        else:
            self._build_plans(self.consts.y_max - y0d, presorted=descending)

    def _device_comm(self):
        """The extension's RCCL communicator of the group (None: single rank, gloo, DIRECT mode)."""
        if self.group is None or self.lompc.mode == "direct":
            return None
        from .dist import device_comm

        return device_comm(self.group, self.lompc.device)

    def _native_ok(self) -> bool:
        """The whole loop in C++: a PATH plan, single rank or combined on the device."""
        p = self._plan
        return (self.native_loop and p is not None and not p.direct
                and (self.group is None or p.comm is not None))

    def _global_levels(self, y0d):
        """Global max / min / mean / count of a sharded y0: one all-gather, one host sync."""
        from .dist import global_levels

        y_hi, y_lo, y_mean, n, bad = global_levels(y0d, self.consts.y_max, self.group)
        assert bad == 0  # price_solver.py:71 (0 <= y0 <= y_max on every rank)
        self.nEVs = n
        return y_hi, y_lo, y_mean

    _PART_STATE = ("y0", "nEVs", "_y_hi", "_y_lo", "y0_rng", "gamma_sc", "gamma_sm", "_gam", "_gam_w0", "_gcentral",
                   "_plan", "_B")

    @_solver_stream
    def stage_partition(self, p: int, y0d, n: int, y_hi: float, y_lo: float, y_sum: float,
                        descending: bool = False, gamma_view=None) -> None:
        """set_charge_levels_stats for partition p ahead of its price loop: the partition's own
        loop plan is (re)prepared now, on the solver's stream, and kept with its levels until
        use_partition(p).  ChargingStation stages every partition of a step before the BiMPC
        solve, so the plans' device preparation overlaps the host interior point instead of
        sitting in front of each partition's loop (every partition keeps its own warm start)."""
        cur = {k: getattr(self, k, None) for k in self._PART_STATE}
        st = self._staged.get(p)
        if st is not None:  # the partition's plan from the previous step: re-targeted
            for k in self._PART_STATE:
                setattr(self, k, st[k])
        else:
            self._plan = None
        try:
            self.set_charge_levels_stats(y0d, n, y_hi, y_lo, y_sum, descending=descending, gamma_view=gamma_view)
            self._staged[p] = {k: getattr(self, k) for k in self._PART_STATE}
        finally:
            for k in self._PART_STATE:
                setattr(self, k, cur[k])

    def prewarm_partitions(self, parts) -> None:
        """Create the loop plan of every partition in ``parts`` now (ChargingStation: at
        construction), on a one-EV placeholder batch: with ``reserve_evs`` its workspaces are sized
        for the whole population at once, so the steps' staging re-targets plans
        (lompc_plan_update) and allocates nothing.  A placeholder plan has never run: its first
        staging and loop are those of a fresh plan (``tests/test_gpu_pipeline.py``: update = fresh)."""
        torch = _torch()
        y = torch.full((1,), 0.5 * float(self.consts.y_max), dtype=torch.float64, device=self._dev)
        v = 0.5 * float(self.consts.y_max)
        for p in parts:
            if p not in self._staged:
                self.stage_partition(p, y, 1, v, v, v, descending=True)

    def use_partition(self, p: int) -> None:
        """Make the plan and levels staged for partition p current (set_charge_levels done)."""
        for k, v in self._staged[p].items():
            setattr(self, k, v)
        self._w0_live = False

    def _build_plans(self, gamma, presorted: bool = False, prebuilt=None) -> None:
        """Batch layout of one price iteration: set 0 = this rank's EVs, set 1 = the central QP.
        The loop plan holds set 0's gamma in ascending order (LOMPC_PLAN_SORTED_GAMMA: its runs
        aggregate per certified piece, O(pieces) per iteration; only the per-set sums leave the
        loop, price_solver.py:196-214, so the EV order does not matter there); the w0 plan keeps
        the caller's order (get_w0_price0 returns w0 per EV).  ``prebuilt``: that batch already
        laid out by the caller — a contiguous device view [gamma ascending | gamma_sc (rank 0)]
        (ChargingStation builds every partition's in one pass per type and step)."""
        torch = _torch()
        central = 1 if self._rank() == 0 else 0
        if prebuilt is not None:
            B = int(prebuilt.numel()) - central
            self._gam = prebuilt
            self._gam_w0 = prebuilt[:B]
            self._gcentral = None if not central else prebuilt[B:]
        else:
            B = int(gamma.numel())
            gamma = gamma.reshape(-1).to(dtype=torch.float64).contiguous()
            self._gam = torch.empty(B + central, dtype=torch.float64, device=self._dev)
            self._gam[:B] = gamma if presorted else torch.sort(gamma).values
            self._gam_w0 = gamma
            self._gcentral = None if not central else self._gam[B:]
            if central:
                self._gam[B] = float(self.gamma_sc)
        off = np.array([0, B, B + central], dtype=np.int64)
        # gamma = y_max - y0 with 0 <= y0 <= y_max asserted in set_charge_levels.  The price
        # iterations change the prices a little at a time: each gamma cell's exact solve starts
        # from the working set the previous iteration ended with there.  The plans are built once
        # and re-targeted at every partition (lompc_plan_update: no allocation, no device sync).
        if self._plan is None:
            self._plan = BatchPlan(self.lompc, self._gam, off, w_ref=self._wr2, want_w=False, want_cost=False,
                                   want_set=True, validate=False, warm_start=True,
                                   sorted_gamma=self.lompc.mode != "direct", cells=self.loop_cells)
            if self.reserve_evs:  # (its later partitions' batches: no reallocation, lompc_plan_reserve)
                self._plan.reserve(self.reserve_evs + central)
            comm = self._device_comm()
            if comm is not None:
                self._plan.set_comm(comm)
        else:
            self._plan.update(self._gam, off, w_ref=self._wr2, validate=False)
        self._w0_live = False  # the w0 plan follows lazily (get_w0_price0_device)
        self._B = B


    @_solver_stream
    def compute_optimal_prices(self, w_ref: np.ndarray, lmbd_r: float) -> tuple[np.ndarray, dict]:
        """
        Inputs:
            w_ref:  Reference w vector (team-optimal solution) from the BiMPC.
            lmbd_r: Robustness price parameter.
        Outputs:
            lmbd:           Optimal unit price (incentive) vector.
            solver_stats:   Additional solver info (price_solver.py:90-95).
        """
        PRINT_LEVEL = _settings.PRINT_LEVEL
        w_ref = np.asarray(w_ref, dtype=np.float64)
        # Convergence tolerance.
        tol, w0_err_bound = self.get_robustness_bounds(lmbd_r)
        # w-inner product metric.
        A_bar, A_bar_inv = self._get_w_inner_product_metric(lmbd_r)

        # Initialize price iterate from previous prices.
        lmbd_k, lmbd_k_new = np.zeros((3 * self.N)), np.zeros((3 * self.N))
        lmbd_k[: self.r] = self.prev_prices
        if PRINT_LEVEL < 2 and self._native_ok():  # the whole loop in one C-ABI call
            if not self.profile_loops:
                return self._finish_prices(*self._native_loop(lmbd_k, lmbd_r, w_ref, A_bar, tol), lmbd_r, w_ref,
                                           A_bar, tol, w0_err_bound)
            t0 = time.perf_counter()
            res = self._native_loop(lmbd_k, lmbd_r, w_ref, A_bar, tol)
            t1 = time.perf_counter()
            out = self._finish_prices(*res, lmbd_r, w_ref, A_bar, tol, w0_err_bound)
            self.loop_host_ms["native_loop"] += (t1 - t0) * 1e3
            self.loop_host_ms["finish_prices"] += (time.perf_counter() - t1) * 1e3
            return out
        phi_w_ref = self.lompc.phi(w_ref)
        # one engine call: the batch error at lmbd_k and the central solve (price_solver.py:106)
        errs, (w_k, dual_cost) = self._iterate(lmbd_k, lmbd_r, w_ref, A_bar)
        dual_cost_decrease_ac = []
        dual_cost_decrease_pred = []
        # Gradient descent till convergence (price_solver.py:111-140):
        for iter in range(_settings.MAX_PRICE_SOLVER_ITERATIONS):
            w_err_max, _, w_avg_err = errs
            if PRINT_LEVEL >= 2:
                print(
                    f"Iteration     : {iter:4d} || Error (max): {w_err_max:13.8f} | Tolerance: {tol:13.8f} "
                    f"|| Error (avg): {w_avg_err:13.8f} | Tolerance: {tol:13.8f}",
                    end="\r",
                )
                if iter % 10 == 0:
                    print("")
            if _settings.PRICE_SOLVER_TOL_TYPE == "max":
                w_err = w_err_max
            else:
                w_err = w_avg_err
            if w_err <= tol:
                if (PRINT_LEVEL >= 2) and not (iter % 10 == 0):
                    print("")
                break
            lmbd_k_new[: self.r], dual_cost_derease = self._price_gradient_descent_step(
                A_bar_inv, w_ref, w_k, lmbd_k[: self.r]
            )
            # one engine call: central solve at lmbd_k_new (:132) + next iteration's batch error
            errs, (w_k, dual_cost_new) = self._iterate(lmbd_k_new, lmbd_r, w_ref, A_bar)
            dual_cost_decrease_ac.append(
                dual_cost_new - dual_cost + (lmbd_k - lmbd_k_new) @ phi_w_ref
            )
            dual_cost_decrease_pred.append(dual_cost_derease)
            dual_cost = dual_cost_new
            lmbd_k = lmbd_k_new
        return self._finish_prices(lmbd_k, w_k, iter, dual_cost_decrease_ac, dual_cost_decrease_pred, lmbd_r, w_ref,
                                   A_bar, tol, w0_err_bound)

    def chain_ok(self, parts) -> bool:
        """compute_optimal_prices_chain applies: PRINT_LEVEL 0 (nothing printed per partition), one
        rank, the native loop on (not profiling it), every staged partition's plan a PATH plan."""
        if _settings.PRINT_LEVEL >= 1 or not self.native_loop or self.group is not None:
            return False
        return all(p in self._staged and self._staged[p]["_plan"] is not None and not self._staged[p]["_plan"].direct
                   for p in parts)

    def compute_optimal_prices_chain(self, parts, w_refs, lmbd_r: float):
        """compute_optimal_prices for the staged partitions ``parts`` in order, each starting from
        the previous one's prices (charging_station.py:275-307 with price_solver.py:79-174), in ONE
        native call (lompc_price_chain): no Python between the partitions' loops.  w_refs: (len(parts),
        N).  Returns [(lmbd (3N,), solver_stats)] per part, as compute_optimal_prices would; the
        solver's prev_prices end as the last part's."""
        MAX = _settings.MAX_PRICE_SOLVER_ITERATIONS
        N, r = self.N, self.r
        n = len(parts)
        if n == 0:
            return []
        A_bar, A_bar_inv = self._get_w_inner_product_metric(lmbd_r)
        A_bar = np.ascontiguousarray(A_bar, dtype=np.float64)
        w_refs = np.ascontiguousarray(np.asarray(w_refs, dtype=np.float64).reshape(n, N))
        lm = np.zeros((n, 3 * N))
        wk = np.zeros((n, N))
        dec = np.zeros((n, 2, MAX))
        arr = (_lib.PriceChainPart * n)()
        for k, p in enumerate(parts):
            st = self._staged[p]
            plan = st["_plan"]
            plan._usable()
            tol = np.sqrt(self.N) * st["y0_rng"] + self.eps_tol  # get_robustness_bounds (price_solver.py:182-186)
            q = arr[k]
            q.plan = plan._plan.value
            q.n_evs, q.tol = float(st["nEVs"]), float(tol)
            q.w_ref = w_refs[k].ctypes.data
            q.dev_sw, q.dev_st = plan.out["set_sum_w"].data_ptr(), plan.out["set_stats"].data_ptr()
            q.lmbd, q.w_k = lm[k].ctypes.data, wk[k].ctypes.data
            q.dec_actual, q.dec_pred = dec[k, 0].ctypes.data, dec[k, 1].ctypes.data
        args = _lib.PriceLoopArgs(
            N, r, MAX, 1 if _settings.PRICE_SOLVER_TOL_TYPE != "max" else 0, float(self.consts.theta),
            float(self.consts.w_max), float(self.m), float(self._kappa_of(A_bar_inv)), float(self.eps_reg), 0.0, 0.0,
            float(lmbd_r), A_bar.ctypes.data, None, self._in.data_ptr(), self._h_in.data_ptr(), None, None,
            self._h_sw.data_ptr(), self._h_st.data_ptr(), self.loop_prof.ctypes.data if self.profile_loops else None,
            1 if self.device_loop else 0)
        prev = np.ascontiguousarray(self.prev_prices, dtype=np.float64).copy()
        t0 = time.perf_counter()
        rc = self._lib.lompc_price_chain(n, ctypes.cast(arr, ctypes.c_void_p), ctypes.byref(args), prev.ctypes.data,
                                         self._stream.cuda_stream)
        if self.profile_loops:
            self.loop_host_ms["native_loop"] += (time.perf_counter() - t0) * 1e3
        self.n_batched_calls += sum(int(arr[k].calls) for k in range(n))
        if rc != _lib.LOMPC_OK:
            k = next((k for k in range(n) if arr[k].rc), n - 1)
            text = self._lib.lompc_plan_last_error(arr[k].plan).decode(errors="replace")
            if rc == _lib.LOMPC_ERR_NOT_CONVERGED:
                raise SolverError(text)
            if "gamma" in text:
                raise AssertionError(text)
            raise ValueError(text or _lib.status_text(self._lib, None, rc))
        self.prev_prices = prev
        out = []
        for k in range(n):
            q = arr[k]
            m = q.calls - 1  # (decreases recorded: one per step taken)
            out.append((lm[k], {"iter": int(q.iterations), "price_before_reg": float(q.price_before_reg),
                                "price_after_reg": float(q.price_after_reg),
                                "dual_cost_decrease_actual": dec[k, 0, :m].copy(),
                                "dual_cost_decrease_predicted": dec[k, 1, :m].copy()}))
        return out

    def _native_loop(self, lmbd_k, lmbd_r, w_ref, A_bar, tol):
        """price_solver.py:106-140 in ONE call (lompc_price_loop): plan runs, copies, syncs and
        price steps stay in C++ until convergence."""
        if self._plan is None:
            raise RuntimeError("set_charge_levels first")
        self._plan._usable()  # (a closed communicator: raise instead of a collective on freed memory)
        MAX = _settings.MAX_PRICE_SOLVER_ITERATIONS
        A_bar = np.ascontiguousarray(A_bar, dtype=np.float64)
        w_ref = np.ascontiguousarray(w_ref, dtype=np.float64)
        args = _lib.PriceLoopArgs(
            self.N, self.r, MAX, 1 if _settings.PRICE_SOLVER_TOL_TYPE != "max" else 0, float(self.consts.theta),
            float(self.consts.w_max), float(self.m), float(self._kappa_of(self._A_bar_inv)), float(self.eps_reg),
            float(tol), float(self.nEVs), float(lmbd_r), A_bar.ctypes.data, w_ref.ctypes.data, self._in.data_ptr(),
            self._h_in.data_ptr(), self._plan.out["set_sum_w"].data_ptr(), self._plan.out["set_stats"].data_ptr(),
            self._h_sw.data_ptr(), self._h_st.data_ptr(), self.loop_prof.ctypes.data if self.profile_loops else None,
            1 if self.device_loop else 0)
        lm = np.ascontiguousarray(lmbd_k, dtype=np.float64).copy()
        w_k = np.empty(self.N)
        dec_ac, dec_pred = np.empty(MAX), np.empty(MAX)
        dual_cost, it = ctypes.c_double(0.0), ctypes.c_int(0)
        errs = np.empty(3)
        rc = self._lib.lompc_price_loop(self._plan._plan, ctypes.byref(args), lm.ctypes.data, w_k.ctypes.data,
                                        ctypes.byref(dual_cost), dec_ac.ctypes.data, dec_pred.ctypes.data,
                                        ctypes.byref(it), errs.ctypes.data, self._plan._stream)
        if rc != _lib.LOMPC_OK:
            text = self._lib.lompc_plan_last_error(self._plan._plan).decode(errors="replace")
            if rc == _lib.LOMPC_ERR_NOT_CONVERGED:
                raise SolverError(text)
            if "gamma" in text:
                raise AssertionError(text)
            raise ValueError(text)
        n = it.value
        self.n_batched_calls += n + 1
        return lm, w_k, min(n, MAX - 1), list(dec_ac[:n]), list(dec_pred[:n])

    def _finish_prices(self, lmbd_k, w_k, iter, dual_cost_decrease_ac, dual_cost_decrease_pred, lmbd_r, w_ref,
                       A_bar, tol, w0_err_bound):
        PRINT_LEVEL = _settings.PRINT_LEVEL
        # Regularize prices (price_solver.py:145-147): the native routine the chain uses too
        # (lompc_price_regularize: the same LP as _regularize_prices, the same bits as the chain)
        lmbd_k = np.ascontiguousarray(lmbd_k, dtype=np.float64)
        w_k = np.ascontiguousarray(w_k, dtype=np.float64)
        pre, post = ctypes.c_double(0.0), ctypes.c_double(0.0)
        rc = self._lib.lompc_price_regularize(self.N, self.r, float(self.consts.theta), float(self.consts.w_max),
                                              w_k.ctypes.data, lmbd_k.ctypes.data, ctypes.byref(pre),
                                              ctypes.byref(post))
        if rc != _lib.LOMPC_OK:
            raise PriceRegularizerError("LP infeasible: " + _lib.status_text(self._lib, None, rc))
        price_pre, price_new = pre.value, post.value
        if PRINT_LEVEL >= 1:
            (w_err_max, w0_err, w_avg_err), (w_k_, _) = self._iterate(lmbd_k, lmbd_r, w_ref, A_bar)
            if PRINT_LEVEL >= 2:
                print(f"Regularization: Price  : {price_pre:9.3f} -> {price_new:9.3f}")
                print(f"                w-error: {np.linalg.norm(w_k - w_k_):13.8f}")
                print(f"w-error (max) : {w_err_max:13.8f} | Tolerance     : {tol:13.8f}")
                print(f"w-error (avg) : {w_avg_err:13.8f} | Tolerance     : {tol:13.8f}")
            if self._rank() == 0:
                print(f"w0-error      : {w0_err:13.8f} | w0 error bound: {w0_err_bound:13.8f}")
        # Update previous prices.
        self.prev_prices = lmbd_k[: self.r]
        solver_stats = {
            "iter": iter,
            "price_before_reg": price_pre,
            "price_after_reg": price_new,
            "dual_cost_decrease_actual": np.array(dual_cost_decrease_ac),
            "dual_cost_decrease_predicted": np.array(dual_cost_decrease_pred),
        }
        return lmbd_k, solver_stats

    def get_gamma_sc(self) -> float:
        return self.gamma_sc

    def get_gamma_sm(self) -> float:
        return self.gamma_sm

    def get_robustness_bounds(self, lmbd_r: float) -> tuple[float, float]:
        """price_solver.py:182-186."""
        kappa = lmbd_r / self.consts.delta + 1e-5
        w_err_bound = np.sqrt(self.N) * self.y0_rng + self.eps_tol
        w0_err_bound = w_err_bound * np.min((1, 1 / np.sqrt(kappa)))
        return w_err_bound, w0_err_bound

    def _get_w_inner_product_metric(self, lmbd_r: float) -> tuple[np.ndarray, np.ndarray]:
        """price_solver.py:188-194."""
        kappa = lmbd_r / self.consts.delta
        if self._kappa == kappa and self._A_bar_inv is not None:  # every partition of a step: same metric
            return self._A_bar, self._A_bar_inv
        A_bar = self.A.T @ self.A + kappa * np.eye(self.N)
        A_bar_inv = np.linalg.inv(A_bar)
        self._A_bar, self._A_bar_inv, self._kappa = A_bar, A_bar_inv, kappa
        return A_bar, A_bar_inv

    # ------------------------------------------------------------ engine calls
    def _iterate(self, lmbd: np.ndarray, lmbd_r: float, w_ref: np.ndarray, A_bar: np.ndarray):
        """ONE batched call at prices lmbd: returns
        ((w_err_max, w0_err, w_avg_err) of price_solver.py:196-214, (w_central, cost_central))."""
        torch = _torch()
        if self._plan is None:
            raise RuntimeError("set_charge_levels first")
        N3 = 3 * self.N
        h = self._h_in_np  # free: the previous call synchronised after its copy
        h[:N3] = lmbd
        h[N3:2 * N3] = lmbd
        h[2 * N3:2 * N3 + 2] = float(lmbd_r)
        h[2 * N3 + 2:2 * N3 + 2 + self.N] = w_ref
        h[2 * N3 + 2 + self.N:] = w_ref
        self._in.copy_(self._h_in, non_blocking=True)
        out = self._plan.run(self._lm2, self._lr2)
        self.n_batched_calls += 1
        sw, st = out["set_sum_w"], out["set_stats"]
        if self.group is not None and self._plan.comm is None:  # (with a comm: combined by the run)
            from .dist import allreduce_set_results

            allreduce_set_results(sw, st, group=self.group)
        self._h_sw.copy_(sw, non_blocking=True)
        self._h_st.copy_(st, non_blocking=True)
        self._stream.synchronize()
        sw, st = self._h_sw.numpy(), self._h_st.numpy()
        self._check_stats(st)
        # price_solver.py:210-214 from the fused sums
        w_avg = sw[0] / self.nEVs
        w_avg_err = np.sqrt((w_avg - w_ref) @ A_bar @ (w_avg - w_ref))
        w0_err = np.abs(w_avg[0] - w_ref[0])
        w_err_max = float(st[0, _lib.LOMPC_STAT_MAX_ERR])
        w_c = sw[1].copy()
        return (w_err_max, w0_err, w_avg_err), (w_c, float(st[1, _lib.LOMPC_STAT_SUM_COST]))

    @staticmethod
    def _check_stats(st: np.ndarray) -> None:
        if np.any(st[:, _lib.LOMPC_STAT_N_INVALID] > 0):
            raise AssertionError("gamma outside [0, y_max]")
        if np.any(st[:, _lib.LOMPC_STAT_N_FAILED] > 0):
            raise SolverError("LoMPC QPs without a certified optimum")


    @_solver_stream
    def _get_w_err(self, lmbd: np.ndarray, lmbd_r: float, w_ref: np.ndarray,
                   A_bar: np.ndarray) -> tuple[float, float, float]:
        """price_solver.py:196-214: (w_err_max, w0_err, w_avg_err) with the per-EV loop batched."""
        kappa = lmbd_r / self.consts.delta
        if not np.allclose(A_bar, self.A.T @ self.A + kappa * np.eye(self.N), rtol=1e-12, atol=1e-12):
            raise ValueError("A_bar must be A'A + (lmbd_r/delta) I (price_solver.py:191-192)")
        errs, _ = self._iterate(np.asarray(lmbd, dtype=np.float64), lmbd_r, np.asarray(w_ref, dtype=np.float64),
                                A_bar)
        return errs

    def _kappa_of(self, A_bar_inv: np.ndarray) -> float:
        if A_bar_inv is self._A_bar_inv:
            return self._kappa
        A_bar = np.linalg.inv(A_bar_inv)
        kappa = A_bar[-1, -1] - 1.0
        if not np.allclose(A_bar, self.A.T @ self.A + kappa * np.eye(self.N), rtol=1e-9, atol=1e-9):
            raise ValueError("A_bar_inv must be (A'A + kappa I)^-1 (price_solver.py:191-193)")
        return max(kappa, 0.0)

    def _price_gradient_descent_step(self, A_bar_inv: np.ndarray, w_ref: np.ndarray, w: np.ndarray,
                                     lmbd: np.ndarray) -> tuple[np.ndarray, float]:
        """price_solver.py:216-246 -> (lmbd_next, dual_cost_decrease), exact on the host."""
        w_ref = np.ascontiguousarray(w_ref, dtype=np.float64)
        w = np.ascontiguousarray(w, dtype=np.float64)
        lm = np.ascontiguousarray(lmbd, dtype=np.float64)
        if w.shape != (self.N,) or w_ref.shape != (self.N,) or lm.shape != (self.r,):
            raise ValueError("price step: w, w_ref (N,) and lmbd (r,) required")
        out = np.empty(self.r)
        dec = ctypes.c_double(0.0)
        iters = ctypes.c_int(0)
        rc = self._lib.lompc_price_step(self.N, self.r, float(self.consts.theta), float(self.consts.w_max),
                                        float(self.m), float(self._kappa_of(A_bar_inv)), float(self.eps_reg),
                                        w_ref.ctypes.data, w.ctypes.data, lm.ctypes.data, out.ctypes.data,
                                        ctypes.byref(dec), ctypes.byref(iters))
        if rc == _lib.LOMPC_ERR_NOT_CONVERGED:
            raise SolverError("price-gradient QP: no certified optimum")
        if rc != _lib.LOMPC_OK:
            raise ValueError(_lib.status_text(self._lib, None, rc))
        self.last_step_iterations = iters.value
        return out, dec.value

    def _regularize_prices(self, w: np.ndarray, lmbd: np.ndarray) -> np.ndarray:
        """price_solver.py:248-255."""
        phi = self.lompc.phi(w)[: self.r]
        Dphi = self.lompc.Dphi(w)[: self.r, :]
        lmbd_reg = self.price_reg.solve_price_regularization(Dphi.T, Dphi.T @ lmbd, phi)
        return lmbd_reg

    def get_w0_price0(self, lmbd: np.ndarray, lmbd_r: float) -> tuple[np.ndarray, float]:
        """price_solver.py:272-285 as one batched solve: (w0 of this rank's EVs, mean price0)."""
        w0, price0_sum = self.get_w0_price0_device(lmbd, lmbd_r)
        return (w0.cpu().numpy() if w0 is not None else np.zeros(0)), price0_sum / self.nEVs


    @_solver_stream
    def get_w0_price0_device(self, lmbd: np.ndarray, lmbd_r: float):
        """(w0 device tensor of this rank's EVs, global sum of price0) — no host copy of w0."""
        torch = _torch()
        N3 = 3 * self.N
        h = self._h_in_np
        h[:N3] = 0.0
        h[: self.r] = lmbd
        h[2 * N3:2 * N3 + 2] = float(lmbd_r)
        self._in.copy_(self._h_in, non_blocking=True)
        B = self._B
        if B and not self._w0_live:
            if self._plan_w0 is None:
                self._plan_w0 = BatchPlan(self.lompc, self._gam_w0, np.array([0, B], dtype=np.int64), want_w=False,
                                          want_cost=False, want_w0=True, want_set=True, validate=False)
            else:
                self._plan_w0.update(self._gam_w0, np.array([0, B], dtype=np.int64), validate=False)
            self._w0_live = True
        if B:
            out = self._plan_w0.run(self._lm2[:1], self._lr2[:1])
            st = out["set_stats"]
            w0 = out["w0"]
        else:
            st = torch.zeros((1, _lib.LOMPC_SET_STATS), dtype=torch.float64, device=self._dev)
            w0 = None
        if self.group is not None:
            import torch.distributed as dist

            st = st.clone()
            dist.all_reduce(st, op=dist.ReduceOp.SUM, group=self.group)
        st = st.cpu().numpy()
        self._check_stats(st)
        return w0, float(st[0, _lib.LOMPC_STAT_SUM_PRICE0])
