"""CVXPY-free ``ChargingStation`` (chargingstation/charging_station.py:15-433): the closed-loop
BiMPC step on the batched engine.

Same constants dataclass, constructor checks, ``simulate() -> logs`` and logs schema
(charging_station.py:118-149) as the reference.  What runs where:

* EV state (SoCs ``y_s``/``y_l``, partition index) lives on the device (torch fp64);
  the full-charge re-draws come from the reference's legacy global ``np.random``
  stream in EV-index order (charging_station.py:95-100, :339-341, :348-350), drawn
  on the host and scattered, so a seeded run draws the same numbers.
* partition statistics (count, min, max, mean per partition; charging_station.py:196-210
  via price_solver.py:66-77, :182-186) are one device reduction per EV type;
* the BiMPC (bimpc.py) is the host interior point of ``lompc_bimpc_solve``;
* each (type, partition) price loop is ``PriceSolver.compute_optimal_prices`` (one
  engine call per price iteration), in the reference's sequential order because
  ``prev_prices`` chains the partitions (charging_station.py:275-307);
* ``_get_w0_price0`` (charging_station.py:310-329) is ONE batched engine call per EV
  type over all partitions (the prices are fixed by then), with fused price0 sums.

Sharded mode (``group``): every rank holds a contiguous slice of each type's EVs (the per-EV
state, the w0 / price0 pass and the state update are sharded).  Default ``sharded_loops =
"replicated"``: ONE all-gather of both types' charge levels per step gives every rank the whole
population, from which every rank builds the same partition statistics and layouts and runs every
(type, partition) price loop itself (k_agg is O(pieces): a loop costs the same whatever the EV
count, so replicating it costs nothing, and no collective runs inside a loop — ~600 per step with
one per price iteration); the w0 / price0 pass runs on this rank's EVs, and its per-partition sums
(the aggregate demand, charging_station.py:356-366) are combined by ONE all-reduce; the state
update's residual sum and global redraw counts are the step's remaining exchanges.  The first
step's prices, iterations and statistics are then bit for bit the single process's; later steps
differ only through the w0 sums' order (and the per-rank plans' gamma windows) at rounding level.
``sharded_loops = "exchange"``: every price iteration all-gathers the per-rank set reductions
(the round-4/5 form, kept for A/B).  The BiMPC and the price steps run redundantly on identical
inputs; the re-draw replays the global random stream.
"""
from __future__ import annotations

import concurrent.futures
import ctypes
import time

from dataclasses import dataclass

import numpy as np

from . import _lib
from . import settings as _settings
from .bimpc import BiMPC, BiMPCConstants, BiMPCParameters
from .lompc import LoMPCConstants, SolverError
from .price_solver import PriceSolver
from .settings import ADD_RESIDUAL_CHARGE_TO_BATTERY, MAX_INITIAL_SOC, MIN_FULL_CHARGE_FRACTION, MIN_INITIAL_SOC


def _torch():
    import torch

    return torch


@dataclass
class ChargingStationConstants:
    """
    simulation_length:  Length of the simulation [hours].
    horizon_bimpc:      BiMPC horizon.
    horizon_lompc:      LoMPC horizon (<= BiMPC horizon).
    nEVs_per_EV_type:   Number of small (and large) EVs.
    npartitions:        Number of partitions per EV type.
    demand:             External demand vector.
    bimpc_consts:       Normalized constants for the BiMPC.
    small_EV_consts:    Constants for the small EV LoMPC.
    large_EV_consts:    Constants for the large EV LoMPC.
    price_type:         "linear" or "linear-convex".
    """

    simulation_length: int
    horizon_bimpc: int
    horizon_lompc: int
    nEVs_per_EV_type: int
    npartitions: int
    demand: np.ndarray
    bimpc_consts: BiMPCConstants
    small_EV_consts: LoMPCConstants
    large_EV_consts: LoMPCConstants
    price_type: str


# ----------------------------------------------------------------- sharded helpers
def shard_bounds(n: int, rank: int, world: int) -> tuple[int, int]:
    base, rem = divmod(n, world)
    lo = rank * base + min(rank, rem)
    return lo, lo + base + (1 if rank < rem else 0)


def partition_stats(y, idx, P: int, group=None) -> np.ndarray:
    """Per partition (count, max, min, sum) of y over the EVs with idx == p, combined over
    ranks (one all-gather of the per-rank records, reduced locally in rank order).  Returns a
    host (P, 4) array; empty partitions have count 0."""
    torch = _torch()
    # masked column reductions over an (n, P) view: P is small, and scatter/atomic forms
    # (bincount, index_add_, scatter_reduce) serialise n updates on P addresses
    onehot = idx.unsqueeze(1) == torch.arange(P, device=y.device).unsqueeze(0)
    yy = y.unsqueeze(1)
    cnt = onehot.sum(0).to(torch.float64)
    sm = torch.where(onehot, yy, 0.0).sum(0)
    mx = torch.where(onehot, yy, -float("inf")).amax(0)
    mn = torch.where(onehot, yy, float("inf")).amin(0)
    rec = torch.stack([cnt, mx, mn, sm], dim=1)
    if group is None:
        return rec.cpu().numpy()
    import torch.distributed as dist

    world = dist.get_world_size(group)
    out = torch.empty((world * P, 4), dtype=torch.float64, device=y.device)
    dist.all_gather_into_tensor(out, rec.contiguous(), group=group)
    rows = out.view(world, P, 4).cpu().numpy()  # the one host sync
    tot = rows[0].copy()
    for r in range(1, world):  # fixed rank order
        tot[:, 0] += rows[r, :, 0]
        tot[:, 3] += rows[r, :, 3]
    tot[:, 1] = rows[:, :, 1].max(axis=0)
    tot[:, 2] = rows[:, :, 2].min(axis=0)
    return tot


def redraw_full(y, mask, lo_val: float, hi_val: float, rng_random, group=None) -> int:
    """y[mask] = lo + (hi - lo) * rng_random(count) with the draws in GLOBAL EV-index order
    (charging_station.py:339-341): every rank draws the global vector from the same
    (replicated) stream and keeps its own slice.  Returns the global count."""
    torch = _torch()
    local = int(mask.sum().item())
    if group is None:
        total, before = local, 0
    else:
        import torch.distributed as dist

        world = dist.get_world_size(group)
        t = torch.tensor([local], dtype=torch.int64, device=y.device)
        allc = [torch.zeros_like(t) for _ in range(world)]
        dist.all_gather(allc, t, group=group)
        counts = [int(c.item()) for c in allc]
        total = sum(counts)
        before = sum(counts[: dist.get_rank(group)])
    draws = lo_val + (hi_val - lo_val) * rng_random((total,))
    if local:
        y[mask] = torch.as_tensor(draws[before:before + local], dtype=torch.float64, device=y.device)
    return total


class ChargingStation:
    def __init__(self, consts: ChargingStationConstants, device: int | None = None, mode: str | None = None,
                 group=None, sharded_loops: str = "replicated") -> None:
        # charging_station.py:44-53
        assert consts.simulation_length >= 1
        assert (consts.horizon_bimpc >= consts.horizon_lompc) and (consts.horizon_lompc >= 1)
        assert consts.nEVs_per_EV_type >= 1
        assert consts.npartitions >= 1
        assert (len(consts.demand.shape) == 1) and (
            consts.demand.shape[0] >= consts.simulation_length + consts.horizon_bimpc + 1)
        torch = _torch()
        self.group = group
        if sharded_loops not in ("replicated", "exchange"):
            raise ValueError("sharded_loops: 'replicated' or 'exchange'")
        # sharded with every price loop replicated on every rank (no collective inside a loop)
        self.replicated = group is not None and sharded_loops == "replicated"
        # sharded with one all-gather of the set reductions per price iteration
        self._exchange = group is not None and not self.replicated
        self._yfull = None  # replicated: this step's whole-population levels {kind: device tensor}
        self._idxfull = {}  # replicated, index path only: the whole population's partition indices
        self._layout_w0 = {}  # replicated: this rank's EVs in the loops' layout order, per type
        self._pool = None  # one worker thread: the large-EV price chain beside the small one
        self._stage_pool = None  # two worker threads: the partition plans staged beside the BiMPC solve
        self.profile_phases = False  # accumulate per-phase wall times of _step in phase_ms (synchronising)
        # every partition's loop plan of a step prepared beside the BiMPC solve (False: each partition's
        # plan prepared when its loop starts — for A/B timing)
        self.stage_partitions = True
        # the partitions' loop-plan batches laid out in one launch per type (False: per partition — A/B timing)
        self.gamma_layout = True
        self.phase_ms = {}
        self.last_step_ms = {}  # host time of the last step's phases (_tick)
        self.chain_ms = {}  # the last step's price chain per EV type (host time of its native call)
        self.stage_ms = {}  # the last step's staging thread per EV type (host time)
        self.bimpc_split = {}  # the last step's BiMPC phase split (_get_bimpc_solution)
        self._gl_host, self._gl_keep = {}, {}  # _gamma_layout's pinned run bounds per price solver
        # the w0 / price0 pass of both types in one engine run (False: one per type — A/B timing)
        self.w0_one_call = True
        self._w0plan, self._w0_host, self._w0_keep = None, None, None
        self.device = torch.cuda.current_device() if device is None else int(device)
        self._dev = f"cuda:{self.device}"
        # Set constants, initialize PriceSolvers and BiMPC.
        self._set_constants(consts)
        self.bimpc = BiMPC(self.N_bi, self.P, self.consts_bi, self.consts_s, self.consts_l)
        lgroup = group if self._exchange else None  # (replicated: every rank's loops see the whole population)
        self.price_solver_s = PriceSolver(self.N_lo, self.consts_s, self.price_type, device=self.device, mode=mode,
                                          group=lgroup)
        self.price_solver_l = PriceSolver(self.N_lo, self.consts_l, self.price_type, device=self.device, mode=mode,
                                          group=lgroup)
        # every partition's loop plan is sized for the whole population of its type at its first
        # growth (partitions gain and lose EVs step to step: no reallocation inside the later steps)
        for ps in (self.price_solver_s, self.price_solver_l):
            ps.reserve_evs = self.M_2
            if not self._exchange and self.stage_partitions:  # (the plans made now: no allocation in a step)
                ps.prewarm_partitions(range(self.P))
        # Initialize state variables = (EV SoCs, charge stored).
        self._init_states()
        # Initialize logs.
        self._init_logs(consts)

    def _set_constants(self, consts: ChargingStationConstants) -> None:
        # charging_station.py:67-92
        self.Tf = consts.simulation_length
        self.N_bi = consts.horizon_bimpc
        self.N_lo = consts.horizon_lompc
        self.M_2 = consts.nEVs_per_EV_type
        self.P = consts.npartitions
        self.demand = consts.demand
        self.consts_bi = consts.bimpc_consts
        self.consts_s = consts.small_EV_consts
        self.consts_l = consts.large_EV_consts
        self.price_type = consts.price_type
        if self.price_type == "linear":
            self.r = 2 * self.N_lo
        else:
            self.r = 3 * self.N_lo
        self.y0_min = MIN_INITIAL_SOC
        self.y0_max = MAX_INITIAL_SOC
        self.y0_s_rng = np.linspace(self.y0_min, self.consts_s.y_max, self.P + 1)
        self.y0_l_rng = np.linspace(self.y0_min, self.consts_l.y_max, self.P + 1)
        self.B = (self.consts_s.theta + self.consts_l.theta) * self.M_2
        if self.group is None:
            self._lo, self._hi = 0, self.M_2
        else:
            import torch.distributed as dist

            self._lo, self._hi = shard_bounds(self.M_2, dist.get_rank(self.group), dist.get_world_size(self.group))

    def _rank0(self) -> bool:
        if self.group is None:
            return True
        import torch.distributed as dist

        return dist.get_rank(self.group) == 0

    # ------------------------------------------------------------------ replicated sharding
    def _gather_levels(self) -> None:
        """Replicated sharding: both types' charge levels of every rank in ONE all-gather (each rank's
        contiguous slice, padded to the largest shard), concatenated in rank order — the whole
        population in EV-index order, exactly the single process's level vectors."""
        torch = _torch()
        import torch.distributed as dist

        world = dist.get_world_size(self.group)
        bounds = [shard_bounds(self.M_2, r, world) for r in range(world)]
        pad = max(b - a for a, b in bounds)
        n = self._hi - self._lo
        send = torch.zeros((2, pad), dtype=torch.float64, device=self._dev)
        send[0, :n] = self.y_s
        send[1, :n] = self.y_l
        recv = torch.empty(world * 2 * pad, dtype=torch.float64, device=self._dev)
        dist.all_gather_into_tensor(recv, send.reshape(-1), group=self.group)
        r = recv.view(world, 2, pad)
        self._yfull = {kind: torch.cat([r[k, t, : b - a] for k, (a, b) in enumerate(bounds)])
                       for t, kind in enumerate(("Small", "Large"))}

    def _gather_idx(self, kind):
        """Replicated sharding, index path only (a type whose levels left the partition range, so its
        EVs keep their previous partition index, charging_station.py:111-116): the whole population's
        partition indices of one type (every rank takes this path together: they all see the same
        levels)."""
        torch = _torch()
        import torch.distributed as dist

        world = dist.get_world_size(self.group)
        bounds = [shard_bounds(self.M_2, r, world) for r in range(world)]
        pad = max(b - a for a, b in bounds)
        idx = self.idx_s if kind == "Small" else self.idx_l
        send = torch.zeros(pad, dtype=torch.int64, device=self._dev)
        send[: idx.numel()] = idx
        recv = torch.empty(world * pad, dtype=torch.int64, device=self._dev)
        dist.all_gather_into_tensor(recv, send, group=self.group)
        r = recv.view(world, pad)
        return torch.cat([r[k, : b - a] for k, (a, b) in enumerate(bounds)])

    def _loop_levels(self, kind):
        """(levels, partition indices) the price loops' layout is built from: this rank's EVs, or with
        replicated sharding the whole population (indices None: gathered only if the index path is
        taken)."""
        if self.replicated:
            return self._yfull[kind], None
        return (self.y_s, self.idx_s) if kind == "Small" else (self.y_l, self.idx_l)

    def _w0_layout(self, kind, reader=None):
        """Replicated sharding: this rank's EVs of one type in the loops' layout order (each partition's
        run of the whole population's layout restricted to global indices [lo, hi): still in descending
        charge level), for the sharded w0 / price0 pass — (local permutation, levels, {p: (start, end)}),
        the run bounds in one host copy.  Made by the type's staging thread (beside the interior point)
        or on first use."""
        torch = _torch()
        got = self._layout_w0.get(kind)
        if got is not None:
            return got
        lo, hi, P = self._lo, self._hi, self.P
        perm, ys, seg = self._partition_layout(kind, *self._loop_levels(kind))
        m = (perm >= lo) & (perm < hi)
        order = sorted(range(P), key=lambda p: seg[p])
        c = torch.cumsum(m.to(torch.int64), 0)
        e = torch.as_tensor([seg[p][1] - 1 for p in order], dtype=torch.int64, device=m.device)
        nz = torch.nonzero_static(m, size=hi - lo).squeeze(1)
        lperm, lys = perm[nz] - lo, ys[nz]
        if reader is not None:  # (made on a staging stream, read on `reader`: the allocator keeps them)
            lperm.record_stream(reader)
            lys.record_stream(reader)
        cnt = torch.where(e >= 0, c[e.clamp(min=0)], 0).cpu().numpy()  # the one host sync
        seg_l, prev = {}, 0
        for k, p in enumerate(order):
            seg_l[p] = (prev, int(cnt[k]))
            prev = int(cnt[k])
        self._layout_w0[kind] = (lperm, lys, seg_l)
        return self._layout_w0[kind]

    def _w0_layouts(self):
        return {kind: self._w0_layout(kind) for kind in ("Small", "Large")}

    def _init_states(self) -> None:
        # charging_station.py:94-109 (global draws, this rank keeps its slice)
        torch = _torch()
        y_s = self.y0_min + (self.y0_max - self.y0_min) * np.random.random((self.M_2,))
        y_l = self.y0_min + (self.y0_max - self.y0_min) * np.random.random((self.M_2,))
        self.y_s = torch.as_tensor(y_s[self._lo:self._hi].copy(), device=self._dev)
        self.y_l = torch.as_tensor(y_l[self._lo:self._hi].copy(), device=self._dev)
        self.x = 0  # Storage battery SoC, normalized wrt B.
        self.t = 0
        self.ncharged_s = 0
        self.ncharged_l = 0
        n = self._hi - self._lo
        self._bounds = {}
        self._lv = {}  # lompc_levels_layout's buffers per EV type
        self.idx_s = torch.zeros((n,), dtype=torch.int64, device=self._dev)
        self.idx_l = torch.zeros((n,), dtype=torch.int64, device=self._dev)
        self._update_indices()

    def _update_indices(self) -> None:
        # charging_station.py:111-116: partition p takes the EVs with rng[p] <= y <= rng[p+1], later
        # partitions winning on shared edges, EVs outside [rng[0], rng[P]] keeping their index.  The
        # boundaries increase, so that is the last boundary <= y (one searchsorted, clamped for
        # y == rng[P]); no host sync, a fixed handful of launches instead of four per partition
        torch = _torch()
        for idx, y, rng in ((self.idx_s, self.y_s, self.y0_s_rng), (self.idx_l, self.y_l, self.y0_l_rng)):
            b = self._bounds.get(id(rng))
            if b is None:  # the boundaries on the device once (a per-call copy would sync)
                b = self._bounds[id(rng)] = torch.as_tensor(rng, dtype=y.dtype, device=y.device)
            p = (torch.searchsorted(b, y, right=True) - 1).clamp_(0, self.P - 1)
            idx.copy_(torch.where((y >= b[0]) & (y <= b[-1]), p, idx))
        self._layout = {}
        self._pending = {}  # (types whose statistics came without the sort: _partition_layout sorts them)
        self._yfull = None
        self._idxfull = {}
        self._layout_w0 = {}

    def _init_logs(self, consts: ChargingStationConstants) -> None:
        # charging_station.py:118-149
        self.logs = {}
        self.logs["constants"] = consts
        self.logs["inputs"] = {
            "w_s": np.zeros((self.P, self.Tf)),
            "w_l": np.zeros((self.P, self.Tf)),
            "w_hat_s": np.zeros((self.P, self.Tf)),
            "w_hat_l": np.zeros((self.P, self.Tf)),
            "u_g": np.zeros((self.Tf,)),
        }
        self.logs["states"] = {"x": np.zeros((self.Tf,))}
        self.logs["bounds"] = {"beta_s": np.zeros((self.P, self.Tf)), "beta_l": np.zeros((self.P, self.Tf))}
        self.logs["statistics"] = {
            "ncharged_s": 0,
            "ncharged_l": 0,
            "gamma_sm": np.zeros((self.P, self.Tf)),
            "gamma_lm": np.zeros((self.P, self.Tf)),
            "niter_s": np.zeros((self.P, self.Tf), dtype=int),
            "niter_l": np.zeros((self.P, self.Tf), dtype=int),
            "Mp_s": np.zeros((self.P, self.Tf), dtype=int),
            "Mp_l": np.zeros((self.P, self.Tf), dtype=int),
        }
        self.logs["prices"] = {
            "lmbd_r": np.zeros((self.Tf)),
            "avg_price_s": np.zeros((self.P, self.Tf)),
            "avg_price_l": np.zeros((self.P, self.Tf)),
            "price_red_s": np.zeros((self.P, self.Tf)),
            "price_red_l": np.zeros((self.P, self.Tf)),
        }

    def simulate(self) -> dict:
        for _ in range(self.Tf):
            self._step()
        return self.logs

    def _step(self):
        # charging_station.py:156-185
        PRINT_LEVEL = _settings.PRINT_LEVEL
        if PRINT_LEVEL >= 1 and self._rank0():
            print("-" * 50)
            print(f"Iteration {self.t}")
            print("-" * 50)
        lmbd_r = 0
        tick = self._tick()
        w_hat_s, w_hat_l, u_g, stats_bi = self._get_bimpc_solution(lmbd_r)
        tick("bimpc")
        prices_s, prices_l, stats_s, stats_l = self._get_optimal_prices(w_hat_s, w_hat_l, lmbd_r)
        tick("prices")
        w0_s, w0_l, price0_s, price0_l, w0_stats = self._get_w0_price0(prices_s, prices_l, lmbd_r)
        tick("w0_price0")
        nu = (w_hat_s, w_hat_l, u_g, w0_s, w0_l)
        stats = (stats_bi, stats_s, stats_l)
        price0 = (price0_s, price0_l)
        self._update_logs(lmbd_r, nu, stats, price0, w0_stats)
        self._update_state(w0_s, w0_l, u_g[0], w0_stats)
        tick("state")
        self.t += 1

    def _tick(self):
        """Phase timer of _step.  profile_phases: synchronises the device at each boundary and
        accumulates phase_ms.  Otherwise host timestamps only (no synchronisation; every phase but
        the BiMPC's ends in a host sync or a native call that waits for its loops, so the host time
        covers its device work): last_step_ms, per step."""
        if not self.profile_phases:
            marks = {}
            last = [time.perf_counter()]

            def mark(name):
                t = time.perf_counter()
                marks[name] = (t - last[0]) * 1e3
                last[0] = t

            self.last_step_ms = marks
            return mark
        torch = _torch()
        torch.cuda.synchronize(self.device)
        last = [time.perf_counter()]

        def tick(name):
            torch.cuda.synchronize(self.device)
            t = time.perf_counter()
            self.phase_ms[name] = self.phase_ms.get(name, 0.0) + (t - last[0]) * 1e3
            last[0] = t

        return tick

    # ------------------------------------------------------------------ BiMPC
    def _robustness(self, solver: PriceSolver, st_row, lmbd_r):
        """set_charge_levels + get_robustness_bounds + get_gamma_sm (price_solver.py:66-77,
        :182-186) from one row of partition statistics (count, max, min, sum)."""
        n, ymax, ymin, ysum = st_row
        y0_rng = (ymax - ymin) / 2
        kappa = lmbd_r / solver.consts.delta + 1e-5
        w_err_bound = np.sqrt(solver.N) * y0_rng + solver.eps_tol
        beta = w_err_bound * np.min((1, 1 / np.sqrt(kappa)))
        gamma_sm = solver.consts.y_max - ysum / n
        return beta, gamma_sm

    def _get_bimpc_solution(self, lmbd_r: float):
        # charging_station.py:187-266
        t_in = time.perf_counter()
        Mp_s, Mp_l = np.zeros((self.P,), dtype=int), np.zeros((self.P,), dtype=int)
        beta_s, beta_l = np.zeros((self.P,)), np.zeros((self.P,))
        gamma_sm, gamma_lm = np.zeros((self.P,)), np.zeros((self.P,))
        # one rank: each type's EVs sorted once by charge level, the partitions' statistics from that
        # order (both types in one host sync); the layout the price loops need comes with it
        if self.replicated:
            self._gather_levels()  # (the step's one exchange of levels: every rank then sees every EV)
        sl = self._sorted_layouts()

        def index_stats(kind):  # a type the sorted layout left out: the index path
            if self.replicated:
                self._idxfull[kind] = self._gather_idx(kind)  # (for _partition_layout too)
                return partition_stats(self._yfull[kind], self._idxfull[kind], self.P)
            y, idx = self._loop_levels(kind)
            return partition_stats(y, idx, self.P, self.group)

        st_s = sl["Small"] if sl and "Small" in sl else index_stats("Small")
        st_l = sl["Large"] if sl and "Large" in sl else index_stats("Large")
        for p in range(self.P):
            Mp_s[p] = int(st_s[p, 0])
            if Mp_s[p] > 0:
                assert st_s[p, 2] >= 0 and st_s[p, 1] <= self.consts_s.y_max  # price_solver.py:71
                beta_s[p], gamma_sm[p] = self._robustness(self.price_solver_s, st_s[p], lmbd_r)
            Mp_l[p] = int(st_l[p, 0])
            if Mp_l[p] > 0:
                assert st_l[p, 2] >= 0 and st_l[p, 1] <= self.consts_l.y_max
                beta_l[p], gamma_lm[p] = self._robustness(self.price_solver_l, st_l[p], lmbd_r)
        self._pstats = (st_s, st_l)
        self._staged = self.stage_partitions
        self.stage_ms = {}
        t_stage = time.perf_counter()
        staging = self._stage_partitions() if self._staged else []
        Mp_s_ = Mp_s / self.B
        Mp_l_ = Mp_l / self.B
        demand = self.demand[self.t: self.t + self.N_bi] / self.B
        bimpc_params = BiMPCParameters(Mp_s_, Mp_l_, beta_s, beta_l, gamma_sm, gamma_lm, self.x, demand)
        t_call = time.perf_counter()
        try:
            w_hat_s, w_hat_l, u_g = self.bimpc.solve_bimpc(bimpc_params)
        finally:
            t_wait = time.perf_counter()
            for f in staging:  # (the partition plans were staged beside the host interior point)
                f.result()
        t_out = time.perf_counter()
        # where the BiMPC phase's host time goes (bench.py's station attribution): the partition
        # statistics before the staging starts, the staging threads' submit, the solve call, and the
        # wait for staging the solve did not hide; stage_ms: each staging thread's own duration
        self.bimpc_split = {"stats_ms": (t_stage - t_in) * 1e3, "submit_ms": (t_call - t_stage) * 1e3,
                            "solve_call_ms": (t_wait - t_call) * 1e3, "stage_wait_ms": (t_out - t_wait) * 1e3,
                            "stage_thread_ms": dict(self.stage_ms)}
        stats_bi = {"Mp_s": Mp_s, "Mp_l": Mp_l, "beta_s": beta_s, "beta_l": beta_l, "gamma_sm": gamma_sm,
                    "gamma_lm": gamma_lm}
        if _settings.PRINT_LEVEL >= 1 and self._rank0():
            total_w0_hat = self.consts_s.theta * Mp_s_ @ w_hat_s[:, 0] + self.consts_l.theta * Mp_l_ @ w_hat_l[:, 0]
            u0_b_hat = u_g[0] - demand[0] - total_w0_hat
            u0_b_err = self.consts_s.theta * Mp_s_ @ beta_s + self.consts_l.theta * Mp_l_ @ beta_l
            x_hat = self.x + u0_b_hat
            print("EV distribution (small): " + " + ".join("{:4d}".format(n) for n in Mp_s)
                  + " = {:4d}".format(np.sum(Mp_s)))
            print("EV distribution (large): " + " + ".join("{:4d}".format(n) for n in Mp_l)
                  + " = {:4d}".format(np.sum(Mp_l)))
            print(f"Electricity generated  : {u_g[0]:13.8f} | Max: {self.consts_bi.u_g_max:13.8f}")
            print(f"Demand                 : {demand[0]:13.8f}")
            print(f"Predicted output (EVs) : {total_w0_hat:13.8f}")
            print(f"Predicted battery input: [{u0_b_hat - u0_b_err:8.5f}, {u0_b_hat + u0_b_err:8.5f}] "
                  f"| Max (mag): {self.consts_bi.u_b_max:8.5f}")
            print(f"Current battery state  : {self.x}")
            print(f"Predicted battery state: Min: 0 | [{x_hat - u0_b_err:8.5f}, {x_hat + u0_b_err:8.5f}] "
                  f"| Max: {self.consts_bi.x_max:8.5f}")
            if _settings.PRINT_LEVEL >= 2:
                print("")
        return w_hat_s, w_hat_l, u_g, stats_bi

    # ------------------------------------------------------------------ prices
    def _get_optimal_prices(self, w_hat_s, w_hat_l, lmbd_r: float):
        # charging_station.py:268-308.  Within one EV type the partitions are sequential
        # (prev_prices chains them); the two types are independent, so without printing (whose
        # order is the reference's interleaving) and on one rank their chains run side by side:
        # one host thread each (the price loops spend their time in C-ABI calls, outside the
        # GIL) on each solver's own stream.
        PRINT_LEVEL = _settings.PRINT_LEVEL
        self.chain_ms = {}
        w_hat_s_opt, w_hat_l_opt = w_hat_s[:, : self.N_lo], w_hat_l[:, : self.N_lo]
        prices_s, prices_l = np.zeros((self.P, self.r)), np.zeros((self.P, self.r))
        stats_s, stats_l = [], []
        st_s, st_l = self._pstats
        chains = (("Small", self.price_solver_s, *self._loop_levels("Small"), st_s, w_hat_s_opt, prices_s, stats_s),
                  ("Large", self.price_solver_l, *self._loop_levels("Large"), st_l, w_hat_l_opt, prices_l, stats_l))
        for kind, _, y, idx, *_ in chains:  # (on this thread: the layouts' host sync)
            self._partition_layout(kind, y, idx)

        prof = self.profile_phases

        def one(chain, p):
            kind, solver, y, idx, st, w_hat, prices, stats = chain
            if st[p, 0] > 0:
                t0 = time.perf_counter() if prof else 0.0
                if self._staged:
                    solver.use_partition(p)  # (staged before the BiMPC solve, _stage_partitions)
                else:
                    ys, (a, b) = self._part_slice(kind, y, idx, p)
                    solver.set_charge_levels_stats(ys[a:b], st[p, 0], st[p, 1], st[p, 2], st[p, 3], descending=True)
                if PRINT_LEVEL >= 1 and self._rank0():
                    print(f"{kind} EVs, partition {p:2d}: ", end="")
                    if PRINT_LEVEL >= 2:
                        print("\n" + "-" * 27)
                t1 = time.perf_counter() if prof else 0.0
                lmbd_, stats_ = solver.compute_optimal_prices(w_hat[p, :], lmbd_r)
                if prof:
                    t2 = time.perf_counter()
                    acc = self.phase_ms
                    acc[f"prices/{kind}/levels"] = acc.get(f"prices/{kind}/levels", 0.0) + (t1 - t0) * 1e3
                    acc[f"prices/{kind}/optimal_prices"] = acc.get(f"prices/{kind}/optimal_prices", 0.0) + (t2 - t1) * 1e3
                prices[p, :] = lmbd_[: self.r]
                stats.append(stats_)
                if PRINT_LEVEL >= 2:
                    print("")
            else:
                stats.append({})

        if PRINT_LEVEL == 0 and not self._exchange:
            torch = _torch()
            main = torch.cuda.current_stream(self.device)

            def run_chain(chain):
                kind, solver, _, _, st, w_hat, prices, stats = chain
                # the chain's thread works on its solver's stream (no waits through a shared one)
                with torch.cuda.device(self.device), torch.cuda.stream(solver._stream):
                    parts = [p for p in range(self.P) if st[p, 0] > 0]
                    if self._staged and solver.chain_ok(parts):
                        # every partition's loop and regularisation in ONE native call (no Python
                        # between the partitions: the other type's chain runs beside it)
                        t0 = time.perf_counter()
                        res = dict(zip(parts, solver.compute_optimal_prices_chain(parts, w_hat[parts, :], lmbd_r)))
                        self.chain_ms[kind] = (time.perf_counter() - t0) * 1e3
                        if prof:
                            key = f"prices/{kind}/optimal_prices"
                            self.phase_ms[key] = self.phase_ms.get(key, 0.0) + (time.perf_counter() - t0) * 1e3
                        for p in range(self.P):
                            if p in res:
                                prices[p, :] = res[p][0][: self.r]
                                stats.append(res[p][1])
                            else:
                                stats.append({})
                        return
                    for p in range(self.P):
                        one(chain, p)

            for chain in chains:
                chain[1]._stream.wait_stream(main)  # the layouts were made on the main stream
            if self._pool is None:
                self._pool = concurrent.futures.ThreadPoolExecutor(max_workers=1)
            fut = self._pool.submit(run_chain, chains[1])
            try:
                run_chain(chains[0])
            finally:
                # the large chain has finished (or failed) before anything is re-raised or the next
                # step reuses its plans and pinned buffers; the main stream then follows both chains
                try:
                    fut.result()
                finally:
                    for chain in chains:
                        main.wait_stream(chain[1]._stream)
        else:
            # sharded: the two chains in the reference's interleaved order on this thread — every
            # rank must issue the plans' device collectives in the same order.  Each loop's stream
            # first waits for the previous loop's (its last engine calls and their collectives may
            # still be queued), so no two collectives on the shared communicator run concurrently,
            # and the main stream waits for both before any torch.distributed collective follows
            torch = _torch()
            main = torch.cuda.current_stream(self.device)
            prev = main
            for p in range(self.P):
                for chain in chains:
                    chain[1]._stream.wait_stream(prev)
                    one(chain, p)
                    prev = chain[1]._stream
            for chain in chains:
                main.wait_stream(chain[1]._stream)
        return prices_s, prices_l, stats_s, stats_l

    def _stage_partitions(self):
        """Every partition's loop plan of this step, prepared (PriceSolver.stage_partition) on one
        host thread per EV type and on the price solvers' streams WHILE the main thread runs the
        BiMPC interior point (a C call without the GIL): the partitions' price loops then start at
        once.  The partitions' levels depend only on the state, not on the BiMPC.  Returns the
        futures (waited for after the solve).  Sharded: on this thread, in order (every rank
        creates its plans' device communicators in the same order)."""
        torch = _torch()
        st_s, st_l = self._pstats
        main = torch.cuda.current_stream(self.device)
        jobs = []
        for kind, solver, st in (("Small", self.price_solver_s, st_s), ("Large", self.price_solver_l, st_l)):
            solver._stream.wait_stream(main)  # (the state the layout sorts is the main stream's)
            jobs.append((kind, solver, *self._loop_levels(kind), st))

        def stage(job):
            kind, solver, y, idx, st = job
            t0 = time.perf_counter()
            try:
                stage_body(kind, solver, y, idx, st)
            finally:
                self.stage_ms[kind] = (time.perf_counter() - t0) * 1e3

        def stage_body(kind, solver, y, idx, st):
            with torch.cuda.device(self.device), torch.cuda.stream(solver._stream):
                # the type's partition layout too (its sorts and one host sync: on this thread, beside
                # the interior point, not before it); its tensors are read on the main stream later
                t0 = time.perf_counter()
                _, ys, seg = self._partition_layout(kind, y, idx, main)
                t1 = time.perf_counter()
                gam, at = self._gamma_layout(solver, ys, seg, st) if self.gamma_layout else (None, None)
                if self.replicated:  # (this rank's EVs in that layout, for the w0 pass: made here, off the step's path)
                    self._w0_layout(kind, main)
                t2 = time.perf_counter()
                self.stage_ms[kind + "/layout"] = (t1 - t0) * 1e3
                self.stage_ms[kind + "/gamma"] = (t2 - t1) * 1e3
                for p in range(self.P):
                    if st[p, 0] > 0:
                        a, b = seg[p]
                        solver.stage_partition(p, ys[a:b], st[p, 0], st[p, 1], st[p, 2], st[p, 3], descending=True,
                                               gamma_view=None if gam is None else gam[at[p][0]:at[p][1]])

        if self._exchange:  # (every rank creates its plans' device communicators in the same order)
            for job in jobs:
                stage(job)
            return []
        if self._stage_pool is None:
            self._stage_pool = concurrent.futures.ThreadPoolExecutor(max_workers=2)
        return [self._stage_pool.submit(stage, job) for job in jobs]

    def _gamma_layout(self, solver: PriceSolver, ys, seg, st):
        """Every partition's loop-plan batch of one EV type in ONE launch (lompc_levels_gamma, for
        PriceSolver._build_plans' ``prebuilt``): gamma = y_max - y0 of the layout's levels (ascending
        within each partition's run, whose levels descend), and on rank 0 each partition's central QP
        (gamma_sc = y_max - (y_hi + y_lo) / 2, price_solver.py:73-76) right after its run.  The runs'
        bounds and central gammas go up in one copy from pinned memory.  Returns (the buffer,
        {p: (start, end)} of its views)."""
        torch = _torch()
        P, ym = self.P, float(solver.consts.y_max)
        central = 1 if solver._rank() == 0 else 0
        order = sorted(range(P), key=lambda p: seg[p])  # the runs in storage order
        n = int(ys.numel())
        hb = self._gl_host.get(solver)
        if hb is None:  # (per solver: the two types' staging threads run at once)
            hb = self._gl_host[solver] = torch.empty(2 * P + 1, dtype=torch.float64).pin_memory()
        h = hb.numpy()
        runs = h[: P + 1].view(np.int64)
        runs[0] = seg[order[0]][0]
        for k, p in enumerate(order):
            runs[k + 1] = seg[p][1]
            h[P + 1 + k] = ym - (float(st[p, 1]) + float(st[p, 2])) / 2 if st[p, 0] > 0 else 0.0
        if runs[0] != 0 or runs[P] != n:
            raise RuntimeError("partition layout: the runs do not tile the levels")
        dev = hb.to(ys.device, non_blocking=True)
        gam = torch.empty(n + central * P, dtype=torch.float64, device=ys.device)
        lib = _lib.load()
        rc = lib.lompc_levels_gamma(ys.data_ptr(), n, dev.data_ptr(), P, ym, central, dev.data_ptr() + 8 * (P + 1),
                                    gam.data_ptr(), torch.cuda.current_stream(ys.device).cuda_stream)
        if rc != _lib.LOMPC_OK:
            raise RuntimeError(_lib.status_text(lib, None, rc))
        at = {p: (seg[p][0] + k * central, seg[p][1] + (k + 1) * central) for k, p in enumerate(order)}
        self._gl_keep[solver] = (hb, dev)  # (the copy's source stays alive until it has run)
        return gam, at

    def _sorted_layouts(self):
        """Both EV types' partition layouts and statistics from ONE sort per type and rank, by the
        extension's lompc_levels_layout: this rank's levels sorted descending, so partition p (charge
        levels in [rng[p], rng[p+1]], later partitions winning on shared edges, charging_station.py:
        111-116) is one contiguous run — partition P-1 first — in descending charge level (ascending
        gamma, as the loop plans want), with its count / max / min / sum (price_solver.py:66-77)
        computed on the device.  Sharded: the ranks' records all-gathered and combined in rank order
        (counts and sums added rank 0 first, max / min), as partition_stats does; one host sync for
        both types.  A type with a charge level outside [rng[0], rng[P]] on any rank (whose EVs keep
        their previous partition index, :111-116, so the runs would not be the partitions) is left out
        of the result: the caller takes the index-based path for it.  Returns {kind: (P, 4) host
        statistics (count, max, min, sum)}; the layouts go to self._layout."""
        torch = _torch()
        P = self.P
        lib = _lib.load()
        stream = torch.cuda.current_stream(self.device).cuda_stream
        parts, recs = [], []
        group = None if self.replicated else self.group  # (replicated: the whole population is here)
        for kind, rng in (("Small", self.y0_s_rng), ("Large", self.y0_l_rng)):
            y = self._loop_levels(kind)[0]
            n = int(y.numel())
            b = self._bounds.get(id(rng))
            if b is None:
                b = self._bounds[id(rng)] = torch.as_tensor(rng, dtype=y.dtype, device=y.device)
            if n == 0:  # (an empty shard: no levels, the empty record)
                e = np.array([0.0, -np.inf, np.inf, 0.0] * P + [-np.inf, np.inf, rng[0], rng[P]])
                recs.append(torch.as_tensor(e, device=y.device))
                parts.append((kind, y.new_empty(0), torch.zeros(0, dtype=torch.int64, device=y.device)))
                continue
            lv = self._lv.get(kind)
            if lv is None or lv["n"] != n:  # (buffers per type, reused from step to step)
                wb, hb = ctypes.c_size_t(0), ctypes.c_size_t(0)
                rc = lib.lompc_levels_layout(None, n, None, P, None, None, None, None, ctypes.byref(wb), None)
                if rc != _lib.LOMPC_OK:
                    raise ValueError(_lib.status_text(lib, None, rc))
                rc = lib.lompc_levels_stats(None, n, None, P, None, None, ctypes.byref(hb), None)
                e = lambda m, dt: torch.empty(m, dtype=dt, device=y.device)
                lv = self._lv[kind] = {"n": n, "ys": e(n, torch.float64), "perm": e(n, torch.int64),
                                       "stats": e(4 * P + 4, torch.float64), "stats_sort": e(4 * P + 4, torch.float64),
                                       "work": e(max(wb.value, hb.value), torch.uint8), "wb": wb.value,
                                       "hb": hb.value if rc == _lib.LOMPC_OK else 0}
            if lv["hb"]:  # the statistics alone now; the sort when the layout is first needed (beside the IPM)
                hb = ctypes.c_size_t(lv["hb"])
                rc = lib.lompc_levels_stats(y.data_ptr(), n, b.data_ptr(), P, lv["stats"].data_ptr(),
                                            lv["work"].data_ptr(), ctypes.byref(hb), stream)
                if rc != _lib.LOMPC_OK:
                    raise RuntimeError(_lib.status_text(lib, None, rc))
                parts.append((kind, None, None))
            else:
                wb = ctypes.c_size_t(lv["wb"])
                rc = lib.lompc_levels_layout(y.data_ptr(), n, b.data_ptr(), P, lv["ys"].data_ptr(),
                                             lv["perm"].data_ptr(), lv["stats"].data_ptr(), lv["work"].data_ptr(),
                                             ctypes.byref(wb), stream)
                if rc != _lib.LOMPC_OK:
                    raise RuntimeError(_lib.status_text(lib, None, rc))
                parts.append((kind, lv["ys"], lv["perm"]))
            recs.append(lv["stats"])
        rec = torch.stack(recs)  # (2, 4P + 4)
        if group is None:
            h = rec.cpu().numpy()[None]  # the one host sync
        else:
            import torch.distributed as dist

            world = dist.get_world_size(group)
            # (the concatenated output form: gloo rejects the stacked (world, ...) one)
            allr = torch.empty((world * rec.shape[0], rec.shape[1]), dtype=rec.dtype, device=rec.device)
            dist.all_gather_into_tensor(allr, rec.contiguous(), group=group)
            h = allr.view(world, *rec.shape).cpu().numpy()  # the one host sync
        out = {}
        for j, (kind, ys, perm) in enumerate(parts):
            rows = h[:, j]  # (ranks, 4P + 4)
            st = rows[0, : 4 * P].reshape(P, 4).copy()  # count, max, min, sum; the other ranks in rank order
            for r in range(1, rows.shape[0]):
                o = rows[r, : 4 * P].reshape(P, 4)
                st[:, 0] += o[:, 0]
                st[:, 3] += o[:, 3]
                st[:, 1] = np.maximum(st[:, 1], o[:, 1])
                st[:, 2] = np.minimum(st[:, 2], o[:, 2])
            ymax, ymin = rows[:, 4 * P].max(), rows[:, 4 * P + 1].min()
            lo, hi = rows[0, 4 * P + 2], rows[0, 4 * P + 3]
            if not (ymin >= lo and ymax <= hi):  # (NaN fails too; every rank decides the same)
                continue
            mine = dist.get_rank(group) if group is not None else 0
            cnt = rows[mine, : 4 * P].reshape(P, 4)[:, 0].astype(np.int64)  # this rank's runs
            ends = np.cumsum(cnt[::-1])  # runs in storage order, partition P-1 first
            seg = {p: (int(ends[k] - cnt[p]), int(ends[k])) for k, p in enumerate(range(P - 1, -1, -1))}
            if ys is None:
                self._pending[kind] = seg  # (sorted by _partition_layout)
            else:
                self._layout[kind] = (perm, ys, seg)
            out[kind] = st
        return out

    def _partition_layout(self, kind, y, idx, reader=None):
        """This rank's EVs of one type grouped by partition, each partition in descending charge
        level (ascending gamma = y_max - y: the price loops' plans aggregate per certified piece,
        LOMPC_PLAN_SORTED_GAMMA), once per step: (permutation, charge levels in that order, host
        {partition: (start, end)}) — per-partition slices without boolean indexing (one host sync per
        type and step instead of one per partition).  Made by _sorted_layouts on one rank; otherwise
        here from the partition indices."""
        torch = _torch()
        if kind not in self._layout and kind in self._pending:
            # the sort the statistics pass deferred: this rank's levels descending (lompc_levels_layout, on
            # the current stream), the runs from the statistics' counts
            seg = self._pending.pop(kind)
            lv, lib = self._lv[kind], _lib.load()
            b = self._bounds[id(self.y0_s_rng if kind == "Small" else self.y0_l_rng)]
            wb = ctypes.c_size_t(lv["wb"])
            rc = lib.lompc_levels_layout(y.data_ptr(), int(y.numel()), b.data_ptr(), self.P, lv["ys"].data_ptr(),
                                         lv["perm"].data_ptr(), lv["stats_sort"].data_ptr(), lv["work"].data_ptr(),
                                         ctypes.byref(wb), torch.cuda.current_stream(self.device).cuda_stream)
            if rc != _lib.LOMPC_OK:
                raise RuntimeError(_lib.status_text(lib, None, rc))
            self._layout[kind] = (lv["perm"], lv["ys"], seg)
        if kind not in self._layout:
            if idx is None:  # (replicated: the whole population's indices, gathered by index_stats)
                idx = self._idxfull[kind]
            # (partition, -y) order exactly: a stable sort by descending y, then a stable sort by
            # partition (a composite float key would round near-equal charge levels out of order)
            by_y = torch.argsort(y, descending=True, stable=True)
            perm = by_y[torch.argsort(idx[by_y], stable=True)]
            counts = torch.bincount(idx, minlength=self.P)[: self.P].cpu().numpy()
            off = np.concatenate([[0], np.cumsum(counts)]).astype(np.int64)
            ys = y[perm]
            if reader is not None:  # (made on another stream: the allocator keeps them until `reader` is done)
                perm.record_stream(reader)
                ys.record_stream(reader)
            self._layout[kind] = (perm, ys, {p: (int(off[p]), int(off[p + 1])) for p in range(self.P)})
        return self._layout[kind]

    def _part_slice(self, kind, y, idx, p):
        """(charge levels in layout order, (start, end) of partition p in it)."""
        perm, ys, seg = self._partition_layout(kind, y, idx)
        return ys, seg[p]

    def _w0_batched(self, kind, solver: PriceSolver, y, idx, prices, lmbd_r):
        """All partitions of one EV type in ONE engine call (price_solver.py:272-285 per partition).
        Returns (w0 in EV order, the device rows per partition (sum w0, sum price0, count, failed,
        invalid) combined over ranks — `_w0_checked` reads and checks them)."""
        torch = _torch()
        N, P = self.N_lo, self.P
        perm, ys, seg = self._w0_layouts()[kind] if self.replicated else self._partition_layout(kind, y, idx)
        # the sets in layout order (each partition's run of EVs; _sorted_layouts stores partition P-1
        # first): set k = partition order[k]
        order = sorted(range(P), key=lambda p: seg[p])
        off = np.array([seg[order[0]][0]] + [seg[p][1] for p in order], dtype=np.int64)
        gamma = (solver.consts.y_max - ys).contiguous()
        lm = np.zeros((P, 3 * N))
        lm[:, : self.r] = prices[order]
        lompc = solver.lompc
        lompc.set_params(lm, np.full(P, float(lmbd_r)))
        res = lompc.solve_batch(gamma, off, want_w=False, want_cost=False, want_w0=True, want_set=True, check=False)
        st = res["set_stats"]
        back = torch.as_tensor(np.argsort(order), device=st.device)  # partition p's row: set back[p]
        red = torch.stack([st[:, _lib.LOMPC_STAT_SUM_W0], st[:, _lib.LOMPC_STAT_SUM_PRICE0],
                           st[:, _lib.LOMPC_STAT_COUNT], st[:, _lib.LOMPC_STAT_N_FAILED],
                           st[:, _lib.LOMPC_STAT_N_INVALID]], dim=1)[back].contiguous()
        if self.group is not None:
            import torch.distributed as dist

            dist.all_reduce(red, op=dist.ReduceOp.SUM, group=self.group)
        w0 = torch.empty_like(y)
        w0[perm] = res["w0"]
        return w0, red  # (red on the device: both types' engine calls are issued before one host sync)

    @staticmethod
    def _w0_checked(red) -> np.ndarray:
        red = red.cpu().numpy()
        if np.any(red[:, 4] > 0):
            raise AssertionError("gamma outside [0, y_max]")
        if np.any(red[:, 3] > 0):
            raise SolverError("LoMPC QPs without a certified optimum")
        return red[:, :3]

    def _w0_both(self, prices_s, prices_l, lmbd_r):
        """Both EV types' w0 / price0 pass (price_solver.py:272-285 for every partition) in ONE engine
        run of one plan over both contexts (kept across steps, re-targeted by lompc_plan_update): the
        sets are the partitions in layout order, small type first.  Returns (w0_s, w0_l in EV order,
        the device rows per (type, partition) (sum w0, sum price0, count, failed, invalid) combined over
        ranks, partition order, small type's P rows first)."""
        torch = _torch()
        from .lompc import BatchPlan

        N, P = self.N_lo, self.P
        gams, offs, lm, per = [], [0], np.zeros((2 * P, 3 * N)), []
        for t, (kind, solver, y, idx, prices) in enumerate(
                (("Small", self.price_solver_s, self.y_s, self.idx_s, prices_s),
                 ("Large", self.price_solver_l, self.y_l, self.idx_l, prices_l))):
            perm, ys, seg = self._w0_layouts()[kind] if self.replicated else self._partition_layout(kind, y, idx)
            order = sorted(range(P), key=lambda p: seg[p])  # set t P + k = partition order[k]
            gams.append(solver.consts.y_max - ys)
            offs += [offs[-1] - seg[order[0]][0] + seg[p][1] for p in order]
            lm[t * P:(t + 1) * P, : self.r] = prices[order]
            per.append((perm, order, int(ys.numel())))
        gamma = torch.cat(gams)
        off = np.asarray(offs, dtype=np.int64)
        plan = self._w0plan
        if plan is None:
            plan = self._w0plan = BatchPlan([self.price_solver_s.lompc, self.price_solver_l.lompc], gamma, off,
                                            sets_per_ctx=[P, P], want_w=False, want_cost=False, want_w0=True,
                                            want_set=True, validate=False)
        else:
            plan.update(gamma, off, validate=False)
        hb = self._w0_host
        if hb is None:
            hb = self._w0_host = torch.empty(2 * P * (3 * N + 1), dtype=torch.float64).pin_memory()
        h = hb.numpy()
        h[: 2 * P * 3 * N] = lm.reshape(-1)
        h[2 * P * 3 * N:] = float(lmbd_r)
        dev = hb.to(gamma.device, non_blocking=True)
        res = plan.run(dev[: 2 * P * 3 * N], dev[2 * P * 3 * N:])
        st = res["set_stats"]
        back = np.concatenate([t * P + np.argsort(per[t][1]) for t in range(2)])  # partition p of type t: its set
        red = torch.stack([st[:, _lib.LOMPC_STAT_SUM_W0], st[:, _lib.LOMPC_STAT_SUM_PRICE0],
                           st[:, _lib.LOMPC_STAT_COUNT], st[:, _lib.LOMPC_STAT_N_FAILED],
                           st[:, _lib.LOMPC_STAT_N_INVALID]], dim=1)[torch.as_tensor(back, device=st.device)]
        if self.group is not None:
            import torch.distributed as dist

            dist.all_reduce(red, op=dist.ReduceOp.SUM, group=self.group)
        w0s, o = [], 0
        for (perm, _, n), y in zip(per, (self.y_s, self.y_l)):
            w0 = torch.empty_like(y)
            w0[perm] = res["w0"][o:o + n]
            w0s.append(w0)
            o += n
        self._w0_keep = dev  # (the prices' copy source stays alive until it has run)
        return w0s[0], w0s[1], red

    def _get_w0_price0(self, prices_s, prices_l, lmbd_r: float):
        # charging_station.py:310-329
        if self.w0_one_call and self.price_solver_s.lompc.mode != "direct":  # (DIRECT plans: one context each)
            w0_s, w0_l, red = self._w0_both(prices_s, prices_l, lmbd_r)
            red = self._w0_checked(red)
            red_s, red_l = red[: self.P], red[self.P:]
        else:
            w0_s, red_s = self._w0_batched("Small", self.price_solver_s, self.y_s, self.idx_s, prices_s, lmbd_r)
            w0_l, red_l = self._w0_batched("Large", self.price_solver_l, self.y_l, self.idx_l, prices_l, lmbd_r)
            red_s, red_l = self._w0_checked(red_s), self._w0_checked(red_l)
        price0_s, price0_l = np.zeros((self.P,)), np.zeros((self.P,))
        for p in range(self.P):
            if red_s[p, 2] > 0:
                price0_s[p] = red_s[p, 1] / red_s[p, 2]
            if red_l[p, 2] > 0:
                price0_l[p] = red_l[p, 1] / red_l[p, 2]
        return w0_s, w0_l, price0_s, price0_l, (red_s, red_l)

    # ------------------------------------------------------------------ state
    def _update_state(self, w0_s, w0_l, u0_g: float, w0_stats) -> None:
        # charging_station.py:331-370
        torch = _torch()
        residual_charge = 0
        thr_s = MIN_FULL_CHARGE_FRACTION * self.consts_s.y_max
        thr_l = MIN_FULL_CHARGE_FRACTION * self.consts_l.y_max
        if self.group is None:
            # both types' residual sums and full counts in ONE host sync; the redraws then fill the
            # full EVs in index order (masked_scatter_: no further sync), small type's draws first
            self.y_s += w0_s
            self.y_l += w0_l
            mask_s, mask_l = self.y_s > thr_s, self.y_l > thr_l
            h = torch.stack([torch.where(mask_s, self.y_s - thr_s, 0.0).sum(), torch.where(mask_l, self.y_l - thr_l, 0.0).sum(),
                             mask_s.sum().to(torch.float64), mask_l.sum().to(torch.float64)]).cpu().numpy()
            residual_charge += self.consts_s.theta * float(h[0])
            for y, mask, n in ((self.y_s, mask_s, int(h[2])), (self.y_l, mask_l, int(h[3]))):
                if n:
                    draws = self.y0_min + (self.y0_max - self.y0_min) * np.random.random((n,))
                    y.masked_scatter_(mask, torch.as_tensor(draws, dtype=torch.float64, device=y.device))
            self.ncharged_s += int(h[2])
            self.ncharged_l += int(h[3])
            residual_charge += self.consts_l.theta * float(h[1])
        else:
            # sharded: both types' local residual sums and full counts in ONE all-gather (one host sync);
            # the residual sums combined in rank order, the redraws in global EV order (every rank draws
            # the global vector from the replicated stream and keeps its slice)
            import torch.distributed as dist

            self.y_s += w0_s
            self.y_l += w0_l
            mask_s, mask_l = self.y_s > thr_s, self.y_l > thr_l
            rec = torch.stack([torch.where(mask_s, self.y_s - thr_s, 0.0).sum(), torch.where(mask_l, self.y_l - thr_l, 0.0).sum(),
                               mask_s.sum().to(torch.float64), mask_l.sum().to(torch.float64)])
            world = dist.get_world_size(self.group)
            allr = torch.empty(4 * world, dtype=torch.float64, device=rec.device)
            dist.all_gather_into_tensor(allr, rec, group=self.group)
            h = allr.view(world, 4).cpu().numpy()  # the one host sync
            me = dist.get_rank(self.group)
            res = h[0, :2].copy()
            for r in range(1, world):  # fixed rank order
                res += h[r, :2]
            residual_charge += self.consts_s.theta * float(res[0]) + self.consts_l.theta * float(res[1])
            for j, (y, mask) in enumerate(((self.y_s, mask_s), (self.y_l, mask_l))):
                cnt = h[:, 2 + j].astype(np.int64)
                total, before, local = int(cnt.sum()), int(cnt[:me].sum()), int(cnt[me])
                if total:
                    draws = self.y0_min + (self.y0_max - self.y0_min) * np.random.random((total,))
                    if local:
                        y.masked_scatter_(mask, torch.as_tensor(draws[before:before + local], dtype=torch.float64,
                                                                 device=y.device))
                if j == 0:
                    self.ncharged_s += total
                else:
                    self.ncharged_l += total
        self._update_indices()
        if not ADD_RESIDUAL_CHARGE_TO_BATTERY:
            residual_charge = 0
        red_s, red_l = w0_stats
        sum_w0_s, sum_w0_l = float(np.sum(red_s[:, 0])), float(np.sum(red_l[:, 0]))
        u0_b = u0_g + (-self.consts_s.theta * sum_w0_s - self.consts_l.theta * sum_w0_l + residual_charge
                       - self.demand[self.t]) / self.B
        self.x += u0_b
        if _settings.PRINT_LEVEL >= 1 and self._rank0():
            print(f"# small EVs charged    : {self.ncharged_s:5d}")
            print(f"# large EVs charged    : {self.ncharged_l:5d}")
            print("")

    def _update_logs(self, lmbd_r: float, nu: tuple, stats: tuple, price0: tuple, w0_stats) -> None:
        # charging_station.py:372-433
        w_hat_s, w_hat_l, u_g, w0_s, w0_l = nu
        stats_bi, stats_s, stats_l = stats
        price0_s, price0_l = price0
        red_s, red_l = w0_stats
        for p in range(self.P):  # mean w0 per partition (:380-384)
            if red_s[p, 2] > 0:
                self.logs["inputs"]["w_s"][p, self.t] = red_s[p, 0] / red_s[p, 2]
            if red_l[p, 2] > 0:
                self.logs["inputs"]["w_l"][p, self.t] = red_l[p, 0] / red_l[p, 2]
        self.logs["inputs"]["w_hat_s"][:, self.t] = w_hat_s[:, 0]
        self.logs["inputs"]["w_hat_l"][:, self.t] = w_hat_l[:, 0]
        self.logs["inputs"]["u_g"][self.t] = u_g[0]
        self.logs["states"]["x"][self.t] = self.x
        self.logs["bounds"]["beta_s"][:, self.t] = stats_bi["beta_s"]
        self.logs["bounds"]["beta_l"][:, self.t] = stats_bi["beta_l"]
        self.logs["statistics"]["ncharged_s"] = self.ncharged_s
        self.logs["statistics"]["ncharged_l"] = self.ncharged_l
        self.logs["statistics"]["gamma_sm"][:, self.t] = stats_bi["gamma_sm"]
        self.logs["statistics"]["gamma_lm"][:, self.t] = stats_bi["gamma_lm"]
        for p in range(self.P):
            self.logs["statistics"]["niter_s"][p, self.t] = stats_s[p]["iter"] if stats_s[p] else -1
            self.logs["statistics"]["niter_l"][p, self.t] = stats_l[p]["iter"] if stats_l[p] else -1
        self.logs["statistics"]["Mp_s"][:, self.t] = stats_bi["Mp_s"]
        self.logs["statistics"]["Mp_l"][:, self.t] = stats_bi["Mp_l"]
        self.logs["prices"]["lmbd_r"][self.t] = lmbd_r
        self.logs["prices"]["avg_price_s"][:, self.t] = price0_s
        self.logs["prices"]["avg_price_l"][:, self.t] = price0_l
        for p in range(self.P):
            self.logs["prices"]["price_red_s"][p, self.t] = (
                stats_s[p]["price_after_reg"] - stats_s[p]["price_before_reg"] if stats_s[p] else np.nan)
            self.logs["prices"]["price_red_l"][p, self.t] = (
                stats_l[p]["price_after_reg"] - stats_l[p]["price_before_reg"] if stats_l[p] else np.nan)
