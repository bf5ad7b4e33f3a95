"""Multi-GPU sharding of the EV batch (one process per GPU, torch.distributed).

The per-EV QPs are independent (price_solver.py:203-209); the only exchange
step of a price iteration is the set of per-partition reductions the
PriceSolver consumes (sum of w, max A_bar error, sum of w0 / price0 — the
aggregate demand of charging_station.py:356-366).  Each rank solves a
contiguous shard of every set's EVs; ``combine_set_results`` then combines
the fused per-set reductions (of one or several contexts, e.g. both EV types)
with ONE all-gather and a local rank-ordered sum / max (RCCL over xGMI with
the "nccl" backend; gloo on CPU in the tests).  Payload is S * (N + 8) doubles
per rank — a few KB — so the collective is latency-bound and one collective
per step beats a sum plus a max all-reduce per context.

On RCCL the product path does NOT go through ``combine_set_results``: ``RcclComm`` is the
extension's own communicator, attached to a plan, and every run of the plan all-gathers and
combines the same records on the device inside the C-ABI call (include/lompc_amd.h,
lompc_plan_set_comm) — the sharded price loop and ``run_steps`` issue no Python per iteration.
``combine_set_results`` is the same rank-ordered combine for backends without a device
communicator (gloo in the CPU tests).
"""
from __future__ import annotations

import numpy as np

from . import _lib


def shard_range(n: int, rank: int, world: int) -> tuple[int, int]:
    """Contiguous block [lo, hi) of n items owned by ``rank``."""
    base, rem = divmod(n, world)
    lo = rank * base + min(rank, rem)
    return lo, lo + base + (1 if rank < rem else 0)


def shard_sets(set_offsets: np.ndarray, rank: int, world: int) -> tuple[np.ndarray, np.ndarray]:
    """Shard every set's EV range across ranks.

    Returns (index of the global EVs owned by this rank, local set_offsets)."""
    set_offsets = np.asarray(set_offsets, dtype=np.int64)
    idx = []
    loc = [0]
    for s in range(len(set_offsets) - 1):
        a, b = int(set_offsets[s]), int(set_offsets[s + 1])
        lo, hi = shard_range(b - a, rank, world)
        idx.append(np.arange(a + lo, a + hi, dtype=np.int64))
        loc.append(loc[-1] + (hi - lo))
    return (np.concatenate(idx) if idx else np.zeros(0, np.int64)), np.asarray(loc, dtype=np.int64)


def allreduce_set_results(set_sum_w, set_stats, group=None):
    """Combine per-rank fused reductions in place (torch tensors, any device).

    Sum columns: set_sum_w and the count/sum/number columns of set_stats;
    max column: LOMPC_STAT_MAX_ERR."""
    combine_set_results([(set_sum_w, set_stats)], group=group)
    return set_sum_w, set_stats


def combine_set_results(pairs, group=None):
    """Combine several (set_sum_w, set_stats) pairs (e.g. both EV types of a step) with ONE
    collective: every rank's packed records are all-gathered (RCCL over xGMI; ~KB payload, so
    one latency instead of a sum and a max all-reduce per pair), then reduced locally in rank
    order — sums for every column, max for LOMPC_STAT_MAX_ERR.  In place; deterministic."""
    import torch
    import torch.distributed as dist

    world = dist.get_world_size(group)
    flat = [torch.cat([sw.reshape(-1), st.reshape(-1)]) for sw, st in pairs]
    packed = torch.cat(flat) if len(flat) > 1 else flat[0]
    L = packed.numel()
    # the same collective on every backend (RCCL on the GPUs; gloo in the CPU tests)
    out = torch.empty(world * L, dtype=packed.dtype, device=packed.device)
    dist.all_gather_into_tensor(out, packed, group=group)
    combine_rows(out.view(world, L), pairs)


def combine_rows(rows, pairs) -> None:
    """The rank-ordered combine of all-gathered records ``rows`` [world, L] (L = the packed
    (set_sum_w, set_stats) pairs) into ``pairs`` in place: column sums in rank order, the max for
    LOMPC_STAT_MAX_ERR — what the device combine (lompc_combine_records, k_combine) computes on the
    same bytes, bit for bit."""
    world = rows.shape[0]
    tot = rows[0].clone()
    for r in range(1, world):  # fixed rank order
        tot += rows[r]
    mx = rows.amax(dim=0)
    off = 0
    for sw, st in pairs:
        S, N = sw.shape
        sw.copy_(tot[off:off + S * N].view(S, N))
        off += S * N
        K = st.shape[1]
        sums = tot[off:off + S * K].view(S, K)
        maxes = mx[off:off + S * K].view(S, K)
        st.copy_(sums)
        st[:, _lib.LOMPC_STAT_MAX_ERR] = maxes[:, _lib.LOMPC_STAT_MAX_ERR]
        off += S * K


class RcclComm:
    """The extension's own RCCL communicator over the ranks of a torch.distributed group
    (``lompc_comm_*``, include/lompc_amd.h).  Attached to a plan (``BatchPlan.set_comm``) it makes
    every run combine the per-set reductions across ranks ON THE DEVICE (one ncclAllGather over
    xGMI + one rank-ordered combine kernel on the run's stream), so the C++ price loop and
    ``run_steps`` stay in C++ on a sharded batch.  The unique id is made on the group's rank 0
    and broadcast once over torch.distributed; creation is collective over the group."""

    def __init__(self, group=None, device: int | None = None):
        import ctypes

        import torch
        import torch.distributed as dist

        self._lib = _lib.load()
        self.device = torch.cuda.current_device() if device is None else int(device)
        self.rank = dist.get_rank(group)
        self.nranks = dist.get_world_size(group)
        uid = (ctypes.c_ubyte * _lib.LOMPC_COMM_ID_BYTES)()
        if self.rank == 0:
            rc = self._lib.lompc_comm_get_unique_id(uid)
            if rc != _lib.LOMPC_OK:
                raise RuntimeError("lompc_comm_get_unique_id: " + _lib.status_text(self._lib, None, rc))
        dev = f"cuda:{self.device}" if dist.get_backend(group) == "nccl" else "cpu"
        t = torch.tensor(list(bytes(uid)), dtype=torch.uint8, device=dev)
        dist.broadcast(t, src=dist.get_global_rank(group, 0) if group is not None else 0, group=group)
        raw = bytes(t.cpu().tolist())
        uid = (ctypes.c_ubyte * _lib.LOMPC_COMM_ID_BYTES).from_buffer_copy(raw)
        comm = ctypes.c_void_p()
        rc = self._lib.lompc_comm_create(uid, self.nranks, self.rank, self.device, ctypes.byref(comm))
        if rc != _lib.LOMPC_OK:
            raise RuntimeError("lompc_comm_create: " + _lib.status_text(self._lib, None, rc))
        self._comm = comm

    @property
    def handle(self):
        return self._comm

    def close(self) -> None:
        if getattr(self, "_comm", None) is not None:
            self._lib.lompc_comm_destroy(self._comm)
            self._comm = None


_COMMS: dict = {}


def device_comm(group, device: int):
    """The process's RcclComm for (group, device), created on first use (collective), or None when
    the group does not run on RCCL (gloo: the Python fallback combines the reductions)."""
    import torch.distributed as dist

    if group is None or dist.get_backend(group) != "nccl":
        return None
    key = (id(group), int(device))
    if key not in _COMMS:
        _COMMS[key] = RcclComm(group, device)
    return _COMMS[key]


def release_comms() -> None:
    """Destroy every cached communicator (before destroy_process_group)."""
    for c in _COMMS.values():
        c.close()
    _COMMS.clear()


def global_levels(y, y_max: float, group=None) -> tuple[float, float, float, int, int]:
    """(max, min, mean, count, out-of-range count) of a sharded charge-level vector y (any
    device) over all ranks: ONE all-gather of a 5-value record per rank and ONE host sync
    (the reference's per-partition statistics, price_solver.py:66-77, over a sharded batch)."""
    import torch
    import torch.distributed as dist

    n = y.numel()
    inf = torch.tensor(float("inf"), dtype=torch.float64, device=y.device)
    rec = torch.stack([y.max() if n else -inf, -y.min() if n else -inf, y.sum(),
                       torch.tensor(float(n), dtype=torch.float64, device=y.device),
                       torch.logical_not((y >= 0) & (y <= y_max)).sum().to(torch.float64)])
    world = dist.get_world_size(group)
    out = torch.empty(world * 5, dtype=torch.float64, device=y.device)
    dist.all_gather_into_tensor(out, rec, group=group)
    rows = out.view(world, 5).cpu().numpy()  # the one host sync
    mx = rows[:, :2].max(axis=0)
    sm = rows[:, 2:].sum(axis=0)
    count = int(sm[1])
    return float(mx[0]), float(-mx[1]), float(sm[0] / count) if count else float("nan"), count, int(sm[2])
