"""Multi-GPU sharding of the EV batch (one process per GPU, torch.distributed).

The per-EV QPs are independent (price_solver.py:203-209); the only exchange
step of a price iteration is the set of per-partition reductions the
PriceSolver consumes (sum of w, max A_bar error, sum of w0 / price0 — the
aggregate demand of charging_station.py:356-366).  Each rank solves a
contiguous shard of every set's EVs; ``allreduce_set_results`` then combines
the fused per-set reductions with ONE sum all-reduce and ONE max all-reduce
(RCCL over xGMI with the "nccl" backend; gloo on CPU in the tests).  Payload
is S * (N + 7) doubles — a few KB — so the collective is latency-bound.
"""
from __future__ import annotations

import numpy as np

from . import _lib

_SUM_COLS = [_lib.LOMPC_STAT_COUNT, _lib.LOMPC_STAT_SUM_W0, _lib.LOMPC_STAT_SUM_PRICE0,
             _lib.LOMPC_STAT_SUM_COST, _lib.LOMPC_STAT_N_REPAIRED, _lib.LOMPC_STAT_N_FAILED,
             _lib.LOMPC_STAT_N_INVALID]
_COLS = {}


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
    import torch
    import torch.distributed as dist

    S, N = set_sum_w.shape
    cols = _COLS.get(set_stats.device)
    if cols is None:  # cached: a fresh host->device index copy per call would stall the stream
        cols = _COLS[set_stats.device] = torch.as_tensor(_SUM_COLS, device=set_stats.device)
    packed = torch.cat([set_sum_w.reshape(-1), set_stats[:, cols].reshape(-1)])
    dist.all_reduce(packed, op=dist.ReduceOp.SUM, group=group)
    mx = set_stats[:, _lib.LOMPC_STAT_MAX_ERR].contiguous()
    dist.all_reduce(mx, op=dist.ReduceOp.MAX, group=group)
    set_sum_w.copy_(packed[: S * N].reshape(S, N))
    set_stats[:, cols] = packed[S * N:].reshape(S, len(_SUM_COLS))
    set_stats[:, _lib.LOMPC_STAT_MAX_ERR] = mx
    return set_sum_w, set_stats
