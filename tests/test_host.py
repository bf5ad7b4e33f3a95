"""CPU tests of the host logic around the kernels: EV sharding, the RCCL/gloo
combine of fused per-set reductions (world_size 2 over gloo), and the
price_solver.py error formulas applied to fused reductions."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from lompc_amd import _lib
from lompc_amd.dist import allreduce_set_results, shard_range, shard_sets
from lompc_amd.price_ops import set_errors, structured_abar

import lompc_oracle as O


def test_shard_range_partitions():
    for n in (0, 1, 7, 1000, 262144):
        for world in (1, 2, 3, 8):
            spans = [shard_range(n, r, world) for r in range(world)]
            assert spans[0][0] == 0 and spans[-1][1] == n
            assert all(spans[i][1] == spans[i + 1][0] for i in range(world - 1))
            sizes = [b - a for a, b in spans]
            assert max(sizes) - min(sizes) <= 1


def test_shard_sets_keeps_set_contiguity():
    off = np.array([0, 5, 5, 17, 40], dtype=np.int64)  # includes an empty set
    seen = []
    for r in range(3):
        idx, loc = shard_sets(off, r, 3)
        assert loc[0] == 0 and loc[-1] == len(idx) and np.all(np.diff(loc) >= 0)
        for s in range(4):
            part = idx[loc[s]:loc[s + 1]]
            assert np.all((part >= off[s]) & (part < off[s + 1]))
        seen.append(idx)
    allidx = np.sort(np.concatenate(seen))
    np.testing.assert_array_equal(allidx, np.arange(40))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _rank_main(rank, world, port, sums, stats, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    sw = torch.tensor(sums[rank])
    st = torch.tensor(stats[rank])
    allreduce_set_results(sw, st)
    q.put((rank, sw.numpy(), st.numpy()))
    dist.barrier()
    dist.destroy_process_group()


def test_allreduce_set_results_gloo_world2():
    """Per-rank fused reductions of two shards combine to the single-rank
    answer (sum columns add, the max-error column takes the max)."""
    rng = np.random.default_rng(0)
    S, N, world = 3, 12, 2
    sums = [rng.random((S, N)) for _ in range(world)]
    stats = [rng.random((S, _lib.LOMPC_SET_STATS)) for _ in range(world)]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_rank_main, args=(r, world, port, sums, stats, q)) for r in range(world)]
    for p in procs:
        p.start()
    out = [q.get(timeout=120) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    exp_sw = sums[0] + sums[1]
    exp_st = stats[0] + stats[1]
    exp_st[:, _lib.LOMPC_STAT_MAX_ERR] = np.maximum(stats[0][:, 3], stats[1][:, 3])
    for _, sw, st in out:
        np.testing.assert_allclose(sw, exp_sw, rtol=1e-15)
        np.testing.assert_allclose(st, exp_st, rtol=1e-15)


def test_set_errors_match_price_solver_formulas(golden):
    """Sharded fused reductions + set_errors == price_solver.py:196-214."""
    for case in golden[:6]:
        N = case["N"]
        W = case["w"]
        A = np.tril(np.ones((N, N)))
        A_bar = structured_abar(A, case["delta"], case["lmbd_r"])
        # two shards, reduced like allreduce_set_results would
        halves = (W[:7], W[7:])
        sum_w = sum(h.sum(axis=0) for h in halves)[None, :]
        dv = W - case["w_ref"]
        errs = np.sqrt(np.einsum("bi,ij,bj->b", dv, A_bar, dv))
        stats = np.zeros((1, _lib.LOMPC_SET_STATS))
        stats[0, _lib.LOMPC_STAT_COUNT] = len(W)
        stats[0, _lib.LOMPC_STAT_MAX_ERR] = max(errs[:7].max(), errs[7:].max())
        emax, w0e, avge = set_errors(A_bar, case["w_ref"][None, :], sum_w, stats)
        assert abs(emax[0] - case["w_err_max"]) <= 1e-10
        assert abs(w0e[0] - case["w0_err"]) <= 1e-10
        assert abs(avge[0] - case["w_avg_err"]) <= 1e-10


def test_structured_abar_is_reference_metric():
    A = np.tril(np.ones((24, 24)))
    A_bar, _ = O.w_inner_product_metric(A, 0.025, 0.3)
    np.testing.assert_allclose(structured_abar(A, 0.025, 0.3), A_bar)


def test_settings_mirror_reference_values():
    from lompc_amd import settings as S

    assert (S.MIN_MAX_BAT_SOC, S.MAX_MAX_BAT_SOC, S.MAX_BAT_CHARGE_RATE) == (0.75, 0.9, 0.25)
    assert S.MAX_PRICE_SOLVER_ITERATIONS == 1000 and S.PRICE_SOLVER_TOL_TYPE == "avg"
    assert (S.MIN_INITIAL_SOC, S.MAX_INITIAL_SOC, S.MIN_FULL_CHARGE_FRACTION) == (0.3, 0.5, 0.95)


def test_lompc_constructor_checks_match_reference():
    """lompc.py:36-38 asserts fire before any device work."""
    from lompc_amd import LoMPC, LoMPCConstants

    with pytest.raises(AssertionError):
        LoMPC(12, LoMPCConstants(0.05, 10, 0.95, 0.25, "small"))
    with pytest.raises(AssertionError):
        LoMPC(12, LoMPCConstants(0.05, 10, 0.9, 0.3, "small"))
    with pytest.raises(AssertionError):
        LoMPC(12, LoMPCConstants(0.05, 10, 0.9, 0.25, "medium"))
    with pytest.raises(ZeroDivisionError):  # q_scale = 3 theta / (4 w_max), lompc.py:67
        LoMPC(12, LoMPCConstants(0.05, 10, 0.9, 0, "small"))


def test_check_last_raises_solver_error_without_plan():
    """LoMPC.check_last on a failed batch raises SolverError with the context's text (a LoMPC has
    no plan handle).  The C library is replaced by a stub reporting one failed QP."""
    import ctypes

    from lompc_amd.lompc import BatchPlan, LoMPC, SolverError

    class FakeLib:
        def lompc_last_status(self, ctx, stream, rep, fail, inv):
            ctypes.cast(fail, ctypes.POINTER(ctypes.c_int64)).contents.value = 1
            return _lib.LOMPC_OK

        lompc_plan_status = None

        def lompc_last_error(self, ctx):
            return b"context text"

    lm = object.__new__(LoMPC)
    lm._lib, lm._ctx, lm.device = FakeLib(), None, 0
    lm._stream = lambda: 0
    with pytest.raises(SolverError, match="1 EVs failed: context text"):
        lm.check_last()

    class FakePlanLib(FakeLib):
        def lompc_plan_status(self, plan, stream, rep, fail, inv):
            return self.lompc_last_status(None, stream, rep, fail, inv)

        def lompc_plan_last_error(self, plan):
            return b""

    bp = object.__new__(BatchPlan)
    bp._lib, bp._plan, bp._stream, bp.direct = FakePlanLib(), None, 0, False
    with pytest.raises(SolverError, match="without a certified optimum"):
        bp.check()
