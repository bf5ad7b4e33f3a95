"""GPU tests of the sharded product path on RCCL (include/lompc_amd.h lompc_comm_* /
lompc_plan_set_comm): a plan with the extension's own communicator all-gathers every rank's
per-set reduction record and combines it in rank order on the device, inside the same C-ABI call
as the run (run_steps, the C++ price loop).

RCCL refuses two ranks on one device, so on the one-GPU box the RCCL code path runs with a
world-size-1 "nccl" process group: the same calls (unique id broadcast, ncclCommInitRank,
ncclAllGather on the plan's stream, the combine kernel, the station's torch.distributed
collectives) as an 8-GPU job, with one record to combine.  The multi-rank arithmetic (sharded =
single, rank-ordered sums) is covered by the world-2 gloo tests (test_gpu_station.py,
test_host.py), which run the same record layout through dist.combine_set_results.

Bar: a world-1 sharded run equals the unsharded run BITWISE (the combine of one record is a copy;
the price steps and the station logs then follow identically).
"""
import os
import socket

import numpy as np
import pytest
import torch

import lompc_oracle as O
from lompc_amd import BatchPlan, LoMPC, LoMPCConstants, settings
from lompc_amd.lompc import LoMPCConstants as LC

pytestmark = pytest.mark.gpu


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.fixture(scope="module")
def nccl1(gpu):
    import torch.distributed as dist

    from lompc_amd import dist as ldist

    dist.init_process_group("nccl", init_method=f"tcp://127.0.0.1:{_free_port()}", rank=0, world_size=1,
                            device_id=torch.device("cuda:0"))
    yield dist.group.WORLD
    ldist.release_comms()
    dist.destroy_process_group()


def _two_type_batch(rng, N, P, M, K):
    cs = [O.small_consts(), O.large_consts()]
    lompcs = [LoMPC(N, LoMPCConstants(c.delta, c.theta, c.y_max, c.w_max, c.ev_type), device=0) for c in cs]
    off1 = [np.array([(m * p) // P for p in range(P + 1)], dtype=np.int64) for m in M]
    off = np.concatenate([off1[0], M[0] + off1[1][1:]])
    g = torch.as_tensor(np.concatenate([c.y_max - (0.3 + 0.2 * rng.random(m)) for c, m in zip(cs, M)]), device="cuda:0")
    wr = torch.as_tensor(np.concatenate([c.w_max * rng.random((P, N)) for c in cs]), device="cuda:0")
    lm = torch.as_tensor(np.stack([np.concatenate([c.theta * rng.random((P, 3 * N)) for c in cs]) for _ in range(K)]),
                         device="cuda:0")
    lr = torch.as_tensor(0.05 * rng.random((K, 2 * P)), device="cuda:0")
    return lompcs, off, g, wr, lm, lr


@pytest.mark.parametrize("want_w", [True, False])
def test_plan_with_comm_equals_plain(nccl1, want_w):
    """run / run_steps with the communicator attached write bitwise the plain plan's outputs; the
    run is two launches longer (all-gather + combine)."""
    from lompc_amd.dist import device_comm

    N, P, K = 24, 6, 5
    lompcs, off, g, wr, lm, lr = _two_type_batch(np.random.default_rng(3), N, P, [20000, 17001], K)
    plain = BatchPlan(lompcs, g, off, sets_per_ctx=[P, P], w_ref=wr, want_w=want_w, want_status=True)
    shard = BatchPlan(lompcs, g, off, sets_per_ctx=[P, P], w_ref=wr, want_w=want_w, want_status=True)
    shard.set_comm(device_comm(nccl1, 0))
    assert shard.launches_per_run() == plain.launches_per_run() + 2
    for k in range(K):
        plain.run(lm[k], lr[k])
        shard.run(lm[k], lr[k])
        torch.cuda.synchronize()
        for key, v in plain.out.items():
            if v is not None:
                assert torch.equal(v, shard.out[key]), (k, key)
    assert shard.check()[1:] == (0, 0)
    shard.run_steps(lm, lr, K, lm[0].numel(), lr[0].numel())
    plain.run_steps(lm, lr, K, lm[0].numel(), lr[0].numel())
    assert shard.check()[1:] == (0, 0) and plain.check()[1:] == (0, 0)
    for key, v in plain.out.items():
        if v is not None:
            assert torch.equal(v, shard.out[key]), key
    # run_steps with the communicator (wide form: ONE all-gather of the group's runs' records after their
    # closings and one combine kernel; the split form: one all-gather + combine per run), every run's
    # records kept: the plain plan's, both issue forms
    for per_kernel in (False, True):
        for per_run in (False, True):  # (per_run: every output per run)
            o_s = shard.run_steps(lm, lr, K, lm[0].numel(), lr[0].numel(), per_run_sets=True, per_run=per_run,
                                  per_kernel=per_kernel)
            o_p = plain.run_steps(lm, lr, K, lm[0].numel(), lr[0].numel(), per_run_sets=True, per_run=per_run)
            assert shard.check()[1:] == (0, 0) and plain.check()[1:] == (0, 0)
            assert shard.info()["steps_group"] == plain.info()["steps_group"] == 1
            for key, v in o_p.items():
                if v is not None:
                    assert torch.equal(v, o_s[key]), (per_kernel, per_run, key)


def test_sorted_wide_with_comm_equals_plain(nccl1):
    """run_steps over gamma-sorted sets without per-EV output (k_paths + k_aggs per group) with the
    communicator: the group's per-set records go to its contiguous send records, ONE all-gather and one
    combine per group — bitwise the plain plan's outputs, per run and shared, both issue forms."""
    from lompc_amd.dist import device_comm

    N, P, K = 24, 6, 9
    lompcs, off, g, wr, lm, lr = _two_type_batch(np.random.default_rng(5), N, P, [20000, 17001], K)
    gs = g.clone()
    for s in range(2 * P):  # each set's gamma ascending
        gs[off[s]:off[s + 1]] = torch.sort(g[off[s]:off[s + 1]]).values
    kw = dict(sets_per_ctx=[P, P], w_ref=wr, want_w=False, want_cost=False, sorted_gamma=True)
    plain = BatchPlan(lompcs, gs, off, **kw)
    shard = BatchPlan(lompcs, gs, off, **kw).set_comm(device_comm(nccl1, 0))
    st = (lm[0].numel(), lr[0].numel())
    for per_kernel in (False, True):
        for per_run_sets in (False, True):
            o_s = shard.run_steps(lm, lr, K, *st, per_run_sets=per_run_sets, per_kernel=per_kernel)
            o_p = plain.run_steps(lm, lr, K, *st, per_run_sets=per_run_sets)
            assert shard.check()[1:] == (0, 0) and plain.check()[1:] == (0, 0)
            for key in ("set_sum_w", "set_stats"):
                assert torch.equal(o_p[key], o_s[key]), (per_kernel, per_run_sets, key)


@pytest.mark.parametrize("nranks", [2, 3, 8])
@pytest.mark.parametrize("S,N", [(24, 24), (24, 48), (5000, 64)])
def test_combine_records_matches_python_combine(gpu, nranks, S, N):
    """The device combine that every sharded run issues after its all-gather (k_combine, exposed as
    lompc_combine_records) on nranks synthetic rank records equals dist.combine_rows (the combine of
    the gloo path, dist.combine_set_results) on the same bytes bit for bit: rank-ordered sums of every
    column, the max of LOMPC_STAT_MAX_ERR.  S (N + 8) = 5000 x 72 doubles exceeds the kernel's
    1024 x 256-thread grid (its grid-stride loop) and any record a plan has all-gathered before."""
    from lompc_amd import _lib
    from lompc_amd.dist import combine_rows

    lib = _lib.load()
    rng = np.random.default_rng(nranks * 1000 + S + N)
    K = _lib.LOMPC_SET_STATS
    L = S * (N + K)
    rows = rng.standard_normal((nranks, L)) * 10.0 ** rng.integers(-6, 6, size=(nranks, L))
    st = rows[:, S * N:].reshape(nranks, S, K)
    st[:, :, _lib.LOMPC_STAT_MAX_ERR] = np.abs(st[:, :, _lib.LOMPC_STAT_MAX_ERR]) + 1e-300  # errors >= 0
    recv = torch.as_tensor(rows, device="cuda:0").contiguous()
    sw_d = torch.full((S, N), np.nan, dtype=torch.float64, device="cuda:0")
    st_d = torch.full((S, K), np.nan, dtype=torch.float64, device="cuda:0")
    stream = torch.cuda.current_stream().cuda_stream
    assert lib.lompc_combine_records(recv.data_ptr(), nranks, S, N, sw_d.data_ptr(), st_d.data_ptr(), 0, stream) == 0
    sw_h = torch.empty((S, N), dtype=torch.float64)
    st_h = torch.empty((S, K), dtype=torch.float64)
    combine_rows(torch.as_tensor(rows), [(sw_h, st_h)])
    torch.cuda.synchronize()
    assert torch.equal(sw_d.cpu(), sw_h) and torch.equal(st_d.cpu(), st_h)
    # one output only (the other may be NULL), and bad arguments refused
    st_d.fill_(np.nan)
    assert lib.lompc_combine_records(recv.data_ptr(), nranks, S, N, None, st_d.data_ptr(), 0, stream) == 0
    torch.cuda.synchronize()
    assert torch.equal(st_d.cpu(), st_h)
    assert lib.lompc_combine_records(recv.data_ptr(), 0, S, N, None, None, 0, stream) == _lib.LOMPC_ERR_INVALID_ARG
    assert lib.lompc_combine_records(None, nranks, S, N, None, None, 0, stream) == _lib.LOMPC_ERR_INVALID_ARG


def test_sharded_price_loop_runs_native(nccl1, monkeypatch):
    """PriceSolver on a process group takes the C++ price loop (lompc_price_loop with the plan's
    communicator) and returns bitwise the single-rank prices and solver_stats."""
    from lompc_amd.price_solver import PriceSolver

    monkeypatch.setattr(settings, "PRINT_LEVEL", 0)
    rng = np.random.default_rng(11)
    N = 24
    for c, price_type in ((LC(0.025, 50, 0.9, 0.15, "large"), "linear-convex"), (LC(0.05, 10, 0.9, 0.25, "small"), "linear")):
        y0 = 0.3 + 0.2 * rng.random(5000)
        w_ref = c.w_max * rng.random(N) * 0.5
        out = []
        for group in (None, nccl1):
            ps = PriceSolver(N, c, price_type, device=0, group=group)
            ps.set_charge_levels(torch.as_tensor(y0, device="cuda:0"))
            if group is not None:
                assert ps._plan.comm is not None and ps._native_ok()
            calls = []
            orig = ps._iterate
            monkeypatch.setattr(ps, "_iterate", lambda *a, **k: (calls.append(1), orig(*a, **k))[1])
            lm, stats = ps.compute_optimal_prices(w_ref, 0.0)
            assert not calls  # no per-iteration Python engine call
            out.append((lm.copy(), stats, ps.n_batched_calls))
        (l0, s0, n0), (l1, s1, n1) = out
        assert np.array_equal(l0, l1) and n0 == n1
        assert s0["iter"] == s1["iter"]
        for k in ("dual_cost_decrease_actual", "dual_cost_decrease_predicted"):
            assert np.array_equal(s0[k], s1[k]), k


@pytest.mark.parametrize("mode", ["replicated", "exchange"])
def test_station_world1_nccl_equals_single(nccl1, monkeypatch, mode):
    """The closed loop on a world-1 RCCL group gives bitwise the single-process trajectory in both
    sharded forms — replicated (the default: the levels all-gathered once per step, every price loop
    on every rank as one persistent launch, the w0 sums / re-draw counts / residual charge combined
    through torch.distributed) and exchange (device-combined set reductions per price iteration)."""
    from lompc_amd.charging_station import ChargingStation
    from test_gpu_station import consts

    monkeypatch.setattr(settings, "PRINT_LEVEL", 0)
    M_2 = 61
    np.random.seed(5)
    ref = ChargingStation(consts(M_2, Tf=3), device=0)
    rl = ref.simulate()
    np.random.seed(5)
    sh = ChargingStation(consts(M_2, Tf=3), device=0, group=nccl1, sharded_loops=mode)
    sl = sh.simulate()
    if mode == "exchange":
        assert sh.price_solver_s._plan.comm is not None and sh.price_solver_l._plan.comm is not None
    else:  # (the loops see the whole population: no communicator, the device loop)
        assert sh.price_solver_s.group is None and sh.price_solver_s.device_loop and sh.replicated
    for sec in ("inputs", "bounds", "prices", "states", "statistics"):
        for k, v in rl[sec].items():
            a, b = np.asarray(v), np.asarray(sl[sec][k])
            assert np.array_equal(a, b, equal_nan=True), (sec, k)
    assert torch.equal(ref.y_s, sh.y_s) and torch.equal(ref.y_l, sh.y_l)
    assert sh.price_solver_s.n_batched_calls == ref.price_solver_s.n_batched_calls
