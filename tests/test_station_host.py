"""CPU tests of the closed loop's sharded host logic (charging_station.py): partition
statistics combined over ranks (charging_station.py:196-210 / price_solver.py:66-77)
and the full-charge re-draw replaying the reference's global np.random stream in EV
order (charging_station.py:339-341) — world_size 2 over gloo on CPU tensors."""
import os
import socket

import numpy as np
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from lompc_amd.charging_station import partition_stats, redraw_full, shard_bounds


def test_shard_bounds_cover():
    for n in (1, 2, 61, 1000):
        for w in (1, 2, 3, 8):
            b = [shard_bounds(n, r, w) for r in range(w)]
            assert b[0][0] == 0 and b[-1][1] == n and all(b[i][1] == b[i + 1][0] for i in range(w - 1))


def test_partition_stats_single_process():
    rng = np.random.default_rng(0)
    y = torch.as_tensor(0.3 + 0.6 * rng.random(200))
    idx = torch.as_tensor(rng.integers(0, 5, 200))
    st = partition_stats(y, idx, 6)
    yn, ix = y.numpy(), idx.numpy()
    for p in range(6):
        m = ix == p
        assert st[p, 0] == m.sum()
        if m.any():
            assert st[p, 1] == yn[m].max() and st[p, 2] == yn[m].min()
            assert abs(st[p, 3] - yn[m].sum()) <= 1e-12


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _rank(rank, world, port, y_all, idx_all, mask_all, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    lo, hi = shard_bounds(len(y_all), rank, world)
    y = torch.as_tensor(y_all[lo:hi].copy())
    idx = torch.as_tensor(idx_all[lo:hi].copy())
    st = partition_stats(y, idx, 6, group=dist.group.WORLD)
    np.random.seed(42)  # replicated stream on every rank
    n = redraw_full(y, torch.as_tensor(mask_all[lo:hi].copy()), 0.3, 0.5, np.random.random, group=dist.group.WORLD)
    q.put((rank, st, n, y.numpy()))
    dist.barrier()
    dist.destroy_process_group()


def test_sharded_stats_and_redraw_world2():
    rng = np.random.default_rng(1)
    n = 37
    y_all = 0.3 + 0.6 * rng.random(n)
    idx_all = rng.integers(0, 5, n)
    mask_all = rng.random(n) < 0.4
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _port()
    procs = [ctx.Process(target=_rank, args=(r, 2, port, y_all, idx_all, mask_all, q)) for r in range(2)]
    for p in procs:
        p.start()
    outs = sorted([q.get(timeout=120) for _ in range(2)], key=lambda o: o[0])
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    ref_st = partition_stats(torch.as_tensor(y_all), torch.as_tensor(idx_all), 6)
    # the reference's single-process re-draw (charging_station.py:339-341)
    np.random.seed(42)
    y_ref = y_all.copy()
    y_ref[mask_all] = 0.3 + (0.5 - 0.3) * np.random.random((mask_all.sum(),))
    y_got = np.concatenate([o[3] for o in outs])
    for _, st, cnt, _ in outs:
        np.testing.assert_array_equal(st[:, :3], ref_st[:, :3])
        np.testing.assert_allclose(st[:, 3], ref_st[:, 3], rtol=1e-14)
        assert cnt == mask_all.sum()
    np.testing.assert_array_equal(y_got, y_ref)


def _ref_indices(y, rng, idx0):
    """charging_station.py:111-116 as written: the masked loop, later partitions winning."""
    idx = idx0.copy()
    for p in range(len(rng) - 1):
        idx[(y >= rng[p]) & (y <= rng[p + 1])] = p
    return idx


def test_update_indices_matches_reference_loop_on_edges():
    """The searchsorted form of _update_indices equals the reference's masked loop on every
    boundary value, below rng[0], above rng[P], and with repeated boundaries."""
    from lompc_amd.charging_station import ChargingStation

    rs = np.random.default_rng(3)
    cases = [np.linspace(0.2, 0.9, 13), np.array([0.0, 0.0, 0.5, 1.0]), np.array([0.0, 0.5, 1.0, 1.0]),
             np.array([0.1, 0.4, 0.4, 0.4, 0.8]), np.array([0.3, 0.3])]
    for rng in cases:
        P = len(rng) - 1
        eps = 1e-12
        y = np.concatenate([rng, np.nextafter(rng, -np.inf), np.nextafter(rng, np.inf), [rng[0] - 0.1, rng[-1] + 0.1,
                            rng[0] - eps, rng[-1] + eps], rng[0] + (rng[-1] - rng[0]) * rs.random(50)])
        idx0 = rs.integers(0, P, len(y))
        cs = object.__new__(ChargingStation)
        cs.P = P
        cs.y_s = torch.as_tensor(y)
        cs.y_l = torch.as_tensor(y[::-1].copy())
        cs.idx_s = torch.as_tensor(idx0.copy())
        cs.idx_l = torch.as_tensor(idx0[::-1].copy())
        cs.y0_s_rng, cs.y0_l_rng = rng, rng.copy()
        cs._bounds = {}
        ChargingStation._update_indices(cs)
        assert np.array_equal(cs.idx_s.numpy(), _ref_indices(y, rng, idx0)), rng
        assert np.array_equal(cs.idx_l.numpy(), _ref_indices(y[::-1], rng, idx0[::-1])), rng



def _rank_rep(rank, world, port, ys_all, yl_all, P, q):
    """Replicated sharding's host logic on CPU tensors: the levels' all-gather and this rank's EVs in
    the whole population's layout order (ChargingStation._gather_levels / _w0_layouts)."""
    from lompc_amd.charging_station import ChargingStation

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    cs = object.__new__(ChargingStation)
    cs.group, cs.M_2, cs.P, cs._dev = dist.group.WORLD, len(ys_all), P, "cpu"
    cs._lo, cs._hi = shard_bounds(cs.M_2, rank, world)
    cs.y_s = torch.as_tensor(ys_all[cs._lo:cs._hi].copy())
    cs.y_l = torch.as_tensor(yl_all[cs._lo:cs._hi].copy())
    cs.replicated, cs._exchange = True, False
    cs._layout, cs._pending, cs._layout_w0 = {}, {}, {}
    ChargingStation._gather_levels(cs)
    full = {k: v.numpy().copy() for k, v in cs._yfull.items()}
    rng = np.linspace(0.3, 0.9, P + 1)
    cs._idxfull = {k: (torch.searchsorted(torch.as_tensor(rng), cs._yfull[k], right=True) - 1).clamp_(0, P - 1)
                   for k in ("Small", "Large")}
    lay = ChargingStation._w0_layouts(cs)
    q.put((rank, full, {k: (v[0].numpy(), v[1].numpy(), v[2]) for k, v in lay.items()},
           {k: cs._layout[k][2] for k in cs._layout}))
    dist.barrier()
    dist.destroy_process_group()


def test_replicated_levels_and_local_layout_world2():
    """world 2 (unequal shards): every rank holds the whole population's levels in EV order after the
    one all-gather, and its w0 layout is exactly its own EVs in the loops' layout order (partition runs
    in descending charge level), each run bounded by this rank's count in that partition."""
    rng = np.random.default_rng(7)
    n, P = 53, 6
    ys_all, yl_all = 0.3 + 0.6 * rng.random(n), 0.3 + 0.6 * rng.random(n)
    ys_all[5] = ys_all[9]  # (a tie)
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _port()
    procs = [ctx.Process(target=_rank_rep, args=(r, 2, port, ys_all, yl_all, P, q)) for r in range(2)]
    for p in procs:
        p.start()
    outs = sorted([q.get(timeout=120) for _ in range(2)], key=lambda o: o[0])
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    edges = np.linspace(0.3, 0.9, P + 1)
    for rank, full, lay, seg_full in outs:
        np.testing.assert_array_equal(full["Small"], ys_all)
        np.testing.assert_array_equal(full["Large"], yl_all)
        lo, hi = shard_bounds(n, rank, 2)
        for kind, y_all in (("Small", ys_all), ("Large", yl_all)):
            lperm, lys, seg = lay[kind]
            assert sorted(lperm.tolist()) == list(range(hi - lo))
            np.testing.assert_array_equal(lys, y_all[lo:hi][lperm])
            part = np.clip(np.searchsorted(edges, y_all, side="right") - 1, 0, P - 1)
            for p in range(P):
                a, b = seg[p]
                got = lperm[a:b] + lo
                want = np.nonzero(part[lo:hi] == p)[0] + lo
                assert sorted(got.tolist()) == want.tolist(), (kind, p)
                assert np.all(np.diff(lys[a:b]) <= 0)
                # the same EVs in the same order as the whole layout's run, restricted to this rank
                fa, fb = seg_full[kind][p]
                assert fb - fa == (part == p).sum()
