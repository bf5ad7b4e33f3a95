"""GPU tests of the station's partition layout (lompc_levels_layout, ChargingStation._sorted_layouts):
one descending sort per EV type gives the statistics the reference's index masks define
(charging_station.py:111-116 with price_solver.py:66-77) and each partition's EVs as one run in
descending charge level; levels exactly on boundaries, ties and an out-of-range level included."""
import numpy as np
import pytest
import torch

from lompc_amd.charging_station import ChargingStation, partition_stats

pytestmark = pytest.mark.gpu


def _ref_indices(y, rng, idx0):
    idx = idx0.copy()
    for p in range(len(rng) - 1):
        idx[(y >= rng[p]) & (y <= rng[p + 1])] = p
    return idx


@pytest.mark.parametrize("case", range(5))
def test_sorted_layouts_match_index_partitions(gpu, case):
    rs = np.random.default_rng(80 + case)
    P = 12 if case != 4 else 1
    rng_s, rng_l = np.linspace(0.3, 0.9, P + 1), np.linspace(0.3, 0.85, P + 1)
    n_s, n_l = (5000, 4000) if case != 2 else (300000, 1)
    y_s = 0.3 + 0.2 * rs.random(n_s)
    y_l = 0.3 + 0.55 * rs.random(n_l)
    y_s[:20] = rng_s[rs.integers(0, P + 1, 20)]  # levels exactly on the boundaries
    if n_l > 4:
        y_l[:3] = y_l[3]  # ties
    if case == 3:
        y_l[min(7, n_l - 1)] = 0.2  # below rng[0]: the large type takes the index path
    cs = object.__new__(ChargingStation)
    cs.P, cs.group, cs.device = P, None, 0
    cs.replicated, cs._exchange = False, False
    cs.y_s, cs.y_l = torch.as_tensor(y_s, device="cuda:0"), torch.as_tensor(y_l, device="cuda:0")
    cs.y0_s_rng, cs.y0_l_rng = rng_s, rng_l
    cs.idx_s = torch.zeros(n_s, dtype=torch.int64, device="cuda:0")
    cs.idx_l = torch.zeros(n_l, dtype=torch.int64, device="cuda:0")
    cs._bounds, cs._lv = {}, {}
    ChargingStation._update_indices(cs)  # (resets cs._layout)
    out = ChargingStation._sorted_layouts(cs)
    assert set(out) == ({"Small"} if case == 3 else {"Small", "Large"})
    for kind, y, idx, rng in (("Small", y_s, cs.idx_s, rng_s), ("Large", y_l, cs.idx_l, rng_l)):
        if kind not in out:
            continue
        ix = idx.cpu().numpy()
        np.testing.assert_array_equal(ix, _ref_indices(y, rng, np.zeros(len(y), dtype=np.int64)))
        ref = partition_stats(torch.as_tensor(y), torch.as_tensor(ix), P)
        st = out[kind]
        np.testing.assert_array_equal(st[:, 0], ref[:, 0])
        np.testing.assert_array_equal(st[:, 1:3], ref[:, 1:3])
        np.testing.assert_allclose(st[:, 3], ref[:, 3], rtol=1e-13)
        yt = cs.y_s if kind == "Small" else cs.y_l
        perm, ys, seg = ChargingStation._partition_layout(cs, kind, yt, idx)  # (the deferred sort, if any)
        if P <= 16:  # (the statistics came without the sort: the sort's own equal them, sums to rounding)
            srt = cs._lv[kind]["stats_sort"].cpu().numpy()[: 4 * P].reshape(P, 4)
            np.testing.assert_array_equal(srt[:, :3], st[:, :3])
            np.testing.assert_allclose(srt[:, 3], st[:, 3], rtol=1e-13)
        perm, ys = perm.cpu().numpy(), ys.cpu().numpy()
        assert np.array_equal(np.sort(perm), np.arange(len(y)))
        np.testing.assert_array_equal(ys, y[perm])
        for p in range(P):
            a, b = seg[p]
            assert np.array_equal(np.sort(perm[a:b]), np.nonzero(ix == p)[0])
            assert np.all(np.diff(ys[a:b]) <= 0)
            # stable: equal levels keep index order
            eq = np.diff(ys[a:b]) == 0
            assert np.all(np.diff(perm[a:b])[eq] > 0)


class _Solver:  # (what ChargingStation._gamma_layout reads of a PriceSolver)
    def __init__(self, y_max, rank):
        self.consts = type("C", (), {"y_max": y_max})()
        self._r = rank

    def _rank(self):
        return self._r


@pytest.mark.parametrize("rank", [0, 1])
def test_gamma_layout_matches_per_partition_batches(gpu, rank):
    """ChargingStation._gamma_layout (lompc_levels_gamma: every partition's loop-plan batch of a type in
    one launch) equals the per-partition construction of PriceSolver._build_plans bit for bit: each
    partition's y_max - y (ascending), then on rank 0 its central QP's gamma_sc = y_max - (y_hi + y_lo) / 2;
    empty partitions included."""
    rs = np.random.default_rng(90 + rank)
    P = 12
    rng_s = np.linspace(0.3, 0.9, P + 1)
    y = 0.3 + 0.35 * rs.random(40000)  # (partitions 7 .. 11 empty)
    y[:10] = rng_s[rs.integers(0, 7, 10)]
    cs = object.__new__(ChargingStation)
    cs.P, cs.group, cs.device = P, None, 0
    cs.replicated, cs._exchange = False, False
    cs.y_s, cs.y_l = torch.as_tensor(y, device="cuda:0"), torch.as_tensor(y[:5000].copy(), device="cuda:0")
    cs.y0_s_rng, cs.y0_l_rng = rng_s, rng_s
    cs.idx_s = torch.zeros(len(y), dtype=torch.int64, device="cuda:0")
    cs.idx_l = torch.zeros(5000, dtype=torch.int64, device="cuda:0")
    cs._bounds, cs._lv, cs._gl_host, cs._gl_keep = {}, {}, {}, {}
    ChargingStation._update_indices(cs)
    out = ChargingStation._sorted_layouts(cs)
    st = out["Small"]
    _, ys, seg = ChargingStation._partition_layout(cs, "Small", cs.y_s, cs.idx_s)
    sol = _Solver(0.9, rank)
    gam, at = ChargingStation._gamma_layout(cs, sol, ys, seg, st)
    g = gam.cpu().numpy()
    for p in range(P):
        a, b = seg[p]
        ref = (0.9 - ys[a:b]).cpu().numpy()
        v = g[at[p][0]:at[p][1]]
        assert len(v) == b - a + (1 if rank == 0 else 0)
        np.testing.assert_array_equal(v[: b - a], ref)
        assert np.all(np.diff(v[: b - a]) >= 0)
        if rank == 0 and st[p, 0] > 0:
            assert v[-1] == 0.9 - (float(st[p, 1]) + float(st[p, 2])) / 2


@pytest.mark.parametrize("where", [0, 777, 39999])
def test_levels_stats_nan_fails_the_range_check(gpu, where):
    """A NaN charge level reaches the caller: lompc_levels_stats' whole-type max y / min y propagate it
    (fmax / fmin would drop it), so _sorted_layouts' range check fails and the type takes the index
    path — instead of a NaN counted in partition 0 while the deferred sort puts it elsewhere."""
    rs = np.random.default_rng(95)
    P = 12
    rng_s = np.linspace(0.3, 0.9, P + 1)
    y = 0.3 + 0.55 * rs.random(40000)
    y[where] = np.nan
    cs = object.__new__(ChargingStation)
    cs.P, cs.group, cs.device = P, None, 0
    cs.replicated, cs._exchange = False, False
    cs.y_s, cs.y_l = torch.as_tensor(y, device="cuda:0"), torch.as_tensor(y[:5000].copy(), device="cuda:0")
    cs.y_l[:] = 0.5  # (the large type: no NaN)
    cs.y0_s_rng, cs.y0_l_rng = rng_s, rng_s
    cs.idx_s = torch.zeros(len(y), dtype=torch.int64, device="cuda:0")
    cs.idx_l = torch.zeros(5000, dtype=torch.int64, device="cuda:0")
    cs._bounds, cs._lv = {}, {}
    ChargingStation._update_indices(cs)
    out = ChargingStation._sorted_layouts(cs)
    assert set(out) == {"Large"}
    rec = cs._lv["Small"]["stats"].cpu().numpy()
    assert np.isnan(rec[4 * P]) and np.isnan(rec[4 * P + 1])
