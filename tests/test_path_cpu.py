"""The path engine's algorithm on the host (oracle/path_cpu.cpp, bench.py's same-algorithm CPU
baseline) against the dense oracle (oracle/lompc_oracle.c) and the 50-digit golden vectors.

It is a second, sequential restatement of the device path engine (lompc_plan.hip: per (set, gamma
cell) exact start solve + parametric active-set tracking with KKT-certified pieces, per-EV lookup,
per-set reductions), so these tests pin the ALGORITHM the GPU runs — piecewise-affine w*(gamma),
piece certificates, cost / error quadratics — independently of the device code.  Tolerances as the
GPU parity tests: |dw| <= 1e-9, cost 1e-9 relative, set sums 1e-10 relative.
"""
import numpy as np
import pytest

import lompc_oracle as O
import oracle_c

TOL_W = 1e-9


def _sets(rng, cs, sizes, N, lr_values):
    P = len(sizes[0])
    off = np.concatenate([[0], np.cumsum(np.concatenate(sizes))]).astype(np.int64)
    ctx = np.repeat(np.arange(len(cs)), [len(s) for s in sizes])
    g = np.concatenate([cs[ctx[s]].y_max * rng.random(off[s + 1] - off[s]) for s in range(len(ctx))])
    lm = np.concatenate([c.theta * rng.random((P, 3 * N)) for c in cs])
    lr = np.asarray(lr_values * len(cs), dtype=np.float64)
    wr = np.concatenate([c.w_max * rng.random((P, N)) for c in cs])
    return off, ctx, g, lm, lr, wr


def _check(o, cs, ctx, off, g, lm, lr, wr, N):
    for s in range(len(ctx)):
        a, b = off[s], off[s + 1]
        st = o["set_stats"][s]
        assert st[0] == b - a and st[6] == 0 and st[7] == 0
        if b == a:
            assert np.all(o["set_sum_w"][s] == 0)
            continue
        c = cs[ctx[s]]
        wo, co, nf = oracle_c.solve_batch(N, c, lm[s], lr[s], g[a:b])
        assert nf == 0
        np.testing.assert_allclose(o["w"][a:b], wo, atol=TOL_W, rtol=0)
        np.testing.assert_allclose(o["cost"][a:b], co, rtol=1e-9, atol=1e-9)
        np.testing.assert_allclose(o["set_sum_w"][s], wo.sum(0), rtol=1e-10, atol=1e-9)
        np.testing.assert_allclose(st[4], co.sum(), rtol=1e-10, atol=1e-9)
        np.testing.assert_allclose(st[1], wo[:, 0].sum(), rtol=1e-10, atol=1e-9)
        # max A_bar error (price_solver.py:207-209) from the oracle's w
        kappa = lr[s] / c.delta
        dv = wo - wr[s]
        err = np.sqrt(np.sum(np.cumsum(dv, axis=1) ** 2, axis=1) + kappa * np.sum(dv * dv, axis=1))
        np.testing.assert_allclose(st[3], err.max(), rtol=1e-7, atol=1e-9)


@pytest.mark.parametrize("N", [12, 24, 48])
def test_path_cpu_matches_dense_oracle(N):
    """Both EV types in one call, ragged sets (empty, one EV, small, a few thousand), lmbd_r = 0 and
    > 0, gamma over the whole [0, y_max] (box bounds and PWL kinks are crossed along the paths)."""
    rng = np.random.default_rng(100 + N)
    cs = [O.small_consts(), O.large_consts()]
    sizes = [[0, 1, 300, 2500], [1700, 64, 0, 3]]
    off, ctx, g, lm, lr, wr = _sets(rng, cs, sizes, N, [0.0, 0.2, 0.0, 3 * N * 0.025])
    o = oracle_c.path_run(N, cs, [4, 4], lm, lr, g, off, w_ref=wr)
    assert o["info"][3] == 0
    _check(o, cs, ctx, off, g, lm, lr, wr, N)


def test_path_cpu_cells_and_bounds():
    """The answer does not depend on the cell count (1 / 8 / 64 cells), and gammas at 0 and y_max and
    invalid ones (NaN, negative, above y_max: counted, NaN outputs) are handled as on the device."""
    rng = np.random.default_rng(7)
    N = 24
    c = O.large_consts()
    g = np.concatenate([np.zeros(50), np.full(50, c.y_max), c.y_max * rng.random(900)])
    off = np.array([0, 1000], dtype=np.int64)
    lm = c.theta * rng.random((1, 3 * N))
    lr = np.array([0.1])
    ref = None
    for cells in (1, 8, 64):
        o = oracle_c.path_run(N, [c], [1], lm, lr, g, off, cells=cells)
        if ref is None:
            ref = o
            _check(o, [c], [0], off, g, lm, lr, np.zeros((1, N)), N)
        np.testing.assert_allclose(o["w"], ref["w"], atol=1e-12, rtol=0)
    g2 = g.copy()
    g2[[3, 4, 5]] = [np.nan, -1.0, 2.0]
    o = oracle_c.path_run(N, [c], [1], lm, lr, g2, off)
    assert o["set_stats"][0][7] == 3 and np.isnan(o["w"][3:6]).all() and np.isnan(o["cost"][3:6]).all()


def test_path_cpu_golden(golden):
    """Every 50-digit certified golden case (tests/golden, N in {12, 24, 48}, both EV types, zero /
    linear / linear-convex prices, lmbd_r in {0, random}) to 1e-9."""
    for case in golden:
        c = O.OracleConstants(case["delta"], case["theta"], case["y_max"], case["w_max"], case["ev_type"])
        N = int(case["N"])
        g = np.asarray(case["gamma"], dtype=np.float64)
        off = np.array([0, g.size], dtype=np.int64)
        o = oracle_c.path_run(N, [c], [1], case["lmbd"][None, :], np.array([case["lmbd_r"]]), g, off)
        assert o["info"][3] == 0
        np.testing.assert_allclose(o["w"], case["w"], atol=TOL_W, rtol=0)
        np.testing.assert_allclose(o["cost"], case["cost"], rtol=1e-9, atol=1e-9)
