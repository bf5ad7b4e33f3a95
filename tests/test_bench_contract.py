"""CPU tests of bench.py's launch contract and of the rank-ordered combine (no GPU needed).

* ``--gpus N`` must describe the ranks that ran: a launcher's WORLD_SIZE that differs from N is
  refused before any measurement; without a launcher, N > 1 starts N rank processes itself
  (bench.spawn_ranks, exercised on the GPU box by scripts/gpu_session.sh `bdist2`).
* No ``LOMPC_*`` diagnostic variable may be set for a measured run.
* ``dist.combine_rows`` (the gloo path's combine, and the reference for the device combine
  ``lompc_combine_records`` in tests/test_gpu_comm.py) sums the ranks' records in rank order and
  takes the max of the A_bar-error column.
"""
import os
import subprocess
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _bench(env_extra, *args):
    env = {k: v for k, v in os.environ.items() if not k.startswith("LOMPC_")}
    env.update(env_extra)
    return subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), *args], env=env, capture_output=True,
                          text=True, timeout=300)


def test_bench_refuses_world_mismatch():
    r = _bench({"WORLD_SIZE": "1", "RANK": "0", "LOCAL_RANK": "0"}, "--gpus", "2")
    assert r.returncode != 0 and "--gpus 2 but WORLD_SIZE 1" in (r.stderr + r.stdout)


def test_bench_refuses_diagnostic_env():
    r = _bench({"LOMPC_HOST_LOOP": "1"}, "--gpus", "1")
    assert r.returncode != 0 and "LOMPC_HOST_LOOP" in (r.stderr + r.stdout)


def test_combine_rows_rank_order():
    from lompc_amd import _lib
    from lompc_amd.dist import combine_rows

    rng = np.random.default_rng(1)
    world, S, N, K = 5, 3, 4, _lib.LOMPC_SET_STATS
    L = S * (N + K)
    rows = rng.standard_normal((world, L)) * 10.0 ** rng.integers(-8, 8, size=(world, L))
    sw, st = torch.empty((S, N), dtype=torch.float64), torch.empty((S, K), dtype=torch.float64)
    combine_rows(torch.as_tensor(rows), [(sw, st)])
    tot = rows[0].copy()
    for r in range(1, world):  # the same sequence of IEEE additions
        tot = tot + rows[r]
    assert np.array_equal(sw.numpy().ravel(), tot[: S * N])
    want = tot[S * N:].reshape(S, K).copy()
    want[:, _lib.LOMPC_STAT_MAX_ERR] = rows[:, S * N:].reshape(world, S, K)[:, :, _lib.LOMPC_STAT_MAX_ERR].max(0)
    assert np.array_equal(st.numpy(), want)
