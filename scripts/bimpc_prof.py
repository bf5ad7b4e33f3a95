"""Diagnostic: the host BiMPC interior point's phases on one instance (N = 48, P = 12, EXP_UNWEIGHTED:
config 5's planner), from a -DLQ_BIMPC_PROF variant library (stderr: factor / directions / residuals /
polish), or wall time only from the product library.

    python scripts/build_variant.py bprof LQ_BIMPC_PROF
    python scripts/bimpc_prof.py [liblompc_amd_bprof.so] [--cases FILE.npz]
"""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "tests"), os.path.join(ROOT, "oracle"), os.path.join(ROOT, "incentive-design-mpc_amd")]
from lompc_amd import _lib  # noqa: E402

libname = next((a for a in sys.argv[1:] if a.endswith(".so")), "liblompc_amd.so")
_lib._lib = _lib.load(os.path.join(ROOT, "incentive-design-mpc_amd", "lompc_amd", libname))
from test_bimpc_host import instance, solve  # noqa: E402

N, P = 48, 12
reps = 20
for seed in (5, 6):
    bi, params, _ = instance(N, P, seed=seed, cost_type=2, u_g_max=1.0, x_max=0.5, u_b_max=0.5)
    solve(N, P, bi, params)
    ts = []
    for _ in range(reps):
        t = time.perf_counter()
        b, *_ = solve(N, P, bi, params)
        ts.append((time.perf_counter() - t) * 1e3)
    print(f"seed {seed}: min {min(ts):7.3f} ms, median {np.median(ts):7.3f} ms per solve, "
          f"{b.last_info['iterations']} iterations", flush=True)
