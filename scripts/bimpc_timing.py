"""Diagnostic: host BiMPC solve time at N = 16 / 48, P = 12 (the example's and config 5's
horizons) for several worker-pool sizes (LOMPC_HOST_THREADS, one subprocess each)."""
import os
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

if len(sys.argv) > 1 and sys.argv[1] == "child":
    sys.path[:0] = [os.path.join(ROOT, "tests"), os.path.join(ROOT, "oracle"), os.path.join(ROOT, "incentive-design-mpc_amd")]
    from test_bimpc_host import instance, solve

    for N in (16, 48):
        bi, params, _ = instance(N, 12, seed=5, cost_type=2, u_g_max=1.0, x_max=0.5, u_b_max=0.5)
        solve(N, 12, bi, params)
        t = time.perf_counter()
        for _ in range(10):
            b, *_ = solve(N, 12, bi, params)
        print(f"  threads {os.environ.get('LOMPC_HOST_THREADS')}: N={N} {(time.perf_counter() - t) / 10 * 1e3:7.2f} ms "
              f"({b.last_info['iterations']} iterations)", flush=True)
else:
    for nt in (1, 2, 4, 8, 16):
        subprocess.run([sys.executable, __file__, "child"], env={**os.environ, "LOMPC_HOST_THREADS": str(nt)}, check=True)
