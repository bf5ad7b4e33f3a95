"""Diagnostic: run the config-1 example (lompc_amd.example) and, if a BiMPC solve fails,
dump its parameters to gpurun_out/bimpc_fail.npz (the BiMPC is a host solver, so the
failure can then be replayed on the CPU)."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "incentive-design-mpc_amd"))
from lompc_amd import example  # noqa: E402
from lompc_amd.bimpc import BiMPC  # noqa: E402

orig = BiMPC.solve_bimpc
calls = []


def solve(self, params):
    calls.append(params)
    try:
        return orig(self, params)
    except Exception:
        d = {k: np.asarray(getattr(params, k), dtype=float) for k in
             ("Mp_s", "Mp_l", "beta_s", "beta_l", "gamma_sm", "gamma_lm", "x0", "demand")}
        d.update(N=self.N, P=self.P, step=len(calls) - 1, info=np.array([self.last_info[k] for k in
                 ("iterations", "objective", "primal_residual", "dual_residual", "complementarity")]))
        os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
        seed = sys.argv[sys.argv.index("--seed") + 1] if "--seed" in sys.argv else "0"
        np.savez(os.path.join(ROOT, "gpurun_out", f"bimpc_fail_seed{seed}.npz"), **d)
        print("BiMPC failure at step", len(calls) - 1, self.last_info)
        raise


BiMPC.solve_bimpc = solve
example.main(sys.argv[1:])
