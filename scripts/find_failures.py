"""Diagnostic: search random price vectors (bench distribution) for uncertified QPs.

Runs PATH and DIRECT mode over many seeded lambda draws (12 sets x 131072 EVs per
type, N=24, gamma = y_max - U[0.3, 0.5]) and dumps every failing (lambda, gamma)
case to gpurun_out/failures.npz for offline analysis against the oracle.
"""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "incentive-design-mpc_amd"))
from lompc_amd import BatchPlan, LoMPC, LoMPCConstants, _lib  # noqa: E402

N, P, M = int(os.environ.get("FF_N", "24")), 12, 131072
DRAWS = int(os.environ.get("FF_DRAWS", "64"))
out = {}
for name, c in (("small", LoMPCConstants(0.05, 10.0, 0.9, 0.25, "small")),
                ("large", LoMPCConstants(0.025, 50.0, 0.9, 0.15, "large"))):
    rng = np.random.default_rng(0)
    off = np.array([(M * p) // P for p in range(P + 1)], dtype=np.int64)
    g = torch.as_tensor(c.y_max - (0.3 + 0.2 * rng.random(M)), device="cuda")
    lr = torch.zeros(P, dtype=torch.float64, device="cuda")
    for mode in ("path", "direct"):
        lompc = LoMPC(N, c, device=0, mode=mode)
        plan = BatchPlan(lompc, g, off, want_status=True)
        rng_l = np.random.default_rng(123)
        nbad = 0
        for k in range(DRAWS):
            lm = torch.as_tensor(c.theta * rng_l.random((P, 3 * N)), device="cuda")
            o = plan.run(lm, lr)
            st = o["status"].cpu().numpy()
            bad = np.nonzero(st == _lib.LOMPC_QP_FAILED)[0]
            rep = int((st == _lib.LOMPC_QP_REPAIRED).sum())
            if len(bad) or rep:
                sets = np.searchsorted(off, bad, side="right") - 1
                print(f"{name} {mode} draw {k}: failed {len(bad)} (sets {sorted(set(sets.tolist()))}), repaired {rep}")
            if len(bad) and nbad < 4:
                s0 = int(sets[0])
                out[f"{name}_{mode}_{k}_lmbd"] = lm[s0].cpu().numpy()
                out[f"{name}_{mode}_{k}_gamma"] = g.cpu().numpy()[bad[sets == s0][:64]]
                nbad += 1
        print(f"{name} {mode}: {DRAWS} draws done")
os.makedirs("gpurun_out", exist_ok=True)
np.savez("gpurun_out/failures.npz", **out)
print("saved", len(out) // 2, "cases")
