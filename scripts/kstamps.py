"""Diagnostic: k_solve phase timing from s_memtime stamps (LOMPC_STAMPS build).

    python scripts/kstamps.py --build     # here: builds lompc_amd/liblompc_amd_stamps.so
    python scripts/kstamps.py [N]         # on the GPU box: bench workload (both EV types, 24 sets)

Per wave (= (set, gamma cell)): setup (lambda loads), exact solve at the cell start (PDAS),
path tracking, EV phase, epilogue; shader cycles, mean / p90 / max over waves, per EV type.
"""
import ctypes
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "incentive-design-mpc_amd"))
from lompc_amd import _lib, build  # noqa: E402

DBG = os.path.join(ROOT, "incentive-design-mpc_amd", "lompc_amd", "liblompc_amd_stamps.so")
if "--build" in sys.argv:
    print(build.build(force=True, verbose=True, out=DBG, defines=("LOMPC_STAMPS",)))
    sys.exit(0)

import torch  # noqa: E402

lib = _lib.load(DBG)
_lib._lib = lib
lib.lompc_debug_stamps.restype = ctypes.c_int
lib.lompc_debug_stamps.argtypes = [ctypes.c_void_p, ctypes.c_int]
from lompc_amd import BatchPlan, LoMPC, LoMPCConstants  # noqa: E402

N = int(sys.argv[1]) if len(sys.argv) > 1 and sys.argv[1].isdigit() else 24
P, B = 12, 262144
outputs = os.environ.get("KS_OUTPUTS", "full")
rng = np.random.default_rng(0)
cs = [LoMPCConstants(0.05, 10.0, 0.9, 0.25, "small"), LoMPCConstants(0.025, 50.0, 0.9, 0.15, "large")]
lompcs = [LoMPC(N, c, device=0) for c in cs]
M = B // 2
off1 = np.array([(M * p) // P for p in range(P + 1)], dtype=np.int64)
off = np.concatenate([off1, M + off1[1:]])
g = torch.as_tensor(np.concatenate([c.y_max - (0.3 + 0.2 * rng.random(M)) for c in cs]), device="cuda")
lm = torch.as_tensor(np.concatenate([c.theta * rng.random((P, 3 * N)) for c in cs]), device="cuda")
wr = torch.as_tensor(np.concatenate([c.w_max * rng.random((P, N)) for c in cs]), device="cuda")
lr = torch.zeros(2 * P, dtype=torch.float64, device="cuda")
plan = BatchPlan(lompcs, g, off, sets_per_ctx=[P, P], w_ref=wr, want_w=outputs == "full", want_cost=outputs != "set",
                 warm_start=os.environ.get("KS_WARM") == "1")
for _ in range(5):
    plan.run(lm, lr)
plan.check()
G1 = plan.cells + 1
nb = 2 * P * G1
buf = np.zeros(nb * 8, dtype=np.int64)
assert lib.lompc_debug_stamps(buf.ctypes.data, buf.size) == 0
st = buf.reshape(nb, 8)
valid = st[:, 7] > 0
cell = np.arange(nb) % G1
valid &= cell < G1 - 1
t = st[:, :6].astype(np.float64)
names = ["setup", "solve@start", "tracking", "EV phase", "epilogue", "total"]
d = np.stack([t[:, 1] - t[:, 0], t[:, 2] - t[:, 1], t[:, 3] - t[:, 2], t[:, 4] - t[:, 3], t[:, 5] - t[:, 4],
              t[:, 5] - t[:, 0]], 1)
start0 = t[valid, 0].min()
print(f"N={N} outputs={outputs} cells={plan.cells}  (shader cycles; s_memtime)")
for k, name in enumerate(("small", "large")):
    sel = valid & (np.arange(nb) // G1 // P == k)
    print(f"{name}: waves {sel.sum()}, EVs/wave mean {st[sel, 7].mean():.0f}, pieces mean {st[sel, 6].mean():.2f} "
          f"max {st[sel, 6].max()}")
    for j, nm in enumerate(names):
        x = d[sel, j]
        print(f"   {nm:12s} mean {x.mean():8.0f}  p90 {np.percentile(x, 90):8.0f}  max {x.max():8.0f}")
    print(f"   wave start offset (vs first wave): mean {(t[sel, 0] - start0).mean():.0f} max {(t[sel, 0] - start0).max():.0f};"
          f" end max {(t[sel, 5] - start0).max():.0f}")
