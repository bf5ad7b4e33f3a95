"""Diagnostic: k_solve phase timing from s_memtime stamps (LOMPC_STAMPS build).

    python scripts/kstamps.py --build     # here: builds lompc_amd/liblompc_amd_stamps.so
    python scripts/kstamps.py [N]         # on the GPU box: bench workload (both EV types, 24 sets)

Per k_path wave (= (set, gamma cell)): setup (lambda loads), exact solve at the cell start
(fp32 search + fp64 PDAS), path tracking; shader cycles, mean / p90 / max over waves, per EV type.
"""
import ctypes
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "incentive-design-mpc_amd"))
from lompc_amd import _lib, build  # noqa: E402

# KS_VARIANT=name: lompc_amd/liblompc_amd_stamps_<name>.so built with KS_DEFINES (comma list)
VAR = os.environ.get("KS_VARIANT")
DBG = os.path.join(ROOT, "incentive-design-mpc_amd", "lompc_amd",
                   f"liblompc_amd_stamps_{VAR}.so" if VAR else "liblompc_amd_stamps.so")
if "--build" in sys.argv:
    extra = tuple(d for d in os.environ.get("KS_DEFINES", "").split(",") if d)
    print(build.build(force=True, verbose=True, out=DBG, defines=("LOMPC_STAMPS",) + extra))
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
G = plan.cells
nb = 2 * P * G
buf = np.zeros(nb * 8, dtype=np.int64)
assert lib.lompc_debug_stamps(buf.ctypes.data, buf.size) == 0
st = buf.reshape(nb, 8)
t = st[:, :4].astype(np.float64)
names = ["setup", "solve@start", "tracking", "total"]
d = np.stack([t[:, 1] - t[:, 0], t[:, 2] - t[:, 1], t[:, 3] - t[:, 2], t[:, 3] - t[:, 0]], 1)
print(f"N={N} cells={plan.cells} k_path waves (shader cycles; s_memtime)")
for k, name in enumerate(("small", "large")):
    sel = np.arange(nb) // G // P == k
    print(f"{name}: waves {sel.sum()}, pieces mean {st[sel, 6].mean():.2f} max {st[sel, 6].max()}")
    nit = st[sel, 4]
    n64, n32, pas = nit % 256, (nit // 256) % 256, nit // 65536
    print(f"   iterations: fp32 mean {n32.mean():.2f} max {n32.max()}  fp64 mean {n64.mean():.2f} max {n64.max()}"
          f"  primal-AS {pas.sum()}  tracking mean {st[sel, 5].mean():.2f} max {st[sel, 5].max()}")
    for j, nm in enumerate(names):
        x = d[sel, j]
        print(f"   {nm:12s} mean {x.mean():8.0f}  p90 {np.percentile(x, 90):8.0f}  max {x.max():8.0f}")

# k_eval workgroups (stamps at (32768 + b) * 8)
ev = np.zeros(32768 * 8, dtype=np.int64)
buf2 = np.zeros(65536 * 8, dtype=np.int64)
assert lib.lompc_debug_stamps(buf2.ctypes.data, buf2.size) == 0
e = buf2[32768 * 8:].reshape(32768, 8)[: min(32768, (B + 255) // 256)]
e = e[e[:, 0] != 0].astype(np.float64)
print(f"k_eval workgroups {len(e)} (shader cycles)")
for (a, b), nm in (((0, 1), "loads+stage"), ((1, 4), "lookup+rows"), ((4, 5), "record")):
    x = e[:, b] - e[:, a]
    print(f"   {nm:15s} mean {x.mean():8.0f}  p90 {np.percentile(x, 90):8.0f}  max {x.max():8.0f}")
# wave launch: each wave's start vs its workgroup's wave 0, and the workgroups' starts over the grid
lib.lompc_debug_wstart.restype = ctypes.c_int
lib.lompc_debug_wstart.argtypes = [ctypes.c_void_p, ctypes.c_int]
ws = np.zeros(32768 * 8, dtype=np.int64)
assert lib.lompc_debug_wstart(ws.ctypes.data, ws.size) == 0
wsr = ws.reshape(32768, 8)[:plan.info()["workgroups"]].astype(np.float64)
wsr = wsr[wsr[:, 0] != 0]
t0 = wsr[:, 0].min()
print(f"   wave launch: wave k - wave 0 of its workgroup: mean {np.mean(wsr.max(1) - wsr[:, 0]):.0f} max "
      f"{np.max(wsr.max(1) - wsr[:, 0]):.0f};  workgroup starts over the grid: p50 {np.percentile(wsr[:, 0] - t0, 50):.0f}"
      f" p90 {np.percentile(wsr[:, 0] - t0, 90):.0f} max {np.max(wsr[:, 0] - t0):.0f}")
x = e[:, 5] - e[:, 0]
print(f"   {'total':15s} mean {x.mean():8.0f}  p90 {np.percentile(x, 90):8.0f}  max {x.max():8.0f}")
if os.environ.get("KS_RT") == "1":  # s_memrealtime build (10 ns ticks, one clock for every XCD)
    z = e[:, 0].min()
    for j, nm in ((0, "start"), (6, "block map"), (2, "round 1"), (3, "pieces"), (1, "staged"), (4, "rows done"),
                  (5, "end")):
        x = (e[:, j] - z) / 100.0
        print(f"   timeline {nm:10s} us: p10 {np.percentile(x, 10):6.2f} p50 {np.percentile(x, 50):6.2f}"
              f" p90 {np.percentile(x, 90):6.2f} max {x.max():6.2f}")
