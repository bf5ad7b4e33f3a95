"""Diagnostic: the wide form's batched evaluation (k_evals) on a timeline, from s_memrealtime stamps.

    python scripts/evals_stamps.py --build   # here: lompc_amd/liblompc_amd_stamps_rt.so (LOMPC_STAMPS, _RT)
    python scripts/evals_stamps.py           # on the GPU box: config 3, K = 20 steps in one run_steps call

Per (workgroup, run): start, staging done (the barrier after the piece table is in LDS), rows issued,
end (after the record).  Prints per-run phase medians / p90, the launch's span, and a timeline of how
many workgroups are in each phase (10 bins per run-equivalent).  100 MHz clock (10 ns).
"""
import ctypes
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "incentive-design-mpc_amd"))
from lompc_amd import _lib, build  # noqa: E402

NOSTAGE = "--nostage" in sys.argv  # (runs after the first keep run 0's staged table: LQ_EVALS_NOSTAGE)
DBG = os.path.join(ROOT, "incentive-design-mpc_amd", "lompc_amd",
                   os.environ.get("ES_LIB", "liblompc_amd_stamps_rt%s.so" % ("_nostage" if NOSTAGE else "")))
if "--build" in sys.argv:
    print(build.build(force=True, out=DBG, defines=("LOMPC_STAMPS", "LOMPC_STAMPS_RT") +
                      (("LQ_EVALS_NOSTAGE",) if NOSTAGE else ())))
    sys.exit(0)

import torch  # noqa: E402

lib = _lib.load(DBG)
_lib._lib = lib
lib.lompc_debug_stamps.restype = ctypes.c_int
lib.lompc_debug_stamps.argtypes = [ctypes.c_void_p, ctypes.c_int]
from lompc_amd import BatchPlan, LoMPC, LoMPCConstants  # noqa: E402

N, P, B, K = 24, 12, 262144, 20
rng = np.random.default_rng(0)
cs = [LoMPCConstants(0.05, 10.0, 0.9, 0.25, "small"), LoMPCConstants(0.025, 50.0, 0.9, 0.15, "large")]
lompcs = [LoMPC(N, c, device=0) for c in cs]
M = B // 2
off1 = np.array([(M * p) // P for p in range(P + 1)], dtype=np.int64)
off = np.concatenate([off1, M + off1[1:]])
g = torch.as_tensor(np.concatenate([c.y_max - (0.3 + 0.2 * rng.random(M)) for c in cs]), device="cuda")
lm = torch.as_tensor(np.stack([np.concatenate([c.theta * rng.random((P, 3 * N)) for c in cs]) for _ in range(K)]),
                     device="cuda")
lr = torch.zeros((K, 2 * P), dtype=torch.float64, device="cuda")
wr = torch.as_tensor(np.concatenate([c.w_max * rng.random((P, N)) for c in cs]), device="cuda")
SET_ONLY = "--set" in sys.argv  # (the reductions-only contract: no per-EV outputs, the per-piece sums)
CELLS = int(os.environ.get("ES_CELLS", "4"))
plan = BatchPlan(lompcs, g, off, sets_per_ctx=[P, P], w_ref=wr, want_w=not SET_ONLY, want_cost=not SET_ONLY,
                 cells=CELLS)
for _ in range(3):
    plan.run_steps(lm, lr, K, lm[0].numel(), lr[0].numel(), per_run_sets=True)
plan.check()
torch.cuda.synchronize()
nb = plan.info()["workgroups"]
buf = np.zeros(512 * 32 * 8, dtype=np.int64)
assert lib.lompc_debug_stamps(buf.ctypes.data, buf.size) == 0
st8 = buf.reshape(512, 32, 8)[:nb, :K].astype(np.float64) * 10e-3  # us
t0 = st8[:, 0, 0].min()
st8 -= t0
st = st8[:, :, [0, 5, 6, 7]]  # start, staged, rows done, end
span = st[:, :, 3].max()
print(f"workgroups {nb}, runs {K}, cells {CELLS}{' (nostage)' if NOSTAGE else ''}{' (set only)' if SET_ONLY else ''}: launch span (first start .. last end) "
      f"{span:.2f} us = {span / K:.2f} us per run")
ph = {"blockmap": st8[:, :, 1] - st8[:, :, 0], "scalars": st8[:, :, 2] - st8[:, :, 1],
      "counts": st8[:, :, 3] - st8[:, :, 2], "pieces": st8[:, :, 4] - st8[:, :, 3],
      "lds+bar": st8[:, :, 5] - st8[:, :, 4], "staging": st[:, :, 1] - st[:, :, 0],
      "rows": st[:, :, 2] - st[:, :, 1], "record": st[:, :, 3] - st[:, :, 2], "run": st[:, :, 3] - st[:, :, 0]}
for k, v in ph.items():
    v = v[:, 1:]  # (runs after the first)
    print(f"  {k:8s} median {np.median(v):6.2f}  p10 {np.percentile(v, 10):6.2f}  p90 {np.percentile(v, 90):6.2f}  "
          f"max {v.max():6.2f} us")
print("  per run (median over workgroups): start / staged / rows done / end")
for r in range(K):
    print(f"   run {r:2d}: " + " ".join(f"{np.median(st[:, r, k]):7.2f}" for k in range(4)) +
          f"   spread of starts {np.percentile(st[:, r, 0], 90) - np.percentile(st[:, r, 0], 10):5.2f}")
# timeline: workgroups staging / writing rows / in the record at each instant
bins = np.linspace(0, span, 10 * K + 1)
mid = 0.5 * (bins[1:] + bins[:-1])
stag = ((st[:, :, 0][..., None] <= mid) & (mid < st[:, :, 1][..., None])).sum(axis=(0, 1))
rows = ((st[:, :, 1][..., None] <= mid) & (mid < st[:, :, 2][..., None])).sum(axis=(0, 1))
print("  timeline (bin, us, WGs staging, WGs in rows):")
for i in range(0, len(mid), 2):
    print(f"   {mid[i]:7.2f}  {stag[i]:4d}  {rows[i]:4d}")
# per-workgroup totals: the launch ends with its slowest workgroup (static block map)
tot = st[:, -1, 3] - st[:, 0, 0]
print(f"  per-workgroup total: min {tot.min():.1f} p10 {np.percentile(tot, 10):.1f} median {np.median(tot):.1f} "
      f"p90 {np.percentile(tot, 90):.1f} max {tot.max():.1f} us (mean {tot.mean():.1f}); span {span:.1f}")
per = nb // (2 * P)
if per > 0:
    ms = [float(np.mean(tot[s * per:(s + 1) * per])) for s in range(2 * P)]
    print("  mean total by set (blocks in order):", " ".join(f"{m:.0f}" for m in ms))
print("  mean total by b % 8 (dispatch XCD):", " ".join(f"{np.mean(tot[x::8]):.1f}" for x in range(8)))
slow = np.argsort(tot)[-10:]
print("  slowest workgroups (b, total):", [(int(b), round(float(tot[b]), 1)) for b in slow])
half = (nb // (2 * P)) * P
for nm, sl in (("small sets", slice(0, half)), ("large sets", slice(half, nb))):
    print(f"  {nm}: " + "  ".join(f"{k} {np.median(v[sl, 1:]):.2f}" for k, v in ph.items()))
cnt = np.zeros(2 * P * CELLS, dtype=np.int32)
lib.lompc_debug_plan_tables.argtypes = [ctypes.c_void_p] * 7
lib.lompc_debug_plan_tables(plan._plan, cnt.ctypes.data, None, None, None, None, None)
print("  pieces per cell (last single-run table) small:", cnt[:P * CELLS].mean(), " large:", cnt[P * CELLS:].mean())
