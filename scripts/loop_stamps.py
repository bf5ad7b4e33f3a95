"""Diagnostic: where a fused device price-loop iteration (k_loop_iter) spends its time.

    python scripts/loop_stamps.py --build   # here: lompc_amd/liblompc_amd_lstamps.so (LOMPC_STAMPS)
    python scripts/loop_stamps.py [N] [EVS] # on the GPU box (default N 48, 87381 EVs: one config-5 partition)

Runs a large-EV PriceSolver's device loop a few times on the diagnostic build and prints, per
phase, the mean s_memrealtime span per wave and launch (path, aggregation, record + arrival), per
set closing and per loop step, plus the closing and stepping waves' own path + aggregation (the
launch's critical path: the last arrivers).
"""
import ctypes
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "incentive-design-mpc_amd"))
from lompc_amd import _lib, build  # noqa: E402

DBG = os.path.join(ROOT, "incentive-design-mpc_amd", "lompc_amd", "liblompc_amd_lstamps.so")
if "--build" in sys.argv:
    print(build.build(force=True, out=DBG, defines=("LOMPC_STAMPS", "LOMPC_STAMPS_RT")))
    sys.exit(0)

lib = _lib.load(DBG)
_lib._lib = lib
lib.lompc_debug_loopstamps.restype = ctypes.c_int
lib.lompc_debug_loopstamps.argtypes = [ctypes.c_void_p, ctypes.c_int]

import torch  # noqa: E402

from lompc_amd import LoMPCConstants, settings  # noqa: E402
from lompc_amd.price_solver import PriceSolver  # noqa: E402

settings.PRINT_LEVEL = 0
N = int(sys.argv[1]) if len(sys.argv) > 1 else 48
EVS = int(sys.argv[2]) if len(sys.argv) > 2 else 87381
lc = LoMPCConstants(0.025, 50.0, 0.9, 0.15, "large")
rng = np.random.default_rng(3)
ps = PriceSolver(N, lc, "linear-convex", device=0)
buf = np.zeros(64 * 8, dtype=np.uint64)
tot = np.zeros((64, 8))
iters = 0
for call in range(6):
    ps.set_charge_levels(0.3 + 0.3 * lc.y_max * rng.random(EVS))
    w_ref = lc.w_max * (0.2 + 0.6 * rng.random(N))
    assert lib.lompc_debug_loopstamps(buf.ctypes.data, 1) == 0
    _, st = ps.compute_optimal_prices(w_ref, 0.0)
    torch.cuda.synchronize()
    assert lib.lompc_debug_loopstamps(buf.ctypes.data, 0) == 0
    if call == 0:
        continue  # (first call: allocation, plan build)
    tot += buf.reshape(64, 8).astype(np.float64)
    iters += st["iter"] + 1
G = ps._plan.cells
W = 2 * G
t = tot[:W]
us = 0.01  # s_memrealtime: 100 MHz
launches = t[:, 5].sum() / W
print(f"N={N} EVs={EVS} cells={G} launches={launches:.0f} (engine calls {iters})")
for k, nm in enumerate(("path", "aggregation", "record+arrival")):
    print(f"   {nm:16s} mean {t[:, k].sum() / t[:, 5].sum() * us:6.2f} us per wave")
print(f"   {'set closing':16s} mean {t[:, 3].sum() / max(t[:, 6].sum(), 1) * us:6.2f} us ({t[:, 6].sum():.0f} closings)")
print(f"   {'loop step':16s} mean {t[:, 4].sum() / max(t[:, 7].sum(), 1) * us:6.2f} us ({t[:, 7].sum():.0f} steps)")
print("   per wave: path mean us " + " ".join(f"{x:5.1f}" for x in t[:, 0] / np.maximum(t[:, 5], 1) * us))
print("             agg  mean us " + " ".join(f"{x:5.1f}" for x in t[:, 1] / np.maximum(t[:, 5], 1) * us))
print("             closings     " + " ".join(f"{x:5.0f}" for x in t[:, 6]))
