"""Diagnostic: per-cell K1 (k_path) counters — PDAS iterations, pieces, shader cycles.

Loads the LOMPC_K1_STATS build (lompc_amd/liblompc_amd_k1stats.so, built by
``python scripts/k1_stats.py --build`` here) instead of the product library and
runs the bench's parameter sets (12 partitions, N=24, lambda ~ theta U[0,1]).
"""
import ctypes
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "incentive-design-mpc_amd"))
from lompc_amd import _lib, build  # noqa: E402

DBG = os.path.join(ROOT, "incentive-design-mpc_amd", "lompc_amd", "liblompc_amd_k1stats.so")

if "--build" in sys.argv:
    print(build.build(force=True, verbose=True, out=DBG, defines=("LOMPC_K1_STATS",)))
    sys.exit(0)

import torch  # noqa: E402

lib = _lib.load(DBG)
_lib._lib = lib
lib.lompc_debug_k1_stats.restype = ctypes.c_int
lib.lompc_debug_k1_stats.argtypes = [ctypes.c_void_p, ctypes.c_int]
from lompc_amd import LoMPC, LoMPCConstants  # noqa: E402

N, P, G = int(os.environ.get("K1_N", "24")), 12, int(os.environ.get("K1_G", "64"))
rng = np.random.default_rng(0)
for name, c in [("small", LoMPCConstants(0.05, 10.0, 0.9, 0.25, "small")),
                ("large", LoMPCConstants(0.025, 50.0, 0.9, 0.15, "large"))]:
    lompc = LoMPC(N, c, device=0, mode="path")
    for rep in range(3):
        lm = torch.as_tensor(c.theta * rng.random((P, 3 * N)), device="cuda")
        lompc.set_params(lm, torch.zeros(P, dtype=torch.float64, device="cuda"),
                         w_ref=torch.as_tensor(c.w_max * rng.random((P, N)), device="cuda"))
        torch.cuda.synchronize()
        buf = np.zeros(P * G * 4, dtype=np.int64)
        assert lib.lompc_debug_k1_stats(buf.ctypes.data, buf.size) == 0
        st = buf.reshape(P, G, 4)
        nit, npc, cs, ct = st[..., 0], st[..., 1], st[..., 2], st[..., 3]
        tot = cs + ct
        i = np.unravel_index(np.argmax(tot), tot.shape)
        print(f"{name} rep{rep}: pdas it mean {nit.mean():.2f} max {nit.max()} | pieces mean {npc.mean():.2f} "
              f"max {npc.max()} total/set {npc.sum(1).mean():.1f} | cyc solve mean {cs.mean():.0f} max {cs.max()} "
              f"| track mean {ct.mean():.0f} max {ct.max()} | slowest cell {i} nit {nit[i]} npc {npc[i]} "
              f"solve {cs[i]} track {ct[i]} | per PDAS it {(cs / np.maximum(nit, 1)).mean():.0f} "
              f"per piece {(ct / np.maximum(npc, 1)).mean():.0f}")
        if rep == 2:
            print("  nit histogram", np.bincount(nit.ravel()))
            print("  npc histogram", np.bincount(npc.ravel()))
