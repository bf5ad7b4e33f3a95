"""Diagnostic: where a fused device price-loop iteration (k_loop_iter) spends its time.

    python scripts/loop_stamps.py --build   # here: lompc_amd/liblompc_amd_lstamps.so (LOMPC_STAMPS)
    python scripts/loop_stamps.py [station]  # on the GPU box: 3 config-5 closed-loop steps (default)
    python scripts/loop_stamps.py N [EVS]    # one large-EV PriceSolver, 5 calls of its device loop

Runs device price loops on the diagnostic build and prints, per
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

# --lib NAME: lompc_amd/liblompc_amd_NAME.so (a variant: scripts/build_variant.py NAME LOMPC_STAMPS
# LOMPC_STAMPS_RT ...); default the plain diagnostic build
LIB = sys.argv[sys.argv.index("--lib") + 1] if "--lib" in sys.argv else "lstamps"
if "--lib" in sys.argv:
    i = sys.argv.index("--lib")
    del sys.argv[i:i + 2]
CELLS = None  # --cells G: the station's loop plans with G path cells per set
if "--cells" in sys.argv:
    i = sys.argv.index("--cells")
    CELLS = int(sys.argv[i + 1])
    del sys.argv[i:i + 2]
DBG = os.path.join(ROOT, "incentive-design-mpc_amd", "lompc_amd", f"liblompc_amd_{LIB}.so")
if "--build" in sys.argv:
    print(build.build(force=True, out=DBG, defines=("LOMPC_STAMPS", "LOMPC_STAMPS_RT")))
    sys.exit(0)

import torch  # noqa: E402

torch.zeros(1, device="cuda")  # (HIP initialised by torch before the diagnostic library loads)
print("torch devices:", torch.cuda.device_count(), flush=True)
lib = _lib.load(DBG)
_lib._lib = lib
lib.lompc_debug_loopstamps.restype = ctypes.c_int
lib.lompc_debug_loopstamps.argtypes = [ctypes.c_void_p, ctypes.c_int]

from lompc_amd import LoMPCConstants, settings  # noqa: E402
from lompc_amd.price_solver import PriceSolver  # noqa: E402

settings.PRINT_LEVEL = 0
mode = sys.argv[1] if len(sys.argv) > 1 else "station"
buf = np.zeros(64 * 16, dtype=np.uint64)
tot = np.zeros((64, 16))
if mode == "station":
    # config 5 on one GPU (bench.py's station leg): 3 closed-loop steps after one warmup step
    from lompc_amd.charging_station import ChargingStation  # noqa: E402
    from lompc_amd.example import DEMAND_SCALE, NUM_EVS_PER_EV_TYPE, station_consts  # noqa: E402

    M_2, N, P = 1048576, 48, 12
    consts = station_consts(8, M_2, n_lo=N, n_bi=N, partitions=P, price_type="linear-convex",
                            demand_scale=DEMAND_SCALE * M_2 / NUM_EVS_PER_EV_TYPE, u_b_max=0.5, x_max=0.5)
    np.random.seed(0)
    st = ChargingStation(consts, device=0)
    st.price_solver_s.loop_cells = st.price_solver_l.loop_cells = CELLS
    st._step()
    torch.cuda.synchronize()
    assert lib.lompc_debug_loopstamps(buf.ctypes.data, 1) == 0
    for _ in range(3):
        st._step()
    torch.cuda.synchronize()
    assert lib.lompc_debug_loopstamps(buf.ctypes.data, 0) == 0
    tot += buf.reshape(64, 16).astype(np.float64)
    ps_l = st.price_solver_l
    last = max(ps_l._staged)  # (the chains run the staged plans: take the large type's last partition)
    ps_l.use_partition(last)
    G = ps_l._plan.cells
    # one more price loop of the large type's last partition, warm (its plan and prices as left):
    # the per-wave path phases of its last k_loop_iter launch (path_cell's stamps)
    lib.lompc_debug_stamps.restype = ctypes.c_int
    lib.lompc_debug_stamps.argtypes = [ctypes.c_void_p, ctypes.c_int]
    ps_l.compute_optimal_prices(0.5 * ps_l.consts.w_max * np.ones(N), 0.0)
    torch.cuda.synchronize()
    sb = np.zeros(65536 * 8, dtype=np.int64)
    assert lib.lompc_debug_stamps(sb.ctypes.data, sb.size) == 0
    ws = sb.reshape(65536, 8)[: 2 * G].astype(np.float64)
    d = np.stack([ws[:, 1] - ws[:, 0], ws[:, 2] - ws[:, 1], ws[:, 3] - ws[:, 2], ws[:, 3] - ws[:, 0]], 1) * 0.01
    for k, nm in enumerate(("setup", "solve@start", "tracking", "total")):
        print(f"   path {nm:12s} us: set 0 mean {d[:G, k].mean():5.2f} max {d[:G, k].max():5.2f};"
              f" set 1 mean {d[G:, k].mean():5.2f} max {d[G:, k].max():5.2f}")
    nit = sb.reshape(65536, 8)[: 2 * G, 4]
    print("   path iterations fp32 / fp64 per wave:", [(int(x // 256 % 256), int(x % 256)) for x in nit[:G]],
          " pieces:", [int(x) for x in sb.reshape(65536, 8)[:G, 6]])
    iters = -1
    EVS = M_2 // P
else:
    N = int(mode)
    EVS = int(sys.argv[2]) if len(sys.argv) > 2 else 87381
    lc = LoMPCConstants(0.025, 50.0, 0.9, 0.15, "large")
    rng = np.random.default_rng(3)
    ps = PriceSolver(N, lc, "linear-convex", device=0)
    ps.loop_cells = CELLS
    iters = 0
    for call in range(6):
        ps.set_charge_levels(0.3 + 0.3 * lc.y_max * rng.random(EVS))
        w_ref = lc.w_max * (0.2 + 0.6 * rng.random(N))
        assert lib.lompc_debug_loopstamps(buf.ctypes.data, 1) == 0
        _, res = ps.compute_optimal_prices(w_ref, 0.0)
        torch.cuda.synchronize()
        assert lib.lompc_debug_loopstamps(buf.ctypes.data, 0) == 0
        if call == 0:
            continue  # (first call: allocation, plan build)
        tot += buf.reshape(64, 16).astype(np.float64)
        iters += res["iter"] + 1
    G = ps._plan.cells
W = 2 * G
t = tot[:W]
us = 0.01  # s_memrealtime: 100 MHz
launches = t[:, 5].sum() / W
print(f"{LIB}: N={N} EVs={EVS} cells={G} launches={launches:.0f} (engine calls {iters})")
for k, nm in enumerate(("path", "aggregation", "record+arrival")):
    print(f"   {nm:16s} mean {t[:, k].sum() / t[:, 5].sum() * us:6.2f} us per wave")
print(f"   {'set closing':16s} mean {(t[:, 3] + t[:, 10]).sum() / max(t[:, 6].sum(), 1) * us:6.2f} us ({t[:, 6].sum():.0f} closings)")
print(f"   {'loop step':16s} mean {(t[:, 4] + t[:, 8] + t[:, 9]).sum() / max(t[:, 7].sum(), 1) * us:6.2f} us ({t[:, 7].sum():.0f} steps)")
ns, nc = max(t[:, 7].sum(), 1), max(t[:, 6].sum(), 1)
print(f"      closing: records' load round {t[:, 10].sum() / nc * us:5.2f}, sums + stores {t[:, 3].sum() / nc * us:5.2f};"
      f"  step: inputs + error {t[:, 8].sum() / ns * us:5.2f}, price QP {t[:, 9].sum() / ns * us:5.2f},"
      f" next prices + publish {t[:, 4].sum() / ns * us:5.2f}")
print("   per wave: path mean us " + " ".join(f"{x:5.1f}" for x in t[:, 0] / np.maximum(t[:, 5], 1) * us))
print("             agg  mean us " + " ".join(f"{x:5.1f}" for x in t[:, 1] / np.maximum(t[:, 5], 1) * us))
print("             closings     " + " ".join(f"{x:5.0f}" for x in t[:, 6]))
