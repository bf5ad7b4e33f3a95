"""Diagnostic: K1 (k_path) per-cell counters on the closed-loop station's own price iterations
(config-5 shape, N = 48).  Runs the station on the LOMPC_K1_STATS build (LOMPC_LIB, built by
``python scripts/k1_stats.py --build``) and reads the counters after every engine call."""
import ctypes
import os
import sys

os.environ["LOMPC_LIB"] = os.environ.get("K1_LIB", "liblompc_amd_k1stats.so")
import numpy as np  # noqa: E402
import torch  # noqa: E402

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "incentive-design-mpc_amd"))
from lompc_amd import _lib, settings  # noqa: E402
from lompc_amd import lompc as L  # noqa: E402
from lompc_amd.charging_station import ChargingStation  # noqa: E402
from lompc_amd.example import DEMAND_SCALE, NUM_EVS_PER_EV_TYPE, station_consts  # noqa: E402

N, M_2 = 48, int(os.environ.get("M2", "131072"))
settings.PRINT_LEVEL = 0
torch.cuda.set_device(0)
lib = _lib.load()
lib.lompc_debug_k1_stats.restype = ctypes.c_int
lib.lompc_debug_k1_stats.argtypes = [ctypes.c_void_p, ctypes.c_int]
rows = []
orig = L.BatchPlan.run


def run(self, lmbd, lmbd_r):
    out = orig(self, lmbd, lmbd_r)
    torch.cuda.synchronize()
    buf = np.zeros(self.S * 64 * 4, dtype=np.int64)
    assert lib.lompc_debug_k1_stats(buf.ctypes.data, buf.size) == 0
    st = buf.reshape(self.S, 64, 4)
    rows.append((self.lompc.ev_type, self.S, st[..., 0].max(), st[..., 1].max(), (st[..., 2] + st[..., 3]).max(),
                 st[..., 2].max(), st[..., 3].max()))
    return out


L.BatchPlan.run = run
consts = station_consts(3, M_2, n_lo=N, n_bi=N, demand_scale=DEMAND_SCALE * M_2 / NUM_EVS_PER_EV_TYPE,
                        u_b_max=0.5, x_max=0.5)
np.random.seed(0)
st = ChargingStation(consts, device=0)
for _ in range(2):
    st._step() if hasattr(st, "_step") else st.step()
r = np.array([x[2:] for x in rows], dtype=np.float64)
print(f"{len(rows)} engine calls; per call max over cells: nit mean {r[:, 0].mean():.1f} max {r[:, 0].max():.0f} | "
      f"pieces mean {r[:, 1].mean():.1f} max {r[:, 1].max():.0f} | cycles mean {r[:, 2].mean():.0f} "
      f"max {r[:, 2].max():.0f} (solve max {r[:, 3].max():.0f}, track max {r[:, 4].max():.0f})")
for ev in ("small", "large"):
    rr = np.array([x[2:] for x in rows if x[0] == ev])
    if len(rr):
        print(ev, len(rr), "calls: cycles mean %.0f p90 %.0f max %.0f; nit mean %.1f max %.0f" % (
            rr[:, 2].mean(), np.percentile(rr[:, 2], 90), rr[:, 2].max(), rr[:, 0].mean(), rr[:, 0].max()))
