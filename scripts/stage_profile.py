"""Diagnostic: the Python / C-ABI cost of a closed-loop station step's partition staging
(ChargingStation._stage_partitions: per EV type the partition layout, the gamma layout and one
PriceSolver.stage_partition per partition).  The staging threads run synchronously on the main
thread here (a stand-in executor), so cProfile sees them; config-5 shape (M2 EVs per type)."""
import concurrent.futures
import cProfile
import os
import pstats
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "incentive-design-mpc_amd"))
from lompc_amd import settings  # noqa: E402
from lompc_amd.charging_station import ChargingStation  # noqa: E402
from lompc_amd.example import DEMAND_SCALE, NUM_EVS_PER_EV_TYPE, station_consts  # noqa: E402

M_2 = int(os.environ.get("M2", "1048576"))
settings.PRINT_LEVEL = 0
torch.cuda.set_device(0)
WARM = int(os.environ.get("WARM", "20"))
consts = station_consts(WARM + 12, M_2, n_lo=48, n_bi=48, demand_scale=DEMAND_SCALE * M_2 / NUM_EVS_PER_EV_TYPE,
                        u_b_max=0.5, x_max=0.5)
np.random.seed(0)
st = ChargingStation(consts, device=0)


class Inline:  # runs each job at submit, on this thread
    def submit(self, fn, *a):
        f = concurrent.futures.Future()
        f.set_result(fn(*a))
        return f


for _ in range(WARM):
    st._step()
torch.cuda.synchronize()
print("---- steady state (threaded staging):", file=sys.stderr, flush=True)
for _ in range(4):
    st._step()
    torch.cuda.synchronize()
    print({k: (round(v, 3) if isinstance(v, float) else {a: round(x, 3) for a, x in v.items()})
           for k, v in st.bimpc_split.items()}, flush=True)
print("---- inline staging:", file=sys.stderr, flush=True)
st._stage_pool = Inline()
st._step()
torch.cuda.synchronize()
pr = cProfile.Profile()
steps = 3
t0 = time.perf_counter()
pr.enable()
for _ in range(steps):
    st._step()
pr.disable()
torch.cuda.synchronize()
print(f"step (staging inline) {(time.perf_counter() - t0) / steps * 1e3:.2f} ms; last split {st.bimpc_split}")
pstats.Stats(pr).sort_stats("tottime").print_stats(30)
pstats.Stats(pr).sort_stats("cumulative").print_stats(40)
