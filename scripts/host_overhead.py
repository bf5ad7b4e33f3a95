"""Diagnostic: host enqueue cost of one lompc_run (BatchPlan.run) vs. GPU time per step.

Prints, for the bench workload (131072 EVs per type, N=24, 12 sets):
  enqueue-only time per call (no synchronisation, queue kept shallow),
  wall time per step with one type and with both types on two streams,
  with and without the HIP-event profiling the bench uses.
"""
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "incentive-design-mpc_amd"))
from lompc_amd import BatchPlan, LoMPC, LoMPCConstants  # noqa: E402

N, P, M = 24, 12, 131072
rng = np.random.default_rng(0)
eng = []
for c in (LoMPCConstants(0.05, 10.0, 0.9, 0.25, "small"), LoMPCConstants(0.025, 50.0, 0.9, 0.15, "large")):
    lompc = LoMPC(N, c, device=0)
    off = np.array([(M * p) // P for p in range(P + 1)], dtype=np.int64)
    g = torch.as_tensor(c.y_max - (0.3 + 0.2 * rng.random(M)), device="cuda")
    lm = torch.as_tensor(c.theta * rng.random((8, P, 3 * N)), device="cuda")
    lr = torch.zeros(P, dtype=torch.float64, device="cuda")
    st = torch.cuda.Stream()
    plan = BatchPlan(lompc, g, off, want_w=True, want_cost=True, want_set=True, stream=st)
    eng.append(dict(lompc=lompc, plan=plan, lm=[lm[k].data_ptr() for k in range(8)], lr=lr.data_ptr(), st=st,
                    lm_t=lm, g=g, off=off))


def steps(n, which, prof):
    for e in which:
        e["lompc"].profile(enable=prof)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    tq = 0.0
    for k in range(n):
        for e in which:
            a = time.perf_counter()
            e["plan"].run(e["lm"][k % 8], e["lr"])
            tq += time.perf_counter() - a
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    for e in which:
        e["lompc"].profile(read=True, reset=True)
        e["lompc"].profile(enable=False)
        e["rep"] = int(e["plan"].out["set_stats"][:, 5].sum().item()), int(e["plan"].out["set_stats"][:, 6].sum().item())
    return dt / n * 1e6, tq / (n * len(which)) * 1e6


for prof in (False, True):
    steps(20, eng, prof)
    for name, which in (("small only", eng[:1]), ("large only", eng[1:]), ("both types", eng)):
        per_step, per_call = steps(200, which, prof)
        print(f"profile={prof!s:5s} {name:11s}: {per_step:7.1f} us/step, host enqueue {per_call:6.1f} us per lompc_run"
              f"  (repaired, failed in last step: {[e['rep'] for e in which]})")

# per price vector: repairs / failures and GPU time of one run (synchronised)
dump = {}
for e, name in zip(eng, ("small", "large")):
    for k in range(8):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        o = e["plan"].run(e["lm"][k], e["lr"])
        torch.cuda.synchronize()
        dt = 1e6 * (time.perf_counter() - t0)
        st = o["status"].cpu().numpy() if o["status"] is not None else None
        stats = o["set_stats"].cpu().numpy()
        nrep = int(stats[:, 5].sum())
        nfail = int(stats[:, 6].sum())
        print(f"{name} lambda[{k}]: {dt:8.1f} us (incl. sync), repaired {nrep}, failed {nfail}, "
              f"failed per set {stats[:, 6].astype(int).tolist()}")
        if nfail:
            s_bad = int(np.argmax(stats[:, 6]))
            dump[f"{name}_{k}_lmbd"] = e["lm_t"][k][s_bad].cpu().numpy()
            dump[f"{name}_{k}_gamma"] = e["g"].cpu().numpy()[e["off"][s_bad]:e["off"][s_bad + 1]]
os.makedirs("gpurun_out", exist_ok=True)
np.savez("gpurun_out/host_failures.npz", **dump)
