"""Kernel-time sweep over the batch size (diagnostic): k_eval / k_direct average
launch time (HIP events) and effective GB/s at 8(N+2) B per QP."""
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "incentive-design-mpc_amd"))
from lompc_amd import BatchPlan, LoMPC, LoMPCConstants  # noqa: E402

torch.cuda.set_device(0)
N = int(os.environ.get("N", "24"))
P = 12
for mode in ("path", "direct"):
    for ev, c in (("small", LoMPCConstants(0.05, 10.0, 0.9, 0.25, "small")),
                  ("large", LoMPCConstants(0.025, 50.0, 0.9, 0.15, "large"))):
        for M in (16384, 131072, 1048576, 4194304):
            if mode == "direct" and M > 1048576:
                continue
            rng = np.random.default_rng(0)
            lo = LoMPC(N, c, device=0, mode=mode)
            off = np.array([(M * p) // P for p in range(P + 1)], dtype=np.int64)
            g = torch.as_tensor(c.y_max - (0.3 + 0.2 * rng.random(M)), device="cuda:0")
            lm = torch.as_tensor(c.theta * rng.random((P, 3 * N)), device="cuda:0")
            lr = torch.zeros(P, dtype=torch.float64, device="cuda:0")
            plan = BatchPlan(lo, g, off, w_ref=torch.zeros(P, N, dtype=torch.float64, device="cuda:0"))
            for _ in range(3):
                plan.run(lm, lr)
            lo.check_last()
            lo.profile(enable=True)
            lo.profile(read=True, reset=True)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            reps = 20
            for _ in range(reps):
                plan.run(lm, lr)
            torch.cuda.synchronize()
            dt = (time.perf_counter() - t0) / reps
            ms, n = lo.profile(read=True)
            us = ms / n * 1e3
            print(f"{mode:6s} {ev:5s} N={N} M={M:8d}  kernel {us:8.1f} us  {8*(N+2)*M/us/1e3:7.1f} GB/s  "
                  f"{M/us*1e6:.3e} QP/s(kernel)  call {dt*1e6:8.1f} us  {M/dt:.3e} QP/s(call)", flush=True)
            del plan, lo
