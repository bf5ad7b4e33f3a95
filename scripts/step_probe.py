"""Diagnostics: the stepped run_steps at config 3 on one or several library builds, one process.

    python scripts/step_probe.py [lib.so ...] [--cells G] [--steps K] [--reps R] [--outputs full|set]

For every in-tree library (lompc_amd/<lib>.so, default the product library; variants are -D builds
made by scripts/build_variant.py) and every cell count: K steps per lompc_plan_run_steps call with
per-step set outputs, R calls; prints the per-step wall time (median over the calls), the k_step
average from one HIP-event pair spanning the steady-state launches, and the standalone kernels
(k_path / k_eval / k_finalize as their own launches, 20 single runs).  Not a measurement of record:
bench.py is (it refuses variant libraries).
"""
import argparse
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "incentive-design-mpc_amd"))
ap = argparse.ArgumentParser()
ap.add_argument("libs", nargs="*", default=["liblompc_amd.so"])
ap.add_argument("--cells", type=int, nargs="*", default=[0])
ap.add_argument("--steps", type=int, default=20)
ap.add_argument("--reps", type=int, default=5)
ap.add_argument("--outputs", default="full")
ap.add_argument("--horizon", type=int, default=24)
ap.add_argument("--evs", type=int, default=262144)
ap.add_argument("--warmup", type=int, default=0, help="warmup call's runs (0: --steps)")
ap.add_argument("--gpu-span", action="store_true", help="torch events around each timed call")
ap.add_argument("--idle-ms", type=float, default=0.0, help="host sleep before each timed call (GPU idle)")
ap.add_argument("--warm-events", action="store_true", help="the warmup call carries the span events")
ap.add_argument("--spin", action="store_true", help="hipSetDeviceFlags(hipDeviceScheduleSpin) before torch")
args = ap.parse_args()

if args.spin:
    import ctypes

    _hip = ctypes.CDLL("libamdhip64.so")
    print("hipSetDeviceFlags(spin):", _hip.hipSetDeviceFlags(1), flush=True)

import torch  # noqa: E402

from lompc_amd import _lib  # noqa: E402

N, P, B = args.horizon, 12, args.evs
for libname in args.libs:
    lib = _lib.load(os.path.join(ROOT, "incentive-design-mpc_amd", "lompc_amd", libname))
    _lib._lib = lib
    from lompc_amd import BatchPlan, LoMPC, LoMPCConstants  # noqa: E402

    rng = np.random.default_rng(0)
    cs = [LoMPCConstants(0.05, 10.0, 0.9, 0.25, "small"), LoMPCConstants(0.025, 50.0, 0.9, 0.15, "large")]
    lompcs = [LoMPC(N, c, device=0) for c in cs]
    M = B // 2
    off1 = np.array([(M * p) // P for p in range(P + 1)], dtype=np.int64)
    off = np.concatenate([off1, M + off1[1:]])
    g = torch.as_tensor(np.concatenate([c.y_max - (0.3 + 0.2 * rng.random(M)) for c in cs]), device="cuda")
    K = args.steps
    lm = torch.as_tensor(np.stack([np.concatenate([c.theta * rng.random((P, 3 * N)) for c in cs]) for _ in range(K)]),
                         device="cuda")
    lr = torch.zeros((K, 2 * P), dtype=torch.float64, device="cuda")
    wr = torch.as_tensor(np.concatenate([c.w_max * rng.random((P, N)) for c in cs]), device="cuda")
    for cells in args.cells:
        plan = BatchPlan(lompcs, g, off, sets_per_ctx=[P, P], w_ref=wr, want_w=args.outputs == "full",
                         want_cost=args.outputs != "set", cells=cells or None)
        if args.warm_events:
            plan.profile(enable=("k_eval",))
        plan.run_steps(lm, lr, args.warmup or K, lm[0].numel(), lr[0].numel(), per_run_sets=True,
                       span_events=args.warm_events)
        plan.check()
        walls, ks, spans = [], [], []
        go, _ = plan.steps_call(lm, lr, K, lm[0].numel(), lr[0].numel(), per_run_sets=True, span_events=True)
        ea, eb = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        for _ in range(args.reps):
            plan.profile(enable=("k_eval",))
            plan.profile(read=True, reset=True)
            torch.cuda.synchronize()
            if args.idle_ms:
                time.sleep(args.idle_ms / 1e3)
            t0 = time.perf_counter()
            if args.gpu_span:
                ea.record()
            go()
            if args.gpu_span:
                eb.record()
            torch.cuda.synchronize()
            walls.append((time.perf_counter() - t0) / K * 1e6)
            if args.gpu_span:
                spans.append(ea.elapsed_time(eb) * 1e3 / K)
            ms, n = plan.profile(read=True)
            ks.append(ms / max(n, 1) * 1e3)
            rep = plan.check()[0]
        plan.profile(enable=("k_path", "k_eval", "k_finalize"))
        for k in ("k_path", "k_eval", "k_finalize"):
            plan.profile(read=True, reset=True, kernel=k)
        wide = []
        for _ in range(3):  # the wide call's own kernels: k_paths per launch, k_evals / k_closes per run
            plan.run_steps(lm, lr, K, lm[0].numel(), lr[0].numel(), per_run_sets=True)
            wide.append({k: plan.profile(read=True, reset=True, kernel=k) for k in ("k_path", "k_eval", "k_finalize")})
        print("   wide call: " + " | ".join(
            "  ".join(f"{k} {ms * 1e3:.1f} us / {n}" for k, (ms, n) in w.items()) for w in wide), flush=True)
        for j in range(20):
            plan.run(lm[j % K], lr[j % K])
        plan.check()
        alone = {k: plan.profile(read=True, kernel=k) for k in ("k_path", "k_eval", "k_finalize")}
        plan.profile(enable=False)
        # host cost of the call itself (Python wrapper + C-ABI entry, no launch: n_runs = 0) — GPU idle
        # time at the start of a timed call
        outs = {k: torch.empty((0,) + tuple(plan.out[k].shape), dtype=torch.float64, device="cuda")
                for k in ("set_sum_w", "set_stats")}
        t0 = time.perf_counter()
        for _ in range(200):
            plan.run_steps(lm, lr, 0, lm[0].numel(), lr[0].numel(), out=outs)
        wrap_us = (time.perf_counter() - t0) / 200 * 1e6
        print(f"   run_steps call overhead (n_runs = 0, out given): {wrap_us:6.1f} us", flush=True)
        print(f"{libname} cells {plan.cells} {args.outputs}: per step {np.median(walls):6.2f} us (min {min(walls):6.2f})"
              f"  k_step {np.median(ks):6.2f} us  alone: " +
              "  ".join(f"{k} {ms / max(n, 1) * 1e3:6.2f}" for k, (ms, n) in alone.items()) +
              f"  repaired per step {rep / K:.0f}", flush=True)
        print("   every call (us per step): " + " ".join(f"{v:.2f}" for v in walls), flush=True)
        if spans:
            print("   GPU span (us per step):   " + " ".join(f"{v:.2f}" for v in spans), flush=True)
        del plan
