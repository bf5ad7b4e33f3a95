"""Benchmark: LoMPC QP solves/sec on MI355X (BASELINE.json metric, config 3/4).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--mode path|direct]
    torchrun --nproc-per-node N bench.py --gpus N ...   (one rank per GPU, RCCL)

One step = one batched price iteration of a whole charging-station time step on
this rank's EV shard: for each EV type (small, large) load P = 12 fresh
partition price vectors (lambda ~ theta U[0,1]^{3N}, test_lompc.py:34) and
solve every EV's LoMPC QP (gamma_i = y_max - y0_i, y0 ~ U[0.3, 0.5],
settings.py:27-28) with full outputs (w, cost) plus the fused per-partition
reductions of price_solver.py:203-214; with N > 1 ranks the per-partition
reductions of both types are exchanged by ONE RCCL all-gather per group of up to
64 steps (the extension's communicator, inside the same C-ABI call) and combined
in rank order on the device (k_combine_runs: local sum / max).  Weak scaling:
262 144 EVs per GPU (config 3; at 8 GPUs this is config 4's 2 097 152).

A single plan run is three kernels: k_path (per (set, gamma cell) solution paths), k_eval (per-EV
evaluation + rows) and k_finalize (per-set reductions and any individual re-solve).  The K timed
steps are independent runs (fresh prices each), issued by ONE lompc_plan_run_steps call in its
WIDE form: per group of up to 64 steps three launches — k_paths (every step's paths at once:
thousands of independent latency-bound chains), k_evals (each workgroup evaluates its block of EVs
for every step of the group in turn, no kernel boundary between steps) and k_closes (one workgroup
per (step, set): the closings).  Every step's work is done in full inside the timed region, and
the results equal the launch-per-kernel form bit for bit (verified after the timed region).

Rank 0 prints ONE JSON line.  ``roofline`` prices k_evals — the kernel that carries the per-EV
work — by the evaluation's algorithmic bytes per QP (gamma in 8 B, w out 8N B, cost out 8 B) over
its duration per step: ONE HIP-event pair around the first group's k_evals launch in the timed
region (hipExtLaunchKernel events on its own stream) divided by the group's steps; ``kernels``
gives each plan kernel's average duration as its own launch from a separate 20-step pass (after
the timed region) and PMC figures from profiles/ when they match this configuration;
``contracts`` the reference's other per-iteration shapes (reductions only, w0 only, every step's
rows to fresh HBM buffers, dependent steps); ``cpu_baseline`` the same path algorithm and the
dense C oracle (oracle/) on the host's cores over a bounded sample of the same workload;
``direct_mode`` the per-EV DIRECT mode on the same batch; ``bimpc`` the config-5 closed-loop
station step (BiMPC steps/sec).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "incentive-design-mpc_amd"))

HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: HBM3E 8.0 TB/s (spec)
FP64_VALU_PEAK_TFLOPS = 78.6  # vendor datasheet (not in the container guide)


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=100)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--evs-per-gpu", type=int, default=262144)
    ap.add_argument("--horizon", type=int, default=24)
    ap.add_argument("--partitions", type=int, default=12)
    ap.add_argument("--mode", choices=["path", "direct"], default="path")
    ap.add_argument("--seed", type=int, default=0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cells", type=int, default=4,
                    help="gamma cells per parameter set of the benchmark's plan (0: the plan's default, 16 at these "
                         "set sizes); 4 measured best for the wide run_steps form (scripts/step_probe.py, K = 20: "
                         "13.4 vs 14.3 us per step at 12 cells — k_paths 28 vs 38 us per call, k_evals 10.7 vs 11.1 "
                         "us per run; K = 100: 12.2 vs 12.5), at +2.6 us for one run's path alone (18.3 vs 15.7 us)")
    ap.add_argument("--warm", action="store_true",
                    help="plan warm start: every gamma cell's exact solve starts from the working set the "
                         "previous step ended with there (as a price loop's plan does)")
    ap.add_argument("--outputs", choices=["full", "cost", "set"], default="full",
                    help="diagnostics: full = w + cost + reductions (the metric's workload); cost = no w rows; "
                         "set = reductions only")
    ap.add_argument("--split-types", action="store_true",
                    help="path mode: one plan per EV type, each on its own stream (overlapping)")
    ap.add_argument("--no-kernel-events", action="store_true", help="= --kernel-events none")
    ap.add_argument("--kernel-events", choices=["span", "sampled", "none"], default="span",
                    help="HIP events of the timed region's stepped launches: span = ONE pair from the start of "
                         "the first full k_step dispatch to the end of the last (hipExtLaunchKernel events), "
                         "read as that many launches (each event boundary costs ~4.5 us of idle GPU, so no "
                         "boundary inside the steady state); sampled = a pair on every E-th launch")
    ap.add_argument("--event-every", type=int, default=4, help="--kernel-events sampled: every E-th launch")
    ap.add_argument("--per-step-issue", action="store_true",
                    help="diagnostics: issue each timed step from Python (one lompc_plan_run per step)")
    ap.add_argument("--cpu-seconds", type=float, default=10.0)
    ap.add_argument("--no-station", action="store_true", help="skip the BiMPC steps/sec leg")
    ap.add_argument("--station-evs-per-gpu", type=int, default=2097152,
                    help="EVs per GPU, half per type (default: config 5's 2 097 152 on one GPU)")
    ap.add_argument("--station-horizon", type=int, default=48)
    ap.add_argument("--station-steps", type=int, default=20)
    ap.add_argument("--station-warmup", type=int, default=3)
    ap.add_argument("--no-direct", action="store_true", help="skip the DIRECT-mode comparison leg")
    ap.add_argument("--dist-backend", choices=["nccl", "gloo"], default="nccl",
                    help="nccl = RCCL (the product path); gloo only to rehearse world > 1 on one GPU")
    ap.add_argument("--force-dist", action="store_true",
                    help="the sharded (N > 1) code path on one rank: a world-size-1 nccl group, every step's set "
                         "reductions all-gathered by the extension's RCCL communicator and combined on the device")
    ap.add_argument("--no-contracts", action="store_true",
                    help="skip the reductions-only / w0-only contract legs (the reference's _get_w_err / get_w0_price0)")
    ap.add_argument("--station-pl1-steps", type=int, default=4,
                    help="extra station steps at the reference's default PRINT_LEVEL = 1 (prints captured)")
    ap.add_argument("--station-prof-steps", type=int, default=4,
                    help="extra station steps with the price loops' per-part timing (after the timed steps)")
    return ap.parse_args()


def spawn_ranks(args) -> int:
    """--gpus N > 1 without a launcher: start the N rank processes (torch.distributed.run, one rank
    per GPU) from this process, which never touches HIP, and return their exit code; rank 0 prints
    the line."""
    import socket
    import subprocess

    so = socket.socket()
    so.bind(("127.0.0.1", 0))
    port = so.getsockname()[1]
    so.close()
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={args.gpus}",
           "--master-addr=127.0.0.1", f"--master-port={port}", os.path.abspath(__file__)] + sys.argv[1:]
    return subprocess.call(cmd)


def check_env():
    """No diagnostic knob may be set for a measured run (they select other libraries / forms)."""
    bad = sorted(k for k in os.environ if k.startswith("LOMPC_"))
    if bad:
        raise SystemExit(f"bench.py: diagnostic variables set ({', '.join(bad)}); unset them for a measured run")


def main():
    args = parse()
    if args.no_kernel_events:
        args.kernel_events = "none"
    check_env()
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(spawn_ranks(args))
    import torch
    import torch.distributed as dist

    from lompc_amd import BatchPlan, LoMPC, LoMPCConstants, _lib
    from lompc_amd.dist import combine_set_results

    from lompc_amd.dist import device_comm, release_comms

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:  # (a line must describe the ranks that ran)
        raise SystemExit(f"bench.py: --gpus {args.gpus} but WORLD_SIZE {world}")
    sharded = world > 1 or args.force_dist
    if world > 1:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        # one rank per GPU; with fewer GPUs than ranks (a gloo rehearsal on one card) ranks share
        ndev = torch.cuda.device_count()
        idx = local % max(ndev, 1)
        torch.cuda.set_device(idx)
        if args.dist_backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device(f"cuda:{idx}"))
        else:
            dist.init_process_group("gloo")
    else:
        torch.cuda.set_device(0)
        if args.force_dist:  # the N > 1 code path with one rank (RCCL allows one rank per device)
            import socket

            so = socket.socket()
            so.bind(("127.0.0.1", 0))
            port = so.getsockname()[1]
            so.close()
            if args.dist_backend == "nccl":
                dist.init_process_group("nccl", init_method=f"tcp://127.0.0.1:{port}", rank=0, world_size=1,
                                        device_id=torch.device("cuda:0"))
            else:
                dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=0, world_size=1)
    dev = torch.device(f"cuda:{torch.cuda.current_device()}")

    N, P = args.horizon, args.partitions
    B = args.evs_per_gpu
    types = [("small", LoMPCConstants(0.05, 10.0, 0.9, 0.25, "small")),
             ("large", LoMPCConstants(0.025, 50.0, 0.9, 0.15, "large"))]  # real_time_price_control.py:26-39
    rng = np.random.default_rng(args.seed * 1000 + rank)
    per_type = [B // 2, B - B // 2]
    nsteps = args.steps + args.warmup
    eng = []
    for (name, c), M in zip(types, per_type):
        lompc = LoMPC(N, c, device=dev.index, mode=args.mode)
        off = np.array([(M * p) // P for p in range(P + 1)], dtype=np.int64)  # P partitions
        y0 = 0.3 + 0.2 * rng.random(M)
        gamma = torch.as_tensor(c.y_max - y0, device=dev)
        lm = torch.as_tensor(c.theta * rng.random((nsteps, P, 3 * N)), device=dev)
        wr = torch.as_tensor(c.w_max * rng.random((P, N)), device=dev)
        eng.append(dict(name=name, c=c, lompc=lompc, off=off, gamma=gamma, lm=lm, wr=wr, M=M))

    main = torch.cuda.current_stream()
    if args.mode == "path" and args.split_types:
        runs = []
        for e in eng:
            st = torch.cuda.Stream()
            st.wait_stream(main)
            lr = torch.zeros(P, dtype=torch.float64, device=dev)
            plan = BatchPlan(e["lompc"], e["gamma"], e["off"], w_ref=e["wr"], want_w=args.outputs == "full",
                             want_cost=args.outputs != "set", want_set=True, stream=st, warm_start=args.warm)
            runs.append(dict(plan=plan, stream=st, lm_ptr=[e["lm"][k].data_ptr() for k in range(nsteps)],
                             lr_ptr=lr.data_ptr(), qps=e["M"], keep=(lr,)))
    elif args.mode == "path":
        # ONE plan over both EV types: their 2P parameter sets stacked (small first), every step
        # is one fused k_solve launch over all (set, gamma cell) waves + one k_reduce
        off = np.concatenate([eng[0]["off"], eng[0]["M"] + eng[1]["off"][1:]])
        gamma = torch.cat([e["gamma"] for e in eng])
        lm = torch.cat([e["lm"] for e in eng], dim=1).contiguous()  # (nsteps, 2P, 3N)
        wr = torch.cat([e["wr"] for e in eng]).contiguous()
        lr = torch.zeros(2 * P, dtype=torch.float64, device=dev)
        runs = [dict(plan=BatchPlan([e["lompc"] for e in eng], gamma, off, sets_per_ctx=[P, P], w_ref=wr,
                                    want_w=args.outputs == "full", want_cost=args.outputs != "set", want_set=True,
                                    stream=main, warm_start=args.warm, cells=args.cells or None), stream=main, lm_ptr=[lm[k].data_ptr() for k in range(nsteps)], lr_ptr=lr.data_ptr(),
                     lm_stride=int(lm[0].numel()),
                     qps=B, keep=(gamma, lm, wr, lr))]
    else:
        # DIRECT mode: one context per EV type, each on its own stream
        runs = []
        for e in eng:
            st = torch.cuda.Stream()
            st.wait_stream(main)
            lr = torch.zeros(P, dtype=torch.float64, device=dev)
            plan = BatchPlan(e["lompc"], e["gamma"], e["off"], w_ref=e["wr"], gamma_ref=torch.full(
                (P,), e["c"].y_max - 0.4, dtype=torch.float64, device=dev), want_w=True, want_cost=True,
                want_set=True, stream=st)
            runs.append(dict(plan=plan, stream=st, lm_ptr=[e["lm"][k].data_ptr() for k in range(nsteps)],
                             lr_ptr=lr.data_ptr(), qps=e["M"], keep=(lr,)))
    torch.cuda.synchronize()

    multi = len(runs) > 1
    # sharded on RCCL: the plan carries the extension's communicator, so every run all-gathers and
    # combines the set reductions on the device inside the same C-ABI call (no Python per step)
    comm = device_comm(dist.group.WORLD, dev.index) if sharded and args.mode == "path" and not multi else None
    if comm is not None:
        runs[0]["plan"].set_comm(comm)
    py_combine = sharded and comm is None  # gloo rehearsal / split plans: torch.distributed per step

    def step(k):
        if py_combine or multi:  # the previous step's collective reads the output buffers
            for r in runs:
                r["stream"].wait_stream(main)
        for r in runs:
            r["plan"].run(r["lm_ptr"][k], r["lr_ptr"])
        if multi:
            for r in runs:
                main.wait_stream(r["stream"])
        if py_combine:
            # every set's reductions (both EV types) in ONE collective
            combine_set_results([(r["plan"].out["set_sum_w"], r["plan"].out["set_stats"]) for r in runs])

    # one plan: the K timed steps are issued by ONE C-ABI call (lompc_plan_run_steps: the same
    # launches per step at that step's prices — plus the RCCL all-gather and the combine kernel
    # when sharded — the HIP events on every E-th step's k_step), so host issue stays far below
    # the GPU time even on a slow host CPU; every step's set reductions are kept ([K][S][...])
    batched = len(runs) == 1 and "lm_stride" in runs[0] and not args.per_step_issue and not py_combine
    # every timed step writes its own set reductions ([K][S][...]), so every step is observable afterwards
    # (verify_steps); the per-EV outputs (w, cost) are one buffer that every step rewrites, as a price
    # loop's iterations do (price_solver.py:203-209), the last step's remaining.  (Allocated before the
    # warmup: no allocation between the warmup and the timed region.)
    outs_t = outs_v = None
    if batched:
        pl = runs[0]["plan"]
        K = args.steps
        outs_t = {k: torch.empty((K,) + tuple(pl.out[k].shape), dtype=torch.float64, device=dev)
                  for k in ("set_sum_w", "set_stats") if pl.out.get(k) is not None}
        outs_v = {k: torch.empty_like(v) for k, v in outs_t.items()}
    # warmup (and correctness gate: every QP certified) — in the timed region's own form, so its
    # one-time setup (the stepped form's tables and block map) is not timed; the warmup carries the
    # timed call's HIP events too (the runtime's first timed dispatch on a queue costs host time), and
    # its event readings are discarded
    ev_every = max(1, args.event_every)
    no_events = args.kernel_events == "none"
    for r in runs:
        r["plan"].profile(enable=("k_eval",) if not no_events else False)
    if batched:
        r = runs[0]
        r["plan"].run_steps(r["lm_ptr"][0], r["lr_ptr"], max(args.warmup, 1), r["lm_stride"], 0,
                            profile_every=0 if no_events else ev_every, span_events=args.kernel_events == "span")
    else:
        for k in range(args.warmup):
            step(k)
    for r in runs:
        rep, fail, inv = r["plan"].check()  # (sticky tallies: every warmup step)
        assert fail == 0 and inv == 0, (fail, inv)
    for r in runs:
        r["plan"].profile(read=True, reset=True)
    go = None
    if batched:  # the timed call prepared (its arguments converted) before the clock starts
        r = runs[0]
        go, _ = r["plan"].steps_call(r["lm_ptr"][args.warmup], r["lr_ptr"], args.steps, r["lm_stride"], 0,
                                     profile_every=0 if no_events else ev_every, out=outs_t,
                                     span_events=args.kernel_events == "span")
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    if batched:
        go()
    else:
        for k in range(args.warmup, nsteps):
            sample = not no_events and (k - args.warmup) % ev_every == 0
            if ev_every > 1 and not no_events:
                for r in runs:
                    r["plan"].profile(enable=("k_eval",) if sample else False)
            step(k)
    t_issue = time.perf_counter() - t0  # host time to enqueue the K steps (GPU-bound if << dt)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    dt = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([dt], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dt = float(t.item())
    repaired = 0
    for r in runs:
        rep, fail, inv = r["plan"].check()  # sticky device tallies: EVERY timed step's QPs
        assert fail == 0 and inv == 0, (fail, inv)
        repaired += rep
    # the per-EV kernel's timing over the timed region: HIP events on its own dispatches
    k_ms, k_n, k_qps = 0.0, 0, 0
    for r in runs:
        ms, n = r["plan"].profile(read=True)
        k_ms += ms
        k_n += n
        k_qps += r["qps"] * n
    verified = verify_steps(runs[0], args, outs_t, outs_v, torch) if batched else None
    gpu_last = None  # the last timed step's GPU outputs (host copies), for the CPU engine's parity check
    if batched and args.mode == "path" and not args.no_cpu_baseline and runs[0]["plan"].out.get("w") is not None:
        pl = runs[0]["plan"]
        gpu_last = {"w": pl.out["w"].cpu().numpy(), "cost": pl.out["cost"].cpu().numpy(),
                    "set_sum_w": outs_t["set_sum_w"][-1].cpu().numpy(), "set_stats": outs_t["set_stats"][-1].cpu().numpy()}
    avg_launch_s = (k_ms / 1e3) / max(k_n, 1)
    qp_per_launch = k_qps / max(k_n, 1)
    bytes_per_qp = 8 * (N + 2)
    achieved_gbs = bytes_per_qp * qp_per_launch / avg_launch_s / 1e9 if k_n else 0.0
    # the stepped form (lompc_plan_run_steps, full outputs, no communicator): the timed region's
    # events sit on its k_step launches
    stepped = batched and args.mode == "path" and runs[0]["plan"].info()["cells"] % 4 == 0
    # wide form (no warm start): per group of <= 64 steps k_paths (the paths), k_evals (every step's
    # evaluation, each workgroup through its block of every step) and k_closes (the closings); its events
    # sit on k_evals and read as one launch per step
    wide = stepped and not args.warm
    rkernel = (("k_step (step k+1's path + step k's evaluation + step k-1's closing)" if args.warm else
                "k_evals (the K steps' evaluations in ONE launch, read per step: its duration / K; the K paths in "
                "one k_paths launch before it, the K closings in one k_closes launch after it)")
               if stepped else ("k_eval" if args.mode == "path" else "k_direct"))
    kname = rkernel.split()[0]

    total_qp = world * B * args.steps
    value = total_qp / dt
    path = args.mode == "path"
    line = {
        "metric": "LoMPC QP solves/sec",
        "value": value,
        "unit": "QP/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": dt / args.steps * 1e3,
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "f64",
        "data": "synthetic (seeded EV populations and price vectors; reference ships no data for this path)",
        "config": {
            "workload": (f"config3/4: {B} EVs per GPU, horizon {N}, 50% small / 50% large EVs, "
                         f"{P} partitions per type ({2 * P} parameter sets), fresh prices every step, "
                         "full outputs (w, cost) + fused per-partition reductions"),
            "evs_per_gpu": B,
            "horizon": N,
            "parameter_sets": 2 * P,
            "mode": args.mode,
            "outputs": args.outputs,
            "warm_start": bool(args.warm),
            "cells_per_set": (runs[0]["plan"].info()["cells"] if args.mode == "path" else None),
            "parallelism": (f"dp{world} (EV shards; ONE RCCL all-gather of both types' per-set reductions per "
                            "group of up to 64 steps + a rank-ordered combine kernel, issued inside the C-ABI call)"
                            if comm is not None else (f"dp{world} (EV shards, torch.distributed all-gather per step)"
                                                      if sharded else "dp1")),
            "sharded_code_path": bool(sharded),
            "dist_backend": (args.dist_backend if sharded else None),
            "launches_per_step": (("3 per group of up to 64 steps (k_paths, k_evals, k_closes)" if wide else
                                   "1 (k_step) + 2 for the K steps' pipeline fill and drain")
                                  + ("; + per step the all-gather and the combine kernel" if comm is not None else "")
                                  if stepped else sum(r["plan"].launches_per_run() for r in runs)),
            "step_outputs": ("set reductions: every step's own [K][S][...]; w, cost: one buffer every step rewrites"
                             if batched else "shared buffers (the last step's remain)"),
            "kernel_events": ("none" if no_events else
                              ((f"k_evals: one pair around its launch, read as its {k_n} steps" if wide else
                                f"{kname}: one pair spanning {k_n} steady-state launches") if args.kernel_events == "span"
                               else f"{kname}, 1 in {ev_every} timed launches")),
            "issue": ("one lompc_plan_run_steps call for the K timed steps" +
                      ((" (wide form)" if wide else " (stepped form)") if stepped else ""))
                     if batched else "per-step lompc_plan_run",
            "correctness_gate": "sticky device tallies: no failed / invalid QP in any warmup or timed step",
        },
        "roofline": {
            "bound": "hbm",
            "achieved": achieved_gbs,
            "peak": HBM_PEAK_GBS,
            "unit": "GB/s",
            "frac": achieved_gbs / HBM_PEAK_GBS,
            "traffic": None,
            "kernel": rkernel,
            "bytes_per_qp": bytes_per_qp,
            "bytes_note": ("the evaluation's algorithmic bytes (gamma in, w and cost out); the path's table "
                           "writes (~1 MB per launch) are not counted") if stepped else "gamma in, w and cost out",
            "qp_per_launch": qp_per_launch,
            "avg_launch_us": avg_launch_s * 1e6,
        },
        "repaired_qps": repaired,
        "host_issue_us_per_step": t_issue / args.steps * 1e6,
        "verified_steps": verified["steps"] if verified else 0,
        "verification": verified or "per-step issue: no per-step records kept",
    }
    if sharded:
        line["collective"] = collective_cost(runs, args, world, dev, torch, dist, comm, batched, dt)
    pmc = load_pmc(args, N, qp_per_launch)
    pk = kname if stepped else "k_eval"
    if pmc and pk in pmc and "hbm_bytes_per_launch" in pmc[pk]:
        line["roofline"]["traffic"] = pmc[pk]["hbm_bytes_per_launch"]
        line["roofline"]["traffic_source"] = pmc["source"]
    if path and world == 1 and len(runs) == 1:
        line["kernels"] = kernel_breakdown(runs[0], step, args, nsteps, pmc, torch)
        if stepped:
            line["kernels"][kname] = {"avg_us": avg_launch_s * 1e6, "launches_timed": k_n,
                                      "note": ("the timed region's evaluation launch, per step (its duration / K); the "
                                               "entries above: each kernel of a single run as its own launch") if wide else
                                              ("the timed region's launches (each as k_path + k_eval + k_finalize of "
                                               "three different steps); the entries above: each kernel as its own launch")}
            if pmc and kname in pmc:
                line["kernels"][kname]["pmc"] = {x: pmc[kname][x] for x in pmc[kname] if x != "hbm_bytes_per_launch"}
    if path and world == 1 and not multi and not args.no_contracts:
        line["contracts"] = contract_legs(eng, runs[0], N, P, args, nsteps, dev, torch, comm, pmc)
        if batched and comm is None:
            line["contracts"]["sequential"] = sequential_leg(runs[0], eng, N, P, args, torch)
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        line["cpu_baseline"] = cpu_baseline(eng, N, args.cpu_seconds, args.seed)
        if path:
            line["cpu_baseline"]["same_algorithm"] = cpu_same_algorithm(eng, N, P, args, gpu_last)
    if path and world == 1 and not args.no_direct:
        line["direct_mode"] = direct_leg(eng, N, P, args, nsteps, dev, torch)
    if not args.no_station:
        del eng, runs
        line["bimpc"] = station_leg(args, world, dev, sharded)
    if rank == 0:
        print(json.dumps(line), flush=True)
    if sharded:
        release_comms()
        dist.destroy_process_group()
    if "error" in line.get("bimpc", {}):
        sys.exit(1)  # the QP/s line is printed; a failed station leg still fails the run


def verify_steps(run, args, outs_t, outs_v, torch):
    """Every timed step checked after the timed region: the same K prices re-run through
    lompc_plan_run_steps in its LOMPC_STEPS_PER_KERNEL form (the same kernels on the same arguments,
    one part per launch: no overlap inside a launch) must give every step's set reductions (sums of w,
    counts, sums of cost / w0 / price0, max A_bar error, tallies) and the last step's per-EV w and cost
    bit for bit.  A mismatch fails the run."""
    plan = run["plan"]
    plan.profile(enable=False)
    last = {k: plan.out[k].clone() for k in ("w", "cost") if plan.out.get(k) is not None}
    plan.run_steps(run["lm_ptr"][args.warmup], run["lr_ptr"], args.steps, run["lm_stride"], 0, per_kernel=True,
                   out=outs_v)
    rep, fail, inv = plan.check()
    assert fail == 0 and inv == 0, (fail, inv)
    ok = [all(bool(torch.equal(outs_t[key][k], outs_v[key][k])) for key in outs_t) for k in range(args.steps)]
    rows = all(bool(torch.equal(v, plan.out[k])) for k, v in last.items())
    if not (all(ok) and rows):
        raise SystemExit(f"bench.py: timed steps differ from their re-run: per-step sets {ok}, last step's rows {rows}")
    st = outs_t.get("set_stats")
    return {"steps": sum(ok), "how": "every timed step's set reductions and the last step's w / cost re-run through "
                                     "lompc_plan_run_steps(LOMPC_STEPS_PER_KERNEL) after the timed region: bitwise equal",
            "counts_ok": bool((st[:, :, 0].sum(dim=1) == plan.B).all()) if st is not None else None}


def collective_cost(runs, args, world, dev, torch, dist, comm, batched, dt):
    """The per-step cost of the cross-rank exchange, so a scaling run is attributable: the same K
    timed steps again WITHOUT the exchange (RCCL: the plan's communicator detached, so no all-gather /
    combine kernel; gloo: no torch.distributed combine), max over ranks; collective_us_per_step =
    timed step - that step.  Also the exchange alone (RCCL: ceil(K / 64) all-gathers of a group's packed
    set records through torch.distributed on the same communicator size; gloo: K combine_set_results
    calls)."""
    from lompc_amd.dist import combine_set_results

    K = args.steps
    r = runs[0]

    def timed(fn):
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        fn()
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()
        t = time.perf_counter() - t0
        if world > 1:
            x = torch.tensor([t], dtype=torch.float64, device=dev)
            dist.all_reduce(x, op=dist.ReduceOp.MAX)
            t = float(x.item())
        return t

    if comm is not None and batched:
        plan = r["plan"]
        plan.set_comm(None)
        try:
            plan.run_steps(r["lm_ptr"][args.warmup], r["lr_ptr"], K, r["lm_stride"], 0)
            t_no = timed(lambda: plan.run_steps(r["lm_ptr"][args.warmup], r["lr_ptr"], K, r["lm_stride"], 0))
        finally:
            plan.set_comm(comm)
        S, N = plan.S, plan.N
        G = 64  # (the wide form's group: one all-gather of its runs' contiguous records)
        rec = torch.zeros(min(K, G) * S * (N + 8), dtype=torch.float64, device=dev)
        recv = torch.empty(world * rec.numel(), dtype=torch.float64, device=dev)

        def gathers():
            for _ in range((K + G - 1) // G):
                dist.all_gather_into_tensor(recv, rec)

        gathers()
        t_ag = timed(gathers)
        how = ("RCCL: ONE all-gather of a group's (up to 64 steps') packed set records + the k_combine_runs kernel "
               "after the group's closings, inside the run_steps call")
    else:
        outs = [(x["plan"].out["set_sum_w"], x["plan"].out["set_stats"]) for x in runs]

        def without():
            for k in range(args.warmup, args.warmup + K):
                for x in runs:
                    x["plan"].run(x["lm_ptr"][k], x["lr_ptr"])

        def combines():
            for _ in range(K):
                combine_set_results(outs)

        without()
        t_no = timed(without)
        t_ag = timed(combines)
        how = f"torch.distributed ({args.dist_backend}) all-gather + host-ordered combine after each step's run"
    return {"how": how, "steps": K, "ms_per_step_with": dt / K * 1e3, "ms_per_step_without": t_no / K * 1e3,
            "collective_us_per_step": (dt - t_no) / K * 1e6, "exchange_alone_us_per_step": t_ag / K * 1e6,
            "ranks": world}


def load_pmc(args, N, qp_per_launch):
    """profiles/pmc.json (scripts/make_traffic.py over a rocprofv3 --pmc session of this bench):
    per-kernel counters, used only when it was collected on this configuration."""
    f = os.path.join(ROOT, "profiles", "pmc.json")
    try:
        d = json.load(open(f))
    except (OSError, ValueError):
        return None
    ok = d.get("mode") == args.mode and d.get("horizon") == N and d.get("qp_per_launch") == qp_per_launch
    return d if ok else None


def kernel_breakdown(run, step, args, nsteps, pmc, torch):
    """Average duration of each of the plan's kernels over 20 more steps with HIP events on
    all three dispatches (outside the timed region), and k_path's roof: it is latency-bound
    (one wave per (set, gamma cell), a chain of dependent DPP scans; far fewer waves than
    SIMDs), so it is priced by the fraction of its waves' cycles that issue VALU work (PMC)."""
    plan = run["plan"]
    kernels = ("k_path", "k_eval", "k_finalize")
    plan.profile(enable=kernels)
    for k in kernels:
        plan.profile(read=True, reset=True, kernel=k)
    n = 20
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for j in range(n):
        step(args.warmup + j % max(nsteps - args.warmup, 1))
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    out = {"steps": n, "ms_per_step_with_events": dt / n * 1e3}
    for k in kernels:
        ms, cnt = plan.profile(read=True, kernel=k)
        if cnt:  # (no k_finalize launches when the sets close inside k_eval)
            out[k] = {"avg_us": ms / cnt * 1e3, "launches": cnt}
    plan.profile(enable=False)
    info = plan.info()
    out["k_path"].update({"waves": info["sets"] * info["cells"], "cells_per_set": info["cells"],
                          "bound": "latency (dependent DPP-scan chains, one wave per SIMD at most)"})
    out["k_eval"]["workgroups"] = info["workgroups"]
    if pmc:
        for k in kernels:
            if k in pmc and k in out:
                out[k]["pmc"] = {x: pmc[k][x] for x in pmc[k] if x != "hbm_bytes_per_launch"}
        if "k_path" in pmc and "valu_issue_frac" in pmc["k_path"]:
            kp = pmc["k_path"]
            out["k_path"]["valu_issue_frac"] = kp["valu_issue_frac"]  # of a wave's own lifetime
            # chip level: the waves' VALU-busy cycles over every SIMD (256 CUs x 4) for the
            # launch's duration at the 2.4 GHz max clock (MI355X_MICROARCH.md) — a lower bound
            # on the true fraction if the clock ran lower
            if "waves" in kp and "wave_cycles_avg" in kp and out["k_path"].get("avg_us"):
                busy = kp["valu_issue_frac"] * kp["wave_cycles_avg"] * kp["waves"]
                out["k_path"]["valu_chip_frac"] = busy / (1024 * out["k_path"]["avg_us"] * 1e-6 * 2.4e9)
    return out


def direct_leg(eng, N, P, args, nsteps, dev, torch):
    """The same batch in DIRECT mode (every EV solved by its own lane from a per-set working
    set, no gamma paths): QP/s over 20 steps, for comparison with the PATH plan above."""
    from lompc_amd import BatchPlan, LoMPC

    runs = []
    for e in eng:
        lo = LoMPC(N, e["c"], device=dev.index, mode="direct")
        lr = torch.zeros(P, dtype=torch.float64, device=dev)
        plan = BatchPlan(lo, e["gamma"], e["off"], w_ref=e["wr"], gamma_ref=torch.full(
            (P,), e["c"].y_max - 0.4, dtype=torch.float64, device=dev), want_w=True, want_cost=True,
            want_set=True)
        runs.append((plan, lo, [e["lm"][k].data_ptr() for k in range(nsteps)], lr))
    n = 20
    for plan, _, lm, lr in runs:
        plan.run(lm[0], lr.data_ptr())
        plan.check()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for j in range(n):
        for plan, _, lm, lr in runs:
            plan.run(lm[args.warmup + j % max(nsteps - args.warmup, 1)], lr.data_ptr())
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    rep = 0
    for plan, _, _, _ in runs:
        r_, f_, i_ = plan.check()
        assert f_ == 0 and i_ == 0
        rep += r_
    B = sum(e["M"] for e in eng)
    return {"value": B * n / dt, "unit": "QP/s", "ms_per_step": dt / n * 1e3, "steps": n, "repaired_qps": rep}


def sorted_reductions_leg(base, lm_ptr, lr_ptr, stride, args, torch, comm, red):
    """``reductions`` through a ``sort_sets`` plan over the headline's unsorted batch (contract_legs);
    ``vs_caller_order``: the largest relative difference of its last step's per-set sums of w and
    costs from the ``reductions_in_caller_order`` leg's (the same EVs: only the summation order and
    the 2^-40 quantisation differ)."""
    from lompc_amd import BatchPlan
    from lompc_amd import _lib

    K = args.steps
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    plan = BatchPlan(base.lompcs, base.gamma, base.off, sets_per_ctx=base.sets_per_ctx, w_ref=base.w_ref,
                     want_set=True, stream=torch.cuda.current_stream(), cells=base.info()["cells"], want_w=False,
                     want_cost=False, sort_sets=True, validate=False)
    torch.cuda.synchronize()
    prep_ms = (time.perf_counter() - t0) * 1e3
    if comm is not None:
        plan.set_comm(comm)
    plan.run_steps(lm_ptr[0], lr_ptr, max(args.warmup, 1), stride, 0)
    assert plan.check()[1:] == (0, 0)
    plan.profile(enable=("k_eval", "k_path"))
    call, res = plan.steps_call(lm_ptr[args.warmup], lr_ptr, K, stride, 0, span_events=True, per_run_sets=True)
    call()  # (the same call once untimed: its outputs and events warm)
    plan.check()
    plan.profile(read=True, reset=True)
    plan.profile(read=True, reset=True, kernel="k_path")
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    call()
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    rep, fail, inv = plan.check()
    assert fail == 0 and inv == 0, ("reductions", fail, inv)
    ms_a, n_a = plan.profile(read=True)
    ms_p, n_p = plan.profile(read=True, kernel="k_path")
    plan.profile(enable=False)
    sw, ss = res["set_sum_w"][-1], res["set_stats"][-1]
    rw, rs = red["set_sum_w"][-1], red["set_stats"][-1]
    dw = float(((sw - rw).abs() / rw.abs().clamp_min(1e-300)).max())
    c = _lib.LOMPC_STAT_SUM_COST
    dc = float(((ss[:, c] - rs[:, c]).abs() / rs[:, c].abs().clamp_min(1e-300)).max())
    B = plan.B
    del plan
    return {"value": B * K / dt, "unit": "QP/s", "ms_per_step": dt / K * 1e3, "steps": K,
            "outputs": "every step's set reductions its own ([K][S][...])", "repaired_qps": rep,
            "k_aggs_us_per_step": ms_a / max(n_a, 1) * 1e3, "k_paths_us_per_step": ms_p / K * 1e3 if n_p else None,
            "launches": "per group of up to 64 steps: k_paths + k_aggs (one workgroup per (step, set))",
            "prepare_ms": prep_ms,
            "prepare": "once per population (BatchPlan(sort_sets=True) construction): each set's gamma sorted on the "
                       "device, the fixed-point prefix sums and the fine bucket index of every set, allocation included",
            "vs_caller_order": {"max_rel_set_sum_w": dw, "max_rel_sum_cost": dc},
            "roofline": None,
            "roofline_note": "O(pieces) per set: no per-EV bytes move per step; bound by the path and aggregation "
                             "latency chains"}


def contract_legs(eng, run, N, P, args, nsteps, dev, torch, comm, pmc):
    """The per-iteration contracts the reference actually runs on the same batch (both EV types,
    2P sets, fresh prices every step), each K steps in one lompc_plan_run_steps call (the wide
    form: per group of up to 64 steps one k_paths, one k_evals and one k_closes launch):

    * ``reductions`` — PriceSolver._get_w_err (price_solver.py:196-214): only the per-set sums of
      w, the max A_bar error and the counts leave the engine (the reference drops w0, :206), so the
      EVs' order inside a set is free: the plan (``BatchPlan(sort_sets=True)``) snapshots the same
      unsorted batch with each set sorted once at prepare (``prepare_ms``, not per step) and every
      step is one k_paths + one k_aggs launch per group — O(pieces) per set, no per-EV bytes;
    * ``reductions_in_caller_order`` — the same contract without the prepare-time sort: k_evals sums
      each certified piece's EVs from their count and fixed-point gamma sum (no rows evaluated);
      algorithmic HBM bytes = gamma in = 8 B per QP;
    * ``w0`` — get_w0_price0 (price_solver.py:272-285): w0 per EV out + price0 sums: 16 B per QP.

    Each reports QP/s, ms per step and the evaluation launch's time per step (one HIP-event pair around
    the launch, read as its steps) with its HBM roofline at that contract's bytes (latency-bound: 8-16 B
    per QP is far below what one launch can move; staging and lookup rounds set the launch time)."""
    from lompc_amd import BatchPlan

    base = run["plan"]
    out = {}
    lm_ptr, lr_ptr, stride = run["lm_ptr"], run["lr_ptr"], run["lm_stride"]
    K = args.steps
    for name, kw, bpq in (("reductions_in_caller_order", dict(want_w=False, want_cost=False), 8),
                          ("w0", dict(want_w=False, want_cost=False, want_w0=True), 16)):
        plan = BatchPlan(base.lompcs, base.gamma, base.off, sets_per_ctx=base.sets_per_ctx, w_ref=base.w_ref,
                         want_set=True, stream=torch.cuda.current_stream(), warm_start=args.warm,
                         cells=base.info()["cells"], **kw)
        if comm is not None:
            plan.set_comm(comm)
        plan.run_steps(lm_ptr[0], lr_ptr, max(args.warmup, 1), stride, 0)
        assert plan.check()[1:] == (0, 0)
        plan.profile(enable=("k_eval",))
        plan.profile(read=True, reset=True)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        res = plan.run_steps(lm_ptr[args.warmup], lr_ptr, K, stride, 0, span_events=True, per_run_sets=True)
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
        if name == "reductions_in_caller_order":
            red = {k: res[k].clone() for k in ("set_sum_w", "set_stats")}
        rep, fail, inv = plan.check()
        assert fail == 0 and inv == 0, (name, fail, inv)
        ms_e, n_e = plan.profile(read=True)
        B = plan.B
        ev_us = ms_e / max(n_e, 1) * 1e3
        gbs = bpq * B / (ev_us * 1e-6) / 1e9 if n_e else 0.0
        out[name] = {"value": B * K / dt, "unit": "QP/s", "ms_per_step": dt / K * 1e3, "steps": K,
                     "outputs": "every step's set reductions its own ([K][S][...]); w0 one buffer every step rewrites",
                     "repaired_qps": rep, "k_evals_avg_us": ev_us, "k_evals_steps_timed": n_e,
                     "roofline": {"bound": "hbm", "kernel": "k_evals", "bytes_per_qp": bpq,
                                  "achieved": gbs, "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": gbs / HBM_PEAK_GBS,
                                  "note": ("the evaluation launch of the wide form per step (the K paths run in "
                                           "one k_paths launch before, the closings in one k_closes launch after, "
                                           "neither in this duration): latency-bound, its staging and lookup rounds, "
                                           "not 8-16 B per QP, set its time")}}
        plan.profile(enable=False)
        del plan
    out["reductions"] = sorted_reductions_leg(base, lm_ptr, lr_ptr, stride, args, torch, comm, red)
    # the headline's workload with every step's rows in their OWN buffer (w at a per-step stride: K x 50 MB
    # of fresh lines, which the 256 MB Infinity Cache cannot hold — the HBM-resident form of the roofline)
    base.profile(enable=("k_eval",))
    o = {"w": torch.empty((K, base.B, N), dtype=torch.float64, device=dev),
         "cost": torch.empty((K, base.B), dtype=torch.float64, device=dev)}
    base.run_steps(lm_ptr[args.warmup], lr_ptr, K, stride, 0, out=o)
    assert base.check()[1:] == (0, 0)
    base.profile(read=True, reset=True)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    base.run_steps(lm_ptr[args.warmup], lr_ptr, K, stride, 0, out=o, span_events=True)
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    rep, fail, inv = base.check()
    assert fail == 0 and inv == 0, ("fresh_rows", fail, inv)
    ms_e, n_e = base.profile(read=True)
    base.profile(enable=False)
    B, bpq = base.B, 8 * (N + 2)
    ev_us = ms_e / max(n_e, 1) * 1e3
    gbs = bpq * B / (ev_us * 1e-6) / 1e9 if n_e else 0.0
    out["fresh_rows"] = {"value": B * K / dt, "unit": "QP/s", "ms_per_step": dt / K * 1e3, "steps": K,
                         "outputs": "w and cost of every step in their own buffers ([K][B][N], [K][B]): no step "
                                    "rewrites another's lines",
                         "k_evals_avg_us": ev_us,
                         "roofline": {"bound": "hbm", "kernel": "k_evals", "bytes_per_qp": bpq, "achieved": gbs,
                                      "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": gbs / HBM_PEAK_GBS}}
    del o
    return out


def sequential_leg(run, eng, N, P, args, torch):
    """The reference's call pattern at config 3: K DEPENDENT steps, step k+1's prices computed on the
    device from step k's set reductions (lompc_plan_run_chain: a projected dual-gradient step
    max(0, lmbd + step (phi(mean w) - phi(w_ref))) per set, as each price iteration of
    price_solver.py:111-140 depends on the previous one's reductions), so no two steps overlap: every
    step is its own path -> evaluation -> closing chain (+ the price update launch).  Same batch, outputs
    (w, cost, set reductions) and roofline bytes as the headline, on the headline's plan; the same chain
    on a warm-started plan (each gamma cell's exact solve from the working set the previous step ended
    with, the form of the engine's price loops) beside it (``warm``).  ms_per_step from the timed call, per-kernel durations from a second call with
    HIP events on every launch; every step's reductions re-computed afterwards by the headline plan's
    independent wide run_steps over the recorded prices (verified_steps: equal to 1e-12 relative;
    bitwise_steps: bit for bit)."""
    from lompc_amd import BatchPlan

    base = run["plan"]
    K = args.steps
    S = base.S
    dev = base.gamma.device
    lm0 = torch.as_tensor(np.concatenate([e["lm"][args.warmup].cpu().numpy() for e in eng]), device=dev)
    lr = torch.zeros(S, dtype=torch.float64, device=dev)
    wt = base.w_ref
    step = 0.5
    warm = BatchPlan(base.lompcs, base.gamma, base.off, sets_per_ctx=base.sets_per_ctx, w_ref=base.w_ref,
                     want_w=True, want_cost=True, want_set=True, stream=torch.cuda.current_stream(), warm_start=True,
                     cells=base.info()["cells"])

    def timed(plan):
        out = {k: torch.empty(s, dtype=torch.float64, device=dev) for k, s in
               (("lmbd", (K, S, 3 * N)), ("set_sum_w", (K, S, N)), ("set_stats", (K, S, 8)))}
        plan.profile(enable=False)
        kw = max(1, min(args.warmup, K))  # (untimed: the chain's first launches, same form)
        plan.run_chain(lm0, lr, wt, step, kw, out={k: v[:kw] for k, v in out.items()})
        assert plan.check()[1:] == (0, 0)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        plan.run_chain(lm0, lr, wt, step, K, out=out)
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
        rep, fail, inv = plan.check()
        assert fail == 0 and inv == 0, (fail, inv)
        last = {k: plan.out[k].clone() for k in ("w", "cost") if plan.out.get(k) is not None}
        # per-kernel durations: the same chain again with a HIP-event pair on every launch
        kernels = ("k_path", "k_eval", "k_finalize")
        plan.profile(enable=kernels)
        for k in kernels:
            plan.profile(read=True, reset=True, kernel=k)
        plan.run_chain(lm0, lr, wt, step, K)
        assert plan.check()[1:] == (0, 0)
        kus = {}
        for k in kernels:
            ms, n = plan.profile(read=True, kernel=k)
            if n:
                kus[k] = {"avg_us": ms / n * 1e3, "launches": n}
        plan.profile(enable=False)
        return dt, rep, out, last, kus

    dt, rep, out, last, kus = timed(base)
    dt_w, _, _, _, kus_w = timed(warm)
    # verification: an independent wide run_steps over the chain's K price vectors
    vo = {k: torch.empty_like(out[k]) for k in ("set_sum_w", "set_stats")}
    base.run_steps(out["lmbd"], lr, K, S * 3 * N, 0, out=vo)
    assert base.check()[1:] == (0, 0)
    bit = [all(bool(torch.equal(out[k][j], vo[k][j])) for k in vo) for j in range(K)]
    close = [bool(torch.allclose(out[k][j], vo[k][j], rtol=1e-12, atol=1e-12)) for k in vo for j in range(K)]
    ok = [all(close[i * K + j] for i in range(len(vo))) for j in range(K)]
    rows_d = max(float((v - base.out[k]).abs().max()) for k, v in last.items())
    if not (all(ok) and rows_d <= 1e-12):
        raise SystemExit(f"bench.py: sequential steps differ from their independent re-run: {ok}, rows {rows_d}")
    moved = float((out["lmbd"][-1] - out["lmbd"][0]).abs().max())
    B = base.B
    bpq = 8 * (N + 2)
    ev_us = kus.get("k_eval", {}).get("avg_us", 0.0)
    gbs = bpq * B / (ev_us * 1e-6) / 1e9 if ev_us else 0.0
    return {"value": B * K / dt, "unit": "QP/s", "ms_per_step": dt / K * 1e3, "steps": K,
            "plan": "the headline's (no warm start)",
            "issue": "one lompc_plan_run_chain call: per step the price update (k_chain_price) then k_path, k_eval, "
                     "k_finalize of that step (4 launches; no overlap between steps is possible)",
            "price_rule": f"lmbd_(k+1) = max(0, lmbd_k + {step} (phi(sum_w / count) - phi(w_ref))) per set, on the device",
            "max_price_change": moved, "repaired_qps": rep, "kernels": kus,
            "verified_steps": sum(ok), "bitwise_steps": sum(bit),
            "verification": "every step's set reductions (and the last step's w / cost) re-computed by an independent "
                            "wide lompc_plan_run_steps over the recorded prices: equal to 1e-12 relative (bitwise: "
                            f"{sum(bit)} of {K} — the wide form's staged evaluation sums a block's rows over seven "
                            f"row waves, a single run's k_eval over eight; the last step's rows within {rows_d:.1e})",
            "warm": {"value": B * K / dt_w, "ms_per_step": dt_w / K * 1e3, "kernels": kus_w,
                     "plan": "warm-started: large price steps leave the stored working sets of little use"},
            "roofline": {"bound": "hbm", "kernel": "k_eval", "bytes_per_qp": bpq, "achieved": gbs,
                         "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": gbs / HBM_PEAK_GBS,
                         "note": "k_eval's duration from the events pass; the step adds the path (latency-bound) and "
                                 "the closing, which no other step can hide here"}}


def station_leg(args, world, dev, sharded=False):
    """BiMPC steps/sec (the second half of BASELINE.json's metric; config 5 weak-scaled).

    One step = ``ChargingStation._step`` (charging_station.py:156-185) on the engine: partition
    statistics, the BiMPC planner (host interior point), the 2 x P sequential price loops
    (one batched engine call per price iteration + host price QP, regularizer LP at the end)
    and the batched w0 / price0 pass, then the state update with the aggregate demand.
    Config 5 shape: horizon N_lo = N_bi = 48, P = 12 partitions, linear-convex prices,
    regularizer on, the example's BiMPC constants (real_time_price_control.py:42-52), demand
    scaled by M_2 / 500; ``--station-evs-per-gpu`` EVs per rank (2 097 152
    at 8 GPUs), sharded by EV index with the station's all-reduces."""
    import torch
    import torch.distributed as dist

    from lompc_amd import settings
    from lompc_amd.charging_station import ChargingStation
    from lompc_amd.example import DEMAND_SCALE, NUM_EVS_PER_EV_TYPE, station_consts

    settings.PRINT_LEVEL = 0
    N, P = args.station_horizon, args.partitions
    M_2 = (args.station_evs_per_gpu // 2) * world  # EVs per type, whole job
    steps, warm = args.station_steps, args.station_warmup
    # storage rate / capacity 0.5 (x_max = 0.5 is one of the example's listed values, :47): at
    # horizon 48 the example's 0.3 / 0.3 makes the first BiMPC infeasible (example.station_consts)
    pl1 = max(args.station_pl1_steps, 0)
    consts = station_consts(steps + warm + max(args.station_prof_steps, 0) + pl1, M_2, n_lo=N, n_bi=N, partitions=P,
                            price_type="linear-convex",
                            demand_scale=DEMAND_SCALE * M_2 / NUM_EVS_PER_EV_TYPE, u_b_max=0.5, x_max=0.5)
    group = dist.group.WORLD if sharded else None
    is_c5 = 2 * M_2 == 2097152 and N == 48 and P == 12
    out = {"metric": "BiMPC steps/sec", "unit": "steps/s", "steps": steps, "warmup": warm,
           "config": {"workload": (f"{'config5' if is_c5 else 'config5 shape'}: {2 * M_2} EVs "
                                   f"({args.station_evs_per_gpu} per GPU), horizon {N}, {P} partitions per type, "
                                   "linear-convex prices, regularizer on, full closed-loop step"),
                      "evs_total": 2 * M_2, "evs_per_gpu": args.station_evs_per_gpu, "horizon_lompc": N,
                      "horizon_bimpc": N, "partitions": P, "price_type": "linear-convex",
                      "bimpc_cost": "EXP_UNWEIGHTED, exp_rate 5", "demand_scale": f"DEMAND_SCALE * {M_2} / 500",
                      "storage": {"u_b_max": 0.5, "x_max": 0.5,
                                  "why": "the example lists x_max in {0.3, 0.5} and u_b_max in {0.15, 0.3} "
                                         "(real_time_price_control.py:46-47); at horizon 48 the first BiMPC from an "
                                         "empty battery needs u_b_max >= 2 d_e ~ 0.37 (beta = 0.183), so 0.3 is "
                                         "infeasible and u_b_max = 0.5 is used"},
                      "sharded_code_path": bool(sharded),
                      "print_level": 0,
                      "print_level_note": ("timed at settings.PRINT_LEVEL = 0; the reference's default is 1 "
                                           "(settings.py:4), which prints per partition and adds one more batched "
                                           "solve (the batch error at the final prices, price_solver.py:150-152) per "
                                           "partition — logging-only work; print_level_1 below times steps at 1")}}
    try:
        np.random.seed(args.seed)  # the reference's legacy global stream (charging_station.py:95-100)
        st = ChargingStation(consts, device=dev.index, group=group)
        for _ in range(warm):
            st._step()

        def calls():
            return st.price_solver_s.n_batched_calls + st.price_solver_l.n_batched_calls

        c0 = calls()
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize()
        per_step, parts = [], []
        t0 = time.perf_counter()
        for _ in range(steps):
            ts = time.perf_counter()
            st._step()
            torch.cuda.synchronize()
            per_step.append(time.perf_counter() - ts)
            parts.append((dict(st.last_step_ms), dict(st.chain_ms), (st.bimpc.last_info or {}).get("solve_ms", 0.0),
                          dict(st.bimpc_split)))
            check_station_state(st, consts)
        if world > 1:
            dist.barrier()
        dt = time.perf_counter() - t0
        if world > 1:
            t = torch.tensor([dt], dtype=torch.float64, device=dev)
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            dt = float(t.item())
        stats = st.logs["statistics"]
        it = np.concatenate([stats["niter_s"][:, warm:warm + steps].ravel(), stats["niter_l"][:, warm:warm + steps].ravel()])
        ncalls = calls() - c0
        ms = np.asarray(per_step) * 1e3
        # the step-to-step spread: a step's time against its price iterations (both types, all
        # partitions) — a least-squares line ms = fixed + per_iteration * iterations
        its = np.zeros(steps)
        for key in ("niter_s", "niter_l"):
            a = np.asarray(stats[key][:, warm:warm + steps], dtype=np.float64)
            its += np.where(a >= 0, a, 0).sum(axis=0)
        spread = {"ms": [round(float(v), 3) for v in ms], "price_iterations": [int(v) for v in its]}
        if steps >= 3 and np.ptp(its) > 0:
            b, a0 = np.polyfit(its, ms, 1)
            r = np.corrcoef(its, ms)[0, 1]
            spread.update({"fit_ms_fixed": float(a0), "fit_us_per_iteration": float(b * 1e3), "fit_r2": float(r * r),
                           "fit_note": "against the price iterations of BOTH types (their chains run concurrently)"})
        spread["attribution"] = station_attribution(ms, parts, stats, warm, steps)
        info = st.bimpc.last_info or {}
        loop = price_loop_breakdown(st, args.station_prof_steps, consts, torch)
        out["print_level_1"] = print_level_leg(st, pl1, consts, torch) if pl1 and world == 1 else None
        out.update({"value": steps / dt, "ms_per_step": dt / steps * 1e3,
                    "ms_per_step_median": float(np.median(ms)), "ms_per_step_min": float(ms.min()),
                    "ms_per_step_max": float(ms.max()),
                    "price_iterations_per_step": float(np.sum(it[it >= 0])) / steps,
                    "engine_calls_per_step": ncalls / steps,
                    "per_step": spread,
                    # (an equivalent, not a measurement: k_agg aggregates certified pieces from prefix sums
                    # and solves no per-EV QP; it counts M_p QPs per engine call)
                    "equivalent_qps_per_sec_k_agg_no_per_ev_solves": (ncalls + 2 * P * steps) * M_2 / P / dt,
                    "checks": {"storage_x_final": float(st.x), "x_max": float(consts.bimpc_consts.x_max),
                               "bimpc_iterations_last": info.get("iterations"),
                               "bimpc_primal_residual_last": info.get("primal_residual"),
                               "bimpc_dual_residual_last": info.get("dual_residual"),
                               "evs_per_type_counted": int(stats["Mp_s"][:, warm + steps - 1].sum())},
                    "price_iteration": loop})
    except Exception as e:  # reported, never hides the QP/s line
        out["error"] = f"{type(e).__name__}: {e}"
    return out


def station_attribution(ms, parts, stats, warm, steps):
    """Where each timed station step's time goes, from host timestamps taken inside _step (no extra
    synchronisation): the BiMPC phase = the host interior point + the partition staging it does not
    hide; the price phase = the longer of the two EV types' chains (each one native call: its
    partitions' loops and regularisations) + what follows them; the w0 / price0 pass; the state update.
    The parts sum to the step; the step is fitted against the SLOWER chain's price iterations."""
    its = {k: np.asarray(stats[key][:, warm:warm + steps], dtype=np.float64) for k, key in
           (("Small", "niter_s"), ("Large", "niter_l"))}
    its = {k: np.where(v >= 0, v, 0).sum(axis=0) for k, v in its.items()}
    rows = []
    for j, (marks, chains, ipm, split) in enumerate(parts):
        b = marks.get("bimpc", 0.0)
        slow = max(chains, key=chains.get) if chains else None
        rows.append({"ms": float(ms[j]), "bimpc_ipm": float(ipm), "bimpc_exposed_staging": float(b - ipm),
                     "prices": float(marks.get("prices", 0.0)),
                     "chain_small": float(chains.get("Small", 0.0)), "chain_large": float(chains.get("Large", 0.0)),
                     "slower_chain": slow, "slower_chain_iterations": int(its[slow][j]) if slow else None,
                     "w0_price0": float(marks.get("w0_price0", 0.0)), "state": float(marks.get("state", 0.0)),
                     "bimpc_split": {k: (round(v, 3) if isinstance(v, float) else {a: round(x, 3) for a, x in v.items()})
                                     for k, v in split.items()}})
    out = {"per_step": rows}
    tot = np.array([r["bimpc_ipm"] + r["bimpc_exposed_staging"] + r["prices"] + r["w0_price0"] + r["state"]
                    for r in rows])
    out["parts_sum_over_step"] = {"min": float((tot / ms).min()), "max": float((tot / ms).max())}
    for k in ("bimpc_ipm", "bimpc_exposed_staging", "prices", "chain_small", "chain_large", "w0_price0", "state"):
        out[f"mean_{k}_ms"] = float(np.mean([r[k] for r in rows]))
    x = np.array([r["slower_chain_iterations"] or 0 for r in rows], dtype=np.float64)
    if len(x) >= 3 and np.ptp(x) > 0:
        b1, a1 = np.polyfit(x, ms, 1)
        r1 = np.corrcoef(x, ms)[0, 1]
        out["fit_slower_chain"] = {"ms_fixed": float(a1), "us_per_iteration": float(b1 * 1e3), "r2": float(r1 * r1)}
    return out


def price_loop_breakdown(st, n, consts, torch):
    """Where a price iteration's time goes: ``n`` more station steps (after the timed ones) with
    the C++ price loops' per-part timing on (lompc_price_loop_args.prof): per engine call, the host
    time issuing the copies / launches (/ the RCCL collective), the host time blocked in the
    stream sync, the GPU span of the call (HIP events from the H2D copy to the D2H copy), the host
    price-gradient QP and the rest of the loop's host work.  The two EV types' loops run on two
    host threads side by side on one rank, so their parts overlap in wall time."""
    from lompc_amd import _lib

    if n <= 0:
        return None
    sols = (st.price_solver_s, st.price_solver_l)
    for s in sols:
        s.loop_prof[:] = 0.0
        s.loop_host_ms = {k: 0.0 for k in s.loop_host_ms}
        s.profile_loops = True
    st.phase_ms = {}
    st.profile_phases = True
    bimpc_ms = 0.0
    t0 = time.perf_counter()
    try:
        for _ in range(n):
            st._step()
            torch.cuda.synchronize()
            bimpc_ms += (st.bimpc.last_info or {}).get("solve_ms", 0.0)
            check_station_state(st, consts)
    finally:
        st.profile_phases = False
        for s in sols:
            s.profile_loops = False
    wall = time.perf_counter() - t0
    tot = sols[0].loop_prof + sols[1].loop_prof
    calls = tot[_lib.LOMPC_LOOP_PROF_ITERS]
    if calls <= 0:
        return {"steps": n, "note": "no native price loop ran"}
    per = lambda k: float(tot[k] / calls)
    return {"steps": n, "engine_calls": int(calls), "ms_per_step": wall / n * 1e3,
            "phase_ms_per_step": {**{k: v / n for k, v in st.phase_ms.items()}, "bimpc_host_ipm": bimpc_ms / n},
            "price_loops_ms_per_step_per_type": float(tot[_lib.LOMPC_LOOP_PROF_WALL] / n / 2e3),
            "price_solver_ms_per_step": {f"{t}/{k}": v / n for t, s in zip(("small", "large"), sols)
                                         for k, v in s.loop_host_ms.items()},
            "per_engine_call_us": {"total": per(_lib.LOMPC_LOOP_PROF_WALL), "issue": per(_lib.LOMPC_LOOP_PROF_ISSUE),
                                   "wait_sync": per(_lib.LOMPC_LOOP_PROF_WAIT), "gpu_span": per(_lib.LOMPC_LOOP_PROF_GPU),
                                   "host_price_qp": per(_lib.LOMPC_LOOP_PROF_STEP),
                                   "host_other": per(_lib.LOMPC_LOOP_PROF_HOST)}}


def print_level_leg(st, n, consts, torch):
    """``n`` more station steps at the reference's default settings.PRINT_LEVEL = 1 (settings.py:4): the
    per-partition prints (captured here, never on stdout: the line stays the only output), the extra
    batched solve per partition that feeds them (price_solver.py:150-152), and the two EV types' chains
    in the reference's interleaved order on one thread (the printing order), so no chain overlap."""
    import contextlib
    import io

    from lompc_amd import settings

    stats = st.logs["statistics"]
    t_first = st.t
    buf = io.StringIO()
    settings.PRINT_LEVEL = 1
    ms = []
    try:
        with contextlib.redirect_stdout(buf):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(n):
                ts = time.perf_counter()
                st._step()
                torch.cuda.synchronize()
                ms.append((time.perf_counter() - ts) * 1e3)
                check_station_state(st, consts)
            dt = time.perf_counter() - t0
    finally:
        settings.PRINT_LEVEL = 0
    its = 0
    for key in ("niter_s", "niter_l"):
        a = np.asarray(stats[key][:, t_first:st.t])
        its += int(a[a >= 0].sum())
    return {"steps": n, "value": n / dt, "unit": "steps/s", "ms_per_step": dt / n * 1e3,
            "ms_per_step_median": float(np.median(ms)), "price_iterations_per_step": its / n,
            "printed_lines": buf.getvalue().count("\n"),
            "note": "the steps after the timed and profiled ones (another part of the trajectory: compare per "
                    "price iteration, not per step)"}


def check_station_state(st, consts):
    """Invariants of a closed-loop step (raise -> the leg reports "error" and the run fails):
    storage state within [0, x_max] up to the BiMPC's robustness margin, the planner converged
    with small residuals, every EV counted in exactly one partition."""
    x_max = consts.bimpc_consts.x_max
    tol = 1e-6 + 0.05 * x_max
    if not (-tol <= st.x <= x_max + tol):
        raise AssertionError(f"storage state {st.x} outside [0, {x_max}]")
    info = st.bimpc.last_info or {}
    scale = 1.0 + abs(info.get("objective", 0.0))
    for k in ("primal_residual", "dual_residual"):
        if not (info.get(k, 0.0) <= 1e-6 * scale):
            raise AssertionError(f"BiMPC {k} {info.get(k)} (objective {info.get('objective')})")
    t = st.t - 1
    for key in ("Mp_s", "Mp_l"):
        if int(st.logs["statistics"][key][:, t].sum()) != st.M_2:
            raise AssertionError(f"{key} does not count every EV once")


def host_threads_note(threads: int) -> dict:
    """Where the CPU baselines' thread count comes from: OpenMP's default is OMP_NUM_THREADS when set
    (the GPU box exports 16, its CPU share per GPU), otherwise the process's CPU affinity."""
    env = os.environ.get("OMP_NUM_THREADS")
    aff = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else os.cpu_count()
    return {"host_cpus": os.cpu_count(), "affinity_cpus": aff,
            "threads_source": (f"OMP_NUM_THREADS={env} in the environment (the box's CPU share per GPU; "
                               f"{aff} CPUs in this process's affinity, {os.cpu_count()} on the machine)"
                               if env else f"OpenMP default: the {aff} CPUs of this process's affinity"),
            "threads_used": threads}


def cpu_same_algorithm(eng, N, P, args, ref):
    """The PATH engine's own algorithm on this host's cores (oracle/path_cpu.cpp, C++ / OpenMP: per
    (set, gamma cell) exact start solve + parametric active-set tracking with certified pieces, per-EV
    lookup and row write, per-set reductions — SURVEY.md §8(d)(1)) on the SAME workload as the GPU line:
    all 262 144 EVs of both types, 24 sets, full outputs (w, cost, set reductions), the timed steps'
    fresh prices in turn; all host threads and one thread.  Its outputs for the last timed step are
    compared with the GPU's (``parity``): the two implementations of one algorithm, fp64 both."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle_c  # baseline only

    oracle_c.build()
    threads = oracle_c.max_threads()
    cs = [e["c"] for e in eng]
    off = np.concatenate([eng[0]["off"], eng[0]["M"] + eng[1]["off"][1:]])
    g = np.concatenate([e["gamma"].cpu().numpy() for e in eng])
    wr = np.concatenate([e["wr"].cpu().numpy() for e in eng])
    lms = [np.concatenate([e["lm"][k].cpu().numpy() for e in eng]) for k in range(args.warmup, args.warmup + args.steps)]
    lr = np.zeros(2 * P)
    B = int(off[-1])

    def timed(nt, budget):
        # (one output buffer set every run rewrites, as the GPU line's steps do: warm-up touches its pages)
        o = oracle_c.path_run(N, cs, [P, P], lms[0], lr, g, off, w_ref=wr, nthreads=nt, cells=args.cells)
        done, t0, k = 0, time.perf_counter(), 0
        while True:
            o = oracle_c.path_run(N, cs, [P, P], lms[k % len(lms)], lr, g, off, w_ref=wr, nthreads=nt, out=o,
                                  cells=args.cells)
            assert o["info"][3] == 0
            done += B
            k += 1
            dt = time.perf_counter() - t0
            if dt >= budget:
                return done / dt, k, dt

    v, runs, dt = timed(threads, args.cpu_seconds / 2)
    v1, runs1, dt1 = timed(1, args.cpu_seconds / 4)
    out = {"value": v, "unit": "QP/s", "cores": threads, "kind": "port (same algorithm as the GPU path engine)",
           "sample": f"{runs} runs x {B} EVs (horizon {N}, 24 sets, full outputs, the timed steps' prices) in {dt:.1f} s, "
                     f"OpenMP {threads} threads (oracle/path_cpu.cpp, {args.cells or 'default'} cells per set as the GPU plan)",
           "single_thread": {"value": v1, "sample": f"{runs1} runs x {B} EVs in {dt1:.1f} s, 1 thread"},
           **host_threads_note(threads)}
    if ref is not None:
        o = oracle_c.path_run(N, cs, [P, P], lms[-1], lr, g, off, w_ref=wr, nthreads=threads, cells=args.cells)
        out["parity"] = {"step": "the last timed step (all EVs)",
                         "max_abs_dw": float(np.abs(o["w"] - ref["w"]).max()),
                         "max_rel_dcost": float((np.abs(o["cost"] - ref["cost"]) / np.maximum(1.0, np.abs(ref["cost"]))).max()),
                         "max_rel_dset_sum_w": float((np.abs(o["set_sum_w"] - ref["set_sum_w"])
                                                      / np.maximum(1.0, np.abs(ref["set_sum_w"]))).max()),
                         "counts_equal": bool(np.array_equal(o["set_stats"][:, 0], ref["set_stats"][:, 0]))}
        if not out["parity"]["max_abs_dw"] <= 1e-9:
            raise SystemExit(f"bench.py: CPU path engine and GPU differ: {out['parity']}")
    return out


def cpu_baseline(eng, N, seconds, seed=0):
    """C oracle (dense primal active set, oracle/lompc_oracle.c) on this host's cores over a
    bounded sample of the same workload (both EV types, the last step's partition-0 prices):
    the headline figure on every host thread, plus one thread (the reference's per-EV loop on
    one core) and the lmbd_r = 3 N delta U variant (test_lompc.py:35) on every thread."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle_c  # checker / baseline only

    oracle_c.build()
    threads = oracle_c.max_threads()
    rng = np.random.default_rng(seed + 7)
    samples = []
    for e in eng:
        g = e["gamma"].cpu().numpy()
        lm = e["lm"][-1, 0].cpu().numpy()
        samples.append((e["c"], lm, g, 3 * N * e["c"].delta * rng.random()))

    def timed(nthreads, budget, lr_on):
        for c, lm, g, lr in samples:  # warm-up (page-in, thread pool) before the calibration
            oracle_c.solve_batch(N, c, lm, lr if lr_on else 0.0, g[:64 * nthreads], nthreads=nthreads)
        n_cal = 256 * nthreads
        t0 = time.perf_counter()
        for c, lm, g, lr in samples:
            oracle_c.solve_batch(N, c, lm, lr if lr_on else 0.0, g[:n_cal], nthreads=nthreads)
        rate = 2 * n_cal / (time.perf_counter() - t0)
        n = int(min(len(samples[0][2]), max(n_cal, rate * budget / 2)))
        # a batch smaller than `budget` of CPU work is repeated (the same QPs solved from scratch
        # each pass, as the reference's per-EV loop does at every price iteration)
        reps = max(1, int(round(rate * budget / (2 * n))))
        t0 = time.perf_counter()
        done = 0
        for _ in range(reps):
            for c, lm, g, lr in samples:
                _, _, nf = oracle_c.solve_batch(N, c, lm, lr if lr_on else 0.0, g[:n], nthreads=nthreads)
                assert nf == 0
                done += n
        dt = time.perf_counter() - t0
        return done / dt, done, reps, n, dt

    v, done, reps, n, dt = timed(threads, seconds, False)
    v1, done1, _, n1, dt1 = timed(1, seconds / 3, False)
    vr, doner, _, nr, dtr = timed(threads, seconds / 3, True)
    return {"value": v, "unit": "QP/s", "cores": threads, "kind": "port",
            "sample": f"{done} QPs ({reps} passes over {n} small + {n} large EVs, horizon {N}, partition-0 "
                      f"prices, lmbd_r = 0) in {dt:.1f} s, C oracle dense active set, OpenMP {threads} threads",
            **host_threads_note(threads), "seed": seed,
            "single_thread": {"value": v1, "sample": f"{done1} QPs in {dt1:.1f} s, 1 thread"},
            "lmbd_r_random": {"value": vr, "sample": f"{doner} QPs in {dtr:.1f} s, {threads} threads, "
                                                     "lmbd_r = 3 N delta U[0,1] per type"}}


if __name__ == "__main__":
    main()
