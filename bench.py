"""Benchmark: LoMPC QP solves/sec on MI355X (BASELINE.json metric, config 3/4).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--mode path|direct]
    torchrun --nproc-per-node N bench.py --gpus N ...   (one rank per GPU, RCCL)

One step = one batched price iteration of a whole charging-station time step on
this rank's EV shard: for each EV type (small, large) load P = 12 fresh
partition price vectors (lambda ~ theta U[0,1]^{3N}, test_lompc.py:34) and
solve every EV's LoMPC QP (gamma_i = y_max - y0_i, y0 ~ U[0.3, 0.5],
settings.py:27-28) with full outputs (w, cost) plus the fused per-partition
reductions of price_solver.py:203-214; with N > 1 ranks the per-partition
reductions are combined by one RCCL sum + one max all-reduce.  Weak scaling:
262 144 EVs per GPU (config 3; at 8 GPUs this is config 4's 2 097 152).

Rank 0 prints ONE JSON line.  ``roofline`` prices the per-EV kernel (k_eval in
PATH mode, the only kernel whose work scales with the EV count) by its
algorithmic bytes per QP (gamma in 8 B, w out 8N B, cost out 8 B) over its
launch duration from HIP events attached to its dispatch; ``cpu_baseline`` times the C
oracle (oracle/, dense active set) on a bounded sample of the same workload.
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
    ap.add_argument("--warm", action="store_true",
                    help="plan warm start: every gamma cell's exact solve starts from the working set the "
                         "previous step ended with there (as a price loop's plan does)")
    ap.add_argument("--outputs", choices=["full", "cost", "set"], default="full",
                    help="diagnostics: full = w + cost + reductions (the metric's workload); cost = no w rows; "
                         "set = reductions only")
    ap.add_argument("--split-types", action="store_true",
                    help="path mode: one plan per EV type, each on its own stream (overlapping)")
    ap.add_argument("--no-kernel-events", action="store_true",
                    help="diagnostics: no HIP events on the per-EV kernel's dispatches in the timed region")
    ap.add_argument("--cpu-seconds", type=float, default=10.0)
    ap.add_argument("--no-station", action="store_true", help="skip the BiMPC steps/sec leg")
    ap.add_argument("--station-evs-per-gpu", type=int, default=262144, help="EVs per GPU, half per type")
    ap.add_argument("--station-horizon", type=int, default=48)
    ap.add_argument("--station-steps", type=int, default=3)
    ap.add_argument("--station-warmup", type=int, default=1)
    ap.add_argument("--dist-backend", choices=["nccl", "gloo"], default="nccl",
                    help="nccl = RCCL (the product path); gloo only to rehearse world > 1 on one GPU")
    return ap.parse_args()


def main():
    args = parse()
    import torch
    import torch.distributed as dist

    from lompc_amd import BatchPlan, LoMPC, LoMPCConstants, _lib
    from lompc_amd.dist import combine_set_results

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
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
                                    stream=main, warm_start=args.warm), stream=main, lm_ptr=[lm[k].data_ptr() for k in range(nsteps)], lr_ptr=lr.data_ptr(),
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

    def step(k):
        if world > 1 or multi:  # the previous step's collective reads the output buffers
            for r in runs:
                r["stream"].wait_stream(main)
        for r in runs:
            r["plan"].run(r["lm_ptr"][k], r["lr_ptr"])
        if multi:
            for r in runs:
                main.wait_stream(r["stream"])
        if world > 1:
            # every set's reductions (both EV types) in ONE collective
            combine_set_results([(r["plan"].out["set_sum_w"], r["plan"].out["set_stats"]) for r in runs])

    # warmup (and correctness gate: every QP certified)
    for k in range(args.warmup):
        step(k)
    for r in runs:
        rep, fail, inv = r["plan"].check()
        assert fail == 0 and inv == 0, (fail, inv)
    for r in runs:
        r["plan"].profile(enable=("k_eval",) if not args.no_kernel_events else False)
        r["plan"].profile(read=True, reset=True)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for k in range(args.warmup, nsteps):
        step(k)
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
        rep, fail, inv = r["plan"].check()
        assert fail == 0 and inv == 0
        repaired += rep
    # per-EV kernel (k_solve / k_direct) timing: HIP events on its own dispatch (hipExtLaunchKernel)
    k_ms, k_n, k_qps = 0.0, 0, 0
    for r in runs:
        ms, n = r["plan"].profile(read=True)
        k_ms += ms
        k_n += n
        k_qps += r["qps"] * n
    avg_launch_s = (k_ms / 1e3) / max(k_n, 1)
    qp_per_launch = k_qps / max(k_n, 1)
    bytes_per_qp = 8 * (N + 2)
    achieved_gbs = bytes_per_qp * qp_per_launch / avg_launch_s / 1e9 if k_n else 0.0

    total_qp = world * B * args.steps
    value = total_qp / dt
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
            "parallelism": f"dp{world} (EV shards, one RCCL all-gather of both types' per-set reductions per step)",
            "launches_per_step": 2 if args.mode == "path" else 6,
        },
        "roofline": {
            "bound": "hbm",
            "achieved": achieved_gbs,
            "peak": HBM_PEAK_GBS,
            "unit": "GB/s",
            "frac": achieved_gbs / HBM_PEAK_GBS,
            "traffic": None,
            "kernel": "k_solve" if args.mode == "path" else "k_direct",
            "bytes_per_qp": bytes_per_qp,
            "qp_per_launch": qp_per_launch,
            "avg_launch_us": avg_launch_s * 1e6,
        },
        "repaired_qps": repaired,
    }
    traffic_file = os.path.join(ROOT, "profiles", "traffic.json")
    if os.path.exists(traffic_file):
        try:
            tr = json.load(open(traffic_file))
            if tr.get("mode") == args.mode and tr.get("horizon") == N and tr.get("qp_per_launch") == qp_per_launch:
                line["roofline"]["traffic"] = tr["hbm_bytes_per_launch"]
                line["roofline"]["traffic_source"] = tr.get("source")
        except Exception:
            pass
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        line["cpu_baseline"] = cpu_baseline(eng, N, args.cpu_seconds)
    if not args.no_station:
        del eng, runs
        line["bimpc"] = station_leg(args, world, dev)
    if rank == 0:
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.destroy_process_group()


def station_leg(args, world, dev):
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
    consts = station_consts(steps + warm, M_2, n_lo=N, n_bi=N, partitions=P, price_type="linear-convex",
                            demand_scale=DEMAND_SCALE * M_2 / NUM_EVS_PER_EV_TYPE, u_b_max=0.5, x_max=0.5)
    group = dist.group.WORLD if world > 1 else None
    out = {"metric": "BiMPC steps/sec", "unit": "steps/s", "steps": steps, "warmup": warm,
           "config": {"workload": f"config5 shape: {2 * M_2} EVs ({args.station_evs_per_gpu} per GPU), horizon {N}, "
                                  f"{P} partitions per type, linear-convex prices, regularizer on, storage "
                                  "u_b_max = x_max = 0.5, full closed-loop step",
                      "evs_total": 2 * M_2, "horizon": N, "partitions": P}}
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
        t0 = time.perf_counter()
        for _ in range(steps):
            st._step()
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()
        dt = time.perf_counter() - t0
        if world > 1:
            t = torch.tensor([dt], dtype=torch.float64, device=dev)
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            dt = float(t.item())
        stats = st.logs["statistics"]
        it = np.concatenate([stats["niter_s"][:, warm:].ravel(), stats["niter_l"][:, warm:].ravel()])
        ncalls = calls() - c0
        out.update({"value": steps / dt, "ms_per_step": dt / steps * 1e3,
                    "price_iterations_per_step": float(np.sum(it[it >= 0])) / steps,
                    "engine_calls_per_step": ncalls / steps,
                    "lompc_qps_per_sec_est": (ncalls + 2 * P * steps) * M_2 / P / dt})
    except Exception as e:  # reported, never hides the QP/s line
        out["error"] = f"{type(e).__name__}: {e}"
    return out


def cpu_baseline(eng, N, seconds):
    """C oracle (dense primal active set, oracle/lompc_oracle.c) on this host's
    cores over a bounded sample of the same workload (both EV types, the
    last step's partition prices)."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle_c  # checker / baseline only

    oracle_c.build()
    threads = oracle_c.max_threads()
    # calibrate, then size the sample to ~`seconds` of CPU work
    samples = []
    for e in eng:
        g = e["gamma"].cpu().numpy()
        lm = e["lm"][-1, 0].cpu().numpy()
        samples.append((e["c"], lm, g))
    t0 = time.perf_counter()
    n_cal = 256 * threads
    for c, lm, g in samples:
        oracle_c.solve_batch(N, c, lm, 0.0, g[:n_cal], nthreads=threads)
    rate = 2 * n_cal / (time.perf_counter() - t0)
    n = int(min(len(samples[0][2]), max(n_cal, rate * seconds / 2)))
    # the batch holds fewer QPs than `seconds` of CPU work: repeat it (the same QPs, solved
    # from scratch each pass, as the reference's per-EV loop would at every price iteration)
    reps = max(1, int(round(rate * seconds / (2 * n))))
    t0 = time.perf_counter()
    done = 0
    for _ in range(reps):
        for c, lm, g in samples:
            _, _, nf = oracle_c.solve_batch(N, c, lm, 0.0, g[:n], nthreads=threads)
            assert nf == 0
            done += n
    dt = time.perf_counter() - t0
    return {"value": done / dt, "unit": "QP/s", "cores": threads, "kind": "port",
            "sample": f"{done} QPs ({reps} passes over {n} small + {n} large EVs, horizon {N}, partition-0 "
                      f"prices) in {dt:.1f} s, C oracle dense active set, OpenMP {threads} threads"}


if __name__ == "__main__":
    main()
