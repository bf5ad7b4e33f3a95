"""profiles/pmc.json from a PMC session (scripts/pmc_session.sh: one rocprofv3 --pmc pass per
counter group over `bench.py --steps 3 --warmup 2`), per plan kernel, per dispatch:

* k_step: the launches that carry an evaluation (the fill / drain launches of a call excluded);
* k_eval HBM traffic = 2 x FETCH_SIZE (gfx950 reports half of the bytes of wide coalesced
  reads, MI355X_MICROARCH.md "HBM") + WRITE_SIZE, both KiB per dispatch -> bytes;
* SQ counters (SQ_WAVE_CYCLES, SQ_ACTIVE_INST_* and SQ_WAIT_* count quad-cycles): the VALU-issue
  fraction of a wave's lifetime = SQ_ACTIVE_INST_VALU / SQ_WAVE_CYCLES, the stall split
  WAIT_ANY (parked on s_waitcnt / barriers) and WAIT_INST_ANY (issue stalls).

* k_evals (the wide run_steps' batched evaluation: one dispatch carries R runs): traffic per RUN =
  per dispatch / R (the session runs bench.py with --warmup R --steps R, so every k_evals dispatch
  carries R runs).

usage: python scripts/make_pmc.py [pmc_dir] [out] [evs] [horizon] [runs per k_evals dispatch]
"""
import collections
import csv
import glob
import json
import sys

root = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/pmc"
out = sys.argv[2] if len(sys.argv) > 2 else "profiles/pmc.json"
qp = float(sys.argv[3]) if len(sys.argv) > 3 else 262144.0
N = int(sys.argv[4]) if len(sys.argv) > 4 else 24
R = int(sys.argv[5]) if len(sys.argv) > 5 else 3
KERNELS = ("k_evals", "k_closes", "k_step", "k_paths", "k_path", "k_eval", "k_finalize")
vals = {k: collections.defaultdict(list) for k in KERNELS}
for f in sorted(glob.glob(f"{root}/p*/run_counter_collection.csv")):
    for r in csv.DictReader(open(f)):
        name = r["Kernel_Name"].replace("void ", "").replace("(anonymous namespace)::", "")
        for k in KERNELS:
            if name.startswith(k + "(") or name.startswith(k + "<"):  # (exact-N template instances)
                vals[k][r["Counter_Name"]].append(float(r["Counter_Value"]))


# k_step: only the steady-state launches (an evaluation's rows written: WRITE_SIZE at least half the
# largest); a run_steps call's first launch (path only) and last (closing only) write almost
# nothing.  Every pass runs the same dispatch sequence, so one mask selects the same launches in each
ws_k = vals["k_step"].get("WRITE_SIZE")
if ws_k:
    top = max(ws_k)
    mask = [w >= 0.5 * top for w in ws_k]
    for c, v in list(vals["k_step"].items()):
        if len(v) % len(mask) == 0:  # (a counter collected in several passes: the passes in order)
            vals["k_step"][c] = [x for x, m in zip(v, mask * (len(v) // len(mask))) if m]


def mean(k, c):
    v = vals[k].get(c)
    return sum(v) / len(v) if v else None


rec = {"mode": "path", "horizon": N, "qp_per_launch": qp,
       "source": "rocprofv3 --kernel-trace --pmc, one pass per counter group (scripts/pmc_session.sh), "
                 "bench.py --steps 3 --warmup 3; FETCH_SIZE doubled per MI355X_MICROARCH.md; KiB -> bytes"}
for k in KERNELS:
    d = {}
    waves, cyc = mean(k, "SQ_WAVES"), mean(k, "SQ_WAVE_CYCLES")
    if waves and cyc:
        d["waves"] = waves
        d["wave_cycles_avg"] = 4.0 * cyc / waves
        d["valu_insts_per_wave"] = mean(k, "SQ_INSTS_VALU") / waves
        av, wa, wi = mean(k, "SQ_ACTIVE_INST_VALU"), mean(k, "SQ_WAIT_ANY"), mean(k, "SQ_WAIT_INST_ANY")
        if av is not None:
            d["valu_issue_frac"] = av / cyc
        if wa is not None:
            d["wait_any_frac"] = wa / cyc
        if wi is not None:
            d["wait_inst_frac"] = wi / cyc
    bc, ia = mean(k, "SQ_LDS_BANK_CONFLICT"), mean(k, "SQ_LDS_IDX_ACTIVE")
    if bc is not None and ia:
        d["lds_bank_conflict_frac"] = bc / ia  # conflict cycles / all LDS-array cycles
    fs, ws = mean(k, "FETCH_SIZE"), mean(k, "WRITE_SIZE")
    if fs is not None and ws is not None:
        per = R if k == "k_evals" else 1  # (k_evals: per run)
        d["fetch_bytes_per_launch"] = 2.0 * fs * 1024.0 / per
        d["write_bytes_per_launch"] = ws * 1024.0 / per
        if per > 1:
            d["runs_per_dispatch"] = per
        d["hbm_bytes_per_launch"] = d["fetch_bytes_per_launch"] + d["write_bytes_per_launch"]
        if k in ("k_eval", "k_step", "k_evals"):
            d["algorithmic_bytes_per_launch"] = 8.0 * (N + 2) * qp
    d["dispatches"] = max((len(v) for v in vals[k].values()), default=0)
    if d["dispatches"]:
        rec[k] = d
json.dump(rec, open(out, "w"), indent=1)
print(json.dumps(rec, indent=1))
