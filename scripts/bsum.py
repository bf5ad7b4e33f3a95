"""Summarise bench JSON lines in gpurun_out/*.log (diagnostics)."""
import glob
import json
import sys

for f in (sys.argv[1:] or sorted(glob.glob("gpurun_out/b*.log"))):
    for x in open(f):
        if x.startswith("{"):
            d = json.loads(x)
            r = d["roofline"]
            extra = ""
            if "bimpc" in d:
                b = d["bimpc"]
                extra = f" | bimpc {b.get('value', 0):.1f} steps/s {b.get('error', '')}"
            print(f"{f}: {d['value']:.3e} QP/s, {d['ms_per_step'] * 1e3:.1f} us/step, {r['kernel']} "
                  f"{r['avg_launch_us']:.1f} us, frac {r['frac']:.3f}, repaired {d.get('repaired_qps')}{extra}")
            ks = d.get("kernels", {})
            print("   kernels:", {k: round(v["avg_us"], 2) for k, v in ks.items() if isinstance(v, dict) and "avg_us" in v})
            for k, v in d.get("contracts", {}).items():
                print(f"   {k}: {v['value']:.3e} QP/s, {v['ms_per_step'] * 1e3:.1f} us/step, path {v['k_path_avg_us']:.1f}"
                      f" eval {v['k_eval_avg_us']:.1f} us")
