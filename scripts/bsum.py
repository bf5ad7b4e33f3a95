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
