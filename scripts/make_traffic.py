"""profiles/traffic.json from a PMC session (scripts/pmc_session.sh): HBM-side bytes per
k_eval launch = 2 x FETCH_SIZE (gfx950 reports half of the bytes of wide coalesced reads,
MI355X_MICROARCH.md "HBM") + WRITE_SIZE, both in KiB per dispatch."""
import collections
import csv
import glob
import json
import sys

root = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/pmc"
out = sys.argv[2] if len(sys.argv) > 2 else "profiles/traffic.json"
vals = collections.defaultdict(list)
for f in sorted(glob.glob(f"{root}/p*/run_counter_collection.csv")):
    for r in csv.DictReader(open(f)):
        if r["Kernel_Name"].replace("void ", "").startswith("k_eval"):
            vals[r["Counter_Name"]].append(float(r["Counter_Value"]))
fetch = sum(vals["FETCH_SIZE"]) / len(vals["FETCH_SIZE"]) * 1024.0
write = sum(vals["WRITE_SIZE"]) / len(vals["WRITE_SIZE"]) * 1024.0
qp = 131072.0
rec = {
    "kernel": "k_eval<24,24>", "mode": "path", "horizon": 24, "qp_per_launch": qp,
    "fetch_bytes_per_launch": 2.0 * fetch, "write_bytes_per_launch": write,
    "hbm_bytes_per_launch": 2.0 * fetch + write,
    "algorithmic_bytes_per_launch": 208.0 * qp,
    "dispatches": len(vals["FETCH_SIZE"]),
    "source": "rocprofv3 --kernel-trace --pmc FETCH_SIZE / WRITE_SIZE (separate passes), bench.py --steps 3 --warmup 2; "
              "FETCH_SIZE doubled per MI355X_MICROARCH.md; KiB -> bytes",
}
json.dump(rec, open(out, "w"), indent=1)
print(json.dumps(rec, indent=1))
