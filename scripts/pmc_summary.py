"""Per-kernel PMC summary (per dispatch) from gpurun_out/pmc/p*/run_counter_collection.csv."""
import collections
import csv
import glob
import sys

root = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/pmc"
agg = collections.defaultdict(lambda: collections.defaultdict(float))
disp = collections.defaultdict(lambda: collections.defaultdict(set))
for f in sorted(glob.glob(f"{root}/p*/run_counter_collection.csv")):
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"].split("(")[0].replace("void ", "")[:28]
        agg[k][r["Counter_Name"]] += float(r["Counter_Value"])
        disp[k][r["Counter_Name"]].add(r["Dispatch_Id"])
for k, d in agg.items():
    if not k.startswith("k_"):
        continue
    per = {c: v / max(1, len(disp[k][c])) for c, v in d.items()}
    waves = per.get("SQ_WAVES", 1)
    print(f"== {k}  dispatches={len(disp[k]['SQ_WAVES'])}  waves/dispatch={waves:.0f}")
    for c in sorted(per):
        extra = ""
        if c.startswith("SQ_INSTS"):
            extra = f"  ({per[c] / waves:.1f} per wave)"
        print(f"   {c:22s} {per[c]:16.1f}{extra}")
    wc = per.get("SQ_WAVE_CYCLES")
    if wc:
        for c in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY"):
            if c in per:
                print(f"   {c} / WAVE_CYCLES = {per[c] / wc:.2f}")
