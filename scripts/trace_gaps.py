"""Print the per-kernel summary and the last steps' kernel timeline of a rocprofv3 run.

usage: python scripts/trace_gaps.py [prof_dir] [n_last]
"""
import csv
import os
import sys

d = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/prof"
n = int(sys.argv[2]) if len(sys.argv) > 2 else 24
for r in list(csv.DictReader(open(os.path.join(d, "run_kernel_stats.csv"))))[:6]:
    print(f'{r["Name"][:60]:62s} calls {r["Calls"]:>4s} avg {float(r["AverageNs"]) / 1000:7.2f} us  {float(r["Percentage"]):5.1f}%')
t = [r for r in csv.DictReader(open(os.path.join(d, "run_kernel_trace.csv")))
     if "k_" in r["Kernel_Name"][:40]]
t.sort(key=lambda r: int(r["Start_Timestamp"]))
t = t[-n:]
t0 = int(t[0]["Start_Timestamp"])
for r in t:
    s, e = int(r["Start_Timestamp"]) - t0, int(r["End_Timestamp"]) - t0
    print(f'{r["Kernel_Name"].replace("void ", "").replace("(anonymous namespace)::", "")[:12]:13s} q{r.get("Queue_Id", "?"):>2s} '
          f'{s / 1000:8.2f} -> {e / 1000:8.2f}  ({(e - s) / 1000:6.2f} us)')
