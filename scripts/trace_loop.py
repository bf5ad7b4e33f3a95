"""Price-loop timeline from a rocprofv3 kernel trace (bench.py station leg / station_profile.py):
per queue, the average duration of each plan kernel and of the idle gap in front of it (end of
the previous kernel on that queue -> its start), i.e. where a device-resident price iteration's
time goes.

usage: python scripts/trace_loop.py [prof_dir] [kernel substring filter]
"""
import collections
import csv
import os
import sys

d = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/sprofk"
flt = sys.argv[2] if len(sys.argv) > 2 else ""
f = next(os.path.join(r, x) for r, _, fs in os.walk(d) for x in fs if x.endswith("kernel_trace.csv"))
rows = list(csv.DictReader(open(f)))


def short(n):
    n = n.replace("void ", "").replace("(anonymous namespace)::", "")
    return n.split("(")[0][:28]


byq = collections.defaultdict(list)
for r in rows:
    byq[r["Queue_Id"]].append(r)
for q, rs in sorted(byq.items()):
    rs.sort(key=lambda r: int(r["Start_Timestamp"]))
    dur = collections.defaultdict(list)
    gap = collections.defaultdict(list)
    prev_end = None
    for r in rs:
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        k = short(r["Kernel_Name"])
        dur[k].append(e - s)
        if prev_end is not None and s - prev_end < 200_000:  # gaps > 200 us: host phases, not the loop
            gap[k].append(s - prev_end)
        prev_end = e
    span = (int(rs[-1]["End_Timestamp"]) - int(rs[0]["Start_Timestamp"])) / 1e3
    print(f"queue {q}: {len(rs)} dispatches over {span:.0f} us")
    for k in sorted(dur, key=lambda k: -sum(dur[k])):
        if flt and flt not in k:
            continue
        g = gap[k]
        print(f"  {k:30s} n {len(dur[k]):6d}  avg {sum(dur[k]) / len(dur[k]) / 1e3:8.2f} us"
              f"  gap before avg {sum(g) / max(len(g), 1) / 1e3:7.2f} us")
