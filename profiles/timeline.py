#!/usr/bin/env python3
"""Print the dispatch timeline (gap before, duration) of the last wave in a rocprofv3 kernel trace.
Usage: python profiles/timeline.py gpurun_out/trace_<tag>/trace/run_kernel_trace.csv"""
import csv
import sys

tr = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
starts = [i for i, r in enumerate(tr) if r["Kernel_Name"].startswith("k_roots")]
lo = starts[-2] + 1 if len(starts) > 1 else 0
while lo < len(tr) and not tr[lo]["Kernel_Name"].startswith("k_roots"):
    lo += 1
hi = len(tr)
prev = None
tot = {}
for r in tr[max(0, lo - 8):hi]:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    name = r["Kernel_Name"].split("(")[0][:40]
    print(f"{name:40s} gap {((s - prev) / 1000 if prev else 0):8.2f} dur {(e - s) / 1000:8.2f}")
    prev = e
    tot[name] = tot.get(name, 0) + (e - s) / 1000
print({k: round(v, 1) for k, v in sorted(tot.items(), key=lambda x: -x[1])})
