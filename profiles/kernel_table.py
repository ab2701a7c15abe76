#!/usr/bin/env python3
"""Per-kernel launch counts and average / total durations from a rocprofv3 kernel trace, over the
dispatches after the first `skip` fraction of the run. Usage: python profiles/kernel_table.py <trace.csv> [skip]"""
import csv
import sys
from collections import defaultdict

rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
skip = float(sys.argv[2]) if len(sys.argv) > 2 else 0.5
rows = rows[int(len(rows) * skip):]
agg = defaultdict(lambda: [0, 0])
for r in rows:
    k = r["Kernel_Name"].split("(")[0].split("<")[0].replace("void ", "")
    agg[k][0] += 1
    agg[k][1] += int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
span = (int(rows[-1]["End_Timestamp"]) - int(rows[0]["Start_Timestamp"])) / 1e3
for k, (n, t) in sorted(agg.items(), key=lambda x: -x[1][1]):
    print(f"{k:40s} n={n:6d} avg={t / n / 1e3:9.2f} us total={t / 1e3:10.1f} us")
print(f"span {span:.1f} us")
