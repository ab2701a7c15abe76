#!/usr/bin/env python3
"""k_level counters of the in-process partitioned waves (profiles/r14e_session.sh: rocprofv3 --pmc over
profiles/part_local_timing.py): per wave and rank, the summed counters of all k_level dispatches and of the
largest one per rank (a wave's level-1 pull). Usage: python profiles/pmc_part.py <dir> <waves> <ranks>"""
import csv
import glob
import os
import sys
from collections import defaultdict

root, waves, ranks = sys.argv[1], int(sys.argv[2]), int(sys.argv[3])
rows = defaultdict(dict)
for f in glob.glob(os.path.join(root, "**", "*counter_collection.csv"), recursive=True):
    for r in csv.DictReader(open(f)):
        key = int(r["Dispatch_Id"])
        rows[key]["name"] = r["Kernel_Name"]
        rows[key][r["Counter_Name"]] = rows[key].get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
lv = [v for _, v in sorted(rows.items()) if "k_level" in v["name"]]
counters = sorted({k for v in lv for k in v if k != "name"})
# the measured waves are the last `waves` of the run; each has `ranks` k_level launches per level
tot = {c: sum(v.get(c, 0.0) for v in lv) for c in counters}
top = sorted(lv, key=lambda v: -v.get(counters[0], 0.0))[: waves * ranks]
print(f"{root}: {len(lv)} k_level dispatches")
for c in counters:
    print(f"  {c}: all k_level {tot[c] / 1e6:.1f} M; largest {waves * ranks} dispatches (level-1 pulls) "
          f"mean {sum(v.get(c, 0.0) for v in top) / max(1, len(top)) / 1e6:.2f} M per rank-dispatch")
