#!/usr/bin/env python3
"""Per-dispatch counters of the last wave's kernels from profiles/pmc_levels.sh output.
Usage: python profiles/pmc_levels.py gpurun_out/pmcl_<tag>"""
import csv
import glob
import os
import sys
from collections import defaultdict

root = sys.argv[1]
rows = defaultdict(dict)   # dispatch id -> {counter: value, name}
for f in glob.glob(os.path.join(root, "p*", "**", "*counter_collection.csv"), recursive=True):
    for r in csv.DictReader(open(f)):
        key = (os.path.dirname(f), int(r["Dispatch_Id"]))
        rows[key]["name"] = r["Kernel_Name"].split("(")[0]
        rows[key][r["Counter_Name"]] = rows[key].get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
by_pass = defaultdict(list)
for (d, i), v in sorted(rows.items()):
    by_pass[d].append(v)
names = ("k_roots", "k_collect", "k_level", "k_final_count", "k_final_write", "k_final")
for d, lst in sorted(by_pass.items()):
    # the last wave: from its k_roots on (round 6: a steady-state wave has no k_wave_init)
    starts = [i for i, v in enumerate(lst) if v["name"].startswith("k_roots")]
    tail = lst[starts[-1]:] if starts else lst
    print(f"== {os.path.relpath(d, root)}")
    for v in tail:
        if not v["name"].startswith(names):
            continue
        cs = {k: x for k, x in v.items() if k != "name"}
        print(f"  {v['name'][:16]:16s} " + " ".join(f"{k}={x:.4g}" for k, x in sorted(cs.items())))
