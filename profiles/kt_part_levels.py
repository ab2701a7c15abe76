"""k_level durations of the in-process partitioned wave from a rocprofv3 kernel trace taken under a counter
pass (dispatches serialised, so each rank's kernel ran alone): the total per rank-wave and the largest
dispatches (the level-1 pulls), per stream (rank).
Usage: python profiles/kt_part_levels.py <trace dir> <waves in the run> [ranks]"""
import collections
import csv
import os
import re
import sys


def main():
    d = sys.argv[1]
    waves = int(sys.argv[2])
    ranks = int(sys.argv[3]) if len(sys.argv) > 3 else 8
    rows = list(csv.DictReader(open(os.path.join(d, "run_kernel_trace.csv"))))
    t0 = min(int(r["Start_Timestamp"]) for r in rows if "k_roots" in r["Kernel_Name"])
    rows = [r for r in rows if int(r["Start_Timestamp"]) >= t0]   # the waves (after the generator)
    key = "Stream_Id" if "Stream_Id" in rows[0] else "Queue_Id"
    lv = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3 for r in rows if "k_level" in r["Kernel_Name"]]
    per = collections.defaultdict(float)
    for r in rows:
        if "k_level" in r["Kernel_Name"]:
            per[r[key]] += (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
    other = collections.defaultdict(float)
    for r in rows:
        m = re.search(r"(k_\w+)", r["Kernel_Name"])
        if m and m.group(1) != "k_level":
            n = m.group(1)
            other[n] += (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
    nw = waves * ranks
    top = sorted(lv, reverse=True)
    print(f"{d}: {len(lv)} k_level dispatches over {nw} rank-waves")
    print(f"  k_level per rank-wave {sum(lv) / nw:.1f} us; per rank (all waves): " +
          " ".join(f"{v / waves:.0f}" for _, v in sorted(per.items())))
    print(f"  largest {ranks * waves} dispatches: mean {sum(top[:nw]) / nw:.1f} us, max {top[0]:.1f}, "
          f"min {top[nw - 1]:.1f}; next {ranks * waves}: mean {sum(top[nw:2 * nw]) / nw:.1f}")
    print("  other wave kernels per rank-wave: " +
          ", ".join(f"{n} {t / nw:.1f}" for n, t in sorted(other.items(), key=lambda x: -x[1])[:8]))


if __name__ == "__main__":
    main()
