"""Per-wave launch patterns, busy time, span and the idle gap before the next wave, from a rocprofv3 kernel
trace of bench.py (synchronous waves and the pipelined leg's asynchronous ones, told apart by k_wave_tail).
Usage: python profiles/wave_gaps.py <trace dir>"""
import collections
import csv
import glob
import os
import re
import sys


def name(r):
    m = re.search(r"(k_\w+)", r["Kernel_Name"])
    return m.group(1) if m else r["Kernel_Name"].split("(")[0][:24]


def main():
    f = glob.glob(os.path.join(sys.argv[1], "**", "*kernel_trace.csv"), recursive=True)[0]
    rows = sorted(csv.DictReader(open(f)), key=lambda r: int(r["Start_Timestamp"]))
    starts = [i for i, r in enumerate(rows) if name(r) == "k_roots"]
    waves = []
    for a, b in zip(starts, starts[1:] + [len(rows)]):
        seq = rows[a:b]
        # a wave ends at its publish; what follows (restore copies, the next wave's init) is between waves
        end = max(i for i, r in enumerate(seq) if name(r) == "k_publish") if any(name(r) == "k_publish" for r in seq) else len(seq) - 1
        w = seq[:end + 1]
        t0, t1 = int(w[0]["Start_Timestamp"]), int(w[-1]["End_Timestamp"])
        busy = sum(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in w)
        nxt = int(rows[b]["Start_Timestamp"]) if b < len(rows) else None
        kinds = collections.Counter(name(r) for r in w)
        waves.append(dict(async_=kinds.get("k_wave_tail", 0) > 0, launches=len(w), span=(t1 - t0) / 1e3,
                          busy=busy / 1e3, gap=(nxt - t1) / 1e3 if nxt else None,
                          pattern=" ".join(name(r).replace("k_", "") for r in w), kinds=kinds,
                          per={k: sum(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in w if name(r) == k) / 1e3
                               for k in kinds}))
    for label, sel in (("synchronous", False), ("asynchronous", True)):
        ws = [w for w in waves if w["async_"] == sel][-10:]
        if not ws:
            continue
        n = len(ws)
        gaps = [w["gap"] for w in ws if w["gap"] is not None]
        print(f"{label}: {n} waves, launches {ws[-1]['launches']}: {ws[-1]['pattern']}")
        print(f"  span {sum(w['span'] for w in ws) / n:.1f} us, busy {sum(w['busy'] for w in ws) / n:.1f} us, "
              f"gap to the next wave {sum(gaps) / max(1, len(gaps)):.1f} us")
        ks = sorted({k for w in ws for k in w["per"]})
        print("  per wave: " + ", ".join(f"{k} {sum(w['per'].get(k, 0) for w in ws) / n:.1f}" for k in ks))


if __name__ == "__main__":
    main()
