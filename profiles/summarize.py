#!/usr/bin/env python3
"""Summarise a profiles/run_profile.sh output directory (gpurun_out/prof_<tag>) into
profiles/<tag>_summary.json + profiles/<tag>_kernel_stats.csv.

Per wave kernel, over the timed steps only (the last `--steps` waves, each wave starting at a
k_roots dispatch): launches per wave, average launch duration (kernel trace), and per-launch PMC
values from the separate counter passes. HBM traffic follows MI355X_MICROARCH.md §HBM:
FETCH_SIZE (KiB) is doubled (gfx950 tallies 128-B requests at 64 B), WRITE_SIZE taken as is; the
doubling holds for the engine's narrow gathers too (profiles/r13e_fetch_calib.txt: one 128-B line
request per miss for 4-B and 8-B gathers, 16-B streams and 256-B runs alike). Usage: python profiles/summarize.py gpurun_out/prof_r02 r02 [--steps 5]
"""
import argparse
import csv
import json
import os
import shutil

WAVE_KERNELS = ("k_roots", "k_level_begin", "k_scan_reduce", "k_scan_apply", "k_mark", "k_expand", "k_pull",
                "k_pull_long", "k_clear_front", "k_level", "k_collect", "k_wave_init",
                "k_final_count", "k_final_write", "k_final", "k_wave_tail", "k_publish")


def base_name(n):
    n = n.strip('"')
    for k in WAVE_KERNELS:
        if n == k or n.startswith(k + "<") or n.startswith("void " + k) or n.startswith(k + "("):
            return k
    return n.split("(")[0].split("<")[0]


def last_waves(rows, steps, name_key, t_key):
    """Dispatches of the last `steps` waves (a wave starts at k_roots)."""
    rows = sorted(rows, key=lambda r: int(r[t_key]))
    starts = [i for i, r in enumerate(rows) if base_name(r[name_key]) == "k_roots"]
    if len(starts) < steps:
        return [], 0
    lo = starts[-steps]
    return [r for r in rows[lo:] if base_name(r[name_key]) in WAVE_KERNELS], steps


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("tag")
    ap.add_argument("--steps", type=int, default=5)
    a = ap.parse_args()
    here = os.path.dirname(os.path.abspath(__file__))
    trace = list(csv.DictReader(open(os.path.join(a.dir, "trace", "run_kernel_trace.csv"))))
    tr, n_w = last_waves(trace, a.steps, "Kernel_Name", "Start_Timestamp")
    out = {"tag": a.tag, "waves": n_w, "kernels": {}}
    for r in tr:
        k = base_name(r["Kernel_Name"])
        d = out["kernels"].setdefault(k, {"launches": 0, "total_ns": 0})
        d["launches"] += 1
        d["total_ns"] += int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
    for k, d in out["kernels"].items():
        d["launches_per_wave"] = d["launches"] / n_w
        d["avg_launch_us"] = d["total_ns"] / d["launches"] / 1e3
        d["ms_per_wave"] = d["total_ns"] / n_w / 1e6
    if tr:
        t0 = min(int(r["Start_Timestamp"]) for r in tr)
        t1 = max(int(r["End_Timestamp"]) for r in tr)
        out["wave_span_ms"] = (t1 - t0) / n_w / 1e6
        out["wave_busy_ms"] = sum(d["total_ns"] for d in out["kernels"].values()) / n_w / 1e6
    for sub in sorted(os.listdir(a.dir)):
        if not sub.startswith("pmc_"):
            continue
        f = os.path.join(a.dir, sub, "run_counter_collection.csv")
        if not os.path.exists(f):
            continue
        rows = list(csv.DictReader(open(f)))
        by_disp = {}
        for r in rows:
            by_disp.setdefault(r["Dispatch_Id"], []).append(r)
        disp = [v[0] | {"_vals": {x["Counter_Name"]: float(x["Counter_Value"]) for x in v}} for v in by_disp.values()]
        sel, n = last_waves(disp, a.steps, "Kernel_Name", "Start_Timestamp")
        for r in sel:
            k = base_name(r["Kernel_Name"])
            d = out["kernels"].setdefault(k, {})
            for c, v in r["_vals"].items():
                d.setdefault("pmc_sum", {}).setdefault(c, 0.0)
                d["pmc_sum"][c] += v
    for k, d in out["kernels"].items():
        s = d.get("pmc_sum", {})
        L = d.get("launches", 0) or 1
        d["pmc_per_launch"] = {c: v / L for c, v in s.items()}
        if "FETCH_SIZE" in s and "WRITE_SIZE" in s:
            d["hbm_bytes_per_launch"] = (2 * s["FETCH_SIZE"] + s["WRITE_SIZE"]) * 1024 / L
            d["hbm_bytes_per_wave"] = (2 * s["FETCH_SIZE"] + s["WRITE_SIZE"]) * 1024 / n_w
            if d.get("total_ns"):
                d["hbm_gbs_pmc"] = (2 * s["FETCH_SIZE"] + s["WRITE_SIZE"]) * 1024 / d["total_ns"]
    dst = os.path.join(here, f"{a.tag}_summary.json")
    json.dump(out, open(dst, "w"), indent=1, sort_keys=True)
    shutil.copy(os.path.join(a.dir, "trace", "run_kernel_stats.csv"), os.path.join(here, f"{a.tag}_kernel_stats.csv"))
    bj = os.path.join(a.dir, "trace_bench.json")
    if os.path.exists(bj):
        shutil.copy(bj, os.path.join(here, f"{a.tag}_bench_under_rocprof.json"))
    print(json.dumps({k: {kk: (round(vv, 3) if isinstance(vv, float) else vv) for kk, vv in d.items()
                          if kk not in ("pmc_sum", "pmc_per_launch")} for k, d in out["kernels"].items()}, indent=1))
    print("wave span %.3f ms, busy %.3f ms" % (out.get("wave_span_ms", 0), out.get("wave_busy_ms", 0)))


if __name__ == "__main__":
    main()
