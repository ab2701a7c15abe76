#!/usr/bin/env python3
"""configs[3]'s prune without torch (measurement only): build R-MAT 24 with 50% stale edges, run one
wave from host roots (it builds the dependency lists, so fgi_prune takes its fast path; FGI_PRUNE_GATHER=1
pins the gathers), then fgi_prune. Only the HIP runtime libfgi links is loaded, so rocprofv3's exit-time
fault was expected not to occur; it does (round 3, profiles/r6m_*), so FGI_RESET_AT_EXIT=1 calls
hipDeviceReset before the interpreter exits, while the profiler is still active.
Usage: python3 profiles/prune_pmc.py   (prints one JSON line)"""
import ctypes
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import _pkg  # noqa: E402

pkg = _pkg.load()
from stl_fusion_amd import workloads as W  # noqa: E402

cfg = W.CONFIGS["rmat24_churn"]
g = pkg.Graph(W.n_slots(cfg))
W.build(g, cfg)
roots = W.roots_for(g, cfg)
g.snapshot()
ws = pkg.WaveStats()
g.invalidate(roots, stats=ws)   # builds the dependency lists
g.restore()                     # every node Consistent again, as bench_configs.py's configs[3] prune
ps = g.prune()
print(json.dumps({"v_inv": int(ws.v_inv), "old_edges": int(ps.old_edges), "new_edges": int(ps.new_edges),
                  "kernel_ms": ps.kernel_ms, "gather": bool(os.environ.get("FGI_PRUNE_GATHER"))}), flush=True)
g.close()
if os.environ.get("FGI_RESET_AT_EXIT"):
    hip = ctypes.CDLL("libamdhip64.so")
    print(json.dumps({"hipDeviceReset": hip.hipDeviceReset()}), flush=True)
