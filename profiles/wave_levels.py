#!/usr/bin/env python3
"""Per-level trace of the configs[1] wave (measurement only): builds R-MAT 24, runs a few waves with
FGI_TRACE=1 (the engine prints each level's direction, frontier, edges, chunking and k_level time,
and the wave's pull statistics to stderr).  Usage: FGI_TRACE=1 [WL_OPTS=1=0,...] python profiles/wave_levels.py [config]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402
import torch  # noqa: E402

import _pkg  # noqa: E402

pkg = _pkg.load()
from stl_fusion_amd import workloads as W  # noqa: E402

cfg = dict(W.CONFIGS[sys.argv[1] if len(sys.argv) > 1 else "rmat24"])
g = pkg.Graph(W.n_slots(cfg))
W.build(g, cfg)
roots = W.roots_for(g, cfg)
d_roots = torch.from_numpy(roots.astype(np.int32)).cuda()
for kv in filter(None, os.environ.get("WL_OPTS", "").split(",")):   # option=value pairs (fgi.h FGI_OPT_*)
    k, v = kv.split("=")
    g.set_option(int(k), int(v))
g.snapshot()
for k in range(3):
    g.restore()
    st = pkg.WaveStats()
    g.invalidate_dev(len(roots), d_roots.data_ptr(), 0, st)
    print(f"wave {k}: v_inv {st.v_inv} e_trav {st.e_trav} kernel {st.kernel_ms:.3f} ms pull {st.pull_ms:.3f} "
          f"push {st.expand_ms:.3f}", file=sys.stderr, flush=True)
