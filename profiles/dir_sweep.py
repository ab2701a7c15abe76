#!/usr/bin/env python3
"""Measurement only: ms per (restore + wave) step of one configuration under each traversal
direction and a few Beamer alpha / beta values (results never depend on them; the tests pin that).
Usage: python profiles/dir_sweep.py [layered_1m|rmat24|rmat24_churn] [steps]"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402
import torch  # noqa: E402

import _pkg  # noqa: E402

pkg = _pkg.load()
from stl_fusion_amd import workloads as W  # noqa: E402

name = sys.argv[1] if len(sys.argv) > 1 else "layered_1m"
steps = int(sys.argv[2]) if len(sys.argv) > 2 else 20
cfg = dict(W.CONFIGS[name])
g = pkg.Graph(W.n_slots(cfg))
W.build(g, cfg)
roots = W.roots_for(g, cfg)
d_roots = torch.from_numpy(roots.astype(np.int32)).cuda()
g.snapshot()


def run(direction, alpha, beta):
    g.set_option(pkg.fgi.OPT_DIRECTION, direction)
    g.set_option(pkg.fgi.OPT_PULL_ALPHA, alpha)
    g.set_option(pkg.fgi.OPT_PULL_BETA, beta)
    g.set_option(pkg.fgi.OPT_LEVEL_TIMING, 0)
    for _ in range(3):
        g.restore()
        g.invalidate_dev(len(roots), d_roots.data_ptr(), 0, pkg.WaveStats())
    st = pkg.WaveStats()
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(steps):
        g.restore()
        g.invalidate_dev(len(roots), d_roots.data_ptr(), 0, st)
    torch.cuda.synchronize()
    ms = (time.perf_counter() - t) / steps * 1e3
    return {"config": name, "direction": direction, "alpha": alpha, "beta": beta, "ms_per_step": ms,
            "v_inv": st.v_inv // steps, "levels": st.levels / steps, "pull_levels": st.pull_levels / steps}


for d, a, b in [(1, 14, 24), (2, 14, 24), (0, 14, 24), (0, 4, 24), (0, 8, 24), (0, 28, 24), (0, 56, 24),
                (0, 14, 4), (0, 14, 96), (0, 28, 96)]:
    print(json.dumps(run(d, a, b)), flush=True)
