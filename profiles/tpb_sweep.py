#!/usr/bin/env python3
"""Pull tiles per block (FGI_OPT_PULL_TPB) against wave time on one device (measurement only): a pull
block owns a fixed run of tpb tiles, so with one resident wave of blocks the slowest block sets the
level; more, smaller blocks let the hardware's block scheduler balance them. Restore + device-root wave,
median over K waves per setting, two alternating passes.
Usage: python profiles/tpb_sweep.py [config, default rmat24] [K] [tpb,tpb,...]"""
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

name = sys.argv[1] if len(sys.argv) > 1 else "rmat24"
K = int(sys.argv[2]) if len(sys.argv) > 2 else 30
tpbs = [int(x) for x in (sys.argv[3] if len(sys.argv) > 3 else "0,8,4,2").split(",")]
cfg = dict(W.CONFIGS[name])
g = pkg.Graph(W.n_slots(cfg))
W.build(g, cfg)
roots = W.roots_for(g, cfg)
d_roots = torch.from_numpy(roots.astype(np.int32)).cuda()
g.snapshot()
ref = None
for rep in range(2):
    for tpb in tpbs:
        g.set_option(pkg.fgi.OPT_PULL_TPB, tpb)
        ts, pulls = [], []
        for k in range(K + 3):
            g.restore()
            st = pkg.WaveStats()
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            g.invalidate_dev(len(roots), d_roots.data_ptr(), 0, st)
            torch.cuda.synchronize()
            if k >= 3:
                ts.append((time.perf_counter() - t0) * 1e3)
                pulls.append(st.pull_ms)
        if ref is None:
            ref = (st.v_inv, st.e_trav)
        assert (st.v_inv, st.e_trav) == ref, ((st.v_inv, st.e_trav), ref)
        print(f"{name} tpb={tpb} v_inv={st.v_inv} levels={st.levels} pull_levels={st.pull_levels} "
              f"wave_ms median={np.median(ts):.4f} min={np.min(ts):.4f} pull_ms median={np.median(pulls):.4f}",
              flush=True)
