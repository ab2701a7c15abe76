"""Diagnostic (round 5): why labelled graphs ran no pull level (FGI_TRACE=1 prints the candidates'
build and every level's direction)."""
import os
import sys

import numpy as np

sys.path.insert(0, ".")
sys.path.insert(0, "oracle")
import _pkg  # noqa: E402
import fgo as O  # noqa: E402

pkg = _pkg.load()
scale, ef, seed = 16, 16, 0x5EED0027
n = 1 << scale
for labels in (-1, 1):
    for direction in (2, 0):
        g = pkg.Graph(n, labels=labels)
        g.set_option(pkg.fgi.OPT_DIRECTION, direction)
        g.synth_rmat(scale, ef, seed)
        s, _ = O.gen_rmat(scale, ef, seed)
        roots = O.gen_roots(1024, n, 0x5EED1027, np.bincount(s, minlength=n))
        g.snapshot()
        for rep in range(2):
            g.restore()
            ws = pkg.WaveStats()
            ids = g.invalidate(roots, stats=ws)
            print(f"labels {labels} direction {direction} wave {rep}: v_inv {ws.v_inv} levels {ws.levels} "
                  f"pull levels {ws.pull_levels} e_trav {ws.e_trav}", file=sys.stderr, flush=True)
        g.close()
