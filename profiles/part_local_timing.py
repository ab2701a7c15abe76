"""Wall time of the 8-rank partitioned wave (run_part_wave with the in-process PartComm: every rank
in its own host thread, the collectives are device copies) on one GPU: restore every partition,
then one fgi_part_local_invalidate of 4,096 roots, K times. Levels and host synchronisations per
level are those of the RCCL path; the collectives are not. Used to A/B level-loop changes
(FGI_LIBRARY selects another build).
Usage: python profiles/part_local_timing.py [scale] [P] [K] [edge factor, default 16]"""
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import _pkg  # noqa: E402

pkg = _pkg.load()
from stl_fusion_amd.workloads import pick_roots  # noqa: E402


def main():
    scale = int(sys.argv[1]) if len(sys.argv) > 1 else 22
    P = int(sys.argv[2]) if len(sys.argv) > 2 else 8
    K = int(sys.argv[3]) if len(sys.argv) > 3 else 20
    ef = int(sys.argv[4]) if len(sys.argv) > 4 else 16
    n = 1 << scale
    block = -(-n // P)
    gs = [pkg.Graph(block, rank=r, world=P) for r in range(P)]
    pkg.fgi.part_init_local(gs, n)
    for g in gs:
        g.part_synth_rmat(scale, ef, 0x5EED0027)
        g.snapshot()
    roots = pick_roots(4096, n, 0x5EED1027, np.ones(n, np.uint8))   # uniform roots
    ts, st = [], None
    for k in range(K + 3):
        for g in gs:
            g.restore()
        t0 = time.perf_counter()
        st = pkg.fgi.part_local_invalidate(gs, roots)
        if k >= 3:
            ts.append(time.perf_counter() - t0)
    ts = np.array(ts) * 1e3
    print(f"lib={os.path.basename(pkg.fgi.LIB_PATH)} labels={os.environ.get('FGI_LABELS', 'auto')} scale={scale} ef={ef} P={P} v_inv={sum(x.v_inv for x in st)} "
          f"levels={st[0].levels} pull_levels={st[0].pull_levels} remote={sum(x.remote_msgs for x in st)} "
          f"wall_ms median={np.median(ts):.3f} min={ts.min():.3f}")


if __name__ == "__main__":
    main()
