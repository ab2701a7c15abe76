"""Debug: pull-only first wave of the streaming mix on 2 ranks; full per-rank stats by exchange mode."""
import sys
import numpy as np
sys.path.insert(0, ".")
import _pkg  # noqa
pkg = _pkg.load()
from stl_fusion_amd import workloads as W

for L_, H_ in ((40, 64), (40, 96)):
    for fx in (1, 2):
        mix = W.StreamMix(H_, L_, 8, 10, 0x5EED00E0)
        n = mix.n
        P = 2
        block = -(-n // P)
        gs = [pkg.Graph(block, rank=r, world=P) for r in range(P)]
        pkg.fgi.part_init_local(gs, n)
        used, dep, tag = mix.initial_edges()
        for g in gs:
            g.part_register_nodes(np.arange(n, dtype=np.uint32), mix.version, mix.state_flags())
            g.part_load_edges(used, dep, tag)
            g.set_option(pkg.fgi.OPT_DIRECTION, 2)
            g.set_option(pkg.fgi.OPT_FRONT_EXCHANGE, fx)
        prev = mix.roots(0)
        st = pkg.fgi.part_local_invalidate(gs, prev)
        print("H", H_, "n", n, "block", block, "fx", fx, flush=True)
        for r, x in enumerate(st):
            print("  rank", r, {k: getattr(x, k) for k, _ in x._fields_ if not k.endswith("_ms")}, flush=True)
        print("  front stats", [g.part_front_stats() for g in gs], flush=True)
        for g in gs:
            g.close()
