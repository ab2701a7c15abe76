"""Debug: the streaming mix's first wave on 2 in-process ranks by direction; per-rank stats."""
import sys
import numpy as np
sys.path.insert(0, ".")
import _pkg  # noqa
pkg = _pkg.load()
from stl_fusion_amd import workloads as W

for direction in (1, 2, 0):
    for plan in (0, 1):
        mix = W.StreamMix(64, 40, 8, 10, 0x5EED00E0)
        n = mix.n
        P = 2
        block = -(-n // P)
        gs = [pkg.Graph(block, rank=r, world=P) for r in range(P)]
        pkg.fgi.part_init_local(gs, n)
        used, dep, tag = mix.initial_edges()
        for g in gs:
            g.part_register_nodes(np.arange(n, dtype=np.uint32), mix.version, mix.state_flags())
            g.part_load_edges(used, dep, tag)
            g.set_option(pkg.fgi.OPT_DIRECTION, direction)
            g.set_option(pkg.fgi.OPT_PART_PLAN, plan)
        v1, f1 = gs[1].dump_states()
        print("rank1 states before:", np.bincount(f1[: n - block] & 3, minlength=3), "versions nonzero", int((v1[: n - block] != 0).sum()))
        print("rank1 used_by rows of 0..3:", [gs[1].used_by(i)[0][:3].tolist() for i in range(3)])
        print("rank0 used_by row of hub 31:", gs[0].used_by(31)[0][-5:].tolist(), gs[0].used_by(31)[1][-2:].tolist(), mix.version[1340:1342].tolist())
        prev = mix.roots(0)
        st = pkg.fgi.part_local_invalidate(gs, prev)
        print(direction, plan, [(x.v_inv, x.levels, x.pull_levels, x.remote_msgs, x.e_trav) for x in st], flush=True)
        for g in gs:
            g.close()
