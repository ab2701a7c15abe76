"""Debug: the streaming mix's first wave on 2 in-process ranks, through fgi_part_local_invalidate and
fgi_part_local_run_batch, with and without detached handles; per-rank V_inv and ids."""
import sys
import numpy as np
sys.path.insert(0, ".")
import _pkg  # noqa
pkg = _pkg.load()
sys.path.insert(0, "oracle")
import fgo as O
from stl_fusion_amd import workloads as W

for nd in (0, 256):
    for via in ("invalidate", "batch"):
        mix = W.StreamMix(64, 40, 8, 10, 0x5EED00E0)
        n = mix.n
        P = 2
        block = -(-n // P)
        gs = [pkg.Graph(block, n_detached=nd, rank=r, world=P) for r in range(P)]
        pkg.fgi.part_init_local(gs, n)
        used, dep, tag = mix.initial_edges()
        for g in gs:
            g.part_register_nodes(np.arange(n, dtype=np.uint32), mix.version, mix.state_flags())
            g.part_load_edges(used, dep, tag)
        prev = mix.roots(0)
        if via == "invalidate":
            st = pkg.fgi.part_local_invalidate(gs, prev)
            ids = [g.part_export_ids() for g in gs]
            print(nd, via, [x.v_inv for x in st], [len(i) for i in ids], flush=True)
        else:
            ids, outs, st = pkg.fgi.part_local_run_batch(gs, [("invalidate", prev)])
            print(nd, via, [x.v_inv for x in st], len(ids), [g.part_export_ids().size for g in gs], flush=True)
        for g in gs:
            g.close()
