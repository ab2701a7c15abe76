"""The RCCL partition path itself (fgi_part_init + fgi_part_invalidate: the code bench.py runs for
N > 1), at world size 1 on one GPU: the level loop, its all-reduces and exchanges go through a real
RCCL communicator (FGI_OPT_PART_COLLECTIVES=1; a one-rank partition otherwise skips them, which
is what bench.py --partition measures at N=1 — both are checked). Results must equal the oracle's
bit-exactly (invalidated set, V_inv, E_trav, final node states), for push-only, pull-only and
automatic direction, with and without stale edges."""
import numpy as np
import pytest
import torch

import fgo as O

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("direction", [0, 1, 2])      # auto, push only, pull only
@pytest.mark.parametrize("stale", [0, 50])
@pytest.mark.parametrize("collectives", [1, 0])
def test_rccl_partition_world1_matches_oracle(pkg, gpu_available, stale, direction, collectives):
    scale, ef, seed, sseed = 12, 16, 0x5EED0027, 0x5EED00C0
    n = 1 << scale
    g = pkg.Graph(n, rank=0, world=1)
    g.part_init(n, pkg.fgi.part_unique_id())
    g.part_synth_rmat(scale, ef, seed, stale, sseed)
    g.set_option(2, direction)
    g.set_option(pkg.fgi.OPT_PART_COLLECTIVES, collectives)
    s, d = O.gen_rmat(scale, ef, seed)
    o = O.Oracle(n)
    o.load_graph(O.version_of(seed, np.arange(n)), None, s, d, O.gen_tags(s, d, seed, stale, sseed))
    deg = np.bincount(s, minlength=n)
    for wave, (k, rseed) in enumerate(((48, 0x5EED1027), (16, 99))):
        roots = O.gen_roots(k, n, rseed, deg)
        imm = (np.arange(len(roots)) % 5 == 0).astype(np.uint8)
        o.clear_log()
        st = o.invalidate_slots(roots, imm)
        d_roots = torch.from_numpy(roots.astype(np.int32)).cuda()
        d_imm = torch.from_numpy(imm).cuda()
        stats = pkg.fgi.WaveStats()
        n_inv = g.part_invalidate(len(roots), d_roots.data_ptr(), d_imm.data_ptr(), stats)
        ids = g.part_export_ids()
        assert n_inv == len(ids) == st.v_inv, wave
        assert np.array_equal(np.sort(ids), np.sort(o.inv_log())), wave
        if wave == 0:
            # later waves: the engine drops RemoveUsedBy'd entries lazily (Computed.cs:387-398 removes
            # them eagerly), so E_trav is pinned on the first wave from a fresh graph, as in
            # test_gpu_part.py; sets and states are pinned on every wave
            assert stats.e_trav == st.e_trav, wave
        if direction == 2:
            assert stats.pull_levels == stats.levels
        ov, of = o.dump_states()
        v, f = g.dump_states()
        assert np.array_equal(v[:n], ov), wave
        assert np.array_equal(f[:n], of), wave
