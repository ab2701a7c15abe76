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


@pytest.mark.parametrize("collectives", [1, 0])
def test_rccl_partition_world1_mutations_match_oracle(pkg, gpu_available, collectives):
    """fgi_part_run_batch / fgi_part_invalidate_all / fgi_part_prune through a real RCCL communicator
    (world size 1): the add_used and begin_compute all-reduces, the cascades and the prune's
    current-node all-gather. Per batch: the invalidated slots, add_used codes, set flags and every
    node word against the oracle; then InvalidateEverything."""
    from harness import canon_edges, random_states
    from test_gpu_part_mutations import _churn_batch
    scale, ef, seed, sseed = 11, 8, 3, 0x5EED00C0
    n = 1 << scale
    rng = np.random.default_rng(77)
    versions, flags = random_states(n, rng, seed=seed)
    s, d = O.gen_rmat(scale, ef, seed)
    live = (versions[s] != 0) & ((flags[s] & 3) == 1)   # only Consistent nodes hold `_usedBy`
    s, d = s[live], d[live]
    tags = versions[d].astype(np.uint64).copy()
    tags[tags == 0] = 7
    tags[rng.random(len(s)) < 0.2] += np.uint64(1)
    g = pkg.Graph(n, n_detached=256, rank=0, world=1)
    g.part_init(n, pkg.fgi.part_unique_id())
    g.set_option(pkg.fgi.OPT_PART_COLLECTIVES, collectives)
    present = np.nonzero(versions)[0].astype(np.uint32)
    g.part_register_nodes(present, versions[present], flags[present])
    g.part_load_edges(s, d, tags)
    o = O.Oracle(n)
    o.load_graph(versions, flags, s, d, tags)
    nv = (1 << 41) | 1
    for b in range(4):
        ov, _ = o.dump_states()
        steps, nv = _churn_batch(rng, n, ov != 0, nv)
        ids, outs = g.part_run_batch(steps)
        o.clear_log()
        for sp in steps:
            if sp[0] == "invalidate":
                o.invalidate_slots(sp[1], sp[2] if len(sp) > 2 else None)
            elif sp[0] == "begin_compute":
                o.begin_compute_slots(sp[1], sp[2], sp[3])
            elif sp[0] == "add_used":
                assert np.array_equal(outs[2], o.add_used_slots(sp[1], sp[2])), b
            else:
                assert int(outs[3].sum()) == o.set_output_slots(sp[1]), b
        assert np.array_equal(np.sort(ids), np.sort(o.inv_log())), b
        v, f = g.dump_states()
        ov, of = o.dump_states()
        assert np.array_equal(v[:n], ov) and np.array_equal(f[:n], of), b
    ps = g.part_prune()
    _, ne = o.prune()
    assert ps.new_edges == ne
    u, dd, t = g.export_edges()
    keep = u < n
    assert np.array_equal(canon_edges(u[keep], dd[keep], t[keep]), canon_edges(*o.export_used_by()))
    o.clear_log()
    ids = g.part_invalidate_all()
    o.invalidate_everything()
    assert np.array_equal(np.sort(ids), np.sort(o.inv_log()))
    v, f = g.dump_states()
    ov, of = o.dump_states()
    assert np.array_equal(v[:n], ov) and np.array_equal(f[:n], of)
    o.close()
    g.close()


def test_rccl_partition_world1_single_mutation_calls(pkg, gpu_available):
    """The standalone partition mutation entry points (fgi_part_begin_compute / add_used / set_output /
    invalidate_all) at world size 1 over RCCL, against the oracle's calls one by one."""
    from harness import random_states
    scale, ef, seed = 10, 8, 11
    n = 1 << scale
    rng = np.random.default_rng(5)
    versions, flags = random_states(n, rng, p_empty=0.0, seed=seed)
    s, d = O.gen_rmat(scale, ef, seed)
    live = (flags[s] & 3) == 1
    s, d = s[live], d[live]
    tags = versions[d].astype(np.uint64).copy()
    g = pkg.Graph(n, n_detached=128, rank=0, world=1)
    g.part_init(n, pkg.fgi.part_unique_id())
    g.set_option(pkg.fgi.OPT_PART_COLLECTIVES, 1)
    g.part_register_nodes(np.arange(n, dtype=np.uint32), versions, flags)
    g.part_load_edges(s, d, tags)
    o = O.Oracle(n)
    o.load_graph(versions, flags, s, d, tags)

    def same_states():
        v, f = g.dump_states()
        ov, of = o.dump_states()
        return np.array_equal(v[:n], ov) and np.array_equal(f[:n], of)

    bc = rng.choice(n, 40, replace=False).astype(np.uint32)
    ver = np.arange(1 << 44, (1 << 44) + 2 * len(bc), 2, dtype=np.uint64) | np.uint64(1)
    hd = (rng.random(len(bc)) < 0.3).astype(np.uint8)
    o.clear_log()
    det, ids = g.part_begin_compute(bc, ver, hd)
    o.begin_compute_slots(bc, ver, hd)
    assert np.array_equal(np.sort(ids), np.sort(o.inv_log()))
    assert same_states()
    dep = rng.choice(bc, 60).astype(np.uint32)
    use = rng.choice(n, 60).astype(np.uint32)
    assert np.array_equal(g.part_add_used(dep, use), o.add_used_slots(dep, use))
    assert same_states()
    o.clear_log()
    out_set, ids = g.part_set_output(bc)
    assert int(out_set.sum()) == o.set_output_slots(bc)
    assert np.array_equal(np.sort(ids), np.sort(o.inv_log()))
    assert same_states()
    o.clear_log()
    ids = g.part_invalidate_all()
    o.invalidate_everything()
    assert np.array_equal(np.sort(ids), np.sort(o.inv_log()))
    assert same_states()
    o.close()
    g.close()
