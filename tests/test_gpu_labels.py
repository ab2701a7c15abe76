"""Hub-first labels (stl.fusion_amd/csrc/labels.hip), forced on small graphs
(fgi_config.labels = 1; graphs of at least 2^25 slots get them automatically, e.g. configs[2] in
test_gpu_configs.py, and FGI_LABELS=1 forces them on every graph of the whole suite).

The labels must be invisible at the boundary: every entry point takes and returns slots and handles
as the host numbers them. Checked against the oracle (Computed.cs:162-230 cascade, 141-160
TrySetOutput, 347-385 AddUsed, 400-419 PruneUsedBy, ComputedRegistry.cs:72-105 Register): the
invalidated ids in ascending slot order (the final collect's fold of the hot labels), the bitmap output,
every node word, degrees, exported edges, `_usedBy` of single nodes, the single mutation calls, streaming
batches with detached handles, and the pruner's walk over handle ranges."""
import numpy as np
import pytest

import fgo as O
from harness import assert_states_equal, canon_edges, oracle_edges, random_states
from test_gpu_part_mutations import _churn_batch

pytestmark = pytest.mark.gpu

SSEED = 0x5EED00C0


def _alive_pairs(o):
    """(slot, version) of every oracle node that is not Invalidated (current or displaced)."""
    import ctypes as C
    out, h = set(), 0
    sl, v, f = C.c_uint32(), C.c_uint64(), C.c_uint32()
    while o.l.fgo_node_info(o.o, h, C.byref(sl), C.byref(v), C.byref(f)) == 0:
        if v.value and (f.value & 3) != 2:
            out.add((sl.value, v.value))
        h += 1
    return out


def _rmat(pkg, scale, ef, seed, stale, labels):
    n = 1 << scale
    g = pkg.Graph(n, n_detached=64, labels=labels)
    g.synth_rmat(scale, ef, seed, stale, SSEED)
    return g


def _oracle_rmat(scale, ef, seed, stale):
    n = 1 << scale
    s, d = O.gen_rmat(scale, ef, seed)
    o = O.Oracle(n)
    o.load_graph(O.version_of(seed, np.arange(n)), None, s, d, O.gen_tags(s, d, seed, stale, SSEED))
    return o, s


@pytest.mark.parametrize("stale", [0, 50])
@pytest.mark.parametrize("direction", [0, 1, 2])
def test_labelled_rmat_waves_match_oracle(pkg, gpu_available, stale, direction):
    scale, ef, seed = 16, 16, 0x5EED0027
    n = 1 << scale
    g = _rmat(pkg, scale, ef, seed, stale, 1)
    plain = _rmat(pkg, scale, ef, seed, stale, -1)
    o, s = _oracle_rmat(scale, ef, seed, stale)
    g.set_option(pkg.fgi.OPT_DIRECTION, direction)
    # the boundary's views of the graph equal the unlabelled engine's
    dg, tg = g.degrees()
    dp, tp = plain.degrees()
    assert tg == tp and np.array_equal(dg, dp)
    assert np.array_equal(canon_edges(*g.export_edges()), canon_edges(*plain.export_edges()))
    deg = np.bincount(s, minlength=n)
    for w, (k, rseed) in enumerate(((256, 0x5EED1027), (16, 99), (1024, 7))):
        roots = O.gen_roots(k, n, rseed, deg)
        imm = (np.arange(len(roots)) % 7 == 0).astype(np.uint8)
        o.clear_log()
        st = o.invalidate_slots(roots, imm)
        ws = pkg.WaveStats()
        ids = g.invalidate(roots, imm, stats=ws)
        assert np.all(np.diff(ids.astype(np.int64)) > 0), "ids not in ascending slot order"
        assert np.array_equal(ids, np.sort(o.inv_log())), w
        assert ws.v_inv == st.v_inv
        if w == 0:
            assert ws.e_trav == st.e_trav
        assert_states_equal(g, o, n)
    # the bitmap output: the same wave as a bitmap over slots
    roots = O.gen_roots(64, n, 12345, deg)
    o.clear_log()
    o.invalidate_slots(roots)
    bits, nb = g.invalidate_bits(roots)
    assert np.array_equal(pkg.fgi.bits_to_ids(bits), np.sort(o.inv_log())) and nb == len(o.inv_log())
    assert np.array_equal(g.last_wave_ids(), np.sort(o.inv_log()))
    assert_states_equal(g, o, n)
    o.close()
    g.close()
    plain.close()


def test_labelled_device_roots_and_snapshot(pkg, gpu_available):
    """fgi_invalidate_dev (the bench's call: roots in device memory, as boundary slots) and
    fgi_restore on a labelled graph: repeated waves give the same ids as the oracle."""
    import torch
    scale, ef, seed = 15, 8, 0x5EED0027
    n = 1 << scale
    g = _rmat(pkg, scale, ef, seed, 0, 1)
    o, s = _oracle_rmat(scale, ef, seed, 0)
    roots = O.gen_roots(128, n, 0x5EED1027, np.bincount(s, minlength=n))
    o.snapshot()
    g.snapshot()
    want = None
    d_roots = torch.from_numpy(roots.astype(np.int32)).cuda()
    for rep in range(3):
        g.restore()
        o.restore()
        o.clear_log()
        o.invalidate_slots(roots)
        want = np.sort(o.inv_log())
        n_inv = g.invalidate_dev(len(roots), d_roots.data_ptr(), 0, pkg.WaveStats())
        assert n_inv == len(want)
        assert np.array_equal(g.last_wave_ids(), want), rep
        assert_states_equal(g, o, n)
    o.close()
    g.close()


@pytest.mark.parametrize("labels", [1, -1])
def test_labelled_mutations_batches_and_prune(pkg, gpu_available, labels):
    """Mixed states (Computing, delays, Invalidated and empty slots, stale edges) loaded through
    fgi_register_nodes + fgi_load_edges into a labelled graph; the single mutation calls, streaming
    batches (detached handles, displacement, add_used, set_output cascades), fgi_get_used_by, the
    pruner's walk over handle ranges and a full prune, each against the oracle."""
    scale, ef, seed = 12, 8, 3
    n = 1 << scale
    rng = np.random.default_rng(91)
    versions, flags = random_states(n, rng, seed=seed)
    s, d = O.gen_rmat(scale, ef, seed)
    live = (versions[s] != 0) & ((flags[s] & 3) == 1)
    s, d = s[live], d[live]
    tags = versions[d].astype(np.uint64).copy()
    tags[tags == 0] = 7
    tags[rng.random(len(s)) < 0.25] += np.uint64(1)
    g = pkg.Graph(n, n_detached=256, labels=labels)
    present = np.nonzero(versions)[0].astype(np.uint32)
    g.register_nodes(present, versions[present], flags[present])
    g.load_edges(s, d, tags)
    o = O.Oracle(n)
    o.load_graph(versions, flags, s, d, tags)
    assert_states_equal(g, o, n)
    # single calls
    bc = rng.choice(n, 40, replace=False).astype(np.uint32)
    ver = np.arange(1 << 44, (1 << 44) + 2 * len(bc), 2, dtype=np.uint64) | np.uint64(1)
    hd = (rng.random(len(bc)) < 0.3).astype(np.uint8)
    o.clear_log()
    det = g.begin_compute(bc, ver, hd)
    o.begin_compute_slots(bc, ver, hd)
    assert np.array_equal(np.sort(g.last_wave_ids()), np.sort(o.inv_log()))
    assert np.all((det == pkg.fgi.NONE) | ((det >= n) & (det < n + 256))), det
    assert_states_equal(g, o, n)
    dep = rng.choice(bc, 60).astype(np.uint32)
    ov, _ = o.dump_states()
    use = rng.choice(np.nonzero(ov)[0], 60).astype(np.uint32)   # AddUsed takes a node: slots that hold one
    ga, oa = g.add_used(dep, use), o.add_used_slots(dep, use)
    assert np.array_equal(ga, oa), np.nonzero(ga != oa)[0]
    assert_states_equal(g, o, n)
    o.clear_log()
    out_set, ids = g.set_output(bc)
    assert int(out_set.sum()) == o.set_output_slots(bc)
    assert np.array_equal(np.sort(ids), np.sort(o.inv_log()))
    assert_states_equal(g, o, n)
    # streaming batches
    nv = (1 << 45) | 1
    for b in range(4):
        ov, _ = o.dump_states()
        steps, nv = _churn_batch(rng, n, ov != 0, nv)
        ids, outs = g.run_batch(steps)
        o.clear_log()
        for k, sp in enumerate(steps):
            if sp[0] == "invalidate":
                o.invalidate_slots(sp[1], sp[2] if len(sp) > 2 else None)
            elif sp[0] == "begin_compute":
                o.begin_compute_slots(sp[1], sp[2], sp[3])
                det = outs[k]
                assert np.all((det == pkg.fgi.NONE) | (det >= n)), det
            elif sp[0] == "add_used":
                assert np.array_equal(outs[k], o.add_used_slots(sp[1], sp[2])), b
            else:
                assert int(outs[k].sum()) == o.set_output_slots(sp[1]), b
        assert np.array_equal(np.sort(ids), np.sort(o.inv_log())), b
        assert_states_equal(g, o, n)
    # `_usedBy` of single nodes: fgi_get_used_by lists the live entries (fgi.h: a dependant d@t that
    # is still alive and not Invalidated; the rows keep the others until a prune, as the reference's
    # sets keep entries of collected nodes until PruneUsedBy, Computed.cs:400-419)
    live = _alive_pairs(o)
    for x in rng.choice(n, 64, replace=False):
        gd, gt = g.used_by(int(x))
        oh = o.current(int(x))
        od, ot = o.used_by(oh) if oh != O.NONE else (np.zeros(0, np.uint32), np.zeros(0, np.uint64))
        keep = np.array([(int(a), int(b)) in live for a, b in zip(od, ot)], bool)
        od, ot = od[keep] if len(od) else od, ot[keep] if len(ot) else ot
        assert np.array_equal(canon_edges(np.full(len(gd), x), gd, gt), canon_edges(np.full(len(od), x), od, ot)), x
    # the pruner's walk over handle ranges, then a full prune
    batch = 1000
    for lo in range(0, g.n_handles, batch):
        ps = g.prune_range(lo, batch)
        _, ne = o.prune_range(lo, batch)
        assert ps.new_edges == ne and (ps.first, ps.count) == (lo, min(batch, g.n_handles - lo)), lo
    u, dd, t = g.export_edges()
    ge = canon_edges(u, dd, t)
    ge = ge[ge[:, 0] < n] if len(ge) else ge
    assert np.array_equal(ge, oracle_edges(o, n))
    ps = g.prune()
    _, ne = o.prune()
    assert ps.new_edges == ne
    o.clear_log()
    ids = g.invalidate_all()
    o.invalidate_everything()
    assert np.array_equal(np.sort(ids), np.sort(o.inv_log()))
    assert_states_equal(g, o, n)
    o.close()
    g.close()
