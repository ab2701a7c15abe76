"""GPU parity: the HIP engine (through the C-ABI) against the CPU oracle on identical inputs.

Bar: bit-exact — same invalidated set, same final (version, state, flags) for every slot, same
V_inv / E_trav / E_match / flag counts, same `_usedBy` edge sets after a prune on both sides.
"""
import numpy as np
import pytest

import _pkg
import fgo as O
from harness import (COMPUTING, CONSISTENT, F_DS, F_HD, F_IOSO, INVALIDATED, assert_states_equal, build_pair,
                     canon_edges, oracle_edges, random_states)

pytestmark = pytest.mark.gpu


def _edges_from_live(versions, flags, rng, m, n, stale_p=0.3):
    # only Consistent nodes have `_usedBy` entries: AddUsedBy throws on a Computing node
    # (Computed.cs:374-375) and an Invalidated node's set is cleared (Computed.cs:217)
    live = np.nonzero((versions != 0) & ((flags & 3) == CONSISTENT))[0].astype(np.uint32)
    src = rng.choice(live, m).astype(np.uint32)
    dst = rng.integers(0, n, m).astype(np.uint32)
    tags = versions[dst].astype(np.uint64).copy()
    tags[tags == 0] = 7
    stale = rng.random(m) < stale_p
    tags[stale] += np.uint64(1)
    return src, dst, tags


def _compare_wave(g, o, n, roots, imm=None, exact_match=False):
    """One wave on both sides. V_inv, E_trav and the sets/states are always exact; E_match is
    exact only on the push path with the dead-edge filter off (otherwise it counts examined edges)."""
    st = O.Stats()
    o.clear_log()
    o.invalidate_slots(roots, imm, stats=st)
    ws = _pkg.load().WaveStats()
    ids = g.invalidate(roots, imm, stats=ws)
    oids = o.inv_log()
    assert np.array_equal(np.sort(ids), np.sort(oids)), f"invalidated sets differ: {len(ids)} vs {len(oids)}"
    assert len(np.unique(ids)) == len(ids), "a node was invalidated twice"
    assert ws.v_inv == st.v_inv and ws.e_trav == st.e_trav, (ws.v_inv, st.v_inv, ws.e_trav, st.e_trav)
    if exact_match:
        assert ws.e_match == st.e_match, (ws.e_match, st.e_match)
    # n_flagged is informational: which visit sets a flag first is order-dependent
    assert_states_equal(g, o, n)
    return ids, ws


def test_synth_layered_matches_cpu_definition(pkg, gpu_available):
    levels, width, fanout, seed = 5, 300, 4, 0x5EED0001
    g = pkg.Graph(levels * width)
    g.synth_layered(levels, width, fanout, seed)
    u, d, t = g.export_edges()
    s, dd = O.gen_layered(levels, width, fanout, seed)
    tt = O.gen_tags(s, dd, seed)
    assert np.array_equal(canon_edges(u, d, t), canon_edges(s, dd, tt))
    v, f = g.dump_states()
    assert np.array_equal(v[:levels * width], O.version_of(seed, np.arange(levels * width)))
    assert np.all(f[:levels * width] == CONSISTENT)


@pytest.mark.parametrize("scale,ef,stale", [(10, 8, 0), (12, 16, 50)])
def test_synth_rmat_matches_cpu_definition(pkg, gpu_available, scale, ef, stale):
    seed, sseed = 0x5EED0024, 0x5EED00C0
    g = pkg.Graph(1 << scale)
    g.synth_rmat(scale, ef, seed, stale, sseed)
    u, d, t = g.export_edges()
    s, dd = O.gen_rmat(scale, ef, seed)
    tt = O.gen_tags(s, dd, seed, stale, sseed)
    assert np.array_equal(canon_edges(u, d, t), canon_edges(s, dd, tt))


def _oracle_from_synth(n, seed, s, dd, tt):
    o = O.Oracle(n)
    o.load_graph(O.version_of(seed, np.arange(n)), None, s, dd, tt)
    return o


def test_wave_layered_config1_shape(pkg, gpu_available):
    """BASELINE config 1 shape (fan-out 8, depth 6) at reduced width."""
    levels, width, fanout, seed = 7, 2000, 8, 0x5EED0001
    n = levels * width
    g = pkg.Graph(n)
    g.synth_layered(levels, width, fanout, seed)
    s, dd = O.gen_layered(levels, width, fanout, seed)
    o = _oracle_from_synth(n, seed, s, dd, O.gen_tags(s, dd, seed))
    deg = np.bincount(s, minlength=n)
    roots = O.gen_roots(20, width, 0x5EED1001, deg[:width])
    ids, ws = _compare_wave(g, o, n, roots)
    assert ws.levels >= 5 and len(ids) > 1000


PATHS = {  # name -> (direction, dead filter)
    "push_nofilter": (1, 0), "push": (1, 1), "pull": (2, 1), "auto": (0, 1), "auto_alpha2": (0, 1),
    # 256 hot heads at most: on these small graphs most list heads are then probed in the invalidated
    # bitmap itself instead of the hot snapshot
    "pull_cold": (2, 1), "auto_cold": (0, 1)}


def _set_path(g, name):
    d, f = PATHS[name]
    g.set_option(2, d)
    g.set_option(1, f)
    if name == "auto_alpha2":
        g.set_option(3, 2)
    if name.endswith("_cold"):
        g.set_option(10, 256)   # FGI_OPT_HOT_HEADS


@pytest.mark.parametrize("path", list(PATHS))
@pytest.mark.parametrize("stale", [0, 50])
def test_wave_rmat(pkg, gpu_available, stale, path):
    scale, ef, seed = 13, 16, 0x5EED0024
    n = 1 << scale
    g = pkg.Graph(n)
    _set_path(g, path)
    g.synth_rmat(scale, ef, seed, stale, 0x5EED00C0)
    s, dd = O.gen_rmat(scale, ef, seed)
    o = _oracle_from_synth(n, seed, s, dd, O.gen_tags(s, dd, seed, stale, 0x5EED00C0))
    deg = np.bincount(s, minlength=n)
    roots = O.gen_roots(64, n, 0x5EED1024, deg)
    ids, ws = _compare_wave(g, o, n, roots, exact_match=(path == "push_nofilter"))
    assert len(ids) > 64
    if path == "pull":
        assert ws.pull_levels == ws.levels
    # second wave on the already-invalidated graph is a no-op
    ids2, ws2 = _compare_wave(g, o, n, roots)
    assert len(ids2) == 0


@pytest.mark.parametrize("path", ["push_nofilter", "push", "pull", "pull_cold"])
def test_wave_mixed_states_and_immediately(pkg, gpu_available, path):
    rng = np.random.default_rng(7)
    n = 5000
    versions, flags = random_states(n, rng)
    src, dst, tags = _edges_from_live(versions, flags, rng, 40000, n)
    g, o = build_pair(pkg, n, versions, flags, src, dst, tags)
    _set_path(g, path)
    assert_states_equal(g, o, n)
    roots = rng.integers(0, n, 300).astype(np.uint32)   # duplicates and empty slots included
    imm = (rng.random(300) < 0.3).astype(np.uint8)
    _compare_wave(g, o, n, roots, imm, exact_match=(path == "push_nofilter"))


@pytest.mark.parametrize("path", ["push", "pull"])
def test_hub_row_spans_many_chunks(pkg, gpu_available, path):
    """One `Everything()`-style hub with 200k dependants (UserService.cs:178-179 shape)."""
    n = 300_000
    versions = O.version_of(3, np.arange(n))
    flags = np.full(n, CONSISTENT, np.uint32)
    dst = np.arange(1, 200_001, dtype=np.uint32)
    src = np.zeros(len(dst), np.uint32)
    tags = versions[dst].copy()
    tags[::7] += np.uint64(1)     # some stale
    # second level: each dependant feeds one more node
    src2 = dst[:50_000]
    dst2 = (dst[:50_000] + 200_000).astype(np.uint32) % n
    src = np.concatenate([src, src2])
    dst = np.concatenate([dst, dst2])
    tags = np.concatenate([tags, versions[dst2]])
    g, o = build_pair(pkg, n, versions, flags, src, dst, tags)
    _set_path(g, path)
    _compare_wave(g, o, n, np.array([0], np.uint32))


@pytest.mark.parametrize("path", ["push", "pull", "pull_cold"])
def test_cycles_and_self_loops(pkg, gpu_available, path):
    n = 1000
    versions = O.version_of(5, np.arange(n))
    flags = np.full(n, CONSISTENT, np.uint32)
    src = np.arange(n, dtype=np.uint32)
    dst = ((src + 1) % n).astype(np.uint32)            # one big cycle
    src = np.concatenate([src, np.arange(0, n, 10, dtype=np.uint32)])
    dst = np.concatenate([dst, np.arange(0, n, 10, dtype=np.uint32)])   # self loops
    tags = versions[dst]
    g, o = build_pair(pkg, n, versions, flags, src, dst, tags)
    _set_path(g, path)
    ids, ws = _compare_wave(g, o, n, np.array([17], np.uint32))
    assert len(ids) == n and ws.levels == n


@pytest.mark.parametrize("labels", [-1, 1])
def test_deep_waves_through_the_tail(pkg, gpu_available, labels):
    """A 1,000-level wave (one cycle with self loops), repeated from a snapshot: the first wave runs as
    level groups; the repeats know the wave is deeper than its head and run its levels in the
    persistent tail (k_wave_tail), far past the 64-entry level ring, with one host synchronisation.
    Every wave equals the oracle: the set, V_inv, E_trav, the level count and every node word; the
    asynchronous entry point (the tail with every level) too."""
    import torch
    n = 1000
    versions = O.version_of(5, np.arange(n))
    flags = np.full(n, CONSISTENT, np.uint32)
    src = np.arange(n, dtype=np.uint32)
    dst = ((src + 1) % n).astype(np.uint32)
    src = np.concatenate([src, np.arange(0, n, 10, dtype=np.uint32)])
    dst = np.concatenate([dst, np.arange(0, n, 10, dtype=np.uint32)])
    tags = versions[dst]
    g = pkg.Graph(n, labels=labels)
    g.register_nodes(np.arange(n, dtype=np.uint32), versions, flags)
    g.load_edges(src, dst, tags)
    o = O.Oracle(n)
    o.load_graph(versions, flags, src, dst, tags)
    g.snapshot()
    o.snapshot()
    roots = np.array([17], np.uint32)
    for rep in range(3):
        g.restore()
        o.restore()
        ids, ws = _compare_wave(g, o, n, roots)
        assert len(ids) == n and ws.levels == n, (rep, ws.levels)
        if rep:
            assert ws.host_syncs == 1, (rep, ws.host_syncs)
    d_roots = torch.from_numpy(roots.astype(np.int32)).cuda()
    torch.cuda.synchronize()
    for rep in range(2):
        g.restore()
        ws = pkg.WaveStats()
        nv, _ = g.wave_wait(g.invalidate_async(1, d_roots.data_ptr()), ws)
        assert nv == n and ws.v_inv == n and ws.e_trav == 1100 and ws.levels == n, (ws.v_inv, ws.e_trav, ws.levels)
    o.restore()
    o.invalidate_slots(roots)
    assert_states_equal(g, o, n)
    g.close()
    o.close()


def test_empty_and_noop_waves(pkg, gpu_available):
    n = 100
    versions = O.version_of(9, np.arange(n))
    flags = np.full(n, CONSISTENT, np.uint32)
    g, o = build_pair(pkg, n, versions, flags, np.zeros(0, np.uint32), np.zeros(0, np.uint32), np.zeros(0, np.uint64))
    assert len(g.invalidate(np.zeros(0, np.uint32))) == 0
    _compare_wave(g, o, n, np.array([3, 3, 3], np.uint32))   # no edges, duplicate root
    _compare_wave(g, o, n, np.array([3], np.uint32))         # already invalidated


def test_invalidate_all(pkg, gpu_available):
    rng = np.random.default_rng(11)
    n = 3000
    versions, flags = random_states(n, rng)
    src, dst, tags = _edges_from_live(versions, flags, rng, 20000, n)
    g, o = build_pair(pkg, n, versions, flags, src, dst, tags)
    st = O.Stats()
    o.clear_log()
    o.invalidate_everything(st)
    ids = g.invalidate_all()
    assert np.array_equal(np.sort(ids), np.sort(o.inv_log()))
    assert_states_equal(g, o, n)


def test_prune_matches_pruner(pkg, gpu_available):
    rng = np.random.default_rng(13)
    n = 4000
    versions, flags = random_states(n, rng, p_delay=0.0)
    src, dst, tags = _edges_from_live(versions, flags, rng, 30000, n, stale_p=0.5)
    g, o = build_pair(pkg, n, versions, flags, src, dst, tags)
    roots = rng.integers(0, n, 50).astype(np.uint32)
    _compare_wave(g, o, n, roots)
    ps = g.prune()
    oe, ne = o.prune()
    assert (ps.old_edges, ps.new_edges) != (0, 0)
    assert ps.new_edges == ne
    u, d, t = g.export_edges()
    assert np.array_equal(canon_edges(u, d, t), oracle_edges(o, n))
    # a wave after compaction still agrees
    _compare_wave(g, o, n, rng.integers(0, n, 50).astype(np.uint32))


class Pair:
    """Engine + oracle driven by the same compute-method operations; handles mapped both ways."""

    def __init__(self, pkg, n, n_detached=256):
        self.g = pkg.Graph(n, n_detached=n_detached)
        self.o = O.Oracle(n)
        self.n = n
        self.o2g = {}        # oracle node handle -> engine handle
        self.home = {}       # engine detached handle -> slot

    def begin(self, slots, versions, has_delay):
        det = self.g.begin_compute(slots, versions, has_delay)
        for s, v, hd, dh in zip(slots, versions, has_delay, det):
            cur = self.o.current(int(s))
            new, displaced = self.o.begin_compute(int(s), int(v), bool(hd))
            if displaced != O.NONE and cur != O.NONE:
                ost = self.o.node_info(displaced)[2] & 3
                if ost != INVALIDATED:
                    assert dh != 0xFFFFFFFF, "engine did not detach a surviving displaced node"
                    self.o2g[displaced] = int(dh)
                    self.home[int(dh)] = int(s)
                else:
                    self.o2g.pop(displaced, None)
            self.o2g[new] = int(s)

    def node(self, slot):
        return self.o.last(slot)


@pytest.mark.parametrize("path", ["auto", "pull", "pull_cold"])
def test_compute_method_lifecycle_random(pkg, gpu_available, path):
    """Random begin_compute / add_used / set_output / invalidate sequences (streaming-mix shape).
    Under "pull" every level is bottom-up, so the dependency-list cache is rebuilt after each
    mutation batch (detached nodes, displaced rows, appended rows)."""
    rng = np.random.default_rng(21)
    n = 600
    p = Pair(pkg, n)
    _set_path(p.g, path)
    versions = O.version_of(77, np.arange(n))
    next_ver = versions.copy()
    # everything starts Consistent via a compute + set_output round
    slots = np.arange(n, dtype=np.uint32)
    p.begin(slots, next_ver, (rng.random(n) < 0.1).astype(np.uint8))
    p.g.set_output(slots)
    for s in slots:
        p.o.set_output(p.node(int(s)))
    for step in range(25):
        # 1. a batch of recomputations
        k = int(rng.integers(5, 60))
        bs = rng.choice(n, k, replace=False).astype(np.uint32)
        next_ver[bs] += np.uint64(1000)
        hd = (rng.random(k) < 0.15).astype(np.uint8)
        p.begin(bs, next_ver[bs], hd)
        # 2. dependency capture: each recomputed node uses a few others
        dep, use = [], []
        for s in bs:
            for u in rng.choice(n, int(rng.integers(1, 5)), replace=False):
                dep.append(int(s))
                use.append(int(u))
        dep = np.array(dep, np.uint32)
        use = np.array(use, np.uint32)
        res = p.g.add_used(dep, use)
        ores = [p.o.add_used(p.node(int(d)), p.node(int(u))) for d, u in zip(dep, use)]
        assert list(res) == ores, f"add_used results differ at step {step}"
        # 3. some computations finish (in order; duplicates of a node are no-ops)
        fin = bs[rng.random(len(bs)) < 0.8]
        oset, ids = p.g.set_output(fin)
        o_set = [p.o.set_output(p.node(int(s))) for s in fin]
        assert list(oset) == o_set
        # 4. an invalidation wave (immediately for some roots)
        roots = rng.integers(0, n, 8).astype(np.uint32)
        imm = (rng.random(8) < 0.25).astype(np.uint8)
        p.o.clear_log()
        p.o.invalidate_slots(roots, imm)
        gids = p.g.invalidate(roots, imm)
        assert np.array_equal(np.sort(gids), np.sort(p.o.inv_log())), f"step {step}"
        assert_states_equal(p.g, p.o, n)
        # 5. a delayed invalidation firing on detached nodes: Invalidate(true) on the object
        det = [(oh, gh) for oh, gh in p.o2g.items() if gh >= n]
        if det and step % 3 == 0:
            oh, gh = det[int(rng.integers(0, len(det)))]
            p.o.clear_log()
            p.o.invalidate_nodes([oh], [1])
            gids = p.g.invalidate(np.array([gh], np.uint32), np.array([1], np.uint8))
            # engine ids are handles: a detached node reports its own handle, the oracle its slot
            gslots = np.array([p.home.get(int(x), int(x)) for x in gids], np.uint32)
            assert np.array_equal(np.sort(gslots), np.sort(p.o.inv_log()))
            assert_states_equal(p.g, p.o, n)
    # used counts and edge sets after a prune on both sides
    for s in range(0, n, 37):
        assert p.g.used_count(s) == p.o.used_count(p.node(s))
    p.g.prune()
    p.o.prune()
    u, d, t = p.g.export_edges()
    ge = canon_edges(u, d, t)
    ge = ge[ge[:, 0] < n] if len(ge) else ge
    assert np.array_equal(ge, oracle_edges(p.o, n))


def test_waves_of_alternating_shapes(pkg, gpu_available):
    """One graph, restored between waves whose shapes alternate (a 256-root wave that pulls, a
    one-node wave without levels): each wave matches the oracle bit-exactly, whatever the previous
    wave's level grouping and pull-list state."""
    scale, ef, seed = 13, 16, 0x5EED0024
    n = 1 << scale
    g = pkg.Graph(n)
    g.synth_rmat(scale, ef, seed, 0, 0)
    s, dd = O.gen_rmat(scale, ef, seed)
    o = _oracle_from_synth(n, seed, s, dd, O.gen_tags(s, dd, seed))
    deg = np.bincount(s, minlength=n)
    big = O.gen_roots(256, n, 0x5EED1024, deg)
    small = np.nonzero(deg == 0)[0][:1].astype(np.uint32)   # a node without dependants
    g.snapshot()
    o.snapshot()
    shapes = []
    for roots in (big, small, big, small, small, big, big):
        g.restore()
        o.restore()
        ids, ws = _compare_wave(g, o, n, roots)
        shapes.append(ws.pull_levels)
    # (the first wave builds the pull-list cache and runs push-only)
    assert max(shapes) > 0 and shapes[1] == 0, shapes


@pytest.mark.parametrize("scale,stale", [(13, 0), (20, 50)])
def test_bitmap_output_equals_id_list(pkg, gpu_available, scale, stale):
    """fgi_invalidate_bits returns the wave's invalidated set as a bitmap over handles: the same set
    as fgi_invalidate's id list, the same statistics and final states; the id list is still
    available afterwards (fgi_last_wave_ids builds it from the bitmap on demand)."""
    seed, sseed = 0x5EED0024, 0x5EED00C0
    n = 1 << scale
    g = pkg.Graph(n, n_detached=64)
    g.synth_rmat(scale, 16, seed, stale, sseed)
    deg, _ = g.degrees()
    roots = O.gen_roots(4096 if scale > 13 else 64, n, 0x5EED1024, deg[:n])
    imm = (np.arange(len(roots)) % 7 == 0).astype(np.uint8)
    g.snapshot()
    ws = pkg.WaveStats()
    ids = g.invalidate(roots, imm, stats=ws)
    v1, f1 = g.dump_states()
    for pinned in (False, True):
        g.restore()
        wb = pkg.WaveStats()
        if pinned:
            buf = pkg.fgi.Pinned(((g.n_handles + 63) // 64) * 8, np.uint64)
            _, nb = g.invalidate_bits(roots, imm, stats=wb, out_ptr=buf.ptr)
            bits = buf.array.copy()
            buf.close()
        else:
            bits, nb = g.invalidate_bits(roots, imm, stats=wb)
        got = pkg.fgi.bits_to_ids(bits)
        assert nb == len(ids) == wb.v_inv and np.array_equal(got, np.sort(ids))
        assert (wb.v_inv, wb.e_trav) == (ws.v_inv, ws.e_trav)
        assert np.array_equal(g.last_wave_ids(), np.sort(ids))   # the list, made on demand
        v2, f2 = g.dump_states()
        assert np.array_equal(v1, v2) and np.array_equal(f1, f2)
    g.close()
