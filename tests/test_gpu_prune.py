"""Incremental pruning (ComputedGraphPruner.cs:79-94, Computed.cs:400-419).

(a) A batched prune sequence: fgi_prune_range over consecutive handle ranges (the pruner's walk
    over the registry in batches), checked after every batch against the oracle's prune of the
    same slots, and, once the walk has covered every handle, the whole edge set.
(b) Long rows (hubs past the one-wave path): their in-place compaction keeps exactly the live
    entries, in order.
(c) fgi_prune_step runs only once waves have made enough entries stale, then walks the handles.
(d) A full prune with and without defragmentation gives the same rows; defragmenting shrinks the
    pool and leaves row slack.
(e) The walk interleaved with recompute / AddUsed / wave churn, through both prune paths.
"""
import numpy as np
import pytest

import fgo as O
from harness import CONSISTENT, assert_states_equal, build_pair, canon_edges, oracle_edges, random_states
from test_gpu_parity import _compare_wave, _edges_from_live

pytestmark = pytest.mark.gpu


def _rows_of(g, lo, hi, n):
    """Engine rows of slots [lo, hi) as canonical (u, d, t) triples."""
    u, d, t = g.export_edges()
    a = canon_edges(u, d, t)
    if len(a) == 0:
        return a
    return a[(a[:, 0] >= lo) & (a[:, 0] < min(hi, n))]


def _oracle_rows(o, lo, hi, n):
    a = oracle_edges(o, n)
    if len(a) == 0:
        return a
    return a[(a[:, 0] >= lo) & (a[:, 0] < hi)]


@pytest.mark.parametrize("batch", [500, 1337, 4000])
def test_batched_prune_sequence_matches_pruner(pkg, gpu_available, batch):
    rng = np.random.default_rng(29 + batch)
    n = 4000
    versions, flags = random_states(n, rng, p_delay=0.0)
    src, dst, tags = _edges_from_live(versions, flags, rng, 40000, n, stale_p=0.5)
    g, o = build_pair(pkg, n, versions, flags, src, dst, tags)
    _compare_wave(g, o, n, rng.integers(0, n, 40).astype(np.uint32))   # lazily removed entries
    olds = news = 0
    for lo in range(0, g.n_handles, batch):
        ps = g.prune_range(lo, batch)
        oe, ne = o.prune_range(lo, batch)
        assert (ps.first, ps.count) == (lo, min(batch, g.n_handles - lo))
        # new counts agree; old ones may not: the engine keeps RemoveUsedBy'd entries until now
        assert ps.new_edges == ne and ps.old_edges >= oe, (lo, ps.old_edges, ps.new_edges, oe, ne)
        olds += ps.old_edges
        news += ne
        hi = min(lo + batch, n)
        if lo < n:
            assert np.array_equal(_rows_of(g, lo, hi, n), _oracle_rows(o, lo, hi, n)), lo
    u, d, t = g.export_edges()
    ge = canon_edges(u, d, t)
    ge = ge[ge[:, 0] < n] if len(ge) else ge
    assert np.array_equal(ge, oracle_edges(o, n))
    assert news < olds
    # waves after the walk agree
    _compare_wave(g, o, n, rng.integers(0, n, 40).astype(np.uint32))
    g.close()
    o.close()


@pytest.mark.parametrize("lists", [False, True])
def test_long_rows_compact_in_place(pkg, gpu_available, lists):
    """lists=True: a pull-only wave first builds the dependency lists, so the prune reads the entries'
    liveness recorded at that build (fgi_prune's fast path) instead of gathering node words."""
    n = 20000
    rng = np.random.default_rng(31)
    versions = O.version_of(5, np.arange(n))
    flags = np.full(n, CONSISTENT, np.uint32)
    # three hubs with 1,500 / 6,000 / 15,000 entries (the one-block path), 60% stale
    src, dst = [], []
    for hub, m in ((0, 1500), (1, 6000), (2, 15000)):
        src.append(np.full(m, hub, np.uint32))
        dst.append(rng.choice(np.arange(10, n, dtype=np.uint32), m, replace=False))
    src = np.concatenate(src)
    dst = np.concatenate(dst)
    tags = versions[dst].copy()
    tags[rng.random(len(tags)) < 0.6] += np.uint64(2)
    g, o = build_pair(pkg, n, versions, flags, src, dst, tags)
    if lists:   # slot 5 has no row: the wave invalidates it alone
        g.set_option(2, 2)
        _compare_wave(g, o, n, np.array([5], np.uint32))
    before = [g.used_by(hub) for hub in (0, 1, 2)]
    ps = g.prune()
    oe, ne = o.prune()
    assert (ps.old_edges, ps.new_edges) == (oe, ne)
    u, d, t = g.export_edges()
    assert np.array_equal(canon_edges(u, d, t), oracle_edges(o, n))
    for hub, (bd, bt) in zip((0, 1, 2), before):   # the kept entries, in their order
        dd, tt = g.used_by(hub)
        keep = bt == versions[bd]
        assert np.array_equal(dd, bd[keep]) and np.array_equal(tt, bt[keep])
    assert 0 < ps.new_edges < ps.old_edges
    g.close()
    o.close()


def test_prune_step_waits_for_stale_entries(pkg, gpu_available):
    rng = np.random.default_rng(37)
    n = 3000
    versions, flags = random_states(n, rng, p_delay=0.0)
    src, dst, tags = _edges_from_live(versions, flags, rng, 30000, n, stale_p=0.0)
    g, o = build_pair(pkg, n, versions, flags, src, dst, tags)
    ps = g.prune_step(1000, 1)
    assert ps.count == 0 and ps.old_edges == 0                # nothing stale yet: no work
    _compare_wave(g, o, n, rng.integers(0, n, 200).astype(np.uint32))
    covered = 0
    while covered < g.n_handles:
        ps = g.prune_step(1000, 1)
        if ps.count == 0:
            break
        assert ps.stale_estimate > 0
        covered += ps.count
    assert covered >= n
    o.prune()
    u, d, t = g.export_edges()
    ge = canon_edges(u, d, t)
    ge = ge[ge[:, 0] < n] if len(ge) else ge
    assert np.array_equal(ge, oracle_edges(o, n))
    g.close()
    o.close()


def test_defragmentation_keeps_rows(pkg, gpu_available):
    rng = np.random.default_rng(41)
    n = 5000
    versions, flags = random_states(n, rng, p_delay=0.0)
    src, dst, tags = _edges_from_live(versions, flags, rng, 60000, n, stale_p=0.7)
    res = []
    for pct in (0, 30):
        g, o = build_pair(pkg, n, versions, flags, src, dst, tags)
        g.set_option(pkg.fgi.OPT_DEFRAG_PCT, pct)
        ps = g.prune()
        u, d, t = g.export_edges()
        res.append((canon_edges(u, d, t), ps.pool_before, ps.pool_after))
        if pct:
            assert ps.pool_after < ps.pool_before
            # waves over the copied rows still agree
            o.prune()
            _compare_wave(g, o, n, rng.integers(0, n, 30).astype(np.uint32))
        else:
            assert ps.pool_after == ps.pool_before
        g.close()
        o.close()
    assert np.array_equal(res[0][0], res[1][0])


def test_restore_after_in_place_prune(pkg, gpu_available):
    """snapshot -> begin_compute -> fgi_prune_range (rows compacted in place) -> fgi_restore: the
    snapshot's row descriptors no longer describe the compacted rows, so restore must refuse
    (FGI_ESTATE) — or, if it restores, leave a graph whose waves still match the oracle's."""
    rng = np.random.default_rng(43)
    n = 3000
    versions, flags = random_states(n, rng, p_delay=0.0)
    src, dst, tags = _edges_from_live(versions, flags, rng, 30000, n, stale_p=0.5)
    g, o = build_pair(pkg, n, versions, flags, src, dst, tags)
    g.snapshot()
    o.snapshot()
    slots = rng.choice(np.nonzero(versions)[0], 40, replace=False).astype(np.uint32)
    newv = (versions[slots] + np.uint64(2)).astype(np.uint64)
    g.begin_compute(slots, newv)
    for s_, v_ in zip(slots, newv):
        o.begin_compute(int(s_), int(v_))
    g.prune_range(0, g.n_handles)
    try:
        g.restore()
    except pkg.FgiError as e:
        assert e.status == pkg.fgi.ESTATE
        return
    o.restore()
    _compare_wave(g, o, n, rng.integers(0, n, 60).astype(np.uint32))


def test_prune_after_recompute_sees_new_versions(pkg, gpu_available):
    """Lists built by a pull wave, then some nodes recomputed (new versions: the entries that captured
    their old versions go stale) before the prune: the liveness recorded at the list build no longer
    holds, so the prune must check the current versions (mut_epoch moved) and drop those entries."""
    from test_gpu_parity import Pair
    rng = np.random.default_rng(41)
    n = 3000
    p = Pair(pkg, n)
    ver = O.version_of(91, np.arange(n))
    slots = np.arange(n, dtype=np.uint32)
    p.begin(slots, ver, np.zeros(n, np.uint8))
    p.g.set_output(slots)
    for s_ in slots:
        p.o.set_output(p.node(int(s_)))
    # dependencies: every node uses a few others (AddUsed while Computing: recompute a batch first)
    batch = rng.choice(n, 1500, replace=False).astype(np.uint32)
    ver[batch] += np.uint64(1000)
    p.begin(batch, ver[batch], np.zeros(len(batch), np.uint8))
    dep = np.repeat(batch, 4)
    use = rng.integers(0, n, len(dep)).astype(np.uint32)
    res = p.g.add_used(dep, use)
    assert list(res) == [p.o.add_used(p.node(int(d)), p.node(int(u))) for d, u in zip(dep, use)]
    p.g.set_output(batch)
    for s_ in batch:
        p.o.set_output(p.node(int(s_)))
    # a pull-only wave builds the lists (and the pool's liveness bits)
    p.g.set_option(2, 2)
    roots = rng.integers(0, n, 3).astype(np.uint32)
    p.o.clear_log()
    p.o.invalidate_slots(roots)
    gids = p.g.invalidate(roots)
    assert np.array_equal(np.sort(gids), np.sort(p.o.inv_log()))
    # recompute nodes other rows point at: their old-version entries go stale
    used = np.unique(use)
    again = used[rng.random(len(used)) < 0.5].astype(np.uint32)
    ver[again] += np.uint64(7)
    p.begin(again, ver[again], np.zeros(len(again), np.uint8))
    p.g.set_output(again)
    for s_ in again:
        p.o.set_output(p.node(int(s_)))
    ps = p.g.prune()
    oe, ne = p.o.prune()
    assert ps.new_edges == ne, (ps.new_edges, ne)
    u, d, t = p.g.export_edges()
    ge = canon_edges(u, d, t)
    ge = ge[ge[:, 0] < n] if len(ge) else ge
    assert np.array_equal(ge, oracle_edges(p.o, n))


@pytest.mark.parametrize("path", ["auto", "pull"])
def test_prune_windows_interleaved_with_churn(pkg, gpu_available, path):
    """The pruner's walk interleaved with a compute-method workload: each step recomputes a batch,
    captures dependencies, finishes most computations, runs a wave, then prunes one window of slots
    (fgi_prune_range; every third step a whole fgi_prune). Under "pull" every wave rebuilds the
    dependency lists, so the prunes alternate between the liveness recorded at a list build and the
    node-word gather (any mutation in between moves mut_epoch). After every prune the window's rows
    equal the oracle's, and every wave matches the oracle's cascade."""
    from test_gpu_parity import Pair, _set_path
    rng = np.random.default_rng(53)
    n = 2500
    p = Pair(pkg, n, n_detached=8192)
    _set_path(p.g, path)
    ver = O.version_of(17, np.arange(n))
    slots = np.arange(n, dtype=np.uint32)
    p.begin(slots, ver, np.zeros(n, np.uint8))
    p.g.set_output(slots)
    for s_ in slots:
        p.o.set_output(p.node(int(s_)))
    win = 700
    lo = 0
    for step in range(18):
        k = int(rng.integers(50, 400))
        bs = rng.choice(n, k, replace=False).astype(np.uint32)
        ver[bs] += np.uint64(1000)
        p.begin(bs, ver[bs], (rng.random(k) < 0.1).astype(np.uint8))
        dep = np.repeat(bs, rng.integers(1, 6, k))
        use = rng.integers(0, n, len(dep)).astype(np.uint32)
        res = p.g.add_used(dep, use)
        assert list(res) == [p.o.add_used(p.node(int(d)), p.node(int(u))) for d, u in zip(dep, use)]
        fin = bs[rng.random(k) < 0.85]
        p.g.set_output(fin)
        for s_ in fin:
            p.o.set_output(p.node(int(s_)))
        roots = rng.integers(0, n, int(rng.integers(1, 40))).astype(np.uint32)
        p.o.clear_log()
        p.o.invalidate_slots(roots)
        gids = p.g.invalidate(roots)
        assert np.array_equal(np.sort(gids), np.sort(p.o.inv_log())), step
        if step % 3 == 2:
            ps = p.g.prune()
            oe, ne = p.o.prune()
            a, b = 0, n
        else:
            ps = p.g.prune_range(lo, win)
            oe, ne = p.o.prune_range(lo, win)
            a, b = lo, min(lo + win, n)
            lo = 0 if lo + win >= n else lo + win
        assert ps.new_edges >= ne and ps.old_edges >= oe, (step, ps.new_edges, ne)
        assert np.array_equal(_rows_of(p.g, a, b, n), _oracle_rows(p.o, a, b, n)), step
        assert_states_equal(p.g, p.o, n)
    p.g.prune()
    p.o.prune()
    u, d, t = p.g.export_edges()
    ge = canon_edges(u, d, t)
    ge = ge[ge[:, 0] < n] if len(ge) else ge
    assert np.array_equal(ge, oracle_edges(p.o, n))
