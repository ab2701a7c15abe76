"""Every BASELINE.json configuration exercised on the GPU at its own size.

configs[0]  layered compute-method graph, 7 x 150,000 slots, fan-out 8, 1,000 roots: the engine
            against the oracle bit-exactly (set, V_inv, E_trav, every final node word) on the
            push, pull and automatic paths.
configs[3]  configs[1]'s generator with 50% stale edges at R-MAT scale 20 (1M slots, 16M edges):
            fgi_prune and a fgi_prune_range walk against the oracle's PruneUsedBy pass
            (Computed.cs:400-419, ComputedGraphPruner.cs:79-94) — identical `_usedBy` edge sets —
            and the waves before and after the prune bit-exact. (The full-scale 50%-stale wave is in
            test_gpu_scale.py.)
configs[2]  R-MAT scale 27, edge factor 8 (134M slots, 1.07G edges, 4,096 roots) on one MI355X:
            the oracle's object graph does not fit a test's time at this size, so each wave is
            checked against the least closure computed independently with torch over the exported
            edge set (closure, witness, E_trav, exact set; tests/closure_check.py), on the
            automatic path (its first wave builds the pull lists), again from the snapshot (pull
            lists ready) and push-only; then 8 vertex-range partitions of the same graph (the
            multi-GPU engine's level loop, in one process) against the single engine, with the
            resident memory per partition measured after the build.
"""
import os

import numpy as np
import pytest

import fgo as O
from harness import CONSISTENT, INVALIDATED, canon_edges

pytestmark = pytest.mark.gpu

THREADS = max(1, min(16, len(os.sched_getaffinity(0))))


def test_configs0_full_size_bit_exact(pkg, gpu_available):
    from stl_fusion_amd import workloads as W
    cfg = W.CONFIGS["layered_1m"]
    levels, width, fanout, seed = cfg["levels"], cfg["width"], cfg["fanout"], cfg["seed"]
    n = levels * width
    O.set_threads(THREADS)
    s, d = O.gen_layered(levels, width, fanout, seed)
    assert len(s) == (levels - 1) * width * fanout   # 7,200,000 edges, fan-out 8
    o = O.Oracle(n)
    o.load_graph(O.version_of(seed, np.arange(n)), None, s, d, O.gen_tags(s, d, seed))
    deg = np.bincount(s, minlength=n)
    roots = O.gen_roots(cfg["roots"], cfg["roots_range"], cfg["roots_seed"], deg[:width])
    assert len(roots) == 1000
    st = o.invalidate_slots(roots, threads=THREADS)
    want = np.sort(o.inv_log())
    ov, of = o.dump_states()
    o.close()
    g = pkg.Graph(n)
    W.build(g, cfg)
    assert np.array_equal(np.sort(W.roots_for(g, cfg)), np.sort(roots))   # bench.py's roots
    g.snapshot()
    for name, direction in (("push", 1), ("pull", 2), ("auto", 0), ("auto_warm", 0)):
        g.restore()
        g.set_option(pkg.fgi.OPT_DIRECTION, direction)
        ws = pkg.WaveStats()
        ids = g.invalidate(roots, stats=ws)
        assert len(np.unique(ids)) == len(ids), name
        assert np.array_equal(np.sort(ids), want), (name, len(ids), len(want))
        assert (ws.v_inv, ws.e_trav) == (st.v_inv, st.e_trav), (name, ws.v_inv, st.v_inv, ws.e_trav, st.e_trav)
        if name == "pull":
            assert ws.pull_levels == ws.levels
        v, f = g.dump_states()
        assert np.array_equal(v[:n], ov), name
        bad = np.nonzero(f[:n] != of)[0]
        assert len(bad) == 0, (name, bad[:8])
    assert 600_000 < len(want) < 700_000   # levels 3-6 saturate (~0.6M)
    g.close()


def _engine_edges(g, n):
    u, d, t = g.export_edges()
    a = canon_edges(u, d, t)
    return a[a[:, 0] < n] if len(a) else a


def _oracle_edges(o):
    return canon_edges(*o.export_used_by())


@pytest.mark.parametrize("mode", ["prune", "prune_gather", "prune_range"])
def test_configs3_scale20_prune_parity(pkg, gpu_available, mode, monkeypatch):
    """The first wave builds the dependency lists, so "prune" runs the fast path (liveness recorded at
    list build + a bitmap of current nodes); "prune_gather" pins the node-word gathers; "prune_range"
    runs its first batch on the fast path and the later ones (after the first compaction) on gathers."""
    if mode == "prune_gather":
        monkeypatch.setenv("FGI_PRUNE_GATHER", "1")
    scale, ef, seed, sseed, rseed = 20, 16, 0x5EED0024, 0x5EED00C0, 0x5EED1024
    n = 1 << scale
    O.set_threads(THREADS)
    s, d = O.gen_rmat(scale, ef, seed)
    tags = O.gen_tags(s, d, seed, 50, sseed)
    o = O.Oracle(n)
    o.load_graph(O.version_of(seed, np.arange(n)), None, s, d, tags)
    roots = O.gen_roots(4096, n, rseed, np.bincount(s, minlength=n))
    roots2 = O.gen_roots(512, n, rseed + 1, np.bincount(s, minlength=n))
    del s, d, tags
    g = pkg.Graph(n)
    g.synth_rmat(scale, ef, seed, 50, sseed)
    # wave 1: invalidated nodes' rows are cleared, entries pointing at them go stale
    st = o.invalidate_slots(roots, threads=THREADS)
    ws = pkg.WaveStats()
    ids = g.invalidate(roots, stats=ws)
    assert np.array_equal(np.sort(ids), np.sort(o.inv_log())) and (ws.v_inv, ws.e_trav) == (st.v_inv, st.e_trav)
    o.clear_log()
    if mode in ("prune", "prune_gather"):
        ps = g.prune()
        oe, ne = o.prune()
        assert ps.new_edges == ne and ps.old_edges >= oe, (ps.old_edges, ps.new_edges, oe, ne)
    else:   # the pruner's batched walk over the registry
        batch = 300_000
        news = 0
        for lo in range(0, g.n_handles, batch):
            ps = g.prune_range(lo, batch)
            oe, ne = o.prune_range(lo, batch)
            assert ps.new_edges == ne, (lo, ps.new_edges, ne)
            news += ne
        assert news > 0
    ge, oe_ = _engine_edges(g, n), _oracle_edges(o)
    assert len(ge) == len(oe_) and np.array_equal(ge, oe_), (len(ge), len(oe_))
    live = ge[:, 2] == O.version_of(seed, ge[:, 1].astype(np.int64))
    assert live.all(), "a pruned row kept a version-mismatched entry"
    # wave 2 after the prune: identical on both sides
    st2 = o.invalidate_slots(roots2, threads=THREADS)
    ws2 = pkg.WaveStats()
    ids2 = g.invalidate(roots2, stats=ws2)
    assert np.array_equal(np.sort(ids2), np.sort(o.inv_log()))
    assert (ws2.v_inv, ws2.e_trav) == (st2.v_inv, st2.e_trav)
    v, f = g.dump_states()
    ov, of = o.dump_states()
    assert np.array_equal(v[:n], ov) and np.array_equal(f[:n], of)
    o.close()
    g.close()


@pytest.fixture(scope="module")
def rmat27(pkg, gpu_available):
    """configs[2]'s graph on one device, its exported edge set on the device for the checks."""
    from closure_check import DeviceEdges
    from stl_fusion_amd import workloads as W
    cfg = W.CONFIGS["rmat27"]
    n = W.n_slots(cfg)
    g = pkg.Graph(n)
    W.build(g, cfg)
    roots = W.roots_for(g, cfg)
    u, d, t = g.export_edges()
    ver = O.version_of(cfg["seed"], np.arange(n, dtype=np.int64))
    edges = DeviceEdges(n, u, d, t, ver)
    m = len(u)
    del u, d, t, ver
    g.snapshot()
    yield g, roots, edges, m
    g.close()


def test_configs2_rmat27_single_gpu_wave(pkg, rmat27):
    g, roots, edges, m = rmat27
    assert len(roots) == 4096 and m > 1_000_000_000   # 1.07G generated, multi-edges removed
    sets = []
    for name, direction in (("auto_first", 0), ("auto", 0), ("push", 1)):
        g.restore()
        g.set_option(pkg.fgi.OPT_DIRECTION, direction)
        ws = pkg.WaveStats()
        ids = g.invalidate(roots, stats=ws)
        assert len(ids) == ws.v_inv
        if name == "auto":
            assert ws.pull_levels > 0, "configs[2]'s whole graph pulls on one device (DESIGN.md §7a)"
        edges.check_wave(ids, roots, ws.e_trav)
        v, f = g.dump_states()
        st = f[:g.n_slots] & 3
        inv = np.zeros(g.n_slots, bool)
        inv[ids] = True
        assert np.array_equal(st == INVALIDATED, inv) and np.all(st[~inv] == CONSISTENT), name
        sets.append(np.sort(ids))
    assert all(np.array_equal(sets[0], x) for x in sets[1:])
    assert 40_000_000 < len(sets[0]) < 43_000_000   # 41.3M
    g.set_option(pkg.fgi.OPT_DIRECTION, 0)


def test_configs2_rmat27_eight_partitions_match_single_engine(pkg, rmat27):
    """configs[2] as the multi-GPU engine runs it: 8 vertex-range partitions of the R-MAT 27 graph
    (each generated by row range, fgi_part_synth_rmat), driven in one process by run_part_wave's
    level loop on 8 host threads (fgi_part_local_invalidate: device copies for the collectives),
    against the single engine on the same graph and roots — the same invalidated set, V_inv, E_trav
    and final node words, slot by slot."""
    from stl_fusion_amd import workloads as W
    g, roots, edges, m = rmat27
    cfg = W.CONFIGS["rmat27"]
    n = W.n_slots(cfg)
    g.restore()
    g.set_option(pkg.fgi.OPT_DIRECTION, 0)
    ws = pkg.WaveStats()
    ids1 = np.sort(g.invalidate(roots, stats=ws))
    v1, f1 = g.dump_states()
    P = 8
    block = -(-n // P)
    import json
    import torch
    free0 = torch.cuda.mem_get_info()[0]
    gs = [pkg.Graph(block, rank=r, world=P) for r in range(P)]
    pkg.fgi.part_init_local(gs, n)
    for x in gs:
        x.part_synth_rmat(cfg["scale"], cfg["edge_factor"], cfg["seed"])
    torch.cuda.synchronize()
    per_rank_gb = (free0 - torch.cuda.mem_get_info()[0]) / P / 2**30   # resident after the build
    if os.environ.get("FGI_PART_MEM_OUT"):
        json.dump({"workload": "configs[2] R-MAT 27, 8 partitions", "resident_gib_per_rank": per_rank_gb},
                  open(os.environ["FGI_PART_MEM_OUT"], "w"))
    assert per_rank_gb < 16, per_rank_gb
    assert sum(x.degrees()[1] for x in gs) == m   # the rows of the 8 ranks are the whole edge set
    stats = pkg.fgi.part_local_invalidate(gs, roots)
    ids = np.sort(np.concatenate([x.part_export_ids() for x in gs]))
    assert np.array_equal(ids, ids1), (len(ids), len(ids1))
    assert sum(s.v_inv for s in stats) == ws.v_inv and sum(s.e_trav for s in stats) == ws.e_trav
    assert sum(s.pull_levels for s in stats) > 0 and sum(s.remote_msgs for s in stats) > 0
    for r, x in enumerate(gs):
        v, f = x.dump_states()
        lo, hi = r * block, min(n, (r + 1) * block)
        assert np.array_equal(v[:hi - lo], v1[lo:hi]) and np.array_equal(f[:hi - lo], f1[lo:hi]), r
    for x in gs:
        x.close()
