"""The two configurations round 3 left unchecked at their own size.

configs[4]  the streaming mix at BASELINE.json's size: 10,000 hubs x 1,000 leaves (10,010,000 slots),
            1% delayed leaves, 100-hub waves. A priming wave, then rounds of one fgi_run_batch each
            (delay timers with immediately = true -> begin_compute / set_output on the previous
            round's hubs -> begin_compute / add_used / set_output on their 100,000 leaves -> a wave on
            100 new hubs), exactly as bench_configs.py submits them. The oracle applies the same calls
            one by one (Computed.cs:141-160 TrySetOutput, 347-385 AddUsed / AddUsedBy,
            ComputedRegistry.cs:72-105 Register with displacement, Computed.cs:162-230 Invalidate).
            Every round: every cascade's ids in step order and every slot's final node word. At this
            size a cascade's leaf level (100,000 edges) is split into multi-fine chunks over the
            cascade grid, and the final collect owns more bitmap words per block than it stages in
            LDS — the paths the small mixes of test_gpu_batch.py never reach.
configs[3]  R-MAT 24 with 50% stale edges at full size (263.4 M entries). PruneUsedBy (Computed.cs:400-419)
            on every registered Consistent node, reached by the pruner's walk (ComputedGraphPruner.cs:
            79-94), keeps an entry iff the dependant's current node exists with the entry's version.
            Checked exactly over the exported edge sets, twice: bench_configs.py's prune (restored
            graph, the fast path) and a prune after a wave (the gather path); the kept entries are
            exactly the live pre-prune ones and PruneStats.new_edges is their count. Then a wave on the
            pruned graph against the independent least closure (tests/closure_check.py).
"""
import numpy as np
import pytest

import fgo as O
from harness import CONSISTENT, INVALIDATED, assert_states_equal

pytestmark = pytest.mark.gpu


def _oracle_round(o, mix, timers, hubs, leaves, vh, vl, roots):
    """The round's calls on the oracle, one by one; returns (timer cascade ids, wave ids)."""
    o.clear_log()
    if len(timers):
        o.invalidate_slots(timers, np.ones(len(timers), np.uint8))
    t_ids = o.inv_log()
    o.begin_compute_slots(hubs, vh)
    assert o.set_output_slots(hubs) == len(hubs)
    o.begin_compute_slots(leaves, vl, mix.has_delay[leaves])
    codes = o.add_used_slots(leaves, mix.hub_of(leaves))
    assert np.all(codes == 0)   # FGO_USED_ADDED
    assert o.set_output_slots(leaves) == len(leaves)
    # nothing above cascades: the recomputed nodes were all invalidated (wave or timer) before
    assert len(o.inv_log()) == len(t_ids)
    o.clear_log()
    o.invalidate_slots(roots)
    return t_ids, o.inv_log()


def test_configs4_full_size_batches_match_oracle(pkg, gpu_available):
    from stl_fusion_amd import workloads as W
    p = W.STREAM
    mix = W.StreamMix(p["hubs"], p["leaves_per_hub"], p["hubs_per_round"], p["delay_pct"], p["seed"])
    n = mix.n
    assert n == 10_010_000
    used, dep, tag = mix.initial_edges()
    flags = mix.state_flags()
    # as bench_configs.py: every slot registered, 10 M leaf -> hub entries, room for the churn
    g = pkg.Graph(n, edge_capacity=3 * (n - p["hubs"]))
    g.register_nodes(np.arange(n, dtype=np.uint32), mix.version, flags)
    g.load_edges(used, dep, tag)
    O.set_threads(16)
    o = O.Oracle(n)
    o.load_graph(mix.version, flags, used, dep, tag)
    del used, dep, tag
    prev = mix.roots(0)
    ids = g.invalidate(prev)
    o.invalidate_slots(prev)
    assert np.array_equal(np.sort(ids), np.sort(o.inv_log()))
    n_delayed = 0
    for r in range(1, 6):
        timers, hs, ls = mix.plan(prev)
        vh = mix.new_versions(hs).copy()
        vl = mix.new_versions(ls).copy()
        roots = mix.roots(r)
        steps = []
        if len(timers):
            steps.append(("invalidate", timers, np.ones(len(timers), np.uint8)))
        steps += [("begin_compute", hs, vh), ("set_output", hs), ("begin_compute", ls, vl, mix.has_delay[ls]),
                  ("add_used", ls, mix.hub_of(ls)), ("set_output", ls), ("invalidate", roots)]
        st = pkg.fgi.BatchStats()
        ids, outs = g.run_batch(steps, stats=st)
        t_ids, w_ids = _oracle_round(o, mix, timers, hs, ls, vh, vl, roots)
        assert len(ls) == 100_000 and len(w_ids) > 90_000, (len(ls), len(w_ids))
        assert np.all(outs[-3] == pkg.fgi.USED_ADDED), f"round {r}: add_used results"
        assert np.all(outs[-2] == 1) and np.all(outs[-5] == 1), f"round {r}: set_output results"
        # cascades in step order: the timers' immediate roots, the (empty) displacement and
        # InvalidateOnSetOutput cascades, the hub wave; each cascade's ids ascending
        want = np.concatenate([np.sort(t_ids), np.sort(w_ids)]).astype(np.uint32)
        assert len(ids) == len(want), f"round {r}: {len(ids)} ids, oracle {len(want)}"
        assert np.array_equal(ids, want), f"round {r}: ids differ at {np.nonzero(ids != want)[0][:8]}"
        assert st.v_inv == len(want)
        # the wave is the root hubs plus their undelayed leaves; the delayed ones only start a timer
        ch = mix.children(roots)
        assert np.array_equal(np.sort(w_ids), np.sort(np.concatenate([roots, ch[mix.has_delay[ch] == 0]])))
        n_delayed += len(timers)
        assert_states_equal(g, o, n)
        prev = roots
    assert n_delayed > 0, "no delay timer fired"
    g.close()
    o.close()


def _sorted_keys(u, d):
    """(used << 32 | dependant) of every entry, sorted on the device (slots < 2^24: no sign issue)."""
    import torch
    k = (torch.from_numpy(u.astype(np.int64)).cuda() << 32) | torch.from_numpy(d.astype(np.int64)).cuda()
    return torch.sort(k).values


def _live_keys(g, n, v, st):
    """The exported entries PruneUsedBy keeps (Computed.cs:400-419): rows of Consistent nodes (the
    export holds the rows of current nodes), dependant registered (not Invalidated) at the entry's tag;
    as sorted (used << 32 | dependant) keys, and the export's size."""
    u, d, t = g.export_edges()
    keep = (u < n) & (d < n)
    keep[keep] &= st[u[keep]] == CONSISTENT
    keep[keep] &= st[d[keep]] != INVALIDATED
    keep[keep] &= t[keep] == v[d[keep]]
    return _sorted_keys(u[keep], d[keep]), len(u)


def _check_prune(g, n, want, old_export):
    import torch
    ps = g.prune()
    assert ps.new_edges == len(want), (ps.new_edges, len(want))
    assert ps.new_edges < old_export, (ps.new_edges, old_export)
    v, _ = g.dump_states()
    u1, d1, t1 = g.export_edges()
    assert len(u1) == len(want)
    assert np.all(t1 == v[:n][d1]), "a kept entry's tag differs from its dependant's version"
    assert torch.equal(_sorted_keys(u1, d1), want), "the kept entries differ from the live pre-prune entries"
    return u1, d1, t1


def test_configs3_full_size_prune_keeps_exactly_the_live_entries(pkg, gpu_available):
    """(a) bench_configs.py's flow: a wave (it builds the pull lists), fgi_restore, fgi_prune on the fast
    path — every node Consistent, so exactly the entries whose tag is their dependant's version stay
    (131.7 M of 263.4 M); (b) a wave, then a second prune (the gather path, after (a)'s compaction) —
    the rows of invalidated nodes are dropped and entries pointing at them too; (c) a third wave on the
    twice-pruned graph against the independent least closure over the kept entries."""
    from closure_check import DeviceEdges
    from stl_fusion_amd import workloads as W
    cfg = W.CONFIGS["rmat24_churn"]
    n = W.n_slots(cfg)
    g = pkg.Graph(n)
    W.build(g, cfg)
    roots = W.roots_for(g, cfg)
    deg, _ = g.degrees()
    roots2 = O.gen_roots(4096, n, cfg["roots_seed"] + 1, deg[:n])
    g.snapshot()
    ws = pkg.WaveStats()
    g.invalidate(roots, stats=ws)
    assert ws.v_inv > 5_000_000
    g.restore()
    # (a)
    v, f = g.dump_states()
    v, st = v[:n], f[:n] & 3
    assert np.all(st == CONSISTENT)
    want, m0 = _live_keys(g, n, v, st)
    assert m0 == 263_432_932 and 0.49 < len(want) / m0 < 0.51, (m0, len(want))
    _check_prune(g, n, want, m0)
    del want
    # (b)
    g.snapshot()
    ws = pkg.WaveStats()
    ids = g.invalidate(roots, stats=ws)
    v, f = g.dump_states()
    v, st = v[:n], f[:n] & 3
    want, m1 = _live_keys(g, n, v, st)
    u1, d1, t1 = _check_prune(g, n, want, m1 + 1)
    del want
    # (c) the pruned rows hold only entries of Consistent nodes to registered dependants at their
    # versions, so the least closure over them from the roots still Consistent is the wave exactly
    edges = DeviceEdges(n, u1, d1, t1, v)
    del u1, d1, t1
    fresh = roots2[st[roots2] == CONSISTENT]
    ws2 = pkg.WaveStats()
    ids2 = g.invalidate(roots2, stats=ws2)
    inv1 = np.zeros(n, bool)
    inv1[ids] = True
    assert not inv1[ids2].any(), "an already invalidated node was invalidated again"
    edges.check_wave(ids2, fresh, ws2.e_trav)
    _, f2 = g.dump_states()
    inv2 = np.zeros(n, bool)
    inv2[ids2] = True
    assert np.array_equal((f2[:n] & 3) == INVALIDATED, inv1 | inv2)
    g.close()
