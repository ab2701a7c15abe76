"""Pull levels answering cold probes from the nonzero-word summary (FGI_OPT_PROBE_SUMMARY):
while few invalidated-bitmap words can be nonzero, k_collect builds one bit per 64-bit word and a pull
level reads a cold head's or tail entry's bitmap word only when its summary bit is set. The default
builds it only for bitmaps larger than an XCD's L2 (configs[2]); here it is forced on small graphs
(option 0) with the hot heads capped (most probes cold), and every wave must equal the oracle's —
invalidated set, V_inv, E_trav on a fresh graph, node words — and the same graph with the summary off."""
import numpy as np
import pytest

import fgo as O

pytestmark = [pytest.mark.gpu, pytest.mark.usefixtures("variants")]


def _pair(pkg, scale, ef, seed, stale, sseed=0x5EED00C0):
    n = 1 << scale
    g = pkg.Graph(n)
    g.synth_rmat(scale, ef, seed, stale, sseed)
    s, d = O.gen_rmat(scale, ef, seed)
    o = O.Oracle(n)
    o.load_graph(O.version_of(seed, np.arange(n)), None, s, d, O.gen_tags(s, d, seed, stale, sseed))
    return g, o, s, n


@pytest.mark.parametrize("direction", [0, 2])
@pytest.mark.parametrize("hot", [0, 256])
@pytest.mark.parametrize("stale", [0, 30])
def test_summary_waves_match_oracle(pkg, gpu_available, direction, hot, stale):
    g, o, s, n = _pair(pkg, 16, 16, 0x5EED0016, stale)
    g.set_option(pkg.fgi.OPT_DIRECTION, direction)
    g.set_option(pkg.fgi.OPT_HOT_HEADS, hot)
    deg = np.bincount(s, minlength=n)
    g.snapshot()
    o.snapshot()
    results = {}
    for mode in (0, -1, 0):   # summary forced, off, forced again (lists and snapshots reused)
        g.restore()
        o.restore()
        g.set_option(pkg.fgi.OPT_PROBE_SUMMARY, mode)
        for k, (nr, rs) in enumerate(((16, 5), (64, 6), (8, 7))):
            roots = O.gen_roots(nr, n, rs, deg)
            o.clear_log()
            st = o.invalidate_slots(roots)
            ws = pkg.WaveStats()
            ids = g.invalidate(roots, stats=ws)
            assert np.array_equal(np.sort(ids), np.sort(o.inv_log())), (mode, k, len(ids), len(o.inv_log()))
            assert ws.v_inv == st.v_inv, (mode, k)
            if k == 0:
                assert ws.e_trav == st.e_trav, (mode, k)
            results.setdefault(k, []).append(np.sort(ids))
        v, f = g.dump_states()
        ov, of = o.dump_states()
        assert np.array_equal(v[:n], ov) and np.array_equal(f[:n], of), mode
    for k, runs in results.items():
        assert all(np.array_equal(r, runs[0]) for r in runs), k
    o.close()
    g.close()


def test_summary_after_mutations(pkg, gpu_available):
    """The summary is rebuilt per pull level from the live bitmap: a wave after recomputes (new
    versions, new edges) and a partial earlier wave still matches."""
    g, o, s, n = _pair(pkg, 14, 16, 0x5EED0014, 20)
    g.set_option(pkg.fgi.OPT_PROBE_SUMMARY, 0)
    g.set_option(pkg.fgi.OPT_HOT_HEADS, 256)
    deg = np.bincount(s, minlength=n)
    r1 = O.gen_roots(4, n, 11, deg)
    ids = g.invalidate(r1)
    o.invalidate_slots(r1)
    assert np.array_equal(np.sort(ids), np.sort(o.inv_log()))
    # recompute what the wave invalidated: new versions, then each re-captures two dependencies
    inv = np.sort(ids)[:200].astype(np.uint32)
    ver = (np.arange(len(inv), dtype=np.uint64) * 2 + (1 << 50) + 1)
    g.begin_compute(inv, ver)
    o.begin_compute_slots(inv, ver)
    rng = np.random.default_rng(3)
    live = np.setdiff1d(np.arange(n, dtype=np.uint32), np.sort(ids))
    used = rng.choice(live, len(inv)).astype(np.uint32)
    codes = g.add_used(inv, used)
    assert np.array_equal(codes, o.add_used_slots(inv, used))
    g.set_output(inv)
    o.set_output_slots(inv)
    o.clear_log()
    r2 = O.gen_roots(32, n, 12, deg)
    st = o.invalidate_slots(r2)
    ws = pkg.WaveStats()
    ids2 = g.invalidate(r2, stats=ws)
    assert np.array_equal(np.sort(ids2), np.sort(o.inv_log()))
    assert ws.v_inv == st.v_inv
    v, f = g.dump_states()
    ov, of = o.dump_states()
    assert np.array_equal(v[:n], ov) and np.array_equal(f[:n], of)
    o.close()
    g.close()


@pytest.mark.parametrize("P", [2, 4])
def test_summary_on_partitions(pkg, gpu_available, P):
    """A partition's pull levels probe the all-gathered bitmap through the same summary (built over
    front_global on each rank): planned and host-driven waves match the oracle with it forced on."""
    scale, ef, seed, stale, sseed = 14, 16, 0x5EED0027, 20, 0x5EED00C0
    n = 1 << scale
    block = -(-n // P)
    gs = [pkg.Graph(block, rank=r, world=P) for r in range(P)]
    pkg.fgi.part_init_local(gs, n)
    for g in gs:
        g.part_synth_rmat(scale, ef, seed, stale, sseed)
        g.set_option(pkg.fgi.OPT_PROBE_SUMMARY, 0)
        g.set_option(pkg.fgi.OPT_HOT_HEADS, 256)
        g.set_option(pkg.fgi.OPT_DIRECTION, 2)
        g.snapshot()
    s, d = O.gen_rmat(scale, ef, seed)
    o = O.Oracle(n)
    o.load_graph(O.version_of(seed, np.arange(n)), None, s, d, O.gen_tags(s, d, seed, stale, sseed))
    o.snapshot()
    roots = O.gen_roots(24, n, 9, np.bincount(s, minlength=n))
    for rep in range(3):   # learning wave, then planned ones
        for g in gs:
            g.restore()
        o.restore()
        o.clear_log()
        st = o.invalidate_slots(roots)
        stats = pkg.fgi.part_local_invalidate(gs, roots)
        ids = np.concatenate([g.part_export_ids() for g in gs])
        assert np.array_equal(np.sort(ids), np.sort(o.inv_log())), rep
        assert sum(x.v_inv for x in stats) == st.v_inv
        assert sum(x.e_trav for x in stats) == st.e_trav
        assert all(x.pull_levels >= 1 for x in stats)
    o.close()
