"""Multi-GPU partition path, exercised on one GPU: P partitions of one R-MAT graph run in one
process (fgi_part_init_local). fgi_part_local_invalidate runs the RCCL path's own level loop
(run_part_wave) on every rank in its own host thread; only the collectives are device copies
instead of RCCL. Results must be exactly the oracle's invalidated set and final node states,
including consecutive pull levels (direction 2: the pull->pull frontier-bitmap copy)."""
import numpy as np
import pytest

import fgo as O

pytestmark = pytest.mark.gpu


FRONT = {"auto": 0, "full": 1, "delta": 2}   # FGI_OPT_FRONT_EXCHANGE: the pull levels' bitmap exchange


@pytest.mark.parametrize("front", ["full", "delta"])
@pytest.mark.parametrize("direction", [0, 1, 2])      # auto, push only, pull only
@pytest.mark.parametrize("P", [2, 3, 4, 8])
@pytest.mark.parametrize("stale", [0, 50])
def test_partitioned_wave_matches_oracle(pkg, gpu_available, P, stale, direction, front):
    if direction == 1 and front == "delta":
        pytest.skip("push-only waves exchange no frontier bitmap")
    scale, ef, seed, sseed = 12, 16, 0x5EED0027, 0x5EED00C0
    n = 1 << scale
    block = -(-n // P)
    gs = [pkg.Graph(block, rank=r, world=P) for r in range(P)]
    pkg.fgi.part_init_local(gs, n)
    for g in gs:
        g.part_synth_rmat(scale, ef, seed, stale, sseed)
        g.set_option(2, direction)
        g.set_option(pkg.fgi.OPT_FRONT_EXCHANGE, FRONT[front])
    s, d = O.gen_rmat(scale, ef, seed)
    o = O.Oracle(n)
    o.load_graph(O.version_of(seed, np.arange(n)), None, s, d, O.gen_tags(s, d, seed, stale, sseed))
    roots = O.gen_roots(48, n, 0x5EED1027, np.bincount(s, minlength=n))
    imm = (np.arange(len(roots)) % 5 == 0).astype(np.uint8)
    st = o.invalidate_slots(roots, imm)
    stats = pkg.fgi.part_local_invalidate(gs, roots, imm)
    ids = np.concatenate([g.part_export_ids() for g in gs])
    assert len(np.unique(ids)) == len(ids)
    assert np.array_equal(np.sort(ids), np.sort(o.inv_log()))
    assert sum(x.v_inv for x in stats) == st.v_inv
    assert sum(x.e_trav for x in stats) == st.e_trav
    if direction == 1:
        assert sum(x.remote_msgs for x in stats) > 0
    if direction == 2 and block % 32 == 0:
        assert all(x.pull_levels == x.levels for x in stats)
        full, delta, _ = gs[0].part_front_stats()
        assert (delta == 0) if front == "full" else (full == 0 and delta > 0)
    # final states, gathered from the owners
    ov, of = o.dump_states()
    for r, g in enumerate(gs):
        v, f = g.dump_states()
        lo, hi = r * block, min(n, (r + 1) * block)
        assert np.array_equal(v[:hi - lo], ov[lo:hi])
        assert np.array_equal(f[:hi - lo], of[lo:hi])
    # a second wave with other roots continues from the partitioned state
    roots2 = O.gen_roots(16, n, 99, np.bincount(s, minlength=n))
    o.clear_log()
    o.invalidate_slots(roots2)
    pkg.fgi.part_local_invalidate(gs, roots2)
    ids2 = np.concatenate([g.part_export_ids() for g in gs])
    assert np.array_equal(np.sort(ids2), np.sort(o.inv_log()))


def test_partition_owns_rows_of_its_slots(pkg, gpu_available):
    scale, ef, seed, P = 10, 8, 7, 4
    n = 1 << scale
    block = n // P
    gs = [pkg.Graph(block, rank=r, world=P) for r in range(P)]
    pkg.fgi.part_init_local(gs, n)
    rows = []
    for r, g in enumerate(gs):
        g.part_synth_rmat(scale, ef, seed)
        u, dd, t = g.export_edges()
        rows.append(np.stack([u.astype(np.uint64) + r * block, dd, t], 1))
    got = np.concatenate(rows)
    s, d = O.gen_rmat(scale, ef, seed)
    want = np.stack([s.astype(np.uint64), d, O.gen_tags(s, d, seed)], 1)
    key = lambda a: a[np.lexsort((a[:, 2], a[:, 1], a[:, 0]))]
    assert np.array_equal(key(got), key(want))


def test_single_engine_calls_refuse_a_partitioned_graph(pkg, gpu_available):
    """A partition's rows hold global dependant ids: the single-device wave and mutation entry
    points must refuse it (FGI_ESTATE) instead of indexing past the partition's arrays."""
    scale, ef, seed, P = 10, 8, 7, 2
    n = 1 << scale
    gs = [pkg.Graph(n // P, rank=r, world=P) for r in range(P)]
    pkg.fgi.part_init_local(gs, n)
    for g in gs:
        g.part_synth_rmat(scale, ef, seed)
    g = gs[1]
    calls = [lambda: g.invalidate(np.array([1], np.uint32)), lambda: g.invalidate_all(), lambda: g.prune(),
             lambda: g.begin_compute(np.array([1], np.uint32), np.array([3], np.uint64)),
             lambda: g.add_used(np.array([1], np.uint32), np.array([2], np.uint32)),
             lambda: g.set_output(np.array([1], np.uint32))]
    for c in calls:
        with pytest.raises(pkg.FgiError) as e:
            c()
        assert e.value.status == pkg.fgi.ESTATE
    # the partitioned wave still works afterwards
    s, d = O.gen_rmat(scale, ef, seed)
    o = O.Oracle(n)
    o.load_graph(O.version_of(seed, np.arange(n)), None, s, d, O.gen_tags(s, d, seed))
    roots = O.gen_roots(8, n, 5, np.bincount(s, minlength=n))
    o.invalidate_slots(roots)
    pkg.fgi.part_local_invalidate(gs, roots)
    ids = np.concatenate([x.part_export_ids() for x in gs])
    assert np.array_equal(np.sort(ids), np.sort(o.inv_log()))


@pytest.mark.parametrize("front", ["auto", "delta"])
@pytest.mark.parametrize("stale", [0, 50])
def test_partitioned_8_ranks_at_scale_matches_single_engine(pkg, gpu_available, stale, front):
    """The 8-rank level loop (run_part_wave: remote targets forwarded, frontier bitmaps all-gathered,
    direction and termination from summed counters) at a size where every level does real work: R-MAT
    22 (4.2M slots, 67M edges) in 8 in-process partitions against the single-device engine on the same
    graph and 4,096 roots — the same invalidated set, V_inv, E_trav and final node words — then a
    second wave from the partitioned state."""
    scale, ef, seed, sseed, P = 22, 16, 0x5EED0027, 0x5EED00C0, 8
    n = 1 << scale
    block = -(-n // P)
    one = pkg.Graph(n)
    one.synth_rmat(scale, ef, seed, stale, sseed)
    deg, _ = one.degrees()
    roots = O.gen_roots(4096, n, 0x5EED1027, deg[:n])
    roots2 = O.gen_roots(512, n, 0x5EED2027, deg[:n])
    ws = pkg.WaveStats()
    ids1 = np.sort(one.invalidate(roots, stats=ws))
    v1, f1 = one.dump_states()
    ids1b = np.sort(one.invalidate(roots2))
    v1b, f1b = one.dump_states()
    one.close()
    gs = [pkg.Graph(block, rank=r, world=P) for r in range(P)]
    pkg.fgi.part_init_local(gs, n)
    for g in gs:
        g.part_synth_rmat(scale, ef, seed, stale, sseed)
        g.set_option(pkg.fgi.OPT_FRONT_EXCHANGE, FRONT[front])
    stats = pkg.fgi.part_local_invalidate(gs, roots)
    ids = np.sort(np.concatenate([g.part_export_ids() for g in gs]))
    assert np.array_equal(ids, ids1), (len(ids), len(ids1))
    assert sum(x.v_inv for x in stats) == ws.v_inv and sum(x.e_trav for x in stats) == ws.e_trav
    assert sum(x.pull_levels for x in stats) > 0 and sum(x.remote_msgs for x in stats) > 0
    # push levels decide from the counts all-gather's bound, pull levels and an all-remote tail from
    # the all-reduce: the loop runs exactly the cascade's depth (no empty level)
    assert all(x.levels == ws.levels for x in stats), ([x.levels for x in stats], ws.levels)
    for r, g in enumerate(gs):
        v, f = g.dump_states()
        lo, hi = r * block, min(n, (r + 1) * block)
        assert np.array_equal(v[:hi - lo], v1[lo:hi]) and np.array_equal(f[:hi - lo], f1[lo:hi]), r
    pkg.fgi.part_local_invalidate(gs, roots2)
    ids = np.sort(np.concatenate([g.part_export_ids() for g in gs]))
    assert np.array_equal(ids, ids1b)
    for r, g in enumerate(gs):
        v, f = g.dump_states()
        lo, hi = r * block, min(n, (r + 1) * block)
        assert np.array_equal(v[:hi - lo], v1b[lo:hi]) and np.array_equal(f[:hi - lo], f1b[lo:hi]), r
    for g in gs:
        g.close()
