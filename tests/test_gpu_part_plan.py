"""Planned partitioned waves (FGI_OPT_PART_PLAN): after a wave whose levels the host
decided one by one (an all-reduce and a host synchronisation per level), the next waves follow its
directions with fixed-size, stream-ordered collectives — the full invalidated-bitmap all-gather before
a pull level, buckets of forwarded targets after a push level — and wait for the device once, at a
closing all-reduce (twice with remote ranks: the start's all-reduce too). Ids that do not fit a
bucket wait for the next push level, and push levels follow the plan while any are left.

Run on one GPU with P partitions in one process (LocalComm: the same level sequence as RCCL; its
stream-ordered exchanges order the ranks' streams with events, no host wait). Every wave must match
the oracle exactly: the invalidated set, V_inv, E_trav on a fresh graph, every node word.
"""
import numpy as np
import pytest

import fgo as O

pytestmark = pytest.mark.gpu


def _build(pkg, P, scale, ef, seed, stale, sseed=0x5EED00C0):
    n = 1 << scale
    block = -(-n // P)
    gs = [pkg.Graph(block, rank=r, world=P) for r in range(P)]
    pkg.fgi.part_init_local(gs, n)
    for g in gs:
        g.part_synth_rmat(scale, ef, seed, stale, sseed)
    s, d = O.gen_rmat(scale, ef, seed)
    o = O.Oracle(n)
    o.load_graph(O.version_of(seed, np.arange(n)), None, s, d, O.gen_tags(s, d, seed, stale, sseed))
    return gs, o, s, n, block


def _check(pkg, gs, o, n, block, roots, want_etrav=True):
    o.clear_log()
    st = o.invalidate_slots(roots)
    stats = pkg.fgi.part_local_invalidate(gs, roots)
    ids = np.concatenate([g.part_export_ids() for g in gs])
    assert len(np.unique(ids)) == len(ids)
    assert np.array_equal(np.sort(ids), np.sort(o.inv_log())), (len(ids), len(o.inv_log()))
    assert sum(x.v_inv for x in stats) == st.v_inv
    if want_etrav:
        assert sum(x.e_trav for x in stats) == st.e_trav
    ov, of = o.dump_states()
    for r, g in enumerate(gs):
        v, f = g.dump_states()
        lo, hi = r * block, min(n, (r + 1) * block)
        assert np.array_equal(v[:hi - lo], ov[lo:hi]) and np.array_equal(f[:hi - lo], of[lo:hi]), r
    return stats


@pytest.mark.parametrize("direction", [0, 1, 2])
@pytest.mark.parametrize("P", [2, 3, 8])
@pytest.mark.parametrize("stale", [0, 50])
def test_planned_waves_match_oracle(pkg, gpu_available, P, stale, direction):
    gs, o, s, n, block = _build(pkg, P, 16, 16, 0x5EED0027, stale)
    for g in gs:
        g.set_option(pkg.fgi.OPT_DIRECTION, direction)
        g.snapshot()
    o.snapshot()
    roots = O.gen_roots(256, n, 0x5EED1027, np.bincount(s, minlength=n))
    learnt = _check(pkg, gs, o, n, block, roots)            # the host-driven levels (learns the plan)
    assert all(x.host_syncs == 0 or x.host_syncs > 2 for x in learnt)
    for rep in range(2):
        for g in gs:
            g.restore()
        o.restore()
        planned = _check(pkg, gs, o, n, block, roots)
        assert all(x.host_syncs == 2 for x in planned), [x.host_syncs for x in planned]
        assert sum(x.levels for x in planned) >= 1
    # other roots on the planned graph state (no restore): a plan learnt from another wave is only a
    # cost choice
    roots2 = O.gen_roots(64, n, 77, np.bincount(s, minlength=n))
    _check(pkg, gs, o, n, block, roots2, want_etrav=False)
    o.close()


@pytest.mark.parametrize("bucket,scale", [(2, 13), (2, 15), (3, 13), (17, 13), (1000, 13)])
def test_planned_waves_with_small_buckets(pkg, gpu_available, bucket, scale):
    """Buckets of `bucket` words per peer (2, the smallest the clamp accepts: a count and one id):
    most forwarded ids wait for later push levels (which the planned wave appends while any are
    left); the wave is still exactly the oracle's."""
    P = 4
    gs, o, s, n, block = _build(pkg, P, scale, 16, 0x5EED0027, 30)
    for g in gs:
        g.snapshot()
    o.snapshot()
    roots = O.gen_roots(200, n, 0x5EED1027, np.bincount(s, minlength=n))
    _check(pkg, gs, o, n, block, roots)
    for g in gs:
        g.set_option(pkg.fgi.OPT_PART_BUCKET, bucket)
        g.restore()
    o.restore()
    planned = _check(pkg, gs, o, n, block, roots)
    assert all(x.remote_msgs > 0 for x in planned)
    o.close()


def test_plan_off_keeps_the_host_driven_levels(pkg, gpu_available):
    P = 3
    gs, o, s, n, block = _build(pkg, P, 14, 16, 0x5EED0027, 0)
    for g in gs:
        g.set_option(pkg.fgi.OPT_PART_PLAN, 0)
        g.snapshot()
    o.snapshot()
    roots = O.gen_roots(128, n, 0x5EED1027, np.bincount(s, minlength=n))
    for rep in range(2):
        for g in gs:
            g.restore()
        o.restore()
        st = _check(pkg, gs, o, n, block, roots)
        assert all(x.host_syncs > 2 for x in st)
    o.close()
