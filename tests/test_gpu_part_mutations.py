"""The registry's mutations on a partitioned graph.

P ranks of an in-process group on one GPU (LocalComm: the RCCL path's own calls, only the collectives
are device copies inside the group). Every batch goes to every rank (fgi_part_local_run_batch): each
rank applies the items of its own slots, the cascades run as partitioned waves, and the pair state of an
add_used crosses ranks through all-reduces. The oracle applies the same calls one by one on the whole
graph (Computed.cs:141-160 TrySetOutput, 347-385 AddUsed / AddUsedBy, ComputedRegistry.cs:72-105
Register with displacement, Computed.cs:162-230 Invalidate, 400-419 PruneUsedBy). Checked after every
batch: the invalidated slots (as a multiset: a slot can fall in two cascades of one batch), the
add_used result codes, the set_output flags, and every slot's node word on its owner. After the churn a
partitioned prune must keep exactly the oracle's entries, and a wave on the pruned graph must match.
"""
import numpy as np
import pytest

import fgo as O
from harness import COMPUTING, CONSISTENT, canon_edges, random_states

pytestmark = pytest.mark.gpu


def _group(pkg, P, n, n_detached=256):
    block = -(-n // P)
    gs = [pkg.Graph(block, n_detached=n_detached, rank=r, world=P) for r in range(P)]
    pkg.fgi.part_init_local(gs, n)
    return gs, block


def _check_states(gs, o, n, block):
    ov, of = o.dump_states()
    for r, g in enumerate(gs):
        v, f = g.dump_states()
        lo, hi = r * block, min(n, (r + 1) * block)
        assert np.array_equal(v[:hi - lo], ov[lo:hi]), f"rank {r}: versions differ"
        bad = np.nonzero(f[:hi - lo] != of[lo:hi])[0]
        assert len(bad) == 0, f"rank {r}: flags differ at {bad[:8] + lo}: {f[bad[:8]]} vs {of[lo + bad[:8]]}"


def _part_edges(gs, block):
    rows = []
    for r, g in enumerate(gs):
        u, d, t = g.export_edges()
        keep = u < block
        rows.append(canon_edges(u[keep].astype(np.uint64) + np.uint64(r * block), d[keep], t[keep]))
    a = np.concatenate(rows) if rows else np.zeros((0, 3), np.uint64)
    return canon_edges(*a.T) if len(a) else a


def _oracle_batch(o, steps):
    """The batch's calls on the oracle, one by one: (invalidated slots, per-step outputs)."""
    o.clear_log()
    outs = []
    for sp in steps:
        if sp[0] == "invalidate":
            o.invalidate_slots(sp[1], sp[2] if len(sp) > 2 else None)
            outs.append(None)
        elif sp[0] == "begin_compute":
            o.begin_compute_slots(sp[1], sp[2], sp[3] if len(sp) > 3 else None)
            outs.append(None)
        elif sp[0] == "add_used":
            outs.append(o.add_used_slots(sp[1], sp[2]))
        else:
            outs.append(o.set_output_slots(sp[1]))
    return o.inv_log(), outs


def _run_both(pkg, gs, o, steps, n, block):
    ids, outs, stats = pkg.fgi.part_local_run_batch(gs, steps)
    want, oouts = _oracle_batch(o, steps)
    assert len(ids) == len(want) and np.array_equal(np.sort(ids), np.sort(want)), (len(ids), len(want))
    assert sum(s.v_inv for s in stats) == len(want)
    for k, sp in enumerate(steps):
        if sp[0] == "add_used":
            assert np.array_equal(outs[k], oouts[k]), f"step {k}: add_used codes {outs[k]} vs {oouts[k]}"
        elif sp[0] == "set_output":
            assert int(outs[k].sum()) == oouts[k], f"step {k}: {int(outs[k].sum())} set, oracle {oouts[k]}"
        elif sp[0] == "begin_compute":
            # a detached handle is reported by the slot's owner, in its own handle space
            det = outs[k][outs[k] != pkg.fgi.NONE]
            assert np.all(det >= block), det
    _check_states(gs, o, n, block)
    return ids, outs, stats


@pytest.mark.parametrize("P", [2, 3, 8])
def test_streaming_mix_on_partitions(pkg, gpu_available, P):
    """BASELINE.json configs[4]'s operation schedule at a small size (64 hubs x 40 leaves, 10% delayed
    leaves): delay timers, recompute of the previous round's hubs and their leaves (every leaf depends
    on its hub: the pairs cross ranks), then a wave on new hubs — one batch per round."""
    from stl_fusion_amd import workloads as W
    mix = W.StreamMix(64, 40, 8, 10, 0x5EED00E0)
    n = mix.n
    gs, block = _group(pkg, P, n)
    used, dep, tag = mix.initial_edges()
    flags = mix.state_flags()
    slots = np.arange(n, dtype=np.uint32)
    for g in gs:
        g.part_register_nodes(slots, mix.version, flags)
        g.part_load_edges(used, dep, tag)
    o = O.Oracle(n)
    o.load_graph(mix.version, flags, used, dep, tag)
    prev = mix.roots(0)
    _run_both(pkg, gs, o, [("invalidate", prev)], n, block)
    fired = 0
    for r in range(1, 7):
        timers, hs, ls = mix.plan(prev)
        vh = mix.new_versions(hs).copy()
        vl = mix.new_versions(ls).copy()
        roots = mix.roots(r)
        steps = []
        if len(timers):
            steps.append(("invalidate", timers, np.ones(len(timers), np.uint8)))
        steps += [("begin_compute", hs, vh), ("set_output", hs), ("begin_compute", ls, vl, mix.has_delay[ls]),
                  ("add_used", ls, mix.hub_of(ls)), ("set_output", ls), ("invalidate", roots)]
        ids, outs, _ = _run_both(pkg, gs, o, steps, n, block)
        assert np.all(outs[-3] == pkg.fgi.USED_ADDED)
        ch = mix.children(roots)
        assert len(ids) >= len(roots) + int((mix.has_delay[ch] == 0).sum())
        fired += len(timers)
        prev = roots
    assert fired > 0
    o.close()


def _churn_batch(rng, n, present, next_version):
    """A random batch: invalidations (some immediate), recomputes (displacing Consistent, delayed and
    Computing nodes), add_used pairs whose two ends fall anywhere (Computing / Consistent / Invalidated
    used nodes, non-Computing dependants), set_output on part of the recomputed slots."""
    inv = rng.choice(n, 24, replace=False).astype(np.uint32)
    bc = rng.choice(n, 48, replace=False).astype(np.uint32)
    ver = np.arange(next_version, next_version + 2 * len(bc), 2, dtype=np.uint64)
    hd = (rng.random(len(bc)) < 0.2).astype(np.uint8)
    pool = np.union1d(np.nonzero(present)[0], bc).astype(np.uint32)
    dep = np.concatenate([rng.choice(bc, 96), rng.choice(pool, 32)]).astype(np.uint32)
    use = rng.choice(pool, len(dep)).astype(np.uint32)
    dep = np.concatenate([dep, dep[:8]])   # repeated pairs within the batch: set semantics
    use = np.concatenate([use, use[:8]])
    so = bc[rng.random(len(bc)) < 0.7]
    inv2 = rng.choice(n, 8, replace=False).astype(np.uint32)
    steps = [("invalidate", inv, (rng.random(len(inv)) < 0.5).astype(np.uint8)),
             ("begin_compute", bc, ver, hd),
             ("add_used", dep, use),
             ("set_output", so),
             ("invalidate", inv2)]
    return steps, next_version + 2 * len(bc)


@pytest.mark.parametrize("direction", [0, 2])
@pytest.mark.parametrize("P", [2, 3, 8])
def test_random_churn_then_prune_on_partitions(pkg, gpu_available, P, direction):
    """Mixed node states on an R-MAT 12 graph (20% stale entries), eight random batches, then a
    partitioned prune (prune-after-churn) and a wave on the pruned graph; auto and pull-only levels
    (P = 3's ragged ranges have no pull lists: push). The first batch recomputes a delayed node that
    holds a live entry of an undelayed dependant: the old node is detached, so the wave on the new node
    must not reach the dependant through the pull lists, which named the used node by its slot."""
    scale, ef, seed, sseed = 12, 8, 7, 0x5EED00C0
    n = 1 << scale
    rng = np.random.default_rng(1000 + P)
    versions, flags = random_states(n, rng, seed=seed)
    s, d = O.gen_rmat(scale, ef, seed)
    live = (versions[s] != 0) & ((flags[s] & 3) == CONSISTENT)   # only Consistent nodes hold `_usedBy`
    s, d = s[live], d[live]
    tags = versions[d].astype(np.uint64).copy()
    tags[tags == 0] = 7                                            # an entry of an empty slot: never live
    tags[rng.random(len(s)) < 0.2] += np.uint64(1)                 # 20% stale entries
    gs, block = _group(pkg, P, n)
    present = np.nonzero(versions)[0].astype(np.uint32)
    for g in gs:
        g.part_register_nodes(present, versions[present], flags[present])
        g.part_load_edges(s, d, tags)
    o = O.Oracle(n)
    o.load_graph(versions, flags, s, d, tags)
    _check_states(gs, o, n, block)
    for g in gs:
        g.set_option(pkg.fgi.OPT_DIRECTION, direction)
    st = flags & 3
    ok = ((st[s] == CONSISTENT) & ((flags[s] & 16) != 0) & (versions[s] != 0) & (st[d] == CONSISTENT) &
          ((flags[d] & 16) == 0) & (tags == versions[d]))
    u = int(s[np.nonzero(ok)[0][0]])
    ids, _, _ = _run_both(pkg, gs, o, [("begin_compute", [u], [(1 << 45) | 1], [0]), ("set_output", [u]),
                                       ("invalidate", [u])], n, block)
    assert list(ids) == [u]
    nv = 1 << 40 | 1
    codes = set()
    for b in range(8):
        ov, _ = o.dump_states()
        steps, nv = _churn_batch(rng, n, ov != 0, nv)
        _, outs, _ = _run_both(pkg, gs, o, steps, n, block)
        codes |= set(int(c) for c in outs[2])
    # every AddUsed outcome occurred
    assert codes >= {pkg.fgi.USED_ADDED, pkg.fgi.USED_DROPPED, pkg.fgi.USED_INVALIDATED, pkg.fgi.USED_ESTATE}, codes
    ps = pkg.fgi.part_local_prune(gs)
    oe, ne = o.prune()
    assert sum(p.new_edges for p in ps) == ne, ([p.new_edges for p in ps], ne)
    ge, oe_ = _part_edges(gs, block), canon_edges(*o.export_used_by())
    assert len(ge) == len(oe_) and np.array_equal(ge, oe_), (len(ge), len(oe_))
    _check_states(gs, o, n, block)
    ov, of = o.dump_states()
    live = np.nonzero((of & 3) == CONSISTENT)[0]
    roots = rng.choice(live, 64, replace=False).astype(np.uint32)
    ids, _, stats = _run_both(pkg, gs, o, [("invalidate", roots)], n, block)
    assert len(ids) > 0   # delayed roots only start their delay
    o.close()


@pytest.mark.parametrize("P", [2, 3])
def test_batch_errors_on_partitions(pkg, gpu_available, P):
    """A repeated slot in one begin_compute, or a slot out of range, is refused on every rank with
    nothing applied; the group stays usable."""
    n = 1000
    gs, block = _group(pkg, P, n)
    v = O.version_of(3, np.arange(n, dtype=np.uint64))
    for g in gs:
        g.part_register_nodes(np.arange(n, dtype=np.uint32), v, np.full(n, CONSISTENT, np.uint32))
    with pytest.raises(pkg.fgi.FgiError):
        pkg.fgi.part_local_run_batch(gs, [("begin_compute", [5, 5], [11, 13])])
    with pytest.raises(pkg.fgi.FgiError):
        pkg.fgi.part_local_run_batch(gs, [("invalidate", [n])])
    o = O.Oracle(n)
    o.load_graph(v, np.full(n, CONSISTENT, np.uint32), np.zeros(0, np.uint32), np.zeros(0, np.uint32),
                 np.zeros(0, np.uint64))
    _run_both(pkg, gs, o, [("begin_compute", [1, 999], [11, 13]), ("set_output", [1]), ("invalidate", [1, 2])],
              n, block)
    _, f = gs[-1].dump_states()
    assert f[999 - (P - 1) * block] & 3 == COMPUTING
    o.close()


@pytest.mark.parametrize("P", [2, 4])
@pytest.mark.parametrize("direction", [0, 2])
def test_pull_on_a_rank_without_roots(pkg, gpu_available, P, direction):
    """Hubs all on rank 0, their leaves spread over every rank: the other ranks start a pull level with
    an empty local frontier, and must still build their hot-head snapshot and pull (regression: k_collect
    returned on an empty local frontier, so their leaves were never reached)."""
    from stl_fusion_amd import workloads as W
    mix = W.StreamMix(64, 40, 8, 10, 0x5EED00E0)
    n = mix.n
    gs, block = _group(pkg, P, n, n_detached=0)
    used, dep, tag = mix.initial_edges()
    for g in gs:
        g.part_register_nodes(np.arange(n, dtype=np.uint32), mix.version, mix.state_flags())
        g.part_load_edges(used, dep, tag)
        g.set_option(pkg.fgi.OPT_DIRECTION, direction)
    o = O.Oracle(n)
    o.load_graph(mix.version, mix.state_flags(), used, dep, tag)
    for r in range(3):
        roots = mix.roots(r)
        o.clear_log()
        st = o.invalidate_slots(roots)
        stats = pkg.fgi.part_local_invalidate(gs, roots)
        ids = np.concatenate([g.part_export_ids() for g in gs])
        assert np.array_equal(np.sort(ids), np.sort(o.inv_log())), (r, len(ids), len(o.inv_log()))
        assert sum(x.v_inv for x in stats) == st.v_inv
    _check_states(gs, o, n, block)
    o.close()
