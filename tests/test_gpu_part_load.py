"""A partitioned engine loaded by a host (fgi_part_register_nodes / fgi_part_load_edges): the
registry and edge import of ComputedRegistry.Register (ComputedRegistry.cs:72-105) and AddUsedBy
(Computed.cs:381-382) with global ids, every rank given the same arrays. P in-process partitions
(fgi_part_init_local: run_part_wave's level loop on every rank, device copies for the collectives)
must reproduce the oracle on the committed golden fixtures and on random mixed-state graphs
(Computing nodes, invalidation delays, Invalidated and empty slots, stale edges, immediately roots):
the same invalidated set, V_inv, E_trav and final node words, over consecutive waves."""
import glob
import json
import os

import numpy as np
import pytest

import fgo as O
from harness import random_states
from test_gpu_parity import _edges_from_live

pytestmark = pytest.mark.gpu

GOLDEN = sorted(glob.glob(os.path.join(os.path.dirname(__file__), "golden", "*.json")))


def _partitioned(pkg, n, P, versions, flags, used, dep, tags, direction, labels=0, tpb=0):
    block = -(-n // P)
    gs = [pkg.Graph(block, rank=r, world=P, labels=labels) for r in range(P)]
    pkg.fgi.part_init_local(gs, n)
    present = np.nonzero(versions)[0].astype(np.uint32)
    for g in gs:
        g.set_option(pkg.fgi.OPT_DIRECTION, direction)
        if tpb:
            g.set_option(pkg.fgi.OPT_PULL_TPB, tpb)
        g.part_register_nodes(present, versions[present], flags[present])
        if len(used):
            g.part_load_edges(used, dep, tags)
    return gs, block


def _check(pkg, gs, block, n, o, roots, imm):
    st = o.invalidate_slots(roots, imm)
    stats = pkg.fgi.part_local_invalidate(gs, roots, imm)
    ids = np.concatenate([g.part_export_ids() for g in gs])
    assert len(np.unique(ids)) == len(ids)
    assert np.array_equal(np.sort(ids), np.sort(o.inv_log())), (len(ids), len(o.inv_log()))
    assert sum(x.v_inv for x in stats) == st.v_inv
    assert sum(x.e_trav for x in stats) == st.e_trav
    ov, of = o.dump_states()
    for r, g in enumerate(gs):
        v, f = g.dump_states()
        lo, hi = r * block, min(n, (r + 1) * block)
        assert np.array_equal(v[:hi - lo], ov[lo:hi]), r
        bad = np.nonzero(f[:hi - lo] != of[lo:hi])[0]
        assert len(bad) == 0, (r, bad[:8], f[bad[:8]], of[lo + bad[:8]])
    o.clear_log()
    return stats


@pytest.mark.parametrize("direction", [1, 0])
@pytest.mark.parametrize("P", [2, 3, 8])
@pytest.mark.parametrize("path", GOLDEN, ids=[os.path.basename(p)[:-5] for p in GOLDEN])
def test_partition_loads_golden_fixture(pkg, gpu_available, path, P, direction):
    doc = json.load(open(path))
    n = doc["n_slots"]
    v = np.array(doc["versions"], np.uint64)
    f = np.array(doc["state_flags"], np.uint32)
    u = np.array(doc["used"], np.uint32)
    d = np.array(doc["dependant"], np.uint32)
    t = np.array(doc["tags"], np.uint64)
    gs, block = _partitioned(pkg, n, P, v, f, u, d, t, direction)
    o = O.Oracle(n)
    o.load_graph(v, f, u, d, t)
    roots = np.array(doc["roots"], np.uint32)
    imm = np.array(doc["immediately"], np.uint8)
    _check(pkg, gs, block, n, o, roots, imm)
    exp = doc["expected"]
    ids = np.sort(np.concatenate([g.part_export_ids() for g in gs]))
    assert ids.tolist() == exp["inv"]
    for g in gs:
        g.close()
    o.close()


@pytest.mark.parametrize("direction", [1, 2, 0])
@pytest.mark.parametrize("P", [2, 3, 8])
def test_partition_loads_mixed_state_graph(pkg, gpu_available, P, direction, labels=0, tpb=0):
    rng = np.random.default_rng(100 + 10 * P + direction)
    n = 4096
    versions, flags = random_states(n, rng)
    src, dst, tags = _edges_from_live(versions, flags, rng, 60000, n, stale_p=0.3)
    # a second batch (incremental load: set semantics across batches, duplicates included)
    src2, dst2, tags2 = _edges_from_live(versions, flags, rng, 20000, n, stale_p=0.3)
    src2 = np.concatenate([src2, src[:500]])
    dst2 = np.concatenate([dst2, dst[:500]])
    tags2 = np.concatenate([tags2, tags[:500]])
    gs, block = _partitioned(pkg, n, P, versions, flags, src, dst, tags, direction, labels, tpb)
    for g in gs:
        g.part_load_edges(src2, dst2, tags2)
    o = O.Oracle(n)
    o.load_graph(versions, flags, np.concatenate([src, src2]), np.concatenate([dst, dst2]),
                 np.concatenate([tags, tags2]))
    # the rows each rank owns are exactly the loaded set (global ids)
    rows = []
    for r, g in enumerate(gs):
        u, d, t = g.export_edges()
        rows.append(np.stack([u.astype(np.uint64) + r * block, d, t], 1))
    got = np.unique(np.concatenate(rows), axis=0)
    want = np.unique(np.stack([np.concatenate([src, src2]).astype(np.uint64), np.concatenate([dst, dst2]),
                               np.concatenate([tags, tags2])], 1), axis=0)
    live_src = ((versions != 0) & ((flags & 3) != 2))[want[:, 0].astype(np.int64)]
    assert np.array_equal(got, want[live_src])
    roots = rng.integers(0, n, 200).astype(np.uint32)   # duplicates and empty slots included
    imm = (rng.random(200) < 0.3).astype(np.uint8)
    stats = _check(pkg, gs, block, n, o, roots, imm)
    if direction == 2 and block % 32 == 0:
        assert all(x.pull_levels == x.levels for x in stats)
    if direction == 1:
        assert sum(x.remote_msgs for x in stats) > 0
    # a second wave from the partitioned state
    roots2 = rng.integers(0, n, 64).astype(np.uint32)
    _check(pkg, gs, block, n, o, roots2, None)
    for g in gs:
        g.close()
    o.close()


@pytest.mark.parametrize("tpb", [0, 1])
@pytest.mark.parametrize("direction", [2, 0])
@pytest.mark.parametrize("P", [2, 3, 8])
def test_partition_codes_mixed_state_graph(pkg, gpu_available, P, direction, tpb):
    """Partition codes (labels=1: hub-first numbering inside each rank's range, chosen at the first bulk
    load, dealt over the runs of slots the pull blocks own: one tile per block with tpb=1, so P=2's
    2,048-slot ranges become two runs) on the mixed-state graphs, twice in a row: the second set of
    graphs gets the first one's freed device memory, whose version replica held every slot's version, so
    an empty slot's replica entry must start at 0 (stale edges into empty slots carry exactly those
    versions)."""
    for _ in range(2):
        test_partition_loads_mixed_state_graph(pkg, gpu_available, P, direction, labels=1, tpb=tpb)


def test_partition_codes_disagreement_fails_every_rank(pkg, gpu_available):
    """Each rank chooses its partition codes alone, from the arrays it is given; the host contract is that
    every rank gets the same ones. A rank given other arrays (here rank 0 misses one registration, so the
    heavy slot 700 weighs nothing in its replica) numbers the slots differently, and the wave's first
    all-reduce (the codes' fingerprint) fails the wave on every rank instead of returning wrong ids."""
    n, P = 1024, 2
    block = n // P
    gs = [pkg.Graph(block, rank=r, world=P, labels=1) for r in range(P)]
    pkg.fgi.part_init_local(gs, n)
    versions = O.version_of(1, np.arange(n, dtype=np.uint64))
    rng = np.random.default_rng(7)
    src = rng.integers(0, n, 4000).astype(np.uint32)
    dst = rng.integers(0, n, 4000).astype(np.uint32)
    dst[:600] = 700                                  # slot 700 (rank 1's) is the heaviest dependant
    tags = versions[dst]
    allslots = np.arange(n, dtype=np.uint32)
    for r, g in enumerate(gs):
        reg = allslots if r == 1 else allslots[allslots != 700]
        g.part_register_nodes(reg, versions[reg])
        g.part_load_edges(src, dst, tags)
    with pytest.raises(pkg.FgiError) as e:
        pkg.fgi.part_local_invalidate(gs, np.array([1, 2, 3], np.uint32))
    assert e.value.status == pkg.fgi.ESTATE and "numbered their slots differently" in str(e.value)
    for g in gs:
        g.close()


def test_part_load_refusals(pkg, gpu_available):
    n, P = 1024, 2
    gs = [pkg.Graph(n // P, rank=r, world=P) for r in range(P)]
    pkg.fgi.part_init_local(gs, n)
    g = gs[0]
    with pytest.raises(pkg.FgiError) as e:
        g.part_register_nodes(np.array([n], np.uint32), np.array([3], np.uint64))
    assert e.value.status == pkg.fgi.EINVAL
    g.part_register_nodes(np.array([5, 700], np.uint32), np.array([3, 9], np.uint64))
    with pytest.raises(pkg.FgiError) as e:   # slot 5 is owned by rank 0 and already has a node
        g.part_register_nodes(np.array([5], np.uint32), np.array([7], np.uint64))
    assert e.value.status == pkg.fgi.ESTATE
    with pytest.raises(pkg.FgiError) as e:
        g.part_load_edges(np.array([5], np.uint32), np.array([700], np.uint32), np.array([0], np.uint64))
    assert e.value.status == pkg.fgi.EINVAL
    # the single-device imports refuse a partition
    for call in (lambda: g.register_nodes(np.array([1], np.uint32), np.array([3], np.uint64)),
                 lambda: g.load_edges(np.array([1], np.uint32), np.array([2], np.uint32), np.array([3], np.uint64))):
        with pytest.raises(pkg.FgiError) as e:
            call()
        assert e.value.status == pkg.fgi.ESTATE
    for x in gs:
        x.close()
