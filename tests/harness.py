"""Shared helpers: drive the engine (stl.fusion_amd) and the CPU oracle with the same operations
and compare their observable state. Only tests/ (and smoke/bench cpu leg) use the oracle."""
import numpy as np

import fgo as O

COMPUTING, CONSISTENT, INVALIDATED = 0, 1, 2
F_IOSO, F_DS, F_HD = 4, 8, 16


def random_states(n, rng, p_empty=0.05, p_computing=0.1, p_delay=0.1, p_invalidated=0.05, seed=1):
    """Per-slot (version, state_flags) with a mix of states (all versions LTag-like)."""
    versions = O.version_of(seed, np.arange(n, dtype=np.uint64))
    u = rng.random(n)
    flags = np.full(n, CONSISTENT, np.uint32)
    flags[u < p_computing] = COMPUTING
    hd = rng.random(n) < p_delay
    flags[hd] |= F_HD
    inv = (u >= p_computing) & (u < p_computing + p_invalidated)
    flags[inv] = INVALIDATED | (flags[inv] & F_HD)
    empty = rng.random(n) < p_empty
    versions = versions.copy()
    versions[empty] = 0
    flags[empty] = 0
    # a few Computing nodes already flagged, a few delayed nodes already started
    ds = (rng.random(n) < 0.02) & ((flags & 3) == CONSISTENT) & ((flags & F_HD) != 0)
    flags[ds] |= F_DS
    io = (rng.random(n) < 0.02) & ((flags & 3) == COMPUTING)
    flags[io] |= F_IOSO
    return versions, flags


def build_pair(pkg, n_slots, versions, flags, src, dst, tags, n_detached=64):
    g = pkg.Graph(n_slots, n_detached=n_detached)
    present = np.nonzero(versions)[0].astype(np.uint32)
    g.register_nodes(present, versions[present], flags[present])
    if len(src):
        g.load_edges(src, dst, tags)
    o = O.Oracle(n_slots)
    o.load_graph(versions, flags, src, dst, tags)
    return g, o


def canon_edges(u, d, t):
    a = np.stack([np.asarray(u, np.uint64), np.asarray(d, np.uint64), np.asarray(t, np.uint64)], axis=1)
    if len(a) == 0:
        return a
    order = np.lexsort((a[:, 2], a[:, 1], a[:, 0]))
    return a[order]


def oracle_edges(o, n_slots):
    """All live `_usedBy` entries of the oracle's current + last nodes, keyed by slot."""
    rows = []
    for s in range(n_slots):
        h = o.last(s)
        if h == O.NONE:
            continue
        d, t = o.used_by(h)
        if len(d):
            rows.append(canon_edges(np.full(len(d), s, np.uint64), d, t))
    if not rows:
        return np.zeros((0, 3), np.uint64)
    return canon_edges(*np.concatenate(rows).T)


def assert_states_equal(g, o, n_slots):
    gv, gf = g.dump_states()
    ov, of = o.dump_states()
    assert np.array_equal(gv[:n_slots], ov), "versions differ"
    bad = np.nonzero(gf[:n_slots] != of)[0]
    assert len(bad) == 0, f"state_flags differ at {bad[:10]}: engine {gf[bad[:10]]} oracle {of[bad[:10]]}"
