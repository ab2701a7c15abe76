#!/usr/bin/env python3
"""Regenerates tests/golden/*.json: small invalidation cases frozen from the CPU oracle.

Each fixture holds the inputs (per-slot version + state_flags, `_usedBy` edges, roots,
immediately flags) and the expected outputs (sorted invalidated slots, final canonical
version/state_flags per slot, V_inv, E_trav, and the `_usedBy` edge set after a prune).
tests/test_oracle_golden.py checks them against the oracle and against an independent pure-Python
restatement; tests/test_gpu_golden.py checks the engine against them.

    python tests/golden/make_golden.py
"""
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
sys.path.insert(0, os.path.join(ROOT, "tests"))
import fgo as O  # noqa: E402
from harness import random_states  # noqa: E402


def live_edges(versions, flags, rng, m, n, stale_p):
    live = np.nonzero((versions != 0) & ((flags & 3) == 1))[0]
    src = rng.choice(live, m)
    dst = rng.integers(0, n, m)
    tags = versions[dst].astype(np.uint64).copy()
    tags[tags == 0] = 7
    tags[rng.random(m) < stale_p] += np.uint64(1)
    return src.astype(np.uint32), dst.astype(np.uint32), tags


def case_random(name, seed, n, m, n_roots, stale_p, p_imm):
    rng = np.random.default_rng(seed)
    versions, flags = random_states(n, rng)
    src, dst, tags = live_edges(versions, flags, rng, m, n, stale_p)
    roots = rng.integers(0, n, n_roots).astype(np.uint32)
    imm = (rng.random(n_roots) < p_imm).astype(np.uint8)
    return dict(name=name, n=n, versions=versions, flags=flags, src=src, dst=dst, tags=tags, roots=roots, imm=imm)


def case_rmat(name, scale, ef, seed, stale, n_roots):
    n = 1 << scale
    s, d = O.gen_rmat(scale, ef, seed)
    versions = O.version_of(seed, np.arange(n))
    flags = np.full(n, 1, np.uint32)
    tags = O.gen_tags(s, d, seed, stale, 0x5EED00C0)
    roots = O.gen_roots(n_roots, n, seed + 1, np.bincount(s, minlength=n))
    return dict(name=name, n=n, versions=versions, flags=flags, src=s, dst=d, tags=tags, roots=roots,
                imm=np.zeros(len(roots), np.uint8))


def case_layered(name, levels, width, fanout, seed, n_roots):
    n = levels * width
    s, d = O.gen_layered(levels, width, fanout, seed)
    versions = O.version_of(seed, np.arange(n))
    roots = O.gen_roots(n_roots, width, seed + 1, np.bincount(s, minlength=n)[:width])
    return dict(name=name, n=n, versions=versions, flags=np.full(n, 1, np.uint32), src=s, dst=d,
                tags=O.gen_tags(s, d, seed), roots=roots, imm=np.zeros(len(roots), np.uint8))


def solve(c):
    o = O.Oracle(c["n"])
    o.load_graph(c["versions"], c["flags"], c["src"], c["dst"], c["tags"])
    st = o.invalidate_slots(c["roots"], c["imm"])
    inv = sorted(int(x) for x in o.inv_log())
    v, f = o.dump_states()
    o.prune()
    rows = []
    for slot in range(c["n"]):
        h = o.last(slot)
        if h == O.NONE:
            continue
        dd, tt = o.used_by(h)
        rows += [[slot, int(a), int(b)] for a, b in zip(dd, tt)]
    rows.sort()
    return dict(inv=inv, v_inv=int(st.v_inv), e_trav=int(st.e_trav), final_versions=[int(x) for x in v],
                final_flags=[int(x) for x in f], pruned_edges=rows)


def main():
    cases = [
        case_random("mixed_states_imm", 1, 300, 2000, 25, 0.3, 0.3),
        case_random("mostly_stale", 2, 200, 1500, 10, 0.8, 0.0),
        case_random("dense_small", 3, 64, 1200, 4, 0.1, 0.5),
        case_rmat("rmat8_live", 8, 8, 0x5EED0024, 0, 8),
        case_rmat("rmat9_churn50", 9, 8, 0x5EED0024, 50, 8),
        case_layered("layered_7x40_f4", 7, 40, 4, 0x5EED0001, 5),
    ]
    for c in cases:
        out = solve(c)
        doc = dict(name=c["name"], generator="tests/golden/make_golden.py", n_slots=c["n"],
                   versions=[int(x) for x in c["versions"]], state_flags=[int(x) for x in c["flags"]],
                   used=[int(x) for x in c["src"]], dependant=[int(x) for x in c["dst"]],
                   tags=[int(x) for x in c["tags"]], roots=[int(x) for x in c["roots"]],
                   immediately=[int(x) for x in c["imm"]], expected=out)
        with open(os.path.join(HERE, c["name"] + ".json"), "w") as fh:
            json.dump(doc, fh, separators=(",", ":"))
        print(c["name"], "v_inv", out["v_inv"], "e_trav", out["e_trav"], "pruned", len(out["pruned_edges"]))


if __name__ == "__main__":
    main()
