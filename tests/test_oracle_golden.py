"""Golden fixtures (tests/golden/*.json, made by tests/golden/make_golden.py from the oracle) checked
against (a) the oracle itself — regressions — and (b) an independent pure-Python restatement of the
reference cascade (Computed.cs:162-230, ComputedRegistry.cs:57-70, Computed.cs:400-419) written
directly from the rules, so the C++ oracle is cross-checked by a second implementation."""
import glob
import json
import os

import numpy as np
import pytest

import fgo as O

GOLDEN = sorted(glob.glob(os.path.join(os.path.dirname(__file__), "golden", "*.json")))
IOSO, DS, HD = 4, 8, 16


def load(path):
    with open(path) as fh:
        return json.load(fh)


def py_restatement(doc):
    """Sequential, recursion-free restatement over the slot model; returns the same fields."""
    n = doc["n_slots"]
    ver = list(doc["versions"])
    flags = list(doc["state_flags"])
    state = [f & 3 for f in flags]
    rows = {}
    for u, d, t in zip(doc["used"], doc["dependant"], doc["tags"]):
        rows.setdefault(u, set()).add((d, t))
    deg0 = {u: len(r) for u, r in rows.items()}
    inv, e_trav = [], 0

    def current(s):
        return ver[s] != 0 and state[s] != 2

    def visit(s, imm, stack):
        nonlocal e_trav
        if not current(s):
            return
        if state[s] == 0:                                  # Computing
            flags[s] |= IOSO | (DS if imm else 0)
            return
        if imm or not (flags[s] & HD):                     # Consistent -> Invalidated
            state[s] = 2
            inv.append(s)
            e_trav += deg0.get(s, 0)
            stack.extend(rows.get(s, ()))
            return
        flags[s] |= DS                                     # delayed

    for r, imm in zip(doc["roots"], doc["immediately"]):
        stack = []
        visit(r, bool(imm), stack)
        while stack:
            d, t = stack.pop()
            if current(d) and ver[d] == t:
                visit(d, False, stack)
    final = []
    for s in range(n):
        if ver[s] == 0:
            final.append(0)
            continue
        f = state[s] | (flags[s] & HD)
        if state[s] == 0:
            f |= flags[s] & (IOSO | DS)
        elif state[s] == 1:
            f |= flags[s] & DS
        final.append(f)
    pruned = []
    for u in range(n):
        if not (current(u) and state[u] == 1):
            # Computing nodes keep their (empty) sets; invalidated ones were cleared
            if current(u):
                pruned += [[u, d, t] for d, t in rows.get(u, ())]
            continue
        pruned += [[u, d, t] for d, t in rows.get(u, ()) if current(d) and ver[d] == t]
    pruned.sort()
    return dict(inv=sorted(inv), v_inv=len(inv), e_trav=e_trav, final_versions=ver, final_flags=final,
                pruned_edges=pruned)


@pytest.mark.parametrize("path", GOLDEN, ids=[os.path.basename(p)[:-5] for p in GOLDEN])
def test_oracle_reproduces_golden(path):
    doc = load(path)
    exp = doc["expected"]
    o = O.Oracle(doc["n_slots"])
    o.load_graph(np.array(doc["versions"], np.uint64), np.array(doc["state_flags"], np.uint32),
                 np.array(doc["used"], np.uint32), np.array(doc["dependant"], np.uint32),
                 np.array(doc["tags"], np.uint64))
    st = o.invalidate_slots(np.array(doc["roots"], np.uint32), np.array(doc["immediately"], np.uint8))
    assert sorted(o.inv_log().tolist()) == exp["inv"]
    assert (st.v_inv, st.e_trav) == (exp["v_inv"], exp["e_trav"])
    v, f = o.dump_states()
    assert v.tolist() == exp["final_versions"] and f.tolist() == exp["final_flags"]


@pytest.mark.parametrize("path", GOLDEN, ids=[os.path.basename(p)[:-5] for p in GOLDEN])
def test_python_restatement_agrees_with_golden(path):
    doc = load(path)
    exp = doc["expected"]
    got = py_restatement(doc)
    assert got["inv"] == exp["inv"]
    assert got["v_inv"] == exp["v_inv"] and got["e_trav"] == exp["e_trav"]
    assert got["final_versions"] == exp["final_versions"]
    assert got["final_flags"] == exp["final_flags"]
    assert got["pruned_edges"] == exp["pruned_edges"]


def test_golden_fixtures_present():
    assert len(GOLDEN) >= 6
    for p in GOLDEN:
        doc = load(p)
        assert doc["generator"] == "tests/golden/make_golden.py"
        assert len(doc["used"]) == len(doc["dependant"]) == len(doc["tags"])
