"""The engine (through the C-ABI) reproduces every committed golden fixture, on each traversal path."""
import glob
import json
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

GOLDEN = sorted(glob.glob(os.path.join(os.path.dirname(__file__), "golden", "*.json")))


@pytest.mark.parametrize("direction", [1, 2, 0])
@pytest.mark.parametrize("path", GOLDEN, ids=[os.path.basename(p)[:-5] for p in GOLDEN])
def test_engine_reproduces_golden(pkg, gpu_available, path, direction):
    doc = json.load(open(path))
    exp = doc["expected"]
    n = doc["n_slots"]
    g = pkg.Graph(n, n_detached=8)
    g.set_option(2, direction)
    v = np.array(doc["versions"], np.uint64)
    f = np.array(doc["state_flags"], np.uint32)
    present = np.nonzero(v)[0].astype(np.uint32)
    g.register_nodes(present, v[present], f[present])
    g.load_edges(doc["used"], doc["dependant"], doc["tags"])
    ws = pkg.WaveStats()
    ids = g.invalidate(doc["roots"], doc["immediately"], stats=ws)
    assert sorted(ids.tolist()) == exp["inv"]
    assert (ws.v_inv, ws.e_trav) == (exp["v_inv"], exp["e_trav"])
    gv, gf = g.dump_states()
    assert gv[:n].tolist() == exp["final_versions"]
    assert gf[:n].tolist() == exp["final_flags"]
    g.prune()
    u, d, t = g.export_edges()
    rows = sorted([int(a), int(b), int(c)] for a, b, c in zip(u, d, t) if a < n)
    assert rows == exp["pruned_edges"]
