"""Debug: engine vs golden fixtures per direction, with details on mismatching nodes."""
import glob, json, os, sys
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
import _pkg
pkg = _pkg.load()
for path in sorted(glob.glob(os.path.join(ROOT, "tests", "golden", "*.json"))):
    doc = json.load(open(path))
    exp = doc["expected"]
    n = doc["n_slots"]
    for direction in (1, 2, 0):
        for use_imm in (True, False):
            if not use_imm and direction != 2:
                continue
            g = pkg.Graph(n, n_detached=8)
            g.set_option(2, direction)
            v = np.array(doc["versions"], np.uint64)
            f = np.array(doc["state_flags"], np.uint32)
            present = np.nonzero(v)[0].astype(np.uint32)
            g.register_nodes(present, v[present], f[present])
            g.load_edges(doc["used"], doc["dependant"], doc["tags"])
            ws = pkg.WaveStats()
            imm = doc["immediately"] if use_imm else None
            ids = g.invalidate(doc["roots"], imm, stats=ws)
            got = sorted(ids.tolist())
            tag = f"{os.path.basename(path)} dir={direction} imm={use_imm}"
            if not use_imm:
                print(tag, "v_inv", ws.v_inv, "levels", ws.levels, "pull_levels", ws.pull_levels)
                g.close()
                continue
            ok = got == exp["inv"]
            print(tag, "OK" if ok else "MISMATCH", "v_inv", ws.v_inv, exp["v_inv"], "levels", ws.levels,
                  "pull", ws.pull_levels, "dups", len(got) - len(set(got)))
            if not ok:
                a, b = set(got), set(exp["inv"])
                for x in sorted(b - a)[:5]:
                    ins = [(int(u), int(t)) for u, d, t in zip(doc["used"], doc["dependant"], doc["tags"]) if d == x]
                    print("  missing", x, "ver", v[x], "flags", f[x], "root", x in doc["roots"],
                          "parents(tag match)", [(u, u in b, t == int(v[x])) for u, t in ins][:12])
                for x in sorted(a - b)[:5]:
                    print("  extra", x, "flags", f[x])
            g.close()
