"""Diagnostic (round 5): test_labelled_mutations_batches_and_prune's `_usedBy` mismatch, for labels
on and off: after the same mutations, every slot whose fgi_get_used_by differs from the oracle's, with
the node words on both sides of each differing entry."""
import sys

import numpy as np

sys.path.insert(0, ".")
sys.path.insert(0, "tests")
sys.path.insert(0, "oracle")
import fgo as O  # noqa: E402
import _pkg  # noqa: E402
pkg = _pkg.load()
from harness import assert_states_equal, canon_edges, random_states  # noqa: E402
from test_gpu_part_mutations import _churn_batch  # noqa: E402


def run(labels, stop_after):
    scale, ef, seed = 12, 8, 3
    n = 1 << scale
    rng = np.random.default_rng(91)
    versions, flags = random_states(n, rng, seed=seed)
    s, d = O.gen_rmat(scale, ef, seed)
    live = (versions[s] != 0) & ((flags[s] & 3) == 1)
    s, d = s[live], d[live]
    tags = versions[d].astype(np.uint64).copy()
    tags[tags == 0] = 7
    tags[rng.random(len(s)) < 0.25] += np.uint64(1)
    g = pkg.Graph(n, n_detached=256, labels=labels)
    present = np.nonzero(versions)[0].astype(np.uint32)
    g.register_nodes(present, versions[present], flags[present])
    g.load_edges(s, d, tags)
    o = O.Oracle(n)
    o.load_graph(versions, flags, s, d, tags)

    def check(tag):
        bad = []
        for x in range(n):
            gd, gt = g.used_by(x)
            oh = o.current(x)
            od, ot = o.used_by(oh) if oh != O.NONE else (np.zeros(0, np.uint32), np.zeros(0, np.uint64))
            a = canon_edges(np.full(len(gd), x), gd, gt)
            b = canon_edges(np.full(len(od), x), od, ot)
            if not np.array_equal(a, b):
                bad.append((x, a.tolist(), b.tolist()))
        ov, of = o.dump_states()
        gv, gf = g.dump_states()
        print(f"labels={labels} after {tag}: {len(bad)} slots differ", flush=True)
        for x, a, b in bad[:6]:
            print(f"  slot {x}: engine {a} oracle {b} word v={ov[x]} f={of[x]} / v={gv[x]} f={gf[x]}", flush=True)
            for e in b:
                dd = int(e[1])
                print(f"    dependant {dd}: oracle v={ov[dd]} f={of[dd]} engine v={gv[dd]} f={gf[dd]} tag {e[2]}", flush=True)
        return len(bad)

    check("load")
    bc = rng.choice(n, 40, replace=False).astype(np.uint32)
    ver = np.arange(1 << 44, (1 << 44) + 2 * len(bc), 2, dtype=np.uint64) | np.uint64(1)
    hd = (rng.random(len(bc)) < 0.3).astype(np.uint8)
    o.clear_log()
    g.begin_compute(bc, ver, hd)
    o.begin_compute_slots(bc, ver, hd)
    check("begin_compute")
    dep = rng.choice(bc, 60).astype(np.uint32)
    ov, _ = o.dump_states()
    use = rng.choice(np.nonzero(ov)[0], 60).astype(np.uint32)
    g.add_used(dep, use)
    o.add_used_slots(dep, use)
    check("add_used")
    o.clear_log()
    g.set_output(bc)
    o.set_output_slots(bc)
    check("set_output")
    nv = (1 << 45) | 1
    for b in range(4):
        ov, _ = o.dump_states()
        steps, nv = _churn_batch(rng, n, ov != 0, nv)
        g.run_batch(steps)
        for k, sp in enumerate(steps):
            if sp[0] == "invalidate":
                o.invalidate_slots(sp[1], sp[2] if len(sp) > 2 else None)
            elif sp[0] == "begin_compute":
                o.begin_compute_slots(sp[1], sp[2], sp[3])
            elif sp[0] == "add_used":
                o.add_used_slots(sp[1], sp[2])
            else:
                o.set_output_slots(sp[1])
        assert_states_equal(g, o, n)
        if check(f"batch {b}") and stop_after:
            break
    g.close()
    o.close()


if __name__ == "__main__":
    run(-1, True)
    run(1, True)
