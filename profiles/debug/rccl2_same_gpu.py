"""Debug: can two RCCL ranks share the one GPU of the box (the N=2 partitioned path through real RCCL)?
Two processes, each one partition rank on device 0, an R-MAT 14 wave against the oracle."""
import os
import sys
import numpy as np
import torch.multiprocessing as mp


def worker(rank, world, q_uid, q_out):
    sys.path.insert(0, ".")
    sys.path.insert(0, "oracle")
    import _pkg
    pkg = _pkg.load()
    try:
        scale, ef, seed = 14, 16, 0x5EED0027
        n = 1 << scale
        block = -(-n // world)
        g = pkg.Graph(block, device=0, rank=rank, world=world)
        if rank == 0:
            uid = pkg.fgi.part_unique_id()
            for _ in range(world - 1):
                q_uid.put(uid)
        else:
            uid = q_uid.get(timeout=60)
        g.part_init(n, uid)
        g.part_synth_rmat(scale, ef, seed, 20, 0x5EED00C0)
        import fgo as O
        s, d = O.gen_rmat(scale, ef, seed)
        roots = O.gen_roots(64, n, 5, np.bincount(s, minlength=n))
        import torch
        dr = torch.from_numpy(roots.astype(np.int32)).cuda()
        out = []
        for plan in (0, 1, 1):
            g.set_option(pkg.fgi.OPT_PART_PLAN, plan)
            g.snapshot() if plan == 0 and not out else g.restore()
            st = pkg.fgi.WaveStats()
            nv = g.part_invalidate(len(roots), dr.data_ptr(), 0, st)
            out.append((plan, nv, st.levels, st.host_syncs, sorted(g.part_export_ids().tolist())))
        q_out.put((rank, out))
    except Exception as e:
        import traceback
        q_out.put((rank, "error: " + traceback.format_exc()))


if __name__ == "__main__":
    world = 2
    ctx = mp.get_context("spawn")
    q_uid, q_out = ctx.Queue(), ctx.Queue()
    ps = [ctx.Process(target=worker, args=(r, world, q_uid, q_out)) for r in range(world)]
    for p in ps:
        p.start()
    res = {}
    for _ in range(world):
        r, o = q_out.get(timeout=240)
        res[r] = o
    for p in ps:
        p.join(timeout=60)
    for r in sorted(res):
        o = res[r]
        if isinstance(o, str):
            print("rank", r, o[-2000:])
        else:
            print("rank", r, [(a, b, c, d, len(e)) for a, b, c, d, e in o])
    if all(not isinstance(o, str) for o in res.values()):
        sys.path.insert(0, "oracle")
        import fgo as O
        scale, ef, seed = 14, 16, 0x5EED0027
        n = 1 << scale
        s, d = O.gen_rmat(scale, ef, seed)
        o = O.Oracle(n)
        o.load_graph(O.version_of(seed, np.arange(n)), None, s, d, O.gen_tags(s, d, seed, 20, 0x5EED00C0))
        roots = O.gen_roots(64, n, 5, np.bincount(s, minlength=n))
        o.invalidate_slots(roots)
        want = np.sort(o.inv_log())
        for k in range(3):
            got = np.sort(np.concatenate([np.asarray(res[r][k][4], np.uint32) for r in sorted(res)]))
            print("wave", k, "matches oracle:", np.array_equal(got, want), len(got), len(want))
