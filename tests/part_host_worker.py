"""One rank of the multi-process partition tests (tests/test_gpu_part_host.py): libfgi's partitioned
engine (fgi_part_init_host: every collective an all-gather through torch.distributed over gloo) in a
process of its own, all ranks on GPU 0. Launched by torch.distributed.run; writes this rank's results
to <out>/rank<r>.npz for the parent to compare with the oracle (test infrastructure; the oracle is used
here only to pick the same roots the parent's oracle run uses)."""
import argparse
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))

# the scenarios (shared with the parent test)
RMAT = dict(scale=13, ef=8, seed=0x5EED0027, sseed=0x5EED00C0)
WAVES = [(48, 0x5EED1027), (16, 99), (48, 0x5EED1027)]
MIX = dict(hubs=64, leaves=40, per_round=8, delay_pct=10, seed=0x5EED00E0, rounds=5)


def mix_schedule(W):
    """The streaming mix's batches (test_gpu_part_mutations.py's schedule), as (kind, args...) steps."""
    mix = W.StreamMix(MIX["hubs"], MIX["leaves"], MIX["per_round"], MIX["delay_pct"], MIX["seed"])
    prev = mix.roots(0)
    batches = [[("invalidate", prev)]]
    for r in range(1, MIX["rounds"]):
        timers, hs, ls = mix.plan(prev)
        vh = mix.new_versions(hs).copy()
        vl = mix.new_versions(ls).copy()
        roots = mix.roots(r)
        steps = []
        if len(timers):
            steps.append(("invalidate", timers, np.ones(len(timers), np.uint8)))
        steps += [("begin_compute", hs, vh), ("set_output", hs), ("begin_compute", ls, vl, mix.has_delay[ls]),
                  ("add_used", ls, mix.hub_of(ls)), ("set_output", ls), ("invalidate", roots)]
        batches.append(steps)
        prev = roots
    return batches


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--scenario", required=True, choices=["rmat", "mix"])
    ap.add_argument("--out", required=True)
    ap.add_argument("--stale", type=int, default=0)
    ap.add_argument("--bucket", type=int, default=0)
    ap.add_argument("--plan", type=int, default=1)
    args = ap.parse_args()

    import torch
    import torch.distributed as dist
    dist.init_process_group("gloo")
    rank, world = dist.get_rank(), dist.get_world_size()
    torch.cuda.set_device(0)
    import _pkg
    import fgo as O
    pkg = _pkg.load()
    from stl_fusion_amd import workloads as W
    res = {}
    if args.scenario == "rmat":
        n = 1 << RMAT["scale"]
        block = -(-n // world)
        g = pkg.Graph(block, rank=rank, world=world)
        g.part_init_host(n)
        g.part_synth_rmat(RMAT["scale"], RMAT["ef"], RMAT["seed"], args.stale, RMAT["sseed"])
        g.set_option(pkg.fgi.OPT_PART_PLAN, args.plan)
        if args.bucket:
            g.set_option(pkg.fgi.OPT_PART_BUCKET, args.bucket)
        s, _ = O.gen_rmat(RMAT["scale"], RMAT["ef"], RMAT["seed"])
        deg = np.bincount(s, minlength=n)
        for w, (k, rseed) in enumerate(WAVES):
            roots = O.gen_roots(k, n, rseed, deg)
            imm = (np.arange(len(roots)) % 5 == 0).astype(np.uint8)
            d_roots = torch.from_numpy(roots.astype(np.int32)).cuda()
            d_imm = torch.from_numpy(imm).cuda()
            st = pkg.WaveStats()
            g.part_invalidate(len(roots), d_roots.data_ptr(), d_imm.data_ptr(), st)
            res[f"w{w}_ids"] = g.part_export_ids()
            res[f"w{w}_stats"] = np.array([st.v_inv, st.e_trav, st.levels, st.host_syncs, st.pull_levels], np.uint64)
            v, f = g.dump_states()
            res[f"w{w}_ver"], res[f"w{w}_flags"] = v, f
    else:
        mix = W.StreamMix(MIX["hubs"], MIX["leaves"], MIX["per_round"], MIX["delay_pct"], MIX["seed"])
        n = mix.n
        block = -(-n // world)
        g = pkg.Graph(block, n_detached=256, rank=rank, world=world)
        g.part_init_host(n)
        used, dep, tag = mix.initial_edges()
        g.part_register_nodes(np.arange(n, dtype=np.uint32), mix.version, mix.state_flags())
        g.part_load_edges(used, dep, tag)
        for b, steps in enumerate(mix_schedule(W)):
            ids, outs = g.part_run_batch(steps)
            res[f"b{b}_ids"] = ids
            for k, o in enumerate(outs):
                if o is not None:
                    res[f"b{b}_out{k}"] = o
            v, f = g.dump_states()
            res[f"b{b}_ver"], res[f"b{b}_flags"] = v, f
        ps = g.part_prune()
        res["prune"] = np.array([ps.old_edges, ps.new_edges], np.uint64)
        u, d, t = g.export_edges()
        res["edges_u"], res["edges_d"], res["edges_t"] = u, d, t
        st = pkg.WaveStats()
        roots = mix.roots(99)
        d_roots = torch.from_numpy(roots.astype(np.int32)).cuda()
        g.part_invalidate(len(roots), d_roots.data_ptr(), 0, st)
        res["last_ids"] = g.part_export_ids()
        v, f = g.dump_states()
        res["last_ver"], res["last_flags"] = v, f
    res["block"] = np.array([block, n, world], np.uint64)
    np.savez(os.path.join(args.out, f"rank{rank}.npz"), **res)
    g.close()
    dist.barrier()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
