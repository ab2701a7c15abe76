"""The partitioned engine across real process boundaries.

Two or three processes, launched by torch.distributed.run, each hold one rank's partition on GPU 0
(RCCL refuses two ranks on one GPU, so their collectives go through fgi_part_init_host: every exchange
of run_part_wave, the mutations' all-reduces and the prune's all-gather as a host all-gather over
gloo). Everything else is the code an N-GPU run executes: the planned waves with their fixed buckets
and carry-over, the host-driven level loop, fgi_part_run_batch's steps and fgi_part_prune. The parent
runs the oracle on the whole graph (Computed.cs:162-230 cascade, 141-160 TrySetOutput, 347-385
AddUsed, ComputedRegistry.cs:72-105 Register with displacement, Computed.cs:400-419 PruneUsedBy) and
checks every rank's invalidated slots, add_used codes, set flags and node words, and the pruned edge
sets. World size 3 is ragged (the slot count is not a multiple of 3)."""
import os
import socket
import subprocess
import sys

import numpy as np
import pytest

import fgo as O
from harness import canon_edges

pytestmark = pytest.mark.gpu

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
import part_host_worker as PW  # noqa: E402


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _launch(P, tmp_path, *args):
    out = tmp_path / f"p{P}"
    out.mkdir()
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={P}",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()),
           os.path.join(HERE, "part_host_worker.py"), "--out", str(out), *map(str, args)]
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    env["OMP_NUM_THREADS"] = "2"
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=110, env=env)
    assert r.returncode == 0, r.stderr[-3000:]
    return [dict(np.load(out / f"rank{q}.npz")) for q in range(P)]


def _states_match(ranks, key, ov, of):
    for q, res in enumerate(ranks):
        block, n, _ = (int(x) for x in res["block"])
        lo, hi = q * block, min(n, (q + 1) * block)
        v, f = res[f"{key}_ver"], res[f"{key}_flags"]
        assert np.array_equal(v[:hi - lo], ov[lo:hi]), f"{key}: rank {q} versions differ"
        assert np.array_equal(f[:hi - lo], of[lo:hi]), f"{key}: rank {q} flags differ"


@pytest.mark.parametrize("P,stale,bucket,plan", [(2, 0, 0, 1), (3, 50, 0, 1), (2, 0, 2, 1), (3, 0, 0, 0)])
def test_rmat_waves_across_processes(gpu_available, tmp_path, P, stale, bucket, plan):
    """Three waves (the second from other roots, the third repeating the first, which a planned wave
    follows with one host synchronisation), mixed immediate roots, 0% / 50% stale edges, buckets of 2
    words (one id per peer per push level: most ids wait for later push levels), the plan off."""
    ranks = _launch(P, tmp_path, "--scenario", "rmat", "--stale", stale, "--bucket", bucket, "--plan", plan)
    c = PW.RMAT
    n = 1 << c["scale"]
    s, d = O.gen_rmat(c["scale"], c["ef"], c["seed"])
    o = O.Oracle(n)
    o.load_graph(O.version_of(c["seed"], np.arange(n)), None, s, d, O.gen_tags(s, d, c["seed"], stale, c["sseed"]))
    deg = np.bincount(s, minlength=n)
    for w, (k, rseed) in enumerate(PW.WAVES):
        roots = O.gen_roots(k, n, rseed, deg)
        imm = (np.arange(len(roots)) % 5 == 0).astype(np.uint8)
        o.clear_log()
        st = o.invalidate_slots(roots, imm)
        ids = np.concatenate([r[f"w{w}_ids"] for r in ranks])
        assert np.array_equal(np.sort(ids), np.sort(o.inv_log())), f"wave {w}: {len(ids)} vs {st.v_inv}"
        assert sum(int(r[f"w{w}_stats"][0]) for r in ranks) == st.v_inv
        if w == 0:
            assert sum(int(r[f"w{w}_stats"][1]) for r in ranks) == st.e_trav
        ov, of = o.dump_states()
        _states_match(ranks, f"w{w}", ov, of)
    if plan:
        # the repeated wave follows the learnt plan: its start and end all-reduces only
        assert all(int(r["w2_stats"][3]) == 2 for r in ranks), [int(r["w2_stats"][3]) for r in ranks]
    o.close()


@pytest.mark.parametrize("P", [2, 3])
def test_streaming_batches_and_prune_across_processes(gpu_available, tmp_path, P):
    """BASELINE.json configs[4]'s schedule at 64 hubs x 40 leaves (10% delayed) through
    fgi_part_run_batch in P processes: delay timers, begin_compute with displacement, add_used pairs
    crossing ranks, set_output, waves; then fgi_part_prune and a wave on the pruned graph."""
    ranks = _launch(P, tmp_path, "--scenario", "mix")
    from stl_fusion_amd import workloads as W
    mix = W.StreamMix(PW.MIX["hubs"], PW.MIX["leaves"], PW.MIX["per_round"], PW.MIX["delay_pct"], PW.MIX["seed"])
    n = mix.n
    used, dep, tag = mix.initial_edges()
    o = O.Oracle(n)
    o.load_graph(mix.version, mix.state_flags(), used, dep, tag)
    for b, steps in enumerate(PW.mix_schedule(W)):
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
        ids = np.concatenate([r[f"b{b}_ids"] for r in ranks])
        assert np.array_equal(np.sort(ids), np.sort(o.inv_log())), f"batch {b}"
        for k, sp in enumerate(steps):
            for q, r in enumerate(ranks):
                if sp[0] == "add_used":
                    assert np.array_equal(r[f"b{b}_out{k}"], outs[k]), f"batch {b} step {k} rank {q}"
                elif sp[0] == "set_output":
                    assert int(r[f"b{b}_out{k}"].sum()) == outs[k], f"batch {b} step {k} rank {q}"
        ov, of = o.dump_states()
        _states_match(ranks, f"b{b}", ov, of)
    _, ne = o.prune()
    assert sum(int(r["prune"][1]) for r in ranks) == ne
    rows = []
    for q, r in enumerate(ranks):
        block = int(r["block"][0])
        keep = r["edges_u"] < block
        rows.append(canon_edges(r["edges_u"][keep].astype(np.uint64) + np.uint64(q * block), r["edges_d"][keep],
                                r["edges_t"][keep]))
    got = np.concatenate(rows)
    assert np.array_equal(canon_edges(*got.T), canon_edges(*o.export_used_by()))
    o.clear_log()
    o.invalidate_slots(mix.roots(99))
    ids = np.concatenate([r["last_ids"] for r in ranks])
    assert np.array_equal(np.sort(ids), np.sort(o.inv_log()))
    ov, of = o.dump_states()
    _states_match(ranks, "last", ov, of)
    o.close()
