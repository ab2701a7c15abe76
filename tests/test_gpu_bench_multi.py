"""bench.py's N > 1 path on a one-GPU box: two ranks launched by
torch.distributed.run share the GPU, so the engine's collectives go through the host (gloo,
fgi_part_init_host) — the same run_part_wave, planned waves and bench bookkeeping an 8-GPU RCCL run
executes. The line must carry the N = 2 record with the invalidated-node count of the single engine on
the same graph and roots (Computed.cs:162-230 cascade, checked here against the single-device engine,
itself oracle-pinned). A rank that dies before its first wave makes the other fail within the bounded
waits: non-zero exit, the rank and the failing collective named, no hang."""
import json
import os
import socket
import subprocess
import sys

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SCALE = 16


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _bench(P, extra_env=None, timeout=110):
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={P}",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()),
           os.path.join(ROOT, "bench.py"), "--gpus", str(P), "--steps", "3", "--warmup", "1", "--no-cpu",
           "--no-e2e", "--no-secondary", "--scale", str(SCALE)]
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    env["OMP_NUM_THREADS"] = "2"
    env.update(extra_env or {})
    return subprocess.run(cmd, capture_output=True, text=True, timeout=timeout, env=env, cwd=ROOT)


def test_bench_two_ranks_host_collectives(pkg, gpu_available):
    from stl_fusion_amd import workloads as W
    r = _bench(2)
    assert r.returncode == 0, r.stderr[-3000:]
    line = [x for x in r.stdout.splitlines() if x.startswith("{")]
    assert len(line) == 1, r.stdout[-2000:]
    d = json.loads(line[0])
    assert d["n_gpus"] == 2 and d["scaling"] == "strong" and "x2 (host (gloo) collectives)" in d["config"]["parallelism"]
    assert d["config"]["scale"] == SCALE and d["config"]["edge_factor"] == 8
    # the single engine on the same graph (configs[2]'s generator at SCALE) and the bench's roots
    cfg = dict(W.CONFIGS["rmat27"])
    cfg["scale"] = SCALE
    n = W.n_slots(cfg)
    g = pkg.Graph(n)
    W.build(g, cfg)
    roots = W.roots_for(g, cfg)
    ws = pkg.WaveStats()
    ids = g.invalidate(roots, stats=ws)
    g.close()
    assert d["v_inv_per_step"] == len(ids) == ws.v_inv
    assert d["e_trav_per_step"] == ws.e_trav
    assert d["value"] > 0 and d["ms_per_step"] > 0


def test_bench_rank_lost_fails_fast(gpu_available):
    r = _bench(2, {"FGI_BENCH_DROP_RANK": "1", "FGI_BENCH_TIMEOUT_S": "20", "FGI_WAIT_TIMEOUT_S": "20"}, timeout=100)
    assert r.returncode != 0
    err = r.stderr
    assert "[rank 0 of 2] bench failed" in err, err[-3000:]
    assert "rank 0 of 2" in err and ("all-gather" in err or "barrier" in err.lower()), err[-3000:]
