"""N>1 path on the CPU: the partitioned wave's exchange protocol (tests/dist_model.py, the same
decomposition as stl.fusion_amd/csrc/part.hip) over a real torch.distributed gloo group at
world sizes 2 and 3 (ragged last partition), checked bit-exactly against the oracle: the union of
the per-rank invalidated sets and the owners' final state flags."""
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp

import fgo as O
from harness import random_states


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _case(seed, scale=9, ef=8, stale=30):
    rng = np.random.default_rng(seed)
    n = 1 << scale
    versions, flags = random_states(n, rng, seed=seed)
    s, d = O.gen_rmat(scale, ef, 0x5EED0000 + seed)
    live = (versions[s] != 0) & ((flags[s] & 3) == 1)      # only Consistent nodes hold `_usedBy`
    s, d = s[live], d[live]
    tags = versions[d].astype(np.uint64).copy()
    tags[tags == 0] = 7
    st = rng.random(len(s)) < stale / 100
    tags[st] += np.uint64(1)
    deg = np.bincount(s, minlength=n)
    roots = O.gen_roots(24, n, 0x5EED1000 + seed, deg)
    imm = (rng.random(len(roots)) < 0.25).astype(np.uint8)
    return n, versions, flags, s, d, tags, roots, imm


def _worker(rank, world, port, seed, direction, q):
    import torch.distributed as dist
    from dist_model import RankModel
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        n, versions, flags, s, d, tags, roots, imm = _case(seed)
        m = RankModel(rank, world, n, versions, flags, s, d, tags)
        levels = m.wave(roots, imm, direction=direction, alpha=6)
        inv, fl = m.gather_results()
        if rank == 0:
            q.put((inv, fl.tolist(), levels))
        dist.barrier()
    except Exception:
        import traceback
        q.put(("error", rank, traceback.format_exc()))
        raise
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
@pytest.mark.parametrize("direction", ["push", "pull", "auto"])
@pytest.mark.parametrize("seed", [1, 2])
def test_partitioned_protocol_matches_oracle(world, direction, seed):
    n, versions, flags, s, d, tags, roots, imm = _case(seed)
    o = O.Oracle(n)
    o.load_graph(versions, flags, s, d, tags)
    o.invalidate_slots(roots, imm)
    o_inv = sorted(int(x) for x in o.inv_log())
    _, o_flags = o.dump_states()
    o.close()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, seed, direction, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = q.get(timeout=120)
    assert res[0] != "error", res
    inv, fl, levels = res
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert len(o_inv) > 10 and levels >= 2
    assert inv == o_inv
    assert np.array_equal(np.asarray(fl, np.uint32)[:n], o_flags[:n])
