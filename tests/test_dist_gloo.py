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


def _delayed_displacement(versions, flags, s, d, tags):
    """A batch that recomputes a Consistent delayed node u holding a live entry of a Consistent
    undelayed dependant: the old u is detached (ComputedRegistry.cs:91-96 only starts its delay), so
    invalidating the new u must not reach the dependant — also not through a pull level, whose
    dependency lists named u by its slot."""
    st = flags & 3
    ok = ((st[s] == 1) & ((flags[s] & 16) != 0) & (versions[s] != 0) & (st[d] == 1) & ((flags[d] & 16) == 0) &
          (tags == versions[d]))
    k = np.nonzero(ok)[0]
    assert len(k), "no delayed node with a live undelayed dependant in this case"
    u = int(s[k[0]])
    return [("begin_compute", np.array([u]), np.array([(1 << 45) | 1], np.uint64), np.zeros(1, np.uint8)),
            ("set_output", np.array([u])), ("invalidate", np.array([u]), None)]


def _churn(seed, n, versions, flags, n_batches=5, first=None):
    """Random batches for the mutation protocol: (kind, args) lists, same on every rank."""
    rng = np.random.default_rng(seed + 99)
    present = versions != 0
    nv = (1 << 40) | 1
    batches = [first] if first else []
    for b in range(n_batches):
        inv = rng.choice(n, 12, replace=False)
        bc = rng.choice(n, 24, replace=False)
        ver = np.arange(nv, nv + 2 * len(bc), 2, dtype=np.uint64)
        nv += 2 * len(bc)
        hd = (rng.random(len(bc)) < 0.25).astype(np.uint8)
        present[bc] = True
        pool = np.nonzero(present)[0]
        dep = np.concatenate([rng.choice(bc, 40), rng.choice(pool, 16)])
        use = rng.choice(pool, len(dep))
        so = bc[rng.random(len(bc)) < 0.7]
        batches.append([("invalidate", inv, (rng.random(len(inv)) < 0.5).astype(np.uint8)),
                        ("begin_compute", bc, ver, hd), ("add_used", dep, use), ("set_output", so),
                        ("invalidate", rng.choice(n, 6, replace=False), None)])
    return batches


def _mut_worker(rank, world, port, seed, direction, q):
    import torch.distributed as dist
    import dist_model as DM
    import torch
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        n, versions, flags, s, d, tags, roots, imm = _case(seed)
        m = DM.RankModel(rank, world, n, versions, flags, s, d, tags)
        out = []
        for batch in _churn(seed, n, versions.copy(), flags, first=_delayed_displacement(versions, flags, s, d, tags)):
            before = len(m.inv)
            res = []
            for sp in batch:
                if sp[0] == "invalidate":
                    m.wave([int(x) for x in sp[1]], sp[2], direction=direction, alpha=6)
                    res.append(None)
                elif sp[0] == "begin_compute":
                    DM.begin_compute(m, sp[1], sp[2], sp[3], direction=direction)
                    res.append(None)
                elif sp[0] == "add_used":
                    res.append(DM.add_used(m, sp[1], sp[2]).tolist())
                else:
                    res.append(DM.set_output(m, sp[1], direction=direction))
            mine = [None] * world
            dist.all_gather_object(mine, sorted(m.inv[before:]))
            out.append((sorted(x for p in mine for x in p), res))
        left = torch.tensor([DM.prune(m)], dtype=torch.int64)
        dist.all_reduce(left)
        rows = [None] * world
        dist.all_gather_object(rows, DM.live_rows(m))
        vers = [None] * world
        dist.all_gather_object(vers, m.ver.tolist())
        inv, fl = m.gather_results()
        if rank == 0:
            q.put((out, int(left[0]), sorted(r for p in rows for r in p), [v for p in vers for v in p], fl.tolist()))
        dist.barrier()
    except Exception:
        import traceback
        q.put(("error", rank, traceback.format_exc()))
        raise
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
@pytest.mark.parametrize("direction", ["push", "pull"])
def test_partitioned_mutation_protocol_matches_oracle(world, direction):
    """The mutation protocol of the partitioned engine (graph.hip part_*: begin_compute with
    displacement, AddUsed's two all-reduces, TrySetOutput's cascade, a partitioned prune) over a gloo
    group, against the oracle applying the same calls one by one: per batch the invalidated multiset,
    AddUsed codes and set counts; at the end every version and flag and the pruned rows."""
    seed = 5
    n, versions, flags, s, d, tags, roots, imm = _case(seed)
    batches = _churn(seed, n, versions.copy(), flags, first=_delayed_displacement(versions, flags, s, d, tags))
    o = O.Oracle(n)
    o.load_graph(versions, flags, s, d, tags)
    want = []
    for batch in batches:
        o.clear_log()
        res = []
        for sp in batch:
            if sp[0] == "invalidate":
                o.invalidate_slots(sp[1], sp[2])
                res.append(None)
            elif sp[0] == "begin_compute":
                o.begin_compute_slots(sp[1], sp[2], sp[3])
                res.append(None)
            elif sp[0] == "add_used":
                res.append(o.add_used_slots(sp[1], sp[2]).tolist())
            else:
                res.append(o.set_output_slots(sp[1]))
        want.append((sorted(int(x) for x in o.inv_log()), res))
    _, ne = o.prune()
    ov, of = o.dump_states()
    us, ud, ut = o.export_used_by()
    live = (ov[us] != 0) & ((of[us] & 3) != 2)
    o_rows = sorted((int(a), int(b), int(c)) for a, b, c in zip(us[live], ud[live], ut[live]))
    o.close()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_mut_worker, args=(r, world, port, seed, direction, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = q.get(timeout=180)
    assert res[0] != "error", res
    out, left, rows, vers, fl = res
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    codes = set()
    for b, ((inv, r), (winv, wr)) in enumerate(zip(out, want)):
        assert inv == winv, (b, len(inv), len(winv))
        assert r == wr, b
        for x in r:
            if isinstance(x, list):
                codes |= set(x)
    assert codes >= {0, 1, 2, 3}, codes
    assert np.array_equal(np.asarray(vers, np.uint64)[:n], ov)
    assert np.array_equal(np.asarray(fl, np.uint32)[:n], of)
    assert rows == o_rows and left == ne, (left, ne, len(rows), len(o_rows))


def _plan_worker(rank, world, port, seed, plan, C, q):
    import torch.distributed as dist
    import dist_model as DM
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        n, versions, flags, s, d, tags, roots, imm = _case(seed)
        m = DM.RankModel(rank, world, n, versions, flags, s, d, tags)
        levels, rounds = DM.planned_wave(m, roots, plan, C, imm)
        inv, fl = m.gather_results()
        if rank == 0:
            q.put((inv, fl.tolist(), levels, rounds))
        dist.barrier()
    except Exception:
        import traceback
        q.put(("error", rank, traceback.format_exc()))
        raise
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
@pytest.mark.parametrize("plan,C", [((0, 1, 1, 0), 1000), ((0, 0, 0), 3), ((1, 1), 17), ((), 5)])
def test_planned_wave_protocol_matches_oracle(world, plan, C):
    """The planned partitioned wave (run_part_planned: the previous wave's directions, full bitmap
    all-gathers before pull levels, fixed-size all-to-all buckets with carry-over after push levels, push
    levels appended while ids wait, one closing all-reduce per round) over a gloo group: whatever the
    plan and however small the buckets, the invalidated set and final flags equal the oracle's."""
    seed = 3
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
    procs = [ctx.Process(target=_plan_worker, args=(r, world, port, seed, list(plan), C, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = q.get(timeout=180)
    assert res[0] != "error", res
    inv, fl, levels, rounds = res
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert inv == o_inv
    assert np.array_equal(np.asarray(fl, np.uint32)[:n], o_flags[:n])
    if C <= 5:
        assert rounds > 1   # small buckets: ids wait for appended push levels
