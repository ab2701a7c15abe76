"""Asynchronous waves (fgi_invalidate_async / fgi_wave_wait; ComputedExt.WhenInvalidated,
/root/reference/src/Stl.Fusion/ComputedExt.cs:99-125, awaited at Client/Internal/RpcInboundComputeCall.cs:53).

Waves are pipelined the way bench.py's pipelined leg runs them — the next wave queued before the
previous one is waited for, with fgi_restore between them — and every wave's invalidated ids (read
from its own device buffer while the next wave runs) and V_inv are checked against the oracle
(Computed.cs:162-230). Also: waves on an evolving graph (no restore, each wave sees the previous one's
effects), a synchronous call after queued waves (it waits for them first), immediate roots, and
labelled graphs (their ids fold back to slot order in each ticket's buffer)."""
import ctypes

import numpy as np
import pytest
import torch

import fgo as O
from harness import assert_states_equal

pytestmark = pytest.mark.gpu

_hip = None


def _d2h(ptr, n):
    """n uint32 from device memory (a completed wave's id buffer; another wave may still be running)."""
    global _hip
    if _hip is None:
        _hip = ctypes.CDLL("libamdhip64.so")
        _hip.hipMemcpy.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int]
    out = np.zeros(n, np.uint32)
    if n:
        assert _hip.hipMemcpy(out.ctypes.data, ctypes.c_void_p(ptr), 4 * n, 2) == 0   # hipMemcpyDeviceToHost
    return out


def _pair(pkg, scale, ef, seed, labels):
    n = 1 << scale
    g = pkg.Graph(n, labels=labels)
    g.synth_rmat(scale, ef, seed)
    s, d = O.gen_rmat(scale, ef, seed)
    o = O.Oracle(n)
    o.load_graph(O.version_of(seed, np.arange(n)), None, s, d, O.gen_tags(s, d, seed))
    return g, o, np.bincount(s, minlength=n)


@pytest.mark.parametrize("labels", [-1, 1])
def test_pipelined_waves_with_restore(pkg, gpu_available, labels):
    scale, ef, seed = 16, 16, 0x5EED0024
    n = 1 << scale
    g, o, deg = _pair(pkg, scale, ef, seed, labels)
    g.snapshot()
    o.snapshot()
    sets = [O.gen_roots(k, n, 0x5EED1024 + k, deg) for k in (256, 16, 1024)]
    want = []
    for r in sets:
        o.restore()
        o.clear_log()
        o.invalidate_slots(r)
        want.append(np.sort(o.inv_log()))
    d_sets = [torch.from_numpy(r.astype(np.int32)).cuda() for r in sets]
    torch.cuda.synchronize()
    prev = None
    seen = 0
    for k in range(9):
        g.restore()
        t = g.invalidate_async(len(sets[k % 3]), d_sets[k % 3].data_ptr())
        assert t == k + 1
        if prev is not None:
            st = pkg.WaveStats()
            nv, ptr = g.wave_wait(prev, st)
            w = want[(prev - 1) % 3]
            assert nv == len(w) == st.v_inv, (prev, nv, len(w))
            assert np.array_equal(_d2h(ptr, nv), w), prev
            seen += 1
        prev = t
    nv, ptr = g.wave_wait(prev)
    assert np.array_equal(_d2h(ptr, nv), want[(prev - 1) % 3])
    assert seen == 8
    # waiting again for a completed ticket returns its results again
    assert g.wave_wait(prev)[0] == nv
    g.close()
    o.close()


def test_async_waves_on_an_evolving_graph(pkg, gpu_available):
    """No restore: each wave runs on the state the previous ones left (the queue keeps their order);
    immediate roots; a synchronous wave and a state query after queued waves wait for them first."""
    scale, ef, seed = 15, 8, 0x5EED0027
    n = 1 << scale
    g, o, deg = _pair(pkg, scale, ef, seed, 1)
    tickets, want = [], []
    rng = np.random.default_rng(3)
    d_keep = []
    for k in range(4):
        r = O.gen_roots(8 + 8 * k, n, 77 + k, deg)
        imm = (rng.random(len(r)) < 0.3).astype(np.uint8)
        o.clear_log()
        st = o.invalidate_slots(r, imm)
        want.append((np.sort(o.inv_log()), st.v_inv))
        dr, di = torch.from_numpy(r.astype(np.int32)).cuda(), torch.from_numpy(imm).cuda()
        d_keep += [dr, di]
        torch.cuda.synchronize()
        tickets.append(g.invalidate_async(len(r), dr.data_ptr(), di.data_ptr()))
        if 1 <= k <= 2:   # the previous wave, while this one is queued
            nv, ptr = g.wave_wait(tickets[k - 1])
            assert nv == want[k - 1][1] and np.array_equal(_d2h(ptr, nv), want[k - 1][0]), k
    # waves 3 and 4 still in flight: the state query waits for them
    assert_states_equal(g, o, n)
    for t in tickets[2:]:   # waited for by the query; their results stay until two later waves
        nv, ptr = g.wave_wait(t)
        assert nv == want[t - 1][1] and np.array_equal(_d2h(ptr, nv), want[t - 1][0]), t
    r = O.gen_roots(64, n, 999, deg)
    o.clear_log()
    o.invalidate_slots(r)
    d_r = torch.from_numpy(r.astype(np.int32)).cuda()
    torch.cuda.synchronize()
    t = g.invalidate_async(len(r), d_r.data_ptr())
    ids = g.invalidate(O.gen_roots(4, n, 5, deg))   # synchronous: waits for ticket t first
    o_ids = np.sort(o.inv_log())
    o.clear_log()
    o.invalidate_slots(O.gen_roots(4, n, 5, deg))
    assert np.array_equal(ids, np.sort(o.inv_log()))
    assert g.wave_wait(t)[0] == len(o_ids)
    assert_states_equal(g, o, n)
    g.close()
    o.close()


def _layered_pair(pkg, levels, width, fanout, seed):
    n = levels * width
    g = pkg.Graph(n)
    g.synth_layered(levels, width, fanout, seed)
    s, d = O.gen_layered(levels, width, fanout, seed)
    o = O.Oracle(n)
    o.load_graph(O.version_of(seed, np.arange(n)), None, s, d, O.gen_tags(s, d, seed))
    return g, o, n


@pytest.mark.parametrize("mode", ["async", "sync"])
def test_wave_tail_timeout_poisons_until_restore(pkg, gpu_available, mode):
    """A wave whose tail (the persistent launch running its last small push levels) loses a block at a grid
    barrier (FGI_OPT_FAULT_INJECT_TAIL) is half applied: fgi_wave_wait (async) or fgi_invalidate (sync)
    returns FGI_EDEVICE, every later call FGI_ESTATE until fgi_restore, and the graph then runs the same
    waves as the oracle again — including a second tail, whose barrier word the failure path reset."""
    fgi = pkg.fgi
    levels, width, fanout, seed = 14, 64, 2, 0x5EED0031
    g, o, n = _layered_pair(pkg, levels, width, fanout, seed)
    # push only: every level after the first group is a small push level, which the tail runs (a pull level
    # would end a synchronous wave's tail before its first barrier)
    g.set_option(fgi.OPT_DIRECTION, 1)
    g.snapshot()
    o.snapshot()
    roots = np.arange(8, dtype=np.uint32)   # level 0: the wave runs every one of the 14 levels
    o.clear_log()
    o.invalidate_slots(roots)
    want = np.sort(o.inv_log())
    assert len(want) > 12 * 8
    o.restore()   # the oracle back at the snapshot: the states a restored graph must show
    d_r = torch.from_numpy(roots.astype(np.int32)).cuda()
    torch.cuda.synchronize()

    def wave():
        if mode == "async":
            t = g.invalidate_async(len(roots), d_r.data_ptr())
            nv, ptr = g.wave_wait(t)
            return _d2h(ptr, nv)
        return g.invalidate(roots)

    # a first wave teaches the engine the wave's depth: the next one runs its levels past the first
    # group in the tail (the async queue runs every level past its group there anyway)
    assert np.array_equal(wave(), want)
    g.restore()
    g.set_option(fgi.OPT_FAULT_INJECT_TAIL, 1)
    with pytest.raises(fgi.FgiError) as e:
        wave()
    assert e.value.status == fgi.EDEVICE, e.value
    for call in (lambda: g.get_state([0]), lambda: g.invalidate(roots), lambda: g.snapshot()):
        with pytest.raises(fgi.FgiError) as e2:
            call()
        assert e2.value.status == fgi.ESTATE
    g.restore()
    assert_states_equal(g, o, n)
    for _ in range(2):
        assert np.array_equal(wave(), want)
        g.restore()
    g.close()
    o.close()


def test_ticket_results_forgotten_once_their_buffer_is_rewritten(pkg, gpu_available):
    """A completed ticket's ids can be read again only while its buffer is its own: a synchronous wave (which
    lists its ids into the even tickets' buffer) makes a later wait on an even ticket fail with FGI_EINVAL
    instead of returning the other wave's ids."""
    fgi = pkg.fgi
    g, o, n = _layered_pair(pkg, 6, 256, 4, 0x5EED0032)
    roots = np.arange(16, dtype=np.uint32)
    d_r = torch.from_numpy(roots.astype(np.int32)).cuda()
    torch.cuda.synchronize()
    g.snapshot()
    t1 = g.invalidate_async(len(roots), d_r.data_ptr())
    g.wave_wait(t1)
    g.restore()
    t2 = g.invalidate_async(len(roots), d_r.data_ptr())
    n2 = g.wave_wait(t2)[0]
    assert g.wave_wait(t2)[0] == n2           # repeated wait: same results
    g.restore()
    g.invalidate(roots[:1])                   # writes the even tickets' buffer
    with pytest.raises(fgi.FgiError) as e:
        g.wave_wait(t2)
    assert e.value.status == fgi.EINVAL
    assert g.wave_wait(t1)[0] > 0             # odd ticket: its buffer was not touched
    g.close()
    o.close()


@pytest.mark.parametrize("labels", [-1, 1])
def test_async_host_roots_and_ids_match_oracle(pkg, gpu_available, labels):
    """fgi_invalidate_async_host / fgi_wave_wait_ids (the host layer's scope flush awaited later): roots and
    immediately flags from host memory, two waves in flight on an evolving graph, each wave's ids brought
    back to the host against the oracle (Computed.cs:162-230), node states after them."""
    scale, ef, seed = 14, 8, 0x5EED0033
    n = 1 << scale
    g, o, deg = _pair(pkg, scale, ef, seed, labels)
    rng = np.random.default_rng(11)
    tickets, want = [], []
    for k in range(5):
        r = O.gen_roots(4 + 12 * k, n, 300 + k, deg)
        imm = (rng.random(len(r)) < 0.25).astype(np.uint8)
        o.clear_log()
        st = o.invalidate_slots(r, imm)
        want.append((np.sort(o.inv_log()), st.v_inv))
        tickets.append(g.invalidate_async_host(r, imm))
        if k >= 1:   # the previous wave, while this one is in flight
            t = tickets[k - 1]
            ws = pkg.WaveStats()
            ids = g.wave_wait_ids(t, ws)
            assert ws.v_inv == want[k - 1][1] and np.array_equal(ids, want[k - 1][0]), k
    ids = g.wave_wait_ids(tickets[-1])
    assert np.array_equal(ids, want[-1][0])
    assert_states_equal(g, o, n)
    g.close()
    o.close()


def test_async_wave_reports_pull_levels_run_as_push(pkg, gpu_available):
    """A queued wave runs every level past its group in the tail as push levels: with pull-only waves on a
    14-level graph, the first queued wave's group (4 levels: nothing learnt yet) leaves 10 levels that would
    pull to the tail — counted in pull_pushed — and still matches the oracle; the next wave's group is sized
    from it (8 levels), so fewer are left.""" 
    fgi = pkg.fgi
    g, o, n = _layered_pair(pkg, 14, 256, 2, 0x5EED0034)
    g.set_option(fgi.OPT_DIRECTION, 2)
    g.snapshot()
    o.snapshot()
    roots = np.arange(32, dtype=np.uint32)
    o.clear_log()
    o.invalidate_slots(roots)
    want = np.sort(o.inv_log())
    pushed, levels = [], []
    for _ in range(2):
        g.restore()
        ws = pkg.WaveStats()
        ids = g.wave_wait_ids(g.invalidate_async_host(roots), ws)
        assert np.array_equal(ids, want)
        levels.append(ws.levels)   # levels with frontier entries (the last level's nodes have no rows)
        pushed.append(ws.pull_pushed)
    assert levels[0] == levels[1] >= 12, levels
    assert pushed == [levels[0] - 4, levels[0] - 8], (pushed, levels)
    g.close()
    o.close()
