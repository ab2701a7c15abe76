"""fgi_run_batch (streaming batches) against the oracle.

(a) The streaming mix (BASELINE.json configs[4], workloads.StreamMix) with one batch per round:
    timers (Invalidate(true)) -> begin_compute(hubs) -> set_output(hubs) -> begin_compute(leaves) ->
    add_used(leaves -> hubs) -> set_output(leaves) -> the round's hub wave, checked round by round
    (every node word, every cascade's ids) against the oracle applying the same calls one by one.
(b) Every behaviour scenario of tests/test_oracle_scenarios.py with each engine call made as a
    one-step batch (displacement and InvalidateOnSetOutput cascades included).
(c) A batch whose add_used step outgrows the pool headroom (the call grows the pool and resumes).
(d) A batch that runs out of detached handles: FGI_ECAPACITY, the steps before it applied.
(e) A batch with a bad argument in any step (a slot repeated in one begin_compute step, a slot or a
    handle out of range, a bad version): FGI_EINVAL, nothing applied.
"""
import functools

import numpy as np
import pytest

import fgo as O
import test_oracle_scenarios as S
from harness import assert_states_equal, build_pair
from test_gpu_scenarios import SCENARIOS, EngineOracle
from test_gpu_stream import _mix, _oracle_round

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("hubs,leaves,k,delay_pct", [(40, 30, 4, 10), (64, 200, 8, 5), (7, 1, 7, 50)])
def test_stream_mix_batches_match_oracle(pkg, gpu_available, hubs, leaves, k, delay_pct):
    mix = _mix(pkg, hubs, leaves, k, delay_pct, 0x5EED00E0)
    n = mix.n
    used, dep, tag = mix.initial_edges()
    g, o = build_pair(pkg, n, mix.version.copy(), mix.state_flags(), used, dep, tag)
    prev = np.zeros(0, np.uint32)
    for r in range(8):
        timers, hs, ls = mix.plan(prev)
        vh = mix.new_versions(hs).copy()
        vl = mix.new_versions(ls).copy()
        t_oracle = _oracle_round(o, mix, timers, hs, ls, vh, vl)
        roots = mix.roots(r)
        o.clear_log()
        o.invalidate_slots(roots)
        w_oracle = o.inv_log()
        steps = []
        if len(timers):
            steps.append(("invalidate", timers, np.ones(len(timers), np.uint8)))
        steps += [("begin_compute", hs, vh), ("set_output", hs), ("begin_compute", ls, vl, mix.has_delay[ls]),
                  ("add_used", ls, mix.hub_of(ls)), ("set_output", ls), ("invalidate", roots)]
        st = pkg.fgi.BatchStats()
        ids, outs = g.run_batch(steps, stats=st)
        assert st.host_syncs <= 2, st.as_dict()
        res = outs[-3]
        assert np.all(res == pkg.fgi.USED_ADDED)
        assert np.all(outs[-2] == 1)
        # cascades in step order: timers, (empty displacement / IOSO cascades), the hub wave
        want = np.concatenate([np.sort(t_oracle), np.sort(w_oracle)]).astype(np.uint32)
        assert np.array_equal(ids, want), f"round {r}"
        assert st.v_inv == len(want)
        assert_states_equal(g, o, n)
        prev = roots
    g.close()
    o.close()


class BatchEngineOracle(EngineOracle):
    """EngineOracle whose engine calls are one-step batches."""

    def begin_compute(self, slot, version, has_delay=False, stats=None):
        old = self.slot_last.get(slot)
        ids, outs = self.g.run_batch([("begin_compute", [slot], [version], [int(has_delay)])])
        self._log(ids)
        det = int(outs[0][0])
        if old is not None and det != O.NONE:
            self.nodes[old][3] = det
            self.home[det] = slot
        self.nodes.append([slot, version, bool(has_delay), slot])
        nid = len(self.nodes) - 1
        self.slot_last[slot] = nid
        return nid, (old if old is not None else O.NONE)

    def set_output(self, h, stats=None):
        ids, outs = self.g.run_batch([("set_output", [self.nodes[h][3]])])
        self._log(ids)
        return int(outs[0][0])

    def add_used(self, dependant_h, used_h):
        _, outs = self.g.run_batch([("add_used", [self.nodes[dependant_h][3]], [self.nodes[used_h][3]])])
        return int(outs[0][0])

    def invalidate_slots(self, slots, immediately=None, threads=1, stats=None):
        self._log(self.g.run_batch([("invalidate", slots, immediately)])[0])

    def invalidate_nodes(self, handles, immediately=None, stats=None):
        self._log(self.g.run_batch([("invalidate", [self.nodes[h][3] for h in handles], immediately)])[0])


@pytest.mark.parametrize("scenario", SCENARIOS, ids=[f.__name__[5:] for f in SCENARIOS])
def test_scenarios_as_batches(pkg, gpu_available, scenario):
    scenario(W=functools.partial(S.World, make=lambda n: BatchEngineOracle(pkg, n)))


def test_batch_grows_the_pool(pkg, gpu_available):
    """Used node 0 holds 3M entries in a full row; one batch adds a dependant to it, which needs a
    relocation larger than the call's headroom: the batch grows the pool, finishes the step and
    the remaining steps, with the same result as the single calls."""
    n = 3_000_010
    ver = O.version_of(11, np.arange(n))
    flags = np.full(n, 1, np.uint32)
    src = np.zeros(n - 10, np.uint32)
    dst = np.arange(10, n, dtype=np.uint32)
    states = []
    for use_batch in (False, True):
        g = pkg.Graph(n, n_detached=16)
        g.register_nodes(np.arange(n, dtype=np.uint32), ver, flags)
        g.load_edges(src, dst, ver[dst])
        if use_batch:
            st = pkg.fgi.BatchStats()
            ids, outs = g.run_batch([("begin_compute", [5], [ver[5] + 2]), ("add_used", [5], [0]),
                                     ("set_output", [5]), ("invalidate", [0])], stats=st)
            assert st.host_syncs >= 2
            assert outs[1][0] == pkg.fgi.USED_ADDED
            assert ids[0] == 5                       # the displacement cascade of step 0
            ids = ids[1:]                            # the last step's wave
        else:
            g.begin_compute([5], [ver[5] + 2])
            assert g.add_used([5], [0])[0] == pkg.fgi.USED_ADDED
            g.set_output([5])
            ids = g.invalidate([0])
        states.append((np.sort(ids), g.dump_states()))
        g.close()
    assert np.array_equal(states[0][0], states[1][0]) and len(states[0][0]) == n - 10 + 2
    assert np.array_equal(states[0][1][0], states[1][1][0]) and np.array_equal(states[0][1][1], states[1][1][1])


def test_batch_out_of_detached_handles(pkg, gpu_available):
    g = pkg.Graph(8, n_detached=1)
    g.register_nodes(np.arange(8, dtype=np.uint32), np.arange(8, dtype=np.uint64) * 2 + 1,
                     np.zeros(8, np.uint32))   # all Computing: a new computation detaches them
    with pytest.raises(pkg.fgi.FgiError) as e:
        g.run_batch([("set_output", [7]), ("begin_compute", [0, 1], [101, 103])])
    assert e.value.status == 3
    v, f = g.get_state([7, 0, 1])
    assert (f[0] & 3) == 1                  # step 0 applied
    assert (f[1] & 3) == 0 and v[1] == 1    # step 1 not
    g.close()


@pytest.mark.parametrize("bad", ["repeat", "slot_range", "version0", "version_big", "used_range", "dep_range"])
def test_batch_bad_argument_applies_nothing(pkg, gpu_available, bad):
    rng = np.random.default_rng(61)
    n = 2000
    from harness import random_states
    from test_gpu_parity import _edges_from_live
    versions, flags = random_states(n, rng, p_delay=0.0)
    src, dst, tags = _edges_from_live(versions, flags, rng, 8000, n, stale_p=0.2)
    g, o = build_pair(pkg, n, versions, flags, src, dst, tags)
    before = g.dump_states()
    edges = g.export_edges()
    slots = rng.choice(n, 500, replace=False).astype(np.uint32)
    ver = (versions[slots] + np.uint64(5)).astype(np.uint64)
    dep = slots[:300].copy()
    use = rng.integers(0, n, 300).astype(np.uint32)
    if bad == "repeat":
        slots[400] = slots[17]
    elif bad == "slot_range":
        slots[250] = n + 3
    elif bad == "version0":
        ver[99] = 0
    elif bad == "version_big":
        ver[499] = np.uint64(1) << np.uint64(60)
    elif bad == "used_range":
        use[123] = g.n_handles
    elif bad == "dep_range":
        dep[299] = g.n_handles + 7
    steps = [("invalidate", rng.integers(0, n, 20).astype(np.uint32)),
             ("begin_compute", slots, ver),
             ("add_used", dep, use),
             ("set_output", slots[:100])]
    with pytest.raises(pkg.FgiError) as e:
        g.run_batch(steps)
    assert e.value.status == pkg.fgi.EINVAL
    after = g.dump_states()
    assert all(np.array_equal(a, b) for a, b in zip(before, after))
    assert all(np.array_equal(a, b) for a, b in zip(edges, g.export_edges()))
    # the graph still takes a good batch (the scratch the checks used is clean again)
    slots2 = np.unique(slots[slots < n])[:200].astype(np.uint32)
    g.run_batch([("begin_compute", slots2, (versions[slots2] + np.uint64(9)).astype(np.uint64))])
    g.close()
    o.close()


@pytest.mark.parametrize("skip,block", [(1, 1), (1, 128), (0, 7)])
def test_batch_barrier_timeout_poisons_until_restore(pkg, gpu_available, skip, block):
    """A cascade whose grid barrier times out (FGI_OPT_FAULT_INJECT: one block leaves without arriving)
    fails the batch with FGI_EDEVICE; the graph then refuses every call with FGI_ESTATE until
    fgi_restore, after which the same batch (detached handles included) matches the oracle, and so
    does a second one. skip = 1: the fault is in the batch's second cascade (the first, a displacement
    cascade, has completed and detached the delayed leaves it displaced). The invalidated hubs and the
    displaced leaves lie in disjoint parts of the graph, so the step order does not change the result."""
    fgi = pkg.fgi
    mix = _mix(pkg, 48, 120, 6, 20, 0x5EED00E0)
    n = mix.n
    used, dep, tag = mix.initial_edges()
    g, o = build_pair(pkg, n, mix.version.copy(), mix.state_flags(), used, dep, tag, n_detached=512)
    g.snapshot()
    hubs = mix.roots(0)
    leaves = mix.children(hubs[:2])
    delayed = leaves[mix.has_delay[leaves] != 0]
    assert len(delayed) > 0
    vd = (mix.version[delayed] + np.uint64(2)).astype(np.uint64)
    roots = hubs[2:]
    bc = ("begin_compute", delayed, vd, np.ones(len(delayed), np.uint8))   # displaced + detached
    # skip = 0: the fault hits the batch's first cascade, which must have roots on the host's side (a
    # displacement cascade of delayed nodes has none: they only start their delay, without a launch)
    steps = [bc, ("invalidate", roots)] if skip else [("invalidate", roots), bc]
    steps.append(("set_output", delayed))
    i_bc = 0 if skip else 1
    g.set_option(fgi.OPT_FAULT_INJECT, (skip << 16) | block)
    with pytest.raises(fgi.FgiError) as e:
        g.run_batch(steps)
    assert e.value.status == fgi.EDEVICE, e.value
    for call in (lambda: g.get_state([0]), lambda: g.dump_states(), lambda: g.invalidate(roots),
                 lambda: g.run_batch([("invalidate", roots)]), lambda: g.prune(), lambda: g.snapshot()):
        with pytest.raises(fgi.FgiError) as e2:
            call()
        assert e2.value.status == fgi.ESTATE
    g.restore()
    assert_states_equal(g, o, n)            # the snapshot's states again
    ids, outs = g.run_batch(steps)
    o.clear_log()
    for s_, v in zip(delayed, vd):
        o.begin_compute(int(s_), int(v), True)
    disp = o.inv_log()
    assert len(disp) == 0                   # displaced delayed nodes only start their delay
    o.invalidate_slots(roots)
    w = o.inv_log()
    for s_ in delayed:
        assert o.set_output(o.last(int(s_))) == 1
    assert np.array_equal(ids, np.sort(w).astype(np.uint32))
    assert np.all(outs[i_bc] != fgi.NONE)   # every displaced delayed leaf was detached
    assert np.all(outs[2] == 1)
    assert_states_equal(g, o, n)
    # a second batch on the recovered graph
    r2 = mix.roots(1)
    ids2, _ = g.run_batch([("invalidate", r2)])
    o.clear_log()
    o.invalidate_slots(r2)
    assert np.array_equal(ids2, np.sort(o.inv_log()).astype(np.uint32))
    assert_states_equal(g, o, n)
    g.close()
    o.close()


def test_restore_without_snapshot_keeps_the_graph_poisoned(pkg, gpu_available):
    fgi = pkg.fgi
    mix = _mix(pkg, 8, 50, 2, 0, 0x5EED00E0)
    used, dep, tag = mix.initial_edges()
    g, o = build_pair(pkg, mix.n, mix.version.copy(), mix.state_flags(), used, dep, tag)
    o.close()
    g.set_option(fgi.OPT_FAULT_INJECT, 1)
    with pytest.raises(fgi.FgiError) as e:
        g.run_batch([("invalidate", mix.roots(0))])
    assert e.value.status == fgi.EDEVICE
    with pytest.raises(fgi.FgiError) as e:
        g.restore()
    assert e.value.status == fgi.ESTATE
    with pytest.raises(fgi.FgiError) as e:
        g.invalidate(mix.roots(0))
    assert e.value.status == fgi.ESTATE
    g.close()
