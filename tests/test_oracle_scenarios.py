"""Known-answer scenarios that pin the CPU oracle to the reference's own behavioural tests.

The reference (C#) holds no numeric golden vectors for the cascade; its pins are the behaviour
tests listed in SURVEY.md §4 / §8(c). Each scenario below restates one of them over the slot
model (a slot = a compute-method input, a node = one Computed instance) and checks the oracle.
Each World-based scenario takes the world factory as a default argument, so
tests/test_gpu_scenarios.py replays the same function against the engine (through the C-ABI).
"""
import numpy as np
import pytest

import fgo as O

C, K, I = 0, 1, 2                     # Computing, Consistent, Invalidated
IOSO, DS, HD = 4, 8, 16
ADDED, DROPPED, USED_INV, ESTATE = 0, 1, 2, 3


class World:
    """A tiny compute-service world over the oracle: compute(slot, deps) = begin + AddUsed + set."""

    def __init__(self, n=64, make=O.Oracle):
        self.o = make(n)
        self.ver = {}
        self.next_v = 1000

    def begin(self, slot, delay=False):
        self.next_v += 7                  # LTagVersionGenerator: a fresh version != the old one
        h, displaced = self.o.begin_compute(slot, self.next_v, delay)
        self.ver[slot] = self.next_v
        return h, displaced

    def compute(self, slot, deps=(), delay=False):
        h, _ = self.begin(slot, delay)
        for d in deps:
            assert self.o.add_used(h, self.o.last(d)) == ADDED
        assert self.o.set_output(h) == 1
        return h

    def state(self, slot):
        return self.o.node_info(self.o.last(slot))[2]

    def invalidate(self, *slots, imm=None):
        self.o.clear_log()
        self.o.invalidate_slots(list(slots), imm)
        return sorted(self.o.inv_log().tolist())


def test_counter_service_basic(W=World):
    """CounterServiceTest.BasicTest (CounterServiceTest.cs:12-30): invalidation makes the computed
    inconsistent and removes it from the registry (GetExisting -> null)."""
    w = W()
    h = w.compute(0)
    assert w.o.current(0) == h and w.state(0) == K
    assert w.invalidate(0) == [0]
    assert w.state(0) == I and w.o.current(0) == O.NONE


def test_counter_service_long_wait(W=World):
    """CounterServiceTest.LongWaitTest (:32-58): invalidating a Computing node keeps it Computing
    and registered; once its output is set it becomes Invalidated and unregistered."""
    w = W()
    h, _ = w.begin(0)
    assert w.invalidate(0) == []
    assert w.o.current(0) == h and w.state(0) == C | IOSO
    assert w.o.set_output(h) == 1
    assert w.state(0) == I and w.o.current(0) == O.NONE


def test_counter_service_concurrent_wait(W=World):
    """CounterServiceTest.ConcurrentWaitTest (:60-98): a dependency that completes after the
    dependant is not recorded (AddUsed drops it, Computed.cs:351-364): Used.Length == 1."""
    w = W()
    x = w.compute(1)
    yh, _ = w.begin(2)                      # "y wait" still computing
    dh, _ = w.begin(3)                      # GetFirstNonZero(x, y)
    assert w.o.add_used(dh, x) == ADDED
    assert w.o.set_output(dh) == 1          # returns after x alone
    assert w.o.set_output(yh) == 1
    assert w.o.add_used(dh, yh) == DROPPED  # late completion: dropped
    assert w.o.used_count(dh) == 1
    # case 2: both used
    dh2 = w.compute(3, deps=[1, 2])
    assert w.o.used_count(dh2) == 2


def test_simplest_provider_cascade_and_new_version(W=World):
    """SimplestProviderTest.BasicTest (SimplestProviderTest.cs:9-32) + EdgeCaseServiceTest
    (EdgeCaseServiceTest.cs:52): SetValue invalidates GetValue, which cascades to GetCharCount;
    recomputation produces a new version."""
    w = W()
    w.compute(0)                  # GetValue
    w.compute(1, deps=[0])        # GetCharCount uses GetValue
    v0 = w.ver[1]
    assert w.invalidate(0) == [0, 1]
    w.compute(0)
    w.compute(1, deps=[0])
    assert w.ver[1] != v0 and w.state(1) == K


def test_mutable_state_two_dependants(W=World):
    """MutableStateTest.CounterServiceTest (MutableStateTest.cs:82-116): one root (the offset
    state) invalidates both Get("a") and Get("b")."""
    w = W()
    w.compute(0)
    w.compute(1, deps=[0])
    w.compute(2, deps=[0])
    assert w.invalidate(0) == [0, 1, 2]


def test_user_provider_invalidate_everything_hub(W=World):
    """UserProviderTest.InvalidateEverythingTest (UserProviderTest.cs:12-36): the Everything() hub
    (UserService.cs:178-179) invalidates every Get(id) and Count(); recomputed nodes are new."""
    w = W(200)
    w.compute(0)                                       # Everything()
    hs = [w.compute(s, deps=[0]) for s in range(1, 101)]   # Get(id) x100 + Count()
    assert w.invalidate(0) == list(range(0, 101))
    w.compute(0)                  # Get(id) awaits Everything() first: the hub is recomputed
    hs2 = [w.compute(s, deps=[0]) for s in range(1, 101)]
    assert all(a != b for a, b in zip(hs, hs2))


def test_nested_operation_multi_root_batch(W=World):
    """NestedOperationLoggerTest.BasicTest (Extensions/NestedOperationLoggerTest.cs:11-38): one
    Computed.Invalidate() scope with several roots invalidates all of them."""
    w = W()
    for s in (0, 1, 2):
        w.compute(s)
    assert w.invalidate(0, 1, 2) == [0, 1, 2]


def test_invalidation_delay_then_timer(W=World):
    """Computed.cs:186-198 + Timeouts.cs:22-28: a node with InvalidationDelay is only flagged
    (DelayStarted) by the cascade; the timer later calls Invalidate(true)."""
    w = W()
    w.compute(0)
    d = w.compute(1, deps=[0], delay=True)
    w.compute(2, deps=[1])
    assert w.invalidate(0) == [0]
    assert w.state(1) == K | DS | HD and w.state(2) == K
    assert w.invalidate(0) == []                       # already started: no-op
    w.o.clear_log()
    w.o.invalidate_nodes([d], [1])                     # timer fires
    assert sorted(w.o.inv_log().tolist()) == [1, 2]


def test_computing_immediately_quirk(W=World):
    """Computed.cs:175-176 / 187-188: Invalidate(true) on a Computing node with a delay sets both
    flags; after TrySetOutput the node stays Consistent (the delayed invalidation never runs)."""
    w = W()
    h, _ = w.begin(0, delay=True)
    w.o.invalidate_nodes([h], [1])
    assert w.state(0) == C | IOSO | DS | HD
    assert w.o.set_output(h) == 1
    assert w.state(0) == K | DS | HD
    assert w.invalidate(0) == [] and w.state(0) == K | DS | HD


def test_add_used_by_on_invalidated_and_computing(W=World):
    """Computed.cs:370-385: AddUsedBy on an Invalidated node invalidates the dependant (it gets
    InvalidateOnSetOutput while Computing); on a Computing node it throws."""
    w = W()
    u = w.compute(0)
    w.invalidate(0)
    dh, _ = w.begin(1)
    assert w.o.add_used(dh, u) == USED_INV
    assert w.state(1) == C | IOSO
    assert w.o.set_output(dh) == 1 and w.state(1) == I
    ch, _ = w.begin(2)
    eh, _ = w.begin(3)
    assert w.o.add_used(eh, ch) == ESTATE


def test_register_displacement(W=World):
    """ComputedRegistry.Register (ComputedRegistry.cs:83-97): a new computation of a slot
    invalidates the current Consistent node (cascading) before replacing it."""
    w = W()
    w.compute(0)
    w.compute(1, deps=[0])
    w.o.clear_log()
    h, displaced = w.begin(0)
    assert displaced != O.NONE and sorted(w.o.inv_log().tolist()) == [0, 1]
    assert w.o.current(0) == h and w.state(0) == C


def test_register_displacement_with_delay_detaches(W=World):
    """A displaced node with an InvalidationDelay is only flagged and dropped from the registry;
    its dependants stay Consistent until its timer fires."""
    w = W()
    w.compute(0, delay=True)
    w.compute(1, deps=[0])
    w.o.clear_log()
    h, displaced = w.begin(0)
    assert w.o.inv_log().tolist() == []
    assert w.o.node_info(displaced)[2] == K | DS | HD and w.state(1) == K
    w.o.clear_log()
    w.o.invalidate_nodes([displaced], [1])
    assert sorted(w.o.inv_log().tolist()) == [0, 1]
    assert w.state(0) == C        # the slot's current node is the new computation


def test_stale_edges_do_not_cascade(W=World):
    """Computed.cs:213-214: an entry whose version no longer matches is skipped."""
    w = W()
    w.compute(0)
    w.compute(1, deps=[0])
    w.compute(2)
    w.o.clear_log()
    h, _ = w.begin(1)             # recompute 1 (0's usedBy entry for 1 is now stale)
    w.o.add_used(h, w.o.last(2))
    w.o.set_output(h)
    assert w.invalidate(0) == [0]
    assert w.state(1) == K


def test_prune_used_by_drops_only_stale_entries(W=World):
    """PruneUsedBy (Computed.cs:400-419) keeps (input, version) entries whose computed is current."""
    w = W()
    w.compute(0)
    w.compute(1, deps=[0])
    w.compute(2, deps=[0])
    w.begin(1)                    # 1 displaced (invalidated) -> its entry in 0 is removed by RemoveUsedBy
    w.o.set_output(w.o.last(1))
    h2, _ = w.begin(2)            # 2 recomputed; entry for old 2 removed by RemoveUsedBy too
    assert len(w.o.used_by(w.o.last(0))[0]) == 0
    old, new = w.o.prune()
    assert new <= old


def test_hashsetslim3_set_semantics_and_spill(W=World):
    """HashSetSlim3 (HashSetSlim3.cs:31-95; HashSetSlimTest.cs:10-86): duplicates collapse, more
    than three entries spill to a hash set, removal works in both representations."""
    w = W(64)
    w.compute(0)
    hs = []
    for s in range(1, 11):
        h, _ = w.begin(s)
        assert w.o.add_used(h, w.o.last(0)) == ADDED
        assert w.o.add_used(h, w.o.last(0)) == ADDED   # duplicate: no second entry
        w.o.set_output(h)
        hs.append(h)
    d, t = w.o.used_by(w.o.last(0))
    assert sorted(d.tolist()) == list(range(1, 11)) and len(set(zip(d.tolist(), t.tolist()))) == 10
    w.invalidate(5)               # RemoveUsedBy(5) from the spilled set
    assert sorted(w.o.used_by(w.o.last(0))[0].tolist()) == [1, 2, 3, 4, 6, 7, 8, 9, 10]
    assert w.invalidate(0) == [0, 1, 2, 3, 4, 6, 7, 8, 9, 10]


def test_cycle_terminates(W=World):
    """AddUsed cannot close a cycle of current nodes (AddUsedBy throws on a Computing node), but
    imported graphs may hold one; the cascade still visits each node once."""
    w = W()
    a, _ = w.begin(0)
    b, _ = w.begin(1)
    w.o.set_output(b)
    assert w.o.add_used(a, b) == ADDED
    w.o.set_output(a)
    h, _ = w.begin(1)             # displacing b invalidates it and cascades to a
    assert w.state(0) == I
    n = 10
    ver = O.version_of(3, np.arange(n))
    o = O.Oracle(n)
    src = np.arange(n, dtype=np.uint32)
    dst = ((src + 1) % n).astype(np.uint32)
    o.load_graph(ver, None, src, dst, ver[dst])
    o.invalidate_slots([4])
    assert sorted(o.inv_log().tolist()) == list(range(n))


def test_parallel_over_roots_equals_sequential():
    rng = np.random.default_rng(5)
    n = 2000
    src = rng.integers(0, n, 20000).astype(np.uint32)
    dst = rng.integers(0, n, 20000).astype(np.uint32)
    ver = O.version_of(1, np.arange(n))
    tags = ver[dst]
    roots = rng.integers(0, n, 64).astype(np.uint32)
    res = []
    for th in (1, 4, 8):
        o = O.Oracle(n)
        o.load_graph(ver, None, src, dst, tags)
        st = o.invalidate_slots(roots, threads=th)
        res.append((sorted(o.inv_log().tolist()), st.e_trav, o.dump_states()[1].tolist()))
    assert res[0] == res[1] == res[2]


def test_generators_are_deterministic():
    s1, d1 = O.gen_rmat(10, 8, 0x5EED0024)
    s2, d2 = O.gen_rmat(10, 8, 0x5EED0024)
    assert np.array_equal(s1, s2) and np.array_equal(d1, d2)
    assert np.all(np.diff(s1.astype(np.int64) * (1 << 32) + d1) > 0)   # sorted, unique
    s, d = O.gen_layered(3, 100, 4, 1)
    assert len(s) == 2 * 100 * 4
    assert np.all(s // 100 + 1 == d // 100)                            # edges go one level up
    v = O.version_of(7, np.arange(1000))
    assert np.all(v & np.uint64(1)) and np.all(v < np.uint64(1 << 55))
