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


def test_counter_service_concurrent_wait_error(W=World):
    """CounterServiceTest.ConcurrentWaitTest case 3 (:87-97): the first dependency ("x fail")
    completes with an error, so GetFirstNonZero returns (with that error) before "y wait" completes:
    the error result is a recorded dependency, the late one is dropped (Used.Length == 1), and
    invalidating the failing dependency invalidates the dependant like any other output."""
    w = W()
    xf = w.compute(4)                       # Get("x fail"): an error output is still an output
    yh, _ = w.begin(5)                      # Get("y wait"): still computing
    dh, _ = w.begin(6)                      # GetFirstNonZero("x fail", "y wait")
    assert w.o.add_used(dh, xf) == ADDED
    assert w.o.set_output(dh) == 1          # completes with x fail's error
    assert w.o.set_output(yh) == 1
    assert w.o.add_used(dh, yh) == DROPPED
    assert w.o.used_count(dh) == 1
    assert w.invalidate(4) == [4, 6]        # Set("x fail", 0) invalidates Get and the dependant
    assert w.state(5) == K


def test_anonymous_computed_basic(W=World):
    """AnonymousComputedTest.BasicTest (AnonymousComputedTest.cs:9-36): an AnonymousComputedSource
    has no computed until first used; Use() computes once (value 1) and keeps returning the cached
    node while it is Consistent; ci.Computed.Invalidate() makes the next Use() compute value 2."""
    w = W()
    made = []
    val = {}

    def use():
        h = w.o.current(0)
        if h == O.NONE:
            h = w.compute(0)
            made.append(h)
            val[h] = len(made)
        return val[h]

    assert w.o.last(0) == O.NONE                     # IsComputed == false
    assert use() == 1 and use() == 1 and len(made) == 1
    h = w.o.last(0)
    assert w.state(0) == K
    w.o.clear_log()
    w.o.invalidate_nodes([h], [0])                   # ci.Computed.Invalidate()
    assert w.o.inv_log().tolist() == [0] and w.state(0) == I
    assert use() == 2 and use() == 2 and len(made) == 2


def test_anonymous_computed_auto_invalidation(W=World):
    """AnonymousComputedTest.ComputedOptionsTest (:38-60): AutoInvalidationDelay = 0.2 s. Each new
    output schedules Invalidate(true) on the timer set (StartAutoInvalidation, Computed.cs:235-246;
    ComputedExt.cs:10-24; Timeouts.cs:22-28); a firing invalidates the node (and anything that used
    it) and the next Use() computes a new value. Changes().Take(3) sees three firings, after which
    Use() returns a value > 3. A timer that fires after the node was already invalidated is a no-op."""
    w = W()
    val = {}
    n = 0

    def use():
        nonlocal n
        h = w.o.current(0)
        if h == O.NONE:
            n += 1
            h = w.compute(0)
            val[h] = n
        return val[h]

    assert use() == 1
    reader = w.compute(1, deps=[0])                  # a computed observing the source
    for k in range(3):                               # three timer rounds
        h = w.o.last(0)
        w.o.clear_log()
        w.o.invalidate_nodes([h], [1])               # the auto-invalidation timer fires
        assert sorted(w.o.inv_log().tolist()) == ([0, 1] if k == 0 else [0])
        w.o.clear_log()
        w.o.invalidate_nodes([h], [1])               # a second firing: already invalidated
        assert w.o.inv_log().tolist() == []
        assert use() == k + 2
    assert use() > 3
    assert w.o.node_info(reader)[2] == I


def test_computed_concurrency_counter_sum(W=World, iterations=120):
    """ConcurrencyTest.ComputedConcurrencyTest (ConcurrencyTest.cs:143-223) over CounterSumService
    (tests/Stl.Fusion.Tests/Services/CounterSumService.cs): Sum(0, 1) = Get0(0) + Get1(1), where
    Get1 has InvalidationDelay = 0.2 s. Readers — Computed.Capture(Sum) and an
    AnonymousComputedSource over Sum — follow the changes while a mutator sets one counter
    `iterations` times; the update delayer (ZeroUnsafe / Instant / 0.1 s) sets how often the readers
    catch up, and every `delay_frequency` mutations the delay timers get to fire. After the final
    wait (500 ms > the 0.2 s delay) every reader sees the registry's Sum node, with value
    2 * iterations.

    Slot model: counters c0, c1 are MutableStates (a set = invalidate the state's node + a new
    node); Get0(0), Get1(1), Sum and the reader sources are compute methods. Along the way:
    a Consistent Get0 always holds the current counter value; a Consistent Get1 without
    DelayStarted does too; a counter change reaches Get1 only as DelayStarted (Computed.cs:186-198),
    so Sum stays Consistent with the old value until the timer's Invalidate(true)."""
    C0, C1, G0, G1, S = 0, 1, 2, 3, 4
    R = 4                                         # HardwareInfo.GetProcessorCountFactor() readers
    SRC = list(range(5, 5 + R))
    deps = {G0: [C0], G1: [C1], S: [G0, G1], **{r: [S] for r in SRC}}
    for delayer, readers_every in (("zero", 1), ("instant", 2), ("0.1s", 7)):
        for delay_frequency in (50, 1000):
            w = W(32)
            val, cv = {}, [0, 0]
            pending = set()
            fired = [0]

            def set_counter(i, v):
                if w.o.last(i) != O.NONE:
                    w.invalidate(i)
                h = w.compute(i)
                val[h] = v
                cv[i] = v
                track_timers()

            def track_timers():
                h = w.o.last(G1)
                if h != O.NONE:
                    st = w.o.node_info(h)[2]
                    if st & 3 == K and st & DS:
                        pending.add(h)

            def fire_timers():
                for h in sorted(pending):
                    w.o.invalidate_nodes([h], [1])   # Timeouts: t.Invalidate(true)
                    fired[0] += 1
                pending.clear()

            def use(slot):
                h = w.o.current(slot)
                if h != O.NONE and w.o.node_info(h)[2] & 3 == K:
                    return val[h]
                if slot in (C0, C1):
                    return val[w.o.last(slot)]
                vals = [use(d) for d in deps[slot]]
                h = w.compute(slot, deps=deps[slot], delay=(slot == G1))
                val[h] = vals[0] if slot in (G0, G1) or slot in SRC else vals[0] + vals[1]
                return val[h]

            def check_invariants():
                for slot, ci in ((G0, 0), (G1, 1)):
                    h = w.o.last(slot)
                    st = w.o.node_info(h)[2]
                    if st & 3 == K and not (st & DS):
                        assert val[h] == cv[ci], (delayer, slot, val[h], cv[ci])
                hs = w.o.last(S)
                if w.o.node_info(hs)[2] & 3 == K:
                    assert val[hs] in (cv[0] + cv[1], val[w.o.last(G0)] + val[w.o.last(G1)])

            set_counter(C0, 0)
            set_counter(C1, 0)
            for r in SRC:
                use(r)
            for used in (0, 1):
                for i in (0, 1):
                    set_counter(i, iterations)
                set_counter(used, 0)
                for k in range(1, iterations + 1):          # Mutator
                    set_counter(used, k)
                    if k % readers_every == 0:
                        for r in SRC:
                            use(r)
                        check_invariants()
                    if k % delay_frequency == 0:            # await Task.Delay(1)
                        fire_timers()
                assert cv[used] == iterations
                fire_timers()                               # await Task.Delay(500)
                expected = 2 * iterations
                assert use(S) == expected, delayer
                s_node = w.o.current(S)
                for r in SRC:                               # every reader: same Sum node, value
                    assert use(r) == expected
                    assert w.o.current(S) == s_node
                check_invariants()
            assert fired[0] >= 1, delayer                   # Get1's delay was exercised


def test_invalidated_handler_set():
    """InvalidatedHandlerSetTest (Internal/InvalidatedHandlerSetTest.cs:10-48) over the fan-out
    model the host mirror implements (InvalidatedHandlerSet.cs: a single item, then a 5-slot
    array, then a hash set; Add is idempotent per handler; Remove keeps the order of the rest):
    for sizes 0..9 and removal probabilities (k + 1) / 200, Invoke calls every remaining handler
    exactly once and never a removed one."""
    rng = np.random.default_rng(0x1A5E7)
    for iteration in range(200):
        p = (iteration + 1.0) / 200
        for size in range(10):
            used = []
            hs = HandlerSet()
            handlers = [(lambda i: (lambda: used.append(i)))(i) for i in range(size)]
            for h in handlers:
                hs.add(h)
                hs.add(h)                                   # idempotent
            hs.invoke()
            assert sorted(used) == list(range(size))
            removed = {i for i in range(size) if rng.random() < p}
            for i in removed:
                hs.remove(handlers[i])
            used.clear()
            hs.invoke()
            assert len(used) == len(set(used)) == size - len(removed)
            assert not (set(used) & removed)


class HandlerSet:
    """InvalidatedHandlerSet (Internal/InvalidatedHandlerSet.cs:3-128) restated: storage is None,
    one handler, a list of up to 5, or a set (insertion-ordered here; the reference's HashSet order
    is unspecified and nothing depends on it)."""
    LIST = 5

    def __init__(self):
        self.st = None

    def add(self, h):
        st = self.st
        if st is None:
            self.st = h
        elif callable(st):
            if st is not h:
                self.st = [st, h]
        elif isinstance(st, list):
            if h in st:
                return
            if len(st) < self.LIST:
                st.append(h)
            else:
                self.st = dict.fromkeys(st + [h])
        else:
            st[h] = None

    def remove(self, h):
        st = self.st
        if st is None:
            return
        if callable(st):
            if st is h:
                self.st = None
        elif isinstance(st, list):
            if h in st:
                st.remove(h)
        else:
            st.pop(h, None)

    def invoke(self):
        st = self.st
        if st is None:
            return
        for h in ([st] if callable(st) else list(st)):
            h()


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
