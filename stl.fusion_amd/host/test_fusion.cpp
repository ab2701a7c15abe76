// test_fusion.cpp — the reference's behaviour tests replayed through the C++ host
// mirror (fusion.hpp) over the fgi engine. Needs a GPU; run by tests/test_gpu_host.py.
// Each case names the reference test it restates; tests/test_oracle_scenarios.py holds the same
// cases against the CPU oracle.
#include <cstdio>
#include <cstdlib>
#include <string>

#include "fusion.hpp"

using namespace fusion;

static int g_fail = 0, g_checks = 0;
#define CHECK(cond)                                                              \
    do {                                                                         \
        ++g_checks;                                                              \
        if (!(cond)) {                                                           \
            std::fprintf(stderr, "%s:%d: CHECK(%s) failed\n", __FILE__, __LINE__, #cond); \
            ++g_fail;                                                            \
        }                                                                        \
    } while (0)

// compute(input, deps) = ComputeMethodFunctionBase.Compute: begin, AddUsed each dep, TrySetOutput
static std::shared_ptr<Computed> Compute(ComputedRegistry& r, const std::string& in,
                                         std::initializer_list<std::shared_ptr<Computed>> deps = {},
                                         bool delay = false) {
    auto c = r.BeginCompute(in, delay);
    for (auto& d : deps) CHECK(r.AddUsed(*c, *d) == FGI_USED_ADDED);
    CHECK(r.SetOutput(*c));
    return c;
}

// CounterServiceTest.BasicTest (CounterServiceTest.cs:12-30)
static void counter_basic() {
    ComputedRegistry r(64);
    int unreg = 0;
    r.OnUnregister = [&](Computed&) { ++unreg; };
    auto c = Compute(r, "count(a)");
    CHECK(r.Get("count(a)") == c && c->IsConsistent());
    int fired = 0;
    c->OnInvalidated([&](Computed&) { ++fired; });
    c->Invalidate();
    CHECK(c->IsInvalidated() && fired == 1 && unreg == 1);
    CHECK(r.Get("count(a)") == nullptr);
    c->Invalidate();                      // no-op on an invalidated node
    CHECK(fired == 1);
    int late = 0;
    c->OnInvalidated([&](Computed&) { ++late; });   // added after: fires at once (Computed.cs:84-97)
    CHECK(late == 1);
}

// CounterServiceTest.LongWaitTest (:32-58)
static void counter_long_wait() {
    ComputedRegistry r(64);
    auto c = r.BeginCompute("wait(a)");
    int fired = 0;
    c->OnInvalidated([&](Computed&) { ++fired; });
    c->Invalidate();
    CHECK(c->State() == ConsistencyState::Computing && (c->Flags() & FGI_F_INVALIDATE_ON_SET_OUTPUT) && fired == 0);
    CHECK(r.Get("wait(a)") == c);
    CHECK(r.SetOutput(*c));
    CHECK(c->IsInvalidated() && fired == 1 && r.Get("wait(a)") == nullptr);
}

// CounterServiceTest.ConcurrentWaitTest (:60-98)
static void counter_concurrent_wait() {
    ComputedRegistry r(64);
    auto x = Compute(r, "x");
    auto y = r.BeginCompute("y");
    auto d = r.BeginCompute("first(x,y)");
    CHECK(r.AddUsed(*d, *x) == FGI_USED_ADDED);
    CHECK(r.SetOutput(*d));
    CHECK(r.SetOutput(*y));
    CHECK(r.AddUsed(*d, *y) == FGI_USED_DROPPED);
    CHECK(d->UsedCount() == 1);
    auto d2 = Compute(r, "first(x,y)", {x, y});
    CHECK(d2->UsedCount() == 2);
}

// SimplestProviderTest.BasicTest (SimplestProviderTest.cs:9-32)
static void simplest_provider() {
    ComputedRegistry r(64);
    auto v = Compute(r, "GetValue");
    auto cc = Compute(r, "GetCharCount", {v});
    int fired = 0;
    cc->OnInvalidated([&](Computed&) { ++fired; });
    v->Invalidate();                      // SetValue: using (Computed.Invalidate()) GetValue()
    CHECK(cc->IsInvalidated() && fired == 1);
    CHECK(r.LastWave().v_inv == 2);
    auto v2 = Compute(r, "GetValue");
    auto cc2 = Compute(r, "GetCharCount", {v2});
    CHECK(cc2->Version() != cc->Version() && cc2->IsConsistent());
}

// UserProviderTest.InvalidateEverythingTest (UserProviderTest.cs:12-36) inside a scope
static void invalidate_everything_hub() {
    ComputedRegistry r(256);
    auto hub = Compute(r, "Everything()");
    std::vector<std::shared_ptr<Computed>> users;
    for (int i = 0; i < 100; ++i) users.push_back(Compute(r, "Get(" + std::to_string(i) + ")", {hub}));
    int fired = 0;
    for (auto& u : users) u->OnInvalidated([&](Computed&) { ++fired; });
    {
        auto scope = r.Invalidate();
        CHECK(r.IsInvalidating());
        r.InvalidateInput("Everything()");
        CHECK(fired == 0);                // batched until the scope closes
    }
    CHECK(!r.IsInvalidating() && fired == 100 && r.LastWave().v_inv == 101);
    for (auto& u : users) CHECK(r.Get(u->Input()) == nullptr);
}

// NestedOperationLoggerTest.BasicTest (Extensions/NestedOperationLoggerTest.cs:11-38)
static void nested_scope_multi_root() {
    ComputedRegistry r(64);
    auto a = Compute(r, "a"), b = Compute(r, "b"), c = Compute(r, "c");
    {
        auto outer = r.Invalidate();
        a->Invalidate();
        {
            auto inner = r.Invalidate();
            b->Invalidate();
            r.InvalidateInput("c");
        }
        CHECK(a->IsConsistent() && b->IsConsistent());   // nested scope: still batching
    }
    CHECK(a->IsInvalidated() && b->IsInvalidated() && c->IsInvalidated());
    CHECK(r.LastWave().roots == 3);
}

// Computed.cs:186-198 + Timeouts.cs:22-28: InvalidationDelay
static void invalidation_delay() {
    ComputedRegistry r(64);
    auto s = Compute(r, "state");
    auto d = Compute(r, "delayed", {s}, true);
    auto t = Compute(r, "top", {d});
    s->Invalidate();
    CHECK(s->IsInvalidated() && d->IsConsistent() && (d->Flags() & FGI_F_INVALIDATION_DELAY_STARTED));
    CHECK(t->IsConsistent());
    d->Invalidate(true);                  // the timer fires
    CHECK(d->IsInvalidated() && t->IsInvalidated());
}

// Computed.cs:370-385: AddUsedBy on Invalidated / Computing
static void add_used_states() {
    ComputedRegistry r(64);
    auto u = Compute(r, "u");
    u->Invalidate();
    auto d = r.BeginCompute("d");
    CHECK(r.AddUsed(*d, *u) == FGI_USED_INVALIDATED);
    CHECK(d->Flags() & FGI_F_INVALIDATE_ON_SET_OUTPUT);
    CHECK(r.SetOutput(*d) && d->IsInvalidated());
    auto c = r.BeginCompute("c");
    auto e = r.BeginCompute("e");
    CHECK(r.AddUsed(*e, *c) == FGI_USED_ESTATE);
}

// ComputedRegistry.Register (ComputedRegistry.cs:83-97): displacement
static void register_displacement() {
    ComputedRegistry r(64);
    auto a = Compute(r, "a");
    auto b = Compute(r, "b", {a});
    int fa = 0, fb = 0;
    a->OnInvalidated([&](Computed&) { ++fa; });
    b->OnInvalidated([&](Computed&) { ++fb; });
    auto a2 = r.BeginCompute("a");
    CHECK(fa == 1 && fb == 1 && a->IsInvalidated() && b->IsInvalidated());
    CHECK(r.Get("a") == a2 && a2->State() == ConsistencyState::Computing);
    // a displaced Computing node keeps working on a detached handle; Register's Invalidate()
    // flagged it InvalidateOnSetOutput, so its completion invalidates it (Computed.cs:145-146)
    auto a3 = r.BeginCompute("a");
    CHECK(a2->Handle() != a3->Handle() && a2->State() == ConsistencyState::Computing);
    CHECK(a2->Flags() & FGI_F_INVALIDATE_ON_SET_OUTPUT);
    int f2 = 0;
    a2->OnInvalidated([&](Computed&) { ++f2; });
    CHECK(r.SetOutput(*a2) && a2->IsInvalidated() && f2 == 1);
    CHECK(a3->State() == ConsistencyState::Computing && r.Get("a") == a3);
    // a displaced delayed node is detached Consistent; its timer invalidates it later
    CHECK(r.SetOutput(*a3));
    auto b3 = Compute(r, "b3", {a3});
    r.BeginCompute("x");   // unrelated
    ComputedRegistry r2(64);
    auto d1 = Compute(r2, "d", {}, true);
    auto top = Compute(r2, "top", {d1});
    auto d2 = r2.BeginCompute("d");
    CHECK(d1->IsConsistent() && (d1->Flags() & FGI_F_INVALIDATION_DELAY_STARTED) && top->IsConsistent());
    CHECK(d1->Handle() != d2->Handle());
    d1->Invalidate(true);
    CHECK(d1->IsInvalidated() && top->IsInvalidated() && d2->State() == ConsistencyState::Computing);
    (void)b3;
}

// ComputedGraphPruner pass (Internal/ComputedGraphPruner.cs:79-94)
static void prune() {
    ComputedRegistry r(64);
    auto a = Compute(r, "a");
    auto b = Compute(r, "b", {a});
    Compute(r, "c", {a});
    b->Invalidate();   // RemoveUsedBy: b's entry leaves a's set (lazily in the engine's pool)
    CHECK(a->UsedBy().size() == 1);
    auto pr = r.Prune();   // the pruner compacts the stale entry away
    CHECK(pr.first == 2 && pr.second == 1 && a->UsedBy().size() == 1);
}

int main() {
    try {
        counter_basic();
        counter_long_wait();
        counter_concurrent_wait();
        simplest_provider();
        invalidate_everything_hub();
        nested_scope_multi_root();
        invalidation_delay();
        add_used_states();
        register_displacement();
        prune();
    } catch (const FgiError& e) {
        std::fprintf(stderr, "FgiError %d: %s\n", (int)e.status, e.what());
        return 2;
    }
    std::printf("%d/%d checks passed\n", g_checks - g_fail, g_checks);
    return g_fail ? 1 : 0;
}
