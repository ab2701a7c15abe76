// test_fusion.cpp — the reference's behaviour tests replayed through the C++ host
// mirror (fusion.hpp) over the fgi engine. Needs a GPU; run by tests/test_gpu_host.py.
// Each case names the reference test it restates; tests/test_oracle_scenarios.py holds the same
// cases against the CPU oracle.
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

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

// Handlers that run waves of their own (a normal pattern in the reference: an Invalidated handler
// invalidating another node, MutableState.OnInvalidated recomputing). The nested waves must not
// disturb the outer fan-out: every invalidated node fires once, the outer wave's handlers stay on
// the nodes it invalidated even when a handler replaces a slot's node (BeginCompute).
static void reentrant_handlers() {
    ComputedRegistry r(64);
    auto a = Compute(r, "a");
    auto b = Compute(r, "b", {a});
    auto x = Compute(r, "x");
    auto y = Compute(r, "y", {x});
    auto z = Compute(r, "z");
    int fa = 0, fb = 0, fy = 0, fz = 0, fa2 = 0, batches = 0;
    std::shared_ptr<Computed> a2;
    a->OnInvalidated([&](Computed&) { ++fa; });
    y->OnInvalidated([&](Computed&) { ++fy; });
    z->OnInvalidated([&](Computed&) { ++fz; });
    b->OnInvalidated([&](Computed&) {
        ++fb;
        x->Invalidate();   // a nested wave from an Invalidated handler
    });
    r.OnInvalidatedBatch = [&](const uint32_t*, size_t) {
        if (batches++) return;
        z->Invalidate();             // a nested wave from the batch handler
        a2 = r.BeginCompute("a");    // ... and a recompute of a slot the outer wave invalidated
        CHECK(r.SetOutput(*a2));
        a2->OnInvalidated([&](Computed&) { ++fa2; });
    };
    a->Invalidate();
    r.OnInvalidatedBatch = nullptr;
    CHECK(fa == 1 && fb == 1 && fy == 1 && fz == 1 && fa2 == 0);
    CHECK(a->IsInvalidated() && b->IsInvalidated() && x->IsInvalidated() && y->IsInvalidated() && z->IsInvalidated());
    CHECK(a2 && r.Get("a") == a2 && a2->IsConsistent());
    a2->Invalidate();
    CHECK(fa2 == 1 && fa == 1);
}

// TodoApp-style replica fan-out at BASELINE.json configs[4]'s size (DESIGN.md §Host fan-out):
// 10,000 hubs x 1,000 leaves = 10M leaves (1% with an invalidation delay), every leaf computed
// held by one RPC client (peer = leaf % 100, call id = leaf), as RpcInboundComputeCall keeps the
// computed it served (Client/Internal/RpcInboundComputeCall.cs:53-62). One scope invalidates all
// hubs: the wave invalidates 10k hubs + 9.9M undelayed leaves; every undelayed leaf's call id
// must reach its peer exactly once, in handle order, in batches of PeerBatch. Runs the dispatch
// with 16 threads and with 1 and prints one JSON line.
static void fanout_10m() {
    const uint32_t H = 10000, Lh = 1000, P = 100;
    const uint32_t N = H + H * Lh;
    ComputedRegistry r(N, 64);
    std::vector<uint32_t> slot(N), flags(N);
    std::vector<uint64_t> ver(N);
    for (uint32_t s = 0; s < N; ++s) {
        slot[s] = s;
        uint64_t x = (uint64_t)s * 0x9E3779B97F4A7C15ull + 0x5EED00E0;
        x ^= x >> 31;
        ver[s] = ((x * 0xBF58476D1CE4E5B9ull) & ((1ull << 54) - 1)) | 1ull;
        const bool delayed = s >= H && (x % 100) == 0;
        flags[s] = FGI_CONSISTENT | (delayed ? 16u : 0u);
    }
    if (fgi_register_nodes(r.Graph(), N, slot.data(), ver.data(), flags.data()) != FGI_OK) throw FgiError(FGI_EDEVICE, "register");
    std::vector<uint32_t> hub(N - H), leaf(N - H);
    std::vector<uint64_t> tag(N - H);
    uint64_t undelayed = 0;
    for (uint32_t k = 0; k < N - H; ++k) {
        leaf[k] = H + k;
        hub[k] = k / Lh;
        tag[k] = ver[H + k];
        undelayed += (flags[H + k] & 16u) ? 0 : 1;
    }
    if (fgi_load_edges(r.Graph(), N - H, hub.data(), leaf.data(), tag.data()) != FGI_OK) throw FgiError(FGI_EDEVICE, "load");
    if (fgi_snapshot(r.Graph()) != FGI_OK) throw FgiError(FGI_EDEVICE, "snapshot");
    // peers: count calls and check order per peer
    std::vector<uint64_t> got(P, 0), last(P, 0), sum(P, 0);
    uint64_t order_bad = 0;
    for (uint32_t q = 0; q < P; ++q)
        r.AddPeer([&](uint32_t peer, const uint64_t* ids, size_t n) {
            for (size_t i = 0; i < n; ++i) {
                order_bad += (ids[i] <= last[peer] && got[peer]) ? 1 : 0;
                last[peer] = ids[i];
                sum[peer] += ids[i];
            }
            got[peer] += n;
        });
    std::vector<uint32_t> roots(H);
    for (uint32_t h = 0; h < H; ++h) roots[h] = h;
    std::vector<uint32_t> sh(N - H), sp(N - H);
    std::vector<uint64_t> sc(N - H);
    for (uint32_t k = 0; k < N - H; ++k) {
        sh[k] = H + k;
        sp[k] = (H + k) % P;
        sc[k] = H + k;
    }
    std::string runs;
    const uint32_t run_threads[3] = {16u, 16u, 1u}, run_output[3] = {1u, 2u, 2u};   // id list, then bitmap
    for (int run = 0; run < 3; ++run) {
        const uint32_t threads = run_threads[run];
        r.WaveOutput = (int)run_output[run];
        std::fill(got.begin(), got.end(), 0);
        std::fill(sum.begin(), sum.end(), 0);
        std::fill(last.begin(), last.end(), 0);
        order_bad = 0;
        const auto t0 = std::chrono::steady_clock::now();
        r.Subscribe(sh.size(), sh.data(), sp.data(), sc.data());
        const double sub_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
        r.FanoutThreads = threads;
        const auto t1 = std::chrono::steady_clock::now();
        r.InvalidateSlots(roots);
        const double call_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t1).count();
        const FanoutStats& f = r.LastFanout();
        const fgi_wave_stats& w = r.LastWave();
        CHECK(w.v_inv == H + undelayed);
        CHECK(f.ids == w.v_inv && f.calls == undelayed && order_bad == 0);
        CHECK(f.bitmap == (run_output[run] == 2 ? 1u : 0u));
        uint64_t min_b = ~0ull, max_b = 0, tot = 0;
        bool sums_ok = true;
        for (uint32_t q = 0; q < P; ++q) {
            min_b = std::min(min_b, f.peer_batches[q]);
            max_b = std::max(max_b, f.peer_batches[q]);
            tot += got[q];
            CHECK(f.peer_calls[q] == got[q]);
            CHECK(f.peer_batches[q] == (got[q] + r.PeerBatch - 1) / r.PeerBatch);
        }
        // expected per-peer sums of the undelayed leaves' call ids
        std::vector<uint64_t> want(P, 0);
        for (uint32_t k = 0; k < N - H; ++k)
            if (!(flags[H + k] & 16u)) want[(H + k) % P] += H + k;
        for (uint32_t q = 0; q < P; ++q) sums_ok &= want[q] == sum[q];
        CHECK(tot == undelayed && sums_ok);
        char line[768];
        std::snprintf(line, sizeof line,
                      "%s{\"threads\": %u, \"output\": \"%s\", \"v_inv\": %llu, \"wave_kernel_ms\": %.3f, \"wave_call_ms\": %.3f, "
                      "\"invalidate_call_ms\": %.3f, \"dispatch_ms\": %.3f, \"gather_ms\": %.3f, \"subscribe_ms\": %.1f, "
                      "\"calls\": %llu, \"batches\": %llu, \"peers\": %u, \"batches_per_peer\": [%llu, %llu], "
                      "\"peer_batch\": %zu}",
                      runs.empty() ? "" : ", ", f.threads, f.bitmap ? "bitmap" : "ids", (unsigned long long)w.v_inv, w.kernel_ms, w.total_ms, call_ms,
                      f.dispatch_ms, f.gather_ms, sub_ms, (unsigned long long)f.calls, (unsigned long long)f.batches,
                      f.peers_hit, (unsigned long long)min_b, (unsigned long long)max_b, r.PeerBatch);
        runs += line;
        if (fgi_restore(r.Graph()) != FGI_OK) throw FgiError(FGI_EDEVICE, "restore");
    }
    std::printf("FANOUT {\"workload\": \"10000 hubs x 1000 leaves, 1%% delayed, 100 peers, all hubs in one scope\", "
                "\"runs\": [%s]}\n", runs.c_str());
}

// ComputedExt.WhenInvalidated (ComputedExt.cs:99-125) awaited across pipelined waves: two scopes flushed
// as asynchronous waves (fgi_invalidate_async_host), both in flight before either is completed; the
// futures and handlers complete with their own wave's fan-out, in ticket order. Then OnAccess
// (ComputedRegistry.cs:36, 172-176) through TryUseExisting / GetExisting / UseNew (Internal/ComputedExt.cs).
static void when_invalidated_async() {
    using namespace std::chrono_literals;
    ComputedRegistry r(256);
    auto a = Compute(r, "a");
    auto b = Compute(r, "b", {a});
    auto c = Compute(r, "c", {b});
    auto x = Compute(r, "x");
    auto y = Compute(r, "y", {x});
    auto fc = c->WhenInvalidated();
    auto fy = y->WhenInvalidated();
    CHECK(fc.wait_for(0s) == std::future_status::timeout);
    int fired_c = 0, fired_y = 0;
    c->OnInvalidated([&](Computed&) { ++fired_c; });
    y->OnInvalidated([&](Computed&) {
        CHECK(fired_c == 1);   // the first wave's fan-out ran first
        ++fired_y;
    });
    {
        auto scope = r.InvalidateAsync();
        r.InvalidateInput("a");
    }
    const uint64_t t1 = r.LastTicket();
    CHECK(t1 > 0 && r.PendingWaves() == 1);
    {
        auto scope = r.InvalidateAsync();   // queued while the first wave may still run
        r.InvalidateInput("x");
    }
    const uint64_t t2 = r.LastTicket();
    CHECK(t2 == t1 + 1 && r.PendingWaves() == 2);
    CHECK(fired_c == 0 && fc.wait_for(0s) == std::future_status::timeout);   // nothing fans out before completion
    r.Complete(t1);
    CHECK(fc.wait_for(0s) == std::future_status::ready && fired_c == 1 && r.LastWave().v_inv == 3);
    CHECK(fy.wait_for(0s) == std::future_status::timeout && fired_y == 0 && r.PendingWaves() == 1);
    r.CompletePending();
    CHECK(fy.wait_for(0s) == std::future_status::ready && fired_y == 1 && r.LastWave().v_inv == 2);
    CHECK(b->IsInvalidated() && c->IsInvalidated() && y->IsInvalidated() && r.PendingWaves() == 0);
    CHECK(b->WhenInvalidated().wait_for(0s) == std::future_status::ready);   // already invalidated
    CHECK(fc.wait_for(0s) == std::future_status::ready && c->WhenInvalidated().valid());
    // any other registry call completes the waves in flight first (its view includes them)
    auto p = Compute(r, "p");
    auto q = Compute(r, "q", {p});
    auto fq = q->WhenInvalidated();
    {
        auto scope = r.InvalidateAsync();
        r.InvalidateInput("p");
    }
    CHECK(r.PendingWaves() == 1);
    CHECK(r.Get("q") == nullptr && r.PendingWaves() == 0);
    CHECK(fq.wait_for(0s) == std::future_status::ready);
    // OnAccess: TryUseExisting -> RenewTimeouts(true), GetExisting -> RenewTimeouts(false), UseNew -> true
    std::vector<std::pair<std::string, bool>> acc;
    r.OnAccess = [&](Computed& cc, bool is_new) { acc.emplace_back(cc.Input(), is_new); };
    auto m = Compute(r, "m");
    auto n = r.BeginCompute("n");
    CHECK(r.TryUseExisting("m", n.get()) == m);   // n now depends on m
    CHECK(acc.size() == 1 && acc[0].first == "m" && acc[0].second);
    CHECK(r.SetOutput(*n));
    r.UseNew(*n);
    CHECK(acc.size() == 2 && acc[1].first == "n" && acc[1].second);
    CHECK(r.GetExisting("m") == m && acc.size() == 3 && acc[2].first == "m" && !acc[2].second);
    CHECK(n->UsedCount() == 1);
    m->Invalidate();   // the edge TryUseExisting captured carries the cascade
    CHECK(n->IsInvalidated());
    CHECK(r.TryUseExisting("m") == nullptr && r.GetExisting("m") == m && acc.size() == 3);   // Invalidated: no report
}

int main(int argc, char** argv) {
    if (argc > 1 && std::strcmp(argv[1], "--fanout") == 0) {
        try {
            fanout_10m();
        } catch (const FgiError& e) {
            std::fprintf(stderr, "FgiError %d: %s\n", (int)e.status, e.what());
            return 2;
        }
        std::printf("%d/%d checks passed\n", g_checks - g_fail, g_checks);
        return g_fail ? 1 : 0;
    }
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
        reentrant_handlers();
        when_invalidated_async();
    } catch (const FgiError& e) {
        std::fprintf(stderr, "FgiError %d: %s\n", (int)e.status, e.what());
        return 2;
    }
    std::printf("%d/%d checks passed\n", g_checks - g_fail, g_checks);
    return g_fail ? 1 : 0;
}
