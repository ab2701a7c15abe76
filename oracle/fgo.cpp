// fgo.cpp — TEST INFRASTRUCTURE ONLY: CPU restatement of Stl.Fusion's invalidation cascade.
// Used by tests/ (parity checker) and bench.py's cpu_baseline leg; never by the product.
// Pinning status: see fgo.h header and DESIGN.md §Oracle (behaviour pins only; numeric
// large-graph parity is unpinned by the reference, which holds no golden vectors).
//
// Each function cites the reference code it restates (paths relative to the reference root).
// The one deliberate deviation: the recursive cascade of Computed.cs:212-216 is run with an
// explicit stack of pending (slot, version) entries, resolved at pop time, so that deep R-MAT
// chains cannot overflow the native stack. The invalidated set is a monotone closure and does
// not depend on visit order.
#include "fgo.h"

#include <algorithm>
#include <atomic>
#include <chrono>
#include <deque>
#include <memory>
#include <mutex>
#include <thread>
#include <vector>

namespace {

constexpr uint32_t kComputing = FGO_COMPUTING;
constexpr uint32_t kConsistent = FGO_CONSISTENT;
constexpr uint32_t kInvalidated = FGO_INVALIDATED;
constexpr uint32_t kIOSO = 1;            // ComputedFlags.InvalidateOnSetOutput (ComputedFlags.cs:6)
constexpr uint32_t kDelayStarted = 2;    // ComputedFlags.InvalidationDelayStarted (ComputedFlags.cs:7)

inline uint64_t mix64(uint64_t x) {
    x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
    x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
    return x ^ (x >> 31);
}

// HashSet<T> stand-in for the spill of HashSetSlim3: array-backed open addressing (linear
// probing, backward-shift deletion), like .NET's HashSet<T> keeps its entries in flat arrays.
template <class T, class H>
struct FlatSet {
    std::vector<T> keys;
    std::vector<uint8_t> used;
    size_t count = 0;
    size_t mask = 0;

    size_t size() const { return count; }
    void grow() {
        std::vector<T> ok;
        std::vector<uint8_t> ou;
        ok.swap(keys);
        ou.swap(used);
        const size_t cap = ok.empty() ? 8 : ok.size() * 2;
        keys.assign(cap, T{});
        used.assign(cap, 0);
        mask = cap - 1;
        count = 0;
        for (size_t i = 0; i < ok.size(); ++i)
            if (ou[i]) insert(ok[i]);
    }
    bool insert(const T& x) {
        if ((count + 1) * 2 > keys.size()) grow();
        size_t i = H()(x) & mask;
        while (used[i]) {
            if (keys[i] == x) return false;
            i = (i + 1) & mask;
        }
        keys[i] = x;
        used[i] = 1;
        ++count;
        return true;
    }
    bool erase(const T& x) {
        if (!count) return false;
        size_t i = H()(x) & mask;
        while (true) {
            if (!used[i]) return false;
            if (keys[i] == x) break;
            i = (i + 1) & mask;
        }
        used[i] = 0;
        size_t j = i;
        while (true) {
            j = (j + 1) & mask;
            if (!used[j]) break;
            const size_t k = H()(keys[j]) & mask;
            const bool move = (j > i) ? (k <= i || k > j) : (k <= i && k > j);
            if (move) {
                keys[i] = keys[j];
                used[i] = 1;
                used[j] = 0;
                i = j;
            }
        }
        --count;
        return true;
    }
    template <class F> void for_each(F&& f) const {
        for (size_t i = 0; i < keys.size(); ++i)
            if (used[i]) f(keys[i]);
    }
};

// HashSetSlim3<T> (src/Stl/Collections/Slim/HashSetSlim3.cs:3-181): three inline items, then
// a spill to HashSet<T> holding everything. Add of a duplicate is a no-op (returns true there).
template <class T, class H>
struct SmallSet3 {
    uint32_t count = 0;
    T item[3];
    std::unique_ptr<FlatSet<T, H>> set;

    size_t size() const { return set ? set->size() : count; }
    void add(const T& x) {                                   // HashSetSlim3.cs:31-64
        if (set) { set->insert(x); return; }
        for (uint32_t i = 0; i < count; ++i)
            if (item[i] == x) return;
        if (count < 3) { item[count++] = x; return; }
        set.reset(new FlatSet<T, H>());
        for (uint32_t i = 0; i < 3; ++i) set->insert(item[i]);
        set->insert(x);
        count = 0;
    }
    bool remove(const T& x) {                                // HashSetSlim3.cs:66-95
        if (set) return set->erase(x);
        for (uint32_t i = 0; i < count; ++i) {
            if (item[i] == x) {
                for (uint32_t j = i + 1; j < count; ++j) item[j - 1] = item[j];
                --count;
                return true;
            }
        }
        return false;
    }
    void clear() { set.reset(); count = 0; }                 // HashSetSlim3.cs:97-102
    template <class F> void apply(F&& f) const {             // HashSetSlim3.cs:120-133
        if (set) { set->for_each(f); return; }
        for (uint32_t i = 0; i < count; ++i) f(item[i]);
    }
    void copy_from(const SmallSet3& o) {
        count = o.count;
        for (uint32_t i = 0; i < 3; ++i) item[i] = o.item[i];
        set.reset(o.set ? new FlatSet<T, H>(*o.set) : nullptr);
    }
};

struct UsedByEntry {            // (ComputedInput Input, LTag Version) — Computed.cs:37
    uint32_t slot = 0;
    uint64_t version = 0;
    bool operator==(const UsedByEntry& o) const { return slot == o.slot && version == o.version; }
};
struct UsedByHash {
    size_t operator()(const UsedByEntry& e) const { return mix64(e.version * 31 + e.slot); }
};
struct PtrHash {
    size_t operator()(const void* p) const { return mix64((uint64_t)(uintptr_t)p); }
};

struct Node {                   // Computed<T> fields, Computed.cs:30-39
    uint32_t slot = 0;
    uint32_t handle = 0;
    uint64_t version = 0;       // LTag Version (Computed.cs:48)
    bool has_delay = false;     // Options.InvalidationDelay != default (Computed.cs:183)
    std::atomic<uint32_t> state{kComputing};   // volatile int _state
    uint32_t flags = 0;                       // volatile ComputedFlags _flags
    std::mutex lock;                          // lock(this) — Computed.cs:42
    SmallSet3<Node*, PtrHash> used;           // RefHashSetSlim3<IComputedImpl> _used
    SmallSet3<UsedByEntry, UsedByHash> used_by;  // HashSetSlim3<(ComputedInput, LTag)> _usedBy
    // statistics only: entries removed from used_by by RemoveUsedBy during the current wave, so
    // that E_trav counts the out-degree at wave start
    uint64_t rm_wave = 0;
    uint32_t rm_count = 0;
};

// ComputedRegistry (ComputedRegistry.cs:22): ConcurrentDictionary<ComputedInput, GCHandle>.
// Restated as an open-addressing table with lock-free reads (ConcurrentDictionary reads take no
// lock) and CAS updates of the value; keys are inserted once and never removed (a removed entry
// is a null value, which Get treats exactly like a missing key, ComputedRegistry.cs:61-69).
// GC weak-handle liveness is not modelled: every node is strongly held.
struct Registry {
    std::vector<uint32_t> keys;
    std::unique_ptr<std::atomic<Node*>[]> vals;
    uint64_t mask = 0;
    std::mutex insert_lock;

    void init(uint32_t n_slots) {
        uint64_t cap = 16;
        while (cap < 2ull * n_slots + 16) cap <<= 1;
        keys.assign(cap, FGO_NONE);
        vals.reset(new std::atomic<Node*>[cap]);
        for (uint64_t i = 0; i < cap; ++i) vals[i].store(nullptr, std::memory_order_relaxed);
        mask = cap - 1;
    }
    // returns the table index of `slot`, or -1 if the key was never inserted
    int64_t find(uint32_t slot) const {
        uint64_t i = mix64(slot) & mask;
        while (true) {
            uint32_t k = keys[i];
            if (k == slot) return (int64_t)i;
            if (k == FGO_NONE) return -1;
            i = (i + 1) & mask;
        }
    }
    uint64_t find_or_insert(uint32_t slot) {
        int64_t f = find(slot);
        if (f >= 0) return (uint64_t)f;
        std::lock_guard<std::mutex> g(insert_lock);
        uint64_t i = mix64(slot) & mask;
        while (keys[i] != FGO_NONE && keys[i] != slot) i = (i + 1) & mask;
        keys[i] = slot;
        return i;
    }
    Node* get(uint32_t slot) const {                     // ComputedRegistry.Get, 57-70
        int64_t i = find(slot);
        return i < 0 ? nullptr : vals[i].load(std::memory_order_acquire);
    }
};

// Worker threads for bulk work (graph import, snapshot/restore, generators); 1 = serial. Results
// do not depend on it: each thread owns a disjoint set of nodes and visits the edges in input order.
uint32_t g_threads = 1;

template <class F>
void parallel_for_threads(uint32_t T, F&& f) {
    if (T <= 1) {
        f(0u, 1u);
        return;
    }
    std::vector<std::thread> ts;
    for (uint32_t t = 0; t < T; ++t) ts.emplace_back([&, t]() { f(t, T); });
    for (auto& t : ts) t.join();
}

struct Ctx {                     // per-thread cascade state
    std::vector<UsedByEntry> stack;
    std::vector<uint32_t> log;
    uint64_t v_inv = 0, e_trav = 0, e_match = 0, n_flagged = 0;
};

struct SavedNode {
    uint32_t state, flags;
    SmallSet3<Node*, PtrHash> used;
    SmallSet3<UsedByEntry, UsedByHash> used_by;
};

}  // namespace

struct fgo {
    uint32_t n_slots = 0;
    uint64_t wave = 1;                      // statistics epoch (one per public cascade call)
    std::deque<Node> nodes;                 // arena; handle = index
    std::vector<Node*> last;                // slot -> most recently created node
    Registry reg;
    std::vector<uint32_t> log;              // invalidation log (slots)
    std::mutex log_lock;
    // snapshot
    std::vector<SavedNode> saved;
    std::vector<Node*> saved_reg;
    size_t saved_node_count = 0;

    Node* new_node(uint32_t slot, uint64_t version, bool has_delay, uint32_t state, uint32_t flags,
                   bool set_last = true) {
        nodes.emplace_back();
        Node& n = nodes.back();
        n.slot = slot;
        n.handle = (uint32_t)(nodes.size() - 1);
        n.version = version;
        n.has_delay = has_delay;
        n.state.store(state, std::memory_order_relaxed);
        n.flags = flags;
        if (set_last) last[slot] = &n;
        return &n;
    }

    // ComputedRegistry.Unregister (ComputedRegistry.cs:107-132), called from
    // ComputeMethodComputed.OnInvalidated (Interception/ComputeMethodComputed.cs:25-29).
    void unregister(Node* n) {
        int64_t i = reg.find(n->slot);
        if (i < 0) return;
        Node* expected = n;
        reg.vals[i].compare_exchange_strong(expected, nullptr, std::memory_order_acq_rel);
    }

    // IComputedImpl.RemoveUsedBy (Computed.cs:387-398)
    void remove_used_by(Node* c, Node* used_by) {
        std::lock_guard<std::mutex> g(c->lock);
        if (c->state.load(std::memory_order_relaxed) == kInvalidated) return;
        if (c->used_by.remove(UsedByEntry{used_by->slot, used_by->version})) {
            if (c->rm_wave != wave) {
                c->rm_wave = wave;
                c->rm_count = 0;
            }
            c->rm_count++;
        }
    }

    // Computed<T>.Invalidate(bool immediately) prologue + instant-invalidation body
    // (Computed.cs:162-230). The usedBy entries are pushed onto ctx.stack instead of being
    // resolved and recursed into inline (212-216); cascade() drains them.
    void visit(Node* n, bool immediately, Ctx& cx) {
        if (n->state.load(std::memory_order_acquire) == kInvalidated) return;     // 164-165
        {
            std::lock_guard<std::mutex> g(n->lock);                                 // 168
            uint32_t flags = n->flags;
            uint32_t st = n->state.load(std::memory_order_relaxed);
            if (st == kInvalidated) return;                                         // 171-172
            if (st == kComputing) {                                                 // 173-178
                flags |= kIOSO;
                if (immediately) flags |= kDelayStarted;
                if (flags != n->flags) cx.n_flagged++;
                n->flags = flags;
                return;
            }
            immediately |= !n->has_delay;                                           // 183
            if (immediately) {
                n->state.store(kInvalidated, std::memory_order_release);            // 185
            } else {
                if (flags & kDelayStarted) return;                                  // 187-188
                n->flags = flags | kDelayStarted;                                   // 190
                cx.n_flagged++;
                return;   // 194-197: the delayed Invalidate(TimeSpan) timer is host-side
            }
        }
        // Instant invalidation — happens once per node (200-219)
        cx.v_inv++;
        cx.log.push_back(n->slot);
        unregister(n);                                                              // 204
        // 205: Invalidated handlers are dispatched by the host after the wave.
        n->used.apply([&](Node* c) { remove_used_by(c, n); });                      // 210
        n->used.clear();                                                            // 211
        // E_trav / E_match count the wave-start out-degree: entries RemoveUsedBy dropped earlier in
        // this wave pointed at dependants invalidated in it (each matched its dependant's version).
        const uint64_t removed = (n->rm_wave == wave) ? n->rm_count : 0;
        cx.e_trav += n->used_by.size() + removed;
        cx.e_match += removed;
        n->used_by.apply([&](const UsedByEntry& e) {                                // 212
            Node* l = last[e.slot];
            if (l && l->version == e.version) cx.e_match++;
            cx.stack.push_back(e);
        });
        n->used_by.clear();                                                         // 217
    }

    void cascade(Ctx& cx) {
        while (!cx.stack.empty()) {
            UsedByEntry e = cx.stack.back();
            cx.stack.pop_back();
            Node* c = reg.get(e.slot);                       // 213: Input.GetExistingComputed()
            if (c != nullptr && c->version == e.version)     // 214
                visit(c, false, cx);                         // 215
        }
    }

    void invalidate(Node* n, bool immediately, Ctx& cx) {
        visit(n, immediately, cx);
        cascade(cx);
    }

    void flush(Ctx& cx, fgo_stats* st) {
        {
            std::lock_guard<std::mutex> g(log_lock);
            log.insert(log.end(), cx.log.begin(), cx.log.end());
        }
        if (st) {
            st->v_inv += cx.v_inv;
            st->e_trav += cx.e_trav;
            st->e_match += cx.e_match;
            st->n_flagged += cx.n_flagged;
        }
        cx.log.clear();
        cx.v_inv = cx.e_trav = cx.e_match = cx.n_flagged = 0;
    }

    // ComputedRegistry.Register (ComputedRegistry.cs:72-105)
    void register_node(Node* n, Ctx& cx) {
        uint64_t i = reg.find_or_insert(n->slot);
        while (n->state.load(std::memory_order_acquire) != kInvalidated) {          // 83
            Node* target = reg.vals[i].load(std::memory_order_acquire);
            if (target != nullptr) {                                                // 84
                if (target == n) return;                                            // 86-90
                if (target->state.load() != kInvalidated)                           // 91-94
                    invalidate(target, false, cx);
                reg.vals[i].compare_exchange_strong(target, nullptr);               // 95-96
            } else {
                Node* expected = nullptr;                                           // 99-101
                if (reg.vals[i].compare_exchange_strong(expected, n)) return;
            }
        }
    }

    static uint32_t canonical_flags(const Node* n) {
        uint32_t st = n->state.load(std::memory_order_relaxed);
        uint32_t f = st;
        if (st == kComputing) {
            if (n->flags & kIOSO) f |= FGO_F_IOSO;
            if (n->flags & kDelayStarted) f |= FGO_F_DELAY_STARTED;
        } else if (st == kConsistent) {
            if (n->flags & kDelayStarted) f |= FGO_F_DELAY_STARTED;
        }
        if (n->has_delay) f |= FGO_F_HAS_DELAY;
        return f;
    }
};

extern "C" {

fgo* fgo_create(uint32_t n_slots) {
    fgo* o = new fgo();
    o->n_slots = n_slots;
    o->last.assign(n_slots, nullptr);
    o->reg.init(n_slots);
    return o;
}

void fgo_destroy(fgo* o) { delete o; }

int fgo_load_graph(fgo* o, uint32_t n, const uint64_t* version, const uint32_t* state_flags,
                   uint64_t m, const uint32_t* src, const uint32_t* dst, const uint64_t* tag) {
    if (n > o->n_slots) return 1;
    for (uint32_t s = 0; s < n; ++s) {
        if (version[s] == 0) continue;
        uint32_t sf = state_flags ? state_flags[s] : FGO_CONSISTENT;
        uint32_t st = sf & 3u;
        uint32_t fl = ((sf & FGO_F_IOSO) ? kIOSO : 0) | ((sf & FGO_F_DELAY_STARTED) ? kDelayStarted : 0);
        Node* nd = o->new_node(s, version[s], (sf & FGO_F_HAS_DELAY) != 0, st, fl);
        if (st != kInvalidated) {
            uint64_t i = o->reg.find_or_insert(s);
            o->reg.vals[i].store(nd);
        }
    }
    for (uint64_t e = 0; e < m; ++e)
        if (src[e] >= n || !o->last[src[e]] || dst[e] >= o->n_slots) return 1;
    // thread t owns the sets of the nodes whose slot is t mod T; every thread walks the edges in
    // input order, so each set sees the same insertion sequence as a serial import
    parallel_for_threads(g_threads, [&](uint32_t t, uint32_t T) {
        for (uint64_t e = 0; e < m; ++e) {
            Node* s = o->last[src[e]];
            if (src[e] % T == t) s->used_by.add(UsedByEntry{dst[e], tag[e]});
            if (dst[e] % T == t) {
                Node* d = o->last[dst[e]];
                if (d && d->version == tag[e]) d->used.add(s);
            }
        }
    });
    return 0;
}

void fgo_set_threads(uint32_t n) { g_threads = n ? n : 1; }
uint32_t fgo_get_threads(void) { return g_threads; }

uint32_t fgo_current(const fgo* o, uint32_t slot) {
    if (slot >= o->n_slots) return FGO_NONE;
    Node* n = o->reg.get(slot);
    return n ? n->handle : FGO_NONE;
}

uint32_t fgo_last(const fgo* o, uint32_t slot) {
    if (slot >= o->n_slots || !o->last[slot]) return FGO_NONE;
    return o->last[slot]->handle;
}

uint32_t fgo_node_count(const fgo* o) { return (uint32_t)o->nodes.size(); }

int fgo_node_info(const fgo* o, uint32_t h, uint32_t* slot, uint64_t* version, uint32_t* state_flags) {
    if (h >= o->nodes.size()) return 1;
    const Node& n = o->nodes[h];
    if (slot) *slot = n.slot;
    if (version) *version = n.version;
    if (state_flags) *state_flags = fgo::canonical_flags(&n);
    return 0;
}

void fgo_dump_states(const fgo* o, uint64_t* version, uint32_t* state_flags) {
    for (uint32_t s = 0; s < o->n_slots; ++s) {
        const Node* n = o->last[s];
        version[s] = n ? n->version : 0;
        state_flags[s] = n ? fgo::canonical_flags(n) : 0;
    }
}

// ComputeMethodFunctionBase.Compute (ComputeMethodFunctionBase.cs:19-27):
// new ComputeMethodComputed (registered in its ctor, ComputeMethodComputed.cs:9-11).
int fgo_begin_compute(fgo* o, uint32_t slot, uint64_t version, int has_delay,
                      uint32_t* out_new, uint32_t* out_displaced, fgo_stats* st) {
    o->wave++;
    if (slot >= o->n_slots || version == 0) return 1;
    Node* prev = o->reg.get(slot);
    Ctx cx;
    // last[] is updated after registration so that the displacement cascade's E_match statistic
    // is measured against the node that was current when the wave started.
    Node* n = o->new_node(slot, version, has_delay != 0, kComputing, 0, false);
    o->register_node(n, cx);
    o->last[slot] = n;
    o->flush(cx, st);
    if (out_new) *out_new = n->handle;
    if (out_displaced) *out_displaced = prev ? prev->handle : FGO_NONE;
    return 0;
}

// Computed<T>.TrySetOutput (Computed.cs:141-160)
int fgo_set_output(fgo* o, uint32_t h, fgo_stats* st) {
    o->wave++;
    if (h >= o->nodes.size()) return 0;
    Node* n = &o->nodes[h];
    bool must_invalidate;
    {
        std::lock_guard<std::mutex> g(n->lock);
        if (n->state.load() != kComputing) return 0;                        // 145-146
        n->state.store(kConsistent);                                        // 148
        must_invalidate = (n->flags & kIOSO) != 0;                          // 150
    }
    if (must_invalidate) {                                                  // 153-156
        Ctx cx;
        o->invalidate(n, false, cx);
        o->flush(cx, st);
    }
    // 158: StartAutoInvalidation — timers are host-side
    return 1;
}

// IComputedImpl.AddUsed / AddUsedBy (Computed.cs:347-385)
uint32_t fgo_add_used(fgo* o, uint32_t dependant_h, uint32_t used_h, fgo_stats* st) {
    (void)st;
    if (dependant_h >= o->nodes.size() || used_h >= o->nodes.size()) return FGO_USED_ESTATE;
    Node* d = &o->nodes[dependant_h];
    Node* u = &o->nodes[used_h];
    std::lock_guard<std::mutex> g(d->lock);                                 // 350
    if (d->state.load() != kComputing) return FGO_USED_DROPPED;             // 351-364
    uint32_t result;
    {
        // used.AddUsedBy(this)
        std::unique_lock<std::mutex> gu(u->lock, std::defer_lock);
        if (u != d) gu.lock();                                              // 372 (Monitor is re-entrant)
        uint32_t ust = u->state.load();
        if (ust == kComputing) {
            result = FGO_USED_ESTATE;                                       // 374-375: throws
        } else if (ust == kInvalidated) {
            result = FGO_USED_INVALIDATED;                                  // 376-378
        } else {
            u->used_by.add(UsedByEntry{d->slot, d->version});               // 381-382
            result = FGO_USED_ADDED;
        }
    }
    if (result == FGO_USED_INVALIDATED) {
        // usedBy.Invalidate(): the dependant is Computing (checked above under its lock), so
        // Computed.cs:173-178 applies: flags |= InvalidateOnSetOutput.
        d->flags |= kIOSO;
    } else if (result == FGO_USED_ADDED) {
        d->used.add(u);                                                     // 365-366
    }
    return result;
}

// Batches of the three calls above over slots (each slot's most recent node), applied one by one
// in order: the same calls a test would make per element, without a foreign call per element.
int fgo_begin_compute_n(fgo* o, uint32_t n, const uint32_t* slots, const uint64_t* versions,
                        const uint8_t* has_delay, fgo_stats* st) {
    for (uint32_t i = 0; i < n; ++i)
        if (fgo_begin_compute(o, slots[i], versions[i], has_delay ? has_delay[i] : 0, nullptr, nullptr, st)) return 1;
    return 0;
}

uint32_t fgo_set_output_n(fgo* o, uint32_t n, const uint32_t* slots, fgo_stats* st) {
    uint32_t set = 0;
    for (uint32_t i = 0; i < n; ++i) set += (uint32_t)fgo_set_output(o, fgo_last(o, slots[i]), st);
    return set;
}

void fgo_add_used_n(fgo* o, uint32_t n, const uint32_t* dependant_slots, const uint32_t* used_slots,
                    uint32_t* out_codes, fgo_stats* st) {
    for (uint32_t i = 0; i < n; ++i) {
        const uint32_t r = fgo_add_used(o, fgo_last(o, dependant_slots[i]), fgo_last(o, used_slots[i]), st);
        if (out_codes) out_codes[i] = r;
    }
}

int fgo_invalidate_slots(fgo* o, uint32_t n, const uint32_t* slots, const uint8_t* immediately,
                         uint32_t n_threads, fgo_stats* st) {
    o->wave++;
    auto t0 = std::chrono::steady_clock::now();
    if (n_threads <= 1) {
        Ctx cx;
        for (uint32_t i = 0; i < n; ++i) {
            if (slots[i] >= o->n_slots) continue;
            Node* c = o->reg.get(slots[i]);       // TryUseExisting: existing == null -> no-op
            if (c) o->invalidate(c, immediately ? immediately[i] != 0 : false, cx);
        }
        o->flush(cx, st);
    } else {
        std::vector<std::thread> ts;
        std::vector<Ctx> cxs(n_threads);
        for (uint32_t t = 0; t < n_threads; ++t) {
            ts.emplace_back([&, t]() {
                Ctx& cx = cxs[t];
                for (uint32_t i = t; i < n; i += n_threads) {
                    if (slots[i] >= o->n_slots) continue;
                    Node* c = o->reg.get(slots[i]);
                    if (c) o->invalidate(c, immediately ? immediately[i] != 0 : false, cx);
                }
            });
        }
        for (auto& t : ts) t.join();
        for (auto& cx : cxs) o->flush(cx, st);
    }
    if (st) {
        st->wall_ns += (uint64_t)std::chrono::duration_cast<std::chrono::nanoseconds>(
                           std::chrono::steady_clock::now() - t0).count();
        st->threads = n_threads ? n_threads : 1;
    }
    return 0;
}

int fgo_invalidate_nodes(fgo* o, uint32_t n, const uint32_t* handles, const uint8_t* immediately,
                         fgo_stats* st) {
    o->wave++;
    Ctx cx;
    for (uint32_t i = 0; i < n; ++i) {
        if (handles[i] >= o->nodes.size()) continue;
        o->invalidate(&o->nodes[handles[i]], immediately ? immediately[i] != 0 : false, cx);
    }
    o->flush(cx, st);
    return 0;
}

// ComputedRegistry.InvalidateEverything (ComputedRegistry.cs:142-147)
int fgo_invalidate_everything(fgo* o, fgo_stats* st) {
    o->wave++;
    std::vector<uint32_t> keys;
    for (uint32_t k : o->reg.keys)
        if (k != FGO_NONE) keys.push_back(k);
    std::sort(keys.begin(), keys.end());
    Ctx cx;
    for (uint32_t k : keys) {
        Node* c = o->reg.get(k);
        if (c) o->invalidate(c, false, cx);
    }
    o->flush(cx, st);
    return 0;
}

// ComputedGraphPruner.OnRun batch loop (Internal/ComputedGraphPruner.cs:79-94) calling
// IComputedImpl.PruneUsedBy (Computed.cs:400-419) on every registered Consistent node.
int fgo_prune(fgo* o, uint64_t* old_edges, uint64_t* new_edges) {
    return fgo_prune_range(o, 0, 0xFFFFFFFFu, old_edges, new_edges);
}

// One batch of ComputedGraphPruner's walk over the registry (ComputedGraphPruner.cs:79-94): the
// registered keys (slots) in [first, first + count).
int fgo_prune_range(fgo* o, uint32_t first, uint32_t count, uint64_t* old_edges, uint64_t* new_edges) {
    uint64_t oe = 0, ne = 0;
    const uint64_t last = (uint64_t)first + count;
    for (uint32_t k : o->reg.keys) {
        if (k == FGO_NONE || k < first || (uint64_t)k >= last) continue;
        Node* c = o->reg.get(k);
        if (!c || c->state.load() != kConsistent) continue;
        std::lock_guard<std::mutex> g(c->lock);
        if (c->state.load() != kConsistent) continue;                        // 403-407
        SmallSet3<UsedByEntry, UsedByHash> repl;                            // 409
        oe += c->used_by.size();
        c->used_by.apply([&](const UsedByEntry& e) {                        // 411-415
            Node* x = o->reg.get(e.slot);
            if (x != nullptr && x->version == e.version) repl.add(e);
        });
        c->used_by.clear();
        c->used_by.copy_from(repl);                                         // 416
        ne += c->used_by.size();
    }
    if (old_edges) *old_edges = oe;
    if (new_edges) *new_edges = ne;
    return 0;
}

uint64_t fgo_inv_log(const fgo* o, uint32_t* out, uint64_t cap) {
    uint64_t n = o->log.size();
    if (out) for (uint64_t i = 0; i < n && i < cap; ++i) out[i] = o->log[i];
    return n;
}

void fgo_clear_log(fgo* o) { o->log.clear(); }

uint64_t fgo_used_by(const fgo* o, uint32_t h, uint32_t* dst, uint64_t* tag, uint64_t cap) {
    if (h >= o->nodes.size()) return 0;
    const Node& n = o->nodes[h];
    uint64_t i = 0;
    n.used_by.apply([&](const UsedByEntry& e) {
        if (i < cap) {
            if (dst) dst[i] = e.slot;
            if (tag) tag[i] = e.version;
        }
        ++i;
    });
    return i;
}

uint64_t fgo_export_used_by(const fgo* o, uint32_t* slot, uint32_t* dst, uint64_t* tag, uint64_t cap) {
    uint64_t i = 0;
    for (uint32_t s = 0; s < o->n_slots; ++s) {
        const Node* n = o->last[s];
        if (!n) continue;
        n->used_by.apply([&](const UsedByEntry& e) {
            if (i < cap) {
                if (slot) slot[i] = s;
                if (dst) dst[i] = e.slot;
                if (tag) tag[i] = e.version;
            }
            ++i;
        });
    }
    return i;
}

uint32_t fgo_used_count(const fgo* o, uint32_t h) {
    if (h >= o->nodes.size()) return 0;
    return (uint32_t)o->nodes[h].used.size();
}

uint64_t fgo_total_used_by(const fgo* o) {
    uint64_t t = 0;
    for (const Node& n : o->nodes) t += n.used_by.size();
    return t;
}

int fgo_snapshot(fgo* o) {
    o->saved_node_count = o->nodes.size();
    o->saved.clear();
    o->saved.resize(o->nodes.size());
    const size_t N = o->nodes.size();
    parallel_for_threads(g_threads, [&](uint32_t t, uint32_t T) {
        for (size_t i = t; i < N; i += T) {
            Node& n = o->nodes[i];
            SavedNode& s = o->saved[i];
            s.state = n.state.load();
            s.flags = n.flags;
            s.used.copy_from(n.used);
            s.used_by.copy_from(n.used_by);
        }
    });
    o->saved_reg.resize(o->reg.mask + 1);
    for (uint64_t i = 0; i <= o->reg.mask; ++i) o->saved_reg[i] = o->reg.vals[i].load();
    return 0;
}

int fgo_restore(fgo* o) {
    if (o->saved.empty() || o->nodes.size() != o->saved_node_count) return 1;
    const size_t N = o->nodes.size();
    parallel_for_threads(g_threads, [&](uint32_t t, uint32_t T) {
        for (size_t i = t; i < N; i += T) {
            Node& n = o->nodes[i];
            SavedNode& s = o->saved[i];
            n.state.store(s.state);
            n.flags = s.flags;
            n.used.copy_from(s.used);
            n.used_by.copy_from(s.used_by);
        }
    });
    for (uint64_t i = 0; i <= o->reg.mask; ++i) o->reg.vals[i].store(o->saved_reg[i]);
    o->log.clear();
    return 0;
}

}  // extern "C"
