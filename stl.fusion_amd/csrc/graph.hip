// graph.hip — node table, edge pool and the graph-mutation entry points of the fgi C-ABI.
//
// Reference members restated here (paths relative to the Stl.Fusion tree):
//   ComputedRegistry.Register / Get / InvalidateEverything   ComputedRegistry.cs:57-147
//   ComputeMethodFunctionBase.Compute (new Computing node)   Interception/ComputeMethodFunctionBase.cs:19-27
//   IComputedImpl.AddUsed / AddUsedBy                        Computed.cs:347-385
//   Computed<T>.TrySetOutput                                 Computed.cs:141-160
//   IComputedImpl.PruneUsedBy + ComputedGraphPruner          Computed.cs:400-419, Internal/ComputedGraphPruner.cs:79-94
#include <hip/hip_runtime.h>
#include <hip/hip_cooperative_groups.h>

#include <rocprim/device/device_radix_sort.hpp>
#include <rocprim/device/device_reduce.hpp>
#include <rocprim/device/device_segmented_radix_sort.hpp>
#include <rocprim/device/device_scan.hpp>

#include <algorithm>
#include <cstddef>
#include <chrono>
#include <cstdarg>
#include <cstdio>
#include <cstring>

#include "fgi_internal.h"

namespace fgi {

fgi_status set_err(fgi_graph* g, fgi_status st, const char* fmt, ...) {
    if (g) {
        char buf[512];
        va_list ap;
        va_start(ap, fmt);
        vsnprintf(buf, sizeof(buf), fmt, ap);
        va_end(ap);
        g->err = buf;
    }
    return st;
}

fgi_status hip_check(fgi_graph* g, hipError_t e, const char* what) {
    if (e == hipSuccess) return FGI_OK;
    return set_err(g, e == hipErrorOutOfMemory ? FGI_ENOMEM : FGI_EDEVICE, "%s: %s", what, hipGetErrorString(e));
}

namespace {

template <class T>
fgi_status dmalloc(fgi_graph* g, T** p, size_t count) {
    *p = nullptr;
    if (count == 0) count = 1;
    hipError_t e = hipMalloc(reinterpret_cast<void**>(p), count * sizeof(T));
    if (e != hipSuccess) return hip_check(g, e, "hipMalloc");
    return FGI_OK;
}

template <class T>
void dfree(T*& p) {
    if (p) hipFree(p);
    p = nullptr;
}

// RAII device temporaries for non-hot-path operations
// Device temporaries of one ABI call. Small ones (power-of-two size classes up to kTmpKeepMax,
// kTmpKeepTotal in all) go back to the graph's cache when the call ends; every user of a
// temporary runs on the graph's stream, so a later reuse is ordered after it.
constexpr size_t kTmpKeepMax = 64ull << 20;
constexpr size_t kTmpKeepTotal = 512ull << 20;

void tmp_release(fgi_graph* g, void* p, size_t bytes) {
    if (g && bytes <= kTmpKeepMax && g->tmp_cached + bytes <= kTmpKeepTotal) {
        g->tmp_cache.emplace_back(bytes, p);
        g->tmp_cached += bytes;
        return;
    }
    hipFree(p);
}

void tmp_drain(fgi_graph* g) {
    for (auto& e : g->tmp_cache) hipFree(e.second);
    g->tmp_cache.clear();
    g->tmp_cached = 0;
}

struct Tmp {
    fgi_graph* g = nullptr;
    void* p = nullptr;
    size_t bytes = 0;
    ~Tmp() {
        if (p) tmp_release(g, p, bytes);
    }
};
template <class T>
fgi_status tmalloc(fgi_graph* g, Tmp& t, T** p, size_t count) {
    size_t want = 4096;
    while (want < (count ? count : 1) * sizeof(T)) want <<= 1;
    t.g = g;
    for (size_t i = 0; i < g->tmp_cache.size(); ++i) {
        if (g->tmp_cache[i].first == want) {
            t.p = g->tmp_cache[i].second;
            t.bytes = want;
            g->tmp_cache[i] = g->tmp_cache.back();
            g->tmp_cache.pop_back();
            g->tmp_cached -= want;
            *p = reinterpret_cast<T*>(t.p);
            return FGI_OK;
        }
    }
    hipError_t e = hipMalloc(&t.p, want);
    if (e != hipSuccess && !g->tmp_cache.empty()) {   // give the cache back and retry once
        hipStreamSynchronize(g->stream);
        tmp_drain(g);
        e = hipMalloc(&t.p, want);
    }
    if (e != hipSuccess) {
        t.p = nullptr;
        return hip_check(g, e, "hipMalloc(tmp)");
    }
    t.bytes = want;
    *p = reinterpret_cast<T*>(t.p);
    return FGI_OK;
}

__device__ __forceinline__ uint32_t home_of(uint32_t h, uint32_t n_slots, const uint32_t* home) {
    return h < n_slots ? h : home[h - n_slots];
}

// ---- bulk row build -------------------------------------------------------------------------
__global__ void k_mark_unique(uint64_t m, const uint64_t* __restrict__ keys, const uint64_t* __restrict__ tags,
                              uint32_t* __restrict__ keep) {
    const uint64_t e = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (e >= m) return;
    const uint64_t k = keys[e];
    uint32_t kp = 1;
    if (e > 0 && keys[e - 1] == k) {
        if (!tags) {
            kp = 0;
        } else {
            // run of equal (used, dependant): a tag already seen earlier in the run is a duplicate
            const uint64_t t = tags[e];
            for (uint64_t q = e; q > 0 && keys[q - 1] == k; --q)
                if (tags[q - 1] == t) {
                    kp = 0;
                    break;
                }
        }
    }
    keep[e] = kp;
}

__device__ __forceinline__ uint64_t edge_tag(uint64_t ver_seed, uint32_t stale_pct, uint64_t stale_seed,
                                             uint32_t src, uint32_t dst) {
    uint64_t v = synth_version(ver_seed, dst);
    if (stale_pct) {
        const uint64_t h = sm64(stale_seed ^ sm64(((uint64_t)src << 32) | dst));
        if (h % 100 < stale_pct) v += 1;
    }
    return v;
}

__global__ void k_scatter_rows(uint64_t m, const uint64_t* __restrict__ keys, const uint64_t* __restrict__ tags,
                               const uint32_t* __restrict__ keep, const uint32_t* __restrict__ pos,
                               uint64_t ver_seed, uint32_t stale_pct, uint64_t stale_seed, uint32_t* pool_col,
                               uint64_t* pool_tag, uint64_t* row_off, uint32_t* row_len, uint32_t* used_cnt,
                               const unsigned long long* node, uint32_t n_slots, uint32_t src_base,
                               uint32_t dst_base) {
    const uint64_t e = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (e >= m) return;
    const uint64_t k = keys[e];
    const uint32_t src = (uint32_t)(k >> 32), dst = (uint32_t)k;
    const uint32_t p = pos[e];
    if (keep[e]) {
        const uint64_t t = tags ? tags[e] : edge_tag(ver_seed, stale_pct, stale_seed, src + src_base, dst);
        pool_col[p] = dst;
        pool_tag[p] = t;
        // the forward link dependant._used += used exists iff the tag is the dependant's version
        const uint32_t ld = dst - dst_base;
        if (ld < n_slots && (node[ld] & kVMask) == t && t != 0) atomicAdd(&used_cnt[ld], 1u);
    }
    const bool first = (e == 0) || (uint32_t)(keys[e - 1] >> 32) != src;
    const bool last = (e + 1 == m) || (uint32_t)(keys[e + 1] >> 32) != src;
    if (first) row_off[src] = p;
    if (last) row_len[src] = p + keep[e];   // temporarily the row end
}

__global__ void k_fix_rows(uint32_t n, const uint64_t* __restrict__ row_off, uint32_t* row_len, uint32_t* row_cap) {
    const uint32_t h = blockIdx.x * blockDim.x + threadIdx.x;
    if (h >= n) return;
    const uint32_t end = row_len[h];
    const uint32_t len = end ? (uint32_t)(end - row_off[h]) : 0u;
    row_len[h] = len;
    row_cap[h] = len;
}

// Live edges of every row (rows of Invalidated / empty nodes are logically empty) as keys+tags.
__global__ void k_live_len(uint32_t n, const unsigned long long* node, const uint32_t* row_len, uint32_t* out) {
    const uint32_t h = blockIdx.x * blockDim.x + threadIdx.x;
    if (h >= n) return;
    const unsigned long long w = node[h];
    out[h] = word_is_current(w) ? row_len[h] : 0u;
}

__global__ void k_gather_live(uint32_t n, const uint32_t* __restrict__ live_len, const uint64_t* __restrict__ dst_off,
                              const uint64_t* __restrict__ row_off, const uint32_t* __restrict__ pool_col,
                              const uint64_t* __restrict__ pool_tag, uint64_t* keys, uint64_t* tags) {
    // one wave per row
    const uint64_t wave = ((uint64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
    const uint32_t lane = threadIdx.x & 63;
    const uint64_t nw = ((uint64_t)gridDim.x * blockDim.x) >> 6;
    for (uint64_t h = wave; h < n; h += nw) {
        const uint32_t len = live_len[h];
        const uint64_t o = row_off[h], d = dst_off[h];
        for (uint32_t i = lane; i < len; i += 64) {
            keys[d + i] = ((uint64_t)h << 32) | pool_col[o + i];
            tags[d + i] = pool_tag[o + i];
        }
    }
}

// ---- node import / query ---------------------------------------------------------------------
__global__ void k_register(uint32_t n, const uint32_t* slot, const uint64_t* version, const uint32_t* flags,
                           unsigned long long* node, uint32_t* row_len, unsigned long long* err) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const uint32_t s = slot[i];
    if (word_is_current(node[s])) {
        atomicAdd(err, 1ull);
        return;
    }
    node[s] = version[i] ? flags_to_word(version[i], flags ? flags[i] : FGI_CONSISTENT) : 0ull;
    row_len[s] = 0;
}

__global__ void k_gather_words(uint32_t n, const uint32_t* __restrict__ h, const unsigned long long* node,
                               unsigned long long* out) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) out[i] = node[h[i]];
}

__global__ void k_degree_of(uint32_t n, const uint32_t* __restrict__ h, const unsigned long long* __restrict__ node,
                            const uint32_t* __restrict__ row_len, uint32_t* out) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) out[i] = word_is_current(node[h[i]]) ? row_len[h[i]] : 0u;
}

__global__ void k_iota(uint32_t n, uint32_t* out) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) out[i] = i;
}

// ---- begin_compute ---------------------------------------------------------------------------
// class: 0 nothing current, 1 displacement root (Consistent, no delay), 2 detach (Computing, or
// Consistent with a delay: ComputedRegistry.cs:91-96 invalidates it, which only flags it).
__device__ __forceinline__ void bc_classify(uint32_t i, const uint32_t* __restrict__ slot, const unsigned long long* node,
                                            uint8_t* cls, uint32_t* roots, unsigned long long* cnt) {
    const unsigned long long w = node[slot[i]];
    uint8_t c = 0;
    if (word_is_current(w)) {
        if (word_state(w) == FGI_CONSISTENT && !(w & kW_HasDelay)) c = 1;
        else c = 2;
    }
    cls[i] = c;
    if (c == 1) roots[atomicAdd(&cnt[0], 1ull)] = slot[i];
    if (c == 2) atomicAdd(&cnt[1], 1ull);
}

__global__ void k_bc_classify(uint32_t n, const uint32_t* __restrict__ slot, const unsigned long long* node,
                              uint8_t* cls, uint32_t* roots, unsigned long long* cnt /*[0]=roots,[1]=detach*/) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) bc_classify(i, slot, node, cls, roots, cnt);
}

struct InstallArgs {
    const uint32_t* slot;
    const uint64_t* version;
    const uint8_t* has_delay;
    const uint8_t* cls;
    const uint32_t* free_h;
    unsigned long long* cursor;
    uint32_t n_slots;
    unsigned long long* node;
    uint64_t* row_off;
    uint32_t* row_len;
    uint32_t* row_cap;
    uint32_t* used_cnt;
    uint32_t* home;
    uint32_t* out_det;
};

__device__ __forceinline__ void bc_install(uint32_t i, const InstallArgs& a) {
    const uint32_t* slot = a.slot;
    const uint64_t* version = a.version;
    const uint8_t* has_delay = a.has_delay;
    const uint8_t* cls = a.cls;
    const uint32_t* free_h = a.free_h;
    unsigned long long* cursor = a.cursor;
    const uint32_t n_slots = a.n_slots;
    unsigned long long* node = a.node;
    uint64_t* row_off = a.row_off;
    uint32_t* row_len = a.row_len;
    uint32_t* row_cap = a.row_cap;
    uint32_t* used_cnt = a.used_cnt;
    uint32_t* home = a.home;
    uint32_t* out_det = a.out_det;
    const uint32_t s = slot[i];
    uint32_t det = FGI_NONE;
    if (cls[i] == 2) {
        const uint32_t h = free_h[atomicAdd(cursor, 1ull)];
        unsigned long long w = node[s];
        // Register's displacement Invalidate() (ComputedRegistry.cs:91-94, Computed.cs:173-191)
        if (word_state(w) == FGI_COMPUTING) w |= kW_IOSO;
        else if (word_state(w) == FGI_CONSISTENT) w |= kW_DS;
        node[h] = w;
        row_off[h] = row_off[s];
        row_len[h] = row_len[s];
        row_cap[h] = row_cap[s];
        used_cnt[h] = used_cnt[s];
        home[h - n_slots] = s;
        row_off[s] = 0;
        row_cap[s] = 0;
        det = h;
    }
    row_len[s] = 0;   // the new node starts with an empty `_usedBy`; an invalidated row is reused
    used_cnt[s] = 0;
    node[s] = (version[i] & kVMask) | kW_Computing | ((has_delay && has_delay[i]) ? kW_HasDelay : 0ull);
    out_det[i] = det;
}

__global__ void k_bc_install(uint32_t n, InstallArgs a) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) bc_install(i, a);
}

// ---- add_used --------------------------------------------------------------------------------
struct Cand {
    uint32_t used, dep_handle, dep_slot, pad;
    uint64_t tag;
};

struct AuArgs {
    const uint32_t* dep;
    const uint32_t* used;
    uint32_t n_slots;
    const uint32_t* home;
    unsigned long long* node;
    uint64_t* row_off;
    uint32_t* row_len;
    uint32_t* row_cap;
    uint32_t* used_cnt;
    uint32_t* pool_col;
    uint64_t* pool_tag;
    unsigned long long* hset;
    uint64_t hmask;
    uint32_t* result;
    Cand* cand;
    uint32_t* pend_pos;
    uint32_t* ovf_rows;
    unsigned long long* cnt;   // [0] candidates [1] pending [2] overflow rows [3] entries the overflow rows need
};

// one pair: its result code; true (and *out) if it is a new `_usedBy` entry to append
__device__ __forceinline__ bool au_classify_pair(uint32_t i, const AuArgs& a, Cand* out) {
    const uint32_t* dep = a.dep;
    const uint32_t* used = a.used;
    const uint32_t n_slots = a.n_slots;
    const uint32_t* home = a.home;
    unsigned long long* node = a.node;
    const uint64_t* row_off = a.row_off;
    const uint32_t* row_len = a.row_len;
    const uint32_t* used_cnt = a.used_cnt;
    const uint32_t* pool_col = a.pool_col;
    const uint64_t* pool_tag = a.pool_tag;
    unsigned long long* hset = a.hset;
    const uint64_t hmask = a.hmask;
    uint32_t* result = a.result;
    const uint32_t d = dep[i], u = used[i];
    const unsigned long long wd = node[d];
    if ((wd & kVMask) == 0 || word_state(wd) != FGI_COMPUTING) {   // Computed.cs:351-364
        result[i] = FGI_USED_DROPPED;
        return false;
    }
    const unsigned long long wu = node[u];
    if ((wu & kVMask) == 0 || word_state(wu) == FGI_INVALIDATED) {  // Computed.cs:376-378
        atomicOr(node + d, kW_IOSO);
        result[i] = FGI_USED_INVALIDATED;
        return false;
    }
    if (word_state(wu) == FGI_COMPUTING) {                           // Computed.cs:374-375
        result[i] = FGI_USED_ESTATE;
        return false;
    }
    result[i] = FGI_USED_ADDED;                                      // Computed.cs:381-383
    // set semantics: (u, d) within this batch ...
    const unsigned long long key = ((unsigned long long)u << 32) | d;
    uint64_t p = sm64(key) & hmask;
    while (true) {
        const unsigned long long prev = atomicCAS(hset + p, ~0ull, key);
        if (prev == ~0ull) break;
        if (prev == key) return false;
        p = (p + 1) & hmask;
    }
    const uint32_t ds = home_of(d, n_slots, home);
    const uint64_t tag = wd & kVMask;
    // ... and across batches: only a dependant that already captured deps can repeat one
    if (used_cnt[d]) {
        const uint64_t o = row_off[u];
        const uint32_t len = row_len[u];
        for (uint32_t k = 0; k < len; ++k)
            if (pool_col[o + k] == ds && pool_tag[o + k] == tag) return false;
    }
    *out = Cand{u, d, ds, 0, tag};
    return true;
}

// Pairs [blockIdx.x * blockDim.x, ...): block-uniform call. The block's new candidates are appended
// with one reservation per block (a single counter word serialises ~88 atomics per microsecond).
__device__ __forceinline__ void au_classify_block(uint32_t i, bool valid, const AuArgs& a) {
    __shared__ uint32_t s_w[8];
    __shared__ unsigned long long s_base;
    Cand cd{};
    const bool want = valid && au_classify_pair(i, a, &cd);
    const unsigned long long m = __ballot(want);
    const uint32_t lane = threadIdx.x & 63, wid = threadIdx.x >> 6, nw = blockDim.x >> 6;
    if (lane == 0) s_w[wid] = (uint32_t)__popcll(m);
    __syncthreads();
    uint32_t before = 0, total = 0;
    for (uint32_t w = 0; w < nw; ++w) {
        before += w < wid ? s_w[w] : 0u;
        total += s_w[w];
    }
    if (threadIdx.x == 0) s_base = total ? atomicAdd(a.cnt, (unsigned long long)total) : 0ull;
    __syncthreads();
    if (want) {
        const uint32_t r = __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
        a.cand[s_base + before + r] = cd;
    }
}

__global__ void k_au_classify(uint32_t n, AuArgs a) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    au_classify_block(i, i < n, a);
}

// Candidate i (valid) per lane; every lane of the wave calls it. Consecutive candidates with the same
// used node (a hub's dependants, appended by one batch) reserve their row slots with one atomic per
// run of equal keys in the wave instead of one each (the row-length word of a hub otherwise takes
// a thousand serialised atomics).
__device__ __forceinline__ void au_reserve(uint64_t i, bool valid, const AuArgs& a) {
    const uint64_t* row_off = a.row_off;
    uint32_t* row_len = a.row_len;
    const uint32_t* row_cap = a.row_cap;
    uint32_t* used_cnt = a.used_cnt;
    uint32_t* pool_col = a.pool_col;
    uint64_t* pool_tag = a.pool_tag;
    uint32_t* pend_pos = a.pend_pos;
    uint32_t* ovf_rows = a.ovf_rows;
    unsigned long long* cnt = a.cnt + 1;
    const uint32_t lane = threadIdx.x & 63;
    const Cand c = valid ? a.cand[i] : Cand{FGI_NONE, 0u, 0u, 0u, 0ull};
    const uint32_t prev = __shfl_up(c.used, 1, 64);
    const bool head = valid && (lane == 0 || prev != c.used);
    const unsigned long long heads = __ballot(head), vm = __ballot(valid);
    // this lane's run: from the nearest head at or below it to the next head (or the last valid lane)
    const unsigned long long below = heads & (lane == 63 ? ~0ull : ((2ull << lane) - 1ull));
    const uint32_t start = below ? 63u - (uint32_t)__builtin_clzll(below) : 0u;
    const unsigned long long above = heads & ~((2ull << lane) - 1ull) & (lane == 63 ? 0ull : ~0ull);
    const uint32_t end = above ? (uint32_t)__builtin_ctzll(above) : 64u - (uint32_t)__builtin_clzll(vm | 1ull);
    uint32_t base = 0;
    if (head) base = atomicAdd(&row_len[c.used], end - start);
    base = __shfl(base, start, 64);
    if (!valid) return;
    const uint32_t pos = base + (lane - start);
    const uint32_t cap = row_cap[c.used];
    if (used_cnt) atomicAdd(&used_cnt[c.dep_handle], 1u);            // dependant._used.Add (365-366); a
                                                                     // partition's owner of it counts it
    if (pos < cap) {
        pool_col[row_off[c.used] + pos] = c.dep_slot;
        pool_tag[row_off[c.used] + pos] = c.tag;
        pend_pos[i] = FGI_NONE;
    } else {
        pend_pos[i] = pos;
        atomicAdd(&cnt[0], 1ull);
        // performed at the coherence point: a batch's last reserve block reads the list (kb_au_reserve)
        if (pos == cap) __hip_atomic_exchange(&ovf_rows[atomicAdd(&cnt[1], 1ull)], c.used, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
}

__global__ void k_au_reserve(uint64_t nc, AuArgs a) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    au_reserve(i, i < nc, a);
}

__device__ __forceinline__ uint32_t grow_cap(uint32_t need) {
    const uint64_t c = (uint64_t)need + (need >> 1);
    return (uint32_t)(c < 4 ? 4 : (c > 0xFFFFFFF0ull ? 0xFFFFFFF0ull : c));
}

__global__ void k_au_size(uint64_t no, const uint32_t* __restrict__ ovf_rows, const uint32_t* __restrict__ row_len,
                          unsigned long long* sum) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < no) atomicAdd(sum, (unsigned long long)grow_cap(row_len[ovf_rows[i]]));
}

// one wave per overflowing row: allocate a larger run at the pool top and move the old entries
__device__ __forceinline__ void au_relocate_row(uint64_t wave, const uint32_t* __restrict__ ovf_rows, uint64_t* row_off,
                                                const uint32_t* __restrict__ row_len, uint32_t* row_cap,
                                                uint32_t* pool_col, uint64_t* pool_tag, unsigned long long* top) {
    const uint32_t lane = threadIdx.x & 63;
    const uint32_t u = ovf_rows[wave];
    const uint32_t ncap = grow_cap(row_len[u]);
    unsigned long long base = 0;
    if (lane == 0) base = atomicAdd(top, (unsigned long long)ncap);
    base = __shfl(base, 0, 64);
    const uint64_t o = row_off[u];
    const uint32_t old_cap = row_cap[u];
    for (uint32_t k = lane; k < old_cap; k += 64) {
        pool_col[base + k] = pool_col[o + k];
        pool_tag[base + k] = pool_tag[o + k];
    }
    if (lane == 0) {
        row_off[u] = base;
        row_cap[u] = ncap;
    }
}

__global__ void k_au_relocate(uint64_t no, const uint32_t* __restrict__ ovf_rows, uint64_t* row_off,
                              const uint32_t* __restrict__ row_len, uint32_t* row_cap, uint32_t* pool_col,
                              uint64_t* pool_tag, unsigned long long* top) {
    const uint64_t wave = ((uint64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
    if (wave < no) au_relocate_row(wave, ovf_rows, row_off, row_len, row_cap, pool_col, pool_tag, top);
}

__device__ __forceinline__ void au_pending(uint64_t i, const Cand* __restrict__ cand, const uint32_t* __restrict__ pend_pos,
                                           const uint64_t* __restrict__ row_off, uint32_t* pool_col, uint64_t* pool_tag) {
    if (pend_pos[i] == FGI_NONE) return;
    const Cand c = cand[i];
    pool_col[row_off[c.used] + pend_pos[i]] = c.dep_slot;
    pool_tag[row_off[c.used] + pend_pos[i]] = c.tag;
}

__global__ void k_au_pending(uint64_t nc, const Cand* __restrict__ cand, const uint32_t* __restrict__ pend_pos,
                             const uint64_t* __restrict__ row_off, uint32_t* pool_col, uint64_t* pool_tag) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < nc) au_pending(i, cand, pend_pos, row_off, pool_col, pool_tag);
}

// ---- set_output ------------------------------------------------------------------------------
__device__ __forceinline__ void set_output(uint32_t i, const uint32_t* __restrict__ h, uint32_t n_handles,
                                           unsigned long long* node, uint8_t* out_set, uint32_t* roots,
                                           unsigned long long* nroots) {
    uint8_t set = 0;
    const uint32_t x = h[i];
    if (x < n_handles) {
        unsigned long long w = node[x];
        while ((w & kVMask) != 0 && word_state(w) == FGI_COMPUTING) {      // Computed.cs:145-146
            const unsigned long long nw = (w & ~(kStateBits | kW_IOSO)) | kW_Consistent;   // 148
            const unsigned long long prev = atomicCAS(node + x, w, nw);
            if (prev == w) {
                set = 1;
                if (w & kW_IOSO) roots[atomicAdd(nroots, 1ull)] = x;     // 150-156
                break;
            }
            w = prev;
        }
    }
    out_set[i] = set;
}

__global__ void k_set_output(uint32_t n, const uint32_t* __restrict__ h, uint32_t n_handles, unsigned long long* node,
                             uint8_t* out_set, uint32_t* roots, unsigned long long* nroots) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) set_output(i, h, n_handles, node, out_set, roots, nroots);
}

// ---- streaming batches (fgi_run_batch) ------------------------------------------------------------
// A batch's kernels read their item counts from the device and do nothing once the batch's abort
// word is set (a step that cannot complete here: the host finishes it, or reports it, after its one
// synchronisation). Abort word: reason << 32 | (step + 1) (kAbort*, fgi_internal.h).

__device__ __forceinline__ bool batch_aborted(const unsigned long long* ab) {
    return __hip_atomic_load(ab, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0;
}

__device__ __forceinline__ uint64_t grid_tid() { return (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; }
__device__ __forceinline__ uint64_t grid_threads() { return (uint64_t)gridDim.x * blockDim.x; }

// Block-uniform: true in the block that arrives last at this launch's completion counter
// (fgi_internal.h). Any wave of a batch kernel may have issued the returnless atomics the last block
// reads (classify counts, the overflow-row list), so every wave drains before the block arrives; the
// last block reads them at the coherence point (bcoh_read).
__device__ __forceinline__ unsigned long long bcoh_read(unsigned long long* p) {
    return __hip_atomic_fetch_add(p, 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ bool batch_last_block(unsigned long long* done, uint64_t G) {
    return last_block_arrive<true>(done, G);
}

__device__ __forceinline__ void batch_abort(unsigned long long* ab, unsigned long long code) {
    __hip_atomic_exchange(ab, code, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// classify, then (last block) the check: the displaced nodes that survive (cnt[1]) need detached
// handles, and the batch's list has n_take (one launch instead of classify + a one-thread check)
__global__ void kb_bc_classify_check(unsigned long long* ab, uint32_t n, const uint32_t* __restrict__ slot,
                                     const unsigned long long* node, uint8_t* cls, uint32_t* roots, unsigned long long* cnt,
                                     unsigned long long* cursor, uint64_t n_take, uint32_t step, unsigned long long* done) {
    if (batch_aborted(ab)) return;   // uniform over the grid: nothing in this launch sets the word before its end
    const uint64_t i = grid_tid();
    if (i < n) bc_classify((uint32_t)i, slot, node, cls, roots, cnt);
    if (!batch_last_block(done, gridDim.x)) return;
    if (threadIdx.x == 0 && bcoh_read(cursor) + bcoh_read(cnt + 1) > n_take) batch_abort(ab, (kAbortDetach << 32) | (step + 1ull));
}

__global__ void kb_bc_install(const unsigned long long* ab, uint32_t n, InstallArgs a) {
    if (batch_aborted(ab)) return;
    const uint64_t i = grid_tid();
    if (i < n) bc_install((uint32_t)i, a);
}

__global__ void kb_au_classify(const unsigned long long* ab, uint32_t n, AuArgs a) {
    if (batch_aborted(ab)) return;
    const uint64_t i = grid_tid();
    au_classify_block((uint32_t)i, i < n, a);
}

// reserve, then (last block) the overflowing rows' new capacities (cnt[3]) and whether they fit the
// pool (otherwise the host grows it and finishes the step): one launch instead of reserve + size + check
__global__ void kb_au_reserve(unsigned long long* ab, AuArgs a, const unsigned long long* top, uint64_t cap, uint32_t step,
                              unsigned long long* done) {
    if (batch_aborted(ab)) return;   // uniform over the grid
    const uint64_t nc = a.cnt[0];
    for (uint64_t i0 = grid_tid() - (threadIdx.x & 63); i0 < nc; i0 += grid_threads())   // wave-uniform
        au_reserve(i0 + (threadIdx.x & 63), i0 + (threadIdx.x & 63) < nc, a);
    if (!batch_last_block(done, gridDim.x)) return;
    __shared__ unsigned long long s_need[kBlock / 64];
    const uint64_t no = bcoh_read(a.cnt + 2);
    unsigned long long need = 0;
    for (uint64_t i = threadIdx.x; i < no; i += blockDim.x) {
        const uint32_t u = __hip_atomic_fetch_add(a.ovf_rows + i, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        need += grow_cap(__hip_atomic_fetch_add(a.row_len + u, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
    }
#pragma unroll
    for (int d = 32; d >= 1; d >>= 1) need += __shfl_xor(need, d, 64);
    if ((threadIdx.x & 63) == 0) s_need[threadIdx.x >> 6] = need;
    __syncthreads();
    if (threadIdx.x == 0) {
        unsigned long long all = 0;
        for (uint32_t w = 0; w < blockDim.x / 64; ++w) all += s_need[w];
        __hip_atomic_exchange(a.cnt + 3, all, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (no && bcoh_read(const_cast<unsigned long long*>(top)) + all > cap)
            batch_abort(ab, (kAbortPool << 32) | (step + 1ull));
    }
}

__global__ void kb_au_relocate(const unsigned long long* ab, AuArgs a, unsigned long long* top) {
    if (batch_aborted(ab)) return;
    const uint64_t no = a.cnt[2];
    for (uint64_t w = grid_tid() >> 6; w < no; w += grid_threads() >> 6)   // wave-uniform
        au_relocate_row(w, a.ovf_rows, a.row_off, a.row_len, a.row_cap, a.pool_col, a.pool_tag, top);
}

__global__ void kb_au_pending(const unsigned long long* ab, AuArgs a) {
    if (batch_aborted(ab)) return;
    const uint64_t nc = a.cnt[0];
    for (uint64_t i = grid_tid(); i < nc; i += grid_threads()) au_pending(i, a.cand, a.pend_pos, a.row_off, a.pool_col, a.pool_tag);
}

// the values the host reads after the batch, next to its counters (one copy back)
__global__ void kb_finish(const unsigned long long* top, unsigned long long* dst) {
    if (threadIdx.x == 0 && blockIdx.x == 0) *dst = *top;
}

__global__ void kb_set_output(const unsigned long long* ab, uint32_t n, const uint32_t* __restrict__ h, uint32_t n_handles,
                              unsigned long long* node, uint8_t* out_set, uint32_t* roots, unsigned long long* nroots) {
    if (batch_aborted(ab)) return;
    const uint64_t i = grid_tid();
    if (i < n) set_output((uint32_t)i, h, n_handles, node, out_set, roots, nroots);
}

// ---- prune -----------------------------------------------------------------------------------
// keep(h): 0 = drop the whole row, 1 = PruneUsedBy filter, 2 = keep all
__device__ __forceinline__ int prune_mode(uint32_t h, uint32_t n_slots, unsigned long long w) {
    if (!word_is_current(w)) return 0;                 // Invalidated / empty: `_usedBy` cleared (217)
    if (h < n_slots && word_state(w) == FGI_CONSISTENT) return 1;   // registered Consistent (ComputedGraphPruner.cs:87-90)
    return 2;                                          // Computing, or detached (not in the registry)
}

#ifndef FGI_SHORT_PER
#define FGI_SHORT_PER 4   // 64-entry slices a wave loads per step of the short-row prune
#endif

__device__ __forceinline__ bool edge_live(const unsigned long long* node, uint32_t dst, uint64_t tag) {
    const unsigned long long w = node[dst];              // Computed.cs:412-413
    return word_is_current(w) && (w & kVMask) == tag;
}

// pool accesses of a prune (plain: non-temporal loads and stores measured slower together, 6.6 against
// 5.5 ms on configs[3], round 2)
template <class T> __device__ __forceinline__ T pr_ld(const T* p) { return *p; }
template <class T> __device__ __forceinline__ void pr_st(T* p, T v) { *p = v; }

__device__ __forceinline__ uint32_t wave_excl_scan32(uint32_t v, uint32_t& total) {
    const uint32_t lane = threadIdx.x & 63;
    uint32_t x = v;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        const uint32_t y = __shfl_up(x, d, 64);
        if (lane >= (uint32_t)d) x += y;
    }
    total = __shfl(x, 63, 64);
    return x - v;
}

// PruneUsedBy in place, rows of handles [lo, hi), two launches (k_prune_rows, k_prune_chunks): an Invalidated /
// empty node's row is dropped (len 0), a registered Consistent node's row keeps the entries whose
// slot's current node is at the entry's version, every other row is kept whole. Rows keep their
// offsets and capacities (the freed entries are slack the row grows into).
//   phase 1: waves take 64 consecutive rows and filter the rows of at most kPruneLong entries as
//            one flattened sequence; the longer rows are listed as chunks of kChunk entries
//            (chunk map: handle | first chunk of the row << 32), one atomic per block.
//   kernel boundary
//   phase 2: blocks take chunks in index order. A chunk loads and checks its entries, publishes
//            its kept count, then sums the counts of the row's earlier chunks (each published only
//            after that chunk's loads, so no store of this chunk can pass an unread entry) and
//            stores; the row's last chunk sets its length. Chunks wait only on lower chunk
//            indices, and blocks start in index order: the lowest unfinished chunk always proceeds.
constexpr uint32_t kPruneLong = 1024;
constexpr uint32_t kBlockLong = 64;     // long rows a block lists with one atomic
constexpr int kChunkPer = 8;
constexpr uint32_t kChunk = 256 * kChunkPer;
constexpr uint32_t kChunkDone = 1u << 31;
enum : int { kPrOld, kPrNew, kPrChunks, kPrDropped, kPrLive, kPrN };

struct PruneArgs {
    uint32_t lo, hi, n_slots;
    // [lo, hi) are boundary handles: row of handle x = its label (hot: s2l[x], else K + x)
    const uint32_t* s2l;
    uint32_t ext_slots, K;
    const unsigned long long* node;
    const uint64_t* row_off;
    uint32_t* row_len;
    uint32_t* pool_col;
    uint64_t* pool_tag;
    uint64_t* chunk_map;        // chunk -> handle | first chunk of its row << 32
    uint32_t* chunk_st;         // zeroed; kChunkDone | kept entries once a chunk has loaded
    unsigned long long* st;     // kPrN counters
    // fast path (fgi_graph::pool_live valid, else null): liveness at list build per pool position,
    // and the handles whose node is current
    const unsigned long long* live_bm;
    const uint32_t* cur_bm;
    // partitions (rows keep global dependant ids): a dependant is current iff its bit in the
    // all-gathered current bitmaps (rank q's pw64 words at q * pw64, one per pblock slots) is set, and
    // its version is the replica's
    const uint64_t* ver_all;
    const unsigned long long* cur_all;
    uint32_t pblock, pw64;
};

// Computed.cs:412-413 for the entry at pool position pos: through the two bitmaps on the fast path,
// else from the dependant's node word
__device__ __forceinline__ bool entry_live(const PruneArgs& a, uint64_t pos, uint32_t dst, uint64_t tag) {
    if (a.ver_all) {
        const uint32_t q = dst / a.pblock, l = dst - q * a.pblock;
        return ((a.cur_all[(uint64_t)q * a.pw64 + (l >> 6)] >> (l & 63)) & 1ull) && a.ver_all[dst] == tag;
    }
    if (a.live_bm) return ((a.live_bm[pos >> 6] >> (pos & 63)) & 1ull) && ((a.cur_bm[dst >> 5] >> (dst & 31)) & 1u);
    return edge_live(a.node, dst, tag);
}

// the chunk map entries of one long row (nch chunks from cb), by the calling threads
__device__ __forceinline__ void prune_map_row(uint64_t* map, uint32_t h, uint32_t cb, uint32_t nch, uint32_t t,
                                              uint32_t nt) {
    for (uint32_t j = t; j < nch; j += nt) map[cb + j] = (uint64_t)h | ((uint64_t)cb << 32);
}

__device__ void prune_short_rows(const PruneArgs& a, uint32_t* s_lh, uint32_t* s_lc, uint32_t& s_nl,
                                 unsigned long long* acc) {
    __shared__ uint32_t s_pre[4][65];    // flattened start of each lane's row (+ the total)
    __shared__ uint32_t s_kept[4][64];   // kept entries so far, per row
    __shared__ uint64_t s_off[4][64];    // row offsets
    const uint32_t lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    const uint64_t nw = ((uint64_t)gridDim.x * blockDim.x) >> 6;
    const uint64_t n_rows = a.hi - a.lo;
    for (uint64_t r0 = (((uint64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6) * 64; r0 < n_rows; r0 += nw * 64) {
        const uint64_t x = a.lo + r0 + lane;
        uint64_t h = x + a.K;
        if (a.s2l && x < a.ext_slots && r0 + lane < n_rows) {
            const uint32_t l = a.s2l[x];
            if (l != FGI_NONE) h = l;
        }
        uint32_t len = 0, eff = 0;
        uint64_t off = 0;
        int mode = 2;
        if (r0 + lane < n_rows) {   // one round: length, word and offset
            len = a.row_len[h];
            const unsigned long long w = a.node[h];
            off = a.row_off[h];
            mode = prune_mode((uint32_t)h, a.n_slots, w);
        }
        if (len && mode == 0) {
            a.row_len[h] = 0;
            acc[2] += len;
        } else if (len && mode == 2) {
            acc[3] += len;
        } else if (len > kPruneLong) {
            const uint32_t nch = (len + kChunk - 1) / kChunk;
            const uint32_t q = atomicAdd(&s_nl, 1u);
            if (q < kBlockLong) {
                s_lh[q] = (uint32_t)h;
                s_lc[q] = nch;
            } else {   // list full: a row of its own
                const uint32_t cb = (uint32_t)atomicAdd(&a.st[kPrChunks], (unsigned long long)nch);
                prune_map_row(a.chunk_map, (uint32_t)h, cb, nch, 0, 1);
            }
        } else if (len) {
            eff = len;
        }
        uint32_t total;
        const uint32_t pre = wave_excl_scan32(eff, total);
        s_pre[wid][lane] = pre;
        if (lane == 0) s_pre[wid][64] = total;
        s_kept[wid][lane] = 0;
        s_off[wid][lane] = off;
        __builtin_amdgcn_wave_barrier();
        // kShortPer slices of 64 flattened entries per step: every load and liveness gather of the
        // step is issued before the first store (a slice's stores never pass its own loads, and the
        // later slices are already in registers)
        constexpr int kShortPer = FGI_SHORT_PER;
        for (uint32_t s0 = 0; s0 < total; s0 += 64 * kShortPer) {   // wave-uniform
            uint32_t rr[kShortPer], col[kShortPer];
            uint64_t tag[kShortPer], ro[kShortPer];
            bool keep[kShortPer];
#pragma unroll
            for (int q = 0; q < kShortPer; ++q) {
                const uint32_t f = s0 + 64 * q + lane;
                uint32_t r = 0;
                if (f < total) {
#pragma unroll
                    for (uint32_t step = 32; step >= 1; step >>= 1)   // the largest r with start <= f
                        if (r + step < 64 && s_pre[wid][r + step] <= f) r += step;
                }
                rr[q] = r;
                ro[q] = s_off[wid][r];
                const uint32_t k = f < total ? f - s_pre[wid][r] : 0u;
                col[q] = f < total ? pr_ld(a.pool_col + ro[q] + k) : 0u;
                tag[q] = f < total ? pr_ld(a.pool_tag + ro[q] + k) : 0ull;
            }
#pragma unroll
            for (int q = 0; q < kShortPer; ++q) {
                const uint32_t f = s0 + 64 * q + lane;
                keep[q] = f < total && entry_live(a, ro[q] + (f - s_pre[wid][rr[q]]), col[q], tag[q]);
            }
#pragma unroll
            for (int q = 0; q < kShortPer; ++q) {
                const uint32_t sq = s0 + 64 * q;
                if (sq >= total) break;   // wave-uniform
                const uint32_t f = sq + lane;
                const bool in = f < total;
                const uint32_t r = rr[q];
                const unsigned long long km = __ballot(keep[q]);
                // lanes of this slice in the same row: from the row's first lane in the slice
                const uint32_t first = in ? (s_pre[wid][r] > sq ? s_pre[wid][r] - sq : 0u) : 0u;
                const unsigned long long seg = ((1ull << lane) - 1ull) & ~((1ull << first) - 1ull);
                const uint32_t before = (uint32_t)__popcll(km & seg);
                const uint32_t base_kept = in ? s_kept[wid][r] : 0u;
                __builtin_amdgcn_wave_barrier();
                if (keep[q]) {
                    pr_st(a.pool_col + ro[q] + base_kept + before, col[q]);
                    pr_st(a.pool_tag + ro[q] + base_kept + before, tag[q]);
                }
                // the row's last lane of this slice adds the slice's kept entries of the row
                const bool last = in && (f + 1 == s_pre[wid][r + 1] || lane == 63 || f + 1 == total);
                if (last) s_kept[wid][r] = base_kept + before + (keep[q] ? 1u : 0u);
                __builtin_amdgcn_wave_barrier();
            }
        }
        if (eff) {
            const uint32_t kept = s_kept[wid][lane];
            a.row_len[h] = kept;
            acc[0] += len;
            acc[1] += kept;
            acc[3] += kept;
        }
        __builtin_amdgcn_wave_barrier();
    }
}

// one chunk of a long row (phase 2); thread t holds entries [8t, 8t + 8) of the chunk, in order
__device__ void prune_chunk(const PruneArgs& a, uint32_t c, uint32_t* s_w, uint32_t& s_pfx, unsigned long long* acc) {
    const uint32_t lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    const uint64_t m = a.chunk_map[c];
    const uint32_t h = (uint32_t)m, first = (uint32_t)(m >> 32);
    const uint32_t len = a.row_len[h];   // the row's last chunk rewrites it only after this chunk published
    const uint64_t o = a.row_off[h];
    const uint32_t base = (c - first) * kChunk;
    uint32_t col[kChunkPer];
    uint64_t tag[kChunkPer];
#pragma unroll
    for (int j = 0; j < kChunkPer; ++j) {
        const uint32_t k = base + threadIdx.x * kChunkPer + j;
        col[j] = k < len ? pr_ld(a.pool_col + o + k) : 0u;
        tag[j] = k < len ? pr_ld(a.pool_tag + o + k) : 0ull;
    }
    uint32_t keep = 0;
#pragma unroll
    for (int j = 0; j < kChunkPer; ++j) {
        const uint32_t k = base + threadIdx.x * kChunkPer + j;
        keep |= (k < len && entry_live(a, o + k, col[j], tag[j])) ? (1u << j) : 0u;
    }
    const uint32_t cnt = (uint32_t)__popc(keep);
    uint32_t x = cnt;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        const uint32_t y = __shfl_up(x, d, 64);
        if (lane >= (uint32_t)d) x += y;
    }
    if (lane == 63) s_w[wid] = x;
    __syncthreads();   // every entry of the chunk is in registers (its liveness used them)
    uint32_t before = x - cnt, all = 0;
#pragma unroll
    for (uint32_t q = 0; q < 4; ++q) {
        before += q < wid ? s_w[q] : 0u;
        all += s_w[q];
    }
    // the flag hands over no data (the count travels in it): relaxed, no release / acquire fences
    // (MI355X_MICROARCH.md: an agent release writes back the XCD's L2, an acquire poll invalidates L1)
    if (threadIdx.x == 0) __hip_atomic_store(&a.chunk_st[c], kChunkDone | all, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (wid == 0) {   // the row's earlier chunks: all published (loaded), their kept counts summed
        uint32_t pfx = 0;
        for (uint32_t j = first + lane; j < c; j += 64) {
            uint32_t v = __hip_atomic_load(&a.chunk_st[j], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            while (!(v & kChunkDone)) {
                __builtin_amdgcn_s_sleep(2);
                v = __hip_atomic_load(&a.chunk_st[j], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            }
            pfx += v & ~kChunkDone;
        }
        for (int d = 32; d >= 1; d >>= 1) pfx += __shfl_xor(pfx, d, 64);
        if (lane == 0) s_pfx = pfx;
    }
    __syncthreads();
    const uint32_t pfx = s_pfx;
    uint32_t at = pfx + before;
#pragma unroll
    for (int j = 0; j < kChunkPer; ++j)
        if ((keep >> j) & 1u) {
            pr_st(a.pool_col + o + at, col[j]);
            pr_st(a.pool_tag + o + at, tag[j]);
            ++at;
        }
    if (threadIdx.x == 0 && base + kChunk >= len) {   // the row's last chunk
        a.row_len[h] = pfx + all;
        acc[0] += len;
        acc[1] += pfx + all;
        acc[3] += pfx + all;
    }
    __syncthreads();   // s_w, s_pfx reused by the next chunk
}

__global__ void k_coop_warm(uint32_t) {}

// bit h: handle h's node is current (not Invalidated, not empty) — the prune's fast path
__global__ void k_build_cur(uint32_t n, const unsigned long long* __restrict__ node, unsigned long long* cur64) {
    const uint64_t nthr = (uint64_t)gridDim.x * blockDim.x;
    const uint64_t lim = ((uint64_t)n + 63) / 64 * 64;
    for (uint64_t h = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; h < lim; h += nthr) {
        const bool c = h < n && word_is_current(node[h]);
        const unsigned long long m = __ballot(c);
        if ((threadIdx.x & 63) == 0) cur64[h >> 6] = m;
    }
}

}  // namespace

// The runtime sets up cooperative launches on their first use in a process, which costs tens of ms:
// paid once per graph before the first timed cooperative launch (prune, streaming batches), not at
// fgi_create, so processes that never launch cooperatively never pay it.
fgi_status coop_warm(fgi_graph* g) {
    if (g->coop_warm) return FGI_OK;
    uint32_t zero = 0;
    void* args[] = {&zero};
    FGI_HIP(g, hipLaunchCooperativeKernel(reinterpret_cast<const void*>(k_coop_warm), dim3(1), dim3(64), args, 0, g->stream));
    FGI_HIP(g, hipStreamSynchronize(g->stream));
    g->coop_warm = true;
    return FGI_OK;
}

namespace {

// Block-reduced prune counters added to st[] (one atomic per wave and counter).
__device__ __forceinline__ void prune_flush(const PruneArgs& a, unsigned long long (&acc)[4]) {
    const uint32_t lane = threadIdx.x & 63;
#pragma unroll
    for (int q = 0; q < 4; ++q)
        for (int d = 32; d >= 1; d >>= 1) acc[q] += __shfl_xor(acc[q], d, 64);
    if (lane == 0) {
        if (acc[0]) atomicAdd(&a.st[kPrOld], acc[0]);
        if (acc[1]) atomicAdd(&a.st[kPrNew], acc[1]);
        if (acc[2]) atomicAdd(&a.st[kPrDropped], acc[2]);
        if (acc[3]) atomicAdd(&a.st[kPrLive], acc[3]);
    }
}

// Phase 1 of a prune: the short rows (one wave each) and, for each long row, its chunks' entries in
// the chunk map. Phase 2 (k_prune_chunks) runs in the next launch: the kernel boundary is the grid
// barrier between them (plain launches: a cooperative launch's dispatch gap is ~11.7 us).
__global__ __launch_bounds__(256) void k_prune_rows(PruneArgs a) {
    __shared__ uint32_t s_lh[kBlockLong], s_lc[kBlockLong];
    __shared__ uint32_t s_nl, s_cb;
    if (threadIdx.x == 0) s_nl = 0;
    __syncthreads();
    unsigned long long acc[4] = {0, 0, 0, 0};   // old, new, dropped, live
    prune_short_rows(a, s_lh, s_lc, s_nl, acc);
    __syncthreads();
    // this block's long rows: one range of chunk indices
    const uint32_t nl = std::min<uint32_t>(s_nl, kBlockLong);
    if (threadIdx.x == 0) {
        uint32_t tot = 0;
        for (uint32_t q = 0; q < nl; ++q) tot += s_lc[q];
        s_cb = tot ? (uint32_t)atomicAdd(&a.st[kPrChunks], (unsigned long long)tot) : 0u;
    }
    __syncthreads();
    uint32_t cb = s_cb;
    for (uint32_t q = 0; q < nl; ++q) {
        prune_map_row(a.chunk_map, s_lh[q], cb, s_lc[q], threadIdx.x, blockDim.x);
        cb += s_lc[q];
    }
    prune_flush(a, acc);
}

// Phase 2: the long rows' chunks, each compacted in place after its row's earlier chunks (chunk_st).
__global__ __launch_bounds__(256) void k_prune_chunks(PruneArgs a) {
    __shared__ uint32_t s_w[4], s_pfx;
    unsigned long long acc[4] = {0, 0, 0, 0};
    const uint32_t n_chunks = (uint32_t)__hip_atomic_load(&a.st[kPrChunks], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    for (uint32_t c = blockIdx.x; c < n_chunks; c += gridDim.x) prune_chunk(a, c, s_w, s_pfx, acc);
    prune_flush(a, acc);
}

// Defragmentation: every row copied to a fresh pool at the exclusive scan of its new capacity
// (length + slack); one wave per row.
__global__ void k_defrag_rows(uint32_t n, const uint64_t* __restrict__ new_off, const uint64_t* __restrict__ row_off,
                              const uint32_t* __restrict__ row_len, const uint32_t* __restrict__ pool_col,
                              const uint64_t* __restrict__ pool_tag, uint32_t* ncol, uint64_t* ntag) {
    const uint32_t lane = threadIdx.x & 63;
    const uint64_t nw = ((uint64_t)gridDim.x * blockDim.x) >> 6;
    for (uint64_t h = ((uint64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6; h < n; h += nw) {
        const uint32_t len = row_len[h];
        const uint64_t o = row_off[h], d = new_off[h];
        for (uint32_t k = lane; k < len; k += 64) {
            ncol[d + k] = pool_col[o + k];
            ntag[d + k] = pool_tag[o + k];
        }
    }
}

__device__ __forceinline__ uint32_t row_slack_cap(uint32_t len) { return len == 0 ? 0u : len + std::max<uint32_t>(4u, len / 8); }

__global__ void k_defrag_caps(uint32_t n, const uint32_t* __restrict__ row_len, uint64_t* cap64) {
    const uint32_t h = blockIdx.x * blockDim.x + threadIdx.x;
    if (h < n) cap64[h] = row_slack_cap(row_len[h]);
}

__global__ void k_defrag_apply(uint32_t n, const uint64_t* __restrict__ new_off, const uint64_t* __restrict__ cap64,
                               uint64_t* row_off, uint32_t* row_cap) {
    const uint32_t h = blockIdx.x * blockDim.x + threadIdx.x;
    if (h >= n) return;
    row_off[h] = new_off[h];
    row_cap[h] = (uint32_t)cap64[h];
}

// ---- dependency-list cache (pull levels) ------------------------------------------------------
// For every `_usedBy` entry (d, tag) of every row owner u with tag == version(d): d depends on u.
// Inclusion depends only on rows and versions, never on node states, so the cache survives waves
// and fgi_restore; every mutation of rows or versions invalidates it (touch()).
__global__ void k_in_count(uint32_t n, const unsigned long long* __restrict__ node, const uint64_t* __restrict__ row_off,
                           const uint32_t* __restrict__ row_len, const uint32_t* __restrict__ pool_col,
                           const uint64_t* __restrict__ pool_tag, uint32_t* cnt) {
    const uint64_t wave = ((uint64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
    const uint32_t lane = threadIdx.x & 63;
    const uint64_t nw = ((uint64_t)gridDim.x * blockDim.x) >> 6;
    for (uint64_t u = wave; u < n; u += nw) {
        const uint32_t len = row_len[u];
        const uint64_t o = row_off[u];
        for (uint32_t k = lane; k < len; k += 64) {
            const uint32_t d = pool_col[o + k];
            const uint64_t t = pool_tag[o + k];
            if (t != 0 && (node[d] & kVMask) == t) atomicAdd(&cnt[d], 1u);
        }
    }
}

// One sort pair per pool position: a live entry (d, tag == version(d)) of row u gives
// key = (d << wbits) | (wmax - weight(u)), value = u; dead entries and row slack get a key past every
// live one (bit `top`), so an ascending stable sort leaves the lists, each ordered by weight
// descending, in the first `total` positions.
__global__ void k_in_pairs(uint32_t n, uint32_t n_slots, const unsigned long long* __restrict__ node,
                           const uint64_t* __restrict__ row_off, const uint32_t* __restrict__ row_len,
                           const uint32_t* __restrict__ pool_col, const uint64_t* __restrict__ pool_tag,
                           const uint32_t* __restrict__ weight, uint32_t wbits, uint32_t wmax, uint32_t top,
                           uint64_t* keys, uint32_t* vals, unsigned long long* live_bm) {
    const uint64_t wave = ((uint64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
    const uint32_t lane = threadIdx.x & 63;
    const uint64_t nw = ((uint64_t)gridDim.x * blockDim.x) >> 6;
    const uint64_t dead = 1ull << top;
    for (uint64_t u = wave; u < n; u += nw) {
        const uint32_t len = row_len[u];
        const uint64_t o = row_off[u];
        const uint64_t wk = (uint64_t)(wmax - (u < n_slots ? weight[u] : 0u));
        for (uint32_t k0 = 0; k0 < len; k0 += 64) {   // wave-uniform
            const uint32_t k = k0 + lane;
            bool live = false;
            if (k < len) {
                const uint32_t d = pool_col[o + k];
                const uint64_t t = pool_tag[o + k];
                live = t != 0 && (node[d] & kVMask) == t;
                keys[o + k] = live ? (((uint64_t)d << wbits) | wk) : dead;
                vals[o + k] = (uint32_t)u;
            }
            // positions o + k0 .. + 63: at most two words of the liveness bitmap (rows share words)
            const unsigned long long m = __ballot(live);
            if (live_bm && lane == 0 && m) {
                const uint64_t p0 = o + k0;
                const uint32_t sh = (uint32_t)(p0 & 63);
                atomicOr(live_bm + (p0 >> 6), m << sh);
                if (sh && (m >> (64 - sh))) atomicOr(live_bm + (p0 >> 6) + 1, m >> (64 - sh));
            }
        }
    }
}

// heads (first two entries) and the "more than two entries" bitmap, one 64-bit word per wave
__global__ void k_in_head(uint32_t n, const uint64_t* __restrict__ uin_off, const uint32_t* __restrict__ uin_len,
                          const uint32_t* __restrict__ uin_src, uint64_t* head, unsigned long long* more64) {
    const uint32_t d = blockIdx.x * blockDim.x + threadIdx.x;
    const uint32_t len = d < n ? uin_len[d] : 0u;
    const unsigned long long m = __ballot(len > 2);
    if ((threadIdx.x & 63) == 0 && d < n) more64[d >> 6] = m;
    if (d >= n) return;
    const uint64_t off = uin_off[d];
    const uint32_t h0 = len > 0 ? uin_src[off] : FGI_NONE;
    const uint32_t h1 = len > 1 ? uin_src[off + 1] : FGI_NONE;
    head[d] = (uint64_t)h0 | ((uint64_t)h1 << 32);
}

// Sort keys of the dependency lists: (weight of the entry << ubits) | entry, weight = the entry's
// own number of dependencies (its list length; 0 for detached handles).
__global__ void k_in_keys(uint64_t m, const uint32_t* __restrict__ uin_src, const uint32_t* __restrict__ uin_len,
                          uint32_t n_slots, uint32_t ubits, uint64_t* keys) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= m) return;
    const uint32_t u = uin_src[i];
    const uint64_t w = u < n_slots ? uin_len[u] : 0u;
    keys[i] = (w << ubits) | u;
}

__global__ void k_in_unkey(uint64_t m, const uint64_t* __restrict__ keys, uint32_t ubits, uint32_t* uin_src) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < m) uin_src[i] = (uint32_t)(keys[i] & ((1ull << ubits) - 1ull));
}

__global__ void k_in_ends(uint32_t n, const uint64_t* __restrict__ off, const uint32_t* __restrict__ len, uint64_t* end) {
    const uint32_t d = blockIdx.x * blockDim.x + threadIdx.x;
    if (d < n) end[d] = off[d] + len[d];
}

// pull candidates: slots with a non-empty dependency list, in slot order
__global__ void k_cand_flag(uint32_t n, const uint32_t* __restrict__ uin_len, uint32_t* flag) {
    const uint32_t d = blockIdx.x * blockDim.x + threadIdx.x;
    if (d < n) flag[d] = uin_len[d] ? 1u : 0u;
}

// how often each handle heads a candidate's list (first or second entry)
__global__ void k_head_count(uint32_t n, const uint32_t* __restrict__ flag, const uint64_t* __restrict__ uin_head,
                             uint32_t* cnt) {
    const uint32_t d = blockIdx.x * blockDim.x + threadIdx.x;
    if (d >= n || !flag[d]) return;
    const uint64_t h = uin_head[d];
    const uint32_t h0 = (uint32_t)h, h1 = (uint32_t)(h >> 32);
    if (h0 != FGI_NONE) atomicAdd(cnt + h0, 1u);
    if (h1 != FGI_NONE) atomicAdd(cnt + h1, 1u);
}

__global__ void k_head_keys(uint32_t n, const uint32_t* __restrict__ cnt, uint64_t* keys) {
    const uint32_t u = blockIdx.x * blockDim.x + threadIdx.x;
    if (u < n) keys[u] = ((uint64_t)cnt[u] << 32) | u;
}

// ranks 0..kHot-1 to the most frequent heads (keys sorted by count, descending)
__global__ void k_hot_pick(uint32_t k_max, uint32_t n_hot, const uint64_t* __restrict__ sorted, uint32_t* hot_id,
                           uint32_t* hot_rank) {
    const uint32_t k = blockIdx.x * blockDim.x + threadIdx.x;
    if (k >= n_hot) return;
    const uint64_t key = k < k_max ? sorted[k] : 0ull;
    if ((key >> 32) == 0) {
        hot_id[k] = FGI_NONE;
        return;
    }
    hot_id[k] = (uint32_t)key;
    hot_rank[(uint32_t)key] = k;
}

// a list head as the pull level probes it: its bit in the invalidated bitmap, or, for a hot head, its
// bit in the snapshot that follows the bitmap (bit hot_bit0 + rank)
__device__ __forceinline__ uint32_t head_code(uint32_t h, const uint32_t* hot_rank, uint32_t hot_bit0) {
    if (h == FGI_NONE || !hot_rank) return h;
    const uint32_t r = hot_rank[h];
    return r != FGI_NONE ? (hot_bit0 + r) : h;
}

__global__ void k_cand_fill(uint32_t n, const uint32_t* __restrict__ flag, const uint32_t* __restrict__ pos,
                            const uint64_t* __restrict__ uin_head, const uint32_t* __restrict__ uin_len,
                            const uint32_t* __restrict__ row_len, const uint32_t* __restrict__ hot_rank,
                            uint32_t hot_bit0, uint4* cand, unsigned long long* too_long) {
    const uint32_t d = blockIdx.x * blockDim.x + threadIdx.x;
    if (d >= n || !flag[d]) return;
    const uint32_t p = pos[d], rl = row_len[d];
    if (rl >> 31) atomicAdd(too_long, 1ull);
    const uint64_t h = uin_head[d];
    cand[p] = make_uint4(d, (rl & 0x7FFFFFFFu) | (uin_len[d] > 2 ? 0x80000000u : 0u),
                         head_code((uint32_t)h, hot_rank, hot_bit0), head_code((uint32_t)(h >> 32), hot_rank, hot_bit0));
}

// segment base of pull block b: the candidates before its first slot b * tpb * kPullTile
__global__ void k_cand_seg(uint32_t G, uint64_t span, uint32_t n, const uint32_t* __restrict__ pos, uint32_t total,
                           uint32_t* seg) {
    const uint32_t b = blockIdx.x * blockDim.x + threadIdx.x;
    if (b > G) return;
    const uint64_t s0 = (uint64_t)b * span;
    seg[b] = s0 < n ? pos[s0] : total;
}

__global__ void k_invalidate_all_roots(uint32_t n_slots, const unsigned long long* node, uint32_t* roots,
                                       unsigned long long* cnt) {
    const uint32_t s = blockIdx.x * blockDim.x + threadIdx.x;
    if (s < n_slots && word_is_current(node[s])) roots[atomicAdd(cnt, 1ull)] = s;
}

inline uint32_t nblk(uint64_t n, uint32_t b = 256) { return (uint32_t)((n + b - 1) / b); }

template <class T>
fgi_status h2d(fgi_graph* g, T* dst, const T* src, size_t count) {
    if (count == 0) return FGI_OK;
    FGI_HIP(g, hipMemcpyAsync(dst, src, count * sizeof(T), hipMemcpyHostToDevice, g->stream));
    return FGI_OK;
}
template <class T>
fgi_status d2h(fgi_graph* g, T* dst, const T* src, size_t count) {
    if (count == 0) return FGI_OK;
    FGI_HIP(g, hipMemcpyAsync(dst, src, count * sizeof(T), hipMemcpyDeviceToHost, g->stream));
    FGI_HIP(g, hipStreamSynchronize(g->stream));
    return FGI_OK;
}

// gather all live edges (rows of current nodes) into fresh device arrays keys/tags
fgi_status gather_live(fgi_graph* g, Tmp& tk, Tmp& tt, uint64_t** keys, uint64_t** tags, uint64_t extra,
                       uint64_t* out_m) {
    const uint32_t H = g->n_handles;
    Tmp tl, to, ts;
    uint32_t* live;
    uint64_t* off;
    FGI_TRY(tmalloc(g, tl, &live, H));
    FGI_TRY(tmalloc(g, to, &off, (size_t)H + 1));
    hipLaunchKernelGGL(k_live_len, dim3(nblk(H)), dim3(256), 0, g->stream, H,
                       reinterpret_cast<const unsigned long long*>(g->node), g->row_len, live);
    size_t tb = 0;
    FGI_HIP(g, rocprim::exclusive_scan(nullptr, tb, live, off, (uint64_t)0, (size_t)H + 0, rocprim::plus<uint64_t>(),
                                       g->stream));
    void* tmp;
    FGI_TRY(tmalloc(g, ts, reinterpret_cast<char**>(&tmp), tb));
    FGI_HIP(g, rocprim::exclusive_scan(tmp, tb, live, off, (uint64_t)0, (size_t)H, rocprim::plus<uint64_t>(), g->stream));
    uint64_t last_off = 0;
    uint32_t last_len = 0;
    FGI_TRY(d2h(g, &last_off, off + H - 1, 1));
    FGI_TRY(d2h(g, &last_len, live + H - 1, 1));
    const uint64_t m = last_off + last_len;
    FGI_TRY(tmalloc(g, tk, keys, m + extra));
    FGI_TRY(tmalloc(g, tt, tags, m + extra));
    if (m)
        hipLaunchKernelGGL(k_gather_live, dim3(std::min<uint64_t>(nblk((uint64_t)H * 64), 65536)), dim3(256), 0,
                           g->stream, H, live, off, g->row_off, g->pool_col, g->pool_tag, *keys, *tags);
    FGI_HIP(g, hipGetLastError());
    *out_m = m;
    return FGI_OK;
}

}  // namespace

// the chunk maps of the two frontier lists: one entry per kFine edges of a level's frontier
fgi_status ensure_cstart(fgi_graph* g, uint64_t total_edges) {
    const uint64_t need = total_edges / kFine + 4;
    if (g->cstart_cap >= need) return FGI_OK;
    dfree(g->cstart[0]);
    dfree(g->cstart[1]);
    const uint64_t cap = std::max<uint64_t>(need, g->cstart_cap * 3 / 2);
    FGI_TRY(dmalloc(g, &g->cstart[0], cap));
    FGI_TRY(dmalloc(g, &g->cstart[1], cap));
    g->cstart_cap = cap;
    return FGI_OK;
}

fgi_status ensure_pool(fgi_graph* g, uint64_t entries) {
    if (g->pool_cap >= entries && g->pool_col) return FGI_OK;
    // pool positions are 32-bit inside the expand kernel's LDS chunk map: 2^32 entries (48 GB of
    // pool) per device; beyond that, partition the graph over more devices
    constexpr uint64_t kMaxPool = 1ull << 32;
    if (entries > kMaxPool)
        return set_err(g, FGI_ENOTSUP, "edge pool of %llu entries exceeds 2^32 per device", (unsigned long long)entries);
    const uint64_t cap = std::min<uint64_t>(std::max<uint64_t>({entries, g->pool_cap + g->pool_cap / 2, (uint64_t)1024}),
                                            kMaxPool);
    uint32_t* col = nullptr;
    uint64_t* tag = nullptr;
    FGI_TRY(dmalloc(g, &col, cap));
    fgi_status st = dmalloc(g, &tag, cap);
    if (st != FGI_OK) {
        hipFree(col);
        return st;
    }
    if (g->pool_top) {
        FGI_HIP(g, hipMemcpyAsync(col, g->pool_col, g->pool_top * sizeof(uint32_t), hipMemcpyDeviceToDevice, g->stream));
        FGI_HIP(g, hipMemcpyAsync(tag, g->pool_tag, g->pool_top * sizeof(uint64_t), hipMemcpyDeviceToDevice, g->stream));
        FGI_HIP(g, hipStreamSynchronize(g->stream));
    }
    dfree(g->pool_col);
    dfree(g->pool_tag);
    g->pool_col = col;
    g->pool_tag = tag;
    g->pool_cap = cap;
    return ensure_cstart(g, cap);
}

fgi_status ensure_in_lists(fgi_graph* g) {
    if (g->uin_epoch == g->mut_epoch && g->uin_src) return FGI_OK;
    hipStream_t s = g->stream;
    const uint32_t H = g->n_handles, N = g->n_slots;
    const uint32_t grid = std::min<uint64_t>(nblk((uint64_t)H * 64), 16384);
    FGI_HIP(g, hipMemsetAsync(g->uin_len, 0, (size_t)N * 4, s));
    hipLaunchKernelGGL(k_in_count, dim3(grid), dim3(256), 0, s, H, reinterpret_cast<const unsigned long long*>(g->node),
                       g->row_off, g->row_len, g->pool_col, g->pool_tag, g->uin_len);
    Tmp ts;
    size_t tb = 0;
    FGI_HIP(g, rocprim::exclusive_scan(nullptr, tb, g->uin_len, g->uin_off, (uint64_t)0, (size_t)N,
                                       rocprim::plus<uint64_t>(), s));
    char* tmp;
    FGI_TRY(tmalloc(g, ts, &tmp, tb));
    FGI_HIP(g, rocprim::exclusive_scan(tmp, tb, g->uin_len, g->uin_off, (uint64_t)0, (size_t)N,
                                       rocprim::plus<uint64_t>(), s));
    uint64_t last_off = 0;
    uint32_t last_len = 0;
    FGI_TRY(d2h(g, &last_off, g->uin_off + N - 1, 1));
    FGI_TRY(d2h(g, &last_len, g->uin_len + N - 1, 1));
    const uint64_t total = last_off + last_len;
    if (total > g->uin_cap || !g->uin_src) {
        dfree(g->uin_src);
        const uint64_t cap = std::max<uint64_t>(total, 1024);
        FGI_TRY(dmalloc(g, &g->uin_src, cap));
        g->uin_cap = cap;
    }
    // Fill and order the lists with one stable radix sort of (dependant, weight) pairs over the pool:
    // every list ordered by its entries' own dependency counts (descending; ties in pool order), so a
    // pull level finds a parent in the frontier among the first entries (in the two heads, mostly).
    uint32_t wmax = 0;
    {
        Tmp tr, tm;
        uint32_t* dmax;
        FGI_TRY(tmalloc(g, tm, &dmax, 1));
        size_t rb = 0;
        FGI_HIP(g, rocprim::reduce(nullptr, rb, g->uin_len, dmax, 0u, (size_t)N, rocprim::maximum<uint32_t>(), s));
        char* rt;
        FGI_TRY(tmalloc(g, tr, &rt, rb));
        FGI_HIP(g, rocprim::reduce(rt, rb, g->uin_len, dmax, 0u, (size_t)N, rocprim::maximum<uint32_t>(), s));
        FGI_TRY(d2h(g, &wmax, dmax, 1));
    }
    uint32_t wbits = 1, dbits = 1;
    while (wbits < 32 && (1ull << wbits) <= wmax) ++wbits;
    while (dbits < 32 && (1ull << dbits) < N) ++dbits;
    const uint32_t top = dbits + wbits;   // the dead-entry bit
    const uint64_t P = g->pool_top;
    if (total && P) {
        if (top >= 64) return set_err(g, FGI_EINVAL, "dependency-list sort key needs %u bits", top + 1);
        Tmp tk0, tk1, tv0, tv1, tt;
        uint64_t *k0, *k1;
        uint32_t *v0, *v1;
        FGI_TRY(tmalloc(g, tk0, &k0, P));
        FGI_TRY(tmalloc(g, tk1, &k1, P));
        FGI_TRY(tmalloc(g, tv0, &v0, P));
        FGI_TRY(tmalloc(g, tv1, &v1, P));
        FGI_HIP(g, hipMemsetAsync(k0, 0xFF, P * sizeof(uint64_t), s));   // row slack: dead keys
        // the pool's liveness bitmap (fgi_prune's fast path) comes with the lists
        const uint64_t lw = (P + 63) / 64 + 1;
        if (g->pool_live_cap < lw * 64) {
            dfree(g->pool_live);
            g->pool_live_cap = 0;
            FGI_TRY(dmalloc(g, &g->pool_live, lw + lw / 8));
            g->pool_live_cap = (lw + lw / 8) * 64;
        }
        FGI_HIP(g, hipMemsetAsync(g->pool_live, 0, lw * 8, s));
        hipLaunchKernelGGL(k_in_pairs, dim3(grid), dim3(256), 0, s, H, N,
                           reinterpret_cast<const unsigned long long*>(g->node), g->row_off, g->row_len, g->pool_col,
                           g->pool_tag, g->uin_len, wbits, wmax, top, k0, v0, g->pool_live);
        FGI_HIP(g, hipGetLastError());
        size_t sb = 0;
        FGI_HIP(g, rocprim::radix_sort_pairs(nullptr, sb, k0, k1, v0, v1, (size_t)P, 0, top + 1, s));
        char* st;
        FGI_TRY(tmalloc(g, tt, &st, sb));
        FGI_HIP(g, rocprim::radix_sort_pairs(st, sb, k0, k1, v0, v1, (size_t)P, 0, top + 1, s));
        FGI_HIP(g, hipMemcpyAsync(g->uin_src, v1, total * sizeof(uint32_t), hipMemcpyDeviceToDevice, s));
        FGI_HIP(g, hipStreamSynchronize(s));   // the temporaries go back to the cache
    }
    FGI_TRY(build_in_heads(g));
    FGI_HIP(g, hipStreamSynchronize(s));
    g->uin_epoch = g->mut_epoch;
    g->pl_mut_epoch = (total && P) ? g->mut_epoch : 0;
    g->pl_pool_epoch = g->pool_epoch;
    return FGI_OK;
}

// Orders every dependency list by weight[entry] (descending; ties by the larger id; entries at or
// past n_weight weigh 0). total = entries over all lists.
fgi_status sort_in_lists(fgi_graph* g, uint64_t total, const uint32_t* weight, uint32_t n_weight) {
    if (total <= 1) return FGI_OK;
    hipStream_t s = g->stream;
    const uint32_t N = g->n_slots;
    const uint64_t ids = std::max<uint64_t>(g->n_handles, n_weight);
    uint32_t ubits = 1;
    while (ubits < 32 && (1ull << ubits) < ids) ++ubits;
    uint32_t max_w = 0;
    {
        Tmp tr, tm;
        uint32_t* dmax;
        FGI_TRY(tmalloc(g, tm, &dmax, 1));
        size_t rb = 0;
        FGI_HIP(g, rocprim::reduce(nullptr, rb, weight, dmax, 0u, (size_t)n_weight, rocprim::maximum<uint32_t>(), s));
        char* rt;
        FGI_TRY(tmalloc(g, tr, &rt, rb));
        FGI_HIP(g, rocprim::reduce(rt, rb, weight, dmax, 0u, (size_t)n_weight, rocprim::maximum<uint32_t>(), s));
        FGI_TRY(d2h(g, &max_w, dmax, 1));
    }
    uint32_t wbits = 1;
    while (wbits < 32 && (1ull << wbits) <= max_w) ++wbits;
    Tmp tk0, tk1, te, tt;
    uint64_t *k0, *k1, *ends;
    FGI_TRY(tmalloc(g, tk0, &k0, total));
    FGI_TRY(tmalloc(g, tk1, &k1, total));
    FGI_TRY(tmalloc(g, te, &ends, N));
    hipLaunchKernelGGL(k_in_keys, dim3(nblk(total)), dim3(256), 0, s, total, g->uin_src, weight, n_weight, ubits, k0);
    hipLaunchKernelGGL(k_in_ends, dim3(nblk(N)), dim3(256), 0, s, N, g->uin_off, g->uin_len, ends);
    size_t sb = 0;
    FGI_HIP(g, rocprim::segmented_radix_sort_keys_desc(nullptr, sb, k0, k1, (unsigned)total, N, g->uin_off, ends, 0,
                                                       ubits + wbits, s));
    char* st;
    FGI_TRY(tmalloc(g, tt, &st, sb));
    FGI_HIP(g, rocprim::segmented_radix_sort_keys_desc(st, sb, k0, k1, (unsigned)total, N, g->uin_off, ends, 0,
                                                       ubits + wbits, s));
    hipLaunchKernelGGL(k_in_unkey, dim3(nblk(total)), dim3(256), 0, s, total, k1, ubits, g->uin_src);
    FGI_HIP(g, hipGetLastError());
    FGI_HIP(g, hipStreamSynchronize(s));
    return FGI_OK;
}

fgi_status build_in_heads(fgi_graph* g) {
    const uint32_t N = g->n_slots;
    hipLaunchKernelGGL(k_in_head, dim3(nblk(N)), dim3(256), 0, g->stream, N, g->uin_off, g->uin_len, g->uin_src,
                       g->uin_head, reinterpret_cast<unsigned long long*>(g->uin_more));
    FGI_HIP(g, hipGetLastError());
    return build_candidates(g);
}

// The pull candidate segments for the graph's pull geometry (see fgi_internal.h). A graph too large
// to pull on one device, or with a row of 2^31 entries or more, gets none (its waves push).
// Hot heads for a graph of n handles: one per 256 handles, a power of two in [kHotMin, kHot]. A/B on
// one box (profiles/r5e_ab.txt): 64 Ki -> 256 Ki heads took configs[2]'s pull levels from 1.105 to
// 1.020 ms per wave; round 4 (profiles/r8d_hot_ab.txt): 512 Ki heads 0.989 ms (1.202-1.206 ms/step
// against 1.215-1.221), 1 Mi 0.983 ms of pull levels but no faster a step (the snapshot's refresh),
// 2 Mi slower; on configs[1] (65,536 heads either way) a snapshot past 64 Ki costs more to refresh
// than it saves.
#ifndef FGI_HOT_DIV
#define FGI_HOT_DIV 256   // measurement builds: make variant-hot HOT=<n> HOT_DIV=<handles per hot head>
#endif
uint32_t hot_count(uint64_t n) {
    uint32_t k = kHotMin;
    while (k < kHot && k < n / FGI_HOT_DIV) k <<= 1;
    return k;
}

fgi_status build_candidates(fgi_graph* g) {
    g->cand_grid = 0;
    uint32_t G = 0, tpb = 0;
    pull_geometry(g, &G, &tpb);
    if (G == 0) return FGI_OK;
    hipStream_t s = g->stream;
    const uint32_t N = g->n_slots;
    if (g->cand_cap < N || !g->cand) {
        dfree(g->cand);
        dfree(g->wl);
        for (int k = 0; k < 2; ++k) dfree(g->sv[k]);
        g->cand_cap = 0;
        FGI_TRY(dmalloc(g, &g->cand, N));
        FGI_TRY(dmalloc(g, &g->wl, N));
        for (int k = 0; k < 2; ++k) FGI_TRY(dmalloc(g, &g->sv[k], N));
        g->cand_cap = N;
    }
    if (!g->cand_seg) {   // sized for the largest pull grid
        FGI_TRY(dmalloc(g, &g->cand_seg, (size_t)kStatBlocks + 1));
        FGI_TRY(dmalloc(g, &g->sv_cnt[0], kStatBlocks));
        FGI_TRY(dmalloc(g, &g->sv_cnt[1], kStatBlocks));
    }
    Tmp tf, tp, ts;
    uint32_t *flag, *pos;
    FGI_TRY(tmalloc(g, tf, &flag, N));
    FGI_TRY(tmalloc(g, tp, &pos, N));
    hipLaunchKernelGGL(k_cand_flag, dim3(nblk(N)), dim3(256), 0, s, N, g->uin_len, flag);
    size_t tb = 0;
    FGI_HIP(g, rocprim::exclusive_scan(nullptr, tb, flag, pos, 0u, (size_t)N, rocprim::plus<uint32_t>(), s));
    char* tmp;
    FGI_TRY(tmalloc(g, ts, &tmp, tb));
    FGI_HIP(g, rocprim::exclusive_scan(tmp, tb, flag, pos, 0u, (size_t)N, rocprim::plus<uint32_t>(), s));
    uint32_t lp = 0, lf = 0;
    FGI_TRY(d2h(g, &lp, pos + N - 1, 1));
    FGI_TRY(d2h(g, &lf, flag + N - 1, 1));
    const uint32_t total = lp + lf;
    // hot heads (a partition's heads are global ids: ranked over all n_global slots, their snapshot
    // taken from the all-gathered invalidated bitmap)
    Tmp th;
    uint32_t* hot_rank = nullptr;
    g->n_hot = 0;
    PartView pv;
    const bool part = part_view(g, &pv);
    const uint32_t NH = part ? pv.n_global : g->n_handles;
    // the snapshot sits past the end of the bitmap a pull level probes (allocated with kHot / 32
    // spare words): the single engine's invalidated bitmap, a partition's all-gathered one
    g->hot_w0 = part ? pv.front_words_global : g->bm_words;
    if (g->hot_w0 * 32 + kHot < (uint64_t)FGI_NONE) {
        if (!g->hot_id) FGI_TRY(dmalloc(g, &g->hot_id, kHot));
        Tmp tc, tk0, tk1, tt;
        uint32_t* cnt;
        uint64_t *k0, *k1;
        FGI_TRY(tmalloc(g, tc, &cnt, NH));
        FGI_TRY(tmalloc(g, th, &hot_rank, NH));
        FGI_TRY(tmalloc(g, tk0, &k0, NH));
        FGI_TRY(tmalloc(g, tk1, &k1, NH));
        FGI_HIP(g, hipMemsetAsync(cnt, 0, (size_t)NH * 4, s));
        FGI_HIP(g, hipMemsetAsync(hot_rank, 0xFF, (size_t)NH * 4, s));
        hipLaunchKernelGGL(k_head_count, dim3(nblk(N)), dim3(256), 0, s, N, flag, g->uin_head, cnt);
        hipLaunchKernelGGL(k_head_keys, dim3(nblk(NH)), dim3(256), 0, s, NH, cnt, k0);
        size_t sb = 0;
        FGI_HIP(g, rocprim::radix_sort_keys_desc(nullptr, sb, k0, k1, (size_t)NH, 0, 64, s));
        char* st;
        FGI_TRY(tmalloc(g, tt, &st, sb));
        FGI_HIP(g, rocprim::radix_sort_keys_desc(st, sb, k0, k1, (size_t)NH, 0, 64, s));
        uint32_t n_hot = hot_count(NH);
        if (g->opt_hot_heads > 0)   // tests: most heads probed in the invalidated bitmap itself
            n_hot = std::min<uint32_t>(n_hot, (uint32_t)(g->opt_hot_heads + 255) / 256 * 256);
        hipLaunchKernelGGL(k_hot_pick, dim3(n_hot / 256), dim3(256), 0, s, NH, n_hot, k1, g->hot_id, hot_rank);
        FGI_HIP(g, hipGetLastError());
        FGI_HIP(g, hipStreamSynchronize(s));
        g->n_hot = n_hot;
    }
    FGI_HIP(g, hipMemsetAsync(g->misc_dev + 15, 0, sizeof(unsigned long long), s));
    hipLaunchKernelGGL(k_cand_fill, dim3(nblk(N)), dim3(256), 0, s, N, flag, pos, g->uin_head, g->uin_len, g->row_len,
                       hot_rank, (uint32_t)(g->hot_w0 * 32), g->cand, g->misc_dev + 15);
    hipLaunchKernelGGL(k_cand_seg, dim3(nblk(G + 1)), dim3(256), 0, s, G, (uint64_t)tpb * kPullTile, N, pos, total,
                       g->cand_seg);
    FGI_HIP(g, hipGetLastError());
    unsigned long long too_long = 0;
    FGI_TRY(d2h(g, &too_long, g->misc_dev + 15, 1));
    if (too_long == 0) g->cand_grid = G;
    if (getenv("FGI_TRACE"))
        fprintf(stderr, "[fgi] candidates: %u of %u slots, pull grid %u x %u tiles, %u hot heads, %llu rows too long\n", total,
                N, G, tpb, g->n_hot, (unsigned long long)too_long);
    return FGI_OK;
}

fgi_status build_rows_from_keys(fgi_graph* g, uint64_t m, uint64_t* keys, uint64_t* tags, uint64_t ver_seed,
                                uint32_t stale_pct, uint64_t stale_seed, uint32_t src_base, uint32_t dst_base) {
    hipStream_t s = g->stream;
    const uint32_t H = g->n_handles;
    // reset all rows (the pool is rebuilt from scratch)
    FGI_HIP(g, hipMemsetAsync(g->row_off, 0, (size_t)H * sizeof(uint64_t), s));
    FGI_HIP(g, hipMemsetAsync(g->row_len, 0, (size_t)H * sizeof(uint32_t), s));
    FGI_HIP(g, hipMemsetAsync(g->row_cap, 0, (size_t)H * sizeof(uint32_t), s));
    FGI_HIP(g, hipMemsetAsync(g->used_cnt, 0, (size_t)H * sizeof(uint32_t), s));
    g->pool_top = 0;
    g->pool_epoch++;
    touch(g);
    if (m == 0) return FGI_OK;
    if (m >= 0xFFFFFFF0ull) return set_err(g, FGI_ENOTSUP, "more than 2^32 edges on one device");
    // 1. sort by (used, dependant) [, tag as payload]
    Tmp tk2, tt2, ttmp;
    uint64_t *k2 = nullptr, *t2 = nullptr;
    FGI_TRY(tmalloc(g, tk2, &k2, m));
    if (tags) FGI_TRY(tmalloc(g, tt2, &t2, m));
    size_t tb = 0;
    if (tags)
        FGI_HIP(g, rocprim::radix_sort_pairs(nullptr, tb, keys, k2, tags, t2, (size_t)m, 0, 64, s));
    else
        FGI_HIP(g, rocprim::radix_sort_keys(nullptr, tb, keys, k2, (size_t)m, 0, 64, s));
    char* tmp;
    FGI_TRY(tmalloc(g, ttmp, &tmp, tb));
    if (tags)
        FGI_HIP(g, rocprim::radix_sort_pairs(tmp, tb, keys, k2, tags, t2, (size_t)m, 0, 64, s));
    else
        FGI_HIP(g, rocprim::radix_sort_keys(tmp, tb, keys, k2, (size_t)m, 0, 64, s));
    // 2. set semantics: mark the first of each (used, dependant, tag)
    Tmp tkeep, tpos, tsc;
    uint32_t *keep, *pos;
    FGI_TRY(tmalloc(g, tkeep, &keep, m));
    FGI_TRY(tmalloc(g, tpos, &pos, m));
    hipLaunchKernelGGL(k_mark_unique, dim3(nblk(m)), dim3(256), 0, s, m, k2, t2, keep);
    size_t sb = 0;
    FGI_HIP(g, rocprim::exclusive_scan(nullptr, sb, keep, pos, 0u, (size_t)m, rocprim::plus<uint32_t>(), s));
    char* stmp;
    FGI_TRY(tmalloc(g, tsc, &stmp, sb));
    FGI_HIP(g, rocprim::exclusive_scan(stmp, sb, keep, pos, 0u, (size_t)m, rocprim::plus<uint32_t>(), s));
    uint32_t lastp = 0, lastk = 0;
    FGI_TRY(d2h(g, &lastp, pos + m - 1, 1));
    FGI_TRY(d2h(g, &lastk, keep + m - 1, 1));
    const uint64_t total = (uint64_t)lastp + lastk;
    // validate handles of the sorted keys: largest used handle is in the last key
    uint64_t maxkey = 0;
    FGI_TRY(d2h(g, &maxkey, k2 + m - 1, 1));
    if ((maxkey >> 32) >= H) return set_err(g, FGI_EINVAL, "used handle %u out of range", (unsigned)(maxkey >> 32));
    FGI_TRY(ensure_pool(g, total));
    hipLaunchKernelGGL(k_scatter_rows, dim3(nblk(m)), dim3(256), 0, s, m, k2, t2, keep, pos, ver_seed, stale_pct,
                       stale_seed, g->pool_col, g->pool_tag, g->row_off, g->row_len, g->used_cnt,
                       reinterpret_cast<const unsigned long long*>(g->node), g->n_slots, src_base, dst_base);
    hipLaunchKernelGGL(k_fix_rows, dim3(nblk(H)), dim3(256), 0, s, H, g->row_off, g->row_len, g->row_cap);
    FGI_HIP(g, hipGetLastError());
    FGI_HIP(g, hipStreamSynchronize(s));
    g->pool_top = total;
    FGI_HIP(g, hipMemcpy(g->pool_top_dev, &g->pool_top, sizeof(uint64_t), hipMemcpyHostToDevice));
    return FGI_OK;
}

// Existing live rows + m new entries (host keys: used handle << 32 | dependant id, host tags),
// rebuilt in one sort (set semantics across both).
fgi_status load_rows(fgi_graph* g, uint64_t m, const uint64_t* host_keys, const uint64_t* host_tags, uint32_t src_base,
                     uint32_t dst_base) {
    FGI_TRY(fold(g));
    Tmp tk, tt;
    uint64_t *keys, *tags, m0 = 0;
    FGI_TRY(gather_live(g, tk, tt, &keys, &tags, m, &m0));
    FGI_TRY(h2d(g, keys + m0, host_keys, m));
    FGI_TRY(h2d(g, tags + m0, host_tags, m));
    if (!g->part) {   // boundary handles -> labels (the first bulk load chooses the hot labels)
        if (m0 == 0) FGI_TRY(labels_choose(g, keys, m));
        FGI_TRY(labels_map_keys(g, keys + m0, m));
    }
    return build_rows_from_keys(g, m0 + m, keys, tags, 0, 0, 0, src_base, dst_base);
}

namespace {
// ---- partitioned mutations (part_* below): the kernels that differ from the single device's -----
// A partition's rows hold (global dependant, tag); node words, rows and |_used| counts are its own
// slots' (local handles), and every rank keeps a replica of all versions (ver_all).

__global__ void k_add_base(uint32_t n, uint32_t* a, uint32_t base) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) a[i] += base;
}

// the recomputed slots' new versions into the replica (every rank, every slot of the call)
__global__ void k_set_versions(uint32_t n, const uint32_t* __restrict__ slot, const uint64_t* __restrict__ ver,
                               uint64_t* ver_all) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) ver_all[slot[i]] = ver[i];
}

// AddUsed, phase A (Computed.cs:350-364), on the ranks owning dependants: 1 if the dependant is
// Computing, | 2 if it has captured dependencies before (only then can the used row hold the pair)
__global__ void k_pau_dep(uint32_t n, const uint32_t* __restrict__ dep, uint32_t base, uint32_t n_local,
                          const unsigned long long* __restrict__ node, const uint32_t* __restrict__ used_cnt, uint32_t* flag) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const uint32_t d = dep[i] - base;
    uint32_t f = 0;
    if (d < n_local) {
        const unsigned long long w = node[d];
        if ((w & kVMask) != 0 && word_state(w) == FGI_COMPUTING) f = 1u | (used_cnt[d] ? 2u : 0u);
    }
    flag[i] = f;
}

struct PauArgs {
    const uint32_t* dep;        // global dependant slots
    const uint32_t* used;       // global used slots
    uint32_t base, n_local;
    const unsigned long long* node;
    const uint64_t* ver_all;
    const uint32_t* dflag;      // phase A, all-reduced
    const uint64_t* row_off;
    const uint32_t* row_len;
    const uint32_t* pool_col;
    const uint64_t* pool_tag;
    unsigned long long* hset;
    uint64_t hmask;
    uint32_t* res;              // (code + 1) | appended << 8 on the used node's owner, else 0
    Cand* cand;
    unsigned long long* cnt;
};

// AddUsed, phase B, on the ranks owning the used nodes: AddUsedBy's rules (Computed.cs:370-385) and
// the entry (dependant, dependant's version) for the used row, set semantics within the batch and
// against the row
__device__ __forceinline__ bool pau_pair(uint32_t i, const PauArgs& a, Cand* out) {
    const uint32_t u = a.used[i] - a.base;
    if (u >= a.n_local) {
        a.res[i] = 0;
        return false;
    }
    const uint32_t d = a.dep[i], f = a.dflag[i];
    uint32_t code;
    bool add = false;
    const unsigned long long wu = a.node[u];
    if (!(f & 1u)) code = FGI_USED_DROPPED;
    else if ((wu & kVMask) == 0 || word_state(wu) == FGI_INVALIDATED) code = FGI_USED_INVALIDATED;
    else if (word_state(wu) == FGI_COMPUTING) code = FGI_USED_ESTATE;
    else {
        code = FGI_USED_ADDED;
        add = true;
        const unsigned long long key = ((unsigned long long)u << 32) | d;
        uint64_t p = sm64(key) & a.hmask;
        while (true) {
            const unsigned long long prev = atomicCAS(a.hset + p, ~0ull, key);
            if (prev == ~0ull) break;
            if (prev == key) {
                add = false;
                break;
            }
            p = (p + 1) & a.hmask;
        }
        const uint64_t tag = a.ver_all[d];
        if (add && (f & 2u)) {
            const uint64_t o = a.row_off[u];
            const uint32_t len = a.row_len[u];
            for (uint32_t k = 0; k < len && add; ++k)
                if (a.pool_col[o + k] == d && a.pool_tag[o + k] == tag) add = false;
        }
        if (add) *out = Cand{u, FGI_NONE, d, 0, tag};
    }
    a.res[i] = (code + 1u) | (add ? 0x100u : 0u);
    return add;
}

__global__ void k_pau_classify(uint32_t n, PauArgs a) {
    __shared__ uint32_t s_w[8];
    __shared__ unsigned long long s_base;
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    Cand cd{};
    const bool want = i < n && pau_pair(i, a, &cd);
    const unsigned long long m = __ballot(want);
    const uint32_t lane = threadIdx.x & 63, wid = threadIdx.x >> 6, nw = blockDim.x >> 6;
    if (lane == 0) s_w[wid] = (uint32_t)__popcll(m);
    __syncthreads();
    uint32_t before = 0, total = 0;
    for (uint32_t w = 0; w < nw; ++w) {
        before += w < wid ? s_w[w] : 0u;
        total += s_w[w];
    }
    if (threadIdx.x == 0) s_base = total ? atomicAdd(a.cnt, (unsigned long long)total) : 0ull;
    __syncthreads();
    if (want) {
        const uint32_t r = __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
        a.cand[s_base + before + r] = cd;
    }
}

// AddUsed, phase C, on the ranks owning dependants: InvalidateOnSetOutput for a used node found
// Invalidated (Computed.cs:376-378); for an appended entry, |_used| and the dependency-entry store
// (the dependant's pull list: used global id at the dependant's version)
__global__ void k_pau_apply(uint32_t n, const uint32_t* __restrict__ dep, const uint32_t* __restrict__ used,
                            uint32_t base, uint32_t n_local, const uint32_t* __restrict__ res, unsigned long long* node,
                            uint32_t* used_cnt, const uint64_t* __restrict__ ver_all, uint64_t* in_keys, uint64_t* in_tags,
                            unsigned long long* in_cnt) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const uint32_t d = dep[i] - base;
    if (d >= n_local) return;
    const uint32_t r = res[i];
    if ((r & 0xFFu) == FGI_USED_INVALIDATED + 1u) atomicOr(node + d, kW_IOSO);
    if (r & 0x100u) {
        atomicAdd(used_cnt + d, 1u);
        const unsigned long long k = atomicAdd(in_cnt, 1ull);
        in_keys[k] = ((uint64_t)d << 32) | used[i];
        in_tags[k] = ver_all[dep[i]];
    }
}
}  // namespace

}  // namespace fgi

using namespace fgi;

static fgi_status single_only(fgi_graph* g, const char* what);
// A graph a failed batch poisoned (fgi_run_batch, FGI_EDEVICE) takes no call but fgi_restore,
// fgi_destroy, fgi_last_error and fgi_set_option.
// a boundary handle's label, on the host (one lookup for a hot slot)
static fgi_status label_of(fgi_graph* g, uint32_t x, uint32_t* out) {
    if (g->lbl_perm) {   // a partition's local handle -> its code's local index
        *out = part_code_local_h(g, x, false);
        return FGI_OK;
    }
    if (!g->lbl_K) {
        *out = x;
        return FGI_OK;
    }
    if (g->lbl_hot && x < g->ext_slots) {
        uint32_t l = FGI_NONE;
        FGI_TRY(d2h(g, &l, g->s2l + x, 1));
        if (l != FGI_NONE) {
            *out = l;
            return FGI_OK;
        }
    }
    *out = x + g->lbl_K;
    return FGI_OK;
}

static fgi_status usable_now(fgi_graph* g) {
    return g->failed ? set_err(g, FGI_ESTATE, "a batch or wave failed on the device (%s); fgi_restore or fgi_destroy",
                               "grid barrier timeout or device wait")
                     : FGI_OK;
}
// every call but fgi_restore, fgi_set_option and the asynchronous wave calls first waits for the
// asynchronous waves in flight (their results are the graph's state the call sees)
static fgi_status usable(fgi_graph* g) {
    FGI_TRY(usable_now(g));
    if (g->aw[0].busy || g->aw[1].busy) {
        hipSetDevice(g->device);
        FGI_TRY(drain_async(g));
    }
    return FGI_OK;
}

extern "C" {

fgi_status fgi_version(uint32_t* major, uint32_t* minor) {
    if (major) *major = 0;
    if (minor) *minor = 1;
    return FGI_OK;
}

const char* fgi_last_error(const fgi_graph* g) { return g ? g->err.c_str() : "null graph"; }

fgi_status fgi_create(const fgi_config* cfg, fgi_graph** out) {
    // callers built against the fgi_config before `labels` pass the shorter struct (labels: auto)
    if (!cfg || !out || cfg->struct_size < offsetof(fgi_config, labels) || cfg->n_slots == 0) return FGI_EINVAL;
    const int labels = cfg->struct_size >= offsetof(fgi_config, labels) + sizeof(int32_t) ? cfg->labels : 0;
    const uint32_t K = cfg->world > 1 ? 0u : labels_capacity(cfg->n_slots, labels);
    if ((uint64_t)K + cfg->n_slots + cfg->n_detached >= 0xFFFFFFF0ull) return FGI_EINVAL;
    *out = nullptr;
    fgi_graph* g = new fgi_graph();
    g->device = cfg->device;
    g->opt_labels = labels;
    g->lbl_K = K;
    g->ext_slots = cfg->n_slots;
    g->ext_handles = cfg->n_slots + cfg->n_detached;
    g->n_slots = K + cfg->n_slots;
    g->n_detached = cfg->n_detached;
    g->n_handles = g->n_slots + cfg->n_detached;
    g->rank = cfg->rank;
    g->world = cfg->world > 0 ? cfg->world : 1;
    auto fail = [&](fgi_status st) {
        fgi_destroy(g);
        return st;
    };
    if (hipSetDevice(g->device) != hipSuccess) return fail(FGI_EDEVICE);
    if (hipStreamCreateWithFlags(&g->stream, hipStreamNonBlocking) != hipSuccess) return fail(FGI_EDEVICE);
    if (hipDeviceGetAttribute(&g->n_cu, hipDeviceAttributeMultiprocessorCount, g->device) != hipSuccess || g->n_cu <= 0)
        g->n_cu = 256;
    const size_t H = g->n_handles;
    if (dmalloc(g, &g->node, H) || dmalloc(g, &g->row_off, H) || dmalloc(g, &g->row_len, H) ||
        dmalloc(g, &g->row_cap, H) || dmalloc(g, &g->used_cnt, H) || dmalloc(g, &g->home, g->n_detached + 1) ||
        dmalloc(g, &g->inv, H) || dmalloc(g, &g->fr_off[0], H) || dmalloc(g, &g->fr_off[1], H) ||
        dmalloc(g, &g->fr_len[0], H) || dmalloc(g, &g->fr_len[1], H) || dmalloc(g, &g->escan[0], H) ||
        dmalloc(g, &g->escan[1], H) || dmalloc(g, &g->bsum, 8ull * kStatBlocks) ||
        dmalloc(g, &g->done, (size_t)(kDoneGroups + 1) * kDoneStride) || dmalloc(g, &g->ctr, 1) || dmalloc(g, &g->gbar, kGbarWords) ||
        dmalloc(g, &g->blk_stats, (size_t)kStatBlocks * kStatCols) || dmalloc(g, &g->misc_dev, 16) ||
        dmalloc(g, &g->pool_top_dev, 1) || dmalloc(g, &g->uin_off, H) || dmalloc(g, &g->uin_len, H) ||
        dmalloc(g, &g->uin_head, g->n_slots + 1))
        return fail(FGI_ENOMEM);
    g->bm_words = (H + 63) / 64 * 2 + 2;
    // the invalidated bitmap carries the hot heads' snapshot past its end (build_candidates)
    if (K && (dmalloc(g, &g->xbm, ((uint64_t)g->ext_handles + 63) / 64 + 2) ||
              dmalloc(g, &g->fold_status, ((uint64_t)g->ext_handles + kFoldTile - 1) / kFoldTile + kStatCols + 1)))
        return fail(FGI_ENOMEM);
    if (dmalloc(g, &g->vis_bm, g->bm_words) || dmalloc(g, &g->vis_spare, g->bm_words) ||
        dmalloc(g, &g->inv_bm, g->bm_words + kHot / 32) ||
        dmalloc(g, &g->cls_bm, g->bm_words) || dmalloc(g, &g->uin_more, g->bm_words) ||
        dmalloc(g, &g->sum_bm, ((uint64_t)H + 4095) / 4096 * 2 + 2))
        return fail(FGI_ENOMEM);
    hipMemset(g->done, 0, (size_t)(kDoneGroups + 1) * kDoneStride * sizeof(unsigned long long));
    hipMemset(g->bsum, 0, 8ull * kStatBlocks * sizeof(unsigned long long));
    hipMemset(g->gbar, 0, kGbarWords * sizeof(unsigned long long));
    hipMemset(g->vis_bm, 0, g->bm_words * 4);
    hipMemset(g->vis_spare, 0, g->bm_words * 4);
    hipMemset(g->inv_bm, 0, g->bm_words * 4);
    hipMemset(g->uin_more, 0, g->bm_words * 4);
    if (hipHostMalloc(reinterpret_cast<void**>(&g->ctr_host), sizeof(WaveCtr)) != hipSuccess ||
        hipHostMalloc(reinterpret_cast<void**>(&g->misc_host), 16 * sizeof(unsigned long long)) != hipSuccess ||
        hipHostMalloc(reinterpret_cast<void**>(&g->ctr_pub), sizeof(WaveCtr) + 128, hipHostMallocCoherent) != hipSuccess ||
        hipHostMalloc(reinterpret_cast<void**>(&g->red_pub), (kPartRedMax + 16) * 8, hipHostMallocCoherent) != hipSuccess)
        return fail(FGI_ENOMEM);
    memset(g->ctr_pub, 0, sizeof(WaveCtr) + 128);
    memset(g->red_pub, 0, (kPartRedMax + 16) * 8);
    hipMemset(g->node, 0, H * sizeof(uint64_t));
    hipMemset(g->row_off, 0, H * sizeof(uint64_t));
    hipMemset(g->row_len, 0, H * sizeof(uint32_t));
    hipMemset(g->row_cap, 0, H * sizeof(uint32_t));
    hipMemset(g->used_cnt, 0, H * sizeof(uint32_t));
    hipMemset(g->pool_top_dev, 0, sizeof(unsigned long long));
    if (hipEventCreateWithFlags(&g->ev_w0, hipEventDisableSystemFence) != hipSuccess ||
        hipEventCreateWithFlags(&g->ev_w1, hipEventDisableSystemFence) != hipSuccess) return fail(FGI_EDEVICE);
    g->free_detached.reserve(g->n_detached);
    for (uint32_t i = g->n_detached; i > 0; --i) g->free_detached.push_back(g->n_slots + i - 1);
    if (ensure_pool(g, std::max<uint64_t>(cfg->edge_capacity, 1024)) != FGI_OK) return fail(FGI_ENOMEM);
    if (hipDeviceSynchronize() != hipSuccess) return fail(FGI_EDEVICE);
    *out = g;
    return FGI_OK;
}

fgi_status fgi_destroy(fgi_graph* g) {
    if (!g) return FGI_OK;
    hipSetDevice(g->device);
    if (g->stream) hipStreamSynchronize(g->stream);
    fgi::part_destroy(g);
    fgi::tmp_drain(g);
    dfree(g->node);
    dfree(g->row_off);
    dfree(g->row_len);
    dfree(g->row_cap);
    dfree(g->used_cnt);
    dfree(g->home);
    dfree(g->pool_col);
    dfree(g->pool_tag);
    dfree(g->pool_top_dev);
    dfree(g->inv);
    dfree(g->inv_alt);
    for (int k = 0; k < 2; ++k) {
        if (g->ar_h[k]) (void)hipHostFree(g->ar_h[k]);
        dfree(g->ar_d[k]);
    }
    for (int k = 0; k < 2; ++k)
        if (g->apub[k]) hipHostFree(g->apub[k]);
    for (int i = 0; i < 2; ++i) {
        dfree(g->fr_off[i]);
        dfree(g->fr_len[i]);
    }
    for (int i = 0; i < 2; ++i) {
        dfree(g->escan[i]);
        dfree(g->cstart[i]);
    }
    dfree(g->uin_off);
    dfree(g->uin_len);
    dfree(g->uin_src);
    dfree(g->uin_head);
    dfree(g->pool_live);
    dfree(g->cand);
    dfree(g->wl);
    dfree(g->cand_seg);
    dfree(g->hot_id);
    for (int k = 0; k < 2; ++k) {
        dfree(g->sv[k]);
        dfree(g->sv_cnt[k]);
    }
    dfree(g->vis_bm);
    dfree(g->vis_spare);
    dfree(g->cls_bm);
    dfree(g->uin_more);
    dfree(g->sum_bm);
    dfree(g->inv_bm);
    dfree(g->bsum);
    dfree(g->done);
    dfree(g->ctr);
    dfree(g->gbar);
    dfree(g->blk_stats);
    dfree(g->roots_buf);
    dfree(g->imm_buf);
    dfree(g->misc_dev);
    dfree(g->snap_node);
    dfree(g->snap_row_off);
    dfree(g->snap_row_len);
    dfree(g->snap_row_cap);
    dfree(g->snap_used);
    dfree(g->snap_home);
    dfree(g->s2l);
    dfree(g->l2s);
    dfree(g->fold_start);
    dfree(g->fold_off);
    dfree(g->fold_base);
    dfree(g->xbm);
    dfree(g->fold_status);
    if (g->scratch) hipFree(g->scratch);
    if (g->ctr_host) hipHostFree(g->ctr_host);
    if (g->ctr_pub) hipHostFree(g->ctr_pub);
    if (g->red_pub) hipHostFree(g->red_pub);
    if (g->misc_host) hipHostFree(g->misc_host);
    for (hipEvent_t e : g->ev) hipEventDestroy(e);
    for (hipEvent_t e : g->batch_ev) hipEventDestroy(e);
    if (g->bst_h) hipHostFree(g->bst_h);
    dfree(g->bst_d);
    dfree(g->bout);
    if (g->ev_w0) hipEventDestroy(g->ev_w0);
    if (g->ev_w1) hipEventDestroy(g->ev_w1);
    if (g->stream) hipStreamDestroy(g->stream);
    delete g;
    return FGI_OK;
}

fgi_status fgi_stream(fgi_graph* g, void** stream) {
    if (!g || !stream) return FGI_EINVAL;
    *stream = g->stream;
    return FGI_OK;
}

fgi_status fgi_register_nodes(fgi_graph* g, uint32_t n, const uint32_t* slot, const uint64_t* version,
                              const uint32_t* state_flags) {
    if (!g || (n && (!slot || !version))) return FGI_EINVAL;
    FGI_TRY(single_only(g, "fgi_register_nodes"));
    for (uint32_t i = 0; i < n; ++i) {
        if (slot[i] >= g->ext_slots) return set_err(g, FGI_EINVAL, "slot %u out of range", slot[i]);
        if (version[i] > kVMask) return set_err(g, FGI_EINVAL, "version of slot %u exceeds 2^56-1", slot[i]);
        if (state_flags && (state_flags[i] & 3u) == 3u) return set_err(g, FGI_EINVAL, "bad state for slot %u", slot[i]);
    }
    if (n == 0) return FGI_OK;
    hipSetDevice(g->device);
    Tmp ts, tv, tf;
    uint32_t *ds, *df = nullptr;
    uint64_t* dv;
    FGI_TRY(tmalloc(g, ts, &ds, n));
    FGI_TRY(tmalloc(g, tv, &dv, n));
    if (state_flags) FGI_TRY(tmalloc(g, tf, &df, n));
    FGI_TRY(h2d(g, ds, slot, n));
    FGI_TRY(labels_map_in(g, ds, n));
    FGI_TRY(h2d(g, dv, version, n));
    if (state_flags) FGI_TRY(h2d(g, df, state_flags, n));
    FGI_TRY(fold(g));
    FGI_HIP(g, hipMemsetAsync(g->misc_dev, 0, sizeof(unsigned long long), g->stream));
    touch(g);
    note_words(g);
    hipLaunchKernelGGL(k_register, dim3(nblk(n)), dim3(256), 0, g->stream, n, ds, dv, df,
                       reinterpret_cast<unsigned long long*>(g->node), g->row_len, g->misc_dev);
    FGI_HIP(g, hipGetLastError());
    unsigned long long bad = 0;
    FGI_TRY(d2h(g, &bad, g->misc_dev, 1));
    if (bad) return set_err(g, FGI_ESTATE, "%llu slots already had a current node", bad);
    return FGI_OK;
}

fgi_status fgi_load_edges(fgi_graph* g, uint64_t m, const uint32_t* used, const uint32_t* dependant_slot,
                          const uint64_t* tag) {
    if (!g || (m && (!used || !dependant_slot || !tag))) return FGI_EINVAL;
    FGI_TRY(single_only(g, "fgi_load_edges"));
    for (uint64_t e = 0; e < m; ++e) {
        if (used[e] >= g->ext_handles || dependant_slot[e] >= g->ext_slots)
            return set_err(g, FGI_EINVAL, "edge %llu out of range", (unsigned long long)e);
        if (tag[e] == 0) return set_err(g, FGI_EINVAL, "edge %llu has tag 0 (LTags are positive)", (unsigned long long)e);
    }
    hipSetDevice(g->device);
    std::vector<uint64_t> hk(m);
    for (uint64_t e = 0; e < m; ++e) hk[e] = ((uint64_t)used[e] << 32) | dependant_slot[e];
    return load_rows(g, m, hk.data(), tag, 0, 0);
}

fgi_status fgi_get_state(fgi_graph* g, uint32_t n, const uint32_t* handle, uint64_t* version, uint32_t* state_flags) {
    if (!g || (n && !handle)) return FGI_EINVAL;
    FGI_TRY(usable(g));
    for (uint32_t i = 0; i < n; ++i)
        if (handle[i] >= g->ext_handles) return set_err(g, FGI_EINVAL, "handle %u out of range", handle[i]);
    if (n == 0) return FGI_OK;
    hipSetDevice(g->device);
    FGI_TRY(fold(g));
    Tmp th, tw;
    uint32_t* dh;
    unsigned long long* dw;
    FGI_TRY(tmalloc(g, th, &dh, n));
    FGI_TRY(tmalloc(g, tw, &dw, n));
    FGI_TRY(h2d(g, dh, handle, n));
    FGI_TRY(labels_map_in(g, dh, n));
    hipLaunchKernelGGL(k_gather_words, dim3(nblk(n)), dim3(256), 0, g->stream, n, dh,
                       reinterpret_cast<const unsigned long long*>(g->node), dw);
    std::vector<unsigned long long> w(n);
    FGI_TRY(d2h(g, w.data(), dw, n));
    for (uint32_t i = 0; i < n; ++i) {
        if (version) version[i] = w[i] & kVMask;
        if (state_flags) state_flags[i] = word_to_flags(w[i]);
    }
    return FGI_OK;
}

fgi_status fgi_dump_states(fgi_graph* g, uint64_t* version, uint32_t* state_flags) {
    if (!g) return FGI_EINVAL;
    FGI_TRY(usable(g));
    hipSetDevice(g->device);
    FGI_TRY(fold(g));
    const uint32_t H = g->ext_handles;
    std::vector<uint64_t> w(H);
    if (g->lbl_K || g->lbl_perm) {   // the words of boundary handles 0 .. H-1 at their labels (codes)
        Tmp th, tw;
        uint32_t* dh;
        unsigned long long* dw;
        FGI_TRY(tmalloc(g, th, &dh, H));
        FGI_TRY(tmalloc(g, tw, &dw, H));
        hipLaunchKernelGGL(k_iota, dim3(nblk(H)), dim3(256), 0, g->stream, H, dh);
        FGI_TRY(labels_map_in(g, dh, H));
        hipLaunchKernelGGL(k_gather_words, dim3(nblk(H)), dim3(256), 0, g->stream, H, dh,
                           reinterpret_cast<const unsigned long long*>(g->node), dw);
        FGI_TRY(d2h(g, reinterpret_cast<unsigned long long*>(w.data()), dw, H));
    } else {
        FGI_TRY(d2h(g, w.data(), g->node, H));
    }
    for (uint32_t h = 0; h < H; ++h) {
        if (version) version[h] = w[h] & kVMask;
        if (state_flags) state_flags[h] = word_to_flags(w[h]);
    }
    return FGI_OK;
}

// Marks the row entries the reference would still hold. RemoveUsedBy (Computed.cs:387-398) drops
// (d, t) from every dependency when d@t is invalidated; the engine drops such entries lazily
// (version filter in the wave, compaction in fgi_prune), so the observable set is: entries whose
// node d@t is still alive — the slot's current node at version t, or a detached node of slot d at
// version t (displaced while Computing / delayed) — and not Invalidated.
__global__ void k_used_by_live(uint32_t len, const uint32_t* __restrict__ col, const uint64_t* __restrict__ tag,
                               const unsigned long long* __restrict__ node, uint32_t n_slots, uint32_t n_detached,
                               const uint32_t* __restrict__ home, uint8_t* keep) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= len) return;
    const uint32_t d = col[i];
    const uint64_t t = tag[i];
    bool k = false;
    if (d < n_slots) {
        const unsigned long long w = node[d];
        if ((w & kVMask) == t) {
            k = word_is_current(w);
        } else {
            for (uint32_t j = 0; j < n_detached && !k; ++j) {
                const unsigned long long wd = node[n_slots + j];
                k = home[j] == d && (wd & kVMask) == t && word_is_current(wd);
            }
        }
    }
    keep[i] = k ? 1 : 0;
}

fgi_status fgi_get_used_by(fgi_graph* g, uint32_t handle, uint32_t* dep, uint64_t* tag, uint64_t cap, uint64_t* out_n) {
    if (!g || handle >= g->ext_handles) return FGI_EINVAL;
    FGI_TRY(usable(g));
    hipSetDevice(g->device);
    FGI_TRY(fold(g));
    FGI_TRY(label_of(g, handle, &handle));
    uint64_t w = 0, off = 0;
    uint32_t len = 0;
    FGI_TRY(d2h(g, &w, g->node + handle, 1));
    FGI_TRY(d2h(g, &off, g->row_off + handle, 1));
    FGI_TRY(d2h(g, &len, g->row_len + handle, 1));
    if (!word_is_current(w)) len = 0;   // `_usedBy` of an Invalidated node is cleared (Computed.cs:217)
    std::vector<uint32_t> d(len);
    std::vector<uint64_t> t(len);
    std::vector<uint8_t> keep(len);
    if (len) {
        Tmp tk;
        uint8_t* dkeep = nullptr;
        FGI_TRY(tmalloc(g, tk, &dkeep, len));
        hipLaunchKernelGGL(k_used_by_live, dim3((len + 255) / 256), dim3(256), 0, g->stream, len, g->pool_col + off,
                           g->pool_tag + off, reinterpret_cast<const unsigned long long*>(g->node), g->n_slots,
                           g->n_detached, g->home, dkeep);
        FGI_HIP(g, hipGetLastError());
        if (g->lbl_perm) {   // a partition's entries hold global codes: their slots
            FGI_TRY(d2h(g, d.data(), g->pool_col + off, len));
            for (uint32_t i = 0; i < len; ++i) d[i] = part_slot_of(g, d[i]);
        } else if (g->lbl_K) {   // the entries' dependants as boundary slots
            Tmp tc;
            uint32_t* dc;
            FGI_TRY(tmalloc(g, tc, &dc, len));
            FGI_HIP(g, hipMemcpyAsync(dc, g->pool_col + off, (size_t)len * 4, hipMemcpyDeviceToDevice, g->stream));
            FGI_TRY(labels_map_out(g, dc, len));
            FGI_TRY(d2h(g, d.data(), dc, len));
        } else {
            FGI_TRY(d2h(g, d.data(), g->pool_col + off, len));
        }
        FGI_TRY(d2h(g, t.data(), g->pool_tag + off, len));
        FGI_TRY(d2h(g, keep.data(), dkeep, len));
    }
    uint64_t n = 0;
    for (uint32_t i = 0; i < len; ++i) n += keep[i];
    if (out_n) *out_n = n;
    if (n > cap) return FGI_ECAPACITY;
    for (uint32_t i = 0, o = 0; i < len; ++i) {
        if (!keep[i]) continue;
        if (dep) dep[o] = d[i];
        if (tag) tag[o] = t[i];
        ++o;
    }
    return FGI_OK;
}

fgi_status fgi_get_used_count(fgi_graph* g, uint32_t handle, uint32_t* out) {
    if (!g || !out || handle >= g->ext_handles) return FGI_EINVAL;
    FGI_TRY(usable(g));
    hipSetDevice(g->device);
    FGI_TRY(fold(g));
    FGI_TRY(label_of(g, handle, &handle));
    uint64_t w = 0;
    uint32_t c = 0;
    FGI_TRY(d2h(g, &w, g->node + handle, 1));
    FGI_TRY(d2h(g, &c, g->used_cnt + handle, 1));
    *out = word_is_current(w) ? c : 0;   // `_used` is cleared on invalidation (Computed.cs:210-211)
    return FGI_OK;
}

fgi_status fgi_get_degrees(fgi_graph* g, uint32_t* degree, uint64_t* total) {
    if (!g) return FGI_EINVAL;
    FGI_TRY(usable(g));
    hipSetDevice(g->device);
    FGI_TRY(fold(g));
    const uint32_t H = g->ext_handles;
    std::vector<uint32_t> deg(H);
    {   // |_usedBy| of boundary handles 0 .. H-1 (at their labels)
        Tmp th, td;
        uint32_t *dh, *dd;
        FGI_TRY(tmalloc(g, th, &dh, H));
        FGI_TRY(tmalloc(g, td, &dd, H));
        hipLaunchKernelGGL(k_iota, dim3(nblk(H)), dim3(256), 0, g->stream, H, dh);
        FGI_TRY(labels_map_in(g, dh, H));
        hipLaunchKernelGGL(k_degree_of, dim3(nblk(H)), dim3(256), 0, g->stream, H, dh,
                           reinterpret_cast<const unsigned long long*>(g->node), g->row_len, dd);
        FGI_HIP(g, hipGetLastError());
        FGI_TRY(d2h(g, deg.data(), dd, H));
    }
    uint64_t t = 0;
    for (uint32_t h = 0; h < H; ++h) {
        if (degree) degree[h] = deg[h];
        t += deg[h];
    }
    if (total) *total = t;
    return FGI_OK;
}

fgi_status fgi_export_edges(fgi_graph* g, uint32_t* used, uint32_t* dep, uint64_t* tag, uint64_t cap, uint64_t* out_n) {
    if (!g) return FGI_EINVAL;
    FGI_TRY(usable(g));
    hipSetDevice(g->device);
    FGI_TRY(fold(g));
    Tmp tk, tt;
    uint64_t *keys, *tags, m = 0;
    FGI_TRY(gather_live(g, tk, tt, &keys, &tags, 0, &m));
    if (out_n) *out_n = m;
    if (m > cap) return FGI_ECAPACITY;
    Tmp tk2, tt2, ts;
    if (g->lbl_K && m) {   // as boundary handles, in (used, dependant) order again
        FGI_TRY(labels_unmap_keys(g, keys, m));
        uint64_t *k2, *t2;
        FGI_TRY(tmalloc(g, tk2, &k2, m));
        FGI_TRY(tmalloc(g, tt2, &t2, m));
        size_t tb = 0;
        FGI_HIP(g, rocprim::radix_sort_pairs(nullptr, tb, keys, k2, tags, t2, (size_t)m, 0, 64, g->stream));
        char* st;
        FGI_TRY(tmalloc(g, ts, &st, tb));
        FGI_HIP(g, rocprim::radix_sort_pairs(st, tb, keys, k2, tags, t2, (size_t)m, 0, 64, g->stream));
        keys = k2;
        tags = t2;
    }
    std::vector<uint64_t> hk(m);
    FGI_TRY(d2h(g, hk.data(), keys, m));
    if (tag) FGI_TRY(d2h(g, tag, tags, m));
    if (g->lbl_perm && m) {   // partition codes: (local used handle, dependant slot), in that order again
        std::vector<uint64_t> ht(m);
        FGI_TRY(d2h(g, ht.data(), tags, m));
        std::vector<uint64_t> idx(m);
        for (uint64_t e = 0; e < m; ++e) {
            hk[e] = ((uint64_t)part_code_local_h(g, (uint32_t)(hk[e] >> 32), true) << 32) | part_slot_of(g, (uint32_t)hk[e]);
            idx[e] = e;
        }
        std::sort(idx.begin(), idx.end(), [&](uint64_t a, uint64_t b) { return hk[a] != hk[b] ? hk[a] < hk[b] : ht[a] < ht[b]; });
        std::vector<uint64_t> k2(m);
        for (uint64_t e = 0; e < m; ++e) {
            k2[e] = hk[idx[e]];
            if (tag) tag[e] = ht[idx[e]];
        }
        hk.swap(k2);
    }
    for (uint64_t e = 0; e < m; ++e) {
        if (used) used[e] = (uint32_t)(hk[e] >> 32);
        if (dep) dep[e] = (uint32_t)hk[e];
    }
    return FGI_OK;
}

fgi_status fgi_snapshot(fgi_graph* g) {
    if (!g) return FGI_EINVAL;
    FGI_TRY(usable(g));
    hipSetDevice(g->device);
    const size_t H = g->n_handles;
    if (!g->snap_node) {
        if (dmalloc(g, &g->snap_node, H) || dmalloc(g, &g->snap_row_off, H) || dmalloc(g, &g->snap_row_len, H) ||
            dmalloc(g, &g->snap_row_cap, H) || dmalloc(g, &g->snap_used, H))
            return FGI_ENOMEM;
    }
    hipStream_t s = g->stream;
    FGI_TRY(fold(g));
    FGI_HIP(g, hipMemcpyAsync(g->snap_node, g->node, H * 8, hipMemcpyDeviceToDevice, s));
    FGI_HIP(g, hipMemcpyAsync(g->snap_row_off, g->row_off, H * 8, hipMemcpyDeviceToDevice, s));
    FGI_HIP(g, hipMemcpyAsync(g->snap_row_len, g->row_len, H * 4, hipMemcpyDeviceToDevice, s));
    FGI_HIP(g, hipMemcpyAsync(g->snap_row_cap, g->row_cap, H * 4, hipMemcpyDeviceToDevice, s));
    FGI_HIP(g, hipMemcpyAsync(g->snap_used, g->used_cnt, H * 4, hipMemcpyDeviceToDevice, s));
    if (g->n_detached) {
        if (!g->snap_home && dmalloc(g, &g->snap_home, g->n_detached)) return FGI_ENOMEM;
        FGI_HIP(g, hipMemcpyAsync(g->snap_home, g->home, (size_t)g->n_detached * 4, hipMemcpyDeviceToDevice, s));
    }
    g->snap_free_detached = g->free_detached;
    FGI_HIP(g, hipStreamSynchronize(s));
    g->snap_epoch = g->pool_epoch;
    g->snap_mut_epoch = g->mut_epoch;
    g->words_dirty = false;
    return FGI_OK;
}

// Restores the node table; the edge pool is append-only between compactions, so the saved row
// descriptors still address the saved rows unless fgi_prune / a bulk load ran in between. A node's
// state is its word plus its visit bit: waves only set bits, so after waves alone the words are the
// snapshot's and clearing the bitmap restores every node; words are copied back only if something
// else (a fold, a mutation, an immediate root) changed them.
fgi_status fgi_restore(fgi_graph* g) {
    if (!g) return FGI_EINVAL;
    if (!g->snap_node) return g->failed ? usable(g) : FGI_EINVAL;
    if (g->snap_epoch != g->pool_epoch) return set_err(g, FGI_ESTATE, "edge pool was rebuilt since the snapshot");
    hipSetDevice(g->device);
    const size_t H = g->n_handles;
    hipStream_t s = g->stream;
    if (g->failed) {
        // a failed batch or wave: words, visit / invalidated bits and the wave counters are undefined. Every
        // saved table is copied back and the wave state cleared before the graph is usable again (the
        // copies are stream-ordered after any wave still in flight; its results are forgotten).
        g->aw[0] = fgi_graph::AsyncWave{};
        g->aw[1] = fgi_graph::AsyncWave{};
        FGI_HIP(g, hipMemcpyAsync(g->node, g->snap_node, H * 8, hipMemcpyDeviceToDevice, s));
        FGI_HIP(g, hipMemsetAsync(g->vis_bm, 0, g->bm_words * 4, s));
        FGI_HIP(g, hipMemsetAsync(g->vis_spare, 0, g->bm_words * 4, s));
        FGI_HIP(g, hipMemsetAsync(g->inv_bm, 0, g->bm_words * 4, s));
        FGI_HIP(g, hipMemsetAsync(g->gbar, 0, kGbarWords * sizeof(unsigned long long), s));
        g->spare_dirty = false;
        g->wave_clean = false;
        g->words_dirty = false;
        g->cls_valid = false;
        g->v_dirty = false;
        g->vis_stale = false;
        g->coop_clean = false;   // the next cascade re-initialises the wave counters
        g->ids_valid = false;
        g->mut_epoch = ~0ull;    // forces the row tables' copy below
    }
    if (g->words_dirty) {
        FGI_HIP(g, hipMemcpyAsync(g->node, g->snap_node, H * 8, hipMemcpyDeviceToDevice, s));
        g->words_dirty = false;
        g->cls_valid = false;
    }
    // the visit bits are forgotten: the clean spare bitmap takes the visit bitmap's place, and the next
    // wave's list kernel clears the old one; without a clean spare, the next wave's init kernel clears it
    // (or flush_vis before any other use)
    if (g->v_dirty) {
        if (!g->spare_dirty && !g->vis_stale) {
            std::swap(g->vis_bm, g->vis_spare);
            g->spare_dirty = true;
        } else {
            g->vis_stale = true;
        }
    }
    g->v_dirty = false;
    if (g->mut_epoch == g->snap_mut_epoch) {
        // nothing but waves ran since the snapshot: rows and |_used| counts are unchanged. The
        // copies are stream-ordered before every later call on this graph, so no host wait here.
        FGI_HIP(g, hipGetLastError());
        return FGI_OK;
    }
    FGI_HIP(g, hipMemcpyAsync(g->row_off, g->snap_row_off, H * 8, hipMemcpyDeviceToDevice, s));
    FGI_HIP(g, hipMemcpyAsync(g->row_len, g->snap_row_len, H * 4, hipMemcpyDeviceToDevice, s));
    FGI_HIP(g, hipMemcpyAsync(g->row_cap, g->snap_row_cap, H * 4, hipMemcpyDeviceToDevice, s));
    FGI_HIP(g, hipMemcpyAsync(g->used_cnt, g->snap_used, H * 4, hipMemcpyDeviceToDevice, s));
    // the detached handles the mutations since the snapshot took are free again (their words and rows
    // are the snapshot's)
    if (g->n_detached && g->snap_home)
        FGI_HIP(g, hipMemcpyAsync(g->home, g->snap_home, (size_t)g->n_detached * 4, hipMemcpyDeviceToDevice, s));
    g->free_detached = g->snap_free_detached;
    FGI_HIP(g, hipStreamSynchronize(s));
    g->mut_epoch = g->snap_mut_epoch;   // rows and versions are those of the snapshot again
    g->failed = false;
    return FGI_OK;
}

fgi_status fgi_set_option(fgi_graph* g, int option, int64_t value) {
    if (!g) return FGI_EINVAL;
    switch (option) {
    case FGI_OPT_DEAD_FILTER: g->opt_dead_filter = value ? 1 : 0; return FGI_OK;
    case FGI_OPT_PART_COLLECTIVES: g->opt_part_coll = value ? 1 : 0; return FGI_OK;
    case FGI_OPT_FRONT_EXCHANGE:
        if (value < 0 || value > 2) return set_err(g, FGI_EINVAL, "frontier exchange must be 0, 1 or 2");
        g->opt_front_exchange = (int)value;
        return FGI_OK;
    case FGI_OPT_DEFRAG_PCT: g->opt_defrag_pct = (int)std::max<int64_t>(0, std::min<int64_t>(100, value)); return FGI_OK;
    case FGI_OPT_DIRECTION:
        if (value < 0 || value > 2) return set_err(g, FGI_EINVAL, "direction must be 0, 1 or 2");
        g->opt_direction = (int)value;
        return FGI_OK;
    case FGI_OPT_PULL_ALPHA:
        if (value < 1) return set_err(g, FGI_EINVAL, "alpha must be >= 1");
        g->opt_pull_alpha = (int)value;
        return FGI_OK;
    case FGI_OPT_LEVEL_TIMING: g->opt_level_timing = value ? 1 : 0; return FGI_OK;
    case FGI_OPT_PULL_TPB:
        if (value < 0 || value > 32) return set_err(g, FGI_EINVAL, "pull tiles per block must be 0..32");
        g->opt_pull_tpb = (int)value;
        // the candidate lists are segmented per pull block: rebuilt for the new grid. A partition's
        // dependency lists come from its load (part_build_in_lists), which a wave never redoes, so its
        // candidates are re-segmented here over the lists it has.
        if (!g->part) {
            g->uin_epoch = 0;
        } else if (g->uin_src && g->uin_epoch == g->mut_epoch) {
            hipSetDevice(g->device);
            return build_candidates(g);
        }
        return FGI_OK;
    case FGI_OPT_HOT_HEADS:
        if (value < 0 || value > (int64_t)kHot) return set_err(g, FGI_EINVAL, "hot heads must be 0..%u", kHot);
        g->opt_hot_heads = (int)value;
        // the candidates' head codes depend on the hot set: rebuilt (as for FGI_OPT_PULL_TPB)
        if (!g->part) {
            g->uin_epoch = 0;
        } else if (g->uin_src && g->uin_epoch == g->mut_epoch) {
            hipSetDevice(g->device);
            return build_candidates(g);
        }
        return FGI_OK;
    case FGI_OPT_PULL_BETA:
        if (value < 0) return set_err(g, FGI_EINVAL, "beta must be >= 0");
        g->opt_pull_beta = (int)value;
        return FGI_OK;
    case FGI_OPT_PART_PLAN: g->opt_part_plan = value ? 1 : 0; return FGI_OK;
    case FGI_OPT_PART_BUCKET: return part_set_bucket(g, value);
    case FGI_OPT_PROBE_SUMMARY:
        if (value < -1 || value > (int64_t)FGI_NONE) return set_err(g, FGI_EINVAL, "probe summary: -1 or a word count");
        if (!FGI_VARIANTS && value != -1)
            return set_err(g, FGI_ENOTSUP, "the probe summary is in the variant build only (make variant-all)");
        g->opt_sum_min = value;
        return FGI_OK;
    case FGI_OPT_FUSED:
        if (value < 0 || value > 15) return set_err(g, FGI_EINVAL, "fused-wave bits must be 0..15");
        if (!FGI_VARIANTS && value != 0)
            return set_err(g, FGI_ENOTSUP, "fused waves are in the variant build only (make variant-all)");
        g->opt_fused = (int)value;
        return FGI_OK;
    case FGI_OPT_FAULT_INJECT:
        if (value < 0 || ((value & 0xFFFF) == 0 && value != 0) || value >= (1ll << 32))
            return set_err(g, FGI_EINVAL, "fault injection: (launches to skip << 16) | (block + 1), block + 1 > 0");
        g->fault_block = (uint32_t)(value & 0xFFFF);
        g->fault_skip = (uint32_t)(value >> 16);
        return FGI_OK;
    case FGI_OPT_FAULT_INJECT_TAIL:
        if (value < 0 || ((value & 0xFFFF) == 0 && value != 0) || value >= (1ll << 32))
            return set_err(g, FGI_EINVAL, "fault injection: (tail launches to skip << 16) | (block + 1), block + 1 > 0");
        g->fault_tail_block = (uint32_t)(value & 0xFFFF);
        g->fault_tail_skip = (uint32_t)(value >> 16);
        return FGI_OK;
    default: return set_err(g, FGI_EINVAL, "unknown option %d", option);
    }
}

// ---- invalidation entry points ----------------------------------------------------------------
// The single-device wave and mutation entry points address rows whose entries are local handles; a
// partitioned graph's rows hold global dependant ids (part.hip), so they must go through fgi_part_*.
static fgi_status single_only(fgi_graph* g, const char* what) {
    FGI_TRY(usable(g));
    return g->part ? set_err(g, FGI_ESTATE, "%s: partitioned graph, use the fgi_part_* entry points", what) : FGI_OK;
}
static fgi_status stage_roots(fgi_graph* g, uint64_t n) {
    if (g->roots_cap >= n && g->roots_buf) return FGI_OK;
    dfree(g->roots_buf);
    dfree(g->imm_buf);
    const uint64_t cap = std::max<uint64_t>(n, 4096);
    FGI_TRY(dmalloc(g, &g->roots_buf, cap));
    FGI_TRY(dmalloc(g, &g->imm_buf, cap));
    g->roots_cap = cap;
    return FGI_OK;
}

static fgi_status copy_ids(fgi_graph* g, uint32_t* out_ids, uint64_t cap, uint64_t* out_n) {
    const uint64_t n = g->last_wave_n;
    if (out_n) *out_n = n;
    if (!out_ids) return FGI_OK;
    if (n > cap) return FGI_ECAPACITY;
    FGI_TRY(ensure_ids(g));
    return d2h(g, out_ids, g->inv_cur ? g->inv_cur : g->inv, n);
}

fgi_status fgi_invalidate(fgi_graph* g, uint32_t n_roots, const uint32_t* roots, const uint8_t* immediately,
                          uint32_t* out_ids, uint64_t cap, uint64_t* out_n, fgi_wave_stats* stats) {
    if (!g || (n_roots && !roots)) return FGI_EINVAL;
    FGI_TRY(single_only(g, "fgi_invalidate"));
    hipSetDevice(g->device);
    FGI_TRY(stage_roots(g, n_roots));
    FGI_TRY(h2d(g, g->roots_buf, roots, n_roots));
    if (immediately) FGI_TRY(h2d(g, g->imm_buf, immediately, n_roots));
    FGI_TRY(run_wave(g, n_roots, g->roots_buf, immediately ? g->imm_buf : nullptr, stats, true));
    return copy_ids(g, out_ids, cap, out_n);
}

fgi_status fgi_invalidate_dev(fgi_graph* g, uint32_t n_roots, const uint32_t* roots_dev, const uint8_t* imm_dev,
                              uint32_t* out_ids_dev, uint64_t* out_n, fgi_wave_stats* stats) {
    if (!g || (n_roots && !roots_dev)) return FGI_EINVAL;
    FGI_TRY(single_only(g, "fgi_invalidate_dev"));
    hipSetDevice(g->device);
    FGI_TRY(run_wave(g, n_roots, roots_dev, imm_dev, stats, true));
    if (out_n) *out_n = g->last_wave_n;
    if (out_ids_dev && g->last_wave_n) {
        FGI_TRY(ensure_ids(g));
        FGI_HIP(g, hipMemcpyAsync(out_ids_dev, g->inv, g->last_wave_n * 4, hipMemcpyDeviceToDevice, g->stream));
        FGI_HIP(g, hipStreamSynchronize(g->stream));
    }
    return FGI_OK;
}

fgi_status fgi_invalidate_bits(fgi_graph* g, uint32_t n_roots, const uint32_t* roots, const uint8_t* immediately,
                               uint64_t* out_bits, uint64_t words, uint64_t* out_n, fgi_wave_stats* stats) {
    if (!g || (n_roots && !roots)) return FGI_EINVAL;
    FGI_TRY(single_only(g, "fgi_invalidate_bits"));
    hipSetDevice(g->device);
    const uint64_t need = ((uint64_t)g->ext_handles + 63) / 64;
    if (out_bits && words < need)
        return set_err(g, FGI_ECAPACITY, "bitmap of %llu words needs %llu", (unsigned long long)words,
                       (unsigned long long)need);
    FGI_TRY(stage_roots(g, n_roots));
    FGI_TRY(h2d(g, g->roots_buf, roots, n_roots));
    if (immediately) FGI_TRY(h2d(g, g->imm_buf, immediately, n_roots));
    g->want_ids = false;   // the final collect only counts; the list is made on demand (ensure_ids)
    const fgi_status st = run_wave(g, n_roots, g->roots_buf, immediately ? g->imm_buf : nullptr, stats, true);
    g->want_ids = true;
    FGI_TRY(st);
    if (out_n) *out_n = g->last_wave_n;
    if (!out_bits) return FGI_OK;
    // the wave's invalidated bitmap over boundary handles (bit h of 32-bit word h / 32 = bit h of 64-bit
    // word h / 64): the labels' own, or, with hot labels, the one the final collect folded (xbm)
    return d2h(g, out_bits, g->xbm ? reinterpret_cast<const uint64_t*>(g->xbm) : reinterpret_cast<const uint64_t*>(g->inv_bm),
               need);
}

fgi_status fgi_invalidate_async(fgi_graph* g, uint32_t n_roots, const uint32_t* roots_dev, const uint8_t* imm_dev,
                                uint64_t* ticket) {
    if (!g || (n_roots && !roots_dev) || !ticket) return FGI_EINVAL;
    FGI_TRY(usable_now(g));
    if (g->part) return set_err(g, FGI_ESTATE, "fgi_invalidate_async: partitioned graph, use fgi_part_invalidate");
    hipSetDevice(g->device);
    return run_wave_async(g, n_roots, roots_dev, imm_dev, ticket);
}

fgi_status fgi_wave_wait(fgi_graph* g, uint64_t ticket, uint64_t* out_n, const uint32_t** ids_dev, fgi_wave_stats* stats) {
    if (!g) return FGI_EINVAL;
    FGI_TRY(usable_now(g));
    hipSetDevice(g->device);
    return wave_wait(g, ticket, out_n, ids_dev, stats);
}

fgi_status fgi_invalidate_async_host(fgi_graph* g, uint32_t n_roots, const uint32_t* roots, const uint8_t* immediately,
                                     uint64_t* ticket) {
    if (!g || (n_roots && !roots) || !ticket) return FGI_EINVAL;
    FGI_TRY(usable_now(g));
    if (g->part) return set_err(g, FGI_ESTATE, "fgi_invalidate_async_host: partitioned graph, use fgi_part_invalidate");
    hipSetDevice(g->device);
    return run_wave_async_host(g, n_roots, roots, immediately, ticket);
}

fgi_status fgi_wave_wait_ids(fgi_graph* g, uint64_t ticket, uint32_t* out_ids, uint64_t cap, uint64_t* out_n,
                             fgi_wave_stats* stats) {
    if (!g) return FGI_EINVAL;
    FGI_TRY(usable_now(g));
    hipSetDevice(g->device);
    uint64_t n = 0;
    const uint32_t* ids = nullptr;
    FGI_TRY(wave_wait(g, ticket, &n, &ids, stats));
    if (out_n) *out_n = n;
    if (!out_ids || n == 0) return FGI_OK;
    if (n > cap) return set_err(g, FGI_ECAPACITY, "wave %llu invalidated %llu handles, the buffer holds %llu",
                                (unsigned long long)ticket, (unsigned long long)n, (unsigned long long)cap);
    // a blocking copy on the null stream: the graph's stream is non-blocking, so a wave queued after this
    // ticket's keeps running (the ticket's buffer is its own until the wave two tickets later is queued)
    FGI_HIP(g, hipMemcpy(out_ids, ids, (size_t)n * 4, hipMemcpyDeviceToHost));
    return FGI_OK;
}

fgi_status fgi_alloc_pinned(uint64_t bytes, void** out) {
    if (!out) return FGI_EINVAL;
    *out = nullptr;
    if (bytes == 0) return FGI_OK;
    return hipHostMalloc(out, bytes, hipHostMallocDefault) == hipSuccess ? FGI_OK : FGI_ENOMEM;
}

fgi_status fgi_free_pinned(void* p) {
    if (!p) return FGI_OK;
    return hipHostFree(p) == hipSuccess ? FGI_OK : FGI_EINVAL;
}

fgi_status fgi_wave_ids_dev(fgi_graph* g, const uint32_t** ids_dev, uint64_t* n) {
    if (!g || !ids_dev) return FGI_EINVAL;
    FGI_TRY(usable(g));
    hipSetDevice(g->device);
    if (!g->part) FGI_TRY(ensure_ids(g));
    *ids_dev = (!g->part && g->inv_cur) ? g->inv_cur : g->inv;
    if (n) *n = g->last_wave_n;
    return FGI_OK;
}

fgi_status fgi_last_wave_ids(fgi_graph* g, uint32_t* out_ids, uint64_t cap, uint64_t* out_n) {
    if (!g) return FGI_EINVAL;
    FGI_TRY(usable(g));
    hipSetDevice(g->device);
    return copy_ids(g, out_ids, cap, out_n);
}

fgi_status fgi_invalidate_all(fgi_graph* g, uint32_t* out_ids, uint64_t cap, uint64_t* out_n, fgi_wave_stats* stats) {
    if (!g) return FGI_EINVAL;
    FGI_TRY(single_only(g, "fgi_invalidate_all"));
    hipSetDevice(g->device);
    FGI_TRY(stage_roots(g, g->n_slots));
    FGI_TRY(fold(g));
    FGI_HIP(g, hipMemsetAsync(g->misc_dev, 0, sizeof(unsigned long long), g->stream));
    hipLaunchKernelGGL(k_invalidate_all_roots, dim3(nblk(g->n_slots)), dim3(256), 0, g->stream, g->n_slots,
                       reinterpret_cast<const unsigned long long*>(g->node), g->roots_buf, g->misc_dev);
    unsigned long long n = 0;
    FGI_TRY(d2h(g, &n, g->misc_dev, 1));
    FGI_TRY(run_wave(g, (uint32_t)n, g->roots_buf, nullptr, stats));
    return copy_ids(g, out_ids, cap, out_n);
}

fgi_status fgi_begin_compute(fgi_graph* g, uint32_t n, const uint32_t* slot, const uint64_t* version,
                             const uint8_t* has_delay, uint32_t* out_detached, fgi_wave_stats* stats) {
    if (!g || (n && (!slot || !version))) return FGI_EINVAL;
    if (n == 0) return FGI_OK;
    {
        // O(n) validation over a reusable slot bitmap (cleared again bit by bit)
        std::vector<uint64_t>& seen = g->seen_bits;
        if (seen.size() < ((size_t)g->ext_slots + 63) / 64) seen.assign(((size_t)g->ext_slots + 63) / 64, 0);
        uint32_t bad = FGI_NONE;
        const char* why = nullptr;
        uint32_t i = 0;
        for (; i < n; ++i) {
            const uint32_t x = slot[i];
            if (x >= g->ext_slots) { why = "slot out of range"; bad = x; break; }
            if (version[i] == 0 || version[i] > kVMask) { why = "bad version"; bad = i; break; }
            const uint64_t m = 1ull << (x & 63);
            if (seen[x >> 6] & m) { why = "slot repeated in one batch"; bad = x; break; }
            seen[x >> 6] |= m;
        }
        for (uint32_t j = 0; j < i; ++j) seen[slot[j] >> 6] = 0;
        if (why) return set_err(g, FGI_EINVAL, "%s (%u)", why, bad);
    }
    FGI_TRY(single_only(g, "fgi_begin_compute"));
    hipSetDevice(g->device);
    hipStream_t st = g->stream;
    Tmp ts, tv, td, tc, tr, tf, to;
    uint32_t *ds, *droots, *dfree_h, *dout;
    uint64_t* dv;
    uint8_t *dd = nullptr, *dcls;
    FGI_TRY(tmalloc(g, ts, &ds, n));
    FGI_TRY(tmalloc(g, tv, &dv, n));
    FGI_TRY(tmalloc(g, tc, &dcls, n));
    FGI_TRY(tmalloc(g, tr, &droots, n));
    FGI_TRY(tmalloc(g, to, &dout, n));
    if (has_delay) {
        FGI_TRY(tmalloc(g, td, &dd, n));
        FGI_TRY(h2d(g, dd, has_delay, n));
    }
    FGI_TRY(h2d(g, ds, slot, n));
    FGI_TRY(labels_map_in(g, ds, n));
    FGI_TRY(h2d(g, dv, version, n));
    FGI_TRY(fold(g));
    FGI_HIP(g, hipMemsetAsync(g->misc_dev, 0, 4 * sizeof(unsigned long long), st));
    hipLaunchKernelGGL(k_bc_classify, dim3(nblk(n)), dim3(256), 0, st, n, ds,
                       reinterpret_cast<const unsigned long long*>(g->node), dcls, droots, g->misc_dev);
    unsigned long long cnt[2];
    FGI_TRY(d2h(g, cnt, g->misc_dev, 2));
    if (cnt[1] > g->free_detached.size())
        return set_err(g, FGI_ECAPACITY, "out of detached handles (%zu free, %llu needed)", g->free_detached.size(),
                       cnt[1]);
    // displacement cascade first (ComputedRegistry.cs:91-94), then detach + install
    g->last_wave_n = 0;
    if (cnt[0]) FGI_TRY(run_wave(g, (uint32_t)cnt[0], droots, nullptr, stats));
    std::vector<uint32_t> take(g->free_detached.end() - (ptrdiff_t)cnt[1], g->free_detached.end());
    FGI_TRY(tmalloc(g, tf, &dfree_h, take.size() + 1));
    FGI_TRY(h2d(g, dfree_h, take.data(), take.size()));
    FGI_TRY(fold(g));   // the displacement cascade's visits
    FGI_HIP(g, hipMemsetAsync(g->misc_dev + 2, 0, sizeof(unsigned long long), st));
    touch(g);
    note_words(g);
    const InstallArgs ia{ds,          dv,          dd,         dcls,       dfree_h, g->misc_dev + 2, g->n_slots,
                         reinterpret_cast<unsigned long long*>(g->node), g->row_off, g->row_len, g->row_cap,
                         g->used_cnt, g->home, dout};
    hipLaunchKernelGGL(k_bc_install, dim3(nblk(n)), dim3(256), 0, st, n, ia);
    FGI_HIP(g, hipGetLastError());
    FGI_TRY(labels_map_out(g, dout, n));   // detached handles as the boundary numbers them
    std::vector<uint32_t> od(n);
    FGI_TRY(d2h(g, od.data(), dout, n));
    g->free_detached.resize(g->free_detached.size() - take.size());
    if (out_detached) std::memcpy(out_detached, od.data(), n * sizeof(uint32_t));
    return FGI_OK;
}

fgi_status fgi_add_used(fgi_graph* g, uint32_t n, const uint32_t* dependant, const uint32_t* used, uint32_t* out_result) {
    if (!g || (n && (!dependant || !used))) return FGI_EINVAL;
    for (uint32_t i = 0; i < n; ++i)
        if (dependant[i] >= g->ext_handles || used[i] >= g->ext_handles)
            return set_err(g, FGI_EINVAL, "handle out of range at %u", i);
    if (n == 0) return FGI_OK;
    FGI_TRY(single_only(g, "fgi_add_used"));
    hipSetDevice(g->device);
    hipStream_t st = g->stream;
    uint64_t hcap = 64;
    while (hcap < 2ull * n) hcap <<= 1;
    Tmp tdep, tuse, tres, thash, tcand, tpend, tovf;
    uint32_t *ddep, *duse, *dres, *dpend, *dovf;
    unsigned long long* dhash;
    Cand* dcand;
    FGI_TRY(tmalloc(g, tdep, &ddep, n));
    FGI_TRY(tmalloc(g, tuse, &duse, n));
    FGI_TRY(tmalloc(g, tres, &dres, n));
    FGI_TRY(tmalloc(g, thash, &dhash, hcap));
    FGI_TRY(tmalloc(g, tcand, &dcand, n));
    FGI_TRY(tmalloc(g, tpend, &dpend, n));
    FGI_TRY(tmalloc(g, tovf, &dovf, n));
    FGI_TRY(h2d(g, ddep, dependant, n));
    FGI_TRY(h2d(g, duse, used, n));
    FGI_TRY(labels_map_in(g, ddep, n));
    FGI_TRY(labels_map_in(g, duse, n));
    FGI_TRY(fold(g));
    note_words(g);   // may set InvalidateOnSetOutput (Computed.cs:376-378)
    FGI_HIP(g, hipMemsetAsync(dhash, 0xFF, hcap * sizeof(unsigned long long), st));
    FGI_HIP(g, hipMemsetAsync(g->misc_dev, 0, 8 * sizeof(unsigned long long), st));
    const AuArgs aa{ddep,        duse,       g->n_slots,   g->home,     reinterpret_cast<unsigned long long*>(g->node),
                    g->row_off,  g->row_len, g->row_cap,   g->used_cnt, g->pool_col,
                    g->pool_tag, dhash,      hcap - 1,     dres,        dcand,
                    dpend,       dovf,       g->misc_dev};
    hipLaunchKernelGGL(k_au_classify, dim3(nblk(n)), dim3(256), 0, st, n, aa);
    unsigned long long nc = 0;
    FGI_TRY(d2h(g, &nc, g->misc_dev, 1));
    if (nc) {
        touch(g);
        hipLaunchKernelGGL(k_au_reserve, dim3(nblk(nc)), dim3(256), 0, st, (uint64_t)nc, aa);
        unsigned long long c2[2];
        FGI_TRY(d2h(g, c2, g->misc_dev + 1, 2));
        if (c2[1]) {   // some rows outgrew their capacity: relocate them to the pool top
            hipLaunchKernelGGL(k_au_size, dim3(nblk(c2[1])), dim3(256), 0, st, (uint64_t)c2[1], dovf, g->row_len,
                               g->misc_dev + 3);
            unsigned long long need = 0;
            FGI_TRY(d2h(g, &need, g->misc_dev + 3, 1));
            FGI_TRY(ensure_pool(g, g->pool_top + need));
            FGI_HIP(g, hipMemcpyAsync(g->pool_top_dev, &g->pool_top, sizeof(uint64_t), hipMemcpyHostToDevice, st));
            hipLaunchKernelGGL(k_au_relocate, dim3(nblk(c2[1] * 64)), dim3(256), 0, st, (uint64_t)c2[1], dovf,
                               g->row_off, g->row_len, g->row_cap, g->pool_col, g->pool_tag, g->pool_top_dev);
            hipLaunchKernelGGL(k_au_pending, dim3(nblk(nc)), dim3(256), 0, st, (uint64_t)nc, dcand, dpend, g->row_off,
                               g->pool_col, g->pool_tag);
            g->pool_top += need;
            FGI_TRY(ensure_cstart(g, g->pool_top));
        }
    }
    FGI_HIP(g, hipGetLastError());
    if (out_result) FGI_TRY(d2h(g, out_result, dres, n));
    else FGI_HIP(g, hipStreamSynchronize(st));
    return FGI_OK;
}

fgi_status fgi_set_output(fgi_graph* g, uint32_t n, const uint32_t* handle, uint8_t* out_set, uint32_t* out_ids,
                          uint64_t cap, uint64_t* out_n, fgi_wave_stats* stats) {
    if (!g || (n && !handle)) return FGI_EINVAL;
    if (out_n) *out_n = 0;
    if (n == 0) return FGI_OK;
    FGI_TRY(single_only(g, "fgi_set_output"));
    hipSetDevice(g->device);
    hipStream_t st = g->stream;
    Tmp th, ts, tr;
    uint32_t *dh, *droots;
    uint8_t* dset;
    FGI_TRY(tmalloc(g, th, &dh, n));
    FGI_TRY(tmalloc(g, ts, &dset, n));
    FGI_TRY(tmalloc(g, tr, &droots, n));
    FGI_TRY(h2d(g, dh, handle, n));
    FGI_TRY(labels_map_in(g, dh, n));
    FGI_TRY(fold(g));
    note_words(g);
    FGI_HIP(g, hipMemsetAsync(g->misc_dev, 0, sizeof(unsigned long long), st));
    hipLaunchKernelGGL(k_set_output, dim3(nblk(n)), dim3(256), 0, st, n, dh, g->n_handles,
                       reinterpret_cast<unsigned long long*>(g->node), dset, droots, g->misc_dev);
    unsigned long long nr = 0;
    FGI_TRY(d2h(g, &nr, g->misc_dev, 1));
    if (out_set) FGI_TRY(d2h(g, out_set, dset, n));
    g->last_wave_n = 0;
    if (nr) FGI_TRY(run_wave(g, (uint32_t)nr, droots, nullptr, stats));   // Invalidate() (Computed.cs:153-156)
    return copy_ids(g, out_ids, cap, out_n);
}

// ---- streaming batches ---------------------------------------------------------------------------
namespace {

constexpr size_t kStageAlign = 256;
inline size_t stage_round(size_t b) { return (b + kStageAlign - 1) / kStageAlign * kStageAlign; }

// Per-step device state of a batch (kept until the call returns: a pool growth resumes a step).
struct BatchStep {
    const uint32_t* h = nullptr;     // staged inputs (device)
    const uint32_t* used = nullptr;
    const uint64_t* ver = nullptr;
    const uint8_t* flags = nullptr;
    uint8_t* cls = nullptr;          // begin_compute
    uint32_t* roots = nullptr;       // begin_compute / set_output cascade roots
    uint32_t* out32 = nullptr;       // detached handles / add_used results
    uint8_t* out8 = nullptr;         // set_output flags
    unsigned long long* hash = nullptr;
    uint64_t hcap = 0;
    Cand* cand = nullptr;
    uint32_t* pend = nullptr;
    uint32_t* ovf = nullptr;
    unsigned long long* cnt = nullptr;   // 4 counters
    size_t out_off = 0;              // where its output lands in the pinned staging
    std::vector<Tmp> tmp;
};

}  // namespace

// Launches steps [from, n) of a batch; returns with the work queued (no synchronisation).
static fgi_status batch_launch(fgi_graph* g, uint32_t from, uint32_t n_steps, const fgi_step* steps,
                               std::vector<BatchStep>& bs, unsigned long long* scr, const uint32_t* take,
                               uint64_t n_take, bool timed, std::vector<std::pair<hipEvent_t, hipEvent_t>>& wave_ev) {
    FGI_TRY(flush_vis(g));
    hipStream_t st = g->stream;
    unsigned long long* abort = scr;
    unsigned long long* out_n = scr + 1;
    unsigned long long* cursor = scr + 2;
    unsigned long long* acc = scr + 3;
    auto* node = reinterpret_cast<unsigned long long*>(g->node);
    // per-cascade timing (the wave share of fgi_batch_stats) only when asked for: timestamped
    // markers between the launches cost device time of their own; the events are the graph's pool
    auto wave = [&](uint32_t n_max, const uint32_t* roots, const uint8_t* imm, const unsigned long long* n_dev) -> fgi_status {
        hipEvent_t e0 = nullptr, e1 = nullptr;
        if (timed) {
            const size_t i = wave_ev.size();
            while (g->batch_ev.size() < 2 * (i + 1)) {
                hipEvent_t e;
                FGI_HIP(g, hipEventCreate(&e));
                g->batch_ev.push_back(e);
            }
            e0 = g->batch_ev[2 * i];
            e1 = g->batch_ev[2 * i + 1];
            wave_ev.emplace_back(e0, e1);
            FGI_HIP(g, hipEventRecord(e0, st));
        }
        FGI_TRY(run_wave_coop(g, n_max, roots, imm, n_dev, g->bout, out_n, acc, abort));
        if (e1) FGI_HIP(g, hipEventRecord(e1, st));
        return fold(g);
    };
    for (uint32_t k = from; k < n_steps; ++k) {
        const fgi_step& sp = steps[k];
        BatchStep& b = bs[k];
        const uint32_t n = sp.n;
        if (n == 0) continue;
        const uint32_t grid = (uint32_t)std::min<uint64_t>(nblk(n), 8192);
        switch (sp.kind) {
            case FGI_STEP_INVALIDATE:
                FGI_TRY(fold(g));
                FGI_TRY(wave(n, b.h, b.flags, nullptr));
                break;
            case FGI_STEP_BEGIN_COMPUTE: {
                FGI_TRY(fold(g));
                hipLaunchKernelGGL(kb_bc_classify_check, dim3(nblk(n)), dim3(256), 0, st, abort, n, b.h, node, b.cls, b.roots,
                                   b.cnt, cursor, n_take, k, g->done);
                FGI_TRY(wave(n, b.roots, nullptr, b.cnt));   // displacement cascade (ComputedRegistry.cs:91-94)
                touch(g);
                note_words(g);
                const InstallArgs ia{b.h,        b.ver,      b.flags,    b.cls,       take, cursor, g->n_slots, node,
                                     g->row_off, g->row_len, g->row_cap, g->used_cnt, g->home, b.out32};
                hipLaunchKernelGGL(kb_bc_install, dim3(nblk(n)), dim3(256), 0, st, abort, n, ia);
                break;
            }
            case FGI_STEP_ADD_USED: {
                FGI_TRY(fold(g));
                note_words(g);
                touch(g);
                const AuArgs aa{b.h,        b.used,     g->n_slots, g->home,     node,        g->row_off,
                                g->row_len, g->row_cap, g->used_cnt, g->pool_col, g->pool_tag, b.hash,
                                b.hcap - 1, b.out32,    b.cand,     b.pend,      b.ovf,       b.cnt};
                if (from == k && b.hcap == 0) {   // resumed after a pool growth: relocate and finish
                    hipLaunchKernelGGL(kb_au_relocate, dim3(grid), dim3(256), 0, st, abort, aa, g->pool_top_dev);
                    hipLaunchKernelGGL(kb_au_pending, dim3(grid), dim3(256), 0, st, abort, aa);
                    break;
                }
                FGI_HIP(g, hipMemsetAsync(b.hash, 0xFF, b.hcap * sizeof(unsigned long long), st));
                hipLaunchKernelGGL(kb_au_classify, dim3(nblk(n)), dim3(256), 0, st, abort, n, aa);
                hipLaunchKernelGGL(kb_au_reserve, dim3(grid), dim3(256), 0, st, abort, aa,
                                   reinterpret_cast<const unsigned long long*>(g->pool_top_dev), g->pool_cap, k, g->done);
                hipLaunchKernelGGL(kb_au_relocate, dim3(grid), dim3(256), 0, st, abort, aa, g->pool_top_dev);
                hipLaunchKernelGGL(kb_au_pending, dim3(grid), dim3(256), 0, st, abort, aa);
                break;
            }
            case FGI_STEP_SET_OUTPUT:
                FGI_TRY(fold(g));
                note_words(g);
                hipLaunchKernelGGL(kb_set_output, dim3(nblk(n)), dim3(256), 0, st, abort, n, b.h, g->n_handles, node,
                                   b.out8, b.roots, b.cnt);
                FGI_TRY(wave(n, b.roots, nullptr, b.cnt));   // Invalidate() of InvalidateOnSetOutput nodes (153-156)
                break;
            default:
                break;
        }
    }
    FGI_HIP(g, hipGetLastError());
    return FGI_OK;
}

fgi_status fgi_run_batch(fgi_graph* g, uint32_t n_steps, const fgi_step* steps, uint32_t* out_ids, uint64_t cap,
                         uint64_t* out_n, fgi_batch_stats* stats) {
    if (!g || (n_steps && !steps)) return FGI_EINVAL;
    if (coop_launch_mode()) FGI_TRY(coop_warm(g));   // once per graph, before the call's timed span
    const auto t0 = std::chrono::steady_clock::now();
    if (out_n) *out_n = 0;
    uint64_t n_waves = 0, n_begin = 0, n_add = 0;
    for (uint32_t k = 0; k < n_steps; ++k) {   // step kinds and pointers (the elements: while staging)
        const fgi_step& sp = steps[k];
        if (sp.n && !sp.handles) return set_err(g, FGI_EINVAL, "step %u: no handles", k);
        switch (sp.kind) {
            case FGI_STEP_INVALIDATE:
            case FGI_STEP_SET_OUTPUT:
                ++n_waves;
                break;
            case FGI_STEP_BEGIN_COMPUTE:
                if (sp.n && !sp.version) return set_err(g, FGI_EINVAL, "step %u: no versions", k);
                ++n_waves;
                n_begin += sp.n;
                break;
            case FGI_STEP_ADD_USED:
                if (sp.n && !sp.used) return set_err(g, FGI_EINVAL, "step %u: no used handles", k);
                n_add += sp.n;
                break;
            default:
                return set_err(g, FGI_EINVAL, "step %u: unknown kind %u", k, sp.kind);
        }
    }
    FGI_TRY(single_only(g, "fgi_run_batch"));
    const auto t_check = std::chrono::steady_clock::now();
    hipSetDevice(g->device);
    hipStream_t st = g->stream;
    // capacities, before anything is queued: the ids of every cascade, pool headroom for the rows
    // the add_used steps may relocate (an add_used step that needs more resumes after a growth)
    const uint64_t need_out = std::max<uint64_t>(1, n_waves) * g->n_handles;
    if (g->bout_cap < need_out) {
        dfree(g->bout);
        g->bout_cap = 0;
        FGI_TRY(dmalloc(g, &g->bout, need_out));
        g->bout_cap = need_out;
    }
    if (n_add) FGI_TRY(ensure_pool(g, g->pool_top + std::max<uint64_t>(1ull << 20, 4 * n_add)));
    FGI_TRY(ensure_cstart(g, std::max<uint64_t>(g->pool_top, g->pool_cap)));
    const auto t_cap = std::chrono::steady_clock::now();
    // detached handles the begin_compute steps may take (top of the free list)
    const uint64_t n_take = std::min<uint64_t>(n_begin, g->free_detached.size());
    // staging: inputs (uploaded once) | the detached-handle list | outputs (downloaded once)
    size_t in_bytes = stage_round(n_take * 4), out_bytes = 0;
    std::vector<size_t> in_off(n_steps * 4, 0);
    for (uint32_t k = 0; k < n_steps; ++k) {
        const fgi_step& sp = steps[k];
        const size_t n = sp.n;
        in_off[4 * k] = in_bytes;
        in_bytes += stage_round(n * 4);
        if (sp.kind == FGI_STEP_ADD_USED) {
            in_off[4 * k + 1] = in_bytes;
            in_bytes += stage_round(n * 4);
        }
        if (sp.kind == FGI_STEP_BEGIN_COMPUTE) {
            in_off[4 * k + 2] = in_bytes;
            in_bytes += stage_round(n * 8);
        }
        if (sp.flags && (sp.kind == FGI_STEP_BEGIN_COMPUTE || sp.kind == FGI_STEP_INVALIDATE)) {
            in_off[4 * k + 3] = in_bytes;
            in_bytes += stage_round(n);
        }
    }
    std::vector<BatchStep> bs(n_steps);
    for (uint32_t k = 0; k < n_steps; ++k) {
        const fgi_step& sp = steps[k];
        bs[k].out_off = out_bytes;
        if (sp.kind == FGI_STEP_BEGIN_COMPUTE || sp.kind == FGI_STEP_ADD_USED) out_bytes += stage_round(sp.n * 4);
        if (sp.kind == FGI_STEP_SET_OUTPUT) out_bytes += stage_round(sp.n);
    }
    // scratch words: abort, ids, detached taken, accumulators, 4 counters per step, the pool top
    const size_t scr_words = 3 + kAccCount + 4 * (size_t)n_steps + 1;
    const size_t scr_bytes = stage_round(scr_words * 8);
    const size_t ptop_word = scr_words - 1;
    // the ids are copied back with the results when they fit the previous batch's count (+25%)
    const uint64_t spec = out_ids ? std::min<uint64_t>(cap, g->batch_ids_hint + g->batch_ids_hint / 4 + 4096) : 0;
    const size_t res_off = in_bytes + scr_bytes;   // outputs follow the scratch words
    const size_t ids_off = res_off + out_bytes;
    const size_t total = ids_off + stage_round(spec * 4);
    if (g->bst_cap < total) {
        if (g->bst_h) hipHostFree(g->bst_h);
        dfree(g->bst_d);
        g->bst_h = nullptr;
        g->bst_cap = 0;
        const size_t c = std::max(total, g->bst_cap * 2);
        if (hipHostMalloc(reinterpret_cast<void**>(&g->bst_h), c) != hipSuccess) return set_err(g, FGI_ENOMEM, "pinned staging");
        FGI_TRY(dmalloc(g, &g->bst_d, c));
        g->bst_cap = c;
    }
    char* H = g->bst_h;
    char* D = g->bst_d;
    // The single calls' argument checks, made while the inputs are staged (one pass over the caller's
    // arrays): range and version checks as branch-free reductions beside the copies (they vectorise),
    // then a slot-repeat test over the staged copy with a byte per slot (independent stores, no
    // read-modify-write chain through one bitmap word). The first offender is searched for only on
    // failure. Nothing has been queued yet, so a bad step applies nothing.
    for (uint32_t k = 0; k < n_steps; ++k) {
        const fgi_step& sp = steps[k];
        const uint32_t n = sp.n;
        uint32_t* hh = reinterpret_cast<uint32_t*>(H + in_off[4 * k]);
        bs[k].h = reinterpret_cast<const uint32_t*>(D + in_off[4 * k]);
        if (sp.kind == FGI_STEP_BEGIN_COMPUTE) {
            uint64_t* hv = reinterpret_cast<uint64_t*>(H + in_off[4 * k + 2]);
            uint32_t hmax = 0;
            uint64_t vbad = 0;
            for (uint32_t i = 0; i < n; ++i) {
                const uint32_t x = sp.handles[i];
                const uint64_t v = sp.version[i];
                hh[i] = x;
                hv[i] = v;
                hmax = std::max(hmax, x);
                vbad |= (uint64_t)(v - 1 >= kVMask);   // version 0 or > kVMask
            }
            std::vector<uint8_t>& seen = g->seen_slots;
            if (seen.size() < g->ext_slots) seen.assign(g->ext_slots, 0);
            uint32_t dup = 0;
            if (hmax < g->ext_slots && !vbad) {
                for (uint32_t i = 0; i < n; ++i) {
                    dup |= seen[hh[i]];
                    seen[hh[i]] = 1;
                }
                for (uint32_t i = 0; i < n; ++i) seen[hh[i]] = 0;
            }
            if (hmax >= g->ext_slots || vbad || dup) {
                const char* why = "bad step";
                uint32_t i = 0, bad = 0;
                for (; i < n; ++i) {
                    const uint32_t x = sp.handles[i];
                    if (x >= g->ext_slots) { why = "slot out of range"; bad = x; break; }
                    if (sp.version[i] == 0 || sp.version[i] > kVMask) { why = "bad version"; bad = i; break; }
                    if (seen[x]) { why = "slot repeated in one step"; bad = x; break; }
                    seen[x] = 1;
                }
                for (uint32_t j = 0; j < i; ++j) seen[sp.handles[j]] = 0;
                return set_err(g, FGI_EINVAL, "step %u: %s (%u)", k, why, bad);
            }
            bs[k].ver = reinterpret_cast<const uint64_t*>(D + in_off[4 * k + 2]);
        } else if (sp.kind == FGI_STEP_ADD_USED) {
            uint32_t* hu = reinterpret_cast<uint32_t*>(H + in_off[4 * k + 1]);
            uint32_t hmax = 0;
            for (uint32_t i = 0; i < n; ++i) {
                const uint32_t d = sp.handles[i], u = sp.used[i];
                hh[i] = d;
                hu[i] = u;
                hmax = std::max(hmax, std::max(d, u));
            }
            if (n && hmax >= g->ext_handles)
                for (uint32_t i = 0; i < n; ++i)
                    if (sp.handles[i] >= g->ext_handles || sp.used[i] >= g->ext_handles)
                        return set_err(g, FGI_EINVAL, "step %u: handle out of range at %u", k, i);
            bs[k].used = reinterpret_cast<const uint32_t*>(D + in_off[4 * k + 1]);
        } else {
            std::memcpy(hh, sp.handles, (size_t)n * 4);
        }
        if (in_off[4 * k + 3]) {
            std::memcpy(H + in_off[4 * k + 3], sp.flags, n);
            bs[k].flags = reinterpret_cast<const uint8_t*>(D + in_off[4 * k + 3]);
        }
    }
    if (n_take) std::memcpy(H, g->free_detached.data() + (g->free_detached.size() - n_take), n_take * 4);
    const auto t_stage = std::chrono::steady_clock::now();
    unsigned long long* scr = reinterpret_cast<unsigned long long*>(D + in_bytes);
    unsigned long long* scr_h = reinterpret_cast<unsigned long long*>(H + in_bytes);
    std::memset(scr_h, 0, scr_words * 8);
    hipEvent_t b0 = g->ev_w0, b1 = g->ev_w1;
    // FGI_BATCH_TIMES=1: the call's host phases on stderr (staging, enqueue, wait, unpacking; us)
    static const bool times = getenv("FGI_BATCH_TIMES") != nullptr;
    using clk = std::chrono::steady_clock;
    const clk::time_point t_pack = times ? clk::now() : t0;
    clk::time_point t_enq = t_pack, t_wait = t_pack;
    FGI_HIP(g, hipEventRecord(b0, st));
    FGI_HIP(g, hipMemcpyAsync(D, H, in_bytes + scr_words * 8, hipMemcpyHostToDevice, st));   // one upload
    for (uint32_t k = 0; k < n_steps && g->lbl_K; ++k) {   // the steps' handles as labels
        const fgi_step& sp = steps[k];
        FGI_TRY(labels_map_in(g, reinterpret_cast<uint32_t*>(D + in_off[4 * k]), sp.n));
        if (sp.kind == FGI_STEP_ADD_USED) FGI_TRY(labels_map_in(g, reinterpret_cast<uint32_t*>(D + in_off[4 * k + 1]), sp.n));
    }
    // per-step device temporaries
    for (uint32_t k = 0; k < n_steps; ++k) {
        const fgi_step& sp = steps[k];
        BatchStep& b = bs[k];
        const uint32_t n = sp.n;
        b.cnt = scr + 3 + kAccCount + 4 * k;
        if (!n) continue;
        b.tmp.resize(8);
        switch (sp.kind) {
            case FGI_STEP_BEGIN_COMPUTE:
                FGI_TRY(tmalloc(g, b.tmp[0], &b.cls, n));
                FGI_TRY(tmalloc(g, b.tmp[1], &b.roots, n));
                b.out32 = reinterpret_cast<uint32_t*>(D + res_off + b.out_off);
                break;
            case FGI_STEP_ADD_USED:
                b.hcap = 64;
                while (b.hcap < 2ull * n) b.hcap <<= 1;
                FGI_TRY(tmalloc(g, b.tmp[0], &b.hash, b.hcap));
                FGI_TRY(tmalloc(g, b.tmp[1], &b.cand, n));
                FGI_TRY(tmalloc(g, b.tmp[2], &b.pend, n));
                FGI_TRY(tmalloc(g, b.tmp[3], &b.ovf, n));
                b.out32 = reinterpret_cast<uint32_t*>(D + res_off + b.out_off);
                break;
            case FGI_STEP_SET_OUTPUT:
                b.out8 = reinterpret_cast<uint8_t*>(D + res_off + b.out_off);
                FGI_TRY(tmalloc(g, b.tmp[1], &b.roots, n));
                break;
            default:
                break;
        }
    }
    const uint32_t* take = reinterpret_cast<const uint32_t*>(D);
    std::vector<std::pair<hipEvent_t, hipEvent_t>> wave_ev;
    const bool timed = stats && g->opt_level_timing;
    uint32_t syncs = 0, from = 0;
    g->last_wave_n = 0;
    while (true) {
        fgi_status s = batch_launch(g, from, n_steps, steps, bs, scr, take, n_take, timed, wave_ev);
        if (s != FGI_OK) return s;
        // results: the counters, the pool top and every step's output in one copy, the ids (as
        // many as the previous batch had, +25%) in a second, then one wait
        hipLaunchKernelGGL(kb_finish, dim3(1), dim3(64), 0, st, g->pool_top_dev, scr + ptop_word);
        FGI_HIP(g, hipMemcpyAsync(H + in_bytes, D + in_bytes, scr_bytes + out_bytes, hipMemcpyDeviceToHost, st));
        if (spec) FGI_HIP(g, hipMemcpyAsync(H + ids_off, g->bout, spec * 4, hipMemcpyDeviceToHost, st));
        FGI_HIP(g, hipEventRecord(b1, st));
        if (times) t_enq = clk::now();
#if FGI_SPIN_WAIT
        // the host spins on a published sequence word behind the copies (wave.hip publish_wait) instead
        // of a stream synchronisation; b1 is complete by then, so its wait returns at once
        FGI_TRY(publish_wait(g, st, g->pool_top_dev, 0, g->red_pub));
        FGI_HIP(g, hipEventSynchronize(b1));
#else
        FGI_HIP(g, hipStreamSynchronize(st));
#endif
        if (times) t_wait = clk::now();
        ++syncs;
        g->pool_top = scr_h[ptop_word];
        const unsigned long long ab = scr_h[0];
        if (scr_h[3 + kAccBarrierIdx] || (ab >> 32) == kAbortBarrier) {
            // a cascade's grid barrier timed out: its blocks left without finishing, the batch's later
            // kernels did nothing. The detached handles the device consumed are accounted for, the
            // barrier counter restarts, and the graph is poisoned until fgi_restore (fgi.h).
            g->free_detached.resize(g->free_detached.size() - (size_t)std::min<uint64_t>(scr_h[2], n_take));
            FGI_HIP(g, hipMemsetAsync(g->gbar, 0, kGbarWords * sizeof(unsigned long long), st));
            FGI_HIP(g, hipStreamSynchronize(st));
            g->failed = true;
            g->coop_clean = false;
            note_words(g);
            touch(g);
            return set_err(g, FGI_EDEVICE,
                           "a cascade's grid barrier timed out (blocks of one grid were not resident together); "
                           "the batch is half-applied and the graph unusable until fgi_restore");
        }
        if (!ab) break;
        const uint32_t k = (uint32_t)(ab & 0xFFFFFFFFull) - 1;
        if ((ab >> 32) == kAbortPool) {   // grow the pool, then finish step k and run the rest
            const unsigned long long need = bs[k].cnt ? scr_h[3 + kAccCount + 4 * k + 3] : 0;
            FGI_TRY(ensure_pool(g, g->pool_top + need + std::max<uint64_t>(1ull << 20, 4 * n_add)));
            scr_h[0] = 0;
            FGI_HIP(g, hipMemcpyAsync(scr, scr_h, 8, hipMemcpyHostToDevice, st));
            bs[k].hcap = 0;   // marks the resumed step: relocation and pending entries only
            from = k;
            continue;
        }
        // out of detached handles at step k: steps before it are applied
        g->free_detached.resize(g->free_detached.size() - (size_t)scr_h[2]);
        return set_err(g, FGI_ECAPACITY, "step %u: out of detached handles (%zu free)", k, g->free_detached.size());
    }
    // host bookkeeping: the detached handles taken, the per-step outputs
    g->free_detached.resize(g->free_detached.size() - (size_t)scr_h[2]);
    for (uint32_t k = 0; k < n_steps; ++k) {
        const fgi_step& sp = steps[k];
        if (!sp.out || !sp.n) continue;
        const char* src = H + res_off + bs[k].out_off;
        if (sp.kind == FGI_STEP_SET_OUTPUT) std::memcpy(sp.out, src, sp.n);
        else if (sp.kind == FGI_STEP_BEGIN_COMPUTE || sp.kind == FGI_STEP_ADD_USED) std::memcpy(sp.out, src, sp.n * 4);
        if (sp.kind == FGI_STEP_BEGIN_COMPUTE && g->lbl_K) {   // detached handles: label K + handle
            uint32_t* o = static_cast<uint32_t*>(sp.out);
            for (uint32_t i = 0; i < sp.n; ++i)
                if (o[i] != FGI_NONE) o[i] -= g->lbl_K;
        }
    }
    g->stale_est += scr_h[3 + 3] + scr_h[3 + 4];   // the cascades' E_trav + E_match (fgi_prune_step)
#if FGI_PROBE
    if (getenv("FGI_TRACE")) print_coop_probe();
#endif
    const uint64_t n_ids = scr_h[1];
    if (out_n) *out_n = n_ids;
    g->batch_ids_hint = n_ids;
    fgi_status ret = FGI_OK;
    if (out_ids) {
        if (n_ids > cap) {
            ret = FGI_ECAPACITY;
        } else if (n_ids <= spec && from == 0) {
            std::memcpy(out_ids, H + ids_off, n_ids * 4);
        } else if (n_ids) {
            FGI_HIP(g, hipMemcpyAsync(out_ids, g->bout, n_ids * 4, hipMemcpyDeviceToHost, st));
            FGI_HIP(g, hipStreamSynchronize(st));
            ++syncs;
        }
    }
    if (times) {
        const clk::time_point t_end = clk::now();
        auto us = [](clk::time_point a, clk::time_point b) { return std::chrono::duration<double, std::micro>(b - a).count(); };
        fprintf(stderr, "[fgi] batch check %.1f cap %.1f stage %.1f pack %.1f enqueue %.1f wait %.1f unpack %.1f total %.1f us (%u steps)\n",
                us(t0, t_check), us(t_check, t_cap), us(t_cap, t_stage), us(t_check, t_pack),
                us(t_pack, t_enq), us(t_enq, t_wait), us(t_wait, t_end), us(t0, t_end), n_steps);
    }
    if (stats) {
        const unsigned long long* acc = scr_h + 3;
        stats->waves += acc[0];
        stats->levels += acc[1];
        stats->v_inv += acc[2];
        stats->e_trav += acc[3];
        stats->e_match += acc[4];
        stats->n_flagged += acc[5];
        float ms = 0;
        if (hipEventElapsedTime(&ms, b0, b1) == hipSuccess) stats->kernel_ms += ms;
        for (auto& e : wave_ev)
            if (hipEventElapsedTime(&ms, e.first, e.second) == hipSuccess) stats->wave_ms += ms;
        stats->host_syncs += syncs;
        stats->total_ms += std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    }
    return ret;
}

// PruneUsedBy over the rows of handles [lo, hi) in place (queued, no synchronisation): the
// counters land in st[kPrN].
// e0 (nullable) is recorded right before the launch: the temporaries, their clearing and the first
// occupancy query (which loads the kernel's code object) stay outside the timed span
static fgi_status prune_range_launch(fgi_graph* g, uint32_t lo, uint32_t hi, Tmp& tmap, Tmp& tcst, Tmp& tcur,
                                     unsigned long long* st, hipEvent_t e0) {
    hipStream_t s = g->stream;
    // every chunk holds more than kPruneLong / 2 entries of a row: the pool bounds their number
    const uint64_t max_chunks = g->pool_top / (kPruneLong / 2) + 1;
    PruneArgs a{};
    FGI_TRY(tmalloc(g, tmap, &a.chunk_map, max_chunks));
    FGI_TRY(tmalloc(g, tcst, &a.chunk_st, max_chunks));
    FGI_HIP(g, hipMemsetAsync(a.chunk_st, 0, max_chunks * sizeof(uint32_t), s));
    // each phase on the blocks the chip holds at once (chunks wait on earlier chunks: a second round
    // of blocks would leave a tail)
    static int per_cu = 0, per_cu2 = 0;
    if (per_cu == 0 && (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, k_prune_rows, 256, 0) != hipSuccess || per_cu < 1))
        per_cu = 1;
    if (per_cu2 == 0 &&
        (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu2, k_prune_chunks, 256, 0) != hipSuccess || per_cu2 < 1))
        per_cu2 = 1;
    const uint64_t resident = (uint64_t)per_cu * (uint64_t)std::max(g->n_cu, 1);
    const uint32_t grid = (uint32_t)std::max<uint64_t>(1, std::min<uint64_t>(resident, nblk((uint64_t)(hi - lo) * 64)));
    a.lo = lo;
    a.hi = hi;
    a.n_slots = g->n_slots;
    a.s2l = g->lbl_hot ? g->s2l : nullptr;
    a.ext_slots = g->ext_slots;
    a.K = g->lbl_K;
    a.node = reinterpret_cast<const unsigned long long*>(g->node);
    a.row_off = g->row_off;
    a.row_len = g->row_len;
    a.pool_col = g->pool_col;
    a.pool_tag = g->pool_tag;
    a.st = st;
    PartView pv;
    if (part_view(g, &pv)) {   // a partition: the dependants' current bits and versions of every rank
        unsigned long long *cl, *ca;
        uint64_t w64 = 0;
        FGI_TRY(part_cur_buffers(g, &cl, &ca, &w64));
        FGI_HIP(g, hipMemsetAsync(cl, 0, w64 * 8, s));
        hipLaunchKernelGGL(k_build_cur, dim3(std::min<uint32_t>((pv.n_local + 255) / 256 + 1, 8192)), dim3(256), 0, s,
                           pv.n_local, a.node, cl);
        FGI_TRY(part_allgather_cur(g));
        a.ver_all = pv.ver_all;
        a.cur_all = ca;
        a.pblock = pv.block;
        a.pw64 = (uint32_t)w64;
    } else
    // fast path: the entries' liveness at list build still holds (no mutation, no compaction since)
    if (g->pool_live && g->pl_mut_epoch == g->mut_epoch && g->pl_pool_epoch == g->pool_epoch &&
        g->pool_top <= g->pool_live_cap && !getenv("FGI_PRUNE_GATHER")) {
        uint32_t* cur;
        FGI_TRY(tmalloc(g, tcur, &cur, g->bm_words));
        const uint32_t H = g->n_handles;
        hipLaunchKernelGGL(k_build_cur, dim3(std::min<uint32_t>((H + 255) / 256 + 1, 8192)), dim3(256), 0, s, H,
                           a.node, reinterpret_cast<unsigned long long*>(cur));
        a.live_bm = g->pool_live;
        a.cur_bm = cur;
    }
    if (getenv("FGI_TRACE")) fprintf(stderr, "[fgi] prune [%u, %u): %u blocks (%d per CU)\n", lo, hi, grid, per_cu);
    if (e0) FGI_HIP(g, hipEventRecord(e0, s));
    hipLaunchKernelGGL(k_prune_rows, dim3(grid), dim3(256), 0, s, a);
    const uint64_t resident2 = (uint64_t)per_cu2 * (uint64_t)std::max(g->n_cu, 1);
    hipLaunchKernelGGL(k_prune_chunks, dim3((uint32_t)std::min<uint64_t>(resident2, max_chunks)), dim3(256), 0, s, a);
    FGI_HIP(g, hipGetLastError());
    return FGI_OK;
}

// Copy every row to a fresh pool with slack (len + max(4, len / 8)): the holes pruning left go away.
static fgi_status defragment(fgi_graph* g) {
    hipStream_t s = g->stream;
    const uint32_t H = g->n_handles;
    Tmp tc, to, ts;
    uint64_t *cap64, *noff;
    FGI_TRY(tmalloc(g, tc, &cap64, H));
    FGI_TRY(tmalloc(g, to, &noff, H));
    hipLaunchKernelGGL(k_defrag_caps, dim3(nblk(H)), dim3(256), 0, s, H, g->row_len, cap64);
    size_t tb = 0;
    FGI_HIP(g, rocprim::exclusive_scan(nullptr, tb, cap64, noff, (uint64_t)0, (size_t)H, rocprim::plus<uint64_t>(), s));
    char* tmp;
    FGI_TRY(tmalloc(g, ts, &tmp, tb));
    FGI_HIP(g, rocprim::exclusive_scan(tmp, tb, cap64, noff, (uint64_t)0, (size_t)H, rocprim::plus<uint64_t>(), s));
    uint64_t last_off = 0, last_cap = 0;
    FGI_TRY(d2h(g, &last_off, noff + H - 1, 1));
    FGI_TRY(d2h(g, &last_cap, cap64 + H - 1, 1));
    const uint64_t total = last_off + last_cap;
    // pool positions are 32-bit in the traversal kernels (ensure_pool's limit): a defragmented pool
    // that would not fit below 2^32 is not made — the rows stay where they are
    constexpr uint64_t kMaxPool = 1ull << 32;
    if (total > kMaxPool) return FGI_OK;
    const uint64_t cap = std::min<uint64_t>(std::max<uint64_t>(total + total / 8, 1024), kMaxPool);
    uint32_t* ncol = nullptr;
    uint64_t* ntag = nullptr;
    FGI_TRY(dmalloc(g, &ncol, cap));
    if (dmalloc(g, &ntag, cap) != FGI_OK) {
        hipFree(ncol);
        return FGI_ENOMEM;
    }
    const uint32_t grid = (uint32_t)std::min<uint64_t>(nblk((uint64_t)H * 64), 8192);
    hipLaunchKernelGGL(k_defrag_rows, dim3(grid), dim3(256), 0, s, H, noff, g->row_off, g->row_len, g->pool_col,
                       g->pool_tag, ncol, ntag);
    hipLaunchKernelGGL(k_defrag_apply, dim3(nblk(H)), dim3(256), 0, s, H, noff, cap64, g->row_off, g->row_cap);
    FGI_HIP(g, hipGetLastError());
    FGI_HIP(g, hipStreamSynchronize(s));
    dfree(g->pool_col);
    dfree(g->pool_tag);
    g->pool_col = ncol;
    g->pool_tag = ntag;
    g->pool_cap = cap;
    g->pool_top = total;
    g->pool_epoch++;
    FGI_HIP(g, hipMemcpy(g->pool_top_dev, &g->pool_top, sizeof(uint64_t), hipMemcpyHostToDevice));
    return ensure_cstart(g, cap);
}

static fgi_status prune_rows(fgi_graph* g, uint32_t lo, uint32_t hi, bool allow_defrag, fgi_prune_stats* stats,
                             bool part_ok = false) {
    if (part_ok) FGI_TRY(usable(g));
    else FGI_TRY(single_only(g, "fgi_prune"));
    hipSetDevice(g->device);
    const auto t0 = std::chrono::steady_clock::now();
    FGI_TRY(fold(g));
    hipStream_t s = g->stream;
    unsigned long long* st = g->misc_dev;
    FGI_HIP(g, hipMemsetAsync(st, 0, kPrN * sizeof(unsigned long long), s));
    hipEvent_t e0 = g->ev_w0, e1 = g->ev_w1;
    Tmp tmap, tcst, tcur;
    if (hi > lo) FGI_TRY(prune_range_launch(g, lo, hi, tmap, tcst, tcur, st, e0));
    else FGI_HIP(g, hipEventRecord(e0, s));
    FGI_HIP(g, hipEventRecord(e1, s));
    unsigned long long c[kPrN];
    FGI_TRY(d2h(g, c, st, kPrN));
    float ms = 0;
    hipEventElapsedTime(&ms, e0, e1);
    touch(g);
    // rows compacted in place: a snapshot's row descriptors no longer describe them (entries moved
    // left, freed slack reused by later appends), so fgi_restore must refuse as after a rebuild
    if (c[kPrNew] != c[kPrOld] || c[kPrDropped] != 0) g->pool_epoch++;
    const uint64_t pool_before = g->pool_top;
    // the full pass knows every row's length: defragment when holes are most of the pool
    if (allow_defrag && lo == 0 && hi == g->ext_handles && g->opt_defrag_pct > 0 &&
        (g->pool_top - std::min<uint64_t>(g->pool_top, c[kPrLive])) * 100 > (uint64_t)g->opt_defrag_pct * g->pool_top)
        FGI_TRY(defragment(g));
    if (stats) {
        stats->old_edges = c[kPrOld];
        stats->new_edges = c[kPrNew];
        stats->pool_before = pool_before;
        stats->pool_after = g->pool_top;
        stats->kernel_ms = ms;
        stats->total_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
        stats->live_edges = c[kPrLive];
        stats->dropped_edges = c[kPrDropped];
        stats->first = lo;
        stats->count = hi - lo;
    }
    g->stale_est = 0;
    return FGI_OK;
}

fgi_status fgi_prune(fgi_graph* g, fgi_prune_stats* stats) {
    if (!g) return FGI_EINVAL;
    FGI_TRY(usable(g));
    if (stats) *stats = fgi_prune_stats{};
    return prune_rows(g, 0, g->ext_handles, true, stats);
}

fgi_status fgi_prune_range(fgi_graph* g, uint32_t first, uint32_t count, fgi_prune_stats* stats) {
    if (!g) return FGI_EINVAL;
    FGI_TRY(usable(g));
    if (stats) *stats = fgi_prune_stats{};
    if (first > g->ext_handles) return set_err(g, FGI_EINVAL, "first handle %u out of range", first);
    const uint32_t hi = (uint32_t)std::min<uint64_t>((uint64_t)first + count, g->ext_handles);
    return prune_rows(g, first, hi, false, stats);
}

fgi_status fgi_prune_step(fgi_graph* g, uint32_t batch, uint32_t stale_pct, fgi_prune_stats* stats) {
    if (!g || batch == 0) return FGI_EINVAL;
    FGI_TRY(usable(g));
    if (stats) *stats = fgi_prune_stats{};
    // ComputedGraphPruner (Internal/ComputedGraphPruner.cs:50-110) walks the registry in batches;
    // here a batch runs only while the estimated stale entries exceed stale_pct of the pool
    if ((uint64_t)g->stale_est * 100 < (uint64_t)stale_pct * std::max<uint64_t>(g->pool_top, 1)) return FGI_OK;
    const uint32_t lo = g->prune_cursor;
    const uint32_t hi = (uint32_t)std::min<uint64_t>((uint64_t)lo + batch, g->ext_handles);
    const uint64_t est = g->stale_est;
    FGI_TRY(prune_rows(g, lo, hi, false, stats));
    g->prune_cursor = hi >= g->ext_handles ? 0 : hi;
    // the estimate shrinks by the share of the handles this batch covered
    g->stale_est = hi >= g->ext_handles ? 0 : est - est * (uint64_t)(hi - lo) / std::max<uint32_t>(g->ext_handles, 1);
    if (stats) stats->stale_estimate = est;
    return FGI_OK;
}

fgi_status fgi_release(fgi_graph* g, uint32_t n, const uint32_t* handle) {
    if (!g || (n && !handle)) return FGI_EINVAL;
    FGI_TRY(usable(g));
    hipSetDevice(g->device);
    FGI_TRY(fold(g));
    if (n) note_words(g);
    for (uint32_t i = 0; i < n; ++i) {
        if (handle[i] < g->ext_slots || handle[i] >= g->ext_handles)
            return set_err(g, FGI_EINVAL, "handle %u is not detached", handle[i]);
        const uint32_t h = handle[i] + g->lbl_K;   // a detached handle's label
        if (std::find(g->free_detached.begin(), g->free_detached.end(), h) != g->free_detached.end())
            return set_err(g, FGI_EINVAL, "handle %u released twice", h);
        const uint64_t zero = 0;
        const uint32_t z32 = 0;
        FGI_TRY(h2d(g, g->node + h, &zero, 1));
        FGI_TRY(h2d(g, g->row_len + h, &z32, 1));
        FGI_TRY(h2d(g, g->row_cap + h, &z32, 1));
        FGI_TRY(h2d(g, g->row_off + h, &zero, 1));
        FGI_HIP(g, hipStreamSynchronize(g->stream));
        g->free_detached.push_back(h);
        touch(g);
    }
    return FGI_OK;
}

// ---- partitioned mutations, prune and batches ----------------------
// A partitioned graph takes the registry's mutations too. Every rank makes the same call with the same
// arguments (global slot ids), in the same order: each applies the items of the slots it owns, writes
// every listed version into its replica (ver_all), and joins the call's collectives — the cascades
// (run_part_wave: displacement, InvalidateOnSetOutput, the invalidation steps) and the all-reduces
// that carry a pair's state between the ranks owning its two ends (AddUsed / AddUsedBy).
namespace {

fgi_status part_check(fgi_graph* g, PartView* pv, const char* what) {
    if (!g->part || !part_view(g, pv)) return set_err(g, FGI_ESTATE, "%s: partition not initialised", what);
    return usable(g);
}

// this rank's ids of the last partitioned wave (global, ascending) appended to *ids
fgi_status part_take_ids(fgi_graph* g, const PartView& pv, std::vector<uint32_t>* ids) {
    if (!ids || g->last_wave_n == 0) return FGI_OK;
    const size_t at = ids->size();
    ids->resize(at + g->last_wave_n);
    FGI_TRY(d2h(g, ids->data() + at, g->inv, g->last_wave_n));
    for (size_t i = at; i < ids->size(); ++i) (*ids)[i] = part_slot_of(g, (*ids)[i] + pv.base);
    if (g->lbl_perm) std::sort(ids->begin() + (ptrdiff_t)at, ids->end());   // the cascade's slots, ascending
    return FGI_OK;
}

fgi_status part_check_slots(fgi_graph* g, const PartView& pv, uint32_t n, const uint32_t* slot, bool distinct) {
    for (uint32_t i = 0; i < n; ++i)
        if (slot[i] >= pv.n_global) return set_err(g, FGI_EINVAL, "slot %u out of range", slot[i]);
    if (distinct && n > 1) {
        std::vector<uint32_t> c(slot, slot + n);
        std::sort(c.begin(), c.end());
        for (uint32_t i = 1; i < n; ++i)
            if (c[i] == c[i - 1]) return set_err(g, FGI_EINVAL, "slot repeated in one batch (%u)", c[i]);
    }
    return FGI_OK;
}

// a cascade from host root slots (global ids; each rank starts the ones it owns), on every rank
fgi_status part_wave_host(fgi_graph* g, const PartView& pv, uint32_t n, const uint32_t* slots, const uint8_t* imm,
                          fgi_wave_stats* stats, std::vector<uint32_t>* ids) {
    (void)pv;
    Tmp tr, ti;
    uint32_t* dr = nullptr;
    uint8_t* di = nullptr;
    if (n) {
        FGI_TRY(tmalloc(g, tr, &dr, n));
        FGI_TRY(h2d(g, dr, slots, n));
        if (imm) {
            FGI_TRY(tmalloc(g, ti, &di, n));
            FGI_TRY(h2d(g, di, imm, n));
        }
    }
    g->last_wave_n = 0;
    FGI_TRY(run_part_wave(g, n, dr, di, stats));
    return part_take_ids(g, pv, ids);
}

// ComputeMethodFunctionBase.Compute + ComputedRegistry.Register with displacement (as
// fgi_begin_compute) over a partition: out_detached[i] is the detached local handle on the slot's
// owner (FGI_NONE elsewhere and for nodes not detached)
fgi_status part_begin_compute(fgi_graph* g, uint32_t n, const uint32_t* slot, const uint64_t* version,
                              const uint8_t* has_delay, uint32_t* out_detached, fgi_wave_stats* stats,
                              std::vector<uint32_t>* ids) {
    PartView pv;
    FGI_TRY(part_check(g, &pv, "fgi_part_begin_compute"));
    if (n && (!slot || !version)) return FGI_EINVAL;
    FGI_TRY(part_check_slots(g, pv, n, slot, true));
    for (uint32_t i = 0; i < n; ++i)
        if (version[i] == 0 || version[i] > kVMask) return set_err(g, FGI_EINVAL, "bad version (%u)", i);
    hipSetDevice(g->device);
    hipStream_t st = g->stream;
    std::vector<uint32_t> li, ls;
    std::vector<uint64_t> lv;
    std::vector<uint8_t> ld;
    for (uint32_t i = 0; i < n; ++i)
        if (slot[i] - pv.base < pv.n_local) {
            li.push_back(i);
            ls.push_back(slot[i] - pv.base);
            lv.push_back(version[i]);
            ld.push_back(has_delay ? has_delay[i] : 0);
        }
    const uint32_t m = (uint32_t)li.size();
    Tmp ts, tv, td, tc, tr, to, tf, tflag, tall, tallv;
    uint32_t *ds = nullptr, *droots = nullptr, *dout = nullptr, *dfree_h = nullptr, *dflag = nullptr;
    uint64_t* dv = nullptr;
    uint8_t *dd = nullptr, *dcls = nullptr;
    FGI_TRY(fold(g));
    FGI_HIP(g, hipMemsetAsync(g->misc_dev, 0, 4 * sizeof(unsigned long long), st));
    if (m) {
        FGI_TRY(tmalloc(g, ts, &ds, m));
        FGI_TRY(tmalloc(g, tv, &dv, m));
        FGI_TRY(tmalloc(g, td, &dd, m));
        FGI_TRY(tmalloc(g, tc, &dcls, m));
        FGI_TRY(tmalloc(g, tr, &droots, m));
        FGI_TRY(tmalloc(g, to, &dout, m));
        FGI_TRY(h2d(g, ds, ls.data(), m));
        FGI_TRY(h2d(g, dv, lv.data(), m));
        FGI_TRY(h2d(g, dd, ld.data(), m));
        hipLaunchKernelGGL(k_bc_classify, dim3(nblk(m)), dim3(256), 0, st, m, ds,
                           reinterpret_cast<const unsigned long long*>(g->node), dcls, droots, g->misc_dev);
    }
    unsigned long long cnt[2];
    FGI_TRY(d2h(g, cnt, g->misc_dev, 2));
    // one all-reduce: which items each owner detaches (their slots' nodes stay current), and whether
    // any rank is short of detached handles — then every rank applies the call, or none does
    std::vector<uint8_t> cls(m);
    if (m) FGI_TRY(d2h(g, cls.data(), dcls, m));
    std::vector<uint32_t> fl(n + 1, 0);
    for (uint32_t j = 0; j < m; ++j) fl[li[j]] = cls[j] == 2 ? 1u : 0u;
    fl[n] = cnt[1] > g->free_detached.size() ? 1u : 0u;
    FGI_TRY(tmalloc(g, tflag, &dflag, n + 1));
    FGI_TRY(h2d(g, dflag, fl.data(), n + 1));
    FGI_TRY(part_allreduce_u32(g, dflag, n + 1));
    FGI_TRY(d2h(g, fl.data(), dflag, n + 1));
    if (fl[n])
        return set_err(g, FGI_ECAPACITY, "a rank is out of detached handles (this one: %zu free, %llu needed)",
                       g->free_detached.size(), cnt[1]);
    // A detached node keeps its row under a local handle no slot id reaches, so its dependants' entries
    // must leave their pull lists (push levels start from the slot's new, empty row); this rank's
    // dependency entries on any rank's detached slots die
    {
        std::vector<uint32_t> det;
        for (uint32_t i = 0; i < n; ++i)
            if (fl[i]) det.push_back(slot[i]);
        FGI_TRY(part_kill_used(g, std::move(det)));
    }
    // the displacement cascade (ComputedRegistry.cs:91-94) on every rank, then versions and installs
    if (cnt[0]) hipLaunchKernelGGL(k_add_base, dim3(nblk(cnt[0])), dim3(256), 0, st, (uint32_t)cnt[0], droots, pv.base);
    g->last_wave_n = 0;
    FGI_TRY(run_part_wave(g, (uint32_t)cnt[0], droots, nullptr, stats));
    FGI_TRY(part_take_ids(g, pv, ids));
    if (n) {
        uint32_t* as = nullptr;
        uint64_t* av = nullptr;
        FGI_TRY(tmalloc(g, tall, &as, n));
        FGI_TRY(tmalloc(g, tallv, &av, n));
        FGI_TRY(h2d(g, as, slot, n));
        FGI_TRY(h2d(g, av, version, n));
        hipLaunchKernelGGL(k_set_versions, dim3(nblk(n)), dim3(256), 0, st, n, as, av, pv.ver_all);
    }
    std::vector<uint32_t> od(m, FGI_NONE);
    if (m) {
        std::vector<uint32_t> take(g->free_detached.end() - (ptrdiff_t)cnt[1], g->free_detached.end());
        FGI_TRY(tmalloc(g, tf, &dfree_h, take.size() + 1));
        FGI_TRY(h2d(g, dfree_h, take.data(), take.size()));
        FGI_TRY(fold(g));   // the displacement cascade's visits
        FGI_HIP(g, hipMemsetAsync(g->misc_dev + 2, 0, sizeof(unsigned long long), st));
        const InstallArgs ia{ds,         dv,          dd,        dcls,      dfree_h, g->misc_dev + 2, g->n_slots,
                             reinterpret_cast<unsigned long long*>(g->node), g->row_off, g->row_len, g->row_cap,
                             g->used_cnt, g->home, dout};
        hipLaunchKernelGGL(k_bc_install, dim3(nblk(m)), dim3(256), 0, st, m, ia);
        FGI_HIP(g, hipGetLastError());
        FGI_TRY(d2h(g, od.data(), dout, m));
        g->free_detached.resize(g->free_detached.size() - take.size());
    } else {
        FGI_HIP(g, hipStreamSynchronize(st));
    }
    if (out_detached) {
        for (uint32_t i = 0; i < n; ++i) out_detached[i] = FGI_NONE;
        for (uint32_t j = 0; j < m; ++j) out_detached[li[j]] = od[j];
    }
    touch(g);
    note_words(g);
    return FGI_OK;
}

// dependant.AddUsed(used) over a partition (Computed.cs:347-385) for pairs of global slots (their
// current nodes): the dependant's owner says whether it is Computing (all-reduce), the used node's
// owner applies AddUsedBy's rules and appends the entry to its row, the results are all-reduced, and
// the dependant's owner applies InvalidateOnSetOutput / counts the new dependency and records it
// for its pull lists. out_result (every pair, every rank): FGI_USED_*
fgi_status part_add_used(fgi_graph* g, uint32_t n, const uint32_t* dep, const uint32_t* used, uint32_t* out_result) {
    PartView pv;
    FGI_TRY(part_check(g, &pv, "fgi_part_add_used"));
    if (n && (!dep || !used)) return FGI_EINVAL;
    FGI_TRY(part_check_slots(g, pv, n, dep, false));
    FGI_TRY(part_check_slots(g, pv, n, used, false));
    if (n == 0) return FGI_OK;
    hipSetDevice(g->device);
    hipStream_t st = g->stream;
    uint64_t hcap = 64;
    while (hcap < 2ull * n) hcap <<= 1;
    Tmp tdep, tuse, tflag, tres, thash, tcand, tpend, tovf, tik, tit;
    uint32_t *ddep, *duse, *dflag, *dres, *dpend, *dovf;
    unsigned long long* dhash;
    Cand* dcand;
    uint64_t *ik, *it;
    FGI_TRY(tmalloc(g, tdep, &ddep, n));
    FGI_TRY(tmalloc(g, tuse, &duse, n));
    FGI_TRY(tmalloc(g, tflag, &dflag, n));
    FGI_TRY(tmalloc(g, tres, &dres, n));
    FGI_TRY(tmalloc(g, thash, &dhash, hcap));
    FGI_TRY(tmalloc(g, tcand, &dcand, n));
    FGI_TRY(tmalloc(g, tpend, &dpend, n));
    FGI_TRY(tmalloc(g, tovf, &dovf, n));
    FGI_TRY(tmalloc(g, tik, &ik, n));
    FGI_TRY(tmalloc(g, tit, &it, n));
    FGI_TRY(h2d(g, ddep, dep, n));
    FGI_TRY(h2d(g, duse, used, n));
    FGI_TRY(fold(g));
    note_words(g);
    auto* node = reinterpret_cast<unsigned long long*>(g->node);
    hipLaunchKernelGGL(k_pau_dep, dim3(nblk(n)), dim3(256), 0, st, n, ddep, pv.base, pv.n_local, node, g->used_cnt, dflag);
    FGI_TRY(part_allreduce_u32(g, dflag, n));
    FGI_HIP(g, hipMemsetAsync(dhash, 0xFF, hcap * sizeof(unsigned long long), st));
    FGI_HIP(g, hipMemsetAsync(g->misc_dev, 0, 8 * sizeof(unsigned long long), st));
    const PauArgs pa{ddep, duse, pv.base, pv.n_local, node, pv.ver_all, dflag, g->row_off, g->row_len, g->pool_col,
                     g->pool_tag, dhash, hcap - 1, dres, dcand, g->misc_dev};
    hipLaunchKernelGGL(k_pau_classify, dim3(nblk(n)), dim3(256), 0, st, n, pa);
    unsigned long long nc = 0;
    FGI_TRY(d2h(g, &nc, g->misc_dev, 1));
    if (nc) {
        touch(g);
        const AuArgs aa{nullptr,     nullptr,    g->n_slots,  g->home,     node,        g->row_off,
                        g->row_len,  g->row_cap, nullptr,     g->pool_col, g->pool_tag, dhash,
                        hcap - 1,    nullptr,    dcand,       dpend,       dovf,        g->misc_dev};
        hipLaunchKernelGGL(k_au_reserve, dim3(nblk(nc)), dim3(256), 0, st, (uint64_t)nc, aa);
        unsigned long long c2[2];
        FGI_TRY(d2h(g, c2, g->misc_dev + 1, 2));
        if (c2[1]) {   // rows that outgrew their capacity: relocated to the pool top
            hipLaunchKernelGGL(k_au_size, dim3(nblk(c2[1])), dim3(256), 0, st, (uint64_t)c2[1], dovf, g->row_len,
                               g->misc_dev + 3);
            unsigned long long need = 0;
            FGI_TRY(d2h(g, &need, g->misc_dev + 3, 1));
            FGI_TRY(ensure_pool(g, g->pool_top + need));
            FGI_HIP(g, hipMemcpyAsync(g->pool_top_dev, &g->pool_top, sizeof(uint64_t), hipMemcpyHostToDevice, st));
            hipLaunchKernelGGL(k_au_relocate, dim3(nblk(c2[1] * 64)), dim3(256), 0, st, (uint64_t)c2[1], dovf,
                               g->row_off, g->row_len, g->row_cap, g->pool_col, g->pool_tag, g->pool_top_dev);
            hipLaunchKernelGGL(k_au_pending, dim3(nblk(nc)), dim3(256), 0, st, (uint64_t)nc, dcand, dpend, g->row_off,
                               g->pool_col, g->pool_tag);
            g->pool_top += need;
            FGI_TRY(ensure_cstart(g, g->pool_top));
        }
    }
    FGI_TRY(part_allreduce_u32(g, dres, n));
    FGI_HIP(g, hipMemsetAsync(g->misc_dev + 5, 0, sizeof(unsigned long long), st));
    hipLaunchKernelGGL(k_pau_apply, dim3(nblk(n)), dim3(256), 0, st, n, ddep, duse, pv.base, pv.n_local, dres, node,
                       g->used_cnt, pv.ver_all, ik, it, g->misc_dev + 5);
    FGI_HIP(g, hipGetLastError());
    unsigned long long ni = 0;
    FGI_TRY(d2h(g, &ni, g->misc_dev + 5, 1));
    if (ni) {
        FGI_TRY(part_store_in_dev(g, ik, it, ni));
        touch(g);
    }
    std::vector<uint32_t> r(n);
    FGI_TRY(d2h(g, r.data(), dres, n));
    if (out_result)
        for (uint32_t i = 0; i < n; ++i) out_result[i] = (r[i] & 0xFFu) - 1u;
    return FGI_OK;
}

// Computed.TrySetOutput (Computed.cs:141-160) over a partition; the nodes flagged
// InvalidateOnSetOutput are the roots of one cascade on every rank. out_set: every item, every rank
fgi_status part_set_output(fgi_graph* g, uint32_t n, const uint32_t* slot, uint8_t* out_set, fgi_wave_stats* stats,
                           std::vector<uint32_t>* ids) {
    PartView pv;
    FGI_TRY(part_check(g, &pv, "fgi_part_set_output"));
    if (n && !slot) return FGI_EINVAL;
    FGI_TRY(part_check_slots(g, pv, n, slot, false));
    hipSetDevice(g->device);
    hipStream_t st = g->stream;
    std::vector<uint32_t> li, lh;
    for (uint32_t i = 0; i < n; ++i)
        if (slot[i] - pv.base < pv.n_local) {
            li.push_back(i);
            lh.push_back(slot[i] - pv.base);
        }
    const uint32_t m = (uint32_t)li.size();
    Tmp th, ts, tr, tfl;
    uint32_t *dh = nullptr, *droots = nullptr, *dfl = nullptr;
    uint8_t* dset = nullptr;
    FGI_TRY(fold(g));
    note_words(g);
    FGI_HIP(g, hipMemsetAsync(g->misc_dev, 0, sizeof(unsigned long long), st));
    std::vector<uint8_t> set(m, 0);
    if (m) {
        FGI_TRY(tmalloc(g, th, &dh, m));
        FGI_TRY(tmalloc(g, ts, &dset, m));
        FGI_TRY(tmalloc(g, tr, &droots, m));
        FGI_TRY(h2d(g, dh, lh.data(), m));
        hipLaunchKernelGGL(k_set_output, dim3(nblk(m)), dim3(256), 0, st, m, dh, g->n_handles,
                           reinterpret_cast<unsigned long long*>(g->node), dset, droots, g->misc_dev);
        FGI_TRY(d2h(g, set.data(), dset, m));
    }
    unsigned long long nr = 0;
    FGI_TRY(d2h(g, &nr, g->misc_dev, 1));
    if (nr) hipLaunchKernelGGL(k_add_base, dim3(nblk(nr)), dim3(256), 0, st, (uint32_t)nr, droots, pv.base);
    g->last_wave_n = 0;
    FGI_TRY(run_part_wave(g, (uint32_t)nr, droots, nullptr, stats));   // Invalidate() (Computed.cs:153-156)
    FGI_TRY(part_take_ids(g, pv, ids));
    if (n) {
        std::vector<uint32_t> all(n, 0);
        for (uint32_t j = 0; j < m; ++j) all[li[j]] = set[j];
        FGI_TRY(tmalloc(g, tfl, &dfl, n));
        FGI_TRY(h2d(g, dfl, all.data(), n));
        FGI_TRY(part_allreduce_u32(g, dfl, n));
        FGI_TRY(d2h(g, all.data(), dfl, n));
        if (out_set)
            for (uint32_t i = 0; i < n; ++i) out_set[i] = (uint8_t)(all[i] != 0);
    }
    return FGI_OK;
}

// ComputedRegistry.InvalidateEverything (ComputedRegistry.cs:142-147) over a partition: every rank's
// current nodes are the roots of one cascade
fgi_status part_invalidate_all(fgi_graph* g, fgi_wave_stats* stats, std::vector<uint32_t>* ids) {
    PartView pv;
    FGI_TRY(part_check(g, &pv, "fgi_part_invalidate_all"));
    hipSetDevice(g->device);
    hipStream_t st = g->stream;
    FGI_TRY(fold(g));
    Tmp tr;
    uint32_t* roots;
    FGI_TRY(tmalloc(g, tr, &roots, std::max<uint32_t>(pv.n_local, 1)));
    FGI_HIP(g, hipMemsetAsync(g->misc_dev, 0, sizeof(unsigned long long), st));
    hipLaunchKernelGGL(k_invalidate_all_roots, dim3(nblk(pv.n_local)), dim3(256), 0, st, pv.n_local,
                       reinterpret_cast<const unsigned long long*>(g->node), roots, g->misc_dev);
    unsigned long long nr = 0;
    FGI_TRY(d2h(g, &nr, g->misc_dev, 1));
    if (nr) hipLaunchKernelGGL(k_add_base, dim3(nblk(nr)), dim3(256), 0, st, (uint32_t)nr, roots, pv.base);
    g->last_wave_n = 0;
    FGI_TRY(run_part_wave(g, (uint32_t)nr, roots, nullptr, stats));
    return part_take_ids(g, pv, ids);
}

fgi_status part_copy_ids(fgi_graph* g, const std::vector<uint32_t>& ids, uint32_t* out_ids, uint64_t cap, uint64_t* out_n) {
    if (out_n) *out_n = ids.size();
    if (!out_ids) return FGI_OK;
    if (ids.size() > cap) return FGI_ECAPACITY;
    std::memcpy(out_ids, ids.data(), ids.size() * 4);
    (void)g;
    return FGI_OK;
}

}  // namespace

fgi_status fgi_part_begin_compute(fgi_graph* g, uint32_t n, const uint32_t* slot, const uint64_t* version,
                                  const uint8_t* has_delay, uint32_t* out_detached, uint32_t* out_ids, uint64_t cap,
                                  uint64_t* out_n, fgi_wave_stats* stats) {
    if (!g) return FGI_EINVAL;
    std::vector<uint32_t> ids, ms;
    slot = part_codes_in(g, n, slot, ms);   // partition codes; outputs are slots again
    FGI_TRY(part_begin_compute(g, n, slot, version, has_delay, out_detached, stats, &ids));
    return part_copy_ids(g, ids, out_ids, cap, out_n);
}

fgi_status fgi_part_add_used(fgi_graph* g, uint32_t n, const uint32_t* dependant, const uint32_t* used,
                             uint32_t* out_result) {
    if (!g) return FGI_EINVAL;
    std::vector<uint32_t> md, mu;
    return part_add_used(g, n, part_codes_in(g, n, dependant, md), part_codes_in(g, n, used, mu), out_result);
}

fgi_status fgi_part_set_output(fgi_graph* g, uint32_t n, const uint32_t* slot, uint8_t* out_set, uint32_t* out_ids,
                               uint64_t cap, uint64_t* out_n, fgi_wave_stats* stats) {
    if (!g) return FGI_EINVAL;
    std::vector<uint32_t> ids, ms;
    slot = part_codes_in(g, n, slot, ms);
    FGI_TRY(part_set_output(g, n, slot, out_set, stats, &ids));
    return part_copy_ids(g, ids, out_ids, cap, out_n);
}

fgi_status fgi_part_invalidate_all(fgi_graph* g, uint32_t* out_ids, uint64_t cap, uint64_t* out_n,
                                   fgi_wave_stats* stats) {
    if (!g) return FGI_EINVAL;
    std::vector<uint32_t> ids;
    FGI_TRY(part_invalidate_all(g, stats, &ids));
    return part_copy_ids(g, ids, out_ids, cap, out_n);
}

fgi_status fgi_part_prune(fgi_graph* g, fgi_prune_stats* stats) {
    PartView pv;
    if (!g) return FGI_EINVAL;
    FGI_TRY(part_check(g, &pv, "fgi_part_prune"));
    if (stats) *stats = fgi_prune_stats{};
    return prune_rows(g, 0, g->n_handles, true, stats, true);
}

fgi_status fgi_part_run_batch(fgi_graph* g, uint32_t n_steps, const fgi_step* steps, uint32_t* out_ids, uint64_t cap,
                              uint64_t* out_n, fgi_batch_stats* stats) {
    PartView pv;
    if (!g || (n_steps && !steps)) return FGI_EINVAL;
    FGI_TRY(part_check(g, &pv, "fgi_part_run_batch"));
    const auto t0 = std::chrono::steady_clock::now();
    if (out_n) *out_n = 0;
    // a bad argument in any step applies nothing (every rank sees the same batch and refuses it alike)
    for (uint32_t k = 0; k < n_steps; ++k) {
        const fgi_step& sp = steps[k];
        if (sp.kind < FGI_STEP_INVALIDATE || sp.kind > FGI_STEP_SET_OUTPUT)
            return set_err(g, FGI_EINVAL, "step %u: unknown kind %u", k, sp.kind);
        if (sp.n && (!sp.handles || (sp.kind == FGI_STEP_ADD_USED && !sp.used) ||
                     (sp.kind == FGI_STEP_BEGIN_COMPUTE && !sp.version)))
            return set_err(g, FGI_EINVAL, "step %u: missing arrays", k);
        FGI_TRY(part_check_slots(g, pv, sp.n, sp.handles, sp.kind == FGI_STEP_BEGIN_COMPUTE));
        if (sp.kind == FGI_STEP_ADD_USED) FGI_TRY(part_check_slots(g, pv, sp.n, sp.used, false));
        if (sp.kind == FGI_STEP_BEGIN_COMPUTE)
            for (uint32_t i = 0; i < sp.n; ++i)
                if (sp.version[i] == 0 || sp.version[i] > kVMask)
                    return set_err(g, FGI_EINVAL, "step %u: bad version (%u)", k, i);
    }
    std::vector<uint32_t> ids;
    fgi_wave_stats ws{};
    for (uint32_t k = 0; k < n_steps; ++k) {
        fgi_step sp = steps[k];   // its slots as codes (partition codes)
        std::vector<uint32_t> mh, mu;
        sp.handles = part_codes_in(g, sp.n, sp.handles, mh);
        if (sp.kind == FGI_STEP_ADD_USED) sp.used = part_codes_in(g, sp.n, sp.used, mu);
        if (sp.n && !sp.handles) return set_err(g, FGI_EINVAL, "step %u: no handles", k);
        const uint64_t before = ws.v_inv;
        switch (sp.kind) {
            case FGI_STEP_INVALIDATE: {
                FGI_TRY(part_check_slots(g, pv, sp.n, sp.handles, false));
                FGI_TRY(part_wave_host(g, pv, sp.n, sp.handles, sp.flags, &ws, &ids));
                break;
            }
            case FGI_STEP_BEGIN_COMPUTE:
                FGI_TRY(part_begin_compute(g, sp.n, sp.handles, sp.version, sp.flags, static_cast<uint32_t*>(sp.out), &ws,
                                           &ids));
                break;
            case FGI_STEP_ADD_USED:
                FGI_TRY(part_add_used(g, sp.n, sp.handles, sp.used, static_cast<uint32_t*>(sp.out)));
                break;
            case FGI_STEP_SET_OUTPUT:
                FGI_TRY(part_set_output(g, sp.n, sp.handles, static_cast<uint8_t*>(sp.out), &ws, &ids));
                break;
            default:
                return set_err(g, FGI_EINVAL, "step %u: unknown kind %u", k, sp.kind);
        }
        if (stats && sp.kind != FGI_STEP_ADD_USED) stats->waves += 1;
        (void)before;
    }
    if (stats) {
        stats->levels += ws.levels;
        stats->v_inv += ws.v_inv;
        stats->e_trav += ws.e_trav;
        stats->e_match += ws.e_match;
        stats->n_flagged += ws.n_flagged;
        stats->kernel_ms += ws.kernel_ms;
        stats->wave_ms += ws.kernel_ms;
        stats->host_syncs += (uint32_t)ws.host_syncs;
        stats->total_ms += std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    }
    return part_copy_ids(g, ids, out_ids, cap, out_n);
}

}  // extern "C"
