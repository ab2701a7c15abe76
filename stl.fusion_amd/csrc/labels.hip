// labels.hip — hub-first internal labels.
//
// A pull level probes, for every live candidate, the invalidated bits of the heads of its dependency
// list (the reference's `_used`, Computed.cs:36, restricted to entries whose `_usedBy` tag matches:
// Computed.cs:212-216). Heads are the candidate's heaviest parents, so the probes concentrate on the
// slots that many nodes depend on. With slots numbered as the host numbers its ComputedInputs, those
// hubs are scattered over the whole bitmap: at configs[2] (R-MAT 27) the 16 MB invalidated bitmap
// misses every XCD's 4 MB L2 (level 1 fetches 2.46 GB, profiles/r8f_pmc_levels_rmat27.txt).
//
// So the engine numbers its nodes itself. At a graph's first bulk edge load it weighs every slot by
// its dependency count (|_used|, the same weight that orders the lists), sorts the slots by (weight
// class, slot) — eight classes per octave of weight + 1 — and gives the heaviest ones, at most an
// eighth of the slots, the labels [0, lbl_hot): the hubs' bits, node words and rows sit in a compact
// prefix (2 MB of bitmap at R-MAT 27). Every other slot or detached handle x keeps label K + x (K =
// the prefix capacity), so the boundary's handles map to labels with one table lookup and back with
// one subtraction or table read, and the bitmap over boundary handles is the labels' bitmap shifted
// by K words, ORed with the hot labels' bits at their slots (the fold, wave.hip). Within a class the
// hot labels keep slot order, so the hot labels of a range of slots form one run per class
// (fold_start), and the fold reads them in order.
//
// Measured on the generator's graphs before building this (profiles/r10_relabel_experiments.txt,
// same wave, relabelled keys): configs[2] 1.18 -> 0.96-0.97 ms/step with every slot in weight order,
// the same with (class, slot) order at 4-8 classes per octave; a weight-ordered prefix of 1/8 of the
// slots takes most of it (0.97). configs[1] (whose 2 MB bitmap already fits L2) gains nothing, so
// labels are automatic only from 2^25 slots on.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <vector>

#include <rocprim/device/device_radix_sort.hpp>

#include "fgi_internal.h"

namespace fgi {
namespace {

inline uint32_t nblk(uint64_t n, uint32_t b = 256) { return (uint32_t)((n + b - 1) / b); }

// weight class of a slot with w dependencies: kClassPerOctave classes per octave of w + 1
__device__ __forceinline__ uint32_t weight_class(uint32_t w) {
    const uint32_t x = w + 1u;   // w < 2^32 - 1 (a slot has fewer dependencies than the pool has entries)
    const uint32_t l = 31u - (uint32_t)__builtin_clz(x);
    const uint32_t frac = l >= 3 ? (x >> (l - 3)) & 7u : (x << (3 - l)) & 7u;   // the 3 bits after the leading one
    return l * kClassPerOctave + frac;
}

__device__ __forceinline__ uint32_t map_in(uint32_t x, uint32_t ext_slots, const uint32_t* __restrict__ s2l, uint32_t K) {
    if (x == FGI_NONE) return x;
    if (s2l && x < ext_slots) {
        const uint32_t l = s2l[x];
        if (l != FGI_NONE) return l;
    }
    return x + K;
}
__device__ __forceinline__ uint32_t map_out(uint32_t l, const uint32_t* __restrict__ l2s, uint32_t K) {
    if (l == FGI_NONE) return l;
    return l < K ? l2s[l] : l - K;
}

__global__ void k_lbl_map_in(uint64_t n, uint32_t* a, uint32_t ext_slots, const uint32_t* __restrict__ s2l, uint32_t K) {
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x)
        a[i] = map_in(a[i], ext_slots, s2l, K);
}
__global__ void k_lbl_map_out(uint64_t n, uint32_t* a, const uint32_t* __restrict__ l2s, uint32_t K) {
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x)
        a[i] = map_out(a[i], l2s, K);
}
__global__ void k_lbl_map_keys(uint64_t m, uint64_t* keys, uint32_t ext_slots, const uint32_t* __restrict__ s2l,
                               uint32_t K, int out, const uint32_t* __restrict__ l2s) {
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < m; i += (uint64_t)gridDim.x * blockDim.x) {
        const uint64_t k = keys[i];
        const uint32_t u = (uint32_t)(k >> 32), d = (uint32_t)k;
        const uint32_t u2 = out ? map_out(u, l2s, K) : map_in(u, ext_slots, s2l, K);
        const uint32_t d2 = out ? map_out(d, l2s, K) : map_in(d, ext_slots, s2l, K);
        keys[i] = ((uint64_t)u2 << 32) | d2;
    }
}

// dependency counts of the boundary's slots from edge keys (used << 32 | dependant)
__global__ void k_lbl_weights(uint64_t m, const uint64_t* __restrict__ keys, uint32_t ext_slots, uint32_t* cnt) {
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < m; i += (uint64_t)gridDim.x * blockDim.x) {
        const uint32_t d = (uint32_t)keys[i];
        if (d < ext_slots) atomicAdd(cnt + d, 1u);
    }
}

// sort key: class descending, then slot ascending (sorted descending: ~slot); the class histogram
__global__ void k_lbl_keys(uint32_t n, const uint32_t* __restrict__ cnt, uint64_t* key, uint32_t* hist) {
    const uint32_t s = blockIdx.x * blockDim.x + threadIdx.x;
    if (s >= n) return;
    const uint32_t c = weight_class(cnt[s]);
    key[s] = ((uint64_t)c << 32) | (uint32_t)~s;
    atomicAdd(hist + c, 1u);
}

// the hot labels: rank r < H of the sorted order -> its slot
__global__ void k_lbl_assign(uint32_t H, const uint64_t* __restrict__ sorted, uint32_t* s2l, uint32_t* l2s) {
    const uint32_t r = blockIdx.x * blockDim.x + threadIdx.x;
    if (r >= H) return;
    const uint32_t s = ~(uint32_t)sorted[r];
    l2s[r] = s;
    s2l[s] = r;
}

// fold_start[t][j] (tile-major: a fold tile reads its row and the next, two contiguous runs): the first
// hot label of hot class j (labels [cb[j], cb[j + 1]), slots ascending) whose slot is >= t * kFoldTile;
// t = tiles gives the class's end
__global__ void k_lbl_fold_start(uint32_t ncls, uint32_t tiles, const uint32_t* __restrict__ cb,
                                 const uint32_t* __restrict__ l2s, uint32_t* fs) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= (uint64_t)ncls * (tiles + 1)) return;
    const uint32_t t = (uint32_t)(i / ncls), j = (uint32_t)(i % ncls);
    uint32_t lo = cb[j], hi = cb[j + 1];
    const uint64_t x = (uint64_t)t * kFoldTile;
    while (lo < hi) {
        const uint32_t mid = lo + (hi - lo) / 2;
        if ((uint64_t)l2s[mid] < x) lo = mid + 1;
        else hi = mid;
    }
    fs[i] = lo;
}

// each fold tile's hot-label count (its runs over the classes)
__global__ void k_lbl_tile_tot(uint32_t ncls, uint32_t tiles, const uint32_t* __restrict__ fs, uint32_t* tot) {
    const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= tiles) return;
    uint32_t c = 0;
    for (uint32_t j = 0; j < ncls; ++j) c += fs[(uint64_t)(t + 1) * ncls + j] - fs[(uint64_t)t * ncls + j];
    tot[t] = c;
}

// fold_off: block t lists its tile's hot labels in the fold's order (class by class, each class's run in
// slot order) as their slots' offsets in the tile, at base[t]: the fold then reads one contiguous run
// of 2-byte offsets per tile instead of a label-map entry per hot label (a cache line per class run)
__global__ __launch_bounds__(256) void k_lbl_fold_off(uint32_t ncls, const uint32_t* __restrict__ fs,
                                                      const uint32_t* __restrict__ base, const uint32_t* __restrict__ l2s,
                                                      uint16_t* off) {
    __shared__ uint32_t s_a[kMaxHotClasses + 1], s_o[kMaxHotClasses + 1];
    const uint32_t t = blockIdx.x;
    if (threadIdx.x == 0) {
        uint32_t o = 0;
        for (uint32_t j = 0; j < ncls; ++j) {
            const uint32_t a = fs[(uint64_t)t * ncls + j];
            s_a[j] = a;
            s_o[j] = o;
            o += fs[(uint64_t)(t + 1) * ncls + j] - a;
        }
        s_o[ncls] = o;
    }
    __syncthreads();
    const uint32_t total = s_o[ncls], b = base[t];
    const uint64_t tile0 = (uint64_t)t * kFoldTile;
    for (uint32_t k = threadIdx.x; k < total; k += blockDim.x) {
        uint32_t lo = 0, hi = ncls;   // the last class j with s_o[j] <= k
        while (hi - lo > 1) {
            const uint32_t mid = (lo + hi) >> 1;
            if (s_o[mid] <= k) lo = mid;
            else hi = mid;
        }
        off[b + k] = (uint16_t)(l2s[s_a[lo] + (k - s_o[lo])] - tile0);
    }
}

// the registered node words of hot slots move from their cold label K + s to their hot label; a
// detached node's home slot follows its slot
__global__ void k_lbl_move_words(uint32_t H, const uint32_t* __restrict__ l2s, uint32_t K, unsigned long long* node) {
    const uint32_t r = blockIdx.x * blockDim.x + threadIdx.x;
    if (r >= H) return;
    const uint32_t s = l2s[r];
    node[r] = node[K + s];
    node[K + s] = 0ull;
}
__global__ void k_lbl_home(uint32_t n, uint32_t* home, uint32_t ext_slots, const uint32_t* __restrict__ s2l, uint32_t K) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const uint32_t h = home[i];   // a slot's label (K + slot before labels are chosen)
    if (h != FGI_NONE && h >= K && h - K < ext_slots) home[i] = map_in(h - K, ext_slots, s2l, K);
}

}  // namespace

uint32_t labels_capacity(uint32_t n_slots, int opt) {
    static const int env = [] {
        const char* e = getenv("FGI_LABELS");   // tests / measurement: 1 always, -1 never
        return e && *e ? atoi(e) : 0;
    }();
    if (env) opt = env;
    if (opt < 0 || n_slots == 0) return 0;
    if (opt == 0 && n_slots < kLabelAutoSlots) return 0;
    const uint64_t want = std::max<uint64_t>(1, n_slots / 8);
    return (uint32_t)((want + kFoldTile - 1) / kFoldTile * kFoldTile);
}

fgi_status labels_map_in(fgi_graph* g, uint32_t* dev, uint64_t n) {
    if (g->lbl_perm) return part_codes_local(g, dev, n, false);
    if (!g->lbl_K || n == 0) return FGI_OK;
    hipLaunchKernelGGL(k_lbl_map_in, dim3(std::min<uint32_t>(nblk(n), 8192)), dim3(256), 0, g->stream, n, dev, g->ext_slots,
                       g->lbl_hot ? g->s2l : nullptr, g->lbl_K);
    FGI_HIP(g, hipGetLastError());
    return FGI_OK;
}

fgi_status labels_map_out(fgi_graph* g, uint32_t* dev, uint64_t n) {
    if (g->lbl_perm) return part_codes_local(g, dev, n, true);
    if (!g->lbl_K || n == 0) return FGI_OK;
    hipLaunchKernelGGL(k_lbl_map_out, dim3(std::min<uint32_t>(nblk(n), 8192)), dim3(256), 0, g->stream, n, dev, g->l2s,
                       g->lbl_K);
    FGI_HIP(g, hipGetLastError());
    return FGI_OK;
}

fgi_status labels_map_keys(fgi_graph* g, uint64_t* keys, uint64_t m) {
    if (!g->lbl_K || m == 0) return FGI_OK;
    hipLaunchKernelGGL(k_lbl_map_keys, dim3(std::min<uint32_t>(nblk(m), 16384)), dim3(256), 0, g->stream, m, keys,
                       g->ext_slots, g->lbl_hot ? g->s2l : nullptr, g->lbl_K, 0, g->l2s);
    FGI_HIP(g, hipGetLastError());
    return FGI_OK;
}

fgi_status labels_unmap_keys(fgi_graph* g, uint64_t* keys, uint64_t m) {
    if (!g->lbl_K || m == 0) return FGI_OK;
    hipLaunchKernelGGL(k_lbl_map_keys, dim3(std::min<uint32_t>(nblk(m), 16384)), dim3(256), 0, g->stream, m, keys,
                       g->ext_slots, g->s2l, g->lbl_K, 1, g->l2s);
    FGI_HIP(g, hipGetLastError());
    return FGI_OK;
}

fgi_status labels_choose(fgi_graph* g, const uint64_t* keys, uint64_t m) {
    if (!g->lbl_K || g->lbl_done || g->part) return FGI_OK;
    hipStream_t s = g->stream;
    const uint32_t n = g->ext_slots;
    FGI_TRY(fold(g));   // node words are moved below: no visit may be pending
    uint32_t *cnt = nullptr, *hist = nullptr, *cb = nullptr;
    uint64_t *k0 = nullptr, *k1 = nullptr;
    void* tmp = nullptr;
    auto cleanup = [&]() {
        for (void* p : {(void*)cnt, (void*)hist, (void*)cb, (void*)k0, (void*)k1, tmp})
            if (p) hipFree(p);
    };
    // a failure leaves no hot set (lbl_hot stays 0, lbl_done false) and no half-built fold tables: a retry
    // starts from the same state
    auto fail = [&](hipError_t e, const char* what) {
        cleanup();
        for (void** p : {(void**)&g->fold_start, (void**)&g->fold_off, (void**)&g->fold_base}) {
            if (*p) hipFree(*p);
            *p = nullptr;
        }
        return hip_check(g, e, what);
    };
    hipError_t e;
    if ((e = hipMalloc(&cnt, (size_t)n * 4)) != hipSuccess) return fail(e, "labels: weights");
    if ((e = hipMalloc(&hist, kLabelClasses * 4)) != hipSuccess) return fail(e, "labels: histogram");
    if ((e = hipMalloc(&k0, (size_t)n * 8)) != hipSuccess) return fail(e, "labels: keys");
    if ((e = hipMalloc(&k1, (size_t)n * 8)) != hipSuccess) return fail(e, "labels: keys");
    (void)hipMemsetAsync(cnt, 0, (size_t)n * 4, s);
    (void)hipMemsetAsync(hist, 0, kLabelClasses * 4, s);
    if (m) hipLaunchKernelGGL(k_lbl_weights, dim3(std::min<uint32_t>(nblk(m), 16384)), dim3(256), 0, s, m, keys, n, cnt);
    hipLaunchKernelGGL(k_lbl_keys, dim3(nblk(n)), dim3(256), 0, s, n, cnt, k0, hist);
    size_t tb = 0;
    if ((e = rocprim::radix_sort_keys_desc(nullptr, tb, k0, k1, (size_t)n, 0, 64, s)) != hipSuccess) return fail(e, "labels: sort");
    if ((e = hipMalloc(&tmp, tb)) != hipSuccess) return fail(e, "labels: sort");
    if ((e = rocprim::radix_sort_keys_desc(tmp, tb, k0, k1, (size_t)n, 0, 64, s)) != hipSuccess) return fail(e, "labels: sort");
    std::vector<uint32_t> h(kLabelClasses);
    if ((e = hipMemcpyAsync(h.data(), hist, kLabelClasses * 4, hipMemcpyDeviceToHost, s)) != hipSuccess ||
        (e = hipStreamSynchronize(s)) != hipSuccess)
        return fail(e, "labels: histogram");
    // the hot set: whole classes from the heaviest down, at most an eighth of the slots (and the
    // prefix capacity), at most kMaxHotClasses classes; weightless slots stay cold
    const uint64_t cap = std::min<uint64_t>(g->lbl_K, std::max<uint64_t>(1, n / 8));
    uint64_t H = 0;
    std::vector<uint32_t> bases;   // class bases of the hot classes, heaviest first
    for (int c = (int)kLabelClasses - 1; c > 0 && bases.size() < kMaxHotClasses; --c) {
        if (!h[c]) continue;
        if (H + h[c] > cap) break;
        bases.push_back((uint32_t)H);
        H += h[c];
    }
    const uint32_t ncls = (uint32_t)bases.size();
    bases.push_back((uint32_t)H);
    const uint32_t tiles = (uint32_t)(((uint64_t)g->ext_handles + kFoldTile - 1) / kFoldTile);
    // each map on its own: a retry after a failed allocation finds the one that exists and makes the other
    if (!g->s2l && (e = hipMalloc(&g->s2l, (size_t)n * 4)) != hipSuccess) {
        g->s2l = nullptr;
        return fail(e, "labels: slot map");
    }
    if (!g->l2s && (e = hipMalloc(&g->l2s, (size_t)g->lbl_K * 4)) != hipSuccess) {
        g->l2s = nullptr;
        return fail(e, "labels: label map");
    }
    (void)hipMemsetAsync(g->s2l, 0xFF, (size_t)n * 4, s);
    (void)hipMemsetAsync(g->l2s, 0xFF, (size_t)g->lbl_K * 4, s);
    if (H) {
        hipLaunchKernelGGL(k_lbl_assign, dim3(nblk(H)), dim3(256), 0, s, (uint32_t)H, k1, g->s2l, g->l2s);
        if (g->fold_start) hipFree(g->fold_start);
        g->fold_start = nullptr;
        if ((e = hipMalloc(&g->fold_start, (size_t)ncls * (tiles + 1) * 4)) != hipSuccess) return fail(e, "labels: fold table");
        if ((e = hipMalloc(&cb, bases.size() * 4)) != hipSuccess) return fail(e, "labels: class bases");
        if ((e = hipMemcpyAsync(cb, bases.data(), bases.size() * 4, hipMemcpyHostToDevice, s)) != hipSuccess)
            return fail(e, "labels: class bases");
        hipLaunchKernelGGL(k_lbl_fold_start, dim3(nblk((uint64_t)ncls * (tiles + 1))), dim3(256), 0, s, ncls, tiles, cb,
                           g->l2s, g->fold_start);
        // the fold's per-tile offset runs: tile counts, their prefix (host: tiles words), the offsets
        for (void* p : {(void*)g->fold_off, (void*)g->fold_base})
            if (p) hipFree(p);
        g->fold_off = nullptr;
        g->fold_base = nullptr;
        if ((e = hipMalloc(&g->fold_off, ((size_t)H + 8ull * tiles + 8) * 2)) != hipSuccess ||
            (e = hipMalloc(&g->fold_base, (size_t)(tiles + 1) * 4)) != hipSuccess)
            return fail(e, "labels: fold offsets");
        hipLaunchKernelGGL(k_lbl_tile_tot, dim3(nblk(tiles)), dim3(256), 0, s, ncls, tiles, g->fold_start, g->fold_base);
        std::vector<uint32_t> tb_host(tiles + 1, 0);
        if ((e = hipMemcpyAsync(tb_host.data(), g->fold_base, (size_t)tiles * 4, hipMemcpyDeviceToHost, s)) != hipSuccess ||
            (e = hipStreamSynchronize(s)) != hipSuccess)
            return fail(e, "labels: fold tile counts");
        // each tile's run starts 16-byte aligned (8 entries): the fold stages it with 16-byte loads
        uint64_t run = 0, covered = 0;
        for (uint32_t t = 0; t <= tiles; ++t) {
            const uint32_t c = t < tiles ? tb_host[t] : 0u;
            tb_host[t] = (uint32_t)run;
            run += (c + 7u) & ~7u;
            covered += c;
        }
        if (covered != H) {
            cleanup();
            return set_err(g, FGI_EDEVICE, "labels: fold runs cover %llu of %llu hot labels", (unsigned long long)covered,
                           (unsigned long long)H);
        }
        if (run > (1ull << 32)) {
            cleanup();
            return set_err(g, FGI_ENOTSUP, "labels: fold offsets exceed 2^32 entries");
        }
        if ((e = hipMemcpyAsync(g->fold_base, tb_host.data(), (size_t)(tiles + 1) * 4, hipMemcpyHostToDevice, s)) != hipSuccess)
            return fail(e, "labels: fold bases");
        hipLaunchKernelGGL(k_lbl_fold_off, dim3(tiles), dim3(256), 0, s, ncls, g->fold_start, g->fold_base, g->l2s,
                           g->fold_off);
        hipLaunchKernelGGL(k_lbl_move_words, dim3(nblk(H)), dim3(256), 0, s, (uint32_t)H, g->l2s, g->lbl_K,
                           reinterpret_cast<unsigned long long*>(g->node));
        if (g->n_detached)
            hipLaunchKernelGGL(k_lbl_home, dim3(nblk(g->n_detached)), dim3(256), 0, s, g->n_detached, g->home, n, g->s2l,
                               g->lbl_K);
    }
    if ((e = hipGetLastError()) != hipSuccess || (e = hipStreamSynchronize(s)) != hipSuccess) return fail(e, "labels");
    cleanup();
    g->lbl_hot = (uint32_t)H;
    g->lbl_ncls = ncls;
    g->fold_tiles = tiles;
    g->lbl_done = true;
    touch(g);
    note_words(g);
    if (getenv("FGI_TRACE"))
        fprintf(stderr, "[fgi] labels: %llu hot slots of %u in %u classes (capacity %u)\n", (unsigned long long)H, n, ncls,
                g->lbl_K);
    return FGI_OK;
}

}  // namespace fgi
