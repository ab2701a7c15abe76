// synth.hip — device generators for the benchmark workloads.
// Same definitions as the CPU oracle's oracle/synth.cpp (checked equal in tests), written for the
// device so a 256M-edge graph is generated and turned into rows in HBM in well under a second.
#include <hip/hip_runtime.h>
#include <stdio.h>

#include <algorithm>

#include <rocprim/device/device_radix_sort.hpp>
#include <rocprim/device/device_scan.hpp>

#include "fgi_internal.h"

namespace fgi {
namespace {

// slot s's node at label K + s (labels.hip moves the hot ones when it chooses them)
__global__ void k_versions(uint32_t n, uint64_t seed, uint32_t K, unsigned long long* node) {
    const uint32_t s = blockIdx.x * blockDim.x + threadIdx.x;
    if (s < n) node[K + s] = synth_version(seed, s) | kW_Consistent;
}

// the generated edges' tags, from boundary slots (before the keys become labels)
__global__ void k_synth_tags(uint64_t m, const uint64_t* __restrict__ keys, uint64_t seed, uint32_t stale_pct,
                             uint64_t stale_seed, uint64_t* tags) {
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < m; i += (uint64_t)gridDim.x * blockDim.x) {
        const uint64_t k = keys[i];
        const uint32_t src = (uint32_t)(k >> 32), dst = (uint32_t)k;
        tags[i] = synth_version(seed, dst) + (synth_stale(stale_pct, stale_seed, src, dst) ? 1ull : 0ull);
    }
}

__global__ void k_gen_layered(uint32_t levels, uint32_t width, uint32_t fanout, uint64_t seed, uint64_t* keys) {
    const uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const uint64_t n = (uint64_t)(levels - 1) * width;
    if (t >= n) return;
    const uint32_t l = (uint32_t)(t / width) + 1, i = (uint32_t)(t % width);
    uint32_t chosen[64];
    uint32_t c = 0;
    for (uint64_t attempt = 0; c < fanout; ++attempt) {
        const uint64_t key = ((uint64_t)l << 56) ^ ((uint64_t)i << 20) ^ attempt;
        const uint32_t j = (uint32_t)(sm64(seed ^ sm64(key)) % width);
        bool dup = false;
        for (uint32_t q = 0; q < c; ++q) dup |= (chosen[q] == j);
        if (!dup) chosen[c++] = j;
    }
    const uint64_t d = (uint64_t)l * width + i;
    for (uint32_t k = 0; k < fanout; ++k) {
        const uint64_t s = (uint64_t)(l - 1) * width + chosen[k];
        keys[t * fanout + k] = (s << 32) | d;
    }
}

__global__ void k_gen_rmat(uint64_t m, uint32_t scale, uint64_t seed, uint64_t* keys) {
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < m; i += (uint64_t)gridDim.x * blockDim.x) {
        uint32_t s, d;
        rmat_edge(i, scale, seed, &s, &d);
        keys[i] = ((uint64_t)s << 32) | d;
    }
}

// ---- measurement experiment: R-MAT keys relabelled by degree (FGI_EXP_RELABEL) -------------------
__global__ void kx_deg(uint64_t m, const uint64_t* __restrict__ keys, uint32_t which, uint32_t* cnt) {
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < m; i += (uint64_t)gridDim.x * blockDim.x) {
        const uint64_t k = keys[i];
        if (which != 1) atomicAdd(cnt + (uint32_t)(k >> 32), 1u);
        if (which != 2) atomicAdd(cnt + (uint32_t)k, 1u);
    }
}
// weight classes: `per` classes per octave of (w + 1)
__device__ __forceinline__ uint32_t kx_class(uint32_t w, uint32_t per) {
    const uint32_t x = w + 1u;
    const uint32_t l = 31u - (uint32_t)__builtin_clz(x);
    const uint32_t frac = l ? ((x << (31u - l)) >> 28) & 7u : 0u;   // the 3 bits after the leading one
    return l * per + (per == 4 ? frac >> 1 : per == 2 ? frac >> 2 : per == 8 ? frac : 0u);
}
// order 3 / 4 / 5: (weight class, slot) with 4 / 1 / 8 classes per octave, else (weight, slot)
__global__ void kx_sortkey(uint32_t n, const uint32_t* __restrict__ cnt, uint32_t order, uint64_t* key) {
    const uint32_t u = blockIdx.x * blockDim.x + threadIdx.x;
    if (u >= n) return;
    const uint32_t w = order == 3 ? kx_class(cnt[u], 4) : order == 4 ? kx_class(cnt[u], 1) : order == 5 ? kx_class(cnt[u], 8) : cnt[u];
    key[u] = ((uint64_t)w << 32) | (uint32_t)~u;
}
// hot[u] = rank + 1 for the K heaviest, 0 otherwise
__global__ void kx_hot(uint32_t n, uint32_t K, const uint64_t* __restrict__ sorted, uint32_t* hot) {
    const uint32_t r = blockIdx.x * blockDim.x + threadIdx.x;
    if (r < K && r < n) hot[~(uint32_t)sorted[r]] = r + 1;
}
__global__ void kx_cold(uint32_t n, const uint32_t* __restrict__ hot, uint32_t* cold) {
    const uint32_t u = blockIdx.x * blockDim.x + threadIdx.x;
    if (u < n) cold[u] = hot[u] ? 0u : 1u;
}
// swizzle of a weight rank inside superblocks of 32,768 labels (32 lines x 32 words x 32 bits of a
// bitmap): consecutive ranks fall in different 128-byte lines, then different words, so the heaviest
// slots do not share a bitmap word or line (push levels' atomics), while the superblock stays compact
__device__ __forceinline__ uint32_t kx_swz(uint32_t r) {
    const uint32_t i = r & 32767u;
    return (r & ~32767u) | ((i & 31u) << 10) | (((i >> 5) & 31u) << 5) | (i >> 10);
}
__global__ void kx_perm(uint32_t n, uint32_t K, const uint32_t* __restrict__ hot, const uint32_t* __restrict__ cold_pos,
                        uint32_t slot_order, uint32_t* perm) {
    const uint32_t u = blockIdx.x * blockDim.x + threadIdx.x;
    // slot_order: the hot labels keep the slots' order among themselves (hot position = u - cold before u);
    // 2: weight order, swizzled within superblocks (K a multiple of 32,768)
    if (u < n)
        perm[u] = hot[u] ? (slot_order == 1 ? u - cold_pos[u] : slot_order == 2 ? kx_swz(hot[u] - 1) : hot[u] - 1)
                         : K + cold_pos[u];
}
__global__ void kx_apply(uint64_t m, const uint32_t* __restrict__ perm, uint64_t* keys) {
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < m; i += (uint64_t)gridDim.x * blockDim.x) {
        const uint64_t k = keys[i];
        keys[i] = ((uint64_t)perm[(uint32_t)(k >> 32)] << 32) | perm[(uint32_t)k];
    }
}

}  // namespace

// FGI_EXP_RELABEL=K (measurement only): the K heaviest slots (FGI_EXP_RELABEL_W: 0 total degree, 1 as
// dependant, 2 as used) take labels 0..K-1 by weight, the others keep their order after them; K < 0:
// every slot by weight. The graph is isomorphic to the unrelabelled one.
static fgi_status exp_relabel(fgi_graph* g, uint32_t n, uint64_t* keys, uint64_t m) {
    const char* e = getenv("FGI_EXP_RELABEL");
    if (!e || !*e) return FGI_OK;
    long long K = atoll(e);
    if (K == 0) return FGI_OK;
    if (K < 0 || K > n) K = n;
    const char* w = getenv("FGI_EXP_RELABEL_W");
    const uint32_t which = w ? (uint32_t)atoi(w) : 0u;
    const char* o = getenv("FGI_EXP_RELABEL_ORDER");
    const uint32_t slot_order = o ? (uint32_t)atoi(o) : 0u;
    hipStream_t s = g->stream;
    uint32_t *cnt, *hot, *cold, *pos, *perm;
    uint64_t *k0, *k1;
    FGI_HIP(g, hipMalloc(&cnt, (size_t)n * 4));
    FGI_HIP(g, hipMalloc(&hot, (size_t)n * 4));
    FGI_HIP(g, hipMalloc(&cold, (size_t)n * 4));
    FGI_HIP(g, hipMalloc(&pos, (size_t)n * 4));
    FGI_HIP(g, hipMalloc(&perm, (size_t)n * 4));
    FGI_HIP(g, hipMalloc(&k0, (size_t)n * 8));
    FGI_HIP(g, hipMalloc(&k1, (size_t)n * 8));
    FGI_HIP(g, hipMemsetAsync(cnt, 0, (size_t)n * 4, s));
    FGI_HIP(g, hipMemsetAsync(hot, 0, (size_t)n * 4, s));
    hipLaunchKernelGGL(kx_deg, dim3(8192), dim3(256), 0, s, m, keys, which, cnt);
    hipLaunchKernelGGL(kx_sortkey, dim3((n + 255) / 256), dim3(256), 0, s, n, cnt, slot_order, k0);
    size_t tb = 0;
    FGI_HIP(g, rocprim::radix_sort_keys_desc(nullptr, tb, k0, k1, (size_t)n, 0, 64, s));
    void* tmp;
    FGI_HIP(g, hipMalloc(&tmp, tb));
    FGI_HIP(g, rocprim::radix_sort_keys_desc(tmp, tb, k0, k1, (size_t)n, 0, 64, s));
    hipLaunchKernelGGL(kx_hot, dim3((uint32_t)((K + 255) / 256)), dim3(256), 0, s, n, (uint32_t)K, k1, hot);
    hipLaunchKernelGGL(kx_cold, dim3((n + 255) / 256), dim3(256), 0, s, n, hot, cold);
    size_t sb = 0;
    FGI_HIP(g, rocprim::exclusive_scan(nullptr, sb, cold, pos, 0u, (size_t)n, rocprim::plus<uint32_t>(), s));
    void* stmp;
    FGI_HIP(g, hipMalloc(&stmp, sb));
    FGI_HIP(g, rocprim::exclusive_scan(stmp, sb, cold, pos, 0u, (size_t)n, rocprim::plus<uint32_t>(), s));
    hipLaunchKernelGGL(kx_perm, dim3((n + 255) / 256), dim3(256), 0, s, n, (uint32_t)K, hot, pos, slot_order, perm);
    hipLaunchKernelGGL(kx_apply, dim3(8192), dim3(256), 0, s, m, perm, keys);
    FGI_HIP(g, hipStreamSynchronize(s));
    for (void* p : {(void*)cnt, (void*)hot, (void*)cold, (void*)pos, (void*)perm, (void*)k0, (void*)k1, tmp, stmp})
        hipFree(p);
    fprintf(stderr, "[fgi] FGI_EXP_RELABEL: %lld heaviest of %u slots (weight %u) relabelled first (slot order %u)\n", K, n, which, slot_order);
    return FGI_OK;
}

fgi_status synth_rmat_keys(fgi_graph* g, uint32_t scale, uint32_t edge_factor, uint64_t seed, uint64_t** keys,
                           uint64_t* m) {
    *m = (uint64_t)edge_factor << scale;
    FGI_HIP(g, hipMalloc(reinterpret_cast<void**>(keys), *m * sizeof(uint64_t)));
    hipLaunchKernelGGL(k_gen_rmat, dim3(8192), dim3(256), 0, g->stream, *m, scale, seed, *keys);
    FGI_HIP(g, hipGetLastError());
    return FGI_OK;
}

// rows from generated keys (boundary slots): with hub-first labels the tags are computed from the
// slots first, then the first load chooses the labels and the keys become labels
static fgi_status synth_rows(fgi_graph* g, uint64_t m, uint64_t* keys, uint64_t seed, uint32_t stale_pct, uint64_t stale_seed) {
    if (!g->lbl_K) return build_rows_from_keys(g, m, keys, nullptr, seed, stale_pct, stale_seed);
    uint64_t* tags = nullptr;
    FGI_HIP(g, hipMalloc(reinterpret_cast<void**>(&tags), std::max<uint64_t>(m, 1) * sizeof(uint64_t)));
    hipLaunchKernelGGL(k_synth_tags, dim3(8192), dim3(256), 0, g->stream, m, keys, seed, stale_pct, stale_seed, tags);
    fgi_status st = hipGetLastError() == hipSuccess ? FGI_OK : FGI_EDEVICE;
    if (st == FGI_OK) st = labels_choose(g, keys, m);
    if (st == FGI_OK) st = labels_map_keys(g, keys, m);
    if (st == FGI_OK) st = build_rows_from_keys(g, m, keys, tags, seed, stale_pct, stale_seed);
    hipFree(tags);
    return st;
}

fgi_status synth_versions(fgi_graph* g, uint32_t n, uint64_t seed) {
    FGI_HIP(g, hipMemsetAsync(g->node, 0, (size_t)g->n_handles * 8, g->stream));
    FGI_HIP(g, hipMemsetAsync(g->vis_bm, 0, g->bm_words * 4, g->stream));   // a new node table
    g->v_dirty = false;
    g->vis_stale = false;
    note_words(g);
    hipLaunchKernelGGL(k_versions, dim3((n + 255) / 256), dim3(256), 0, g->stream, n, seed, g->lbl_K,
                       reinterpret_cast<unsigned long long*>(g->node));
    FGI_HIP(g, hipGetLastError());
    return FGI_OK;
}

}  // namespace fgi

using namespace fgi;

extern "C" {

fgi_status fgi_synth_layered(fgi_graph* g, uint32_t levels, uint32_t width, uint32_t fanout, uint64_t seed) {
    if (!g || levels < 2 || width == 0 || fanout == 0 || fanout > 64 || fanout > width) return FGI_EINVAL;
    const uint64_t n = (uint64_t)levels * width;
    if (n > g->ext_slots) return set_err(g, FGI_EINVAL, "graph needs %llu slots", (unsigned long long)n);
    hipSetDevice(g->device);
    FGI_TRY(synth_versions(g, (uint32_t)n, seed));
    const uint64_t m = (uint64_t)(levels - 1) * width * fanout;
    uint64_t* keys = nullptr;
    FGI_HIP(g, hipMalloc(reinterpret_cast<void**>(&keys), m * sizeof(uint64_t)));
    const uint64_t threads = (uint64_t)(levels - 1) * width;
    hipLaunchKernelGGL(k_gen_layered, dim3((uint32_t)((threads + 255) / 256)), dim3(256), 0, g->stream, levels, width,
                       fanout, seed, keys);
    fgi_status st = hipGetLastError() == hipSuccess ? synth_rows(g, m, keys, seed, 0, 0) : FGI_EDEVICE;
    hipFree(keys);
    return st;
}

fgi_status fgi_synth_rmat(fgi_graph* g, uint32_t scale, uint32_t edge_factor, uint64_t seed, uint32_t stale_pct,
                          uint64_t stale_seed) {
    if (!g || scale == 0 || scale > 31 || edge_factor == 0 || stale_pct > 100) return FGI_EINVAL;
    if ((1ull << scale) > g->ext_slots) return set_err(g, FGI_EINVAL, "graph needs 2^%u slots", scale);
    hipSetDevice(g->device);
    FGI_TRY(synth_versions(g, 1u << scale, seed));
    uint64_t* keys = nullptr;
    uint64_t m = 0;
    FGI_TRY(synth_rmat_keys(g, scale, edge_factor, seed, &keys, &m));
    if (!g->lbl_K) FGI_TRY(exp_relabel(g, 1u << scale, keys, m));
    fgi_status st = synth_rows(g, m, keys, seed, stale_pct, stale_seed);
    hipFree(keys);
    return st;
}

}  // extern "C"
