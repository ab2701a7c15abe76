// synth.hip — device generators for the benchmark workloads.
// Same definitions as the CPU oracle's oracle/synth.cpp (checked equal in tests), written for the
// device so a 256M-edge graph is generated and turned into rows in HBM in well under a second.
#include <hip/hip_runtime.h>

#include "fgi_internal.h"

namespace fgi {
namespace {

__global__ void k_versions(uint32_t n, uint64_t seed, unsigned long long* node) {
    const uint32_t s = blockIdx.x * blockDim.x + threadIdx.x;
    if (s < n) node[s] = synth_version(seed, s) | kW_Consistent;
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

}  // namespace

fgi_status synth_rmat_keys(fgi_graph* g, uint32_t scale, uint32_t edge_factor, uint64_t seed, uint64_t** keys,
                           uint64_t* m) {
    *m = (uint64_t)edge_factor << scale;
    FGI_HIP(g, hipMalloc(reinterpret_cast<void**>(keys), *m * sizeof(uint64_t)));
    hipLaunchKernelGGL(k_gen_rmat, dim3(8192), dim3(256), 0, g->stream, *m, scale, seed, *keys);
    FGI_HIP(g, hipGetLastError());
    return FGI_OK;
}

fgi_status synth_versions(fgi_graph* g, uint32_t n, uint64_t seed) {
    FGI_HIP(g, hipMemsetAsync(g->node, 0, (size_t)g->n_handles * 8, g->stream));
    FGI_HIP(g, hipMemsetAsync(g->vis_bm, 0, g->bm_words * 4, g->stream));   // a new node table
    g->v_dirty = false;
    g->vis_stale = false;
    note_words(g);
    hipLaunchKernelGGL(k_versions, dim3((n + 255) / 256), dim3(256), 0, g->stream, n, seed,
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
    if (n > g->n_slots) return set_err(g, FGI_EINVAL, "graph needs %llu slots", (unsigned long long)n);
    hipSetDevice(g->device);
    FGI_TRY(synth_versions(g, (uint32_t)n, seed));
    const uint64_t m = (uint64_t)(levels - 1) * width * fanout;
    uint64_t* keys = nullptr;
    FGI_HIP(g, hipMalloc(reinterpret_cast<void**>(&keys), m * sizeof(uint64_t)));
    const uint64_t threads = (uint64_t)(levels - 1) * width;
    hipLaunchKernelGGL(k_gen_layered, dim3((uint32_t)((threads + 255) / 256)), dim3(256), 0, g->stream, levels, width,
                       fanout, seed, keys);
    fgi_status st = hipGetLastError() == hipSuccess ? build_rows_from_keys(g, m, keys, nullptr, seed, 0, 0) : FGI_EDEVICE;
    hipFree(keys);
    return st;
}

fgi_status fgi_synth_rmat(fgi_graph* g, uint32_t scale, uint32_t edge_factor, uint64_t seed, uint32_t stale_pct,
                          uint64_t stale_seed) {
    if (!g || scale == 0 || scale > 31 || edge_factor == 0 || stale_pct > 100) return FGI_EINVAL;
    if ((1ull << scale) > g->n_slots) return set_err(g, FGI_EINVAL, "graph needs 2^%u slots", scale);
    hipSetDevice(g->device);
    FGI_TRY(synth_versions(g, 1u << scale, seed));
    uint64_t* keys = nullptr;
    uint64_t m = 0;
    FGI_TRY(synth_rmat_keys(g, scale, edge_factor, seed, &keys, &m));
    fgi_status st = build_rows_from_keys(g, m, keys, nullptr, seed, stale_pct, stale_seed);
    hipFree(keys);
    return st;
}

}  // extern "C"
