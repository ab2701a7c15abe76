// Microbenchmark (measurement only, not part of the engine): a pull level's probe mix on MI355X.
// Streams N 16-byte candidates (non-temporal, 4 per lane per step like pull_level) and probes two
// random 32-bit words per candidate: a fraction HOT of them in an 8 KB hot region (the hot heads'
// snapshot), the rest in a cold table of B bytes. configs[1] today: 80% hot, cold table = the 2 MB
// invalidated bitmap; configs[2]: cold table 16 MB. A head-only cold bitmap (one bit per distinct
// list head, slot order) shrinks the cold table to ~140 KB (R-MAT 24) / ~1-2 MB (R-MAT 27).
//   hipcc --offload-arch=gfx950 -O3 -o probe_mix probe_mix.hip && ./probe_mix
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <vector>

#define CHECK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); return 1; } } while (0)

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ uint32_t word_of(uint32_t r, uint32_t hot_pct, uint32_t cold_words) {
    // r's top bits choose hot vs cold, the rest the word
    const bool hot = ((r >> 25) * 100u) >> 7 < hot_pct;
    return hot ? (r & 2047u) : 2048u + (r % cold_words);
}

__global__ __launch_bounds__(256, 5) void k_probe(const u32x4* __restrict__ cand, uint64_t n, const uint32_t* __restrict__ bm,
                                                  uint32_t hot_pct, uint32_t cold_words, uint32_t* out) {
    uint32_t acc = 0;
    const uint64_t stride = (uint64_t)gridDim.x * 1024;
    for (uint64_t base = (uint64_t)blockIdx.x * 1024 + (threadIdx.x >> 6) * 256; base < n; base += stride) {
        u32x4 c[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const uint64_t i = base + j * 64 + (threadIdx.x & 63);
            c[j] = i < n ? __builtin_nontemporal_load(cand + i) : u32x4{0, 0, 0, 0};
        }
        uint32_t f[8];
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            f[2 * j] = bm[word_of(c[j].z, hot_pct, cold_words)];
            f[2 * j + 1] = bm[word_of(c[j].w, hot_pct, cold_words)];
        }
#pragma unroll
        for (int j = 0; j < 4; ++j) acc += ((f[2 * j] >> (c[j].z & 31)) | (f[2 * j + 1] >> (c[j].w & 31))) & 1u;
    }
    if (acc == 0xFFFFFFFFu) out[0] = acc;   // never: keeps the loads
}

int main() {
    const uint64_t n = 8ull << 20;   // 8 M candidates = 128 MB (configs[1]'s first pull level)
    u32x4* cand;
    uint32_t *bm, *out;
    CHECK(hipMalloc(&cand, n * 16));
    CHECK(hipMalloc(&bm, 64u << 20));
    CHECK(hipMalloc(&out, 4));
    std::vector<u32x4> h(n);
    uint64_t s = 88172645463325252ull;
    for (uint64_t i = 0; i < n; ++i) {
        s ^= s << 13; s ^= s >> 7; s ^= s << 17;
        h[i] = u32x4{(uint32_t)i, 0, (uint32_t)s, (uint32_t)(s >> 32)};
    }
    CHECK(hipMemcpy(cand, h.data(), n * 16, hipMemcpyHostToDevice));
    CHECK(hipMemset(bm, 0x55, 64u << 20));
    hipEvent_t e0, e1;
    CHECK(hipEventCreate(&e0));
    CHECK(hipEventCreate(&e1));
    const uint32_t hots[] = {0, 80, 90, 100};
    const uint32_t tables[] = {32u << 10, 128u << 10, 512u << 10, 2u << 20, 16u << 20};
    for (uint32_t hp : hots) {
        for (uint32_t tb : tables) {
            if (hp == 100 && tb != tables[0]) continue;
            const uint32_t cw = tb / 4;
            for (int w = 0; w < 3; ++w) hipLaunchKernelGGL(k_probe, dim3(1280), dim3(256), 0, 0, cand, n, bm, hp, cw, out);
            CHECK(hipEventRecord(e0));
            const int R = 20;
            for (int r = 0; r < R; ++r) hipLaunchKernelGGL(k_probe, dim3(1280), dim3(256), 0, 0, cand, n, bm, hp, cw, out);
            CHECK(hipEventRecord(e1));
            CHECK(hipEventSynchronize(e1));
            float ms;
            CHECK(hipEventElapsedTime(&ms, e0, e1));
            const double us = ms * 1000.0 / R;
            printf("hot %3u%% cold table %8u B  %8.1f us  %7.0f GB/s candidates  %6.1f G probes/s\n", hp, tb, us,
                   n * 16 / us / 1e3, 2.0 * n / us / 1e3);
        }
    }
    return 0;
}
