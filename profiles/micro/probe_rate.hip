// Microbenchmark (measurement only, not part of the engine): the memory shapes of a pull level on
// MI355X. Streams N 16-byte candidates (non-temporal, 4 per lane per step like pull_level) and, per
// candidate, probes 0, 1 or 2 random 32-bit words of a bitmap of B bytes (L2-resident at 2 MB,
// MALL-resident at 16 MB, L1-resident at 8 KB). Reports GB/s of candidates and probes per second.
//   hipcc --offload-arch=gfx950 -O3 -o probe_rate probe_rate.hip && ./probe_rate
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <vector>

#define CHECK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); return 1; } } while (0)

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

template <int PROBES, int STREAM>
__global__ __launch_bounds__(256, 5) void k_probe(const u32x4* __restrict__ cand, uint64_t n, const uint32_t* __restrict__ bm,
                                                   uint32_t mask_words, uint32_t* out) {
    uint32_t acc = 0;
    const uint64_t stride = (uint64_t)gridDim.x * 1024;
    for (uint64_t base = (uint64_t)blockIdx.x * 1024 + (threadIdx.x >> 6) * 256; base < n; base += stride) {
        u32x4 c[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const uint64_t i = base + j * 64 + (threadIdx.x & 63);
            if (STREAM) c[j] = i < n ? __builtin_nontemporal_load(cand + i) : u32x4{0, 0, 0, 0};
            else {   // addresses from a hash of the index: no stream
                uint32_t h = (uint32_t)i * 2654435761u;
                c[j] = u32x4{(uint32_t)i, 0, h ^ (h >> 13), (h * 40503u) ^ (h >> 7)};
            }
        }
        uint32_t f[8];
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            f[2 * j] = PROBES >= 1 ? bm[(c[j].z >> 5) & mask_words] : c[j].z;
            f[2 * j + 1] = PROBES >= 2 ? bm[(c[j].w >> 5) & mask_words] : c[j].w;
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
    const uint32_t grids[] = {1280, 2560};
    const uint32_t tables[] = {8u << 10, 2u << 20, 16u << 20};
    for (uint32_t G : grids) {
        for (uint32_t tb : tables) {
            const uint32_t mw = tb / 4 - 1;
            auto run = [&](auto kern, const char* name) -> int {
                for (int w = 0; w < 3; ++w) hipLaunchKernelGGL(kern, dim3(G), dim3(256), 0, 0, cand, n, bm, mw, out);
                CHECK(hipEventRecord(e0));
                const int R = 20;
                for (int r = 0; r < R; ++r) hipLaunchKernelGGL(kern, dim3(G), dim3(256), 0, 0, cand, n, bm, mw, out);
                CHECK(hipEventRecord(e1));
                CHECK(hipEventSynchronize(e1));
                float ms;
                CHECK(hipEventElapsedTime(&ms, e0, e1));
                const double us = ms * 1000.0 / R;
                printf("grid %u table %7u B %-22s %8.1f us  %7.0f GB/s candidates  %6.1f G probes/s\n", G, tb, name, us,
                       n * 16 / us / 1e3, (double)n * (name[0] == '2' ? 2 : name[0] == '1' ? 1 : 0) / us / 1e3);
                return 0;
            };
            if (tb == tables[0]) if (run(k_probe<0, 1>, "0 probes, stream")) return 1;
            if (run(k_probe<1, 1>, "1 probe, stream")) return 1;
            if (run(k_probe<2, 1>, "2 probes, stream")) return 1;
            if (run(k_probe<2, 0>, "2 probes, no stream")) return 1;
        }
    }
    return 0;
}
