// Microbenchmark (measurement only, not part of the engine): where a pull level's head probes should
// read the hot heads' snapshot from. N 16-byte candidates are streamed (non-temporal, 4 per lane per
// step); each probes two heads. A fraction P of the heads is hot (a code below HOT), the rest probe a
// 2 MB bitmap (L2-resident, configs[1]'s 16.7 M slots). The hot snapshot is read either from global
// memory (a HOT / 8-byte table: L1-resident at 8 KB) or from LDS, filled once per block.
//   hipcc --offload-arch=gfx950 -O3 -o snap_rate snap_rate.hip && ./snap_rate
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <vector>

#define CHECK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); return 1; } } while (0)

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

// LDS = 0: the snapshot is read from global memory; otherwise staged into LDS first
template <uint32_t HOT, int LDS, int BLOCK>
__global__ __launch_bounds__(BLOCK) void k_snap(const u32x4* __restrict__ cand, uint64_t n, const uint32_t* __restrict__ snap,
                                               const uint32_t* __restrict__ bm, uint32_t* out) {
    __shared__ uint32_t s_snap[LDS ? HOT / 32 : 1];
    if (LDS) {
        for (uint32_t i = threadIdx.x; i < HOT / 32; i += BLOCK) s_snap[i] = snap[i];
        __syncthreads();
    }
    uint32_t acc = 0;
    constexpr uint32_t kStep = BLOCK * 4;
    const uint64_t stride = (uint64_t)gridDim.x * kStep;
    for (uint64_t base = (uint64_t)blockIdx.x * kStep + (threadIdx.x >> 6) * 256; base < n; base += stride) {
        u32x4 c[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const uint64_t i = base + j * 64 + (threadIdx.x & 63);
            c[j] = i < n ? __builtin_nontemporal_load(cand + i) : u32x4{0, 0, 0, 0};
        }
        uint32_t f[8];
#pragma unroll
        for (int j = 0; j < 4; ++j) {
#pragma unroll
            for (int k = 0; k < 2; ++k) {
                const uint32_t h = k ? c[j].w : c[j].z;
                uint32_t v;
                if (h < HOT) v = LDS ? s_snap[h >> 5] : snap[h >> 5];
                else v = bm[((h - HOT) >> 5) & ((2u << 20) / 4 - 1)];
                f[2 * j + k] = v;
            }
        }
#pragma unroll
        for (int j = 0; j < 4; ++j) acc += ((f[2 * j] >> (c[j].z & 31)) | (f[2 * j + 1] >> (c[j].w & 31))) & 1u;
    }
    if (acc == 0xFFFFFFFFu) out[0] = acc;   // never: keeps the loads
}

int main() {
    const uint64_t n = 8ull << 20;   // 8 M candidates = 128 MB
    u32x4* cand;
    uint32_t *bm, *snap, *out;
    CHECK(hipMalloc(&cand, n * 16));
    CHECK(hipMalloc(&bm, 2u << 20));
    CHECK(hipMalloc(&snap, 1u << 20));
    CHECK(hipMalloc(&out, 4));
    CHECK(hipMemset(bm, 0x55, 2u << 20));
    CHECK(hipMemset(snap, 0x33, 1u << 20));
    hipEvent_t e0, e1;
    CHECK(hipEventCreate(&e0));
    CHECK(hipEventCreate(&e1));
    std::vector<u32x4> h(n);
    const double fracs[] = {0.8, 0.95, 1.0};
    for (double p : fracs) {
        auto fill = [&](uint32_t hot) {
            uint64_t s = 88172645463325252ull;
            auto rnd = [&]() { s ^= s << 13; s ^= s >> 7; s ^= s << 17; return s; };
            for (uint64_t i = 0; i < n; ++i) {
                uint32_t hd[2];
                for (int k = 0; k < 2; ++k) {
                    const uint64_t r = rnd();
                    const bool is_hot = (double)(r & 0xFFFFFF) / 16777216.0 < p;
                    hd[k] = is_hot ? (uint32_t)((r >> 24) % hot) : hot + (uint32_t)((r >> 24) % (16u << 20));
                }
                h[i] = u32x4{(uint32_t)i, 0, hd[0], hd[1]};
            }
            return hipMemcpy(cand, h.data(), n * 16, hipMemcpyHostToDevice);
        };
        auto time = [&](auto kern, uint32_t grid, uint32_t block, const char* name) -> int {
            for (int w = 0; w < 3; ++w) hipLaunchKernelGGL(kern, dim3(grid), dim3(block), 0, 0, cand, n, snap, bm, out);
            CHECK(hipEventRecord(e0));
            const int R = 20;
            for (int r = 0; r < R; ++r) hipLaunchKernelGGL(kern, dim3(grid), dim3(block), 0, 0, cand, n, snap, bm, out);
            CHECK(hipGetLastError());
            CHECK(hipEventRecord(e1));
            CHECK(hipEventSynchronize(e1));
            float ms;
            CHECK(hipEventElapsedTime(&ms, e0, e1));
            printf("hot %.2f %-40s %7.1f us\n", p, name, ms * 1000.0 / R);
            return 0;
        };
        CHECK(fill(65536));
        if (time(k_snap<65536, 0, 256>, 1280, 256, "64 Ki heads, global (8 KB), 5x256/CU")) return 1;
        if (time(k_snap<65536, 1, 256>, 1280, 256, "64 Ki heads, LDS (8 KB), 5x256/CU")) return 1;
        CHECK(fill(262144));
        if (time(k_snap<262144, 0, 256>, 1280, 256, "256 Ki heads, global (32 KB), 5x256/CU")) return 1;
        if (time(k_snap<262144, 1, 256>, 1024, 256, "256 Ki heads, LDS (32 KB), 4x256/CU")) return 1;
        if (time(k_snap<262144, 1, 512>, 512, 512, "256 Ki heads, LDS (32 KB), 2x512/CU")) return 1;
        CHECK(fill(524288));
        if (time(k_snap<524288, 0, 256>, 1280, 256, "512 Ki heads, global (64 KB), 5x256/CU")) return 1;
        if (time(k_snap<524288, 1, 512>, 512, 512, "512 Ki heads, LDS (64 KB), 2x512/CU")) return 1;
        if (time(k_snap<524288, 1, 1024>, 256, 1024, "512 Ki heads, LDS (64 KB), 1x1024/CU")) return 1;
        CHECK(fill(1048576));
        (void)time(k_snap<1048576, 1, 1024>, 256, 1024, "1 Mi heads, LDS (128 KB), 1x1024/CU");   // may exceed the static LDS limit
    }
    return 0;
}
