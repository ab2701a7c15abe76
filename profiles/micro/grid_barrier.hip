// Microbenchmark (measurement only, not part of the engine): the cost of one software grid barrier
// of a plain launch on MI355X (k_wave_coop / k_wave_fused use one per level), by grid size and by
// how the barrier orders memory:
//   0  every thread: agent-scope seq_cst fence, block barrier, thread 0 arrives (relaxed atomic) and
//      polls (relaxed atomic loads, s_sleep 1), block barrier, every thread fences again (the engine's)
//   1  no fences at all (relaxed arrival and polls only: the pure counter cost; not a valid barrier)
//   2  thread 0 only: release-ordered arrival, acquire-ordered polls (one wave per block does the cache
//      maintenance instead of every wave)
//   3  as 2 without s_sleep in the poll
//   4  as 2, the arrival counted per XCD group first (blockIdx % 8), the last of a group arrives on the
//      top counter; waiters poll the top counter
// Each block also writes `dirty` KB of plain stores between barriers (lines its L2 must write back).
//   hipcc --offload-arch=gfx950 -O3 -o grid_barrier grid_barrier.hip && ./grid_barrier
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>

#define CHECK(x)                                                              \
    do {                                                                      \
        hipError_t e = (x);                                                   \
        if (e != hipSuccess) {                                                \
            printf("%s: %s\n", #x, hipGetErrorString(e));                     \
            return 1;                                                         \
        }                                                                     \
    } while (0)

template <int V>
__device__ __forceinline__ void bar(unsigned long long* cnt, unsigned long long* grp, uint32_t G) {
    __shared__ int dummy;
    if (V == 0) __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "agent");
    __syncthreads();
    if (threadIdx.x == 0) {
        if (V == 4) {
            const uint32_t g = blockIdx.x % 8;
            const uint32_t gsize = (G - g + 7) / 8;
            const unsigned long long a = __hip_atomic_fetch_add(grp + g * 16, 1ull, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
            if ((a + 1) % gsize == 0) __hip_atomic_fetch_add(cnt, 1ull, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
            const unsigned long long rounds = a / gsize + 1;   // this barrier's index (1-based)
            const unsigned long long ng = G < 8 ? G : 8;
            while (__hip_atomic_load(cnt, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT) < rounds * ng) __builtin_amdgcn_s_sleep(1);
        } else {
            const int order = V >= 2 ? __ATOMIC_RELEASE : __ATOMIC_RELAXED;
            const unsigned long long arrived = __hip_atomic_fetch_add(cnt, 1ull, order, __HIP_MEMORY_SCOPE_AGENT);
            const unsigned long long target = (arrived / G + 1) * G;
            while (__hip_atomic_load(cnt, V >= 2 ? __ATOMIC_ACQUIRE : __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < target)
                if (V != 3) __builtin_amdgcn_s_sleep(1);
        }
        dummy = 0;
    }
    __syncthreads();
    if (V == 0) __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "agent");
}

template <int V>
__global__ __launch_bounds__(256) void k_bars(int K, unsigned long long* cnt, unsigned long long* grp, uint32_t* scratch,
                                              uint32_t dirty_words) {
    uint32_t* mine = scratch + (uint64_t)blockIdx.x * dirty_words;
    for (int k = 0; k < K; ++k) {
        for (uint32_t i = threadIdx.x; i < dirty_words; i += blockDim.x) mine[i] = k + i;
        bar<V>(cnt, grp, gridDim.x);
    }
}

template <int V>
int run(uint32_t G, uint32_t dirty_kb, unsigned long long* cnt, unsigned long long* grp, uint32_t* scratch) {
    const int K = 2000;
    hipEvent_t a, b;
    CHECK(hipEventCreate(&a));
    CHECK(hipEventCreate(&b));
    for (int rep = 0; rep < 2; ++rep) {
        CHECK(hipMemset(cnt, 0, 8));
        CHECK(hipMemset(grp, 0, 8 * 16 * 8));
        CHECK(hipDeviceSynchronize());
        CHECK(hipEventRecord(a));
        hipLaunchKernelGGL(k_bars<V>, dim3(G), dim3(256), 0, 0, K, cnt, grp, scratch, dirty_kb * 256);
        CHECK(hipEventRecord(b));
        CHECK(hipEventSynchronize(b));
        float ms = 0;
        CHECK(hipEventElapsedTime(&ms, a, b));
        if (rep) printf("variant %d grid %4u dirty %3u KB/block: %.3f us per barrier\n", V, G, dirty_kb, ms * 1e3 / K);
    }
    CHECK(hipEventDestroy(a));
    CHECK(hipEventDestroy(b));
    return 0;
}

int main() {
    unsigned long long *cnt, *grp;
    uint32_t* scratch;
    CHECK(hipMalloc(&cnt, 64));
    CHECK(hipMalloc(&grp, 8 * 16 * 8));
    CHECK(hipMalloc(&scratch, (size_t)1024 * 64 * 1024));
    for (uint32_t dirty : {0u, 16u}) {
        for (uint32_t G : {32u, 64u, 128u, 256u}) {
            if (run<0>(G, dirty, cnt, grp, scratch)) return 1;
            if (run<1>(G, dirty, cnt, grp, scratch)) return 1;
            if (run<2>(G, dirty, cnt, grp, scratch)) return 1;
            if (run<3>(G, dirty, cnt, grp, scratch)) return 1;
            if (run<4>(G, dirty, cnt, grp, scratch)) return 1;
        }
    }
    return 0;
}
