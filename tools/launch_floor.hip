// Kernel-boundary cost on one stream (measurement tool, not part of the engine): N dependent launches
// queued behind a spinning kernel, so the host's launch rate does not set the pace; the device time of
// the N launches / N is the boundary + dispatch cost of one launch of that shape.
//   hipcc --offload-arch=gfx950 -O3 -o tools/launch_floor tools/launch_floor.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <cstring>

#define CK(x)                                                                                   \
    do {                                                                                        \
        hipError_t e_ = (x);                                                                    \
        if (e_ != hipSuccess) {                                                                 \
            fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_));           \
            exit(1);                                                                            \
        }                                                                                       \
    } while (0)

struct Big {
    unsigned long long w[160];   // 1,280 B of kernel arguments (k_level's are ~1.2 KB)
};

__global__ void k_spin(unsigned long long cycles) {   // ~cycles of the 100 MHz wall clock
    const unsigned long long t0 = wall_clock64();
    while (wall_clock64() - t0 < cycles) __builtin_amdgcn_s_sleep(8);
}
__global__ void k_empty(int) {}
__global__ void k_big(Big b, unsigned long long* out) {
    if (threadIdx.x == 0 && blockIdx.x == 0 && b.w[7] == 12345ull) out[0] = 1;
}
__global__ void k_lds(unsigned long long* out, int z) {
    __shared__ unsigned long long s[4096];   // 32 KB static LDS
    s[threadIdx.x] = threadIdx.x;
    __syncthreads();
    if (z && threadIdx.x == 0) out[blockIdx.x] = s[(threadIdx.x + 1) & 255];
}
__global__ void k_host_word(unsigned long long* host, unsigned long long v) {
    if (threadIdx.x == 0 && blockIdx.x == 0) host[0] = v;
}
__global__ void k_dirty(uint4* p, size_t n) {   // leaves n * 16 B dirty in L2
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
        p[i] = make_uint4((uint32_t)i, 1u, 2u, 3u);
}

int main(int argc, char** argv) {
    const int N = argc > 1 ? atoi(argv[1]) : 2000;
    hipStream_t s;
    CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    unsigned long long* dev;
    CK(hipMalloc(&dev, 1 << 20));
    unsigned long long* host;
    CK(hipHostMalloc(reinterpret_cast<void**>(&host), 4096, hipHostMallocCoherent));
    uint4* dirty;
    const size_t dn = (8u << 20) / 16;   // 8 MB
    CK(hipMalloc(&dirty, dn * 16));
    Big big;
    memset(&big, 0, sizeof(big));

    auto run = [&](const char* name, auto launch, int per, int cnt = 0) {
        const int n = cnt ? cnt : N;
        // warm
        for (int i = 0; i < 50; ++i) launch(i);
        CK(hipStreamSynchronize(s));
        hipLaunchKernelGGL(k_spin, dim3(1), dim3(64), 0, s, 100000ull * (N / 100 + 4));   // ~N * 10 us
        CK(hipEventRecord(a, s));
        for (int i = 0; i < n; ++i) launch(i);
        CK(hipEventRecord(b, s));
        CK(hipStreamSynchronize(s));
        float ms = 0;
        CK(hipEventElapsedTime(&ms, a, b));
        printf("%-44s %7.3f us per launch (%d launches x %d)\n", name, ms * 1000.0 / n / per, n, per);
    };
    run("empty <<<1,256>>>", [&](int) { hipLaunchKernelGGL(k_empty, dim3(1), dim3(256), 0, s, 0); }, 1);
    run("empty <<<256,256>>>", [&](int) { hipLaunchKernelGGL(k_empty, dim3(256), dim3(256), 0, s, 0); }, 1);
    run("empty <<<1024,256>>>", [&](int) { hipLaunchKernelGGL(k_empty, dim3(1024), dim3(256), 0, s, 0); }, 1);
    run("empty <<<4096,256>>>", [&](int) { hipLaunchKernelGGL(k_empty, dim3(4096), dim3(256), 0, s, 0); }, 1);
    run("1.3 KB kernarg <<<1,256>>>", [&](int) { hipLaunchKernelGGL(k_big, dim3(1), dim3(256), 0, s, big, dev); }, 1);
    run("1.3 KB kernarg <<<1024,256>>>", [&](int) { hipLaunchKernelGGL(k_big, dim3(1024), dim3(256), 0, s, big, dev); }, 1);
    run("32 KB LDS <<<1024,256>>>", [&](int) { hipLaunchKernelGGL(k_lds, dim3(1024), dim3(256), 0, s, dev, 0); }, 1);
    run("store to coherent host word <<<1,256>>>",
        [&](int i) { hipLaunchKernelGGL(k_host_word, dim3(1), dim3(256), 0, s, host, (unsigned long long)i); }, 1);
    run("8 MB dirty + empty (pair)", [&](int) {
        hipLaunchKernelGGL(k_dirty, dim3(2048), dim3(256), 0, s, dirty, dn);
        hipLaunchKernelGGL(k_empty, dim3(1), dim3(256), 0, s, 0);
    }, 1);
    run("8 MB dirty alone", [&](int) { hipLaunchKernelGGL(k_dirty, dim3(2048), dim3(256), 0, s, dirty, dn); }, 1);
    // a captured graph of 100 empty launches, replayed
    {
        hipGraph_t g;
        hipGraphExec_t ge;
        CK(hipStreamBeginCapture(s, hipStreamCaptureModeThreadLocal));
        for (int i = 0; i < 100; ++i) hipLaunchKernelGGL(k_empty, dim3(1), dim3(256), 0, s, 0);
        CK(hipStreamEndCapture(s, &g));
        CK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
        const int n0 = N;
        run("graph of 100 empty <<<1,256>>> (per node)", [&](int) { CK(hipGraphLaunch(ge, s)); }, 100, N / 20);
        (void)n0;
        CK(hipGraphExecDestroy(ge));
        CK(hipGraphDestroy(g));
    }
    CK(hipStreamDestroy(s));
    return 0;
}
