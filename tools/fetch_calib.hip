// FETCH_SIZE calibration for the engine's access shapes (measurement tool, not part of the engine).
// MI355X_MICROARCH.md: on gfx950 FETCH_SIZE reports half the bytes of a WIDE coalesced read (128-B
// requests tallied at 64 B); other widths are uncalibrated. The engine's k_level is mostly narrow random
// gathers (4-8 B per lane into distinct lines) and bitmap probes, so each shape below touches a KNOWN set
// of lines once, and the rocprofv3 counters per kernel are compared with that count:
//   k_stream   16 B per lane, coalesced, `bytes` bytes
//   k_gather4  one 4-B load in each of `lines` distinct 128-B lines (random order)
//   k_gather8  one 8-B load in each of `lines` distinct 128-B lines
//   k_gather4x2 two 4-B loads 64 B apart in each line (both halves of the line)
//   k_run      64 lanes read 256 contiguous bytes (4 B each) at random 256-B-aligned offsets (row reads)
//   hipcc --offload-arch=gfx950 -O3 -o tools/fetch_calib tools/fetch_calib.hip
#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstdio>
#include <cstdlib>

#define CK(x)                                                                                   \
    do {                                                                                        \
        hipError_t e_ = (x);                                                                    \
        if (e_ != hipSuccess) {                                                                 \
            fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_));           \
            exit(1);                                                                            \
        }                                                                                       \
    } while (0)

// a permutation of [0, n) for n a power of two: odd multiplier, xor-shift (bijective mod 2^k)
__device__ __forceinline__ uint64_t perm(uint64_t i, uint64_t mask) {
    i = (i * 0x9E3779B97F4A7C15ull) & mask;
    i ^= i >> 7;
    i = (i * 0xBF58476D1CE4E5B9ull) & mask;
    return i;
}

__global__ void k_stream(const uint4* __restrict__ p, uint64_t n, unsigned long long* out) {
    uint32_t acc = 0;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
        const uint4 v = p[i];
        acc ^= v.x ^ v.y ^ v.z ^ v.w;
    }
    if (acc == 0x12345678u) out[0] = acc;
}
__global__ void k_gather4(const uint32_t* __restrict__ p, uint64_t lines, unsigned long long* out) {
    uint32_t acc = 0;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < lines; i += (uint64_t)gridDim.x * blockDim.x)
        acc ^= p[perm(i, lines - 1) * 32 + (i & 31)];
    if (acc == 0x12345678u) out[0] = acc;
}
__global__ void k_gather8(const uint64_t* __restrict__ p, uint64_t lines, unsigned long long* out) {
    uint64_t acc = 0;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < lines; i += (uint64_t)gridDim.x * blockDim.x)
        acc ^= p[perm(i, lines - 1) * 16 + (i & 15)];
    if (acc == 0x12345678ull) out[0] = acc;
}
__global__ void k_gather4x2(const uint32_t* __restrict__ p, uint64_t lines, unsigned long long* out) {
    uint32_t acc = 0;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < lines; i += (uint64_t)gridDim.x * blockDim.x) {
        const uint64_t l = perm(i, lines - 1) * 32;
        acc ^= p[l + (i & 15)] ^ p[l + 16 + (i & 15)];
    }
    if (acc == 0x12345678u) out[0] = acc;
}
__global__ void k_run(const uint32_t* __restrict__ p, uint64_t runs, unsigned long long* out) {
    uint32_t acc = 0;
    const uint32_t lane = threadIdx.x & 63;
    const uint64_t w0 = ((uint64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6, W = ((uint64_t)gridDim.x * blockDim.x) >> 6;
    for (uint64_t r = w0; r < runs; r += W) acc ^= p[perm(r, runs - 1) * 64 + lane];
    if (acc == 0x12345678u) out[0] = acc;
}

int main(int argc, char** argv) {
    const uint64_t bytes = 1ull << 30;   // 1 GiB array: 8 M lines of 128 B
    const uint64_t lines = bytes / 128;
    const uint64_t glines = 1ull << 21;   // 2 M distinct lines gathered (256 MB of lines)
    void* a;
    CK(hipMalloc(&a, bytes));
    CK(hipMemset(a, 1, bytes));
    unsigned long long* out;
    CK(hipMalloc(&out, 64));
    CK(hipDeviceSynchronize());
    const dim3 grid(4096), blk(256);
    hipLaunchKernelGGL(k_stream, grid, blk, 0, 0, (const uint4*)a, bytes / 16 / 4, out);   // 256 MB
    hipLaunchKernelGGL(k_gather4, grid, blk, 0, 0, (const uint32_t*)a, glines, out);
    hipLaunchKernelGGL(k_gather8, grid, blk, 0, 0, (const uint64_t*)a + (bytes / 8 / 2), glines, out);
    hipLaunchKernelGGL(k_gather4x2, grid, blk, 0, 0, (const uint32_t*)a + (bytes / 4 / 4) * 1, glines / 2, out);
    hipLaunchKernelGGL(k_run, grid, blk, 0, 0, (const uint32_t*)a, glines / 2, out);
    CK(hipDeviceSynchronize());
    printf("k_stream    %llu bytes read (16 B per lane)\n", (unsigned long long)(bytes / 4));
    printf("k_gather4   %llu distinct 128-B lines, one 4-B load each (%llu B of lines)\n", (unsigned long long)glines,
           (unsigned long long)glines * 128);
    printf("k_gather8   %llu distinct 128-B lines, one 8-B load each (%llu B of lines)\n", (unsigned long long)glines,
           (unsigned long long)glines * 128);
    printf("k_gather4x2 %llu distinct 128-B lines, both 64-B halves read (%llu B of lines)\n",
           (unsigned long long)glines / 2, (unsigned long long)glines / 2 * 128);
    printf("k_run       %llu distinct 256-B runs, 64 lanes x 4 B (%llu B)\n", (unsigned long long)glines / 2,
           (unsigned long long)glines / 2 * 256);
    (void)lines;
    return 0;
}
