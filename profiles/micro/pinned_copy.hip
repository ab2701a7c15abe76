// Host copy rates into hipHostMalloc'd staging vs ordinary memory (fgi_run_batch stages its inputs in
// pinned memory): 2.5 MB per copy, cold source (a fresh 2.5 MB slice of a 256 MB array each time).
// Build: hipcc -O3 --offload-arch=gfx950 -o pinned_copy pinned_copy.hip
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

int main() {
    const size_t B = 2500000, N = 256u << 20;
    std::vector<char> src(N, 1);
    char* pinned = nullptr;
    char* pinned_wc = nullptr;
    if (hipHostMalloc(reinterpret_cast<void**>(&pinned), B) != hipSuccess) return 1;
    if (hipHostMalloc(reinterpret_cast<void**>(&pinned_wc), B, hipHostMallocWriteCombined) != hipSuccess) return 1;
    std::vector<char> plain(B, 0);
    struct Dst { const char* name; char* p; } dsts[] = {{"pinned(default)", pinned}, {"pinned(write-combined)", pinned_wc}, {"malloc", plain.data()}};
    for (auto& d : dsts) {
        for (int hot = 0; hot < 2; ++hot) {
            double best = 1e9, sum = 0;
            const int R = 40;
            for (int r = 0; r < R; ++r) {
                const size_t off = hot ? 0 : (size_t)r * B % (N - B);
                auto t0 = std::chrono::steady_clock::now();
                std::memcpy(d.p, src.data() + off, B);
                auto t1 = std::chrono::steady_clock::now();
                const double us = std::chrono::duration<double, std::micro>(t1 - t0).count();
                best = us < best ? us : best;
                sum += us;
            }
            std::printf("%-24s %s source: median-ish avg %.1f us, best %.1f us (%.1f GB/s)\n", d.name, hot ? "hot " : "cold",
                        sum / R, best, B / best / 1e3);
        }
    }
    hipHostFree(pinned);
    hipHostFree(pinned_wc);
    return 0;
}
