// synth.cpp — TEST INFRASTRUCTURE ONLY: CPU definition of the synthetic workloads
// (DESIGN.md §Workloads). The engine generates the same graphs on the device with its own code
// (stl.fusion_amd/csrc/synth.hip); tests/test_gpu_parity.py checks the two edge sets are equal.
#include "fgo.h"

#include <algorithm>
#include <atomic>
#include <thread>
#include <vector>

namespace {
constexpr uint64_t kGolden = 0x9E3779B97F4A7C15ull;
constexpr uint64_t kVersionMask = (1ull << 55) - 1;   // ConcurrentLTagGenerator mask: long.MaxValue >> 8

inline uint64_t sm64(uint64_t x) {
    x += kGolden;
    x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
    x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
    return x ^ (x >> 31);
}

// Bijective scramble of [0, 2^scale): odd multiply, xorshift, add, odd multiply, xorshift.
inline uint32_t scramble(uint64_t x, uint32_t scale, uint64_t seed) {
    const uint64_t mask = (scale >= 64) ? ~0ull : ((1ull << scale) - 1);
    const uint64_t k1 = sm64(seed ^ 0xA5A5A5A5A5A5A5A5ull) | 1ull;
    const uint64_t k2 = sm64(seed ^ 0x5A5A5A5A5A5A5A5Aull) | 1ull;
    const uint64_t c = sm64(seed ^ 0x0123456789ABCDEFull);
    const uint32_t s1 = (scale + 1) / 2, s2 = scale / 2 ? scale / 2 : 1;
    x = (x * k1) & mask;
    x ^= x >> s1;
    x = (x + c) & mask;
    x = (x * k2) & mask;
    x ^= x >> s2;
    return (uint32_t)x;
}

template <class F>
void par(uint32_t T, F&& f) {
    if (T <= 1) {
        f(0u, 1u);
        return;
    }
    std::vector<std::thread> ts;
    for (uint32_t t = 0; t < T; ++t) ts.emplace_back([&, t]() { f(t, T); });
    for (auto& t : ts) t.join();
}

uint64_t finish(std::vector<uint64_t>& keys, uint32_t* src, uint32_t* dst) {
    std::sort(keys.begin(), keys.end());
    keys.erase(std::unique(keys.begin(), keys.end()), keys.end());
    if (src && dst) {
        for (size_t i = 0; i < keys.size(); ++i) {
            src[i] = (uint32_t)(keys[i] >> 32);
            dst[i] = (uint32_t)keys[i];
        }
    }
    return keys.size();
}

// Sorted, deduplicated (src, dst) of `keys` (src < 2^scale in the high word) with T threads:
// bucket by the top bits of src, sort and deduplicate the buckets independently (equal keys share
// a bucket), concatenate. Same output as finish().
uint64_t finish_parallel(std::vector<uint64_t>& keys, uint32_t scale, uint32_t T, uint32_t* src, uint32_t* dst) {
    const uint32_t bb = scale < 10 ? scale : 10;
    const uint32_t NB = 1u << bb;
    const uint32_t shift = 32 + scale - bb;
    const uint64_t m = keys.size();
    std::vector<uint64_t> cnt((size_t)T * NB, 0);
    par(T, [&](uint32_t t, uint32_t TT) {
        const uint64_t lo = m * t / TT, hi = m * (t + 1) / TT;
        for (uint64_t i = lo; i < hi; ++i) cnt[(size_t)t * NB + (keys[i] >> shift)]++;
    });
    std::vector<uint64_t> boff(NB + 1, 0), pos((size_t)T * NB);
    uint64_t run = 0;
    for (uint32_t b = 0; b < NB; ++b) {
        boff[b] = run;
        for (uint32_t t = 0; t < T; ++t) {
            pos[(size_t)t * NB + b] = run;
            run += cnt[(size_t)t * NB + b];
        }
    }
    boff[NB] = run;
    std::vector<uint64_t> out(m);
    par(T, [&](uint32_t t, uint32_t TT) {
        const uint64_t lo = m * t / TT, hi = m * (t + 1) / TT;
        uint64_t* p = &pos[(size_t)t * NB];
        for (uint64_t i = lo; i < hi; ++i) out[p[keys[i] >> shift]++] = keys[i];
    });
    std::vector<uint64_t>().swap(keys);
    std::vector<uint64_t> ulen(NB, 0);
    std::atomic<uint32_t> next{0};
    par(T, [&](uint32_t, uint32_t) {
        for (uint32_t b; (b = next.fetch_add(1)) < NB;) {
            auto first = out.begin() + (ptrdiff_t)boff[b], last = out.begin() + (ptrdiff_t)boff[b + 1];
            std::sort(first, last);
            ulen[b] = (uint64_t)(std::unique(first, last) - first);
        }
    });
    std::vector<uint64_t> uoff(NB + 1, 0);
    for (uint32_t b = 0; b < NB; ++b) uoff[b + 1] = uoff[b] + ulen[b];
    if (src && dst) {
        par(T, [&](uint32_t t, uint32_t TT) {
            for (uint32_t b = t; b < NB; b += TT)
                for (uint64_t i = 0; i < ulen[b]; ++i) {
                    const uint64_t k = out[boff[b] + i];
                    src[uoff[b] + i] = (uint32_t)(k >> 32);
                    dst[uoff[b] + i] = (uint32_t)k;
                }
        });
    }
    return uoff[NB];
}
}  // namespace

extern "C" uint32_t fgo_get_threads(void);

extern "C" {

uint64_t fgo_splitmix64(uint64_t x) { return sm64(x); }

uint64_t fgo_version_of(uint64_t seed, uint32_t slot) {
    return (sm64(seed ^ (uint64_t)slot) & kVersionMask) | 1ull;
}

uint64_t fgo_gen_layered(uint32_t levels, uint32_t width, uint32_t fanout, uint64_t seed,
                         uint32_t* src, uint32_t* dst) {
    if (levels < 2 || width == 0) return 0;
    if (fanout > width) fanout = width;
    const uint64_t m = (uint64_t)(levels - 1) * width * fanout;
    if (!src || !dst) return m;
    std::vector<uint64_t> keys;
    keys.reserve(m);
    std::vector<uint32_t> chosen;
    for (uint32_t l = 1; l < levels; ++l) {
        for (uint32_t i = 0; i < width; ++i) {
            chosen.clear();
            for (uint64_t attempt = 0; chosen.size() < fanout; ++attempt) {
                const uint64_t key = ((uint64_t)l << 56) ^ ((uint64_t)i << 20) ^ attempt;
                const uint32_t j = (uint32_t)(sm64(seed ^ sm64(key)) % width);
                if (std::find(chosen.begin(), chosen.end(), j) == chosen.end()) chosen.push_back(j);
            }
            for (uint32_t j : chosen) {
                const uint64_t s = (uint64_t)(l - 1) * width + j;
                const uint64_t d = (uint64_t)l * width + i;
                keys.push_back((s << 32) | d);
            }
        }
    }
    return finish(keys, src, dst);
}

uint64_t fgo_gen_rmat(uint32_t scale, uint32_t edge_factor, uint64_t seed, uint32_t* src, uint32_t* dst) {
    const uint64_t m = (uint64_t)edge_factor << scale;
    // quadrant thresholds on 53-bit uniforms: a = 0.57, a+b = 0.76, a+b+c = 0.95
    const uint64_t one = 1ull << 53;
    const uint64_t tA = one / 100 * 57, tAB = one / 100 * 76, tABC = one / 100 * 95;
    const uint64_t ks = sm64(seed);
    const uint32_t T = fgo_get_threads();
    std::vector<uint64_t> keys(m);
    par(T, [&](uint32_t t, uint32_t TT) {
    for (uint64_t i = m * t / TT; i < m * (t + 1) / TT; ++i) {
        uint64_t s = 0, d = 0;
        for (uint32_t l = 0; l < scale; ++l) {
            const uint64_t u = sm64(ks ^ ((i << 6) | l)) >> 11;
            const uint64_t bit = 1ull << (scale - 1 - l);
            if (u < tA) {
            } else if (u < tAB) {
                d |= bit;
            } else if (u < tABC) {
                s |= bit;
            } else {
                s |= bit;
                d |= bit;
            }
        }
        const uint64_t ps = scramble(s, scale, seed), pd = scramble(d, scale, seed);
        keys[i] = (ps << 32) | pd;
    }
    });
    return T > 1 ? finish_parallel(keys, scale, T, src, dst) : finish(keys, src, dst);
}

void fgo_gen_tags(uint64_t m, const uint32_t* src, const uint32_t* dst, uint64_t ver_seed,
                  uint32_t stale_pct, uint64_t stale_seed, uint64_t* tag) {
    par(fgo_get_threads(), [&](uint32_t t, uint32_t T) {
        for (uint64_t e = m * t / T; e < m * (t + 1) / T; ++e) {
            uint64_t v = fgo_version_of(ver_seed, dst[e]);
            if (stale_pct) {
                const uint64_t h = sm64(stale_seed ^ sm64(((uint64_t)src[e] << 32) | dst[e]));
                if (h % 100 < stale_pct) v += 1;
            }
            tag[e] = v;
        }
    });
}

uint32_t fgo_gen_roots(uint32_t n_roots, uint32_t range, uint64_t seed, const uint32_t* out_degree,
                       uint32_t* roots) {
    std::vector<uint8_t> taken(range, 0);
    uint32_t n = 0;
    const uint64_t limit = (uint64_t)range * 64 + 1024;
    for (uint64_t k = 0; n < n_roots && k < limit; ++k) {
        const uint32_t c = (uint32_t)(sm64(seed + k) % range);
        if (taken[c] || (out_degree && out_degree[c] == 0)) continue;
        taken[c] = 1;
        roots[n++] = c;
    }
    return n;
}

}  // extern "C"
