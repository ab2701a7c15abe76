// wave.hip — batched multi-root invalidation as a level-synchronous frontier BFS on gfx950.
//
// Restates the cascade of Computed<T>.Invalidate (src/Stl.Fusion/Computed.cs:162-230):
//   visit(dst, tag): the dst slot's current node n exists and n.Version == tag
//                    (Computed.cs:213-214, ComputedInput.GetExistingComputed) ->
//     Invalidated              : no-op                                  (164-165, 171-172)
//     Computing                : flags |= InvalidateOnSetOutput          (173-178)
//     Consistent, hasDelay     : flags |= InvalidationDelayStarted once  (186-191; timer host-side)
//     Consistent, no delay     : state := Invalidated, expand every `_usedBy` entry (185, 212-216)
// Each rule is one 64-bit CAS on the packed node word, so a node is invalidated (and expanded)
// exactly once however many frontier edges reach it. The union over roots is order-independent
// (DESIGN.md §Semantics), so one BFS wave replaces the reference's sequence of per-root DFS.
//
// Per level L (all launches stream-ordered, no host round trip inside a group of levels):
//   k_scan_reduce / k_scan_apply : exclusive scan of the frontier's row lengths (two passes over
//                                  4 B/entry), chunk->first-entry map for load balancing
//   k_expand                     : edge-parallel expansion, kChunk edges per block iteration;
//                                  each edge: col (4 B) + tag (8 B) streamed non-temporally,
//                                  node word (8 B) gathered, CAS on a version match. Winners are
//                                  appended (wave-aggregated atomics) to the invalidated list and,
//                                  with their row, to the next frontier.
#include <hip/hip_runtime.h>

#include <chrono>

#include "fgi_internal.h"

namespace fgi {
namespace {

__device__ __forceinline__ uint32_t lane_id() { return __lane_id(); }

// CAS state transition of one node word; w is a (possibly stale) observed value with the right
// version. Returns 1 if this call moved Consistent -> Invalidated, 2 if it only set a flag.
__device__ __forceinline__ int visit_word(unsigned long long* p, unsigned long long w, bool imm) {
    while (true) {
        const uint32_t st = word_state(w);
        unsigned long long nw;
        if (st == FGI_INVALIDATED) return 0;
        if (st == FGI_COMPUTING) {
            nw = w | kW_IOSO | (imm ? kW_DS : 0ull);
            if (nw == w) return 0;
        } else if (imm || !(w & kW_HasDelay)) {
            nw = (w & (kVMask | kW_HasDelay)) | kW_Invalidated;   // canonical: flags cleared
        } else {
            if (w & kW_DS) return 0;
            nw = w | kW_DS;
        }
        const unsigned long long prev = atomicCAS(p, w, nw);
        if (prev == w) return word_state(nw) == FGI_INVALIDATED ? 1 : 2;
        w = prev;
    }
}

__device__ __forceinline__ uint32_t wave_excl_scan(uint32_t v, uint32_t& total) {
    const uint32_t lane = lane_id();
    uint32_t x = v;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        const uint32_t y = __shfl_up(x, d, 64);
        if (lane >= (uint32_t)d) x += y;
    }
    total = __shfl(x, 63, 64);
    return x - v;
}

__device__ __forceinline__ uint32_t wave_sum(uint32_t v) {
#pragma unroll
    for (int d = 32; d >= 1; d >>= 1) v += __shfl_xor(v, d, 64);
    return v;
}

// Reserve `n_inv` slots in the invalidated list and `n_fr` in the next frontier for this lane;
// one atomic per list per wave. Returns the lane's bases.
__device__ __forceinline__ void wave_reserve(uint32_t n_inv, uint32_t n_fr, unsigned long long* inv_ctr,
                                             unsigned long long* fr_ctr, uint64_t& inv_base,
                                             uint64_t& fr_base) {
    uint32_t tot;
    const uint32_t packed = n_inv | (n_fr << 16);
    const uint32_t ex = wave_excl_scan(packed, tot);
    const uint32_t lane = lane_id();
    unsigned long long b_inv = 0, b_fr = 0;
    if (lane == 0 && (tot & 0xFFFFu)) b_inv = atomicAdd(inv_ctr, (unsigned long long)(tot & 0xFFFFu));
    if (lane == 0 && (tot >> 16)) b_fr = atomicAdd(fr_ctr, (unsigned long long)(tot >> 16));
    b_inv = __shfl(b_inv, 0, 64);
    b_fr = __shfl(b_fr, 0, 64);
    inv_base = b_inv + (ex & 0xFFFFu);
    fr_base = b_fr + (ex >> 16);
}

// ---- roots (level 0) ------------------------------------------------------------------------
// Roots are resolved like ComputedExt.TryUseExisting (Internal/ComputedExt.cs:25-35): the
// handle's current node, no tag check; immediately[i] selects Invalidate(true).
__global__ __launch_bounds__(kBlock) void k_roots(const uint32_t* __restrict__ roots,
                                                  const uint8_t* __restrict__ imm, uint32_t n,
                                                  uint32_t n_handles, unsigned long long* node,
                                                  const uint64_t* __restrict__ row_off,
                                                  const uint32_t* __restrict__ row_len,
                                                  uint32_t* __restrict__ inv, uint64_t* __restrict__ fr_off,
                                                  uint32_t* __restrict__ fr_len, WaveCtr* ctr) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    uint32_t win = 0, flagged = 0, h = 0, len = 0;
    uint64_t off = 0;
    if (i < n) {
        h = roots[i];
        if (h < n_handles) {
            const unsigned long long w = node[h];
            if ((w & kVMask) != 0) {
                const int r = visit_word(node + h, w, imm ? imm[i] != 0 : false);
                if (r == 1) {
                    win = 1;
                    len = row_len[h];
                    off = row_off[h];
                } else if (r == 2) {
                    flagged = 1;
                }
            }
        }
    }
    uint64_t ib, fb;
    const uint32_t has_row = (win && len) ? 1u : 0u;
    wave_reserve(win, has_row, &ctr->inv, &ctr->lvl[0].F, ib, fb);
    if (win) inv[ib] = h;
    if (has_row) {
        fr_off[fb] = off;
        fr_len[fb] = len;
    }
    const uint32_t fs = wave_sum(flagged), ws = wave_sum(win);
    if (lane_id() == 0 && fs) atomicAdd(&ctr->n_flagged, (unsigned long long)fs);
    if (lane_id() == 0 && ws) atomicAdd(&ctr->root_inv, (unsigned long long)ws);
}

// ---- frontier scan ----------------------------------------------------------------------------
__device__ __forceinline__ unsigned long long block_sum(unsigned long long v, unsigned long long* s_red) {
#pragma unroll
    for (int d = 32; d >= 1; d >>= 1) v += __shfl_xor(v, d, 64);
    const int wid = threadIdx.x >> 6;
    __syncthreads();
    if (lane_id() == 0) s_red[wid] = v;
    __syncthreads();
    unsigned long long t = 0;
    for (int k = 0; k < (int)(blockDim.x >> 6); ++k) t += s_red[k];
    return t;
}

__global__ __launch_bounds__(kBlock) void k_scan_reduce(int L, const uint32_t* __restrict__ fr_len,
                                                        unsigned long long* __restrict__ partials,
                                                        WaveCtr* ctr) {
    __shared__ unsigned long long s_red[kBlock / 64];
    const uint64_t F = ctr->lvl[L % kRing].F;
    const uint64_t b = blockIdx.x, G = gridDim.x;
    const uint64_t lo = F * b / G, hi = F * (b + 1) / G;
    unsigned long long s = 0;
    for (uint64_t i = lo + threadIdx.x; i < hi; i += blockDim.x) s += fr_len[i];
    s = block_sum(s, s_red);
    if (threadIdx.x == 0) partials[b] = s;
}

// Exclusive scan of fr_len into escan; records for every chunk of kChunk edges the frontier
// entry holding its first edge (cstart), and the level's edge total.
__global__ __launch_bounds__(kBlock) void k_scan_apply(int L, const uint32_t* __restrict__ fr_len,
                                                       const unsigned long long* __restrict__ partials,
                                                       uint64_t* __restrict__ escan, uint32_t* __restrict__ cstart,
                                                       WaveCtr* ctr) {
    __shared__ unsigned long long s_red[kBlock / 64];
    __shared__ unsigned long long s_wave[kBlock / 64];
    LevelCtr& lc = ctr->lvl[L % kRing];
    const uint64_t F = lc.F;
    const uint64_t b = blockIdx.x, G = gridDim.x;
    // prefix of partials before this block, and the grand total
    unsigned long long before = 0, all = 0;
    for (uint64_t k = threadIdx.x; k < G; k += blockDim.x) {
        const unsigned long long p = partials[k];
        all += p;
        if (k < b) before += p;
    }
    before = block_sum(before, s_red);
    all = block_sum(all, s_red);
    if (b == 0 && threadIdx.x == 0) {
        lc.T = all;
        lc.nchunks = (all + kChunk - 1) / kChunk;
    }
    if (F == 0) return;
    const uint64_t lo = F * b / G, hi = F * (b + 1) / G;
    unsigned long long run = before;
    const uint32_t lane = lane_id(), wid = threadIdx.x >> 6;
    for (uint64_t base = lo; base < hi; base += blockDim.x) {
        const uint64_t i = base + threadIdx.x;
        const unsigned long long v = (i < hi) ? fr_len[i] : 0ull;
        // inclusive wave scan (64-bit)
        unsigned long long x = v;
#pragma unroll
        for (int d = 1; d < 64; d <<= 1) {
            const unsigned long long y = __shfl_up(x, d, 64);
            if (lane >= (uint32_t)d) x += y;
        }
        __syncthreads();
        if (lane == 63) s_wave[wid] = x;
        __syncthreads();
        unsigned long long woff = 0, tile = 0;
        for (uint32_t k = 0; k < (blockDim.x >> 6); ++k) {
            const unsigned long long t = s_wave[k];
            if (k < wid) woff += t;
            tile += t;
        }
        const unsigned long long es = run + woff + x - v;
        if (i < hi) {
            escan[i] = es;
            const unsigned long long c_lo = (es + kChunk - 1) / kChunk;
            const unsigned long long c_hi = (es + v - 1) / kChunk;
            for (unsigned long long c = c_lo; c <= c_hi; ++c) cstart[c] = (uint32_t)i;
        }
        run += tile;
    }
}

// ---- expansion --------------------------------------------------------------------------------
__device__ __forceinline__ uint32_t lds_upper_bound(const uint32_t* s, uint32_t n, uint32_t x) {
    uint32_t lo = 0, hi = n;   // first k with s[k] > x
    while (lo < hi) {
        const uint32_t mid = (lo + hi) >> 1;
        if (s[mid] <= x) lo = mid + 1;
        else hi = mid;
    }
    return lo;
}

__global__ __launch_bounds__(kBlock) void k_expand(int L, const uint64_t* __restrict__ fr_off,
                                                   const uint64_t* __restrict__ escan,
                                                   const uint32_t* __restrict__ cstart,
                                                   const uint32_t* __restrict__ pool_col,
                                                   const uint64_t* __restrict__ pool_tag,
                                                   unsigned long long* node, const uint64_t* __restrict__ row_off,
                                                   const uint32_t* __restrict__ row_len,
                                                   uint32_t* __restrict__ inv, uint64_t* __restrict__ nfr_off,
                                                   uint32_t* __restrict__ nfr_len, WaveCtr* ctr) {
    __shared__ uint32_t s_rel[kChunk + 1];
    __shared__ uint64_t s_base[kChunk + 1];
    LevelCtr& lc = ctr->lvl[L % kRing];
    LevelCtr& ln = ctr->lvl[(L + 1) % kRing];
    if (blockIdx.x == 0 && threadIdx.x < sizeof(LevelCtr) / 8)
        reinterpret_cast<unsigned long long*>(&ctr->lvl[(L + 2) % kRing])[threadIdx.x] = 0ull;
    const uint64_t T = lc.T, F = lc.F, nch = lc.nchunks;
    uint32_t matched = 0, flagged = 0;
    for (uint64_t c = blockIdx.x; c < nch; c += gridDim.x) {
        const uint64_t cbase = c * kChunk;
        const uint32_t clen = (uint32_t)((T - cbase) < (uint64_t)kChunk ? (T - cbase) : (uint64_t)kChunk);
        const uint32_t i0 = cstart[c];
        const uint32_t i1 = (c + 1 < nch) ? cstart[c + 1] : (uint32_t)(F - 1);
        const uint32_t n = i1 - i0 + 1;
        for (uint32_t k = threadIdx.x; k < n; k += kBlock) {
            const uint64_t es = escan[i0 + k];
            s_rel[k] = es > cbase ? (uint32_t)(es - cbase) : 0u;
            s_base[k] = fr_off[i0 + k] + cbase - es;
        }
        __syncthreads();
        uint32_t dst[kEPT];
        uint64_t tag[kEPT];
#pragma unroll
        for (int j = 0; j < kEPT; ++j) {
            const uint32_t local = threadIdx.x + j * kBlock;
            dst[j] = 0xFFFFFFFFu;
            tag[j] = 0;
            if (local < clen) {
                const uint32_t k = lds_upper_bound(s_rel, n, local) - 1;
                const uint64_t p = s_base[k] + local;
                dst[j] = __builtin_nontemporal_load(pool_col + p);
                tag[j] = __builtin_nontemporal_load(pool_tag + p);
            }
        }
        unsigned long long w[kEPT];
#pragma unroll
        for (int j = 0; j < kEPT; ++j) w[j] = (dst[j] != 0xFFFFFFFFu) ? node[dst[j]] : 0ull;
        uint32_t win_mask = 0;
#pragma unroll
        for (int j = 0; j < kEPT; ++j) {
            if (tag[j] != 0 && (w[j] & kVMask) == tag[j]) {
                ++matched;
                const int r = visit_word(node + dst[j], w[j], false);
                if (r == 1) win_mask |= 1u << j;
                else if (r == 2) ++flagged;
            }
        }
        uint32_t lens[kEPT];
        uint64_t offs[kEPT];
        uint32_t n_inv = 0, n_fr = 0;
#pragma unroll
        for (int j = 0; j < kEPT; ++j) {
            lens[j] = 0;
            offs[j] = 0;
            if (win_mask & (1u << j)) {
                lens[j] = row_len[dst[j]];
                offs[j] = row_off[dst[j]];
                ++n_inv;
                if (lens[j]) ++n_fr;
            }
        }
        uint64_t ib, fb;
        wave_reserve(n_inv, n_fr, &ctr->inv, &ln.F, ib, fb);
#pragma unroll
        for (int j = 0; j < kEPT; ++j) {
            if (win_mask & (1u << j)) {
                inv[ib++] = dst[j];
                if (lens[j]) {
                    nfr_off[fb] = offs[j];
                    nfr_len[fb] = lens[j];
                    ++fb;
                }
            }
        }
        __syncthreads();
    }
    const uint32_t ms = wave_sum(matched), fs = wave_sum(flagged);
    if (lane_id() == 0) {
        if (ms) atomicAdd(&ctr->e_match, (unsigned long long)ms);
        if (fs) atomicAdd(&ctr->n_flagged, (unsigned long long)fs);
    }
}

}  // namespace

fgi_status run_wave(fgi_graph* g, uint32_t n_roots, const uint32_t* roots_dev, const uint8_t* imm_dev,
                    fgi_wave_stats* stats) {
    const auto t0 = std::chrono::steady_clock::now();
    hipStream_t s = g->stream;
    FGI_TRY(ensure_cstart(g, g->pool_top));
    FGI_HIP(g, hipMemsetAsync(g->ctr, 0, sizeof(WaveCtr), s));
    const bool timing = stats != nullptr;
    if (timing) FGI_HIP(g, hipEventRecord(g->ev_w0, s));
    if (n_roots) {
        const uint32_t nb = (n_roots + kBlock - 1) / kBlock;
        hipLaunchKernelGGL(k_roots, dim3(nb), dim3(kBlock), 0, s, roots_dev, imm_dev, n_roots, g->n_handles,
                           reinterpret_cast<unsigned long long*>(g->node), g->row_off, g->row_len, g->inv,
                           g->fr_off[0], g->fr_len[0], g->ctr);
    }
    // Persistent grid for the expansion: 6 resident 256-thread blocks per CU (LDS 24.6 KB each).
    int n_cu = 256;
    hipDeviceGetAttribute(&n_cu, hipDeviceAttributeMultiprocessorCount, g->device);
    const uint32_t expand_grid = (uint32_t)n_cu * 6;
    constexpr int kGroup = 4;
    int L = 0;
    uint64_t levels = 0, e_trav = 0, f_total = 0;
    double expand_ms = 0;
    uint64_t expand_launches = 0;
    bool done = (n_roots == 0);
    std::vector<int> ev_level;
    while (!done) {
        const int L0 = L;
        for (int k = 0; k < kGroup; ++k, ++L) {
            const int buf = L & 1;
            hipLaunchKernelGGL(k_scan_reduce, dim3(kScanBlocks), dim3(kBlock), 0, s, L, g->fr_len[buf], g->partials,
                               g->ctr);
            hipLaunchKernelGGL(k_scan_apply, dim3(kScanBlocks), dim3(kBlock), 0, s, L, g->fr_len[buf], g->partials,
                               g->escan, g->cstart, g->ctr);
            if (timing) {
                while (g->ev.size() < 2 * (size_t)(L + 1)) {
                    hipEvent_t e;
                    FGI_HIP(g, hipEventCreate(&e));
                    g->ev.push_back(e);
                }
                FGI_HIP(g, hipEventRecord(g->ev[2 * L], s));
            }
            hipLaunchKernelGGL(k_expand, dim3(expand_grid), dim3(kBlock), 0, s, L, g->fr_off[buf], g->escan, g->cstart,
                               g->pool_col, g->pool_tag, reinterpret_cast<unsigned long long*>(g->node), g->row_off,
                               g->row_len, g->inv, g->fr_off[buf ^ 1], g->fr_len[buf ^ 1], g->ctr);
            if (timing) FGI_HIP(g, hipEventRecord(g->ev[2 * L + 1], s));
        }
        FGI_HIP(g, hipGetLastError());
        FGI_HIP(g, hipMemcpyAsync(g->ctr_host, g->ctr, sizeof(WaveCtr), hipMemcpyDeviceToHost, s));
        FGI_HIP(g, hipStreamSynchronize(s));
        for (int l = L0; l < L; ++l) {
            const LevelCtr& lc = g->ctr_host->lvl[l % kRing];
            if (lc.F) {
                ++levels;
                e_trav += lc.T;
                f_total += lc.F;
                if (timing) {
                    float ms = 0;
                    FGI_HIP(g, hipEventElapsedTime(&ms, g->ev[2 * l], g->ev[2 * l + 1]));
                    expand_ms += ms;
                    ++expand_launches;
                }
            }
        }
        if (g->ctr_host->lvl[L % kRing].F == 0) done = true;
    }
    if (n_roots == 0) {
        FGI_HIP(g, hipMemcpyAsync(g->ctr_host, g->ctr, sizeof(WaveCtr), hipMemcpyDeviceToHost, s));
        FGI_HIP(g, hipStreamSynchronize(s));
    }
    if (timing) {
        FGI_HIP(g, hipEventRecord(g->ev_w1, s));
        FGI_HIP(g, hipEventSynchronize(g->ev_w1));
    }
    g->last_wave_n = g->ctr_host->inv;
    if (stats) {
        const uint64_t v = g->ctr_host->inv;
        stats->roots += n_roots;
        stats->levels += levels;
        stats->v_inv += v;
        stats->e_trav += e_trav;
        stats->e_match += g->ctr_host->e_match;
        stats->n_flagged += g->ctr_host->n_flagged;
        // Algorithmic bytes of the wave:
        //   per traversed edge     20 B  (col 4 + tag 8 + node-word gather 8)
        //   per frontier entry     44 B  (fr_len 4 x2 scan passes, escan 8 w + 8 r, fr_off 8 r,
        //                                 frontier write 12 by the producer)
        //   per invalidated node   24 B  (CAS 8 + row_len/row_off gather 12 + list write 4)
        //   per root                5 B
        stats->alg_bytes += 20 * e_trav + 44 * f_total + 24 * v + 5ull * n_roots;
        float wave_ms = 0;
        hipEventElapsedTime(&wave_ms, g->ev_w0, g->ev_w1);
        stats->kernel_ms += wave_ms;
        stats->expand_ms += expand_ms;
        stats->expand_launches += expand_launches;
        // expand kernel alone: edges 20 B, frontier entries read 16 B (escan + fr_off), winners
        // 24 B (CAS + row gathers + list write), next-frontier entries written 12 B.
        const uint64_t v_exp = v - g->ctr_host->root_inv;
        const uint64_t f0 = g->ctr_host->lvl[0].F;   // level-0 frontier is written by k_roots
        stats->expand_bytes += 20 * e_trav + 16 * f_total + 24 * v_exp + 12 * (f_total - f0);
        stats->f_total += f_total;
        stats->total_ms += std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    }
    return FGI_OK;
}

}  // namespace fgi
