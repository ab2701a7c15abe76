// wave.hip — batched multi-root invalidation as a level-synchronous, direction-optimizing BFS.
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
// Per level L (stream-ordered launches; the host only synchronises once per group of levels):
//   k_scan_reduce / k_scan_apply : exclusive scan of the frontier's row lengths, chunk->entry map,
//                                  level edge total, and the push/pull decision for the level
//   k_mark                       : the previous level's winners -> dead bitmap (+ frontier bitmap)
//   k_expand  (push levels)      : edge-parallel expansion of the frontier's `_usedBy` rows;
//                                  edges to nodes already dead skip the tag load and the gather
//   k_pull / k_pull_long (pull)  : every live slot scans its dependency list (the reference's
//                                  `_used`: in-edges whose tag matches its version) for a parent
//                                  in the frontier bitmap, with early exit (Beamer's bottom-up step)
//   k_clear_front                : reset the frontier bitmap
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>

#include "fgi_internal.h"

namespace fgi {
namespace {

constexpr uint32_t kPullCap = 16;   // in-list entries a k_pull thread scans before handing off

__device__ __forceinline__ uint32_t lane_id() { return __lane_id(); }

__device__ __forceinline__ bool bit_of(const uint32_t* __restrict__ bm, uint32_t h) {
    return (bm[h >> 5] >> (h & 31)) & 1u;
}

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
// one atomic per list per wave. Every lane of the wave must call it.
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

// Append one (possibly absent) winner per lane: invalidated list + next frontier with its row.
__device__ __forceinline__ void emit_one(bool win, uint32_t h, const uint64_t* __restrict__ row_off,
                                         const uint32_t* __restrict__ row_len, uint32_t* __restrict__ inv,
                                         uint64_t* __restrict__ nfr_off, uint32_t* __restrict__ nfr_len,
                                         unsigned long long* inv_ctr, unsigned long long* fr_ctr) {
    uint32_t len = 0;
    uint64_t off = 0;
    if (win) {
        len = row_len[h];
        off = row_off[h];
    }
    uint64_t ib, fb;
    wave_reserve(win ? 1u : 0u, (win && len) ? 1u : 0u, inv_ctr, fr_ctr, ib, fb);
    if (win) inv[ib] = h;
    if (win && len) {
        nfr_off[fb] = off;
        nfr_len[fb] = len;
    }
}

// Block-level emission: winners are staged in LDS and appended to the global lists in batches
// (one pair of global atomics per batch instead of one per wave per iteration: the two list
// counters are single words, and same-address atomics saturate at ~88/us chip-wide).
constexpr uint32_t kEmitCap = 1024;
struct Emit {
    uint32_t n;
    uint32_t pad;
    unsigned long long base_inv, base_fr;
    uint32_t wsum[kBlock / 64];
    uint32_t h[kEmitCap];
};

__device__ __forceinline__ void emit_init(Emit& e) {
    if (threadIdx.x == 0) e.n = 0;
    __syncthreads();
}

// Every lane of the calling wave must call it (ballot); lanes beyond the LDS capacity fall back
// to direct appends.
__device__ __forceinline__ void emit_push(Emit& e, bool win, uint32_t h, const uint64_t* __restrict__ row_off,
                                          const uint32_t* __restrict__ row_len, uint32_t* __restrict__ inv,
                                          uint64_t* __restrict__ nfr_off, uint32_t* __restrict__ nfr_len,
                                          unsigned long long* inv_ctr, unsigned long long* fr_ctr) {
    const unsigned long long m = __ballot(win);
    if (!m) return;
    uint32_t base = 0;
    if (lane_id() == 0) base = atomicAdd(&e.n, (uint32_t)__popcll(m));
    base = __shfl(base, 0, 64);
    if (win) {
        const uint32_t idx = base + (uint32_t)__popcll(m & ((1ull << lane_id()) - 1ull));
        if (idx < kEmitCap) {
            e.h[idx] = h;
        } else {
            inv[atomicAdd(inv_ctr, 1ull)] = h;
            const uint32_t len = row_len[h];
            if (len) {
                const unsigned long long fb = atomicAdd(fr_ctr, 1ull);
                nfr_off[fb] = row_off[h];
                nfr_len[fb] = len;
            }
        }
    }
}

// Block-uniform call. Flushes when at least `at` winners are staged (at = 1: flush anything).
__device__ __forceinline__ void emit_flush(Emit& e, uint32_t at, const uint64_t* __restrict__ row_off,
                                           const uint32_t* __restrict__ row_len, uint32_t* __restrict__ inv,
                                           uint64_t* __restrict__ nfr_off, uint32_t* __restrict__ nfr_len,
                                           unsigned long long* inv_ctr, unsigned long long* fr_ctr) {
    __syncthreads();
    const uint32_t n = e.n < kEmitCap ? e.n : kEmitCap;
    __syncthreads();   // every thread has read e.n before any wave can push again
    if (n < at || n == 0) return;   // uniform decision
    constexpr int kPer = kEmitCap / kBlock;
    uint32_t hh[kPer], len[kPer];
    uint64_t off[kPer];
    uint32_t cnt = 0;
#pragma unroll
    for (int k = 0; k < kPer; ++k) {
        const uint32_t i = threadIdx.x + k * kBlock;
        hh[k] = 0;
        len[k] = 0;
        off[k] = 0;
        if (i < n) {
            hh[k] = e.h[i];
            len[k] = row_len[hh[k]];
            off[k] = row_off[hh[k]];
            cnt += len[k] ? 1u : 0u;
        }
    }
    uint32_t wtot;
    const uint32_t wex = wave_excl_scan(cnt, wtot);
    const uint32_t wid = threadIdx.x >> 6;
    if (lane_id() == 0) e.wsum[wid] = wtot;
    __syncthreads();
    uint32_t before = 0, total = 0;
    for (uint32_t k = 0; k < kBlock / 64; ++k) {
        if (k < wid) before += e.wsum[k];
        total += e.wsum[k];
    }
    if (threadIdx.x == 0) {
        e.base_inv = atomicAdd(inv_ctr, (unsigned long long)n);
        e.base_fr = total ? atomicAdd(fr_ctr, (unsigned long long)total) : 0ull;
    }
    __syncthreads();
    uint64_t fb = e.base_fr + before + wex;
#pragma unroll
    for (int k = 0; k < kPer; ++k) {
        const uint32_t i = threadIdx.x + k * kBlock;
        if (i < n) {
            inv[e.base_inv + i] = hh[k];
            if (len[k]) {
                nfr_off[fb] = off[k];
                nfr_len[fb] = len[k];
                ++fb;
            }
        }
    }
    __syncthreads();
    if (threadIdx.x == 0) e.n = 0;
    __syncthreads();
}

// ---- multi-GPU: remote targets staged per block and bucketed by owner ------------------------
constexpr uint32_t kMaxWorld = 8;
constexpr uint32_t kMsgCap = 1024;
struct RemoteArgs {
    uint32_t base, n_local, block, world;
    const uint64_t* ver_all;
    uint32_t* sent_bm;
    uint32_t* send_buf;
    unsigned long long* send_cnt;
};
template <bool PART> struct MsgEmit {
    uint32_t n;
    uint32_t cnt[kMaxWorld], cur[kMaxWorld];
    unsigned long long base[kMaxWorld];
    uint32_t d[kMsgCap];
};
template <> struct MsgEmit<false> {
    uint32_t n;
};

__device__ __forceinline__ void msg_push(MsgEmit<true>& me, bool send, uint32_t dst, const RemoteArgs& ra) {
    const unsigned long long m = __ballot(send);
    if (!m) return;
    uint32_t base = 0;
    if (lane_id() == 0) base = atomicAdd(&me.n, (uint32_t)__popcll(m));
    base = __shfl(base, 0, 64);
    if (send) {
        const uint32_t idx = base + (uint32_t)__popcll(m & ((1ull << lane_id()) - 1ull));
        if (idx < kMsgCap) {
            me.d[idx] = dst;
        } else {
            const uint32_t q = dst / ra.block;
            ra.send_buf[(uint64_t)q * ra.block + atomicAdd(&ra.send_cnt[q], 1ull)] = dst;
        }
    }
}

__device__ __forceinline__ void msg_flush(MsgEmit<true>& me, uint32_t at, const RemoteArgs& ra) {
    __syncthreads();
    const uint32_t n = me.n < kMsgCap ? me.n : kMsgCap;
    if (threadIdx.x < kMaxWorld) {
        me.cnt[threadIdx.x] = 0;
        me.cur[threadIdx.x] = 0;
    }
    __syncthreads();
    if (n < at || n == 0) return;
    for (uint32_t i = threadIdx.x; i < n; i += blockDim.x) atomicAdd(&me.cnt[me.d[i] / ra.block], 1u);
    __syncthreads();
    if (threadIdx.x < ra.world && me.cnt[threadIdx.x])
        me.base[threadIdx.x] = atomicAdd(&ra.send_cnt[threadIdx.x], (unsigned long long)me.cnt[threadIdx.x]);
    __syncthreads();
    for (uint32_t i = threadIdx.x; i < n; i += blockDim.x) {
        const uint32_t dst = me.d[i], q = dst / ra.block;
        ra.send_buf[(uint64_t)q * ra.block + me.base[q] + atomicAdd(&me.cur[q], 1u)] = dst;
    }
    __syncthreads();
    if (threadIdx.x == 0) me.n = 0;
    __syncthreads();
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
    uint32_t win = 0, flagged = 0, h = 0;
    if (i < n) {
        h = roots[i];
        if (h < n_handles) {
            const unsigned long long w = node[h];
            if ((w & kVMask) != 0) {
                const int r = visit_word(node + h, w, imm ? imm[i] != 0 : false);
                win = (r == 1);
                flagged = (r == 2);
            }
        }
    }
    emit_one(win, h, row_off, row_len, inv, fr_off, fr_len, &ctr->inv, &ctr->lvl[0].F);
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
// entry holding its first edge (cstart), the level's edge total, and push-vs-pull.
__global__ __launch_bounds__(kBlock) void k_scan_apply(int L, const uint32_t* __restrict__ fr_len,
                                                       const unsigned long long* __restrict__ partials,
                                                       uint64_t* __restrict__ escan, uint32_t* __restrict__ cstart,
                                                       WaveCtr* ctr, int direction, uint64_t pull_threshold) {
    __shared__ unsigned long long s_red[kBlock / 64];
    __shared__ unsigned long long s_wave[kBlock / 64];
    LevelCtr& lc = ctr->lvl[L % kRing];
    const uint64_t F = lc.F;
    const uint64_t b = blockIdx.x, G = gridDim.x;
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
        // direction: 1 push only, 2 pull only, 0 auto (pull when the frontier's rows are heavy)
        lc.pull = (F != 0 && (direction == 2 || (direction == 0 && all > pull_threshold))) ? 1ull : 0ull;
    }
    if (F == 0) return;
    const uint64_t lo = F * b / G, hi = F * (b + 1) / G;
    unsigned long long run = before;
    const uint32_t lane = lane_id(), wid = threadIdx.x >> 6;
    for (uint64_t base = lo; base < hi; base += blockDim.x) {
        const uint64_t i = base + threadIdx.x;
        const unsigned long long v = (i < hi) ? fr_len[i] : 0ull;
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

// ---- bitmaps ----------------------------------------------------------------------------------
// Nodes that won Consistent -> Invalidated since the last mark become dead (and frontier, on pull
// levels). The range [marked, inv) is exactly the previous level's winners.
__global__ __launch_bounds__(kBlock) void k_mark(int L, const uint32_t* __restrict__ inv, uint32_t* dead_bm,
                                                 uint32_t* front_bm, WaveCtr* ctr) {
    LevelCtr& lc = ctr->lvl[L % kRing];
    const uint64_t lo = ctr->marked, hi = ctr->inv;
    if (blockIdx.x == 0 && threadIdx.x == 0) {
        lc.mark_lo = lo;
        lc.mark_hi = hi;
    }
    const bool front = lc.pull != 0;
    for (uint64_t i = lo + (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < hi;
         i += (uint64_t)gridDim.x * blockDim.x) {
        const uint32_t h = inv[i];
        atomicOr(dead_bm + (h >> 5), 1u << (h & 31));
        if (front) atomicOr(front_bm + (h >> 5), 1u << (h & 31));
    }
}

__global__ __launch_bounds__(kBlock) void k_clear_front(int L, const uint32_t* __restrict__ inv, uint32_t* front_bm,
                                                        WaveCtr* ctr) {
    LevelCtr& lc = ctr->lvl[L % kRing];
    const uint64_t lo = lc.mark_lo, hi = lc.mark_hi;
    if (blockIdx.x == 0 && threadIdx.x == 0) ctr->marked = hi;
    if (!lc.pull) return;
    for (uint64_t i = lo + (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < hi;
         i += (uint64_t)gridDim.x * blockDim.x)
        front_bm[inv[i] >> 5] = 0u;   // every set bit of the word belongs to this level's frontier
}

// ---- push: edge-parallel expansion ------------------------------------------------------------
__device__ __forceinline__ uint32_t lds_upper_bound(const uint32_t* s, uint32_t n, uint32_t x) {
    uint32_t lo = 0, hi = n;   // first k with s[k] > x
    while (lo < hi) {
        const uint32_t mid = (lo + hi) >> 1;
        if (s[mid] <= x) lo = mid + 1;
        else hi = mid;
    }
    return lo;
}

// PART: multi-GPU rank — dependant slots outside [ra.base, ra.base + ra.n_local) are remote: their
// tag is checked against the version replica and matching targets are forwarded once per wave.
template <bool PART>
__global__ __launch_bounds__(kBlock) void k_expand(int L, const uint64_t* __restrict__ fr_off,
                                                   const uint64_t* __restrict__ escan,
                                                   const uint32_t* __restrict__ cstart,
                                                   const uint32_t* __restrict__ pool_col,
                                                   const uint64_t* __restrict__ pool_tag,
                                                   unsigned long long* node, const uint64_t* __restrict__ row_off,
                                                   const uint32_t* __restrict__ row_len,
                                                   const uint32_t* __restrict__ dead_bm, int dead_filter,
                                                   uint32_t* __restrict__ inv, uint64_t* __restrict__ nfr_off,
                                                   uint32_t* __restrict__ nfr_len, WaveCtr* ctr, RemoteArgs ra) {
    __shared__ uint32_t s_rel[kChunk + 1];
    __shared__ uint64_t s_base[kChunk + 1];
    __shared__ Emit em;
    __shared__ MsgEmit<PART> me;
    LevelCtr& lc = ctr->lvl[L % kRing];
    LevelCtr& ln = ctr->lvl[(L + 1) % kRing];
    if (blockIdx.x == 0 && threadIdx.x < sizeof(LevelCtr) / 8)
        reinterpret_cast<unsigned long long*>(&ctr->lvl[(L + 2) % kRing])[threadIdx.x] = 0ull;
    if (lc.pull) return;
    emit_init(em);
    if constexpr (PART) {
        if (threadIdx.x == 0) me.n = 0;
    }
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
        uint64_t pos[kEPT];
#pragma unroll
        for (int j = 0; j < kEPT; ++j) {
            const uint32_t local = threadIdx.x + j * kBlock;
            dst[j] = 0xFFFFFFFFu;
            pos[j] = 0;
            if (local < clen) {
                const uint32_t k = lds_upper_bound(s_rel, n, local) - 1;
                pos[j] = s_base[k] + local;
                dst[j] = __builtin_nontemporal_load(pool_col + pos[j]);
            }
        }
        // remote dependants (PART): forwarded at most once per wave, only on a version match
        if constexpr (PART) {
#pragma unroll
            for (int j = 0; j < kEPT; ++j) {
                bool send = false;
                const uint32_t d = dst[j];
                if (d != 0xFFFFFFFFu && d - ra.base >= ra.n_local) {
                    if (!bit_of(ra.sent_bm, d)) {
                        const uint64_t t = __builtin_nontemporal_load(pool_tag + pos[j]);
                        if (t != 0 && ra.ver_all[d] == t) {
                            ++matched;
                            const uint32_t b = 1u << (d & 31);
                            send = !(atomicOr(ra.sent_bm + (d >> 5), b) & b);
                        }
                    }
                    dst[j] = 0xFFFFFFFFu;
                }
                msg_push(me, send, d, ra);
            }
#pragma unroll
            for (int j = 0; j < kEPT; ++j)
                if (dst[j] != 0xFFFFFFFFu) dst[j] -= ra.base;   // local handle
        }
        // edges to nodes invalidated in an earlier level need neither the tag nor the gather
        if (dead_filter) {
#pragma unroll
            for (int j = 0; j < kEPT; ++j)
                if (dst[j] != 0xFFFFFFFFu && bit_of(dead_bm, dst[j])) dst[j] = 0xFFFFFFFFu;
        }
        uint64_t tag[kEPT];
        unsigned long long w[kEPT];
#pragma unroll
        for (int j = 0; j < kEPT; ++j) {
            tag[j] = 0;
            w[j] = 0;
            if (dst[j] != 0xFFFFFFFFu) {
                tag[j] = __builtin_nontemporal_load(pool_tag + pos[j]);
                w[j] = node[dst[j]];
            }
        }
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
#pragma unroll
        for (int j = 0; j < kEPT; ++j)
            emit_push(em, (win_mask >> j) & 1u, dst[j], row_off, row_len, inv, nfr_off, nfr_len, &ctr->inv, &ln.F);
        emit_flush(em, kEmitCap / 2, row_off, row_len, inv, nfr_off, nfr_len, &ctr->inv, &ln.F);
        if constexpr (PART) msg_flush(me, kMsgCap / 2, ra);
    }
    emit_flush(em, 1, row_off, row_len, inv, nfr_off, nfr_len, &ctr->inv, &ln.F);
    if constexpr (PART) msg_flush(me, 1, ra);
    const uint32_t ms = wave_sum(matched), fs = wave_sum(flagged);
    if (lane_id() == 0) {
        if (ms) atomicAdd(&ctr->e_match, (unsigned long long)ms);
        if (fs) atomicAdd(&ctr->n_flagged, (unsigned long long)fs);
    }
}

// ---- pull: every live slot looks for a parent in the frontier ---------------------------------
// uin_* is the dependency-list cache: for slot d, the handles u whose `_usedBy` row holds
// (d, version(d)) — the reference's d._used (Computed.cs:36, 365-366). A parent in the frontier
// bitmap (u invalidated in the previous level) means the push step would visit d from u.
__global__ __launch_bounds__(kBlock) void k_pull(int L, uint32_t n_slots, const uint64_t* __restrict__ uin_off,
                                                 const uint32_t* __restrict__ uin_len,
                                                 const uint32_t* __restrict__ uin_src,
                                                 const uint32_t* __restrict__ dead_bm,
                                                 const uint32_t* __restrict__ front_bm, unsigned long long* node,
                                                 const uint64_t* __restrict__ row_off,
                                                 const uint32_t* __restrict__ row_len, uint32_t* __restrict__ inv,
                                                 uint64_t* __restrict__ nfr_off, uint32_t* __restrict__ nfr_len,
                                                 uint32_t* __restrict__ ovf, WaveCtr* ctr) {
    __shared__ Emit em;
    LevelCtr& lc = ctr->lvl[L % kRing];
    LevelCtr& ln = ctr->lvl[(L + 1) % kRing];
    if (!lc.pull) return;
    emit_init(em);
    uint32_t flagged = 0, cand = 0, examined = 0, live = 0, wins = 0;
    const uint32_t stride = gridDim.x * blockDim.x;
    const uint32_t n_iter = (n_slots + stride - 1) / stride;   // uniform trip count: flushes are block-wide
    for (uint32_t it = 0; it < n_iter; ++it) {
        const uint32_t d = it * stride + blockIdx.x * blockDim.x + threadIdx.x;
        bool win = false, long_list = false;
        if (d < n_slots && !bit_of(dead_bm, d)) {
            ++live;
            const uint32_t len = uin_len[d];
            if (len) {
                ++cand;
                const uint64_t off = uin_off[d];
                const uint32_t lim = len < kPullCap ? len : kPullCap;
                bool found = false;
                uint32_t k = 0;
                for (; k < lim; ++k) {
                    if (bit_of(front_bm, uin_src[off + k])) {
                        found = true;
                        ++k;
                        break;
                    }
                }
                examined += k;
                if (found) {
                    const int r = visit_word(node + d, node[d], false);
                    win = (r == 1);
                    flagged += (r == 2);
                } else if (len > kPullCap) {
                    long_list = true;
                }
            }
        }
        // long dependency lists continue in k_pull_long (one wave per node)
        const unsigned long long lm = __ballot(long_list);
        if (lm) {
            unsigned long long base = 0;
            if (lane_id() == 0) base = atomicAdd(&lc.ovf, (unsigned long long)__popcll(lm));
            base = __shfl(base, 0, 64);
            if (long_list) ovf[base + __popcll(lm & ((1ull << lane_id()) - 1ull))] = d;
        }
        wins += win ? 1u : 0u;
        emit_push(em, win, d, row_off, row_len, inv, nfr_off, nfr_len, &ctr->inv, &ln.F);
        emit_flush(em, kEmitCap - kBlock, row_off, row_len, inv, nfr_off, nfr_len, &ctr->inv, &ln.F);
    }
    emit_flush(em, 1, row_off, row_len, inv, nfr_off, nfr_len, &ctr->inv, &ln.F);
    const uint32_t fs = wave_sum(flagged), cs = wave_sum(cand), es = wave_sum(examined);
    const uint32_t ls = wave_sum(live), ws = wave_sum(wins);
    if (lane_id() == 0) {
        if (fs) atomicAdd(&ctr->n_flagged, (unsigned long long)fs);
        if (cs) atomicAdd(&ctr->pull_cand, (unsigned long long)cs);
        if (es) atomicAdd(&ctr->pull_edges, (unsigned long long)es);
        if (ls) atomicAdd(&ctr->pull_live, (unsigned long long)ls);
        if (ws) atomicAdd(&ctr->pull_win, (unsigned long long)ws);
    }
    if (blockIdx.x == 0 && threadIdx.x == 0) atomicAdd(&ctr->pull_scan, (unsigned long long)n_slots);
}

__global__ __launch_bounds__(kBlock) void k_pull_long(int L, const uint64_t* __restrict__ uin_off,
                                                      const uint32_t* __restrict__ uin_len,
                                                      const uint32_t* __restrict__ uin_src,
                                                      const uint32_t* __restrict__ front_bm, unsigned long long* node,
                                                      const uint64_t* __restrict__ row_off,
                                                      const uint32_t* __restrict__ row_len,
                                                      uint32_t* __restrict__ inv, uint64_t* __restrict__ nfr_off,
                                                      uint32_t* __restrict__ nfr_len,
                                                      const uint32_t* __restrict__ ovf, WaveCtr* ctr) {
    LevelCtr& lc = ctr->lvl[L % kRing];
    LevelCtr& ln = ctr->lvl[(L + 1) % kRing];
    if (!lc.pull) return;
    const uint64_t n = lc.ovf;
    const uint32_t lane = lane_id();
    const uint64_t wave0 = ((uint64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
    const uint64_t nwaves = ((uint64_t)gridDim.x * blockDim.x) >> 6;
    uint32_t flagged = 0, examined = 0;
    for (uint64_t q = wave0; q < n; q += nwaves) {
        const uint32_t d = ovf[q];
        const uint32_t len = uin_len[d];
        const uint64_t off = uin_off[d];
        bool found = false;
        for (uint32_t base = kPullCap; base < len && !found; base += 64) {
            const uint32_t k = base + lane;
            const bool hit = k < len && bit_of(front_bm, uin_src[off + k]);
            found = __ballot(hit) != 0;
            examined += (k < len) ? 1 : 0;
        }
        bool win = false;
        if (found && lane == 0) {
            const int r = visit_word(node + d, node[d], false);
            win = (r == 1);
            flagged += (r == 2);
        }
        emit_one(win, d, row_off, row_len, inv, nfr_off, nfr_len, &ctr->inv, &ln.F);
    }
    const uint32_t fs = wave_sum(flagged), es = wave_sum(examined);
    if (lane == 0) {
        if (fs) atomicAdd(&ctr->n_flagged, (unsigned long long)fs);
        if (es) atomicAdd(&ctr->pull_edges, (unsigned long long)es);
    }
}

// multi-GPU roots: every rank gets the global list and visits the slots it owns
__global__ __launch_bounds__(kBlock) void k_part_roots(const uint32_t* __restrict__ roots, const uint8_t* __restrict__ imm,
                                                       uint32_t n, uint32_t base, uint32_t n_local,
                                                       unsigned long long* node, const uint64_t* __restrict__ row_off,
                                                       const uint32_t* __restrict__ row_len,
                                                       uint32_t* __restrict__ inv, uint64_t* __restrict__ fr_off,
                                                       uint32_t* __restrict__ fr_len, WaveCtr* ctr) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    uint32_t win = 0, flagged = 0, h = 0;
    if (i < n) {
        h = roots[i] - base;
        if (h < n_local) {
            const unsigned long long w = node[h];
            if ((w & kVMask) != 0) {
                const int r = visit_word(node + h, w, imm ? imm[i] != 0 : false);
                win = (r == 1);
                flagged = (r == 2);
            }
        }
    }
    emit_one(win, h, row_off, row_len, inv, fr_off, fr_len, &ctr->inv, &ctr->lvl[0].F);
    const uint32_t fs = wave_sum(flagged), ws = wave_sum(win);
    if (lane_id() == 0 && fs) atomicAdd(&ctr->n_flagged, (unsigned long long)fs);
    if (lane_id() == 0 && ws) atomicAdd(&ctr->root_inv, (unsigned long long)ws);
}

// multi-GPU: apply the targets other ranks forwarded (their versions were checked by the sender)
__global__ __launch_bounds__(kBlock) void k_apply_recv(int L, uint64_t n, const uint32_t* __restrict__ recv, uint32_t base,
                                                       unsigned long long* node, const uint64_t* __restrict__ row_off,
                                                       const uint32_t* __restrict__ row_len,
                                                       uint32_t* __restrict__ inv, uint64_t* __restrict__ nfr_off,
                                                       uint32_t* __restrict__ nfr_len, WaveCtr* ctr) {
    __shared__ Emit em;
    LevelCtr& ln = ctr->lvl[(L + 1) % kRing];
    emit_init(em);
    uint32_t flagged = 0;
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    const uint64_t n_iter = (n + stride - 1) / stride;
    for (uint64_t it = 0; it < n_iter; ++it) {
        const uint64_t i = it * stride + (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
        bool win = false;
        uint32_t h = 0;
        if (i < n) {
            h = recv[i] - base;
            const unsigned long long w = node[h];
            if ((w & kVMask) != 0) {
                const int r = visit_word(node + h, w, false);
                win = (r == 1);
                flagged += (r == 2);
            }
        }
        emit_push(em, win, h, row_off, row_len, inv, nfr_off, nfr_len, &ctr->inv, &ln.F);
        emit_flush(em, kEmitCap - kBlock, row_off, row_len, inv, nfr_off, nfr_len, &ctr->inv, &ln.F);
    }
    emit_flush(em, 1, row_off, row_len, inv, nfr_off, nfr_len, &ctr->inv, &ln.F);
    const uint32_t fs = wave_sum(flagged);
    if (lane_id() == 0 && fs) atomicAdd(&ctr->n_flagged, (unsigned long long)fs);
}

}  // namespace

fgi_status run_wave(fgi_graph* g, uint32_t n_roots, const uint32_t* roots_dev, const uint8_t* imm_dev,
                    fgi_wave_stats* stats) {
    const auto t0 = std::chrono::steady_clock::now();
    hipStream_t s = g->stream;
    static const bool trace = getenv("FGI_TRACE") != nullptr;
    const bool timing = stats != nullptr || trace;
    FGI_TRY(ensure_cstart(g, g->pool_top));
    // Pull levels need the dependency-list cache. It is built lazily: while it is stale, levels
    // run push-only; once a level group shows a frontier heavy enough to pull, the cache is
    // (re)built and later groups may pull. Small waves (streaming mixes) never pay for it.
    const int direction = g->opt_direction;
    const uint64_t pull_threshold = g->pool_top / (uint64_t)(g->opt_pull_alpha > 0 ? g->opt_pull_alpha : 1);
    if (direction == 2 && n_roots) FGI_TRY(ensure_in_lists(g));
    bool allow_pull = direction != 1 && g->uin_src && g->uin_epoch == g->mut_epoch;
    FGI_HIP(g, hipMemsetAsync(g->ctr, 0, sizeof(WaveCtr), s));
    FGI_HIP(g, hipMemsetAsync(g->dead_bm, 0, g->bm_words * 4, s));
    if (timing) FGI_HIP(g, hipEventRecord(g->ev_w0, s));
    if (n_roots) {
        const uint32_t nb = (n_roots + kBlock - 1) / kBlock;
        hipLaunchKernelGGL(k_roots, dim3(nb), dim3(kBlock), 0, s, roots_dev, imm_dev, n_roots, g->n_handles,
                           reinterpret_cast<unsigned long long*>(g->node), g->row_off, g->row_len, g->inv,
                           g->fr_off[0], g->fr_len[0], g->ctr);
    }
    int n_cu = 256;
    hipDeviceGetAttribute(&n_cu, hipDeviceAttributeMultiprocessorCount, g->device);
    const uint32_t expand_grid = (uint32_t)n_cu * 5;     // 5 resident blocks per CU (LDS 28.8 KB each)
    const uint32_t pull_grid = (uint32_t)n_cu * 8;
    const uint32_t mark_grid = (uint32_t)n_cu * 2;
    constexpr int kGroup = 4;
    int L = 0;
    uint64_t levels = 0, e_trav = 0, f_total = 0, pull_levels = 0;
    double expand_ms = 0, pull_ms = 0;
    uint64_t expand_launches = 0, expand_edges = 0, expand_f = 0, pull_launches = 0, pull_f = 0;
    int dir_eff_of[kRing];
    bool done = (n_roots == 0);
    while (!done) {
        const int L0 = L;
        const int dir_eff = allow_pull ? direction : 1;
        for (int k = 0; k < kGroup; ++k, ++L) {
            const int buf = L & 1;
            dir_eff_of[L % kRing] = dir_eff;
            hipLaunchKernelGGL(k_scan_reduce, dim3(kScanBlocks), dim3(kBlock), 0, s, L, g->fr_len[buf], g->partials,
                               g->ctr);
            hipLaunchKernelGGL(k_scan_apply, dim3(kScanBlocks), dim3(kBlock), 0, s, L, g->fr_len[buf], g->partials,
                               g->escan, g->cstart, g->ctr, dir_eff, pull_threshold);
            hipLaunchKernelGGL(k_mark, dim3(mark_grid), dim3(kBlock), 0, s, L, g->inv, g->dead_bm, g->front_bm, g->ctr);
            if (timing) {
                while (g->ev.size() < 4 * (size_t)(L + 1) + 4) {
                    hipEvent_t e;
                    FGI_HIP(g, hipEventCreate(&e));
                    g->ev.push_back(e);
                }
                FGI_HIP(g, hipEventRecord(g->ev[4 * L], s));
            }
            hipLaunchKernelGGL(k_expand<false>, dim3(expand_grid), dim3(kBlock), 0, s, L, g->fr_off[buf], g->escan,
                               g->cstart, g->pool_col, g->pool_tag, reinterpret_cast<unsigned long long*>(g->node),
                               g->row_off, g->row_len, g->dead_bm, g->opt_dead_filter, g->inv, g->fr_off[buf ^ 1],
                               g->fr_len[buf ^ 1], g->ctr, RemoteArgs{});
            if (timing) FGI_HIP(g, hipEventRecord(g->ev[4 * L + 1], s));
            if (dir_eff != 1) {
                hipLaunchKernelGGL(k_pull, dim3(pull_grid), dim3(kBlock), 0, s, L, g->n_slots, g->uin_off, g->uin_len,
                                   g->uin_src, g->dead_bm, g->front_bm, reinterpret_cast<unsigned long long*>(g->node),
                                   g->row_off, g->row_len, g->inv, g->fr_off[buf ^ 1], g->fr_len[buf ^ 1], g->pull_ovf,
                                   g->ctr);
                if (timing) FGI_HIP(g, hipEventRecord(g->ev[4 * L + 3], s));
                hipLaunchKernelGGL(k_pull_long, dim3(pull_grid), dim3(kBlock), 0, s, L, g->uin_off, g->uin_len,
                                   g->uin_src, g->front_bm, reinterpret_cast<unsigned long long*>(g->node), g->row_off,
                                   g->row_len, g->inv, g->fr_off[buf ^ 1], g->fr_len[buf ^ 1], g->pull_ovf, g->ctr);
            }
            if (timing) FGI_HIP(g, hipEventRecord(g->ev[4 * L + 2], s));
            hipLaunchKernelGGL(k_clear_front, dim3(mark_grid), dim3(kBlock), 0, s, L, g->inv, g->front_bm, g->ctr);
        }
        FGI_HIP(g, hipGetLastError());
        FGI_HIP(g, hipMemcpyAsync(g->ctr_host, g->ctr, sizeof(WaveCtr), hipMemcpyDeviceToHost, s));
        FGI_HIP(g, hipStreamSynchronize(s));
        for (int l = L0; l < L; ++l) {
            const LevelCtr& lc = g->ctr_host->lvl[l % kRing];
            float ms_e = 0, ms_p = 0;
            if (timing) {
                // every launch counts (empty and no-op levels too), so the average launch
                // durations are the ones rocprofv3 reports for k_expand and k_pull
                FGI_HIP(g, hipEventElapsedTime(&ms_e, g->ev[4 * l], g->ev[4 * l + 1]));
                expand_ms += ms_e;
                ++expand_launches;
                if (dir_eff_of[l % kRing] != 1) {
                    FGI_HIP(g, hipEventElapsedTime(&ms_p, g->ev[4 * l + 1], g->ev[4 * l + 3]));
                    pull_ms += ms_p;
                    ++pull_launches;
                }
            }
            if (lc.F) {
                ++levels;
                e_trav += lc.T;
                f_total += lc.F;
                if (lc.pull) {
                    ++pull_levels;
                    pull_f += lc.F;
                } else {
                    expand_edges += lc.T;
                    expand_f += lc.F;
                }
            }
            if (trace)
                fprintf(stderr, "[fgi] level %d %s: frontier %llu edges %llu expand %.3f ms pull %.3f ms ovf %llu\n", l,
                        lc.pull ? "pull" : "push", (unsigned long long)lc.F, (unsigned long long)lc.T, ms_e, ms_p,
                        (unsigned long long)lc.ovf);
        }
        if (g->ctr_host->lvl[L % kRing].F == 0) done = true;
        if (!done && !allow_pull && direction == 0) {
            bool heavy = false;
            for (int l = L0; l < L; ++l) heavy |= g->ctr_host->lvl[l % kRing].T > pull_threshold;
            if (heavy) {
                FGI_TRY(ensure_in_lists(g));
                allow_pull = true;
            }
        }
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
    if (trace)
        fprintf(stderr, "[fgi] wave: %llu invalidated, pull candidates %llu, pull dependencies examined %llu\n",
                (unsigned long long)g->ctr_host->inv, (unsigned long long)g->ctr_host->pull_cand,
                (unsigned long long)g->ctr_host->pull_edges);
    if (stats) {
        const uint64_t v = g->ctr_host->inv;
        stats->roots += n_roots;
        stats->levels += levels;
        stats->v_inv += v;
        stats->e_trav += e_trav;
        stats->e_match += g->ctr_host->e_match;
        stats->n_flagged += g->ctr_host->n_flagged;
        stats->pull_levels += pull_levels;
        stats->pull_edges += g->ctr_host->pull_edges;
        // Algorithmic bytes of the wave. Push level, per traversed edge:
        // col 4 + tag 8 + node-word gather 8; per frontier entry: fr_len 4 x2, escan 8 w + 8 r,
        // fr_off 8 r, written 12 by the producer. Pull level: per candidate with a dependency list
        // uin_len 4 + uin_off 8, per examined dependency 4. Per invalidated node: CAS 8 + row
        // gathers 12 + list write 4. Per root 5.
        const uint64_t push_b = 20 * expand_edges + 44 * expand_f;
        // k_pull alone: dead-bitmap scan 1/8 B per slot, uin_len 4 B per live slot, uin_off 8 B per
        // slot with a dependency list, 4 B per dependency examined (its frontier-bitmap probe is an
        // L2 hit and not counted), and per winner 24 B (CAS 8 + row gathers 12 + list write 4)
        // plus 12 B per next-frontier entry written.
        const WaveCtr& c = *g->ctr_host;
        const uint64_t pull_b = c.pull_scan / 8 + 4 * c.pull_live + 8 * c.pull_cand + 4 * c.pull_edges +
                                36 * c.pull_win;
        stats->alg_bytes += push_b + pull_b + 24 * v + 5ull * n_roots;
        float wave_ms = 0;
        hipEventElapsedTime(&wave_ms, g->ev_w0, g->ev_w1);
        stats->kernel_ms += wave_ms;
        stats->expand_ms += expand_ms;
        stats->pull_ms += pull_ms;
        stats->expand_launches += expand_launches;
        stats->expand_bytes += 20 * expand_edges + 16 * expand_f;
        stats->pull_bytes += pull_b;
        stats->pull_launches += pull_launches;
        stats->f_total += f_total;
        stats->total_ms += std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    }
    return FGI_OK;
}

// ---- multi-GPU wave, split into phases shared by the RCCL driver (one process per GPU) and the
// in-process driver (several partitions of one graph on one device, exchange by device copies).
fgi_status part_wave_begin(fgi_graph* g, uint32_t n_roots, const uint32_t* roots_dev, const uint8_t* imm_dev) {
    PartView pv;
    if (!part_view(g, &pv)) return set_err(g, FGI_ESTATE, "partition not initialised");
    hipStream_t s = g->stream;
    g->pw = PartWave{};
    g->pw.t0 = std::chrono::steady_clock::now();
    g->pw.n_roots = n_roots;
    FGI_TRY(ensure_cstart(g, g->pool_top));
    FGI_HIP(g, hipMemsetAsync(g->ctr, 0, sizeof(WaveCtr), s));
    FGI_HIP(g, hipMemsetAsync(g->dead_bm, 0, g->bm_words * 4, s));
    FGI_HIP(g, hipMemsetAsync(pv.sent_bm, 0, pv.sent_words * 4, s));
    while (g->ev.size() < 3) {
        hipEvent_t e;
        FGI_HIP(g, hipEventCreate(&e));
        g->ev.push_back(e);
    }
    FGI_HIP(g, hipEventRecord(g->ev_w0, s));
    if (n_roots)
        hipLaunchKernelGGL(k_part_roots, dim3((n_roots + kBlock - 1) / kBlock), dim3(kBlock), 0, s, roots_dev, imm_dev,
                           n_roots, pv.base, pv.n_local, reinterpret_cast<unsigned long long*>(g->node), g->row_off,
                           g->row_len, g->inv, g->fr_off[0], g->fr_len[0], g->ctr);
    FGI_HIP(g, hipGetLastError());
    return FGI_OK;
}

const unsigned long long* part_level_frontier_dev(fgi_graph* g, int L) { return &g->ctr->lvl[L % kRing].F; }
const unsigned long long* part_level_edges_dev(fgi_graph* g, int L) { return &g->ctr->lvl[L % kRing].T; }

// scan of the local frontier (its edge total T decides push vs pull for every rank)
fgi_status part_level_scan(fgi_graph* g, int L) {
    PartView pv;
    part_view(g, &pv);
    hipStream_t s = g->stream;
    const int buf = L & 1;
    FGI_HIP(g, hipMemsetAsync(pv.send_cnt, 0, (size_t)pv.world * 8, s));
    hipLaunchKernelGGL(k_scan_reduce, dim3(kScanBlocks), dim3(kBlock), 0, s, L, g->fr_len[buf], g->partials, g->ctr);
    hipLaunchKernelGGL(k_scan_apply, dim3(kScanBlocks), dim3(kBlock), 0, s, L, g->fr_len[buf], g->partials, g->escan,
                       g->cstart, g->ctr, 1, (uint64_t)0);
    FGI_HIP(g, hipGetLastError());
    return FGI_OK;
}

// marks the previous level's winners (dead; frontier bitmap on pull levels); on a pull level the
// local frontier words front_bm[0, block/32) are then all-gathered into pv.front_global
fgi_status part_level_mark(fgi_graph* g, int L, bool pull) {
    hipStream_t s = g->stream;
    int n_cu = 256;
    hipDeviceGetAttribute(&n_cu, hipDeviceAttributeMultiprocessorCount, g->device);
    static const unsigned long long one = 1;
    if (pull)
        FGI_HIP(g, hipMemcpyAsync(&g->ctr->lvl[L % kRing].pull, &one, 8, hipMemcpyHostToDevice, s));
    hipLaunchKernelGGL(k_mark, dim3((uint32_t)n_cu * 2), dim3(kBlock), 0, s, L, g->inv, g->dead_bm, g->front_bm, g->ctr);
    FGI_HIP(g, hipGetLastError());
    return FGI_OK;
}

// push: expand (remote targets staged for the exchange); pull: scan local dependency lists
// against the global frontier bitmap
fgi_status part_level_work(fgi_graph* g, int L, bool pull) {
    PartView pv;
    part_view(g, &pv);
    hipStream_t s = g->stream;
    int n_cu = 256;
    hipDeviceGetAttribute(&n_cu, hipDeviceAttributeMultiprocessorCount, g->device);
    const RemoteArgs ra{pv.base, pv.n_local, pv.block, pv.world, pv.ver_all, pv.sent_bm, pv.send_buf, pv.send_cnt};
    const int buf = L & 1;
    FGI_HIP(g, hipEventRecord(g->ev[0], s));
    // launched on pull levels too: it clears the counters of level L + 2 and returns
    hipLaunchKernelGGL(k_expand<true>, dim3((uint32_t)n_cu * 4), dim3(kBlock), 0, s, L, g->fr_off[buf], g->escan,
                       g->cstart, g->pool_col, g->pool_tag, reinterpret_cast<unsigned long long*>(g->node), g->row_off,
                       g->row_len, g->dead_bm, g->opt_dead_filter, g->inv, g->fr_off[buf ^ 1], g->fr_len[buf ^ 1],
                       g->ctr, ra);
    FGI_HIP(g, hipEventRecord(g->ev[1], s));
    if (pull) {
        const uint32_t pull_grid = (uint32_t)n_cu * 8;
        hipLaunchKernelGGL(k_pull, dim3(pull_grid), dim3(kBlock), 0, s, L, pv.n_local, g->uin_off, g->uin_len, g->uin_src,
                           g->dead_bm, pv.front_global, reinterpret_cast<unsigned long long*>(g->node), g->row_off,
                           g->row_len, g->inv, g->fr_off[buf ^ 1], g->fr_len[buf ^ 1], g->pull_ovf, g->ctr);
        FGI_HIP(g, hipEventRecord(g->ev[2], s));
        hipLaunchKernelGGL(k_pull_long, dim3(pull_grid), dim3(kBlock), 0, s, L, g->uin_off, g->uin_len, g->uin_src,
                           pv.front_global, reinterpret_cast<unsigned long long*>(g->node), g->row_off, g->row_len,
                           g->inv, g->fr_off[buf ^ 1], g->fr_len[buf ^ 1], g->pull_ovf, g->ctr);
        FGI_HIP(g, hipMemsetAsync(pv.front_global, 0, pv.front_words_global * 4, s));
    }
    FGI_HIP(g, hipGetLastError());
    g->pw.pulled = pull;
    return FGI_OK;
}

fgi_status part_level_apply(fgi_graph* g, int L, uint64_t n_recv, uint64_t n_sent) {
    PartView pv;
    part_view(g, &pv);
    hipStream_t s = g->stream;
    int n_cu = 256;
    hipDeviceGetAttribute(&n_cu, hipDeviceAttributeMultiprocessorCount, g->device);
    const int buf = L & 1;
    if (n_recv)
        hipLaunchKernelGGL(k_apply_recv, dim3(std::min<uint64_t>((n_recv + kBlock - 1) / kBlock, (uint64_t)n_cu * 8)),
                           dim3(kBlock), 0, s, L, n_recv, pv.recv_buf, pv.base,
                           reinterpret_cast<unsigned long long*>(g->node), g->row_off, g->row_len, g->inv,
                           g->fr_off[buf ^ 1], g->fr_len[buf ^ 1], g->ctr);
    hipLaunchKernelGGL(k_clear_front, dim3((uint32_t)n_cu * 2), dim3(kBlock), 0, s, L, g->inv, g->front_bm, g->ctr);
    FGI_HIP(g, hipGetLastError());
    g->pw.sent += n_sent;
    return FGI_OK;
}

// after the level's frontier total is known (the stream has been synchronised by then)
fgi_status part_level_account(fgi_graph* g, int L) {
    FGI_HIP(g, hipMemcpyAsync(g->ctr_host, g->ctr, sizeof(WaveCtr), hipMemcpyDeviceToHost, g->stream));
    FGI_HIP(g, hipStreamSynchronize(g->stream));
    const LevelCtr& lc = g->ctr_host->lvl[L % kRing];
    g->pw.levels++;
    g->pw.e_trav += lc.T;
    g->pw.f_total += lc.F;
    if (!lc.pull) g->pw.push_edges += lc.T, g->pw.push_f += lc.F;
    float ms = 0;
    FGI_HIP(g, hipEventElapsedTime(&ms, g->ev[0], g->ev[1]));
    g->pw.expand_ms += ms;
    g->pw.expand_launches++;
    if (g->pw.pulled) {
        FGI_HIP(g, hipEventElapsedTime(&ms, g->ev[1], g->ev[2]));
        g->pw.pull_ms += ms;
        g->pw.pull_launches++;
        g->pw.pull_levels++;
    }
    return FGI_OK;
}

fgi_status part_wave_end(fgi_graph* g, fgi_wave_stats* stats) {
    hipStream_t s = g->stream;
    FGI_HIP(g, hipMemcpyAsync(g->ctr_host, g->ctr, sizeof(WaveCtr), hipMemcpyDeviceToHost, s));
    FGI_HIP(g, hipEventRecord(g->ev_w1, s));
    FGI_HIP(g, hipStreamSynchronize(s));
    g->last_wave_n = g->ctr_host->inv;
    if (stats) {
        const PartWave& w = g->pw;
        const uint64_t v = g->ctr_host->inv;
        stats->roots += w.n_roots;
        stats->levels += w.levels;
        stats->v_inv += v;
        stats->e_trav += w.e_trav;
        stats->e_match += g->ctr_host->e_match;
        stats->n_flagged += g->ctr_host->n_flagged;
        stats->remote_msgs += w.sent;
        // as run_wave (push and pull levels), plus 8 B per forwarded target (written + received)
        const WaveCtr& c = *g->ctr_host;
        const uint64_t pull_b = c.pull_scan / 8 + 4 * c.pull_live + 8 * c.pull_cand + 4 * c.pull_edges +
                                36 * c.pull_win;
        stats->alg_bytes += 20 * w.push_edges + 44 * w.push_f + pull_b + 24 * v + 8 * w.sent + 5ull * w.n_roots;
        stats->pull_levels += w.pull_levels;
        stats->pull_edges += c.pull_edges;
        stats->pull_ms += w.pull_ms;
        stats->pull_bytes += pull_b;
        stats->pull_launches += w.pull_launches;
        float wave_ms = 0;
        hipEventElapsedTime(&wave_ms, g->ev_w0, g->ev_w1);
        stats->kernel_ms += wave_ms;
        stats->expand_ms += w.expand_ms;
        stats->expand_launches += w.expand_launches;
        stats->expand_bytes += 20 * w.push_edges + 16 * w.push_f;
        stats->f_total += w.f_total;
        stats->total_ms += std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - w.t0).count();
    }
    return FGI_OK;
}

// One process per GPU: levels in lockstep over RCCL.
fgi_status run_part_wave(fgi_graph* g, uint32_t n_roots, const uint32_t* roots_dev, const uint8_t* imm_dev,
                         fgi_wave_stats* stats) {
    PartView pv;
    part_view(g, &pv);
    FGI_TRY(part_wave_begin(g, n_roots, roots_dev, imm_dev));
    const bool allow_pull = g->opt_direction != 1 && g->uin_src && g->uin_epoch == g->mut_epoch;
    uint64_t e_global = 0, f_global = 0, t_global = 0;
    FGI_HIP(g, hipMemcpy(pv.scratch_u64, &g->pool_top, 8, hipMemcpyHostToDevice));
    FGI_TRY(part_allreduce_sum(g, pv.scratch_u64, &e_global));
    const uint64_t threshold = e_global / (uint64_t)(g->opt_pull_alpha > 0 ? g->opt_pull_alpha : 1);
    FGI_TRY(part_allreduce_sum(g, part_level_frontier_dev(g, 0), &f_global));
    for (int L = 0; f_global != 0; ++L) {
        FGI_TRY(part_level_scan(g, L));
        FGI_TRY(part_allreduce_sum(g, part_level_edges_dev(g, L), &t_global));
        const bool pull = allow_pull && (g->opt_direction == 2 || t_global > threshold);
        FGI_TRY(part_level_mark(g, L, pull));
        if (pull) FGI_TRY(part_allgather_front(g));
        FGI_TRY(part_level_work(g, L, pull));
        uint64_t n_recv = 0, n_sent = 0;
        if (!pull) FGI_TRY(part_exchange(g, &n_recv, &n_sent));
        FGI_TRY(part_level_apply(g, L, n_recv, n_sent));
        FGI_TRY(part_allreduce_sum(g, part_level_frontier_dev(g, L + 1), &f_global));
        FGI_TRY(part_level_account(g, L));
    }
    return part_wave_end(g, stats);
}

}  // namespace fgi
