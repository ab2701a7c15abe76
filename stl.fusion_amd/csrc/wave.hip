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
//   k_level_begin : push/pull decision for the level (from the frontier totals F and T that the
//                   previous level's emitters accumulated), dead/frontier bitmap upkeep for the
//                   previous level's push winners, partial sums of the frontier's row lengths
//   k_scan_apply  : (push levels) exclusive scan of the row lengths and the chunk->entry map
//   k_level       : push — edge-parallel expansion of the frontier's `_usedBy` rows (edges to
//                   nodes already dead skip the tag load and the gather); or pull — every live
//                   slot probes its dependency list (the reference's `_used`: in-edges whose tag
//                   matches its version) for a parent in the frontier bitmap, head first, with
//                   early exit (Beamer's bottom-up step), storing its winners' bitmap words itself
// Multi-GPU levels (run_part_wave) use k_scan_reduce / k_scan_apply / k_mark / k_level<true> /
// k_apply_recv / k_clear_front, with the exchange between them.
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>

#include "fgi_internal.h"

namespace fgi {
namespace {

constexpr uint32_t kPullCap = 16;   // list entries one lane scans; longer lists go to the whole wave

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

// Where a level's winners go: the invalidated list (all winners) and the next frontier (winners
// with a non-empty row, with that row's offset/length); the next level's F and T accumulate in ln.
struct Out {
    const uint64_t* __restrict__ row_off;
    const uint32_t* __restrict__ row_len;
    uint32_t* __restrict__ inv;
    uint64_t* __restrict__ nfr_off;
    uint32_t* __restrict__ nfr_len;
    unsigned long long* inv_ctr;
    LevelCtr* ln;
};

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

__device__ __forceinline__ unsigned long long wave_sum64(unsigned long long v) {
#pragma unroll
    for (int d = 32; d >= 1; d >>= 1) v += __shfl_xor(v, d, 64);
    return v;
}

// Per-block statistics: hot kernels keep their counters per block (plain read-modify-write of the
// block's own row by one thread, launches of a wave are stream-ordered) instead of per-wave
// atomics on a few words: a single device-scope word saturates near 88 atomics/us, so 6,000 waves
// adding to it would serialise for ~70 us. k_stats_reduce folds the rows into WaveCtr.
enum : int { kStEMatch, kStFlagged, kStPullCand, kStPullEdges, kStPullLive, kStPullWin, kStPullTail, kStPullScan, kStats };
static_assert(kStats == kStatCols, "statistics columns");

// Block-uniform call: adds each thread's v[k] into the block's row.
__device__ __forceinline__ void block_stats_add(unsigned long long* blk, unsigned long long (*s)[kStats],
                                                const uint32_t (&v)[kStats]) {
    const uint32_t wid = threadIdx.x >> 6;
#pragma unroll
    for (int k = 0; k < kStats; ++k) {
        unsigned long long x = v[k];
#pragma unroll
        for (int d = 32; d >= 1; d >>= 1) x += __shfl_xor(x, d, 64);
        if (lane_id() == 0) s[wid][k] = x;
    }
    __syncthreads();
    if (threadIdx.x < kStats) {
        unsigned long long t = 0;
        for (uint32_t q = 0; q < kBlock / 64; ++q) t += s[q][threadIdx.x];
        if (t) blk[(uint64_t)blockIdx.x * kStats + threadIdx.x] += t;
    }
}

// Append one (possibly absent) winner per lane. Every lane of the wave must call it.
__device__ __forceinline__ void emit_one(bool win, uint32_t h, const Out& o) {
    uint32_t len = 0;
    uint64_t off = 0;
    if (win) {
        len = o.row_len[h];
        off = o.row_off[h];
    }
    uint64_t ib, fb;
    wave_reserve(win ? 1u : 0u, (win && len) ? 1u : 0u, o.inv_ctr, &o.ln->F, ib, fb);
    if (win) o.inv[ib] = h;
    if (win && len) {
        o.nfr_off[fb] = off;
        o.nfr_len[fb] = len;
    }
    const unsigned long long ls = wave_sum64(len);
    if (lane_id() == 0 && ls) atomicAdd(&o.ln->T, ls);
}

// Block-level emission: winners are staged in LDS and appended to the global lists in batches
// (one pair of global atomics per batch instead of one per wave per iteration: the two list
// counters are single words, and same-address atomics saturate at ~88/us chip-wide). The staging
// buffer (CAP entries) is passed separately: pull levels stage into the expand LDS arrays.
constexpr uint32_t kEmitCap = 1024;
struct Emit {
    uint32_t n;
    uint32_t pad;
    unsigned long long base_inv, base_fr;
    uint32_t wsum[kBlock / 64];
    unsigned long long wlen[kBlock / 64];
};

__device__ __forceinline__ void emit_init(Emit& e) {
    if (threadIdx.x == 0) e.n = 0;
    __syncthreads();
}

// Every lane of the calling wave must call it (ballot); lanes beyond the LDS capacity fall back
// to direct appends.
template <uint32_t CAP>
__device__ __forceinline__ void emit_push(Emit& e, uint32_t* buf, bool win, uint32_t h, const Out& o) {
    const unsigned long long m = __ballot(win);
    if (!m) return;
    uint32_t base = 0;
    if (lane_id() == 0) base = atomicAdd(&e.n, (uint32_t)__popcll(m));
    base = __shfl(base, 0, 64);
    if (win) {
        const uint32_t idx = base + (uint32_t)__popcll(m & ((1ull << lane_id()) - 1ull));
        if (idx < CAP) {
            buf[idx] = h;
        } else {
            o.inv[atomicAdd(o.inv_ctr, 1ull)] = h;
            const uint32_t len = o.row_len[h];
            if (len) {
                const unsigned long long fb = atomicAdd(&o.ln->F, 1ull);
                o.nfr_off[fb] = o.row_off[h];
                o.nfr_len[fb] = len;
                atomicAdd(&o.ln->T, (unsigned long long)len);
            }
        }
    }
}

// Block-uniform call. Flushes when at least `at` winners are staged (at = 1: flush anything).
template <uint32_t CAP>
__device__ __forceinline__ void emit_flush(Emit& e, uint32_t* buf, uint32_t at, const Out& o) {
    __syncthreads();
    const uint32_t n = e.n < CAP ? e.n : CAP;
    __syncthreads();   // every thread has read e.n before any wave can push again
    if (n < at || n == 0) return;   // uniform decision
    constexpr int kPer = CAP / kBlock;
    // pass 1: this thread's entries (i = tid + k * kBlock) with a row, and their row lengths
    uint32_t cnt = 0;
    unsigned long long lsum = 0;
#pragma unroll
    for (int k = 0; k < kPer; ++k) {
        const uint32_t i = threadIdx.x + k * kBlock;
        if (i < n) {
            const uint32_t len = o.row_len[buf[i]];
            cnt += len ? 1u : 0u;
            lsum += len;
        }
    }
    uint32_t wtot;
    const uint32_t wex = wave_excl_scan(cnt, wtot);
    lsum = wave_sum64(lsum);
    const uint32_t wid = threadIdx.x >> 6;
    if (lane_id() == 0) {
        e.wsum[wid] = wtot;
        e.wlen[wid] = lsum;
    }
    __syncthreads();
    uint32_t before = 0, total = 0;
    for (uint32_t k = 0; k < kBlock / 64; ++k) {
        if (k < wid) before += e.wsum[k];
        total += e.wsum[k];
    }
    if (threadIdx.x == 0) {
        unsigned long long tl = 0;
        for (uint32_t k = 0; k < kBlock / 64; ++k) tl += e.wlen[k];
        e.base_inv = atomicAdd(o.inv_ctr, (unsigned long long)n);
        e.base_fr = total ? atomicAdd(&o.ln->F, (unsigned long long)total) : 0ull;
        if (tl) atomicAdd(&o.ln->T, tl);
    }
    __syncthreads();
    // pass 2: the same entries in the same order (row lengths are L2 hits now)
    uint64_t fb = e.base_fr + before + wex;
#pragma unroll
    for (int k = 0; k < kPer; ++k) {
        const uint32_t i = threadIdx.x + k * kBlock;
        if (i < n) {
            const uint32_t h = buf[i];
            o.inv[e.base_inv + i] = h;
            const uint32_t len = o.row_len[h];
            if (len) {
                o.nfr_off[fb] = o.row_off[h];
                o.nfr_len[fb] = len;
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
                                                  uint32_t n_handles, unsigned long long* node, Out o,
                                                  WaveCtr* ctr) {
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
    emit_one(win, h, o);
    const uint32_t fs = wave_sum(flagged), ws = wave_sum(win);
    if (lane_id() == 0 && fs) atomicAdd(&ctr->root_flagged, (unsigned long long)fs);
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

__device__ __forceinline__ void scan_partial(uint64_t F, const uint32_t* __restrict__ fr_len,
                                             unsigned long long* __restrict__ partials, unsigned long long* s_red) {
    const uint64_t b = blockIdx.x, G = gridDim.x;
    const uint64_t lo = F * b / G, hi = F * (b + 1) / G;
    unsigned long long s = 0;
    for (uint64_t i = lo + threadIdx.x; i < hi; i += blockDim.x) s += fr_len[i];
    s = block_sum(s, s_red);
    if (threadIdx.x == 0) partials[b] = s;
}

// multi-GPU levels: partial sums of the frontier's row lengths
__global__ __launch_bounds__(kBlock) void k_scan_reduce(int L, const uint32_t* __restrict__ fr_len,
                                                        unsigned long long* __restrict__ partials,
                                                        WaveCtr* ctr) {
    __shared__ unsigned long long s_red[kBlock / 64];
    scan_partial(ctr->lvl[L % kRing].F, fr_len, partials, s_red);
}

// Single-GPU level prologue (one launch, grid kScanBlocks):
//  - the push/pull decision for level L from the frontier totals F, T its producers accumulated;
//  - bitmap upkeep for the previous level's winners inv[mark_hi(L-1), inv): winners of a push level
//    (or the roots) are marked dead here, and into the frontier bitmap fb_cur if level L pulls;
//    winners of a pull level were marked by the pull itself. fb_nxt (written by a pull at level
//    L) is cleared when level L pushes, so a later push->pull switch finds it empty;
//  - on push levels, the partial sums of the frontier's row lengths for k_scan_apply.
__global__ __launch_bounds__(kBlock) void k_level_begin(int L, WaveCtr* ctr, const uint32_t* __restrict__ inv,
                                                        uint32_t* dead_bm, uint32_t* fb_cur, uint32_t* fb_nxt,
                                                        uint64_t bm_words, uint64_t slot_words,
                                                        const uint32_t* __restrict__ fr_len,
                                                        unsigned long long* __restrict__ partials, int direction,
                                                        uint64_t pull_threshold) {
    __shared__ unsigned long long s_red[kBlock / 64];
    LevelCtr& lc = ctr->lvl[L % kRing];
    const uint64_t F = lc.F, T = lc.T;
    const bool pull = F != 0 && (direction == 2 || (direction == 0 && T > pull_threshold));
    const bool prev_pull = L > 0 && ctr->lvl[(L + kRing - 1) % kRing].pull != 0;
    const uint64_t lo = L > 0 ? ctr->lvl[(L + kRing - 1) % kRing].mark_hi : 0ull;
    const uint64_t hi = ctr->inv;
    const uint64_t tid = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const uint64_t nthr = (uint64_t)gridDim.x * blockDim.x;
    if (tid == 0) {
        lc.pull = pull ? 1ull : 0ull;
        lc.nchunks = (T + kChunk - 1) / kChunk;
        lc.mark_lo = lo;
        lc.mark_hi = hi;
    }
    if (!prev_pull) {
        for (uint64_t i = lo + tid; i < hi; i += nthr) {
            const uint32_t h = inv[i];
            atomicOr(dead_bm + (h >> 5), 1u << (h & 31));
            if (pull) atomicOr(fb_cur + (h >> 5), 1u << (h & 31));
        }
    }
    // a pull at level L stores every slot word of fb_nxt; the words past the slots (detached
    // handles) are never winners of a pull and must read as zero
    for (uint64_t w = (pull ? slot_words : 0ull) + tid; w < bm_words; w += nthr) fb_nxt[w] = 0u;
    if (!pull && F) scan_partial(F, fr_len, partials, s_red);
}

// Exclusive scan of fr_len into escan; records for every chunk of kChunk edges the frontier
// entry holding its first edge (cstart). decide = 1 (multi-GPU levels): also sets T, nchunks and
// a push decision (the driver overrides it for pull levels); decide = 0: k_level_begin decided.
__global__ __launch_bounds__(kBlock) void k_scan_apply(int L, const uint32_t* __restrict__ fr_len,
                                                       const unsigned long long* __restrict__ partials,
                                                       uint64_t* __restrict__ escan, uint32_t* __restrict__ cstart,
                                                       WaveCtr* ctr, int decide) {
    __shared__ unsigned long long s_red[kBlock / 64];
    __shared__ unsigned long long s_wave[kBlock / 64];
    LevelCtr& lc = ctr->lvl[L % kRing];
    const uint64_t F = lc.F;
    if (!decide && (lc.pull || F == 0)) return;
    const uint64_t b = blockIdx.x, G = gridDim.x;
    unsigned long long before = 0, all = 0;
    for (uint64_t k = threadIdx.x; k < G; k += blockDim.x) {
        const unsigned long long p = partials[k];
        all += p;
        if (k < b) before += p;
    }
    before = block_sum(before, s_red);
    all = block_sum(all, s_red);
    if (decide && b == 0 && threadIdx.x == 0) {
        lc.T = all;
        lc.nchunks = (all + kChunk - 1) / kChunk;
        lc.pull = 0ull;
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

// ---- multi-GPU bitmaps ------------------------------------------------------------------------
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

struct ExpandArgs {
    const uint64_t* __restrict__ fr_off;
    const uint64_t* __restrict__ escan;
    const uint32_t* __restrict__ cstart;
    const uint32_t* __restrict__ pool_col;
    const uint64_t* __restrict__ pool_tag;
    const uint32_t* __restrict__ dead_bm;
    int dead_filter;
};

// PART: multi-GPU rank — dependant slots outside [ra.base, ra.base + ra.n_local) are remote: their
// tag is checked against the version replica and matching targets are forwarded once per wave.
template <bool PART>
__device__ __forceinline__ void expand_level(const LevelCtr& lc, const ExpandArgs& x, unsigned long long* node,
                                             const Out& o, Emit& em, uint32_t* eb, MsgEmit<PART>& me, uint32_t* s_rel,
                                             uint32_t* s_base, unsigned long long* blk,
                                             unsigned long long (*s_st)[kStats], const RemoteArgs& ra) {
    if constexpr (PART) {
        if (threadIdx.x == 0) me.n = 0;
    }
    const uint64_t T = lc.T, F = lc.F, nch = lc.nchunks;
    uint32_t matched = 0, flagged = 0;
    for (uint64_t c = blockIdx.x; c < nch; c += gridDim.x) {
        const uint64_t cbase = c * kChunk;
        const uint32_t clen = (uint32_t)((T - cbase) < (uint64_t)kChunk ? (T - cbase) : (uint64_t)kChunk);
        const uint32_t i0 = x.cstart[c];
        const uint32_t i1 = (c + 1 < nch) ? x.cstart[c + 1] : (uint32_t)(F - 1);
        const uint32_t n = i1 - i0 + 1;
        for (uint32_t k = threadIdx.x; k < n; k += kBlock) {
            const uint64_t es = x.escan[i0 + k];
            s_rel[k] = es > cbase ? (uint32_t)(es - cbase) : 0u;
            s_base[k] = (uint32_t)(x.fr_off[i0 + k] + cbase - es);   // pool positions < 2^32
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
                dst[j] = __builtin_nontemporal_load(x.pool_col + pos[j]);
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
                        const uint64_t t = __builtin_nontemporal_load(x.pool_tag + pos[j]);
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
        if (x.dead_filter) {
#pragma unroll
            for (int j = 0; j < kEPT; ++j)
                if (dst[j] != 0xFFFFFFFFu && bit_of(x.dead_bm, dst[j])) dst[j] = 0xFFFFFFFFu;
        }
        uint64_t tag[kEPT];
        unsigned long long w[kEPT];
#pragma unroll
        for (int j = 0; j < kEPT; ++j) {
            tag[j] = 0;
            w[j] = 0;
            if (dst[j] != 0xFFFFFFFFu) {
                tag[j] = __builtin_nontemporal_load(x.pool_tag + pos[j]);
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
        for (int j = 0; j < kEPT; ++j) emit_push<kEmitCap>(em, eb, (win_mask >> j) & 1u, dst[j], o);
        emit_flush<kEmitCap>(em, eb, kEmitCap / 2, o);
        if constexpr (PART) msg_flush(me, kMsgCap / 2, ra);
    }
    emit_flush<kEmitCap>(em, eb, 1, o);
    if constexpr (PART) msg_flush(me, 1, ra);
    const uint32_t v[kStats] = {matched, flagged, 0, 0, 0, 0, 0, 0};
    block_stats_add(blk, s_st, v);
}

// ---- pull: every live slot looks for a parent in the frontier ---------------------------------
// uin_* is the dependency-list cache: for slot d, the handles u whose `_usedBy` row holds
// (d, version(d)) — the reference's d._used (Computed.cs:36, 365-366). A parent in the frontier
// bitmap (u invalidated in the previous level) means the push step would visit d from u.
struct PullArgs {
    uint32_t n_slots;
    const uint64_t* __restrict__ uin_off;
    const uint32_t* __restrict__ uin_len;
    const uint32_t* __restrict__ uin_src;
    const uint64_t* __restrict__ uin_head;   // first two list entries (lo | hi << 32)
    const uint32_t* __restrict__ front_rd;   // frontier bitmap (handles; multi-GPU: global ids)
    uint32_t* front_wr;                      // single GPU: next frontier bitmap, stored whole
    uint32_t* dead_bm;
};

// Each wave owns kPS x 64 consecutive slots (2 x kPS bitmap words); a lane handles kPS slots 64
// apart, so every step issues kPS independent loads (dead word, head, frontier bit, node word, CAS)
// per lane. A live slot probes the two heads of its list first (lists are ordered so that the
// entries a wave reaches earliest come first), then the next kPullCap entries of a list that
// missed (4 loads in flight), and the rest of a longer list with the whole wave. The
// wave stores its winners' dead bits and next-frontier words itself — no atomics, no marking pass.
constexpr uint32_t kPS = 4;
#ifndef FGI_DIAG
#define FGI_DIAG 0   // instrumented builds only (make diag): bits switch parts of the pull off
#endif
constexpr uint32_t kPullEmitCap = 2048;   // staged in the expand LDS array s_base (8 KB)

__device__ __forceinline__ bool probe_tail(const PullArgs& p, uint64_t off, uint32_t len, uint32_t& examined) {
    const uint32_t lim = len < kPullCap ? len : kPullCap;
    bool hit = false;
    for (uint32_t k = 0; k < lim && !hit; k += 4) {
        uint32_t u[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) u[j] = (k + j < lim) ? p.uin_src[off + k + j] : FGI_NONE;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            if (u[j] != FGI_NONE) {
                ++examined;
                hit |= bit_of(p.front_rd, u[j]);
            }
        }
    }
    return hit;
}

__device__ __forceinline__ void pull_level(const PullArgs& p, unsigned long long* node, const Out& o, Emit& em,
                                           uint32_t* eb, unsigned long long* blk, unsigned long long (*s_st)[kStats]) {
    uint32_t flagged = 0, cand = 0, examined = 0, live = 0, wins = 0, tails = 0;
    const uint32_t lane = lane_id();
    const uint32_t per_block = kBlock * kPS;
    const uint32_t stride = gridDim.x * per_block;
    const uint32_t n_iter = (p.n_slots + stride - 1) / stride;   // uniform trip count: flushes are block-wide
    for (uint32_t it = 0; it < n_iter; ++it) {
        const uint32_t d0 = it * stride + blockIdx.x * per_block + (threadIdx.x >> 6) * (64 * kPS);
        uint32_t d[kPS];
        uint64_t hd[kPS];
        bool lv[kPS], hit[kPS], long_rest[kPS];
#pragma unroll
        for (int j = 0; j < (int)kPS; ++j) {
            d[j] = d0 + j * 64 + lane;
            const uint32_t dw = d[j] < p.n_slots ? p.dead_bm[d[j] >> 5] : 0xFFFFFFFFu;
            lv[j] = d[j] < p.n_slots && !((dw >> (d[j] & 31)) & 1u);
        }
        constexpr uint64_t kNoHeads = ((uint64_t)FGI_NONE << 32) | FGI_NONE;
#pragma unroll
        for (int j = 0; j < (int)kPS; ++j)
            hd[j] = lv[j] ? ((FGI_DIAG & 32) ? (uint64_t)((d[j] * 2654435761u) % p.n_slots) | ((uint64_t)FGI_NONE << 32)
                                             : p.uin_head[d[j]])
                          : kNoHeads;
#pragma unroll
        for (int j = 0; j < (int)kPS; ++j) {
            live += lv[j] ? 1u : 0u;
            hit[j] = false;
            long_rest[j] = false;
            const uint32_t h0 = (uint32_t)hd[j], h1 = (uint32_t)(hd[j] >> 32);
            if (h0 != FGI_NONE) {
                ++cand;
                ++examined;
                if (FGI_DIAG & 16) {
                    hit[j] = ((h0 * 2654435761u) >> 31) != 0;
                } else {
                    const bool b0 = bit_of(p.front_rd, h0);
                    const bool b1 = h1 != FGI_NONE && bit_of(p.front_rd, h1);
                    examined += (!b0 && h1 != FGI_NONE) ? 1u : 0u;
                    hit[j] = b0 || b1;
                }
            }
        }
        // both heads missed: the next kPullCap entries of the list, then the whole wave on the rest
#pragma unroll
        for (int j = 0; j < (int)kPS && !(FGI_DIAG & 4); ++j) {
            uint32_t len = 0;
            uint64_t off = 0;
            if ((uint32_t)hd[j] != FGI_NONE && !hit[j]) {
                len = p.uin_len[d[j]];
                if (len > 2) {
                    off = p.uin_off[d[j]];
                    ++tails;
                    hit[j] = probe_tail(p, off + 2, len - 2, examined);
                    long_rest[j] = !hit[j] && len > 2 + kPullCap;
                }
            }
            unsigned long long lm = __ballot(long_rest[j]);
            while (lm) {
                const int l = __ffsll((long long)lm) - 1;
                lm &= lm - 1;
                const uint64_t lo = __shfl(off, l, 64);
                const uint32_t ln = __shfl(len, l, 64);
                bool f = false;
                for (uint32_t b = 2 + kPullCap; b < ln && !f; b += 64) {
                    const uint32_t k = b + lane;
                    const bool x = k < ln && bit_of(p.front_rd, p.uin_src[lo + k]);
                    examined += (k < ln) ? 1u : 0u;
                    f = __ballot(x) != 0;
                }
                if ((int)lane == l) hit[j] = f;
            }
        }
        unsigned long long w[kPS];
#pragma unroll
        for (int j = 0; j < (int)kPS; ++j) w[j] = (hit[j] && !(FGI_DIAG & 2)) ? node[d[j]] : 0ull;
        bool win[kPS];
#pragma unroll
        for (int j = 0; j < (int)kPS; ++j) {
            win[j] = (FGI_DIAG & 2) ? hit[j] : false;
            if (hit[j] && !(FGI_DIAG & 2)) {
                const int r = visit_word(node + d[j], w[j], false);
                win[j] = (r == 1);
                flagged += (r == 2);
            }
            wins += win[j] ? 1u : 0u;
        }
        if (p.front_wr && !(FGI_DIAG & 8)) {
#pragma unroll
            for (int j = 0; j < (int)kPS; ++j) {
                const unsigned long long wm = __ballot(win[j]);
                const uint32_t u0 = d0 + j * 64;
                if (lane == 0 && u0 < p.n_slots) {
                    unsigned long long* dp = reinterpret_cast<unsigned long long*>(p.dead_bm) + (u0 >> 6);
                    if (wm) *dp |= wm;
                    reinterpret_cast<unsigned long long*>(p.front_wr)[u0 >> 6] = wm;
                }
            }
        }
#pragma unroll
        for (int j = 0; j < (int)kPS; ++j) emit_push<kPullEmitCap>(em, eb, (FGI_DIAG & 1) ? false : win[j], d[j], o);
        // at most kPS x kBlock winners per step
        emit_flush<kPullEmitCap>(em, eb, kPullEmitCap - kPS * kBlock, o);
    }
    emit_flush<kPullEmitCap>(em, eb, 1, o);
    const uint32_t scan = (blockIdx.x == 0 && threadIdx.x == 0) ? p.n_slots : 0u;
    const uint32_t v[kStats] = {0, flagged, cand, examined, live, wins, tails, scan};
    block_stats_add(blk, s_st, v);
}

// One level's traversal: push (expand) or pull, as decided for the level on the device.
template <bool PART>
__global__ __launch_bounds__(kBlock) void k_level(int L, ExpandArgs x, PullArgs p, unsigned long long* node, Out o,
                                                  WaveCtr* ctr, unsigned long long* blk, RemoteArgs ra) {
    __shared__ uint32_t s_rel[kChunk + 1];
    __shared__ uint32_t s_base[kChunk + 1];
    __shared__ Emit em;
    __shared__ uint32_t eb[kEmitCap];
    __shared__ MsgEmit<PART> me;
    __shared__ unsigned long long s_st[kBlock / 64][kStats];
    static_assert(kChunk + 1 >= kPullEmitCap, "pull staging");
    const LevelCtr& lc = ctr->lvl[L % kRing];
    o.ln = &ctr->lvl[(L + 1) % kRing];
    if (blockIdx.x == 0 && threadIdx.x < sizeof(LevelCtr) / 8)
        reinterpret_cast<unsigned long long*>(&ctr->lvl[(L + 2) % kRing])[threadIdx.x] = 0ull;
    // multi-GPU pull levels run on every rank (parents may be remote); otherwise no frontier, no work
    if (!lc.pull && lc.F == 0) return;
    emit_init(em);
    if (lc.pull) pull_level(p, node, o, em, s_base, blk, s_st);
    else expand_level<PART>(lc, x, node, o, em, eb, me, s_rel, s_base, blk, s_st, ra);
}

// multi-GPU roots: every rank gets the global list and visits the slots it owns
__global__ __launch_bounds__(kBlock) void k_part_roots(const uint32_t* __restrict__ roots, const uint8_t* __restrict__ imm,
                                                       uint32_t n, uint32_t base, uint32_t n_local,
                                                       unsigned long long* node, Out o, WaveCtr* ctr) {
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
    emit_one(win, h, o);
    const uint32_t fs = wave_sum(flagged), ws = wave_sum(win);
    if (lane_id() == 0 && fs) atomicAdd(&ctr->root_flagged, (unsigned long long)fs);
    if (lane_id() == 0 && ws) atomicAdd(&ctr->root_inv, (unsigned long long)ws);
}

// multi-GPU: apply the targets other ranks forwarded (their versions were checked by the sender)
__global__ __launch_bounds__(kBlock) void k_apply_recv(int L, uint64_t n, const uint32_t* __restrict__ recv, uint32_t base,
                                                       unsigned long long* node, Out o, WaveCtr* ctr,
                                                       unsigned long long* blk) {
    __shared__ unsigned long long s_st[kBlock / 64][kStats];
    __shared__ Emit em;
    __shared__ uint32_t eb[kEmitCap];
    o.ln = &ctr->lvl[(L + 1) % kRing];
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
        emit_push<kEmitCap>(em, eb, win, h, o);
        emit_flush<kEmitCap>(em, eb, kEmitCap - kBlock, o);
    }
    emit_flush<kEmitCap>(em, eb, 1, o);
    const uint32_t v[kStats] = {0, flagged, 0, 0, 0, 0, 0, 0};
    block_stats_add(blk, s_st, v);
}

// Folds the per-block statistics rows into the wave counters (one block; idempotent, so it can
// run after every level group).
__global__ __launch_bounds__(kBlock) void k_stats_reduce(const unsigned long long* __restrict__ blk, WaveCtr* ctr) {
    __shared__ unsigned long long s_red[kBlock / 64];
    unsigned long long* dst[kStats] = {&ctr->e_match,   &ctr->n_flagged, &ctr->pull_cand, &ctr->pull_edges,
                                       &ctr->pull_live, &ctr->pull_win,  &ctr->pull_tail, &ctr->pull_scan};
    for (int k = 0; k < kStats; ++k) {
        unsigned long long t = 0;
        for (uint32_t b = threadIdx.x; b < kStatBlocks; b += blockDim.x) t += blk[(uint64_t)b * kStats + k];
        t = block_sum(t, s_red);
        if (threadIdx.x == 0) *dst[k] = t + (k == kStFlagged ? ctr->root_flagged : 0ull);
    }
}

}  // namespace

// Algorithmic bytes of the pull levels of a wave (k_level on pull levels): per slot scanned the
// dead-bitmap read and the next-frontier store (1/8 B each); per live slot its head (4 B); per
// head miss the list's offset and length (12 B) and 4 B per further dependency examined (the
// frontier-bitmap probes hit L2 and are not counted); per winner CAS 8 + row gathers 12 + list
// write 4 + frontier entry 12.
static uint64_t pull_level_bytes(const WaveCtr& c) {
    const uint64_t tail_deps = c.pull_edges > c.pull_cand ? c.pull_edges - c.pull_cand : 0;
    return c.pull_scan / 4 + 4 * c.pull_live + 12 * c.pull_tail + 4 * tail_deps + 36 * c.pull_win;
}

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
    uint32_t* fb[2] = {g->front_bm, g->front_nx};
    FGI_HIP(g, hipMemsetAsync(g->ctr, 0, sizeof(WaveCtr), s));
    FGI_HIP(g, hipMemsetAsync(g->blk_stats, 0, sizeof(unsigned long long) * kStatBlocks * kStatCols, s));
    FGI_HIP(g, hipMemsetAsync(g->dead_bm, 0, g->bm_words * 4, s));
    FGI_HIP(g, hipMemsetAsync(fb[0], 0, g->bm_words * 4, s));
    if (timing) FGI_HIP(g, hipEventRecord(g->ev_w0, s));
    Out o{g->row_off, g->row_len, g->inv, g->fr_off[0], g->fr_len[0], &g->ctr->inv, &g->ctr->lvl[0]};
    if (n_roots) {
        const uint32_t nb = (n_roots + kBlock - 1) / kBlock;
        hipLaunchKernelGGL(k_roots, dim3(nb), dim3(kBlock), 0, s, roots_dev, imm_dev, n_roots, g->n_handles,
                           reinterpret_cast<unsigned long long*>(g->node), o, g->ctr);
    }
    int n_cu = 256;
    hipDeviceGetAttribute(&n_cu, hipDeviceAttributeMultiprocessorCount, g->device);
    // 6 resident blocks per CU (LDS 20.6 KB, 76 VGPRs); per-block statistics rows bound the grid
    const uint32_t level_grid = std::min<uint32_t>((uint32_t)n_cu * 6, kStatBlocks);
    const uint64_t slot_words = ((uint64_t)g->n_slots + 63) / 64 * 2;
    constexpr int kGroup = 4;
    int L = 0;
    uint64_t levels = 0, e_trav = 0, f_total = 0, pull_levels = 0;
    double expand_ms = 0, pull_ms = 0;
    uint64_t expand_launches = 0, expand_edges = 0, expand_f = 0, pull_launches = 0;
    bool done = (n_roots == 0);
    while (!done) {
        const int L0 = L;
        const int dir_eff = allow_pull ? direction : 1;
        for (int k = 0; k < kGroup; ++k, ++L) {
            const int buf = L & 1;
            hipLaunchKernelGGL(k_level_begin, dim3(kScanBlocks), dim3(kBlock), 0, s, L, g->ctr, g->inv, g->dead_bm,
                               fb[buf], fb[buf ^ 1], g->bm_words, slot_words, g->fr_len[buf], g->partials, dir_eff,
                               pull_threshold);
            hipLaunchKernelGGL(k_scan_apply, dim3(kScanBlocks), dim3(kBlock), 0, s, L, g->fr_len[buf], g->partials,
                               g->escan, g->cstart, g->ctr, 0);
            if (timing) {
                while (g->ev.size() < 2 * (size_t)(L + 1) + 2) {
                    hipEvent_t e;
                    FGI_HIP(g, hipEventCreate(&e));
                    g->ev.push_back(e);
                }
                FGI_HIP(g, hipEventRecord(g->ev[2 * L], s));
            }
            const ExpandArgs xa{g->fr_off[buf], g->escan, g->cstart, g->pool_col, g->pool_tag, g->dead_bm,
                                g->opt_dead_filter};
            const PullArgs pa{g->n_slots, g->uin_off, g->uin_len, g->uin_src, g->uin_head, fb[buf], fb[buf ^ 1],
                              g->dead_bm};
            Out ol{g->row_off, g->row_len, g->inv, g->fr_off[buf ^ 1], g->fr_len[buf ^ 1], &g->ctr->inv, nullptr};
            hipLaunchKernelGGL(k_level<false>, dim3(level_grid), dim3(kBlock), 0, s, L, xa, pa,
                               reinterpret_cast<unsigned long long*>(g->node), ol, g->ctr, g->blk_stats, RemoteArgs{});
            if (timing) FGI_HIP(g, hipEventRecord(g->ev[2 * L + 1], s));
        }
        hipLaunchKernelGGL(k_stats_reduce, dim3(1), dim3(kBlock), 0, s, g->blk_stats, g->ctr);
        FGI_HIP(g, hipGetLastError());
        FGI_HIP(g, hipMemcpyAsync(g->ctr_host, g->ctr, sizeof(WaveCtr), hipMemcpyDeviceToHost, s));
        FGI_HIP(g, hipStreamSynchronize(s));
        for (int l = L0; l < L; ++l) {
            const LevelCtr& lc = g->ctr_host->lvl[l % kRing];
            float ms = 0;
            if (timing) {
                // every k_level launch counts (empty levels too), so the average launch duration
                // is the one rocprofv3 reports for k_level
                FGI_HIP(g, hipEventElapsedTime(&ms, g->ev[2 * l], g->ev[2 * l + 1]));
                if (lc.pull) {
                    pull_ms += ms;
                    ++pull_launches;
                } else {
                    expand_ms += ms;
                    ++expand_launches;
                }
            }
            if (lc.F) {
                ++levels;
                e_trav += lc.T;
                f_total += lc.F;
                if (lc.pull) {
                    ++pull_levels;
                } else {
                    expand_edges += lc.T;
                    expand_f += lc.F;
                }
            }
            if (trace)
                fprintf(stderr, "[fgi] level %d %s: frontier %llu edges %llu k_level %.3f ms\n", l,
                        lc.pull ? "pull" : "push", (unsigned long long)lc.F, (unsigned long long)lc.T, ms);
        }
        if (g->ctr_host->lvl[L % kRing].F == 0) done = true;
        if (!done && !allow_pull && direction == 0) {
            bool heavy = false;
            for (int l = L0; l <= L; ++l) heavy |= g->ctr_host->lvl[l % kRing].T > pull_threshold;
            if (heavy) {
                FGI_TRY(ensure_in_lists(g));
                allow_pull = true;
            }
        }
    }
    if (n_roots == 0) {
        hipLaunchKernelGGL(k_stats_reduce, dim3(1), dim3(kBlock), 0, s, g->blk_stats, g->ctr);
        FGI_HIP(g, hipMemcpyAsync(g->ctr_host, g->ctr, sizeof(WaveCtr), hipMemcpyDeviceToHost, s));
        FGI_HIP(g, hipStreamSynchronize(s));
    }
    if (timing) {
        FGI_HIP(g, hipEventRecord(g->ev_w1, s));
        FGI_HIP(g, hipEventSynchronize(g->ev_w1));
    }
    g->last_wave_n = g->ctr_host->inv;
    const WaveCtr& c = *g->ctr_host;
    if (trace)
        fprintf(stderr,
                "[fgi] wave: %llu invalidated; pull: live %llu, candidates %llu, head misses %llu, dependencies "
                "examined %llu, winners %llu\n",
                (unsigned long long)c.inv, (unsigned long long)c.pull_live, (unsigned long long)c.pull_cand,
                (unsigned long long)c.pull_tail, (unsigned long long)c.pull_edges, (unsigned long long)c.pull_win);
    if (stats) {
        const uint64_t v = c.inv;
        stats->roots += n_roots;
        stats->levels += levels;
        stats->v_inv += v;
        stats->e_trav += e_trav;
        stats->e_match += c.e_match;
        stats->n_flagged += c.n_flagged;
        stats->pull_levels += pull_levels;
        stats->pull_edges += c.pull_edges;
        // Algorithmic bytes. Push level, per traversed edge: col 4 + tag 8 +
        // node-word gather 8; per frontier entry: fr_len 4 x2, escan 8 w + 8 r, fr_off 8 r, written
        // 12 by the producer. Per invalidated node: CAS 8 + row gathers 12 + list write 4. Per root 5.
        const uint64_t push_b = 20 * expand_edges + 44 * expand_f;
        const uint64_t pull_b = pull_level_bytes(c);
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
    FGI_HIP(g, hipMemsetAsync(g->blk_stats, 0, sizeof(unsigned long long) * kStatBlocks * kStatCols, s));
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
                           n_roots, pv.base, pv.n_local, reinterpret_cast<unsigned long long*>(g->node),
                           Out{g->row_off, g->row_len, g->inv, g->fr_off[0], g->fr_len[0], &g->ctr->inv, &g->ctr->lvl[0]},
                           g->ctr);
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
                       g->cstart, g->ctr, 1);
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
    const ExpandArgs xa{g->fr_off[buf], g->escan, g->cstart, g->pool_col, g->pool_tag, g->dead_bm, g->opt_dead_filter};
    const PullArgs pa{pv.n_local, g->uin_off, g->uin_len, g->uin_src, g->uin_head, pv.front_global, nullptr, g->dead_bm};
    const Out o{g->row_off, g->row_len, g->inv, g->fr_off[buf ^ 1], g->fr_len[buf ^ 1], &g->ctr->inv, nullptr};
    hipLaunchKernelGGL(k_level<true>, dim3((uint32_t)n_cu * 5), dim3(kBlock), 0, s, L, xa, pa,
                       reinterpret_cast<unsigned long long*>(g->node), o, g->ctr, g->blk_stats, ra);
    FGI_HIP(g, hipEventRecord(g->ev[1], s));
    if (pull) FGI_HIP(g, hipMemsetAsync(pv.front_global, 0, pv.front_words_global * 4, s));
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
                           reinterpret_cast<unsigned long long*>(g->node),
                           Out{g->row_off, g->row_len, g->inv, g->fr_off[buf ^ 1], g->fr_len[buf ^ 1], &g->ctr->inv,
                               nullptr},
                           g->ctr, g->blk_stats);
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
    if (g->pw.pulled) {
        g->pw.pull_ms += ms;
        g->pw.pull_launches++;
        g->pw.pull_levels++;
    } else {
        g->pw.expand_ms += ms;
        g->pw.expand_launches++;
    }
    return FGI_OK;
}

fgi_status part_wave_end(fgi_graph* g, fgi_wave_stats* stats) {
    hipStream_t s = g->stream;
    hipLaunchKernelGGL(k_stats_reduce, dim3(1), dim3(kBlock), 0, s, g->blk_stats, g->ctr);
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
        const uint64_t pull_b = pull_level_bytes(c);
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
