// wave.hip — batched multi-root invalidation as a level-synchronous, direction-optimizing BFS.
//
// Restates the cascade of Computed<T>.Invalidate (src/Stl.Fusion/Computed.cs:162-230):
//   visit(dst, tag): the dst slot's current node n exists and n.Version == tag
//                    (Computed.cs:213-214, ComputedInput.GetExistingComputed) ->
//     Invalidated              : no-op                                  (164-165, 171-172)
//     Computing                : flags |= InvalidateOnSetOutput          (173-178)
//     Consistent, hasDelay     : flags |= InvalidationDelayStarted once  (186-191; timer host-side)
//     Consistent, no delay     : state := Invalidated, expand every `_usedBy` entry (185, 212-216)
// Every rule is idempotent (a second visit is always a no-op) and its effect depends only on the
// node word, which no wave changes. So a wave records visits in a bitmap: one atomicOr per visit
// decides the first visitor, and the first visitor of a node of the expandable class (Consistent,
// no delay) is its one invalidation winner. fold() applies the bits to the words before anything
// else reads them. The union over roots is order-independent, so one
// BFS wave replaces the reference's sequence of per-root DFS.
//
// Per level L (stream-ordered launches; the host synchronises once per group of levels):
//   k_level_begin : push/pull decision for the level, frontier bitmap upkeep for the previous
//                   level's push winners, partial sums of the frontier's row lengths; after a pull
//                   level: partial sums of its per-tile winner counts (collect, pass 1)
//   k_scan_apply  : push — exclusive scan of the row lengths and the chunk->entry map; after a pull
//                   level: the winners bitmap -> invalidated list + frontier list (collect, pass 2)
//   k_level       : push — edge-parallel expansion of the frontier's `_usedBy` rows; or pull — every
//                   live slot probes its dependency list (the reference's `_used`) for a parent in
//                   the frontier bitmap (Beamer's bottom-up step), writing only bitmaps and counts
// Multi-GPU levels (run_part_wave) use k_scan_reduce / k_scan_apply / k_mark / k_level<true> /
// k_apply_recv / k_clear_front, with the exchange between them.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <vector>
#include <cstdio>
#include <cstdlib>

#include "fgi_internal.h"

namespace fgi {
namespace {

__device__ __forceinline__ uint32_t lane_id() { return __lane_id(); }

__device__ __forceinline__ bool bit_of(const uint32_t* __restrict__ bm, uint32_t h) {
    return (bm[h >> 5] >> (h & 31)) & 1u;
}

// Effect of a node's first visit in a wave: 1 = Consistent -> Invalidated (expands), 2 = a flag
// is newly set (Computing: InvalidateOnSetOutput; Consistent with delay: InvalidationDelayStarted),
// 0 = nothing (Invalidated, or the flag was already set).
__device__ __forceinline__ int first_visit(unsigned long long w) {
    const uint32_t st = word_state(w);
    if (st == FGI_CONSISTENT) return (w & kW_HasDelay) ? ((w & kW_DS) ? 0 : 2) : 1;
    if (st == FGI_COMPUTING) return (w & kW_IOSO) ? 0 : 2;
    return 0;
}

// The node word after a (non-immediate) visit: canonical, flags of an Invalidated node cleared.
__host__ __device__ __forceinline__ unsigned long long visited_word(unsigned long long w) {
    if ((w & kVMask) == 0) return w;
    const uint32_t st = word_state(w);
    if (st == FGI_COMPUTING) return w | kW_IOSO;
    if (st == FGI_CONSISTENT)
        return (w & kW_HasDelay) ? (w | kW_DS) : ((w & (kVMask | kW_HasDelay)) | kW_Invalidated);
    return w;
}

// Invalidate(immediately: true) on a canonical word (Computed.cs:162-191: the delay is ignored).
__device__ __forceinline__ unsigned long long imm_word(unsigned long long w) {
    const uint32_t st = word_state(w);
    if (st == FGI_COMPUTING) return w | kW_IOSO | kW_DS;
    if (st == FGI_CONSISTENT) return (w & (kVMask | kW_HasDelay)) | kW_Invalidated;
    return w;
}

// One visit of node h (word w, version already matched): a single atomicOr on the visit bitmap.
__device__ __forceinline__ int visit_bit(uint32_t* vis, uint32_t h, unsigned long long w) {
    const uint32_t b = 1u << (h & 31);
    if (atomicOr(vis + (h >> 5), b) & b) return 0;
    return first_visit(w);
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

__device__ __forceinline__ unsigned long long wave_sum64(unsigned long long v) {
#pragma unroll
    for (int d = 32; d >= 1; d >>= 1) v += __shfl_xor(v, d, 64);
    return v;
}

__device__ __forceinline__ unsigned long long lanemask_lt() { return (1ull << lane_id()) - 1ull; }

// Where a level's winners go: the invalidated list (all winners) and the next frontier (winners
// with a non-empty row: row offset and length); the next level's F and T accumulate in ln.
struct Out {
    const uint64_t* __restrict__ row_off;
    const uint32_t* __restrict__ row_len;
    uint32_t* __restrict__ inv;
    uint32_t* __restrict__ nfr_off;   // row offsets (edge pool positions < 2^32)
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

// Per-block statistics: hot kernels keep their counters per block (plain read-modify-write of the
// block's own column entry by one thread, launches of a wave are stream-ordered) instead of per-wave
// atomics on a few words: a single device-scope word saturates near 88 atomics/us. Column-major
// ([column][block]) so k_stats_reduce sweeps each column coalesced.
enum : int { kStEMatch, kStFlagged, kStPullCand, kStPullEdges, kStPullLive, kStPullWin, kStPullTail, kStPullScan, kStats };
static_assert(kStats == kStatCols, "statistics columns");

// Block-uniform call: adds each thread's v[k] into the block's entries.
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
        for (uint32_t q = 0; q < blockDim.x / 64; ++q) t += s[q][threadIdx.x];
        if (t) blk[(uint64_t)threadIdx.x * kStatBlocks + blockIdx.x] += t;
    }
}

// Append one (possibly absent) winner per lane. Every lane of the wave must call it.
__device__ __forceinline__ void emit_one(bool win, uint32_t h, const Out& o) {
    const uint32_t len = win ? o.row_len[h] : 0u;
    const uint32_t off = (win && len) ? (uint32_t)o.row_off[h] : 0u;
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

// Block-level emission (push levels): winners are staged in LDS and appended to the global lists
// in batches (one pair of global atomics per batch instead of one per wave per iteration).
constexpr uint32_t kEmitCap = 1024;
constexpr uint32_t kChunkEmitCap = 2 * kChunk;   // push levels: staged over the chunk map
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
        const uint32_t idx = base + (uint32_t)__popcll(m & lanemask_lt());
        if (idx < CAP) {
            buf[idx] = h;
        } else {
            o.inv[atomicAdd(o.inv_ctr, 1ull)] = h;
            const uint32_t len = o.row_len[h];
            if (len) {
                const unsigned long long fb = atomicAdd(&o.ln->F, 1ull);
                o.nfr_off[fb] = (uint32_t)o.row_off[h];
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
    // the three counters from three waves, so the atomics are in flight together
    if (threadIdx.x == 0) e.base_inv = atomicAdd(o.inv_ctr, (unsigned long long)n);
    if (threadIdx.x == 64) e.base_fr = total ? atomicAdd(&o.ln->F, (unsigned long long)total) : 0ull;
    if (threadIdx.x == 128) {
        unsigned long long tl = 0;
        for (uint32_t k = 0; k < kBlock / 64; ++k) tl += e.wlen[k];
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
                o.nfr_off[fb] = (uint32_t)o.row_off[h];
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
        const uint32_t idx = base + (uint32_t)__popcll(m & lanemask_lt());
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
// handle's current node, no tag check. Global root ids; this device owns [base, base + n_range).
// IMM = 1: only the roots with immediately[i] set (Invalidate(true) ignores the delay, so it can
// change the node word; CAS on the word with the visit bit folded in), launched before IMM = 0,
// which visits the other roots through the visit bitmap.
template <int IMM>
__global__ __launch_bounds__(kBlock) void k_roots(const uint32_t* __restrict__ roots, const uint8_t* __restrict__ imm,
                                                  uint32_t n, uint32_t base, uint32_t n_range, unsigned long long* node,
                                                  uint32_t* vis, Out o, WaveCtr* ctr) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    uint32_t win = 0, flagged = 0, h = 0;
    if (i < n) {
        h = roots[i] - base;
        const bool is_imm = imm ? imm[i] != 0 : false;
        if (h < n_range && is_imm == (IMM != 0)) {
            unsigned long long w = node[h];
            if ((w & kVMask) != 0) {
                int r = 0;
                if (IMM) {
                    const bool v = bit_of(vis, h);
                    while (true) {
                        const unsigned long long cw = v ? visited_word(w) : w;
                        const unsigned long long nw = imm_word(cw);
                        if (nw == cw) break;
                        const unsigned long long prev = atomicCAS(node + h, w, nw);
                        if (prev == w) {
                            r = (word_state(nw) == FGI_INVALIDATED) ? 1 : 2;
                            break;
                        }
                        w = prev;
                    }
                    if (r == 1) atomicOr(vis + (h >> 5), 1u << (h & 31));
                } else {
                    r = visit_bit(vis, h, w);
                }
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
constexpr int kScanThreads = 256;   // threads per block of the collect / scan kernel (k_scan_apply): at its
                                     // register budget (4 waves/SIMD) all kScanBlocks blocks are resident
constexpr int kMaxWaves = kScanThreads / 64;

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

// Called by every block of a pass-1 grid with its per-block sums v[q] (q < ncols) in thread 0: the
// last block to finish turns src's columns into exclusive prefixes dst[q * G + k] and totals
// dst[3 * G + q] — O(G) work, instead of every pass-2 block re-reading all G sums. The sums and the
// counter are agent-scope atomic RMWs, performed at the coherence point shared by the XCDs (their
// L2s are not coherent with each other); a block's counter increment is issued only after its sum
// exchanges have returned, so the last block reads every sum. No L2 write-back fence is needed.
constexpr int kDoneGroups = 16;
constexpr int kDoneStride = 16;
__device__ __forceinline__ unsigned long long coh_xchg(unsigned long long* p, unsigned long long v) {
    return __hip_atomic_exchange(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ unsigned long long coh_read(unsigned long long* p) {
    return __hip_atomic_fetch_add(p, 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// The completion counter is two-level (one counter word serialises near 88 atomics/us,
// MI355X_MICROARCH.md): block b counts into group b % kDoneGroups, the last block of a group into
// the top word done[0]; groups live kDoneStride words (128 B) apart.
__device__ void finish_prefix(unsigned long long* src, unsigned long long* dst, int ncols, uint64_t G,
                              unsigned long long* done, unsigned long long* s_red, const unsigned long long* v) {
    __shared__ bool s_last;
    if (threadIdx.x == 0) {
        unsigned long long r = 0;
        for (int q = 0; q < ncols; ++q) r |= coh_xchg(src + q * G + blockIdx.x, v[q]);
        __builtin_amdgcn_s_waitcnt(0);   // the exchanges have been performed
        const uint32_t grp = blockIdx.x % kDoneGroups;
        const uint64_t gsize = (G - grp + kDoneGroups - 1) / kDoneGroups;
        const unsigned long long t = __hip_atomic_fetch_add(done + (1 + grp) * kDoneStride, 1ull + (r & 0ull),
                                                            __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        bool last = false;
        if (t == gsize - 1) {
            __builtin_amdgcn_s_waitcnt(0);
            const uint64_t ng = G < (uint64_t)kDoneGroups ? G : (uint64_t)kDoneGroups;
            last = __hip_atomic_fetch_add(done, 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == ng - 1;
        }
        s_last = last;
    }
    __syncthreads();
    if (!s_last) return;
    // every sum this thread needs is read in one round (G <= kScanBlocks, blockDim.x == kBlock)
    constexpr uint32_t kPer = (kScanBlocks + kBlock - 1) / kBlock;
    const uint64_t k0 = (uint64_t)threadIdx.x * kPer;
    const uint32_t lane = lane_id(), wid = threadIdx.x >> 6;
    unsigned long long xs[3][kPer];
#pragma unroll
    for (int q = 0; q < 3; ++q)
#pragma unroll
        for (uint32_t j = 0; j < kPer; ++j) xs[q][j] = (q < ncols && k0 + j < G) ? coh_read(src + q * G + k0 + j) : 0ull;
#pragma unroll
    for (int q = 0; q < 3; ++q) {
        if (q >= ncols) break;
        unsigned long long loc = 0;
#pragma unroll
        for (uint32_t j = 0; j < kPer; ++j) loc += xs[q][j];
        unsigned long long x = loc;
#pragma unroll
        for (int d = 1; d < 64; d <<= 1) {
            const unsigned long long y = __shfl_up(x, d, 64);
            if (lane >= (uint32_t)d) x += y;
        }
        __syncthreads();
        if (lane == 63) s_red[wid] = x;
        __syncthreads();
        unsigned long long run = x - loc, tot = 0;
        for (uint32_t k = 0; k < (blockDim.x >> 6); ++k) {
            if (k < wid) run += s_red[k];
            tot += s_red[k];
        }
#pragma unroll
        for (uint32_t j = 0; j < kPer; ++j)
            if (k0 + j < G) {
                dst[q * G + k0 + j] = run;
                run += xs[q][j];
            }
        if (threadIdx.x == 0) dst[3 * G + q] = tot;
    }
    if (threadIdx.x <= (uint32_t)kDoneGroups) coh_xchg(done + threadIdx.x * kDoneStride, 0ull);
}

__device__ __forceinline__ void scan_partial(uint64_t F, const uint32_t* __restrict__ fr_len,
                                             unsigned long long* __restrict__ partials, unsigned long long* s_red,
                                             unsigned long long* done) {
    const uint64_t b = blockIdx.x, G = gridDim.x;
    const uint64_t lo = F * b / G, hi = F * (b + 1) / G;
    unsigned long long s = 0;
    for (uint64_t i = lo + threadIdx.x; i < hi; i += blockDim.x) s += fr_len[i];
    s = block_sum(s, s_red);
    const unsigned long long v[1] = {s};
    finish_prefix(partials, partials + 4 * G, 1, G, done, s_red, v);   // prefixes for k_scan_apply
}

__device__ __forceinline__ void probe_at(unsigned long long* pr, int k);

// ---- collect: a pull level's winners bitmap -> invalidated list (+ next frontier) -------------
// The pull level counted its winners per tile (kPullTile slots; tile t = iteration * pgrid + block,
// slots [it * pgrid * kPullTile + block * kPullTile, +kPullTile)). Pass 1 sums the tiles of every
// block of the collect grid; pass 2 turns each tile's bitmap words into list entries at offsets
// from those sums — deterministic, no atomics. Entries come out in tile order.
struct CollectArgs {
    const PullTile* __restrict__ tiles;
    uint64_t n_tiles;
    uint32_t pgrid, n_slots;
    uint32_t* fb;                // winners bitmap of the pull level
    uint32_t n_handles;          // rows: row_len has n_handles entries
    int fr_multi;                // multi-GPU collects: also write the frontier list (the next level pushes)
    const uint32_t* __restrict__ row_len;
    uint32_t* inv;
    const uint64_t* __restrict__ row_off;
    uint32_t* fr_off;
    uint32_t* fr_len;
    uint64_t* escan;
    uint32_t* cstart;
    unsigned long long* part3;   // [3][G] pass-1 sums: winners, expandable winners, row lengths
    uint64_t stay_pull_f;        // a pull level is followed by another while the frontier exceeds this
    unsigned long long* probe;   // measurement only (FGI_PROBE): phase stamps of collect pass 2
    unsigned long long* pre3;    // [3][G] exclusive prefixes of part3's columns, then the 3 totals
    unsigned long long* done;    // pass-1 blocks finished (the last one scans part3; zero between uses)
};

__device__ __forceinline__ void collect_pass1(const CollectArgs& c, unsigned long long* s_red) {
    const uint64_t b = blockIdx.x, G = gridDim.x;
    const uint64_t lo = c.n_tiles * b / G, hi = c.n_tiles * (b + 1) / G;
    unsigned long long w = 0, e = 0, l = 0;
    for (uint64_t t = lo + threadIdx.x; t < hi; t += blockDim.x) {
        const PullTile x = c.tiles[t];
        w += x.w;
        e += x.e;
        l += x.len;
    }
    w = block_sum(w, s_red);
    e = block_sum(e, s_red);
    l = block_sum(l, s_red);
    const unsigned long long v[3] = {w, e, l};
    finish_prefix(c.part3, c.pre3, 3, G, c.done, s_red, v);
}

// One tile by one wave: lane l owns the 16 slots s0 + 16l .. s0 + 16l + 15 (one 16-bit chunk of the
// winners bitmap). Two wave scans place every lane's entries (winners; expandable winners and their
// row lengths); the entries are staged in the wave's LDS buffer and stored coalesced, in slot order,
// at bw (inv) and be / bl (frontier index / edge offset). write_fr: also the frontier entries, their
// scan and the chunk map.
// The lane's 16-bit chunk of tile t's winners bitmap (loaded ahead of the tile's collect).
__device__ __forceinline__ uint32_t collect_bits(const CollectArgs& c, uint64_t t) {
    const uint64_t base = t * kPullTile + 16ull * lane_id();
    return base < c.n_slots ? (uint32_t)reinterpret_cast<const uint16_t*>(c.fb)[base / 16] : 0u;
}

__device__ __forceinline__ void collect_tile(const CollectArgs& c, uint64_t t, uint32_t m, uint64_t bw, uint64_t be,
                                             uint64_t bl, bool write_fr, uint32_t* __restrict__ stage) {
    const uint32_t lane = lane_id();
    const uint64_t s0 = t * kPullTile;   // tile t = it * pgrid + block covers slots [t * kPullTile, +kPullTile)
    const uint64_t base = s0 + 16ull * lane;
    uint32_t rl[16];
    uint32_t em = 0, len = 0;
#pragma unroll
    for (int k = 0; k < 16; ++k) rl[k] = 0;
    if (write_fr && m) {
        if (base + 16 <= c.n_handles) {
            const uint4* p = reinterpret_cast<const uint4*>(c.row_len + base);
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                const uint4 v = p[q];
                rl[4 * q] = v.x;
                rl[4 * q + 1] = v.y;
                rl[4 * q + 2] = v.z;
                rl[4 * q + 3] = v.w;
            }
        } else {
#pragma unroll
            for (int k = 0; k < 16; ++k) rl[k] = ((m >> k) & 1u) ? c.row_len[base + k] : 0u;
        }
#pragma unroll
        for (int k = 0; k < 16; ++k) {
            if (!((m >> k) & 1u)) rl[k] = 0;
            em |= (rl[k] != 0 ? 1u : 0u) << k;
            len += rl[k];
        }
    }
    uint32_t tot_p, tot_l;
    const uint32_t pw = wave_excl_scan((uint32_t)__popc(m) | ((uint32_t)__popc(em) << 16), tot_p);
    const uint32_t pl = write_fr ? wave_excl_scan(len, tot_l) : 0u;
    const uint32_t n_w = tot_p & 0xFFFFu, n_e = tot_p >> 16;
    // winners -> inv
    {
        uint32_t o = pw & 0xFFFFu;
        for (uint32_t mm = m; mm; mm &= mm - 1) stage[o++] = (uint32_t)base + (uint32_t)(__ffs(mm) - 1);
        __builtin_amdgcn_wave_barrier();
        for (uint32_t i = lane; i < n_w; i += 64) c.inv[bw + i] = stage[i];
        __builtin_amdgcn_wave_barrier();
    }
    if (!write_fr || n_e == 0) return;
    // expandable winners -> fr_len, escan (+ cstart for every chunk whose first edge they hold), fr_off
    const uint32_t pe = pw >> 16;
    {
        uint32_t o = pe;
#pragma unroll
        for (int k = 0; k < 16; ++k)
            if (rl[k]) stage[o++] = rl[k];
        __builtin_amdgcn_wave_barrier();
        for (uint32_t i = lane; i < n_e; i += 64) c.fr_len[be + i] = stage[i];
        __builtin_amdgcn_wave_barrier();
    }
    {
        uint32_t o = pe, r = pl;
#pragma unroll
        for (int k = 0; k < 16; ++k) {
            if (!rl[k]) continue;
            const uint64_t es = bl + r, idx = be + o;
            const uint64_t c_lo = (es + kChunk - 1) / kChunk, c_hi = (es + rl[k] - 1) / kChunk;
            for (uint64_t q = c_lo; q <= c_hi; ++q) c.cstart[q] = (uint32_t)idx;
            stage[o++] = r;
            r += rl[k];
        }
        __builtin_amdgcn_wave_barrier();
        for (uint32_t i = lane; i < n_e; i += 64) c.escan[be + i] = bl + stage[i];
        __builtin_amdgcn_wave_barrier();
    }
    {
        // row offsets of the expandable slots only (sparse: a whole 128-B run per lane would fetch
        // mostly unused offsets); low words suffice, pool positions are < 2^32
        const uint32_t* off32 = reinterpret_cast<const uint32_t*>(c.row_off);
        uint32_t ro[16];
#pragma unroll
        for (int k = 0; k < 16; ++k) ro[k] = ((em >> k) & 1u) ? off32[2 * (base + k)] : 0u;
        uint32_t o = pe;
#pragma unroll
        for (int k = 0; k < 16; ++k)
            if ((em >> k) & 1u) stage[o++] = ro[k];
        __builtin_amdgcn_wave_barrier();
        for (uint32_t i = lane; i < n_e; i += 64) c.fr_off[be + i] = stage[i];
        __builtin_amdgcn_wave_barrier();
    }
}

// Pass 2 (kScanThreads-thread blocks, same grid as pass 1); block 0 publishes the level's totals.
// single: the push/pull decision for this level is made here and the frontier list is written
// only for a push; multi-GPU levels always write it (the drivers decide after an all-reduce).
__device__ __forceinline__ void collect_pass2(const CollectArgs& c, LevelCtr& lc, WaveCtr* ctr, bool single,
                                              int direction, uint64_t pull_threshold, uint32_t* fb_nxt,
                                              uint64_t slot_words, unsigned long long* s_red) {
    __shared__ uint32_t s_ow[64], s_oe[64], s_nz[64];
    __shared__ unsigned long long s_ol[64], s_tot[3];
    __shared__ uint32_t s_stage[kMaxWaves][kPullTile];   // per-wave staging of one tile's entries
    if (c.probe && threadIdx.x == 0 && blockIdx.x < kProbeBlocks)
        c.probe[blockIdx.x * kProbePhases] = __builtin_amdgcn_s_memrealtime();
    const uint64_t b = blockIdx.x, G = gridDim.x;
    // the block's offsets (sums over blocks < b) and the level totals: every pass-1 sum is loaded
    // at once (kScanBlocks / kScanThreads per thread, independent loads), one fused reduction
    const uint64_t inv_base = lc.mark_lo;   // set by pass 1's kernel
    const unsigned long long bw = c.pre3[b], be = c.pre3[G + b], bl = c.pre3[2 * G + b];
    const unsigned long long tw = c.pre3[3 * G], te = c.pre3[3 * G + 1], tl = c.pre3[3 * G + 2];
    // Beamer's two rules: pull when the frontier's edges exceed E / alpha; after a pull, keep pulling
    // while the frontier holds more than n / beta nodes (a large frontier of short rows is cheaper
    // to pull than to expand edge by edge)
    const bool pull = single && te != 0 &&
                      (direction == 2 || (direction == 0 && (tl > pull_threshold || te > c.stay_pull_f)));
    const bool write_fr = single ? !pull : c.fr_multi != 0;
    __syncthreads();   // block 0's threads have all read lc.mark_lo before thread 0 writes lc
    if (b == 0 && threadIdx.x == 0) {
        lc.F = te;
        lc.T = tl;
        lc.nchunks = (tl + kChunk - 1) / kChunk;
        lc.pull = pull ? 1ull : 0ull;
        lc.mark_hi = inv_base + tw;
        ctr->inv = inv_base + tw;
    }
    // a push level after a pull: the next frontier bitmap (last written by the pull before) is
    // cleared so a later push->pull switch marks into an empty one
    if (single && !pull) {
        const uint64_t nthr = G * blockDim.x;
        for (uint64_t w = b * blockDim.x + threadIdx.x; w < slot_words; w += nthr) fb_nxt[w] = 0u;
    }
    probe_at(c.probe, 2);
    const uint64_t lo = c.n_tiles * b / G, hi = c.n_tiles * (b + 1) / G;
    const uint32_t W = blockDim.x >> 6, wid = threadIdx.x >> 6, lane = lane_id();
    uint64_t rw = inv_base + bw, re = be, rl = bl;
    // chunks of up to 64 tiles: wave 0 loads their counts and scans them (offsets within the
    // chunk into LDS), then the waves take the chunk's tiles round-robin with no further barrier
    for (uint64_t cb = lo; cb < hi; cb += 64) {   // block-uniform
        const uint32_t nt = (uint32_t)std::min<uint64_t>(64, hi - cb);
        if (wid == 0) {
            PullTile x{0, 0, 0ull};
            if (lane < nt) x = c.tiles[cb + lane];
            uint32_t tw_, te_;
            const uint32_t ow = wave_excl_scan(x.w, tw_), oe = wave_excl_scan(x.e, te_);
            unsigned long long il = x.len;
#pragma unroll
            for (int d = 1; d < 64; d <<= 1) {
                const unsigned long long y = __shfl_up(il, d, 64);
                if (lane >= (uint32_t)d) il += y;
            }
            s_ow[lane] = ow;
            s_oe[lane] = oe;
            s_ol[lane] = il - x.len;
            s_nz[lane] = x.w;
            if (lane == 63) {
                s_tot[0] = tw_;
                s_tot[1] = te_;
                s_tot[2] = il;
            }
        }
        __syncthreads();
        // the next tile's bitmap chunk is loaded while the current one is collected
        uint32_t j = wid;
        while (j < nt && !s_nz[j]) j += W;
        uint32_t m = j < nt ? collect_bits(c, cb + j) : 0u;
        while (j < nt) {
            uint32_t jn = j + W;
            while (jn < nt && !s_nz[jn]) jn += W;
            const uint32_t mn = jn < nt ? collect_bits(c, cb + jn) : 0u;
            collect_tile(c, cb + j, m, rw + s_ow[j], re + s_oe[j], rl + s_ol[j], write_fr, s_stage[wid]);
            j = jn;
            m = mn;
        }
        rw += s_tot[0];
        re += s_tot[1];
        rl += s_tot[2];
        if (cb == lo) probe_at(c.probe, 3);
        __syncthreads();   // the next chunk overwrites the offsets
    }
    probe_at(c.probe, 10);
}

// multi-GPU levels: partial sums of the frontier's row lengths, or collect pass 1 after a pull
__global__ __launch_bounds__(kBlock) void k_scan_reduce(int L, const uint32_t* __restrict__ fr_len,
                                                        unsigned long long* __restrict__ partials,
                                                        WaveCtr* ctr, CollectArgs ca) {
    __shared__ unsigned long long s_red[kBlock / 64];
    if (L > 0 && ctr->lvl[(L + kRing - 1) % kRing].pull) {
        if (blockIdx.x == 0 && threadIdx.x == 0) ctr->lvl[L % kRing].mark_lo = ctr->inv;
        collect_pass1(ca, s_red);
        return;
    }
    scan_partial(ctr->lvl[L % kRing].F, fr_len, partials, s_red, ca.done);
}

// Single-GPU level prologue (one launch, grid kScanBlocks):
//  - after a push level (or the roots): the push/pull decision for level L from the frontier
//    totals F, T its producers accumulated; its winners inv[mark_hi(L-1), inv) are marked into the
//    frontier bitmap fb_cur if level L pulls; fb_nxt is cleared when level L pushes, so a later
//    push->pull switch finds it empty; partial sums of the frontier's row lengths on a push;
//  - after a pull level: collect pass 1 (the decision follows in k_scan_apply).
__global__ __launch_bounds__(kBlock) void k_level_begin(int L, WaveCtr* ctr, const uint32_t* __restrict__ inv,
                                                        uint32_t* fb_cur, uint32_t* fb_nxt, uint64_t bm_words,
                                                        uint64_t slot_words, const uint32_t* __restrict__ fr_len,
                                                        unsigned long long* __restrict__ partials, int direction,
                                                        uint64_t pull_threshold, CollectArgs ca) {
    __shared__ unsigned long long s_red[kBlock / 64];
    LevelCtr& lc = ctr->lvl[L % kRing];
    const uint64_t tid = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const uint64_t nthr = (uint64_t)gridDim.x * blockDim.x;
    const bool prev_pull = L > 0 && ctr->lvl[(L + kRing - 1) % kRing].pull != 0;
    if (prev_pull) {
        if (tid == 0) lc.mark_lo = ctr->inv;
        // words past the slots (detached handles) are never written by a pull: keep them zero
        for (uint64_t w = slot_words + tid; w < bm_words; w += nthr) fb_nxt[w] = 0u;
        collect_pass1(ca, s_red);
        return;
    }
    const uint64_t F = lc.F, T = lc.T;
    const bool pull = F != 0 && (direction == 2 || (direction == 0 && T > pull_threshold));
    const uint64_t lo = L > 0 ? ctr->lvl[(L + kRing - 1) % kRing].mark_hi : 0ull;
    const uint64_t hi = ctr->inv;
    if (tid == 0) {
        lc.pull = pull ? 1ull : 0ull;
        lc.nchunks = (T + kChunk - 1) / kChunk;
        lc.mark_lo = lo;
        lc.mark_hi = hi;
    }
    if (pull) {
        for (uint64_t i = lo + tid; i < hi; i += nthr) {
            const uint32_t h = inv[i];
            atomicOr(fb_cur + (h >> 5), 1u << (h & 31));
        }
    }
    // a pull at level L stores every slot word of fb_nxt; the words past the slots (detached
    // handles) are never winners of a pull and must read as zero
    for (uint64_t w = (pull ? slot_words : 0ull) + tid; w < bm_words; w += nthr) fb_nxt[w] = 0u;
    if (!pull && F) scan_partial(F, fr_len, partials, s_red, ca.done);
}

// Exclusive scan of fr_len into escan; records for every chunk of kChunk edges the frontier
// entry holding its first edge (cstart). decide = 1 (multi-GPU levels): also sets T, nchunks and
// a push decision (the driver overrides it for pull levels); decide = 0: k_level_begin decided.
// After a pull level: collect pass 2 instead. kScanThreads-thread blocks.
__global__ __launch_bounds__(kScanThreads, 4) void k_scan_apply(int L, const uint32_t* __restrict__ fr_len,
                                                     const unsigned long long* __restrict__ partials,
                                                     uint64_t* __restrict__ escan, uint32_t* __restrict__ cstart,
                                                     WaveCtr* ctr, int decide, CollectArgs ca, int direction,
                                                     uint64_t pull_threshold, uint32_t* fb_nxt, uint64_t slot_words) {
    __shared__ unsigned long long s_red[kMaxWaves];
    __shared__ unsigned long long s_wave[kMaxWaves];
    LevelCtr& lc = ctr->lvl[L % kRing];
    if (L > 0 && ctr->lvl[(L + kRing - 1) % kRing].pull) {
        collect_pass2(ca, lc, ctr, !decide, direction, pull_threshold, fb_nxt, slot_words, s_red);
        return;
    }
    const uint64_t F = lc.F;
    if (!decide && (lc.pull || F == 0)) return;
    const uint64_t b = blockIdx.x, G = gridDim.x;
    // exclusive prefix and total of the per-block sums (the last pass-1 block wrote them)
    const unsigned long long before = partials[4 * G + b], all = partials[7 * G];
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
// The previous level's winners (pushed, received or collected after a pull: the range [marked,
// inv)) become the frontier bitmap of a pull level.
__global__ __launch_bounds__(kBlock) void k_mark(int L, const uint32_t* __restrict__ inv, uint32_t* front_bm,
                                                 WaveCtr* ctr, int copied) {
    LevelCtr& lc = ctr->lvl[L % kRing];
    const uint64_t lo = ctr->marked, hi = ctr->inv;
    if (blockIdx.x == 0 && threadIdx.x == 0) {
        lc.mark_lo = lo;
        lc.mark_hi = hi;
    }
    if (!lc.pull || copied) return;   // copied: the previous pull's winners bitmap was copied in whole
    for (uint64_t i = lo + (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < hi;
         i += (uint64_t)gridDim.x * blockDim.x) {
        const uint32_t h = inv[i];
        atomicOr(front_bm + (h >> 5), 1u << (h & 31));
    }
}

// Tile totals of a pull level into the next level's F and T, and its winner count into pad0
// (winners still to be collected into the invalidated list; one block).
__device__ __forceinline__ void tile_totals(const PullTile* __restrict__ tiles, uint64_t n_tiles, LevelCtr& ln,
                                            unsigned long long* s_red) {
    unsigned long long w = 0, e = 0, l = 0;
    for (uint64_t t = threadIdx.x; t < n_tiles; t += blockDim.x) {
        w += tiles[t].w;
        e += tiles[t].e;
        l += tiles[t].len;
    }
    w = block_sum(w, s_red);
    e = block_sum(e, s_red);
    l = block_sum(l, s_red);
    if (threadIdx.x == 0) {
        ln.F = e;
        ln.T = l;
        ln.pad0 = w;
    }
}

__global__ __launch_bounds__(kBlock) void k_clear_front(int L, const uint32_t* __restrict__ inv, uint32_t* front_bm,
                                                        WaveCtr* ctr, const PullTile* __restrict__ tiles,
                                                        uint64_t n_tiles, int wiped) {
    __shared__ unsigned long long s_red[kBlock / 64];
    LevelCtr& lc = ctr->lvl[L % kRing];
    const uint64_t lo = lc.mark_lo, hi = lc.mark_hi;
    if (blockIdx.x == 0 && threadIdx.x == 0) ctr->marked = hi;
    if (!lc.pull) return;
    if (blockIdx.x == 0) tile_totals(tiles, n_tiles, ctr->lvl[(L + 1) % kRing], s_red);
    if (wiped) return;   // the host cleared the whole bitmap (one memset instead of a store per winner)
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
    const uint32_t* __restrict__ fr_off;
    const uint64_t* __restrict__ escan;
    const uint32_t* __restrict__ cstart;
    const uint32_t* __restrict__ pool_col;
    const uint64_t* __restrict__ pool_tag;
    int dead_filter;
    unsigned long long* probe;   // measurement only (FGI_PROBE): per-block phase timestamps, else null
};

// FGI_PROBE: all of the block's memory operations drained, then a 100 MHz timestamp for phase k
__device__ __forceinline__ void probe_at(unsigned long long* pr, int k) {
    if (!pr) return;
    __builtin_amdgcn_s_waitcnt(0);
    __syncthreads();
    if (threadIdx.x == 0 && blockIdx.x < kProbeBlocks) pr[blockIdx.x * kProbePhases + k] = __builtin_amdgcn_s_memrealtime();
}

// PART: multi-GPU rank — dependant slots outside [ra.base, ra.base + ra.n_local) are remote: their
// tag is checked against the version replica and matching targets are forwarded once per wave.
template <bool PART>
__device__ __forceinline__ void expand_level(const LevelCtr& lc, const ExpandArgs& x, const unsigned long long* node,
                                             uint32_t* vis, const Out& o, Emit& em, uint32_t* eb, MsgEmit<PART>& me,
                                             uint32_t* s_rel, uint32_t* s_base, unsigned long long* blk,
                                             unsigned long long (*s_st)[kStats], const RemoteArgs& ra) {
    if constexpr (PART) {
        if (threadIdx.x == 0) me.n = 0;
    }
    const uint64_t T = lc.T, F = lc.F, nch = lc.nchunks;
    uint32_t matched = 0, flagged = 0;
    probe_at(x.probe, 1);
    for (uint64_t c = blockIdx.x; c < nch; c += gridDim.x) {
        const uint64_t cbase = c * kChunk;
        const uint32_t clen = (uint32_t)((T - cbase) < (uint64_t)kChunk ? (T - cbase) : (uint64_t)kChunk);
        const uint32_t i0 = x.cstart[c];
        const uint32_t i1 = (c + 1 < nch) ? x.cstart[c + 1] : (uint32_t)(F - 1);
        const uint32_t n = i1 - i0 + 1;
        // n <= kChunk + 1 entries: every load issued before the first use
        uint64_t fes[kEPT + 1];
        uint32_t fof[kEPT + 1];
#pragma unroll
        for (int j = 0; j <= kEPT; ++j) {
            const uint32_t k = threadIdx.x + j * kBlock;
            fes[j] = k < n ? x.escan[i0 + k] : 0ull;
            fof[j] = k < n ? x.fr_off[i0 + k] : 0u;
        }
#pragma unroll
        for (int j = 0; j <= kEPT; ++j) {
            const uint32_t k = threadIdx.x + j * kBlock;
            if (k < n) {
                s_rel[k] = fes[j] > cbase ? (uint32_t)(fes[j] - cbase) : 0u;
                s_base[k] = (uint32_t)((uint64_t)fof[j] + cbase - fes[j]);   // pool positions < 2^32
            }
        }
        __syncthreads();
        probe_at(x.probe, 2);
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
        probe_at(x.probe, 3);
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
        // edges to nodes visited earlier need neither the tag nor the gather (the bitmap is read
        // without synchronisation: a stale 0 only costs the gather and an atomic that finds the bit)
        if (x.dead_filter) {
#pragma unroll
            for (int j = 0; j < kEPT; ++j)
                if (dst[j] != 0xFFFFFFFFu && bit_of(vis, dst[j])) dst[j] = 0xFFFFFFFFu;
        }
        probe_at(x.probe, 4);
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
        probe_at(x.probe, 5);
        uint32_t win_mask = 0;
#pragma unroll
        for (int j = 0; j < kEPT; ++j) {
            if (tag[j] != 0 && (w[j] & kVMask) == tag[j]) {
                ++matched;
                const int r = visit_bit(vis, dst[j], w[j]);
                if (r == 1) win_mask |= 1u << j;
                else if (r == 2) ++flagged;
            }
        }
        probe_at(x.probe, 6);
        // the chunk's winners (at most kChunk) are staged over the chunk map, flushed before the
        // next chunk refills it
        __syncthreads();
#pragma unroll
        for (int j = 0; j < kEPT; ++j) emit_push<kChunkEmitCap>(em, eb, (win_mask >> j) & 1u, dst[j], o);
        probe_at(x.probe, 7);
        emit_flush<kChunkEmitCap>(em, eb, 1, o);
        probe_at(x.probe, 8);
        if constexpr (PART) msg_flush(me, kMsgCap / 2, ra);
    }
    probe_at(x.probe, 9);
    if constexpr (PART) msg_flush(me, 1, ra);
    const uint32_t v[kStats] = {matched, flagged, 0, 0, 0, 0, 0, 0};
    block_stats_add(blk, s_st, v);
    probe_at(x.probe, 10);
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
    const uint32_t* __restrict__ uin_more;   // bitmap: the list has more than two entries
    const uint32_t* __restrict__ front_rd;   // frontier bitmap (handles; multi-GPU: global ids)
    uint32_t* front_wr;                      // this level's winners, stored whole per tile
    const uint32_t* __restrict__ cls;        // expandable-class bitmap
    const uint32_t* __restrict__ row_len;
    PullTile* tiles;
    unsigned long long* probe;   // measurement only (FGI_PROBE)
};

// A block owns tile (it, block) of every iteration: kPullTile consecutive slots, kPS per lane
// (64 apart), so a lane issues kPS independent loads of each kind. Per slot: the visit, class and
// "more" bitmap words (one 64-bit word per 64 slots), the two list heads and the row length, all
// unconditional and coalesced; then the frontier bits of the heads (L2); a hit is a visit. The
// wave's visits and wins go to LDS as 64-bit ballot words; slots whose heads missed but whose
// list goes on are queued in LDS and scanned at the flush by 8-lane groups (8 entries per probe
// step, early exit). The flush (every kMaxIter iterations and at the end) writes the owned
// visit and frontier words and the per-tile counts — a pull level does no global atomics.
constexpr uint32_t kPS = kPullTile / kBlock;
constexpr uint32_t kMaxIter = 16;           // iterations buffered in LDS between flushes
constexpr uint32_t kTailCap = kChunk;       // queued slots (s_rel)
constexpr uint32_t kTileWords = kPullTile / 64;
static_assert(kPS == 4 && kTileWords == 16, "pull geometry");

__device__ __forceinline__ void pull_flush(const PullArgs& p, const unsigned long long* node, uint32_t* vis,
                                           uint32_t it_base, uint32_t nbuf, const uint32_t* q, uint32_t nq,
                                           unsigned long long* s_vm, unsigned long long* s_wm, uint32_t* s_cw,
                                           uint32_t* s_ce, unsigned long long* s_cl, uint32_t& flagged,
                                           uint32_t& examined, uint32_t& wins, uint32_t& tails) {
    const uint64_t stride = (uint64_t)gridDim.x * kPullTile;
    const uint32_t lane = lane_id(), sub = lane & 7, grp = threadIdx.x >> 3;
    __syncthreads();
    // queued slots: 8 lanes per slot, entries 2.. of its list; the next slot's list length and
    // offset are loaded while the current list is scanned
    const uint32_t G8 = blockDim.x / 8;
    uint32_t d_n = 0, len_n = 0;
    uint64_t off_n = 0;
    if (grp < nq) {
        d_n = q[grp];
        len_n = p.uin_len[d_n];
        off_n = p.uin_off[d_n];
    }
    for (uint32_t e = grp; e < nq; e += G8) {
        const uint32_t d = d_n, len = len_n;
        const uint64_t off = off_n;
        if (e + G8 < nq) {
            d_n = q[e + G8];
            len_n = p.uin_len[d_n];
            off_n = p.uin_off[d_n];
        }
        bool found = false;
        for (uint32_t r = 2; r < len && !found; r += 8) {   // group-uniform
            const uint32_t i = r + sub;
            const bool x = i < len && bit_of(p.front_rd, p.uin_src[off + i]);
            examined += (i < len) ? 1u : 0u;
            found = ((__ballot(x) >> (lane & ~7u)) & 0xFFull) != 0;
        }
        if (found && sub == 0) {
            const uint64_t it = d / stride;
            const uint32_t k = (uint32_t)(it - it_base);
            const uint32_t wq = (uint32_t)((d - it * stride - (uint64_t)blockIdx.x * kPullTile) >> 6);
            const unsigned long long bit = 1ull << (d & 63);
            atomicOr(&s_vm[k * kTileWords + wq], bit);
            if (bit_of(p.cls, d)) {
                atomicOr(&s_wm[k * kTileWords + wq], bit);
                const uint32_t rl = p.row_len[d];
                atomicAdd(&s_cw[k], 1u);
                if (rl) {
                    atomicAdd(&s_ce[k], 1u);
                    atomicAdd(&s_cl[k], (unsigned long long)rl);
                }
                ++wins;
            } else {
                flagged += first_visit(node[d]) == 2 ? 1u : 0u;
            }
        }
        tails += sub == 0 ? 1u : 0u;
    }
    __syncthreads();
    unsigned long long* vis64 = reinterpret_cast<unsigned long long*>(vis);
    unsigned long long* fw64 = reinterpret_cast<unsigned long long*>(p.front_wr);
    for (uint32_t i = threadIdx.x; i < nbuf * kTileWords; i += blockDim.x) {
        const uint32_t k = i / kTileWords, wq = i % kTileWords;
        const uint64_t s = (it_base + k) * stride + (uint64_t)blockIdx.x * kPullTile + (uint64_t)wq * 64;
        if (s < p.n_slots) {
            const unsigned long long vm = s_vm[i];
            if (vm) vis64[s >> 6] |= vm;   // the block owns these words during the level
            fw64[s >> 6] = s_wm[i];
        }
    }
    for (uint32_t k = threadIdx.x; k < nbuf; k += blockDim.x) {
        p.tiles[(uint64_t)(it_base + k) * gridDim.x + blockIdx.x] = PullTile{s_cw[k], s_ce[k], s_cl[k]};
        s_cw[k] = 0;
        s_ce[k] = 0;
        s_cl[k] = 0;
    }
    __syncthreads();
}

// One iteration's per-slot words of a wave (kPS slots per lane, 64 apart): visit, class and "more"
// bitmap words (the 32-bit word holding the lane's bit), the two list heads and the row length.
struct PullSlots {
    uint32_t vw[kPS], cw[kPS], mw[kPS], rl[kPS];
    uint64_t hd[kPS];
};

__device__ __forceinline__ void pull_load(const PullArgs& p, const uint32_t* vis, uint64_t d0, uint32_t lane,
                                          PullSlots& x) {
#pragma unroll
    for (int j = 0; j < (int)kPS; ++j) {
        const uint64_t d = d0 + j * 64 + lane;
        const bool in = d < p.n_slots;
        x.vw[j] = in ? vis[d >> 5] : ~0u;
        x.cw[j] = in ? p.cls[d >> 5] : 0u;
        x.mw[j] = in ? p.uin_more[d >> 5] : 0u;
        x.hd[j] = in ? __builtin_nontemporal_load(p.uin_head + d) : ~0ull;
        x.rl[j] = in ? p.row_len[d] : 0u;
    }
}

__device__ __forceinline__ void pull_level(const PullArgs& p, const unsigned long long* node, uint32_t* vis,
                                           uint32_t* lds_q, unsigned long long* lds_buf, unsigned long long* blk,
                                           unsigned long long (*s_st)[kStats]) {
    uint32_t flagged = 0, cand = 0, examined = 0, live = 0, wins = 0, tails = 0, examined_tail = 0, wins_tail = 0;
    const uint32_t lane = lane_id(), wid = threadIdx.x >> 6;
    const uint64_t stride = (uint64_t)gridDim.x * kPullTile;
    const uint32_t n_iter = (uint32_t)pull_iters(p.n_slots, gridDim.x);
    unsigned long long* s_vm = lds_buf;                                   // [kMaxIter][16]
    unsigned long long* s_wm = s_vm + kMaxIter * kTileWords;              // [kMaxIter][16]
    unsigned long long* s_cl = s_wm + kMaxIter * kTileWords;              // [kMaxIter]
    uint32_t* s_cw = reinterpret_cast<uint32_t*>(s_cl + kMaxIter);        // [kMaxIter]
    uint32_t* s_ce = s_cw + kMaxIter;                                     // [kMaxIter]
    uint32_t* s_qn = s_ce + kMaxIter;
    if (threadIdx.x < kMaxIter) {
        s_cw[threadIdx.x] = 0;
        s_ce[threadIdx.x] = 0;
        s_cl[threadIdx.x] = 0;
    }
    if (threadIdx.x == 0) *s_qn = 0;
    __syncthreads();
    uint32_t it_base = 0;
    // the slot words of iteration it + 1 are loaded while iteration it waits for its frontier bits
    PullSlots cur;
    pull_load(p, vis, (uint64_t)blockIdx.x * kPullTile + wid * (64 * kPS), lane, cur);
    for (uint32_t it = 0; it < n_iter; ++it) {
        const uint32_t k = it - it_base;
        const uint64_t s0 = (uint64_t)it * stride + (uint64_t)blockIdx.x * kPullTile;
        const uint64_t d0 = s0 + wid * (64 * kPS);
        const uint32_t* vw = cur.vw;
        const uint32_t* cw = cur.cw;
        const uint32_t* mw = cur.mw;
        const uint32_t* rl = cur.rl;
        bool c[kPS];
        uint32_t f0[kPS], f1[kPS];
#pragma unroll
        for (int j = 0; j < (int)kPS; ++j) {
            const uint64_t d = d0 + j * 64 + lane;
            const bool lv = d < p.n_slots && !((vw[j] >> (lane & 31)) & 1u);
            const uint32_t h0 = (uint32_t)cur.hd[j], h1 = (uint32_t)(cur.hd[j] >> 32);
            c[j] = lv && h0 != FGI_NONE;
            f0[j] = c[j] ? p.front_rd[h0 >> 5] : 0u;
            f1[j] = (c[j] && h1 != FGI_NONE) ? p.front_rd[h1 >> 5] : 0u;
            live += (uint32_t)__popcll(__ballot(lv));
        }
        PullSlots nxt;
        pull_load(p, vis, d0 + stride, lane, nxt);
        bool hit[kPS], tail[kPS];
#pragma unroll
        for (int j = 0; j < (int)kPS; ++j) {
            const uint32_t h0 = (uint32_t)cur.hd[j], h1 = (uint32_t)(cur.hd[j] >> 32);
            const bool b0 = c[j] && ((f0[j] >> (h0 & 31)) & 1u);
            const bool b1 = c[j] && h1 != FGI_NONE && ((f1[j] >> (h1 & 31)) & 1u);
            // statistics as wave-uniform counts (scalar registers), reported by lane 0
            cand += (uint32_t)__popcll(__ballot(c[j]));
            examined += (uint32_t)__popcll(__ballot(c[j])) + (uint32_t)__popcll(__ballot(c[j] && h1 != FGI_NONE && !b0));
            hit[j] = b0 || b1;
            tail[j] = c[j] && !hit[j] && ((mw[j] >> (lane & 31)) & 1u);
        }
        uint32_t nw = 0, ne = 0;
        unsigned long long nl = 0;
        uint32_t q_end = 0;
#pragma unroll
        for (int j = 0; j < (int)kPS; ++j) {
            const uint64_t d = d0 + j * 64 + lane;
            const bool win = hit[j] && ((cw[j] >> (lane & 31)) & 1u);
            if (hit[j] && !win) flagged += first_visit(node[d]) == 2 ? 1u : 0u;
            const unsigned long long vm = __ballot(hit[j]), wm = __ballot(win);
            if (lane == 0) {
                s_vm[k * kTileWords + wid * kPS + j] = vm;
                s_wm[k * kTileWords + wid * kPS + j] = wm;
            }
            nw += (uint32_t)__popcll(wm);
            ne += (uint32_t)__popcll(__ballot(win && rl[j]));
            nl += win ? rl[j] : 0u;
            const unsigned long long tm = __ballot(tail[j]);
            if (tm) {
                uint32_t qb = 0;
                if (lane == 0) qb = atomicAdd(s_qn, (uint32_t)__popcll(tm));
                qb = __shfl(qb, 0, 64);
                if (tail[j]) lds_q[qb + __popcll(tm & lanemask_lt())] = (uint32_t)d;
                q_end = qb + (uint32_t)__popcll(tm);
            }
        }
        wins += nw;
        nl = wave_sum64(nl);
        if (lane == 0) {
            if (nw) atomicAdd(&s_cw[k], nw);
            if (ne) atomicAdd(&s_ce[k], ne);
            if (nl) atomicAdd(&s_cl[k], nl);
        }
        if (it == 0) probe_at(p.probe, 1);
        // flush when the LDS buffers are full, the queue could overflow next time, or at the end
        const bool full = k + 1 == kMaxIter || it + 1 == n_iter;
        if (__syncthreads_or(full || q_end > kTailCap - kPullTile)) {
            const uint32_t nq = *s_qn;
            probe_at(p.probe, it + 1 == n_iter ? 4 : 2);
            pull_flush(p, node, vis, it_base, k + 1, lds_q, nq, s_vm, s_wm, s_cw, s_ce, s_cl, flagged, examined_tail,
                       wins_tail, tails);
            if (threadIdx.x == 0) *s_qn = 0;
            __syncthreads();
            probe_at(p.probe, it + 1 == n_iter ? 5 : 3);
            it_base = it + 1;
        }
        cur = nxt;
    }
    const uint32_t scan = (blockIdx.x == 0 && threadIdx.x == 0) ? p.n_slots : 0u;
    // cand, live, wins and the head probes of `examined` are wave-uniform counts; the tail probes
    // and flag counts are per lane
    const bool l0 = lane == 0;
    const uint32_t v[kStats] = {0, flagged, l0 ? cand : 0u, examined_tail + (l0 ? examined : 0u), l0 ? live : 0u,
                                wins_tail + (l0 ? wins : 0u), tails, scan};
    block_stats_add(blk, s_st, v);
    probe_at(p.probe, 10);
}

// One level's traversal: push (expand) or pull, as decided for the level on the device.
template <bool PART>
__global__ __launch_bounds__(kBlock, 5) void k_level(int L, ExpandArgs x, PullArgs p, const unsigned long long* node,
                                                  uint32_t* vis, Out o, WaveCtr* ctr, unsigned long long* blk,
                                                  RemoteArgs ra) {
    // push: the chunk map (s_rel, s_base), then the chunk's winners over it; pull: queue + buffers
    __shared__ __align__(16) uint32_t s_x[kChunkEmitCap + 8];
    uint32_t* s_rel = s_x;                    // [kChunk + 1]
    uint32_t* s_base = s_x + kChunk + 4;      // [kChunk + 2], 16-byte aligned
    __shared__ Emit em;
    __shared__ MsgEmit<PART> me;
    __shared__ unsigned long long s_st[kBlock / 64][kStats];
    static_assert((2 * kMaxIter * kTileWords + kMaxIter) * 8 + 3 * kMaxIter * 4 + 4 <= (kChunk + 2) * 4, "pull LDS");
    if ((x.probe || p.probe) && threadIdx.x == 0 && blockIdx.x < kProbeBlocks)
        (x.probe ? x.probe : p.probe)[blockIdx.x * kProbePhases] = __builtin_amdgcn_s_memrealtime();
    const LevelCtr& lc = ctr->lvl[L % kRing];
    o.ln = &ctr->lvl[(L + 1) % kRing];
    if (blockIdx.x == 0 && threadIdx.x < sizeof(LevelCtr) / 8)
        reinterpret_cast<unsigned long long*>(&ctr->lvl[(L + 2) % kRing])[threadIdx.x] = 0ull;
    // multi-GPU pull levels run on every rank (parents may be remote); otherwise no frontier, no work
    if (!lc.pull && lc.F == 0) return;
    if (lc.pull) {
        pull_level(p, node, vis, s_rel, reinterpret_cast<unsigned long long*>(s_base), blk, s_st);
    } else {
        emit_init(em);
        expand_level<PART>(lc, x, node, vis, o, em, s_x, me, s_rel, s_base, blk, s_st, ra);
    }
}

// multi-GPU: apply the targets other ranks forwarded (their versions were checked by the sender)
__global__ __launch_bounds__(kBlock) void k_apply_recv(int L, uint64_t n, const uint32_t* __restrict__ recv, uint32_t base,
                                                       const unsigned long long* node, uint32_t* vis, Out o,
                                                       WaveCtr* ctr, unsigned long long* blk) {
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
                const int r = visit_bit(vis, h, w);
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

// Folds the per-block statistics into the wave counters: one block per column (coalesced sweeps).
// Block kStats: if level L_next follows a pull level, its F and T from the pull's tiles (the host
// reads them to decide termination before k_level_begin(L_next) has run).
// Wave prologue in one launch (instead of three fills): the counter ring, the per-block
// statistics and the first frontier bitmap start at zero.
__global__ __launch_bounds__(kBlock) void k_wave_init(WaveCtr* ctr, unsigned long long* blk, uint32_t* fb0,
                                                      uint64_t fb_words, unsigned long long* done) {
    const uint64_t tid = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const uint64_t nthr = (uint64_t)gridDim.x * blockDim.x;
    // finish_prefix's completion counters (normally left at zero by their last user)
    if (tid <= (uint64_t)kDoneGroups) coh_xchg(done + tid * kDoneStride, 0ull);
    unsigned long long* c = reinterpret_cast<unsigned long long*>(ctr);
    for (uint64_t i = tid; i < sizeof(WaveCtr) / 8; i += nthr) c[i] = 0ull;
    for (uint64_t i = tid; i < (uint64_t)kStatBlocks * kStatCols; i += nthr) blk[i] = 0ull;
    uint4* f4 = reinterpret_cast<uint4*>(fb0);
    for (uint64_t i = tid; i < fb_words / 4; i += nthr) f4[i] = make_uint4(0u, 0u, 0u, 0u);
    for (uint64_t i = fb_words / 4 * 4 + tid; i < fb_words; i += nthr) fb0[i] = 0u;
}

__global__ __launch_bounds__(kBlock) void k_stats_reduce(const unsigned long long* __restrict__ blk, WaveCtr* ctr,
                                                         int L_next, const PullTile* __restrict__ tiles,
                                                         uint64_t n_tiles) {
    __shared__ unsigned long long s_red[kBlock / 64];
    const int k = blockIdx.x;
    if (k == kStats) {
        if (L_next > 0 && ctr->lvl[(L_next + kRing - 1) % kRing].pull)
            tile_totals(tiles, n_tiles, ctr->lvl[L_next % kRing], s_red);
        return;
    }
    unsigned long long* dst[kStats] = {&ctr->e_match,   &ctr->n_flagged, &ctr->pull_cand, &ctr->pull_edges,
                                       &ctr->pull_live, &ctr->pull_win,  &ctr->pull_tail, &ctr->pull_scan};
    const unsigned long long* col = blk + (uint64_t)k * kStatBlocks;
    unsigned long long t = 0;
#pragma unroll
    for (uint32_t b = 0; b < kStatBlocks / kBlock; ++b) t += col[b * kBlock + threadIdx.x];
    t = block_sum(t, s_red);
    if (threadIdx.x == 0) *dst[k] = t + (k == kStFlagged ? ctr->root_flagged : 0ull);
}

// ---- fold / class bitmap -----------------------------------------------------------------------
__global__ __launch_bounds__(kBlock) void k_fold(uint32_t n, const uint32_t* __restrict__ vis,
                                                 unsigned long long* node) {
    for (uint64_t h = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; h < n; h += (uint64_t)gridDim.x * blockDim.x)
        if (bit_of(vis, (uint32_t)h)) node[h] = visited_word(node[h]);
}

__global__ __launch_bounds__(kBlock) void k_build_cls(uint32_t n, const unsigned long long* __restrict__ node,
                                                      unsigned long long* cls64) {
    const uint64_t nthr = (uint64_t)gridDim.x * blockDim.x;
    const uint64_t lim = ((uint64_t)n + 63) / 64 * 64;
    for (uint64_t h = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; h < lim; h += nthr) {
        bool c = false;
        if (h < n) {
            const unsigned long long w = node[h];
            c = (w & kVMask) != 0 && word_state(w) == FGI_CONSISTENT && !(w & kW_HasDelay);
        }
        const unsigned long long m = __ballot(c);
        if (lane_id() == 0) cls64[h >> 6] = m;
    }
}

}  // namespace

fgi_status fold(fgi_graph* g) {
    if (!g->v_dirty) return FGI_OK;
    const uint32_t H = g->n_handles;
    hipLaunchKernelGGL(k_fold, dim3(std::min<uint32_t>((H + kBlock - 1) / kBlock, 8192)), dim3(kBlock), 0, g->stream, H,
                       g->vis_bm, reinterpret_cast<unsigned long long*>(g->node));
    FGI_HIP(g, hipGetLastError());
    FGI_HIP(g, hipMemsetAsync(g->vis_bm, 0, g->bm_words * 4, g->stream));
    g->v_dirty = false;
    note_words(g);
    return FGI_OK;
}

fgi_status ensure_cls(fgi_graph* g) {
    if (g->cls_valid) return FGI_OK;
    const uint32_t H = g->n_handles;
    hipLaunchKernelGGL(k_build_cls, dim3(std::min<uint32_t>((H + kBlock - 1) / kBlock + 1, 8192)), dim3(kBlock), 0,
                       g->stream, H, reinterpret_cast<const unsigned long long*>(g->node),
                       reinterpret_cast<unsigned long long*>(g->cls_bm));
    FGI_HIP(g, hipGetLastError());
    g->cls_valid = true;
    return FGI_OK;
}

// Algorithmic bytes of the pull levels of a wave (k_level on pull levels): per slot scanned its
// two list heads and row length (12 B) and the visit / class / "more" / frontier words (1/2 B);
// per queued slot its list offset and length (12 B) and 4 B per further dependency examined (the
// frontier-bitmap probes hit L2 and are not counted). Winners cost only bitmap bits and counts.
static uint64_t pull_level_bytes(const WaveCtr& c) {
    const uint64_t head_probes = c.pull_cand;   // >= 1 examined per candidate in the head step
    const uint64_t tail_deps = c.pull_edges > head_probes ? c.pull_edges - head_probes : 0;
    return c.pull_scan * 12 + c.pull_scan / 2 + 12 * c.pull_tail + 4 * tail_deps;
}

// Flags of the per-level timing events (FGI_EVENT_FLAGS overrides, for measurement). Without the
// system-scope fence a record costs ~1 us instead of ~6 us between kernels (profiles/, e1).
static unsigned event_flags() {
    static const unsigned f = getenv("FGI_EVENT_FLAGS") ? (unsigned)strtoul(getenv("FGI_EVENT_FLAGS"), nullptr, 0)
                                                       : (unsigned)hipEventDisableSystemFence;
    return f;
}

// FGI_PROBE (measurement only): median per-phase offsets (us) of a push level's stamped blocks
static fgi_status probe_report(fgi_graph* g, int L, uint32_t grid, const char* what = "level") {
    std::vector<unsigned long long> h((size_t)kProbeBlocks * kProbePhases);
    FGI_HIP(g, hipStreamSynchronize(g->stream));
    FGI_HIP(g, hipMemcpy(h.data(), g->probe, h.size() * 8, hipMemcpyDeviceToHost));
    const uint32_t nb = std::min<uint32_t>(grid, kProbeBlocks);
    unsigned long long t0 = ~0ull, t_end = 0;
    for (uint32_t b = 0; b < nb; ++b)
        if (h[(size_t)b * kProbePhases]) {
            t0 = std::min(t0, h[(size_t)b * kProbePhases]);
            t_end = std::max(t_end, h[(size_t)b * kProbePhases + 10]);
        }
    fprintf(stderr, "[probe] %s %d span %.2f us; median phase stamps (us after first block start):", what, L,
            t0 == ~0ull ? 0.0 : (t_end - t0) / 100.0);
    for (int k = 0; k <= 10; ++k) {
        std::vector<double> v;
        for (uint32_t b = 0; b < nb; ++b) {
            const unsigned long long x = h[(size_t)b * kProbePhases + k];
            if (x && (h[(size_t)b * kProbePhases + 2] || h[(size_t)b * kProbePhases + 4]))
                v.push_back((x - t0) / 100.0);   // blocks with a chunk (push) / pulling blocks
        }
        if (v.empty()) continue;
        std::sort(v.begin(), v.end());
        fprintf(stderr, " p%d=%.2f/%.2f", k, v[v.size() / 2], v.back());
    }
    fprintf(stderr, "\n");
    return FGI_OK;
}

static CollectArgs collect_args(fgi_graph* g, uint32_t n_slots, uint32_t pgrid, uint32_t* fb, int fr_multi, int buf) {
    CollectArgs c;
    c.tiles = g->tiles;
    c.n_tiles = pull_iters(n_slots, pgrid) * pgrid;
    c.pgrid = pgrid;
    c.n_slots = n_slots;
    c.fb = fb;
    c.n_handles = g->n_handles;
    c.stay_pull_f = g->opt_pull_beta > 0 ? n_slots / (uint64_t)g->opt_pull_beta : ~0ull;
    c.fr_multi = fr_multi;
    c.row_len = g->row_len;
    c.inv = g->inv;
    c.row_off = g->row_off;
    c.fr_off = g->fr_off[buf];
    c.fr_len = g->fr_len[buf];
    c.escan = g->escan;
    c.cstart = g->cstart;
    c.part3 = g->partials + kScanBlocks;
    c.pre3 = g->partials + 4 * kScanBlocks;
    c.done = g->partials + 8 * kScanBlocks;   // (kDoneGroups + 1) counters, kDoneStride apart
    c.probe = nullptr;
    return c;
}

static uint32_t level_grid_for(fgi_graph* g, uint32_t per_cu) {
    return std::min<uint32_t>((uint32_t)g->n_cu * per_cu, kStatBlocks);
}

fgi_status run_wave(fgi_graph* g, uint32_t n_roots, const uint32_t* roots_dev, const uint8_t* imm_dev,
                    fgi_wave_stats* stats) {
    const auto t0 = std::chrono::steady_clock::now();
    hipStream_t s = g->stream;
    static const bool trace = getenv("FGI_TRACE") != nullptr;
    static const bool no_level_events = getenv("FGI_NO_LEVEL_EVENTS") != nullptr;   // measurement only
    static const bool probe = getenv("FGI_PROBE") != nullptr;                        // measurement only
    if (probe && !g->probe) FGI_HIP(g, hipMalloc(&g->probe, sizeof(unsigned long long) * kProbeBlocks * kProbePhases));
    const bool timing = (stats != nullptr || trace) && !no_level_events && g->opt_level_timing;
    FGI_TRY(ensure_cstart(g, g->pool_top));
    FGI_TRY(ensure_cls(g));
    // Pull levels need the dependency-list cache. It is built lazily: while it is stale, levels
    // run push-only; once a level group shows a frontier heavy enough to pull, the cache is
    // (re)built and later groups may pull. Small waves (streaming mixes) never pay for it.
    const int direction = g->opt_direction;
    const uint64_t pull_threshold = g->pool_top / (uint64_t)(g->opt_pull_alpha > 0 ? g->opt_pull_alpha : 1);
    if (direction == 2 && n_roots) FGI_TRY(ensure_in_lists(g));
    bool allow_pull = direction != 1 && g->uin_src && g->uin_epoch == g->mut_epoch;
    uint32_t* fb[2] = {g->front_bm, g->front_nx};
    static_assert(sizeof(WaveCtr) % 8 == 0, "WaveCtr is cleared as 64-bit words");
    hipLaunchKernelGGL(k_wave_init, dim3(512), dim3(kBlock), 0, s, g->ctr, g->blk_stats, fb[0], (uint64_t)g->bm_words,
                       g->partials + 8 * kScanBlocks);
    if (timing || stats) FGI_HIP(g, hipEventRecord(g->ev_w0, s));
    Out o{g->row_off, g->row_len, g->inv, g->fr_off[0], g->fr_len[0], &g->ctr->inv, &g->ctr->lvl[0]};
    if (n_roots) {
        g->v_dirty = true;
        const uint32_t nb = (n_roots + kBlock - 1) / kBlock;
        auto* node = reinterpret_cast<unsigned long long*>(g->node);
        if (imm_dev) {
            hipLaunchKernelGGL(k_roots<1>, dim3(nb), dim3(kBlock), 0, s, roots_dev, imm_dev, n_roots, 0u, g->n_handles,
                               node, g->vis_bm, o, g->ctr);
        }
        hipLaunchKernelGGL(k_roots<0>, dim3(nb), dim3(kBlock), 0, s, roots_dev, imm_dev, n_roots, 0u, g->n_handles, node,
                           g->vis_bm, o, g->ctr);
    }
    // 5 resident blocks per CU (k_level launch bounds); per-block statistics bound the grid
    const uint32_t level_grid = level_grid_for(g, 5);
    const uint64_t slot_words = ((uint64_t)g->n_slots + 63) / 64 * 2;
    const uint64_t n_tiles = pull_iters(g->n_slots, level_grid) * level_grid;
    // Levels run in groups between host synchronisations (one ~30 us round trip each); the first
    // group is sized by the previous wave's depth, so a repeated workload syncs once per wave and an
    // overshoot costs only empty levels (three ~4 us launches each).
    int group = std::min(8, std::max(2, g->last_levels));
    int L = 0;
    uint64_t levels = 0, e_trav = 0, f_total = 0, pull_levels = 0;
    double expand_ms = 0, pull_ms = 0;
    uint64_t expand_launches = 0, expand_edges = 0, expand_f = 0, pull_launches = 0;
    bool done = (n_roots == 0);
    while (!done) {
        const int L0 = L;
        const int dir_eff = allow_pull ? direction : 1;
        for (int k = 0; k < group; ++k, ++L) {
            const int buf = L & 1;
            CollectArgs ca = collect_args(g, g->n_slots, level_grid, fb[buf], 0, buf);
            hipLaunchKernelGGL(k_level_begin, dim3(kScanBlocks), dim3(kBlock), 0, s, L, g->ctr, g->inv, fb[buf],
                               fb[buf ^ 1], g->bm_words, slot_words, g->fr_len[buf], g->partials, dir_eff,
                               pull_threshold, ca);
            if (probe) {
                FGI_HIP(g, hipMemsetAsync(g->probe, 0, sizeof(unsigned long long) * kProbeBlocks * kProbePhases, s));
                ca.probe = g->probe;
            }
            hipLaunchKernelGGL(k_scan_apply, dim3(kScanBlocks), dim3(kScanThreads), 0, s, L, g->fr_len[buf], g->partials,
                               g->escan, g->cstart, g->ctr, 0, ca, dir_eff, pull_threshold, fb[buf ^ 1], slot_words);
            if (probe && L > 0) FGI_TRY(probe_report(g, L, kScanBlocks, "collect"));
            if (timing) {
                while (g->ev.size() < 2 * (size_t)(L + 1) + 2) {
                    hipEvent_t e;
                    FGI_HIP(g, hipEventCreateWithFlags(&e, event_flags()));
                    g->ev.push_back(e);
                }
                FGI_HIP(g, hipEventRecord(g->ev[2 * L], s));
            }
            if (probe) FGI_HIP(g, hipMemsetAsync(g->probe, 0, sizeof(unsigned long long) * kProbeBlocks * kProbePhases, s));
            const ExpandArgs xa{g->fr_off[buf], g->escan,    g->cstart,
                                g->pool_col, g->pool_tag, g->opt_dead_filter, probe ? g->probe : nullptr};
            const PullArgs pa{g->n_slots, g->uin_off, g->uin_len, g->uin_src,  g->uin_head,
                              g->uin_more, fb[buf], fb[buf ^ 1], g->cls_bm, g->row_len,
                              g->tiles,   probe ? g->probe : nullptr};
            Out ol{g->row_off, g->row_len, g->inv, g->fr_off[buf ^ 1], g->fr_len[buf ^ 1], &g->ctr->inv, nullptr};
            hipLaunchKernelGGL(k_level<false>, dim3(level_grid), dim3(kBlock), 0, s, L, xa, pa,
                               reinterpret_cast<const unsigned long long*>(g->node), g->vis_bm, ol, g->ctr,
                               g->blk_stats, RemoteArgs{});
            if (timing) FGI_HIP(g, hipEventRecord(g->ev[2 * L + 1], s));
            if (probe) FGI_TRY(probe_report(g, L, level_grid));
        }
        hipLaunchKernelGGL(k_stats_reduce, dim3(kStats + 1), dim3(kBlock), 0, s, g->blk_stats, g->ctr, L, g->tiles,
                           n_tiles);
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
        if (g->ctr_host->lvl[L % kRing].F == 0) {
            done = true;
            // a last pull level's winners (all without rows) are still only in its bitmap: run
            // level L's collect (k_level_begin + k_scan_apply; there is nothing to traverse)
            if (L > 0 && g->ctr_host->lvl[(L - 1) % kRing].pull && g->ctr_host->lvl[L % kRing].pad0) {
                const int buf = L & 1;
                const CollectArgs ca = collect_args(g, g->n_slots, level_grid, fb[buf], 0, buf);
                hipLaunchKernelGGL(k_level_begin, dim3(kScanBlocks), dim3(kBlock), 0, s, L, g->ctr, g->inv, fb[buf],
                                   fb[buf ^ 1], g->bm_words, slot_words, g->fr_len[buf], g->partials, dir_eff,
                                   pull_threshold, ca);
                hipLaunchKernelGGL(k_scan_apply, dim3(kScanBlocks), dim3(kScanThreads), 0, s, L, g->fr_len[buf],
                                   g->partials, g->escan, g->cstart, g->ctr, 0, ca, dir_eff, pull_threshold,
                                   fb[buf ^ 1], slot_words);
                FGI_HIP(g, hipGetLastError());
                FGI_HIP(g, hipMemcpyAsync(g->ctr_host, g->ctr, sizeof(WaveCtr), hipMemcpyDeviceToHost, s));
                FGI_HIP(g, hipStreamSynchronize(s));
            }
        }
        group = 4;
        // also when the wave is already done (its level groups are sized from the previous wave's
        // depth, so a repeated wave after a mutation finishes in one group): the next wave pulls
        if (!allow_pull && direction == 0) {
            bool heavy = false;
            for (int l = L0; l <= L; ++l) heavy |= g->ctr_host->lvl[l % kRing].T > pull_threshold;
            if (heavy) {
                FGI_TRY(ensure_in_lists(g));
                allow_pull = true;
            }
        }
    }
    if (n_roots == 0) {
        hipLaunchKernelGGL(k_stats_reduce, dim3(kStats + 1), dim3(kBlock), 0, s, g->blk_stats, g->ctr, 0, g->tiles,
                           n_tiles);
        FGI_HIP(g, hipMemcpyAsync(g->ctr_host, g->ctr, sizeof(WaveCtr), hipMemcpyDeviceToHost, s));
        FGI_HIP(g, hipStreamSynchronize(s));
    }
    if (timing || stats) {
        FGI_HIP(g, hipEventRecord(g->ev_w1, s));
        FGI_HIP(g, hipEventSynchronize(g->ev_w1));
    }
    if (imm_dev && n_roots) note_words(g);   // immediate roots changed node words
    g->last_wave_n = g->ctr_host->inv;
    if (n_roots) g->last_levels = (int)levels;
    const WaveCtr& c = *g->ctr_host;
    if (trace)
        fprintf(stderr,
                "[fgi] wave: %llu invalidated; pull: live %llu, candidates %llu, queued %llu, dependencies "
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
        // node-word gather 8; per frontier entry: fr_len 4 x2, escan 8 w + 8 r, fr_off 4 r, written
        // 8 (offset, length) by the producer. Per invalidated node: row gathers 12 + list write 4.
        // Per root 5.
        const uint64_t push_b = 20 * expand_edges + 36 * expand_f;
        const uint64_t pull_b = pull_level_bytes(c);
        stats->alg_bytes += push_b + pull_b + 16 * v + 5ull * n_roots;
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
static uint32_t part_grid(fgi_graph* g) { return level_grid_for(g, 5); }

fgi_status part_wave_begin(fgi_graph* g, uint32_t n_roots, const uint32_t* roots_dev, const uint8_t* imm_dev) {
    PartView pv;
    if (!part_view(g, &pv)) return set_err(g, FGI_ESTATE, "partition not initialised");
    hipStream_t s = g->stream;
    g->pw = PartWave{};
    g->pw.t0 = std::chrono::steady_clock::now();
    g->pw.n_roots = n_roots;
    FGI_TRY(ensure_cstart(g, g->pool_top));
    FGI_TRY(ensure_cls(g));
    FGI_HIP(g, hipMemsetAsync(g->ctr, 0, sizeof(WaveCtr), s));
    FGI_HIP(g, hipMemsetAsync(g->blk_stats, 0, sizeof(unsigned long long) * kStatBlocks * kStatCols, s));
    FGI_HIP(g, hipMemsetAsync(pv.sent_bm, 0, pv.sent_words * 4, s));
    while (g->ev.size() < 3) {
        hipEvent_t e;
        FGI_HIP(g, hipEventCreateWithFlags(&e, event_flags()));
        g->ev.push_back(e);
    }
    FGI_HIP(g, hipEventRecord(g->ev_w0, s));
    g->v_dirty = true;
    const Out o{g->row_off, g->row_len, g->inv, g->fr_off[0], g->fr_len[0], &g->ctr->inv, &g->ctr->lvl[0]};
    auto* node = reinterpret_cast<unsigned long long*>(g->node);
    if (n_roots) {
        const uint32_t nb = (n_roots + kBlock - 1) / kBlock;
        if (imm_dev)
            hipLaunchKernelGGL(k_roots<1>, dim3(nb), dim3(kBlock), 0, s, roots_dev, imm_dev, n_roots, pv.base, pv.n_local,
                               node, g->vis_bm, o, g->ctr);
        hipLaunchKernelGGL(k_roots<0>, dim3(nb), dim3(kBlock), 0, s, roots_dev, imm_dev, n_roots, pv.base, pv.n_local,
                           node, g->vis_bm, o, g->ctr);
        if (imm_dev) note_words(g);
    }
    FGI_HIP(g, hipGetLastError());
    return FGI_OK;
}

const unsigned long long* part_level_frontier_dev(fgi_graph* g, int L) { return &g->ctr->lvl[L % kRing].F; }
const unsigned long long* part_level_edges_dev(fgi_graph* g, int L) { return &g->ctr->lvl[L % kRing].T; }

// Level L's list work before its traversal. After a pull level (prev_pull): collect its winners
// bitmap (front_nx) into the invalidated list, and into the frontier list if level L pushes
// (write_fr). After a push level, a push level L needs the exclusive scan of its frontier's row
// lengths (escan) and the chunk map; a pull level L needs neither (part_level_mark marks its frontier).
fgi_status part_level_scan(fgi_graph* g, int L, bool prev_pull, bool write_fr) {
    PartView pv;
    part_view(g, &pv);
    hipStream_t s = g->stream;
    const int buf = L & 1;
    const CollectArgs ca = collect_args(g, pv.n_local, part_grid(g), g->front_nx, write_fr ? 1 : 0, buf);
    FGI_HIP(g, hipMemsetAsync(pv.send_cnt, 0, (size_t)pv.world * 8, s));
    if (!prev_pull && !write_fr) return FGI_OK;
    hipLaunchKernelGGL(k_scan_reduce, dim3(kScanBlocks), dim3(kBlock), 0, s, L, g->fr_len[buf], g->partials, g->ctr, ca);
    hipLaunchKernelGGL(k_scan_apply, dim3(kScanBlocks), dim3(kScanThreads), 0, s, L, g->fr_len[buf], g->partials, g->escan,
                       g->cstart, g->ctr, 1, ca, 1, ~0ull, g->front_nx, (uint64_t)0);
    FGI_HIP(g, hipGetLastError());
    return FGI_OK;
}

// Marks the previous level's winners into the local frontier bitmap on a pull level; the local
// frontier words front_bm[0, block/32) are then all-gathered into pv.front_global. After a pull
// level (prev_pull) its winners bitmap front_nx is exactly the set [marked, inv) just collected:
// a pull level L copies it whole instead of one atomic per winner; either way front_nx is cleared
// here, so no later level or wave reads a stale winner.
fgi_status part_level_mark(fgi_graph* g, int L, bool pull, bool prev_pull) {
    hipStream_t s = g->stream;
    const int n_cu = g->n_cu;
    // the flag's high word is zero (the ring slot was cleared two levels ago or at wave start), so a
    // 32-bit device-side set of the low word is the whole store, with no pageable host copy
    if (pull)
        FGI_HIP(g, hipMemsetD32Async(reinterpret_cast<hipDeviceptr_t>(&g->ctr->lvl[L % kRing].pull), 1, 1, s));
    const bool copy = pull && prev_pull;
    if (copy) FGI_HIP(g, hipMemcpyAsync(g->front_bm, g->front_nx, g->bm_words * 4, hipMemcpyDeviceToDevice, s));
    if (prev_pull) FGI_HIP(g, hipMemsetAsync(g->front_nx, 0, g->bm_words * 4, s));
    hipLaunchKernelGGL(k_mark, dim3((uint32_t)n_cu * 2), dim3(kBlock), 0, s, L, g->inv, g->front_bm, g->ctr,
                       copy ? 1 : 0);
    FGI_HIP(g, hipGetLastError());
    return FGI_OK;
}

// push: expand (remote targets staged for the exchange); pull: scan local dependency lists
// against the global frontier bitmap
fgi_status part_level_work(fgi_graph* g, int L, bool pull) {
    PartView pv;
    part_view(g, &pv);
    hipStream_t s = g->stream;
    const RemoteArgs ra{pv.base, pv.n_local, pv.block, pv.world, pv.ver_all, pv.sent_bm, pv.send_buf, pv.send_cnt};
    const int buf = L & 1;
    if (g->opt_level_timing) FGI_HIP(g, hipEventRecord(g->ev[0], s));
    const ExpandArgs xa{g->fr_off[buf], g->escan, g->cstart, g->pool_col, g->pool_tag, g->opt_dead_filter, nullptr};
    const PullArgs pa{pv.n_local,      g->uin_off,  g->uin_len, g->uin_src,  g->uin_head, g->uin_more,
                      pv.front_global, g->front_nx, g->cls_bm,  g->row_len, g->tiles, nullptr};
    const Out o{g->row_off, g->row_len, g->inv, g->fr_off[buf ^ 1], g->fr_len[buf ^ 1], &g->ctr->inv, nullptr};
    hipLaunchKernelGGL(k_level<true>, dim3(part_grid(g)), dim3(kBlock), 0, s, L, xa, pa,
                       reinterpret_cast<const unsigned long long*>(g->node), g->vis_bm, o, g->ctr, g->blk_stats, ra);
    if (g->opt_level_timing) FGI_HIP(g, hipEventRecord(g->ev[1], s));
    if (pull) FGI_HIP(g, hipMemsetAsync(pv.front_global, 0, pv.front_words_global * 4, s));
    FGI_HIP(g, hipGetLastError());
    g->pw.pulled = pull;
    return FGI_OK;
}

fgi_status part_level_apply(fgi_graph* g, int L, uint64_t n_recv, uint64_t n_sent) {
    PartView pv;
    part_view(g, &pv);
    hipStream_t s = g->stream;
    const int n_cu = g->n_cu;
    const int buf = L & 1;
    if (n_recv)
        hipLaunchKernelGGL(k_apply_recv, dim3(std::min<uint64_t>((n_recv + kBlock - 1) / kBlock, (uint64_t)n_cu * 8)),
                           dim3(kBlock), 0, s, L, n_recv, pv.recv_buf, pv.base,
                           reinterpret_cast<const unsigned long long*>(g->node), g->vis_bm,
                           Out{g->row_off, g->row_len, g->inv, g->fr_off[buf ^ 1], g->fr_len[buf ^ 1], &g->ctr->inv,
                               nullptr},
                           g->ctr, g->blk_stats);
    const uint64_t n_tiles = pull_iters(pv.n_local, part_grid(g)) * part_grid(g);
    // after a pull level every set bit of the frontier bitmap is this level's (it is all-zero
    // otherwise), so one memset replaces the per-winner clears
    const bool wipe = g->pw.pulled;
    if (wipe) FGI_HIP(g, hipMemsetAsync(g->front_bm, 0, g->bm_words * 4, s));
    hipLaunchKernelGGL(k_clear_front, dim3((uint32_t)n_cu * 2), dim3(kBlock), 0, s, L, g->inv, g->front_bm, g->ctr,
                       g->tiles, n_tiles, wipe ? 1 : 0);
    FGI_HIP(g, hipGetLastError());
    g->pw.sent += n_sent;
    return FGI_OK;
}

// after the level's frontier total is known (the stream has been synchronised by then).
// fetched: the caller already enqueued the counter copy (part_level_fetch) ahead of the
// synchronisation it waited on, so the copy needs no sync of its own.
fgi_status part_level_fetch(fgi_graph* g) {
    FGI_HIP(g, hipMemcpyAsync(g->ctr_host, g->ctr, sizeof(WaveCtr), hipMemcpyDeviceToHost, g->stream));
    return FGI_OK;
}

fgi_status part_level_account(fgi_graph* g, int L, bool fetched) {
    if (!fetched) {
        FGI_TRY(part_level_fetch(g));
        FGI_HIP(g, hipStreamSynchronize(g->stream));
    }
    const LevelCtr& lc = g->ctr_host->lvl[L % kRing];
    g->pw.levels++;
    g->pw.e_trav += lc.T;
    g->pw.f_total += lc.F;
    if (!lc.pull) g->pw.push_edges += lc.T, g->pw.push_f += lc.F;
    float ms = 0;
    if (g->opt_level_timing) FGI_HIP(g, hipEventElapsedTime(&ms, g->ev[0], g->ev[1]));
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
    hipLaunchKernelGGL(k_stats_reduce, dim3(kStats + 1), dim3(kBlock), 0, s, g->blk_stats, g->ctr, 0, g->tiles,
                       (uint64_t)0);
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
        stats->alg_bytes += 20 * w.push_edges + 36 * w.push_f + pull_b + 16 * v + 8 * w.sent + 5ull * w.n_roots;
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

// The partitioned wave, one call per rank: levels in lockstep, collectives through the rank's
// PartComm (RCCL over xGMI with one process per GPU, or device copies between the graphs of an
// in-process group, one host thread per rank — the same level sequence either way). Per level one
// all-reduce of {frontier, frontier edges} decides push vs pull (Beamer's alpha / beta rules, as
// run_wave) and termination; push levels add the exchange (counts all-gather, then payloads).
fgi_status run_part_wave(fgi_graph* g, uint32_t n_roots, const uint32_t* roots_dev, const uint8_t* imm_dev,
                         fgi_wave_stats* stats) {
    PartView pv;
    part_view(g, &pv);
    FGI_TRY(part_wave_begin(g, n_roots, roots_dev, imm_dev));
    hipStream_t s = g->stream;
    // one all-reduce of {local edges, level-0 frontier, its edges, ranks without pull lists}
    const bool can_pull = g->opt_direction != 1 && g->uin_src && g->uin_epoch == g->mut_epoch;
    const uint64_t head[2] = {g->pool_top, 0};
    const uint64_t tail[2] = {0, can_pull ? 0ull : 1ull};
    FGI_HIP(g, hipMemcpyAsync(pv.scratch_u64, head, 8, hipMemcpyHostToDevice, s));
    FGI_HIP(g, hipMemcpyAsync(pv.scratch_u64 + 1, part_level_frontier_dev(g, 0), 16, hipMemcpyDeviceToDevice, s));
    FGI_HIP(g, hipMemcpyAsync(pv.scratch_u64 + 3, tail + 1, 8, hipMemcpyHostToDevice, s));
    uint64_t sums[4] = {0, 0, 0, 0};
    FGI_TRY(part_allreduce_sum(g, pv.scratch_u64, sums, 4));
    const uint64_t threshold = sums[0] / (uint64_t)(g->opt_pull_alpha > 0 ? g->opt_pull_alpha : 1);
    const uint64_t stay_pull_f = g->opt_pull_beta > 0 ? pv.n_global / (uint64_t)g->opt_pull_beta : ~0ull;
    const bool allow_pull = sums[3] == 0;
    const int direction = g->opt_direction;
    uint64_t f_global = sums[1], t_global = sums[2];
    int L = 0;
    bool last_pull = false;
    for (; f_global != 0; ++L) {
        const bool pull = allow_pull && t_global != 0 &&
                          (direction == 2 || (direction == 0 && (t_global > threshold ||
                                                                 (last_pull && f_global > stay_pull_f))));
        FGI_TRY(part_level_scan(g, L, last_pull, !pull));
        FGI_TRY(part_level_mark(g, L, pull, last_pull));
        if (pull) FGI_TRY(part_allgather_front(g));
        FGI_TRY(part_level_work(g, L, pull));
        uint64_t n_recv = 0, n_sent = 0;
        if (!pull) FGI_TRY(part_exchange(g, &n_recv, &n_sent));
        FGI_TRY(part_level_apply(g, L, n_recv, n_sent));
        // the counter copy rides on the all-reduce's stream synchronisation
        FGI_TRY(part_level_fetch(g));
        uint64_t ft[2] = {0, 0};
        FGI_TRY(part_allreduce_sum(g, part_level_frontier_dev(g, L + 1), ft, 2));
        f_global = ft[0];
        t_global = ft[1];
        FGI_TRY(part_level_account(g, L, true));
        last_pull = pull;
    }
    // the last pull level's winners (without rows) are collected into the invalidated list
    if (last_pull) {
        FGI_TRY(part_level_scan(g, L, true, false));
        FGI_HIP(g, hipMemsetAsync(g->front_nx, 0, g->bm_words * 4, s));
    }
    return part_wave_end(g, stats);
}

}  // namespace fgi
