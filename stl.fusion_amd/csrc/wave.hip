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
// Launches of a wave:
//   k_wave_init, k_roots           — counters, the invalidated bitmap, level 0's frontier list
//   per level L: k_collect(L)      — only after a pull level when level L pushes: the pull's
//                                    winners bitmap -> level L's frontier list (else it exits)
//                k_level(L)        — push: edge-parallel expansion of the frontier's `_usedBy`
//                                    rows, winners appended to level L+1's list already scanned
//                                    (one packed atomic per block batch); or pull: every live slot
//                                    probes its dependency list (the reference's `_used`) for an
//                                    invalidated parent (Beamer's bottom-up step); its last block
//                                    publishes level L+1's frontier size
//   k_final                        — the invalidated bitmap -> the invalidated list (ascending)
// The push/pull choice of a level is a pure function of device counters that every block of the
// level's kernels evaluates the same way; the host synchronises once per group of levels.
#include <hip/hip_cooperative_groups.h>
#include <hip/hip_runtime.h>

#include <sched.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstring>
#include <cstdlib>
#include <vector>

#include "fgi_internal.h"

// measurement-only build (make variant-probe): k_level stamps per-block phase times (100 MHz wall
// clock) into d_probe; run_wave prints per-level medians with FGI_TRACE=1
#ifndef FGI_PROBE
#define FGI_PROBE 0
#endif

namespace fgi {
namespace {

__device__ __forceinline__ uint32_t lane_id() { return __lane_id(); }
constexpr int kProbeLevelsOff = 1 << 20;   // a level index no probe records (cooperative waves)

#if FGI_PROBE
constexpr int kProbeLevels = 8, kProbePts = 8, kProbeBlocks = 2048;
__device__ unsigned long long d_probe[kProbeLevels][kProbeBlocks][kProbePts];
#define PROBE(L, k)                                                                    \
    do {                                                                               \
        if (threadIdx.x == 0 && (L) < kProbeLevels && blockIdx.x < (uint32_t)kProbeBlocks) \
            d_probe[(L)][blockIdx.x][(k)] = wall_clock64();                            \
    } while (0)
// cooperative waves: block 0's phase stamps per launch (ring of 64 launches)
__device__ unsigned long long d_cprobe[64][10];
__device__ unsigned int d_cprobe_n;
#define CPROBE(k)                                                               \
    do {                                                                        \
        if (blockIdx.x == 0 && threadIdx.x == 0) d_cprobe[s_cp][(k)] = wall_clock64(); \
    } while (0)
#else
#define CPROBE(k) \
    do {          \
    } while (0)
#define PROBE(L, k) \
    do {            \
    } while (0)
#endif

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
// A plain read first: a bit already set (an earlier level's visit, or another block's in this one that
// has reached L2) needs no atomic. Within a launch the bits only go from 0 to 1, so a stale read can only
// show 0, and then the atomic decides; hub slots that many edges of a level reach stop contending on one
// word (level 0 of configs[1]: 4,096 degree-weighted roots, 125 k edges onto a few thousand hubs).
__device__ __forceinline__ int visit_bit(uint32_t* vis, uint32_t h, unsigned long long w) {
    const uint32_t b = 1u << (h & 31);
    if (vis[h >> 5] & b) return 0;
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

__device__ __forceinline__ unsigned long long wave_excl_scan64(unsigned long long v, unsigned long long& total) {
    const uint32_t lane = lane_id();
    unsigned long long x = v;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        const unsigned long long y = __shfl_up(x, d, 64);
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

// lane 0's value in every lane (a scalar read; every lane of the wave active)
__device__ __forceinline__ uint32_t from_lane0(uint32_t v) { return __builtin_amdgcn_readfirstlane(v); }
__device__ __forceinline__ unsigned long long from_lane0(unsigned long long v) {
    return ((unsigned long long)__builtin_amdgcn_readfirstlane((uint32_t)(v >> 32)) << 32) |
           __builtin_amdgcn_readfirstlane((uint32_t)v);
}
// set bits of the wave-uniform mask m below this lane (two mbcnt instructions)
__device__ __forceinline__ uint32_t rank_in(unsigned long long m) {
    return __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
}

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

// Per-block statistics: hot kernels keep their counters per block (plain read-modify-write of the
// block's own column entry by one thread, launches of a wave are stream-ordered) instead of per-wave
// atomics on a few words: a single device-scope word saturates near 88 atomics/us. Column-major
// ([column][block]) so k_final sweeps each column coalesced.
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
        // a returnless atomic: nothing in this launch reads the columns, so no round trip is waited for
        if (t) __hip_atomic_fetch_add(blk + (uint64_t)threadIdx.x * kStatBlocks + blockIdx.x, t, __ATOMIC_RELAXED,
                                      __HIP_MEMORY_SCOPE_AGENT);
    }
}

// ---- cross-block hand-offs ----------------------------------------------------------------------
// Agent-scope atomic RMWs are performed at the coherence point shared by the XCDs (their L2s are
// not coherent with each other); a block's completion-counter increment is issued only after its
// own atomics have returned, so the block that arrives last sees every other block's atomics.
__device__ __forceinline__ unsigned long long coh_xchg(unsigned long long* p, unsigned long long v) {
    return __hip_atomic_exchange(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ unsigned long long coh_read(unsigned long long* p) {
    return __hip_atomic_fetch_add(p, 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// the traversal kernels' completion counter (fgi_internal.h): their hand-off values are written by
// thread 0 (coh_xchg) or by atomics whose result was waited for
__device__ __forceinline__ bool last_block(unsigned long long* done, uint64_t G) { return last_block_arrive<false>(done, G); }

// Called by the last block: exclusive prefixes over blocks of three columns, packed per block in
// src[k] (bits 48-63, 32-47, 0-31: pack3), into dst[q * G + k], column totals into tot[q]. In rounds
// of kBlock * kEpiloguePer blocks (one round up to 2,048 blocks): every word of a round is read at
// once (thread t holds kEpiloguePer consecutive blocks; the reads are agent-scope atomics, performed
// at the coherence point, each a round trip: one CU's atomics are the epilogue's cost, so the columns
// are read as one word), then one block scan per column, carried across rounds.
constexpr uint32_t kEpiloguePer = 8;
__host__ __device__ constexpr unsigned long long pack3(unsigned long long a, unsigned long long b, unsigned long long c) {
    return (a << 48) | (b << 32) | c;
}
__device__ void prefix_columns(unsigned long long* src, unsigned long long* dst, uint64_t G, unsigned long long* tot) {
    constexpr int ncols = 3;
    __shared__ unsigned long long s_sc[3][kBlock / 64];
    const uint32_t lane = lane_id(), wid = threadIdx.x >> 6, W = blockDim.x >> 6;
    const uint64_t R = (uint64_t)blockDim.x * kEpiloguePer;
    unsigned long long carry[3] = {0, 0, 0};
    for (uint64_t r0 = 0; r0 < G; r0 += R) {   // block-uniform
        const uint64_t k0 = r0 + (uint64_t)threadIdx.x * kEpiloguePer;
        unsigned long long xs[3][kEpiloguePer];
#pragma unroll
        for (uint32_t j = 0; j < kEpiloguePer; ++j) {
            const unsigned long long v = k0 + j < G ? coh_read(src + k0 + j) : 0ull;
            xs[0][j] = v >> 48;
            xs[1][j] = (v >> 32) & 0xFFFFull;
            xs[2][j] = v & 0xFFFFFFFFull;
        }
        // the three columns' wave scans share one pair of barriers
        unsigned long long x[3];
#pragma unroll
        for (int q = 0; q < 3; ++q) {
            unsigned long long loc = 0;
#pragma unroll
            for (uint32_t j = 0; j < kEpiloguePer; ++j) loc += xs[q][j];
            unsigned long long t;
            x[q] = wave_excl_scan64(loc, t);
            if (lane == 0) s_sc[q][wid] = t;
        }
        __syncthreads();
#pragma unroll
        for (int q = 0; q < 3; ++q) {
            unsigned long long run = carry[q] + x[q], all = 0;
            for (uint32_t j = 0; j < W; ++j) {
                if (j < wid) run += s_sc[q][j];
                all += s_sc[q][j];
            }
#pragma unroll
            for (uint32_t j = 0; j < kEpiloguePer; ++j)
                if (k0 + j < G) {
                    dst[q * G + k0 + j] = run;
                    run += xs[q][j];
                }
            carry[q] += all;
        }
        __syncthreads();   // s_sc is rewritten by the next round
    }
    if (threadIdx.x == 0)
        for (int q = 0; q < ncols; ++q) tot[q] = carry[q];
}

// ---- frontier lists -------------------------------------------------------------------------------
// Where a level's winners go: the invalidated bitmap and, for winners with a non-empty row, the next
// level's frontier list (row offset, length, exclusive edge offset; cstart for every fine chunk
// whose first edge the entry holds), reserved through the next level's packed counter.
struct Out {
    const uint64_t* __restrict__ row_off;
    const uint32_t* __restrict__ row_len;
    uint32_t* inv_bm;
    uint32_t* __restrict__ nfr_off;   // row offsets (edge pool positions < 2^32)
    uint32_t* __restrict__ nfr_len;
    uint64_t* __restrict__ nescan;
    uint32_t* __restrict__ ncstart;
    LevelCtr* ln;
};

// A frontier entry: its row (offset, length) and exclusive edge offset es, and the chunk map entries
// of the fine chunks whose first edge lies in [es, es + len). Lane-local form (rare overflow paths).
__device__ __forceinline__ void write_entry(const Out& o, uint64_t idx, uint64_t es, uint32_t off, uint32_t len) {
    o.nfr_off[idx] = off;
    o.nfr_len[idx] = len;
    o.nescan[idx] = es;
    const uint64_t c_lo = (es + kFine - 1) / kFine, c_hi = (es + len - 1) / kFine;
    for (uint64_t c = c_lo; c <= c_hi; ++c) o.ncstart[c] = (uint32_t)idx;
}

// The chunk map entries of one frontier entry per lane (has: the lane holds an entry, len > 0). A
// hub's row spans thousands of fine chunks: a span longer than kSpanSerial chunks is written by the
// whole wave, one lane per chunk, instead of by its own lane (a 1 M-edge row would otherwise be
// ~4,000 dependent store issues in one lane, the push level's slowest block). Edge offsets < 2^32.
// Every lane of the wave calls it.
constexpr uint32_t kSpanSerial = 4;
__device__ __forceinline__ void write_span(uint32_t* cstart, bool has, uint32_t idx, uint64_t es, uint32_t len) {
    uint32_t c_lo = 0, c_hi = 0;
    bool big = false;
    if (has) {
        c_lo = (uint32_t)((es + kFine - 1) / kFine);
        c_hi = (uint32_t)((es + len - 1) / kFine);
        if (c_hi + 1 - c_lo <= kSpanSerial) {
            for (uint32_t c = c_lo; c <= c_hi; ++c) cstart[c] = idx;
        } else {
            big = true;
        }
    }
    unsigned long long m = __ballot(big);
    while (m) {   // wave-uniform
        const int src = __builtin_ctzll(m);
        m &= m - 1;
        const uint32_t lo = __builtin_amdgcn_readlane(c_lo, src), hi = __builtin_amdgcn_readlane(c_hi, src);
        const uint32_t id = __builtin_amdgcn_readlane(idx, src);
        for (uint32_t c = lo + lane_id(); c <= hi; c += 64) cstart[c] = id;
    }
}

// write_entry for one entry per lane; every lane of the wave calls it
__device__ __forceinline__ void write_entry_wave(const Out& o, bool has, uint64_t idx, uint64_t es, uint32_t off,
                                                 uint32_t len) {
    if (has) {
        o.nfr_off[idx] = off;
        o.nfr_len[idx] = len;
        o.nescan[idx] = es;
    }
    write_span(o.ncstart, has, (uint32_t)idx, es, len);
}

__device__ __forceinline__ void mark_invalidated(uint32_t* inv_bm, uint32_t h) { atomicOr(inv_bm + (h >> 5), 1u << (h & 31)); }

// One (possibly absent) winner per lane. Every lane of the wave must call it.
__device__ __forceinline__ void emit_one(bool win, uint32_t h, const Out& o) {
    const uint32_t len = win ? o.row_len[h] : 0u;
    const uint32_t off = win ? (uint32_t)o.row_off[h] : 0u;   // requested with the length
    if (win) mark_invalidated(o.inv_bm, h);
    const unsigned long long mine = (win && len) ? ((1ull << 32) | len) : 0ull;
    unsigned long long tot;
    const unsigned long long ex = wave_excl_scan64(mine, tot);
    unsigned long long base = 0;
    if (lane_id() == 0 && tot) base = atomicAdd(&o.ln->ft, tot);
    base = from_lane0(base) + ex;
    write_entry_wave(o, win && len, base >> 32, base & 0xFFFFFFFFull, off, len);
}

// Block-level emission: winners are staged in LDS (buf) and appended in batches: one packed
// reservation per batch.
constexpr uint32_t kEmitCap = 1024;
constexpr uint32_t kChunkEmitCap = 2 * kChunk;   // push levels: staged over the chunk map
struct Emit {
    uint32_t n;
    uint32_t pad;
    unsigned long long base;
    uint32_t we[kBlock / 64];
    uint32_t wl[kBlock / 64];
};

__device__ __forceinline__ void emit_init(Emit& e) {
    if (threadIdx.x == 0) e.n = 0;
    __syncthreads();
}

// Every lane of the calling wave must call it (ballot); lanes beyond the LDS capacity append their
// winner alone.
template <uint32_t CAP>
__device__ __forceinline__ void emit_push(Emit& e, uint32_t* buf, bool win, uint32_t h, const Out& o) {
    const unsigned long long m = __ballot(win);
    if (!m) return;
    uint32_t base = 0;
    if (lane_id() == 0) base = atomicAdd(&e.n, (uint32_t)__popcll(m));
    base = from_lane0(base);
    if (win) {
        const uint32_t idx = base + rank_in(m);
        if (idx < CAP) {
            buf[idx] = h;
        } else {
            mark_invalidated(o.inv_bm, h);
            const uint32_t len = o.row_len[h];
            if (len) {
                const unsigned long long r = atomicAdd(&o.ln->ft, (1ull << 32) | len);
                write_entry(o, r >> 32, r & 0xFFFFFFFFull, (uint32_t)o.row_off[h], len);
            }
        }
    }
}

// Push chunks: the winner's row (offset, length) was gathered right after its visit (and its
// invalidated bit set there), so the flush reads both from LDS. A chunk stages at most kChunk
// winners: offsets in buf[0, kChunk), lengths in buf[kChunk, 2 kChunk). Every lane of the calling
// wave must call it.
__device__ __forceinline__ void emit_push_row(Emit& e, uint32_t* buf, bool win, uint32_t off, uint32_t len) {
    const unsigned long long m = __ballot(win);
    if (!m) return;
    uint32_t base = 0;
    if (lane_id() == 0) base = atomicAdd(&e.n, (uint32_t)__popcll(m));
    base = from_lane0(base);
    if (win) {
        const uint32_t idx = base + rank_in(m);
        buf[idx] = off;
        buf[kChunk + idx] = len;
    }
}

// Block-uniform call. Flushes when at least `at` winners are staged (at = 1: flush anything).
// Pass 1: every thread's entries (i = tid + k * kBlock) — invalidated bit, row length; one block
// scan of (entries with rows, edges) and one packed reservation. Pass 2: the entries in the same
// order at their reserved index and edge offset.
template <uint32_t CAP>
__device__ __forceinline__ void emit_flush(Emit& e, uint32_t* buf, uint32_t at, const Out& o) {
    __syncthreads();
    const uint32_t n = e.n < CAP ? e.n : CAP;
    __syncthreads();   // every thread has read e.n before any wave can push again
    if (n < at || n == 0) return;   // uniform decision
    // a push chunk stages each winner's row offset and length (emit_push_row): no gathers here, and
    // at most kChunk of them
    constexpr bool kStage2 = CAP == kChunkEmitCap;
    constexpr int kPer = (kStage2 ? kChunk : CAP) / kBlock;
    static_assert(!kStage2 || 2 * kChunk <= CAP, "push winners fit half the buffer");
    uint32_t cnt = 0, lsum = 0;
#pragma unroll
    for (int k = 0; k < kPer; ++k) {
        const uint32_t i = threadIdx.x + k * kBlock;
        if (i < n) {
            uint32_t len;
            if constexpr (kStage2) {
                len = buf[kChunk + i];
            } else {
                const uint32_t h = buf[i];
                mark_invalidated(o.inv_bm, h);
                len = o.row_len[h];
            }
            cnt += len ? 1u : 0u;
            lsum += len;
        }
    }
    uint32_t wtot_e, wtot_l;
    const uint32_t wex_e = wave_excl_scan(cnt, wtot_e), wex_l = wave_excl_scan(lsum, wtot_l);
    const uint32_t wid = threadIdx.x >> 6;
    if (lane_id() == 0) {
        e.we[wid] = wtot_e;
        e.wl[wid] = wtot_l;
    }
    __syncthreads();
    uint32_t be = 0, bl = 0, te = 0, tl = 0;
    for (uint32_t k = 0; k < kBlock / 64; ++k) {
        if (k < wid) {
            be += e.we[k];
            bl += e.wl[k];
        }
        te += e.we[k];
        tl += e.wl[k];
    }
    if (threadIdx.x == 0) e.base = te ? atomicAdd(&o.ln->ft, ((unsigned long long)te << 32) | tl) : 0ull;
    __syncthreads();
    uint64_t idx = (e.base >> 32) + be + wex_e;
    uint64_t es = (e.base & 0xFFFFFFFFull) + bl + wex_l;
#pragma unroll
    for (int k = 0; k < kPer; ++k) {   // block-uniform: every lane calls write_entry_wave
        const uint32_t i = threadIdx.x + k * kBlock;
        uint32_t len = 0, off = 0;
        if (i < n) {
            if constexpr (kStage2) {
                off = buf[i];
                len = buf[kChunk + i];
            } else {
                const uint32_t h = buf[i];
                len = o.row_len[h];   // an L2 hit now
                off = len ? (uint32_t)o.row_off[h] : 0u;
            }
        }
        write_entry_wave(o, len != 0, idx, es, off, len);
        if (len) {
            ++idx;
            es += len;
        }
    }
    __syncthreads();
    if (threadIdx.x == 0) e.n = 0;
    __syncthreads();
}

// Last block of a producer kernel (roots, push level, received targets): level L+1's F and T from
// the packed counter.
__device__ __forceinline__ void publish_ft(LevelCtr* ln, unsigned long long* done, uint64_t G) {
    if (last_block(done, G) && threadIdx.x == 0) {
        const unsigned long long ft = coh_read(&ln->ft);
        ln->F = ft >> 32;
        ln->T = ft & 0xFFFFFFFFull;
    }
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
    base = from_lane0(base);
    if (send) {
        const uint32_t idx = base + rank_in(m);
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
// One root per lane (i < n), every lane of the wave calls it: the visit, the frontier entry, the
// root counters.
// Roots given as boundary handles (fgi_invalidate*, labels active): handle x is label s2l[x] if hot,
// else K + x; anything past ext_handles is no handle (ignored like any out-of-range root)
struct RootMap {
    const uint32_t* s2l;
    uint32_t ext_slots, ext_handles, K;
    int on;
};
__device__ __forceinline__ uint32_t root_label(const RootMap& m, uint32_t x) {
    if (x >= m.ext_handles) return FGI_NONE;
    if (m.s2l && x < m.ext_slots) {
        const uint32_t l = m.s2l[x];
        if (l != FGI_NONE) return l;
    }
    return x + m.K;
}

template <int IMM>
__device__ __forceinline__ void root_step(uint32_t i, const uint32_t* __restrict__ roots, const uint8_t* __restrict__ imm,
                                          uint32_t n, uint32_t base, uint32_t n_range, unsigned long long* node,
                                          uint32_t* vis, const Out& o, WaveCtr* ctr, const RootMap& rm = RootMap{}) {
    uint32_t win = 0, flagged = 0, h = 0;
    if (i < n) {
        h = rm.on ? root_label(rm, roots[i]) : roots[i] - base;
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

// publish: unpack level 0's totals into F / T (the partitioned wave all-reduces those words);
// the single engine reads the packed counter (lvl_F / lvl_T) and skips the hand-off
template <int IMM>
// stamp: no k_wave_init ran before this wave (the previous one left the state clean): the wave's start on
// the device wall clock is stamped here instead (WaveCtr::t0)
__global__ __launch_bounds__(kBlock) void k_roots(const uint32_t* __restrict__ roots, const uint8_t* __restrict__ imm,
                                                  uint32_t n, uint32_t base, uint32_t n_range, unsigned long long* node,
                                                  uint32_t* vis, Out o, WaveCtr* ctr, unsigned long long* done,
                                                  int publish, RootMap rm, int stamp) {
    if (stamp && blockIdx.x == 0 && threadIdx.x == 0) ctr->t0 = wall_clock64();
    root_step<IMM>(blockIdx.x * blockDim.x + threadIdx.x, roots, imm, n, base, n_range, node, vis, o, ctr, rm);
    if (publish) publish_ft(o.ln, done, gridDim.x);
}

// ---- the level's direction ------------------------------------------------------------------------
struct WaveParams {
    int multi;                  // partitioned wave: the host sets lvl[L].pull after its all-reduce
    int direction;              // 0 auto, 1 push only, 2 pull only
    uint64_t pull_threshold;    // alpha rule: pull when the frontier's edges exceed E / alpha
    uint64_t stay_pull_f;       // beta rule: after a pull, pull again while F exceeds n / beta
    uint32_t grid;              // blocks of k_level / k_collect
    uint32_t tpb;               // pull tiles per block
    uint64_t n_tiles;
};

// Beamer's two rules, as a pure function of the counters (every block decides the same).
__device__ __forceinline__ bool level_pulls(const WaveCtr* ctr, int L, const WaveParams& wp, uint64_t F, uint64_t T) {
    if (F == 0 || wp.direction == 1) return false;
    if (wp.direction == 2) return true;
    const bool prev_pull = L > 0 && ctr->lvl[(L + kRing - 1) % kRing].pull != 0;
    return T > wp.pull_threshold || (prev_pull && F > wp.stay_pull_f);
}
__device__ __forceinline__ bool level_pulls(const WaveCtr* ctr, int L, const WaveParams& wp) {
    const LevelCtr& lc = ctr->lvl[L % kRing];
    if (wp.multi) return lc.pull != 0;
    return level_pulls(ctr, L, wp, lvl_F(lc), lvl_T(lc));
}

// A level group's end (run_wave): the wave is over when the level after the group's last one — or after
// the last one its tail ran (ctr->cur) — has no frontier. The host decides the same from the published
// counters, so the final kernels and the publish can leave the wave state clean for the next wave
// (WaveEnd) exactly when the host will not run another group.
struct WaveEnd {
    WaveCtr* ctr;            // null: the state is left as it is
    int L;                   // the first level the group did not launch
    int tail;                // the group ended with k_wave_tail
    unsigned long long* blk; // per-block statistics, cleared with the invalidated bitmap
    uint32_t* inv_bm;        // the labels' invalidated bitmap: ext words of it cleared (64-bit words)
    uint64_t words;          // 64-bit words of inv_bm the wave can have set (n_handles / 64, rounded up)
    uint32_t* spare;         // the other visit bitmap, cleared whether the wave is over or not (nullable)
};
__device__ __forceinline__ bool wave_over(const WaveEnd& e) {
    const uint64_t stop = e.tail ? max((uint64_t)e.L, (uint64_t)e.ctr->cur) : (uint64_t)e.L;
    return lvl_F(e.ctr->lvl[stop % kRing]) == 0;
}

// fine chunks per expand chunk: as large as kEPT allows while every block still gets two chunks
__device__ __forceinline__ uint32_t level_mult(uint64_t T, uint32_t grid) {
    const uint64_t nfine = (T + kFine - 1) / kFine;
    uint32_t m = 1;
    while (m < (uint32_t)kEPT && (nfine + 2 * m - 1) / (2 * m) >= 2ull * grid) m <<= 1;
    return m;
}

// A cascade's grid (k_wave_coop) is one block per CU and its levels are small: the largest chunks
// that still leave every chunk its own block, so a level is one round of chunks (each chunk is a chain
// of dependent round trips; a second round doubles the level). A 100-hub wave's leaf level (100 k
// edges) takes 196 chunks of 512 edges instead of 391 of 256 over 256 blocks.
__device__ __forceinline__ uint32_t level_mult_one_round(uint64_t T, uint32_t grid) {
    const uint64_t nfine = (T + kFine - 1) / kFine;
    uint32_t m = 1;
    while (m < (uint32_t)kEPT && (nfine + m - 1) / m > grid) m <<= 1;
    return m;
}

// ---- collect: a pull level's winners lists -> the next level's frontier list ------------------
// Pull block b listed its expandable winners at wl[seg[b] ..); the pull's last block left the
// exclusive prefixes of the per-block (winners, expandable winners, row lengths) sums in pre[].
// One wave per pull block: 64 entries per step, their row lengths and offsets gathered together,
// a wave scan for the edge offsets, the entries written at the block's offsets (frontier order is
// the lists' order: a push does not depend on it).
struct CollectArgs {
    const uint32_t* __restrict__ wl;
    const uint32_t* __restrict__ seg;
    const uint32_t* __restrict__ row_len;
    const uint64_t* __restrict__ row_off;
    const unsigned long long* __restrict__ pre;   // [3][grid]: winners, expandable winners, lengths
    uint32_t* fr_off;
    uint32_t* fr_len;
    uint64_t* escan;
    uint32_t* cstart;
    // hot heads: before a pull level, hot_bm = the invalidated bits of hot_id[0 .. n_hot)
    const uint32_t* __restrict__ hot_id;
    uint32_t* hot_bm;
    uint32_t n_hot;
    const uint32_t* inv;
    // probe summary (single engine; null for a partition): one bit per 64-bit word of inv
    unsigned long long* sum_bm;
    uint64_t n64;               // 64-bit words of inv the pull levels probe
    int64_t sum_min;            // fewest words for a summary (< 0: never)
};

constexpr int kCollectThreads = 256;

// The hot heads' snapshot before a pull level: one entry per lane, 64 bits per wave (n_hot and the
// thread stride are multiples of 64).
__device__ __forceinline__ void collect_hot(const CollectArgs& c, uint64_t tid, uint64_t stride) {
    unsigned long long* hot64 = reinterpret_cast<unsigned long long*>(c.hot_bm);
    for (uint64_t k = tid; k < c.n_hot; k += stride) {
        const uint32_t u = c.hot_id[k];
        const unsigned long long m = __ballot(u != FGI_NONE && bit_of(c.inv, u));
        if (lane_id() == 0) hot64[k >> 6] = m;
    }
}

// Before pull level L, while few bitmap words can be nonzero (at most the invalidated count so far,
// estimated from the levels' frontiers: sum * 8 < words), one bit per 64-bit word of the invalidated
// bitmap, set iff the word is nonzero: a cold probe that would miss (most of them, that early) reads
// the L2-resident summary instead of a line of a bitmap larger than L2 (R-MAT 27: 16 MB against 4 MB
// of L2 per XCD). Level L's `sum` word says whether the pull level may use it; every pull level's
// k_collect writes it. One summary word per wave and step (64 coalesced bitmap words).
__device__ __forceinline__ void collect_sum(const CollectArgs& c, WaveCtr* ctr, int L, uint64_t wave, uint64_t waves) {
    bool use = c.sum_bm != nullptr && c.sum_min >= 0 && c.n64 >= (uint64_t)c.sum_min && L < kRing - 4;
    if (use) {
        uint64_t S = 0;
        for (int l = 0; l <= L; ++l) S += lvl_F(ctr->lvl[l]);
        use = S * 8 < c.n64;
    }
    if (blockIdx.x == 0 && threadIdx.x == 0) ctr->lvl[L % kRing].sum = use ? 1ull : 0ull;
    if (!use) return;
    const unsigned long long* inv64 = reinterpret_cast<const unsigned long long*>(c.inv);
    const uint32_t lane = lane_id();
    for (uint64_t w = wave; w * 64 < c.n64; w += waves) {   // wave-uniform
        const uint64_t i = w * 64 + lane;
        const unsigned long long m = __ballot(i < c.n64 && inv64[i] != 0ull);
        if (lane == 0) c.sum_bm[w] = m;
    }
}

// Push level L's frontier list from pull level L-1's per-block winners lists: one wave per pull block
// (waves w0, w0 + W, ... of the caller's grid).
__device__ __forceinline__ void collect_front(const LevelCtr& lc, uint64_t G, const CollectArgs& c, uint64_t w0,
                                              uint64_t W) {
    const uint32_t lane = lane_id();
    for (uint64_t b = w0; b < G; b += W) {   // wave-uniform
        const uint64_t e0 = c.pre[G + b], e1 = b + 1 < G ? c.pre[G + b + 1] : lvl_F(lc);
        uint64_t es = c.pre[2 * G + b];
        const uint64_t base = c.seg[b];
        for (uint64_t i0 = 0; i0 < e1 - e0; i0 += 64) {
            const uint64_t i = i0 + lane;
            const bool in = i < e1 - e0;
            const uint32_t d = in ? c.wl[base + i] : 0u;
            const uint32_t len = in ? c.row_len[d] : 0u;
            const uint32_t off = in ? (uint32_t)c.row_off[d] : 0u;   // pool positions are < 2^32
            uint32_t tot;
            const uint32_t ex = wave_excl_scan(len, tot);
            const uint64_t idx = e0 + i, e = es + ex;
            if (in) {
                c.fr_off[idx] = off;
                c.fr_len[idx] = len;
                c.escan[idx] = e;
            }
            write_span(c.cstart, in && len, (uint32_t)idx, e, len);
            es += tot;
        }
    }
}

// A fused wave's k_collect / k_level launch with mid index i (passed as L = -1 - i): its level is
// mid_base + i, run only while it is still the wave's current level (a launch past the levels that
// need one, or a block reading `cur` after its own launch advanced it, finds another level and does
// nothing). Returns -1 if there is nothing to do.
__device__ __forceinline__ int mid_level(const WaveCtr* ctr, int L) {
    if (L >= 0) return L;
    if (ctr->phase == kPhaseDone || ctr->broken) return -1;
    const uint64_t want = ctr->mid_base + (uint64_t)(-1 - L);
    return ctr->cur == want ? (int)want : -1;
}

// Level L's frontier list when level L-1 pulled and level L pushes; before a pull level, the hot
// heads' snapshot; otherwise nothing to do. Fused waves (L < 0, mid index): only for the levels the
// k_level launch will run (pull, or a push of more than big_push edges); the small push levels and
// their collect run in the fused tail kernel.
__global__ __launch_bounds__(kCollectThreads) void k_collect(int L, WaveCtr* ctr, WaveParams wp, CollectArgs c,
                                                             CollectArgs c1, uint64_t big_push) {
    const bool fused = FGI_VARIANTS && L < 0;
    L = mid_level(ctr, L);
    if (L < 0) return;
    if (fused && (L & 1)) c = c1;   // a fused wave's level is known on the device only: odd levels, buffer 1
    const LevelCtr& lc = ctr->lvl[L % kRing];
    // a partition's pull level runs on every rank, also on one whose own frontier is empty (its
    // candidates' parents may be remote): its hot snapshot is needed all the same
    if (lvl_F(lc) == 0 && !wp.multi) return;
    if (level_pulls(ctr, L, wp)) {
        collect_hot(c, (uint64_t)blockIdx.x * blockDim.x + threadIdx.x, (uint64_t)gridDim.x * blockDim.x);
        if (FGI_VARIANTS && c.sum_bm)
            collect_sum(c, ctr, L, (uint64_t)blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6),
                        (uint64_t)gridDim.x * (blockDim.x >> 6));
        return;
    }
    if (lvl_F(lc) == 0 || (fused && lvl_T(lc) <= big_push)) return;
    if (L == 0 || !ctr->lvl[(L + kRing - 1) % kRing].pull) return;
    collect_front(lc, wp.grid, c, (uint64_t)blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6),
                  (uint64_t)gridDim.x * (blockDim.x >> 6));
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

// measured slower on configs[1] (0.2354-0.2362 against 0.2333-0.2340 ms/step off, one box,
// profiles/r11_tail_ab.txt r12f): off by default, FGI_PUSH_SMALL=<edges> for measurement
constexpr uint64_t kPushSmallMax = 0;

struct ExpandArgs {
    const uint32_t* __restrict__ fr_off;
    const uint64_t* __restrict__ escan;
    const uint32_t* __restrict__ cstart;
    const uint32_t* __restrict__ pool_col;
    const uint64_t* __restrict__ pool_tag;
    int dead_filter;
    // levels of fewer edges (a measurement knob, FGI_PUSH_SMALL): no separate dead-edge filter trip
    // (visited targets are caught by the visit's plain read) and the winners' rows gathered with the
    // tags, speculatively (12 B per matched edge). 0: never (the default)
    uint64_t small_max = kPushSmallMax;
};

// PART: multi-GPU rank — dependant slots outside [ra.base, ra.base + ra.n_local) are remote: their
// tag is checked against the version replica and matching targets are forwarded once per wave.
template <bool PART>
__device__ __forceinline__ void expand_level(int L, uint64_t F, uint64_t T, uint32_t mult, const ExpandArgs& x,
                                             const unsigned long long* node, uint32_t* vis, const Out& o, Emit& em,
                                             uint32_t* eb, MsgEmit<PART>& me, uint32_t* s_rel, uint32_t* s_base,
                                             unsigned long long* blk, unsigned long long (*s_st)[kStats],
                                             const RemoteArgs& ra) {
    if constexpr (PART) {
        if (threadIdx.x == 0) me.n = 0;
    }
    const uint64_t nfine = (T + kFine - 1) / kFine;
    const uint64_t nch = (nfine + mult - 1) / mult;
    const uint64_t cedges = (uint64_t)mult * kFine;
    uint32_t matched = 0, flagged = 0;
    for (uint64_t c = blockIdx.x; c < nch; c += gridDim.x) {
        const uint64_t cbase = c * cedges;
        const uint32_t clen = (uint32_t)((T - cbase) < cedges ? (T - cbase) : cedges);
        const uint32_t i0 = x.cstart[c * mult];
        const uint32_t i1 = (c + 1 < nch) ? x.cstart[(c + 1) * mult] : (uint32_t)(F - 1);
        const uint32_t n = i1 - i0 + 1;
        // n <= cedges + 1 entries: every load issued before the first use
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
        PROBE(L, 4);
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
        // edges to nodes visited earlier need neither the tag nor the gather (the bitmap is read
        // without synchronisation: a stale 0 only costs the gather and an atomic that finds the bit).
        // Kept on small levels too (round 3 measured the alternative: no gain)
        const bool small = T < x.small_max;   // level-uniform
        if (x.dead_filter && !small) {
#pragma unroll
            for (int j = 0; j < kEPT; ++j)
                if (dst[j] != 0xFFFFFFFFu && bit_of(vis, dst[j])) dst[j] = 0xFFFFFFFFu;
        }
        PROBE(L, 5);
        uint64_t tag[kEPT];
        unsigned long long w[kEPT];
        uint32_t rl[kEPT], ro[kEPT];
#pragma unroll
        for (int j = 0; j < kEPT; ++j) {
            tag[j] = 0;
            w[j] = 0;
            rl[j] = 0;
            ro[j] = 0;
            if (dst[j] != 0xFFFFFFFFu) {
                tag[j] = __builtin_nontemporal_load(x.pool_tag + pos[j]);
                w[j] = node[dst[j]];
                if (small) {
                    rl[j] = o.row_len[dst[j]];
                    ro[j] = (uint32_t)o.row_off[dst[j]];   // pool positions are < 2^32
                }
            }
        }
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
        // a winner's invalidated bit and its row, requested as soon as its visit has returned (the
        // flush then needs no gather round trip); a small level has its rows already
#pragma unroll
        for (int j = 0; j < kEPT; ++j) {
            if ((win_mask >> j) & 1u) {
                mark_invalidated(o.inv_bm, dst[j]);
                if (!small) {
                    rl[j] = o.row_len[dst[j]];
                    ro[j] = (uint32_t)o.row_off[dst[j]];   // pool positions are < 2^32
                }
            } else {
                rl[j] = 0;
                ro[j] = 0;
            }
        }
        // the chunk's winners (at most cedges) are staged over the chunk map, flushed before the
        // next chunk refills it
        __syncthreads();
        PROBE(L, 6);
#pragma unroll
        for (int j = 0; j < kEPT; ++j) emit_push_row(em, eb, (win_mask >> j) & 1u, ro[j], rl[j]);
        emit_flush<kChunkEmitCap>(em, eb, 1, o);
        PROBE(L, 7);
        if constexpr (PART) msg_flush(me, kMsgCap / 2, ra);
    }
    if constexpr (PART) msg_flush(me, 1, ra);
    const uint32_t v[kStats] = {matched, flagged, 0, 0, 0, 0, 0, 0};
    block_stats_add(blk, s_st, v);
}

// ---- pull: every live candidate looks for an invalidated parent --------------------------------
// uin_* is the dependency-list cache: for slot d, the handles u whose `_usedBy` row holds
// (d, version(d)) — the reference's d._used (Computed.cs:36, 365-366). An invalidated parent means
// the push step would visit d from it (in this level or already in the previous one).
// Only slots with a non-empty list can ever be reached bottom-up (R-MAT 24: about half of them), and
// each pull level leaves fewer unvisited: a level reads the candidate list of its block (the static
// list on the wave's first pull, the previous pull's survivors after that) and writes its own
// survivors forward.
struct PullArgs {
    uint32_t n_slots;
    const uint64_t* __restrict__ uin_off;
    const uint32_t* __restrict__ uin_len;
    const uint32_t* __restrict__ uin_src;
    const uint32_t* front_rd;                // invalidated bitmap (multi-GPU: all-gathered, global ids)
    const uint32_t* sum;                     // probe summary of front_rd (null: none; level's `sum` word)
    uint32_t hot_bit0;                       // a hot head's code: hot_bit0 + rank (its snapshot bit)
    uint32_t hot_lds;                        // hot snapshot words staged into LDS per block (<= kLdsHot)
    uint32_t* inv_bm;                        // this device's invalidated bitmap (owned words |= winners)
    const uint32_t* __restrict__ cls;        // expandable-class bitmap
    uint32_t* wl;                            // per block (at its segment base): expandable winners
    unsigned long long* bsum;                // [3][grid] per-block sums, then [3][grid] prefixes
    const uint32_t* __restrict__ cand_seg;   // [grid + 1] segment bases
    const uint4* c[3];                       // [0] the static candidates, [1 + k] survivors buffer k
    uint4* sv[2];
    uint32_t* sv_cnt[2];                     // [grid] survivors per block
};

// A block owns the tiles [b * tpb, (b + 1) * tpb) (tpb <= kMaxIter): their visit, class and winners
// words live in LDS for the whole level (loaded once, coalesced) and the visit / winners words are
// written back once (owned words, plain stores), so a pull level does no global atomics and a
// candidate's only global gathers are the invalidated bits of its two list heads (hot heads: an
// L1-resident snapshot). Candidates are read 4 per lane per batch (one 16-byte entry each,
// streamed); a hit is a visit. A winner with a non-empty row is appended to the block's winners
// list (for the collect, if the next level pushes); the block's winner / expandable / row-length
// totals are per-thread register sums. Candidates whose heads missed but whose list goes on are
// queued in LDS and scanned at the wave's flush (pull_tails). Candidates neither hit nor queued,
// and queued ones whose scan found nothing, are this level's survivors.
constexpr uint32_t kMaxIter = 32;           // tiles per pull block (kMaxIter * kPullTile slots)
#ifndef FGI_CPL
#define FGI_CPL 4          // measurement builds: make variant-cpl CPL=<candidates per lane> TCAP=<queue words>
#endif
#ifndef FGI_TAIL_CAP
#define FGI_TAIL_CAP kChunk
#endif
constexpr uint32_t kCPL = FGI_CPL;          // candidates per lane per step
constexpr uint32_t kTailCap = FGI_TAIL_CAP; // queued candidates
constexpr uint32_t kTileWords = kPullTile / 64;
constexpr uint32_t kOwnWords = 2 * kMaxIter * kTileWords;   // owned 32-bit bitmap words
constexpr uint32_t kCandBatch = kCPL * kBlock; // candidates per block step (kCPL per lane)
constexpr uint32_t kWaveBatch = kCPL * 64;     // a wave's run per step
constexpr uint32_t kWaveTailCap = kTailCap / (kBlock / 64);   // queued candidates per wave
constexpr uint32_t kLaneTail = 12;          // lists a lane scans alone in a tail pass (entries 4..11)

// visits / winners / classes of the owned tiles in LDS: 32-bit words (two lanes of a wave that
// share a word serialise their atomics; narrower words halve how many do)
struct PullLds {
    uint32_t hot[kLdsHot];                          // the hot heads' snapshot (first hot_lds words)
    uint32_t vm[kOwnWords];                         // visits: the level's start, | this level's non-winners
    uint32_t wm[kOwnWords];                         // winners
    uint32_t cs[kOwnWords];                         // expandable class (read only)
    uint32_t sn;                                    // survivors written
    uint32_t wn;                                    // expandable winners listed
};

// k_level's LDS (32-bit words): push — the chunk map, then the chunk's winners; pull — the tail queue
// (kTailCap) and PullLds at kTailCap + 4
// the multi-GPU push's per-owner staging (MsgEmit<true>) follows the push region
constexpr uint32_t kPushLds = kChunkEmitCap + 8;
constexpr uint32_t kLevelLds =
    std::max<uint32_t>(kPushLds + (sizeof(MsgEmit<true>) + 7) / 8 * 2, kTailCap + 4 + (sizeof(PullLds) + 3) / 4);
static_assert(kTailCap % 4 == 0 && kWaveBatch <= kTailCap / (kBlock / 64), "pull tail queue");

// a thread's winners: count, those with a non-empty row, their row lengths
struct WinSum {
    uint32_t w = 0, e = 0;
    unsigned long long l = 0;
};

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

// the bitmap word holding a list head's invalidated bit: a hot head's code indexes the snapshot
// that follows the invalidated bitmap (g->hot_w0), any other head the bitmap itself. The snapshot's
// first hot_lds words are read from the block's LDS copy: a random probe of an L2-resident bitmap
// costs ~4x an L1 hit and ~5x an LDS read (profiles/r5f_probe_rate.txt, r5g_snap_rate.txt)
__device__ __forceinline__ bool sum_zero(const PullArgs& p, uint32_t h) {
    return !((p.sum[h >> 11] >> ((h >> 6) & 31)) & 1u);   // h's 64-bit bitmap word is zero
}
__device__ __forceinline__ uint32_t head_bits(const PullArgs& p, const PullLds& s, uint32_t h, bool sum) {
    const uint32_t r = (h - p.hot_bit0) >> 5;   // wraps past hot_lds for a cold head
    if (r < p.hot_lds) return s.hot[r];
    if (sum && h < p.hot_bit0 && sum_zero(p, h)) return 0u;   // a cold head in a zero word
    return p.front_rd[h >> 5];
}
// a tail entry's invalidated bit (entries are handles, never hot codes)
__device__ __forceinline__ bool front_bit(const PullArgs& p, uint32_t u, bool sum) {
    return !(sum && sum_zero(p, u)) && bit_of(p.front_rd, u);
}

// an entry past the list reads as a dead candidate at the block's first slot
__device__ __forceinline__ uint4 load_cand(const uint4* p, bool in, uint32_t s_lo) {
    if (!in) return make_uint4(s_lo, 0u, FGI_NONE, FGI_NONE);
    const u32x4 v = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(p));
    return make_uint4(v.x, v.y, v.z, v.w);
}

// one lane's hit (tails): visit bits, and a winner's sums and list entry
__device__ __forceinline__ void pull_hit(const PullArgs& p, PullLds& s, uint64_t s_lo, uint64_t seg, uint32_t d, bool win,
                                         uint32_t aux, WinSum& ws) {
    const uint32_t rel = (uint32_t)(d - s_lo);
    const uint32_t bit = 1u << (d & 31);
    if (win) {
        atomicOr(&s.wm[rel >> 5], bit);
        const uint32_t rl = aux & 0x7FFFFFFFu;
        ++ws.w;
        if (rl) {
            ++ws.e;
            ws.l += rl;
            p.wl[seg + atomicAdd(&s.wn, 1u)] = d;
        }
    } else {
        atomicOr(&s.vm[rel >> 5], bit);
    }
}

// A wave's queued candidates (both heads missed, the list goes on). Pass 1: one lane per candidate
// probes entries 2 and 3 (both in flight together) — most queued candidates settle here. Pass 2a:
// lists of at most kLaneTail entries that go past entry 3 without a hit, one lane per candidate with
// all of entries 4.. in flight (configs[0]'s 8-entry lists of nodes two levels ahead: 64 per step
// instead of 8). Pass 2b: the longer lists, 8 lanes per candidate over entries 4.. in steps of 8
// (early exit); the next candidate's list is located while the current one is scanned. q (the wave's
// queue of candidate indices) is reused for pass 2's lists (bit 31: longer than kLaneTail).
__device__ __forceinline__ void pull_tails(const PullArgs& p, const uint4* src, uint4* sv_out, const unsigned long long* node,
                                           uint64_t s_lo, uint64_t seg, uint32_t* q, uint32_t nq, PullLds& s,
                                           uint32_t& flagged, uint32_t& examined, uint32_t& tails, WinSum& ws, bool sum) {
    const uint32_t lane = lane_id();
    uint32_t nlong = 0;
    for (uint32_t r0 = 0; r0 < nq; r0 += 64) {   // wave-uniform
        const uint32_t e = r0 + lane;
        const bool in = e < nq;
        uint32_t qi = 0, len = 0;
        uint64_t off = 0;
        uint4 c = make_uint4(0u, 0u, 0u, 0u);
        if (in) {
            qi = q[e];
            c = src[seg + qi];
            len = p.uin_len[c.x];
            off = p.uin_off[c.x];
        }
        const uint32_t u2 = (in && len > 2) ? p.uin_src[off + 2] : FGI_NONE;
        const uint32_t u3 = (in && len > 3) ? p.uin_src[off + 3] : FGI_NONE;
        const bool hit = (u2 != FGI_NONE && front_bit(p, u2, sum)) || (u3 != FGI_NONE && front_bit(p, u3, sum));
        examined += (u2 != FGI_NONE ? 1u : 0u) + (u3 != FGI_NONE ? 1u : 0u);
        const bool more = in && !hit && len > 4;
        const unsigned long long mm = __ballot(more);
        if (more) q[nlong + rank_in(mm)] = qi | (len > kLaneTail ? 0x80000000u : 0u);   // below every entry still unread
        nlong += (uint32_t)__popcll(mm);
        if (in && hit) {
            const uint32_t d = c.x, rel = (uint32_t)(d - s_lo);
            const bool win = (s.cs[rel >> 5] >> (d & 31)) & 1u;
            pull_hit(p, s, s_lo, seg, d, win, c.y, ws);
            if (!win) flagged += first_visit(node[d]) == 2 ? 1u : 0u;
        }
        const bool surv = in && !hit && !more;
        const unsigned long long sm = __ballot(surv);
        if (sm) {
            uint32_t sb = 0;
            if (lane == 0) sb = atomicAdd(&s.sn, (uint32_t)__popcll(sm));
            sb = from_lane0(sb);
            if (surv) sv_out[sb + rank_in(sm)] = c;
        }
        tails += in ? 1u : 0u;
    }
    __builtin_amdgcn_wave_barrier();
    // pass 2a: the short lists, one lane each; the long ones compacted to the queue's front
    uint32_t nl2 = 0;
    for (uint32_t r0 = 0; r0 < nlong; r0 += 64) {   // wave-uniform
        const uint32_t e = r0 + lane;
        const uint32_t v = e < nlong ? q[e] : 0u;
        const bool in = e < nlong && !(v >> 31);
        const bool lng = e < nlong && (v >> 31);
        const unsigned long long lm = __ballot(lng);
        if (lng) q[nl2 + rank_in(lm)] = v & 0x7FFFFFFFu;   // below every entry still unread
        nl2 += (uint32_t)__popcll(lm);
        uint4 c = make_uint4(0u, 0u, 0u, 0u);
        uint32_t len = 0;
        uint64_t off = 0;
        if (in) {
            c = src[seg + v];
            len = p.uin_len[c.x];
            off = p.uin_off[c.x];
        }
        uint32_t u[kLaneTail - 4];
#pragma unroll
        for (uint32_t k = 0; k < kLaneTail - 4; ++k) u[k] = (in && 4 + k < len) ? p.uin_src[off + 4 + k] : FGI_NONE;
        bool found = false;
#pragma unroll
        for (uint32_t k = 0; k < kLaneTail - 4; ++k)
            if (u[k] != FGI_NONE) {
                found |= front_bit(p, u[k], sum);
                ++examined;
            }
        if (in && found) {
            const uint32_t d = c.x, rel = (uint32_t)(d - s_lo);
            const bool win = (s.cs[rel >> 5] >> (d & 31)) & 1u;
            pull_hit(p, s, s_lo, seg, d, win, c.y, ws);
            if (!win) flagged += first_visit(node[d]) == 2 ? 1u : 0u;
        }
        const bool surv = in && !found;
        const unsigned long long sm = __ballot(surv);
        if (sm) {
            uint32_t sb = 0;
            if (lane == 0) sb = atomicAdd(&s.sn, (uint32_t)__popcll(sm));
            sb = from_lane0(sb);
            if (surv) sv_out[sb + rank_in(sm)] = c;
        }
    }
    nlong = nl2;
    __builtin_amdgcn_wave_barrier();
    const uint32_t sub = lane & 7, grp = lane >> 3;
    constexpr uint32_t G8 = 8;
    uint4 c_n = make_uint4(0u, 0u, 0u, 0u);
    uint32_t len_n = 0;
    uint64_t off_n = 0;
    if (grp < nlong) {
        c_n = src[seg + q[grp]];
        len_n = p.uin_len[c_n.x];
        off_n = p.uin_off[c_n.x];
    }
    for (uint32_t e = grp; e < nlong; e += G8) {
        const uint4 c = c_n;
        const uint32_t len = len_n;
        const uint64_t off = off_n;
        if (e + G8 < nlong) {
            c_n = src[seg + q[e + G8]];
            len_n = p.uin_len[c_n.x];
            off_n = p.uin_off[c_n.x];
        }
        bool found = false;
        for (uint32_t r = 4; r < len && !found; r += 8) {   // group-uniform
            const uint32_t k = r + sub;
            const bool x = k < len && front_bit(p, p.uin_src[off + k], sum);
            examined += (k < len) ? 1u : 0u;
            found = ((__ballot(x) >> (lane & ~7u)) & 0xFFull) != 0;
        }
        if (sub == 0) {
            const uint32_t d = c.x;
            if (found) {
                const uint32_t rel = (uint32_t)(d - s_lo);
                const bool win = (s.cs[rel >> 5] >> (d & 31)) & 1u;
                pull_hit(p, s, s_lo, seg, d, win, c.y, ws);
                if (!win) flagged += first_visit(node[d]) == 2 ? 1u : 0u;
            } else {
                sv_out[atomicAdd(&s.sn, 1u)] = c;
            }
        }
    }
}

__device__ __forceinline__ void pull_level(int L, const PullArgs& p, const WaveParams& wp, uint64_t npull, bool sum,
                                           const unsigned long long* node, uint32_t* vis, uint32_t* lds_q, PullLds& s,
                                           unsigned long long* blk, unsigned long long (*s_st)[kStats],
                                           unsigned long long (&bs)[3]) {
    uint32_t flagged = 0, examined = 0, live = 0, tails = 0, examined_tail = 0;
    const uint32_t lane = lane_id();
    const uint32_t b = blockIdx.x;
    const uint64_t s_lo = (uint64_t)b * wp.tpb * kPullTile;
    const uint64_t seg = p.cand_seg[b];
    const int sid = npull == 0 ? 0 : 1 + (int)((npull - 1) & 1);
    const int dst = (int)(npull & 1);
    const uint4* src = p.c[sid];
    // a block's survivors are a subset of its candidate segment: the count read back is clamped to it,
    // so a corrupt count cannot walk into the next block's segment
    const uint32_t seg_n = (uint32_t)(p.cand_seg[b + 1] - seg);
    const uint32_t cnt = npull == 0 ? seg_n : min(p.sv_cnt[sid - 1][b], seg_n);
    uint4* const sv_out = p.sv[dst] + seg;     // this level's survivors (the block's segment)
    uint32_t* const wl_out = p.wl + seg;       // this level's expandable winners
    // the first batch's entries are requested before the owned words are staged
    uint4 c[kCPL];
#pragma unroll
    for (int j = 0; j < (int)kCPL; ++j) {
        const uint32_t i = (threadIdx.x >> 6) * kWaveBatch + j * 64 + lane;
        c[j] = load_cand(src + seg + i, i < cnt, (uint32_t)s_lo);
    }
    {
        // every word's loads are issued before the first LDS store (one memory round trip, not one
        // per grid-stride step)
        const uint64_t w_lo = s_lo >> 5, w_end = ((uint64_t)p.n_slots + 31) >> 5;
        const uint32_t nw = 2 * wp.tpb * kTileWords;
        constexpr uint32_t kPer = kOwnWords / kBlock;
        constexpr uint32_t kHotPer = kLdsHot / kBlock;
        uint32_t vv[kPer], cc[kPer], hh[kHotPer];
#pragma unroll
        for (uint32_t k = 0; k < kPer; ++k) {
            const uint32_t i = threadIdx.x + k * kBlock;
            const bool in = i < nw && w_lo + i < w_end;
            vv[k] = in ? vis[w_lo + i] : ~0u;
            cc[k] = in ? p.cls[w_lo + i] : 0u;
        }
        const uint32_t* hot = p.front_rd + (p.hot_bit0 >> 5);
#pragma unroll
        for (uint32_t k = 0; k < kHotPer; ++k) {
            const uint32_t i = threadIdx.x + k * kBlock;
            hh[k] = i < p.hot_lds ? hot[i] : 0u;
        }
#pragma unroll
        for (uint32_t k = 0; k < kPer; ++k) {
            const uint32_t i = threadIdx.x + k * kBlock;
            if (i < nw) {
                s.vm[i] = vv[k];
                s.cs[i] = cc[k];
                s.wm[i] = 0;
            }
        }
#pragma unroll
        for (uint32_t k = 0; k < kHotPer; ++k) s.hot[threadIdx.x + k * kBlock] = hh[k];
    }
    if (threadIdx.x == 0) {
        s.sn = 0;
        s.wn = 0;
    }
    __syncthreads();
    PROBE(L, 1);
    WinSum ws;
    // every wave streams its own 256-candidate runs (4 entries per lane) and scans its own tail
    // queue: no block barrier until the write-back
    const uint32_t wid = threadIdx.x >> 6;
    uint32_t* wq = lds_q + wid * kWaveTailCap;
    uint32_t qn = 0;
    for (uint32_t base = wid * kWaveBatch; base < cnt; base += kCandBatch) {   // wave-uniform
        bool lv[kCPL];
        uint32_t f0[kCPL], f1[kCPL];
#pragma unroll
        for (int j = 0; j < (int)kCPL; ++j) {
            const bool in = base + j * 64 + lane < cnt;
            const uint32_t rel = c[j].x - (uint32_t)s_lo;
            lv[j] = in && !((s.vm[rel >> 5] >> (c[j].x & 31)) & 1u);
            f0[j] = lv[j] ? head_bits(p, s, c[j].z, sum) : 0u;
            f1[j] = (lv[j] && c[j].w != FGI_NONE) ? head_bits(p, s, c[j].w, sum) : 0u;
        }
        // the next run's entries are requested before this run's probes are consumed
        uint4 cn[kCPL];
#pragma unroll
        for (int j = 0; j < (int)kCPL; ++j) {
            const uint32_t i = base + kCandBatch + j * 64 + lane;
            cn[j] = load_cand(src + seg + i, i < cnt, (uint32_t)s_lo);
        }
#pragma unroll
        for (int j = 0; j < (int)kCPL; ++j) {
            const uint32_t i = base + j * 64 + lane;
            const uint32_t d = c[j].x, h0 = c[j].z, h1 = c[j].w, aux = c[j].y;
            const bool b0 = lv[j] && ((f0[j] >> (h0 & 31)) & 1u);
            const bool b1 = lv[j] && h1 != FGI_NONE && ((f1[j] >> (h1 & 31)) & 1u);
            const bool hit = b0 || b1;
            const bool tail = lv[j] && !hit && (aux >> 31);
            const bool surv = lv[j] && !hit && !tail;
            live += lv[j] ? 1u : 0u;
            examined += (lv[j] ? 1u : 0u) + ((lv[j] && h1 != FGI_NONE && !b0) ? 1u : 0u);
            bool win = false;
            if (hit) {
                const uint32_t rel = d - (uint32_t)s_lo;
                const uint32_t bit = 1u << (d & 31);
                win = (s.cs[rel >> 5] & bit) != 0;
                if (win) {   // a winner's visit bit is folded in from wm at the write-back
                    atomicOr(&s.wm[rel >> 5], bit);
                    const uint32_t rl = aux & 0x7FFFFFFFu;
                    ++ws.w;
                    ws.e += rl ? 1u : 0u;
                    ws.l += rl;
                } else {
                    atomicOr(&s.vm[rel >> 5], bit);
                    flagged += first_visit(node[d]) == 2 ? 1u : 0u;
                }
            }
            const bool xw = win && (aux & 0x7FFFFFFFu);
            const unsigned long long xm = __ballot(xw);
            if (xm) {
                uint32_t xb = 0;
                if (lane == 0) xb = atomicAdd(&s.wn, (uint32_t)__popcll(xm));
                xb = from_lane0(xb);
                if (xw) wl_out[xb + rank_in(xm)] = d;
            }
            const unsigned long long tm = __ballot(tail);
            if (tail) wq[qn + rank_in(tm)] = i;
            qn += (uint32_t)__popcll(tm);
            const unsigned long long sm = __ballot(surv);
            if (sm) {
                uint32_t sb = 0;
                if (lane == 0) sb = atomicAdd(&s.sn, (uint32_t)__popcll(sm));
                sb = from_lane0(sb);
                if (surv) sv_out[sb + rank_in(sm)] = c[j];
            }
        }
        // scan the queued tails when the queue could overflow next batch, or at the wave's end
        if (base + kCandBatch >= cnt) PROBE(L, 7);
        if (qn > kWaveTailCap - kWaveBatch || base + kCandBatch >= cnt) {
            __builtin_amdgcn_wave_barrier();
            pull_tails(p, src, sv_out, node, s_lo, seg, wq, qn, s, flagged, examined_tail, tails, ws,
                       sum);
            __builtin_amdgcn_wave_barrier();
            qn = 0;
        }
#pragma unroll
        for (int j = 0; j < (int)kCPL; ++j) c[j] = cn[j];
    }
    PROBE(L, 2);
    __syncthreads();
    PROBE(L, 3);
    // write back the owned words (visits before this level | this level's)
    unsigned long long* vis64 = reinterpret_cast<unsigned long long*>(vis);
    unsigned long long* inv64 = reinterpret_cast<unsigned long long*>(p.inv_bm);
    for (uint32_t i = threadIdx.x; i < wp.tpb * kTileWords; i += blockDim.x) {
        const uint64_t sl = s_lo + (uint64_t)i * 64;
        if (sl < p.n_slots) {
            const unsigned long long wm = s.wm[2 * i] | ((unsigned long long)s.wm[2 * i + 1] << 32);
            vis64[sl >> 6] = wm | s.vm[2 * i] | ((unsigned long long)s.vm[2 * i + 1] << 32);
            // returnless: the word's earlier bits need not be read back (nothing in this launch reads it)
            if (wm) __hip_atomic_fetch_or(inv64 + (sl >> 6), wm, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
    }
    bs[0] = ws.w;
    bs[1] = ws.e;
    bs[2] = ws.l;
    if (threadIdx.x == 0) p.sv_cnt[dst][b] = s.sn;
    // the tail probes, flag counts, live and head probes are per lane; the winners are the per-thread
    // sums (bs[0]); the scanned count is the block's list length
    const uint32_t v[kStats] = {0, flagged, threadIdx.x == 0 ? s.sn : 0u, examined_tail + examined,
                                live, (uint32_t)bs[0], tails, threadIdx.x == 0 ? cnt : 0u};
    block_stats_add(blk, s_st, v);
}

// The last block of a pull level: prefixes of the per-block (winners, expandable winners, row
// lengths) for a possible collect, and level L+1's frontier totals.
__device__ __forceinline__ void pull_epilogue(int L, const PullArgs& p, LevelCtr* ln, unsigned long long* done,
                                              const unsigned long long (&bs)[3], unsigned long long* s_red,
                                              unsigned long long* cur = nullptr) {
    __shared__ unsigned long long s_tot[3];
    const uint64_t G = gridDim.x;
    // per-thread partial sums -> the block's sums, one packed word: a block owns at most
    // kMaxIter * kPullTile = 32,768 slots (winners < 2^16) and its winners' rows hold < 2^32 edges
    static_assert(kMaxIter * kPullTile < 65536, "pull block sums pack into 16 bits");
    const unsigned long long b0 = block_sum(bs[0], s_red), b1 = block_sum(bs[1], s_red), b2 = block_sum(bs[2], s_red);
    if (threadIdx.x == 0) coh_xchg(p.bsum + blockIdx.x, pack3(b0, b1, b2));
    PROBE(L, 5);
    if (!last_block(done, gridDim.x)) {
        PROBE(L, 6);
        return;
    }
    prefix_columns(p.bsum, p.bsum + 3 * G, G, s_tot);
    __syncthreads();
    if (threadIdx.x == 0) {
        ln->w = s_tot[0];
        ln->F = s_tot[1];
        ln->T = s_tot[2];
        if (cur) *cur = (unsigned long long)L + 1;   // a fused wave's next level (every block has finished)
    }
    PROBE(L, 6);
}

// One level's traversal: push (expand) or pull, as decided for the level on the device.
// Larg >= 0: level Larg (run_wave's level groups, the partitioned wave). Larg < 0: a fused wave's
// launch with mid index -1 - Larg (mid_level): it runs its level if that level pulls or pushes more
// than big_push edges (the fused tail kernel runs the smaller push levels), adds the level to the
// wave's device-side totals and, from its last block, advances the wave's current level. The
// frontier buffers alternate with the level's parity: x / o serve even levels, x1 / o1 odd ones.
template <bool PART>
__global__ __launch_bounds__(kBlock, kLevelOcc) void k_level(int Larg, WaveParams wp, ExpandArgs x, ExpandArgs x1, PullArgs p,
                                                  const unsigned long long* node, uint32_t* vis, Out o, Out o1, WaveCtr* ctr,
                                                  unsigned long long* blk, unsigned long long* done, RemoteArgs ra,
                                                  uint64_t big_push) {
    // push: the chunk map (s_rel, s_base), then the chunk's winners over it; pull: queue + buffers
    __shared__ __align__(16) uint32_t s_x[kLevelLds];
    uint32_t* s_rel = s_x;                    // [kChunk + 1]
    uint32_t* s_base = s_x + kChunk + 4;      // [kChunk + 2], 16-byte aligned
    __shared__ Emit em;
    MsgEmit<PART>& me = *reinterpret_cast<MsgEmit<PART>*>(s_x + kPushLds);   // push levels only
    __shared__ unsigned long long s_st[kBlock / 64][kStats];
    __shared__ unsigned long long s_red[kBlock / 64];
    static_assert(sizeof(PullLds) <= (kLevelLds - kTailCap - 4) * 4, "pull LDS");
    static_assert(kPushLds % 2 == 0 && (kPushLds + sizeof(MsgEmit<true>) / 4) <= kLevelLds, "push LDS");
    const bool fused = FGI_VARIANTS && !PART && Larg < 0;
    const int L = mid_level(ctr, Larg);
    if (L < 0) return;
    if (fused && (L & 1)) {
        x = x1;
        o = o1;
    }
    PROBE(L, 0);
    LevelCtr& lc = ctr->lvl[L % kRing];
    o.ln = &ctr->lvl[(L + 1) % kRing];
    if (fused && lvl_F(lc) == 0) return;   // the wave is done: the tail kernel runs the final count
    const bool pull = level_pulls(ctr, L, wp);
    if (fused && !pull && lvl_T(lc) <= big_push) return;   // the tail kernel's
    if (blockIdx.x == 0 && threadIdx.x < sizeof(LevelCtr) / 8)
        reinterpret_cast<unsigned long long*>(&ctr->lvl[(L + 2) % kRing])[threadIdx.x] = 0ull;
    const uint64_t npull = lc.npull;
    if (blockIdx.x == 0 && threadIdx.x == 0) {
        if (!PART) {
            lc.pull = pull ? 1ull : 0ull;
            WaveParams wr = wp;   // what the automatic choice would be (the next wave's launch plan)
            wr.direction = 0;
            lc.want = (wp.direction == 0 ? pull : level_pulls(ctr, L, wr)) ? 1ull : 0ull;
        }
        o.ln->npull = npull + (pull ? 1 : 0);
        if (fused) {
            ctr->n_levels += 1;
            ctr->e_trav += lvl_T(lc);
            ctr->f_total += lvl_F(lc);
            ctr->n_pull += pull ? 1 : 0;
            ctr->n_mid += 1;
            ctr->mid_kind[(-1 - Larg) % kMidMax] = pull ? 2 : 1;
            if (!pull) {
                ctr->mid_push_edges += lvl_T(lc);
                ctr->mid_push_f += lvl_F(lc);
            }
        }
    }
    // multi-GPU pull levels run on every rank (parents may be remote); otherwise no frontier, no work
    if (pull) {
        unsigned long long bs[3] = {0, 0, 0};
        const bool sum = FGI_VARIANTS && p.sum != nullptr && lc.sum != 0;
        pull_level(L, p, wp, npull, sum, node, vis, s_rel, *reinterpret_cast<PullLds*>(s_x + kTailCap + 4), blk, s_st, bs);
        PROBE(L, 4);
        pull_epilogue(L, p, o.ln, done, bs, s_red, fused ? &ctr->cur : nullptr);
        return;
    }
    const uint64_t F = lvl_F(lc), T = lvl_T(lc);
    if (F == 0) return;
    const uint32_t mult = level_mult(T, gridDim.x);
    if (blockIdx.x == 0 && threadIdx.x == 0) lc.mult = mult;
    // blocks without a chunk leave at once and are not counted (a small level costs its chunks only)
    const uint64_t nch = ((T + kFine - 1) / kFine + mult - 1) / mult;
    const uint64_t active = nch < gridDim.x ? nch : gridDim.x;
    if (blockIdx.x >= active) return;
    emit_init(em);
    PROBE(L, 1);
    expand_level<PART>(L, F, T, mult, x, node, vis, o, em, s_x, me, s_rel, s_base, blk, s_st, ra);
    PROBE(L, 2);
    if constexpr (PART) publish_ft(o.ln, done, active);   // the host all-reduces F / T
    else if (fused && last_block(done, active) && threadIdx.x == 0) ctr->cur = (unsigned long long)L + 1;
    PROBE(L, 3);
}

// multi-GPU: apply the targets other ranks forwarded (their versions were checked by the sender)
// C > 0 (planned waves): recv holds n / (C - 1) buckets of C words, a count then up to C - 1 ids, and
// entry i is id i % (C - 1) of bucket i / (C - 1), if within its count.
__global__ __launch_bounds__(kBlock) void k_apply_recv(int L, uint64_t n, const uint32_t* __restrict__ recv, uint32_t base,
                                                       const unsigned long long* node, uint32_t* vis, Out o,
                                                       WaveCtr* ctr, unsigned long long* blk, unsigned long long* done,
                                                       uint32_t C) {
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
        bool in = i < n;
        uint64_t at = i;
        if (C && in) {
            const uint64_t q = i / (C - 1), j = i % (C - 1);
            in = j < recv[q * C];
            at = q * C + 1 + j;
        }
        if (in) {
            h = recv[at] - base;
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
    publish_ft(o.ln, done, gridDim.x);
}

// Planned multi-GPU waves: one block per owner q moves the next ids it forwarded to q (send_buf slice
// q, cumulative over the wave: each target at most once, sent_bm) into bucket q of the fixed-size
// all-to-all: the count, then up to C - 1 ids; the rest waits for the next push level's pack.
__global__ __launch_bounds__(kBlock) void k_a2a_pack(uint32_t R, uint32_t C, const uint32_t* __restrict__ send_buf,
                                                     uint32_t block, const unsigned long long* send_cnt,
                                                     unsigned long long* cur, uint32_t* a2a_send) {
    const uint32_t q = blockIdx.x;
    const unsigned long long c0 = cur[q], tot = send_cnt[q];
    const uint32_t n = q == R ? 0u : (uint32_t)std::min<unsigned long long>(tot - c0, (unsigned long long)(C - 1));
    uint32_t* dst = a2a_send + (uint64_t)q * C;
    for (uint32_t i = threadIdx.x; i < n; i += blockDim.x) dst[1 + i] = send_buf[(uint64_t)q * block + c0 + i];
    if (threadIdx.x == 0) {
        dst[0] = n;
        cur[q] = c0 + n;
    }
}

// The planned wave's closing all-reduce: red[0] the next level's local frontier, red[1] the forwarded
// ids still waiting in send_buf, red[2 + 2l .. + 1] level L0 + l's local {F, T}, l < K (the next
// wave's plan).
__global__ void k_part_tail(const WaveCtr* ctr, int L0, int L, uint32_t W, const unsigned long long* send_cnt,
                            const unsigned long long* cur, unsigned long long* red, int K) {
    if (threadIdx.x != 0) return;
    red[0] = lvl_F(ctr->lvl[L % kRing]);
    unsigned long long pend = 0;
    for (uint32_t q = 0; q < W; ++q) pend += send_cnt[q] - cur[q];
    red[1] = pend;
    for (int l = 0; l < K; ++l) {
        red[2 + 2 * l] = lvl_F(ctr->lvl[(L0 + l) % kRing]);
        red[3 + 2 * l] = lvl_T(ctr->lvl[(L0 + l) % kRing]);
    }
}

// ---- final collect: the invalidated bitmap -> the invalidated list -----------------------------
// Two launches, no inter-block waiting (a cooperative launch costs ~11 us of dispatch gap on this
// stack, a ticket counter serialises ~1,000 atomics on one word): k_final_count — block t counts the
// set bits of its 64-bit words [t * wpb, (t + 1) * wpb) and stores the count; tickets 0..kStats-1
// also fold the per-block statistics into the wave counters (one column each, coalesced sweeps).
// k_final_write — block t adds up its predecessors' counts (all of them in one round) and writes
// every set bit's handle at that offset, in ascending order: one 1,024-handle tile per wave, 16
// handles per lane, staged in LDS and stored coalesced.
// total = 1 (bitmap mode, no k_final_write follows): the last block also sums the counts into
// ctr->inv (V_inv).
// Hub-first labels (labels.hip): the bitmap over boundary handles of fold tile t
// (handles [t * kFoldTile, + kFoldTile), kFoldWords 64-bit words) is the labels' bitmap shifted by K
// (K + x is the label of every handle x that has no hot label; K is a multiple of kFoldTile), ORed with
// the tile's hot labels' bits at their slots: per hot class j, the labels [fold_start[t][j],
// fold_start[t + 1][j]), which keep slot order. Written to f.xbm; returns the tile's set bits (every
// thread). Block-uniform call; s_w: kFoldWords words, s_a / s_o: kMaxHotClasses + 1 words of LDS.
constexpr uint32_t kFoldStage = 12288;   // a fold tile's slot offsets staged in LDS (24 KB; ~8,200 per tile at configs[2])

__device__ unsigned long long fold_tile(const FoldArgs& f, const unsigned long long* __restrict__ inv64, uint64_t ext_words,
                                        uint32_t t, unsigned long long* s_w, uint32_t* s_a, uint32_t* s_o,
                                        unsigned long long* s_red) {
    const uint64_t w0 = (uint64_t)t * kFoldWords;
    const uint32_t nw = (uint32_t)std::min<uint64_t>(kFoldWords, ext_words > w0 ? ext_words - w0 : 0);
    const uint64_t kw = f.K / 64;
    __shared__ uint32_t s_wt[2][kBlock / 64];
    __shared__ uint32_t s_i[kMaxHotClasses + 1];
    __shared__ __align__(16) uint16_t s_off[kFoldStage];
    __shared__ uint32_t s_eb[kFoldStage / 32 + 2];   // the staged entries' bits, in entry order
    const bool hot = f.l2s && f.ncls && !(f.exp & 1);
    for (uint32_t i = threadIdx.x; i < kFoldStage / 32 + 2; i += blockDim.x) s_eb[i] = 0u;
    // every independent load first — the tile's run bounds, its classes' runs, the cold words, the slot
    // offsets — then the LDS stores: a block's fold is a chain of round trips, so fewer links
    const uint32_t b0 = hot ? f.base[t] : 0u, b1 = hot ? f.base[t + 1] : 0u;
    uint32_t len = 0, a = 0;
    if (hot && threadIdx.x < f.ncls) {
        const uint32_t* fs = f.fold_start + (uint64_t)t * f.ncls + threadIdx.x;   // rows t and t + 1
        a = fs[0];
        len = fs[f.ncls] - a;
    }
    constexpr uint32_t kU = kFoldWords / kBlock;
    static_assert(kFoldWords % kBlock == 0, "fold tile words per thread");
    unsigned long long cw[kU];
#pragma unroll
    for (uint32_t u = 0; u < kU; ++u) {
        const uint32_t i = u * kBlock + threadIdx.x;
        cw[u] = i < nw && !(f.exp & 2) ? inv64[kw + w0 + i] : 0ull;
    }
    // the tile's slot offsets (fold_off: labels.hip k_lbl_fold_off, the same order, 2 bytes each; a tile's
    // run starts 16-byte aligned and is padded to 8 entries) staged in LDS by 16-byte loads; a tile with
    // more than kFoldStage reads the rest from memory
    const uint16_t* toff = f.off + b0;
    constexpr uint32_t kV = (kFoldStage / 8 + kBlock - 1) / kBlock;
    const uint32_t n16 = (f.exp & 8) ? 0u : min(b1 - b0, kFoldStage) / 8;
    uint4 v[kV];
#pragma unroll
    for (uint32_t u = 0; u < kV; ++u) {
        const uint32_t i = u * kBlock + threadIdx.x;
        if (i < n16) v[u] = reinterpret_cast<const uint4*>(toff)[i];
    }
#pragma unroll
    for (uint32_t u = 0; u < kU; ++u) s_w[u * kBlock + threadIdx.x] = cw[u];
#pragma unroll
    for (uint32_t u = 0; u < kV; ++u) {
        const uint32_t i = u * kBlock + threadIdx.x;
        if (i < n16) reinterpret_cast<uint4*>(s_off)[i] = v[u];
    }
    if (hot) {
        // this tile's run of each hot class, cut into chunks of up to 64 labels (one 64-bit window of the
        // hot bitmap each): per class its first label (s_a), its first entry in the tile's fold_off run
        // (s_o) and its first chunk (s_i), by one block scan over the classes
        const uint32_t nch = (len + 63) >> 6;
        uint32_t tot_l, tot_c;
        const uint32_t ex_l = wave_excl_scan(len, tot_l);
        const uint32_t ex_c = wave_excl_scan(nch, tot_c);
        const uint32_t wid = threadIdx.x >> 6;
        if (lane_id() == 0) {
            s_wt[0][wid] = tot_l;
            s_wt[1][wid] = tot_c;
        }
        __syncthreads();
        uint32_t before_l = 0, before_c = 0, labels = 0, chunks = 0;
        for (uint32_t k = 0; k < blockDim.x / 64; ++k) {
            before_l += k < wid ? s_wt[0][k] : 0u;
            before_c += k < wid ? s_wt[1][k] : 0u;
            labels += s_wt[0][k];
            chunks += s_wt[1][k];
        }
        if (threadIdx.x < f.ncls) {
            s_a[threadIdx.x] = a;
            s_o[threadIdx.x] = before_l + ex_l;
            s_i[threadIdx.x] = before_c + ex_c;
        }
        if (threadIdx.x == 0) {
            s_o[f.ncls] = labels;
            s_i[f.ncls] = chunks;
        }
        __syncthreads();
        // one chunk per thread: its class by a search over the chunk offsets, its labels' bits as one
        // 64-bit window of the hot bitmap (two words at most), then per set bit its slot's offset (LDS)
        // and the bit in the tile's words (LDS)
        const uint32_t staged = n16 * 8;   // entries [0, staged) are in LDS
        // per chunk (one per thread): its class by a search over the chunk offsets, its labels' bits as
        // one 64-bit window of the hot bitmap (two words at most), copied into the tile's entry-order
        // bitmap s_eb at its first entry (LDS); a chunk past the staged entries folds its bits itself
        uint32_t* s_w32 = reinterpret_cast<uint32_t*>(s_w);   // 32-bit LDS atomics (little endian)
        for (uint32_t q = threadIdx.x; q < ((f.exp & 4) ? 0u : chunks); q += blockDim.x) {
            uint32_t lo = 0;   // the last class j with s_i[j] <= q
#pragma unroll
            for (uint32_t step = kMaxHotClasses / 2; step; step >>= 1) {
                const uint32_t j = lo + step;
                if (j < f.ncls && s_i[j] <= q) lo = j;
            }
            const uint32_t c0 = (q - s_i[lo]) << 6;      // the chunk's first label in its class's run
            const uint32_t lab0 = s_a[lo] + c0;
            const uint32_t e0 = s_o[lo] + c0;            // its first entry in the tile's offsets
            const uint32_t m = min(64u, s_o[lo + 1] - s_o[lo] - c0);
            const uint32_t wq = lab0 >> 6, sh = lab0 & 63;
            unsigned long long bits = inv64[wq] >> sh;
            if (sh && sh + m > 64) bits |= inv64[wq + 1] << (64 - sh);
            if (m < 64) bits &= (1ull << m) - 1ull;
            if (!bits) continue;
            if (e0 + m <= staged) {
                const uint32_t w = e0 >> 5, b = e0 & 31;
                const uint32_t v0 = (uint32_t)bits, v1 = (uint32_t)(bits >> 32);
                if (v0) {
                    atomicOr(&s_eb[w], v0 << b);
                    if (b) atomicOr(&s_eb[w + 1], v0 >> (32 - b));
                }
                if (v1) {
                    atomicOr(&s_eb[w + 1], v1 << b);
                    if (b) atomicOr(&s_eb[w + 2], v1 >> (32 - b));
                }
                continue;
            }
            for (; bits; bits &= bits - 1) {   // past the LDS stage (rare: > kFoldStage hot labels in a tile)
                const uint32_t e = e0 + (uint32_t)(__ffsll((long long)bits) - 1);
                const uint32_t x = e < staged ? s_off[e] : toff[e];   // < kFoldTile
                atomicOr(&s_w32[x >> 5], 1u << (x & 31));
            }
        }
        __syncthreads();
        // one staged entry per lane: its bit from s_eb, its slot's offset from s_off, the bit in the tile's
        // words — no search, no divergence
        const uint32_t ne = min(labels, staged);
        for (uint32_t k0 = 0; k0 < ne; k0 += 4 * blockDim.x) {   // block-uniform
            uint32_t x[4];
#pragma unroll
            for (int u = 0; u < 4; ++u) {
                const uint32_t k = k0 + u * blockDim.x + threadIdx.x;
                x[u] = (k < ne && ((s_eb[k >> 5] >> (k & 31)) & 1u)) ? (uint32_t)s_off[k] : FGI_NONE;
            }
#pragma unroll
            for (int u = 0; u < 4; ++u)
                if (x[u] != FGI_NONE) atomicOr(&s_w32[x[u] >> 5], 1u << (x[u] & 31));
        }
    }
    __syncthreads();
    unsigned long long c = 0;
    for (uint32_t i = threadIdx.x; i < nw; i += blockDim.x) {
        const unsigned long long v = s_w[i];
        c += (unsigned long long)__popcll(v);
        f.xbm[w0 + i] = v;
    }
    c = block_sum(c, s_red);
    __syncthreads();   // s_w, s_a, s_o are reused by the block's next tile
    return c;
}

constexpr uint32_t kFoldBlocks = 4096;   // k_final_count's grid with hot labels: one fold tile per block up to 2^28 handles

// The final count: tickets 0..kStats-1 fold the per-block statistics into the wave counters; every
// block counts the set bits of its 64-bit words [t * wpb, (t + 1) * wpb) into status[t]. With hot labels
// (f.xbm), block t is fold tile t instead: it writes the tile's bitmap over boundary handles into xbm
// and counts that.
__global__ __launch_bounds__(kBlock) void k_final_count(const unsigned long long* __restrict__ inv64, uint64_t words,
                                                        uint64_t wpb, unsigned long long* status, WaveCtr* ctr,
                                                        const unsigned long long* __restrict__ blk, int total,
                                                        unsigned long long* done, FoldArgs f) {
    __shared__ unsigned long long s_red[kBlock / 64];
    const uint32_t t = blockIdx.x;
    if (t < (uint32_t)kStats) {
        const int k = t;
        unsigned long long* dst[kStats] = {&ctr->e_match,   &ctr->n_flagged, &ctr->pull_surv, &ctr->pull_edges,
                                           &ctr->pull_live, &ctr->pull_win,  &ctr->pull_tail, &ctr->pull_scan};
        const unsigned long long* col = blk + (uint64_t)k * kStatBlocks;
        unsigned long long x = 0;
#pragma unroll
        for (uint32_t q = 0; q < kStatBlocks / kBlock; ++q) x += col[q * kBlock + threadIdx.x];
        x = block_sum(x, s_red);
        if (threadIdx.x == 0) *dst[k] = x + (k == kStFlagged ? ctr->root_flagged : 0ull);
    }
    unsigned long long c = 0;
    if (f.xbm) {
        // fold tiles t, t + G, ...: one status word per tile (k_final_write's spb groups); one tile per
        // block up to kFoldBlocks tiles
        __shared__ unsigned long long s_w[kFoldWords];
        __shared__ uint32_t s_a[kMaxHotClasses + 1], s_o[kMaxHotClasses + 1];
        for (uint32_t tt = t; (uint64_t)tt * kFoldWords < words; tt += gridDim.x) {   // block-uniform
            const unsigned long long ct = fold_tile(f, inv64, words, tt, s_w, s_a, s_o, s_red);
            if (!total) {
                if (threadIdx.x == 0) status[tt] = ct;
            } else {
                c += ct;
            }
        }
        if (!total) return;
    } else {
        const uint64_t lo = t * wpb, hi = std::min<uint64_t>(words, lo + wpb);
        for (uint64_t w = lo + threadIdx.x; w < hi; w += blockDim.x) c += (unsigned long long)__popcll(inv64[w]);
        c = block_sum(c, s_red);
    }
    if (!total) {
        if (threadIdx.x == 0) status[t] = c;
        return;
    }
    if (threadIdx.x == 0) coh_xchg(status + t, c);
    if (!last_block(done, gridDim.x)) return;
    unsigned long long all = 0;
    for (uint32_t k = threadIdx.x; k < gridDim.x; k += blockDim.x) all += coh_read(status + k);
    all = block_sum(all, s_red);
    if (threadIdx.x == 0) ctr->inv = all;
}

// The list: block t writes the set bits of its words [t * wpb, + wpb) of inv64 (the boundary's bitmap:
// the labels' own, or xbm) in ascending order, after the sum of the counts of the status entries
// before its own (spb entries per block: 1, or its fold tiles).
// With pub (a synchronous wave's list, run_wave): the last block to finish also publishes the wave's
// counters to fine-grained host memory and then the sequence word (k_publish's protocol, one launch
// fewer). The asynchronous waves keep k_publish: their ids are read by other streams after the wait, so
// the word must follow the whole kernel.
struct ListPub {
    unsigned long long* dst;   // null: no publish
    unsigned long long seq;
    unsigned long long* done;
    uint32_t words;
};

// With end.ctr (a level group's list, run_wave): once the wave is over (wave_over), every block also
// zeroes its share of the invalidated bitmap (its own words, after reading them, when it lists that
// bitmap; hot labels: k_final_count has read it) and of the statistics rows, and with end.spare its share
// of the swapped-out visit bitmap, so that the next wave needs no init kernel.
__global__ __launch_bounds__(kBlock) void k_final_write(const unsigned long long* __restrict__ inv64, uint64_t words,
                                                        uint64_t wpb, const unsigned long long* __restrict__ status,
                                                        WaveCtr* ctr, uint32_t* out, int need_done, uint32_t spb,
                                                        ListPub pub, WaveEnd end) {
    if (need_done && ctr->phase != kPhaseDone) return;   // a fused wave whose tail stopped early: not yet
    __shared__ unsigned long long s_red[kBlock / 64];
    __shared__ unsigned long long s_wbase[kBlock / 64];
    __shared__ uint32_t s_stage[kBlock / 64][kPullTile];
    const uint32_t t = blockIdx.x;
    const uint32_t lane = lane_id(), wid = threadIdx.x >> 6;
    constexpr uint32_t W = kBlock / 64;
    // each wave owns a contiguous run of the block's words: counted first, then written with a
    // wave-local running offset (no block barrier per tile)
    const uint64_t lo = t * wpb, hi = std::min<uint64_t>(words, lo + wpb);
    const uint64_t ww = (wpb + W - 1) / W;
    const uint64_t wlo = std::min<uint64_t>(hi, lo + wid * ww), whi = std::min<uint64_t>(hi, wlo + ww);
    unsigned long long part = 0;
    for (uint64_t k = threadIdx.x; k < (uint64_t)t * spb; k += blockDim.x) part += status[k];
    uint32_t wc = 0;
    for (uint64_t x = wlo + lane; x < whi; x += 64) wc += (uint32_t)__popcll(inv64[x]);
#pragma unroll
    for (int d = 32; d >= 1; d >>= 1) wc += __shfl_xor(wc, d, 64);
    const unsigned long long excl = block_sum(part, s_red);   // its barriers also publish s_wbase below
    if (lane == 0) s_wbase[wid] = wc;
    __syncthreads();
    unsigned long long run = excl;
    for (uint32_t k = 0; k < wid; ++k) run += s_wbase[k];
    if (t == gridDim.x - 1 && threadIdx.x == blockDim.x - 1) ctr->inv = run + wc;
    const uint16_t* bits16 = reinterpret_cast<const uint16_t*>(inv64);
    // tiles of 16 words per wave, 16 handles per lane
    for (uint64_t tw = wlo; tw < whi; tw += kTileWords) {   // wave-uniform
        const uint64_t q = tw * 4 + lane;                    // the lane's 16-bit chunk
        const uint32_t m = (tw + lane / 4 >= whi) ? 0u : (uint32_t)bits16[q];
        uint32_t tot;
        const uint32_t ex = wave_excl_scan((uint32_t)__popc(m), tot);
        uint32_t o = ex;
        for (uint32_t mm = m; mm; mm &= mm - 1) s_stage[wid][o++] = (uint32_t)(q * 16 + (uint32_t)(__ffs(mm) - 1));
        __builtin_amdgcn_wave_barrier();
        for (uint32_t i = lane; i < tot; i += 64) out[run + i] = s_stage[wid][i];
        __builtin_amdgcn_wave_barrier();
        run += tot;
    }
    if (end.ctr) {   // block-uniform
        const bool over = wave_over(end);
        __syncthreads();   // the block's waves have read their words
        // the block's share of the labels' bitmap: its own read range when it lists that bitmap (the
        // partition is the launch's: ceil(words / grid) per block)
        const uint64_t P = (end.words + gridDim.x - 1) / gridDim.x;
        const uint64_t z0 = min(end.words, (uint64_t)t * P), z1 = min(end.words, z0 + P);
        unsigned long long* iw = reinterpret_cast<unsigned long long*>(end.inv_bm);
        unsigned long long* sw = reinterpret_cast<unsigned long long*>(end.spare);
        for (uint64_t x = z0 + threadIdx.x; x < z1; x += blockDim.x) {
            if (over) iw[x] = 0ull;
            if (sw) sw[x] = 0ull;
        }
        if (over) {
            constexpr uint64_t kBlk = (uint64_t)kStatBlocks * kStatCols;
            const uint64_t Q = (kBlk + gridDim.x - 1) / gridDim.x;
            const uint64_t b0 = min(kBlk, (uint64_t)t * Q), b1 = min(kBlk, b0 + Q);
            for (uint64_t x = b0 + threadIdx.x; x < b1; x += blockDim.x) end.blk[x] = 0ull;
        }
    }
    if (pub.dst && last_block_arrive<true>(pub.done, gridDim.x)) {
        if (threadIdx.x == 0) pub.dst[pub.words + 1] = wall_clock64();
        unsigned long long* src = reinterpret_cast<unsigned long long*>(ctr);
        for (uint32_t i = threadIdx.x; i < pub.words; i += blockDim.x) pub.dst[i] = coh_read(src + i);
        __threadfence_system();
        __syncthreads();
        if (threadIdx.x == 0) __hip_atomic_store(pub.dst + pub.words, pub.seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
    }
}

constexpr uint32_t kFinalStage = 1024;   // bitmap words a block keeps in LDS (8 KB), k_wave_coop

// ---- a whole (push-only) wave in one launch ---------------------------------------------------
// Streaming batches (fgi_run_batch) queue mutation steps and waves back to back and synchronise once
// at the end, so their waves cannot come back to the host between levels. A cooperative grid (every
// block resident) runs the roots (immediate ones first), every level and the final collect, with a
// grid barrier where run_wave has a kernel boundary. The root count may be read from the device
// (roots produced by an earlier step). The invalidated handles are appended at out[*out_n ..) in
// ascending order and *out_n advanced; acc accumulates the batch's totals.
enum : int { kAccWaves, kAccLevels, kAccInv, kAccETrav, kAccEMatch, kAccFlagged, kAccFTotal, kAccBarrier, kAccN };
static_assert(kAccN <= kAccCount && kAccBarrier == kAccBarrierIdx, "batch accumulators");

struct CoopArgs {
    const uint32_t* roots;
    const uint8_t* imm;
    uint32_t n_max;
    const unsigned long long* n_dev;   // nullable: n_max roots
    unsigned long long* node;
    uint32_t* vis;
    uint32_t* inv_bm;
    const uint64_t* row_off;
    const uint32_t* row_len;
    uint32_t* fr_off[2];
    uint32_t* fr_len[2];
    uint64_t* escan[2];
    uint32_t* cstart[2];
    const uint32_t* pool_col;
    const uint64_t* pool_tag;
    int dead_filter;
    uint32_t n_handles;
    WaveCtr* ctr;
    unsigned long long* blk;
    unsigned long long* cnt;           // [grid] final collect counts
    uint32_t* out;
    unsigned long long* out_n;
    unsigned long long* acc;           // [kAccN]
    const unsigned long long* abort;   // nullable: a batch's abort word (set: the wave does nothing)
    unsigned long long* abort_w;       // the same word, set (kAbortBarrier) when a grid barrier times out
    uint64_t bar_timeout;              // grid barrier timeout, 100 MHz ticks
    uint32_t fault_block;              // fault injection: block fault_block - 1 skips its first barrier
    int bar_mode;                      // soft_grid_sync's memory ordering (FGI_BAR_MODE)
    unsigned long long* gbar;          // plain launch: the grid barrier's arrival counter (monotonic)
    int one_round;                     // chunk size by level_mult_one_round (FGI_COOP_CHUNKS=0: level_mult)
    FoldArgs fold;                     // hot labels: the ids come from the folded bitmap (fold_tile)
    uint64_t ext_words;                // words of the bitmap over boundary handles
};

// Grid barrier of a plain (non-cooperative) launch of k_wave_coop. A cooperative launch goes to the
// runtime's cooperative queue: ~11.7 us of dispatch gap before each, where plain launches follow
// each other within 0.1 us (profiles/r6n_stream_kernels.txt), and a streaming round makes six of
// them, four with no roots. The grid is one block per two CUs, far below what the chip holds
// resident, so every block runs at once without the cooperative guarantee. As the device library's
// barrier: agent-scope fences on both sides; one thread per block arrives on a monotonic counter and
// waits for the next multiple of the grid size.
// Failure is defined, never a hang or a half-synchronised grid: a wait longer than the timeout (2 s
// of the 100 MHz wall clock) marks the grid broken (acc[kAccBarrier]) and sets the batch's abort word
// (kAbortBarrier: the batch's later kernels and cascades do nothing); a block waiting at a barrier
// leaves as soon as it sees the broken mark. Returns false in every block that did not see the
// barrier complete: the caller returns at once, writing nothing more. A block that did see it
// complete went on with complete data; it leaves at its next barrier. fgi_run_batch then fails with
// FGI_EDEVICE and poisons the graph until fgi_restore (graph.hip).
// skip (fault injection, FGI_OPT_FAULT_INJECT): this block leaves without arriving, as a block that
// is never resident would never arrive.
// mode (measurement, FGI_BAR_MODE): 0 every thread fences (agent scope, seq_cst) on both sides; 1 the
// block's stores are ordered by its block barrier and one wave (thread 0) makes them visible with an
// agent-scope release fence before it arrives and an acquire fence after its wait (the L2 write-back
// and invalidate are per XCD and the L1 per CU, so one wave's fences serve the block).
constexpr uint64_t kGridBarTimeout = 200000000ull;
__device__ __forceinline__ bool soft_grid_sync(unsigned long long* cnt, unsigned long long* broken,
                                               unsigned long long* abort_w, uint64_t timeout, bool skip, int mode = 0) {
    __shared__ int s_ok;
    if (skip) return false;   // block-uniform
    if (mode == 0) __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "agent");
    __syncthreads();
    if (threadIdx.x == 0) {
        if (mode != 0) __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
        const unsigned long long arrived = __hip_atomic_fetch_add(cnt, 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        const unsigned long long target = (arrived / gridDim.x + 1) * gridDim.x;
        const uint64_t t0 = wall_clock64();
        int ok = 1;
        while (__hip_atomic_load(cnt, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < target) {
            if (__hip_atomic_load(broken, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0) {
                ok = 0;
                break;
            }
            __builtin_amdgcn_s_sleep(1);
            if (wall_clock64() - t0 > timeout) {
                __hip_atomic_store(broken, 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                if (abort_w) atomicCAS(abort_w, 0ull, kAbortBarrier << 32);
                ok = 0;
                break;
            }
        }
        if (mode != 0) __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
        s_ok = ok;
    }
    __syncthreads();
    if (mode == 0) __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "agent");
    return s_ok != 0;
}

template <bool SOFT>
__global__ __launch_bounds__(kBlock) void k_wave_coop(CoopArgs a) {
    // false: the grid is broken (soft barrier only); the block returns at once
    int n_sync = 0;
    auto grid_sync = [&]() -> bool {
        if constexpr (SOFT) {
            const bool skip = a.fault_block != 0 && n_sync == 0 && blockIdx.x + 1 == a.fault_block;
            ++n_sync;
            return soft_grid_sync(a.gbar, a.acc + kAccBarrier, a.abort_w, a.bar_timeout, skip, a.bar_mode);
        } else {
            cooperative_groups::this_grid().sync();
            return true;
        }
    };
    __shared__ __align__(16) uint32_t s_x[kChunkEmitCap + 8];
    uint32_t* s_rel = s_x;
    uint32_t* s_base = s_x + kChunk + 4;
    __shared__ Emit em;
    __shared__ MsgEmit<false> me;
    __shared__ unsigned long long s_st[kBlock / 64][kStats];
    __shared__ unsigned long long s_red[kBlock / 64];
    __shared__ unsigned long long s_ft, s_base_out;
    __shared__ uint32_t s_w[kBlock / 64];
    __shared__ unsigned long long s_words[kFinalStage];
    // uniform across the grid: the word is written before the launch and not during it
    if (a.abort && __hip_atomic_load(a.abort, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0) return;
#if FGI_PROBE
    __shared__ uint32_t s_cp;
    if (threadIdx.x == 0 && blockIdx.x == 0) {
        s_cp = atomicAdd(&d_cprobe_n, 1u) % 64;
        for (int k = 0; k < 10; ++k) d_cprobe[s_cp][k] = 0;
    }
    __syncthreads();
#endif
    CPROBE(0);
    WaveCtr* ctr = a.ctr;
    const uint32_t n = a.n_dev ? (uint32_t)std::min<unsigned long long>(*a.n_dev, a.n_max) : a.n_max;
    if (n == 0) {   // an empty cascade (no displaced node, nothing flagged InvalidateOnSetOutput)
        if (blockIdx.x == 0 && threadIdx.x == 0) a.acc[kAccWaves] += 1;
        return;
    }
    const uint32_t gsize = gridDim.x * blockDim.x;
    const Out o0{a.row_off, a.row_len, a.inv_bm, a.fr_off[0], a.fr_len[0], a.escan[0], a.cstart[0], &ctr->lvl[0]};
    if (a.imm) {   // Invalidate(true) roots first: their CAS may change node words
        for (uint32_t i0 = blockIdx.x * blockDim.x; i0 < n; i0 += gsize)
            root_step<1>(i0 + threadIdx.x, a.roots, a.imm, n, 0u, a.n_handles, a.node, a.vis, o0, ctr);
        if (!grid_sync()) return;
    }
    for (uint32_t i0 = blockIdx.x * blockDim.x; i0 < n; i0 += gsize)
        root_step<0>(i0 + threadIdx.x, a.roots, a.imm, n, 0u, a.n_handles, a.node, a.vis, o0, ctr);
    CPROBE(1);
    uint64_t levels = 0, e_trav = 0, f_total = 0;
    for (int L = 0;; ++L) {
        if (!grid_sync()) return;   // level L's frontier (and its counter) is complete
        if (L < 4) CPROBE(2 + L);
        if (threadIdx.x == 0) s_ft = coh_read(&ctr->lvl[L % kRing].ft);
        __syncthreads();
        const uint64_t F = s_ft >> 32, T = s_ft & 0xFFFFFFFFull;
        if (blockIdx.x == 0 && threadIdx.x == 0) {
            ctr->lvl[L % kRing].F = F;
            ctr->lvl[L % kRing].T = T;
        }
        // level L + 1's counter accumulates during this level; L + 2's is cleared for the next one
        if (blockIdx.x == 0 && threadIdx.x < sizeof(LevelCtr) / 8)
            reinterpret_cast<unsigned long long*>(&ctr->lvl[(L + 2) % kRing])[threadIdx.x] = 0ull;
        if (F == 0) break;
        ++levels;
        e_trav += T;
        f_total += F;
        const int buf = L & 1;
        const ExpandArgs x{a.fr_off[buf], a.escan[buf], a.cstart[buf], a.pool_col, a.pool_tag, a.dead_filter};
        const Out o{a.row_off, a.row_len,        a.inv_bm, a.fr_off[buf ^ 1], a.fr_len[buf ^ 1],
                    a.escan[buf ^ 1], a.cstart[buf ^ 1], &ctr->lvl[(L + 1) % kRing]};
        emit_init(em);
        const uint32_t mult = a.one_round ? level_mult_one_round(T, gridDim.x) : level_mult(T, gridDim.x);
        expand_level<false>(kProbeLevelsOff, F, T, mult, x, a.node, a.vis, o, em, s_x, me, s_rel, s_base, a.blk,
                            s_st, RemoteArgs{});
    }
    // final collect (as k_final, with a grid barrier instead of waiting on status words)
    const uint64_t words = ((uint64_t)a.n_handles + 63) / 64;
    const uint64_t wpb = (words + gridDim.x - 1) / gridDim.x;
    const uint64_t lo = std::min<uint64_t>(words, blockIdx.x * wpb), hi = std::min<uint64_t>(words, lo + wpb);
    const unsigned long long* inv64 = reinterpret_cast<const unsigned long long*>(a.inv_bm);
    if (threadIdx.x == 0) s_base_out = *a.out_n;   // advanced only after the barrier below
    if (blockIdx.x < (uint32_t)kStats) {
        const int k = blockIdx.x;
        unsigned long long* dst[kStats] = {&ctr->e_match,   &ctr->n_flagged, &ctr->pull_surv, &ctr->pull_edges,
                                           &ctr->pull_live, &ctr->pull_win,  &ctr->pull_tail, &ctr->pull_scan};
        const unsigned long long* col = a.blk + (uint64_t)k * kStatBlocks;
        unsigned long long x = 0;
        // only this grid's rows are written (the others were cleared by k_wave_init or by the previous
        // cooperative wave's own blocks): one load per thread instead of a 16-deep chain of loads
        for (uint32_t q = threadIdx.x; q < gridDim.x; q += blockDim.x) x += col[q];
        x = block_sum(x, s_red);
        if (threadIdx.x == 0) {
            const unsigned long long v = x + (k == kStFlagged ? ctr->root_flagged : 0ull);
            *dst[k] = v;
            if (k == kStEMatch) atomicAdd(a.acc + kAccEMatch, v);
            if (k == kStFlagged) atomicAdd(a.acc + kAccFlagged, v);
        }
    }
    unsigned long long c = 0;
    // hot labels: this block's fold tiles (the list is written from their bitmap over boundary handles)
    const bool folded = a.fold.xbm != nullptr;
    const uint64_t tiles = folded ? (a.ext_words + kFoldWords - 1) / kFoldWords : 0;
    const uint64_t tpb = folded ? (tiles + gridDim.x - 1) / gridDim.x : 0;
    const uint64_t f_lo = std::min<uint64_t>(a.ext_words, blockIdx.x * tpb * kFoldWords);
    const uint64_t f_hi = std::min<uint64_t>(a.ext_words, f_lo + tpb * kFoldWords);
    if (folded) {
        static_assert((kChunkEmitCap + 8) * 4 >= kFoldWords * 8, "a fold tile's words fit the coop wave's LDS");
        unsigned long long* s_fw = reinterpret_cast<unsigned long long*>(s_x);   // kFoldWords words
        __shared__ uint32_t s_fa[kMaxHotClasses + 1], s_fo[kMaxHotClasses + 1];
        for (uint64_t t = blockIdx.x * tpb; t < std::min<uint64_t>(tiles, (blockIdx.x + 1) * tpb); ++t)
            c += fold_tile(a.fold, inv64, a.ext_words, (uint32_t)t, s_fw, s_fa, s_fo, s_red);
    } else {
        for (uint64_t w = lo + threadIdx.x; w < hi; w += blockDim.x) {
            const unsigned long long v = inv64[w];
            if (w - lo < kFinalStage) s_words[w - lo] = v;
            c += (unsigned long long)__popcll(v);
        }
        c = block_sum(c, s_red);
    }
    if (threadIdx.x == 0) coh_xchg(a.cnt + blockIdx.x, c);
    CPROBE(6);
    if (!grid_sync()) return;
    CPROBE(7);
    unsigned long long part = 0;
    for (uint32_t k = threadIdx.x; k < blockIdx.x; k += blockDim.x) part += coh_read(a.cnt + k);
    const unsigned long long excl = block_sum(part, s_red);
    if (blockIdx.x == gridDim.x - 1 && threadIdx.x == 0) {
        ctr->inv = excl + c;
        *a.out_n = s_base_out + excl + c;
        a.acc[kAccWaves] += 1;
        a.acc[kAccLevels] += levels;
        a.acc[kAccInv] += excl + c;
        a.acc[kAccETrav] += e_trav;
        a.acc[kAccFTotal] += f_total;
    }
    const uint32_t lane = lane_id(), wid = threadIdx.x >> 6;
    const uint16_t* bits16 = reinterpret_cast<const uint16_t*>(folded ? a.fold.xbm : inv64);
    uint64_t run = s_base_out + excl;
    const uint64_t o_lo = folded ? f_lo : lo, o_hi = folded ? f_hi : hi;   // the words listed
    for (uint64_t w0 = o_lo; w0 < o_hi; w0 += (uint64_t)(blockDim.x >> 6) * kTileWords) {   // block-uniform
        const uint64_t tw = w0 + (uint64_t)wid * kTileWords;
        const uint64_t q = tw * 4 + lane;
        const uint64_t wl = tw - o_lo + lane / 4;
        const uint32_t m = (tw + lane / 4 >= o_hi) ? 0u
                           : (!folded && wl < kFinalStage) ? (uint32_t)(s_words[wl] >> (16 * (lane & 3))) & 0xFFFFu
                                                           : (uint32_t)bits16[q];
        uint32_t tot;
        const uint32_t ex = wave_excl_scan((uint32_t)__popc(m), tot);
        __syncthreads();
        if (lane == 0) s_w[wid] = tot;
        __syncthreads();
        uint32_t before = 0, all = 0;
        for (uint32_t k = 0; k < blockDim.x / 64; ++k) {
            if (k < wid) before += s_w[k];
            all += s_w[k];
        }
        // the chunk map's LDS is free now: one 1,024-handle tile per wave
        uint32_t* stage = s_x + wid * kPullTile;
        uint32_t o = ex;
        for (uint32_t mm = m; mm; mm &= mm - 1) stage[o++] = (uint32_t)(q * 16 + (uint32_t)(__ffs(mm) - 1));
        __builtin_amdgcn_wave_barrier();
        for (uint32_t i = lane; i < tot; i += 64) a.out[run + before + i] = stage[i];
        __builtin_amdgcn_wave_barrier();
        run += all;
    }
    // leave the state clean for the next cooperative wave (no k_wave_init, no k_fold between
    // them): this block's visits folded into the node words, its bitmap words, its statistics
    // entries and (block 0) the level counters this wave used cleared
    __syncthreads();
    CPROBE(8);
    unsigned long long* vis64 = reinterpret_cast<unsigned long long*>(a.vis);
    unsigned long long* invw = reinterpret_cast<unsigned long long*>(a.inv_bm);
    // Visits folded into the node words. The final collect does not read visit or node words, so
    // the fold needs no barrier and spreads over the whole grid: each wave takes runs of 64 visit words
    // (one per lane), then folds its non-zero words one lane per handle, eight words' node words in
    // flight at a time. (A block folding its own range bit by bit serialised tens of thousands of
    // read-modify-writes in the few blocks that own a hub's consecutive dependants.)
    {
        const uint32_t W = blockDim.x >> 6;
        const uint64_t step = (uint64_t)gridDim.x * W * 64;
        for (uint64_t w0 = ((uint64_t)blockIdx.x * W + wid) * 64; w0 < words; w0 += step) {   // wave-uniform
            const uint64_t w = w0 + lane;
            const unsigned long long mine = w < words ? vis64[w] : 0ull;
            if (mine) vis64[w] = 0ull;
            unsigned long long nz = __ballot(mine != 0ull);
            while (nz) {   // wave-uniform
                uint32_t idx[8];
                bool m[8];
                unsigned long long nv[8];
#pragma unroll
                for (int j = 0; j < 8; ++j) {
                    idx[j] = nz ? (uint32_t)__builtin_ctzll(nz) : 64u;
                    nz &= nz ? nz - 1 : 0ull;
                    const unsigned long long wj = idx[j] < 64u ? __shfl(mine, (int)idx[j], 64) : 0ull;
                    m[j] = (wj >> lane) & 1ull;
                    nv[j] = m[j] ? a.node[(w0 + idx[j]) * 64 + lane] : 0ull;
                }
#pragma unroll
                for (int j = 0; j < 8; ++j)
                    if (m[j]) a.node[(w0 + idx[j]) * 64 + lane] = visited_word(nv[j]);
            }
        }
    }
    for (uint64_t w = lo + threadIdx.x; w < hi; w += blockDim.x)
        if (folded || w - lo >= kFinalStage || s_words[w - lo]) invw[w] = 0ull;
    if (threadIdx.x < (uint32_t)kStats) a.blk[(uint64_t)threadIdx.x * kStatBlocks + blockIdx.x] = 0ull;
    if (blockIdx.x == 0) {
        if (threadIdx.x == 0) {
            ctr->root_inv = 0;
            ctr->root_flagged = 0;
        }
        const uint64_t used = std::min<uint64_t>(levels + 3, (uint64_t)kRing);
        for (uint64_t i = threadIdx.x; i < used * (sizeof(LevelCtr) / 8); i += blockDim.x)
            reinterpret_cast<unsigned long long*>(&ctr->lvl[0])[i] = 0ull;
    }
    CPROBE(9);
}

// ---- the wave's tail: its last, small push levels in one persistent launch -------------------------
// After a level group's k_collect + k_level launches, k_wave_tail (kTailBlocks blocks, software grid
// barriers between levels, one wave per block fencing: 1.3 us per barrier at 32 blocks,
// profiles/r7i_grid_barrier.txt) runs the levels that follow while they are small push levels: the
// collect after a pull level, then one push level after the other, until the frontier is empty or a
// level pulls or has more than max_edges edges (that level is left to the host's next group). It
// records where it stopped in ctr->cur. A level group thus ends with one launch however many small push
// levels the wave's tail has (configs[1]: levels 4 and 5, four launches before), and a wave whose pull
// levels fit the group never needs a second group (the asynchronous waves rely on that: max_edges = ~0).
constexpr uint32_t kTailBlocks = 32;

// measurement knobs: the tail's grid (FGI_TAIL_BLOCKS, default kTailBlocks; its blocks must be resident
// together) and whether the push level after a pull stays in the group (FGI_TAIL_HEAD=1: the tail runs it,
// with the collect of the pull's winners)
static uint32_t tail_blocks(const fgi_graph* g) {
    static const uint32_t env = [] {
        const char* e = getenv("FGI_TAIL_BLOCKS");
        return e && *e ? (uint32_t)atoi(e) : 0u;
    }();
    const uint32_t b = env ? env : kTailBlocks;
    return std::max<uint32_t>(1, std::min<uint32_t>(b, (uint32_t)std::max(1, g->n_cu)));
}
static int tail_head_after_pull() {
    static const int v = [] {
        const char* e = getenv("FGI_TAIL_HEAD");
        return e && e[0] == '1' ? 1 : 2;
    }();
    return v;
}
constexpr int kGbarTail = 8;   // g->gbar word of the tail's barrier (its own grid size)

struct TailArgs {
    int grp0;                          // the group's first level (its levels' counters are summed here)
    int L0;                            // the first level the group did not launch
    WaveParams wp;
    CollectArgs col[2];                // frontier buffers by level parity (collect after a pull level)
    ExpandArgs x[2];
    Out o[2];
    const unsigned long long* node;
    uint32_t* vis;
    WaveCtr* ctr;
    unsigned long long* blk;
    unsigned long long* gbar;
    uint64_t bar_timeout;
    uint64_t max_edges;                // a level with more edges is left to the host's next group
    int all;                           // run every remaining level (asynchronous waves: no second group)
    uint32_t fault_block;              // fault injection (FGI_OPT_FAULT_INJECT_TAIL): block fault_block - 1
                                       // leaves at its first grid barrier without arriving
};

// A level-group wave's totals on the device (one writer: block 0's first thread of the tail), so that
// the host need not read them from the level ring, which a tail of more than kRing levels rolls over:
// WaveCtr n_levels / e_trav / f_total / n_pull over the non-empty levels, push_edges / push_f over
// the push levels, mid_push_edges / mid_push_f over those the tail ran, t_max the largest level's edges.
// Summed in registers over the launch and added to the counters once at its end.
struct TailSums {
    unsigned long long n = 0, e = 0, f = 0, np = 0, pe = 0, pf = 0, te = 0, tf = 0, tmax = 0;
    __device__ void add(uint64_t F, uint64_t T, bool pull, bool in_tail) {
        if (!F) return;
        n += 1;
        e += T;
        f += F;
        if (pull) {
            np += 1;
        } else {
            pe += T;
            pf += F;
        }
        if (in_tail) {
            te += T;
            tf += F;
        }
        if (T > tmax) tmax = T;
    }
    __device__ void commit(WaveCtr* c) const {
        c->n_levels += n;
        c->e_trav += e;
        c->f_total += f;
        c->n_pull += np;
        c->push_edges += pe;
        c->push_f += pf;
        c->mid_push_edges += te;
        c->mid_push_f += tf;
        if (tmax > c->t_max) c->t_max = tmax;
    }
};

__global__ __launch_bounds__(kBlock) void k_wave_tail(TailArgs a) {
    __shared__ __align__(16) uint32_t s_x[kChunkEmitCap + 8];
    uint32_t* s_rel = s_x;
    uint32_t* s_base = s_x + kChunk + 4;
    __shared__ Emit em;
    __shared__ MsgEmit<false> me;
    __shared__ unsigned long long s_st[kBlock / 64][kStats];
    __shared__ unsigned long long s_ft;
    WaveCtr* ctr = a.ctr;
    bool first_sync = true;
    auto grid_sync = [&]() -> bool {
        const bool skip = a.fault_block != 0 && first_sync && blockIdx.x + 1 == a.fault_block;
        first_sync = false;
        return soft_grid_sync(a.gbar, &ctr->broken, nullptr, a.bar_timeout, skip, 1);
    };
    // the wave's totals (WaveCtr n_levels ..): the group's levels, read before the ring rolls over — one
    // level per lane of block 0's first wave, every load in flight together, then lane 0 adds them up
    TailSums acc;
    if (blockIdx.x == 0 && threadIdx.x < 64) {
        const int n = a.L0 - a.grp0;
        for (int l0 = 0; l0 < n; l0 += 64) {
            const int l = a.grp0 + l0 + (int)threadIdx.x;
            uint64_t F = 0, T = 0, P = 0;
            if (l < a.L0) {
                const LevelCtr& g = ctr->lvl[l % kRing];
                F = lvl_F(g);
                T = lvl_T(g);
                P = g.pull;
            }
            const int m = min(64, n - l0);
            for (int k = 0; k < m; ++k) {   // lane 0 accounts for lane k's level (in level order)
                const uint64_t Fk = __shfl(F, k, 64), Tk = __shfl(T, k, 64), Pk = __shfl(P, k, 64);
                if (threadIdx.x == 0) acc.add(Fk, Tk, Pk != 0, false);
            }
        }
    }
    int L = a.L0;
    for (bool first = true;; ++L, first = false) {
        LevelCtr& lc = ctr->lvl[L % kRing];
        if (threadIdx.x == 0) s_ft = coh_read(&lc.ft);   // a push producer's packed counter (or the pull's F / T)
        __syncthreads();
        const uint64_t F = lc.F ? lc.F : (s_ft >> 32), T = lc.F ? lc.T : (s_ft & 0xFFFFFFFFull);
        const bool wants_pull = F != 0 && level_pulls(ctr, L, a.wp, F, T);
        if (F == 0 || (!a.all && (wants_pull || T > a.max_edges))) break;
        if (blockIdx.x == 0 && threadIdx.x == 0) {
            acc.add(F, T, false, true);
            if (wants_pull) ctr->pull_pushed += 1;   // an asynchronous wave's level past its queued group
        }
        if (first && L > 0 && ctr->lvl[(L + kRing - 1) % kRing].pull) {   // after a pull level: its frontier list
            collect_front(lc, a.wp.grid, a.col[L & 1], (uint64_t)blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6),
                          (uint64_t)gridDim.x * (blockDim.x >> 6));
            if (!grid_sync()) return;
        }
        if (blockIdx.x == 0) {
            if (threadIdx.x == 0) {
                lc.pull = 0ull;
                lc.mult = level_mult_one_round(T, gridDim.x);
                ctr->lvl[(L + 1) % kRing].npull = lc.npull;
            }
            // level L + 1's counter accumulates during this level; L + 2's is cleared for the next one
            if (threadIdx.x < sizeof(LevelCtr) / 8)
                reinterpret_cast<unsigned long long*>(&ctr->lvl[(L + 2) % kRing])[threadIdx.x] = 0ull;
        }
        const int buf = L & 1;
        Out o = a.o[buf ^ 1];
        o.ln = &ctr->lvl[(L + 1) % kRing];
        emit_init(em);
        expand_level<false>(kProbeLevelsOff, F, T, level_mult_one_round(T, gridDim.x), a.x[buf], a.node, a.vis, o, em, s_x,
                            me, s_rel, s_base, a.blk, s_st, RemoteArgs{});
        if (!grid_sync()) {
            if (blockIdx.x == 0 && threadIdx.x == 0) acc.commit(ctr);
            return;
        }
    }
    if (blockIdx.x == 0 && threadIdx.x == 0) {
        acc.commit(ctr);
        ctr->cur = (unsigned long long)L;
    }
}

#if FGI_VARIANTS   // measured slower than the level groups: variant builds only
// ---- fused waves: the small push levels of a wave inside two persistent launches -----------------
// run_wave's launch sequence is: k_wave_fused<false> (head) — the wave's counters, bitmaps and
// statistics cleared, the roots, then push levels while they are small; k_collect + k_level pairs
// (mid launches) — the pull levels, and push levels of more than big_push edges; k_wave_fused<true>
// (tail) — the collect of a push level that follows a pull level, the remaining small push levels and
// the final count (V_inv, the per-block counts k_final_write lists the ids from). A small push level
// is a chain of dependent round trips over a few thousand edges: inside a persistent grid (one block
// per CU) its cost is one software grid barrier instead of a kernel launch and a collect launch each
// (DESIGN.md §3). The head and the tail each stop at the first level that needs a k_level launch
// (the wave's current level, ctr->cur); the host launches a predicted number of mid pairs (the previous
// wave's), then the tail, and synchronises once; a tail that stopped early (more mid levels than
// predicted) is followed by another round.
struct FusedArgs {
    const uint32_t* roots;
    const uint8_t* imm;
    uint32_t n_roots;
    uint32_t n_handles;
    unsigned long long* node;
    uint32_t* vis;
    uint32_t* inv_bm;
    const uint64_t* row_off;
    const uint32_t* row_len;
    uint32_t* fr_off[2];
    uint32_t* fr_len[2];
    uint64_t* escan[2];
    uint32_t* cstart[2];
    const uint32_t* pool_col;
    const uint64_t* pool_tag;
    int dead_filter;
    int clear_vis;                     // fgi_restore's deferred clear of the visit bitmap
    uint64_t bm_words;
    WaveCtr* ctr;
    unsigned long long* blk;
    unsigned long long* gbar;          // grid-barrier arrival counter (monotonic; g->gbar + kGbarFused)
    unsigned long long* done;          // completion counters (last_block)
    uint64_t bar_timeout;
    int bar_mode;                      // soft_grid_sync's memory ordering (FGI_BAR_MODE)
    int do_init;                       // the head clears the wave state itself (else k_wave_init ran before)
    WaveParams wp;
    CollectArgs col;
    uint64_t big_push;                 // push levels with more edges run as k_level launches
    unsigned long long* status;        // [fin_G] per-block invalidated counts for k_final_write
    uint32_t fin_G;
    uint64_t fin_wpb;
};

template <bool TAIL>
__global__ __launch_bounds__(kBlock) void k_wave_fused(FusedArgs a) {
    __shared__ __align__(16) uint32_t s_x[kChunkEmitCap + 8];
    uint32_t* s_rel = s_x;
    uint32_t* s_base = s_x + kChunk + 4;
    __shared__ Emit em;
    __shared__ MsgEmit<false> me;
    __shared__ unsigned long long s_st[kBlock / 64][kStats];
    __shared__ unsigned long long s_red[kBlock / 64];
    __shared__ unsigned long long s_ft;
    WaveCtr* ctr = a.ctr;
    auto grid_sync = [&]() -> bool {
        return soft_grid_sync(a.gbar, &ctr->broken, nullptr, a.bar_timeout, false, a.bar_mode);
    };
    const uint64_t tid = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const uint64_t nthr = (uint64_t)gridDim.x * blockDim.x;
    int L = 0;
    if constexpr (!TAIL) {
      if (a.do_init) {
        // the wave's counters (broken too: nothing can have set it before the first barrier), the
        // per-block statistics, the invalidated bitmap and the hot snapshot past it, the visit bitmap
        unsigned long long* c64 = reinterpret_cast<unsigned long long*>(ctr);
        for (uint64_t i = tid; i < sizeof(WaveCtr) / 8; i += nthr) c64[i] = 0ull;
        for (uint64_t i = tid; i < (uint64_t)kStatBlocks * kStatCols; i += nthr) a.blk[i] = 0ull;
        uint4* f4 = reinterpret_cast<uint4*>(a.inv_bm);
        for (uint64_t i = tid; i < a.bm_words / 4; i += nthr) f4[i] = make_uint4(0u, 0u, 0u, 0u);
        for (uint64_t i = a.bm_words / 4 * 4 + tid; i < a.bm_words; i += nthr) a.inv_bm[i] = 0u;
        if (a.clear_vis) {
            uint4* v4 = reinterpret_cast<uint4*>(a.vis);
            for (uint64_t i = tid; i < a.bm_words / 4; i += nthr) v4[i] = make_uint4(0u, 0u, 0u, 0u);
            for (uint64_t i = a.bm_words / 4 * 4 + tid; i < a.bm_words; i += nthr) a.vis[i] = 0u;
        }
        if (!grid_sync()) return;
      }
        const Out o0{a.row_off, a.row_len, a.inv_bm, a.fr_off[0], a.fr_len[0], a.escan[0], a.cstart[0], &ctr->lvl[0]};
        const uint32_t gsize = gridDim.x * blockDim.x;
        if (a.imm) {   // Invalidate(true) roots first: their CAS may change node words
            for (uint32_t i0 = blockIdx.x * blockDim.x; i0 < a.n_roots; i0 += gsize)
                root_step<1>(i0 + threadIdx.x, a.roots, a.imm, a.n_roots, 0u, a.n_handles, a.node, a.vis, o0, ctr);
            if (!grid_sync()) return;
        }
        for (uint32_t i0 = blockIdx.x * blockDim.x; i0 < a.n_roots; i0 += gsize)
            root_step<0>(i0 + threadIdx.x, a.roots, a.imm, a.n_roots, 0u, a.n_handles, a.node, a.vis, o0, ctr);
        if (!grid_sync()) return;
    } else {
        // uniform: written by earlier launches only
        if (ctr->phase == kPhaseDone || ctr->broken) return;
        L = (int)ctr->cur;
        const LevelCtr& lc = ctr->lvl[L % kRing];
        const uint64_t F = lvl_F(lc), T = lvl_T(lc);
        if (F != 0) {
            if (level_pulls(ctr, L, a.wp, F, T) || T > a.big_push) {   // a mid level: the host runs another round
                if (blockIdx.x == 0 && threadIdx.x == 0) ctr->mid_base = (unsigned long long)L;
                return;
            }
            if (L > 0 && ctr->lvl[(L + kRing - 1) % kRing].pull) {   // after a pull level: its frontier list
                CollectArgs c = a.col;
                const int buf = L & 1;
                c.fr_off = a.fr_off[buf];
                c.fr_len = a.fr_len[buf];
                c.escan = a.escan[buf];
                c.cstart = a.cstart[buf];
                collect_front(lc, a.wp.grid, c, (uint64_t)blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6),
                              (uint64_t)gridDim.x * (blockDim.x >> 6));
                if (!grid_sync()) return;
            }
        }
    }
    // the push levels while they are small (level L's frontier and counters are complete here)
    for (;; ++L) {
        LevelCtr& lc = ctr->lvl[L % kRing];
        if (threadIdx.x == 0) s_ft = coh_read(&lc.ft);
        __syncthreads();
        const uint64_t F = lc.F ? lc.F : (s_ft >> 32), T = lc.F ? lc.T : (s_ft & 0xFFFFFFFFull);
        if (F == 0) break;
        if (level_pulls(ctr, L, a.wp, F, T) || T > a.big_push) {
            if (blockIdx.x == 0 && threadIdx.x == 0) {
                ctr->cur = (unsigned long long)L;
                ctr->mid_base = (unsigned long long)L;
            }
            return;
        }
        if (blockIdx.x == 0) {
            if (threadIdx.x == 0) {
                ctr->lvl[(L + 1) % kRing].npull = lc.npull;
                ctr->n_levels += 1;
                ctr->e_trav += T;
                ctr->f_total += F;
                ctr->push_edges += T;
                ctr->push_f += F;
            }
            // level L + 1's counter accumulates during this level; L + 2's is cleared for the next one
            if (threadIdx.x < sizeof(LevelCtr) / 8)
                reinterpret_cast<unsigned long long*>(&ctr->lvl[(L + 2) % kRing])[threadIdx.x] = 0ull;
        }
        const int buf = L & 1;
        const ExpandArgs x{a.fr_off[buf], a.escan[buf], a.cstart[buf], a.pool_col, a.pool_tag, a.dead_filter};
        const Out o{a.row_off,          a.row_len,         a.inv_bm, a.fr_off[buf ^ 1], a.fr_len[buf ^ 1],
                    a.escan[buf ^ 1], a.cstart[buf ^ 1], &ctr->lvl[(L + 1) % kRing]};
        emit_init(em);
        expand_level<false>(kProbeLevelsOff, F, T, level_mult_one_round(T, gridDim.x), x, a.node, a.vis, o, em, s_x, me,
                            s_rel, s_base, a.blk, s_st, RemoteArgs{});
        if (!grid_sync()) return;
    }
    // the wave is done: statistics folded into the wave counters, the per-block counts of the final
    // collect (k_final_write's geometry), V_inv by the last block
    if (blockIdx.x < (uint32_t)kStats) {
        const int k = blockIdx.x;
        unsigned long long* dst[kStats] = {&ctr->e_match,   &ctr->n_flagged, &ctr->pull_surv, &ctr->pull_edges,
                                           &ctr->pull_live, &ctr->pull_win,  &ctr->pull_tail, &ctr->pull_scan};
        const unsigned long long* col = a.blk + (uint64_t)k * kStatBlocks;
        unsigned long long x = 0;
#pragma unroll
        for (uint32_t q = 0; q < kStatBlocks / kBlock; ++q) x += col[q * kBlock + threadIdx.x];
        x = block_sum(x, s_red);
        if (threadIdx.x == 0) *dst[k] = x + (k == kStFlagged ? ctr->root_flagged : 0ull);
    }
    const uint64_t words = ((uint64_t)a.n_handles + 63) / 64;
    const unsigned long long* inv64 = reinterpret_cast<const unsigned long long*>(a.inv_bm);
    for (uint32_t t = blockIdx.x; t < a.fin_G; t += gridDim.x) {   // block-uniform
        const uint64_t lo = t * a.fin_wpb, hi = std::min<uint64_t>(words, lo + a.fin_wpb);
        unsigned long long c = 0;
        for (uint64_t w = lo + threadIdx.x; w < hi; w += blockDim.x) c += (unsigned long long)__popcll(inv64[w]);
        c = block_sum(c, s_red);
        if (threadIdx.x == 0) coh_xchg(a.status + t, c);
    }
    if (!last_block(a.done, gridDim.x)) return;
    unsigned long long all = 0;
    for (uint32_t k = threadIdx.x; k < a.fin_G; k += blockDim.x) all += coh_read(a.status + k);
    all = block_sum(all, s_red);
    if (threadIdx.x == 0) {
        ctr->inv = all;
        ctr->cur = (unsigned long long)L;
        ctr->phase = kPhaseDone;
    }
}

#endif  // FGI_VARIANTS

__global__ __launch_bounds__(kBlock) void k_wave_init(WaveCtr* ctr, unsigned long long* blk, uint32_t* inv_bm,
                                                      uint32_t* vis_bm, uint64_t bm_words) {
    const uint64_t tid = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const uint64_t nthr = (uint64_t)gridDim.x * blockDim.x;
    unsigned long long* c = reinterpret_cast<unsigned long long*>(ctr);
    // the word's one writer stamps the wave's start (statistics without stream events, run_wave)
    for (uint64_t i = tid; i < sizeof(WaveCtr) / 8; i += nthr) c[i] = i == offsetof(WaveCtr, t0) / 8 ? wall_clock64() : 0ull;
    for (uint64_t i = tid; i < (uint64_t)kStatBlocks * kStatCols; i += nthr) blk[i] = 0ull;
    uint4* f4 = reinterpret_cast<uint4*>(inv_bm);
    for (uint64_t i = tid; i < bm_words / 4; i += nthr) f4[i] = make_uint4(0u, 0u, 0u, 0u);
    for (uint64_t i = bm_words / 4 * 4 + tid; i < bm_words; i += nthr) inv_bm[i] = 0u;
    if (vis_bm) {   // fgi_restore's deferred clear
        uint4* v4 = reinterpret_cast<uint4*>(vis_bm);
        for (uint64_t i = tid; i < bm_words / 4; i += nthr) v4[i] = make_uint4(0u, 0u, 0u, 0u);
        for (uint64_t i = bm_words / 4 * 4 + tid; i < bm_words; i += nthr) vis_bm[i] = 0u;
    }
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

fgi_status flush_vis(fgi_graph* g) {
    if (!g->vis_stale) return FGI_OK;
    FGI_HIP(g, hipMemsetAsync(g->vis_bm, 0, g->bm_words * 4, g->stream));
    g->vis_stale = false;
    return FGI_OK;
}

fgi_status fold(fgi_graph* g) {
    FGI_TRY(flush_vis(g));
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

namespace {

// Algorithmic bytes of the pull levels of a wave (k_level on pull levels): per candidate scanned
// its entry (slot 4, heads 8, row length 4) and the visit / class words (1/4 B); per survivor its
// entry written forward (16 B); per queued candidate its list offset and length (12 B) and entry
// re-read (4 B), and 4 B per further dependency examined. The invalidated-bitmap probes hit L2 and
// are not counted.
uint64_t pull_level_bytes(const WaveCtr& c) {
    const uint64_t head_probes = c.pull_live;   // >= 1 examined per live candidate in the head step
    const uint64_t tail_deps = c.pull_edges > head_probes ? c.pull_edges - head_probes : 0;
    return 16 * c.pull_scan + c.pull_scan / 4 + 16 * c.pull_surv + 16 * c.pull_tail + 4 * tail_deps;
}

// Flags of the per-level timing events (FGI_EVENT_FLAGS overrides, for measurement). Without the
// system-scope fence a record costs ~1 us instead of ~6 us between kernels (profiles/, e1).
unsigned event_flags() {
    static const unsigned f = getenv("FGI_EVENT_FLAGS") ? (unsigned)strtoul(getenv("FGI_EVENT_FLAGS"), nullptr, 0)
                                                       : (unsigned)hipEventDisableSystemFence;
    return f;
}

// the level grid is bounded by the per-block statistics rows (the epilogues take any grid)
constexpr uint32_t kLevelGridMax = kStatBlocks;
static_assert(kFinalBlocks <= kLevelGridMax, "epilogue geometry");

}  // namespace

// kLevelOcc resident blocks per CU (k_level launch bounds); a pull block owns at most kMaxIter tiles, so a
// larger graph gets more blocks, up to kLevelGridMax (268M slots per device, hub-first labels included); beyond that, no pull.
// FGI_OPT_PULL_TPB fixes the tiles per block instead (tests: every grid takes the same results).
void pull_geometry(const fgi_graph* g, uint32_t* grid, uint32_t* tpb) {
    const uint64_t n_tiles = ((uint64_t)g->n_slots + kPullTile - 1) / kPullTile;
    uint64_t G = std::min<uint64_t>((uint64_t)g->n_cu * kLevelOcc, kLevelGridMax);
    uint64_t t = (n_tiles + G - 1) / G;
    if (g->opt_pull_tpb > 0) {
        t = std::min<uint64_t>((uint64_t)g->opt_pull_tpb, kMaxIter);
        G = (n_tiles + t - 1) / t;
    }
    if (t > kMaxIter) {
        t = kMaxIter;
        G = (n_tiles + t - 1) / t;
    }
    *grid = G <= kLevelGridMax ? (uint32_t)G : 0u;
    *tpb = (uint32_t)std::max<uint64_t>(t, 1);
}

namespace {

WaveParams wave_params(fgi_graph* g, int multi, int direction, uint64_t total_edges, uint64_t n_beta) {
    WaveParams wp;
    wp.multi = multi;
    wp.direction = direction;
    wp.pull_threshold = total_edges / (uint64_t)(g->opt_pull_alpha > 0 ? g->opt_pull_alpha : 1);
    wp.stay_pull_f = g->opt_pull_beta > 0 ? n_beta / (uint64_t)g->opt_pull_beta : ~0ull;
    pull_geometry(g, &wp.grid, &wp.tpb);
    if (wp.grid == 0) {   // no pull levels: the traversal grid of a push level
        wp.grid = std::min<uint32_t>((uint32_t)g->n_cu * kLevelOcc, kLevelGridMax);
        wp.tpb = 0;
        if (wp.direction != 1) wp.direction = 1;
    }
    wp.n_tiles = ((uint64_t)g->n_slots + kPullTile - 1) / kPullTile;
    return wp;
}

bool pull_ready(const fgi_graph* g, const WaveParams& wp) {
    return wp.tpb != 0 && g->uin_src && g->uin_epoch == g->mut_epoch && g->cand_grid == wp.grid;
}

Out out_for(fgi_graph* g, int buf, LevelCtr* ln) {
    return Out{g->row_off, g->row_len, g->inv_bm, g->fr_off[buf], g->fr_len[buf], g->escan[buf], g->cstart[buf], ln};
}

CollectArgs collect_args(fgi_graph* g, uint32_t n_slots, const WaveParams& wp, int buf) {
    CollectArgs c;
    (void)n_slots;
    c.wl = g->wl;
    c.seg = g->cand_seg;
    c.row_len = g->row_len;
    c.row_off = g->row_off;
    c.pre = g->bsum + 3ull * wp.grid;
    c.fr_off = g->fr_off[buf];
    c.fr_len = g->fr_len[buf];
    c.escan = g->escan[buf];
    c.cstart = g->cstart[buf];
    c.hot_id = g->hot_id;
    c.hot_bm = g->inv_bm + g->hot_w0;
    c.n_hot = g->n_hot;
    c.inv = g->inv_bm;
    c.sum_bm = g->part ? nullptr : reinterpret_cast<unsigned long long*>(g->sum_bm);   // over inv_bm only
    c.n64 = ((uint64_t)g->n_handles + 63) / 64;
    c.sum_min = g->opt_sum_min;
    return c;
}

// k_collect: one wave per pull block (a grid-stride loop covers any grid)
uint32_t collect_grid(const fgi_graph* g, const WaveParams& wp) {
    (void)g;
    constexpr uint32_t W = kCollectThreads / 64;
    return std::max<uint32_t>(1, (wp.grid + W - 1) / W);
}

// Level L's collect grid: the full one unless the previous wave's directions say the collect has nothing
// to do (level L pushes and level L - 1 did not pull); a small grid then still does everything if the
// prediction is wrong (k_collect's loops stride over any grid), only slower. An empty launch of the full
// grid costs ~3.8 us on configs[1] (profiles/r12c1).
uint32_t collect_grid_at(const fgi_graph* g, const WaveParams& wp, int L) {
    const uint32_t full = collect_grid(g, wp);
    const std::vector<uint8_t>& d = g->last_dirs;
    if (L < 0 || (size_t)L >= d.size()) return full;
    const bool needed = d[L] || (L > 0 && d[L - 1]);
    return needed ? full : std::min<uint32_t>(full, 4u);
}

PullArgs pull_args(fgi_graph* g, uint32_t n_slots, const uint32_t* front_rd) {
    PullArgs p;
    p.n_slots = n_slots;
    p.uin_off = g->uin_off;
    p.uin_len = g->uin_len;
    p.uin_src = g->uin_src;
    p.front_rd = front_rd;
    // the summary of the bitmap this level probes: inv_bm, or a partition's all-gathered front_global
    // (used only where the level's k_collect built it: its `sum` word)
    p.sum = ((g->part != nullptr) == (front_rd != g->inv_bm)) ? g->sum_bm : nullptr;
    p.hot_bit0 = (uint32_t)(g->hot_w0 * 32);
    p.hot_lds = std::min<uint32_t>(g->n_hot / 32, kLdsHot);
    p.inv_bm = g->inv_bm;
    p.wl = g->wl;
    p.cls = g->cls_bm;
    p.bsum = g->bsum;
    p.cand_seg = g->cand_seg;
    p.c[0] = g->cand;
    for (int k = 0; k < 2; ++k) {
        p.c[1 + k] = g->sv[k];
        p.sv[k] = g->sv[k];
        p.sv_cnt[k] = g->sv_cnt[k];
    }
    return p;
}

ExpandArgs expand_args(fgi_graph* g, int buf) {
    static const uint64_t small_max = [] {
        const char* e = getenv("FGI_PUSH_SMALL");   // measurement: the small-level threshold (0 off)
        return e && *e ? (uint64_t)strtoull(e, nullptr, 10) : kPushSmallMax;
    }();
    ExpandArgs x{g->fr_off[buf], g->escan[buf], g->cstart[buf], g->pool_col, g->pool_tag, g->opt_dead_filter};
    x.small_max = small_max;
    return x;
}

// the invalidated bitmap -> V_inv (ctr->inv) and, with ids, the invalidated list
hipError_t launch_final(fgi_graph* g, uint32_t n_handles, bool ids = true, uint32_t* out = nullptr, ListPub pub = ListPub{},
                        WaveEnd end = WaveEnd{}) {
    if (!ids) pub.dst = nullptr;   // no list kernel: the caller publishes
    if (!end.ctr) g->wave_clean = false;   // the counters (inv, ...) are written and nothing clears them
    if (!out) out = g->inv;
    const auto* inv64 = reinterpret_cast<const unsigned long long*>(g->inv_bm);
    const FoldArgs f = fold_args(g);
    if (f.xbm) {   // hot labels: one fold tile per counting block, the list from the folded bitmap
        const uint64_t words = ((uint64_t)g->ext_handles + 63) / 64;
        const uint32_t tiles = (uint32_t)((words + kFoldWords - 1) / kFoldWords);
        unsigned long long* st = g->fold_status;
        const uint32_t Gc = std::max<uint32_t>(std::min<uint32_t>(tiles, kFoldBlocks), kStats);
        hipLaunchKernelGGL(k_final_count, dim3(Gc), dim3(kBlock), 0, g->stream, inv64, words,
                           (uint64_t)kFoldWords, st, g->ctr, (const unsigned long long*)g->blk_stats, ids ? 0 : 1, g->done, f);
        if (ids) {
            const uint32_t G = std::min<uint32_t>(kFinalBlocks, tiles), spb = (tiles + G - 1) / G;
            const uint32_t G2 = (tiles + spb - 1) / spb;
            hipLaunchKernelGGL(k_final_write, dim3(G2), dim3(kBlock), 0, g->stream, (const unsigned long long*)g->xbm, words,
                               (uint64_t)spb * kFoldWords, (const unsigned long long*)st, g->ctr, out, 0, spb, pub, end);
        }
        return hipGetLastError();
    }
    const uint64_t words = ((uint64_t)n_handles + 63) / 64;
    uint32_t G = (uint32_t)std::min<uint64_t>(kFinalBlocks, std::max<uint64_t>(kStats, (words + kFinalWpb - 1) / kFinalWpb));
    const uint64_t wpb = (words + G - 1) / G;
    // per-block counts apart from the pull prefixes a collect may still read
    unsigned long long* st = g->bsum + 6ull * kStatBlocks;
    hipLaunchKernelGGL(k_final_count, dim3(G), dim3(kBlock), 0, g->stream, inv64, words, wpb, st, g->ctr,
                       (const unsigned long long*)g->blk_stats, ids ? 0 : 1, g->done, FoldArgs{});
    if (ids)
        hipLaunchKernelGGL(k_final_write, dim3(G), dim3(kBlock), 0, g->stream, inv64, words, wpb,
                           (const unsigned long long*)st, g->ctr, out, 0, 1u, pub, end);
    return hipGetLastError();
}

TailArgs tail_args(fgi_graph* g, int grp0, int L0, const WaveParams& wp, uint64_t max_edges) {
    TailArgs ta{};
    ta.grp0 = grp0;
    ta.L0 = L0;
    ta.wp = wp;
    for (int b = 0; b < 2; ++b) {
        ta.col[b] = collect_args(g, g->n_slots, wp, b);
        ta.x[b] = expand_args(g, b);
        ta.o[b] = out_for(g, b, nullptr);
    }
    ta.node = reinterpret_cast<const unsigned long long*>(g->node);
    ta.vis = g->vis_bm;
    ta.ctr = g->ctr;
    ta.blk = g->blk_stats;
    ta.gbar = g->gbar + kGbarTail;
    ta.bar_timeout = kGridBarTimeout;
    ta.max_edges = max_edges;
    // fault injection (tests): the (k+1)-th tail launched from the option on loses a block at its first
    // barrier, which then times out after 20 ms (the failure path of run_wave / wave_wait)
    if (g->fault_tail_block) {
        if (g->fault_tail_skip == 0) {
            ta.fault_block = g->fault_tail_block;
            ta.bar_timeout = 2000000ull;
            g->fault_tail_block = 0;
        } else {
            --g->fault_tail_skip;
        }
    }
    return ta;
}

#ifndef FGI_ROOT_BLOCK
#define FGI_ROOT_BLOCK 256   // measurement builds: make variant-rootblk RB=<threads> (a multiple of 64)
#endif
void launch_roots(fgi_graph* g, uint32_t n_roots, const uint32_t* roots_dev, const uint8_t* imm_dev, uint32_t base,
                  uint32_t n_range, int publish, bool ext_roots = false, int stamp = 0) {
    const RootMap rm{g->lbl_hot ? g->s2l : nullptr, g->ext_slots, g->ext_handles, g->lbl_K, ext_roots && g->lbl_K ? 1 : 0};
    constexpr uint32_t kRootBlock = FGI_ROOT_BLOCK;
    static_assert(kRootBlock % 64 == 0 && kRootBlock <= kBlock, "root block");
    const uint32_t nb = (n_roots + kRootBlock - 1) / kRootBlock;
    auto* node = reinterpret_cast<unsigned long long*>(g->node);
    const Out o = out_for(g, 0, &g->ctr->lvl[0]);
    // the immediate roots' launch never publishes: the second launch adds to the same counter
    if (imm_dev)
        hipLaunchKernelGGL(k_roots<1>, dim3(nb), dim3(kRootBlock), 0, g->stream, roots_dev, imm_dev, n_roots, base, n_range,
                           node, g->vis_bm, o, g->ctr, g->done, 0, rm, stamp);
    hipLaunchKernelGGL(k_roots<0>, dim3(nb), dim3(kRootBlock), 0, g->stream, roots_dev, imm_dev, n_roots, base, n_range, node,
                       g->vis_bm, o, g->ctr, g->done, publish, rm, imm_dev ? 0 : stamp);
}

}  // namespace

#if FGI_PROBE
// block 0's phase times of the last cooperative waves (FGI_TRACE=1, probe build): entry -> roots
// done -> level barriers -> final counts -> prefix barrier -> ids written -> cleaned up
void print_coop_probe() {
    static unsigned long long h[64][10];
    unsigned int n = 0;
    if (hipMemcpyFromSymbol(h, HIP_SYMBOL(d_cprobe), sizeof(h)) != hipSuccess ||
        hipMemcpyFromSymbol(&n, HIP_SYMBOL(d_cprobe_n), sizeof(n)) != hipSuccess)
        return;
    for (unsigned int i = (n > 8 ? n - 8 : 0); i < n; ++i) {
        const unsigned long long* t = h[i % 64];
        fprintf(stderr, "[coop] wave %u:", i);
        for (int k = 1; k < 10; ++k)
            if (t[k]) fprintf(stderr, " %d:+%.1f", k, (t[k] - t[0]) / 100.0);
        fprintf(stderr, " us\n");
    }
}
#endif

// soft_grid_sync's memory ordering (FGI_BAR_MODE, measurement; default 1: one wave per block fences)
static int bar_mode() {
    static const int m = [] {
        const char* e = getenv("FGI_BAR_MODE");
        return e ? atoi(e) : 1;
    }();
    return m;
}

// FGI_COOP_LAUNCH=1: k_wave_coop as a cooperative launch (grid barriers by the device library)
// instead of a plain launch with soft_grid_sync. Nothing else launches cooperatively.
bool coop_launch_mode() {
#if FGI_VARIANTS
    static const bool coop = [] {
        const char* e = getenv("FGI_COOP_LAUNCH");
        return e && e[0] == '1';
    }();
    return coop;
#else
    return false;   // the cooperative launch of round 3 (and its exit-time fault under rocprofv3): variant builds only
#endif
}

// One push-only wave in a single launch of k_wave_coop (one block per CU, grid barriers between its
// phases): no host synchronisation. The roots
// (n_max, or *n_dev of them) are device-resident; the invalidated handles are appended at
// out[*out_n ..). The wave folds its visits into the node words itself.
fgi_status run_wave_coop(fgi_graph* g, uint32_t n_max, const uint32_t* roots_dev, const uint8_t* imm_dev,
                         const unsigned long long* n_dev, uint32_t* out, unsigned long long* out_n,
                         unsigned long long* acc, unsigned long long* abort) {
    hipStream_t s = g->stream;
    FGI_TRY(ensure_cstart(g, std::max<uint64_t>(g->pool_top, g->pool_cap)));
    const bool coop = coop_launch_mode();
    // resident blocks per CU, per graph (its device): the launch-time residency bound below. The grid
    // is half the CUs, a quarter of what the kernel's resources allow, so other work on the device
    // would have to hold most of it for blocks to wait on each other; if it does, the barrier's timeout
    // fails the batch cleanly (soft_grid_sync) instead of hanging.
    int& per_cu = g->coop_per_cu;
    if (per_cu == 0 &&
        (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, k_wave_coop<true>, kBlock, 0) !=
             hipSuccess ||
         per_cu < 1))
        per_cu = 1;
    static const uint32_t g_env = [] {   // FGI_COOP_BLOCKS: measurement knob (grid size)
        const char* e = getenv("FGI_COOP_BLOCKS");
        return e ? (uint32_t)strtoul(e, nullptr, 10) : 0u;
    }();
    // one block per two CUs: with the software barrier a grid of 128 runs a configs[4] round's cascades
    // in 0.24 ms of kernels against 0.32 ms with 256 blocks (profiles/r6zl_coop_blocks.txt)
    const uint32_t G = std::max<uint32_t>((uint32_t)kStats, g_env ? g_env : (uint32_t)std::max(g->n_cu / 2, 1));
    if ((uint64_t)G > (uint64_t)per_cu * (uint64_t)std::max(g->n_cu, 1))
        return set_err(g, FGI_ENOTSUP, "cooperative wave: %u blocks cannot be resident", G);
    FGI_TRY(fold(g));   // visits of a level-launched wave
    if (coop) FGI_TRY(coop_warm(g));
    g->wave_clean = false;   // this path dirties the wave state (run_wave re-inits)
    if (!g->coop_clean)
        hipLaunchKernelGGL(k_wave_init, dim3(kInitBlocks), dim3(kBlock), 0, s, g->ctr, g->blk_stats, g->inv_bm,
                           (uint32_t*)nullptr, (uint64_t)g->bm_words);
    CoopArgs a{};
    a.roots = roots_dev;
    a.imm = imm_dev;
    a.n_max = n_max;
    a.n_dev = n_dev;
    a.node = reinterpret_cast<unsigned long long*>(g->node);
    a.vis = g->vis_bm;
    a.inv_bm = g->inv_bm;
    a.row_off = g->row_off;
    a.row_len = g->row_len;
    for (int k = 0; k < 2; ++k) {
        a.fr_off[k] = g->fr_off[k];
        a.fr_len[k] = g->fr_len[k];
        a.escan[k] = g->escan[k];
        a.cstart[k] = g->cstart[k];
    }
    a.pool_col = g->pool_col;
    a.pool_tag = g->pool_tag;
    a.dead_filter = g->opt_dead_filter;
    a.n_handles = g->n_handles;
    a.ctr = g->ctr;
    a.blk = g->blk_stats;
    a.cnt = g->bsum + 5ull * kStatBlocks;   // apart from the pull prefixes and k_final's status words
    a.out = out;
    a.out_n = out_n;
    a.acc = acc;
    a.abort = abort;
    a.abort_w = abort;
    a.gbar = g->gbar;
    a.bar_mode = bar_mode();
    // fault injection (FGI_OPT_FAULT_INJECT, tests): after fault_skip more cascade launches, one block
    // of the cascade leaves at its first barrier without arriving; the others give up after 20 ms
    uint32_t fb = 0;
    if (g->fault_block) {
        if (g->fault_skip == 0) {
            fb = g->fault_block;
            g->fault_block = 0;
        } else {
            --g->fault_skip;
        }
    }
    a.fault_block = fb;
    a.bar_timeout = fb ? 2000000ull : kGridBarTimeout;
    static const int one_round = [] {
        const char* e = getenv("FGI_COOP_CHUNKS");
        return e && e[0] == '0' ? 0 : 1;
    }();
    a.one_round = one_round;
    a.fold = fold_args(g);
    a.ext_words = ((uint64_t)g->ext_handles + 63) / 64;
    if (coop) {
#if FGI_VARIANTS
        void* args[] = {&a};
        FGI_HIP(g, hipLaunchCooperativeKernel(reinterpret_cast<const void*>(k_wave_coop<false>), dim3(G), dim3(kBlock), args, 0, s));
#endif
    } else {
        hipLaunchKernelGGL(k_wave_coop<true>, dim3(G), dim3(kBlock), 0, s, a);
        FGI_HIP(g, hipGetLastError());
    }
    g->coop_clean = true;   // the wave folded its visits and cleared what it used
    note_words(g);
    return FGI_OK;
}

#if FGI_PROBE
// per level: kernel span, dispatch skew, and per-phase medians / maxima over the blocks (us)
void print_probe(fgi_graph* g, int L0, int L1) {
    static unsigned long long h[kProbeLevels][kProbeBlocks][kProbePts];
    if (hipMemcpyFromSymbol(h, HIP_SYMBOL(d_probe), sizeof(h)) != hipSuccess) return;
    for (int l = L0; l < L1 && l < kProbeLevels; ++l) {
        const bool pull = g->ctr_host->lvl[l % kRing].pull != 0;
        // phase boundaries in order: pull 0 entry, 1 staged, 7 last batch (wave 0), 2 loop done
        // (wave 0), 3 all waves, 4 write-back + stats, 5 sums published, 6 exit; push 0 entry,
        // 1 set up, 4 chunk map (last chunk), 5 edges + dead filter, 6 tags / words / visits,
        // 7 winners emitted, 2 expanded, 3 published
        const int pull_pts[] = {0, 1, 7, 2, 3, 4, 5, 6};
        const int push_pts[] = {0, 1, 4, 5, 6, 7, 2, 3};
        const int* pts = pull ? pull_pts : push_pts;
        const int np = 8;
        unsigned long long t_lo = ~0ull, t_hi = 0, s_hi = 0;
        std::vector<std::vector<double>> d(np);
        for (int b = 0; b < kProbeBlocks; ++b) {
            const unsigned long long* t = h[l][b];
            if (!t[0]) continue;
            t_lo = std::min(t_lo, t[0]);
            s_hi = std::max(s_hi, t[0]);
            for (int k = 0; k < np; ++k) t_hi = std::max(t_hi, t[pts[k]]);
            for (int k = 1; k < np; ++k)
                if (t[pts[k]] && t[pts[k - 1]]) d[k].push_back((double)(t[pts[k]] - t[pts[k - 1]]) / 100.0);
        }
        if (t_lo == ~0ull) continue;
        fprintf(stderr, "[probe] level %d %s: span %.1f us, start skew %.1f us; phases (median/max us):", l,
                pull ? "pull" : "push", (t_hi - t_lo) / 100.0, (s_hi - t_lo) / 100.0);
        for (int k = 1; k < np; ++k) {
            auto& v = d[k];
            if (v.empty()) continue;
            std::sort(v.begin(), v.end());
            fprintf(stderr, " %d:%.1f/%.1f", k, v[v.size() / 2], v.back());
        }
        fprintf(stderr, "\n");
    }
}
#endif

namespace {

#if FGI_VARIANTS
// FGI_FUSED_BLOCKS: the fused kernels' grid (default one block per CU; measurement)

bool fused_init_in_head() {
    static const bool h = [] {
        const char* e = getenv("FGI_FUSED_INIT");
        return e && e[0] == '1';
    }();
    return h;
}

uint32_t fused_grid(const fgi_graph* g) {
    static const uint32_t env = [] {
        const char* e = getenv("FGI_FUSED_BLOCKS");
        return e ? (uint32_t)strtoul(e, nullptr, 10) : 0u;
    }();
    return std::max<uint32_t>((uint32_t)kStats, env ? env : (uint32_t)std::max(g->n_cu, 1));
}

#endif  // FGI_VARIANTS

hipError_t ensure_events(fgi_graph* g, size_t n) {
    while (g->ev.size() < n) {
        hipEvent_t e;
        const hipError_t r = hipEventCreateWithFlags(&e, event_flags());
        if (r != hipSuccess) return r;
        g->ev.push_back(e);
    }
    return hipSuccess;
}

}  // namespace

#if FGI_VARIANTS
// A wave as fused launches (k_wave_fused head, k_collect + k_level mid pairs, k_wave_fused tail; see
// above): one host synchronisation when the predicted number of mid pairs suffices. Returns
// FGI_ENOTSUP (nothing launched) if the fused grid cannot be resident on this device.
static fgi_status run_wave_fused(fgi_graph* g, uint32_t n_roots, const uint32_t* roots_dev, const uint8_t* imm_dev,
                                 fgi_wave_stats* stats, WaveParams wp, bool timing,
                                 std::chrono::steady_clock::time_point t0) {
    hipStream_t s = g->stream;
    const uint32_t G = fused_grid(g);
    if (g->fused_per_cu == 0) {
        int a = 0, b = 0;
        if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&a, k_wave_fused<false>, kBlock, 0) != hipSuccess ||
            hipOccupancyMaxActiveBlocksPerMultiprocessor(&b, k_wave_fused<true>, kBlock, 0) != hipSuccess)
            a = b = 0;
        g->fused_per_cu = std::max(1, std::min(a, b));
    }
    if ((uint64_t)G > (uint64_t)g->fused_per_cu * (uint64_t)std::max(g->n_cu, 1)) return FGI_ENOTSUP;
    FusedArgs a{};
    a.roots = roots_dev;
    a.imm = imm_dev;
    a.n_roots = n_roots;
    a.n_handles = g->n_handles;
    a.node = reinterpret_cast<unsigned long long*>(g->node);
    a.vis = g->vis_bm;
    a.inv_bm = g->inv_bm;
    a.row_off = g->row_off;
    a.row_len = g->row_len;
    for (int k = 0; k < 2; ++k) {
        a.fr_off[k] = g->fr_off[k];
        a.fr_len[k] = g->fr_len[k];
        a.escan[k] = g->escan[k];
        a.cstart[k] = g->cstart[k];
    }
    a.pool_col = g->pool_col;
    a.pool_tag = g->pool_tag;
    a.dead_filter = g->opt_dead_filter;
    a.clear_vis = g->vis_stale ? 1 : 0;
    a.bm_words = g->bm_words;
    a.ctr = g->ctr;
    a.blk = g->blk_stats;
    a.gbar = g->gbar + kGbarFused;
    a.done = g->done;
    a.bar_timeout = kGridBarTimeout;
    a.bar_mode = bar_mode();
    a.do_init = fused_init_in_head() ? 1 : 0;
    a.wp = wp;
    a.col = collect_args(g, g->n_slots, wp, 0);   // frontier buffers chosen per level on the device
    a.big_push = (uint64_t)G * kChunk;            // one round of the largest chunks over the grid
    if (g->opt_fused & kFusedMidPush) a.big_push = 0;          // tests: every push level as a k_level launch
    if (g->opt_fused & kFusedTailPush) a.big_push = ~0ull;     // tests: every push level in the fused grid
    const uint64_t words = ((uint64_t)g->n_handles + 63) / 64;
    a.fin_G = (uint32_t)std::min<uint64_t>(kFinalBlocks, std::max<uint64_t>(kStats, (words + kFinalWpb - 1) / kFinalWpb));
    a.fin_wpb = (words + a.fin_G - 1) / a.fin_G;
    a.status = g->bsum + 6ull * kStatBlocks;
    g->vis_stale = false;
    g->coop_clean = false;
    if (n_roots) g->v_dirty = true;
    const auto* node = reinterpret_cast<const unsigned long long*>(g->node);
    FGI_HIP(g, ensure_events(g, 2 * (size_t)kMidMax + 4));
    hipEvent_t* ev = g->ev.data();
    const size_t eh = 2 * (size_t)kMidMax;   // the head's / tail's event pair
    if (timing || stats) FGI_HIP(g, hipEventRecord(g->ev_w0, s));
    g->wave_clean = false;   // this path dirties the wave state (run_wave re-inits)
    if (!a.do_init)   // the wave state cleared by its own launch: the head's first barrier has no dirty 4 MB
        hipLaunchKernelGGL(k_wave_init, dim3(kInitBlocks), dim3(kBlock), 0, s, g->ctr, g->blk_stats, g->inv_bm,
                           a.clear_vis ? g->vis_bm : nullptr, (uint64_t)g->bm_words);
    if (timing) FGI_HIP(g, hipEventRecord(ev[eh], s));
    hipLaunchKernelGGL(k_wave_fused<false>, dim3(G), dim3(kBlock), 0, s, a);
    if (timing) FGI_HIP(g, hipEventRecord(ev[eh + 1], s));
    FGI_HIP(g, hipGetLastError());
    const ExpandArgs x0 = expand_args(g, 0), x1 = expand_args(g, 1);
    const Out o0 = out_for(g, 1, nullptr), o1 = out_for(g, 0, nullptr);
    const PullArgs pa = pull_args(g, g->n_slots, g->inv_bm);
    const CollectArgs c0 = collect_args(g, g->n_slots, wp, 0), c1 = collect_args(g, g->n_slots, wp, 1);
    int P = (g->opt_fused & kFusedNoPredict) ? 0 : std::min(kMidMax, std::max(0, g->last_mid));
    double pull_ms = 0, expand_ms = 0, fused_ms = 0;
    uint64_t pull_launches = 0, expand_launches = 0, fused_launches = 1, syncs = 0;
    float ms = 0;
    for (int round = 0;; ++round) {
        if (round > 0) FGI_HIP(g, hipMemsetAsync(g->ctr->mid_kind, 0, sizeof(g->ctr->mid_kind), s));
        for (int i = 0; i < P; ++i) {
            // the level (mid_base + i) is known on the device only: its parity picks the buffers there
            hipLaunchKernelGGL(k_collect, dim3(collect_grid(g, wp)), dim3(kCollectThreads), 0, s, -1 - i, g->ctr, wp,
                               c0, c1, a.big_push);
            if (timing) FGI_HIP(g, hipEventRecord(ev[2 * i], s));
            hipLaunchKernelGGL(k_level<false>, dim3(wp.grid), dim3(kBlock), 0, s, -1 - i, wp, x0, x1, pa, node, g->vis_bm,
                               o0, o1, g->ctr, g->blk_stats, g->done, RemoteArgs{}, a.big_push);
            if (timing) FGI_HIP(g, hipEventRecord(ev[2 * i + 1], s));
        }
        if (timing) FGI_HIP(g, hipEventRecord(ev[eh + 2], s));
        hipLaunchKernelGGL(k_wave_fused<true>, dim3(G), dim3(kBlock), 0, s, a);
        if (timing) FGI_HIP(g, hipEventRecord(ev[eh + 3], s));
        ++fused_launches;
        if (g->want_ids) {
            const auto* inv64 = reinterpret_cast<const unsigned long long*>(g->inv_bm);
            hipLaunchKernelGGL(k_final_write, dim3(a.fin_G), dim3(kBlock), 0, s, inv64, words, a.fin_wpb,
                               (const unsigned long long*)a.status, g->ctr, g->inv, 1, 1u, ListPub{}, WaveEnd{});
        }
        FGI_HIP(g, hipGetLastError());
        FGI_HIP(g, hipMemcpyAsync(g->ctr_host, g->ctr, sizeof(WaveCtr), hipMemcpyDeviceToHost, s));
        if (timing || stats) FGI_HIP(g, hipEventRecord(g->ev_w1, s));   // the round's end (re-recorded if it goes on)
        FGI_HIP(g, hipStreamSynchronize(s));
        ++syncs;
        const WaveCtr& c = *g->ctr_host;
        if (timing) {
            if (round == 0 && hipEventElapsedTime(&ms, ev[eh], ev[eh + 1]) == hipSuccess) fused_ms += ms;
            if (hipEventElapsedTime(&ms, ev[eh + 2], ev[eh + 3]) == hipSuccess) fused_ms += ms;
            for (int i = 0; i < P; ++i) {
                const unsigned long long kind = c.mid_kind[i];
                if (!kind || hipEventElapsedTime(&ms, ev[2 * i], ev[2 * i + 1]) != hipSuccess) continue;
                if (kind == 2) {
                    pull_ms += ms;
                    ++pull_launches;
                } else {
                    expand_ms += ms;
                    ++expand_launches;
                }
            }
        } else {
            for (int i = 0; i < P; ++i) {
                pull_launches += c.mid_kind[i] == 2;
                expand_launches += c.mid_kind[i] == 1;
            }
        }
        if (c.broken) {
            g->failed = true;
            FGI_HIP(g, hipMemsetAsync(g->gbar, 0, kGbarWords * sizeof(unsigned long long), s));
            FGI_HIP(g, hipStreamSynchronize(s));
            return set_err(g, FGI_EDEVICE, "a fused wave's grid barrier timed out; the graph is unusable until fgi_restore");
        }
        if (c.phase == kPhaseDone) break;
        if (round > 4096) return set_err(g, FGI_EDEVICE, "fused wave: no progress");
        P = (g->opt_fused & kFusedNoPredict) ? 1 : kMidMax;   // more mid levels than predicted
    }
    const WaveCtr& c = *g->ctr_host;
    g->last_mid = (int)c.n_mid;
    if (imm_dev && n_roots) note_words(g);   // immediate roots changed node words
    g->last_wave_n = c.inv;
    g->ids_valid = g->want_ids;
    g->stale_est += c.e_trav + c.e_match;
    if (n_roots) g->last_levels = (int)std::max<uint64_t>(c.n_levels, 1);
    static const bool trace = getenv("FGI_TRACE") != nullptr;
    if (trace)
        fprintf(stderr,
                "[fgi] fused wave: %llu invalidated, %llu levels (%llu pull, %llu by k_level), %llu edges; push levels "
                "in the fused grid: %llu entries / %llu edges; %llu host syncs; head+tail %.3f ms, pull %.3f ms\n",
                (unsigned long long)c.inv, (unsigned long long)c.n_levels, (unsigned long long)c.n_pull,
                (unsigned long long)c.n_mid, (unsigned long long)c.e_trav, (unsigned long long)c.push_f,
                (unsigned long long)c.push_edges, (unsigned long long)syncs, fused_ms, pull_ms);
    if (stats) {
        const uint64_t v = c.inv;
        stats->roots += n_roots;
        stats->levels += c.n_levels;
        stats->v_inv += v;
        stats->e_trav += c.e_trav;
        stats->e_match += c.e_match;
        stats->n_flagged += c.n_flagged;
        stats->pull_levels += c.n_pull;
        stats->pull_edges += c.pull_edges;
        const uint64_t pull_b = pull_level_bytes(c);
        const uint64_t mid_push_b = 20 * c.mid_push_edges + 40 * c.mid_push_f;
        const uint64_t fused_push_b = 20 * c.push_edges + 40 * c.push_f;
        stats->alg_bytes += mid_push_b + fused_push_b + pull_b + 4 * v + 5ull * n_roots;
        float wave_ms = 0;
        hipEventElapsedTime(&wave_ms, g->ev_w0, g->ev_w1);
        stats->kernel_ms += wave_ms;
        stats->expand_ms += expand_ms;
        stats->pull_ms += pull_ms;
        stats->expand_launches += expand_launches;
        stats->expand_bytes += mid_push_b;
        stats->pull_bytes += pull_b;
        stats->pull_launches += pull_launches;
        stats->f_total += c.f_total;
        stats->fused_launches += fused_launches;
        stats->fused_ms += fused_ms;
        stats->fused_push_bytes += fused_push_b;
        stats->host_syncs += syncs;
        stats->total_ms += std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    }
    return FGI_OK;
}

#endif  // FGI_VARIANTS

// The end of a level group: the counters to the host and the host's wait for them. With
// FGI_SPIN_WAIT a one-block kernel writes the counters into fine-grained host memory, then (after a
// system-scope fence) a sequence word the host spins on: the wait ends when that word lands instead of
// when the runtime observes the stream's completion, and no copy command is issued. The spin polls the
// stream every 1,024 pauses, so a fault or a lost write still ends the wait. `mark` records the wave's
// end event before the publish kernel (complete once the word is seen, so its wait costs nothing);
// the publish kernel also leaves its start on the device wall clock at ctr_pub[kPubWords + 1], which
// with WaveCtr::t0 times a wave without stream events (each event record costs the stream ~5 us).
[[maybe_unused]] constexpr uint32_t kPubWords = sizeof(WaveCtr) / 8;
namespace {
// end.ctr (a level group's counters, run_wave): once the wave is over, the counters are zeroed after
// the copy — the next wave starts from them without an init kernel (WaveEnd)
__global__ __launch_bounds__(256) void k_publish(const unsigned long long* __restrict__ src, uint32_t words,
                                                 unsigned long long* dst, unsigned long long seq, WaveEnd end) {
    const bool over = end.ctr && wave_over(end);
    if (threadIdx.x == 0) dst[words + 1] = wall_clock64();
    for (uint32_t i = threadIdx.x; i < words; i += blockDim.x) dst[i] = src[i];
    __threadfence_system();
    __syncthreads();
    if (threadIdx.x == 0) __hip_atomic_store(dst + words, seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
    if (over) {
        unsigned long long* c = reinterpret_cast<unsigned long long*>(end.ctr);
        for (uint32_t i = threadIdx.x; i < (uint32_t)(sizeof(WaveCtr) / 8); i += blockDim.x) c[i] = 0ull;
    }
}

}  // namespace

// src[0, words) into the fine-grained host buffer dst (words + 2 long), waiting for the sequence word
// dst[words]; dst[words + 1] is the publish kernel's start on the device wall clock
// The host's wait for a published sequence word: x86 `pause` while the device works (the common case
// ends within a wave's few hundred us), a hipStreamQuery every 1,024 pauses so a fault or a lost write
// still ends the wait, then sched_yield between polls once the wait has lasted ~10 ms (a rank spinning
// on a peer leaves its core to the collective's proxy threads), and FGI_EDEVICE after
// FGI_WAIT_TIMEOUT_S (default 300) seconds: a collective whose peer never arrives fails the call
// instead of spinning forever.
static fgi_status wait_word(fgi_graph* g, hipStream_t s, const unsigned long long* word, unsigned long long seq) {
    static const double limit_s = [] {
        const char* e = getenv("FGI_WAIT_TIMEOUT_S");
        return e && *e ? atof(e) : 300.0;
    }();
    const auto t0 = std::chrono::steady_clock::now();
    for (uint64_t k = 1; __atomic_load_n(word, __ATOMIC_ACQUIRE) != seq; ++k) {
        if (k < (1u << 15)) {
            __builtin_ia32_pause();
        } else {
            sched_yield();
        }
        if ((k & 1023) == 0) {
            const hipError_t e = hipStreamQuery(s);
            if (e == hipErrorNotReady) {
                if (std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count() > limit_s)
                    return set_err(g, FGI_EDEVICE, "wait: the device did not publish within %.0f s (a collective's peer missing?)",
                                   limit_s);
                continue;
            }
            if (e != hipSuccess) FGI_HIP(g, e);
            if (__atomic_load_n(word, __ATOMIC_ACQUIRE) != seq)
                return set_err(g, FGI_EDEVICE, "publish: the stream completed without the sequence word");
        }
    }
    return FGI_OK;
}

fgi_status publish_wait(fgi_graph* g, hipStream_t s, const unsigned long long* src, uint32_t words, unsigned long long* dst) {
    const unsigned long long seq = ++g->pub_seq;
    hipLaunchKernelGGL(k_publish, dim3(1), dim3(256), 0, s, src, words, dst, seq, WaveEnd{});
    FGI_HIP(g, hipGetLastError());
    FGI_TRY(wait_word(g, s, dst + words, seq));
    g->last_pub_t = dst[words + 1];
    return FGI_OK;
}

// src[0, words) into dst (fine-grained host memory) without waiting: a later publish_wait on the same
// stream covers it (its sequence word lands after this kernel's system-scope fence)
static fgi_status publish_async(fgi_graph* g, hipStream_t s, const unsigned long long* src, uint32_t words, unsigned long long* dst) {
    hipLaunchKernelGGL(k_publish, dim3(1), dim3(256), 0, s, src, words, dst, 0ull, WaveEnd{});
    FGI_HIP(g, hipGetLastError());
    return FGI_OK;
}

// the device wall clock in ms between two stamps (0 if unknown)
float wall_ms(fgi_graph* g, uint64_t t0, uint64_t t1) {
    if (!g->wall_khz && hipDeviceGetAttribute(&g->wall_khz, hipDeviceAttributeWallClockRate, g->device) != hipSuccess)
        g->wall_khz = -1;
    return t1 > t0 && g->wall_khz > 0 ? (float)((double)(t1 - t0) / g->wall_khz) : 0.f;
}

namespace {

// The same wait when the wave's list kernel published the counters itself (launch_final with a ListPub of
// sequence `seq`): the end marker is recorded behind that kernel.
static fgi_status counters_published(fgi_graph* g, hipStream_t s, bool mark, unsigned long long seq) {
    if (mark) FGI_HIP(g, hipEventRecord(g->ev_w1, s));
    FGI_TRY(wait_word(g, s, g->ctr_pub + kPubWords, seq));
    g->last_pub_t = g->ctr_pub[kPubWords + 1];
    memcpy(g->ctr_host, g->ctr_pub, sizeof(WaveCtr));
    if (mark) FGI_HIP(g, hipEventSynchronize(g->ev_w1));
    return FGI_OK;
}

static fgi_status counters_to_host(fgi_graph* g, hipStream_t s, bool mark, const WaveEnd& end = WaveEnd{}) {
#if FGI_SPIN_WAIT
    if (mark) FGI_HIP(g, hipEventRecord(g->ev_w1, s));
    const unsigned long long seq = ++g->pub_seq;
    hipLaunchKernelGGL(k_publish, dim3(1), dim3(256), 0, s, reinterpret_cast<const unsigned long long*>(g->ctr),
                       (uint32_t)kPubWords, g->ctr_pub, seq, end);
    FGI_HIP(g, hipGetLastError());
    FGI_TRY(wait_word(g, s, g->ctr_pub + kPubWords, seq));
    g->last_pub_t = g->ctr_pub[kPubWords + 1];
    memcpy(g->ctr_host, g->ctr_pub, sizeof(WaveCtr));
    if (mark) FGI_HIP(g, hipEventSynchronize(g->ev_w1));
#else
    (void)end;
    FGI_HIP(g, hipMemcpyAsync(g->ctr_host, g->ctr, sizeof(WaveCtr), hipMemcpyDeviceToHost, s));
    if (mark) FGI_HIP(g, hipEventRecord(g->ev_w1, s));
    FGI_HIP(g, hipStreamSynchronize(s));
#endif
    return FGI_OK;
}

}  // namespace

// A completed asynchronous wave's ids stay readable (fgi_wave_wait again) only while its buffer is its own:
// a synchronous wave or a list made on demand that writes the buffer forgets the ticket's results
static void forget_async_results(fgi_graph* g, const uint32_t* buf) {
    for (fgi_graph::AsyncWave& a : g->aw)
        if (!a.busy && a.ticket && ((a.ticket & 1) ? g->inv_alt : g->inv) == buf) a.ticket = 0;
}

// k_collect has nothing to do before a push level that follows a push level (no hot snapshot, no pull
// winners to list). Where the previous wave's directions (what the automatic choice wanted:
// LevelCtr::want) say so, a level group leaves the launch out and pins both levels to push — a cost
// choice, the result does not depend on it; a wave whose shape changed pushes there once, records what
// the rule wanted, and the next wave's plan follows. Bit k of *skip / *pin: level L0 + k. prev_pull: the
// level before L0 pulled (-1: L0 is the wave's first level or the group follows nothing known).
static void plan_collects(const fgi_graph* g, const WaveParams& wp, int L0, int group, int prev_pull, uint32_t* skip,
                          uint32_t* pin) {
    const std::vector<uint8_t>& d = g->last_dirs;
    auto pushes = [&](int l) -> bool {
        if (wp.direction != 0) return wp.direction == 1;
        if (l < L0) return prev_pull == 0;   // only the level just before the group is known (it ran)
        return (size_t)l < d.size() && !d[l];
    };
    *skip = *pin = 0;
    for (int k = 0; k < group && k < 32; ++k) {
        const int l = L0 + k;
        if (pushes(l) && (l == 0 || pushes(l - 1))) {
            *skip |= 1u << k;
            *pin |= 1u << k;
            if (k > 0) *pin |= 1u << (k - 1);
        }
    }
}

fgi_status run_wave(fgi_graph* g, uint32_t n_roots, const uint32_t* roots_dev, const uint8_t* imm_dev,
                    fgi_wave_stats* stats, bool ext_roots) {
    const auto t0 = std::chrono::steady_clock::now();
    forget_async_results(g, g->inv);   // the list goes to g->inv (now, or on demand: ensure_ids)
    hipStream_t s = g->stream;
    static const bool trace = getenv("FGI_TRACE") != nullptr;
    static const bool no_level_events = getenv("FGI_NO_LEVEL_EVENTS") != nullptr;   // measurement only
    const bool timing = (stats != nullptr || trace) && !no_level_events && g->opt_level_timing;
    FGI_TRY(ensure_cstart(g, g->pool_top));
    FGI_TRY(ensure_cls(g));
    // Pull levels need the dependency-list cache. It is built lazily: while it is stale, levels
    // run push-only; once a level group shows a frontier heavy enough to pull, the cache is
    // (re)built and later groups may pull. Small waves (streaming mixes) never pay for it.
    const int direction = g->opt_direction;
    // Beamer's beta rule counts the graph's nodes: the boundary's slots (hub-first labels add K empty ones)
    const WaveParams wp0 = wave_params(g, 0, direction, g->pool_top, g->ext_slots);
    if (wp0.direction == 2 && n_roots) FGI_TRY(ensure_in_lists(g));
    bool allow_pull = wp0.direction != 1 && pull_ready(g, wp0);
    static_assert(sizeof(WaveCtr) % 8 == 0, "WaveCtr is cleared as 64-bit words");
    // fused launches when the wave's directions are settled (lists ready, or push only); a wave that
    // may still have to build the dependency lists part-way runs as level groups below
#if FGI_VARIANTS
    if ((g->opt_fused & kFusedOn) && !g->lbl_K && (allow_pull || wp0.direction == 1)) {   // labels: level groups
        WaveParams wp = wp0;
        if (!allow_pull) wp.direction = 1;
        const fgi_status r = run_wave_fused(g, n_roots, roots_dev, imm_dev, stats, wp, timing, t0);
        if (r != FGI_ENOTSUP) return r;
    }
#endif
    // the previous wave left the counters, statistics and invalidated bitmap zeroed (WaveEnd) and the visit
    // bitmap is clean (fgi_restore swapped in the spare): no init kernel, the roots kernel stamps t0
    const bool clean_start = g->wave_clean && !g->vis_stale && n_roots != 0;
    g->wave_clean = false;
    if (!clean_start)
        hipLaunchKernelGGL(k_wave_init, dim3(kInitBlocks), dim3(kBlock), 0, s, g->ctr, g->blk_stats, g->inv_bm,
                           g->vis_stale ? g->vis_bm : nullptr, (uint64_t)g->bm_words);
    g->vis_stale = false;
    g->coop_clean = false;
#if FGI_PROBE
    {
        void* pp = nullptr;
        if (hipGetSymbolAddress(&pp, HIP_SYMBOL(d_probe)) == hipSuccess) (void)hipMemsetAsync(pp, 0, sizeof(d_probe), s);
    }
#endif
    // the wave's span: stream events with per-level timing, else the device wall clock (spin waits)
    const bool events = timing || (stats && !FGI_SPIN_WAIT);
    if (events) FGI_HIP(g, hipEventRecord(g->ev_w0, s));
    if (n_roots) {
        g->v_dirty = true;
        launch_roots(g, n_roots, roots_dev, imm_dev, 0u, g->n_handles, 0, ext_roots, clean_start ? 1 : 0);
    }
    const auto* node = reinterpret_cast<const unsigned long long*>(g->node);
    // the list kernel and the publish of a group leave the state clean once the wave is over (WaveEnd):
    // only when the list kernel runs (ids wanted, not the measurement-only merged publish)
    static const bool list_pub = getenv("FGI_LIST_PUBLISH") && getenv("FGI_LIST_PUBLISH")[0] == '1';
    const bool merged = FGI_SPIN_WAIT && g->want_ids && list_pub;
    const bool leave_clean = g->want_ids && !merged && FGI_SPIN_WAIT;
    // Levels run in groups between host synchronisations (one ~30 us round trip each); the first
    // group is sized by the previous wave's depth, so a repeated workload syncs once per wave and an
    // overshoot costs only empty levels (two ~2 us launches each). Every group ends with the final
    // collect, so the group that ends the wave needs no further round trip.
    // With the tail (k_wave_tail, default on; FGI_TAIL=0 off for measurement) a group launches the
    // levels up to the previous wave's last pull or large push level and the tail runs the rest.
    static const uint64_t tail_edges = [] {
        const char* e = getenv("FGI_TAIL");
        if (e && e[0] == '0') return 0ull;
        const char* m = getenv("FGI_TAIL_EDGES");
        return m && *m ? (unsigned long long)strtoull(m, nullptr, 10) : (unsigned long long)kTailBlocks * kChunk;   // by the default grid
    }();
    // the tail only where the previous wave had at least two levels past its head (a pull level and the
    // push level after it stay in the group: that level's collect scans the pull's winners, a full-grid
    // job; one small level costs less as a k_level launch than as the tail: profiles/r11_tail_ab.txt)
    const bool use_tail = tail_edges != 0 && g->last_levels >= g->last_head + 2;
    int group = use_tail ? std::min(8, std::max(1, g->last_head)) : std::min(8, std::max(2, g->last_levels));
    int L = 0, head = 1;
    std::vector<uint8_t> dirs;   // this wave's directions (the next wave's collect grids)
    bool dirs_ok = true;
    uint64_t levels = 0, e_trav = 0, f_total = 0, pull_levels = 0;
    double expand_ms = 0, pull_ms = 0, tail_ms = 0;
    uint64_t expand_launches = 0, expand_edges = 0, expand_f = 0, pull_launches = 0, syncs = 0;
    uint64_t tail_launches = 0, tail_edges_run = 0, tail_f = 0;
    bool done = (n_roots == 0);
    bool final_done = false;
    while (!done) {
        const int L0 = L;
        WaveParams wp = wp0;
        if (!allow_pull) wp.direction = 1;
        uint32_t skip = 0, pin = 0;   // left-out collects, levels pinned to push (plan_collects)
        plan_collects(g, wp, L0, group, L0 > 0 ? (g->ctr_host->lvl[(L0 - 1) % kRing].pull ? 1 : 0) : -1, &skip, &pin);
        for (int k = 0; k < group; ++k, ++L) {
            const int buf = L & 1;
            WaveParams wl = wp;
            if (k < 32 && ((pin >> k) & 1u)) wl.direction = 1;
            if (!(k < 32 && ((skip >> k) & 1u)))
                hipLaunchKernelGGL(k_collect, dim3(collect_grid_at(g, wl, L)), dim3(kCollectThreads), 0, s, L, g->ctr, wl,
                                   collect_args(g, g->n_slots, wl, buf), collect_args(g, g->n_slots, wl, buf), ~0ull);
            if (timing) {
                while (g->ev.size() < 2 * (size_t)(L + 1) + 2) {
                    hipEvent_t e;
                    FGI_HIP(g, hipEventCreateWithFlags(&e, event_flags()));
                    g->ev.push_back(e);
                }
                FGI_HIP(g, hipEventRecord(g->ev[2 * L], s));
            }
            hipLaunchKernelGGL(k_level<false>, dim3(wl.grid), dim3(kBlock), 0, s, L, wl, expand_args(g, buf),
                               expand_args(g, buf), pull_args(g, g->n_slots, g->inv_bm), node, g->vis_bm,
                               out_for(g, buf ^ 1, nullptr), out_for(g, buf ^ 1, nullptr), g->ctr, g->blk_stats,
                               g->done, RemoteArgs{}, ~0ull);
            if (timing) FGI_HIP(g, hipEventRecord(g->ev[2 * L + 1], s));
        }
        if (use_tail) {   // the wave's small push levels after the group: one persistent launch
            const TailArgs ta = tail_args(g, L0, L, wp, tail_edges);
            if (timing) {
                while (g->ev.size() < 2 * (size_t)(L + 1) + 4) {
                    hipEvent_t e;
                    FGI_HIP(g, hipEventCreateWithFlags(&e, event_flags()));
                    g->ev.push_back(e);
                }
                FGI_HIP(g, hipEventRecord(g->ev[2 * L], s));
            }
            hipLaunchKernelGGL(k_wave_tail, dim3(tail_blocks(g)), dim3(kBlock), 0, s, ta);
            if (timing) FGI_HIP(g, hipEventRecord(g->ev[2 * L + 1], s));
        }
        // the list kernel may publish the counters itself (one launch fewer), but its last block's
        // system-scope release then writes back the whole list first: 11.6 -> 33.7 us for configs[1]'s
        // k_final_write, 0.231 -> 0.262 ms/step (profiles/r12c); measurement only (FGI_LIST_PUBLISH=1)
        ListPub lp{};
        if (merged) lp = ListPub{g->ctr_pub, ++g->pub_seq, g->done, (uint32_t)kPubWords};
        WaveEnd we{};
        if (leave_clean) {
            we = WaveEnd{g->ctr, L, use_tail ? 1 : 0, g->blk_stats, g->inv_bm, ((uint64_t)g->n_handles + 63) / 64,
                         g->spare_dirty ? g->vis_spare : nullptr};
            g->spare_dirty = false;   // the list kernel clears it whether the wave goes on or not
        }
        FGI_HIP(g, launch_final(g, g->n_handles, g->want_ids, nullptr, lp, we));   // idempotent: repeated if the wave goes on
        final_done = true;
        FGI_HIP(g, hipGetLastError());
        // the wave's end marker rides on the group's synchronisation (re-recorded if the wave goes on):
        // recording it after the wait would cost the call a further device round trip
        if (merged) FGI_TRY(counters_published(g, s, events, lp.seq));
        else FGI_TRY(counters_to_host(g, s, events, we));
        ++syncs;
        if (use_tail && g->ctr_host->broken) {   // half a wave is applied: poisoned until fgi_restore (fgi.h)
            FGI_HIP(g, hipMemsetAsync(g->gbar + kGbarTail, 0, sizeof(unsigned long long), s));
            FGI_HIP(g, hipStreamSynchronize(s));
            g->failed = true;
            return set_err(g, FGI_EDEVICE, "the wave tail's grid barrier timed out (its blocks were not resident together)");
        }
        // the tail ran levels [L, stop); the ring holds the last kRing levels' counters only (the wave's
        // totals come from the device, tail_account), so a tail that ran more leaves the group's
        // per-level figures (timing, trace, head) unread
        const int stop = use_tail ? std::max<int>(L, (int)g->ctr_host->cur) : L;
        const bool ring_ok = stop - L0 < kRing - 4;
        if (use_tail) {
            float ms = 0;
            if (timing && hipEventElapsedTime(&ms, g->ev[2 * L], g->ev[2 * L + 1]) == hipSuccess) tail_ms += ms;
            ++tail_launches;
            for (int l = std::max(L, stop - (kRing - 4)); trace && l < stop; ++l) {
                const LevelCtr& lc = g->ctr_host->lvl[l % kRing];
                fprintf(stderr, "[fgi] level %d push (tail): frontier %llu edges %llu chunk x%llu\n", l,
                        (unsigned long long)lvl_F(lc), (unsigned long long)lvl_T(lc), (unsigned long long)lc.mult);
            }
        }
        if (ring_ok) {
            dirs.resize(std::max<size_t>(dirs.size(), (size_t)stop), 0);
            for (int l = L0; l < L; ++l) dirs[l] = g->ctr_host->lvl[l % kRing].want ? 1 : 0;
        } else {
            dirs_ok = false;
        }
        for (int l = L0; l < L && ring_ok; ++l) {
            const LevelCtr& lc = g->ctr_host->lvl[l % kRing];
            if (lvl_F(lc) && (lc.pull || lvl_T(lc) > tail_edges)) head = l + (lc.pull ? tail_head_after_pull() : 1);
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
            const uint64_t lF = lvl_F(lc), lT = lvl_T(lc);
            if (lF && !use_tail) {
                ++levels;
                e_trav += lT;
                f_total += lF;
                if (lc.pull) {
                    ++pull_levels;
                } else {
                    expand_edges += lT;
                    expand_f += lF;
                }
            }
            if (trace)
                fprintf(stderr, "[fgi] level %d %s: frontier %llu edges %llu chunk x%llu k_level %.3f ms\n", l,
                        lc.pull ? "pull" : "push", (unsigned long long)lF, (unsigned long long)lT,
                        (unsigned long long)lc.mult, ms);
        }
#if FGI_PROBE
        if (trace) print_probe(g, L0, L);
#endif
        if (use_tail && trace && stop > L)
            fprintf(stderr, "[fgi] tail: levels %d..%d in one launch\n", L, stop - 1);
        L = stop;
        done = lvl_F(g->ctr_host->lvl[L % kRing]) == 0;
        group = 4;
        // also when the wave is already done (its level groups are sized from the previous wave's
        // depth, so a repeated wave after a mutation finishes in one group): the next wave pulls
        if (!allow_pull && wp0.direction == 0) {
            bool heavy = use_tail && g->ctr_host->t_max > wp.pull_threshold;
            for (int l = L0; l <= L && ring_ok; ++l) heavy |= lvl_T(g->ctr_host->lvl[l % kRing]) > wp.pull_threshold;
            if (heavy) {
                g->lists_wanted = true;
                FGI_TRY(ensure_in_lists(g));
                allow_pull = pull_ready(g, wp0);
            }
        }
    }
    if (!final_done) {   // no roots
        FGI_HIP(g, launch_final(g, g->n_handles, g->want_ids));
        FGI_HIP(g, hipGetLastError());
        FGI_TRY(counters_to_host(g, s, events));
    }
    if (use_tail && final_done) {   // the device's totals (tail_account)
        const WaveCtr& c = *g->ctr_host;
        levels = c.n_levels;
        e_trav = c.e_trav;
        f_total = c.f_total;
        pull_levels = c.n_pull;
        tail_edges_run = c.mid_push_edges;
        tail_f = c.mid_push_f;
        expand_edges = c.push_edges - c.mid_push_edges;
        expand_f = c.push_f - c.mid_push_f;
    }
    if (imm_dev && n_roots) note_words(g);   // immediate roots changed node words
    // the last group's list kernel and publish saw the wave over (the host's loop ends on the same test)
    g->wave_clean = leave_clean && final_done;
    g->last_wave_n = g->ctr_host->inv;
    g->ids_valid = g->want_ids;
    g->inv_cur = g->inv;
    // entries this wave made stale: the invalidated nodes' rows and the matched entries pointing at
    // them (fgi_prune_step's trigger)
    g->stale_est += e_trav + g->ctr_host->e_match;
    if (n_roots) {
        g->last_levels = (int)std::max<uint64_t>(levels, 1);
        g->last_head = head;
        if (dirs_ok) g->last_dirs.swap(dirs);
        else g->last_dirs.clear();
    }
    const WaveCtr& c = *g->ctr_host;
    if (trace)
        fprintf(stderr,
                "[fgi] wave: %llu invalidated; pull: live %llu, survivors %llu, queued %llu, dependencies "
                "examined %llu, winners %llu\n",
                (unsigned long long)c.inv, (unsigned long long)c.pull_live, (unsigned long long)c.pull_surv,
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
        // node-word gather 8; per frontier entry: fr_off 4 + escan 8 read, fr_off 4 + fr_len 4 +
        // escan 8 written by the producer, its row length and offset 12 gathered. Final collect:
        // 4 B per invalidated node. Per root 5.
        const uint64_t push_b = 20 * (expand_edges + tail_edges_run) + 40 * (expand_f + tail_f);
        const uint64_t pull_b = pull_level_bytes(c);
        stats->alg_bytes += push_b + pull_b + 4 * v + 5ull * n_roots;
        float wave_ms = 0;
        if (events) {
            hipEventElapsedTime(&wave_ms, g->ev_w0, g->ev_w1);
        } else {
            wave_ms = wall_ms(g, c.t0, g->last_pub_t);
        }
        stats->kernel_ms += wave_ms;
        stats->expand_ms += expand_ms;
        stats->pull_ms += pull_ms;
        stats->expand_launches += expand_launches;
        stats->expand_bytes += 20 * expand_edges + 40 * expand_f;
        stats->fused_launches += tail_launches;
        stats->fused_ms += tail_ms;
        stats->fused_push_bytes += 20 * tail_edges_run + 40 * tail_f;
        stats->pull_bytes += pull_b;
        stats->pull_launches += pull_launches;
        stats->f_total += f_total;
        stats->host_syncs += syncs + (final_done ? 0 : 1);
        stats->total_ms += std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    }
    return FGI_OK;
}

// ---- asynchronous waves -------------------------------------------------------------------------------
// fgi_invalidate_async queues one whole wave — init, roots, a level group sized by the previous wave
// (its pull levels and large push levels), the tail with every remaining level (all = 1: no level is
// left to a second group, so the wave is complete in its queue), the final collect into the ticket's
// id buffer and a publish of the counters into the ticket's host buffer — and returns. A wave whose
// pull levels outnumber the group runs its later pull levels as push levels inside the tail: the
// result is the same, only slower, and the next wave's group is sized from this one. The next call's
// host work (restore, root upload, the launches) thus overlaps the device's previous wave
// (ComputedExt.WhenInvalidated: the caller awaits the wave instead of blocking on it).
fgi_status run_wave_async(fgi_graph* g, uint32_t n_roots, const uint32_t* roots_dev, const uint8_t* imm_dev,
                          uint64_t* ticket) {
    const uint64_t t = g->next_ticket;
    fgi_graph::AsyncWave& a = g->aw[t & 1];
    if (a.busy) FGI_TRY(wave_wait(g, a.ticket, nullptr, nullptr, nullptr));   // at most two in flight
    const auto t0 = std::chrono::steady_clock::now();
    hipStream_t s = g->stream;
    if (!g->apub[0]) {
        for (int k = 0; k < 2; ++k)
            if (hipHostMalloc(reinterpret_cast<void**>(&g->apub[k]), sizeof(WaveCtr) + 128, hipHostMallocCoherent) != hipSuccess)
                return set_err(g, FGI_ENOMEM, "async wave: published counters");
        for (int k = 0; k < 2; ++k) memset(g->apub[k], 0, sizeof(WaveCtr) + 128);
    }
    if (!g->inv_alt) FGI_HIP(g, hipMalloc(reinterpret_cast<void**>(&g->inv_alt), (size_t)g->n_handles * 4));
    FGI_TRY(ensure_cstart(g, g->pool_top));
    FGI_TRY(ensure_cls(g));
    const WaveParams wp0 = wave_params(g, 0, g->opt_direction, g->pool_top, g->ext_slots);
    // the dependency lists a pull level needs are built here, before anything is queued, once a wave
    // has shown a frontier heavy enough to pull (as run_wave builds them after such a group)
    if (n_roots && wp0.direction != 1 && (g->lists_wanted || wp0.direction == 2)) FGI_TRY(ensure_in_lists(g));
    WaveParams wp = wp0;
    if (!(wp0.direction != 1 && pull_ready(g, wp0))) wp.direction = 1;
    // as run_wave: no init kernel after a wave that left the state clean (the queue is stream-ordered)
    const bool clean_start = g->wave_clean && !g->vis_stale && n_roots != 0;
    g->wave_clean = false;
    if (!clean_start)
        hipLaunchKernelGGL(k_wave_init, dim3(kInitBlocks), dim3(kBlock), 0, s, g->ctr, g->blk_stats, g->inv_bm,
                           g->vis_stale ? g->vis_bm : nullptr, (uint64_t)g->bm_words);
    g->vis_stale = false;
    g->coop_clean = false;
    const auto* node = reinterpret_cast<const unsigned long long*>(g->node);
    // the previous wave's levels in the group (up to 8), its head at least; the tail runs the rest
    int group = std::min(8, std::max(std::max(1, g->last_head), g->last_levels));
    if (n_roots) {
        g->v_dirty = true;
        launch_roots(g, n_roots, roots_dev, imm_dev, 0u, g->n_handles, 0, true, clean_start ? 1 : 0);
        uint32_t skip = 0, pin = 0;
        plan_collects(g, wp, 0, group, -1, &skip, &pin);
        for (int L = 0; L < group; ++L) {
            const int buf = L & 1;
            WaveParams wl = wp;
            if (L < 32 && ((pin >> L) & 1u)) wl.direction = 1;
            if (!(L < 32 && ((skip >> L) & 1u)))
                hipLaunchKernelGGL(k_collect, dim3(collect_grid_at(g, wl, L)), dim3(kCollectThreads), 0, s, L, g->ctr, wl,
                                   collect_args(g, g->n_slots, wl, buf), collect_args(g, g->n_slots, wl, buf), ~0ull);
            hipLaunchKernelGGL(k_level<false>, dim3(wl.grid), dim3(kBlock), 0, s, L, wl, expand_args(g, buf),
                               expand_args(g, buf), pull_args(g, g->n_slots, g->inv_bm), node, g->vis_bm,
                               out_for(g, buf ^ 1, nullptr), out_for(g, buf ^ 1, nullptr), g->ctr, g->blk_stats,
                               g->done, RemoteArgs{}, ~0ull);
        }
        TailArgs ta = tail_args(g, 0, group, wp, ~0ull);
        ta.all = 1;
        hipLaunchKernelGGL(k_wave_tail, dim3(tail_blocks(g)), dim3(kBlock), 0, s, ta);
    } else {
        group = 0;
    }
    uint32_t* out = (t & 1) ? g->inv_alt : g->inv;
    // the queue runs every level (the tail's `all`), so the wave is over after it: its list kernel and
    // publish leave the state clean for the next wave (WaveEnd)
    const WaveEnd we{g->ctr, group, 1, g->blk_stats, g->inv_bm, ((uint64_t)g->n_handles + 63) / 64,
                     g->spare_dirty ? g->vis_spare : nullptr};
    g->spare_dirty = false;
    FGI_HIP(g, launch_final(g, g->n_handles, true, out, ListPub{}, we));
    const unsigned long long seq = ++g->apub_seq;
    hipLaunchKernelGGL(k_publish, dim3(1), dim3(256), 0, s, reinterpret_cast<const unsigned long long*>(g->ctr),
                       (uint32_t)kPubWords, g->apub[t & 1], seq, we);
    FGI_HIP(g, hipGetLastError());
    g->wave_clean = true;   // once the queue has run (every later launch is stream-ordered after it)
    if (imm_dev && n_roots) note_words(g);   // immediate roots change node words (fgi_restore copies them back)
    a.ticket = t;
    a.seq = seq;
    a.n_roots = n_roots;
    a.imm = imm_dev != nullptr;
    a.group = group;
    a.t0 = t0;
    a.busy = true;
    g->ids_valid = false;
    g->next_ticket = t + 1;
    if (ticket) *ticket = t;
    return FGI_OK;
}

// fgi_invalidate_async with roots in host memory: the ticket parity's pinned buffer takes a copy (its
// previous wave, two tickets back, has completed before its slot is reused: run_wave_async waits for it)
// and a stream-ordered copy moves it to the device, so the call still returns without waiting.
fgi_status run_wave_async_host(fgi_graph* g, uint32_t n_roots, const uint32_t* roots, const uint8_t* imm, uint64_t* ticket) {
    const uint64_t t = g->next_ticket;
    const int k = (int)(t & 1);
    fgi_graph::AsyncWave& a = g->aw[k];
    if (a.busy) FGI_TRY(wave_wait(g, a.ticket, nullptr, nullptr, nullptr));   // its staged roots are consumed
    const uint64_t need = std::max<uint64_t>(n_roots, 1);
    if (g->ar_cap[k] < need) {
        if (g->ar_h[k]) (void)hipHostFree(g->ar_h[k]);
        if (g->ar_d[k]) (void)hipFree(g->ar_d[k]);
        g->ar_h[k] = g->ar_d[k] = nullptr;
        g->ar_cap[k] = 0;
        const uint64_t cap = std::max<uint64_t>(need, 4096);
        // roots (4 B each) then the immediately flags (1 B each), in one pinned and one device buffer
        if (hipHostMalloc(reinterpret_cast<void**>(&g->ar_h[k]), cap * 5, hipHostMallocDefault) != hipSuccess ||
            hipMalloc(reinterpret_cast<void**>(&g->ar_d[k]), cap * 5) != hipSuccess)
            return set_err(g, FGI_ENOMEM, "async wave: root staging");
        g->ar_cap[k] = cap;
    }
    uint8_t* imm_h = reinterpret_cast<uint8_t*>(g->ar_h[k] + g->ar_cap[k]);
    uint8_t* imm_d = reinterpret_cast<uint8_t*>(g->ar_d[k] + g->ar_cap[k]);
    if (n_roots) {
        memcpy(g->ar_h[k], roots, (size_t)n_roots * 4);
        FGI_HIP(g, hipMemcpyAsync(g->ar_d[k], g->ar_h[k], (size_t)n_roots * 4, hipMemcpyHostToDevice, g->stream));
        if (imm) {
            memcpy(imm_h, imm, n_roots);
            FGI_HIP(g, hipMemcpyAsync(imm_d, imm_h, n_roots, hipMemcpyHostToDevice, g->stream));
        }
    }
    return run_wave_async(g, n_roots, g->ar_d[k], imm && n_roots ? imm_d : nullptr, ticket);
}

fgi_status wave_wait(fgi_graph* g, uint64_t ticket, uint64_t* out_n, const uint32_t** ids_dev, fgi_wave_stats* stats) {
    if (ticket == 0 || ticket >= g->next_ticket) return set_err(g, FGI_EINVAL, "no wave with ticket %llu", (unsigned long long)ticket);
    // the older one first: waves complete in ticket order
    fgi_graph::AsyncWave& o = g->aw[(ticket + 1) & 1];
    if (o.busy && o.ticket < ticket) FGI_TRY(wave_wait(g, o.ticket, nullptr, nullptr, nullptr));
    fgi_graph::AsyncWave& a = g->aw[ticket & 1];
    if (!a.busy || a.ticket != ticket) {   // already waited for: its count, its buffer (if still its own)
        if (a.ticket != ticket)
            return set_err(g, FGI_EINVAL, "the results of wave %llu are gone (a later wave took its buffers)",
                           (unsigned long long)ticket);
        if (out_n) *out_n = a.n_inv;
        if (ids_dev) *ids_dev = (ticket & 1) ? g->inv_alt : g->inv;
        return FGI_OK;
    }
    unsigned long long* pub = g->apub[ticket & 1];
    const fgi_status ws = wait_word(g, g->stream, pub + kPubWords, a.seq);
    if (ws != FGI_OK) {
        // the wave may still be running (a timeout) or the stream failed: its buffers stay its own and the
        // graph is poisoned until fgi_restore (which orders its copies after the wave on the stream)
        g->failed = true;
        return ws;
    }
    a.busy = false;
    const WaveCtr& c = *reinterpret_cast<const WaveCtr*>(pub);
    if (c.broken) {
        // the wave's tail left at a timed-out grid barrier: the wave is half applied (as run_wave's level
        // groups, fgi.h). The other wave in flight, queued behind it, is drained first (its tail starts from
        // the misaligned barrier counter and times out too), then the barrier word is reset.
        g->aw[0].busy = g->aw[1].busy = false;
        FGI_HIP(g, hipStreamSynchronize(g->stream));
        FGI_HIP(g, hipMemsetAsync(g->gbar + kGbarTail, 0, sizeof(unsigned long long), g->stream));
        FGI_HIP(g, hipStreamSynchronize(g->stream));
        g->failed = true;
        return set_err(g, FGI_EDEVICE, "wave %llu: the wave tail's grid barrier timed out (its blocks were not resident "
                                       "together); the graph is unusable until fgi_restore", (unsigned long long)ticket);
    }
    // the wave's totals from the device (tail_account); the group's levels from the ring while it has not
    // rolled over (the next wave's group size)
    const uint64_t levels = c.n_levels, e_trav = c.e_trav, f_total = c.f_total, pull_levels = c.n_pull;
    const uint64_t push_e = c.push_edges, push_f = c.push_f;
    uint64_t head = (uint64_t)std::max(1, g->last_head);
    const uint64_t stop = a.group ? std::max<uint64_t>((uint64_t)a.group, c.cur) : 0;
    if (stop < (uint64_t)kRing - 4) {
        head = 1;
        std::vector<uint8_t> dirs(stop, 0);   // the next waves' launch plans (plan_collects); the tail's levels push
        for (uint64_t l = 0; l < (uint64_t)a.group; ++l) {
            const LevelCtr& lc = c.lvl[l % kRing];
            dirs[l] = lc.want ? 1 : 0;
            if (lvl_F(lc) && (lc.pull || lvl_T(lc) > (uint64_t)tail_blocks(g) * kChunk))
                head = l + (lc.pull ? tail_head_after_pull() : 1);
        }
        if (a.n_roots) g->last_dirs.swap(dirs);
    } else if (a.n_roots) {
        g->last_dirs.clear();
    }
    a.n_inv = c.inv;
    g->last_wave_n = c.inv;
    g->inv_cur = (ticket & 1) ? g->inv_alt : g->inv;
    g->ids_valid = true;
    g->stale_est += e_trav + c.e_match;
    if (a.n_roots) {
        g->last_levels = (int)std::max<uint64_t>(levels, 1);
        g->last_head = (int)head;
        if (c.t_max > g->pool_top / (uint64_t)std::max(1, g->opt_pull_alpha)) g->lists_wanted = true;
    }
    if (out_n) *out_n = c.inv;
    if (ids_dev) *ids_dev = g->inv_cur;
    if (stats) {
        stats->roots += a.n_roots;
        stats->levels += levels;
        stats->v_inv += c.inv;
        stats->e_trav += e_trav;
        stats->e_match += c.e_match;
        stats->n_flagged += c.n_flagged;
        stats->pull_levels += pull_levels;
        stats->pull_edges += c.pull_edges;
        stats->alg_bytes += 20 * push_e + 40 * push_f + pull_level_bytes(c) + 4 * c.inv + 5ull * a.n_roots;
        stats->kernel_ms += wall_ms(g, c.t0, pub[kPubWords + 1]);
        stats->f_total += f_total;
        stats->host_syncs += 1;
        stats->pull_pushed += c.pull_pushed;
        stats->total_ms += std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - a.t0).count();
    }
    return FGI_OK;
}

fgi_status drain_async(fgi_graph* g) {
    for (int k = 0; k < 2; ++k) {
        fgi_graph::AsyncWave& x = g->aw[k];
        fgi_graph::AsyncWave& y = g->aw[k ^ 1];
        if (x.busy && (!y.busy || x.ticket < y.ticket)) FGI_TRY(wave_wait(g, x.ticket, nullptr, nullptr, nullptr));
    }
    for (int k = 0; k < 2; ++k)
        if (g->aw[k].busy) FGI_TRY(wave_wait(g, g->aw[k].ticket, nullptr, nullptr, nullptr));
    return FGI_OK;
}

fgi_status ensure_ids(fgi_graph* g) {
    if (g->ids_valid) return FGI_OK;
    // the bitmap of the last wave is intact until the next wave starts: list it now
    if (!g->inv_cur) g->inv_cur = g->inv;
    forget_async_results(g, g->inv_cur);
    FGI_HIP(g, launch_final(g, g->n_handles, true, g->inv_cur));
    FGI_HIP(g, hipStreamSynchronize(g->stream));
    g->ids_valid = true;
    return FGI_OK;
}

// ---- multi-GPU wave -------------------------------------------------------------------------------
// The partitioned wave, one call per rank: levels in lockstep, collectives through the rank's
// PartComm (RCCL over xGMI with one process per GPU, or device copies between the graphs of an
// in-process group, one host thread per rank — the same level sequence either way). A pull level
// all-gathers the invalidated bitmap, pulls, and all-reduces {frontier, frontier edges} of the next
// level, which decide push vs pull (Beamer's alpha / beta rules, as run_wave) and termination. A
// push level synchronises the host once: its counts all-gather (payload sizes, then the payloads;
// the received targets are applied) also carries every rank's local next {F, T}. The targets
// forwarded bound the winners they add, so F + sent >= the next frontier (0: the wave is done) and T
// scales by the local edges per winner — direction is a cost choice, the result does not depend on
// it. A level whose winners are all remote falls back to the all-reduce (termination is exact).
// The plan's key: a plan follows the levels of the wave it was learnt from; any mutation or option
// change since then starts a new one. Every rank computes it from its own calls, which are the same on
// all ranks (the start all-reduce also checks that every rank can follow its plan).
uint64_t part_plan_key(const fgi_graph* g) {
    return (uint64_t)g->mut_epoch * 1000003ull ^ ((uint64_t)g->opt_direction << 56) ^ ((uint64_t)g->opt_pull_alpha << 40) ^
           ((uint64_t)g->opt_pull_beta << 24) ^ ((uint64_t)g->opt_front_exchange << 20) ^ (uint64_t)g->uin_epoch;
}

// A planned partitioned wave (every rank follows the previous wave's directions, g->part_plan): the
// levels' collectives are stream-ordered and fixed in size — a pull level all-gathers the whole
// invalidated bitmap, a push level moves its forwarded targets in fixed-size buckets (what does not
// fit waits for the next push level: a later visit of a node changes nothing, so the result is the
// same) — so the host queues the whole plan and waits once, at a closing all-reduce of the next
// frontier, the ids still waiting and every level's {F, T}. If that finds work left, push levels
// follow, planned the same way, until none is left. The direction of a level is a cost choice:
// results do not depend on the plan.
// a partitioned wave times itself with stream events only when per-level timing is on (or without the
// spin wait); otherwise by the device wall clock between WaveCtr::t0 and the wave's last publish
static inline bool part_events(const fgi_graph* g) { return g->opt_level_timing != 0 || !FGI_SPIN_WAIT; }

static fgi_status run_part_planned(fgi_graph* g, const PartView& pv, const WaveParams& wp, const PartBuckets& pb,
                                   uint32_t n_roots, fgi_wave_stats* stats, std::chrono::steady_clock::time_point t0) {
    hipStream_t s = g->stream;
    const bool coll = pv.world > 1 || g->opt_part_coll;
    const auto* node = reinterpret_cast<const unsigned long long*>(g->node);
    const RemoteArgs ra{pv.base, pv.n_local, pv.block, pv.world, pv.ver_all, pv.sent_bm, pv.send_buf, pv.send_cnt};
    // one rank without collectives: the pull levels probe the invalidated bitmap itself (no copy into
    // front_global per pull level) when its hot snapshot sits where the partition's would (the same
    // word count: no detached handles)
    const bool alias = !coll && g->hot_w0 == g->bm_words;
    const uint32_t* front = alias ? g->inv_bm : pv.front_global;
    uint32_t* const hot_base = alias ? g->inv_bm : pv.front_global;
    if (coll) {
        FGI_HIP(g, hipMemsetAsync(pv.send_cnt, 0, (size_t)pv.world * 8, s));
        FGI_HIP(g, hipMemsetAsync(pb.cur, 0, (size_t)pv.world * 8, s));
    }
    std::vector<uint8_t> plan = g->part_plan;
    const bool timing = g->opt_level_timing != 0;
    FGI_HIP(g, ensure_events(g, 2 * (size_t)kPlanMax + 2));
    uint64_t syncs = 0, rounds = 0;
    int L = 0;
    std::vector<uint64_t> glob, plan_ft;
    double pull_ms = 0, expand_ms = 0;
    uint64_t pull_launches = 0, expand_launches = 0;
    uint64_t levels = 0, e_trav = 0, f_total = 0, push_edges = 0, push_f = 0, pull_levels = 0;
    while (true) {
        const int L0 = L;
        for (size_t k = 0; k < plan.size(); ++k, ++L) {
            const bool pull = plan[k] != 0;
            const int buf = L & 1;
            const int e = 2 * (L - L0);
            if (pull) {
                FGI_HIP(g, hipMemsetD32Async(reinterpret_cast<hipDeviceptr_t>(&g->ctr->lvl[L % kRing].pull), 1, 1, s));
                if (coll) FGI_TRY(part_allgather_front_async(g));
                else if (!alias)
                    FGI_HIP(g, hipMemcpyAsync(pv.front_global, g->inv_bm, (size_t)pv.block / 32 * 4, hipMemcpyDeviceToDevice, s));
            }
            CollectArgs ca = collect_args(g, pv.n_local, wp, buf);
            ca.inv = front;   // hot heads are global ids
            ca.hot_bm = hot_base + g->hot_w0;
            ca.sum_bm = reinterpret_cast<unsigned long long*>(g->sum_bm);   // over front_global (part init)
            ca.n64 = pv.front_words_global / 2;
            hipLaunchKernelGGL(k_collect, dim3(collect_grid(g, wp)), dim3(kCollectThreads), 0, s, L, g->ctr, wp, ca, ca,
                               ~0ull);
            if (timing) FGI_HIP(g, hipEventRecord(g->ev[e], s));
            hipLaunchKernelGGL(k_level<true>, dim3(wp.grid), dim3(kBlock), 0, s, L, wp, expand_args(g, buf),
                               expand_args(g, buf), pull_args(g, g->n_slots, front), node, g->vis_bm,
                               out_for(g, buf ^ 1, nullptr), out_for(g, buf ^ 1, nullptr), g->ctr, g->blk_stats, g->done,
                               ra, ~0ull);
            if (timing) FGI_HIP(g, hipEventRecord(g->ev[e + 1], s));
            if (!pull && coll) {
                hipLaunchKernelGGL(k_a2a_pack, dim3(pv.world), dim3(kBlock), 0, s, pv.rank, pb.C, pv.send_buf, pv.block,
                                   pv.send_cnt, pb.cur, pb.send);
                FGI_TRY(part_alltoall_async(g));
                const uint64_t n = (uint64_t)pv.world * (pb.C - 1);
                hipLaunchKernelGGL(k_apply_recv, dim3(std::min<uint64_t>((n + kBlock - 1) / kBlock, (uint64_t)g->n_cu * 8)),
                                   dim3(kBlock), 0, s, L, n, pb.recv, pv.base, node, g->vis_bm, out_for(g, buf ^ 1, nullptr),
                                   g->ctr, g->blk_stats, g->done, pb.C);
            }
            FGI_HIP(g, hipGetLastError());
        }
        // the final collect may be repeated if the wave goes on (it only reads the invalidated bitmap)
        FGI_HIP(g, launch_final(g, pv.n_local));
#if FGI_SPIN_WAIT
        // the counters ride to fine-grained host memory ahead of the all-reduce's published result
        FGI_TRY(publish_async(g, s, reinterpret_cast<const unsigned long long*>(g->ctr), kPubWords, g->ctr_pub));
#else
        FGI_HIP(g, hipMemcpyAsync(g->ctr_host, g->ctr, sizeof(WaveCtr), hipMemcpyDeviceToHost, s));
#endif
        // the first round's levels decide the next wave's plan: their {F, T} ride on the all-reduce
        const int K = rounds == 0 ? L - L0 : 0;
        const uint32_t cnt = 2 + 2 * (uint32_t)K;
        hipLaunchKernelGGL(k_part_tail, dim3(1), dim3(64), 0, s, g->ctr, L0, L, coll ? pv.world : 0u, pv.send_cnt, pb.cur,
                           pb.red, K);
        glob.assign(cnt, 0);
        if (part_events(g)) FGI_HIP(g, hipEventRecord(g->ev_w1, s));   // the round's end (re-recorded if the wave goes on)
        FGI_TRY(part_allreduce_sum(g, pb.red, glob.data(), cnt));   // the wave's one host synchronisation
#if FGI_SPIN_WAIT
        memcpy(g->ctr_host, g->ctr_pub, sizeof(WaveCtr));
#endif
        if (timing) FGI_HIP(g, hipEventSynchronize(g->ev_w1));       // complete already: the level events too
        if (rounds == 0) plan_ft.assign(glob.begin() + 2, glob.end());
        ++syncs;
        ++rounds;
        for (int l = L0; l < L; ++l) {   // the round's levels (a round has at most kPlanMax < kRing)
            const LevelCtr& lc = g->ctr_host->lvl[l % kRing];
            const uint64_t F = lvl_F(lc), T = lvl_T(lc);
            // a level counts as the host-driven loop counts it: if any rank had a frontier (round 0: the
            // all-reduced F; later rounds, push levels: this rank's); a plan's surplus levels do not
            const bool ran = rounds == 1 ? plan_ft[2 * (l - L0)] != 0 : F != 0;
            if (lc.pull && ran) ++pull_levels;
            if (ran) ++levels;
            if (F) {
                e_trav += T;
                f_total += F;
                if (!lc.pull) {
                    push_edges += T;
                    push_f += F;
                }
            }
            float ms = 0;
            if (!timing || hipEventElapsedTime(&ms, g->ev[2 * (l - L0)], g->ev[2 * (l - L0) + 1]) != hipSuccess) continue;
            if (lc.pull) {
                pull_ms += ms;
                ++pull_launches;
            } else {
                expand_ms += ms;
                ++expand_launches;
            }
        }
        if (glob[0] == 0 && glob[1] == 0) break;
        // work left (a longer wave than the plan, or ids waiting in send_buf): push levels; each moves
        // at least one waiting id per peer, so the wave ends
        if (rounds > (1u << 20)) return set_err(g, FGI_EDEVICE, "planned partitioned wave: no end in sight");
        plan.assign(16, 0);
    }
    // the next wave's plan: Beamer's rules over this wave's global levels (as the host-driven loop
    // decides them), computed alike on every rank from the all-reduced {F, T}
    {
        std::vector<uint8_t> next;
        bool last_pull = false;
        const bool allow_pull = g->part_plan_pull;
        for (size_t l = 0; 2 * l + 1 < plan_ft.size() && next.size() < kPlanMax; ++l) {
            const uint64_t F = plan_ft[2 * l], T = plan_ft[2 * l + 1];
            if (F == 0) break;
            const bool pull = allow_pull && T != 0 &&
                              (wp.direction == 2 ||
                               (wp.direction == 0 && (T > wp.pull_threshold || (last_pull && F > wp.stay_pull_f))));
            next.push_back(pull ? 1 : 0);
            last_pull = pull;
        }
        if (!next.empty()) g->part_plan = next;
    }
    const WaveCtr& c = *g->ctr_host;
    g->last_wave_n = c.inv;
    g->ids_valid = true;
    if (stats) {
        uint64_t sent_total = 0;
        if (coll) {
            std::vector<unsigned long long> sc(pv.world, 0);
            FGI_HIP(g, hipMemcpy(sc.data(), pv.send_cnt, (size_t)pv.world * 8, hipMemcpyDeviceToHost));
            for (uint32_t q = 0; q < pv.world; ++q) sent_total += sc[q];
        }
        const uint64_t v = c.inv;
        stats->roots += n_roots;
        stats->levels += levels;
        stats->v_inv += v;
        stats->e_trav += e_trav;
        stats->e_match += c.e_match;
        stats->n_flagged += c.n_flagged;
        stats->remote_msgs += sent_total;
        const uint64_t pull_b = pull_level_bytes(c);
        stats->alg_bytes += 20 * push_edges + 40 * push_f + pull_b + 4 * v + 8 * sent_total + 5ull * n_roots;
        stats->pull_levels += pull_levels;
        stats->pull_edges += c.pull_edges;
        stats->pull_ms += pull_ms;
        stats->pull_bytes += pull_b;
        stats->pull_launches += pull_launches;
        float wave_ms = 0;
        if (part_events(g)) hipEventElapsedTime(&wave_ms, g->ev_w0, g->ev_w1);
        else wave_ms = wall_ms(g, c.t0, g->last_pub_t);
        stats->kernel_ms += wave_ms;
        stats->expand_ms += expand_ms;
        stats->expand_launches += expand_launches;
        stats->expand_bytes += 20 * push_edges + 40 * push_f;
        stats->f_total += f_total;
        stats->host_syncs += syncs + (coll ? 1 : 0);   // + the start all-reduce
        stats->total_ms += std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    }
    return FGI_OK;
}

fgi_status run_part_wave(fgi_graph* g, uint32_t n_roots, const uint32_t* roots_dev, const uint8_t* imm_dev,
                         fgi_wave_stats* stats) {
    PartView pv;
    if (!part_view(g, &pv)) return set_err(g, FGI_ESTATE, "partition not initialised");
    const auto t0 = std::chrono::steady_clock::now();
    hipStream_t s = g->stream;
    FGI_TRY(part_ensure_lists(g));
    FGI_TRY(ensure_cstart(g, g->pool_top));
    FGI_TRY(ensure_cls(g));
    // one rank: nothing is remote, the collectives are identities (skipped unless FGI_OPT_PART_COLLECTIVES)
    const bool coll = pv.world > 1 || g->opt_part_coll;
    if (coll) FGI_HIP(g, hipMemsetAsync(pv.sent_bm, 0, pv.sent_words * 4, s));
    g->wave_clean = false;   // this path dirties the wave state (run_wave re-inits)
    if (coll) FGI_TRY(part_front_reset(g));
    hipLaunchKernelGGL(k_wave_init, dim3(kInitBlocks), dim3(kBlock), 0, s, g->ctr, g->blk_stats, g->inv_bm,
                       g->vis_stale ? g->vis_bm : nullptr, (uint64_t)g->bm_words);
    g->vis_stale = false;
    g->coop_clean = false;
    while (g->ev.size() < 2) {
        hipEvent_t e;
        FGI_HIP(g, hipEventCreateWithFlags(&e, event_flags()));
        g->ev.push_back(e);
    }
    // the wave's span: stream events with per-level timing, else the device wall clock (spin waits:
    // WaveCtr::t0 from k_wave_init, the end from the last publish)
    if (part_events(g)) FGI_HIP(g, hipEventRecord(g->ev_w0, s));
    g->v_dirty = true;
    if (n_roots) launch_roots(g, n_roots, roots_dev, imm_dev, pv.base, pv.n_local, 1);
    if (imm_dev && n_roots) note_words(g);
    FGI_HIP(g, hipGetLastError());
    const auto* node = reinterpret_cast<const unsigned long long*>(g->node);
    // one all-reduce of {local edges, level-0 frontier, its edges, ranks without pull lists, ranks
    // that can follow the previous wave's plan, the partition codes' fingerprint and its square}
    const WaveParams wp0 = wave_params(g, 1, g->opt_direction, g->pool_top, pv.n_global);
    const bool can_pull = wp0.direction != 1 && pull_ready(g, wp0);
    const PartBuckets pb = part_buckets(g);
    const uint64_t key = part_plan_key(g);
    // (a plan learnt while some rank had no pull lists stays valid only while this rank has none either:
    // a rank whose lists appeared since votes no, and the wave learns a new plan)
    const bool plan_ok = g->opt_part_plan && !g->part_plan.empty() && g->opt_front_exchange != 2 &&
                         g->part_plan_key == key && (can_pull || !g->part_plan_pull);
    uint64_t sums[7] = {0, 0, 0, 0, 0, 0, 0};
    if (!coll && plan_ok) {
        // one rank without collectives: nothing to agree on (the plan is this rank's own)
        sums[0] = g->pool_top;
        sums[4] = 1;
    } else {
        const uint64_t head[1] = {g->pool_top};
        const uint64_t tail[4] = {can_pull ? 0ull : 1ull, plan_ok ? 1ull : 0ull, g->pg_hash, g->pg_hash * g->pg_hash};
        FGI_HIP(g, hipMemcpyAsync(pb.red, head, 8, hipMemcpyHostToDevice, s));
        FGI_HIP(g, hipMemcpyAsync(pb.red + 1, &g->ctr->lvl[0].F, 16, hipMemcpyDeviceToDevice, s));
        FGI_HIP(g, hipMemcpyAsync(pb.red + 3, tail, 32, hipMemcpyHostToDevice, s));
        FGI_TRY(part_allreduce_sum(g, pb.red, sums, 7));
        // every rank sees the same sums, so every rank fails here together when the ranks' codes differ
        // (sum h = W h and sum h^2 = W h^2 for every rank's h only when all are equal)
        if (sums[5] != (uint64_t)pv.world * g->pg_hash || sums[6] != (uint64_t)pv.world * g->pg_hash * g->pg_hash) {
            g->failed = true;
            return set_err(g, FGI_ESTATE, "rank %u of %u: the ranks numbered their slots differently (partition codes "
                                          "chosen from different arrays: every rank must be given the same "
                                          "fgi_part_register_nodes / fgi_part_load_edges arrays)", pv.rank, pv.world);
        }
    }
    const WaveParams wp = wave_params(g, 1, g->opt_direction, sums[0], pv.n_global);
    if (sums[4] == pv.world)   // every rank follows the plan: no host synchronisation until the wave's end
        return run_part_planned(g, pv, wp, pb, n_roots, stats, t0);
    g->part_plan.clear();      // learnt again by this wave's levels
    g->part_plan_key = key;
    g->part_plan_pull = sums[3] == 0;   // every rank's pull lists were ready (the same on all ranks)
    const uint64_t stay_pull_f = wp.stay_pull_f;
    const bool allow_pull = sums[3] == 0;
    const int direction = wp.direction;
    const RemoteArgs ra{pv.base, pv.n_local, pv.block, pv.world, pv.ver_all, pv.sent_bm, pv.send_buf, pv.send_cnt};
    // the invalidated bitmap over all slots: all-gathered before pull levels (one rank without
    // collectives: its own words copied in, so the hot snapshot past its end is where the candidates
    // expect it)
    // one rank without collectives: the pull levels probe the invalidated bitmap itself (no copy into
    // front_global per pull level) when its hot snapshot sits where the partition's would (the same
    // word count: no detached handles)
    const bool alias = !coll && g->hot_w0 == g->bm_words;
    const uint32_t* front = alias ? g->inv_bm : pv.front_global;
    uint32_t* const hot_base = alias ? g->inv_bm : pv.front_global;
    uint64_t f_global = sums[1], t_global = sums[2];
    const double avg_deg = (double)sums[0] / std::max<uint64_t>(1, pv.n_global);
    uint64_t levels = 0, e_trav = 0, f_total = 0, sent_total = 0, push_edges = 0, push_f = 0;
    uint64_t pull_levels = 0, pull_launches = 0, expand_launches = 0;
    uint64_t syncs = 1;   // the start's all-reduce
    double expand_ms = 0, pull_ms = 0;
    int L = 0;
    bool last_pull = false;
    for (; f_global != 0; ++L) {
        const bool pull = allow_pull && t_global != 0 &&
                          (direction == 2 || (direction == 0 && (t_global > wp.pull_threshold ||
                                                                 (last_pull && f_global > stay_pull_f))));
        if (g->part_plan.size() < kPlanMax) g->part_plan.push_back(pull ? 1 : 0);
        const int buf = L & 1;
        if (coll) FGI_HIP(g, hipMemsetAsync(pv.send_cnt, 0, (size_t)pv.world * 8, s));
        // the level's direction for its kernels: the flag's high word is zero (the ring slot was
        // cleared two levels ago or at wave start), so a 32-bit device-side set is the whole store
        if (pull) {
            FGI_HIP(g, hipMemsetD32Async(reinterpret_cast<hipDeviceptr_t>(&g->ctr->lvl[L % kRing].pull), 1, 1, s));
            if (coll) {
                uint64_t f0 = 0, d0 = 0, d1 = 0, b = 0;
                FGI_TRY(part_front_stats(g, &f0, &d0, &b));
                FGI_TRY(part_allgather_front(g));
                FGI_TRY(part_front_stats(g, &f0, &d1, &b));
                syncs += g->opt_front_exchange != 1 ? 1 : 0;   // the delta count's read-back (auto or delta)
            } else if (!alias) {
                FGI_HIP(g, hipMemcpyAsync(pv.front_global, g->inv_bm, (size_t)pv.block / 32 * 4, hipMemcpyDeviceToDevice, s));
            }
        }
        CollectArgs ca = collect_args(g, pv.n_local, wp, buf);
        ca.inv = front;   // hot heads are global ids
        ca.hot_bm = hot_base + g->hot_w0;
        ca.sum_bm = reinterpret_cast<unsigned long long*>(g->sum_bm);   // over front_global (part init)
        ca.n64 = pv.front_words_global / 2;
        hipLaunchKernelGGL(k_collect, dim3(collect_grid(g, wp)), dim3(kCollectThreads), 0, s, L, g->ctr, wp, ca, ca, ~0ull);
        if (g->opt_level_timing) FGI_HIP(g, hipEventRecord(g->ev[0], s));
        hipLaunchKernelGGL(k_level<true>, dim3(wp.grid), dim3(kBlock), 0, s, L, wp, expand_args(g, buf),
                           expand_args(g, buf), pull_args(g, g->n_slots, front), node, g->vis_bm,
                           out_for(g, buf ^ 1, nullptr), out_for(g, buf ^ 1, nullptr), g->ctr, g->blk_stats, g->done,
                           ra, ~0ull);
        if (g->opt_level_timing) FGI_HIP(g, hipEventRecord(g->ev[1], s));
        FGI_HIP(g, hipGetLastError());
        uint64_t n_recv = 0, n_sent = 0, glob[3] = {0, 0, 0};
        const bool exch = !pull && coll;
        if (exch) {
            FGI_HIP(g, hipMemcpyAsync(pv.send_cnt + pv.world, &g->ctr->lvl[(L + 1) % kRing].F, 16,
                                      hipMemcpyDeviceToDevice, s));
            // the level's counters ride on the exchange's stream synchronisation
            FGI_HIP(g, hipMemcpyAsync(g->ctr_host, g->ctr, sizeof(WaveCtr), hipMemcpyDeviceToHost, s));
            FGI_TRY(part_exchange(g, &n_recv, &n_sent, glob));
        }
        if (n_recv)
            hipLaunchKernelGGL(k_apply_recv, dim3(std::min<uint64_t>((n_recv + kBlock - 1) / kBlock, (uint64_t)g->n_cu * 8)),
                               dim3(kBlock), 0, s, L, n_recv, pv.recv_buf, pv.base, node, g->vis_bm,
                               out_for(g, buf ^ 1, nullptr), g->ctr, g->blk_stats, g->done, 0u);
        FGI_HIP(g, hipGetLastError());
        sent_total += n_sent;
        ++syncs;   // the level's count all-gather or all-reduce
        // every winner remote (the wave's tail): whether the received targets add any is known only
        // after they are applied, so the exact all-reduce decides termination (no empty level)
        if (exch && (glob[0] != 0 || glob[2] == 0)) {
            f_global = glob[0] + glob[2];
            t_global = glob[0] ? (uint64_t)((double)glob[1] * (double)f_global / (double)glob[0])
                               : (uint64_t)((double)glob[2] * avg_deg);
            if (glob[2] && !t_global) t_global = 1;
        } else {
            // the counter copy rides on the all-reduce's stream synchronisation
            FGI_HIP(g, hipMemcpyAsync(g->ctr_host, g->ctr, sizeof(WaveCtr), hipMemcpyDeviceToHost, s));
            uint64_t ft[2] = {0, 0};
            FGI_TRY(part_allreduce_sum(g, &g->ctr->lvl[(L + 1) % kRing].F, ft, 2));
            f_global = ft[0];
            t_global = ft[1];
        }
        const LevelCtr& lc = g->ctr_host->lvl[L % kRing];
        ++levels;
        e_trav += lc.T;
        f_total += lc.F;
        float ms = 0;
        if (g->opt_level_timing) FGI_HIP(g, hipEventElapsedTime(&ms, g->ev[0], g->ev[1]));
        if (pull) {
            ++pull_levels;
            ++pull_launches;
            pull_ms += ms;
        } else {
            push_edges += lc.T;
            push_f += lc.F;
            ++expand_launches;
            expand_ms += ms;
        }
        last_pull = pull;
    }
    FGI_HIP(g, launch_final(g, pv.n_local));
    FGI_HIP(g, hipGetLastError());
    FGI_TRY(counters_to_host(g, s, part_events(g)));
    g->last_wave_n = g->ctr_host->inv;
    g->ids_valid = true;
    if (stats) {
        const WaveCtr& c = *g->ctr_host;
        const uint64_t v = c.inv;
        stats->roots += n_roots;
        stats->levels += levels;
        stats->v_inv += v;
        stats->e_trav += e_trav;
        stats->e_match += c.e_match;
        stats->n_flagged += c.n_flagged;
        stats->remote_msgs += sent_total;
        stats->host_syncs += syncs + 1;   // + the final collect's
        // as run_wave, plus 8 B per forwarded target (written + received)
        const uint64_t pull_b = pull_level_bytes(c);
        stats->alg_bytes += 20 * push_edges + 40 * push_f + pull_b + 4 * v + 8 * sent_total + 5ull * n_roots;
        stats->pull_levels += pull_levels;
        stats->pull_edges += c.pull_edges;
        stats->pull_ms += pull_ms;
        stats->pull_bytes += pull_b;
        stats->pull_launches += pull_launches;
        float wave_ms = 0;
        if (part_events(g)) hipEventElapsedTime(&wave_ms, g->ev_w0, g->ev_w1);
        else wave_ms = wall_ms(g, c.t0, g->last_pub_t);
        stats->kernel_ms += wave_ms;
        stats->expand_ms += expand_ms;
        stats->expand_launches += expand_launches;
        stats->expand_bytes += 20 * push_edges + 40 * push_f;
        stats->f_total += f_total;
        stats->total_ms += std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    }
    return FGI_OK;
}

}  // namespace fgi
