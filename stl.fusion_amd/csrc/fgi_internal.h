// fgi_internal.h — device data layout and shared helpers of the fgi engine (gfx950 only).
//
// HBM layout, one entry per handle h in [0, n_slots + n_detached):
//   node[h]    u64  packed node word: bits 0-55 version (LTag; 0 = no node), bits 56-57
//                   ConsistencyState, bit 58 InvalidateOnSetOutput, bit 59 InvalidationDelayStarted,
//                   bit 60 hasDelay. One 64-bit CAS checks the version and moves the state.
//   row_off[h] u64  start of h's `_usedBy` row in the edge pool
//   row_len[h] u32  entries in the row (logical length is 0 once the node is Invalidated)
//   row_cap[h] u32  reserved entries (appends go in place while len < cap)
//   used_cnt[h]u32  |_used| of the node (forward links created while it was Computing)
// Edge pool (structure of arrays, rows are contiguous runs):
//   pool_col[p] u32 dependant slot (ComputedInput of the `_usedBy` entry)
//   pool_tag[p] u64 dependant version at capture time (LTag of the `_usedBy` entry)
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <chrono>
#include <cstdlib>
#include <string>
#include <utility>
#include <vector>

#include "../../include/fgi.h"
#include "../../include/fgi_variants.h"

// Measurement variants (make variant-all -> libfgi_variants.so): the fused waves, the probe summary and
// the cooperative launch of streaming cascades, each measured slower than the shipping paths on MI355X
// (DESIGN.md §3, §7b). The shipping library leaves them out: their options return FGI_ENOTSUP.
#ifndef FGI_VARIANTS
#define FGI_VARIANTS 0
#endif

namespace fgi {

constexpr uint64_t kVMask = (1ull << 56) - 1;
constexpr int kStateShift = 56;
constexpr uint64_t kStateBits = 3ull << kStateShift;
constexpr uint64_t kW_IOSO = 1ull << 58;
constexpr uint64_t kW_DS = 1ull << 59;
constexpr uint64_t kW_HasDelay = 1ull << 60;
constexpr uint64_t kW_Computing = 0ull;
constexpr uint64_t kW_Consistent = 1ull << kStateShift;
constexpr uint64_t kW_Invalidated = 2ull << kStateShift;

__host__ __device__ inline uint32_t word_state(uint64_t w) { return (uint32_t)((w >> kStateShift) & 3u); }
__host__ __device__ inline bool word_is_current(uint64_t w) {
    return (w & kVMask) != 0 && word_state(w) != FGI_INVALIDATED;
}

// Host-visible state_flags <-> node word (canonical flags, fgi.h)
__host__ __device__ inline uint32_t word_to_flags(uint64_t w) {
    if ((w & kVMask) == 0) return 0;
    uint32_t st = word_state(w);
    uint32_t f = st;
    if (st == FGI_COMPUTING) {
        if (w & kW_IOSO) f |= FGI_F_INVALIDATE_ON_SET_OUTPUT;
        if (w & kW_DS) f |= FGI_F_INVALIDATION_DELAY_STARTED;
    } else if (st == FGI_CONSISTENT) {
        if (w & kW_DS) f |= FGI_F_INVALIDATION_DELAY_STARTED;
    }
    if (w & kW_HasDelay) f |= FGI_F_HAS_DELAY;
    return f;
}
__host__ __device__ inline uint64_t flags_to_word(uint64_t version, uint32_t f) {
    uint64_t w = (version & kVMask) | ((uint64_t)(f & 3u) << kStateShift);
    if (f & FGI_F_INVALIDATE_ON_SET_OUTPUT) w |= kW_IOSO;
    if (f & FGI_F_INVALIDATION_DELAY_STARTED) w |= kW_DS;
    if (f & FGI_F_HAS_DELAY) w |= kW_HasDelay;
    return w;
}

// splitmix64 finaliser
__host__ __device__ inline uint64_t sm64(uint64_t x) {
    x += 0x9E3779B97F4A7C15ull;
    x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
    x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
    return x ^ (x >> 31);
}
__host__ __device__ inline uint64_t synth_version(uint64_t seed, uint32_t slot) {
    return (sm64(seed ^ (uint64_t)slot) & ((1ull << 55) - 1)) | 1ull;
}

// R-MAT edge i of a (scale, seed) graph (oracle/synth.cpp): per level l,
// u = sm64(sm64(seed) ^ (i << 6 | l)) >> 11 against 0.57 / 0.76 / 0.95 * 2^53, endpoints scrambled by
// a bijection of [0, 2^scale)
__host__ __device__ inline uint32_t rmat_scramble(uint64_t x, uint32_t scale, uint64_t seed) {
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
__host__ __device__ inline void rmat_edge(uint64_t i, uint32_t scale, uint64_t seed, uint32_t* src, uint32_t* dst) {
    const uint64_t one = 1ull << 53;
    const uint64_t tA = one / 100 * 57, tAB = one / 100 * 76, tABC = one / 100 * 95;
    const uint64_t ks = sm64(seed);
    uint64_t s = 0, d = 0;
    for (uint32_t l = 0; l < scale; ++l) {
        const uint64_t u = sm64(ks ^ ((i << 6) | l)) >> 11;
        const uint64_t bit = 1ull << (scale - 1 - l);
        if (u >= tA) {
            if (u < tAB) d |= bit;
            else if (u < tABC) s |= bit;
            else {
                s |= bit;
                d |= bit;
            }
        }
    }
    *src = rmat_scramble(s, scale, seed);
    *dst = rmat_scramble(d, scale, seed);
}
// stale edge of the churn workloads (configs[3]): tag = version + 1
__host__ __device__ inline bool synth_stale(uint32_t stale_pct, uint64_t stale_seed, uint32_t src, uint32_t dst) {
    return stale_pct && (sm64(stale_seed ^ sm64(((uint64_t)src << 32) | dst)) % 100) < stale_pct;
}

// ---- wave bookkeeping -------------------------------------------------------------------------
constexpr int kRing = 64;               // per-level counters live in a ring (deep waves roll over)
constexpr int kBlock = 256;             // threads per block for the traversal kernels
constexpr int kEPT = 8;                 // edges per thread per chunk (largest chunk)
constexpr int kChunk = kBlock * kEPT;   // edges per expand chunk (largest chunk)
constexpr int kFine = 256;              // edges per fine chunk of the chunk map (cstart granularity);
                                        // a push level expands chunks of 1..kEPT fine chunks
constexpr uint32_t kStatBlocks = 8192;  // per-block statistics rows (grid limit of the hot kernels: 268M slots pull)
constexpr int kStatCols = 8;
constexpr int kPullTile = 1024;         // slots per pull tile (one block iteration of a pull level)
constexpr int kDoneGroups = 16;         // two-level completion counters (last-block epilogues)
constexpr int kDoneStride = 16;         // 128 B apart
#ifndef FGI_FINAL_BLOCKS
#define FGI_FINAL_BLOCKS 1024               // measurement builds: make variant-grid FINAL=<blocks> WPB=<words> INIT=<blocks>
#endif
#ifndef FGI_FINAL_WPB
#define FGI_FINAL_WPB 256
#endif
#ifndef FGI_INIT_BLOCKS
#define FGI_INIT_BLOCKS 2048
#endif
constexpr uint32_t kFinalBlocks = FGI_FINAL_BLOCKS; // grid of the final collect (invalidated bitmap -> list)
constexpr uint32_t kFinalWpb = FGI_FINAL_WPB;       // fewest 64-bit bitmap words per final-collect block
constexpr uint32_t kInitBlocks = FGI_INIT_BLOCKS;   // grid of k_wave_init
#ifndef FGI_SPIN_WAIT
#define FGI_SPIN_WAIT 1                     // measurement builds: make variant-nospin (stream synchronisation)
#endif
#ifndef FGI_HOT
#define FGI_HOT 524288                  // measurement builds: make variant-hot HOT=<n> (a multiple of 256)
#endif
constexpr uint32_t kHot = FGI_HOT;      // most hot list heads (pull probes through a snapshot of kHot / 8 B)
#ifndef FGI_LDS_HOT
#define FGI_LDS_HOT 4096                // measurement builds: make variant-ldshot LDSHOT=<words>
#endif
// hot snapshot words a pull block keeps in LDS (16 KB): 4,096 against 2,048 measured -1% on configs[1]
// and -2% on configs[2] with hub-first labels; 8,192 pulls faster still but its lower occupancy makes
// the push levels 4x slower (round 5, profiles/r12i_ldshot_ab.txt)
constexpr uint32_t kLdsHot = FGI_LDS_HOT;
// fewest hot heads: 8 KB, or what the LDS copy holds (a graph's count: build_candidates, hot_count)
#ifdef FGI_HOT_MIN
constexpr uint32_t kHotMin = FGI_HOT_MIN;   // measurement builds (variant-cpl HOTMIN=)
#else
constexpr uint32_t kHotMin = kLdsHot * 32 > 65536 ? kLdsHot * 32 : 65536;
#endif
// resident k_level blocks per CU: LDS-bound once the LDS snapshot passes 8 KB (160 KB per CU)
#ifdef FGI_LEVEL_OCC
constexpr uint32_t kLevelOcc = FGI_LEVEL_OCC;   // measurement builds (variant-cpl)
#else
constexpr uint32_t kLevelOcc = kLdsHot <= 2048 ? 5 : kLdsHot <= 4096 ? 4 : 3;
#endif
constexpr int kAccCount = 8;            // batch accumulators (fgi_run_batch; run_wave_coop's acc)
// A batch's abort word (fgi_run_batch): reason << 32 | (step + 1). kAbortBarrier: a cascade's grid
// barrier timed out (no step index; the graph is poisoned until fgi_restore).
constexpr unsigned long long kAbortDetach = 1, kAbortPool = 2, kAbortBarrier = 3;
constexpr int kAccBarrierIdx = 7;       // acc[7]: a cascade's grid barrier timed out
// grid-barrier arrival counters (g->gbar, monotonic, a multiple of the grid size between launches):
// word 0 k_wave_coop's (streaming cascades), word kGbarFused k_wave_fused's (their grids differ)
constexpr int kGbarWords = 32, kGbarFused = 16;

// Per-level counters. The producers of level L's frontier (roots, push emits, received targets)
// reserve list space with ONE packed 64-bit atomic on `ft` (frontier entries << 32 | edges): the
// returned value is both the entry index and the exclusive edge offset (escan) of the reserving
// batch, so the frontier list comes out already scanned. The last block of each producer kernel
// unpacks ft into F / T (a pull level sums its per-block counts instead).
struct LevelCtr {
    unsigned long long F;       // frontier entries (expandable = invalidated with |row| > 0)
    unsigned long long T;       // edges of the frontier (sum of row lengths)
    unsigned long long ft;      // packed reservation counter (F << 32 | T)
    unsigned long long pull;    // 1 if this level runs bottom-up (pull)
    unsigned long long w;       // pull level L-1: its winners (the frontier count before rows)
    unsigned long long mult;    // push: fine chunks per expand chunk
    unsigned long long npull;   // pull levels of the wave before this one (which candidate list to read)
    unsigned long long sum;     // pull level: 1 if k_collect built the nonzero-word summary for its probes
    unsigned long long want;    // 1 if the automatic choice (Beamer's rules) is pull, whatever the level ran
                                // as (a level the host pinned to push, push-only options): the next wave's
                                // launch plan (run_wave's left-out collects) learns from it
};

// A level's frontier totals: a push producer leaves them packed in ft (the single engine does not
// unpack them: the next kernel and the host read ft directly, which saves the producer's last-block
// hand-off; a partition's producers unpack them into F / T for the all-reduce), a pull level's last
// block writes F / T (ft stays 0). F == 0 means no frontier entry, and then T == 0 too.
__host__ __device__ inline uint64_t lvl_F(const LevelCtr& c) { return c.F ? c.F : (c.ft >> 32); }
__host__ __device__ inline uint64_t lvl_T(const LevelCtr& c) { return c.F ? c.T : (c.ft & 0xFFFFFFFFull); }

struct WaveCtr {
    unsigned long long inv;         // invalidated handles of the wave (V_inv; the final collect)
    unsigned long long e_match;
    unsigned long long n_flagged;
    unsigned long long root_inv;    // winners of the roots kernel
    unsigned long long pull_surv;   // pull: candidates still unvisited after their level (written forward)
    unsigned long long pull_edges;  // pull: dependency entries examined
    unsigned long long pull_live;   // pull: slots not yet dead when scanned
    unsigned long long pull_win;    // pull: nodes invalidated by pull levels
    unsigned long long pull_scan;   // pull: slots scanned (bitmap reads), summed over pull levels
    unsigned long long pull_tail;   // pull: candidates whose head dependency missed (list scanned)
    unsigned long long root_flagged;  // flag-only visits of the roots kernel
    // fused waves (run_wave): the head / tail kernels run the small push levels inside
    // one launch each; k_level launches in between run the pull levels (and push levels too large for
    // the fused grid), each reading its level from here
    unsigned long long cur;         // the next level to run
    unsigned long long mid_base;    // the level of the round's first k_level launch (mid index 0)
    unsigned long long phase;       // kPhaseDone once the final count has run
    unsigned long long broken;      // a fused kernel's grid barrier timed out
    unsigned long long n_levels;    // device-side totals of the wave: non-empty levels,
    unsigned long long e_trav;      //   their frontier edges (E_trav),
    unsigned long long f_total;     //   their frontier entries,
    unsigned long long n_pull;      //   pull levels,
    unsigned long long push_edges;  //   edges / entries of the push levels run inside the fused kernels
    unsigned long long push_f;
    unsigned long long n_mid;       //   levels run by k_level launches
    unsigned long long mid_kind[16];  // per k_level launch of the round (mid index): 0 nothing, 1 push, 2 pull
    unsigned long long mid_push_edges;  // edges / entries of the push levels run by k_level launches
    unsigned long long mid_push_f;
    unsigned long long t0;          // device wall clock at k_wave_init (a wave's kernel span without events)
    unsigned long long t_max;       // the wave's largest level, in edges (level-group waves: tail_account)
    unsigned long long pull_pushed; // levels the automatic choice would pull that a tail ran as push (async `all`)
    LevelCtr lvl[kRing];
};
constexpr unsigned long long kPhaseDone = 1;
constexpr uint32_t kPlanMax = 48;   // levels of a planned partitioned wave
constexpr int kMidMax = 16;         // k_level launches per round of a fused wave

// per-wave accounting of a partitioned wave
struct PartWave {
    std::chrono::steady_clock::time_point t0;
    uint64_t n_roots = 0, levels = 0, e_trav = 0, f_total = 0, sent = 0, expand_launches = 0;
    uint64_t push_edges = 0, push_f = 0, pull_launches = 0, pull_levels = 0;
    double expand_ms = 0, pull_ms = 0;
    bool pulled = false;
};

// FGI_OPT_FUSED bits: fused waves on; tests: no mid-pair prediction (every k_level level found by an
// extra round), every push level as a k_level launch, every push level in the fused grid
constexpr int kFusedOn = 1, kFusedNoPredict = 2, kFusedMidPush = 4, kFusedTailPush = 8;
// Fused waves are off by default: on MI355X they measured slower than the level groups (DESIGN.md
// §3: a grid barrier's cache maintenance costs what a launch does, and the fused grid runs the push
// levels' dependent round trips with fewer blocks). FGI_FUSED=1 in the environment turns them on.
inline int fused_default() {
#if FGI_VARIANTS
    const char* e = getenv("FGI_FUSED");
    return (e && e[0] == '1') ? kFusedOn : 0;
#else
    return 0;
#endif
}

// ---- cross-block hand-off shared by the kernels' last-block epilogues (wave.hip, graph.hip) ---------
// Block-uniform: true in the block that arrives last at this launch's completion counter, over the
// blocks [0, G) taking part. The counter is two-level (one word serialises near 88 atomics/us,
// MI355X_MICROARCH.md "dequeue"): block b counts into group b % kDoneGroups, the last block of a group
// into the top word; the last block resets every word for the next launch. Agent-scope atomic RMWs are
// performed at the coherence point shared by the XCDs, so what the last block must see has to be
// performed before its block arrives:
//   kDrainAll = false: the block's hand-off values are written by thread 0 (or by atomics whose result
//     a thread waited for); wave 0 drains its own memory counter before the arrival (the traversal
//     kernels: one wave's wait, not every wave's, sits on their critical path);
//   kDrainAll = true: any wave may have issued returnless atomics the last block reads (a batch's
//     classify counts, the overflow-row list): every wave drains its vector-memory counter (returnless
//     atomics included, gfx9 counts them in vmcnt) before the block's barrier, and the arrivals are
//     acquire-release at agent scope.
template <bool kDrainAll>
__device__ inline bool last_block_arrive(unsigned long long* done, uint64_t G) {
    __shared__ bool s_last;
    if (kDrainAll) __builtin_amdgcn_s_waitcnt(0);
    __syncthreads();
    if (threadIdx.x == 0) {
        __builtin_amdgcn_s_waitcnt(0);
        constexpr int kOrd = kDrainAll ? __ATOMIC_ACQ_REL : __ATOMIC_RELAXED;
        const uint32_t grp = blockIdx.x % kDoneGroups;
        const uint64_t gsize = (G - grp + kDoneGroups - 1) / kDoneGroups;
        const unsigned long long t =
            __hip_atomic_fetch_add(done + (1 + grp) * kDoneStride, 1ull, kOrd, __HIP_MEMORY_SCOPE_AGENT);
        bool last = false;
        if (t == gsize - 1) {
            const uint64_t ng = G < (uint64_t)kDoneGroups ? G : (uint64_t)kDoneGroups;
            last = __hip_atomic_fetch_add(done, 1ull, kOrd, __HIP_MEMORY_SCOPE_AGENT) == ng - 1;
        }
        s_last = last;
    }
    __syncthreads();
    const bool last = s_last;
    if (last && threadIdx.x <= (uint32_t)kDoneGroups)
        __hip_atomic_exchange(done + threadIdx.x * kDoneStride, 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    return last;
}

// ---- host-side graph object -------------------------------------------------------------------
struct DevBuf {
    void* p = nullptr;
    size_t bytes = 0;
};

}  // namespace fgi

struct fgi_graph {
    int device = 0;
    int n_cu = 256;                    // compute units of the device (queried once at create)
    hipStream_t stream = nullptr;
    // Internal handle space (labels). n_slots / n_handles count the engine's labels:
    // K hot labels [0, K) for the heaviest slots, then label K + x for every other slot or detached
    // handle x (the labels K + x of hot slots stay empty). ext_slots / ext_handles are the boundary's
    // counts (fgi_config.n_slots, + n_detached). K = 0 (labels are the handles) unless the graph uses
    // hub-first labels.
    uint32_t n_slots = 0, n_detached = 0, n_handles = 0;
    uint32_t ext_slots = 0, ext_handles = 0;
    uint32_t lbl_K = 0;                // label capacity of the hot prefix (a multiple of kFoldTile)
    uint32_t lbl_hot = 0;              // hot labels in use (<= lbl_K), set at the first bulk edge load
    int opt_labels = 0;                // fgi_config.labels: 0 auto, 1 always, -1 never
    bool lbl_done = false;             // the hot set has been chosen (first bulk edge load)
    bool nodes_written = false;        // node words were written since create (note_words): at labels, if any
    // Partition codes: a partition renumbers the slots within each rank's range, heaviest
    // first, so that the all-gathered invalidated bitmap the pull levels probe holds every rank's hubs in a
    // compact run at the start of its range. Ownership is unchanged (a slot's code lies in its owner's
    // range). Every fgi_part_* entry point and every query maps slots <-> codes; the engine runs on codes.
    bool lbl_perm = false;
    uint32_t* pg_gc = nullptr;         // [n_global] slot -> code (device)
    uint32_t* pg_ig = nullptr;         // [n_global] code -> slot (device)
    std::vector<uint32_t> pg_gc_h, pg_ig_h;   // host copies
    uint64_t pg_hash = 0;               // of the slot -> code table (0: no codes); every rank's must agree
    uint32_t* s2l = nullptr;           // [ext_slots] hot label of a slot, FGI_NONE if cold
    uint32_t* l2s = nullptr;           // [lbl_K] slot of a hot label
    uint32_t* fold_start = nullptr;    // [fold_tiles + 1][lbl_ncls] first hot label of class c at slots >= t * kFoldTile
    uint16_t* fold_off = nullptr;      // [lbl_hot] per tile, its hot labels in (class, slot) order: slot - tile base
    uint32_t* fold_base = nullptr;     // [fold_tiles + 1] each tile's first entry in fold_off
    uint32_t lbl_ncls = 0, fold_tiles = 0;
    unsigned long long* xbm = nullptr; // [ext words] the wave's invalidated set over the boundary's handles
    unsigned long long* fold_status = nullptr;   // [fold tiles, >= kStats] per-tile counts of the final collect
    int rank = 0, world = 1;

    // node table
    uint64_t* node = nullptr;
    uint64_t* row_off = nullptr;
    uint32_t* row_len = nullptr;
    uint32_t* row_cap = nullptr;
    uint32_t* used_cnt = nullptr;
    uint32_t* home = nullptr;          // [n_detached]: home slot of a detached handle
    std::vector<uint32_t> free_detached;  // host free list of detached handles
    std::vector<uint64_t> seen_bits;      // host scratch bitmap over slots (batch duplicate checks)
    std::vector<uint8_t> seen_slots;      // host scratch, a byte per slot (fgi_run_batch's duplicate checks)
    // device temporaries of the mutation calls, kept for reuse (same stream, so reuse is ordered
    // after the previous user) instead of a hipMalloc + hipFree (an implicit device sync) per call
    std::vector<std::pair<size_t, void*>> tmp_cache;
    size_t tmp_cached = 0;

    // edge pool
    uint32_t* pool_col = nullptr;
    uint64_t* pool_tag = nullptr;
    uint64_t pool_cap = 0;             // entries
    uint64_t pool_top = 0;             // bump pointer (host mirror of device counter)
    unsigned long long* pool_top_dev = nullptr;
    uint64_t pool_epoch = 0;           // bumped on compaction (invalidates snapshots)

    // wave workspace
    uint32_t* inv = nullptr;           // [n_handles] invalidated handles of the last wave (ascending)
    uint32_t* fr_off[2] = {nullptr, nullptr};  // frontier lists: row offsets (pool positions < 2^32)
    uint32_t* fr_len[2] = {nullptr, nullptr};
    uint64_t* escan[2] = {nullptr, nullptr};   // exclusive edge offset of every frontier entry
    uint32_t* cstart[2] = {nullptr, nullptr};  // fine chunk -> frontier entry holding its first edge
    uint64_t cstart_cap = 0;
    unsigned long long* bsum = nullptr;  // [8][kStatBlocks] per-block sums / prefixes of the epilogues
    unsigned long long* done = nullptr;  // completion counters of the last-block epilogues
    fgi::WaveCtr* ctr = nullptr;
    unsigned long long* gbar = nullptr;   // [kGbarWords] grid-barrier counters (k_wave_coop, k_wave_fused)
    unsigned long long* blk_stats = nullptr;   // [kStatBlocks][kStatCols] per-block wave statistics
    fgi::WaveCtr* ctr_host = nullptr;  // pinned
    // fine-grained host memory the wave's publish kernel writes: the counters, then a sequence word
    // (ctr_pub[kPubWords]) the host spins on instead of a stream synchronisation (run_wave)
    unsigned long long* ctr_pub = nullptr;
    uint64_t pub_seq = 0;
    int wall_khz = 0;                   // device wall-clock rate (WaveCtr::t0 and the publish time)
    uint64_t last_pub_t = 0;            // the last publish_wait's device wall-clock stamp
    unsigned long long* red_pub = nullptr;   // fine-grained host words of the partition's all-reduce results
    uint32_t* roots_buf = nullptr;     // staging for host roots
    uint8_t* imm_buf = nullptr;
    uint64_t roots_cap = 0;
    uint64_t last_wave_n = 0;
    // asynchronous waves (fgi_invalidate_async / fgi_wave_wait): at most two in flight (tickets t and
    // t + 1), each with its own published counters (apub[t % 2]) and id buffer (inv for even tickets,
    // inv_alt for odd ones); inv_cur is the id list of the last wave a caller waited for
    struct AsyncWave {
        uint64_t ticket = 0, seq = 0;
        uint64_t n_inv = 0;            // V_inv, once waited for
        uint32_t n_roots = 0;
        bool busy = false, imm = false, timing = false;
        int group = 0;
        std::chrono::steady_clock::time_point t0;
    };
    AsyncWave aw[2];
    unsigned long long* apub[2] = {nullptr, nullptr};
    uint64_t apub_seq = 0;
    uint64_t next_ticket = 1;
    uint32_t* inv_alt = nullptr;
    uint32_t* inv_cur = nullptr;
    // fgi_invalidate_async_host: per ticket parity, the roots staged in pinned memory and their device copy
    uint32_t* ar_h[2] = {nullptr, nullptr};
    uint32_t* ar_d[2] = {nullptr, nullptr};
    uint64_t ar_cap[2] = {0, 0};
    bool lists_wanted = false;         // a wave met a frontier heavy enough to pull (async waves build lists first)
    bool want_ids = true;              // run_wave writes the invalidated list (false: bitmap and count only)
    bool ids_valid = false;            // inv holds the last wave's list (else ensure_ids rebuilds it)
    int last_levels = 4;               // non-empty levels of the last wave (sizes the first level group)
    int last_head = 4;                 // levels up to the last one the tail cannot run (pull, or large push)
    std::vector<uint8_t> last_dirs;    // the last synchronous wave's levels: 1 pull, 0 push (k_collect grids)
    int last_mid = 3;                  // k_level launches the last fused wave needed (its mid pairs)
    int fused_per_cu = 0;              // resident k_wave_fused blocks per CU (0: not queried yet)
    bool coop_warm = false;            // a cooperative launch has run (coop_warm)

    // Visit bitmap over handles: bit h set = node h was visited by a wave since the
    // last fold. A visit's effect is a pure function of the node word, and every second visit is a
    // no-op, so the pair (node word, visit bit) is the node's state; one atomicOr decides the first
    // visitor. fold() applies the bits to the words before any mutation or state query.
    uint32_t* vis_bm = nullptr;
    // fgi_restore swaps in a clean second visit bitmap instead of leaving the clear to the next wave's init
    // kernel; the next wave's list kernel clears the swapped-out one (spare_dirty) as it goes
    uint32_t* vis_spare = nullptr;
    bool spare_dirty = false;
    // the last level-group wave left its counters, statistics and invalidated bitmap zeroed (its final
    // kernels and publish did, WaveEnd): the next wave runs without k_wave_init
    bool wave_clean = false;
    bool v_dirty = false;              // vis_bm may hold set bits
    bool vis_stale = false;            // fgi_restore left vis_bm's clearing to the next wave (flush_vis)
    bool coop_clean = false;           // wave counters, statistics and bitmaps clear (a cooperative wave left them so)
    // Expandable-class bitmap (Consistent, no delay: a first visit invalidates and expands), built
    // from the node words; pull levels read it instead of the words (2 MB vs 128 MB at 16M slots).
    uint32_t* cls_bm = nullptr;
    bool cls_valid = false;
    bool words_dirty = true;           // node words changed since the snapshot
    // Invalidated bitmap: bit h set = node h was invalidated by this wave. It is the frontier of a
    // pull level: every node invalidated before the previous level already had all its dependants
    // visited, so "an invalidated parent" and "a parent in the previous level's frontier" select
    // the same unvisited slots. Multi-GPU: all-gathered into front_global.
    uint32_t* inv_bm = nullptr;
    uint64_t bm_words = 0;             // words per bitmap (even: pull levels store 64-bit words)

    // dependency-list cache for pull levels: for slot d, the handles whose `_usedBy` row holds
    // (d, version(d)) (= the reference's d._used). Rebuilt from the rows when stale.
    uint64_t* uin_off = nullptr;
    uint32_t* uin_len = nullptr;
    uint32_t* uin_src = nullptr;
    uint64_t* uin_head = nullptr;      // [n_slots] the list's first two entries (lo | hi << 32, FGI_NONE
                                       // if absent), probed first: lists are ordered by the number of
                                       // dependencies of each entry, the ones a wave reaches earliest
    uint32_t* uin_more = nullptr;      // bitmap: the list has more than two entries
    uint64_t uin_cap = 0;
    // Per pool position: the entry was live (tag == its dependant's version) when the dependency lists
    // were built. Versions change only through mutations (mut_epoch) and entries move only through
    // compaction (pool_epoch), so while both are unchanged an entry is live iff its bit is set and its
    // dependant is current: fgi_prune then reads this bitmap and a bitmap of current nodes (2 MB at 16 M
    // slots, L2-resident) instead of gathering every dependant's 8-byte node word.
    unsigned long long* pool_live = nullptr;
    uint64_t pool_live_cap = 0;              // positions covered
    uint64_t pl_mut_epoch = 0, pl_pool_epoch = ~0ull;
    // Pull candidates: the slots with a non-empty dependency list, grouped by the
    // pull block owning their tile range (segment [cand_seg[b], cand_seg[b + 1]), slot order), as
    // (slot, list heads, row length | more-than-two-entries bit << 31). A pull level reads the
    // static list (first pull of a wave) or the survivors of the previous pull level, and writes its
    // own survivors (still unvisited) into the other survivor buffer at the same segment bases.
    // One 16-byte entry per candidate: {slot, row length | more << 31, head 0, head 1}.
    uint4* cand = nullptr;
    uint32_t* cand_seg = nullptr;      // [pull grid + 1]
    uint32_t* wl = nullptr;            // [n_slots] a pull level's expandable winners, per block at cand_seg
    // Hot heads: the (at most kHot) handles that head the most lists get a rank; candidate entries
    // name them by a bit index past the bitmap's end (hot_w0), where a pull level finds a snapshot of their
    // invalidated bits taken before the level (8 KB: L1-resident) instead of the whole bitmap.
    uint32_t* hot_id = nullptr;        // [kHot] rank -> handle (FGI_NONE past n_hot)
    uint32_t n_hot = 0;
    uint64_t hot_w0 = 0;               // the snapshot's first word in the bitmap a pull level probes
                                       // (inv_bm, or a partition's front_global): kHot / 32 words
                                       // allocated past its end; a hot head's code is 32 * hot_w0 + rank
    uint4* sv[2] = {nullptr, nullptr};
    uint32_t* sv_cnt[2] = {nullptr, nullptr};   // [pull grid] survivors per block
    uint64_t cand_cap = 0;
    uint32_t cand_grid = 0;            // pull grid the segments were built for (0 = none)
    uint64_t uin_epoch = 0;            // mut_epoch the cache was built at (0 = never)
    uint64_t mut_epoch = 1;            // changes on every mutation of rows or versions
    uint64_t epoch_counter = 1;
    uint64_t snap_mut_epoch = 0;

    // options (fgi_set_option)
    int opt_dead_filter = 1;
    int opt_defrag_pct = 60;
    int opt_part_coll = 0;             // FGI_OPT_PART_COLLECTIVES
    int opt_front_exchange = 0;        // FGI_OPT_FRONT_EXCHANGE: 0 auto, 1 full all-gather, 2 delta
    uint64_t stale_est = 0;            // entries waves made stale since the last prune (fgi_prune_step)
    uint32_t prune_cursor = 0;         // next handle of fgi_prune_step's walk
    int opt_direction = 0;
    int opt_pull_alpha = 28;           // profiles/r2y_direction_sweep.jsonl: 28 beats 14 on configs[0] (-6%) and [1] (-1%)
    int opt_pull_tpb = 0;             // pull tiles per block (0: from the CU count; tests)
    int opt_hot_heads = 0;            // FGI_OPT_HOT_HEADS: cap on the hot heads (0: by graph size)
    // probe summary: one bit per 64-bit word of the invalidated bitmap (set iff the word is nonzero),
    // built before a pull level while few words can be nonzero, so cold head and tail probes that
    // would miss are answered from an L2-resident table (FGI_OPT_PROBE_SUMMARY)
    uint32_t* sum_bm = nullptr;
    int64_t opt_sum_min = -1;         // fewest 64-bit bitmap words for a summary (-1: never; measured
                                      // slower on configs[2])
    int opt_pull_beta = 32;           // after a pull, pull again while the frontier exceeds n / beta
    int opt_level_timing = 1;         // HIP events around each level's k_level launch (statistics)
    int opt_fused = fgi::fused_default();  // FGI_OPT_FUSED (kFused* bits)

    // generic scratch (sorts, batches)
    void* scratch = nullptr;
    size_t scratch_bytes = 0;
    unsigned long long* misc_dev = nullptr;   // small device counters [16]
    unsigned long long* misc_host = nullptr;  // pinned [16]

    // snapshot
    uint64_t* snap_node = nullptr;
    uint64_t* snap_row_off = nullptr;
    uint32_t* snap_row_len = nullptr;
    uint32_t* snap_row_cap = nullptr;
    uint32_t* snap_used = nullptr;
    uint64_t snap_epoch = ~0ull;
    uint32_t* snap_home = nullptr;           // [n_detached]
    std::vector<uint32_t> snap_free_detached;

    // A failed streaming batch (a cascade's grid barrier timed out) left the graph half-applied: every
    // entry point but fgi_restore / fgi_destroy / fgi_last_error / fgi_set_option returns FGI_ESTATE
    // until fgi_restore brings back the snapshot (graph.hip, usable()).
    bool failed = false;
    int coop_per_cu = 0;                     // resident k_wave_coop blocks per CU on this graph's device
    uint32_t fault_block = 0;                // FGI_OPT_FAULT_INJECT: block + 1 of a cascade that skips a barrier
    uint32_t fault_skip = 0;                 // ... after this many more cascade launches
    uint32_t fault_tail_block = 0;           // FGI_OPT_FAULT_INJECT_TAIL: the same for a wave tail (k_wave_tail)
    uint32_t fault_tail_skip = 0;

    // timing
    std::vector<hipEvent_t> ev;        // pairs around expand launches
    // streaming batches (fgi_run_batch): pinned host staging + its device copy, the ids output
    char* bst_h = nullptr;
    char* bst_d = nullptr;
    size_t bst_cap = 0;
    uint32_t* bout = nullptr;
    uint64_t bout_cap = 0;
    uint64_t batch_ids_hint = 0;       // the previous batch's id count (sizes the copy made with the results)
    std::vector<hipEvent_t> batch_ev;  // fgi_run_batch per-cascade timing events (pairs)
    hipEvent_t ev_w0 = nullptr, ev_w1 = nullptr;

    // multi-GPU
    void* part = nullptr;
    fgi::PartWave pw;
    // planned partitioned waves (run_part_wave): the directions of the previous wave's levels (1 pull),
    // the key they were learnt under, and whether the pull lists were ready then
    std::vector<uint8_t> part_plan;
    uint64_t part_plan_key = 0;
    bool part_plan_pull = false;
    int opt_part_plan = 1;             // FGI_OPT_PART_PLAN

    std::string err;
};

// ---- internal entry points shared between translation units ----------------------------------
namespace fgi {
// ---- hub-first labels (labels.hip) ----
constexpr uint32_t kFoldTile = 65536;            // slots per fold tile (1,024 bitmap words; offsets fit 16 bits)
constexpr uint32_t kFoldWords = kFoldTile / 64;
constexpr uint32_t kLabelAutoSlots = 1u << 25;   // auto: graphs whose bitmap outgrows one XCD's L2 (4 MB)
constexpr uint32_t kClassPerOctave = 8;          // weight classes per octave of (dependencies + 1)
constexpr uint32_t kLabelClasses = 33 * kClassPerOctave;
constexpr uint32_t kMaxHotClasses = 256;        // hot classes (one per thread of a fold block)
// hot-prefix capacity of a graph of n boundary slots (0: the graph keeps labels = handles)
uint32_t labels_capacity(uint32_t n_slots, int opt);
// boundary handle x -> label (x < ext_handles) and back, on the device (in place; no-ops with K = 0)
fgi_status labels_map_in(fgi_graph* g, uint32_t* dev, uint64_t n);
fgi_status labels_map_out(fgi_graph* g, uint32_t* dev, uint64_t n);
// both halves of edge keys (used << 32 | dependant), boundary -> labels / labels -> boundary
fgi_status labels_map_keys(fgi_graph* g, uint64_t* keys, uint64_t m);
fgi_status labels_unmap_keys(fgi_graph* g, uint64_t* keys, uint64_t m);
// first bulk edge load (keys in boundary handles): choose the hot set from the keys' dependants and
// move the node words already registered to their labels. No-op unless the graph wants labels and has
// not chosen them yet.
fgi_status labels_choose(fgi_graph* g, const uint64_t* keys, uint64_t m);
// ---- partition codes (part.hip) ----
// whether a partition of n_global slots renumbers its slots (fgi_config.labels / FGI_LABELS, auto from 2^25)
bool part_codes_wanted(const fgi_graph* g, uint32_t n_global);
// global slots -> codes (host arrays, into out; returns the array to use: `in` itself without codes)
const uint32_t* part_codes_in(const fgi_graph* g, uint64_t n, const uint32_t* in, std::vector<uint32_t>& out);
// a partition's local handles (owned slots base + h, h < n_local; detached handles unchanged) <-> the
// engine's local indices, in place on the device (out: engine -> boundary), or one on the host
fgi_status part_codes_local(fgi_graph* g, uint32_t* dev, uint64_t n, bool out);
uint32_t part_code_local_h(const fgi_graph* g, uint32_t h, bool out);
// a global code -> its slot on the host (ids and dependants leaving the engine)
inline uint32_t part_slot_of(const fgi_graph* g, uint32_t code) {
    return (g->lbl_perm && code < g->pg_ig_h.size()) ? g->pg_ig_h[code] : code;
}
// the words of a fold tile's slots: per hot class, the hot labels of the tile's slots, or none
struct FoldArgs {
    const uint32_t* l2s;           // null: no hot labels (the bitmap of handles is the labels' own)
    const uint32_t* fold_start;
    const uint16_t* off;           // fold_off / fold_base (fgi_graph)
    const uint32_t* base;
    uint32_t ncls, tiles;          // fold_start is [tiles + 1][ncls]
    uint32_t K;                    // cold label of handle x: K + x
    unsigned long long* xbm;       // out: the invalidated set over boundary handles
    uint32_t exp;                  // measurement only (FGI_FOLD_EXP, results wrong): 1 no hot labels, 2 no cold copy, 4 no chunks, 8 no staging
};
// active (xbm set) iff the graph has a hot-label prefix (K > 0): the boundary's bitmap is then the
// labels' one shifted by K, ORed with the hot labels' bits at their slots
inline FoldArgs fold_args(const fgi_graph* g) {
    static const uint32_t exp = [] {
        const char* e = getenv("FGI_FOLD_EXP");
        return e && *e ? (uint32_t)atoi(e) : 0u;
    }();
    return FoldArgs{g->lbl_hot ? g->l2s : nullptr, g->fold_start, g->fold_off, g->fold_base, g->lbl_hot ? g->lbl_ncls : 0u,
                    g->fold_tiles, g->lbl_K, g->lbl_K ? g->xbm : nullptr, exp};
}

fgi_status set_err(fgi_graph* g, fgi_status st, const char* fmt, ...);
fgi_status hip_check(fgi_graph* g, hipError_t e, const char* what);
fgi_status ensure_scratch(fgi_graph* g, size_t bytes);
fgi_status ensure_pool(fgi_graph* g, uint64_t entries);
fgi_status ensure_cstart(fgi_graph* g, uint64_t total_edges);
// Run one cascade wave from `n_roots` device-resident roots. Fills stats (nullable).
// ext_roots: the roots are boundary handles (the entry points' own arrays), mapped to labels by the
// roots kernel; internal callers pass labels.
fgi_status run_wave(fgi_graph* g, uint32_t n_roots, const uint32_t* roots_dev, const uint8_t* imm_dev,
                    fgi_wave_stats* stats, bool ext_roots = false);
// The last single-device wave's invalidated list in g->inv (rebuilt from the invalidated bitmap if
// the wave ran in bitmap mode).
fgi_status ensure_ids(fgi_graph* g);
// Build rows from device edge keys (src << 32 | dst) + optional tags; pool must be empty.
// Consumes `keys`/`tags` buffers (they may be overwritten). If tags == nullptr the tag of each
// edge is synth_version(ver_seed, dst) (+1 if stale by hash).
// src_base / dst_base translate partition-local ids to global ones (multi-GPU): keys hold
// (local used handle << 32 | global dependant slot); tags and the stale hash use global ids.
fgi_status build_rows_from_keys(fgi_graph* g, uint64_t m, uint64_t* keys, uint64_t* tags,
                                uint64_t ver_seed, uint32_t stale_pct, uint64_t stale_seed,
                                uint32_t src_base = 0, uint32_t dst_base = 0);
// Existing live rows + m new entries given as host arrays (keys: used handle << 32 | dependant id).
fgi_status load_rows(fgi_graph* g, uint64_t m, const uint64_t* host_keys, const uint64_t* host_tags, uint32_t src_base,
                     uint32_t dst_base);
// Build the pull dependency-list cache if the graph changed since it was built.
fgi_status ensure_in_lists(fgi_graph* g);
// Copy the first two entries of every slot's list into uin_head, then (re)build the pull
// candidate segments (wave.hip).
// orders every dependency list by weight[entry], descending (graph.hip)
fgi_status sort_in_lists(fgi_graph* g, uint64_t total, const uint32_t* weight, uint32_t n_weight);
fgi_status build_in_heads(fgi_graph* g);
fgi_status build_candidates(fgi_graph* g);
// Pull geometry of a graph: blocks of a pull level and the tiles each owns (0 blocks: the graph is
// too large to pull on one device; its waves push).
void pull_geometry(const fgi_graph* g, uint32_t* grid, uint32_t* tpb);
// Record a mutation of rows or versions (invalidates the dependency-list cache).
inline void touch(fgi_graph* g) { g->mut_epoch = ++g->epoch_counter; }
// Record a change of node words (class bitmap rebuilt before the next wave; restore copies words).
inline void note_words(fgi_graph* g) {
    g->cls_valid = false;
    g->words_dirty = true;
    g->nodes_written = true;
}
// Apply the visit bitmap to the node words and clear it (wave.hip). Every entry point that reads or
// mutates node words outside a wave calls it first.
fgi_status fold(fgi_graph* g);
fgi_status flush_vis(fgi_graph* g);
bool coop_launch_mode();                 // FGI_COOP_LAUNCH=1: streaming waves as cooperative launches
fgi_status coop_warm(fgi_graph* g);   // first cooperative launch of the graph's process, outside timed spans   // fgi_restore's deferred visit-bitmap clear, before any use but a wave's init
#if FGI_PROBE
void print_coop_probe();
#endif
// A push-only wave in one launch (k_wave_coop), without host synchronisation (streaming batches):
// device-resident roots (n_max, or *n_dev of them), ids appended at out[*out_n ..), totals added to
// acc[0..6] (waves, levels, invalidated, E_trav, E_match, flagged, frontier entries; acc[7] set if a
// grid barrier timed out); nothing
// happens if *abort (nullable) is set when the wave starts.
fgi_status run_wave_coop(fgi_graph* g, uint32_t n_max, const uint32_t* roots_dev, const uint8_t* imm_dev,
                         const unsigned long long* n_dev, uint32_t* out, unsigned long long* out_n,
                         unsigned long long* acc, unsigned long long* abort);
// Asynchronous waves (wave.hip): queue a wave and return (ticket), wait for one (and every earlier
// one), wait for all in flight. Every entry point but fgi_restore, fgi_set_option and the async calls
// themselves drains first (usable()).
fgi_status run_wave_async(fgi_graph* g, uint32_t n_roots, const uint32_t* roots_dev, const uint8_t* imm_dev,
                          uint64_t* ticket);
fgi_status wave_wait(fgi_graph* g, uint64_t ticket, uint64_t* out_n, const uint32_t** ids_dev, fgi_wave_stats* stats);
// the same wave from roots in host memory: staged through the ticket parity's pinned buffer
fgi_status run_wave_async_host(fgi_graph* g, uint32_t n_roots, const uint32_t* roots, const uint8_t* imm, uint64_t* ticket);
fgi_status drain_async(fgi_graph* g);
// Rebuild the expandable-class bitmap if node words changed (wave.hip).
fgi_status ensure_cls(fgi_graph* g);
// Pull tiles of a level over n slots with `grid` blocks.
__host__ __device__ inline uint64_t pull_iters(uint64_t n, uint32_t grid) { return (n + (uint64_t)grid * kPullTile - 1) / ((uint64_t)grid * kPullTile); }
// ---- multi-GPU partition (part.hip) ----
// Release multi-GPU resources.
fgi_status part_destroy(fgi_graph* g);
struct PartView {
    uint32_t rank, world;
    uint32_t base, n_local, n_global, block;   // this rank owns [base, base + n_local); block = ceil(N/world)
    uint64_t* ver_all;          // [n_global] replica of every node's version (immutable during a wave)
    uint32_t* sent_bm;          // [n_global bits] remote targets already sent in this wave
    uint64_t sent_words;
    uint32_t* send_buf;         // [world][block] outgoing target ids per owner
    uint32_t* recv_buf;         // [world * block] incoming, concatenated
    unsigned long long* send_cnt;   // [world + 2] device counters (targets per owner, then next F, T)
    uint32_t* front_global;     // [n_global bits] all-gathered invalidated bitmap (pull levels)
    uint64_t front_words_global;
    unsigned long long* scratch_u64;
};
bool part_view(fgi_graph* g, PartView* v);
// Exchange this level's messages: counts by all-gather, payload by grouped send/recv over RCCL.
// Returns the number of target ids received (concatenated at recv_buf) and sent.
fgi_status part_exchange(fgi_graph* g, uint64_t* n_recv, uint64_t* n_sent, uint64_t* glob);
// Sum of count (1..kPartRedMax) device u64 over all ranks, returned on the host.
// src[0, words) of device memory into the fine-grained host buffer dst (words + 2 long), the host
// spinning on the sequence word dst[words]; dst[words + 1] = the publish's device wall-clock stamp
// (wave.hip). wall_ms: milliseconds between two such stamps (WaveCtr::t0 is one).
fgi_status publish_wait(fgi_graph* g, hipStream_t s, const unsigned long long* src, uint32_t words, unsigned long long* dst);
float wall_ms(fgi_graph* g, uint64_t t0, uint64_t t1);
fgi_status part_allreduce_sum(fgi_graph* g, const unsigned long long* dev_val, uint64_t* out,
                              uint32_t count = 1);
// all-gather every rank's local invalidated-bitmap words into front_global (part.hip)
fgi_status part_allgather_front(fgi_graph* g);
// zero front_global at a wave's start (the delta exchange's baseline)
fgi_status part_front_reset(fgi_graph* g);
// Planned waves (run_part_wave): the full frontier all-gather and the fixed-size bucket all-to-all,
// stream-ordered (no host synchronisation), and the buffers they move.
constexpr uint32_t kPartRedMax = 160;   // words of one all-reduce (part_allreduce_sum)
struct PartBuckets {
    uint32_t C;                        // words per peer: count, then up to C - 1 target ids
    uint32_t* send;                    // [world][C]
    uint32_t* recv;                    // [world][C]
    unsigned long long* cur;           // [world] the next send_buf id to pack per owner
    unsigned long long* red;           // [kPartRedMax] device all-reduce source
};
fgi_status part_allgather_front_async(fgi_graph* g);
uint64_t part_plan_key(const fgi_graph* g);
fgi_status part_alltoall_async(fgi_graph* g);
PartBuckets part_buckets(fgi_graph* g);
// FGI_OPT_PART_BUCKET: words per peer of the planned waves' buckets (0: all that is allocated)
fgi_status part_set_bucket(fgi_graph* g, int64_t words);
// Partitioned mutations (graph.hip): a u32 array summed over the ranks in place (synchronises); the
// current-node bitmaps of the partitioned prune (this rank's, every rank's all-gathered); the
// dependency-entry store's append from device arrays.
fgi_status part_allreduce_u32(fgi_graph* g, uint32_t* dev, uint64_t n);
fgi_status part_cur_buffers(fgi_graph* g, unsigned long long** local, unsigned long long** all, uint64_t* w64);
fgi_status part_allgather_cur(fgi_graph* g);
fgi_status part_store_in_dev(fgi_graph* g, const uint64_t* keys, const uint64_t* tags, uint64_t m);
// the dependency entries whose used end is one of the global slots listed (host, any order) die:
// their node was displaced while it stayed current (Computing, or a delayed invalidation pending)
fgi_status part_kill_used(fgi_graph* g, std::vector<uint32_t> slots);
// frontier exchanges of each kind so far and the bytes this rank received through them
fgi_status part_front_stats(fgi_graph* g, uint64_t* full, uint64_t* delta, uint64_t* bytes);
// Rebuild a partition's pull lists from its dependency-entry store if rows or versions changed.
fgi_status part_ensure_lists(fgi_graph* g);
// Partitioned wave over global root ids (wave.hip): run_part_wave drives the phases below.
fgi_status run_part_wave(fgi_graph* g, uint32_t n_roots, const uint32_t* roots_dev, const uint8_t* imm_dev,
                         fgi_wave_stats* stats);
// Append (used, dependant slot, tag) entries to rows (set semantics, no state checks).
fgi_status append_edges(fgi_graph* g, uint64_t m, const uint32_t* used_dev, const uint32_t* dep_dev,
                        const uint64_t* tag_dev, const uint32_t* dep_handle_dev);
}  // namespace fgi

#define FGI_HIP(g, call)                                                   \
    do {                                                                   \
        hipError_t _e = (call);                                            \
        if (_e != hipSuccess) return fgi::hip_check((g), _e, #call);       \
    } while (0)
#define FGI_TRY(call)                          \
    do {                                       \
        fgi_status _s = (call);                \
        if (_s != FGI_OK) return _s;           \
    } while (0)
