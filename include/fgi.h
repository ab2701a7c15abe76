/*
 * fgi.h — C-ABI of the MI355X cascading-invalidation engine ("fgi": Fusion Graph Invalidation).
 *
 * The engine keeps Stl.Fusion's reverse dependency graph (every Computed's `_usedBy` set) in HBM
 * and runs `Computed.Invalidate()` cascades as batched frontier BFS waves in gfx950 HIP kernels.
 * The reference exposes no FFI seam for the cascade (Computed<T>.Invalidate is non-virtual,
 * `_usedBy` private: src/Stl.Fusion/Computed.cs:36-37, 162); the boundary is a host layer that
 * mirrors ComputedRegistry / `using (Computed.Invalidate())` / IComputed.Invalidated and calls
 * this library (C# `[LibraryImport("fgi")]` stubs in INTEGRATION.md; the C++ mirror is
 * stl.fusion_amd/host/fusion.hpp). Every entry point below names the reference member it
 * replaces.
 *
 * Conventions
 *   - Plain C types only; all arrays are HOST pointers unless the name ends in `_dev`.
 *   - Every function returns an fgi_status; nothing throws or aborts, mirroring
 *     "Invalidate doesn't throw - ever" (Computed.cs:200-229). fgi_last_error() describes the
 *     last failure on a graph.
 *   - A graph is externally synchronised: one caller thread at a time (the host layer funnels
 *     all calls through one dispatcher, which replaces the per-node `lock(this)` of
 *     Computed.cs:42). Calls are synchronous: they return after the device work completed.
 *
 * Node model ("handles")
 *   - A slot is a ComputedInput (ComputedInput.cs / ComputeMethodInput.cs); the host maps each
 *     input to a dense slot id in [0, n_slots). Handle h < n_slots addresses the slot's current
 *     node (the registry entry, ComputedRegistry.cs:22).
 *   - Handles >= n_slots are "detached" nodes: nodes displaced from the registry by a newer
 *     computation while still Computing or while a delayed invalidation is pending
 *     (ComputedRegistry.cs:91-96 leaves such an object alive and unregistered). They keep their
 *     own `_usedBy` row and state; fgi_begin_compute hands them out.
 *   - state_flags word: bits 0-1 ConsistencyState (Computing 0, Consistent 1, Invalidated 2 —
 *     ConsistencyState.cs:5-10), bit 2 InvalidateOnSetOutput, bit 3 InvalidationDelayStarted
 *     (ComputedFlags.cs:4-8), bit 4 hasDelay (ComputedOptions.InvalidationDelay != 0).
 *     Reported flags are canonical: an Invalidated node reports no IOSO/DelayStarted bits and a
 *     non-Computing node no IOSO bit (the reference never reads them again, Computed.cs:145,
 *     164-172), so results are independent of the order in which a batch is applied.
 *   - version: the node's LTag (LTag.cs:13-22), 1 <= version < 2^56 (ConcurrentLTagGenerator
 *     yields values in [1, 2^55]). Edge tags are full 64-bit LTags.
 */
#ifndef FGI_H
#define FGI_H
#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef int fgi_status;
#define FGI_OK 0
#define FGI_EINVAL 1     /* bad argument */
#define FGI_ENOMEM 2     /* device allocation failed */
#define FGI_ECAPACITY 3  /* output buffer too small: *out_n holds the required size */
#define FGI_EDEVICE 4    /* HIP / RCCL runtime error */
#define FGI_ESTATE 5     /* operation invalid in the node's state */
#define FGI_ENOTSUP 6    /* not supported in this configuration */

#define FGI_NONE 0xFFFFFFFFu

#define FGI_COMPUTING 0u
#define FGI_CONSISTENT 1u
#define FGI_INVALIDATED 2u
#define FGI_STATE_MASK 3u
#define FGI_F_INVALIDATE_ON_SET_OUTPUT 4u
#define FGI_F_INVALIDATION_DELAY_STARTED 8u
#define FGI_F_HAS_DELAY 16u

/* fgi_add_used per-item outcome (Computed.cs:347-385) */
#define FGI_USED_ADDED 0u        /* (dependant.input, dependant.version) added to used._usedBy */
#define FGI_USED_DROPPED 1u      /* dependant not Computing: no-op (Computed.cs:351-364) */
#define FGI_USED_INVALIDATED 2u  /* used already Invalidated: dependant gets InvalidateOnSetOutput (376-378) */
#define FGI_USED_ESTATE 3u       /* used is Computing: the reference throws WrongComputedState (374-375) */

typedef struct fgi_graph fgi_graph;

typedef struct fgi_config {
    uint32_t struct_size;      /* sizeof(fgi_config) */
    int32_t device;            /* HIP device ordinal */
    uint32_t n_slots;          /* slot capacity (registry keys) */
    uint32_t n_detached;       /* capacity for detached nodes (handles n_slots .. n_slots+n_detached) */
    uint64_t edge_capacity;    /* initial edge-pool capacity (grows on demand) */
    /* multi-GPU 1-D vertex partition (fgi_part_*); 0/1 for a single device */
    int32_t rank;
    int32_t world;
    /* Internal labels: 0 auto — a single-device graph of at least 2^25 slots (an
     * invalidated bitmap larger than one XCD's L2) relabels its heaviest slots into a prefix of the
     * engine's handle space at its first bulk edge load; 1 always (tests); -1 never. Invisible at the
     * boundary: every entry point takes and returns slots and handles as before. Callers built against
     * the previous layout of this struct (struct_size without this field) get 0. */
    int32_t labels;
    int32_t reserved;
} fgi_config;

typedef struct fgi_wave_stats {
    uint64_t roots;            /* root entries submitted */
    uint64_t levels;           /* BFS levels with a non-empty frontier */
    uint64_t v_inv;            /* Consistent -> Invalidated transitions (= expanded nodes) */
    uint64_t e_trav;           /* sum of |_usedBy| over invalidated nodes (TEPS numerator). Exact on a
                                  graph's first wave (and after fgi_restore / fgi_prune); after earlier
                                  waves it also counts the entries RemoveUsedBy would have removed
                                  (Computed.cs:387-398), which the engine drops lazily at the next prune,
                                  so it can exceed the reference's count until then */
    uint64_t e_match;          /* traversed edges whose tag == version of the dst slot's node */
    uint64_t n_flagged;        /* visits that only set InvalidateOnSetOutput / DelayStarted */
    uint64_t alg_bytes;        /* algorithmic HBM bytes of the wave */
    double kernel_ms;          /* device time of the wave's kernels (HIP events) */
    double total_ms;           /* wall time of the call */
    uint64_t remote_msgs;      /* multi-GPU: frontier messages sent to other partitions */
    uint64_t f_total;          /* frontier entries expanded (invalidated nodes with |_usedBy| > 0) */
    uint64_t expand_launches;  /* expand kernel launches that had work */
    double expand_ms;          /* summed device time of those launches (HIP events) */
    uint64_t expand_bytes;     /* algorithmic bytes of those launches */
    uint64_t pull_levels;      /* levels run bottom-up */
    uint64_t pull_edges;       /* dependency-list entries examined by pull levels */
    double pull_ms;            /* device time of the k_pull launches (HIP events) */
    uint64_t pull_bytes;       /* algorithmic bytes of the k_pull launches */
    uint64_t pull_launches;    /* k_pull launches (every level of a wave that may pull) */
    /* fused waves: the head and tail launches that run the roots, the small push levels,
       the collect after a pull level and the final count inside one persistent grid each */
    uint64_t fused_launches;   /* persistent launches: the wave tail (k_wave_tail), or a fused wave's head / tail */
    double fused_ms;           /* their summed device time (HIP events, FGI_OPT_LEVEL_TIMING) */
    uint64_t fused_push_bytes; /* algorithmic bytes of the push levels they ran (20 B per edge + 40 B
                                  per frontier entry, as a k_level push) */
    uint64_t host_syncs;       /* times the wave waited for the device */
    uint64_t pull_pushed;      /* asynchronous waves: levels past the queued group that the automatic
                                  direction choice would pull and the wave ran as push (same result,
                                  slower; the next queued wave's group covers them) */
} fgi_wave_stats;

typedef struct fgi_prune_stats {
    uint64_t old_edges;        /* sum of |_usedBy| over pruned (Consistent, registered) nodes before */
    uint64_t new_edges;        /* ... and after (ComputedGraphPruner.cs:91-93) */
    uint64_t pool_before;      /* edge-pool slots in use (pool top) before */
    uint64_t pool_after;       /* ... and after (smaller only if the pass defragmented the pool) */
    double kernel_ms;          /* device time of the pruning kernels (HIP events) */
    double total_ms;           /* wall time of the call */
    uint64_t live_edges;       /* entries left in the rows the call visited */
    uint64_t dropped_edges;    /* entries of Invalidated nodes' rows dropped (their `_usedBy` was cleared) */
    uint32_t first, count;     /* the handle range visited */
    uint64_t stale_estimate;   /* fgi_prune_step: the estimate that triggered the batch */
} fgi_prune_stats;

/* ---- lifetime ------------------------------------------------------------------------------ */
fgi_status fgi_create(const fgi_config* cfg, fgi_graph** out);      /* new ComputedRegistry (ComputedRegistry.cs:38-52) */
fgi_status fgi_destroy(fgi_graph* g);                                /* ComputedRegistry.Dispose (54-55) */
const char* fgi_last_error(const fgi_graph* g);
fgi_status fgi_version(uint32_t* major, uint32_t* minor);

/* ---- registry / node state ---------------------------------------------------------------- */
/* Bulk import of current nodes (ComputedRegistry.Register, ComputedRegistry.cs:72-105, without
 * displacement: the slots must be empty). version[i] == 0 leaves the slot empty. */
fgi_status fgi_register_nodes(fgi_graph* g, uint32_t n, const uint32_t* slot, const uint64_t* version,
                              const uint32_t* state_flags);
/* Bulk import of `_usedBy` entries: used[i]._usedBy += (dependant_slot[i], tag[i])
 * (IComputedImpl.AddUsedBy body, Computed.cs:381-382, no state checks). Set semantics
 * (HashSetSlim3.Add, HashSetSlim3.cs:31-64): duplicate entries collapse. */
fgi_status fgi_load_edges(fgi_graph* g, uint64_t m, const uint32_t* used, const uint32_t* dependant_slot,
                          const uint64_t* tag);
/* IComputed.Version / ConsistencyState / flags for handles (Computed.cs:46-48). */
fgi_status fgi_get_state(fgi_graph* g, uint32_t n, const uint32_t* handle, uint64_t* version,
                         uint32_t* state_flags);
/* Whole-table dump (n_slots + n_detached entries) — for parity checks. */
fgi_status fgi_dump_states(fgi_graph* g, uint64_t* version, uint32_t* state_flags);
/* IComputedImpl.UsedBy (Computed.cs:337-345): the `_usedBy` entries of one node as the reference
 * would hold them: an entry (d, t) whose node d@t was invalidated is gone (RemoveUsedBy,
 * Computed.cs:387-398; the engine removes it lazily), and an Invalidated node reports none (its
 * set was cleared, Computed.cs:217). fgi_export_edges shows the raw pool instead. */
fgi_status fgi_get_used_by(fgi_graph* g, uint32_t handle, uint32_t* dependant_slot, uint64_t* tag,
                           uint64_t cap, uint64_t* out_n);
/* IComputedImpl.Used.Length for a node (Computed.cs:327-335). */
fgi_status fgi_get_used_count(fgi_graph* g, uint32_t handle, uint32_t* out);
/* Out-degree (|_usedBy|) of every handle, and the total. */
fgi_status fgi_get_degrees(fgi_graph* g, uint32_t* degree /*n_slots+n_detached, nullable*/, uint64_t* total);

/* ---- dependency capture (compute-method call path) ----------------------------------------- */
/* ComputeMethodFunctionBase.Compute (ComputeMethodFunctionBase.cs:19-27): a new Computing node of
 * version[i] becomes the current node of slot[i] (registered in its ctor,
 * ComputeMethodComputed.cs:9-11). A current node is displaced as ComputedRegistry.Register does
 * (ComputedRegistry.cs:83-97): it is invalidated (immediately=false) — a cascade root — and, if it
 * survives that (Computing, or Consistent with an invalidation delay), it is detached and its
 * handle returned in out_detached[i] (FGI_NONE otherwise). Slots must be distinct in one call. */
fgi_status fgi_begin_compute(fgi_graph* g, uint32_t n, const uint32_t* slot, const uint64_t* version,
                             const uint8_t* has_delay /*nullable*/, uint32_t* out_detached /*nullable*/,
                             fgi_wave_stats* stats /*nullable*/);
/* dependant.AddUsed(used) for each pair (IComputedImpl.AddUsed/AddUsedBy, Computed.cs:347-385,
 * reached from ComputedExt.UseNew / TryUseExisting, Internal/ComputedExt.cs:13-22, 70-76).
 * out_result[i] gets an FGI_USED_* code. Pairs in one call are applied as one batch.
 * Deviation from SURVEY.md §8(b)'s sketch `(src_slot, dst_slot, dst_version)`: the pairs are node
 * handles, as the reference's AddUsed takes node objects (Computed.cs:347, `AddUsed(IComputedImpl
 * used)`), not (input, version) keys. The dependant's version is its node's own (a handle names one
 * node: a slot's current node, or a detached one), so an entry can never carry a version the
 * dependant node does not have, and a detached (displaced, still Computing) dependant is addressable. */
fgi_status fgi_add_used(fgi_graph* g, uint32_t n, const uint32_t* dependant, const uint32_t* used,
                        uint32_t* out_result /*nullable*/);
/* Computed<T>.TrySetOutput (Computed.cs:141-160) for each handle: Computing -> Consistent;
 * nodes flagged InvalidateOnSetOutput are invalidated at once in one cascade wave.
 * out_set[i] = 1 if the node was Computing. */
fgi_status fgi_set_output(fgi_graph* g, uint32_t n, const uint32_t* handle, uint8_t* out_set /*nullable*/,
                          uint32_t* out_ids /*nullable*/, uint64_t cap, uint64_t* out_n /*nullable*/,
                          fgi_wave_stats* stats /*nullable*/);

/* ---- invalidation (the hot path) ----------------------------------------------------------- */
/* One batched cascade: for each root handle, `existing.Invalidate(immediately[i])`
 * (Computed.Invalidate() scope -> ComputedExt.TryUseExisting -> Computed.cs:162-230, recursing
 * through every `_usedBy` entry whose version still matches, 212-216). immediately may be NULL
 * (all false — what the scope does). The invalidated set is written to out_ids (handles, in
 * ascending order); if cap is too small, FGI_ECAPACITY is returned with *out_n = required size (the
 * wave itself has completed). out_ids may be NULL to skip the copy. */
fgi_status fgi_invalidate(fgi_graph* g, uint32_t n_roots, const uint32_t* roots, const uint8_t* immediately,
                          uint32_t* out_ids, uint64_t cap, uint64_t* out_n, fgi_wave_stats* stats);
/* Same with device-resident roots / flags / output (bench and pipelined host layers). out_ids_dev
 * may be NULL (the ids stay in the engine's own buffer, see fgi_wave_ids_dev). */
fgi_status fgi_invalidate_dev(fgi_graph* g, uint32_t n_roots, const uint32_t* roots_dev,
                              const uint8_t* immediately_dev, uint32_t* out_ids_dev, uint64_t* out_n,
                              fgi_wave_stats* stats);
/* The same wave as fgi_invalidate, with the invalidated set returned as a bitmap over handles: bit h of
 * out_bits[h / 64] set = handle h was invalidated by this wave; `words` >= (n_slots + n_detached + 63)
 * / 64 (else FGI_ECAPACITY). *out_n = V_inv. A 16.8M-slot graph's bitmap is 2 MB against 29.5 MB of
 * ids for configs[1]'s 7.4M-node wave: the host decodes it where it consumes the set. The id list
 * stays available through fgi_last_wave_ids / fgi_wave_ids_dev (made on demand). out_bits may be NULL. */
fgi_status fgi_invalidate_bits(fgi_graph* g, uint32_t n_roots, const uint32_t* roots, const uint8_t* immediately,
                               uint64_t* out_bits, uint64_t words, uint64_t* out_n, fgi_wave_stats* stats);
/* Asynchronous waves (ComputedExt.WhenInvalidated, ComputedExt.cs:99-125, which the RPC server awaits
 * at Client/Internal/RpcInboundComputeCall.cs:53): fgi_invalidate_async queues the wave
 * fgi_invalidate_dev would run (device-resident roots, boundary handles) on the graph's stream and
 * returns without waiting; *ticket names it (1, 2, ...). At most two waves are in flight: a third call
 * first waits for the oldest. The next call's host work (fgi_restore, root uploads, its launches)
 * overlaps the device's previous wave. fgi_wave_wait waits for the ticket's wave (and every earlier
 * one) and returns its V_inv, its statistics and a device pointer to its invalidated ids (ascending;
 * valid until the wave two tickets later is queued, or any synchronous wave runs); waiting again for a
 * completed ticket returns its results again until the wave two tickets later is queued (FGI_EINVAL
 * after that). Every other entry point except fgi_restore and
 * fgi_set_option first waits for the waves in flight. A wave queued this way runs all its levels in
 * one queue (no second level group): its later pull levels, if the previous wave's shape predicted
 * fewer, run as push levels — same result, slower, and counted in fgi_wave_stats.pull_pushed. A wave
 * whose tail's grid barrier times out fails its fgi_wave_wait with FGI_EDEVICE and poisons the graph
 * until fgi_restore, as a synchronous wave does. */
fgi_status fgi_invalidate_async(fgi_graph* g, uint32_t n_roots, const uint32_t* roots_dev, const uint8_t* imm_dev,
                                uint64_t* ticket);
fgi_status fgi_wave_wait(fgi_graph* g, uint64_t ticket, uint64_t* out_n, const uint32_t** ids_dev,
                         fgi_wave_stats* stats);
/* The same pair for a host layer that holds its roots and wants its ids in host memory (the scope-dispose
 * flush of `using (Computed.Invalidate())` with ComputedExt.WhenInvalidated awaited later): the roots
 * (boundary handles, as fgi_invalidate) are staged through a pinned buffer of the ticket's own and copied
 * on the graph's stream, so the call returns without waiting; fgi_wave_wait_ids waits like fgi_wave_wait
 * and copies the ticket's ids (ascending) into out_ids (FGI_ECAPACITY with *out_n set if cap is short;
 * out_ids may be NULL for the count). A wave queued after the ticket keeps running during the copy. */
fgi_status fgi_invalidate_async_host(fgi_graph* g, uint32_t n_roots, const uint32_t* roots, const uint8_t* immediately,
                                     uint64_t* ticket);
fgi_status fgi_wave_wait_ids(fgi_graph* g, uint64_t ticket, uint32_t* out_ids, uint64_t cap, uint64_t* out_n,
                             fgi_wave_stats* stats);
/* Page-locked host memory for the calls' host arrays (roots in, ids / bitmaps out): copies from and
 * to it run at full PCIe rate without a staging copy (SURVEY.md §8(b) "Ownership"). */
fgi_status fgi_alloc_pinned(uint64_t bytes, void** out);
fgi_status fgi_free_pinned(void* p);
/* Device pointer to the last wave's invalidated-slot list (valid until the next call). */
fgi_status fgi_wave_ids_dev(fgi_graph* g, const uint32_t** ids_dev, uint64_t* n);
/* Host copy of the last wave's invalidated handles — e.g. the displacement cascade of
 * fgi_begin_compute, whose Invalidated handlers the host must still run. */
fgi_status fgi_last_wave_ids(fgi_graph* g, uint32_t* out_ids, uint64_t cap, uint64_t* out_n);
/* ComputedRegistry.InvalidateEverything (ComputedRegistry.cs:142-147). */
fgi_status fgi_invalidate_all(fgi_graph* g, uint32_t* out_ids, uint64_t cap, uint64_t* out_n,
                              fgi_wave_stats* stats);

/* ---- streaming batches (BASELINE.json configs[4]) ------------------------------- */
/* One step of a batch: the arguments of the matching single call. */
#define FGI_STEP_INVALIDATE 1     /* fgi_invalidate: handles, flags = immediately (nullable) */
#define FGI_STEP_BEGIN_COMPUTE 2  /* fgi_begin_compute: handles = slots, version, flags = has_delay (nullable) */
#define FGI_STEP_ADD_USED 3       /* fgi_add_used: handles = dependants, used */
#define FGI_STEP_SET_OUTPUT 4     /* fgi_set_output: handles */
typedef struct fgi_step {
    uint32_t kind;
    uint32_t n;
    const uint32_t* handles;
    const uint32_t* used;
    const uint64_t* version;
    const uint8_t* flags;
    void* out;   /* nullable: BEGIN_COMPUTE uint32_t detached[n]; ADD_USED uint32_t result[n];
                    SET_OUTPUT uint8_t set[n] */
} fgi_step;

typedef struct fgi_batch_stats {
    uint64_t waves;        /* cascade waves run (steps with a non-empty root set count; empty ones too) */
    uint64_t levels;       /* BFS levels with a non-empty frontier, summed over the waves */
    uint64_t v_inv;        /* Consistent -> Invalidated transitions, summed over the waves */
    uint64_t e_trav;
    uint64_t e_match;
    uint64_t n_flagged;
    double kernel_ms;      /* device time from the batch's first launch to its last (HIP events) */
    double wave_ms;        /* of which the cascades' one-launch waves (HIP events) */
    double total_ms;       /* wall time of the call */
    uint32_t host_syncs;   /* times the call waited for the device */
    uint32_t pad;
} fgi_batch_stats;

/* A host layer's batch of compute-method work in one call: the steps are applied in order, each
 * exactly as the matching single call would apply it (fgi_invalidate, fgi_begin_compute — its
 * displacement cascade included —, fgi_add_used, fgi_set_output — its InvalidateOnSetOutput cascade
 * included; Computed.cs:141-230, 347-385, ComputedRegistry.cs:83-97), but every count stays on the
 * device and each cascade runs as one launch (one block per CU, grid barriers between its levels): the
 * call uploads the batch once and waits for the device once (once more if an add_used step must grow
 * the edge pool, and once more to copy out_ids). out_ids gets the handles invalidated by the batch's
 * cascades, cascade after cascade (each in ascending order); FGI_ECAPACITY with *out_n = the count if
 * cap is too small. If the batch runs out of detached handles, FGI_ECAPACITY names the step: the
 * steps before it are applied, it and the later ones are not. FGI_EINVAL (a bad argument in any step)
 * applies nothing.
 * FGI_EDEVICE if a cascade's grid barrier timed out (blocks of one cascade's grid were not resident
 * together, e.g. other work held the device). The batch is then half-applied: the steps before the
 * failed cascade are, the cascade may have been partly folded into node words, the later steps are
 * not. The graph is poisoned: every later call but fgi_restore, fgi_destroy, fgi_last_error and
 * fgi_set_option returns FGI_ESTATE until fgi_restore brings back the last snapshot (node words, rows,
 * detached handles); without a snapshot, only fgi_destroy remains. This mirrors the reference's
 * "Invalidate never throws" (Computed.cs:200-229) as far as a device fault allows: the failure is
 * reported once and nothing later runs on an undefined registry. */
fgi_status fgi_run_batch(fgi_graph* g, uint32_t n_steps, const fgi_step* steps, uint32_t* out_ids, uint64_t cap,
                         uint64_t* out_n, fgi_batch_stats* stats);

/* ---- graph maintenance ---------------------------------------------------------------------- */
/* One ComputedGraphPruner pass (Internal/ComputedGraphPruner.cs:79-94): PruneUsedBy on every
 * registered Consistent node (Computed.cs:400-419) — keep (slot, tag) iff the slot's current node
 * exists with version == tag — then compact the edge pool. While no mutation and no compaction has
 * happened since the pull dependency lists were built, the version half of that test is read from the
 * liveness the list build recorded per pool entry, and only "current" from a bitmap of the node words
 * (same result, no per-entry gather of the dependant's node word). */
fgi_status fgi_prune(fgi_graph* g, fgi_prune_stats* stats);
/* The same PruneUsedBy pass over the rows of handles [first, first + count) only (one batch of
 * ComputedGraphPruner's walk, ComputedGraphPruner.cs:79-94). Rows are compacted in place: their
 * offsets and capacities stay, the freed entries become slack the rows grow into. fgi_prune visits
 * every row and, when holes exceed FGI_OPT_DEFRAG_PCT of the pool, copies the rows to a fresh pool
 * (each with max(4, len / 8) slack). */
fgi_status fgi_prune_range(fgi_graph* g, uint32_t first, uint32_t count, fgi_prune_stats* stats);
/* Incremental pruning: the next `batch` handles after the previous step's (wrapping around), but
 * only while the engine's estimate of stale entries exceeds stale_pct of the pool (waves add the
 * entries they make stale: the rows of invalidated nodes and the entries pointing at them);
 * otherwise returns at once with zero counts. */
fgi_status fgi_prune_step(fgi_graph* g, uint32_t batch, uint32_t stale_pct, fgi_prune_stats* stats);
/* Release a detached handle once the host no longer references the node. */
fgi_status fgi_release(fgi_graph* g, uint32_t n, const uint32_t* handle);

/* ---- bench / test support ------------------------------------------------------------------- */
/* Save / restore node states and row lengths on the device (reset from a pristine copy).
 * fgi_restore is stream-ordered: it may return before the device copies finish; every later call
 * on the graph runs after them. On a poisoned graph (a failed fgi_run_batch, FGI_EDEVICE) fgi_restore
 * copies back every saved table, clears the wave bitmaps and the detached-handle list to the
 * snapshot's, and makes the graph usable again. fgi_restore refuses (FGI_ESTATE) once the edge pool
 * was rebuilt or rows were compacted since the snapshot (a bulk load, fgi_prune / fgi_prune_range that
 * moved entries, a defragmentation): a poisoned graph then stays poisoned, and fgi_destroy is all that
 * is left for it — take a new snapshot after such a call. */
fgi_status fgi_snapshot(fgi_graph* g);
fgi_status fgi_restore(fgi_graph* g);
/* Device-side synthetic workloads. All nodes Consistent with
 * version (splitmix64(seed ^ slot) & (2^55-1)) | 1. stale_pct% of edges (by hash with
 * stale_seed) carry tag = version + 1. The graph must be empty. */
fgi_status fgi_synth_layered(fgi_graph* g, uint32_t levels, uint32_t width, uint32_t fanout, uint64_t seed);
fgi_status fgi_synth_rmat(fgi_graph* g, uint32_t scale, uint32_t edge_factor, uint64_t seed,
                          uint32_t stale_pct, uint64_t stale_seed);
/* Copy the full edge set (sorted by (used, dependant, tag)) to the host: parity tests. */
fgi_status fgi_export_edges(fgi_graph* g, uint32_t* used, uint32_t* dependant_slot, uint64_t* tag,
                            uint64_t cap, uint64_t* out_n);
/* HIP stream the graph's kernels run on (as void* = hipStream_t) — for event timing in bench. */
fgi_status fgi_stream(fgi_graph* g, void** stream);
/* Traversal options (defaults in brackets). Results never depend on them; they exist so tests can
 * pin each code path and benches can compare them.
 *   FGI_OPT_DEAD_FILTER [1]  skip edges whose dependant was invalidated in an earlier level using
 *                            a per-wave bitmap (E_match then counts examined edges only)
 *   FGI_OPT_DIRECTION   [0]  0 auto (push/pull per level), 1 push only, 2 pull only
 *   FGI_OPT_PULL_ALPHA  [28] auto: pull when frontier edges > total edges / alpha
 *   FGI_OPT_PULL_BETA   [32] auto: after a pull level, pull again while the frontier holds more
 *                            than n_slots / beta nodes (0: the alpha rule only)
 *   FGI_OPT_LEVEL_TIMING [1] with a stats argument, time every level's traversal launch with HIP
 *                            events (per-kernel figures for the roofline); 0 keeps only the
 *                            wave-boundary events, so measured waves carry no per-level markers
 *   FGI_OPT_DEFRAG_PCT  [60] fgi_prune copies the rows to a fresh pool when holes exceed this % of
 *                            it (0: never)
 *   FGI_OPT_PULL_TPB    [0]  pull tiles (1,024 slots) per block, 1..32; 0 sizes the grid from the CU
 *                            count (measurement / tests: results never depend on it)
 *   FGI_OPT_PART_COLLECTIVES [0] a one-rank partition skips its collectives (identities there);
 *                            1 runs them anyway (tests of the RCCL level loop on one GPU)
 *   FGI_OPT_FRONT_EXCHANGE [0] partitions, before a pull level: 0 per level whichever moves fewer
 *                            bytes, 1 all-gather of the whole invalidated bitmap, 2 only the words
 *                            that changed since the previous exchange (8 B each, to every rank);
 *                            all ranks of a partition must set the same value
 *   FGI_OPT_HOT_HEADS   [0]  most list heads a pull level probes through the hot snapshot: 0 sizes
 *                            it from the graph (65,536-262,144); n > 0 caps it at n rounded up to 256,
 *                            so the other heads are probed in the invalidated bitmap itself (tests pin
 *                            that path on small graphs; results never depend on it)
 *   FGI_OPT_PART_PLAN   [1]  partitions: a wave follows the previous wave's directions (when every
 *                            rank can) and queues all its levels' collectives at fixed sizes, with one
 *                            host synchronisation at its end (two with remote ranks: the start's
 *                            all-reduce too); 0 decides every level on the host after an all-reduce.
 *                            All ranks must set the same value
 *   FGI_OPT_PART_BUCKET [0]  partitions, planned waves: words per peer of a push level's bucket (a
 *                            count, then ids; 0 = the allocated 65,536); smaller buckets only delay
 *                            ids to later push levels (tests pin that path; results never change)
 *   FGI_OPT_FAULT_INJECT [0] tests only: value (k << 16) | b, b > 0: in the (k+1)-th streaming
 *                            cascade launched from now (fgi_run_batch), block b - 1 leaves at its first
 *                            grid barrier without arriving, and that cascade's barrier times out after
 *                            20 ms: the failure path runs deterministically (FGI_EDEVICE, then the
 *                            poisoned graph)
 *   FGI_OPT_FAULT_INJECT_TAIL [0] tests only: the same for the (k+1)-th wave tail (the persistent
 *                            launch that runs a wave's last small push levels, synchronous or
 *                            asynchronous waves): fgi_invalidate* / fgi_wave_wait return FGI_EDEVICE and
 *                            the graph is poisoned until fgi_restore */
#define FGI_OPT_DEAD_FILTER 1
#define FGI_OPT_DIRECTION 2
#define FGI_OPT_PULL_ALPHA 3
#define FGI_OPT_LEVEL_TIMING 4
#define FGI_OPT_PULL_BETA 5
#define FGI_OPT_DEFRAG_PCT 6
#define FGI_OPT_PART_COLLECTIVES 7
#define FGI_OPT_PULL_TPB 8
#define FGI_OPT_FRONT_EXCHANGE 9
#define FGI_OPT_HOT_HEADS 10
#define FGI_OPT_FAULT_INJECT 11
#define FGI_OPT_PART_PLAN 13
#define FGI_OPT_PART_BUCKET 14
#define FGI_OPT_FAULT_INJECT_TAIL 16
/* 12 and 15: the measurement variants' options (include/fgi_variants.h); FGI_ENOTSUP here */
fgi_status fgi_set_option(fgi_graph* g, int option, int64_t value);

/* ---- multi-GPU (1-D vertex-range partition, RCCL all-to-all frontier exchange) --------------- */
/* RCCL unique id (128 bytes) made by rank 0 and broadcast by the caller (e.g. torch.distributed). */
fgi_status fgi_part_unique_id(uint8_t* id128);
/* Join the partitioned engine: this graph owns slots [rank*ceil(N/world), ...) of a global
 * N = n_global slots; cfg->rank/world must be set. */
fgi_status fgi_part_init(fgi_graph* g, uint32_t n_global, const uint8_t* id128);
/* Join the partitioned engine with the host's own transport instead of RCCL: every collective of the
 * partition (the waves' exchanges, the mutations' all-reduces, the prune's all-gather) reduces to
 * fn(ctx, send, bytes, recv) — an all-gather of `bytes` from every rank into recv (world * bytes,
 * rank-major; 0 = success), e.g. torch.distributed over gloo. The ranks may then share a GPU (RCCL
 * refuses two ranks on one device): the multi-process path runs on any box. Every collective
 * synchronises the rank's stream (correct, not fast). Same results as fgi_part_init's. */
typedef int (*fgi_allgather_fn)(void* ctx, const void* send, uint64_t bytes, void* recv);
fgi_status fgi_part_init_host(fgi_graph* g, uint32_t n_global, fgi_allgather_fn fn, void* ctx);
/* Partitioned R-MAT: every rank walks the global edge sequence by index (edge i is a pure function of
 * i) and keeps only its share — the rows of its slots and the dependency entries of its slots —
 * without materialising the global edge list. */
fgi_status fgi_part_synth_rmat(fgi_graph* g, uint32_t scale, uint32_t edge_factor, uint64_t seed,
                               uint32_t stale_pct, uint64_t stale_seed);
/* Bulk import into a partitioned graph (ComputedRegistry.Register, ComputedRegistry.cs:72-105, without
 * displacement; the single-device fgi_register_nodes refuses a partition). Every rank is given the
 * same global node list (the host broadcasts it): each rank installs the nodes of the slots it owns
 * and records every listed version in its replica (ver_all), against which it checks the tags of
 * edges into other ranks' slots. No collective runs. */
fgi_status fgi_part_register_nodes(fgi_graph* g, uint32_t n, const uint32_t* slot, const uint64_t* version,
                                   const uint32_t* state_flags);
/* Bulk import of `_usedBy` entries with global ids (IComputedImpl.AddUsedBy body, Computed.cs:381-382;
 * set semantics). Every rank is given the same batch: it keeps the rows of the `used` slots it owns
 * (entries keep global dependant ids) and the dependency entries of the dependants it owns, from
 * which it rebuilds its pull lists (the reference's `_used`, Computed.cs:36, 365-366). No collective
 * runs. The first bulk load of a partition that uses partition codes (labels: automatic from 2^25
 * slots, fgi_config.labels = 1 forces them) also numbers every rank's slots by weight, each rank on
 * its own from the arrays it was given; ranks given different arrays number them differently, and
 * the next collective wave then fails on every rank with FGI_ESTATE. */
fgi_status fgi_part_load_edges(fgi_graph* g, uint64_t m, const uint32_t* used, const uint32_t* dependant,
                               const uint64_t* tag);
/* Collective wave: every rank passes the same global root list; each rank reports the
 * invalidated slots it owns (global ids) and its own share of the statistics. */
fgi_status fgi_part_invalidate(fgi_graph* g, uint32_t n_roots, const uint32_t* roots_dev,
                               const uint8_t* immediately_dev, uint64_t* out_n, fgi_wave_stats* stats);
fgi_status fgi_part_export_ids(fgi_graph* g, uint32_t* out_ids, uint64_t cap, uint64_t* out_n);
/* In-process partition group: `p` graphs (created with rank = i, world = p) emulate p ranks in
 * one process — on one device or several. fgi_part_local_invalidate runs the RCCL path's own level
 * loop on every rank (one host thread per rank); only the collectives differ (device copies
 * between the group's buffers instead of RCCL). Used to test and rehearse the multi-GPU engine on
 * one GPU. */
fgi_status fgi_part_init_local(fgi_graph* const* gs, uint32_t p, uint32_t n_global);
fgi_status fgi_part_local_invalidate(fgi_graph* const* gs, uint32_t p, uint32_t n_roots, const uint32_t* roots,
                                     const uint8_t* immediately /*nullable*/, fgi_wave_stats* stats /*p entries*/);
/* ---- mutations, batches and pruning on a partition ----------------
 * The registry's mutations on a partitioned graph. Every rank makes the same call with the same
 * arguments — global slot ids, the whole batch — in the same order (the host broadcasts them): each
 * rank applies the items of the slots it owns, records every listed version in its replica (ver_all),
 * and joins the call's collectives: the cascades (displacement, InvalidateOnSetOutput, invalidation
 * steps) run as partitioned waves, and an all-reduce carries a pair's state between the ranks owning
 * its two ends. Results are those of the single-device call on the whole graph: out_ids gets this
 * rank's invalidated slots (global ids; cascade after cascade, each ascending).
 *   fgi_part_begin_compute  fgi_begin_compute; out_detached[i]: the detached local handle on the
 *                           slot's owner (FGI_NONE on the other ranks). FGI_ECAPACITY on every rank
 *                           when any rank is out of detached handles (nothing applied)
 *   fgi_part_add_used       fgi_add_used for pairs of global slots (their current nodes); out_result
 *                           (FGI_USED_*) on every rank
 *   fgi_part_set_output     fgi_set_output for global slots; out_set on every rank
 *   fgi_part_invalidate_all fgi_invalidate_all
 *   fgi_part_run_batch      fgi_run_batch's steps (handles are global slots) applied in order; each
 *                           cascade is a partitioned wave
 *   fgi_part_prune          fgi_prune on this rank's rows (an all-gather of the current-node bitmap
 *                           decides the entries into other ranks' slots; no other collective)
 * fgi_part_local_run_batch / fgi_part_local_prune run the same on every rank of an in-process group
 * (fgi_part_init_local): the out arrays are merged (out_detached from each slot's owner; the results
 * every rank computes must agree), out_ids gets rank 0's ids, then rank 1's, ...; stats: p entries. */
fgi_status fgi_part_begin_compute(fgi_graph* g, uint32_t n, const uint32_t* slot, const uint64_t* version,
                                  const uint8_t* has_delay /*nullable*/, uint32_t* out_detached /*nullable*/,
                                  uint32_t* out_ids, uint64_t cap, uint64_t* out_n, fgi_wave_stats* stats);
fgi_status fgi_part_add_used(fgi_graph* g, uint32_t n, const uint32_t* dependant, const uint32_t* used,
                             uint32_t* out_result /*nullable*/);
fgi_status fgi_part_set_output(fgi_graph* g, uint32_t n, const uint32_t* slot, uint8_t* out_set /*nullable*/,
                               uint32_t* out_ids, uint64_t cap, uint64_t* out_n, fgi_wave_stats* stats);
fgi_status fgi_part_invalidate_all(fgi_graph* g, uint32_t* out_ids, uint64_t cap, uint64_t* out_n,
                                   fgi_wave_stats* stats);
fgi_status fgi_part_run_batch(fgi_graph* g, uint32_t n_steps, const fgi_step* steps, uint32_t* out_ids, uint64_t cap,
                              uint64_t* out_n, fgi_batch_stats* stats);
fgi_status fgi_part_prune(fgi_graph* g, fgi_prune_stats* stats);
fgi_status fgi_part_local_run_batch(fgi_graph* const* gs, uint32_t p, uint32_t n_steps, const fgi_step* steps,
                                    uint32_t* out_ids, uint64_t cap, uint64_t* out_n,
                                    fgi_batch_stats* stats /*p entries*/);
fgi_status fgi_part_local_prune(fgi_graph* const* gs, uint32_t p, fgi_prune_stats* stats /*p entries*/);
/* Frontier exchanges of a partition rank so far (full all-gathers, delta exchanges) and the bytes it
 * received through them (FGI_OPT_FRONT_EXCHANGE). */
fgi_status fgi_part_front_stats(fgi_graph* g, uint64_t* full, uint64_t* delta, uint64_t* bytes);
/* ncclGetVersion of the RCCL the engine's collectives are bound to, and the file it was loaded
 * from: /opt/rocm/lib/librccl.so.1 (or $FGI_RCCL_LIBRARY), opened by path with RTLD_LOCAL on first
 * use, so an RCCL the process loaded before (torch's bundled copy) is not the one bound. */
fgi_status fgi_rccl_info(int* version, char* path /*nullable*/, uint64_t cap);

#ifdef __cplusplus
}
#endif
#endif /* FGI_H */
