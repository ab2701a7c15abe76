/*
 * fgo.h — TEST INFRASTRUCTURE ONLY. CPU oracle for the cascading-invalidation path.
 *
 * This is a plain C++ restatement of Stl.Fusion's `Computed.Invalidate()` cascade and the
 * graph operations around it, used (a) by tests/ as the parity checker for the HIP engine and
 * (b) by bench.py's `cpu_baseline` leg as the host-CPU reference timing. Nothing in the
 * product (stl.fusion_amd/, include/fgi.h) links, loads or calls it.
 *
 * Pinning: the reference is C# and no .NET toolchain exists in this image, so
 * the reference cannot be built or run here and it holds no numeric golden vectors. The oracle
 * is pinned against the reference's own behavioural tests, restated as known-answer scenarios in
 * tests/test_oracle_scenarios.py (CounterServiceTest, SimplestProviderTest, MutableStateTest,
 * UserProviderTest.InvalidateEverythingTest, NestedOperationLoggerTest, EdgeCaseServiceTest,
 * HashSetSlimTest set semantics). Large-graph outputs have no reference vectors: "parity
 * unpinned" beyond those behaviour pins.
 *
 * Model (follows the reference object graph, not the engine's slot layout):
 *   - a node is a `Computed` instance (src/Stl.Fusion/Computed.cs:28-39): input slot, version,
 *     state, flags, hasDelay (= Options.InvalidationDelay != 0), `_used` (RefHashSetSlim3 of
 *     nodes) and `_usedBy` (HashSetSlim3 of (slot, version));
 *   - the registry maps slot -> current node (src/Stl.Fusion/ComputedRegistry.cs:22, 57-132);
 *   - node handles are arena indices; a slot may have several nodes over time.
 */
#ifndef FGO_H
#define FGO_H
#include <stdint.h>
#include <stddef.h>

#ifdef __cplusplus
extern "C" {
#endif

#define FGO_NONE 0xFFFFFFFFu

/* ConsistencyState (src/Stl.Fusion/ConsistencyState.cs:5-10) */
#define FGO_COMPUTING 0u
#define FGO_CONSISTENT 1u
#define FGO_INVALIDATED 2u
/* state_flags packing shared with include/fgi.h: bits 0-1 state, bit 2 InvalidateOnSetOutput,
 * bit 3 InvalidationDelayStarted (ComputedFlags.cs:4-8), bit 4 hasDelay. */
#define FGO_F_IOSO 4u
#define FGO_F_DELAY_STARTED 8u
#define FGO_F_HAS_DELAY 16u

/* AddUsed outcome codes (Computed.cs:347-385) — identical values to FGI_USED_* */
#define FGO_USED_ADDED 0u           /* edge (dst.slot, dst.version) added to src._usedBy */
#define FGO_USED_DROPPED 1u         /* dependant no longer Computing: call is a no-op (351-364) */
#define FGO_USED_INVALIDATED 2u     /* src already Invalidated: dependant.Invalidate() (376-378) */
#define FGO_USED_ESTATE 3u          /* src is Computing: the reference throws (374-375) */

typedef struct fgo fgo;

typedef struct fgo_stats {
    uint64_t v_inv;      /* Consistent -> Invalidated transitions */
    uint64_t e_trav;     /* sum of |_usedBy| over invalidated nodes */
    uint64_t e_match;    /* traversed edges whose tag equals the dst slot's node version at wave start */
    uint64_t n_flagged;  /* visits that set a flag (Computing -> IOSO, delay -> DelayStarted) */
    uint64_t wall_ns;    /* wall time of the cascade(s) */
    uint32_t threads;
    uint32_t pad;
} fgo_stats;

fgo* fgo_create(uint32_t n_slots);
void fgo_destroy(fgo* o);

/* Bulk import: one Consistent/Computing node per slot with version != 0 (registered), and the
 * reverse edges src._usedBy += (dst, tag). If node(dst).version == tag, src is also added to
 * dst._used (the forward link AddUsed would have created). Set semantics (HashSetSlim3). */
int fgo_load_graph(fgo* o, uint32_t n, const uint64_t* version, const uint32_t* state_flags,
                   uint64_t m, const uint32_t* src, const uint32_t* dst, const uint64_t* tag);

/* Worker threads for the bulk operations (fgo_load_graph, snapshot/restore, fgo_gen_rmat,
 * fgo_gen_tags); default 1. Results are identical for any value. */
void fgo_set_threads(uint32_t n);
uint32_t fgo_get_threads(void);

uint32_t fgo_current(const fgo* o, uint32_t slot);   /* registry Get (ComputedRegistry.cs:57-70) */
uint32_t fgo_last(const fgo* o, uint32_t slot);      /* most recently created node of the slot */
uint32_t fgo_node_count(const fgo* o);
/* Canonical node state: flags of an Invalidated node and IOSO of a non-Computing node are
 * unobservable in the reference (Computed.cs:145,164-172) and reported as 0. */
int fgo_node_info(const fgo* o, uint32_t h, uint32_t* slot, uint64_t* version, uint32_t* state_flags);
/* Per-slot canonical state of fgo_last(slot) (version 0 / flags 0 for never-used slots). */
void fgo_dump_states(const fgo* o, uint64_t* version, uint32_t* state_flags);

/* ComputeMethodFunctionBase.Compute (ComputeMethodFunctionBase.cs:19-27) + Register with
 * displacement (ComputedRegistry.cs:72-105). Returns the new node handle in *out_new and the
 * displaced node (if one was current) in *out_displaced (FGO_NONE otherwise). */
int fgo_begin_compute(fgo* o, uint32_t slot, uint64_t version, int has_delay,
                      uint32_t* out_new, uint32_t* out_displaced, fgo_stats* st);
/* TrySetOutput (Computed.cs:141-160): 1 if the node was Computing, else 0. */
int fgo_set_output(fgo* o, uint32_t h, fgo_stats* st);
/* dependant.AddUsed(used) (Computed.cs:347-368): returns an FGO_USED_* code. */
uint32_t fgo_add_used(fgo* o, uint32_t dependant_h, uint32_t used_h, fgo_stats* st);
/* The three calls above over slots (each resolved to fgo_last(slot)), one by one in order.
 * has_delay and out_codes may be NULL. fgo_set_output_n returns how many nodes were Computing. */
int fgo_begin_compute_n(fgo* o, uint32_t n, const uint32_t* slots, const uint64_t* versions,
                        const uint8_t* has_delay, fgo_stats* st);
uint32_t fgo_set_output_n(fgo* o, uint32_t n, const uint32_t* slots, fgo_stats* st);
void fgo_add_used_n(fgo* o, uint32_t n, const uint32_t* dependant_slots, const uint32_t* used_slots,
                    uint32_t* out_codes, fgo_stats* st);

/* `using (Computed.Invalidate()) svc.Get(slot)` for each root slot in order
 * (Internal/ComputedExt.cs:29-35 -> Computed.cs:162-230). immediately may be NULL.
 * n_threads > 1 splits roots round-robin across threads (parallel-over-roots baseline). */
int fgo_invalidate_slots(fgo* o, uint32_t n, const uint32_t* slots, const uint8_t* immediately,
                         uint32_t n_threads, fgo_stats* st);
/* IComputed.Invalidate(immediately) on node handles (e.g. a delay timer firing). */
int fgo_invalidate_nodes(fgo* o, uint32_t n, const uint32_t* handles, const uint8_t* immediately,
                         fgo_stats* st);
/* ComputedRegistry.InvalidateEverything (ComputedRegistry.cs:142-147). */
int fgo_invalidate_everything(fgo* o, fgo_stats* st);
/* ComputedGraphPruner pass: PruneUsedBy on every registered Consistent node
 * (ComputedGraphPruner.cs:79-94, Computed.cs:400-419). */
int fgo_prune(fgo* o, uint64_t* old_edges, uint64_t* new_edges);
/* The same over the registered slots in [first, first + count) (one batch of the pruner's walk). */
int fgo_prune_range(fgo* o, uint32_t first, uint32_t count, uint64_t* old_edges, uint64_t* new_edges);

/* Slots invalidated since the last fgo_clear_log, in transition order. */
uint64_t fgo_inv_log(const fgo* o, uint32_t* out, uint64_t cap);
void fgo_clear_log(fgo* o);

/* IComputedImpl.UsedBy / Used (Computed.cs:327-345). */
uint64_t fgo_used_by(const fgo* o, uint32_t h, uint32_t* dst, uint64_t* tag, uint64_t cap);
uint32_t fgo_used_count(const fgo* o, uint32_t h);
uint64_t fgo_total_used_by(const fgo* o);   /* sum of |_usedBy| over all live nodes */
/* Every slot's most recent node's `_usedBy` entries as (slot, dependant slot, tag) triples, slots
 * ascending (test bulk export; *_used_by per node for the same thing one node at a time). */
uint64_t fgo_export_used_by(const fgo* o, uint32_t* slot, uint32_t* dst, uint64_t* tag, uint64_t cap);

/* Snapshot / restore of the whole object graph (bench: reset from a pristine copy). */
int fgo_snapshot(fgo* o);
int fgo_restore(fgo* o);

/* ---- synthetic workloads (the engine has its own device generator) ---- */
uint64_t fgo_splitmix64(uint64_t x);
uint64_t fgo_version_of(uint64_t seed, uint32_t slot);
/* Config 1: levels x width nodes; every node of level >= 1 uses `fanout` distinct nodes of the
 * previous level. Writes edges sorted by (src, dst). Returns m (call with NULL to size). */
uint64_t fgo_gen_layered(uint32_t levels, uint32_t width, uint32_t fanout, uint64_t seed,
                         uint32_t* src, uint32_t* dst);
/* R-MAT (a,b,c) = (0.57,0.19,0.19) with a bijective vertex scramble, deduplicated, sorted by
 * (src, dst). Returns m (unique edges). Call with NULL to get the count. */
uint64_t fgo_gen_rmat(uint32_t scale, uint32_t edge_factor, uint64_t seed, uint32_t* src, uint32_t* dst);
/* Edge tags: ver(dst), or ver(dst)+1 when the edge is stale (p = stale_p_pct / 100 by hash). */
void fgo_gen_tags(uint64_t m, const uint32_t* src, const uint32_t* dst, uint64_t ver_seed,
                  uint32_t stale_pct, uint64_t stale_seed, uint64_t* tag);
/* Distinct roots with out-degree > 0 drawn from splitmix64(seed + k) % range. */
uint32_t fgo_gen_roots(uint32_t n_roots, uint32_t range, uint64_t seed, const uint32_t* out_degree,
                       uint32_t* roots);

#ifdef __cplusplus
}
#endif
#endif
