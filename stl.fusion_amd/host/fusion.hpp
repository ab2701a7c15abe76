// fusion.hpp — host-layer mirror of Stl.Fusion's invalidation API over the fgi C-ABI.
//
// This is the layer a Fusion host keeps in front of the engine. It mirrors:
//   ComputedRegistry.Get / Register / InvalidateEverything / OnRegister / OnUnregister / OnAccess
//                                                   (src/Stl.Fusion/ComputedRegistry.cs:34-147, 172-176)
//   ComputedExt.TryUseExisting / UseNew -> RenewTimeouts -> ReportAccess
//                                                   (Internal/ComputedExt.cs:10-76, Computed.cs:248-262)
//   ComputedExt.WhenInvalidated                      (ComputedExt.cs:99-125): a future completed by the
//                                                   node's Invalidated handler, also across asynchronous
//                                                   (pipelined) waves (fgi_invalidate_async_host)
//   Computed.Invalidate() scope, Computed.IsInvalidating()   (Computed.Static.cs:41-47)
//   IComputed.Invalidate(immediately), ConsistencyState, Version, event Invalidated
//                                                   (Computed.cs:11-26, 84-105, 162)
//   InvalidatedHandlerSet                            (Internal/InvalidatedHandlerSet.cs:3-128)
//   ComputeMethodFunctionBase.Compute -> new Computing node (ComputeMethodFunctionBase.cs:19-27)
//   IComputedImpl.AddUsed, TrySetOutput, UsedBy      (Computed.cs:141-160, 327-385)
//   ComputedGraphPruner pass                         (Internal/ComputedGraphPruner.cs:79-94)
//   RPC replica invalidation: an inbound compute call waits for its computed's invalidation and
//   then sends `$sys-c.Invalidate(callId)` to its peer (Client/Internal/RpcInboundComputeCall.cs:
//   53-62, 102-106) — here a subscription (handle -> peer, call id), delivered per peer in batches
//   after the wave.
// The C# host this stands in for is sketched in INTEGRATION.md ([LibraryImport] stubs); no .NET
// SDK exists in this image, so the mirror is C++ and is exercised by host/test_fusion.cpp.
//
// Threading: one registry = one dispatcher thread (the ABI is externally synchronised). After each
// wave the dispatcher fans the returned ids out (Dispatch):
//   1. in parallel over contiguous id ranges (ids come in ascending order), or over ranges of the
//      wave's invalidated bitmap when the wave returned one (large waves): per-peer call-id lists
//      (subscriptions are consumed: a call completes once), and the ids that have host objects;
//   2. per peer, its call ids in handle order, cut into batches of at most PeerBatch — one sink
//      call per batch (what one `$sys-c.Invalidate` message per peer per batch would carry);
//   3. registry-level batch handlers get the whole id list in chunks of BatchChunk;
//   4. per host object: OnUnregister, then its InvalidatedHandlerSet, each handler exactly once.
#pragma once

#include <cstdint>
#include <deque>
#include <functional>
#include <future>
#include <memory>
#include <stdexcept>
#include <string>
#include <unordered_map>
#include <unordered_set>
#include <vector>

#include "../../include/fgi.h"

namespace fusion {

using LTag = uint64_t;
enum class ConsistencyState : uint32_t { Computing = 0, Consistent = 1, Invalidated = 2 };

class Computed;
class ComputedRegistry;

class FgiError : public std::runtime_error {
   public:
    FgiError(fgi_status s, const std::string& what) : std::runtime_error(what), status(s) {}
    fgi_status status;
};

// A handler's identity is its shared_ptr (the reference compares delegates).
using InvalidatedHandler = std::shared_ptr<const std::function<void(Computed&)>>;

// InvalidatedHandlerSet (Internal/InvalidatedHandlerSet.cs:3-128): empty, one handler, a list of up
// to ListSize, then a hash set. Add of a handler already present is a no-op; Remove keeps the order
// of the rest; Invoke calls each handler once (list order; set order unspecified, as there).
class InvalidatedHandlerSet {
   public:
    static constexpr size_t ListSize = 5;
    void Add(const InvalidatedHandler& h);
    void Remove(const InvalidatedHandler& h);
    void Clear() {
        list_.clear();
        set_.reset();
    }
    size_t Size() const { return set_ ? set_->size() : list_.size(); }
    bool Spilled() const { return (bool)set_; }
    void Invoke(Computed& c) const;

   private:
    std::vector<InvalidatedHandler> list_;                         // <= ListSize entries
    std::unique_ptr<std::unordered_set<InvalidatedHandler>> set_;  // after the list overflows
};

// One Computed instance (a node). Holds the engine handle: the input's slot while it is the
// registered node, or a detached handle once a newer computation displaced it.
class Computed {
   public:
    const std::string& Input() const { return input_; }
    LTag Version() const { return version_; }
    uint32_t Handle() const { return handle_; }
    ConsistencyState State() const;
    uint32_t Flags() const;   // fgi state_flags (InvalidateOnSetOutput, DelayStarted, hasDelay)
    bool IsConsistent() const { return State() == ConsistencyState::Consistent; }
    bool IsInvalidated() const { return State() == ConsistencyState::Invalidated; }
    // IComputed.Invalidate(immediately): inside a Computed.Invalidate() scope the node joins the
    // scope's batch; otherwise one wave runs now.
    void Invalidate(bool immediately = false);
    // event Invalidated += / -= (Computed.cs:84-105): fires once; added after invalidation it fires
    // at once. Returns the handler's identity for RemoveOnInvalidated.
    InvalidatedHandler OnInvalidated(std::function<void(Computed&)> handler);
    void OnInvalidated(const InvalidatedHandler& handler);
    void RemoveOnInvalidated(const InvalidatedHandler& handler);
    std::vector<std::pair<uint32_t, LTag>> UsedBy() const;   // IComputedImpl.UsedBy
    uint32_t UsedCount() const;                               // IComputedImpl.Used.Length
    // ComputedExt.WhenInvalidated (ComputedExt.cs:99-125): ready at once for an Invalidated node, else
    // completed by the node's Invalidated event — after a synchronous wave's fan-out, or when the
    // registry completes the asynchronous wave that invalidated it (Complete / CompletePending). Every call
    // returns the same future.
    std::shared_future<void> WhenInvalidated();

   private:
    friend class ComputedRegistry;
    ComputedRegistry* reg_ = nullptr;
    std::string input_;
    uint32_t slot_ = 0, handle_ = 0;
    LTag version_ = 0;
    bool fired_ = false;
    InvalidatedHandlerSet handlers_;
    std::shared_ptr<std::promise<void>> when_;   // WhenInvalidated's promise, once asked for
    std::shared_future<void> when_f_;
};

// Per-wave fan-out statistics (the last Dispatch).
struct FanoutStats {
    uint64_t ids = 0;            // invalidated handles dispatched
    uint64_t objects = 0;        // of which had host objects (handlers / OnUnregister ran)
    uint64_t calls = 0;          // peer call ids delivered
    uint64_t batches = 0;        // peer sink invocations
    uint32_t peers_hit = 0;      // peers that received at least one batch
    uint32_t threads = 0;        // threads of the parallel phase
    uint32_t bitmap = 0;         // 1: dispatched from the wave's invalidated bitmap (fgi_invalidate_bits)
    double dispatch_ms = 0;      // whole Dispatch
    double gather_ms = 0;        // parallel phase (subscriptions -> per-peer lists)
    std::vector<uint64_t> peer_calls, peer_batches;   // per peer id
};

class ComputedRegistry {
   public:
    ComputedRegistry(uint32_t n_slots, uint32_t n_detached = 1024, int device = 0);
    ~ComputedRegistry();
    ComputedRegistry(const ComputedRegistry&) = delete;
    ComputedRegistry& operator=(const ComputedRegistry&) = delete;

    // ComputedRegistry.Get: the current (registered, not invalidated) node of an input, or null
    std::shared_ptr<Computed> Get(const std::string& input);
    // ComputeMethodFunctionBase.Compute: a new Computing node of `input` replaces (and, per
    // Register, invalidates) the current one
    std::shared_ptr<Computed> BeginCompute(const std::string& input, bool has_delay = false);
    // dependant.AddUsed(used); returns the FGI_USED_* outcome (FGI_USED_ESTATE = the reference throws)
    uint32_t AddUsed(Computed& dependant, Computed& used);
    // TrySetOutput: true if the node was Computing; an InvalidateOnSetOutput node cascades at once
    bool SetOutput(Computed& c);
    void InvalidateEverything();
    // one ComputedGraphPruner pass; returns (old, new) `_usedBy` totals of the pruned nodes
    std::pair<uint64_t, uint64_t> Prune();

    // ComputedExt.TryUseExisting with no call options (Internal/ComputedExt.cs:10-23): the input's
    // Consistent current node, made a dependency of usedBy (nullable) and reported as accessed
    // (RenewTimeouts(true) -> OnAccess); null if there is none (the caller computes it)
    std::shared_ptr<Computed> TryUseExisting(const std::string& input, Computed* usedBy = nullptr);
    // CallOptions.GetExisting (ComputedExt.cs:38-42): the current node in any state, reported as
    // accessed with isNew = false unless it is Invalidated (RenewTimeouts returns early then)
    std::shared_ptr<Computed> GetExisting(const std::string& input);
    // ComputedExt.UseNew (ComputedExt.cs:70-76) after a computation: AddUsed from usedBy, then the access
    // report with isNew = true
    void UseNew(Computed& computed, Computed* usedBy = nullptr);

    // `using (Computed.Invalidate()) { ... }`: roots collected while the scope is open are
    // invalidated as one batched wave when the outermost scope closes.
    class InvalidationScope {
       public:
        explicit InvalidationScope(ComputedRegistry* r) : r_(r) { ++r_->scope_depth_; }
        InvalidationScope(InvalidationScope&& o) noexcept : r_(o.r_) { o.r_ = nullptr; }
        ~InvalidationScope() {
            if (r_ && --r_->scope_depth_ == 0) r_->FlushScope();
        }

       private:
        ComputedRegistry* r_;
    };
    InvalidationScope Invalidate() { return InvalidationScope(this); }
    bool IsInvalidating() const { return scope_depth_ > 0; }
    // The same scope, flushed as an asynchronous wave (fgi_invalidate_async_host): closing the outermost
    // scope queues the wave and returns; the nodes' Invalidated handlers (and WhenInvalidated futures) run
    // when the registry completes the wave — Complete(ticket), CompletePending(), or any other registry
    // call, which completes the waves in flight first. LastTicket() names the last queued wave.
    InvalidationScope InvalidateAsync() {
        async_scope_ = true;
        return InvalidationScope(this);
    }
    uint64_t LastTicket() const { return last_ticket_; }
    // Queue one wave from slot / handle roots without waiting (what an async scope's flush does)
    uint64_t InvalidateSlotsAsync(const std::vector<uint32_t>& roots, const std::vector<uint8_t>* immediately = nullptr);
    // Wait for the asynchronous waves up to `ticket` (in order) and fan their results out (Dispatch)
    void Complete(uint64_t ticket);
    void CompletePending();
    size_t PendingWaves() const { return pending_.size(); }
    // `_ = svc.Get(input)` inside a scope: TryUseExisting's Invalidate branch (ComputedExt.cs:29-35)
    void InvalidateInput(const std::string& input);
    // Slot-level roots (inputs already resolved by the host, e.g. bulk-registered nodes)
    void InvalidateSlots(const std::vector<uint32_t>& slots);

    // ---- RPC replica fan-out -----------------------------------------------------------------
    // A peer's sink receives its invalidated call ids, in handle order, PeerBatch at most per call.
    using PeerSink = std::function<void(uint32_t peer, const uint64_t* call_ids, size_t n)>;
    uint32_t AddPeer(PeerSink sink);
    // An inbound compute call of `peer` (call id) now waits for the node `handle`'s invalidation.
    void Subscribe(uint32_t handle, uint32_t peer, uint64_t call_id);
    void Subscribe(size_t n, const uint32_t* handles, const uint32_t* peers, const uint64_t* call_ids);
    size_t PeerBatch = 4096;
    uint32_t FanoutThreads = 0;   // 0: hardware concurrency, capped at 16

    // how a wave's invalidated set comes back: 0 auto (the bitmap once the previous wave invalidated
    // more than 1/32 of the handles), 1 the id list, 2 the bitmap (fgi_invalidate_bits)
    int WaveOutput = 0;

    std::function<void(Computed&)> OnRegister, OnUnregister;
    // event OnAccess (ComputedRegistry.cs:36, ReportAccess 172-176): a compute-method node was used —
    // isNew is RenewTimeouts' argument (TryUseExisting / UseNew: true, GetExisting: false)
    std::function<void(Computed&, bool)> OnAccess;
    // registry-level handler class: the wave's invalidated handles, BatchChunk at a time
    std::function<void(const uint32_t* ids, size_t n)> OnInvalidatedBatch;
    size_t BatchChunk = 65536;

    fgi_graph* Graph() const { return g_; }
    const fgi_wave_stats& LastWave() const { return last_; }
    const FanoutStats& LastFanout() const { return fan_; }

   private:
    friend class Computed;
    struct Sub {
        uint64_t call_id;
        uint32_t peer, next;
    };
    void Check(fgi_status s, const char* what) const;
    uint32_t SlotOf(const std::string& input, bool create);
    void RunWave(const uint32_t* roots, size_t n, const uint8_t* imm);
    // the engine's ids of the last call into ids_ (grown without zero-fill, reused across waves)
    uint32_t* IdsBuffer(uint64_t need);
    void Dispatch(const uint32_t* ids, uint64_t n);
    void DispatchBits(const uint64_t* bits, uint64_t words, uint64_t n);
    void DispatchImpl(const uint32_t* ids, const uint64_t* bits, uint64_t words, uint64_t n);
    void FlushScope();
    void ReportAccess(Computed& c, bool is_new);
    LTag NextVersion(LTag current);
    void MoveSubs(uint32_t from, uint32_t to);

    fgi_graph* g_ = nullptr;
    uint32_t n_slots_ = 0, n_handles_ = 0;
    std::unordered_map<std::string, uint32_t> slots_;
    std::vector<std::shared_ptr<Computed>> current_;                 // slot -> newest node
    std::unordered_map<uint32_t, std::shared_ptr<Computed>> detached_;  // detached handle -> node
    std::vector<uint8_t> has_obj_;                                   // handle -> host object exists
    std::vector<uint32_t> scope_roots_;
    std::vector<uint8_t> scope_imm_;
    int scope_depth_ = 0;
    bool async_scope_ = false;               // the outermost open scope flushes asynchronously
    std::deque<uint64_t> pending_;           // asynchronous waves queued, not yet completed (ticket order)
    uint64_t last_ticket_ = 0;
    LTag ltag_ = 0x100000;
    fgi_wave_stats last_{};
    FanoutStats fan_;
    std::unique_ptr<uint32_t[]> ids_;
    uint64_t ids_cap_ = 0;
    std::unique_ptr<uint64_t[]> bits_;   // the last bitmap-mode wave's invalidated bitmap
    uint64_t pred_v_ = 0;                // the previous wave's V_inv (picks the output form)
    // subscriptions: per handle a singly-linked list in one pool (kNone-terminated), free list
    std::vector<PeerSink> peers_;
    std::vector<uint32_t> sub_head_;
    std::vector<Sub> subs_;
    std::vector<uint32_t> sub_free_;
};

}  // namespace fusion
