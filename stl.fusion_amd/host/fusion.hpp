// fusion.hpp — host-layer mirror of Stl.Fusion's invalidation API over the fgi C-ABI.
//
// This is the layer a Fusion host keeps in front of the engine. It mirrors:
//   ComputedRegistry.Get / Register / InvalidateEverything / OnRegister / OnUnregister
//                                                   (src/Stl.Fusion/ComputedRegistry.cs:34-147)
//   Computed.Invalidate() scope, Computed.IsInvalidating()   (Computed.Static.cs:41-47)
//   IComputed.Invalidate(immediately), ConsistencyState, Version, event Invalidated
//                                                   (Computed.cs:11-26, 84-105, 162)
//   ComputeMethodFunctionBase.Compute -> new Computing node (ComputeMethodFunctionBase.cs:19-27)
//   IComputedImpl.AddUsed, TrySetOutput, UsedBy      (Computed.cs:141-160, 327-385)
//   ComputedGraphPruner pass                         (Internal/ComputedGraphPruner.cs:79-94)
// The C# host this stands in for is sketched in INTEGRATION.md ([LibraryImport] stubs); no .NET
// SDK exists in this image, so the mirror is C++ and is exercised by host/test_fusion.cpp.
//
// Threading: one registry = one dispatcher thread (the ABI is externally synchronised). Invalidated
// handlers run on that thread after each wave, each exactly once (InvalidatedHandlerSet.cs:100-127).
#pragma once

#include <cstdint>
#include <functional>
#include <memory>
#include <stdexcept>
#include <string>
#include <unordered_map>
#include <vector>

#include "../../include/fgi.h"

namespace fusion {

using LTag = uint64_t;
enum class ConsistencyState : uint32_t { Computing = 0, Consistent = 1, Invalidated = 2 };

class ComputedRegistry;

class FgiError : public std::runtime_error {
   public:
    FgiError(fgi_status s, const std::string& what) : std::runtime_error(what), status(s) {}
    fgi_status status;
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
    // event Invalidated: fires once; added after invalidation it fires at once (Computed.cs:84-97)
    void OnInvalidated(std::function<void(Computed&)> handler);
    std::vector<std::pair<uint32_t, LTag>> UsedBy() const;   // IComputedImpl.UsedBy
    uint32_t UsedCount() const;                               // IComputedImpl.Used.Length

   private:
    friend class ComputedRegistry;
    ComputedRegistry* reg_ = nullptr;
    std::string input_;
    uint32_t slot_ = 0, handle_ = 0;
    LTag version_ = 0;
    bool fired_ = false;
    std::vector<std::function<void(Computed&)>> handlers_;
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
    // `_ = svc.Get(input)` inside a scope: TryUseExisting's Invalidate branch (ComputedExt.cs:29-35)
    void InvalidateInput(const std::string& input);

    std::function<void(Computed&)> OnRegister, OnUnregister;
    fgi_graph* Graph() const { return g_; }
    const fgi_wave_stats& LastWave() const { return last_; }

   private:
    friend class Computed;
    void Check(fgi_status s, const char* what) const;
    uint32_t SlotOf(const std::string& input, bool create);
    void RunWave(const std::vector<uint32_t>& roots, const std::vector<uint8_t>& imm);
    void Dispatch(const uint32_t* ids, uint64_t n);
    void FlushScope();
    LTag NextVersion(LTag current);

    fgi_graph* g_ = nullptr;
    uint32_t n_slots_ = 0;
    std::unordered_map<std::string, uint32_t> slots_;
    std::vector<std::shared_ptr<Computed>> current_;                 // slot -> newest node
    std::unordered_map<uint32_t, std::shared_ptr<Computed>> detached_;  // detached handle -> node
    std::vector<uint32_t> scope_roots_;
    std::vector<uint8_t> scope_imm_;
    int scope_depth_ = 0;
    LTag ltag_ = 0x100000;
    fgi_wave_stats last_{};
};

}  // namespace fusion
