// fusion.cpp — implementation of the host-layer mirror (see fusion.hpp).
#include "fusion.hpp"

#include <algorithm>
#include <chrono>
#include <thread>

namespace fusion {

namespace {
constexpr uint32_t kNone = 0xFFFFFFFFu;
constexpr uint64_t kParallelMin = 1u << 16;   // ids below this fan out on the dispatcher thread

double ms_since(std::chrono::steady_clock::time_point t0) {
    return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
}
}  // namespace

// ---- InvalidatedHandlerSet ------------------------------------------------------------------------
void InvalidatedHandlerSet::Add(const InvalidatedHandler& h) {
    if (!h) return;
    if (set_) {
        set_->insert(h);
        return;
    }
    for (const auto& x : list_)
        if (x == h) return;
    if (list_.size() < ListSize) {
        list_.push_back(h);
        return;
    }
    set_ = std::make_unique<std::unordered_set<InvalidatedHandler>>(list_.begin(), list_.end());
    set_->insert(h);
    list_.clear();
}

void InvalidatedHandlerSet::Remove(const InvalidatedHandler& h) {
    if (!h) return;
    if (set_) {
        set_->erase(h);
        return;
    }
    auto it = std::find(list_.begin(), list_.end(), h);
    if (it != list_.end()) list_.erase(it);
}

void InvalidatedHandlerSet::Invoke(Computed& c) const {
    if (set_) {
        for (const auto& h : *set_) (*h)(c);
        return;
    }
    for (const auto& h : list_) (*h)(c);
}

// ---- registry -------------------------------------------------------------------------------------
ComputedRegistry::ComputedRegistry(uint32_t n_slots, uint32_t n_detached, int device) : n_slots_(n_slots) {
    fgi_config cfg{};
    cfg.struct_size = sizeof(cfg);
    cfg.device = device;
    cfg.n_slots = n_slots;
    cfg.n_detached = n_detached;
    cfg.world = 1;
    fgi_status s = fgi_create(&cfg, &g_);
    if (s != FGI_OK) throw FgiError(s, "fgi_create failed (no GPU?)");
    n_handles_ = n_slots + n_detached;
    current_.resize(n_slots);
    has_obj_.assign(n_handles_, 0);
}

ComputedRegistry::~ComputedRegistry() { fgi_destroy(g_); }

void ComputedRegistry::Check(fgi_status s, const char* what) const {
    if (s != FGI_OK) throw FgiError(s, std::string(what) + ": " + fgi_last_error(g_));
}

uint32_t ComputedRegistry::SlotOf(const std::string& input, bool create) {
    auto it = slots_.find(input);
    if (it != slots_.end()) return it->second;
    if (!create) return FGI_NONE;
    if (slots_.size() >= n_slots_) throw FgiError(FGI_ECAPACITY, "registry is full");
    const uint32_t s = (uint32_t)slots_.size();
    slots_.emplace(input, s);
    return s;
}

// LTagVersionGenerator.NextVersion (LTagVersionGenerator.cs:13-20): a fresh positive tag != current
LTag ComputedRegistry::NextVersion(LTag current) {
    do {
        ltag_ = ((ltag_ + 1) & ((1ull << 55) - 1));
    } while (ltag_ == 0 || ltag_ == current);
    return ltag_;
}

uint32_t* ComputedRegistry::IdsBuffer(uint64_t need) {
    if (need > ids_cap_) {
        const uint64_t cap = std::max<uint64_t>(need, ids_cap_ + ids_cap_ / 2);
        ids_.reset(new uint32_t[cap]);   // default-initialised: no zero-fill
        ids_cap_ = cap;
    }
    return ids_.get();
}

std::shared_ptr<Computed> ComputedRegistry::Get(const std::string& input) {
    CompletePending();
    const uint32_t s = SlotOf(input, false);
    if (s == FGI_NONE || !current_[s]) return nullptr;
    const ConsistencyState st = current_[s]->State();
    if (st == ConsistencyState::Invalidated) return nullptr;   // unregistered on invalidation
    return current_[s];
}

void ComputedRegistry::MoveSubs(uint32_t from, uint32_t to) {
    if (from >= sub_head_.size() || sub_head_[from] == kNone) return;
    if (to >= sub_head_.size()) sub_head_.resize(n_handles_, kNone);
    sub_head_[to] = sub_head_[from];
    sub_head_[from] = kNone;
}

std::shared_ptr<Computed> ComputedRegistry::BeginCompute(const std::string& input, bool has_delay) {
    CompletePending();
    const uint32_t s = SlotOf(input, true);
    auto c = std::make_shared<Computed>();
    c->reg_ = this;
    c->input_ = input;
    c->slot_ = s;
    c->handle_ = s;
    c->version_ = NextVersion(current_[s] ? current_[s]->version_ : 0);
    const uint8_t hd = has_delay ? 1 : 0;
    uint32_t detached = FGI_NONE;
    fgi_wave_stats ws{};
    Check(fgi_begin_compute(g_, 1, &s, &c->version_, &hd, &detached, &ws), "fgi_begin_compute");
    auto old = current_[s];
    if (detached != FGI_NONE) {   // displaced but alive (Computing / delayed): its handle moves
        if (old) {
            old->handle_ = detached;
            detached_[detached] = old;
            has_obj_[detached] = 1;
        }
        MoveSubs(s, detached);   // the replicas follow the old node
    }
    // the displacement cascade's invalidated nodes (the old node among them) get their handlers
    if (ws.v_inv) {
        uint64_t n = 0;
        uint32_t* ids = IdsBuffer(ws.v_inv);
        Check(fgi_last_wave_ids(g_, ids, ws.v_inv, &n), "fgi_last_wave_ids");
        last_ = ws;
        Dispatch(ids, n);
    }
    current_[s] = c;
    has_obj_[s] = 1;
    if (OnRegister) OnRegister(*c);
    return c;
}

uint32_t ComputedRegistry::AddUsed(Computed& dependant, Computed& used) {
    CompletePending();
    uint32_t out = 0;
    const uint32_t d = dependant.handle_, u = used.handle_;
    Check(fgi_add_used(g_, 1, &d, &u, &out), "fgi_add_used");
    return out;
}

bool ComputedRegistry::SetOutput(Computed& c) {
    CompletePending();
    uint8_t set = 0;
    const uint32_t h = c.handle_;
    uint64_t n = 0;
    uint32_t* ids = IdsBuffer(1024);
    fgi_status s = fgi_set_output(g_, 1, &h, &set, ids, ids_cap_, &n, &last_);
    if (s == FGI_ECAPACITY) {   // the cascade completed; fetch its ids with the right size
        ids = IdsBuffer(n);
        s = fgi_last_wave_ids(g_, ids, n, &n);
    }
    Check(s, "fgi_set_output");
    Dispatch(ids, n);
    return set != 0;
}

void ComputedRegistry::RunWave(const uint32_t* roots, size_t n_roots, const uint8_t* imm) {
    CompletePending();
    uint64_t n = 0;
    last_ = fgi_wave_stats{};
    // the bitmap (n_handles / 8 bytes) costs less to bring back than the id list (4 B per node) once a
    // wave invalidates more than 1/32 of the handles; the previous wave's size predicts this one's
    const uint64_t words = ((uint64_t)n_handles_ + 63) / 64;
    const bool use_bits = WaveOutput == 2 || (WaveOutput == 0 && pred_v_ * 32 > (uint64_t)n_handles_);
    if (use_bits) {
        if (!bits_) bits_.reset(new uint64_t[words]);
        uint64_t* bits = bits_.get();
        Check(fgi_invalidate_bits(g_, (uint32_t)n_roots, roots, imm, bits, words, &n, &last_), "fgi_invalidate_bits");
        pred_v_ = n;
        DispatchBits(bits, words, n);
        return;
    }
    uint32_t* ids = IdsBuffer(1024);
    fgi_status s = fgi_invalidate(g_, (uint32_t)n_roots, roots, imm, ids, ids_cap_, &n, &last_);
    if (s == FGI_ECAPACITY) {   // the wave itself completed; fetch the ids with the right size
        ids = IdsBuffer(n);
        s = fgi_last_wave_ids(g_, ids, n, &n);
    }
    Check(s, "fgi_invalidate");
    pred_v_ = n;
    Dispatch(ids, n);
}

// The post-wave fan-out (fusion.hpp, "Threading"). Reference: InvalidatedHandlerSet.Invoke
// (Internal/InvalidatedHandlerSet.cs:100-127) per node; one `$sys-c.Invalidate` per replica call
// (Client/Internal/RpcInboundComputeCall.cs:53-62, 102-106), batched per peer here.
// Reentrant: peer sinks, batch handlers and Invalidated handlers are user code and may run waves
// themselves (a handler invalidating another node is the reference's normal pattern). While this
// fan-out runs it owns the ids buffer (a nested wave gets a fresh one) and its host objects are
// resolved before the first callback, so a nested BeginCompute that replaces a slot's node cannot
// redirect this wave's handlers to the new node.
void ComputedRegistry::Dispatch(const uint32_t* ids, uint64_t n) { DispatchImpl(ids, nullptr, 0, n); }

// The same fan-out over the wave's invalidated bitmap (fgi_invalidate_bits): each gather thread
// decodes its own range of words, so the ids are never materialised as a list (unless a batch
// handler wants them: chunks of BatchChunk are decoded for it).
void ComputedRegistry::DispatchBits(const uint64_t* bits, uint64_t words, uint64_t n) {
    DispatchImpl(nullptr, bits, words, n);
}

void ComputedRegistry::DispatchImpl(const uint32_t* ids, const uint64_t* bits, uint64_t words, uint64_t n) {
    const auto t0 = std::chrono::steady_clock::now();
    std::unique_ptr<uint32_t[]> own;
    uint64_t own_cap = 0;
    if (ids_ && ids && ids == ids_.get()) {
        own = std::move(ids_);
        own_cap = ids_cap_;
        ids_cap_ = 0;
    }
    std::unique_ptr<uint64_t[]> own_bits;
    if (bits_ && bits && bits == bits_.get()) own_bits = std::move(bits_);
    const uint32_t P = (uint32_t)peers_.size();
    FanoutStats fan;
    fan.ids = n;
    fan.peer_calls.assign(P, 0);
    fan.peer_batches.assign(P, 0);
    // 1. parallel gather: per thread, per peer call ids (ids ascending -> handle order), freed
    //    subscription entries, and the host objects of the ids (read-only lookups)
    uint32_t T = 1;
    if (n >= kParallelMin) {
        T = FanoutThreads ? FanoutThreads : std::min(16u, std::max(1u, std::thread::hardware_concurrency()));
        T = (uint32_t)std::min<uint64_t>(T, (n + kParallelMin - 1) / kParallelMin * 4);
    }
    fan.threads = T;
    fan.bitmap = bits ? 1u : 0u;
    struct Part {
        std::vector<std::vector<uint64_t>> calls;
        std::vector<uint32_t> freed;
        std::vector<std::pair<uint32_t, std::shared_ptr<Computed>>> objs;
    };
    std::vector<Part> parts(T);
    const bool any_subs = !subs_.empty() && !sub_head_.empty();
    auto gather = [&](uint32_t t) {
        Part& pt = parts[t];
        pt.calls.resize(P);
        auto visit = [&](const uint32_t h) {
            if (h >= n_handles_) return;
            if (has_obj_[h]) {
                std::shared_ptr<Computed> c;
                if (h < n_slots_) {
                    c = current_[h];
                } else {
                    auto it = detached_.find(h);
                    if (it != detached_.end()) c = it->second;
                }
                pt.objs.emplace_back(h, std::move(c));
            }
            if (!any_subs || h >= sub_head_.size()) return;
            uint32_t e = sub_head_[h];
            if (e == kNone) return;
            sub_head_[h] = kNone;   // a call completes once (each handle is in one range only)
            while (e != kNone) {
                const Sub& sb = subs_[e];
                pt.calls[sb.peer].push_back(sb.call_id);
                pt.freed.push_back(e);
                e = sb.next;
            }
        };
        if (bits) {   // ascending handles of this thread's words
            const uint64_t lo = words * t / T, hi = words * (t + 1) / T;
            for (uint64_t w = lo; w < hi; ++w)
                for (uint64_t m = bits[w]; m; m &= m - 1) visit((uint32_t)(w * 64 + (uint64_t)__builtin_ctzll(m)));
        } else {
            const uint64_t lo = n * t / T, hi = n * (t + 1) / T;
            for (uint64_t i = lo; i < hi; ++i) visit(ids[i]);
        }
    };
    if (T == 1) {
        gather(0);
    } else {
        std::vector<std::thread> th;
        th.reserve(T - 1);
        for (uint32_t t = 1; t < T; ++t) th.emplace_back(gather, t);
        gather(0);
        for (auto& x : th) x.join();
    }
    for (auto& pt : parts) sub_free_.insert(sub_free_.end(), pt.freed.begin(), pt.freed.end());
    // detached nodes leave the engine now (before any callback can hand their handles out again)
    for (auto& pt : parts)
        for (auto& o : pt.objs) {
            const uint32_t h = o.first;
            if (h < n_slots_ || !o.second) continue;
            auto it = detached_.find(h);
            if (it != detached_.end() && it->second == o.second) {
                detached_.erase(it);
                has_obj_[h] = 0;
                fgi_release(g_, 1, &h);
            }
        }
    fan.gather_ms = ms_since(t0);
    // 2. per peer: its call ids in handle order, PeerBatch per sink call
    std::vector<uint64_t> buf;
    for (uint32_t q = 0; q < P; ++q) {
        uint64_t tot = 0;
        for (auto& pt : parts) tot += pt.calls[q].size();
        if (!tot) continue;
        const uint64_t* data;
        if (T == 1) {
            data = parts[0].calls[q].data();
        } else {
            buf.clear();
            buf.reserve(tot);
            for (auto& pt : parts) buf.insert(buf.end(), pt.calls[q].begin(), pt.calls[q].end());
            data = buf.data();
        }
        const size_t B = std::max<size_t>(1, PeerBatch);
        for (uint64_t o = 0; o < tot; o += B) {
            const size_t k = (size_t)std::min<uint64_t>(B, tot - o);
            if (q < peers_.size() && peers_[q]) peers_[q](q, data + o, k);
            ++fan.peer_batches[q];
        }
        fan.peer_calls[q] = tot;
        fan.calls += tot;
        fan.batches += fan.peer_batches[q];
        ++fan.peers_hit;
    }
    // 3. the registry-level handler class, over the whole list
    if (OnInvalidatedBatch) {
        const size_t C = std::max<size_t>(1, BatchChunk);
        if (bits) {
            std::vector<uint32_t> chunk;
            chunk.reserve((size_t)std::min<uint64_t>(C, n));
            for (uint64_t w = 0; w < words; ++w)
                for (uint64_t m = bits[w]; m; m &= m - 1) {
                    chunk.push_back((uint32_t)(w * 64 + (uint64_t)__builtin_ctzll(m)));
                    if (chunk.size() == C) {
                        OnInvalidatedBatch(chunk.data(), chunk.size());
                        chunk.clear();
                    }
                }
            if (!chunk.empty()) OnInvalidatedBatch(chunk.data(), chunk.size());
        } else {
            for (uint64_t o = 0; o < n; o += C) OnInvalidatedBatch(ids + o, (size_t)std::min<uint64_t>(C, n - o));
        }
    }
    // 4. host objects: OnUnregister, then each node's handler set, exactly once
    for (auto& pt : parts) {
        for (auto& o : pt.objs) {
            Computed* c = o.second.get();
            if (!c || c->fired_) continue;
            ++fan.objects;
            c->fired_ = true;
            if (o.first < n_slots_ && OnUnregister) OnUnregister(*c);
            InvalidatedHandlerSet hs = std::move(c->handlers_);
            c->handlers_.Clear();
            hs.Invoke(*c);
        }
    }
    fan.dispatch_ms = ms_since(t0);
    fan_ = std::move(fan);
    if (own && own_cap > ids_cap_) {   // hand the (larger) buffer back for the next wave
        ids_ = std::move(own);
        ids_cap_ = own_cap;
    }
    if (own_bits && !bits_) bits_ = std::move(own_bits);
}

uint32_t ComputedRegistry::AddPeer(PeerSink sink) {
    peers_.push_back(std::move(sink));
    return (uint32_t)peers_.size() - 1;
}

void ComputedRegistry::Subscribe(uint32_t handle, uint32_t peer, uint64_t call_id) {
    Subscribe(1, &handle, &peer, &call_id);
}

void ComputedRegistry::Subscribe(size_t n, const uint32_t* handles, const uint32_t* peers, const uint64_t* call_ids) {
    if (sub_head_.empty()) sub_head_.assign(n_handles_, kNone);   // once, on the first subscription
    for (size_t i = 0; i < n; ++i) {
        const uint32_t h = handles[i];
        if (h >= n_handles_ || peers[i] >= peers_.size()) throw FgiError(FGI_EINVAL, "Subscribe: bad handle or peer");
        uint32_t e;
        if (!sub_free_.empty()) {
            e = sub_free_.back();
            sub_free_.pop_back();
        } else {
            e = (uint32_t)subs_.size();
            subs_.push_back({});
        }
        subs_[e] = Sub{call_ids[i], peers[i], sub_head_[h]};
        sub_head_[h] = e;
    }
}

void ComputedRegistry::InvalidateInput(const std::string& input) {
    const uint32_t s = SlotOf(input, false);
    if (s == FGI_NONE) return;   // TryUseExisting: no existing computed -> nothing to invalidate
    if (IsInvalidating()) {
        scope_roots_.push_back(s);
        scope_imm_.push_back(0);
    } else {
        RunWave(&s, 1, nullptr);
    }
}

void ComputedRegistry::InvalidateSlots(const std::vector<uint32_t>& slots) {
    if (IsInvalidating()) {
        scope_roots_.insert(scope_roots_.end(), slots.begin(), slots.end());
        scope_imm_.insert(scope_imm_.end(), slots.size(), 0);
    } else {
        RunWave(slots.data(), slots.size(), nullptr);
    }
}

void ComputedRegistry::FlushScope() {
    const bool async = async_scope_;
    async_scope_ = false;
    if (scope_roots_.empty()) return;
    std::vector<uint32_t> roots;
    std::vector<uint8_t> imm;
    roots.swap(scope_roots_);
    imm.swap(scope_imm_);
    if (async) {
        InvalidateSlotsAsync(roots, &imm);
        return;
    }
    RunWave(roots.data(), roots.size(), imm.data());
}

// ---- asynchronous waves (ComputedExt.WhenInvalidated over fgi_invalidate_async_host) ------------------
// The engine keeps at most two waves in flight (a third call waits for the oldest inside the library);
// the mirror completes a wave — its ids brought back and fanned out exactly as a synchronous wave's —
// when asked, or before any other registry call (whose view of the registry must include the wave).
uint64_t ComputedRegistry::InvalidateSlotsAsync(const std::vector<uint32_t>& roots, const std::vector<uint8_t>* imm) {
    // a third wave makes the library wait for the oldest: complete it here so its fan-out runs in order
    while (pending_.size() >= 2) Complete(pending_.front());
    uint64_t t = 0;
    Check(fgi_invalidate_async_host(g_, (uint32_t)roots.size(), roots.data(),
                                    imm && imm->size() == roots.size() ? imm->data() : nullptr, &t),
          "fgi_invalidate_async_host");
    pending_.push_back(t);
    last_ticket_ = t;
    return t;
}

void ComputedRegistry::Complete(uint64_t ticket) {
    while (!pending_.empty() && pending_.front() <= ticket) {
        const uint64_t t = pending_.front();
        pending_.pop_front();   // before the fan-out: its handlers may call back into the registry
        fgi_wave_stats ws{};
        uint64_t n = 0;
        uint32_t* ids = IdsBuffer(1024);
        fgi_status s = fgi_wave_wait_ids(g_, t, ids, ids_cap_, &n, &ws);
        if (s == FGI_ECAPACITY) {   // the wave completed; fetch its ids with the right size
            ids = IdsBuffer(n);
            s = fgi_wave_wait_ids(g_, t, ids, n, &n, nullptr);
        }
        Check(s, "fgi_wave_wait_ids");
        last_ = ws;
        pred_v_ = n;
        Dispatch(ids, n);
    }
}

void ComputedRegistry::CompletePending() {
    if (!pending_.empty()) Complete(pending_.back());
}

// ---- access reports (ComputedRegistry.ReportAccess, Computed.RenewTimeouts) -----------------------
void ComputedRegistry::ReportAccess(Computed& c, bool is_new) {
    if (!OnAccess) return;
    if (c.IsInvalidated()) return;   // RenewTimeouts returns early for an Invalidated node (Computed.cs:250-251)
    OnAccess(c, is_new);
}

std::shared_ptr<Computed> ComputedRegistry::TryUseExisting(const std::string& input, Computed* usedBy) {
    auto existing = Get(input);
    if (!existing || !existing->IsConsistent()) return nullptr;
    if (usedBy) AddUsed(*usedBy, *existing);
    if (OnAccess) OnAccess(*existing, true);   // Consistent: RenewTimeouts(true) reports it
    return existing;
}

std::shared_ptr<Computed> ComputedRegistry::GetExisting(const std::string& input) {
    CompletePending();
    const uint32_t s = SlotOf(input, false);
    if (s == FGI_NONE || !current_[s]) return nullptr;
    ReportAccess(*current_[s], false);
    return current_[s];
}

void ComputedRegistry::UseNew(Computed& computed, Computed* usedBy) {
    if (usedBy) AddUsed(*usedBy, computed);
    ReportAccess(computed, true);
}

void ComputedRegistry::InvalidateEverything() {
    CompletePending();
    uint64_t n = 0;
    last_ = fgi_wave_stats{};
    uint32_t* ids = IdsBuffer(1024);
    fgi_status s = fgi_invalidate_all(g_, ids, ids_cap_, &n, &last_);
    if (s == FGI_ECAPACITY) {
        ids = IdsBuffer(n);
        s = fgi_last_wave_ids(g_, ids, n, &n);
    }
    Check(s, "fgi_invalidate_all");
    Dispatch(ids, n);
}

std::pair<uint64_t, uint64_t> ComputedRegistry::Prune() {
    CompletePending();
    fgi_prune_stats ps{};
    Check(fgi_prune(g_, &ps), "fgi_prune");
    return {ps.old_edges, ps.new_edges};
}

// ---- Computed --------------------------------------------------------------------------------------
ConsistencyState Computed::State() const { return (ConsistencyState)(Flags() & FGI_STATE_MASK); }

uint32_t Computed::Flags() const {
    reg_->CompletePending();   // the state includes the waves in flight (their handlers run first)
    uint64_t v = 0;
    uint32_t f = 0;
    reg_->Check(fgi_get_state(reg_->g_, 1, &handle_, &v, &f), "fgi_get_state");
    if (v != version_) return FGI_INVALIDATED;   // the slot moved on: this node is gone
    return f;
}

void Computed::Invalidate(bool immediately) {
    if (reg_->IsInvalidating()) {
        reg_->scope_roots_.push_back(handle_);
        reg_->scope_imm_.push_back(immediately ? 1 : 0);
    } else {
        const uint8_t imm = immediately ? 1 : 0;
        reg_->RunWave(&handle_, 1, &imm);
    }
}

InvalidatedHandler Computed::OnInvalidated(std::function<void(Computed&)> handler) {
    auto h = std::make_shared<const std::function<void(Computed&)>>(std::move(handler));
    OnInvalidated(h);
    return h;
}

void Computed::OnInvalidated(const InvalidatedHandler& handler) {
    if (fired_ || IsInvalidated()) {   // Computed.cs:84-97: added after invalidation -> fires now
        (*handler)(*this);
        return;
    }
    handlers_.Add(handler);
}

void Computed::RemoveOnInvalidated(const InvalidatedHandler& handler) { handlers_.Remove(handler); }

std::shared_future<void> Computed::WhenInvalidated() {
    if (when_) return when_f_;
    when_ = std::make_shared<std::promise<void>>();
    when_f_ = when_->get_future().share();
    // ComputedExt.cs:101-102: already Invalidated -> completed. Every invalidation of a node the mirror
    // holds goes through its fan-out (fired_), so the test needs no device query — which would complete
    // the asynchronous waves in flight, while the caller wants to await them.
    if (fired_) {
        when_->set_value();
        return when_f_;
    }
    std::shared_ptr<std::promise<void>> p = when_;
    handlers_.Add(std::make_shared<const std::function<void(Computed&)>>([p](Computed&) { p->set_value(); }));
    return when_f_;
}

std::vector<std::pair<uint32_t, LTag>> Computed::UsedBy() const {
    uint64_t n = 0;
    fgi_get_used_by(reg_->g_, handle_, nullptr, nullptr, 0, &n);
    std::vector<uint32_t> d(n);
    std::vector<uint64_t> t(n);
    reg_->Check(fgi_get_used_by(reg_->g_, handle_, d.data(), t.data(), n, &n), "fgi_get_used_by");
    std::vector<std::pair<uint32_t, LTag>> out;
    for (uint64_t i = 0; i < n; ++i) out.emplace_back(d[i], t[i]);
    return out;
}

uint32_t Computed::UsedCount() const {
    uint32_t c = 0;
    reg_->Check(fgi_get_used_count(reg_->g_, handle_, &c), "fgi_get_used_count");
    return c;
}

}  // namespace fusion
