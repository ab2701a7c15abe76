// fusion.cpp — implementation of the host-layer mirror (see fusion.hpp).
#include "fusion.hpp"

#include <algorithm>

namespace fusion {

ComputedRegistry::ComputedRegistry(uint32_t n_slots, uint32_t n_detached, int device) : n_slots_(n_slots) {
    fgi_config cfg{};
    cfg.struct_size = sizeof(cfg);
    cfg.device = device;
    cfg.n_slots = n_slots;
    cfg.n_detached = n_detached;
    cfg.world = 1;
    fgi_status s = fgi_create(&cfg, &g_);
    if (s != FGI_OK) throw FgiError(s, "fgi_create failed (no GPU?)");
    current_.resize(n_slots);
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

std::shared_ptr<Computed> ComputedRegistry::Get(const std::string& input) {
    const uint32_t s = SlotOf(input, false);
    if (s == FGI_NONE || !current_[s]) return nullptr;
    const ConsistencyState st = current_[s]->State();
    if (st == ConsistencyState::Invalidated) return nullptr;   // unregistered on invalidation
    return current_[s];
}

std::shared_ptr<Computed> ComputedRegistry::BeginCompute(const std::string& input, bool has_delay) {
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
    if (old) {
        if (detached != FGI_NONE) {
            old->handle_ = detached;       // displaced but alive (Computing / delayed)
            detached_[detached] = old;
        }
    }
    // the displacement cascade's invalidated nodes (the old node among them) get their handlers
    if (ws.v_inv) {
        std::vector<uint32_t> ids(ws.v_inv);
        uint64_t n = 0;
        Check(fgi_last_wave_ids(g_, ids.data(), ids.size(), &n), "fgi_last_wave_ids");
        Dispatch(ids.data(), n);
        last_ = ws;
    }
    current_[s] = c;
    if (OnRegister) OnRegister(*c);
    return c;
}

uint32_t ComputedRegistry::AddUsed(Computed& dependant, Computed& used) {
    uint32_t out = 0;
    const uint32_t d = dependant.handle_, u = used.handle_;
    Check(fgi_add_used(g_, 1, &d, &u, &out), "fgi_add_used");
    return out;
}

bool ComputedRegistry::SetOutput(Computed& c) {
    uint8_t set = 0;
    const uint32_t h = c.handle_;
    std::vector<uint32_t> ids(n_slots_ + 1024);
    uint64_t n = 0;
    Check(fgi_set_output(g_, 1, &h, &set, ids.data(), ids.size(), &n, &last_), "fgi_set_output");
    Dispatch(ids.data(), n);
    return set != 0;
}

void ComputedRegistry::RunWave(const std::vector<uint32_t>& roots, const std::vector<uint8_t>& imm) {
    std::vector<uint32_t> ids(n_slots_ + detached_.size() + 1);
    uint64_t n = 0;
    last_ = fgi_wave_stats{};
    fgi_status s = fgi_invalidate(g_, (uint32_t)roots.size(), roots.data(), imm.empty() ? nullptr : imm.data(),
                                  ids.data(), ids.size(), &n, &last_);
    if (s == FGI_ECAPACITY) {   // the wave itself completed; fetch the ids with the right size
        ids.resize(n);
        s = fgi_last_wave_ids(g_, ids.data(), ids.size(), &n);
    }
    Check(s, "fgi_invalidate");
    Dispatch(ids.data(), n);
}

// Invalidated handlers: once per node, after the wave (InvalidatedHandlerSet.Invoke, :100-127);
// OnUnregister for registry nodes (ComputeMethodComputed.OnInvalidated -> Unregister).
void ComputedRegistry::Dispatch(const uint32_t* ids, uint64_t n) {
    for (uint64_t i = 0; i < n; ++i) {
        const uint32_t h = ids[i];
        std::shared_ptr<Computed> c;
        if (h < n_slots_) {
            c = current_[h];
        } else {
            auto it = detached_.find(h);
            if (it != detached_.end()) {
                c = it->second;
                detached_.erase(it);
                fgi_release(g_, 1, &h);
            }
        }
        if (!c || c->fired_) continue;
        c->fired_ = true;
        if (h < n_slots_ && OnUnregister) OnUnregister(*c);
        auto hs = std::move(c->handlers_);
        c->handlers_.clear();
        for (auto& f : hs) f(*c);
    }
}

void ComputedRegistry::InvalidateInput(const std::string& input) {
    const uint32_t s = SlotOf(input, false);
    if (s == FGI_NONE) return;   // TryUseExisting: no existing computed -> nothing to invalidate
    if (IsInvalidating()) {
        scope_roots_.push_back(s);
        scope_imm_.push_back(0);
    } else {
        RunWave({s}, {});
    }
}

void ComputedRegistry::FlushScope() {
    if (scope_roots_.empty()) return;
    std::vector<uint32_t> roots;
    std::vector<uint8_t> imm;
    roots.swap(scope_roots_);
    imm.swap(scope_imm_);
    RunWave(roots, imm);
}

void ComputedRegistry::InvalidateEverything() {
    std::vector<uint32_t> ids(n_slots_ + detached_.size() + 1);
    uint64_t n = 0;
    last_ = fgi_wave_stats{};
    Check(fgi_invalidate_all(g_, ids.data(), ids.size(), &n, &last_), "fgi_invalidate_all");
    Dispatch(ids.data(), n);
}

std::pair<uint64_t, uint64_t> ComputedRegistry::Prune() {
    fgi_prune_stats ps{};
    Check(fgi_prune(g_, &ps), "fgi_prune");
    return {ps.old_edges, ps.new_edges};
}

ConsistencyState Computed::State() const { return (ConsistencyState)(Flags() & FGI_STATE_MASK); }

uint32_t Computed::Flags() const {
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
        reg_->RunWave({handle_}, {static_cast<uint8_t>(immediately ? 1 : 0)});
    }
}

void Computed::OnInvalidated(std::function<void(Computed&)> handler) {
    if (fired_ || IsInvalidated()) {
        handler(*this);
        return;
    }
    handlers_.push_back(std::move(handler));
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
