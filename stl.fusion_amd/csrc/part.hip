// part.hip — multi-GPU engine: 1-D vertex-range partition of the slots over the GPUs of one node
// (one process per GPU), frontier exchange with RCCL over xGMI.
//
// Rank p owns slots [p*B, p*B + n_local), B = ceil(N / world): their node words and their
// `_usedBy` rows (entries keep the GLOBAL dependant slot). Every rank also holds a replica of all
// N versions (versions never change during a wave), so the rank that traverses an edge to a
// remote slot checks the tag against the version itself and forwards only matching targets. A
// per-wave "sent" bitmap forwards each remote target at most once per wave: a node's first visit
// in a wave is the only one that can change it (Computed.cs:164-191 — later visits find it
// Invalidated, or the flag already set), so dropping the repeats is exact.
//
// Per level (run_part_wave, wave.hip): all-reduce of the level's frontier and its edges (push vs
// pull, termination); a push level expands locally (k_level<true>), all-gathers the per-owner
// counts, moves the targets by grouped send/recv and the owners apply them (k_apply_recv); a pull
// level all-gathers the frontier bitmap and every rank pulls its own slots.
//
// The collectives sit behind PartComm: RcclComm (one process per GPU, RCCL over xGMI) or
// LocalComm (an in-process group of P graphs driven by P host threads, device copies between their
// buffers). Both run the same run_part_wave, so the in-process tests execute exactly the level
// sequence a multi-GPU run does.
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>
#include <dlfcn.h>
#include <sched.h>

#include <algorithm>
#include <condition_variable>
#include <cstdio>
#include <cstring>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <type_traits>
#include <vector>

#include <rocprim/device/device_radix_sort.hpp>
#include <rocprim/device/device_scan.hpp>

#include "fgi_internal.h"

namespace fgi {

// Collectives of a partitioned wave (every rank calls them in the same order).
struct PartComm {
    virtual ~PartComm() {}
    // sum of `count` device u64 over all ranks, returned on the host (synchronises the stream)
    virtual fgi_status allreduce_sum(fgi_graph* g, const unsigned long long* dev_val, uint64_t* out, uint32_t count) = 0;
    // this level's forwarded targets: send_buf[q] (send_cnt[q] entries) to owner q; the targets
    // received from every other rank are concatenated at recv_buf. send_cnt[world, world + 1] carry
    // the rank's local {F, T} of the next level, summed with the targets sent by all ranks into
    // glob = {sum F, sum T, sum sent} on the way (the count all-gather doubles as the level's
    // all-reduce, so a push level synchronises the host once)
    virtual fgi_status exchange(fgi_graph* g, uint64_t* n_recv, uint64_t* n_sent, uint64_t* glob) = 0;
    // every rank's local invalidated-bitmap words inv_bm[0, block/32) into front_global
    virtual fgi_status allgather_front(fgi_graph* g) = 0;
    // every rank's u64 `mine` into all[0, world) (host), synchronising the stream
    virtual fgi_status allgather_count(fgi_graph* g, uint64_t mine, uint64_t* all) = 0;
    // every rank's delta entries dbuf[0, cnt[rank]) (global word << 32 | word) to every other rank:
    // concatenated at rbuf, returns the number received
    virtual fgi_status exchange_delta(fgi_graph* g, const uint64_t* cnt, uint64_t* n_recv) = 0;
    // Planned waves (no host synchronisation): stream-ordered collectives of fixed size.
    // allgather_front without waiting for the host (the next kernels on the stream see front_global)
    virtual fgi_status allgather_front_async(fgi_graph* g) = 0;
    // a2a_send[q * C, + C) to rank q, into a2a_recv[r * C, + C) from every rank r
    virtual fgi_status alltoall_async(fgi_graph* g) = 0;
    // Partitioned mutations: the element-wise sum of a device u32 array over all ranks, in place
    // (synchronises); every rank's cur_local (W64 words) into cur_all[q * W64, + W64) (stream-ordered)
    virtual fgi_status allreduce_u32(fgi_graph* g, uint32_t* dev, uint64_t n) = 0;
    virtual fgi_status allgather_cur_async(fgi_graph* g) = 0;
};

struct PartState {
    PartView v{};
    ncclComm_t comm = nullptr;
    std::unique_ptr<PartComm> ops;
    unsigned long long* all_cnt = nullptr;     // [world * (world + 2)] device
    unsigned long long* all_cnt_host = nullptr;
    unsigned long long* scalar = nullptr;      // device scratch for all-reduce
    unsigned long long* scalar_host = nullptr;
    // In-store: the dependency entries of the owned slots, as loaded (dependant local << 32 | used
    // global, tag). The owners of the `used` ends hold these entries in their rows; the owner of the
    // dependant keeps its own copy so it can rebuild its pull lists (part_rebuild_lists) without an
    // exchange whenever its node versions change.
    uint64_t* in_keys = nullptr;
    uint64_t* in_tags = nullptr;
    uint64_t in_n = 0, in_cap = 0;
    uint32_t* weight = nullptr;                // [n_global] live dependencies per slot (list order)
    // delta frontier exchange (part_allgather_front): this rank's changed bitmap words since the last
    // exchange, and the other ranks' received ones (global word index << 32 | word)
    uint64_t* dbuf = nullptr;                  // [block / 32]
    uint64_t* rbuf = nullptr;                  // [(world - 1) * block / 32]
    unsigned long long* dcnt = nullptr;        // device count of dbuf
    uint64_t front_full = 0, front_delta = 0;  // exchanges of each kind (statistics)
    uint64_t front_bytes = 0;                  // bytes received by this rank's frontier exchanges
    // planned waves (run_part_wave): the targets a push level forwards move in fixed-size buckets,
    // a2a_C words per peer (count, then up to a2a_C - 1 ids); what does not fit waits in send_buf
    // (a2a_cur: the next id to pack per owner) for the next push level
    uint32_t a2a_C = 0;                        // words per peer in use (<= a2a_cap; FGI_OPT_PART_BUCKET)
    uint32_t a2a_cap = 0;                      // words per peer allocated
    uint32_t* a2a_send = nullptr;              // [world][a2a_C]
    uint32_t* a2a_recv = nullptr;              // [world][a2a_C]
    unsigned long long* a2a_cur = nullptr;     // [world]
    unsigned long long* red = nullptr;         // [kPartRedMax] device all-reduce buffer (planned waves)
    unsigned long long* red_host = nullptr;
    // partitioned prune: the current-node bits of the owned slots (W64 words, padded per rank) and
    // every rank's, all-gathered (allocated on first use)
    uint64_t cur_w64 = 0;
    unsigned long long* cur_local = nullptr;
    unsigned long long* cur_all = nullptr;
    std::vector<uint32_t> u32_host;            // allreduce_u32's host copy (in-process groups)
    uint32_t* roots_codes = nullptr;           // fgi_part_invalidate's roots as codes (partition codes)
    uint32_t roots_cap = 0;
};

static PartState* ps(fgi_graph* g) { return reinterpret_cast<PartState*>(g->part); }

// ---- the RCCL the engine binds to ----------------------------------------------------------------
// libfgi does not link librccl: a process that loaded another librccl with the same soname first
// (torch's bundled copy) would otherwise bind the engine's collectives to that one. The entry points
// are resolved from /opt/rocm's librccl (the one the engine is built against, FGI_RCCL_LIBRARY
// overrides the path), opened RTLD_LOCAL, once per process: every collective below goes through
// this table.
struct RcclApi {
    void* lib = nullptr;
    std::string path;
    decltype(&ncclGetVersion) GetVersion = nullptr;
    decltype(&ncclGetUniqueId) GetUniqueId = nullptr;
    decltype(&ncclCommInitRank) CommInitRank = nullptr;
    decltype(&ncclCommInitRankConfig) CommInitRankConfig = nullptr;
    decltype(&ncclCommGetAsyncError) CommGetAsyncError = nullptr;
    decltype(&ncclCommAbort) CommAbort = nullptr;
    decltype(&ncclCommDestroy) CommDestroy = nullptr;
    decltype(&ncclGetErrorString) GetErrorString = nullptr;
    decltype(&ncclAllReduce) AllReduce = nullptr;
    decltype(&ncclAllGather) AllGather = nullptr;
    decltype(&ncclAllToAll) AllToAll = nullptr;
    decltype(&ncclSend) Send = nullptr;
    decltype(&ncclRecv) Recv = nullptr;
    decltype(&ncclGroupStart) GroupStart = nullptr;
    decltype(&ncclGroupEnd) GroupEnd = nullptr;
    std::string err;
};

static const RcclApi& rccl() {
    static const RcclApi api = [] {
        RcclApi a;
        const char* env = getenv("FGI_RCCL_LIBRARY");
        a.path = env && *env ? env : "/opt/rocm/lib/librccl.so.1";
        a.lib = dlopen(a.path.c_str(), RTLD_NOW | RTLD_LOCAL);
        if (!a.lib) {
            const char* e = dlerror();
            a.err = e ? e : "dlopen failed";
            return a;
        }
        bool ok = true;
        auto sym = [&](auto& fn, const char* name) {
            fn = reinterpret_cast<std::remove_reference_t<decltype(fn)>>(dlsym(a.lib, name));
            if (!fn) {
                ok = false;
                a.err = std::string("missing ") + name;
            }
        };
        sym(a.GetVersion, "ncclGetVersion");
        sym(a.GetUniqueId, "ncclGetUniqueId");
        sym(a.CommInitRank, "ncclCommInitRank");
        sym(a.CommInitRankConfig, "ncclCommInitRankConfig");
        sym(a.CommGetAsyncError, "ncclCommGetAsyncError");
        sym(a.CommAbort, "ncclCommAbort");
        sym(a.CommDestroy, "ncclCommDestroy");
        sym(a.GetErrorString, "ncclGetErrorString");
        sym(a.AllReduce, "ncclAllReduce");
        sym(a.AllGather, "ncclAllGather");
        sym(a.AllToAll, "ncclAllToAll");
        sym(a.Send, "ncclSend");
        sym(a.Recv, "ncclRecv");
        sym(a.GroupStart, "ncclGroupStart");
        sym(a.GroupEnd, "ncclGroupEnd");
        if (!ok) {
            dlclose(a.lib);
            a.lib = nullptr;
        }
        return a;
    }();
    return api;
}

static bool rccl_ok() { return rccl().lib != nullptr; }

// c: [W][W + 2] all-gathered counts (targets sent by q to r, then q's next-level F, T)
template <typename C>
static void sum_counts(const C* c, uint32_t W, uint64_t* glob) {
    const uint32_t S = W + 2;
    glob[0] = glob[1] = glob[2] = 0;
    for (uint32_t q = 0; q < W; ++q) {
        glob[0] += c[(size_t)q * S + W];
        glob[1] += c[(size_t)q * S + W + 1];
        for (uint32_t r = 0; r < W; ++r)
            if (r != q) glob[2] += c[(size_t)q * S + r];
    }
}

fgi_status part_destroy(fgi_graph* g) {
    PartState* p = ps(g);
    if (!p) return FGI_OK;
    p->ops.reset();
    if (p->comm) rccl().CommDestroy(p->comm);
    hipFree(p->v.ver_all);
    hipFree(p->v.sent_bm);
    hipFree(p->v.send_buf);
    hipFree(p->v.recv_buf);
    hipFree(p->v.send_cnt);
    hipFree(p->all_cnt);
    hipFree(p->scalar);
    hipFree(p->v.front_global);
    hipFree(p->v.scratch_u64);
    hipFree(p->in_keys);
    hipFree(p->in_tags);
    hipFree(p->weight);
    hipFree(p->dbuf);
    hipFree(p->rbuf);
    hipFree(p->dcnt);
    hipFree(p->a2a_send);
    hipFree(p->a2a_recv);
    hipFree(p->a2a_cur);
    hipFree(p->red);
    hipFree(p->cur_local);
    hipFree(p->cur_all);
    hipFree(p->roots_codes);
    if (p->red_host) hipHostFree(p->red_host);
    if (p->all_cnt_host) hipHostFree(p->all_cnt_host);
    if (p->scalar_host) hipHostFree(p->scalar_host);
    delete p;
    g->part = nullptr;
    hipFree(g->pg_gc);
    hipFree(g->pg_ig);
    g->pg_gc = g->pg_ig = nullptr;
    g->pg_gc_h.clear();
    g->pg_ig_h.clear();
    g->lbl_perm = false;
    g->pg_hash = 0;
    return FGI_OK;
}

bool part_view(fgi_graph* g, PartView* v) {
    PartState* p = ps(g);
    if (!p) return false;
    *v = p->v;
    return true;
}

// ---- bounded waits on the RCCL path (fail fast, never hang) ------------------------------------------
// A rank whose peer never joins a collective would otherwise wait forever: in ncclCommInitRank, in a
// grouped send/recv's connection setup, or on its stream behind a collective kernel. The communicator
// is non-blocking (ncclConfig_t.blocking = 0): every RCCL call that reports ncclInProgress is polled
// through ncclCommGetAsyncError, and every host wait behind a collective polls the stream, each for at
// most FGI_WAIT_TIMEOUT_S seconds (default 300; FGI_RCCL_INIT_TIMEOUT_S, default 120, for the
// communicator's creation). On timeout the communicator is aborted (its kernels leave), the graph is
// marked failed and the call returns FGI_EDEVICE naming the rank and the collective.
static double wait_limit_s(const char* var, double dflt) {
    const char* e = getenv(var);
    return e && *e ? atof(e) : dflt;
}

static fgi_status comm_fail(fgi_graph* g, const char* what, double limit_s) {
    PartState* p = ps(g);
    if (p && p->comm && rccl().CommAbort) {
        rccl().CommAbort(p->comm);
        p->comm = nullptr;
    }
    g->failed = true;
    return set_err(g, FGI_EDEVICE, "rank %d of %d: %s did not complete within %.0f s (a peer missing or stuck); "
                                   "the communicator was aborted", g->rank, g->world, what, limit_s);
}

// an RCCL call's result: ncclInProgress (non-blocking communicator) is waited out, bounded
static fgi_status nccl_settle(fgi_graph* g, ncclComm_t comm, ncclResult_t r, const char* what, double limit_s) {
    if (r == ncclInProgress && comm && rccl().CommGetAsyncError) {
        const auto t0 = std::chrono::steady_clock::now();
        for (uint64_t k = 0; r == ncclInProgress; ++k) {
            if (rccl().CommGetAsyncError(comm, &r) != ncclSuccess) break;
            if (r != ncclInProgress) break;
            if (std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count() > limit_s)
                return comm_fail(g, what, limit_s);
            if (k > 1024) sched_yield();
        }
    }
    if (r == ncclSuccess) return FGI_OK;
    g->failed = true;
    return set_err(g, FGI_EDEVICE, "rank %d of %d: %s: %s", g->rank, g->world, what, rccl().GetErrorString(r));
}
#define FGI_NCCL(g, call)                                                                                  \
    do {                                                                                                   \
        ncclResult_t _r = (call);                                                                          \
        if (_r != ncclSuccess)                                                                             \
            FGI_TRY(nccl_settle((g), ps(g) ? ps(g)->comm : nullptr, _r, #call,                             \
                                wait_limit_s("FGI_WAIT_TIMEOUT_S", 300.0)));                                \
    } while (0)

// the host's wait behind this rank's collectives: the stream polled, bounded
static fgi_status comm_sync(fgi_graph* g, hipStream_t s, const char* what) {
    const double limit_s = wait_limit_s("FGI_WAIT_TIMEOUT_S", 300.0);
    const auto t0 = std::chrono::steady_clock::now();
    for (uint64_t k = 0;; ++k) {
        const hipError_t e = hipStreamQuery(s);
        if (e == hipSuccess) return FGI_OK;
        if (e != hipErrorNotReady) return hip_check(g, e, what);
        if ((k & 255) == 0 &&
            std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count() > limit_s)
            return comm_fail(g, what, limit_s);
        if (k < 4096) __builtin_ia32_pause();
        else sched_yield();
    }
}

// ---- RCCL (one process per GPU) ----------------------------------------------------------------
struct RcclComm final : PartComm {
    fgi_status allreduce_sum(fgi_graph* g, const unsigned long long* dev_val, uint64_t* out, uint32_t count) override {
        PartState* p = ps(g);
        hipStream_t s = g->stream;
        const bool big = count > 4;
        unsigned long long* dst = big ? p->red : p->scalar;
        unsigned long long* host = big ? p->red_host : p->scalar_host;
        const unsigned long long* src = dev_val;   // one rank: the sum is the value
        if (p->v.world > 1 || g->opt_part_coll) {
            FGI_NCCL(g, rccl().AllReduce(dev_val, dst, count, ncclUint64, ncclSum, p->comm, s));
            src = dst;
        }
#if FGI_SPIN_WAIT
        (void)host;
        // the host spins instead of a stream sync (publish_wait is bounded by FGI_WAIT_TIMEOUT_S too)
        if (publish_wait(g, s, src, count, g->red_pub) != FGI_OK)
            return comm_fail(g, "all-reduce (wave counters)", wait_limit_s("FGI_WAIT_TIMEOUT_S", 300.0));
        for (uint32_t i = 0; i < count; ++i) out[i] = g->red_pub[i];
#else
        FGI_HIP(g, hipMemcpyAsync(host, src, 8 * count, hipMemcpyDeviceToHost, s));
        FGI_TRY(comm_sync(g, s, "all-reduce (wave counters)"));
        for (uint32_t i = 0; i < count; ++i) out[i] = host[i];
#endif
        return FGI_OK;
    }
    fgi_status allgather_front_async(fgi_graph* g) override { return allgather_front(g); }   // stream-ordered
    fgi_status alltoall_async(fgi_graph* g) override {
        PartState* p = ps(g);
        FGI_NCCL(g, rccl().AllToAll(p->a2a_send, p->a2a_recv, p->a2a_C, ncclUint32, p->comm, g->stream));
        return FGI_OK;
    }
    fgi_status allreduce_u32(fgi_graph* g, uint32_t* dev, uint64_t n) override {
        PartState* p = ps(g);
        if (n && (p->v.world > 1 || g->opt_part_coll))
            FGI_NCCL(g, rccl().AllReduce(dev, dev, n, ncclUint32, ncclSum, p->comm, g->stream));
        return comm_sync(g, g->stream, "all-reduce (u32)");
    }
    fgi_status allgather_cur_async(fgi_graph* g) override {
        PartState* p = ps(g);
        if (p->v.world > 1 || g->opt_part_coll)
            FGI_NCCL(g, rccl().AllGather(p->cur_local, p->cur_all, p->cur_w64, ncclUint64, p->comm, g->stream));
        else
            FGI_HIP(g, hipMemcpyAsync(p->cur_all, p->cur_local, p->cur_w64 * 8, hipMemcpyDeviceToDevice, g->stream));
        return FGI_OK;
    }
    fgi_status exchange(fgi_graph* g, uint64_t* n_recv, uint64_t* n_sent, uint64_t* glob) override {
        PartState* p = ps(g);
        const uint32_t W = p->v.world, R = p->v.rank, S = W + 2;
        hipStream_t s = g->stream;
        FGI_NCCL(g, rccl().AllGather(p->v.send_cnt, p->all_cnt, S, ncclUint64, p->comm, s));
        FGI_HIP(g, hipMemcpyAsync(p->all_cnt_host, p->all_cnt, (size_t)W * S * 8, hipMemcpyDeviceToHost, s));
        FGI_TRY(comm_sync(g, s, "all-gather of the push level's counts"));
        const unsigned long long* c = p->all_cnt_host;   // c[q * S + r]: sent by q to r; c[q * S + W + i]: q's F, T
        sum_counts(c, W, glob);
        uint64_t recv = 0, sent = 0;
        FGI_NCCL(g, rccl().GroupStart());
        for (uint32_t q = 0; q < W; ++q) {
            if (q == R) continue;
            const uint64_t to_q = c[R * S + q], from_q = c[q * S + R];
            if (to_q)
                FGI_NCCL(g, rccl().Send(p->v.send_buf + (uint64_t)q * p->v.block, to_q, ncclUint32, (int)q, p->comm, s));
            if (from_q) FGI_NCCL(g, rccl().Recv(p->v.recv_buf + recv, from_q, ncclUint32, (int)q, p->comm, s));
            recv += from_q;
            sent += to_q;
        }
        FGI_NCCL(g, rccl().GroupEnd());
        *n_recv = recv;
        *n_sent = sent;
        return FGI_OK;
    }
    fgi_status allgather_front(fgi_graph* g) override {
        PartState* p = ps(g);
        FGI_NCCL(g, rccl().AllGather(g->inv_bm, p->v.front_global, p->v.block / 32, ncclUint32, p->comm, g->stream));
        return FGI_OK;
    }
    fgi_status allgather_count(fgi_graph* g, uint64_t mine, uint64_t* all) override {
        PartState* p = ps(g);
        const uint32_t W = p->v.world;
        p->scalar_host[0] = mine;
        FGI_HIP(g, hipMemcpyAsync(p->scalar, p->scalar_host, 8, hipMemcpyHostToDevice, g->stream));
        FGI_NCCL(g, rccl().AllGather(p->scalar, p->all_cnt, 1, ncclUint64, p->comm, g->stream));
        FGI_HIP(g, hipMemcpyAsync(p->all_cnt_host, p->all_cnt, (size_t)W * 8, hipMemcpyDeviceToHost, g->stream));
        FGI_TRY(comm_sync(g, g->stream, "all-gather of a count"));
        for (uint32_t q = 0; q < W; ++q) all[q] = p->all_cnt_host[q];
        return FGI_OK;
    }
    fgi_status exchange_delta(fgi_graph* g, const uint64_t* cnt, uint64_t* n_recv) override {
        PartState* p = ps(g);
        const uint32_t W = p->v.world, R = p->v.rank;
        uint64_t recv = 0;
        FGI_NCCL(g, rccl().GroupStart());
        for (uint32_t q = 0; q < W; ++q) {
            if (q == R) continue;
            if (cnt[R]) FGI_NCCL(g, rccl().Send(p->dbuf, cnt[R], ncclUint64, (int)q, p->comm, g->stream));
            if (cnt[q]) FGI_NCCL(g, rccl().Recv(p->rbuf + recv, cnt[q], ncclUint64, (int)q, p->comm, g->stream));
            recv += cnt[q];
        }
        FGI_NCCL(g, rccl().GroupEnd());
        *n_recv = recv;
        return FGI_OK;
    }
};

// ---- host collectives (one process per rank, the host's own transport) -------------------------------
// Every collective reduces to one primitive the caller supplies (fgi_part_init_host): an all-gather of
// equal-size host buffers, e.g. torch.distributed over gloo. The ranks then need not sit on distinct
// GPUs (RCCL refuses two ranks on one device), so the planned and host-driven waves, the mutations and
// the prune of run_part_wave execute across real process boundaries on any box. Each collective
// synchronises the rank's stream, moves its part through host memory and copies the result back:
// correct, not fast (the async variants are synchronous here).
struct HostComm final : PartComm {
    fgi_allgather_fn fn;
    void* ctx;
    std::vector<uint8_t> sbuf, rbuf;
    HostComm(fgi_allgather_fn f, void* c) : fn(f), ctx(c) {}

    // all-gather `bytes` from sbuf into rbuf (world * bytes)
    fgi_status gather(fgi_graph* g, uint64_t bytes) {
        const uint32_t W = ps(g)->v.world;
        rbuf.resize((size_t)W * bytes + 1);
        if (sbuf.size() < bytes) sbuf.resize(bytes);
        const int rc = fn(ctx, sbuf.data(), bytes, rbuf.data());
        if (rc == 0) return FGI_OK;
        g->failed = true;   // a collective of the wave's protocol is missing on this rank: its state is undefined
        return set_err(g, FGI_EDEVICE, "rank %d of %d: host all-gather of %llu bytes failed (%d; a peer missing?)", g->rank,
                       g->world, (unsigned long long)bytes, rc);
    }
    // device -> sbuf (synchronises the stream: the device words are final)
    fgi_status stage(fgi_graph* g, const void* dev, uint64_t bytes, uint64_t at = 0) {
        if (sbuf.size() < at + bytes) sbuf.resize(at + bytes);
        if (bytes) FGI_HIP(g, hipMemcpyAsync(sbuf.data() + at, dev, bytes, hipMemcpyDeviceToHost, g->stream));
        FGI_HIP(g, hipStreamSynchronize(g->stream));
        return FGI_OK;
    }
    fgi_status upload(fgi_graph* g, void* dev, const void* host, uint64_t bytes) {
        if (bytes) FGI_HIP(g, hipMemcpyAsync(dev, host, bytes, hipMemcpyHostToDevice, g->stream));
        FGI_HIP(g, hipStreamSynchronize(g->stream));   // the host buffer is reused by the next collective
        return FGI_OK;
    }
    const uint64_t* u64(uint32_t q, uint64_t words) const { return reinterpret_cast<const uint64_t*>(rbuf.data()) + q * words; }

    fgi_status allreduce_sum(fgi_graph* g, const unsigned long long* dev_val, uint64_t* out, uint32_t count) override {
        FGI_TRY(stage(g, dev_val, 8ull * count));
        FGI_TRY(gather(g, 8ull * count));
        for (uint32_t i = 0; i < count; ++i) {
            uint64_t t = 0;
            for (uint32_t q = 0; q < ps(g)->v.world; ++q) t += u64(q, count)[i];
            out[i] = t;
        }
        return FGI_OK;
    }
    fgi_status exchange(fgi_graph* g, uint64_t* n_recv, uint64_t* n_sent, uint64_t* glob) override {
        PartState* p = ps(g);
        const uint32_t W = p->v.world, R = p->v.rank, S = W + 2;
        FGI_TRY(stage(g, p->v.send_cnt, 8ull * S));
        FGI_TRY(gather(g, 8ull * S));
        std::vector<uint64_t> c(reinterpret_cast<const uint64_t*>(rbuf.data()),
                                reinterpret_cast<const uint64_t*>(rbuf.data()) + (size_t)W * S);
        sum_counts(c.data(), W, glob);
        uint64_t mx = 0;   // the payload moves as one all-gather of [W][mx] ids per rank
        for (uint32_t q = 0; q < W; ++q)
            for (uint32_t r = 0; r < W; ++r)
                if (r != q) mx = std::max<uint64_t>(mx, c[(size_t)q * S + r]);
        uint64_t sent = 0, recv = 0;
        if (mx) {
            sbuf.assign((size_t)W * mx * 4, 0);
            for (uint32_t q = 0; q < W; ++q) {
                const uint64_t to_q = q == R ? 0 : c[(size_t)R * S + q];
                if (to_q)
                    FGI_HIP(g, hipMemcpyAsync(sbuf.data() + (size_t)q * mx * 4, p->v.send_buf + (uint64_t)q * p->v.block,
                                              to_q * 4, hipMemcpyDeviceToHost, g->stream));
                sent += to_q;
            }
            FGI_HIP(g, hipStreamSynchronize(g->stream));
            FGI_TRY(gather(g, (uint64_t)W * mx * 4));
            std::vector<uint32_t> in;
            for (uint32_t q = 0; q < W; ++q) {
                if (q == R) continue;
                const uint64_t from_q = c[(size_t)q * S + R];
                const uint32_t* src = reinterpret_cast<const uint32_t*>(rbuf.data() + ((size_t)q * W + R) * mx * 4);
                in.insert(in.end(), src, src + from_q);
            }
            recv = in.size();
            FGI_TRY(upload(g, p->v.recv_buf, in.data(), recv * 4));
        }
        *n_recv = recv;
        *n_sent = sent;
        return FGI_OK;
    }
    fgi_status allgather_front(fgi_graph* g) override {
        PartState* p = ps(g);
        const uint64_t bytes = (uint64_t)(p->v.block / 32) * 4;
        FGI_TRY(stage(g, g->inv_bm, bytes));
        FGI_TRY(gather(g, bytes));
        return upload(g, p->v.front_global, rbuf.data(), (uint64_t)p->v.world * bytes);
    }
    fgi_status allgather_count(fgi_graph* g, uint64_t mine, uint64_t* all) override {
        sbuf.resize(std::max<size_t>(sbuf.size(), 8));
        std::memcpy(sbuf.data(), &mine, 8);
        FGI_TRY(gather(g, 8));
        for (uint32_t q = 0; q < ps(g)->v.world; ++q) all[q] = u64(q, 1)[0];
        return FGI_OK;
    }
    fgi_status exchange_delta(fgi_graph* g, const uint64_t* cnt, uint64_t* n_recv) override {
        PartState* p = ps(g);
        const uint32_t W = p->v.world, R = p->v.rank;
        uint64_t mx = 0;
        for (uint32_t q = 0; q < W; ++q) mx = std::max<uint64_t>(mx, cnt[q]);
        uint64_t recv = 0;
        if (mx) {
            sbuf.assign(mx * 8, 0);
            FGI_TRY(stage(g, p->dbuf, cnt[R] * 8));
            FGI_TRY(gather(g, mx * 8));
            std::vector<uint64_t> in;
            for (uint32_t q = 0; q < W; ++q)
                if (q != R) in.insert(in.end(), u64(q, mx), u64(q, mx) + cnt[q]);
            recv = in.size();
            FGI_TRY(upload(g, p->rbuf, in.data(), recv * 8));
        }
        *n_recv = recv;
        return FGI_OK;
    }
    fgi_status allgather_front_async(fgi_graph* g) override { return allgather_front(g); }
    fgi_status alltoall_async(fgi_graph* g) override {
        PartState* p = ps(g);
        const uint32_t W = p->v.world, R = p->v.rank;
        const uint64_t C = p->a2a_C;
        FGI_TRY(stage(g, p->a2a_send, (uint64_t)W * C * 4));
        FGI_TRY(gather(g, (uint64_t)W * C * 4));
        std::vector<uint32_t> in((size_t)W * C);
        for (uint32_t q = 0; q < W; ++q)
            std::memcpy(in.data() + (size_t)q * C, rbuf.data() + ((size_t)q * W + R) * C * 4, C * 4);
        return upload(g, p->a2a_recv, in.data(), (uint64_t)W * C * 4);
    }
    fgi_status allreduce_u32(fgi_graph* g, uint32_t* dev, uint64_t n) override {
        const uint32_t W = ps(g)->v.world;
        FGI_TRY(stage(g, dev, n * 4));
        FGI_TRY(gather(g, n * 4));
        std::vector<uint32_t> sum(n, 0);
        for (uint32_t q = 0; q < W; ++q) {
            const uint32_t* v = reinterpret_cast<const uint32_t*>(rbuf.data() + (size_t)q * n * 4);
            for (uint64_t i = 0; i < n; ++i) sum[i] += v[i];
        }
        return upload(g, dev, sum.data(), n * 4);
    }
    fgi_status allgather_cur_async(fgi_graph* g) override {
        PartState* p = ps(g);
        FGI_TRY(stage(g, p->cur_local, p->cur_w64 * 8));
        FGI_TRY(gather(g, p->cur_w64 * 8));
        return upload(g, p->cur_all, rbuf.data(), (uint64_t)p->v.world * p->cur_w64 * 8);
    }
};

// ---- in-process group (P graphs, one host thread per rank) ---------------------------------------
// The ranks meet at a generation barrier; a rank that fails marks the group failed and releases
// the others, whose collectives then return FGI_EDEVICE instead of waiting forever.
struct LocalGroup {
    std::vector<fgi_graph*> gs;
    std::mutex mu;
    std::condition_variable cv;
    uint32_t arrived = 0;
    uint64_t gen = 0;
    bool failed = false;
    std::vector<uint64_t> vals;   // [P][kPartRedMax] all-reduce contributions
    std::vector<uint64_t> cnt;    // [P][P + 2] targets rank r forwards to owner q, then r's F, T
    // stream-ordered exchanges (planned waves): rank r records ready[r] when its source is final and
    // done[r] when its copies from the others are queued; the others' streams wait on them
    std::vector<hipEvent_t> ready, done;

    explicit LocalGroup(std::vector<fgi_graph*> g) : gs(std::move(g)) {
        vals.assign(gs.size() * kPartRedMax, 0);
        cnt.assign(gs.size() * (gs.size() + 2), 0);
        ready.assign(gs.size(), nullptr);
        done.assign(gs.size(), nullptr);
        for (size_t r = 0; r < gs.size(); ++r) {
            hipSetDevice(gs[r]->device);
            hipEventCreateWithFlags(&ready[r], hipEventDisableTiming);
            hipEventCreateWithFlags(&done[r], hipEventDisableTiming);
        }
    }
    ~LocalGroup() {
        for (hipEvent_t e : ready)
            if (e) hipEventDestroy(e);
        for (hipEvent_t e : done)
            if (e) hipEventDestroy(e);
    }
    bool arrive() {
        std::unique_lock<std::mutex> lk(mu);
        if (failed) return false;
        const uint64_t my = gen;
        if (++arrived == gs.size()) {
            arrived = 0;
            ++gen;
            cv.notify_all();
            return true;
        }
        cv.wait(lk, [&] { return gen != my || failed; });
        return !failed;
    }
    void fail() {
        std::lock_guard<std::mutex> lk(mu);
        failed = true;
        cv.notify_all();
    }
    void reset() {
        std::lock_guard<std::mutex> lk(mu);
        failed = false;
        arrived = 0;
    }
};

struct LocalComm final : PartComm {
    std::shared_ptr<LocalGroup> grp;
    uint32_t rank;
    LocalComm(std::shared_ptr<LocalGroup> g, uint32_t r) : grp(std::move(g)), rank(r) {}

    fgi_status peer_failed(fgi_graph* g) { return set_err(g, FGI_EDEVICE, "another rank of the in-process group failed"); }

    fgi_status allreduce_sum(fgi_graph* g, const unsigned long long* dev_val, uint64_t* out, uint32_t count) override {
        PartState* p = ps(g);
#if FGI_SPIN_WAIT
        (void)p;
        FGI_TRY(publish_wait(g, g->stream, dev_val, count, g->red_pub));
        const unsigned long long* host = g->red_pub;
#else
        unsigned long long* host = count > 4 ? p->red_host : p->scalar_host;
        FGI_HIP(g, hipMemcpyAsync(host, dev_val, 8 * count, hipMemcpyDeviceToHost, g->stream));
        FGI_HIP(g, hipStreamSynchronize(g->stream));
#endif
        {
            std::lock_guard<std::mutex> lk(grp->mu);
            for (uint32_t i = 0; i < count; ++i) grp->vals[(size_t)rank * kPartRedMax + i] = host[i];
        }
        if (!grp->arrive()) return peer_failed(g);
        for (uint32_t i = 0; i < count; ++i) {
            uint64_t t = 0;
            for (size_t r = 0; r < grp->gs.size(); ++r) t += grp->vals[r * kPartRedMax + i];
            out[i] = t;
        }
        if (!grp->arrive()) return peer_failed(g);   // nobody overwrites vals before all have read them
        return FGI_OK;
    }
    fgi_status exchange(fgi_graph* g, uint64_t* n_recv, uint64_t* n_sent, uint64_t* glob) override {
        PartState* p = ps(g);
        const uint32_t W = p->v.world, R = rank, S = W + 2;
        FGI_HIP(g, hipMemcpyAsync(p->all_cnt_host, p->v.send_cnt, (size_t)S * 8, hipMemcpyDeviceToHost, g->stream));
        FGI_HIP(g, hipStreamSynchronize(g->stream));   // also: this rank's send buffers are complete
        {
            std::lock_guard<std::mutex> lk(grp->mu);
            for (uint32_t q = 0; q < S; ++q) grp->cnt[(size_t)R * S + q] = p->all_cnt_host[q];
        }
        if (!grp->arrive()) return peer_failed(g);
        sum_counts(grp->cnt.data(), W, glob);
        uint64_t recv = 0, sent = 0;
        for (uint32_t q = 0; q < W; ++q) {
            if (q == R) continue;
            const uint64_t from_q = grp->cnt[(size_t)q * S + R];
            if (from_q) {
                PartState* pq = ps(grp->gs[q]);
                FGI_HIP(g, hipMemcpyAsync(p->v.recv_buf + recv, pq->v.send_buf + (uint64_t)R * pq->v.block, from_q * 4,
                                          hipMemcpyDefault, g->stream));
            }
            recv += from_q;
            sent += grp->cnt[(size_t)R * S + q];
        }
        // the senders refill their buffers (and counts) only after every rank's copies are done
        FGI_HIP(g, hipStreamSynchronize(g->stream));
        if (!grp->arrive()) return peer_failed(g);
        *n_recv = recv;
        *n_sent = sent;
        return FGI_OK;
    }
    fgi_status allgather_front(fgi_graph* g) override {
        PartState* p = ps(g);
        FGI_HIP(g, hipStreamSynchronize(g->stream));   // this rank's invalidated words are final
        if (!grp->arrive()) return peer_failed(g);
        const uint64_t words = p->v.block / 32;
        for (size_t q = 0; q < grp->gs.size(); ++q)
            FGI_HIP(g, hipMemcpyAsync(p->v.front_global + q * words, grp->gs[q]->inv_bm, words * 4, hipMemcpyDefault,
                                      g->stream));
        FGI_HIP(g, hipStreamSynchronize(g->stream));
        if (!grp->arrive()) return peer_failed(g);     // the sources stay untouched until all copies are done
        return FGI_OK;
    }
    fgi_status allgather_count(fgi_graph* g, uint64_t mine, uint64_t* all) override {
        const size_t W = grp->gs.size();
        {
            std::lock_guard<std::mutex> lk(grp->mu);
            grp->vals[(size_t)rank * kPartRedMax] = mine;
        }
        if (!grp->arrive()) return peer_failed(g);
        for (size_t q = 0; q < W; ++q) all[q] = grp->vals[q * kPartRedMax];
        if (!grp->arrive()) return peer_failed(g);
        return FGI_OK;
    }
    fgi_status exchange_delta(fgi_graph* g, const uint64_t* cnt, uint64_t* n_recv) override {
        PartState* p = ps(g);
        FGI_HIP(g, hipStreamSynchronize(g->stream));   // this rank's delta list is complete
        if (!grp->arrive()) return peer_failed(g);
        uint64_t recv = 0;
        for (uint32_t q = 0; q < (uint32_t)grp->gs.size(); ++q) {
            if (q == rank) continue;
            if (cnt[q])
                FGI_HIP(g, hipMemcpyAsync(p->rbuf + recv, ps(grp->gs[q])->dbuf, cnt[q] * 8, hipMemcpyDefault, g->stream));
            recv += cnt[q];
        }
        FGI_HIP(g, hipStreamSynchronize(g->stream));
        if (!grp->arrive()) return peer_failed(g);     // the senders keep their lists until every copy is done
        *n_recv = recv;
        return FGI_OK;
    }
    // Stream-ordered copies between the group's graphs, no host wait: this rank's source is marked
    // ready on its stream; once every rank has queued its mark (a host-thread barrier, no device
    // synchronisation), each stream waits for the others' marks and copies; then each stream waits
    // until every rank's copies are queued behind its own marks, so no source is overwritten early.
    template <class F>
    fgi_status exchange_async(fgi_graph* g, F copies) {
        FGI_HIP(g, hipEventRecord(grp->ready[rank], g->stream));
        if (!grp->arrive()) return peer_failed(g);
        for (size_t q = 0; q < grp->gs.size(); ++q)
            if (q != rank) FGI_HIP(g, hipStreamWaitEvent(g->stream, grp->ready[q], 0));
        FGI_TRY(copies());
        FGI_HIP(g, hipEventRecord(grp->done[rank], g->stream));
        if (!grp->arrive()) return peer_failed(g);
        for (size_t q = 0; q < grp->gs.size(); ++q)
            if (q != rank) FGI_HIP(g, hipStreamWaitEvent(g->stream, grp->done[q], 0));
        return FGI_OK;
    }
    fgi_status allgather_front_async(fgi_graph* g) override {
        PartState* p = ps(g);
        const uint64_t words = p->v.block / 32;
        return exchange_async(g, [&]() -> fgi_status {
            for (size_t q = 0; q < grp->gs.size(); ++q)
                FGI_HIP(g, hipMemcpyAsync(p->v.front_global + q * words, grp->gs[q]->inv_bm, words * 4, hipMemcpyDefault,
                                          g->stream));
            return FGI_OK;
        });
    }
    fgi_status alltoall_async(fgi_graph* g) override {
        PartState* p = ps(g);
        const uint64_t C = p->a2a_C;
        return exchange_async(g, [&]() -> fgi_status {
            for (size_t q = 0; q < grp->gs.size(); ++q)
                FGI_HIP(g, hipMemcpyAsync(p->a2a_recv + q * C, ps(grp->gs[q])->a2a_send + (uint64_t)rank * C, C * 4,
                                          hipMemcpyDefault, g->stream));
            return FGI_OK;
        });
    }
    fgi_status allgather_cur_async(fgi_graph* g) override {
        PartState* p = ps(g);
        const uint64_t W = p->cur_w64;
        return exchange_async(g, [&]() -> fgi_status {
            for (size_t q = 0; q < grp->gs.size(); ++q)
                FGI_HIP(g, hipMemcpyAsync(p->cur_all + q * W, ps(grp->gs[q])->cur_local, W * 8, hipMemcpyDefault, g->stream));
            return FGI_OK;
        });
    }
    // host-side sum: every rank copies its array out, the group adds them, every rank copies the sum in
    fgi_status allreduce_u32(fgi_graph* g, uint32_t* dev, uint64_t n) override {
        PartState* p = ps(g);
        p->u32_host.resize(n);
        if (n) FGI_HIP(g, hipMemcpyAsync(p->u32_host.data(), dev, n * 4, hipMemcpyDeviceToHost, g->stream));
        FGI_HIP(g, hipStreamSynchronize(g->stream));
        if (!grp->arrive()) return peer_failed(g);
        std::vector<uint32_t> sum(n, 0);
        for (size_t q = 0; q < grp->gs.size(); ++q) {
            const std::vector<uint32_t>& h = ps(grp->gs[q])->u32_host;
            for (uint64_t i = 0; i < n; ++i) sum[i] += h[i];
        }
        if (!grp->arrive()) return peer_failed(g);   // nobody changes its copy before all have read it
        if (n) FGI_HIP(g, hipMemcpyAsync(dev, sum.data(), n * 4, hipMemcpyHostToDevice, g->stream));
        FGI_HIP(g, hipStreamSynchronize(g->stream));
        return FGI_OK;
    }
};

fgi_status part_exchange(fgi_graph* g, uint64_t* n_recv, uint64_t* n_sent, uint64_t* glob) {
    return ps(g)->ops->exchange(g, n_recv, n_sent, glob);
}

fgi_status part_allgather_front_async(fgi_graph* g) {
    PartState* p = ps(g);
    ++p->front_full;
    p->front_bytes += (uint64_t)(p->v.world - 1) * p->v.block / 8;
    return p->ops->allgather_front_async(g);
}

fgi_status part_alltoall_async(fgi_graph* g) { return ps(g)->ops->alltoall_async(g); }

fgi_status part_allreduce_u32(fgi_graph* g, uint32_t* dev, uint64_t n) { return ps(g)->ops->allreduce_u32(g, dev, n); }

// every rank's current-node bits (its owned slots: W64 = ceil(block / 64) words each, rank q's at
// q * W64) into the returned all-gathered array; the caller builds cur_local first (its W64 words)
fgi_status part_cur_buffers(fgi_graph* g, unsigned long long** local, unsigned long long** all, uint64_t* w64) {
    PartState* p = ps(g);
    if (!p->cur_local) {
        p->cur_w64 = ((uint64_t)p->v.block + 63) / 64;
        if (hipMalloc(&p->cur_local, p->cur_w64 * 8) != hipSuccess ||
            hipMalloc(&p->cur_all, p->cur_w64 * 8 * p->v.world) != hipSuccess)
            return set_err(g, FGI_ENOMEM, "current-node bitmaps");
    }
    *local = p->cur_local;
    *all = p->cur_all;
    *w64 = p->cur_w64;
    return FGI_OK;
}

fgi_status part_allgather_cur(fgi_graph* g) { return ps(g)->ops->allgather_cur_async(g); }

static fgi_status part_store_in(fgi_graph* g, const uint64_t* keys, const uint64_t* tags, uint64_t m);

// device entries (dependant local << 32 | used global, tag) appended to the in-store
fgi_status part_store_in_dev(fgi_graph* g, const uint64_t* keys, const uint64_t* tags, uint64_t m) {
    return part_store_in(g, keys, tags, m);
}

namespace {
// entries (dependant local << 32 | used global) whose used end is in the sorted list: tag 0 (a
// version is never 0, so the list build reads them as dead)
__global__ void k_in_kill(uint64_t m, const uint64_t* __restrict__ keys, uint64_t* tags, const uint32_t* __restrict__ list,
                          uint32_t nl) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= m) return;
    const uint32_t u = (uint32_t)keys[i];
    uint32_t lo = 0, hi = nl;
    while (lo < hi) {
        const uint32_t mid = (lo + hi) >> 1;
        if (list[mid] < u) lo = mid + 1;
        else hi = mid;
    }
    if (lo < nl && list[lo] == u) tags[i] = 0;
}
}  // namespace

fgi_status part_kill_used(fgi_graph* g, std::vector<uint32_t> slots) {
    PartState* p = ps(g);
    if (slots.empty() || p->in_n == 0) return FGI_OK;
    std::sort(slots.begin(), slots.end());
    slots.erase(std::unique(slots.begin(), slots.end()), slots.end());
    uint32_t* d = nullptr;
    if (hipMalloc(&d, slots.size() * 4) != hipSuccess) return set_err(g, FGI_ENOMEM, "displaced-slot list");
    hipMemcpyAsync(d, slots.data(), slots.size() * 4, hipMemcpyHostToDevice, g->stream);
    hipLaunchKernelGGL(k_in_kill, dim3((uint32_t)((p->in_n + 255) / 256)), dim3(256), 0, g->stream, p->in_n, p->in_keys, p->in_tags, d,
                       (uint32_t)slots.size());
    const hipError_t e = hipStreamSynchronize(g->stream);
    hipFree(d);
    FGI_HIP(g, e);
    return FGI_OK;
}

fgi_status part_set_bucket(fgi_graph* g, int64_t words) {
    PartState* p = ps(g);
    if (!p) return set_err(g, FGI_ESTATE, "partition not initialised");
    if (words < 0) return set_err(g, FGI_EINVAL, "bucket words must be >= 0");
    p->a2a_C = words == 0 ? p->a2a_cap : (uint32_t)std::max<int64_t>(2, std::min<int64_t>(words, p->a2a_cap));
    return FGI_OK;
}

PartBuckets part_buckets(fgi_graph* g) {
    PartState* p = ps(g);
    return PartBuckets{p->a2a_C, p->a2a_send, p->a2a_recv, p->a2a_cur, p->red};
}

namespace {
// this rank's bitmap words that changed since the last exchange (front_global holds what the other
// ranks last received): listed as (global word << 32 | word) and written into front_global's own range
__global__ void k_front_delta(uint32_t words, const uint32_t* __restrict__ inv, uint32_t* own_front, uint32_t word_base,
                              uint64_t* dbuf, unsigned long long* dcnt) {
    const uint32_t w = blockIdx.x * blockDim.x + threadIdx.x;
    const uint32_t v = w < words ? inv[w] : 0u;
    const bool ch = w < words && v != own_front[w];
    const unsigned long long m = __ballot(ch);
    if (!m) return;
    const uint32_t lane = threadIdx.x & 63;
    unsigned long long b = 0;
    if (lane == 0) b = atomicAdd(dcnt, (unsigned long long)__popcll(m));
    b = __shfl(b, 0, 64);
    if (ch) {
        dbuf[b + __popcll(m & ((1ull << lane) - 1ull))] = ((uint64_t)(word_base + w) << 32) | v;
        own_front[w] = v;
    }
}

__global__ void k_front_apply(uint64_t n, const uint64_t* __restrict__ rbuf, uint32_t* front) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) {
        const uint64_t e = rbuf[i];
        front[e >> 32] = (uint32_t)e;
    }
}
}  // namespace

// The invalidated bitmap over all ranks' slots before a pull level (front_global). Full mode: an
// all-gather of every rank's block/32 words — (world - 1) * block / 8 bytes into every rank. Delta mode:
// each rank lists the words that gained bits since the previous exchange of the wave (8 B each) and
// sends the list to every other rank; the receivers patch their copy. FGI_OPT_FRONT_EXCHANGE 0 picks
// per level whichever moves fewer bytes (every rank decides alike from the all-gathered list sizes),
// 1 always full, 2 always delta. Either way front_global ends up identical.
fgi_status part_allgather_front(fgi_graph* g) {
    PartState* p = ps(g);
    const int mode = g->opt_front_exchange;
    if (mode == 1) {
        ++p->front_full;
        p->front_bytes += (uint64_t)(p->v.world - 1) * p->v.block / 8;
        return p->ops->allgather_front(g);
    }
    hipStream_t s = g->stream;
    const uint32_t words = p->v.block / 32, W = p->v.world;
    FGI_HIP(g, hipMemsetAsync(p->dcnt, 0, 8, s));
    hipLaunchKernelGGL(k_front_delta, dim3((words + 255) / 256), dim3(256), 0, s, words, g->inv_bm,
                       p->v.front_global + (uint64_t)p->v.rank * words, p->v.rank * words, p->dbuf, p->dcnt);
    FGI_HIP(g, hipGetLastError());
    uint64_t mine = 0;
    FGI_HIP(g, hipMemcpyAsync(&mine, p->dcnt, 8, hipMemcpyDeviceToHost, s));
    FGI_HIP(g, hipStreamSynchronize(s));
    uint64_t cnt[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    FGI_TRY(p->ops->allgather_count(g, mine, cnt));
    uint64_t total = 0;
    for (uint32_t q = 0; q < W; ++q) total += cnt[q];
    const uint64_t full_bytes = (uint64_t)(W - 1) * words * 4;
    if (mode == 0 && 8 * total >= full_bytes) {   // dense: the plain all-gather moves fewer bytes
        ++p->front_full;
        p->front_bytes += full_bytes;
        return p->ops->allgather_front(g);
    }
    ++p->front_delta;
    uint64_t n_recv = 0;
    FGI_TRY(p->ops->exchange_delta(g, cnt, &n_recv));
    p->front_bytes += 8 * n_recv;
    if (n_recv)
        hipLaunchKernelGGL(k_front_apply, dim3((uint32_t)((n_recv + 255) / 256)), dim3(256), 0, s, n_recv, p->rbuf,
                           p->v.front_global);
    FGI_HIP(g, hipGetLastError());
    return FGI_OK;
}

// a wave's first exchange is relative to an empty bitmap (every rank's inv_bm starts cleared)
fgi_status part_front_reset(fgi_graph* g) {
    PartState* p = ps(g);
    if (g->opt_front_exchange == 1) return FGI_OK;   // every exchange overwrites the whole bitmap
    FGI_HIP(g, hipMemsetAsync(p->v.front_global, 0, p->v.front_words_global * 4, g->stream));
    return FGI_OK;
}

fgi_status part_front_stats(fgi_graph* g, uint64_t* full, uint64_t* delta, uint64_t* bytes) {
    PartState* p = ps(g);
    if (!p) return FGI_EINVAL;
    *full = p->front_full;
    *delta = p->front_delta;
    *bytes = p->front_bytes;
    return FGI_OK;
}

fgi_status part_allreduce_sum(fgi_graph* g, const unsigned long long* dev_val, uint64_t* out, uint32_t count) {
    if (count < 1 || count > kPartRedMax) return set_err(g, FGI_EINVAL, "part_allreduce_sum: count %u", count);
    return ps(g)->ops->allreduce_sum(g, dev_val, out, count);
}

namespace {

// versions by slot; with partition codes (ig: code -> slot) entry c holds the version of slot ig[c]
__global__ void k_versions_all(uint32_t n, uint64_t seed, uint64_t* ver, const uint32_t* __restrict__ ig) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) ver[i] = synth_version(seed, ig ? ig[i] : (uint32_t)i);
}

__global__ void k_versions_local(uint32_t n, uint32_t base, uint64_t seed, unsigned long long* node,
                                 const uint32_t* __restrict__ ig) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) node[i] = synth_version(seed, ig ? ig[base + i] : base + i) | kW_Consistent;
}

// Row-range R-MAT (fgi_part_synth_rmat): edge i is a pure function of i, so every rank walks the
// global edge sequence and keeps only its share — the rows of the slots it owns (used == src) and the
// dependency-list entries of the slots it owns (dependant == dst, not stale) — without materialising
// the global edge list (at configs[2] that is 1.07G edges, 8.6 GB of keys per rank). Block b walks the
// contiguous edges [b * per, (b + 1) * per). Pass 0 counts both shares per block and adds every live
// edge to its dependant's weight (the list order: a slot's live dependencies over the whole graph);
// pass 1 writes the shares at the blocks' exclusive offsets (wave ballots, LDS cursors).
constexpr uint32_t kGenBlocks = 4096;
// With partition codes (gc: slot -> code, fill pass only) the kept keys hold codes, and each row entry's tag
// (computed from the slot ids, as build_rows_from_keys would: the dependant's version, + 1 if stale) goes to
// rtags. A slot's code has the slot's owner, so the shares and counts are those of the slot ids.
__global__ __launch_bounds__(256) void k_rmat_part(uint64_t m, uint64_t per, uint32_t scale, uint64_t seed, uint32_t base,
                                                   uint32_t n_local, uint32_t stale_pct, uint64_t stale_seed, int fill,
                                                   unsigned long long* blk_cnt, const unsigned long long* blk_off,
                                                   uint64_t* rows, uint64_t* ins, uint32_t* weight,
                                                   const uint32_t* __restrict__ gc, uint64_t* rtags) {
    __shared__ unsigned long long s_cur[2];
    __shared__ unsigned long long s_red[2][4];
    const uint64_t lo = (uint64_t)blockIdx.x * per, hi = lo + per < m ? lo + per : m;
    const uint32_t lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    if (fill && threadIdx.x < 2) s_cur[threadIdx.x] = blk_off[threadIdx.x * kGenBlocks + blockIdx.x];
    __syncthreads();
    unsigned long long nr = 0, ni = 0;
    for (uint64_t i0 = lo; i0 < hi; i0 += blockDim.x) {   // block-uniform
        const uint64_t i = i0 + threadIdx.x;
        bool own_row = false, own_in = false;
        uint32_t s = 0, d = 0;
        if (i < hi) {
            rmat_edge(i, scale, seed, &s, &d);
            own_row = s - base < n_local;
            const bool live = !synth_stale(stale_pct, stale_seed, s, d);
            own_in = live && d - base < n_local;
            if (!fill && live) atomicAdd(weight + d, 1u);
        }
        if (!fill) {
            nr += own_row;
            ni += own_in;
            continue;
        }
        const unsigned long long mr = __ballot(own_row), mi = __ballot(own_in);
        unsigned long long br = 0, bi = 0;
        if (lane == 0) {
            if (mr) br = atomicAdd(&s_cur[0], (unsigned long long)__popcll(mr));
            if (mi) bi = atomicAdd(&s_cur[1], (unsigned long long)__popcll(mi));
        }
        br = __shfl(br, 0, 64);
        bi = __shfl(bi, 0, 64);
        const unsigned long long lt = (1ull << lane) - 1ull;
        uint32_t sc = s, dc = d;
        if (gc && (own_row || own_in)) {
            sc = gc[s];
            dc = gc[d];
        }
        if (own_row) {
            const uint64_t at = br + __popcll(mr & lt);
            rows[at] = ((uint64_t)(sc - base) << 32) | dc;
            if (rtags) rtags[at] = synth_version(seed, d) + (synth_stale(stale_pct, stale_seed, s, d) ? 1u : 0u);
        }
        if (own_in) ins[bi + __popcll(mi & lt)] = ((uint64_t)(dc - base) << 32) | sc;
    }
    if (fill) return;
    for (int dd = 32; dd >= 1; dd >>= 1) {
        nr += __shfl_xor(nr, dd, 64);
        ni += __shfl_xor(ni, dd, 64);
    }
    if (lane == 0) {
        s_red[0][wid] = nr;
        s_red[1][wid] = ni;
    }
    __syncthreads();
    if (threadIdx.x < 2) {
        unsigned long long t = 0;
        for (uint32_t q = 0; q < blockDim.x / 64; ++q) t += s_red[threadIdx.x][q];
        blk_cnt[threadIdx.x * kGenBlocks + blockIdx.x] = t;
    }
}

__global__ void k_in_tags_synth(uint64_t m, const uint64_t* __restrict__ keys, uint32_t base, uint64_t seed,
                                uint64_t* tags, const uint32_t* __restrict__ ig) {
    const uint64_t e = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (e >= m) return;
    const uint32_t c = (uint32_t)(keys[e] >> 32) + base;   // the dependant (its code, with partition codes)
    tags[e] = synth_version(seed, ig ? ig[c] : c);
}

// the in-store's live entries (tag == version of the dependant's node): flag for the compaction
__global__ void k_in_live(uint64_t m, const uint64_t* __restrict__ keys, const uint64_t* __restrict__ tags,
                          const unsigned long long* __restrict__ node, uint32_t* flag) {
    const uint64_t e = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (e >= m) return;
    const uint64_t t = tags[e];
    flag[e] = (t != 0 && (node[(uint32_t)(keys[e] >> 32)] & kVMask) == t) ? 1u : 0u;
}

__global__ void k_compact64(uint64_t m, const uint64_t* __restrict__ in, const uint32_t* __restrict__ flag,
                            const uint32_t* __restrict__ pos, uint64_t* out) {
    const uint64_t e = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (e < m && flag[e]) out[pos[e]] = in[e];
}

__global__ void k_in_part_unique(uint64_t m, const uint64_t* __restrict__ k, uint32_t* keep) {
    const uint64_t e = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (e < m) keep[e] = (e == 0 || k[e] != k[e - 1]) ? 1u : 0u;
}

__global__ void k_in_part_rows(uint64_t m, const uint64_t* __restrict__ k, const uint32_t* __restrict__ keep,
                               const uint32_t* __restrict__ pos, uint32_t* src_out, uint64_t* off, uint32_t* len) {
    const uint64_t e = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (e >= m) return;
    const uint32_t d = (uint32_t)(k[e] >> 32);
    if (keep[e]) src_out[pos[e]] = (uint32_t)k[e];
    if (e == 0 || (uint32_t)(k[e - 1] >> 32) != d) off[d] = pos[e];
    if (e + 1 == m || (uint32_t)(k[e + 1] >> 32) != d) len[d] = pos[e] + keep[e];   // row end, fixed below
}

__global__ void k_in_part_fix(uint32_t n, const uint64_t* __restrict__ off, uint32_t* len) {
    const uint32_t d = blockIdx.x * blockDim.x + threadIdx.x;
    if (d < n && len[d]) len[d] -= (uint32_t)off[d];
}

// fgi_part_register_nodes: every listed slot's version goes into the replica; the owner installs the
// node (as fgi_register_nodes: the slot must be empty)
__global__ void k_part_register(uint32_t n, const uint32_t* __restrict__ slot, const uint64_t* __restrict__ version,
                                const uint32_t* __restrict__ flags, uint32_t base, uint32_t n_local, uint64_t* ver_all,
                                unsigned long long* node, uint32_t* row_len, unsigned long long* err) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const uint32_t s = slot[i];
    const uint64_t v = version[i];
    ver_all[s] = v;
    const uint32_t h = s - base;
    if (h >= n_local) return;
    if (word_is_current(node[h])) {
        atomicAdd(err, 1ull);
        return;
    }
    node[h] = v ? flags_to_word(v, flags ? flags[i] : FGI_CONSISTENT) : 0ull;
    row_len[h] = 0;
}

// fgi_part_load_edges: every edge of the batch that is live when loaded adds to its dependant's weight
__global__ void k_part_weight(uint64_t m, const uint32_t* __restrict__ dep, const uint64_t* __restrict__ tag,
                              const uint64_t* __restrict__ ver_all, uint32_t* weight) {
    const uint64_t e = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (e < m && tag[e] == ver_all[dep[e]]) atomicAdd(weight + dep[e], 1u);
}

inline uint32_t nblk(uint64_t n) { return (uint32_t)((n + 255) / 256); }

// ---- partition codes ------------------------------------------------------------------
// The code order: each rank's range sorted by weight class (8 classes per octave of weight + 1, the
// heaviest first, as the single device's labels), ties in slot order. A slot's code comes from its position
// in that order (pc_code), inside its owner's range ([q * block, q * block + n_local)), so a slot keeps its
// owner and every rank computes the same tables from the same global weights.
__device__ __forceinline__ uint32_t pc_class(uint32_t w) {
    const uint32_t x = w + 1u;
    const uint32_t l = 31u - (uint32_t)__builtin_clz(x);
    const uint32_t frac = l >= 3 ? (x >> (l - 3)) & 7u : (x << (3 - l)) & 7u;
    return l * kClassPerOctave + frac;
}
__global__ void k_pc_keys(uint32_t N, uint32_t B, const uint32_t* __restrict__ w, uint64_t* keys) {
    const uint32_t x = blockIdx.x * blockDim.x + threadIdx.x;
    if (x >= N) return;
    keys[x] = ((uint64_t)(x / B) << 48) | ((uint64_t)(kLabelClasses - 1u - pc_class(w[x])) << 32) | x;
}
// Position i of that order (rank q's range [q * B, q * B + n_q)) -> its code. Contiguous (T = 0), the heaviest
// slots of a rank would all fall to its first pull blocks (a pull block owns a fixed run of T slots); so the
// order is dealt round-robin over the runs of T slots instead: run j gets positions j, j + S, j + 2S, ... (S
// runs, the last one short; once the short run is full the rest are dealt over the S - 1 full runs), and
// every pull block starts with its share of the hubs, in weight order.
__device__ __forceinline__ uint32_t pc_code(uint32_t i, uint32_t N, uint32_t B, uint32_t T) {
    const uint32_t q = i / B, base = q * B, nq = min(B, N - base), r = i - base;
    if (T == 0 || nq <= T) return i;
    const uint32_t S = (nq + T - 1) / T, last = nq - (S - 1) * T, A = last * S;
    uint32_t run, k;
    if (r < A) {
        run = r % S;
        k = r / S;
    } else {
        run = (r - A) % (S - 1);
        k = last + (r - A) / (S - 1);
    }
    return base + run * T + k;
}
__global__ void k_pc_tables(uint32_t N, uint32_t B, uint32_t T, const uint64_t* __restrict__ sorted, uint32_t* gc,
                            uint32_t* ig) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= N) return;
    const uint32_t x = (uint32_t)sorted[i];
    const uint32_t c = pc_code(i, N, B, T);
    gc[x] = c;
    ig[c] = x;
}
// what was installed before the codes (registered nodes, versions, weights), moved to the codes
__global__ void k_pc_move_local(uint32_t nl, uint32_t base, const uint32_t* __restrict__ gc,
                                const unsigned long long* __restrict__ node_old, unsigned long long* node,
                                const uint32_t* __restrict__ used_old, uint32_t* used) {
    const uint32_t h = blockIdx.x * blockDim.x + threadIdx.x;
    if (h >= nl) return;
    const uint32_t c = gc[base + h] - base;
    node[c] = node_old[h];
    used[c] = used_old[h];
}
__global__ void k_pc_move_global(uint32_t N, const uint32_t* __restrict__ gc, const uint64_t* __restrict__ ver_old,
                                 uint64_t* ver, const uint32_t* __restrict__ w_old, uint32_t* w) {
    const uint32_t x = blockIdx.x * blockDim.x + threadIdx.x;
    if (x >= N) return;
    const uint32_t c = gc[x];
    ver[c] = ver_old[x];
    w[c] = w_old[x];
}
// local handles <-> local code indices (owned range only), in place
__global__ void k_pc_local(uint64_t n, uint32_t* a, const uint32_t* __restrict__ table, uint32_t base, uint32_t nl) {
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
        const uint32_t h = a[i];
        if (h < nl) a[i] = table[base + h] - base;
    }
}
// global slots -> codes, in place
__global__ void k_pc_global(uint64_t n, uint32_t* a, const uint32_t* __restrict__ gc, uint32_t N) {
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
        const uint32_t x = a[i];
        if (x < N) a[i] = gc[x];
    }
}

// exclusive scan of flag[0, m) into pos; returns the total (synchronises the stream)
fgi_status scan_flags(fgi_graph* g, const uint32_t* flag, uint32_t* pos, uint64_t m, uint64_t* total) {
    hipStream_t s = g->stream;
    size_t tb = 0;
    rocprim::exclusive_scan(nullptr, tb, flag, pos, 0u, (size_t)m, rocprim::plus<uint32_t>(), s);
    void* tmp = nullptr;
    FGI_HIP(g, hipMalloc(&tmp, std::max<size_t>(tb, 16)));
    rocprim::exclusive_scan(tmp, tb, flag, pos, 0u, (size_t)m, rocprim::plus<uint32_t>(), s);
    uint32_t lp = 0, lf = 0;
    hipMemcpyAsync(&lp, pos + m - 1, 4, hipMemcpyDeviceToHost, s);
    hipMemcpyAsync(&lf, flag + m - 1, 4, hipMemcpyDeviceToHost, s);
    const hipError_t e = hipStreamSynchronize(s);
    hipFree(tmp);
    FGI_HIP(g, e);
    *total = (uint64_t)lp + lf;
    return FGI_OK;
}

}  // namespace

// The owned slots' dependency lists (pull levels) from the in-store: its live entries (tag == the
// owned dependant node's version: the reference's d._used, Computed.cs:365-366) sorted and
// deduplicated into lists of global used ids, each ordered by the entries' weights (as the single
// engine: most-depended-on first), then the heads and the pull candidates. Local to the rank.
// Choose the codes from every slot's weight (weight_dev: [n_global], by slot; replaced by the weights in
// code order) and move what is already installed: the owned node words and |_used| counts, the version
// replica. Only before any row or dependency entry exists and while no detached handle is taken.
static fgi_status part_codes_choose(fgi_graph* g, uint32_t* weight_dev) {
    PartState* p = ps(g);
    const uint32_t N = p->v.n_global, B = p->v.block, base = p->v.base, nl = p->v.n_local;
    hipStream_t s = g->stream;
    FGI_TRY(fold(g));
    uint64_t *k0 = nullptr, *k1 = nullptr, *ver_old = nullptr;
    uint32_t *w_old = nullptr, *used_old = nullptr;
    unsigned long long* node_old = nullptr;
    void* tmp = nullptr;
    fgi_status st = FGI_OK;
    do {
        if (!g->pg_gc && (hipMalloc(&g->pg_gc, (size_t)N * 4) != hipSuccess || hipMalloc(&g->pg_ig, (size_t)N * 4) != hipSuccess)) {
            st = set_err(g, FGI_ENOMEM, "partition codes");
            break;
        }
        if (hipMalloc(&k0, (size_t)N * 8) != hipSuccess || hipMalloc(&k1, (size_t)N * 8) != hipSuccess) {
            st = set_err(g, FGI_ENOMEM, "partition code keys");
            break;
        }
        hipLaunchKernelGGL(k_pc_keys, dim3(nblk(N)), dim3(256), 0, s, N, B, weight_dev, k0);
        size_t tb = 0;
        rocprim::radix_sort_keys(nullptr, tb, k0, k1, (size_t)N, 0, 56, s);
        if (hipMalloc(&tmp, std::max<size_t>(tb, 16)) != hipSuccess) {
            st = set_err(g, FGI_ENOMEM, "partition code sort");
            break;
        }
        rocprim::radix_sort_keys(tmp, tb, k0, k1, (size_t)N, 0, 56, s);
        uint32_t pgrid = 0, ptpb = 0;
        pull_geometry(g, &pgrid, &ptpb);
        const uint32_t T = pgrid ? ptpb * kPullTile : 0u;   // the slots a pull block owns
        hipLaunchKernelGGL(k_pc_tables, dim3(nblk(N)), dim3(256), 0, s, N, B, T, k1, g->pg_gc, g->pg_ig);
        if (hipMalloc(&ver_old, (size_t)N * 8) != hipSuccess || hipMalloc(&w_old, (size_t)N * 4) != hipSuccess ||
            hipMalloc(&node_old, (size_t)std::max<uint32_t>(nl, 1) * 8) != hipSuccess ||
            hipMalloc(&used_old, (size_t)std::max<uint32_t>(nl, 1) * 4) != hipSuccess) {
            st = set_err(g, FGI_ENOMEM, "partition code moves");
            break;
        }
        hipMemcpyAsync(ver_old, p->v.ver_all, (size_t)N * 8, hipMemcpyDeviceToDevice, s);
        hipMemcpyAsync(w_old, weight_dev, (size_t)N * 4, hipMemcpyDeviceToDevice, s);
        hipMemcpyAsync(node_old, g->node, (size_t)nl * 8, hipMemcpyDeviceToDevice, s);
        hipMemcpyAsync(used_old, g->used_cnt, (size_t)nl * 4, hipMemcpyDeviceToDevice, s);
        hipLaunchKernelGGL(k_pc_move_global, dim3(nblk(N)), dim3(256), 0, s, N, g->pg_gc, ver_old, p->v.ver_all, w_old,
                           weight_dev);
        if (nl)
            hipLaunchKernelGGL(k_pc_move_local, dim3(nblk(nl)), dim3(256), 0, s, nl, base, g->pg_gc, node_old,
                               reinterpret_cast<unsigned long long*>(g->node), used_old, g->used_cnt);
        g->pg_gc_h.resize(N);
        g->pg_ig_h.resize(N);
        if (hipMemcpyAsync(g->pg_gc_h.data(), g->pg_gc, (size_t)N * 4, hipMemcpyDeviceToHost, s) != hipSuccess ||
            hipMemcpyAsync(g->pg_ig_h.data(), g->pg_ig, (size_t)N * 4, hipMemcpyDeviceToHost, s) != hipSuccess ||
            hipStreamSynchronize(s) != hipSuccess) {
            st = set_err(g, FGI_EDEVICE, "partition codes");
            break;
        }
    } while (0);
    for (void* q : {(void*)k0, (void*)k1, (void*)ver_old, (void*)w_old, (void*)node_old, (void*)used_old, tmp})
        if (q) hipFree(q);
    if (st != FGI_OK) return st;
    // the table's fingerprint: the wave's first all-reduce checks that every rank chose the same codes (each
    // rank chooses them alone, from the same arrays; a rank given other arrays would number slots otherwise)
    uint64_t hsh = 0xcbf29ce484222325ull;
    for (uint32_t x = 0; x < N; ++x) hsh = (hsh ^ g->pg_gc_h[x]) * 0x100000001b3ull;
    g->pg_hash = hsh ? hsh : 1;
    g->lbl_perm = true;
    touch(g);
    note_words(g);
    if (getenv("FGI_TRACE")) fprintf(stderr, "[fgi] partition codes: rank %u of %u, %u slots\n", p->v.rank, p->v.world, N);
    return FGI_OK;
}

// the first bulk load of a partition that wants codes (nothing loaded, no detached handle taken)
static bool part_codes_now(fgi_graph* g) {
    PartState* p = ps(g);
    return !g->lbl_perm && part_codes_wanted(g, p->v.n_global) && g->pool_top == 0 && p->in_n == 0 &&
           g->free_detached.size() == g->n_detached;
}

static fgi_status part_rebuild_lists(fgi_graph* g) {
    PartState* p = ps(g);
    hipStream_t s = g->stream;
    const uint64_t m = p->in_n;
    g->uin_epoch = 0;
    if (p->v.block % 32 != 0) return FGI_OK;   // pull levels all-gather whole bitmap words per rank
    FGI_HIP(g, hipMemsetAsync(g->uin_len, 0, (size_t)g->n_slots * 4, s));
    FGI_HIP(g, hipMemsetAsync(g->uin_off, 0, (size_t)g->n_slots * 8, s));
    if (!g->uin_src) {
        FGI_HIP(g, hipMalloc(&g->uin_src, 1024 * 4));
        g->uin_cap = 1024;
    }
    uint32_t *flag = nullptr, *pos = nullptr, *keep = nullptr, *kpos = nullptr;
    uint64_t *k1 = nullptr, *k2 = nullptr;
    void* st = nullptr;
    fgi_status rc = FGI_OK;
    uint64_t mi = 0;
    do {
        if (m) {
            if (hipMalloc(&flag, m * 4) != hipSuccess || hipMalloc(&pos, m * 4) != hipSuccess) {
                rc = set_err(g, FGI_ENOMEM, "dependency-list build buffers");
                break;
            }
            hipLaunchKernelGGL(k_in_live, dim3(nblk(m)), dim3(256), 0, s, m, p->in_keys, p->in_tags,
                               reinterpret_cast<const unsigned long long*>(g->node), flag);
            rc = scan_flags(g, flag, pos, m, &mi);
            if (rc != FGI_OK) break;
        }
        if (mi == 0) {
            rc = build_in_heads(g);
            break;
        }
        if (hipMalloc(&k1, mi * 8) != hipSuccess || hipMalloc(&k2, mi * 8) != hipSuccess ||
            hipMalloc(&keep, mi * 4) != hipSuccess || hipMalloc(&kpos, mi * 4) != hipSuccess) {
            rc = set_err(g, FGI_ENOMEM, "dependency-list build buffers");
            break;
        }
        hipLaunchKernelGGL(k_compact64, dim3(nblk(m)), dim3(256), 0, s, m, p->in_keys, flag, pos, k1);
        hipFree(flag);
        hipFree(pos);
        flag = pos = nullptr;
        size_t sb = 0;
        rocprim::radix_sort_keys(nullptr, sb, k1, k2, (size_t)mi, 0, 64, s);
        if (hipMalloc(&st, std::max(sb, (size_t)16)) != hipSuccess) {
            rc = set_err(g, FGI_ENOMEM, "sort temp");
            break;
        }
        rocprim::radix_sort_keys(st, sb, k1, k2, (size_t)mi, 0, 64, s);
        hipLaunchKernelGGL(k_in_part_unique, dim3(nblk(mi)), dim3(256), 0, s, mi, k2, keep);
        uint64_t total = 0;
        rc = scan_flags(g, keep, kpos, mi, &total);
        if (rc != FGI_OK) break;
        if (total > g->uin_cap) {
            hipFree(g->uin_src);
            g->uin_src = nullptr;
            if (hipMalloc(&g->uin_src, std::max<uint64_t>(total, 1024) * 4) != hipSuccess) {
                rc = set_err(g, FGI_ENOMEM, "dependency lists");
                break;
            }
            g->uin_cap = std::max<uint64_t>(total, 1024);
        }
        hipLaunchKernelGGL(k_in_part_rows, dim3(nblk(mi)), dim3(256), 0, s, mi, k2, keep, kpos, g->uin_src, g->uin_off,
                           g->uin_len);
        hipLaunchKernelGGL(k_in_part_fix, dim3(nblk(g->n_slots)), dim3(256), 0, s, g->n_slots, g->uin_off, g->uin_len);
        rc = sort_in_lists(g, total, p->weight, p->v.n_global);
        if (rc != FGI_OK) break;
        rc = build_in_heads(g);
        if (rc != FGI_OK) break;
        if (hipStreamSynchronize(s) != hipSuccess) rc = set_err(g, FGI_EDEVICE, "dependency-list build");
    } while (0);
    hipFree(flag);
    hipFree(pos);
    hipFree(k1);
    hipFree(k2);
    hipFree(keep);
    hipFree(kpos);
    hipFree(st);
    if (rc == FGI_OK) g->uin_epoch = g->mut_epoch;   // rows, versions and lists agree
    return rc;
}

fgi_status part_ensure_lists(fgi_graph* g) {
    PartState* p = ps(g);
    if (!p || g->uin_epoch == g->mut_epoch || p->in_n == 0) return FGI_OK;
    return part_rebuild_lists(g);
}

bool part_codes_wanted(const fgi_graph* g, uint32_t n_global) {
    return labels_capacity(n_global, g->opt_labels) != 0;   // fgi_config.labels / FGI_LABELS, auto from 2^25
}

const uint32_t* part_codes_in(const fgi_graph* g, uint64_t n, const uint32_t* in, std::vector<uint32_t>& out) {
    if (!g->lbl_perm || !in || n == 0) return in;
    out.resize(n);
    const uint64_t N = g->pg_gc_h.size();
    for (uint64_t i = 0; i < n; ++i) out[i] = in[i] < N ? g->pg_gc_h[in[i]] : in[i];
    return out.data();
}

fgi_status part_codes_local(fgi_graph* g, uint32_t* dev, uint64_t n, bool out) {
    PartState* p = ps(g);
    if (!g->lbl_perm || !p || n == 0) return FGI_OK;
    hipLaunchKernelGGL(k_pc_local, dim3(std::min<uint32_t>(nblk(n), 8192)), dim3(256), 0, g->stream, n, dev,
                       out ? g->pg_ig : g->pg_gc, p->v.base, p->v.n_local);
    FGI_HIP(g, hipGetLastError());
    return FGI_OK;
}

uint32_t part_code_local_h(const fgi_graph* g, uint32_t h, bool out) {
    const PartState* p = reinterpret_cast<const PartState*>(g->part);
    if (!g->lbl_perm || !p || h >= p->v.n_local) return h;
    return (out ? g->pg_ig_h : g->pg_gc_h)[p->v.base + h] - p->v.base;
}

// append m device entries (keys: dependant local << 32 | used global, tags) to the in-store
static fgi_status part_store_in(fgi_graph* g, const uint64_t* keys, const uint64_t* tags, uint64_t m) {
    PartState* p = ps(g);
    if (m == 0) return FGI_OK;
    if (p->in_n + m > p->in_cap) {
        const uint64_t cap = std::max<uint64_t>(p->in_n + m, p->in_cap + p->in_cap / 2);
        uint64_t *nk = nullptr, *nt = nullptr;
        if (hipMalloc(&nk, cap * 8) != hipSuccess || hipMalloc(&nt, cap * 8) != hipSuccess) {
            hipFree(nk);
            return set_err(g, FGI_ENOMEM, "dependency-entry store");
        }
        if (p->in_n) {
            FGI_HIP(g, hipMemcpyAsync(nk, p->in_keys, p->in_n * 8, hipMemcpyDeviceToDevice, g->stream));
            FGI_HIP(g, hipMemcpyAsync(nt, p->in_tags, p->in_n * 8, hipMemcpyDeviceToDevice, g->stream));
            FGI_HIP(g, hipStreamSynchronize(g->stream));
        }
        hipFree(p->in_keys);
        hipFree(p->in_tags);
        p->in_keys = nk;
        p->in_tags = nt;
        p->in_cap = cap;
    }
    FGI_HIP(g, hipMemcpyAsync(p->in_keys + p->in_n, keys, m * 8, hipMemcpyDefault, g->stream));
    FGI_HIP(g, hipMemcpyAsync(p->in_tags + p->in_n, tags, m * 8, hipMemcpyDefault, g->stream));
    FGI_HIP(g, hipStreamSynchronize(g->stream));
    p->in_n += m;
    return FGI_OK;
}

static void part_clear_store(PartState* p) {
    hipFree(p->in_keys);
    hipFree(p->in_tags);
    p->in_keys = p->in_tags = nullptr;
    p->in_n = p->in_cap = 0;
}

}  // namespace fgi

using namespace fgi;

extern "C" {

fgi_status fgi_part_unique_id(uint8_t* id128) {
    if (!id128) return FGI_EINVAL;
    if (!rccl_ok()) return FGI_ENOTSUP;
    ncclUniqueId id;
    if (rccl().GetUniqueId(&id) != ncclSuccess) return FGI_EDEVICE;
    std::memcpy(id128, id.internal, NCCL_UNIQUE_ID_BYTES);
    return FGI_OK;
}

static fgi_status part_alloc(fgi_graph* g, uint32_t n_global);

fgi_status fgi_part_init(fgi_graph* g, uint32_t n_global, const uint8_t* id128) {
    if (!g || !id128) return FGI_EINVAL;
    if (g->part) return set_err(g, FGI_ESTATE, "partition already initialised");
    if (!rccl_ok())
        return set_err(g, FGI_ENOTSUP, "RCCL not available (%s: %s)", rccl().path.c_str(), rccl().err.c_str());
    FGI_TRY(part_alloc(g, n_global));
    PartState* p = ps(g);
    ncclUniqueId id;
    std::memcpy(id.internal, id128, NCCL_UNIQUE_ID_BYTES);
    // non-blocking communicator: its creation (every rank must join) and every later call that reports
    // ncclInProgress are waited out with a bound (nccl_settle); FGI_RCCL_BLOCKING=1 makes the plain
    // blocking communicator instead (no bounds)
    const char* blk = getenv("FGI_RCCL_BLOCKING");
    ncclResult_t r;
    if (blk && blk[0] == '1') {
        r = rccl().CommInitRank(&p->comm, (int)p->v.world, id, g->rank);
    } else {
        ncclConfig_t cfg = NCCL_CONFIG_INITIALIZER;
        cfg.blocking = 0;
        r = rccl().CommInitRankConfig(&p->comm, (int)p->v.world, id, g->rank, &cfg);
        if (r == ncclInProgress) {
            const fgi_status st = nccl_settle(g, p->comm, r, "ncclCommInitRankConfig (every rank must join)",
                                              wait_limit_s("FGI_RCCL_INIT_TIMEOUT_S", 120.0));
            if (st != FGI_OK) {
                const std::string err = g->err;
                part_destroy(g);
                g->failed = false;   // the graph itself is intact: the partition was not created
                return set_err(g, st, "%s", err.c_str());
            }
            r = ncclSuccess;
        }
    }
    if (r != ncclSuccess) {
        part_destroy(g);
        return set_err(g, FGI_EDEVICE, "rank %d of %d: ncclCommInitRank: %s", g->rank, g->world, rccl().GetErrorString(r));
    }
    p->ops.reset(new RcclComm());
    return FGI_OK;
}

fgi_status fgi_part_init_host(fgi_graph* g, uint32_t n_global, fgi_allgather_fn fn, void* ctx) {
    if (!g || !fn) return FGI_EINVAL;
    if (g->part) return set_err(g, FGI_ESTATE, "partition already initialised");
    FGI_TRY(part_alloc(g, n_global));
    ps(g)->ops.reset(new HostComm(fn, ctx));
    return FGI_OK;
}

static fgi_status part_alloc(fgi_graph* g, uint32_t n_global) {
    if (!g || g->world < 1 || g->rank < 0 || g->rank >= g->world) return FGI_EINVAL;
    if (g->lbl_K) {   // a partition numbers its slots by rank ranges: no hub-first labels (a fresh graph drops them)
        // node words already written sit at labels K + x (and detached homes hold K + slot): dropping K
        // would lose them, so only a graph with nothing in it yet may join
        if (g->lbl_done || g->pool_top || g->nodes_written)
            return set_err(g, FGI_ESTATE, "a graph with registered nodes or loaded edges cannot join a partition");
        g->lbl_K = 0;
        g->n_slots = g->ext_slots;
        g->n_handles = g->ext_handles;
        g->free_detached.clear();
        for (uint32_t i = g->n_detached; i > 0; --i) g->free_detached.push_back(g->n_slots + i - 1);
    }
    if ((uint32_t)g->world > 8) return set_err(g, FGI_ENOTSUP, "at most 8 partitions (one node)");
    if (g->part) return set_err(g, FGI_ESTATE, "partition already initialised");
    const uint32_t W = (uint32_t)g->world;
    const uint32_t block = (uint32_t)(((uint64_t)n_global + W - 1) / W);
    if (g->n_slots < block) return set_err(g, FGI_EINVAL, "graph has %u slots, partition needs %u", g->n_slots, block);
    hipSetDevice(g->device);
    PartState* p = new PartState();
    g->part = p;
    p->v.rank = (uint32_t)g->rank;
    p->v.world = W;
    p->v.n_global = n_global;
    p->v.block = block;
    p->v.base = (uint32_t)std::min<uint64_t>((uint64_t)block * g->rank, n_global);
    p->v.n_local = (uint32_t)std::min<uint64_t>(block, n_global - p->v.base);
    p->v.sent_words = (uint64_t)n_global / 32 + 2;
    auto fail = [&](const char* what) {
        part_destroy(g);
        return set_err(g, FGI_ENOMEM, "partition allocation failed: %s", what);
    };
    // an empty slot's version is 0 in the replica (fgi_part_register_nodes writes only the present ones)
    if (hipMalloc(&p->v.ver_all, (size_t)n_global * 8) != hipSuccess ||
        hipMemset(p->v.ver_all, 0, (size_t)n_global * 8) != hipSuccess)
        return fail("versions");
    if (hipMalloc(&p->v.sent_bm, p->v.sent_words * 4) != hipSuccess) return fail("sent bitmap");
    if (hipMalloc(&p->v.send_buf, (size_t)W * block * 4) != hipSuccess) return fail("send buffer");
    if (hipMalloc(&p->v.recv_buf, (size_t)W * block * 4) != hipSuccess) return fail("recv buffer");
    if (hipMalloc(&p->v.send_cnt, (size_t)(W + 2) * 8) != hipSuccess) return fail("counts");
    if (hipMalloc(&p->all_cnt, (size_t)W * (W + 2) * 8) != hipSuccess) return fail("counts");
    if (hipMalloc(&p->scalar, 32) != hipSuccess) return fail("scalar");
    // even, so the hot heads' snapshot past its end (kHot / 32 words, build_candidates) is 64-bit aligned
    p->v.front_words_global = ((uint64_t)n_global / 32 + 3) & ~1ull;
    if (hipMalloc(&p->v.front_global, (p->v.front_words_global + kHot / 32) * 4) != hipSuccess) return fail("frontier bitmap");
    // the pull levels' probe summary covers the all-gathered bitmap: one bit per 64-bit word of it
    hipFree(g->sum_bm);
    g->sum_bm = nullptr;
    if (hipMalloc(&g->sum_bm, ((uint64_t)n_global / 4096 + 4) * 8) != hipSuccess) return fail("probe summary");
    if (hipMemset(p->v.front_global, 0, (p->v.front_words_global + kHot / 32) * 4) != hipSuccess) return fail("frontier bitmap");
    if (hipMalloc(&p->v.scratch_u64, 32) != hipSuccess) return fail("scratch");
    if (hipMalloc(&p->weight, (size_t)n_global * 4) != hipSuccess) return fail("list weights");
    if (hipMalloc(&p->dbuf, (size_t)(block / 32 + 1) * 8) != hipSuccess ||
        hipMalloc(&p->rbuf, (size_t)(W > 1 ? W - 1 : 1) * (block / 32 + 1) * 8) != hipSuccess ||
        hipMalloc(&p->dcnt, 8) != hipSuccess)
        return fail("frontier delta buffers");
    if (hipMemset(p->weight, 0, (size_t)n_global * 4) != hipSuccess) return fail("list weights");
    if (hipHostMalloc(reinterpret_cast<void**>(&p->all_cnt_host), (size_t)W * (W + 2) * 8) != hipSuccess)
        return fail("host");
    if (hipHostMalloc(reinterpret_cast<void**>(&p->scalar_host), 32) != hipSuccess) return fail("host");
    // planned waves: buckets of a2a_C words per peer (a push level's forwarded targets beyond that wait
    // for the next push level); 64 K ids per peer moves (world - 1) * 256 KB per rank and level
    p->a2a_C = p->a2a_cap = (uint32_t)std::min<uint64_t>(65536, (uint64_t)block + 1);
    if (hipMalloc(&p->a2a_send, (size_t)W * p->a2a_C * 4) != hipSuccess ||
        hipMalloc(&p->a2a_recv, (size_t)W * p->a2a_C * 4) != hipSuccess || hipMalloc(&p->a2a_cur, (size_t)W * 8) != hipSuccess ||
        hipMalloc(&p->red, (size_t)kPartRedMax * 8) != hipSuccess)
        return fail("planned-wave buffers");
    if (hipMemset(p->a2a_send, 0, (size_t)W * p->a2a_C * 4) != hipSuccess ||
        hipMemset(p->a2a_recv, 0, (size_t)W * p->a2a_C * 4) != hipSuccess)
        return fail("planned-wave buffers");
    if (hipHostMalloc(reinterpret_cast<void**>(&p->red_host), (size_t)kPartRedMax * 8) != hipSuccess) return fail("host");
    return FGI_OK;
}

fgi_status fgi_part_init_local(fgi_graph* const* gs, uint32_t P, uint32_t n_global) {
    if (!gs || P == 0) return FGI_EINVAL;
    for (uint32_t r = 0; r < P; ++r) {
        if (!gs[r] || gs[r]->rank != (int)r || gs[r]->world != (int)P) return FGI_EINVAL;
        FGI_TRY(part_alloc(gs[r], n_global));
    }
    auto grp = std::make_shared<LocalGroup>(std::vector<fgi_graph*>(gs, gs + P));
    for (uint32_t r = 0; r < P; ++r) ps(gs[r])->ops.reset(new LocalComm(grp, r));
    return FGI_OK;
}

// In-process driver: run_part_wave on every rank, one host thread per rank; the collectives meet
// in the group's LocalComm (exactly the level sequence of the RCCL path).
fgi_status fgi_part_local_invalidate(fgi_graph* const* gs, uint32_t P, uint32_t n_roots, const uint32_t* roots,
                                     const uint8_t* immediately, fgi_wave_stats* stats) {
    if (!gs || P == 0 || (n_roots && !roots)) return FGI_EINVAL;
    LocalComm* c0 = nullptr;
    for (uint32_t r = 0; r < P; ++r) {
        if (!gs[r] || !gs[r]->part || ps(gs[r])->v.world != P) return FGI_EINVAL;
        LocalComm* c = dynamic_cast<LocalComm*>(ps(gs[r])->ops.get());
        if (!c || c->rank != r) return set_err(gs[r], FGI_EINVAL, "graph is not rank %u of an in-process group", r);
        if (c0 && c->grp != c0->grp) return set_err(gs[r], FGI_EINVAL, "graphs of different in-process groups");
        c0 = c;
    }
    c0->grp->reset();
    std::vector<fgi_status> st(P, FGI_OK);
    std::vector<std::thread> ts;
    for (uint32_t r = 0; r < P; ++r) {
        ts.emplace_back([&, r]() {
            fgi_graph* g = gs[r];
            hipSetDevice(g->device);
            uint32_t* rd = nullptr;
            uint8_t* id = nullptr;
            fgi_status s = FGI_OK;
            if (n_roots && (hipMalloc(&rd, n_roots * 4) != hipSuccess ||
                            (immediately && hipMalloc(&id, n_roots) != hipSuccess)))
                s = set_err(g, FGI_ENOMEM, "root buffers");
            std::vector<uint32_t> mapped;
            const uint32_t* rr = part_codes_in(g, n_roots, roots, mapped);
            if (s == FGI_OK && n_roots) {
                if (hipMemcpy(rd, rr, n_roots * 4, hipMemcpyHostToDevice) != hipSuccess ||
                    (immediately && hipMemcpy(id, immediately, n_roots, hipMemcpyHostToDevice) != hipSuccess))
                    s = set_err(g, FGI_EDEVICE, "root copy");
            }
            if (s == FGI_OK) s = run_part_wave(g, n_roots, rd, id, stats ? stats + r : nullptr);
            if (s != FGI_OK) c0->grp->fail();
            hipFree(rd);
            hipFree(id);
            st[r] = s;
        });
    }
    for (auto& t : ts) t.join();
    for (uint32_t r = 0; r < P; ++r)
        if (st[r] != FGI_OK) return st[r];
    return FGI_OK;
}

// Checks that gs[0..P) is one in-process group, rank by rank; returns its first member's comm.
static fgi_status local_group(fgi_graph* const* gs, uint32_t P, LocalComm** out) {
    if (!gs || P == 0) return FGI_EINVAL;
    LocalComm* c0 = nullptr;
    for (uint32_t r = 0; r < P; ++r) {
        if (!gs[r] || !gs[r]->part || ps(gs[r])->v.world != P) return FGI_EINVAL;
        LocalComm* c = dynamic_cast<LocalComm*>(ps(gs[r])->ops.get());
        if (!c || c->rank != r) return set_err(gs[r], FGI_EINVAL, "graph is not rank %u of an in-process group", r);
        if (c0 && c->grp != c0->grp) return set_err(gs[r], FGI_EINVAL, "graphs of different in-process groups");
        c0 = c;
    }
    *out = c0;
    return FGI_OK;
}

// Runs fn(rank) on one host thread per rank of an in-process group (the ranks' collectives meet
// in the group); a failing rank fails the group so that the others leave their collectives.
extern "C++" template <class F>
static fgi_status local_run(fgi_graph* const* gs, uint32_t P, LocalComm* c0, F fn) {
    c0->grp->reset();
    std::vector<fgi_status> st(P, FGI_OK);
    std::vector<std::thread> ts;
    for (uint32_t r = 0; r < P; ++r) {
        ts.emplace_back([&, r]() {
            hipSetDevice(gs[r]->device);
            const fgi_status s = fn(r);
            if (s != FGI_OK) c0->grp->fail();
            st[r] = s;
        });
    }
    for (auto& t : ts) t.join();
    for (uint32_t r = 0; r < P; ++r)
        if (st[r] != FGI_OK) return st[r];
    return FGI_OK;
}

// fgi_part_run_batch on every rank of an in-process group. Each rank writes its step outputs into
// private buffers; they are merged afterwards: a detached handle comes from the slot's owner, the
// add_used results and set flags (which every rank computes) must agree across the ranks.
fgi_status fgi_part_local_run_batch(fgi_graph* const* gs, uint32_t P, uint32_t n_steps, const fgi_step* steps,
                                    uint32_t* out_ids, uint64_t cap, uint64_t* out_n, fgi_batch_stats* stats) {
    LocalComm* c0 = nullptr;
    FGI_TRY(local_group(gs, P, &c0));
    if (n_steps && !steps) return FGI_EINVAL;
    std::vector<std::vector<fgi_step>> rs(P, std::vector<fgi_step>(steps, steps + n_steps));
    std::vector<std::vector<std::vector<uint32_t>>> outs(P, std::vector<std::vector<uint32_t>>(n_steps));
    for (uint32_t r = 0; r < P; ++r)
        for (uint32_t k = 0; k < n_steps; ++k)
            if (steps[k].out) {
                outs[r][k].assign(steps[k].n, 0);   // u8 flags fit in the first quarter
                rs[r][k].out = outs[r][k].data();
            }
    std::vector<std::vector<uint32_t>> ids(P);
    std::vector<uint64_t> nid(P, 0);
    FGI_TRY(local_run(gs, P, c0, [&](uint32_t r) -> fgi_status {
        fgi_batch_stats* sr = stats ? stats + r : nullptr;
        if (sr) *sr = fgi_batch_stats{};
        if (out_ids) ids[r].resize(cap);
        return fgi_part_run_batch(gs[r], n_steps, rs[r].data(), out_ids ? ids[r].data() : nullptr, cap, &nid[r], sr);
    }));
    uint64_t total = 0;
    for (uint32_t r = 0; r < P; ++r) total += nid[r];
    if (out_n) *out_n = total;
    if (out_ids && total > cap) return FGI_ECAPACITY;
    for (uint32_t r = 0, at = 0; out_ids && r < P; at += (uint32_t)nid[r], ++r)
        std::memcpy(out_ids + at, ids[r].data(), nid[r] * 4);
    for (uint32_t k = 0; k < n_steps; ++k) {
        const fgi_step& sp = steps[k];
        if (!sp.out) continue;
        if (sp.kind == FGI_STEP_BEGIN_COMPUTE) {
            auto* o = static_cast<uint32_t*>(sp.out);
            for (uint32_t i = 0; i < sp.n; ++i) {
                o[i] = FGI_NONE;
                for (uint32_t r = 0; r < P; ++r) {
                    const PartView& v = ps(gs[r])->v;
                    if (sp.handles[i] - v.base < v.n_local) o[i] = outs[r][k][i];
                }
            }
        } else {
            const size_t bytes = sp.kind == FGI_STEP_SET_OUTPUT ? sp.n : (size_t)sp.n * 4;
            for (uint32_t r = 1; r < P; ++r)
                if (std::memcmp(outs[r].at(k).data(), outs[0][k].data(), bytes) != 0)
                    return set_err(gs[r], FGI_ESTATE, "step %u: rank %u's results differ from rank 0's", k, r);
            std::memcpy(sp.out, outs[0][k].data(), bytes);
        }
    }
    return FGI_OK;
}

// fgi_part_prune on every rank of an in-process group (stats: P entries, nullable).
fgi_status fgi_part_local_prune(fgi_graph* const* gs, uint32_t P, fgi_prune_stats* stats) {
    LocalComm* c0 = nullptr;
    FGI_TRY(local_group(gs, P, &c0));
    return local_run(gs, P, c0, [&](uint32_t r) { return fgi_part_prune(gs[r], stats ? stats + r : nullptr); });
}

// The RCCL library the engine's collectives bind to: the file its entry points were resolved from
// (rccl(): /opt/rocm's librccl, opened privately, whatever other RCCL the process has loaded).
fgi_status fgi_rccl_info(int* version, char* path, uint64_t cap) {
    if (!rccl_ok()) return FGI_ENOTSUP;
    int v = 0;
    if (rccl().GetVersion(&v) != ncclSuccess) return FGI_EDEVICE;
    if (version) *version = v;
    if (path && cap) {
        Dl_info info{};
        const char* f = (dladdr(reinterpret_cast<void*>(rccl().GetVersion), &info) && info.dli_fname) ? info.dli_fname
                                                                                                      : rccl().path.c_str();
        std::strncpy(path, f, cap - 1);
        path[cap - 1] = 0;
    }
    return FGI_OK;
}

fgi_status fgi_part_synth_rmat(fgi_graph* g, uint32_t scale, uint32_t edge_factor, uint64_t seed, uint32_t stale_pct,
                               uint64_t stale_seed) {
    if (!g || !g->part || scale == 0 || scale > 31 || edge_factor == 0 || stale_pct > 100) return FGI_EINVAL;
    PartState* p = ps(g);
    if ((1ull << scale) != p->v.n_global) return set_err(g, FGI_EINVAL, "partition was initialised for %u slots",
                                                         p->v.n_global);
    hipSetDevice(g->device);
    hipStream_t s = g->stream;
    const uint32_t N = p->v.n_global, base = p->v.base, nl = p->v.n_local;
    FGI_HIP(g, hipMemsetAsync(g->node, 0, (size_t)g->n_handles * 8, s));
    FGI_HIP(g, hipMemsetAsync(g->vis_bm, 0, g->bm_words * 4, s));   // a new node table
    g->v_dirty = false;
    g->vis_stale = false;
    note_words(g);
    // partition codes: chosen after the count pass (the weights); a graph that already has codes keeps them
    const bool choose = !g->lbl_perm && part_codes_wanted(g, N) && g->free_detached.size() == g->n_detached;
    hipLaunchKernelGGL(k_versions_local, dim3((nl + 255) / 256), dim3(256), 0, s, nl, base, seed,
                       reinterpret_cast<unsigned long long*>(g->node), g->lbl_perm ? g->pg_ig : (const uint32_t*)nullptr);
    hipLaunchKernelGGL(k_versions_all, dim3((N + 255) / 256), dim3(256), 0, s, N, seed, p->v.ver_all,
                       g->lbl_perm ? g->pg_ig : (const uint32_t*)nullptr);
    part_clear_store(p);
    FGI_HIP(g, hipMemsetAsync(p->weight, 0, (size_t)N * 4, s));
    // the rank's rows and dependency entries, generated by edge-index range (k_rmat_part)
    const uint64_t m = (uint64_t)edge_factor << scale;
    const uint64_t per = (m + kGenBlocks - 1) / kGenBlocks;
    unsigned long long *cnt = nullptr, *off = nullptr;
    uint64_t *rows = nullptr, *ins = nullptr, *tags = nullptr, *rtags = nullptr;
    auto cleanup = [&]() {
        hipFree(cnt);
        hipFree(off);
        hipFree(rows);
        hipFree(ins);
        hipFree(tags);
        hipFree(rtags);
    };
    fgi_status st = FGI_OK;
    do {
        if (hipMalloc(&cnt, 2 * kGenBlocks * 8) != hipSuccess || hipMalloc(&off, 2 * kGenBlocks * 8) != hipSuccess) {
            st = set_err(g, FGI_ENOMEM, "generator counts");
            break;
        }
        hipLaunchKernelGGL(k_rmat_part, dim3(kGenBlocks), dim3(256), 0, s, m, per, scale, seed, base, nl, stale_pct,
                           stale_seed, 0, cnt, (const unsigned long long*)nullptr, (uint64_t*)nullptr, (uint64_t*)nullptr,
                           p->weight, (const uint32_t*)nullptr, (uint64_t*)nullptr);
        if (choose) {   // the weights by slot are complete: codes, then the versions at them
            g->pool_top = 0;   // the rows are rebuilt below
            st = part_codes_choose(g, p->weight);
            if (st != FGI_OK) break;
            hipLaunchKernelGGL(k_versions_local, dim3((nl + 255) / 256), dim3(256), 0, s, nl, base, seed,
                               reinterpret_cast<unsigned long long*>(g->node), (const uint32_t*)g->pg_ig);
            hipLaunchKernelGGL(k_versions_all, dim3((N + 255) / 256), dim3(256), 0, s, N, seed, p->v.ver_all,
                               (const uint32_t*)g->pg_ig);
        } else if (g->lbl_perm) {   // the weights by slot into code order
            uint32_t* w2 = nullptr;
            if (hipMalloc(&w2, (size_t)N * 4) != hipSuccess) {
                st = set_err(g, FGI_ENOMEM, "weights");
                break;
            }
            hipMemcpyAsync(w2, p->weight, (size_t)N * 4, hipMemcpyDeviceToDevice, s);
            hipLaunchKernelGGL(k_pc_move_global, dim3(nblk(N)), dim3(256), 0, s, N, (const uint32_t*)g->pg_gc,
                               (const uint64_t*)p->v.ver_all, p->v.ver_all, (const uint32_t*)w2, p->weight);
            hipStreamSynchronize(s);
            hipFree(w2);
            // k_pc_move_global also moved ver_all: write it again at the codes
            hipLaunchKernelGGL(k_versions_all, dim3((N + 255) / 256), dim3(256), 0, s, N, seed, p->v.ver_all,
                               (const uint32_t*)g->pg_ig);
        }
        std::vector<unsigned long long> hc(2 * kGenBlocks), ho(2 * kGenBlocks);
        if (hipMemcpyAsync(hc.data(), cnt, hc.size() * 8, hipMemcpyDeviceToHost, s) != hipSuccess ||
            hipStreamSynchronize(s) != hipSuccess) {
            st = set_err(g, FGI_EDEVICE, "generator count pass");
            break;
        }
        uint64_t tot[2] = {0, 0};
        for (int c = 0; c < 2; ++c)
            for (uint32_t b = 0; b < kGenBlocks; ++b) {
                ho[c * kGenBlocks + b] = tot[c];
                tot[c] += hc[c * kGenBlocks + b];
            }
        const uint64_t mo = tot[0], mi = tot[1];
        if (hipMalloc(&rows, std::max<uint64_t>(mo, 1) * 8) != hipSuccess ||
            hipMalloc(&ins, std::max<uint64_t>(mi, 1) * 8) != hipSuccess ||
            hipMalloc(&tags, std::max<uint64_t>(mi, 1) * 8) != hipSuccess ||
            (g->lbl_perm && hipMalloc(&rtags, std::max<uint64_t>(mo, 1) * 8) != hipSuccess)) {
            st = set_err(g, FGI_ENOMEM, "owned edges");
            break;
        }
        FGI_HIP(g, hipMemcpyAsync(off, ho.data(), ho.size() * 8, hipMemcpyHostToDevice, s));
        hipLaunchKernelGGL(k_rmat_part, dim3(kGenBlocks), dim3(256), 0, s, m, per, scale, seed, base, nl, stale_pct,
                           stale_seed, 1, cnt, (const unsigned long long*)off, rows, ins, (uint32_t*)nullptr,
                           g->lbl_perm ? (const uint32_t*)g->pg_gc : (const uint32_t*)nullptr, rtags);
        if (mi)
            hipLaunchKernelGGL(k_in_tags_synth, dim3(nblk(mi)), dim3(256), 0, s, mi, ins, base, seed, tags,
                               g->lbl_perm ? (const uint32_t*)g->pg_ig : (const uint32_t*)nullptr);
        if (hipStreamSynchronize(s) != hipSuccess) {
            st = set_err(g, FGI_EDEVICE, "generator fill pass");
            break;
        }
        hipFree(cnt);
        hipFree(off);
        cnt = off = nullptr;
        // rows: (owned used << 32 | global dependant), tags synthesised from global ids (with codes: from the
        // slot ids, by the generator)
        st = build_rows_from_keys(g, mo, rows, rtags, seed, stale_pct, stale_seed, base, base);
        if (st != FGI_OK) break;
        hipFree(rows);
        rows = nullptr;
        st = part_store_in(g, ins, tags, mi);
        if (st != FGI_OK) break;
        st = part_rebuild_lists(g);
    } while (0);
    cleanup();
    return st;
}

fgi_status fgi_part_register_nodes(fgi_graph* g, uint32_t n, const uint32_t* slot, const uint64_t* version,
                                   const uint32_t* state_flags) {
    if (!g || (n && (!slot || !version))) return FGI_EINVAL;
    if (!g->part) return set_err(g, FGI_ESTATE, "fgi_part_register_nodes: partition not initialised");
    PartState* p = ps(g);
    for (uint32_t i = 0; i < n; ++i) {
        if (slot[i] >= p->v.n_global) return set_err(g, FGI_EINVAL, "slot %u out of range", slot[i]);
        if (version[i] > kVMask) return set_err(g, FGI_EINVAL, "version of slot %u exceeds 2^56-1", slot[i]);
        if (state_flags && (state_flags[i] & 3u) == 3u) return set_err(g, FGI_EINVAL, "bad state for slot %u", slot[i]);
    }
    if (n == 0) return FGI_OK;
    std::vector<uint32_t> mapped;
    slot = part_codes_in(g, n, slot, mapped);   // partition codes
    hipSetDevice(g->device);
    hipStream_t s = g->stream;
    FGI_TRY(fold(g));
    uint32_t *ds = nullptr, *df = nullptr;
    uint64_t* dv = nullptr;
    fgi_status st = FGI_OK;
    if (hipMalloc(&ds, (size_t)n * 4) != hipSuccess || hipMalloc(&dv, (size_t)n * 8) != hipSuccess ||
        (state_flags && hipMalloc(&df, (size_t)n * 4) != hipSuccess)) {
        st = set_err(g, FGI_ENOMEM, "register buffers");
    } else {
        hipMemcpyAsync(ds, slot, (size_t)n * 4, hipMemcpyHostToDevice, s);
        hipMemcpyAsync(dv, version, (size_t)n * 8, hipMemcpyHostToDevice, s);
        if (df) hipMemcpyAsync(df, state_flags, (size_t)n * 4, hipMemcpyHostToDevice, s);
        hipMemsetAsync(p->scalar, 0, 8, s);
        hipLaunchKernelGGL(k_part_register, dim3(nblk(n)), dim3(256), 0, s, n, ds, dv, df, p->v.base, p->v.n_local,
                           p->v.ver_all, reinterpret_cast<unsigned long long*>(g->node), g->row_len, p->scalar);
        unsigned long long bad = 0;
        hipMemcpyAsync(&bad, p->scalar, 8, hipMemcpyDeviceToHost, s);
        if (hipStreamSynchronize(s) != hipSuccess) st = set_err(g, FGI_EDEVICE, "register");
        else if (bad) st = set_err(g, FGI_ESTATE, "%llu owned slots already had a current node", bad);
    }
    hipFree(ds);
    hipFree(dv);
    hipFree(df);
    touch(g);          // versions changed: the pull lists are rebuilt before the next wave
    note_words(g);
    return st;
}

fgi_status fgi_part_load_edges(fgi_graph* g, uint64_t m, const uint32_t* used, const uint32_t* dependant,
                               const uint64_t* tag) {
    if (!g || (m && (!used || !dependant || !tag))) return FGI_EINVAL;
    if (!g->part) return set_err(g, FGI_ESTATE, "fgi_part_load_edges: partition not initialised");
    PartState* p = ps(g);
    const uint32_t base = p->v.base, nl = p->v.n_local, N = p->v.n_global;
    for (uint64_t e = 0; e < m; ++e) {
        if (used[e] >= N || dependant[e] >= N)
            return set_err(g, FGI_EINVAL, "edge %llu out of range", (unsigned long long)e);
        if (tag[e] == 0) return set_err(g, FGI_EINVAL, "edge %llu has tag 0 (LTags are positive)", (unsigned long long)e);
    }
    hipSetDevice(g->device);
    // list weights: every rank sees the whole batch (and every version, ver_all). At the first bulk load of a
    // partition that wants codes they decide the codes (by slot), which then number the batch and all else.
    const bool choose = m && part_codes_now(g);
    std::vector<uint32_t> mu, md;
    if (!choose) {
        used = part_codes_in(g, m, used, mu);
        dependant = part_codes_in(g, m, dependant, md);
    }
    if (m) {
        hipStream_t s = g->stream;
        uint32_t* dd = nullptr;
        uint64_t* dt = nullptr;
        fgi_status st = FGI_OK;
        if (hipMalloc(&dd, m * 4) != hipSuccess || hipMalloc(&dt, m * 8) != hipSuccess) {
            st = set_err(g, FGI_ENOMEM, "weight buffers");
        } else {
            hipMemcpyAsync(dd, dependant, m * 4, hipMemcpyHostToDevice, s);
            hipMemcpyAsync(dt, tag, m * 8, hipMemcpyHostToDevice, s);
            hipLaunchKernelGGL(k_part_weight, dim3(nblk(m)), dim3(256), 0, s, m, dd, dt, p->v.ver_all, p->weight);
            if (hipStreamSynchronize(s) != hipSuccess) st = set_err(g, FGI_EDEVICE, "weights");
        }
        hipFree(dd);
        hipFree(dt);
        FGI_TRY(st);
    }
    if (choose) {
        FGI_TRY(part_codes_choose(g, p->weight));
        used = part_codes_in(g, m, used, mu);
        dependant = part_codes_in(g, m, dependant, md);
    }
    std::vector<uint64_t> rk, rt, ik, it;
    for (uint64_t e = 0; e < m; ++e) {
        if (used[e] - base < nl) {   // a row this rank owns: (local used, global dependant)
            rk.push_back(((uint64_t)(used[e] - base) << 32) | dependant[e]);
            rt.push_back(tag[e]);
        }
        if (dependant[e] - base < nl) {   // a dependency entry of a slot this rank owns
            ik.push_back(((uint64_t)(dependant[e] - base) << 32) | used[e]);
            it.push_back(tag[e]);
        }
    }
    FGI_TRY(load_rows(g, rk.size(), rk.data(), rt.data(), base, base));
    FGI_TRY(part_store_in(g, ik.data(), it.data(), ik.size()));
    return part_rebuild_lists(g);
}

fgi_status fgi_part_invalidate(fgi_graph* g, uint32_t n_roots, const uint32_t* roots_dev, const uint8_t* imm_dev,
                               uint64_t* out_n, fgi_wave_stats* stats) {
    if (!g || !g->part || (n_roots && !roots_dev)) return FGI_EINVAL;
    hipSetDevice(g->device);
    if (g->lbl_perm && n_roots) {   // the roots' codes (the caller's buffer stays as it is)
        PartState* p = ps(g);
        if (p->roots_cap < n_roots) {
            hipFree(p->roots_codes);
            p->roots_codes = nullptr;
            p->roots_cap = 0;
            FGI_HIP(g, hipMalloc(&p->roots_codes, (size_t)n_roots * 4));
            p->roots_cap = n_roots;
        }
        FGI_HIP(g, hipMemcpyAsync(p->roots_codes, roots_dev, (size_t)n_roots * 4, hipMemcpyDeviceToDevice, g->stream));
        hipLaunchKernelGGL(k_pc_global, dim3(std::min<uint32_t>(nblk(n_roots), 4096)), dim3(256), 0, g->stream,
                           (uint64_t)n_roots, p->roots_codes, (const uint32_t*)g->pg_gc, p->v.n_global);
        roots_dev = p->roots_codes;
    }
    FGI_TRY(run_part_wave(g, n_roots, roots_dev, imm_dev, stats));
    if (out_n) *out_n = g->last_wave_n;
    return FGI_OK;
}

fgi_status fgi_part_front_stats(fgi_graph* g, uint64_t* full, uint64_t* delta, uint64_t* bytes) {
    if (!g || !g->part || !full || !delta || !bytes) return FGI_EINVAL;
    return part_front_stats(g, full, delta, bytes);
}

fgi_status fgi_part_export_ids(fgi_graph* g, uint32_t* out_ids, uint64_t cap, uint64_t* out_n) {
    if (!g || !g->part) return FGI_EINVAL;
    const uint64_t n = g->last_wave_n;
    if (out_n) *out_n = n;
    if (!out_ids) return FGI_OK;
    if (n > cap) return FGI_ECAPACITY;
    hipSetDevice(g->device);
    FGI_HIP(g, hipMemcpy(out_ids, g->inv, n * 4, hipMemcpyDeviceToHost));
    const uint32_t base = ps(g)->v.base;
    for (uint64_t i = 0; i < n; ++i) out_ids[i] = part_slot_of(g, out_ids[i] + base);   // local -> global slot
    if (g->lbl_perm) std::sort(out_ids, out_ids + n);   // ascending slots
    return FGI_OK;
}

}  // extern "C"
