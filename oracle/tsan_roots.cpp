// tsan_roots.cpp — TEST INFRASTRUCTURE ONLY. Drives the oracle's threaded paths under
// -fsanitize=thread (oracle/Makefile target `tsan`, run by tests/test_oracle_tsan.py):
//   - parallel-over-roots cascade (fgo_invalidate_slots with n_threads > 1), the cpu_baseline leg;
//   - the threaded bulk operations (fgo_gen_rmat, fgo_gen_tags, fgo_load_graph, snapshot/restore).
// Every thread count must give the sequential result: the same invalidated set, E_trav and final
// state of every node (the restatement of tests/test_oracle_scenarios.py's
// test_parallel_over_roots_equals_sequential, on a larger R-MAT graph with 25% stale edges).
#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "fgo.h"

struct Result {
    std::vector<uint32_t> inv;
    uint64_t e_trav = 0, v_inv = 0;
    std::vector<uint64_t> ver;
    std::vector<uint32_t> flags;
};

static Result run(fgo* o, uint32_t n, const std::vector<uint32_t>& roots, uint32_t threads) {
    Result r;
    if (fgo_restore(o) != 0) std::abort();
    fgo_clear_log(o);
    fgo_stats st{};
    if (fgo_invalidate_slots(o, (uint32_t)roots.size(), roots.data(), nullptr, threads, &st) != 0) std::abort();
    r.inv.resize(fgo_inv_log(o, nullptr, 0));
    fgo_inv_log(o, r.inv.data(), r.inv.size());
    std::sort(r.inv.begin(), r.inv.end());
    r.e_trav = st.e_trav;
    r.v_inv = st.v_inv;
    r.ver.resize(n);
    r.flags.resize(n);
    fgo_dump_states(o, r.ver.data(), r.flags.data());
    return r;
}

int main(int argc, char** argv) {
    const uint32_t scale = argc > 1 ? (uint32_t)std::atoi(argv[1]) : 13;
    const uint32_t n = 1u << scale, ef = 8;
    const uint64_t seed = 0x5EED7541;
    fgo_set_threads(8);
    const uint64_t m = fgo_gen_rmat(scale, ef, seed, nullptr, nullptr);
    std::vector<uint32_t> src(m), dst(m);
    fgo_gen_rmat(scale, ef, seed, src.data(), dst.data());
    std::vector<uint64_t> tag(m), ver(n);
    fgo_gen_tags(m, src.data(), dst.data(), seed, 25, seed ^ 0xC0, tag.data());
    for (uint32_t s = 0; s < n; ++s) ver[s] = fgo_version_of(seed, s);
    // a mix of states: some Computing, some with a delay
    std::vector<uint32_t> flags(n);
    for (uint32_t s = 0; s < n; ++s) {
        const uint64_t h = fgo_splitmix64(seed ^ s);
        flags[s] = (h % 10 == 0) ? FGO_COMPUTING : FGO_CONSISTENT;
        if ((h >> 8) % 10 == 0) flags[s] |= FGO_F_HAS_DELAY;
    }
    std::vector<uint32_t> deg(n, 0);
    for (uint64_t i = 0; i < m; ++i) ++deg[src[i]];
    std::vector<uint32_t> roots(256);
    roots.resize(fgo_gen_roots(256, n, seed ^ 0x1, deg.data(), roots.data()));

    fgo* o = fgo_create(n);
    if (!o || fgo_load_graph(o, n, ver.data(), flags.data(), m, src.data(), dst.data(), tag.data()) != 0) return 2;
    if (fgo_snapshot(o) != 0) return 2;
    const Result base = run(o, n, roots, 1);
    int bad = 0;
    for (uint32_t t : {2u, 4u, 8u}) {
        const Result r = run(o, n, roots, t);
        const bool same = r.inv == base.inv && r.e_trav == base.e_trav && r.v_inv == base.v_inv &&
                          r.ver == base.ver && r.flags == base.flags;
        std::printf("threads=%u v_inv=%llu e_trav=%llu %s\n", t, (unsigned long long)r.v_inv,
                    (unsigned long long)r.e_trav, same ? "same" : "DIFFERENT");
        bad += !same;
    }
    fgo_destroy(o);
    std::printf("edges=%llu roots=%zu v_inv=%llu: %s\n", (unsigned long long)m, roots.size(),
                (unsigned long long)base.v_inv, bad ? "FAIL" : "ok");
    return bad ? 1 : 0;
}
