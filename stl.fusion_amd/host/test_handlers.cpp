// test_handlers.cpp — InvalidatedHandlerSetTest (tests/Stl.Fusion.Tests/Internal/
// InvalidatedHandlerSetTest.cs:10-48) restated over the host mirror's InvalidatedHandlerSet.
// Host code only (no engine call): runs on the CPU, from tests/test_gpu_host.py.
#include <cstdio>
#include <random>
#include <set>
#include <vector>

#include "fusion.hpp"

using namespace fusion;

static int g_fail = 0, g_checks = 0;
#define CHECK(cond)                                                                       \
    do {                                                                                  \
        ++g_checks;                                                                       \
        if (!(cond)) {                                                                    \
            std::fprintf(stderr, "%s:%d: CHECK(%s) failed\n", __FILE__, __LINE__, #cond); \
            ++g_fail;                                                                     \
        }                                                                                 \
    } while (0)

static std::mt19937_64 rng(0x1A5E7);

// RunTest(size, removalProbability): every handler runs once; after removing a random subset,
// exactly the rest run, once each, and no removed one
static void run_test(int size, double p) {
    std::multiset<int> used;
    std::vector<InvalidatedHandler> actions;
    for (int i = 0; i < size; ++i)
        actions.push_back(std::make_shared<const std::function<void(Computed&)>>([&used, i](Computed&) { used.insert(i); }));
    InvalidatedHandlerSet set;
    for (auto& a : actions) set.Add(a);
    for (auto& a : actions) set.Add(a);   // Add is idempotent per handler
    Computed none;                        // handlers ignore the argument (the reference passes null)
    set.Invoke(none);
    CHECK((int)used.size() == size && (int)std::set<int>(used.begin(), used.end()).size() == size);
    CHECK(set.Spilled() == (size > (int)InvalidatedHandlerSet::ListSize));
    std::bernoulli_distribution sample(p);
    std::set<int> removed;
    for (int i = 0; i < size; ++i)
        if (sample(rng)) removed.insert(i);
    for (int i : removed) set.Remove(actions[i]);
    used.clear();
    set.Invoke(none);
    CHECK((int)used.size() == size - (int)removed.size());
    CHECK(std::set<int>(used.begin(), used.end()).size() == used.size());
    for (int i : used) CHECK(!removed.count(i));
    CHECK(set.Size() == used.size());
}

int main() {
    const int iterations = 200;
    for (int it = 0; it < iterations; ++it)
        for (int size = 0; size < 10; ++size) run_test(size, (it + 1.0) / iterations);
    // list order is kept by Remove (InvalidatedHandlerSet.cs:88-91)
    std::vector<int> order;
    std::vector<InvalidatedHandler> hs;
    for (int i = 0; i < 5; ++i)
        hs.push_back(std::make_shared<const std::function<void(Computed&)>>([&order, i](Computed&) { order.push_back(i); }));
    InvalidatedHandlerSet set;
    for (auto& h : hs) set.Add(h);
    set.Remove(hs[1]);
    set.Remove(nullptr);
    Computed none;
    set.Invoke(none);
    CHECK((order == std::vector<int>{0, 2, 3, 4}));
    std::printf("%d/%d checks passed\n", g_checks - g_fail, g_checks);
    return g_fail ? 1 : 0;
}
