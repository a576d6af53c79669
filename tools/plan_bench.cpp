// plan_bench.cpp -- host-only timing of the GN elimination planner (sparse_plan.h) on a graph's
// directed edge list, without a GPU.  Input (stdin): "N E" then E lines "ii jj" (global keyframe
// ids, the op's ii/jj).  The pose pairs are formed exactly as gn_driver.hip's build_plan does
// (unique ids, first pose pinned, pairs in first-appearance order).
//   hipcc -O2 -std=c++17 -I mast3r-slam_amd/csrc tools/plan_bench.cpp -o /tmp/plan_bench
//   python tools/plan_graph.py cfg4 | /tmp/plan_bench
#include <chrono>
#include <cstdio>
#include <map>

#include "sparse_plan.h"

using namespace m3s;

int main() {
    long long N = 0, E = 0;
    if (scanf("%lld %lld", &N, &E) != 2) return 1;
    std::vector<long long> ii(E), jj(E);
    for (long long e = 0; e < E; e++)
        if (scanf("%lld %lld", &ii[e], &jj[e]) != 2) return 1;
    std::vector<long long> u(ii);
    u.insert(u.end(), jj.begin(), jj.end());
    std::sort(u.begin(), u.end());
    u.erase(std::unique(u.begin(), u.end()), u.end());
    auto row = [&](long long id) { return (int)(std::lower_bound(u.begin(), u.end(), id) - u.begin()) - 1; };
    const int npose = (int)N - 1;
    std::vector<int> slot((size_t)npose * npose, -1);
    std::vector<std::pair<int, int>> pairs;
    int nblk = npose;
    for (long long e = 0; e < E; e++) {
        const int i = row(ii[e]), j = row(jj[e]);
        if (i >= 0 && j >= 0 && i != j && slot[(size_t)i * npose + j] < 0) {
            slot[(size_t)i * npose + j] = slot[(size_t)j * npose + i] = nblk++;
            pairs.push_back({std::min(i, j), std::max(i, j)});
        }
    }
    struct P {
        const char* name;
        RoundPolicy pol;
    };
    // the driver's defaults (gn_driver.hip fused_policy / hybrid_policy / multi_policy)
    const P pols[] = {{"fused", {true, 64, 1, 64, kTailPoseMax, 4, true}},
                      {"hybrid", {false, 64, 1, 64, kTailPoseMax, 4, true}},
                      {"multi", {false, 32, 2, 64, 0, 0, false}}};
    printf("{\"npose\": %d, \"pairs\": %zu, \"plans\": {", npose, pairs.size());
    bool first = true;
    for (const P& p : pols) {
        SparsePlan sp;
        std::vector<double> t;
        for (int rep = 0; rep < 21; rep++) {
            const auto a = std::chrono::steady_clock::now();
            build_sparse_plan(pairs, nblk, npose, p.pol, sp);
            t.push_back(std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - a).count());
        }
        std::sort(t.begin(), t.end());
        size_t fmax = 0;
        for (size_t k = 0; k + 1 < sp.fptr.size(); k++) fmax = std::max(fmax, (size_t)(sp.fptr[k + 1] - sp.fptr[k]));
        printf("%s\"%s\": {\"us_median\": %.1f, \"us_min\": %.1f, \"rounds\": %zu, \"ntail\": %d, \"eliminated\": %zu, "
               "\"front_max\": %zu, \"targets\": %zu, \"contribs\": %zu, \"inl_ints\": %zu}",
               first ? "" : ", ", p.name, t[t.size() / 2], t[0], sp.rounds.size(), sp.ntail, sp.nodes.size(), fmax,
               sp.tg.size() / 3, sp.tc.size() / 2, sp.inl.size());
        first = false;
    }
    printf("}}\n");
    return 0;
}
