// knn_unit -- C++ unit tests.
//   knn_unit cpu   : host-only checks (xyz round trip, normalisation, kd-tree and CPU grid
//                    vs brute force, checker self-test)
//   knn_unit gpu   : device checks through the C API (tile vs exact path vs oracle for
//                    several K / N / distributions, permutation bijection, stored-space
//                    semantics, set_k, save/load, N <= K edge cases)
// Exit code = number of failed checks.
// -DKN_UNIT_CPU_ONLY builds the host checks alone (no HIP / C API): the sanitizer build
// (`python -m cuda_knearests_amd._build --asan` -> bin/knn_unit_asan).
#ifndef KN_UNIT_CPU_ONLY
#include <hip/hip_runtime.h>
#endif

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#ifndef KN_UNIT_CPU_ONLY
#include "knearests.h"
#endif
#include "../host/host.hpp"

static int g_fail = 0, g_pass = 0;
#define EXPECT(cond, ...)                                          \
    do {                                                           \
        if (cond) { ++g_pass; }                                    \
        else { ++g_fail; fprintf(stderr, "FAIL %s:%d: ", __FILE__, __LINE__); fprintf(stderr, __VA_ARGS__); fprintf(stderr, "\n"); } \
    } while (0)

static void cpu_tests() {
    // xyz round trip + normalisation
    std::vector<float> a;
    knh::gen_uniform(1000, 7, a);
    std::string err;
    EXPECT(knh::write_xyz("/tmp/knn_unit.xyz", a.data(), 1000, &err), "write_xyz: %s", err.c_str());
    std::vector<float> b;
    EXPECT(knh::read_xyz("/tmp/knn_unit.xyz", b, false, &err), "read_xyz: %s", err.c_str());
    EXPECT(a == b, "xyz round trip differs");
    knh::normalize_1000(b);
    float lo = 1e30f, hi = -1e30f;
    for (float v : b) { lo = std::min(lo, v); hi = std::max(hi, v); }
    EXPECT(lo > 0.f && hi < 1000.f && hi > 990.f, "normalisation range [%g,%g]", lo, hi);
    // oracle vs brute force, several K and distributions (incl. duplicates)
    for (int dist = 0; dist < 3; ++dist) {
        std::vector<float> p;
        if (dist == 0) knh::gen_uniform(3000, 1, p);
        else if (dist == 1) knh::gen_clustered(3000, 2, p);
        else { knh::gen_uniform(1500, 3, p); p.insert(p.end(), p.begin(), p.end()); }  // exact duplicates
        const int n = (int)p.size() / 3;
        for (int k : {1, 8, 16, 50}) {
            std::vector<uint32_t> bi((size_t)n * k), ki((size_t)n * k), gi((size_t)n * k);
            std::vector<float> bd((size_t)n * k), kd((size_t)n * k), gd((size_t)n * k);
            knh::brute_knn_all(p.data(), n, k, bi.data(), bd.data(), 0);
            knh::kdtree_knn_all(p.data(), n, k, ki.data(), kd.data(), 0);
            const float inf[3] = {INFINITY, INFINITY, INFINITY}, ninf[3] = {-INFINITY, -INFINITY, -INFINITY};
            std::vector<uint32_t> unc;
            knh::grid_knn_cpu(p.data(), n, n, k, 0.f, ninf, inf, gi.data(), gd.data(), &unc, 0);
            EXPECT(ki == bi && kd == bd, "kdtree != brute (dist %d, k %d)", dist, k);
            EXPECT(gi == bi && gd == bd, "grid_cpu != brute (dist %d, k %d)", dist, k);
            EXPECT(unc.empty(), "grid_cpu uncertified %zu", unc.size());
            auto r = knh::check_knn(p.data(), n, n, k, gi.data(), bi.data(), bd.data());
            EXPECT(r.bad_rows == 0, "checker: %s", r.message.c_str());
        }
    }
    // checker must catch a wrong result
    {
        std::vector<float> p;
        knh::gen_uniform(500, 4, p);
        std::vector<uint32_t> bi(500 * 4);
        std::vector<float> bd(500 * 4);
        knh::brute_knn_all(p.data(), 500, 4, bi.data(), bd.data(), 0);
        auto bad = bi;
        std::swap(bad[0], bad[3]);
        EXPECT(knh::check_knn(p.data(), 500, 500, 4, bad.data(), bi.data(), bd.data()).bad_rows == 1, "checker missed a swap");
        bad = bi;
        bad[7] = bad[6];
        EXPECT(knh::check_knn(p.data(), 500, 500, 4, bad.data(), bi.data(), bd.data()).bad_rows == 1, "checker missed a dupe");
    }
    // tiny N (N <= K): slots beyond N-1 stay empty
    {
        std::vector<float> p = {0, 0, 0, 1, 0, 0, 0, 2, 0};
        std::vector<uint32_t> gi(3 * 5);
        std::vector<float> gd(3 * 5);
        const float inf[3] = {INFINITY, INFINITY, INFINITY}, ninf[3] = {-INFINITY, -INFINITY, -INFINITY};
        knh::grid_knn_cpu(p.data(), 3, 3, 5, 0.f, ninf, inf, gi.data(), gd.data(), nullptr, 0);
        EXPECT(gi[0] == 1 && gi[1] == 2 && gi[2] == 0xFFFFFFFFu, "tiny N row 0: %u %u %u", gi[0], gi[1], gi[2]);
    }
}

#ifndef KN_UNIT_CPU_ONLY
static bool run_case(const std::vector<float>& p, int k, int exact, const char* tag, float ppc = 0.f) {
    const int n = (int)p.size() / 3;
    kn_config cfg = kn_default_config();
    cfg.k = k;
    cfg.exact_only = exact;
    cfg.points_per_cell = ppc;
    kn_problem* kn = kn_prepare_ex(reinterpret_cast<const kn_float3*>(p.data()), n, &cfg);
    if (!kn) { EXPECT(false, "%s: prepare failed: %s", tag, kn_last_error()); return false; }
    EXPECT(kn_solve_ex(kn) == KN_OK, "%s: solve failed: %s", tag, kn_last_error());
    unsigned* knn = kn_get_knearests(kn);
    unsigned* perm = kn_get_permutation(kn);
    unsigned* orig = kn_get_neighbors(kn);
    kn_stats st;
    kn_get_stats(kn, &st);
    std::vector<uint32_t> nb((size_t)n * k);
    for (int i = 0; i < n; ++i)
        for (int j = 0; j < k; ++j) {
            const unsigned v = knn[(size_t)i * k + j];
            nb[(size_t)perm[i] * k + j] = v == 0xFFFFFFFFu ? v : perm[v];
        }
    EXPECT(std::equal(nb.begin(), nb.end(), orig), "%s: stored-space view != original-space result", tag);
    std::vector<unsigned> ps(perm, perm + n);
    std::sort(ps.begin(), ps.end());
    bool bij = true;
    for (int i = 0; i < n; ++i) bij = bij && ps[i] == (unsigned)i;
    EXPECT(bij, "%s: permutation not a bijection", tag);
    std::vector<uint32_t> oi((size_t)n * k);
    std::vector<float> od((size_t)n * k);
    knh::kdtree_knn_all(p.data(), n, k, oi.data(), od.data(), 0);
    auto r = knh::check_knn(p.data(), n, n, k, nb.data(), oi.data(), od.data());
    EXPECT(r.bad_rows == 0, "%s: %ld bad rows: %s", tag, r.bad_rows, r.message.c_str());
    fprintf(stderr, "  %-28s n=%-8d k=%-3d exact-path=%-7d build %.3f ms solve %.3f ms  %s\n", tag, n, k,
            st.fallback_queries, st.ms_build, st.ms_solve, r.bad_rows ? "BAD" : "ok");
    free(knn); free(perm); free(orig);
    kn_free(&kn);
    EXPECT(kn == nullptr, "kn_free must null the pointer");
    return r.bad_rows == 0;
}

static void gpu_tests() {
    int nd = 0;
    if (hipGetDeviceCount(&nd) != hipSuccess || nd == 0) { fprintf(stderr, "no HIP device: GPU tests skipped\n"); return; }
    std::vector<float> p;
    knh::gen_uniform(20000, 11, p);
    for (int k : {1, 8, 16, 32, 50, 64}) {
        run_case(p, k, 0, "uniform20K tile");
        run_case(p, k, 1, "uniform20K exact");
    }
    knh::gen_blue(30000, 5, p);
    run_case(p, 16, 0, "blue30K tile");
    knh::gen_clustered(30000, 6, p);
    run_case(p, 16, 0, "clustered30K tile");
    run_case(p, 16, 1, "clustered30K exact");
    knh::gen_uniform(1500, 9, p);
    p.insert(p.end(), p.begin(), p.end());
    run_case(p, 8, 0, "duplicates3K tile");
    for (int n : {1, 2, 5, 17, 100}) {
        knh::gen_uniform(n, 12 + n, p);
        run_case(p, 8, 0, "tinyN tile");
    }
    knh::gen_uniform(300000, 13, p);
    run_case(p, 16, 0, "uniform300K tile");
    // set_k + save/load
    {
        knh::gen_uniform(50000, 21, p);
        kn_config cfg = kn_default_config();
        cfg.k = 8;
        kn_problem* kn = kn_prepare_ex(reinterpret_cast<const kn_float3*>(p.data()), 50000, &cfg);
        EXPECT(kn && kn_solve_ex(kn) == KN_OK, "prepare/solve");
        EXPECT(kn_set_k(kn, 24) == KN_OK && kn_solve_ex(kn) == KN_OK, "set_k: %s", kn_last_error());
        unsigned* a = kn_get_neighbors(kn);
        EXPECT(kn_save(kn, "/tmp/knn_unit.kng") == KN_OK, "save: %s", kn_last_error());
        kn_free(&kn);
        cfg.k = 24;
        kn_problem* kl = kn_load("/tmp/knn_unit.kng", &cfg);
        EXPECT(kl && kn_solve_ex(kl) == KN_OK, "load/solve: %s", kn_last_error());
        unsigned* b = kl ? kn_get_neighbors(kl) : nullptr;
        EXPECT(a && b && std::equal(a, a + 50000 * 24, b), "save/load result differs");
        free(a); free(b);
        kn_free(&kl);
    }
}

#endif  // KN_UNIT_CPU_ONLY

int main(int argc, char** argv) {
    const std::string what = argc > 1 ? argv[1] : "all";
    if (what == "cpu" || what == "all") cpu_tests();
#ifndef KN_UNIT_CPU_ONLY
    if (what == "gpu" || what == "all") gpu_tests();
#endif
    fprintf(stderr, "knn_unit: %d passed, %d failed\n", g_pass, g_fail);
    return g_fail;
}
