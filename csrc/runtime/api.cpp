// api.cpp -- C API (knearests.h) on top of kn::Engine.
// Reference: knearests.cu:235-466 (kn_prepare / kn_solve / kn_free / getters / stats).
#include <cctype>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "engine.hpp"
#include "hostio.hpp"
#include "../host/host.hpp"
#include "knearests.h"

namespace {
thread_local std::string g_err;

kn::Engine* eng(kn_problem* kn) { return kn ? static_cast<kn::Engine*>(kn->impl) : nullptr; }

void sync_fields(kn_problem* kn) {
    kn::Engine* e = eng(kn);
    kn->allocated_points = e->n();
    kn->dimx = e->dims()[0];
    kn->dimy = e->dims()[1];
    kn->dimz = e->dims()[2];
    kn->num_cell_offsets = 0;
    kn->d_cell_offsets = nullptr;
    kn->d_cell_offset_dists = nullptr;
    kn->d_cell_max = nullptr;
    kn->d_counters = nullptr;
    kn->d_globcounter = nullptr;
    kn->k = e->k();
    kn->d_permutation = e->d_perm();
    kn->d_ptrs = e->d_cell_start();
    kn->d_stored_points4 = reinterpret_cast<float*>(e->d_sorted());
    kn->d_stored_points = reinterpret_cast<kn_float3*>(e->d_points3());
    kn->d_knearests = e->d_knn_stored_if_valid();
}

kn::EngineConfig to_engine(const kn_config* c) {
    kn::EngineConfig e;
    if (!c) return e;
    e.k = c->k > 0 ? c->k : KN_DEFAULT_K;
    e.points_per_cell = c->points_per_cell;
    for (int a = 0; a < 3; ++a) e.tile[a] = c->tile[a];
    e.halo = c->halo;
    e.deterministic = c->deterministic;
    e.device = c->device;
    e.verbose = c->verbose;
    e.use_tiles = c->exact_only ? 0 : 1;
    e.adaptive = c->fixed_grid ? 0 : 1;
    e.algo = c->algo;
    return e;
}
}  // namespace

// Log level from the environment, shared with the Python package (utils.get_logger):
// KN_LOG = DEBUG -> 2 (debug), INFO -> 1 (timings, as the reference's IF_VERBOSE), WARNING /
// ERROR -> 0; KN_VERBOSE=<int> overrides. `dflt` when neither is set.
static int env_verbosity(int dflt) {
    if (const char* v = std::getenv("KN_VERBOSE")) return std::atoi(v);
    if (const char* l = std::getenv("KN_LOG")) {
        std::string s(l);
        for (auto& ch : s) ch = (char)std::toupper((unsigned char)ch);
        if (s == "DEBUG") return 2;
        if (s == "INFO") return 1;
        if (s == "WARNING" || s == "WARN" || s == "ERROR" || s == "CRITICAL") return 0;
    }
    return dflt;
}

extern "C" {

void kn_set_last_error_internal(const char* msg) { g_err = msg ? msg : ""; }

kn_config kn_default_config(void) {
    kn_config c;
    std::memset(&c, 0, sizeof(c));
    c.k = KN_DEFAULT_K;
    c.deterministic = 1;
    c.verbose = env_verbosity(0);
    return c;
}

const char* kn_last_error(void) { return g_err.c_str(); }

kn_problem* kn_prepare_ex(const kn_float3* points, int numpoints, const kn_config* cfg) {
    kn_config c = cfg ? *cfg : kn_default_config();
    auto* e = new kn::Engine(to_engine(&c));
    if (e->prepare_host(reinterpret_cast<const float*>(points), numpoints) != KN_OK) {
        g_err = e->error();
        delete e;
        return nullptr;
    }
    auto* kn = static_cast<kn_problem*>(std::calloc(1, sizeof(kn_problem)));
    kn->impl = e;
    sync_fields(kn);
    return kn;
}

kn_problem* kn_prepare(const kn_float3* points, int numpoints) {
    kn_config c = kn_default_config();
    c.verbose = env_verbosity(1);  // reference prints its timings (IF_VERBOSE, params.h:6)
    return kn_prepare_ex(points, numpoints, &c);
}

kn_status kn_solve_ex(kn_problem* kn) {
    kn::Engine* e = eng(kn);
    if (!e) { g_err = "null problem"; return KN_ERR_INVALID_ARGUMENT; }
    kn_status s = e->solve();
    // reference semantics: d_knearests holds the stored-space result after kn_solve
    // (knearests.cu:329-364); the engine solves in original space, one remap kernel converts
    // (N*K ids + N inverse permutation). Non-fatal: if that buffer does not fit, the solve still
    // succeeded, d_knearests stays NULL and the getters convert on demand.
    if (s == KN_OK && !e->d_knn_stored()) g_err = "kn_solve: stored-space d_knearests not materialised: " + e->error();
    if (s != KN_OK) g_err = e->error();
    sync_fields(kn);
    return s;
}

void kn_solve(kn_problem* kn) { (void)kn_solve_ex(kn); }

kn_status kn_solve_range(kn_problem* kn, int first, int count, unsigned int* out_ids, float* out_d2) {
    kn::Engine* e = eng(kn);
    if (!e) { g_err = "null problem"; return KN_ERR_INVALID_ARGUMENT; }
    if (count < 0 || first < 0 || (long long)first + count > (long long)e->n()) {
        g_err = "query range outside [0, N)";
        return KN_ERR_INVALID_ARGUMENT;
    }
    if (count > 0 && !out_ids) { g_err = "null output"; return KN_ERR_INVALID_ARGUMENT; }
    if (count == 0) return KN_OK;
    const size_t nk = (size_t)count * e->k();
    // the batch buffers are the engine's grow-only scratch: a sequence of batches allocates once
    // (no synchronising hipMalloc / hipFree per batch)
    const size_t bi = (nk * sizeof(unsigned) + 255) & ~(size_t)255;
    char* scr = static_cast<char*>(e->scratch(bi + (out_d2 ? nk * sizeof(float) : 0)));
    unsigned* d_idx = scr ? reinterpret_cast<unsigned*>(scr) : nullptr;
    float* d_d2 = (scr && out_d2) ? reinterpret_cast<float*>(scr + bi) : nullptr;
    kn_status s = KN_OK;
    if (!scr) {
        g_err = "hipMalloc(query range)";
        s = KN_ERR_DEVICE;
    }
    if (s == KN_OK && (s = e->solve_range(first, count, d_idx, d_d2)) != KN_OK) g_err = e->error();
    if (s == KN_OK && (hipMemcpy(out_ids, d_idx, nk * sizeof(unsigned), hipMemcpyDeviceToHost) != hipSuccess ||
                       (out_d2 && hipMemcpy(out_d2, d_d2, nk * sizeof(float), hipMemcpyDeviceToHost) != hipSuccess))) {
        g_err = "D2H (query range)";
        s = KN_ERR_DEVICE;
    }
    return s;
}

kn_status kn_set_k(kn_problem* kn, int k) {
    kn::Engine* e = eng(kn);
    if (!e) { g_err = "null problem"; return KN_ERR_INVALID_ARGUMENT; }
    kn_status s = e->set_k(k);
    if (s != KN_OK) g_err = e->error();
    sync_fields(kn);  // d_knearests is stale until the next kn_solve
    return s;
}

void kn_free(kn_problem** kn) {
    if (!kn || !*kn) return;
    delete eng(*kn);
    std::free(*kn);
    *kn = nullptr;  // reference knearests.cu:407
}

kn_float3* kn_get_points(kn_problem* kn) {
    kn::Engine* e = eng(kn);
    if (!e) return nullptr;
    float* p = e->get_points_sorted();
    if (!p) g_err = e->error();
    return reinterpret_cast<kn_float3*>(p);
}

unsigned int* kn_get_permutation(kn_problem* kn) {
    kn::Engine* e = eng(kn);
    if (!e) return nullptr;
    unsigned* p = e->get_permutation();
    if (!p) g_err = e->error();
    return p;
}

unsigned int* kn_get_knearests(kn_problem* kn) {
    kn::Engine* e = eng(kn);
    if (!e) return nullptr;
    unsigned* p = e->get_knearests_stored();
    if (!p) g_err = e->error();
    kn->d_knearests = e->d_knn_stored_if_valid();
    return p;
}

float* kn_get_distances(kn_problem* kn) {
    kn::Engine* e = eng(kn);
    if (!e) return nullptr;
    float* p = e->get_distances_stored();
    if (!p) g_err = e->error();
    return p;
}

unsigned int* kn_get_neighbors(kn_problem* kn) {
    kn::Engine* e = eng(kn);
    if (!e) return nullptr;
    unsigned* p = e->get_neighbors_original();
    if (!p) g_err = e->error();
    return p;
}

kn_status kn_get_stats(kn_problem* kn, kn_stats* out) {
    kn::Engine* e = eng(kn);
    if (!e || !out) { g_err = "null argument"; return KN_ERR_INVALID_ARGUMENT; }
    kn_status s = e->stats(out, nullptr);
    if (s != KN_OK) g_err = e->error();
    return s;
}

void kn_print_stats(kn_problem* kn) {
    kn::Engine* e = eng(kn);
    if (!e) return;
    kn_stats st;
    std::vector<int> hist;
    if (e->stats(&st, &hist) != KN_OK) { fprintf(stderr, "kn_print_stats: %s\n", e->error().c_str()); return; }
    fprintf(stderr, "grid %dx%dx%d (%d cells), %d points, K=%d\n", st.dims[0], st.dims[1], st.dims[2],
            st.num_cells, st.num_points, st.k);
    fprintf(stderr, "points per cell: min %d, max %d, avg %.3f, empty cells %d\n", st.min_cell,
            st.max_cell, st.avg_cell, st.empty_cells);
    for (size_t i = 0; i < hist.size(); ++i)
        if (hist[i]) fprintf(stderr, "  [%2zu%s] %d\n", i, i + 1 == hist.size() ? "+" : " ", hist[i]);
    fprintf(stderr, "exact-path queries %d, uncertified %d, build %.3f ms, solve %.3f ms\n",
            st.fallback_queries, st.uncertified_queries, st.ms_build, st.ms_solve);
}

kn_status kn_save(kn_problem* kn, const char* path) {
    kn::Engine* e = eng(kn);
    if (!e || !path) { g_err = "null argument"; return KN_ERR_INVALID_ARGUMENT; }
    kn_status s = e->save(path);
    if (s != KN_OK) g_err = e->error();
    return s;
}

kn_problem* kn_load(const char* path, const kn_config* cfg) {
    kn_config c = cfg ? *cfg : kn_default_config();
    kn::EngineConfig ec = to_engine(&c);
    if (!cfg) ec.k = 0;  // take K from the file
    std::string err;
    kn::Engine* e = kn::Engine::load(path, ec, &err);
    if (!e) { g_err = err; return nullptr; }
    auto* kn = static_cast<kn_problem*>(std::calloc(1, sizeof(kn_problem)));
    kn->impl = e;
    sync_fields(kn);
    return kn;
}

void kn_release_cached_memory(void) { kn::arena_release_all(); }

size_t kn_struct_size(int which) {
    switch (which) {
        case 0: return sizeof(kn_config);
        case 1: return sizeof(kn_problem);
        case 2: return sizeof(kn_stats);
        case 3: return sizeof(kn_multi_options);
        case 4: return sizeof(kn_multi_stats);
        default: return 0;
    }
}

kn_float3* kn_read_xyz(const char* path, int* n, int normalize) {
    std::vector<float> xyz;
    std::string err;
    if (!path || !knh::read_xyz(path, xyz, normalize != 0, &err)) { g_err = err; if (n) *n = 0; return nullptr; }
    const size_t cnt = xyz.size() / 3;
    float* out = static_cast<float*>(std::malloc(std::max<size_t>(1, xyz.size()) * sizeof(float)));
    std::memcpy(out, xyz.data(), xyz.size() * sizeof(float));
    if (n) *n = (int)cnt;
    return reinterpret_cast<kn_float3*>(out);
}

kn_status kn_write_xyz(const char* path, const kn_float3* pts, int n) {
    std::string err;
    if (!knh::write_xyz(path, reinterpret_cast<const float*>(pts), n, &err)) { g_err = err; return KN_ERR_IO; }
    return KN_OK;
}

}  // extern "C"
