// engine.cpp -- single-GPU host runtime. See engine.hpp.
// Replaces the reference's kn_prepare / kn_firstbuild / kn_solve / kn_free (knearests.cu:152-438):
// one arena instead of per-buffer gpuMalloc* (:205-335), deterministic scan instead of the
// atomic `reserve` bump allocator, hipGraph replay of the whole build+solve step.
#include "engine.hpp"

#include <chrono>

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <string>
#include <cstring>
#include <fstream>

#include "hostio.hpp"

namespace kn {

namespace {
constexpr size_t kAlign = 256;
size_t align_up(size_t v) { return (v + kAlign - 1) & ~(kAlign - 1); }
template <class T>
T* carve(char*& p, size_t count) {
    T* r = reinterpret_cast<T*>(p);
    p += align_up(count * sizeof(T));
    return r;
}
}  // namespace

Engine::Engine(const EngineConfig& cfg) : cfg_(cfg) {
    if (cfg_.k <= 0) cfg_.k = KN_DEFAULT_K;
}

Engine::~Engine() {
    const auto t0 = std::chrono::steady_clock::now();
    release();
    if (std::getenv("KN_PREP_TIMING"))
        fprintf(stderr, "kn_free: release %.3f ms\n",
                std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count());
}

void Engine::release() {
    if (graph_) { (void)hipGraphExecDestroy(graph_); graph_ = nullptr; }
    drop_pipeline();
    // the arena goes back to the process-wide cache (hostio.hpp): the next kn_prepare of a similar
    // size skips hipMalloc
    if (stream_) (void)hipStreamSynchronize(stream_);
    if (arena_) { arena_release(cfg_.device, arena_, arena_bytes_); arena_ = nullptr; arena_bytes_ = 0; }
    if (out_idx_) { dfree(out_idx_); out_idx_ = nullptr; }
    if (out_dist_) { dfree(out_dist_); out_dist_ = nullptr; }
    if (inv_perm_) { dfree(inv_perm_); inv_perm_ = nullptr; }
    if (knn_stored_) { dfree(knn_stored_); knn_stored_ = nullptr; }
    if (points3_) { dfree(points3_); points3_ = nullptr; }
    if (tree_ws_) { dfree(tree_ws_); tree_ws_ = nullptr; }
    if (tree_nodes_) { dfree(tree_nodes_); tree_nodes_ = nullptr; }
    if (scratch_) { dfree(scratch_); scratch_ = nullptr; scratch_bytes_ = 0; }
    // the (idle) stream and its events go back to the pool; the reference leaks its events (D6)
    if (stream_) {
        (void)hipStreamSynchronize(stream_);
        StreamSet ss;
        ss.stream = stream_;
        for (int i = 0; i < 4; ++i) ss.ev[i] = ev_[i];
        streamset_release(cfg_.device, ss);
    }
    stream_ = nullptr;
    for (auto& e : ev_) e = nullptr;
}

hipError_t Engine::dmalloc(void** p, size_t bytes) {
    bytes = std::max<size_t>(bytes, 1);
    size_t got = 0;
    if (void* c = arena_acquire(cfg_.device, bytes, &got)) {
        *p = c;
        dsize_[c] = got;
        return hipSuccess;
    }
    hipError_t e = device_malloc(p, bytes);
    if (e == hipSuccess) dsize_[*p] = bytes;
    return e;
}

void Engine::dfree(void* p) {
    if (!p) return;
    // a parked block may go to another engine (another stream) at once: this engine's pending
    // work on it must have drained
    if (stream_) (void)hipStreamSynchronize(stream_);
    auto it = dsize_.find(p);
    if (it == dsize_.end()) { (void)hipFree(p); return; }
    arena_release(cfg_.device, p, it->second);
    dsize_.erase(it);
}

void* Engine::scratch(size_t bytes) {
    if (bytes <= scratch_bytes_) return scratch_;
    if (scratch_) { dfree(scratch_); scratch_ = nullptr; scratch_bytes_ = 0; }
    void* p = nullptr;
    if (dmalloc(&p, bytes) != hipSuccess) return nullptr;
    scratch_ = p;
    scratch_bytes_ = bytes;
    ++scratch_allocs_;
    return p;
}

kn_status Engine::fail(kn_status s, const std::string& msg) {
    err_ = msg;
    if (cfg_.verbose) fprintf(stderr, "[knearests] error: %s\n", msg.c_str());
    return s;
}

kn_status Engine::check(hipError_t e, const char* what) {
    if (e == hipSuccess) return KN_OK;
    return fail(e == hipErrorOutOfMemory ? KN_ERR_OUT_OF_MEMORY : KN_ERR_DEVICE,
                std::string(what) + ": " + hipGetErrorString(e));
}

kn_status Engine::allocate(int n, const int* dims_override, bool refined, int xsub_override) {
    if (n < 0) return fail(KN_ERR_INVALID_ARGUMENT, "negative point count");
    if (cfg_.k < 1 || cfg_.k > KN_MAX_K) return fail(KN_ERR_INVALID_ARGUMENT, "k out of range [1,128]");
    kn_status st;
    if ((st = check(hipSetDevice(cfg_.device), "hipSetDevice")) != KN_OK) return st;
    const auto ta0 = std::chrono::steady_clock::now();
    if (!stream_) {
        // from the process-wide pool (hostio.hpp): stream + event creation cost 2-8 ms per engine
        StreamSet ss;
        if ((st = check(streamset_acquire(cfg_.device, &ss), "hipStreamCreate")) != KN_OK) return st;
        stream_ = ss.stream;
        for (int i = 0; i < 4; ++i) ev_[i] = ss.ev[i];
    }
    ap_ = auto_params(n, cfg_.k, cfg_.points_per_cell, cfg_.tile, cfg_.halo, nullptr);
    if (dims_override && refined) {
        // occupancy refinement: finer isotropic cells (xsub 1), same tile / halo / LDS capacity
        // (occupied cells keep about the target density)
        for (int a = 0; a < 3; ++a) ap_.dims[a] = std::max(1, dims_override[a]);
        ap_.tile[0] = std::max(1, ap_.tile[0] / std::max(1, ap_.xsub));
        ap_.xsub = 1;
        ap_.lds_bytes = query_lds_bytes(ap_.tile, ap_.halo, ap_.lds_capacity, 1);
    } else if (dims_override) {
        // a given grid (kn_load): its x subdivision comes with it (default: none)
        const int xs = std::max(1, xsub_override);
        ap_.tile[0] = std::max(1, ap_.tile[0] / std::max(1, ap_.xsub)) * xs;
        ap_.xsub = xs;
        for (int a = 0; a < 3; ++a) ap_.dims[a] = std::max(1, dims_override[a]);
        const double ppc = (double)std::max(1, n) / ((double)ap_.dims[0] * ap_.dims[1] * ap_.dims[2]);
        ap_.lds_capacity = lds_capacity_for(staged_points(ap_, ppc));
        ap_.lds_bytes = query_lds_bytes(ap_.tile, ap_.halo, ap_.lds_capacity, ap_.xsub);
    }
    const int C = ap_.dims[0] * ap_.dims[1] * ap_.dims[2];
    const size_t nb = scan_block_count(C) + 1;
    size_t bytes = 0;
    bytes += align_up((size_t)n * 3 * sizeof(float));
    bytes += align_up(kBBoxWords * sizeof(unsigned));
    bytes += align_up(sizeof(GridGeom));
    bytes += 3 * align_up((size_t)(C + 1) * sizeof(int));
    bytes += align_up(nb * sizeof(int));
    bytes += align_up((size_t)n * sizeof(float4));  // bin_tmp (cell_rank aliases it)
    bytes += align_up((size_t)n * sizeof(float4));
    bytes += 2 * align_up((size_t)n * sizeof(unsigned));
    bytes += align_up(kNumCounters * sizeof(unsigned));
    bytes += align_up(sizeof(unsigned long long));
    if (graph_) { (void)hipGraphExecDestroy(graph_); graph_ = nullptr; }
    drop_pipeline();
    if (bytes > arena_bytes_) {
        if (arena_) {
            if (stream_) (void)hipStreamSynchronize(stream_);
            arena_release(cfg_.device, arena_, arena_bytes_);
        }
        arena_ = nullptr;
        arena_bytes_ = 0;
        size_t got = 0;
        if (void* c = arena_acquire(cfg_.device, bytes, &got)) {
            arena_ = static_cast<char*>(c);
            arena_bytes_ = got;
        } else {
            if ((st = check(device_malloc(reinterpret_cast<void**>(&arena_), bytes), "hipMalloc(arena)")) != KN_OK) return st;
            arena_bytes_ = bytes;
        }
    }
    arena_used_ = bytes;
    if (std::getenv("KN_PREP_TIMING"))
        fprintf(stderr, "allocate: stream/events + arena %.3f ms (arena %zu B)\n",
                std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - ta0).count(), arena_bytes_);
    char* p = arena_;
    points_ = carve<float>(p, (size_t)n * 3);
    bbox_ = carve<unsigned>(p, kBBoxWords);
    geom_ = carve<GridGeom>(p, 1);
    cell_count_ = carve<int>(p, C + 1);
    cell_scan_ = carve<int>(p, C + 1);
    cell_start_ = carve<int>(p, C + 1);
    block_sums_ = carve<int>(p, nb);
    bin_tmp_ = carve<float4>(p, n);
    cell_rank_ = reinterpret_cast<int2*>(bin_tmp_);
    sorted_ = carve<float4>(p, n);
    perm_ = carve<unsigned>(p, n);
    fallback_ = carve<unsigned>(p, n);
    counters_ = carve<unsigned>(p, kNumCounters);
    occ_ = carve<unsigned long long>(p, 1);
    live_ = 0;
    graph_set_ = -1;
    set_[0] = members();
    // outputs
    for (void** q : {(void**)&out_idx_, (void**)&out_dist_, (void**)&inv_perm_, (void**)&knn_stored_,
                     (void**)&points3_})
        if (*q) { dfree(*q); *q = nullptr; }
    // the N x K outputs are allocated on the first whole solve (ensure_outputs): a caller that
    // only solves query ranges (solve_range, kn_solve_range) never holds them
    const size_t nk = std::max<size_t>(1, (size_t)n * cfg_.k);
    n_ = n;
    C_ = C;
    built_ = solved_ = stored_valid_ = points3_valid_ = false;
    if (cfg_.verbose)
        fprintf(stderr, "[knearests] N=%d K=%d grid %dx%dx%d tile %dx%dx%d halo %d lds %zu B, GPU memory %.1f MB\n",
                n, cfg_.k, ap_.dims[0], ap_.dims[1], ap_.dims[2], ap_.tile[0], ap_.tile[1],
                ap_.tile[2], ap_.halo, ap_.lds_bytes,
                (bytes + nk * (sizeof(unsigned) + (cfg_.with_distances ? 4 : 0))) / 1048576.0);
    return KN_OK;
}

BuildBuffers Engine::build_buffers() const {
    BuildBuffers b{};
    b.points = points_;
    b.n = n_;
    for (int a = 0; a < 3; ++a) b.dims[a] = ap_.dims[a];
    b.bbox_words = bbox_;
    b.geom = geom_;
    b.cell_count = cell_count_;
    b.cell_scan = cell_scan_;
    b.block_sums = block_sums_;
    b.cell_start = cell_start_;
    b.cell_rank = cell_rank_;
    b.bin_tmp = bin_tmp_;
    b.sorted = sorted_;
    b.perm = perm_;
    b.deterministic = cfg_.deterministic;
    b.use_box = 0;
    return b;
}

QueryBuffers Engine::query_buffers() const {
    QueryBuffers q{};
    q.sorted = sorted_;
    q.cell_start = cell_start_;
    q.perm = perm_;
    q.geom = geom_;
    q.n = n_;
    for (int a = 0; a < 3; ++a) q.dims[a] = ap_.dims[a];
    q.k = cfg_.k;
    q.n_queries = n_;
    q.id_map = nullptr;
    for (int a = 0; a < 3; ++a) { q.complete.lo[a] = -INFINITY; q.complete.hi[a] = INFINITY; }
    q.out_idx = out_idx_;
    q.out_dist = out_dist_;
    if (out_ref_slot_ >= 0) {  // a batch step: output pointers from the table (stream_batch)
        q.out_idx_ref = reinterpret_cast<unsigned* const*>(tab_ + kBatchMax + out_ref_slot_);
        q.out_dist_ref = reinterpret_cast<float* const*>(tab_ + 2 * kBatchMax + out_ref_slot_);
    }
    if (out_ovr_set_ >= 0) {  // an eager batch step: the caller's buffers
        q.out_idx = bout_idx_[out_ovr_set_];
        q.out_dist = bout_dist_[out_ovr_set_];
    }
    q.fallback_list = fallback_;
    q.counters = counters_;
    for (int a = 0; a < 3; ++a) q.tile[a] = ap_.tile[a];
    q.halo = ap_.halo;
    q.xsub = ap_.xsub;
    q.lds_capacity = ap_.lds_capacity;
    q.use_tiles = cfg_.use_tiles;
    // fallback grid from the last observed fallback count: 32 workgroups when it was (nearly)
    // empty -- a launch beside the running queries whose workgroups all find nothing to do --,
    // 256 when it was short, the default (KN_EXACT_GRID) otherwise
    q.exact_grid = last_fallback_ < 128u ? 32 : last_fallback_ < 4096u ? 256 : 0;
    // many cooperative re-rank finishes last time (exactly equal distances): the wide window
    if ((unsigned long long)last_coop_ * 64 > (unsigned long long)n_) q.flags |= kQueryFlagWide;
    return q;
}

// fused_step: build + grid query in one stream-ordered step (the captured graph): the build's
// first binning kernel zeroes the query counters, so the step has no memset node
kn_status Engine::build_async(bool fused_step, bool serial) {
    BuildBuffers b = build_buffers();
    b.serial = serial ? 1 : 0;
    if (fused_step && !use_tree_) {
        b.zero_words = counters_;
        b.n_zero_words = kNumCounters;
    }
    return check(launch_build(b, stream_), "build");
}
kn_status Engine::query_async(bool fused_step) {
    if (use_tree_) return tree_query();
    QueryBuffers q = query_buffers();
    q.counters_zeroed = fused_step ? 1 : 0;
    return check(launch_query(q, stream_), "query");
}

// Tree buffers for the current grid: workspace (sized by n and the grid dims) and the node
// buffer (P = pow2 >= n leaf slots, any leaf count fits). Allocated outside any graph capture.
kn_status Engine::ensure_tree() {
    kn_status st;
    const size_t need = tree_workspace_bytes(n_, ap_.dims);
    if (tree_ws_bytes_ < need) {
        if (tree_ws_) dfree(tree_ws_);
        tree_ws_ = nullptr;
        tree_ws_bytes_ = 0;
        if ((st = check(dmalloc(&tree_ws_, need), "hipMalloc(tree)")) != KN_OK) return st;
        tree_ws_bytes_ = need;
    }
    const size_t nb = tree_node_bytes(n_);
    if (tree_nodes_bytes_ < nb) {
        if (tree_nodes_) dfree(tree_nodes_);
        tree_nodes_ = nullptr;
        tree_nodes_bytes_ = 0;
        if ((st = check(dmalloc(&tree_nodes_, nb), "hipMalloc(tree nodes)")) != KN_OK) return st;
        tree_nodes_bytes_ = nb;
    }
    set_[live_].tree_ws = tree_ws_;
    set_[live_].tree_nodes = tree_nodes_;
    return KN_OK;
}

// Stream-ordered, no host synchronisation (the leaf count stays on the device): capturable.
kn_status Engine::tree_query() {
    kn_status st;
    if ((st = tree_build_async()) != KN_OK) return st;
    return tree_query_async();
}

kn_status Engine::tree_build_async() {
    kn_status st;
    if ((st = ensure_tree()) != KN_OK) return st;
    TreeView t = tree_view(tree_ws_, n_, ap_.dims);
    tree_attach_nodes(t, tree_nodes_);
    if ((st = check(launch_tree_leaves(sorted_, cell_start_, geom_, t, stream_), "tree leaves")) != KN_OK) return st;
    return check(launch_tree_nodes(t, stream_), "tree nodes");
}

kn_status Engine::tree_query_async() {
    TreeView t = tree_view(tree_ws_, n_, ap_.dims);
    tree_attach_nodes(t, tree_nodes_);
    TreeQuery q{};
    q.k = cfg_.k;
    q.n_queries = n_;
    q.out_idx = out_idx_;
    q.out_dist = out_dist_;
    if (out_ref_slot_ >= 0) {
        q.out_idx_ref = reinterpret_cast<unsigned* const*>(tab_ + kBatchMax + out_ref_slot_);
        q.out_dist_ref = reinterpret_cast<float* const*>(tab_ + 2 * kBatchMax + out_ref_slot_);
    }
    if (out_ovr_set_ >= 0) {
        q.out_idx = bout_idx_[out_ovr_set_];
        q.out_dist = bout_dist_[out_ovr_set_];
    }
    q.counters = counters_;
    return check(launch_tree_query(t, q, stream_), "tree query");
}

int Engine::tree_leaves() {
    if (!use_tree_ || !tree_ws_ || !solved_) return 0;
    TreeView t = tree_view(tree_ws_, n_, ap_.dims);
    unsigned L = 0;
    return tree_leaf_count(t, &L, stream_) == hipSuccess ? (int)L : -1;
}

kn_status Engine::occupancy(double* w) {
    unsigned long long s = 0;
    kn_status st;
    if ((st = check(launch_cell_occupancy(cell_start_, C_, occ_, stream_), "occupancy")) != KN_OK) return st;
    if ((st = check(hipMemcpyAsync(&s, occ_, sizeof(s), hipMemcpyDeviceToHost, stream_), "D2H occupancy")) != KN_OK)
        return st;
    if ((st = check(hipStreamSynchronize(stream_), "occupancy sync")) != KN_OK) return st;
    *w = n_ > 0 ? (double)s / n_ : 0.0;
    return KN_OK;
}

// Upload + build; with cfg_.adaptive, re-bin with finer cells while the mean occupancy of a
// point's cell is far above a Poisson grid's (at most 3 refinements, cell_start <= 64 B/point).
kn_status Engine::prepare_from(const float* src, int n, hipMemcpyKind kind) {
    kn_status st;
    if (!src && n > 0) return fail(KN_ERR_INVALID_ARGUMENT, "null points");
    using clk = std::chrono::steady_clock;
    const auto t0 = clk::now();
    if ((st = allocate(n)) != KN_OK) return st;
    const auto t1 = clk::now();
    bool refined = false;
    for (int round = 0;; ++round) {
        // host points: through the pinned staging ring (hostio.hpp), device points: D2D
        const hipError_t ce = kind == hipMemcpyHostToDevice
                                  ? copy_h2d_staged(points_, src, (size_t)n * 12, stream_)
                                  : hipMemcpyAsync(points_, src, (size_t)n * 12, kind, stream_);
        if (n > 0 && (st = check(ce, "copy points")) != KN_OK) return st;
        const auto tc = clk::now();
        (void)hipEventRecord(ev_[0], stream_);
        points3_valid_ = false;
        // adaptive: probe grids are binned without the in-cell order (see launch_cell_sort)
        BuildBuffers b = build_buffers();
        b.serial = 1;
        if (cfg_.adaptive) b.deterministic = 0;
        if ((st = check(launch_build(b, stream_), "build")) != KN_OK) return st;
        (void)hipEventRecord(ev_[1], stream_);
        if ((st = check(hipEventSynchronize(ev_[1]), "build sync")) != KN_OK) return st;
        (void)hipEventElapsedTime(&ms_build_, ev_[0], ev_[1]);
        if (std::getenv("KN_PREP_TIMING")) {
            auto ms = [](clk::duration d) { return std::chrono::duration<double, std::milli>(d).count(); };
            fprintf(stderr, "prepare round %d: copy enqueue %.3f ms, build + sync %.3f ms (device build %.3f ms)\n", round,
                    ms(tc - t1), ms(clk::now() - tc), ms_build_);
        }
        if (!cfg_.adaptive || n == 0) break;
        double w = 0.0;
        int nd[3];
        if (round < 3 && (st = occupancy(&w)) != KN_OK) return st;
        if (round == 3 || !refine_dims(ap_.dims, w, cfg_.k, cfg_.points_per_cell, n, nd, ap_.xsub)) {
            if (cfg_.deterministic &&
                (st = check(launch_cell_sort(cell_start_, geom_, n, sorted_, perm_, bin_tmp_, stream_), "cell sort")) != KN_OK)
                return st;
            break;
        }
        if (cfg_.verbose)
            fprintf(stderr, "kn: cell occupancy %.1f -> grid %dx%dx%d\n", w, nd[0], nd[1], nd[2]);
        if ((st = allocate(n, nd, true)) != KN_OK) return st;
        refined = true;
    }
    // A grid that had to be refined serves a cloud whose density varies too much for one cell
    // size (900K clustered, K=16: grid query 7.5 ms, tree 1.6 ms + 0.27 ms build; surfaces
    // 1.27 vs 0.96 + 0.27; profiles/diag_r2_tree.jsonl): the tree path takes it.
    refined_ = refined;
    use_tree_ = cfg_.use_tiles && (cfg_.algo == 2 || (cfg_.algo == 0 && refined)) && tree_supports(ap_.dims);
    if (graph_) { (void)hipGraphExecDestroy(graph_); graph_ = nullptr; }
    drop_pipeline();  // grid or tree step of the new plan
    if (cfg_.verbose) fprintf(stderr, "kn_firstbuild: %.3f msec\n", ms_build_);
    if (cfg_.verbose > 1 || std::getenv("KN_PREP_TIMING")) {
        const auto t2 = clk::now();
        auto ms = [](clk::duration d) { return std::chrono::duration<double, std::milli>(d).count(); };
        fprintf(stderr, "kn_prepare host phases: allocate %.3f ms, upload + build + plan %.3f ms\n", ms(t1 - t0),
                ms(t2 - t1));
    }
    built_ = true;
    return KN_OK;
}

kn_status Engine::prepare_host(const float* pts, int n) { return prepare_from(pts, n, hipMemcpyHostToDevice); }

kn_status Engine::prepare_device(const float* d_pts, int n) { return prepare_from(d_pts, n, hipMemcpyDeviceToDevice); }

kn_status Engine::upload_device(const float* d_pts, int n) {
    kn_status st;
    if (!arena_ || n != n_) {
        if ((st = allocate(n)) != KN_OK) return st;
    }
    // the primed pipelined build (if any) reads the other set's input: let it finish, it is stale
    if ((st = check(pipe_.unprime(), "pipeline")) != KN_OK) return st;
    other_stale_ = true;
    stream_mode_ = false;
    if (n > 0 && (st = check(hipMemcpyAsync(points_, d_pts, (size_t)n * 12, hipMemcpyDeviceToDevice, stream_),
                             "D2D points")) != KN_OK)
        return st;
    built_ = true;  // the next launch_graph() (or solve after a build) owns the grid
    points3_valid_ = stored_valid_ = false;
    return KN_OK;
}

kn_status Engine::ensure_outputs() {
    const size_t nk = std::max<size_t>(1, (size_t)n_ * cfg_.k);
    kn_status st;
    if (!out_idx_ && (st = check(dmalloc(&out_idx_, nk * sizeof(unsigned)), "hipMalloc(knn)")) != KN_OK) return st;
    if (cfg_.with_distances && !out_dist_ &&
        (st = check(dmalloc(&out_dist_, nk * sizeof(float)), "hipMalloc(dist)")) != KN_OK)
        return st;
    set_[live_].out_idx = out_idx_;
    set_[live_].out_dist = out_dist_;
    if (use_tree_ && (st = ensure_tree()) != KN_OK) return st;
    return KN_OK;
}

// Queries of the original indices [first, first + count) only, rows written to caller device
// buffers (count x K ids in original space, optional distances). The whole-solve outputs are
// never allocated, so a cloud whose N x K result does not fit next to the grid is solved in
// batches. Grid kernels (also for clouds the tree path serves).
kn_status Engine::solve_range(int first, int count, unsigned* d_idx, float* d_dist) {
    if (!built_) return fail(KN_ERR_STATE, "solve_range() before prepare()");
    if (first < 0 || count < 0 || (long long)first + count > (long long)n_)
        return fail(KN_ERR_INVALID_ARGUMENT, "query range outside [0, N)");
    if (count > 0 && !d_idx) return fail(KN_ERR_INVALID_ARGUMENT, "null output buffer");
    if (count == 0) return KN_OK;
    QueryBuffers q = query_buffers();
    q.q_lo = first;
    q.n_queries = first + count;
    q.out_idx = d_idx;
    q.out_dist = d_dist;
    q.exact_grid = 0;
    kn_status st;
    if ((st = check(launch_query(q, stream_), "query range")) != KN_OK) return st;
    return check(hipStreamSynchronize(stream_), "query range sync");
}

kn_status Engine::solve() {
    if (!built_) return fail(KN_ERR_STATE, "solve() before prepare()");
    kn_status st;
    if ((st = ensure_outputs()) != KN_OK) return st;
    (void)hipEventRecord(ev_[2], stream_);
    if ((st = query_async()) != KN_OK) return st;
    (void)hipEventRecord(ev_[3], stream_);
    if ((st = check(hipEventSynchronize(ev_[3]), "solve sync")) != KN_OK) return st;
    (void)hipEventElapsedTime(&ms_solve_, ev_[2], ev_[3]);
    // the stream is idle: the counters tell the next launches how long the fallback list runs
    // and how many queries needed the cooperative re-rank
    unsigned cw[4] = {~0u, 0, 0, 0};
    if (hipMemcpy(cw, counters_, sizeof(cw), hipMemcpyDeviceToHost) != hipSuccess) cw[0] = ~0u;
    last_fallback_ = cw[0];
    if (!use_tree_) last_coop_ = cw[3];
    if (cfg_.verbose) {
        unsigned c[kNumCounters] = {0};
        (void)hipMemcpy(c, counters_, sizeof(c), hipMemcpyDeviceToHost);
        fprintf(stderr, "kn_solve: %.3f msec (exact-path queries %u, uncertified %u, dense tiles %u)\n",
                ms_solve_, c[0], c[1], c[2]);
    }
    solved_ = true;
    stored_valid_ = false;
    return KN_OK;
}

kn_status Engine::set_k(int k) {
    if (k < 1 || k > KN_MAX_K) return fail(KN_ERR_INVALID_ARGUMENT, "k out of range [1,128]");
    if (!built_) return fail(KN_ERR_STATE, "set_k() before prepare()");
    if (k == cfg_.k) return KN_OK;
    cfg_.k = k;
    // grid density stays; the halo/LDS plan follows K
    // (the grid's x subdivision stays with the grid)
    const AutoParams np = auto_params(n_, k, cfg_.points_per_cell, cfg_.tile, cfg_.halo, nullptr, ap_.xsub);
    ap_.tile[0] = np.tile[0]; ap_.tile[1] = np.tile[1]; ap_.tile[2] = np.tile[2];
    ap_.halo = np.halo;
    {
        // occupied cells hold about the target density (refined grids have many empty cells)
        const double ppc = std::max((double)n_ / std::max(1, C_),
                                    (double)(cfg_.points_per_cell > 0.f ? cfg_.points_per_cell
                                                                        : default_points_per_cell(k)) / ap_.xsub);
        ap_.lds_capacity = lds_capacity_for(staged_points(ap_, ppc));
        ap_.lds_bytes = query_lds_bytes(ap_.tile, ap_.halo, ap_.lds_capacity, ap_.xsub);
    }
    if (graph_) { (void)hipGraphExecDestroy(graph_); graph_ = nullptr; }
    drop_pipeline(true);  // the grid stays: the next solve() queries it with the new K
    for (void** q : {(void**)&out_idx_, (void**)&out_dist_, (void**)&knn_stored_})
        if (*q) { dfree(*q); *q = nullptr; }
    set_[0].out_idx = nullptr;
    set_[0].out_dist = nullptr;
    solved_ = stored_valid_ = false;
    return KN_OK;
}

kn_status Engine::run_graph(int iters, float* ms_per_iter) {
    if (!built_) return fail(KN_ERR_STATE, "run_graph() before prepare()");
    kn_status st;
    if ((st = ensure_outputs()) != KN_OK) return st;  // not inside the capture
    if (graph_ && graph_set_ != live_) { (void)hipGraphExecDestroy(graph_); graph_ = nullptr; }
    if (!graph_) {
        graph_set_ = live_;
        hipGraph_t g;
        if ((st = check(hipStreamBeginCapture(stream_, hipStreamCaptureModeThreadLocal), "capture")) != KN_OK) return st;
        kn_status s1 = build_async(true);
        kn_status s2 = query_async(true);
        hipError_t e = hipStreamEndCapture(stream_, &g);
        if (s1 != KN_OK) return s1;
        if (s2 != KN_OK) return s2;
        if ((st = check(e, "end capture")) != KN_OK) return st;
        e = hipGraphInstantiate(&graph_, g, nullptr, nullptr, 0);
        (void)hipGraphDestroy(g);
        if ((st = check(e, "graph instantiate")) != KN_OK) return st;
    }
    (void)hipEventRecord(ev_[0], stream_);
    for (int i = 0; i < iters; ++i)
        if ((st = check(hipGraphLaunch(graph_, stream_), "graph launch")) != KN_OK) return st;
    (void)hipEventRecord(ev_[1], stream_);
    if ((st = check(hipEventSynchronize(ev_[1]), "graph sync")) != KN_OK) return st;
    float ms = 0.f;
    (void)hipEventElapsedTime(&ms, ev_[0], ev_[1]);
    if (ms_per_iter) *ms_per_iter = iters > 0 ? ms / iters : 0.f;
    solved_ = true;
    stored_valid_ = points3_valid_ = false;  // the graph rebuilt the grid
    return KN_OK;
}

// build stream priority of the pipeline: 0 default, 1 the device's greatest, 2 its least
static int pipe_prio() {
    const char* v = std::getenv("KN_PIPE_PRIO");
    const int p = v ? std::atoi(v) : 0;
    return (p == 1 || p == 2) ? p : 0;
}

Engine::GridSet Engine::members() const {
    return GridSet{points_, bbox_, geom_, cell_count_, cell_scan_, block_sums_, cell_start_, cell_rank_, bin_tmp_,
                   sorted_, perm_, fallback_, counters_, occ_, tree_ws_, tree_nodes_, out_idx_, out_dist_};
}

void Engine::view_set(int s) {
    const GridSet& g = set_[s];
    points_ = g.points; bbox_ = g.bbox; geom_ = g.geom; cell_count_ = g.cell_count; cell_scan_ = g.cell_scan;
    block_sums_ = g.block_sums; cell_start_ = g.cell_start; cell_rank_ = g.cell_rank; bin_tmp_ = g.bin_tmp;
    sorted_ = g.sorted; perm_ = g.perm; fallback_ = g.fallback; counters_ = g.counters; occ_ = g.occ;
    tree_ws_ = g.tree_ws; tree_nodes_ = g.tree_nodes;
    out_idx_ = g.out_idx; out_dist_ = g.out_dist;
    live_ = s;
}

void Engine::drop_pipeline(bool keep_grid) {
    drop_batch();   // batch graphs are captured against both sets
    pipe_.reset();  // waits for both streams, destroys the stage graphs
    if (bstream_) {
        StreamSet ss;
        ss.stream = bstream_;
        for (int i = 0; i < 4; ++i) ss.ev[i] = pev_[i];
        streamset_release(cfg_.device, ss, pipe_prio());
        bstream_ = nullptr;
        for (auto& e : pev_) e = nullptr;
    }
    if (live_ != 0) {
        // the live grid sits in arena2_ / arena3_, which is about to go back to the block cache:
        // copy it (with its input points) to arena_ when it is still needed, view set 0 again and
        // drop the graph captured against the live set
        if (graph_) { (void)hipGraphExecDestroy(graph_); graph_ = nullptr; }
        char* src = live_ == 1 ? arena2_ : arena3_;
        if (keep_grid && src && arena_used_)
            (void)hipMemcpyAsync(arena_, src, arena_used_, hipMemcpyDeviceToDevice, stream_);
        // the live tree and result buffers (same sizes in every set) stay with the live view
        std::swap(set_[0].tree_ws, set_[live_].tree_ws);
        std::swap(set_[0].tree_nodes, set_[live_].tree_nodes);
        std::swap(set_[0].out_idx, set_[live_].out_idx);
        std::swap(set_[0].out_dist, set_[live_].out_dist);
        view_set(0);
    }
    if (arena2_) { dfree(arena2_); arena2_ = nullptr; }  // dfree waits for stream_ (the copy)
    if (arena3_) { dfree(arena3_); arena3_ = nullptr; }
    for (int s = 1; s < 3; ++s) {
        if (set_[s].tree_ws) dfree(set_[s].tree_ws);
        if (set_[s].tree_nodes) dfree(set_[s].tree_nodes);
        if (set_[s].out_idx) dfree(set_[s].out_idx);
        if (set_[s].out_dist) dfree(set_[s].out_dist);
        set_[s] = GridSet{};
    }
    set_[0] = members();
    other_stale_ = true;
}

// Stage bodies of the pipeline (captured once per set): the members view set s while the stage
// enqueues, then the live view comes back.
kn_status Engine::stage_build(int s, hipStream_t st) {
    const int keep = live_;
    hipStream_t ks = stream_;
    view_set(s);
    stream_ = st;
    kn_status r = build_async(true, /*serial=*/false);  // beside the running queries
    if (r == KN_OK && use_tree_) r = tree_build_async();
    stream_ = ks;
    view_set(keep);
    return r;
}

// The tile kernel's exact finish as an epilogue on the build stream instead of right after the
// tile kernel on the query stream: default for the K buckets 32..64, where it wins -- 900K K=50
// (the lane walk's 1-slot top-K margin sends ~360 queries to the exact kernel, ~38 us) 200
// steps 0.913 -> 0.855 ms, 20 steps 0.90 -> 0.868 (interleaved processes on one box,
// profiles/ab_r4_exact_k50.txt); K=32 0.518 -> 0.500 (profiles/ab_r4_m1_epilogue.txt). At K=16
// and K=24 it loses (0.2946 -> 0.2976, 0.396 -> 0.403; r3: 0.2954 -> 0.3016,
// profiles/r4_ab_exact.txt): the extra cross-stream dependency and the exact kernel's workgroups
// competing with the next query cost more than the few us of exact work. Round 5 (two query
// streams, two margin slots at every K): above K = 40 the exact finish on the query stream
// overlaps the next step's query on the other query stream and wins again (900K K=50 100 / 30
// steps 0.7358 -> 0.7276 ms, K=64 equal; profiles/ab_r5_k50.txt), so the epilogue covers the
// buckets 25..40. KN_PIPE_EXACT=0 / 1 forces it off / on.
bool exact_epilogue(int k) {
    static const int mode = [] {
        const char* v = std::getenv("KN_PIPE_EXACT");
        return v ? std::atoi(v) : -1;
    }();
    return mode == 1 || (mode < 0 && k > 24 && k <= 40);
}

kn_status Engine::stage_query(int s, hipStream_t st) {
    const int keep = live_;
    hipStream_t ks = stream_;
    view_set(s);
    stream_ = st;
    kn_status r;
    if (use_tree_) {
        r = tree_query_async();
    } else if (!exact_epilogue(cfg_.k)) {
        r = query_async(true);
    } else {
        // the tile kernel only: its fallback list's exact finish is the epilogue on the build
        // stream, so the next step's queries follow this one's without waiting for it
        QueryBuffers q = query_buffers();
        q.counters_zeroed = 1;
        q.exact_mode = 1;
        r = check(launch_query(q, stream_), "query");
    }
    stream_ = ks;
    view_set(keep);
    return r;
}

kn_status Engine::stage_exact(int s, hipStream_t st) {
    const int keep = live_;
    view_set(s);
    QueryBuffers q = query_buffers();
    q.counters_zeroed = 1;
    q.exact_mode = 2;
    const kn_status r = check(launch_query(q, st), "exact finish");
    view_set(keep);
    return r;
}

// Grid set s carved from base (the carve of allocate(), its own input points).
kn_status Engine::carve_set(int s, char* base) {
    const int C = C_, n = n_;
    const size_t nb = scan_block_count(C) + 1;
    char* p = base;
    GridSet& g = set_[s];
    g.points = carve<float>(p, (size_t)n * 3);
    g.bbox = carve<unsigned>(p, kBBoxWords);
    g.geom = carve<GridGeom>(p, 1);
    g.cell_count = carve<int>(p, C + 1);
    g.cell_scan = carve<int>(p, C + 1);
    g.cell_start = carve<int>(p, C + 1);
    g.block_sums = carve<int>(p, nb);
    g.bin_tmp = carve<float4>(p, n);
    g.cell_rank = reinterpret_cast<int2*>(g.bin_tmp);
    g.sorted = carve<float4>(p, n);
    g.perm = carve<unsigned>(p, n);
    g.fallback = carve<unsigned>(p, n);
    g.counters = carve<unsigned>(p, kNumCounters);
    g.occ = carve<unsigned long long>(p, 1);
    g.tree_ws = g.tree_nodes = nullptr;
    g.out_idx = nullptr;
    g.out_dist = nullptr;
    if (use_tree_) {
        kn_status st;
        if ((st = check(dmalloc(&g.tree_ws, tree_workspace_bytes(n_, ap_.dims)), "hipMalloc(tree 2)")) != KN_OK ||
            (st = check(dmalloc(&g.tree_nodes, tree_node_bytes(n_)), "hipMalloc(tree nodes 2)")) != KN_OK)
            return st;
    }
    return KN_OK;
}

// The other grid sets + the build stream + the pipeline's stage graphs.
kn_status Engine::ensure_pipeline() {
    kn_status st;
    if ((st = ensure_outputs()) != KN_OK) return st;
    set_[live_] = members();  // tree buffers allocated since the last carve
    // Two query streams (default; KN_PIPE_QSTREAMS=1: one): odd steps' queries on a second
    // stream, so step i+1's queries start as soon as its build is done instead of after step
    // i's last workgroup and the kernel boundary (~15 us per step inside a 10-step graph,
    // profiles/r4_pipe_unroll.txt). 900K K=16, interleaved processes on one box: 200 steps
    // 0.2894 -> 0.2756 ms, the driver's 20 / 5 0.3080 -> 0.3048 (profiles/r5_qstreams.txt)
    static const int qstreams_env = [] {
        const char* v = std::getenv("KN_PIPE_QSTREAMS");
        return v ? std::atoi(v) : 2;
    }();
    const int qstreams = qstreams_cfg_ > 0 ? qstreams_cfg_ : qstreams_env;
    if (!pipe_.ready()) {
        // Three grid sets with two query streams (KN_PIPE_SETS=2: two): step i+1's build then
        // waits for step i-2's query instead of step i-1's, which still runs beside step i's; with
        // two sets the build (~170 us beside a query) ran only after step i-1's query ended and
        // step i+1's query started after step i's, leaving the GPU without any query kernel 10 %
        // of the time (rocprof, gpurun_out/r5engprof2). Needs one more set in memory: only when it
        // fits comfortably.
        static const int sets_env0 = [] {
            const char* v = std::getenv("KN_PIPE_SETS");
            return v ? std::atoi(v) : 3;
        }();
        const int sets_env = sets_cfg_ > 0 ? sets_cfg_ : sets_env0;
        nsets_ = 2;
        if (qstreams >= 2 && sets_env >= 3) {
            size_t fr = 0, tot = 0;
            const size_t need = arena_bytes_ + 2 * std::max<size_t>(1, (size_t)n_ * cfg_.k) * sizeof(float) +
                                (use_tree_ ? tree_workspace_bytes(n_, ap_.dims) + tree_node_bytes(n_) : 0);
            if (hipMemGetInfo(&fr, &tot) == hipSuccess && need < fr / 4) nsets_ = 3;
        }
    }
    for (int s = 1; s < nsets_; ++s) {
        char*& ar = s == 1 ? arena2_ : arena3_;
        if (ar) continue;
        if ((st = check(dmalloc(&ar, arena_bytes_), s == 1 ? "hipMalloc(grid set 2)" : "hipMalloc(grid set 3)")) != KN_OK)
            return st;
        if ((st = carve_set(s, ar)) != KN_OK) {
            drop_pipeline();
            return st;
        }
        other_stale_ = true;
    }
    for (int s = 0; s < nsets_; ++s) {
        // the other sets' results (per-set outputs: the exact finish of step i runs while step
        // i+1 queries)
        if (s == live_) continue;
        GridSet& g = set_[s];
        const size_t nk = std::max<size_t>(1, (size_t)n_ * cfg_.k);
        if (!g.out_idx && (st = check(dmalloc(&g.out_idx, nk * sizeof(unsigned)), "hipMalloc(knn 2)")) != KN_OK) return st;
        if (cfg_.with_distances && !g.out_dist &&
            (st = check(dmalloc(&g.out_dist, nk * sizeof(float)), "hipMalloc(dist 2)")) != KN_OK)
            return st;
    }
    if (!bstream_) {
        // KN_PIPE_PRIO=1: the build stream at the device's highest priority (its latency-bound
        // kernels then take CU slots as soon as the query's workgroups free them)
        StreamSet ss;
        if ((st = check(streamset_acquire(cfg_.device, &ss, pipe_prio()), "hipStreamCreate")) != KN_OK) return st;
        bstream_ = ss.stream;
        for (int i = 0; i < 4; ++i) pev_[i] = ss.ev[i];
    }
    if (!pipe_.ready()) {
        auto b = [this](int s, hipStream_t st2) { return stage_build(s, st2) == KN_OK ? hipSuccess : hipErrorUnknown; };
        auto q = [this](int s, hipStream_t st2) { return stage_query(s, st2) == KN_OK ? hipSuccess : hipErrorUnknown; };
        Pipeline::Stage x;
        if (!use_tree_ && exact_epilogue(cfg_.k))  // the tree query finishes its own exact-path queries
            x = [this](int s, hipStream_t st2) { return stage_exact(s, st2) == KN_OK ? hipSuccess : hipErrorUnknown; };
        if ((st = check(pipe_.init(stream_, bstream_, b, q, x, false, qstreams, nsets_), "pipeline init")) != KN_OK)
            return st;
        // KN_PIPE_EAGER=1 (diagnostics): the resident pipeline's stages enqueued per step instead of
        // replayed from their graphs (the 20-step cold start, profiles/r6_coldstart.txt)
        static const bool eager_env = [] {
            const char* v = std::getenv("KN_PIPE_EAGER");
            return v && v[0] == '1';
        }();
        if (eager_env) pipe_.set_eager(true);
    }
    return KN_OK;
}

kn_status Engine::set_pipeline_shape(int query_streams, int sets) {
    if (query_streams != -1 && query_streams != 1 && query_streams != 2)
        return fail(KN_ERR_INVALID_ARGUMENT, "set_pipeline_shape: query streams must be 1, 2 or -1");
    if (sets != -1 && sets != 2 && sets != 3) return fail(KN_ERR_INVALID_ARGUMENT, "set_pipeline_shape: sets must be 2, 3 or -1");
    if (query_streams == qstreams_cfg_ && sets == sets_cfg_) return KN_OK;
    qstreams_cfg_ = query_streams;
    sets_cfg_ = sets;
    if (pipe_.ready()) drop_pipeline(/*keep_grid=*/true);  // rebuilt with the new shape on next use
    return KN_OK;
}

// Steps per graph launch of the resident pipeline: 10 (900K, K=16, 200 steps: 0.310 ms per step
// with one graph per stage and step, 0.296 with 4 steps per graph, 0.293 with 10; at the
// driver's 20 steps 0.318 / 0.310 for 4 / 10; profiles/r4_pipe_unroll.txt)
static int pipe_unroll_default() {
    const char* v = std::getenv("KN_PIPE_UNROLL");
    return v ? std::atoi(v) : 10;
}

// Software-pipelined steps over two grid sets (pipeline.hpp): build(i+1) on bstream_ while
// query(i) runs on stream_. The query kernel fills the chip and the build's five latency-bound
// kernels (~50 us at 900K, ~15 % of a step) run in its shadow. Resident mode: every step bins
// and queries the engine's current cloud (both sets hold it as input).
kn_status Engine::launch_pipelined(int iters, int unroll) {
    if (!built_) return fail(KN_ERR_STATE, "launch_pipelined() before prepare()");
    kn_status st;
    if ((st = ensure_pipeline()) != KN_OK) return st;
    if (other_stale_) {
        // the other set's input takes the live cloud (resident mode: both sets bin it); the
        // primed build of a previous stream read other points
        if ((st = check(pipe_.unprime(), "pipeline")) != KN_OK) return st;
        for (int s = 0; s < nsets_; ++s)
            if (s != live_ && n_ > 0 &&
                (st = check(hipMemcpyAsync(set_[s].points, points_, (size_t)n_ * 12, hipMemcpyDeviceToDevice, stream_),
                            "D2D points")) != KN_OK)
                return st;
        if ((st = check(hipStreamSynchronize(stream_), "sync")) != KN_OK) return st;
        other_stale_ = false;
    }
    stream_mode_ = false;
    if (iters <= 0) return KN_OK;
    if (unroll < 0) unroll = pipe_unroll_default();
    hipError_t e = pipe_.launch(iters, unroll);
    // later work on stream_ (getters, serial steps) follows the last step's epilogue (its exact
    // finish runs on the build stream)
    if (e == hipSuccess) e = hipStreamWaitEvent(stream_, pipe_.last_done(), 0);
    if (e != hipSuccess) {
        drop_pipeline();
        return check(e == hipErrorUnknown ? hipErrorLaunchFailure : e, "pipelined launch");
    }
    // the last step's grid is the engine's current grid (getters, stats, stored-space views);
    // later getters are stream-ordered after its query (stream_), and the primed build writes the
    // other set
    view_set(pipe_.last_set());
    solved_ = true;
    stored_valid_ = points3_valid_ = false;
    return KN_OK;
}

kn_status Engine::stream_step(const float* d_pts, const float* d_next) {
    if (!built_) return fail(KN_ERR_STATE, "stream_step() before prepare()");
    if (!d_pts && n_ > 0) return fail(KN_ERR_INVALID_ARGUMENT, "null points");
    kn_status st;
    if ((st = ensure_pipeline()) != KN_OK) return st;
    const size_t bytes = (size_t)n_ * 12;
    auto copy_in = [this, bytes](const float* src) {
        return [this, bytes, src](int s, hipStream_t sd) {
            return bytes ? hipMemcpyAsync(set_[s].points, src, bytes, hipMemcpyDeviceToDevice, sd) : hipSuccess;
        };
    };
    if (!stream_mode_) {
        // a resident-mode prime read the resident cloud: this stream's first step bins its own
        if ((st = check(pipe_.unprime(), "pipeline")) != KN_OK) return st;
        stream_mode_ = true;
    }
    Pipeline::Stage pre = copy_in(d_pts);
    Pipeline::Stage nxt = copy_in(d_next);
    hipError_t e = pipe_.step_with(pre, d_next ? &nxt : nullptr);
    if (e == hipSuccess) e = hipStreamWaitEvent(stream_, pipe_.last_done(), 0);
    if (e != hipSuccess) {
        drop_pipeline();
        return check(e == hipErrorUnknown ? hipErrorLaunchFailure : e, "stream step");
    }
    view_set(pipe_.last_set());
    other_stale_ = true;
    solved_ = true;
    stored_valid_ = points3_valid_ = false;
    return KN_OK;
}

void Engine::drop_batch() {
    if (stream_) (void)hipStreamSynchronize(stream_);
    if (bstream_) (void)hipStreamSynchronize(bstream_);
    bpipe_.reset();  // (shares pipe_'s second query stream: reset before pipe_)
    for (auto& kv : bgraphs_) (void)hipGraphExecDestroy(kv.second);
    bgraphs_.clear();
    for (auto e : bev_) (void)hipEventDestroy(e);
    bev_.clear();
    if (qstream2_) {
        (void)hipStreamSynchronize(qstream2_);
        (void)hipStreamDestroy(qstream2_);
        qstream2_ = nullptr;
    }
    if (tab_) { dfree(tab_); tab_ = nullptr; }
}

// Steps 0..L-1 of a batch in one graph, sets alternating (step j: set j & 1). Build stream: copy-in
// + build of step 0; then per step j: (epilogue of step j-1 after its query) and the copy-in +
// build of step j+1 into the set step j-1 released. Main stream: query of step j after its build.
kn_status Engine::batch_graph(int L, hipGraphExec_t* out) {
    auto it = bgraphs_.find(L);
    if (it != bgraphs_.end()) { *out = it->second; return KN_OK; }
    // KN_BATCH_QSTREAMS=2 (diagnostics): consecutive steps' queries on two streams inside the
    // graph. Crashes the HIP runtime during capture (segfault after the first graphs, as the
    // resident pipeline's unrolled graphs with two query streams, profiles/r5_qstreams.txt): the
    // eager batch pipeline (stream_batch_eager) overlaps consecutive clouds' queries instead
    static const int bqs = [] {
        const char* v = std::getenv("KN_BATCH_QSTREAMS");
        return v ? std::atoi(v) : 1;
    }();
    if (bqs >= 2 && !qstream2_ &&
        hipStreamCreateWithFlags(&qstream2_, hipStreamNonBlocking) != hipSuccess)
        return fail(KN_ERR_DEVICE, "hipStreamCreate");
    hipStream_t qst[2] = {stream_, bqs >= 2 ? qstream2_ : stream_};
    while (bev_.size() < 2 * (size_t)L + 3) {
        hipEvent_t e = nullptr;
        if (hipEventCreateWithFlags(&e, hipEventDisableTiming) != hipSuccess) return fail(KN_ERR_DEVICE, "hipEventCreate");
        bev_.push_back(e);
    }
    hipEvent_t fork = bev_[0], join = bev_[1], join2 = bev_[2 + 2 * L];
    hipEvent_t* eb = bev_.data() + 2;      // step j built
    hipEvent_t* eq = bev_.data() + 2 + L;  // step j queried
    const bool epi = !use_tree_ && exact_epilogue(cfg_.k);
    const size_t nf = (size_t)n_ * 3;
    hipError_t e = hipStreamBeginCapture(stream_, hipStreamCaptureModeThreadLocal);
    if (e != hipSuccess) return check(e, "batch capture");
    kn_status st = KN_OK;
    auto H = [&](hipError_t r) { if (st == KN_OK && r != hipSuccess) st = check(r, "batch capture"); };
    auto S = [&](kn_status r) { if (st == KN_OK) st = r; };
    auto build = [&](int j) {
        const int s = j & 1;
        H(launch_copy_from_ref(reinterpret_cast<const float* const*>(tab_ + j), set_[s].points, nf, bstream_));
        if (st == KN_OK) S(stage_build(s, bstream_));
        H(hipEventRecord(eb[j], bstream_));
    };
    auto exact = [&](int j) {
        out_ref_slot_ = j;
        S(stage_exact(j & 1, bstream_));
        out_ref_slot_ = -1;
    };
    H(hipEventRecord(fork, stream_));
    H(hipStreamWaitEvent(bstream_, fork, 0));
    if (qst[1] != stream_) H(hipStreamWaitEvent(qst[1], fork, 0));
    build(0);
    for (int j = 0; j < L && st == KN_OK; ++j) {
        hipStream_t qs = qst[j & 1];
        H(hipStreamWaitEvent(qs, eb[j], 0));
        out_ref_slot_ = j;
        if (st == KN_OK) S(stage_query(j & 1, qs));
        out_ref_slot_ = -1;
        H(hipEventRecord(eq[j], qs));
        if (j >= 1) {
            H(hipStreamWaitEvent(bstream_, eq[j - 1], 0));
            if (epi && st == KN_OK) exact(j - 1);
        }
        if (j + 1 < L && st == KN_OK) build(j + 1);
    }
    if (epi && st == KN_OK) {
        H(hipStreamWaitEvent(bstream_, eq[L - 1], 0));
        exact(L - 1);
    }
    H(hipEventRecord(join, bstream_));
    H(hipStreamWaitEvent(stream_, join, 0));
    if (qst[1] != stream_) {
        H(hipEventRecord(join2, qst[1]));
        H(hipStreamWaitEvent(stream_, join2, 0));
    }
    hipGraph_t g = nullptr;
    const hipError_t ee = hipStreamEndCapture(stream_, &g);
    if (st != KN_OK) {
        if (g) (void)hipGraphDestroy(g);
        return st;
    }
    if ((st = check(ee, "batch end capture")) != KN_OK) return st;
    hipGraphExec_t x = nullptr;
    e = hipGraphInstantiate(&x, g, nullptr, nullptr, 0);
    (void)hipGraphDestroy(g);
    if ((st = check(e, "batch graph instantiate")) != KN_OK) return st;
    bgraphs_[L] = x;
    *out = x;
    return KN_OK;
}

// Eager batch (default, KN_BATCH_MODE=graph: the captured batch graphs below): the clouds go
// through a second Pipeline over the same grid sets and streams in eager mode, one step_with()
// per cloud -- copy-in + build on the build stream, queries alternating between the two query
// streams (consecutive clouds' queries overlap as in the resident pipeline; a captured graph whose
// queries alternate between two streams crashes the HIP runtime), rows
// straight into the caller's buffers (set s's stages read bout_*_[s] when they are enqueued).
kn_status Engine::stream_batch_eager(int m, const float* const* d_in, unsigned* const* d_idx, float* const* d_dist) {
    kn_status st;
    if (!bpipe_.ready()) {
        auto b = [this](int s, hipStream_t st2) { return stage_build(s, st2) == KN_OK ? hipSuccess : hipErrorUnknown; };
        auto q = [this](int s, hipStream_t st2) {
            out_ovr_set_ = s;
            const kn_status r = stage_query(s, st2);
            out_ovr_set_ = -1;
            return r == KN_OK ? hipSuccess : hipErrorUnknown;
        };
        Pipeline::Stage x;
        if (!use_tree_ && exact_epilogue(cfg_.k))
            x = [this](int s, hipStream_t st2) {
                out_ovr_set_ = s;
                const kn_status r = stage_exact(s, st2);
                out_ovr_set_ = -1;
                return r == KN_OK ? hipSuccess : hipErrorUnknown;
            };
        hipStream_t aux = pipe_.aux_stream();
        // as many grid sets as the resident pipeline (three with two query streams)
        if ((st = check(bpipe_.init(stream_, bstream_, b, q, x, false, aux ? 2 : 1, nsets_, aux), "batch pipeline init")) !=
            KN_OK)
            return st;
        bpipe_.set_eager(true);
    }
    // the resident pipeline's last queries (joined into stream_ by launch_pipelined / stream_step)
    // read the sets this batch rebuilds: its builds wait for stream_'s tail
    if ((st = check(pipe_.unprime(), "pipeline")) != KN_OK) return st;
    if (bev_.empty()) {
        hipEvent_t ev = nullptr;
        if (hipEventCreateWithFlags(&ev, hipEventDisableTiming) != hipSuccess) return fail(KN_ERR_DEVICE, "hipEventCreate");
        bev_.push_back(ev);
    }
    if ((st = check(hipEventRecord(bev_[0], stream_), "batch event")) != KN_OK) return st;
    if ((st = check(hipStreamWaitEvent(bstream_, bev_[0], 0), "batch event")) != KN_OK) return st;
    const size_t bytes = (size_t)n_ * 12;
    auto pre = [this, bytes, d_in, d_idx, d_dist](int j) {
        const float* src = d_in[j];
        unsigned* oi = d_idx[j];
        float* od = d_dist ? d_dist[j] : nullptr;
        return Pipeline::Stage([this, bytes, src, oi, od](int s, hipStream_t sd) {
            bout_idx_[s] = oi;
            bout_dist_[s] = od;
            return bytes ? hipMemcpyAsync(set_[s].points, src, bytes, hipMemcpyDeviceToDevice, sd) : hipSuccess;
        });
    };
    hipError_t e = hipSuccess;
    for (int j = 0; j < m && e == hipSuccess; ++j) {
        const Pipeline::Stage p = pre(j);
        if (j + 1 < m) {
            const Pipeline::Stage nx = pre(j + 1);
            e = bpipe_.step_with(p, &nx);
        } else {
            e = bpipe_.step_with(p, nullptr);
        }
    }
    // later work on either stream (getters, resident or stream steps) follows the batch
    if (e == hipSuccess) e = hipStreamWaitEvent(stream_, bpipe_.last_done(), 0);
    if (e == hipSuccess) e = hipStreamWaitEvent(bstream_, bpipe_.last_done(), 0);
    if (e != hipSuccess) {
        drop_pipeline();
        return check(e == hipErrorUnknown ? hipErrorLaunchFailure : e, "batch step");
    }
    view_set(bpipe_.last_set());
    other_stale_ = true;
    stream_mode_ = true;
    solved_ = false;
    stored_valid_ = points3_valid_ = false;
    return KN_OK;
}

kn_status Engine::stream_batch(int m, const float* const* d_in, unsigned* const* d_idx, float* const* d_dist) {
    if (!built_) return fail(KN_ERR_STATE, "stream_batch() before prepare()");
    if (m < 0 || (m > 0 && (!d_in || !d_idx))) return fail(KN_ERR_INVALID_ARGUMENT, "stream_batch: null tables");
    for (int j = 0; j < m; ++j)
        if ((n_ > 0 && !d_in[j]) || !d_idx[j] || (d_dist && !d_dist[j]))
            return fail(KN_ERR_INVALID_ARGUMENT, "stream_batch: null pointer in a table");
    if (m == 0) return KN_OK;
    kn_status st;
    if ((st = ensure_pipeline()) != KN_OK) return st;
    static const bool graph_mode = [] {
        const char* v = std::getenv("KN_BATCH_MODE");
        return v && std::string(v) == "graph";
    }();
    if (!(batch_mode_ >= 0 ? batch_mode_ == 1 : graph_mode)) return stream_batch_eager(m, d_in, d_idx, d_dist);
    if (!tab_ && (st = check(dmalloc(reinterpret_cast<void**>(&tab_), 3 * kBatchMax * sizeof(void*)), "hipMalloc(batch table)")) != KN_OK)
        return st;
    // everything the pipeline enqueued (a primed build, an epilogue) is done before the batch
    // graphs reuse both sets: the side stream's tail joins the main stream
    if ((st = check(pipe_.unprime(), "pipeline")) != KN_OK) return st;
    // chunks of power-of-two lengths (largest first, <= kBatchMax): six graphs serve any m, all
    // captured at the first call, so a later (timed) call never captures. Each chunk starts with
    // its first build not overlapped by a query (the chunk's graph follows the previous one).
    if (bgraphs_.empty()) {
        for (int L = 1; L <= kBatchMax; L *= 2) {
            hipGraphExec_t g = nullptr;
            if ((st = batch_graph(L, &g)) != KN_OK) return st;
        }
    }
    int last_L = 1;
    for (int c0 = 0; c0 < m;) {
        int L = kBatchMax;
        while (L > m - c0) L >>= 1;
        hipGraphExec_t g = nullptr;
        if ((st = batch_graph(L, &g)) != KN_OK) return st;
        void* tab[3 * kBatchMax];
        for (int j = 0; j < 3 * kBatchMax; ++j) tab[j] = nullptr;
        for (int j = 0; j < L; ++j) {
            tab[j] = const_cast<float*>(d_in[c0 + j]);
            tab[kBatchMax + j] = d_idx[c0 + j];
            tab[2 * kBatchMax + j] = d_dist ? d_dist[c0 + j] : nullptr;
        }
        if ((st = check(launch_set_ptr_table(tab, 3 * kBatchMax, tab_, stream_), "batch table")) != KN_OK) return st;
        if ((st = check(hipGraphLaunch(g, stream_), "batch graph launch")) != KN_OK) return st;
        c0 += L;
        last_L = L;
    }
    // the last step's grid is the engine's grid (stats, stored-space views); its rows went to the
    // caller, so the engine's own results are stale
    view_set((last_L - 1) & 1);
    // later pipeline work on the build stream (resident or stream steps) waits for the batch
    if ((st = check(hipEventRecord(bev_[0], stream_), "batch event")) != KN_OK) return st;
    if ((st = check(hipStreamWaitEvent(bstream_, bev_[0], 0), "batch event")) != KN_OK) return st;
    other_stale_ = true;
    stream_mode_ = true;
    solved_ = false;
    stored_valid_ = points3_valid_ = false;
    return KN_OK;
}

kn_status Engine::launch_graph(int iters) {
    if (!built_) return fail(KN_ERR_STATE, "launch_graph() before prepare()");
    kn_status st;
    if ((st = ensure_outputs()) != KN_OK) return st;  // not inside the capture
    if (graph_ && graph_set_ != live_) { (void)hipGraphExecDestroy(graph_); graph_ = nullptr; }
    if (!graph_) {
        graph_set_ = live_;
        hipGraph_t g;
        if ((st = check(hipStreamBeginCapture(stream_, hipStreamCaptureModeThreadLocal), "capture")) != KN_OK) return st;
        kn_status s1 = build_async(true);
        kn_status s2 = query_async(true);
        hipError_t e = hipStreamEndCapture(stream_, &g);
        if (s1 != KN_OK) return s1;
        if (s2 != KN_OK) return s2;
        if ((st = check(e, "end capture")) != KN_OK) return st;
        e = hipGraphInstantiate(&graph_, g, nullptr, nullptr, 0);
        (void)hipGraphDestroy(g);
        if ((st = check(e, "graph instantiate")) != KN_OK) return st;
    }
    for (int i = 0; i < iters; ++i)
        if ((st = check(hipGraphLaunch(graph_, stream_), "graph launch")) != KN_OK) return st;
    solved_ = true;
    stored_valid_ = points3_valid_ = false;  // the graph rebuilds the grid
    return KN_OK;
}

kn_status Engine::sync() {
    kn_status st;
    if ((st = check(pipe_.sync(), "pipeline sync")) != KN_OK) return st;
    return check(hipStreamSynchronize(stream_), "stream sync");
}

kn_status Engine::copy_results(unsigned* d_idx, float* d_dist) {
    if (!solved_) return fail(KN_ERR_STATE, "not solved");
    const size_t nk = (size_t)n_ * cfg_.k;
    kn_status st;
    if (d_idx && nk && (st = check(hipMemcpyAsync(d_idx, out_idx_, nk * 4, hipMemcpyDeviceToDevice, stream_), "D2D idx")) != KN_OK)
        return st;
    if (d_dist && out_dist_ && nk &&
        (st = check(hipMemcpyAsync(d_dist, out_dist_, nk * 4, hipMemcpyDeviceToDevice, stream_), "D2D dist")) != KN_OK)
        return st;
    return sync();
}

kn_status Engine::counters(unsigned out[kNumCounters]) {
    kn_status st;
    if ((st = check(hipMemcpyAsync(out, counters_, kNumCounters * sizeof(unsigned), hipMemcpyDeviceToHost, stream_), "D2H counters")) != KN_OK) return st;
    return sync();
}

unsigned* Engine::d_knn_stored() {
    if (!solved_) return nullptr;
    if (stored_valid_) return knn_stored_;
    // ids only: the reference exposes no distances (knearests.h:3-16), so the stored-space
    // distance copy is made on demand by get_distances_stored()
    const size_t nk = std::max<size_t>(1, (size_t)n_ * cfg_.k);
    if (!inv_perm_ && check(dmalloc(&inv_perm_, std::max<size_t>(1, n_) * sizeof(unsigned)), "hipMalloc(inv)") != KN_OK)
        return nullptr;
    if (!knn_stored_ && check(dmalloc(&knn_stored_, nk * sizeof(unsigned)), "hipMalloc(knn_stored)") != KN_OK)
        return nullptr;
    if (check(launch_invert_perm(perm_, n_, inv_perm_, stream_), "invert perm") != KN_OK) return nullptr;
    if (check(launch_to_stored_space(out_idx_, perm_, inv_perm_, n_, cfg_.k, knn_stored_, nullptr, nullptr, stream_),
              "to stored space") != KN_OK)
        return nullptr;
    if (check(hipStreamSynchronize(stream_), "sync") != KN_OK) return nullptr;
    stored_valid_ = true;
    return knn_stored_;
}

float* Engine::d_points3() {
    if (!built_) return nullptr;
    if (points3_valid_) return points3_;
    if (!points3_ && check(dmalloc(&points3_, std::max<size_t>(1, (size_t)n_ * 3) * sizeof(float)),
                           "hipMalloc(points3)") != KN_OK)
        return nullptr;
    if (check(launch_sorted_xyz(sorted_, n_, points3_, stream_), "sorted xyz") != KN_OK) return nullptr;
    if (check(hipStreamSynchronize(stream_), "sync") != KN_OK) return nullptr;
    points3_valid_ = true;
    return points3_;
}

// malloc'd host copy (the reference getters' contract: the caller free()s it), through the
// pinned staging ring
template <class T>
static T* d2h(const T* d, size_t count, hipStream_t s) {
    T* h = (T*)malloc(std::max<size_t>(1, count) * sizeof(T));
    if (!h) return nullptr;
    if (count && copy_d2h_staged(h, d, count * sizeof(T), s) != hipSuccess) {
        free(h);
        return nullptr;
    }
    return h;
}

float* Engine::get_points_sorted() {
    if (!built_) { fail(KN_ERR_STATE, "not prepared"); return nullptr; }
    const float* d = d_points3();  // float3 view of the stored points (one device pass)
    if (!d) return nullptr;
    return d2h(d, (size_t)n_ * 3, stream_);
}
unsigned* Engine::get_permutation() {
    if (!built_) { fail(KN_ERR_STATE, "not prepared"); return nullptr; }
    return d2h(perm_, (size_t)n_, stream_);
}
unsigned* Engine::get_knearests_stored() {
    // KN_GET_TRACE=1: the getter's phases on stderr (stored-space conversion, host copy)
    static const bool trace = [] {
        const char* v = std::getenv("KN_GET_TRACE");
        return v && std::atoi(v) != 0;
    }();
    const auto t0 = std::chrono::steady_clock::now();
    unsigned* d = d_knn_stored();
    if (!d) { if (err_.empty()) fail(KN_ERR_STATE, "not solved"); return nullptr; }
    const auto t1 = std::chrono::steady_clock::now();
    unsigned* h = d2h(d, (size_t)n_ * cfg_.k, stream_);
    if (trace) {
        const auto t2 = std::chrono::steady_clock::now();
        fprintf(stderr, "get_knearests: to_stored %.3f ms, copy %.3f ms\n",
                std::chrono::duration<double, std::milli>(t1 - t0).count(),
                std::chrono::duration<double, std::milli>(t2 - t1).count());
    }
    return h;
}
float* Engine::get_distances_stored() {
    if (!out_dist_) { fail(KN_ERR_STATE, "distances disabled"); return nullptr; }
    if (!d_knn_stored()) return nullptr;  // also builds inv_perm_
    // stored-space distances: a temporary device buffer, freed before returning
    const size_t nk = (size_t)n_ * cfg_.k;
    float* tmp = nullptr;
    if (check(dmalloc(&tmp, std::max<size_t>(1, nk) * sizeof(float)), "hipMalloc(dist_stored)") != KN_OK) return nullptr;
    float* out = nullptr;
    // the id half rewrites knn_stored_ with the values it already holds
    if (check(launch_to_stored_space(out_idx_, perm_, inv_perm_, n_, cfg_.k, knn_stored_, out_dist_, tmp, stream_),
              "to stored space") == KN_OK)
        out = d2h(tmp, nk, stream_);
    dfree(tmp);
    return out;
}
unsigned* Engine::get_neighbors_original() {
    if (!solved_) { fail(KN_ERR_STATE, "not solved"); return nullptr; }
    return d2h(out_idx_, (size_t)n_ * cfg_.k, stream_);
}
float* Engine::get_distances_original() {
    if (!solved_ || !out_dist_) { fail(KN_ERR_STATE, "not solved / distances disabled"); return nullptr; }
    return d2h(out_dist_, (size_t)n_ * cfg_.k, stream_);
}

kn_status Engine::stats(kn_stats* out, std::vector<int>* hist) {
    if (!built_) return fail(KN_ERR_STATE, "not prepared");
    constexpr int H = 64;
    kn_status st;
    if ((st = check(launch_cell_stats(cell_start_, C_, cell_count_, H, stream_), "cell stats")) != KN_OK) return st;
    std::vector<int> v(3 + H);
    if ((st = check(hipMemcpyAsync(v.data(), cell_count_, v.size() * sizeof(int), hipMemcpyDeviceToHost, stream_), "D2H")) != KN_OK) return st;
    unsigned c[kNumCounters] = {0};
    if ((st = check(hipMemcpyAsync(c, counters_, sizeof(c), hipMemcpyDeviceToHost, stream_), "D2H")) != KN_OK) return st;
    if ((st = check(hipStreamSynchronize(stream_), "sync")) != KN_OK) return st;
    std::memset(out, 0, sizeof(*out));
    out->num_points = n_;
    out->k = cfg_.k;
    for (int a = 0; a < 3; ++a) out->dims[a] = ap_.dims[a];
    out->num_cells = C_;
    out->min_cell = C_ ? v[0] : 0;
    out->max_cell = v[1];
    out->avg_cell = C_ ? (float)n_ / C_ : 0.f;
    out->empty_cells = v[2];
    out->fallback_queries = solved_ ? (int)c[0] : 0;
    out->uncertified_queries = solved_ ? (int)c[1] : 0;
    out->ms_build = ms_build_;
    out->ms_solve = ms_solve_;
    out->range_allocations = (int)scratch_allocs_;
    if (hist) hist->assign(v.begin() + 3, v.end());
    // the stats kernel used cell_count_ as scratch: it is rebuilt by every build
    return KN_OK;
}

namespace {
constexpr unsigned kMagicV1 = 0x4b4e4731;  // "KNG1": {magic, n, dims[3], k}
constexpr unsigned kMagic = 0x4b4e4732;    // "KNG2": + {tile[3], halo, lds_capacity, flags}
// KNG2 flags word: bit 0 = the plan words are valid, bit 1 = the grid was refined (the cloud's
// density varies: algo auto serves it with the tree path)
constexpr int kPlanValid = 1, kPlanRefined = 2, kPlanXsubShift = 8;  // flags: bits 8-11 = xsub
constexpr size_t kMaxLdsBytes = 160 * 1024;  // gfx950 LDS per workgroup
}  // namespace

kn_status Engine::save(const char* path) {
    if (!built_) return fail(KN_ERR_STATE, "not prepared");
    std::ofstream f(path, std::ios::binary);
    if (!f) return fail(KN_ERR_IO, std::string("cannot open ") + path);
    GridGeom g;
    kn_status st;
    if ((st = check(hipMemcpy(&g, geom_, sizeof(g), hipMemcpyDeviceToHost), "D2H geom")) != KN_OK) return st;
    std::vector<float4> s(n_);
    std::vector<int> cs(C_ + 1);
    if (n_ && (st = check(hipMemcpy(s.data(), sorted_, (size_t)n_ * sizeof(float4), hipMemcpyDeviceToHost), "D2H")) != KN_OK) return st;
    if ((st = check(hipMemcpy(cs.data(), cell_start_, ((size_t)C_ + 1) * sizeof(int), hipMemcpyDeviceToHost), "D2H")) != KN_OK) return st;
    // the tile / halo / LDS plan travels with the grid: a refined (occupancy-adaptive) grid keeps
    // the plan of the target density, which allocate() cannot re-derive from n / C
    const int hdr[12] = {(int)kMagic, n_, ap_.dims[0], ap_.dims[1], ap_.dims[2], cfg_.k,
                         ap_.tile[0], ap_.tile[1], ap_.tile[2], ap_.halo, ap_.lds_capacity,
                         kPlanValid | (refined_ ? kPlanRefined : 0) | (ap_.xsub << kPlanXsubShift)};
    f.write((const char*)hdr, sizeof(hdr));
    f.write((const char*)&g, sizeof(g));
    f.write((const char*)s.data(), s.size() * sizeof(float4));
    f.write((const char*)cs.data(), cs.size() * sizeof(int));
    return f ? KN_OK : fail(KN_ERR_IO, "write failed");
}

Engine* Engine::load(const char* path, const EngineConfig& cfg, std::string* err) {
    std::ifstream f(path, std::ios::binary);
    if (!f) { if (err) *err = std::string("cannot open ") + path; return nullptr; }
    int hdr[12] = {0};
    f.read((char*)hdr, 6 * sizeof(int));
    const bool v2 = f && hdr[0] == (int)kMagic;
    if (!f || (!v2 && hdr[0] != (int)kMagicV1) || hdr[1] < 0) { if (err) *err = "bad file header"; return nullptr; }
    if (v2) f.read((char*)(hdr + 6), 6 * sizeof(int));
    GridGeom g;
    f.read((char*)&g, sizeof(g));
    const int n = hdr[1];
    const long C = (long)hdr[2] * hdr[3] * hdr[4];
    if (hdr[2] <= 0 || hdr[3] <= 0 || hdr[4] <= 0 || C > 400000000L) { if (err) *err = "bad grid"; return nullptr; }
    std::vector<float4> s(n);
    std::vector<int> cs(C + 1);
    f.read((char*)s.data(), s.size() * sizeof(float4));
    f.read((char*)cs.data(), cs.size() * sizeof(int));
    if (!f) { if (err) *err = "truncated file"; return nullptr; }
    // validate before anything reaches the device: the query kernels index with these values
    if (cs[0] != 0 || cs[C] != n) { if (err) *err = "corrupt file: cell_start bounds"; return nullptr; }
    for (long c = 0; c < C; ++c)
        if (cs[c + 1] < cs[c]) { if (err) *err = "corrupt file: cell_start not monotone"; return nullptr; }
    std::vector<unsigned> perm(n);
    std::vector<unsigned char> seen(n, 0);
    for (int i = 0; i < n; ++i) {
        unsigned u;
        std::memcpy(&u, &s[i].w, 4);
        if (u >= (unsigned)n || seen[u]) { if (err) *err = "corrupt file: ids are not a permutation"; return nullptr; }
        seen[u] = 1;
        perm[i] = u;
    }
    for (int a = 0; a < 3; ++a)
        if (g.dims[a] != hdr[2 + a]) { if (err) *err = "corrupt file: geometry / dims mismatch"; return nullptr; }
    EngineConfig c = cfg;
    if (c.k <= 0) c.k = hdr[5];
    Engine* e = new Engine(c);
    const int dims[3] = {hdr[2], hdr[3], hdr[4]};
    const int xs = v2 ? std::max(1, std::min(4, (hdr[11] >> kPlanXsubShift) & 15)) : 1;
    if (e->allocate(n, dims, false, xs) != KN_OK) { if (err) *err = e->error(); delete e; return nullptr; }
    if (v2 && (hdr[11] & kPlanValid) && c.k == hdr[5]) {
        // same K: restore the saved plan (refined grids keep the target density's LDS plan);
        // a plan the device cannot launch (corrupt / hostile file) is rejected here, not at the
        // first query launch
        int tile[3];
        for (int a = 0; a < 3; ++a) tile[a] = hdr[6 + a];
        const bool sane = tile[0] >= 1 && tile[1] >= 1 && tile[2] >= 1 && tile[0] <= 64 && tile[1] <= 64 &&
                          tile[2] <= 64 && hdr[9] >= 1 && hdr[9] <= 16 && hdr[10] >= 64 && hdr[10] <= 8192;
        if (!sane || query_lds_bytes(tile, hdr[9], hdr[10], xs) > kMaxLdsBytes) {
            if (err) *err = "corrupt file: query plan exceeds the device's LDS";
            delete e;
            return nullptr;
        }
        for (int a = 0; a < 3; ++a) e->ap_.tile[a] = tile[a];
        e->ap_.halo = hdr[9];
        e->ap_.lds_capacity = hdr[10];
        e->ap_.lds_bytes = query_lds_bytes(e->ap_.tile, e->ap_.halo, e->ap_.lds_capacity, xs);
    }
    // the refined state travels with the grid: algo auto serves a refined grid with the tree
    e->refined_ = v2 && (hdr[11] & kPlanRefined);
    e->use_tree_ = c.use_tiles && (c.algo == 2 || (c.algo == 0 && e->refined_)) && tree_supports(e->ap_.dims);
    bool ok = hipMemcpy(e->geom_, &g, sizeof(g), hipMemcpyHostToDevice) == hipSuccess &&
              (n == 0 || hipMemcpy(e->sorted_, s.data(), (size_t)n * sizeof(float4), hipMemcpyHostToDevice) == hipSuccess) &&
              (n == 0 || hipMemcpy(e->perm_, perm.data(), (size_t)n * sizeof(unsigned), hipMemcpyHostToDevice) == hipSuccess) &&
              hipMemcpy(e->cell_start_, cs.data(), (C + 1) * sizeof(int), hipMemcpyHostToDevice) == hipSuccess;
    if (!ok) { if (err) *err = "upload failed"; delete e; return nullptr; }
    e->built_ = true;
    return e;
}

}  // namespace kn
