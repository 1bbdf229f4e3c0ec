// engine.hpp -- single-GPU host runtime (replaces reference knearests.cu:205-466).
//
// * One device arena sized up front (reference allocates 9 buffers with an over-allocation
//   bug, knearests.cu:329-335 / defect D3).
// * Stream-ordered, allocation-free build + solve; both can be captured once into a hipGraph
//   and replayed (run_graph), which removes the per-launch host overhead of the ~8 kernels.
// * Errors are returned as kn_status + message, never exit() (reference defect D7).
#pragma once

#include <unordered_map>

#include <hip/hip_runtime.h>

#include <string>
#include <vector>

#include "knearests.h"
#include "kn/kernels.h"
#include "kn/tree.h"
#include "pipeline.hpp"

namespace kn {

struct EngineConfig {
    int k = KN_DEFAULT_K;
    float points_per_cell = 0.f;
    int tile[3] = {0, 0, 0};
    int halo = 0;
    int deterministic = 1;
    int device = 0;
    int verbose = 0;
    int use_tiles = 1;
    int with_distances = 1;
    int adaptive = 1;  // refine the grid when cells are over-occupied (clusters, surfaces)
    int algo = 0;      // query structure: 0 auto (tree when the adaptive grid was refined), 1 grid, 2 tree
};

class Engine {
public:
    explicit Engine(const EngineConfig& cfg);
    ~Engine();
    Engine(const Engine&) = delete;
    Engine& operator=(const Engine&) = delete;

    // Upload host points (N x 3 floats) and build the grid.
    kn_status prepare_host(const float* pts, int n);
    // Build from device points already resident (N x 3 floats). The engine keeps a copy.
    kn_status prepare_device(const float* d_pts, int n);
    // Copy device points into the arena WITHOUT building (for graph replay: the captured graph
    // rebuilds the grid itself). Re-plans (and drops the graph) only when n changes.
    kn_status upload_device(const float* d_pts, int n);
    kn_status solve();
    // Queries [first, first + count) only, into caller device buffers (count x K; d_dist may be
    // null): batched solves of clouds whose whole N x K result does not fit on the device.
    kn_status solve_range(int first, int count, unsigned* d_idx, float* d_dist);
    // Grow-only device scratch owned by the engine (kn_solve_range's batch buffers): a batched
    // solve allocates once, at its first (largest-so-far) batch, not per batch. nullptr on failure.
    void* scratch(size_t bytes);
    size_t scratch_allocations() const { return scratch_allocs_; }
    kn_status set_k(int k);
    // Capture build+solve into a graph once, then replay it `iters` times (bench path).
    kn_status run_graph(int iters, float* ms_per_iter);
    // Enqueue `iters` graph replays without waiting (capturing on first use); sync() waits.
    kn_status launch_graph(int iters);
    // Enqueue `iters` PIPELINED steps: two grid sets (and tree buffers on the tree path), the
    // build of step i+1 runs on a second stream while step i queries (a stream of clouds: each
    // step still bins and queries the whole cloud). sync() waits; results are the last step's.
    // unroll >= 2 (even): groups of `unroll` steps per graph (pipeline.hpp); < 0: KN_PIPE_UNROLL.
    // The pipeline stays primed between calls (the next step's build is already enqueued).
    kn_status launch_pipelined(int iters, int unroll = -1);
    // A stream of distinct clouds (n points each, device pointers): the step's cloud is copied
    // into the free grid set's input on the build stream, then binned and queried; `d_next`
    // (may be null) is the next step's cloud, binned now, while this step queries. The results
    // (original space) and the grid are this step's until the next call; sync() waits.
    kn_status stream_step(const float* d_pts, const float* d_next);
    // A batch of m distinct clouds of n points each (device pointers; the reference's repeated
    // kn_prepare + kn_solve on new points, knearests.cu:235-392): step j bins d_in[j] and writes its
    // original-space rows to d_idx[j] (n x K) and d_dist[j] (n x K, may be null). Steps run through
    // graphs of up to kBatchMax steps, captured once per batch length: each replays its steps'
    // copy-in + build on the build stream and queries on the main stream, step j+1's build under
    // step j's queries (as the resident unrolled pipeline); the steps' pointers come from a device
    // table written by a one-block kernel before each launch. Asynchronous (sync() waits). The
    // engine's own result buffers are not written (results() after a batch is an error); the
    // grid of the last step stays (stats, stored-space views of the last cloud).
    static constexpr int kBatchMax = kPtrTableMax / 3;
    kn_status stream_batch(int m, const float* const* d_in, unsigned* const* d_idx, float* const* d_dist);
    // stream_batch mode: 0 eager batch pipeline, 1 captured batch graphs, -1 KN_BATCH_MODE (default eager)
    void set_batch_mode(int mode) { batch_mode_ = mode; }
    // Shape of the resident / batch pipeline for THIS engine (-1: the process-wide KN_PIPE_QSTREAMS /
    // KN_PIPE_SETS defaults, read once): query streams 1 or 2, grid sets 2 or 3. A change drops a
    // pipeline already built (its graphs and extra grid sets); tests use it to cover the unrolled
    // one-query-stream path in-process.
    kn_status set_pipeline_shape(int query_streams, int sets);
    kn_status sync();  // both streams
    // Device-to-device copy of the original-space results into caller buffers.
    kn_status copy_results(unsigned* d_idx, float* d_dist);
    kn_status counters(unsigned out[kNumCounters]);

    // Host copies (caller frees with free()).
    float* get_points_sorted();            // N x 3
    unsigned* get_permutation();
    unsigned* get_knearests_stored();      // N x K stored space (reference semantics)
    float* get_distances_stored();
    unsigned* get_neighbors_original();    // N x K original space
    float* get_distances_original();
    kn_status stats(kn_stats* out, std::vector<int>* hist);

    kn_status save(const char* path);
    static Engine* load(const char* path, const EngineConfig& cfg, std::string* err);

    const std::string& error() const { return err_; }
    int n() const { return n_; }
    int k() const { return cfg_.k; }
    const int* dims() const { return ap_.dims; }
    int num_cells() const { return C_; }
    float ms_build() const { return ms_build_; }
    float ms_solve() const { return ms_solve_; }
    bool uses_tree() const { return use_tree_; }
    int tree_leaves();  // leaf count of the last tree step (diagnostics: one host sync)

    // raw device pointers (C API struct fields)
    float4* d_sorted() const { return sorted_; }
    int* d_cell_start() const { return cell_start_; }
    unsigned* d_perm() const { return perm_; }
    unsigned* d_knn_stored();                    // converts on first use after a solve
    unsigned* d_knn_stored_if_valid() const { return stored_valid_ ? knn_stored_ : nullptr; }
    float* d_points3();                          // stored-order float3 view (reference field)

private:
    kn_status fail(kn_status s, const std::string& msg);
    kn_status check(hipError_t e, const char* what);
    kn_status allocate(int n, const int* dims_override = nullptr, bool refined = false, int xsub_override = 0);
    kn_status prepare_from(const float* src, int n, hipMemcpyKind kind);
    kn_status occupancy(double* w);
    kn_status ensure_outputs();
    // serial: alone on the device (BuildBuffers::serial); the pipeline stages pass false
    kn_status build_async(bool fused_step = false, bool serial = true);
    kn_status query_async(bool fused_step = false);
    // Morton-leaf tree over the built grid's points + its query (stream-ordered, capturable)
    kn_status tree_query();
    kn_status tree_build_async();  // leaves + node boxes of the current grid (stream-ordered)
    kn_status tree_query_async();  // the tree query over them
    kn_status ensure_tree();
    QueryBuffers query_buffers() const;
    BuildBuffers build_buffers() const;
    void release();
    // pipelined steps (pipeline.hpp): two or three grid sets, set 0 carved from arena_, set 1 from
    // arena2_, set 2 from arena3_ (same carve, input points included); the members above always
    // view the LIVE set (the one the last step queried), so getters, stats and serial steps see the
    // last step's grid
    struct GridSet {
        float* points; unsigned* bbox; GridGeom* geom; int* cell_count; int* cell_scan; int* block_sums;
        int* cell_start; int2* cell_rank; float4* bin_tmp; float4* sorted; unsigned* perm; unsigned* fallback;
        unsigned* counters; unsigned long long* occ;
        void* tree_ws;
        void* tree_nodes;
        unsigned* out_idx;  // per-set results (dmalloc'd): step i's rows stay while step i+1 queries
        float* out_dist;
    };
    GridSet members() const;
    void view_set(int s);  // members <- set_[s]
    kn_status ensure_pipeline();
    kn_status stage_build(int s, hipStream_t st);
    kn_status stage_query(int s, hipStream_t st);
    kn_status stage_exact(int s, hipStream_t st);  // the fallback list's exact finish (epilogue)
    // keep_grid: the live grid (maybe in arena2_) must survive into arena_ (set_k keeps solving it)
    void drop_pipeline(bool keep_grid = false);
    int qstreams_cfg_ = -1, sets_cfg_ = -1;  // set_pipeline_shape (-1: environment defaults)
    GridSet set_[3]{};
    int nsets_ = 2;            // grid sets of the resident pipeline (3 with two query streams)
    kn_status carve_set(int s, char* base);
    int live_ = 0;             // set the members view
    int graph_set_ = -1;       // set graph_ was captured against
    bool other_stale_ = true;  // another set's input differs from the live input
    bool stream_mode_ = false; // the last pipelined steps were stream_step()s (distinct clouds)
    char* arena2_ = nullptr;
    char* arena3_ = nullptr;
    hipStream_t bstream_ = nullptr;
    hipEvent_t pev_[4] = {nullptr, nullptr, nullptr, nullptr};  // the side stream's pooled events
    Pipeline pipe_;
    // batched streams (stream_batch): device pointer table {in, idx, dist} x kBatchMax, graphs by
    // batch length, capture events; out_ref_slot_ >= 0 while a batch step is captured (its
    // query / exact / tree launches read their output pointers from the table slot)
    void** tab_ = nullptr;
    std::unordered_map<int, hipGraphExec_t> bgraphs_;
    std::vector<hipEvent_t> bev_;
    hipStream_t qstream2_ = nullptr;  // batch graphs: odd steps' queries (KN_BATCH_QSTREAMS=2)
    // eager batch pipeline (stream_batch default): the same stages over the same grid sets and
    // streams as pipe_, enqueued per step; a step's outputs are the caller's buffers of set s
    Pipeline bpipe_;
    unsigned* bout_idx_[3] = {nullptr, nullptr, nullptr};
    float* bout_dist_[3] = {nullptr, nullptr, nullptr};
    int out_ovr_set_ = -1;  // >= 0 while a batch stage of that set is enqueued
    int batch_mode_ = -1;
    kn_status stream_batch_eager(int m, const float* const* d_in, unsigned* const* d_idx, float* const* d_dist);
    int out_ref_slot_ = -1;
    kn_status batch_graph(int L, hipGraphExec_t* out);
    void drop_batch();
    size_t arena_used_ = 0;  // bytes of arena_ carved by allocate() (arena2_ has the same carve)

    EngineConfig cfg_;
    AutoParams ap_{};
    std::string err_;
    hipStream_t stream_ = nullptr;
    hipEvent_t ev_[4] = {nullptr, nullptr, nullptr, nullptr};
    hipGraphExec_t graph_ = nullptr;
    int n_ = 0, C_ = 0;
    size_t arena_bytes_ = 0;
    // result / tree buffers through the process-wide device block cache (hostio.hpp)
    std::unordered_map<void*, size_t> dsize_;
    void* scratch_ = nullptr;
    size_t scratch_bytes_ = 0, scratch_allocs_ = 0;
    hipError_t dmalloc(void** p, size_t bytes);
    template <class T>
    hipError_t dmalloc(T** p, size_t bytes) { return dmalloc(reinterpret_cast<void**>(p), bytes); }
    void dfree(void* p);
    char* arena_ = nullptr;
    float* points_ = nullptr;
    unsigned* bbox_ = nullptr;
    GridGeom* geom_ = nullptr;
    int* cell_count_ = nullptr;
    int* cell_scan_ = nullptr;
    int* block_sums_ = nullptr;
    int* cell_start_ = nullptr;
    int2* cell_rank_ = nullptr;
    float4* bin_tmp_ = nullptr;
    float4* sorted_ = nullptr;
    unsigned* perm_ = nullptr;
    unsigned* fallback_ = nullptr;
    unsigned* counters_ = nullptr;
    unsigned long long* occ_ = nullptr;
    // outputs (re-allocated when K changes)
    unsigned* out_idx_ = nullptr;
    float* out_dist_ = nullptr;
    unsigned* inv_perm_ = nullptr;
    unsigned* knn_stored_ = nullptr;
    float* points3_ = nullptr;  // stored-order float3 copy of sorted_ (reference d_stored_points)
    bool points3_valid_ = false;
    bool built_ = false, solved_ = false, stored_valid_ = false;
    unsigned last_fallback_ = ~0u;  // fallback-list length of the last eager solve (~0: unknown)
    unsigned last_coop_ = 0;        // cooperative re-rank finishes of the last eager solve
    bool use_tree_ = false;         // chosen at prepare (EngineConfig::algo)
    bool refined_ = false;          // the occupancy-adaptive grid was refined (saved with the grid)
    void* tree_ws_ = nullptr;
    size_t tree_ws_bytes_ = 0;
    void* tree_nodes_ = nullptr;
    size_t tree_nodes_bytes_ = 0;
    float ms_build_ = 0.f, ms_solve_ = 0.f;
};

}  // namespace kn
