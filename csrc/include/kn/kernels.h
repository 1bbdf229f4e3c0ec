// kn/kernels.h -- host-side launchers for the gfx950 HIP kernels.
//
// Every launcher is stream-ordered, allocation-free and synchronisation-free, so the
// whole build+solve pipeline can be captured into a hipGraph (engine.cpp) or run on the
// current PyTorch stream (torch/bindings.cpp). Buffers are owned by the caller.
//
// Pipeline (replaces reference knearests.cu:152-201 kn_firstbuild and :348-392 kn_solve):
//   bbox -> geom -> count(+rank) -> scan(blocks, top) -> scatter(+cell_start) [-> cell sort]
//   -> knn_tile (LDS-staged, certified) -> knn_fallback (exact ring walk for the rest)
#pragma once

#include <hip/hip_runtime_api.h>
#include <math.h>
#include <stddef.h>
#include <stdint.h>

namespace kn {

// Device-resident grid geometry. Written by geom_kernel (or geom_from_box) so the host
// never has to read the data-dependent bounding box back (graph-capturable pipeline).
struct GridGeom {
    float origin[3];    // world position of cell (0,0,0)'s lower corner
    float cell[3];      // cell edge per axis
    float inv_cell[3];  // 1 / cell
    float eps;          // conservative slack for box-distance bounds (world units)
    int dims[3];
    int pad;
};

// Box inside which the local point set is complete (all points of the global cloud that lie
// in it are present). Single GPU: infinite. Multi-GPU: the rank's owned box grown by its halo.
// Position-dependent halo (round 4, kn/route.h): points within the wide zone (distance <= w to
// a face of the global domain) were routed with the edge width h_e, the others with the
// interior width h_i <= h_e. lo / hi are the own box grown by h_i; a face's margin grows by
// `wide` = h_e - h_i when the query's distance to the domain plus that margin stays below
// `zlim` (w minus a rounding slack): every point of the ball it certifies then lies in the wide
// zone. wide = 0: one width (single GPU: all zero, the margins are infinite anyway).
// Density-adaptive halo (round 4, kn/route.h): a width field over a G^3 cell grid of the global
// domain. Every routing, splat and certification kernel maps a point to its cell with this one
// function, so the three agree bit for bit.
struct FieldGeom {
    float lo[3];
    float inv[3];  // G / domain extent
    int g;         // cells per axis (0: no field)
    float rstep;   // radius certified per neighbourhood ring: level m covers r <= m * rstep
};
__host__ __device__ inline FieldGeom field_geom(const float lo[3], const float hi[3], int g) {
    FieldGeom f{};
    float inv_max = 0.f;
    for (int a = 0; a < 3; ++a) {
        f.lo[a] = lo[a];
        const float ext = hi[a] - lo[a] > 1e-30f ? hi[a] - lo[a] : 1e-30f;
        f.inv[a] = (float)g / ext;
        inv_max = f.inv[a] > inv_max ? f.inv[a] : inv_max;
    }
    f.g = g;
    // 0.2 % below a cell: a point within m * rstep of a query lies within m cells of it on every
    // axis despite the rounding of the cell coordinates
    f.rstep = g > 0 ? 0.998f / inv_max : 0.f;
    return f;
}
__host__ __device__ inline int field_axis(const FieldGeom& f, float v, int a) {
    int i = (int)floorf((v - f.lo[a]) * f.inv[a]);
    i = i < 0 ? 0 : i;
    return i > f.g - 1 ? f.g - 1 : i;
}
__host__ __device__ inline int field_cell(const FieldGeom& f, float x, float y, float z) {
    return field_axis(f, x, 0) + f.g * (field_axis(f, y, 1) + f.g * field_axis(f, z, 2));
}
constexpr int kFieldLevels = 3;  // neighbourhood rings of the splat / certification

struct CompleteBox {
    float lo[3];
    float hi[3];
    float wide;
    float zlim;
    float dlo[3];
    float dhi[3];
    // density-adaptive halo: radius certified at each field cell (null: none). The own box
    // (lo / hi, no halo) certifies a query's ball inside it; cfield[cell] one that reaches out.
    const float* cfield;
    FieldGeom fg;
};

constexpr int kScanItems = 4096;  // elements per scan block (256 threads x 16)

// Bounding box: each of <= kBBoxBlocks blocks writes its 6 partial (lo, hi) encodings, the
// single-block finaliser reduces them -- no same-address atomics, no memset.
constexpr int kBBoxBlocks = 256;
constexpr int kBBoxWords = 6 * kBBoxBlocks;
int bbox_block_count(int n);
// partials[a * kBBoxBlocks + b]: a < 3: max of ~ord(min_a), a >= 3: max of ord(max_a) over
// block b's points (ord = order-preserving float -> uint). Blocks past bbox_block_count(n)
// are not written.
// zero_ints / n_zero: ints block 0 zeroes on the way (the bucketed build's bucket totals)
hipError_t launch_bbox_partials(const float* pts, int n, unsigned* partials, hipStream_t s, int* zero_ints = nullptr,
                                int n_zero = 0);

// Query counters (device, zeroed by every launch_query):
//  [0] queries sent to the exact kernel   [1] uncertified (multi-GPU: K-th leaves complete box)
//  [2] LDS-overflow (dense) tiles         [3] in-wave cooperative re-ranks / exact re-scans
//  [4] rows streamed (per wave)           [5] candidates streamed (per wave)
//  [6] insertion networks executed        [7] query chunks (waves x chunk iterations)
constexpr int kNumCounters = 8;

// QueryBuffers::flags
constexpr int kQueryFlagForceRescan = 1;  // exact re-scan for every query (tests)
constexpr int kQueryFlagStream = 2;       // staging-free stream kernel
constexpr int kQueryFlagTile = 4;         // LDS-staged tile kernel, row walk
constexpr int kQueryFlagLane = 8;         // LDS-staged tile kernel, lane walk (default; env KN_QUERY_ALGO)
// Second, wider exact re-rank window (query.hip kWin2): for point sets with many exactly equal
// distances (lattice-like / symmetric samplings), whose truncated keys run longer than the
// default window and would otherwise take the wave-serial cooperative sort. Costs ~3 % (900K
// K=16) to 15 % (100K) where it is not needed, so callers set it from the previous solve's
// counters[3] (cooperative finishes; kn::Engine: more than 1/64 of the queries).
constexpr int kQueryFlagWide = 16;

struct BuildBuffers {
    // inputs
    const float* points;      // N x 3 floats (AoS, 12-byte stride)
    int n;
    int dims[3];
    // scratch / outputs (caller-allocated)
    unsigned* bbox_words;     // kBBoxWords words of per-block partials (no zeroing needed)
    GridGeom* geom;           // 1
    int* cell_count;          // C      (zeroed by the launcher)
    int* cell_scan;           // C      block-local exclusive scan
    int* block_sums;          // ceil(C / kScanItems) + 1
    int* cell_start;          // C + 1  final exclusive scan, cell_start[C] = N
    int2* cell_rank;          // N      (cell, rank inside cell) -- atomic binning only
    float4* bin_tmp;          // N      bucketed binning scratch (may alias cell_rank)
    float4* sorted;           // N      {x, y, z, bits(original index)}
    unsigned* perm;           // N      perm[stored] = original index
    int deterministic;        // 1: sort each cell by original index
    // optional fixed domain (multi-GPU ranks): if use_box, bbox is not computed
    int use_box;
    float box_lo[3], box_hi[3];
    // optional: words (<= 64) the build zeroes on the device (the following query's counters,
    // so the step needs no memset node; then QueryBuffers::counters_zeroed = 1)
    unsigned* zero_words;
    int n_zero_words;
    // optional global-id mode (multi-GPU ranks, query.hip row_of): every stored point's w becomes
    // gids[local index] | 0x80000000 on non-owned points (local index >= n_owned); perm keeps the
    // local index. Fused into the bucket sort (non-deterministic bucketed build), else one extra pass.
    const int* gids;
    int n_owned;
    // points per bucketed-binning block (0: automatic, build.hip bin_plan)
    int bin_items;
    // launch context of the build (build.hip launch_build): 0 = pipelined (beside running query
    // kernels: 256-thread streaming blocks of ~16K points up to 4M points), 1 = serial (alone on the
    // device: 1024-thread blocks of 4096 points, one block per CU at 900K)
    int serial;
    // 1: a kernel earlier on the stream zeroed cell_scan[0, bin_totals_words(C)) (the bucketed
    // build's totals; DistPipeline's route_count): no memset node with a fixed box
    int totals_zeroed = 0;
};
// ints of cell_scan that hold the bucketed build's bucket totals at most (nbuckets <= 4096, <= C + 1)
inline int bin_totals_words(int num_cells) { return num_cells + 1 < 4096 ? num_cells + 1 : 4096; }

size_t scan_block_count(int num_cells);

// Bucketed binning (two-level counting sort, LDS atomics only): points are first split into
// buckets of 2^shift consecutive cells by `nblocks` streaming blocks, then one workgroup per
// bucket counts, scans and places its points. Used when the (bucket x block) count table fits
// in the C+1-entry cell_count buffer; otherwise the build falls back to global-atomic binning.
struct BinPlan {
    int shift;     // log2(cells per bucket), 8..14
    int nbuckets;  // ceil(C / 2^shift) <= 4096
    int nblocks;   // streaming blocks
    int per_block; // points per streaming block (multiple of 256)
};
bool bin_plan(int n, int num_cells, BinPlan* out, int items = 0);
hipError_t launch_build(const BuildBuffers& b, hipStream_t stream);

// Batched streams of clouds (Engine::stream_batch): write `count` (<= kPtrTableMax) pointers into
// the device table `dst` (kernel arguments carry them: the host array may go at once), and copy
// n floats from the buffer whose address sits in the device slot `src_ref`.
constexpr int kPtrTableMax = 96;
hipError_t launch_set_ptr_table(void* const* ptrs, int count, void** dst, hipStream_t stream);
hipError_t launch_copy_from_ref(const float* const* src_ref, float* dst, size_t n, hipStream_t stream);
// The deterministic in-cell order (by original index) of launch_build, alone (rank of each point
// in its cell, O(N x mean cell occupancy) parallel work; tmp: N float4 scratch). The occupancy-
// adaptive build bins its probe grids without it (a clustered cloud's first grid has cells of
// thousands of points) and orders the final grid once.
hipError_t launch_cell_sort(const int* cell_start, const GridGeom* geom, int n, float4* sorted, unsigned* perm,
                            float4* tmp, hipStream_t stream);

// A distributed step's steady-state check run by the last workgroup of the exact finish kernel
// (deferred mode, DistPipeline::stage_query): the arguments of steady_flag_partials_kernel
// (route.hip, kn/step_flag.h) plus the max-accumulator and the kernel's workgroup ticket (zeroed
// at allocation; the last workgroup resets it).
struct StepFlagJob {
    const unsigned* partials;  // route_count's bbox partials: 6 x stride words
    int nb, stride, n;         // partial blocks, their stride, the share's true size
    const double* planned;     // planned {lo, hi, n} meta (8 doubles)
    const int* totals;         // this step's send counts ...
    const int* ptotals;        // ... and the planned ones
    int nt;
    int* flag;                 // the set's flag word
    int* pending;              // atomicMax accumulator of the launch's steps
    unsigned* ticket;          // workgroup ticket (self-resetting)
};

struct QueryBuffers {
    const float4* sorted;
    const int* cell_start;
    const unsigned* perm;
    const GridGeom* geom;
    int n;                    // number of stored points
    int dims[3];
    int k;
    int n_queries;            // points with original index < n_queries are queries
    int q_lo;                 // ... and >= q_lo (query ranges; out row = original index - q_lo)
    const unsigned* id_map;   // optional: output id = id_map[original index]
    const unsigned* row_of;   // optional: global-id mode -- each stored point's w is its global id
                              // (| 0x80000000 on non-query halo points) and a query's output row
                              // is row_of[stored index]; id_map is then unused
    CompleteBox complete;
    unsigned* out_idx;        // n_queries x k   (row = original index), UINT_MAX = empty
    float* out_dist;          // optional n_queries x k squared distances
    // optional: device slots holding the output pointers, read by the kernels at launch time
    // instead of out_idx / out_dist (a graph captured once writes each replay's rows where the
    // slot points: batched streams of clouds, Engine::stream_batch)
    unsigned* const* out_idx_ref = nullptr;
    float* const* out_dist_ref = nullptr;
    unsigned* fallback_list;  // n   (stored indices of queries needing the exact path)
    unsigned* counters;       // kNumCounters words, see below
    unsigned* uncert_list;    // optional n_queries: original indices of uncertified queries
    int tile[3];
    int halo;                 // halo rings of cells in y and z
    int xsub = 1;             // x sub-cells per y/z cell width (AutoParams::xsub): x halo = halo * xsub
    int lds_capacity;         // points staged per workgroup (power of two)
    int use_tiles;            // 0: exact ring walk for every query (debug / reference path)
    int flags;                // kQueryFlag* below
    int counters_zeroed;      // 1: the preceding build zeroed `counters` (no memset here)
    int exact_grid;           // workgroups of the fallback launch; 0 = default (sized for long
                              // lists). The engine passes a small grid when the previous solve's
                              // list was short (the launch then costs ~3 us less).
    // 0: the tile kernel then the exact finish of its fallback list; 1: the tile kernel only;
    // 2: the exact finish only (after a mode-1 launch on the same counters / list: pipelined
    // steps run it on the build stream, off the query stream's critical path)
    int exact_mode;
    // optional (exact modes 0 and 2): DEVICE pointer to the step check the exact kernel's last
    // workgroup runs
    const StepFlagJob* step_flag = nullptr;
};

hipError_t launch_query(const QueryBuffers& q, hipStream_t stream);
// Complete-box certification of `rows` finished rows (row r = local point r of `pts`, N x 3):
// uncertified rows are appended to uncert_list and counted in counters[1].
hipError_t launch_certify_rows(const float* pts, int rows, int k, const float* out_dist, const CompleteBox& cb,
                               const GridGeom* geom, unsigned* counters, unsigned* uncert_list, hipStream_t stream);
// Exact K nearest of EXTERNAL points {x, y, z, bits(global id)} among the grid's points (multi-GPU
// query forwarding): row t of q.out_idx / q.out_dist; a point with the query's global id is
// skipped (self). Uses q.sorted / cell_start / geom / dims / k / row_of / counters.
hipError_t launch_query_external(const QueryBuffers& q, const float4* ext, int n_ext, hipStream_t stream);
// Forwarding slots of a sync-free multi-GPU step (kn/route.h launch_fwd_pack): n_slots queries,
// 2 float4 each ({x, y, z, bits(gid)}, {origin K-th d2, -, -, -}); gid 0xFFFFFFFF = empty. Rows
// t of out_idx / out_dist (global ids, ascending (d2, id), <= K points within the seed) for every
// filled slot; empty slots' rows are left untouched.
hipError_t launch_query_external_slots(const QueryBuffers& q, const float4* slots, int n_slots, hipStream_t s);

// out_sorted[i*k + j] = inv(out_orig[perm[i]*k + j]) : reference (stored-space) view.
hipError_t launch_to_stored_space(const unsigned* out_orig, const unsigned* perm,
                                  const unsigned* inv_perm, int n, int k,
                                  unsigned* out_sorted, const float* dist_orig,
                                  float* dist_sorted, hipStream_t stream);
hipError_t launch_invert_perm(const unsigned* perm, int n, unsigned* inv, hipStream_t stream);
// xyz[3i..3i+2] = sorted[i].xyz : the reference's float3 stored-point view (kn_problem field).
hipError_t launch_sorted_xyz(const float4* sorted, int n, float* xyz, hipStream_t stream);

// Grid-occupancy statistics (reference kn_print_stats, knearests.cu:440-466):
// out[0]=min, out[1]=max, out[2]=empty cells, out[3..3+hist_len) = histogram of counts.
// Occupancy-adaptive grid: out[0] = sum over cells of count^2 (= N x the mean occupancy of a
// point's own cell; a Poisson(l) grid gives N (1 + l)). Clustered clouds and points on surfaces
// give far more; refine_dims then proposes finer dims (see query.hip).
hipError_t launch_cell_occupancy(const int* cell_start, int num_cells, unsigned long long* out,
                                 hipStream_t stream);
// Finer dims for an over-occupied grid (w = sum count^2 / N), or false if the grid is fine.
// The refined dims are isotropic (their grid has xsub 1).
bool refine_dims(const int dims[3], double w, int k, float points_per_cell, int n, int out[3], int xsub = 1);
float default_points_per_cell(int k);
hipError_t launch_cell_stats(const int* cell_start, int num_cells, int* out, int hist_len,
                             hipStream_t stream);

// Heuristics shared by the engine, the torch binding and the CLI.
// xsub: the grid's cells are xsub times finer along x (the axis of the contiguous cell rows) than
// along y and z; dims[0] and tile[0] count x sub-cells, halo counts y/z cells (x halo = halo *
// xsub sub-cells). A lane's row x-range is then cut at sub-cell granularity for the same row
// count (query.hip, lane walk).
struct AutoParams {
    int dims[3];
    int tile[3];
    int halo;
    int lds_capacity;
    size_t lds_bytes;
    int xsub = 1;
};
AutoParams auto_params(int n, int k, float points_per_cell, const int* tile_hint, int halo_hint,
                       const float* extent /* nullable: cubic grid */, int xsub_hint = 0 /* 0 = auto */);
// points staged per query workgroup of the plan at `ppc` points per (y/z-sized) cell
double staged_points(const AutoParams& p, double ppc);
// Checked builds only (KN_CHECKED): first out-of-bounds report of each kernel file
// {site code, index, limit, index high word}; all 0xFFFFFFFF in release builds.
hipError_t debug_words_build(unsigned out[4], bool reset);
hipError_t debug_words_query(unsigned out[4], bool reset);
// -DKN_PHASES=1 builds: wave cycles of knn_tile_kernel per phase, summed over waves:
// {stage (+ the kernel tail), chunk setup, scan (hot loop), re-rank, certify, chunks, waves, -}.
// Other builds: hipErrorNotSupported.
hipError_t debug_phase_cycles(unsigned long long out[8], bool reset);

size_t query_lds_bytes(const int tile[3], int halo, int lds_capacity, int xsub = 1);
int lds_capacity_for(double staged_points);

}  // namespace kn
