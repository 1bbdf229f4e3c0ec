// kn/tree.h -- Morton-leaf tree kNN path (csrc/kernels/tree.hip).
//
// The uniform grid (kn/kernels.h) is the fastest structure for near-uniform clouds, but one cell
// size cannot serve a cloud whose density varies by 10^4 (Gaussian clusters over a sparse
// background, scans): dense cells hold hundreds of points, sparse queries need many rings, tiles
// overflow the LDS budget. The tree path adapts to any density:
//
//   build:  the grid's points (already grouped by cell) in the Morton order of their CELLS,
//           without sorting: 8^3-cell bricks numbered by the Morton code of their brick
//           coordinates, one exclusive scan of the brick counts, one workgroup per brick scans
//           its 512 cells in Morton order and copies their point runs -> leaves = the maximal
//           binary-prefix (radix) nodes of <= 32 points (runs of one cell chunked) -> leaf
//           boxes (wave DPP reductions) -> implicit complete binary tree of boxes over P = pow2
//           >= n leaf slots (heap index, root 1, leaf l = node P + l; nodes past the leaf count
//           are never written nor entered), reduced bottom-up 6 levels per launch in LDS.
//           Every launch is sized from n and the grid dims alone and the leaf count stays on
//           the device: the whole tree step is stream-ordered and graph-capturable.
//   query:  one wave per 64 consecutive points of the Morton order (lanes = queries).
//           Wave-uniform near-first traversal
//           (a node is entered when ANY lane's box distance is within its own K-th bound);
//           every visited leaf is staged once in the wave's LDS slice and streamed to all
//           lanes (broadcast reads) into the same packed-key / v_med3_u32 register top-K as the
//           grid kernels, key slot = (visit index, point in leaf). Exact re-rank of the kept
//           slots by (d2, id) and certification against the truncation floor; uncertified
//           queries (near-ties, > 256 visited leaves) go to a list finished by a wave-per-query
//           exact traversal with threshold compaction (same semantics as the grid's exact
//           kernel, so results are identical to the oracle's).
//
// Output format is that of launch_query: row = the point's original index (w field), ids are
// original indices (or id_map[...]).
#pragma once

#include <hip/hip_runtime_api.h>
#include <stddef.h>

#include "kn/kernels.h"

namespace kn {

// Leaves of <= 64 points (round 5; 32 before): half the traversal rounds for the latency-bound
// query waves, one 64-lane load per leaf visit. 900K, pipelined: clustered K=16 1.193 -> 1.096
// ms, surfaces 0.751 -> 0.744, clustered K=50 4.30 -> 3.78 (more waves pass the 128-leaf visit
// cap and finish in the exact kernel: 2,135 -> 8,145 queries); profiles/ab_r5_tree_leaf64.txt.
#ifndef KN_TREE_LEAF_BITS
#define KN_TREE_LEAF_BITS 6
#endif
constexpr int kTreeLeaf = 1 << KN_TREE_LEAF_BITS;  // points per leaf (at most)

// A tree: one workspace (carved by tree_view) plus a node buffer sized from n.
struct TreeView {
    float4* pts;          // n points in Morton order {x, y, z, w} (w copied from the input)
    unsigned* leaf_start; // L + 1 leaf boundaries (<= 64 points per leaf)
    unsigned* seg_start;  // scratch: segment boundaries between forced cuts
    unsigned* list;       // n: tree positions of queries for the exact finish
    float* thr;           // n: their distance bound
    unsigned* flag;       // n scratch
    unsigned* incl;       // n scratch
    unsigned long long* codes;  // n: the Morton code of each tree point's cell
    unsigned* vals;       // n: input (grid slot) index of each tree point
    unsigned* info;       // [0] = L after launch_tree_leaves (device; the query kernels read it)
    float4* tmp_pts;      // n: points in cell order (before the sub-cell order)
    unsigned* tmp_vals;   // n
    unsigned long long* cell_code;  // n: Morton code of each point's cell (brick code << 9 | in-brick code)
    uint2* cell_span;     // n: tree range [first, end) of each point's cell
    unsigned* bcount;     // padded brick space + 1: brick counts, scanned in place to bases
    unsigned* scan_sums;  // block sums of the device scans
    size_t nbricks_pad;   // 8^bb brick slots (bb = ceil(log2(max bricks per axis)))
    int nbricks[3];       // bricks per axis
    int dims[3];          // grid dims
    float4* nlo;          // 2P node boxes (lower corner; heap index, root 1, leaf l = node P + l)
    float4* nhi;          // 2P upper corners
    int n, P;             // points, P = next power of two >= n (leaf slots)
};

// dims: the grid's dims (host copy of GridGeom::dims)
size_t tree_workspace_bytes(int n, const int dims[3]);
// The Morton brick codes hold 10 bits of brick coordinate per axis (8 cells a brick): grids of at
// most 8,192 cells per axis. Larger grids stay on the grid path (callers check this).
constexpr int kTreeMaxAxisCells = 8192;
// The brick counts live in a cube of pow2(max bricks per axis)^3 slots (Morton order over the
// longest axis), so an elongated grid (8192 x 8 x 8 cells: 1024^3 slots, 4 GB) would cost far more
// than its cells. Bound the padded space itself: 2^24 slots (64 MB, e.g. 2048 x 8 x 8 or 2048^3
// cells); larger spaces stay on the grid path.
constexpr size_t kTreeMaxBrickSlots = (size_t)1 << 24;
inline size_t tree_brick_slots(const int dims[3]) {
    int m = 1;  // bricks along the longest axis
    for (int a = 0; a < 3; ++a) {
        const int b = (dims[a] + 7) / 8;
        if (b > m) m = b;
    }
    size_t side = 1;
    while ((int)side < m) side <<= 1;
    return side * side * side;
}
inline bool tree_supports(const int dims[3]) {
    return dims[0] <= kTreeMaxAxisCells && dims[1] <= kTreeMaxAxisCells && dims[2] <= kTreeMaxAxisCells &&
           tree_brick_slots(dims) <= kTreeMaxBrickSlots;
}
TreeView tree_view(void* ws, int n, const int dims[3]);
// Phase 1 (stream-ordered, no host sync): the grid's sorted points in the Morton order of their
// cells, leaf boundaries; the leaf count lands in t.info[0] on the device.
hipError_t launch_tree_leaves(const float4* in, const int* cell_start, const GridGeom* geom, const TreeView& t,
                              hipStream_t s);
size_t tree_node_bytes(int n);
void tree_attach_nodes(TreeView& t, void* nodes);
// Phase 2: leaf boxes and the implicit tree's node boxes.
hipError_t launch_tree_nodes(const TreeView& t, hipStream_t s);
// Diagnostics: the leaf count (one host sync).
hipError_t tree_leaf_count(const TreeView& t, unsigned* L, hipStream_t s);

struct TreeQuery {
    int k;
    int n_queries;            // points whose w < n_queries are queries
    const unsigned* id_map;   // optional output id map (as QueryBuffers::id_map)
    const unsigned* row_of;   // optional global-id mode (as QueryBuffers::row_of: w = global id |
                              // halo bit, output row = row_of[stored index]; multi-GPU ranks)
    unsigned* out_idx;        // n_queries x k, row = original index
    float* out_dist;          // optional
    unsigned* const* out_idx_ref = nullptr;  // optional pointer slots (QueryBuffers::out_idx_ref)
    float* const* out_dist_ref = nullptr;
    unsigned* counters;       // kNumCounters words: [0] exact-finish queries, [2] waves over the
                              // visit cap, [3] queries whose re-rank stayed unsorted, [4] queries
                              // whose K-th is not below the truncation floor, [5] leaves
                              // visited, [6] insertion networks (checked builds), [7] waves
    int flags;                // 1: every query takes the exact finish (tests)
};
hipError_t launch_tree_query(const TreeView& t, const TreeQuery& q, hipStream_t s);
hipError_t debug_words_tree(unsigned out[4], bool reset);

}  // namespace kn
