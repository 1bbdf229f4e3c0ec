// kn/route.h -- multi-GPU routing launchers (csrc/kernels/route.hip).
//
// One solve of the distributed engine moves every point once: to its owner rank and, as a
// halo copy, to each rank whose box is within h. The launchers below build the send buffer
// of that single all-to-all-v and unpack what arrives. Stream-ordered, allocation-free.
#pragma once

#include <hip/hip_runtime_api.h>
#include <stddef.h>

#include "kn/kernels.h"

namespace kn {

constexpr int kRouteMaxWorld = 64;
#ifndef KN_ROUTE_ITEMS
#define KN_ROUTE_ITEMS 1024
#endif
constexpr int kRouteItems = KN_ROUTE_ITEMS;  // points per routing block

struct RouteParams {
    float lo[3];    // global domain lower corner
    float ext[3];   // domain extent (hi - lo, clamped > 0)
    float g[3];     // decomposition grid (px, py, pz) as floats
    int grid[3];
    int world;      // px * py * pz <= kRouteMaxWorld
    float h2;       // squared halo send width (edge width h_e: points in the wide zone)
    // Position-dependent halo: a point farther than wz from every face of the global domain is
    // sent with the interior width (hi2 <= h2) -- an interior query's K-th ball is a whole ball,
    // a query near a domain face sees a truncated one (x 4^(1/3) at an edge). hi2 == h2: one width.
    float hi2;
    float wz;
    float dom_hi[3];  // global domain upper corner (lower: lo)
    int pad0;         // explicit padding (plans are compared byte for byte): always 0
    // Density-adaptive halo (field != null): a point in field cell c is sent to every rank whose
    // box is within field[c] (+ fslack) -- the widths splatted from the previous full step's
    // measured K-th distances (launch_field_splat); h2 / hi2 / wz are then unused.
    const float* field;
    FieldGeom fg;
    float fslack;
    int id_offset;  // global id of this rank's first point (route_scatter with ids == nullptr)
    float box_lo[kRouteMaxWorld][3];  // rank boxes (same formula as SpatialDecomposition.rank_box)
    float box_hi[kRouteMaxWorld][3];
    // Count-balanced decomposition (balanced = 1): the owner comes from kd splits instead of the
    // equal-volume grid formula -- x splits, then y splits per x slab, then z splits per (x, y)
    // column, each set chosen at global quantiles (SpatialDecomposition.splits, the same layout):
    //   xs[0..px]                       (xs[0] = lo, xs[px] = hi)
    //   ys[ix * (py + 1) + j], j <= py
    //   zs[(ix + px * iy) * (pz + 1) + j], j <= pz
    int balanced;
    float xs[kRouteMaxWorld + 1];
    float ys[2 * kRouteMaxWorld];
    float zs[2 * kRouteMaxWorld];
};
static_assert(sizeof(RouteParams) == offsetof(RouteParams, zs) + sizeof(float) * 2 * kRouteMaxWorld,
              "RouteParams has hidden tail padding");
static_assert(offsetof(RouteParams, field) == offsetof(RouteParams, pad0) + sizeof(int), "RouteParams padding");
// floats in a splits array for decomposition grid g (kd layout above)
inline int route_split_count(const int g[3]) { return (g[0] + 1) + g[0] * (g[1] + 1) + g[0] * g[1] * (g[2] + 1); }

// Device-side plan header (doubles) written by launch_route_plan for the host's one sync:
constexpr int kPlanHdr = 24;
// [0..2] global lo  [3..5] global hi  [6] h (certification halo, edge width h_e)  [7] h_send
// [8] n_total  [9] id offset of this rank  [10] 1 if the halo covers the whole domain
// [11] domain diagonal  [12..14] this rank's box lo  [15..17] its box hi
// [18] h_i (interior width)  [19] its send width  [20] wide-zone width w  [21] w - rounding slack
// [22] 1 if the plan routes with a halo field (then [6] = [18] = 0: the complete box is the own
//      box, the field certifies the rest)  [23] the field's largest width

// The local geometry of `rank` from its plan header -- ONE definition for every distributed
// runtime (the torch binding's dist_local and the C-API kn_solve_multi): the complete box (own box
// grown by the certification halo h, unbounded on domain faces or when the halo covers the
// domain), the local grid box (own box grown by the send halo, clipped to the domain) and its
// extent (the grid plan's aspect).
struct RankLocal {
    CompleteBox complete;
    double box[6];  // lo[3], hi[3]
    float ext[3];
};
// cert_field (optional): the rank's certification field (launch_field_cert) for a field plan.
RankLocal rank_local(const double* hdr, int rank, const int grid[3], const float* cert_field = nullptr,
                     int field_g = 0);

// Receive-side table: source s's segment starts at seg[s], holds own[s] owned rows then its
// halo rows; owned rows of all sources go first (own_pref), then halo rows (halo_pref).
// Self-last layout (launch_route_scatter with self_last = rank): the rank's own segment is
// not sent through the collective; recv then holds only the other sources' segments
// (rows_cross rows, self's seg[] entry is a zero-length placeholder) and the self segment is
// read from a separate buffer.
struct UnpackTable {
    int world;
    int n_own;
    int rows_cross;  // rows in recv; rows past it come from the self buffer
    int self;        // source whose segment is the self buffer (-1: none)
    int out_rows;    // rows of the output arrays (0: the rows processed; bounds checks only)
    int seg[kRouteMaxWorld];
    int own[kRouteMaxWorld];
    int own_pref[kRouteMaxWorld];
    int halo_pref[kRouteMaxWorld];
};

// Direct placement of the self segment (steady-state steps, split sizes known): the rank's own
// owned / halo rows go straight to their local rows -- owned row j at own_base + j, halo row j
// at halo_base + j of the (rows, 3) points / (rows,) global ids the local build reads -- instead of
// into the send buffer and through the unpack.
struct SelfPlace {
    float* pts;
    int* gids;
    int own_base;   // sum of recv_own over the sources before this rank
    int halo_base;  // n_own + sum of recv_halo over the sources before this rank
    int rows;       // local rows: every write is checked against it
    // the planned size of the self segment (validated step): a step whose own / halo counts for
    // this rank differ writes NOTHING (its rows would land at other offsets, possibly past
    // `rows`); the steady flag, which compares every count with the plan, rejects the step
    int own_cnt;
    int halo_cnt;
};

int route_block_count(int n);
// Every launcher reads the routing parameters from DEVICE memory (`p`), so the whole
// meta -> plan -> count chain is enqueued without a host round trip. `world` = p->world.
// block_counts: 2*world*route_block_count(n) ints (column-major, scanned in place);
// totals: 2*world ints = (owned, halo) rows per destination.
// zero_ints / n_zero (optional): ints block 0 zeroes on the way (the following build's bucket
// totals, BuildBuffers::totals_zeroed)
hipError_t launch_route_count(const float* pts, int n, const RouteParams* p, int world, int* block_counts,
                              int* totals, hipStream_t s,
                              unsigned* partials = nullptr, int* zero_ints = nullptr, int n_zero = 0);
// ids == nullptr: global id = p->id_offset + local index.
// self_last < 0: segments in destination order 0..world-1. self_last = rank: the other
// destinations in order, then the rank's own segment at the end (kept out of the collective).
// If the rows do not fit in send_rows the kernel writes nothing (the caller sees the totals
// after its sync and re-launches with a larger buffer) -- so the scatter can be enqueued
// before the host knows the sizes.
hipError_t launch_route_scatter(const float* pts, const int* ids, int n, const RouteParams* p, int world,
                                const int* block_offsets, const int* totals, float4* send, int send_rows,
                                int self_last, hipStream_t s,
                                const SelfPlace* self_place = nullptr);
// rows = t.rows_cross + rows of the self buffer (self_rows may be null when t.self < 0)
// sorted[i].w = gid[perm[i]] | (perm[i] >= n_owned ? 0x80000000 : 0): prepares a rank's grid
// for the query kernels' global-id mode (QueryBuffers::row_of = perm).
hipError_t launch_global_w(float4* sorted, const unsigned* perm, const int* gids, int n, int n_owned,
                           hipStream_t stream);
hipError_t launch_route_unpack(const float4* recv, const float4* self_rows, int rows, const UnpackTable& t,
                               float* pts, int* gids, hipStream_t s);
// metas: world x 8 doubles (every rank's launch_local_meta output, all-gathered on device).
// Writes the RouteParams for decomposition `grid` (px*py*pz == world) and the plan header:
// global domain, h = halo_factor x expected K-th neighbour radius of the whole cloud, the
// send width (h plus rounding slack; the whole domain once h reaches its diagonal), id offset.
// inner_factor > 0: the interior width h_i = min(h, inner_factor x that radius) for points
// farther than w = h + h_i from the domain faces (0: one width).
// splits: optional device array (route_split_count(grid) floats): count-balanced boxes.
// field (optional, device, field_g^3 widths): route with the density-adaptive halo field instead
// of the global widths (unless its largest width reaches the domain diagonal).
hipError_t launch_route_plan(const double* metas, int world, int rank, const int grid[3], int k,
                             double halo_factor, const float* splits, RouteParams* p, double* hdr, hipStream_t s,
                             double inner_factor = 0.0, const float* field = nullptr, int field_g = 0);
// ---- density-adaptive halo field (round 4) ----------------------------------------------------
// After a full step: every owned query whose K-th ball leaves the own box (own_lo / own_hi, +-inf
// on domain faces) raises the width of every field cell within m rings of its own cell to its
// K-th distance R (atomic max; m = the smallest ring count with R <= m * rstep, <= kFieldLevels).
// The ranks' fields are then MAX-all-reduced. pts: the rank's local rows (owned first), d2:
// (n_owned, k) squared distances. stat[0] += queries with fewer than K neighbours, stat[1] += queries
// beyond kFieldLevels rings (neither can be certified by the field). slack: absolute width added
// to R (>= the certification's rounding slack).
hipError_t launch_field_splat(const float* pts, int n_owned, const float* d2, int k, const float own_lo[3],
                              const float own_hi[3], const FieldGeom& fg, float slack, float* field, unsigned* stat,
                              hipStream_t s);
// cert[c] = max over m <= kFieldLevels of min(m * rstep, min of field over the m-ring
// neighbourhood of c): the radius up to which a query in cell c has every point of its ball.
hipError_t launch_field_cert(const float* field, const FieldGeom& fg, float* cert, hipStream_t s);
// The field geometry of a plan header (global domain [0..5]) with G cells per axis.
FieldGeom field_geom_hdr(const double* hdr, int g);
// Interior halo factor for K neighbours: the smallest f (steps of 0.05) for which a uniform
// cloud's K-th neighbour distance exceeds f x the expected (K+1)-point radius with probability
// <= 1e-12 (Poisson tail P[Poisson((K+1) f^3) <= K-1]); K=16 -> 1.55, K=1 -> 2.4, K=50 -> 1.35.
double inner_halo_factor(int k);
// Local meta of a rank's share: out = {lo[3], hi[3], n, 0} (doubles; +-inf box when n == 0).
// words: kBBoxWords scratch words (kn/kernels.h). One all_gather of `out` gives the global
// domain and the id offsets.
hipError_t launch_local_meta(const float* pts, int n, unsigned* words, double* out, hipStream_t s);
// Steady-state check of a sync-free distributed step, one wave: flag[0] = (this rank's meta or
// send counts differ from the planned ones) + (any uncertified query). No host involvement.
// Steady step check with the share's bbox taken from route_count's partials (route_block_count(n)
// blocks x 6 words, [a * nb + block]) instead of a local_meta pass.
// n_routed: rows route_count ran over (the partials' block count and stride); n: the share's true
// size (the meta comparison). n_routed <= n.
hipError_t launch_steady_flag_partials(const unsigned* partials, int n_routed, int n, const double* planned_meta,
                                       const int* totals, const int* planned_totals, int n_totals,
                                       const unsigned* counters, int* flag, hipStream_t stream);
// World-1 steady step check (no routing pass): one bbox pass over the share + the same flag
// kernel. sticky / host_flag (both or neither): also max-accumulate the flag into the device word
// `sticky` and store it to `host_flag`, a device-visible pointer to pinned host memory.
hipError_t launch_steady_flag_local(const float* pts, int n, unsigned* words, const double* planned_meta,
                                    const unsigned* counters, int* flag, int* sticky, int* host_flag, hipStream_t s);
// Sticky step flag (pipelined distributed steps, after the flag's all-reduce): sticky =
// max(sticky, flag), also stored to host_flag (device pointer to pinned host memory).
hipError_t launch_flag_sink(const int* flag, int* sticky, int* host_flag, hipStream_t s);
// *pending = max(*pending, *flag), atomically (steps on different streams accumulate into one word)
hipError_t launch_flag_accum(const int* flag, int* pending, hipStream_t s);
hipError_t launch_steady_flag(const double* local, const double* planned_meta, const int* totals,
                              const int* planned_totals, int n_totals, const unsigned* counters, int* flag,
                              hipStream_t s);
// Query forwarding inside a sync-free multi-GPU step (fixed-capacity slots, no host sync):
//   launch_fwd_pack    -> send: world x F slots of 2 float4 ({x, y, z, bits(gid)}, {K-th d2, ...}),
//                         the uncertified queries (uncert[0 .. *ucount), local rows; their K-th
//                         squared distance from d2 (rows x k)) to every other rank whose box is
//                         within it; slot_row (world x F) / slot_of (umax x world, -1 = none);
//                         overflow (> F per destination or > umax queries) counted in stat[1]
//   (equal-split all-to-all of send; launch_query_external_slots answers the received slots;
//    equal-split all-to-all of the answers back)
//   launch_fwd_merge   -> each forwarded row merged with its answers: K smallest (d2, gid), no
//                         duplicates (idx: global ids, -1 = empty)
hipError_t launch_fwd_pack(const RouteParams* p, int world, int rank, int F, int k, const unsigned* uncert,
                           const unsigned* ucount, int umax, const float* pts, const int* gids, const float* d2,
                           float4* send, int* slot_row, int* slot_of, int* cnt, unsigned* stat, hipStream_t s);
hipError_t launch_fwd_merge(int world, int F, int k, const unsigned* uncert, const unsigned* ucount, int umax,
                            const int* slot_of, const int* back_idx, const float* back_d2, int* idx, float* d2,
                            hipStream_t s);
// Count-balanced kd splits (parallel/decomposition.py balanced_splits, the same bins and
// slab / column assignment): the histogram stage of one rank's share. stage 0: x bins (1 row);
// stage 1: y bins per x slab (px rows, slabs from xs); stage 2: z bins per (x, y) column
// (px * py rows, columns from xs and ys). The caller sums the ranks' histograms and takes the
// quantile edges (multi.cpp split_edges), then runs the next stage with them.
constexpr int kSplitBins = 4096;
struct SplitHistArgs {
    float lo[3];
    float ext[3];  // hi - lo in float32, clamped >= 1e-30
    int grid[3];
    int stage;
    float xs[kRouteMaxWorld + 1];  // xs[0..px] (stages 1, 2)
    float ys[2 * kRouteMaxWorld];  // ys[ix * (py + 1) + j] (stage 2)
};
inline int split_hist_rows(const int g[3], int stage) { return stage == 0 ? 1 : stage == 1 ? g[0] : g[0] * g[1]; }
// scratch words launch_split_hist needs (per-block partial histograms)
size_t split_hist_scratch_words(int n, const int grid[3], int stage);
// hist: split_hist_rows x kSplitBins uint32, overwritten (stream-ordered, no host sync)
hipError_t launch_split_hist(const float* pts, int n, const SplitHistArgs& a, unsigned* hist, unsigned* scratch,
                             hipStream_t s);
hipError_t debug_words_route(unsigned out[4], bool reset);

}  // namespace kn
