// kn/route.h -- multi-GPU routing launchers (csrc/kernels/route.hip).
//
// One solve of the distributed engine moves every point once: to its owner rank and, as a
// halo copy, to each rank whose box is within h. The launchers below build the send buffer
// of that single all-to-all-v and unpack what arrives. Stream-ordered, allocation-free.
#pragma once

#include <hip/hip_runtime_api.h>

namespace kn {

constexpr int kRouteMaxWorld = 64;
constexpr int kRouteItems = 1024;  // points per routing block

struct RouteParams {
    float lo[3];    // global domain lower corner
    float ext[3];   // domain extent (hi - lo, clamped > 0)
    float g[3];     // decomposition grid (px, py, pz) as floats
    int grid[3];
    int world;      // px * py * pz <= kRouteMaxWorld
    float h2;       // squared halo send width
    float box_lo[kRouteMaxWorld][3];  // rank boxes (host-computed, same as SpatialDecomposition)
    float box_hi[kRouteMaxWorld][3];
};

// Receive-side table: source s's segment starts at seg[s], holds own[s] owned rows then its
// halo rows; owned rows of all sources go first (own_pref), then halo rows (halo_pref).
struct UnpackTable {
    int world;
    int n_own;
    int seg[kRouteMaxWorld];
    int own[kRouteMaxWorld];
    int own_pref[kRouteMaxWorld];
    int halo_pref[kRouteMaxWorld];
};

int route_block_count(int n);
// block_counts: 2*world*route_block_count(n) ints (column-major, scanned in place);
// totals: 2*world ints = (owned, halo) rows per destination.
hipError_t launch_route_count(const float* pts, int n, const RouteParams& p, int* block_counts, int* totals,
                              hipStream_t s);
hipError_t launch_route_scatter(const float* pts, const int* ids, int n, const RouteParams& p,
                                const int* block_offsets, const int* totals, float4* send, int send_rows,
                                hipStream_t s);
hipError_t launch_route_unpack(const float4* recv, int rows, const UnpackTable& t, float* pts, int* gids,
                               hipStream_t s);
// Local meta of a rank's share: out = {lo[3], hi[3], n, 0} (doubles; +-inf box when n == 0).
// words: 8 scratch words. One all_gather of `out` gives the global domain and the id offsets.
hipError_t launch_local_meta(const float* pts, int n, unsigned* words, double* out, hipStream_t s);
hipError_t debug_words_route(unsigned out[4], bool reset);

}  // namespace kn
