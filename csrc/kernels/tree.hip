// tree.hip -- Morton-leaf tree kNN for strongly non-uniform clouds (design: kn/tree.h).
//
// Reference: knearests.cu:93-148 walks a uniform grid whose cell size is fixed by the point count
// (knearests.cu:249); its README scopes it to uniformly distributed points. The grid path of this
// framework (query.hip) keeps that structure for uniform clouds; this file is the density-
// adaptive path: an implicit box tree over 64-point Morton leaves, traversed one wave per leaf.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <type_traits>

#include "kn/knn_device.h"
#include "kn/tree.h"
#include "kn/wave.h"

namespace kn {

namespace {

constexpr unsigned SENT = 0xFFFFFFFFu;
constexpr int kLeafBits = KN_TREE_LEAF_BITS;  // kTreeLeaf = 64 points per leaf (default)
#ifndef KN_TREE_SLOT_BITS
#define KN_TREE_SLOT_BITS 13
#endif
constexpr int kVisitBits = KN_TREE_SLOT_BITS - kLeafBits;  // key slot = visit index | point in leaf
static_assert(kLeafBits <= 6, "a leaf is scanned by one wave (<= 64 points)");
constexpr int kMaxVisit = 1 << kVisitBits;    // leaves a wave may visit before its queries go exact
constexpr unsigned kMask = (1u << (kVisitBits + kLeafBits)) - 1u;
static_assert((1 << kLeafBits) == kTreeLeaf, "leaf size");
constexpr int kStack = 64;  // traversal stack: <= 3 pending siblings per 2 levels of log2(P) <= 31
constexpr int kTCap = 256;                    // exact-finish candidate buffer per wave (u64 keys)
constexpr int kSortPasses = 3;                // odd-even passes of the exact re-rank (then checked)
// A point inside a box can compute a squared distance a few ulps below the box's: nodes are
// pruned only when the box distance exceeds the bound by more than that.
constexpr float kShrink = 0.99999f;
constexpr int kExactGrid = 512;
constexpr int kFrontier = 256;  // exact kernel: breadth-first frontier / leaf list per wave
// Round-3 A/Bs of the traversal that LOST (900K, identical rows): a breadth-first sweep with the
// bounds frozen after the own leaves (profiles/ab_r3_tree_bfs.jsonl, 1.3-3.5x slower: a sparse
// query near a cluster keeps a loose bound until the cluster's nearest leaves shrink it, which
// only the depth-first order does); per-lane box distances stacked in LDS instead of re-loading a
// popped node's box (profiles/ab_r3_tree_stackdist.jsonl, K=16 +16 %: the 10 KB per wave cost
// more in resident waves than the loads it saved). Session 2: a leaf-filtered variant (the traversal
// only lists the leaves it enters; every 32 listed leaves each lane box-tests them against its own
// bound and scans just the ones it needs with per-lane 4-wide global gathers) lost everywhere
// (profiles/ab_r3_tree_filter.jsonl, K=16: clustered 1.59 -> 2.29 ms, surface 0.96 -> 1.34,
// uniform 1.36 -> 1.88; K=50 +10-40 %): the divergent global-memory gathers and the bounds frozen
// between chunks (+20 % listed leaves) cost more than the broadcast union stream of staged leaves.
// Leaves of 16 instead of 32 points (KN_TREE_LEAF_BITS=4: tighter boxes, twice the visits) lost too
// (profiles/ab_r3_tree_leaf16.jsonl: clustered K=16 1.61 -> 2.03 ms, surface 0.97 -> 1.46).
// Grouped traversal (G = 2 / 4 groups of 32 / 16 queries per wave, each with its own near-first
// traversal, stack, visit list and leaf buffer; rounds alternate node steps and leaf streams) lost
// 1.5-4x (profiles/ab_r3_tree_groups{2,4}.jsonl): a group's union is far more than 1/G of the
// wave's (clustered K=16: 709K leaf visits per solve -> 1.06M / 1.62M summed over groups), and
// each round waits for the slowest group.

struct TArgs {
    const float4* pts;
    const unsigned* leaf_start;  // L + 1
    const float4* nlo;
    const float4* nhi;
    unsigned* list;
    float* thr;
    const unsigned* Lp;  // device leaf count (written by the build: no host read, graph-capturable)
    int n, P, logP;      // P = the node buffer's leaf capacity (power of two >= n)
    int k;
    int n_queries;
    int q_lo;  // always 0: the tree path serves whole solves (ranges use the grid kernels)
    const unsigned* id_map;
    const unsigned* row_of;  // null: local mode of w_live / w_id / w_row / out_id; else global-id mode
    const unsigned* src;     // tree point -> input (grid slot) index: row_of is indexed by grid slot
    unsigned* out_idx;
    float* out_dist;
    unsigned* const* out_idx_ref;  // non-null: output pointers read from these slots at launch
    float* const* out_dist_ref;
    unsigned* counters;
    int flags;
};


__device__ __forceinline__ unsigned ordf(float f) {
    const unsigned u = __float_as_uint(f);
    return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
}
__device__ __forceinline__ float unordf(unsigned u) {
    return __uint_as_float((u & 0x80000000u) ? (u & 0x7FFFFFFFu) : ~u);
}

// 10 bits -> every third bit of 30
__device__ __forceinline__ unsigned spread10(unsigned v) {
    v &= 0x3FFu;
    v = (v | (v << 16)) & 0x030000FFu;
    v = (v | (v << 8)) & 0x0300F00Fu;
    v = (v | (v << 4)) & 0x030C30C3u;
    v = (v | (v << 2)) & 0x09249249u;
    return v;
}

__device__ __forceinline__ float box_d2(float qx, float qy, float qz, const float4& lo, const float4& hi) {
    const float dx = fmaxf(fmaxf(lo.x - qx, qx - hi.x), 0.f);
    const float dy = fmaxf(fmaxf(lo.y - qy, qy - hi.y), 0.f);
    const float dz = fmaxf(fmaxf(lo.z - qz, qz - hi.z), 0.f);
    return fmaf(dz, dz, fmaf(dy, dy, dx * dx));
}

// ---- build: Morton order of the grid's CELLS, no sort ------------------------------------------
// The input is the grid's sorted array: points already grouped by cell (x-fastest). The tree order
// is the Morton order of the cells: cells are grouped in 8x8x8 bricks, bricks are numbered by
// the Morton code of their brick coordinates (a padded power-of-two brick space) and the cells of
// a brick by their 9-bit in-brick Morton code, so (brick code << 9 | cell code) IS the cell's
// Morton code. One exclusive scan over the brick counts places every brick; one workgroup per
// brick scans its 512 cells in Morton order and copies their point runs. Counting, no sorting:
// replaces the round-2 30-bit radix sort of point codes (hipCUB) and needs no host round trip.
constexpr int kBrickBits = 3;            // 8 cells per brick axis
constexpr int kBrickCells = 1 << (3 * kBrickBits);

__device__ __forceinline__ unsigned compact3(unsigned v) {  // inverse of spread10
    v &= 0x09249249u;
    v = (v | (v >> 2)) & 0x030C30C3u;
    v = (v | (v >> 4)) & 0x0300F00Fu;
    v = (v | (v >> 8)) & 0x030000FFu;
    v = (v | (v >> 16)) & 0x000003FFu;
    return v;
}

// One 64-thread workgroup per real brick: lane = one (y, z) row of the brick's 8x8 rows; the
// brick's point count lands at its Morton slot of the (pre-zeroed) padded count array.
__global__ __launch_bounds__(64) void brick_count_kernel(const int* __restrict__ cell_start, const GridGeom* __restrict__ geom,
                                                         int nbx, int nby, unsigned* __restrict__ bcount) {
    const GridGeom g = *geom;
    const int b = blockIdx.x, bx = b % nbx, by = (b / nbx) % nby, bz = b / (nbx * nby);
    const int lane = threadIdx.x;
    const int y = by * 8 + (lane & 7), z = bz * 8 + (lane >> 3);
    const int x0 = bx * 8, x1 = min(g.dims[0], x0 + 8);
    unsigned c = 0;
    if (y < g.dims[1] && z < g.dims[2]) {
        const size_t row = ((size_t)z * g.dims[1] + y) * g.dims[0];
        c = (unsigned)(cell_start[row + x1] - cell_start[row + x0]);
    }
    c = wave_sum_u32(c);
    if (lane == 0) bcount[spread10(bx) | (spread10(by) << 1) | (spread10(bz) << 2)] = c;
}

// One 256-thread workgroup per real brick: in-brick Morton scan of the 512 cell counts, then every
// point of the brick to its cell's tree range (thread per point, cell found by binary search),
// in input order within the cell: tmp_pts / tmp_vals (input index), the cell's Morton code and
// tree range [first, end) per point (subcell_rank_kernel orders the cell).
__global__ __launch_bounds__(256) void brick_scatter_kernel(const float4* __restrict__ in, const int* __restrict__ cell_start,
                                                            const GridGeom* __restrict__ geom, int nbx, int nby,
                                                            const unsigned* __restrict__ bbase, float4* __restrict__ tmp_pts,
                                                            unsigned* __restrict__ tmp_vals,
                                                            unsigned long long* __restrict__ cell_code,
                                                            uint2* __restrict__ cell_span) {
    __shared__ int s_base[kBrickCells + 1];
    __shared__ int s_start[kBrickCells];
    __shared__ int s_wsum[4];
    const GridGeom g = *geom;
    const int b = blockIdx.x, bx = b % nbx, by = (b / nbx) % nby, bz = b / (nbx * nby);
    const unsigned bcode = spread10(bx) | (spread10(by) << 1) | (spread10(bz) << 2);
    const int t = threadIdx.x, lane = t & 63, wid = t >> 6;
    int cnt[2];
#pragma unroll
    for (int h = 0; h < 2; ++h) {
        const int m = 2 * t + h;  // a thread owns two consecutive Morton slots
        const int x = bx * 8 + (int)compact3((unsigned)m), y = by * 8 + (int)compact3((unsigned)m >> 1),
                  z = bz * 8 + (int)compact3((unsigned)m >> 2);
        cnt[h] = 0;
        int st = 0;
        if (x < g.dims[0] && y < g.dims[1] && z < g.dims[2]) {
            const size_t c = ((size_t)z * g.dims[1] + y) * g.dims[0] + x;
            st = cell_start[c];
            cnt[h] = cell_start[c + 1] - st;
        }
        s_start[m] = st;
    }
    const int tsum = cnt[0] + cnt[1];
    const int incl = wave_inclusive_scan_add(tsum);
    if (lane == 63) s_wsum[wid] = incl;
    __syncthreads();
    int off = incl - tsum;
    for (int w = 0; w < wid; ++w) off += s_wsum[w];
    s_base[2 * t] = off;
    s_base[2 * t + 1] = off + cnt[0];
    if (t == 255) s_base[kBrickCells] = off + tsum;
    __syncthreads();
    const int total = s_base[kBrickCells];
    const unsigned out0 = bbase[bcode];
    for (int j = t; j < total; j += 256) {
        int lo = 0, hi = kBrickCells - 1;  // last slot whose base <= j (the non-empty cell holding j)
        while (lo < hi) {
            const int mid = (lo + hi + 1) >> 1;
            if (s_base[mid] <= j) lo = mid; else hi = mid - 1;
        }
        const unsigned src = (unsigned)(s_start[lo] + (j - s_base[lo]));
        const unsigned dst = out0 + (unsigned)j;
        tmp_pts[dst] = in[src];
        tmp_vals[dst] = src;
        // the cell's Morton code: up to 30 brick bits + 9 in-brick bits (64-bit: an axis of more than
        // 1,024 cells -- 128 bricks -- takes the brick code past 23 bits)
        cell_code[dst] = ((unsigned long long)bcode << (3 * kBrickBits)) | (unsigned long long)lo;
        cell_span[dst] = make_uint2(out0 + (unsigned)s_base[lo], out0 + (unsigned)s_base[lo + 1]);
    }
}

// Within a cell, points follow the Morton order of their 8x8x8 sub-cell (ties: input order), so
// leaves may split a dense cell into compact parts (cell-granular leaves cost the tree query
// ~20 %). One thread per point ranks it by counting over its cell's points: sum of count^2 work
// (~8n for an occupancy-adaptive grid), spread evenly over the points -- done per brick, the
// few bricks holding a cluster's core serialised it (230 us at 900K clustered).
__device__ __forceinline__ unsigned subcell_code(const GridGeom& g, const float4& p, unsigned long long cc) {
    // cell coordinates: brick coordinates (the high bits) * 8 + the in-brick Morton bits
    const unsigned bc = (unsigned)(cc >> (3 * kBrickBits)), ic = (unsigned)cc & (kBrickCells - 1);
    const int cx = (int)((compact3(bc) << kBrickBits) | compact3(ic));
    const int cy = (int)((compact3(bc >> 1) << kBrickBits) | compact3(ic >> 1));
    const int cz = (int)((compact3(bc >> 2) << kBrickBits) | compact3(ic >> 2));
    const int sx = clampi((int)((p.x - (g.origin[0] + cx * g.cell[0])) * g.inv_cell[0] * 8.f), 0, 7);
    const int sy = clampi((int)((p.y - (g.origin[1] + cy * g.cell[1])) * g.inv_cell[1] * 8.f), 0, 7);
    const int sz = clampi((int)((p.z - (g.origin[2] + cz * g.cell[2])) * g.inv_cell[2] * 8.f), 0, 7);
    return spread10((unsigned)sx) | (spread10((unsigned)sy) << 1) | (spread10((unsigned)sz) << 2);
}
__global__ __launch_bounds__(256) void subcell_rank_kernel(const float4* __restrict__ tmp_pts, const unsigned* __restrict__ tmp_vals,
                                                           const unsigned long long* __restrict__ cell_code,
                                                           const uint2* __restrict__ cell_span,
                                                           const GridGeom* __restrict__ geom, int n, float4* __restrict__ pts,
                                                           unsigned* __restrict__ vals, unsigned long long* __restrict__ codes) {
    const int j = blockIdx.x * blockDim.x + threadIdx.x;
    if (j >= n) return;
    const GridGeom g = *geom;
    const unsigned long long cc = cell_code[j];
    const uint2 sp = cell_span[j];
    const float4 p = tmp_pts[j];
    const unsigned sc = subcell_code(g, p, cc);
    unsigned r = 0;
    if (sp.y - sp.x > 1)
        for (unsigned i = sp.x; i < sp.y; ++i) {
            const unsigned si = subcell_code(g, tmp_pts[i], cc);
            r += (si < sc || (si == sc && i < (unsigned)j)) ? 1u : 0u;
        }
    const unsigned dst = sp.x + r;
    pts[dst] = p;
    vals[dst] = tmp_vals[j];
    codes[dst] = (cc << 9) | sc;  // <= 48 bits
}

// ---- device-wide scan of u32 (block sums -> one-workgroup scan of the sums -> block scans) ------
constexpr int kTScanItems = 4096;  // 256 threads x 16
__global__ __launch_bounds__(256) void tscan_sums_kernel(const unsigned* __restrict__ in, int n, unsigned* __restrict__ sums) {
    const int base = blockIdx.x * kTScanItems;
    unsigned s = 0;
    for (int i = base + threadIdx.x; i < min(n, base + kTScanItems); i += 256) s += in[i];
    __shared__ unsigned ws[4];
    s = wave_sum_u32(s);
    if ((threadIdx.x & 63) == 0) ws[threadIdx.x >> 6] = s;
    __syncthreads();
    if (threadIdx.x == 0) sums[blockIdx.x] = ws[0] + ws[1] + ws[2] + ws[3];
}
// (256 threads: a 1024-thread block beside the running query kernels waits for 16 free wave slots
// on one CU)
constexpr int kTScanTop = 256;
__global__ __launch_bounds__(kTScanTop) void tscan_top_kernel(unsigned* __restrict__ sums, int nb) {
    __shared__ unsigned wsum[kTScanTop / 64];
    __shared__ unsigned carry_s;
    if (threadIdx.x == 0) carry_s = 0;
    __syncthreads();
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    for (int base = 0; base < nb; base += kTScanTop) {
        const int i = base + threadIdx.x;
        const unsigned v = (i < nb) ? sums[i] : 0u;
        const unsigned incl = (unsigned)wave_inclusive_scan_add((int)v);
        if (lane == 63) wsum[wid] = incl;
        __syncthreads();
        unsigned woff = 0;
        for (int w = 0; w < wid; ++w) woff += wsum[w];
        const unsigned carry = carry_s;
        if (i < nb) sums[i] = carry + woff + incl - v;
        __syncthreads();
        if (threadIdx.x == kTScanTop - 1) carry_s = carry + woff + incl;
        __syncthreads();
    }
}
// out = scan(in) with the block offsets from tscan_top (inclusive or exclusive); in may == out
__global__ __launch_bounds__(256) void tscan_apply_kernel(const unsigned* __restrict__ in, int n, const unsigned* __restrict__ sums,
                                                          unsigned* __restrict__ out, int inclusive) {
    constexpr int I = kTScanItems / 256;
    const int base = blockIdx.x * kTScanItems + threadIdx.x * I;
    unsigned v[I];
#pragma unroll
    for (int j = 0; j < I; ++j) v[j] = (base + j < n) ? in[base + j] : 0u;
    unsigned s = 0;
#pragma unroll
    for (int j = 0; j < I; ++j) { const unsigned x = v[j]; v[j] = inclusive ? s + x : s; s += x; }
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    const unsigned incl = (unsigned)wave_inclusive_scan_add((int)s);
    __shared__ unsigned wsum[4];
    if (lane == 63) wsum[wid] = incl;
    __syncthreads();
    unsigned off = sums[blockIdx.x] + incl - s;
    for (int w = 0; w < wid; ++w) off += wsum[w];
#pragma unroll
    for (int j = 0; j < I; ++j)
        if (base + j < n) out[base + j] = v[j] + off;
}
inline unsigned cdiv_(size_t a, size_t b) { return (unsigned)((a + b - 1) / b); }
hipError_t tscan(const unsigned* in, int n, unsigned* out, unsigned* sums, bool inclusive, hipStream_t s) {
    if (n <= 0) return hipSuccess;
    const unsigned nb = cdiv_((size_t)n, kTScanItems);
    tscan_sums_kernel<<<nb, 256, 0, s>>>(in, n, sums);
    tscan_top_kernel<<<1, kTScanTop, 0, s>>>(sums, (int)nb);
    tscan_apply_kernel<<<nb, 256, 0, s>>>(in, n, sums, out, inclusive ? 1 : 0);
    return hipGetLastError();
}

// Leaf boundaries: leaves are the maximal binary-prefix (radix) nodes of the sorted Morton codes
// holding <= kTreeLeaf points -- boxes of aspect <= 2 that never straddle a jump of the curve
// (fixed runs of the Morton order do: measured ~2x the candidates per query). Positions b-1 and b
// are in different leaves iff their lowest common prefix node holds more than kTreeLeaf points;
// its extent is found by two binary searches inside the kTreeLeaf + 1 window around b. Runs of
// equal codes (one finest cell) longer than a leaf are chunked by leaf_flag_kernel.
__device__ __forceinline__ int hibit(unsigned long long x) { return x ? 63 - __builtin_clzll(x) : -1; }

// codes: 64-bit Morton codes of each point's sub-cell (3 bits per brick level, 9 in-brick cell
// bits, 9 sub-cell bits: > 32 bits for any grid of more than one brick level)
__global__ void cut_kernel(const unsigned long long* __restrict__ c, int n, unsigned* __restrict__ flag) {
    const int b = blockIdx.x * blockDim.x + threadIdx.x;
    if (b >= n) return;
    unsigned f = 1u;
    if (b > 0) {
        const unsigned long long x = c[b - 1] ^ c[b];
        f = 0u;
        if (x) {
            const int sh = hibit(x) + 1;
            const unsigned long long p = sh >= 64 ? 0ull : c[b] >> sh;
            int lo = max(0, b - 1 - kTreeLeaf), hi = b - 1;  // first index with prefix p
            while (lo < hi) {
                const int mid = (lo + hi) >> 1;
                if ((sh >= 64 ? 0ull : c[mid] >> sh) == p) hi = mid; else lo = mid + 1;
            }
            const int s0 = lo;
            lo = b; hi = min(n, b + kTreeLeaf + 1);  // first index past the prefix
            while (lo < hi) {
                const int mid = (lo + hi) >> 1;
                if ((sh >= 64 ? 0ull : c[mid] >> sh) == p) lo = mid + 1; else hi = mid;
            }
            f = (lo - s0 > kTreeLeaf) ? 1u : 0u;
        }
    }
    flag[b] = f;
}

// incl = inclusive scan of flag: segment (or leaf) id of b = incl[b] - 1; starts[id] = b at flagged
// positions, starts[count] = n, count -> *total
__global__ void starts_kernel(const unsigned* __restrict__ flag, const unsigned* __restrict__ incl, int n,
                              unsigned* __restrict__ starts, unsigned* __restrict__ total) {
    const int b = blockIdx.x * blockDim.x + threadIdx.x;
    if (b >= n) return;
    if (flag[b]) starts[incl[b] - 1] = (unsigned)b;
    if (b == n - 1) {
        starts[incl[b]] = (unsigned)n;
        if (total) *total = incl[b];
    }
}

// flag[b] = b starts a leaf: segment [s, e) splits at s + floor(j len / c), c = ceil(len / kTreeLeaf)
__global__ void leaf_flag_kernel(const unsigned* __restrict__ incl, const unsigned* __restrict__ seg_start, int n,
                                 unsigned* __restrict__ flag) {
    const int b = blockIdx.x * blockDim.x + threadIdx.x;
    if (b >= n) return;
    const unsigned sg = incl[b] - 1;
    const unsigned long long s0 = seg_start[sg], len = seg_start[sg + 1] - s0;
    const unsigned long long c = (len + kTreeLeaf - 1) / kTreeLeaf, o = (unsigned long long)b - s0;
    const unsigned long long j = (o * c + len - 1) / len;
    flag[b] = (j * len / c == o) ? 1u : 0u;
}

// One wave per leaf, grid-stride over the device leaf count (leaves past it are never read:
// the traversal and node_box_kernel test a node's first leaf against L instead).
__global__ __launch_bounds__(256) void leaf_box_kernel(const float4* __restrict__ pts, const unsigned* __restrict__ leaf_start,
                                                       const unsigned* __restrict__ Lp, int P, float4* __restrict__ nlo,
                                                       float4* __restrict__ nhi) {
    const int L = (int)*Lp, lane = threadIdx.x & 63;
    for (int leaf = blockIdx.x * 4 + (threadIdx.x >> 6); leaf < L; leaf += gridDim.x * 4) {
        const unsigned i = leaf_start[leaf] + lane;
        const bool v = i < leaf_start[leaf + 1];
        const float4 p = v ? pts[i] : make_float4(0.f, 0.f, 0.f, 0.f);
        const unsigned lx = wave_min_u32(v ? ordf(p.x) : SENT), hx = wave_max_u32(v ? ordf(p.x) : 0u);
        const unsigned ly = wave_min_u32(v ? ordf(p.y) : SENT), hy = wave_max_u32(v ? ordf(p.y) : 0u);
        const unsigned lz = wave_min_u32(v ? ordf(p.z) : SENT), hz = wave_max_u32(v ? ordf(p.z) : 0u);
        if (lane == 0) {
            // w words: the leaf's first point and count, so a traversal that tests the leaf's box
            // has its point range in the same load (no dependent leaf_start round before the points)
            const unsigned b0 = leaf_start[leaf], cnt = leaf_start[leaf + 1] - b0;
            nlo[P + leaf] = make_float4(unordf(lx), unordf(ly), unordf(lz), __uint_as_float(b0));
            nhi[P + leaf] = make_float4(unordf(hx), unordf(hy), unordf(hz), __uint_as_float(cnt));
        }
    }
}

// First leaf of heap node v (root 1, leaves at [P, 2P), P = 2^logP). Nodes whose first leaf is
// at or past the leaf count L are empty; they are never written, never entered.
__device__ __forceinline__ int first_leaf(int v, int logP) {
    const int d = 31 - __builtin_clz((unsigned)v);
    return (v << (logP - d)) - (1 << logP);
}

// Nodes [m, 2m) -> their ancestors up to log2(min(m, 64)) levels, one 64-thread workgroup per
// group of min(m, 64) siblings, in LDS.
__global__ __launch_bounds__(64) void node_box_kernel(float4* __restrict__ nlo, float4* __restrict__ nhi, int m,
                                                      int logP, const unsigned* __restrict__ Lp) {
    __shared__ float4 slo[64], shi[64];
    const int t = threadIdx.x;
    const int cnt = min(m, 64);
    int nb = m + blockIdx.x * cnt;
    const int L = (int)*Lp;
    if (first_leaf(nb, logP) >= L) return;  // the whole group is past the last leaf
    if (t < cnt) {
        // empty nodes (first leaf >= L) were never written: read as empty boxes
        const bool e = first_leaf(nb + t, logP) >= L;
        slo[t] = e ? make_float4(INFINITY, INFINITY, INFINITY, 0.f) : nlo[nb + t];
        shi[t] = e ? make_float4(-INFINITY, -INFINITY, -INFINITY, 0.f) : nhi[nb + t];
    }
    __syncthreads();
    for (int c = cnt; c > 1; c >>= 1) {
        const int h = c >> 1;
        float4 l = make_float4(0.f, 0.f, 0.f, 0.f), u = l;
        if (t < h) {
            const float4 a0 = slo[2 * t], a1 = slo[2 * t + 1], b0 = shi[2 * t], b1 = shi[2 * t + 1];
            l = make_float4(fminf(a0.x, a1.x), fminf(a0.y, a1.y), fminf(a0.z, a1.z), 0.f);
            u = make_float4(fmaxf(b0.x, b1.x), fmaxf(b0.y, b1.y), fmaxf(b0.z, b1.z), 0.f);
        }
        __syncthreads();
        nb >>= 1;
        if (t < h) { slo[t] = l; shi[t] = u; nlo[nb + t] = l; nhi[nb + t] = u; }
        __syncthreads();
    }
}

// ---- query: one wave per 64 consecutive points of the Morton order (lanes = queries) -------------
// (Round 4, 32-point leaves: asking the compiler for 6 / 8 waves per SIMD at K <= 16 (82 -> 80 / 64
// VGPRs, 3 / 12 spilled) was mixed -- clustered 1.440 -> 1.422 / 1.404 ms, surfaces 0.825 -> 0.854 /
// 0.853; profiles/ab_r4_tree_waves.txt. Round 5, 64-point leaves: 8 waves wins, KN_TREE_WPE.)
// Waves per SIMD requested for the K <= 16 buckets (a VGPR cap: K=16 82 -> 64 VGPRs, 12 spilled).
// With 64-point leaves the latency-bound traversal gains from the occupancy: 900K, pipelined,
// clustered K=16 1.098 -> 1.041 ms, surfaces 0.742 -> 0.717, K=8 unchanged (6 waves: +0..2 %;
// profiles/ab_r5_tree_waves.txt; with 32-point leaves it was mixed, round 4). KN_TREE_WPE=1: no cap.
#ifndef KN_TREE_WPE
#define KN_TREE_WPE 8
#endif
// K=24 / K=32 buckets: 5 / 4 waves (114 -> 96 VGPRs, 7 spilled; 146 -> 128, 5 spilled): clustered
// K=24 1.368 -> 1.296 ms, K=32 1.893 -> 1.672, surfaces K=32 1.022 -> 0.995 (profiles/ab_r5_tree_waves.txt)
#ifndef KN_TREE_WPE24
#define KN_TREE_WPE24 5
#endif
#ifndef KN_TREE_WPE32
#define KN_TREE_WPE32 4
#endif
// K=40 / K=50 buckets: 3 waves (178 / 222 -> 168 VGPRs, 3 / 25 spilled): clustered K=40 3.09 -> 2.38
// ms, K=50 3.80 -> 2.82, surfaces K=50 1.96 -> 1.56 (profiles/ab_r5_tree_waves.txt)
#ifndef KN_TREE_WPE50
#define KN_TREE_WPE50 3
#endif
// K=64 bucket: 2 waves (259 -> 256 VGPRs, 3 spilled): clustered K=64 8.78 -> 5.02 ms, surfaces
// 4.64 -> 2.65
#ifndef KN_TREE_WPE64
#define KN_TREE_WPE64 2
#endif
// Gated-tier top-K networks in the tree query (kn/knn_device.h topk_tiers): KN_TREE_TIERS = T > 0
// forces T, -1 = the tile kernel's rule (3 tiers for the K=50 bucket, 4 for K=64), 0 (default)
// one network
#ifndef KN_TREE_TIERS
#define KN_TREE_TIERS 0
#endif
template <int KT>
constexpr int tree_tiers() {
    return KN_TREE_TIERS > 0 ? KN_TREE_TIERS : KN_TREE_TIERS < 0 ? (KT > 50 ? 4 : KT > 40 ? 3 : 1) : 1;
}
template <int KT>
constexpr int tree_wpe() {
    return KT <= 16 ? KN_TREE_WPE
                    : KT <= 24 ? KN_TREE_WPE24 : KT <= 32 ? KN_TREE_WPE32 : KT <= 50 ? KN_TREE_WPE50 : KN_TREE_WPE64;
}
template <int KT, int M>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(tree_wpe<KT>(), 8))) void knn_tree_kernel(TArgs a) {
    // output pointers: the launch's, or read from device slots (graph replays of a batched
    // stream of clouds); locals, so the kernel argument block stays read-only
    out_u32_t* const o_idx = out_ptr(a.out_idx_ref ? *a.out_idx_ref : a.out_idx);
    out_f32_t* const o_dist = out_ptr(a.out_idx_ref ? (a.out_dist_ref ? *a.out_dist_ref : nullptr) : a.out_dist);
    constexpr int KM = KT + M + 1;  // + 1: the query itself enters its own list at d2 = 0
    __shared__ float4 s_pts[4][kTreeLeaf];
    __shared__ int s_visit[4][kMaxVisit];  // first point of each visited leaf
    __shared__ int s_stack[4][kStack];
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    const int w = xcd_remap(blockIdx.x, gridDim.x) * 4 + wid;
    const int base = w * 64;
    if (base >= a.n) return;
    float4* buf = s_pts[wid];
    int* vis = s_visit[wid];
    int* stk = s_stack[wid];
    const int qcnt = min(64, a.n - base);
    // lanes past the last point duplicate it (same candidate stream, never written back)
    const unsigned qpos = (unsigned)(base + min(lane, qcnt - 1));
    const float4 qp = a.pts[KN_IDX(qpos, (unsigned)a.n, 401)];
    const unsigned qw = __float_as_uint(qp.w);
    const bool live = lane < qcnt && w_live(a, qw);
    if (!__builtin_amdgcn_ballot_w64(live)) return;
    const float qx = qp.x, qy = qp.y, qz = qp.z;

    unsigned keys[KM];
#pragma unroll
    for (int j = 0; j < KM; ++j) keys[j] = SENT;
    unsigned nnet = 0;
    int nv = 0;
    bool over = false;

    // stage the leaf of points [b, b + cnt) in the wave's LDS slice and stream its points to every
    // lane (broadcast reads)
    auto visit_range = [&](int b, int cnt) __attribute__((always_inline)) {
        if (lane < cnt) buf[lane] = a.pts[KN_IDX(b + lane, a.n, 402)];
        if (lane == 0) vis[nv] = b;
        __builtin_amdgcn_wave_barrier();
        const int sb = nv << kLeafBits;
#pragma unroll 4
        for (int j = 0; j < cnt; ++j) {
            const float4 c = buf[j];
            nnet += topk_push<KM, KN_TOPK_SPLIT, tree_tiers<KT>()>(keys, cand_key(c, qx, qy, qz, ~kMask, sb + j, 0));
        }
        ++nv;
        __builtin_amdgcn_wave_barrier();
    };
    auto visit = [&](int lf) __attribute__((always_inline)) {
        const int b = (int)a.leaf_start[lf];
        visit_range(b, (int)a.leaf_start[lf + 1] - b);
    };
    // the leaves holding the wave's own 64 points first: every lane starts the traversal with a
    // bound from ~64 nearby candidates (small leaves alone leave the early bounds loose, and a
    // loose bound of any lane opens nodes for the whole wave)
    const int L = (int)*a.Lp;
    int l0 = 0, l1 = L - 1;
    while (l0 < l1) {  // last leaf starting at or before base
        const int mid = (l0 + l1 + 1) >> 1;
        if ((int)a.leaf_start[mid] <= base) l0 = mid; else l1 = mid - 1;
    }
    l1 = l0;
    while (l1 + 1 < L && (int)a.leaf_start[l1 + 1] < base + qcnt) ++l1;
    for (int lf = l0; lf <= l1 && nv < kMaxVisit; ++lf) visit(lf);

    // wave-uniform near-first traversal from the root: a node is entered when any live lane's
    // box distance is within its bound (the (K+M+1)-th key, rounded up)
    int sp = 1;
    if (lane == 0) stk[0] = 1;
    __builtin_amdgcn_wave_barrier();
    while (sp > 0) {
        --sp;
        const int node = __builtin_amdgcn_readfirstlane(stk[sp]);
        const unsigned last = keys[KM - 1];
        const float ub = last == SENT ? INFINITY : __uint_as_float(last | kMask);
        if (node >= a.P) {
            // a leaf is re-tested against the bounds tightened since its push (a visit stages and
            // scores its points); an inner node is not: its children are tested below anyway,
            // and a child's box lies inside its parent's, so skipping the parent's re-test prunes
            // the same subtrees one dependent box load sooner (900K K=16: clustered 1.578 ->
            // 1.453 ms/step, surfaces 0.972 -> 0.930, the same leaf visits and rows;
            // profiles/ab_r4_tree_pop_retest.txt)
            const float4 blo = a.nlo[node], bhi = a.nhi[node];
            const float bd = box_d2(qx, qy, qz, blo, bhi);
            if (!__builtin_amdgcn_ballot_w64(live && bd < INFINITY && bd * kShrink <= ub)) continue;
            const int lf = node - a.P;
            if (lf >= l0 && lf <= l1) continue;  // visited first
            if (nv == kMaxVisit) { over = true; break; }
            // the point range rides in the box's w words (leaf_box_kernel)
            visit_range(__builtin_amdgcn_readfirstlane((int)__float_as_uint(blo.w)),
                        __builtin_amdgcn_readfirstlane((int)__float_as_uint(bhi.w)));
            continue;
        }
        const int c0 = 2 * node;
        // the grandchildren of an inner node whose children are inner nodes, tested and pushed
        // directly (a grandchild's box lies inside its parent's, so one that passes has a passing
        // parent): one dependent round of box loads per two levels instead of per level. A node is
        // empty when its first leaf lies past L (the leftmost descendant never is). 900K K=16:
        // clustered 1.479 -> 1.449 ms/step, surfaces 0.951 -> 0.825; three levels (8 boxes per
        // round) lost, 2.11 / 1.16 (profiles/ab_r4_tree_fan.txt)
        auto enter_descendants = [&](auto fan_c) __attribute__((always_inline)) {
            constexpr int FAN = decltype(fan_c)::value;
            const int g0 = node * FAN;
            float gd[FAN];
            unsigned need = 0u;  // bit j: descendant j is entered
#pragma unroll
            for (int j = 0; j < FAN; ++j) {
                const int g = g0 + j;
                gd[j] = (j == 0 || first_leaf(g, a.logP) < L) ? box_d2(qx, qy, qz, a.nlo[g], a.nhi[g]) : INFINITY;
                if (__builtin_amdgcn_ballot_w64(live && gd[j] < INFINITY && gd[j] * kShrink <= ub)) need |= 1u << j;
            }
            // near-first: the descendant nearest for most live lanes goes on top
            int am = 0;
#pragma unroll
            for (int j = 1; j < FAN; ++j) am = gd[j] < gd[am] ? j : am;
            int ord[FAN], vote[FAN];
#pragma unroll
            for (int j = 0; j < FAN; ++j) {
                vote[j] = (need >> j) & 1u ? __builtin_popcountll(__builtin_amdgcn_ballot_w64(live && am == j)) : -1;
                ord[j] = j;
            }
#pragma unroll
            for (int i = 1; i < FAN; ++i)  // ascending votes: the most-voted pushed last (top)
#pragma unroll
                for (int j = i; j > 0; --j)
                    if (vote[ord[j]] < vote[ord[j - 1]]) { const int t = ord[j]; ord[j] = ord[j - 1]; ord[j - 1] = t; }
#pragma unroll
            for (int i = 0; i < FAN; ++i) {
                const int j = ord[i];
                if ((need >> j) & 1u) {
                    if (lane == 0) stk[sp] = g0 + j;
                    ++sp;
                }
            }
            __builtin_amdgcn_wave_barrier();
        };
        if (sp + 4 > kStack) { over = true; break; }  // (unreachable for P <= 2^31) exact path
        if (c0 < a.P) {  // the children are inner nodes
            enter_descendants(std::integral_constant<int, 4>());
            continue;
        }
        // the left child shares the node's first leaf (non-empty); the right one may lie past L
        const float b0 = box_d2(qx, qy, qz, a.nlo[c0], a.nhi[c0]);
        const float b1 = first_leaf(c0 + 1, a.logP) < L ? box_d2(qx, qy, qz, a.nlo[c0 + 1], a.nhi[c0 + 1]) : INFINITY;
        const bool need0 = __builtin_amdgcn_ballot_w64(live && b0 < INFINITY && b0 * kShrink <= ub) != 0;
        const bool need1 = __builtin_amdgcn_ballot_w64(live && b1 < INFINITY && b1 * kShrink <= ub) != 0;
        // nearer child (for most live lanes) on top of the stack
        const int votes = __builtin_popcountll(__builtin_amdgcn_ballot_w64(live && b0 <= b1));
        const bool first0 = 2 * votes >= __builtin_popcountll(__builtin_amdgcn_ballot_w64(live));
        const int nearc = first0 ? c0 : c0 + 1, farc = first0 ? c0 + 1 : c0;
        const bool nn = first0 ? need0 : need1, nf = first0 ? need1 : need0;
        if (lane == 0) {
            if (nf) stk[sp] = farc;
            if (nn) stk[sp + (nf ? 1 : 0)] = nearc;
        }
        sp += (nf ? 1 : 0) + (nn ? 1 : 0);
        __builtin_amdgcn_wave_barrier();
    }

    // exact re-rank of the kept slots by (d2, id). The query itself gets the smallest key (it sits
    // in the run of d2 = 0 keys, so it moves to the front within the passes below) and is dropped
    // from the front; were it pushed out by more than K+M exact duplicates, nothing is dropped.
    unsigned long long e[KM];
    bool has_self = false;
#pragma unroll
    for (int j = 0; j < KM; ++j) {
        const unsigned key = keys[j];
        unsigned long long v = ~0ull;
        if (key != SENT) {
            const unsigned slot = key & kMask;
            const unsigned pidx = (unsigned)vis[slot >> kLeafBits] + (slot & ((1u << kLeafBits) - 1u));
            if (pidx != qpos) {
                const float4 c = a.pts[KN_IDX(pidx, (unsigned)a.n, 403)];
                const float dx = c.x - qx, dy = c.y - qy, dz = c.z - qz;
                v = pack_key64(fmaf(dz, dz, fmaf(dy, dy, dx * dx)), w_id(a, __float_as_uint(c.w)));
            } else {
                v = 0ull;
                has_self = true;
            }
        }
        e[j] = v;
    }
    // keys order the slots by truncated distance: only slots of equal truncation buckets can be
    // out of exact order, so a few odd-even passes sort them; checked below (else: exact finish)
#pragma unroll
    for (int r = 0; r < kSortPasses; ++r) {
#pragma unroll
        for (int j = r & 1; j + 1 < KM; j += 2) {
            const unsigned long long x = e[j], y = e[j + 1];
            const bool s = y < x;
            e[j] = s ? y : x;
            e[j + 1] = s ? x : y;
        }
    }
    bool sorted = true;
#pragma unroll
    for (int j = 0; j + 1 < KM; ++j) sorted = sorted && !(e[j + 1] < e[j]);
    const int k = a.k;
    const int off = has_self ? 1 : 0;
    unsigned long long ek = ~0ull;
    unsigned kb = SENT;
#pragma unroll
    for (int j = 0; j < KT + 2; ++j) {
        if (j == k - 1 + off) ek = e[j];
        if (j == k) kb = keys[j];
    }
    const unsigned last = keys[KM - 1];
    const bool full = last != SENT;
    // nothing truncated away (exact d2 >= its key's floor >= the last key's floor) can precede the
    // K-th exact neighbour when that lies strictly below the floor
    bool cert = !over && sorted &&
                (!full || (ek != ~0ull && __uint_as_float((unsigned)(ek >> 32)) < __uint_as_float(last & ~kMask)));
    if (a.flags & 1) cert = false;
    const unsigned long long unc = __builtin_amdgcn_ballot_w64(live && !cert);
    if (unc) {
        unsigned pos0 = 0;
        if (lane == 0) pos0 = atomicAdd(a.counters + 0, (unsigned)__builtin_popcountll(unc));
        pos0 = (unsigned)__builtin_amdgcn_readfirstlane((int)pos0);
        if (live && !cert) {
            const unsigned long long lt = (lane == 0) ? 0ull : (~0ull >> (64 - lane));
            const unsigned pos = pos0 + (unsigned)__builtin_popcountll(unc & lt);
            a.list[KN_IDX(pos, (unsigned)a.n, 404)] = qpos;
            // the K+1 smallest keys hold at most one self: a bound on the K-th distance
            a.thr[KN_IDX(pos, (unsigned)a.n, 405)] = kb == SENT ? INFINITY : __uint_as_float(kb | kMask);
        }
    }
    if (lane == 0) {
        if (over) atomicAdd(a.counters + 2, 1u);
        atomicAdd(a.counters + 5, (unsigned)nv);  // leaves visited
        atomicAdd(a.counters + 7, 1u);            // waves
    }
    if (unc) {  // causes (diagnostics): [3] re-rank left unsorted, [4] K-th not below the floor
        const unsigned nu = (unsigned)__builtin_popcountll(__builtin_amdgcn_ballot_w64(live && !over && !sorted));
        const unsigned nf = (unsigned)__builtin_popcountll(__builtin_amdgcn_ballot_w64(live && !over && sorted && !cert));
        if (lane == 0 && nu) atomicAdd(a.counters + 3, nu);
        if (lane == 0 && nf) atomicAdd(a.counters + 4, nf);
    }
    if (kStats) {
        const unsigned nets = (unsigned)__builtin_amdgcn_readfirstlane((int)nnet);
        if (lane == 0) atomicAdd(a.counters + 6, nets);
    }
    // KN_VEC_OUT (kn/knn_device.h): V positions of the row per global store when k % V == 0 and the
    // output pointers are V-aligned, instead of one scattered 4-byte store per entry and array
    constexpr int V = out_vec_width<KT>();
    const bool vec = out_vec_ok<V>(k, (const void*)o_idx, (const void*)o_dist);
    if (live && cert && vec) {
        const unsigned row = w_row(a, qw, a.row_of ? a.src[KN_IDX(qpos, (unsigned)a.n, 419)] : qpos);
#pragma unroll
        for (int j0 = 0; j0 < KT; j0 += V) {
            // a whole group, or (K % 4 == 2) the row's last two positions
            const bool whole = j0 + (V - 1) < k;
            if (whole || (V == 4 && KN_VEC_TAIL && j0 + 1 == k - 1)) {
                unsigned vi[V];
                float vd[V];
#pragma unroll
                for (int u = 0; u < V; ++u) {
                    const int j = j0 + u < KT ? j0 + u : KT - 1;
                    const unsigned long long v = has_self ? e[j + 1] : e[j];
                    const bool empty = v == ~0ull;
                    vi[u] = empty ? SENT : out_id(a, (unsigned)v);
                    vd[u] = empty ? INFINITY : __uint_as_float((unsigned)(v >> 32));
                }
                if (whole) {
                    const size_t o = KN_IDX((size_t)row * (size_t)k + j0 + (V - 1), (size_t)a.n_queries * k, 407) - (V - 1);
                    store_vec<V>(o_idx + o, vi);
                    if (o_dist) store_vec<V>(o_dist + o, vd);
                } else {
                    const size_t o = KN_IDX((size_t)row * (size_t)k + j0 + 1, (size_t)a.n_queries * k, 408) - 1;
                    const unsigned ti[2] = {vi[0], vi[1]};
                    const float td[2] = {vd[0], vd[1]};
                    store_vec<2>(o_idx + o, ti);
                    if (o_dist) store_vec<2>(o_dist + o, td);
                }
            }
        }
    } else if (live && cert) {
        const unsigned row = w_row(a, qw, a.row_of ? a.src[KN_IDX(qpos, (unsigned)a.n, 419)] : qpos);
#pragma unroll
        for (int j = 0; j < KT; ++j) {
            if (j < k) {
                const size_t o = KN_IDX((size_t)row * (size_t)k + j, (size_t)a.n_queries * k, 406);
                const unsigned long long v = has_self ? e[j + 1] : e[j];
                const bool empty = v == ~0ull;
                o_idx[o] = empty ? SENT : out_id(a, (unsigned)v);
                if (o_dist) o_dist[o] = empty ? INFINITY : __uint_as_float((unsigned)(v >> 32));
            }
        }
    }
}

// ---- exact finish: one wave per listed query (or every point: list == nullptr) ------------------
// Near-first traversal with the query's distance bound; every candidate with d2 <= thr is
// ballot-compacted into the wave's LDS buffer, which is bitonic-sorted by (d2, id) and cut to K
// (thr = K-th distance) when it could overflow -- the semantics of query.hip's exact kernel.
__global__ __launch_bounds__(256) void knn_tree_exact_kernel(TArgs a, int all) {
    // output pointers: the launch's, or read from device slots (graph replays of a batched
    // stream of clouds); locals, so the kernel argument block stays read-only
    out_u32_t* const o_idx = out_ptr(a.out_idx_ref ? *a.out_idx_ref : a.out_idx);
    out_f32_t* const o_dist = out_ptr(a.out_idx_ref ? (a.out_dist_ref ? *a.out_dist_ref : nullptr) : a.out_dist);
    __shared__ unsigned long long s_buf[4][kTCap];
    __shared__ int s_stack[4][kStack];
    __shared__ float s_sbd[4][kStack];  // box distance of each stacked node (computed by its parent)
    __shared__ int s_fr[4][2][kFrontier];
    __shared__ int s_lf[4][kFrontier];
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    unsigned long long* buf = s_buf[wid];
    int* stk = s_stack[wid];
    float* sbd = s_sbd[wid];
    const unsigned long long lt = (lane == 0) ? 0ull : (~0ull >> (64 - lane));
    const int total = all ? a.n : (int)a.counters[0];
    const int k = a.k;
    const int L = (int)*a.Lp;
    for (int t = blockIdx.x * 4 + wid; t < total; t += gridDim.x * 4) {
        const unsigned qpos = all ? (unsigned)t : (unsigned)__builtin_amdgcn_readfirstlane((int)a.list[KN_IDX(t, a.n, 411)]);
        const float4 qp = a.pts[KN_IDX(qpos, (unsigned)a.n, 412)];
        const unsigned qw = __float_as_uint(qp.w);
        if (!w_live(a, qw)) continue;
        const float qx = qp.x, qy = qp.y, qz = qp.z;
        float thr = all ? INFINITY : a.thr[KN_IDX(t, a.n, 413)];
        int cnt = 0;
        auto compact = [&]() __attribute__((always_inline)) {
            __builtin_amdgcn_wave_barrier();
            unsigned long long v[kTCap / 64];
#pragma unroll
            for (int e = 0; e < kTCap / 64; ++e) v[e] = (64 * e + lane < cnt) ? buf[64 * e + lane] : ~0ull;
            __builtin_amdgcn_wave_barrier();
            wave_bitonic_sort_u64<kTCap / 64>(v, lane);
#pragma unroll
            for (int e = 0; e < kTCap / 64; ++e)
                if (64 * e + lane < k) buf[64 * e + lane] = v[e];
            cnt = min(cnt, k);
            if (cnt >= k) {
                unsigned hb = 0;
#pragma unroll
                for (int e = 0; e < kTCap / 64; ++e)
                    if ((k - 1) / 64 == e) hb = (unsigned)__builtin_amdgcn_readlane((int)(unsigned)(v[e] >> 32), (k - 1) & 63);
                thr = __uint_as_float(hb);
            }
            __builtin_amdgcn_wave_barrier();
        };
        // A finite bound (listed queries: the (K+1)-th truncated key, rounded up) is already tight:
        // sweep the tree breadth-first, 64 nodes per step (one dependent global round per level
        // instead of per node), collect the leaves within the bound, then scan them 64 / kTreeLeaf
        // per step (one lane per point). The kept set is order-independent (the bound only ever
        // tightens to a K-th distance found, ties break by id), so rows equal the depth-first walk's. A
        // frontier or leaf list past kFrontier falls back to that walk.
        bool dfs = !(thr < INFINITY);
        if (!dfs) {
            int* cur = s_fr[wid][0];
            int* nxt = s_fr[wid][1];
            int* lfl = s_lf[wid];
            if (lane == 0) cur[0] = 1;
            int ncur = 1, nleaf = 0;
            __builtin_amdgcn_wave_barrier();
            while (ncur > 0 && !dfs) {
                int nn = 0;
                for (int i0 = 0; i0 < ncur; i0 += 64) {
                    const int i = i0 + lane;
                    const int node = i < ncur ? cur[i] : 0;
                    bool isleaf = false, p0 = false, p1 = false;
                    if (i < ncur) {
                        if (node >= a.P) {
                            isleaf = true;
                        } else {
                            const int c0 = 2 * node;
                            const float b0 = box_d2(qx, qy, qz, a.nlo[c0], a.nhi[c0]);
                            const float b1 = first_leaf(c0 + 1, a.logP) < L
                                                 ? box_d2(qx, qy, qz, a.nlo[c0 + 1], a.nhi[c0 + 1]) : INFINITY;
                            p0 = b0 < INFINITY && b0 * kShrink <= thr;
                            p1 = b1 < INFINITY && b1 * kShrink <= thr;
                        }
                    }
                    const unsigned long long bl = __builtin_amdgcn_ballot_w64(isleaf);
                    const unsigned long long q0 = __builtin_amdgcn_ballot_w64(p0);
                    const unsigned long long q1 = __builtin_amdgcn_ballot_w64(p1);
                    const int nl = __builtin_popcountll(bl), nc = __builtin_popcountll(q0) + __builtin_popcountll(q1);
                    if (nleaf + nl > kFrontier || nn + nc > kFrontier) { dfs = true; break; }
                    if (isleaf) lfl[nleaf + __builtin_popcountll(bl & lt)] = node - a.P;
                    const int off = nn + __builtin_popcountll(q0 & lt) + __builtin_popcountll(q1 & lt);
                    if (p0) nxt[off] = 2 * node;
                    if (p1) nxt[off + (p0 ? 1 : 0)] = 2 * node + 1;
                    nleaf += nl;
                    nn += nc;
                }
                __builtin_amdgcn_wave_barrier();
                int* t = cur; cur = nxt; nxt = t;
                ncur = nn;
            }
            if (!dfs) {
                // 64 / kTreeLeaf leaves per step, one lane per point
                constexpr int LPS = 64 / kTreeLeaf;
                const int grp = lane / kTreeLeaf, sub = lane % kTreeLeaf;
                for (int j = 0; j < nleaf; j += LPS) {
                    if (cnt + 64 > kTCap) compact();
                    bool pass = false;
                    unsigned long long key = 0;
                    if (j + grp < nleaf) {
                        const int lf = lfl[j + grp];
                        const int p = (int)a.leaf_start[lf] + sub;
                        if (p < (int)a.leaf_start[lf + 1] && (unsigned)p != qpos) {
                            const float4 c = a.pts[KN_IDX(p, a.n, 416)];
                            const float dx = c.x - qx, dy = c.y - qy, dz = c.z - qz;
                            const float d2 = fmaf(dz, dz, fmaf(dy, dy, dx * dx));
                            pass = d2 <= thr;
                            key = pack_key64(d2, w_id(a, __float_as_uint(c.w)));
                        }
                    }
                    const unsigned long long bal = __builtin_amdgcn_ballot_w64(pass);
                    if (pass) buf[cnt + __builtin_popcountll(bal & lt)] = key;
                    cnt += __builtin_popcountll(bal);
                }
            }
            __builtin_amdgcn_wave_barrier();
        }
        // one query per wave: box distances are wave-uniform, so a node's distance is stacked with
        // it by its parent and the pop re-tests it against the (possibly tighter) bound without
        // re-loading the node's box -- one dependent global round per node instead of two for a
        // lone, latency-bound wave. The root holds the query: distance 0.
        int sp = dfs ? 1 : 0;
        if (lane == 0) { stk[0] = 1; sbd[0] = 0.f; }
        __builtin_amdgcn_wave_barrier();
        while (sp > 0) {
            --sp;
            const int node = __builtin_amdgcn_readfirstlane(stk[sp]);
            const float bd = __int_as_float(__builtin_amdgcn_readfirstlane(__float_as_int(sbd[sp])));
            if (!(bd < INFINITY && bd * kShrink <= thr)) continue;
            if (node >= a.P) {
                if (cnt + 64 > kTCap) compact();
                const int lf = node - a.P;
                const int p = (int)a.leaf_start[lf] + lane;
                bool pass = false;
                unsigned long long key = 0;
                if (p < (int)a.leaf_start[lf + 1] && (unsigned)p != qpos) {
                    const float4 c = a.pts[KN_IDX(p, a.n, 414)];
                    const float dx = c.x - qx, dy = c.y - qy, dz = c.z - qz;
                    const float d2 = fmaf(dz, dz, fmaf(dy, dy, dx * dx));
                    pass = d2 <= thr;
                    key = pack_key64(d2, w_id(a, __float_as_uint(c.w)));
                }
                const unsigned long long bal = __builtin_amdgcn_ballot_w64(pass);
                if (pass) buf[cnt + __builtin_popcountll(bal & lt)] = key;
                cnt += __builtin_popcountll(bal);
                continue;
            }
            const int c0 = 2 * node;
            const float b0 = box_d2(qx, qy, qz, a.nlo[c0], a.nhi[c0]);
            const float b1 = first_leaf(c0 + 1, a.logP) < L ? box_d2(qx, qy, qz, a.nlo[c0 + 1], a.nhi[c0 + 1]) : INFINITY;
            const bool need0 = b0 < INFINITY && b0 * kShrink <= thr;
            const bool need1 = b1 < INFINITY && b1 * kShrink <= thr;
            const bool first0 = b0 <= b1;
            const int nearc = first0 ? c0 : c0 + 1, farc = first0 ? c0 + 1 : c0;
            const float nearb = first0 ? b0 : b1, farb = first0 ? b1 : b0;
            const bool nn = first0 ? need0 : need1, nf = first0 ? need1 : need0;
            if (lane == 0) {
                if (nf) { stk[sp] = farc; sbd[sp] = farb; }
                if (nn) { stk[sp + (nf ? 1 : 0)] = nearc; sbd[sp + (nf ? 1 : 0)] = nearb; }
            }
            sp += (nf ? 1 : 0) + (nn ? 1 : 0);
            __builtin_amdgcn_wave_barrier();
        }
        compact();
        const unsigned row = w_row(a, qw, a.row_of ? a.src[KN_IDX(qpos, (unsigned)a.n, 419)] : qpos);
        for (int j = lane; j < k; j += 64) {
            const size_t o = KN_IDX((size_t)row * (size_t)k + j, (size_t)a.n_queries * k, 415);
            const unsigned long long v = (j < cnt) ? buf[j] : ~0ull;
            const bool empty = (v == ~0ull);
            o_idx[o] = empty ? SENT : out_id(a, (unsigned)v);
            if (o_dist) o_dist[o] = empty ? INFINITY : __uint_as_float((unsigned)(v >> 32));
        }
        __builtin_amdgcn_wave_barrier();
    }
}

inline unsigned cdiv(size_t a, size_t b) { return (unsigned)((a + b - 1) / b); }
inline size_t align256(size_t b) { return (b + 255) & ~(size_t)255; }

}  // namespace

static int tree_pow2(int L) {
    int P = 1;
    while (P < L) P <<= 1;
    return P;
}
static int tree_log2(int P) { return 31 - __builtin_clz((unsigned)P); }

// padded brick space of a grid: (8^bb entries, bricks per axis)
static size_t brick_space(const int dims[3], int nb3[3]) {
    int m = 1;
    for (int a = 0; a < 3; ++a) {
        nb3[a] = std::max(1, (dims[a] + 7) / 8);
        m = std::max(m, nb3[a]);
    }
    const size_t side = (size_t)tree_pow2(m);
    return side * side * side;
}

size_t tree_workspace_bytes(int n, const int dims[3]) {
    if (n <= 0) return 256;
    int nb3[3];
    const size_t NB = brick_space(dims, nb3);
    const size_t sums = cdiv(std::max<size_t>(n, NB), kTScanItems) + 1;
    size_t b = align256((size_t)n * 16);         // pts
    b += 2 * align256(((size_t)n + 1) * 4);      // leaf_start, seg_start
    b += 4 * align256((size_t)n * 4);            // list, thr, flag, incl
    b += align256((size_t)n * 8);                // codes (u64)
    b += align256((size_t)n * 4);                // vals
    b += align256(16);                           // info
    b += align256((size_t)n * 16);               // tmp_pts
    b += align256((size_t)n * 4);                // tmp_vals
    b += align256((size_t)n * 8);                // cell_code (u64)
    b += align256((size_t)n * 8);                // cell_span
    b += align256((NB + 1) * 4);                 // brick counts -> bases
    b += align256(sums * 4);                     // scan block sums
    return b;
}

TreeView tree_view(void* ws, int n, const int dims[3]) {
    TreeView t{};
    t.n = std::max(n, 0);
    if (n <= 0) return t;
    char* p = static_cast<char*>(ws);
    auto take = [&](size_t bytes) { char* r = p; p += align256(bytes); return r; };
    t.pts = reinterpret_cast<float4*>(take((size_t)n * 16));
    t.leaf_start = reinterpret_cast<unsigned*>(take(((size_t)n + 1) * 4));
    t.seg_start = reinterpret_cast<unsigned*>(take(((size_t)n + 1) * 4));
    t.list = reinterpret_cast<unsigned*>(take((size_t)n * 4));
    t.thr = reinterpret_cast<float*>(take((size_t)n * 4));
    t.flag = reinterpret_cast<unsigned*>(take((size_t)n * 4));
    t.incl = reinterpret_cast<unsigned*>(take((size_t)n * 4));
    t.codes = reinterpret_cast<unsigned long long*>(take((size_t)n * 8));
    t.vals = reinterpret_cast<unsigned*>(take((size_t)n * 4));
    t.info = reinterpret_cast<unsigned*>(take(16));
    t.tmp_pts = reinterpret_cast<float4*>(take((size_t)n * 16));
    t.tmp_vals = reinterpret_cast<unsigned*>(take((size_t)n * 4));
    t.cell_code = reinterpret_cast<unsigned long long*>(take((size_t)n * 8));
    t.cell_span = reinterpret_cast<uint2*>(take((size_t)n * 8));
    for (int a = 0; a < 3; ++a) t.dims[a] = dims[a];
    t.nbricks_pad = brick_space(dims, t.nbricks);
    t.bcount = reinterpret_cast<unsigned*>(take((t.nbricks_pad + 1) * 4));
    t.scan_sums = reinterpret_cast<unsigned*>(take((cdiv(std::max<size_t>(n, t.nbricks_pad), kTScanItems) + 1) * 4));
    return t;
}

// the node buffer holds a tree over P = pow2 >= n leaf slots: every possible leaf count (a leaf
// holds >= 1 point) fits without knowing L on the host
size_t tree_node_bytes(int n) { return 2 * (size_t)tree_pow2(std::max(n, 1)) * 2 * sizeof(float4); }

void tree_attach_nodes(TreeView& t, void* nodes) {
    t.P = tree_pow2(std::max(t.n, 1));
    t.nlo = static_cast<float4*>(nodes);
    t.nhi = t.nlo + 2 * (size_t)t.P;
}

hipError_t launch_tree_leaves(const float4* in, const int* cell_start, const GridGeom* geom, const TreeView& t,
                              hipStream_t s) {
    const int n = t.n;
    if (n <= 0) return hipSuccess;
    if (!tree_supports(t.dims)) return hipErrorInvalidValue;
    hipError_t e;
    // Morton order of the cells (brick counts -> brick bases -> per-brick cell scan + copy)
    const unsigned nreal = (unsigned)(t.nbricks[0] * t.nbricks[1] * t.nbricks[2]);
    if ((e = hipMemsetAsync(t.bcount, 0, t.nbricks_pad * sizeof(unsigned), s)) != hipSuccess) return e;
    brick_count_kernel<<<nreal, 64, 0, s>>>(cell_start, geom, t.nbricks[0], t.nbricks[1], t.bcount);
    if ((e = tscan(t.bcount, (int)t.nbricks_pad, t.bcount, t.scan_sums, false, s)) != hipSuccess) return e;
    brick_scatter_kernel<<<nreal, 256, 0, s>>>(in, cell_start, geom, t.nbricks[0], t.nbricks[1], t.bcount,
                                               t.tmp_pts, t.tmp_vals, t.cell_code, t.cell_span);
    subcell_rank_kernel<<<cdiv(n, 256), 256, 0, s>>>(t.tmp_pts, t.tmp_vals, t.cell_code, t.cell_span, geom, n, t.pts,
                                                     t.vals, t.codes);
    // leaves: maximal prefix nodes of <= kTreeLeaf points, long equal-code runs chunked
    cut_kernel<<<cdiv(n, 256), 256, 0, s>>>(t.codes, n, t.flag);
    if ((e = tscan(t.flag, n, t.incl, t.scan_sums, true, s)) != hipSuccess) return e;
    starts_kernel<<<cdiv(n, 256), 256, 0, s>>>(t.flag, t.incl, n, t.seg_start, nullptr);
    leaf_flag_kernel<<<cdiv(n, 256), 256, 0, s>>>(t.incl, t.seg_start, n, t.flag);
    if ((e = tscan(t.flag, n, t.incl, t.scan_sums, true, s)) != hipSuccess) return e;
    starts_kernel<<<cdiv(n, 256), 256, 0, s>>>(t.flag, t.incl, n, t.leaf_start, t.info);
    return hipGetLastError();
}

hipError_t launch_tree_nodes(const TreeView& t, hipStream_t s) {
    if (t.n <= 0) return hipSuccess;
    if (!t.nlo) return hipErrorInvalidValue;
    const int logP = tree_log2(t.P);
    leaf_box_kernel<<<std::max(1u, std::min(cdiv(t.n, 4 * 8), 4096u)), 256, 0, s>>>(t.pts, t.leaf_start, t.info, t.P,
                                                                                     t.nlo, t.nhi);
    for (int m = t.P; m > 1; m /= std::min(m, 64))
        node_box_kernel<<<m / std::min(m, 64), 64, 0, s>>>(t.nlo, t.nhi, m, logP, t.info);
    return hipGetLastError();
}

hipError_t launch_tree_query(const TreeView& t, const TreeQuery& q, hipStream_t s) {
    if (q.k <= 0 || q.k > 128) return hipErrorInvalidValue;
    hipError_t e = hipMemsetAsync(q.counters, 0, kNumCounters * sizeof(unsigned), s);
    if (e != hipSuccess || t.n == 0 || q.n_queries == 0) return e;
    if (!t.nlo) return hipErrorInvalidValue;
    TArgs a{};
    a.pts = t.pts; a.leaf_start = t.leaf_start; a.nlo = t.nlo; a.nhi = t.nhi; a.list = t.list; a.thr = t.thr;
    a.Lp = t.info; a.n = t.n; a.P = t.P; a.logP = tree_log2(t.P);
    a.k = q.k; a.n_queries = q.n_queries; a.q_lo = 0; a.id_map = q.id_map;
    a.row_of = q.row_of; a.src = t.vals; a.out_idx = q.out_idx; a.out_dist = q.out_dist; a.counters = q.counters;
    a.out_idx_ref = q.out_idx_ref; a.out_dist_ref = q.out_dist_ref;
    a.flags = q.flags;
    constexpr int M = 2;
    const unsigned grid = cdiv(cdiv(t.n, 64), 4);
    const int k = q.k;
    bool all = false;
    if (k <= 4) knn_tree_kernel<4, M><<<grid, 256, 0, s>>>(a);
    else if (k <= 8) knn_tree_kernel<8, M><<<grid, 256, 0, s>>>(a);
    else if (k <= 12) knn_tree_kernel<12, M><<<grid, 256, 0, s>>>(a);
    else if (k <= 16) knn_tree_kernel<16, M><<<grid, 256, 0, s>>>(a);
    else if (k <= 24) knn_tree_kernel<24, M><<<grid, 256, 0, s>>>(a);
    else if (k <= 32) knn_tree_kernel<32, M><<<grid, 256, 0, s>>>(a);
    else if (k <= 40) knn_tree_kernel<40, M><<<grid, 256, 0, s>>>(a);
    else if (k <= 50) knn_tree_kernel<50, M><<<grid, 256, 0, s>>>(a);
    else if (k <= 64) knn_tree_kernel<64, M><<<grid, 256, 0, s>>>(a);
    else all = true;  // K > 64: the exact traversal serves every query
    if ((e = hipGetLastError()) != hipSuccess) return e;
    const unsigned eg = all ? std::max(1u, std::min(cdiv(t.n, 4), 16384u)) : (unsigned)kExactGrid;
    knn_tree_exact_kernel<<<eg, 256, 0, s>>>(a, all ? 1 : 0);
    return hipGetLastError();
}

hipError_t tree_leaf_count(const TreeView& t, unsigned* L, hipStream_t s) {
    *L = 0;
    if (t.n <= 0) return hipSuccess;
    hipError_t e = hipMemcpyAsync(L, t.info, sizeof(unsigned), hipMemcpyDeviceToHost, s);
    return e != hipSuccess ? e : hipStreamSynchronize(s);
}

KN_DEFINE_DEBUG_READER(debug_words_tree)

}  // namespace kn
