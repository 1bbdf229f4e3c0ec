// build.hip -- grid construction on gfx950 (wave64).
//
// Replaces the reference's count / reserve / store kernels (knearests.cu:32-60,152-201):
//  * bbox_kernel     : data-driven domain (reference hard-codes [0,1000]^3, knearests.cu:21)
//  * count_kernel    : per-point cell id + atomic *rank* capture, so the scatter needs no
//                      second atomic pass (reference re-zeroes and re-counts, :183-187)
//  * scan_*          : deterministic exclusive scan (reference uses an unordered atomic bump
//                      allocator, `reserve` :40-48, which scatters cells randomly in memory)
//  * scatter_kernel  : counting-sort scatter into float4 {x,y,z,bits(orig)} + permutation,
//                      and finalises cell_start in the same launch
//  * cell_sort_kernel: optional stable in-cell order (by original index) for bitwise
//                      reproducible output (reference order is nondeterministic, :56)
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdlib>

#include "kn/kernels.h"
#include "kn/route.h"
#include "kn/wave.h"

// A/B knobs of round-3 build variants (scripts/ab_build.py, profiles/ab_r3_build.jsonl; eager
// C.build, 900K K=16 / 12.5M):
//  * KN_BUILD_BATCH: bucket count / scatter load 4 points per thread before their LDS atomics
//    (3 float4 loads at a 48-B lane stride): 900K +2.1 us, 12.5M -1 % -> off
//  * KN_SORT_REGS: the bucket sort keeps its points in registers between its two passes:
//    900K -0.3 us, 12.5M -1.3 % -> on
//  * KN_BBOX_THREADS 1024 (one float4 triple per thread): 900K +2.0 us -> 256
#ifndef KN_BUILD_BATCH
#define KN_BUILD_BATCH 0
#endif
#ifndef KN_SORT_REGS
#define KN_SORT_REGS 1
#endif
#ifndef KN_BBOX_THREADS
#define KN_BBOX_THREADS 256
#endif

namespace kn {

namespace {

__device__ __forceinline__ unsigned ord_float(float f) {
    unsigned u = __float_as_uint(f);
    return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
}
__device__ __forceinline__ float unord_float(unsigned u) {
    return __uint_as_float((u & 0x80000000u) ? (u & 0x7fffffffu) : ~u);
}

// Per-block partial bbox (see launch_bbox_partials). VEC: 4 points = 3 aligned float4 loads
// per iteration (x0 y0 z0 x1 | y1 z1 x2 y2 | z2 x3 y3 z3); needs a 16-B aligned base.
template <bool VEC>
__global__ __launch_bounds__(KN_BBOX_THREADS) void bbox_partials_kernel(const float* __restrict__ pts, int n,
                                                            unsigned* __restrict__ partials,
                                                            int* __restrict__ zero_ints, int n_zero) {
    if (blockIdx.x == 0)
        for (int j = threadIdx.x; j < n_zero; j += blockDim.x) zero_ints[j] = 0;
    float mn[3] = {INFINITY, INFINITY, INFINITY};
    float mx[3] = {-INFINITY, -INFINITY, -INFINITY};
    auto acc = [&](int a, float v) { mn[a] = fminf(mn[a], v); mx[a] = fmaxf(mx[a], v); };
    const int tid = blockIdx.x * blockDim.x + threadIdx.x, nth = gridDim.x * blockDim.x;
    int i0 = tid;
    if (VEC) {
        const float4* p4 = reinterpret_cast<const float4*>(pts);
        const int ng = n >> 2;
        for (int g = tid; g < ng; g += nth) {
            const size_t g3 = 3 * (size_t)g;
            const float4 a = p4[g3], b = p4[g3 + 1], c = p4[g3 + 2];
            acc(0, a.x); acc(1, a.y); acc(2, a.z);
            acc(0, a.w); acc(1, b.x); acc(2, b.y);
            acc(0, b.z); acc(1, b.w); acc(2, c.x);
            acc(0, c.y); acc(1, c.z); acc(2, c.w);
        }
        i0 = 4 * ng + tid;
    }
    for (int i = i0; i < n; i += nth) {
        acc(0, pts[3 * (size_t)i]); acc(1, pts[3 * (size_t)i + 1]); acc(2, pts[3 * (size_t)i + 2]);
    }
    __shared__ unsigned red[6][16];
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
#pragma unroll
    for (int a = 0; a < 3; ++a) {
        const unsigned lo = wave_max_u32(~ord_float(mn[a]));
        const unsigned hi = wave_max_u32(ord_float(mx[a]));
        if (lane == 0) { red[a][wid] = lo; red[3 + a][wid] = hi; }
    }
    __syncthreads();
    if (threadIdx.x < 6) {
        unsigned v = red[threadIdx.x][0];
        for (int w = 1; w < (int)(blockDim.x >> 6); ++w) v = max(v, red[threadIdx.x][w]);
        partials[threadIdx.x * kBBoxBlocks + blockIdx.x] = v;
    }
}

__device__ void write_geom(GridGeom* g, const float lo[3], const float hi[3], const int dims[3]) {
    float maxext = 0.f;
    for (int a = 0; a < 3; ++a) maxext = fmaxf(maxext, hi[a] - lo[a]);
    if (!(maxext > 0.f)) maxext = 1.f;
    for (int a = 0; a < 3; ++a) {
        float ext = hi[a] - lo[a];
        // pad so that the max point falls strictly inside the last cell; keep degenerate
        // (flat) axes at a sane size relative to the cloud.
        ext = fmaxf(ext, maxext * 1e-3f);
        const float pad = ext * 1e-5f + fabsf(lo[a]) * 1e-6f + 1e-30f;
        const float o = lo[a] - pad;
        const float e = ext + 2.f * pad + fabsf(hi[a]) * 1e-6f;
        g->origin[a] = o;
        g->cell[a] = e / (float)dims[a];
        g->inv_cell[a] = (float)dims[a] / e;
        g->dims[a] = dims[a];
    }
    g->eps = maxext * 2e-6f + 1e-30f;
    g->pad = 0;
}

// Grid geometry from the bbox partials; called by one full wave (the reduction is wave-wide),
// every lane gets the same result.
__device__ void geom_from_partials(const unsigned* __restrict__ partials, int nblocks, const int dims[3],
                                   GridGeom* g) {
    unsigned words[6];
    bbox_reduce_partials(partials, nblocks, kBBoxBlocks, words);
    float lo[3], hi[3];
    for (int a = 0; a < 3; ++a) {
        lo[a] = unord_float(~words[a]);
        hi[a] = unord_float(words[3 + a]);
        if (!(hi[a] >= lo[a])) { lo[a] = 0.f; hi[a] = 1.f; }  // empty input
    }
    write_geom(g, lo, hi, dims);
}

__global__ void geom_kernel(const unsigned* __restrict__ partials, int nblocks, int d0, int d1, int d2,
                            GridGeom* g) {
    const int dims[3] = {d0, d1, d2};
    GridGeom t;
    geom_from_partials(partials, nblocks, dims, &t);  // wave 0 (the only one)
    if (threadIdx.x == 0 && blockIdx.x == 0) *g = t;
}

// Where the bucketed build's first kernel takes the grid geometry from (folded into it, so
// no separate geometry launch): a fixed box, or the bbox partials.
struct GeomSrc {
    const unsigned* partials;
    int nbb;
    int use_box;
    float lo[3], hi[3];
    int dims[3];
};

__global__ void geom_box_kernel(float l0, float l1, float l2, float h0, float h1, float h2, int d0,
                                int d1, int d2, GridGeom* g) {
    if (threadIdx.x != 0 || blockIdx.x != 0) return;
    const float lo[3] = {l0, l1, l2}, hi[3] = {h0, h1, h2};
    const int dims[3] = {d0, d1, d2};
    write_geom(g, lo, hi, dims);
}

__global__ __launch_bounds__(256) void count_kernel(const float* __restrict__ pts, int n,
                                                    const GridGeom* __restrict__ g,
                                                    int* __restrict__ cell_count,
                                                    int2* __restrict__ cell_rank) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const size_t i3 = 3 * (size_t)i;  // 64-bit: 3*i overflows int above 715M points
    const float p[3] = {pts[i3 + 0], pts[i3 + 1], pts[i3 + 2]};
    const int c = cell_of(*g, p);
    const int r = atomicAdd(cell_count + c, 1);
    cell_rank[i] = make_int2(c, r);
    (void)KN_IDX(c, g->dims[0] * g->dims[1] * g->dims[2], 101);
}

// Block-local exclusive scan of kScanItems ints (256 threads x 16 items), block total out.
__global__ __launch_bounds__(256) void scan_blocks_kernel(const int* __restrict__ in, int n,
                                                          int* __restrict__ out,
                                                          int* __restrict__ block_sums) {
    constexpr int T = 256, I = kScanItems / T;
    const int base = blockIdx.x * kScanItems + threadIdx.x * I;
    int v[I];
    if (base + I <= n) {
        const int4* p = reinterpret_cast<const int4*>(in + base);
#pragma unroll
        for (int j = 0; j < I / 4; ++j) {
            int4 q = p[j];
            v[4 * j] = q.x; v[4 * j + 1] = q.y; v[4 * j + 2] = q.z; v[4 * j + 3] = q.w;
        }
    } else {
#pragma unroll
        for (int j = 0; j < I; ++j) v[j] = (base + j < n) ? in[base + j] : 0;
    }
    int s = 0;
#pragma unroll
    for (int j = 0; j < I; ++j) { const int t = v[j]; v[j] = s; s += t; }
    // wave inclusive scan of the per-thread totals
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    const int incl = wave_inclusive_scan_add(s);
    __shared__ int wsum[4];
    if (lane == 63) wsum[wid] = incl;
    __syncthreads();
    int woff = 0;
    for (int w = 0; w < wid; ++w) woff += wsum[w];
    const int off = woff + incl - s;
    if (base + I <= n) {
        int4* p = reinterpret_cast<int4*>(out + base);
#pragma unroll
        for (int j = 0; j < I / 4; ++j)
            p[j] = make_int4(v[4 * j] + off, v[4 * j + 1] + off, v[4 * j + 2] + off, v[4 * j + 3] + off);
    } else {
#pragma unroll
        for (int j = 0; j < I; ++j)
            if (base + j < n) out[base + j] = v[j] + off;
    }
    if (threadIdx.x == T - 1) block_sums[blockIdx.x] = off + s;
}

// Single workgroup: exclusive scan of the block totals (any count, chunks of 1024).
__global__ __launch_bounds__(1024) void scan_top_kernel(int* __restrict__ sums, int nb) {
    __shared__ int wsum[16];
    __shared__ int carry_s;
    if (threadIdx.x == 0) carry_s = 0;
    __syncthreads();
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    for (int base = 0; base < nb; base += 1024) {
        const int i = base + threadIdx.x;
        const int v = (i < nb) ? sums[i] : 0;
        const int incl = wave_inclusive_scan_add(v);
        if (lane == 63) wsum[wid] = incl;
        __syncthreads();
        int woff = 0;
        for (int w = 0; w < wid; ++w) woff += wsum[w];
        const int carry = carry_s;
        if (i < nb) sums[i] = carry + woff + incl - v;
        __syncthreads();
        if (threadIdx.x == 1023) carry_s = carry + woff + incl;
        __syncthreads();
    }
    if (threadIdx.x == 0) sums[nb] = carry_s;
}

__global__ __launch_bounds__(256) void scatter_kernel(
    const float* __restrict__ pts, int n, const int2* __restrict__ cell_rank,
    const int* __restrict__ cell_scan, const int* __restrict__ block_sums, int num_cells,
    int* __restrict__ cell_start, float4* __restrict__ sorted, unsigned* __restrict__ perm) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) {
        const int2 cr = cell_rank[i];
        const int pos = KN_IDX(cell_scan[KN_IDX(cr.x, num_cells, 103)] + block_sums[cr.x / kScanItems] + cr.y, n, 102);
        const size_t i3 = 3 * (size_t)i;
        sorted[pos] = make_float4(pts[i3], pts[i3 + 1], pts[i3 + 2], __uint_as_float((unsigned)i));
        perm[pos] = (unsigned)i;
    }
    // finalise cell_start (grid-stride; the scatter grid has >= num_cells+1 threads only if
    // N >= C, so loop)
    for (int c = i; c <= num_cells; c += gridDim.x * blockDim.x) {
        cell_start[c] = (c < num_cells) ? cell_scan[c] + block_sums[c / kScanItems] : n;
    }
}

// One thread per cell: insertion sort of the cell's entries by original index.
__global__ __launch_bounds__(256) void cell_sort_kernel(const int* __restrict__ cell_start,
                                                        int num_cells, float4* __restrict__ sorted,
                                                        unsigned* __restrict__ perm) {
    const int c = blockIdx.x * blockDim.x + threadIdx.x;
    if (c >= num_cells) return;
    const int a = cell_start[c], b = cell_start[c + 1];
    (void)KN_IDX(b, a + 100000000, 105);
    for (int i = a + 1; i < b; ++i) {
        const float4 v = sorted[i];
        const unsigned key = __float_as_uint(v.w);
        int j = i - 1;
        while (j >= a && __float_as_uint(sorted[j].w) > key) {
            sorted[j + 1] = sorted[j];
            perm[j + 1] = perm[j];
            --j;
        }
        sorted[j + 1] = v;
        perm[j + 1] = key;
    }
}

// Deterministic in-cell order without a per-cell serial sort: every point counts the points of
// its cell with a smaller original index (its rank) and moves to cell start + rank in `tmp`; a
// copy pass writes the result back. O(sum over cells of count^2) = O(N x mean occupancy of a
// point's cell) work, all of it parallel (the one-thread-per-cell insertion sort is serial in the
// largest cell: 0.58 ms on a clustered cloud's 216-point cells).
__global__ __launch_bounds__(256) void cell_rank_kernel(const float4* __restrict__ sorted, const int* __restrict__ cell_start,
                                                        const GridGeom* __restrict__ gp, int n, float4* __restrict__ tmp) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const GridGeom g = *gp;
    const float4 v = sorted[i];
    const float p[3] = {v.x, v.y, v.z};
    const int c = cell_of(g, p);
    const int a = cell_start[c], b = cell_start[c + 1];
    const unsigned key = __float_as_uint(v.w);
    int r = 0;
    for (int j = a; j < b; ++j) r += __float_as_uint(sorted[j].w) < key ? 1 : 0;
    tmp[KN_IDX(a + r, n, 108)] = v;
}

__global__ void cell_copy_kernel(const float4* __restrict__ tmp, int n, float4* __restrict__ sorted,
                                 unsigned* __restrict__ perm) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const float4 v = tmp[i];
    sorted[i] = v;
    perm[i] = __float_as_uint(v.w);
}

__global__ __launch_bounds__(256) void cell_occupancy_kernel(const int* __restrict__ cell_start, int num_cells,
                                                             unsigned long long* __restrict__ out) {
    unsigned long long acc = 0;
    for (int c = blockIdx.x * blockDim.x + threadIdx.x; c < num_cells; c += gridDim.x * blockDim.x) {
        const unsigned long long cnt = (unsigned long long)(cell_start[c + 1] - cell_start[c]);
        acc += cnt * cnt;
    }
    // wave reduction (two 32-bit halves through DPP-free shuffles), then one atomic per wave
    for (int off = 32; off > 0; off >>= 1) {
        const unsigned lo = (unsigned)__shfl_xor((int)(unsigned)acc, off, 64);
        const unsigned hi = (unsigned)__shfl_xor((int)(unsigned)(acc >> 32), off, 64);
        acc += ((unsigned long long)hi << 32) | lo;
    }
    if ((threadIdx.x & 63) == 0 && acc) atomicAdd(out, acc);
}

__global__ __launch_bounds__(256) void cell_stats_kernel(const int* __restrict__ cell_start,
                                                         int num_cells, int* __restrict__ out,
                                                         int hist_len) {
    const int c = blockIdx.x * blockDim.x + threadIdx.x;
    if (c >= num_cells) return;
    const int cnt = cell_start[c + 1] - cell_start[c];
    atomicMin(out + 0, cnt);
    atomicMax(out + 1, cnt);
    if (cnt == 0) atomicAdd(out + 2, 1);
    atomicAdd(out + 3 + min(cnt, hist_len - 1), 1);
}

inline unsigned cdiv(size_t a, size_t b) { return (unsigned)((a + b - 1) / b); }

}  // namespace

size_t scan_block_count(int num_cells) { return cdiv((size_t)num_cells, kScanItems); }

int bbox_block_count(int n) {
    return std::max(1, std::min((int)cdiv((size_t)std::max(n, 0), KN_BBOX_THREADS == 1024 ? 1024 * 4 : 256 * 8),
                                kBBoxBlocks));
}

hipError_t launch_bbox_partials(const float* pts, int n, unsigned* partials, hipStream_t s, int* zero_ints,
                                int n_zero) {
    if (n <= 0) return hipSuccess;
    const int grid = bbox_block_count(n);
    if (!zero_ints) n_zero = 0;
    if ((reinterpret_cast<uintptr_t>(pts) & 15u) == 0)
        bbox_partials_kernel<true><<<grid, KN_BBOX_THREADS, 0, s>>>(pts, n, partials, zero_ints, n_zero);
    else
        bbox_partials_kernel<false><<<grid, KN_BBOX_THREADS, 0, s>>>(pts, n, partials, zero_ints, n_zero);
    return hipGetLastError();
}

// ---- bucketed binning ---------------------------------------------------------------
// A streaming block's points [i0, i1) (i0 a multiple of 4), 4 per thread and pass: thread t
// takes points i0 + 4 (t + j blockDim) .. +3 -- 3 aligned float4 loads when the base is 16-B
// aligned and the group is whole -- so every load of a pass is in flight before the first LDS
// atomic (the compiler does not hoist global loads over LDS atomics by itself).
struct Pts4 {
    float p[4][3];
    int i;  // first point index; points i..i+3 valid below `lim`
};
__device__ __forceinline__ void load_pts4(const float* __restrict__ pts, int i, int i1, bool vec, Pts4& q) {
    q.i = i;
    if (vec && i + 4 <= i1) {
        const float4* p4 = reinterpret_cast<const float4*>(pts + 3 * (size_t)i);
        const float4 a = p4[0], b = p4[1], c = p4[2];
        q.p[0][0] = a.x; q.p[0][1] = a.y; q.p[0][2] = a.z;
        q.p[1][0] = a.w; q.p[1][1] = b.x; q.p[1][2] = b.y;
        q.p[2][0] = b.z; q.p[2][1] = b.w; q.p[2][2] = c.x;
        q.p[3][0] = c.y; q.p[3][1] = c.z; q.p[3][2] = c.w;
    } else {
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            const size_t j = 3 * (size_t)min(i + u, i1 - 1);
            q.p[u][0] = pts[j]; q.p[u][1] = pts[j + 1]; q.p[u][2] = pts[j + 2];
        }
    }
}

// Bucket offsets without a table scan (KN_BIN_ATOMIC, default): every streaming block claims its
// sub-range of every bucket with ONE device-scope atomicAdd on the bucket's total (the returned old
// total is the block's offset inside the bucket, in arrival order); the scatter blocks scan the
// <= 4096 bucket totals themselves, so the build has no scan kernel between count and scatter.
// The totals are zeroed by the bbox kernel (or a memset with a fixed box) earlier in the same
// build. Bucket segments hold their blocks' points in arrival order; the bucket sort places them
// with LDS atomics anyway (the in-cell order is only fixed by the deterministic cell sort).
// KN_BIN_ATOMIC=0: the bucket-major table + scan_blocks_kernel of rounds 2-5.
// KN_BIN_PREFETCH: points per thread the count / scatter blocks load before their set-up
// (geometry, bucket offsets), so the load latency overlaps it.
#ifndef KN_BIN_ATOMIC
#define KN_BIN_ATOMIC 1
#endif
#ifndef KN_BIN_PREFETCH
#define KN_BIN_PREFETCH 4
#endif

template <int R>
struct PrefetchPts {
    float p[R > 0 ? R : 1][3];
    __device__ __forceinline__ void load(const float* __restrict__ pts, int i0, int i1) {
#pragma unroll
        for (int r = 0; r < R; ++r) {
            const size_t j = 3 * (size_t)min(i0 + (int)threadIdx.x + r * (int)blockDim.x, i1 - 1);
            p[r][0] = pts[j]; p[r][1] = pts[j + 1]; p[r][2] = pts[j + 2];
        }
    }
    // first index the plain loop continues at
    __device__ __forceinline__ static int rest(int i0) { return i0 + (int)threadIdx.x + R * (int)blockDim.x; }
    __device__ __forceinline__ static bool valid(int i0, int i1, int r) {
        return i0 + (int)threadIdx.x + r * (int)blockDim.x < i1;
    }
};

// A1: per-(bucket, block) counts with LDS atomics. KN_BIN_ATOMIC: block-major offsets
// table[block][bucket] from the totals' atomics; else the bucket-major count table (its exclusive
// scan gives every block its write offset inside every bucket).
__global__ __launch_bounds__(1024) void bucket_count_kernel(const float* __restrict__ pts, int n, GeomSrc src,
                                                           GridGeom* __restrict__ gout, int shift,
                                                           int nbuckets, int nblocks, int per_block,
                                                           int* __restrict__ table, int* __restrict__ totals,
                                                           unsigned* __restrict__ zero_words, int n_zero_words) {
    extern __shared__ int hist[];
    __shared__ GridGeom gs;
    const int i0 = blockIdx.x * per_block, i1 = min(n, i0 + per_block);
#if !KN_BUILD_BATCH
    constexpr int R = KN_BIN_PREFETCH;
    PrefetchPts<R> pf;
    pf.load(pts, i0, i1);
#endif
    // the step's query counters, zeroed here instead of by a separate memset node
    if (blockIdx.x == 0 && (int)threadIdx.x < n_zero_words) zero_words[threadIdx.x] = 0u;
    for (int j = threadIdx.x; j < nbuckets; j += blockDim.x) hist[j] = 0;
    if (threadIdx.x < 64) {  // every block derives the geometry; block 0 publishes it
        GridGeom t;
        if (src.use_box) write_geom(&t, src.lo, src.hi, src.dims);
        else geom_from_partials(src.partials, src.nbb, src.dims, &t);
        if (threadIdx.x == 0) {
            gs = t;
            if (blockIdx.x == 0) *gout = t;
        }
    }
    __syncthreads();
    const GridGeom g = gs;
#if KN_BUILD_BATCH
    const bool vec = (reinterpret_cast<uintptr_t>(pts) & 15u) == 0;
    for (int i = i0 + 4 * threadIdx.x; i < i1; i += 4 * blockDim.x) {
        Pts4 q;
        load_pts4(pts, i, i1, vec, q);
#pragma unroll
        for (int u = 0; u < 4; ++u)
            if (i + u < i1) atomicAdd(&hist[cell_of(g, q.p[u]) >> shift], 1);
    }
#else
#pragma unroll
    for (int r = 0; r < R; ++r)
        if (pf.valid(i0, i1, r)) atomicAdd(&hist[cell_of(g, pf.p[r]) >> shift], 1);
    for (int i = pf.rest(i0); i < i1; i += blockDim.x) {
        const float p[3] = {pts[3 * (size_t)i], pts[3 * (size_t)i + 1], pts[3 * (size_t)i + 2]};
        atomicAdd(&hist[cell_of(g, p) >> shift], 1);
    }
#endif
    __syncthreads();
#if KN_BIN_ATOMIC
    int* row = table + (size_t)blockIdx.x * nbuckets;
    for (int j = threadIdx.x; j < nbuckets; j += blockDim.x) {
        const int h = hist[j];
        row[j] = h ? atomicAdd(&totals[j], h) : 0;
    }
#else
    (void)totals;
    for (int j = threadIdx.x; j < nbuckets; j += blockDim.x) table[(size_t)j * nblocks + blockIdx.x] = hist[j];
#endif
}

// A3: every point to its bucket's segment of bin_tmp as {x, y, z, bits(original index)}.
// KN_BIN_ATOMIC: the block scans the bucket totals (-> bucket starts; block 0 publishes them in
// bstart[0..nbuckets], bstart[nbuckets] = n, for the bucket sort) and adds its own offsets.
__global__ __launch_bounds__(1024) void bucket_scatter_kernel(const float* __restrict__ pts, int n,
                                                             const GridGeom* __restrict__ gp, int shift,
                                                             int nbuckets, int nblocks, int per_block,
                                                             const int* __restrict__ tscan,
                                                             const int* __restrict__ tsums, int nbt,
                                                             const int* __restrict__ totals,
                                                             int* __restrict__ bstart,
                                                             float4* __restrict__ tmp) {
    extern __shared__ int cur[];
    const int i0 = blockIdx.x * per_block, i1 = min(n, i0 + per_block);
#if !KN_BUILD_BATCH
    constexpr int R = KN_BIN_PREFETCH;
    PrefetchPts<R> pf;
    pf.load(pts, i0, i1);
#endif
#if KN_BIN_ATOMIC
    (void)tscan; (void)tsums; (void)nbt; (void)nblocks;
    {
        // thread t owns buckets [t * per, t * per + per), per <= 16 (nbuckets <= 4096, >= 256 threads)
        __shared__ int wsum[16];
        const int per = (nbuckets + (int)blockDim.x - 1) / (int)blockDim.x;
        const int j0 = threadIdx.x * per;
        const int* mine = tscan + (size_t)blockIdx.x * nbuckets;  // this block's offsets (count kernel)
        int tv[16], ov[16];
        int s = 0;
#pragma unroll
        for (int q = 0; q < 16; ++q) {
            const bool v = q < per && j0 + q < nbuckets;
            tv[q] = v ? totals[j0 + q] : 0;
            ov[q] = v ? mine[j0 + q] : 0;
            s += tv[q];
        }
        const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
        const int incl = wave_inclusive_scan_add(s);
        if (lane == 63) wsum[wid] = incl;
        __syncthreads();
        int run = incl - s;
        for (int w = 0; w < wid; ++w) run += wsum[w];
#pragma unroll
        for (int q = 0; q < 16; ++q) {
            if (q < per && j0 + q < nbuckets) {
                cur[j0 + q] = run + ov[q];
                if (blockIdx.x == 0) bstart[j0 + q] = run;
                run += tv[q];
            }
        }
        if (blockIdx.x == 0 && threadIdx.x == 0) bstart[nbuckets] = n;
    }
#else
    (void)totals; (void)bstart;
    __shared__ int pre[1024];  // exclusive prefix of the scan blocks' totals (nbt <= 1024)
    if (threadIdx.x < 64) {
        const int per = (nbt + 63) >> 6, j0 = threadIdx.x * per;
        int s = 0;
        for (int j = 0; j < per; ++j) s += (j0 + j < nbt) ? tsums[j0 + j] : 0;
        int run = wave_inclusive_scan_add(s) - s;
        for (int j = 0; j < per; ++j)
            if (j0 + j < nbt) { pre[j0 + j] = run; run += tsums[j0 + j]; }
    }
    __syncthreads();
    for (int j = threadIdx.x; j < nbuckets; j += blockDim.x) {
        const size_t t = (size_t)j * nblocks + blockIdx.x;
        cur[j] = tscan[t] + pre[t / kScanItems];
    }
#endif
    __syncthreads();
    const GridGeom g = *gp;
#if KN_BUILD_BATCH
    const bool vec = (reinterpret_cast<uintptr_t>(pts) & 15u) == 0;
    for (int i = i0 + 4 * threadIdx.x; i < i1; i += 4 * blockDim.x) {
        Pts4 q;
        load_pts4(pts, i, i1, vec, q);
        int pos[4];
#pragma unroll
        for (int u = 0; u < 4; ++u)
            pos[u] = (i + u < i1) ? atomicAdd(&cur[cell_of(g, q.p[u]) >> shift], 1) : -1;
#pragma unroll
        for (int u = 0; u < 4; ++u)
            if (pos[u] >= 0)
                tmp[KN_IDX(pos[u], n, 104)] =
                    make_float4(q.p[u][0], q.p[u][1], q.p[u][2], __uint_as_float((unsigned)(i + u)));
    }
#else
    int pos[R > 0 ? R : 1];
#pragma unroll
    for (int r = 0; r < R; ++r)
        pos[r] = pf.valid(i0, i1, r) ? atomicAdd(&cur[cell_of(g, pf.p[r]) >> shift], 1) : -1;
#pragma unroll
    for (int r = 0; r < R; ++r)
        if (pos[r] >= 0)
            tmp[KN_IDX(pos[r], n, 104)] = make_float4(pf.p[r][0], pf.p[r][1], pf.p[r][2],
                                                      __uint_as_float((unsigned)(i0 + (int)threadIdx.x + r * (int)blockDim.x)));
    for (int i = pf.rest(i0); i < i1; i += blockDim.x) {
        const float p[3] = {pts[3 * (size_t)i], pts[3 * (size_t)i + 1], pts[3 * (size_t)i + 2]};
        const int pos = atomicAdd(&cur[cell_of(g, p) >> shift], 1);
        tmp[KN_IDX(pos, n, 104)] = make_float4(p[0], p[1], p[2], __uint_as_float((unsigned)i));
    }
#endif
}

// B: one workgroup per bucket: LDS histogram of its 2^shift cells, LDS exclusive scan ->
// cell_start, then every point to its final slot (LDS cursor atomics).
__global__ __launch_bounds__(256) void bucket_sort_kernel(const float4* __restrict__ tmp, int n,
                                                          const GridGeom* __restrict__ gp, int shift,
                                                          int nbuckets, int nblocks,
                                                          const int* __restrict__ tscan,
                                                          const int* __restrict__ tsums,
                                                          const int* __restrict__ bstart, int num_cells,
                                                          int* __restrict__ cell_start,
                                                          float4* __restrict__ sorted,
                                                          unsigned* __restrict__ perm,
                                                          const int* __restrict__ gids, int n_owned) {
    extern __shared__ int cur[];  // 2^shift cells
    __shared__ int wsum[4];
    __shared__ int seg[2];
    const int b = blockIdx.x;
    const int cells = 1 << shift;
    const int c0 = b << shift;
    for (int j = threadIdx.x; j < cells; j += 256) cur[j] = 0;
#if KN_BIN_ATOMIC
    (void)tscan; (void)tsums;
    if (threadIdx.x == 0) {  // bucket segment [bs, be): the starts the scatter's block 0 published
        seg[0] = bstart[b];
        seg[1] = bstart[b + 1];
    }
#else
    (void)bstart;
    if (threadIdx.x < 64) {  // bucket segment [bs, be): scanned table + prefix of raw block totals
        const size_t t0 = (size_t)b * nblocks, t1 = (size_t)(b + 1) * nblocks;
        const int i0 = (int)(t0 / kScanItems);
        const int i1 = (b + 1 < nbuckets) ? (int)(t1 / kScanItems) : 0;
        int s0 = 0, s1 = 0;
        for (int j = threadIdx.x; j < max(i0, i1); j += 64) {
            const int v = tsums[j];
            s0 += j < i0 ? v : 0;
            s1 += j < i1 ? v : 0;
        }
        s0 = __shfl(wave_inclusive_scan_add(s0), 63, 64);
        s1 = __shfl(wave_inclusive_scan_add(s1), 63, 64);
        if (threadIdx.x == 0) {
            seg[0] = tscan[t0] + s0;
            seg[1] = (b + 1 < nbuckets) ? tscan[t1] + s1 : n;
        }
    }
#endif
    __syncthreads();
    const int bs = seg[0], be = seg[1];
    const GridGeom g = *gp;
    // the bucket's first R x 256 points stay in registers between the two passes (a bucket holds
    // ~2^shift x points-per-cell points: all of them at the usual densities); all R loads are
    // issued before the first LDS atomic
    constexpr int R = KN_SORT_REGS ? 4 : 0;
    float4 v[R > 0 ? R : 1];
    int cl[R > 0 ? R : 1];
#pragma unroll
    for (int r = 0; r < R; ++r) {
        const int k = bs + threadIdx.x + r * 256;
        v[r] = k < be ? tmp[KN_IDX(k, n, 105)] : make_float4(0.f, 0.f, 0.f, 0.f);
    }
#pragma unroll
    for (int r = 0; r < R; ++r) {
        const float p[3] = {v[r].x, v[r].y, v[r].z};
        cl[r] = bs + threadIdx.x + r * 256 < be ? KN_IDX(cell_of(g, p) - c0, cells, 106) : -1;
        if (cl[r] >= 0) atomicAdd(&cur[cl[r]], 1);
    }
    for (int k = bs + threadIdx.x + R * 256; k < be; k += 256) {
        const float4 w = tmp[KN_IDX(k, n, 105)];
        const float p[3] = {w.x, w.y, w.z};
        atomicAdd(&cur[KN_IDX(cell_of(g, p) - c0, cells, 106)], 1);
    }
    __syncthreads();
    // exclusive scan of cur[0, cells): thread t owns `per` consecutive cells
    const int per = cells >> 8;
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    int s = 0;
    for (int j = 0; j < per; ++j) s += cur[threadIdx.x * per + j];
    const int incl = wave_inclusive_scan_add(s);
    if (lane == 63) wsum[wid] = incl;
    __syncthreads();
    int run = incl - s;
    for (int w = 0; w < wid; ++w) run += wsum[w];
    for (int j = 0; j < per; ++j) {
        const int c = threadIdx.x * per + j;
        const int cnt = cur[c];
        cur[c] = bs + run;
        if (c0 + c < num_cells) cell_start[c0 + c] = bs + run;
        run += cnt;
    }
    if (b == nbuckets - 1 && threadIdx.x == 0) cell_start[num_cells] = n;
    __syncthreads();
    auto place = [&](const float4& w, int pos) {
        const unsigned local = __float_as_uint(w.w);
        float4 o = w;
        if (gids) {  // global-id mode (see BuildBuffers::gids)
            // (A/B: carrying the ids through the bucket scatter instead -- a second scattered store
            // stream -- cost 4 us more at 900K than this gather)
            const unsigned gid = (unsigned)gids[KN_IDX(local, (unsigned)n, 108)];
            o.w = __uint_as_float((gid & 0x7FFFFFFFu) | ((int)local >= n_owned ? 0x80000000u : 0u));
        }
        sorted[KN_IDX(pos, n, 107)] = o;
        perm[pos] = local;
    };
#pragma unroll
    for (int r = 0; r < R; ++r)
        if (cl[r] >= 0) place(v[r], atomicAdd(&cur[cl[r]], 1));
    for (int k = bs + threadIdx.x + R * 256; k < be; k += 256) {
        const float4 w = tmp[KN_IDX(k, n, 105)];
        const float p[3] = {w.x, w.y, w.z};
        place(w, atomicAdd(&cur[cell_of(g, p) - c0], 1));
    }
}

// ---- small clouds: the whole build in ONE workgroup (no inter-kernel round trips) ----------------
// For small clouds the multi-kernel build is latency-bound (pts20K: 5 kernels, ~30 us for ~1 us of
// bandwidth). One 1024-thread workgroup instead: every thread loads its <= kSmallP points ONCE
// (all loads in flight together) and keeps them in registers through the bbox (block
// reduction, the same geometry function as the multi-block path), the LDS cell histogram and
// scan (-> cell_start) and the LDS-cursor scatter of point indices into an LDS slot array; each
// cell's slots are then ordered by original index in LDS (thread per cell) and the rows are
// written with one gather. The layout is that of the deterministic multi-kernel build, so the
// queries see identical input. LDS: C counts + n slots (small_build_fits).
constexpr int kSmallP = 24;                  // points per thread (registers): n <= 24576
constexpr int kSmallLdsWords = 150 * 256;    // 150 KB of the 160 KB LDS
bool small_build_fits(int n, int C) {
    return n > 0 && n <= 1024 * kSmallP && (size_t)C + (size_t)n <= (size_t)kSmallLdsWords;
}
__global__ __launch_bounds__(1024) void small_build_kernel(const float* __restrict__ pts, int n, int d0, int d1, int d2,
                                                           int use_box, float bl0, float bl1, float bl2, float bh0,
                                                           float bh1, float bh2, GridGeom* __restrict__ geom,
                                                           int* __restrict__ cell_start, float4* __restrict__ sorted,
                                                           unsigned* __restrict__ perm, unsigned* __restrict__ zero_words,
                                                           int n_zero) {
    extern __shared__ int sm[];
    const int C = d0 * d1 * d2;
    int* cnt = sm;      // C: counts, then cursors
    int* slot = sm + C; // n: original index of every stored slot
    __shared__ unsigned red[6][16];
    __shared__ int wsum[16];
    __shared__ GridGeom sg;
    const int t = threadIdx.x, lane = t & 63, wid = t >> 6;
    if (t < n_zero) zero_words[t] = 0u;
    float p[kSmallP][3];
#pragma unroll
    for (int j = 0; j < kSmallP; ++j) {
        const int i = min(t + 1024 * j, n - 1);  // clamped: duplicates of the last point are harmless
        p[j][0] = pts[3 * (size_t)i];
        p[j][1] = pts[3 * (size_t)i + 1];
        p[j][2] = pts[3 * (size_t)i + 2];
    }
    for (int c = t; c < C; c += 1024) cnt[c] = 0;
    // 1. bbox -> geometry
    if (!use_box) {
#pragma unroll
        for (int a = 0; a < 3; ++a) {
            float mn = INFINITY, mx = -INFINITY;
#pragma unroll
            for (int j = 0; j < kSmallP; ++j) { mn = fminf(mn, p[j][a]); mx = fmaxf(mx, p[j][a]); }
            const unsigned lo = wave_max_u32(~ord_float(mn)), hi = wave_max_u32(ord_float(mx));
            if (lane == 0) { red[a][wid] = lo; red[3 + a][wid] = hi; }
        }
    }
    __syncthreads();
    if (t == 0) {
        float lo[3], hi[3];
        const int dims[3] = {d0, d1, d2};
        if (use_box) {
            lo[0] = bl0; lo[1] = bl1; lo[2] = bl2; hi[0] = bh0; hi[1] = bh1; hi[2] = bh2;
        } else {
            for (int a = 0; a < 3; ++a) {
                unsigned wl = 0, wh = 0;
                for (int w = 0; w < 16; ++w) { wl = max(wl, red[a][w]); wh = max(wh, red[3 + a][w]); }
                lo[a] = unord_float(~wl);
                hi[a] = unord_float(wh);
            }
        }
        write_geom(&sg, lo, hi, dims);
        *geom = sg;
    }
    __syncthreads();
    const GridGeom g = sg;
    // 2. histogram (cells stay in registers)
    int cl[kSmallP];
#pragma unroll
    for (int j = 0; j < kSmallP; ++j) {
        cl[j] = t + 1024 * j < n ? cell_of(g, p[j]) : -1;
        if (cl[j] >= 0) atomicAdd(&cnt[cl[j]], 1);
    }
    __syncthreads();
    // 3. exclusive scan (each thread a contiguous run of cells) -> cell_start, cursors
    const int per = (C + 1023) / 1024, c0 = min(C, t * per), c1 = min(C, c0 + per);
    int s = 0;
    for (int c = c0; c < c1; ++c) s += cnt[c];
    const int incl = wave_inclusive_scan_add(s);
    if (lane == 63) wsum[wid] = incl;
    __syncthreads();
    int off = incl - s;
    for (int w = 0; w < wid; ++w) off += wsum[w];
    for (int c = c0; c < c1; ++c) {
        const int v = cnt[c];
        cell_start[c] = off;
        cnt[c] = off;
        off += v;
    }
    if (t == 1023) cell_start[C] = off;
    __syncthreads();
    // 4. scatter of indices (LDS cursors)
#pragma unroll
    for (int j = 0; j < kSmallP; ++j)
        if (cl[j] >= 0) slot[atomicAdd(&cnt[cl[j]], 1)] = t + 1024 * j;
    __syncthreads();
    // 5. in-cell order by original index: cnt[c] is now the cell's end, its start the previous
    //    cell's end (insertion sort in LDS; cells hold a few points)
    for (int c = t; c < C; c += 1024) {
        const int a = c ? cnt[c - 1] : 0, b = cnt[c];
        for (int i = a + 1; i < b; ++i) {
            const int key = slot[i];
            int j = i - 1;
            while (j >= a && slot[j] > key) {
                slot[j + 1] = slot[j];
                --j;
            }
            slot[j + 1] = key;
        }
    }
    __syncthreads();
    // 6. rows: one gather (all loads of a thread in flight together)
#pragma unroll
    for (int j = 0; j < kSmallP; ++j) {
        const int pos = t + 1024 * j;
        if (pos < n) {
            const int i = slot[pos];
            sorted[pos] = make_float4(pts[3 * (size_t)i], pts[3 * (size_t)i + 1], pts[3 * (size_t)i + 2],
                                      __uint_as_float((unsigned)i));
            perm[pos] = (unsigned)i;
        }
    }
}

hipError_t launch_cell_sort(const int* cell_start, const GridGeom* geom, int n, float4* sorted, unsigned* perm,
                            float4* tmp, hipStream_t s) {
    if (n <= 0) return hipSuccess;
    cell_rank_kernel<<<cdiv(n, 256), 256, 0, s>>>(sorted, cell_start, geom, n, tmp);
    cell_copy_kernel<<<cdiv(n, 256), 256, 0, s>>>(tmp, n, sorted, perm);
    return hipGetLastError();
}

bool bin_plan(int n, int num_cells, BinPlan* out, int items_req) {
    if (n <= 0 || num_cells <= 0) return false;
    // Points per streaming block (KN_BIN_ITEMS overrides): ~64 blocks up to 4M points (the power
    // of two nearest n / 64, within 4096..16384), 4096 above. Beside the running query kernels a
    // few large 256-thread blocks finish sooner than many small ones: 900K K=16 20 / 5 steps 0.282
    // -> 0.273 ms, 200 / 50 0.244 -> 0.241 (three sets), world-1 distributed 0.270 -> 0.262; 300K
    // and pts20K want 4096 (16384: +9 % / +31 %); 10M equal (profiles/ab_r5_bin_items.txt)
    static const int items_env = [] {
        const char* v = std::getenv("KN_BIN_ITEMS");
        const int t = v ? std::atoi(v) : 0;
        return (t >= 512 && t <= 65536) ? t : 0;
    }();
    // (above 4M points, 1024-thread blocks of 16384 points: 12.5M K=16 distributed share 4.616
    // -> 4.554 ms, 10M K=32 equal; profiles/ab_r5_bin_items.txt)
    int items = items_env ? items_env : items_req;
    if (!items) {
        items = 16384;
        if (n <= (4 << 20)) {
            const double l = std::log2(std::max(1.0, (double)n / 64.0));
            items = 1 << std::max(12, std::min(14, (int)std::lround(l)));
        }
    }
    const int nblocks = std::max(1, std::min((int)cdiv((size_t)n, (size_t)items), 1024));
    const int per_block = (int)(cdiv(cdiv((size_t)n, nblocks), 256) * 256);
    for (int shift = 8; shift <= 14; ++shift) {
        const long long nbuckets = ((long long)num_cells + (1ll << shift) - 1) >> shift;
        if (nbuckets > 4096) continue;
        if (nbuckets * nblocks > (long long)num_cells + 1) continue;
        if (2 * nbuckets + 2 > (long long)num_cells + 1) continue;  // bucket totals + starts (KN_BIN_ATOMIC)
        *out = BinPlan{shift, (int)nbuckets, (int)cdiv((size_t)n, per_block), per_block};
        return true;
    }
    return false;
}

hipError_t launch_build(const BuildBuffers& b, hipStream_t s) {
    const int C = b.dims[0] * b.dims[1] * b.dims[2];
    const int n = b.n;
    hipError_t e;
    BinPlan bp{};
    static const bool force_atomic = [] {
        const char* v = std::getenv("KN_BUILD_ALGO");
        return v && std::atoi(v) == 1;
    }();
    // KN_SMALL_BUILD=1: the one-workgroup build below for small clouds (read per launch: tests A/B
    // both paths). Off by default: measured on MI355X it takes 42 us for pts20K where the
    // multi-kernel build takes 25-27 us (step 0.107 vs 0.089 ms serial, equal when pipelined;
    // profiles/ab_r3_small_cloud.jsonl)
    const char* small_env = std::getenv("KN_SMALL_BUILD");
    const bool no_small = !(small_env && std::atoi(small_env) == 1);
    if (!no_small && !force_atomic && small_build_fits(n, C) && !b.gids && b.n_zero_words <= 1024) {
        // one workgroup, one launch (deterministic layout whatever b.deterministic says)
        static const bool attr = [] {
            // dynamic + static LDS may not pass 160 KB: the kernel's static words (~0.5 KB) come
            // off the opt-in (asking for the whole 160 KB is rejected and leaves the 64 KB default)
            (void)hipFuncSetAttribute((const void*)small_build_kernel, hipFuncAttributeMaxDynamicSharedMemorySize,
                                      kSmallLdsWords * 4);
            return true;
        }();
        (void)attr;
        small_build_kernel<<<1, 1024, ((size_t)C + (size_t)n) * sizeof(int), s>>>(
            b.points, n, b.dims[0], b.dims[1], b.dims[2], b.use_box, b.box_lo[0], b.box_lo[1], b.box_lo[2], b.box_hi[0],
            b.box_hi[1], b.box_hi[2], b.geom, b.cell_start, b.sorted, b.perm, b.zero_words,
            b.zero_words ? b.n_zero_words : 0);
        return hipGetLastError();
    }
    // Serial builds (nothing else on the device: kn_prepare, the serial graph step) use 1024-thread
    // blocks of 4096 points up to 4M points: ~220 blocks at 900K, one per CU, 16 waves each to hide
    // the LDS-atomic latency (900K build 0.050 ms vs 0.054 with 256-thread blocks and 0.083 with the
    // pipelined ~16K-point blocks; profiles/ab_r5_bin_threads.txt, BENCH_r04/r05 ms_build)
    const bool serial_small = b.serial && n <= (4 << 20);
    const int items_req = b.bin_items ? b.bin_items : (serial_small ? 4096 : 0);
    if (b.bin_tmp && !force_atomic && bin_plan(n, C, &bp, items_req)) {
        // geometry folded into bucket_count; scan top level folded into its consumers
        GeomSrc src{};
        src.use_box = b.use_box;
        for (int a = 0; a < 3; ++a) { src.lo[a] = b.box_lo[a]; src.hi[a] = b.box_hi[a]; src.dims[a] = b.dims[a]; }
        // KN_BIN_ATOMIC: bucket totals + published bucket starts in the (otherwise unused)
        // cell_scan buffer (bin_plan keeps 2 nbuckets + 2 <= C + 1), zeroed before the count
        int* totals = b.cell_scan;
        int* bstart = b.cell_scan + bp.nbuckets + 1;
        const int n_tot = KN_BIN_ATOMIC ? bp.nbuckets : 0;
        if (!b.use_box) {
            if ((e = launch_bbox_partials(b.points, n, b.bbox_words, s, totals, n_tot)) != hipSuccess) return e;
            src.partials = b.bbox_words;
            src.nbb = bbox_block_count(n);
        } else if (n_tot && !b.totals_zeroed &&
                   (e = hipMemsetAsync(totals, 0, (size_t)n_tot * sizeof(int), s)) != hipSuccess) {
            return e;
        }
        const size_t T = (size_t)bp.nbuckets * bp.nblocks;
        // global ids fused into the sort unless the in-cell order pass follows (it orders by w)
        const bool fuse_gid = b.gids && !b.deterministic;
        // Streaming blocks of 256 threads up to 4M points, 1024 above (KN_BIN_THREADS overrides).
        // Serially 1024 is faster (~220 blocks at 900K points is one block per CU, and the
        // LDS-atomic loops need 16 waves per CU: 900K build 0.050 vs 0.054 ms), but the pipelined
        // build runs beside one or two query kernels, where a 1024-thread block must find 16 free
        // wave slots on one CU and waits: 900K K=16 200 / 50 steps 0.2669 -> 0.2541 ms, the
        // driver's 20 / 5 0.296 -> 0.287, K=32 0.474 -> 0.410, clustered 1.044 -> 0.952, surfaces
        // 0.712 -> 0.652, world-1 distributed 0.286 -> 0.274; 10M K=32 +1.5 % (kept at 1024
        // there). Two interleaved passes, profiles/ab_r5_bin_threads.txt
        static const int bin_env = [] {
            const char* v = std::getenv("KN_BIN_THREADS");
            const int t = v ? std::atoi(v) : 0;
            return (t == 256 || t == 512 || t == 1024) ? t : 0;
        }();
        const int bin_threads = bin_env ? bin_env : (n <= (4 << 20) && !b.serial ? 256 : 1024);
        bucket_count_kernel<<<bp.nblocks, bin_threads, bp.nbuckets * sizeof(int), s>>>(
            b.points, n, src, b.geom, bp.shift, bp.nbuckets, bp.nblocks, bp.per_block, b.cell_count, totals,
            b.zero_words, b.n_zero_words);
        const unsigned nbt = (unsigned)scan_block_count((int)T);
        if (!KN_BIN_ATOMIC) scan_blocks_kernel<<<nbt, 256, 0, s>>>(b.cell_count, (int)T, b.cell_scan, b.block_sums);
        const int* tscan = KN_BIN_ATOMIC ? b.cell_count : b.cell_scan;
        bucket_scatter_kernel<<<bp.nblocks, bin_threads, bp.nbuckets * sizeof(int), s>>>(
            b.points, n, b.geom, bp.shift, bp.nbuckets, bp.nblocks, bp.per_block, tscan, b.block_sums,
            (int)nbt, totals, bstart, b.bin_tmp);
        bucket_sort_kernel<<<bp.nbuckets, 256, (1u << bp.shift) * sizeof(int), s>>>(
            b.bin_tmp, n, b.geom, bp.shift, bp.nbuckets, bp.nblocks, b.cell_scan, b.block_sums, bstart, C,
            b.cell_start, b.sorted, b.perm, fuse_gid ? b.gids : nullptr, b.n_owned);
        if (b.deterministic && (e = launch_cell_sort(b.cell_start, b.geom, n, b.sorted, b.perm, b.bin_tmp, s)) != hipSuccess)
            return e;
        if (b.gids && !fuse_gid) return launch_global_w(b.sorted, b.perm, b.gids, n, b.n_owned, s);
        return hipGetLastError();
    }
    // global-atomic binning (fallback)
    if (b.zero_words && b.n_zero_words > 0 &&
        (e = hipMemsetAsync(b.zero_words, 0, (size_t)b.n_zero_words * sizeof(unsigned), s)) != hipSuccess)
        return e;
    if (b.use_box) {
        geom_box_kernel<<<1, 64, 0, s>>>(b.box_lo[0], b.box_lo[1], b.box_lo[2], b.box_hi[0],
                                         b.box_hi[1], b.box_hi[2], b.dims[0], b.dims[1],
                                         b.dims[2], b.geom);
    } else {
        if ((e = launch_bbox_partials(b.points, n, b.bbox_words, s)) != hipSuccess) return e;
        geom_kernel<<<1, 64, 0, s>>>(b.bbox_words, n > 0 ? bbox_block_count(n) : 0, b.dims[0], b.dims[1],
                                     b.dims[2], b.geom);
    }
    if ((e = hipMemsetAsync(b.cell_count, 0, (size_t)C * sizeof(int), s)) != hipSuccess) return e;
    if (n > 0) count_kernel<<<cdiv(n, 256), 256, 0, s>>>(b.points, n, b.geom, b.cell_count, b.cell_rank);
    const unsigned nb = (unsigned)scan_block_count(C);
    scan_blocks_kernel<<<nb, 256, 0, s>>>(b.cell_count, C, b.cell_scan, b.block_sums);
    scan_top_kernel<<<1, 1024, 0, s>>>(b.block_sums, (int)nb);
    const size_t threads = std::max((size_t)n, (size_t)C + 1);
    scatter_kernel<<<cdiv(threads, 256), 256, 0, s>>>(b.points, n, b.cell_rank, b.cell_scan,
                                                      b.block_sums, C, b.cell_start, b.sorted,
                                                      b.perm);
    if (b.deterministic)
        cell_sort_kernel<<<cdiv(C, 256), 256, 0, s>>>(b.cell_start, C, b.sorted, b.perm);
    if (b.gids) {
        if ((e = hipGetLastError()) != hipSuccess) return e;
        return launch_global_w(b.sorted, b.perm, b.gids, n, b.n_owned, s);
    }
    return hipGetLastError();
}

KN_DEFINE_DEBUG_READER(debug_words_build)

hipError_t launch_cell_occupancy(const int* cell_start, int num_cells, unsigned long long* out, hipStream_t s) {
    hipError_t e;
    if ((e = hipMemsetAsync(out, 0, sizeof(unsigned long long), s)) != hipSuccess) return e;
    if (num_cells > 0) {
        const unsigned grid = std::max(1u, std::min(cdiv(num_cells, 256 * 8), 2048u));
        cell_occupancy_kernel<<<grid, 256, 0, s>>>(cell_start, num_cells, out);
    }
    return hipGetLastError();
}

hipError_t launch_cell_stats(const int* cell_start, int num_cells, int* out, int hist_len,
                             hipStream_t s) {
    hipError_t e;
    const int init[3] = {0x7fffffff, 0, 0};
    (void)init;
    if ((e = hipMemsetAsync(out, 0, (size_t)(3 + hist_len) * sizeof(int), s)) != hipSuccess) return e;
    if ((e = hipMemsetAsync(out, 0x7f, sizeof(int), s)) != hipSuccess) return e;
    if (num_cells > 0)
        cell_stats_kernel<<<cdiv(num_cells, 256), 256, 0, s>>>(cell_start, num_cells, out, hist_len);
    return hipGetLastError();
}

// ---- pointer tables of batched streams of clouds (Engine::stream_batch) ----------------------
// A graph captured once per batch length reads its steps' input / output pointers from a device
// table; one tiny kernel writes the table (its values travel as kernel arguments, so the host
// array need not outlive the enqueue) before each graph launch, stream-ordered.
struct PtrTable {
    void* p[kPtrTableMax];
};
__global__ void set_ptr_table_kernel(PtrTable t, int count, void** dst) {
    const int i = threadIdx.x;
    if (i < count) dst[i] = t.p[i];
}
// dst[0, n) = (*src_ref)[0, n): 16-byte vector copy where the source is aligned, else scalar
__global__ __launch_bounds__(256) void copy_from_ref_kernel(const float* const* src_ref, float* __restrict__ dst,
                                                            size_t n) {
    const float* src = *src_ref;
    const size_t tid = (size_t)blockIdx.x * blockDim.x + threadIdx.x, stride = (size_t)gridDim.x * blockDim.x;
    if (((reinterpret_cast<uintptr_t>(src) | reinterpret_cast<uintptr_t>(dst)) & 15u) == 0) {
        const size_t n4 = n / 4;
        const float4* s4 = reinterpret_cast<const float4*>(src);
        float4* d4 = reinterpret_cast<float4*>(dst);
        for (size_t i = tid; i < n4; i += stride) d4[i] = s4[i];
        for (size_t i = 4 * n4 + tid; i < n; i += stride) dst[i] = src[i];
    } else {
        for (size_t i = tid; i < n; i += stride) dst[i] = src[i];
    }
}

hipError_t launch_set_ptr_table(void* const* ptrs, int count, void** dst, hipStream_t s) {
    if (count < 0 || count > kPtrTableMax) return hipErrorInvalidValue;
    if (count == 0) return hipSuccess;
    PtrTable t{};
    for (int i = 0; i < count; ++i) t.p[i] = ptrs[i];
    set_ptr_table_kernel<<<1, kPtrTableMax, 0, s>>>(t, count, dst);
    return hipGetLastError();
}

hipError_t launch_copy_from_ref(const float* const* src_ref, float* dst, size_t n, hipStream_t s) {
    if (n == 0) return hipSuccess;
    const unsigned grid = std::max(1u, std::min(cdiv(n / 4 + 1, 256), 2048u));
    copy_from_ref_kernel<<<grid, 256, 0, s>>>(src_ref, dst, n);
    return hipGetLastError();
}

}  // namespace kn
