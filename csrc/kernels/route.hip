// route.hip -- multi-GPU point routing on gfx950: owner + halo destinations in ONE exchange.
//
// NEW component (the reference is single-GPU, knearests.cu has no partitioning). A rank's
// points go, in one all-to-all-v over RCCL/xGMI, to
//   * their OWNER (the rank box of the px*py*pz spatial decomposition that contains them), and
//   * every other rank whose box lies within the halo width h (HALO copies),
// so redistribution and halo exchange cost a single collective per solve. The send buffer is
// laid out per destination d as [owned rows for d][halo rows for d], rows are float4
// {x, y, z, bits(global id)} (16-B aligned, one dwordx4 per row on both sides of the copy).
//
// Order is deterministic and stable (by input index) -- no atomics decide positions:
//   route_count_kernel   : per-block counts of every (destination, kind) column (LDS atomics)
//   route_scan_kernel    : one workgroup per column, exclusive scan over blocks + column total
//   route_scatter_kernel : per-wave ballots give in-wave ranks, LDS gives wave offsets
//   route_unpack_kernel  : received [owned|halo] segments of every source -> owned points first
//                          (queries), halo after, as (N,3) points + int32 global ids
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>

#include "kn/route.h"
#include "kn/step_flag.h"
#include "kn/wave.h"

namespace kn {

namespace {

constexpr int kRT = 256;                      // threads per routing block
constexpr int kRounds = kRouteItems / kRT;    // points per thread

__device__ __forceinline__ int route_owner(const RouteParams& p, float x, float y, float z) {
    if (p.balanced) {
        // kd splits: the number of inner splits <= the coordinate on each level (a point on a
        // split belongs to the upper box), as SpatialDecomposition.owner
        const int px = p.grid[0], py = p.grid[1], pz = p.grid[2];
        int ix = 0, iy = 0, iz = 0;
        for (int j = 1; j < px; ++j) ix += p.xs[j] <= x ? 1 : 0;
        for (int j = 1; j < py; ++j) iy += p.ys[ix * (py + 1) + j] <= y ? 1 : 0;
        const int col = ix + px * iy;
        for (int j = 1; j < pz; ++j) iz += p.zs[col * (pz + 1) + j] <= z ? 1 : 0;
        return ix + px * (iy + py * iz);
    }
    const float v[3] = {x, y, z};
    int c[3];
#pragma unroll
    for (int a = 0; a < 3; ++a) {
        // same operation order as SpatialDecomposition.owner: (p - lo) / ext * g
        const float f = __fmul_rn(__fdiv_rn(__fsub_rn(v[a], p.lo[a]), p.ext[a]), p.g[a]);
        int i = (int)floorf(f);
        i = i < 0 ? 0 : i;
        c[a] = i > p.grid[a] - 1 ? p.grid[a] - 1 : i;
    }
    return c[0] + p.grid[0] * (c[1] + p.grid[1] * c[2]);
}

// Bit r set: point must be sent to rank r as halo (r != owner, squared distance to r's box
// within h2). Un-fused arithmetic, same order as SpatialDecomposition.box_dist2.
__device__ __forceinline__ unsigned long long route_halo(const RouteParams& p, float x, float y, float z,
                                                         int owner) {
    unsigned long long m = 0;
    float h2;
    if (p.field) {
        // density-adaptive halo: the width of the point's field cell
        const float w = fmaf(p.field[field_cell(p.fg, x, y, z)], 1.0001f, p.fslack);
        h2 = w * w;
    } else {
        // position-dependent width: the edge width in the wide zone near the domain faces
        const float zp = fminf(fminf(fminf(x - p.lo[0], p.dom_hi[0] - x), fminf(y - p.lo[1], p.dom_hi[1] - y)),
                               fminf(z - p.lo[2], p.dom_hi[2] - z));
        h2 = zp <= p.wz ? p.h2 : p.hi2;
    }
    for (int r = 0; r < p.world; ++r) {
        if (r == owner) continue;
        const float dx = __fadd_rn(fmaxf(__fsub_rn(p.box_lo[r][0], x), 0.f), fmaxf(__fsub_rn(x, p.box_hi[r][0]), 0.f));
        const float dy = __fadd_rn(fmaxf(__fsub_rn(p.box_lo[r][1], y), 0.f), fmaxf(__fsub_rn(y, p.box_hi[r][1]), 0.f));
        const float dz = __fadd_rn(fmaxf(__fsub_rn(p.box_lo[r][2], z), 0.f), fmaxf(__fsub_rn(z, p.box_hi[r][2]), 0.f));
        const float d2 = __fadd_rn(__fadd_rn(__fmul_rn(dx, dx), __fmul_rn(dy, dy)), __fmul_rn(dz, dz));
        if (d2 <= h2) m |= 1ull << r;
    }
    return m;
}

__device__ __forceinline__ unsigned meta_ord(float f) {
    const unsigned u = __float_as_uint(f);
    return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
}
__device__ __forceinline__ float meta_unord(unsigned u) {
    return __uint_as_float((u & 0x80000000u) ? (u & 0x7fffffffu) : ~u);
}

// partials (optional): the block's bbox as 6 words at partials[a * nb + block] (the encoding of
// launch_bbox_partials) -- the steady-state step checks its share's bbox from these instead of a
// separate pass over the points (steady_flag_partials_kernel)
__global__ __launch_bounds__(kRT) void route_count_kernel(const float* __restrict__ pts, int n,
                                                          const RouteParams* __restrict__ pp,
                                                          int* __restrict__ block_counts, int nb,
                                                          unsigned* __restrict__ partials,
                                                          int* __restrict__ zero_ints, int n_zero) {
    const RouteParams& p = *pp;
    if (blockIdx.x == 0)
        for (int j = threadIdx.x; j < n_zero; j += blockDim.x) zero_ints[j] = 0;
    __shared__ int cnt[2 * kRouteMaxWorld];
    __shared__ unsigned red[6][kRT / 64];
    const int cols = 2 * p.world;
    for (int c = threadIdx.x; c < cols; c += kRT) cnt[c] = 0;
    __syncthreads();
    unsigned bw[6] = {0u, 0u, 0u, 0u, 0u, 0u};  // max of ~ord(min) / ord(max); 0 = empty
    const bool lead = (threadIdx.x & 63) == 0;
#pragma unroll
    for (int r = 0; r < kRounds; ++r) {
        const int i = blockIdx.x * kRouteItems + r * kRT + threadIdx.x;
        int o = -1;
        unsigned long long m = 0;
        if (i < n) {
            const size_t i3 = 3 * (size_t)i;  // 64-bit: 3*i overflows int above 715M points
            const float x = pts[i3], y = pts[i3 + 1], z = pts[i3 + 2];
            bw[0] = max(bw[0], ~meta_ord(x)); bw[1] = max(bw[1], ~meta_ord(y)); bw[2] = max(bw[2], ~meta_ord(z));
            bw[3] = max(bw[3], meta_ord(x)); bw[4] = max(bw[4], meta_ord(y)); bw[5] = max(bw[5], meta_ord(z));
            o = route_owner(p, x, y, z);
            m = route_halo(p, x, y, z, o);
        }
        // per-wave column counts from ballots, one LDS atomic per wave and column: per-lane
        // atomics on one address (every point of a share has the same few owners) serialise
        // 64-fold (48 us for 900K points at world 1 vs the ~10 us the loads take)
        for (int d = 0; d < p.world; ++d) {
            const unsigned long long bo = __builtin_amdgcn_ballot_w64(o == d);
            const unsigned long long bh = __builtin_amdgcn_ballot_w64((m >> d) & 1ull);
            if (lead && bo) atomicAdd(&cnt[2 * d], __builtin_popcountll(bo));
            if (lead && bh) atomicAdd(&cnt[2 * d + 1], __builtin_popcountll(bh));
        }
    }
    if (partials) {
        const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
#pragma unroll
        for (int a = 0; a < 6; ++a) {
            const unsigned v = wave_max_u32(bw[a]);
            if (lane == 0) red[a][wid] = v;
        }
    }
    __syncthreads();
    for (int c = threadIdx.x; c < cols; c += kRT) block_counts[(size_t)c * nb + blockIdx.x] = cnt[c];
    if (partials && threadIdx.x < 6) {
        unsigned v = red[threadIdx.x][0];
        for (int w = 1; w < kRT / 64; ++w) v = max(v, red[threadIdx.x][w]);
        partials[(size_t)threadIdx.x * nb + blockIdx.x] = v;
    }
}

// One workgroup per column: exclusive scan of the column's nb block counts; total -> totals[c].
__global__ __launch_bounds__(kRT) void route_scan_kernel(int* __restrict__ block_counts, int nb,
                                                         int* __restrict__ totals) {
    __shared__ int wsum[kRT / 64];
    __shared__ int carry_s;
    int* col = block_counts + (size_t)blockIdx.x * nb;
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    if (threadIdx.x == 0) carry_s = 0;
    __syncthreads();
    for (int base = 0; base < nb; base += kRT) {
        const int i = base + threadIdx.x;
        const int v = (i < nb) ? col[i] : 0;
        const int incl = wave_inclusive_scan_add(v);
        if (lane == 63) wsum[wid] = incl;
        __syncthreads();
        int woff = 0;
        for (int w = 0; w < wid; ++w) woff += wsum[w];
        const int carry = carry_s;
        if (i < nb) col[i] = carry + woff + incl - v;
        __syncthreads();
        if (threadIdx.x == kRT - 1) carry_s = carry + woff + incl;
        __syncthreads();
    }
    if (threadIdx.x == 0) totals[blockIdx.x] = carry_s;
}

__global__ __launch_bounds__(kRT) void route_scatter_kernel(const float* __restrict__ pts,
                                                            const int* __restrict__ ids, int n,
                                                            const RouteParams* __restrict__ pp,
                                                            const int* __restrict__ block_offsets, int nb,
                                                            const int* __restrict__ totals,
                                                            float4* __restrict__ send, int send_rows,
                                                            int self_last, SelfPlace sp) {
    __shared__ int base[2 * kRouteMaxWorld];            // block's next row of every column
    __shared__ int wcnt[kRT / 64][2 * kRouteMaxWorld];  // per-wave counts of the current round
    __shared__ int overflow;
    __shared__ int seg_self;                            // first row of the self segment
    const RouteParams& p = *pp;
    const int cols = 2 * p.world;
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    if (threadIdx.x == 0) {
        int seg = 0;
        for (int t = 0; t < p.world; ++t) {
            // self_last >= 0: every other destination in order, then self
            const int d = self_last < 0 ? t : (t == p.world - 1 ? self_last : (t < self_last ? t : t + 1));
            const int own = totals[2 * d], halo = totals[2 * d + 1];
            base[2 * d] = seg + block_offsets[(size_t)(2 * d) * nb + blockIdx.x];
            base[2 * d + 1] = seg + own + block_offsets[(size_t)(2 * d + 1) * nb + blockIdx.x];
            if (d == self_last) seg_self = seg;
            seg += own + halo;
        }
        // same decision in every block: nothing is written. With direct self placement the
        // self segment does not occupy the send buffer.
        overflow = (sp.pts ? seg_self : seg) > send_rows;
        if (sp.pts && (totals[2 * self_last] != sp.own_cnt || totals[2 * self_last + 1] != sp.halo_cnt))
            overflow = 1;  // self segment differs from the plan: placing it could overrun `rows`
    }
    __syncthreads();
    if (overflow) return;
    const unsigned long long lt = (lane == 0) ? 0ull : (~0ull >> (64 - lane));
    for (int r = 0; r < kRounds; ++r) {
        const int i = blockIdx.x * kRouteItems + r * kRT + threadIdx.x;
        const bool valid = i < n;
        float x = 0.f, y = 0.f, z = 0.f;
        int o = -1;
        unsigned long long m = 0;
        if (valid) {
            const size_t i3 = 3 * (size_t)i;
            x = pts[i3]; y = pts[i3 + 1]; z = pts[i3 + 2];
            o = route_owner(p, x, y, z);
            m = route_halo(p, x, y, z, o);
        }
        // phase A: per-wave column counts
        for (int d = 0; d < p.world; ++d) {
            const unsigned long long bo = __builtin_amdgcn_ballot_w64(o == d);
            const unsigned long long bh = __builtin_amdgcn_ballot_w64((m >> d) & 1ull);
            if (lane == 0) {
                wcnt[wid][2 * d] = __builtin_popcountll(bo);
                wcnt[wid][2 * d + 1] = __builtin_popcountll(bh);
            }
        }
        __syncthreads();
        // phase B: rows (in-wave rank from the ballot, earlier waves from LDS)
        if (__builtin_amdgcn_ballot_w64(valid)) {
            const int gid = valid ? (ids ? ids[i] : p.id_offset + i) : 0;
            const float4 row = make_float4(x, y, z, __int_as_float(gid));
            for (int d = 0; d < p.world; ++d) {
                const bool po = o == d, ph = (m >> d) & 1ull;
                const unsigned long long bo = __builtin_amdgcn_ballot_w64(po);
                const unsigned long long bh = __builtin_amdgcn_ballot_w64(ph);
                if (po || ph) {
                    const int c = 2 * d + (po ? 0 : 1);
                    int off = base[c];
                    for (int w = 0; w < wid; ++w) off += wcnt[w][c];
                    off += __builtin_popcountll((po ? bo : bh) & lt);
                    if (sp.pts && d == self_last) {
                        // the rank's own segment straight to its local rows (what the unpack
                        // would compute): owned first over all sources, halo after
                        const int j = off - seg_self;
                        const int loc = po ? sp.own_base + j : sp.halo_base + (j - totals[2 * d]);
                        if (loc < 0 || loc >= sp.rows) continue;  // unreachable after the prologue check
                        const size_t l3 = 3 * (size_t)KN_IDX(loc, sp.rows, 403);
                        sp.pts[l3] = x;
                        sp.pts[l3 + 1] = y;
                        sp.pts[l3 + 2] = z;
                        sp.gids[loc] = gid;
                    } else {
                        send[KN_IDX(off, send_rows, 401)] = row;
                    }
                }
            }
        }
        __syncthreads();
        for (int c = threadIdx.x; c < cols; c += kRT) {
            int s = 0;
            for (int w = 0; w < kRT / 64; ++w) s += wcnt[w][c];
            base[c] += s;
        }
        __syncthreads();
    }
}

__global__ __launch_bounds__(kRT) void route_unpack_kernel(const float4* __restrict__ recv,
                                                           const float4* __restrict__ self_rows, int rows,
                                                           UnpackTable t, float* __restrict__ pts,
                                                           int* __restrict__ gids) {
    const int j = blockIdx.x * kRT + threadIdx.x;
    if (j >= rows) return;
    int lo, o;
    float4 v;
    if (j >= t.rows_cross) {  // the self segment (kept out of the collective)
        lo = t.self;
        o = j - t.rows_cross;
        v = self_rows[o];
    } else {
        lo = 0;
        int hi = t.world - 1;  // last source whose segment starts at or before j
        while (lo < hi) {
            const int mid = (lo + hi + 1) >> 1;
            if (t.seg[mid] <= j) lo = mid; else hi = mid - 1;
        }
        o = j - t.seg[lo];
        v = recv[j];
    }
    const int out = (o < t.own[lo]) ? t.own_pref[lo] + o : t.n_own + t.halo_pref[lo] + (o - t.own[lo]);
    const int oo = KN_IDX(out, t.out_rows > 0 ? t.out_rows : rows, 402);
    const size_t o3 = 3 * (size_t)oo;
    pts[o3] = v.x;
    pts[o3 + 1] = v.y;
    pts[o3 + 2] = v.z;
    gids[oo] = __float_as_int(v.w);
}


// One thread: global domain, halo width, rank boxes and id offset from the gathered metas.
// Formulas follow SpatialDecomposition / DistributedKNearests (parallel/*.py) in double.
__global__ void route_plan_kernel(const double* __restrict__ metas, int world, int rank, int gx, int gy, int gz,
                                  int k, double halo_factor, double inner_factor, const float* __restrict__ splits,
                                  RouteParams* __restrict__ p, double* __restrict__ hdr,
                                  const float* __restrict__ field, int field_g) {
    // the halo field's largest width (one wave; widths >= 0 order as their bits)
    unsigned fmax_bits = 0u;
    if (field) {
        const int cells = field_g * field_g * field_g;
        for (int c = threadIdx.x; c < cells; c += 64) fmax_bits = max(fmax_bits, __float_as_uint(field[c]));
        fmax_bits = wave_max_u32(fmax_bits);
    }
    if (threadIdx.x != 0 || blockIdx.x != 0) return;
    double lo[3], hi[3];
    double ntot = 0.0, off = 0.0;
    for (int a = 0; a < 3; ++a) { lo[a] = INFINITY; hi[a] = -INFINITY; }
    for (int r = 0; r < world; ++r) {
        for (int a = 0; a < 3; ++a) {
            lo[a] = fmin(lo[a], metas[8 * r + a]);
            hi[a] = fmax(hi[a], metas[8 * r + 3 + a]);
        }
        if (r < rank) off += metas[8 * r + 6];
        ntot += metas[8 * r + 6];
    }
    bool finite = true;
    for (int a = 0; a < 3; ++a) finite = finite && isfinite(lo[a]) && isfinite(hi[a]);
    if (!finite)
        for (int a = 0; a < 3; ++a) { lo[a] = 0.0; hi[a] = 1.0; }  // empty global cloud
    double vol = 1.0, diag2 = 0.0, scale = 0.0;
    for (int a = 0; a < 3; ++a) {
        const double e = hi[a] - lo[a];
        vol *= e;
        diag2 += e * e;
        scale = fmax(scale, fmax(fabs(lo[a]), fmax(fabs(hi[a]), e)));
    }
    vol = fmax(vol, 1e-30);
    const double rk = cbrt(3.0 * (k + 1) * vol / (4.0 * M_PI * fmax(1.0, ntot)));
    const double diag = sqrt(diag2);
    // halo field: the send width of a cell is its field value (x 1.0001 + fslack); the complete
    // box is the own box (certification width 0) plus the field's certified radii. A field whose
    // widest cell reaches the diagonal falls back to the global widths.
    const double fslack = 1e-5 * scale;
    const double fmax = (double)__uint_as_float(fmax_bits);
    const bool use_field = field && field_g > 0 && fmax * 1.0001 + fslack < diag;
    const double h = use_field ? 0.0 : halo_factor * rk;
    const bool full = h >= diag;
    const double hs = use_field ? fmax * 1.0001 + 2.0 * fslack
                    : full ? 2.0 * diag + 1.0 : h * (1.0 + 1e-5) + 1e-5 * scale;
    // interior width (position-dependent halo): h_i <= h, sent to points farther than w = h + h_i
    // from the domain faces; the certification's zone limit keeps a rounding slack below w
    const double hi_ = inner_factor > 0.0 ? fmin(h, inner_factor * rk) : h;
    const double his = full || use_field ? hs : hi_ * (1.0 + 1e-5) + 1e-5 * scale;
    const double wz = h + hi_;
    const int g[3] = {gx, gy, gz};
    for (int a = 0; a < 3; ++a) {
        const float l = (float)lo[a], u = (float)hi[a];
        p->lo[a] = l;
        p->ext[a] = fmaxf(u - l, 1e-30f);
        p->g[a] = (float)g[a];
        p->grid[a] = g[a];
    }
    p->world = world;
    const float hf = (float)hs;
    p->h2 = hf * hf;
    const float hif = (float)his;
    p->hi2 = hif * hif;
    p->wz = (float)wz;
    for (int a = 0; a < 3; ++a) p->dom_hi[a] = (float)hi[a];
    p->pad0 = 0;
    p->field = use_field ? field : nullptr;
    {
        const float fl[3] = {(float)lo[0], (float)lo[1], (float)lo[2]};
        const float fh[3] = {(float)hi[0], (float)hi[1], (float)hi[2]};
        p->fg = field_geom(fl, fh, use_field ? field_g : 0);
    }
    p->fslack = (float)fslack;
    p->id_offset = (int)off;
    p->balanced = splits ? 1 : 0;
    const int nxs = gx + 1, nys = gx * (gy + 1), nzs = gx * gy * (gz + 1);
    for (int j = 0; j < kRouteMaxWorld + 1; ++j) p->xs[j] = (splits && j < nxs) ? splits[j] : 0.f;
    for (int j = 0; j < 2 * kRouteMaxWorld; ++j) p->ys[j] = (splits && j < nys) ? splits[nxs + j] : 0.f;
    for (int j = 0; j < 2 * kRouteMaxWorld; ++j) p->zs[j] = (splits && j < nzs) ? splits[nxs + nys + j] : 0.f;
    double own_lo[3] = {0, 0, 0}, own_hi[3] = {0, 0, 0};
    for (int r = 0; r < world; ++r) {
        const int c[3] = {r % gx, (r / gx) % gy, r / (gx * gy)};
        double blo[3], bhi[3];
        if (splits) {
            const int col = c[0] + gx * c[1];
            blo[0] = p->xs[c[0]];
            bhi[0] = p->xs[c[0] + 1];
            blo[1] = p->ys[c[0] * (gy + 1) + c[1]];
            bhi[1] = p->ys[c[0] * (gy + 1) + c[1] + 1];
            blo[2] = p->zs[col * (gz + 1) + c[2]];
            bhi[2] = p->zs[col * (gz + 1) + c[2] + 1];
        } else {
            for (int a = 0; a < 3; ++a) {
                const double w = (hi[a] - lo[a]) / g[a];
                blo[a] = __dadd_rn(lo[a], __dmul_rn((double)c[a], w));
                bhi[a] = c[a] == g[a] - 1 ? hi[a] : __dadd_rn(lo[a], __dmul_rn((double)(c[a] + 1), w));
            }
        }
        for (int a = 0; a < 3; ++a) {
            p->box_lo[r][a] = (float)blo[a];
            p->box_hi[r][a] = (float)bhi[a];
            if (r == rank) { own_lo[a] = blo[a]; own_hi[a] = bhi[a]; }
        }
    }
    for (int r = world; r < kRouteMaxWorld; ++r)  // unused slots: defined bytes (plans compare equal)
        for (int a = 0; a < 3; ++a) p->box_lo[r][a] = p->box_hi[r][a] = 0.f;
    for (int a = 0; a < 3; ++a) { hdr[a] = lo[a]; hdr[3 + a] = hi[a]; }
    for (int a = 0; a < 3; ++a) { hdr[12 + a] = own_lo[a]; hdr[15 + a] = own_hi[a]; }
    hdr[6] = h;
    hdr[7] = hs;
    hdr[8] = ntot;
    hdr[9] = off;
    hdr[10] = full ? 1.0 : 0.0;
    hdr[11] = diag;
    for (int i = 18; i < kPlanHdr; ++i) hdr[i] = 0.0;
    hdr[18] = hi_;
    hdr[19] = his;
    hdr[20] = wz;
    hdr[21] = wz - 1e-5 * scale;
    hdr[22] = use_field ? 1.0 : 0.0;
    hdr[23] = use_field ? fmax : 0.0;
}

// ---- density-adaptive halo field ------------------------------------------------------------
__global__ void field_splat_kernel(const float* __restrict__ pts, int n_owned, const float* __restrict__ d2, int k,
                                   float3 olo, float3 ohi, FieldGeom fg, float slack, unsigned* __restrict__ field,
                                   unsigned* __restrict__ stat) {
    const int j = blockIdx.x * blockDim.x + threadIdx.x;
    if (j >= n_owned) return;
    const float dk = d2[(size_t)j * k + (k - 1)];
    if (!(dk < INFINITY)) {  // fewer than K neighbours in the whole cloud
        atomicAdd(stat + 0, 1u);
        return;
    }
    const float x = pts[3 * (size_t)j], y = pts[3 * (size_t)j + 1], z = pts[3 * (size_t)j + 2];
    const float margin = fminf(fminf(fminf(x - olo.x, ohi.x - x), fminf(y - olo.y, ohi.y - y)),
                               fminf(z - olo.z, ohi.z - z));
    // R: the K-th distance rounded up, plus the slack the certification subtracts
    const float R = fmaf(sqrtf(dk), 1.000001f, slack);
    if (R <= margin) return;  // the ball stays in the own box
    int m = 1;
    while (m < kFieldLevels && R > (float)m * fg.rstep) ++m;
    if (R > (float)m * fg.rstep) atomicAdd(stat + 1, 1u);  // past the field's reach: forwarded
    const int cx = field_axis(fg, x, 0), cy = field_axis(fg, y, 1), cz = field_axis(fg, z, 2);
    const unsigned rb = __float_as_uint(R);
    for (int zz = max(0, cz - m); zz <= min(fg.g - 1, cz + m); ++zz)
        for (int yy = max(0, cy - m); yy <= min(fg.g - 1, cy + m); ++yy)
            for (int xx = max(0, cx - m); xx <= min(fg.g - 1, cx + m); ++xx)
                atomicMax(field + (xx + fg.g * (yy + fg.g * zz)), rb);
}

__global__ void field_cert_kernel(const float* __restrict__ field, FieldGeom fg, float* __restrict__ cert) {
    const int G = fg.g;
    const int c = blockIdx.x * blockDim.x + threadIdx.x;
    if (c >= G * G * G) return;
    const int cx = c % G, cy = (c / G) % G, cz = c / (G * G);
    float mn[kFieldLevels + 1];
#pragma unroll
    for (int m = 0; m <= kFieldLevels; ++m) mn[m] = INFINITY;
    constexpr int L = kFieldLevels;
    for (int dz = -L; dz <= L; ++dz) {
        const int zz = cz + dz;
        if (zz < 0 || zz >= G) continue;
        for (int dy = -L; dy <= L; ++dy) {
            const int yy = cy + dy;
            if (yy < 0 || yy >= G) continue;
            for (int dx = -L; dx <= L; ++dx) {
                const int xx = cx + dx;
                if (xx < 0 || xx >= G) continue;
                const int ring = max(max(abs(dx), abs(dy)), abs(dz));
                const float v = field[xx + G * (yy + G * zz)];
#pragma unroll
                for (int m = 1; m <= L; ++m)
                    if (ring <= m) mn[m] = fminf(mn[m], v);
            }
        }
    }
    float r = 0.f;
#pragma unroll
    for (int m = 1; m <= L; ++m) r = fmaxf(r, fminf(mn[m], (float)m * fg.rstep));
    cert[c] = r;
}

inline unsigned cdiv(size_t a, size_t b) { return (unsigned)((a + b - 1) / b); }


// ---- local meta of a rank's share: {lo[3], hi[3], n, 0} as doubles ---------------------
// (replaces a strided torch.aminmax over dim 0, which costs ~0.34 ms at 900K points)
// words: the per-block partials of launch_bbox_partials (build.hip), same encoding
__global__ void meta_finalize_kernel(const unsigned* __restrict__ partials, int nblocks, int n,
                                     double* __restrict__ out) {
    unsigned words[6];
    bbox_reduce_partials(partials, nblocks, kBBoxBlocks, words);
    const int t = threadIdx.x;
    if (t >= 8) return;
    double v;
    unsigned wt = words[0];  // words[t] without dynamic register indexing
#pragma unroll
    for (int a = 1; a < 6; ++a) wt = (t == a) ? words[a] : wt;
    if (t < 3) v = n > 0 ? (double)meta_unord(~wt) : (double)INFINITY;
    else if (t < 6) v = n > 0 ? (double)meta_unord(wt) : -(double)INFINITY;
    else if (t == 6) v = (double)n;
    else v = 0.0;
    out[t] = v;
}

// Global-id mode of the query kernels (query.hip, w_live / w_id / w_row): the stored point at
// sorted slot i gets w = gid[perm[i]], with the halo bit on non-owned points (perm[i] >=
// n_owned). One coalesced pass over the N stored points replaces K random id_map gathers per
// query in the query epilogue.
__global__ void global_w_kernel(float4* __restrict__ sorted, const unsigned* __restrict__ perm,
                                const int* __restrict__ gids, int n, int n_owned) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const unsigned local = perm[KN_IDX(i, n, 420)];
    const unsigned gid = (unsigned)gids[KN_IDX(local, (unsigned)n, 421)];
    sorted[i].w = __uint_as_float((gid & 0x7FFFFFFFu) | ((int)local >= n_owned ? 0x80000000u : 0u));
}

__global__ void steady_flag_kernel(const double* __restrict__ local, const double* __restrict__ planned,
                                   const int* __restrict__ totals, const int* __restrict__ ptotals, int nt,
                                   const unsigned* __restrict__ counters, int* __restrict__ flag) {
    const int lane = threadIdx.x;
    bool diff = false;
    if (lane < 8) diff = local[lane] != planned[lane];  // {lo, hi, n}: a NaN never matches either
    for (int i = lane; i < nt; i += 64) diff |= totals[i] != ptotals[i];
    const bool any = __builtin_amdgcn_ballot_w64(diff) != 0ull;
    if (lane == 0) flag[0] = (any ? 1 : 0) + (counters[1] != 0u ? 1 : 0);
}

// Steady-state check from the routing pass's bbox partials (route_count_kernel): this share's
// {lo, hi, n} against the planned meta (the same double conversion as meta_finalize_kernel), the
// send counts against the planned ones, and no uncertified query.
// partials[a * stride + b] for the nb blocks b < nb. sticky / host_flag (optional, graph-replayed
// world-1 steps): the flag is also max-accumulated into sticky and stored to host_flag (a device
// pointer to pinned host memory), so no copy node follows the step.
__global__ __launch_bounds__(1024) void steady_flag_partials_kernel(const unsigned* __restrict__ partials, int nb,
                                            int stride, int n,
                                            const double* __restrict__ planned, const int* __restrict__ totals,
                                            const int* __restrict__ ptotals, int nt,
                                            const unsigned* __restrict__ counters, int* __restrict__ flag,
                                            int* __restrict__ sticky, int* __restrict__ host_flag) {
    // block-wide reduction of the nb x 6 partials (launched with 256 threads: a 1024-thread block
    // beside the running query kernels waits for 16 free wave slots on one CU); kn/step_flag.h
    int f = step_flag_eval(partials, nb, stride, n, planned, totals, ptotals, nt, counters[1]);
    if (threadIdx.x == 0) {
        if (sticky) {
            f = max(f, sticky[0]);
            sticky[0] = f;
            host_flag[0] = f;
        }
        flag[0] = f;
    }
}

// Sticky flag of a pipelined distributed step, after its all-reduce: sticky = max(sticky, flag),
// stored to pinned host memory (a device pointer), so the host reading it sees this step's flag or
// a later step's -- never "valid" after an invalid step.
__global__ void flag_sink_kernel(const int* __restrict__ flag, int* __restrict__ sticky, int* __restrict__ host_flag) {
    if (threadIdx.x == 0) {
        const int f = max(flag[0], sticky[0]);
        sticky[0] = f;
        host_flag[0] = f;
    }
}

// ---- query forwarding inside a sync-free step (fixed-capacity slots, no host round trip) -------
// Every uncertified query of this rank (local row, K-th squared distance r2 of its local answer)
// goes to each OTHER rank whose box lies within r2 (conservative slack), into that destination's
// fixed slot block: slot = atomic counter, row pair {x, y, z, bits(gid)}, {r2, -, -, -}. A
// destination block that would overflow F slots counts in stat[1] (the step's flag then fails it
// and the caller re-solves the full way). slot_of[u * world + d] = the slot of query u at d (-1).
__global__ __launch_bounds__(256) void fwd_pack_kernel(const RouteParams* __restrict__ pp, int rank, int F, int k,
                                                       const unsigned* __restrict__ uncert,
                                                       const unsigned* __restrict__ ucount, int umax,
                                                       const float* __restrict__ pts, const int* __restrict__ gids,
                                                       const float* __restrict__ d2, float4* __restrict__ send,
                                                       int* __restrict__ slot_row, int* __restrict__ slot_of,
                                                       int* __restrict__ cnt, unsigned* __restrict__ stat) {
    const RouteParams& p = *pp;
    const int world = p.world;
    const int nu = (int)*ucount;
    if (blockIdx.x == 0 && threadIdx.x == 0 && nu > umax) atomicAdd(stat + 1, (unsigned)(nu - umax));
    for (int u = blockIdx.x * blockDim.x + threadIdx.x; u < min(nu, umax); u += gridDim.x * blockDim.x) {
        const int row = (int)uncert[u];
        const float x = pts[3 * (size_t)row], y = pts[3 * (size_t)row + 1], z = pts[3 * (size_t)row + 2];
        const float r2 = d2[(size_t)row * k + (k - 1)];
        // the float box arithmetic may not miss a rank: same slack as the host-synchronised round
        const float r2c = (r2 < INFINITY) ? r2 * (1.0f + 1e-5f) + 1e-6f : INFINITY;
        for (int d = 0; d < world; ++d) {
            int sl = -1;
            if (d != rank) {
                const float dx = __fadd_rn(fmaxf(__fsub_rn(p.box_lo[d][0], x), 0.f), fmaxf(__fsub_rn(x, p.box_hi[d][0]), 0.f));
                const float dy = __fadd_rn(fmaxf(__fsub_rn(p.box_lo[d][1], y), 0.f), fmaxf(__fsub_rn(y, p.box_hi[d][1]), 0.f));
                const float dz = __fadd_rn(fmaxf(__fsub_rn(p.box_lo[d][2], z), 0.f), fmaxf(__fsub_rn(z, p.box_hi[d][2]), 0.f));
                const float bd = __fadd_rn(__fadd_rn(__fmul_rn(dx, dx), __fmul_rn(dy, dy)), __fmul_rn(dz, dz));
                if (bd <= r2c) {
                    const int s = atomicAdd(&cnt[d], 1);
                    if (s < F) {
                        const size_t o = (size_t)d * F + s;
                        send[2 * o] = make_float4(x, y, z, __int_as_float(gids[row]));
                        send[2 * o + 1] = make_float4(r2, 0.f, 0.f, 0.f);
                        slot_row[o] = row;
                        sl = s;
                    } else {
                        atomicAdd(stat + 1, 1u);
                    }
                }
            }
            slot_of[(size_t)u * world + d] = sl;
        }
    }
}

// Merge of the answers: one thread per forwarded query. Its row (ascending (d2, id), K entries)
// is merged with each destination's answer list (<= K, ascending) keeping the K smallest
// (d2, gid), duplicates (a halo copy answered by its owner too) dropped.
__global__ __launch_bounds__(256) void fwd_merge_kernel(int world, int F, int k, const unsigned* __restrict__ uncert,
                                                        const unsigned* __restrict__ ucount, int umax,
                                                        const int* __restrict__ slot_of, const int* __restrict__ back_idx,
                                                        const float* __restrict__ back_d2, int* __restrict__ idx,
                                                        float* __restrict__ d2) {
    constexpr int kMaxK = 128;
    const int nu = min((int)*ucount, umax);
    for (int u = blockIdx.x * blockDim.x + threadIdx.x; u < nu; u += gridDim.x * blockDim.x) {
        const int row = (int)uncert[u];
        int* ri = idx + (size_t)row * k;
        float* rd = d2 + (size_t)row * k;
        for (int d = 0; d < world; ++d) {
            const int sl = slot_of[(size_t)u * world + d];
            if (sl < 0) continue;
            const int* ai = back_idx + ((size_t)d * F + sl) * k;
            const float* ad = back_d2 + ((size_t)d * F + sl) * k;
            int oi[kMaxK];
            float od[kMaxK];
            int i = 0, j = 0, m = 0;
            unsigned lastid = 0xFFFFFFFFu;
            float lastd = -1.f;
            while (m < k && (i < k || j < k)) {
                const bool vi = i < k && ri[i] != -1, vj = j < k && ai[j] != -1;
                if (!vi && !vj) break;
                bool takei;
                if (!vj) takei = true;
                else if (!vi) takei = false;
                else takei = rd[i] < ad[j] || (rd[i] == ad[j] && (unsigned)ri[i] <= (unsigned)ai[j]);
                const int ci = takei ? ri[i] : ai[j];
                const float cd = takei ? rd[i] : ad[j];
                if (takei) ++i; else ++j;
                if ((unsigned)ci == lastid && cd == lastd) continue;  // duplicate point
                oi[m] = ci;
                od[m] = cd;
                lastid = (unsigned)ci;
                lastd = cd;
                ++m;
            }
            for (int t = 0; t < k; ++t) {
                ri[t] = t < m ? oi[t] : -1;
                rd[t] = t < m ? od[t] : INFINITY;
            }
        }
    }
}

// ---- count-balanced split histograms (launch_split_hist) --------------------------------
__device__ __forceinline__ int split_bin_row(const SplitHistArgs& a, float x, float y, float z, int* row) {
    const int px = a.grid[0], py = a.grid[1];
    int ix = 0, iy = 0;
    if (a.stage >= 1)
        for (int j = 1; j < px; ++j) ix += x >= a.xs[j] ? 1 : 0;
    if (a.stage >= 2)
        for (int j = 1; j < py; ++j) iy += y >= a.ys[ix * (py + 1) + j] ? 1 : 0;
    *row = a.stage == 0 ? 0 : a.stage == 1 ? ix : ix + px * iy;
    const int ax = a.stage;
    const float v = ax == 0 ? x : ax == 1 ? y : z;
    // (p - lo) / ext * B, float32 as balanced_splits
    const float f = __fmul_rn(__fdiv_rn(__fsub_rn(v, a.lo[ax]), a.ext[ax]), (float)kSplitBins);
    const int b = (int)floorf(f);
    return b < 0 ? 0 : (b > kSplitBins - 1 ? kSplitBins - 1 : b);
}

constexpr int kSplitLdsBins = 16384;  // 64 KB of LDS: per-block partials up to 4 rows

__global__ __launch_bounds__(1024) void split_hist_lds_kernel(const float* __restrict__ pts, int n, SplitHistArgs a,
                                                              int bins, unsigned* __restrict__ part) {
    __shared__ unsigned h[kSplitLdsBins];
    for (int j = threadIdx.x; j < bins; j += 1024) h[j] = 0u;
    __syncthreads();
    const int per = (n + gridDim.x - 1) / gridDim.x, i0 = blockIdx.x * per, i1 = min(n, i0 + per);
    for (int i = i0 + threadIdx.x; i < i1; i += 1024) {
        int row;
        const int b = split_bin_row(a, pts[3 * (size_t)i], pts[3 * (size_t)i + 1], pts[3 * (size_t)i + 2], &row);
        atomicAdd(&h[row * kSplitBins + b], 1u);
    }
    __syncthreads();
    for (int j = threadIdx.x; j < bins; j += 1024) part[(size_t)blockIdx.x * bins + j] = h[j];
}

__global__ __launch_bounds__(256) void split_hist_sum_kernel(const unsigned* __restrict__ part, int nb, int bins,
                                                             unsigned* __restrict__ hist) {
    const int j = blockIdx.x * 256 + threadIdx.x;
    if (j >= bins) return;
    unsigned s = 0;
    for (int b = 0; b < nb; ++b) s += part[(size_t)b * bins + j];
    hist[j] = s;
}

__global__ __launch_bounds__(256) void split_hist_global_kernel(const float* __restrict__ pts, int n, SplitHistArgs a,
                                                                unsigned* __restrict__ hist) {
    for (int i = blockIdx.x * 256 + threadIdx.x; i < n; i += gridDim.x * 256) {
        int row;
        const int b = split_bin_row(a, pts[3 * (size_t)i], pts[3 * (size_t)i + 1], pts[3 * (size_t)i + 2], &row);
        atomicAdd(&hist[(size_t)row * kSplitBins + b], 1u);
    }
}

int split_hist_blocks(int n) { return std::max(1, std::min((int)cdiv((size_t)n, 8192), 128)); }

}  // namespace

int route_block_count(int n) { return std::max(1, (int)cdiv((size_t)std::max(n, 0), kRouteItems)); }

hipError_t launch_route_count(const float* pts, int n, const RouteParams* p, int world, int* block_counts,
                              int* totals, hipStream_t s, unsigned* partials, int* zero_ints, int n_zero) {
    if (world < 1 || world > kRouteMaxWorld) return hipErrorInvalidValue;
    const int nb = route_block_count(n);
    if (!zero_ints) n_zero = 0;
    route_count_kernel<<<nb, kRT, 0, s>>>(pts, n, p, block_counts, nb, partials, zero_ints, n_zero);
    route_scan_kernel<<<2 * world, kRT, 0, s>>>(block_counts, nb, totals);
    return hipGetLastError();
}

hipError_t launch_route_scatter(const float* pts, const int* ids, int n, const RouteParams* p, int world,
                                const int* block_offsets, const int* totals, float4* send, int send_rows,
                                int self_last, hipStream_t s, const SelfPlace* self_place) {
    if (world < 1 || world > kRouteMaxWorld || self_last >= world) return hipErrorInvalidValue;
    SelfPlace sp{};
    if (self_place) {
        if (self_last < 0 || !self_place->pts || !self_place->gids) return hipErrorInvalidValue;
        sp = *self_place;
    }
    const int nb = route_block_count(n);
    if (n > 0)
        route_scatter_kernel<<<nb, kRT, 0, s>>>(pts, ids, n, p, block_offsets, nb, totals, send, send_rows,
                                                self_last, sp);
    return hipGetLastError();
}


hipError_t launch_route_plan(const double* metas, int world, int rank, const int grid[3], int k,
                             double halo_factor, const float* splits, RouteParams* p, double* hdr, hipStream_t s,
                             double inner_factor, const float* field, int field_g) {
    if (world < 1 || world > kRouteMaxWorld || grid[0] * grid[1] * grid[2] != world || rank < 0 || rank >= world)
        return hipErrorInvalidValue;
    if (field && (field_g < 1 || field_g > 256)) return hipErrorInvalidValue;
    route_plan_kernel<<<1, 64, 0, s>>>(metas, world, rank, grid[0], grid[1], grid[2], k, halo_factor, inner_factor,
                                       splits, p, hdr, field, field ? field_g : 0);
    return hipGetLastError();
}

hipError_t launch_field_splat(const float* pts, int n_owned, const float* d2, int k, const float own_lo[3],
                              const float own_hi[3], const FieldGeom& fg, float slack, float* field, unsigned* stat,
                              hipStream_t s) {
    if (fg.g < 1 || fg.g > 256 || k < 1 || n_owned < 0) return hipErrorInvalidValue;
    if (n_owned > 0)
        field_splat_kernel<<<cdiv((size_t)n_owned, 256), 256, 0, s>>>(
            pts, n_owned, d2, k, make_float3(own_lo[0], own_lo[1], own_lo[2]),
            make_float3(own_hi[0], own_hi[1], own_hi[2]), fg, slack, reinterpret_cast<unsigned*>(field), stat);
    return hipGetLastError();
}

hipError_t launch_field_cert(const float* field, const FieldGeom& fg, float* cert, hipStream_t s) {
    if (fg.g < 1 || fg.g > 256) return hipErrorInvalidValue;
    const size_t cells = (size_t)fg.g * fg.g * fg.g;
    field_cert_kernel<<<cdiv(cells, 256), 256, 0, s>>>(field, fg, cert);
    return hipGetLastError();
}

FieldGeom field_geom_hdr(const double* hd, int g) {
    const float lo[3] = {(float)hd[0], (float)hd[1], (float)hd[2]};
    const float hi[3] = {(float)hd[3], (float)hd[4], (float)hd[5]};
    return field_geom(lo, hi, g);
}

hipError_t launch_route_unpack(const float4* recv, const float4* self_rows, int rows, const UnpackTable& t,
                               float* pts, int* gids, hipStream_t s) {
    if (t.world < 1 || t.world > kRouteMaxWorld || t.rows_cross > rows || t.self >= t.world ||
        (rows > t.rows_cross && (t.self < 0 || self_rows == nullptr)))
        return hipErrorInvalidValue;
    if (rows > 0) route_unpack_kernel<<<cdiv(rows, kRT), kRT, 0, s>>>(recv, self_rows, rows, t, pts, gids);
    return hipGetLastError();
}

hipError_t launch_local_meta(const float* pts, int n, unsigned* words, double* out, hipStream_t s) {
    hipError_t e;
    if ((e = launch_bbox_partials(pts, n, words, s)) != hipSuccess) return e;
    meta_finalize_kernel<<<1, 64, 0, s>>>(words, n > 0 ? bbox_block_count(n) : 0, n, out);
    return hipGetLastError();
}

hipError_t launch_steady_flag(const double* local, const double* planned_meta, const int* totals,
                              const int* planned_totals, int n_totals, const unsigned* counters, int* flag,
                              hipStream_t s) {
    steady_flag_kernel<<<1, 64, 0, s>>>(local, planned_meta, totals, planned_totals, n_totals, counters, flag);
    return hipGetLastError();
}

hipError_t launch_steady_flag_partials(const unsigned* partials, int n_routed, int n, const double* planned_meta,
                                       const int* totals, const int* planned_totals, int n_totals,
                                       const unsigned* counters, int* flag, hipStream_t s) {
    // the partials' layout is route_count's over the ROUTED rows (block count and stride); n is the
    // share's true size, compared with the planned meta (a grown share routes only the planned rows)
    if (n_routed < 0 || n_routed > n) return hipErrorInvalidValue;
    const int nb = n_routed > 0 ? route_block_count(n_routed) : 0;
    steady_flag_partials_kernel<<<1, 256, 0, s>>>(partials, nb, nb, n, planned_meta, totals, planned_totals, n_totals,
                                                 counters, flag, nullptr, nullptr);
    return hipGetLastError();
}

hipError_t launch_steady_flag_local(const float* pts, int n, unsigned* words, const double* planned_meta,
                                    const unsigned* counters, int* flag, int* sticky, int* host_flag, hipStream_t s) {
    if ((sticky == nullptr) != (host_flag == nullptr)) return hipErrorInvalidValue;
    hipError_t e;
    if ((e = launch_bbox_partials(pts, n, words, s)) != hipSuccess) return e;
    steady_flag_partials_kernel<<<1, 256, 0, s>>>(words, n > 0 ? bbox_block_count(n) : 0, kBBoxBlocks, n,
                                                 planned_meta, nullptr, nullptr, 0, counters, flag, sticky, host_flag);
    return hipGetLastError();
}

hipError_t launch_flag_sink(const int* flag, int* sticky, int* host_flag, hipStream_t s) {
    flag_sink_kernel<<<1, 64, 0, s>>>(flag, sticky, host_flag);
    return hipGetLastError();
}

__global__ void flag_accum_kernel(const int* __restrict__ flag, int* __restrict__ pending) {
    if (threadIdx.x == 0) atomicMax(pending, flag[0]);
}
hipError_t launch_flag_accum(const int* flag, int* pending, hipStream_t s) {
    flag_accum_kernel<<<1, 64, 0, s>>>(flag, pending);
    return hipGetLastError();
}

hipError_t launch_global_w(float4* sorted, const unsigned* perm, const int* gids, int n, int n_owned, hipStream_t s) {
    if (n > 0) global_w_kernel<<<cdiv(n, kRT), kRT, 0, s>>>(sorted, perm, gids, n, n_owned);
    return hipGetLastError();
}

hipError_t launch_fwd_pack(const RouteParams* p, int world, int rank, int F, int k, const unsigned* uncert,
                           const unsigned* ucount, int umax, const float* pts, const int* gids, const float* d2,
                           float4* send, int* slot_row, int* slot_of, int* cnt, unsigned* stat, hipStream_t s) {
    if (world < 1 || world > kRouteMaxWorld || rank < 0 || rank >= world || F < 1 || k < 1 || umax < 0)
        return hipErrorInvalidValue;
    hipError_t e;
    // empty slots: gid 0xFFFFFFFF (every float NaN); counters zeroed
    if ((e = hipMemsetAsync(send, 0xFF, (size_t)world * F * 2 * sizeof(float4), s)) != hipSuccess) return e;
    if ((e = hipMemsetAsync(cnt, 0, (size_t)world * sizeof(int), s)) != hipSuccess) return e;
    if (umax > 0)
        fwd_pack_kernel<<<std::max(1u, std::min(cdiv((size_t)umax, 256), 64u)), 256, 0, s>>>(
            p, rank, F, k, uncert, ucount, umax, pts, gids, d2, send, slot_row, slot_of, cnt, stat);
    return hipGetLastError();
}

hipError_t launch_fwd_merge(int world, int F, int k, const unsigned* uncert, const unsigned* ucount, int umax,
                            const int* slot_of, const int* back_idx, const float* back_d2, int* idx, float* d2,
                            hipStream_t s) {
    if (world < 1 || F < 1 || k < 1 || k > 128 || umax < 0) return hipErrorInvalidValue;
    if (umax > 0)
        fwd_merge_kernel<<<std::max(1u, std::min(cdiv((size_t)umax, 256), 64u)), 256, 0, s>>>(
            world, F, k, uncert, ucount, umax, slot_of, back_idx, back_d2, idx, d2);
    return hipGetLastError();
}

RankLocal rank_local(const double* hd, int rank, const int grid[3], const float* cert_field, int field_g) {
    RankLocal r{};
    if (hd[22] != 0.0 && cert_field && field_g > 0) {
        // a field plan ([6] = [18] = 0 below: the complete box is the own box)
        r.complete.cfield = cert_field;
        r.complete.fg = field_geom_hdr(hd, field_g);
    }
    const double h = hd[6], hs = hd[7];
    const bool full = hd[10] != 0.0;
    // interior width (position-dependent halo); a header without one (0): the single width
    const double hi_ = hd[18] > 0.0 ? hd[18] : h;
    const int c[3] = {rank % grid[0], (rank / grid[0]) % grid[1], rank / (grid[0] * grid[1])};
    r.complete.wide = full ? 0.f : (float)(h - hi_);
    r.complete.zlim = (float)hd[21];
    for (int a = 0; a < 3; ++a) {
        const double lo = hd[a], hi = hd[3 + a];
        const double blo = hd[12 + a], bhi = hd[15 + a];  // equal-volume or count-balanced box
        r.complete.dlo[a] = (float)lo;
        r.complete.dhi[a] = (float)hi;
        r.complete.lo[a] = full || c[a] == 0 ? -INFINITY : (float)(blo - hi_);
        r.complete.hi[a] = full || c[a] == grid[a] - 1 ? INFINITY : (float)(bhi + hi_);
        r.box[a] = std::max(lo, blo - hs);
        r.box[3 + a] = std::min(hi, bhi + hs);
        r.ext[a] = (float)(r.box[3 + a] - r.box[a]);
    }
    return r;
}

double inner_halo_factor(int k) {
    k = std::max(1, k);
    for (int i = 0; i <= 60; ++i) {
        const double f = 1.0 + 0.05 * i;
        const double lam = (double)(k + 1) * f * f * f;
        // P[Poisson(lam) <= k - 1], summed in log space
        double cdf = 0.0;
        for (int j = 0; j < k; ++j) cdf += std::exp(-lam + j * std::log(lam) - std::lgamma(j + 1.0));
        if (cdf <= 1e-12) return f;
    }
    return 4.0;
}

size_t split_hist_scratch_words(int n, const int grid[3], int stage) {
    const int bins = split_hist_rows(grid, stage) * kSplitBins;
    return bins <= kSplitLdsBins ? (size_t)split_hist_blocks(n) * bins : 1;
}

hipError_t launch_split_hist(const float* pts, int n, const SplitHistArgs& a, unsigned* hist, unsigned* scratch,
                             hipStream_t s) {
    // px * py <= 64 keeps xs / ys (px * (py + 1) <= 128) and the rows in range
    if (a.stage < 0 || a.stage > 2 || a.grid[0] < 1 || a.grid[1] < 1 || a.grid[0] * a.grid[1] > kRouteMaxWorld)
        return hipErrorInvalidValue;
    const int bins = split_hist_rows(a.grid, a.stage) * kSplitBins;
    if (n <= 0) return hipMemsetAsync(hist, 0, (size_t)bins * sizeof(unsigned), s);
    if (bins <= kSplitLdsBins) {
        const int nb = split_hist_blocks(n);
        split_hist_lds_kernel<<<nb, 1024, 0, s>>>(pts, n, a, bins, scratch);
        split_hist_sum_kernel<<<(int)cdiv((size_t)bins, 256), 256, 0, s>>>(scratch, nb, bins, hist);
    } else {
        hipError_t e = hipMemsetAsync(hist, 0, (size_t)bins * sizeof(unsigned), s);
        if (e != hipSuccess) return e;
        split_hist_global_kernel<<<std::min((int)cdiv((size_t)n, 256), 2048), 256, 0, s>>>(pts, n, a, hist);
    }
    return hipGetLastError();
}

KN_DEFINE_DEBUG_READER(debug_words_route)

}  // namespace kn
