// kn/wave.h -- wave64 device helpers for gfx950 (DPP reductions, med3, cell mapping).
#pragma once

#include <hip/hip_runtime.h>

#include "kn/kernels.h"

namespace kn {

// ---- checked builds (-DKN_CHECKED=1): bounds-checked indexing --------------------------
// Every wrapped index is tested against its buffer's extent; a violation is recorded in a
// per-translation-unit device word (first failing site code, index, limit) and the access is
// redirected to element 0, so a bug shows up as a report instead of a GPU memory fault.
// The release build compiles the macro away.
#if defined(KN_CHECKED) && KN_CHECKED
static __device__ unsigned kn_dbg_words[4];
__device__ __noinline__ long long kn_dbg_fail(unsigned code, long long i, long long n) {
    if (atomicCAS(&kn_dbg_words[0], 0u, code) == 0u) {
        kn_dbg_words[1] = (unsigned)i;
        kn_dbg_words[2] = (unsigned)n;
        kn_dbg_words[3] = (unsigned)(i >> 32);
    }
    return 0;
}
#define KN_IDX(i, n, code) \
    (((unsigned long long)(long long)(i) < (unsigned long long)(long long)(n)) \
         ? (i)                                                                 \
         : (__decltype_nr(i))kn_dbg_fail((code), (long long)(i), (long long)(n)))
template <class T> struct kn_nr { using type = T; };
template <class T> struct kn_nr<T&> { using type = T; };
#define __decltype_nr(x) typename kn::kn_nr<decltype(x)>::type
#define KN_DEFINE_DEBUG_READER(NAME)                                                     \
    hipError_t NAME(unsigned out[4], bool reset) {                                        \
        hipError_t e = hipMemcpyFromSymbol(out, HIP_SYMBOL(kn_dbg_words), 16, 0, hipMemcpyDeviceToHost); \
        if (e == hipSuccess && reset) {                                                   \
            const unsigned z[4] = {0, 0, 0, 0};                                           \
            e = hipMemcpyToSymbol(HIP_SYMBOL(kn_dbg_words), z, 16, 0, hipMemcpyHostToDevice); \
        }                                                                                 \
        return e;                                                                         \
    }
#else
#define KN_IDX(i, n, code) (i)
#define KN_DEFINE_DEBUG_READER(NAME)                       \
    hipError_t NAME(unsigned out[4], bool) {               \
        out[0] = out[1] = out[2] = out[3] = 0xFFFFFFFFu;   \
        return hipSuccess;                                 \
    }
#endif

// DPP controls (gfx9 encoding)
#define KN_DPP_QUAD_1032 0xB1
#define KN_DPP_QUAD_2301 0x4E
#define KN_DPP_ROW_MIRROR 0x140
#define KN_DPP_ROW_HALF_MIRROR 0x141

// Row (16-lane) reduction with DPP, then combine the 4 rows through readlane (SGPR result,
// wave-uniform). ~12 instructions, no LDS traffic.
#define KN_WAVE_REDUCE(NAME, T, OP)                                                            \
    __device__ __forceinline__ T NAME(T x) {                                                   \
        x = OP(x, (T)__builtin_amdgcn_update_dpp((int)x, (int)x, KN_DPP_QUAD_1032, 0xF, 0xF, false)); \
        x = OP(x, (T)__builtin_amdgcn_update_dpp((int)x, (int)x, KN_DPP_QUAD_2301, 0xF, 0xF, false)); \
        x = OP(x, (T)__builtin_amdgcn_update_dpp((int)x, (int)x, KN_DPP_ROW_HALF_MIRROR, 0xF, 0xF, false)); \
        x = OP(x, (T)__builtin_amdgcn_update_dpp((int)x, (int)x, KN_DPP_ROW_MIRROR, 0xF, 0xF, false)); \
        const T a = (T)__builtin_amdgcn_readlane((int)x, 0);                                   \
        const T b = (T)__builtin_amdgcn_readlane((int)x, 16);                                  \
        const T c = (T)__builtin_amdgcn_readlane((int)x, 32);                                  \
        const T d = (T)__builtin_amdgcn_readlane((int)x, 48);                                  \
        return OP(OP(a, b), OP(c, d));                                                         \
    }

__device__ __forceinline__ unsigned kn_umin(unsigned a, unsigned b) { return a < b ? a : b; }
__device__ __forceinline__ unsigned kn_umax(unsigned a, unsigned b) { return a > b ? a : b; }
__device__ __forceinline__ int kn_imin(int a, int b) { return a < b ? a : b; }
__device__ __forceinline__ int kn_imax(int a, int b) { return a > b ? a : b; }

KN_WAVE_REDUCE(wave_min_u32, unsigned, kn_umin)
KN_WAVE_REDUCE(wave_max_u32, unsigned, kn_umax)

// One wave reduces the per-block bbox partials of launch_bbox_partials (kn/kernels.h):
// out[a] = max over blocks of partials[a * stride + b], a < 6. Result wave-uniform.
__device__ __forceinline__ void bbox_reduce_partials(const unsigned* __restrict__ partials, int nblocks,
                                                     int stride, unsigned out[6]) {
    const int lane = threadIdx.x & 63;
#pragma unroll
    for (int a = 0; a < 6; ++a) {
        unsigned v = 0u;
        for (int b = lane; b < nblocks; b += 64) v = v > partials[a * stride + b] ? v : partials[a * stride + b];
        out[a] = wave_max_u32(v);
    }
}
KN_WAVE_REDUCE(wave_min_i32, int, kn_imin)
KN_WAVE_REDUCE(wave_max_i32, int, kn_imax)

// Wave-wide (min(mn), max(mx)) of small ints (|v| < 32767; INT_MAX / INT_MIN sentinels
// saturate) in ONE reduction: (-mn, mx) packed as two int16 and reduced with v_pk_max_i16.
// Result is wave-uniform (scalar registers).
__device__ __forceinline__ unsigned pk_max_i16(unsigned a, unsigned b) {
    unsigned r;
    asm("v_pk_max_i16 %0, %1, %2" : "=v"(r) : "v"(a), "v"(b));
    return r;
}
__device__ __forceinline__ int2 wave_minmax_i32(int mn, int mx) {
    mn = mn < -32767 ? -32767 : (mn > 32767 ? 32767 : mn);
    mx = mx < -32768 ? -32768 : (mx > 32767 ? 32767 : mx);
    unsigned v = ((unsigned)(-mn) & 0xFFFFu) | ((unsigned)mx << 16);
    v = pk_max_i16(v, (unsigned)__builtin_amdgcn_update_dpp((int)v, (int)v, KN_DPP_QUAD_1032, 0xF, 0xF, false));
    v = pk_max_i16(v, (unsigned)__builtin_amdgcn_update_dpp((int)v, (int)v, KN_DPP_QUAD_2301, 0xF, 0xF, false));
    v = pk_max_i16(v, (unsigned)__builtin_amdgcn_update_dpp((int)v, (int)v, KN_DPP_ROW_HALF_MIRROR, 0xF, 0xF, false));
    v = pk_max_i16(v, (unsigned)__builtin_amdgcn_update_dpp((int)v, (int)v, KN_DPP_ROW_MIRROR, 0xF, 0xF, false));
    int lo = -32768, hi = -32768;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
        const unsigned u = (unsigned)__builtin_amdgcn_readlane((int)v, 16 * r);
        lo = max(lo, (int)(short)(u & 0xFFFFu));
        hi = max(hi, (int)(short)(u >> 16));
    }
    return make_int2(-lo, hi);
}

// Inclusive prefix sum over the 64 lanes.
__device__ __forceinline__ int wave_inclusive_scan_add(int v) {
    const int lane = threadIdx.x & 63;
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) {
        const int t = __shfl_up(v, off, 64);
        if (lane >= off) v += t;
    }
    return v;
}

// v_med3_u32: the median of three. With lo <= hi this is clamp(x, lo, hi), the single-op
// step of a sorted-array insertion (new[j] = med3(old[j-1], x, old[j])).
__device__ __forceinline__ unsigned med3_u32(unsigned a, unsigned b, unsigned c) {
    unsigned r;
    asm("v_med3_u32 %0, %1, %2, %3" : "=v"(r) : "v"(a), "v"(b), "v"(c));
    return r;
}

__device__ __forceinline__ int clampi(int v, int lo, int hi) { return v < lo ? lo : (v > hi ? hi : v); }

// Point -> cell coordinate along one axis. Identical arithmetic everywhere (binning, queries,
// fallback) so a point's cell is reproducible bit-for-bit.
// floor((p - origin) * inv_cell) clamped to [0, dims - 1]: clamping the float to [0, dims - 1/2]
// first makes the truncating convert a floor and the integer clamp unnecessary (same integer for
// every input, NaN -> 0; dims < 2^22), 4 VALU instead of 8 on the lane walk's per-row path
#ifndef KN_FAST_CELL
#define KN_FAST_CELL 1
#endif
__device__ __forceinline__ int cell_coord(const GridGeom& g, int a, float p) {
    const float f = (p - g.origin[a]) * g.inv_cell[a];
#if KN_FAST_CELL
    return (int)fminf(fmaxf(f, 0.f), (float)g.dims[a] - 0.5f);
#else
    const int i = (int)floorf(fminf(fmaxf(f, -1.f), (float)g.dims[a]));
    return clampi(i, 0, g.dims[a] - 1);
#endif
}
__device__ __forceinline__ int cell_of(const GridGeom& g, const float p[3]) {
    const int i = cell_coord(g, 0, p[0]);
    const int j = cell_coord(g, 1, p[1]);
    const int k = cell_coord(g, 2, p[2]);
    return i + g.dims[0] * (j + g.dims[1] * k);
}

// Square root of a search-radius bound: the hardware v_sqrt_f32 (<= 1 ulp) without the
// correctly-rounded expansion sqrtf() compiles to (~20 VALU: denormal scaling + two refinement
// FMAs + class fix-up). Every caller scales the result by 1 + 1e-6 and adds the grid eps, which
// covers the ulp, so the row cuts stay conservative. Row setup is on the lane walk's per-row path.
#ifndef KN_FAST_SQRT
#define KN_FAST_SQRT 1
#endif
__device__ __forceinline__ float sqrt_bound(float x) {
#if KN_FAST_SQRT
    return __builtin_amdgcn_sqrtf(x);
#else
    return sqrtf(x);
#endif
}

// Lower bound of the distance from coordinate q to the slab of cells [c0, c1] on axis a
// (conservative by g.eps so rounding in binning can never make it exceed a true distance).
__device__ __forceinline__ float slab_dist(const GridGeom& g, int a, float q, int c0, int c1) {
    const float lo = g.origin[a] + (float)c0 * g.cell[a] - g.eps;
    const float hi = g.origin[a] + (float)(c1 + 1) * g.cell[a] + g.eps;
    return fmaxf(0.f, fmaxf(lo - q, q - hi));
}

}  // namespace kn
