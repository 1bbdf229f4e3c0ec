// step_flag.h -- device side of the distributed step's steady-state check (route.hip
// steady_flag_partials_kernel, and the last workgroup of the exact finish kernel in deferred mode,
// query.hip). Device code only: include from .hip sources.
//
// The check: this share's {lo, hi, n} (reduced from the routing pass's per-block bbox partials,
// the encoding of launch_bbox_partials) equals the planned meta, every send count equals the
// planned one, and no query of the step was left uncertified (counters[1]). 0 = steady.
#pragma once

#include <hip/hip_runtime.h>

#include "kn/kernels.h"
#include "kn/wave.h"

namespace kn {

__device__ __forceinline__ float step_flag_unord(unsigned u) {
    return __uint_as_float((u & 0x80000000u) ? (u & 0x7fffffffu) : ~u);
}

// Whole workgroup (any multiple of 64 threads <= 1024) calls it; returns the flag in thread 0
// (other threads: 0). uncertified: the step's counters[1], read by the caller.
__device__ inline int step_flag_eval(const unsigned* __restrict__ partials, int nb, int stride, int n,
                                     const double* __restrict__ planned, const int* __restrict__ totals,
                                     const int* __restrict__ ptotals, int nt, unsigned uncertified) {
    __shared__ unsigned red[6][16];
    __shared__ unsigned words_s[6];
    __shared__ int out_s;
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    const int nbr = n > 0 ? nb : 0;
#pragma unroll
    for (int a = 0; a < 6; ++a) {
        unsigned v = 0u;
        for (int b = threadIdx.x; b < nbr; b += blockDim.x) v = max(v, partials[(size_t)a * stride + b]);
        v = wave_max_u32(v);
        if (lane == 0) red[a][wid] = v;
    }
    __syncthreads();
    if (threadIdx.x < 6) {
        unsigned v = 0u;
        for (int w = 0; w < (int)(blockDim.x >> 6); ++w) v = max(v, red[threadIdx.x][w]);
        words_s[threadIdx.x] = v;
    }
    __syncthreads();
    if (wid == 0) {
        unsigned words[6];
#pragma unroll
        for (int a = 0; a < 6; ++a) words[a] = words_s[a];
        bool diff = false;
        if (lane < 8) {
            unsigned wt = words[0];
#pragma unroll
            for (int a = 1; a < 6; ++a) wt = (lane == a) ? words[a] : wt;
            double v;
            if (lane < 3) v = n > 0 ? (double)step_flag_unord(~wt) : (double)INFINITY;
            else if (lane < 6) v = n > 0 ? (double)step_flag_unord(wt) : -(double)INFINITY;
            else if (lane == 6) v = (double)n;
            else v = 0.0;
            diff = v != planned[lane];  // a NaN never matches
        }
        for (int i = lane; i < nt; i += 64) diff |= totals[i] != ptotals[i];
        const bool any = __builtin_amdgcn_ballot_w64(diff) != 0ull;
        if (lane == 0) out_s = (any ? 1 : 0) + (uncertified != 0u ? 1 : 0);
    }
    __syncthreads();
    return threadIdx.x == 0 ? out_s : 0;
}

}  // namespace kn
