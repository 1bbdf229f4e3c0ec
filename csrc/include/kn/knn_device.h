// kn/knn_device.h -- device helpers shared by the grid kernels (query.hip) and the tree
// kernels (tree.hip): packed 32-bit candidate keys, the v_med3_u32 top-K insertion, the
// local / global-id modes of a stored point's w field, the XCD-aware block remap and a wave
// bitonic sort of 64-bit (d2, id) keys.
#pragma once

#include <hip/hip_runtime.h>

#include "kn/kernels.h"
#include "kn/wave.h"

namespace kn {

// checked builds also count work (query counters [4..7])
#if defined(KN_CHECKED) && KN_CHECKED
constexpr bool kStats = true;
#else
constexpr bool kStats = false;
#endif

__device__ __forceinline__ float complete_margin(const CompleteBox& cb, float q, int a) {
    return fminf(q - cb.lo[a], cb.hi[a] - q);
}

// Radius up to which the query's K-th ball is certified by the rank's complete box: the smallest
// face margin, each face widened by cb.wide when the whole ball then stays in the wide zone
// (position-dependent halo, CompleteBox). wide = 0 (uniform halo, single GPU): the box margin.
// Density-adaptive halo (cb.cfield): the larger of the own-box margin and the radius the field
// certifies at the query's cell.
__device__ __forceinline__ float complete_margin3(const CompleteBox& cb, float x, float y, float z) {
    float m = INFINITY;
    if (!(cb.wide > 0.f)) {
        m = fminf(fminf(complete_margin(cb, x, 0), complete_margin(cb, y, 1)), complete_margin(cb, z, 2));
    } else {
        const float q[3] = {x, y, z};
        float zq = INFINITY;
#pragma unroll
        for (int a = 0; a < 3; ++a) zq = fminf(zq, fminf(q[a] - cb.dlo[a], cb.dhi[a] - q[a]));
#pragma unroll
        for (int a = 0; a < 3; ++a) {
            float lo = q[a] - cb.lo[a], hi = cb.hi[a] - q[a];  // +inf on domain faces
            if (zq + lo + cb.wide <= cb.zlim) lo += cb.wide;
            if (zq + hi + cb.wide <= cb.zlim) hi += cb.wide;
            m = fminf(m, fminf(lo, hi));
        }
    }
    if (cb.cfield) m = fmaxf(m, cb.cfield[field_cell(cb.fg, x, y, z)]);
    return m;
}

// Output pointers in the global address space. The kernels pick their output pointers at run time
// (the launch's, or a device slot's for batched graphs), which leaves them generic to the compiler:
// it then emits FLAT stores, which count on the LDS counter as well, so every later LDS wait (the
// re-rank's point reads) also waits for the stores in flight. A global pointer gives global_store.
// KN_GLOBAL_OUT=0: the generic pointers (round 5).
#ifndef KN_GLOBAL_OUT
#define KN_GLOBAL_OUT 1
#endif
#if KN_GLOBAL_OUT
typedef __attribute__((address_space(1))) unsigned out_u32_t;
typedef __attribute__((address_space(1))) float out_f32_t;
#else
typedef unsigned out_u32_t;
typedef float out_f32_t;
#endif
__device__ __forceinline__ out_u32_t* out_ptr(unsigned* p) { return (out_u32_t*)p; }
__device__ __forceinline__ out_f32_t* out_ptr(float* p) { return (out_f32_t*)p; }

// Row stores of the query kernels (KN_VEC_OUT: query.hip re-rank window pass, tree.hip leaf
// search): positions per global store -- 4 where the K
// bucket is a multiple of 4, 2 for K=50 (200-byte rows: 8-byte aligned); 0 = per-entry stores
#ifndef KN_VEC_OUT
#define KN_VEC_OUT 1
#endif
#ifndef KN_VEC_TAIL
#define KN_VEC_TAIL 0
#endif
template <int KT>
constexpr int out_vec_width() {
    return !KN_VEC_OUT ? 1 : (KT % 4 == 0 || (KN_VEC_TAIL && KT % 4 == 2) ? 4 : KT % 2 == 0 ? 2 : 1);
}
// KN_VEC_TAIL: a k with k % 4 == 2 (K=50, or k=6 in the K=8 bucket) is also stored 4 positions
// at a time -- its rows are only 8-byte aligned (dword alignment is what the 16-byte global
// stores need) -- plus one 2-position store for the row's last two. 0 (default): the K=50 bucket
// stores 2 positions at a time, and other buckets' k % 4 == 2 queries one entry per store.
// Measured: K=50 query 0.664 -> 0.729 ms with the tail, 100 / 30 steps 0.536 -> 0.600 (the
// 16-byte stores at 8-byte aligned rows split); tree surfaces -1 % (profiles/ab_r6_vec_tail.txt).
// run-time check of a query's k against the store width V (and the 2-position tail)
template <int V>
__device__ __forceinline__ bool out_vec_ok(int k, const void* p0, const void* p1) {
    const bool kk = V == 4 ? ((k & 3) == 0 || (KN_VEC_TAIL && (k & 3) == 2)) : (k % V) == 0;
    // row starts: k * 4 bytes apart; with the tail they are 8-byte aligned only
    const uintptr_t amask = V == 4 && (k & 3) != 0 ? 7u : (uintptr_t)(4 * V - 1);
    return V > 1 && kk && ((reinterpret_cast<uintptr_t>(p0) | reinterpret_cast<uintptr_t>(p1)) & amask) == 0;
}
typedef unsigned kn_u32x2 __attribute__((ext_vector_type(2)));
typedef unsigned kn_u32x4 __attribute__((ext_vector_type(4)));
typedef float kn_f32x2 __attribute__((ext_vector_type(2)));
typedef float kn_f32x4 __attribute__((ext_vector_type(4)));
template <int V>
__device__ __forceinline__ void store_vec(out_u32_t* p, const unsigned (&v)[V]) {
    if constexpr (V == 4) *(__attribute__((address_space(1))) kn_u32x4*)p = kn_u32x4{v[0], v[1], v[2], v[3]};
    else if constexpr (V == 2) *(__attribute__((address_space(1))) kn_u32x2*)p = kn_u32x2{v[0], v[1]};
    else *p = v[0];
}
template <int V>
__device__ __forceinline__ void store_vec(out_f32_t* p, const float (&v)[V]) {
    if constexpr (V == 4) *(__attribute__((address_space(1))) kn_f32x4*)p = kn_f32x4{v[0], v[1], v[2], v[3]};
    else if constexpr (V == 2) *(__attribute__((address_space(1))) kn_f32x2*)p = kn_f32x2{v[0], v[1]};
    else *p = v[0];
}
__device__ __forceinline__ bool pair_less(float da, unsigned ia, float db, unsigned ib) {
    return da < db || (da == db && ia < ib);
}

// The w field of a stored point. Default mode: its original (local) index -- queries are the
// indices < n_queries, the output row is that index, and the output id is id_map[index].
// Global-id mode (row_of != nullptr, multi-GPU ranks): w already holds the point's GLOBAL id,
// with kHaloBit set on halo (non-query) points, and row_of[stored index] gives a query's output
// row. The output ids then need no gather through id_map: at 12.5M points per rank that
// random gather (K per query from a 50 MB table) cost more than the whole lane-walk search.
constexpr unsigned kHaloBit = 0x80000000u;
template <class A>
__device__ __forceinline__ bool w_live(const A& a, unsigned w) {
    return a.row_of ? !(w & kHaloBit) : ((int)w >= a.q_lo && (int)w < a.n_queries);
}
template <class A>
__device__ __forceinline__ unsigned w_id(const A& a, unsigned w) { return a.row_of ? (w & ~kHaloBit) : w; }
template <class A>
__device__ __forceinline__ unsigned w_row(const A& a, unsigned w, unsigned sidx) {
    return a.row_of ? a.row_of[KN_IDX(sidx, (unsigned)a.n, 231)] : w - (unsigned)a.q_lo;
}
template <class A>
__device__ __forceinline__ unsigned out_id(const A& a, unsigned id) {
    return (a.row_of || !a.id_map) ? id : a.id_map[KN_IDX(id, (unsigned)a.n, 232)];
}

// Bijective XCD-aware remap: consecutive tiles (which share halo cells) land on one XCD's L2.
__device__ __forceinline__ int xcd_remap(int b, int nblocks) {
    const int xcd = b & 7, idx = b >> 3;
    const int q = nblocks >> 3, r = nblocks & 7;
    return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + idx;
}

__device__ __forceinline__ unsigned long long pack_key64(float d, unsigned id) {
    return ((unsigned long long)__float_as_uint(d) << 32) | id;
}

// Ascending bitonic sort of E*64 64-bit keys held E per lane (element index e*64 + lane):
// cross-lane stages exchange through ds_bpermute (__shfl_xor), the stride-64 stage of E = 2
// compares a lane's two elements.
template <int E>
__device__ __forceinline__ void wave_bitonic_sort_u64(unsigned long long (&v)[E], int lane) {
    constexpr int N = 64 * E;
#pragma clang loop unroll(full)
    for (int size = 2; size <= N; size <<= 1) {
#pragma clang loop unroll(full)
        for (int stride = size >> 1; stride > 0; stride >>= 1) {
            if (stride >= 64) {
#pragma unroll
                for (int e = 0; e < E; ++e) {
                    const int f = e ^ (stride >> 6);
                    if (e < f) {
                        const bool up = (((e << 6) | lane) & size) == 0;
                        const unsigned long long mn = v[e] < v[f] ? v[e] : v[f], mx = v[e] < v[f] ? v[f] : v[e];
                        v[e] = up ? mn : mx;
                        v[f] = up ? mx : mn;
                    }
                }
            } else {
#pragma unroll
                for (int e = 0; e < E; ++e) {
                    const unsigned lo = (unsigned)__shfl_xor((int)(unsigned)v[e], stride, 64);
                    const unsigned hi = (unsigned)__shfl_xor((int)(unsigned)(v[e] >> 32), stride, 64);
                    const unsigned long long o = ((unsigned long long)hi << 32) | lo;
                    const bool up = (((e << 6) | lane) & size) == 0;
                    const bool lower = (lane & stride) == 0;
                    const unsigned long long mn = v[e] < o ? v[e] : o, mx = v[e] < o ? o : v[e];
                    v[e] = (up == lower) ? mn : mx;
                }
            }
        }
    }
}

// Packed 32-bit key of one candidate: squared-distance float bits with the low SB mantissa
// bits replaced by the candidate's LDS slot (one v_bfi_b32).
__device__ __forceinline__ unsigned cand_key(const float4& p, float qx, float qy, float qz, unsigned himask,
                                             int s, int /*qslot*/) {
    const float dx = p.x - qx, dy = p.y - qy, dz = p.z - qz;
    const float d2 = fmaf(dz, dz, fmaf(dy, dy, dx * dx));
    unsigned key;
    // VOP3 reads at most one SGPR on gfx9: keep the (loop-invariant) mask in a VGPR
    asm("v_bfi_b32 %0, %1, %2, %3" : "=v"(key) : "v"(himask), "v"(__float_as_uint(d2)), "s"((unsigned)s));
    return key;
}

// cand_key with a per-lane (VGPR) slot: the lane-walk variant's candidates differ per lane.
__device__ __forceinline__ unsigned cand_key_v(const float4& p, float qx, float qy, float qz, unsigned himask,
                                               int s) {
    const float dx = p.x - qx, dy = p.y - qy, dz = p.z - qz;
    const float d2 = fmaf(dz, dz, fmaf(dy, dy, dx * dx));
    unsigned key;
    // himask is wave-uniform: an SGPR operand (a VGPR constraint re-materialised it with a v_mov
    // per candidate inside the unrolled loop)
    asm("v_bfi_b32 %0, %1, %2, %3" : "=v"(key) : "s"(himask), "v"(__float_as_uint(d2)), "v"((unsigned)s));
    return key;
}

// Sorted-array insertion of `key` into keys[0..KM) (ascending), dropping the largest:
// new[j] = med3(old[j-1], key, old[j]) -- one v_med3_u32 per slot, all independent. Skipped
// (uniform branch) when no lane of the wave improves; a non-improving key is a no-op anyway.
//
// Split networks (KN_TOPK_SPLIT): slots below the lowest insertion position of the wave's
// inserting lanes do not change, so when every inserting lane's key is >= keys[LO-1] (a uniform
// ballot) the network starts at LO. A new candidate inside the K-th ball is uniformly placed in
// it, i.e. at a uniform rank: late in a walk, when few lanes insert at once, the wave's lowest
// position is often in the upper half. Numpy lockstep replay of the lane walk
// (scripts/sim_wave_order.py machinery, /tmp replays recorded in DESIGN.md): med3 slots per wave
// K=16 -8 % (half) / -6 % (quarters), K=50 -13 % / -17 %. 0 = one network, 1 = halves,
// 2 = quarters.
//
// Gated tiers (KN_TOPK_TIERS = T > 1, round 6): the SAME network, run top-down in T slices, each
// lower slice behind its own uniform ballot. new[j] only reads old[j-1], old[j] and the key, so
// slices [LO, HI) computed from the top keep every read an old value; and for a lane whose key is
// >= old[LO-1], every slot below LO is unchanged by its own formula, so a slice that no lane of
// the wave reaches is skipped exactly. Unlike the split networks above there is ONE copy of every
// med3 (no duplicated upper part): per candidate step a slice costs one compare + branch, and saves
// its med3s whenever no inserting lane's key falls into it (late in a walk most insertions land in
// the upper ranks of a full list).
#ifndef KN_TOPK_SPLIT
#define KN_TOPK_SPLIT 0
#endif
#ifndef KN_TOPK_TIERS
#define KN_TOPK_TIERS 1
#endif
template <int KM, int LO>
__device__ __forceinline__ void topk_net(unsigned (&keys)[KM], unsigned key) {
#pragma unroll
    for (int j = KM - 1; j > LO; --j) keys[j] = med3_u32(keys[j - 1], key, keys[j]);
    if constexpr (LO == 0) keys[0] = min(keys[0], key);
    else keys[LO] = med3_u32(keys[LO - 1], key, keys[LO]);
}
// slots [LO, HI) of the network (top-down); LO = 0 takes the plain min at slot 0
template <int KM, int LO, int HI>
__device__ __forceinline__ void topk_slice(unsigned (&keys)[KM], unsigned key) {
#pragma unroll
    for (int j = HI - 1; j >= LO; --j) keys[j] = j == 0 ? min(keys[0], key) : med3_u32(keys[j - 1], key, keys[j]);
}
// tier t of T covers slots [lo(t), lo(t - 1)) from the top: t = 0 is the top slice
template <int KM, int T, int t>
__device__ __forceinline__ void topk_tiers(unsigned (&keys)[KM], unsigned key) {
    constexpr int HI = t == 0 ? KM : (KM * (T - t)) / T;
    constexpr int LO = (KM * (T - t - 1)) / T;
    topk_slice<KM, LO, HI>(keys, key);
    if constexpr (t + 1 < T && LO > 0) {
        // the next slice changes only lanes whose key is below old[LO - 1] (still old: the slices
        // above never write below LO)
        if (__builtin_amdgcn_ballot_w64(key < keys[LO - 1])) topk_tiers<KM, T, t + 1>(keys, key);
    }
}
template <int KM, int SPLIT = KN_TOPK_SPLIT, int TIERS = KN_TOPK_TIERS>
__device__ __forceinline__ unsigned topk_push(unsigned (&keys)[KM], unsigned key) {
    if (__builtin_amdgcn_ballot_w64(key < keys[KM - 1])) {
        if constexpr (TIERS > 1 && KM >= 2 * TIERS) {
            topk_tiers<KM, TIERS, 0>(keys, key);
        } else if constexpr (SPLIT == 0 || KM < 8) {
            topk_net<KM, 0>(keys, key);
        } else if constexpr (SPLIT == 1) {
            constexpr int H = KM / 2;
            if (__builtin_amdgcn_ballot_w64(key < keys[H - 1])) topk_net<KM, 0>(keys, key);
            else topk_net<KM, H>(keys, key);
        } else {
            constexpr int Q = KM / 4, H = KM / 2, T = (3 * KM) / 4;
            if (__builtin_amdgcn_ballot_w64(key < keys[H - 1])) {
                if (__builtin_amdgcn_ballot_w64(key < keys[Q - 1])) topk_net<KM, 0>(keys, key);
                else topk_net<KM, Q>(keys, key);
            } else {
                if (__builtin_amdgcn_ballot_w64(key < keys[T - 1])) topk_net<KM, H>(keys, key);
                else topk_net<KM, T>(keys, key);
            }
        }
        return 1u;
    }
    return 0u;
}

// Wave-wide sum (DPP within rows of 16, then the 4 row totals).
__device__ __forceinline__ unsigned wave_sum_u32(unsigned x) {
    x += (unsigned)__builtin_amdgcn_update_dpp(0, (int)x, KN_DPP_QUAD_1032, 0xF, 0xF, false);
    x += (unsigned)__builtin_amdgcn_update_dpp(0, (int)x, KN_DPP_QUAD_2301, 0xF, 0xF, false);
    x += (unsigned)__builtin_amdgcn_update_dpp(0, (int)x, KN_DPP_ROW_HALF_MIRROR, 0xF, 0xF, false);
    x += (unsigned)__builtin_amdgcn_update_dpp(0, (int)x, KN_DPP_ROW_MIRROR, 0xF, 0xF, false);
    return (unsigned)__builtin_amdgcn_readlane((int)x, 0) + (unsigned)__builtin_amdgcn_readlane((int)x, 16) +
           (unsigned)__builtin_amdgcn_readlane((int)x, 32) + (unsigned)__builtin_amdgcn_readlane((int)x, 48);
}

}  // namespace kn
