// query.hip -- k-nearest-neighbour queries on gfx950 (wave64, LDS-staged, certified).
//
// Reference hot path: knearests.cu:93-148 (`knearest`): one 32-thread block per 32 points,
// per-thread K-entry max-heap in shared memory, ring walk over a 29,791-entry offset table,
// racy early-exit bookkeeping. This file re-designs it for CDNA4:
//
// knn_tile_kernel  -- one 256-thread workgroup per TX*TY*TZ cell tile.
//   1. The tile plus H halo rings of cells is staged into LDS as float4 {x,y,z,bits(orig)}
//      (rows of the x-fastest grid are contiguous runs of the sorted array -> coalesced
//      16-B loads).
//   2. Each wave takes 64 of the tile's queries (lanes = queries). The candidate stream is
//      WAVE-UNIFORM: rows (y,z) of the wave's region are visited centre-out, every lane
//      derives the x-range of cells its current K-th distance still needs, and a DPP
//      min/max gives the union; every lane then reads the same LDS point (broadcast).
//   3. Top-K lives in registers as K+M packed 32-bit keys: the squared distance's float
//      bits with the low SB mantissa bits replaced by the candidate's LDS slot. Positive
//      float bits order like the floats, so insertion into the sorted key array is ONE
//      v_med3_u32 per slot (new[j] = med3(old[j-1], key, old[j])), branch-free; the whole
//      network is skipped by a uniform ballot when no lane improves.
//   4. Exact re-rank: the K+M kept slots are re-evaluated in full fp32 and ordered by
//      (distance, original id) with a streaming window (a slot's position = its valid
//      predecessors +- the same-bucket neighbours that cross it), rare long runs of equal
//      buckets and truncation near-ties by a wave-cooperative bitonic sort / exact re-scan.
//      A query is CERTIFIED when (a) its exact K-th distance does not exceed the truncation
//      floor of the (K+M)-th key, so nothing truncated away can be closer, and (b) the K-th
//      distance is within the distance to the boundary of the region it scanned (and of the
//      rank's complete box in multi-GPU runs). Uncertified queries (rare) are appended to a
//      list for the exact kernel below. (Reference defect D1: its "no guarantee" flag never
//      fires, knearests.cu:136-139.)
//
// knn_exact_coop_kernel -- one WAVE per query: analytic Chebyshev shell walk from the query's
//   cell, candidates tested 64 at a time, those within the current K-th distance compacted
//   into a per-wave LDS buffer that is bitonic-sorted and truncated to K whenever it fills;
//   a true per-query stopping rule (distance to the scanned block). Serves the fallback list,
//   and every query when tiles are disabled.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <climits>
#include <cmath>
#include <cstdlib>
#include <cstring>
#include <type_traits>

#include "kn/kernels.h"
#include "kn/knn_device.h"
#include "kn/step_flag.h"
#include "kn/wave.h"

namespace kn {

namespace {

constexpr unsigned SENT = 0xFFFFFFFFu;
// Threads per tile workgroup. 512 threads with taller tiles lost the round-4 A/B at every tile
// shape (900K K=16 0.294 -> 0.325-0.360 ms/step, K=50 0.967 -> 0.944-1.147;
// profiles/ab_r4_tiles_margin.txt)
constexpr int kWG = 256;
constexpr int kWaves = kWG / 64;

struct TileArgs {
    const float4* sorted;
    const int* cell_start;
    const GridGeom* geom;
    int n;
    int X, Y, Z;
    int k;
    int n_queries;
    int q_lo;                // local mode: queries are original indices [q_lo, n_queries), row = w - q_lo
    const unsigned* id_map;
    const unsigned* row_of;  // non-null: global-id mode (see w_live / w_id / w_row)
    CompleteBox complete;
    unsigned* out_idx;
    float* out_dist;
    unsigned* const* out_idx_ref;  // non-null: the output pointers are read from these slots
    float* const* out_dist_ref;
    unsigned* fallback_list;
    unsigned* counters;
    int TX, TY, TZ, H;
    int Hx;         // x halo in x sub-cells (H * xsub)
    int cap;        // LDS point capacity (multiple of 64)
    int slot_bits;  // log2(cap)
    int ntx, nty, ntz;
    int tblock;     // tile blocking of the workgroup order (tile_coords; KN_TILE_BLOCK)
    int cb_stride;  // max staged cells per row + 1
    int max_rows;
    int flags;      // kQueryForceRescan: every query takes the exact re-scan (tests)
    // lane walk row order (KN_ROW_ORDER): the (2H+1)^2 row offsets (oy, oz), one byte each
    // ((oy + 8) | (oz + 8) << 4), sorted by their expected squared distance with +1 on the near
    // side of the query's cell; each lane mirrors it to its own position (row_order_table)
    unsigned row_order[32];
    int row_mirror;  // 1: each lane mirrors the table to its own cell position (distance order)
    int n_outer;     // KN_OUTER_PACK: row_order holds the n_outer rows of Chebyshev ring >= 2
};
constexpr int kRowOrderMax = 128;

// gathers in flight per lane in the K=50 bucket's walk: 1 measured best in round 2; with the round-6
// gated-tier networks and grouped re-rank, 2 (together with KN_RERANK_GROUP=8): K=50 query 0.854 ->
// 0.810 ms, pipelined 100 / 30 0.559 -> 0.546, 20 / 5 0.626 -> 0.612 (profiles/ab_r6_k50.txt)
// ... and in the K <= 40 buckets (3 since round 2, profiles/ab_r2_lane_unroll.txt)
#ifndef KN_LANE_UNROLL40
#define KN_LANE_UNROLL40 3
#endif
#ifndef KN_LANE_UNROLL50
#define KN_LANE_UNROLL50 2
#endif
#ifndef KN_LANE_UNROLL
#define KN_LANE_UNROLL 2
#endif
// Lane walk region: the lane's own cell +- H, then (full mode) the rest of the staged block
// (tile + H) for the lanes whose bound still reaches past their own box. KN_LANE_FULL: 0 never,
// 1 for K buckets > 40 (measured: 900K K=50 2.41 -> 2.22 ms with 2728 -> 638 exact-path
// queries, K=64 3.31 -> 3.29; but K=16 0.349 -> 0.366, K=32 0.947 -> 0.966 from the extra
// code; profiles/ab_r1_lane_full.jsonl), 2 always.
#ifndef KN_LANE_FULL
#define KN_LANE_FULL 1
#endif
// Lane walk row order: z-slab then y centre-out (0, +1, -1, +2, -2) for every lane, or the
// host-built distance-sorted table of TileArgs::row_order, mirrored per lane so the near side of
// the query's own cell comes first (rows closer to the query tighten its bound sooner; numpy
// replay at 3.4 points/cell, K=16: 115 -> 103 candidates per query). KN_ROW_ORDER 0 = never,
// 1 = always, 2 = the whole-block walk only (K > 40). Interleaved in-process A/B, 900K uniform,
// identical rows (profiles/ab_r3_row_order.jsonl): K=50 query 0.943 -> 0.794 ms, but K=8 +4 %,
// K=16 -1 %, K=32 +13 % (the row-synchronous wave pays the longest lane span of every row, and
// the per-lane mirror makes the spans of one row iteration more uneven).
#ifndef KN_ROW_ORDER
#define KN_ROW_ORDER 2
#endif
// (A ring-order table without the mirror for K <= 40 lost too: K=8 +8 %, K=32 +8 %,
// profiles/ab_r3_ring.jsonl; removed in round 4.)
// KN_OUTER_PACK (lane walk, K <= 40, the fixed order): the 3x3 rows around the query's row stay
// row-synchronous, the outer rows (Chebyshev ring >= 2 of the (2H+1)^2 block) are PACKED: each
// lane marks the outer rows its bound still reaches (a 64-bit mask, distances from 8 per-lane
// slab gaps selected by the uniform table entry), then iteration i visits every lane's i-th marked
// row. The row-synchronous loop paid, for each of up to 16 outer rows, the longest span of the
// few lanes whose bound was still wide (numpy replay: outer rows 56 candidate steps over 9.2 row
// iterations per wave at K=16 -> 26 over 3.8). Interleaved A/B, 900K uniform, identical rows
// (profiles/ab_r3_outer_pack.jsonl): query K=12 -5 %, K=16 -2 %, K=24 -17 %, K=32 -3 %, K=40 -6 %,
// blue noise K=16 -5 %, 300K K=16 -12 %; K=8 +9 % (its outer rows are almost never needed, the
// mask costs more): 0 = off, 1 = every K <= 40 bucket, 2 = the K buckets 12..40 and 64 (default),
// 3 = the K buckets 12..64. Round 4, the whole-block walk (K > 40) packing its outer ring instead
// of the distance-sorted table (interleaved, identical rows, profiles/ab_r4_outer_pack_k64.txt):
// K=64 1.189 -> 1.128 ms/step, but K=50 0.912 -> 0.932 (the sorted table stays there).
// Oracle check on clustered clouds (profiles/diag_r3_outer_pack_oracle.txt).
#ifndef KN_OUTER_PACK
#define KN_OUTER_PACK 2
#endif
// (Round 4: the packed walk's 3x3 inner rows in the mirrored expected-distance order instead of
// centre-out z/y lost at every K: K=16 +1.3 %, K=32 +0.8 %, K=50 +2 %, K=64 +2.5 %;
// profiles/ab_r4_pack_inner_sorted.txt. Removed.)
template <int KT>
constexpr bool outer_pack_k() {
    return KN_OUTER_PACK == 1 ? KT <= 40
         : KN_OUTER_PACK == 2 ? ((KT >= 12 && KT <= 40) || KT == 64)
         : KN_OUTER_PACK == 3 ? (KT >= 12 && KT <= 64) : false;
}
// Default AutoParams::xsub of the tile path for K <= KN_XSUB_MAX_K. Interleaved A/B at 900K
// uniform (profiles/ab_r3_xsub.jsonl): xsub 2 query K=8 0.207 -> 0.198, K=16 0.305 -> 0.292 ms
// (build +3 us), K=32 +2 %, K=50 +4 %; xsub 4 at K=16 0.318 -> 0.301 but build +11 us.
#ifndef KN_DEFAULT_XSUB
#define KN_DEFAULT_XSUB 2
#endif
#ifndef KN_XSUB_MAX_K
#define KN_XSUB_MAX_K 16
#endif
// Re-rank of the kept keys: 1 = streaming window (O(kWin) live registers), 0 = odd-even
// transposition over (d2, id) arrays of KM entries each plus the in-wave exact re-scan of
// truncation near-ties (round 1).
#ifndef KN_WIN
#define KN_WIN 1
#endif
// Unrolled re-rank walk for the K buckets with KM <= 24 (key shifts and window rotations become
// register renames). Round 5 measured it at +-1 %; with the pairwise compare below it wins:
// in-process A/B, 900K uniform, identical rows (profiles/ab_r6_rerank.txt): K=16 query 0.2878 ->
// 0.2804 ms, K=8 0.2013 -> 0.1966; K=32 (KM = 35, rolled either way) unchanged.
#ifndef KN_RERANK_UNROLL
#define KN_RERANK_UNROLL 1
#endif
// Staging of the tile + halo rows (knn_tile_kernel steps 1 and 3): 1 = per-row (cell bounds by
// half-wave rows without integer division; points by one direct global -> LDS load per 64 points of
// a row), 0 = round 5 (boundaries with a division per entry, points with a binary search each)
#ifndef KN_STAGE_ROWS
#define KN_STAGE_ROWS 1
#endif
#if defined(KN_CHECKED) && KN_CHECKED
constexpr bool kChecked = true;
#else
constexpr bool kChecked = false;
#endif
typedef __attribute__((address_space(3))) void* lds_ptr_t;
// Lane walk: 1 = the query itself in its own top-K list (default), 0 = its own row scanned as two
// spans around it, no self slot (see knn_tile_kernel's KM). Measured: no gain -- the extra span
// pass costs what the med3 slot and the re-rank entry save (900K, in-process A/B, identical rows:
// K=16 0.2762 vs 0.2784 ms, K=50 0.845 vs 0.848, K=64 0.885 vs 0.888; profiles/ab_r6_self_slot.txt)
#ifndef KN_SELF_SLOT
#define KN_SELF_SLOT 1
#endif
// x halo of the tile path in x sub-cells (xsub > 1): 0 = halo * xsub (whole cells, the y / z halo
// width), T > 0 = min(T, halo * xsub). The lane walk's own box is the query's sub-cell +- this many
// sub-cells in x, and certification measures against that box, so a narrower x halo stays exact.
// Measured with its own plan (scripts/ab_plan.py, profiles/ab_r6_xhalo.txt): T = 3 (1.5 cells)
// shrinks the K <= 16 plan to 32.5 KB (5 workgroups per CU) but sends 72 / 27 queries of 900K /
// 300K to the exact path at K=16: 900K K=16 0.280 -> 0.306 ms, 300K 0.145 -> 0.177; only K=8 and 3M
// gain (-1 %, -5..-7 %). Off.
#ifndef KN_XHALO_SUB
#define KN_XHALO_SUB 0
#endif
inline int x_halo(int halo, int xsub) {
    const int full = halo * std::max(1, xsub);
    return (KN_XHALO_SUB > 0 && xsub > 1) ? std::min(KN_XHALO_SUB, full) : full;
}
// Checked builds, diagnostics: counters [4] / [5] count the lane walk's wave-uniform row
// iterations and lockstep candidate steps (0: per-lane rows / candidates summed over live lanes)
#ifndef KN_WALK_STATS
#define KN_WALK_STATS 0
#endif
// kWin = 1: compare each adjacent pair of kept keys once (see window_pass): 900K K=16 query
// 0.2914 -> 0.2880 ms, K=32 0.5273 -> 0.5209, K=8 0.2026 -> 0.1992 (profiles/ab_r6_rerank.txt)
#ifndef KN_RERANK_PAIR
#define KN_RERANK_PAIR 1
#endif
constexpr int kWin = KN_WIN;  // exact re-rank window: same-bucket neighbours within +-kWin
// Second, wider window for the lanes whose bucket runs overflow +-kWin but fit +-kWin2 (point
// sets with many exactly equal distances -- symmetric / lattice-like samplings: pts20K has runs
// of >= 3 equal buckets in 55 % of its K=8 queries, and sending them all to the wave-serial
// cooperative sort made its query kernel 5x slower). The lanes run one of the two passes each
// (divergent, but in parallel), only runs longer than kWin2 + 1 go cooperative. 0 = off.
#ifndef KN_WIN2
#define KN_WIN2 4
#endif
constexpr int kWin2 = KN_WIN2 > kWin ? KN_WIN2 : 0;
template <int V>
struct IntC {
    static constexpr int value = V;
};
// f(IntC<I>{}) ... f(IntC<N - 1>{}): a compile-time unrolled loop whose body sees a constant index
template <int I, int N, class F>
__device__ __forceinline__ void static_for(F& f) {
    if constexpr (I < N) {
        f(IntC<I>{});
        static_for<I + 1, N>(f);
    }
}
// entries per shift of the rolled re-rank walk (KM > 24; see window_pass): 4 against 1 measured
// K=50 -2 %, K=64 -3.6 % (profiles/ab_r6_rerank_group.txt); 8 a further -1 % at K=50, equal at K=32
// and K=64 (profiles/ab_r6_k50.txt)
// KN_DIAG_SKIP_OUT=1 (diagnostics only, wrong results): the re-rank writes no rows -- the cost
// of the scattered per-entry output stores
#ifndef KN_DIAG_SKIP_OUT
#define KN_DIAG_SKIP_OUT 0
#endif
#ifndef KN_RERANK_GROUP
#define KN_RERANK_GROUP 8
#endif
// Round-3 A/Bs of the lane walk that LOST against this kernel (900K uniform, interleaved in
// process, identical rows; profiles/ab_r3_lane_variants.jsonl, profiles/ab_r3_collect.jsonl):
//  * collect-then-select (d2-only scan + per-lane LDS queue of candidate slots, bulk med3
//    insertion): K=16 0.30 -> 0.49 ms. The ballot-gated insertion already skips ~45 % of the
//    candidate steps (98 networks per 64-query chunk for ~172 steps, checked-build counters),
//    so the queue saved less than its LDS traffic and the lost workgroup slot cost.
//  * fast re-rank (rows straight from the keys unless two adjacent keys share a truncation
//    bucket): 2 % of the lanes have such a pair, and the cooperative sort they fall back to
//    costs more than the window pass saves (K=16 +4 %, K=50 2.2x).
//  * software-pipelined lane gathers: +0-3 %. R-capped lane bound (Poisson-quantile ball at the
//    tile density): K=16 +6 %, K=50 +8 %.
//  * query groups (G = 2 or 4 adjacent lanes per query, slots interleaved, group-min bound, DPP
//    merge of the lists): never faster -- u20000 K=8 0.039 (G=1) / 0.039 / 0.044 ms, u100000
//    K=8 0.051 / 0.075 / 0.122, 900K K=16 0.29 / 0.46 / 0.79 (profiles/ab_r3_qgroup.jsonl).
//    Small clouds are bound by the per-workgroup fixed costs (cell bounds, prefix scans,
//    staging round trips), not by the per-lane candidate chain.

constexpr int kCoopCap = 128;  // per-wave LDS buffer of the cooperative re-scan (u64 keys)
constexpr int kQueryForceRescan = kQueryFlagForceRescan;
// fallback-list entry flag: the query's output row holds K real candidates (their K-th squared
// distance is an upper bound the exact kernel seeds its threshold with); stored indices < 2^31
constexpr unsigned kSeedBit = 0x80000000u;
constexpr int kQueryAlgoStream = kQueryFlagStream;
constexpr int kQueryAlgoTile = kQueryFlagTile;
constexpr int kQueryAlgoLane = kQueryFlagLane;
// lane walk with the second re-rank window (kQueryFlagWide; profiles/ab_r3_win2.jsonl: pts20K
// K=8 query 0.19 -> 0.07 ms with it, 900K uniform K=16 +3 %, 100K +15 % without need)
constexpr int kQueryWide = kQueryFlagWide;

// Shared device helpers (key packing, med3 top-K insertion, id modes, wave sort): kn/knn_device.h

// Per-phase wave-cycle census of knn_tile_kernel (diagnostic builds only, -DKN_PHASES=1; the
// s_memtime stamps cost ~10 % themselves): every wave accumulates the shader cycles it spends
// in each phase and lane 0 adds them to g_phase[] at the end. Read with debug_phase_cycles().
#ifndef KN_PHASES
#define KN_PHASES 0
#endif
enum { kPhStage = 0, kPhSetup, kPhScan, kPhRerank, kPhCertify, kPhChunks, kPhWaves, kPhN = 8 };
#if KN_PHASES
// One VGPR holds the 8 accumulators (lane p = phase p): no SGPR pressure in a kernel that is
// already near its SGPR budget (an SGPR-array version spilled and tripled the kernel time).
__device__ unsigned long long g_phase[kPhN];
#define KN_PH_DECL unsigned ph_acc = 0; unsigned long long ph_last = __builtin_amdgcn_s_memtime(); int ph_cur = kPhStage;
#define KN_PH_MARK(p)                                                                \
    do {                                                                             \
        const unsigned long long ph_now_ = __builtin_amdgcn_s_memtime();             \
        ph_acc += ((int)(threadIdx.x & 63) == ph_cur) ? (unsigned)(ph_now_ - ph_last) : 0u; \
        ph_last = ph_now_;                                                           \
        ph_cur = (p);                                                                \
    } while (0)
#define KN_PH_COUNT(p) (ph_acc += ((int)(threadIdx.x & 63) == (p)) ? 1u : 0u)
#define KN_PH_FLUSH()                                                                     \
    do {                                                                                  \
        const int l_ = threadIdx.x & 63;                                                  \
        if (l_ == kPhWaves) ph_acc += 1u;                                                 \
        if (l_ < kPhN) atomicAdd(&g_phase[l_], (unsigned long long)ph_acc);             \
    } while (0)
#else
#define KN_PH_DECL
#define KN_PH_MARK(p) ((void)0)
#define KN_PH_COUNT(p) ((void)0)
#define KN_PH_FLUSH() ((void)0)
#endif

// Tile of a workgroup. xcd_remap gives each XCD a contiguous run of tile numbers; with B > 1 the
// numbers run through B x B x B blocks of tiles (x-fastest blocks, x-fastest inside a block; edge
// blocks are partial), so the ~128 workgroups an XCD holds at once form compact 3-D groups whose
// halos overlap in that XCD's L2 -- x-fastest order makes them a 1-2 tile-row slab, whose z halos
// are fetched again by the next slab (10M K=32: FETCH_SIZE 1.43x the sorted array, SQ_WAIT_ANY
// 59 % of wave cycles vs 34 % at 900K; profiles/pmc_r5_10m_k32.txt). A bijection of [0, ntiles).
__device__ __forceinline__ void tile_coords(int lin, int ntx, int nty, int ntz, int B, int& tx, int& ty, int& tz) {
    if (B <= 1) {
        tx = lin % ntx;
        ty = (lin / ntx) % nty;
        tz = lin / (ntx * nty);
        return;
    }
    const int slab = B * nty * ntx;             // tiles of a full z-slab of blocks
    const int bz = min(lin / slab, (ntz - 1) / B);
    int r = lin - bz * slab;
    const int hz = min(B, ntz - bz * B);        // this slab's height
    const int row = B * ntx * hz;               // tiles of a full y-row of blocks in the slab
    const int by = min(r / row, (nty - 1) / B);
    r -= by * row;
    const int hy = min(B, nty - by * B);
    const int blk = B * hy * hz;                // tiles of a full block in the row
    const int bx = min(r / blk, (ntx - 1) / B);
    r -= bx * blk;
    const int hx = min(B, ntx - bx * B);
    tx = bx * B + r % hx;
    ty = by * B + (r / hx) % hy;
    tz = bz * B + r / (hx * hy);
}

// LANE = false: wave-uniform candidate stream over the union of the chunk's needs (LDS
// broadcast reads). LANE = true ("lane walk"): each lane walks ITS OWN rows of the staged
// block -- centre-out over the (2H+1)^2 row offsets around its cell, x-range cut by its own
// bound -- as a divergent loop with per-lane LDS gathers. ~90 candidates per query instead of
// the ~535 the union stream feeds every lane, at the price of divergent trip counts.
// Waves per SIMD requested for the K > 50 buckets (a VGPR cap: 145 -> 128 VGPRs, 13 spilled): the
// LDS plan allows 4 workgroups per CU, the registers 3 without the cap. 900K K=64 0.909 -> 0.848
// ms/step (profiles/ab_r5_tree_waves.txt). KN_TILE_WPE64=1: no cap.
#ifndef KN_TILE_WPE64
#define KN_TILE_WPE64 4
#endif
template <int KT>
constexpr int tile_wpe() { return KT > 50 ? KN_TILE_WPE64 : 1; }
// Gated-tier top-K networks (kn/knn_device.h topk_tiers) per K bucket: in-process A/B at 900K
// uniform, identical rows (profiles/ab_r6_tiers.txt): K=50 bucket 3 tiers 0.904 -> 0.877 ms
// (2 tiers -1.6 %), K=64 bucket 4 tiers 1.009 -> 0.912 (3 tiers -8 %); at K <= 32 every tier count
// lost (K=16 +0.2 / +2 / +6.5 %, K=32 +2.4 ... +12 %, K=8 +1.6 ... +5 %): their lists are short and
// a slice's compare + branch costs more than the med3s it skips. KN_TILE_TIERS=T forces T.
#ifndef KN_TILE_TIERS
#define KN_TILE_TIERS 0
#endif
template <int KT>
constexpr int tile_tiers() { return KN_TILE_TIERS > 0 ? KN_TILE_TIERS : KT > 50 ? 4 : KT > 40 ? 3 : 1; }
template <int KT, int M, bool LANE, bool WIDE = false>
__global__ __launch_bounds__(kWG) __attribute__((amdgpu_waves_per_eu(tile_wpe<KT>(), 8))) void knn_tile_kernel(TileArgs a) {
    // output pointers: the launch's, or read from device slots (graph replays of a batched
    // stream of clouds); locals, so the kernel argument block stays read-only
    out_u32_t* const o_idx = out_ptr(a.out_idx_ref ? *a.out_idx_ref : a.out_idx);
    out_f32_t* const o_dist = out_ptr(a.out_idx_ref ? (a.out_dist_ref ? *a.out_dist_ref : nullptr) : a.out_dist);
    // K + M margin slots (+ 1 for the query itself on the union stream, where it enters its own
    // list at d2 = 0 and is dropped at the re-rank). The lane walk scans the query's own row as two
    // spans around the query's slot instead (KN_SELF_SLOT=0), so its list has no self slot: one
    // med3 less per network and one re-rank entry less, for one extra span per walk.
    constexpr bool kSelfSlot = !LANE || KN_SELF_SLOT;
    constexpr int KM = KT + M + (kSelfSlot ? 1 : 0);
    constexpr bool kFull = LANE && (KN_LANE_FULL == 2 || (KN_LANE_FULL == 1 && KT > 40));
    // (KN_OUTER_PACK=3: the whole-block walk packs its outer rows instead of the sorted table)
    constexpr bool kRowOrder = LANE && (KN_ROW_ORDER == 1 || (KN_ROW_ORDER == 2 && kFull && !outer_pack_k<KT>()));
    // row-cut square roots: the bare v_sqrt_f32 (kn/wave.h sqrt_bound) for the walks of K <= 40
    // (900K, interleaved A/B: K=16 query -2.5 %, K=32 -3 %); the whole-block walk (K > 40) keeps
    // the correctly rounded sqrtf, which measured 11 % FASTER there (K=50 0.949 -> 0.838 ms) with
    // identical rows and near-identical code (profiles/ab_r5_query_variants.txt)
    auto rsqrt = [](float x) __attribute__((always_inline)) { return kFull ? sqrtf(x) : sqrt_bound(x); };
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    KN_PH_DECL
    float4* pts = reinterpret_cast<float4*>(smem);
    // cell boundaries of the staged rows, RELATIVE to the row's first point (u16: half the LDS of
    // int offsets, which buys the x sub-cells); rows of >= 65536 points only occur in tiles far
    // beyond the LDS capacity (the dense path below reads cell_start directly)
    unsigned short* cbr = reinterpret_cast<unsigned short*>(smem + (size_t)a.cap * sizeof(float4));
    int* rowbase = reinterpret_cast<int*>(smem + (size_t)a.cap * sizeof(float4) +
                                          (((size_t)a.max_rows * a.cb_stride * 2 + 3) & ~(size_t)3));
    int* rowst = rowbase + a.max_rows + 1;  // global sorted index of each row's first point
    int* rowend = rowst + a.max_rows;       // ... and one past its last
    int* qpref = rowend + a.max_rows;       // TY*TZ + 1 entries
    int* misc = qpref + a.TY * a.TZ + 1;

    const GridGeom g = *a.geom;
    const int ntiles = a.ntx * a.nty * a.ntz;
    int tx, ty, tz;
    tile_coords(xcd_remap(blockIdx.x, ntiles), a.ntx, a.nty, a.ntz, a.tblock, tx, ty, tz);
    const int tx0 = tx * a.TX, ty0 = ty * a.TY, tz0 = tz * a.TZ;
    const int tx1 = min(a.X, tx0 + a.TX), ty1 = min(a.Y, ty0 + a.TY), tz1 = min(a.Z, tz0 + a.TZ);
    // Staged block: the tile + H rings, clipped to the grid. With the whole-block lane walk
    // (kFull, K > 40) a block that would be clipped at a domain face is SHIFTED inward instead:
    // the same number of cells (so the same LDS plan), but the tile's boundary queries -- whose
    // K-th ball is a half/quarter/eighth ball up to 2x the interior radius -- reach T + 2H - 1
    // cells inward instead of H and certify on the tile path instead of the exact kernel.
    int sx0, sx1, sy0, sy1, sz0, sz1;
    if constexpr (kFull) {
        const int wx = a.TX + 2 * a.Hx, wy = a.TY + 2 * a.H, wz = a.TZ + 2 * a.H;
        sx0 = max(0, min(tx0 - a.Hx, a.X - wx)); sx1 = min(a.X, sx0 + wx);
        sy0 = max(0, min(ty0 - a.H, a.Y - wy)); sy1 = min(a.Y, sy0 + wy);
        sz0 = max(0, min(tz0 - a.H, a.Z - wz)); sz1 = min(a.Z, sz0 + wz);
    } else {
        sx0 = max(0, tx0 - a.Hx); sx1 = min(a.X, tx1 + a.Hx);
        sy0 = max(0, ty0 - a.H); sy1 = min(a.Y, ty1 + a.H);
        sz0 = max(0, tz0 - a.H); sz1 = min(a.Z, tz1 + a.H);
    }
    const int nxs = sx1 - sx0, nys = sy1 - sy0, nzs = sz1 - sz0;
    const int nrows = nys * nzs;
    const int cbs = nxs + 1;
    const int ntry = ty1 - ty0, ntrz = tz1 - tz0, ntr = ntry * ntrz;
    const int hx = tx0 - sx0;
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;

    // ---- 1. cell boundaries of every staged row ----------------------------------------
    auto row_cell = [&](int r) { return ((sz0 + r / nys) * a.Y + sy0 + r % nys) * a.X + sx0; };
    if constexpr (KN_STAGE_ROWS) {
        // one row per half-wave (cbs <= 32) or per wave: no integer division per boundary, the row's
        // first boundary broadcast from its first lane instead of loaded again by every lane
        const int seg = cbs <= 32 ? 32 : 64;
        const int rpw = 64 / seg;  // rows per wave iteration
        const int sl = lane & (seg - 1), sbase = lane & ~(seg - 1);
        for (int r0 = wid * rpw; r0 < nrows; r0 += kWaves * rpw) {
            const int r = r0 + (lane >> (seg == 32 ? 5 : 6));
            const int c0 = r < nrows ? row_cell(r) : 0;
            int v0 = 0;
            for (int i0 = 0; i0 < cbs; i0 += seg) {
                const int i = i0 + sl;
                const int v = (r < nrows && i < cbs) ? a.cell_start[KN_IDX(c0 + i, a.X * a.Y * a.Z + 1, 201)] : 0;
                if (i0 == 0) v0 = __shfl(v, sbase, 64);  // the row's first boundary (uniform loop)
                if (r < nrows && i < cbs) {
                    cbr[r * cbs + i] = (unsigned short)(v - v0);
                    if (i == 0) rowst[r] = v;
                    if (i == nxs) rowend[r] = v;
                }
            }
        }
    } else {
    for (int t = threadIdx.x; t < nrows * cbs; t += kWG) {
        const int r = t / cbs, i = t - r * cbs;
        const int c0 = row_cell(r);
        const int v = a.cell_start[KN_IDX(c0 + i, a.X * a.Y * a.Z + 1, 201)];
        const int v0 = a.cell_start[KN_IDX(c0, a.X * a.Y * a.Z + 1, 201)];
        cbr[r * cbs + i] = (unsigned short)(v - v0);
        if (i == 0) rowst[r] = v;
        if (i == nxs) rowend[r] = v;
    }
    }
    __syncthreads();
    // ---- 2. row prefix (LDS offsets) and tile-row query prefix (wave 0) ----------------
    if (wid == 0) {
        int carry = 0;
        bool big = false;  // a row too long for u16 offsets: the tile takes the dense path
        for (int base = 0; base < nrows; base += 64) {
            const int r = base + lane;
            const int len = (r < nrows) ? rowend[r] - rowst[r] : 0;
            big = big || __builtin_amdgcn_ballot_w64(len > 65535) != 0;
            const int incl = wave_inclusive_scan_add(len);
            if (r < nrows) rowbase[r] = carry + incl - len;
            carry += __shfl(incl, 63, 64);
        }
        if (lane == 0) rowbase[nrows] = carry;
        int qc = 0;
        for (int base = 0; base < ntr; base += 64) {
            const int t = base + lane;
            int len = 0;
            if (t < ntr) {
                const int r = (ty0 - sy0 + t % ntry) + nys * (tz0 - sz0 + t / ntry);
                len = big ? a.cell_start[row_cell(r) + hx + (tx1 - tx0)] - a.cell_start[row_cell(r) + hx]
                          : (int)cbr[r * cbs + hx + (tx1 - tx0)] - (int)cbr[r * cbs + hx];
            }
            const int incl = wave_inclusive_scan_add(len);
            if (t < ntr) qpref[t] = qc + incl - len;
            qc += __shfl(incl, 63, 64);
        }
        if (lane == 0) qpref[ntr] = qc;
    }
    __syncthreads();
    const int S = rowbase[nrows];
    const int Q = qpref[ntr];
    if (Q == 0) return;
    if (S > a.cap) {
        // Tile too dense for the LDS budget: every query of the tile takes the exact path.
        for (int t = threadIdx.x; t < Q; t += kWG) {
            int lo = 0, hi = ntr - 1;
            while (lo < hi) { const int mid = (lo + hi + 1) >> 1; if (qpref[mid] <= t) lo = mid; else hi = mid - 1; }
            const int r = (ty0 - sy0 + lo % ntry) + nys * (tz0 - sz0 + lo / ntry);
            const unsigned sidx = (unsigned)(a.cell_start[row_cell(r) + hx] + (t - qpref[lo]));
            const unsigned orig = __float_as_uint(a.sorted[KN_IDX(sidx, (unsigned)a.n, 204)].w);
            if (w_live(a, orig)) {
                const unsigned pos = atomicAdd(a.counters + 0, 1u);
                a.fallback_list[KN_IDX(pos, (unsigned)a.n, 205)] = sidx;
            }
        }
        if (threadIdx.x == 0) atomicAdd(a.counters + 2, 1u);
        return;
    }
    // ---- 3. stage the points ------------------------------------------------------------
    if constexpr (KN_STAGE_ROWS && !kChecked) {
        // one row per wave iteration: its points are one contiguous run of the sorted array and
        // land in one contiguous LDS range, so a wave copies 64 of them with ONE direct
        // global -> LDS load (global_load_lds_dwordx4: per-lane source, LDS base in M0 + lane * 16;
        // lanes past the row end are masked off). No per-point binary search, no VGPR round trip.
        // The barrier below waits for the loads (vmcnt) before any wave reads the points.
        for (int r = wid; r < nrows; r += kWaves) {
            const int st = __builtin_amdgcn_readfirstlane(rowst[r]);
            const int len = __builtin_amdgcn_readfirstlane(rowend[r]) - st;
            const int dst = __builtin_amdgcn_readfirstlane(rowbase[r]);
            for (int c = 0; c < len; c += 64) {
                if (c + lane < len)
                    __builtin_amdgcn_global_load_lds(a.sorted + st + c + lane, (lds_ptr_t)(pts + dst + c), 16, 0, 0);
            }
        }
    } else if constexpr (KN_STAGE_ROWS) {
        // checked builds: the same per-row copy through registers, every index bounds-checked
        for (int r = wid; r < nrows; r += kWaves) {
            const int st = rowst[r], len = rowend[r] - st, dst = rowbase[r];
            for (int c = lane; c < len; c += 64) pts[KN_IDX(dst + c, a.cap, 203)] = a.sorted[KN_IDX(st + c, a.n, 202)];
        }
    } else {
    // (round 5: 16-B coalesced loads, each point's row found by binary search over rowbase)
    for (int s = threadIdx.x; s < S; s += kWG) {
        int lo = 0, hi = nrows - 1;
        while (lo < hi) { const int mid = (lo + hi + 1) >> 1; if (rowbase[mid] <= s) lo = mid; else hi = mid - 1; }
        pts[KN_IDX(s, a.cap, 203)] = a.sorted[KN_IDX(rowst[lo] + (s - rowbase[lo]), a.n, 202)];
    }
    }
    __syncthreads();
    (void)misc;

    const unsigned MASK = (1u << a.slot_bits) - 1u;
    const unsigned HIMASK = ~MASK;

    // ---- 4. query chunks: 64 queries per wave ------------------------------------------
    // Lanes past the tile's last query duplicate that query (identical candidate tests, so
    // they never add work to the uniform stream); only lanes < Q are written back.
    for (int chunk = wid; chunk * 64 < Q; chunk += kWaves) {
        KN_PH_MARK(kPhSetup);
        KN_PH_COUNT(kPhChunks);
        const int qi_raw = chunk * 64 + lane;
        const bool in_range = qi_raw < Q;
        const int qi = in_range ? qi_raw : Q - 1;
        int lo = 0, hi = ntr - 1;
        while (lo < hi) { const int mid = (lo + hi + 1) >> 1; if (qpref[mid] <= qi) lo = mid; else hi = mid - 1; }
        const int qrow = (ty0 - sy0 + lo % ntry) + nys * (tz0 - sz0 + lo / ntry);
        const int qoff = (int)cbr[qrow * cbs + hx] + (qi - qpref[lo]);
        const int qslot = rowbase[qrow] + qoff;
        const unsigned qsidx = (unsigned)(rowst[qrow] + qoff);
        const float4 qp = pts[KN_IDX(qslot, S, 206)];
        const unsigned qorig = __float_as_uint(qp.w);
        const bool live = w_live(a, qorig);  // halo points of a multi-GPU rank are not queries
        const float qx = qp.x, qy = qp.y, qz = qp.z;
        const int cx = cell_coord(g, 0, qx) - sx0;
        const int cy = cell_coord(g, 1, qy) - sy0;
        const int cz = cell_coord(g, 2, qz) - sz0;
        // scanned region: the wave's bounding box of the live queries' cells + H (union
        // stream), or each lane's own cell + H (lane walk)
        int rx0, rx1, ry0, ry1, rz0, rz1, zc = 0, yc = 0, nzt = 0, nyt = 0;
        // lane walk: the lane's own cell +- H (phase 1 of the walk)
        int hx0 = 0, hx1 = -1, hy0 = 0, hy1 = -1, hz0 = 0, hz1 = -1;
        if constexpr (LANE) {
            if (!__builtin_amdgcn_ballot_w64(live)) continue;  // no live query in this chunk
            hx0 = max(0, cx - a.Hx); hx1 = min(nxs - 1, cx + a.Hx);
            hy0 = max(0, cy - a.H); hy1 = min(nys - 1, cy + a.H);
            hz0 = max(0, cz - a.H); hz1 = min(nzs - 1, cz + a.H);
            if constexpr (kFull) {
                rx0 = 0; rx1 = nxs - 1;
                ry0 = 0; ry1 = nys - 1;
                rz0 = 0; rz1 = nzs - 1;
            } else {
                rx0 = hx0; rx1 = hx1; ry0 = hy0; ry1 = hy1; rz0 = hz0; rz1 = hz1;
            }
        } else {
            // 3 packed (-min, max) reductions
            const int2 bx = wave_minmax_i32(live ? cx : INT_MAX, live ? cx : INT_MIN);
            if (bx.x > bx.y) continue;  // no live query in this chunk (uniform)
            const int2 by = wave_minmax_i32(live ? cy : INT_MAX, live ? cy : INT_MIN);
            const int2 bz = wave_minmax_i32(live ? cz : INT_MAX, live ? cz : INT_MIN);
            rx0 = max(0, bx.x - a.Hx); rx1 = min(nxs - 1, bx.y + a.Hx);
            ry0 = max(0, by.x - a.H); ry1 = min(nys - 1, by.y + a.H);
            rz0 = max(0, bz.x - a.H); rz1 = min(nzs - 1, bz.y + a.H);
            zc = (bz.x + bz.y) >> 1; yc = (by.x + by.y) >> 1;
            nzt = 2 * max(zc - rz0, rz1 - zc) + 1;
            nyt = 2 * max(yc - ry0, ry1 - yc) + 1;
        }

        // Visit the region's rows centre-out; for each row every live lane derives the x-range of
        // cells its current bound `tau` still needs (|x - qx|^2 <= tau - dyz^2). Union stream: the
        // wave takes the union, and `body(s0, s1)` streams the uniform LDS slot range [s0, s1).
        // Lane walk: the row offset is uniform, the row itself and [s0, s1) are per lane.
        auto scan_region = [&](auto&& lane_tau, auto&& body2) {
          if constexpr (LANE) {
            const int side = 2 * a.H + 1;
            // LDS slot range [s0, s1) of cells [x0, x1] of staged row (y, z); empty if x0 > x1
            // (row index r and r * cbs given: the row-synchronous inner loop derives both from the
            // lane's own row plus a uniform offset, without a per-row integer multiply)
            auto lane_span_r = [&](int r, int rcb, int x0, int x1) {
                int2 sp = make_int2(0, 0);
                if (x0 <= x1) {
                    const int rb = rowbase[r];
                    sp.x = rb + (int)cbr[rcb + x0];
                    sp.y = KN_IDX(rb + (int)cbr[rcb + x1 + 1], S + 1, 212);
                }
                return sp;
            };
            auto lane_span = [&](int y, int z, int x0, int x1) {
                const int r = y + nys * z;
                return lane_span_r(r, r * cbs, x0, x1);
            };
            const int qr0 = cy + nys * cz, qr0cb = qr0 * cbs;  // the lane's own row
            // own (uniform): the query's own row (offset (0, 0)). Without a self slot it is scanned as
            // the two spans around the query's own slot (either may be empty), through the SAME call
            // site in a uniform loop of two passes: a second inlined copy of the scan loop raised the
            // register allocation of the large-K buckets (K=50 119 -> 177 VGPRs, K=64 spills)
            auto body = [&](int2 sp, bool own = false) {
                int e = sp.y;
                if (!kSelfSlot && own) e = min(sp.y, qslot);
                const int passes = (!kSelfSlot && own) ? 2 : 1;
#pragma unroll 1
                for (int pass = 0; pass < passes; ++pass) {
                    body2(sp.x, e);
                    sp.x = max(sp.x, qslot + 1);
                    e = sp.y;
                }
            };
            if constexpr (kRowOrder) {
            const int nent = side * side;
            // mirror the table so that offset +1 is the near neighbour row of the query's cell
            const float fy = (qy - g.origin[1]) * g.inv_cell[1] - (float)(sy0 + cy);
            const float fz = (qz - g.origin[2]) * g.inv_cell[2] - (float)(sz0 + cz);
            const int sgy = (a.row_mirror && fy < 0.5f) ? -1 : 1, sgz = (a.row_mirror && fz < 0.5f) ? -1 : 1;
            for (int t = 0; t < nent; ++t) {
                int oy, oz;
                if (nent <= kRowOrderMax) {
                    const unsigned e = (a.row_order[t >> 2] >> ((t & 3) * 8)) & 255u;
                    oy = (int)(e & 15u) - 8;
                    oz = (int)(e >> 4) - 8;
                } else {
                    const int iz = t / side, iy = t - iz * side;
                    oz = (iz & 1) ? ((iz + 1) >> 1) : -(iz >> 1);
                    oy = (iy & 1) ? ((iy + 1) >> 1) : -(iy >> 1);
                }
                const int z = cz + sgz * oz, y = cy + sgy * oy;
                const float dzb = slab_dist(g, 2, qz, sz0 + z, sz0 + z);
                const float dyb = slab_dist(g, 1, qy, sy0 + y, sy0 + y);
                const float dyz2 = fmaf(dyb, dyb, dzb * dzb);
                const float tau = lane_tau();
                int lx0 = 0, lx1 = -1;
                if (live && z >= hz0 && z <= hz1 && y >= hy0 && y <= hy1 && dyz2 <= tau) {
                    if (tau == INFINITY) {
                        lx0 = hx0; lx1 = hx1;
                    } else {
                        const float rr = rsqrt(tau - dyz2) * 1.000001f + g.eps;
                        lx0 = max(hx0, cell_coord(g, 0, qx - rr) - sx0);
                        lx1 = min(hx1, cell_coord(g, 0, qx + rr) - sx0);
                    }
                }
                if (!__builtin_amdgcn_ballot_w64(lx0 <= lx1)) continue;
                body(lane_span(y, z, lx0, lx1), oy == 0 && oz == 0);
            }
            } else {
            const bool pack = outer_pack_k<KT>() && a.n_outer > 0;
            const int sidein = pack ? 3 : side;  // rows visited row-synchronously
            for (int tz_ = 0; tz_ < sidein; ++tz_) {
                const int oz = (tz_ & 1) ? ((tz_ + 1) >> 1) : -(tz_ >> 1);
                const int z = cz + oz;
                const float dzb = slab_dist(g, 2, qz, sz0 + z, sz0 + z);
                const float dz2 = dzb * dzb;
                const bool zin = live && z >= hz0 && z <= hz1;
                if (!__builtin_amdgcn_ballot_w64(zin && dz2 <= lane_tau())) continue;
                for (int ty_ = 0; ty_ < sidein; ++ty_) {
                    const int oy = (ty_ & 1) ? ((ty_ + 1) >> 1) : -(ty_ >> 1);
                    const int y = cy + oy;
                    const float dyb = slab_dist(g, 1, qy, sy0 + y, sy0 + y);
                    const float dyz2 = fmaf(dyb, dyb, dz2);
                    const float tau = lane_tau();
                    int lx0 = 0, lx1 = -1;
                    if (zin && y >= hy0 && y <= hy1 && dyz2 <= tau) {
                        if (tau == INFINITY) {
                            lx0 = hx0; lx1 = hx1;
                        } else {
                            const float rr = rsqrt(tau - dyz2) * 1.000001f + g.eps;
                            lx0 = max(hx0, cell_coord(g, 0, qx - rr) - sx0);
                            lx1 = min(hx1, cell_coord(g, 0, qx + rr) - sx0);
                        }
                    }
                    if (!__builtin_amdgcn_ballot_w64(lx0 <= lx1)) continue;
                    const int ro = oy + nys * oz;  // uniform
                    body(lane_span_r(qr0 + ro, qr0cb + ro * cbs, lx0, lx1), ro == 0);
                }
            }
            if (outer_pack_k<KT>() && pack) {
                // per-lane slab gaps of offsets +-1, +-2 on y and z (the table holds ring >= 2 rows
                // with |offset| <= H; offsets beyond +-2 use the exact slab distance)
                const float fy = (qy - g.origin[1]) * g.inv_cell[1] - (float)(sy0 + cy);
                const float fz = (qz - g.origin[2]) * g.inv_cell[2] - (float)(sz0 + cz);
                const int sgy = fy < 0.5f ? -1 : 1, sgz = fz < 0.5f ? -1 : 1;
                auto gap = [&](int axis, int o) {
                    const int c = axis == 1 ? cy + sgy * o : cz + sgz * o;
                    const int s0c = axis == 1 ? sy0 : sz0;
                    const float qv = axis == 1 ? qy : qz;
                    const int lo = axis == 1 ? hy0 : hz0, hi = axis == 1 ? hy1 : hz1;
                    return (c >= lo && c <= hi) ? slab_dist(g, axis, qv, s0c + c, s0c + c) : INFINITY;
                };
                const float y1p = gap(1, 1), y1m = gap(1, -1), y2p = gap(1, 2), y2m = gap(1, -2);
                const float z1p = gap(2, 1), z1m = gap(2, -1), z2p = gap(2, 2), z2m = gap(2, -2);
                const float y0 = gap(1, 0), z0 = gap(2, 0);
                auto sel = [](int o, float m2, float m1, float c0, float p1, float p2, float far) {
                    return o == 0 ? c0 : o == 1 ? p1 : o == -1 ? m1 : o == 2 ? p2 : o == -2 ? m2 : far;
                };
                const float tau0 = lane_tau();
                unsigned long long mask = 0;
                for (int t = 0; t < a.n_outer; ++t) {
                    const unsigned e = (a.row_order[t >> 2] >> ((t & 3) * 8)) & 255u;  // uniform
                    const int oy = (int)(e & 15u) - 8, oz = (int)(e >> 4) - 8;
                    const float gy = sel(oy, y2m, y1m, y0, y1p, y2p, gap(1, oy));
                    const float gz = sel(oz, z2m, z1m, z0, z1p, z2p, gap(2, oz));
                    // out-of-box rows have an infinite gap: excluded explicitly (a lane whose bound is
                    // still infinite would otherwise take them, INF <= INF)
                    const bool in = gy < INFINITY && gz < INFINITY;
                    mask |= (live && in && fmaf(gy, gy, gz * gz) <= tau0) ? (1ull << t) : 0ull;
                }
                while (__builtin_amdgcn_ballot_w64(mask != 0ull)) {
                    int y = cy, z = cz, lx0 = 0, lx1 = -1;
                    if (mask) {
                        const int t = __builtin_ctzll(mask);
                        mask &= mask - 1;
                        const unsigned e = (a.row_order[t >> 2] >> ((t & 3) * 8)) & 255u;
                        y = cy + sgy * ((int)(e & 15u) - 8);
                        z = cz + sgz * ((int)(e >> 4) - 8);
                        const float dyb = slab_dist(g, 1, qy, sy0 + y, sy0 + y);
                        const float dzb = slab_dist(g, 2, qz, sz0 + z, sz0 + z);
                        const float dyz2 = fmaf(dyb, dyb, dzb * dzb);
                        const float tau = lane_tau();
                        if (dyz2 <= tau) {
                            const float rr = rsqrt(tau - dyz2) * 1.000001f + g.eps;
                            lx0 = max(hx0, cell_coord(g, 0, qx - rr) - sx0);
                            lx1 = min(hx1, cell_coord(g, 0, qx + rr) - sx0);
                        }
                    }
                    if (!__builtin_amdgcn_ballot_w64(lx0 <= lx1)) continue;
                    body(lane_span(y, z, lx0, lx1));
                }
            }
            }
            if constexpr (kFull) {
            // Phase 2: the rest of the staged block, only for lanes whose bound still reaches
            // a cell outside their own +-H box (the slabs just outside it are the nearest such
            // cells on each axis). Centre-out per axis; a magnitude no lane reaches on either
            // side ends the axis loop (slab distance grows with it, the bound only shrinks).
            // Rows of the phase-1 band skip the x-interval phase 1 already scanned.
            bool more = false;
            {
                const float t = lane_tau();
                auto out = [&](int axis, float q, int c, int s0c) {
                    const float d = slab_dist(g, axis, q, s0c + c, s0c + c);
                    return d * d <= t;
                };
                more = (hx0 > rx0 && out(0, qx, hx0 - 1, sx0)) || (hx1 < rx1 && out(0, qx, hx1 + 1, sx0)) ||
                       (hy0 > ry0 && out(1, qy, hy0 - 1, sy0)) || (hy1 < ry1 && out(1, qy, hy1 + 1, sy0)) ||
                       (hz0 > rz0 && out(2, qz, hz0 - 1, sz0)) || (hz1 < rz1 && out(2, qz, hz1 + 1, sz0));
                more = more && live;
            }
            if (__builtin_amdgcn_ballot_w64(more)) {
                for (int tz_ = 0; tz_ < 2 * nzs; ++tz_) {
                    const int mz = (tz_ + 1) >> 1;
                    const int z = cz + ((tz_ & 1) ? mz : -mz);
                    if (tz_ & 1) {
                        const float t = lane_tau();
                        bool reach = false;
                        if (more) {
                            if (cz + mz <= rz1) { const float d = slab_dist(g, 2, qz, sz0 + cz + mz, sz0 + cz + mz); reach |= d * d <= t; }
                            if (cz - mz >= rz0) { const float d = slab_dist(g, 2, qz, sz0 + cz - mz, sz0 + cz - mz); reach |= d * d <= t; }
                        }
                        if (!__builtin_amdgcn_ballot_w64(reach)) break;
                    }
                    const float dzb = slab_dist(g, 2, qz, sz0 + z, sz0 + z);
                    const float dz2 = dzb * dzb;
                    const bool zin = more && z >= rz0 && z <= rz1;
                    if (!__builtin_amdgcn_ballot_w64(zin && dz2 <= lane_tau())) continue;
                    const bool zband = z >= hz0 && z <= hz1;
                    for (int ty_ = 0; ty_ < 2 * nys; ++ty_) {
                        const int my = (ty_ + 1) >> 1;
                        const int y = cy + ((ty_ & 1) ? my : -my);
                        if (ty_ & 1) {
                            const float t = lane_tau();
                            bool reach = false;
                            if (zin) {
                                if (cy + my <= ry1) { const float d = slab_dist(g, 1, qy, sy0 + cy + my, sy0 + cy + my); reach |= fmaf(d, d, dz2) <= t; }
                                if (cy - my >= ry0) { const float d = slab_dist(g, 1, qy, sy0 + cy - my, sy0 + cy - my); reach |= fmaf(d, d, dz2) <= t; }
                            }
                            if (!__builtin_amdgcn_ballot_w64(reach)) break;
                        }
                        const float dyb = slab_dist(g, 1, qy, sy0 + y, sy0 + y);
                        const float dyz2 = fmaf(dyb, dyb, dz2);
                        const float tau = lane_tau();
                        int lx0 = 0, lx1 = -1;
                        if (zin && y >= ry0 && y <= ry1 && dyz2 <= tau) {
                            if (tau == INFINITY) {
                                lx0 = rx0; lx1 = rx1;
                            } else {
                                const float rr = rsqrt(tau - dyz2) * 1.000001f + g.eps;
                                lx0 = max(rx0, cell_coord(g, 0, qx - rr) - sx0);
                                lx1 = min(rx1, cell_coord(g, 0, qx + rr) - sx0);
                            }
                        }
                        if (!__builtin_amdgcn_ballot_w64(lx0 <= lx1)) continue;
                        int bx0 = 0, bx1 = -1;  // right part of a phase-1 band row
                        if (zband && y >= hy0 && y <= hy1) {
                            bx0 = max(lx0, hx1 + 1); bx1 = lx1;
                            lx1 = min(lx1, hx0 - 1);
                        }
                        body(lane_span(y, z, lx0, lx1));
                        if (__builtin_amdgcn_ballot_w64(bx0 <= bx1)) body(lane_span(y, z, bx0, bx1));
                    }
                }
            }
            }
          } else {
            for (int tz_ = 0; tz_ < nzt; ++tz_) {
                const int z = zc + ((tz_ & 1) ? ((tz_ + 1) >> 1) : -(tz_ >> 1));
                if (z < rz0 || z > rz1) continue;
                const float dzb = slab_dist(g, 2, qz, sz0 + z, sz0 + z);
                const float dz2 = dzb * dzb;
                // rows of this slab any live lane can still need (bound at slab start: superset)
                int yl0 = ry0, yl1 = ry1;
                {
                    const float tz = lane_tau();
                    int ly0 = INT_MAX, ly1 = INT_MIN;
                    if (tz == INFINITY) {
                        ly0 = ry0; ly1 = ry1;
                    } else if (dz2 <= tz) {
                        const float rr = rsqrt(tz - dz2) * 1.000001f + g.eps;
                        ly0 = max(ry0, cell_coord(g, 1, qy - rr) - sy0);
                        ly1 = min(ry1, cell_coord(g, 1, qy + rr) - sy0);
                    }
                    if (!live) { ly0 = INT_MAX; ly1 = INT_MIN; }
                    const int2 Yr = wave_minmax_i32(ly0, ly1);
                    if (Yr.x > Yr.y) continue;
                    yl0 = Yr.x; yl1 = Yr.y;
                }
                for (int ty_ = 0; ty_ < nyt; ++ty_) {
                    const int y = yc + ((ty_ & 1) ? ((ty_ + 1) >> 1) : -(ty_ >> 1));
                    if (y < yl0 || y > yl1) continue;
                    const float dyb = slab_dist(g, 1, qy, sy0 + y, sy0 + y);
                    const float dyz2 = fmaf(dyb, dyb, dz2);
                    const float tau = lane_tau();
                    int lx0 = INT_MAX, lx1 = INT_MIN;
                    if (tau == INFINITY) {
                        lx0 = rx0; lx1 = rx1;
                    } else if (dyz2 <= tau) {
                        const float rr = rsqrt(tau - dyz2) * 1.000001f + g.eps;
                        lx0 = max(rx0, cell_coord(g, 0, qx - rr) - sx0);
                        lx1 = min(rx1, cell_coord(g, 0, qx + rr) - sx0);
                    }
                    if (!live) { lx0 = INT_MAX; lx1 = INT_MIN; }
                    const int2 X = wave_minmax_i32(lx0, lx1);
                    if (X.x > X.y) continue;
                    const int r = y + nys * z;
                    const int rb = rowbase[r];
                    // uniform bounds -> scalar loop control
                    const int s0 = __builtin_amdgcn_readfirstlane(rb + (int)cbr[r * cbs + X.x]);
                    const int s1 = __builtin_amdgcn_readfirstlane(KN_IDX(rb + (int)cbr[r * cbs + X.y + 1], S + 1, 207));
                    body2(s0, s1);
                }
            }
          }
        };

        unsigned keys[KM];
#pragma unroll
        for (int j = 0; j < KM; ++j) keys[j] = SENT;
        // uniform per-chunk work statistics: diagnostics builds only (KN_CHECKED), they cost
        // SGPRs in the hot loop
        unsigned st_rows = 0, st_cand = 0, st_ins = 0;
        KN_PH_MARK(kPhScan);
        scan_region(
            [&]() {
                const unsigned last = keys[KM - 1];
                return last == SENT ? INFINITY : __uint_as_float(last | MASK);
            },
            [&](int s0, int s1) {
                int s = s0;
                if constexpr (LANE) {
                    // divergent per-lane walk: kUnroll gathers in flight per lane, per K bucket from
                    // interleaved A/Bs at 900K (profiles/ab_r2_lane_unroll.txt): 3 for K <= 40
                    // (vs 2: K=8 -3.8 %, 16 -1.5 %, 24 -3.6 %, 32 -1 to -3 %, 40 -3.1 %), 1 for
                    // the K=50 bucket (-2.4 %), 2 for K=64 (1 and 3 lose or tie)
                    constexpr int kUnroll = KT <= 40 ? KN_LANE_UNROLL40 : (KT <= 50 ? KN_LANE_UNROLL50 : KN_LANE_UNROLL);
                    if constexpr (kStats && KN_WALK_STATS) {
                        // wave-uniform: row iterations and lockstep candidate steps (the unrolled
                        // loop runs to the longest span, then the remainder loop)
                        const unsigned L = (unsigned)max(0, s1 - s0);
                        const unsigned steps = (unsigned)kUnroll * wave_max_u32(L / (unsigned)kUnroll) +
                                               wave_max_u32(L % (unsigned)kUnroll);
                        st_rows += steps > 0u ? 1u : 0u;
                        st_cand += steps;
                    } else if constexpr (kStats) {
                        st_rows += (s1 > s0) ? 1u : 0u;
                        st_cand += (unsigned)max(0, s1 - s0);
                    }
                    for (; s + kUnroll <= s1; s += kUnroll) {
                        float4 p[kUnroll];
                        unsigned kk[kUnroll];
#pragma unroll
                        for (int u = 0; u < kUnroll; ++u) p[u] = pts[s + u];
#pragma unroll
                        for (int u = 0; u < kUnroll; ++u) kk[u] = cand_key_v(p[u], qx, qy, qz, HIMASK, s + u);
#pragma unroll
                        for (int u = 0; u < kUnroll; ++u) {
                            const unsigned i0 = topk_push<KM, KN_TOPK_SPLIT, tile_tiers<KT>()>(keys, kk[u]);
                            if constexpr (kStats) st_ins += i0;
                        }
                    }
                    for (; s < s1; ++s) {
                        const unsigned i0 = topk_push<KM, KN_TOPK_SPLIT, tile_tiers<KT>()>(keys, cand_key_v(pts[s], qx, qy, qz, HIMASK, s));
                        if constexpr (kStats) st_ins += i0;
                    }
                    return;
                } else {
                if constexpr (kStats) {
                    st_rows += 1u;
                    st_cand += (unsigned)(s1 - s0);
                }
                // software-pipelined: the next 4 broadcast reads are issued before the current 4
                // candidates are scored (two register sets, no loop-carried copies); reads past
                // s1 stay inside the workgroup's LDS and are never scored
                if (s + 4 <= s1) {
                    float4 a0 = pts[s], a1 = pts[s + 1], a2 = pts[s + 2], a3 = pts[s + 3];
                    auto score4 = [&](const float4& p0, const float4& p1, const float4& p2, const float4& p3, int sb) {
                        const unsigned k0 = cand_key(p0, qx, qy, qz, HIMASK, sb, qslot);
                        const unsigned k1 = cand_key(p1, qx, qy, qz, HIMASK, sb + 1, qslot);
                        const unsigned k2 = cand_key(p2, qx, qy, qz, HIMASK, sb + 2, qslot);
                        const unsigned k3 = cand_key(p3, qx, qy, qz, HIMASK, sb + 3, qslot);
                        asm volatile("" ::"v"(k0), "v"(k1), "v"(k2), "v"(k3));
                        const unsigned i0 = topk_push<KM, KN_TOPK_SPLIT, tile_tiers<KT>()>(keys, k0);
                        const unsigned i1 = topk_push<KM, KN_TOPK_SPLIT, tile_tiers<KT>()>(keys, k1);
                        const unsigned i2 = topk_push<KM, KN_TOPK_SPLIT, tile_tiers<KT>()>(keys, k2);
                        const unsigned i3 = topk_push<KM, KN_TOPK_SPLIT, tile_tiers<KT>()>(keys, k3);
                        if constexpr (kStats) st_ins += i0 + i1 + i2 + i3;
                    };
                    while (true) {
                        const float4 b0 = pts[s + 4], b1 = pts[s + 5], b2 = pts[s + 6], b3 = pts[s + 7];
                        score4(a0, a1, a2, a3, s);
                        s += 4;
                        if (s + 4 > s1) break;
                        a0 = pts[s + 4]; a1 = pts[s + 5]; a2 = pts[s + 6]; a3 = pts[s + 7];
                        score4(b0, b1, b2, b3, s);
                        s += 4;
                        if (s + 4 > s1) break;
                    }
                }
                for (; s < s1; ++s) {
                    const unsigned i0 = topk_push<KM, KN_TOPK_SPLIT, tile_tiers<KT>()>(keys, cand_key(pts[s], qx, qy, qz, HIMASK, s, qslot));
                    if constexpr (kStats) st_ins += i0;
                }
                }
            });
        if (kStats && LANE && KN_WALK_STATS) {  // wave-uniform row iterations / steps / networks
            if (lane == 0) {
                atomicAdd(a.counters + 4, st_rows);
                atomicAdd(a.counters + 5, st_cand);
                atomicAdd(a.counters + 6, st_ins);
                atomicAdd(a.counters + 7, 1u);
            }
        } else if (kStats && LANE) {  // lane walk: per-lane rows / candidates, summed over live lanes
            if (live && in_range) {
                atomicAdd(a.counters + 4, st_rows);
                atomicAdd(a.counters + 5, st_cand);
            }
            if (lane == 0) {
                atomicAdd(a.counters + 6, st_ins);
                atomicAdd(a.counters + 7, 1u);
            }
        } else if (kStats && lane == 0) {  // wave-uniform work statistics (4 atomics per chunk)
            atomicAdd(a.counters + 4, st_rows);
            atomicAdd(a.counters + 5, st_cand);
            atomicAdd(a.counters + 6, st_ins);
            atomicAdd(a.counters + 7, 1u);
        }

        KN_PH_MARK(kPhRerank);
        const int k = a.k;
        const bool act = in_range && live;
        // ---- exact re-rank: streaming window ---------------------------------------------
        // keys are sorted by (truncated d2, slot); the exact (d2, id) order can differ only
        // inside a run of equal truncation buckets. A kept candidate's output position is its
        // number of valid predecessors in key order plus the signed count of same-bucket
        // neighbours within +-kWin that cross it in exact order. Computed on the fly, so only a
        // window of 2*kWin+1 exact (d2, id) pairs is live instead of two KM-arrays (the odd-even
        // transposition re-rank held both: K=50 176 VGPRs = 2 waves/SIMD). Rows are written
        // before certification; a row that fails it is rewritten by the exact kernel, which
        // runs later on the same stream. Runs longer than kWin + 1 (lattices, heavy
        // duplication) take the wave-cooperative sort below.
        const unsigned qs = (unsigned)qslot;
        auto kvalid = [&](unsigned key) { return key != SENT && (!kSelfSlot || (key & MASK) != qs); };
        // precision reference taken before the window pass consumes the keys (and before the
        // self key is dropped below)
        const unsigned last = keys[KM - 1];
        if constexpr (kSelfSlot && KN_VEC_OUT) {
            // drop the query's own key (d2 = 0: nearly always keys[0]) so the valid keys form a
            // prefix and entry j lands at position j (+-1): the in-order row stores of the window
            // pass rely on it. One compare and select per key; the self mask is a scalar OR.
            bool seen = false;
#pragma unroll
            for (int t = 0; t < KM; ++t) {
                seen = seen | ((keys[t] != SENT) & ((keys[t] & MASK) == qs));
                keys[t] = seen ? (t + 1 < KM ? keys[t + 1 < KM ? t + 1 : KM - 1] : SENT) : keys[t];
            }
        }
        const bool force = (a.flags & kQueryForceRescan) != 0;
        bool ovf = force;
        // wider-window overflow (== ovf when the second window is off)
        bool ovf2 = force;
        int nfound = 0;
#pragma unroll
        for (int j = 0; j + kWin + 1 < KM; ++j)
            ovf |= keys[j + kWin + 1] != SENT && ((keys[j] ^ keys[j + kWin + 1]) & HIMASK) == 0u;
        if constexpr (WIDE && kWin2 > 0) {
#pragma unroll
            for (int j = 0; j + kWin2 + 1 < KM; ++j)
                ovf2 |= keys[j + kWin2 + 1] != SENT && ((keys[j] ^ keys[j + kWin2 + 1]) & HIMASK) == 0u;
        } else {
            ovf2 = ovf;
        }
        const unsigned orow = act ? w_row(a, qorig, qsidx) : 0u;
        const size_t row = (size_t)orow * (size_t)k;
        float dK2 = INFINITY;
        auto window_pass = [&](auto wc) {
            constexpr int W = decltype(wc)::value;
            // Rolled loop over the kept keys with constant register indices only: the key array
            // shifts down one slot per step (KM moves) and the window rotates, so no unrolled
            // straight-line code gives the scheduler room to pull every entry's LDS read and
            // compare forward (fully unrolled, K=50 needed 214 VGPRs; rolled it stays near the
            // scan loop's own pressure).
            constexpr int NW = 2 * W + 1;
            float wd[NW];
            unsigned wi[NW], wk[NW];
            auto ld = [&](unsigned key, int t) {
                const bool v = kvalid(key);
                const float4 p = pts[KN_IDX(v ? (key & MASK) : 0u, (unsigned)S, 208)];
                const float dx = p.x - qx, dy = p.y - qy, dz = p.z - qz;
                wk[t] = v ? key : SENT;
                wd[t] = v ? fmaf(dz, dz, fmaf(dy, dy, dx * dx)) : INFINITY;
                wi[t] = v ? w_id(a, __float_as_uint(p.w)) : SENT;
            };
#pragma unroll
            for (int t = 0; t < NW; ++t) ld((t >= W && t - W < KM) ? keys[t - W] : SENT, t);
            int base = 0;
            // W = 1 (KN_RERANK_PAIR): each adjacent pair is compared ONCE. c = "entry j+1 precedes
            // entry j in exact (d2, id) order and shares its truncation bucket"; entry j's position
            // is base - c(j-1, j) + c(j, j+1), the first term carried from the previous entry. (The
            // general form compares j with both neighbours, i.e. every pair twice. The validity
            // test of the earlier entry can be dropped: a SENT key never shares a finite key's
            // bucket, and an invalid entry's own position is never used.)
            int c_prev = 0;
            // KN_VEC_OUT (window W = 1): with disjoint swaps, POSITION j's final entry is known at
            // step j -- entry j-1 if it swapped forward (c_prev), entry j+1 if j swaps with it
            // (c_next), else entry j -- so the row is written in order, V positions per global
            // store instead of one scattered 4-byte store per entry and array (those stores were
            // 8 % of the K=16 kernel and 23 % at K=50: profiles/ab_r6_vec_out.txt). Positions past
            // the valid prefix get don't-care values: such a row has nfound < k, fails
            // certification and is rewritten by the exact path. Needs k % V == 0 and V-aligned
            // output pointers (checked here, uniform), else the per-entry stores below.
            constexpr int V = out_vec_width<KT>();
            constexpr bool kVec = W == 1 && KN_RERANK_PAIR && V > 1;
            const bool vec = kVec && out_vec_ok<V>(k, (const void*)o_idx, (const void*)o_dist);
            unsigned ob_i[V];
            float ob_d[V];
            int jb = 0;  // absolute index of the entry at u = 0 (the rolled loop's group base)
            // entry(u): the next kept key; u = its compile-time offset since the last shift of keys[]
            auto entry = [&](auto uc) __attribute__((always_inline)) {
                constexpr int u = decltype(uc)::value;
                const bool vj = wk[W] != SENT;
                int pos = base;
                if constexpr (W == 1 && KN_RERANK_PAIR) {
                    const int same = (int)(wk[2] != SENT) & (int)(((wk[2] ^ wk[1]) & HIMASK) == 0u);
                    const int lt = (int)(wd[2] < wd[1]) | ((int)(wd[2] == wd[1]) & (int)(wi[2] < wi[1]));
                    const int c_next = same & lt;
                    pos += c_next - c_prev;
                    if constexpr (kVec) {
                        if (vec) {
                            constexpr int sl = u % V;
                            ob_d[sl] = c_prev ? wd[0] : (c_next ? wd[2] : wd[1]);
                            // (an invalid entry's id is SENT: never through out_id's id_map gather)
                            const unsigned oid = c_prev ? wi[0] : (c_next ? wi[2] : wi[1]);
                            ob_i[sl] = oid == SENT ? SENT : out_id(a, oid);
                            if constexpr (sl == V - 1) {
                                const int j0 = jb + u - (V - 1);
                                if (act && j0 + (V - 1) < k && !KN_DIAG_SKIP_OUT) {
                                    const size_t o = KN_IDX(row + (size_t)j0 + (V - 1), (size_t)a.n_queries * k, 210) - (V - 1);
                                    store_vec<V>(o_idx + o, ob_i);
                                    if (o_dist) store_vec<V>(o_dist + o, ob_d);
                                }
                            }
                            if constexpr (V == 4 && KN_VEC_TAIL && sl == 1) {
                                // the row's last two positions (k % 4 == 2)
                                if (act && jb + u == k - 1 && !KN_DIAG_SKIP_OUT) {
                                    const size_t o = KN_IDX(row + (size_t)k - 1, (size_t)a.n_queries * k, 211) - 1;
                                    const unsigned ti[2] = {ob_i[0], ob_i[1]};
                                    const float td[2] = {ob_d[0], ob_d[1]};
                                    store_vec<2>(o_idx + o, ti);
                                    if (o_dist) store_vec<2>(o_dist + o, td);
                                }
                            }
                        }
                    }
                    c_prev = c_next;
                } else {
#pragma unroll
                for (int t = 0; t < NW; ++t) {
                    if (t == W) continue;
                    // branch-free: bitwise &/| (short-circuit forms compile to exec-mask branches)
                    const int same = (int)(wk[t] != SENT) & (int)(((wk[t] ^ wk[W]) & HIMASK) == 0u);
                    const float da = t > W ? wd[t] : wd[W], db = t > W ? wd[W] : wd[t];
                    const unsigned ia = t > W ? wi[t] : wi[W], ib = t > W ? wi[W] : wi[t];
                    const int lt = (int)(da < db) | ((int)(da == db) & (int)(ia < ib));
                    pos += (t > W ? 1 : -1) * (same & lt);
                }
                }
                if (!vec && vj && act && pos < k && !KN_DIAG_SKIP_OUT) {
                    const size_t o = KN_IDX(row + pos, (size_t)a.n_queries * k, 209);
                    o_idx[o] = out_id(a, wi[W]);
                    if (o_dist) o_dist[o] = wd[W];
                }
                dK2 = (vj && pos == k - 1) ? wd[W] : dK2;
                base += vj ? 1 : 0;
#pragma unroll
                for (int t = 0; t + 1 < NW; ++t) { wk[t] = wk[t + 1]; wd[t] = wd[t + 1]; wi[t] = wi[t + 1]; }
                // entry j + W + 1 sits at keys[W + 1 + u] (keys[] shifted j - u times so far)
                constexpr int nx = W + 1 + u;
                ld(nx < KM ? keys[nx < KM ? nx : KM - 1] : SENT, NW - 1);
            };
            // KN_RERANK_UNROLL: the K buckets with KM <= 24 unroll the whole walk (no key shifts:
            // register renames). Larger lists run a rolled loop over groups of KN_RERANK_GROUP
            // entries, shifting keys[] once per group (KM - G moves per G entries instead of per
            // entry; the < G padding entries past the end see SENT keys and write nothing).
            if constexpr (KN_RERANK_UNROLL && KM <= 24) {
                static_for<0, KM>(entry);
            } else {
                constexpr int G = KN_RERANK_GROUP;
#pragma unroll 1
                for (int jj = 0; jj < KM; jj += G) {
                    jb = jj;
                    static_for<0, G>(entry);
#pragma unroll
                    for (int t = 0; t < KM; ++t) keys[t] = t + G < KM ? keys[t + G < KM ? t + G : KM - 1] : SENT;
                }
            }
            nfound = base;
        };
        if (!ovf) window_pass(IntC<kWin>{});
        if constexpr (WIDE && kWin2 > 0) {
            if (ovf && !ovf2) window_pass(IntC<kWin2>{});
        }
        ovf = ovf2;  // what is left for the cooperative sort
        // Wave-cooperative finish of ONE lane's query at a time (rare paths): the wave holds
        // 64-bit (d2 bits, id) keys, E per lane, bitonic-sorts them across lanes and writes the
        // lane's row; the lane gets its exact K-th distance and found count back.
        const size_t rowq = row;
        auto coop_finish = [&](int L, auto& v) {
            constexpr int E = (int)std::extent<std::remove_reference_t<decltype(v)>>::value;
            wave_bitonic_sort_u64<E>(v, lane);
            const size_t rowL = (size_t)__builtin_amdgcn_readlane((int)(rowq / (size_t)k), L) * (size_t)k;
            int nf = 0;
#pragma unroll
            for (int e = 0; e < E; ++e) nf += __builtin_popcountll(__builtin_amdgcn_ballot_w64(v[e] != ~0ull));
#pragma unroll
            for (int e = 0; e < E; ++e) {
                const int r = 64 * e + lane;
                if (r < k && v[e] != ~0ull) {
                    const size_t o = KN_IDX(rowL + r, (size_t)a.n_queries * k, 214);
                    o_idx[o] = out_id(a, (unsigned)v[e]);
                    if (o_dist) o_dist[o] = __uint_as_float((unsigned)(v[e] >> 32));
                }
            }
            float dk = INFINITY;
#pragma unroll
            for (int e = 0; e < E; ++e)
                if ((k - 1) / 64 == e)
                    dk = __uint_as_float((unsigned)__builtin_amdgcn_readlane((int)(unsigned)(v[e] >> 32), (k - 1) & 63));
            if (nf < k) dk = INFINITY;
            if (lane == L) { dK2 = dk; nfound = nf; }
        };
        // (1) window overflow (or every lane under kQueryForceRescan): sort the lane's KM kept keys
        for (unsigned long long om = __builtin_amdgcn_ballot_w64(ovf && act); om; om &= om - 1) {
            const int L = __builtin_ctzll(om);
            constexpr int E = (KM + 63) / 64;
            const unsigned qsL = (unsigned)__builtin_amdgcn_readlane((int)qs, L);
            const float qxL = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(qx), L));
            const float qyL = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(qy), L));
            const float qzL = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(qz), L));
            unsigned long long v[E];
#pragma unroll
            for (int e = 0; e < E; ++e) {
                unsigned key = SENT;
#pragma unroll
                for (int j = 64 * e; j < KM && j < 64 * (e + 1); ++j) {
                    const unsigned kj = (unsigned)__builtin_amdgcn_readlane((int)keys[j], L);
                    key = (lane == j - 64 * e) ? kj : key;
                }
                const bool valid = key != SENT && (key & MASK) != qsL;
                const float4 p = pts[KN_IDX(valid ? (key & MASK) : 0u, (unsigned)S, 213)];
                const float dx = p.x - qxL, dy = p.y - qyL, dz = p.z - qzL;
                const float d = fmaf(dz, dz, fmaf(dy, dy, dx * dx));
                v[e] = valid ? pack_key64(d, w_id(a, __float_as_uint(p.w))) : ~0ull;
            }
            coop_finish(L, v);
            if (lane == 0) atomicAdd(a.counters + 3, 1u);  // cooperative re-ranks (diagnostic)
        }
        // (2) precision: everything truncated away has exact d2 >= the floor of the last key's
        // bucket. If the exact K-th distance reaches into it (K-th and last kept candidates
        // within one truncation ulp), the wave re-scans the lane's region exactly: every point
        // with d2 <= that K-th distance (an upper bound of the true one) is compacted into a
        // per-wave LDS buffer, then sorted and written as above. More than kCoopCap such
        // points (heavy duplication) leave the query to the exact kernel.
        bool prec_fail = last != SENT && !(dK2 <= __uint_as_float(last & HIMASK));
        // The wave's re-scan buffer lives in the unused tail of the staged-point area (slots
        // [S, cap)): no LDS is reserved for this rare path, which keeps the workgroup's LDS (and
        // so the workgroups per CU) at the staging's. A wave whose slice does not fit leaves
        // the query to the exact kernel (prec_fail stays set).
        constexpr int kCoopSlots = kCoopCap * 8 / (int)sizeof(float4);
        const bool coop_ok = S + (wid + 1) * kCoopSlots <= a.cap;
        for (unsigned long long om = __builtin_amdgcn_ballot_w64(prec_fail && act && coop_ok); om; om &= om - 1) {
            const int L = __builtin_ctzll(om);
            auto rl = [&](int v) { return __builtin_amdgcn_readlane(v, L); };
            auto rlf = [&](float v) { return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), L)); };
            const int qsL = rl(qslot);
            const float qxL = rlf(qx), qyL = rlf(qy), qzL = rlf(qz), thr = rlf(dK2);
            const int x0 = rl(rx0), x1 = rl(rx1), y0 = rl(ry0), y1 = rl(ry1), z0 = rl(rz0), z1 = rl(rz1);
            unsigned long long* buf = reinterpret_cast<unsigned long long*>(pts + S) + wid * kCoopCap;
            const unsigned long long lt = (lane == 0) ? 0ull : (~0ull >> (64 - lane));
            int cnt = 0;
            for (int z = z0; z <= z1; ++z) {
                const float dzb = slab_dist(g, 2, qzL, sz0 + z, sz0 + z);
                const float dz2 = dzb * dzb;
                if (!(dz2 <= thr)) continue;
                for (int y = y0; y <= y1; ++y) {
                    const float dyb = slab_dist(g, 1, qyL, sy0 + y, sy0 + y);
                    const float dyz2 = fmaf(dyb, dyb, dz2);
                    if (!(dyz2 <= thr)) continue;
                    const float rr = rsqrt(thr - dyz2) * 1.000001f + g.eps;
                    const int lx0 = max(x0, cell_coord(g, 0, qxL - rr) - sx0);
                    const int lx1 = min(x1, cell_coord(g, 0, qxL + rr) - sx0);
                    if (lx0 > lx1) continue;
                    const int r = y + nys * z;
                    const int rb = rowbase[r];
                    const int s0 = __builtin_amdgcn_readfirstlane(rb + (int)cbr[r * cbs + lx0]);
                    const int s1 = __builtin_amdgcn_readfirstlane(KN_IDX(rb + (int)cbr[r * cbs + lx1 + 1], S + 1, 215));
                    for (int sb = s0; sb < s1; sb += 64) {
                        const int sl = sb + lane;
                        bool pass = false;
                        unsigned long long key = 0;
                        if (sl < s1 && sl != qsL) {
                            const float4 p = pts[sl];
                            const float dx = p.x - qxL, dy = p.y - qyL, dz = p.z - qzL;
                            const float d = fmaf(dz, dz, fmaf(dy, dy, dx * dx));
                            pass = d <= thr;
                            key = pack_key64(d, w_id(a, __float_as_uint(p.w)));
                        }
                        const unsigned long long bal = __builtin_amdgcn_ballot_w64(pass);
                        const int at = cnt + __builtin_popcountll(bal & lt);
                        if (pass && at < kCoopCap) buf[at] = key;
                        cnt += __builtin_popcountll(bal);
                    }
                }
            }
            __builtin_amdgcn_wave_barrier();
            if (cnt <= kCoopCap) {
                unsigned long long v[kCoopCap / 64];
#pragma unroll
                for (int e = 0; e < kCoopCap / 64; ++e) v[e] = (64 * e + lane < cnt) ? buf[64 * e + lane] : ~0ull;
                __builtin_amdgcn_wave_barrier();
                coop_finish(L, v);
                if (lane == L) prec_fail = false;
            }
            if (lane == 0) atomicAdd(a.counters + 3, 1u);  // cooperative re-ranks (diagnostic)
        }
        KN_PH_MARK(kPhCertify);
        if (!act) continue;

        // distance to the boundary of the scanned region (grid faces do not count: no points
        // exist beyond the grid) and to the complete box (multi-GPU halo limit)
        float m = INFINITY;
        {
            const int gx0 = sx0 + rx0, gx1 = sx0 + rx1, gy0 = sy0 + ry0, gy1 = sy0 + ry1;
            const int gz0 = sz0 + rz0, gz1 = sz0 + rz1;
            if (gx0 > 0) m = fminf(m, qx - (g.origin[0] + gx0 * g.cell[0]));
            if (gx1 < a.X - 1) m = fminf(m, g.origin[0] + (gx1 + 1) * g.cell[0] - qx);
            if (gy0 > 0) m = fminf(m, qy - (g.origin[1] + gy0 * g.cell[1]));
            if (gy1 < a.Y - 1) m = fminf(m, g.origin[1] + (gy1 + 1) * g.cell[1] - qy);
            if (gz0 > 0) m = fminf(m, qz - (g.origin[2] + gz0 * g.cell[2]));
            if (gz1 < a.Z - 1) m = fminf(m, g.origin[2] + (gz1 + 1) * g.cell[2] - qz);
            m = fminf(m, complete_margin3(a.complete, qx, qy, qz));
            m -= g.eps;
        }
        const bool geo_ok = !prec_fail && (nfound >= k) && (m > 0.f) && (m == INFINITY || dK2 <= m * m);
        if (!geo_ok) {
            const unsigned pos = atomicAdd(a.counters + 0, 1u);
            // the row already holds K real candidates: their K-th distance bounds the true one,
            // and the exact kernel starts its walk with it (kSeedBit)
            const bool seed = o_dist && nfound >= k && dK2 < INFINITY;
            a.fallback_list[KN_IDX(pos, (unsigned)a.n, 210)] = qsidx | (seed ? kSeedBit : 0u);
        }
    }
    KN_PH_MARK(kPhStage);
    KN_PH_FLUSH();
}

// ---------------------------------------------------------------------------------------
// knn_stream_kernel -- the tile kernel's algorithm (one workgroup per cell tile, 64 queries
// per wave, wave-uniform candidate stream, med3 top-K, exact re-rank, certification) WITHOUT
// the workgroup-wide LDS staging of the tile + halo points. Each wave streams the cell rows
// it needs straight from the cell-sorted array (L2-resident; one point per lane, 16-B
// coalesced), ONE ROW AHEAD: the next row's extent is derived with the current (stale, hence
// conservative) bound and its load is in flight while the current row is scored. A 64-entry
// wave-private LDS ring turns the per-lane loads into broadcast reads for the hot loop.
//   * no staging phase, no per-tile LDS capacity (dense tiles no longer spill to the exact
//     kernel), ~11 KB of LDS per workgroup -> occupancy is set by VGPRs, and waves of a
//     workgroup run independently (a wave without a chunk exits at once);
//   * top-K keys carry the candidate's STREAM POSITION in their low SB bits; a per-wave row
//     table {position of the row's first candidate, its stored index} maps a kept key back to
//     its point at the re-rank (binary lifting, all K+M keys in lockstep).
// PMC that motivated it (900K, k=16, tile kernel): SQ_WAIT_ANY 35 % of wave cycles (staging
// loads + barriers), ~2.6 resident waves/SIMD of the 5 the LDS budget allows.
constexpr int kRing = 64;
constexpr int kMaxRowsPerChunk = 128;
constexpr int kStreamSlotBits = 11;  // stream positions per chunk: 2048

// Occupancy target: the scheduler otherwise trades waves for ILP (unconstrained: 112-187
// VGPRs = 2-4 waves/SIMD); 5 waves/SIMD fits in 94 VGPRs without spills.
#ifndef KN_STREAM_WPE
#define KN_STREAM_WPE 5
#endif
template <int KT, int M>
__global__ __launch_bounds__(kWG) __attribute__((amdgpu_waves_per_eu(KN_STREAM_WPE, 8))) void knn_stream_kernel(
    TileArgs a) {
    // output pointers: the launch's, or read from device slots (graph replays of a batched
    // stream of clouds); locals, so the kernel argument block stays read-only
    out_u32_t* const o_idx = out_ptr(a.out_idx_ref ? *a.out_idx_ref : a.out_idx);
    out_f32_t* const o_dist = out_ptr(a.out_idx_ref ? (a.out_dist_ref ? *a.out_dist_ref : nullptr) : a.out_dist);
    constexpr int KM = KT + M + 1;
    constexpr unsigned MASK = (1u << kStreamSlotBits) - 1u;
    constexpr unsigned HIMASK = ~MASK;
    __shared__ __attribute__((aligned(16))) float4 ring_all[kWaves][kRing];
    __shared__ int rpos_all[kWaves][kMaxRowsPerChunk];
    __shared__ int rsid_all[kWaves][kMaxRowsPerChunk];
    extern __shared__ __attribute__((aligned(16))) int dyn[];
    int* cb = dyn;
    int* qpref = cb + a.max_rows * a.cb_stride;  // TY*TZ + 1 entries

    const GridGeom g = *a.geom;
    const int ntiles = a.ntx * a.nty * a.ntz;
    const int tile = xcd_remap(blockIdx.x, ntiles);
    const int tx = tile % a.ntx, ty = (tile / a.ntx) % a.nty, tz = tile / (a.ntx * a.nty);
    const int tx0 = tx * a.TX, ty0 = ty * a.TY, tz0 = tz * a.TZ;
    const int tx1 = min(a.X, tx0 + a.TX), ty1 = min(a.Y, ty0 + a.TY), tz1 = min(a.Z, tz0 + a.TZ);
    const int sx0 = max(0, tx0 - a.Hx), sx1 = min(a.X, tx1 + a.Hx);
    const int sy0 = max(0, ty0 - a.H), sy1 = min(a.Y, ty1 + a.H);
    const int sz0 = max(0, tz0 - a.H), sz1 = min(a.Z, tz1 + a.H);
    const int nxs = sx1 - sx0, nys = sy1 - sy0, nzs = sz1 - sz0;
    const int nrows = nys * nzs;
    const int cbs = nxs + 1;
    const int ntry = ty1 - ty0, ntrz = tz1 - tz0, ntr = ntry * ntrz;
    const int hx = tx0 - sx0;
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    float4* ring = ring_all[wid];
    int* rpos = rpos_all[wid];
    int* rsid = rsid_all[wid];

    // ---- 1. cell boundaries of every row of the tile + halo box (as knn_tile_kernel) ----
    for (int t = threadIdx.x; t < nrows * cbs; t += kWG) {
        const int r = t / cbs, i = t - r * cbs;
        const int y = sy0 + r % nys, z = sz0 + r / nys;
        cb[r * cbs + i] = a.cell_start[KN_IDX((z * a.Y + y) * a.X + sx0 + i, a.X * a.Y * a.Z + 1, 221)];
    }
    __syncthreads();
    // ---- 2. query prefix over the tile's rows (wave 0) ----------------------------------
    if (wid == 0) {
        int qc = 0;
        for (int base = 0; base < ntr; base += 64) {
            const int t = base + lane;
            int len = 0;
            if (t < ntr) {
                const int r = (ty0 - sy0 + t % ntry) + nys * (tz0 - sz0 + t / ntry);
                len = cb[r * cbs + hx + (tx1 - tx0)] - cb[r * cbs + hx];
            }
            const int incl = wave_inclusive_scan_add(len);
            if (t < ntr) qpref[t] = qc + incl - len;
            qc += __shfl(incl, 63, 64);
        }
        if (lane == 0) qpref[ntr] = qc;
    }
    __syncthreads();
    const int Q = qpref[ntr];

    // ---- 3. query chunks: 64 queries per wave -------------------------------------------
    for (int chunk = wid; chunk * 64 < Q; chunk += kWaves) {
        const int qi_raw = chunk * 64 + lane;
        const bool in_range = qi_raw < Q;
        const int qi = in_range ? qi_raw : Q - 1;
        int lo = 0, hi = ntr - 1;
        while (lo < hi) { const int mid = (lo + hi + 1) >> 1; if (qpref[mid] <= qi) lo = mid; else hi = mid - 1; }
        const int qrow = (ty0 - sy0 + lo % ntry) + nys * (tz0 - sz0 + lo / ntry);
        const unsigned qsidx = (unsigned)(cb[qrow * cbs + hx] + (qi - qpref[lo]));
        const float4 qp = a.sorted[KN_IDX(qsidx, (unsigned)a.n, 222)];
        const unsigned qorig = __float_as_uint(qp.w);
        const bool live = w_live(a, qorig);
        const float qx = qp.x, qy = qp.y, qz = qp.z;
        const int cx = cell_coord(g, 0, qx) - sx0;
        const int cy = cell_coord(g, 1, qy) - sy0;
        const int cz = cell_coord(g, 2, qz) - sz0;
        const int2 bx = wave_minmax_i32(live ? cx : INT_MAX, live ? cx : INT_MIN);
        if (bx.x > bx.y) continue;  // no live query in this chunk (uniform)
        const int2 by = wave_minmax_i32(live ? cy : INT_MAX, live ? cy : INT_MIN);
        const int2 bz = wave_minmax_i32(live ? cz : INT_MAX, live ? cz : INT_MIN);
        const int rx0 = max(0, bx.x - a.Hx), rx1 = min(nxs - 1, bx.y + a.Hx);
        const int ry0 = max(0, by.x - a.H), ry1 = min(nys - 1, by.y + a.H);
        const int rz0 = max(0, bz.x - a.H), rz1 = min(nzs - 1, bz.y + a.H);
        const int zc = (bz.x + bz.y) >> 1, yc = (by.x + by.y) >> 1;
        const int nzt = 2 * max(zc - rz0, rz1 - zc) + 1;
        const int nyt = 2 * max(yc - ry0, ry1 - yc) + 1;
        const int nit = nzt * nyt;

        // union x-range (local cells) of the row visited at iteration `it` under bound `tau`;
        // returns false (uniform) when the row lies outside the region or no lane needs it
        auto row_range = [&](int it, float tau, int& r, int& X0, int& X1) -> bool {
            const int tz_ = it / nyt, ty_ = it - tz_ * nyt;
            const int z = zc + ((tz_ & 1) ? ((tz_ + 1) >> 1) : -(tz_ >> 1));
            const int y = yc + ((ty_ & 1) ? ((ty_ + 1) >> 1) : -(ty_ >> 1));
            if (z < rz0 || z > rz1 || y < ry0 || y > ry1) return false;
            const float dzb = slab_dist(g, 2, qz, sz0 + z, sz0 + z);
            const float dyb = slab_dist(g, 1, qy, sy0 + y, sy0 + y);
            const float dyz2 = fmaf(dyb, dyb, dzb * dzb);
            int lx0 = INT_MAX, lx1 = INT_MIN;
            if (tau == INFINITY) {
                lx0 = rx0; lx1 = rx1;
            } else if (dyz2 <= tau) {
                const float rr = sqrt_bound(tau - dyz2) * 1.000001f + g.eps;
                lx0 = max(rx0, cell_coord(g, 0, qx - rr) - sx0);
                lx1 = min(rx1, cell_coord(g, 0, qx + rr) - sx0);
            }
            if (!live) { lx0 = INT_MAX; lx1 = INT_MIN; }
            const int2 X = wave_minmax_i32(lx0, lx1);
            r = y + nys * z;
            X0 = X.x; X1 = X.y;
            return X.x <= X.y;
        };

        unsigned keys[KM];
#pragma unroll
        for (int j = 0; j < KM; ++j) keys[j] = SENT;
        auto lane_tau = [&]() {
            const unsigned last = keys[KM - 1];
            return last == SENT ? INFINITY : __uint_as_float(last | MASK);
        };

        // prefetch state: the next non-empty row (iteration, staged-row, stored range)
        int it = 0;
        int pf_it = -1, pf_r = 0, pf_p0 = 0, pf_p1 = 0;
        float4 pf = make_float4(0.f, 0.f, 0.f, 0.f);
        auto prefetch_next = [&]() {
            const float tau = lane_tau();
            pf_it = -1;
            for (; it < nit; ++it) {
                int r, X0, X1;
                if (row_range(it, tau, r, X0, X1)) {
                    pf_it = it; pf_r = r;
                    pf_p0 = __builtin_amdgcn_readfirstlane(cb[r * cbs + X0]);
                    pf_p1 = __builtin_amdgcn_readfirstlane(cb[r * cbs + X1 + 1]);
                    if (lane < pf_p1 - pf_p0) pf = a.sorted[KN_IDX(pf_p0 + lane, a.n, 223)];
                    ++it;
                    return;
                }
            }
        };

        int nrow = 0;         // rows recorded in the row table (uniform)
        unsigned pos = 0;     // stream position of the next candidate (uniform)
        bool overflow = false;
        prefetch_next();
        while (pf_it >= 0) {
            const int cur_it = pf_it, cur_r = pf_r, cur_p0 = pf_p0, cur_p1 = pf_p1;
            if (lane < cur_p1 - cur_p0) ring[lane] = pf;
            prefetch_next();  // next row's load overlaps this row's scoring
            int r, X0, X1;
            if (!row_range(cur_it, lane_tau(), r, X0, X1)) continue;  // bound shrank past it
            const int s0 = __builtin_amdgcn_readfirstlane(cb[cur_r * cbs + X0]);
            const int s1 = __builtin_amdgcn_readfirstlane(cb[cur_r * cbs + X1 + 1]);
            if (s0 >= s1) continue;
            if (nrow >= kMaxRowsPerChunk || pos + (unsigned)(s1 - s0) > MASK + 1u) { overflow = true; break; }
            if (lane == 0) { rpos[nrow] = (int)pos; rsid[nrow] = s0; }
            ++nrow;
            // rows longer than the ring are scored in 64-point pieces (the first is prefetched)
            for (int base = cur_p0; base < s1; base += kRing) {
                if (base != cur_p0) {
                    const int len = min(kRing, cur_p1 - base);
                    float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
                    if (lane < len) v = a.sorted[KN_IDX(base + lane, a.n, 224)];
                    if (lane < len) ring[lane] = v;
                }
                const int i0 = max(s0, base) - base, i1 = min(s1, base + kRing) - base;
                if (i0 >= i1) continue;
                unsigned pp = pos + (unsigned)(base + i0 - s0);
                int i = i0;
                for (; i + 4 <= i1; i += 4, pp += 4) {
                    const float4 p0 = ring[i], p1 = ring[i + 1], p2 = ring[i + 2], p3 = ring[i + 3];
                    const unsigned k0 = cand_key(p0, qx, qy, qz, HIMASK, (int)pp, 0);
                    const unsigned k1 = cand_key(p1, qx, qy, qz, HIMASK, (int)pp + 1, 0);
                    const unsigned k2 = cand_key(p2, qx, qy, qz, HIMASK, (int)pp + 2, 0);
                    const unsigned k3 = cand_key(p3, qx, qy, qz, HIMASK, (int)pp + 3, 0);
                    asm volatile("" ::"v"(k0), "v"(k1), "v"(k2), "v"(k3));
                    topk_push<KM, KN_TOPK_SPLIT, tile_tiers<KT>()>(keys, k0);
                    topk_push<KM, KN_TOPK_SPLIT, tile_tiers<KT>()>(keys, k1);
                    topk_push<KM, KN_TOPK_SPLIT, tile_tiers<KT>()>(keys, k2);
                    topk_push<KM, KN_TOPK_SPLIT, tile_tiers<KT>()>(keys, k3);
                }
                for (; i < i1; ++i, ++pp) topk_push<KM, KN_TOPK_SPLIT, tile_tiers<KT>()>(keys, cand_key(ring[i], qx, qy, qz, HIMASK, (int)pp, 0));
            }
            pos += (unsigned)(s1 - s0);
        }
        if (overflow) {
            // stream too long for the key's slot bits / row table: the chunk's live queries
            // take the exact kernel (drain the prefetch first)
            if (live && in_range) {
                const unsigned p = atomicAdd(a.counters + 0, 1u);
                a.fallback_list[KN_IDX(p, (unsigned)a.n, 225)] = qsidx;
            }
            if (lane == 0) atomicAdd(a.counters + 2, 1u);
            continue;
        }

        // ---- exact re-rank: slot -> stored index via the row table (binary lifting) ------
        const unsigned last_key = keys[KM - 1];
        int rl[KM];
#pragma unroll
        for (int j = 0; j < KM; ++j) {
            keys[j] = keys[j] == SENT ? SENT : (keys[j] & MASK);  // slot (SENT stays)
            rl[j] = 0;
        }
#pragma unroll 1
        for (int st = kMaxRowsPerChunk / 2; st > 0; st >>= 1) {
            if (st >= nrow) continue;  // uniform
#pragma unroll
            for (int j = 0; j < KM; ++j) {
                const int c = min(rl[j] + st, kMaxRowsPerChunk - 1);
                if (rl[j] + st < nrow && rpos[c] <= (int)keys[j]) rl[j] = c;
                if ((j & 3) == 3) __builtin_amdgcn_sched_barrier(0);
            }
        }
#pragma unroll
        for (int j = 0; j < KM; ++j) {
            const unsigned sidx = (unsigned)(rsid[rl[j]] + ((int)keys[j] - rpos[rl[j]]));
            rl[j] = (keys[j] != SENT && sidx != qsidx) ? (int)sidx : -1;  // stored index or -1
        }
        float dd[KM];
        unsigned ii[KM];
#pragma unroll
        for (int j = 0; j < KM; ++j) {
            const unsigned sidx = (unsigned)rl[j];
            const bool valid = rl[j] >= 0;
            const float4 p = a.sorted[KN_IDX(valid ? sidx : qsidx, (unsigned)a.n, 226)];
            const float dx = p.x - qx, dy = p.y - qy, dz = p.z - qz;
            const float d = fmaf(dz, dz, fmaf(dy, dy, dx * dx));
            dd[j] = valid ? d : INFINITY;
            ii[j] = valid ? w_id(a, __float_as_uint(p.w)) : SENT;
            // at most 4 gathers in flight: 19 float4 loads hoisted together cost 76 VGPRs
            if ((j & 3) == 3) __builtin_amdgcn_sched_barrier(0);
        }
        const unsigned last = last_key;
        for (int round = 0; round < (KM + 1) / 2; ++round) {
            bool swapped = false;
#pragma unroll
            for (int pass = 0; pass < 2; ++pass) {
#pragma unroll
                for (int j = pass; j + 1 < KM; j += 2) {
                    const bool sw = pair_less(dd[j + 1], ii[j + 1], dd[j], ii[j]);
                    const float d0 = sw ? dd[j + 1] : dd[j], d1 = sw ? dd[j] : dd[j + 1];
                    const unsigned i0 = sw ? ii[j + 1] : ii[j], i1 = sw ? ii[j] : ii[j + 1];
                    dd[j] = d0; dd[j + 1] = d1; ii[j] = i0; ii[j + 1] = i1;
                    swapped |= sw;
                }
            }
            if (!__builtin_amdgcn_ballot_w64(swapped)) break;
        }
        const int k = a.k;
        auto kth = [&]() {
            float v = INFINITY;
#pragma unroll
            for (int j = 0; j < KM; ++j) if (j == k - 1) v = dd[j];
            return v;
        };
        float dK2 = kth();
        const bool need = live && ((last != SENT && !(dK2 <= __uint_as_float(last & HIMASK))) ||
                                   (a.flags & kQueryForceRescan));
        if (__builtin_amdgcn_ballot_w64(need)) {
            // truncation near-tie (rare): exact (d2, id) re-scan of the region, from global
            const float thr = need ? ((a.flags & kQueryForceRescan) ? INFINITY : dK2) : -1.f;
#pragma unroll
            for (int j = 0; j < KM; ++j) {
                dd[j] = need ? INFINITY : dd[j];
                ii[j] = need ? SENT : ii[j];
            }
            for (int it2 = 0; it2 < nit; ++it2) {
                int r, X0, X1;
                if (!row_range(it2, need ? thr : -1.f, r, X0, X1)) continue;
                const int s0 = __builtin_amdgcn_readfirstlane(cb[r * cbs + X0]);
                const int s1 = __builtin_amdgcn_readfirstlane(cb[r * cbs + X1 + 1]);
                for (int s = s0; s < s1; ++s) {
                    const float4 p = a.sorted[KN_IDX(s, a.n, 227)];
                    const float dx = p.x - qx, dy = p.y - qy, dz = p.z - qz;
                    const float d2 = fmaf(dz, dz, fmaf(dy, dy, dx * dx));
                    const unsigned id = w_id(a, __float_as_uint(p.w));
                    const bool take = (unsigned)s != qsidx && d2 <= thr && pair_less(d2, id, dd[KM - 1], ii[KM - 1]);
                    if (__builtin_amdgcn_ballot_w64(take)) {
                        if (take) {
#pragma unroll
                            for (int j = KM - 1; j > 0; --j) {
                                const bool bp = pair_less(d2, id, dd[j - 1], ii[j - 1]);
                                const bool bc = pair_less(d2, id, dd[j], ii[j]);
                                const float nd = bp ? dd[j - 1] : (bc ? d2 : dd[j]);
                                const unsigned ni = bp ? ii[j - 1] : (bc ? id : ii[j]);
                                dd[j] = nd; ii[j] = ni;
                            }
                            if (pair_less(d2, id, dd[0], ii[0])) { dd[0] = d2; ii[0] = id; }
                        }
                    }
                }
            }
            if (need && in_range) atomicAdd(a.counters + 3, 1u);
            dK2 = kth();
        }
        int nfound = 0;
#pragma unroll
        for (int j = 0; j < KM; ++j) nfound += (ii[j] != SENT) ? 1 : 0;
        if (!(in_range && live)) continue;
        float m = INFINITY;
        {
            const int gx0 = sx0 + rx0, gx1 = sx0 + rx1, gy0 = sy0 + ry0, gy1 = sy0 + ry1;
            const int gz0 = sz0 + rz0, gz1 = sz0 + rz1;
            if (gx0 > 0) m = fminf(m, qx - (g.origin[0] + gx0 * g.cell[0]));
            if (gx1 < a.X - 1) m = fminf(m, g.origin[0] + (gx1 + 1) * g.cell[0] - qx);
            if (gy0 > 0) m = fminf(m, qy - (g.origin[1] + gy0 * g.cell[1]));
            if (gy1 < a.Y - 1) m = fminf(m, g.origin[1] + (gy1 + 1) * g.cell[1] - qy);
            if (gz0 > 0) m = fminf(m, qz - (g.origin[2] + gz0 * g.cell[2]));
            if (gz1 < a.Z - 1) m = fminf(m, g.origin[2] + (gz1 + 1) * g.cell[2] - qz);
            m = fminf(m, complete_margin3(a.complete, qx, qy, qz));
            m -= g.eps;
        }
        const bool geo_ok = (nfound >= k) && (m > 0.f) && (m == INFINITY || dK2 <= m * m);
        if (geo_ok) {
            const size_t row = (size_t)w_row(a, qorig, qsidx) * (size_t)k;
#pragma unroll
            for (int j = 0; j < KM; ++j) {
                if (j < k) {
                    const size_t o = KN_IDX(row + j, (size_t)a.n_queries * k, 228);
                    o_idx[o] = out_id(a, ii[j]);
                    if (o_dist) o_dist[o] = dd[j];
                }
            }
        } else {
            const unsigned p = atomicAdd(a.counters + 0, 1u);
            a.fallback_list[KN_IDX(p, (unsigned)a.n, 230)] = qsidx;
        }
    }
}

struct ExactArgs {
    const float4* sorted;
    const int* cell_start;
    const GridGeom* geom;
    int n;
    int X, Y, Z;
    int k;
    int n_queries;
    int q_lo;                // local mode: queries are original indices [q_lo, n_queries), row = w - q_lo
    const unsigned* id_map;
    const unsigned* row_of;
    CompleteBox complete;
    unsigned* out_idx;
    float* out_dist;
    unsigned* const* out_idx_ref;
    float* const* out_dist_ref;
    const unsigned* list;      // stored indices (nullptr: all stored points)
    const unsigned* list_count;
    unsigned* counters;        // [1] uncertified count
    unsigned* uncert_list;     // optional: original indices of uncertified queries
    const float4* ext;         // external queries {x, y, z, bits(global id)} (nullptr: stored points)
    int n_ext;
    // 2: slot layout of the multi-GPU forwarding (launch_query_external_slots): query t is
    // ext[2t] = {x, y, z, bits(gid)} and ext[2t + 1].x its origin's K-th squared distance (an
    // upper bound: seeds the threshold); gid 0xFFFFFFFF = empty slot, skipped
    int ext_stride;
    // deferred distributed steps: the step check run by the last workgroup (kn/step_flag.h); a
    // DEVICE pointer (the job's fields as kernel arguments pushed the kernel past its SGPR budget
    // into scratch)
    const StepFlagJob* fjp = nullptr;
    int has_fj = 0;
};

// ---- wave-per-query exact kernel: threshold compaction + wave bitonic sort (any K <= 128) ----
// One wave serves one query of the fallback list (or every query without tiles). It walks the
// query's Chebyshev shells of cells; candidates are tested 64 at a time (dense shells: a row's
// points dealt to the lanes; sparse shells: one row per lane) and every candidate with
// d2 <= thr is appended to a per-wave LDS buffer by ballot compaction. When the buffer could
// overflow, and after each shell once K candidates are held, the wave bitonic-sorts the buffer
// by (d2 bits, id), keeps the first K and lowers thr to the K-th distance, so the buffer stays
// small however dense the cells are (clustered clouds). A shell ends the walk once the K-th
// distance lies inside the scanned block. Registers hold 4 keys per lane for any K, instead of
// a per-lane K-entry (d2, id) list (K=50: 256 VGPRs plus scratch in the round-1 kernel).
constexpr int kXCap = 256;
// Workgroups of the fallback launch (4 query waves each). The list length is only known on the
// device, so the grid is fixed: enough waves to hide the walk's load latency when the list is
// long (clustered clouds) at a small fixed cost when it is empty.
#ifndef KN_EXACT_GRID
#define KN_EXACT_GRID 1024
#endif  // per-wave candidate buffer (u64 keys); >= K + 64 for K <= 128
__global__ __launch_bounds__(256) void knn_exact_coop_kernel(ExactArgs a) {
    // output pointers: the launch's, or read from device slots (graph replays of a batched
    // stream of clouds); locals, so the kernel argument block stays read-only
    out_u32_t* const o_idx = out_ptr(a.out_idx_ref ? *a.out_idx_ref : a.out_idx);
    out_f32_t* const o_dist = out_ptr(a.out_idx_ref ? (a.out_dist_ref ? *a.out_dist_ref : nullptr) : a.out_dist);
    __shared__ unsigned long long s_buf[4][kXCap];
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    unsigned long long* buf = s_buf[wid];
    const unsigned long long lt = (lane == 0) ? 0ull : (~0ull >> (64 - lane));
    const GridGeom g = *a.geom;
    const int total = a.ext ? a.n_ext : (a.list ? (int)*a.list_count : a.n);
    const int k = a.k;
    for (int t = blockIdx.x * 4 + wid; t < total; t += gridDim.x * 4) {
        // external queries (multi-GPU forwarding): a point of another rank, self = same global id
        const unsigned entry = a.ext ? ~0u : (unsigned)__builtin_amdgcn_readfirstlane(
            (int)(a.list ? a.list[KN_IDX(t, a.n, 311)] : (unsigned)t));
        const bool seeded = !a.ext && a.list && (entry & kSeedBit) && o_dist;
        const unsigned sidx = a.ext ? ~0u : (entry & ~kSeedBit);
        const float4 qp = a.ext ? a.ext[(size_t)t * a.ext_stride] : a.sorted[KN_IDX(sidx, (unsigned)a.n, 312)];
        const unsigned qw = __float_as_uint(qp.w);
        if (!a.ext && !w_live(a, qw)) continue;
        if (a.ext && a.ext_stride == 2 && qw == SENT) continue;  // empty forwarding slot
        const unsigned qorig = a.ext ? (unsigned)t : w_row(a, qw, sidx);
        const unsigned qid = a.ext ? w_id(a, qw) : ~0u;
        const float qx = qp.x, qy = qp.y, qz = qp.z;
        const int cx = cell_coord(g, 0, qx), cy = cell_coord(g, 1, qy), cz = cell_coord(g, 2, qz);
        int cnt = 0;            // keys in buf (uniform)
        float thr = INFINITY;   // current K-th distance bound (uniform)
        if (a.ext && a.ext_stride == 2) {
            // forwarded query: only points within the origin's K-th distance can improve its row
            const float s0 = a.ext[(size_t)t * 2 + 1].x;
            if (s0 >= 0.f && s0 < INFINITY) thr = s0;
        }
        if (seeded) {
            // the tile kernel's K-th distance for this row (K real points within it): every true
            // neighbour passes d2 <= thr from the first shell on, rows are cut by the ball at once
            const float s0 = __int_as_float(__builtin_amdgcn_readfirstlane(__float_as_int(
                o_dist[KN_IDX((size_t)qorig * (size_t)k + (size_t)(k - 1), (size_t)a.n_queries * k, 317)])));
            if (s0 >= 0.f && s0 < INFINITY) thr = s0;
        }
        // sort buf[0, cnt), keep the first min(cnt, k), thr = K-th distance once K are held
        auto compact = [&]() __attribute__((always_inline)) {
            __builtin_amdgcn_wave_barrier();
            unsigned long long v[kXCap / 64];
#pragma unroll
            for (int e = 0; e < kXCap / 64; ++e) v[e] = (64 * e + lane < cnt) ? buf[64 * e + lane] : ~0ull;
            __builtin_amdgcn_wave_barrier();
            wave_bitonic_sort_u64<kXCap / 64>(v, lane);
#pragma unroll
            for (int e = 0; e < kXCap / 64; ++e)
                if (64 * e + lane < k) buf[64 * e + lane] = v[e];
            cnt = min(cnt, k);
            if (cnt >= k) {
                unsigned hb = 0;
#pragma unroll
                for (int e = 0; e < kXCap / 64; ++e)
                    if ((k - 1) / 64 == e) hb = (unsigned)__builtin_amdgcn_readlane((int)(unsigned)(v[e] >> 32), (k - 1) & 63);
                thr = __uint_as_float(hb);
            }
            __builtin_amdgcn_wave_barrier();
        };
        // test one candidate per lane (p < 0: none) and append the passing ones
        auto offer = [&](int p) __attribute__((always_inline)) {
            if (cnt + 64 > kXCap) compact();
            bool pass = false;
            unsigned long long key = 0;
            if (p >= 0 && (unsigned)p != sidx) {
                const float4 c = a.sorted[KN_IDX(p, a.n, 313)];
                const float dx = c.x - qx, dy = c.y - qy, dz = c.z - qz;
                const float d2 = fmaf(dz, dz, fmaf(dy, dy, dx * dx));
                const unsigned cid = w_id(a, __float_as_uint(c.w));
                pass = d2 <= thr && cid != qid;
                key = pack_key64(d2, cid);
            }
            const unsigned long long bal = __builtin_amdgcn_ballot_w64(pass);
            if (pass) buf[cnt + __builtin_popcountll(bal & lt)] = key;
            cnt += __builtin_popcountll(bal);
        };
        const int rmax = max(max(max(cx, a.X - 1 - cx), max(cy, a.Y - 1 - cy)), max(cz, a.Z - 1 - cz));
        bool certified = false, sorted_now = false;
        bool dense = true;  // ring 0 is one row: candidate-parallel
        for (int r = 0; r <= rmax; ++r) {
            const int z0 = max(0, cz - r), z1 = min(a.Z - 1, cz + r);
            const int y0 = max(0, cy - r), y1 = min(a.Y - 1, cy + r);
            const int ny = y1 - y0 + 1, nrows = (z1 - z0 + 1) * ny;
            // stored range of part `part` of shell row `tr`: rows on the shell's y/z faces are
            // whole x-runs, interior rows contribute their two x-end cells
            auto seg = [&](int tr, int part, int& p0, int& p1) -> bool {
                const int z = z0 + tr / ny, y = y0 + tr % ny;
                const bool shell = (z == cz - r) || (z == cz + r) || (y == cy - r) || (y == cy + r);
                if (shell ? part == 1 : (r == 0 && part == 1)) return false;
                int xa, xb;
                if (shell) { xa = max(0, cx - r); xb = min(a.X - 1, cx + r); }
                else if (part == 0) { xa = cx - r; xb = cx - r; }
                else { xa = cx + r; xb = cx + r; }
                if (xa < 0 || xb > a.X - 1 || xa > xb) return false;
                if (thr != INFINITY) {
                    // only the cells of the row that reach into the current K-th ball (dense
                    // clusters: the ball is far smaller than a shell, most rows are skipped)
                    const float dyb = slab_dist(g, 1, qy, y, y), dzb = slab_dist(g, 2, qz, z, z);
                    const float dyz2 = fmaf(dyb, dyb, dzb * dzb);
                    if (!(dyz2 <= thr)) return false;
                    const float rr = sqrt_bound(thr - dyz2) * 1.000001f + g.eps;
                    xa = max(xa, cell_coord(g, 0, qx - rr));
                    xb = min(xb, cell_coord(g, 0, qx + rr));
                    if (xa > xb) return false;
                }
                const int rowc = (z * a.Y + y) * a.X;
                p0 = a.cell_start[KN_IDX(rowc + xa, a.X * a.Y * a.Z + 1, 314)];
                p1 = a.cell_start[KN_IDX(rowc + xb + 1, a.X * a.Y * a.Z + 1, 314)];
                return p0 < p1;
            };
            unsigned shell_pts = 0;
            if (dense) {
                for (int tr = 0; tr < nrows; ++tr)
                    for (int part = 0; part < 2; ++part) {
                        int p0, p1;
                        if (!seg(tr, part, p0, p1)) continue;
                        shell_pts += (unsigned)(p1 - p0);
                        for (int pb = p0; pb < p1; pb += 64) offer(pb + lane < p1 ? pb + lane : -1);
                    }
            } else {
                for (int tb = 0; tb < nrows; tb += 64) {
                    // one row per lane: walk its (up to two) segments, 64 candidates per step
                    int c0 = 0, c1 = 0, d0 = 0, d1 = 0;
                    if (tb + lane < nrows) {
                        if (!seg(tb + lane, 0, c0, c1)) c0 = c1 = 0;
                        if (!seg(tb + lane, 1, d0, d1)) d0 = d1 = 0;
                    }
                    shell_pts += (unsigned)((c1 - c0) + (d1 - d0));
                    while (__builtin_amdgcn_ballot_w64(c0 < c1 || d0 < d1)) {
                        int p = -1;
                        if (c0 < c1) p = c0++;
                        else if (d0 < d1) p = d0++;
                        offer(p);
                    }
                }
                shell_pts = wave_sum_u32(shell_pts);
            }
            if (dense) shell_pts = (unsigned)__builtin_amdgcn_readfirstlane((int)shell_pts);
            dense = shell_pts > 32u * (unsigned)nrows;  // the next shell is probably alike
            // stopping rule: distance from q to the outside of the scanned block
            float m = INFINITY;
            if (cx - r > 0) m = fminf(m, qx - (g.origin[0] + (cx - r) * g.cell[0]));
            if (cx + r < a.X - 1) m = fminf(m, g.origin[0] + (cx + r + 1) * g.cell[0] - qx);
            if (cy - r > 0) m = fminf(m, qy - (g.origin[1] + (cy - r) * g.cell[1]));
            if (cy + r < a.Y - 1) m = fminf(m, g.origin[1] + (cy + r + 1) * g.cell[1] - qy);
            if (cz - r > 0) m = fminf(m, qz - (g.origin[2] + (cz - r) * g.cell[2]));
            if (cz + r < a.Z - 1) m = fminf(m, g.origin[2] + (cz + r + 1) * g.cell[2] - qz);
            m -= g.eps;
            if (m == INFINITY) { compact(); sorted_now = true; certified = true; break; }
            if (cnt >= k) {
                compact();
                sorted_now = true;
                if (m > 0.f && thr <= m * m) { certified = true; break; }
            } else {
                sorted_now = false;
            }
        }
        if (!sorted_now) compact();
        // certification against the rank's complete box (multi-GPU); needs the K-th distance
        const float dk = (cnt < k) ? INFINITY : thr;
        const float mc = complete_margin3(a.complete, qx, qy, qz) - g.eps;
        const bool cert = certified && (mc == INFINITY || (mc > 0.f && dk <= mc * mc));
        if (!cert && lane == 0) {
            const unsigned pos = atomicAdd(a.counters + 1, 1u);
            if (a.uncert_list) a.uncert_list[KN_IDX(pos, (unsigned)a.n_queries, 316)] = qorig;
        }
        __builtin_amdgcn_wave_barrier();
        for (int j = lane; j < k; j += 64) {
            const size_t o = KN_IDX((size_t)qorig * (size_t)k + j, (size_t)a.n_queries * k, 315);
            const unsigned long long v = (j < cnt) ? buf[j] : ~0ull;
            const bool empty = (v == ~0ull);
            o_idx[o] = empty ? SENT : out_id(a, (unsigned)v);
            if (o_dist) o_dist[o] = empty ? INFINITY : __uint_as_float((unsigned)(v >> 32));
        }
        __builtin_amdgcn_wave_barrier();
    }
    if (a.has_fj) {
        const StepFlagJob& fj = *a.fjp;
        // last workgroup (device-scope ticket; every workgroup reaches this point: the query loop
        // has no early exit): the step check once every query of the step, tile and exact, has
        // counted its uncertified rows; then the ticket is reset for the next launch. Replaces two
        // one-block kernels on the query stream (flag partials + accumulate) that each waited for a
        // free CU slot beside the other query stream's tile kernel.
        // No release / acquire fences (on gfx950 an agent-scope fence writes back the L2, per
        // workgroup): the only value read across workgroups is counters[1], and every workgroup's
        // increments of it are RETURNING device-scope atomics, complete (vmcnt) before the barrier
        // that precedes its ticket; the last workgroup reads it with another atomic on the same
        // address (RMWs of one address are performed in one coherence order). The partials and
        // totals come from earlier kernels (stream order).
        __shared__ int last_s;
        __builtin_amdgcn_s_waitcnt(0);  // every wave's counter atomics returned (vmcnt = 0) ...
        __syncthreads();                // ... before workgroup thread 0 takes the ticket
        if (threadIdx.x == 0) last_s = atomicAdd(fj.ticket, 1u) == gridDim.x - 1 ? 1 : 0;
        __syncthreads();
        if (last_s) {
            const unsigned unc = atomicAdd(a.counters + 1, 0u);
            const int f = step_flag_eval(fj.partials, fj.nb, fj.stride, fj.n, fj.planned, fj.totals,
                                         fj.ptotals, fj.nt, unc);
            if (threadIdx.x == 0) {
                fj.flag[0] = f;
                atomicMax(fj.pending, f);
                __hip_atomic_store(fj.ticket, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            }
        }
    }
}

// Complete-box certification of finished rows (multi-GPU ranks on the tree path, whose kernels
// search the whole local point set): row r (= local point r) is certified when its K-th squared
// distance lies inside the rank's complete box margin; otherwise it is listed for the
// query-forwarding round (counters[1], uncert_list), as the grid kernels list theirs.
__global__ void certify_rows_kernel(const float* __restrict__ pts, int rows, int k, const float* __restrict__ out_dist,
                                    CompleteBox cb, const GridGeom* __restrict__ geom, unsigned* __restrict__ counters,
                                    unsigned* __restrict__ uncert_list) {
    const int r = blockIdx.x * blockDim.x + threadIdx.x;
    if (r >= rows) return;
    const float dk = out_dist[(size_t)r * k + (k - 1)];  // INFINITY when fewer than K were found
    const float x = pts[3 * (size_t)r], y = pts[3 * (size_t)r + 1], z = pts[3 * (size_t)r + 2];
    const float m = complete_margin3(cb, x, y, z) - geom->eps;
    const bool cert = (m == INFINITY) || (m > 0.f && dk <= m * m);
    if (!cert) {
        const unsigned pos = atomicAdd(counters + 1, 1u);
        uncert_list[KN_IDX(pos, (unsigned)rows, 318)] = (unsigned)r;
    }
}

__global__ void invert_perm_kernel(const unsigned* __restrict__ perm, int n, unsigned* __restrict__ inv) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) inv[perm[i]] = (unsigned)i;
}

__global__ void sorted_xyz_kernel(const float4* __restrict__ sorted, int n, float* __restrict__ xyz) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const float4 v = sorted[i];
    const size_t o = 3 * (size_t)i;
    xyz[o] = v.x;
    xyz[o + 1] = v.y;
    xyz[o + 2] = v.z;
}

__global__ void to_stored_kernel(const unsigned* __restrict__ out_orig, const unsigned* __restrict__ perm,
                                 const unsigned* __restrict__ inv, int n, int k,
                                 unsigned* __restrict__ out_sorted, const float* __restrict__ dist_orig,
                                 float* __restrict__ dist_sorted) {
    const size_t t = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= (size_t)n * k) return;
    const size_t i = t / k, j = t - i * k;
    const size_t src = (size_t)perm[i] * k + j;
    const unsigned v = out_orig[src];
    out_sorted[t] = (v == SENT) ? SENT : inv[v];
    if (dist_sorted) dist_sorted[t] = dist_orig[src];
}

inline unsigned cdiv(size_t a, size_t b) { return (unsigned)((a + b - 1) / b); }

// Query algorithm: flags bit 1 -> stream kernel, bit 2 -> LDS-staged tile kernel (union
// stream), bit 3 -> tile kernel (lane walk); none -> the process default (env KN_QUERY_ALGO =
// "tile" | "stream" | "lane", else the measured default: the lane walk for every K (900K
// uniform, MI355X: K=16 0.513 -> 0.331 ms, K=32 1.21 -> 0.95, K=64 4.01 -> 3.26,
// profiles/ab_r1_lane_walk.jsonl; K=50 2.27 -> 2.22 once the lane walk covers the whole staged
// block above K=40, profiles/ab_r1_lane_full.jsonl).
constexpr int kAlgoTile = 1, kAlgoStream = 2, kAlgoLane = 3;
inline int default_algo(int) { return kAlgoLane; }
inline int query_algo(int flags, int k) {
    if (flags & kQueryAlgoStream) return kAlgoStream;
    if (flags & kQueryAlgoTile) return kAlgoTile;
    if (flags & kQueryAlgoLane) return kAlgoLane;
    static const int def = [] {
        const char* e = std::getenv("KN_QUERY_ALGO");
        if (e && std::strcmp(e, "stream") == 0) return kAlgoStream;
        if (e && std::strcmp(e, "tile") == 0) return kAlgoTile;
        if (e && std::strcmp(e, "lane") == 0) return kAlgoLane;
        return 0;
    }();
    return def ? def : default_algo(k);
}

// Lane walk row order for halo H: the (2H+1)^2 offsets (oy, oz) sorted by expected squared
// distance from a query in the near half of its cell (offset m > 0 is the near side: expected
// gap m - 0.75 cells; m < 0: |m| - 0.25), ties by |oz|, |oy|, then value. Empty when > 128.
// ring = true: by Chebyshev ring max(|oy|, |oz|), then the centre-out z-slab / y order.
void row_order_table(int H, unsigned out[32], bool ring) {
    for (int i = 0; i < 32; ++i) out[i] = 0;
    const int side = 2 * H + 1;
    if (side * side > kRowOrderMax) return;
    struct E { double key; int oy, oz; };
    E e[kRowOrderMax];
    int n = 0;
    auto gap = [](int m) { return m > 0 ? m - 0.75 : (m < 0 ? -m - 0.25 : 0.0); };
    auto co = [](int m) { return m > 0 ? 2 * m - 1 : -2 * m; };  // centre-out rank 0, +1, -1, +2, ...
    for (int oz = -H; oz <= H; ++oz)
        for (int oy = -H; oy <= H; ++oy)
            e[n++] = {ring ? 1e4 * std::max(std::abs(oy), std::abs(oz)) + 100.0 * co(oz) + co(oy)
                           : gap(oy) * gap(oy) + gap(oz) * gap(oz), oy, oz};
    std::stable_sort(e, e + n, [](const E& u, const E& v) {
        if (u.key != v.key) return u.key < v.key;
        if (std::abs(u.oz) != std::abs(v.oz)) return std::abs(u.oz) < std::abs(v.oz);
        if (std::abs(u.oy) != std::abs(v.oy)) return std::abs(u.oy) < std::abs(v.oy);
        return u.oz != v.oz ? u.oz > v.oz : u.oy > v.oy;
    });
    for (int t = 0; t < n; ++t)
        out[t >> 2] |= (unsigned)((e[t].oy + 8) | ((e[t].oz + 8) << 4)) << ((t & 3) * 8);
}

template <int KT>
hipError_t launch_k(const QueryBuffers& q, hipStream_t s) {
    // margin slots beyond K: a query is lost to the exact path only if the K-th and (K+M)-th
    // distances collide within one truncation ulp (~2^-(23-SB)); M=3 makes that ~1e-7/query.
    // Round 4 gave the lane-walk kernel (the default) M = 1 above K = 32: at K = 50 one slot less
    // per candidate outweighed the 3x longer exact list then (900K uniform: 0.967 -> 0.884
    // ms/step, 110 -> 360 exact queries; profiles/ab_r4_tiles_margin.txt); at K = 16 M = 1 loses,
    // 0.294 -> 0.329. The union-stream and staging-free kernels keep M = 2 (the stream kernel's
    // rows differ from the oracle with M = 1 at K = 50). KN_TOPK_MARGIN=m forces m for the lane walk.
#ifndef KN_TOPK_MARGIN
#define KN_TOPK_MARGIN -1
#endif
    constexpr int M = 2;
    // Round 5: with two query streams the longer exact list of M = 1 no longer pays for the slot
    // it saves: M = 2 at K = 50 0.748 -> 0.736 ms (110 instead of 360 exact queries), K = 64
    // 0.949 -> 0.917 (profiles/ab_r5_k50.txt)
    constexpr int ML = KN_TOPK_MARGIN >= 0 ? KN_TOPK_MARGIN : 2;
    const int X = q.dims[0], Y = q.dims[1], Z = q.dims[2];
    hipError_t e = hipSuccess;
    if (q.exact_mode != 2 && !q.counters_zeroed &&
        (e = hipMemsetAsync(q.counters, 0, kNumCounters * sizeof(unsigned), s)) != hipSuccess)
        return e;
    if (q.n == 0 || q.n_queries <= q.q_lo) return hipSuccess;
    // the register-resident tile path covers K <= 64; larger K use the exact ring walk
    const bool tiles = q.use_tiles && KT <= 64;
    if (!tiles && q.exact_mode == 2) return hipSuccess;  // the exact kernel served every query already
    if (tiles && q.exact_mode != 2) {
        TileArgs a;
        a.sorted = q.sorted; a.cell_start = q.cell_start; a.geom = q.geom; a.n = q.n;
        a.X = X; a.Y = Y; a.Z = Z; a.k = q.k; a.n_queries = q.n_queries; a.q_lo = q.q_lo; a.id_map = q.id_map;
        a.row_of = q.row_of;
        a.complete = q.complete; a.out_idx = q.out_idx; a.out_dist = q.out_dist;
        a.out_idx_ref = q.out_idx_ref; a.out_dist_ref = q.out_dist_ref;
        a.fallback_list = q.fallback_list; a.counters = q.counters;
        a.TX = q.tile[0]; a.TY = q.tile[1]; a.TZ = q.tile[2]; a.H = q.halo;
        a.Hx = x_halo(q.halo, q.xsub);
        a.cap = q.lds_capacity;
        a.flags = q.flags;
        {
            // the distance-sorted, mirrored table for the whole-block walk (K > 40), or the
            // outer-ring rows of the packed walk
            row_order_table(a.H, a.row_order, false);
            a.row_mirror = 1;
            a.n_outer = 0;
            if (outer_pack_k<KT>() && !(KN_ROW_ORDER == 1) && a.H >= 2 &&
                (2 * a.H + 1) * (2 * a.H + 1) - 9 <= 64) {
                // the distance-sorted table minus the 3x3 rows around the query's own row
                unsigned all[32];
                row_order_table(a.H, all, false);
                for (int i = 0; i < 32; ++i) a.row_order[i] = 0;
                const int nent = (2 * a.H + 1) * (2 * a.H + 1);
                for (int t = 0; t < nent; ++t) {
                    const unsigned e = (all[t >> 2] >> ((t & 3) * 8)) & 255u;
                    const int oy = (int)(e & 15u) - 8, oz = (int)(e >> 4) - 8;
                    if (std::max(std::abs(oy), std::abs(oz)) < 2) continue;
                    a.row_order[a.n_outer >> 2] |= e << ((a.n_outer & 3) * 8);
                    ++a.n_outer;
                }
            }
        }
        int sb = 0;
        while ((1 << sb) < q.lds_capacity) ++sb;
        a.slot_bits = sb;
        a.ntx = (X + a.TX - 1) / a.TX; a.nty = (Y + a.TY - 1) / a.TY; a.ntz = (Z + a.TZ - 1) / a.TZ;
        // workgroup order in blocks of tiles (tile_coords): 900K / 10M uniform, 200 / 30 / 100 steps,
        // two interleaved passes (profiles/ab_r5_tile_block.txt): 10M K=32 6.56 -> 6.37 ms (B 2 or
        // 4), K=50 0.777 -> 0.759 (B 4), K=16 within +-0.5 % for B 2 (+1 % for B 4).
        // KN_TILE_BLOCK=B overrides (1 = plain x-fastest order)
        static const int tblock_env = [] {
            const char* v = std::getenv("KN_TILE_BLOCK");
            return v ? std::max(1, std::atoi(v)) : 0;
        }();
        // round 5 (two query streams, three sets, 16K-point binning blocks): the K=32 bucket at 900K
        // runs fastest in plain order (0.451 -> 0.408 ms, two passes; K=24 / 50 / 64 and 10M keep
        // their blocks; profiles/ab_r5_tile_block.txt)
        // K <= 16 and K=32 by cloud size (gpurun_out/r5tb4, r5tb6, two passes, B 1 / 2 / 4): K=16
        // 300K 0.136 / 0.134 / 0.130 ms, 2M 0.594 / 0.575 / 0.565, 4M 1.35 / 1.30 / 1.22, 600K-900K
        // plain order by 0-1 % (900K 200 / 50 0.238 / 0.239 / 0.240); K=32 300K 0.246 / 0.264 /
        // 0.216, 4M 2.50 / 2.37 / 2.35; K=8 300K 0.096 / 0.094 / 0.087
        const bool mid = q.n >= (512 << 10) && q.n <= (1536 << 10);
        a.tblock = tblock_env ? tblock_env : ((KT <= 16 || KT == 32) && mid) ? 1 : 4;
        a.cb_stride = std::min(X, a.TX + 2 * a.Hx) + 1;
        a.max_rows = std::min(Y, a.TY + 2 * a.H) * std::min(Z, a.TZ + 2 * a.H);
        const unsigned nt = (unsigned)(a.ntx * a.nty * a.ntz);
        if (query_algo(q.flags, q.k) == kAlgoStream) {
            a.flags = q.flags & kQueryForceRescan;
            const size_t dyn = ((size_t)a.max_rows * a.cb_stride + (size_t)a.TY * a.TZ + 1) * sizeof(int);
            if constexpr (KT <= 64) knn_stream_kernel<KT, M><<<nt, kWG, dyn, s>>>(a);
        } else {
        // KN_LDS_EXTRA (bytes, diagnostics): pad the workgroup's LDS to measure how the query
        // kernel responds to fewer resident workgroups per CU
        static const size_t lds_extra = [] {
            const char* v = std::getenv("KN_LDS_EXTRA");
            return v ? (size_t)std::max(0, std::atoi(v)) : (size_t)0;
        }();
        const size_t lds = query_lds_bytes(q.tile, q.halo, q.lds_capacity, q.xsub) + lds_extra;
        static bool attr_set = false;
        if (!attr_set) {
            if constexpr (KT <= 64) {
                (void)hipFuncSetAttribute((const void*)knn_tile_kernel<KT, M, false>,
                                          hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
                (void)hipFuncSetAttribute((const void*)knn_tile_kernel<KT, ML, true>,
                                          hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
                (void)hipFuncSetAttribute((const void*)knn_tile_kernel<KT, ML, true, true>,
                                          hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
            }
            attr_set = true;
        }
        if constexpr (KT <= 64) {
            const bool wide = kWin2 > 0 && (q.flags & kQueryWide);
            if (query_algo(q.flags, q.k) != kAlgoLane) knn_tile_kernel<KT, M, false><<<nt, kWG, lds, s>>>(a);
            else if (wide) knn_tile_kernel<KT, ML, true, true><<<nt, kWG, lds, s>>>(a);
            else knn_tile_kernel<KT, ML, true><<<nt, kWG, lds, s>>>(a);
        }
        }
        if ((e = hipGetLastError()) != hipSuccess) return e;
        if (q.exact_mode == 1) return hipSuccess;
    }
    ExactArgs b;
    b.sorted = q.sorted; b.cell_start = q.cell_start; b.geom = q.geom; b.n = q.n;
    b.X = X; b.Y = Y; b.Z = Z; b.k = q.k; b.n_queries = q.n_queries; b.q_lo = q.q_lo; b.id_map = q.id_map;
    b.row_of = q.row_of;
    b.complete = q.complete; b.out_idx = q.out_idx; b.out_dist = q.out_dist;
    b.out_idx_ref = q.out_idx_ref; b.out_dist_ref = q.out_dist_ref;
    b.list = tiles ? q.fallback_list : nullptr;
    b.list_count = q.counters + 0;
    b.counters = q.counters;
    b.uncert_list = q.uncert_list;
    b.ext = nullptr;
    b.n_ext = 0;
    if (q.step_flag) {
        b.fjp = q.step_flag;
        b.has_fj = 1;
    }
    // one wave per query (threshold compaction, any K): 1024 waves for the fallback list
    const unsigned grid = tiles ? (unsigned)(q.exact_grid > 0 ? q.exact_grid : KN_EXACT_GRID)
                                : std::max(1u, std::min(cdiv(q.n, 4), 16384u));
    knn_exact_coop_kernel<<<grid, 256, 0, s>>>(b);
    return hipGetLastError();
}

}  // namespace

size_t query_lds_bytes(const int tile[3], int halo, int lds_capacity, int xsub) {
    const int rows = (tile[1] + 2 * halo) * (tile[2] + 2 * halo);
    const int cbs = tile[0] + 2 * x_halo(halo, xsub) + 1;
    size_t b = (size_t)lds_capacity * 16;
    b += ((size_t)rows * cbs * 2 + 3) & ~(size_t)3;  // u16 row-relative cell boundaries
    b += (size_t)(rows + 1) * 4;                      // rowbase
    b += (size_t)rows * 2 * 4;                        // rowst, rowend
    b += (size_t)(tile[1] * tile[2] + 1) * 4;
    b += 16;
    b = (b + 15) & ~(size_t)15;  // (cooperative re-scan buffers: the staged area's unused tail)
    return b;
}

KN_DEFINE_DEBUG_READER(debug_words_query)

hipError_t debug_phase_cycles(unsigned long long out[8], bool reset) {
#if KN_PHASES
    hipError_t e = hipMemcpyFromSymbol(out, HIP_SYMBOL(g_phase), sizeof(unsigned long long) * kPhN);
    if (e == hipSuccess && reset) {
        unsigned long long z[kPhN] = {0};
        e = hipMemcpyToSymbol(HIP_SYMBOL(g_phase), z, sizeof(z));
    }
    return e;
#else
    for (int i = 0; i < 8; ++i) out[i] = 0;
    (void)reset;
    return hipErrorNotSupported;
#endif
}

hipError_t launch_certify_rows(const float* pts, int rows, int k, const float* out_dist, const CompleteBox& cb,
                               const GridGeom* geom, unsigned* counters, unsigned* uncert_list, hipStream_t s) {
    if (rows < 0 || k < 1 || !out_dist) return hipErrorInvalidValue;
    if (rows > 0) certify_rows_kernel<<<cdiv(rows, 256), 256, 0, s>>>(pts, rows, k, out_dist, cb, geom, counters, uncert_list);
    return hipGetLastError();
}

hipError_t launch_query_external(const QueryBuffers& q, const float4* ext, int n_ext, hipStream_t s) {
    if (q.k <= 0 || q.k > 128 || n_ext < 0) return hipErrorInvalidValue;
    if (n_ext == 0) return hipSuccess;
    ExactArgs b{};
    b.sorted = q.sorted; b.cell_start = q.cell_start; b.geom = q.geom; b.n = q.n;
    b.X = q.dims[0]; b.Y = q.dims[1]; b.Z = q.dims[2]; b.k = q.k; b.n_queries = n_ext; b.q_lo = 0;
    b.id_map = q.id_map; b.row_of = q.row_of;
    for (int a = 0; a < 3; ++a) { b.complete.lo[a] = -INFINITY; b.complete.hi[a] = INFINITY; }
    b.out_idx = q.out_idx; b.out_dist = q.out_dist;
    b.list = nullptr; b.list_count = nullptr;
    b.counters = q.counters;
    b.uncert_list = nullptr;
    b.ext = ext;
    b.n_ext = n_ext;
    b.ext_stride = 1;
    knn_exact_coop_kernel<<<std::max(1u, std::min(cdiv((size_t)n_ext, 4), 16384u)), 256, 0, s>>>(b);
    return hipGetLastError();
}

hipError_t launch_query_external_slots(const QueryBuffers& q, const float4* slots, int n_slots, hipStream_t s) {
    if (q.k <= 0 || q.k > 128 || n_slots < 0) return hipErrorInvalidValue;
    if (n_slots == 0) return hipSuccess;
    ExactArgs b{};
    b.sorted = q.sorted; b.cell_start = q.cell_start; b.geom = q.geom; b.n = q.n;
    b.X = q.dims[0]; b.Y = q.dims[1]; b.Z = q.dims[2]; b.k = q.k; b.n_queries = n_slots; b.q_lo = 0;
    b.id_map = q.id_map; b.row_of = q.row_of;
    for (int a = 0; a < 3; ++a) { b.complete.lo[a] = -INFINITY; b.complete.hi[a] = INFINITY; }
    b.out_idx = q.out_idx; b.out_dist = q.out_dist;
    b.counters = q.counters;
    b.ext = slots;
    b.n_ext = n_slots;
    b.ext_stride = 2;
    // fixed grid (the number of filled slots is only known on the device); empty slots are skipped
    knn_exact_coop_kernel<<<std::max(1u, std::min(cdiv((size_t)n_slots, 4), 512u)), 256, 0, s>>>(b);
    return hipGetLastError();
}

hipError_t launch_query(const QueryBuffers& q, hipStream_t s) {
    const int k = q.k;
    if (k <= 0 || k > 128) return hipErrorInvalidValue;
    if (k <= 4) return launch_k<4>(q, s);
    if (k <= 8) return launch_k<8>(q, s);
    if (k <= 12) return launch_k<12>(q, s);
    if (k <= 16) return launch_k<16>(q, s);
    if (k <= 24) return launch_k<24>(q, s);
    if (k <= 32) return launch_k<32>(q, s);
    if (k <= 40) return launch_k<40>(q, s);
    if (k <= 50) return launch_k<50>(q, s);
    if (k <= 64) return launch_k<64>(q, s);
    if (k <= 96) return launch_k<96>(q, s);
    return launch_k<128>(q, s);
}

hipError_t launch_invert_perm(const unsigned* perm, int n, unsigned* inv, hipStream_t s) {
    if (n > 0) invert_perm_kernel<<<cdiv(n, 256), 256, 0, s>>>(perm, n, inv);
    return hipGetLastError();
}

hipError_t launch_sorted_xyz(const float4* sorted, int n, float* xyz, hipStream_t s) {
    if (n > 0) sorted_xyz_kernel<<<cdiv(n, 256), 256, 0, s>>>(sorted, n, xyz);
    return hipGetLastError();
}

hipError_t launch_to_stored_space(const unsigned* out_orig, const unsigned* perm, const unsigned* inv,
                                  int n, int k, unsigned* out_sorted, const float* dist_orig,
                                  float* dist_sorted, hipStream_t s) {
    const size_t tot = (size_t)n * k;
    if (tot > 0)
        to_stored_kernel<<<cdiv(tot, 256), 256, 0, s>>>(out_orig, perm, inv, n, k, out_sorted,
                                                        dist_orig, dist_sorted);
    return hipGetLastError();
}

// Expected staged points -> LDS slot capacity (multiple of 64, not necessarily a power of two:
// the key's slot field is ceil(log2(cap)) bits either way). The staged count of a tile is
// ~Poisson(staged) (sd = sqrt(staged)); staged + 5 sd + 64 makes an overflow (-> exact path)
// negligible for near-uniform clouds while keeping the 4x4x4/H2 plan at ~31 KB per workgroup,
// i.e. 5 workgroups (20 waves) per CU instead of 4 with a power-of-two 2048.
int lds_capacity_for(double staged) {
    // KN_LDS_SD: slack in standard deviations of the staged count (default 5; sweeps)
    static const double sd = [] {
        const char* v = std::getenv("KN_LDS_SD");
        return v ? std::max(0.0, std::atof(v)) : 5.0;
    }();
    double c = staged + sd * std::sqrt(std::max(staged, 1.0)) + 64.0;
    int cap = ((int)std::ceil(c) + 63) & ~63;
    return std::max(128, std::min(cap, 8192));
}

// Target density after whole-tile rounding. The reference uses 3.1 (knearests.cu:249). With the
// union-stream kernel (profiles/sweep_r1_tiles*.txt) K <= 40 was fastest at ~3.4 points/cell
// (64^3 for 900K: K=16 0.503 ms vs 0.542 at 68^3 and 0.635 at 60^3) and K=50 at ~2.9.
// Lane-walk density targets from sweeps on MI355X (profiles/sweep_r1_lane.txt,
// profiles/sweep_r1_lane_k32_k50.txt, profiles/sweep_r1_lane_k64.txt): 3.4 pts/cell with 4x4x4
// tiles for every tile-path K (<= 64); above K=40 with a 3-ring halo (K=50 at 900K 2.20 ->
// 1.96 ms; K=64 vs 2.9 pts/cell: 900K 3.26 -> 2.81 ms, 3M 9.43 -> 8.70). K=32 at 5.0 pts/cell
// with 4x4x2 tiles won at 900K (0.94 -> 0.79 ms) but lost at 3M (2.31 -> 2.66) and 10M
// (6.94 -> 8.01), so it is not the default. K > 64 (exact kernel only): 2.9.
float default_points_per_cell(int k) { return k <= 64 ? 3.4f : 2.9f; }

bool refine_dims(const int dims[3], double w, int k, float ppc, int n, int out[3], int xsub) {
    if (!(ppc > 0.f)) ppc = default_points_per_cell(k);
    const double wt = 1.0 + ppc / std::max(1, xsub);  // a Poisson grid at the target density
    if (!(w > 2.0 * wt) || n <= 0) return false;
    double f = std::cbrt(w / wt);
    // refined grids are isotropic (xsub 1): the x sub-cells serve the uniform tile path only
    const int xs = std::max(1, xsub);
    const int base[3] = {std::max(1, dims[0] / xs), dims[1], dims[2]};
    const double c0 = (double)base[0] * base[1] * base[2];
    const double cmax = std::min(4.0e8, std::max(16.0 * n, 1048576.0));  // cell_start <= 64 B/point
    if (c0 * f * f * f > cmax) f = std::cbrt(cmax / c0);
    if (f < 1.2) return false;
    for (int a = 0; a < 3; ++a) out[a] = std::max(4, (int)std::ceil(base[a] * f / 4.0) * 4);  // whole 4-cell tiles
    return true;
}

// Default x subdivision of the tile-path grid (AutoParams::xsub); KN_XSUB overrides.
int default_xsub(int k) {
    static const int env = [] {
        const char* v = std::getenv("KN_XSUB");
        return v ? std::max(1, std::min(4, std::atoi(v))) : 0;
    }();
    if (env) return env;
    return k <= KN_XSUB_MAX_K ? KN_DEFAULT_XSUB : 1;
}

double staged_points(const AutoParams& p, double ppc_cell) {
    return (double)(p.tile[0] + 2 * x_halo(p.halo, p.xsub)) * (p.tile[1] + 2 * p.halo) * (p.tile[2] + 2 * p.halo) *
           ppc_cell;
}

AutoParams auto_params(int n, int k, float ppc, const int* tile_hint, int halo_hint,
                       const float* extent, int xsub_hint) {
    AutoParams p;
    p.xsub = xsub_hint > 0 ? std::min(4, xsub_hint) : default_xsub(k);
    if (!(ppc > 0.f)) ppc = default_points_per_cell(k);
    const double cells = std::max(1.0, (double)n / ppc);
    for (int a = 0; a < 3; ++a) p.tile[a] = (tile_hint && tile_hint[a] > 0) ? tile_hint[a] : 4;
    double x[3];  // real-valued cells per axis
    if (extent && extent[0] > 0 && extent[1] > 0 && extent[2] > 0) {
        const double vol = (double)extent[0] * extent[1] * extent[2];
        const double h = std::cbrt(vol / cells);
        for (int a = 0; a < 3; ++a) x[a] = extent[a] / h;
    } else {
        x[0] = x[1] = x[2] = std::cbrt(cells);
    }
    // Small clouds: fewer 4^3 tiles than CUs leave most of the chip idle; 2^3 tiles give 8x the
    // workgroups (20K points, K=8: 0.049 -> 0.046 ms; at 300K 4^3 stays faster, 0.185 vs 0.197
    // for 4x4x2; profiles/sweep_r1_small.txt)
    // KN_HALF_TILE_MAX=T: 4x2x4 tiles below T 4^3 tiles (0 = never). Round 5
    // (bench.py, two passes, profiles/sweep_r5_tiles.txt): 200K 0.098 -> 0.093 ms, 300K 0.130 ->
    // 0.108, but 350K 0.101 -> 0.122 and 450K 0.126 -> 0.154. The per-query cost of the 4^3 plan
    // depends on the density after whole-tile rounding: 300K / 400K (3.5-3.6 points per cell)
    // 0.43 / 0.39 ns per query, 350K / 450K (3.2) 0.29 / 0.28; a power-of-two LDS capacity (11-bit
    // slot field) at 300K / 400K was neutral, so the cause is open.
    // Candidate default: T = 1,500 (~1.4 rounds of 1,024 workgroup slots): 200K (1,000 tiles) and
    // 300K (1,331) win, 350K / 400K (1,728) and 450K (2,197) lose or tie; not yet measured at
    // 100K-320K with bench.py (scripts/gpu/r5_half3.sh), so off by default.
    static const double half_max = [] {
        const char* v = std::getenv("KN_HALF_TILE_MAX");
        return v ? std::atof(v) : 0.0;
    }();
    const double tiles4 = std::ceil(x[0] / 4) * std::ceil(x[1] / 4) * std::ceil(x[2] / 4);
    if (!(tile_hint && (tile_hint[0] > 0 || tile_hint[1] > 0 || tile_hint[2] > 0))) {
        if (tiles4 < 256.0)
            for (int a = 0; a < 3; ++a) p.tile[a] = 2;
        else if (std::lround(x[0] / 4) * std::lround(x[1] / 4) * std::lround(x[2] / 4) < half_max)
            p.tile[1] = 2;  // (whole 4^3 tiles after rounding: 300K 11^3, 350K 12^3)
    }
    // Whole tiles: a partial edge tile costs a full halo staging for a fraction of the queries
    // (66 cells = 16.5 tiles of 4 -> 17 % of the tiles partial), so axes of >= 4 tiles are
    // rounded to a multiple of the tile edge (900K, K=16: 66^3 -> 64^3, solve 0.566 -> 0.505 ms).
    for (int a = 0; a < 3; ++a) {
        p.dims[a] = std::max(1, (int)std::lround(x[a]));
        if (x[a] >= 4.0 * p.tile[a]) p.dims[a] = std::max(p.tile[a], (int)std::lround(x[a] / p.tile[a]) * p.tile[a]);
    }
    // guard against int overflow of the cell count
    while ((double)p.dims[0] * p.dims[1] * p.dims[2] * p.xsub > 4.0e8)
        for (int a = 0; a < 3; ++a) p.dims[a] = std::max(1, p.dims[a] * 4 / 5);
    if (n > 0)  // the halo (K-th radius in cells) and the LDS plan follow the ACTUAL density
        ppc = (float)((double)n / ((double)p.dims[0] * p.dims[1] * p.dims[2]));
    // x sub-cells: same rows, xsub x the cell boundaries per row
    p.dims[0] *= p.xsub;
    p.tile[0] *= p.xsub;
    if (halo_hint > 0) {
        p.halo = halo_hint;
    } else {
        // K-th neighbour radius in cells for a uniform cloud: (3(K+1)/(4 pi ppc))^(1/3)
        const double rk = std::cbrt(3.0 * (k + 1) / (4.0 * M_PI * ppc));
        p.halo = std::max(1, (int)std::ceil(rk + 0.35));
        // 40 < K <= 64: the lane walk scans the whole staged block (KN_LANE_FULL), so 2 rings
        // certify all but the domain-boundary queries, which the exact kernel finishes; 2 rings
        // keep the workgroup at ~40 KB of LDS (4 per CU) where 3 rings took 70 KB (2 per CU).
        // 900K uniform: K=50 1.31 -> 0.95 ms, K=64 1.68 -> 1.33 ms (profiles/ab_r2_exact.log)
        if (k > 40 && k <= 64) p.halo = std::min(p.halo, 2);
    }
    p.lds_capacity = lds_capacity_for(staged_points(p, ppc / p.xsub));
    p.lds_bytes = query_lds_bytes(p.tile, p.halo, p.lds_capacity, p.xsub);
    return p;
}

}  // namespace kn
