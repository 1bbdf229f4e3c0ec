// multi.cpp -- single-process multi-GPU solve through the C API (kn_prepare_multi & co).
//
// NEW component (the reference is single-GPU, knearests.cu). The same algorithm as the Python
// DistributedKNearests (cuda_knearests_amd/parallel/distributed.py), driven from one host
// thread over R ranks, each bound to a HIP device:
//   1. rank r holds a contiguous chunk of the input (global id = chunk offset + index);
//   2. local metas (launch_local_meta) -> the host -> global domain and px*py*pz rank grid;
//   3. count-balanced boxes (default): three histogram stages on every rank
//      (launch_split_hist: x; y per x slab; z per column), summed on the host, quantile edges
//      (split_edges, the arithmetic of parallel/decomposition.py balanced_splits);
//   4. device plan of every rank (launch_route_plan: halo width, rank boxes) + per-destination
//      (owned, halo) counts (launch_route_count) -> the host learns the split sizes -> send
//      buffers (launch_route_scatter, destination order);
//   5. ONE exchange of rows between every pair of ranks: RCCL grouped ncclSend / ncclRecv over
//      one communicator per device (ncclCommInitAll) when the ranks' devices are all distinct,
//      device-to-device copies otherwise (several virtual ranks on one GPU: lets the whole path
//      run on a 1-GPU box);
//   6. per rank: unpack (owned first), grid build over the rank box grown by the send halo,
//      global-id stored points, certified queries of the owned points (complete box);
//   7. uncertified queries (K-th neighbour reaches past the halo): query forwarding (default) --
//      launch_fwd_pack puts each into a slot per rank whose box its K-th sphere reaches, one
//      equal-split exchange, launch_query_external_slots answers on the destination's grid, one
//      exchange back, launch_fwd_merge -- or, with forwarding off, a halo-doubling round;
//   8. rows are gathered to the host in original order.
// Every device buffer is persistent and grow-only (DBuf): a repeated solve of the same cloud
// (or of kn_update_multi coordinates of similar extent) makes no device allocation
// (kn_multi_stats::device_allocations). Everything runs on per-rank streams; the host
// synchronises at the meta, split-histogram, count, certification and result copies.
#include <hip/hip_runtime.h>

#include "hostio.hpp"

#include <algorithm>
#include <array>
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <functional>
#include <limits>
#include <string>
#include <vector>

#ifdef KN_HAVE_RCCL
#include <rccl/rccl.h>
#endif

#include "knearests.h"
#include "kn/kernels.h"
#include "kn/route.h"

extern "C" void kn_set_last_error_internal(const char* msg);

namespace {

// Grow-only device buffer (bytes); reallocated only when a solve needs more.
struct DBuf {
    void* p = nullptr;
    size_t cap = 0;
    template <class T>
    T* as() const { return static_cast<T*>(p); }
};

constexpr int kMaxSplits = (kn::kRouteMaxWorld + 1) + 4 * kn::kRouteMaxWorld;

struct RankState {
    int dev = 0;
    hipStream_t s = nullptr;
    int n = 0;  // points of the share
    // persistent small buffers
    DBuf pts, words, meta, metas, plan, hdr, bc, totals, splits, hist, hist_scratch, geom, counters, fcounters,
        fstat, fcnt;
    // per-solve buffers (grow-only)
    DBuf send, recv, lpts, lgids, ws, cell_start, sorted, perm, out_idx, out_dist, fallback, uncert;
    DBuf fsend, frecv, slot_row, slot_of, aidx, ad2, bidx, bd2;
    // host view of the current round
    std::array<double, kn::kPlanHdr> hdr_host{};
    std::vector<int> tot;  // 2 * world: (owned, halo) rows to each destination
    int nl = 0, n_owned = 0;
    int dims[3] = {1, 1, 1};
    unsigned unc = 0;  // uncertified queries of the round
};

// Balanced 3-factorisation of world (minimum rank-box surface, ties within 1 % resolved in a
// fixed order) -- parallel/decomposition.py factor3.
void factor3(int world, const double ext[3], int out[3]) {
    double best = std::numeric_limits<double>::infinity();
    std::vector<std::pair<std::array<int, 3>, double>> c;
    for (int a = 1; a <= world; ++a) {
        if (world % a) continue;
        for (int b = 1; b <= world / a; ++b) {
            if ((world / a) % b) continue;
            const int d = world / a / b;
            const double bx = ext[0] / a, by = ext[1] / b, bz = ext[2] / d;
            const double cost = bx * by + by * bz + bx * bz;
            c.push_back({{a, b, d}, cost});
            best = std::min(best, cost);
        }
    }
    for (auto& e : c)
        if (e.second <= best * (1.0 + 1e-2)) { out[0] = e.first[0]; out[1] = e.first[1]; out[2] = e.first[2]; return; }
}

// Quantile edges of each row of `hist` (rows x kSplitBins counts) -> rows x (parts + 1) floats:
// first = lo, last = hi, inner edges at the upper edge of the bin holding the j/parts quantile
// (decomposition.py _edges: t = ceil(tot j / parts), first bin whose cumulative count >= t).
std::vector<float> split_edges(const std::vector<unsigned long long>& hist, int rows, int parts, double lo, double hi) {
    constexpr int B = kn::kSplitBins;
    std::vector<float> out((size_t)rows * (parts + 1));
    std::vector<long long> cs(B);
    for (int r = 0; r < rows; ++r) {
        long long run = 0;
        for (int b = 0; b < B; ++b) cs[b] = run += (long long)hist[(size_t)r * B + b];
        const long long tot = cs[B - 1];
        float* o = &out[(size_t)r * (parts + 1)];
        o[0] = (float)lo;
        for (int j = 1; j < parts; ++j) {
            const long long t = (tot * j + parts - 1) / parts;
            const long long b = std::lower_bound(cs.begin(), cs.end(), t) - cs.begin();
            double inner = lo + ((double)b + 1.0) * (hi - lo) / B;
            inner = std::min(std::max(inner, lo), hi);
            o[j] = (float)inner;
        }
        o[parts] = (float)hi;
    }
    return out;
}

}  // namespace

struct kn_multi {
    std::vector<RankState> r;
    int n = 0;
    kn_config cfg{};
    kn_multi_options opt{};
    bool rccl = false;
    // last solve
    int rounds = 0, halo_points = 0, forwarded = 0, allocations = 0;
    bool balanced = false;
    float ms_total = 0.f;
    std::vector<unsigned> idx;
    std::vector<float> dist;
    bool solved = false;
    int host_syncs = 0;
    // plan reuse: the count-balanced kd splits of the last solve stay valid while every rank's
    // meta (bbox, count) is unchanged -- a repeated solve skips the split histograms' syncs
    std::vector<double> plan_metas;
    bool splits_valid = false;
#ifdef KN_HAVE_RCCL
    std::vector<ncclComm_t> comms;
#endif
    std::string err;
};

namespace {

#define KN_M(expr)                                                                      \
    do {                                                                                \
        hipError_t e_ = (expr);                                                         \
        if (e_ != hipSuccess) {                                                         \
            m->err = std::string(#expr) + ": " + hipGetErrorString(e_);                 \
            return KN_ERR_DEVICE;                                                       \
        }                                                                               \
    } while (0)
#define KN_TRY(expr)                           \
    do {                                       \
        const kn_status st_ = (expr);          \
        if (st_ != KN_OK) return st_;          \
    } while (0)

// Grows `b` to at least `bytes` (the caller has selected the rank's device). 1/8 headroom so
// that a slightly larger halo on the next solve does not reallocate.
hipError_t ensure(kn_multi* m, DBuf& b, size_t bytes) {
    bytes = std::max<size_t>(bytes, 16);
    if (b.cap >= bytes) return hipSuccess;
    if (b.p) (void)hipFree(b.p);
    b.p = nullptr;
    b.cap = 0;
    const size_t want = bytes + bytes / 8;
    hipError_t e = kn::device_malloc(&b.p, want);
    if (e != hipSuccess) return e;
    b.cap = want;
    ++m->allocations;
    return hipSuccess;
}
template <class T>
hipError_t ensure_n(kn_multi* m, DBuf& b, size_t count) { return ensure(m, b, count * sizeof(T)); }

void free_buf(DBuf& b) {
    if (b.p) (void)hipFree(b.p);
    b = DBuf{};
}

kn_status sync_all(kn_multi* m) {
    for (auto& R : m->r) { KN_M(hipSetDevice(R.dev)); KN_M(hipStreamSynchronize(R.s)); }
    ++m->host_syncs;
    return KN_OK;
}

// One transfer per ordered pair (s -> d), s == d included (a local device copy).
struct Xfer {
    const void* src;
    void* dst;
    size_t bytes;
};

// All pairs' transfers of one exchange: RCCL grouped send/recv (distinct devices) or device
// copies issued on the destination's stream after every source's stream has drained.
kn_status exchange(kn_multi* m, const std::function<Xfer(int, int)>& f) {
    const int W = (int)m->r.size();
    if (m->rccl) {
#ifdef KN_HAVE_RCCL
        if (ncclGroupStart() != ncclSuccess) { m->err = "ncclGroupStart failed"; return KN_ERR_DEVICE; }
        for (int i = 0; i < W; ++i) {
            RankState& R = m->r[i];
            for (int p = 0; p < W; ++p) {
                const Xfer out = f(i, p), in = f(p, i);
                if (p == i) {
                    if (out.bytes && hipMemcpyAsync(out.dst, out.src, out.bytes, hipMemcpyDeviceToDevice, R.s) != hipSuccess) {
                        (void)ncclGroupEnd();
                        m->err = "local copy failed";
                        return KN_ERR_DEVICE;
                    }
                    continue;
                }
                if ((out.bytes && ncclSend(out.src, out.bytes, ncclChar, p, m->comms[i], R.s) != ncclSuccess) ||
                    (in.bytes && ncclRecv(in.dst, in.bytes, ncclChar, p, m->comms[i], R.s) != ncclSuccess)) {
                    (void)ncclGroupEnd();
                    m->err = "ncclSend / ncclRecv failed";
                    return KN_ERR_DEVICE;
                }
            }
        }
        if (ncclGroupEnd() != ncclSuccess) { m->err = "ncclGroupEnd failed"; return KN_ERR_DEVICE; }
        return KN_OK;
#endif
    }
    KN_TRY(sync_all(m));  // every source buffer complete
    for (int d = 0; d < W; ++d) {
        RankState& D = m->r[d];
        KN_M(hipSetDevice(D.dev));
        for (int s = 0; s < W; ++s) {
            const Xfer x = f(s, d);
            if (x.bytes) KN_M(hipMemcpyPeerAsync(x.dst, D.dev, x.src, m->r[s].dev, x.bytes, D.s));
        }
    }
    return KN_OK;
}

// 2. metas -> global domain (lo, hi) and rank grid
kn_status phase_meta(kn_multi* m, double lo[3], double hi[3], int grid[3]) {
    const int W = (int)m->r.size();
    std::vector<double> metas((size_t)8 * W);
    for (int i = 0; i < W; ++i) {
        RankState& R = m->r[i];
        KN_M(hipSetDevice(R.dev));
        KN_M(kn::launch_local_meta(R.pts.as<float>(), R.n, R.words.as<unsigned>(), R.meta.as<double>(), R.s));
        KN_M(hipMemcpyAsync(&metas[(size_t)8 * i], R.meta.p, 8 * sizeof(double), hipMemcpyDeviceToHost, R.s));
    }
    KN_TRY(sync_all(m));
    if (metas != m->plan_metas) {  // a rank's bbox or count changed: the splits are re-planned
        m->plan_metas = metas;
        m->splits_valid = false;
    }
    for (int a = 0; a < 3; ++a) { lo[a] = INFINITY; hi[a] = -INFINITY; }
    for (int i = 0; i < W; ++i)
        for (int a = 0; a < 3; ++a) { lo[a] = std::min(lo[a], metas[8 * i + a]); hi[a] = std::max(hi[a], metas[8 * i + 3 + a]); }
    double ext[3];
    for (int a = 0; a < 3; ++a) {
        if (!std::isfinite(lo[a]) || !std::isfinite(hi[a])) { lo[a] = 0.0; hi[a] = 1.0; }  // empty cloud
        ext[a] = std::max(hi[a] - lo[a], 1e-30);
    }
    factor3(W, ext, grid);
    for (int i = 0; i < W; ++i) {
        RankState& R = m->r[i];
        KN_M(hipSetDevice(R.dev));
        KN_M(hipMemcpyAsync(R.metas.p, metas.data(), metas.size() * sizeof(double), hipMemcpyHostToDevice, R.s));
    }
    return KN_OK;
}

// 3. count-balanced kd splits -> every rank's `splits` buffer
kn_status phase_splits(kn_multi* m, const double lo[3], const double hi[3], const int grid[3]) {
    const int W = (int)m->r.size();
    constexpr int B = kn::kSplitBins;
    kn::SplitHistArgs a{};
    for (int d = 0; d < 3; ++d) {
        a.lo[d] = (float)lo[d];
        a.ext[d] = std::max((float)(hi[d] - lo[d]), 1e-30f);
        a.grid[d] = grid[d];
    }
    std::vector<float> e[3];
    const int parts[3] = {grid[0], grid[1], grid[2]};
    for (int stage = 0; stage < 3; ++stage) {
        a.stage = stage;
        const int rows = kn::split_hist_rows(grid, stage);
        if (parts[stage] == 1) {  // one part: the edges are the domain, no histogram needed
            e[stage].assign((size_t)rows * 2, 0.f);
            for (int r = 0; r < rows; ++r) { e[stage][2 * r] = (float)lo[stage]; e[stage][2 * r + 1] = (float)hi[stage]; }
        } else {
            std::vector<unsigned> h((size_t)W * rows * B);
            for (int i = 0; i < W; ++i) {
                RankState& R = m->r[i];
                KN_M(hipSetDevice(R.dev));
                KN_M(ensure_n<unsigned>(m, R.hist, (size_t)rows * B));
                KN_M(ensure_n<unsigned>(m, R.hist_scratch, kn::split_hist_scratch_words(R.n, grid, stage)));
                KN_M(kn::launch_split_hist(R.pts.as<float>(), R.n, a, R.hist.as<unsigned>(), R.hist_scratch.as<unsigned>(), R.s));
                KN_M(hipMemcpyAsync(&h[(size_t)i * rows * B], R.hist.p, (size_t)rows * B * sizeof(unsigned),
                                    hipMemcpyDeviceToHost, R.s));
            }
            KN_TRY(sync_all(m));
            std::vector<unsigned long long> sum((size_t)rows * B, 0ull);
            for (int i = 0; i < W; ++i)
                for (size_t j = 0; j < sum.size(); ++j) sum[j] += h[(size_t)i * rows * B + j];
            e[stage] = split_edges(sum, rows, parts[stage], lo[stage], hi[stage]);
        }
        if (stage == 0) std::copy(e[0].begin(), e[0].end(), a.xs);
        if (stage == 1) std::copy(e[1].begin(), e[1].end(), a.ys);
    }
    std::vector<float> all;
    for (auto& v : e) all.insert(all.end(), v.begin(), v.end());
    if ((int)all.size() != kn::route_split_count(grid)) { m->err = "split layout mismatch"; return KN_ERR_STATE; }
    for (int i = 0; i < W; ++i) {
        RankState& R = m->r[i];
        KN_M(hipSetDevice(R.dev));
        KN_M(hipMemcpyAsync(R.splits.p, all.data(), all.size() * sizeof(float), hipMemcpyHostToDevice, R.s));
    }
    return KN_OK;
}

// 4.-6. one routing round with halo factor hf: plan, counts, exchange, local solves; sets unc
kn_status solve_round(kn_multi* m, double hf, const int grid[3], bool balanced, bool* full) {
    const int W = (int)m->r.size();
    const int k = m->cfg.k;
    for (int i = 0; i < W; ++i) {
        RankState& R = m->r[i];
        KN_M(hipSetDevice(R.dev));
        // position-dependent halo: the interior width scales with the round's halo factor
        const double inner = kn::inner_halo_factor(k) * hf / std::max(1e-30, m->opt.halo_factor);
        KN_M(kn::launch_route_plan(R.metas.as<double>(), W, i, grid, k, hf, balanced ? R.splits.as<float>() : nullptr,
                                   R.plan.as<kn::RouteParams>(), R.hdr.as<double>(), R.s, inner));
        KN_M(kn::launch_route_count(R.pts.as<float>(), R.n, R.plan.as<kn::RouteParams>(), W, R.bc.as<int>(),
                                    R.totals.as<int>(), R.s));
        R.tot.assign((size_t)2 * W, 0);
        KN_M(hipMemcpyAsync(R.tot.data(), R.totals.p, 2 * W * sizeof(int), hipMemcpyDeviceToHost, R.s));
        KN_M(hipMemcpyAsync(R.hdr_host.data(), R.hdr.p, kn::kPlanHdr * sizeof(double), hipMemcpyDeviceToHost, R.s));
    }
    KN_TRY(sync_all(m));
    auto own = [&](int s, int d) { return m->r[s].tot[2 * d]; };
    auto halo = [&](int s, int d) { return m->r[s].tot[2 * d + 1]; };
    auto rows = [&](int s, int d) { return own(s, d) + halo(s, d); };
    *full = m->r[0].hdr_host[10] != 0.0;
    // send buffers (destination order) and receive buffers (source order)
    std::vector<std::vector<size_t>> soff(W, std::vector<size_t>(W + 1, 0)), roff(W, std::vector<size_t>(W + 1, 0));
    for (int i = 0; i < W; ++i) {
        for (int d = 0; d < W; ++d) {
            soff[i][d + 1] = soff[i][d] + (size_t)rows(i, d);
            roff[i][d + 1] = roff[i][d] + (size_t)rows(d, i);
        }
        RankState& R = m->r[i];
        KN_M(hipSetDevice(R.dev));
        KN_M(ensure_n<float4>(m, R.send, soff[i][W]));
        KN_M(ensure_n<float4>(m, R.recv, roff[i][W]));
        KN_M(kn::launch_route_scatter(R.pts.as<float>(), nullptr, R.n, R.plan.as<kn::RouteParams>(), W, R.bc.as<int>(),
                                      R.totals.as<int>(), R.send.as<float4>(), (int)soff[i][W], -1, R.s));
    }
    KN_TRY(exchange(m, [&](int s, int d) {
        return Xfer{m->r[s].send.as<float4>() + soff[s][d], m->r[d].recv.as<float4>() + roff[d][s],
                    (size_t)rows(s, d) * sizeof(float4)};
    }));
    // local solve on every rank
    m->halo_points = 0;
    for (int i = 0; i < W; ++i) {
        RankState& R = m->r[i];
        KN_M(hipSetDevice(R.dev));
        kn::UnpackTable t{};
        t.world = W;
        int seg = 0, no = 0, nh = 0;
        for (int s = 0; s < W; ++s) {
            t.seg[s] = seg;
            t.own[s] = own(s, i);
            t.own_pref[s] = no;
            t.halo_pref[s] = nh;
            seg += rows(s, i);
            no += own(s, i);
            nh += halo(s, i);
        }
        t.n_own = no;
        t.rows_cross = seg;
        t.self = -1;
        const int nl = seg, n_owned = no;
        R.nl = nl;
        R.n_owned = n_owned;
        m->halo_points += nh;
        KN_M(ensure_n<float>(m, R.lpts, (size_t)nl * 3));
        KN_M(ensure_n<int>(m, R.lgids, nl));
        KN_M(kn::launch_route_unpack(R.recv.as<float4>(), nullptr, nl, t, R.lpts.as<float>(), R.lgids.as<int>(), R.s));
        // rank box / complete box / local grid box from the plan header (kn::rank_local, shared
        // with the torch binding's dist_local)
        const kn::RankLocal rl = kn::rank_local(R.hdr_host.data(), i, grid);
        const double* box = rl.box;
        const kn::CompleteBox comp = rl.complete;
        const float* fext = rl.ext;
        const int th[3] = {m->cfg.tile[0], m->cfg.tile[1], m->cfg.tile[2]};
        const kn::AutoParams ap = kn::auto_params(nl, k, m->cfg.points_per_cell, th, m->cfg.halo, fext);
        for (int a = 0; a < 3; ++a) R.dims[a] = ap.dims[a];
        const int C = ap.dims[0] * ap.dims[1] * ap.dims[2];
        const size_t nb = kn::scan_block_count(C) + 1;
        size_t rank_off = kn::kBBoxWords + 16 + 2 * ((size_t)C + 1) + nb;
        rank_off = (rank_off + 3) & ~(size_t)3;
        KN_M(ensure_n<int>(m, R.ws, rank_off + 4 * (size_t)nl));
        KN_M(ensure_n<int>(m, R.cell_start, (size_t)C + 1));
        KN_M(ensure_n<float4>(m, R.sorted, nl));
        KN_M(ensure_n<unsigned>(m, R.perm, nl));
        KN_M(ensure_n<unsigned>(m, R.out_idx, (size_t)n_owned * k));
        KN_M(ensure_n<float>(m, R.out_dist, (size_t)n_owned * k));
        KN_M(ensure_n<unsigned>(m, R.fallback, nl));
        KN_M(ensure_n<unsigned>(m, R.uncert, n_owned));
        int* ws = R.ws.as<int>();
        kn::BuildBuffers b{};
        b.points = R.lpts.as<float>();
        b.n = nl;
        for (int a = 0; a < 3; ++a) b.dims[a] = ap.dims[a];
        b.bbox_words = reinterpret_cast<unsigned*>(ws);
        b.geom = R.geom.as<kn::GridGeom>();
        b.cell_count = ws + kn::kBBoxWords + 16;
        b.cell_scan = b.cell_count + (C + 1);
        b.block_sums = b.cell_scan + (C + 1);
        b.cell_rank = reinterpret_cast<int2*>(ws + rank_off);
        b.bin_tmp = reinterpret_cast<float4*>(ws + rank_off);
        b.cell_start = R.cell_start.as<int>();
        b.sorted = R.sorted.as<float4>();
        b.perm = R.perm.as<unsigned>();
        b.deterministic = m->cfg.deterministic;
        b.use_box = 1;
        for (int a = 0; a < 3; ++a) { b.box_lo[a] = (float)box[a]; b.box_hi[a] = (float)box[3 + a]; }
        KN_M(kn::launch_build(b, R.s));
        KN_M(kn::launch_global_w(R.sorted.as<float4>(), R.perm.as<unsigned>(), R.lgids.as<int>(), nl, n_owned, R.s));
        kn::QueryBuffers q{};
        q.sorted = R.sorted.as<float4>();
        q.cell_start = R.cell_start.as<int>();
        q.perm = R.perm.as<unsigned>();
        q.geom = R.geom.as<kn::GridGeom>();
        q.n = nl;
        for (int a = 0; a < 3; ++a) q.dims[a] = ap.dims[a];
        q.k = k;
        q.n_queries = n_owned;
        q.row_of = R.perm.as<unsigned>();
        q.complete = comp;
        q.out_idx = R.out_idx.as<unsigned>();
        q.out_dist = R.out_dist.as<float>();
        q.fallback_list = R.fallback.as<unsigned>();
        q.counters = R.counters.as<unsigned>();
        q.uncert_list = R.uncert.as<unsigned>();
        for (int a = 0; a < 3; ++a) q.tile[a] = ap.tile[a];
        q.halo = ap.halo;
        q.xsub = ap.xsub;
        q.lds_capacity = ap.lds_capacity;
        q.use_tiles = m->cfg.exact_only ? 0 : 1;
        KN_M(kn::launch_query(q, R.s));
        R.unc = 0;
        KN_M(hipMemcpyAsync(&R.unc, R.counters.as<unsigned>() + 1, sizeof(unsigned), hipMemcpyDeviceToHost, R.s));
    }
    return sync_all(m);
}

// 7. query forwarding of the round's uncertified queries (exact: every rank whose box the
// query's K-th sphere reaches answers it from its grid)
kn_status forward(kn_multi* m) {
    const int W = (int)m->r.size();
    const int k = m->cfg.k;
    unsigned umax = 0;
    for (auto& R : m->r) umax = std::max(umax, R.unc);
    // slots per rank pair: a pair carries at most the source's uncertified count -> no overflow
    int F = 64;
    while ((unsigned)F < umax) F <<= 1;
    const size_t slots = (size_t)W * F;
    for (int i = 0; i < W; ++i) {
        RankState& R = m->r[i];
        KN_M(hipSetDevice(R.dev));
        KN_M(ensure_n<float4>(m, R.fsend, 2 * slots));
        KN_M(ensure_n<float4>(m, R.frecv, 2 * slots));
        KN_M(ensure_n<int>(m, R.slot_row, slots));
        KN_M(ensure_n<int>(m, R.slot_of, std::max<size_t>(1, (size_t)R.unc * W)));
        KN_M(ensure_n<int>(m, R.aidx, slots * k));
        KN_M(ensure_n<float>(m, R.ad2, slots * k));
        KN_M(ensure_n<int>(m, R.bidx, slots * k));
        KN_M(ensure_n<float>(m, R.bd2, slots * k));
        KN_M(hipMemsetAsync(R.fstat.p, 0, 2 * sizeof(unsigned), R.s));
        KN_M(kn::launch_fwd_pack(R.plan.as<kn::RouteParams>(), W, i, F, k, R.uncert.as<unsigned>(),
                                 R.counters.as<unsigned>() + 1, (int)R.unc, R.lpts.as<float>(), R.lgids.as<int>(),
                                 R.out_dist.as<float>(), R.fsend.as<float4>(), R.slot_row.as<int>(),
                                 R.slot_of.as<int>(), R.fcnt.as<int>(), R.fstat.as<unsigned>(), R.s));
    }
    const size_t slot_bytes = (size_t)F * 2 * sizeof(float4);
    KN_TRY(exchange(m, [&](int s, int d) {
        return Xfer{m->r[s].fsend.as<float4>() + (size_t)d * F * 2, m->r[d].frecv.as<float4>() + (size_t)s * F * 2,
                    slot_bytes};
    }));
    for (int i = 0; i < W; ++i) {
        RankState& R = m->r[i];
        KN_M(hipSetDevice(R.dev));
        KN_M(hipMemsetAsync(R.fcounters.p, 0, kn::kNumCounters * sizeof(unsigned), R.s));
        kn::QueryBuffers q{};
        q.sorted = R.sorted.as<float4>();
        q.cell_start = R.cell_start.as<int>();
        q.geom = R.geom.as<kn::GridGeom>();
        q.n = R.nl;
        for (int a = 0; a < 3; ++a) q.dims[a] = R.dims[a];
        q.k = k;
        q.row_of = R.perm.as<unsigned>();
        q.out_idx = R.aidx.as<unsigned>();
        q.out_dist = R.ad2.as<float>();
        q.counters = R.fcounters.as<unsigned>();
        KN_M(kn::launch_query_external_slots(q, R.frecv.as<float4>(), (int)slots, R.s));
    }
    const size_t ans = (size_t)F * k;
    KN_TRY(exchange(m, [&](int s, int d) {  // answers of rank s to rank d's queries
        return Xfer{m->r[s].aidx.as<int>() + (size_t)d * ans, m->r[d].bidx.as<int>() + (size_t)s * ans,
                    ans * sizeof(int)};
    }));
    KN_TRY(exchange(m, [&](int s, int d) {
        return Xfer{m->r[s].ad2.as<float>() + (size_t)d * ans, m->r[d].bd2.as<float>() + (size_t)s * ans,
                    ans * sizeof(float)};
    }));
    m->forwarded = 0;
    std::vector<std::array<unsigned, 2>> stat(W);
    for (int i = 0; i < W; ++i) {
        RankState& R = m->r[i];
        KN_M(hipSetDevice(R.dev));
        KN_M(kn::launch_fwd_merge(W, F, k, R.uncert.as<unsigned>(), R.counters.as<unsigned>() + 1, (int)R.unc,
                                  R.slot_of.as<int>(), R.bidx.as<int>(), R.bd2.as<float>(), R.out_idx.as<int>(),
                                  R.out_dist.as<float>(), R.s));
        KN_M(hipMemcpyAsync(stat[i].data(), R.fstat.p, 2 * sizeof(unsigned), hipMemcpyDeviceToHost, R.s));
        m->forwarded += (int)R.unc;
    }
    KN_TRY(sync_all(m));
    for (auto& s : stat)
        if (s[1]) { m->err = "forwarding slots overflowed"; return KN_ERR_STATE; }
    return KN_OK;
}

// 8. rows in original order
kn_status gather(kn_multi* m) {
    const int k = m->cfg.k;
    const int W = (int)m->r.size();
    m->idx.assign((size_t)m->n * k, 0xFFFFFFFFu);
    m->dist.assign((size_t)m->n * k, INFINITY);
    // every rank's rows copied back at once, ONE sync for all of them
    std::vector<std::vector<int>> g(W);
    std::vector<std::vector<unsigned>> ix(W);
    std::vector<std::vector<float>> ds(W);
    for (int i = 0; i < W; ++i) {
        RankState& R = m->r[i];
        KN_M(hipSetDevice(R.dev));
        const int n_owned = R.n_owned;
        g[i].resize(n_owned);
        ix[i].resize((size_t)n_owned * k);
        ds[i].resize((size_t)n_owned * k);
        if (n_owned) {
            KN_M(hipMemcpyAsync(g[i].data(), R.lgids.p, n_owned * sizeof(int), hipMemcpyDeviceToHost, R.s));
            KN_M(hipMemcpyAsync(ix[i].data(), R.out_idx.p, ix[i].size() * sizeof(unsigned), hipMemcpyDeviceToHost, R.s));
            KN_M(hipMemcpyAsync(ds[i].data(), R.out_dist.p, ds[i].size() * sizeof(float), hipMemcpyDeviceToHost, R.s));
        }
    }
    KN_TRY(sync_all(m));
    for (int i = 0; i < W; ++i) {
        for (int j = 0; j < m->r[i].n_owned; ++j) {
            if (g[i][j] < 0 || g[i][j] >= m->n) { m->err = "global id out of range"; return KN_ERR_DEVICE; }
            const size_t dst = (size_t)g[i][j] * k;
            std::memcpy(&m->idx[dst], &ix[i][(size_t)j * k], k * sizeof(unsigned));
            std::memcpy(&m->dist[dst], &ds[i][(size_t)j * k], k * sizeof(float));
        }
    }
    return KN_OK;
}

kn_status solve(kn_multi* m) {
    const int W = (int)m->r.size();
    double lo[3], hi[3];
    int grid[3];
    m->host_syncs = 0;
    KN_TRY(phase_meta(m, lo, hi, grid));
    m->balanced = m->opt.balance != 0 && W > 1 && grid[0] * grid[1] <= kn::kRouteMaxWorld;
    if (m->balanced && !m->splits_valid) {
        KN_TRY(phase_splits(m, lo, hi, grid));
        m->splits_valid = true;  // the ranks' `splits` buffers hold them until a meta changes
    }
    double hf = m->opt.halo_factor;
    m->forwarded = 0;
    for (int round = 0; round < m->opt.max_rounds; ++round) {
        bool full = false;
        KN_TRY(solve_round(m, hf, grid, m->balanced, &full));
        m->rounds = round + 1;
        unsigned unc = 0;
        for (auto& R : m->r) unc += R.unc;
        if (unc == 0 || full) return gather(m);
        if (m->opt.forward) {
            KN_TRY(forward(m));
            return gather(m);
        }
        hf *= 2.0;  // uncertified queries: grow the halo
    }
    m->err = "queries still uncertified after the maximum number of halo growth rounds";
    return KN_ERR_STATE;
}

}  // namespace

extern "C" {

kn_multi_options kn_default_multi_options(void) {
    kn_multi_options o{};
    o.halo_factor = 2.5;
    o.balance = 1;
    o.forward = 1;
    o.max_rounds = 8;
    return o;
}

kn_multi* kn_prepare_multi(const kn_float3* points, int numpoints, const int* devices, int ndevices,
                           const kn_config* cfg) {
    if (!points && numpoints > 0) { kn_set_last_error_internal("null points"); return nullptr; }
    if (numpoints < 0 || ndevices < 1 || ndevices > kn::kRouteMaxWorld) {
        kn_set_last_error_internal("bad point or device count (1..64 ranks)");
        return nullptr;
    }
    auto* m = new kn_multi();
    m->cfg = cfg ? *cfg : kn_default_config();
    m->opt = kn_default_multi_options();
    if (m->cfg.k <= 0) m->cfg.k = KN_DEFAULT_K;
    if (m->cfg.k > KN_MAX_K) { kn_set_last_error_internal("k out of range [1,128]"); delete m; return nullptr; }
    m->n = numpoints;
    std::vector<int> devs(ndevices);
    for (int i = 0; i < ndevices; ++i) devs[i] = devices ? devices[i] : i;
    bool distinct = true;
    for (int i = 0; i < ndevices; ++i)
        for (int j = 0; j < i; ++j) distinct = distinct && devs[i] != devs[j];
#ifdef KN_HAVE_RCCL
    m->rccl = distinct && std::getenv("KN_MULTI_COPY") == nullptr;
#else
    m->rccl = false;
#endif
    const float* src = reinterpret_cast<const float*>(points);
    m->r.resize(ndevices);
    for (int i = 0; i < ndevices; ++i) {
        RankState& R = m->r[i];
        R.dev = devs[i];
        const int a = (int)((long long)numpoints * i / ndevices), b = (int)((long long)numpoints * (i + 1) / ndevices);
        R.n = b - a;
        const int W = ndevices;
        bool ok = hipSetDevice(R.dev) == hipSuccess && hipStreamCreateWithFlags(&R.s, hipStreamNonBlocking) == hipSuccess &&
                  ensure_n<float>(m, R.pts, (size_t)R.n * 3) == hipSuccess &&
                  ensure_n<unsigned>(m, R.words, kn::kBBoxWords) == hipSuccess &&
                  ensure_n<double>(m, R.meta, 8) == hipSuccess && ensure_n<double>(m, R.metas, (size_t)8 * W) == hipSuccess &&
                  ensure_n<kn::RouteParams>(m, R.plan, 1) == hipSuccess &&
                  ensure_n<double>(m, R.hdr, kn::kPlanHdr) == hipSuccess &&
                  ensure_n<int>(m, R.bc, (size_t)2 * W * kn::route_block_count(R.n)) == hipSuccess &&
                  ensure_n<int>(m, R.totals, (size_t)2 * W) == hipSuccess &&
                  ensure_n<float>(m, R.splits, kMaxSplits) == hipSuccess &&
                  ensure_n<kn::GridGeom>(m, R.geom, 1) == hipSuccess &&
                  ensure_n<unsigned>(m, R.counters, kn::kNumCounters) == hipSuccess &&
                  ensure_n<unsigned>(m, R.fcounters, kn::kNumCounters) == hipSuccess &&
                  ensure_n<unsigned>(m, R.fstat, 2) == hipSuccess && ensure_n<int>(m, R.fcnt, W) == hipSuccess &&
                  (R.n == 0 || hipMemcpy(R.pts.p, src + (size_t)3 * a, (size_t)R.n * 12, hipMemcpyHostToDevice) == hipSuccess);
        if (!ok) {
            kn_set_last_error_internal("device allocation / upload failed");
            kn_free_multi(&m);
            return nullptr;
        }
    }
#ifdef KN_HAVE_RCCL
    if (m->rccl) {
        m->comms.resize(ndevices);
        if (ncclCommInitAll(m->comms.data(), ndevices, devs.data()) != ncclSuccess) {
            m->comms.clear();
            m->rccl = false;  // fall back to device copies
        }
    }
#endif
    return m;
}

kn_status kn_set_multi_options(kn_multi* m, const kn_multi_options* o) {
    if (!m || !o) { kn_set_last_error_internal("null argument"); return KN_ERR_INVALID_ARGUMENT; }
    if (!(o->halo_factor > 0.0) || o->max_rounds < 1 || o->max_rounds > 64) {
        kn_set_last_error_internal("bad multi options (halo_factor > 0, max_rounds 1..64)");
        return KN_ERR_INVALID_ARGUMENT;
    }
    m->opt = *o;
    m->solved = false;
    return KN_OK;
}

kn_status kn_update_multi(kn_multi* m, const kn_float3* points) {
    if (!m || (!points && m->n > 0)) { kn_set_last_error_internal("null argument"); return KN_ERR_INVALID_ARGUMENT; }
    const float* src = reinterpret_cast<const float*>(points);
    const int W = (int)m->r.size();
    for (int i = 0; i < W; ++i) {
        RankState& R = m->r[i];
        const size_t a = (size_t)((long long)m->n * i / W);
        if (hipSetDevice(R.dev) != hipSuccess ||
            (R.n && hipMemcpyAsync(R.pts.p, src + 3 * a, (size_t)R.n * 12, hipMemcpyHostToDevice, R.s) != hipSuccess)) {
            kn_set_last_error_internal("point upload failed");
            return KN_ERR_DEVICE;
        }
    }
    for (auto& R : m->r)
        if (hipSetDevice(R.dev) != hipSuccess || hipStreamSynchronize(R.s) != hipSuccess) {
            kn_set_last_error_internal("point upload failed");
            return KN_ERR_DEVICE;
        }
    m->solved = false;
    return KN_OK;
}

kn_status kn_solve_multi(kn_multi* m) {
    if (!m) { kn_set_last_error_internal("null problem"); return KN_ERR_INVALID_ARGUMENT; }
    const auto t0 = std::chrono::steady_clock::now();
    m->allocations = 0;
    m->rounds = 0;
    m->solved = false;
    const kn_status st = solve(m);
    if (st != KN_OK) {
        (void)sync_all(m);  // no work of this solve left in flight
        kn_set_last_error_internal(m->err.c_str());
        return st;
    }
    m->ms_total = std::chrono::duration<float, std::milli>(std::chrono::steady_clock::now() - t0).count();
    m->solved = true;
    return KN_OK;
}

unsigned int* kn_get_neighbors_multi(kn_multi* m) {
    if (!m || !m->solved) { kn_set_last_error_internal("not solved"); return nullptr; }
    auto* out = static_cast<unsigned*>(std::malloc(std::max<size_t>(1, m->idx.size()) * sizeof(unsigned)));
    if (out && !m->idx.empty()) std::memcpy(out, m->idx.data(), m->idx.size() * sizeof(unsigned));
    return out;
}

float* kn_get_distances_multi(kn_multi* m) {
    if (!m || !m->solved) { kn_set_last_error_internal("not solved"); return nullptr; }
    auto* out = static_cast<float*>(std::malloc(std::max<size_t>(1, m->dist.size()) * sizeof(float)));
    if (out && !m->dist.empty()) std::memcpy(out, m->dist.data(), m->dist.size() * sizeof(float));
    return out;
}

kn_status kn_get_multi_info(kn_multi* m, int* ranks, int* rounds, int* halo_points, int* uses_rccl) {
    if (!m) { kn_set_last_error_internal("null problem"); return KN_ERR_INVALID_ARGUMENT; }
    if (ranks) *ranks = (int)m->r.size();
    if (rounds) *rounds = m->rounds;
    if (halo_points) *halo_points = m->halo_points;
    if (uses_rccl) *uses_rccl = m->rccl ? 1 : 0;
    return KN_OK;
}

kn_status kn_get_multi_stats(kn_multi* m, kn_multi_stats* out) {
    if (!m || !out) { kn_set_last_error_internal("null argument"); return KN_ERR_INVALID_ARGUMENT; }
    kn_multi_stats s{};
    s.ranks = (int)m->r.size();
    s.rounds = m->rounds;
    s.halo_points = m->halo_points;
    s.forwarded = m->forwarded;
    s.uses_rccl = m->rccl ? 1 : 0;
    s.balanced = m->balanced ? 1 : 0;
    s.min_owned = m->r.empty() ? 0 : INT32_MAX;
    s.max_owned = 0;
    for (auto& R : m->r) { s.min_owned = std::min(s.min_owned, R.n_owned); s.max_owned = std::max(s.max_owned, R.n_owned); }
    s.device_allocations = m->allocations;
    s.ms_total = m->ms_total;
    s.host_syncs = m->host_syncs;
    *out = s;
    return KN_OK;
}

void kn_free_multi(kn_multi** pm) {
    if (!pm || !*pm) return;
    kn_multi* m = *pm;
#ifdef KN_HAVE_RCCL
    for (auto& c : m->comms) (void)ncclCommDestroy(c);
#endif
    for (auto& R : m->r) {
        (void)hipSetDevice(R.dev);
        if (R.s) (void)hipStreamSynchronize(R.s);
        for (DBuf* b : {&R.pts, &R.words, &R.meta, &R.metas, &R.plan, &R.hdr, &R.bc, &R.totals, &R.splits, &R.hist,
                        &R.hist_scratch, &R.geom, &R.counters, &R.fcounters, &R.fstat, &R.fcnt, &R.send, &R.recv,
                        &R.lpts, &R.lgids, &R.ws, &R.cell_start, &R.sorted, &R.perm, &R.out_idx, &R.out_dist,
                        &R.fallback, &R.uncert, &R.fsend, &R.frecv, &R.slot_row, &R.slot_of, &R.aidx, &R.ad2,
                        &R.bidx, &R.bd2})
            free_buf(*b);
        if (R.s) (void)hipStreamDestroy(R.s);
    }
    delete m;
    *pm = nullptr;
}

}  // extern "C"
