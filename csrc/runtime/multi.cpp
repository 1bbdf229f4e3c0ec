// multi.cpp -- single-process multi-GPU solve through the C API (kn_prepare_multi & co).
//
// NEW component (the reference is single-GPU, knearests.cu). The same algorithm as the Python
// DistributedKNearests (cuda_knearests_amd/parallel/distributed.py), driven from one host
// thread over R ranks, each bound to a HIP device:
//   1. rank r holds a contiguous chunk of the input (global id = chunk offset + index);
//   2. local metas (launch_local_meta) -> gathered on the host -> device plan of every rank
//      (launch_route_plan: global domain, halo width, rank boxes of the px*py*pz split);
//   3. per-destination (owned, halo) counts (launch_route_count) -> the host learns the
//      split sizes -> send buffers (launch_route_scatter, destination order);
//   4. ONE exchange of rows between every pair of ranks: RCCL grouped ncclSend / ncclRecv
//      over one communicator per device (ncclCommInitAll) when the ranks' devices are all
//      distinct, device-to-device copies otherwise (several virtual ranks on one GPU: lets the
//      whole path run on a 1-GPU box);
//   5. per rank: unpack (owned first), grid build over the rank box grown by the send halo,
//      global-id stored points, certified queries of the owned points (complete box);
//   6. a rank with uncertified queries doubles the halo and the step repeats (growth round);
//   7. rows are gathered to the host in original order.
// Everything runs on per-rank streams; the host synchronises at the count and result copies.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <array>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
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

struct RankState {
    int dev = 0;
    hipStream_t s = nullptr;
    int n = 0;               // points of the share
    float* pts = nullptr;    // share (n x 3)
    unsigned* words = nullptr;
    double* meta = nullptr;  // 8 doubles
    double* metas = nullptr; // world x 8 doubles (host-gathered)
    kn::RouteParams* plan = nullptr;
    double* hdr = nullptr;
    int* bc = nullptr;
    int* totals = nullptr;
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

}  // namespace

struct kn_multi {
    std::vector<RankState> r;
    int n = 0;
    kn_config cfg{};
    bool rccl = false;
    double halo_factor = 2.5;
    int max_rounds = 8;
    int rounds = 0, halo_points = 0;
    std::vector<unsigned> idx;
    std::vector<float> dist;
    bool solved = false;
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

template <class T>
hipError_t dalloc(T** p, size_t count) { return hipMalloc(reinterpret_cast<void**>(p), std::max<size_t>(1, count) * sizeof(T)); }

// Buffers of one round on one rank, freed at the end of the round.
struct Round {
    float4* send = nullptr;
    float4* recv = nullptr;
    float* lpts = nullptr;
    int* lgids = nullptr;
    int* ws = nullptr;
    int* cell_start = nullptr;
    float4* sorted = nullptr;
    unsigned* perm = nullptr;
    kn::GridGeom* geom = nullptr;
    unsigned* out_idx = nullptr;
    float* out_dist = nullptr;
    unsigned* fallback = nullptr;
    unsigned* counters = nullptr;
    unsigned* uncert = nullptr;
    void release() {
        for (void* p : {(void*)send, (void*)recv, (void*)lpts, (void*)lgids, (void*)ws, (void*)cell_start, (void*)sorted,
                        (void*)perm, (void*)geom, (void*)out_idx, (void*)out_dist, (void*)fallback, (void*)counters,
                        (void*)uncert})
            if (p) (void)hipFree(p);
        *this = Round{};
    }
};

kn_status solve_round(kn_multi* m, double hf, std::vector<Round>& rd, bool* done) {
    const int W = (int)m->r.size();
    const int k = m->cfg.k > 0 ? m->cfg.k : KN_DEFAULT_K;
    // 2. metas -> host -> every rank; decomposition grid from the global extent
    std::vector<double> metas((size_t)8 * W);
    for (int i = 0; i < W; ++i) {
        RankState& R = m->r[i];
        KN_M(hipSetDevice(R.dev));
        KN_M(kn::launch_local_meta(R.pts, R.n, R.words, R.meta, R.s));
        KN_M(hipMemcpyAsync(&metas[(size_t)8 * i], R.meta, 8 * sizeof(double), hipMemcpyDeviceToHost, R.s));
    }
    for (auto& R : m->r) { KN_M(hipSetDevice(R.dev)); KN_M(hipStreamSynchronize(R.s)); }
    double lo[3] = {INFINITY, INFINITY, INFINITY}, hi[3] = {-INFINITY, -INFINITY, -INFINITY};
    for (int i = 0; i < W; ++i)
        for (int a = 0; a < 3; ++a) { lo[a] = std::min(lo[a], metas[8 * i + a]); hi[a] = std::max(hi[a], metas[8 * i + 3 + a]); }
    double ext[3];
    for (int a = 0; a < 3; ++a) ext[a] = std::isfinite(lo[a]) && std::isfinite(hi[a]) ? std::max(hi[a] - lo[a], 1e-30) : 1.0;
    int grid[3];
    factor3(W, ext, grid);
    // 3. plan + counts on every rank, one host sync for all totals
    std::vector<int> tot((size_t)2 * W * W);
    std::vector<double> hdr(kn::kPlanHdr);
    for (int i = 0; i < W; ++i) {
        RankState& R = m->r[i];
        KN_M(hipSetDevice(R.dev));
        KN_M(hipMemcpyAsync(R.metas, metas.data(), metas.size() * sizeof(double), hipMemcpyHostToDevice, R.s));
        KN_M(kn::launch_route_plan(R.metas, W, i, grid, k, hf, nullptr, R.plan, R.hdr, R.s));
        KN_M(kn::launch_route_count(R.pts, R.n, R.plan, W, R.bc, R.totals, R.s));
        KN_M(hipMemcpyAsync(&tot[(size_t)2 * W * i], R.totals, 2 * W * sizeof(int), hipMemcpyDeviceToHost, R.s));
        if (i == 0) KN_M(hipMemcpyAsync(hdr.data(), R.hdr, kn::kPlanHdr * sizeof(double), hipMemcpyDeviceToHost, R.s));
    }
    for (auto& R : m->r) { KN_M(hipSetDevice(R.dev)); KN_M(hipStreamSynchronize(R.s)); }
    auto own = [&](int s, int d) { return tot[(size_t)2 * W * s + 2 * d]; };
    auto halo = [&](int s, int d) { return tot[(size_t)2 * W * s + 2 * d + 1]; };
    auto rows = [&](int s, int d) { return own(s, d) + halo(s, d); };
    const double h = hdr[6], hs = hdr[7];
    const bool full = hdr[10] != 0.0;
    // send buffers (destination order) and receive buffers (source order)
    for (int i = 0; i < W; ++i) {
        RankState& R = m->r[i];
        KN_M(hipSetDevice(R.dev));
        int ns = 0, nr = 0;
        for (int d = 0; d < W; ++d) { ns += rows(i, d); nr += rows(d, i); }
        KN_M(dalloc(&rd[i].send, ns));
        KN_M(dalloc(&rd[i].recv, nr));
        KN_M(kn::launch_route_scatter(R.pts, nullptr, R.n, R.plan, W, R.bc, R.totals, rd[i].send, ns, -1, R.s));
    }
    // 4. the exchange
    if (m->rccl) {
#ifdef KN_HAVE_RCCL
        if (ncclGroupStart() != ncclSuccess) { m->err = "ncclGroupStart failed"; return KN_ERR_DEVICE; }
        for (int i = 0; i < W; ++i) {
            RankState& R = m->r[i];
            size_t so = 0, ro = 0;
            for (int d = 0; d < W; ++d) {
                const size_t sc = (size_t)rows(i, d), rc = (size_t)rows(d, i);
                if (sc && ncclSend(rd[i].send + so, sc * 4, ncclFloat, d, m->comms[i], R.s) != ncclSuccess) {
                    m->err = "ncclSend failed";
                    (void)ncclGroupEnd();
                    return KN_ERR_DEVICE;
                }
                if (rc && ncclRecv(rd[i].recv + ro, rc * 4, ncclFloat, d, m->comms[i], R.s) != ncclSuccess) {
                    m->err = "ncclRecv failed";
                    (void)ncclGroupEnd();
                    return KN_ERR_DEVICE;
                }
                so += sc;
                ro += rc;
            }
        }
        if (ncclGroupEnd() != ncclSuccess) { m->err = "ncclGroupEnd failed"; return KN_ERR_DEVICE; }
#endif
    } else {
        for (auto& R : m->r) { KN_M(hipSetDevice(R.dev)); KN_M(hipStreamSynchronize(R.s)); }  // scatters done
        for (int d = 0; d < W; ++d) {
            RankState& D = m->r[d];
            KN_M(hipSetDevice(D.dev));
            size_t ro = 0;
            for (int s = 0; s < W; ++s) {
                size_t so = 0;
                for (int t = 0; t < d; ++t) so += (size_t)rows(s, t);
                const size_t rc = (size_t)rows(s, d);
                if (rc) KN_M(hipMemcpyPeerAsync(rd[d].recv + ro, D.dev, rd[s].send + so, m->r[s].dev, rc * sizeof(float4), D.s));
                ro += rc;
            }
        }
    }
    // 5. local solve on every rank
    m->halo_points = 0;
    for (int i = 0; i < W; ++i) {
        RankState& R = m->r[i];
        Round& B = rd[i];
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
        m->halo_points += nh;
        KN_M(dalloc(&B.lpts, (size_t)nl * 3));
        KN_M(dalloc(&B.lgids, nl));
        KN_M(kn::launch_route_unpack(B.recv, nullptr, nl, t, B.lpts, B.lgids, R.s));
        // rank box / complete box / local grid box from the plan header (bindings.cpp dist_local)
        const int c[3] = {i % grid[0], (i / grid[0]) % grid[1], i / (grid[0] * grid[1])};
        double box[6];
        kn::CompleteBox comp;
        float fext[3];
        for (int a = 0; a < 3; ++a) {
            const double l = hdr[a], u = hdr[3 + a];
            const double w = (u - l) / (double)grid[a];
            const double blo = l + (double)c[a] * w;
            const double bhi = c[a] == grid[a] - 1 ? u : l + (double)(c[a] + 1) * w;
            comp.lo[a] = full || c[a] == 0 ? -INFINITY : (float)(blo - h);
            comp.hi[a] = full || c[a] == grid[a] - 1 ? INFINITY : (float)(bhi + h);
            box[a] = std::max(l, blo - hs);
            box[3 + a] = std::min(u, bhi + hs);
            fext[a] = (float)(box[3 + a] - box[a]);
        }
        const int th[3] = {m->cfg.tile[0], m->cfg.tile[1], m->cfg.tile[2]};
        const kn::AutoParams ap = kn::auto_params(nl, k, m->cfg.points_per_cell, th, m->cfg.halo, fext);
        const int C = ap.dims[0] * ap.dims[1] * ap.dims[2];
        const size_t nb = kn::scan_block_count(C) + 1;
        size_t rank_off = kn::kBBoxWords + 16 + 2 * ((size_t)C + 1) + nb;
        rank_off = (rank_off + 3) & ~(size_t)3;
        KN_M(dalloc(&B.ws, rank_off + 4 * (size_t)nl));
        KN_M(dalloc(&B.cell_start, (size_t)C + 1));
        KN_M(dalloc(&B.sorted, nl));
        KN_M(dalloc(&B.perm, nl));
        KN_M(dalloc(&B.geom, 1));
        kn::BuildBuffers b{};
        b.points = B.lpts;
        b.n = nl;
        for (int a = 0; a < 3; ++a) b.dims[a] = ap.dims[a];
        b.bbox_words = reinterpret_cast<unsigned*>(B.ws);
        b.geom = B.geom;
        b.cell_count = B.ws + kn::kBBoxWords + 16;
        b.cell_scan = b.cell_count + (C + 1);
        b.block_sums = b.cell_scan + (C + 1);
        b.cell_rank = reinterpret_cast<int2*>(B.ws + rank_off);
        b.bin_tmp = reinterpret_cast<float4*>(B.ws + rank_off);
        b.cell_start = B.cell_start;
        b.sorted = B.sorted;
        b.perm = B.perm;
        b.deterministic = m->cfg.deterministic;
        b.use_box = 1;
        for (int a = 0; a < 3; ++a) { b.box_lo[a] = (float)box[a]; b.box_hi[a] = (float)box[3 + a]; }
        KN_M(kn::launch_build(b, R.s));
        KN_M(kn::launch_global_w(B.sorted, B.perm, B.lgids, nl, n_owned, R.s));
        KN_M(dalloc(&B.out_idx, (size_t)n_owned * k));
        KN_M(dalloc(&B.out_dist, (size_t)n_owned * k));
        KN_M(dalloc(&B.fallback, nl));
        KN_M(dalloc(&B.counters, kn::kNumCounters));
        KN_M(dalloc(&B.uncert, n_owned));
        kn::QueryBuffers q{};
        q.sorted = B.sorted;
        q.cell_start = B.cell_start;
        q.perm = B.perm;
        q.geom = B.geom;
        q.n = nl;
        for (int a = 0; a < 3; ++a) q.dims[a] = ap.dims[a];
        q.k = k;
        q.n_queries = n_owned;
        q.row_of = B.perm;
        q.complete = comp;
        q.out_idx = B.out_idx;
        q.out_dist = B.out_dist;
        q.fallback_list = B.fallback;
        q.counters = B.counters;
        q.uncert_list = B.uncert;
        for (int a = 0; a < 3; ++a) q.tile[a] = ap.tile[a];
        q.halo = ap.halo;
        q.lds_capacity = ap.lds_capacity;
        q.use_tiles = m->cfg.exact_only ? 0 : 1;
        KN_M(kn::launch_query(q, R.s));
    }
    // 6. certification: any uncertified query -> growth round
    unsigned unc = 0;
    for (int i = 0; i < W; ++i) {
        RankState& R = m->r[i];
        KN_M(hipSetDevice(R.dev));
        unsigned c[kn::kNumCounters];
        KN_M(hipMemcpyAsync(c, rd[i].counters, sizeof(c), hipMemcpyDeviceToHost, R.s));
        KN_M(hipStreamSynchronize(R.s));
        unc += c[1];
    }
    *done = unc == 0 || full;
    if (!*done) return KN_OK;
    // 7. rows in original order
    m->idx.assign((size_t)m->n * k, 0xFFFFFFFFu);
    m->dist.assign((size_t)m->n * k, INFINITY);
    for (int i = 0; i < W; ++i) {
        RankState& R = m->r[i];
        KN_M(hipSetDevice(R.dev));
        int n_owned = 0;
        for (int s = 0; s < W; ++s) n_owned += own(s, i);
        std::vector<int> g(n_owned);
        std::vector<unsigned> ix((size_t)n_owned * k);
        std::vector<float> ds((size_t)n_owned * k);
        if (n_owned) {
            KN_M(hipMemcpyAsync(g.data(), rd[i].lgids, n_owned * sizeof(int), hipMemcpyDeviceToHost, R.s));
            KN_M(hipMemcpyAsync(ix.data(), rd[i].out_idx, ix.size() * sizeof(unsigned), hipMemcpyDeviceToHost, R.s));
            KN_M(hipMemcpyAsync(ds.data(), rd[i].out_dist, ds.size() * sizeof(float), hipMemcpyDeviceToHost, R.s));
        }
        KN_M(hipStreamSynchronize(R.s));
        for (int j = 0; j < n_owned; ++j) {
            const size_t dst = (size_t)g[j] * k;
            if (g[j] < 0 || g[j] >= m->n) { m->err = "global id out of range"; return KN_ERR_DEVICE; }
            std::memcpy(&m->idx[dst], &ix[(size_t)j * k], k * sizeof(unsigned));
            std::memcpy(&m->dist[dst], &ds[(size_t)j * k], k * sizeof(float));
        }
    }
    return KN_OK;
}

}  // namespace

extern "C" {

kn_multi* kn_prepare_multi(const kn_float3* points, int numpoints, const int* devices, int ndevices,
                           const kn_config* cfg) {
    if (!points && numpoints > 0) { kn_set_last_error_internal("null points"); return nullptr; }
    if (numpoints < 0 || ndevices < 1 || ndevices > kn::kRouteMaxWorld) {
        kn_set_last_error_internal("bad point or device count (1..64 ranks)");
        return nullptr;
    }
    auto* m = new kn_multi();
    m->cfg = cfg ? *cfg : kn_default_config();
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
        bool ok = hipSetDevice(R.dev) == hipSuccess && hipStreamCreateWithFlags(&R.s, hipStreamNonBlocking) == hipSuccess &&
                  dalloc(&R.pts, (size_t)R.n * 3) == hipSuccess && dalloc(&R.words, kn::kBBoxWords) == hipSuccess &&
                  dalloc(&R.meta, 8) == hipSuccess && dalloc(&R.metas, (size_t)8 * ndevices) == hipSuccess &&
                  dalloc(&R.plan, 1) == hipSuccess && dalloc(&R.hdr, kn::kPlanHdr) == hipSuccess &&
                  dalloc(&R.bc, (size_t)2 * ndevices * kn::route_block_count(R.n)) == hipSuccess &&
                  dalloc(&R.totals, (size_t)2 * ndevices) == hipSuccess &&
                  (R.n == 0 || hipMemcpy(R.pts, src + (size_t)3 * a, (size_t)R.n * 12, hipMemcpyHostToDevice) == hipSuccess);
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

kn_status kn_solve_multi(kn_multi* m) {
    if (!m) { kn_set_last_error_internal("null problem"); return KN_ERR_INVALID_ARGUMENT; }
    const int W = (int)m->r.size();
    double hf = m->halo_factor;
    kn_status st = KN_OK;
    m->rounds = 0;
    for (int round = 0; round < m->max_rounds; ++round) {
        std::vector<Round> rd(W);
        bool done = false;
        st = solve_round(m, hf, rd, &done);
        for (int i = 0; i < W; ++i) {
            (void)hipSetDevice(m->r[i].dev);
            (void)hipStreamSynchronize(m->r[i].s);
            rd[i].release();
        }
        m->rounds = round + 1;
        if (st != KN_OK) { kn_set_last_error_internal(m->err.c_str()); return st; }
        if (done) { m->solved = true; return KN_OK; }
        hf *= 2.0;  // uncertified queries: grow the halo
    }
    kn_set_last_error_internal("queries still uncertified after the maximum number of halo growth rounds");
    return KN_ERR_STATE;
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

void kn_free_multi(kn_multi** pm) {
    if (!pm || !*pm) return;
    kn_multi* m = *pm;
#ifdef KN_HAVE_RCCL
    for (auto& c : m->comms) (void)ncclCommDestroy(c);
#endif
    for (auto& R : m->r) {
        (void)hipSetDevice(R.dev);
        for (void* p : {(void*)R.pts, (void*)R.words, (void*)R.meta, (void*)R.metas, (void*)R.plan, (void*)R.hdr,
                        (void*)R.bc, (void*)R.totals})
            if (p) (void)hipFree(p);
        if (R.s) (void)hipStreamDestroy(R.s);
    }
    delete m;
    *pm = nullptr;
}

}  // extern "C"
