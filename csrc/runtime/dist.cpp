// dist.cpp -- see dist.hpp.
#include "dist.hpp"

#include <rccl/rccl.h>

#include <algorithm>
#include <chrono>
#include <cmath>
#include <cstdlib>
#include <cstring>
#include <thread>

#include "hostio.hpp"

namespace kn {

bool exact_epilogue(int k);

  // engine.cpp: KN_PIPE_EXACT

namespace {
#define KN_TRY(expr)                     \
    do {                                 \
        hipError_t e_ = (expr);          \
        if (e_ != hipSuccess) return e_; \
    } while (0)

constexpr size_t kAlign = 256;
size_t align_up(size_t v) { return (v + kAlign - 1) & ~(kAlign - 1); }
template <class T>
T* carve(char*& p, size_t count) {
    T* r = reinterpret_cast<T*>(p);
    p += align_up(std::max<size_t>(count, 1) * sizeof(T));
    return r;
}
ncclComm_t as_comm(RankComm* c) { return static_cast<ncclComm_t>(c->comm); }
}  // namespace

// ---------------------------------------------------------------- communicator --------
bool comm_unique_id(unsigned char out[kCommIdBytes], std::string* err) {
    static_assert(sizeof(ncclUniqueId) == kCommIdBytes, "ncclUniqueId is 128 bytes");
    ncclUniqueId id;
    const ncclResult_t r = ncclGetUniqueId(&id);
    if (r != ncclSuccess) {
        if (err) *err = std::string("ncclGetUniqueId: ") + ncclGetErrorString(r);
        return false;
    }
    std::memcpy(out, &id, kCommIdBytes);
    return true;
}

RankComm* comm_create(const unsigned char id[kCommIdBytes], int world, int rank, int device, std::string* err) {
    if (world < 1 || world > kRouteMaxWorld || rank < 0 || rank >= world) {
        if (err) *err = "bad world / rank";
        return nullptr;
    }
    if (hipSetDevice(device) != hipSuccess) {
        if (err) *err = "hipSetDevice failed";
        return nullptr;
    }
    ncclUniqueId uid;
    std::memcpy(&uid, id, kCommIdBytes);
    ncclComm_t comm = nullptr;
    const ncclResult_t r = ncclCommInitRank(&comm, world, uid, rank);
    if (r != ncclSuccess) {
        if (err) *err = std::string("ncclCommInitRank: ") + ncclGetErrorString(r);
        return nullptr;
    }
    RankComm* c = new RankComm();
    c->comm = comm;
    c->world = world;
    c->rank = rank;
    c->device = device;
    return c;
}

void comm_destroy(RankComm* c) {
    if (!c) return;
    if (c->comm && !c->aborted) (void)ncclCommDestroy(as_comm(c));
    delete c;
}

std::string comm_async_error(RankComm* c) {
    if (!c || !c->comm) return "no communicator";
    if (c->aborted) return "communicator aborted";
    ncclResult_t r = ncclSuccess;
    if (ncclCommGetAsyncError(as_comm(c), &r) != ncclSuccess) return "ncclCommGetAsyncError failed";
    if (r == ncclSuccess || r == ncclInProgress) return "";
    return std::string("RCCL async error: ") + ncclGetErrorString(r);
}

void comm_abort(RankComm* c) {
    if (!c || !c->comm || c->aborted) return;
    (void)ncclCommAbort(as_comm(c));
    c->aborted = true;
}

// ---------------------------------------------------------------- pipeline ------------
DistPipeline::DistPipeline(const DistPlan& p, RankComm* comm) : p_(p), comm_(comm) {
    const int W = p_.world;
    if (comm_ && (comm_->world != W || comm_->rank != p_.rank)) { fail("communicator does not match the plan"); return; }
    if (W < 1 || W > kRouteMaxWorld || p_.rank < 0 || p_.rank >= W || p_.k < 1 || p_.k > KN_MAX_K || p_.n < 0 ||
        (int)p_.recv_own.size() != W || (int)p_.recv_halo.size() != W || (int)p_.cross_send.size() != W ||
        (int)p_.cross_recv.size() != W || (int)p_.tot.size() != 2 * W || (int)p_.hdr.size() < kPlanHdr ||
        p_.grid[0] * p_.grid[1] * p_.grid[2] != W || !p_.route || !p_.metas || (p_.n > 0 && !p_.points)) {
        fail("inconsistent distributed plan");
        return;
    }
    if (p_.self_via_comm && W != 1) { fail("self_via_comm is the world-1 forced-collective mode"); return; }
    if (hipSetDevice(p_.device) != hipSuccess) { fail("hipSetDevice"); return; }
    long long own = 0, halo = 0;
    for (int s = 0; s < W; ++s) {
        if (p_.recv_own[s] < 0 || p_.recv_halo[s] < 0 || p_.cross_send[s] < 0 || p_.cross_recv[s] < 0) {
            fail("negative split size");
            return;
        }
        own += p_.recv_own[s];
        halo += p_.recv_halo[s];
    }
    if (own + halo >= (1ll << 31) - 1) { fail("too many local rows"); return; }
    n_owned_ = (int)own;
    n_route_ = n_flag_ = p_.n;
    rows_ = (int)(own + halo);
    // send / receive layouts (route_scatter self-last: the other destinations in rank order, then
    // the rank's own segment; the receive buffer holds the other sources in rank order)
    soff_.assign(W, 0);
    roff_.assign(W, 0);
    long long so = 0, ro = 0;
    for (int d = 0; d < W; ++d) {
        if (d == p_.rank) continue;
        soff_[d] = so;
        roff_[d] = ro;
        so += p_.cross_send[d];
        ro += p_.cross_recv[d];
    }
    const long long nself = (long long)p_.tot[2 * p_.rank] + p_.tot[2 * p_.rank + 1];
    if (so + nself > p_.cap) { fail("send buffer smaller than the planned rows"); return; }
    table_ = UnpackTable{};
    table_.world = W;
    if (p_.self_via_comm) {
        // world 1: the own rows travel through the communicator and the unpack like any source's
        soff_[0] = so;  // the self segment follows the (no) other destinations
        roff_[0] = 0;
        recv_rows_ = (int)nself;
        table_.seg[0] = 0;
        table_.own[0] = p_.recv_own[0];
        table_.own_pref[0] = 0;
        table_.halo_pref[0] = 0;
        table_.n_own = n_owned_;
        table_.rows_cross = recv_rows_;
        table_.self = -1;
        table_.out_rows = rows_;
        rows_cross_ = recv_rows_;
    } else {
        long long seg = 0, o = 0, h = 0;
        for (int s = 0; s < W; ++s) {
            table_.seg[s] = (int)seg;
            table_.own[s] = p_.recv_own[s];
            table_.own_pref[s] = (int)o;
            table_.halo_pref[s] = (int)h;
            if (s != p_.rank) seg += (long long)p_.recv_own[s] + p_.recv_halo[s];
            o += p_.recv_own[s];
            h += p_.recv_halo[s];
        }
        if (seg != ro) { fail("receive split sizes do not add up"); return; }
        table_.n_own = n_owned_;
        table_.rows_cross = (int)seg;
        table_.self = p_.rank;
        table_.out_rows = rows_;
        rows_cross_ = (int)seg;
        recv_rows_ = (int)seg;
        if (p_.place[2] != rows_) { fail("self placement does not match the local rows"); return; }
    }
    // local geometry and the query plan: the same arithmetic as the torch binding's dist_local
    const RankLocal rl = rank_local(p_.hdr.data(), p_.rank, p_.grid, p_.cert_field, p_.field_g);
    complete_ = rl.complete;
    const int th[3] = {0, 0, 0};
    AutoParams ap = auto_params(rows_, p_.k, p_.ppc, th, 0, rl.ext);
    if (p_.dims[0] != ap.dims[0] || p_.dims[1] != ap.dims[1] || p_.dims[2] != ap.dims[2]) {
        ap.tile[0] = std::max(1, ap.tile[0] / std::max(1, ap.xsub));  // a refined grid: isotropic
        ap.xsub = 1;
    }
    const long long C = (long long)p_.dims[0] * p_.dims[1] * p_.dims[2];
    if (p_.dims[0] < 1 || p_.dims[1] < 1 || p_.dims[2] < 1 || C >= (1ll << 31) - 1) { fail("bad local grid"); return; }
    C_ = (int)C;
    bproto_ = BuildBuffers{};
    bproto_.n = rows_;
    for (int a = 0; a < 3; ++a) bproto_.dims[a] = p_.dims[a];
    bproto_.deterministic = p_.deterministic;
    bproto_.use_box = 1;
    for (int a = 0; a < 3; ++a) {
        bproto_.box_lo[a] = (float)rl.box[a];
        bproto_.box_hi[a] = (float)rl.box[3 + a];
    }
    bproto_.n_owned = n_owned_;
    // forced collectives (world 1, the own rows through RCCL): the build follows the 14 MB self
    // exchange on the build stream, where the automatic large binning blocks cost 8 % (0.333 ->
    // 0.359 ms); plain steps keep them (0.270 -> 0.262)
    bproto_.bin_items = p_.self_via_comm ? 4096 : 0;
    bproto_.n_zero_words = kNumCounters;
    qproto_ = QueryBuffers{};
    qproto_.n = rows_;
    for (int a = 0; a < 3; ++a) qproto_.dims[a] = p_.dims[a];
    qproto_.k = p_.k;
    qproto_.n_queries = n_owned_;
    qproto_.complete = complete_;
    for (int a = 0; a < 3; ++a) qproto_.tile[a] = ap.tile[a];
    qproto_.halo = ap.halo;
    qproto_.xsub = ap.xsub;
    qproto_.lds_capacity = ap.lds_capacity;
    qproto_.use_tiles = 1;
    qproto_.counters_zeroed = 1;
    qproto_.exact_grid = p_.exact_grid;

    // buffers: one block per set
    const int nb = route_block_count(p_.n);
    const size_t nbs = scan_block_count(C_) + 1;
    const size_t K = (size_t)p_.k;
    auto layout = [&](char* base, Set& S) {
        char* q = base;
        S.send = carve<float4>(q, (size_t)p_.cap);
        S.bc = carve<int>(q, (size_t)2 * W * nb);
        S.totals = carve<int>(q, (size_t)2 * W);
        S.partials = carve<unsigned>(q, (size_t)6 * nb);
        S.recv = carve<float4>(q, (size_t)recv_rows_);
        S.lpts = carve<float>(q, (size_t)rows_ * 3);
        S.lgids = carve<int>(q, (size_t)rows_);
        S.bbox = carve<unsigned>(q, kBBoxWords);
        S.geom = carve<GridGeom>(q, 1);
        S.cell_count = carve<int>(q, (size_t)C_ + 1);
        S.cell_scan = carve<int>(q, (size_t)C_ + 1);
        S.block_sums = carve<int>(q, nbs);
        S.cell_start = carve<int>(q, (size_t)C_ + 1);
        S.bin_tmp = carve<float4>(q, (size_t)rows_);
        S.sorted = carve<float4>(q, (size_t)rows_);
        S.perm = carve<unsigned>(q, (size_t)rows_);
        S.fallback = carve<unsigned>(q, (size_t)rows_);
        S.counters = carve<unsigned>(q, kNumCounters);
        S.uncert = carve<unsigned>(q, (size_t)n_owned_);
        S.idx = carve<int>(q, (size_t)n_owned_ * K);
        S.d2 = carve<float>(q, (size_t)n_owned_ * K);
        S.flag = carve<int>(q, 1);
        S.ticket = carve<unsigned>(q, 1);
        return (size_t)(q - base);
    };
    Set probe{};
    const size_t bytes = layout(nullptr, probe);
    // KN_DIST_QSTREAMS: query streams of the rank pipeline (pipeline.hpp). Two query streams run
    // three grid sets (the next step's route + exchange + build then waits for the query two steps
    // back, not the previous one still in flight)
    // Default two (900K K=16 world 1, 200 / 50 steps, two passes: one stream 0.3145 / 0.3196 ms,
    // two streams + three sets + per-launch flag 0.2838 / 0.2886; profiles/r5_dist.txt). They lost
    // until the second query stream ran at the device's least priority no more (pipeline.cpp).
    const char* qsv = std::getenv("KN_DIST_QSTREAMS");
    const int qstreams = comm_ ? (qsv ? std::atoi(qsv) : 2) : 1;
    const char* nsv = std::getenv("KN_DIST_SETS");  // A/B override: 2 or 3 grid sets
    nsets_ = nsv ? std::max(2, std::min(Pipeline::kMaxSets, std::atoi(nsv))) : (qstreams >= 2 ? 3 : 2);
    // With two query streams the step's flag is reduced once per launch() (KN_DIST_DEFER=0: per step):
    // a per-step epilogue on the build stream (flag + all-reduce) would wait for each query and hold
    // the next build behind it, and an all-reduce on a third stream could reorder RCCL calls of one
    // communicator across ranks
    const char* dfv = std::getenv("KN_DIST_DEFER");
    deferred_ = comm_ && qstreams >= 2 && !(dfv && dfv[0] == '0');
    // KN_DIST_TAIL=1: tail mode (measured neutral at world 1: 200 / 50 0.2661 vs 0.2657 ms, 20 / 5
    // -1.5 %, K=50 equal; profiles/r5_dist.txt), off by default
    const char* tlv = std::getenv("KN_DIST_TAIL");
    tail_ = deferred_ && (tlv && tlv[0] == '1');
    // KN_DIST_FUSED_FLAG=0: the step check as its own two kernels on the query stream (rounds 5-6)
    const char* ffv = std::getenv("KN_DIST_FUSED_FLAG");
    fused_flag_ = deferred_ && !tail_ && !(ffv && ffv[0] == '0');
    for (int s = 0; s < nsets_; ++s) {
        Set& S = set_[s];
        void* b = nullptr;
        if (device_malloc(&b, bytes) != hipSuccess) { fail("hipMalloc(distributed set)"); return; }
        S.block = static_cast<char*>(b);
        layout(S.block, S);
        if (hipMemset(S.flag, 0, sizeof(int)) != hipSuccess || hipMemset(S.ticket, 0, sizeof(unsigned)) != hipSuccess) {
            fail("hipMemset");
            return;
        }
        S.tree_ws = S.tree_nodes = nullptr;
        if (p_.use_tree) {
            if (device_malloc(&S.tree_ws, std::max<size_t>(1, tree_workspace_bytes(rows_, p_.dims))) != hipSuccess ||
                device_malloc(&S.tree_nodes, std::max<size_t>(1, tree_node_bytes(rows_))) != hipSuccess) {
                fail("hipMalloc(distributed tree)");
                return;
            }
        }
    }
    void* v = nullptr;
    if (device_malloc(&v, sizeof(RouteParams)) != hipSuccess) { fail("hipMalloc(route)"); return; }
    route_dev_ = v;
    if (device_malloc(&v, (size_t)W * 8 * sizeof(double)) != hipSuccess) { fail("hipMalloc(metas)"); return; }
    metas_dev_ = static_cast<double*>(v);
    if (device_malloc(&v, (size_t)2 * W * sizeof(int)) != hipSuccess) { fail("hipMalloc(totals)"); return; }
    tot_dev_ = static_cast<int*>(v);
    if (device_malloc(&v, sizeof(int)) != hipSuccess) { fail("hipMalloc(sticky)"); return; }
    sticky_ = static_cast<int*>(v);
    if (device_malloc(&v, 2 * sizeof(int)) != hipSuccess) { fail("hipMalloc(pending)"); return; }
    pending_ = static_cast<int*>(v);
    reduced_ = pending_ + 1;
    if (hipMemset(pending_, 0, 2 * sizeof(int)) != hipSuccess) { fail("hipMemset"); return; }
    if (hipHostMalloc(&v, sizeof(int), hipHostMallocDefault) != hipSuccess) { fail("hipHostMalloc(flag)"); return; }
    host_flag_ = static_cast<int*>(v);
    *host_flag_ = 0;
    if (hipHostGetDevicePointer(&v, host_flag_, 0) != hipSuccess) { fail("hipHostGetDevicePointer"); return; }
    host_flag_dev_ = static_cast<int*>(v);
    if (device_malloc(&v, (size_t)Pipeline::kMaxSets * sizeof(StepFlagJob)) != hipSuccess) { fail("hipMalloc(jobs)"); return; }
    jobs_dev_ = static_cast<StepFlagJob*>(v);
    if (upload_jobs() != hipSuccess) { fail("step check upload"); return; }
    if (hipMemcpy(route_dev_, p_.route, sizeof(RouteParams), hipMemcpyDeviceToDevice) != hipSuccess ||
        hipMemcpy(metas_dev_, p_.metas, (size_t)W * 8 * sizeof(double), hipMemcpyDeviceToDevice) != hipSuccess ||
        hipMemcpy(tot_dev_, p_.tot.data(), (size_t)2 * W * sizeof(int), hipMemcpyHostToDevice) != hipSuccess ||
        hipMemset(sticky_, 0, sizeof(int)) != hipSuccess) {
        fail("plan upload");
        return;
    }
    // KN_DIST_SIDE_PRIO (A/B): 1 the build stream at the device's greatest priority, 2 at its least
    const char* spv = std::getenv("KN_DIST_SIDE_PRIO");
    const int sprio = spv ? std::atoi(spv) : 0;
    int p_least = 0, p_greatest = 0;
    (void)hipDeviceGetStreamPriorityRange(&p_least, &p_greatest);
    if (hipStreamCreateWithFlags(&main_, hipStreamNonBlocking) != hipSuccess ||
        ((sprio == 1 || sprio == 2)
             ? hipStreamCreateWithPriority(&side_, hipStreamNonBlocking, sprio == 2 ? p_least : p_greatest)
             : hipStreamCreateWithFlags(&side_, hipStreamNonBlocking)) != hipSuccess) {
        fail("hipStreamCreate");
        return;
    }
    if (hipEventCreateWithFlags(&in_ev_, hipEventDisableTiming) != hipSuccess) { fail("hipEventCreate"); return; }
    for (int i = 0; i < 8; ++i) {
        hipEvent_t e = nullptr;
        if (hipEventCreateWithFlags(&e, hipEventDisableTiming) != hipSuccess) { fail("hipEventCreate"); return; }
        ring_.push_back(e);
    }
    auto b = [this](int s, hipStream_t st) { return stage_build(s, st); };
    auto q = [this](int s, hipStream_t st) { return stage_query(s, st); };
    auto r = [this](int s, hipStream_t st) { return stage_flag(s, st); };
    auto t = [this](int s, hipStream_t st) { return stage_tail(s, st); };
    if (!comm_) {  // loopback mode: eager stages driven by the caller
        ok_ = true;
        return;
    }
    // KN_DIST_CAPTURE_JOINED=1 (diagnostics): start unrolled captures on the main stream, so the
    // RCCL calls of the build stage are captured on a JOINED stream (the round-4 segfault)
    const char* joined = std::getenv("KN_DIST_CAPTURE_JOINED");
    const Pipeline::Stage rs = !deferred_ ? Pipeline::Stage(r) : tail_ ? Pipeline::Stage(t) : Pipeline::Stage();
    if (pipe_.init(main_, side_, b, q, rs, !(joined && joined[0] == '1'), qstreams, nsets_, nullptr, tail_) != hipSuccess) {
        fail("pipeline init");
        return;
    }
    // RCCL stages run eagerly until prepare_graphs() captured them (set_eager(false) below)
    pipe_.set_eager(true);
    ok_ = true;
}

kn_status DistPipeline::poll(hipEvent_t ev, double timeout_s, const char* what) {
    using clk = std::chrono::steady_clock;
    const auto t0 = clk::now();
    int polls = 0;
    for (;;) {
        const hipError_t q = hipEventQuery(ev);
        if (q == hipSuccess) return KN_OK;
        if (q != hipErrorNotReady) { err_ = std::string(what) + ": " + hipGetErrorString(q); return KN_ERR_DEVICE; }
        if ((++polls & 63) == 0) {
            // a dead or hung peer: RCCL's async error, or the deadline
            const std::string ae = comm_ ? comm_async_error(comm_) : std::string();
            if (!ae.empty()) {
                comm_abort(comm_);
                err_ = ae;
                return KN_ERR_DEVICE;
            }
            if (std::chrono::duration<double>(clk::now() - t0).count() > timeout_s) {
                if (comm_) comm_abort(comm_);
                err_ = std::string(what) + " did not complete within the deadline (peer dead or hung?)";
                return KN_ERR_DEVICE;
            }
        }
        std::this_thread::sleep_for(std::chrono::microseconds(polls < 256 ? 2 : 50));
    }
}

kn_status DistPipeline::warmup(double timeout_s) {
    if (!ok_ || !comm_) return KN_ERR_STATE;
    if (warm_) return KN_OK;
    // one eager (uncaptured) step on set 1: RCCL connects to the step's peers and sets up the
    // all-reduce before anything is captured (collective: every rank calls it at the same step)
    hipError_t e = stage_build(1, main_);
    if (e == hipSuccess) e = stage_query(1, main_);
    if (e == hipSuccess) e = stage_flag(1, main_);
    if (e == hipSuccess) e = hipEventRecord(ring_[0], main_);
    if (e != hipSuccess) { err_ = std::string("eager warm-up step: ") + hipGetErrorString(e); return KN_ERR_DEVICE; }
    const kn_status st = poll(ring_[0], timeout_s, "eager warm-up step");
    if (st == KN_OK) warm_ = true;
    return st;
}

kn_status DistPipeline::prepare_graphs(int unroll) {
    if (!ok_ || !comm_) return KN_ERR_STATE;
    if (!warm_) { err_ = "prepare_graphs() before warmup()"; return KN_ERR_STATE; }
    pipe_.set_eager(false);
    // test hook: an injected capture failure (the fallback path of tests/test_gpu_distributed.py)
    const char* inj = std::getenv("KN_DIST_CAPTURE_FAIL");
    hipError_t e = (inj && inj[0] == '1') ? hipErrorStreamCaptureUnsupported : pipe_.prepare(unroll);
    if (e != hipSuccess) {
        pipe_.set_eager(true);
        err_ = std::string("graph capture of the distributed step: ") + hipGetErrorString(e);
        return KN_ERR_DEVICE;
    }
    return KN_OK;
}

void DistPipeline::set_eager(bool eager) { pipe_.set_eager(eager); }

kn_status DistPipeline::rebind(const float* points, const int* ids, int n) {
    if (!ok_) return KN_ERR_STATE;
    if (n < 0 || (n > 0 && !points)) {
        err_ = "rebind: bad input";
        return KN_ERR_INVALID_ARGUMENT;
    }
    if (points == p_.points && ids == p_.ids && n == n_flag_) return KN_OK;
    if (!pipe_.eager()) pipe_.set_eager(true);
    // a primed build read the old input: the next launch rebuilds from the new one
    if (pipe_.unprime() != hipSuccess) { err_ = "rebind: sync"; return KN_ERR_DEVICE; }
    p_.points = points;
    p_.ids = ids;
    // A share of another size cannot be the validated plan's: route at most the planned number of
    // points (the buffers' size) and let the step's flag see the true count, so the step is
    // invalid on every rank (MAX all-reduce) while every rank issues the same collectives
    n_route_ = std::min(n, p_.n);
    n_flag_ = n;
    if (upload_jobs() != hipSuccess) { err_ = "rebind: step check upload"; return KN_ERR_DEVICE; }
    return KN_OK;
}

// the sets' step checks (step_flag_job) in device memory, for the exact kernel (fused flag)
hipError_t DistPipeline::upload_jobs() {
    StepFlagJob h[Pipeline::kMaxSets]{};
    for (int s = 0; s < nsets_; ++s) h[s] = step_flag_job(s);
    return hipMemcpy(jobs_dev_, h, sizeof(h), hipMemcpyHostToDevice);
}

DistPipeline::~DistPipeline() {
    pipe_.reset();
    if (main_) (void)hipStreamSynchronize(main_);
    if (side_) (void)hipStreamSynchronize(side_);
    for (auto& S : set_) {
        if (S.block) (void)hipFree(S.block);
        if (S.tree_ws) (void)hipFree(S.tree_ws);
        if (S.tree_nodes) (void)hipFree(S.tree_nodes);
    }
    for (void* v : {route_dev_, (void*)metas_dev_, (void*)tot_dev_, (void*)sticky_, (void*)pending_, (void*)jobs_dev_})
        if (v) (void)hipFree(v);
    if (host_flag_) (void)hipHostFree(host_flag_);
    for (auto e : ring_) (void)hipEventDestroy(e);
    if (in_ev_) (void)hipEventDestroy(in_ev_);
    if (main_) (void)hipStreamDestroy(main_);
    if (side_) (void)hipStreamDestroy(side_);
}

hipError_t DistPipeline::exchange(int s, hipStream_t st) {
    if (!comm_) return hipSuccess;  // loopback mode: the caller moved the rows
    const Set& S = set_[s];
    const int W = p_.world;
    ncclComm_t comm = as_comm(comm_);
    if (ncclGroupStart() != ncclSuccess) return hipErrorUnknown;
    bool bad = false;
    for (int d = 0; d < W && !bad; ++d) {
        size_t sc, rc;
        if (d == p_.rank) {
            if (!p_.self_via_comm) continue;
            sc = rc = (size_t)recv_rows_;
        } else {
            sc = (size_t)p_.cross_send[d];
            rc = (size_t)p_.cross_recv[d];
        }
        if (sc && ncclSend(reinterpret_cast<const float*>(S.send + soff_[d]), sc * 4, ncclFloat, d, comm, st) != ncclSuccess)
            bad = true;
        if (rc && ncclRecv(reinterpret_cast<float*>(S.recv + roff_[d]), rc * 4, ncclFloat, d, comm, st) != ncclSuccess)
            bad = true;
    }
    const ncclResult_t r = ncclGroupEnd();
    return bad || r != ncclSuccess ? hipErrorUnknown : hipSuccess;
}

// marks (profile only): events recorded after the routing and after the exchange
hipError_t DistPipeline::stage_build(int s, hipStream_t st, const std::vector<hipEvent_t>* marks) {
    Set& S = set_[s];
    const auto* rp = static_cast<const RouteParams*>(route_dev_);
    if (n_route_ > 0) {
        // block 0 also zeroes the build's bucket totals (no memset node before the build)
        KN_TRY(launch_route_count(p_.points, n_route_, rp, p_.world, S.bc, S.totals, st, S.partials, S.cell_scan,
                                  bin_totals_words(C_)));
        if (p_.self_via_comm) {
            KN_TRY(launch_route_scatter(p_.points, p_.ids, n_route_, rp, p_.world, S.bc, S.totals, S.send, p_.cap, p_.rank, st));
        } else {
            SelfPlace sp{S.lpts, S.lgids, p_.place[0], p_.place[1], p_.place[2], p_.place[3], p_.place[4]};
            KN_TRY(launch_route_scatter(p_.points, p_.ids, n_route_, rp, p_.world, S.bc, S.totals, S.send, p_.cap, p_.rank,
                                        st, &sp));
        }
    } else {
        // an empty share: nothing to route, the counts are all zero
        KN_TRY(hipMemsetAsync(S.totals, 0, (size_t)2 * p_.world * sizeof(int), st));
    }
    if (marks) KN_TRY(hipEventRecord((*marks)[0], st));
    KN_TRY(exchange(s, st));
    if (marks) KN_TRY(hipEventRecord((*marks)[1], st));
    if (rows_cross_ > 0) KN_TRY(launch_route_unpack(S.recv, nullptr, rows_cross_, table_, S.lpts, S.lgids, st));
    BuildBuffers b = bproto_;
    b.points = S.lpts;
    b.bbox_words = S.bbox;
    b.geom = S.geom;
    b.cell_count = S.cell_count;
    b.cell_scan = S.cell_scan;
    b.block_sums = S.block_sums;
    b.cell_start = S.cell_start;
    b.cell_rank = reinterpret_cast<int2*>(S.bin_tmp);
    b.bin_tmp = S.bin_tmp;
    b.sorted = S.sorted;
    b.perm = S.perm;
    b.gids = S.lgids;
    b.zero_words = S.counters;
    b.totals_zeroed = n_route_ > 0 ? 1 : 0;
    KN_TRY(launch_build(b, st));
    if (p_.use_tree && rows_ > 0) {
        TreeView t = tree_view(S.tree_ws, rows_, p_.dims);
        tree_attach_nodes(t, S.tree_nodes);
        KN_TRY(launch_tree_leaves(S.sorted, S.cell_start, S.geom, t, st));
        KN_TRY(launch_tree_nodes(t, st));
    }
    return hipSuccess;
}

hipError_t DistPipeline::stage_query(int s, hipStream_t st) {
    Set& S = set_[s];
    if (p_.use_tree) {
        if (rows_ > 0) {
            TreeView t = tree_view(S.tree_ws, rows_, p_.dims);
            tree_attach_nodes(t, S.tree_nodes);
            TreeQuery q{};
            q.k = p_.k;
            q.n_queries = n_owned_;
            q.row_of = S.perm;
            q.out_idx = reinterpret_cast<unsigned*>(S.idx);
            q.out_dist = S.d2;
            q.counters = S.counters;
            KN_TRY(launch_tree_query(t, q, st));
            // the complete-box certification the grid kernels do inline
            KN_TRY(launch_certify_rows(S.lpts, n_owned_, p_.k, S.d2, complete_, S.geom, S.counters, S.uncert, st));
        }
        if (deferred_ && !tail_) KN_TRY(step_flag(s, st));
        return hipSuccess;
    }
    // the tile kernel and its exact finish (KN_PIPE_EXACT=1: the exact finish opens the epilogue
    // on the side stream instead, engine.cpp exact_epilogue; deferred mode: always here)
    QueryBuffers q = query_proto(s);
    q.exact_mode = tail_ ? 1 : (!deferred_ && exact_epilogue(p_.k)) ? 1 : 0;
    if (fused_flag_ && n_route_ <= n_flag_) {
        // the same check as step_flag(), in the exact finish kernel's last workgroup
        q.step_flag = jobs_dev_ + s;
        return launch_query(q, st);
    }
    KN_TRY(launch_query(q, st));
    if (deferred_ && !tail_) KN_TRY(step_flag(s, st));
    return hipSuccess;
}

// Tail mode: the fallback list's exact finish and the step's local flag, on the pipeline's tail
// stream after the step's tile kernel (pipeline.hpp tail_stream).
hipError_t DistPipeline::stage_tail(int s, hipStream_t st) {
    if (!p_.use_tree) {
        QueryBuffers q = query_proto(s);
        q.exact_mode = 2;
        KN_TRY(launch_query(q, st));
    }
    return step_flag(s, st);
}

StepFlagJob DistPipeline::step_flag_job(int s) const {
    const Set& S = set_[s];
    StepFlagJob j{};
    j.partials = S.partials;
    j.nb = j.stride = n_route_ > 0 ? route_block_count(n_route_) : 0;  // launch_steady_flag_partials' layout
    j.n = n_flag_;
    j.planned = metas_dev_ + 8 * p_.rank;
    j.totals = S.totals;
    j.ptotals = tot_dev_;
    j.nt = 2 * p_.world;
    j.flag = S.flag;
    j.pending = pending_;
    j.ticket = S.ticket;
    return j;
}

// deferred mode: the step's local flag on its query stream, max-accumulated into pending_
hipError_t DistPipeline::step_flag(int s, hipStream_t st) {
    Set& S = set_[s];
    KN_TRY(launch_steady_flag_partials(S.partials, n_route_, n_flag_, metas_dev_ + 8 * p_.rank, S.totals, tot_dev_, 2 * p_.world,
                                       S.counters, S.flag, st));
    return launch_flag_accum(S.flag, pending_, st);
}

QueryBuffers DistPipeline::query_proto(int s) const {
    const Set& S = set_[s];
    QueryBuffers q = qproto_;
    q.sorted = S.sorted;
    q.cell_start = S.cell_start;
    q.geom = S.geom;
    q.row_of = S.perm;
    q.out_idx = reinterpret_cast<unsigned*>(S.idx);
    q.out_dist = S.d2;
    q.fallback_list = S.fallback;
    q.counters = S.counters;
    q.uncert_list = S.uncert;
    return q;
}

// Epilogue of step s (side stream, after its queries): the exact finish of the fallback list,
// this step's check (the share's bbox and count from the routing partials and every send count
// as planned, no uncertified row), its MAX all-reduce and the sticky host flag.
hipError_t DistPipeline::stage_flag(int s, hipStream_t st) {
    Set& S = set_[s];
    if (!p_.use_tree && (exact_epilogue(p_.k) || tail_)) {  // (tail mode: the query left the list)
        QueryBuffers q = query_proto(s);
        q.exact_mode = 2;
        KN_TRY(launch_query(q, st));
    }
    KN_TRY(launch_steady_flag_partials(S.partials, n_route_, n_flag_, metas_dev_ + 8 * p_.rank, S.totals, tot_dev_, 2 * p_.world,
                                       S.counters, S.flag, st));
    if (!comm_) return hipSuccess;  // loopback mode: the caller reduces the ranks' flags
    if (ncclAllReduce(S.flag, S.flag, 1, ncclInt32, ncclMax, as_comm(comm_), st) != ncclSuccess) return hipErrorUnknown;
    return launch_flag_sink(S.flag, sticky_, host_flag_dev_, st);
}

kn_status DistPipeline::loopback_stage(int stage) {
    if (!ok_ || comm_) return KN_ERR_STATE;
    hipError_t e = hipSuccess;
    if (stage == 0) {
        // the routing half of stage_build (exchange and local build follow in stage 1)
        Set& S = set_[0];
        const auto* rp = static_cast<const RouteParams*>(route_dev_);
        if (n_route_ > 0) {
            e = launch_route_count(p_.points, n_route_, rp, p_.world, S.bc, S.totals, main_, S.partials);
            SelfPlace sp{S.lpts, S.lgids, p_.place[0], p_.place[1], p_.place[2], p_.place[3], p_.place[4]};
            if (e == hipSuccess)
                e = launch_route_scatter(p_.points, p_.ids, n_route_, rp, p_.world, S.bc, S.totals, S.send, p_.cap, p_.rank,
                                         main_, &sp);
        } else {
            e = hipMemsetAsync(S.totals, 0, (size_t)2 * p_.world * sizeof(int), main_);
        }
    } else {
        Set& S = set_[0];
        if (rows_cross_ > 0) e = launch_route_unpack(S.recv, nullptr, rows_cross_, table_, S.lpts, S.lgids, main_);
        if (e == hipSuccess) {
            BuildBuffers b = bproto_;
            b.points = S.lpts; b.bbox_words = S.bbox; b.geom = S.geom; b.cell_count = S.cell_count;
            b.cell_scan = S.cell_scan; b.block_sums = S.block_sums; b.cell_start = S.cell_start;
            b.cell_rank = reinterpret_cast<int2*>(S.bin_tmp); b.bin_tmp = S.bin_tmp; b.sorted = S.sorted;
            b.perm = S.perm; b.gids = S.lgids; b.zero_words = S.counters;
            e = launch_build(b, main_);
        }
        if (e == hipSuccess && p_.use_tree && rows_ > 0) {
            TreeView t = tree_view(S.tree_ws, rows_, p_.dims);
            tree_attach_nodes(t, S.tree_nodes);
            e = launch_tree_leaves(S.sorted, S.cell_start, S.geom, t, main_);
            if (e == hipSuccess) e = launch_tree_nodes(t, main_);
        }
        if (e == hipSuccess) e = stage_query(0, main_);
        if (e == hipSuccess) e = stage_flag(0, main_);
    }
    if (e == hipSuccess) e = hipStreamSynchronize(main_);
    if (e != hipSuccess) { err_ = std::string("loopback stage: ") + hipGetErrorString(e); return KN_ERR_DEVICE; }
    return KN_OK;
}

int DistPipeline::flag_local(int s) const {
    int f = -1;
    (void)hipStreamSynchronize(main_);
    (void)hipMemcpy(&f, set_[s].flag, sizeof(int), hipMemcpyDeviceToHost);
    return f;
}

kn_status DistPipeline::launch(int iters, int unroll, bool keep_primed, hipStream_t caller, long long* last_step) {
    if (!ok_) return KN_ERR_STATE;
    if (!comm_) { err_ = "loopback pipelines run loopback_stage() only"; return KN_ERR_STATE; }
    if (comm_->aborted) { err_ = "communicator aborted"; return KN_ERR_DEVICE; }
    if (!warm_) { err_ = "launch() before warmup()"; return KN_ERR_STATE; }
    if (iters <= 0) {
        if (last_step) *last_step = pipe_.steps() - 1;
        return KN_OK;
    }
    hipError_t e = hipSuccess;
    if (caller) {
        // the first build reads the caller's points after the caller's earlier writes
        e = hipEventRecord(in_ev_, caller);
        if (e == hipSuccess) e = hipStreamWaitEvent(side_, in_ev_, 0);
    }
    if (e == hipSuccess) e = pipe_.launch(iters, unroll, keep_primed);
    if (e == hipSuccess && deferred_) {
        // one all-reduce for the call's steps: after both query streams' last steps (last_done),
        // on the build stream, in the same place of every rank's RCCL call sequence
        e = hipStreamWaitEvent(side_, pipe_.last_done(), 0);
        if (e == hipSuccess && ncclAllReduce(pending_, reduced_, 1, ncclInt32, ncclMax, as_comm(comm_), side_) != ncclSuccess)
            e = hipErrorUnknown;
        if (e == hipSuccess) e = launch_flag_sink(reduced_, sticky_, host_flag_dev_, side_);
    }
    if (e == hipSuccess && caller) {
        // later work on the caller's stream (e.g. refilling the points) waits for the builds
        for (int s = 0; s < nsets_ && e == hipSuccess; ++s) e = hipStreamWaitEvent(caller, pipe_.build_event(s), 0);
    }
    if (e != hipSuccess) {
        err_ = std::string("distributed pipelined launch: ") + hipGetErrorString(e);
        return KN_ERR_DEVICE;
    }
    const long long last = pipe_.steps() - 1;
    const int slot = ring_next_;
    ring_next_ = (ring_next_ + 1) % (int)ring_.size();
    if (hipEventRecord(ring_[slot], side_) != hipSuccess) { err_ = "hipEventRecord"; return KN_ERR_DEVICE; }
    done_.emplace_back(last, slot);
    while (done_.size() > ring_.size()) done_.pop_front();
    if (last_step) *last_step = last;
    return KN_OK;
}

kn_status DistPipeline::wait(long long step, double timeout_s, int* flag) {
    if (!ok_ || !comm_) return KN_ERR_STATE;
    hipEvent_t ev = nullptr;
    for (const auto& d : done_)
        if (d.first >= step) { ev = ring_[d.second]; break; }
    if (!ev) {
        if (done_.empty() || step > done_.back().first) { err_ = "wait() for a step not launched"; return KN_ERR_STATE; }
        ev = ring_[done_.front().second];  // older than the ring: its flag is final (sticky)
    }
    const kn_status st = poll(ev, timeout_s, "distributed step");
    if (st != KN_OK) {
        err_ = "step " + std::to_string(step) + ", " + pending_stage(step) + ": " + err_;
        return st;
    }
    if (flag) *flag = *reinterpret_cast<volatile int*>(host_flag_);
    return KN_OK;
}

std::string DistPipeline::pending_stage(long long step) const {
    const int s = (int)(step % nsets_);
    const hipEvent_t eb = pipe_.build_event(s), eq = pipe_.query_event(s);
    if (eb && hipEventQuery(eb) == hipErrorNotReady) {
        // the build stage holds the grouped send / recv: name the peers it exchanges rows with
        std::string peers;
        for (int d = 0; d < p_.world; ++d)
            if (d != p_.rank && (p_.cross_send[d] > 0 || p_.cross_recv[d] > 0))
                peers += (peers.empty() ? "" : ",") + std::to_string(d) + "(send " + std::to_string(p_.cross_send[d]) +
                         " recv " + std::to_string(p_.cross_recv[d]) + ")";
        return "stage route+exchange+build pending, peers [" + peers + "]";
    }
    if (eq && hipEventQuery(eq) == hipErrorNotReady) return "stage query pending";
    return "stage flag all-reduce pending (all " + std::to_string(p_.world) + " ranks)";
}

kn_status DistPipeline::sync() {
    if (pipe_.sync() != hipSuccess) { err_ = "distributed pipeline sync"; return KN_ERR_DEVICE; }
    return KN_OK;
}

kn_status DistPipeline::profile(float ms[5]) {
    if (!ok_ || !comm_) return KN_ERR_STATE;
    if (pipe_.sync() != hipSuccess || pipe_.unprime() != hipSuccess) { err_ = "sync"; return KN_ERR_DEVICE; }
    std::vector<hipEvent_t> ev(6, nullptr);
    for (auto& e : ev)
        if (hipEventCreate(&e) != hipSuccess) { err_ = "hipEventCreate"; return KN_ERR_DEVICE; }
    // the set the pipeline will build next is free (nothing primed): profile in it
    const int s = (int)(pipe_.steps() % nsets_);
    std::vector<hipEvent_t> marks = {ev[1], ev[2]};
    hipError_t e = hipEventRecord(ev[0], main_);
    if (e == hipSuccess) e = stage_build(s, main_, &marks);
    if (e == hipSuccess) e = hipEventRecord(ev[3], main_);
    if (e == hipSuccess) e = stage_query(s, main_);
    if (e == hipSuccess) e = hipEventRecord(ev[4], main_);
    if (e == hipSuccess) e = stage_flag(s, main_);
    if (e == hipSuccess) e = hipEventRecord(ev[5], main_);
    if (e == hipSuccess) e = hipStreamSynchronize(main_);
    for (int i = 0; i < 5 && e == hipSuccess; ++i) e = hipEventElapsedTime(&ms[i], ev[i], ev[i + 1]);
    for (auto x : ev) (void)hipEventDestroy(x);
    if (e != hipSuccess) { err_ = std::string("profile: ") + hipGetErrorString(e); return KN_ERR_DEVICE; }
    return KN_OK;
}

}  // namespace kn
