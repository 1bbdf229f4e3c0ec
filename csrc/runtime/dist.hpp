// dist.hpp -- one rank's pipelined distributed step over RCCL (NEW: the reference is single-GPU,
// knearests.cu has no streams, devices or collectives).
//
// One process per GPU. After a validated full step (parallel/distributed.py: global domain, rank
// boxes, halo width, split sizes), every steady step is the 1-GPU pipelined step plus the
// communication, all in hipGraphs replayed by kn::Pipeline (pipeline.hpp):
//   B(i)  side stream   route this rank's share (owner + halo destinations, its own rows placed
//                       straight into the local set) -> grouped ncclSend / ncclRecv of the rows
//                       that change rank -> unpack -> local grid build (global ids in the points)
//   Q(i)  main stream   queries of the owned points (the tile kernel, or the Morton-leaf tree
//                       path + complete-box certification)
//   R(i)  side stream   exact finish of the tile kernel's fallback list -> the step's flag (share /
//                       counts as planned, all rows certified) -> ncclAllReduce(MAX) -> sticky flag
//                       in pinned host memory
// B(i+1), with its all-to-all, runs while Q(i) fills the chip; both RCCL calls live on the side
// stream, in the same order on every rank (one communicator, no cross-stream collectives).
#pragma once

#include <hip/hip_runtime.h>

#include <deque>
#include <string>
#include <utility>
#include <vector>

#include "knearests.h"
#include "kn/kernels.h"
#include "kn/route.h"
#include "kn/tree.h"
#include "pipeline.hpp"

namespace kn {

// One rank's RCCL communicator (ncclComm_t behind an opaque pointer, so this header needs no RCCL
// include). The ranks share the 128-byte unique id through their own channel (the Python layer
// all-gathers it over torch.distributed).
struct RankComm {
    void* comm = nullptr;
    int world = 0, rank = 0, device = 0;
    bool aborted = false;
};
constexpr int kCommIdBytes = 128;
bool comm_unique_id(unsigned char out[kCommIdBytes], std::string* err);
RankComm* comm_create(const unsigned char id[kCommIdBytes], int world, int rank, int device, std::string* err);
void comm_destroy(RankComm* c);
// ncclCommGetAsyncError: "" when healthy
std::string comm_async_error(RankComm* c);
void comm_abort(RankComm* c);

// The validated steady plan (a full step's routing decisions, parallel/distributed.py _steady).
struct DistPlan {
    int world = 1, rank = 0, k = 16, device = 0;
    int n = 0;                       // points of this rank's share (every step)
    const float* points = nullptr;   // device (n x 3), read in place by every step
    const int* ids = nullptr;        // device (n) global ids, or null: id offset + i
    const void* route = nullptr;     // device RouteParams of the validated step (copied)
    std::vector<double> hdr;         // kPlanHdr plan header doubles
    const double* metas = nullptr;   // device (world x 8) metas of the validated step (copied)
    std::vector<int> tot;            // 2*world planned (owned, halo) send counts
    int grid[3] = {1, 1, 1};         // rank grid
    int dims[3] = {1, 1, 1};         // local grid dims of the validated step (maybe refined)
    int use_tree = 0;
    float ppc = 0.f;
    int deterministic = 1;
    int exact_grid = 0;
    int cap = 0;                     // send buffer rows
    std::vector<int> recv_own, recv_halo, cross_send, cross_recv;
    int place[5] = {0, 0, 0, 0, 0};  // SelfPlace: own_base, halo_base, rows, own count, halo count
    // world 1, forced collectives: the rank's own rows go through an RCCL self send / recv and
    // the unpack instead of straight into the local set (exercises the exchange on one GPU)
    int self_via_comm = 0;
    // halo field plan (hdr[22] != 0): the certified radii of the field cells (device, G^3 floats,
    // alive as long as the pipeline); the route plan holds the width field's pointer itself
    const float* cert_field = nullptr;
    int field_g = 0;
};

class DistPipeline {
public:
    // comm == nullptr: LOOPBACK mode (tests): no communicator, no graphs -- the caller drives one
    // eager step per rank through loopback_stage() and moves the rows between the ranks' send /
    // receive buffers itself (one process, W virtual ranks on one GPU), which checks the send /
    // receive layouts, the unpack table and the local solve against the torch path at world > 1.
    DistPipeline(const DistPlan& p, RankComm* comm);
    ~DistPipeline();
    DistPipeline(const DistPipeline&) = delete;
    DistPipeline& operator=(const DistPipeline&) = delete;
    const std::string& error() const { return err_; }
    bool ok() const { return ok_; }

    // Construction is LOCAL (plan checks, allocation, streams): nothing collective runs, so a rank
    // whose construction fails can tell its peers before any of them enters a collective.
    // warmup(): one eager step (collective; RCCL connects to the step's peers), waited for under
    // the deadline while polling RCCL's async error. Required before launch().
    kn_status warmup(double timeout_s);
    // Capture every stage graph and both unrolled graphs now (nothing runs). On failure the
    // pipeline stays eager and an error is returned; callers all-reduce the outcome and pick one
    // mode for every rank. Until this succeeds the stages run eagerly (the default at world > 1:
    // RCCL point-to-point calls inside graphs have never run on more than one rank here).
    kn_status prepare_graphs(int unroll);
    void set_eager(bool eager);
    bool eager() const { return pipe_.eager(); }
    // Read the steps' input from other device buffers (ids null: id offset + i): a caller passing a
    // fresh tensor every step keeps its pipeline, without anything collective. Eager stages read
    // the new pointers at once; captured graphs hold the old ones, so a graph-mode pipeline
    // switches to eager (one wait for the streams, once). A share of another size n routes at most
    // the planned rows and fails the step's flag on every rank. The launch() caller-stream
    // ordering still covers the old buffers' last reads.
    kn_status rebind(const float* points, const int* ids, int n);
    int capture_fallbacks() const { return pipe_.fallbacks(); }
    // Enqueue `iters` pipelined steps (unroll >= 2, even: steps per graph launch); *last_step = the
    // index of the last one. The steps read the caller's points in place: `caller` (may be null)
    // is the stream that wrote them -- the first build waits for it, and it waits (on the device)
    // for the builds that read them. keep_primed: also enqueue the next step's build now (the
    // caller promises the points stay unchanged until the next launch).
    kn_status launch(int iters, int unroll, bool keep_primed, hipStream_t caller, long long* last_step);
    // Wait (polling RCCL's async error, at most timeout_s) until step `step`'s flag is final;
    // *flag = the sticky flag (0: every step so far valid).
    kn_status wait(long long step, double timeout_s, int* flag);
    kn_status sync();
    int last_set() const { return pipe_.last_set(); }
    int sets() const { return nsets_; }
    // One serial step on the main stream with events between its phases (ms): route, exchange,
    // unpack + build, query (tile kernel / tree + certification), epilogue (exact finish, flag,
    // all-reduce). Unprimes the pipeline.
    kn_status profile(float ms[5]);

    // loopback mode: stage 0 = route (send buffer + own rows placed), 1 = unpack + build + query
    // + the step's local flag (no all-reduce); set 0 is used; synchronous
    kn_status loopback_stage(int stage);
    float4* send_rows(int s) const { return set_[s].send; }
    float4* recv_rows(int s) const { return set_[s].recv; }
    long long send_offset(int d) const { return soff_[d]; }
    long long recv_offset(int src) const { return roff_[src]; }
    int flag_local(int s) const;  // synchronous read of set s's flag word

    int rows() const { return rows_; }
    int n_owned() const { return n_owned_; }
    int k() const { return p_.k; }
    // buffers of set s (the last step: last_set()); valid until the step after next
    const int* gids(int s) const { return set_[s].lgids; }
    const int* idx(int s) const { return set_[s].idx; }
    const float* d2(int s) const { return set_[s].d2; }
    const unsigned* counters(int s) const { return set_[s].counters; }
    const int* totals(int s) const { return set_[s].totals; }
    int share_rows() const { return p_.n; }
    const unsigned* partials(int s) const { return set_[s].partials; }

private:
    struct Set {
        char* block;
        float4* send; int* bc; int* totals; unsigned* partials; float4* recv;
        float* lpts; int* lgids;
        unsigned* bbox; GridGeom* geom; int* cell_count; int* cell_scan; int* block_sums; int* cell_start;
        float4* bin_tmp; float4* sorted; unsigned* perm;
        unsigned* fallback; unsigned* counters; unsigned* uncert;
        int* idx; float* d2; int* flag; unsigned* ticket;
        void* tree_ws; void* tree_nodes;
    };
    hipError_t stage_build(int s, hipStream_t st, const std::vector<hipEvent_t>* marks = nullptr);
    hipError_t stage_query(int s, hipStream_t st);
    hipError_t stage_tail(int s, hipStream_t st);  // tail mode: the exact finish + the step's flag
    hipError_t stage_flag(int s, hipStream_t st);  // epilogue: exact finish, flag, all-reduce
    hipError_t step_flag(int s, hipStream_t st);   // deferred mode: local flag -> pending_
    StepFlagJob step_flag_job(int s) const;        // step_flag's arguments (fused into the exact kernel)
    QueryBuffers query_proto(int s) const;
    // wait for `ev`, polling RCCL's async error; past the deadline the communicator is aborted
    kn_status poll(hipEvent_t ev, double timeout_s, const char* what);
    // which stage of step `step` is still pending (route + exchange + build with its peers /
    // query / flag all-reduce): prefixed to wait()'s error, so a CollectiveError names it
    std::string pending_stage(long long step) const;
    hipError_t exchange(int s, hipStream_t st);
    bool fail(const std::string& m) { err_ = m; ok_ = false; return false; }

    DistPlan p_;
    RankComm* comm_;
    std::string err_;
    bool ok_ = false;
    bool warm_ = false;
    int rows_ = 0, n_owned_ = 0, C_ = 0;
    int n_route_ = 0, n_flag_ = 0;  // rows routed per step / the share's true size (rebind)
    int rows_cross_ = 0, recv_rows_ = 0;
    std::vector<long long> soff_, roff_;  // send / recv row offsets per peer
    UnpackTable table_{};
    BuildBuffers bproto_{};
    QueryBuffers qproto_{};
    CompleteBox complete_{};
    Set set_[Pipeline::kMaxSets]{};
    int nsets_ = 2;
    void* route_dev_ = nullptr;
    double* metas_dev_ = nullptr;
    int* tot_dev_ = nullptr;
    int* sticky_ = nullptr;
    // deferred flag reduction (two query streams): every step's flag is max-accumulated on the
    // device (pending_, atomic), one all-reduce per launch() call into reduced_ then the sticky flag
    bool deferred_ = false;
    // deferred mode, KN_DIST_TAIL=1 (opt-in): the exact finish and the step's flag run as the
    // pipeline's epilogue on a stream of their own, so a query stream's next tile follows its tile
    bool tail_ = false;
    // deferred grid steps (KN_DIST_FUSED_FLAG, default on): the step's check runs in the exact
    // finish kernel's last workgroup (QueryBuffers::step_flag) instead of two kernels after it
    bool fused_flag_ = false;
    StepFlagJob* jobs_dev_ = nullptr;  // per set, device copies of step_flag_job (upload_jobs)
    hipError_t upload_jobs();
    int* pending_ = nullptr;
    int* reduced_ = nullptr;
    int* host_flag_ = nullptr;      // pinned
    int* host_flag_dev_ = nullptr;  // its device pointer
    hipStream_t main_ = nullptr, side_ = nullptr;
    Pipeline pipe_;
    // host waits: (last step covered, event) ring, recorded after each launch's last epilogue
    std::vector<hipEvent_t> ring_;
    hipEvent_t in_ev_ = nullptr;  // the caller's input is ready
    std::deque<std::pair<long long, int>> done_;
    int ring_next_ = 0;
};

}  // namespace kn
