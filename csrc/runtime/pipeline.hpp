// pipeline.hpp -- two-set software pipeline over two HIP streams (used by kn::Engine and the
// distributed rank pipeline, kn::DistPipeline).
//
// The reference runs one cloud at a time: kn_prepare (bin) then kn_solve (query), serially on the
// default stream (knearests.cu:235-392). Here step i works on buffer set s = i & 1 in up to three
// stages, each captured once per set into a hipGraph:
//   B(i)  side stream  produce set s (bin the cloud; distributed: route + exchange + bin)
//   Q(i)  main stream  consume set s (the queries)
//   R(i)  side stream  optional epilogue after Q(i) (distributed: all-reduce of the step's flag)
// B(i+1) runs on the side stream while Q(i) fills the chip: set s^1 is free once Q(i-1) and
// R(i-1) are done. The latency-bound binning kernels hide in the query's shadow.
//
// Priming. A call enqueues, per step, Q(i) and the NEXT step's build B(i+1). In resident mode
// (every step reads the same input buffer) the pipeline stays primed between calls: a call of U
// steps enqueues U queries and U builds and starts with a query, as a continuous stream would.
// A changed input (or new stages) unprimes it; the next call then builds first.
//
// Unrolled launches (unroll U >= 2, even): U steps per graph, captured across both streams
// (fork / join through events), so consecutive queries follow each other inside one graph launch
// instead of paying a graph launch + cross-stream event per step.
#pragma once

#include <hip/hip_runtime.h>

#include <functional>
#include <vector>

namespace kn {

class Pipeline {
public:
    using Stage = std::function<hipError_t(int set, hipStream_t s)>;
    Pipeline() = default;
    ~Pipeline() { reset(); }
    Pipeline(const Pipeline&) = delete;
    Pipeline& operator=(const Pipeline&) = delete;

    // Stages (r may be empty). Streams stay owned by the caller. Graphs are captured lazily.
    // capture_from_side: unrolled captures start on the side stream (the main stream joins it):
    // RCCL point-to-point calls in the build stage crash when captured on a JOINED stream
    // (measured on MI355X, RCCL 2.26.6), so the stages with collectives must be on the origin.
    // query_streams = 2: the queries of odd sets go to a second (pipeline-owned) stream, so a
    // step's queries need not wait for the previous step's last workgroups: each depends only on
    // its own build (sets, counters and outputs are per set)
    // sets = 3: step i uses set i % 3, so step i+1's build waits for step i-2's query instead of
    // step i-1's (with two query streams two queries are in flight; the build of the next step
    // then need not wait for the older of them). Unrolled graphs need 2 sets and one query stream.
    static constexpr int kMaxSets = 3;
    // aux (query_streams = 2): an existing stream for the odd steps' queries (not owned, e.g. a
    // second pipeline over the same grid sets sharing the first one's), else one is created
    // tail_stream: the epilogue R runs on a pipeline-owned stream of its own instead of the side
    // stream (it then delays neither the next build nor the next query on its query stream)
    hipError_t init(hipStream_t main, hipStream_t side, Stage b, Stage q, Stage r = Stage(),
                    bool capture_from_side = false, int query_streams = 1, int sets = 2,
                    hipStream_t aux = nullptr, bool tail_stream = false);
    hipStream_t aux_stream() const { return aux_; }
    int sets() const { return ns_; }
    bool ready() const { return main_ != nullptr; }
    // Enqueue `iters` resident-mode steps; unroll >= 2 (even): whole groups of `unroll` steps go
    // through one unrolled graph, the rest through per-step graphs. keep_primed = false: the call
    // ends without the next step's build (its input may change before the next call).
    hipError_t launch(int iters, int unroll = 0, bool keep_primed = true);
    // Capture every stage graph (and both unrolled graphs when unroll >= 2, even) now, without
    // running anything: a capture error surfaces here, before any step is enqueued, so a caller
    // can decide (collectively, over several ranks) to run eagerly instead. No-op in eager mode.
    hipError_t prepare(int unroll);
    // Eager mode: the stage bodies are enqueued directly on the two streams at every step (same
    // stages, same event order, nothing captured). Switching waits for both streams and drops the
    // captured graphs (ending a capture a failed stage left open).
    void set_eager(bool eager);
    bool eager() const { return eager_; }
    // captures that failed inside launch() / step_with() and switched the pipeline to eager mode
    int fallbacks() const { return fallbacks_; }
    // Event recorded after the most recent build of set s (its input has been read).
    hipEvent_t build_event(int s) const { return evB_[s]; }
    // Event recorded after the most recent query of set s (diagnostics: which stage is pending)
    hipEvent_t query_event(int s) const { return evQ_[s]; }
    // One step whose input is provided by `pre` (run on the side stream before B, e.g. a copy of
    // the step's cloud into set s's input buffer); `next_pre` != null: also the next step's input
    // is known, so its build is enqueued now (overlapping this step's queries). Unprimes the
    // resident state.
    hipError_t step_with(const Stage& pre, const Stage* next_pre);
    // R(i) of the last step when it is still pending (launch() and step_with() end with it).
    hipError_t flush();
    // Wait for both streams.
    hipError_t sync();
    // Drop the primed build (the input it read changed): waits for the side stream.
    hipError_t unprime();
    int last_set() const { return last_set_; }
    long long steps() const { return next_; }
    // Event recorded after the last step's final stage (R if present, else Q).
    hipEvent_t last_done() const { return last_done_; }
    // Destroy graphs and events (init() again before the next launch).
    void reset();

private:
    hipError_t graphs();          // per-set stage graphs
    hipError_t fallback_if(hipError_t capture_error);
    hipError_t unrolled(int start_set, int U);
    hipError_t capture(const Stage& st, int set, hipGraphExec_t* out);
    hipError_t enqueue_build(int set);   // side: wait set free, B(set), record evB
    hipError_t enqueue_query(int set);   // query stream of the set: wait evB, Q(set), record evQ

    hipError_t enqueue_epilogue(int set);

    hipStream_t main_ = nullptr, side_ = nullptr;
    hipStream_t aux_ = nullptr;  // second query stream of the unrolled graphs (KN_PIPE_QSTREAMS=2)
    bool aux_owned_ = false;
    hipStream_t tail_ = nullptr;  // epilogue stream (init tail_stream), else R runs on side_
    hipStream_t rstream() const { return tail_ ? tail_ : side_; }
    bool capture_from_side_ = false;
    bool eager_ = false;
    int fallbacks_ = 0;
    Stage b_, q_, r_;
    int ns_ = 2;  // grid sets
    hipGraphExec_t gB_[kMaxSets] = {}, gQ_[kMaxSets] = {}, gR_[kMaxSets] = {};
    hipGraphExec_t gU_[2] = {nullptr, nullptr};
    int gU_len_[2] = {0, 0};
    hipEvent_t evB_[kMaxSets] = {};  // set built
    hipEvent_t evQ_[kMaxSets] = {};  // set queried
    hipEvent_t evF_[kMaxSets] = {};  // set free (after Q and R)
    hipEvent_t evQS_[2] = {nullptr, nullptr};  // tail of each query stream (two query streams)
    int last_qs_ = 0;                          // query stream of the last query
    hipEvent_t last_done_ = nullptr;
    std::vector<hipEvent_t> cap_ev_;  // fork / join events of the unrolled captures
    long long next_ = 0;       // index of the next step to query
    bool primed_ = false;      // B(next_) enqueued (resident input)
    bool r_pending_ = false;   // R(next_ - 1) not yet enqueued
    int last_set_ = -1;
};

}  // namespace kn
