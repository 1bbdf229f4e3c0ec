// pipeline.cpp -- see pipeline.hpp.
#include "pipeline.hpp"

#include <cstdio>
#include <cstdlib>

namespace kn {

namespace {
#define KN_TRY(expr)                          \
    do {                                      \
        hipError_t e_ = (expr);               \
        if (e_ != hipSuccess) return e_;      \
    } while (0)

void destroy(hipGraphExec_t& g) {
    if (g) (void)hipGraphExecDestroy(g);
    g = nullptr;
}
void destroy(hipEvent_t& e) {
    if (e) (void)hipEventDestroy(e);
    e = nullptr;
}
// Flags of the events that order the pipeline's streams on the device (never waited on by the
// host). KN_EVENT_SCOPE (A/B): 0 default system-scope release, 1 device-scope release
// (hipEventReleaseToDevice), 2 no system fence (hipEventDisableSystemFence).
unsigned order_event_flags() {
    static const unsigned f = [] {
        const char* v = std::getenv("KN_EVENT_SCOPE");
        const int m = v ? std::atoi(v) : 0;
        return (unsigned)hipEventDisableTiming |
               (m == 1 ? (unsigned)hipEventReleaseToDevice : m == 2 ? (unsigned)hipEventDisableSystemFence : 0u);
    }();
    return f;
}
}  // namespace

hipError_t Pipeline::init(hipStream_t main, hipStream_t side, Stage b, Stage q, Stage r, bool capture_from_side,
                          int query_streams, int sets, hipStream_t aux, bool tail_stream) {
    reset();
    if (sets < 2 || sets > kMaxSets) return hipErrorInvalidValue;
    ns_ = sets;
    main_ = main;
    side_ = side;
    capture_from_side_ = capture_from_side;
    b_ = std::move(b);
    q_ = std::move(q);
    r_ = std::move(r);
    for (int s = 0; s < ns_; ++s) {
        for (hipEvent_t* e : {&evB_[s], &evQ_[s], &evF_[s]})
            KN_TRY(hipEventCreateWithFlags(e, order_event_flags()));
        // both sets start free
        KN_TRY(hipEventRecord(evF_[s], main_));
        KN_TRY(hipEventRecord(evQ_[s], main_));
    }
    KN_TRY(hipEventCreateWithFlags(&last_done_, hipEventDisableTiming));
    KN_TRY(hipEventRecord(last_done_, main_));
    if (tail_stream && r_) KN_TRY(hipStreamCreateWithFlags(&tail_, hipStreamNonBlocking));
    if (query_streams >= 2) {
        int lo = 0, hi = 0;
        KN_TRY(hipDeviceGetStreamPriorityRange(&lo, &hi));
        (void)hi;
        // the second query stream at the default priority, like the first (the device's least
        // priority, KN_PIPE_AUXPRIO=0, measured slower: 900K K=16 200 / 50 steps 0.276 -> 0.268
        // ms, the driver's 20 / 5 0.304 -> 0.297, K=50 0.766 -> 0.747; three interleaved passes,
        // profiles/ab_r5_stream_prio.txt)
        const char* ap = std::getenv("KN_PIPE_AUXPRIO");
        if (aux) aux_ = aux;
        else if (ap && std::atoi(ap) == 0) KN_TRY(hipStreamCreateWithPriority(&aux_, hipStreamNonBlocking, lo));
        else KN_TRY(hipStreamCreateWithFlags(&aux_, hipStreamNonBlocking));
        aux_owned_ = !aux;
        for (auto& e : evQS_) {
            KN_TRY(hipEventCreateWithFlags(&e, order_event_flags()));
            KN_TRY(hipEventRecord(e, main_));
        }
    }
    return hipSuccess;
}

void Pipeline::reset() {
    if (main_) (void)hipStreamSynchronize(main_);
    if (side_) (void)hipStreamSynchronize(side_);
    if (tail_) {
        (void)hipStreamSynchronize(tail_);
        (void)hipStreamDestroy(tail_);
        tail_ = nullptr;
    }
    for (int s = 0; s < kMaxSets; ++s) {
        destroy(gB_[s]);
        destroy(gQ_[s]);
        destroy(gR_[s]);
        destroy(evB_[s]);
        destroy(evQ_[s]);
        destroy(evF_[s]);
    }
    for (int s = 0; s < 2; ++s) {
        destroy(gU_[s]);
        gU_len_[s] = 0;
        destroy(evQS_[s]);
    }
    destroy(last_done_);
    if (aux_) {
        (void)hipStreamSynchronize(aux_);
        if (aux_owned_) (void)hipStreamDestroy(aux_);
        aux_ = nullptr;
        aux_owned_ = false;
    }
    for (auto& e : cap_ev_) destroy(e);
    cap_ev_.clear();
    main_ = side_ = nullptr;
    next_ = 0;
    primed_ = r_pending_ = false;
    last_set_ = -1;
}

hipError_t Pipeline::capture(const Stage& st, int set, hipGraphExec_t* out) {
    hipGraph_t g = nullptr;
    KN_TRY(hipStreamBeginCapture(main_, hipStreamCaptureModeThreadLocal));
    const hipError_t e1 = st(set, main_);
    const hipError_t e2 = hipStreamEndCapture(main_, &g);
    if (e1 != hipSuccess) {
        if (g) (void)hipGraphDestroy(g);
        return e1;
    }
    KN_TRY(e2);
    const hipError_t e3 = hipGraphInstantiate(out, g, nullptr, nullptr, 0);
    (void)hipGraphDestroy(g);
    // KN_PIPE_GRAPH_UPLOAD=1 (diagnostics): upload the executable graph to the device now instead
    // of at its first launches (the 20-step cold start, profiles/r6_coldstart.txt)
    static const bool upload = [] {
        const char* v = std::getenv("KN_PIPE_GRAPH_UPLOAD");
        return v && v[0] == '1';
    }();
    if (e3 == hipSuccess && upload) KN_TRY(hipGraphUpload(*out, main_));
    return e3;
}

hipError_t Pipeline::graphs() {
    if (eager_) return hipSuccess;
    for (int s = 0; s < ns_; ++s) {
        if (!gB_[s]) KN_TRY(capture(b_, s, &gB_[s]));
        if (!gQ_[s]) KN_TRY(capture(q_, s, &gQ_[s]));
        if (r_ && !gR_[s]) KN_TRY(capture(r_, s, &gR_[s]));
    }
    return hipSuccess;
}

// U steps starting at set s0, both streams in one graph. Step j: Q(j) on the main branch after
// B(j) (j = 0: built before the graph) and Q(j-1); on the side branch R(j-1) after Q(j-1), then
// B(j+1) into the set Q(j-1) released. Ends after Q(U-1) and B(U) (R(U-1) is flushed after it).
hipError_t Pipeline::unrolled(int s0, int U) {
    if (gU_[s0] && gU_len_[s0] == U) return hipSuccess;
    destroy(gU_[s0]);
    gU_len_[s0] = 0;
    const size_t need = 2 * (size_t)U + 3;
    while (cap_ev_.size() < need) {
        hipEvent_t e = nullptr;
        KN_TRY(hipEventCreateWithFlags(&e, order_event_flags()));
        cap_ev_.push_back(e);
    }
    hipEvent_t fork = cap_ev_[0], join = cap_ev_[1], join2 = cap_ev_[2];
    hipEvent_t* eq = cap_ev_.data() + 3;      // after Q(j)
    hipEvent_t* eb = cap_ev_.data() + 3 + U;  // after B(j+1)
    hipGraph_t g = nullptr;
    // origin stream of the capture; the other one joins it through the fork event
    hipStream_t origin = capture_from_side_ ? side_ : main_, other = capture_from_side_ ? main_ : side_;
    // query streams: Q(j) on qst[j & 1]. With the second query stream (KN_PIPE_QSTREAMS=2), the
    // queries of consecutive steps (different grid sets, different outputs) depend only on their
    // own builds, so step j+1's workgroups fill the CUs that step j's tail leaves idle instead of
    // waiting for its last workgroup and the kernel boundary
    hipStream_t qst[2] = {main_, aux_ ? aux_ : main_};
    // KN_PIPE_TRACE=1 (diagnostics): stderr marks around the capture's phases
    static const bool trace = [] {
        const char* v = std::getenv("KN_PIPE_TRACE");
        return v && v[0] == '1';
    }();
    if (trace) std::fprintf(stderr, "[pipeline] unrolled(%d, U=%d): begin capture (aux %d)\n", s0, U, aux_ ? 1 : 0);
    KN_TRY(hipStreamBeginCapture(origin, hipStreamCaptureModeThreadLocal));
    hipError_t e = hipEventRecord(fork, origin);
    if (e == hipSuccess) e = hipStreamWaitEvent(other, fork, 0);
    if (e == hipSuccess && aux_) e = hipStreamWaitEvent(aux_, fork, 0);
    for (int j = 0; j < U && e == hipSuccess; ++j) {
        const int s = (s0 + j) & 1;
        hipStream_t qs = qst[j & 1];
        if (j >= 1) e = hipStreamWaitEvent(qs, eb[j - 1], 0);  // B(j) (built during Q(j-1))
        if (e == hipSuccess) e = q_(s, qs);
        if (e == hipSuccess) e = hipEventRecord(eq[j], qs);
        if (e == hipSuccess && j >= 1) {
            e = hipStreamWaitEvent(side_, eq[j - 1], 0);
            if (e == hipSuccess && r_) e = r_(s ^ 1, side_);
        }
        if (e == hipSuccess) e = b_(s ^ 1, side_);
        if (e == hipSuccess) e = hipEventRecord(eb[j], side_);
    }
    if (e == hipSuccess) e = hipEventRecord(join, other);
    if (e == hipSuccess) e = hipStreamWaitEvent(origin, join, 0);
    if (e == hipSuccess && aux_) e = hipEventRecord(join2, aux_);
    if (e == hipSuccess && aux_) e = hipStreamWaitEvent(origin, join2, 0);
    if (trace) std::fprintf(stderr, "[pipeline] unrolled(%d): stages enqueued (%s), end capture\n", s0, hipGetErrorString(e));
    const hipError_t ee = hipStreamEndCapture(origin, &g);
    if (trace) std::fprintf(stderr, "[pipeline] unrolled(%d): captured (%s), instantiate\n", s0, hipGetErrorString(ee));
    if (e != hipSuccess) {
        if (g) (void)hipGraphDestroy(g);
        return e;
    }
    KN_TRY(ee);
    e = hipGraphInstantiate(&gU_[s0], g, nullptr, nullptr, 0);
    if (trace) std::fprintf(stderr, "[pipeline] unrolled(%d): instantiated (%s)\n", s0, hipGetErrorString(e));
    (void)hipGraphDestroy(g);
    if (e == hipSuccess) gU_len_[s0] = U;
    return e;
}

// Eager mode runs the stage bodies directly on the streams (same stages, same event order as
// the graphs): nothing is captured, so a stage whose calls cannot be captured (RCCL at world > 1
// by default, dist.cpp) or whose capture failed still runs.
hipError_t Pipeline::enqueue_build(int s) {
    // without an epilogue the set is free once its query is done
    KN_TRY(hipStreamWaitEvent(side_, r_ ? evF_[s] : evQ_[s], 0));
    KN_TRY(eager_ ? b_(s, side_) : hipGraphLaunch(gB_[s], side_));
    return hipEventRecord(evB_[s], side_);
}

hipError_t Pipeline::enqueue_query(int s) {
    // with two query streams, consecutive STEPS alternate streams (whatever the number of sets)
    const int qi = (aux_ && (next_ & 1)) ? 1 : 0;
    hipStream_t qs = qi ? aux_ : main_;
    KN_TRY(hipStreamWaitEvent(qs, evB_[s], 0));
    KN_TRY(eager_ ? q_(s, qs) : hipGraphLaunch(gQ_[s], qs));
    KN_TRY(hipEventRecord(evQ_[s], qs));
    last_qs_ = qi;
    return aux_ ? hipEventRecord(evQS_[qi], qs) : hipSuccess;
}

hipError_t Pipeline::enqueue_epilogue(int s) {
    hipStream_t rs = rstream();
    KN_TRY(hipStreamWaitEvent(rs, evQ_[s], 0));
    KN_TRY(eager_ ? r_(s, rs) : hipGraphLaunch(gR_[s], rs));
    return hipEventRecord(evF_[s], rs);
}

hipError_t Pipeline::prepare(int unroll) {
    if (!main_) return hipErrorNotInitialized;
    if (eager_) return hipSuccess;
    KN_TRY(graphs());
    if (unroll >= 2 && !(unroll & 1) && ns_ == 2 && !aux_) {  // (launch() runs unrolled graphs only then)
        KN_TRY(unrolled(0, unroll));
        KN_TRY(unrolled(1, unroll));
    }
    return hipSuccess;
}

void Pipeline::set_eager(bool eager) {
    if (eager == eager_) return;
    if (main_) (void)hipStreamSynchronize(main_);
    if (side_) (void)hipStreamSynchronize(side_);
    if (aux_) (void)hipStreamSynchronize(aux_);
    if (tail_) (void)hipStreamSynchronize(tail_);
    // a failed capture may have left a stream in capture mode: end it (the graph is dropped)
    for (hipStream_t st : {main_, side_}) {
        hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
        if (st && hipStreamIsCapturing(st, &cs) == hipSuccess && cs != hipStreamCaptureStatusNone) {
            hipGraph_t g = nullptr;
            (void)hipStreamEndCapture(st, &g);
            if (g) (void)hipGraphDestroy(g);
        }
    }
    (void)hipGetLastError();
    for (int s = 0; s < kMaxSets; ++s) {
        destroy(gB_[s]);
        destroy(gQ_[s]);
        destroy(gR_[s]);
    }
    for (int s = 0; s < 2; ++s) {
        destroy(gU_[s]);
        gU_len_[s] = 0;
    }
    eager_ = eager;
}

hipError_t Pipeline::flush() {
    if (r_pending_) {
        r_pending_ = false;
        KN_TRY(enqueue_epilogue(last_set_));
        return hipEventRecord(last_done_, rstream());
    }
    if (!r_ && last_set_ >= 0) {
        hipStream_t ql = last_qs_ ? aux_ : main_;
        // both query streams' last queries (they do not depend on each other) before last_done
        if (aux_) KN_TRY(hipStreamWaitEvent(ql, evQS_[last_qs_ ^ 1], 0));
        return hipEventRecord(last_done_, ql);
    }
    return hipSuccess;
}

hipError_t Pipeline::fallback_if(hipError_t e) {
    if (e == hipSuccess) return e;
    // a capture or instantiation failed (nothing ran): the same stages eagerly from now on
    set_eager(true);
    ++fallbacks_;
    return hipSuccess;
}

hipError_t Pipeline::launch(int iters, int unroll, bool keep_primed) {
    if (!main_) return hipErrorNotInitialized;
    KN_TRY(fallback_if(graphs()));
    if (unroll < 2 || (unroll & 1) || eager_) unroll = 0;
    // Two query streams run per-step graphs: a graph whose queries alternate between two streams
    // crashes the HIP runtime from 4 unrolled steps on (ROCm 7.0: unbounded recursion in
    // libamdhip64 while capturing, profiles/r5_qstreams.txt), and 2-step graphs measured slower
    // than per-step launches (900K K=16, 200 steps: 0.2828 vs 0.2756 ms; one query stream with
    // 10-step graphs 0.2894)
    // (KN_PIPE_UNROLL_QS2=1, diagnostics: capture the unrolled graphs with both query streams anyway;
    // tools/repro_capture.hip is the standalone reproducer, profiles/r6_capture_repro.txt)
    static const bool force_qs2 = [] {
        const char* v = std::getenv("KN_PIPE_UNROLL_QS2");
        return v && v[0] == '1';
    }();
    if ((aux_ && !force_qs2) || ns_ != 2) unroll = 0;
    if (unroll) {
        // both start parities up front (also by a call of fewer steps, e.g. a warm-up): a capture
        // never lands inside a later (timed) call
        hipError_t e = unrolled(0, unroll);
        if (e == hipSuccess) e = unrolled(1, unroll);
        KN_TRY(fallback_if(e));
        if (eager_) unroll = 0;
    }
    int done = 0;
    while (done < iters) {
        const int s = (int)(next_ % ns_);
        // an unrolled graph ends with the next step's build: only when the call keeps it primed,
        // or more steps follow in this call
        if (unroll && iters - done >= unroll + (keep_primed ? 0 : 1)) {
            if (!primed_) KN_TRY(enqueue_build(s));
            if (r_pending_) {
                r_pending_ = false;
                KN_TRY(enqueue_epilogue(last_set_));
            }
            // the graph's first query reads set s (built on the side stream); its first build
            // writes set s^1, released by the last query (main, stream order) and R (side)
            KN_TRY(hipStreamWaitEvent(main_, evB_[s], 0));
            if (r_) KN_TRY(hipStreamWaitEvent(main_, evF_[s ^ 1], 0));
            KN_TRY(hipGraphLaunch(gU_[s], main_));
            // U is even: the last query used set s^1, the primed build (B(next)) wrote set s.
            // Every per-set event is re-recorded after the graph: its queries read both sets and
            // its last epilogue inside it (R(U-2)) released set s, so a later step_with() or build
            // of either set waits for the whole graph (not for a stale pre-graph event)
            last_set_ = s ^ 1;
            KN_TRY(hipEventRecord(evQ_[s ^ 1], main_));
            KN_TRY(hipEventRecord(evQ_[s], main_));
            KN_TRY(hipEventRecord(evB_[s], main_));
            if (r_) KN_TRY(hipEventRecord(evF_[s], main_));
            primed_ = true;
            r_pending_ = (bool)r_;
            next_ += unroll;
            done += unroll;
            continue;
        }
        if (!primed_) KN_TRY(enqueue_build(s));
        KN_TRY(enqueue_query(s));
        if (r_pending_) {  // R(i-1) (last_set_ is still step i-1's set)
            r_pending_ = false;
            KN_TRY(enqueue_epilogue(last_set_));
        }
        last_set_ = s;
        if (keep_primed || done + 1 < iters) {
            KN_TRY(enqueue_build((s + 1) % ns_));  // B(i+1) overlaps Q(i)
            primed_ = true;
        } else {
            primed_ = false;
        }
        r_pending_ = (bool)r_;
        ++next_;
        ++done;
    }
    return flush();
}

hipError_t Pipeline::step_with(const Stage& pre, const Stage* next_pre) {
    if (!main_) return hipErrorNotInitialized;
    KN_TRY(fallback_if(graphs()));
    const int s = (int)(next_ % ns_);
    const int sn = (s + 1) % ns_;
    if (!primed_) {
        // this step's input into set s, then its build
        KN_TRY(hipStreamWaitEvent(side_, r_ ? evF_[s] : evQ_[s], 0));
        KN_TRY(pre(s, side_));
        KN_TRY(enqueue_build(s));
    }
    KN_TRY(enqueue_query(s));
    if (r_pending_) {
        r_pending_ = false;
        KN_TRY(enqueue_epilogue(last_set_));
    }
    last_set_ = s;
    primed_ = false;
    if (next_pre) {
        KN_TRY(hipStreamWaitEvent(side_, r_ ? evF_[sn] : evQ_[sn], 0));
        KN_TRY((*next_pre)(sn, side_));
        KN_TRY(enqueue_build(sn));
        primed_ = true;
    }
    r_pending_ = (bool)r_;
    ++next_;
    return flush();
}

hipError_t Pipeline::sync() {
    if (!main_) return hipSuccess;
    if (aux_) KN_TRY(hipStreamSynchronize(aux_));
    if (tail_) KN_TRY(hipStreamSynchronize(tail_));
    KN_TRY(hipStreamSynchronize(side_));
    return hipStreamSynchronize(main_);
}

hipError_t Pipeline::unprime() {
    if (!main_) return hipSuccess;
    KN_TRY(hipStreamSynchronize(side_));
    if (tail_) KN_TRY(hipStreamSynchronize(tail_));
    primed_ = false;
    return hipSuccess;
}

}  // namespace kn
