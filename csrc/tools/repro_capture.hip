// repro_capture.hip -- standalone reproducer (plain hipcc: no torch, no RCCL) of the unrolled
// pipeline capture that crashed inside the HIP runtime with two query streams (DESIGN.md round 5,
// profiles/r5_capture_crash.txt).
//
// The capture has exactly kn::Pipeline::unrolled's event pattern (csrc/runtime/pipeline.cpp:143-195)
// with empty kernels for the stages: three streams (main = capture origin, side = builds, aux =
// second query stream), U steps; step j: Q(j) on qst[j & 1] after B(j) (event eb[j-1]); then,
// on the side stream, after Q(j-1) (event eq[j-1]) the optional epilogue R(j-1), and B(j+1).
//   repro_capture [U=4] [aux=1] [epilogue=0] [build_kernels=5] [query_kernels=2] [from_side=0] [captures=2] [pre=1]
// captures = 2: both start parities are captured with the SAME events, one after the other, as
// Pipeline::launch does (unrolled(0), unrolled(1)). Run it against torch's bundled HIP runtime
// (LD_LIBRARY_PATH=<torch>/lib) to match the extension's process: the round-5 crash was there.
// Prints "captured ... launched ... ok" or dies (a host crash inside the runtime is a segfault:
// exit status 139).
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                                                      \
    do {                                                                                           \
        hipError_t e_ = (x);                                                                       \
        if (e_ != hipSuccess) {                                                                    \
            std::fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
            return 1;                                                                              \
        }                                                                                          \
    } while (0)

__global__ void empty_kernel(int* p, int v) {
    if (p && threadIdx.x == 0 && blockIdx.x == 0) p[0] = v;
}

int main(int argc, char** argv) {
    const int U = argc > 1 ? std::atoi(argv[1]) : 4;
    const bool use_aux = argc > 2 ? std::atoi(argv[2]) != 0 : true;
    const bool use_r = argc > 3 ? std::atoi(argv[3]) != 0 : false;
    const int nb = argc > 4 ? std::atoi(argv[4]) : 5;
    const int nq = argc > 5 ? std::atoi(argv[5]) : 2;
    const bool from_side = argc > 6 ? std::atoi(argv[6]) != 0 : false;
    const int ncap = argc > 7 ? std::atoi(argv[7]) : 2;
    // pre = 1: first capture every stage alone on the main stream, per set (Pipeline::graphs()),
    // as launch() does before the unrolled captures
    const bool pre = argc > 8 ? std::atoi(argv[8]) != 0 : true;
    int rtv = 0, drv = 0;
    CK(hipRuntimeGetVersion(&rtv));
    CK(hipDriverGetVersion(&drv));
    std::printf("HIP runtime %d driver %d; U=%d aux=%d epilogue=%d build_kernels=%d query_kernels=%d "
                "capture_from_side=%d captures=%d pre=%d\n", rtv, drv, U, use_aux, use_r, nb, nq, from_side, ncap, pre);
    std::fflush(stdout);
    int* d = nullptr;
    CK(hipMalloc(&d, 64 * sizeof(int)));
    hipStream_t main_s, side_s, aux_s = nullptr;
    CK(hipStreamCreateWithFlags(&main_s, hipStreamNonBlocking));
    CK(hipStreamCreateWithFlags(&side_s, hipStreamNonBlocking));
    if (use_aux) CK(hipStreamCreateWithFlags(&aux_s, hipStreamNonBlocking));
    auto stage = [&](int kernels, int tag, hipStream_t s) {
        for (int i = 0; i < kernels; ++i) empty_kernel<<<4, 64, 0, s>>>(d, tag * 16 + i);
        return hipGetLastError();
    };
    std::vector<hipEvent_t> ev(2 * (size_t)U + 3);
    for (auto& e : ev) CK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
    hipEvent_t fork = ev[0], join = ev[1], join2 = ev[2];
    hipEvent_t* eq = ev.data() + 3;
    hipEvent_t* eb = ev.data() + 3 + U;
    hipStream_t origin = from_side ? side_s : main_s, other = from_side ? main_s : side_s;
    hipStream_t qst[2] = {main_s, aux_s ? aux_s : main_s};
    std::vector<hipGraphExec_t> execs;
    if (pre) {
        for (int set = 0; set < 2; ++set)
            for (int kind = 0; kind < (use_r ? 3 : 2); ++kind) {
                hipGraph_t g = nullptr;
                CK(hipStreamBeginCapture(main_s, hipStreamCaptureModeThreadLocal));
                CK(stage(kind == 0 ? nb : kind == 1 ? nq : 1, 10 + kind, main_s));
                CK(hipStreamEndCapture(main_s, &g));
                hipGraphExec_t gx = nullptr;
                CK(hipGraphInstantiate(&gx, g, nullptr, nullptr, 0));
                CK(hipGraphDestroy(g));
                execs.push_back(gx);
            }
        std::printf("per-stage graphs: %zu\n", execs.size());
    }
    for (int c = 0; c < ncap; ++c) {
    hipGraph_t g = nullptr;
    CK(hipStreamBeginCapture(origin, hipStreamCaptureModeThreadLocal));
    CK(hipEventRecord(fork, origin));
    CK(hipStreamWaitEvent(other, fork, 0));
    if (aux_s) CK(hipStreamWaitEvent(aux_s, fork, 0));
    for (int j = 0; j < U; ++j) {
        hipStream_t qs = qst[j & 1];
        if (j >= 1) CK(hipStreamWaitEvent(qs, eb[j - 1], 0));
        CK(stage(nq, 1, qs));
        CK(hipEventRecord(eq[j], qs));
        if (j >= 1) {
            CK(hipStreamWaitEvent(side_s, eq[j - 1], 0));
            if (use_r) CK(stage(1, 2, side_s));
        }
        CK(stage(nb, 3, side_s));
        CK(hipEventRecord(eb[j], side_s));
    }
    CK(hipEventRecord(join, other));
    CK(hipStreamWaitEvent(origin, join, 0));
    if (aux_s) {
        CK(hipEventRecord(join2, aux_s));
        CK(hipStreamWaitEvent(origin, join2, 0));
    }
    CK(hipStreamEndCapture(origin, &g));
    size_t nodes = 0;
    CK(hipGraphGetNodes(g, nullptr, &nodes));
    std::printf("capture %d: %zu nodes\n", c, nodes);
    std::fflush(stdout);
    hipGraphExec_t gx = nullptr;
    CK(hipGraphInstantiate(&gx, g, nullptr, nullptr, 0));
    CK(hipGraphDestroy(g));
    std::printf("instantiated %d\n", c);
    std::fflush(stdout);
    execs.push_back(gx);
    }
    for (int i = 0; i < 3; ++i)
        for (auto gx : execs) CK(hipGraphLaunch(gx, main_s));
    CK(hipStreamSynchronize(main_s));
    std::printf("launched 3x: ok\n");
    for (auto gx : execs) CK(hipGraphExecDestroy(gx));
    for (auto e : ev) CK(hipEventDestroy(e));
    CK(hipFree(d));
    return 0;
}
