// valu_rate.hip -- VALU issue-rate calibration for gfx950 (MI355X).
//
// Question ("roofline mis-calibrated"): how many SIMD cycles does one wave64 VALU
// instruction cost, for the instruction classes the kNN query kernel's hot loop is made of
// (v_med3_u32 insertion network, v_fma_f32 distance, v_bfi_b32 key pack, VOP2 integer ops,
// packed f32), and how does that change with the number of waves per SIMD?
//
// Method: every wave runs 8 independent register chains of one instruction (inline asm, so the
// compiler can neither fold nor reorder them), 64 instructions per loop trip. The grid puts W
// waves on each of the chip's SIMDs at once (256-thread blocks = 4 waves, one per SIMD; 256*W
// blocks). Wall time from hipEvents; the shader clock from s_memtime / s_memrealtime (100 MHz)
// stamped by wave 0 of block 0 around its loop. Reported: SIMD cycles per wave-instruction
//   = wall * f_clk / (W * trips * 64)   (one SIMD's share of the instruction stream).
// The SQ counters SQ_ACTIVE_INST_VALU / SQ_INSTS_VALU count per-wave quad-cycles, so they alone
// cannot tell a 2-cycle SIMD-32 issue from a 4-cycle one once several waves share a SIMD.
//
// Build: hipcc -O3 --offload-arch=gfx950 csrc/tools/valu_rate.hip -o bin/valu_rate
// Run:   bin/valu_rate [trips]     (prints one JSON line per (op, waves/SIMD))
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

#define CHECK(x)                                                                              \
    do {                                                                                      \
        hipError_t e_ = (x);                                                                  \
        if (e_ != hipSuccess) {                                                               \
            std::fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
            std::exit(1);                                                                     \
        }                                                                                     \
    } while (0)

enum Op {
    MED3 = 0, FMA, PKFMA, BFI, MINU, CNDMASK, ADDF,
    MED3F, MINF, MAX3F, ADDU, ANDB, ORB, MOVB, CNDSG, MULF, SUBF, LSHL, CMPF, MED3I, MAXU, NOPS
};
static const char* kName[NOPS] = {"v_med3_u32", "v_fma_f32", "v_pk_fma_f32", "v_bfi_b32", "v_min_u32",
                                  "v_cndmask_b32(vcc from s_mov)", "v_add_f32", "v_med3_f32", "v_min_f32",
                                  "v_max3_f32", "v_add_u32", "v_and_b32", "v_or_b32", "v_mov_b32",
                                  "v_cndmask_b32(sgpr mask)", "v_mul_f32", "v_sub_f32", "v_lshlrev_b32",
                                  "v_cmp_lt_f32(e64)", "v_med3_i32", "v_max_u32"};

template <int OP>
__device__ __forceinline__ void step(unsigned& a, unsigned b, unsigned c) {
    if constexpr (OP == MED3) asm volatile("v_med3_u32 %0, %0, %1, %2" : "+v"(a) : "v"(b), "v"(c));
    if constexpr (OP == FMA) asm volatile("v_fma_f32 %0, %0, %1, %2" : "+v"(a) : "v"(b), "v"(c));
    if constexpr (OP == BFI) asm volatile("v_bfi_b32 %0, %1, %0, %2" : "+v"(a) : "v"(b), "v"(c));
    if constexpr (OP == MINU) asm volatile("v_min_u32 %0, %0, %1" : "+v"(a) : "v"(b));
    if constexpr (OP == CNDMASK) asm volatile("v_cndmask_b32 %0, %0, %1, vcc" : "+v"(a) : "v"(b));
    if constexpr (OP == ADDF) asm volatile("v_add_f32 %0, %0, %1" : "+v"(a) : "v"(b));
    if constexpr (OP == MED3F) asm volatile("v_med3_f32 %0, %0, %1, %2" : "+v"(a) : "v"(b), "v"(c));
    if constexpr (OP == MINF) asm volatile("v_min_f32 %0, %0, %1" : "+v"(a) : "v"(b));
    if constexpr (OP == MAX3F) asm volatile("v_max3_f32 %0, %0, %1, %2" : "+v"(a) : "v"(b), "v"(c));
    if constexpr (OP == ADDU) asm volatile("v_add_u32 %0, %0, %1" : "+v"(a) : "v"(b));
    if constexpr (OP == ANDB) asm volatile("v_and_b32 %0, %0, %1" : "+v"(a) : "v"(b));
    if constexpr (OP == ORB) asm volatile("v_or_b32 %0, %0, %1" : "+v"(a) : "v"(b));
    if constexpr (OP == MOVB) asm volatile("v_mov_b32 %0, %1" : "=v"(a) : "v"(a));
    if constexpr (OP == MULF) asm volatile("v_mul_f32 %0, %0, %1" : "+v"(a) : "v"(b));
    if constexpr (OP == SUBF) asm volatile("v_sub_f32 %0, %0, %1" : "+v"(a) : "v"(b));
    if constexpr (OP == LSHL) asm volatile("v_lshlrev_b32 %0, 1, %0" : "+v"(a));
    if constexpr (OP == MED3I) asm volatile("v_med3_i32 %0, %0, %1, %2" : "+v"(a) : "v"(b), "v"(c));
    if constexpr (OP == MAXU) asm volatile("v_max_u32 %0, %0, %1" : "+v"(a) : "v"(b));
}

template <int OP>
__global__ __launch_bounds__(256) void rate_kernel(unsigned* out, int trips, unsigned long long* clk) {
    unsigned a[8];
    const unsigned b = threadIdx.x * 3u + 1u, c = 0x3f800000u ^ threadIdx.x;
#pragma unroll
    for (int i = 0; i < 8; ++i) a[i] = threadIdx.x + 17u * i;
    unsigned long long t0 = 0, r0 = 0;
    const bool stamp = blockIdx.x == 0 && threadIdx.x == 0;
    if (stamp) { t0 = __builtin_amdgcn_s_memtime(); r0 = __builtin_amdgcn_s_memrealtime(); }
    if constexpr (OP == PKFMA) {
        // 8 independent 64-bit register pairs, v_pk_fma_f32 on each
        typedef float f2 __attribute__((ext_vector_type(2)));
        f2 p[8];
        const f2 pb = {__uint_as_float(b), __uint_as_float(c)}, pc = {1.0f, 2.0f};
#pragma unroll
        for (int i = 0; i < 8; ++i) p[i] = f2{__uint_as_float(a[i]), __uint_as_float(a[i] ^ 5u)};
        for (int t = 0; t < trips; ++t) {
#pragma unroll
            for (int r = 0; r < 8; ++r)
#pragma unroll
                for (int i = 0; i < 8; ++i) asm volatile("v_pk_fma_f32 %0, %0, %1, %2" : "+v"(p[i]) : "v"(pb), "v"(pc));
        }
#pragma unroll
        for (int i = 0; i < 8; ++i) a[i] = __float_as_uint(p[i].x) ^ __float_as_uint(p[i].y);
    } else if constexpr (OP == CNDSG || OP == CMPF) {
        // the realistic select: mask in an SGPR pair written by a VALU compare (v_cmp_*_e64)
        unsigned long long m;
        asm volatile("v_cmp_lt_u32_e64 %0, %1, %2" : "=s"(m) : "v"(b), "v"(c));
        for (int t = 0; t < trips; ++t) {
#pragma unroll
            for (int r = 0; r < 8; ++r)
#pragma unroll
                for (int i = 0; i < 8; ++i) {
                    if constexpr (OP == CNDSG)
                        asm volatile("v_cndmask_b32_e64 %0, %0, %1, %2" : "+v"(a[i]) : "v"(b), "s"(m));
                    else {
                        unsigned long long mm;
                        asm volatile("v_cmp_lt_f32_e64 %0, %1, %2" : "=s"(mm) : "v"(a[i]), "v"(b));
                        a[i] ^= (unsigned)(mm >> 40);  // keeps every compare live (SALU)
                    }
                }
        }
    } else {
        if constexpr (OP == CNDMASK) asm volatile("s_mov_b64 vcc, exec" ::: "vcc");
        for (int t = 0; t < trips; ++t) {
#pragma unroll
            for (int r = 0; r < 8; ++r)
#pragma unroll
                for (int i = 0; i < 8; ++i) step<OP>(a[i], b, c);
        }
    }
    if (stamp) {
        clk[0] = __builtin_amdgcn_s_memtime() - t0;
        clk[1] = __builtin_amdgcn_s_memrealtime() - r0;
    }
    unsigned x = 0;
#pragma unroll
    for (int i = 0; i < 8; ++i) x ^= a[i];
    if (x == 0x12345679u) out[blockIdx.x * 256 + threadIdx.x] = x;  // keeps the chains live
}

template <int OP>
static void run(int cus, int trips, unsigned* out, unsigned long long* clk) {
    const int wps[] = {1, 2, 4, 8};
    for (int w : wps) {
        const int blocks = cus * w;
        hipEvent_t e0, e1;
        CHECK(hipEventCreate(&e0));
        CHECK(hipEventCreate(&e1));
        // warm-up (clocks ramp), then timed launches
        for (int i = 0; i < 3; ++i) rate_kernel<OP><<<blocks, 256>>>(out, trips, clk);
        CHECK(hipGetLastError());
        const int reps = 5;
        CHECK(hipEventRecord(e0));
        for (int i = 0; i < reps; ++i) rate_kernel<OP><<<blocks, 256>>>(out, trips, clk);
        CHECK(hipEventRecord(e1));
        CHECK(hipEventSynchronize(e1));
        float ms = 0.f;
        CHECK(hipEventElapsedTime(&ms, e0, e1));
        ms /= reps;
        unsigned long long hc[2];
        CHECK(hipMemcpy(hc, clk, sizeof(hc), hipMemcpyDeviceToHost));
        const double ghz = hc[1] ? (double)hc[0] / (double)hc[1] * 0.1 : 0.0;  // memrealtime = 100 MHz
        const double insts = (double)w * trips * 64.0;                         // per SIMD
        const double cyc = ms * 1e-3 * ghz * 1e9 / insts;
        std::printf("{\"op\": \"%s\", \"waves_per_simd\": %d, \"ms\": %.4f, \"clock_ghz\": %.3f, "
                    "\"simd_cycles_per_wave_inst\": %.3f, \"wave_inst_per_s_chip\": %.4g}\n",
                    kName[OP], w, ms, ghz, cyc, (double)blocks * 4 * trips * 64.0 / (ms * 1e-3));
        std::fflush(stdout);
        CHECK(hipEventDestroy(e0));
        CHECK(hipEventDestroy(e1));
    }
}

int main(int argc, char** argv) {
    const int trips = argc > 1 ? std::atoi(argv[1]) : 20000;
    hipDeviceProp_t prop;
    CHECK(hipGetDeviceProperties(&prop, 0));
    const int cus = prop.multiProcessorCount;
    std::fprintf(stderr, "%s: %d CUs, trips %d\n", prop.gcnArchName, cus, trips);
    unsigned* out;
    unsigned long long* clk;
    CHECK(hipMalloc(&out, (size_t)cus * 8 * 256 * sizeof(unsigned)));
    CHECK(hipMalloc(&clk, 2 * sizeof(unsigned long long)));
    run<MED3>(cus, trips, out, clk);
    run<FMA>(cus, trips, out, clk);
    run<PKFMA>(cus, trips, out, clk);
    run<BFI>(cus, trips, out, clk);
    run<MINU>(cus, trips, out, clk);
    run<CNDMASK>(cus, trips, out, clk);
    run<ADDF>(cus, trips, out, clk);
    run<MED3F>(cus, trips, out, clk);
    run<MINF>(cus, trips, out, clk);
    run<MAX3F>(cus, trips, out, clk);
    run<ADDU>(cus, trips, out, clk);
    run<ANDB>(cus, trips, out, clk);
    run<ORB>(cus, trips, out, clk);
    run<MOVB>(cus, trips, out, clk);
    run<CNDSG>(cus, trips, out, clk);
    run<MULF>(cus, trips, out, clk);
    run<SUBF>(cus, trips, out, clk);
    run<LSHL>(cus, trips, out, clk);
    run<CMPF>(cus, trips, out, clk);
    run<MED3I>(cus, trips, out, clk);
    run<MAXU>(cus, trips, out, clk);
    CHECK(hipFree(out));
    CHECK(hipFree(clk));
    return 0;
}
