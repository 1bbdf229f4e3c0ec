// hostio_probe.cpp -- where the time of a large device -> pageable-host getter goes (900K x 17
// words = 61.2 MB at K=16): DMA rates (pinned / pageable), host copy-out into fresh malloc'd
// memory (page faults) with 1..16 threads, transparent huge pages, MADV_POPULATE_WRITE, and
// free() of the result. Build: hipcc -O2 -fopenmp --offload-arch=gfx950 scripts/hostio_probe.cpp
// -o bin/hostio_probe. Usage: bin/hostio_probe [MB] [reps]
#include <hip/hip_runtime.h>
#include <omp.h>
#include <sys/mman.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <functional>
#include <vector>

#ifndef MADV_POPULATE_WRITE
#define MADV_POPULATE_WRITE 23
#endif

static double now_ms() {
    return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

#define CK(x)                                                                       \
    do {                                                                            \
        hipError_t e_ = (x);                                                        \
        if (e_ != hipSuccess) {                                                     \
            fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));                 \
            exit(1);                                                                \
        }                                                                           \
    } while (0)

typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
__global__ void copy_kernel(const u32x4* __restrict__ src, u32x4* __restrict__ dst, size_t n4) {
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n4; i += (size_t)gridDim.x * blockDim.x)
        __builtin_nontemporal_store(src[i], &dst[i]);
}

static void par_copy(void* dst, const void* src, size_t bytes, int nt) {
#pragma omp parallel num_threads(nt)
    {
        const int t = omp_get_thread_num(), T = omp_get_num_threads();
        const size_t per = ((bytes + T - 1) / T + 4095) & ~(size_t)4095;
        const size_t a = std::min(bytes, (size_t)t * per), z = std::min(bytes, a + per);
        if (z > a) std::memcpy((char*)dst + a, (const char*)src + a, z - a);
    }
}

static void par_populate(void* p, size_t bytes, int nt) {
    // page-aligned interior, one slice per thread
    const uintptr_t lo = ((uintptr_t)p + 4095) & ~(uintptr_t)4095, hi = ((uintptr_t)p + bytes) & ~(uintptr_t)4095;
    if (hi <= lo) return;
    const size_t len = hi - lo;
#pragma omp parallel num_threads(nt)
    {
        const int t = omp_get_thread_num(), T = omp_get_num_threads();
        const size_t per = ((len + T - 1) / T + 4095) & ~(size_t)4095;
        const size_t a = std::min(len, (size_t)t * per), z = std::min(len, a + per);
        if (z > a) (void)madvise((void*)(lo + a), z - a, MADV_POPULATE_WRITE);
    }
}

static void huge(void* p, size_t bytes) {
    const uintptr_t lo = ((uintptr_t)p + (2u << 20) - 1) & ~(uintptr_t)((2u << 20) - 1);
    const uintptr_t hi = ((uintptr_t)p + bytes) & ~(uintptr_t)((2u << 20) - 1);
    if (hi > lo) (void)madvise((void*)lo, hi - lo, MADV_HUGEPAGE);
}

int main(int argc, char** argv) {
    const double mb = argc > 1 ? atof(argv[1]) : 61.2;
    const int reps = argc > 2 ? atoi(argv[2]) : 5;
    const size_t bytes = (size_t)(mb * 1e6) & ~(size_t)63;
    void* d = nullptr;
    CK(hipMalloc(&d, bytes));
    CK(hipMemset(d, 1, bytes));
    void* pin = nullptr;
    CK(hipHostMalloc(&pin, bytes, hipHostMallocDefault));
    hipStream_t s;
    CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    CK(hipDeviceSynchronize());
    std::vector<char> reused(bytes, 0);
    FILE* thp = fopen("/sys/kernel/mm/transparent_hugepage/enabled", "r");
    char tbuf[256] = {0};
    if (thp) { if (!fgets(tbuf, sizeof tbuf, thp)) tbuf[0] = 0; fclose(thp); }
    tbuf[strcspn(tbuf, "\n")] = 0;
    printf("{\"probe\": \"hostio\", \"mb\": %.1f, \"omp_max\": %d, \"thp\": \"%s\"}\n", bytes / 1e6, omp_get_max_threads(), tbuf);

    auto run = [&](const char* name, const std::function<void(double*)>& body) {
        std::vector<double> t, tf;
        for (int r = 0; r <= reps; ++r) {
            double extra = 0;
            const double a = now_ms();
            body(&extra);
            const double b = now_ms();
            if (r) { t.push_back(b - a - extra); tf.push_back(extra); }
        }
        std::sort(t.begin(), t.end());
        std::sort(tf.begin(), tf.end());
        const double m = t[t.size() / 2];
        printf("{\"case\": \"%s\", \"ms\": %.3f, \"GBps\": %.1f, \"ms_free\": %.3f}\n", name, m, bytes / 1e6 / m,
               tf[tf.size() / 2]);
        fflush(stdout);
    };
    auto timed_free = [](void* p, double* extra) { const double a = now_ms(); free(p); *extra += now_ms() - a; };

    run("dma_pinned", [&](double*) { CK(hipMemcpyAsync(pin, d, bytes, hipMemcpyDeviceToHost, s)); CK(hipStreamSynchronize(s)); });
    {
        hipStream_t ss[4];
        for (auto& x : ss) CK(hipStreamCreateWithFlags(&x, hipStreamNonBlocking));
        for (int parts : {2, 4}) {
            char nm[64];
            snprintf(nm, sizeof nm, "dma_pinned_split%d", parts);
            run(nm, [&](double*) {
                const size_t per = (bytes / parts + 4095) & ~(size_t)4095;
                for (int i = 0; i < parts; ++i) {
                    const size_t a = std::min(bytes, (size_t)i * per), z = std::min(bytes, a + per);
                    if (z > a) CK(hipMemcpyAsync((char*)pin + a, (const char*)d + a, z - a, hipMemcpyDeviceToHost, ss[i]));
                }
                for (int i = 0; i < parts; ++i) CK(hipStreamSynchronize(ss[i]));
            });
        }
        for (int blocks : {64, 256, 1024}) {
            char nm[64];
            snprintf(nm, sizeof nm, "kernel_to_pinned_b%d", blocks);
            run(nm, [&](double*) {
                copy_kernel<<<blocks, 256, 0, s>>>((const u32x4*)d, (u32x4*)pin, bytes / 16);
                CK(hipStreamSynchronize(s));
            });
        }
        for (auto& x : ss) CK(hipStreamDestroy(x));
    }
    run("dma_pageable_reused", [&](double*) { CK(hipMemcpyAsync(reused.data(), d, bytes, hipMemcpyDeviceToHost, s)); CK(hipStreamSynchronize(s)); });
    run("dma_pageable_fresh", [&](double* x) {
        void* h = malloc(bytes);
        CK(hipMemcpyAsync(h, d, bytes, hipMemcpyDeviceToHost, s));
        CK(hipStreamSynchronize(s));
        timed_free(h, x);
    });
    for (int nt : {1, 4, 8, 16}) {
        char nm[64];
        snprintf(nm, sizeof nm, "copyout_fresh_t%d", nt);
        run(nm, [&](double* x) { void* h = malloc(bytes); par_copy(h, pin, bytes, nt); timed_free(h, x); });
        snprintf(nm, sizeof nm, "copyout_fresh_huge_t%d", nt);
        run(nm, [&](double* x) { void* h = malloc(bytes); huge(h, bytes); par_copy(h, pin, bytes, nt); timed_free(h, x); });
        snprintf(nm, sizeof nm, "populate_then_copy_t%d", nt);
        run(nm, [&](double* x) { void* h = malloc(bytes); par_populate(h, bytes, nt); par_copy(h, pin, bytes, nt); timed_free(h, x); });
        snprintf(nm, sizeof nm, "copyout_reused_t%d", nt);
        run(nm, [&](double*) { par_copy(reused.data(), pin, bytes, nt); });
    }
    run("register_dma_unregister_fresh", [&](double* x) {
        void* h = malloc(bytes);
        CK(hipHostRegister(h, bytes, hipHostRegisterDefault));
        CK(hipMemcpyAsync(h, d, bytes, hipMemcpyDeviceToHost, s));
        CK(hipStreamSynchronize(s));
        CK(hipHostUnregister(h));
        timed_free(h, x);
    });
    run("mmap_populate_dma_fresh", [&](double* x) {
        // not free()-able: the ceiling of a getter that could hand out mmap'd memory
        void* h = mmap(nullptr, bytes, PROT_READ | PROT_WRITE, MAP_PRIVATE | MAP_ANONYMOUS | MAP_POPULATE, -1, 0);
        CK(hipMemcpyAsync(h, d, bytes, hipMemcpyDeviceToHost, s));
        CK(hipStreamSynchronize(s));
        const double a = now_ms();
        munmap(h, bytes);
        *x += now_ms() - a;
    });
    return 0;
}
