// hostio.cpp -- staged pageable copies and the device arena cache (see hostio.hpp).
#include "hostio.hpp"

#include <omp.h>
#include <sys/mman.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <vector>

namespace kn {

namespace {

constexpr size_t kChunk = 4u << 20;       // bytes per staging slot
constexpr size_t kDirectBelow = 1u << 20;  // smaller copies skip the ring

bool env_on(const char* name, bool dflt) {
    const char* v = std::getenv(name);
    return v ? std::atoi(v) != 0 : dflt;
}

// Parallel host memcpy in 256 KiB blocks (page-fault and bandwidth bound on freshly malloc'd
// destinations: one thread reaches ~6-10 GB/s).
void par_memcpy(void* dst, const void* src, size_t bytes) {
    constexpr size_t kBlk = 256u << 10;
    const long nb = (long)((bytes + kBlk - 1) / kBlk);
    const int nt = std::max(1, std::min(16, omp_get_max_threads()));
    if (nb <= 1 || nt == 1) { std::memcpy(dst, src, bytes); return; }
#pragma omp parallel for num_threads(nt) schedule(static)
    for (long b = 0; b < nb; ++b) {
        const size_t off = (size_t)b * kBlk;
        std::memcpy((char*)dst + off, (const char*)src + off, std::min(kBlk, bytes - off));
    }
}

struct Ring {
    std::mutex mu;
    void* slot[2] = {nullptr, nullptr};
    hipEvent_t ev[2] = {nullptr, nullptr};
    bool pending[2] = {false, false};
    int dev = -1;

    hipError_t ready() {
        hipError_t e = hipSuccess;
        if (!slot[0]) {
            for (auto& p : slot)
                if ((e = hipHostMalloc(&p, kChunk, hipHostMallocDefault)) != hipSuccess) return e;
        }
        int d = 0;
        if ((e = hipGetDevice(&d)) != hipSuccess) return e;
        if (d != dev) {
            for (int i = 0; i < 2; ++i) {
                if (ev[i]) {
                    if (pending[i]) (void)hipEventSynchronize(ev[i]);
                    (void)hipEventDestroy(ev[i]);
                    ev[i] = nullptr;
                }
                pending[i] = false;
                if ((e = hipEventCreateWithFlags(&ev[i], hipEventDisableTiming)) != hipSuccess) return e;
            }
            dev = d;
        }
        return e;
    }
    hipError_t wait(int i) {
        if (!pending[i]) return hipSuccess;
        pending[i] = false;
        return hipEventSynchronize(ev[i]);
    }
};

Ring& ring() {
    static Ring* r = new Ring();  // never destroyed: pinned memory is released at process exit
    return *r;
}

struct Cached {
    int dev;
    void* p;
    size_t bytes;
};
std::mutex g_pool_mu;
std::vector<Cached> g_pool;
constexpr size_t kPoolMaxBytes = 4ull << 30;
constexpr int kPoolPerDevice = 8;  // an engine's arena + its result / tree buffers

}  // namespace

hipError_t copy_h2d_staged(void* d, const void* h, size_t bytes, hipStream_t s) {
    if (bytes < kDirectBelow || !env_on("KN_HOST_STAGE", false))
        return hipMemcpyAsync(d, h, bytes, hipMemcpyHostToDevice, s);
    Ring& r = ring();
    std::lock_guard<std::mutex> lock(r.mu);
    hipError_t e = r.ready();
    if (e != hipSuccess) return hipMemcpyAsync(d, h, bytes, hipMemcpyHostToDevice, s);
    int i = 0;
    for (size_t off = 0; off < bytes; off += kChunk, i ^= 1) {
        const size_t len = std::min(kChunk, bytes - off);
        if ((e = r.wait(i)) != hipSuccess) return e;  // the slot's previous DMA has drained
        par_memcpy(r.slot[i], (const char*)h + off, len);
        if ((e = hipMemcpyAsync((char*)d + off, r.slot[i], len, hipMemcpyHostToDevice, s)) != hipSuccess) return e;
        if ((e = hipEventRecord(r.ev[i], s)) != hipSuccess) return e;
        r.pending[i] = true;
    }
    return hipSuccess;
}

// Large device -> pageable host copies (the reference getters' malloc'd results): one pinned
// buffer sized to the copy (grow-only, process-wide, <= kBigMax), every chunk's DMA enqueued at
// once (the copy engine streams at PCIe rate), and a team of host threads copying each chunk out
// as soon as its event completes -- the host copy overlaps the DMA of the later chunks. The
// destination's 2 MiB-aligned interior is advised to transparent huge pages first: a freshly
// malloc'd result faults one 2 MiB page per first touch instead of 512 4 KiB ones (61 MB copy-out
// with 8 threads 0.74-0.81 ms vs 3.6-4.4 ms, its free() 2.4-3.0 vs 4.8-7.2 ms; DMA 1.08 ms at
// 56 GB/s; scripts/hostio_probe.cpp, profiles/r4_hostio_probe.txt). The destination is faulted
// in before the first chunk lands (900K K=16 getter 1.69 -> 1.54 ms median, faster in all 6
// interleaved pairs; profiles/api_r4_getter_prefault.jsonl).
namespace {
constexpr size_t kBigChunk = 16u << 20;
constexpr size_t kHuge = 2u << 20;
void advise_huge(void* p, size_t bytes) {
    const uintptr_t lo = ((uintptr_t)p + kHuge - 1) & ~(uintptr_t)(kHuge - 1);
    const uintptr_t hi = ((uintptr_t)p + bytes) & ~(uintptr_t)(kHuge - 1);
    if (hi > lo) (void)madvise((void*)lo, hi - lo, MADV_HUGEPAGE);  // advice only: errors ignored
}
constexpr size_t kBigMax = 1ull << 30;
constexpr int kBigEvents = (int)(kBigMax / kBigChunk);
struct BigStage {
    std::mutex mu;
    void* buf = nullptr;
    size_t cap = 0;
    std::vector<hipEvent_t> ev;
    int dev = -1;
};
BigStage& big() {
    static BigStage* b = new BigStage();  // never destroyed: pinned memory is released at exit
    return *b;
}
}  // namespace

static hipError_t copy_d2h_big(void* h, const void* d, size_t bytes, hipStream_t s) {
    // KN_GET_TRACE=1: enqueue / first chunk ready / last chunk ready / done, on stderr
    static const bool trace = env_on("KN_GET_TRACE", false);
    using clk = std::chrono::steady_clock;
    const auto t0 = clk::now();
    clk::time_point t_enq, t_first, t_last;
    BigStage& b = big();
    std::lock_guard<std::mutex> lock(b.mu);
    hipError_t e;
    int dev = 0;
    if ((e = hipGetDevice(&dev)) != hipSuccess) return e;
    if (b.cap < bytes) {
        if (b.buf) (void)hipHostFree(b.buf);
        b.buf = nullptr;
        b.cap = 0;
        const size_t want = std::min(kBigMax, std::max(bytes, (size_t)64 << 20));
        if ((e = hipHostMalloc(&b.buf, want, hipHostMallocDefault)) != hipSuccess) return e;
        b.cap = want;
    }
    if (b.dev != dev) {
        for (auto x : b.ev) (void)hipEventDestroy(x);
        b.ev.clear();
        b.dev = dev;
    }
    const size_t nchunks = (bytes + kBigChunk - 1) / kBigChunk;
    while (b.ev.size() < nchunks) {
        hipEvent_t x = nullptr;
        if ((e = hipEventCreateWithFlags(&x, hipEventDisableTiming)) != hipSuccess) return e;
        b.ev.push_back(x);
    }
    for (size_t c = 0; c < nchunks; ++c) {
        const size_t off = c * kBigChunk, len = std::min(kBigChunk, bytes - off);
        if ((e = hipMemcpyAsync((char*)b.buf + off, (const char*)d + off, len, hipMemcpyDeviceToHost, s)) != hipSuccess)
            return e;
        if ((e = hipEventRecord(b.ev[c], s)) != hipSuccess) return e;
    }
    t_enq = clk::now();
    advise_huge(h, bytes);
    // 8 threads: the copy-out's best on MI355X hosts (16 contend for the page-fault path;
    // KN_COPY_THREADS, A/B)
    static const int copy_threads = [] {
        const char* v = std::getenv("KN_COPY_THREADS");
        const int t = v ? std::atoi(v) : 8;
        return (t >= 1 && t <= 64) ? t : 8;
    }();
    // KN_COPY_PREFAULT (default on): every thread first faults in its slices of the destination
    // (one store per 4 KiB page) while the first chunk's DMA is still in flight, so the copy-out
    // of each chunk runs at the memcpy rate of mapped pages instead of zeroing fresh huge pages
    // behind the DMA
    static const bool prefault = env_on("KN_COPY_PREFAULT", true);
    const int nt = std::max(1, std::min(copy_threads, omp_get_max_threads()));
    hipError_t err = hipSuccess;
#pragma omp parallel num_threads(nt)
    {
        const int t = omp_get_thread_num(), T = omp_get_num_threads();
        auto slice = [&](size_t c, uintptr_t* a, uintptr_t* z) {
            const size_t off = c * kBigChunk, len = std::min(kBigChunk, bytes - off);
            // slices cut at 2 MiB boundaries of the destination address: every huge page is
            // touched (faulted in) by one thread only
            const uintptr_t beg = (uintptr_t)h + off, end = beg + len, per = (len + T - 1) / T;
            auto cut = [&](int i) -> uintptr_t {
                if (i <= 0) return beg;
                if (i >= T) return end;
                return std::min(end, (beg + (uintptr_t)i * per + kHuge - 1) & ~(uintptr_t)(kHuge - 1));
            };
            *a = cut(t);
            *z = cut(t + 1);
        };
        if (prefault)
            for (size_t c = 0; c < nchunks; ++c) {
                uintptr_t a, z;
                slice(c, &a, &z);
                for (uintptr_t p = a; p < z; p = (p & ~(uintptr_t)4095) + 4096) *(volatile char*)p = 0;
            }
        for (size_t c = 0; c < nchunks; ++c) {
#pragma omp single
            {
                const hipError_t x = hipEventSynchronize(b.ev[c]);
                if (x != hipSuccess) err = x;
                if (trace) (c == 0 ? t_first : t_last) = clk::now();
            }  // implicit barrier: the chunk is in pinned memory
            if (err != hipSuccess) continue;
            uintptr_t a, z;
            slice(c, &a, &z);
            if (z > a) std::memcpy((void*)a, (const char*)b.buf + (a - (uintptr_t)h), z - a);
        }
    }
    if (trace) {
        auto ms = [&](clk::time_point t) { return std::chrono::duration<double, std::milli>(t - t0).count(); };
        fprintf(stderr, "copy_d2h_big %.1f MB: enqueued %.3f, chunk0 %.3f, last %.3f, done %.3f ms\n", bytes / 1e6,
                ms(t_enq), ms(t_first), nchunks > 1 ? ms(t_last) : ms(t_first), ms(clk::now()));
    }
    return err;
}

hipError_t copy_d2h_staged(void* h, const void* d, size_t bytes, hipStream_t s) {
    // big copies: the pinned whole-copy path (KN_HOST_BIG=0: off)
    if (bytes >= (4u << 20) && bytes <= kBigMax && env_on("KN_HOST_BIG", true)) return copy_d2h_big(h, d, bytes, s);
    if (bytes < kDirectBelow || !env_on("KN_HOST_STAGE", false)) {
        hipError_t e = hipMemcpyAsync(h, d, bytes, hipMemcpyDeviceToHost, s);
        return e != hipSuccess ? e : hipStreamSynchronize(s);
    }
    Ring& r = ring();
    std::lock_guard<std::mutex> lock(r.mu);
    hipError_t e = r.ready();
    if (e != hipSuccess) {
        if ((e = hipMemcpyAsync(h, d, bytes, hipMemcpyDeviceToHost, s)) != hipSuccess) return e;
        return hipStreamSynchronize(s);
    }
    for (int i = 0; i < 2; ++i)
        if ((e = r.wait(i)) != hipSuccess) return e;
    const size_t nchunks = (bytes + kChunk - 1) / kChunk;
    auto issue = [&](size_t c) -> hipError_t {
        const int i = (int)(c & 1);
        const size_t off = c * kChunk, len = std::min(kChunk, bytes - off);
        hipError_t x = hipMemcpyAsync(r.slot[i], (const char*)d + off, len, hipMemcpyDeviceToHost, s);
        if (x != hipSuccess) return x;
        if ((x = hipEventRecord(r.ev[i], s)) != hipSuccess) return x;
        r.pending[i] = true;
        return hipSuccess;
    };
    if ((e = issue(0)) != hipSuccess) return e;
    for (size_t c = 0; c < nchunks; ++c) {
        // chunk c + 1 streams into the other slot while the host drains chunk c
        if (c + 1 < nchunks && (e = issue(c + 1)) != hipSuccess) return e;
        const int i = (int)(c & 1);
        if ((e = r.wait(i)) != hipSuccess) return e;
        const size_t off = c * kChunk, len = std::min(kChunk, bytes - off);
        par_memcpy((char*)h + off, r.slot[i], len);
    }
    return hipSuccess;
}

void* arena_acquire(int device, size_t bytes, size_t* got) {
    if (!env_on("KN_ARENA_CACHE", true)) return nullptr;
    std::lock_guard<std::mutex> lock(g_pool_mu);
    int best = -1;
    for (int i = 0; i < (int)g_pool.size(); ++i) {
        const Cached& c = g_pool[i];
        if (c.dev == device && c.bytes >= bytes && c.bytes <= 2 * bytes + (64u << 20) &&
            (best < 0 || c.bytes < g_pool[best].bytes))
            best = i;
    }
    if (best < 0) return nullptr;
    void* p = g_pool[best].p;
    *got = g_pool[best].bytes;
    g_pool.erase(g_pool.begin() + best);
    return p;
}

void arena_release(int device, void* p, size_t bytes) {
    if (!p) return;
    if (env_on("KN_ARENA_CACHE", true)) {
        std::lock_guard<std::mutex> lock(g_pool_mu);
        size_t total = bytes;
        int same = 0;
        for (const Cached& c : g_pool) {
            total += c.bytes;
            same += c.dev == device ? 1 : 0;
        }
        if (total <= kPoolMaxBytes && same < kPoolPerDevice) {
            g_pool.push_back({device, p, bytes});
            return;
        }
    }
    int cur = 0;
    (void)hipGetDevice(&cur);
    (void)hipSetDevice(device);
    (void)hipFree(p);
    (void)hipSetDevice(cur);
}

namespace {
std::mutex g_ss_mu;
std::vector<std::pair<int, StreamSet>> g_ss;  // key: device * 2 + priority
}  // namespace

hipError_t streamset_acquire(int device, StreamSet* out, int priority) {
    const int key = device * 2 + (priority ? 1 : 0);
    {
        std::lock_guard<std::mutex> lock(g_ss_mu);
        for (size_t i = 0; i < g_ss.size(); ++i)
            if (g_ss[i].first == key) {
                *out = g_ss[i].second;
                g_ss.erase(g_ss.begin() + (long)i);
                return hipSuccess;
            }
    }
    StreamSet s;
    hipError_t e;
    if (priority) {
        int least = 0, greatest = 0;
        e = hipDeviceGetStreamPriorityRange(&least, &greatest);
        // 1: the device's greatest priority, 2: its least (KN_PIPE_PRIO)
        if (e == hipSuccess)
            e = hipStreamCreateWithPriority(&s.stream, hipStreamNonBlocking, priority == 2 ? least : greatest);
    } else {
        e = hipStreamCreateWithFlags(&s.stream, hipStreamNonBlocking);
    }
    for (auto& ev : s.ev)
        if (e == hipSuccess) e = hipEventCreate(&ev);
    if (e != hipSuccess) {
        for (auto& ev : s.ev) if (ev) (void)hipEventDestroy(ev);
        if (s.stream) (void)hipStreamDestroy(s.stream);
        return e;
    }
    *out = s;
    return hipSuccess;
}

void streamset_release(int device, const StreamSet& s, int priority) {
    if (!s.stream) return;
    const int key = device * 2 + (priority ? 1 : 0);
    {
        std::lock_guard<std::mutex> lock(g_ss_mu);
        int same = 0;
        for (const auto& p : g_ss) same += p.first == key ? 1 : 0;
        if (same < 8) { g_ss.emplace_back(key, s); return; }
    }
    for (auto ev : s.ev) if (ev) (void)hipEventDestroy(ev);
    (void)hipStreamDestroy(s.stream);
}

hipError_t device_malloc(void** p, size_t bytes) {
    hipError_t e = hipMalloc(p, bytes);
    if (e != hipErrorOutOfMemory) return e;
    // blocks parked in the cache (up to kPoolPerDevice per device, kPoolMaxBytes in all) may be
    // what the device is missing: give them back and retry once
    (void)hipGetLastError();
    arena_release_all();
    return hipMalloc(p, bytes);
}

void arena_release_all() {
    std::lock_guard<std::mutex> lock(g_pool_mu);
    int cur = 0;
    (void)hipGetDevice(&cur);
    for (const Cached& c : g_pool) {
        (void)hipSetDevice(c.dev);
        (void)hipFree(c.p);
    }
    g_pool.clear();
    (void)hipSetDevice(cur);
}

}  // namespace kn
