// cu_mask_probe.hip -- which XCD / CU runs the work of a stream created with a one-bit CU mask
// (hipExtStreamCreateWithCUMask), so a CU partition between the build and query streams can be
// spread evenly over the 8 XCDs (kn::Pipeline).
//
// For every mask bit i < multiProcessorCount: a stream whose mask holds only bit i runs 64
// one-wave workgroups; each records HW_REG_XCC_ID and HW_REG_HW_ID (vector stores). Prints one
// line per bit: its first workgroup's XCC / SE / SH / CU, and how many distinct (xcc, se, sh, cu)
// and XCCs its 64 workgroups saw (1 = the mask pinned them to one CU).
//   hipcc --offload-arch=gfx950 -O2 csrc/tools/cu_mask_probe.hip -o bin/cu_mask_probe
#include <hip/hip_runtime.h>

#include <cstdio>
#include <set>
#include <utility>
#include <vector>

#define CK(x)                                                                             \
    do {                                                                                  \
        hipError_t e_ = (x);                                                              \
        if (e_ != hipSuccess) {                                                           \
            std::fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
            return 1;                                                                     \
        }                                                                                 \
    } while (0)

__global__ void where_kernel(unsigned* out) {
    unsigned xcc, hw;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(hw));
    if (threadIdx.x == 0) {
        out[2 * blockIdx.x] = xcc;
        out[2 * blockIdx.x + 1] = hw;
    }
}

int main() {
    hipDeviceProp_t prop;
    CK(hipGetDeviceProperties(&prop, 0));
    const int ncu = prop.multiProcessorCount;
    const int words = (ncu + 31) / 32;
    constexpr int kBlocks = 64;
    unsigned* d = nullptr;
    CK(hipMalloc(&d, 2 * kBlocks * sizeof(unsigned)));
    std::vector<unsigned> h(2 * kBlocks);
    std::printf("# %s, %d CUs\n", prop.gcnArchName, ncu);
    for (int bit = 0; bit < ncu; ++bit) {
        std::vector<uint32_t> mask(words, 0u);
        mask[bit / 32] = 1u << (bit % 32);
        hipStream_t s;
        CK(hipExtStreamCreateWithCUMask(&s, (uint32_t)words, mask.data()));
        CK(hipMemsetAsync(d, 0xff, 2 * kBlocks * sizeof(unsigned), s));
        where_kernel<<<kBlocks, 64, 0, s>>>(d);
        CK(hipGetLastError());
        CK(hipMemcpyAsync(h.data(), d, h.size() * sizeof(unsigned), hipMemcpyDeviceToHost, s));
        CK(hipStreamSynchronize(s));
        CK(hipStreamDestroy(s));
        // HW_ID: [11:8] cu_id, [12] sh_id, [14:13] se_id (tg / vm / queue ids above vary per launch)
        std::set<std::pair<unsigned, unsigned>> seen;
        std::set<unsigned> xccs;
        for (int b = 0; b < kBlocks; ++b) {
            seen.insert({h[2 * b], (h[2 * b + 1] >> 8) & 0x7fu});
            xccs.insert(h[2 * b]);
        }
        const unsigned w = (h[1] >> 8) & 0x7fu;
        std::printf("%d xcc %u se %u sh %u cu %u distinct %zu xccs %zu\n", bit, h[0], (w >> 5) & 3u, (w >> 4) & 1u,
                    w & 15u, seen.size(), xccs.size());
    }
    CK(hipFree(d));
    return 0;
}
