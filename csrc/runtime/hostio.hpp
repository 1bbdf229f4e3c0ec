// hostio.hpp -- host <-> device transfers of PAGEABLE host memory and a device arena cache, for the
// reference-API path (kn_prepare from host points, the malloc'd getters; reference
// knearests.cu:205-231 gpuMalloc* helpers and :410-438 getters).
//
// * Staged copies (opt-in, KN_HOST_STAGE=1): a process-wide pinned ring (2 slots x 4 MiB,
//   allocated once); host memcpy of chunk i into a slot (OpenMP threads) overlaps the DMA of chunk
//   i-1. Measured on MI355X (profiles/api_r3_host_staging.jsonl): kn_get_knearests 3.34 -> 2.82 ms
//   at K=16 but 7.9 -> 14.3 ms at K=50, and the whole prepare/solve/get/free cycle slower (the
//   runtime's own pageable path already streams at 17-23 GB/s): off by default.
// * Device block cache: kn_free / Engine teardown parks the engine's device arena and result /
//   tree buffers (at most 8 blocks per device, <= 4 GiB in total) and the next Engine takes a block
//   of a size it fits (within 2x + 64 MiB) instead of hipMalloc; a kn_prepare / kn_solve / kn_free
//   cycle then allocates and frees nothing on the device (hipFree of the 3 N x K result buffers
//   alone took ~7 ms per kn_free at 900K, K=16). KN_ARENA_CACHE=0 disables it,
//   kn_release_cached_memory() frees it.
#pragma once

#include <hip/hip_runtime.h>
#include <stddef.h>

namespace kn {

// Stream-ordered copy of `bytes` from pageable host memory into device memory. Returns once the
// host buffer may be reused (the last chunks may still be in flight on `s`).
hipError_t copy_h2d_staged(void* d, const void* h, size_t bytes, hipStream_t s);
// Copy from device memory (stream-ordered after earlier work on `s`) into pageable host memory;
// returns when the host buffer holds the data.
hipError_t copy_d2h_staged(void* h, const void* d, size_t bytes, hipStream_t s);

// Device block cache (see above). acquire: a cached block of >= bytes (and <= 2 x bytes + 64 MiB)
// on `device`, or nullptr; *got = its size. release: park or free.
void* arena_acquire(int device, size_t bytes, size_t* got);
void arena_release(int device, void* p, size_t bytes);
void arena_release_all();
// hipMalloc that, on hipErrorOutOfMemory, frees every parked cache block and retries once (the
// cache must never be why an allocation fails)
hipError_t device_malloc(void** p, size_t bytes);

// Stream + 4 timing events of an engine from a per-device pool (creating a HIP stream and its
// events cost 2-8 ms per kn_prepare on MI355X, measured with KN_PREP_TIMING): acquire creates when
// the pool is empty; release parks up to 8 sets per device (the stream must be idle).
struct StreamSet {
    hipStream_t stream = nullptr;
    hipEvent_t ev[4] = {nullptr, nullptr, nullptr, nullptr};
};
// priority: 0 = default, 1 = the device's highest stream priority (pooled separately)
hipError_t streamset_acquire(int device, StreamSet* out, int priority = 0);
void streamset_release(int device, const StreamSet& s, int priority = 0);

}  // namespace kn
