// hostio.hpp -- host <-> device transfers of PAGEABLE host memory and a device arena cache, for the
// reference-API path (kn_prepare from host points, the malloc'd getters; reference
// knearests.cu:205-231 gpuMalloc* helpers and :410-438 getters).
//
// * Staged copies: a process-wide pinned ring (2 slots x 4 MiB, allocated once). Host memcpy of
//   chunk i into a slot (OpenMP threads) overlaps the DMA of chunk i-1; the runtime's own pageable
//   path copies through its staging buffer with one thread. Copies below 1 MiB go direct.
// * Arena cache: kn_free / Engine teardown parks the engine's device arena (at most 2 per device,
//   <= 4 GiB in total) and the next Engine of a size it fits (within 2x) takes it instead of
//   hipMalloc + hipFree per kn_prepare. KN_ARENA_CACHE=0 disables it, kn_release_cached_memory()
//   frees it.
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

// Device arena cache (see above). acquire: a cached block of >= bytes (and <= 2 x bytes) on
// `device`, or nullptr; *got = its size. release: park or free.
void* arena_acquire(int device, size_t bytes, size_t* got);
void arena_release(int device, void* p, size_t bytes);
void arena_release_all();

}  // namespace kn
