/*
 * knearests.h -- public C API of the MI355X-native k-nearest-neighbour engine.
 *
 * Source-compatible with the reference API (reference knearests.h:3-29):
 *   kn_problem, kn_prepare, kn_solve, kn_free, kn_get_points, kn_get_knearests,
 *   kn_get_permutation, kn_print_stats
 * with the same index-space semantics (reference knearests.cu:129,145 / test_knearests.cu:158):
 *   - kn_get_points()      : points in *stored* (cell-bucketed) order,
 *   - kn_get_permutation() : perm[stored] = original index,
 *   - kn_get_knearests()   : N x K uint32, row i = neighbours of stored point i, values are
 *                            stored indices, ascending by distance, self excluded,
 *                            UINT_MAX marks slots that could not be filled (N <= K).
 * Getters return malloc()'d host buffers that the caller releases with free().
 *
 * Extensions (not in the reference): runtime K and tuning (kn_config / kn_prepare_ex),
 * squared distances (kn_get_distances), original-order results (kn_get_neighbors),
 * per-phase timings and counters (kn_get_stats), error codes instead of exit()
 * (kn_last_error), re-solve without rebuild (kn_set_k), binary save/load of the binned
 * structure (kn_save / kn_load).
 */
#pragma once

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* Host-side 3-float point. Layout-identical to HIP's float3 (12 bytes, 4-byte aligned),
 * so `(float3*)vec.data()` callers of the reference keep working. */
#ifndef KN_HAVE_FLOAT3
#if defined(__HIP__) || defined(__HIPCC__) || defined(HIP_INCLUDE_HIP_HIP_RUNTIME_H) || \
    defined(HIP_INCLUDE_HIP_AMD_DETAIL_HIP_VECTOR_TYPES_H)
#define KN_HAVE_FLOAT3 1
typedef float3 kn_float3;
#else
typedef struct { float x, y, z; } kn_float3;
#endif
#endif

#define KN_DEFAULT_K 50 /* reference params.h:4 (DEFAULT_NB_PLANES) */
#define KN_MAX_K 128

typedef enum {
    KN_OK = 0,
    KN_ERR_INVALID_ARGUMENT = 1,
    KN_ERR_OUT_OF_MEMORY = 2,
    KN_ERR_DEVICE = 3,
    KN_ERR_IO = 4,
    KN_ERR_STATE = 5
} kn_status;

/* Runtime configuration (replaces the reference's compile-time params.h). */
typedef struct {
    int k;                   /* neighbours per point (1..KN_MAX_K), default 50            */
    float points_per_cell;   /* grid density target; <=0 -> automatic (>= 3.1, ref :249)  */
    int tile[3];             /* query tile in cells (x,y,z); 0 -> automatic                */
    int halo;                /* halo rings staged around a tile; 0 -> automatic            */
    int deterministic;       /* 1 -> stable in-cell order (sorted by original id)          */
    int device;              /* HIP device ordinal                                        */
    int verbose;             /* 0 silent, 1 timings (reference IF_VERBOSE), 2 debug        */
    int exact_only;          /* 1 -> skip the LDS tile kernel (exact ring walk for all)      */
    int fixed_grid;          /* 1 -> no occupancy refinement of the grid (clusters/surfaces) */
    int algo;                /* query structure: 0 auto (the Morton-leaf tree when the
                                occupancy-adaptive grid had to be refined), 1 grid, 2 tree    */
} kn_config;

/* Per-solve statistics (reference kn_print_stats + cell_max, knearests.cu:378-466). */
typedef struct {
    int num_points;
    int k;
    int dims[3];
    int num_cells;
    int min_cell, max_cell;   /* occupancy */
    float avg_cell;
    int empty_cells;
    int fallback_queries;     /* queries not certified by the tiled kernel          */
    int uncertified_queries;  /* queries with fewer than K neighbours in the cloud  */
    float ms_build;           /* bbox + count + scan + scatter (device time)        */
    float ms_solve;           /* tiled query + fallback (device time)               */
    int range_allocations;    /* device allocations made by kn_solve_range so far (grow-only
                                 scratch: 1 for any sequence of equal or shrinking batches) */
} kn_stats;

/* The problem handle. Field names follow the reference struct (reference knearests.h:3-16);
 * divergences, all documented here:
 *   - d_cell_offsets / d_cell_offset_dists / d_cell_max / d_globcounter are NULL: the ring walk
 *     is analytic (no offset table), there is no racy max-ring buffer (reference defect D2)
 *     and no atomic bump allocator (cells are laid out by a deterministic scan, defect D5);
 *   - d_ptrs has C+1 entries (exclusive scan, d_ptrs[C] = N); d_counters is NULL: the count
 *     of cell c is d_ptrs[c+1] - d_ptrs[c];
 *   - d_stored_points is a float3 array in stored order, as in the reference; the engine's own
 *     float4 rows {x, y, z, bits(original index)} are d_stored_points4;
 *   - d_knearests holds the N x K stored-space result after kn_solve, as in the reference
 *     (knearests.cu:329-364), with UINT_MAX in slots that cannot be filled;
 *   - k and impl are additions (runtime K, engine state). */
typedef struct {
    int allocated_points;          /* number of input points                                */
    int dimx, dimy, dimz;          /* grid resolution                                       */
    int num_cell_offsets;          /* 0: no offset table (analytic ring walk)               */
    int *d_cell_offsets;           /* NULL (see above)                                      */
    float *d_cell_offset_dists;    /* NULL                                                  */
    float *d_cell_max;             /* NULL                                                  */
    unsigned int *d_permutation;   /* device: perm[stored] = original index                 */
    int *d_counters;               /* NULL: counts are d_ptrs[c+1] - d_ptrs[c]              */
    int *d_ptrs;                   /* device: first stored index of each cell, C+1 entries  */
    int *d_globcounter;            /* NULL                                                  */
    kn_float3 *d_stored_points;    /* device: N points in stored order (float3)             */
    unsigned int *d_knearests;     /* device: N x K neighbours in stored space (after solve) */
    int k;                         /* neighbours per point                                  */
    float *d_stored_points4;       /* device: N float4 {x,y,z,bits(original index)}         */
    void *impl;                    /* engine state (opaque)                                 */
} kn_problem;

/* ---- reference-compatible API ---------------------------------------------------- */
kn_problem *kn_prepare(const kn_float3 *points, int numpoints);
void kn_solve(kn_problem *kn);
void kn_free(kn_problem **kn);

kn_float3 *kn_get_points(kn_problem *kn);
unsigned int *kn_get_knearests(kn_problem *kn);
unsigned int *kn_get_permutation(kn_problem *kn);

void kn_print_stats(kn_problem *kn);

/* ---- extensions ------------------------------------------------------------------- */
kn_config kn_default_config(void);
kn_problem *kn_prepare_ex(const kn_float3 *points, int numpoints, const kn_config *cfg);
kn_status kn_solve_ex(kn_problem *kn);
/* Queries of the original indices [first, first + count) only: count x K original-space ids
 * (row = original index - first) into host buffers, squared distances too when out_d2 != NULL.
 * The whole N x K result is never allocated on the device, so clouds whose result does not fit
 * next to the grid are solved in batches. */
kn_status kn_solve_range(kn_problem *kn, int first, int count, unsigned int *out_ids, float *out_d2);
kn_status kn_set_k(kn_problem *kn, int k);                 /* re-solve with another K, no rebuild */
float *kn_get_distances(kn_problem *kn);                   /* N x K squared distances, stored space */
unsigned int *kn_get_neighbors(kn_problem *kn);            /* N x K, original space (row = original id) */
kn_status kn_get_stats(kn_problem *kn, kn_stats *out);
const char *kn_last_error(void);
kn_status kn_save(kn_problem *kn, const char *path);
kn_problem *kn_load(const char *path, const kn_config *cfg);

/* ---- point-file helpers (reference test_knearests.cu:15-80) --------------------- */
/* Reads a .xyz file (first line = count, then "x y z" per line). If normalize != 0 the
 * cloud is mapped into [0,1000]^3 with a 0.1%-inflated bbox and uniform scale. Returns
 * a malloc()'d array of *n points, or NULL (see kn_last_error()). */
kn_float3 *kn_read_xyz(const char *path, int *n, int normalize);
kn_status kn_write_xyz(const char *path, const kn_float3 *pts, int n);

/* ---- multi-GPU in one process (extension; the reference is single-GPU) --------------- */
/* The cloud is split over `ndevices` ranks (devices[i] = HIP device of rank i; NULL: 0..n-1;
 * repeated devices = virtual ranks on one GPU). A solve routes every point to the owner of
 * its box of a px*py*pz spatial split plus halo copies to the neighbouring boxes, in one
 * exchange (RCCL ncclSend/ncclRecv over one communicator per device when the devices are
 * distinct, device copies otherwise), then every rank solves its owned points with the
 * single-GPU kernels and certifies them against its halo (uncertified -> wider halo). */
typedef struct kn_multi kn_multi;
kn_multi *kn_prepare_multi(const kn_float3 *points, int numpoints, const int *devices, int ndevices,
                           const kn_config *cfg);
kn_status kn_solve_multi(kn_multi *m);
unsigned int *kn_get_neighbors_multi(kn_multi *m);  /* N x K original ids, row = original index */
float *kn_get_distances_multi(kn_multi *m);         /* N x K squared distances */
kn_status kn_get_multi_info(kn_multi *m, int *ranks, int *rounds, int *halo_points, int *uses_rccl);
void kn_free_multi(kn_multi **m);
/* Options of the multi-GPU solve (kn_default_multi_options(); set before kn_solve_multi). */
typedef struct {
    double halo_factor; /* halo send width in expected K-th neighbour radii of the whole cloud (2.5) */
    int balance;        /* 1: count-balanced kd rank boxes (default), 0: equal-volume boxes          */
    int forward;        /* 1: uncertified queries answered by query forwarding (default),
                           0: a halo-doubling round per uncertified step                           */
    int max_rounds;     /* halo growth rounds at most (8)                                            */
} kn_multi_options;
kn_multi_options kn_default_multi_options(void);
kn_status kn_set_multi_options(kn_multi *m, const kn_multi_options *o);
/* New coordinates of the same N points (the next kn_solve_multi re-routes; buffers are kept). */
kn_status kn_update_multi(kn_multi *m, const kn_float3 *points);
typedef struct {
    int ranks, rounds, halo_points;
    int forwarded;          /* uncertified queries answered by query forwarding              */
    int uses_rccl, balanced;
    int min_owned, max_owned;  /* owned points per rank                                    */
    int device_allocations; /* device allocations made by the last solve (0 once buffers fit) */
    float ms_total;         /* host wall time of the last kn_solve_multi                      */
    int host_syncs;         /* host synchronisation points of the last kn_solve_multi: meta,
                               route counts, local solves, rows (+1 per kd split level of a new
                               count-balanced plan; a solve whose ranks' bboxes and counts are
                               unchanged reuses the splits; + forwarding)                        */
} kn_multi_stats;
kn_status kn_get_multi_stats(kn_multi *m, kn_multi_stats *out);

/* ABI self-check for bindings (ctypes, other languages): sizeof of the public structs as
 * compiled into the library. which: 0 kn_config, 1 kn_problem, 2 kn_stats, 3 kn_multi_options,
 * 4 kn_multi_stats. */
size_t kn_struct_size(int which);

/* Extension: free the device blocks that kn_free parks for reuse by the next kn_prepare (a
   process-wide cache of at most 8 blocks per device and 4 GiB in all: arenas, result and tree
   buffers; KN_ARENA_CACHE=0 disables it). An allocation that fails for lack of device memory
   frees the cache and retries once by itself. */
void kn_release_cached_memory(void);

#ifdef __cplusplus
}
#endif
