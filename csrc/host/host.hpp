// host.hpp -- CPU-side components: correctness oracles, CPU grid kNN, .xyz I/O.
//
// * KdTree      : own implementation of the reference's CPU oracle (reference
//                 kd_tree.h/kd_tree.cpp): median split on the widest axis, leaves of <= 16
//                 points, near-child-first descent with box-distance pruning. Unlike the
//                 reference it excludes the query by INDEX (reference drops neighbour 0, which
//                 is wrong with duplicate points, test_knearests.cu:210) and orders results
//                 by (squared distance, index) so ties are deterministic.
// * brute_knn   : O(N^2) oracle for small clouds (tests).
// * grid_knn_cpu: the engine's algorithm on the host (uniform grid + exact ring walk with the
//                 same stopping rule as knn_exact_kernel) -- the CPU backend and the local
//                 solver of the multi-process gloo path.
// * xyz I/O     : reference format (test_knearests.cu:40-80): first line = count, then
//                 "x y z" lines; optional normalisation into [0,1000]^3 with a bbox inflated
//                 by 0.1% of its largest side.
#pragma once

#include <cstdint>
#include <string>
#include <vector>

namespace knh {

class KdTree {
public:
    KdTree() = default;
    void build(const float* pts, int n);
    // K nearest of an arbitrary position (exclude = index to skip, or -1).
    void query(const float q[3], int k, int exclude, uint32_t* idx, float* d2) const;
    int size() const { return n_; }

private:
    struct Node {
        float lo[3], hi[3];  // bounding box of the node's points
        int begin, end;      // range in order_
        int left, right;     // children (-1 for leaves)
    };
    int build_rec(int begin, int end);
    std::vector<float> p_;
    std::vector<int> order_;
    std::vector<Node> nodes_;
    int n_ = 0;
    static constexpr int kLeaf = 16;
};

// All-points kNN (self excluded by index). Rows are ascending by (d2, index); slots beyond
// the available neighbours are UINT32_MAX / +inf.
void kdtree_knn_all(const float* pts, int n, int k, uint32_t* idx, float* d2, int threads);
void brute_knn_all(const float* pts, int n, int k, uint32_t* idx, float* d2, int threads);
// Queries [0, n_queries) against all n points; uncertified gets the query ids whose K-th
// distance reaches past `complete_lo/hi` (multi-rank halo limit; pass +-inf for none).
// complete_ext (nullable): {wide, zlim, domain lo x3, domain hi x3} of a position-dependent halo
// (kn::CompleteBox): a face margin grows by `wide` when the query's distance to the domain plus
// the margin + wide stays <= zlim.
void grid_knn_cpu(const float* pts, int n, int n_queries, int k, float points_per_cell,
                  const float complete_lo[3], const float complete_hi[3], uint32_t* idx,
                  float* d2, std::vector<uint32_t>* uncertified, int threads, const float* complete_ext = nullptr);

// Distance-aware comparison of a kNN result (original space, rows ascending) against an
// oracle: every row must be duplicate-free, exclude its own index, list valid ids in
// ascending distance order, and its distances must equal the oracle's bit for bit (the
// squared distance is the same fp32 fma chain on both sides). Ids may differ only inside
// runs of equal distance (ties), which is where the reference's exact-equality test was
// flaky (test_knearests.cu:215-231).
struct CheckResult {
    long rows_checked = 0;
    long bad_rows = 0;
    long first_bad = -1;
    std::string message;
};
CheckResult check_knn(const float* pts, int n, int n_queries, int k, const uint32_t* idx,
                      const uint32_t* oracle_idx, const float* oracle_d2);

// Synthetic clouds in [0,1000]^3 (the reference's 300K / 900K blue-noise files are missing
// from its snapshot, .MISSING_LARGE_BLOBS): uniform random; a blue-noise stand-in
// (one jittered point per cell of a cubic lattice, jitter 0.35 of the spacing, so the
// minimum spacing is bounded like pts20K.xyz's); Gaussian clusters (stress case).
void gen_uniform(int n, uint64_t seed, std::vector<float>& xyz);
void gen_blue(int n, uint64_t seed, std::vector<float>& xyz);
void gen_clustered(int n, uint64_t seed, std::vector<float>& xyz);

bool read_xyz(const std::string& path, std::vector<float>& xyz, bool normalize, std::string* err);
bool write_xyz(const std::string& path, const float* xyz, int n, std::string* err);
void normalize_1000(std::vector<float>& xyz);

}  // namespace knh
