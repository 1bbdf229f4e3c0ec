// bindings.cpp -- PyTorch (ROCm) extension `cuda_knearests_amd._C`.
//
// Device ops run on the current PyTorch HIP stream with memory from the caching allocator,
// so they compose with torch.cuda graphs and torch.distributed (RCCL) in the Python layer.
// GPU ops throw if called on CPU tensors; there is no silent fallback.
#include <ATen/hip/HIPContext.h>
#include <c10/core/DeviceGuard.h>
#include <torch/extension.h>

#include <execinfo.h>
#include <signal.h>
#include <unistd.h>

#include <cmath>
#include <cstdio>
#include <cstring>
#include <limits>
#include <vector>

#include "kn/kernels.h"
#include "kn/route.h"
#include "kn/tree.h"
#include "../host/host.hpp"
#include "../runtime/engine.hpp"
#include "../runtime/dist.hpp"

#include <memory>

namespace {

#define KN_CHECK_HIP(expr)                                                                 \
    do {                                                                                   \
        hipError_t e_ = (expr);                                                            \
        TORCH_CHECK(e_ == hipSuccess, "HIP error in ", #expr, ": ", hipGetErrorString(e_)); \
    } while (0)

void check_points(const torch::Tensor& p, bool cuda) {
    TORCH_CHECK(p.dim() == 2 && p.size(1) == 3, "points must be (N, 3)");
    TORCH_CHECK(p.scalar_type() == torch::kFloat32, "points must be float32");
    TORCH_CHECK(p.is_contiguous(), "points must be contiguous");
    if (cuda) {
        TORCH_CHECK(p.is_cuda(), "points must be a GPU (HIP) tensor");
    } else {
        TORCH_CHECK(p.device().is_cpu(), "points must be a CPU tensor");
    }
}

// Complete box from its Python list: [lo x3, hi x3] (one halo width) or + [wide, zlim, domain lo
// x3, domain hi x3] (position-dependent halo, kn::CompleteBox)
kn::CompleteBox complete_box(const std::vector<double>& c) {
    TORCH_CHECK(c.size() == 6 || c.size() == 14, "complete must have 6 or 14 entries");
    kn::CompleteBox b{};
    for (int a = 0; a < 3; ++a) { b.lo[a] = (float)c[a]; b.hi[a] = (float)c[3 + a]; }
    if (c.size() == 14) {
        b.wide = (float)c[6];
        b.zlim = (float)c[7];
        for (int a = 0; a < 3; ++a) { b.dlo[a] = (float)c[8 + a]; b.dhi[a] = (float)c[11 + a]; }
    }
    return b;
}

// geom tensor: 16 x int32 (64 bytes) holding a kn::GridGeom
static_assert(sizeof(kn::GridGeom) <= 64, "GridGeom must fit in 64 bytes");

std::vector<torch::Tensor> build_impl(torch::Tensor points, std::vector<int64_t> dims, bool deterministic,
                                      c10::optional<std::vector<double>> box, const int* gids = nullptr,
                                      int n_owned = 0, unsigned* zero_words = nullptr, int n_zero_words = 0) {
    check_points(points, true);
    TORCH_CHECK(dims.size() == 3 && dims[0] > 0 && dims[1] > 0 && dims[2] > 0, "dims must be 3 positive ints");
    const c10::DeviceGuard guard(points.device());
    const int n = (int)points.size(0);
    const int64_t C = dims[0] * dims[1] * dims[2];
    TORCH_CHECK(C < (1ll << 31) - 1, "too many cells");
    auto i32 = points.options().dtype(torch::kInt32);
    auto f32 = points.options().dtype(torch::kFloat32);
    const int64_t nb = (int64_t)kn::scan_block_count((int)C) + 1;
    // workspace (int32 words): bbox partials kBBoxWords | geom-pad 16 | cell_count C+1 | cell_scan C+1
    //                          | block_sums nb | (16-byte aligned) bin_tmp 4N (cell_rank 2N aliases it)
    int64_t rank_off = kn::kBBoxWords + 16 + 2 * (C + 1) + nb;
    rank_off = (rank_off + 3) & ~(int64_t)3;
    auto ws = torch::empty({rank_off + 4 * (int64_t)n}, i32);
    auto cell_start = torch::empty({C + 1}, i32);
    auto sorted = torch::empty({(int64_t)n, 4}, f32);
    auto perm = torch::empty({(int64_t)n}, i32);
    auto geom = torch::empty({16}, i32);
    int* w = ws.data_ptr<int>();
    kn::BuildBuffers b{};
    b.points = points.data_ptr<float>();
    b.n = n;
    for (int a = 0; a < 3; ++a) b.dims[a] = (int)dims[a];
    b.bbox_words = reinterpret_cast<unsigned*>(w);
    b.geom = reinterpret_cast<kn::GridGeom*>(geom.data_ptr<int>());
    b.cell_count = w + kn::kBBoxWords + 16;
    b.cell_scan = b.cell_count + (C + 1);
    b.block_sums = b.cell_scan + (C + 1);
    b.cell_rank = reinterpret_cast<int2*>(w + rank_off);
    b.bin_tmp = reinterpret_cast<float4*>(w + rank_off);
    b.cell_start = cell_start.data_ptr<int>();
    b.sorted = reinterpret_cast<float4*>(sorted.data_ptr<float>());
    b.perm = reinterpret_cast<unsigned*>(perm.data_ptr<int>());
    b.deterministic = deterministic ? 1 : 0;
    b.use_box = 0;
    if (box.has_value()) {
        TORCH_CHECK(box->size() == 6, "box must be [lox, loy, loz, hix, hiy, hiz]");
        b.use_box = 1;
        for (int a = 0; a < 3; ++a) { b.box_lo[a] = (float)(*box)[a]; b.box_hi[a] = (float)(*box)[3 + a]; }
    }
    b.gids = gids;
    b.n_owned = n_owned;
    b.zero_words = zero_words;
    b.n_zero_words = n_zero_words;
    const hipStream_t s = c10::hip::getCurrentHIPStreamMasqueradingAsCUDA().stream();
    KN_CHECK_HIP(kn::launch_build(b, s));
    return {sorted, cell_start, perm, geom};
}

std::vector<torch::Tensor> build(torch::Tensor points, std::vector<int64_t> dims, bool deterministic,
                                 c10::optional<std::vector<double>> box) {
    return build_impl(points, dims, deterministic, box);
}

// cbp (internal callers): the complete box itself (e.g. with a halo field), overriding `complete`
std::vector<torch::Tensor> query_impl(torch::Tensor sorted, torch::Tensor cell_start, torch::Tensor geom,
                                      std::vector<int64_t> dims, int64_t k, int64_t n_queries,
                                      c10::optional<torch::Tensor> id_map, std::vector<double> complete,
                                      std::vector<int64_t> tile, int64_t halo, int64_t lds_capacity,
                                      bool use_tiles, bool with_dist, int64_t flags,
                                      c10::optional<torch::Tensor> row_of, int64_t exact_grid,
                                      c10::optional<torch::Tensor> zeroed_counters, int64_t q_lo,
                                      int64_t xsub, const kn::CompleteBox* cbp) {
    TORCH_CHECK(sorted.is_cuda() && sorted.dim() == 2 && sorted.size(1) == 4 && sorted.scalar_type() == torch::kFloat32,
                "sorted must be a (N,4) float32 GPU tensor");
    TORCH_CHECK(cell_start.is_cuda() && cell_start.scalar_type() == torch::kInt32, "cell_start must be int32 GPU");
    TORCH_CHECK(geom.is_cuda() && geom.numel() == 16, "geom must be a 16-int GPU tensor");
    TORCH_CHECK(dims.size() == 3 && tile.size() == 3 && (complete.size() == 6 || complete.size() == 14),
                "bad dims/tile/complete");
    TORCH_CHECK(k >= 1 && k <= 128, "k must be in [1, 128]");
    TORCH_CHECK(cell_start.numel() == dims[0] * dims[1] * dims[2] + 1, "cell_start size does not match dims");
    const int n = (int)sorted.size(0);
    TORCH_CHECK(n_queries >= 0 && n_queries <= n, "n_queries out of range");
    // query range [q_lo, n_queries) of original indices (local id mode only); rows = n_queries - q_lo
    TORCH_CHECK(q_lo >= 0 && q_lo <= n_queries && (q_lo == 0 || !row_of.has_value()), "bad query range");
    const c10::DeviceGuard guard(sorted.device());
    auto i32 = sorted.options().dtype(torch::kInt32);
    const int64_t rows = n_queries - q_lo;
    auto out_idx = torch::empty({rows, k}, i32);
    torch::Tensor out_dist;
    if (with_dist) out_dist = torch::empty({rows, k}, sorted.options());
    auto fallback = torch::empty({std::max(1, n)}, i32);
    // zeroed_counters: kNumCounters int32 words the preceding build zeroed on the device
    torch::Tensor counters = zeroed_counters.has_value() ? *zeroed_counters : torch::empty({kn::kNumCounters}, i32);
    TORCH_CHECK(counters.is_cuda() && counters.scalar_type() == torch::kInt32 && counters.numel() == kn::kNumCounters,
                "counters must be kNumCounters int32 GPU words");
    auto uncert = torch::empty({std::max<int64_t>(1, n_queries)}, i32);
    kn::QueryBuffers q{};
    q.sorted = reinterpret_cast<const float4*>(sorted.data_ptr<float>());
    q.cell_start = cell_start.data_ptr<int>();
    q.perm = nullptr;
    q.geom = reinterpret_cast<const kn::GridGeom*>(geom.data_ptr<int>());
    q.n = n;
    for (int a = 0; a < 3; ++a) q.dims[a] = (int)dims[a];
    q.k = (int)k;
    q.n_queries = (int)n_queries;
    q.q_lo = (int)q_lo;
    if (id_map.has_value()) {
        TORCH_CHECK(id_map->is_cuda() && id_map->scalar_type() == torch::kInt32 && id_map->numel() >= n,
                    "id_map must be an int32 GPU tensor with >= N entries");
        q.id_map = reinterpret_cast<const unsigned*>(id_map->data_ptr<int>());
    }
    if (row_of.has_value()) {
        TORCH_CHECK(row_of->is_cuda() && row_of->scalar_type() == torch::kInt32 && row_of->numel() >= n,
                    "row_of must be an int32 GPU tensor with >= N entries");
        q.row_of = reinterpret_cast<const unsigned*>(row_of->data_ptr<int>());
    }
    q.complete = cbp ? *cbp : complete_box(complete);
    q.out_idx = reinterpret_cast<unsigned*>(out_idx.data_ptr<int>());
    q.out_dist = with_dist ? out_dist.data_ptr<float>() : nullptr;
    q.fallback_list = reinterpret_cast<unsigned*>(fallback.data_ptr<int>());
    q.counters = reinterpret_cast<unsigned*>(counters.data_ptr<int>());
    q.uncert_list = reinterpret_cast<unsigned*>(uncert.data_ptr<int>());
    for (int a = 0; a < 3; ++a) q.tile[a] = (int)tile[a];
    q.halo = (int)halo;
    TORCH_CHECK(xsub >= 1 && xsub <= 4, "xsub must be in [1, 4]");
    q.xsub = (int)xsub;
    q.lds_capacity = (int)lds_capacity;
    q.use_tiles = use_tiles ? 1 : 0;
    q.flags = (int)flags;
    q.exact_grid = (int)exact_grid;
    q.counters_zeroed = zeroed_counters.has_value() ? 1 : 0;
    TORCH_CHECK(lds_capacity >= 64 && lds_capacity % 64 == 0 && lds_capacity <= 8192,
                "lds_capacity must be a multiple of 64 in [64, 8192]");
    TORCH_CHECK(kn::query_lds_bytes(q.tile, q.halo, q.lds_capacity, q.xsub) <= 160 * 1024, "tile plan exceeds 160 KiB LDS");
    const hipStream_t s = c10::hip::getCurrentHIPStreamMasqueradingAsCUDA().stream();
    KN_CHECK_HIP(kn::launch_query(q, s));
    if (!with_dist) out_dist = torch::empty({0}, sorted.options());
    return {out_idx, out_dist, counters, uncert, fallback};
}

std::vector<torch::Tensor> query(torch::Tensor sorted, torch::Tensor cell_start, torch::Tensor geom,
                                 std::vector<int64_t> dims, int64_t k, int64_t n_queries,
                                 c10::optional<torch::Tensor> id_map, std::vector<double> complete,
                                 std::vector<int64_t> tile, int64_t halo, int64_t lds_capacity,
                                 bool use_tiles, bool with_dist, int64_t flags,
                                 c10::optional<torch::Tensor> row_of, int64_t exact_grid = 0,
                                 c10::optional<torch::Tensor> zeroed_counters = c10::nullopt, int64_t q_lo = 0,
                                 int64_t xsub = 1) {
    return query_impl(sorted, cell_start, geom, dims, k, n_queries, id_map, complete, tile, halo, lds_capacity,
                      use_tiles, with_dist, flags, row_of, exact_grid, zeroed_counters, q_lo, xsub, nullptr);
}

// Morton-leaf tree over a built grid's points (kn/tree.h): (workspace, node buffer, leaf count).
// One host sync (the leaf count sizes the node buffer).
std::tuple<torch::Tensor, torch::Tensor, int64_t> tree_build_impl(torch::Tensor sorted, torch::Tensor cell_start,
                                                                  torch::Tensor geom, std::vector<int64_t> dims,
                                                                  bool count_leaves);

py::tuple tree_build(torch::Tensor sorted, torch::Tensor cell_start, torch::Tensor geom, std::vector<int64_t> dims,
                     bool count_leaves) {
    auto r = tree_build_impl(sorted, cell_start, geom, dims, count_leaves);
    return py::make_tuple(std::get<0>(r), std::get<1>(r), std::get<2>(r));
}

// Stream-ordered tree build (no host sync); the leaf count is read back only on request
// (count_leaves, diagnostics) -- the query kernels take it from the device.
std::tuple<torch::Tensor, torch::Tensor, int64_t> tree_build_impl(torch::Tensor sorted, torch::Tensor cell_start,
                                                                  torch::Tensor geom, std::vector<int64_t> dims,
                                                                  bool count_leaves) {
    TORCH_CHECK(sorted.is_cuda() && sorted.dim() == 2 && sorted.size(1) == 4 && sorted.scalar_type() == torch::kFloat32,
                "sorted must be a (N,4) float32 GPU tensor");
    TORCH_CHECK(geom.is_cuda() && geom.numel() == 16, "geom must be a 16-int GPU tensor");
    TORCH_CHECK(dims.size() == 3 && dims[0] > 0 && dims[1] > 0 && dims[2] > 0, "dims = the grid's [X, Y, Z]");
    TORCH_CHECK(cell_start.is_cuda() && cell_start.scalar_type() == torch::kInt32 &&
                    cell_start.numel() == dims[0] * dims[1] * dims[2] + 1, "cell_start must match dims");
    const c10::DeviceGuard guard(sorted.device());
    const int n = (int)sorted.size(0);
    const int d[3] = {(int)dims[0], (int)dims[1], (int)dims[2]};
    TORCH_CHECK(kn::tree_supports(d), "tree path: grid too elongated / too large (padded brick space > 2^24 slots)");
    auto u8 = sorted.options().dtype(torch::kUInt8);
    auto ws = torch::empty({(int64_t)kn::tree_workspace_bytes(n, d)}, u8);
    auto nodes = torch::empty({(int64_t)kn::tree_node_bytes(n)}, u8);
    kn::TreeView t = kn::tree_view(ws.data_ptr(), n, d);
    kn::tree_attach_nodes(t, nodes.data_ptr());
    const hipStream_t s = c10::hip::getCurrentHIPStreamMasqueradingAsCUDA().stream();
    KN_CHECK_HIP(kn::launch_tree_leaves(reinterpret_cast<const float4*>(sorted.data_ptr<float>()),
                                        cell_start.data_ptr<int>(),
                                        reinterpret_cast<const kn::GridGeom*>(geom.data_ptr<int>()), t, s));
    KN_CHECK_HIP(kn::launch_tree_nodes(t, s));
    unsigned L = 0;
    if (count_leaves) KN_CHECK_HIP(kn::tree_leaf_count(t, &L, s));
    return {ws, nodes, count_leaves ? (int64_t)L : (int64_t)-1};
}

std::vector<torch::Tensor> tree_query(torch::Tensor ws, torch::Tensor nodes, std::vector<int64_t> dims, int64_t n,
                                      int64_t k, int64_t n_queries, c10::optional<torch::Tensor> id_map, bool with_dist,
                                      int64_t flags, c10::optional<torch::Tensor> row_of = c10::nullopt) {
    TORCH_CHECK(dims.size() == 3 && dims[0] > 0 && dims[1] > 0 && dims[2] > 0, "dims = the grid's [X, Y, Z]");
    const int d[3] = {(int)dims[0], (int)dims[1], (int)dims[2]};
    TORCH_CHECK(ws.is_cuda() && ws.scalar_type() == torch::kUInt8, "ws must be a tree_build workspace");
    TORCH_CHECK(n >= 0 && (size_t)ws.numel() >= kn::tree_workspace_bytes((int)n, d), "workspace too small for n");
    TORCH_CHECK(nodes.is_cuda() && (size_t)nodes.numel() >= kn::tree_node_bytes((int)n), "node buffer too small");
    TORCH_CHECK(k >= 1 && k <= 128, "k must be in [1, 128]");
    TORCH_CHECK(n_queries >= 0 && n_queries <= n, "n_queries out of range");
    const c10::DeviceGuard guard(ws.device());
    kn::TreeView t = kn::tree_view(ws.data_ptr(), (int)n, d);
    kn::tree_attach_nodes(t, nodes.data_ptr());
    auto i32 = ws.options().dtype(torch::kInt32);
    auto out_idx = torch::empty({n_queries, k}, i32);
    torch::Tensor out_dist = torch::empty({with_dist ? n_queries : 0, with_dist ? k : 0}, ws.options().dtype(torch::kFloat32));
    auto counters = torch::empty({kn::kNumCounters}, i32);
    kn::TreeQuery q{};
    q.k = (int)k;
    q.n_queries = (int)n_queries;
    if (id_map.has_value()) {
        TORCH_CHECK(id_map->is_cuda() && id_map->scalar_type() == torch::kInt32 && id_map->numel() >= n,
                    "id_map must be an int32 GPU tensor with >= N entries");
        q.id_map = reinterpret_cast<const unsigned*>(id_map->data_ptr<int>());
    }
    if (row_of.has_value()) {
        TORCH_CHECK(row_of->is_cuda() && row_of->scalar_type() == torch::kInt32 && row_of->numel() >= n,
                    "row_of must be an int32 GPU tensor with >= N entries");
        q.row_of = reinterpret_cast<const unsigned*>(row_of->data_ptr<int>());
    }
    q.out_idx = reinterpret_cast<unsigned*>(out_idx.data_ptr<int>());
    q.out_dist = with_dist ? out_dist.data_ptr<float>() : nullptr;
    q.counters = reinterpret_cast<unsigned*>(counters.data_ptr<int>());
    q.flags = (int)flags;
    const hipStream_t s = c10::hip::getCurrentHIPStreamMasqueradingAsCUDA().stream();
    KN_CHECK_HIP(kn::launch_tree_query(t, q, s));
    return {out_idx, out_dist, counters};
}

py::dict auto_params(int64_t n, int64_t k, double ppc, std::vector<int64_t> tile, int64_t halo,
                     c10::optional<std::vector<double>> extent, int64_t xsub) {
    int th[3] = {0, 0, 0};
    for (size_t a = 0; a < tile.size() && a < 3; ++a) th[a] = (int)tile[a];
    float ext[3];
    const float* pe = nullptr;
    if (extent.has_value() && extent->size() == 3) {
        for (int a = 0; a < 3; ++a) ext[a] = (float)(*extent)[a];
        pe = ext;
    }
    const kn::AutoParams p = kn::auto_params((int)n, (int)k, (float)ppc, th, (int)halo, pe, (int)xsub);
    py::dict d;
    d["xsub"] = p.xsub;
    d["dims"] = std::vector<int>{p.dims[0], p.dims[1], p.dims[2]};
    d["tile"] = std::vector<int>{p.tile[0], p.tile[1], p.tile[2]};
    d["halo"] = p.halo;
    d["lds_capacity"] = p.lds_capacity;
    d["lds_bytes"] = (int64_t)p.lds_bytes;
    return d;
}

torch::Tensor to_stored_space(torch::Tensor out_orig, torch::Tensor perm) {
    TORCH_CHECK(out_orig.is_cuda() && perm.is_cuda(), "GPU tensors expected");
    const c10::DeviceGuard guard(out_orig.device());
    const int n = (int)perm.numel();
    const int k = (int)out_orig.size(1);
    auto inv = torch::empty({std::max(1, n)}, perm.options());
    auto out = torch::empty_like(out_orig);
    const hipStream_t s = c10::hip::getCurrentHIPStreamMasqueradingAsCUDA().stream();
    KN_CHECK_HIP(kn::launch_invert_perm(reinterpret_cast<const unsigned*>(perm.data_ptr<int>()), n,
                                        reinterpret_cast<unsigned*>(inv.data_ptr<int>()), s));
    KN_CHECK_HIP(kn::launch_to_stored_space(reinterpret_cast<const unsigned*>(out_orig.data_ptr<int>()),
                                            reinterpret_cast<const unsigned*>(perm.data_ptr<int>()),
                                            reinterpret_cast<const unsigned*>(inv.data_ptr<int>()), n, k,
                                            reinterpret_cast<unsigned*>(out.data_ptr<int>()), nullptr,
                                            nullptr, s));
    return out;
}

// ---- multi-GPU routing (csrc/kernels/route.hip) -------------------------------------
kn::RouteParams route_params(const std::vector<double>& lo, const std::vector<double>& hi,
                             const std::vector<int64_t>& grid, const std::vector<double>& boxes, double h,
                             const c10::optional<std::vector<double>>& splits = c10::nullopt,
                             double h_inner = -1.0, double wz = INFINITY) {
    TORCH_CHECK(lo.size() == 3 && hi.size() == 3 && grid.size() == 3, "lo/hi/grid must have 3 entries");
    const int64_t world = grid[0] * grid[1] * grid[2];
    TORCH_CHECK(world >= 1 && world <= kn::kRouteMaxWorld, "world size must be in [1, 64]");
    TORCH_CHECK((int64_t)boxes.size() == 6 * world, "boxes must hold 6 floats per rank");
    kn::RouteParams p{};
    for (int a = 0; a < 3; ++a) {
        // float32 arithmetic, exactly as SpatialDecomposition.owner evaluates it
        const float l = (float)lo[a], u = (float)hi[a];
        p.lo[a] = l;
        p.ext[a] = std::max(u - l, 1e-30f);
        p.g[a] = (float)grid[a];
        p.grid[a] = (int)grid[a];
    }
    p.world = (int)world;
    const float hf = (float)h;
    p.h2 = hf * hf;
    // position-dependent halo (h_inner < 0: one width)
    const float hif = (float)(h_inner < 0.0 ? h : h_inner);
    p.hi2 = hif * hif;
    p.wz = (float)wz;
    for (int a = 0; a < 3; ++a) p.dom_hi[a] = (float)hi[a];
    for (int r = 0; r < world; ++r)
        for (int a = 0; a < 3; ++a) {
            p.box_lo[r][a] = (float)boxes[6 * r + a];
            p.box_hi[r][a] = (float)boxes[6 * r + 3 + a];
        }
    if (splits.has_value()) {
        const int g[3] = {(int)grid[0], (int)grid[1], (int)grid[2]};
        TORCH_CHECK((int)splits->size() == kn::route_split_count(g), "splits do not match the grid");
        const int nxs = g[0] + 1, nys = g[0] * (g[1] + 1);
        p.balanced = 1;
        for (int j = 0; j < (int)splits->size(); ++j) {
            const float v = (float)(*splits)[j];
            if (j < nxs) p.xs[j] = v;
            else if (j < nxs + nys) p.ys[j - nxs] = v;
            else p.zs[j - nxs - nys] = v;
        }
    }
    return p;
}

// RouteParams on the device (the route kernels read their parameters from device memory)
torch::Tensor upload_params(const kn::RouteParams& p, const torch::Device& dev) {
    auto h = torch::empty({(int64_t)sizeof(kn::RouteParams)}, torch::TensorOptions().dtype(torch::kUInt8));
    std::memcpy(h.data_ptr<uint8_t>(), &p, sizeof(p));
    return h.to(dev, /*non_blocking=*/false);
}

const kn::RouteParams* params_ptr(const torch::Tensor& plan) {
    TORCH_CHECK(plan.is_cuda() && plan.scalar_type() == torch::kUInt8 && plan.numel() == (int64_t)sizeof(kn::RouteParams),
                "plan must be the uint8 device tensor returned by route_plan");
    return reinterpret_cast<const kn::RouteParams*>(plan.data_ptr<uint8_t>());
}

std::vector<torch::Tensor> route_count_impl(const torch::Tensor& points, const kn::RouteParams* p, int world) {
    const int n = (int)points.size(0);
    const int nb = kn::route_block_count(n);
    auto i32 = points.options().dtype(torch::kInt32);
    auto bc = torch::empty({2 * (int64_t)world * nb}, i32);
    auto totals = torch::empty({(int64_t)world, 2}, i32);
    const hipStream_t s = c10::hip::getCurrentHIPStreamMasqueradingAsCUDA().stream();
    KN_CHECK_HIP(kn::launch_route_count(points.data_ptr<float>(), n, p, world, bc.data_ptr<int>(), totals.data_ptr<int>(), s));
    return {bc, totals};
}

torch::Tensor route_scatter_impl(const torch::Tensor& points, const c10::optional<torch::Tensor>& ids,
                                 const kn::RouteParams* p, int world, const torch::Tensor& block_offsets,
                                 const torch::Tensor& totals, int64_t rows, int self_last = -1) {
    const int n = (int)points.size(0);
    const int* idp = nullptr;
    if (ids.has_value()) {
        TORCH_CHECK(ids->is_cuda() && ids->scalar_type() == torch::kInt32 && ids->numel() == n && ids->is_contiguous(),
                    "ids must be a contiguous int32 GPU tensor of N entries");
        idp = ids->data_ptr<int>();
    }
    TORCH_CHECK(block_offsets.numel() == 2 * (int64_t)world * kn::route_block_count(n) &&
                    totals.numel() == 2 * (int64_t)world,
                "block_offsets / totals do not match route_count's output");
    TORCH_CHECK(rows >= 0, "rows must be >= 0");
    auto send = torch::empty({rows, 4}, points.options());
    const hipStream_t s = c10::hip::getCurrentHIPStreamMasqueradingAsCUDA().stream();
    KN_CHECK_HIP(kn::launch_route_scatter(points.data_ptr<float>(), idp, n, p, world, block_offsets.data_ptr<int>(),
                                          totals.data_ptr<int>(), reinterpret_cast<float4*>(send.data_ptr<float>()),
                                          (int)rows, self_last, s));
    return send;
}

// -> (scanned block counts, totals (world, 2) = owned / halo rows per destination)
std::vector<torch::Tensor> route_count(torch::Tensor points, std::vector<double> lo, std::vector<double> hi,
                                       std::vector<int64_t> grid, std::vector<double> boxes, double h,
                                       c10::optional<std::vector<double>> splits, double h_inner, double wz) {
    check_points(points, true);
    const c10::DeviceGuard guard(points.device());
    const kn::RouteParams p = route_params(lo, hi, grid, boxes, h, splits, h_inner, wz);
    auto dp = upload_params(p, points.device());
    return route_count_impl(points, params_ptr(dp), p.world);
}

torch::Tensor route_scatter(torch::Tensor points, torch::Tensor ids, std::vector<double> lo, std::vector<double> hi,
                            std::vector<int64_t> grid, std::vector<double> boxes, double h, torch::Tensor block_offsets,
                            torch::Tensor totals, int64_t rows, c10::optional<std::vector<double>> splits,
                            double h_inner, double wz) {
    check_points(points, true);
    const c10::DeviceGuard guard(points.device());
    const kn::RouteParams p = route_params(lo, hi, grid, boxes, h, splits, h_inner, wz);
    auto dp = upload_params(p, points.device());
    return route_scatter_impl(points, ids, params_ptr(dp), p.world, block_offsets, totals, rows);
}

const float* splits_ptr(const c10::optional<torch::Tensor>& splits, const std::vector<int64_t>& grid) {
    if (!splits.has_value()) return nullptr;
    const int g[3] = {(int)grid[0], (int)grid[1], (int)grid[2]};
    TORCH_CHECK(splits->is_cuda() && splits->scalar_type() == torch::kFloat32 && splits->is_contiguous() &&
                    splits->numel() == kn::route_split_count(g),
                "splits must be a contiguous float32 GPU tensor in the kd layout of the grid");
    return splits->data_ptr<float>();
}

// (pointer, G) of an optional halo-field tensor (G^3 float32 widths or certified radii, on the GPU)
static std::pair<float*, int> field_arg(const c10::optional<torch::Tensor>& f) {
    if (!f.has_value()) return {nullptr, 0};
    TORCH_CHECK(f->is_cuda() && f->scalar_type() == torch::kFloat32 && f->is_contiguous(),
                "a halo field must be a contiguous float32 GPU tensor");
    const int64_t n = f->numel();
    const int g = (int)std::lround(std::cbrt((double)n));
    TORCH_CHECK(g >= 1 && g <= 256 && (int64_t)g * g * g == n, "a halo field holds G^3 floats, G in [1, 256]");
    return {f->data_ptr<float>(), g};
}

// Device-side plan from the all-gathered metas (world x 8 float64, on device): no host sync.
// -> (plan (uint8 RouteParams on device), header (16,) float64 on device, see kn::kPlanHdr)
std::vector<torch::Tensor> route_plan(torch::Tensor metas, int64_t rank, std::vector<int64_t> grid, int64_t k,
                                      double halo_factor, c10::optional<torch::Tensor> splits, double inner_factor,
                                      c10::optional<torch::Tensor> field) {
    const auto fa = field_arg(field);
    TORCH_CHECK(metas.is_cuda() && metas.scalar_type() == torch::kFloat64 && metas.is_contiguous() &&
                    metas.numel() % 8 == 0,
                "metas must be a contiguous (world*8,) float64 GPU tensor");
    TORCH_CHECK(grid.size() == 3, "grid must have 3 entries");
    const int world = (int)(metas.numel() / 8);
    const c10::DeviceGuard guard(metas.device());
    auto plan = torch::empty({(int64_t)sizeof(kn::RouteParams)}, metas.options().dtype(torch::kUInt8));
    auto hdr = torch::empty({kn::kPlanHdr}, metas.options());
    const int g[3] = {(int)grid[0], (int)grid[1], (int)grid[2]};
    const hipStream_t s = c10::hip::getCurrentHIPStreamMasqueradingAsCUDA().stream();
    KN_CHECK_HIP(kn::launch_route_plan(metas.data_ptr<double>(), world, (int)rank, g, (int)k, halo_factor,
                                       splits_ptr(splits, grid), reinterpret_cast<kn::RouteParams*>(plan.data_ptr<uint8_t>()),
                                       hdr.data_ptr<double>(), s, inner_factor, fa.first, fa.second));
    return {plan, hdr};
}

std::vector<torch::Tensor> route_count_dev(torch::Tensor points, torch::Tensor plan, int64_t world) {
    check_points(points, true);
    const c10::DeviceGuard guard(points.device());
    TORCH_CHECK(world >= 1 && world <= kn::kRouteMaxWorld, "world size must be in [1, 64]");
    return route_count_impl(points, params_ptr(plan), (int)world);
}

torch::Tensor route_scatter_dev(torch::Tensor points, c10::optional<torch::Tensor> ids, torch::Tensor plan,
                                int64_t world, torch::Tensor block_offsets, torch::Tensor totals, int64_t rows,
                                int64_t self_last) {
    check_points(points, true);
    const c10::DeviceGuard guard(points.device());
    TORCH_CHECK(world >= 1 && world <= kn::kRouteMaxWorld, "world size must be in [1, 64]");
    TORCH_CHECK(self_last >= -1 && self_last < world, "self_last must be -1 or a rank");
    return route_scatter_impl(points, ids, params_ptr(plan), (int)world, block_offsets, totals, rows, (int)self_last);
}

// The whole pre-sync half of a distributed step in one call (no host round trip inside):
// route plan from the gathered metas -> per-destination counts -> scatter into a send buffer
// of `cap` rows in the self-last layout. If the rows do not fit, `send` is left unwritten and
// the caller re-scatters after its sync (route_scatter_dev with self_last = rank).
// `sync` (int32) packs everything the host reads at its one sync, so it is ONE copy:
//   [0, 2*kPlanHdr)            plan header (kPlanHdr doubles)
//   [2*kPlanHdr, +2*world)     totals: (owned, halo) rows this rank sends to each destination
//   [2*kPlanHdr+2*world, end)  room for the counts all-to-all's output (rows to receive)
// -> (plan, sync, scanned block counts, send (cap, 4))
std::vector<torch::Tensor> route_begin(torch::Tensor points, c10::optional<torch::Tensor> ids, torch::Tensor metas,
                                       int64_t rank, std::vector<int64_t> grid, int64_t k, double halo_factor,
                                       int64_t cap, c10::optional<torch::Tensor> splits, double inner_factor,
                                       c10::optional<torch::Tensor> field) {
    check_points(points, true);
    const auto fa = field_arg(field);
    TORCH_CHECK(cap >= 0 && cap < INT32_MAX, "cap out of range");
    TORCH_CHECK(metas.is_cuda() && metas.scalar_type() == torch::kFloat64 && metas.is_contiguous() &&
                    metas.numel() % 8 == 0 && metas.numel() >= 8,
                "metas must be a contiguous (world*8,) float64 GPU tensor");
    TORCH_CHECK(grid.size() == 3, "grid must have 3 entries");
    const int world = (int)(metas.numel() / 8);
    TORCH_CHECK(world <= kn::kRouteMaxWorld, "world size must be <= 64");
    const c10::DeviceGuard guard(points.device());
    const int n = (int)points.size(0);
    const int* idp = nullptr;
    if (ids.has_value()) {
        TORCH_CHECK(ids->is_cuda() && ids->scalar_type() == torch::kInt32 && ids->numel() == n && ids->is_contiguous(),
                    "ids must be a contiguous int32 GPU tensor of N entries");
        idp = ids->data_ptr<int>();
    }
    auto i32 = points.options().dtype(torch::kInt32);
    auto plan = torch::empty({(int64_t)sizeof(kn::RouteParams)}, i32.dtype(torch::kUInt8));
    auto sync = torch::empty({2 * (int64_t)kn::kPlanHdr + 4 * (int64_t)world}, i32);
    auto bc = torch::empty({2 * (int64_t)world * kn::route_block_count(n)}, i32);
    auto send = torch::empty({cap, 4}, points.options());
    auto* pp = reinterpret_cast<kn::RouteParams*>(plan.data_ptr<uint8_t>());
    int* totals = sync.data_ptr<int>() + 2 * kn::kPlanHdr;
    const int g[3] = {(int)grid[0], (int)grid[1], (int)grid[2]};
    const hipStream_t s = c10::hip::getCurrentHIPStreamMasqueradingAsCUDA().stream();
    KN_CHECK_HIP(kn::launch_route_plan(metas.data_ptr<double>(), world, (int)rank, g, (int)k, halo_factor,
                                       splits_ptr(splits, grid), pp,
                                       reinterpret_cast<double*>(sync.data_ptr<int>()), s, inner_factor, fa.first,
                                       fa.second));
    KN_CHECK_HIP(kn::launch_route_count(points.data_ptr<float>(), n, pp, world, bc.data_ptr<int>(), totals, s));
    KN_CHECK_HIP(kn::launch_route_scatter(points.data_ptr<float>(), idp, n, pp, world, bc.data_ptr<int>(), totals,
                                          reinterpret_cast<float4*>(send.data_ptr<float>()), (int)cap, (int)rank, s));
    return {plan, sync, bc, send};
}

// recv: rows received from every source, source s = [recv_own[s] owned | recv_halo[s] halo].
// -> (points (rows, 3): owned of all sources first, then halo; global ids (rows,))
std::vector<torch::Tensor> route_unpack(torch::Tensor recv, std::vector<int64_t> recv_own, std::vector<int64_t> recv_halo) {
    TORCH_CHECK(recv.is_cuda() && recv.dim() == 2 && recv.size(1) == 4 && recv.scalar_type() == torch::kFloat32 &&
                    recv.is_contiguous(),
                "recv must be a contiguous (R, 4) float32 GPU tensor");
    const int world = (int)recv_own.size();
    TORCH_CHECK(world >= 1 && world <= kn::kRouteMaxWorld && (int)recv_halo.size() == world, "bad source table");
    const c10::DeviceGuard guard(recv.device());
    kn::UnpackTable t{};
    t.world = world;
    int64_t seg = 0, own = 0, halo = 0;
    for (int s = 0; s < world; ++s) {
        TORCH_CHECK(recv_own[s] >= 0 && recv_halo[s] >= 0, "negative counts");
        t.seg[s] = (int)seg;
        t.own[s] = (int)recv_own[s];
        t.own_pref[s] = (int)own;
        t.halo_pref[s] = (int)halo;
        seg += recv_own[s] + recv_halo[s];
        own += recv_own[s];
        halo += recv_halo[s];
    }
    t.n_own = (int)own;
    t.rows_cross = (int)seg;
    t.self = -1;
    TORCH_CHECK(seg == recv.size(0), "source table does not add up to the received rows");
    auto pts = torch::empty({seg, 3}, recv.options());
    auto gids = torch::empty({seg}, recv.options().dtype(torch::kInt32));
    const hipStream_t s = c10::hip::getCurrentHIPStreamMasqueradingAsCUDA().stream();
    KN_CHECK_HIP(kn::launch_route_unpack(reinterpret_cast<const float4*>(recv.data_ptr<float>()), nullptr, (int)seg,
                                         t, pts.data_ptr<float>(), gids.data_ptr<int>(), s));
    return {pts, gids};
}

// Self-last variant: recv holds the other sources' segments only (in source order), the rank's
// own segment (recv_own[rank] + recv_halo[rank] rows) is `self_rows`, taken straight from its
// send buffer. Output order is the same as route_unpack's.
std::vector<torch::Tensor> route_unpack_split(torch::Tensor recv, torch::Tensor self_rows, std::vector<int64_t> recv_own,
                                              std::vector<int64_t> recv_halo, int64_t rank) {
    auto ok = [](const torch::Tensor& x) {
        return x.is_cuda() && x.dim() == 2 && x.size(1) == 4 && x.scalar_type() == torch::kFloat32 && x.is_contiguous();
    };
    TORCH_CHECK(ok(recv) && ok(self_rows), "recv / self_rows must be contiguous (R, 4) float32 GPU tensors");
    const int world = (int)recv_own.size();
    TORCH_CHECK(world >= 1 && world <= kn::kRouteMaxWorld && (int)recv_halo.size() == world && rank >= 0 && rank < world,
                "bad source table");
    const c10::DeviceGuard guard(recv.device());
    kn::UnpackTable t{};
    t.world = world;
    int64_t seg = 0, own = 0, halo = 0;
    for (int s = 0; s < world; ++s) {
        TORCH_CHECK(recv_own[s] >= 0 && recv_halo[s] >= 0, "negative counts");
        t.seg[s] = (int)seg;  // self: zero-length placeholder in recv
        t.own[s] = (int)recv_own[s];
        t.own_pref[s] = (int)own;
        t.halo_pref[s] = (int)halo;
        if (s != rank) seg += recv_own[s] + recv_halo[s];
        own += recv_own[s];
        halo += recv_halo[s];
    }
    t.n_own = (int)own;
    t.rows_cross = (int)seg;
    t.self = (int)rank;
    const int64_t nself = recv_own[rank] + recv_halo[rank];
    TORCH_CHECK(seg == recv.size(0) && nself == self_rows.size(0),
                "source table does not add up to the received / self rows");
    const int64_t rows = seg + nself;
    TORCH_CHECK(rows < INT32_MAX, "too many rows");
    auto pts = torch::empty({rows, 3}, recv.options());
    auto gids = torch::empty({rows}, recv.options().dtype(torch::kInt32));
    const hipStream_t s = c10::hip::getCurrentHIPStreamMasqueradingAsCUDA().stream();
    KN_CHECK_HIP(kn::launch_route_unpack(reinterpret_cast<const float4*>(recv.data_ptr<float>()),
                                         reinterpret_cast<const float4*>(self_rows.data_ptr<float>()), (int)rows, t,
                                         pts.data_ptr<float>(), gids.data_ptr<int>(), s));
    return {pts, gids};
}

// Density-adaptive halo field (kn/route.h): splat this rank's measured K-th distances into
// `field` (G^3 float32, zeroed by the caller, then MAX-all-reduced over the ranks). pts: the local
// rows (owned first), d2: (n_owned, k). -> stat (2 int32 on device: queries with < K neighbours,
// queries beyond the field's reach).
torch::Tensor field_splat(torch::Tensor pts, int64_t n_owned, torch::Tensor d2, int64_t k, std::vector<double> hdr,
                          int64_t rank, std::vector<int64_t> grid, torch::Tensor field) {
    check_points(pts, true);
    TORCH_CHECK(grid.size() == 3 && hdr.size() >= (size_t)kn::kPlanHdr, "grid must have 3 entries, hdr kPlanHdr");
    TORCH_CHECK(n_owned >= 0 && n_owned <= pts.size(0), "n_owned out of range");
    TORCH_CHECK(d2.is_cuda() && d2.scalar_type() == torch::kFloat32 && d2.is_contiguous() && d2.numel() >= n_owned * k,
                "d2 must be a contiguous (n_owned, k) float32 GPU tensor");
    const auto fa = field_arg(field);
    const c10::DeviceGuard guard(pts.device());
    const int gi[3] = {(int)grid[0], (int)grid[1], (int)grid[2]};
    const int c[3] = {(int)(rank % gi[0]), (int)((rank / gi[0]) % gi[1]), (int)(rank / (gi[0] * gi[1]))};
    float lo[3], hi[3];
    for (int a = 0; a < 3; ++a) {  // the own box, unbounded on domain faces (rank_local with h = 0)
        lo[a] = c[a] == 0 ? -INFINITY : (float)hdr[12 + a];
        hi[a] = c[a] == gi[a] - 1 ? INFINITY : (float)hdr[15 + a];
    }
    const kn::FieldGeom fg = kn::field_geom_hdr(hdr.data(), fa.second);
    double scale = 0.0;
    for (int a = 0; a < 3; ++a) scale = std::max({scale, std::fabs(hdr[a]), std::fabs(hdr[3 + a]), hdr[3 + a] - hdr[a]});
    auto stat = torch::zeros({2}, pts.options().dtype(torch::kInt32));
    const hipStream_t s = c10::hip::getCurrentHIPStreamMasqueradingAsCUDA().stream();
    // slack 4e-6 x scale >= the local grids' certification slack (2e-6 x their extent)
    KN_CHECK_HIP(kn::launch_field_splat(pts.data_ptr<float>(), (int)n_owned, d2.data_ptr<float>(), (int)k, lo, hi, fg,
                                        (float)(4e-6 * scale), fa.first,
                                        reinterpret_cast<unsigned*>(stat.data_ptr<int>()), s));
    return stat;
}

// Certified radius of every field cell (launch_field_cert) for a plan header's domain.
torch::Tensor field_cert(torch::Tensor field, std::vector<double> hdr) {
    TORCH_CHECK(hdr.size() >= 6, "hdr needs the domain");
    const auto fa = field_arg(field);
    const c10::DeviceGuard guard(field.device());
    auto cert = torch::empty_like(field);
    const hipStream_t s = c10::hip::getCurrentHIPStreamMasqueradingAsCUDA().stream();
    KN_CHECK_HIP(kn::launch_field_cert(fa.first, kn::field_geom_hdr(hdr.data(), fa.second), cert.data_ptr<float>(), s));
    return cert;
}

// The whole post-sync half of a distributed step in one call: unpack (self-last layout) ->
// rank box / complete box / local grid box from the plan header -> tile plan -> grid build ->
// queries of the owned points. Same arithmetic as the Python local path
// (SpatialDecomposition.rank_box / complete_box, DistributedKNearests.local_solve), so both
// give bit-identical results.
// hdr: the plan header as doubles (kn::kPlanHdr). -> (pts, gids, idx, d2, counters)
std::vector<torch::Tensor> dist_local(torch::Tensor recv, torch::Tensor self_rows, std::vector<int64_t> recv_own,
                                      std::vector<int64_t> recv_halo, int64_t rank, std::vector<int64_t> grid,
                                      std::vector<double> hdr, int64_t k, double ppc, bool deterministic,
                                      int64_t exact_grid = 0, bool adaptive = false,
                                      c10::optional<std::vector<int64_t>> dims_hint = c10::nullopt,
                                      c10::optional<torch::Tensor> pre_pts = c10::nullopt,
                                      c10::optional<torch::Tensor> pre_gids = c10::nullopt,
                                      int64_t use_tree = -1,
                                      c10::optional<torch::Tensor> field_cert = c10::nullopt) {
    TORCH_CHECK(grid.size() == 3 && hdr.size() >= (size_t)kn::kPlanHdr, "grid must have 3 entries, hdr kPlanHdr");
    const auto fc = field_arg(field_cert);
    const int64_t world = grid[0] * grid[1] * grid[2];
    TORCH_CHECK(world == (int64_t)recv_own.size(), "grid does not match the source table");
    std::vector<torch::Tensor> pg;
    if (pre_pts.has_value()) {
        // the self segment is already in place (route_steady with `place`): unpack only the rows
        // received from the other sources into the same local arrays
        TORCH_CHECK(pre_gids.has_value(), "pre_pts needs pre_gids");
        TORCH_CHECK(rank >= 0 && rank < world, "bad rank");
        kn::UnpackTable t{};
        t.world = (int)world;
        int64_t seg = 0, own = 0, halo = 0;
        for (int64_t src = 0; src < world; ++src) {
            t.seg[src] = (int)seg;
            t.own[src] = (int)recv_own[src];
            t.own_pref[src] = (int)own;
            t.halo_pref[src] = (int)halo;
            if (src != rank) seg += recv_own[src] + recv_halo[src];
            own += recv_own[src];
            halo += recv_halo[src];
        }
        t.n_own = (int)own;
        t.rows_cross = (int)seg;
        t.self = (int)rank;
        t.out_rows = (int)(own + halo);  // only the cross rows are processed; outputs span all
        TORCH_CHECK(seg == recv.size(0) && pre_pts->size(0) == own + halo && pre_gids->numel() == own + halo,
                    "source table does not add up to the received / local rows");
        KN_CHECK_HIP(kn::launch_route_unpack(reinterpret_cast<const float4*>(recv.data_ptr<float>()), nullptr,
                                             (int)seg, t, pre_pts->data_ptr<float>(), pre_gids->data_ptr<int>(),
                                             c10::hip::getCurrentHIPStreamMasqueradingAsCUDA().stream()));
        pg = {*pre_pts, *pre_gids};
    } else {
        pg = route_unpack_split(recv, self_rows, recv_own, recv_halo, rank);
    }
    int64_t n_owned = 0;
    for (auto v : recv_own) n_owned += v;
    // the rank's box / complete box / local grid box from the plan header (kn::rank_local, shared
    // with the C-API multi-GPU runtime)
    const int gi[3] = {(int)grid[0], (int)grid[1], (int)grid[2]};
    const kn::RankLocal rl = kn::rank_local(hdr.data(), (int)rank, gi, fc.first, fc.second);
    std::vector<double> complete(6), box(rl.box, rl.box + 6);
    for (int a = 0; a < 3; ++a) {
        complete[a] = (double)rl.complete.lo[a];
        complete[3 + a] = (double)rl.complete.hi[a];
    }
    const int64_t npts = pg[0].size(0);
    float fext[3] = {rl.ext[0], rl.ext[1], rl.ext[2]};
    const int th[3] = {0, 0, 0};
    kn::AutoParams ap = kn::auto_params((int)npts, (int)k, (float)ppc, th, 0, fext);
    std::vector<int64_t> dims = {ap.dims[0], ap.dims[1], ap.dims[2]};
    if (dims_hint.has_value()) {
        TORCH_CHECK(dims_hint->size() == 3 && (*dims_hint)[0] > 0 && (*dims_hint)[1] > 0 && (*dims_hint)[2] > 0,
                    "dims_hint must be 3 positive ints");
        dims = *dims_hint;  // the validated step's (possibly refined) grid: no occupancy sync
    }
    // global-id mode: the stored points carry their global ids (halo bit on non-owned points), so
    // the query epilogue writes ids without a random gather through the id table. The build writes
    // them (fused into its bucket sort) and zeroes the query counters (no memset node).
    auto counters = torch::empty({kn::kNumCounters}, pg[1].options());
    auto g = build_impl(pg[0], dims, deterministic, box, pg[1].data_ptr<int>(), (int)n_owned,
                        reinterpret_cast<unsigned*>(counters.data_ptr<int>()), kn::kNumCounters);
    bool refined = false;
    if (adaptive && !dims_hint.has_value() && npts > 0) {
        // occupancy-adaptive local grid (as kn::Engine::prepare_from): while the mean occupancy of a
        // point's cell is far above a Poisson grid's, re-bin finer (<= 3 rounds); the tile / halo /
        // LDS plan stays that of the target density. One host read per round (full steps only).
        const hipStream_t s = c10::hip::getCurrentHIPStreamMasqueradingAsCUDA().stream();
        auto occ = torch::empty({1}, pg[1].options().dtype(torch::kInt64));
        for (int round = 0; round < 3; ++round) {
            const int C = (int)(dims[0] * dims[1] * dims[2]);
            KN_CHECK_HIP(kn::launch_cell_occupancy(g[1].data_ptr<int>(), C,
                                                   reinterpret_cast<unsigned long long*>(occ.data_ptr<int64_t>()), s));
            const double w = (double)occ.cpu().item<int64_t>() / (double)npts;
            const int cur[3] = {(int)dims[0], (int)dims[1], (int)dims[2]};
            int nd[3];
            if (!kn::refine_dims(cur, w, (int)k, (float)ppc, (int)npts, nd, ap.xsub)) break;
            dims = {nd[0], nd[1], nd[2]};
            g = build_impl(pg[0], dims, deterministic, box, pg[1].data_ptr<int>(), (int)n_owned,
                           reinterpret_cast<unsigned*>(counters.data_ptr<int>()), kn::kNumCounters);
            refined = true;
        }
    }
    // use_tree: -1 auto (the local grid had to be refined: a share too non-uniform for one cell
    // size, as kn::Engine decides on one GPU), 0 grid, 1 tree
    const int dims3[3] = {(int)dims[0], (int)dims[1], (int)dims[2]};
    const bool tree = (use_tree < 0 ? refined : use_tree != 0) && kn::tree_supports(dims3);
    auto dims_t = torch::tensor({dims[0], dims[1], dims[2]}, torch::kInt64);
    auto tree_t = torch::tensor({(int64_t)(tree ? 1 : 0)}, torch::kInt64);
    if (tree && npts > 0) {
        // Morton-leaf tree over the local grid's points in global-id mode (owned points are the
        // queries), then the complete-box certification the grid kernels do inline: uncertified
        // rows go to the forwarding round
        auto tb = tree_build_impl(g[0], g[1], g[3], dims, false);
        auto tq = tree_query(std::get<0>(tb), std::get<1>(tb), dims, npts, k, n_owned, c10::nullopt, true, 0, g[2]);
        auto uncert = torch::empty({std::max<int64_t>(1, n_owned)}, pg[1].options());
        // the rank's whole complete box (wide zone, halo field), as the grid kernels below
        const kn::CompleteBox cb = rl.complete;
        KN_CHECK_HIP(kn::launch_certify_rows(pg[0].data_ptr<float>(), (int)n_owned, (int)k, tq[1].data_ptr<float>(), cb,
                                             reinterpret_cast<const kn::GridGeom*>(g[3].data_ptr<int>()),
                                             reinterpret_cast<unsigned*>(tq[2].data_ptr<int>()),
                                             reinterpret_cast<unsigned*>(uncert.data_ptr<int>()),
                                             c10::hip::getCurrentHIPStreamMasqueradingAsCUDA().stream()));
        return {pg[0], pg[1], tq[0], tq[1], tq[2], g[0], g[1], g[3], g[2], uncert, dims_t, tree_t};
    }
    if (dims[0] != ap.dims[0] || dims[1] != ap.dims[1] || dims[2] != ap.dims[2]) {
        // a refined grid (this step's or the validated step's hint): isotropic, xsub 1
        ap.tile[0] = std::max(1, ap.tile[0] / std::max(1, ap.xsub));
        ap.xsub = 1;
    }
    auto q = query_impl(g[0], g[1], g[3], dims, k, n_owned, c10::nullopt, complete, {ap.tile[0], ap.tile[1], ap.tile[2]},
                        ap.halo, ap.lds_capacity, true, true, 0, g[2], exact_grid, counters, 0, ap.xsub, &rl.complete);
    // + the local grid (global-id mode) and the uncertified list, for query forwarding
    return {pg[0], pg[1], q[0], q[1], q[2], g[0], g[1], g[3], g[2], q[3], dims_t, tree_t};
}

// Exact K nearest of external points (multi-GPU query forwarding) among a global-id-mode local
// grid: ext (M, 4) float32 {x, y, z, bits(global id)} -> (idx (M, k) global ids, d2 (M, k))
std::vector<torch::Tensor> query_external(torch::Tensor sorted, torch::Tensor cell_start, torch::Tensor geom,
                                          std::vector<int64_t> dims, int64_t k, torch::Tensor ext,
                                          torch::Tensor row_of) {
    TORCH_CHECK(sorted.is_cuda() && sorted.dim() == 2 && sorted.size(1) == 4, "sorted must be (N,4) GPU");
    TORCH_CHECK(ext.is_cuda() && ext.dim() == 2 && ext.size(1) == 4 && ext.scalar_type() == torch::kFloat32 &&
                    ext.is_contiguous(), "ext must be a contiguous (M,4) float32 GPU tensor");
    TORCH_CHECK(dims.size() == 3 && cell_start.numel() == dims[0] * dims[1] * dims[2] + 1, "bad dims");
    TORCH_CHECK(k >= 1 && k <= 128, "k must be in [1, 128]");
    TORCH_CHECK(row_of.is_cuda() && row_of.scalar_type() == torch::kInt32 && row_of.numel() >= sorted.size(0),
                "row_of must be the grid's int32 perm");
    const c10::DeviceGuard guard(sorted.device());
    const int64_t m = ext.size(0);
    auto idx = torch::empty({m, k}, sorted.options().dtype(torch::kInt32));
    auto d2 = torch::empty({m, k}, sorted.options());
    auto counters = torch::zeros({kn::kNumCounters}, sorted.options().dtype(torch::kInt32));
    kn::QueryBuffers q{};
    q.sorted = reinterpret_cast<const float4*>(sorted.data_ptr<float>());
    q.cell_start = cell_start.data_ptr<int>();
    q.geom = reinterpret_cast<const kn::GridGeom*>(geom.data_ptr<int>());
    q.n = (int)sorted.size(0);
    for (int a = 0; a < 3; ++a) q.dims[a] = (int)dims[a];
    q.k = (int)k;
    q.row_of = reinterpret_cast<const unsigned*>(row_of.data_ptr<int>());
    q.out_idx = reinterpret_cast<unsigned*>(idx.data_ptr<int>());
    q.out_dist = d2.data_ptr<float>();
    q.counters = reinterpret_cast<unsigned*>(counters.data_ptr<int>());
    const hipStream_t s = c10::hip::getCurrentHIPStreamMasqueradingAsCUDA().stream();
    KN_CHECK_HIP(kn::launch_query_external(q, reinterpret_cast<const float4*>(ext.data_ptr<float>()), (int)m, s));
    return {idx, d2};
}

// ---- query forwarding inside a sync-free step (kn/route.h launch_fwd_pack / launch_fwd_merge) ----
// -> {send (world*F*2, 4) f32, slot_of (umax*world) i32, stat (2) i32: [1] = overflow}
std::vector<torch::Tensor> fwd_pack(torch::Tensor plan, int64_t world, int64_t rank, int64_t F, int64_t k,
                                    torch::Tensor uncert, torch::Tensor counters, int64_t umax, torch::Tensor pts,
                                    torch::Tensor gids, torch::Tensor d2) {
    TORCH_CHECK(plan.is_cuda() && plan.numel() == (int64_t)sizeof(kn::RouteParams), "plan must be a route plan");
    TORCH_CHECK(world >= 1 && world <= kn::kRouteMaxWorld && rank >= 0 && rank < world, "bad world / rank");
    TORCH_CHECK(F >= 1 && F <= (1 << 20) && umax >= 0 && umax <= (1 << 24), "bad slot capacity");
    TORCH_CHECK(k >= 1 && k <= 128, "k must be in [1, 128]");
    TORCH_CHECK(uncert.is_cuda() && uncert.scalar_type() == torch::kInt32, "uncert: int32 GPU list");
    TORCH_CHECK(counters.is_cuda() && counters.scalar_type() == torch::kInt32 && counters.numel() >= 2, "counters");
    TORCH_CHECK(pts.is_cuda() && pts.scalar_type() == torch::kFloat32 && pts.dim() == 2 && pts.size(1) == 3 &&
                    pts.is_contiguous(), "pts: (rows, 3) f32");
    TORCH_CHECK(gids.is_cuda() && gids.scalar_type() == torch::kInt32 && gids.numel() >= pts.size(0), "gids");
    TORCH_CHECK(d2.is_cuda() && d2.scalar_type() == torch::kFloat32 && d2.dim() == 2 && d2.size(1) == k &&
                    d2.is_contiguous(), "d2: (owned, k) f32");
    TORCH_CHECK(uncert.numel() >= std::min<int64_t>(umax, d2.size(0)) || d2.size(0) == 0, "uncert list too short");
    const c10::DeviceGuard guard(pts.device());
    auto f32 = pts.options();
    auto i32 = pts.options().dtype(torch::kInt32);
    auto send = torch::empty({world * F * 2, 4}, f32);
    auto slot_row = torch::empty({world * F}, i32);
    auto slot_of = torch::empty({std::max<int64_t>(1, umax * world)}, i32);
    auto cnt = torch::empty({world}, i32);
    auto stat = torch::zeros({2}, i32);
    const int um = (int)std::min<int64_t>(umax, d2.size(0));
    const hipStream_t s = c10::hip::getCurrentHIPStreamMasqueradingAsCUDA().stream();
    KN_CHECK_HIP(kn::launch_fwd_pack(reinterpret_cast<const kn::RouteParams*>(plan.data_ptr<uint8_t>()), (int)world,
                                     (int)rank, (int)F, (int)k, reinterpret_cast<const unsigned*>(uncert.data_ptr<int>()),
                                     reinterpret_cast<const unsigned*>(counters.data_ptr<int>() + 1), um,
                                     pts.data_ptr<float>(), gids.data_ptr<int>(), d2.data_ptr<float>(),
                                     reinterpret_cast<float4*>(send.data_ptr<float>()), slot_row.data_ptr<int>(),
                                     slot_of.data_ptr<int>(), cnt.data_ptr<int>(),
                                     reinterpret_cast<unsigned*>(stat.data_ptr<int>()), s));
    return {send, slot_of, stat};
}

// Answers to received forwarding slots from the local grid (global-id mode): -> {idx (slots, k)
// global ids, d2 (slots, k)}; rows of empty slots are undefined.
std::vector<torch::Tensor> fwd_answer(torch::Tensor sorted, torch::Tensor cell_start, torch::Tensor geom,
                                      std::vector<int64_t> dims, int64_t k, torch::Tensor slots, torch::Tensor row_of) {
    TORCH_CHECK(sorted.is_cuda() && sorted.dim() == 2 && sorted.size(1) == 4, "sorted must be (N,4) GPU");
    TORCH_CHECK(slots.is_cuda() && slots.dim() == 2 && slots.size(1) == 4 && slots.size(0) % 2 == 0 &&
                    slots.scalar_type() == torch::kFloat32 && slots.is_contiguous(), "slots: (2*S, 4) f32");
    TORCH_CHECK(dims.size() == 3 && cell_start.numel() == dims[0] * dims[1] * dims[2] + 1, "bad dims");
    TORCH_CHECK(k >= 1 && k <= 128, "k must be in [1, 128]");
    TORCH_CHECK(row_of.is_cuda() && row_of.scalar_type() == torch::kInt32 && row_of.numel() >= sorted.size(0),
                "row_of must be the grid's int32 perm");
    const c10::DeviceGuard guard(sorted.device());
    const int64_t m = slots.size(0) / 2;
    auto idx = torch::empty({m, k}, sorted.options().dtype(torch::kInt32));
    auto d2 = torch::empty({m, k}, sorted.options());
    auto counters = torch::zeros({kn::kNumCounters}, sorted.options().dtype(torch::kInt32));
    kn::QueryBuffers q{};
    q.sorted = reinterpret_cast<const float4*>(sorted.data_ptr<float>());
    q.cell_start = cell_start.data_ptr<int>();
    q.geom = reinterpret_cast<const kn::GridGeom*>(geom.data_ptr<int>());
    q.n = (int)sorted.size(0);
    for (int a = 0; a < 3; ++a) q.dims[a] = (int)dims[a];
    q.k = (int)k;
    q.row_of = reinterpret_cast<const unsigned*>(row_of.data_ptr<int>());
    q.out_idx = reinterpret_cast<unsigned*>(idx.data_ptr<int>());
    q.out_dist = d2.data_ptr<float>();
    q.counters = reinterpret_cast<unsigned*>(counters.data_ptr<int>());
    const hipStream_t s = c10::hip::getCurrentHIPStreamMasqueradingAsCUDA().stream();
    KN_CHECK_HIP(kn::launch_query_external_slots(q, reinterpret_cast<const float4*>(slots.data_ptr<float>()), (int)m, s));
    return {idx, d2};
}

// Merges the answers (all-to-all'd back: (world*F, k) each) into the forwarded rows, in place.
void fwd_merge(int64_t world, int64_t F, int64_t k, torch::Tensor uncert, torch::Tensor counters, int64_t umax,
               torch::Tensor slot_of, torch::Tensor back_idx, torch::Tensor back_d2, torch::Tensor idx, torch::Tensor d2) {
    TORCH_CHECK(back_idx.is_cuda() && back_idx.scalar_type() == torch::kInt32 && back_idx.numel() == world * F * k,
                "back_idx: (world*F, k) i32");
    TORCH_CHECK(back_d2.is_cuda() && back_d2.scalar_type() == torch::kFloat32 && back_d2.numel() == world * F * k,
                "back_d2: (world*F, k) f32");
    TORCH_CHECK(idx.is_cuda() && idx.scalar_type() == torch::kInt32 && idx.dim() == 2 && idx.size(1) == k &&
                    idx.is_contiguous(), "idx: (owned, k) i32");
    TORCH_CHECK(d2.is_cuda() && d2.scalar_type() == torch::kFloat32 && d2.sizes() == idx.sizes() && d2.is_contiguous(),
                "d2 like idx");
    TORCH_CHECK(slot_of.is_cuda() && slot_of.numel() >= std::min<int64_t>(umax, idx.size(0)) * world, "slot_of");
    const c10::DeviceGuard guard(idx.device());
    const hipStream_t s = c10::hip::getCurrentHIPStreamMasqueradingAsCUDA().stream();
    KN_CHECK_HIP(kn::launch_fwd_merge((int)world, (int)F, (int)k, reinterpret_cast<const unsigned*>(uncert.data_ptr<int>()),
                                      reinterpret_cast<const unsigned*>(counters.data_ptr<int>() + 1),
                                      (int)std::min<int64_t>(umax, idx.size(0)), slot_of.data_ptr<int>(),
                                      back_idx.data_ptr<int>(), back_d2.data_ptr<float>(), idx.data_ptr<int>(),
                                      d2.data_ptr<float>(), s));
}

// Sync-free distributed step check (one wave, on device): (1,) int32 = mismatch of this rank's
// meta / send counts against the planned ones + (uncertified queries > 0)
torch::Tensor steady_flag(torch::Tensor local, torch::Tensor metas, int64_t rank, torch::Tensor totals,
                          torch::Tensor planned_totals, torch::Tensor counters) {
    TORCH_CHECK(local.is_cuda() && local.scalar_type() == torch::kFloat64 && local.numel() == 8, "local: (8,) f64 GPU");
    TORCH_CHECK(metas.is_cuda() && metas.scalar_type() == torch::kFloat64 && metas.numel() >= 8 * (rank + 1) &&
                    metas.is_contiguous(), "metas: (world*8,) f64 GPU");
    TORCH_CHECK(totals.is_cuda() && planned_totals.is_cuda() && totals.scalar_type() == torch::kInt32 &&
                    planned_totals.scalar_type() == torch::kInt32 && totals.numel() == planned_totals.numel() &&
                    totals.is_contiguous() && planned_totals.is_contiguous(), "totals: matching int32 GPU tensors");
    TORCH_CHECK(counters.is_cuda() && counters.scalar_type() == torch::kInt32 && counters.numel() >= 2, "counters");
    const c10::DeviceGuard guard(local.device());
    auto flag = torch::empty({1}, counters.options());
    const hipStream_t s = c10::hip::getCurrentHIPStreamMasqueradingAsCUDA().stream();
    KN_CHECK_HIP(kn::launch_steady_flag(local.data_ptr<double>(), metas.data_ptr<double>() + 8 * rank,
                                        totals.data_ptr<int>(), planned_totals.data_ptr<int>(), (int)totals.numel(),
                                        reinterpret_cast<const unsigned*>(counters.data_ptr<int>()),
                                        flag.data_ptr<int>(), s));
    return flag;
}

// World-1 steady step check from one bbox pass over the share (no routing pass): (1,) int32 flag.
// sticky ((1,) int32 GPU) + host ((1,) int32 pinned CPU), optional: the flag is max-accumulated
// into sticky and stored to host by the kernel (graph replays need no copy node after the step).
torch::Tensor steady_flag_local(torch::Tensor points, torch::Tensor metas, int64_t rank, torch::Tensor counters,
                                c10::optional<torch::Tensor> sticky, c10::optional<torch::Tensor> host) {
    check_points(points, true);
    TORCH_CHECK(metas.is_cuda() && metas.scalar_type() == torch::kFloat64 && metas.numel() >= 8 * (rank + 1) &&
                    metas.is_contiguous(), "metas: (world*8,) f64 GPU");
    TORCH_CHECK(counters.is_cuda() && counters.scalar_type() == torch::kInt32 && counters.numel() >= 2, "counters");
    TORCH_CHECK(sticky.has_value() == host.has_value(), "sticky and host go together");
    const c10::DeviceGuard guard(points.device());
    int* sp = nullptr;
    int* hp = nullptr;
    if (sticky.has_value()) {
        TORCH_CHECK(sticky->is_cuda() && sticky->scalar_type() == torch::kInt32 && sticky->numel() == 1, "sticky");
        TORCH_CHECK(!host->is_cuda() && host->is_pinned() && host->scalar_type() == torch::kInt32 && host->numel() == 1,
                    "host: (1,) int32 pinned CPU tensor");
        void* d = nullptr;
        KN_CHECK_HIP(hipHostGetDevicePointer(&d, host->data_ptr(), 0));
        sp = sticky->data_ptr<int>();
        hp = static_cast<int*>(d);
    }
    auto words = torch::empty({kn::kBBoxWords}, points.options().dtype(torch::kInt32));
    auto flag = torch::empty({1}, counters.options());
    const hipStream_t s = c10::hip::getCurrentHIPStreamMasqueradingAsCUDA().stream();
    KN_CHECK_HIP(kn::launch_steady_flag_local(points.data_ptr<float>(), (int)points.size(0),
                                              reinterpret_cast<unsigned*>(words.data_ptr<int>()),
                                              metas.data_ptr<double>() + 8 * rank,
                                              reinterpret_cast<const unsigned*>(counters.data_ptr<int>()),
                                              flag.data_ptr<int>(), sp, hp, s));
    return flag;
}

// Pre-collective half of a steady-state step: counts + scatter with the validated step's plan
// (no re-planning; the plan kernel is a serial one-thread pass) and this share's bbox partials
// taken by the counting pass. -> (totals (2*world,) int32, send (cap, 4), partials)
std::vector<torch::Tensor> route_steady(torch::Tensor points, c10::optional<torch::Tensor> ids, torch::Tensor plan,
                                        int64_t world, int64_t cap, int64_t rank,
                                        c10::optional<std::vector<int64_t>> place = c10::nullopt) {
    check_points(points, true);
    TORCH_CHECK(plan.is_cuda() && plan.numel() == (int64_t)sizeof(kn::RouteParams), "plan must be a route plan");
    TORCH_CHECK(world >= 1 && world <= kn::kRouteMaxWorld && rank >= 0 && rank < world, "bad world / rank");
    TORCH_CHECK(cap >= 0 && cap < INT32_MAX, "cap out of range");
    const c10::DeviceGuard guard(points.device());
    const int n = (int)points.size(0);
    const int* idp = nullptr;
    if (ids.has_value()) {
        TORCH_CHECK(ids->is_cuda() && ids->scalar_type() == torch::kInt32 && ids->numel() == n && ids->is_contiguous(),
                    "ids must be a contiguous int32 GPU tensor of N entries");
        idp = ids->data_ptr<int>();
    }
    auto i32 = points.options().dtype(torch::kInt32);
    const int nb = kn::route_block_count(n);
    auto totals = torch::empty({2 * world}, i32);
    auto bc = torch::empty({2 * world * (int64_t)nb}, i32);
    auto partials = torch::empty({6 * (int64_t)nb}, i32);
    auto send = torch::empty({cap, 4}, points.options());
    const auto* pp = reinterpret_cast<const kn::RouteParams*>(plan.data_ptr<uint8_t>());
    const hipStream_t s = c10::hip::getCurrentHIPStreamMasqueradingAsCUDA().stream();
    KN_CHECK_HIP(kn::launch_route_count(points.data_ptr<float>(), n, pp, (int)world, bc.data_ptr<int>(),
                                        totals.data_ptr<int>(), s, reinterpret_cast<unsigned*>(partials.data_ptr<int>())));
    if (place.has_value()) {
        // place = [own_base, halo_base, local rows, planned own, planned halo]: the self segment
        // goes straight to the local (rows, 3) points / global ids (SelfPlace); send holds only the
        // other destinations' rows. A self segment of another size than planned writes nothing.
        TORCH_CHECK(place->size() == 5 && (*place)[2] >= 0 && (*place)[2] < INT32_MAX,
                    "place = [own_base, halo_base, rows, own_cnt, halo_cnt]");
        auto lpts = torch::empty({(*place)[2], 3}, points.options());
        auto lgids = torch::empty({(*place)[2]}, i32);
        kn::SelfPlace sp{lpts.data_ptr<float>(), lgids.data_ptr<int>(), (int)(*place)[0], (int)(*place)[1],
                         (int)(*place)[2], (int)(*place)[3], (int)(*place)[4]};
        KN_CHECK_HIP(kn::launch_route_scatter(points.data_ptr<float>(), idp, n, pp, (int)world, bc.data_ptr<int>(),
                                              totals.data_ptr<int>(), reinterpret_cast<float4*>(send.data_ptr<float>()),
                                              (int)cap, (int)rank, s, &sp));
        return {totals, send, partials, lpts, lgids};
    }
    KN_CHECK_HIP(kn::launch_route_scatter(points.data_ptr<float>(), idp, n, pp, (int)world, bc.data_ptr<int>(),
                                          totals.data_ptr<int>(), reinterpret_cast<float4*>(send.data_ptr<float>()),
                                          (int)cap, (int)rank, s));
    return {totals, send, partials};
}

// Steady-state check from route_steady's partials: (1,) int32, non-zero = the share's meta or send
// counts differ from the validated step's, or a query is uncertified
torch::Tensor steady_flag_partials(torch::Tensor partials, int64_t n, torch::Tensor metas, int64_t rank,
                                   torch::Tensor totals, torch::Tensor planned_totals, torch::Tensor counters) {
    TORCH_CHECK(partials.is_cuda() && partials.scalar_type() == torch::kInt32 &&
                    partials.numel() == 6 * (int64_t)kn::route_block_count((int)n), "partials of route_steady");
    TORCH_CHECK(metas.is_cuda() && metas.scalar_type() == torch::kFloat64 && metas.numel() >= 8 * (rank + 1) &&
                    metas.is_contiguous(), "metas: (world*8,) f64 GPU");
    TORCH_CHECK(totals.is_cuda() && planned_totals.is_cuda() && totals.scalar_type() == torch::kInt32 &&
                    planned_totals.scalar_type() == torch::kInt32 && totals.numel() == planned_totals.numel() &&
                    totals.is_contiguous() && planned_totals.is_contiguous(), "totals: matching int32 GPU tensors");
    TORCH_CHECK(counters.is_cuda() && counters.scalar_type() == torch::kInt32 && counters.numel() >= 2, "counters");
    const c10::DeviceGuard guard(partials.device());
    auto flag = torch::empty({1}, counters.options());
    const hipStream_t s = c10::hip::getCurrentHIPStreamMasqueradingAsCUDA().stream();
    KN_CHECK_HIP(kn::launch_steady_flag_partials(reinterpret_cast<const unsigned*>(partials.data_ptr<int>()), (int)n, (int)n,
                                                 metas.data_ptr<double>() + 8 * rank, totals.data_ptr<int>(),
                                                 planned_totals.data_ptr<int>(), (int)totals.numel(),
                                                 reinterpret_cast<const unsigned*>(counters.data_ptr<int>()),
                                                 flag.data_ptr<int>(), s));
    return flag;
}

void cell_sort(torch::Tensor sorted, torch::Tensor cell_start, torch::Tensor perm, torch::Tensor geom) {
    TORCH_CHECK(sorted.is_cuda() && sorted.dim() == 2 && sorted.size(1) == 4, "sorted must be (N,4) GPU");
    TORCH_CHECK(cell_start.is_cuda() && cell_start.scalar_type() == torch::kInt32, "cell_start must be int32 GPU");
    TORCH_CHECK(perm.is_cuda() && perm.numel() == sorted.size(0), "perm must match sorted");
    TORCH_CHECK(geom.is_cuda() && geom.numel() == 16, "geom must be a 16-int GPU tensor");
    const c10::DeviceGuard guard(sorted.device());
    auto tmp = torch::empty_like(sorted);
    const hipStream_t s = c10::hip::getCurrentHIPStreamMasqueradingAsCUDA().stream();
    KN_CHECK_HIP(kn::launch_cell_sort(cell_start.data_ptr<int>(), reinterpret_cast<const kn::GridGeom*>(geom.data_ptr<int>()),
                                      (int)sorted.size(0), reinterpret_cast<float4*>(sorted.data_ptr<float>()),
                                      reinterpret_cast<unsigned*>(perm.data_ptr<int>()),
                                      reinterpret_cast<float4*>(tmp.data_ptr<float>()), s));
}

// occupancy-adaptive grid: sum over cells of count^2 (int64, on device, no sync)
torch::Tensor occupancy(torch::Tensor cell_start) {
    TORCH_CHECK(cell_start.is_cuda() && cell_start.scalar_type() == torch::kInt32 && cell_start.is_contiguous() &&
                    cell_start.numel() >= 1,
                "cell_start must be a contiguous int32 GPU tensor of C + 1 entries");
    const c10::DeviceGuard guard(cell_start.device());
    auto out = torch::empty({1}, cell_start.options().dtype(torch::kInt64));
    const hipStream_t s = c10::hip::getCurrentHIPStreamMasqueradingAsCUDA().stream();
    KN_CHECK_HIP(kn::launch_cell_occupancy(cell_start.data_ptr<int>(), (int)cell_start.numel() - 1,
                                           reinterpret_cast<unsigned long long*>(out.data_ptr<int64_t>()), s));
    return out;
}

py::object refine_dims(std::vector<int64_t> dims, double w, int64_t k, double ppc, int64_t n, int64_t xsub) {
    TORCH_CHECK(dims.size() == 3, "dims must have 3 entries");
    const int d[3] = {(int)dims[0], (int)dims[1], (int)dims[2]};
    int out[3];
    if (!kn::refine_dims(d, w, (int)k, (float)ppc, (int)n, out, (int)xsub)) return py::none();
    return py::cast(std::vector<int64_t>{out[0], out[1], out[2]});
}

// -> (8,) float64 {lo[3], hi[3], n, 0} of this rank's points (one kernel pass, no host sync)
torch::Tensor local_meta(torch::Tensor points) {
    check_points(points, true);
    const c10::DeviceGuard guard(points.device());
    auto words = torch::empty({kn::kBBoxWords}, points.options().dtype(torch::kInt32));
    auto out = torch::empty({8}, points.options().dtype(torch::kFloat64));
    const hipStream_t s = c10::hip::getCurrentHIPStreamMasqueradingAsCUDA().stream();
    KN_CHECK_HIP(kn::launch_local_meta(points.data_ptr<float>(), (int)points.size(0),
                                       reinterpret_cast<unsigned*>(words.data_ptr<int>()), out.data_ptr<double>(), s));
    return out;
}

// ---- native engine (own arena + own stream + hipGraph), the C API's runtime ------------
class PyEngine {
public:
    PyEngine(int64_t k, double ppc, std::vector<int64_t> tile, int64_t halo, bool deterministic, bool use_tiles,
             bool with_dist, int64_t device, bool adaptive, int64_t algo) {
        kn::EngineConfig c;
        c.k = (int)k;
        c.points_per_cell = (float)ppc;
        for (size_t a = 0; a < 3 && a < tile.size(); ++a) c.tile[a] = (int)tile[a];
        c.halo = (int)halo;
        c.deterministic = deterministic ? 1 : 0;
        c.use_tiles = use_tiles ? 1 : 0;
        c.adaptive = adaptive ? 1 : 0;
        c.algo = (int)algo;
        c.with_distances = with_dist ? 1 : 0;
        c.device = (int)device;
        e_ = std::make_unique<kn::Engine>(c);
    }
    void prepare(torch::Tensor points) {
        check_points(points, true);
        const c10::DeviceGuard guard(points.device());
        // the engine's own stream must see the producer's writes
        KN_CHECK_HIP(hipStreamSynchronize(c10::hip::getCurrentHIPStreamMasqueradingAsCUDA().stream()));
        TORCH_CHECK(e_->prepare_device(points.data_ptr<float>(), (int)points.size(0)) == KN_OK, e_->error());
    }
    void prepare_async(torch::Tensor points) {
        check_points(points, true);
        const c10::DeviceGuard guard(points.device());
        KN_CHECK_HIP(hipStreamSynchronize(c10::hip::getCurrentHIPStreamMasqueradingAsCUDA().stream()));
        TORCH_CHECK(e_->upload_device(points.data_ptr<float>(), (int)points.size(0)) == KN_OK, e_->error());
    }
    void solve() { TORCH_CHECK(e_->solve() == KN_OK, e_->error()); }
    void set_k(int64_t k) { TORCH_CHECK(e_->set_k((int)k) == KN_OK, e_->error()); }
    void launch_graph(int64_t iters) { TORCH_CHECK(e_->launch_graph((int)iters) == KN_OK, e_->error()); }
    void launch_pipelined(int64_t iters, int64_t unroll) {
        TORCH_CHECK(e_->launch_pipelined((int)iters, (int)unroll) == KN_OK, e_->error());
    }
    // One step of a stream of distinct clouds (same N as the prepared cloud): this step's points and
    // optionally the next step's (binned now, while this step queries). Stream-ordered: the
    // caller's tensors must stay unchanged until sync() (or the step after next).
    void stream_step(torch::Tensor points, c10::optional<torch::Tensor> next) {
        check_points(points, true);
        TORCH_CHECK(points.size(0) == e_->n(), "stream_step: every cloud must have the prepared N points");
        const float* np = nullptr;
        if (next.has_value()) {
            check_points(*next, true);
            TORCH_CHECK(next->size(0) == e_->n(), "stream_step: every cloud must have the prepared N points");
            np = next->data_ptr<float>();
        }
        const c10::DeviceGuard guard(points.device());
        // the engine's streams must see the producer's writes
        KN_CHECK_HIP(hipStreamSynchronize(c10::hip::getCurrentHIPStreamMasqueradingAsCUDA().stream()));
        TORCH_CHECK(e_->stream_step(points.data_ptr<float>(), np) == KN_OK, e_->error());
    }
    // a batch of distinct clouds (kn::Engine::stream_batch): points[j] (N, 3) float32 GPU ->
    // idx[j] (N, K) int32 and d2[j] (N, K) float32 (optional) in original space. Asynchronous on
    // the engine's streams: call sync() before reading the outputs.
    // mode: "eager" (default: the eager batch pipeline) or "graph" (captured batch graphs)
    void stream_batch(std::vector<torch::Tensor> points, std::vector<torch::Tensor> idx,
                      c10::optional<std::vector<torch::Tensor>> d2, c10::optional<std::string> mode) {
        if (mode.has_value()) {
            TORCH_CHECK(*mode == "eager" || *mode == "graph", "stream_batch: mode is 'eager' or 'graph'");
            e_->set_batch_mode(*mode == "graph" ? 1 : 0);
        }
        const size_t m = points.size();
        TORCH_CHECK(idx.size() == m && (!d2.has_value() || d2->size() == m), "one output per cloud");
        std::vector<const float*> in(m);
        std::vector<unsigned*> oi(m);
        std::vector<float*> od(m);
        for (size_t j = 0; j < m; ++j) {
            check_points(points[j], true);
            TORCH_CHECK(points[j].size(0) == e_->n(), "stream_batch: every cloud must have the prepared N points");
            TORCH_CHECK(idx[j].is_cuda() && idx[j].scalar_type() == torch::kInt32 && idx[j].is_contiguous() &&
                            idx[j].numel() == (int64_t)e_->n() * e_->k(), "idx[j]: contiguous (N, K) int32 GPU");
            in[j] = points[j].data_ptr<float>();
            oi[j] = reinterpret_cast<unsigned*>(idx[j].data_ptr<int>());
            if (d2.has_value()) {
                const auto& t = (*d2)[j];
                TORCH_CHECK(t.is_cuda() && t.scalar_type() == torch::kFloat32 && t.is_contiguous() &&
                                t.numel() == (int64_t)e_->n() * e_->k(), "d2[j]: contiguous (N, K) float32 GPU");
                od[j] = t.data_ptr<float>();
            }
        }
        if (m == 0) return;
        const c10::DeviceGuard guard(points[0].device());
        KN_CHECK_HIP(hipStreamSynchronize(c10::hip::getCurrentHIPStreamMasqueradingAsCUDA().stream()));
        TORCH_CHECK(e_->stream_batch((int)m, in.data(), oi.data(), d2.has_value() ? od.data() : nullptr) == KN_OK,
                    e_->error());
        // the batch still reads / writes these tensors on the engine's private streams: hold them
        // until sync() (a caller dropping one early must not let the caching allocator
        // hand its memory to other work while the batch runs)
        for (size_t j = 0; j < m; ++j) {
            held_.push_back(points[j]);
            held_.push_back(idx[j]);
            if (d2.has_value()) held_.push_back((*d2)[j]);
        }
    }
    // per-engine pipeline shape (query streams 1 / 2, grid sets 2 / 3; -1: KN_PIPE_* defaults)
    void set_pipeline_shape(int64_t query_streams, int64_t sets) {
        TORCH_CHECK(e_->set_pipeline_shape((int)query_streams, (int)sets) == KN_OK, e_->error());
    }
    // stored -> original permutation of the engine's current grid (host int32)
    torch::Tensor permutation() {
        unsigned* p = e_->get_permutation();
        TORCH_CHECK(p, e_->error());
        auto t = torch::empty({(int64_t)e_->n()}, torch::kInt32);
        std::memcpy(t.data_ptr<int>(), p, (size_t)e_->n() * sizeof(unsigned));
        free(p);
        return t;
    }
    void sync() {
        TORCH_CHECK(e_->sync() == KN_OK, e_->error());
        held_.clear();  // every batch enqueued so far has finished with its tensors
    }
    std::vector<torch::Tensor> results(torch::Device dev) {
        const int64_t n = e_->n(), k = e_->k();
        auto opt = torch::TensorOptions().device(dev);
        auto idx = torch::empty({n, k}, opt.dtype(torch::kInt32));
        auto d2 = torch::empty({n, k}, opt.dtype(torch::kFloat32));
        TORCH_CHECK(e_->copy_results(reinterpret_cast<unsigned*>(idx.data_ptr<int>()), d2.data_ptr<float>()) == KN_OK,
                    e_->error());
        return {idx, d2};
    }
    // queries [first, first + count) only, (count, K) ids (original space) + squared distances
    std::vector<torch::Tensor> solve_range(int64_t first, int64_t count, torch::Device dev) {
        TORCH_CHECK(first >= 0 && count >= 0 && first + count <= e_->n(), "query range outside [0, N)");
        const int64_t k = e_->k();
        auto opt = torch::TensorOptions().device(dev);
        auto idx = torch::empty({count, k}, opt.dtype(torch::kInt32));
        auto d2 = torch::empty({count, k}, opt.dtype(torch::kFloat32));
        TORCH_CHECK(e_->solve_range((int)first, (int)count, reinterpret_cast<unsigned*>(idx.data_ptr<int>()),
                                    d2.data_ptr<float>()) == KN_OK,
                    e_->error());
        return {idx, d2};
    }
    std::vector<int64_t> counters() {
        unsigned c[kn::kNumCounters];
        TORCH_CHECK(e_->counters(c) == KN_OK, e_->error());
        return std::vector<int64_t>(c, c + kn::kNumCounters);
    }
    py::dict info() {
        py::dict d;
        d["n"] = e_->n();
        d["k"] = e_->k();
        d["dims"] = std::vector<int>{e_->dims()[0], e_->dims()[1], e_->dims()[2]};
        d["ms_build"] = e_->ms_build();
        d["ms_solve"] = e_->ms_solve();
        d["algo"] = e_->uses_tree() ? "tree" : "grid";
        d["tree_leaves"] = e_->tree_leaves();
        return d;
    }

private:
    std::unique_ptr<kn::Engine> e_;
    std::vector<torch::Tensor> held_;  // stream_batch inputs / outputs in flight (released by sync())
};

// -DKN_PHASES=1 builds: knn_tile_kernel wave cycles per phase (kn/kernels.h); empty otherwise
std::vector<int64_t> debug_phase_cycles(bool reset) {
    unsigned long long v[8];
    if (kn::debug_phase_cycles(v, reset) != hipSuccess) return {};
    return std::vector<int64_t>(v, v + 8);
}

std::vector<int64_t> debug_words(bool reset) {
    unsigned b[4], q[4], r[4], t[4];
    KN_CHECK_HIP(kn::debug_words_build(b, reset));
    KN_CHECK_HIP(kn::debug_words_query(q, reset));
    KN_CHECK_HIP(kn::debug_words_route(r, reset));
    KN_CHECK_HIP(kn::debug_words_tree(t, reset));
    return {b[0], b[1], b[2], b[3], q[0], q[1], q[2], q[3], r[0], r[1], r[2], r[3], t[0], t[1], t[2], t[3]};
}

// ---- CPU (host) components ----------------------------------------------------------
std::vector<torch::Tensor> kdtree_knn(torch::Tensor points, int64_t k, int64_t threads) {
    check_points(points, false);
    const int n = (int)points.size(0);
    auto idx = torch::empty({n, k}, torch::kInt32);
    auto d2 = torch::empty({n, k}, torch::kFloat32);
    {
        py::gil_scoped_release nogil;
        knh::kdtree_knn_all(points.data_ptr<float>(), n, (int)k, reinterpret_cast<uint32_t*>(idx.data_ptr<int>()),
                            d2.data_ptr<float>(), (int)threads);
    }
    return {idx, d2};
}

std::vector<torch::Tensor> brute_knn(torch::Tensor points, int64_t k, int64_t threads) {
    check_points(points, false);
    const int n = (int)points.size(0);
    auto idx = torch::empty({n, k}, torch::kInt32);
    auto d2 = torch::empty({n, k}, torch::kFloat32);
    {
        py::gil_scoped_release nogil;
        knh::brute_knn_all(points.data_ptr<float>(), n, (int)k, reinterpret_cast<uint32_t*>(idx.data_ptr<int>()),
                           d2.data_ptr<float>(), (int)threads);
    }
    return {idx, d2};
}

std::vector<torch::Tensor> grid_knn_cpu(torch::Tensor points, int64_t n_queries, int64_t k, double ppc,
                                        std::vector<double> complete, int64_t threads) {
    check_points(points, false);
    const kn::CompleteBox cb = complete_box(complete);  // 6 or 14 entries
    const int n = (int)points.size(0);
    TORCH_CHECK(n_queries >= 0 && n_queries <= n, "n_queries out of range");
    auto idx = torch::empty({n_queries, k}, torch::kInt32);
    auto d2 = torch::empty({n_queries, k}, torch::kFloat32);
    const float ext[8] = {cb.wide, cb.zlim, cb.dlo[0], cb.dlo[1], cb.dlo[2], cb.dhi[0], cb.dhi[1], cb.dhi[2]};
    std::vector<uint32_t> unc;
    {
        py::gil_scoped_release nogil;
        knh::grid_knn_cpu(points.data_ptr<float>(), n, (int)n_queries, (int)k, (float)ppc, cb.lo, cb.hi,
                          reinterpret_cast<uint32_t*>(idx.data_ptr<int>()), d2.data_ptr<float>(), &unc,
                          (int)threads, ext);
    }
    auto u = torch::empty({(int64_t)unc.size()}, torch::kInt32);
    for (size_t i = 0; i < unc.size(); ++i) u[i] = (int)unc[i];
    return {idx, d2, u};
}

torch::Tensor read_xyz(const std::string& path, bool normalize) {
    std::vector<float> xyz;
    std::string err;
    TORCH_CHECK(knh::read_xyz(path, xyz, normalize, &err), err);
    auto t = torch::empty({(int64_t)(xyz.size() / 3), 3}, torch::kFloat32);
    std::memcpy(t.data_ptr<float>(), xyz.data(), xyz.size() * sizeof(float));
    return t;
}

void write_xyz(const std::string& path, torch::Tensor points) {
    check_points(points, false);
    std::string err;
    TORCH_CHECK(knh::write_xyz(path, points.data_ptr<float>(), (int)points.size(0), &err), err);
}

torch::Tensor normalize_1000(torch::Tensor points) {
    check_points(points, false);
    std::vector<float> xyz(points.data_ptr<float>(), points.data_ptr<float>() + points.numel());
    knh::normalize_1000(xyz);
    auto t = torch::empty_like(points);
    std::memcpy(t.data_ptr<float>(), xyz.data(), xyz.size() * sizeof(float));
    return t;
}

}  // namespace


// ---- crash diagnostics -----------------------------------------------------------------
// A native backtrace on SIGSEGV / SIGBUS / SIGFPE / SIGILL (faulthandler prints only the Python
// frames): the frames go to stderr with backtrace_symbols_fd (async-signal-safe), then the previous
// disposition is restored and the signal re-raised, so the process still dies as it would have.
namespace crash {
struct sigaction g_prev[32];
void handler(int sig, siginfo_t* info, void*) {
    const char hdr[] = "\n[cuda_knearests_amd] fatal signal; native backtrace:\n";
    (void)!write(2, hdr, sizeof(hdr) - 1);
    char buf[64];
    const int n = std::snprintf(buf, sizeof(buf), "signal %d, fault address %p\n", sig, info ? info->si_addr : nullptr);
    if (n > 0) (void)!write(2, buf, (size_t)n);
    // innermost frames and the outermost ones (a runaway recursion fills the middle)
    static void* frames[1 << 16];
    const int nf = backtrace(frames, 1 << 16);
    if (nf <= 64) {
        backtrace_symbols_fd(frames, nf, 2);
    } else {
        backtrace_symbols_fd(frames, 8, 2);
        const int m = std::snprintf(buf, sizeof(buf), "... %d frames ...\n", nf - 48);
        if (m > 0) (void)!write(2, buf, (size_t)m);
        backtrace_symbols_fd(frames + nf - 40, 40, 2);
    }
    sigaction(sig, &g_prev[sig], nullptr);
    raise(sig);
}
bool install() {
    static bool done = false;
    if (done) return true;
    void* warm[2];
    (void)backtrace(warm, 2);  // loads libgcc's unwinder now, not inside the handler
    // an alternate signal stack for the calling (main) thread: a fault from unbounded recursion
    // (the HIP / RCCL capture crashes of round 5) leaves no stack for the handler otherwise
    static std::vector<char> alt(1 << 18);
    stack_t ss;
    std::memset(&ss, 0, sizeof(ss));
    ss.ss_sp = alt.data();
    ss.ss_size = alt.size();
    (void)sigaltstack(&ss, nullptr);
    struct sigaction sa;
    std::memset(&sa, 0, sizeof(sa));
    sa.sa_sigaction = handler;
    sa.sa_flags = SA_SIGINFO | SA_ONSTACK;
    sigemptyset(&sa.sa_mask);
    for (int sig : {SIGSEGV, SIGBUS, SIGFPE, SIGILL})
        if (sigaction(sig, &sa, &g_prev[sig]) != 0) return false;
    done = true;
    return true;
}
}  // namespace crash

// ---- one rank's pipelined distributed step over RCCL (csrc/runtime/dist.hpp) -------------
py::bytes rccl_unique_id() {
    unsigned char id[kn::kCommIdBytes];
    std::string err;
    TORCH_CHECK(kn::comm_unique_id(id, &err), err);
    return py::bytes(reinterpret_cast<const char*>(id), kn::kCommIdBytes);
}

class PyRankComm {
public:
    PyRankComm(py::bytes id, int64_t world, int64_t rank, int64_t device) {
        const std::string s = id;
        TORCH_CHECK(s.size() == (size_t)kn::kCommIdBytes, "the unique id is 128 bytes");
        std::string err;
        {
            py::gil_scoped_release nogil;  // collective: blocks until every rank joined
            c_ = kn::comm_create(reinterpret_cast<const unsigned char*>(s.data()), (int)world, (int)rank, (int)device, &err);
        }
        TORCH_CHECK(c_, err);
    }
    ~PyRankComm() { kn::comm_destroy(c_); }
    std::string async_error() { return kn::comm_async_error(c_); }
    void abort() { kn::comm_abort(c_); }
    kn::RankComm* c_ = nullptr;
};

class PyDistPipe {
public:
    // comm = None: loopback mode (tests), world / rank from `loopback` = (world, rank)
    PyDistPipe(std::shared_ptr<PyRankComm> comm, torch::Tensor points, c10::optional<torch::Tensor> ids,
               torch::Tensor plan, torch::Tensor metas, std::vector<int64_t> tot, std::vector<double> hdr,
               std::vector<int64_t> grid, std::vector<int64_t> dims, std::vector<int64_t> recv_own,
               std::vector<int64_t> recv_halo, std::vector<int64_t> cross_send, std::vector<int64_t> cross_recv,
               std::vector<int64_t> place, int64_t cap, int64_t k, double ppc, bool deterministic, int64_t exact_grid,
               int64_t use_tree, bool self_via_comm, c10::optional<std::vector<int64_t>> loopback,
               c10::optional<torch::Tensor> field, c10::optional<torch::Tensor> field_cert)
        : comm_(std::move(comm)), points_(points) {
        check_points(points, true);
        TORCH_CHECK(plan.is_cuda() && plan.numel() == (int64_t)sizeof(kn::RouteParams), "plan must be a route plan");
        TORCH_CHECK(metas.is_cuda() && metas.scalar_type() == torch::kFloat64 && metas.is_contiguous(), "metas: f64 GPU");
        TORCH_CHECK(grid.size() == 3 && dims.size() == 3 && place.size() == 5, "grid / dims / place sizes");
        kn::DistPlan p;
        if (comm_) {
            p.world = comm_->c_->world;
            p.rank = comm_->c_->rank;
        } else {
            TORCH_CHECK(loopback.has_value() && loopback->size() == 2, "no communicator: loopback = (world, rank)");
            p.world = (int)(*loopback)[0];
            p.rank = (int)(*loopback)[1];
        }
        comm_world_ = p.world;
        p.device = points.get_device();
        p.k = (int)k;
        p.n = (int)points.size(0);
        p.points = points.data_ptr<float>();
        if (ids.has_value()) {
            TORCH_CHECK(ids->is_cuda() && ids->scalar_type() == torch::kInt32 && ids->numel() == points.size(0) &&
                            ids->is_contiguous(), "ids: contiguous int32 GPU tensor of N entries");
            ids_ = *ids;
            p.ids = ids_.data_ptr<int>();
        }
        plan_ = plan;
        metas_ = metas;
        p.route = plan.data_ptr();
        TORCH_CHECK(metas.numel() == 8 * (int64_t)p.world, "metas: world x 8");
        p.metas = metas.data_ptr<double>();
        p.hdr = hdr;
        for (auto v : tot) p.tot.push_back((int)v);
        for (int a = 0; a < 3; ++a) { p.grid[a] = (int)grid[a]; p.dims[a] = (int)dims[a]; }
        for (auto v : recv_own) p.recv_own.push_back((int)v);
        for (auto v : recv_halo) p.recv_halo.push_back((int)v);
        for (auto v : cross_send) p.cross_send.push_back((int)v);
        for (auto v : cross_recv) p.cross_recv.push_back((int)v);
        for (int i = 0; i < 5; ++i) p.place[i] = (int)place[i];
        p.cap = (int)cap;
        p.ppc = (float)ppc;
        p.deterministic = deterministic ? 1 : 0;
        p.exact_grid = (int)exact_grid;
        p.use_tree = (int)use_tree;
        p.self_via_comm = self_via_comm ? 1 : 0;
        // halo field plan: the route plan points at the width field, the complete box at the
        // certified radii; both stay alive with the pipeline
        TORCH_CHECK(field.has_value() == field_cert.has_value(), "field and field_cert go together");
        if (field.has_value()) {
            const auto fc = field_arg(field_cert);
            TORCH_CHECK(field_arg(field).second == fc.second, "field / field_cert sizes differ");
            field_ = *field;
            field_cert_ = *field_cert;
            p.cert_field = fc.first;
            p.field_g = fc.second;
        }
        const c10::DeviceGuard guard(points.device());
        // the plan tensors (route plan, metas) are copied by the constructor: their producers first
        KN_CHECK_HIP(hipStreamSynchronize(c10::hip::getCurrentHIPStreamMasqueradingAsCUDA().stream()));
        d_ = std::make_shared<kn::DistPipeline>(p, comm_ ? comm_->c_ : nullptr);
        TORCH_CHECK(d_->ok(), d_->error());
    }
    // one eager step, collective (every rank calls it after all constructed their pipelines);
    // waits under the deadline with the GIL released
    void warmup(double timeout_s) {
        kn_status st;
        {
            py::gil_scoped_release nogil;
            st = d_->warmup(timeout_s);
        }
        TORCH_CHECK(st == KN_OK, d_->error());
    }
    // capture the step's graphs now (nothing runs); False: capture failed, the pipeline is eager
    bool prepare_graphs(int64_t unroll) {
        const c10::DeviceGuard guard(points_.device());
        return d_->prepare_graphs((int)unroll) == KN_OK;
    }
    void set_eager(bool eager) { d_->set_eager(eager); }
    // new input tensors for the following steps (same n, same ids presence); keeps them alive
    void rebind(torch::Tensor points, c10::optional<torch::Tensor> ids) {
        check_points(points, true);
        TORCH_CHECK(points.get_device() == points_.get_device(), "rebind: same device");
        const int* ip = nullptr;
        if (ids.has_value()) {
            TORCH_CHECK(ids->is_cuda() && ids->scalar_type() == torch::kInt32 && ids->numel() == points.size(0) &&
                            ids->is_contiguous(), "ids: contiguous int32 GPU tensor of N entries");
            ip = ids->data_ptr<int>();
        }
        const c10::DeviceGuard guard(points.device());
        TORCH_CHECK(d_->rebind(points.data_ptr<float>(), ip, (int)points.size(0)) == KN_OK, d_->error());
        points_ = points;
        ids_ = ids.has_value() ? *ids : torch::Tensor();
    }
    std::string mode() { return d_->eager() ? "eager" : "graph"; }
    int64_t capture_fallbacks() { return d_->capture_fallbacks(); }
    std::string error() { return d_->error(); }
    // loopback mode: one synchronous stage (0 route, 1 unpack + build + query + local flag)
    void loopback_stage(int64_t stage) { TORCH_CHECK(d_->loopback_stage((int)stage) == KN_OK, d_->error()); }
    // views (float32, (rows, 4)) of set 0's send rows for destination d / receive rows from source s.
    // Like outputs(), each view's deleter holds the pipeline, so the buffers outlive the views
    torch::Tensor send_view(int64_t d, int64_t rows) {
        TORCH_CHECK(d >= 0 && d < comm_world_ && rows >= 0, "send_view: destination out of range");
        return owned_view(d_->send_rows(0) + d_->send_offset((int)d), rows);
    }
    torch::Tensor recv_view(int64_t src, int64_t rows) {
        TORCH_CHECK(src >= 0 && src < comm_world_ && rows >= 0, "recv_view: source out of range");
        return owned_view(d_->recv_rows(0) + d_->recv_offset((int)src), rows);
    }
    torch::Tensor owned_view(float4* base, int64_t rows) {
        auto opt = torch::TensorOptions().device(points_.device()).dtype(torch::kFloat32);
        std::shared_ptr<kn::DistPipeline> keep = d_;
        std::shared_ptr<PyRankComm> keepc = comm_;
        return torch::from_blob(reinterpret_cast<float*>(base), {rows, 4}, [keep, keepc](void*) {}, opt);
    }
    int64_t flag_local() { return d_->flag_local(0); }
    // diagnostics (loopback mode): set 0's query counters and routed column totals
    std::vector<int64_t> debug_words(int64_t set) {
        TORCH_CHECK(set == 0 || set == 1, "set must be 0 or 1");
        KN_CHECK_HIP(hipDeviceSynchronize());
        std::vector<unsigned> c(kn::kNumCounters);
        const int W = (int)comm_world_;
        std::vector<int> t((size_t)2 * W);
        KN_CHECK_HIP(hipMemcpy(c.data(), d_->counters((int)set), c.size() * sizeof(unsigned), hipMemcpyDeviceToHost));
        KN_CHECK_HIP(hipMemcpy(t.data(), d_->totals((int)set), t.size() * sizeof(int), hipMemcpyDeviceToHost));
        std::vector<int64_t> out(c.begin(), c.end());
        out.insert(out.end(), t.begin(), t.end());
        return out;
    }
    // enqueue `iters` steps (unroll: steps per graph launch, even >= 2, else one graph per stage)
    // keep_primed: also enqueue the next step's build (the caller promises the points stay
    // unchanged until the next launch); the current torch stream orders the input
    int64_t launch(int64_t iters, int64_t unroll, bool keep_primed) {
        long long last = -1;
        const c10::DeviceGuard guard(points_.device());
        const hipStream_t caller = c10::hip::getCurrentHIPStreamMasqueradingAsCUDA().stream();
        kn_status st;
        {
            // eager mode enqueues RCCL calls: never hold the GIL across them
            py::gil_scoped_release nogil;
            st = d_->launch((int)iters, (int)unroll, keep_primed, caller, &last);
        }
        TORCH_CHECK(st == KN_OK, d_->error());
        return last;
    }
    // wait for step `step` (polls RCCL errors; deadline) -> sticky flag (0 = all steps valid)
    int64_t wait(int64_t step, double timeout_s) {
        int flag = -1;
        kn_status st;
        {
            py::gil_scoped_release nogil;
            st = d_->wait(step, timeout_s, &flag);
        }
        TORCH_CHECK(st == KN_OK, d_->error());
        return flag;
    }
    void sync() { TORCH_CHECK(d_->sync() == KN_OK, d_->error()); }
    int64_t last_set() { return d_->last_set(); }
    int64_t sets() { return d_->sets(); }
    // (owned global ids, idx, d2) of grid set s: views of the pipeline's buffers, overwritten by
    // the step after next. Each view holds a reference to the pipeline (its deleter), so the
    // buffers outlive every tensor that views them, whatever the Python side drops
    std::vector<torch::Tensor> outputs(int64_t s) {
        TORCH_CHECK(s >= 0 && s < d_->sets(), "set out of range");
        auto opt = torch::TensorOptions().device(points_.device());
        const int64_t no = d_->n_owned(), k = d_->k();
        std::shared_ptr<kn::DistPipeline> keep = d_;
        std::shared_ptr<PyRankComm> keepc = comm_;
        auto owner = [keep, keepc](void*) {};
        auto g = torch::from_blob(const_cast<int*>(d_->gids((int)s)), {no}, owner, opt.dtype(torch::kInt32));
        auto i = torch::from_blob(const_cast<int*>(d_->idx((int)s)), {no, k}, owner, opt.dtype(torch::kInt32));
        auto d = torch::from_blob(const_cast<float*>(d_->d2((int)s)), {no, k}, owner, opt.dtype(torch::kFloat32));
        return {g, i, d};
    }
    std::vector<int64_t> counters(int64_t s) {
        TORCH_CHECK(s >= 0 && s < d_->sets(), "set out of range");
        TORCH_CHECK(d_->sync() == KN_OK, d_->error());
        unsigned c[kn::kNumCounters];
        KN_CHECK_HIP(hipMemcpy(c, d_->counters((int)s), sizeof(c), hipMemcpyDeviceToHost));
        return std::vector<int64_t>(c, c + kn::kNumCounters);
    }
    py::dict profile() {
        float ms[5] = {0, 0, 0, 0, 0};
        TORCH_CHECK(d_->profile(ms) == KN_OK, d_->error());
        py::dict r;
        r["ms_route"] = ms[0];
        r["ms_exchange"] = ms[1];
        r["ms_build"] = ms[2];
        r["ms_query"] = ms[3];
        r["ms_finish"] = ms[4];  // exact finish + flag + its all-reduce
        return r;
    }
    int64_t rows() { return d_->rows(); }
    int64_t n_owned() { return d_->n_owned(); }

private:
    std::shared_ptr<PyRankComm> comm_;
    torch::Tensor points_, ids_, plan_, metas_, field_, field_cert_;
    int64_t comm_world_ = 1;
    std::shared_ptr<kn::DistPipeline> d_;
};

PYBIND11_MODULE(TORCH_EXTENSION_NAME, m) {
    m.doc() = "MI355X-native k-nearest-neighbour kernels (gfx950 HIP) and CPU oracles";
    m.def("build", &build, "bin points into the grid (GPU)", py::arg("points"), py::arg("dims"),
          py::arg("deterministic") = true, py::arg("box") = py::none());
    m.def("query", &query, "k-nearest-neighbour queries on a built grid (GPU)", py::arg("sorted"),
          py::arg("cell_start"), py::arg("geom"), py::arg("dims"), py::arg("k"), py::arg("n_queries"),
          py::arg("id_map"), py::arg("complete"), py::arg("tile"), py::arg("halo"), py::arg("lds_capacity"),
          py::arg("use_tiles"), py::arg("with_dist"), py::arg("flags") = 0, py::arg("row_of") = py::none(),
          py::arg("exact_grid") = 0, py::arg("zeroed_counters") = py::none(), py::arg("q_lo") = 0,
          py::arg("xsub") = 1);
    m.def("auto_params", &auto_params, "grid / tile plan", py::arg("n"), py::arg("k"), py::arg("ppc"),
          py::arg("tile"), py::arg("halo"), py::arg("extent") = py::none(), py::arg("xsub") = 0);
    m.def(
        "query_lds_bytes",
        [](std::vector<int64_t> tile, int64_t halo, int64_t cap, int64_t xsub) {
            TORCH_CHECK(tile.size() == 3, "tile must have 3 entries");
            const int t[3] = {(int)tile[0], (int)tile[1], (int)tile[2]};
            return (int64_t)kn::query_lds_bytes(t, (int)halo, (int)cap, (int)xsub);
        },
        "LDS bytes per workgroup of the tile query kernel for a plan", py::arg("tile"), py::arg("halo"),
        py::arg("cap"), py::arg("xsub") = 1);
    m.def("to_stored_space", &to_stored_space, "original-space result -> reference stored-space view");
    m.def(
        "tree_supports",
        [](std::vector<int64_t> dims) {
            TORCH_CHECK(dims.size() == 3, "dims = [X, Y, Z]");
            const int d[3] = {(int)dims[0], (int)dims[1], (int)dims[2]};
            return py::make_tuple(kn::tree_supports(d), (int64_t)kn::tree_brick_slots(d));
        },
        "whether the tree path takes a grid of these dims: (supported, padded brick slots)", py::arg("dims"));
    m.def("tree_build", &tree_build,
          "Morton-leaf tree over a grid's sorted points, stream-ordered: (workspace, nodes, leaves or -1)",
          py::arg("sorted"), py::arg("cell_start"), py::arg("geom"), py::arg("dims"), py::arg("count_leaves") = false);
    m.def("tree_query", &tree_query, "kNN through a tree_build result: (idx, d2, counters)", py::arg("ws"),
          py::arg("nodes"), py::arg("dims"), py::arg("n"), py::arg("k"), py::arg("n_queries"), py::arg("id_map") = py::none(),
          py::arg("with_dist") = true, py::arg("flags") = 0, py::arg("row_of") = py::none());
    m.def("cell_sort", &cell_sort, "in-cell order by original index (deterministic layout) of a built grid");
    m.def("occupancy", &occupancy, "sum over cells of count^2 (occupancy-adaptive grid)");
    m.def("refine_dims", &refine_dims, "finer grid dims for an over-occupied grid, or None", py::arg("dims"),
          py::arg("w"), py::arg("k"), py::arg("ppc"), py::arg("n"), py::arg("xsub") = 1);
    m.def("local_meta", &local_meta, "multi-GPU: {lo[3], hi[3], n, 0} of the local points (float64, on device)");
    m.def("route_count", &route_count, "multi-GPU routing: per-destination (owned, halo) row counts",
          py::arg("points"), py::arg("lo"), py::arg("hi"), py::arg("grid"), py::arg("boxes"), py::arg("h"),
          py::arg("splits") = py::none(), py::arg("h_inner") = -1.0, py::arg("wz") = INFINITY);
    m.def("route_plan", &route_plan, "multi-GPU: device-side routing plan from the gathered metas (no host sync)",
          py::arg("metas"), py::arg("rank"), py::arg("grid"), py::arg("k"), py::arg("halo_factor"),
          py::arg("splits") = py::none(), py::arg("inner_factor") = 0.0, py::arg("field") = py::none());
    m.def("field_splat", &field_splat,
          "multi-GPU halo field: splat the owned queries' K-th distances into a G^3 width field (in place)",
          py::arg("pts"), py::arg("n_owned"), py::arg("d2"), py::arg("k"), py::arg("hdr"), py::arg("rank"),
          py::arg("grid"), py::arg("field"));
    m.def("field_cert", &field_cert, "multi-GPU halo field: certified radius of every field cell",
          py::arg("field"), py::arg("hdr"));
    m.def("inner_halo_factor", &kn::inner_halo_factor,
          "multi-GPU: interior halo width in expected (K+1)-point radii (Poisson tail <= 1e-12)", py::arg("k"));
    m.def("route_count_dev", &route_count_dev, "multi-GPU: route_count with the device plan");
    m.def("route_scatter_dev", &route_scatter_dev, "multi-GPU: route_scatter with the device plan (ids=None: offset + i)",
          py::arg("points"), py::arg("ids"), py::arg("plan"), py::arg("world"), py::arg("block_offsets"),
          py::arg("totals"), py::arg("rows"), py::arg("self_last") = -1);
    m.def("route_begin", &route_begin,
          "multi-GPU: plan + counts + scatter (self-last layout, cap rows) enqueued in one call",
          py::arg("points"), py::arg("ids"), py::arg("metas"), py::arg("rank"), py::arg("grid"), py::arg("k"),
          py::arg("halo_factor"), py::arg("cap"), py::arg("splits") = py::none(), py::arg("inner_factor") = 0.0,
          py::arg("field") = py::none());
    m.def("query_external", &query_external,
          "multi-GPU query forwarding: exact K nearest of external points among a local grid");
    m.def("steady_flag", &steady_flag, "multi-GPU: on-device check of a sync-free steady-state step");
    m.def("fwd_pack", &fwd_pack, "multi-GPU: uncertified queries into fixed forwarding slots (no host sync)");
    m.def("fwd_answer", &fwd_answer, "multi-GPU: answers to received forwarding slots from the local grid");
    m.def("fwd_merge", &fwd_merge, "multi-GPU: merge forwarded answers into the rows, in place");
    m.def("route_steady", &route_steady,
          "multi-GPU steady step: counts + scatter with a validated plan, share bbox partials on the way",
          py::arg("points"), py::arg("ids"), py::arg("plan"), py::arg("world"), py::arg("cap"), py::arg("rank"),
          py::arg("place") = py::none());
    m.def("steady_flag_local", &steady_flag_local,
          "multi-GPU world 1: steady check from one bbox pass (+ optional sticky / pinned host flag)",
          py::arg("points"), py::arg("metas"), py::arg("rank"), py::arg("counters"), py::arg("sticky") = py::none(),
          py::arg("host") = py::none());
    m.def("steady_flag_partials", &steady_flag_partials,
          "multi-GPU: steady-step check with the share bbox from route_steady's partials");
    m.def("dist_local", &dist_local,
          "multi-GPU: unpack + local grid build + owned-point queries from the plan header, one call",
          py::arg("recv"), py::arg("self_rows"), py::arg("recv_own"), py::arg("recv_halo"), py::arg("rank"),
          py::arg("grid"), py::arg("hdr"), py::arg("k"), py::arg("ppc"), py::arg("deterministic"),
          py::arg("exact_grid") = 0, py::arg("adaptive") = false, py::arg("dims_hint") = py::none(),
          py::arg("pre_pts") = py::none(), py::arg("pre_gids") = py::none(), py::arg("use_tree") = -1,
          py::arg("field_cert") = py::none());
    m.def("route_unpack_split", &route_unpack_split,
          "multi-GPU: unpack other sources' rows + this rank's own segment (self-last layout)");
    m.def("route_scatter", &route_scatter, "multi-GPU routing: build the all-to-all send buffer",
          py::arg("points"), py::arg("ids"), py::arg("lo"), py::arg("hi"), py::arg("grid"), py::arg("boxes"),
          py::arg("h"), py::arg("block_offsets"), py::arg("totals"), py::arg("rows"), py::arg("splits") = py::none(),
          py::arg("h_inner") = -1.0, py::arg("wz") = INFINITY);
    m.def("route_unpack", &route_unpack, "multi-GPU routing: received rows -> owned-first points + global ids");
    m.def("install_crash_handler", &crash::install,
          "print a native backtrace on SIGSEGV/SIGBUS/SIGFPE/SIGILL, then die as before");
    m.def("rccl_unique_id", &rccl_unique_id, "multi-GPU: a new RCCL unique id (128 bytes) for RankComm");
    py::class_<PyRankComm, std::shared_ptr<PyRankComm>>(m, "RankComm", "one rank's RCCL communicator (collective init)",
                                                          py::module_local())
        .def(py::init<py::bytes, int64_t, int64_t, int64_t>(), py::arg("uid"), py::arg("world"), py::arg("rank"),
             py::arg("device"))
        .def("async_error", &PyRankComm::async_error)
        .def("abort", &PyRankComm::abort);
    py::class_<PyDistPipe>(m, "DistPipe", "one rank's pipelined distributed step (route + RCCL exchange + build | "
                                          "query | flag all-reduce), hipGraph-replayed",
                          py::module_local())
        .def(py::init<std::shared_ptr<PyRankComm>, torch::Tensor, c10::optional<torch::Tensor>, torch::Tensor,
                      torch::Tensor, std::vector<int64_t>, std::vector<double>, std::vector<int64_t>,
                      std::vector<int64_t>, std::vector<int64_t>, std::vector<int64_t>, std::vector<int64_t>,
                      std::vector<int64_t>, std::vector<int64_t>, int64_t, int64_t, double, bool, int64_t, int64_t,
                      bool, c10::optional<std::vector<int64_t>>, c10::optional<torch::Tensor>,
                      c10::optional<torch::Tensor>>(),
             py::arg("comm"), py::arg("points"), py::arg("ids"), py::arg("plan"), py::arg("metas"), py::arg("tot"),
             py::arg("hdr"), py::arg("grid"), py::arg("dims"), py::arg("recv_own"), py::arg("recv_halo"),
             py::arg("cross_send"), py::arg("cross_recv"), py::arg("place"), py::arg("cap"), py::arg("k"),
             py::arg("ppc"), py::arg("deterministic"), py::arg("exact_grid"), py::arg("use_tree"),
             py::arg("self_via_comm"), py::arg("loopback") = py::none(), py::arg("field") = py::none(),
             py::arg("field_cert") = py::none())
        .def("loopback_stage", &PyDistPipe::loopback_stage)
        .def("send_view", &PyDistPipe::send_view)
        .def("recv_view", &PyDistPipe::recv_view)
        .def("flag_local", &PyDistPipe::flag_local)
        .def("debug_words", &PyDistPipe::debug_words, py::arg("set") = 0)
        .def("warmup", &PyDistPipe::warmup, py::arg("timeout_s") = 300.0)
        .def("prepare_graphs", &PyDistPipe::prepare_graphs, py::arg("unroll"))
        .def("set_eager", &PyDistPipe::set_eager)
        .def("rebind", &PyDistPipe::rebind, py::arg("points"), py::arg("ids") = py::none())
        .def("mode", &PyDistPipe::mode)
        .def("capture_fallbacks", &PyDistPipe::capture_fallbacks)
        .def("error", &PyDistPipe::error)
        .def("launch", &PyDistPipe::launch, py::arg("iters") = 1, py::arg("unroll") = 0, py::arg("keep_primed") = false)
        .def("wait", &PyDistPipe::wait, py::arg("step"), py::arg("timeout_s") = 300.0)
        .def("sync", &PyDistPipe::sync)
        .def("last_set", &PyDistPipe::last_set)
        .def("sets", &PyDistPipe::sets)
        .def("outputs", &PyDistPipe::outputs)
        .def("counters", &PyDistPipe::counters)
        .def("profile", &PyDistPipe::profile)
        .def("rows", &PyDistPipe::rows)
        .def("n_owned", &PyDistPipe::n_owned);
    py::class_<PyEngine>(m, "Engine", "native single-GPU engine (own arena/stream, hipGraph replay)",
                        py::module_local())
        .def(py::init<int64_t, double, std::vector<int64_t>, int64_t, bool, bool, bool, int64_t, bool, int64_t>(),
             py::arg("k") = 16, py::arg("points_per_cell") = 0.0, py::arg("tile") = std::vector<int64_t>{},
             py::arg("halo") = 0, py::arg("deterministic") = true, py::arg("use_tiles") = true,
             py::arg("with_dist") = true, py::arg("device") = 0, py::arg("adaptive") = true,
             py::arg("algo") = 0)
        .def("prepare", &PyEngine::prepare)
        .def("prepare_async", &PyEngine::prepare_async)
        .def("solve", &PyEngine::solve)
        .def("set_k", &PyEngine::set_k)
        .def("launch_graph", &PyEngine::launch_graph, py::arg("iters") = 1)
        .def("launch_pipelined", &PyEngine::launch_pipelined, py::arg("iters") = 1, py::arg("unroll") = -1)
        .def("stream_step", &PyEngine::stream_step, py::arg("points"), py::arg("next") = py::none())
        .def("stream_batch", &PyEngine::stream_batch, py::arg("points"), py::arg("idx"), py::arg("d2") = py::none(),
             py::arg("mode") = py::none())
        .def("set_pipeline_shape", &PyEngine::set_pipeline_shape, py::arg("query_streams") = -1, py::arg("sets") = -1)
        .def("get_permutation", &PyEngine::permutation)
        .def("sync", &PyEngine::sync)
        .def("results", &PyEngine::results)
        .def("solve_range", &PyEngine::solve_range, py::arg("first"), py::arg("count"), py::arg("device"))
        .def("counters", &PyEngine::counters)
        .def("info", &PyEngine::info);
    m.def("debug_phase_cycles", &debug_phase_cycles, "KN_PHASES builds: query-kernel wave cycles per phase",
          py::arg("reset") = false);
    m.def("debug_words", &debug_words, "checked builds: first OOB report {code, index, limit, hi} of build and query kernels",
          py::arg("reset") = false);
#if defined(KN_CHECKED) && KN_CHECKED
    m.attr("CHECKED") = true;
#else
    m.attr("CHECKED") = false;
#endif
    m.def("kdtree_knn", &kdtree_knn, "CPU kd-tree oracle", py::arg("points"), py::arg("k"), py::arg("threads") = 0);
    m.def("brute_knn", &brute_knn, "CPU brute-force oracle", py::arg("points"), py::arg("k"), py::arg("threads") = 0);
    m.def("grid_knn_cpu", &grid_knn_cpu, "CPU grid kNN (engine algorithm on the host)");
    m.def("read_xyz", &read_xyz, "read a .xyz file", py::arg("path"), py::arg("normalize") = false);
    m.def("write_xyz", &write_xyz, "write a .xyz file");
    m.def("normalize_1000", &normalize_1000, "map a cloud into [0,1000]^3 (reference normalisation)");
    m.attr("SENTINEL") = py::int_(-1);
    m.attr("MAX_K") = py::int_(128);
}
