// host.cpp -- CPU oracles, CPU grid kNN and .xyz I/O. See host.hpp.
// Parity map (reference, read for behaviour only):
//   kd-tree oracle      <- kd_tree.cpp:80-300 / kd_tree.h:64-207 (set_points, split, recursive query)
//   .xyz loader + [0,1000]^3 normalisation <- test_knearests.cu:15-81 (get_bbox, load_file)
//   result check vs oracle <- test_knearests.cu:117-236 (main's comparison loop)
#include "host.hpp"

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <fstream>
#include <limits>
#include <sstream>

#ifdef _OPENMP
#include <omp.h>
#endif

namespace knh {

namespace {

constexpr uint32_t SENT = 0xFFFFFFFFu;

inline bool pair_less(float da, uint32_t ia, float db, uint32_t ib) {
    return da < db || (da == db && ia < ib);
}

// Fixed-capacity sorted list of (d2, idx), ascending, ties by index.
struct TopK {
    int k;
    float* d;
    uint32_t* i;
    void init(int kk, float* dd, uint32_t* ii) {
        k = kk; d = dd; i = ii;
        for (int j = 0; j < k; ++j) { d[j] = std::numeric_limits<float>::infinity(); i[j] = SENT; }
    }
    float worst() const { return d[k - 1]; }
    void push(float dd, uint32_t ii) {
        if (!pair_less(dd, ii, d[k - 1], i[k - 1])) return;
        int j = k - 1;
        while (j > 0 && pair_less(dd, ii, d[j - 1], i[j - 1])) { d[j] = d[j - 1]; i[j] = i[j - 1]; --j; }
        d[j] = dd; i[j] = ii;
    }
};

inline float dist2(const float* a, const float* b) {
    const float dx = b[0] - a[0], dy = b[1] - a[1], dz = b[2] - a[2];
    return std::fma(dz, dz, std::fma(dy, dy, dx * dx));
}

int nthreads(int t) {
#ifdef _OPENMP
    return t > 0 ? t : omp_get_max_threads();
#else
    (void)t;
    return 1;
#endif
}

}  // namespace

// ------------------------------------------------------------------ kd-tree oracle ----
void KdTree::build(const float* pts, int n) {
    n_ = n;
    p_.assign(pts, pts + (size_t)n * 3);
    order_.resize(n);
    for (int i = 0; i < n; ++i) order_[i] = i;
    nodes_.clear();
    nodes_.reserve(n > 0 ? 2 * (n / kLeaf + 1) : 1);
    if (n > 0) build_rec(0, n);
}

int KdTree::build_rec(int begin, int end) {
    Node nd;
    for (int a = 0; a < 3; ++a) { nd.lo[a] = std::numeric_limits<float>::infinity(); nd.hi[a] = -nd.lo[a]; }
    for (int t = begin; t < end; ++t) {
        const float* q = &p_[3 * (size_t)order_[t]];
        for (int a = 0; a < 3; ++a) { nd.lo[a] = std::min(nd.lo[a], q[a]); nd.hi[a] = std::max(nd.hi[a], q[a]); }
    }
    nd.begin = begin; nd.end = end; nd.left = nd.right = -1;
    const int id = (int)nodes_.size();
    nodes_.push_back(nd);
    if (end - begin <= kLeaf) return id;
    int axis = 0;
    for (int a = 1; a < 3; ++a)
        if (nd.hi[a] - nd.lo[a] > nd.hi[axis] - nd.lo[axis]) axis = a;
    const int mid = begin + (end - begin) / 2;
    std::nth_element(order_.begin() + begin, order_.begin() + mid, order_.begin() + end,
                     [&](int x, int y) { return p_[3 * (size_t)x + axis] < p_[3 * (size_t)y + axis]; });
    const int l = build_rec(begin, mid);
    const int r = build_rec(mid, end);
    nodes_[id].left = l;
    nodes_[id].right = r;
    return id;
}

void KdTree::query(const float q[3], int k, int exclude, uint32_t* idx, float* d2) const {
    TopK top;
    top.init(k, d2, idx);
    if (n_ == 0) return;
    struct Item { int node; float bd; };
    Item stack[128];
    int sp = 0;
    stack[sp++] = {0, 0.f};
    while (sp) {
        const Item it = stack[--sp];
        if (it.bd > top.worst()) continue;
        const Node& nd = nodes_[it.node];
        if (nd.left < 0) {
            for (int t = nd.begin; t < nd.end; ++t) {
                const int j = order_[t];
                if (j == exclude) continue;
                top.push(dist2(q, &p_[3 * (size_t)j]), (uint32_t)j);
            }
            continue;
        }
        float bd[2];
        const int ch[2] = {nd.left, nd.right};
        for (int c = 0; c < 2; ++c) {
            const Node& cn = nodes_[ch[c]];
            float s = 0.f;
            for (int a = 0; a < 3; ++a) {
                const float e = std::max(0.f, std::max(cn.lo[a] - q[a], q[a] - cn.hi[a]));
                s += e * e;
            }
            bd[c] = s;
        }
        // push the far child first so the near child is visited first
        const int nearc = bd[0] <= bd[1] ? 0 : 1;
        stack[sp++] = {ch[1 - nearc], bd[1 - nearc]};
        stack[sp++] = {ch[nearc], bd[nearc]};
    }
}

void kdtree_knn_all(const float* pts, int n, int k, uint32_t* idx, float* d2, int threads) {
    KdTree t;
    t.build(pts, n);
#pragma omp parallel for schedule(dynamic, 256) num_threads(nthreads(threads))
    for (int i = 0; i < n; ++i) t.query(pts + 3 * (size_t)i, k, i, idx + (size_t)i * k, d2 + (size_t)i * k);
}

void brute_knn_all(const float* pts, int n, int k, uint32_t* idx, float* d2, int threads) {
#pragma omp parallel for schedule(dynamic, 64) num_threads(nthreads(threads))
    for (int i = 0; i < n; ++i) {
        TopK top;
        top.init(k, d2 + (size_t)i * k, idx + (size_t)i * k);
        for (int j = 0; j < n; ++j)
            if (j != i) top.push(dist2(pts + 3 * (size_t)i, pts + 3 * (size_t)j), (uint32_t)j);
    }
}

// ----------------------------------------------------------------- CPU grid kNN -------
void grid_knn_cpu(const float* pts, int n, int n_queries, int k, float ppc, const float clo[3],
                  const float chi[3], uint32_t* idx, float* d2, std::vector<uint32_t>* uncert,
                  int threads, const float* cext) {
    if (n_queries <= 0) return;
    if (!(ppc > 0.f)) ppc = 3.1f;  // same default grid density as the GPU engine
    float lo[3], hi[3];
    for (int a = 0; a < 3; ++a) { lo[a] = std::numeric_limits<float>::infinity(); hi[a] = -lo[a]; }
    for (int i = 0; i < n; ++i)
        for (int a = 0; a < 3; ++a) { lo[a] = std::min(lo[a], pts[3 * (size_t)i + a]); hi[a] = std::max(hi[a], pts[3 * (size_t)i + a]); }
    if (n == 0) { for (int a = 0; a < 3; ++a) { lo[a] = 0; hi[a] = 1; } }
    const int sz = std::max(1, (int)std::lround(std::cbrt(std::max(1.0, (double)n / ppc))));
    const int D[3] = {sz, sz, sz};
    float org[3], cell[3], inv[3];
    float maxext = 0.f;
    for (int a = 0; a < 3; ++a) maxext = std::max(maxext, hi[a] - lo[a]);
    if (!(maxext > 0.f)) maxext = 1.f;
    for (int a = 0; a < 3; ++a) {
        const float ext = std::max(hi[a] - lo[a], maxext * 1e-3f);
        const float pad = ext * 1e-5f + std::fabs(lo[a]) * 1e-6f + 1e-30f;
        org[a] = lo[a] - pad;
        const float e = ext + 2.f * pad + std::fabs(hi[a]) * 1e-6f;
        cell[a] = e / D[a];
        inv[a] = D[a] / e;
    }
    const float eps = maxext * 2e-6f + 1e-30f;
    auto coord = [&](int a, float p) {
        const float f = (p - org[a]) * inv[a];
        int i = (int)std::floor(std::min(std::max(f, -1.f), (float)D[a]));
        return std::min(std::max(i, 0), D[a] - 1);
    };
    const long C = (long)D[0] * D[1] * D[2];
    std::vector<int> start(C + 1, 0), cellof(n);
    for (int i = 0; i < n; ++i) {
        const int c = coord(0, pts[3 * (size_t)i]) + D[0] * (coord(1, pts[3 * (size_t)i + 1]) + D[1] * coord(2, pts[3 * (size_t)i + 2]));
        cellof[i] = c;
        start[c + 1]++;
    }
    for (long c = 0; c < C; ++c) start[c + 1] += start[c];
    std::vector<int> fill(start.begin(), start.end() - 1), order(n);
    for (int i = 0; i < n; ++i) order[fill[cellof[i]]++] = i;  // stable: in-cell order = index order
    std::vector<float> sp((size_t)n * 3);
    for (int t = 0; t < n; ++t)
        for (int a = 0; a < 3; ++a) sp[3 * (size_t)t + a] = pts[3 * (size_t)order[t] + a];
    std::vector<char> bad(n_queries, 0);
#pragma omp parallel for schedule(dynamic, 256) num_threads(nthreads(threads))
    for (int qi = 0; qi < n_queries; ++qi) {
        const float* q = pts + 3 * (size_t)qi;
        TopK top;
        top.init(k, d2 + (size_t)qi * k, idx + (size_t)qi * k);
        const int c[3] = {coord(0, q[0]), coord(1, q[1]), coord(2, q[2])};
        const int rmax = std::max({c[0], D[0] - 1 - c[0], c[1], D[1] - 1 - c[1], c[2], D[2] - 1 - c[2]});
        bool ok = false;
        for (int r = 0; r <= rmax; ++r) {
            for (int z = std::max(0, c[2] - r); z <= std::min(D[2] - 1, c[2] + r); ++z)
                for (int y = std::max(0, c[1] - r); y <= std::min(D[1] - 1, c[1] + r); ++y) {
                    const bool shell = std::abs(z - c[2]) == r || std::abs(y - c[1]) == r;
                    const long row = ((long)z * D[1] + y) * D[0];
                    int xs[2][2];
                    int nr = 0;
                    if (shell) { xs[0][0] = std::max(0, c[0] - r); xs[0][1] = std::min(D[0] - 1, c[0] + r); nr = 1; }
                    else {
                        if (c[0] - r >= 0) { xs[nr][0] = xs[nr][1] = c[0] - r; ++nr; }
                        if (c[0] + r <= D[0] - 1) { xs[nr][0] = xs[nr][1] = c[0] + r; ++nr; }
                    }
                    for (int pr = 0; pr < nr; ++pr)
                        for (int t = start[row + xs[pr][0]]; t < start[row + xs[pr][1] + 1]; ++t) {
                            const int j = order[t];
                            if (j == qi) continue;
                            top.push(dist2(q, &sp[3 * (size_t)t]), (uint32_t)j);
                        }
                }
            float m = std::numeric_limits<float>::infinity();
            for (int a = 0; a < 3; ++a) {
                if (c[a] - r > 0) m = std::min(m, q[a] - (org[a] + (c[a] - r) * cell[a]));
                if (c[a] + r < D[a] - 1) m = std::min(m, org[a] + (c[a] + r + 1) * cell[a] - q[a]);
            }
            m -= eps;
            if (m == std::numeric_limits<float>::infinity() || (m > 0.f && top.d[k - 1] <= m * m)) { ok = true; break; }
        }
        float m = std::numeric_limits<float>::infinity();
        const float wide = cext ? cext[0] : 0.f;
        float zq = std::numeric_limits<float>::infinity();
        if (wide > 0.f)
            for (int a = 0; a < 3; ++a) zq = std::min(zq, std::min(q[a] - cext[2 + a], cext[5 + a] - q[a]));
        for (int a = 0; a < 3; ++a) {
            float lo = q[a] - clo[a], hi = chi[a] - q[a];
            if (wide > 0.f && zq + lo + wide <= cext[1]) lo += wide;
            if (wide > 0.f && zq + hi + wide <= cext[1]) hi += wide;
            m = std::min(m, std::min(lo, hi));
        }
        m -= eps;
        if (!(m == std::numeric_limits<float>::infinity() || (m > 0.f && top.d[k - 1] <= m * m))) ok = false;
        if (!ok) bad[qi] = 1;
    }
    if (uncert) {
        uncert->clear();
        for (int i = 0; i < n_queries; ++i) if (bad[i]) uncert->push_back((uint32_t)i);
    }
}

// ------------------------------------------------------------------ result checker ---
CheckResult check_knn(const float* pts, int n, int nq, int k, const uint32_t* idx, const uint32_t* oidx,
                      const float* od2) {
    CheckResult r;
    r.rows_checked = nq;
    std::string first;
    for (int i = 0; i < nq; ++i) {
        const uint32_t* row = idx + (size_t)i * k;
        const uint32_t* orow = oidx + (size_t)i * k;
        const float* drow = od2 + (size_t)i * k;
        char buf[256];
        buf[0] = 0;
        float prev = -1.f;
        for (int j = 0; j < k && !buf[0]; ++j) {
            const uint32_t v = row[j];
            if (v == SENT) {
                if (orow[j] != SENT) std::snprintf(buf, sizeof(buf), "row %d slot %d empty, oracle has %u", i, j, orow[j]);
                continue;
            }
            if (v >= (uint32_t)n) { std::snprintf(buf, sizeof(buf), "row %d slot %d id %u out of range", i, j, v); break; }
            if (v == (uint32_t)i) { std::snprintf(buf, sizeof(buf), "row %d contains itself", i); break; }
            for (int t = 0; t < j; ++t)
                if (row[t] == v) { std::snprintf(buf, sizeof(buf), "row %d duplicate id %u", i, v); break; }
            const float d = dist2(pts + 3 * (size_t)i, pts + 3 * (size_t)v);
            if (d < prev) { std::snprintf(buf, sizeof(buf), "row %d not ascending at slot %d", i, j); break; }
            prev = d;
            if (d != drow[j])
                std::snprintf(buf, sizeof(buf), "row %d slot %d: d2 %.9g (id %u) vs oracle %.9g (id %u)", i, j, d, v,
                              drow[j], orow[j]);
        }
        if (buf[0]) {
            if (r.bad_rows == 0) { r.first_bad = i; first = buf; }
            ++r.bad_rows;
        }
    }
    r.message = r.bad_rows ? first : "ok";
    return r;
}

// --------------------------------------------------------------------- .xyz I/O -------
static void bbox_inflated(const std::vector<float>& xyz, float lo[3], float hi[3]) {
    const size_t n = xyz.size() / 3;
    for (int a = 0; a < 3; ++a) { lo[a] = hi[a] = n ? xyz[a] : 0.f; }
    for (size_t i = 1; i < n; ++i)
        for (int a = 0; a < 3; ++a) { lo[a] = std::min(lo[a], xyz[3 * (size_t)i + a]); hi[a] = std::max(hi[a], xyz[3 * (size_t)i + a]); }
    const float d = 0.001f * std::max({hi[0] - lo[0], hi[1] - lo[1], hi[2] - lo[2]});
    for (int a = 0; a < 3; ++a) { lo[a] -= d; hi[a] += d; }
}

void normalize_1000(std::vector<float>& xyz) {
    if (xyz.empty()) return;
    float lo[3], hi[3];
    bbox_inflated(xyz, lo, hi);
    float side = std::max({hi[0] - lo[0], hi[1] - lo[1], hi[2] - lo[2]});
    if (!(side > 0.f)) side = 1.f;
    const size_t n = xyz.size() / 3;
#pragma omp parallel for
    for (long i = 0; i < (long)n; ++i)
        for (int a = 0; a < 3; ++a) xyz[3 * (size_t)i + a] = (float)(1000.0 * (xyz[3 * (size_t)i + a] - lo[a]) / side);
}

bool read_xyz(const std::string& path, std::vector<float>& xyz, bool normalize, std::string* err) {
    std::ifstream in(path, std::ios::binary);
    if (!in) { if (err) *err = "cannot open " + path; return false; }
    std::string data((std::istreambuf_iterator<char>(in)), std::istreambuf_iterator<char>());
    const char* p = data.c_str();
    const char* end = p + data.size();
    auto skip_ws = [&]() { while (p < end && (*p == ' ' || *p == '\t' || *p == '\r' || *p == '\n')) ++p; };
    skip_ws();
    char* q = nullptr;
    const long count = std::strtol(p, &q, 10);
    if (q == p || count < 0) { if (err) *err = "bad header in " + path; return false; }
    p = q;
    xyz.clear();
    xyz.reserve((size_t)count * 3);
    while (true) {
        skip_ws();
        if (p >= end) break;
        const float v = std::strtof(p, &q);
        if (q == p) { if (err) *err = "bad number in " + path; return false; }
        xyz.push_back(v);
        p = q;
    }
    if (xyz.size() != (size_t)count * 3) {
        if (err) *err = "point count mismatch in " + path + ": header " + std::to_string(count) +
                        ", found " + std::to_string(xyz.size() / 3.0);
        return false;
    }
    if (normalize) normalize_1000(xyz);
    return true;
}

bool write_xyz(const std::string& path, const float* xyz, int n, std::string* err) {
    FILE* f = std::fopen(path.c_str(), "w");
    if (!f) { if (err) *err = "cannot write " + path; return false; }
    std::fprintf(f, "%d\n", n);
    for (int i = 0; i < n; ++i) std::fprintf(f, "%.9g %.9g %.9g\n", xyz[3 * (size_t)i], xyz[3 * (size_t)i + 1], xyz[3 * (size_t)i + 2]);
    const bool ok = std::fclose(f) == 0;
    if (!ok && err) *err = "write failed: " + path;
    return ok;
}

}  // namespace knh

namespace knh {

namespace {
// splitmix64 -> uniform floats; deterministic across platforms
struct Rng {
    uint64_t s;
    explicit Rng(uint64_t seed) : s(seed * 0x9E3779B97F4A7C15ull + 0x632BE59BD9B4E019ull) {}
    uint64_t next() {
        uint64_t z = (s += 0x9E3779B97F4A7C15ull);
        z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
        z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
        return z ^ (z >> 31);
    }
    float uni() { return (float)((next() >> 40) * (1.0 / 16777216.0)); }  // [0,1)
    float gauss() {
        const float u = std::max(uni(), 1e-7f), v = uni();
        return std::sqrt(-2.f * std::log(u)) * std::cos(6.2831853f * v);
    }
};
}  // namespace

void gen_uniform(int n, uint64_t seed, std::vector<float>& xyz) {
    xyz.resize((size_t)n * 3);
    Rng r(seed);
    for (size_t i = 0; i < xyz.size(); ++i) xyz[i] = 1000.f * r.uni();
}

void gen_blue(int n, uint64_t seed, std::vector<float>& xyz) {
    xyz.clear();
    xyz.reserve((size_t)n * 3);
    const int m = std::max(1, (int)std::ceil(std::cbrt((double)n)));
    const float h = 1000.f / m;
    Rng r(seed);
    // visit lattice cells in a shuffled order so truncation to n points stays space-filling
    std::vector<uint32_t> cells((size_t)m * m * m);
    for (size_t c = 0; c < cells.size(); ++c) cells[c] = (uint32_t)c;
    for (size_t c = cells.size(); c > 1; --c) std::swap(cells[c - 1], cells[r.next() % c]);
    for (int t = 0; t < n; ++t) {
        const uint32_t c = cells[t];
        const int i = c % m, j = (c / m) % m, k = c / ((uint32_t)m * m);
        xyz.push_back((i + 0.5f + 0.7f * (r.uni() - 0.5f)) * h);
        xyz.push_back((j + 0.5f + 0.7f * (r.uni() - 0.5f)) * h);
        xyz.push_back((k + 0.5f + 0.7f * (r.uni() - 0.5f)) * h);
    }
}

void gen_clustered(int n, uint64_t seed, std::vector<float>& xyz) {
    xyz.resize((size_t)n * 3);
    Rng r(seed);
    const int nc = std::max(1, n / 5000);
    std::vector<float> c((size_t)nc * 4);
    for (int i = 0; i < nc; ++i) {
        for (int a = 0; a < 3; ++a) c[4 * i + a] = 100.f + 800.f * r.uni();
        c[4 * i + 3] = 5.f + 40.f * r.uni();
    }
    for (int t = 0; t < n; ++t) {
        if (t % 10 == 0) {  // 10% uniform background
            for (int a = 0; a < 3; ++a) xyz[3 * (size_t)t + a] = 1000.f * r.uni();
            continue;
        }
        const int i = (int)(r.next() % nc);
        for (int a = 0; a < 3; ++a)
            xyz[3 * (size_t)t + a] = std::min(1000.f, std::max(0.f, c[4 * i + a] + c[4 * i + 3] * r.gauss()));
    }
}

}  // namespace knh
