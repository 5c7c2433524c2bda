// bvh.cpp -- binned-SAH build of the exact-pruning sphere BVH (see bvh.h).
#include "bvh.h"

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <limits>
#include <thread>

namespace rtamd {

namespace {

struct Box {
    double lo[3] = {std::numeric_limits<double>::infinity(), std::numeric_limits<double>::infinity(),
                    std::numeric_limits<double>::infinity()};
    double hi[3] = {-std::numeric_limits<double>::infinity(), -std::numeric_limits<double>::infinity(),
                    -std::numeric_limits<double>::infinity()};
    void grow(const Box &b) {
        for (int k = 0; k < 3; ++k) { lo[k] = std::min(lo[k], b.lo[k]); hi[k] = std::max(hi[k], b.hi[k]); }
    }
    void grow(const double p[3]) {
        for (int k = 0; k < 3; ++k) { lo[k] = std::min(lo[k], p[k]); hi[k] = std::max(hi[k], p[k]); }
    }
    double area() const {
        double e[3];
        for (int k = 0; k < 3; ++k) e[k] = std::max(0.0, hi[k] - lo[k]);
        return 2.0 * (e[0] * e[1] + e[1] * e[2] + e[2] * e[0]);
    }
};

struct Prim { Box box; double c[3]; uint32_t id; double n[3] = {0, 0, 0}; };

inline float down(double x) {  // largest float <= x
    float f = (float)x;
    return ((double)f > x) ? std::nextafter(f, -std::numeric_limits<float>::infinity()) : f;
}
inline float up(double x) {  // smallest float >= x
    float f = (float)x;
    return ((double)f < x) ? std::nextafter(f, std::numeric_limits<float>::infinity()) : f;
}
inline float bits_f(uint32_t u) { float f; std::memcpy(&f, &u, 4); return f; }

// set on the threads that build per-cell trees side by side (build_triangle_cells):
// their builders run serially instead of each starting 16 more threads
thread_local bool tl_serial_build = false;

struct Builder {
    std::vector<Prim> &prims;
    uint32_t leaf_size;
    // phantom > 0: triangles.  A node's effective box is its box widened by
    // the phantom offsets 2(n^.o)n^ over its normal box (bvh.h), so the SAH
    // prices that widened box for |o| ~ phantom and may also split on the
    // normal components (axes 3-5).
    double phantom = 0;
    struct Node { Box box; uint32_t a = 0, b = 0; bool leaf = false; };
    std::vector<Node> nodes;
    uint32_t max_depth = 0;

    // SAH bins per axis (RT_AMD_SAH_BINS for sphere trees, RT_AMD_TRI_SAH_BINS
    // for triangle trees; 2 .. kMaxBins).  16 until round 5; A/B in one process
    // (profiles/round5_walk/ab_*_sah_bins.jsonl): C2 lean frame 16 / 32 / 64 /
    // 128 -> 3.754 / 3.745 / 3.712 / 3.718 ms; C5 triangle trees 16 / 32 / 64 ->
    // 148.0 / 144.2 / 144.7 ms (C5 scene load 3.1 -> 3.7 s on 8 host threads).
    // tools/sbvh_sim: a diffuse bounce's walk in RTOW 16.6 -> 15.8 node visits
    // at 64 bins, its wave's longest 29.3 -> 28.6.
    static constexpr int kMaxBins = 128;
    int bins = 16;
    // the binning scratch, reused by every node of this builder (the bins are
    // done before build() recurses): off the stack, which load_world's callers
    // may keep small (secondary threads)
    struct BinScratch { std::vector<Box> bb, nb; std::vector<uint32_t> cnt, lc; std::vector<double> left; };
    BinScratch scr;
    static int env_bins(const char *name, int def) {
        const char *e = std::getenv(name);
        const int b = e ? std::atoi(e) : def;
        return b >= 2 && b <= kMaxBins ? b : def;
    }

    Builder(std::vector<Prim> &p, uint32_t ls, double ph = 0)
        : prims(p), leaf_size(ls), phantom(ph),
          bins(ph > 0 ? env_bins("RT_AMD_TRI_SAH_BINS", 32) : env_bins("RT_AMD_SAH_BINS", 64)) {}

    // Subtrees of at least kParMin prims below depth kParDepth are built on
    // their own threads (they partition disjoint prim ranges) and spliced in
    // afterwards: the same splits as a serial build, only node numbering
    // differs (which no result depends on, bvh.h).  C5's camera tree: 263 ->
    // ~45 ms on 16 threads.
    static constexpr uint32_t kParDepth = 4, kParMin = 512;
    struct Task { uint32_t n, first, count, depth; };
    std::vector<Task> deferred;
    bool defer = false;

    void build_root(uint32_t count) {
        nodes.reserve((size_t)count * 2);
        nodes.emplace_back();
        unsigned hw = std::thread::hardware_concurrency();
        const unsigned threads = tl_serial_build ? 1u : std::min(16u, std::max(1u, hw));
        defer = threads > 1 && count >= 4 * kParMin;
        build(0, 0, count, 0);
        defer = false;
        if (deferred.empty()) return;
        std::vector<Builder> sub(deferred.size(), Builder(prims, leaf_size, phantom));
        std::atomic<size_t> next{0};
        auto work = [&]() {
            for (size_t t; (t = next.fetch_add(1)) < deferred.size();) {
                const Task &k = deferred[t];
                sub[t].nodes.reserve((size_t)k.count * 2);
                sub[t].nodes.emplace_back();
                sub[t].build(0, k.first, k.count, k.depth);
            }
        };
        std::vector<std::thread> pool;
        for (unsigned i = 1; i < std::min<size_t>(threads, deferred.size()); ++i) pool.emplace_back(work);
        work();
        for (auto &t : pool) t.join();
        for (size_t t = 0; t < deferred.size(); ++t) {
            // local node 0 becomes the placeholder n, local i > 0 lands at base + i - 1
            const uint32_t base = (uint32_t)nodes.size();
            auto remap = [&](Node nd) {
                if (!nd.leaf) nd.a = base + nd.a - 1;  // children are never a local root
                return nd;
            };
            nodes[deferred[t].n] = remap(sub[t].nodes[0]);
            for (size_t i = 1; i < sub[t].nodes.size(); ++i) nodes.push_back(remap(sub[t].nodes[i]));
            max_depth = std::max(max_depth, sub[t].max_depth);
        }
        deferred.clear();
    }

    double cost_area(const Box &g, const Box &n) const {
        if (phantom <= 0) return g.area();
        double dn[3], sum = 0, e[3];
        for (int k = 0; k < 3; ++k) { dn[k] = std::max(0.0, n.hi[k] - n.lo[k]); sum += dn[k]; }
        for (int k = 0; k < 3; ++k) {
            const double mid = std::fabs(n.hi[k] + n.lo[k]) / 2;
            e[k] = std::max(0.0, g.hi[k] - g.lo[k]) + 2 * phantom * (dn[k] + mid * sum);
        }
        return 2.0 * (e[0] * e[1] + e[1] * e[2] + e[2] * e[0]);
    }
    static double key(const Prim &p, int ax) { return ax < 3 ? p.c[ax] : p.n[ax - 3]; }

    void make_leaf(uint32_t n, uint32_t first, uint32_t count) {
        nodes[n].leaf = true;
        nodes[n].a = first;
        nodes[n].b = count;
    }

    // Builds node n over prims[first, first + count).
    void build(uint32_t n, uint32_t first, uint32_t count, uint32_t depth) {
        if (defer && depth == kParDepth && count >= kParMin) {
            deferred.push_back({n, first, count, depth});
            return;
        }
        max_depth = std::max(max_depth, depth);
        Box box, cbox, nbox;
        for (uint32_t i = first; i < first + count; ++i) {
            box.grow(prims[i].box);
            cbox.grow(prims[i].c);
            nbox.grow(prims[i].n);
        }
        nodes[n].box = box;
        if (count <= leaf_size) { make_leaf(n, first, count); return; }
        // binned SAH over the centroid box (and the normal box for triangles)
        const int kBins = bins;
        double best_cost = std::numeric_limits<double>::infinity();
        int best_axis = -1, best_split = 0;
        double best_lo = 0, best_ext = 1;
        const int naxes = phantom > 0 ? 6 : 3;
        for (int ax = 0; ax < naxes; ++ax) {
            const double lo = ax < 3 ? cbox.lo[ax] : nbox.lo[ax - 3];
            const double ext = (ax < 3 ? cbox.hi[ax] : nbox.hi[ax - 3]) - lo;
            if (!(ext > 0)) continue;
            scr.bb.assign(kBins, Box());
            scr.nb.assign(kBins, Box());
            scr.cnt.assign(kBins, 0u);
            scr.left.resize(kBins);
            scr.lc.resize(kBins);
            Box *bb = scr.bb.data(), *nb = scr.nb.data();
            uint32_t *cnt = scr.cnt.data();
            // (triangle trees bin with one multiply: the many per-cell builds;
            // sphere trees keep the division their tuned trees were built with)
            const double inv = kBins / ext;
            for (uint32_t i = first; i < first + count; ++i) {
                int b = phantom > 0 ? (int)((key(prims[i], ax) - lo) * inv)
                                    : (int)((key(prims[i], ax) - lo) / ext * kBins);
                b = std::min(kBins - 1, std::max(0, b));
                bb[b].grow(prims[i].box);
                nb[b].grow(prims[i].n);
                ++cnt[b];
            }
            double *left = scr.left.data();
            uint32_t *lc = scr.lc.data();
            Box acc, nacc;
            uint32_t c = 0;
            for (int b = 0; b < kBins; ++b) {
                acc.grow(bb[b]);
                nacc.grow(nb[b]);
                c += cnt[b];
                left[b] = cost_area(acc, nacc);
                lc[b] = c;
            }
            acc = Box();
            nacc = Box();
            c = 0;
            for (int b = kBins - 1; b > 0; --b) {
                acc.grow(bb[b]);
                nacc.grow(nb[b]);
                c += cnt[b];
                if (lc[b - 1] == 0 || c == 0) continue;
                const double cost = left[b - 1] * lc[b - 1] + cost_area(acc, nacc) * c;
                if (cost < best_cost) {
                    best_cost = cost; best_axis = ax; best_split = b; best_lo = lo; best_ext = ext;
                }
            }
        }
        uint32_t mid;
        if (best_axis < 0 || depth > 40) {
            // degenerate centroids (or very deep): median split on the widest axis
            int axis = 0;
            double w = -1;
            for (int k = 0; k < 3; ++k)
                if (cbox.hi[k] - cbox.lo[k] > w) { w = cbox.hi[k] - cbox.lo[k]; axis = k; }
            mid = first + count / 2;
            std::nth_element(prims.begin() + first, prims.begin() + mid, prims.begin() + first + count,
                             [axis](const Prim &x, const Prim &y) { return x.c[axis] < y.c[axis]; });
        } else {
            auto it = std::partition(prims.begin() + first, prims.begin() + first + count,
                                     [&](const Prim &p) {
                                         int b = phantom > 0
                                                     ? (int)((key(p, best_axis) - best_lo) * (kBins / best_ext))
                                                     : (int)((key(p, best_axis) - best_lo) / best_ext * kBins);
                                         b = std::min(kBins - 1, std::max(0, b));
                                         return b < best_split;
                                     });
            mid = (uint32_t)(it - prims.begin());
            if (mid == first || mid == first + count) mid = first + count / 2;
        }
        // Traversal order: the kernel visits child a first unless the ray
        // points down axis b.  b = the axis that best separates the children's
        // mean centroids, with the lower child first.
        double ml[3] = {0, 0, 0}, mr[3] = {0, 0, 0};
        for (uint32_t i = first; i < mid; ++i)
            for (int k = 0; k < 3; ++k) ml[k] += prims[i].c[k] / (mid - first);
        for (uint32_t i = mid; i < first + count; ++i)
            for (int k = 0; k < 3; ++k) mr[k] += prims[i].c[k] / (first + count - mid);
        int axis = 0;
        for (int k = 1; k < 3; ++k)
            if (std::fabs(mr[k] - ml[k]) > std::fabs(mr[axis] - ml[axis])) axis = k;
        if (ml[axis] > mr[axis]) {
            std::rotate(prims.begin() + first, prims.begin() + mid, prims.begin() + first + count);
            mid = first + (first + count - mid);
        }
        const uint32_t l = (uint32_t)nodes.size();
        nodes.emplace_back();
        nodes.emplace_back();
        nodes[n].a = l;
        nodes[n].b = (uint32_t)axis;
        build(l, first, mid - first, depth + 1);
        build(l + 1, mid, first + count - mid, depth + 1);
    }

    // miss links for one octant: DFS successor after a node's subtree
    void links(uint32_t n, uint32_t miss_n, uint32_t oct, std::vector<uint32_t> &miss) const {
        miss[(size_t)n * 8 + oct] = miss_n;
        if (nodes[n].leaf) return;
        const uint32_t l = nodes[n].a, r = l + 1;
        const bool neg = (oct >> nodes[n].b) & 1u;  // ray points down this axis
        const uint32_t first = neg ? r : l, second = neg ? l : r;
        links(first, second, oct, miss);
        links(second, miss_n, oct, miss);
    }
};

bool finite_sphere(const Sphere &s) {
    return std::isfinite(s.center.x) && std::isfinite(s.center.y) && std::isfinite(s.center.z) &&
           std::isfinite(s.radius);
}

}  // namespace

// Box of the unit normals of prims in node n (recursive), rounded outward.
static void normal_boxes(const Builder &b, const std::vector<Prim> &prims, uint32_t n,
                         std::vector<Box> &out) {
    Box nb;
    const auto &nd = b.nodes[n];
    if (nd.leaf) {
        for (uint32_t i = nd.a; i < nd.a + nd.b; ++i) nb.grow(prims[i].n);
    } else {
        normal_boxes(b, prims, nd.a, out);
        normal_boxes(b, prims, nd.a + 1, out);
        nb.grow(out[nd.a]);
        nb.grow(out[nd.a + 1]);
    }
    out[n] = nb;
}

// Classifies triangle i for the trees: 0 = tree primitive (p filled), 1 =
// degenerate (never accepted), 2 = brute force (non-finite data, sliver).
static int triangle_prim(const Triangle &t, const float *h, uint32_t i, Prim &p) {
    const double v[3][3] = {{t.v0.x, t.v0.y, t.v0.z}, {t.v1.x, t.v1.y, t.v1.z},
                            {t.v2.x, t.v2.y, t.v2.z}};
    bool finite = std::isfinite(h[0]) && std::isfinite(h[1]) && std::isfinite(h[2]) &&
                  std::isfinite(h[3]);
    for (int k = 0; k < 3; ++k)
        for (int j = 0; j < 3; ++j) finite = finite && std::isfinite(v[k][j]);
    const double nn = std::sqrt((double)h[0] * h[0] + (double)h[1] * h[1] + (double)h[2] * h[2]);
    if (finite && nn == 0.0) return 1;  // cos == 0 for every finite ray: never accepted
    // The edge tests accept points whose projection along the stored n lies
    // in the triangle.  Keep only triangles whose stored n is within ~2.6
    // degrees of the exact plane normal, so that projection is well
    // conditioned; the rest (slivers, non-finite data) are brute forced.
    double e1[3], e2[3], tn[3];
    for (int k = 0; k < 3; ++k) { e1[k] = v[1][k] - v[0][k]; e2[k] = v[2][k] - v[0][k]; }
    tn[0] = e1[1] * e2[2] - e1[2] * e2[1];
    tn[1] = e1[2] * e2[0] - e1[0] * e2[2];
    tn[2] = e1[0] * e2[1] - e1[1] * e2[0];
    const double tl = std::sqrt(tn[0] * tn[0] + tn[1] * tn[1] + tn[2] * tn[2]);
    const double cosphi = finite && tl > 0 ? (tn[0] * h[0] + tn[1] * h[1] + tn[2] * h[2]) / (tl * nn)
                                           : -1.0;
    if (!(cosphi >= 0.999)) return 2;
    for (int k = 0; k < 3; ++k) p.n[k] = (double)h[k] / nn;
    // Accepted points are q + (2 n^.o) n^ + w n^ with q in the triangle and
    // |w| <= max_i |n^.(v0 - v_i)| (n^ is not exactly normal to the plane).
    double w = 0;
    for (int j = 1; j < 3; ++j) {
        const double d = p.n[0] * (v[0][0] - v[j][0]) + p.n[1] * (v[0][1] - v[j][1]) +
                         p.n[2] * (v[0][2] - v[j][2]);
        w = std::max(w, std::fabs(d));
    }
    double vm = 0;
    for (int k = 0; k < 3; ++k)
        for (int j = 0; j < 3; ++j) vm = std::max(vm, std::fabs(v[k][j]));
    w = w * (1 + 1e-9) + 1e-15 * vm;
    for (int k = 0; k < 3; ++k) {
        const double pad = w * std::fabs(p.n[k]);
        p.box.lo[k] = std::min({v[0][k], v[1][k], v[2][k]}) - pad;
        p.box.hi[k] = std::max({v[0][k], v[1][k], v[2][k]}) + pad;
        p.c[k] = (p.box.lo[k] + p.box.hi[k]) / 2;
    }
    p.id = i;
    return 0;
}

// 16-float records (n, n.v0) (v0, bits(id)) (v1, 0) (v2, 0) in tree order.
static std::vector<float> triangle_records(const std::vector<Prim> &prims,
                                           const std::vector<Triangle> &tris,
                                           const std::vector<float> &tri_hot) {
    std::vector<float> out(prims.size() * 16);
    for (size_t i = 0; i < prims.size(); ++i) {
        const uint32_t id = prims[i].id;
        const Triangle &t = tris[id];
        float *r = &out[i * 16];
        std::memcpy(r, &tri_hot[(size_t)id * 4], 4 * sizeof(float));
        const Vec3 vs[3] = {t.v0, t.v1, t.v2};
        for (int j = 0; j < 3; ++j) {
            r[4 * (j + 1) + 0] = vs[j].x;
            r[4 * (j + 1) + 1] = vs[j].y;
            r[4 * (j + 1) + 2] = vs[j].z;
            r[4 * (j + 1) + 3] = 0.0f;
        }
        r[7] = bits_f(id);
    }
    return out;
}

// ---- quantised kernel nodes (bvh.h QuantGrid)
static float qdec(uint32_t q, float step, float base) { return std::fmaf((float)q, step, base); }

// grid over [lo, hi] with 65535 steps whose decode covers both ends
static void make_grid(float lo, float hi, float &base, float &step) {
    base = lo;
    step = hi > lo ? up(((double)hi - (double)lo) / 65535.0 * (1 + 1e-6))
                   : std::numeric_limits<float>::min();
    while (qdec(65535, step, base) < hi) step = std::nextafter(step, std::numeric_limits<float>::infinity());
}
static uint32_t q_down(float x, float step, float base) {  // largest q: decode(q) <= x
    double g = std::floor(((double)x - base) / step);
    uint32_t q = (uint32_t)std::min(65535.0, std::max(0.0, g));
    while (q > 0 && qdec(q, step, base) > x) --q;
    while (q < 65535 && qdec(q + 1, step, base) <= x) ++q;
    return q;
}
static uint32_t q_up(float x, float step, float base) {  // smallest q: decode(q) >= x
    double g = std::ceil(((double)x - base) / step);
    uint32_t q = (uint32_t)std::min(65535.0, std::max(0.0, g));
    while (q < 65535 && qdec(q, step, base) < x) ++q;
    while (q > 0 && qdec(q - 1, step, base) >= x) --q;
    return q;
}
static uint32_t node_word(const float *lo_a, const float *hi_b) {  // a, b bits -> kernel a
    uint32_t a, b;
    std::memcpy(&a, lo_a, 4);
    std::memcpy(&b, hi_b, 4);
    if (a & kLeafBit) return kLeafBit | ((a & ~kLeafBit) << 3) | b;  // first << 3 | count
    return a | (b << 29);                                             // child | axis << 29
}
// nodes: `stride` floats per node (min.xyz, a) (max.xyz, b) [(nmin) (nmax)].
// Kernel image, 8 u32 per node, one 32-B sector:
//   static: box (3 words) | normal box (3 words) | a | link
//   camera: box (3 words) | a | link | 0 0 0
// link = the DFS successor of a fixed child-a-first order (octant 0 of
// `miss`): octant-ordered links change node visits by 1-3 % at C5
// (tools/tbvh_sim.cpp SIM_FIXED_OCT) but cost a second cache line per step.
static void quantize_boxes(const std::vector<float> &nodes, size_t stride, bool normals,
                           const std::vector<uint32_t> &miss, std::vector<uint32_t> &q, QuantGrid &g,
                           float *nbase, float *nstep, const float *glo = nullptr, const float *ghi = nullptr) {
    const size_t n = nodes.size() / stride;
    float lo[3], hi[3], nlo = 1, nhi = -1;
    for (int k = 0; k < 3; ++k) { lo[k] = nodes[k]; hi[k] = nodes[4 + k]; }  // root holds all
    if (glo)  // a grid over a given box holding the root's (per-cell trees: one grid for all)
        for (int k = 0; k < 3; ++k) { lo[k] = std::min(lo[k], glo[k]); hi[k] = std::max(hi[k], ghi[k]); }
    for (size_t i = 0; i < n && normals; ++i)
        for (int k = 0; k < 3; ++k) {
            nlo = std::min(nlo, nodes[i * stride + 8 + k]);
            nhi = std::max(nhi, nodes[i * stride + 12 + k]);
        }
    for (int k = 0; k < 3; ++k) make_grid(lo[k], hi[k], g.base[k], g.step[k]);
    if (normals) make_grid(nlo, nhi, *nbase, *nstep);
    q.assign(n * 8, 0);
    for (size_t i = 0; i < n; ++i) {
        const float *f = &nodes[i * stride];
        uint32_t b[6];
        for (int k = 0; k < 3; ++k) {
            b[k] = q_down(f[k], g.step[k], g.base[k]);
            b[3 + k] = q_up(f[4 + k], g.step[k], g.base[k]);
        }
        uint32_t *w = &q[i * 8];
        w[0] = b[0] | b[1] << 16;
        w[1] = b[2] | b[3] << 16;
        w[2] = b[4] | b[5] << 16;
        if (normals) {
            uint32_t m[6];
            for (int k = 0; k < 3; ++k) {
                m[k] = q_down(f[8 + k], *nstep, *nbase);
                m[3 + k] = q_up(f[12 + k], *nstep, *nbase);
            }
            w[3] = m[0] | m[1] << 16;
            w[4] = m[2] | m[3] << 16;
            w[5] = m[4] | m[5] << 16;
            w[6] = node_word(&f[3], &f[7]);
            w[7] = miss[i * 8];
        } else {
            w[3] = node_word(&f[3], &f[7]);
            w[4] = miss[i * 8];
        }
    }
}

TriangleBVH build_triangle_bvh(const std::vector<Triangle> &tris, const std::vector<float> &tri_hot,
                               uint32_t leaf_size, const float *oc, double phantom, bool image) {
    TriangleBVH out;
    if (oc)
        for (int k = 0; k < 3; ++k) out.oc[k] = oc[k];
    std::vector<Prim> prims;
    std::vector<Prim> geo_prims;  // unshifted, for the centre / radius bound
    for (uint32_t i = 0; i < tris.size(); ++i) {
        Prim p;
        const int kind = triangle_prim(tris[i], &tri_hot[(size_t)i * 4], i, p);
        if (kind == 2) out.loose.push_back(i);
        if (kind != 0) continue;
        geo_prims.push_back(p);
        if (oc) {  // phantoms of origin oc: + 2(n^.oc)n^ (exact in double, rounded outward below)
            const double sdot = p.n[0] * oc[0] + p.n[1] * oc[1] + p.n[2] * oc[2];
            for (int k = 0; k < 3; ++k) {
                p.box.lo[k] += 2 * sdot * p.n[k];
                p.box.hi[k] += 2 * sdot * p.n[k];
                p.c[k] = (p.box.lo[k] + p.box.hi[k]) / 2;
            }
        }
        prims.push_back(p);
    }
    if (prims.size() < 16 || prims.size() >= (1u << 27)) {
        // not worth a tree (brute force keeps the reference order), or beyond the
        // kernel node encoding (first < 2^28, child < 2^29)
        out.loose.clear();
        return out;
    }
    // phantom scale for the SAH: typical |o| (origins lie on or near the scene)
    Box geo;
    for (const Prim &p : prims) geo.grow(p.box);
    double cn = 0, hd = 0;
    for (int k = 0; k < 3; ++k) {
        const double c = (geo.lo[k] + geo.hi[k]) / 2;
        cn += c * c;
        hd = std::max(hd, (geo.hi[k] - geo.lo[k]) / 2);
    }
    double L = 0.4 * (std::sqrt(cn) + hd / 2);  // A/B on C5 (tools/tbvh_sim.cpp): 1-4 best
    if (const char *e = std::getenv("RT_AMD_TRI_PHANTOM")) L = std::atof(e);
    if (phantom > 0) L = phantom;
    Builder b(prims, std::min(7u, std::max(1u, leaf_size)), L > 0 ? L : 1e-30);  // count: 3 bits
    b.build_root((uint32_t)prims.size());
    out.depth = b.max_depth;
    std::vector<Box> nbox(b.nodes.size());
    normal_boxes(b, prims, 0, nbox);

    Box all;
    double mag = 0;
    for (const Prim &p : geo_prims) {
        all.grow(p.box);
        for (int k = 0; k < 3; ++k) mag = std::max({mag, std::fabs(p.box.lo[k]), std::fabs(p.box.hi[k])});
    }
    for (int k = 0; k < 3; ++k) mag = std::max(mag, (double)std::fabs(out.oc[k]));
    double half = 0;
    for (int k = 0; k < 3; ++k) {
        out.centre[k] = (float)((all.lo[k] + all.hi[k]) / 2);
        half = std::max(half, std::max(all.hi[k] - out.centre[k], out.centre[k] - all.lo[k]));
    }
    out.radius = up(half * std::sqrt(3.0) * (1 + 1e-6));
    out.mag = up(mag);

    out.nodes.resize(b.nodes.size() * 16);
    for (size_t n = 0; n < b.nodes.size(); ++n) {
        const auto &nd = b.nodes[n];
        float *o = &out.nodes[n * 16];
        for (int k = 0; k < 3; ++k) {
            o[k] = down(nd.box.lo[k]);
            o[4 + k] = up(nd.box.hi[k]);
            o[8 + k] = down(nbox[n].lo[k]);
            o[12 + k] = up(nbox[n].hi[k]);
        }
        o[3] = bits_f(nd.leaf ? (nd.a | kLeafBit) : nd.a);
        o[7] = bits_f(nd.b);
    }
    out.miss.assign(b.nodes.size() * 8, kNodeEnd);
    for (uint32_t oct = 0; oct < 8; ++oct) b.links(0, kNodeEnd, oct, out.miss);
    out.tris = triangle_records(prims, tris, tri_hot);
    if (image) {
        quantize_boxes(out.nodes, 16, true, out.miss, out.qnodes, out.qbox, &out.nbase, &out.nstep);
        build_wide_image(out);
    }
    return out;
}

// f16 bits of the largest half <= x (up = false) or the smallest half >= x
// (up = true), for finite x within the half range (the normal boxes: |x| <= 1)
static float half_value(uint16_t h) {
    const int e = (h >> 10) & 31, m = h & 1023;
    const float v = e == 0 ? std::ldexp((float)m, -24) : std::ldexp((float)(1024 + m), e - 25);
    return (h & 0x8000) ? -v : v;
}
static uint16_t half_round(float x, bool up) {
    // every finite half, ascending; built once by a magic static (thread-safe
    // initialisation: two worlds may load at once, the ctypes binding drops the GIL)
    static const std::vector<std::pair<float, uint16_t>> table = [] {
        std::vector<std::pair<float, uint16_t>> t;
        for (uint32_t h = 0; h < 65536; ++h)
            if (((h >> 10) & 31) != 31) t.push_back({half_value((uint16_t)h), (uint16_t)h});
        std::stable_sort(t.begin(), t.end(),
                         [](const std::pair<float, uint16_t> &a, const std::pair<float, uint16_t> &b) {
                             return a.first < b.first;
                         });
        return t;
    }();
    if (up) {
        auto it = std::lower_bound(table.begin(), table.end(), x,
                                   [](const std::pair<float, uint16_t> &a, float v) { return a.first < v; });
        return it == table.end() ? (uint16_t)0x7C00u : it->second;  // (+inf: never for |x| <= 1)
    }
    auto it = std::upper_bound(table.begin(), table.end(), x,
                               [](float v, const std::pair<float, uint16_t> &a) { return v < a.first; });
    return it == table.begin() ? (uint16_t)0xFC00u : std::prev(it)->second;
}

void build_wide_image(TriangleBVH &tb) {
    tb.wnodes.clear();
    tb.wdepth = 0;
    const size_t n = tb.qnodes.size() / 8;
    if (n == 0) return;
    auto word = [&](uint32_t node, int k) { return tb.qnodes[(size_t)node * 8 + k]; };
    auto is_leaf = [&](uint32_t node) { return (word(node, 6) & kLeafBit) != 0; };
    auto child = [&](uint32_t node) { return word(node, 6) & 0x1FFFFFFFu; };
    // the binary nodes a wide node holds: grandchildren of binary node b
    auto slots = [&](uint32_t b, uint32_t out[4]) -> int {
        int m = 0;
        if (is_leaf(b)) {  // (a one-leaf tree: the root record holds node 0 itself)
            out[m++] = b;
            return m;
        }
        for (uint32_t c = child(b); c < child(b) + 2; ++c) {
            if (is_leaf(c)) {
                out[m++] = c;
            } else {
                out[m++] = child(c);
                out[m++] = child(c) + 1;
            }
        }
        return m;
    };
    // breadth-first: wide node w stands for binary node order[w]
    std::vector<uint32_t> order{0}, depth{0};
    for (size_t w = 0; w < order.size(); ++w) {
        if (order.size() > 65535) return;  // u16 stack entries
        uint32_t s[4];
        const int m = slots(order[w], s);
        for (int c = 0; c < m; ++c)
            if (!is_leaf(s[c]) && !(order[w] == 0 && is_leaf(0))) {
                order.push_back(s[c]);
                depth.push_back(depth[w] + 1);
            }
    }
    if (order.size() > 65535) return;
    tb.wnodes.assign(order.size() * 32, 0u);
    uint32_t next = 1;  // wide index of the next internal child, in the push order above
    for (size_t w = 0; w < order.size(); ++w) {
        uint32_t *r = &tb.wnodes[w * 32];
        uint32_t s[4];
        const int m = slots(order[w], s);
        for (int c = 0; c < 4; ++c) {
            if (c >= m) {
                r[24 + c] = kLeafBit;  // empty: a leaf without triangles
                continue;
            }
            for (int k = 0; k < 3; ++k) r[6 * c + k] = word(s[c], k);
            // the normal box as halves, rounded outward from the float box
            // (render.hip tri_wide_child decodes them with v_cvt_f32_f16)
            const float *nf = &tb.nodes[(size_t)s[c] * 16];
            uint16_t h[6];
            for (int k = 0; k < 3; ++k) {
                h[k] = half_round(nf[8 + k], false);
                h[3 + k] = half_round(nf[12 + k], true);
            }
            for (int k = 0; k < 3; ++k) r[6 * c + 3 + k] = (uint32_t)h[2 * k] | ((uint32_t)h[2 * k + 1] << 16);
            r[24 + c] = is_leaf(s[c]) ? word(s[c], 6) : next++;
        }
        tb.wdepth = std::max(tb.wdepth, depth[w]);
    }
}

float triangle_cell_edge(const std::vector<Triangle> &tris, uint32_t max_cells) {
    double lo[3] = {INFINITY, INFINITY, INFINITY}, hi[3] = {-INFINITY, -INFINITY, -INFINITY};
    for (const Triangle &t : tris)
        for (const Vec3 &v : {t.v0, t.v1, t.v2}) {
            const double c[3] = {v.x, v.y, v.z};
            if (!(std::isfinite(c[0]) && std::isfinite(c[1]) && std::isfinite(c[2]))) continue;
            for (int k = 0; k < 3; ++k) { lo[k] = std::min(lo[k], c[k]); hi[k] = std::max(hi[k], c[k]); }
        }
    double ext = 0;
    for (int k = 0; k < 3; ++k) {
        if (!(lo[k] <= hi[k])) return 0.0f;
        ext = std::max(ext, hi[k] - lo[k]);
    }
    if (!(ext > 0) || !std::isfinite(ext)) return 0.0f;
    for (double s = ext / 64; s <= ext * 2; s *= 1.05) {
        double n = 1;
        for (int k = 0; k < 3; ++k) n *= std::max(1.0, std::ceil((hi[k] - (double)(float)lo[k]) / s + 1e-9));
        if (n <= max_cells) return (float)s;
    }
    return (float)ext;
}

TriangleCells build_triangle_cells(const std::vector<Triangle> &tris, const std::vector<float> &tri_hot,
                                   const std::vector<Sphere> &spheres, uint32_t leaf_size, float size,
                                   TriangleBVH &tb) {
    TriangleCells out;
    if (tb.nodes.empty() || tb.wnodes.empty() || !(size > 0)) return out;
    // The grid covers where secondary rays start near the mesh: the box of the
    // mesh's (finite) vertices and of every sphere no larger than the mesh
    // (a ground sphere of radius 1000 would only stretch it; its surface still
    // marks the cells it crosses below).  RT_AMD_TRI_CELL_SCENE=0: the mesh's
    // box alone (the first build, A/B only).
    double lo[3] = {INFINITY, INFINITY, INFINITY}, hi[3] = {-INFINITY, -INFINITY, -INFINITY};
    auto finite3 = [](const Vec3 &v) { return std::isfinite(v.x) && std::isfinite(v.y) && std::isfinite(v.z); };
    for (const Triangle &t : tris)
        for (const Vec3 &v : {t.v0, t.v1, t.v2}) {
            if (!finite3(v)) continue;
            const double c[3] = {v.x, v.y, v.z};
            for (int k = 0; k < 3; ++k) { lo[k] = std::min(lo[k], c[k]); hi[k] = std::max(hi[k], c[k]); }
        }
    double ext = 0;
    for (int k = 0; k < 3; ++k) {
        if (!(lo[k] <= hi[k])) return out;
        ext = std::max(ext, hi[k] - lo[k]);
    }
    const char *scene_env = std::getenv("RT_AMD_TRI_CELL_SCENE");
    if (!(scene_env && std::atoi(scene_env) == 0))
        for (const Sphere &sp : spheres) {
            const double r = std::fabs((double)sp.radius);
            if (!finite3(sp.center) || !(r <= ext)) continue;
            const double c[3] = {sp.center.x, sp.center.y, sp.center.z};
            for (int k = 0; k < 3; ++k) { lo[k] = std::min(lo[k], c[k] - r); hi[k] = std::max(hi[k], c[k] + r); }
        }
    // Every cell gets a tree.  (Only cells that a surface passes through
    // would not do: a triangle's hits lie on its phantom for the ray's origin
    // (common.rs:141, the sign quirk), so secondary rays start all over the
    // region around the mesh.  Trees for occupied cells only, 79 of C5's
    // 189: 106.4 ms; occupancy grown by one cell: 97.7; every cell: 97.7.)
    // The edge grows (5 % steps) until the grid has <= 1024 cells and the
    // trees hold <= 4e7 triangles in all (C5, 2.49 / 2.2 / 2.0-unit cells:
    // 189 / 320 / 396 trees, 97.2 / 91.1 / 88.7 ms).
    // (RT_AMD_TRI_CELL_BUDGET: the triangle budget, tuning only)
    const char *budget_env = std::getenv("RT_AMD_TRI_CELL_BUDGET");
    const double budget = budget_env ? std::atof(budget_env) : 4e7;
    uint64_t ncells = 0;
    for (int attempt = 0; attempt < 400; ++attempt, size *= 1.05f) {
        ncells = 1;
        for (int k = 0; k < 3; ++k) {
            out.lo[k] = (float)lo[k];
            out.n[k] = (uint32_t)std::max(1.0, std::ceil((hi[k] - out.lo[k]) / size + 1e-9));
            ncells *= out.n[k];
        }
        if (ncells <= 1024 && (double)ncells * (double)tris.size() <= budget) break;
    }
    if (ncells > 1024 || (double)ncells * (double)tris.size() > budget) return TriangleCells{};
    out.size = size;
    out.ncells = (uint32_t)ncells;
    // SAH phantom scale in half-diagonals (RT_AMD_TRI_CELL_SAH, tuning only):
    // 0.4, between the two best measured scales (a uniform origin lies 0.55
    // half-diagonals from its cell's centre on average).  C5 lean frames at 2.5-unit cells
    // (profiles/round6_c5_cells/sah_scale_sweep*.log): scale 1e-3 148.1 ms,
    // 0.25 135.1, 0.5 135.3, 1 138.7, 2 145.7, 4 167.8
    const char *sah_env = std::getenv("RT_AMD_TRI_CELL_SAH");
    const double sah = sah_env ? std::max(1e-3, std::atof(sah_env)) : 0.4;
    // one tree per cell, on host threads, built for the cell's centre (the
    // kernel widens from the centre of the origin's cell)
    std::vector<TriangleBVH> trees(ncells);
    std::atomic<uint64_t> next{0};
    auto work = [&]() {
        const bool was_serial = tl_serial_build;  // (the calling thread runs work() too)
        tl_serial_build = true;
        for (uint64_t c; (c = next++) < ncells;) {
            const uint64_t x = c % out.n[0], y = (c / out.n[0]) % out.n[1], z = c / (out.n[0] * out.n[1]);
            const float oc[3] = {out.lo[0] + ((float)x + 0.5f) * size, out.lo[1] + ((float)y + 0.5f) * size,
                                 out.lo[2] + ((float)z + 0.5f) * size};
            trees[c] = build_triangle_bvh(tris, tri_hot, leaf_size, oc, size * 0.866 * sah, false);
        }
        tl_serial_build = was_serial;
    };
    const unsigned nt = std::max(1u, std::min(16u, std::thread::hardware_concurrency()));
    const auto t0 = std::chrono::steady_clock::now();
    std::vector<std::thread> pool;
    for (unsigned i = 1; i < nt; ++i) pool.emplace_back(work);
    work();
    for (auto &t : pool) t.join();
    const auto t1 = std::chrono::steady_clock::now();
    // one grid for every tree (and the static one): the union of their roots
    float glo[3], ghi[3];
    for (int k = 0; k < 3; ++k) { glo[k] = tb.nodes[k]; ghi[k] = tb.nodes[4 + k]; }
    for (uint64_t c = 0; c < ncells; ++c) {
        const TriangleBVH &t = trees[c];
        if (t.nodes.empty()) return TriangleCells{};
        for (int k = 0; k < 3; ++k) { glo[k] = std::min(glo[k], t.nodes[k]); ghi[k] = std::max(ghi[k], t.nodes[4 + k]); }
    }
    trees.push_back(tb);
    {  // every tree (and the static one) on the common grid, on the same threads
        std::atomic<uint64_t> next_q{0};
        auto quant = [&]() {
            for (uint64_t c; (c = next_q++) <= ncells;) {
                TriangleBVH &t = trees[c];
                quantize_boxes(t.nodes, 16, true, t.miss, t.qnodes, t.qbox, &t.nbase, &t.nstep, glo, ghi);
                build_wide_image(t);
                if (c < ncells) {  // a cell tree keeps only its wide image and records (host memory)
                    std::vector<float>().swap(t.nodes);
                    std::vector<uint32_t>().swap(t.miss);
                    std::vector<uint32_t>().swap(t.qnodes);
                }
            }
        };
        std::vector<std::thread> qpool;
        for (unsigned i = 1; i < nt; ++i) qpool.emplace_back(quant);
        quant();
        for (auto &t : qpool) t.join();
    }
    const auto t2 = std::chrono::steady_clock::now();
    if (std::getenv("RT_AMD_TRI_CELLS_DEBUG"))
        std::fprintf(stderr, "cell trees: build %.2f s, quantise + wide images %.2f s\n",
                     std::chrono::duration<double>(t1 - t0).count(), std::chrono::duration<double>(t2 - t1).count());
    uint64_t sw = 0;
    for (uint64_t c = 0; c <= ncells; ++c) {
        TriangleBVH &t = trees[c];
        if (t.wnodes.empty()) return TriangleCells{};
        sw = std::max<uint64_t>(sw, t.wnodes.size() / 32);
        out.wdepth = std::max(out.wdepth, t.wdepth);
        out.mag = std::max(out.mag, t.mag);
    }
    if ((ncells + 1) * sw >= (1ull << 32)) return TriangleCells{};
    // One record array for every tree.  A record holds nothing of its tree
    // ((n, n.v0) (v0, id) (v1) (v2), triangle_records), so the static tree's
    // records serve all of them: a cell tree's leaf is pointed at its
    // triangles' run there, and only a leaf whose triangles are not one run
    // in the static order gets copies appended.  (Per-tree copies took 10 MB
    // per tree: 30 trees pushed C5's records out of the caches.)
    const TriangleBVH &st = trees[ncells];
    auto rec_id = [](const std::vector<float> &r, size_t j) {
        uint32_t id;
        std::memcpy(&id, &r[j * 16 + 7], 4);
        return id;
    };
    std::vector<uint32_t> spos(tris.size(), ~0u);
    for (size_t j = 0; j < st.tris.size() / 16; ++j) spos[rec_id(st.tris, j)] = (uint32_t)j;
    out.tris = st.tris;
    for (uint64_t c = 0; c < ncells; ++c) {
        TriangleBVH &t = trees[c];
        for (size_t w = 0; w < t.wnodes.size() / 32; ++w)
            for (int k = 0; k < 4; ++k) {
                uint32_t &word = t.wnodes[w * 32 + 24 + k];
                if (!(word & kLeafBit) || (word & 7u) == 0) continue;  // inner / empty child
                const uint32_t first = (word & ~kLeafBit) >> 3, count = word & 7u;
                uint32_t s0 = spos[rec_id(t.tris, first)];
                bool run = s0 != ~0u;
                for (uint32_t j = 1; run && j < count; ++j) run = spos[rec_id(t.tris, first + j)] == s0 + j;
                if (!run) {
                    s0 = (uint32_t)(out.tris.size() / 16);
                    out.tris.insert(out.tris.end(), t.tris.begin() + (size_t)first * 16,
                                    t.tris.begin() + (size_t)(first + count) * 16);
                }
                if (s0 >= (1u << 28)) return TriangleCells{};  // the leaf word's first field
                word = kLeafBit | (s0 << 3) | count;
            }
    }
    out.stride_w = (uint32_t)sw;
    out.wnodes.assign((ncells + 1) * sw * 32, 0u);
    for (uint64_t c = 0; c <= ncells; ++c)
        std::copy(trees[c].wnodes.begin(), trees[c].wnodes.end(), out.wnodes.begin() + c * sw * 32);
    tb = trees.back();  // (the static tree on the common grid: its binary walk's nodes too)
    return out;
}

CameraTriangleBVH build_camera_triangle_bvh(const std::vector<Triangle> &tris,
                                            const std::vector<float> &tri_hot, const TriangleBVH &tb,
                                            const float origin[3], uint32_t leaf_size, bool tree) {
    CameraTriangleBVH out;
    for (int k = 0; k < 3; ++k) out.origin[k] = origin[k];
    if (tb.nodes.empty()) return out;
    const double o[3] = {origin[0], origin[1], origin[2]};
    const double onorm = std::fabs(o[0]) + std::fabs(o[1]) + std::fabs(o[2]);
    if (!(onorm < 1e18)) return out;  // the kernel brute-forces such origins
    // the kernel's per-ray margin (render.hip triangles_bvh) for this origin
    double dist = tb.radius + 2 * onorm;
    for (int k = 0; k < 3; ++k) dist += std::fabs(o[k] - tb.centre[k]);
    const double rho = 1e-5 * (dist + onorm + tb.mag) * (1 + 1e-6);
    std::vector<Prim> prims;
    for (uint32_t i = 0; i < tris.size(); ++i) {
        Prim p;
        if (triangle_prim(tris[i], &tri_hot[(size_t)i * 4], i, p) != 0) continue;
        const double sdot = p.n[0] * o[0] + p.n[1] * o[1] + p.n[2] * o[2];
        for (int k = 0; k < 3; ++k) {
            const double off = 2 * sdot * p.n[k];
            p.box.lo[k] += off - rho;
            p.box.hi[k] += off + rho;
            p.c[k] = (p.box.lo[k] + p.box.hi[k]) / 2;
        }
        prims.push_back(p);
    }
    if (prims.empty()) return out;
    auto record_boxes = [&]() {
        out.rec_box.resize(prims.size() * 6);
        for (size_t i = 0; i < prims.size(); ++i)
            for (int k = 0; k < 3; ++k) {
                out.rec_box[i * 6 + k] = down(prims[i].box.lo[k]);
                out.rec_box[i * 6 + 3 + k] = up(prims[i].box.hi[k]);
            }
    };
    if (!tree) {  // records only (any order: candidates merge by (t, index))
        out.tris = triangle_records(prims, tris, tri_hot);
        record_boxes();
        return out;
    }
    Builder b(prims, std::min(7u, std::max(1u, leaf_size)));  // count: 3 bits
    b.build_root((uint32_t)prims.size());
    out.depth = b.max_depth;
    out.nodes.resize(b.nodes.size() * 8);
    for (size_t n = 0; n < b.nodes.size(); ++n) {
        const auto &nd = b.nodes[n];
        float *f = &out.nodes[n * 8];
        for (int k = 0; k < 3; ++k) { f[k] = down(nd.box.lo[k]); f[4 + k] = up(nd.box.hi[k]); }
        f[3] = bits_f(nd.leaf ? (nd.a | kLeafBit) : nd.a);
        f[7] = bits_f(nd.b);
    }
    out.miss.assign(b.nodes.size() * 8, kNodeEnd);
    for (uint32_t oct = 0; oct < 8; ++oct) b.links(0, kNodeEnd, oct, out.miss);
    out.tris = triangle_records(prims, tris, tri_hot);
    quantize_boxes(out.nodes, 8, false, out.miss, out.qnodes, out.qbox, nullptr, nullptr);
    record_boxes();
    return out;
}

SphereBVH build_sphere_bvh(const std::vector<Sphere> &spheres, uint32_t leaf_size) {
    SphereBVH out;
    // Very large spheres (e.g. a r=1000 ground) would inflate every box through
    // |o - c|; they, and anything non-finite, stay in the brute-force list.
    std::vector<double> radii;
    for (const Sphere &s : spheres)
        if (finite_sphere(s)) radii.push_back(std::fabs((double)s.radius));
    double median = 0;
    if (!radii.empty()) {
        std::nth_element(radii.begin(), radii.begin() + radii.size() / 2, radii.end());
        median = radii[radii.size() / 2];
    }
    std::vector<Prim> prims;
    // spheres above big_k x the median radius stay out of the tree (A/B on C2:
    // 4 -> 5.41 ms, 8 -> 5.35, 16 -> 5.34; the ground sphere in the tree -> 97)
    double big_k = 8.0;
    if (const char *e = std::getenv("RT_AMD_BIG_K")) {
        // a typo (0), a negative or non-finite value keeps the default
        const double k = std::atof(e);
        if (std::isfinite(k) && k > 0.0) big_k = k;
    }
    for (uint32_t i = 0; i < spheres.size(); ++i) {
        const Sphere &s = spheres[i];
        const double r = std::fabs((double)s.radius);
        if (!finite_sphere(s) || r > big_k * median) { out.big.push_back(i); continue; }
        Prim p;
        const double c[3] = {s.center.x, s.center.y, s.center.z};
        for (int k = 0; k < 3; ++k) { p.c[k] = c[k]; p.box.lo[k] = c[k] - r; p.box.hi[k] = c[k] + r; }
        p.id = i;
        prims.push_back(p);
    }
    if (prims.size() < 16) {  // not worth a tree
        out.big.clear();
        for (uint32_t i = 0; i < spheres.size(); ++i) out.big.push_back(i);
        return out;
    }
    Builder b(prims, std::max(1u, leaf_size));
    b.build_root((uint32_t)prims.size());
    out.depth = b.max_depth;

    Box all;
    double rmax = 0, rmin = std::numeric_limits<double>::infinity(), mag = 0;
    for (const Prim &p : prims) {
        all.grow(p.c);
        rmax = std::max(rmax, (p.box.hi[0] - p.box.lo[0]) / 2);
        rmin = std::min(rmin, (p.box.hi[0] - p.box.lo[0]) / 2);
        for (int k = 0; k < 3; ++k) mag = std::max({mag, std::fabs(p.box.lo[k]), std::fabs(p.box.hi[k])});
    }
    double half = 0;
    for (int k = 0; k < 3; ++k) {
        out.centre[k] = (float)((all.lo[k] + all.hi[k]) / 2);
        half = std::max(half, std::max(all.hi[k] - out.centre[k], out.centre[k] - all.lo[k]));
    }
    out.radius = up(half * std::sqrt(3.0) * (1 + 1e-6));
    out.rmax = up(rmax);
    // 1/rmin rounded up (rmin rounded down); inf when some radius is 0
    out.inv_rmin = rmin > 0 ? up(1.0 / (double)down(rmin)) : std::numeric_limits<float>::infinity();
    out.mag = up(mag);

    out.nodes.resize(b.nodes.size() * 8);
    for (size_t n = 0; n < b.nodes.size(); ++n) {
        const auto &nd = b.nodes[n];
        float *o = &out.nodes[n * 8];
        for (int k = 0; k < 3; ++k) { o[k] = down(nd.box.lo[k]); o[4 + k] = up(nd.box.hi[k]); }
        o[3] = bits_f(nd.leaf ? (nd.a | kLeafBit) : nd.a);
        o[7] = bits_f(nd.b);
    }
    out.miss.assign(b.nodes.size() * 8, kNodeEnd);
    for (uint32_t oct = 0; oct < 8; ++oct) b.links(0, kNodeEnd, oct, out.miss);
    out.prims.resize(prims.size() * 4);
    out.prim_id.resize(prims.size());
    for (size_t i = 0; i < prims.size(); ++i) {
        const Sphere &s = spheres[prims[i].id];
        out.prims[i * 4 + 0] = s.center.x;
        out.prims[i * 4 + 1] = s.center.y;
        out.prims[i * 4 + 2] = s.center.z;
        out.prims[i * 4 + 3] = s.radius * s.radius;  // same bits as the brute-force table
        out.prim_id[i] = prims[i].id;
    }
    return out;
}

}  // namespace rtamd

namespace rtamd {

// Inverse of the camera map: a primary ray's direction is M (u, v, 1) with
// M = [h | v | llc - o] (camera.rs:84-89), so a point P - o maps to w = Mi (P - o)
// and lies on the ray of (u, v) = (w0 / w2, w1 / w2) when w2 > 0.
static bool camera_inverse(const CameraModel &cam, double Mi[3][3]) {
    double M[3][3];
    const Vec3 cols[3] = {cam.horizontal, cam.vertical, {cam.lower_left.x - cam.origin.x,
                                                         cam.lower_left.y - cam.origin.y,
                                                         cam.lower_left.z - cam.origin.z}};
    for (int j = 0; j < 3; ++j) { M[0][j] = cols[j].x; M[1][j] = cols[j].y; M[2][j] = cols[j].z; }
    const double det = M[0][0] * (M[1][1] * M[2][2] - M[1][2] * M[2][1]) -
                       M[0][1] * (M[1][0] * M[2][2] - M[1][2] * M[2][0]) +
                       M[0][2] * (M[1][0] * M[2][1] - M[1][1] * M[2][0]);
    if (!(std::fabs(det) > 0) || !std::isfinite(det)) return false;
    Mi[0][0] = (M[1][1] * M[2][2] - M[1][2] * M[2][1]) / det;
    Mi[0][1] = (M[0][2] * M[2][1] - M[0][1] * M[2][2]) / det;
    Mi[0][2] = (M[0][1] * M[1][2] - M[0][2] * M[1][1]) / det;
    Mi[1][0] = (M[1][2] * M[2][0] - M[1][0] * M[2][2]) / det;
    Mi[1][1] = (M[0][0] * M[2][2] - M[0][2] * M[2][0]) / det;
    Mi[1][2] = (M[0][2] * M[1][0] - M[0][0] * M[1][2]) / det;
    Mi[2][0] = (M[1][0] * M[2][1] - M[1][1] * M[2][0]) / det;
    Mi[2][1] = (M[0][1] * M[2][0] - M[0][0] * M[2][1]) / det;
    Mi[2][2] = (M[0][0] * M[1][1] - M[0][1] * M[1][0]) / det;
    return true;
}

bool sphere_list_params(const SphereBVH &bv, const CameraModel &cam, size_t width, size_t height,
                        SphereListParams &out) {
    // (the checks and constants of build_primary_sphere_lists below)
    const size_t n = bv.prims.size() / 4;
    if (n == 0 || n >= kSphListWalk || width < 2 || height < 2 || height > (1u << 24) ||
        width > (1u << 24) || width * height > (1ull << 28))
        return false;
    const Vec3 cv[4] = {cam.origin, cam.lower_left, cam.horizontal, cam.vertical};
    double mag = 0;
    for (const Vec3 &v : cv) mag = std::max({mag, std::fabs((double)v.x), std::fabs((double)v.y),
                                             std::fabs((double)v.z)});
    double Mi[3][3];
    if (!(mag < 1e3) || !camera_inverse(cam, Mi)) return false;
    for (int r = 0; r < 3; ++r)
        for (int c = 0; c < 3; ++c) out.Mi[3 * r + c] = Mi[r][c];
    out.o[0] = cam.origin.x; out.o[1] = cam.origin.y; out.o[2] = cam.origin.z;
    out.e_abs = 4e-6 * (std::fabs(out.o[0]) + std::fabs(out.o[1]) + std::fabs(out.o[2]) + bv.mag);
    out.wden = (double)(float)(width - 1);
    out.hden = (double)(float)(height - 1);
    out.n = (uint32_t)n;
    out.width = (uint32_t)width;
    out.height = (uint32_t)height;
    return true;
}

PrimarySphereLists build_primary_sphere_lists(const SphereBVH &bv, const CameraModel &cam,
                                              size_t width, size_t height) {
    PrimarySphereLists out;
    const size_t n = bv.prims.size() / 4;
    if (n == 0 || n >= kSphListWalk || width < 2 || height < 2 || height > (1u << 24) ||
        width > (1u << 24) || width * height > (1ull << 28))
        return out;
    // the one-pixel margins below cover the rounding of u, v and the ray
    // direction (relative ~1e-7 of the camera's coordinates) for cameras near
    // the scene's scale; far-off cameras walk the tree instead
    const Vec3 cv[4] = {cam.origin, cam.lower_left, cam.horizontal, cam.vertical};
    double mag = 0;
    for (const Vec3 &v : cv) mag = std::max({mag, std::fabs((double)v.x), std::fabs((double)v.y),
                                             std::fabs((double)v.z)});
    double Mi[3][3];
    if (!(mag < 1e3) || !camera_inverse(cam, Mi)) return out;
    const double o[3] = {cam.origin.x, cam.origin.y, cam.origin.z};
    const double e_abs = 4e-6 * (std::fabs(o[0]) + std::fabs(o[1]) + std::fabs(o[2]) + bv.mag);
    const double wden = (double)(float)(width - 1), hden = (double)(float)(height - 1);
    const int64_t W = (int64_t)width, H = (int64_t)height;
    std::vector<uint8_t> cnt(width * height, 0);  // kSphListMax + 1 = overflow
    out.rec.assign(2 * width * height, 0);
    for (uint32_t i = 0; i < n; ++i) {
        const float *s = &bv.prims[(size_t)i * 4];
        const double c[3] = {s[0], s[1], s[2]};
        const double r = std::sqrt((double)s[3]) * (1 + 1e-6);
        const double a = std::sqrt((c[0] - o[0]) * (c[0] - o[0]) + (c[1] - o[1]) * (c[1] - o[1]) +
                                   (c[2] - o[2]) * (c[2] - o[2]));
        // the walk's margin (render.hip sph_inflation, K = 3e-3), doubled
        const double R = r + 2 * 3e-3 * (a + r) * 1.01 + 2 * e_abs;
        if (!std::isfinite(R) || !std::isfinite(a)) return PrimarySphereLists{};
        double umin = 1e300, umax = -1e300, vmin = 1e300, vmax = -1e300;
        int front = 0, behind = 0;
        for (int k = 0; k < 8; ++k) {  // corners of the inflated ball's box
            const double P[3] = {c[0] + (k & 1 ? R : -R) - o[0], c[1] + (k & 2 ? R : -R) - o[1],
                                 c[2] + (k & 4 ? R : -R) - o[2]};
            double w[3];
            for (int q = 0; q < 3; ++q) w[q] = Mi[q][0] * P[0] + Mi[q][1] * P[1] + Mi[q][2] * P[2];
            const double wn = std::fabs(w[0]) + std::fabs(w[1]) + std::fabs(w[2]);
            if (w[2] > 1e-6 * wn) {
                ++front;
                umin = std::min(umin, w[0] / w[2]); umax = std::max(umax, w[0] / w[2]);
                vmin = std::min(vmin, w[1] / w[2]); vmax = std::max(vmax, w[1] / w[2]);
            } else if (w[2] < -1e-6 * wn) {
                ++behind;
            }
        }
        if (behind == 8) continue;                         // no point of positive depth
        if (front < 8) return PrimarySphereLists{};        // straddles the camera plane: walk
        // pixel col covers u in [col, col + 1] / wden; one pixel of margin each side
        const double cl = std::floor(umin * wden) - 2, ch = std::floor(umax * wden) + 1;
        const double rl = std::floor(vmin * hden) - 2, rh = std::floor(vmax * hden) + 1;
        if (ch < 0 || cl > (double)(W - 1) || rh < 0 || rl > (double)(H - 1)) continue;
        const int64_t c0 = std::max<int64_t>(0, (int64_t)cl), c1 = std::min<int64_t>(W - 1, (int64_t)ch);
        const int64_t r0 = std::max<int64_t>(0, (int64_t)rl), r1 = std::min<int64_t>(H - 1, (int64_t)rh);
        for (int64_t rb = r0; rb <= r1; ++rb) {  // rb counts from the bottom (common.rs:327)
            const size_t row = (size_t)(H - 1 - rb) * width;
            for (int64_t col = c0; col <= c1; ++col) {
                const size_t px = row + (size_t)col;
                const uint32_t k = cnt[px];
                if (k >= kSphListMax) { cnt[px] = kSphListMax + 1; continue; }
                uint32_t &word = out.rec[2 * px + (k >> 1)];
                word |= i << (16 * (k & 1));
                cnt[px] = (uint8_t)(k + 1);
            }
        }
    }
    for (size_t px = 0; px < width * height; ++px)
        out.rec[2 * px + 1] = (out.rec[2 * px + 1] & 0xFFFFu) |
                              ((cnt[px] > kSphListMax ? kSphListWalk : cnt[px]) << 16);
    return out;
}

PrimaryTriLists build_primary_tri_lists(const CameraTriangleBVH &ct, const CameraModel &cam,
                                        size_t width, size_t height) {
    PrimaryTriLists out;
    const size_t n = ct.rec_box.size() / 6;
    if (n == 0 || width < 2 || height < 2 || height > (1u << 24) || width > (1u << 24)) return out;
    const double o[3] = {cam.origin.x, cam.origin.y, cam.origin.z};
    // ray direction = M (u, v, 1) with M = [h | v | llc - o]  (camera.rs:84-89)
    double M[3][3];
    const Vec3 cols[3] = {cam.horizontal, cam.vertical, {cam.lower_left.x - cam.origin.x,
                                                         cam.lower_left.y - cam.origin.y,
                                                         cam.lower_left.z - cam.origin.z}};
    for (int j = 0; j < 3; ++j) { M[0][j] = cols[j].x; M[1][j] = cols[j].y; M[2][j] = cols[j].z; }
    const double det = M[0][0] * (M[1][1] * M[2][2] - M[1][2] * M[2][1]) -
                       M[0][1] * (M[1][0] * M[2][2] - M[1][2] * M[2][0]) +
                       M[0][2] * (M[1][0] * M[2][1] - M[1][1] * M[2][0]);
    if (!(std::fabs(det) > 0) || !std::isfinite(det)) return out;
    double Mi[3][3];  // inverse via the adjugate
    Mi[0][0] = (M[1][1] * M[2][2] - M[1][2] * M[2][1]) / det;
    Mi[0][1] = (M[0][2] * M[2][1] - M[0][1] * M[2][2]) / det;
    Mi[0][2] = (M[0][1] * M[1][2] - M[0][2] * M[1][1]) / det;
    Mi[1][0] = (M[1][2] * M[2][0] - M[1][0] * M[2][2]) / det;
    Mi[1][1] = (M[0][0] * M[2][2] - M[0][2] * M[2][0]) / det;
    Mi[1][2] = (M[0][2] * M[1][0] - M[0][0] * M[1][2]) / det;
    Mi[2][0] = (M[1][0] * M[2][1] - M[1][1] * M[2][0]) / det;
    Mi[2][1] = (M[0][1] * M[2][0] - M[0][0] * M[2][1]) / det;
    Mi[2][2] = (M[0][0] * M[1][1] - M[0][1] * M[1][0]) / det;
    const double wden = (double)(float)(width - 1), hden = (double)(float)(height - 1);
    const int64_t W = (int64_t)width, H = (int64_t)height;
    const uint32_t spr = (uint32_t)((width + kTriStripW - 1) / kTriStripW);
    out.strips_per_row = spr;
    std::vector<uint32_t> count((size_t)spr * height + 1, 0), always;
    struct Span { uint32_t rec, s0, s1, r0, r1; };
    std::vector<Span> spans;
    spans.reserve(n);
    for (uint32_t i = 0; i < n; ++i) {
        const float *b = &ct.rec_box[(size_t)i * 6];
        double umin = 1e300, umax = -1e300, vmin = 1e300, vmax = -1e300;
        int front = 0, behind = 0;
        for (int c = 0; c < 8; ++c) {
            const double P[3] = {(c & 1 ? b[3] : b[0]) - o[0], (c & 2 ? b[4] : b[1]) - o[1],
                                 (c & 4 ? b[5] : b[2]) - o[2]};
            double w[3];
            for (int r = 0; r < 3; ++r) w[r] = Mi[r][0] * P[0] + Mi[r][1] * P[1] + Mi[r][2] * P[2];
            const double wn = std::fabs(w[0]) + std::fabs(w[1]) + std::fabs(w[2]);
            if (w[2] > 1e-6 * wn) {
                ++front;
                umin = std::min(umin, w[0] / w[2]); umax = std::max(umax, w[0] / w[2]);
                vmin = std::min(vmin, w[1] / w[2]); vmax = std::max(vmax, w[1] / w[2]);
            } else if (w[2] < -1e-6 * wn) {
                ++behind;
            }
        }
        if (behind == 8) continue;  // no point of positive depth
        if (front < 8) { always.push_back(i); continue; }
        // pixel col covers u in [col, col + 1] / wden; one pixel of margin each side
        const double cl = std::floor(umin * wden) - 2, ch = std::floor(umax * wden) + 1;
        const double rl = std::floor(vmin * hden) - 2, rh = std::floor(vmax * hden) + 1;
        if (ch < 0 || cl > (double)(W - 1) || rh < 0 || rl > (double)(H - 1)) continue;
        const int64_t c0 = std::max<int64_t>(0, (int64_t)cl), c1 = std::min<int64_t>(W - 1, (int64_t)ch);
        const int64_t r0 = std::max<int64_t>(0, (int64_t)rl), r1 = std::min<int64_t>(H - 1, (int64_t)rh);
        const Span sp{i, (uint32_t)(c0 / kTriStripW), (uint32_t)(c1 / kTriStripW), (uint32_t)r0, (uint32_t)r1};
        spans.push_back(sp);
        for (uint32_t r = sp.r0; r <= sp.r1; ++r)
            for (uint32_t s = sp.s0; s <= sp.s1; ++s) ++count[(size_t)r * spr + s + 1];
    }
    for (size_t k = 1; k < count.size(); ++k) count[k] += count[k - 1];
    out.offsets = count;
    out.items.assign(count.back() + always.size(), 0);
    std::vector<uint32_t> fill(count.begin(), count.end() - 1);
    for (const Span &sp : spans)
        for (uint32_t r = sp.r0; r <= sp.r1; ++r)
            for (uint32_t s = sp.s0; s <= sp.s1; ++s) out.items[fill[(size_t)r * spr + s]++] = sp.rec;
    std::copy(always.begin(), always.end(), out.items.begin() + count.back());
    return out;
}

}  // namespace rtamd
