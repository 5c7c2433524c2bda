// bvh.cpp -- binned-SAH build of the exact-pruning sphere BVH (see bvh.h).
#include "bvh.h"

#include <algorithm>
#include <cmath>
#include <cstring>
#include <limits>

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

struct Prim { Box box; double c[3]; uint32_t id; };

inline float down(double x) {  // largest float <= x
    float f = (float)x;
    return ((double)f > x) ? std::nextafter(f, -std::numeric_limits<float>::infinity()) : f;
}
inline float up(double x) {  // smallest float >= x
    float f = (float)x;
    return ((double)f < x) ? std::nextafter(f, std::numeric_limits<float>::infinity()) : f;
}
inline float bits_f(uint32_t u) { float f; std::memcpy(&f, &u, 4); return f; }

struct Builder {
    std::vector<Prim> &prims;
    uint32_t leaf_size;
    struct Node { Box box; uint32_t a = 0, b = 0; bool leaf = false; };
    std::vector<Node> nodes;
    uint32_t max_depth = 0;

    Builder(std::vector<Prim> &p, uint32_t ls) : prims(p), leaf_size(ls) {}

    void make_leaf(uint32_t n, uint32_t first, uint32_t count) {
        nodes[n].leaf = true;
        nodes[n].a = first;
        nodes[n].b = count;
    }

    // Builds node n over prims[first, first + count).
    void build(uint32_t n, uint32_t first, uint32_t count, uint32_t depth) {
        max_depth = std::max(max_depth, depth);
        Box box, cbox;
        for (uint32_t i = first; i < first + count; ++i) { box.grow(prims[i].box); cbox.grow(prims[i].c); }
        nodes[n].box = box;
        if (count <= leaf_size) { make_leaf(n, first, count); return; }
        // binned SAH over the centroid box
        constexpr int kBins = 16;
        double best_cost = std::numeric_limits<double>::infinity();
        int best_axis = -1, best_split = 0;
        for (int ax = 0; ax < 3; ++ax) {
            const double ext = cbox.hi[ax] - cbox.lo[ax];
            if (!(ext > 0)) continue;
            Box bb[kBins];
            uint32_t cnt[kBins] = {0};
            for (uint32_t i = first; i < first + count; ++i) {
                int b = (int)((prims[i].c[ax] - cbox.lo[ax]) / ext * kBins);
                b = std::min(kBins - 1, std::max(0, b));
                bb[b].grow(prims[i].box);
                ++cnt[b];
            }
            Box left[kBins];
            uint32_t lc[kBins];
            Box acc;
            uint32_t c = 0;
            for (int b = 0; b < kBins; ++b) { acc.grow(bb[b]); c += cnt[b]; left[b] = acc; lc[b] = c; }
            acc = Box();
            c = 0;
            for (int b = kBins - 1; b > 0; --b) {
                acc.grow(bb[b]);
                c += cnt[b];
                if (lc[b - 1] == 0 || c == 0) continue;
                const double cost = left[b - 1].area() * lc[b - 1] + acc.area() * c;
                if (cost < best_cost) { best_cost = cost; best_axis = ax; best_split = b; }
            }
        }
        uint32_t mid;
        int axis = best_axis;
        if (axis < 0 || depth > 40) {
            // degenerate centroids (or very deep): median split on the widest axis
            axis = 0;
            double w = -1;
            for (int k = 0; k < 3; ++k)
                if (cbox.hi[k] - cbox.lo[k] > w) { w = cbox.hi[k] - cbox.lo[k]; axis = k; }
            mid = first + count / 2;
            std::nth_element(prims.begin() + first, prims.begin() + mid, prims.begin() + first + count,
                             [axis](const Prim &x, const Prim &y) { return x.c[axis] < y.c[axis]; });
        } else {
            const double ext = cbox.hi[axis] - cbox.lo[axis];
            auto it = std::partition(prims.begin() + first, prims.begin() + first + count,
                                     [&](const Prim &p) {
                                         int b = (int)((p.c[axis] - cbox.lo[axis]) / ext * kBins);
                                         b = std::min(kBins - 1, std::max(0, b));
                                         return b < best_split;
                                     });
            mid = (uint32_t)(it - prims.begin());
            if (mid == first || mid == first + count) mid = first + count / 2;
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
    for (uint32_t i = 0; i < spheres.size(); ++i) {
        const Sphere &s = spheres[i];
        const double r = std::fabs((double)s.radius);
        if (!finite_sphere(s) || r > 8.0 * median) { out.big.push_back(i); continue; }
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
    b.nodes.reserve(prims.size() * 2);
    b.nodes.emplace_back();
    b.build(0, 0, (uint32_t)prims.size(), 0);
    out.depth = b.max_depth;

    Box all;
    double rmax = 0, mag = 0;
    for (const Prim &p : prims) {
        all.grow(p.c);
        rmax = std::max(rmax, (p.box.hi[0] - p.box.lo[0]) / 2);
        for (int k = 0; k < 3; ++k) mag = std::max({mag, std::fabs(p.box.lo[k]), std::fabs(p.box.hi[k])});
    }
    double half = 0;
    for (int k = 0; k < 3; ++k) {
        out.centre[k] = (float)((all.lo[k] + all.hi[k]) / 2);
        half = std::max(half, std::max(all.hi[k] - out.centre[k], out.centre[k] - all.lo[k]));
    }
    out.radius = up(half * std::sqrt(3.0) * (1 + 1e-6));
    out.rmax = up(rmax);
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
