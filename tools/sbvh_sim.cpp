// sbvh_sim.cpp -- host emulation of the sphere-tree walk (tuning tool).
// Walks the stackless octant-linked sphere BVH (bvh.h SphereBVH) the way
// render.hip does for rays of a scene -- primary rays of a W x H grid and
// diffuse bounces from their hits -- and reports the distribution of node
// visits per walk and what a 64-lane wave pays for it: a walk loop runs until
// its longest walk ends, so the wave's cost is the max over its lanes.
// Not product code, not a parity check (double arithmetic, no inflation).
//   g++ -O2 -std=c++17 -I../rust-swift-raytracer_amd/csrc sbvh_sim.cpp \
//       ../rust-swift-raytracer_amd/csrc/{bvh,scene}.cpp -o sbvh_sim -lpthread
//   ./sbvh_sim ../scenes/rtow.txt [W H]     (RT_AMD_LEAF: leaf size, default 3;
//   SIM_BVH4=1: node fetches and box tests of the tree collapsed to 4-wide nodes)
#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <sstream>
#include <vector>

#include "bvh.h"
#include "scene.h"

using namespace rtamd;

struct V { double x, y, z; };
static V add(V a, V b) { return {a.x + b.x, a.y + b.y, a.z + b.z}; }
static V sub(V a, V b) { return {a.x - b.x, a.y - b.y, a.z - b.z}; }
static V mul(V a, double s) { return {a.x * s, a.y * s, a.z * s}; }
static double dot(V a, V b) { return a.x * b.x + a.y * b.y + a.z * b.z; }
static V unit(V a) { return mul(a, 1.0 / std::sqrt(dot(a, a))); }

struct Hit { double t = INFINITY; int id = -1; };

static double sphere_t(V o, V d, const float *s) {  // (cx, cy, cz, r^2), |d| = 1
    V oc = sub(o, V{s[0], s[1], s[2]});
    const double hb = dot(oc, d), c = dot(oc, oc) - s[3], disc = hb * hb - c;
    if (disc < 0) return INFINITY;
    const double q = std::sqrt(disc), r1 = -hb - q, r2 = -hb + q;
    return r1 > 1e-3 ? r1 : r2 > 1e-3 ? r2 : INFINITY;
}

// the kernel's walk: big spheres, then the tree from the root along the
// octant links; returns node visits
static int walk(const SphereBVH &b, const std::vector<float> &hot, V o, V d, Hit &h) {
    for (uint32_t i : b.big) {
        const double t = sphere_t(o, d, &hot[(size_t)i * 4]);
        if (t < h.t) { h.t = t; h.id = (int)i; }
    }
    const double inv[3] = {1 / d.x, 1 / d.y, 1 / d.z}, ov[3] = {o.x, o.y, o.z};
    const uint32_t oct = (inv[0] < 0 ? 1u : 0u) | (inv[1] < 0 ? 2u : 0u) | (inv[2] < 0 ? 4u : 0u);
    int visits = 0;
    uint32_t node = 0;
    while (node != kNodeEnd) {
        ++visits;
        const float *n = &b.nodes[(size_t)node * 8];
        double tn = -INFINITY, tf = INFINITY;
        for (int k = 0; k < 3; ++k) {
            const double t0 = (n[k] - ov[k]) * inv[k], t1 = (n[4 + k] - ov[k]) * inv[k];
            tn = std::max(tn, std::min(t0, t1));
            tf = std::min(tf, std::max(t0, t1));
        }
        uint32_t a, bb;
        std::memcpy(&a, &n[3], 4);
        std::memcpy(&bb, &n[7], 4);
        const bool skip = tn > tf || tf < 1e-3 || tn > h.t;
        const bool leaf = a & kLeafBit;
        if (!skip && leaf)
            for (uint32_t j = a & ~kLeafBit; j < (a & ~kLeafBit) + bb; ++j) {
                const double t = sphere_t(o, d, &b.prims[(size_t)j * 4]);
                if (t < h.t) { h.t = t; h.id = (int)b.prim_id[j]; }
            }
        node = (skip || leaf) ? b.miss[(size_t)node * 8 + oct] : a + ((oct >> bb) & 1u);
    }
    return visits;
}

// SIM_BVH4=1: the same tree collapsed to 4 children per node (each internal
// child replaced by its two children), walked with a stack, nearest child
// first.  Returns node fetches; box tests (children tested) go to *tests.
static int walk4(const SphereBVH &b, const std::vector<float> &hot, V o, V d, Hit &h, int *tests) {
    for (uint32_t i : b.big) {
        const double t = sphere_t(o, d, &hot[(size_t)i * 4]);
        if (t < h.t) { h.t = t; h.id = (int)i; }
    }
    const double inv[3] = {1 / d.x, 1 / d.y, 1 / d.z}, ov[3] = {o.x, o.y, o.z};
    auto box = [&](uint32_t n, double &tn) {
        const float *f = &b.nodes[(size_t)n * 8];
        double a = -INFINITY, z = INFINITY;
        for (int k = 0; k < 3; ++k) {
            const double t0 = (f[k] - ov[k]) * inv[k], t1 = (f[4 + k] - ov[k]) * inv[k];
            a = std::max(a, std::min(t0, t1));
            z = std::min(z, std::max(t0, t1));
        }
        tn = a;
        return !(a > z || z < 1e-3 || a > h.t);
    };
    auto word = [&](uint32_t n, int k) { uint32_t w; std::memcpy(&w, &b.nodes[(size_t)n * 8 + k], 4); return w; };
    auto leaf = [&](uint32_t n) {
        const uint32_t a = word(n, 3), cnt = word(n, 7);
        for (uint32_t j = a & ~kLeafBit; j < (a & ~kLeafBit) + cnt; ++j) {
            const double t = sphere_t(o, d, &b.prims[(size_t)j * 4]);
            if (t < h.t) { h.t = t; h.id = (int)b.prim_id[j]; }
        }
    };
    int fetches = 0;
    double t0;
    std::vector<std::pair<double, uint32_t>> st;
    if (!box(0, t0)) return 0;
    if (word(0, 3) & kLeafBit) { leaf(0); return 1; }
    st.push_back({t0, 0});
    while (!st.empty()) {
        auto [tn, n] = st.back();
        st.pop_back();
        if (tn > h.t) continue;
        ++fetches;
        uint32_t kids[4], nk = 0;
        const uint32_t a = word(n, 3);
        for (uint32_t c = a; c < a + 2; ++c) {
            if (word(c, 3) & kLeafBit) kids[nk++] = c;
            else { const uint32_t g = word(c, 3); kids[nk++] = g; kids[nk++] = g + 1; }
        }
        std::pair<double, uint32_t> hit[4];
        int nh = 0;
        for (uint32_t k = 0; k < nk; ++k) {
            ++*tests;
            double t;
            if (box(kids[k], t)) hit[nh++] = {t, kids[k]};
        }
        std::sort(hit, hit + nh, [](auto &x, auto &y) { return x.first > y.first; });  // nearest last
        for (int k = 0; k < nh; ++k) {
            if (word(hit[k].second, 3) & kLeafBit) continue;
            st.push_back(hit[k]);
        }
        for (int k = nh - 1; k >= 0; --k)  // leaves now, nearest first
            if (word(hit[k].second, 3) & kLeafBit) leaf(hit[k].second);
    }
    return fetches;
}

int main(int argc, char **argv) {
    if (argc < 2) { std::fprintf(stderr, "usage: sbvh_sim scene.txt [W H]\n"); return 2; }
    std::ifstream f(argv[1]);
    std::stringstream ss;
    ss << f.rdbuf();
    SceneModel s;
    if (parse_scene(ss.str(), s) != kParseOk) { std::fprintf(stderr, "parse error\n"); return 1; }
    const int W = argc > 3 ? std::atoi(argv[2]) : 192, H = argc > 3 ? std::atoi(argv[3]) : 108;
    const char *lf = std::getenv("RT_AMD_LEAF");
    const SphereBVH b = build_sphere_bvh(s.spheres, lf ? (uint32_t)std::atoi(lf) : 3u);
    std::vector<float> hot(s.spheres.size() * 4);
    for (size_t i = 0; i < s.spheres.size(); ++i) {
        hot[i * 4] = s.spheres[i].center.x; hot[i * 4 + 1] = s.spheres[i].center.y;
        hot[i * 4 + 2] = s.spheres[i].center.z; hot[i * 4 + 3] = s.spheres[i].radius * s.spheres[i].radius;
    }
    const CameraModel &cm = s.camera;
    const V org{cm.origin.x, cm.origin.y, cm.origin.z};
    uint32_t rng = 2547549u;
    auto rnd = [&]() { rng ^= rng << 13; rng ^= rng >> 17; rng ^= rng << 5; return rng * 0x1p-32; };
    std::vector<int> vis[3];  // bounce 0, 1, 2
    const bool bvh4 = std::getenv("SIM_BVH4") != nullptr;
    std::vector<int> box4[3];  // SIM_BVH4: children tested per walk
    for (int j = 0; j < H; ++j)
        for (int i = 0; i < W; ++i) {
            const double u = (i + rnd()) / (W - 1), v = (j + rnd()) / (H - 1);
            V o = org;
            V d = unit(sub(add(add(V{cm.lower_left.x, cm.lower_left.y, cm.lower_left.z},
                                   mul(V{cm.horizontal.x, cm.horizontal.y, cm.horizontal.z}, u)),
                               mul(V{cm.vertical.x, cm.vertical.y, cm.vertical.z}, v)), o));
            for (int bounce = 0; bounce < 3; ++bounce) {
                Hit h;
                if (bvh4) {
                    Hit h2;
                    int tests = 0;
                    vis[bounce].push_back(walk4(b, hot, o, d, h2, &tests));
                    box4[bounce].push_back(tests);
                }
                const int v2 = walk(b, hot, o, d, h);
                if (!bvh4) vis[bounce].push_back(v2);
                if (h.id < 0) break;
                const float *c = &hot[(size_t)h.id * 4];
                const V p = add(o, mul(d, h.t));
                const V n = unit(sub(p, V{c[0], c[1], c[2]}));
                const V r = unit(V{rnd() * 2 - 1, rnd() * 2 - 1, rnd() * 2 - 1});
                o = p;
                d = unit(add(n, r));
            }
        }
    std::printf("nodes %zu leaves<=%s big %zu\n", b.nodes.size() / 8, lf ? lf : "3", b.big.size());
    for (int k = 0; k < 3; ++k) {
        std::vector<int> v = vis[k];
        if (v.empty()) continue;
        double mean = 0;
        for (int x : v) mean += x;
        mean /= v.size();
        // consecutive groups of 64 (neighbouring pixels) and shuffled groups
        double gmax = 0, rmax = 0;
        size_t ng = v.size() / 64;
        for (size_t g = 0; g < ng; ++g) gmax += *std::max_element(v.begin() + g * 64, v.begin() + g * 64 + 64);
        std::vector<int> sh = v;
        for (size_t i = sh.size() - 1; i > 0; --i) std::swap(sh[i], sh[(size_t)(rnd() * (i + 1)) % (i + 1)]);
        for (size_t g = 0; g < ng; ++g) rmax += *std::max_element(sh.begin() + g * 64, sh.begin() + g * 64 + 64);
        if (bvh4 && !box4[k].empty()) {
            double bt = 0, bmax = 0;
            for (int x : box4[k]) bt += x;
            for (size_t g = 0; g < ng; ++g)
                bmax += *std::max_element(box4[k].begin() + g * 64, box4[k].begin() + g * 64 + 64);
            std::printf("bvh4 bounce %d: box tests mean %.1f, E[max of 64] %.1f\n", k, bt / box4[k].size(),
                        ng ? bmax / ng : 0.0);
        }
        std::sort(v.begin(), v.end());
        std::printf("bounce %d: %zu walks, mean %.1f, p50 %d p90 %d p99 %d max %d; E[max of 64] "
                    "neighbours %.1f, shuffled %.1f (lane use %.0f%% / %.0f%%)\n",
                    k, v.size(), mean, v[v.size() / 2], v[v.size() * 9 / 10], v[v.size() * 99 / 100], v.back(),
                    ng ? gmax / ng : 0.0, ng ? rmax / ng : 0.0, ng ? 100 * mean / (gmax / ng) : 0.0,
                    ng ? 100 * mean / (rmax / ng) : 0.0);
    }
}
