// tbvh_sim.cpp -- host emulation of the triangle-BVH traversal (tuning tool).
// Counts node visits and triangle tests per ray for a scene's primary rays and
// for rays from the primary hit points, for any build (RT_AMD_TRI_LEAF etc.).
// Not product code and not a parity check: float arithmetic mirrors the
// kernel's box test; hits use the reference's triangle t (with its sign).
//   g++ -O2 -std=c++17 -I../rust-swift-raytracer_amd/csrc tbvh_sim.cpp \
//       ../rust-swift-raytracer_amd/csrc/{bvh,scene}.cpp -o tbvh_sim
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <fstream>
#include <map>
#include <tuple>
#include <vector>
#include <sstream>

#include "bvh.h"
#include "scene.h"

using namespace rtamd;

struct V { float x, y, z; };
static V sub(V a, V b) { return {a.x - b.x, a.y - b.y, a.z - b.z}; }
static V add(V a, V b) { return {a.x + b.x, a.y + b.y, a.z + b.z}; }
static V mul(V a, float s) { return {a.x * s, a.y * s, a.z * s}; }
static float dot(V a, V b) { return (a.x * b.x + a.y * b.y) + a.z * b.z; }
static V cross(V a, V b) { return {a.y * b.z - a.z * b.y, -(a.x * b.z - a.z * b.x), a.x * b.y - a.y * b.x}; }
static V unit(V a) { float l = std::sqrt(dot(a, a)); return {a.x / l, a.y / l, a.z / l}; }

struct Count { double nodes = 0, tests = 0, rays = 0; };

static bool g_exact = false;  // tree over phantom triangles of one origin (no widening)
static float trace(const TriangleBVH &t, V o, V d, Count &c) {
    c.rays += 1;
    const float onorm = std::fabs(o.x) + std::fabs(o.y) + std::fabs(o.z);
    const float ix = 1.0f / d.x, iy = 1.0f / d.y, iz = 1.0f / d.z;
    const unsigned oct = (ix < 0) | ((iy < 0) << 1) | ((iz < 0) << 2);
    const float dist = std::fabs(o.x - t.centre[0]) + std::fabs(o.y - t.centre[1]) +
                       std::fabs(o.z - t.centre[2]) + t.radius + 2 * onorm;
    const float rho = 1e-5f * (dist + onorm + t.mag);
    float best = INFINITY;
    uint32_t node = 0;
    while (node != kNodeEnd) {
        c.nodes += 1;
        const float *n = &t.nodes[(size_t)node * 16];
        float sl = 0, sh = 0;
        const float ov[3] = {o.x, o.y, o.z}, iv[3] = {ix, iy, iz};
        const float dv[3] = {o.x - t.oc[0], o.y - t.oc[1], o.z - t.oc[2]};
        for (int k = 0; k < 3; ++k) {
            float a = n[8 + k] * dv[k], b = n[12 + k] * dv[k];
            sl += std::fmin(a, b); sh += std::fmax(a, b);
        }
        if (g_exact) sl = sh = 0;
        float tn = -INFINITY, tf = INFINITY;
        for (int k = 0; k < 3; ++k) {
            float a = sl * n[8 + k], b = sl * n[12 + k], cc = sh * n[8 + k], dd = sh * n[12 + k];
            float lo = n[k] + 2 * std::fmin(std::fmin(a, b), std::fmin(cc, dd)) - rho;
            float hi = n[4 + k] + 2 * std::fmax(std::fmax(a, b), std::fmax(cc, dd)) + rho;
            float t0 = (lo - ov[k]) * iv[k], t1 = (hi - ov[k]) * iv[k];
            tn = std::fmax(tn, std::fmin(t0, t1));
            tf = std::fmin(tf, std::fmax(t0, t1));
        }
        uint32_t a, b;
        std::memcpy(&a, &n[3], 4);
        std::memcpy(&b, &n[7], 4);
        const bool skip = tn > tf || tf < 0.001f || tn > best;
        const bool leaf = a & kLeafBit;
        const uint32_t next = (skip || leaf) ? t.miss[(size_t)node * 8 + oct] : a + ((oct >> b) & 1u);
        if (!skip && leaf) {
            for (uint32_t j = a & ~kLeafBit; j < (a & ~kLeafBit) + b; ++j) {
                c.tests += 1;
                const float *r = &t.tris[(size_t)j * 16];
                V N{r[0], r[1], r[2]};
                float cs = dot(N, d);
                if (std::fabs(cs) < 1e-8f) continue;
                float tt = g_exact ? (r[3] - dot(N, o)) / cs : (dot(N, o) + r[3]) / cs;
                if (tt < 0.001f || tt > best) continue;
                V p = add(o, mul(d, tt));
                V v0{r[4], r[5], r[6]}, v1{r[8], r[9], r[10]}, v2{r[12], r[13], r[14]};
                if (dot(N, cross(sub(v1, v0), sub(p, v0))) < 0) continue;
                if (dot(N, cross(sub(v2, v1), sub(p, v1))) < 0) continue;
                if (dot(N, cross(sub(v0, v2), sub(p, v2))) < 0) continue;
                best = tt;
            }
        }
        node = next;
    }
    return best;
}

int main(int argc, char **argv) {
    if (argc < 2) { std::fprintf(stderr, "usage: tbvh_sim scene.txt [W H]\n"); return 2; }
    std::ifstream f(argv[1]);
    std::stringstream ss;
    ss << f.rdbuf();
    SceneModel s;
    if (parse_scene(ss.str(), s) != kParseOk) { std::fprintf(stderr, "parse error\n"); return 1; }
    const int W = argc > 3 ? std::atoi(argv[2]) : 96, H = argc > 3 ? std::atoi(argv[3]) : 54;
    PackedScene p = pack_scene(s, 8, 1);
    const char *lf = std::getenv("RT_AMD_TRI_LEAF");
    TriangleBVH t = build_triangle_bvh(s.triangles, p.tri_hot, lf ? std::atoi(lf) : 4);
    std::printf("tris %zu nodes %zu loose %zu depth %u\n", s.triangles.size(), t.nodes.size() / 16,
                t.loose.size(), t.depth);
    const CameraModel &cm = s.camera;
    if (std::getenv("SIM_EXACT")) {  // phantom triangles of the camera origin
        g_exact = true;
        for (auto &tr : s.triangles) {
            double n[3] = {tr.normal.x, tr.normal.y, tr.normal.z};
            double nn = std::sqrt(n[0] * n[0] + n[1] * n[1] + n[2] * n[2]);
            double sdot = (n[0] * cm.origin.x + n[1] * cm.origin.y + n[2] * cm.origin.z) / nn;
            Vec3 *vs[3] = {&tr.v0, &tr.v1, &tr.v2};
            for (Vec3 *v : vs) {
                v->x += (float)(2 * sdot * n[0] / nn);
                v->y += (float)(2 * sdot * n[1] / nn);
                v->z += (float)(2 * sdot * n[2] / nn);
            }
        }
        p = pack_scene(s, 8, 1);
        t = build_triangle_bvh(s.triangles, p.tri_hot, lf ? std::atoi(lf) : 4);
        std::printf("exact phantom tree: nodes %zu\n", t.nodes.size() / 16);
    }
    V org{cm.origin.x, cm.origin.y, cm.origin.z};
    Count prim, sec;
    uint32_t rng = 2547549u;
    auto rnd = [&]() { rng ^= rng << 13; rng ^= rng >> 17; rng ^= rng << 5; return rng * 0x1p-32f; };
    int hits = 0;
    for (int j = 0; j < H; ++j)
        for (int i = 0; i < W; ++i) {
            float u = (i + 0.5f) / W, v = (j + 0.5f) / H;
            V d = unit(sub(add(add(V{cm.lower_left.x, cm.lower_left.y, cm.lower_left.z},
                                   mul(V{cm.horizontal.x, cm.horizontal.y, cm.horizontal.z}, u)),
                               mul(V{cm.vertical.x, cm.vertical.y, cm.vertical.z}, v)), org));
            float tt = trace(t, org, d, prim);
            if (std::isfinite(tt)) {
                ++hits;
                V o2 = add(org, mul(d, tt));
                V d2 = unit(V{rnd() * 2 - 1, rnd() * 2 - 1, rnd() * 2 - 1});
                trace(t, o2, d2, sec);
            }
        }
    if (const char *cs = std::getenv("SIM_CELL")) {  // per-cell trees for the secondary rays
        const float S = std::atof(cs);
        // secondary origins: the primary hit points (recomputed)
        std::vector<V> o2s, d2s;
        uint32_t rng2 = 2547549u;
        auto rnd2 = [&]() { rng2 ^= rng2 << 13; rng2 ^= rng2 >> 17; rng2 ^= rng2 << 5; return rng2 * 0x1p-32f; };
        Count dummy;
        for (int j = 0; j < H; ++j)
            for (int i = 0; i < W; ++i) {
                float u = (i + 0.5f) / W, v = (j + 0.5f) / H;
                V d = unit(sub(add(add(V{cm.lower_left.x, cm.lower_left.y, cm.lower_left.z},
                                       mul(V{cm.horizontal.x, cm.horizontal.y, cm.horizontal.z}, u)),
                                   mul(V{cm.vertical.x, cm.vertical.y, cm.vertical.z}, v)), org));
                float tt = trace(t, org, d, dummy);
                if (std::isfinite(tt)) {
                    o2s.push_back(add(org, mul(d, tt)));
                    d2s.push_back(unit(V{rnd2() * 2 - 1, rnd2() * 2 - 1, rnd2() * 2 - 1}));
                }
            }
        std::map<std::tuple<int, int, int>, TriangleBVH> trees;
        Count cell;
        for (size_t r = 0; r < o2s.size(); ++r) {
            V o2 = o2s[r];
            auto key = std::make_tuple((int)std::floor(o2.x / S), (int)std::floor(o2.y / S), (int)std::floor(o2.z / S));
            auto it = trees.find(key);
            if (it == trees.end()) {
                float oc[3] = {(std::get<0>(key) + 0.5f) * S, (std::get<1>(key) + 0.5f) * S, (std::get<2>(key) + 0.5f) * S};
                it = trees.emplace(key, build_triangle_bvh(s.triangles, p.tri_hot, lf ? std::atoi(lf) : 4, oc, S * 0.866)).first;
            }
            trace(it->second, o2, d2s[r], cell);
        }
        std::printf("cells S=%g: %zu trees, secondary %.1f nodes/ray, %.1f tests/ray\n", S, trees.size(),
                    cell.nodes / cell.rays, cell.tests / cell.rays);
    }
    std::printf("primary: %.0f rays, %.1f nodes/ray, %.1f tests/ray, hit %.3f\n", prim.rays,
                prim.nodes / prim.rays, prim.tests / prim.rays, hits / prim.rays);
    if (sec.rays)
        std::printf("secondary: %.0f rays, %.1f nodes/ray, %.1f tests/ray\n", sec.rays,
                    sec.nodes / sec.rays, sec.tests / sec.rays);
}
