// bvh_check.cpp -- host-side structural checks of the BVH builders (CPU test
// driver for tests/test_bvh_host.py; compiled with g++ against csrc/bvh.cpp).
// Checks, for the sphere tree, the static triangle tree and the camera tree:
//   * every primitive sits in exactly one leaf, leaves within limits;
//   * every node's float box contains its children's boxes and its prims;
//   * octant links: each link is a valid node index or the end marker, and a
//     full walk entering every node visits each node exactly once per octant;
//   * quantised kernel nodes decode (fmaf(q, step, base)) to boxes containing
//     the float boxes, and the packed child/axis/leaf words round-trip.
// Prints "OK <counts>" or the first failure and exits non-zero.
#include <algorithm>
#include <cmath>
#include <cstdlib>
#include <cstdio>
#include <cstring>
#include <map>
#include <fstream>
#include <sstream>
#include <vector>

#include "bvh.h"
#include "scene.h"

using namespace rtamd;

static int fails = 0;
#define CHECK(c, ...)                                   \
    do {                                                \
        if (!(c)) {                                     \
            if (fails++ < 10) std::printf(__VA_ARGS__); \
        }                                               \
    } while (0)

static uint32_t bits(float f) { uint32_t u; std::memcpy(&u, &f, 4); return u; }

// nodes: stride floats, (min, a) (max, b); walk with links, every node entered
static void check_links(const std::vector<float> &nodes, size_t stride, const std::vector<uint32_t> &miss,
                        const char *what) {
    const size_t n = nodes.size() / stride;
    for (uint32_t oct = 0; oct < 8; ++oct) {
        std::vector<int> seen(n, 0);
        uint32_t node = 0;
        size_t steps = 0;
        while (node != kNodeEnd && steps++ <= n) {
            CHECK(node < n, "%s: link out of range\n", what);
            if (node >= n) return;
            seen[node]++;
            const uint32_t a = bits(nodes[node * stride + 3]), b = bits(nodes[node * stride + 7]);
            node = (a & kLeafBit) ? miss[node * 8 + oct] : a + ((oct >> b) & 1u);
        }
        for (size_t i = 0; i < n; ++i) CHECK(seen[i] == 1, "%s: node %zu seen %d times (oct %u)\n", what, i, seen[i], oct);
    }
}

static void check_tree(const std::vector<float> &nodes, size_t stride, size_t nprims, uint32_t maxleaf,
                       const char *what) {
    const size_t n = nodes.size() / stride;
    std::vector<int> owner(nprims, 0);
    for (size_t i = 0; i < n; ++i) {
        const float *f = &nodes[i * stride];
        const uint32_t a = bits(f[3]), b = bits(f[7]);
        for (int k = 0; k < 3; ++k) CHECK(f[k] <= f[4 + k], "%s: node %zu inverted box\n", what, i);
        if (a & kLeafBit) {
            const uint32_t first = a & ~kLeafBit;
            CHECK(b >= 1 && b <= maxleaf, "%s: leaf %zu count %u\n", what, i, b);
            for (uint32_t j = first; j < first + b && j < nprims; ++j) owner[j]++;
        } else {
            CHECK(a + 1 < n && b < 3, "%s: node %zu child %u axis %u\n", what, i, a, b);
            for (uint32_t c = a; c <= a + 1 && c + 1 <= n; ++c)
                for (int k = 0; k < 3; ++k) {
                    CHECK(nodes[c * stride + k] >= f[k] && nodes[c * stride + 4 + k] <= f[4 + k],
                          "%s: child %u box not inside parent %zu\n", what, c, i);
                    if (stride == 16)
                        CHECK(nodes[c * stride + 8 + k] >= f[8 + k] && nodes[c * stride + 12 + k] <= f[12 + k],
                              "%s: child %u normal box not inside parent %zu\n", what, c, i);
                }
        }
    }
    for (size_t j = 0; j < nprims; ++j) CHECK(owner[j] == 1, "%s: prim %zu in %d leaves\n", what, j, owner[j]);
}

static void check_quant(const std::vector<float> &nodes, size_t stride, const std::vector<uint32_t> &q,
                        const std::vector<uint32_t> &miss, const QuantGrid &g, float nb, float ns,
                        const char *what) {
    const size_t n = nodes.size() / stride, words = 8;
    CHECK(q.size() == n * words, "%s: qnodes size\n", what);
    auto dec = [](uint32_t v, float s, float b) { return std::fmaf((float)v, s, b); };
    for (size_t i = 0; i < n && q.size() == n * words; ++i) {
        const float *f = &nodes[i * stride];
        const uint32_t *w = &q[i * words];
        const uint32_t u[6] = {w[0] & 0xFFFF, w[0] >> 16, w[1] & 0xFFFF, w[1] >> 16, w[2] & 0xFFFF, w[2] >> 16};
        for (int k = 0; k < 3; ++k) {
            CHECK(dec(u[k], g.step[k], g.base[k]) <= f[k], "%s: node %zu lo %d not conservative\n", what, i, k);
            CHECK(dec(u[3 + k], g.step[k], g.base[k]) >= f[4 + k], "%s: node %zu hi %d not conservative\n", what, i, k);
            // and tight: within 2 grid steps
            CHECK(f[k] - dec(u[k], g.step[k], g.base[k]) <= 2 * g.step[k], "%s: node %zu lo %d loose\n", what, i, k);
        }
        if (stride == 16) {
            const uint32_t m[6] = {w[3] & 0xFFFF, w[3] >> 16, w[4] & 0xFFFF, w[4] >> 16, w[5] & 0xFFFF, w[5] >> 16};
            for (int k = 0; k < 3; ++k) {
                CHECK(dec(m[k], ns, nb) <= f[8 + k], "%s: node %zu nlo %d\n", what, i, k);
                CHECK(dec(m[3 + k], ns, nb) >= f[12 + k], "%s: node %zu nhi %d\n", what, i, k);
            }
        }
        const uint32_t a = bits(f[3]), b = bits(f[7]), word = w[stride == 16 ? 6 : 3];
        CHECK(w[stride == 16 ? 7 : 4] == miss[i * 8], "%s: link word %zu\n", what, i);
        if (a & kLeafBit)
            CHECK(word == (kLeafBit | ((a & ~kLeafBit) << 3) | b), "%s: leaf word %zu\n", what, i);
        else
            CHECK((word & 0x1FFFFFFFu) == a && (word >> 29) == b, "%s: internal word %zu\n", what, i);
    }
}

// The 4-wide image (bvh.h TriangleBVH::wnodes): a walk of every slot reaches
// each wide node once and each binary leaf's word once, every child's box
// words are a binary node's, and the stack bound holds (3 * wdepth).
static void check_wide(const TriangleBVH &tb) {
    const size_t nw = tb.wnodes.size() / 32, nq = tb.qnodes.size() / 8;
    CHECK(nw > 0 && tb.wnodes.size() == nw * 32 && nw <= 65535, "wide: %zu records\n", nw);
    if (nw == 0) return;
    std::vector<int> seen(nw, 0);
    std::map<uint32_t, int> leaves;
    std::map<std::vector<uint32_t>, std::vector<uint32_t>> words;  // box words 0-2 -> binary nodes
    for (size_t i = 0; i < nq; ++i) {
        const uint32_t *q = &tb.qnodes[i * 8];
        words[std::vector<uint32_t>(q, q + 3)].push_back((uint32_t)i);
    }
    auto half = [](uint32_t h) {
        const int e = (h >> 10) & 31, m = h & 1023;
        const float v = e == 0 ? std::ldexp((float)m, -24) : std::ldexp((float)(1024 + m), e - 25);
        return (h & 0x8000) ? -v : v;
    };
    std::vector<std::pair<uint32_t, uint32_t>> st{{0u, 0u}};  // (wide node, depth)
    size_t maxstack = 0;
    while (!st.empty()) {
        const auto [w, dpt] = st.back();
        st.pop_back();
        CHECK(w < nw, "wide: index %u out of range\n", w);
        if (w >= nw) return;
        seen[w]++;
        CHECK(dpt <= tb.wdepth, "wide: node %u deeper (%u) than wdepth %u\n", w, dpt, tb.wdepth);
        const uint32_t *r = &tb.wnodes[(size_t)w * 32];
        size_t pushed = 0;
        for (int c = 0; c < 4; ++c) {
            const uint32_t a = r[24 + c];
            if (a == kLeafBit) continue;  // empty slot
            // the slot's words are some binary node's words 0-5 (and its leaf word)
            // the slot is some binary node: its box words, its leaf word, and
            // halves that contain its float normal box
            bool found = false;
            auto it = words.find(std::vector<uint32_t>(r + 6 * c, r + 6 * c + 3));
            if (it != words.end())
                for (uint32_t i : it->second) {
                    const uint32_t qa = tb.qnodes[(size_t)i * 8 + 6];
                    if ((a & kLeafBit) ? qa != a : (qa & kLeafBit) != 0) continue;
                    const float *f = &tb.nodes[(size_t)i * 16];
                    const uint32_t *h = r + 6 * c + 3;
                    const float lo[3] = {half(h[0] & 0xFFFF), half(h[0] >> 16), half(h[1] & 0xFFFF)};
                    const float hi[3] = {half(h[1] >> 16), half(h[2] & 0xFFFF), half(h[2] >> 16)};
                    bool in = true;
                    for (int k = 0; k < 3; ++k) in = in && lo[k] <= f[8 + k] && hi[k] >= f[12 + k] &&
                                                   hi[k] - lo[k] <= f[12 + k] - f[8 + k] + 2e-3f;
                    found = found || in;
                }
            CHECK(found, "wide: node %u slot %d is no binary node\n", w, c);
            if (a & kLeafBit) {
                leaves[a]++;
            } else {
                st.push_back({a, dpt + 1});
                ++pushed;
            }
        }
        maxstack = std::max(maxstack, st.size());
        (void)pushed;
    }
    for (size_t i = 0; i < nw; ++i) CHECK(seen[i] == 1, "wide: node %zu reached %d times\n", i, seen[i]);
    size_t nleaf = 0;
    for (size_t i = 0; i < nq; ++i)
        if (tb.qnodes[i * 8 + 6] & kLeafBit) {
            ++nleaf;
            CHECK(leaves[tb.qnodes[i * 8 + 6]] == 1, "wide: leaf %zu reached %d times\n", i,
                  leaves[tb.qnodes[i * 8 + 6]]);
        }
    CHECK(leaves.size() == nleaf, "wide: %zu leaf words, %zu binary leaves\n", leaves.size(), nleaf);
}

// Per-origin-cell trees (bvh.h TriangleCells, argv[3] = starting cell edge):
// the grid covers the mesh and the spheres no larger than it, the image holds
// ncells + 1 trees of stride_w wide nodes with the static tree last (equal to
// the re-quantised tb), the records begin with the static tree's, and every
// tree's walk reaches each of its wide nodes once and each tree triangle in
// exactly one leaf.
static void check_cells(const SceneModel &s, const TriangleCells &tc, const TriangleBVH &tb) {
    CHECK(tc.ncells == tc.n[0] * tc.n[1] * tc.n[2] && tc.ncells > 0, "cells: %u != grid\n", tc.ncells);
    CHECK(tc.ncells <= 1024, "cells: %u > 1024\n", tc.ncells);
    const size_t sw = tc.stride_w;
    CHECK(tc.wnodes.size() == (size_t)(tc.ncells + 1) * sw * 32, "cells: image size\n");
    double lo[3] = {INFINITY, INFINITY, INFINITY}, hi[3] = {-INFINITY, -INFINITY, -INFINITY}, ext = 0;
    for (const Triangle &t : s.triangles)
        for (const Vec3 &v : {t.v0, t.v1, t.v2}) {
            const double c[3] = {v.x, v.y, v.z};
            for (int k = 0; k < 3; ++k) { lo[k] = std::min(lo[k], c[k]); hi[k] = std::max(hi[k], c[k]); }
        }
    for (int k = 0; k < 3; ++k) ext = std::max(ext, hi[k] - lo[k]);
    for (const Sphere &sp : s.spheres) {
        const double r = std::fabs((double)sp.radius), c[3] = {sp.center.x, sp.center.y, sp.center.z};
        if (!(r <= ext)) continue;
        for (int k = 0; k < 3; ++k) { lo[k] = std::min(lo[k], c[k] - r); hi[k] = std::max(hi[k], c[k] + r); }
    }
    for (int k = 0; k < 3; ++k)
        CHECK(tc.lo[k] <= lo[k] + 1e-6 * (1 + std::fabs(lo[k])) && tc.lo[k] + (double)tc.n[k] * tc.size >= hi[k] - 1e-4,
              "cells: axis %d [%g, %g] not covered\n", k, lo[k], hi[k]);
    CHECK(std::equal(tb.wnodes.begin(), tb.wnodes.end(), tc.wnodes.begin() + (size_t)tc.ncells * sw * 32),
          "cells: static slot differs from tb\n");
    CHECK(tc.tris.size() >= tb.tris.size() && std::equal(tb.tris.begin(), tb.tris.end(), tc.tris.begin()),
          "cells: records do not begin with the static tree's\n");
    std::vector<int> want(s.triangles.size(), 0);
    for (size_t j = 0; j < tb.tris.size() / 16; ++j) {
        uint32_t id;
        std::memcpy(&id, &tb.tris[j * 16 + 7], 4);
        want[id]++;
    }
    for (uint32_t c = 0; c <= tc.ncells; ++c) {
        const uint32_t *img = &tc.wnodes[(size_t)c * sw * 32];
        std::vector<int> seen(sw, 0), got(s.triangles.size(), 0);
        std::vector<uint32_t> st{0u};
        while (!st.empty()) {
            const uint32_t w = st.back();
            st.pop_back();
            CHECK(w < sw, "cells: tree %u node %u out of range\n", c, w);
            if (w >= sw) return;
            seen[w]++;
            for (int k = 0; k < 4; ++k) {
                const uint32_t a = img[(size_t)w * 32 + 24 + k];
                if (!(a & kLeafBit)) { st.push_back(a); continue; }
                const uint32_t first = (a & ~kLeafBit) >> 3, count = a & 7u;
                CHECK((size_t)(first + count) * 16 <= tc.tris.size(), "cells: tree %u leaf past records\n", c);
                for (uint32_t j = first; j < first + count && (size_t)(j + 1) * 16 <= tc.tris.size(); ++j) {
                    uint32_t id;
                    std::memcpy(&id, &tc.tris[(size_t)j * 16 + 7], 4);
                    if (id < got.size()) got[id]++;
                }
            }
        }
        size_t nreached = 0;
        for (size_t w = 0; w < sw; ++w) {
            CHECK(seen[w] <= 1, "cells: tree %u node %zu reached %d times\n", c, w, seen[w]);
            nreached += seen[w];
        }
        CHECK(got == want, "cells: tree %u does not hold every tree triangle once\n", c);
        if (fails) return;
    }
}

int main(int argc, char **argv) {
    std::ifstream fh(argv[1]);
    std::stringstream ss;
    ss << fh.rdbuf();
    SceneModel s;
    if (parse_scene(ss.str(), s) != kParseOk) { std::printf("parse error\n"); return 2; }
    PackedScene p = pack_scene(s, 8, 1);
    const uint32_t leaf = argc > 2 ? (uint32_t)std::atoi(argv[2]) : 2;
    SphereBVH sb = build_sphere_bvh(s.spheres, 3);
    if (!sb.nodes.empty()) {
        check_tree(sb.nodes, 8, sb.prim_id.size(), 3, "sphere");
        check_links(sb.nodes, 8, sb.miss, "sphere");
    }
    TriangleBVH tb = build_triangle_bvh(s.triangles, p.tri_hot, leaf);
    CameraTriangleBVH cb;
    if (!tb.nodes.empty()) {
        check_tree(tb.nodes, 16, tb.tris.size() / 16, leaf, "static");
        check_links(tb.nodes, 16, tb.miss, "static");
        check_quant(tb.nodes, 16, tb.qnodes, tb.miss, tb.qbox, tb.nbase, tb.nstep, "static");
        check_wide(tb);
        const float o[3] = {s.camera.origin.x, s.camera.origin.y, s.camera.origin.z};
        cb = build_camera_triangle_bvh(s.triangles, p.tri_hot, tb, o, leaf);
        check_tree(cb.nodes, 8, cb.tris.size() / 16, leaf, "camera");
        check_links(cb.nodes, 8, cb.miss, "camera");
        check_quant(cb.nodes, 8, cb.qnodes, cb.miss, cb.qbox, 0, 1, "camera");
        CHECK(cb.tris.size() == tb.tris.size(), "camera tree holds %zu records, static %zu\n",
              cb.tris.size() / 16, tb.tris.size() / 16);
    }
    // every triangle is in the tree, brute-forced (loose) or degenerate (n = 0)
    size_t in_tree = tb.tris.size() / 16, degenerate = 0;
    for (size_t i = 0; i < s.triangles.size(); ++i) {
        const float *h = &p.tri_hot[i * 4];
        if (h[0] == 0 && h[1] == 0 && h[2] == 0) ++degenerate;
    }
    if (!tb.nodes.empty())
        CHECK(in_tree + tb.loose.size() + degenerate >= s.triangles.size(),
              "triangles lost: %zu tree + %zu loose + %zu degenerate < %zu\n", in_tree, tb.loose.size(),
              degenerate, s.triangles.size());
    size_t ncells = 0;
    if (argc > 3 && !tb.nodes.empty()) {
        TriangleBVH tb2 = tb;
        const TriangleCells tc = build_triangle_cells(s.triangles, p.tri_hot, s.spheres, leaf,
                                                      (float)std::atof(argv[3]), tb2);
        ncells = tc.ncells;
        if (ncells) check_cells(s, tc, tb2);
        else CHECK(false, "cells: none built\n");
        std::printf("cells %zu\n", ncells);
    }
    if (fails) return 1;
    std::printf("OK spheres %zu nodes %zu | triangles %zu tree %zu loose %zu nodes %zu camera nodes %zu\n",
                s.spheres.size(), sb.nodes.size() / 8, s.triangles.size(), in_tree, tb.loose.size(),
                tb.nodes.size() / 16, cb.nodes.size() / 8);
    return 0;
}
