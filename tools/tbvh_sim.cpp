// tbvh_sim.cpp -- host emulation of the triangle-BVH traversal (tuning tool).
// Counts node visits and triangle tests per ray for a scene's primary rays and
// for rays from the primary hit points, for any build (RT_AMD_TRI_LEAF etc.),
// walking the kernel image (qnodes) of the static tree.  (A DFS-preorder
// image with implicit first children measured 4 % slower on the GPU than the
// builder layout, whose sibling pairs and top levels sit together.)
// Not product code and not a parity check: float arithmetic mirrors the
// kernel's box test; hits use the reference's triangle t (with its sign).
// Experiments:
//   SIM_OC=x,y,z[,L]  static tree built for origin (x,y,z) [SAH phantom scale L]
//   SIM_CELL=S        one tree per S-unit cell of the secondary-ray origins
//   SIM_HYB=D,S       the static topology with per-cell boxes (phantoms at the
//                     cell centre, widened per ray from it) for depth < D
//   SIM_HYB_RANGE=1   ... boxes over the whole cell instead (no widening)
//   SIM_LEVELS=1      share of visits per tree level
//   SIM_BIN=P         secondary rays of P-ray pools, waves in arrival order vs
//                     binned by octant + origin cell (SIM_BIN_KEY, SIM_BIN_CELL)
//   SIM_WIDE=K        the tree collapsed to K-wide nodes, walked with a stack:
//                     fetches (dependent node loads) vs box tests per ray
//                     (SIM_WIDE_LEVEL=1: grandchildren, as bvh.cpp builds it;
//                     SIM_WIDE_ORDER=0: children in slot order, not nearest-first)
//   SIM_Q8=B,N        16-B nodes in DFS preorder: N>0 u8 boxes and normal boxes
//                     on per-block frames (B nodes per block; N=3 per-axis
//                     normal frames), N=0 u16 boxes with one normal box per
//                     block, N=-1 global grids of SIM_G=box_bits,normal_bits
//   g++ -O2 -std=c++17 -I../rust-swift-raytracer_amd/csrc tbvh_sim.cpp \
//       ../rust-swift-raytracer_amd/csrc/{bvh,scene}.cpp -o tbvh_sim
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <fstream>
#include <map>
#include <functional>
#include <algorithm>
#include <tuple>
#include <vector>
#include <limits>
#include <memory>
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
static std::vector<int> g_depth;          // node depth (kernel image), for SIM_LEVELS
static std::vector<double> g_level_visits;

static bool g_exact = false;
static std::vector<uint32_t> *g_visits = nullptr;  // SIM_WAVE: the nodes a ray visits, in order
static int g_hyb_D = 0;                       // SIM_HYB=D,S: per-cell boxes for depth < D
static const std::vector<float> *g_cellbox = nullptr;  // 6 per node (lo, hi) for this ray's cell
static double g_hyb_hits = 0;
static float g_coc[3];
static bool g_hyb_range = false;  // SIM_HYB_RANGE=1: boxes over the whole cell, no widening  // tree over phantom triangles of one origin (no widening)

// Walks the kernel image (bvh.h qnodes: builder layout, fixed child-a-first
// order, one link per node) with the kernel's box arithmetic.
static float trace(const TriangleBVH &t, V o, V d, Count &c) {
    c.rays += 1;
    const float onorm = std::fabs(o.x) + std::fabs(o.y) + std::fabs(o.z);
    const float iv[3] = {1.0f / d.x, 1.0f / d.y, 1.0f / d.z};
    const float dist = std::fabs(o.x - t.centre[0]) + std::fabs(o.y - t.centre[1]) +
                       std::fabs(o.z - t.centre[2]) + t.radius + 2 * onorm;
    const float rho = 1e-5f * (dist + onorm + t.mag);
    const float ov[3] = {o.x, o.y, o.z};
    const float dv[3] = {o.x - t.oc[0], o.y - t.oc[1], o.z - t.oc[2]};
    auto dec = [](uint32_t q, float s, float b) { return std::fmaf((float)q, s, b); };
    float best = INFINITY;
    uint32_t node = 0;
    while (node != kNodeEnd) {
        c.nodes += 1;
        if (g_visits) g_visits->push_back(node);
        if (!g_depth.empty()) g_level_visits[g_depth[node]] += 1;
        const uint32_t *w = &t.qnodes[(size_t)node * 8];
        const uint32_t u[6] = {w[0] & 0xFFFF, w[0] >> 16, w[1] & 0xFFFF, w[1] >> 16, w[2] & 0xFFFF, w[2] >> 16};
        const uint32_t m[6] = {w[3] & 0xFFFF, w[3] >> 16, w[4] & 0xFFFF, w[4] >> 16, w[5] & 0xFFFF, w[5] >> 16};
        float sl = 0, sh = 0, n0[3], n1[3];
        for (int k = 0; k < 3; ++k) {
            n0[k] = g_exact ? 0 : dec(m[k], t.nstep, t.nbase);
            n1[k] = g_exact ? 0 : dec(m[3 + k], t.nstep, t.nbase);
            float a = n0[k] * dv[k], b = n1[k] * dv[k];
            sl += std::fmin(a, b); sh += std::fmax(a, b);
        }
        float tn = -INFINITY, tf = INFINITY;
        if (g_cellbox && g_depth[node] < g_hyb_D) {
            g_hyb_hits += 1;
            const float *cb = &(*g_cellbox)[(size_t)node * 6];
            float csl = 0, csh = 0;
            for (int k = 0; k < 3 && !g_hyb_range; ++k) {
                float a = n0[k] * (ov[k] - g_coc[k]), b = n1[k] * (ov[k] - g_coc[k]);
                csl += std::fmin(a, b); csh += std::fmax(a, b);
            }
            for (int k = 0; k < 3; ++k) {
                float a = csl * n0[k], b = csl * n1[k], cc = csh * n0[k], dd = csh * n1[k];
                float lo = cb[k] + 2 * std::fmin(std::fmin(a, b), std::fmin(cc, dd)) - rho;
                float hi = cb[3 + k] + 2 * std::fmax(std::fmax(a, b), std::fmax(cc, dd)) + rho;
                float t0 = (lo - ov[k]) * iv[k], t1 = (hi - ov[k]) * iv[k];
                tn = std::fmax(tn, std::fmin(t0, t1));
                tf = std::fmin(tf, std::fmax(t0, t1));
            }
        } else
        for (int k = 0; k < 3; ++k) {
            float a = sl * n0[k], b = sl * n1[k], cc = sh * n0[k], dd = sh * n1[k];
            float lo = dec(u[k], t.qbox.step[k], t.qbox.base[k]) + 2 * std::fmin(std::fmin(a, b), std::fmin(cc, dd)) - rho;
            float hi = dec(u[3 + k], t.qbox.step[k], t.qbox.base[k]) + 2 * std::fmax(std::fmax(a, b), std::fmax(cc, dd)) + rho;
            float t0 = (lo - ov[k]) * iv[k], t1 = (hi - ov[k]) * iv[k];
            tn = std::fmax(tn, std::fmin(t0, t1));
            tf = std::fmin(tf, std::fmax(t0, t1));
        }
        const uint32_t a = w[6], link = w[7];
        const bool skip = tn > tf || tf < 0.001f || tn > best;
        const bool leaf = a & kLeafBit;
        const uint32_t next = (skip || leaf) ? link : (a & 0x1FFFFFFFu);
        if (!skip && leaf) {
            const uint32_t first = (a & ~kLeafBit) >> 3, count = a & 7u;
            for (uint32_t j = first; j < first + count; ++j) {
                c.tests += 1;
                const float *r = &t.tris[(size_t)j * 16];
                V N{r[0], r[1], r[2]};
                float cs = dot(N, d);
                if (std::fabs(cs) < 1e-8f) continue;
                float tt = g_exact ? (r[3] - dot(N, o)) / cs : (dot(N, o) + r[3]) / cs;
                if (tt < 0.001f || tt > best) continue;
                V pp = add(o, mul(d, tt));
                V v0{r[4], r[5], r[6]}, v1{r[8], r[9], r[10]}, v2{r[12], r[13], r[14]};
                if (dot(N, cross(sub(v1, v0), sub(pp, v0))) < 0) continue;
                if (dot(N, cross(sub(v2, v1), sub(pp, v1))) < 0) continue;
                if (dot(N, cross(sub(v0, v2), sub(pp, v2))) < 0) continue;
                best = tt;
            }
        }
        node = next;
    }
    return best;
}

// SIM_WIDE=K: the static tree collapsed to K-wide nodes (each node's K child
// boxes fetched together: one dependent round trip per node), walked with a
// per-ray stack, hit children nearest-first, leaves tested as their box is hit.
// Child boxes are the binary image's (same decode and widening arithmetic).
struct Wide {
    std::vector<std::vector<uint32_t>> kids;  // per binary node index: its wide children
};
static float qarea(const TriangleBVH &t, uint32_t n) {
    const uint32_t *w = &t.qnodes[(size_t)n * 8];
    float e[3];
    for (int k = 0; k < 3; ++k) {
        const uint32_t lo = (w[k] & 0xFFFF), hi = w[k] >> 16;
        (void)lo; (void)hi;
    }
    const uint32_t u[6] = {w[0] & 0xFFFF, w[0] >> 16, w[1] & 0xFFFF, w[1] >> 16, w[2] & 0xFFFF, w[2] >> 16};
    for (int k = 0; k < 3; ++k) e[k] = (float)(u[3 + k] - u[k]) * t.qbox.step[k];
    return e[0] * e[1] + e[1] * e[2] + e[0] * e[2];
}
static Wide make_wide(const TriangleBVH &t, int K) {
    Wide W;
    const size_t n = t.qnodes.size() / 8;
    W.kids.resize(n);
    for (size_t i = 0; i < n; ++i) {
        const uint32_t a = t.qnodes[i * 8 + 6];
        if (a & kLeafBit) continue;
        std::vector<uint32_t> k{a & 0x1FFFFFFFu, (a & 0x1FFFFFFFu) + 1};
        static const bool level = std::getenv("SIM_WIDE_LEVEL") != nullptr;  // grandchildren, not largest-area
        while ((int)k.size() < K) {
            int best = -1;
            float ba = -1;
            for (size_t j = 0; j < k.size(); ++j) {
                if (t.qnodes[(size_t)k[j] * 8 + 6] & kLeafBit) continue;
                if (level && j >= 2) break;
                const float ar = level ? 1.0f : qarea(t, k[j]);
                if (ar > ba) { ba = ar; best = (int)j; }
            }
            if (best < 0) break;
            const uint32_t c = t.qnodes[(size_t)k[best] * 8 + 6] & 0x1FFFFFFFu;
            k.erase(k.begin() + best);
            k.push_back(c);
            k.push_back(c + 1);
        }
        W.kids[i] = k;
    }
    // wide nodes reachable from the root, their depth, the stack bound
    std::vector<std::pair<uint32_t, int>> st{{0u, 0}};
    size_t nw = 0;
    int maxd = 0;
    while (!st.empty()) {
        auto [i, dd] = st.back();
        st.pop_back();
        ++nw;
        maxd = std::max(maxd, dd);
        for (uint32_t c : W.kids[i])
            if (!(t.qnodes[(size_t)c * 8 + 6] & kLeafBit)) st.push_back({c, dd + 1});
    }
    std::printf("wide K=%d: %zu wide nodes, max depth %d (stack bound %d)\n", K, nw, maxd, (K - 1) * maxd);
    return W;
}
struct WideCount { double fetches = 0, boxes = 0, tests = 0, rays = 0, maxstack = 0, pops = 0; };
static float trace_wide(const TriangleBVH &t, const Wide &W, V o, V d, WideCount &c) {
    c.rays += 1;
    const float onorm = std::fabs(o.x) + std::fabs(o.y) + std::fabs(o.z);
    const float iv[3] = {1.0f / d.x, 1.0f / d.y, 1.0f / d.z};
    const float dist = std::fabs(o.x - t.centre[0]) + std::fabs(o.y - t.centre[1]) +
                       std::fabs(o.z - t.centre[2]) + t.radius + 2 * onorm;
    const float rho = 1e-5f * (dist + onorm + t.mag);
    const float ov[3] = {o.x, o.y, o.z};
    const float dv[3] = {o.x - t.oc[0], o.y - t.oc[1], o.z - t.oc[2]};
    auto dec = [](uint32_t q, float s, float b) { return std::fmaf((float)q, s, b); };
    // SIM_WIDE_SHARED_N=1: every child of a wide node is widened with the
    // union of the children's normal boxes (one widening per fetch)
    static const bool shared_n = std::getenv("SIM_WIDE_SHARED_N") != nullptr;
    uint32_t shared_m[6] = {0, 0, 0, 0, 0, 0};
    bool use_shared = false;
    auto box = [&](uint32_t node, float &tn, float &tf) {
        const uint32_t *w = &t.qnodes[(size_t)node * 8];
        const uint32_t u[6] = {w[0] & 0xFFFF, w[0] >> 16, w[1] & 0xFFFF, w[1] >> 16, w[2] & 0xFFFF, w[2] >> 16};
        uint32_t m[6] = {w[3] & 0xFFFF, w[3] >> 16, w[4] & 0xFFFF, w[4] >> 16, w[5] & 0xFFFF, w[5] >> 16};
        if (use_shared)
            for (int k = 0; k < 6; ++k) m[k] = shared_m[k];
        float sl = 0, sh = 0, n0[3], n1[3];
        for (int k = 0; k < 3; ++k) {
            n0[k] = dec(m[k], t.nstep, t.nbase);
            n1[k] = dec(m[3 + k], t.nstep, t.nbase);
            float a = n0[k] * dv[k], b = n1[k] * dv[k];
            sl += std::fmin(a, b); sh += std::fmax(a, b);
        }
        tn = -INFINITY; tf = INFINITY;
        // SIM_WIDE_SYM=1: symmetric widening 2 S max|m_k|, S = sum_k max|m d_k| >= |s|
        static const bool sym = std::getenv("SIM_WIDE_SYM") != nullptr;
        float S = 0;
        for (int k = 0; k < 3; ++k) S += std::fmax(std::fabs(n0[k] * dv[k]), std::fabs(n1[k] * dv[k]));
        for (int k = 0; k < 3; ++k) {
            float a = sl * n0[k], b = sl * n1[k], cc = sh * n0[k], dd = sh * n1[k];
            float wl = std::fmin(std::fmin(a, b), std::fmin(cc, dd)), wh = std::fmax(std::fmax(a, b), std::fmax(cc, dd));
            if (sym) { wh = S * std::fmax(std::fabs(n0[k]), std::fabs(n1[k])); wl = -wh; }
            // SIM_WIDE_MR=1: midpoint-radius enclosure of [sl, sh] x [n0, n1]
            static const bool mr = std::getenv("SIM_WIDE_MR") != nullptr;
            if (mr) {
                const float sc = 0.5f * (sl + sh), sr = 0.5f * (sh - sl);
                const float mc = 0.5f * (n0[k] + n1[k]), mrr = 0.5f * (n1[k] - n0[k]);
                const float pm = sc * mc, rad = std::fabs(sc) * mrr + sr * (std::fabs(mc) + mrr);
                wl = pm - rad; wh = pm + rad;
            }
            float lo = dec(u[k], t.qbox.step[k], t.qbox.base[k]) + 2 * wl - rho;
            float hi = dec(u[3 + k], t.qbox.step[k], t.qbox.base[k]) + 2 * wh + rho;
            float t0 = (lo - ov[k]) * iv[k], t1 = (hi - ov[k]) * iv[k];
            tn = std::fmax(tn, std::fmin(t0, t1));
            tf = std::fmin(tf, std::fmax(t0, t1));
        }
    };
    float best = INFINITY;
    auto leaf = [&](uint32_t a) {
        const uint32_t first = (a & ~kLeafBit) >> 3, count = a & 7u;
        for (uint32_t j = first; j < first + count; ++j) {
            c.tests += 1;
            const float *r = &t.tris[(size_t)j * 16];
            V N{r[0], r[1], r[2]};
            float cs = dot(N, d);
            if (std::fabs(cs) < 1e-8f) continue;
            float tt = (dot(N, o) + r[3]) / cs;
            if (tt < 0.001f || tt > best) continue;
            V pp = add(o, mul(d, tt));
            V v0{r[4], r[5], r[6]}, v1{r[8], r[9], r[10]}, v2{r[12], r[13], r[14]};
            if (dot(N, cross(sub(v1, v0), sub(pp, v0))) < 0) continue;
            if (dot(N, cross(sub(v2, v1), sub(pp, v1))) < 0) continue;
            if (dot(N, cross(sub(v0, v2), sub(pp, v2))) < 0) continue;
            best = tt;
        }
    };
    // the root's own box first (as the binary walk does)
    {
        float tn, tf;
        c.boxes += 1;
        box(0, tn, tf);
        if (tn > tf || tf < 0.001f) return best;
        const uint32_t a = t.qnodes[6];
        if (a & kLeafBit) { leaf(a); return best; }
    }
    std::vector<std::pair<float, uint32_t>> st{{-INFINITY, 0u}};
    while (!st.empty()) {
        const auto [etn, node] = st.back();
        st.pop_back();
        c.pops += 1;
        if (etn > best) continue;
        c.fetches += 1;
        std::vector<std::pair<float, uint32_t>> hits;
        if (shared_n) {
            // the union of the children's normal boxes (u16 grid words 3..5)
            for (int k = 0; k < 3; ++k) { shared_m[k] = 0xFFFF; shared_m[3 + k] = 0; }
            for (uint32_t ch : W.kids[node]) {
                const uint32_t *w = &t.qnodes[(size_t)ch * 8];
                const uint32_t m[6] = {w[3] & 0xFFFF, w[3] >> 16, w[4] & 0xFFFF, w[4] >> 16, w[5] & 0xFFFF, w[5] >> 16};
                for (int k = 0; k < 3; ++k) {
                    shared_m[k] = std::min(shared_m[k], m[k]);
                    shared_m[3 + k] = std::max(shared_m[3 + k], m[3 + k]);
                }
            }
            use_shared = true;
        }
        for (uint32_t ch : W.kids[node]) {
            float tn, tf;
            c.boxes += 1;
            box(ch, tn, tf);
            if (tn > tf || tf < 0.001f || tn > best) continue;
            hits.push_back({tn, ch});
        }
        use_shared = false;
        // SIM_WIDE_ORDER=0: slot order (nearest-first otherwise)
        static const bool sorted = !std::getenv("SIM_WIDE_ORDER") || std::atoi(std::getenv("SIM_WIDE_ORDER")) != 0;
        if (sorted) std::sort(hits.begin(), hits.end());
        for (auto &h : hits) {
            const uint32_t a = t.qnodes[(size_t)h.second * 8 + 6];
            if (a & kLeafBit) { if (h.first <= best) leaf(a); }
        }
        for (auto it = hits.rbegin(); it != hits.rend(); ++it) {
            const uint32_t a = t.qnodes[(size_t)it->second * 8 + 6];
            if (!(a & kLeafBit) && it->first <= best) st.push_back(*it);
        }
        c.maxstack = std::max(c.maxstack, (double)st.size());
    }
    return best;
}

// SIM_Q8=B[,N]: 16-B nodes.  The tree in DFS preorder (first child = next
// node, skip = + subtree size); blocks of B consecutive nodes carry a float
// frame (box base + step per axis; normal base + step: one for all axes, or
// per axis with N=3) and every node stores its box and normal box as u8 on its
// block's frame, rounded outward from the u16 image.  Counts node visits and
// frame changes (a header load) per ray.
struct Q8 {
    int B = 64, N = 1;
    std::vector<uint8_t> q;       // 12 per node: box lo xyz, hi xyz, nbox lo xyz, hi xyz
    std::vector<float> hdr;       // 12 per block: base[3] step[3] nbase[3] nstep[3]
    std::vector<uint32_t> size, leaf_a;  // subtree size; builder word a for leaves (0: internal)
    std::vector<float> fbox, nun;  // N=0: u16-image box per node, block union of normal boxes
    std::vector<float> fnb;        // N<0: per-node normal box (global grids, SIM_G)
    size_t n = 0;
};
static float q8_step(float lo, float hi) {
    if (!(hi > lo)) return std::numeric_limits<float>::min();
    float s = (float)(((double)hi - lo) / 255.0 * (1 + 1e-6));
    while (std::fmaf(255.0f, s, lo) < hi) s = std::nextafter(s, INFINITY);
    return s;
}
static uint8_t q8_down(float x, float s, float b) {
    int q = (int)std::floor(((double)x - b) / s);
    q = std::min(255, std::max(0, q));
    while (q > 0 && std::fmaf((float)q, s, b) > x) --q;
    while (q < 255 && std::fmaf((float)(q + 1), s, b) <= x) ++q;
    return (uint8_t)q;
}
static uint8_t q8_up(float x, float s, float b) {
    int q = (int)std::ceil(((double)x - b) / s);
    q = std::min(255, std::max(0, q));
    while (q < 255 && std::fmaf((float)q, s, b) < x) ++q;
    while (q > 0 && std::fmaf((float)(q - 1), s, b) >= x) --q;
    return (uint8_t)q;
}
static Q8 make_q8(const TriangleBVH &t, int B, int N) {
    Q8 o; o.B = B; o.N = N;
    const size_t n = t.qnodes.size() / 8;
    std::vector<uint32_t> order;  // preorder -> builder node
    std::vector<uint32_t> st{0};
    while (!st.empty()) {
        const uint32_t i = st.back(); st.pop_back();
        order.push_back(i);
        const uint32_t a = t.qnodes[(size_t)i * 8 + 6];
        if (!(a & kLeafBit)) { const uint32_t c = a & 0x1FFFFFFFu; st.push_back(c + 1); st.push_back(c); }
    }
    o.n = order.size();
    std::vector<uint32_t> pos(n);
    for (size_t k = 0; k < order.size(); ++k) pos[order[k]] = (uint32_t)k;
    o.size.assign(o.n, 1);
    o.leaf_a.assign(o.n, 0);
    for (size_t k = o.n; k-- > 0;) {
        const uint32_t a = t.qnodes[(size_t)order[k] * 8 + 6];
        if (a & kLeafBit) o.leaf_a[k] = a;
        else { const uint32_t c = a & 0x1FFFFFFFu; o.size[k] = 1 + o.size[pos[c]] + o.size[pos[c + 1]]; }
    }
    auto dec = [](uint32_t q, float s, float b) { return std::fmaf((float)q, s, b); };
    std::vector<float> f(o.n * 12);
    for (size_t k = 0; k < o.n; ++k) {
        const uint32_t *w = &t.qnodes[(size_t)order[k] * 8];
        const uint32_t u[6] = {w[0] & 0xFFFF, w[0] >> 16, w[1] & 0xFFFF, w[1] >> 16, w[2] & 0xFFFF, w[2] >> 16};
        const uint32_t m[6] = {w[3] & 0xFFFF, w[3] >> 16, w[4] & 0xFFFF, w[4] >> 16, w[5] & 0xFFFF, w[5] >> 16};
        for (int j = 0; j < 6; ++j) {
            f[k * 12 + j] = dec(u[j], t.qbox.step[j % 3], t.qbox.base[j % 3]);
            f[k * 12 + 6 + j] = dec(m[j], t.nstep, t.nbase);
        }
    }
    const size_t nb = (o.n + B - 1) / B;
    if (N < 0) {  // SIM_G=Bb,Nb: global grids of 2^Bb / 2^Nb steps from the float nodes
        const char *g = std::getenv("SIM_G");
        int Bb = 10, Nb = 8;
        if (g) std::sscanf(g, "%d,%d", &Bb, &Nb);
        const int mb = (1 << Bb) - 1, mn = (1 << Nb) - 1;
        auto gstep = [](float lo, float hi, int m) {
            float st = (float)(((double)hi - lo) / m * (1 + 1e-6));
            while (std::fmaf((float)m, st, lo) < hi) st = std::nextafter(st, INFINITY);
            return st;
        };
        auto qd = [](float x, float st, float b, int m) {
            int q = (int)std::floor(((double)x - b) / st); q = std::min(m, std::max(0, q));
            while (q > 0 && std::fmaf((float)q, st, b) > x) --q;
            return std::fmaf((float)q, st, b);
        };
        auto qu = [](float x, float st, float b, int m) {
            int q = (int)std::ceil(((double)x - b) / st); q = std::min(m, std::max(0, q));
            while (q < m && std::fmaf((float)q, st, b) < x) ++q;
            return std::fmaf((float)q, st, b);
        };
        const float *root = &t.nodes[0];
        float bb[3], bs[3], nlo = 1, nhi = -1;
        for (int k = 0; k < 3; ++k) { bb[k] = root[k]; bs[k] = gstep(root[k], root[4 + k], mb); }
        for (size_t i = 0; i < n; ++i)
            for (int k = 0; k < 3; ++k) {
                nlo = std::min(nlo, t.nodes[i * 16 + 8 + k]); nhi = std::max(nhi, t.nodes[i * 16 + 12 + k]);
            }
        const float ns = gstep(nlo, nhi, mn);
        o.fbox.resize(o.n * 6);
        o.fnb.resize(o.n * 6);
        for (size_t k = 0; k < o.n; ++k) {
            const float *fn = &t.nodes[(size_t)order[k] * 16];
            for (int j = 0; j < 3; ++j) {
                o.fbox[k * 6 + j] = qd(fn[j], bs[j], bb[j], mb);
                o.fbox[k * 6 + 3 + j] = qu(fn[4 + j], bs[j], bb[j], mb);
                o.fnb[k * 6 + j] = qd(fn[8 + j], ns, nlo, mn);
                o.fnb[k * 6 + 3 + j] = qu(fn[12 + j], ns, nlo, mn);
            }
        }
        return o;
    }
    if (N == 0) {  // u16 boxes as now, one normal box per block
        o.fbox.resize(o.n * 6);
        o.nun.assign(nb * 6, 0);
        for (size_t b = 0; b < nb; ++b) {
            float *u = &o.nun[b * 6];
            for (int j = 0; j < 3; ++j) { u[j] = INFINITY; u[3 + j] = -INFINITY; }
            for (size_t k = b * B; k < std::min(o.n, (b + 1) * B); ++k)
                for (int j = 0; j < 3; ++j) {
                    u[j] = std::min(u[j], f[k * 12 + 6 + j]);
                    u[3 + j] = std::max(u[3 + j], f[k * 12 + 9 + j]);
                }
        }
        for (size_t k = 0; k < o.n; ++k)
            for (int j = 0; j < 6; ++j) o.fbox[k * 6 + j] = f[k * 12 + j];
        return o;
    }
    o.hdr.assign(nb * 12, 0);
    o.q.assign(o.n * 12, 0);
    for (size_t b = 0; b < nb; ++b) {
        float lo[6], hi[6];
        for (int j = 0; j < 6; ++j) { lo[j] = INFINITY; hi[j] = -INFINITY; }
        for (size_t k = b * B; k < std::min(o.n, (b + 1) * B); ++k)
            for (int j = 0; j < 3; ++j) {
                lo[j] = std::min(lo[j], f[k * 12 + j]); hi[j] = std::max(hi[j], f[k * 12 + 3 + j]);
                lo[3 + j] = std::min(lo[3 + j], f[k * 12 + 6 + j]); hi[3 + j] = std::max(hi[3 + j], f[k * 12 + 9 + j]);
            }
        if (N == 1) {
            const float l = std::min({lo[3], lo[4], lo[5]}), h = std::max({hi[3], hi[4], hi[5]});
            for (int j = 3; j < 6; ++j) { lo[j] = l; hi[j] = h; }
        }
        float *hd = &o.hdr[b * 12];
        for (int j = 0; j < 3; ++j) {
            hd[j] = lo[j]; hd[3 + j] = q8_step(lo[j], hi[j]);
            hd[6 + j] = lo[3 + j]; hd[9 + j] = q8_step(lo[3 + j], hi[3 + j]);
        }
        for (size_t k = b * B; k < std::min(o.n, (b + 1) * B); ++k)
            for (int j = 0; j < 3; ++j) {
                o.q[k * 12 + j] = q8_down(f[k * 12 + j], hd[3 + j], hd[j]);
                o.q[k * 12 + 3 + j] = q8_up(f[k * 12 + 3 + j], hd[3 + j], hd[j]);
                o.q[k * 12 + 6 + j] = q8_down(f[k * 12 + 6 + j], hd[9 + j], hd[6 + j]);
                o.q[k * 12 + 9 + j] = q8_up(f[k * 12 + 9 + j], hd[9 + j], hd[6 + j]);
            }
    }
    return o;
}
static double g_q8_hdr = 0;
static float trace_q8(const TriangleBVH &t, const Q8 &Q, V o, V d, Count &c) {
    c.rays += 1;
    const float onorm = std::fabs(o.x) + std::fabs(o.y) + std::fabs(o.z);
    const float iv[3] = {1.0f / d.x, 1.0f / d.y, 1.0f / d.z};
    const float dist = std::fabs(o.x - t.centre[0]) + std::fabs(o.y - t.centre[1]) +
                       std::fabs(o.z - t.centre[2]) + t.radius + 2 * onorm;
    const float rho = 1e-5f * (dist + onorm + t.mag);
    const float ov[3] = {o.x, o.y, o.z};
    const float dv[3] = {o.x - t.oc[0], o.y - t.oc[1], o.z - t.oc[2]};
    float best = INFINITY;
    size_t cur = (size_t)-1;
    for (size_t i = 0; i < Q.n;) {
        c.nodes += 1;
        if (i / Q.B != cur) { cur = i / Q.B; g_q8_hdr += 1; }
        const float *hd = Q.N > 0 ? &Q.hdr[cur * 12] : nullptr;
        const uint8_t *q = Q.N > 0 ? &Q.q[i * 12] : nullptr;
        float sl = 0, sh = 0, n0[3], n1[3], bl[3], bh[3];
        for (int k = 0; k < 3; ++k) {
            if (Q.N > 0) {
                n0[k] = std::fmaf((float)q[6 + k], hd[9 + k], hd[6 + k]);
                n1[k] = std::fmaf((float)q[9 + k], hd[9 + k], hd[6 + k]);
                bl[k] = std::fmaf((float)q[k], hd[3 + k], hd[k]);
                bh[k] = std::fmaf((float)q[3 + k], hd[3 + k], hd[k]);
            } else if (Q.N < 0) {
                n0[k] = Q.fnb[i * 6 + k];
                n1[k] = Q.fnb[i * 6 + 3 + k];
                bl[k] = Q.fbox[i * 6 + k];
                bh[k] = Q.fbox[i * 6 + 3 + k];
            } else {
                n0[k] = Q.nun[cur * 6 + k];
                n1[k] = Q.nun[cur * 6 + 3 + k];
                bl[k] = Q.fbox[i * 6 + k];
                bh[k] = Q.fbox[i * 6 + 3 + k];
            }
            float a = n0[k] * dv[k], b = n1[k] * dv[k];
            sl += std::fmin(a, b); sh += std::fmax(a, b);
        }
        float tn = -INFINITY, tf = INFINITY;
        for (int k = 0; k < 3; ++k) {
            float a = sl * n0[k], b = sl * n1[k], cc = sh * n0[k], dd = sh * n1[k];
            float lo = bl[k] + 2 * std::fmin(std::fmin(a, b), std::fmin(cc, dd)) - rho;
            float hi = bh[k] + 2 * std::fmax(std::fmax(a, b), std::fmax(cc, dd)) + rho;
            float t0 = (lo - ov[k]) * iv[k], t1 = (hi - ov[k]) * iv[k];
            tn = std::fmax(tn, std::fmin(t0, t1));
            tf = std::fmin(tf, std::fmax(t0, t1));
        }
        const bool skip = tn > tf || tf < 0.001f || tn > best;
        const uint32_t a = Q.leaf_a[i];
        if (!skip && a) {
            const uint32_t first = (a & ~kLeafBit) >> 3, count = a & 7u;
            for (uint32_t j = first; j < first + count; ++j) {
                c.tests += 1;
                const float *r = &t.tris[(size_t)j * 16];
                V N{r[0], r[1], r[2]};
                float cs = dot(N, d);
                if (std::fabs(cs) < 1e-8f) continue;
                float tt = (dot(N, o) + r[3]) / cs;
                if (tt < 0.001f || tt > best) continue;
                V pp = add(o, mul(d, tt));
                V v0{r[4], r[5], r[6]}, v1{r[8], r[9], r[10]}, v2{r[12], r[13], r[14]};
                if (dot(N, cross(sub(v1, v0), sub(pp, v0))) < 0) continue;
                if (dot(N, cross(sub(v2, v1), sub(pp, v1))) < 0) continue;
                if (dot(N, cross(sub(v0, v2), sub(pp, v2))) < 0) continue;
                best = tt;
            }
        }
        i = skip ? i + Q.size[i] : i + 1;
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
    float soc[3] = {0, 0, 0};
    const char *socs = std::getenv("SIM_OC");  // static-tree origin "x,y,z" (+ optional ",L")
    double sph = 0;
    if (socs) std::sscanf(socs, "%f,%f,%f,%lf", &soc[0], &soc[1], &soc[2], &sph);
    TriangleBVH t = build_triangle_bvh(s.triangles, p.tri_hot, lf ? std::atoi(lf) : 4, socs ? soc : nullptr, sph);
    std::printf("tris %zu nodes %zu loose %zu depth %u\n", s.triangles.size(), t.nodes.size() / 16,
                t.loose.size(), t.depth);
    if (std::getenv("SIM_LEVELS")) {  // depth of every node (child pair at a & 0x1FFFFFFF)
        const size_t n = t.qnodes.size() / 8;
        g_depth.assign(n, 0);
        g_level_visits.assign(64, 0);
        for (size_t i = 0; i < n; ++i) {  // parents precede children in the builder layout
            const uint32_t a = t.qnodes[i * 8 + 6];
            if (!(a & kLeafBit)) {
                const uint32_t ch = a & 0x1FFFFFFFu;
                g_depth[ch] = g_depth[ch + 1] = g_depth[i] + 1;
            }
        }
    }
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
    Count prim, sec, q8c;
    std::unique_ptr<Wide> wide;
    WideCount wprim, wsec;
    size_t wdiff = 0;
    if (const char *ws = std::getenv("SIM_WIDE")) wide = std::make_unique<Wide>(make_wide(t, std::atoi(ws)));
    std::unique_ptr<Q8> q8;
    size_t q8diff = 0;
    if (const char *qs = std::getenv("SIM_Q8")) {
        int B = 64, N = 1;
        std::sscanf(qs, "%d,%d", &B, &N);
        q8 = std::make_unique<Q8>(make_q8(t, B, N));
    }
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
            if (wide) {
                const float tw = trace_wide(t, *wide, org, d, wprim);
                if (!(tw == tt || (std::isinf(tw) && std::isinf(tt)))) ++wdiff;
            }
            if (std::isfinite(tt)) {
                ++hits;
                V o2 = add(org, mul(d, tt));
                V d2 = unit(V{rnd() * 2 - 1, rnd() * 2 - 1, rnd() * 2 - 1});
                const float t2 = trace(t, o2, d2, sec);
                if (wide) {
                    const float tw = trace_wide(t, *wide, o2, d2, wsec);
                    if (!(tw == t2 || (std::isinf(tw) && std::isinf(t2)))) ++wdiff;
                }
                if (q8) {
                    const float t3 = trace_q8(t, *q8, o2, d2, q8c);
                    if (!(t2 == t3 || (std::isinf(t2) && std::isinf(t3)))) ++q8diff;
                }
            }
        }
    if (const char *ws = std::getenv("SIM_WAVE")) {
        // Wave coherence of secondary rays: groups of G rays whose origins are
        // the hits of G jittered primary rays of one pixel (a wave's lanes hold
        // samples of one or two pixels), directions random.  Per group: lane
        // visits summed, the longest walk, the distinct nodes the lanes touch
        // at each lockstep step (vector loads: one L2 request per distinct
        // 32-B node per instruction), and the union of the walks (a wave-wide
        // packet walk in DFS preorder: one scalar load per node of the union).
        const int G = std::max(1, std::atoi(ws));
        const size_t n = t.qnodes.size() / 8;
        std::vector<uint32_t> rank(n, 0);  // preorder rank of each node
        {
            std::vector<uint32_t> st{0};
            uint32_t r = 0;
            while (!st.empty()) {
                const uint32_t i = st.back(); st.pop_back();
                rank[i] = r++;
                const uint32_t a = t.qnodes[(size_t)i * 8 + 6];
                if (!(a & kLeafBit)) { const uint32_t c = a & 0x1FFFFFFFu; st.push_back(c + 1); st.push_back(c); }
            }
        }
        const bool cosine = std::getenv("SIM_WAVE_COS") != nullptr;  // normal + unit (diffuse) dirs
        uint32_t rng3 = 12345u;
        auto rnd3 = [&]() { rng3 ^= rng3 << 13; rng3 ^= rng3 >> 17; rng3 ^= rng3 << 5; return rng3 * 0x1p-32f; };
        double lanes = 0, maxl = 0, uniq = 0, uni = 0, groups = 0, nonmono = 0;
        Count dummy, wc;
        for (int j = 0; j < H; ++j)
            for (int i = 0; i < W; ++i) {
                std::vector<std::vector<uint32_t>> walks;
                for (int k = 0; k < G; ++k) {
                    const float u = (i + rnd3()) / W, v = (j + rnd3()) / H;
                    V d = unit(sub(add(add(V{cm.lower_left.x, cm.lower_left.y, cm.lower_left.z},
                                           mul(V{cm.horizontal.x, cm.horizontal.y, cm.horizontal.z}, u)),
                                       mul(V{cm.vertical.x, cm.vertical.y, cm.vertical.z}, v)), org));
                    const float tt = trace(t, org, d, dummy);
                    if (!std::isfinite(tt)) continue;
                    V o2 = add(org, mul(d, tt));
                    V d2 = unit(V{rnd3() * 2 - 1, rnd3() * 2 - 1, rnd3() * 2 - 1});
                    if (cosine) {
                        // around the nearest triangle's normal facing the ray origin side
                        V nz{0, 0, 1};
                        d2 = unit(add(nz, d2));
                    }
                    std::vector<uint32_t> vis;
                    g_visits = &vis;
                    trace(t, o2, d2, wc);
                    g_visits = nullptr;
                    walks.push_back(std::move(vis));
                }
                if (walks.empty()) continue;
                groups += 1;
                size_t mx = 0;
                std::vector<uint32_t> all;
                for (auto &w : walks) {
                    lanes += w.size();
                    mx = std::max(mx, w.size());
                    for (size_t q = 1; q < w.size(); ++q) nonmono += rank[w[q]] <= rank[w[q - 1]];
                    all.insert(all.end(), w.begin(), w.end());
                }
                maxl += mx;
                for (size_t s = 0; s < mx; ++s) {
                    std::vector<uint32_t> at;
                    for (auto &w : walks) if (s < w.size()) at.push_back(w[s]);
                    std::sort(at.begin(), at.end());
                    uniq += std::unique(at.begin(), at.end()) - at.begin();
                }
                std::sort(all.begin(), all.end());
                uni += std::unique(all.begin(), all.end()) - all.begin();
            }
        std::printf("waves of %d secondary rays (%s dirs): %.0f groups, per group: lane visits %.0f, longest "
                    "walk %.0f, lockstep distinct nodes %.0f, union %.0f (non-monotone steps %.0f)\n",
                    G, cosine ? "+z diffuse" : "uniform", groups, lanes / groups, maxl / groups, uniq / groups,
                    uni / groups, nonmono);
        return 0;
    }
    if (const char *bs = std::getenv("SIM_BIN")) {
        // Secondary-ray binning: pools of P rays (P/16 consecutive pixels x 16
        // samples, as a workgroup's lanes would hold them), cut into waves of 64
        // either in arrival order (4 pixels per wave) or after sorting the pool
        // by direction octant then origin (SIM_BIN_KEY=1: octant only, 2:
        // octant + 8-unit... origin cell of SIM_BIN_CELL units).  Per wave: lane
        // visits, the longest walk, the lockstep distinct nodes (L2 requests of
        // independent walks) and the union (a packet walk's scalar loads).
        const int P = std::max(64, std::atoi(bs)) / 64 * 64;
        const int key = std::getenv("SIM_BIN_KEY") ? std::atoi(std::getenv("SIM_BIN_KEY")) : 2;
        const float cell = std::getenv("SIM_BIN_CELL") ? (float)std::atof(std::getenv("SIM_BIN_CELL")) : 1.0f;
        uint32_t rng3 = 12345u;
        auto rnd3 = [&]() { rng3 ^= rng3 << 13; rng3 ^= rng3 >> 17; rng3 ^= rng3 << 5; return rng3 * 0x1p-32f; };
        struct R { uint64_t k; std::vector<uint32_t> w; };
        double st[2][4] = {};
        double waves = 0;
        const int ppool = P / 16;
        Count wc, dummy;
        for (int pix0 = 0; pix0 + ppool <= W * H; pix0 += ppool) {
            std::vector<R> pool;
            for (int q = 0; q < ppool; ++q) {
                const int i = (pix0 + q) % W, j = (pix0 + q) / W;
                for (int k = 0; k < 16; ++k) {
                    const float u = (i + rnd3()) / W, v = (j + rnd3()) / H;
                    V d = unit(sub(add(add(V{cm.lower_left.x, cm.lower_left.y, cm.lower_left.z},
                                           mul(V{cm.horizontal.x, cm.horizontal.y, cm.horizontal.z}, u)),
                                       mul(V{cm.vertical.x, cm.vertical.y, cm.vertical.z}, v)), org));
                    const float tt = trace(t, org, d, dummy);
                    V o2 = org, d2 = d;
                    R r;
                    if (std::isfinite(tt)) {
                        o2 = add(org, mul(d, tt));
                        d2 = unit(V{rnd3() * 2 - 1, rnd3() * 2 - 1, rnd3() * 2 - 1});
                        g_visits = &r.w;
                        trace(t, o2, d2, wc);
                        g_visits = nullptr;
                    }
                    const uint64_t oct = (d2.x < 0) | ((d2.y < 0) << 1) | ((d2.z < 0) << 2);
                    auto cq = [&](float x) { return (uint64_t)(int64_t)std::floor(x / cell + 512) & 1023u; };
                    r.k = (oct << 40) | (key >= 2 ? (cq(o2.x) << 20 | cq(o2.y) << 10 | cq(o2.z)) : 0);
                    pool.push_back(std::move(r));
                }
            }
            for (int mode = 0; mode < 2; ++mode) {
                std::vector<R *> order;
                for (auto &r : pool) order.push_back(&r);
                if (mode == 1)
                    std::stable_sort(order.begin(), order.end(), [](const R *a, const R *b) { return a->k < b->k; });
                for (size_t w0 = 0; w0 < order.size(); w0 += 64) {
                    size_t mx = 0;
                    double lanes = 0;
                    std::vector<uint32_t> all;
                    for (size_t l = w0; l < w0 + 64; ++l) {
                        mx = std::max(mx, order[l]->w.size());
                        lanes += order[l]->w.size();
                        all.insert(all.end(), order[l]->w.begin(), order[l]->w.end());
                    }
                    double uq = 0;
                    for (size_t s2 = 0; s2 < mx; ++s2) {
                        std::vector<uint32_t> at;
                        for (size_t l = w0; l < w0 + 64; ++l)
                            if (s2 < order[l]->w.size()) at.push_back(order[l]->w[s2]);
                        std::sort(at.begin(), at.end());
                        uq += std::unique(at.begin(), at.end()) - at.begin();
                    }
                    std::sort(all.begin(), all.end());
                    const double un = (double)(std::unique(all.begin(), all.end()) - all.begin());
                    st[mode][0] += lanes; st[mode][1] += (double)mx; st[mode][2] += uq; st[mode][3] += un;
                    if (mode == 0) waves += 1;
                }
            }
        }
        for (int mode = 0; mode < 2; ++mode)
            std::printf("pool %d, %s: per wave lane visits %.0f, longest %.0f, lockstep distinct %.0f, union %.0f\n",
                        P, mode ? "binned" : "arrival order", st[mode][0] / waves, st[mode][1] / waves,
                        st[mode][2] / waves, st[mode][3] / waves);
        return 0;
    }
    if (const char *hs = std::getenv("SIM_HYB")) {
        float S = 1; std::sscanf(hs, "%d,%f", &g_hyb_D, &S);
        g_hyb_range = std::getenv("SIM_HYB_RANGE") != nullptr;
        const size_t n = t.qnodes.size() / 8;
        g_depth.assign(n, 0);
        g_level_visits.assign(64, 0);
        for (size_t i = 0; i < n; ++i) {
            const uint32_t a = t.qnodes[i * 8 + 6];
            if (!(a & kLeafBit)) { const uint32_t ch = a & 0x1FFFFFFFu; g_depth[ch] = g_depth[ch + 1] = g_depth[i] + 1; }
        }
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
        std::map<std::tuple<int, int, int>, std::vector<float>> cells;
        // per-node box over the node's records' phantoms for o in the cell
        std::function<void(uint32_t, const double *, const double *, std::vector<float> &, float *)> rec;
        rec = [&](uint32_t node, const double *clo, const double *chi, std::vector<float> &out, float *bx) {
            const uint32_t a = t.qnodes[(size_t)node * 8 + 6];
            float b[6] = {INFINITY, INFINITY, INFINITY, -INFINITY, -INFINITY, -INFINITY};
            if (a & kLeafBit) {
                const uint32_t first = (a & ~kLeafBit) >> 3, count = a & 7u;
                for (uint32_t j = first; j < first + count; ++j) {
                    const float *r = &t.tris[(size_t)j * 16];
                    double nn = std::sqrt((double)r[0] * r[0] + (double)r[1] * r[1] + (double)r[2] * r[2]);
                    double nh[3] = {r[0] / nn, r[1] / nn, r[2] / nn};
                    double smin = 0, smax = 0;
                    for (int k = 0; k < 3; ++k) {
                        if (g_hyb_range) {
                            const double p = nh[k] * clo[k], q = nh[k] * chi[k];
                            smin += std::min(p, q);
                            smax += std::max(p, q);
                        } else {
                            smin += nh[k] * (clo[k] + chi[k]) / 2;
                        }
                    }
                    if (!g_hyb_range) smax = smin;
                    for (int k = 0; k < 3; ++k) {
                        double o1 = 2 * nh[k] * smin, o2 = 2 * nh[k] * smax;
                        double vmin = std::min({r[4 + k], r[8 + k], r[12 + k]}), vmax = std::max({r[4 + k], r[8 + k], r[12 + k]});
                        b[k] = std::min(b[k], (float)(vmin + std::min(o1, o2)) - 1e-4f);
                        b[3 + k] = std::max(b[3 + k], (float)(vmax + std::max(o1, o2)) + 1e-4f);
                    }
                }
            } else {
                const uint32_t ch = a & 0x1FFFFFFFu;
                float b1[6], b2[6];
                rec(ch, clo, chi, out, b1); rec(ch + 1, clo, chi, out, b2);
                for (int k = 0; k < 3; ++k) { b[k] = std::min(b1[k], b2[k]); b[3 + k] = std::max(b1[3 + k], b2[3 + k]); }
            }
            for (int k = 0; k < 6; ++k) { bx[k] = b[k]; out[(size_t)node * 6 + k] = b[k]; }
        };
        Count hc;
        for (size_t r = 0; r < o2s.size(); ++r) {
            V o2 = o2s[r];
            auto key = std::make_tuple((int)std::floor(o2.x / S), (int)std::floor(o2.y / S), (int)std::floor(o2.z / S));
            auto it = cells.find(key);
            if (it == cells.end()) {
                double clo[3] = {std::get<0>(key) * S, std::get<1>(key) * S, std::get<2>(key) * S};
                double chi[3] = {clo[0] + S, clo[1] + S, clo[2] + S};
                std::vector<float> bx(n * 6);
                float root[6];
                rec(0, clo, chi, bx, root);
                it = cells.emplace(key, std::move(bx)).first;
            }
            g_cellbox = &it->second;
            for (int k = 0; k < 3; ++k) g_coc[k] = (k == 0 ? std::get<0>(key) : k == 1 ? std::get<1>(key) : std::get<2>(key)) * S + S / 2;
            trace(t, o2, d2s[r], hc);
            g_cellbox = nullptr;
        }
        std::printf("hybrid D=%d S=%g: %zu cells, secondary %.1f nodes/ray (%.1f with cell boxes), %.2f tests/ray\n",
                    g_hyb_D, S, cells.size(), hc.nodes / hc.rays, g_hyb_hits / hc.rays, hc.tests / hc.rays);
        return 0;
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
    if (wide)
        for (const WideCount *w : {&wprim, &wsec})
            std::printf("wide K=%s %s: %.1f fetches/ray, %.1f box tests/ray, %.1f tri tests/ray, "
                        "%.1f pops/ray, max stack %.0f, %zu hits differ\n", std::getenv("SIM_WIDE"),
                        w == &wprim ? "primary" : "secondary", w->fetches / w->rays, w->boxes / w->rays,
                        w->tests / w->rays, w->pops / w->rays, w->maxstack, wdiff);
    if (q8)
        std::printf("q8 B=%d N=%d: secondary %.1f nodes/ray, %.2f frame changes/ray, %.1f tests/ray, %zu hits differ\n",
                    q8->B, q8->N, q8c.nodes / q8c.rays, g_q8_hdr / q8c.rays, q8c.tests / q8c.rays, q8diff);
    if (!g_level_visits.empty()) {  // cumulative share of visits in the top levels
        double tot = 0, acc = 0;
        std::vector<size_t> per_level(64, 0);
        for (int d : g_depth) per_level[d]++;
        for (double v : g_level_visits) tot += v;
        size_t nodes_acc = 0;
        for (int d = 0; d < 64 && per_level[d]; ++d) {
            acc += g_level_visits[d];
            nodes_acc += per_level[d];
            std::printf("levels 0..%d: %zu nodes, %.1f%% of visits\n", d, nodes_acc, 100 * acc / tot);
        }
    }
}
