// render.hip -- the MI355X render path: a persistent path-regenerating trace
// kernel and an ordered resolve kernel, hand-written for gfx950 (CDNA4).
//
// Replaces the reference's ray_trace pixel loop and everything under it
// (Naxaes/Rust-Swift-Raytracer raytracer/src/common.rs:263-361 ray_color /
// ray_trace, common.rs:59-258 Sphere/Triangle/Mesh/World::hit,
// materials.rs:30-102 scatter, camera.rs:84-89 cast_ray, random.rs:15-30).
//
// Numerics: every operation is one IEEE binary32 op in the reference's order
// (-ffp-contract=off, correctly rounded divide/sqrt), so a sample started
// from the same xorshift32 state produces the same bits as the reference.
//
// Work decomposition: one job = one pixel sample.  Each wave
// is persistent: its 64 lanes trace one bounce per loop iteration; a lane
// whose path ends writes the sample colour to a per-sample slab in HBM and
// takes the next job (ballot + mbcnt prefix, one atomic per chunk per wave on
// one of 16-64 partitioned counters), so lanes never idle behind the longest path
// of their wave.  World::hit goes through exact BVHs (spheres: staged in LDS;
// triangles: phantom-aware static and camera-origin trees, primary strip
// lists) whose visiting order provably returns the reference's hit; the
// brute-force loops keep the reference order (RT_ACCEL_BRUTE, small scenes).
// The resolve kernel sums each pixel's samples in sample order (the
// reference's sequential add_with_alpha, common.rs:338-340), applies the
// gamma/`as u8` epilogue (:344-356) and stores RGBA8 rows top-first (:351).
#include <hip/hip_runtime.h>

#include <cstdint>

#include "exactdiv.h"
#include "render.h"

#pragma clang fp contract(off)

namespace rtamd {
namespace {

// ------------------------------------------------------------ device maths
struct F3 { float x, y, z; };

__device__ __forceinline__ F3 f3(float x, float y, float z) { return F3{x, y, z}; }
__device__ __forceinline__ F3 operator+(F3 a, F3 b) { return F3{a.x + b.x, a.y + b.y, a.z + b.z}; }
__device__ __forceinline__ F3 operator-(F3 a, F3 b) { return F3{a.x - b.x, a.y - b.y, a.z - b.z}; }
__device__ __forceinline__ F3 operator-(F3 a) { return F3{-a.x, -a.y, -a.z}; }
__device__ __forceinline__ F3 scale(F3 a, float s) { return F3{a.x * s, a.y * s, a.z * s}; }
// (x*x' + y*y') + z*z'  (maths.rs:82)
__device__ __forceinline__ float dot(F3 a, F3 b) { return (a.x * b.x + a.y * b.y) + a.z * b.z; }
__device__ __forceinline__ F3 cross(F3 a, F3 b) {  // maths.rs:88-94
    return F3{a.y * b.z - a.z * b.y, -(a.x * b.z - a.z * b.x), a.x * b.y - a.y * b.x};
}
// The divisions go through exactdiv.h (one shared correctly rounded
// reciprocal, three corrected quotients: the same bits as `/`) whenever the
// operands are in its guarded range; HIP's divide otherwise (never taken by
// lanes of ordinary scenes, so the branch is skipped wave-wide).
// RT_NO_XDIV builds the plain-divide variant (A/B only).
__device__ __forceinline__ F3 divide_by(F3 a, float b) {
#ifndef RT_NO_XDIV
    // (bitwise: both guards evaluate without a branch)
    if (__builtin_expect((unsigned)xdiv_den_ok(b) & (unsigned)xdiv_num3_ok(a.x, a.y, a.z), 1)) {
        const float y = xdiv_rcp(b);
        return F3{xdiv(a.x, b, y), xdiv(a.y, b, y), xdiv(a.z, b, y)};
    }
#endif
    return F3{a.x / b, a.y / b, a.z / b};
}
__device__ __forceinline__ F3 unit(F3 a) {  // NVec3::new, maths.rs:111-118
    const float len = xsqrt((a.x * a.x + a.y * a.y) + a.z * a.z);
#ifndef RT_NO_XDIV
    // components are bounded by the length: the cheaper numerator guard
    if (__builtin_expect((unsigned)xdiv_den_ok(len) & (unsigned)xdiv_num3_small_ok(a.x, a.y, a.z), 1)) {
        const float y = xdiv_rcp(len);
        return F3{xdiv(a.x, len, y), xdiv(a.y, len, y), xdiv(a.z, len, y)};
    }
#endif
    return F3{a.x / len, a.y / len, a.z / len};
}

// xorshift32 (random.rs:22-30); `x as f32 / u32::MAX as f32` == RN(x) * 2^-32.
__device__ __forceinline__ uint32_t xorshift(uint32_t &s) {
    uint32_t x = s;
    x ^= x << 13;
    x ^= x >> 17;
    x ^= x << 5;
    s = x;
    return x;
}
// `random_f32() * 2.0 - 1.0` (common.rs:32-38, random.rs:27-30): RN(RN(x) 2^-32 2
// - 1) with an exact product (a power-of-two scaling of RN(x), >= 2^-31), so
// one fma gives the same bits.
__device__ __forceinline__ float draw11(uint32_t &s) {
    return __builtin_fmaf((float)xorshift(s), 0x1p-31f, -1.0f);
}
// `n + random_f32()` (camera u, v numerators, common.rs:335-336): the same
// exact product, one rounding
__device__ __forceinline__ float draw_plus(uint32_t &s, float n) {
    return __builtin_fmaf((float)xorshift(s), 0x1p-32f, n);
}
// common.rs:32-38 -- three draws x, y, z, normalised (no rejection sampling).
__device__ __forceinline__ F3 draw_unit(uint32_t &s) {
    float x = draw11(s);
    float y = draw11(s);
    float z = draw11(s);
    return unit(F3{x, y, z});
}

__device__ __forceinline__ uint32_t counter_seed(uint32_t seed, uint64_t job) {
#ifdef RT_ABLATE_SEED  // timing-only diagnostic: wrong seeds
    return ((uint32_t)job * 0x9E3779B9u + seed) | 1u;
#endif
    uint64_t z = job + (uint64_t)seed * 0x9E3779B97F4A7C15ull + 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    z ^= z >> 31;
    uint32_t r = (uint32_t)(z ^ (z >> 32));
    return r ? r : 2547549u;
}

// Rust `f32 as u8`: saturating, NaN -> 0, truncating.
__device__ __forceinline__ uint32_t sat_u8(float x) {
    if (!(x > 0.0f)) return 0u;
    if (x >= 255.0f) return 255u;
    return (uint32_t)x;
}

// Wave-uniform read of scene data through the constant address space, so the
// backend emits s_load (scalar cache -> SGPRs) instead of 64 lane loads.
__device__ __forceinline__ float4 uniform_load(const float4 *base, uint32_t i) {
#if defined(__HIP_DEVICE_COMPILE__)
    typedef const __attribute__((address_space(4))) float *cfloat_ptr;
    const cfloat_ptr q = (cfloat_ptr)(const void *)base + 4u * i;
    return make_float4(q[0], q[1], q[2], q[3]);
#else
    return base[i];
#endif
}

__device__ __forceinline__ uint32_t uniform_load_u32(const uint32_t *base, uint32_t i) {
#if defined(__HIP_DEVICE_COMPILE__)
    typedef const __attribute__((address_space(4))) uint32_t *cu32_ptr;
    return ((cu32_ptr)(const void *)base)[i];
#else
    return base[i];
#endif
}

__device__ __forceinline__ uint4 uniform_load_u4(const uint4 *base, uint32_t i) {
#if defined(__HIP_DEVICE_COMPILE__)
    typedef const __attribute__((address_space(4))) uint32_t *cu32_ptr;
    const cu32_ptr q = (cu32_ptr)(const void *)base + 4u * i;
    return make_uint4(q[0], q[1], q[2], q[3]);
#else
    return base[i];
#endif
}

__device__ __forceinline__ uint32_t fdiv(uint32_t n, const FastDiv &f) { return fastdiv_apply(n, f); }

constexpr uint32_t kWave = 64;
constexpr uint32_t kNodeEndDev = 0xFFFFFFFFu;  // bvh.h kNodeEnd
constexpr uint32_t kLeafBitDev = 0x80000000u;  // bvh.h kLeafBit
constexpr uint32_t kSphListWalk = 0xFFFFu;     // bvh.h kSphListWalk
constexpr uint32_t kSphListMaxDev = 3u;        // bvh.h kSphListMax
constexpr uint32_t kBatch = 8;  // spheres per scalar-load batch (sphere count padded to it)

// ------------------------------------------------------------ sphere stage
// Brute force, file order, shrinking t_max (common.rs:241-247).  Batches of
// kBatch spheres: all scalar loads issue up front, the discriminants
// (independent of t_max) are computed for the whole batch, and the in-order
// root/t_max updates run only when some lane's discriminant is non-negative
// (rare; wave-uniform skip).
// The last batch tests only the scene's spheres: a wave-uniform guard skips
// the padding's arithmetic (world.txt's 9 spheres took 16 tests per ray;
// RT_BRUTE_PADDED restores the padded batches).
__device__ __forceinline__ void spheres_brute(const TraceParams &p, F3 org, F3 dir, float &best_t,
                                              int &best_i) {
    const float tmin = 0.001f;
#ifdef RT_BRUTE_PADDED
    const uint32_t n = p.nsph_padded;
#else
    const uint32_t n = p.nsph;
#endif
    for (uint32_t i0 = 0; i0 < n; i0 += kBatch) {
        const uint32_t m = n - i0;  // spheres left (>= kBatch except in the last batch)
        float hb[kBatch], disc[kBatch];
        bool any = false;
#pragma unroll
        for (uint32_t k = 0; k < kBatch; ++k) {
            hb[k] = 0.0f;
            disc[k] = -1.0f;
            if (k != 0u && k >= m) continue;  // (wave-uniform)
            const float4 S = uniform_load(p.sph_hot, i0 + k);
            const float ocx = org.x - S.x, ocy = org.y - S.y, ocz = org.z - S.z;
            hb[k] = (ocx * dir.x + ocy * dir.y) + ocz * dir.z;
            const float cc = ((ocx * ocx + ocy * ocy) + ocz * ocz) - S.w;
            disc[k] = hb[k] * hb[k] - cc;  // a == 1.0 exactly (maths.rs:127)
            any |= disc[k] >= 0.0f;
        }
        if (!any) continue;
#pragma unroll
        for (uint32_t k = 0; k < kBatch; ++k) {
            if (disc[k] >= 0.0f) {
                const float sq = xsqrt(disc[k]);
                const float r1 = -hb[k] - sq;
                const float r2 = -hb[k] + sq;
                const bool ok1 = (tmin < r1) && (r1 < best_t);
                const bool ok2 = (tmin < r2) && (r2 < best_t);
                if (ok1 || ok2) {
                    best_t = ok1 ? r1 : r2;  // r1 <= r2: the smaller valid root
                    best_i = (int)(i0 + k);
                }
            }
        }
    }
}

// One sphere in any order: same arithmetic as Sphere::hit (common.rs:74-92);
// the candidate (root1 if > t_min, else root2 if > t_min) is independent of
// t_max, and the reference keeps the smallest candidate, lowest index first.
__device__ __forceinline__ bool sphere_candidate(float4 S, F3 org, F3 dir, int idx, float &best_t,
                                                 int &best_i) {
    const float tmin = 0.001f;
    const float ocx = org.x - S.x, ocy = org.y - S.y, ocz = org.z - S.z;
    const float hb = (ocx * dir.x + ocy * dir.y) + ocz * dir.z;
    const float cc = ((ocx * ocx + ocy * ocy) + ocz * ocz) - S.w;
    const float disc = hb * hb - cc;
    if (!(disc >= 0.0f)) return false;
    const float sq = xsqrt(disc);
    const float r1 = -hb - sq;
    const float r2 = -hb + sq;
    const bool v1 = tmin < r1;
    const float c = v1 ? r1 : r2;
    const bool valid = v1 || (tmin < r2);
    // c < best_t || (c == best_t && best_t < inf && idx < best_i) as one
    // unsigned compare of (t bits, index) keys: both t are positive (c > t_min,
    // best_t > t_min or +inf), so their bits order like the values; best_i is
    // -1 (all ones) only while best_t is +inf, and c = +inf, which that rule
    // never takes, is excluded
    const uint64_t kc = ((uint64_t)__float_as_uint(c) << 32) | (uint32_t)idx;
    const uint64_t kb = ((uint64_t)__float_as_uint(best_t) << 32) | (uint32_t)best_i;
    const bool take = valid && c != __builtin_inff() && kc < kb;
    if (take) { best_t = c; best_i = idx; }
    return take;
}

constexpr float kErrK = 3.0e-3f;  // >= 2.7x the derived sqrt(30u) = 1.12e-3

// Where the traversal reads the tree from: global memory (any size) or the
// workgroup's LDS copy (staged once per persistent workgroup).
struct BvhView {
    const float4 *nodes;     // global: 2 per node; LDS: 64-B records (box | 8 x u32 link pairs)
    const uint32_t *miss32;  // global: 8 x u32 per node
    const uint16_t *miss16;  // (unused: the LDS links live in the node records)
    const float4 *prims;
    const uint32_t *ids;
    const float4 *shade;     // per-sphere shading records (2 x float4)
    const uint32_t *kinds;
};

// Spheres through the exact-pruning BVH (bvh.h): big spheres first (brute
// force, wave-uniform), then a stackless octant-ordered traversal that the
// kernel can advance a bounded number of nodes per loop iteration.  Every
// node box is inflated per ray by e, which bounds how far a computed
// candidate's point can lie outside its sphere: with
// s = min(A, best_t + R)(1+3K) + R >= |o - c| + r for every sphere that can
// still win, the squared-distance excess is <= 30u s^2, so the point is
// within min(sqrt(30u) s, 15u s^2 / r) of the surface.  e takes the smaller
// of K s (K = 3e-3) and Kq s^2 / rmin (Kq = 40.5u), both 2.7x the bound,
// plus e_abs for the slab arithmetic.  A node is skipped only when the
// inflated box is certainly missed or certainly starts beyond best_t.
__device__ __forceinline__ float slab_rcp(float d) {
    return __builtin_amdgcn_fmed3f(__builtin_amdgcn_rcpf(d), -1e20f, 1e20f);
}

struct SphBound { float A, e_abs; };  // per-ray inputs of the inflation
__device__ __forceinline__ SphBound sph_bound(const TraceParams &p, F3 org) {
    const float ax = org.x - p.bvh_c[0], ay = org.y - p.bvh_c[1], az = org.z - p.bvh_c[2];
    // (v_sqrt_f32, <= 1 ulp: the 1e-5 factor covers it; A is only a bound)
    return SphBound{__builtin_amdgcn_sqrtf((ax * ax + ay * ay) + az * az) * 1.00001f + p.bvh_r,
                    2e-6f * ((fabsf(org.x) + fabsf(org.y)) + fabsf(org.z) + p.bvh_mag)};
}
constexpr float kErrKq = 40.5f * 0x1p-24f;  // 2.7 x 15u
__device__ __forceinline__ float sph_inflation(const TraceParams &p, SphBound b, float bt) {
    const float s = fminf(b.A, bt + p.bvh_rmax) * (1.0f + 3.0f * kErrK) + p.bvh_rmax;  // fminf(A, inf) = A
    // fminf drops the NaN of 0 * inf (rmin == 0): the linear bound then applies
    return fminf(kErrK * s, (kErrKq * s) * (s * p.bvh_inv_rmin)) + b.e_abs;
}

__device__ __forceinline__ void spheres_big(const TraceParams &p, F3 org, F3 dir, float &best_t,
                                            int &best_i) {
    for (uint32_t k = 0; k < p.nbig; ++k) {
        // (both scalar loads: a vector load here made the ray setup wait on
        // every outstanding vector memory op, vmcnt(0))
        const float4 S = uniform_load(p.big_hot, k);
        sphere_candidate(S, org, dir, (int)uniform_load_u32(p.big_id, k), best_t, best_i);
    }
}

// One node of the sphere tree.  node becomes the end marker when the search
// is over: kNodeEndDev, or 0xFFFF for the LDS copy's u16 links.  A leaf the
// ray enters is handed back in `leaf` as (first << 3) | count for
// sphere_leaf.  (Deferring leaf tests until every lane of the wave has one
// pending -- "while-while" -- measured 6% slower on C2 and 60% on C5.)
// kLds: `ooff` = 4 * octant (the link word's offset in the record); global
// memory: `ooff` = the octant, `octm` unused.
template <bool kLds>
__device__ __forceinline__ bool sphere_node(const BvhView &v, F3 inv, uint32_t ooff, float best_t, F3 nlo,
                                            F3 nhi, uint32_t &node, uint32_t &leaf, uint32_t &node_tests) {
    ++node_tests;
    // LDS copy: `node` is the record's LDS byte address (64-B records: box |
    // per octant one u32 of two u16 links: the node to visit next when the box
    // is entered -- the near child, or for a leaf its miss link -- and when it
    // is skipped), so the next node is one select of a half of one LDS word
    float4 B0, B1;
    uint32_t miss, hit = 0;
    if (kLds) {
#if defined(__HIP_DEVICE_COMPILE__)
        // `node` is the record's LDS address (staged as such: no base add)
        typedef const __attribute__((address_space(3))) char *lds_cptr;
        const lds_cptr rec = (lds_cptr)(uintptr_t)node;
        B0 = *(const __attribute__((address_space(3))) float4 *)rec;
        B1 = *(const __attribute__((address_space(3))) float4 *)(rec + 16);
        const uint32_t lw = *(const __attribute__((address_space(3))) uint32_t *)(rec + 32 + ooff);
        hit = lw & 0xFFFFu;
        miss = lw >> 16;
#else
        B0 = B1 = make_float4(0.0f, 0.0f, 0.0f, 0.0f);
        miss = 0;
#endif
    } else {
        B0 = v.nodes[2 * node];
        B1 = v.nodes[2 * node + 1];
        miss = v.miss32[8 * node + ooff];
    }
    // Slab values b * inv - lo * inv as one fma each, nlo = -(lo * inv) per ray
    // (sphere_slabs): the result is the exact slab value of a face moved by
    // <= u|lo| + 3u|b - lo| (rounded lo * inv, rcp, the fma's rounding), which
    // e_abs = 2e-6 (|o|_1 + M) covers ~8x, so [tn, tf] is the exact interval
    // of a box that still contains every inflated sphere of the node: plain
    // comparisons are safe.  inv is finite (ray setup), so no 0 * inf NaN.
    // lo = o + e, hi = o - e:  (bmin - e) - o == bmin - (o + e)
    const float t0x = __builtin_fmaf(B0.x, inv.x, nlo.x), t1x = __builtin_fmaf(B1.x, inv.x, nhi.x);
    const float t0y = __builtin_fmaf(B0.y, inv.y, nlo.y), t1y = __builtin_fmaf(B1.y, inv.y, nhi.y);
    const float t0z = __builtin_fmaf(B0.z, inv.z, nlo.z), t1z = __builtin_fmaf(B1.z, inv.z, nhi.z);
    const float tn = fmaxf(fmaxf(fminf(t0x, t1x), fminf(t0y, t1y)), fminf(t0z, t1z));
    const float tf = fminf(fminf(fmaxf(t0x, t1x), fmaxf(t0y, t1y)), fmaxf(t0z, t1z));
    // tn > best_t as a signed-integer compare: best_t is positive (or +inf)
    // and tn is finite for any ray that can produce a candidate (inv and the
    // slab offsets are finite), so the orders agree; a NaN ray has no
    // candidate, so skipping for it changes nothing.  (As a float compare the
    // compiler folds it into tn > min(tf, best_t) and canonicalises best_t at
    // every node.)
    const bool skip = tn > tf || tf < 0.001f || __float_as_int(tn) > __float_as_int(best_t);
    if (kLds) {
        // staged leaf word: (first << 3) | count for a leaf (count >= 1), 0 else
        leaf = __float_as_uint(B0.w);
        node = skip ? miss : hit;
        return !skip && leaf != 0u;
    }
    const uint32_t a = __float_as_uint(B0.w);
    const bool is_leaf = (a & kLeafBitDev) != 0;
    // near child first
    const uint32_t child = a + ((ooff >> __float_as_uint(B1.w)) & 1u);
    node = (skip || is_leaf) ? miss : child;
    // (returned as a flag, so the caller branches on it directly; leaf is only
    // read when it is set)
    leaf = ((a & ~kLeafBitDev) << 3) | __float_as_uint(B1.w);
    return !skip && is_leaf;
}

// The walk's first node.  With the LDS tree the root's own box test is
// skipped: the walk starts at the root's near child for the ray's octant (the
// root's `next` link).  The root box holds every tree sphere, so skipping its
// test only forgoes a cull (exact); a ray that starts inside
// the scene's box -- nearly every ray -- enters it anyway (one node test per
// walk fewer).  A one-node tree (the root a leaf) starts at the root.
template <bool kLds>
__device__ __forceinline__ uint32_t sphere_walk_entry(uint32_t root, uint32_t oct, uint32_t nnodes) {
#if defined(__HIP_DEVICE_COMPILE__)
    if (kLds && nnodes > 1u) {
        typedef const __attribute__((address_space(3))) char *lds_cptr;
        return *(const __attribute__((address_space(3))) uint32_t *)((lds_cptr)(uintptr_t)root + 32 + 4u * oct) &
               0xFFFFu;
    }
#endif
    (void)oct;
    (void)nnodes;
    return root;
}

// The walk's per-ray slab offsets for inflation e: nlo = -((o + e) inv),
// nhi = -((o - e) inv).
__device__ __forceinline__ void sphere_slabs(F3 org, F3 inv, float e, F3 &nlo, F3 &nhi) {
    nlo = f3(-((org.x + e) * inv.x), -((org.y + e) * inv.y), -((org.z + e) * inv.z));
    nhi = f3(-((org.x - e) * inv.x), -((org.y - e) * inv.y), -((org.z - e) * inv.z));
}

// Tests a pending leaf.  The node boxes keep the inflation derived from the
// best t at the walk's start: a larger best t only inflates them more (still
// exact), and re-deriving it after every new best (the round-1
// to round-4 code) cost ~20 VALU per improvement for boxes ~1 % tighter.
__device__ __forceinline__ void sphere_leaf(const BvhView &v, F3 org, F3 dir, uint32_t leaf, float &best_t,
                                            int &best_i, uint32_t &sph_tests) {
    const uint32_t first = leaf >> 3, n = leaf & 7u;
#ifndef RT_LEAF_LOOP
    // leaves hold 1 or 2 spheres (leaf size 2): straight-line tests, the loop
    // only for larger leaves (RT_AMD_LEAF)
    sph_tests += n;
    sphere_candidate(v.prims[first], org, dir, (int)v.ids[first], best_t, best_i);
    if (n > 1u) {
        sphere_candidate(v.prims[first + 1], org, dir, (int)v.ids[first + 1], best_t, best_i);
        for (uint32_t j = first + 2; j < first + n; ++j)
            sphere_candidate(v.prims[j], org, dir, (int)v.ids[j], best_t, best_i);
    }
#else
    for (uint32_t j = first; j < first + n; ++j) {
        ++sph_tests;
        sphere_candidate(v.prims[j], org, dir, (int)v.ids[j], best_t, best_i);
    }
#endif
}

// ------------------------------------------------------------ triangle stage
// Triangle::intersect (common.rs:129-166), after the t-range check passed:
// the three edge tests against the hit point o + t*d.
__device__ __forceinline__ bool tri_edges(F3 n, F3 v0, F3 v1, F3 v2, F3 pt) {
    if (dot(n, cross(v1 - v0, pt - v0)) < 0.0f) return false;
    if (dot(n, cross(v2 - v1, pt - v1)) < 0.0f) return false;
    if (dot(n, cross(v0 - v2, pt - v2)) < 0.0f) return false;
    return true;
}

// The reference's plane step and t-range check (common.rs:131-150), with its
// sign: t = (n.o + d) / cos; false when |cos| < 1e-8 or t is out of range.
__device__ __forceinline__ bool tri_plane(float4 N, F3 org, F3 dir, float best_t, float &t) {
    const float cosl = (N.x * dir.x + N.y * dir.y) + N.z * dir.z;
    if (-1e-8f < cosl && cosl < 1e-8f) return false;
    t = (((N.x * org.x + N.y * org.y) + N.z * org.z) + N.w) / cosl;
    return !(t < 0.001f || t > best_t);
}

// Mesh::hit (common.rs:178-223) in file order: t_max = best_t, first wins ties.
__device__ __forceinline__ void triangles_brute(const TraceParams &p, F3 org, F3 dir, float best_t,
                                                float &tri_t, int &tri_i, uint32_t &tri_in) {
    const float tmin = 0.001f;
    for (uint32_t j = 0; j < p.ntri; ++j) {
        const float4 N = p.tri_hot[j];
        const float cosl = (N.x * dir.x + N.y * dir.y) + N.z * dir.z;
        if (-1e-8f < cosl && cosl < 1e-8f) continue;
        const float t = (((N.x * org.x + N.y * org.y) + N.z * org.z) + N.w) / cosl;
        if (t < tmin || t > best_t) continue;
        ++tri_in;
        const float4 *g = p.tri_geo + 4u * j;
        const float4 A = g[0], B = g[1], Cc = g[2];
        if (!tri_edges(f3(N.x, N.y, N.z), f3(A.x, A.y, A.z), f3(B.x, B.y, B.z), f3(Cc.x, Cc.y, Cc.z),
                       org + scale(dir, t)))
            continue;
        if (t < tri_t) { tri_t = t; tri_i = (int)j; }
    }
}

// One triangle in any order, with the reference's winner: the smallest
// accepted t, lowest index on ties (a NaN/inf t is never recorded).
__device__ __forceinline__ bool tri_merge(float t, int idx, float &tri_t, int &tri_i) {
    const bool take = t < tri_t || (t == tri_t && tri_t < __builtin_inff() && idx < tri_i);
    if (take) { tri_t = t; tri_i = idx; }
    return take;
}

// One tree-ordered triangle record (bvh.h TriangleBVH::tris).
__device__ __forceinline__ bool tri_record(const float4 *r, F3 org, F3 dir, float best_t,
                                           float &tri_t, int &tri_i, uint32_t &tri_in) {
    const float4 N = r[0];
    float t;
    if (!tri_plane(N, org, dir, best_t, t)) return false;
    ++tri_in;
    const float4 A = r[1], B = r[2], Cc = r[3];
    if (!tri_edges(f3(N.x, N.y, N.z), f3(A.x, A.y, A.z), f3(B.x, B.y, B.z), f3(Cc.x, Cc.y, Cc.z),
                   org + scale(dir, t)))
        return false;
    return tri_merge(t, (int)__float_as_uint(A.w), tri_t, tri_i);
}

// Triangles through the phantom-aware BVH (bvh.h).  An accepted hit lies on
// its triangle translated by 2(n^.o)n^ (the reference's sign of n.o), up to
// rounding.  Per node the kernel bounds s = n^.o over the node's normal box,
// widens the box by the interval of 2 s m_k on each axis k (m over the normal
// box) plus rho, a rounding margin that dominates every error term
// (<= ~40u (dist + |o| + M)), and skips only nodes the ray
// certainly misses or enters beyond min(best_t, tri_t).
//
// cam (bounce 0, org == camera origin): the lane walks the camera-origin tree
// instead, whose boxes already are the phantoms of that origin padded by rho
// (bvh.h CameraTriangleBVH) -- same step, no widening, so lanes at bounce 0
// and lanes further down their paths do not serialise.
//
// tri_begin: brute-forced triangles, then the walk's margin.  Returns false
// when the walk is not needed (far / non-finite origin: every record is tested
// here instead -- the margins would overflow; same result by the
// order-independent merge).
__device__ __forceinline__ bool tri_begin(const TraceParams &p, F3 org, F3 dir, float best_t,
                                          bool cam, float &rho, float &tri_t, int &tri_i,
                                          uint32_t &tri_in, uint32_t &tri_done) {
    tri_done += p.tloose;
    for (uint32_t k = 0; k < p.tloose; ++k) {  // slivers / non-finite data
        const uint32_t j = p.tbvh_loose[k];
        const float4 N = p.tri_hot[j];
        float t;
        if (!tri_plane(N, org, dir, best_t, t)) continue;
        ++tri_in;
        const float4 *g = p.tri_geo + 4u * j;
        const float4 A = g[0], B = g[1], Cc = g[2];
        if (tri_edges(f3(N.x, N.y, N.z), f3(A.x, A.y, A.z), f3(B.x, B.y, B.z), f3(Cc.x, Cc.y, Cc.z),
                      org + scale(dir, t)))
            tri_merge(t, (int)j, tri_t, tri_i);
    }
    const float onorm = (fabsf(org.x) + fabsf(org.y)) + fabsf(org.z);
    if (!cam && !(onorm < 1e18f)) {
        tri_done += p.ttris;
        for (uint32_t j = 0; j < p.ttris; ++j)
            tri_record(p.tbvh_tris + 4u * j, org, dir, best_t, tri_t, tri_i, tri_in);
        return false;
    }
    // distance from o to any phantom point: |o - c| + radius + 2|o|
    const float dist = ((fabsf(org.x - p.tbvh_c[0]) + fabsf(org.y - p.tbvh_c[1])) +
                        fabsf(org.z - p.tbvh_c[2])) + p.tbvh_r + 2.0f * onorm;
    rho = cam ? 0.0f : 1e-5f * ((dist + onorm) + p.tbvh_mag);
    return true;
}

// One node of the triangle tree (static or camera-origin); an entered leaf is
// handed back in `leaf` as (first << 3) | count, like sphere_node.
__device__ __forceinline__ bool tri_node(const TraceParams &p, F3 nlo, F3 nhi, F3 inv, F3 dlt2, bool cam,
                                         float cap, uint32_t &node, uint32_t &leaf,
                                         uint32_t &node_tests) {
    ++node_tests;
    // Quantised nodes (bvh.h QuantGrid): u16 coordinates decoded with one fma
    // on the tree's grid; the host rounds every face outward *after* this
    // exact decode, so a decoded box contains the float box.
    // one 32-B sector per node: (static) box | normals | a | link,
    // (camera) box | a | link; fixed child-a-first order (bvh.cpp)
    const uint4 *qn = (cam ? p.cam_nodes : p.tbvh_nodes) + 2u * node;
    const uint4 q0 = qn[0], q1 = qn[1];
    const uint32_t a = cam ? q0.w : q1.z;
    const uint32_t miss = cam ? q1.x : q1.w;
    const float gbx = cam ? p.cq_base[0] : p.tq_base[0], gsx = cam ? p.cq_step[0] : p.tq_step[0];
    const float gby = cam ? p.cq_base[1] : p.tq_base[1], gsy = cam ? p.cq_step[1] : p.tq_step[1];
    const float gbz = cam ? p.cq_base[2] : p.tq_base[2], gsz = cam ? p.cq_step[2] : p.tq_step[2];
    auto lo16 = [](uint32_t w) { return (float)(w & 0xFFFFu); };
    auto hi16 = [](uint32_t w) { return (float)(w >> 16); };
    const float4 B0 = make_float4(__builtin_fmaf(lo16(q0.x), gsx, gbx), __builtin_fmaf(hi16(q0.x), gsy, gby),
                                  __builtin_fmaf(lo16(q0.y), gsz, gbz), 0.0f);
    const float4 B1 = make_float4(__builtin_fmaf(hi16(q0.y), gsx, gbx), __builtin_fmaf(lo16(q0.z), gsy, gby),
                                  __builtin_fmaf(hi16(q0.z), gsz, gbz), 0.0f);
    // normal box; the camera tree has none (no widening): its lanes decode
    // with a zero grid, so every word of the node is used on every path and
    // the node stays two 16-B loads (with the decode under `if (!cam)` the
    // compiler split the second half into a dword and a dwordx3 load: three
    // memory instructions per node, C5 +24 %)
    const float nb = cam ? 0.0f : p.tq_nbase, ns = cam ? 0.0f : p.tq_nstep;
    const float4 N0 = make_float4(__builtin_fmaf(lo16(q0.w), ns, nb), __builtin_fmaf(hi16(q0.w), ns, nb),
                                  __builtin_fmaf(lo16(q1.x), ns, nb), 0.0f);
    const float4 N1 = make_float4(__builtin_fmaf(hi16(q1.x), ns, nb), __builtin_fmaf(lo16(q1.y), ns, nb),
                                  __builtin_fmaf(hi16(q1.y), ns, nb), 0.0f);
    // 2s = n^.(2d) over the normal box, d = o - oc (the tree's box origin,
    // bvh.h); dlt2 = 2d is exact, so 2s m below has the bits of 2 (s m)
    const float ax = N0.x * dlt2.x, bx = N1.x * dlt2.x;
    const float ay = N0.y * dlt2.y, by = N1.y * dlt2.y;
    const float az = N0.z * dlt2.z, bz = N1.z * dlt2.z;
    const float sl = (fminf(ax, bx) + fminf(ay, by)) + fminf(az, bz);
    const float sh = (fmaxf(ax, bx) + fmaxf(ay, by)) + fmaxf(az, bz);
    // phantom offset 2 s m_k over 2s in [sl, sh], m_k in [N0.k, N1.k]
    auto widen = [&](float lo, float hi, float m0, float m1, float nl, float nh, float iv, float &t0,
                     float &t1) {
        const float a = sl * m0, b = sl * m1, c = sh * m0, d = sh * m1;
        const float omin = fminf(fminf(a, b), fminf(c, d));
        const float omax = fmaxf(fmaxf(a, b), fmaxf(c, d));
        // (l - (o + rho)) inv and (h - (o - rho)) inv, nl = -((o + rho) inv),
        // nh = -((o - rho) inv) per ray (sphere_slabs with e = rho): the faces
        // move out by rho, plus <= u|o + rho| + 3u|l - o| of rounding, far
        // inside rho
        t0 = __builtin_fmaf(lo + omin, iv, nl);
        t1 = __builtin_fmaf(hi + omax, iv, nh);
    };
    float t0x, t1x, t0y, t1y, t0z, t1z;
    widen(B0.x, B1.x, N0.x, N1.x, nlo.x, nhi.x, inv.x, t0x, t1x);
    widen(B0.y, B1.y, N0.y, N1.y, nlo.y, nhi.y, inv.y, t0y, t1y);
    widen(B0.z, B1.z, N0.z, N1.z, nlo.z, nhi.z, inv.z, t0z, t1z);
    const float tn = fmaxf(fmaxf(fminf(t0x, t1x), fminf(t0y, t1y)), fminf(t0z, t1z));
    const float tf = fminf(fminf(fmaxf(t0x, t1x), fmaxf(t0y, t1y)), fmaxf(t0z, t1z));
    // tn > cap as an integer compare (cap > 0 or +inf; see sphere_node: a
    // NaN tn only comes from a NaN ray, which records no triangle)
    const bool skip = tn > tf || tf < 0.001f || __float_as_int(tn) > __float_as_int(cap);
    // a: child | axis << 29, or leaf bit | first << 3 | count
    const bool is_leaf = (a & kLeafBitDev) != 0;
    const uint32_t child = a & 0x1FFFFFFFu;
    node = (skip || is_leaf) ? miss : child;
    leaf = a & ~kLeafBitDev;  // read only when the flag is set
    return !skip && is_leaf;
}

// One child of a 4-wide static-tree node (bvh.h TriangleBVH::wnodes): the
// same decode, widening and skip rule as tri_node's static branch, from the
// child's six box / normal-box words.  Returns whether the child is entered
// (its entry distance in tn).
__device__ __forceinline__ bool tri_wide_child(const TraceParams &p, uint32_t w0, uint32_t w1, uint32_t w2,
                                               uint32_t w3, uint32_t w4, uint32_t w5, F3 nlo, F3 nhi,
                                               F3 inv, F3 dlt2, float cap, float &tn) {
    auto lo16 = [](uint32_t w) { return (float)(w & 0xFFFFu); };
    auto hi16 = [](uint32_t w) { return (float)(w >> 16); };
    const float gsx = p.tq_step[0], gsy = p.tq_step[1], gsz = p.tq_step[2];
    // normal box: halves (exact in f32), one conversion each
    auto h16lo = [](uint32_t w) { return (float)__builtin_bit_cast(_Float16, (uint16_t)(w & 0xFFFFu)); };
    auto h16hi = [](uint32_t w) { return (float)__builtin_bit_cast(_Float16, (uint16_t)(w >> 16)); };
    // The grid decode is folded into the slab values: nlo / nhi arrive as
    // gb inv + nl and gb inv + nh (the wide walk's set-up), so a face value is
    // (q gs + o) inv + that -- two fmas per face instead of the decode fma, an
    // add and an fma (6 VALU fewer per child; A/B on C5: 149.5 -> 147.6 ms).
    // Rounding: the face moves by <= ~4u (|gb| + |q gs| + |o|) against the
    // exact decode, inside rho = 1e-5 (dist + |o|_1 + M) with the other
    // terms (<= ~40u (dist + |o| + M), tri_begin): the widened box still
    // holds every phantom.
    const float nx0 = h16lo(w3), ny0 = h16hi(w3), nz0 = h16lo(w4);
    const float nx1 = h16hi(w4), ny1 = h16lo(w5), nz1 = h16hi(w5);
    const float ax = nx0 * dlt2.x, bx = nx1 * dlt2.x;
    const float ay = ny0 * dlt2.y, by = ny1 * dlt2.y;
    const float az = nz0 * dlt2.z, bz = nz1 * dlt2.z;
    const float sl = (fminf(ax, bx) + fminf(ay, by)) + fminf(az, bz);
    const float sh = (fmaxf(ax, bx) + fmaxf(ay, by)) + fmaxf(az, bz);
    auto widen = [&](float qlo, float qhi, float m0, float m1, float c0, float c1, float gs, float iv, float &t0,
                     float &t1) {
        const float a = sl * m0, b = sl * m1, c = sh * m0, d = sh * m1;
        const float omin = fminf(fminf(a, b), fminf(c, d));
        const float omax = fmaxf(fmaxf(a, b), fmaxf(c, d));
        t0 = __builtin_fmaf(__builtin_fmaf(qlo, gs, omin), iv, c0);
        t1 = __builtin_fmaf(__builtin_fmaf(qhi, gs, omax), iv, c1);
    };
    float t0x, t1x, t0y, t1y, t0z, t1z;
    widen(lo16(w0), hi16(w1), nx0, nx1, nlo.x, nhi.x, gsx, inv.x, t0x, t1x);
    widen(hi16(w0), lo16(w2), ny0, ny1, nlo.y, nhi.y, gsy, inv.y, t0y, t1y);
    widen(lo16(w1), hi16(w2), nz0, nz1, nlo.z, nhi.z, gsz, inv.z, t0z, t1z);
    tn = fmaxf(fmaxf(fminf(t0x, t1x), fminf(t0y, t1y)), fminf(t0z, t1z));
    const float tf = fminf(fminf(fmaxf(t0x, t1x), fmaxf(t0y, t1y)), fmaxf(t0z, t1z));
    return !(tn > tf || tf < 0.001f || __float_as_int(tn) > __float_as_int(cap));
}

__device__ __forceinline__ void tri_leaf(const TraceParams &p, F3 org, F3 dir, bool cam,
                                         uint32_t leaf, float best_t, float &tri_t, int &tri_i,
                                         uint32_t &tri_in, uint32_t &tri_done, const float4 *wrecs = nullptr) {
    // (wrecs: the wide walk's records, TraceParams::tw_tris)
    const float4 *recs = wrecs ? wrecs : cam ? p.cam_tris : p.tbvh_tris;
    const uint32_t first = leaf >> 3, end = first + (leaf & 7u);
    tri_done += leaf & 7u;
    for (uint32_t j = first; j < end; ++j)
        tri_record(recs + 4u * j, org, dir, best_t, tri_t, tri_i, tri_in);
}

// Job -> (sample, column, row): job = local pixel * spp + s (pixel-major);
// local rows map to image rows through the rank's row blocks (tiles.py);
// row counts from the bottom as ray_trace does (common.rs:327-331).
template <bool kSerial>
__device__ __forceinline__ void job_pixel(const TraceParams &p, uint32_t job, uint32_t &s,
                                          uint32_t &col, uint32_t &row) {
    if (kSerial && p.mode == kRngSerialPixel) {
        // job = local pixel q * E + position: pixel p0 + q (s is not used)
        const uint32_t pix = fdiv(p.cbase, p.div_sspp) + fdiv(job, p.div_spp);
        s = 0;
        row = fdiv(pix, p.div_width);
        col = pix - row * p.width;
        return;
    }
    if (kSerial) {
        // SERIAL passes: job = launch sample * V + variant; frame sample j =
        // (row * W + col) * spp + s in the reference's loop order (common.rs:327-336)
        const uint32_t jl = fdiv(job, p.div_spp);
        const uint32_t j = p.cbase + jl < p.nserial ? p.cbase + jl : p.nserial - 1u;
        const uint32_t pix = fdiv(j, p.div_sspp);
        s = j - pix * p.sspp;
        row = fdiv(pix, p.div_width);
        col = pix - row * p.width;
        return;
    }
    const uint32_t lp = fdiv(job, p.div_spp);
    s = job - lp * p.spp;
    const uint32_t q = fdiv(lp, p.div_width);
    col = lp - q * p.width;
    const uint32_t lr = p.slab_row0 + q;
    const uint32_t blk = fdiv(lr, p.div_rowblock);
    const uint32_t ir = (blk * p.nranks + p.rank) * p.row_block + (lr - blk * p.row_block);
    row = p.height - 1u - ir;
}

// kRngSerialPixel: the stream positions (window indices) local pixel q's
// samples' windows cover: from 2 jf + 3 lo(jf) to 2 jz + 3 (lo(jz) + K - 1),
// jf / jz its first / last sample in the iteration
__device__ __forceinline__ void serial_pixel_span(const TraceParams &p, uint32_t q, uint32_t &plo,
                                                  uint32_t &phi) {
    if (p.spix != nullptr) {  // tabulated by the window kernel: one load
        const uint4 s = p.spix[q];
        plo = s.x;
        phi = s.y;
        return;
    }
    const uint32_t a = p.cbase, ss = p.sspp;
    const uint32_t ln = min(p.sL, p.nserial - a);
    const uint32_t p0 = fdiv(a, p.div_sspp);
    const uint32_t jf = q == 0u ? 0u : (p0 + q) * ss - a;
    const uint32_t jz = min((p0 + q + 1u) * ss - a, ln) - 1u;
    plo = 2u * jf + 3u * p.slo[jf];
    phi = 2u * jz + 3u * (p.slo[jz] + p.sK - 1u);
}

// SERIAL passes: the start state of job (launch sample jl, variant k).
__device__ __forceinline__ uint32_t serial_start(const TraceParams &p, uint32_t job) {
    const uint32_t jl = fdiv(job, p.div_spp);
    const uint32_t k = job - jl * p.spp;
    if (p.mode == kRngSerialCount)
        return p.win[2u * jl + 3u * ((p.slo ? p.slo[jl]
                                            : serial_lo(p.sM, p.cbase, jl, p.spp, (p.max_draws - 2u) / 3u,
                                                        p.nserial)) + k)];
    if (p.mode == kRngSerialCheck) return p.win[p.cbase + jl];
    if (p.mode == kRngSerialPixel) {
        // local pixel q = jl, position plo(q) + k (kept inside the pixel's span:
        // the launch's E is the widest pixel's; jobs past a narrower pixel's
        // span are not traced, serial_pixel_job)
        uint32_t plo, phi;
        serial_pixel_span(p, jl, plo, phi);
        return p.win[min(plo + k, max(phi, plo))];
    }
    return counter_seed(p.seed, (uint64_t)(p.cbase + jl) * p.spp + k);
}

// kRngSerialPixel: false for a job past its pixel's span (the lane stays idle)
__device__ __forceinline__ bool serial_pixel_job(const TraceParams &p, uint32_t job) {
    const uint32_t q = fdiv(job, p.div_spp);
    uint32_t plo, phi;
    serial_pixel_span(p, q, plo, phi);
    return plo + (job - q * p.spp) <= phi;
}

// Primary ray against its pixel strip's candidate records (bvh.h
// PrimaryTriLists) plus the `always` records, in any order (tri_merge).
template <bool kSerial>
__device__ __forceinline__ void tri_primary_list(const TraceParams &p, uint32_t job, F3 org, F3 dir,
                                                 float best_t, float &tri_t, int &tri_i,
                                                 uint32_t &tri_in, uint32_t &tri_done) {
    uint32_t s, col, row;
    job_pixel<kSerial>(p, job, s, col, row);
    const uint32_t strip = row * p.ptl_spr + col / kPrimaryTriStripW;
    const uint32_t b = p.ptl_off[strip], e = p.ptl_off[strip + 1];
    tri_done += (e - b) + (p.ptl_end - p.ptl_always);
    for (uint32_t j = b; j < e; ++j)
        tri_record(p.cam_tris + 4u * p.ptl_items[j], org, dir, best_t, tri_t, tri_i, tri_in);
    for (uint32_t j = p.ptl_always; j < p.ptl_end; ++j)
        tri_record(p.cam_tris + 4u * p.ptl_items[j], org, dir, best_t, tri_t, tri_i, tri_in);
}

// One resolved pixel: gamma + `as u8` (common.rs:344-356), RGBA8 at the
// tile row of launch-local pixel lp.
__device__ __forceinline__ void resolve_store(const TraceParams &p, uint32_t lp, float r, float g,
                                              float b) {
    const uint32_t R = sat_u8(__builtin_sqrtf(r * p.inv_spp) * 255.999f);
    const uint32_t G = sat_u8(__builtin_sqrtf(g * p.inv_spp) * 255.999f);
    const uint32_t B = sat_u8(__builtin_sqrtf(b * p.inv_spp) * 255.999f);
    const uint32_t q = fdiv(lp, p.div_width);
    const uint32_t col = lp - q * p.width;
    p.out[(size_t)(p.slab_row0 + q) * p.width + col] = R | (G << 8) | (B << 16) | (p.alpha_u8 << 24);
}

// Fused resolve of one finished chunk (wave-uniform call, all lanes active):
// jobs [base, base + len) are whole pixels (chunks and partitions are
// pixel-aligned), their samples sit at ring offset `off` of the wave's ring
// (planes `plane` floats apart).  Each pixel's samples are summed in order
// (common.rs:333-341, the same fold as resolve_kernel).  The samples were
// stored by this wave: a workgroup-scope fence orders them (one CU, one L1).
//
// One lane per (pixel, plane) when 3 * pixels <= 64 and spp % 4 == 0: lane
// c * np + g folds plane c of pixel g in sample order from float4 loads (4
// in flight per round), then the pixel's lane collects the G and B sums with
// two shuffles: spp adds and spp / 4 loads per lane (A/B on C2 -1.7 %
// against folding float4 groups through ds_bpermute, 3 * spp bpermutes and
// adds per pixel).  Other chunks, and the triangle kernels (kPlaneLanes
// false: at their 64-VGPR cap the float4 rounds spill, C5 +7 %), sum one
// pixel per lane.
// which kernel families fold with plane lanes: the sphere kernels and the
// wide triangle walk (A/B on C5, 1-pixel chunks: 149.8 -> 148.1 ms, 2 VGPRs
// spilled); the binary triangle walk keeps one lane per pixel
#define RT_PLANE_LANES(mesh) ((mesh) < 2 || (mesh) == 3)
template <bool kPlaneLanes>
__device__ __forceinline__ void resolve_chunk(const TraceParams &p, const float *ring, uint32_t plane,
                                              uint32_t off, uint32_t base, uint32_t len,
                                              uint32_t lane) {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
    const uint32_t spp = p.spp;
    const uint32_t np = fdiv(len, p.div_spp), pix0 = fdiv(base, p.div_spp);
    if (kPlaneLanes && 3u * np <= kWave && (spp & 3u) == 0) {
        const uint32_t c = lane >= np ? (lane >= 2u * np ? 2u : 1u) : 0u;
        const uint32_t g = lane - c * np;
        const bool on = lane < 3u * np;
        const float *src = ring + off + c * plane + (on ? g : 0u) * spp;
        float acc = 0.0f;
        for (uint32_t k = 0; k < spp; k += 16u) {
            float4 v[4];
#pragma unroll
            for (uint32_t q = 0; q < 4; ++q) {
                v[q] = make_float4(0.0f, 0.0f, 0.0f, 0.0f);
                if (on && k + 4u * q < spp) v[q] = *reinterpret_cast<const float4 *>(src + k + 4u * q);
            }
#pragma unroll
            for (uint32_t q = 0; q < 4; ++q) {
                if (k + 4u * q < spp) {  // (wave-uniform)
                    acc = acc + v[q].x;
                    acc = acc + v[q].y;
                    acc = acc + v[q].z;
                    acc = acc + v[q].w;
                }
            }
        }
        const float sg = __shfl(acc, (int)(lane < np ? np + lane : lane));
        const float sb = __shfl(acc, (int)(lane < np ? 2u * np + lane : lane));
        if (lane < np) resolve_store(p, pix0 + lane, acc, sg, sb);
        return;
    }
    for (uint32_t i = lane; i < np; i += kWave) {
        const float *src = ring + off + i * spp;
        float r = 0.0f, g = 0.0f, b = 0.0f;
        for (uint32_t k = 0; k < spp; ++k) {
            r = r + src[k];
            g = g + src[plane + k];
            b = b + src[2 * plane + k];
        }
        resolve_store(p, pix0 + i, r, g, b);
    }
}

// The sphere tree's view for a kernel; kLds: copied into the workgroup's LDS
// (one barrier).  Returns the walk's first node (its LDS address with kLds).
// LDS layout: node records (64 B: box float4 x 2 | 8 x u32 links) | prims
// (float4) | shade (2 x float4 / sphere) | ids (u32) | kinds (u32), at the
// start of the dynamic LDS (trace_lds_bytes).  A record is
//   (lo.xyz, leaf word) (hi.xyz, 0) and, per ray octant o, the u32
//   next(o) | miss(o) << 16: the node to visit when the box is entered (the
//   near child along the split axis for the octant's sign, the DFS order of
//   bvh.h; a leaf's own miss link) and when it is skipped,
// with the leaf word (first << 3) | count for leaves and 0 for inner nodes.
// Node references are record LDS addresses (base + index * 64; the kernels
// have no static LDS before it, so base is 0 and they stay below 0xFFFF: the
// copy holds <= kLdsTreeMaxNodes nodes); 0xFFFF stays the end marker.
template <bool kLds>
__device__ __forceinline__ uint32_t stage_tree(const TraceParams &p, float4 *lds, BvhView &view) {
    if (!kLds) {
        view = BvhView{p.bvh_nodes, p.bvh_miss, nullptr, p.bvh_prims, p.bvh_prim_id,
                       p.sph_shade, p.sph_kind};
        return 0;
    }
    float4 *n4 = lds;
    const uint32_t lbase = (uint32_t)(uintptr_t)(__attribute__((address_space(3))) float4 *)lds;
    float4 *p4 = n4 + 4 * p.nnodes;
    float4 *s4 = p4 + p.nprims;
    uint32_t *id = reinterpret_cast<uint32_t *>(s4 + 2 * p.nsph_padded);
    uint32_t *kd = id + p.nprims;
    const uint16_t *g16 = p.bvh_miss16;
    auto addr = [&](uint32_t l) { return l == 0xFFFFu ? 0xFFFFu : lbase + l * 64u; };
    for (uint32_t i = threadIdx.x; i < p.nnodes; i += blockDim.x) {
        float4 b0 = p.bvh_nodes[2 * i];
        const uint32_t a = __float_as_uint(b0.w);
        float4 b1 = p.bvh_nodes[2 * i + 1];
        const bool is_leaf = (a & kLeafBitDev) != 0;
        const uint32_t axis = __float_as_uint(b1.w);  // (leaves: the count)
        b0.w = __uint_as_float(is_leaf ? ((a & ~kLeafBitDev) << 3) | axis : 0u);
        b1.w = 0.0f;
        n4[4 * i] = b0;
        n4[4 * i + 1] = b1;
        uint32_t w[8];
        for (uint32_t o = 0; o < 8; ++o) {
            const uint32_t miss = addr(g16[8 * i + o]);
            const uint32_t next = is_leaf ? miss : lbase + (a + ((o >> axis) & 1u)) * 64u;
            w[o] = next | (miss << 16);
        }
        n4[4 * i + 2] = make_float4(__uint_as_float(w[0]), __uint_as_float(w[1]), __uint_as_float(w[2]),
                                    __uint_as_float(w[3]));
        n4[4 * i + 3] = make_float4(__uint_as_float(w[4]), __uint_as_float(w[5]), __uint_as_float(w[6]),
                                    __uint_as_float(w[7]));
    }
    for (uint32_t i = threadIdx.x; i < p.nprims; i += blockDim.x) {
        p4[i] = p.bvh_prims[i];
        id[i] = p.bvh_prim_id[i];
    }
    for (uint32_t i = threadIdx.x; i < p.nsph_padded; i += blockDim.x) {
        s4[2 * i] = p.sph_shade[2 * i];
        s4[2 * i + 1] = p.sph_shade[2 * i + 1];
        kd[i] = p.sph_kind[i];
    }
    __syncthreads();
    view = BvhView{n4, nullptr, nullptr, p4, id, s4, kd};
    return lbase;
}

// ------------------------------------------------------------ trace kernel
// kBvh: sphere search through the exact BVH (else brute force).  kLds: the
// tree is copied into the workgroup's LDS once (persistent grid), so every
// traversal step is a ds_read instead of an L2 round trip.  kStep: the BVH
// walks are cut into slices of p.steps nodes, so lanes that finish early are
// shaded and refilled while the wave's long walks continue (triangle scenes:
// walk lengths vary by 10-100x); without it a lane walks to the end in one
// iteration (cheaper per node: sphere-only scenes).
// 6 waves per SIMD = 80 VGPRs: 3 LDS workgroups of 512 per CU (A/B: 5 waves ->
// 2 workgroups costs ~6% at C2)
#ifndef RT_WAVES_PER_EU
#define RT_WAVES_PER_EU 6
#endif
// Waves per SIMD of the lean (uncounted) triangle-scene kernels.  A/B on C5:
// with 256-node walk slices 8 waves beat 6 (264 vs 272 ms; 7: 274), with
// 128- or 96-node slices 6 waves win again (242 / 240 vs 248 / 251 ms at 8).
// The counting variants use RT_WAVES_PER_EU; the host queries occupancy per
// variant (trace_occupancy).
#ifndef RT_WAVES_PER_EU_MESH
#define RT_WAVES_PER_EU_MESH 6
#endif
// LDS workgroup of the sphere-only kernel: 1024 threads, 2 per CU (8 waves
// per SIMD, RT_WAVES_PER_EU_SPHERES).  History (A/B, one process): round 1,
// 512 -> 6.77 ms, 768 -> 6.73, 896 -> 8.41, 1024 -> 7.78 (then the per-wave ray
// state thrashed the L1); round 2, 256 -> 7.90, 384 -> 6.15, 512 -> 5.42 = 768,
// and on the 8-rank tile 768 beat 512 by 3 %.  Round 4, after the kernarg
// reloads freed the SGPRs (profiles/round4_occ/ab_occ_*.log, rank_occ_*.log):
// 768 -> 1024 at 8 waves: C2 4.449 -> 4.444 ms, C3 66.86 -> 62.23 ms, C2 tiles
// of 2 / 8 ranks 2.389 -> 2.336 / 0.772 -> 0.781 ms, C3 8-rank tile 8.78 ->
// 8.33 ms; 896 (7 waves) -> one workgroup per CU, 6.0 ms.  The counting and
// SERIAL sphere variants keep 768 threads at RT_WAVES_PER_EU: at 8 waves their
// extra state spills VGPRs to scratch.
#ifndef RT_WAVES_PER_EU_SPHERES
#define RT_WAVES_PER_EU_SPHERES 8
#endif
#ifndef RT_LDS_BLOCK_SPHERES
#define RT_LDS_BLOCK_SPHERES 1024
#endif
// (the sphere kernels without the LDS tree, 256 threads: A/B 8 vs 6 waves,
// global-memory tree at C2 6.01 vs 5.99 ms, brute force 2.39 vs 2.32 ms)
#ifndef RT_WAVES_PER_EU_SPHERES_GLOBAL
#define RT_WAVES_PER_EU_SPHERES_GLOBAL 6
#endif
#ifndef RT_LDS_BLOCK_SPHERES_AUX
#define RT_LDS_BLOCK_SPHERES_AUX 768
#endif
// LDS workgroup of the triangle-scene kernels (A/B on C5: 256 -> 223 ms,
// 512 -> 221, 768 -> 225)
#ifndef RT_LDS_BLOCK_MESH
#define RT_LDS_BLOCK_MESH 512
#endif
// kMesh: the scene has triangles (else the whole Mesh::hit stage compiles
// away, which keeps the sphere-only kernel's register allocation small).
// kSerial: the SERIAL-mode passes (render.h kRngSerial*): jobs are (sample,
// variant) pairs and store scatter counts -- a separate instance, so the frame
// kernels carry none of its registers.
// kind: 0 lean frame kernel, 1 counting frame kernel, 2 SERIAL pass
// Waves per SIMD of the wide triangle walk (kMesh 3; 80 VGPRs at 6)
#ifndef RT_WAVES_PER_EU_WIDE
#define RT_WAVES_PER_EU_WIDE 6
#endif
#ifndef RT_LDS_BLOCK_WIDE
#define RT_LDS_BLOCK_WIDE 512
#endif
constexpr uint32_t trace_threads(bool lds, int mesh, int kind) {
    return !lds ? 256u : mesh == 3 ? (uint32_t)RT_LDS_BLOCK_WIDE : mesh ? (uint32_t)RT_LDS_BLOCK_MESH
                       : kind == 0 ? (uint32_t)RT_LDS_BLOCK_SPHERES : (uint32_t)RT_LDS_BLOCK_SPHERES_AUX;
}
constexpr int trace_waves_per_eu(bool lds, int mesh, int kind) {
    return kind != 0 ? RT_WAVES_PER_EU : mesh == 3 ? RT_WAVES_PER_EU_WIDE : mesh ? RT_WAVES_PER_EU_MESH
                       : lds ? RT_WAVES_PER_EU_SPHERES : RT_WAVES_PER_EU_SPHERES_GLOBAL;
}
template <bool kBvh, bool kLds, bool kStep, int kMesh, bool kCount, bool kSerial = false>
__global__ __launch_bounds__(trace_threads(kLds, kMesh, kSerial ? 2 : kCount ? 1 : 0))
__attribute__((amdgpu_waves_per_eu(trace_waves_per_eu(kLds, kMesh, kSerial ? 2 : kCount ? 1 : 0), 8)))
void trace_kernel(TraceParams p) {
    // SERIAL count passes: the walk of the previous pass set the first sample
    // and this iteration's candidates per sample (ctrl[5], <= the launch's K)
    if (kSerial && p.ctrl != nullptr) {
        if (p.ctrl[0] != 0u) return;
        p.cbase = p.ctrl[4];  // (the walks advance it)
        const uint32_t K = p.ctrl[5];
        if (p.mode == kRngSerialCount && K != 0u && K < p.spp) {
            // (chunks of whole samples stay whole samples, about as many jobs per atomic)
            if (p.chunk % p.spp == 0u) p.chunk = (p.chunk / K) * K;
            p.spp = K;
            p.div_spp = make_fastdiv(K);
            p.njobs = p.npix * K;
        }
        if (p.mode == kRngSerialPixel) {
            // this iteration's pixels and positions per pixel (the launch was
            // sized for their bounds): job = local pixel q * E + e
            p.sK = K != 0u && K < p.sK ? K : p.sK;  // (serial_k)
            const uint32_t E = min(p.ctrl[7], p.spp);
            const uint32_t ln = min(p.sL, p.nserial - p.cbase);
            const uint32_t p0 = fdiv(p.cbase, p.div_sspp);
            const uint32_t npq = E ? fdiv(p.cbase + ln - 1u, p.div_sspp) - p0 + 1u : 0u;
            p.spp = max(E, 1u);
            p.div_spp = make_fastdiv(p.spp);
            p.npix = npq;
            p.njobs = npq * E;
        }
    }
    // frames: zero the other job-counter set for the launch after this one
    // (stream order: it starts once this grid has finished)
    if (!kSerial && p.job_counter_next != nullptr && blockIdx.x == 0)
        for (uint32_t i = threadIdx.x; i < kMaxJobParts; i += blockDim.x) p.job_counter_next[32u * i] = 0u;
    const uint32_t lane = __lane_id();
    // Each section of the loop (ray setup, sphere walk, triangle setup and
    // walk, shading, the chunk resolve, the refill) re-reads the parameters it
    // needs from the kernarg segment (scalar loads through a pointer the
    // compiler must treat as changed each time) instead of holding all of
    // them in SGPRs across the whole loop: the lean C2 kernel spilled 92 SGPRs
    // to VGPR lanes (252 v_readlane / v_writelane in its code), the C5 kernel
    // 191 plus 13 VGPRs to scratch; now 7 and 0 (+3 VGPRs).  A/B in one
    // process (tools/ab.py, lean frames): C2 4.638 -> 4.451 ms, C3 69.61 ->
    // 66.86 ms, C5 175.1 -> 170.9 ms (profiles/round4_kargs/).
    // RT_NO_KARG_RELOAD builds the previous code.
    // (SERIAL passes rewrite fields of their copy of p at entry -- cbase, spp,
    // the divider, njobs -- so they keep reading that copy)
    auto kargs = [&]() -> const TraceParams & {
#if defined(__HIP_DEVICE_COMPILE__) && !defined(RT_NO_KARG_RELOAD)
        if (kSerial) return p;
        const __attribute__((address_space(4))) TraceParams *kp =
            (const __attribute__((address_space(4))) TraceParams *)__builtin_amdgcn_kernarg_segment_ptr();
        asm volatile("" : "+s"(kp));
        return *(const TraceParams *)kp;
#else
        return p;
#endif
    };
    extern __shared__ float4 lds[];
    BvhView view;
    const uint32_t sph_root = stage_tree<kLds>(p, lds, view);  // the sphere walk's first node
    // kMesh 3: the lane's stack of wide-node indices (u16, entry k at
    // tstack[k * blockDim.x]) after the sphere tree's LDS copy
    uint16_t *const tstack = reinterpret_cast<uint16_t *>(
                                 reinterpret_cast<char *>(lds) +
                                 (kLds ? (trace_tree_lds(p.nnodes, p.nprims, p.nsph_padded) + 15u) & ~(size_t)15u
                                       : 0u)) + threadIdx.x;
    uint32_t tsp = 0;  // (kMesh 3) entries on the stack

    F3 org = f3(0, 0, 0), dir = f3(0, 0, 0), inv = f3(0, 0, 0);
    float thr_r = 1.0f, thr_g = 1.0f, thr_b = 1.0f;  // ray_color's final_color
    uint32_t rng = 0, slot = ~0u, bounce = 0;  // slot ~0: no finished sample to count
    uint32_t nscat = 0;  // (kSerial) the sample's diffuse/metal scatters so far
    uint32_t spl0 = 0, spl1 = kSphListWalk << 16;  // the pixel's primary sphere list (p.spl)
    // lane state between loop iterations (see the bounce loop below)
    enum : uint32_t { kSetup = 0, kSph = 1, kTriInit = 2, kTri = 3, kShade = 4 };
    uint32_t phase = kSetup, node = 0, oct = 0;
    float best_t = 0.0f, tri_t = 0.0f, e = 0.0f;  // e: the triangle walk's margin rho
    int best_i = -1, tri_i = -1;
    bool active = false;
    uint32_t rays = 0, tri_in = 0, sph_tests = 0, node_tests = 0, tnode_tests = 0,
             tri_done = 0;
    // iteration mix (counting variant, lane 0's view; wave-uniform): loop
    // iterations, iterations that walked the sphere tree, active lanes summed
    // over all iterations and over the walking ones (RT_AMD_ITER_DEBUG)
    uint32_t it_all = 0, it_walk = 0, lanes_all = 0, lanes_walk = 0;
#ifdef RT_WALK_MIX
    // diagnostic build only (counting variant): per sphere walk, the walk
    // loop's iterations, those in which some lane tested a leaf, and the leaf
    // loop's sphere trips (each the longest-active lane's view)
    uint32_t wm_iters = 0, wm_leaf_iters = 0, wm_leaf_trips = 0, wm_walks = 0;
#endif

    uint32_t pool_next = 0, pool_end = 0;  // wave-uniform job pool
    // (kSerial pixel pass) jobs [gap_lo, gap_lo + gap_len) of the pool are not
    // handed out: the pool counts jobs without them (copied table entries)
    uint32_t gap_lo = ~0u, gap_len = 0;
    bool exhausted = false;

    // Where a finished sample goes: the slab (slot = job) or, with the fused
    // resolve, the wave's ring (slot = ring offset = (k << ring_shift) + job -
    // rbase[k] for the chunk in ring slot k).  All wave-uniform.
    const bool fused = p.ring != nullptr;
    const uint32_t wave_id = __builtin_amdgcn_readfirstlane(blockIdx.x * (blockDim.x / kWave) +
                                                            threadIdx.x / kWave);
    float *const sbase = fused ? p.ring + (size_t)wave_id * (3u * kTraceRing << p.ring_shift)
                               : p.samples;
    const uint32_t pstride = fused ? (kTraceRing << p.ring_shift) : p.njobs;
    uint32_t rfree = (1u << kTraceRing) - 1u;  // ring slots not holding a chunk
    uint32_t rbase[kTraceRing], rlen[kTraceRing], rleft[kTraceRing];  // chunk jobs, samples not done
#pragma unroll
    for (uint32_t k = 0; k < kTraceRing; ++k) rbase[k] = rlen[k] = rleft[k] = 0;
    uint32_t cur_off = 0;  // slot - job for the pool's chunk
    // a lane's job from its slot (tri_primary_list needs the pixel)
    auto lane_job = [&](uint32_t sl) -> uint32_t {
        if (!fused) return sl;
        const uint32_t k = sl >> p.ring_shift;
        uint32_t b = rbase[0];
#pragma unroll
        for (uint32_t i = 1; i < kTraceRing; ++i) b = k == i ? rbase[i] : b;
        return b + (sl & ((1u << p.ring_shift) - 1u));
    };

#ifdef RT_WAVE_TIMES
    // diagnostic build only: per-wave timeline on the 100 MHz constant clock
    // (start, last chunk pulled, queue found empty, exit; tools/tail_probe.py)
    const uint64_t wt_start = __builtin_amdgcn_s_memrealtime();
    uint64_t wt_pull = wt_start, wt_exh = wt_start;
    uint32_t wt_jobs_tail = 0;  // jobs claimed in the wave's last chunk
#endif
#ifdef RT_STAMPS
    // diagnostic build only: wave cycles per loop segment (s_memtime deltas):
    // 0 direction normalisation + loop back, 1 ray setup, 2 walks, 3 shading,
    // 4 sample store, 5 fused resolve, 6 refill, 7 (unused)
    uint64_t stamp_acc[kStampSegs] = {0, 0, 0, 0, 0, 0, 0, 0};
    uint64_t stamp_prev = __builtin_amdgcn_s_memtime();
#define RT_STAMP(k)                                                       \
    do {                                                                  \
        __builtin_amdgcn_sched_barrier(0);                                \
        const uint64_t t_ = __builtin_amdgcn_s_memtime();                 \
        __builtin_amdgcn_sched_barrier(0);                                \
        stamp_acc[k] += t_ - stamp_prev;                                  \
        stamp_prev = t_;                                                  \
    } while (0)
#else
#define RT_STAMP(k) \
    do {            \
    } while (0)
#endif
    // Job queue: the launch's jobs are split into p.nparts equal partitions,
    // each with its own counter on its own 128-B line (one shared counter
    // serialises at ~12 ns per atomic: 6 ms per C2 frame).  A wave starts on
    // its home partition and moves on when that one is drained.
    uint32_t part = (blockIdx.x * (blockDim.x / kWave) + threadIdx.x / kWave) % p.nparts;
    uint32_t tries = 0;  // partitions found drained (wave-uniform)
    // (pixel-aligned, so every chunk holds whole pixels: the fused resolve)
    auto part_begin = [&](uint32_t k) -> uint32_t {
        return (uint32_t)(((uint64_t)k * p.npix) / p.nparts) * p.spp;
    };
    uint32_t pbegin = part_begin(part), pend = part_begin(part + 1);
    uint32_t prefetch = 0;          // lane 0: counter value of the next chunk, fetched early
    bool prefetch_pending = false;  // wave-uniform
    for (;;) {
        // Directions that need NVec3::new (maths.rs:111-118) this iteration: the
        // scattered rays' and the new primary rays' share one normalisation.
        F3 vdir = dir;
        bool renorm = false;
        bool done = false;
        bool walked = false;  // (kCount: the iteration mix)
        const uint32_t nact = kCount ? (uint32_t)__popcll(__ballot(active)) : 0u;
        if (active) {
            // ---- ray_color's bounce loop (common.rs:267-282) as a lane state
            // machine: setup -> sphere walk -> triangle walk -> shade.  The walks
            // advance at most p.steps nodes per loop iteration, so lanes whose
            // search ends early are shaded and refilled while the others walk on.
            float out_r = 0.0f, out_g = 0.0f, out_b = 0.0f;
            if (phase == kSetup) {
                const TraceParams &p = kargs();  // (ray setup: see kargs)
                if ((int32_t)bounce >= p.depth) {
                    done = true;  // depth exhausted -> (0, 0, 0) (common.rs:284)
                } else {
                    ++rays;
                    // slab-test reciprocals only (not reference arithmetic): v_rcp_f32's
                    // 1-ulp error moves a slab face by <= 4u|b - lo|, inside e_abs and
                    // rho.  Clamped to +-1e20 (+-0 -> +-1e20, sign kept)
                    // so slab products stay finite: an axis with |d| < 1e-20 gets its
                    // t values scaled by 1e20|d| < 1, which keeps its interval's sign
                    // pattern -- the ray lies inside that (inflated) slab for any
                    // finite hit, and the scaled interval still spans [0, >1e9].
                    inv = f3(slab_rcp(dir.x), slab_rcp(dir.y), slab_rcp(dir.z));
                    oct = (inv.x < 0.0f ? 1u : 0u) | (inv.y < 0.0f ? 2u : 0u) | (inv.z < 0.0f ? 4u : 0u);
                    // World::hit, spheres in order with shrinking t_max (common.rs:241-247)
                    best_t = __builtin_inff();
                    best_i = -1;
                    if (kBvh) {
                        spheres_big(p, org, dir, best_t, best_i);
                        node = sphere_walk_entry<kLds>(sph_root, oct, p.nnodes);
                        // (RT_AMD_ABLATE=1: timing-only diagnostic, results are wrong)
                        phase = (p.ablate & 1u) ? kTriInit : kSph;
                        if (!kMesh && bounce == 0 && (spl1 >> 16) != kSphListWalk) {
                            // primary ray: the pixel's candidate spheres instead of
                            // the walk (bvh.h PrimarySphereLists; same candidate
                            // arithmetic and (t, index) argmin as sphere_leaf)
                            const uint32_t nc = spl1 >> 16;
                            sph_tests += nc;
                            if (nc > 0) sphere_candidate(view.prims[spl0 & 0xFFFFu], org, dir,
                                                         (int)view.ids[spl0 & 0xFFFFu], best_t, best_i);
                            if (nc > 1) sphere_candidate(view.prims[spl0 >> 16], org, dir,
                                                         (int)view.ids[spl0 >> 16], best_t, best_i);
                            if (nc > 2) sphere_candidate(view.prims[spl1 & 0xFFFFu], org, dir,
                                                         (int)view.ids[spl1 & 0xFFFFu], best_t, best_i);
                            phase = kTriInit;
                        }
                    } else {
                        spheres_brute(p, org, dir, best_t, best_i);
                        phase = kTriInit;
                    }
                }
            }
            RT_STAMP(1);
            // kStep: at most p.steps node visits per lane per iteration
            uint32_t budget = p.steps;
            // walk_min (sphere-only scenes): while fewer than walk_min lanes wait
            // for a walk and other lanes can advance without one (fresh samples
            // whose primary sphere list replaced the walk), skip this
            // iteration's walk: those lanes are shaded now and join the next
            // walk, so fewer walk segments run with lanes idle in them
            bool walk_now = true;
            if (!kMesh && p.walk_min != 0) {
                const uint32_t nwalk = (uint32_t)__popcll(__ballot(phase == kSph));
                const uint32_t nother = (uint32_t)__popcll(__ballot(phase != kSph && !done));
                walk_now = nwalk >= p.walk_min || nother == 0;
            }
            if (kBvh && phase == kSph && walk_now) {
                const TraceParams &p = kargs();  // (see kargs)
                walked = true;
                constexpr uint32_t kEnd = kLds ? 0xFFFFu : kNodeEndDev;
                const SphBound bnd = sph_bound(p, org);
                F3 nlo, nhi;
                sphere_slabs(org, inv, sph_inflation(p, bnd, best_t), nlo, nhi);
                const uint32_t ooff = kLds ? 4u * oct : oct;
#ifdef RT_WALK_MIX
                uint32_t wi = 0, wl = 0, wt = 0;
#endif
                do {
                    uint32_t leaf;
                    const bool lf = sphere_node<kLds>(view, inv, ooff, best_t, nlo, nhi, node, leaf, node_tests);
#ifdef RT_WALK_MIX
                    if (kCount) {
                        ++wi;
                        const bool any1 = __ballot(lf) != 0;
                        const bool any2 = __ballot(lf && (leaf & 7u) >= 2u) != 0;
                        wl += any1 ? 1u : 0u;
                        wt += any2 ? 2u : any1 ? 1u : 0u;
                    }
#endif
                    if (lf) sphere_leaf(view, org, dir, leaf, best_t, best_i, sph_tests);
                } while (node != kEnd && (!kStep || --budget != 0));
#ifdef RT_WALK_MIX
                if (kCount) {
                    // (wave maxima over the walking lanes: the longest-active lane saw every iteration)
                    for (uint32_t off = 1; off < kWave; off <<= 1) {
                        wi = max(wi, (uint32_t)__shfl_xor((int)wi, (int)off));
                        wl = max(wl, (uint32_t)__shfl_xor((int)wl, (int)off));
                        wt = max(wt, (uint32_t)__shfl_xor((int)wt, (int)off));
                    }
                    wm_iters += wi;
                    wm_leaf_iters += wl;
                    wm_leaf_trips += wt;
                    wm_walks += 1u;
                }
#endif
                if (node == kEnd) phase = kTriInit;
            }
            if (phase == kTriInit) {
                const TraceParams &p = kargs();  // (see kargs)
                // Mesh::hit with t_max = best_t, own closest from +inf (common.rs:178-223)
                tri_t = __builtin_inff();
                tri_i = -1;
                phase = kShade;
                if (kMesh == 0) {
                    // no triangles: Mesh::hit finds nothing
                } else if (kMesh >= 2) {  // (p.tnodes != 0)
                    // (kMesh 3: every lane walks the static tree's wide image)
                    const bool cam = kMesh == 2 && bounce == 0 && p.cam_nnodes != 0;
                    if (tri_begin(p, org, dir, best_t, cam, e, tri_t, tri_i, tri_in, tri_done)) {
                        // (the lists index the camera-origin records, which exist
                        // without the camera tree's nodes: runtime.cpp prepare_camera)
                        if (bounce == 0 && p.ptl_off != nullptr) {
                            tri_primary_list<kSerial>(p, lane_job(slot), org, dir, best_t, tri_t, tri_i, tri_in,
                                             tri_done);
                        } else {
                            node = 0;
                            tsp = 0;
                            phase = kTri;
                        }
                    }
                } else {
                    triangles_brute(p, org, dir, best_t, tri_t, tri_i, tri_in);
                }
            }
            bool tri_now = true;
            if (kMesh >= 2 && p.tri_walk_min != 0) {
                const uint32_t nwalk = (uint32_t)__popcll(__ballot(phase == kTri));
                const uint32_t nother = (uint32_t)__popcll(__ballot(phase != kTri && !done));
                tri_now = nwalk >= p.tri_walk_min || nother == 0;
            }
            if (kMesh == 2 && phase == kTri && tri_now) {
                const TraceParams &p = kargs();  // (see kargs)
                if (kStep) budget = max(budget, p.steps / 2u);  // a lane that just left the sphere walk
                const bool cam = bounce == 0 && p.cam_nnodes != 0;
                const F3 dlt2 = f3(2.0f * (org.x - p.tbvh_oc[0]), 2.0f * (org.y - p.tbvh_oc[1]),
                                   2.0f * (org.z - p.tbvh_oc[2]));
                // rho (e; 0 on the camera tree) folded into the slab offsets
                F3 nlo, nhi;
                sphere_slabs(org, inv, e, nlo, nhi);
                float cap = fminf(best_t, tri_t);
                do {
                    uint32_t leaf;
                    if (tri_node(p, nlo, nhi, inv, dlt2, cam, cap, node, leaf, tnode_tests)) {
                        tri_leaf(p, org, dir, cam, leaf, best_t, tri_t, tri_i, tri_in, tri_done);
                        cap = fminf(best_t, tri_t);
                    }
                } while (node != kNodeEndDev && (!kStep || --budget != 0));
                if (node == kNodeEndDev) phase = kShade;
            }
            if (kMesh == 3 && phase == kTri && tri_now) {
                // The static tree's 4-wide image: one 128-B record per step
                // holds four children's boxes (one round trip where the binary
                // walk takes about four; tools/tbvh_sim.cpp SIM_WIDE=4: 584 ->
                // 146 dependent node loads per secondary ray, the same box
                // tests).  Leaf children are tested at once; of the internal
                // children that are entered, the nearest is walked next and the
                // others are pushed on the lane's LDS stack (A/B on C5 against
                // the lowest slot next: 151.0 -> 150.5 ms).  Any order is exact
                // (tri_merge keeps the (t, index) argmin).
                const TraceParams &p = kargs();  // (see kargs)
                uint32_t wbudget = p.wsteps;
                // Per-origin-cell trees (RT_AMD_TRI_CELLS, off by default): the
                // tree whose phantoms were built for the centre of the cell the
                // origin lies in (the static tree, tc_ncells, outside every cell).
                // The origin does not change during the walk, so every slice
                // picks the same tree.  Any tree is exact for any origin: the
                // widening below covers o - oc (bvh.h TriangleCells).
                F3 oc = f3(p.tbvh_oc[0], p.tbvh_oc[1], p.tbvh_oc[2]);
                uint32_t tree = 0;  // (one register across the walk: the bases follow from it)
                if (p.tc_ncells != 0u) {
                    const float fx = floorf((org.x - p.tc_lo[0]) * p.tc_inv_size);
                    const float fy = floorf((org.y - p.tc_lo[1]) * p.tc_inv_size);
                    const float fz = floorf((org.z - p.tc_lo[2]) * p.tc_inv_size);
                    tree = p.tc_ncells;
                    if (fx >= 0.0f && fx < (float)p.tc_n[0] && fy >= 0.0f && fy < (float)p.tc_n[1] && fz >= 0.0f &&
                        fz < (float)p.tc_n[2]) {
                        tree = ((uint32_t)fz * p.tc_n[1] + (uint32_t)fy) * p.tc_n[0] + (uint32_t)fx;
                        // (bvh.cpp build_triangle_cells' centre, the same operations)
                        oc = f3(p.tc_lo[0] + (fx + 0.5f) * p.tc_size, p.tc_lo[1] + (fy + 0.5f) * p.tc_size,
                                p.tc_lo[2] + (fz + 0.5f) * p.tc_size);
                    }
                }
                const F3 dlt2 = f3(2.0f * (org.x - oc.x), 2.0f * (org.y - oc.y), 2.0f * (org.z - oc.z));
                F3 nlo, nhi;
                sphere_slabs(org, inv, e, nlo, nhi);
                // (the grid base folded in: tri_wide_child)
                nlo = f3(__builtin_fmaf(p.tq_base[0], inv.x, nlo.x), __builtin_fmaf(p.tq_base[1], inv.y, nlo.y),
                         __builtin_fmaf(p.tq_base[2], inv.z, nlo.z));
                nhi = f3(__builtin_fmaf(p.tq_base[0], inv.x, nhi.x), __builtin_fmaf(p.tq_base[1], inv.y, nhi.y),
                         __builtin_fmaf(p.tq_base[2], inv.z, nhi.z));
                float cap = fminf(best_t, tri_t);
                do {
                    const uint4 *wn = p.tw_nodes + 8u * (tree * p.tw_stride + node);
                    tnode_tests += 4;
                    float tn[4];
                    bool in[4];
#ifndef RT_WIDE_ONE_LOAD
                    // two halves: the first brings the 128-B line into the L1,
                    // the second (after a compiler barrier, so that the node
                    // never occupies 28 VGPRs at once) hits it there
                    {
                        const uint4 q0 = wn[0], q1 = wn[1], q2 = wn[2];
                        in[0] = tri_wide_child(p, q0.x, q0.y, q0.z, q0.w, q1.x, q1.y, nlo, nhi, inv, dlt2, cap, tn[0]);
                        in[1] = tri_wide_child(p, q1.z, q1.w, q2.x, q2.y, q2.z, q2.w, nlo, nhi, inv, dlt2, cap, tn[1]);
                    }
                    asm volatile("" ::: "memory");
                    {
                        const uint4 q3 = wn[3], q4 = wn[4], q5 = wn[5];
                        in[2] = tri_wide_child(p, q3.x, q3.y, q3.z, q3.w, q4.x, q4.y, nlo, nhi, inv, dlt2, cap, tn[2]);
                        in[3] = tri_wide_child(p, q4.z, q4.w, q5.x, q5.y, q5.z, q5.w, nlo, nhi, inv, dlt2, cap, tn[3]);
                    }
#else
                    {
                        const uint4 q0 = wn[0], q1 = wn[1], q2 = wn[2], q3 = wn[3], q4 = wn[4], q5 = wn[5];
                        in[0] = tri_wide_child(p, q0.x, q0.y, q0.z, q0.w, q1.x, q1.y, nlo, nhi, inv, dlt2, cap, tn[0]);
                        in[1] = tri_wide_child(p, q1.z, q1.w, q2.x, q2.y, q2.z, q2.w, nlo, nhi, inv, dlt2, cap, tn[1]);
                        in[2] = tri_wide_child(p, q3.x, q3.y, q3.z, q3.w, q4.x, q4.y, nlo, nhi, inv, dlt2, cap, tn[2]);
                        in[3] = tri_wide_child(p, q4.z, q4.w, q5.x, q5.y, q5.z, q5.w, nlo, nhi, inv, dlt2, cap, tn[3]);
                    }
#endif
                    const uint4 qa = wn[6];
                    const uint32_t a[4] = {qa.x, qa.y, qa.z, qa.w};
                    // entered leaf children, one copy of the leaf test for all four
                    uint32_t lmask = 0;
#pragma unroll
                    for (int c = 0; c < 4; ++c) lmask |= (in[c] && (a[c] & kLeafBitDev)) ? 1u << c : 0u;
                    while (lmask != 0) {
                        const uint32_t c = (uint32_t)__builtin_ctz(lmask);
                        lmask &= lmask - 1u;
                        const uint32_t lw = c == 0 ? a[0] : c == 1 ? a[1] : c == 2 ? a[2] : a[3];
                        tri_leaf(p, org, dir, false, lw & ~kLeafBitDev, best_t, tri_t, tri_i, tri_in, tri_done,
                                 p.tw_tris);
                    }
                    cap = fminf(best_t, tri_t);
                    uint32_t nxt = 0xFFFFu;
                    float ntn = 0.0f;
#pragma unroll
                    for (int c = 3; c >= 0; --c) {
                        if (in[c] && !(a[c] & kLeafBitDev) && __float_as_int(tn[c]) <= __float_as_int(cap)) {
                            if (nxt != 0xFFFFu) {
                                // the nearer one next, the other on the stack
                                const bool closer = tn[c] < ntn;
                                tstack[tsp * blockDim.x] = (uint16_t)(closer ? nxt : a[c]);
                                ++tsp;
                                if (closer) { nxt = a[c]; ntn = tn[c]; }
                            } else {
                                nxt = a[c];
                                ntn = tn[c];
                            }
                        }
                    }
                    if (nxt == 0xFFFFu && tsp != 0) {
                        --tsp;
                        nxt = tstack[tsp * blockDim.x];
                    }
                    node = nxt;
                } while (node != 0xFFFFu && (!kStep || --wbudget != 0));
                if (node == 0xFFFFu) phase = kShade;
            }
            RT_STAMP(2);
            if (phase == kShade) {
                const TraceParams &p = kargs();  // (see kargs)
                phase = kSetup;
                // One NVec3::new for both kinds of lane that need one here: a
                // missed ray re-normalises its direction (common.rs:277), a
                // sphere hit normalises (pos - c) / r (common.rs:95), so the
                // wave runs one copy of the sqrt / divide sequence, not two
                const bool sky = tri_i < 0 && best_i < 0;
                const bool sph = tri_i < 0 && best_i >= 0;
                F3 un = dir, spos = dir;
                float4 SS = make_float4(0.0f, 0.0f, 0.0f, 0.0f), SM = SS;
                uint32_t skind = 0;
                if (sph) {
                    // one round trip: centre/radius, colour/param and kind together
                    SS = view.shade[2 * best_i];
                    SM = view.shade[2 * best_i + 1];
                    skind = view.kinds[best_i];
                    spos = org + scale(dir, best_t);
                    un = divide_by(spos - f3(SS.x, SS.y, SS.z), SS.w);
                }
                if (sky || sph) un = unit(un);
                if (sky) {
                    // background (common.rs:276-281): re-normalise, lerp to sky blue
                    const float t = 0.5f * (un.y + 1.0f);
                    const float w = 1.0f - t;
                    out_r = thr_r * (1.0f * w + 0.5f * t);
                    out_g = thr_g * (1.0f * w + 0.7f * t);
                    out_b = thr_b * (1.0f * w + 1.0f * t);
                    done = true;
                } else {
                    F3 pos, nrm;
                    uint32_t kind;
                    float cr, cg, cb, param;
                    if (tri_i >= 0) {  // a triangle wins a tie against a sphere
                        pos = org + scale(dir, tri_t);
                        const float4 *g = p.tri_geo + 4u * (uint32_t)tri_i;
                        const float4 A = g[0], Nn = g[3];
                        nrm = f3(Nn.x, Nn.y, Nn.z);
                        const float *m = p.mats + 8u * __float_as_uint(A.w);
                        kind = __float_as_uint(m[0]);
                        cr = m[1]; cg = m[2]; cb = m[3]; param = m[4];
                    } else {
                        kind = skind;
                        pos = spos;
                        nrm = un;  // common.rs:95, normalised above
                        cr = SM.x; cg = SM.y; cb = SM.z; param = SM.w;
                    }
                    // Each scatter builds an un-normalised direction `v`; the draws
                    // of diffuse and metal (random_unit_sphere, common.rs:32-38) and
                    // the final normalisation are shared code so divergent lanes do
                    // not execute three copies of the divide/sqrt sequences.
                    bool next = true, keep_normal = false;
                    F3 v = nrm;
                    if (kind == kMatDiffuse || kind == kMatMetal) {
                        const F3 ru = draw_unit(rng);
                        if (kSerial) ++nscat;
                        if (kind == kMatDiffuse) {  // materials.rs:42-52
                            v = nrm + ru;
                            const float eps = 1e-8f;
                            keep_normal = fabsf(v.x) < eps && fabsf(v.y) < eps && fabsf(v.z) < eps;
                        } else {  // materials.rs:54-63 (reflect, maths.rs:26-28)
                            const F3 refl = dir - scale(nrm, 2.0f * dot(dir, nrm));
                            v = refl + scale(ru, param);
                            next = dot(v, nrm) >= 0.0f;
                        }
                    } else if (kind == kMatDielectric) {  // materials.rs:65-97
                        F3 n2 = nrm;
                        float eta = param;
                        if (dot(dir, nrm) >= 0.0f) { n2 = -nrm; eta = 1.0f / param; }
                        const float cos_t = dot(-dir, n2);  // maths.rs:31-36
                        const F3 perp = scale(dir + scale(n2, cos_t), eta);
                        const F3 par = scale(n2, -xsqrt(fabsf(1.0f - dot(perp, perp))));
                        v = perp + par;
                        cr = cg = cb = 1.0f;
                    } else {  // Emission (materials.rs:100-102)
                        next = false;
                    }
                    if (next) {
                        thr_r = thr_r * cr;
                        thr_g = thr_g * cg;
                        thr_b = thr_b * cb;
                        org = pos;
                        if (keep_normal) {
                            dir = nrm;
                        } else {
                            vdir = v;  // normalised below, with the new rays' directions
                            renorm = true;
                        }
                        ++bounce;
                    } else {  // common.rs:273-274: final * colour
                        out_r = thr_r * cr;
                        out_g = thr_g * cg;
                        out_b = thr_b * cb;
                        done = true;
                    }
                }
            }
            RT_STAMP(3);
            if (done) {
                if (kSerial && p.mode == kRngSerialCheck) {
                    // the chain check: this sample's end state must be the next
                    // sample's start state (one variant: slot = launch sample)
                    const uint32_t j = p.cbase + slot;
                    out_r = rng == (j + 1u < p.nserial ? p.win[j + 1u] : p.seed) ? 0.0f : 1.0f;
                } else if (kSerial) {
                    // SERIAL passes: the sample's scatter count b instead of its
                    // colour -- it drew 2 + 3b numbers (common.rs:335-336 and one
                    // random_unit_sphere per diffuse/metal scatter, common.rs:32-38),
                    // counted as they were drawn
                    out_r = (float)nscat;
                }
                // planar (R, G, B planes): 12 B per sample, to the slab or the
                // ring (SERIAL passes: plane 0 only)
                sbase[slot] = out_r;
                if (!kSerial) {
                    sbase[pstride + slot] = out_g;
                    sbase[2 * pstride + slot] = out_b;
                }
                active = false;
            }
        }
        RT_STAMP(4);
        if (kCount && nact != 0) {  // (wave-uniform: every lane counts the same)
            const bool wk = __ballot(walked) != 0;
            ++it_all;
            lanes_all += nact;
            it_walk += wk ? 1u : 0u;
            lanes_walk += wk ? nact : 0u;
        }
        const uint64_t dead = __ballot(!active);
        const uint32_t ndead = (uint32_t)__popcll(dead);
        const bool refill = dead != 0 && (ndead >= p.refill_min || ndead == kWave);
        // ---- fused resolve, at refill points: lanes that finished since the
        // last one (slot != ~0) are counted against their chunk's ring slot; a
        // chunk with no samples left is summed now, by this wave, while its
        // samples are still in the cache.  (Every lane is idle in the last
        // iteration, so every chunk is resolved before the wave exits.)
        if (fused && refill) {
            const bool fin = !active && slot != ~0u;
            if (__ballot(fin) != 0) {
                const uint32_t lk = slot >> p.ring_shift;
#pragma unroll
                for (uint32_t k = 0; k < kTraceRing; ++k) {
                    if (rfree & (1u << k)) continue;
                    const uint32_t n = (uint32_t)__popcll(__ballot(fin && lk == k));
                    rleft[k] -= n;
                    if (n != 0 && rleft[k] == 0) {
                        const TraceParams &pc = kargs();
                        if (!(pc.ablate & 2u))
                            resolve_chunk<RT_PLANE_LANES(kMesh)>(pc, sbase, pstride, k << pc.ring_shift, rbase[k],
                                                  rlen[k], lane);
                        rfree |= 1u << k;
                    }
                }
                if (fin) slot = ~0u;
            }
        }
        RT_STAMP(5);
        // ---- refill lanes whose path ended (active-ray compaction) -------
        // (with the fused resolve a new chunk needs a free ring slot: with all
        // kTraceRing slots waiting on unfinished samples the lanes stay idle)
        if (refill && !exhausted && !(fused && rfree == 0 && pool_next >= pool_end)) {
            const TraceParams &pc = kargs();  // (the refill's parameters: see kargs)
            // (a wave-uniform loop only in the pixel table pass, which skips
            // chunks that hold no position of its pixel's span)
            while (pool_next >= pool_end) {
                uint32_t base = 0;
                if (lane == 0) {
                    base = pbegin + (prefetch_pending ? prefetch
                                                      : atomicAdd(pc.job_counter + 32u * part, pc.chunk));
                    while (base >= pend && ++tries < pc.nparts) {
                        part = part + 1 == pc.nparts ? 0 : part + 1;
                        pbegin = part_begin(part);
                        pend = part_begin(part + 1);
                        base = pbegin + atomicAdd(pc.job_counter + 32u * part, pc.chunk);
                    }
                }
                prefetch_pending = false;
                base = __builtin_amdgcn_readfirstlane(base);
                part = __builtin_amdgcn_readfirstlane(part);
                tries = __builtin_amdgcn_readfirstlane(tries);
                pbegin = __builtin_amdgcn_readfirstlane(pbegin);
                pend = __builtin_amdgcn_readfirstlane(pend);
                if (base >= pend) {
                    exhausted = true;
#ifdef RT_WAVE_TIMES
                    wt_exh = __builtin_amdgcn_s_memrealtime();
#endif
                    break;
                } else {
                    pool_next = base;
                    pool_end = min(base + pc.chunk, pend);
                    if (kSerial && pc.mode == kRngSerialPixel && pc.spix != nullptr) {
                        // pixel rows are padded to whole chunks (the row stride E
                        // is a multiple of the chunk: serial_window_kernel), so a
                        // chunk lies in one pixel's row: hand out only its
                        // positions inside the pixel's span (the rest would leave
                        // lanes idle, serial_pixel_job) and skip chunks past it
                        const uint32_t q = fdiv(base, pc.div_spp);
                        const uint4 sq = uniform_load_u4(pc.spix, q);
                        const uint32_t rowb = q * pc.spp;
                        const uint32_t live_end = rowb + (sq.y >= sq.x ? sq.y - sq.x + 1u : 0u);
                        pool_end = min(pool_end, live_end);
                        // the positions the previous iteration traced were copied
                        // (serial_reuse_kernel): the pool skips them
                        gap_lo = ~0u;
                        gap_len = 0;
                        if (sq.z <= sq.w && pool_next < pool_end) {
                            const uint32_t g0 = max(rowb + sq.z, pool_next);
                            const uint32_t g1 = min(rowb + sq.w + 1u, pool_end);
                            if (g0 < g1) {
                                gap_lo = g0;
                                gap_len = g1 - g0;
                                pool_end -= gap_len;
                            }
                        }
                        if (pool_next >= pool_end) continue;
                    }
#ifdef RT_WAVE_TIMES
                    wt_pull = __builtin_amdgcn_s_memrealtime();
                    wt_jobs_tail = pool_end - pool_next;
#endif
                    if (fused) {
                        const uint32_t k = (uint32_t)__builtin_ctz(rfree);
                        rfree &= ~(1u << k);
#pragma unroll
                        for (uint32_t i = 0; i < kTraceRing; ++i)
                            if (i == k) rbase[i] = base, rlen[i] = rleft[i] = pool_end - base;
                        cur_off = (k << pc.ring_shift) - base;
                    }
                }
                if (!kSerial) break;  // (frames: one pass, as the plain `if` it replaces)
            }
            // (the pixel pass's skipped chunks may leave pool_end below pool_next)
            const uint32_t avail = kSerial && exhausted ? 0u : pool_end - pool_next;
            const uint32_t rank = __builtin_amdgcn_mbcnt_hi(
                (uint32_t)(dead >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)dead, 0u));
            if (!active && rank < avail) {
                uint32_t job = pool_next + rank;
                if (kSerial && job >= gap_lo) job += gap_len;
                // Jobs are enumerated pixel-major (job = pixel*spp + s): the
                // lanes refilled together trace samples of one pixel (or of
                // neighbours), so their primary walks visit the same nodes
                // (A/B: C2 trace -5.5 %, C5 -5 % against sample-major), and
                // they store to consecutive slab slots.  Seeds and replay
                // states use the reference's job index below, so the
                // enumeration order changes no bits.
                uint32_t s, col, row;
                uint64_t gjob = 0;
                if (!kSerial && pc.gj32) {
                    // one rank, 32-bit global jobs (TraceParams::gj32)
                    const uint32_t lp = fdiv(job, pc.div_spp);
                    const uint32_t q = fdiv(lp, pc.div_width);
                    col = lp - q * pc.width;
                    row = pc.height - 1u - (pc.slab_row0 + q);
                    gjob = job + pc.gj_c0 - q * pc.gj_2p;
                } else {
                    job_pixel<kSerial>(pc, job, s, col, row);
                    gjob = ((uint64_t)row * pc.width + col) * pc.spp + s;
                }
                slot = job + cur_off;
                bool take = true;
                if (kSerial) {
                    nscat = 0;
                    rng = serial_start(pc, job);
                    if (pc.mode == kRngSerialPixel) take = serial_pixel_job(pc, job);
                } else {
                    rng = (pc.mode == kRngReplay) ? pc.replay[gjob] : counter_seed(pc.seed, gjob);
                }
                // common.rs:335-337: u drawn before v; camera.rs:84-89
                // numerators are in [2^-32, 2^24]: exactdiv.h with the host's
                // reciprocals whenever the denominators are in range
                const float un = draw_plus(rng, (float)col);
                const float vn = draw_plus(rng, (float)row);
#ifndef RT_NO_XDIV
                const bool xd = pc.xdiv_uv != 0;
#else
                const bool xd = false;
#endif
                const float u = xd ? xdiv(un, pc.wden, pc.wrcp) : un / pc.wden;
                const float v = xd ? xdiv(vn, pc.hden, pc.hrcp) : vn / pc.hden;
                const F3 h = f3(pc.cam[6], pc.cam[7], pc.cam[8]);
                const F3 vv = f3(pc.cam[9], pc.cam[10], pc.cam[11]);
                org = f3(pc.cam[0], pc.cam[1], pc.cam[2]);
                const F3 llc = f3(pc.cam[3], pc.cam[4], pc.cam[5]);
                vdir = ((llc + scale(h, u)) + scale(vv, v)) - org;  // normalised below
                renorm = true;
                if (kBvh && !kMesh && pc.spl != nullptr) {
                    // issued after the seed's (replay) load, so nothing waits on it
                    // before the ray's setup in the next iteration
                    if (pc.ablate & 4u) {  // timing-only diagnostic: no record load
                        spl0 = 0;
                        spl1 = 0;
                    } else {
                        // (32-bit index: a frame's pixel count fits)
                        const uint2 r = pc.spl[(pc.height - 1u - row) * pc.width + col];
                        spl0 = r.x;
                        spl1 = r.y;
                    }
                }
                thr_r = thr_g = thr_b = 1.0f;
                bounce = 0;
                phase = kSetup;
                active = take;
            }
            pool_next += min(ndead, avail);
            // ask for the next chunk now; the reply is only waited for when the
            // pool runs dry (hides the ~1-3 us atomic round trip)
            if (!exhausted && !prefetch_pending && pool_end - pool_next < kWave) {
                if (lane == 0) prefetch = atomicAdd(p.job_counter + 32u * part, p.chunk);
                prefetch_pending = true;
            }
        }
        RT_STAMP(6);
        if (renorm) dir = unit(vdir);
        RT_STAMP(0);
        if (__ballot(active) == 0 && exhausted) break;
    }

    // ---- per-wave statistics (stats requested only): each wave adds its
    // counters to its own 16-slot record, no atomics -- 6144 waves' atomics on
    // the same six words serialised at the end of every launch (~0.4 ms, most
    // of a multi-GPU tile's overhead); the host sums the records
    if (!kCount || p.stats == nullptr) return;  // (!kCount: the counters compile away)
    uint64_t c[6] = {rays, tri_in, sph_tests, node_tests, tnode_tests, tri_done};
    const uint64_t mix[4] = {it_all, it_walk, lanes_all, lanes_walk};  // (wave-uniform)
#pragma unroll
    for (int k = 0; k < 6; ++k)
        for (uint32_t off = kWave / 2; off > 0; off >>= 1) c[k] += __shfl_xor(c[k], (int)off);
    if (lane == 0) {
        unsigned long long *w = p.stats + (size_t)wave_id * kStatSlots;
#pragma unroll
        for (int k = 0; k < 6; ++k) w[k < 4 ? k : k + 4] += c[k];
        for (int k = 0; k < 4; ++k) w[10 + k] += mix[k];
#ifdef RT_WALK_MIX
        w[4] += wm_iters; w[5] += wm_leaf_iters; w[6] += wm_leaf_trips; w[7] += wm_walks;
#endif
#ifdef RT_STAMPS
        // coarse shares (stamp_cycles): refill + store + resolve + loop, setup, walks, shade
        w[4] += stamp_acc[0] + stamp_acc[4] + stamp_acc[5] + stamp_acc[6];
        for (int k = 1; k < 4; ++k) w[4 + k] += stamp_acc[k];
        for (uint32_t k = 0; k < kStampSegs; ++k) w[16 + k] += stamp_acc[k];
#endif
#ifdef RT_WAVE_TIMES
        w[4] = wt_start;
        w[5] = wt_pull;
        w[6] = wt_exh;
        w[7] = __builtin_amdgcn_s_memrealtime();
        w[14] = wt_jobs_tail;
#endif
    }
}

// ------------------------------------------------------------ resolve kernel
// Sums each pixel's samples in order (common.rs:333-341), gamma + `as u8`
// (:344-356), one RGBA8 word per pixel.  The slab is planar and pixel-major,
// so one wave's 64 pixels own a contiguous run of 64*spp floats per plane:
// the wave copies it through LDS in chunks of 64 samples (float4 loads
// across the run, coalesced), padded to 65 floats per pixel so that the
// in-order per-lane sums read LDS without bank conflicts.
constexpr uint32_t kResolveWaves = 4;
constexpr uint32_t kResolveChunk = 64;
constexpr uint32_t kResolvePad = kResolveChunk + 1;
__global__ __launch_bounds__(kResolveWaves * 64) void resolve_kernel(
    const float *__restrict__ samples, uint32_t *__restrict__ out, uint32_t npix, uint32_t spp,
    float inv, uint32_t width, uint32_t slab_row0) {
    __shared__ float lds[kResolveWaves][kWave * kResolvePad];
    const uint32_t lane = threadIdx.x % kWave, wave = threadIdx.x / kWave;
    const uint32_t lp0 = (blockIdx.x * kResolveWaves + wave) * kWave;
    if (lp0 >= npix) return;  // whole waves only: no workgroup barrier below
    const uint32_t n = min(kWave, npix - lp0);
    const size_t plane = (size_t)npix * spp;
    float *L = lds[wave];
    float acc[3] = {0.0f, 0.0f, 0.0f};
    float a = 1.0f;  // Color::new(0,0,0): alpha 1
    for (uint32_t k0 = 0; k0 < spp; k0 += kResolveChunk) {
        const uint32_t kc = min(kResolveChunk, spp - k0);
#pragma unroll
        for (uint32_t c = 0; c < 3; ++c) {
            const float *src = samples + c * plane + (size_t)lp0 * spp + k0;
            if (kc == kResolveChunk && spp % 4 == 0) {
                // 16 lanes per pixel, 4 pixels per float4 wave load
                for (uint32_t e = lane; e < n * 16; e += kWave) {
                    const uint32_t pix = e >> 4, k = (e & 15u) * 4;
                    const float4 v = *reinterpret_cast<const float4 *>(src + (size_t)pix * spp + k);
                    float *d = L + pix * kResolvePad + k;
                    d[0] = v.x; d[1] = v.y; d[2] = v.z; d[3] = v.w;
                }
            } else {
                for (uint32_t e = lane; e < n * kc; e += kWave) {
                    const uint32_t pix = e / kc, k = e - pix * kc;
                    L[pix * kResolvePad + k] = src[(size_t)pix * spp + k];
                }
            }
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
            float x = acc[c];
            if (lane < n)
                for (uint32_t k = 0; k < kc; ++k) x = x + L[lane * kResolvePad + k];
            acc[c] = x;
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        }
        for (uint32_t k = 0; k < kc; ++k) a = a + 1.0f;  // every sample's alpha is exactly 1.0
    }
    if (lane >= n) return;
    const uint32_t lp = lp0 + lane;
    const uint32_t R = sat_u8(__builtin_sqrtf(acc[0] * inv) * 255.999f);
    const uint32_t G = sat_u8(__builtin_sqrtf(acc[1] * inv) * 255.999f);
    const uint32_t B = sat_u8(__builtin_sqrtf(acc[2] * inv) * 255.999f);
    const uint32_t A = sat_u8(a * inv * 255.999f);
    const uint32_t q = lp / width;
    const uint32_t col = lp - q * width;
    out[(size_t)(slab_row0 + q) * width + col] = R | (G << 8) | (B << 16) | (A << 24);
}

}  // namespace

uint32_t trace_block_threads(bool lds, int mesh, int kind) { return trace_threads(lds, mesh, kind); }

size_t trace_lds_bytes(const TraceParams &p) {
    // (shading records in global memory instead, which would allow 8 waves per
    // SIMD: A/B +1.7 % at 6 waves, +8 % at 8 waves per SIMD)
    return trace_tree_lds(p.nnodes, p.nprims, p.nsph_padded);
}

size_t trace_dyn_lds(const TraceParams &p, bool lds, bool wide, uint32_t threads) {
    const size_t tree = lds ? (trace_lds_bytes(p) + 15u) & ~(size_t)15u : 0u;
    return tree + (wide ? (size_t)p.tw_depth * threads * 2u : 0u);
}

template <bool kStep, int kMesh, bool kCount, bool kSerial>
static void launch_trace_t(const TraceParams &p, uint32_t blocks, hipStream_t stream) {
    const uint32_t lt = trace_threads(true, kMesh, kSerial ? 2 : kCount ? 1 : 0);
    if (p.nnodes && p.use_lds)
        hipLaunchKernelGGL((trace_kernel<true, true, kStep, kMesh, kCount, kSerial>), dim3(blocks), dim3(lt),
                           trace_dyn_lds(p, true, kMesh == 3, lt), stream, p);
    else if (p.nnodes)
        hipLaunchKernelGGL((trace_kernel<true, false, kStep, kMesh, kCount, kSerial>), dim3(blocks),
                           dim3(256), trace_dyn_lds(p, false, kMesh == 3, 256), stream, p);
    else
        hipLaunchKernelGGL((trace_kernel<false, false, kStep, kMesh, kCount, kSerial>), dim3(blocks),
                           dim3(256), trace_dyn_lds(p, false, kMesh == 3, 256), stream, p);
}

// kMesh: 0 no triangles, 1 brute-force triangles (no triangle tree: small
// meshes), 2 triangle trees -- the tree walk's registers only where it runs
template <bool kCount, bool kSerial>
static void launch_trace_c(const TraceParams &p, uint32_t blocks, hipStream_t stream) {
    const int mesh = trace_mesh_kind(p.ntri != 0, p.tnodes != 0);
    if (!kSerial && mesh == 2 && p.tw_nodes != nullptr) {
        if (p.step) launch_trace_t<true, 3, kCount, false>(p, blocks, stream);
        else launch_trace_t<false, 3, kCount, false>(p, blocks, stream);
        return;
    }
    if (p.step) {
        if (mesh == 2) launch_trace_t<true, 2, kCount, kSerial>(p, blocks, stream);
        else if (mesh == 1) launch_trace_t<true, 1, kCount, kSerial>(p, blocks, stream);
        else launch_trace_t<true, 0, kCount, kSerial>(p, blocks, stream);
    } else {
        if (mesh == 2) launch_trace_t<false, 2, kCount, kSerial>(p, blocks, stream);
        else if (mesh == 1) launch_trace_t<false, 1, kCount, kSerial>(p, blocks, stream);
        else launch_trace_t<false, 0, kCount, kSerial>(p, blocks, stream);
    }
}

// Frames rendered without stats run a variant whose work counters compile away
// (one VALU increment per node / sphere test / ray); SERIAL passes their own.
hipError_t launch_trace(const TraceParams &p, uint32_t blocks, hipStream_t stream) {
    if (p.mode >= kRngSerialCount) launch_trace_c<false, true>(p, blocks, stream);
    else if (p.stats) launch_trace_c<true, false>(p, blocks, stream);
    else launch_trace_c<false, false>(p, blocks, stream);
    return hipGetLastError();
}

hipError_t launch_resolve_ex(const float *samples, uint32_t *out, uint32_t npix, uint32_t spp,
                             float inv_spp, uint32_t width, uint32_t slab_row0,
                             hipStream_t stream) {
    const uint32_t per_block = kResolveWaves * kWave;
    const uint32_t blocks = (npix + per_block - 1) / per_block;
    hipLaunchKernelGGL(resolve_kernel, dim3(blocks), dim3(per_block), 0, stream, samples, out, npix,
                       spp, inv_spp, width, slab_row0);
    return hipGetLastError();
}

template <bool kStep, int kMesh, bool kCount, bool kSerial>
static hipError_t trace_occupancy_t(int *blocks_per_cu, int variant, size_t lds_bytes) {
    constexpr int kind = kSerial ? 2 : kCount ? 1 : 0;
    if (variant == 2)
        return hipOccupancyMaxActiveBlocksPerMultiprocessor(
            blocks_per_cu, trace_kernel<true, true, kStep, kMesh, kCount, kSerial>,
            trace_threads(true, kMesh, kind), lds_bytes);
    if (variant == 1)
        return hipOccupancyMaxActiveBlocksPerMultiprocessor(
            blocks_per_cu, trace_kernel<true, false, kStep, kMesh, kCount, kSerial>, 256, lds_bytes);
    return hipOccupancyMaxActiveBlocksPerMultiprocessor(
        blocks_per_cu, trace_kernel<false, false, kStep, kMesh, kCount, kSerial>, 256, lds_bytes);
}

template <bool kCount, bool kSerial>
static hipError_t trace_occupancy_c(int *blocks_per_cu, int variant, size_t lds_bytes, bool step,
                                    int mesh) {
    if (!kSerial && mesh == 3)
        return step ? trace_occupancy_t<true, 3, kCount, false>(blocks_per_cu, variant, lds_bytes)
                    : trace_occupancy_t<false, 3, kCount, false>(blocks_per_cu, variant, lds_bytes);
    if (mesh == 3) mesh = 2;
    if (step)
        return mesh == 2   ? trace_occupancy_t<true, 2, kCount, kSerial>(blocks_per_cu, variant, lds_bytes)
               : mesh == 1 ? trace_occupancy_t<true, 1, kCount, kSerial>(blocks_per_cu, variant, lds_bytes)
                           : trace_occupancy_t<true, 0, kCount, kSerial>(blocks_per_cu, variant, lds_bytes);
    return mesh == 2   ? trace_occupancy_t<false, 2, kCount, kSerial>(blocks_per_cu, variant, lds_bytes)
           : mesh == 1 ? trace_occupancy_t<false, 1, kCount, kSerial>(blocks_per_cu, variant, lds_bytes)
                       : trace_occupancy_t<false, 0, kCount, kSerial>(blocks_per_cu, variant, lds_bytes);
}

hipError_t trace_occupancy(int *blocks_per_cu, int variant, size_t lds_bytes, bool step, int mesh,
                           int kind) {
    return kind == 2   ? trace_occupancy_c<false, true>(blocks_per_cu, variant, lds_bytes, step, mesh)
           : kind == 1 ? trace_occupancy_c<true, false>(blocks_per_cu, variant, lds_bytes, step, mesh)
                       : trace_occupancy_c<false, false>(blocks_per_cu, variant, lds_bytes, step, mesh);
}

// ------------------------------------------------------------ SERIAL mode
// The reference draws every sample from ONE xorshift32 stream (common.rs:321):
// sample j starts at stream position P_j = 2j + 3B_j, B_j = the diffuse/metal
// scatters of all earlier samples.  runtime.cpp render_frame_serial finds
// every P_j chunk by chunk: trace_kernel (kRngSerialCount) traces each sample
// of the chunk from K candidate positions around its predicted one,
// the walk kernels follow the true path through that table, and the frame
// is then rendered in REPLAY mode from the start states found.

// xorshift32^(2^i) as 32 columns (GF(2) matrix): y = XOR of columns c with bit c of x set
__device__ __forceinline__ uint32_t gf2_apply(const uint32_t *cols, uint32_t x) {
    uint32_t y = 0;
#pragma unroll 8
    for (uint32_t c = 0; c < 32u; ++c) y ^= (x >> c & 1u) ? cols[c] : 0u;
    return y;
}

// the same from a matrix in global memory (tabulated powers), 16-B loads
__device__ __forceinline__ uint32_t gf2_apply_g(const uint32_t *cols, uint32_t x) {
    const uint4 *c4 = reinterpret_cast<const uint4 *>(cols);
    uint32_t y = 0;
#pragma unroll
    for (uint32_t q = 0; q < 8u; ++q) {
        const uint4 m = c4[q];
        y ^= (x >> (4u * q) & 1u) ? m.x : 0u;
        y ^= (x >> (4u * q + 1u) & 1u) ? m.y : 0u;
        y ^= (x >> (4u * q + 2u) & 1u) ? m.z : 0u;
        y ^= (x >> (4u * q + 3u) & 1u) ? m.w : 0u;
    }
    return y;
}

// Window: thread t writes win[4t, 4t + 4): one jump to 4t (two tabulated
// matrices), then plain xorshift steps.  (16 states per thread and one
// matrix apply per set bit of 16t until round 5: a few dozen workgroups of
// long jumps, 16 us per iteration on world.txt 960x540x16.)
constexpr uint32_t kWinPerThread = kSerialWinPerThread;
// It also tabulates the iteration's window bases lo[jl] = serial_lo(a, jl) for
// jl < L (a = ctrl[4], K = the iteration's candidates), which the count pass
// and the walks then load instead of evaluating M twice per step.
// pix_spp != 0 (the pixel table pass follows): ctrl[7] = max over the
// iteration's pixels of the stream positions their samples' windows span.
__global__ __launch_bounds__(256) void serial_window_kernel(uint32_t *__restrict__ ctrl,
                                                            const uint32_t *__restrict__ jump,
                                                            uint32_t *__restrict__ win, uint32_t n,
                                                            SerialPred M, uint32_t *__restrict__ lo,
                                                            uint32_t L, uint32_t Kmax, uint32_t depth,
                                                            uint32_t nserial, uint32_t pix_spp, uint32_t pix_emax,
                                                            uint32_t *__restrict__ counters, uint32_t ncounters,
                                                            uint4 *__restrict__ spix, uint32_t pix_chunk,
                                                            const uint4 *__restrict__ spix_prev) {
    if (ctrl[0] != 0u) return;
    // the following trace pass's job counters (instead of a fill launch)
    for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < ncounters; i += gridDim.x * blockDim.x)
        counters[32u * i] = 0u;
    if (lo != nullptr) {
        const uint32_t k = ctrl[5];
        const uint32_t K = k != 0u && k < Kmax ? k : Kmax;  // (serial_k)
        const uint32_t a = ctrl[4];
        for (uint32_t jl = blockIdx.x * blockDim.x + threadIdx.x; jl < L; jl += gridDim.x * blockDim.x)
            lo[jl] = serial_lo(M, a, jl, K, depth, nserial);
        if (pix_spp != 0u) {
            // local pixel q: samples [jf, jz] of the iteration, windows from
            // 2 jf + 3 lo(jf) to 2 jz + 3 (lo(jz) + K - 1)
            const uint32_t ln = min(L, nserial - a);
            const uint32_t p0 = a / pix_spp, npq = (a + ln - 1u) / pix_spp - p0 + 1u;
            // the previous iteration (serial_walk_finish_kernel: its first sample
            // ctrl[10], its table's row stride ctrl[11], this iteration's window
            // at its stream offset ctrl[8]; ctrl[9] set once one has run)
            const bool reuse = spix_prev != nullptr && ctrl[9] != 0u && ctrl[11] != 0u;
            const uint32_t ap = ctrl[10], D = ctrl[8], Ep = ctrl[11];
            const uint32_t p0p = ap / pix_spp;
            const uint32_t npqp = reuse ? (ap + min(L, nserial - ap) - 1u) / pix_spp - p0p + 1u : 0u;
            uint32_t span = 0;
            for (uint32_t q = blockIdx.x * blockDim.x + threadIdx.x; q < npq; q += gridDim.x * blockDim.x) {
                const uint32_t jf = q == 0u ? 0u : (p0 + q) * pix_spp - a;
                const uint32_t jz = min((p0 + q + 1u) * pix_spp - a, ln) - 1u;
                const uint32_t lf = serial_lo(M, a, jf, K, depth, nserial);
                const uint32_t lz = serial_lo(M, a, jz, K, depth, nserial);
                const uint32_t hi = 2u * jz + 3u * (lz + K - 1u), lo0 = 2u * jf + 3u * lf;
                span = max(span, hi >= lo0 ? hi - lo0 + 1u : 1u);
                if (spix != nullptr) {
                    // the positions of this pixel the previous table holds: its
                    // traced range [plo', min(phi', plo' + E' - 1)] at offset -D,
                    // inside [lo0, hi] (relative to lo0; empty: z > w)
                    uint32_t r0 = 1u, r1 = 0u;
                    const uint32_t pix = p0 + q;
                    if (reuse && pix >= p0p && pix - p0p < npqp) {
                        const uint4 so = spix_prev[pix - p0p];
                        if (so.y >= so.x) {
                            const int64_t olo = (int64_t)so.x - D;
                            const int64_t ohi = (int64_t)min(so.y, so.x + Ep - 1u) - D;
                            const int64_t l = olo > (int64_t)lo0 ? olo : (int64_t)lo0;
                            const int64_t h = ohi < (int64_t)hi ? ohi : (int64_t)hi;
                            if (l <= h) {
                                r0 = (uint32_t)(l - lo0);
                                r1 = (uint32_t)(h - lo0);
                            }
                        }
                    }
                    spix[q] = make_uint4(lo0, hi, r0, r1);
                }
            }
            // (rounded up to whole chunks of the pass's job queue (pix_chunk,
            // spix: rows of one pixel per chunk) and clamped to the table's row
            // stride, a multiple of it: every reader takes ctrl[7] as is, and a
            // position past it reads as "left the window")
            if (spix != nullptr && pix_chunk > 1u) span = (span + pix_chunk - 1u) / pix_chunk * pix_chunk;
            span = min(span, pix_emax);
            if (span) atomicMax(ctrl + 7, span);
        }
    }
    // the jump matrices this workgroup's threads need (bits of i0 below 32),
    // staged in LDS: the jumps then read no global memory
    __shared__ uint32_t jl_lds[32 * 32];
    for (uint32_t i = threadIdx.x; i < 32u * 32u; i += blockDim.x) jl_lds[i] = jump[i];
    __syncthreads();
    const uint32_t i0 = (blockIdx.x * blockDim.x + threadIdx.x) * kWinPerThread;
    if (i0 >= n) return;
    uint32_t x = ctrl[1];
    // the jump to i0: M^(4096 j) M^(4 j') from the tabulated powers (two
    // applies; were one per set bit of i0, ~7 on average), higher bits by
    // powers of two
    x = gf2_apply_g(jump + 32u * (64u + kSerialJumpT1 + ((i0 >> 12) & 255u)), x);
    x = gf2_apply_g(jump + 32u * (64u + ((i0 & 4095u) / kWinPerThread)), x);
    for (uint32_t b = 20; (i0 >> b) != 0u; ++b)
        if ((i0 >> b) & 1u) x = gf2_apply(jl_lds + 32u * b, x);
    for (uint32_t q = 0; q < kWinPerThread && i0 + q < n; ++q) {
        win[i0 + q] = x;
        x ^= x << 13;
        x ^= x >> 17;
        x ^= x << 5;
    }
}

// The walk through an iteration's candidate table (b of chunk sample jl at
// candidate k = table[jl * K + k]; candidate k means B = lo[jl] + k scatters
// since sample a, lo = serial_lo tabulated by serial_window_kernel) in short
// dependent-load chains instead of one of L:
//   blocks: for every block of R samples and every candidate of its first
//     sample, follow R samples: its end offset, or kWalkLeft | the samples
//     walked before one left its window (the path of every walk recorded);
//   super: for every group of kSuperBlocks blocks and every candidate of its
//     first block, chain through the group's block ends (recording each
//     block's start offset);
//   finish: one lane chains the superblock ends from B = 0 as far as they
//     are valid, the workgroup fills the full blocks' path columns from the
//     recorded starts, and serial_states_kernel gathers the start states
//     (win[2 jl + 3 B]) of every resolved sample from the recorded paths; ctrl
//     advances past the resolved samples (>= 1: sample a's own window always
//     holds B = 0).
constexpr uint32_t kWalkInvalid = 0xFFFFFFFFu;
constexpr uint32_t kWalkLeft = 0x80000000u;  // bend: the walk left a window (offsets stay below 2^31)
__device__ __forceinline__ uint32_t walk_step(const float *table, const SerialPred &M, uint32_t a,
                                              uint32_t K, uint32_t depth, uint32_t nserial, uint32_t jl,
                                              uint32_t B, const uint32_t *lo = nullptr) {
    const uint32_t l = lo ? lo[jl] : serial_lo(M, a, jl, K, depth, nserial);
    const float b = (B >= l && B - l < K) ? table[(size_t)jl * K + (B - l)] : -1.0f;
    return b >= 0.0f ? B + (uint32_t)b : kWalkInvalid;
}

// (the iteration's candidates per sample: ctrl[5] when set, else the launch's K)
__device__ __forceinline__ uint32_t serial_k(const uint32_t *ctrl, uint32_t K) {
    const uint32_t k = ctrl[5];
    return k != 0u && k < K ? k : K;
}

// path (optional): the offset B at the start of each of the block's samples,
// sample-major (path[(jl - j0) * nb * K + t], coalesced), so that the states
// of the true path are a gather (serial_states_kernel), not a re-walk
// ptab (the pixel table pass, kRngSerialPixel): b is read from the traced
// (pixel, position) table itself -- b of sample jl at offset B is
// ptab[q E + (2 jl + 3 B - plo(q))], q its local pixel -- instead of a
// gathered L x K count table (a 16 MB table instead of an 80 MB one at 32 k x
// 617, and no gather pass); ppix: the frame's spp as a divider.
__global__ __launch_bounds__(256) void serial_walk_blocks_kernel(
    const uint32_t *__restrict__ ctrl, const float *__restrict__ table, SerialPred M,
    uint32_t *__restrict__ bend, uint32_t *__restrict__ path, const uint32_t *__restrict__ lo, uint32_t L,
    uint32_t K, uint32_t R, uint32_t depth, uint32_t nserial, const float *__restrict__ ptab, FastDiv ppix) {
    if (ctrl[0] != 0u) return;
    K = serial_k(ctrl, K);
    const uint32_t a = ctrl[4];
    const uint32_t n = min(L, nserial - a);
    const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
    const uint32_t nb = (n + R - 1) / R;
    if (t >= nb * K) return;
    const uint32_t blk = t / K, k0 = t - blk * K;
    const uint32_t j0 = blk * R, j1 = min(j0 + R, n);
    const size_t stride = (size_t)nb * K;
    uint32_t B = (lo ? lo[j0] : serial_lo(M, a, j0, K, depth, nserial)) + k0;
    uint32_t jl = j0;
    if (ptab != nullptr) {
        const uint32_t E = ctrl[7], spp = ppix.d;
        const uint32_t p0 = fastdiv_apply(a, ppix);
        uint32_t q = fastdiv_apply(a + j0, ppix) - p0;  // local pixel of sample jl
        uint32_t jf = q == 0u ? 0u : (p0 + q) * spp - a;  // its first sample in the iteration
        uint32_t jnext = (p0 + q + 1u) * spp - a;        // the next pixel's
        uint32_t plo = 2u * jf + 3u * lo[jf];
        for (; jl < j1; ++jl) {
            if (path) path[(size_t)(jl - j0) * stride + t] = B;
            if (jl == jnext) {
                ++q;
                plo = 2u * jnext + 3u * lo[jnext];
                jnext += spp;
            }
            const uint32_t l = lo[jl];
            const uint32_t pos = 2u * jl + 3u * B;
            const float b = (B >= l && B - l < K && pos >= plo && pos - plo < E)
                                ? ptab[(size_t)q * E + (pos - plo)]
                                : -1.0f;
            if (!(b >= 0.0f)) break;
            B += (uint32_t)b;
        }
    } else {
#pragma unroll 4
        for (; jl < j1; ++jl) {
            if (path) path[(size_t)(jl - j0) * stride + t] = B;
            const uint32_t nB = walk_step(table, M, a, K, depth, nserial, jl, B, lo);
            if (nB == kWalkInvalid) break;
            B = nB;
        }
    }
    // the block's end offset, or kWalkLeft | the samples whose end was found
    // (the path then holds the start offset of the sample that left)
    bend[t] = jl == j1 ? B : kWalkLeft | (jl - j0);
}

// ---- pixel table walks with the rows in LDS (kRngSerialPixel, depth < 255)
// One workgroup per block of R samples stages the pixel-table rows of the
// block's pixels -- positions [plo(q), phi(q)] of each local pixel q, the span
// its samples' windows cover (serial_pixel_span), as u8 scatter counts -- and
// then walks from LDS: the per-step reads that were dependent L2 loads (and
// the path of every candidate, 64 stores per lane) become LDS reads.  A
// position outside its pixel's traced span reads as "left the window" (the
// span, not the launch's widest one: positions past a narrower pixel's span
// were not traced).
struct WalkRowsLds {
    uint32_t lo[kMaxWalkR];              // lo[j0 .. j1)
    uint32_t plo[kWalkLdsMaxPix], span[kWalkLdsMaxPix], off[kWalkLdsMaxPix];
    uint32_t qa, nq;
};
// stages the rows of samples [j0, j1) of the iteration (whole workgroup; E:
// the pass's positions per pixel, ctrl[7])
__device__ __forceinline__ void walk_stage_rows(WalkRowsLds &w, uint8_t *rows, uint32_t E, const float *ptab,
                                                const uint32_t *lo, uint32_t a, uint32_t n, uint32_t j0,
                                                uint32_t j1, uint32_t K, FastDiv ppix) {
    const uint32_t spp = ppix.d;
    const uint32_t p0 = fastdiv_apply(a, ppix);
    const uint32_t qa = fastdiv_apply(a + j0, ppix) - p0, qb = fastdiv_apply(a + j1 - 1u, ppix) - p0;
    const uint32_t nq = qb - qa + 1u;
    for (uint32_t i = threadIdx.x; i < j1 - j0; i += blockDim.x) w.lo[i] = lo[j0 + i];
    if (threadIdx.x == 0) {
        w.qa = qa;
        w.nq = nq;
        uint32_t off = 0;
        for (uint32_t i = 0; i < nq; ++i) {
            const uint32_t q = qa + i;
            const uint32_t jf = q == 0u ? 0u : (p0 + q) * spp - a;
            const uint32_t jz = min((p0 + q + 1u) * spp - a, n) - 1u;
            const uint32_t plo = 2u * jf + 3u * lo[jf];
            const uint32_t phi = 2u * jz + 3u * (lo[jz] + K - 1u);
            // the traced positions: plo + e for e < E and plo + e <= phi
            const uint32_t sp = min(phi >= plo ? phi - plo + 1u : 0u, E);
            w.plo[i] = plo;
            w.span[i] = sp;
            w.off[i] = off;
            off += sp;
        }
    }
    __syncthreads();
    for (uint32_t i = 0; i < nq; ++i) {
        const float *src = ptab + (size_t)(qa + i) * E;
        uint8_t *dst = rows + w.off[i];
        for (uint32_t e = threadIdx.x; e < w.span[i]; e += blockDim.x) dst[e] = (uint8_t)src[e];
    }
    __syncthreads();
}

// b of sample jl (local pixel i = q - qa of the rows) at offset B, or -1
__device__ __forceinline__ int walk_lds_b(const WalkRowsLds &w, const uint8_t *rows, uint32_t i, uint32_t jl,
                                          uint32_t j0, uint32_t B, uint32_t K) {
    const uint32_t l = w.lo[jl - j0];
    const uint32_t pos = 2u * jl + 3u * B;
    const uint32_t e = pos - w.plo[i];
    return (B >= l && B - l < K && pos >= w.plo[i] && e < w.span[i]) ? (int)rows[w.off[i] + e] : -1;
}

// Block walks from LDS rows: bend and path as serial_walk_blocks_kernel (one
// workgroup of kWalkLdsThreads per block; the pixel's span and row offset stay
// in registers between pixel changes, so a step is one dependent LDS read).
constexpr uint32_t kWalkLdsThreads = 1024;
__global__ __launch_bounds__(kWalkLdsThreads) void serial_walk_blocks_lds_kernel(
    const uint32_t *__restrict__ ctrl, uint32_t *__restrict__ bend, uint32_t *__restrict__ path,
    const uint32_t *__restrict__ lo, uint32_t L, uint32_t Kmax, uint32_t R, uint32_t nserial,
    const float *__restrict__ ptab, FastDiv ppix) {
    if (ctrl[0] != 0u) return;
    const uint32_t K = serial_k(ctrl, Kmax);
    const uint32_t a = ctrl[4];
    const uint32_t n = min(L, nserial - a);
    const uint32_t nb = (n + R - 1) / R;
    const uint32_t blk = blockIdx.x;
    if (blk >= nb) return;  // (whole workgroups)
    __shared__ WalkRowsLds w;
    extern __shared__ uint8_t rows[];
    const uint32_t j0 = blk * R, j1 = min(j0 + R, n);
    walk_stage_rows(w, rows, ctrl[7], ptab, lo, a, n, j0, j1, K, ppix);
    const uint32_t spp = ppix.d, p0 = fastdiv_apply(a, ppix);
    const size_t stride = (size_t)nb * K;
    for (uint32_t k0 = threadIdx.x; k0 < K; k0 += blockDim.x) {
        const size_t t = (size_t)blk * K + k0;
        uint32_t B = w.lo[0] + k0;
        uint32_t i = 0;                                     // local pixel of sample jl, - qa
        uint32_t jnext = (p0 + w.qa + 1u) * spp - a;        // the next pixel's first sample
        uint32_t plo = w.plo[0], span = w.span[0], off = w.off[0];
        uint32_t jl = j0;
        for (; jl < j1; ++jl) {
#ifndef RT_DIAG_NO_PATH  // (timing-only diagnostic build: no path records, wrong states)
            path[(size_t)(jl - j0) * stride + t] = B;
#endif
            if (jl == jnext) {
                ++i;
                jnext += spp;
                plo = w.plo[i];
                span = w.span[i];
                off = w.off[i];
            }
            const uint32_t l = w.lo[jl - j0];
            const uint32_t pos = 2u * jl + 3u * B;
            const uint32_t e = pos - plo;
            if (!(B >= l && B - l < K && pos >= plo && e < span)) break;
            B += rows[off + e];
        }
        bend[t] = jl == j1 ? B : kWalkLeft | (jl - j0);
    }
}

// Superblocks of kSuperBlocks blocks: for every candidate start of a
// superblock's first block, the chain through its blocks' ends (bend), so that
// the finish kernel's chain is one dependent load per superblock.  sbend[sb *
// K + k]: the superblock's end offset, or kWalkLeft | the block (within it)
// where the chain stopped; sB[blk * K + k]: the offset at the start of its
// block blk (nb * K u32, coalesced over k).
constexpr uint32_t kSuperBlocks = 16;
constexpr size_t kSuperLdsBytes = 48 * 1024;  // serial_walk_super_lds_kernel's staged block ends
__global__ __launch_bounds__(256) void serial_walk_super_kernel(
    const uint32_t *__restrict__ ctrl, const uint32_t *__restrict__ bend, const uint32_t *__restrict__ lo,
    uint32_t *__restrict__ sbend, uint32_t *__restrict__ sB, uint32_t L, uint32_t Kmax, uint32_t R,
    uint32_t nserial) {
    if (ctrl[0] != 0u) return;
    const uint32_t K = serial_k(ctrl, Kmax);
    const uint32_t a = ctrl[4];
    const uint32_t n = min(L, nserial - a);
    const uint32_t nb = (n + R - 1) / R;
    const uint32_t ns = (nb + kSuperBlocks - 1) / kSuperBlocks;
    const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= ns * K) return;
    const uint32_t sb = t / K, k0 = t - sb * K;
    const uint32_t b0 = sb * kSuperBlocks, b1 = min(nb, b0 + kSuperBlocks);
    uint32_t B = lo[b0 * R] + k0;
    uint32_t blk = b0;
    for (; blk < b1; ++blk) {
        sB[(size_t)blk * K + k0] = B;
        const uint32_t l = lo[blk * R];
        if (!(B >= l && B - l < K)) break;
        const uint32_t e = bend[(size_t)blk * K + (B - l)];
        if (e & kWalkLeft) break;
        B = e;
    }
    sbend[t] = blk == b1 ? B : kWalkLeft | (blk - b0);
}

// The same with the superblock's block ends staged in LDS (one workgroup per
// superblock, kSuperBlocks * K u32 <= kSuperLdsBytes): the chain's dependent
// reads come from LDS instead of L2.
__global__ __launch_bounds__(1024) void serial_walk_super_lds_kernel(
    const uint32_t *__restrict__ ctrl, const uint32_t *__restrict__ bend, const uint32_t *__restrict__ lo,
    uint32_t *__restrict__ sbend, uint32_t *__restrict__ sB, uint32_t L, uint32_t Kmax, uint32_t R,
    uint32_t nserial) {
    if (ctrl[0] != 0u) return;
    const uint32_t K = serial_k(ctrl, Kmax);
    const uint32_t a = ctrl[4];
    const uint32_t n = min(L, nserial - a);
    const uint32_t nb = (n + R - 1) / R;
    const uint32_t ns = (nb + kSuperBlocks - 1) / kSuperBlocks;
    const uint32_t sb = blockIdx.x;
    if (sb >= ns) return;  // (whole workgroups)
    extern __shared__ uint32_t be[];  // bend of the superblock's blocks, [blk - b0][k]
    __shared__ uint32_t blo[kSuperBlocks];
    const uint32_t b0 = sb * kSuperBlocks, b1 = min(nb, b0 + kSuperBlocks);
    for (uint32_t i = threadIdx.x; i < (b1 - b0) * K; i += blockDim.x) be[i] = bend[(size_t)b0 * K + i];
    if (threadIdx.x < b1 - b0) blo[threadIdx.x] = lo[(b0 + threadIdx.x) * R];
    __syncthreads();
    for (uint32_t k0 = threadIdx.x; k0 < K; k0 += blockDim.x) {
        uint32_t B = blo[0] + k0;
        uint32_t blk = b0;
        for (; blk < b1; ++blk) {
            sB[(size_t)blk * K + k0] = B;
            const uint32_t l = blo[blk - b0];
            if (!(B >= l && B - l < K)) break;
            const uint32_t e = be[(blk - b0) * K + (B - l)];
            if (e & kWalkLeft) break;
            B = e;
        }
        sbend[(size_t)sb * K + k0] = blk == b1 ? B : kWalkLeft | (blk - b0);
    }
}

__global__ __launch_bounds__(256) void serial_walk_finish_kernel(
    uint32_t *__restrict__ ctrl, const float *__restrict__ table, SerialPred M,
    const double *__restrict__ V, uint32_t npix, uint32_t spp, const uint32_t *__restrict__ win,
    const uint32_t *__restrict__ bend, const uint32_t *__restrict__ path, uint32_t *__restrict__ states,
    uint32_t *__restrict__ fin, const uint32_t *__restrict__ lo, const uint32_t *__restrict__ sbend,
    const uint32_t *__restrict__ sB, uint32_t L, uint32_t Lw, uint32_t Kmax, uint32_t R, uint32_t depth,
    uint32_t nserial, float z, float sfloor) {
    __shared__ uint32_t bstart[kMaxWalkBlocks];
    __shared__ uint32_t blo[kMaxWalkBlocks];
    __shared__ uint32_t nfull;
    __shared__ uint32_t scol[kMaxWalkBlocks / kSuperBlocks + 1];  // the chain's column in each superblock
    __shared__ uint32_t cB, cblk, cleft;
    if (ctrl[0] != 0u) {
        if (fin && threadIdx.x == 0) fin[1] = fin[3] = 0u;  // (the states kernels: nothing)
        return;
    }
    const uint32_t K = serial_k(ctrl, Kmax);
    const uint32_t a = ctrl[4];
    const uint32_t n = min(L, nserial - a);
    const uint32_t nb = (n + R - 1) / R;
    const uint32_t ns = (nb + kSuperBlocks - 1) / kSuperBlocks;
    for (uint32_t blk = threadIdx.x; blk < nb; blk += blockDim.x)
        blo[blk] = lo ? lo[blk * R] : serial_lo(M, a, blk * R, K, depth, nserial);
    __syncthreads();
    // The chain through the superblock ends: one dependent load per
    // superblock (the block-by-block chain was 256 dependent L2 loads, 98 us
    // per iteration on c_raytracer 960x540x16); where it stops, the block and
    // its start offset come from the superblock's recorded block starts.
    if (threadIdx.x == 0) {
        uint32_t B = 0, sb = 0, blk = nb, left = 0;
        for (; sb < ns; ++sb) {
            const uint32_t b0 = sb * kSuperBlocks, l = blo[b0];
            if (!(B >= l && B - l < K)) {  // outside the first block's window
                blk = b0;
                break;
            }
            const uint32_t col = sb * K + (B - l);
            scol[sb] = col;
            const uint32_t e = sbend[col];
            if (e & kWalkLeft) {
                blk = b0 + (e & ~kWalkLeft);
                B = sB[(size_t)blk * K + (col - sb * K)];
                const uint32_t lb = blo[blk];
                if (B >= lb && B - lb < K) {
                    const uint32_t eb = bend[(size_t)blk * K + (B - lb)];
                    left = eb == kWalkInvalid ? 0u : eb & ~kWalkLeft;  // samples resolved in blk
                }
                break;
            }
            B = e;
        }
        cB = B;
        cblk = blk;
        cleft = left;
    }
    __syncthreads();
    // the full blocks' start offsets and path columns, in parallel
    for (uint32_t blk = threadIdx.x; blk < cblk; blk += blockDim.x) {
        const uint32_t sb = blk / kSuperBlocks;
        const uint32_t Bb = sB[(size_t)blk * K + (scol[sb] - sb * K)];
        bstart[blk] = Bb;
        if (fin) fin[4 + blk] = blk * K + (Bb - blo[blk]);  // the block's path column
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        uint32_t B = cB, blk = cblk;
        nfull = blk;
        uint32_t done = min(blk * R, n);
        if (fin) {
            if (blk < nb && cleft > 0u) {
                // the path leaves a window inside this block, after cleft
                // samples whose states the block walk's path holds, as it
                // holds the start offset of the sample that left
                const uint32_t col = blk * K + (B - blo[blk]);
                fin[4 + blk] = col;
                B = path[(size_t)cleft * nb * K + col];
                done = blk * R + cleft;
            }
            fin[0] = a;
            fin[1] = blk;
            fin[2] = nb * K;
            fin[3] = done;  // the states to gather: samples [0, done) of the iteration
        }
        if (blk < nb && fin) {
            ctrl[6] += 1u;
        } else if (blk < nb) {
            // the path leaves a window inside this block: resolve it lane-serially
            // up to that sample (the window of the block's first sample holds B:
            // it was the previous block's valid end, or 0)
            const uint32_t j1 = min(blk * R + R, n);
            for (uint32_t jl = blk * R; jl < j1; ++jl) {
                const uint32_t nB = walk_step(table, M, a, K, depth, nserial, jl, B, lo);
                if (nB == kWalkInvalid) break;
                states[a + jl] = win[2u * jl + 3u * B];
                B = nB;
                done = jl + 1;
            }
            ctrl[6] += 1u;
        }
        ctrl[1] = win[2u * done + 3u * B];
        ctrl[2] += B;
        ctrl[3] += 1u;
        ctrl[4] = a + done;
        // (the next iteration's reuse of this one's pixel table: its window
        // starts at offset D = 2 done + 3 B of this one's; the first sample and
        // the row stride of this one's table)
        ctrl[8] = 2u * done + 3u * B;
        ctrl[9] = 1u;
        ctrl[10] = a;
        ctrl[11] = ctrl[7];
        ctrl[7] = 0u;  // (the next window kernel's pixel span, atomicMax)
        if (a + done >= nserial) ctrl[0] = 1u;
        if (V != nullptr) {
            // the next iteration's windows: +-z sigma of the scatter-count
            // deviation its samples can accumulate (V: prefix sums of the
            // per-sample variances from the estimate pass), plus the spread of
            // one sample; never more than the launch's Kmax
            // V: per-pixel prefix sums P (npix + 1) then variances (npix); the
            // variance of samples [0, j) is P[p] + (j - p spp) var[p], p = j / spp
            auto vsum = [&](uint32_t j) {
                const uint32_t q = min(j / spp, npix);
                return q < npix ? V[q] + (double)(j - q * spp) * V[npix + 1 + q] : V[npix];
            };
            const uint32_t a2 = min(a + done, nserial), e = min(a2 + Lw, nserial);
            const double v = vsum(e) - vsum(a2);
            const double w = ceil(2.0 * (double)z * (sqrt(v > 0.0 ? v : 0.0) + (double)sfloor * sqrt((double)(e - a2)))) +
                             (double)(2u * depth + 2u);
            ctrl[5] = w >= (double)Kmax ? Kmax : (uint32_t)w;
        }
    }
    __syncthreads();
    if (fin) return;  // the full blocks' states: serial_states_kernel (a gather)
    for (uint32_t blk = threadIdx.x; blk < nfull; blk += blockDim.x) {
        uint32_t B = bstart[blk];
        const uint32_t j1 = min(blk * R + R, n);
        for (uint32_t jl = blk * R; jl < j1; ++jl) {
            states[a + jl] = win[2u * jl + 3u * B];
            B = walk_step(table, M, a, K, depth, nserial, jl, B, lo);
        }
    }
}

// The start states of the iteration's full blocks, one thread per sample:
// the path the block walk recorded for the block's true start (fin, written by
// serial_walk_finish_kernel: {a, full blocks, path stride, samples of the
// iteration, column per block}).
__global__ __launch_bounds__(256) void serial_states_kernel(const uint32_t *__restrict__ fin,
                                                            const uint32_t *__restrict__ path,
                                                            const uint32_t *__restrict__ win,
                                                            uint32_t *__restrict__ states, uint32_t R) {
    const uint32_t jl = blockIdx.x * blockDim.x + threadIdx.x;
    if (jl >= fin[3]) return;
    const uint32_t blk = jl / R;
    const uint32_t B = path[(size_t)(jl - blk * R) * fin[2] + fin[4 + blk]];
    states[fin[0] + jl] = win[2u * jl + 3u * B];
}

// ---- coalescing block search (kRngSerialCoalesce)
// The count pass traces every (sample, candidate) pair of an iteration (L K
// traces), yet the candidate paths of a block coalesce: two candidates whose
// offsets meet at some sample share every later step, and in a random walk
// with per-sample variance s^2 only about K / sqrt(pi s^2 n) of K neighbouring
// starts are still distinct after n samples.  Here one workgroup owns one
// block of R samples: it keeps the block's distinct live offsets (sorted, in
// LDS) and the live slot of each of the K candidates of the block's first
// sample, traces each live offset once per sample, and merges equal offsets.
// It writes what serial_walk_blocks_kernel derives from the count table --
// bend (the block end of every candidate, or kWalkLeft | the samples walked)
// and path (the offset of every candidate at every sample) -- so the
// superblock, finish and gather kernels run unchanged.

// One sample of the reference's ray_color (common.rs:263-285) from stream
// state rng, for frame sample j: the number of diffuse/metal scatters b (the
// sample draws 2 + 3b numbers, common.rs:335-336 and 32-38).  The same helper
// arithmetic as trace_kernel's lane state machine, without colours: whole
// walks, the static triangle tree at every bounce (the camera tree and the
// primary lists are exact shortcuts of it), no sphere lists.
template <bool kBvh, bool kLds, int kMesh>
__device__ __forceinline__ uint32_t serial_trace_b(const TraceParams &p, const BvhView &view, uint32_t sph_root,
                                                uint32_t rng, uint32_t j) {
    const uint32_t pix = fdiv(j, p.div_sspp);
    const uint32_t row = fdiv(pix, p.div_width);
    const uint32_t col = pix - row * p.width;
    const float un = draw_plus(rng, (float)col);  // camera.rs:84-89 via common.rs:335-337
    const float vn = draw_plus(rng, (float)row);
#ifndef RT_NO_XDIV
    const bool xd = p.xdiv_uv != 0;
#else
    const bool xd = false;
#endif
    const float u = xd ? xdiv(un, p.wden, p.wrcp) : un / p.wden;
    const float v = xd ? xdiv(vn, p.hden, p.hrcp) : vn / p.hden;
    const F3 h = f3(p.cam[6], p.cam[7], p.cam[8]);
    const F3 vv = f3(p.cam[9], p.cam[10], p.cam[11]);
    F3 org = f3(p.cam[0], p.cam[1], p.cam[2]);
    const F3 llc = f3(p.cam[3], p.cam[4], p.cam[5]);
    F3 dir = unit(((llc + scale(h, u)) + scale(vv, v)) - org);
    uint32_t b = 0, cnt = 0;  // (cnt: the helpers' work counters, unused)
    for (int32_t bounce = 0; bounce < p.depth; ++bounce) {
        const F3 inv = f3(slab_rcp(dir.x), slab_rcp(dir.y), slab_rcp(dir.z));
        const uint32_t oct = (inv.x < 0.0f ? 1u : 0u) | (inv.y < 0.0f ? 2u : 0u) | (inv.z < 0.0f ? 4u : 0u);
        float best_t = __builtin_inff();
        int best_i = -1;
        if (kBvh) {  // World::hit (common.rs:241-247) through the exact tree
            spheres_big(p, org, dir, best_t, best_i);
            constexpr uint32_t kEnd = kLds ? 0xFFFFu : kNodeEndDev;
            const SphBound bnd = sph_bound(p, org);
            F3 nlo, nhi;
            sphere_slabs(org, inv, sph_inflation(p, bnd, best_t), nlo, nhi);
            const uint32_t ooff = kLds ? 4u * oct : oct;
            uint32_t node = sphere_walk_entry<kLds>(sph_root, oct, p.nnodes);
            do {
                uint32_t leaf;
                if (sphere_node<kLds>(view, inv, ooff, best_t, nlo, nhi, node, leaf, cnt))
                    sphere_leaf(view, org, dir, leaf, best_t, best_i, cnt);
            } while (node != kEnd);
        } else {
            spheres_brute(p, org, dir, best_t, best_i);
        }
        float tri_t = __builtin_inff();  // Mesh::hit (common.rs:178-223)
        int tri_i = -1;
        if (kMesh == 2) {
            float e = 0.0f;
            if (tri_begin(p, org, dir, best_t, false, e, tri_t, tri_i, cnt, cnt)) {
                const F3 dlt2 = f3(2.0f * (org.x - p.tbvh_oc[0]), 2.0f * (org.y - p.tbvh_oc[1]),
                                   2.0f * (org.z - p.tbvh_oc[2]));
                F3 nlo, nhi;
                sphere_slabs(org, inv, e, nlo, nhi);
                float cap = fminf(best_t, tri_t);
                uint32_t node = 0;
                do {
                    uint32_t leaf;
                    if (tri_node(p, nlo, nhi, inv, dlt2, false, cap, node, leaf, cnt)) {
                        tri_leaf(p, org, dir, false, leaf, best_t, tri_t, tri_i, cnt, cnt);
                        cap = fminf(best_t, tri_t);
                    }
                } while (node != kNodeEndDev);
            }
        } else if (kMesh == 1) {
            triangles_brute(p, org, dir, best_t, tri_t, tri_i, cnt);
        }
        if (tri_i < 0 && best_i < 0) return b;  // background (common.rs:276-281): no draws
        F3 pos, nrm;
        uint32_t kind;
        float param;
        if (tri_i >= 0) {  // a triangle wins a tie against a sphere
            pos = org + scale(dir, tri_t);
            const float4 *g = p.tri_geo + 4u * (uint32_t)tri_i;
            const float4 A = g[0], Nn = g[3];
            nrm = f3(Nn.x, Nn.y, Nn.z);
            const float *m = p.mats + 8u * __float_as_uint(A.w);
            kind = __float_as_uint(m[0]);
            param = m[4];
        } else {
            const float4 S = view.shade[2 * best_i];
            param = view.shade[2 * best_i + 1].w;
            kind = view.kinds[best_i];
            pos = org + scale(dir, best_t);
            nrm = unit(divide_by(pos - f3(S.x, S.y, S.z), S.w));  // common.rs:95
        }
        F3 v = nrm;
        bool keep_normal = false;
        if (kind == kMatDiffuse || kind == kMatMetal) {
            const F3 ru = draw_unit(rng);
            ++b;
            if (kind == kMatDiffuse) {  // materials.rs:42-52
                v = nrm + ru;
                const float eps = 1e-8f;
                keep_normal = fabsf(v.x) < eps && fabsf(v.y) < eps && fabsf(v.z) < eps;
            } else {  // materials.rs:54-63: absorbed when the scatter points inward
                const F3 refl = dir - scale(nrm, 2.0f * dot(dir, nrm));
                v = refl + scale(ru, param);
                if (!(dot(v, nrm) >= 0.0f)) return b;
            }
        } else if (kind == kMatDielectric) {  // materials.rs:65-97 (no draws)
            F3 n2 = nrm;
            float eta = param;
            if (dot(dir, nrm) >= 0.0f) { n2 = -nrm; eta = 1.0f / param; }
            const float cos_t = dot(-dir, n2);
            const F3 perp = scale(dir + scale(n2, cos_t), eta);
            const F3 par = scale(n2, -xsqrt(fabsf(1.0f - dot(perp, perp))));
            v = perp + par;
        } else {
            return b;  // Emission (materials.rs:100-102)
        }
        org = pos;
        dir = keep_normal ? nrm : unit(v);
    }
    return b;  // depth exhausted (common.rs:284)
}

// Exclusive prefix sum of one u32 per thread over the 256-thread workgroup
// (wave scans, then the 4 wave totals); *total gets the sum.  Contains barriers.
__device__ __forceinline__ uint32_t block_exscan256(uint32_t v, uint32_t *wsum, uint32_t *total) {
    const uint32_t lane = threadIdx.x & (kWave - 1u), wv = threadIdx.x / kWave;
    uint32_t x = v;
#pragma unroll
    for (uint32_t off = 1; off < kWave; off <<= 1) {
        const uint32_t y = __shfl_up(x, off);
        if (lane >= off) x += y;
    }
    if (lane == kWave - 1u) wsum[wv] = x;
    __syncthreads();
    uint32_t before = 0;
    for (uint32_t w = 0; w < wv; ++w) before += wsum[w];
    *total = wsum[0] + wsum[1] + wsum[2] + wsum[3];
    return before + x - v;
}

constexpr uint32_t kCoalesceThreads = 256;
constexpr uint32_t kSlotDead = 0xFFFFFFFFu;

// LDS bytes of the coalescing workgroup after the tree: cand (u16 x K), three
// u32 lists of Kp = K + depth + 1 live offsets, two bitmaps and a prefix of W
// words (all 16-B aligned)
__host__ __device__ inline size_t coalesce_lds_bytes(uint32_t K, uint32_t depth) {
    const size_t Kp = (size_t)K + depth + 1, W = (Kp + 31) / 32;
    auto al = [](size_t x) { return (x + 15) & ~(size_t)15; };
    return al(2 * (size_t)K) + 3 * al(4 * Kp) + 3 * al(4 * W) + 16;
}

// Waves per SIMD the brute-force coalescing kernels are compiled for (their
// live set fits 64 VGPRs without spills at 8; 1 = unconstrained, 76 VGPRs, 6
// waves); the tree variants stay unconstrained (they would spill at 8)
#ifndef RT_COALESCE_WAVES_BRUTE
#define RT_COALESCE_WAVES_BRUTE 8
#endif
template <bool kBvh, bool kLds, int kMesh>
__global__ __launch_bounds__(kCoalesceThreads)
__attribute__((amdgpu_waves_per_eu(kBvh ? 1 : RT_COALESCE_WAVES_BRUTE, 8)))
void serial_coalesce_kernel(TraceParams p, uint32_t *__restrict__ path,
                                                                           uint32_t *__restrict__ bend, uint32_t L,
                                                                           uint32_t Kmax, uint32_t R,
                                                                           uint32_t tree_bytes,
                                                                           unsigned long long *__restrict__ dbg) {
    if (p.ctrl[0] != 0u) return;
    const uint32_t K = serial_k(p.ctrl, Kmax);
    const uint32_t a = p.ctrl[4];
    const uint32_t n = min(L, p.nserial - a);
    const uint32_t nb = (n + R - 1) / R;
    const uint32_t blk = blockIdx.x;
    if (blk >= nb) return;  // (whole workgroup, before any barrier)
    extern __shared__ float4 lds[];
    BvhView view;
    const uint32_t sph_root = stage_tree<kLds>(p, lds, view);
    const uint32_t depth = p.depth > 0 ? (uint32_t)p.depth : 0u;
    const uint32_t Kp = K + depth + 1, W = (Kp + 31) / 32;
    auto al = [](uint32_t x) { return (x + 15u) & ~15u; };
    char *c = reinterpret_cast<char *>(lds) + tree_bytes;
    uint16_t *cand = reinterpret_cast<uint16_t *>(c);  // live slot of each candidate (0xFFFF: left)
    c += al(2 * K);
    uint32_t *LB = reinterpret_cast<uint32_t *>(c);    // live offsets, ascending
    c += al(4 * Kp);
    uint32_t *LBn = reinterpret_cast<uint32_t *>(c);   // the next sample's
    c += al(4 * Kp);
    uint32_t *NB = reinterpret_cast<uint32_t *>(c);    // each live offset's end (kSlotDead: left)
    c += al(4 * Kp);
    uint32_t *bits0 = reinterpret_cast<uint32_t *>(c);  // the ends present, relative to the window
    c += al(4 * W);
    uint32_t *bits1 = reinterpret_cast<uint32_t *>(c);
    c += al(4 * W);
    uint32_t *wpre = reinterpret_cast<uint32_t *>(c);   // exclusive popcount prefix of the bitmap
    c += al(4 * W);
    uint32_t *wsum = reinterpret_cast<uint32_t *>(c);   // block_exscan256's wave totals
    // (all dynamic: the tree's LDS node addresses assume no static LDS below it)
    const uint32_t t = threadIdx.x;
    const uint32_t j0 = blk * R, j1 = min(j0 + R, n);
    const size_t stride = (size_t)nb * K;
    const uint32_t base = p.slo[j0];
    for (uint32_t k = t; k < K; k += kCoalesceThreads) {
        cand[k] = (uint16_t)k;
        LB[k] = base + k;
    }
    for (uint32_t w = t; w < W; w += kCoalesceThreads) bits0[w] = bits1[w] = 0u;
    uint32_t nlive = K;
    uint32_t d_traces = 0, d_passes = 0;  // (dbg: RT_AMD_SERIAL_DEBUG)
    __syncthreads();
    for (uint32_t s = 0; j0 + s < j1; ++s) {
        d_traces += nlive;
        d_passes += (nlive + kCoalesceThreads - 1) / kCoalesceThreads;
        const uint32_t jl = j0 + s;
        const uint32_t l = p.slo[jl];  // the window of sample jl: [l, l + K)
        uint32_t *bits = (s & 1u) ? bits1 : bits0;
        uint32_t *bnext = (s & 1u) ? bits0 : bits1;
        // every distinct live offset once: its sample's end offset
        for (uint32_t i = t; i < nlive; i += kCoalesceThreads) {
            const uint32_t B = LB[i];
            uint32_t e = kSlotDead;
            if (B >= l && B - l < K) {
                e = B + serial_trace_b<kBvh, kLds, kMesh>(p, view, sph_root, p.win[2u * jl + 3u * B], a + jl);
                const uint32_t r = e - l;  // < K + depth
                atomicOr(&bits[r >> 5], 1u << (r & 31u));
            }
            NB[i] = e;
        }
        __syncthreads();
        // ranks of the distinct ends: popcount prefix over the bitmap words
        const uint32_t per = (W + kCoalesceThreads - 1) / kCoalesceThreads;
        const uint32_t w0 = min(t * per, W), w1 = min(w0 + per, W);
        uint32_t cntw = 0;
        for (uint32_t w = w0; w < w1; ++w) cntw += __popc(bits[w]);
        uint32_t total = 0;
        uint32_t run = block_exscan256(cntw, wsum, &total);
        for (uint32_t w = w0; w < w1; ++w) {
            wpre[w] = run;
            run += __popc(bits[w]);
        }
        __syncthreads();
        auto rank = [&](uint32_t e) {
            const uint32_t r = e - l;
            return wpre[r >> 5] + __popc(bits[r >> 5] & ((1u << (r & 31u)) - 1u));
        };
        for (uint32_t i = t; i < nlive; i += kCoalesceThreads) {
            const uint32_t e = NB[i];
            if (e != kSlotDead) LBn[rank(e)] = e;  // (merged slots write the same value)
        }
        for (uint32_t k = t; k < K; k += kCoalesceThreads) {
            const uint32_t sl = cand[k];
            if (sl == 0xFFFFu) continue;
            path[(size_t)s * stride + (size_t)blk * K + k] = LB[sl];
            const uint32_t e = NB[sl];
            if (e == kSlotDead) {
                cand[k] = 0xFFFFu;
                bend[(size_t)blk * K + k] = kWalkLeft | s;
            } else {
                cand[k] = (uint16_t)rank(e);
            }
        }
        for (uint32_t w = t; w < W; w += kCoalesceThreads) bnext[w] = 0u;
        nlive = total;
        uint32_t *sw = LB;
        LB = LBn;
        LBn = sw;
        __syncthreads();
    }
    for (uint32_t k = t; k < K; k += kCoalesceThreads) {
        const uint32_t sl = cand[k];
        if (sl != 0xFFFFu) bend[(size_t)blk * K + k] = LB[sl];
    }
    if (dbg != nullptr && t == 0) {
        atomicAdd(dbg, (unsigned long long)d_traces);
        atomicAdd(dbg + 1, (unsigned long long)d_passes);
        atomicAdd(dbg + 2, 1ull);
        atomicAdd(dbg + 3, (unsigned long long)K * (j1 - j0));
    }
}

template <bool kBvh, bool kLds>
static void launch_coalesce_m(const TraceParams &p, uint32_t *path, uint32_t *bend, uint32_t L, uint32_t Kmax,
                              uint32_t R, size_t tree_bytes, size_t lds, unsigned long long *dbg,
                              hipStream_t stream) {
    const uint32_t nb = (L + R - 1) / R;
    const int mesh = trace_mesh_kind(p.ntri != 0, p.tnodes != 0);
    if (mesh == 2)
        hipLaunchKernelGGL((serial_coalesce_kernel<kBvh, kLds, 2>), dim3(nb), dim3(kCoalesceThreads), lds, stream, p,
                           path, bend, L, Kmax, R, (uint32_t)tree_bytes, dbg);
    else if (mesh == 1)
        hipLaunchKernelGGL((serial_coalesce_kernel<kBvh, kLds, 1>), dim3(nb), dim3(kCoalesceThreads), lds, stream, p,
                           path, bend, L, Kmax, R, (uint32_t)tree_bytes, dbg);
    else
        hipLaunchKernelGGL((serial_coalesce_kernel<kBvh, kLds, 0>), dim3(nb), dim3(kCoalesceThreads), lds, stream, p,
                           path, bend, L, Kmax, R, (uint32_t)tree_bytes, dbg);
}

size_t serial_coalesce_search_lds(uint32_t K, uint32_t depth) { return coalesce_lds_bytes(K, depth); }

size_t serial_coalesce_lds(const TraceParams &p, uint32_t K, bool tree_lds) {
    const size_t tb = tree_lds ? (trace_lds_bytes(p) + 15) & ~(size_t)15 : 0;
    return tb + coalesce_lds_bytes(K, p.depth > 0 ? (uint32_t)p.depth : 0u);
}

hipError_t launch_serial_coalesce(const TraceParams &p, uint32_t *path, uint32_t *bend, uint32_t L, uint32_t Kmax,
                                  uint32_t R, bool tree_lds, unsigned long long *dbg, hipStream_t stream) {
    if (!L || !R) return hipSuccess;
    const size_t tb = tree_lds ? (trace_lds_bytes(p) + 15) & ~(size_t)15 : 0;
    const size_t lds = serial_coalesce_lds(p, Kmax, tree_lds);
    if (p.nnodes && tree_lds) launch_coalesce_m<true, true>(p, path, bend, L, Kmax, R, tb, lds, dbg, stream);
    else if (p.nnodes) launch_coalesce_m<true, false>(p, path, bend, L, Kmax, R, tb, lds, dbg, stream);
    else launch_coalesce_m<false, false>(p, path, bend, L, Kmax, R, tb, lds, dbg, stream);
    return hipGetLastError();
}

// ---- the estimate reduction (render.h serial_tab_doubles for the layout)
// One thread per pixel: its spp * R scatter counts (contiguous) summed in
// double; a negative or NaN count (a lost draw count) raises the flag.
__global__ __launch_bounds__(256) void serial_moments_kernel(const float *__restrict__ est, uint32_t pix0,
                                                             uint32_t n, uint32_t spp, uint32_t R,
                                                             double scale, double *__restrict__ tab,
                                                             uint32_t npix) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const uint32_t per = spp * R;
    const float *src = est + (size_t)i * per;
    double s = 0.0, sq = 0.0;
    bool bad = false;
    for (uint32_t k = 0; k < per; ++k) {
        const float b = src[k];
        bad |= !(b >= 0.0f);
        s += (double)b;
        sq += (double)b * (double)b;
    }
    const uint32_t p = pix0 + i;
    const double mu = s / (double)per;
    const double v = sq / (double)per - mu * mu;
    tab[npix + 1 + p] = mu;
    tab[3 * (size_t)npix + 2 + p] = (v > 0.0 ? v : 0.0) * scale;
    tab[4 * (size_t)npix + 2 + p] = sq - s * mu;
    if (bad) tab[5 * (size_t)npix + 5] = 1.0;
}

// Prefix sums over pixels of (spp mu, spp var, ss) in tiles of kScanTile:
// tile totals, one workgroup's exclusive scan of the totals, then each tile's
// own scan from its offset.  The shape is fixed, so the sums are the same
// bits on every call.
constexpr uint32_t kScanTile = 1024;
__device__ __forceinline__ void scan_inputs(const double *tab, uint32_t npix, uint32_t spp, uint32_t p,
                                            double v[3]) {
    if (p >= npix) { v[0] = v[1] = v[2] = 0.0; return; }
    v[0] = (double)spp * tab[npix + 1 + p];
    v[1] = (double)spp * tab[3 * (size_t)npix + 2 + p];
    v[2] = tab[4 * (size_t)npix + 2 + p];
}

// inclusive scan of 256 values x 3 across the workgroup (Hillis-Steele in LDS)
__device__ __forceinline__ void block_scan3(double (*sh)[256], double v[3]) {
    const uint32_t t = threadIdx.x;
#pragma unroll
    for (int c = 0; c < 3; ++c) sh[c][t] = v[c];
    __syncthreads();
    for (uint32_t off = 1; off < 256; off <<= 1) {
        double a[3];
#pragma unroll
        for (int c = 0; c < 3; ++c) a[c] = t >= off ? sh[c][t - off] : 0.0;
        __syncthreads();
#pragma unroll
        for (int c = 0; c < 3; ++c) sh[c][t] += a[c];
        __syncthreads();
    }
#pragma unroll
    for (int c = 0; c < 3; ++c) v[c] = sh[c][t];
    __syncthreads();
}

__global__ __launch_bounds__(256) void serial_scan_tiles_kernel(const double *__restrict__ tab, uint32_t npix,
                                                                uint32_t spp, double *__restrict__ tsum) {
    __shared__ double sh[3][256];
    const uint32_t p0 = blockIdx.x * kScanTile + threadIdx.x * 4u;
    double acc[3] = {0.0, 0.0, 0.0};
    for (uint32_t k = 0; k < 4; ++k) {
        double v[3];
        scan_inputs(tab, npix, spp, p0 + k, v);
#pragma unroll
        for (int c = 0; c < 3; ++c) acc[c] += v[c];
    }
    block_scan3(sh, acc);
    if (threadIdx.x == 255)
#pragma unroll
        for (int c = 0; c < 3; ++c) tsum[3 * blockIdx.x + c] = acc[c];
}

// one workgroup: exclusive scan of the ntiles totals in place
__global__ __launch_bounds__(256) void serial_scan_totals_kernel(double *__restrict__ tsum, uint32_t ntiles) {
    __shared__ double sh[3][256];
    const uint32_t per = (ntiles + 255u) / 256u;
    const uint32_t b = threadIdx.x * per, e = min(b + per, ntiles);
    double acc[3] = {0.0, 0.0, 0.0};
    for (uint32_t i = b; i < e; ++i)
#pragma unroll
        for (int c = 0; c < 3; ++c) acc[c] += tsum[3 * i + c];
    double inc[3] = {acc[0], acc[1], acc[2]};
    block_scan3(sh, inc);
    double run[3];
#pragma unroll
    for (int c = 0; c < 3; ++c) run[c] = inc[c] - acc[c];  // (exclusive: the sum before b)
    if (threadIdx.x == 0)
#pragma unroll
        for (int c = 0; c < 3; ++c) run[c] = 0.0;
    for (uint32_t i = b; i < e; ++i)
#pragma unroll
        for (int c = 0; c < 3; ++c) {
            const double x = tsum[3 * i + c];
            tsum[3 * i + c] = run[c];
            run[c] += x;
        }
}

__global__ __launch_bounds__(256) void serial_scan_apply_kernel(double *__restrict__ tab, uint32_t npix,
                                                                uint32_t spp, const double *__restrict__ tsum) {
    __shared__ double sh[3][256];
    const uint32_t p0 = blockIdx.x * kScanTile + threadIdx.x * 4u;
    double v[4][3], acc[3] = {0.0, 0.0, 0.0};
    for (uint32_t k = 0; k < 4; ++k) {
        scan_inputs(tab, npix, spp, p0 + k, v[k]);
#pragma unroll
        for (int c = 0; c < 3; ++c) acc[c] += v[k][c];
    }
    double inc[3] = {acc[0], acc[1], acc[2]};
    block_scan3(sh, inc);
    double run[3];
#pragma unroll
    for (int c = 0; c < 3; ++c) run[c] = tsum[3 * blockIdx.x + c] + (inc[c] - acc[c]);
    if (threadIdx.x == 0)
#pragma unroll
        for (int c = 0; c < 3; ++c) run[c] = tsum[3 * blockIdx.x + c];
    if (blockIdx.x == 0 && threadIdx.x == 0) {
        tab[0] = 0.0;                         // P[0]
        tab[2 * (size_t)npix + 1] = 0.0;      // PV[0]
    }
    for (uint32_t k = 0; k < 4; ++k) {
        const uint32_t p = p0 + k;
#pragma unroll
        for (int c = 0; c < 3; ++c) run[c] += v[k][c];
        if (p < npix) {
            tab[p + 1] = run[0];
            tab[2 * (size_t)npix + 2 + p] = run[1];
            if (p + 1 == npix) tab[5 * (size_t)npix + 2] = run[2];  // sum of ss
        }
    }
}

// dmax over the window starts a = i q, q = max(1, L / 4) (atomicMax on the
// bits of a non-negative double orders like the doubles), plus V(n0).
__global__ __launch_bounds__(256) void serial_reach_kernel(double *__restrict__ tab, uint32_t npix, uint32_t spp,
                                                           uint32_t L, uint32_t n0) {
    const SerialPred m{tab, tab + npix + 1, spp, npix};
    const uint32_t N = npix * spp;  // (< 2^32, runtime.cpp)
    const uint32_t q = max(1u, L / 4u);
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    unsigned long long *dmax = reinterpret_cast<unsigned long long *>(tab + 5 * (size_t)npix + 3);
    if (i * q < N) {
        const uint32_t a = (uint32_t)(i * q);
        const uint64_t e = (uint64_t)a + L + L / 4u;
        const double d = serial_M(m, e < N ? (uint32_t)e : N) - serial_M(m, a);
        atomicMax(dmax, (unsigned long long)__double_as_longlong(d > 0.0 ? d : 0.0));
    }
    if (i == 0) {
        const double *PV = tab + 2 * (size_t)npix + 1, *var = tab + 3 * (size_t)npix + 2;
        const uint32_t p = n0 / spp;
        tab[5 * (size_t)npix + 4] = p < npix ? PV[p] + (double)(n0 - p * spp) * var[p] : PV[npix];
    }
}

__global__ __launch_bounds__(256) void serial_check_count_kernel(const float *__restrict__ flags, uint32_t n,
                                                                 unsigned long long *__restrict__ count) {
    uint32_t c = 0;
    for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x)
        c += flags[i] != 0.0f ? 1u : 0u;
    for (uint32_t off = kWave / 2; off > 0; off >>= 1) c += __shfl_xor(c, (int)off);
    if ((threadIdx.x & (kWave - 1u)) == 0 && c != 0) atomicAdd(count, (unsigned long long)c);
}

hipError_t launch_serial_check_count(const float *flags, uint32_t n, unsigned long long *count,
                                     hipStream_t stream) {
    if (!n) return hipSuccess;
    const uint32_t want = (n + 255) / 256, blocks = want < 2048 ? want : 2048;
    hipLaunchKernelGGL(serial_check_count_kernel, dim3(blocks), dim3(256), 0, stream, flags, n, count);
    return hipGetLastError();
}

size_t serial_tab_doubles(uint32_t npix) { return 5 * (size_t)npix + 10; }

size_t serial_scan_scratch(uint32_t npix) { return 3 * (size_t)((npix + kScanTile - 1) / kScanTile) + 3; }

hipError_t launch_serial_moments(const float *est, uint32_t pix0, uint32_t n, uint32_t spp, uint32_t R,
                                 double scale, double *tab, uint32_t npix, hipStream_t stream) {
    if (!n) return hipSuccess;
    hipLaunchKernelGGL(serial_moments_kernel, dim3((n + 255) / 256), dim3(256), 0, stream, est, pix0, n, spp,
                       R, scale, tab, npix);
    return hipGetLastError();
}

hipError_t launch_serial_tables(double *tab, double *scratch, uint32_t npix, uint32_t spp, uint32_t L,
                                uint32_t n0, hipStream_t stream) {
    if (!npix) return hipSuccess;
    const uint32_t ntiles = (npix + kScanTile - 1) / kScanTile;
    hipLaunchKernelGGL(serial_scan_tiles_kernel, dim3(ntiles), dim3(256), 0, stream, tab, npix, spp, scratch);
    hipLaunchKernelGGL(serial_scan_totals_kernel, dim3(1), dim3(256), 0, stream, scratch, ntiles);
    hipLaunchKernelGGL(serial_scan_apply_kernel, dim3(ntiles), dim3(256), 0, stream, tab, npix, spp, scratch);
    const uint32_t N = npix * spp, q = L / 4u > 1u ? L / 4u : 1u;
    const uint64_t pts = ((uint64_t)N + q - 1) / q;
    hipLaunchKernelGGL(serial_reach_kernel, dim3((uint32_t)((pts + 255) / 256)), dim3(256), 0, stream, tab,
                       npix, spp, L, n0);
    return hipGetLastError();
}

hipError_t launch_serial_window(uint32_t *ctrl, const uint32_t *jump, uint32_t *win, uint32_t n,
                                SerialPred M, uint32_t *lo, uint32_t L, uint32_t K, uint32_t depth,
                                uint32_t nserial, uint32_t pix_spp, uint32_t pix_emax, uint32_t *counters,
                                uint32_t ncounters, uint4 *spix, uint32_t pix_chunk, const uint4 *spix_prev,
                                hipStream_t stream) {
    if (!n) return hipSuccess;
    const uint32_t threads = std::max((n + kWinPerThread - 1) / kWinPerThread, lo ? std::min(L, 1u << 16) : 0u);
    hipLaunchKernelGGL(serial_window_kernel, dim3((threads + 255) / 256), dim3(256), 0, stream, ctrl,
                       jump, win, n, M, lo, L, K, depth, nserial, pix_spp, pix_emax, counters,
                       counters ? ncounters : 0u, pix_spp != 0u ? spix : nullptr, pix_chunk,
                       pix_spp != 0u && spix != nullptr ? spix_prev : nullptr);
    return hipGetLastError();
}

// One workgroup per local pixel q of the iteration: the table entries of its
// reused range (spix[q].zw, serial_window_kernel) from the previous table.
// Entry e of pixel q is stream position plo(q) + e of this iteration's window,
// i.e. position plo(q) + e + D of the previous one, entry plo(q) + e + D -
// plo'(q') of its pixel's row there: b of a (pixel, stream position) pair is
// the same whichever iteration traced it.
__global__ __launch_bounds__(256) void serial_reuse_kernel(const uint32_t *__restrict__ ctrl,
                                                           const uint4 *__restrict__ spix,
                                                           const uint4 *__restrict__ spix_prev,
                                                           float *__restrict__ ptab,
                                                           const float *__restrict__ ptab_prev, uint32_t spp,
                                                           uint32_t L, uint32_t nserial) {
    if (ctrl[0] != 0u || ctrl[9] == 0u) return;
    const uint32_t a = ctrl[4];
    const uint32_t ln = min(L, nserial - a);
    const uint32_t p0 = a / spp, npq = (a + ln - 1u) / spp - p0 + 1u;
    const uint32_t q = blockIdx.x;
    if (q >= npq) return;
    const uint4 s = spix[q];
    if (s.z > s.w) return;
    const uint32_t E = ctrl[7], Ep = ctrl[11], D = ctrl[8];
    const uint4 so = spix_prev[p0 + q - ctrl[10] / spp];
    const uint32_t e1 = min(s.w, E - 1u);
    for (uint32_t e = s.z + threadIdx.x; e <= e1; e += blockDim.x)
        ptab[(size_t)q * E + e] = ptab_prev[(size_t)(p0 + q - ctrl[10] / spp) * Ep + (s.x + e + D - so.x)];
}

hipError_t launch_serial_reuse(const uint32_t *ctrl, const uint4 *spix, const uint4 *spix_prev, float *ptab,
                               const float *ptab_prev, uint32_t npq_max, uint32_t spp, uint32_t L,
                               uint32_t nserial, hipStream_t stream) {
    if (!npq_max) return hipSuccess;
    hipLaunchKernelGGL(serial_reuse_kernel, dim3(npq_max), dim3(256), 0, stream, ctrl, spix, spix_prev, ptab,
                       ptab_prev, spp, L, nserial);
    return hipGetLastError();
}

// table[jl * K + k] = b of sample jl at offset lo[jl] + k, i.e. at stream
// position 2 jl + 3 (lo[jl] + k) of the iteration, which the pixel table pass
// traced for the sample's pixel q at ptab[q * E + (position - plo(q))]
__global__ __launch_bounds__(256) void serial_pixtab_gather_kernel(const uint32_t *__restrict__ ctrl,
                                                                   const float *__restrict__ ptab,
                                                                   const uint32_t *__restrict__ lo,
                                                                   float *__restrict__ table, uint32_t L,
                                                                   uint32_t Kmax, uint32_t spp, uint32_t nserial) {
    if (ctrl[0] != 0u) return;
    const uint32_t K = serial_k(ctrl, Kmax);
    const uint32_t E = ctrl[7];
    const uint32_t a = ctrl[4];
    const uint32_t n = min(L, nserial - a);
    const uint32_t p0 = a / spp;
    for (uint32_t t = blockIdx.x * blockDim.x + threadIdx.x; t < n * K; t += gridDim.x * blockDim.x) {
        const uint32_t jl = t / K, k = t - jl * K;
        const uint32_t q = (a + jl) / spp - p0;
        const uint32_t jf = q == 0u ? 0u : (p0 + q) * spp - a;
        const uint32_t plo = 2u * jf + 3u * lo[jf];
        const uint32_t pos = 2u * jl + 3u * (lo[jl] + k);
        // (lo is non-decreasing up to a rounding tie of the double prediction:
        // a position outside the traced span reads as "left the window")
        table[t] = (pos >= plo && pos - plo < E) ? ptab[(size_t)q * E + (pos - plo)] : -1.0f;
    }
}

hipError_t launch_serial_pixtab_gather(const uint32_t *ctrl, const float *ptab, const uint32_t *lo, float *table,
                                       uint32_t L, uint32_t K, uint32_t spp, uint32_t nserial, hipStream_t stream) {
    const uint64_t n = (uint64_t)L * K;
    const uint32_t blocks = (uint32_t)std::min<uint64_t>((n + 255) / 256, 4096);
    hipLaunchKernelGGL(serial_pixtab_gather_kernel, dim3(std::max(blocks, 1u)), dim3(256), 0, stream, ctrl, ptab,
                       lo, table, L, K, spp, nserial);
    return hipGetLastError();
}

uint32_t serial_super_words(uint32_t L, uint32_t K, uint32_t R) {
    const uint32_t nb = (L + R - 1) / R;
    return (nb + kSuperBlocks - 1) / kSuperBlocks * K;
}

uint32_t serial_walk_block(uint32_t L) {
    const uint32_t R = (L + 255) / 256;
    return R < 32u ? 32u : R;
}

hipError_t launch_serial_walk(uint32_t *ctrl, const float *table, SerialPred M, const double *V,
                              uint32_t npix, uint32_t spp, float z, float sfloor, const uint32_t *win,
                              uint32_t *states, uint32_t *bend, uint32_t *path, uint32_t *fin,
                              const uint32_t *lo, uint32_t *sbend, uint32_t *sB, uint32_t L, uint32_t Lw,
                              uint32_t K, uint32_t R, uint32_t depth, uint32_t nserial, const float *ptab,
                              uint32_t lds_rows, hipStream_t stream) {
    if (!L || !R) return hipSuccess;
    const uint32_t nb = (L + R - 1) / R;
    if (nb > kMaxWalkBlocks) return hipErrorInvalidValue;
    const uint64_t nt = (uint64_t)nb * K;
    const uint64_t nst = (uint64_t)((nb + kSuperBlocks - 1) / kSuperBlocks) * K;
    if (!fin) path = nullptr;
    // (the coalescing search and the pixel table need the recorded paths: the
    // finish kernel's lane-serial fallback reads a count table)
    if ((table == nullptr || ptab != nullptr) && !path) return hipErrorInvalidValue;
    const FastDiv ppix = make_fastdiv(spp ? spp : 1u);
    // the pixel table's walks from LDS rows (lds_rows bytes per workgroup)
    if (ptab != nullptr && lds_rows != 0) {
        if (R > kMaxWalkR) return hipErrorInvalidValue;
        hipLaunchKernelGGL(serial_walk_blocks_lds_kernel, dim3(nb), dim3(kWalkLdsThreads), lds_rows, stream, ctrl,
                           bend, path, lo, L, K, R, nserial, ptab, ppix);
    } else if (table != nullptr || ptab != nullptr) {
        hipLaunchKernelGGL(serial_walk_blocks_kernel, dim3((uint32_t)((nt + 255) / 256)), dim3(256), 0, stream,
                           ctrl, table, M, bend, path, lo, L, K, R, depth, nserial, ptab, ppix);
    }
    const uint32_t ns = (nb + kSuperBlocks - 1) / kSuperBlocks;
    if ((size_t)kSuperBlocks * K * 4 <= kSuperLdsBytes)
        hipLaunchKernelGGL(serial_walk_super_lds_kernel, dim3(ns), dim3(1024), (size_t)kSuperBlocks * K * 4, stream,
                           ctrl, bend, lo, sbend, sB, L, K, R, nserial);
    else
        hipLaunchKernelGGL(serial_walk_super_kernel, dim3((uint32_t)((nst + 255) / 256)), dim3(256), 0, stream,
                           ctrl, bend, lo, sbend, sB, L, K, R, nserial);
    hipLaunchKernelGGL(serial_walk_finish_kernel, dim3(1), dim3(256), 0, stream, ctrl, table, M, V, npix,
                       spp ? spp : 1u, win, bend, path, states, path ? fin : nullptr, lo, sbend, sB, L, Lw, K,
                       R, depth, nserial, z, sfloor);
    if (path)
        hipLaunchKernelGGL(serial_states_kernel, dim3((L + 255) / 256), dim3(256), 0, stream, fin, path, win,
                           states, R);
    return hipGetLastError();
}

// ------------------------------------------------------------ primary sphere lists
// Device twin of bvh.cpp build_primary_sphere_lists (same double operations in
// the same order, -ffp-contract=off): per tree sphere, the box of its inflated
// ball projected through the inverse camera map to a pixel rectangle (rows
// counted from the bottom, common.rs:327), empty if behind the camera; flag
// bit 0: some ball straddles the camera plane or is not finite (every pixel
// walks).
struct SplConst { double Mi[9], o[3], e_abs, wden, hden; };
// an empty rectangle that every tile culls (lo above any pixel, hi below)
__device__ __forceinline__ int4 spl_empty() { return make_int4(0x7FFFFFFF, -1, 0x7FFFFFFF, -1); }

__global__ __launch_bounds__(256) void spl_rect_kernel(const float4 *__restrict__ prims, uint32_t n,
                                                       SplConst k, uint32_t W, uint32_t H,
                                                       int4 *__restrict__ rects, uint32_t *__restrict__ flag) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const float4 s = prims[i];
    const double c[3] = {s.x, s.y, s.z};
    const double r = sqrt((double)s.w) * (1 + 1e-6);
    const double a = sqrt((c[0] - k.o[0]) * (c[0] - k.o[0]) + (c[1] - k.o[1]) * (c[1] - k.o[1]) +
                          (c[2] - k.o[2]) * (c[2] - k.o[2]));
    const double R = r + 2 * 3e-3 * (a + r) * 1.01 + 2 * k.e_abs;
    int4 rect = spl_empty();
    if (!isfinite(R) || !isfinite(a)) {
        atomicOr(flag, 1u);
        rects[i] = rect;
        return;
    }
    double umin = 1e300, umax = -1e300, vmin = 1e300, vmax = -1e300;
    int front = 0, behind = 0;
    for (int q = 0; q < 8; ++q) {
        const double P[3] = {c[0] + (q & 1 ? R : -R) - k.o[0], c[1] + (q & 2 ? R : -R) - k.o[1],
                             c[2] + (q & 4 ? R : -R) - k.o[2]};
        double w[3];
        for (int t = 0; t < 3; ++t) w[t] = k.Mi[3 * t] * P[0] + k.Mi[3 * t + 1] * P[1] + k.Mi[3 * t + 2] * P[2];
        const double wn = fabs(w[0]) + fabs(w[1]) + fabs(w[2]);
        if (w[2] > 1e-6 * wn) {
            ++front;
            umin = fmin(umin, w[0] / w[2]); umax = fmax(umax, w[0] / w[2]);
            vmin = fmin(vmin, w[1] / w[2]); vmax = fmax(vmax, w[1] / w[2]);
        } else if (w[2] < -1e-6 * wn) {
            ++behind;
        }
    }
    if (behind != 8 && front < 8) atomicOr(flag, 1u);  // straddles the camera plane
    if (front == 8) {
        const double cl = floor(umin * k.wden) - 2, ch = floor(umax * k.wden) + 1;
        const double rl = floor(vmin * k.hden) - 2, rh = floor(vmax * k.hden) + 1;
        if (!(ch < 0 || cl > (double)(W - 1) || rh < 0 || rl > (double)(H - 1)))
            rect = make_int4(cl < 0 ? 0 : (int)cl, ch > (double)(W - 1) ? (int)(W - 1) : (int)ch,
                             rl < 0 ? 0 : (int)rl, rh > (double)(H - 1) ? (int)(H - 1) : (int)rh);
    }
    rects[i] = rect;
}

// One thread per pixel of a 16 x 16 tile (record row 0 = the top image row):
// the first three tree spheres whose rectangle covers it, or "walk" past three
// (bvh.h PrimarySphereLists).  Rectangles are culled against the tile 256 at a
// time and compacted, in tree order, into LDS; a tile whose pixels have all
// overflowed stops early.
__global__ __launch_bounds__(256) void spl_fill_kernel(const int4 *__restrict__ rects, uint32_t n,
                                                       const uint32_t *__restrict__ flag, uint32_t W, uint32_t H,
                                                       uint2 *__restrict__ rec) {
    __shared__ int4 rl[256];
    __shared__ uint32_t ri[256];
    __shared__ uint32_t wc[4];
    const uint32_t tid = threadIdx.x, lane = tid & 63u, wave = tid >> 6;
    const int col = (int)(blockIdx.x * 16 + (tid & 15u)), row = (int)(blockIdx.y * 16 + (tid >> 4));
    const bool on = col < (int)W && row < (int)H;
    const int rb = (int)H - 1 - row;  // counted from the bottom
    // the tile's extent: columns [tc0, tc1], bottom-counted rows [tr0, tr1]
    const int tc0 = (int)(blockIdx.x * 16), tc1 = min(tc0 + 15, (int)W - 1);
    const int tr1 = (int)H - 1 - (int)(blockIdx.y * 16), tr0 = max(tr1 - 15, 0);
    uint32_t cnt = flag[0] != 0u ? kSphListMaxDev + 1u : 0u, w0 = 0, w1 = 0;
    for (uint32_t b0 = 0; b0 < n; b0 += 256) {
        const uint32_t i = b0 + tid;
        int4 r = spl_empty();
        if (i < n) r = rects[i];
        const bool keep = r.x <= tc1 && r.y >= tc0 && r.z <= tr1 && r.w >= tr0;
        const uint64_t m = __ballot(keep);
        if (lane == 0) wc[wave] = (uint32_t)__popcll(m);
        __syncthreads();
        uint32_t off = 0, total = 0;
        for (uint32_t w = 0; w < 4; ++w) {
            off += w < wave ? wc[w] : 0u;
            total += wc[w];
        }
        if (keep) {
            const uint32_t pos = off + __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32),
                                                                 __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
            rl[pos] = r;
            ri[pos] = i;
        }
        __syncthreads();
        for (uint32_t j = 0; j < total && cnt <= kSphListMaxDev; ++j) {
            const int4 q = rl[j];
            if (col >= q.x && col <= q.y && rb >= q.z && rb <= q.w) {
                const uint32_t idx = ri[j];
                if (cnt == 0) w0 = idx;
                else if (cnt == 1) w0 |= idx << 16;
                else if (cnt == 2) w1 = idx;
                ++cnt;
            }
        }
        if (__syncthreads_and(!on || cnt > kSphListMaxDev)) break;
    }
    if (!on) return;
    const uint32_t c = cnt > kSphListMaxDev ? kSphListWalk : cnt;
    rec[(size_t)row * W + (uint32_t)col] = make_uint2(w0, (w1 & 0xFFFFu) | (c << 16));
}

hipError_t launch_sphere_lists(const float4 *prims, uint32_t n, const double *Mi, const double *o,
                               double e_abs, double wden, double hden, uint32_t width, uint32_t height,
                               int4 *rects, uint32_t *flag, uint2 *rec, hipStream_t stream) {
    SplConst k;
    for (int i = 0; i < 9; ++i) k.Mi[i] = Mi[i];
    for (int i = 0; i < 3; ++i) k.o[i] = o[i];
    k.e_abs = e_abs;
    k.wden = wden;
    k.hden = hden;
    hipError_t e = hipMemsetAsync(flag, 0, 4, stream);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(spl_rect_kernel, dim3((n + 255) / 256), dim3(256), 0, stream, prims, n, k, width, height,
                       rects, flag);
    hipLaunchKernelGGL(spl_fill_kernel, dim3((width + 15) / 16, (height + 15) / 16), dim3(256), 0, stream, rects, n,
                       flag, width, height, rec);
    return hipGetLastError();
}

// Multi-device frames (runtime.cpp render_frame_multi): rank g's tile holds
// the image rows of its row blocks (tile row k = image row tile_row(k)); the
// root's gather buffer holds nranks tiles of max_rows rows each.  One thread
// per RGBA8 word of the frame reads its word from its rank's tile: the frame
// is written once, coalesced, and the gathered tiles are read once.
__global__ __launch_bounds__(256) void assemble_kernel(const uint32_t *__restrict__ gathered,
                                                       uint32_t *__restrict__ out, uint32_t width,
                                                       uint32_t height, uint32_t row_block,
                                                       uint32_t nranks, uint32_t max_rows) {
    const uint64_t n = (uint64_t)width * height;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
         i += (uint64_t)gridDim.x * blockDim.x) {
        const uint32_t row = (uint32_t)(i / width), col = (uint32_t)(i - (uint64_t)row * width);
        const uint32_t b = row / row_block;
        const uint32_t g = b % nranks;
        const uint32_t k = (b / nranks) * row_block + row % row_block;
        out[i] = gathered[((uint64_t)g * max_rows + k) * width + col];
    }
}

hipError_t launch_assemble(const uint32_t *gathered, uint32_t *out, uint32_t width, uint32_t height,
                           uint32_t row_block, uint32_t nranks, uint32_t max_rows,
                           hipStream_t stream) {
    const uint64_t n = (uint64_t)width * height;
    if (!n) return hipSuccess;
    const uint64_t want = (n + 255) / 256, blocks = want < 256 * 64 ? want : 256 * 64;
    hipLaunchKernelGGL(assemble_kernel, dim3((uint32_t)blocks), dim3(256), 0, stream, gathered, out,
                       width, height, row_block ? row_block : 1, nranks ? nranks : 1, max_rows);
    return hipGetLastError();
}

}  // namespace rtamd
