// render.h -- kernel launch interface of the HIP render path (internal).
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>

#include "fastdiv.h"

namespace rtamd {

enum : uint32_t { kRngCounter = 1, kRngReplay = 2 };
// SERIAL-mode passes (runtime.cpp render_frame_serial), kernel-internal modes:
// jobs are (sample, variant) pairs and store the sample's diffuse/metal scatter
// count b (the reference draws 2 + 3b numbers per sample) instead of a colour.
//   kRngSerialCount: variant k = candidate; start state win[2 jl + 3 (lo[jl] + k)]
//   kRngSerialEstimate: variant r = repetition; start state counter_seed(seed, j * V + r)
//   kRngSerialCheck: one variant; start state win[j] (the found start states),
//     stores 1 when the sample's end state is not win[j + 1] (p.seed: the
//     stream state after the frame's last sample), else 0
//   kRngSerialCoalesce: not a trace_kernel pass -- render_frame launches the
//     coalescing block search (launch_serial_coalesce) with the frame's scene
//   kRngSerialPixel: the pixel table pass: a sample's scatter
//     count depends only on its pixel and its start position in the stream, so
//     the iteration's count table is gathered (launch_serial_pixtab_gather)
//     from one trace per (pixel, stream position) its samples' windows cover:
//     variant e of local pixel q starts at win[plo(q) + e] (ctrl[7] = the
//     iteration's positions per pixel, set by serial_window_kernel)
enum : uint32_t { kRngSerialCount = 3, kRngSerialEstimate = 4, kRngSerialCheck = 5, kRngSerialCoalesce = 6,
                  kRngSerialPixel = 7 };
enum : uint32_t { kMatDiffuse = 0, kMatMetal = 1, kMatDielectric = 2, kMatEmission = 3 };
constexpr uint32_t kPrimaryTriStripW = 8;  // bvh.h kTriStripW
#ifndef RT_TRACE_RING
#define RT_TRACE_RING 4
#endif
constexpr uint32_t kTraceRing = RT_TRACE_RING;  // chunk slots per wave (fused resolve)
// u64 counters per wave record (TraceParams::stats); the -DRT_STAMPS
// diagnostic build adds 8 fine segment stamps at slots 16..23
#ifdef RT_STAMPS
constexpr uint32_t kStatSlots = 24;
#else
constexpr uint32_t kStatSlots = 16;
#endif
constexpr uint32_t kStampSegs = 8;

// SERIAL prediction, per pixel (built on the device from the estimate pass,
// render.hip launch_serial_tables): P[q] = sum over pixels p < q of spp mu[p]
// (npix + 1 doubles), mu[p] the pixel's mean scatter count per sample.  The
// predicted scatter count of frame samples [0, j) is
// M(j) = P[p] + (j - p spp) mu[p], p = j / spp (P[npix] for j = npix spp).
struct SerialPred {
    const double *P;
    const double *mu;
    uint32_t spp, npix;
};
RT_HOST_DEVICE inline double serial_M(const SerialPred &m, uint32_t j) {
    const uint32_t p = j / m.spp;
    return p < m.npix ? m.P[p] + (double)(j - p * m.spp) * m.mu[p] : m.P[m.npix];
}

// Kernel argument block (lives in the kernarg segment -> SGPRs).
// job-queue partitions of one launch at most (the counters are kMaxJobParts
// u32 slots, 128 B apart, per set)
constexpr uint32_t kMaxJobParts = 1024;

struct TraceParams {
    const float4 *sph_hot;    // nsph_padded x (cx, cy, cz, r*r); pad = NaN (never hit)
    const float4 *sph_cold;   // nsph_padded x (r, material id bits, 0, 0)
    const float4 *tri_hot;    // ntri x (n.x, n.y, n.z, n.v0), n = cross(v1-v0, v2-v0)
    const float4 *tri_geo;    // ntri x 4: (v0, mat) (v1, 0) (v2, 0) (unit normal, 0)
    const float *mats;        // 8 floats per material: kind bits, r, g, b, param
    float *samples;           // slab-local sample colours: R, G, B planes of njobs floats,
                              // pixel-major (slot = job = local pixel * spp + s)
    // fused resolve (ring != nullptr, else the samples go to the slab above and
    // resolve_kernel sums them): each wave owns kTraceRing slots of 2^ring_shift
    // samples per plane (R, G, B), one chunk per slot; when a chunk's last
    // sample is done the wave sums its pixels in order and stores RGBA8 to out
    float *ring;
    uint32_t ring_shift;
    uint32_t *out;            // tile RGBA8 words (tile row-major)
    float inv_spp;            // 1.0 / spp as f32 (common.rs:345)
    uint32_t alpha_u8;        // the alpha byte: every pixel's is the same (resolve_kernel)
    uint32_t *job_counter;    // nparts counters, 32 u32 apart; zeroed before every launch
    uint32_t *job_counter_next;  // frames: the other set of kMaxParts counters, which this
                                 // launch zeroes for the next one (no fill launch per frame)
    unsigned long long *stats;// nullptr, or kStatSlots per wave (wave = block * waves per
                              // block + wave in block): rays, tri in t-range, BVH sphere
                              // tests, BVH node tests, 4 stamp counters, triangle-BVH node
                              // tests, triangle tests
    const uint32_t *replay;   // REPLAY start states (global job index)
    float cam[12];            // origin, lower_left, horizontal, vertical
    float wden, hden;         // (width-1) as f32, (height-1) as f32
    float wrcp, hrcp;         // RN(1/wden), RN(1/hden) (exactdiv.h) ...
    uint32_t xdiv_uv;         // ... valid when nonzero (both in the exact-division range)
    uint32_t nsph, nsph_padded, ntri;
    uint32_t width, height, spp;
    int32_t depth;            // max_ray_bounces (may be <= 0: zero colour)
    uint32_t mode, seed;
    uint32_t row_block, rank, nranks;
    uint32_t slab_row0;       // first tile row of this launch
    uint32_t njobs;           // samples in this launch
    uint32_t npix;            // pixels in this launch
    uint32_t chunk;           // jobs fetched per atomic by one wave
    uint32_t nparts;          // job-queue partitions (kernel header comment)
    // exact-pruning BVH (bvh.h); nnodes == 0 selects the brute-force kernel
    const float4 *bvh_nodes;  // 2 per node
    const uint32_t *bvh_miss; // 8 per node (one DFS successor per ray octant)
    const uint16_t *bvh_miss16;  // same as u16 (0xFFFF = end), for the LDS copy
    const float4 *bvh_prims;  // (cx, cy, cz, r*r) in BVH order
    const uint32_t *bvh_prim_id;
    const float4 *big_hot;    // spheres kept out of the tree (tested first)
    const uint32_t *big_id;
    uint32_t nnodes, nbig, nprims;
    uint32_t use_lds;         // stage the tree in LDS (trace_lds_bytes per workgroup)
    uint32_t ablate;          // timing-only diagnostics (RT_AMD_ABLATE): 1 = skip the tree walk
    const float4 *sph_shade;  // 2 per sphere: (centre, r) (colour, fuzz|ir)
    const uint32_t *sph_kind; // material kind per sphere
    FastDiv div_spp, div_width, div_rowblock;  // job -> (pixel, sample) mapping
    uint32_t refill_min;      // refill dead lanes once at least this many are idle
    uint32_t walk_min;        // sphere-only: start a walk iteration once this many lanes wait
                              // for one (0: every iteration walks)
    uint32_t tri_walk_min;    // triangle scenes: the same for the triangle walk
    uint32_t steps;           // BVH nodes a lane walks per loop iteration (>= 1) ...
    uint32_t step;            // ... when nonzero (else walks run to the end)
    float bvh_c[3], bvh_r, bvh_rmax, bvh_mag, bvh_inv_rmin;
    // phantom-aware triangle BVH (bvh.h TriangleBVH); tnodes == 0: brute-force Mesh loop
    const uint4 *tbvh_nodes;  // 2 per node: quantised box, normal box, a, link (bvh.h qnodes)
    const float4 *tbvh_tris;  // 4 per triangle in tree order: (n, n.v0) (v0, id) (v1) (v2)
    const uint32_t *tbvh_loose;  // triangles tested by brute force, ascending
    uint32_t tnodes, ttris, tloose;
    float tbvh_c[3], tbvh_r, tbvh_mag;
    float tbvh_oc[3];         // origin the boxes were built for (widening uses o - oc)
    float tq_base[3], tq_step[3], tq_nbase, tq_nstep;  // static-tree grids
    // the static tree's 4-wide image (bvh.h TriangleBVH::wnodes), walked with a
    // per-lane stack of tw_depth u16 entries in LDS (trace_kernel<..., kMesh = 3>);
    // nullptr: the binary walk (kMesh = 2)
    const uint4 *tw_nodes;    // 8 per wide node (128 B)
    uint32_t tw_depth;        // stack entries per lane (3 * TriangleBVH::wdepth, >= 1)
    uint32_t wsteps;          // wide-node fetches per lane per loop iteration (sliced walks)
    float cq_base[3], cq_step[3];                      // camera-tree grid
    // the same triangles' phantoms for the camera origin (bvh.h CameraTriangleBVH),
    // used at bounce 0; cam_nnodes == 0: bounce 0 uses the tree above
    const uint4 *cam_nodes;   // 2 per node: quantised box, a, link
    const float4 *cam_tris;   // 4 per triangle, as tbvh_tris
    uint32_t cam_nnodes;
    // primary-ray triangle lists (bvh.h PrimaryTriLists, camera-tree record
    // indices); ptl_off == nullptr: bounce-0 lanes walk the camera tree
    const uint32_t *ptl_off;  // strips + 1
    const uint32_t *ptl_items;
    uint32_t ptl_spr;         // strips per image row
    uint32_t ptl_always, ptl_end;  // items[ptl_always, ptl_end): tested by every primary ray
    // primary-ray sphere candidates (bvh.h PrimarySphereLists, sphere-only
    // scenes): per image pixel (i0 | i1 << 16, i2 | count << 16); nullptr: walk
    const uint2 *spl;
    // SERIAL-mode passes (mode kRngSerialCount / kRngSerialEstimate): p.spp is
    // the variants per sample V and p.npix the samples of the launch; launch
    // sample jl is frame sample cbase + jl (reference order, common.rs:327-336),
    // clamped to nserial - 1
    const uint32_t *win;      // kRngSerialCount: stream states from sample cbase's start on
    SerialPred sM;            // kRngSerialCount: the predicted scatter counts (per pixel)
    const uint32_t *slo;      // kRngSerialCount (optional): serial_lo of each launch sample,
                              // tabulated by serial_window_kernel
    const uint32_t *ctrl;     // serial control block (kRngSerialCount: cbase = ctrl[4];
                              // ctrl[0] != 0, the frame is resolved: exit at once)
    uint32_t cbase;           // first frame sample of the launch
    uint32_t nserial;         // samples in the frame
    uint32_t sspp;            // the frame's spp ...
    FastDiv div_sspp;         // ... and its divider
    uint32_t max_draws;       // 2 + 3 * max(depth, 0): bound of the draw count search
    uint32_t sL, sK;          // kRngSerialPixel: the iteration length and the launch's K
    // frames of one rank whose global job indices (row * W + col) * spp + s
    // fit 32 bits (gj32 != 0): the global job of launch job j in local row q is
    // j + gj_c0 - q * gj_2p (mod 2^32), gj_c0 = (H - 1 - slab_row0) W spp,
    // gj_2p = 2 W spp -- the refill's job -> (pixel, seed) without the
    // row-block map and the 64-bit products
    uint32_t gj32, gj_c0, gj_2p;
    // (round-6 fields last: the offsets of the fields above stay those the
    // frame kernels' kernarg loads were tuned with)
    // per-origin-cell trees (bvh.h TriangleCells; tc_ncells == 0: the static
    // tree only): tree c's wide nodes from tw_nodes + 8 c tw_stride; tree
    // tc_ncells is the static tree.  tw_tris: the records every wide walk's
    // leaves index (all trees share one array; tbvh_tris without cells)
    const float4 *tw_tris;
    uint32_t tw_stride, tc_ncells;
    uint32_t tc_n[3];
    float tc_lo[3], tc_size, tc_inv_size;
    const uint4 *spix;        // kRngSerialPixel (optional): per local pixel its positions
                              // {plo, phi} and the positions [z, w] (relative to plo; empty
                              // when z > w) copied from the previous iteration's table
                              // (serial_window_kernel, serial_reuse_kernel): not traced
};

// Candidate k of chunk sample jl (frame sample a + jl) means B = serial_lo + k
// scatters since sample a: the predicted offset M(a + jl) - M(a) minus K / 2,
// clamped to the possible [0, depth * jl].  Count kernel and walk kernels use
// this one definition.
RT_HOST_DEVICE inline uint32_t serial_lo(const SerialPred &M, uint32_t a, uint32_t jl, uint32_t K,
                                         uint32_t depth, uint32_t nserial) {
    const uint32_t j = a + jl < nserial ? a + jl : nserial;
    double c = __builtin_floor(serial_M(M, j) - serial_M(M, a)) - (double)(K / 2u);
    const double hi = (double)depth * (double)jl;
    c = c < 0.0 ? 0.0 : c;
    c = c > hi ? hi : c;
    return (uint32_t)c;
}

hipError_t launch_trace(const TraceParams &p, uint32_t blocks, hipStream_t stream);
// Primary sphere lists built on the device (bvh.h build_primary_sphere_lists,
// the same double arithmetic per sphere, then one thread per pixel collecting
// the spheres whose projected box covers it, in tree order): rec gets 2 u32
// per pixel; rects (n int4) and flag (1 u32) are scratch.  Mi: 9 doubles,
// o: 3; every pixel walks when a ball straddles the camera plane.
hipError_t launch_sphere_lists(const float4 *prims, uint32_t n, const double *Mi, const double *o,
                               double e_abs, double wden, double hden, uint32_t width, uint32_t height,
                               int4 *rects, uint32_t *flag, uint2 *rec, hipStream_t stream);
// SERIAL mode, the estimate reduction (render_frame_serial step 1), on the
// device.  tab holds, for a frame of npix pixels (serial_tab_doubles(npix)):
//   P   [0, npix]             prefix sums of spp mu (SerialPred::P)
//   mu  [npix + 1, 2 npix]    per-pixel mean scatter count (SerialPred::mu)
//   V   [2 npix + 1, 4 npix + 1]  prefix sums of spp var (npix + 1), then var (npix)
//   ss  [4 npix + 2, 5 npix + 1]  per-pixel sum of squared deviations of b
//   sum [5 npix + 2, + 8)     {sum of ss, dmax (double bits), V(n0), lost-count flag}
// Moments: pixels [pix0, pix0 + n) of one estimate launch, whose scatter
// counts are est[(p - pix0) spp R + s R + r] (R traces per sample); var is
// scaled by `scale` (the means' estimation error).  Tables: the prefix sums
// (a fixed-shape scan: deterministic), dmax = the largest M(a + L + L/4) -
// M(a) over a = 0, L/4, 2 L/4, ... (the candidate window's reach) and V(n0).
size_t serial_tab_doubles(uint32_t npix);
// Counts the nonzero flags of a kRngSerialCheck pass (plane 0 of the slab)
// into *count (atomics; *count is not reset).
hipError_t launch_serial_check_count(const float *flags, uint32_t n, unsigned long long *count,
                                     hipStream_t stream);
hipError_t launch_serial_moments(const float *est, uint32_t pix0, uint32_t n, uint32_t spp, uint32_t R,
                                 double scale, double *tab, uint32_t npix, hipStream_t stream);
hipError_t launch_serial_tables(double *tab, double *scratch, uint32_t npix, uint32_t spp, uint32_t L,
                                uint32_t n0, hipStream_t stream);
// doubles of launch_serial_tables' scratch
size_t serial_scan_scratch(uint32_t npix);
// SERIAL mode.  ctrl (u32[8]): {resolved, state at sample a, sum of b (low
// bits), iterations, a = first unresolved sample, candidates per sample of the
// next iteration (0: the launch's K), iterations that stopped short, 0}.
// jump: kSerialJumpWords u32, column c of M^(2^i), then of M^(kSerialWinPerThread
// j) and M^(4096 j) (xorshift32 is linear over GF(2)).  Window: win[i] = xorshift32^i(ctrl[1]) for i < n.
// lo (optional): L u32, the iteration's window bases serial_lo(a, jl) with the
// iteration's K (ctrl[5] when set, else K), for the count pass
// (TraceParams::slo) and the walks.
// pix_spp (optional, nonzero: the pixel table pass follows): also sets ctrl[7]
// to the iteration's stream positions per pixel (serial_pixtab_span; ctrl[7]
// must be 0 on entry: the initial block and the finish kernel leave it so),
// clamped to pix_emax (the pixel table's row stride).
// counters (optional): ncounters job-queue counters (32 u32 apart) the next
// trace pass uses, zeroed here instead of by a fill launch.
// the jump table: M^(2^i) (i < 64), M^(kSerialWinPerThread j) (j < 4096 /
// kSerialWinPerThread) and M^(4096 j) (j < 256), 32 u32 each
constexpr uint32_t kSerialWinPerThread = 4;  // window states per thread (serial_window_kernel)
constexpr uint32_t kSerialJumpT1 = 4096 / kSerialWinPerThread;
constexpr uint32_t kSerialJumpWords = 32 * (64 + kSerialJumpT1 + 256);
hipError_t launch_serial_window(uint32_t *ctrl, const uint32_t *jump, uint32_t *win, uint32_t n,
                                SerialPred M, uint32_t *lo, uint32_t L, uint32_t K, uint32_t depth,
                                uint32_t nserial, uint32_t pix_spp, uint32_t pix_emax, uint32_t *counters,
                                uint32_t ncounters, uint4 *spix, uint32_t pix_chunk, const uint4 *spix_prev,
                                hipStream_t stream);
// The pixel table's entries the previous iteration already traced (window
// kernel: spix[q].zw, relative to the pixel's plo) copied from ptab_prev
// (row stride ctrl[11], its pixels from frame pixel ctrl[10] / spp, stream
// offset ctrl[8] between the two iterations' windows) into ptab (ctrl[7]).
hipError_t launch_serial_reuse(const uint32_t *ctrl, const uint4 *spix, const uint4 *spix_prev, float *ptab,
                               const float *ptab_prev, uint32_t npq_max, uint32_t spp, uint32_t L,
                               uint32_t nserial, hipStream_t stream);
// The pixel table pass's result (ptab: b of local pixel q at position plo(q) + e
// = ptab[q * ctrl[7] + e]) gathered into the count table of the iteration
// (table[jl * K + k], the layout the walks read; -1 outside the traced span)
hipError_t launch_serial_pixtab_gather(const uint32_t *ctrl, const float *ptab, const uint32_t *lo, float *table,
                                       uint32_t L, uint32_t K, uint32_t spp, uint32_t nserial, hipStream_t stream);
// the largest positions-per-pixel span an iteration can need (ptab sizing):
// 2 (spp - 1) + 3 (depth (spp - 1) + K) + 1
// (64-bit: the host checks it against the table's bounds before narrowing)
inline uint64_t serial_pixtab_emax64(uint64_t spp, uint64_t K, uint64_t depth) {
    return 2u * (spp - 1u) + 3u * (depth * (spp - 1u) + K) + 1u;
}
// Coalescing block search (render.hip serial_coalesce_kernel): one workgroup
// per block of R samples of the iteration writes bend and path (layouts of
// launch_serial_walk's block walks) by tracing each block's distinct live
// offsets once per sample, from win and lo (p.win, p.slo, p.ctrl set as for a
// count pass; K + depth + 1 < 65535).  tree_lds: stage the sphere tree in LDS
// (serial_coalesce_lds bytes per workgroup, tree included).
// dbg (optional, 4 u64, diagnostics): += live offsets traced, trace passes per
// thread, blocks, the count pass's traces (K x samples) of every block
hipError_t launch_serial_coalesce(const TraceParams &p, uint32_t *path, uint32_t *bend, uint32_t L, uint32_t Kmax,
                                  uint32_t R, bool tree_lds, unsigned long long *dbg, hipStream_t stream);
size_t serial_coalesce_lds(const TraceParams &p, uint32_t K, bool tree_lds);
// the search's own LDS bytes (without the tree) for K candidates at this depth
size_t serial_coalesce_search_lds(uint32_t K, uint32_t depth);
// Walk: from sample a = ctrl[4], follows the true path through the candidate
// table (b of chunk sample jl at candidate k = table[jl * K + k], plane 0 of
// the slab) as far as it stays inside the candidate windows (at least one
// sample), writes those samples' start states to states[a + jl] and advances
// ctrl (a, the state at a, resolved).  bend: scratch of
// ceil(L / R) * K u32, R = the block length (serial_walk_block(L) for the
// count pass; table == nullptr: bend and path were written by the coalescing
// search, the block walks are skipped).
uint32_t serial_walk_block(uint32_t L);
constexpr uint32_t kMaxWalkBlocks = 4096;  // blocks per iteration (the finish kernel's LDS)
// fin (serial_walk_finish_kernel's result): 4 header words, a column per block
constexpr uint32_t kWalkFinWords = 4 + kMaxWalkBlocks;
// pixel table walks from LDS (lds_rows != 0): samples per block at most, and
// the u8 rows' LDS budget per workgroup
constexpr uint32_t kMaxWalkR = 256;
constexpr uint32_t kWalkLdsRowBytes = 48 * 1024;
constexpr uint32_t kWalkLdsMaxPix = 72;  // pixels one block's samples touch: (R - 1) / spp + 2
// path, fin (optional, both or neither): scratch of ceil(L / R) R K u32 for the
// block walks' recorded paths and 4 + kMaxWalkBlocks u32 for the chain's result; with
// them the full blocks' states are gathered by a parallel kernel, not re-walked.
// V (optional): the per-sample scatter-count variances as npix + 1 per-pixel
// prefix sums of spp var followed by npix per-pixel variances; with it
// the walk sets the next iteration's candidates per sample in ctrl[5] (<= K):
// 2 z (sqrt(V over Lw samples) + sfloor sqrt(Lw)) + 2 depth + 2; the count
// pass and the walks use ctrl[5] when it is set.
// ptab (optional, with path and fin): the pixel table pass's table (ptab[q *
// ctrl[7] + e], render.h kRngSerialPixel) read by the block walks directly;
// table is then unused.  lds_rows (with ptab, nonzero): the block walks stage
// each block's pixel rows in LDS as u8 (depth < 255; that many bytes per
// workgroup, <= kWalkLdsRowBytes).
hipError_t launch_serial_walk(uint32_t *ctrl, const float *table, SerialPred M, const double *V,
                              uint32_t npix, uint32_t spp, float z, float sfloor, const uint32_t *win,
                              uint32_t *states, uint32_t *bend, uint32_t *path, uint32_t *fin,
                              const uint32_t *lo, uint32_t *sbend, uint32_t *sB, uint32_t L, uint32_t Lw,
                              uint32_t K, uint32_t R, uint32_t depth, uint32_t nserial, const float *ptab,
                              uint32_t lds_rows, hipStream_t stream);
// (lo: required; sbend, sB: scratch of serial_super_words(L, K, R) and ceil(L / R) K
// u32 for the superblock chain)
uint32_t serial_super_words(uint32_t L, uint32_t K, uint32_t R);
// inv_spp = 1.0 / (spp as f32) computed from the signed spp (common.rs:345).
hipError_t launch_resolve_ex(const float *samples, uint32_t *out, uint32_t npix, uint32_t spp,
                             float inv_spp, uint32_t width, uint32_t slab_row0,
                             hipStream_t stream);
// Reassembles a gathered multi-device frame: gathered holds nranks tiles of
// max_rows rows (row-cyclic blocks of row_block rows), out the width x height
// frame (top row first).
hipError_t launch_assemble(const uint32_t *gathered, uint32_t *out, uint32_t width, uint32_t height,
                           uint32_t row_block, uint32_t nranks, uint32_t max_rows,
                           hipStream_t stream);
// variant: 0 brute force, 1 BVH from global memory, 2 BVH staged in LDS;
// step: the sliced-walk kernel (TraceParams::step); mesh: trace_mesh_kind
// workgroups per CU of one trace_kernel instance (kind: 0 the lean frame
// kernel, 1 the counting frame kernel, 2 the SERIAL passes)
hipError_t trace_occupancy(int *blocks_per_cu, int variant, size_t lds_bytes, bool step, int mesh,
                           int kind);
// The kernel family of a scene: 0 no triangles, 1 triangles searched by brute
// force (no triangle tree), 2 triangle trees (TraceParams::tnodes != 0)
inline int trace_mesh_kind(bool triangles, bool tree) { return !triangles ? 0 : tree ? 2 : 1; }
// kMesh 3: kind 2 walked through the 4-wide image (TraceParams::tw_nodes); the
// SERIAL passes keep the binary walk
size_t trace_lds_bytes(const TraceParams &p);
// the sphere tree's LDS copy (render.hip stage_tree)
__host__ __device__ inline size_t trace_tree_lds(uint32_t nnodes, uint32_t nprims, uint32_t nsph_padded) {
    return (size_t)nnodes * 64 + (size_t)nprims * 20 + (size_t)nsph_padded * 36;
}
// the LDS copy addresses its 64-B node records with u16 byte addresses (0xFFFF: end)
constexpr uint32_t kLdsTreeMaxNodes = 1023;
// threads per trace workgroup: LDS-tree kernels (per kernel family, trace_mesh_kind
// or 3 for the wide walk) vs global
uint32_t trace_block_threads(bool lds, int mesh, int kind);
// dynamic LDS of one trace workgroup: the sphere tree (lds) and, for the wide
// triangle walk, every lane's stack (u16 entries)
size_t trace_dyn_lds(const TraceParams &p, bool lds, bool wide, uint32_t threads);

}  // namespace rtamd
