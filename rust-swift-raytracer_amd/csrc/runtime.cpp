// runtime.cpp -- frame driver of the HIP render path (host side).
//
// Owns each world's device-resident scene (uploaded once per device, reused
// by every frame and every camera move), the per-wave sample rings (or the
// per-sample slab) and the launch sequence: for every launch of tile rows,
// zero the job counters and launch the persistent trace kernel, which
// resolves pixels itself; with RT_FLAG_KEEP_SAMPLES the samples go to the
// slab and the ordered resolve kernel follows.  The reference's equivalent is
// ray_trace's triple loop (common.rs:320-361).
#include "runtime.h"

#include <algorithm>
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#include <rccl/rccl.h>

#include "../../include/raytracer_amd.h"
#include "render.h"

namespace rtamd {

namespace {
thread_local std::string g_error;

uint64_t env_u64(const char *name, uint64_t dflt) {
    const char *v = std::getenv(name);
    if (!v || !*v) return dflt;
    return std::strtoull(v, nullptr, 10);
}
}  // namespace

void set_error(const std::string &msg) { g_error = msg; }
const std::string &last_error() { return g_error; }

#define HIP_TRY(expr)                                                                 \
    do {                                                                              \
        hipError_t e_ = (expr);                                                       \
        if (e_ != hipSuccess) {                                                       \
            set_error(std::string(#expr) + " failed: " + hipGetErrorString(e_));      \
            return -2;                                                                \
        }                                                                             \
    } while (0)

DeviceState::~DeviceState() {
    if (device < 0) return;
    if (hipSetDevice(device) != hipSuccess) return;
    void *bufs[] = {sph_hot, sph_cold, tri_hot, tri_geo, mats, samples, ring, out, replay, counter, stats,
                    bvh_nodes, bvh_prims, big_hot, bvh_miss, bvh_prim_id, big_id, bvh_miss16,
                    sph_shade, sph_kind, tbvh_nodes, tbvh_tris, tbvh_loose, tw_nodes, tw_tris,
                    cam_nodes, cam_tris, ptl_off, ptl_items, spl, tile, gath,
                    sstates, stab, sscan, swin, sjump, sctrl, sbend, spath, sfin,
                    gspl, gspl_rects, gspl_flag, scheck, slo, ssbend, ssb, sptab, sspix, sptab2};
    for (void *b : bufs)
        if (b) (void)hipFree(b);
    for (hipEvent_t e : ev)
        if (e) (void)hipEventDestroy(e);
    for (hipEvent_t e : tev)
        if (e) (void)hipEventDestroy(e);
    if (hrec) (void)hipHostFree(hrec);
    for (hipEvent_t e : sev)
        if (e) (void)hipEventDestroy(e);
    if (done) (void)hipEventDestroy(done);
    if (stream) (void)hipStreamDestroy(stream);
}

size_t tile_rows(size_t height, uint32_t row_block, uint32_t rank, uint32_t nranks) {
    if (nranks <= 1) return height;
    const size_t B = row_block ? row_block : 1;
    const size_t blocks = (height + B - 1) / B;
    size_t rows = 0;
    for (size_t b = rank; b < blocks; b += nranks) rows += std::min(B, height - b * B);
    return rows;
}

size_t tile_row(size_t k, uint32_t row_block, uint32_t rank, uint32_t nranks) {
    if (nranks <= 1) return k;
    const size_t B = row_block ? row_block : 1;
    return ((k / B) * nranks + rank) * B + k % B;
}

static_assert(kPrimaryTriStripW == kTriStripW, "render.h and bvh.h strip widths");
static constexpr uint64_t kMaxParts = kMaxJobParts;  // job-queue partitions (render.h)
static constexpr uint32_t kPixtabParts = 64;  // the pixel table pass's (zeroed by the window kernel)

static int device_for(WorldState &w, int want, DeviceState *&out) {
    int count = 0;
    if (hipGetDeviceCount(&count) != hipSuccess || count <= 0) {
        set_error("no HIP device available: the MI355X render path requires a GPU");
        return -3;
    }
    int dev = want;
    if (dev < 0) HIP_TRY(hipGetDevice(&dev));
    if (dev >= count) {
        set_error("device ordinal out of range");
        return -1;
    }
    HIP_TRY(hipSetDevice(dev));
    auto &slot = w.devices[dev];
    if (!slot) {
        auto d = std::make_unique<DeviceState>();
        d->device = dev;
        HIP_TRY(hipStreamCreateWithFlags(&d->stream, hipStreamNonBlocking));
        for (auto &e : d->ev) HIP_TRY(hipEventCreate(&e));
        for (auto &e : d->sev) HIP_TRY(hipEventCreate(&e));
        HIP_TRY(hipEventCreateWithFlags(&d->done, hipEventDisableTiming));
        hipDeviceProp_t prop;
        HIP_TRY(hipGetDeviceProperties(&prop, dev));
        d->num_cus = prop.multiProcessorCount;
        // the scene's kernel family (render.h trace_mesh_kind; frames rendered with
        // RT_ACCEL_BRUTE run the brute-force triangle kernels on these figures)
        // Triangle trees are walked through their 4-wide image (kMesh 3) when it
        // exists and every lane's stack fits in LDS beside a workgroup's tree
        // (RT_AMD_TRI_WIDE=0: the binary walk)
        const TriangleBVH &tw = w.tbvh;
        const uint32_t tw_depth = std::max<uint32_t>(1u, 3u * std::max(tw.wdepth, w.tcells.wdepth));
        bool wide = !tw.wnodes.empty() && env_u64("RT_AMD_TRI_WIDE", 1) != 0 &&
                    (size_t)tw_depth * trace_block_threads(true, 3, 0) * 2u <= 64u * 1024u;
        int tri = wide ? 3 : trace_mesh_kind(w.packed.ntri > 0, !w.tbvh.nodes.empty());
        // the stack's LDS (kinds 0 and 1: SERIAL passes keep the binary walk)
        auto stack_lds = [&](int c, uint32_t threads) -> size_t {
            return tri == 3 && c != 2 ? (size_t)tw_depth * threads * 2u : 0u;
        };
        // workgroups per CU of the kernels without the LDS sphere tree
        auto occupancy_global = [&]() -> hipError_t {
            for (int c = 0; c < 3; ++c)
                for (int st = 0; st < 2; ++st) {
                    hipError_t e = trace_occupancy(&d->blocks_per_cu[c][st], 0, stack_lds(c, 256), st, tri, c);
                    if (e == hipSuccess)
                        e = trace_occupancy(&d->blocks_per_cu_bvh[c][st], 1, stack_lds(c, 256), st, tri, c);
                    if (e != hipSuccess) return e;
                }
            return hipSuccess;
        };
        HIP_TRY(occupancy_global());
        // scene upload (once per device)
        const PackedScene &p = w.packed;
        auto up = [&](void **dst, const std::vector<float> &src) -> hipError_t {
            hipError_t e = hipMalloc(dst, src.size() * sizeof(float));
            if (e != hipSuccess) return e;
            return hipMemcpy(*dst, src.data(), src.size() * sizeof(float), hipMemcpyHostToDevice);
        };
        HIP_TRY(up((void **)&d->sph_hot, p.sph_hot));
        HIP_TRY(up((void **)&d->sph_cold, p.sph_cold));
        HIP_TRY(up((void **)&d->tri_hot, p.tri_hot));
        HIP_TRY(up((void **)&d->tri_geo, p.tri_geo));
        HIP_TRY(up((void **)&d->mats, p.mats));
        HIP_TRY(up((void **)&d->sph_shade, p.sph_shade));
        HIP_TRY(hipMalloc((void **)&d->sph_kind, p.sph_kind.size() * 4));
        HIP_TRY(hipMemcpy(d->sph_kind, p.sph_kind.data(), p.sph_kind.size() * 4, hipMemcpyHostToDevice));
        d->nsph = p.nsph;
        d->nsph_padded = p.nsph_padded;
        d->ntri = p.ntri;
        const SphereBVH &bv = w.bvh;
        if (!bv.nodes.empty()) {
            auto upu = [&](void **dst, const std::vector<uint32_t> &src) -> hipError_t {
                hipError_t e = hipMalloc(dst, std::max<size_t>(src.size(), 1) * sizeof(uint32_t));
                if (e != hipSuccess || src.empty()) return e;
                return hipMemcpy(*dst, src.data(), src.size() * sizeof(uint32_t), hipMemcpyHostToDevice);
            };
            std::vector<float> big_hot;
            for (uint32_t i : bv.big)
                for (int k = 0; k < 4; ++k) big_hot.push_back(p.sph_hot[(size_t)i * 4 + k]);
            if (big_hot.empty()) big_hot.assign(4, 0.0f);
            HIP_TRY(up((void **)&d->bvh_nodes, bv.nodes));
            HIP_TRY(up((void **)&d->bvh_prims, bv.prims));
            HIP_TRY(up((void **)&d->big_hot, big_hot));
            HIP_TRY(upu((void **)&d->bvh_miss, bv.miss));
            HIP_TRY(upu((void **)&d->bvh_prim_id, bv.prim_id));
            HIP_TRY(upu((void **)&d->big_id, bv.big));
            d->nnodes = (uint32_t)(bv.nodes.size() / 8);
            d->nbig = (uint32_t)bv.big.size();
            d->nprims = (uint32_t)bv.prim_id.size();
            // LDS copy of the tree: 64 B per node + 20 B per sphere, u16 links
            TraceParams lp{};
            lp.nnodes = d->nnodes; lp.nprims = d->nprims; lp.nsph_padded = (uint32_t)p.nsph_padded;
            const size_t lds = trace_lds_bytes(lp);
            // (the LDS copy addresses 64-B node records with u16 byte offsets)
            if (d->nnodes <= kLdsTreeMaxNodes && lds <= env_u64("RT_AMD_LDS_MAX", 64 * 1024)) {
                std::vector<uint16_t> m16(bv.miss.size());
                for (size_t i = 0; i < m16.size(); ++i)
                    m16[i] = bv.miss[i] == kNodeEnd ? (uint16_t)0xFFFF : (uint16_t)bv.miss[i];
                HIP_TRY(hipMalloc((void **)&d->bvh_miss16, m16.size() * 2));
                HIP_TRY(hipMemcpy(d->bvh_miss16, m16.data(), m16.size() * 2, hipMemcpyHostToDevice));
                // every kernel kind must fit its LDS (the tree, plus the wide
                // walk's stacks for the frame kinds); when the stacks are what
                // does not fit, the frames take the binary triangle walk and
                // every kind keeps the LDS sphere tree
                auto occupancy_lds = [&](bool &fits) -> hipError_t {
                    fits = true;
                    for (int c = 0; c < 3; ++c)
                        for (int st = 0; st < 2; ++st) {
                            const uint32_t lt = trace_block_threads(true, tri == 3 && c == 2 ? 2 : tri, c);
                            const size_t sb = stack_lds(c, lt);
                            const hipError_t e = trace_occupancy(&d->blocks_per_cu_lds[c][st], 2,
                                                                 sb ? ((lds + 15u) & ~(size_t)15u) + sb : lds, st,
                                                                 tri, c);
                            if (e != hipSuccess) return e;
                            fits = fits && d->blocks_per_cu_lds[c][st] > 0;
                        }
                    return hipSuccess;
                };
                bool fits = false;
                HIP_TRY(occupancy_lds(fits));
                if (!fits && wide) {
                    wide = false;
                    tri = trace_mesh_kind(w.packed.ntri > 0, !w.tbvh.nodes.empty());
                    HIP_TRY(occupancy_global());
                    HIP_TRY(occupancy_lds(fits));
                    if (!fits) {
                        // the tree itself does not fit: give up the LDS tree, not
                        // the wide triangle walk (its stacks fit without the tree)
                        wide = true;
                        tri = 3;
                        HIP_TRY(occupancy_global());
                    }
                }
                if (fits) d->lds_bytes = lds;
            }
        }
        const TriangleBVH &tb = w.tbvh;
        if (!tb.nodes.empty()) {
            auto upu = [&](void **dst, const std::vector<uint32_t> &src) -> hipError_t {
                hipError_t e = hipMalloc(dst, std::max<size_t>(src.size(), 1) * sizeof(uint32_t));
                if (e != hipSuccess || src.empty()) return e;
                return hipMemcpy(*dst, src.data(), src.size() * sizeof(uint32_t), hipMemcpyHostToDevice);
            };
            HIP_TRY(upu((void **)&d->tbvh_nodes, tb.qnodes));
            HIP_TRY(up((void **)&d->tbvh_tris, tb.tris));
            HIP_TRY(upu((void **)&d->tbvh_loose, tb.loose));
            d->tnodes = (uint32_t)(tb.qnodes.size() / 8);
            if (wide) {
                if (w.tcells.ncells) {  // the per-cell trees + the static one
                    HIP_TRY(upu((void **)&d->tw_nodes, w.tcells.wnodes));
                    HIP_TRY(up((void **)&d->tw_tris, w.tcells.tris));
                } else {
                    HIP_TRY(upu((void **)&d->tw_nodes, tb.wnodes));
                }
                d->tw_depth = tw_depth;
            }
            d->ttris = (uint32_t)(tb.tris.size() / 16);
            d->tloose = (uint32_t)tb.loose.size();
        }
        const uint64_t bpc = env_u64("RT_AMD_BLOCKS_PER_CU", 0);
        for (int c = 0; c < 3; ++c)
            for (int st = 0; st < 2; ++st) {
                if (bpc)
                    d->blocks_per_cu[c][st] = d->blocks_per_cu_bvh[c][st] = d->blocks_per_cu_lds[c][st] =
                        (int)bpc;
                d->blocks_per_cu[c][st] = std::max(d->blocks_per_cu[c][st], 1);
                d->blocks_per_cu_bvh[c][st] = std::max(d->blocks_per_cu_bvh[c][st], 1);
            }
        HIP_TRY(hipMalloc((void **)&d->counter, 2 * kMaxParts * 128));
        slot = std::move(d);
    }
    out = slot.get();
    return 0;
}

static uint32_t cam_leaf() {
    return (uint32_t)env_u64("RT_AMD_CAM_LEAF", 2);  // triangles per camera-tree leaf
}

// The camera-origin phantom records (and, with tree, the camera tree over
// them) for cam's origin.  Frames with primary strip lists need only the
// records: the lists replace every bounce-0 walk (C5: ~3 ms instead of the
// tree's ~50 ms after a camera move).
void prepare_camera(WorldState &w, const CameraModel &cam, bool tree) {
    if (w.tbvh.nodes.empty() || env_u64("RT_AMD_CAMERA_TREE", 1) == 0) return;
    const float o[3] = {cam.origin.x, cam.origin.y, cam.origin.z};
    if (w.ctree_version && std::memcmp(o, w.ctree.origin, sizeof(o)) == 0 && (w.ctree_full || !tree)) return;
    w.ctree = build_camera_triangle_bvh(w.scene.triangles, w.packed.tri_hot, w.tbvh, o, cam_leaf(), tree);
    w.ctree_full = tree;
    ++w.ctree_version;
}

// Primary sphere lists for a new camera or frame size are built on the device
// on the frame's stream, before its trace kernel (RT_AMD_GPU_LISTS, default 1).
// With RT_AMD_GPU_LISTS=0 they are built on a host thread while frames render
// without them (RT_AMD_SYNC_LISTS=1: built before the frame).  Every frame is
// bit-identical either way; only the work per primary ray differs.
static bool sync_lists() { return env_u64("RT_AMD_SYNC_LISTS", 0) != 0; }
static bool gpu_lists() { return env_u64("RT_AMD_GPU_LISTS", 1) != 0; }

template <typename T>
static bool job_ready(const std::future<T> &f) {
    return f.valid() && f.wait_for(std::chrono::seconds(0)) == std::future_status::ready;
}

static bool same_cam(const CameraModel &a, const CameraModel &b) {
    return std::memcmp(&a, &b, sizeof(a)) == 0;
}

// Camera tree (bounce-0 triangle tree for the camera origin) and the primary
// strip lists for (cam, width, height), rebuilt before the frame when either
// changed.  Unlike the sphere lists these are not deferred to a host thread:
// a C5 frame without them costs ~660 ms instead of ~221 ms, while the
// rebuild takes ~50 + 6 ms (subtrees built on 16 host threads, bvh.cpp).
static void prepare_camera_lists(WorldState &w, const CameraModel &cam, size_t width, size_t height,
                                 bool lists) {
    prepare_camera(w, cam, !lists);
    if (!lists || !w.ctree_version) return;
    if (w.ptl_version && w.ptl_w == width && w.ptl_h == height && w.ptl_ctree == w.ctree_version &&
        same_cam(w.ptl_cam, cam))
        return;
    w.ptl = build_primary_tri_lists(w.ctree, cam, width, height);
    w.ptl_cam = cam;
    w.ptl_w = width;
    w.ptl_h = height;
    w.ptl_ctree = w.ctree_version;
    ++w.ptl_version;
}

// Primary sphere candidates per pixel (< 50 ms at 1080p on one host core).
// Returns true when w.spl is current for (cam, width, height).
static bool prepare_primary_sphere_lists(WorldState &w, const CameraModel &cam, size_t width,
                                         size_t height) {
    if (w.spl_version && w.spl_w == width && w.spl_h == height && same_cam(w.spl_cam, cam))
        return true;
    WorldState::SplJob &j = w.spl_job;
    if (sync_lists()) {
        w.spl = build_primary_sphere_lists(w.bvh, cam, width, height);
    } else {
        if (j.f.valid() && !job_ready(j.f)) return false;  // (one build at a time)
        if (j.f.valid() && same_cam(j.cam, cam) && j.w == width && j.h == height) {
            w.spl = j.f.get();
        } else {
            if (j.f.valid()) (void)j.f.get();  // a finished build for another camera
            j.cam = cam;
            j.w = width;
            j.h = height;
            j.f = std::async(std::launch::async, [&w, cam, width, height]() {
                return build_primary_sphere_lists(w.bvh, cam, width, height);
            });
            return false;
        }
    }
    w.spl_cam = cam;
    w.spl_w = width;
    w.spl_h = height;
    ++w.spl_version;
    return true;
}

template <typename T>
static hipError_t grow(T *&buf, size_t &cap, size_t n) {
    if (n <= cap) return hipSuccess;
    if (buf) (void)hipFree(buf);
    buf = nullptr;
    cap = 0;
    hipError_t e = hipMalloc((void **)&buf, n * sizeof(T));
    if (e == hipSuccess) cap = n;
    return e;
}

// The device build of the primary sphere lists for (cam, width, height),
// enqueued on s when either changed; false = no lists (every primary ray
// walks).  RT_AMD_SPL_CHECK=1 (tests): compare them with the host build.
static int device_sphere_lists(WorldState &w, DeviceState *d, const CameraModel &cam, size_t width,
                               size_t height, hipStream_t s, bool &ok) {
    if (!(d->gspl_built && d->gspl_w == width && d->gspl_h == height && same_cam(d->gspl_cam, cam))) {
        SphereListParams sp;
        d->gspl_ok = sphere_list_params(w.bvh, cam, width, height, sp) && (height + 15) / 16 <= 65535 &&
                     sp.n == d->nprims;
        if (d->gspl_ok) {
            HIP_TRY(grow(d->gspl, d->gspl_cap, width * height));
            HIP_TRY(grow(d->gspl_rects, d->gspl_rects_cap, (size_t)sp.n));
            HIP_TRY(grow(d->gspl_flag, d->gspl_flag_cap, 1));
            HIP_TRY(launch_sphere_lists(d->bvh_prims, sp.n, sp.Mi, sp.o, sp.e_abs, sp.wden, sp.hden, sp.width,
                                        sp.height, d->gspl_rects, d->gspl_flag, d->gspl, s));
            if (env_u64("RT_AMD_SPL_CHECK", 0)) {
                const PrimarySphereLists h = build_primary_sphere_lists(w.bvh, cam, width, height);
                std::vector<uint32_t> g(2 * width * height);
                HIP_TRY(hipMemcpyAsync(g.data(), d->gspl, g.size() * 4, hipMemcpyDeviceToHost, s));
                HIP_TRY(hipStreamSynchronize(s));
                for (size_t px = 0; px < width * height; ++px) {
                    const bool same = h.rec.empty() ? (g[2 * px + 1] >> 16) == kSphListWalk
                                                    : g[2 * px] == h.rec[2 * px] && g[2 * px + 1] == h.rec[2 * px + 1];
                    if (!same) {
                        set_error("RT_AMD_SPL_CHECK: device sphere lists differ from the host build at pixel " +
                                  std::to_string(px));
                        return -2;
                    }
                }
            }
        }
        d->gspl_cam = cam;
        d->gspl_w = width;
        d->gspl_h = height;
        d->gspl_built = true;
    }
    ok = d->gspl_ok;
    return 0;
}

int render_frame(WorldState &w, const CameraModel &cam, size_t width, size_t height,
                 const RtRenderOptions &o, uint32_t *d_out, hipStream_t stream,
                 RtRenderStats *stats, const SerialPass *sp, const uint32_t *d_replay, bool defer_stats) {
    if (stats) std::memset(stats, 0, sizeof(*stats));
    const uint32_t nranks = o.nranks ? o.nranks : 1;
    if (o.rank >= nranks) { set_error("rank >= nranks"); return -1; }
    if (o.rng_mode == RT_RNG_SERIAL && !sp && !d_replay)
        return render_frame_serial(w, cam, width, height, o, d_out, stream, stats);
    if (!sp && o.rng_mode != RT_RNG_COUNTER && o.rng_mode != RT_RNG_REPLAY && !d_replay) {
        set_error("rng_mode must be RT_RNG_COUNTER, RT_RNG_REPLAY or RT_RNG_SERIAL");
        return -1;
    }
    if (o.rng_mode == RT_RNG_REPLAY && !o.replay_states && !d_replay) {
        set_error("replay table missing");
        return -1;
    }
    if (sp) d_out = reinterpret_cast<uint32_t *>(1);  // (a pass writes counts, not pixels)
    if (width > 0xFFFFFFu || height > 0xFFFFFFu) { set_error("frame too large"); return -1; }
    const uint32_t B = nranks > 1 ? (o.row_block ? o.row_block : 1) : (uint32_t)std::max<size_t>(height, 1);
    const size_t T = tile_rows(height, B, o.rank, nranks);
    if (width == 0 || T == 0) return 0;
    if (!d_out) { set_error("null output"); return -1; }

    std::lock_guard<std::recursive_mutex> lock(w.mu);
    DeviceState *d = nullptr;
    int rc = device_for(w, o.device, d);
    if (rc) return rc;
    hipStream_t s = stream ? stream : d->stream;
    // the device's scratch (job counters, rings, slab, stats) is shared by every
    // frame on it: a frame enqueued on another stream waits for the last one
    if (d->done_stream && d->done_stream != s) HIP_TRY(hipStreamWaitEvent(s, d->done, 0));

    const uint32_t spp = o.samples_per_pixel > 0 ? (uint32_t)o.samples_per_pixel : 0u;
    const uint64_t jobs_per_row = (uint64_t)width * spp;
    if (jobs_per_row > 0x7FFFFFFFull) { set_error("width*spp too large"); return -1; }
    // Fused resolve (default): samples live in per-wave rings and the trace
    // kernel writes the RGBA8 pixels.  The slab path (every sample to HBM, then
    // resolve_kernel) serves RT_FLAG_KEEP_SAMPLES and spp above 4096 (a ring
    // slot holds at least one whole pixel).
    const bool fused = spp > 0 && spp <= 4096 && !(o.flags & RT_FLAG_KEEP_SAMPLES) &&
                       env_u64("RT_AMD_FUSED", 1) != 0;
    // jobs per launch: 2^31 (fused: C3 in one launch) or 2^30 (a 12 GB slab)
    const uint64_t slab_jobs = env_u64("RT_AMD_SLAB_JOBS", fused ? (1ull << 31) - 1 : 1ull << 30);
    size_t rows_per_slab = jobs_per_row ? (size_t)std::max<uint64_t>(1, slab_jobs / jobs_per_row) : T;
    rows_per_slab = std::min(rows_per_slab, T);
    if (jobs_per_row && !fused)
        HIP_TRY(grow(d->samples, d->samples_cap, 3 * rows_per_slab * jobs_per_row));

    const bool replay = d_replay != nullptr || o.rng_mode == RT_RNG_REPLAY;
    if (!d_replay && !sp && o.rng_mode == RT_RNG_REPLAY && spp) {
        const size_t n = width * height * (size_t)spp;
        HIP_TRY(grow(d->replay, d->replay_cap, n));
        HIP_TRY(hipMemcpyAsync(d->replay, o.replay_states, n * 4, hipMemcpyHostToDevice, s));
    }

    TraceParams p{};
    bool primary_lists = false;  // the frame's primary rays use candidate lists
    p.sph_hot = d->sph_hot; p.sph_cold = d->sph_cold;
    p.tri_hot = d->tri_hot; p.tri_geo = d->tri_geo;
    p.mats = d->mats;
    p.samples = d->samples;
    p.job_counter = d->counter;
    p.job_counter_next = nullptr;
    // (set 0 is also the SERIAL passes' scratch: the double-buffered frame sets
    // start over from a fill after them)
    if (sp) d->cset_clean[0] = d->cset_clean[1] = false;
    p.replay = d_replay ? d_replay : d->replay;
    const Vec3 cv[4] = {cam.origin, cam.lower_left, cam.horizontal, cam.vertical};
    for (int i = 0; i < 4; ++i) { p.cam[3 * i] = cv[i].x; p.cam[3 * i + 1] = cv[i].y; p.cam[3 * i + 2] = cv[i].z; }
    p.wden = (float)(uint64_t)(width - 1);   // (width-1) as f32 (common.rs:335)
    p.hden = (float)(uint64_t)(height - 1);  // (height-1) as f32 (common.rs:336)
    // the camera divisions through exactdiv.h: a denominator in [2^-40, 2^40]
    // and its correctly rounded reciprocal (IEEE division on the host)
    auto den_ok = [](float b) { return b >= 0x1p-40f && b <= 0x1p40f; };
    p.xdiv_uv = den_ok(p.wden) && den_ok(p.hden);
    p.wrcp = p.xdiv_uv ? 1.0f / p.wden : 0.0f;
    p.hrcp = p.xdiv_uv ? 1.0f / p.hden : 0.0f;
    p.nsph = d->nsph; p.nsph_padded = d->nsph_padded; p.ntri = d->ntri;
    p.width = (uint32_t)width; p.height = (uint32_t)height; p.spp = spp;
    p.depth = o.max_ray_bounces;
    p.mode = replay ? (uint32_t)RT_RNG_REPLAY : (uint32_t)RT_RNG_COUNTER;
    p.seed = o.seed;
    p.ablate = (uint32_t)env_u64("RT_AMD_ABLATE", 0);
    p.sph_shade = d->sph_shade;
    p.sph_kind = d->sph_kind;

    p.div_width = make_fastdiv((uint32_t)width);
    p.div_spp = make_fastdiv(spp ? spp : 1);
    p.div_rowblock = make_fastdiv(B);
    // node visits per lane per loop iteration of a sliced walk (A/B on C5, 8
    // waves per SIMD: 32 -> 277 ms, 64 -> 259, 96 -> 252, 128 -> 248, 192 ->
    // 251, 256 -> 263, 512 -> 353; 6 waves: 64 -> 243, 96 -> 240, 128 -> 242)
    p.steps = (uint32_t)std::max<uint64_t>(1, env_u64("RT_AMD_STEPS", 128));
    p.row_block = B; p.rank = o.rank; p.nranks = nranks;
    const bool use_bvh = d->nnodes > 0 && o.accel != RT_ACCEL_BRUTE;
    if (use_bvh) {
        const SphereBVH &bv = w.bvh;
        p.bvh_nodes = d->bvh_nodes; p.bvh_miss = d->bvh_miss;
        p.bvh_prims = d->bvh_prims; p.bvh_prim_id = d->bvh_prim_id;
        p.big_hot = d->big_hot; p.big_id = d->big_id;
        p.nnodes = d->nnodes; p.nbig = d->nbig; p.nprims = d->nprims;
        p.bvh_miss16 = d->bvh_miss16;
        p.use_lds = d->lds_bytes > 0 && env_u64("RT_AMD_LDS", 1) != 0;
        for (int k = 0; k < 3; ++k) p.bvh_c[k] = bv.centre[k];
        p.bvh_r = bv.radius; p.bvh_rmax = bv.rmax; p.bvh_mag = bv.mag;
        p.bvh_inv_rmin = env_u64("RT_AMD_LINEAR_E", 0) ? INFINITY : bv.inv_rmin;
        // sphere-only scenes: primary rays test their pixel's candidates
        if (d->ntri == 0 && env_u64("RT_AMD_SPHERE_LISTS", 1) != 0 && gpu_lists()) {
            bool ok = false;
            rc = device_sphere_lists(w, d, cam, width, height, s, ok);
            if (rc) return rc;
            p.spl = ok ? d->gspl : nullptr;
            primary_lists = ok;
        } else if (d->ntri == 0 && env_u64("RT_AMD_SPHERE_LISTS", 1) != 0 &&
                   prepare_primary_sphere_lists(w, cam, width, height)) {
            if (d->spl_version != w.spl_version) {
                if (d->spl) HIP_TRY(hipFree(d->spl));
                d->spl = nullptr;
                if (!w.spl.rec.empty()) {
                    HIP_TRY(hipMalloc((void **)&d->spl, w.spl.rec.size() * 4));
                    HIP_TRY(hipMemcpy(d->spl, w.spl.rec.data(), w.spl.rec.size() * 4,
                                      hipMemcpyHostToDevice));
                }
                d->spl_version = w.spl_version;
            }
            p.spl = d->spl;
            primary_lists = p.spl != nullptr;
        }
    }
    const bool use_tbvh = d->tnodes > 0 && o.accel != RT_ACCEL_BRUTE;
    const bool want_ptl = width >= 2 && height >= 2 && env_u64("RT_AMD_PRIMARY_LISTS", 1) != 0;
    if (use_tbvh) prepare_camera_lists(w, cam, width, height, want_ptl);
    if (use_tbvh && w.ctree_version && d->cam_version != w.ctree_version) {
        for (void *b : {(void *)d->cam_nodes, (void *)d->cam_tris})
            if (b) HIP_TRY(hipFree(b));
        d->cam_nodes = nullptr;
        d->cam_tris = nullptr;
        d->cam_nnodes = 0;
        const CameraTriangleBVH &ct = w.ctree;
        if (!ct.tris.empty()) {
            HIP_TRY(hipMalloc((void **)&d->cam_tris, ct.tris.size() * 4));
            HIP_TRY(hipMemcpy(d->cam_tris, ct.tris.data(), ct.tris.size() * 4, hipMemcpyHostToDevice));
        }
        if (!ct.nodes.empty()) {
            HIP_TRY(hipMalloc((void **)&d->cam_nodes, ct.qnodes.size() * 4));
            HIP_TRY(hipMemcpy(d->cam_nodes, ct.qnodes.data(), ct.qnodes.size() * 4, hipMemcpyHostToDevice));
            d->cam_nnodes = (uint32_t)(ct.qnodes.size() / 8);
        }
        d->cam_version = w.ctree_version;
    }
    if (use_tbvh) {
        if (d->cam_tris && std::memcmp(w.ctree.origin, &cam.origin, 12) == 0) {
            p.cam_tris = d->cam_tris;
            if (d->cam_nnodes) {
                p.cam_nodes = d->cam_nodes;
                p.cam_nnodes = d->cam_nnodes;
            }
            if (want_ptl && w.ptl_version && w.ptl_w == width && w.ptl_h == height &&
                w.ptl_ctree == w.ctree_version && same_cam(w.ptl_cam, cam)) {
                if (d->ptl_version != w.ptl_version) {
                    for (void *b : {(void *)d->ptl_off, (void *)d->ptl_items})
                        if (b) HIP_TRY(hipFree(b));
                    d->ptl_off = d->ptl_items = nullptr;
                    const PrimaryTriLists &pl = w.ptl;
                    if (!pl.offsets.empty()) {
                        HIP_TRY(hipMalloc((void **)&d->ptl_off, pl.offsets.size() * 4));
                        HIP_TRY(hipMemcpy(d->ptl_off, pl.offsets.data(), pl.offsets.size() * 4,
                                          hipMemcpyHostToDevice));
                        HIP_TRY(hipMalloc((void **)&d->ptl_items, std::max<size_t>(pl.items.size(), 1) * 4));
                        if (!pl.items.empty())
                            HIP_TRY(hipMemcpy(d->ptl_items, pl.items.data(), pl.items.size() * 4,
                                              hipMemcpyHostToDevice));
                    }
                    d->ptl_version = w.ptl_version;
                }
                if (d->ptl_off) {
                    primary_lists = true;
                    p.ptl_off = d->ptl_off;
                    p.ptl_items = d->ptl_items;
                    p.ptl_spr = w.ptl.strips_per_row;
                    p.ptl_always = w.ptl.offsets.back();
                    p.ptl_end = (uint32_t)w.ptl.items.size();
                }
            }
            for (int k = 0; k < 3; ++k) { p.cq_base[k] = w.ctree.qbox.base[k]; p.cq_step[k] = w.ctree.qbox.step[k]; }
        }
        const TriangleBVH &tb = w.tbvh;
        p.tbvh_nodes = d->tbvh_nodes;
        p.tbvh_tris = d->tbvh_tris; p.tbvh_loose = d->tbvh_loose;
        p.tnodes = d->tnodes; p.ttris = d->ttris; p.tloose = d->tloose;
        for (int k = 0; k < 3; ++k) {
            p.tbvh_c[k] = tb.centre[k];
            p.tbvh_oc[k] = tb.oc[k];
            p.tq_base[k] = tb.qbox.base[k];
            p.tq_step[k] = tb.qbox.step[k];
        }
        p.tq_nbase = tb.nbase;
        p.tq_nstep = tb.nstep;
        if (d->tw_nodes) {
            p.tw_nodes = d->tw_nodes;
            p.tw_depth = d->tw_depth;
            p.tw_tris = (const float4 *)d->tbvh_tris;
            if (d->tw_tris) {
                const TriangleCells &tc = w.tcells;
                p.tw_tris = (const float4 *)d->tw_tris;
                p.tw_stride = tc.stride_w;
                p.tc_ncells = tc.ncells;
                for (int k = 0; k < 3; ++k) { p.tc_n[k] = tc.n[k]; p.tc_lo[k] = tc.lo[k]; }
                p.tc_size = tc.size;
                p.tc_inv_size = 1.0f / tc.size;
            }
            // wide-node fetches per lane per loop iteration of a sliced walk (A/B
            // on C5: 16 -> 166.1 ms, 20 -> 163.9, 24 -> 163.5, 28 -> 164.4, 32 -> 166.4)
            p.wsteps = (uint32_t)std::max<uint64_t>(1, env_u64("RT_AMD_WSTEPS", 24));
        }
        p.tbvh_r = tb.radius; p.tbvh_mag = std::max(tb.mag, w.tcells.mag);
    }
    const float inv_spp = 1.0f / (float)o.samples_per_pixel;  // 1.0 / spp as f32 (common.rs:345)
    p.inv_spp = inv_spp;
    {
        // every sample's alpha is exactly 1.0, so each pixel's
        // alpha byte is this one fold, done once (resolve_kernel does it per pixel)
        float a = 1.0f;  // Color::new(0,0,0) has alpha 1 (color.rs:21-23)
        for (uint32_t k = 0; k < spp && a + 1.0f != a; ++k) a = a + 1.0f;
        const float x = a * inv_spp * 255.999f;
        p.alpha_u8 = !(x > 0.0f) ? 0u : x >= 255.0f ? 255u : (uint32_t)x;  // saturating `as u8`
    }
    p.out = d_out;

    // sliced walks pay off when walk lengths vary a lot: scenes with a triangle tree
    p.step = (uint32_t)env_u64("RT_AMD_STEP", use_tbvh ? 1 : 0) != 0;
    // whole walks (sphere scenes): refill once half the wave is idle, so lanes
    // refilled together start samples of the same pixel and their primary
    // walks stay coherent (A/B on C2: 1 -> 6.16 ms, 8 -> 6.14, 16 -> 6.12,
    // 32 -> 6.10); sliced walks refill every iteration (C5: 32 costs +5 %)
    // The wide triangle walk (frames only; SERIAL passes walk the binary tree):
    // refill at 16 idle lanes and walk only when no lane can advance without
    // it (A/B on C5, refill / walk gate: 1 / 32 -> 163.5 ms, 8 / 32 -> 159.7,
    // 8 / 64 -> 156.8, 12 / 64 -> 153.1, 16 / 64 -> 151.8, 20 / 64 -> 152.2,
    // 24 / 64 -> 154.6, 32 / 64 -> 164.7)
    const bool wide_frame = p.tw_nodes != nullptr && sp == nullptr;
    p.refill_min = (uint32_t)std::max<uint64_t>(
        1, env_u64("RT_AMD_REFILL", wide_frame ? 16 : p.step ? 1 : 24));
    p.walk_min = (uint32_t)env_u64("RT_AMD_WALK_MIN", 65);  // sphere-only: walk when nothing else can advance
    p.tri_walk_min = (uint32_t)env_u64("RT_AMD_TRI_WALK_MIN", wide_frame ? 64 : 32);
    const int sv = p.step ? 1 : 0;
    const bool timed = stats != nullptr;  // HIP-event timing + counters need a host wait
    // launch_trace runs the counting variant iff p.stats, the SERIAL instances for sp
    const int ctv = sp ? 2 : timed ? 1 : 0;
    const int bpc = !use_bvh   ? d->blocks_per_cu[ctv][sv]
                    : p.use_lds ? d->blocks_per_cu_lds[ctv][sv]
                                : d->blocks_per_cu_bvh[ctv][sv];
    // (the kernel family launch_trace picks: the wide triangle walk for frames)
    const int fam = p.ntri == 0 ? 0 : p.tnodes == 0 ? 1 : (p.tw_nodes != nullptr && ctv != 2) ? 3 : 2;
    const uint64_t waves_per_block = trace_block_threads(use_bvh && p.use_lds, fam, ctv) / 64;
    const uint64_t full_blocks = (uint64_t)bpc * (uint64_t)d->num_cus;
    uint32_t launches = 0, waves = 0;
    // counters only when asked for: one 16-slot record per wave, summed here
    const uint64_t max_waves = full_blocks * waves_per_block;
    p.stats = nullptr;
    if (timed) {
        HIP_TRY(grow(d->stats, d->stats_cap, max_waves * kStatSlots));
        HIP_TRY(hipMemsetAsync(d->stats, 0, max_waves * kStatSlots * 8, s));
        p.stats = d->stats;
    }
    if (sp) {
        // one SERIAL pass: nsamples x variants jobs (job = launch sample *
        // variants + variant); each stores its scatter count to slab plane 0
        const uint64_t njobs = (uint64_t)sp->nsamples * sp->variants;
        if (njobs == 0) return 0;
        if (njobs > 0x7FFFFFFFull) { set_error("serial pass too large"); return -1; }
        if (sp->mode != kRngSerialCoalesce && sp->mode != kRngSerialPixel)
            HIP_TRY(grow(d->samples, d->samples_cap, 3 * njobs));
        p.samples = sp->mode == kRngSerialPixel ? sp->ptab : d->samples;
        p.sL = sp->L;
        p.sK = sp->Kmax;
        p.ring = nullptr;
        p.ring_shift = 0;
        p.mode = sp->mode;
        p.spp = sp->variants;
        p.div_spp = make_fastdiv(sp->variants);
        p.sspp = spp;
        p.div_sspp = make_fastdiv(spp ? spp : 1);
        p.cbase = sp->cbase;
        p.nserial = (uint32_t)((uint64_t)width * height * spp);
        p.win = sp->win;
        p.sM = sp->M;
        p.slo = sp->lo;
        p.spix = sp->spix;
        p.ctrl = sp->ctrl;
        p.max_draws = 2u + 3u * (uint32_t)std::max(o.max_ray_bounces, 0);
        p.njobs = (uint32_t)njobs;
        p.npix = sp->nsamples;
        p.slab_row0 = 0;
        const uint64_t jobs_per_block = waves_per_block * 256;
        const uint64_t blocks = std::max<uint64_t>(
            1, std::min<uint64_t>(full_blocks, (njobs + jobs_per_block - 1) / jobs_per_block));
        const uint64_t nwaves = blocks * waves_per_block;
        // the count pass: chunks of 128 jobs, not whole samples of K candidates
        // (the end of the launch drains sooner: c_raytracer 960x540x16 SERIAL
        // 671 -> 608 ms; 64: 610 ms; more partitions cost, 64: +8 %, 256: +30 %)
        uint64_t chunk = std::min<uint64_t>(256, std::max<uint64_t>(64, njobs / (nwaves * 16) / 64 * 64));
        chunk = chunk >= sp->variants ? chunk / sp->variants * sp->variants : sp->variants;
        if (sp->mode == kRngSerialCount) chunk = env_u64("RT_AMD_SERIAL_CCHUNK", 128);
        // the pixel table pass: chunks of consecutive positions of one pixel, not
        // whole pixels (a pixel's span is 10^3 positions: whole-pixel chunks
        // left most waves without work); 128 since round 5
        // (profiles/round5_serial/sweep_pchunk.jsonl: 64 / 128 / 192 / 256 / 512
        // -> world.txt 960x540x16 89.1 / 84.6 / 83.9 / 85.0 / 88.9 ms, 1920x1080x16
        // 365 / 337 / 334 / 337 / 355 ms, RTOW at C2 settings 699 / 665 / 670 /
        // 693 / 790 ms)
        if (sp->mode == kRngSerialPixel) chunk = env_u64("RT_AMD_SERIAL_PCHUNK", 128);
        p.chunk = (uint32_t)std::max<uint64_t>(1, chunk);
        uint64_t parts = std::max<uint64_t>(
            1, std::min<uint64_t>({(uint64_t)(p.step ? 64 : 16), kMaxParts, njobs / (16 * chunk) + 1}));
        if (const uint64_t np = env_u64("RT_AMD_SERIAL_PARTS", 0)) parts = std::min<uint64_t>(np, kMaxParts);
        p.nparts = (uint32_t)parts;
        if (sp->mode == kRngSerialPixel) {
            // (job counters zeroed by serial_window_kernel, kPixtabParts of them)
            p.nparts = (uint32_t)std::min<uint64_t>(parts, kPixtabParts);
            HIP_TRY(launch_trace(p, (uint32_t)blocks, s));
        } else if (sp->mode == kRngSerialCoalesce) {
            // one workgroup per block of sp->R samples; the tree in LDS when it
            // fits beside the search's own arrays (64 KB per workgroup)
            const bool tree_lds = p.use_lds && serial_coalesce_lds(p, sp->variants, true) <= 64 * 1024;
            HIP_TRY(launch_serial_coalesce(p, sp->path, sp->bend, sp->nsamples, sp->variants, sp->R, tree_lds,
                                           sp->dbg, s));
        } else {
            HIP_TRY(hipMemsetAsync(d->counter, 0, parts * 128, s));
            HIP_TRY(launch_trace(p, (uint32_t)blocks, s));
        }
        HIP_TRY(hipEventRecord(d->done, s));
        d->done_stream = s;
        d->last_jobs = 0;  // the slab holds counts now, not samples
        return 0;
    }
    // One frame launch's schedule for kernel kind k (0 lean, 1 counting):
    // workgroups, waves, jobs per queue pull (chunk) and job-queue partitions
    struct LaunchPlan { uint64_t blocks, nwaves, chunk, parts, block_threads; };
    auto plan = [&](int k, uint64_t njobs) -> LaunchPlan {
        const int kb = !use_bvh ? d->blocks_per_cu[k][sv] : p.use_lds ? d->blocks_per_cu_lds[k][sv]
                                                                     : d->blocks_per_cu_bvh[k][sv];
        const uint64_t wpb = trace_block_threads(use_bvh && p.use_lds, fam, k) / 64;
        const uint64_t jobs_per_block = wpb * 256;
        uint64_t blocks = std::min<uint64_t>((uint64_t)kb * d->num_cus, (njobs + jobs_per_block - 1) / jobs_per_block);
        blocks = std::max<uint64_t>(blocks, 1);
        const uint64_t nwaves = blocks * wpb;
        uint64_t chunk = env_u64("RT_AMD_CHUNK", 0);
        if (!chunk) chunk = std::min<uint64_t>(256, std::max<uint64_t>(64, njobs / (nwaves * 16) / 64 * 64));
        // whole pixels per chunk (partitions are pixel-aligned too), so a
        // chunk's pixels are complete once its samples are
        chunk = chunk >= spp ? chunk / spp * spp : spp;
        if (fused) {
            // a resolve sums one pixel per lane, so whole-walk kernels take
            // chunks of >= 8 pixels (<= 4096 jobs unless spp is larger;
            // A/B, C2: 4 px 7.10 ms, 8 px 6.79, 16 px 6.83, 32 px 7.36,
            // slab + resolve_kernel 6.94).  Sliced walks keep their chunk
            // (C5: 16 px +1.5 %, 4 px = slab)
            uint64_t px = std::max<uint64_t>(1, std::min<uint64_t>(
                env_u64("RT_AMD_RESOLVE_PIX", p.step ? 1 : 8), 4096 / spp));
            // small launches (multi-GPU tiles) keep >= 16 chunks per wave
            // where 4-pixel chunks allow it (C2 tile of 8 ranks: 8 px 1.12 ms,
            // 4 px 1.04, 2 px 1.22; C3 tile of 8 ranks, 21 chunks of 8 px per
            // wave: 8 px 9.80 ms, 4 px 9.17, 2 px 9.32; of 4 ranks, 42: 8 and
            // 4 px 18.0 ms; of 2 ranks: 8 px 35.0, 4 px 35.5).  Round 5: 32
            // until then, which put the full C2 frame (31.6 chunks of 8 px per
            // wave at 8,192 waves) on 4-pixel chunks: lean frame 3.900 ms
            // against 3.745 ms with 8, 3.811 with 12 and 3.912 with 16 pixels
            // (profiles/round5_walk/ab_c2_chunk.jsonl); the 8-rank tile keeps
            // 4 px (0.678 ms, 8 px 0.849 ms)
            while (px > 4 && njobs / (nwaves * px * spp) < 16) px /= 2;
            chunk = std::max<uint64_t>(chunk, px * spp);
        }
        // job-queue partitions: each keeps >= 16 chunks.  Whole-walk
        // kernels take 8: a wave whose partition is drained probes the
        // others one atomic at a time, so at the end of a launch fewer
        // partitions drain faster (A/B, round 2, C2: 64 -> 5.42 ms, 32 ->
        // 5.38, 16 -> 5.35, 8 -> 5.36; round 4, 8192 waves of 1024-thread
        // workgroups, lean frames: 16 -> 4.453 ms, 12 -> 4.335, 10 -> 4.331,
        // 8 -> 4.346, 4 -> +6 % on the tiles; 8-rank tile 16 -> 0.78, 8 ->
        // 0.76 ms; C3 62.44 -> 62.37 ms).  Sliced walks keep 64 (C5: 16
        // costs +1.6 %).
        uint64_t parts = env_u64("RT_AMD_PARTS", p.step ? 64 : 8);
        parts = std::max<uint64_t>(1, std::min<uint64_t>({parts, kMaxParts, njobs / (16 * chunk) + 1}));
        return LaunchPlan{blocks, nwaves, chunk, parts, wpb * 64};
    };
    LaunchPlan lean_plan{0, 0, 0, 0, 0};  // the uncounted (timed) kernel's schedule of the last launch
    uint32_t nslab = 0;  // (counted frames: event triple per launch)
    for (size_t r0 = 0; r0 < T; r0 += rows_per_slab, ++nslab) {
        const size_t rows = std::min(rows_per_slab, T - r0);
        hipEvent_t *ev3 = nullptr;
        if (timed) {
            while (d->tev.size() < 3 * (size_t)(nslab + 1)) {
                hipEvent_t e;
                HIP_TRY(hipEventCreate(&e));
                d->tev.push_back(e);
            }
            ev3 = &d->tev[3 * (size_t)nslab];
        }
        const uint64_t njobs = rows * jobs_per_row;
        p.slab_row0 = (uint32_t)r0;
        p.gj32 = nranks == 1 && (uint64_t)width * height * spp < (1ull << 32) ? 1u : 0u;
        p.gj_c0 = (uint32_t)(((uint64_t)height - 1 - r0) * width * spp);
        p.gj_2p = (uint32_t)(2ull * width * spp);
        p.njobs = (uint32_t)njobs;
        p.npix = (uint32_t)(rows * width);
        if (timed) HIP_TRY(hipEventRecord(ev3[0], s));
        if (njobs) {
            const LaunchPlan lp = plan(ctv, njobs);
            const uint64_t blocks = lp.blocks, nwaves = lp.nwaves, chunk = lp.chunk, parts = lp.parts;
            p.chunk = (uint32_t)chunk;
            p.ring = nullptr;
            p.ring_shift = 0;
            if (fused) {
                while ((1ull << p.ring_shift) < chunk) ++p.ring_shift;
                HIP_TRY(grow(d->ring, d->ring_cap, nwaves * 3 * (kTraceRing << p.ring_shift)));
                p.ring = d->ring;
            }
            p.nparts = (uint32_t)parts;
            // two counter sets: this launch takes set cset (zeroed by the launch
            // before it, or filled here) and zeroes the other for the next one,
            // so back-to-back frames need no fill launch (a fill plus its gap
            // before the trace kernel was ~20 us of every C2 frame)
            uint32_t *const cur = d->counter + (size_t)d->cset * kMaxParts * 32;
            if (!d->cset_clean[d->cset]) HIP_TRY(hipMemsetAsync(cur, 0, parts * 128, s));
            p.job_counter = cur;
            p.job_counter_next = d->counter + (size_t)(d->cset ^ 1u) * kMaxParts * 32;
            HIP_TRY(launch_trace(p, (uint32_t)blocks, s));
            d->cset_clean[d->cset] = false;
            d->cset ^= 1u;
            d->cset_clean[d->cset] = true;
            p.job_counter = d->counter;
            p.job_counter_next = nullptr;
            lean_plan = ctv == 0 ? lp : plan(0, njobs);
            d->last_jobs = fused ? 0 : njobs;
            d->last_spp = spp;
            d->last_fused = fused;  // rt_read_samples needs the slab
            ++launches;
            waves = (uint32_t)nwaves;
        }
        if (timed) HIP_TRY(hipEventRecord(ev3[1], s));
        if (!fused)  // (spp 0: no samples, the resolve still writes every pixel)
            HIP_TRY(launch_resolve_ex(d->samples, d_out, (uint32_t)(rows * width), spp, inv_spp,
                                      (uint32_t)width, (uint32_t)r0, s));
        if (timed) HIP_TRY(hipEventRecord(ev3[2], s));
    }
    HIP_TRY(hipEventRecord(d->done, s));
    d->done_stream = s;
    // without stats the frame stays asynchronous on the stream (no host wait)
    if (!timed) return 0;
    // the wave records into pinned host memory (an asynchronous copy, so a
    // deferred frame does not wait here)
    const size_t nrec = max_waves * kStatSlots;
    if (d->hrec_cap < nrec) {
        if (d->hrec) HIP_TRY(hipHostFree(d->hrec));
        d->hrec = nullptr;
        d->hrec_cap = 0;
        HIP_TRY(hipHostMalloc((void **)&d->hrec, nrec * 8));
        d->hrec_cap = nrec;
    }
    HIP_TRY(hipMemcpyAsync(d->hrec, d->stats, nrec * 8, hipMemcpyDeviceToHost, s));
    auto &pd = d->pend;
    pd.active = true;
    pd.nrec = nrec;
    pd.nslab = nslab;
    pd.launches = launches;
    pd.samples = (uint64_t)T * jobs_per_row;
    pd.use_bvh = use_bvh;
    pd.use_tbvh = use_tbvh;
    pd.stream = s;
    RtRenderStatsFixed &fx = pd.fixed;
    fx = RtRenderStatsFixed{};
    fx.waves = waves;
    fx.accel = (use_bvh || use_tbvh) ? RT_ACCEL_BVH : RT_ACCEL_BRUTE;
    fx.tri_bvh = use_tbvh ? 1u : 0u;
    fx.fused_resolve = fused ? 1u : 0u;
    fx.primary_lists = primary_lists ? 1u : 0u;
    fx.camera_tree = p.cam_tris != nullptr ? 1u : 0u;  // camera-origin records (tree or lists)
    // (the schedule of the frame's uncounted kernel: what a timed frame runs)
    fx.launch_parts = (uint32_t)lean_plan.parts;
    fx.launch_chunk = (uint32_t)lean_plan.chunk;
    fx.launch_refill_min = p.refill_min;
    fx.launch_walk_min = p.walk_min;
    fx.launch_tri_walk_min = p.tri_walk_min;
    fx.launch_wsteps = p.wsteps;
    fx.launch_block_threads = (uint32_t)lean_plan.block_threads;
    fx.launch_blocks = (uint32_t)lean_plan.blocks;
    fx.nsph = d->nsph;
    fx.ntri = d->ntri;
    fx.nbig = d->nbig;
    if (defer_stats) return 0;
    return collect_frame_stats(d, stats);
}

int collect_frame_stats(DeviceState *d, RtRenderStats *stats) {
    auto &pd = d->pend;
    if (!pd.active) {
        set_error("no counted frame pending on this device");
        return -1;
    }
    pd.active = false;
    HIP_TRY(hipSetDevice(d->device));
    HIP_TRY(hipStreamSynchronize(pd.stream));
    double trace_ms = 0.0, resolve_ms = 0.0;
    for (uint32_t k = 0; k < pd.nslab; ++k) {
        float a = 0, b = 0;
        HIP_TRY(hipEventElapsedTime(&a, d->tev[3 * k], d->tev[3 * k + 1]));
        HIP_TRY(hipEventElapsedTime(&b, d->tev[3 * k + 1], d->tev[3 * k + 2]));
        trace_ms += a;
        resolve_ms += b;
    }
    const unsigned long long *rec = d->hrec;
    if (const char *dump = std::getenv("RT_AMD_WAVE_DUMP")) {  // diagnostic: raw per-wave records
        if (FILE *f = std::fopen(dump, "wb")) {
            std::fwrite(rec, 8, pd.nrec, f);
            std::fclose(f);
        }
    }
    unsigned long long st[kStatSlots] = {};
    for (size_t i = 0; i < pd.nrec; ++i) st[i % kStatSlots] += rec[i];
    if (stats) {
        const RtRenderStatsFixed &fx = pd.fixed;
        const bool use_bvh = pd.use_bvh, use_tbvh = pd.use_tbvh;
        stats->samples = pd.samples;
        stats->rays = st[0];
        stats->sphere_tests = st[0] * (uint64_t)fx.nsph;
        stats->tri_tests = st[0] * (uint64_t)fx.ntri;  // the reference's brute-force count
        stats->tri_in_range = st[1];
        stats->trace_ms = trace_ms;
        stats->resolve_ms = resolve_ms;
        stats->trace_launches = pd.launches;
        stats->waves = fx.waves;
        stats->launch_parts = fx.launch_parts;
        stats->launch_chunk = fx.launch_chunk;
        stats->launch_refill_min = fx.launch_refill_min;
        stats->launch_walk_min = fx.launch_walk_min;
        stats->launch_tri_walk_min = fx.launch_tri_walk_min;
        stats->launch_wsteps = fx.launch_wsteps;
        stats->launch_block_threads = fx.launch_block_threads;
        stats->launch_blocks = fx.launch_blocks;
        stats->accel = fx.accel;
        stats->bvh_sphere_tests = st[2];
        stats->bvh_node_tests = st[3];
        stats->big_sphere_tests = use_bvh ? st[0] * (uint64_t)fx.nbig : st[0] * (uint64_t)fx.nsph;
        for (int k = 0; k < 4; ++k) stats->stamp_cycles[k] = st[4 + k];
#ifdef RT_STAMPS
        {   // fine segments (tools/stamps.py parses this line)
            double tot = 0;
            for (uint32_t k = 0; k < kStampSegs; ++k) tot += (double)st[16 + k];
            std::fprintf(stderr, "stamp segments:");
            for (uint32_t k = 0; k < kStampSegs; ++k) std::fprintf(stderr, " %.4f", st[16 + k] / std::max(1.0, tot));
            std::fprintf(stderr, " cycles %.6e\n", tot);
        }
#endif
        stats->tri_node_tests = st[8];
#ifdef RT_WALK_MIX
        std::fprintf(stderr, "walk mix: %llu walks, %.2f iterations per walk, %.2f with a leaf, %.2f leaf trips\n",
                     st[7], st[4] / std::max(1.0, (double)st[7]), st[5] / std::max(1.0, (double)st[7]),
                     st[6] / std::max(1.0, (double)st[7]));
#endif
        if (env_u64("RT_AMD_ITER_DEBUG", 0))
            std::fprintf(stderr, "iteration mix: %llu iterations (%.1f active lanes), %llu walking (%.1f lanes), "
                         "%llu other (%.1f lanes)\n", st[10], st[12] / std::max(1.0, (double)st[10]), st[11],
                         st[13] / std::max(1.0, (double)st[11]), st[10] - st[11],
                         (st[12] - st[13]) / std::max(1.0, (double)(st[10] - st[11])));
        stats->tri_bvh = fx.tri_bvh;
        stats->fused_resolve = fx.fused_resolve;
        stats->primary_lists = fx.primary_lists;
        stats->camera_tree = fx.camera_tree;
        stats->bvh_tri_tests = use_tbvh ? st[9] : stats->tri_tests;
    }
    return 0;
}

// ------------------------------------------------------------ SERIAL mode
// The reference draws every sample from one xorshift32 stream seeded 2547549
// (common.rs:321, random.rs:8-30): sample j (reference order (row * W + col)
// * spp + s) starts at stream position P_j = 2j + 3 B_j, where B_j counts the
// diffuse/metal scatters of all earlier samples (2 draws for u, v, 3 per
// random_unit_sphere).  That is a sequential dependency, resolved here on the
// device chunk by chunk:
//   1. estimate: each sample traced R times from counter seeds gives every
//      pixel's mean scatter count (kRngSerialEstimate);
//   2. per chunk of L samples, whose first sample's B is known exactly:
//      window: the stream states from that sample's start on (jump matrices);
//      count: every sample traced from K candidate positions centred on its
//        predicted offset (kRngSerialCount), a table of scatter counts;
//      walk: one lane follows the true path through the table, writing each
//        sample's start state and the next chunk's start state;
//      a walk that leaves its window cancels the remaining launches and the
//      host resumes from that chunk with a window twice as wide;
//   3. the frame is rendered in REPLAY mode from the start states.
// The result is the reference's own frame, bit for bit (tests/test_gpu_serial.py).
namespace {
uint32_t xorshift32(uint32_t x) {
    x ^= x << 13;
    x ^= x >> 17;
    x ^= x << 5;
    return x;
}

// columns of M^(2^i), i < 64, M the xorshift32 step as a GF(2) matrix
// xorshift32 jump matrices (GF(2), 32 columns each; render.h
// kSerialJumpWords): M^(2^i) for i < 64, then M^(w j) for j < 4096 / w (w =
// kSerialWinPerThread) and M^(4096 j) for j < 256 (serial_window_kernel: two
// applies reach any multiple of w below 2^20)
std::vector<uint32_t> xorshift_jump_table() {
    std::vector<uint32_t> t(kSerialJumpWords);
    for (uint32_t c = 0; c < 32; ++c) t[c] = xorshift32(1u << c);
    auto apply = [&](const uint32_t *cols, uint32_t x) {
        uint32_t y = 0;
        for (uint32_t c = 0; c < 32; ++c)
            if (x >> c & 1u) y ^= cols[c];
        return y;
    };
    for (int i = 1; i < 64; ++i)
        for (uint32_t c = 0; c < 32; ++c) t[32 * i + c] = apply(&t[32 * (i - 1)], t[32 * (i - 1) + c]);
    static_assert((kSerialWinPerThread & (kSerialWinPerThread - 1)) == 0, "a power of two");
    int wlog = 0;
    while ((1u << wlog) < kSerialWinPerThread) ++wlog;
    for (int lvl = 0; lvl < 2; ++lvl) {
        uint32_t *T = &t[(size_t)32 * (64 + (lvl ? kSerialJumpT1 : 0))];
        const uint32_t *step = &t[32 * (lvl == 0 ? wlog : 12)];  // M^w, M^4096
        const uint32_t cnt = lvl == 0 ? kSerialJumpT1 : 256u;
        for (uint32_t c = 0; c < 32; ++c) T[c] = 1u << c;  // M^0
        for (uint32_t j = 1; j < cnt; ++j)
            for (uint32_t c = 0; c < 32; ++c) T[32 * j + c] = apply(step, T[32 * (j - 1) + c]);
    }
    return t;
}
}  // namespace

// sigma floor of a sample's scatter count (the frame-wide K adds 0.05 to its
// sigma), scaled for the means' estimation error from `per` traces a pixel
static double serial_floor(uint64_t per) { return 0.05 * std::sqrt(1.0 + 1.0 / (double)per); }

static int serial_check_args(size_t width, size_t height, const RtRenderOptions &o) {
    const uint64_t N = (uint64_t)width * height * (uint64_t)std::max(o.samples_per_pixel, 0);
    if (N >= 0xFFFFFFFFull) {
        set_error("RT_RNG_SERIAL: width * height * spp must be below 2^32");
        return -1;
    }
    if (o.max_ray_bounces > 100000) {
        set_error("RT_RNG_SERIAL: max_ray_bounces above 100000");
        return -1;
    }
    return 0;
}

// Steps 1 and 2 of SERIAL mode on device d, stream s: every sample's start
// state of the whole width x height frame into d->sstates (frame sample
// order), the events sev[0] (start), sev[2] (tables done) and sev[1] (states
// found) recorded on s; with RT_FLAG_SERIAL_CHECK the chain is checked after
// sev[1].  stats (optional) gets the serial_* fields.
static int serial_find_states(WorldState &w, const CameraModel &cam, size_t width, size_t height,
                              const RtRenderOptions &o, DeviceState *d, hipStream_t s, RtRenderStats *stats) {
    const uint64_t spp = (uint64_t)std::max(o.samples_per_pixel, 0);
    const uint64_t N = (uint64_t)width * height * spp;
    const uint32_t depth = (uint32_t)std::max(o.max_ray_bounces, 0);
    int rc = 0;
    if (d->done_stream && d->done_stream != s) HIP_TRY(hipStreamWaitEvent(s, d->done, 0));
    HIP_TRY(hipEventRecord(d->sev[0], s));
    HIP_TRY(grow(d->sstates, d->sstates_cap, std::max<uint64_t>(N, 1)));
    RtRenderOptions ob = o;
    // the inner passes read and write d's buffers (d->samples, d->stab, ...):
    // pin them to d's device rather than to whichever device is current
    ob.device = d->device;
    ob.ndevices = 0;
    ob.rng_mode = RT_RNG_COUNTER;
    ob.rank = 0;
    ob.nranks = 1;
    ob.flags = 0;
    uint32_t final_state = o.seed;  // the stream state after the last sample
    if (N > 0) {
        const auto tp0 = std::chrono::steady_clock::now();  // (RT_AMD_SERIAL_DEBUG)
        // 1. per-pixel mean scatter counts from R counter-seeded traces per
        // sample, reduced on the device (per-pixel moments, then prefix sums
        // over pixels): no per-sample table and no host pass over the samples
        // (RT_AMD_SERIAL_EST traces per pixel: the means' error adds to every
        // window's deviation, sweep on the 960x540x16 frames at z 1.5:
        // c_raytracer / RTOW / world.txt 32 -> 457 / 315 / - ms, 128 -> 418 /
        // 281 / 364, 256 -> 416 / 285 / 360, 512 -> 427 / 281 / -; z 1.2 and
        // 1.0 cost more at every EST, 1.8 and 2.1 as much or more)
        // (round 5, with the pixel table: x2 per x4 samples per pixel from 16 spp,
        // like the iteration length -- profiles/round5_serial/sweep_estimate_
        // traces*.jsonl: world.txt 960x540x16 64 / 96 / 128 / 192 -> 84.7 / 84.0 /
        // 83.2 / 84.2 ms; RTOW at C2 settings 128 / 192 / 256 / 320 / 384 -> 639 /
        // 604 / 591 / 588 / 594 ms)
        uint64_t est_def = 128;
        for (uint64_t q = 64; q <= spp; q *= 4) est_def *= 2;
        const uint64_t est = std::max<uint64_t>(1, env_u64("RT_AMD_SERIAL_EST", est_def));
        const uint64_t R = std::max<uint64_t>(
            1, std::min<uint64_t>({(est + spp - 1) / spp, 64, 0x7FFFFFFFull / N}));
        const uint64_t npix = (uint64_t)width * height;
        const double per = (double)(spp * R);
        // The coalescing block search (serial_coalesce_kernel) or the count
        // pass over every (sample, candidate) pair + block walks.  Coalescing
        // traces 0.33-0.45 of the count pass's traces but runs each block's
        // samples in sequence: it wins where a trace is short -- brute-force
        // scenes, i.e. no sphere or triangle tree (< 16 of each: render()'s
        // scenes; 960x540x16 c_raytracer 338 -> 308 ms, world.txt 301 -> 233
        // ms) -- and loses on tree walks (RTOW 238 -> 620 ms).
        // RT_AMD_SERIAL_COALESCE: 0 off, 1 on, unset: that rule.  The rule
        // keys on the scene's size (trees are built for >= 16 spheres or
        // triangles), not on o.accel: a large scene forced to RT_ACCEL_BRUTE
        // has even longer traces and takes the count pass too.
        const bool trees = d->nnodes > 0 || d->tnodes > 0;
        // The pixel table pass (round 4, the default from 4 samples per pixel):
        // a sample's scatter count depends only on its pixel and its start
        // position (the samples of one pixel trace the same camera ray from
        // the same draws), so the count table of an iteration is gathered from
        // one trace per (pixel, stream position) that any of the pixel's
        // samples' windows covers -- about L (3K / spp + 2 + 3 mu) traces
        // instead of the count pass's L K, and independent ones, unlike the
        // coalescing search's chains.  RT_AMD_SERIAL_PIXTAB=0: the searches below.
        bool pixtab = spp >= 4 && env_u64("RT_AMD_SERIAL_PIXTAB", 1) != 0;
        // the pixel pass's per-pixel spans (one load per refill, whole-chunk rows)
        const bool use_spix = env_u64("RT_AMD_SERIAL_SPIX", 1) != 0;
        // ... and an iteration's reuse of the previous one's table (the positions
        // both windows cover, after a stop: DESIGN.md 3.4); two tables, alternating
        const bool reuse = use_spix && env_u64("RT_AMD_SERIAL_REUSE", 1) != 0;
        const uint64_t pchunk = std::max<uint64_t>(1, env_u64("RT_AMD_SERIAL_PCHUNK", 128));
        bool coalesce = false;
        // (iterations of 128 k samples in blocks of 32 for the coalescing search,
        // profiles/round3_serial/coalesce_sweep*.log; 16 k for the count pass;
        // the pixel table: 32 k at 16 spp, x sqrt(spp / 16) in powers of two --
        // its traces per sample grow as K / spp ~ sqrt(L) / spp, its fixed cost
        // per iteration as 1 / L; profiles/round4_serial/pixtab_sweep*.log:
        // world.txt 960x540x16 16 k / 32 k / 64 k -> 141 / 114 / 121 ms, RTOW
        // 1920x1080x64 64 k / 128 k / 256 k -> 1.01 / 1.07 / 1.24 s)
        uint64_t L = 1, Lw = 1, n0 = 1;
        // the iteration length for the search chosen (planned again, without the
        // pixel table, when its table turns out too large below)
        auto plan = [&]() {
            coalesce = !pixtab && env_u64("RT_AMD_SERIAL_COALESCE", trees ? 0 : 1) != 0 && depth < 1024;
            uint64_t Ldef = coalesce ? 131072 : 16384;
            if (pixtab) {
                // (round 5, after the iterations' fixed cost fell from ~90 to ~54
                // us: 48 k at 16 spp, profiles/round5_serial/iteration_length_*.log:
                // world.txt 960x540x16 32 k / 48 k / 64 k / 96 k -> 92.5 / 91.3 /
                // 94.3 / 102.5 ms, 1920x1080x16 400 / 368 / 385 / 425 ms; RTOW
                // 1920x1080x64 64 k / 96 k / 128 k -> 732 / 683 / 689 ms)
                Ldef = 49152;
                for (uint64_t q = 64; q <= spp; q *= 4) Ldef *= 2;        // 64 spp: 96 k, 256 spp: 192 k
                for (uint64_t q = spp; q < 16 && Ldef > 8192; q *= 4) Ldef /= 2;  // 4 spp: 24 k
            }
            L = std::max<uint64_t>(1, std::min<uint64_t>(env_u64("RT_AMD_SERIAL_CHUNK", Ldef), N));
            // windows are sized for the deviation over Lw samples (default L; a
            // longer Lw widens them, a shorter iteration stops less often)
            Lw = std::max<uint64_t>(1, env_u64("RT_AMD_SERIAL_WLEN", L));
            n0 = std::min(N, Lw);
        };
        plan();
        HIP_TRY(grow(d->stab, d->stab_cap, serial_tab_doubles((uint32_t)npix)));
        HIP_TRY(grow(d->sscan, d->sscan_cap, serial_scan_scratch((uint32_t)npix)));
        double *const sums = d->stab + 5 * npix + 2;  // {sum ss, dmax, V(n0), lost count}
        HIP_TRY(hipMemsetAsync(sums, 0, 8 * sizeof(double), s));
        {
            // launches of whole pixels, <= 2^28 traces each
            const uint64_t step_pix = std::max<uint64_t>(1, ((1ull << 28) / R) / spp);
            for (uint64_t p0 = 0; p0 < npix; p0 += step_pix) {
                const uint64_t np = std::min(step_pix, npix - p0);
                const SerialPass sp{kRngSerialEstimate, (uint32_t)(p0 * spp), (uint32_t)(np * spp), (uint32_t)R,
                                    nullptr, SerialPred{}, nullptr};
                rc = render_frame(w, cam, width, height, ob, nullptr, s, nullptr, &sp);
                if (rc) return rc;
                HIP_TRY(launch_serial_moments(d->samples, (uint32_t)p0, (uint32_t)np, (uint32_t)spp, (uint32_t)R,
                                              1.0 + 1.0 / per, d->stab, (uint32_t)npix, s));
            }
        }
        const SerialPred pred{d->stab, d->stab + npix + 1, (uint32_t)spp, (uint32_t)npix};
        const double z = (double)env_u64("RT_AMD_SERIAL_Z10", 15) / 10.0;
        double dmax = 0.0;  // largest predicted offset within L + L/4 samples: the window
        uint64_t K = 0, npq_max = 0, emax = 0;
        double sm[4] = {0.0, 0.0, 0.0, 0.0};  // {sum ss, dmax bits, V(n0), lost-count flag}
        double sigma = 0.0;
        for (;;) {
            HIP_TRY(launch_serial_tables(d->stab, d->sscan, (uint32_t)npix, (uint32_t)spp, (uint32_t)L,
                                         (uint32_t)n0, s));
            HIP_TRY(hipEventRecord(d->sev[2], s));
            HIP_TRY(hipMemcpyAsync(sm, sums, sizeof(sm), hipMemcpyDeviceToHost, s));
            HIP_TRY(hipStreamSynchronize(s));
            if (sm[3] != 0.0) {
                set_error("RT_RNG_SERIAL: estimate pass lost a sample's draw count");
                return -5;
            }
            {
                uint64_t bits;
                std::memcpy(&bits, &sm[1], 8);
                std::memcpy(&dmax, &bits, 8);
            }
            sigma = std::sqrt(std::max(sm[0], 0.0) / (double)(N * R)) + 0.05;
            // 2. iterations of L samples from the first unresolved one (ctrl[4]),
            // K candidates per sample, spanning +-z sigma of the deviation of the
            // true offset from the predicted one at the end of L samples.  Narrow
            // windows trade progress for work: an iteration resolves samples up
            // to where the path leaves a window, and the next one starts there
            // with its windows re-centred (no host round trip).
            // (tools/serial_sweep.sh on the c_raytracer, C1 and RTOW frames: L 2048
            // -> 103 / 9 / 126 ms, 4096 -> 71 / 7 / 85, 16384 -> 56 / 6 / 61, 65536 ->
            // 72 / 6 / 64; z 1.0 / 1.5 / 2.0 within 5 %: short iterations pay the
            // launch tail, long ones the sqrt(L) wider windows)
            const double spread = std::sqrt((double)Lw * (1.0 + 1.0 / (double)(spp * R)));
            K = (uint64_t)std::ceil(2.0 * z * sigma * spread) + 2 * (uint64_t)depth + 2;
            if (const uint64_t k = env_u64("RT_AMD_SERIAL_K", 0)) K = k;  // (tests: narrow windows)
            // sample a + 1's window must hold every b of sample a: K >= 2 depth + 2
            K = std::min<uint64_t>(std::max<uint64_t>(K, 2 * (uint64_t)depth + 2), (uint64_t)depth * L + 1);
            if (L * K > 0x7FFFFFFFull) {
                set_error("RT_RNG_SERIAL: candidate table too large");
                return -5;
            }
            // (the coalescing workgroup keeps K candidates' u16 slots and K + depth
            // + 1 live offsets in LDS, <= 64 KB: wider windows take the count pass)
            if (K > 4096 || serial_coalesce_search_lds((uint32_t)K, depth) > 64 * 1024) coalesce = false;
            // the pixel table's bounds (64-bit: no wrap before the checks): pixels an
            // iteration touches x the widest span of positions one pixel's windows cover
            npq_max = L / spp + 2;
            emax = pixtab ? serial_pixtab_emax64(spp, K, depth) : 0;
            // (rows padded to whole job chunks of the pixel pass: render_frame's chunk)
            if (pixtab && use_spix) emax = (emax + pchunk - 1) / pchunk * pchunk;
            if (!pixtab || (npq_max * emax <= (1ull << 28) && emax <= 0x7FFFFFFFull)) break;
            // too large: plan the iterations as without the pixel table (L, and
            // with it K and the reach; the coalescing search where the rule picks it)
            pixtab = false;
            plan();
            HIP_TRY(hipMemsetAsync(sums + 1, 0, sizeof(double), s));  // (the reach: atomicMax)
        }
        // the block walks read the pixel table directly (RT_AMD_SERIAL_PGATHER=1:
        // through a gathered L x K count table instead, the first build: 27 us per
        // iteration more at 32 k x 617)
        const bool pgather = pixtab && env_u64("RT_AMD_SERIAL_PGATHER", 0) != 0;
        if (pixtab) {
            HIP_TRY(grow(d->sptab, d->sptab_cap, npq_max * emax));
            HIP_TRY(grow(d->sspix, d->sspix_cap, 2 * npq_max));
            if (reuse) HIP_TRY(grow(d->sptab2, d->sptab2_cap, npq_max * emax));
            if (pgather) HIP_TRY(grow(d->samples, d->samples_cap, L * K));
        }
        // The walks size each iteration's windows from the per-pixel variances
        // (V: prefix sums over pixels of spp var, then var; the variance of
        // samples [0, j) is PV[p] + (j - p spp) var[p]): 2 z (sqrt(V) + 0.05
        // sqrt(n scale)) + 2 depth + 2 for n samples -- the frame-wide K above
        // where every pixel has the frame's sigma, narrower over sky and other
        // constant-count pixels
        const bool adapt = env_u64("RT_AMD_SERIAL_ADAPT", 1) != 0;
        const double *Vdev = d->stab + 2 * npix + 1;
        const uint64_t wlen = 2 * L + 3 * ((uint64_t)std::ceil(dmax) + K + (uint64_t)depth) + 8;
        if (wlen >= 0xFFFFFFFFull) {
            set_error("RT_RNG_SERIAL: candidate window too large");
            return -5;
        }
        // block length: the count pass's walks use serial_walk_block(L) (256
        // blocks); the coalescing search RT_AMD_SERIAL_R samples (default 32,
        // <= kMaxWalkBlocks blocks per iteration)
        // (the pixel table's walks: blocks of 64 samples up to 48 k-sample
        // iterations, then about 768 blocks per iteration -- 128 samples at 64
        // spp's 96 k: RTOW at C2 settings 665 -> 645 ms, world.txt unchanged)
        uint64_t walk_r_def = 64;
        while (walk_r_def < kMaxWalkR && L > walk_r_def * 768) walk_r_def *= 2;
        const uint64_t R_walk =
            coalesce ? std::min<uint64_t>(L, std::max<uint64_t>({env_u64("RT_AMD_SERIAL_R", 32), 1,
                                                                 (L + kMaxWalkBlocks - 1) / kMaxWalkBlocks}))
            : pixtab ? std::min<uint64_t>(L, std::max<uint64_t>({env_u64("RT_AMD_SERIAL_WALKR", walk_r_def), 1,
                                                                 (L + kMaxWalkBlocks - 1) / kMaxWalkBlocks}))
                     : serial_walk_block((uint32_t)L);
        // the pixel table's walks read each block's rows from LDS (as u8 counts:
        // depth < 255) when a block's pixels x the row stride fit the budget
        // (RT_AMD_SERIAL_WALK_LDS=0: the walks read the table in global memory)
        uint32_t walk_lds = 0;
        if (pixtab && !pgather && depth < 255 && R_walk <= kMaxWalkR &&
            env_u64("RT_AMD_SERIAL_WALK_LDS", 1) != 0) {
            const uint64_t maxpix = (R_walk - 1) / spp + 2;
            if (maxpix <= kWalkLdsMaxPix && maxpix * emax <= kWalkLdsRowBytes) walk_lds = (uint32_t)(maxpix * emax);
        }
        uint32_t K0 = 0;  // the first iteration's candidates (later ones: the walks)
        if (adapt) {
            const double w0 = 2.0 * z * (std::sqrt(std::max(sm[2], 0.0)) + serial_floor(spp * R) * std::sqrt((double)n0));
            K0 = (uint32_t)std::min<double>((double)K, std::ceil(w0) + 2.0 * depth + 2.0);
        }
        HIP_TRY(grow(d->swin, d->swin_cap, wlen));
        HIP_TRY(grow(d->slo, d->slo_cap, L));
        HIP_TRY(grow(d->sbend, d->sbend_cap, (L + R_walk - 1) / R_walk * K));
        HIP_TRY(grow(d->ssb, d->ssb_cap, (L + R_walk - 1) / R_walk * K));
        HIP_TRY(grow(d->ssbend, d->ssbend_cap, serial_super_words((uint32_t)L, (uint32_t)K, (uint32_t)R_walk)));
        // recorded block paths: the states of resolved samples become a gather
        // (the coalescing search has no count table to re-walk: always)
        const bool gather = coalesce || pixtab || env_u64("RT_AMD_SERIAL_GATHER", 1) != 0;
        if (gather) {
            HIP_TRY(grow(d->spath, d->spath_cap, (L + R_walk - 1) / R_walk * R_walk * K));
            if (!d->sfin) HIP_TRY(hipMalloc((void **)&d->sfin, kWalkFinWords * 4));
        }
        if (!d->sjump) {
            const std::vector<uint32_t> jt = xorshift_jump_table();
            HIP_TRY(hipMalloc((void **)&d->sjump, jt.size() * 4));
            HIP_TRY(hipMemcpy(d->sjump, jt.data(), jt.size() * 4, hipMemcpyHostToDevice));
        }
        if (!d->sctrl) HIP_TRY(hipMalloc((void **)&d->sctrl, 64));
        // Random::new() (random.rs:8-10); words 8-11: the previous iteration (reuse)
        const uint32_t ctrl0[16] = {0u, o.seed, 0u, 0u, 0u, K0, 0u, 0u, 0u, 0u, 0u, 0u, 0u, 0u, 0u, 0u};
        HIP_TRY(hipMemcpyAsync(d->sctrl, ctrl0, 64, hipMemcpyHostToDevice, s));
        uint64_t iter_q = 0;  // iterations queued (table / span buffers alternate)
        // iterations are queued in batches sized by the expected progress;
        // those queued past the end exit at once (ctrl[0])
        uint32_t ctrl[8] = {0, 0, 0, 0, 0, 0, 0, 0};
        double t_enqueue = 0, t_wait = 0;  // (RT_AMD_SERIAL_DEBUG)
        hipEvent_t dbg_ev[2] = {nullptr, nullptr};
        unsigned long long *dbg_cnt = nullptr;  // (coalescing search counters)
        if (env_u64("RT_AMD_SERIAL_DEBUG", 0)) {
            for (auto &e : dbg_ev) HIP_TRY(hipEventCreate(&e));
            HIP_TRY(hipEventRecord(dbg_ev[0], s));
            HIP_TRY(hipMalloc((void **)&dbg_cnt, 4 * 8));
            HIP_TRY(hipMemsetAsync(dbg_cnt, 0, 4 * 8, s));
        }
        const double t_prep = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - tp0).count();
        uint64_t queued = 0;
        while (!ctrl[0]) {
            const uint64_t left = N - ctrl[4];
            const uint64_t it = std::max<uint64_t>(2, (uint64_t)std::ceil((double)left / (0.8 * (double)L)));
            if ((queued += it) > N + 64) {  // (every iteration resolves >= 1 sample)
                set_error("RT_RNG_SERIAL: start states not resolved");
                return -5;
            }
            const auto t0 = std::chrono::steady_clock::now();
            for (uint64_t q = 0; q < it; ++q, ++iter_q) {
                // this iteration's table and spans, and the previous iteration's
                // (reuse: the two alternate)
                const bool odd = reuse && (iter_q & 1u);
                float *const ptab = odd ? d->sptab2 : d->sptab;
                float *const ptab_prev = reuse ? (odd ? d->sptab : d->sptab2) : nullptr;
                uint4 *const spix = d->sspix + (odd ? npq_max : 0);
                const uint4 *const spix_prev = reuse ? d->sspix + (odd ? 0 : npq_max) : nullptr;
                // (the pixel table pass's job counters are zeroed by the window kernel)
                HIP_TRY(launch_serial_window(d->sctrl, d->sjump, d->swin, (uint32_t)wlen, pred, d->slo,
                                             (uint32_t)L, (uint32_t)K, depth, (uint32_t)N,
                                             pixtab ? (uint32_t)spp : 0u, (uint32_t)emax,
                                             pixtab ? d->counter : nullptr, kPixtabParts,
                                             pixtab && use_spix ? spix : nullptr,
                                             (uint32_t)pchunk, spix_prev, s));
                if (pixtab) {
                    if (reuse)
                        HIP_TRY(launch_serial_reuse(d->sctrl, spix, spix_prev, ptab, ptab_prev, (uint32_t)npq_max,
                                                    (uint32_t)spp, (uint32_t)L, (uint32_t)N, s));
                    SerialPass sp{kRngSerialPixel, 0u, (uint32_t)npq_max, (uint32_t)emax, d->swin, pred, d->sctrl,
                                  d->slo};
                    sp.ptab = ptab;
                    sp.spix = use_spix ? spix : nullptr;
                    sp.L = (uint32_t)L;
                    sp.Kmax = (uint32_t)K;
                    rc = render_frame(w, cam, width, height, ob, nullptr, s, nullptr, &sp);
                    if (rc) return rc;
                    if (pgather)
                        HIP_TRY(launch_serial_pixtab_gather(d->sctrl, ptab, d->slo, d->samples, (uint32_t)L,
                                                           (uint32_t)K, (uint32_t)spp, (uint32_t)N, s));
                } else {
                    SerialPass sp{coalesce ? kRngSerialCoalesce : kRngSerialCount, 0u, (uint32_t)L, (uint32_t)K,
                                  d->swin, pred, d->sctrl, d->slo};
                    sp.path = d->spath;
                    sp.bend = d->sbend;
                    sp.R = (uint32_t)R_walk;
                    sp.dbg = dbg_cnt;
                    rc = render_frame(w, cam, width, height, ob, nullptr, s, nullptr, &sp);
                    if (rc) return rc;
                }
                HIP_TRY(launch_serial_walk(d->sctrl, (coalesce || (pixtab && !pgather)) ? nullptr : d->samples, pred,
                                           adapt ? Vdev : nullptr, (uint32_t)npix, (uint32_t)spp, (float)z,
                                           (float)serial_floor(spp * R), d->swin, d->sstates, d->sbend,
                                           gather ? d->spath : nullptr, gather ? d->sfin : nullptr, d->slo,
                                           d->ssbend, d->ssb, (uint32_t)L, (uint32_t)Lw, (uint32_t)K,
                                           (uint32_t)R_walk, depth, (uint32_t)N,
                                           (pixtab && !pgather) ? ptab : nullptr, walk_lds, s));
            }
            const auto t1 = std::chrono::steady_clock::now();
            HIP_TRY(hipMemcpyAsync(ctrl, d->sctrl, 32, hipMemcpyDeviceToHost, s));
            HIP_TRY(hipStreamSynchronize(s));
            const auto t2 = std::chrono::steady_clock::now();
            t_enqueue += std::chrono::duration<double, std::milli>(t1 - t0).count();
            t_wait += std::chrono::duration<double, std::milli>(t2 - t1).count();
        }
        if (stats) {
            stats->serial_retries = ctrl[6];
            stats->serial_iterations = ctrl[3];
        }
        final_state = ctrl[1];
        if (dbg_ev[0]) {
            HIP_TRY(hipEventRecord(dbg_ev[1], s));
            HIP_TRY(hipEventSynchronize(dbg_ev[1]));
            float a = 0, b = 0;
            HIP_TRY(hipEventElapsedTime(&a, d->sev[0], dbg_ev[0]));
            HIP_TRY(hipEventElapsedTime(&b, dbg_ev[0], dbg_ev[1]));
            std::fprintf(stderr, "serial debug: GPU estimate + tables %.1f ms, iterations %.1f ms\n", a, b);
            for (auto &e : dbg_ev) (void)hipEventDestroy(e);
            unsigned long long c[4] = {0, 0, 0, 0};
            HIP_TRY(hipMemcpy(c, dbg_cnt, sizeof(c), hipMemcpyDeviceToHost));
            HIP_TRY(hipFree(dbg_cnt));
            if (coalesce && c[2])
                std::fprintf(stderr, "serial debug: coalesce %llu traces in %llu blocks (%.3f of the count pass's "
                             "%llu), %.1f trace passes per block\n", c[0], c[2], (double)c[0] / std::max(1.0, (double)c[3]),
                             c[3], (double)c[1] / (double)c[2]);
        }
        if (env_u64("RT_AMD_SERIAL_DEBUG", 0) && pixtab) {
            // the pixel table pass's idle jobs: per iteration every pixel's row is E
            // (the widest span) long, a pixel's own span ~ 2 (spp - 1) + 3 (K - 1) +
            // 3 (spp - 1) mu (its predicted scatters)
            std::vector<double> mu(npix);
            HIP_TRY(hipMemcpy(mu.data(), d->stab + npix + 1, npix * sizeof(double), hipMemcpyDeviceToHost));
            const uint64_t npq = std::max<uint64_t>(1, L / spp);
            double used = 0, padded = 0;
            for (uint64_t q0 = 0; q0 < npix; q0 += npq) {
                double mx = 0, sum = 0;
                const uint64_t q1 = std::min(npix, q0 + npq);
                for (uint64_t q = q0; q < q1; ++q) {
                    const double sp = 2.0 * (spp - 1) + 3.0 * (K - 1) + 3.0 * (spp - 1) * mu[q] + 1;
                    mx = std::max(mx, sp);
                    sum += sp;
                }
                used += sum;
                padded += mx * (double)(q1 - q0);
            }
            std::fprintf(stderr, "serial debug: pixel table spans use %.3f of the npq x E jobs (K %llu)\n",
                         used / std::max(padded, 1.0), (unsigned long long)K);
        }
        if (env_u64("RT_AMD_SERIAL_DEBUG", 0)) {
            std::fprintf(stderr, "serial debug: %s N %llu L %llu R %llu K %llu sigma %.3f: %u iterations (%u "
                         "stopped short), %llu queued, estimate + tables %.1f ms, enqueue %.1f ms, wait %.1f ms\n",
                         pixtab ? "pixel table" : coalesce ? "coalesce" : "count", (unsigned long long)N,
                         (unsigned long long)L,
                         (unsigned long long)R_walk, (unsigned long long)K, sigma,
                         ctrl[3], ctrl[6], (unsigned long long)queued, t_prep, t_enqueue, t_wait);
        }
    }
    HIP_TRY(hipEventRecord(d->sev[1], s));
    if (N > 0 && (o.flags & RT_FLAG_SERIAL_CHECK)) {
        // the chain the reference's one stream forms (common.rs:321-341):
        // sample 0 starts at the seed, sample j ends where j + 1 starts,
        // the last one where the search ended (ctrl[1])
        // the states the check traces: d->sstates, or (test hook) a scratch
        // copy with one state corrupted, so the check must see the links into
        // and out of that sample break while the frame still renders from the
        // states the search found
        const uint32_t *checked = d->sstates;
        uint32_t *broken = nullptr;
        if (const char *brk = std::getenv("RT_AMD_SERIAL_BREAK")) {
            const uint64_t j = std::strtoull(brk, nullptr, 10);
            if (j < N) {
                HIP_TRY(hipMalloc((void **)&broken, N * 4));
                HIP_TRY(hipMemcpyAsync(broken, d->sstates, N * 4, hipMemcpyDeviceToDevice, s));
                uint32_t x = 0;
                HIP_TRY(hipMemcpyAsync(&x, broken + j, 4, hipMemcpyDeviceToHost, s));
                HIP_TRY(hipStreamSynchronize(s));
                x = x == 1u ? 2u : 1u;
                HIP_TRY(hipMemcpyAsync(broken + j, &x, 4, hipMemcpyHostToDevice, s));
                HIP_TRY(hipStreamSynchronize(s));
                checked = broken;
            }
        }
        struct FreeScratch {
            uint32_t *p;
            ~FreeScratch() { if (p) (void)hipFree(p); }
        } free_broken{broken};
        uint32_t first = 0;
        HIP_TRY(hipMemcpyAsync(&first, checked, 4, hipMemcpyDeviceToHost, s));
        if (!d->scheck) HIP_TRY(hipMalloc((void **)&d->scheck, 8));
        HIP_TRY(hipMemsetAsync(d->scheck, 0, 8, s));
        const uint64_t step = 1ull << 28;
        for (uint64_t c0 = 0; c0 < N; c0 += step) {
            const uint32_t n = (uint32_t)std::min(step, N - c0);
            const SerialPass sp{kRngSerialCheck, (uint32_t)c0, n, 1u, checked, SerialPred{}, nullptr};
            RtRenderOptions oc = ob;
            oc.seed = final_state;
            rc = render_frame(w, cam, width, height, oc, nullptr, s, nullptr, &sp);
            if (rc) return rc;
            HIP_TRY(launch_serial_check_count(d->samples, n, d->scheck, s));
        }
        unsigned long long breaks = 0;
        HIP_TRY(hipMemcpyAsync(&breaks, d->scheck, 8, hipMemcpyDeviceToHost, s));
        HIP_TRY(hipStreamSynchronize(s));
        if (stats) {
            stats->serial_checked = N;
            stats->serial_chain_breaks = breaks + (first != o.seed ? 1u : 0u);
        }
    }
    return 0;
}

int render_frame_serial(WorldState &w, const CameraModel &cam, size_t width, size_t height,
                        const RtRenderOptions &o, uint32_t *d_out, hipStream_t stream,
                        RtRenderStats *stats) {
    if (stats) std::memset(stats, 0, sizeof(*stats));
    if (width == 0 || height == 0) return 0;
    int rc = serial_check_args(width, height, o);
    if (rc) return rc;
    std::lock_guard<std::recursive_mutex> lock(w.mu);
    DeviceState *d = nullptr;
    rc = device_for(w, o.device, d);
    if (rc) return rc;
    hipStream_t s = stream ? stream : d->stream;
    rc = serial_find_states(w, cam, width, height, o, d, s, stats);
    if (rc) return rc;
    const uint64_t N = (uint64_t)width * height * (uint64_t)std::max(o.samples_per_pixel, 0);
    // 3. the frame (or rank's tile) from the start states
    RtRenderOptions orp = o;
    orp.rng_mode = RT_RNG_REPLAY;
    orp.replay_states = nullptr;
    RtRenderStats keep{};
    if (stats) keep = *stats;
    rc = render_frame(w, cam, width, height, orp, d_out, s, stats, nullptr, d->sstates);
    if (rc) return rc;
    if (stats) {
        stats->serial_retries = keep.serial_retries;
        stats->serial_iterations = keep.serial_iterations;
        stats->serial_checked = keep.serial_checked;
        stats->serial_chain_breaks = keep.serial_chain_breaks;
        float ms = 0.0f;
        HIP_TRY(hipEventSynchronize(d->sev[1]));
        HIP_TRY(hipEventElapsedTime(&ms, d->sev[0], d->sev[1]));
        stats->serial_ms = ms;
        if (N > 0) {
            HIP_TRY(hipEventElapsedTime(&ms, d->sev[0], d->sev[2]));
            stats->serial_setup_ms = ms;
        }
    }
    return 0;
}

long read_samples(WorldState &w, int device, float *out, size_t n) {
    std::lock_guard<std::recursive_mutex> lock(w.mu);  // (device_for may add a device)
    DeviceState *d = nullptr;
    int rc = device_for(w, device, d);
    if (rc) return rc;
    if (d->last_fused) {
        set_error("rt_read_samples: the last launch resolved in the trace kernel "
                  "(render with RT_FLAG_KEEP_SAMPLES to keep the samples)");
        return -1;
    }
    const size_t count = std::min(n / 4, d->last_jobs);
    if (!count) return 0;
    HIP_TRY(hipDeviceSynchronize());
    std::vector<float> planes(3 * d->last_jobs);
    for (int c = 0; c < 3; ++c)
        HIP_TRY(hipMemcpy(planes.data() + c * d->last_jobs, d->samples + c * d->last_jobs,
                          d->last_jobs * sizeof(float), hipMemcpyDeviceToHost));
    // (r, g, b, 0) per sample, as documented: sample-major order (s * npix +
    // pixel) from the pixel-major slab (pixel * spp + s)
    const size_t spp = std::max<size_t>(1, d->last_spp), npix = d->last_jobs / spp;
    for (size_t i = 0; i < count; ++i) {
        const size_t src = (i % npix) * spp + i / npix;
        out[4 * i] = planes[src];
        out[4 * i + 1] = planes[d->last_jobs + src];
        out[4 * i + 2] = planes[2 * d->last_jobs + src];
        out[4 * i + 3] = 0.0f;
    }
    return (long)(count * 4);
}

#define NCCL_TRY(expr)                                                                \
    do {                                                                              \
        ncclResult_t r_ = (expr);                                                     \
        if (r_ != ncclSuccess) {                                                      \
            set_error(std::string(#expr) + " failed: " + ncclGetErrorString(r_));     \
            return -4;                                                                \
        }                                                                             \
    } while (0)

namespace {
// RCCL communicators, one set per device list (ncclCommInitAll is expensive:
// created once per process and kept; map nodes are stable)
std::mutex g_comm_mu;
std::map<std::vector<int>, std::vector<ncclComm_t>> g_comms;

int device_comms(const std::vector<int> &devs, std::vector<ncclComm_t> *&out) {
    std::lock_guard<std::mutex> lock(g_comm_mu);
    auto it = g_comms.find(devs);
    if (it == g_comms.end()) {
        std::vector<ncclComm_t> c(devs.size(), nullptr);
        NCCL_TRY(ncclCommInitAll(c.data(), (int)devs.size(), devs.data()));
        it = g_comms.emplace(devs, std::move(c)).first;
    }
    out = &it->second;
    return 0;
}

int device_list(int first, int n, std::vector<int> &devs) {
    int count = 0;
    if (hipGetDeviceCount(&count) != hipSuccess || count <= 0) {
        set_error("no HIP device available: the MI355X render path requires a GPU");
        return -3;
    }
    if (first < 0) HIP_TRY(hipGetDevice(&first));
    if (n < 1 || first + n > count) {
        set_error("ndevices: devices [" + std::to_string(first) + ", " + std::to_string(first + n) +
                  ") are not all visible (" + std::to_string(count) + " devices)");
        return -1;
    }
    devs.resize(n);
    for (int g = 0; g < n; ++g) devs[g] = first + g;
    return 0;
}
}  // namespace

int comm_count(int first, int n) {
    std::vector<int> devs;
    int rc = device_list(first, n, devs);
    if (rc) return rc;
    std::vector<ncclComm_t> *comms = nullptr;
    rc = device_comms(devs, comms);
    if (rc) return rc;
    int ranks = 0;
    NCCL_TRY(ncclCommCount((*comms)[0], &ranks));
    return ranks;
}

int render_frame_multi(WorldState &w, const CameraModel &cam, size_t width, size_t height,
                       const RtRenderOptions &o, uint32_t *d_out, hipStream_t stream,
                       RtRenderStats *stats) {
    if (stats) std::memset(stats, 0, sizeof(*stats));
    if ((o.nranks > 1) || o.rank) {
        set_error("ndevices renders the whole frame: rank/nranks must be 0/1");
        return -1;
    }
    std::lock_guard<std::recursive_mutex> lock(w.mu);
    std::vector<int> devs;
    int rc = device_list(o.device, o.ndevices, devs);
    if (rc) return rc;
    const uint32_t n = (uint32_t)devs.size();
    const uint32_t B = o.row_block ? o.row_block : 8;
    if (width == 0 || height == 0) return 0;
    if (!d_out) { set_error("null output"); return -1; }
    if (width > 0xFFFFFFu || height > 0xFFFFFFu) { set_error("frame too large"); return -1; }
    size_t max_rows = 0;
    for (uint32_t g = 0; g < n; ++g) max_rows = std::max(max_rows, tile_rows(height, B, g, n));
    std::vector<ncclComm_t> *comms = nullptr;
    rc = device_comms(devs, comms);
    if (rc) return rc;
    std::vector<DeviceState *> ds(n, nullptr);
    std::vector<hipStream_t> ss(n, nullptr);
    for (uint32_t g = 0; g < n; ++g) {
        rc = device_for(w, devs[g], ds[g]);
        if (rc) return rc;
        ss[g] = (g == 0 && stream) ? stream : ds[g]->stream;
        if (n > 1) HIP_TRY(grow(ds[g]->tile, ds[g]->tile_cap, max_rows * width));
    }
    if (n > 1) {
        HIP_TRY(hipSetDevice(devs[0]));
        HIP_TRY(grow(ds[0]->gath, ds[0]->gath_cap, n * max_rows * width));
    }
    // SERIAL: the reference's one stream is a sequential dependency, so the
    // start states are found once, on the first device, and broadcast over
    // RCCL; every device then renders its row blocks from them (REPLAY)
    const bool serial = o.rng_mode == RT_RNG_SERIAL;
    RtRenderStats sst{};
    if (serial) {
        rc = serial_check_args(width, height, o);
        if (rc) return rc;
        HIP_TRY(hipSetDevice(devs[0]));
        rc = serial_find_states(w, cam, width, height, o, ds[0], ss[0], stats ? &sst : nullptr);
        if (rc) return rc;
        const uint64_t N = (uint64_t)width * height * (uint64_t)std::max(o.samples_per_pixel, 0);
        if (n > 1 && N > 0) {
            for (uint32_t g = 1; g < n; ++g) {
                HIP_TRY(hipSetDevice(devs[g]));
                HIP_TRY(grow(ds[g]->sstates, ds[g]->sstates_cap, N));
            }
            NCCL_TRY(ncclGroupStart());
            for (uint32_t g = 0; g < n; ++g) {
                const ncclResult_t r = ncclBroadcast(ds[0]->sstates, ds[g]->sstates, N, ncclUint32, 0,
                                                     (*comms)[g], ss[g]);
                if (r != ncclSuccess) {
                    (void)ncclGroupEnd();
                    set_error(std::string("ncclBroadcast failed: ") + ncclGetErrorString(r));
                    return -4;
                }
            }
            NCCL_TRY(ncclGroupEnd());
        }
    }
    // every device renders its row blocks, all enqueued before any host wait:
    // a counted frame leaves its counters pending on its device
    // (render_frame defer_stats) and they are collected once every device's
    // tile is in flight, so counted frames keep the timed frames' schedule
    for (uint32_t g = 0; g < n; ++g) {
        RtRenderOptions og = o;
        og.ndevices = 0;
        og.rank = g;
        og.nranks = n;
        og.row_block = B;
        og.device = devs[g];
        if (serial) {
            og.rng_mode = RT_RNG_REPLAY;
            og.replay_states = nullptr;
        }
        RtRenderStats sg;
        HIP_TRY(hipSetDevice(devs[g]));
        // (one device: its tile is the frame, rendered in place -- no gather)
        rc = render_frame(w, cam, width, height, og, n == 1 ? d_out : ds[g]->tile, ss[g], stats ? &sg : nullptr,
                          nullptr, serial ? ds[g]->sstates : nullptr, /*defer_stats=*/true);
        if (rc) return rc;
    }
    // RCCL gather of equal-size tiles to the first device (over xGMI); with one
    // device the tile was rendered into d_out (until round 5 a one-rank gather
    // copied it there: one RCCL kernel and ~17 us per frame)
    const size_t bytes = max_rows * width * 4;
    if (n > 1) NCCL_TRY(ncclGroupStart());
    for (uint32_t g = 0; g < n && n > 1; ++g) {
        const ncclResult_t r = ncclGather(ds[g]->tile, n > 1 ? (void *)ds[0]->gath : (void *)d_out, bytes,
                                          ncclUint8, 0, (*comms)[g], ss[g]);
        if (r != ncclSuccess) {
            (void)ncclGroupEnd();  // (never leave this thread's group open)
            set_error(std::string("ncclGather failed: ") + ncclGetErrorString(r));
            return -4;
        }
    }
    if (n > 1) NCCL_TRY(ncclGroupEnd());
    HIP_TRY(hipSetDevice(devs[0]));
    if (n > 1)
        HIP_TRY(launch_assemble(ds[0]->gath, d_out, (uint32_t)width, (uint32_t)height, B, n,
                                (uint32_t)max_rows, ss[0]));
    // the tiles and the gather buffer are reused by the next frame on these streams
    for (uint32_t g = 0; g < n; ++g) {
        HIP_TRY(hipSetDevice(devs[g]));
        HIP_TRY(hipEventRecord(ds[g]->done, ss[g]));
        ds[g]->done_stream = ss[g];
    }
    // the counted tiles' counters, collected only now: every device's tile, the
    // gather and the assembly are enqueued before the host waits on any of them
    for (uint32_t g = 0; g < n && stats; ++g) {
        HIP_TRY(hipSetDevice(devs[g]));
        RtRenderStats sg;
        std::memset(&sg, 0, sizeof(sg));
        rc = collect_frame_stats(ds[g], &sg);
        if (rc) return rc;
        {
            stats->samples += sg.samples; stats->rays += sg.rays;
            stats->sphere_tests += sg.sphere_tests; stats->tri_tests += sg.tri_tests;
            stats->tri_in_range += sg.tri_in_range;
            stats->trace_ms = std::max(stats->trace_ms, sg.trace_ms);
            stats->resolve_ms = std::max(stats->resolve_ms, sg.resolve_ms);
            stats->trace_launches = std::max(stats->trace_launches, sg.trace_launches);
            stats->waves += sg.waves; stats->accel = sg.accel;
            stats->bvh_sphere_tests += sg.bvh_sphere_tests; stats->bvh_node_tests += sg.bvh_node_tests;
            stats->big_sphere_tests += sg.big_sphere_tests;
            for (int k = 0; k < 4; ++k) stats->stamp_cycles[k] += sg.stamp_cycles[k];
            stats->tri_node_tests += sg.tri_node_tests; stats->bvh_tri_tests += sg.bvh_tri_tests;
            stats->tri_bvh = sg.tri_bvh; stats->fused_resolve = sg.fused_resolve;
            stats->primary_lists = sg.primary_lists; stats->camera_tree = sg.camera_tree;
            stats->launch_parts = sg.launch_parts; stats->launch_chunk = sg.launch_chunk;
            stats->launch_refill_min = sg.launch_refill_min; stats->launch_walk_min = sg.launch_walk_min;
            stats->launch_tri_walk_min = sg.launch_tri_walk_min; stats->launch_wsteps = sg.launch_wsteps;
            stats->launch_block_threads = sg.launch_block_threads; stats->launch_blocks = sg.launch_blocks;
        }
    }
    HIP_TRY(hipSetDevice(devs[0]));
    if (stats) {
        HIP_TRY(hipStreamSynchronize(ss[0]));
        if (serial) {
            stats->serial_retries = sst.serial_retries;
            stats->serial_iterations = sst.serial_iterations;
            stats->serial_checked = sst.serial_checked;
            stats->serial_chain_breaks = sst.serial_chain_breaks;
            float ms = 0.0f;
            HIP_TRY(hipEventElapsedTime(&ms, ds[0]->sev[0], ds[0]->sev[1]));
            stats->serial_ms = ms;
            if (width * height * (size_t)std::max(o.samples_per_pixel, 0) > 0) {
                HIP_TRY(hipEventElapsedTime(&ms, ds[0]->sev[0], ds[0]->sev[2]));
                stats->serial_setup_ms = ms;
            }
        }
    }
    return 0;
}

int assemble_tiles(const uint32_t *gathered, uint32_t *out, size_t width, size_t height, uint32_t row_block,
                   uint32_t nranks, size_t max_rows, hipStream_t stream) {
    if (width == 0 || height == 0) return 0;
    if (!gathered || !out) { set_error("rt_assemble_tiles: null buffer"); return -1; }
    if (nranks == 0 || row_block == 0) { set_error("rt_assemble_tiles: nranks and row_block must be >= 1"); return -1; }
    if (width > 0xFFFFFFu || height > 0xFFFFFFu) { set_error("frame too large"); return -1; }
    for (uint32_t g = 0; g < nranks; ++g)
        if (tile_rows(height, row_block, g, nranks) > max_rows) {
            set_error("rt_assemble_tiles: max_rows is smaller than a rank's tile");
            return -1;
        }
    HIP_TRY(launch_assemble(gathered, out, (uint32_t)width, (uint32_t)height, row_block, nranks,
                            (uint32_t)max_rows, stream));
    return 0;
}

int render_frame_host(WorldState &w, const CameraModel &cam, size_t width, size_t height,
                      const RtRenderOptions &o, void *host_out, RtRenderStats *stats) {
    std::lock_guard<std::recursive_mutex> lock(w.mu);
    if (o.ndevices >= 1) {
        if (width == 0 || height == 0) {
            if (stats) std::memset(stats, 0, sizeof(*stats));
            return 0;
        }
        if (!host_out) { set_error("null framebuffer pixels"); return -1; }
        std::vector<int> devs;
        int rc = device_list(o.device, o.ndevices, devs);
        if (rc) return rc;
        DeviceState *root = nullptr;
        rc = device_for(w, devs[0], root);
        if (rc) return rc;
        HIP_TRY(grow(root->out, root->out_cap, width * height));
        rc = render_frame_multi(w, cam, width, height, o, root->out, root->stream, stats);
        if (rc) return rc;
        HIP_TRY(hipSetDevice(devs[0]));
        HIP_TRY(hipMemcpyAsync(host_out, root->out, width * height * 4, hipMemcpyDeviceToHost,
                               root->stream));
        HIP_TRY(hipStreamSynchronize(root->stream));
        return 0;
    }
    const uint32_t nranks = o.nranks ? o.nranks : 1;
    const uint32_t B = nranks > 1 ? (o.row_block ? o.row_block : 1) : (uint32_t)std::max<size_t>(height, 1);
    const size_t T = o.rank < nranks ? tile_rows(height, B, o.rank, nranks) : 0;
    if (width == 0 || T == 0) {
        if (stats) std::memset(stats, 0, sizeof(*stats));
        return o.rank < nranks ? 0 : -1;
    }
    if (!host_out) { set_error("null framebuffer pixels"); return -1; }
    DeviceState *d = nullptr;
    int rc = device_for(w, o.device, d);
    if (rc) return rc;
    HIP_TRY(grow(d->out, d->out_cap, T * width));
    rc = render_frame(w, cam, width, height, o, d->out, d->stream, stats);
    if (rc) return rc;
    HIP_TRY(hipMemcpyAsync(host_out, d->out, T * width * 4, hipMemcpyDeviceToHost, d->stream));
    HIP_TRY(hipStreamSynchronize(d->stream));
    return 0;
}

}  // namespace rtamd
