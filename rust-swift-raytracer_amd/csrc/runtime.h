// runtime.h -- device-side state of a loaded world and the frame driver.
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>
#include <future>
#include <map>
#include <mutex>
#include <memory>
#include <string>
#include <vector>

#include "bvh.h"
#include "render.h"
#include "scene.h"

struct RtRenderOptions;
struct RtRenderStats;

namespace rtamd {

// The RtRenderStats fields of a counted frame that the host knows when it
// enqueues the frame (the rest come from the device's wave records).
struct RtRenderStatsFixed {
    uint32_t waves = 0, accel = 0, tri_bvh = 0, fused_resolve = 0, primary_lists = 0, camera_tree = 0;
    uint32_t launch_parts = 0, launch_chunk = 0, launch_refill_min = 0, launch_walk_min = 0;
    uint32_t launch_tri_walk_min = 0, launch_wsteps = 0, launch_block_threads = 0, launch_blocks = 0;
    uint32_t nsph = 0, ntri = 0, nbig = 0;
};

void set_error(const std::string &msg);
const std::string &last_error();

// One device's copy of a scene plus the scratch a frame needs.  Buffers grow
// on demand and persist across frames (the interactive flow re-renders the
// same scene with a moved camera, GameView.swift:198-219 / lib.rs:60-63).
struct DeviceState {
    int device = -1;
    hipStream_t stream = nullptr;
    hipEvent_t ev[3] = {nullptr, nullptr, nullptr};
    hipEvent_t sev[3] = {nullptr, nullptr, nullptr};  // SERIAL mode: start, tables done, states found
    float4 *sph_hot = nullptr, *sph_cold = nullptr, *tri_hot = nullptr, *tri_geo = nullptr;
    float *mats = nullptr;
    float4 *sph_shade = nullptr;
    uint32_t *sph_kind = nullptr;
    uint32_t nsph = 0, nsph_padded = 0, ntri = 0;
    float4 *bvh_nodes = nullptr, *bvh_prims = nullptr, *big_hot = nullptr;
    uint32_t *bvh_miss = nullptr, *bvh_prim_id = nullptr, *big_id = nullptr;
    uint16_t *bvh_miss16 = nullptr;
    uint32_t nnodes = 0, nbig = 0, nprims = 0;
    uint4 *tbvh_nodes = nullptr;                                // triangle BVH (bvh.h qnodes)
    float4 *tbvh_tris = nullptr;
    uint32_t *tbvh_loose = nullptr;
    uint32_t tnodes = 0, ttris = 0, tloose = 0;
    uint4 *tw_nodes = nullptr;                                  // its 4-wide image (bvh.h wnodes)
    uint32_t tw_depth = 0;                                      // stack entries per lane
    float *tw_tris = nullptr;                                   // per-cell trees' records (tcells)
    uint4 *cam_nodes = nullptr;                                 // camera-origin triangle BVH
    float4 *cam_tris = nullptr;
    uint32_t cam_nnodes = 0;
    uint64_t cam_version = 0;                                  // WorldState::ctree_version uploaded
    uint32_t *ptl_off = nullptr, *ptl_items = nullptr;         // primary-ray triangle lists
    uint64_t ptl_version = 0;
    uint2 *spl = nullptr;                                       // primary sphere lists
    uint64_t spl_version = 0;
    // primary sphere lists built on the device (render.hip launch_sphere_lists)
    uint2 *gspl = nullptr;           size_t gspl_cap = 0;
    int4 *gspl_rects = nullptr;      size_t gspl_rects_cap = 0;
    uint32_t *gspl_flag = nullptr;   size_t gspl_flag_cap = 0;
    CameraModel gspl_cam{};
    size_t gspl_w = 0, gspl_h = 0;
    bool gspl_built = false, gspl_ok = false;
    size_t lds_bytes = 0;                                      // 0: tree not LDS-stageable
    float *samples = nullptr;        size_t samples_cap = 0;   // sample slab (3 planes)
    float *ring = nullptr;           size_t ring_cap = 0;      // per-wave sample rings (fused resolve)
    uint32_t *out = nullptr;         size_t out_cap = 0;       // RGBA8 tile (host path)
    uint32_t *tile = nullptr;        size_t tile_cap = 0;      // multi-device: this rank's tile
    uint32_t *gath = nullptr;        size_t gath_cap = 0;      // multi-device root: gathered tiles
    hipEvent_t done = nullptr;       // end of the last frame enqueued on this device ...
    hipStream_t done_stream = nullptr;  // ... and the stream it was enqueued on
    uint32_t *replay = nullptr;      size_t replay_cap = 0;
    // SERIAL mode (render_frame_serial): start states, candidate offsets, the
    // stream window of a chunk, xorshift jump matrices, control block
    uint32_t *sstates = nullptr;     size_t sstates_cap = 0;
    double *stab = nullptr;          size_t stab_cap = 0;   // prediction tables (render.h serial_tab_doubles)
    double *sscan = nullptr;         size_t sscan_cap = 0;  // their scan's scratch
    uint32_t *slo = nullptr;         size_t slo_cap = 0;    // an iteration's window bases (launch_serial_window)
    uint32_t *ssbend = nullptr;      size_t ssbend_cap = 0; // superblock ends and block starts (launch_serial_walk)
    uint32_t *ssb = nullptr;         size_t ssb_cap = 0;
    uint32_t *swin = nullptr;        size_t swin_cap = 0;
    uint32_t *sbend = nullptr;       size_t sbend_cap = 0;
    uint32_t *spath = nullptr;       size_t spath_cap = 0;  // block walks' paths (L x K)
    float *sptab = nullptr;          size_t sptab_cap = 0;  // pixel table pass: b per (pixel, position)
    uint4 *sspix = nullptr;          size_t sspix_cap = 0;  // pixel table pass: spans per pixel, 2 buffers
    float *sptab2 = nullptr;         size_t sptab2_cap = 0; // (the previous iteration's table: reuse)
    uint32_t *sfin = nullptr;                               // chain result (4 + kMaxWalkBlocks)
    uint32_t *sjump = nullptr;
    uint32_t *sctrl = nullptr;
    unsigned long long *scheck = nullptr;                       // chain-check count
    uint32_t *counter = nullptr;                                // job counters: 2 sets of kMaxParts
    uint32_t cset = 0;              // the set the next frame launch uses ...
    bool cset_clean[2] = {false, false};  // ... and whether each set is known to be zero
    unsigned long long *stats = nullptr; size_t stats_cap = 0;  // per-wave counter records
    // resident workgroups per CU of each kernel variant, [0]: whole walks, [1]: sliced walks
    // [count][step]: workgroups per CU of each kernel instance
    int blocks_per_cu[3][2] = {}, blocks_per_cu_bvh[3][2] = {}, blocks_per_cu_lds[3][2] = {};
    int num_cus = 0;
    // a counted frame's timing events (3 per launch: start, trace end, resolve
    // end) and its wave records copied to pinned host memory; with
    // render_frame(..., defer_stats) the host collects them later
    // (collect_frame_stats), so several devices' counted frames run at once
    std::vector<hipEvent_t> tev;
    unsigned long long *hrec = nullptr; size_t hrec_cap = 0;
    struct PendingStats {
        bool active = false;
        size_t nrec = 0;          // records (waves x kStatSlots) in hrec
        uint32_t nslab = 0;       // event triples in tev (one per slab)
        uint32_t launches = 0;    // trace launches
        uint64_t samples = 0;
        bool use_bvh = false, use_tbvh = false;
        RtRenderStatsFixed fixed; // the fields known before the frame ran
        hipStream_t stream = nullptr;
    } pend;
    size_t last_jobs = 0;                                       // jobs of the last launch
    size_t last_spp = 0;                                        // and its spp
    bool last_fused = false;                                    // it resolved in-kernel (no slab)
    ~DeviceState();
};

struct WorldState {
    SceneModel scene;
    PackedScene packed;
    SphereBVH bvh;
    TriangleBVH tbvh;
    TriangleCells tcells;  // per-origin-cell trees (RT_AMD_TRI_CELLS), usually empty
    CameraTriangleBVH ctree;      // for the camera origin of ctree_version
    uint64_t ctree_version = 0;   // 0: none built
    bool ctree_full = false;      // ctree has its nodes (else records only)
    PrimaryTriLists ptl;          // for ptl_cam at ptl_w x ptl_h (and ctree_version)
    CameraModel ptl_cam{};
    size_t ptl_w = 0, ptl_h = 0;
    uint64_t ptl_ctree = 0, ptl_version = 0;
    PrimarySphereLists spl;       // for spl_cam at spl_w x spl_h
    CameraModel spl_cam{};
    size_t spl_w = 0, spl_h = 0;
    uint64_t spl_version = 0;
    // Primary sphere lists for a new camera or size are built on a host thread
    // while frames render without them (same pixels); adopted by the first
    // frame after the build is done.  (Declared after the structures the
    // build reads: a pending future's destructor waits for its build.)
    struct SplJob { std::future<PrimarySphereLists> f; CameraModel cam{}; size_t w = 0, h = 0; };
    SplJob spl_job;
    std::map<int, std::unique_ptr<DeviceState>> devices;
    // one frame at a time per handle: calls from several host threads are
    // serialised here (render_frame_multi re-enters render_frame)
    std::recursive_mutex mu;
};

// One launch of a SERIAL-mode pass (render_frame_serial): the frame's jobs are
// replaced by nsamples x variants jobs starting at frame sample cbase, each
// storing its sample's diffuse/metal scatter count to plane 0 of the slab
// (DeviceState::samples) instead of a colour (render.h kRngSerial*).
struct SerialPass {
    uint32_t mode;            // kRngSerialCount or kRngSerialEstimate
    uint32_t cbase, nsamples, variants;
    const uint32_t *win;
    SerialPred M;
    const uint32_t *ctrl;
    const uint32_t *lo;       // kRngSerialCount (optional): tabulated window bases
    // kRngSerialCoalesce: the block walks' outputs (launch_serial_coalesce),
    // iteration length (nsamples), candidates (variants) and block length R
    uint32_t *path = nullptr, *bend = nullptr;
    uint32_t R = 0;
    unsigned long long *dbg = nullptr;  // (RT_AMD_SERIAL_DEBUG: launch_serial_coalesce's counters)
    // kRngSerialPixel: the table it writes (nsamples pixels x variants
    // positions, the launch's bounds), the iteration length and its K
    float *ptab = nullptr;
    uint32_t L = 0, Kmax = 0;
    const uint4 *spix = nullptr;  // its pixels' position spans (serial_window_kernel)
};

// Renders rank's tile of a width x height frame into device memory d_out
// (RGBA8 words, tile row-major).  stream may be null (library stream).
// sp: launch that SERIAL pass instead (d_out unused).  d_replay: REPLAY from
// this device-resident start-state table (frame sample order).
// defer_stats (with stats): the counted frame is only enqueued, and its
// counters and times are left pending on its device until
// collect_frame_stats(device state) fills stats.
int render_frame(WorldState &w, const CameraModel &cam, size_t width, size_t height,
                 const RtRenderOptions &opts, uint32_t *d_out, hipStream_t stream,
                 RtRenderStats *stats, const SerialPass *sp = nullptr,
                 const uint32_t *d_replay = nullptr, bool defer_stats = false);
// Waits for device d's pending counted frame and fills stats from it.
int collect_frame_stats(DeviceState *d, RtRenderStats *stats);

// RT_RNG_SERIAL: the reference's single frame-wide xorshift32 stream
// (common.rs:321).  Finds every sample's start state on the device (chunked
// candidate tables + walks), then renders in REPLAY mode.
int render_frame_serial(WorldState &w, const CameraModel &cam, size_t width, size_t height,
                        const RtRenderOptions &opts, uint32_t *d_out, hipStream_t stream,
                        RtRenderStats *stats);

// A frame row-tiled over opts.ndevices devices (first = opts.device, or the
// current device) in this one process: each device renders its row blocks
// (blocks of opts.row_block rows, round-robin) into its own tile, an RCCL
// ncclGather (communicators from ncclCommInitAll, cached per device list)
// collects the tiles on the first device, and assemble_kernel writes the
// frame to d_out there (width x height RGBA8, top row first).  stream (may be
// null) is a stream of the first device; the others use their library streams.
int render_frame_multi(WorldState &w, const CameraModel &cam, size_t width, size_t height,
                       const RtRenderOptions &opts, uint32_t *d_out, hipStream_t stream,
                       RtRenderStats *stats);

// assemble_kernel on its own (rt_assemble_tiles): checks the arguments
// against the tile layout of tile_rows / tile_row, then launches.
int assemble_tiles(const uint32_t *gathered, uint32_t *out, size_t width, size_t height, uint32_t row_block,
                   uint32_t nranks, size_t max_rows, hipStream_t stream);

// Ranks of the cached RCCL communicator of devices [first, first + n)
// (created on first use), or a negative error.
int comm_count(int first, int n);

// Same, into host memory (the reference's synchronous render(), lib.rs:49-57).
int render_frame_host(WorldState &w, const CameraModel &cam, size_t width, size_t height,
                      const RtRenderOptions &opts, void *host_out, RtRenderStats *stats);

// (Re)builds the camera-origin triangle tree when the origin changed
// (load_world, move_camera_position, or a render with another camera).
void prepare_camera(WorldState &w, const CameraModel &cam, bool tree = false);

long read_samples(WorldState &w, int device, float *out, size_t n);

size_t tile_rows(size_t height, uint32_t row_block, uint32_t rank, uint32_t nranks);
size_t tile_row(size_t k, uint32_t row_block, uint32_t rank, uint32_t nranks);

}  // namespace rtamd
