/*
 * raytracer_amd.h -- extensions of the MI355X raytracer library beyond the
 * reference C-ABI (raytracer.h).  Nothing here changes the reference entry
 * points; it exposes what the reference hard-codes (Options, common.rs:288-317,
 * fixed to 16 spp / 8 bounces at lib.rs:51), device-resident rendering for
 * benchmarks, row tiles for multi-GPU, scene introspection and PPM output.
 */
#ifndef RAYTRACER_AMD_H
#define RAYTRACER_AMD_H

#include "raytracer.h"

#ifdef __cplusplus
extern "C" {
#endif

/* RNG modes.  The reference draws every sample from ONE xorshift32 stream
 * seeded 2547549 for the whole frame (common.rs:321, random.rs:8-10), which
 * is a sequential dependency.  The GPU offers:
 *   RT_RNG_SERIAL: that stream, seeded `seed`: the reference's own frame, bit
 *     for bit.  The library finds every sample's start state on the GPU
 *     (chunked candidate tables and walks), then renders as
 *     REPLAY; width*height*spp must be below 2^32.  The default of render().
 *   RT_RNG_COUNTER: sample (pixel p, index s) starts xorshift32 from
 *     rt_sample_seed(seed, p*spp + s); draws inside a sample follow the
 *     reference order exactly.  The fast mode (no sequential dependency);
 *     statistically, not bitwise, equal to the reference.
 *   RT_RNG_REPLAY: sample start states are read from a table (e.g. recorded
 *     from a serial CPU run), which reproduces the serial frame bit-for-bit. */
enum { RT_RNG_COUNTER = 1, RT_RNG_REPLAY = 2, RT_RNG_SERIAL = 3 };

typedef struct RtRenderOptions {
  int32_t samples_per_pixel;      /* Options.samples_per_pixel (common.rs:290) */
  int32_t max_ray_bounces;        /* Options.max_ray_bounces   (common.rs:291) */
  uint32_t rng_mode;              /* RT_RNG_*                                   */
  uint32_t seed;                  /* COUNTER base seed (default 2547549)        */
  const uint32_t *replay_states;  /* REPLAY: host table, width*height*spp u32,
                                     index (row*width + col)*spp + s, row 0 =
                                     bottom (common.rs:327-336 loop order)      */
  uint32_t row_block;             /* multi-GPU tile: image rows are dealt in    */
  uint32_t rank;                  /* blocks of row_block rows, round-robin over */
  uint32_t nranks;                /* nranks; this call renders rank's rows      */
  int32_t device;                 /* HIP device ordinal, -1 = current device    */
  int32_t accel;                  /* RT_ACCEL_*: how World::hit finds spheres   */
  uint32_t flags;                 /* RT_FLAG_* (0 = default)                    */
  int32_t ndevices;               /* 0: one device (`device`), this call renders
                                     rank's tile.  >= 1: the WHOLE frame, row-
                                     tiled (blocks of row_block rows) over
                                     devices [first, first + ndevices), first =
                                     `device` or the current device, in this one
                                     process; an RCCL ncclGather (communicators
                                     from ncclCommInitAll) collects the tiles on
                                     the first device.  rank/nranks must be 0/1. */
} RtRenderOptions;

/* Frame resolve.  By default the trace kernel resolves each pixel itself: a
 * wave keeps its chunks' samples in a small per-wave ring (cache-resident)
 * and sums a pixel's samples in order once its last sample is done, so only
 * the RGBA8 frame reaches HBM.  RT_FLAG_KEEP_SAMPLES writes every sample to a
 * full slab in HBM instead and resolves with a second kernel, which
 * rt_read_samples can then read.  Both give bit-identical frames. */
enum { RT_FLAG_KEEP_SAMPLES = 1 };

/* RT_RNG_SERIAL self-check.  RT_FLAG_SERIAL_CHECK traces every sample once
 * more from the start state found for it and checks the chain the reference's
 * one stream forms (common.rs:321-341): sample 0 starts at the seed, and each
 * sample's end state is the next sample's start state (the last one's: the
 * stream state the search ended on).  Mismatches are counted in
 * RtRenderStats.serial_chain_breaks (0 = the start states are the
 * reference's). */
enum { RT_FLAG_SERIAL_CHECK = 2 };

/* Sphere search.  Both give bit-identical frames:
 *   RT_ACCEL_BRUTE: every sphere in file order (common.rs:241-247).
 *   RT_ACCEL_BVH:   exact-pruning BVHs: spheres (BRUTE below 16 spheres) and
 *                   the phantom-aware triangle tree (BRUTE below 16 triangles).
 *   RT_ACCEL_AUTO:  BVH when the scene has one, else BRUTE.  Default. */
enum { RT_ACCEL_AUTO = 0, RT_ACCEL_BRUTE = 1, RT_ACCEL_BVH = 2 };

typedef struct RtRenderStats {
  uint64_t samples;        /* pixel samples traced                           */
  uint64_t rays;           /* World::hit calls (primary + bounces)           */
  uint64_t sphere_tests;   /* rays * spheres (brute force, common.rs:241)     */
  uint64_t tri_tests;      /* rays * triangles (common.rs:182)               */
  uint64_t tri_in_range;   /* triangle tests that passed the t-range check   */
  double trace_ms;         /* HIP-event time of the trace kernel(s)          */
  double resolve_ms;       /* HIP-event time of the resolve kernel(s)        */
  uint32_t trace_launches; /* number of trace launches (slabs)               */
  uint32_t waves;          /* persistent waves per trace launch              */
  uint32_t accel;          /* RT_ACCEL_BRUTE or RT_ACCEL_BVH (what ran)      */
  uint64_t bvh_sphere_tests; /* sphere tests executed inside the BVH         */
  uint64_t bvh_node_tests;   /* BVH node (box) tests executed                */
  uint64_t big_sphere_tests; /* rays * spheres kept out of the BVH           */
  uint64_t stamp_cycles[4];  /* diagnostic builds (-DRT_STAMPS) only: wave
                                cycles in refill+store / ray setup / BVH
                                walks / shading; zero in the product build             */
  uint64_t tri_node_tests;   /* triangle-BVH node tests executed              */
  uint64_t bvh_tri_tests;    /* triangle tests executed (== tri_tests brute)  */
  uint32_t tri_bvh;          /* 1 when the triangle BVH ran                   */
  uint32_t fused_resolve;    /* 1 when the trace kernel resolved the pixels
                                (no slab, resolve_ms ~ 0)                    */
  double serial_ms;          /* RT_RNG_SERIAL: HIP-event time spent finding the
                                start states (before the REPLAY render)       */
  uint32_t serial_retries;   /* RT_RNG_SERIAL: iterations whose walk stopped
                                short of their samples (the next one resumed) */
  uint32_t primary_lists;    /* 1: primary rays used per-pixel / per-strip
                                candidate lists (0 right after a camera move or
                                resize while they are built on a host thread) */
  uint32_t camera_tree;      /* 1: bounce-0 triangle rays used the camera-origin records (tree or strip lists) */
  uint32_t serial_iterations;   /* RT_RNG_SERIAL: candidate-table iterations run   */
  uint64_t serial_checked;      /* RT_FLAG_SERIAL_CHECK: samples whose chain link
                                   was checked (0 without the flag)             */
  uint64_t serial_chain_breaks; /* RT_FLAG_SERIAL_CHECK: broken links (0 = the
                                   reference's stream)                          */
  double serial_setup_ms;       /* RT_RNG_SERIAL: HIP-event time of the estimate
                                   pass and its tables (part of serial_ms)      */
  /* The frame trace launch's scheduling settings (the last launch of the
   * frame; they decide the schedule, so profiles record them with their
   * counters): job-queue partitions, jobs per queue pull, refill threshold
   * (idle lanes), walk gates (sphere / triangle walks), wide-walk fetches per
   * slice, threads per workgroup and workgroups per launch. */
  uint32_t launch_parts;
  uint32_t launch_chunk;
  uint32_t launch_refill_min;
  uint32_t launch_walk_min;
  uint32_t launch_tri_walk_min;
  uint32_t launch_wsteps;
  uint32_t launch_block_threads;
  uint32_t launch_blocks;
} RtRenderStats;

/* spp 16, depth 8 (lib.rs:51), SERIAL, seed 2547549, one rank, device -1,
 * row_block 8, ndevices 0: render()'s settings.  render() also reads two
 * environment variables: RT_AMD_RNG=counter selects RT_RNG_COUNTER (fast,
 * statistically equal frames) instead of the reference's stream, and
 * RT_AMD_DEVICES=N (N >= 1) row-tiles its frames over N GPUs (in SERIAL mode
 * the first device finds the whole frame's start states -- the stream is one
 * sequential dependency -- and broadcasts them over RCCL; the REPLAY render is
 * split). */
void rt_default_options(RtRenderOptions *opts);

/* Rows of a `height`-row image that belong to `rank` (see RtRenderOptions). */
size_t rt_tile_rows(size_t height, uint32_t row_block, uint32_t rank, uint32_t nranks);
/* Image row (0 = top) of the k-th row of rank's tile. */
size_t rt_tile_row(size_t k, uint32_t row_block, uint32_t rank, uint32_t nranks);

/* Counter-mode seed of global sample `job` (splitmix64 finaliser, nonzero). */
uint32_t rt_sample_seed(uint32_t seed, uint64_t job);

/* Renders `framebuffer` (full image size) with explicit options.  pixels
 * receives rank's tile: rt_tile_rows() rows of `width` pixels, tile row k =
 * image row rt_tile_row(k).  Synchronous.  Returns 0 or a negative error. */
int rt_render_ex(Rust_CFramebuffer framebuffer, const Rust_WorldHandle *handle,
                 const RtRenderOptions *opts, RtRenderStats *stats);

/* Threading: one frame at a time per handle.  Calls from several host threads
 * on one handle are serialised by a lock; frames enqueued on different streams
 * of one device are ordered (the later waits for the earlier: they share the
 * device's scratch). */

/* Same, but the tile is written to DEVICE memory `d_rgba` (rt_tile_rows*width
 * RGBA8; with ndevices >= 1 the whole width*height frame on the first device)
 * on HIP stream `hip_stream` (NULL = the library's stream; with ndevices it is
 * the first device's stream).  The scene
 * stays resident on the device between calls.  With `stats`, returns after the
 * frame is complete (HIP-event timings and counters filled in); with
 * stats == NULL the frame is only enqueued on the stream (no host wait), so
 * consecutive frames and the caller's collectives pipeline -- except in
 * RT_RNG_SERIAL mode, whose start-state search reads its progress back and
 * waits on the host between batches of iterations (the REPLAY render that
 * follows is only enqueued); do not call it inside a stream capture.  Returns
 * 0 or a negative error. */
int rt_render_device(const Rust_WorldHandle *handle, size_t width, size_t height,
                     const RtRenderOptions *opts, void *d_rgba, void *hip_stream,
                     RtRenderStats *stats);

/* Diagnostics: copies the per-sample colours (r, g, b, 0 as 4 f32) of the
 * LAST trace launch on `device` (-1 = current) to host `out` (n floats max).
 * That launch must have been rendered with RT_FLAG_KEEP_SAMPLES.  Output
 * order is sample-major: slot = s*(rows*width) + k*width + col for sample s
 * of tile row k (rows = tile rows of that launch).  Returns the number of
 * floats copied or a negative error. */
long rt_read_samples(const Rust_WorldHandle *handle, int device, float *out, size_t n);

/* Frees a handle from load_world (the reference never frees, lib.rs:42-45). */
void rt_free_world(Rust_WorldHandle *handle);

/* Last error message of this thread ("" if none). */
const char *rt_last_error(void);

/* Host-side scene introspection (no GPU needed). */
size_t rt_world_num_spheres(const Rust_WorldHandle *handle);
size_t rt_world_num_triangles(const Rust_WorldHandle *handle);
/* center(3) radius material(type, r, g, b, a, param) */
int rt_world_sphere(const Rust_WorldHandle *handle, size_t i, float out[10]);
/* v0 v1 v2 normal material(type, r, g, b, a, param) */
int rt_world_triangle(const Rust_WorldHandle *handle, size_t i, float out[18]);
/* Scene editing: replaces sphere / triangle i's material with (type, r, g,
 * b, a, param), type 0 Diffuse, 1 Metal (param = fuzz), 2 Dielectric (param =
 * ir), 3 Emission (materials.rs:7-12, 100-102; the scene grammar cannot
 * produce Emission, parser.rs:175-234).  a must be 1.0 (every reference Color
 * has alpha 1).  The next frame re-uploads the scene.  0 or -1. */
int rt_world_set_sphere_material(Rust_WorldHandle *handle, size_t i, const float material[6]);
int rt_world_set_triangle_material(Rust_WorldHandle *handle, size_t i, const float material[6]);
/* origin, lower_left_corner, horizontal, vertical (camera.rs:8-15) */
void rt_camera_get(const Rust_Camera *camera, float out[12]);
/* ParseError discriminant of the last failed load_world (parser.rs:11-18),
 * 100 = input on which the reference panics, -1 = none. */
int rt_last_parse_error(void);

/* image.rs:59-81: writes an ASCII PPM (P3).  Returns 0 on success. */
int rt_write_ppm(const Rust_CFramebuffer *framebuffer, const char *path);

/* The last step of a multi-device frame (ndevices > 1), on its own: reads
 * `nranks` tiles of `max_rows` rows each from DEVICE memory d_gathered (rank
 * g's tile at row g*max_rows, tile row k = image row rt_tile_row(k), the
 * layout the RCCL gather leaves on the first device) and writes the
 * width x height frame to DEVICE memory d_out, on hip_stream (NULL: the null
 * stream), without waiting.  Lets one GPU check the assembly for any rank
 * count.  Returns 0 or a negative error. */
int rt_assemble_tiles(const void *d_gathered, void *d_out, size_t width, size_t height, uint32_t row_block,
                      uint32_t nranks, size_t max_rows, void *hip_stream);

/* Number of HIP devices visible (0 if the runtime is unavailable). */
int rt_device_count(void);

/* Rank count of the RCCL communicator that multi-device frames (ndevices =
 * n, first device `first`, -1 = current) use; creates it on first use.
 * Returns n, or a negative error (e.g. fewer than first + n devices). */
int rt_comm_count(int first, int n);

#ifdef __cplusplus
}
#endif

#endif /* RAYTRACER_AMD_H */
