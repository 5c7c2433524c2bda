/*
 * rt_oracle.h -- C API of the CPU oracle (TEST INFRASTRUCTURE ONLY).
 *
 * The oracle is a strict-IEEE binary32 C++ restatement of the reference
 * raytracer crate's render path (Naxaes/Rust-Swift-Raytracer,
 * raytracer/src/{random,maths,color,camera,common,materials,parser,image}.rs).
 * Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may load
 * it, and only as the checker / CPU baseline -- never as the product.
 *
 * Parity status: the reference is Rust and no Rust toolchain exists in this
 * pipeline, so no reference output can be produced.  The oracle is pinned by
 * the reference's own known-answer tests (maths.rs:243-286 reflect/refract/
 * negate), by the xorshift32 stream (random.rs:22-30), and cross-checked
 * bit-for-bit against a second, independent numpy-float32 restatement
 * (tests/pyref.py).  Full-frame output is "parity unpinned" by the reference.
 */
#ifndef RT_ORACLE_H
#define RT_ORACLE_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* RNG modes.  SERIAL is the reference's semantics: ONE xorshift32 stream for
 * the whole frame (common.rs:321).  COUNTER seeds every (pixel, sample) from
 * ro_sample_seed().  REPLAY takes each sample's start state from a table. */
enum { RO_RNG_SERIAL = 0, RO_RNG_COUNTER = 1, RO_RNG_REPLAY = 2 };

typedef struct ro_stats {
    uint64_t samples;        /* W*H*spp actually traced                     */
    uint64_t rays;           /* World::hit calls (common.rs:268)            */
    uint64_t sphere_tests;   /* Sphere::hit calls                           */
    uint64_t tri_tests;      /* Triangle::intersect calls                   */
    uint64_t tri_in_range;   /* triangle tests that passed the t-range test */
} ro_stats;

typedef struct ro_scene ro_scene;

/* parser.rs:336-381.  Returns NULL on a parse error (the reference panics). */
ro_scene *ro_parse(const char *source);
void ro_scene_free(ro_scene *s);
int ro_last_parse_error(void);  /* parser.rs:11-18 ParseError discriminant  */
size_t ro_scene_num_spheres(const ro_scene *s);
size_t ro_scene_num_triangles(const ro_scene *s);
/* camera[12] = origin, lower_left_corner, horizontal, vertical (camera.rs:8-15) */
void ro_scene_camera(const ro_scene *s, float camera[12]);
void ro_scene_set_camera(ro_scene *s, const float camera[12]);
/* replaces sphere (triangle != 0: triangle) i's material (type r g b a param) */
int ro_scene_set_material(ro_scene *s, int triangle, size_t i, const float m[6]);
/* sphere i: center(3) radius(1) material(6) = type, r, g, b, a, param */
void ro_scene_sphere(const ro_scene *s, size_t i, float out[10]);
/* triangle i: v0 v1 v2 (9) normal(3) material(6) */
void ro_scene_triangle(const ro_scene *s, size_t i, float out[18]);

/* Camera::new_at (camera.rs:21-33) and move_camera_position (lib.rs:60-63). */
void ro_camera_new_at(const float origin[3], float aspect, float camera[12]);
void ro_camera_move(const float camera_in[12], float x, float y, float z, float camera_out[12]);

/* Counter-mode per-sample seed (documented spec shared with the HIP kernel). */
uint32_t ro_sample_seed(uint32_t base_seed, uint64_t job);

/* ray_trace (common.rs:320-361) generalised with an RNG mode and a row subset:
 * rows row_begin, row_begin+row_step, ... (< height) in reference row order
 * (row 0 = bottom of the image).  out_rgba has width*height*4 bytes, top row
 * first (common.rs:351); untraced rows are left untouched.
 * sample_states (optional, width*height*spp u32): receives (SERIAL/COUNTER)
 * the RNG state at the start of every sample, indexed by the global job id
 * job = (row*width + col)*spp + s.  replay_states: REPLAY input, same index.
 * sample_rgba (optional, width*height*spp*4 f32): every sample's ray_color
 * result (r, g, b, a), same job index -- the bit-level parity surface.
 * nthreads > 1 is allowed for COUNTER/REPLAY (pixels dealt cyclically).
 * Returns 0 on success. */
int ro_render(const ro_scene *s, size_t width, size_t height, int spp, int depth,
              int rng_mode, uint32_t seed, const uint32_t *replay_states,
              size_t row_begin, size_t row_step, int nthreads,
              uint8_t *out_rgba, uint32_t *sample_states, float *sample_rgba,
              ro_stats *stats);

/* Same, over the columns col_begin, col_begin+col_step, ... of those rows only
 * (COUNTER / REPLAY; SERIAL needs whole rows). */
int ro_render_cols(const ro_scene *s, size_t width, size_t height, int spp, int depth,
                   int rng_mode, uint32_t seed, const uint32_t *replay_states,
                   size_t row_begin, size_t row_step, size_t col_begin, size_t col_step,
                   int nthreads, uint8_t *out_rgba, uint32_t *sample_states,
                   float *sample_rgba, ro_stats *stats);

/* ---- known-answer hooks on single functions (tests only) ---------------- */
uint32_t ro_xorshift32(uint32_t *state);                      /* random.rs:22-30 */
float ro_random_f32(uint32_t *state);                         /* random.rs:15-17 */
void ro_reflect(const float v[3], const float n[3], float out[3]);            /* maths.rs:26-28 */
void ro_refract(const float uv[3], const float n[3], float eta, float out[3]);/* maths.rs:31-36 */
void ro_normalize(const float v[3], float out[3]);                          /* maths.rs:111-118 */
/* ray = origin(3) direction(3).  out = t, position(3), normal(3).  1 = hit. */
int ro_sphere_hit(const float ray[6], const float center[3], float radius,
                  float t_min, float t_max, float out[7]);                  /* common.rs:59-98 */
int ro_triangle_intersect(const float ray[6], const float v[9],
                          float t_min, float t_max, float out[7]);           /* common.rs:124-166 */
/* material = type, r, g, b, a, param.  hit = t, position(3), normal(3).
 * Returns 1 if a next ray exists (written to next_ray[6]); color[4] always. */
int ro_scatter(const float material[6], const float ray[6], const float hit[7],
               uint32_t *rng_state, float color[4], float next_ray[6]);     /* materials.rs:30-102 */
void ro_sky(const float dir[3], const float final_color[4], float out[4]);  /* common.rs:276-281 */
void ro_cast_ray(const float camera[12], float s, float t, float ray[6]);   /* camera.rs:84-89 */
uint8_t ro_as_u8(float x);                                    /* Rust `as u8` (saturating) */

/* image.rs:59-81: ASCII PPM (P3), top row first.  Returns bytes written or -1. */
long ro_write_ppm(const uint8_t *rgba, size_t width, size_t height, char *buf, size_t cap);

#ifdef __cplusplus
}
#endif
#endif
