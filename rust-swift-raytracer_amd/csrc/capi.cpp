// capi.cpp -- the C-ABI of the library: the reference's three entry points
// (Naxaes/Rust-Swift-Raytracer raytracer/src/lib.rs:37-63, header
// MacOSPlatform/MacOSPlatform/Engine/includes/raytracer.h:42-47) plus the
// extensions declared in include/raytracer_amd.h.
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>

#include "../../include/raytracer.h"
#include "../../include/raytracer_amd.h"
#include "runtime.h"
#include "scene.h"

// The opaque types of raytracer.h.  Rust_WorldHandle stays two pointers;
// the camera is heap-allocated on its own because callers replace it
// (GameView.swift:200-216 writes handle->camera = move_camera_position(...)).
struct Rust_World {
    rtamd::WorldState state;
};
struct Rust_Camera {
    rtamd::CameraModel cam;
};

namespace {
thread_local int g_parse_status = rtamd::kParseOk;

RtRenderOptions reference_options() {
    RtRenderOptions o;
    rt_default_options(&o);
    return o;
}

// A leaf-size knob (RT_AMD_LEAF / RT_AMD_TRI_LEAF): a whole decimal number in
// [1, 8], else the default (the BVH builders clamp it as well)
uint32_t env_leaf(const char *name, uint32_t dflt) {
    const char *e = std::getenv(name);
    if (!e || !*e) return dflt;
    char *end = nullptr;
    const long n = std::strtol(e, &end, 10);
    return (end && *end == '\0' && n >= 1 && n <= 8) ? (uint32_t)n : dflt;
}

// render()'s device count: RT_AMD_DEVICES=N (N >= 1) row-tiles its frames over
// N devices; unset, invalid or 0 keeps one device
int32_t env_devices() {
    const char *e = std::getenv("RT_AMD_DEVICES");
    if (!e || !*e) return 0;
    char *end = nullptr;
    const long n = std::strtol(e, &end, 10);
    return (end && *end == '\0' && n >= 1 && n <= 64) ? (int32_t)n : 0;
}
}  // namespace

extern "C" {

// lib.rs:37-46
Rust_WorldHandle *load_world(const char *source) {
    if (!source) {
        rtamd::set_error("load_world: null source");
        return nullptr;
    }
    auto *world = new Rust_World();
    g_parse_status = rtamd::parse_scene(std::string(source), world->state.scene);
    if (g_parse_status != rtamd::kParseOk) {
        rtamd::set_error("load_world: parse error " + std::to_string(g_parse_status));
        delete world;
        return nullptr;
    }
    // spheres padded to the kernel's scalar-load batch of 8 with NaN centres
    world->state.packed = rtamd::pack_scene(world->state.scene, 8, 1);
    // spheres per BVH leaf (A/B with walk gating, C2 / C3: 3 -> 4.72 / 70.6 ms,
    // 2 -> 4.65 / 69.6, 1 -> 6.33 / 95.3 -- its tree no longer fits 64 KB of LDS)
    world->state.bvh = rtamd::build_sphere_bvh(world->state.scene.spheres, env_leaf("RT_AMD_LEAF", 2u));
    // triangles per BVH leaf (A/B on C5 at 96-node walk slices: 1 -> 222 ms,
    // 2 -> 240, 3 -> 293)
    world->state.tbvh = rtamd::build_triangle_bvh(world->state.scene.triangles,
                                                  world->state.packed.tri_hot,
                                                  env_leaf("RT_AMD_TRI_LEAF", 1u));
    // per-origin-cell trees: for meshes of >= 64 k triangles
    // by default, over the box of the mesh and the spheres around it, starting
    // from the edge that cuts the mesh's box into <= 1024 cells and grown to the
    // trees' budget (bvh.h TriangleCells; C5: 396 trees of 2-unit cells, static
    // tree 143.6 ms -> 88.7 ms); RT_AMD_TRI_CELLS=<edge> sets the starting
    // edge, 0 switches them off.  The static tree is re-quantised on their
    // common grid.
    {
        float size = 0.0f;
        if (const char *cs = std::getenv("RT_AMD_TRI_CELLS")) {
            size = std::strtof(cs, nullptr);
        } else if (world->state.scene.triangles.size() >= 65536 && !world->state.tbvh.nodes.empty()) {
            size = rtamd::triangle_cell_edge(world->state.scene.triangles, 1024);
        }
        if (size > 0.0f)
            world->state.tcells = rtamd::build_triangle_cells(world->state.scene.triangles,
                                                              world->state.packed.tri_hot,
                                                              world->state.scene.spheres,
                                                              env_leaf("RT_AMD_TRI_LEAF", 1u), size,
                                                              world->state.tbvh);
        const auto &tc = world->state.tcells;
        if (std::getenv("RT_AMD_TRI_CELLS_DEBUG")) std::fprintf(stderr, "tri cells: %u x %u x %u = %u cells of %.3g, %u wide nodes per tree, "
                     "%zu records, %.1f MB\n", tc.n[0], tc.n[1], tc.n[2], tc.ncells, tc.size, tc.stride_w,
                     tc.tris.size() / 16,
                     (tc.wnodes.size() * 4.0 + tc.tris.size() * 4.0) / 1e6);
    }
    // bounce-0 triangle tree for the scene camera (rebuilt by the first render
    // after move_camera_position, which does not see the world)
    rtamd::prepare_camera(world->state, world->state.scene.camera);
    auto *cam = new Rust_Camera{world->state.scene.camera};
    return new Rust_WorldHandle{world, cam};
}

// lib.rs:60-63: consumes the old camera, returns Camera::new_at(pos + d, aspect).
Rust_Camera *move_camera_position(Rust_Camera *camera, float x, float y, float z) {
    if (!camera) return nullptr;
    auto *moved = new Rust_Camera{rtamd::camera_moved(camera->cam, x, y, z)};
    delete camera;
    return moved;
}

// lib.rs:49-57: Options::new(16, 8, None, true); synchronous.  Writes into the
// caller's pixels (the reference returned a pointer into a freed Vec).
Rust_CFramebuffer render(Rust_CFramebuffer framebuffer, const Rust_WorldHandle *handle) {
    RtRenderOptions o = reference_options();
    o.ndevices = env_devices();
    // the reference's own frame (one xorshift32 stream, common.rs:321) unless
    // RT_AMD_RNG=counter asks for the fast per-sample-seeded mode
    const char *rng = std::getenv("RT_AMD_RNG");
    if (rng && std::strcmp(rng, "counter") == 0) o.rng_mode = RT_RNG_COUNTER;
    int rc = rt_render_ex(framebuffer, handle, &o, nullptr);
    if (rc != 0) {
        std::fprintf(stderr, "raytracer render() failed (%d): %s\n", rc, rtamd::last_error().c_str());
        return Rust_CFramebuffer{0, 0, nullptr};
    }
    return framebuffer;
}

void rt_default_options(RtRenderOptions *o) {
    std::memset(o, 0, sizeof(*o));
    o->samples_per_pixel = 16;  // lib.rs:51
    o->max_ray_bounces = 8;     // lib.rs:51
    o->rng_mode = RT_RNG_SERIAL;  // the reference's stream (common.rs:321)
    o->seed = 2547549u;         // random.rs:9
    o->row_block = 8;  // multi-GPU tiles: blocks of 8 rows
    o->rank = 0;
    o->nranks = 1;
    o->device = -1;
    o->accel = RT_ACCEL_AUTO;
}

size_t rt_tile_rows(size_t height, uint32_t row_block, uint32_t rank, uint32_t nranks) {
    if (rank >= (nranks ? nranks : 1)) return 0;
    return rtamd::tile_rows(height, row_block, rank, nranks);
}

size_t rt_tile_row(size_t k, uint32_t row_block, uint32_t rank, uint32_t nranks) {
    return rtamd::tile_row(k, row_block, rank, nranks);
}

uint32_t rt_sample_seed(uint32_t seed, uint64_t job) {
    uint64_t z = job + (uint64_t)seed * 0x9E3779B97F4A7C15ull + 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    z ^= z >> 31;
    uint32_t r = (uint32_t)(z ^ (z >> 32));
    return r ? r : 2547549u;
}

int rt_render_ex(Rust_CFramebuffer fb, const Rust_WorldHandle *h, const RtRenderOptions *opts,
                 RtRenderStats *stats) {
    if (!h || !h->world || !h->camera) {
        rtamd::set_error("render: null world handle");
        return -1;
    }
    RtRenderOptions o = opts ? *opts : reference_options();
    return rtamd::render_frame_host(h->world->state, h->camera->cam, fb.width, fb.height, o,
                                    fb.pixels, stats);
}

int rt_render_device(const Rust_WorldHandle *h, size_t width, size_t height,
                     const RtRenderOptions *opts, void *d_rgba, void *hip_stream,
                     RtRenderStats *stats) {
    if (!h || !h->world || !h->camera) {
        rtamd::set_error("render: null world handle");
        return -1;
    }
    RtRenderOptions o = opts ? *opts : reference_options();
    if (o.ndevices >= 1)
        return rtamd::render_frame_multi(h->world->state, h->camera->cam, width, height, o,
                                         static_cast<uint32_t *>(d_rgba),
                                         static_cast<hipStream_t>(hip_stream), stats);
    return rtamd::render_frame(h->world->state, h->camera->cam, width, height, o,
                               static_cast<uint32_t *>(d_rgba),
                               static_cast<hipStream_t>(hip_stream), stats);
}

long rt_read_samples(const Rust_WorldHandle *h, int device, float *out, size_t n) {
    if (!h || !h->world || !out) {
        rtamd::set_error("rt_read_samples: null argument");
        return -1;
    }
    return rtamd::read_samples(h->world->state, device, out, n);
}

void rt_free_world(Rust_WorldHandle *h) {
    if (!h) return;
    delete h->world;
    delete h->camera;
    delete h;
}

const char *rt_last_error(void) { return rtamd::last_error().c_str(); }

int rt_last_parse_error(void) { return g_parse_status; }

size_t rt_world_num_spheres(const Rust_WorldHandle *h) {
    return h && h->world ? h->world->state.scene.spheres.size() : 0;
}
size_t rt_world_num_triangles(const Rust_WorldHandle *h) {
    return h && h->world ? h->world->state.scene.triangles.size() : 0;
}

// Replaces primitive i's material.  Each primitive owns its material copy
// (parser.rs:237-310 clone the named material), so this changes one primitive.
static int set_material(Rust_WorldHandle *h, bool tri, size_t i, const float *m) {
    if (!h || !h->world || !m) return -1;
    rtamd::WorldState &w = h->world->state;
    std::lock_guard<std::recursive_mutex> lock(w.mu);
    rtamd::SceneModel &sc = w.scene;
    if (tri ? i >= sc.triangles.size() : i >= sc.spheres.size()) {
        rtamd::set_error("set material: primitive index out of range");
        return -1;
    }
    // kinds of materials.rs:7-12; every Color the reference builds has alpha 1.0
    // (color.rs:21-23), which the resolve relies on
    const float k = m[0];
    if (!(k == 0.0f || k == 1.0f || k == 2.0f || k == 3.0f) || m[4] != 1.0f) {
        rtamd::set_error("set material: kind must be 0-3 and alpha 1.0");
        return -1;
    }
    const uint32_t idx = tri ? sc.triangles[i].material : sc.spheres[i].material;
    sc.materials[idx] = rtamd::Material{(uint32_t)k, m[1], m[2], m[3], m[4], m[5]};
    w.packed = rtamd::pack_scene(sc, 8, 1);
    w.devices.clear();  // the next frame uploads the scene again
    return 0;
}

int rt_world_set_sphere_material(Rust_WorldHandle *h, size_t i, const float material[6]) {
    return set_material(h, false, i, material);
}

int rt_world_set_triangle_material(Rust_WorldHandle *h, size_t i, const float material[6]) {
    return set_material(h, true, i, material);
}

static void material_out(const rtamd::Material &m, float *o) {
    o[0] = (float)m.kind; o[1] = m.r; o[2] = m.g; o[3] = m.b; o[4] = m.a; o[5] = m.param;
}

int rt_world_sphere(const Rust_WorldHandle *h, size_t i, float out[10]) {
    if (!h || !h->world || i >= h->world->state.scene.spheres.size()) return -1;
    const auto &sc = h->world->state.scene;
    const auto &s = sc.spheres[i];
    out[0] = s.center.x; out[1] = s.center.y; out[2] = s.center.z; out[3] = s.radius;
    material_out(sc.materials[s.material], out + 4);
    return 0;
}

int rt_world_triangle(const Rust_WorldHandle *h, size_t i, float out[18]) {
    if (!h || !h->world || i >= h->world->state.scene.triangles.size()) return -1;
    const auto &sc = h->world->state.scene;
    const auto &t = sc.triangles[i];
    const rtamd::Vec3 v[4] = {t.v0, t.v1, t.v2, t.normal};
    for (int k = 0; k < 4; ++k) { out[3 * k] = v[k].x; out[3 * k + 1] = v[k].y; out[3 * k + 2] = v[k].z; }
    material_out(sc.materials[t.material], out + 12);
    return 0;
}

void rt_camera_get(const Rust_Camera *c, float out[12]) {
    const rtamd::Vec3 v[4] = {c->cam.origin, c->cam.lower_left, c->cam.horizontal, c->cam.vertical};
    for (int k = 0; k < 4; ++k) { out[3 * k] = v[k].x; out[3 * k + 1] = v[k].y; out[3 * k + 2] = v[k].z; }
}

// image.rs:59-81: "P3\n{w} {h}\n255\n" then "r g b\n" per pixel, top row first.
int rt_write_ppm(const Rust_CFramebuffer *fb, const char *path) {
    if (!fb || !path || (!fb->pixels && fb->width * fb->height)) return -1;
    FILE *f = std::fopen(path, "wb");
    if (!f) return -1;
    std::fprintf(f, "P3\n%zu %zu\n255\n", fb->width, fb->height);
    for (size_t i = 0; i < fb->width * fb->height; ++i) {
        const Rust_ColorU8 &c = fb->pixels[i];
        std::fprintf(f, "%u %u %u\n", (unsigned)c.r, (unsigned)c.g, (unsigned)c.b);
    }
    return std::fclose(f) == 0 ? 0 : -1;
}

int rt_comm_count(int first, int n) { return rtamd::comm_count(first, n); }

int rt_assemble_tiles(const void *d_gathered, void *d_out, size_t width, size_t height, uint32_t row_block,
                      uint32_t nranks, size_t max_rows, void *hip_stream) {
    return rtamd::assemble_tiles(static_cast<const uint32_t *>(d_gathered), static_cast<uint32_t *>(d_out), width,
                                 height, row_block, nranks, max_rows, static_cast<hipStream_t>(hip_stream));
}

int rt_device_count(void) {
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess) return 0;
    return n;
}

}  // extern "C"
