// sphere_list_check.cpp -- host check of the primary-ray sphere lists
// (bvh.cpp build_primary_sphere_lists; CPU test driver for
// tests/test_bvh_host.py).  For every pixel of a W x H frame and several
// sub-pixel offsets (the extremes 2^-32 and 1.0 of random_f32 included), the
// primary ray is built with the reference's f32 arithmetic (common.rs:335-336,
// camera.rs:84-89, maths.rs:111-118) and tested against every tree sphere with
// Sphere::hit's candidate arithmetic (common.rs:74-92).  Any sphere that
// yields a candidate root must be in the pixel's list, unless the pixel walks
// the tree.  Prints "OK <counts>" or the first failures and exits non-zero.
// usage: sphere_list_check scene.txt W H [dx dy dz]   (optional camera move)
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <fstream>
#include <sstream>
#include <vector>

#include "bvh.h"
#include "scene.h"

#pragma STDC FP_CONTRACT OFF

using namespace rtamd;

static uint32_t xs32(uint32_t &s) {
    s ^= s << 13;
    s ^= s >> 17;
    s ^= s << 5;
    return s;
}

int main(int argc, char **argv) {
    if (argc < 4) return 2;
    std::ifstream fh(argv[1]);
    std::stringstream ss;
    ss << fh.rdbuf();
    SceneModel scene;
    if (parse_scene(ss.str(), scene) != kParseOk) return 2;
    const size_t W = (size_t)std::atoi(argv[2]), H = (size_t)std::atoi(argv[3]);
    CameraModel cam = scene.camera;
    if (argc >= 7) cam = camera_moved(cam, std::strtof(argv[4], nullptr), std::strtof(argv[5], nullptr),
                                      std::strtof(argv[6], nullptr));
    const SphereBVH bv = build_sphere_bvh(scene.spheres, 3);
    const PrimarySphereLists L = build_primary_sphere_lists(bv, cam, W, H);
    if (L.rec.empty()) {
        std::printf("OK lists disabled (walk)\n");
        return 0;
    }
    const size_t n = bv.prims.size() / 4;
    const float wden = (float)(W - 1), hden = (float)(H - 1);
    const float offs[3] = {0x1p-32f, 1.0f, 0.5f};
    uint32_t seed = 2547549u;
    size_t rays = 0, hits = 0, walk = 0, listed = 0, fails = 0;
    for (size_t ir = 0; ir < H; ++ir) {
        const size_t row = H - 1 - ir;  // rows count from the bottom (common.rs:327)
        for (size_t col = 0; col < W; ++col) {
            const uint32_t a = L.rec[2 * (ir * W + col)], b = L.rec[2 * (ir * W + col) + 1];
            const uint32_t cnt = b >> 16;
            if (cnt == kSphListWalk) { ++walk; continue; }
            listed += cnt;
            const uint32_t item[3] = {a & 0xFFFFu, a >> 16, b & 0xFFFFu};
            for (int k = 0; k < 8; ++k) {
                const float r1 = k < 3 ? offs[k] : (float)xs32(seed) * 0x1p-32f;
                const float r2 = k < 3 ? offs[2 - k] : (float)xs32(seed) * 0x1p-32f;
                const float u = ((float)col + r1) / wden, v = ((float)row + r2) / hden;
                const Vec3 o = cam.origin, l = cam.lower_left, h = cam.horizontal, vv = cam.vertical;
                float dx = ((l.x + h.x * u) + vv.x * v) - o.x;
                float dy = ((l.y + h.y * u) + vv.y * v) - o.y;
                float dz = ((l.z + h.z * u) + vv.z * v) - o.z;
                const float len = std::sqrt((dx * dx + dy * dy) + dz * dz);
                dx = dx / len; dy = dy / len; dz = dz / len;
                ++rays;
                for (size_t i = 0; i < n; ++i) {
                    const float *s = &bv.prims[4 * i];
                    const float ox = o.x - s[0], oy = o.y - s[1], oz = o.z - s[2];
                    const float hb = (ox * dx + oy * dy) + oz * dz;
                    const float cc = ((ox * ox + oy * oy) + oz * oz) - s[3];
                    const float disc = hb * hb - cc;
                    if (!(disc >= 0.0f)) continue;
                    const float sq = std::sqrt(disc);
                    if (!(0.001f < -hb - sq) && !(0.001f < -hb + sq)) continue;
                    ++hits;
                    bool in = false;
                    for (uint32_t j = 0; j < cnt; ++j) in |= item[j] == i;
                    if (!in && fails++ < 10)
                        std::printf("pixel (%zu, %zu) offset %d: tree sphere %zu has a candidate but is not listed\n",
                                    col, ir, k, i);
                }
            }
        }
    }
    if (fails) return 1;
    std::printf("OK rays %zu candidates %zu walk-pixels %zu listed %zu\n", rays, hits, walk, listed);
    return 0;
}
