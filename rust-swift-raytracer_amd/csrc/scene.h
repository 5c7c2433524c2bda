// scene.h -- host-side scene model of the MI355X raytracer (product code).
//
// Mirrors the reference's World / Camera / MaterialType (raytracer/src/
// common.rs:169-258, camera.rs:8-93, materials.rs:7-12) and packs them into
// the structure-of-arrays layout the HIP kernel reads (DESIGN.md "Data layout
// in HBM").  Contains no device code and no torch types.
#pragma once

#include <cstddef>
#include <cstdint>
#include <string>
#include <vector>

namespace rtamd {

struct Vec3 { float x, y, z; };

enum MaterialKind : uint32_t { kDiffuse = 0, kMetal = 1, kDielectric = 2, kEmission = 3 };

struct Material {           // materials.rs:7-12
    uint32_t kind;
    float r, g, b, a;       // Color (alpha is 1.0 for every parsed material)
    float param;            // Metal fuzz | Dielectric ir
};

struct Sphere { Vec3 center; float radius; uint32_t material; };     // common.rs:54-58
struct Triangle { Vec3 v0, v1, v2, normal; uint32_t material; };    // common.rs:101-107

struct CameraModel {        // camera.rs:8-15
    Vec3 origin, lower_left, horizontal, vertical;
};

// camera.rs:21-33
CameraModel camera_new_at(Vec3 origin, float aspect);
// lib.rs:60-63 (+ camera.rs:70-72 aspect_ratio, :91-93 position)
CameraModel camera_moved(const CameraModel &c, float x, float y, float z);

struct SceneModel {
    std::vector<Material> materials;   // one entry per sphere/triangle reference
    std::vector<Sphere> spheres;       // in file order (ties: first wins)
    std::vector<Triangle> triangles;   // the single Mesh of lib.rs:41
    CameraModel camera;
};

// ParseError discriminants (parser.rs:11-18); 100 = reference would panic.
enum ParseStatus { kParseOk = -1, kMissingCamera = 1, kWrongSyntax = 2, kDidntStartWith = 3,
                   kNotAF32 = 5, kWouldPanic = 100 };

// parser.rs:336-381.  Returns kParseOk or the error kind.
int parse_scene(const std::string &text, SceneModel &out);

// Structure-of-arrays image of a scene, ready for upload.
struct PackedScene {
    // spheres: hot = (cx, cy, cz, r*r); cold = (r, material id bits, 0, 0)
    std::vector<float> sph_hot, sph_cold;
    uint32_t nsph = 0, nsph_padded = 0;
    // triangles: hot = (n.x, n.y, n.z, d) with n = cross(v1-v0, v2-v0), d = n.v0;
    // geo = 4 float4 per triangle: (v0, mat bits) (v1, 0) (v2, 0) (normal, 0)
    std::vector<float> tri_hot, tri_geo;
    uint32_t ntri = 0, ntri_padded = 0;
    // materials: 8 floats each: (kind bits, r, g, b, param, 0, 0, 0)
    std::vector<float> mats;
    // per-sphere shading record (one round trip after the hit): 8 floats
    // (cx, cy, cz, r, colour r, g, b, fuzz|ir) + material kind
    std::vector<float> sph_shade;
    std::vector<uint32_t> sph_kind;
};
PackedScene pack_scene(const SceneModel &s, uint32_t sphere_pad, uint32_t tri_pad);

}  // namespace rtamd
