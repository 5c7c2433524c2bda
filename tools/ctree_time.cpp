// Host timing of the triangle-tree builders on the C5 mesh (tools only):
// usage: ctree_time scene.txt
#include <chrono>
#include <cstdio>
#include <fstream>
#include <sstream>
#include "bvh.h"
#include "scene.h"
using namespace rtamd;
int main(int argc, char **argv) {
    std::ifstream f(argv[1]); std::stringstream ss; ss << f.rdbuf();
    SceneModel sc; if (parse_scene(ss.str(), sc) != kParseOk) return 1;
    PackedScene p = pack_scene(sc, 8, 1);
    auto t0 = std::chrono::steady_clock::now();
    TriangleBVH tb = build_triangle_bvh(sc.triangles, p.tri_hot, 1);
    auto t1 = std::chrono::steady_clock::now();
    CameraModel cam = camera_moved(sc.camera, 0, 0, -0.05f);
    float o[3] = {cam.origin.x, cam.origin.y, cam.origin.z};
    CameraTriangleBVH ct = build_camera_triangle_bvh(sc.triangles, p.tri_hot, tb, o, 2);
    auto t2 = std::chrono::steady_clock::now();
    PrimaryTriLists pl = build_primary_tri_lists(ct, cam, 1920, 1080);
    auto t3 = std::chrono::steady_clock::now();
    auto ms = [](auto a, auto b) { return std::chrono::duration<double, std::milli>(b - a).count(); };
    std::printf("static tree %.1f ms, camera tree %.1f ms, strip lists %.1f ms (%zu nodes)\n", ms(t0, t1), ms(t1, t2), ms(t2, t3), ct.qnodes.size() / 8);
}
