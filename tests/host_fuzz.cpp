// host_fuzz.cpp -- sanitizer driver for the host side of the product (built
// with -fsanitize=address,undefined by tests/test_host_sanitizers.py).
//
// The parser (csrc/scene.cpp, the parser.rs:54-381 grammar with hand-decoded
// UTF-8) and the BVH builders (csrc/bvh.cpp) run on every load_world and
// camera move.  This driver feeds them:
//   * every scene file given on the command line, unchanged;
//   * byte-level mutations of those files (bit flips, byte insertions and
//     deletions, truncations, splices of two files, random UTF-8 sequences
//     including overlong, surrogate and truncated forms);
//   * random well-formed scenes (degenerate, duplicate, huge and non-finite
//     spheres and triangles) so that the builders see unusual geometry.
// Every scene that parses is packed and gets all trees and primary lists
// built for a few cameras and frame sizes.  Any sanitizer report aborts.
//
// usage: host_fuzz <seconds> <seed> scene.txt...
#include <chrono>
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <fstream>
#include <random>
#include <sstream>
#include <string>
#include <vector>

#include "bvh.h"
#include "scene.h"

using namespace rtamd;

namespace {

std::string read_file(const char *path) {
    std::ifstream f(path, std::ios::binary);
    std::stringstream ss;
    ss << f.rdbuf();
    return ss.str();
}

struct Counts {
    uint64_t inputs = 0, parsed = 0, spheres = 0, triangles = 0;
};

void build_everything(const SceneModel &sc, std::mt19937_64 &rng, Counts &cnt) {
    ++cnt.parsed;
    cnt.spheres += sc.spheres.size();
    cnt.triangles += sc.triangles.size();
    const PackedScene packed = pack_scene(sc, 8, 1);
    const uint32_t leaf = 1 + (uint32_t)(rng() % 4);
    const SphereBVH bv = build_sphere_bvh(sc.spheres, leaf);
    const TriangleBVH tb = build_triangle_bvh(sc.triangles, packed.tri_hot, leaf);
    const size_t sizes[][2] = {{1, 1}, {2, 2}, {7, 3}, {64, 36}, {33, 1}};
    CameraModel cam = sc.camera;
    for (int k = 0; k < 3; ++k) {
        const float o[3] = {cam.origin.x, cam.origin.y, cam.origin.z};
        if (!tb.nodes.empty()) {
            const CameraTriangleBVH ct = build_camera_triangle_bvh(sc.triangles, packed.tri_hot, tb, o,
                                                                   1 + (uint32_t)(rng() % 3));
            const auto &sz = sizes[rng() % 5];
            (void)build_primary_tri_lists(ct, cam, sz[0], sz[1]);
        }
        if (!bv.nodes.empty()) {
            const auto &sz = sizes[rng() % 5];
            (void)build_primary_sphere_lists(bv, cam, sz[0], sz[1]);
        }
        std::uniform_real_distribution<float> d(-50.0f, 50.0f);
        cam = camera_moved(cam, d(rng), d(rng), d(rng));
    }
}

std::string mutate(const std::vector<std::string> &corpus, std::mt19937_64 &rng) {
    std::string s = corpus[rng() % corpus.size()];
    const int edits = 1 + (int)(rng() % 8);
    for (int e = 0; e < edits; ++e) {
        const size_t n = s.size();
        switch (rng() % 7) {
        case 0:  // bit flip
            if (n) s[rng() % n] ^= (char)(1u << (rng() % 8));
            break;
        case 1: {  // insert a byte (often structural)
            static const char kStruct[] = ";:.-0123456789 \n\t/ emacrtiuslo";
            const char c = (rng() % 2) ? kStruct[rng() % (sizeof(kStruct) - 1)] : (char)(rng() & 0xFF);
            s.insert(s.begin() + (n ? rng() % (n + 1) : 0), c);
            break;
        }
        case 2:  // delete a run
            if (n) {
                const size_t at = rng() % n;
                s.erase(at, 1 + rng() % std::min<size_t>(16, n - at));
            }
            break;
        case 3:  // truncate
            if (n) s.resize(rng() % n);
            break;
        case 4: {  // splice another file's tail
            const std::string &o = corpus[rng() % corpus.size()];
            if (!o.empty() && n) s = s.substr(0, rng() % n) + o.substr(rng() % o.size());
            break;
        }
        case 5: {  // UTF-8-ish sequences: valid, overlong, surrogates, truncated
            static const char *kSeq[] = {"\xC3\xA9", "\xE2\x80\x83", "\xE3\x80\x80", "\xF0\x9F\x98\x80",
                                         "\xC0\xAF", "\xED\xA0\x80", "\xF4\x90\x80\x80", "\xE2\x82",
                                         "\xF0\x9F", "\xC2", "\xFF", "\xE6\x97\xA5\xE6\x9C\xAC"};
            s.insert(n ? rng() % (n + 1) : 0, kSeq[rng() % 12]);
            break;
        }
        default: {  // duplicate a statement
            const size_t a = n ? s.find(';', rng() % n) : std::string::npos;
            if (a != std::string::npos) {
                const size_t b = s.rfind(';', a ? a - 1 : 0);
                const size_t from = b == std::string::npos ? 0 : b + 1;
                s.insert(a + 1, s.substr(from, a + 1 - from));
            }
        }
        }
    }
    return s;
}

std::string num(std::mt19937_64 &rng) {
    char buf[64];
    switch (rng() % 8) {
    case 0: return "0.0";
    case 1: std::snprintf(buf, sizeof buf, "%.1f", (double)(int64_t)(rng() % 2000001) - 1000000.0); return buf;
    case 2: return "340282350000000000000000000000000000000.0";   // FLT_MAX
    case 3: return "3402823500000000000000000000000000000000.0";  // overflows to inf
    case 4: return "0.0000000000000000000000000000000000000000001";
    default: {
        std::uniform_real_distribution<double> d(-20.0, 20.0);
        std::snprintf(buf, sizeof buf, "%.6f", d(rng));
        return buf;
    }
    }
}

std::string random_scene(std::mt19937_64 &rng) {
    std::string s = "camera origin " + num(rng) + " " + num(rng) + " " + num(rng) + " aspect " +
                    ((rng() % 4) ? std::string("1.77778") : num(rng)) + ";\n";
    s += "material M0 : Diffuse color 0.5 0.5 0.5;\nmaterial M1 : Metal color 0.8 0.6 0.2 fuzz 0.3;\n"
         "material M2 : Dielectric ir 1.5;\n";
    const int ns = (int)(rng() % 60), nt = (int)(rng() % 80);
    for (int i = 0; i < ns; ++i) {
        s += "sphere center " + num(rng) + " " + num(rng) + " " + num(rng) + " radius " +
             ((rng() % 3) ? std::string("0.5") : num(rng)) + " material M" + std::to_string(rng() % 3) + ";\n";
        if (rng() % 10 == 0) s += s.substr(s.rfind("sphere"));  // exact duplicate
    }
    for (int i = 0; i < nt; ++i) {
        std::string v[3];
        for (auto &x : v) x = num(rng) + " " + num(rng) + " " + num(rng);
        if (rng() % 8 == 0) v[2] = v[1];  // degenerate
        s += "triangle v0 " + v[0] + " v1 " + v[1] + " v2 " + v[2] + " material M" +
             std::to_string(rng() % 3) + ";\n";
    }
    return s;
}

}  // namespace

int main(int argc, char **argv) {
    if (argc < 4) {
        std::fprintf(stderr, "usage: host_fuzz <seconds> <seed> scene.txt...\n");
        return 2;
    }
    const double seconds = std::atof(argv[1]);
    std::mt19937_64 rng(std::strtoull(argv[2], nullptr, 10));
    std::vector<std::string> corpus;
    for (int i = 3; i < argc; ++i) corpus.push_back(read_file(argv[i]));
    Counts cnt;
    auto run = [&](const std::string &text) {
        ++cnt.inputs;
        SceneModel sc;
        if (parse_scene(text, sc) == kParseOk) build_everything(sc, rng, cnt);
    };
    for (const auto &c : corpus) run(c);
    const auto t0 = std::chrono::steady_clock::now();
    uint64_t iter = 0;
    while (std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count() < seconds) {
        run((iter++ % 3 == 2) ? random_scene(rng) : mutate(corpus, rng));
    }
    std::printf("inputs %llu parsed %llu spheres %llu triangles %llu\n",
                (unsigned long long)cnt.inputs, (unsigned long long)cnt.parsed,
                (unsigned long long)cnt.spheres, (unsigned long long)cnt.triangles);
    return 0;
}
