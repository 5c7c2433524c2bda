// scene.cpp -- scene DSL parser, camera constructors and SoA packing (host).
//
// The parser accepts exactly the grammar of the reference's parser.rs:326-381
// (camera, then materials, then spheres, then triangles, `//` comments) with
// its quirks: keywords need no trailing whitespace, a float needs >= 3 bytes
// of remaining input (parser.rs:112), floats are [-]digits[.digits] parsed
// with correct rounding (Rust `str::parse::<f32>`), duplicate material names
// overwrite, and a comment is only recognised where parser.rs calls
// skip_comment.  Inputs on which the reference panics return kWouldPanic.
//
// Built with -ffp-contract=off: the triangle constants precomputed here must
// carry the exact bits the reference computes per test (common.rs:131-140).
#include "scene.h"
#include "unicode_alnum.h"

#include <cmath>
#include <cstdlib>
#include <cstring>
#include <locale.h>
#include <unordered_map>

namespace rtamd {

namespace {

inline Vec3 vsub(Vec3 a, Vec3 b) { return {a.x - b.x, a.y - b.y, a.z - b.z}; }
inline Vec3 vadd(Vec3 a, Vec3 b) { return {a.x + b.x, a.y + b.y, a.z + b.z}; }
inline float vdot(Vec3 a, Vec3 b) { return a.x * b.x + a.y * b.y + a.z * b.z; }
inline Vec3 vcross(Vec3 a, Vec3 b) {  // maths.rs:88-94
    return {a.y * b.z - a.z * b.y, -(a.x * b.z - a.z * b.x), a.x * b.y - a.y * b.x};
}
inline Vec3 vnormalize(Vec3 a) {  // maths.rs:111-118
    float len = std::sqrt(a.x * a.x + a.y * a.y + a.z * a.z);
    return {a.x / len, a.y / len, a.z / len};
}

struct ParseError { int status; };

// Unicode helpers for Rust's char::is_whitespace / is_alphanumeric.
uint32_t decode_utf8(const char *p, const char *end, int &len) {
    unsigned char c = (unsigned char)*p;
    if (c < 0x80) { len = 1; return c; }
    len = c >= 0xF0 ? 4 : c >= 0xE0 ? 3 : 2;
    uint32_t cp = c & (0x7Fu >> len);
    for (int k = 1; k < len && p + k < end; ++k) cp = (cp << 6) | ((unsigned char)p[k] & 0x3Fu);
    return cp;
}
bool unicode_space(uint32_t c) {
    if (c <= 0x20) return c == 0x20 || (c >= 0x09 && c <= 0x0D);
    if (c < 0x85) return false;
    return c == 0x85 || c == 0xA0 || c == 0x1680 || (c >= 0x2000 && c <= 0x200A) ||
           c == 0x2028 || c == 0x2029 || c == 0x202F || c == 0x205F || c == 0x3000;
}
// char::is_alphanumeric (parser.rs:60): the Unicode 13.0.0 table of
// unicode_alnum.h (tools/gen_unicode_alnum.py), binary search above ASCII.
bool unicode_alnum(uint32_t c) {
    if (c < 0x80) {
        return (c >= '0' && c <= '9') || ((c | 0x20) >= 'a' && (c | 0x20) <= 'z');
    }
    uint32_t lo = 0, hi = kAlnumRangeCount;  // first range with end >= c
    while (lo < hi) {
        const uint32_t mid = (lo + hi) / 2;
        if (kAlnumRanges[mid][1] < c) lo = mid + 1;
        else hi = mid;
    }
    return lo < kAlnumRangeCount && kAlnumRanges[lo][0] <= c;
}

// A scanner whose position plays the role of the reference's `&str` rest.
class Scanner {
  public:
    Scanner(const char *b, const char *e) : pos_(b), end_(e) {}

    bool at_end() const { return pos_ == end_; }

    void ws() {  // skip_whitespace, parser.rs:54-57
        while (pos_ < end_) {
            int n;
            if (!unicode_space(decode_utf8(pos_, end_, n))) return;
            pos_ += n;
        }
    }
    // starts_with, parser.rs:81-88 -- advance past `kw` if it is a prefix.
    bool eat(const char *kw) {
        size_t n = std::strlen(kw);
        if ((size_t)(end_ - pos_) < n) return false;
        if (pos_ + n < end_ && ((unsigned char)pos_[n] & 0xC0) == 0x80)
            throw ParseError{kWouldPanic};  // &source[0..n] off a char boundary
        if (std::memcmp(pos_, kw, n) != 0) return false;
        pos_ += n;
        return true;
    }
    void need(const char *kw) {
        if (!eat(kw)) throw ParseError{kDidntStartWith};
    }
    // get_identifier, parser.rs:59-62
    std::string ident() {
        const char *b = pos_;
        while (pos_ < end_) {
            int n;
            uint32_t cp = decode_utf8(pos_, end_, n);
            if (!(cp == '_' || unicode_alnum(cp))) break;
            pos_ += n;
        }
        return std::string(b, pos_);
    }
    // parse_float, parser.rs:107-133
    float number() {
        if (end_ - pos_ < 3) throw ParseError{kNotAF32};
        const char *p = pos_;
        if (*p == '-') ++p;
        bool dot = false, digit = false;
        for (; p < end_; ++p) {
            if (*p >= '0' && *p <= '9') { digit = true; continue; }
            if (*p != '.') break;
            if (dot) throw ParseError{kNotAF32};
            dot = true;
        }
        if (!digit) throw ParseError{kNotAF32};  // "", "-", ".", "-."
        std::string lit(pos_, p);
        static locale_t c_loc = newlocale(LC_ALL_MASK, "C", (locale_t)0);
        char *stop = nullptr;
        float v = strtof_l(lit.c_str(), &stop, c_loc);  // correctly rounded
        if (stop != lit.c_str() + lit.size()) throw ParseError{kNotAF32};
        pos_ = p;
        return v;
    }
    Vec3 vec3() {  // parse_vec3, parser.rs:135-142
        Vec3 v;
        v.x = number(); ws();
        v.y = number(); ws();
        v.z = number();
        return v;
    }
    // skip_comment, parser.rs:313-323
    void comments() {
        for (;;) {
            if (end_ - pos_ < 2) return;
            if (pos_ + 2 < end_ && ((unsigned char)pos_[2] & 0xC0) == 0x80)
                throw ParseError{kWouldPanic};  // starts_with(source, "//") slice
            if (pos_[0] != '/' || pos_[1] != '/') return;
            const char *p = pos_ + 2;
            for (;; ++p) {
                if (p >= end_) throw ParseError{kWrongSyntax};
                // find() slices byte by byte: a multi-byte char before '\n' panics
                if (((unsigned char)*p & 0x80) != 0) throw ParseError{kWouldPanic};
                if (*p == '\n') break;
            }
            pos_ = p + 1;
        }
    }

  private:
    const char *pos_, *end_;
};

bool valid_utf8(const std::string &s) {
    for (size_t i = 0; i < s.size();) {
        unsigned char c = (unsigned char)s[i];
        size_t n = c < 0x80 ? 1 : (c & 0xE0) == 0xC0 ? 2 : (c & 0xF0) == 0xE0 ? 3 : (c & 0xF8) == 0xF0 ? 4 : 0;
        if (!n || i + n > s.size()) return false;
        for (size_t k = 1; k < n; ++k)
            if (((unsigned char)s[i + k] & 0xC0) != 0x80) return false;
        i += n;
    }
    return true;
}

}  // namespace

CameraModel camera_new_at(Vec3 origin, float aspect) {
    const float viewport_height = 2.0f;
    const float viewport_width = aspect * viewport_height;
    const float focal_length = 1.0f;
    CameraModel c;
    c.origin = origin;
    c.horizontal = {viewport_width, 0.0f, 0.0f};
    c.vertical = {0.0f, viewport_height, 0.0f};
    c.lower_left = vsub(origin, {viewport_width / 2.0f, viewport_height / 2.0f, focal_length});
    return c;
}

CameraModel camera_moved(const CameraModel &c, float x, float y, float z) {
    const float aspect = c.horizontal.x / c.vertical.y;  // camera.rs:70-72
    return camera_new_at(vadd(c.origin, {x, y, z}), aspect);
}

int parse_scene(const std::string &text, SceneModel &out) {
    if (!valid_utf8(text)) return kWouldPanic;  // CStr::to_str().unwrap(), lib.rs:39
    out = SceneModel{};
    std::unordered_map<std::string, Material> by_name;
    auto lookup = [&](const std::string &name) -> uint32_t {
        auto it = by_name.find(name);
        if (it == by_name.end()) throw ParseError{kWrongSyntax};
        out.materials.push_back(it->second);  // each primitive owns a copy
        return (uint32_t)(out.materials.size() - 1);
    };
    Scanner sc(text.data(), text.data() + text.size());
    try {
        sc.comments();
        if (!sc.eat("camera")) return kMissingCamera;
        sc.ws(); sc.need("origin"); sc.ws();
        Vec3 origin = sc.vec3(); sc.ws();
        sc.need("aspect"); sc.ws();
        float aspect = sc.number(); sc.ws();
        sc.need(";");
        out.camera = camera_new_at(origin, aspect);
        sc.ws();
        sc.comments();

        while (sc.eat("material")) {
            sc.ws();
            std::string name = sc.ident();
            sc.ws(); sc.need(":"); sc.ws();
            Material m{};
            m.a = 1.0f;  // Color::from(Vec3) / Color::new set alpha 1 (color.rs:21-23, 51-54)
            if (sc.eat("Diffuse")) {
                sc.ws(); sc.need("color"); sc.ws();
                Vec3 c = sc.vec3();
                m.kind = kDiffuse; m.r = c.x; m.g = c.y; m.b = c.z;
            } else if (sc.eat("Metal")) {
                sc.ws(); sc.need("color"); sc.ws();
                Vec3 c = sc.vec3(); sc.ws();
                sc.need("fuzz"); sc.ws();
                m.kind = kMetal; m.r = c.x; m.g = c.y; m.b = c.z; m.param = sc.number();
            } else if (sc.eat("Dielectric")) {
                sc.ws(); sc.need("ir"); sc.ws();
                m.kind = kDielectric; m.param = sc.number();
            } else {
                throw ParseError{kWrongSyntax};
            }
            sc.ws(); sc.need(";");
            by_name[name] = m;
            sc.ws();
            sc.comments();
        }
        while (sc.eat("sphere")) {
            sc.ws(); sc.need("center"); sc.ws();
            Sphere s;
            s.center = sc.vec3(); sc.ws();
            sc.need("radius"); sc.ws();
            s.radius = sc.number(); sc.ws();
            sc.need("material"); sc.ws();
            std::string name = sc.ident(); sc.ws();
            sc.need(";");
            s.material = lookup(name);
            out.spheres.push_back(s);
            sc.ws();
            sc.comments();
        }
        while (sc.eat("triangle")) {
            Triangle t;
            Vec3 *v[3] = {&t.v0, &t.v1, &t.v2};
            const char *kw[3] = {"v0", "v1", "v2"};
            sc.ws();
            for (int k = 0; k < 3; ++k) {
                sc.need(kw[k]); sc.ws();
                *v[k] = sc.vec3(); sc.ws();
            }
            sc.need("material"); sc.ws();
            std::string name = sc.ident(); sc.ws();
            sc.need(";");
            t.material = lookup(name);
            t.normal = vnormalize(vcross(vsub(t.v1, t.v0), vsub(t.v2, t.v0)));  // common.rs:116-123
            out.triangles.push_back(t);
            sc.ws();
            sc.comments();
        }
        if (!sc.at_end()) return kWrongSyntax;
    } catch (const ParseError &e) {
        return e.status;
    }
    return kParseOk;
}

static inline float u32_bits(uint32_t u) { float f; std::memcpy(&f, &u, 4); return f; }

PackedScene pack_scene(const SceneModel &s, uint32_t sphere_pad, uint32_t tri_pad) {
    PackedScene p;
    p.nsph = (uint32_t)s.spheres.size();
    p.nsph_padded = (p.nsph + sphere_pad - 1) / sphere_pad * sphere_pad;
    if (p.nsph_padded == 0) p.nsph_padded = sphere_pad;
    p.sph_hot.assign((size_t)p.nsph_padded * 4, std::nanf(""));  // NaN centre: never hit
    p.sph_cold.assign((size_t)p.nsph_padded * 4, 0.0f);
    for (uint32_t i = 0; i < p.nsph; ++i) {
        const Sphere &q = s.spheres[i];
        float *h = &p.sph_hot[(size_t)i * 4];
        h[0] = q.center.x; h[1] = q.center.y; h[2] = q.center.z;
        h[3] = q.radius * q.radius;  // radius.powi(2) (common.rs:77)
        float *c = &p.sph_cold[(size_t)i * 4];
        c[0] = q.radius; c[1] = u32_bits(q.material);
    }
    p.ntri = (uint32_t)s.triangles.size();
    p.ntri_padded = tri_pad ? (p.ntri + tri_pad - 1) / tri_pad * tri_pad : p.ntri;
    if (p.ntri_padded == 0) p.ntri_padded = 1;
    p.tri_hot.assign((size_t)p.ntri_padded * 4, 0.0f);  // n = 0 -> "parallel", never hit
    p.tri_geo.assign((size_t)p.ntri_padded * 16, 0.0f);
    for (uint32_t i = 0; i < p.ntri; ++i) {
        const Triangle &t = s.triangles[i];
        Vec3 n = vcross(vsub(t.v1, t.v0), vsub(t.v2, t.v0));  // common.rs:131-133
        float *h = &p.tri_hot[(size_t)i * 4];
        h[0] = n.x; h[1] = n.y; h[2] = n.z;
        h[3] = vdot(n, t.v0);  // common.rs:140
        float *g = &p.tri_geo[(size_t)i * 16];
        g[0] = t.v0.x; g[1] = t.v0.y; g[2] = t.v0.z; g[3] = u32_bits(t.material);
        g[4] = t.v1.x; g[5] = t.v1.y; g[6] = t.v1.z;
        g[8] = t.v2.x; g[9] = t.v2.y; g[10] = t.v2.z;
        g[12] = t.normal.x; g[13] = t.normal.y; g[14] = t.normal.z;
    }
    p.sph_shade.assign((size_t)p.nsph_padded * 8, 0.0f);
    p.sph_kind.assign(p.nsph_padded, 0u);
    for (uint32_t i = 0; i < p.nsph; ++i) {
        const Sphere &q = s.spheres[i];
        const Material &m = s.materials[q.material];
        float *o = &p.sph_shade[(size_t)i * 8];
        o[0] = q.center.x; o[1] = q.center.y; o[2] = q.center.z; o[3] = q.radius;
        o[4] = m.r; o[5] = m.g; o[6] = m.b; o[7] = m.param;
        p.sph_kind[i] = m.kind;
    }
    p.mats.assign(s.materials.size() ? s.materials.size() * 8 : 8, 0.0f);
    for (size_t i = 0; i < s.materials.size(); ++i) {
        const Material &m = s.materials[i];
        float *o = &p.mats[i * 8];
        o[0] = u32_bits(m.kind); o[1] = m.r; o[2] = m.g; o[3] = m.b; o[4] = m.param;
    }
    return p;
}

}  // namespace rtamd
