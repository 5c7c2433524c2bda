// rt_oracle.cpp -- CPU oracle: strict-IEEE binary32 restatement of the
// reference raytracer crate's render path.  TEST INFRASTRUCTURE ONLY (see
// rt_oracle.h): tests/, __graft_entry__.smoke() and bench.py's cpu_baseline
// leg are the only users.  Never linked into the product library.
//
// Build: g++ -O2 -ffp-contract=off (no fast-math): every `a*b+c` below must
// round twice, exactly like Rust's uncontracted f32 arithmetic.
//
// Parity: "full-frame parity unpinned by the reference" -- the reference is
// Rust and cannot be built here (no cargo/rustc).  Pinned by the reference's
// KATs (maths.rs:243-286) and cross-checked bit-for-bit against the
// independent numpy restatement in tests/pyref.py.
//
// Every function cites the reference file:line it restates.  Paths are
// relative to raytracer/src/ of Naxaes/Rust-Swift-Raytracer.

#include "rt_oracle.h"
#include "../rust-swift-raytracer_amd/csrc/unicode_alnum.h"

#include <clocale>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <locale.h>
#include <limits>
#include <map>
#include <string>
#include <thread>
#include <vector>

namespace {

// ---------------------------------------------------------------- maths.rs
struct V3 { float x, y, z; };

// maths.rs:146 / 152 / 158 / 164 -- component-wise, new_unchecked (no renorm).
inline V3 add(V3 a, V3 b) { return {a.x + b.x, a.y + b.y, a.z + b.z}; }
inline V3 sub(V3 a, V3 b) { return {a.x - b.x, a.y - b.y, a.z - b.z}; }
// maths.rs:204-208: Vec3*f32 -> lhs.x*rhs; f32*Vec3 -> rhs.x*self (same bits).
inline V3 muls(V3 a, float s) { return {a.x * s, a.y * s, a.z * s}; }
// maths.rs:210-214
inline V3 divs(V3 a, float s) { return {a.x / s, a.y / s, a.z / s}; }
// maths.rs:217
inline V3 neg(V3 a) { return {-a.x, -a.y, -a.z}; }
// maths.rs:82 / 125: (x*x' + y*y') + z*z'
inline float dot(V3 a, V3 b) { return a.x * b.x + a.y * b.y + a.z * b.z; }
// maths.rs:88-94
inline V3 cross(V3 a, V3 b) {
    return {a.y * b.z - a.z * b.y, -(a.x * b.z - a.z * b.x), a.x * b.y - a.y * b.x};
}
// maths.rs:111-118 (NVec3::new): len = sqrt((x*x + y*y) + z*z); divide each.
inline V3 normalize(V3 a) {
    float len = std::sqrt(a.x * a.x + a.y * a.y + a.z * a.z);
    return {a.x / len, a.y / len, a.z / len};
}
// maths.rs:46-49
inline bool near_zero(V3 a) {
    const float s = 1e-8f;
    return std::fabs(a.x) < s && std::fabs(a.y) < s && std::fabs(a.z) < s;
}
// maths.rs:26-28: v - 2.0*v.dot(n)*n, evaluated as v - ((2*dot) * n)
inline V3 reflect(V3 v, V3 n) { return sub(v, muls(n, 2.0f * dot(v, n))); }
// maths.rs:31-36
inline V3 refract(V3 uv, V3 n, float eta) {
    float cos_theta = dot(neg(uv), n);                       // NVec3::dot(&-uv, &n)
    V3 perp = muls(add(uv, muls(n, cos_theta)), eta);        // eta * (uv + cos*n)
    float par_s = -std::sqrt(std::fabs(1.0f - dot(perp, perp)));
    V3 par = muls(n, par_s);                                 // (-sqrt|..|) * n
    return add(perp, par);
}

// ---------------------------------------------------------------- color.rs
struct C4 { float r, g, b, a; };
inline C4 color3(float r, float g, float b) { return {r, g, b, 1.0f}; }        // color.rs:21-23
inline C4 add_a(C4 x, C4 y) { return {x.r + y.r, x.g + y.g, x.b + y.b, x.a + y.a}; }  // :30-32
inline C4 mul_a(C4 x, C4 y) { return {x.r * y.r, x.g * y.g, x.b * y.b, x.a * y.a}; }  // :36-38

// ---------------------------------------------------------------- random.rs
struct Rng {
    uint32_t s;
    uint32_t next() {  // random.rs:22-30
        uint32_t x = s;
        x ^= x << 13;
        x ^= x >> 17;
        x ^= x << 5;
        s = x;
        return x;
    }
    // random.rs:15-17: `x as f32 / u32::MAX as f32`; u32::MAX as f32 == 2^32.
    float f32() { return (float)next() / 4294967296.0f; }
    float bilateral() { return f32() * 2.0f - 1.0f; }  // random.rs:19-21
};
const uint32_t kDefaultSeed = 2547549u;  // random.rs:9

// common.rs:32-38: NVec3::new(bx, by, bz) -- args evaluated x, y, z.
inline V3 random_unit_sphere(Rng &r) {
    float x = r.bilateral();
    float y = r.bilateral();
    float z = r.bilateral();
    return normalize({x, y, z});
}

// ---------------------------------------------------------------- materials.rs
enum MatType { DIFFUSE = 0, METAL = 1, DIELECTRIC = 2, EMISSION = 3 };  // materials.rs:7-12
struct Material { int type; C4 color; float param; };  // param = fuzz | ir

// ---------------------------------------------------------------- camera.rs
struct Camera { V3 origin, llc, horizontal, vertical; };  // camera.rs:8-15
Camera camera_new_at(V3 origin, float aspect) {  // camera.rs:21-33
    float vh = 2.0f;
    float vw = aspect * vh;
    float focal = 1.0f;
    Camera c;
    c.origin = origin;
    c.horizontal = {vw, 0.0f, 0.0f};
    c.vertical = {0.0f, vh, 0.0f};
    c.llc = sub(origin, V3{vw / 2.0f, vh / 2.0f, focal});
    return c;
}
struct Ray { V3 o, d; };
// camera.rs:84-89: ((llc + s*h) + t*v) - origin, normalised.
inline Ray cast_ray(const Camera &c, float s, float t) {
    V3 p = sub(add(add(c.llc, muls(c.horizontal, s)), muls(c.vertical, t)), c.origin);
    return {c.origin, normalize(p)};
}
inline V3 ray_at(const Ray &r, float t) { return add(r.o, muls(r.d, t)); }  // common.rs:20

// ---------------------------------------------------------------- common.rs
struct Sphere { V3 center; float radius; Material mat; };
struct Triangle { V3 v0, v1, v2, normal; Material mat; };
struct Hit { V3 position, normal; float t; const Material *mat; };

struct Counters { uint64_t rays = 0, sph = 0, tri = 0, tri_in = 0; };

// common.rs:59-98
bool sphere_hit(const Sphere &sp, const Ray &ray, float t_min, float t_max, Hit &out) {
    V3 oc = sub(ray.o, sp.center);
    float a = 1.0f;  // NVec3::length_squared() returns 1.0 (maths.rs:127)
    float half_b = dot(oc, ray.d);
    float c = dot(oc, oc) - sp.radius * sp.radius;  // powi(2) == r*r
    float disc = half_b * half_b - a * c;
    if (disc < 0.0f) return false;
    float sq = std::sqrt(disc);
    float roots[2] = {(-half_b - sq) / a, (-half_b + sq) / a};
    // filter(t_min < x && x < t_max).min_by(partial_cmp): first minimum wins.
    bool found = false;
    float t = 0.0f;
    for (float x : roots) {
        if (t_min < x && x < t_max) {
            if (!found || x < t) { t = x; found = true; }
        }
    }
    if (!found) return false;
    out.position = ray_at(ray, t);
    out.normal = normalize(divs(sub(out.position, sp.center), sp.radius));
    out.t = t;
    out.mat = &sp.mat;
    return true;
}

// common.rs:124-166 (including the `n.dot(origin) + d` sign quirk at :141).
bool triangle_intersect(const Triangle &tr, const Ray &ray, float t_min, float t_max,
                        Hit &out, Counters *cnt) {
    V3 a = sub(tr.v1, tr.v0);
    V3 b = sub(tr.v2, tr.v0);
    V3 n = cross(a, b);
    float cosl = dot(n, ray.d);
    if (-1e-8f < cosl && cosl < 1e-8f) return false;  // is_zero
    float d = dot(n, tr.v0);
    float t = (dot(n, ray.o) + d) / cosl;
    if (t < t_min || t > t_max) return false;
    if (cnt) cnt->tri_in++;
    V3 p = ray_at(ray, t);
    V3 e0 = sub(tr.v1, tr.v0), vp0 = sub(p, tr.v0);
    if (dot(n, cross(e0, vp0)) < 0.0f) return false;
    V3 e1 = sub(tr.v2, tr.v1), vp1 = sub(p, tr.v1);
    if (dot(n, cross(e1, vp1)) < 0.0f) return false;
    V3 e2 = sub(tr.v0, tr.v2), vp2 = sub(p, tr.v2);
    if (dot(n, cross(e2, vp2)) < 0.0f) return false;
    out.position = p;
    out.normal = tr.normal;
    out.t = t;
    out.mat = &tr.mat;
    return true;
}

struct World {
    std::vector<Sphere> spheres;
    std::vector<Triangle> triangles;  // the single Mesh built by lib.rs:41
};

// common.rs:237-258 (spheres in order, then Mesh::hit common.rs:178-223).
bool world_hit(const World &w, const Ray &ray, Hit &rec, Counters &cnt) {
    cnt.rays++;
    float closest = std::numeric_limits<float>::infinity();
    bool have = false;
    for (const Sphere &s : w.spheres) {
        cnt.sph++;
        Hit h;
        if (sphere_hit(s, ray, 0.001f, closest, h)) { closest = h.t; rec = h; have = true; }
    }
    // Mesh::hit with t_max = closest; its own closest_intersection starts at +inf.
    bool mesh_have = false;
    Hit mrec;
    float mclosest = std::numeric_limits<float>::infinity();
    for (const Triangle &t : w.triangles) {
        cnt.tri++;
        Hit h;
        if (triangle_intersect(t, ray, 0.001f, closest, h, &cnt)) {
            if (h.t < mclosest) { mclosest = h.t; mrec = h; mesh_have = true; }
        }
    }
    if (mesh_have) { rec = mrec; have = true; }
    return have;
}

struct Scatter { C4 color; bool has_next; Ray next; };

// materials.rs:26-28
inline bool hit_front_face(V3 dir, V3 n) { return dot(dir, n) >= 0.0f; }

// materials.rs:30-102
Scatter scatter(const Material &m, const Ray &ray, const Hit &hit, Rng &rng) {
    Scatter s;
    switch (m.type) {
    case DIFFUSE: {  // :42-52
        V3 sc = add(hit.normal, random_unit_sphere(rng));
        s.color = m.color;
        s.has_next = true;
        s.next = near_zero(sc) ? Ray{hit.position, hit.normal} : Ray{hit.position, normalize(sc)};
        break;
    }
    case METAL: {  // :54-63
        V3 reflected = reflect(ray.d, hit.normal);
        V3 dir = add(reflected, muls(random_unit_sphere(rng), m.param));
        s.color = m.color;
        if (hit_front_face(dir, hit.normal)) {
            s.has_next = true;
            s.next = Ray{hit.position, normalize(dir)};
        } else {
            s.has_next = false;
        }
        break;
    }
    case DIELECTRIC: {  // :65-97 (inverted "front face" convention kept)
        V3 n;
        float ratio;
        if (hit_front_face(ray.d, hit.normal)) { n = neg(hit.normal); ratio = 1.0f / m.param; }
        else { n = hit.normal; ratio = m.param; }
        V3 refr = refract(ray.d, n, ratio);
        s.color = color3(1.0f, 1.0f, 1.0f);
        s.has_next = true;
        s.next = Ray{hit.position, normalize(refr)};
        break;
    }
    default: {  // EMISSION :100-102
        s.color = m.color;
        s.has_next = false;
        break;
    }
    }
    return s;
}

// common.rs:276-281: t = 0.5*(dir.normalize().y + 1); lerp((1,1,1),(0.5,0.7,1),t)
inline C4 sky(V3 dir) {
    float t = 0.5f * (normalize(dir).y + 1.0f);
    V3 a = muls(V3{1.0f, 1.0f, 1.0f}, 1.0f - t);
    V3 b = muls(V3{0.5f, 0.7f, 1.0f}, t);
    V3 c = add(a, b);
    return color3(c.x, c.y, c.z);
}

// common.rs:263-285
C4 ray_color(const Ray &ray0, const World &w, Rng &rng, int depth, Counters &cnt) {
    Ray ray = ray0;
    C4 fin = color3(1.0f, 1.0f, 1.0f);
    for (int i = 0; i < depth; ++i) {
        Hit hit;
        if (world_hit(w, ray, hit, cnt)) {
            Scatter sc = scatter(*hit.mat, ray, hit, rng);
            if (sc.has_next) {
                fin = mul_a(fin, sc.color);
                ray = sc.next;
            } else {
                return mul_a(fin, sc.color);
            }
        } else {
            return mul_a(fin, sky(ray.d));
        }
    }
    return color3(0.0f, 0.0f, 0.0f);  // Vec3::new_zero().into()
}

// Rust `f32 as u8`: saturating, NaN -> 0, truncation toward zero.
inline uint8_t as_u8(float x) {
    if (!(x > 0.0f)) return 0;  // NaN, <= 0 (incl. -0.0)
    if (x >= 255.0f) return 255;
    return (uint8_t)x;
}

}  // namespace

// ---------------------------------------------------------------- parser.rs
namespace {

// ParseError discriminants (parser.rs:11-18); 100 = the reference would panic.
enum PErr { P_OK = -1, P_COULDNT_OPEN = 0, P_MISSING_CAMERA = 1, P_WRONG_SYNTAX = 2,
            P_DIDNT_START_WITH = 3, P_NOT_I32 = 4, P_NOT_F32 = 5, P_PANIC = 100 };
thread_local int g_parse_error = P_OK;

struct PFail { int code; };

// Decode one UTF-8 code point at s[i]; returns its length.
size_t utf8_decode(const std::string &s, size_t i, uint32_t &cp) {
    unsigned char c = (unsigned char)s[i];
    if (c < 0x80) { cp = c; return 1; }
    size_t n = (c >= 0xF0) ? 4 : (c >= 0xE0) ? 3 : 2;
    cp = c & (0xFF >> (n + 1));
    for (size_t k = 1; k < n && i + k < s.size(); ++k) cp = (cp << 6) | ((unsigned char)s[i + k] & 0x3F);
    return n;
}
bool is_boundary(const std::string &s, size_t i) {
    return i >= s.size() || ((unsigned char)s[i] & 0xC0) != 0x80;
}
// char::is_whitespace (Unicode White_Space).
bool is_ws(uint32_t c) {
    return (c >= 0x09 && c <= 0x0D) || c == 0x20 || c == 0x85 || c == 0xA0 || c == 0x1680 ||
           (c >= 0x2000 && c <= 0x200A) || c == 0x2028 || c == 0x2029 || c == 0x202F ||
           c == 0x205F || c == 0x3000;
}
// char::is_alphanumeric (parser.rs:60): Alphabetic || Nd/Nl/No, Unicode
// 13.0.0.  The ranges are Unicode data (tools/gen_unicode_alnum.py, from perl's
// unicore Alphabetic table and Python's unicodedata), shared with the product;
// tests/test_parser.py checks both parsers against those sources directly.
bool is_alnum(uint32_t c) {
    if (c < 0x80) return (c >= '0' && c <= '9') || (c >= 'a' && c <= 'z') || (c >= 'A' && c <= 'Z');
    for (uint32_t i = 0; i < rtamd::kAlnumRangeCount; ++i) {  // linear: the oracle favours plainness
        if (c < rtamd::kAlnumRanges[i][0]) return false;
        if (c <= rtamd::kAlnumRanges[i][1]) return true;
    }
    return false;
}

// A cursor over the (NUL-terminated) source, mirroring the &str slices.
struct Src { const std::string *s; size_t i; };

Src skip_whitespace(Src x) {  // parser.rs:54-57
    while (x.i < x.s->size()) {
        uint32_t cp;
        size_t n = utf8_decode(*x.s, x.i, cp);
        if (!is_ws(cp)) break;
        x.i += n;
    }
    return x;
}
std::string get_identifier(Src &x) {  // parser.rs:59-62
    size_t j = x.i;
    while (j < x.s->size()) {
        uint32_t cp;
        size_t n = utf8_decode(*x.s, j, cp);
        if (!(is_alnum(cp) || cp == '_')) break;
        j += n;
    }
    std::string id = x.s->substr(x.i, j - x.i);
    x.i = j;
    return id;
}
// parser.rs:81-88 (a slice end off a char boundary panics in Rust)
bool starts_with(Src x, const char *t, Src &rest) {
    size_t n = std::strlen(t);
    size_t len = x.s->size() - x.i;
    if (len >= n) {
        if (!is_boundary(*x.s, x.i + n)) throw PFail{P_PANIC};
        if (x.s->compare(x.i, n, t) == 0) { rest = Src{x.s, x.i + n}; return true; }
    }
    return false;
}
Src expect(Src x, const char *t) {
    Src r;
    if (!starts_with(x, t, r)) throw PFail{P_DIDNT_START_WITH};
    return r;
}
// parser.rs:65-77 with target "\n" (char-boundary panics reproduced).
bool find_newline(Src x, Src &at) {
    for (size_t i = x.i; i + 1 <= x.s->size(); ++i) {
        if (!is_boundary(*x.s, i) || !is_boundary(*x.s, i + 1)) throw PFail{P_PANIC};
        if ((*x.s)[i] == '\n') { at = Src{x.s, i}; return true; }
    }
    return false;
}

locale_t c_locale() {
    static locale_t loc = newlocale(LC_ALL_MASK, "C", (locale_t)0);
    return loc;
}

// parser.rs:107-133; `parse::<f32>` is correctly rounded -> strtof_l on the slice.
Src parse_float(Src x, float &out) {
    const std::string &s = *x.s;
    size_t len = s.size() - x.i;
    if (len < 3) throw PFail{P_NOT_F32};
    size_t idx = 0;
    if (s[x.i] == '-') idx = 1;
    bool dot = false;
    while (x.i + idx < s.size()) {
        char c = s[x.i + idx];
        if (c >= '0' && c <= '9') ++idx;
        else if (c == '.') { if (dot) throw PFail{P_NOT_F32}; dot = true; ++idx; }
        else break;
    }
    std::string lit = s.substr(x.i, idx);
    // Rust grammar: [-] (Digit+ | Digit+ '.' Digit* | Digit* '.' Digit+)
    bool has_digit = false;
    for (char c : lit) has_digit |= (c >= '0' && c <= '9');
    if (!has_digit) throw PFail{P_NOT_F32};
    char *end = nullptr;
    out = strtof_l(lit.c_str(), &end, c_locale());
    if (end != lit.c_str() + lit.size()) throw PFail{P_NOT_F32};
    return Src{x.s, x.i + idx};
}
Src parse_vec3(Src x, V3 &v) {  // parser.rs:135-142
    x = parse_float(x, v.x);
    x = skip_whitespace(x);
    x = parse_float(x, v.y);
    x = skip_whitespace(x);
    x = parse_float(x, v.z);
    return x;
}
Src skip_comment(Src x) {  // parser.rs:313-323
    Src line;
    while (starts_with(x, "//", line)) {
        Src nl;
        if (find_newline(line, nl)) x = Src{x.s, nl.i + 1};
        else throw PFail{P_WRONG_SYNTAX};
    }
    return x;
}

}  // namespace

struct ro_scene {
    World world;
    Camera camera;
};

extern "C" {

int ro_last_parse_error(void) { return g_parse_error; }

// parser.rs:336-381 (parse_camera 145-167, parse_material 175-234,
// parse_sphere 237-269, parse_triangle 272-310).
ro_scene *ro_parse(const char *source) {
    g_parse_error = P_OK;
    std::string text(source ? source : "");
    // CStr::to_str().unwrap() (lib.rs:39): invalid UTF-8 panics.
    for (size_t i = 0; i < text.size();) {
        unsigned char c = (unsigned char)text[i];
        size_t n = c < 0x80 ? 1 : (c >> 5) == 6 ? 2 : (c >> 4) == 14 ? 3 : (c >> 3) == 30 ? 4 : 0;
        if (n == 0 || i + n > text.size()) { g_parse_error = P_PANIC; return nullptr; }
        for (size_t k = 1; k < n; ++k)
            if (((unsigned char)text[i + k] & 0xC0) != 0x80) { g_parse_error = P_PANIC; return nullptr; }
        i += n;
    }
    ro_scene *scene = new ro_scene();
    try {
        std::map<std::string, Material> materials;
        Src x{&text, 0};
        x = skip_comment(x);
        Src r;
        if (!starts_with(x, "camera", r)) throw PFail{P_MISSING_CAMERA};
        {
            Src y = skip_whitespace(r);
            y = expect(y, "origin");
            y = skip_whitespace(y);
            V3 o;
            y = parse_vec3(y, o);
            y = skip_whitespace(y);
            y = expect(y, "aspect");
            y = skip_whitespace(y);
            float a;
            y = parse_float(y, a);
            y = skip_whitespace(y);
            y = expect(y, ";");
            scene->camera = camera_new_at(o, a);
            x = skip_whitespace(y);
        }
        x = skip_comment(x);
        while (starts_with(x, "material", r)) {
            Src y = skip_whitespace(r);
            std::string name = get_identifier(y);
            y = skip_whitespace(y);
            y = expect(y, ":");
            y = skip_whitespace(y);
            Material m{};
            Src z;
            if (starts_with(y, "Diffuse", z)) {
                z = skip_whitespace(z);
                z = expect(z, "color");
                z = skip_whitespace(z);
                V3 c;
                z = parse_vec3(z, c);
                z = skip_whitespace(z);
                z = expect(z, ";");
                m.type = DIFFUSE; m.color = color3(c.x, c.y, c.z); m.param = 0.0f;
            } else if (starts_with(y, "Metal", z)) {
                z = skip_whitespace(z);
                z = expect(z, "color");
                z = skip_whitespace(z);
                V3 c;
                z = parse_vec3(z, c);
                z = skip_whitespace(z);
                z = expect(z, "fuzz");
                z = skip_whitespace(z);
                float f;
                z = parse_float(z, f);
                z = skip_whitespace(z);
                z = expect(z, ";");
                m.type = METAL; m.color = color3(c.x, c.y, c.z); m.param = f;
            } else if (starts_with(y, "Dielectric", z)) {
                z = skip_whitespace(z);
                z = expect(z, "ir");
                z = skip_whitespace(z);
                float ir;
                z = parse_float(z, ir);
                z = skip_whitespace(z);
                z = expect(z, ";");
                m.type = DIELECTRIC; m.color = color3(0.0f, 0.0f, 0.0f); m.param = ir;
            } else {
                throw PFail{P_WRONG_SYNTAX};
            }
            materials[name] = m;
            x = skip_whitespace(z);
            x = skip_comment(x);
        }
        while (starts_with(x, "sphere", r)) {
            Src y = skip_whitespace(r);
            y = expect(y, "center");
            y = skip_whitespace(y);
            V3 c;
            y = parse_vec3(y, c);
            y = skip_whitespace(y);
            y = expect(y, "radius");
            y = skip_whitespace(y);
            float rad;
            y = parse_float(y, rad);
            y = skip_whitespace(y);
            y = expect(y, "material");
            y = skip_whitespace(y);
            std::string m = get_identifier(y);
            y = skip_whitespace(y);
            y = expect(y, ";");
            auto it = materials.find(m);
            if (it == materials.end()) throw PFail{P_WRONG_SYNTAX};
            scene->world.spheres.push_back(Sphere{c, rad, it->second});
            x = skip_whitespace(y);
            x = skip_comment(x);
        }
        while (starts_with(x, "triangle", r)) {
            Src y = skip_whitespace(r);
            V3 v[3];
            const char *kw[3] = {"v0", "v1", "v2"};
            for (int k = 0; k < 3; ++k) {
                y = expect(y, kw[k]);
                y = skip_whitespace(y);
                y = parse_vec3(y, v[k]);
                y = skip_whitespace(y);
            }
            y = expect(y, "material");
            y = skip_whitespace(y);
            std::string m = get_identifier(y);
            y = skip_whitespace(y);
            y = expect(y, ";");
            auto it = materials.find(m);
            if (it == materials.end()) throw PFail{P_WRONG_SYNTAX};
            // Triangle::new (common.rs:116-123)
            Triangle t;
            t.v0 = v[0]; t.v1 = v[1]; t.v2 = v[2];
            t.normal = normalize(cross(sub(v[1], v[0]), sub(v[2], v[0])));
            t.mat = it->second;
            scene->world.triangles.push_back(t);
            x = skip_whitespace(y);
            x = skip_comment(x);
        }
        if (x.i != text.size()) throw PFail{P_WRONG_SYNTAX};
    } catch (const PFail &f) {
        g_parse_error = f.code;
        delete scene;
        return nullptr;
    }
    return scene;
}

void ro_scene_free(ro_scene *s) { delete s; }
size_t ro_scene_num_spheres(const ro_scene *s) { return s->world.spheres.size(); }
size_t ro_scene_num_triangles(const ro_scene *s) { return s->world.triangles.size(); }

static void cam_out(const Camera &c, float o[12]) {
    const V3 v[4] = {c.origin, c.llc, c.horizontal, c.vertical};
    for (int i = 0; i < 4; ++i) { o[3 * i] = v[i].x; o[3 * i + 1] = v[i].y; o[3 * i + 2] = v[i].z; }
}
static Camera cam_in(const float o[12]) {
    Camera c;
    V3 *v[4] = {&c.origin, &c.llc, &c.horizontal, &c.vertical};
    for (int i = 0; i < 4; ++i) *v[i] = V3{o[3 * i], o[3 * i + 1], o[3 * i + 2]};
    return c;
}
void ro_scene_camera(const ro_scene *s, float camera[12]) { cam_out(s->camera, camera); }
void ro_scene_set_camera(ro_scene *s, const float camera[12]) { s->camera = cam_in(camera); }

static void mat_out(const Material &m, float o[6]) {
    o[0] = (float)m.type; o[1] = m.color.r; o[2] = m.color.g; o[3] = m.color.b; o[4] = m.color.a;
    o[5] = m.param;
}
static Material mat_in(const float o[6]) {
    Material m;
    m.type = (int)o[0]; m.color = C4{o[1], o[2], o[3], o[4]}; m.param = o[5];
    return m;
}

// Test hook: replaces one primitive's material (each owns a copy, as
// parser.rs:237-310 clone the named material), e.g. with Emission
// (materials.rs:100-102), which the grammar cannot produce.
int ro_scene_set_material(ro_scene *s, int triangle, size_t i, const float m[6]) {
    if (triangle) {
        if (i >= s->world.triangles.size()) return -1;
        s->world.triangles[i].mat = mat_in(m);
    } else {
        if (i >= s->world.spheres.size()) return -1;
        s->world.spheres[i].mat = mat_in(m);
    }
    return 0;
}
void ro_scene_sphere(const ro_scene *s, size_t i, float out[10]) {
    const Sphere &sp = s->world.spheres[i];
    out[0] = sp.center.x; out[1] = sp.center.y; out[2] = sp.center.z; out[3] = sp.radius;
    mat_out(sp.mat, out + 4);
}
void ro_scene_triangle(const ro_scene *s, size_t i, float out[18]) {
    const Triangle &t = s->world.triangles[i];
    const V3 v[4] = {t.v0, t.v1, t.v2, t.normal};
    for (int k = 0; k < 4; ++k) { out[3 * k] = v[k].x; out[3 * k + 1] = v[k].y; out[3 * k + 2] = v[k].z; }
    mat_out(t.mat, out + 12);
}

void ro_camera_new_at(const float origin[3], float aspect, float camera[12]) {
    cam_out(camera_new_at(V3{origin[0], origin[1], origin[2]}, aspect), camera);
}
// lib.rs:60-63: Camera::new_at(position + (x,y,z), aspect_ratio()); camera.rs:70-72
void ro_camera_move(const float ci[12], float x, float y, float z, float co[12]) {
    Camera c = cam_in(ci);
    float aspect = c.horizontal.x / c.vertical.y;
    cam_out(camera_new_at(add(c.origin, V3{x, y, z}), aspect), co);
}

// Counter-mode seed: splitmix64 finaliser of (seed, job), folded to a nonzero u32.
uint32_t ro_sample_seed(uint32_t base_seed, uint64_t job) {
    uint64_t z = job + (uint64_t)base_seed * 0x9E3779B97F4A7C15ull + 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    z ^= z >> 31;
    uint32_t s = (uint32_t)(z ^ (z >> 32));
    return s ? s : kDefaultSeed;
}

// ray_trace, common.rs:320-361, generalised (see header).
static void trace_rows(const ro_scene *sc, size_t W, size_t H, int spp, int depth, int mode,
                       uint32_t seed, const uint32_t *replay, size_t row_begin, size_t row_step,
                       size_t col_begin, size_t col_step, size_t thread, size_t nthreads, uint8_t *out,
                       uint32_t *states, float *sample_rgba, Counters &cnt, uint64_t &samples) {
    Rng rng{seed ? seed : kDefaultSeed};
    const float wden = (float)(W - 1);  // (width-1) as f32
    const float hden = (float)(H - 1);
    const float inv_spp = 1.0f / (float)spp;
    size_t k = 0;
    for (size_t row = row_begin; row < H; row += row_step, ++k) {
        for (size_t col = col_begin; col < W; col += col_step) {
            // (pixels dealt cyclically over the threads: a single row still
            // uses every thread; per-sample RNG modes only)
            if ((k * W + col) % nthreads != thread) continue;
            C4 color = color3(0.0f, 0.0f, 0.0f);  // alpha starts at 1.0
            for (int s = 0; s < spp; ++s) {
                uint64_t job = ((uint64_t)row * W + col) * (uint64_t)spp + (uint64_t)s;
                if (mode == RO_RNG_COUNTER) rng.s = ro_sample_seed(seed, job);
                else if (mode == RO_RNG_REPLAY) rng.s = replay[job];
                if (states) states[job] = rng.s;
                float u = ((float)col + rng.f32()) / wden;
                float v = ((float)row + rng.f32()) / hden;
                Ray ray = cast_ray(sc->camera, u, v);
                C4 c = ray_color(ray, sc->world, rng, depth, cnt);
                if (sample_rgba) {
                    float *o = sample_rgba + job * 4;
                    o[0] = c.r; o[1] = c.g; o[2] = c.b; o[3] = c.a;
                }
                color = add_a(color, c);
                ++samples;
            }
            // Gamma (common.rs:344-349): sqrt(c * (1/spp)) * 255.999; alpha without sqrt.
            float r = std::sqrt(color.r * inv_spp) * 255.999f;
            float g = std::sqrt(color.g * inv_spp) * 255.999f;
            float b = std::sqrt(color.b * inv_spp) * 255.999f;
            float a = color.a * inv_spp * 255.999f;
            uint8_t *px = out + ((H - row - 1) * W + col) * 4;  // fb[[H-row-1, col]]
            px[0] = as_u8(r); px[1] = as_u8(g); px[2] = as_u8(b); px[3] = as_u8(a);
        }
    }
}

int ro_render(const ro_scene *s, size_t width, size_t height, int spp, int depth, int rng_mode,
              uint32_t seed, const uint32_t *replay_states, size_t row_begin, size_t row_step,
              int nthreads, uint8_t *out_rgba, uint32_t *sample_states, float *sample_rgba,
              ro_stats *stats) {
    return ro_render_cols(s, width, height, spp, depth, rng_mode, seed, replay_states, row_begin, row_step, 0,
                          1, nthreads, out_rgba, sample_states, sample_rgba, stats);
}

int ro_render_cols(const ro_scene *s, size_t width, size_t height, int spp, int depth, int rng_mode,
                   uint32_t seed, const uint32_t *replay_states, size_t row_begin, size_t row_step,
                   size_t col_begin, size_t col_step, int nthreads, uint8_t *out_rgba,
                   uint32_t *sample_states, float *sample_rgba, ro_stats *stats) {
    if (!s || !out_rgba || row_step == 0 || col_step == 0) return -1;
    if (rng_mode == RO_RNG_SERIAL && (col_begin != 0 || col_step != 1)) return -1;  // (one stream: whole rows)
    if (rng_mode == RO_RNG_REPLAY && !replay_states) return -1;
    if (rng_mode == RO_RNG_SERIAL) nthreads = 1;  // one frame-wide stream: inherently serial
    if (nthreads < 1) nthreads = 1;
    std::vector<Counters> cnt((size_t)nthreads);
    std::vector<uint64_t> samples((size_t)nthreads, 0);
    if (nthreads == 1) {
        trace_rows(s, width, height, spp, depth, rng_mode, seed, replay_states, row_begin, row_step,
                   col_begin, col_step, 0, 1, out_rgba, sample_states, sample_rgba, cnt[0], samples[0]);
    } else {
        std::vector<std::thread> th;
        for (int t = 0; t < nthreads; ++t)
            th.emplace_back([&, t] {
                trace_rows(s, width, height, spp, depth, rng_mode, seed, replay_states, row_begin,
                           row_step, col_begin, col_step, (size_t)t, (size_t)nthreads, out_rgba, sample_states,
                           sample_rgba, cnt[(size_t)t], samples[(size_t)t]);
            });
        for (auto &x : th) x.join();
    }
    if (stats) {
        *stats = ro_stats{};
        for (int t = 0; t < nthreads; ++t) {
            stats->samples += samples[(size_t)t];
            stats->rays += cnt[(size_t)t].rays;
            stats->sphere_tests += cnt[(size_t)t].sph;
            stats->tri_tests += cnt[(size_t)t].tri;
            stats->tri_in_range += cnt[(size_t)t].tri_in;
        }
    }
    return 0;
}

// ---- known-answer hooks ----------------------------------------------------
uint32_t ro_xorshift32(uint32_t *state) { Rng r{*state}; uint32_t x = r.next(); *state = r.s; return x; }
float ro_random_f32(uint32_t *state) { Rng r{*state}; float x = r.f32(); *state = r.s; return x; }
void ro_reflect(const float v[3], const float n[3], float out[3]) {
    V3 r = reflect(V3{v[0], v[1], v[2]}, V3{n[0], n[1], n[2]});
    out[0] = r.x; out[1] = r.y; out[2] = r.z;
}
void ro_refract(const float uv[3], const float n[3], float eta, float out[3]) {
    V3 r = refract(V3{uv[0], uv[1], uv[2]}, V3{n[0], n[1], n[2]}, eta);
    out[0] = r.x; out[1] = r.y; out[2] = r.z;
}
void ro_normalize(const float v[3], float out[3]) {
    V3 r = normalize(V3{v[0], v[1], v[2]});
    out[0] = r.x; out[1] = r.y; out[2] = r.z;
}
static Ray ray_in(const float r[6]) { return Ray{V3{r[0], r[1], r[2]}, V3{r[3], r[4], r[5]}}; }
static void hit_out(const Hit &h, float o[7]) {
    o[0] = h.t; o[1] = h.position.x; o[2] = h.position.y; o[3] = h.position.z;
    o[4] = h.normal.x; o[5] = h.normal.y; o[6] = h.normal.z;
}
int ro_sphere_hit(const float ray[6], const float c[3], float radius, float t_min, float t_max,
                  float out[7]) {
    Sphere sp{V3{c[0], c[1], c[2]}, radius, Material{}};
    Hit h;
    if (!sphere_hit(sp, ray_in(ray), t_min, t_max, h)) return 0;
    hit_out(h, out);
    return 1;
}
int ro_triangle_intersect(const float ray[6], const float v[9], float t_min, float t_max,
                          float out[7]) {
    Triangle t;
    t.v0 = V3{v[0], v[1], v[2]}; t.v1 = V3{v[3], v[4], v[5]}; t.v2 = V3{v[6], v[7], v[8]};
    t.normal = normalize(cross(sub(t.v1, t.v0), sub(t.v2, t.v0)));
    t.mat = Material{};
    Hit h;
    if (!triangle_intersect(t, ray_in(ray), t_min, t_max, h, nullptr)) return 0;
    hit_out(h, out);
    return 1;
}
int ro_scatter(const float material[6], const float ray[6], const float hit[7], uint32_t *rng_state,
               float color[4], float next_ray[6]) {
    Material m = mat_in(material);
    Hit h;
    h.t = hit[0]; h.position = V3{hit[1], hit[2], hit[3]}; h.normal = V3{hit[4], hit[5], hit[6]};
    h.mat = &m;
    Rng r{*rng_state};
    Scatter s = scatter(m, ray_in(ray), h, r);
    *rng_state = r.s;
    color[0] = s.color.r; color[1] = s.color.g; color[2] = s.color.b; color[3] = s.color.a;
    if (s.has_next) {
        next_ray[0] = s.next.o.x; next_ray[1] = s.next.o.y; next_ray[2] = s.next.o.z;
        next_ray[3] = s.next.d.x; next_ray[4] = s.next.d.y; next_ray[5] = s.next.d.z;
    }
    return s.has_next ? 1 : 0;
}
void ro_sky(const float dir[3], const float fin[4], float out[4]) {
    C4 c = mul_a(C4{fin[0], fin[1], fin[2], fin[3]}, sky(V3{dir[0], dir[1], dir[2]}));
    out[0] = c.r; out[1] = c.g; out[2] = c.b; out[3] = c.a;
}
void ro_cast_ray(const float camera[12], float s, float t, float ray[6]) {
    Ray r = cast_ray(cam_in(camera), s, t);
    ray[0] = r.o.x; ray[1] = r.o.y; ray[2] = r.o.z; ray[3] = r.d.x; ray[4] = r.d.y; ray[5] = r.d.z;
}
uint8_t ro_as_u8(float x) { return as_u8(x); }

// image.rs:59-81
long ro_write_ppm(const uint8_t *rgba, size_t W, size_t H, char *buf, size_t cap) {
    std::string o = "P3\n" + std::to_string(W) + " " + std::to_string(H) + "\n255\n";
    for (size_t i = 0; i < W * H; ++i) {
        o += std::to_string(rgba[4 * i]) + " " + std::to_string(rgba[4 * i + 1]) + " " +
             std::to_string(rgba[4 * i + 2]) + "\n";
    }
    if (buf) {
        if (o.size() > cap) return -1;
        std::memcpy(buf, o.data(), o.size());
    }
    return (long)o.size();
}

}  // extern "C"
