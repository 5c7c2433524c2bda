"""Second, independent restatement of the reference render path in numpy float32.

TEST INFRASTRUCTURE ONLY.  Written directly from the reference Rust sources
(Naxaes/Rust-Swift-Raytracer raytracer/src/*.rs), without sharing code with
the C++ oracle, so that the two restatements cross-check each other
bit-for-bit.  Pure-Python scalar loops: use only on tiny frames.

Every numpy float32 scalar op below is one correctly rounded IEEE binary32
operation (numpy never fuses), which is exactly Rust's f32 semantics.
"""
from __future__ import annotations

from fractions import Fraction

import numpy as np

F = np.float32
INF = F(np.inf)
T_MIN = F(0.001)                      # common.rs:242,250
EPS8 = F(1e-8)                        # maths.rs:47, common.rs:135
GAMMA = F(255.999)                    # common.rs:345
U32MAX_F = F(4294967295)              # `u32::MAX as f32` == 2^32

np.seterr(all="ignore")


def dec_to_f32(lit: str) -> np.float32:
    """Correctly rounded decimal -> binary32 (Rust `str::parse::<f32>`)."""
    q = Fraction(lit)
    c = F(float(q))  # may be off by one ulp through double rounding
    best = None
    for cand in (np.nextafter(c, F(-np.inf)), c, np.nextafter(c, F(np.inf))):
        if not np.isfinite(cand):
            continue
        err = abs(Fraction(float(cand)) - q)
        key = (err, int(np.array(cand).view(np.uint32)) & 1)
        if best is None or key < best[0]:
            best = (key, cand)
    return best[1]


# ---------------------------------------------------------------- random.rs
class Random:
    def __init__(self, seed=2547549):
        self.state = seed & 0xFFFFFFFF

    def xor_shift_32(self):  # random.rs:22-30
        x = self.state
        x ^= (x << 13) & 0xFFFFFFFF
        x ^= x >> 17
        x ^= (x << 5) & 0xFFFFFFFF
        self.state = x
        return x

    def random_f32(self):  # random.rs:15-17
        return F(self.xor_shift_32()) / U32MAX_F

    def random_bilateral_f32(self):  # random.rs:19-21
        return self.random_f32() * F(2.0) - F(1.0)


# ---------------------------------------------------------------- maths.rs
def v(x, y, z):
    return (F(x), F(y), F(z))


def vadd(a, b):
    return (a[0] + b[0], a[1] + b[1], a[2] + b[2])


def vsub(a, b):
    return (a[0] - b[0], a[1] - b[1], a[2] - b[2])


def vmuls(a, s):
    return (a[0] * s, a[1] * s, a[2] * s)


def vdivs(a, s):
    return (a[0] / s, a[1] / s, a[2] / s)


def vneg(a):
    return (-a[0], -a[1], -a[2])


def vdot(a, b):
    return (a[0] * b[0] + a[1] * b[1]) + a[2] * b[2]


def vcross(a, b):
    return (a[1] * b[2] - a[2] * b[1], -(a[0] * b[2] - a[2] * b[0]), a[0] * b[1] - a[1] * b[0])


def nvec3(x, y, z):  # maths.rs:111-118
    length = np.sqrt((x * x + y * y) + z * z)
    return (x / length, y / length, z / length)


def normalize(a):
    return nvec3(*a)


def near_zero(a):
    return abs(a[0]) < EPS8 and abs(a[1]) < EPS8 and abs(a[2]) < EPS8


def reflect(vv, n):  # maths.rs:26-28
    return vsub(vv, vmuls(n, F(2.0) * vdot(vv, n)))


def refract(uv, n, eta):  # maths.rs:31-36
    cos_theta = vdot(vneg(uv), n)
    perp = vmuls(vadd(uv, vmuls(n, cos_theta)), eta)
    par = vmuls(n, -np.sqrt(abs(F(1.0) - vdot(perp, perp))))
    return vadd(perp, par)


# ---------------------------------------------------------------- camera.rs
def camera_new_at(origin, aspect):  # camera.rs:21-33
    vh = F(2.0)
    vw = aspect * vh
    horizontal = (vw, F(0.0), F(0.0))
    vertical = (F(0.0), vh, F(0.0))
    llc = vsub(origin, (vw / F(2.0), vh / F(2.0), F(1.0)))
    return {"origin": origin, "llc": llc, "h": horizontal, "v": vertical}


def cast_ray(cam, s, t):  # camera.rs:84-89
    p = vsub(vadd(vadd(cam["llc"], vmuls(cam["h"], s)), vmuls(cam["v"], t)), cam["origin"])
    return (cam["origin"], normalize(p))


def at(ray, t):
    return vadd(ray[0], vmuls(ray[1], t))


# ---------------------------------------------------------------- common.rs
def sphere_hit(center, radius, ray, t_min, t_max):  # common.rs:59-98
    oc = vsub(ray[0], center)
    a = F(1.0)
    half_b = vdot(oc, ray[1])
    c = vdot(oc, oc) - radius * radius
    disc = half_b * half_b - a * c
    if disc < F(0.0):
        return None
    sq = np.sqrt(disc)
    roots = [(-half_b - sq) / a, (-half_b + sq) / a]
    valid = [x for x in roots if t_min < x and x < t_max]
    if not valid:
        return None
    t = valid[0]
    for x in valid[1:]:
        if x < t:
            t = x
    pos = at(ray, t)
    normal = normalize(vdivs(vsub(pos, center), radius))
    return (t, pos, normal)


def triangle_intersect(v0, v1, v2, ray, t_min, t_max):  # common.rs:124-166
    n = vcross(vsub(v1, v0), vsub(v2, v0))
    cosl = vdot(n, ray[1])
    if -EPS8 < cosl and cosl < EPS8:
        return None
    d = vdot(n, v0)
    t = (vdot(n, ray[0]) + d) / cosl
    if t < t_min or t > t_max:
        return None
    p = at(ray, t)
    for (a, b) in ((v0, v1), (v1, v2), (v2, v0)):
        if vdot(n, vcross(vsub(b, a), vsub(p, a))) < F(0.0):
            return None
    return (t, p)


def world_hit(world, ray):  # common.rs:237-258
    closest = INF
    rec = None
    for (c, r, m) in world["spheres"]:
        h = sphere_hit(c, r, ray, T_MIN, closest)
        if h is not None:
            closest = h[0]
            rec = (h[0], h[1], h[2], m)
    mclosest = INF
    mrec = None
    for (v0, v1, v2, nrm, m) in world["triangles"]:
        h = triangle_intersect(v0, v1, v2, ray, T_MIN, closest)
        if h is not None and h[0] < mclosest:
            mclosest = h[0]
            mrec = (h[0], h[1], nrm, m)
    if mrec is not None:
        rec = mrec
    return rec


def random_unit_sphere(rng):  # common.rs:32-38
    x = rng.random_bilateral_f32()
    y = rng.random_bilateral_f32()
    z = rng.random_bilateral_f32()
    return nvec3(x, y, z)


def scatter(mat, ray, hit, rng):  # materials.rs:30-102
    kind = mat[0]
    _, pos, normal, _ = hit
    if kind == "Diffuse":
        s = vadd(normal, random_unit_sphere(rng))
        if near_zero(s):
            return mat[1], (pos, normal)
        return mat[1], (pos, normalize(s))
    if kind == "Metal":
        reflected = reflect(ray[1], normal)
        direction = vadd(reflected, vmuls(random_unit_sphere(rng), mat[2]))
        if vdot(direction, normal) >= F(0.0):
            return mat[1], (pos, normalize(direction))
        return mat[1], None
    if kind == "Dielectric":
        if vdot(ray[1], normal) >= F(0.0):
            n, ratio = vneg(normal), F(1.0) / mat[1]
        else:
            n, ratio = normal, mat[1]
        return (F(1.0), F(1.0), F(1.0), F(1.0)), (pos, normalize(refract(ray[1], n, ratio)))
    return mat[1], None  # Emission


def cmul(a, b):
    return tuple(x * y for x, y in zip(a, b))


def ray_color(ray, world, rng, depth):  # common.rs:263-285
    final = (F(1.0), F(1.0), F(1.0), F(1.0))
    for _ in range(depth):
        hit = world_hit(world, ray)
        if hit is not None:
            color, nxt = scatter(hit[3], ray, hit, rng)
            if nxt is not None:
                final = cmul(final, color)
                ray = nxt
            else:
                return cmul(final, color)
        else:
            t = F(0.5) * (normalize(ray[1])[1] + F(1.0))
            c = vadd(vmuls(v(1.0, 1.0, 1.0), F(1.0) - t), vmuls(v(0.5, 0.7, 1.0), t))
            return cmul(final, (c[0], c[1], c[2], F(1.0)))
    return (F(0.0), F(0.0), F(0.0), F(1.0))


def as_u8(x):
    if not (x > 0):
        return 0
    if x >= 255:
        return 255
    return int(x)


def ray_trace(world, cam, width, height, spp, depth, seed=2547549, states=None, samples=None):
    """common.rs:320-361 with the serial RNG; states: optional per-sample start
    states (replay), indexed by job = (row*W + col)*spp + s.  samples: optional
    float32[W*H*spp, 4] receiving every sample's ray_color result."""
    rng = Random(seed)
    out = np.zeros((height, width, 4), np.uint8)
    wden = F(width - 1)
    hden = F(height - 1)
    inv = F(1.0) / F(spp)
    for row in range(height):
        for col in range(width):
            color = (F(0.0), F(0.0), F(0.0), F(1.0))
            for s in range(spp):
                if states is not None:
                    rng.state = int(states[(row * width + col) * spp + s])
                u = (F(col) + rng.random_f32()) / wden
                vv = (F(row) + rng.random_f32()) / hden
                c = ray_color(cast_ray(cam, u, vv), world, rng, depth)
                if samples is not None:
                    samples[(row * width + col) * spp + s] = c
                color = tuple(x + y for x, y in zip(color, c))
            px = (np.sqrt(color[0] * inv) * GAMMA, np.sqrt(color[1] * inv) * GAMMA,
                  np.sqrt(color[2] * inv) * GAMMA, color[3] * inv * GAMMA)
            out[height - row - 1, col] = [as_u8(x) for x in px]
    return out


# ---------------------------------------------------------------- parser.rs (subset)
def parse(text: str):
    """Whitespace-token parser for the parser.rs grammar (well-formed input only)."""
    import re
    text = re.sub(r"//[^\n]*\n", "", text)
    stmts = [s.strip() for s in text.split(";") if s.strip()]
    cam = None
    mats = {}
    world = {"spheres": [], "triangles": []}
    for st in stmts:
        tok = st.replace(":", " : ").split()
        if tok[0] == "camera":
            o = v(*(dec_to_f32(t) for t in tok[2:5]))
            cam = camera_new_at(o, dec_to_f32(tok[6]))
        elif tok[0] == "material":
            name, kind = tok[1], tok[3]
            if kind == "Diffuse":
                mats[name] = ("Diffuse", tuple(dec_to_f32(t) for t in tok[5:8]) + (F(1.0),))
            elif kind == "Metal":
                mats[name] = ("Metal", tuple(dec_to_f32(t) for t in tok[5:8]) + (F(1.0),),
                              dec_to_f32(tok[9]))
            else:
                mats[name] = ("Dielectric", dec_to_f32(tok[5]))
        elif tok[0] == "sphere":
            c = tuple(dec_to_f32(t) for t in tok[2:5])
            world["spheres"].append((c, dec_to_f32(tok[6]), mats[tok[8]]))
        elif tok[0] == "triangle":
            v0 = tuple(dec_to_f32(t) for t in tok[2:5])
            v1 = tuple(dec_to_f32(t) for t in tok[6:9])
            v2 = tuple(dec_to_f32(t) for t in tok[10:13])
            nrm = normalize(vcross(vsub(v1, v0), vsub(v2, v0)))
            world["triangles"].append((v0, v1, v2, nrm, mats[tok[14]]))
    return cam, world
