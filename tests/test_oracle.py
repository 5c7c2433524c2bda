"""CPU tests of the oracle (the C++ restatement used as the parity checker).

Pins it against (1) the reference's own known-answer tests (maths.rs:243-286),
(2) the xorshift32 stream (random.rs:8-30), (3) hand-derived known answers
for each quirk SURVEY.md 8(a) lists, (4) the independent numpy restatement
(tests/pyref.py) bit-for-bit, and (5) the committed golden fixtures.
"""
import hashlib
import json
import os

import numpy as np
import pytest

import oracle as O
import pyref as P
import scenes as S
from conftest import ROOT, scene_text

GOLD = os.path.join(ROOT, "tests", "golden")
f32 = np.float32


def fa(*x):
    return O.f32arr(x)


def call3(fn, *args):
    out = np.zeros(3, np.float32)
    fn(*args, O.fptr(out))
    return out


def bits(a):
    return np.asarray(a, np.float32).view(np.uint32)


# ---------------------------------------------------------------- random.rs
def test_xorshift_known_answers():
    # first outputs from seed 2547549 (random.rs:9)
    assert O.xorshift_stream(2547549, 6) == [2725201371, 273946257, 3259598226, 2911641871,
                                              471297785, 3369006525]
    r = O.random_f32_stream(2547549, 6)
    assert np.allclose(r, [0.63451040, 0.06378309, 0.75893438, 0.67791945, 0.10973257,
                           0.78440797], atol=5e-8)


def test_random_f32_is_x_times_2_pow_minus_32():
    # u32::MAX as f32 rounds to 2^32, so random_f32 == RNE(x) * 2^-32; 1.0 is reachable
    xs = O.xorshift_stream(2547549, 200)
    fs = O.random_f32_stream(2547549, 200)
    assert all(bits(f) == bits(f32(np.uint32(x)) * f32(2.0 ** -32)) for x, f in zip(xs, fs))
    assert f32(np.uint32(0xFFFFFFFF)) / f32(4294967296.0) == 1.0


def test_rng_golden():
    g = json.load(open(os.path.join(GOLD, "rng.json")))
    assert O.xorshift_stream(g["seed"], 32) == g["xorshift32"]
    assert list(bits(O.random_f32_stream(g["seed"], 32))) == g["random_f32_bits"]
    for j, s in g["counter_seed"].items():
        assert O.sample_seed(2547549, int(j)) == s


# ---------------------------------------------------------------- maths.rs KATs
def test_reference_kat_reflect():  # maths.rs:251-257
    out = call3(O.lib().ro_reflect, O.fptr(fa(1.0, 0.0, -1.0)), O.fptr(fa(0.0, 0.0, 1.0)))
    assert np.all(np.abs(out - fa(1.0, 0.0, 1.0)) < 1e-8)


def test_reference_kat_refract_identity():  # maths.rs:279-286 (eta = 1)
    a = call3(O.lib().ro_normalize, O.fptr(fa(1.0, 0.0, -1.0)))
    out = call3(O.lib().ro_refract, O.fptr(a), O.fptr(fa(0.0, 0.0, 1.0)), 1.0)
    assert np.all(np.abs(out - a) < 1e-8)


def test_reference_kat_negate():  # maths.rs:243-249 (via reflect with n = 0)
    out = call3(O.lib().ro_reflect, O.fptr(fa(-1.0, -2.0, -3.0)), O.fptr(fa(0.0, 0.0, 0.0)))
    assert list(out) == [-1.0, -2.0, -3.0]


def test_normalize_divides_not_multiplies():
    v = fa(1.0, 2.0, 3.0)
    out = call3(O.lib().ro_normalize, O.fptr(v))
    ln = np.sqrt((v[0] * v[0] + v[1] * v[1]) + v[2] * v[2])
    assert list(bits(out)) == list(bits([v[0] / ln, v[1] / ln, v[2] / ln]))


# ---------------------------------------------------------------- as u8
@pytest.mark.parametrize("x,want", [(np.nan, 0), (-1.0, 0), (-0.0, 0), (0.0, 0), (0.99, 0),
                                    (254.9, 254), (255.0, 255), (255.999 * 1.0, 255),
                                    (1e30, 255), (np.inf, 255), (-np.inf, 0)])
def test_as_u8_saturates(x, want):
    assert O.lib().ro_as_u8(x) == want


# ---------------------------------------------------------------- hits
def sphere(ray, c, r, tmin=0.001, tmax=np.inf):
    out = np.zeros(7, np.float32)
    hit = O.lib().ro_sphere_hit(O.fptr(O.f32arr(ray)), O.fptr(O.f32arr(c)), r, tmin, tmax,
                                O.fptr(out))
    return out if hit else None


def tri(ray, v, tmin=0.001, tmax=np.inf):
    out = np.zeros(7, np.float32)
    hit = O.lib().ro_triangle_intersect(O.fptr(O.f32arr(ray)), O.fptr(O.f32arr(v)), tmin, tmax,
                                        O.fptr(out))
    return out if hit else None


def test_sphere_hit_miss_inside():
    h = sphere([0, 0, 0, 0, 0, -1], [0, 0, -2], 0.5)
    assert h is not None and abs(h[0] - 1.5) < 1e-6 and abs(h[6] - 1.0) < 1e-6
    assert sphere([0, 0, 0, 0, 1, 0], [0, 0, -2], 0.5) is None
    # origin inside: root1 < t_min, root2 is taken
    h = sphere([0, 0, -2, 0, 0, -1], [0, 0, -2], 0.5)
    assert h is not None and abs(h[0] - 0.5) < 1e-6
    # strict t_max: a hit exactly at t_max is rejected
    assert sphere([0, 0, 0, 0, 0, -1], [0, 0, -2], 0.5, tmax=1.5) is None
    # sphere behind the ray
    assert sphere([0, 0, 0, 0, 0, 1], [0, 0, -2], 0.5) is None


def test_sphere_uses_a_equal_one():
    # NVec3::length_squared() == 1.0 (maths.rs:127): a non-unit direction is NOT rescaled
    h = sphere([0, 0, 0, 0, 0, -2], [0, 0, -4], 1.0)
    assert h is not None
    half_b = f32(-8.0)     # oc.d = (0,0,4).(0,0,-2)
    c = f32(15.0)          # |oc|^2 - r^2
    t = (-half_b - np.sqrt(half_b * half_b - c)) / f32(1.0)
    assert bits(h[0]) == bits(t) and h[0] == 1.0  # with a = |d|^2 = 4 it would be 0.5


def test_triangle_sign_quirk_from_nonzero_origin():
    # common.rs:141 computes (n.o + d)/cos, not (d - n.o)/cos: exact only when n.o == 0
    v = [-1, -1, -3, 1, -1, -3, 0, 1, -3]
    h0 = tri([0, 0, 0, 0, 0, -1], v)
    assert h0 is not None and abs(h0[0] - 3.0) < 1e-6
    h1 = tri([0, 0, 1, 0, 0, -1], v)  # true distance 4; quirk gives (n.o + d)/cos = 2
    assert h1 is not None and abs(h1[0] - 2.0) < 1e-6


def test_triangle_t_equal_t_max_accepted():
    v = [-1, -1, -3, 1, -1, -3, 0, 1, -3]
    assert tri([0, 0, 0, 0, 0, -1], v, tmax=3.0) is not None  # `t > t_max` rejects only
    assert tri([0, 0, 0, 0, 0, -1], v, tmax=2.9999) is None


def test_triangle_parallel_rejected():
    v = [-1, -1, -3, 1, -1, -3, 0, 1, -3]
    assert tri([0, 0, 0, 1, 0, 0], v) is None


# ---------------------------------------------------------------- scatter
def scatter(mat, ray, hit, state):
    st = O.C.c_uint32(state)
    color = np.zeros(4, np.float32)
    nxt = np.zeros(6, np.float32)
    has = O.lib().ro_scatter(O.fptr(O.f32arr(mat)), O.fptr(O.f32arr(ray)), O.fptr(O.f32arr(hit)),
                             O.C.byref(st), O.fptr(color), O.fptr(nxt))
    return bool(has), color, nxt, st.value


def test_metal_absorb_returns_colour_and_draws_three():
    # ray along +z hitting a surface whose normal is +z: reflected . n < 0 -> absorbed
    has, color, _, s = scatter([1, 0.8, 0.6, 0.2, 1.0, 0.0], [0, 0, 0, 0, 0, 1],
                               [1, 0, 0, 1, 0, 0, 1], 2547549)
    assert not has and list(color) == [f32(0.8), f32(0.6), f32(0.2), 1.0]
    st = O.C.c_uint32(2547549)
    for _ in range(3):
        O.lib().ro_xorshift32(O.C.byref(st))
    assert s == st.value  # 3 draws even with fuzz 0


def test_dielectric_inverted_convention_draws_nothing():
    hit = [1, 0, 0, 1, 0, 0, 1]
    has_in, c_in, n_in, s_in = scatter([2, 0, 0, 0, 1, 1.5], [0, 0, 0, 0, 0, 1], hit, 5)
    has_out, c_out, n_out, s_out = scatter([2, 0, 0, 0, 1, 1.5], [0, 0, 0, 0, 0, -1], hit, 5)
    assert has_in and has_out and s_in == 5 and s_out == 5
    assert list(c_in) == [1, 1, 1, 1]
    # normal incidence passes straight through either way
    assert abs(n_in[5] - 1) < 1e-6 and abs(n_out[5] + 1) < 1e-6


def test_diffuse_scatter_direction_normalised():
    has, color, nxt, s = scatter([0, 0.5, 0.5, 0.5, 1.0, 0.0], [0, 0, 0, 0, 0, -1],
                                 [1, 0, 0, 1, 0, 0, 1], 2547549)
    assert has and abs(np.linalg.norm(nxt[3:]) - 1) < 1e-6


def test_sky_renormalises_direction():
    d = fa(0.3, 0.4, 0.5)  # not unit: the sky term normalises it again (common.rs:278)
    out = np.zeros(4, np.float32)
    O.lib().ro_sky(O.fptr(d), O.fptr(fa(1, 1, 1, 1)), O.fptr(out))
    n = d / np.sqrt((d[0] * d[0] + d[1] * d[1]) + d[2] * d[2])
    t = f32(0.5) * (f32(d[1] / np.sqrt((d[0] * d[0] + d[1] * d[1]) + d[2] * d[2])) + f32(1.0))
    assert bits(out[1]) == bits(f32(1.0) * (f32(1.0) - t) + f32(0.7) * t)
    assert out[3] == 1.0 and n.shape == (3,)


# ---------------------------------------------------------------- frames
@pytest.mark.parametrize("name,w,h,spp,depth", [
    ("c_raytracer_world.txt", 12, 9, 2, 8),
    ("world.txt", 10, 7, 3, 5),
    ("three_spheres.txt", 9, 9, 1, 4),
    ("c_raytracer_world.txt", 1, 4, 2, 8),
    ("c_raytracer_world.txt", 4, 1, 2, 8),
    ("world.txt", 5, 4, 0, 8),
    ("world.txt", 5, 4, 2, 0),
])
def test_oracle_matches_numpy_restatement(name, w, h, spp, depth):
    src = scene_text(name)
    cam, world = P.parse(src)
    ps = np.zeros((w * h * max(spp, 0), 4), np.float32)
    a = P.ray_trace(world, cam, w, h, spp, depth, samples=ps)
    b, _, _, smp = O.Scene(src).render(w, h, spp, depth, record_samples=True)
    assert np.array_equal(a, b)
    assert np.array_equal(ps.view(np.uint32), smp.view(np.uint32))


def test_replay_reproduces_serial():
    src = scene_text("world.txt")
    s = O.Scene(src)
    a, sa, states = s.render(20, 15, 4, 8, record_states=True)
    b, sb, _ = s.render(20, 15, 4, 8, mode=O.RNG_REPLAY, replay=states)
    assert np.array_equal(a, b) and sa == sb


def test_counter_mode_threads_invariant():
    s = O.Scene(S.rtow())
    a, sa, _ = s.render(40, 24, 2, 8, mode=O.RNG_COUNTER, nthreads=1)
    b, sb, _ = s.render(40, 24, 2, 8, mode=O.RNG_COUNTER, nthreads=4)
    assert np.array_equal(a, b) and sa == sb


def test_golden_frames():
    meta = json.load(open(os.path.join(GOLD, "frames.json")))
    arrays = np.load(os.path.join(GOLD, "frames.npz"))
    srcs = {"c1": S.three_spheres(), "c_raytracer": scene_text("c_raytracer_world.txt"),
            "world": scene_text("world.txt"), "rtow": S.rtow()}
    for name, m in meta.items():
        src = srcs[name.split("_")[0] if not name.startswith("c_raytracer") else "c_raytracer"]
        img, st, states, smp = O.Scene(src).render(m["width"], m["height"], m["spp"], m["depth"],
                                                   mode=m["mode"], seed=m["seed"],
                                                   record_states=True, record_samples=True)
        assert np.array_equal(img, arrays[name]), name
        assert hashlib.sha256(img.tobytes()).hexdigest() == m["rgba_sha256"]
        assert hashlib.sha256(states.tobytes()).hexdigest() == m["sample_states_sha256"]
        assert hashlib.sha256(smp.view(np.uint32).tobytes()).hexdigest() == m["sample_bits_sha256"]
        assert st == m["stats"], name


def test_ppm_writer_format():  # image.rs:59-81
    img = np.zeros((2, 3, 4), np.uint8)
    img[0, 0] = [255, 0, 0, 255]
    img[1, 2] = [1, 2, 3, 255]
    txt = O.ppm(img).decode()
    lines = txt.split("\n")
    assert lines[:3] == ["P3", "3 2", "255"]
    assert lines[3] == "255 0 0" and lines[8] == "1 2 3" and txt.endswith("\n")


def test_emission_matches_numpy_restatement():
    """Emission (materials.rs:100-102) via the oracle's material hook: the
    grammar cannot produce it (parser.rs:175-234), so both restatements get
    the same emitters injected after parsing."""
    src = scene_text("c_raytracer_world.txt")
    cam, world = P.parse(src)
    s = O.Scene(src)
    for i, rgb in [(4, (4.0, 3.5, 3.0)), (1, (0.0, 0.9, 2.0))]:
        c, r, _ = world["spheres"][i]
        world["spheres"][i] = (c, r, ("Emission", tuple(np.float32(x) for x in rgb) + (np.float32(1.0),)))
        s.set_material(i, 3, rgb)
    v0, v1, v2, nrm, _ = world["triangles"][1]
    world["triangles"][1] = (v0, v1, v2, nrm, ("Emission", (np.float32(1.5), np.float32(0.25),
                                                           np.float32(0.5), np.float32(1.0))))
    s.set_material(1, 3, (1.5, 0.25, 0.5), triangle=True)
    w, h, spp, depth = 12, 9, 2, 8
    ps = np.zeros((w * h * spp, 4), np.float32)
    a = P.ray_trace(world, cam, w, h, spp, depth, samples=ps)
    b, _, _, smp = s.render(w, h, spp, depth, record_samples=True)
    assert np.array_equal(a, b)
    assert np.array_equal(ps.view(np.uint32), smp.view(np.uint32))
    base, _, _ = O.Scene(src).render(w, h, spp, depth)
    assert not np.array_equal(b, base)
