"""GPU tests of the reference's callers and of the Emission material.

* examples/c_raytracer (the C twin of examples/c_raytracer.rs:48-62) is RUN:
  its 200x200 render() frame (16 spp, depth 8, lib.rs:51) written as a P3 PPM
  (image.rs:59-81) must equal the oracle's PPM of the reference's frame (SERIAL)
  byte for byte, and BASELINE configs[0] (C1: three spheres, 256x256, 1 spp,
  depth 4) is driven through the same binary via rt_render_ex.
* Emission (materials.rs:100-102) is reachable only through the scene-editing
  extension (the grammar cannot produce it, parser.rs:175-234): spheres and a
  triangle turned emissive render bit-exact against the oracle, in COUNTER and
  in REPLAY (the reference's serial stream), brute force and BVH.
"""
import os
import subprocess

import numpy as np
import pytest

import oracle as O
import raytracer_amd as R
import scenes as S
from conftest import ROOT, scene_text
from test_gpu_parity import assert_bits_equal

pytestmark = pytest.mark.gpu

EXE = os.path.join(ROOT, "examples", "c_raytracer")


def _run(args, tmp_path, env=None):
    out = tmp_path / "out.ppm"
    e = dict(os.environ)
    e.update(env or {})
    r = subprocess.run([EXE, str(out)] + args, capture_output=True, text=True, timeout=100, env=e)
    assert r.returncode == 0, r.stderr
    return out.read_bytes()


def test_c_example_default_frame_equals_oracle_ppm(tmp_path):
    """The C twin's render() frame is the reference's own image (SERIAL)."""
    src = scene_text("c_raytracer_world.txt")
    img, _, _ = O.Scene(src).render(200, 200, 16, 8, mode=O.RNG_SERIAL)
    assert _run([], tmp_path) == O.ppm(img)  # the inline world of c_raytracer.rs:15-44
    img, _, _ = O.Scene(src).render(200, 200, 16, 8, mode=O.RNG_COUNTER, nthreads=8)
    assert _run(["-", "200", "200"], tmp_path, {"RT_AMD_DEVICES": "1", "RT_AMD_RNG": "counter"}) \
        == O.ppm(img)


def test_c1_through_the_c_example(tmp_path):
    src = S.three_spheres()
    path = tmp_path / "c1.txt"
    path.write_text(src)
    img, _, _ = O.Scene(src).render(256, 256, 1, 4, mode=O.RNG_SERIAL)
    assert _run([str(path), "256", "256", "1", "4"], tmp_path) == O.ppm(img)


def _emissive(src, spheres, tris):
    world, ref = R.World(src), O.Scene(src)
    for i, rgb in spheres:
        world.set_material(i, 3, rgb)
        ref.set_material(i, 3, rgb)
    for i, rgb in tris:
        world.set_material(i, 3, rgb, triangle=True)
        ref.set_material(i, 3, rgb, triangle=True)
    return world, ref


def test_emission_counter_and_replay():
    src = scene_text("c_raytracer_world.txt")
    world, ref = _emissive(src, [(4, (4.0, 3.5, 3.0)), (1, (0.0, 0.9, 2.0))], [(1, (1.5, 0.25, 0.5))])
    w, h, spp, depth = 48, 27, 6, 8
    img, st, _ = ref.render(w, h, spp, depth, mode=O.RNG_COUNTER, nthreads=8)
    out, gst = world.render(w, h, spp, depth)
    assert_bits_equal(out, img, "emissive COUNTER frame")
    assert gst["rays"] == st["rays"]
    base, _, _ = O.Scene(src).render(w, h, spp, depth, mode=O.RNG_COUNTER, nthreads=8)
    assert not np.array_equal(img, base)  # the emitters are visible
    img, st, states = ref.render(w, h, spp, depth, mode=O.RNG_SERIAL, record_states=True)
    out, gst = world.render(w, h, spp, depth, mode=R.RNG_REPLAY, replay=states)
    assert_bits_equal(out, img, "emissive REPLAY frame")


def test_emission_in_the_sphere_bvh():
    src = S.rtow()
    n = R.World(src).num_spheres
    picks = [(i, (2.0 + (i % 3), 1.5, 1.0)) for i in range(5, n, 37)]
    world, ref = _emissive(src, picks, [])
    for accel in (R.ACCEL_BVH, R.ACCEL_BRUTE):
        out, st = world.render(64, 36, 4, 8, accel=accel)
        img, ost, _ = ref.render(64, 36, 4, 8, mode=O.RNG_COUNTER, nthreads=8)
        assert_bits_equal(out, img, f"emissive RTOW accel={accel}")
        assert st["rays"] == ost["rays"]
    with pytest.raises(ValueError):
        world.set_material(n, 3, (1.0, 1.0, 1.0))


@pytest.mark.parametrize("search", ["pixtab", "count", "coalesce"])
def test_emission_serial_every_search(monkeypatch, search):
    """render()'s mode (SERIAL) with emitters -- the branch that ends a path
    with no draw (materials.rs:100-102) -- beside metal absorption and
    dielectrics (the c_raytracer world), through each start-state search: the
    pixel table, the count pass and the coalescing search must find the states
    of the reference's one stream (oracle SERIAL) for every material branch."""
    env = {"pixtab": dict(RT_AMD_SERIAL_PIXTAB="1"),
           "count": dict(RT_AMD_SERIAL_PIXTAB="0", RT_AMD_SERIAL_COALESCE="0"),
           "coalesce": dict(RT_AMD_SERIAL_PIXTAB="0", RT_AMD_SERIAL_COALESCE="1")}[search]
    for k, v in env.items():
        monkeypatch.setenv(k, v)
    src = scene_text("c_raytracer_world.txt")
    world, ref = _emissive(src, [(4, (4.0, 3.5, 3.0)), (1, (0.0, 0.9, 2.0))], [(1, (1.5, 0.25, 0.5))])
    w, h, spp, depth = 48, 27, 8, 8
    img, st, _ = ref.render(w, h, spp, depth, mode=O.RNG_SERIAL)
    out, gst = world.render(w, h, spp, depth, mode=R.RNG_SERIAL, serial_check=True)
    assert_bits_equal(out, img, f"emissive SERIAL frame ({search})")
    assert gst["rays"] == st["rays"] and gst["serial_chain_breaks"] == 0
