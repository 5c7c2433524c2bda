"""GPU parity of RT_RNG_SERIAL: the reference's single frame-wide xorshift32
stream (common.rs:321, random.rs:8-30) found on the device -- no replay table
from a CPU run -- against the oracle's SERIAL mode, bit for bit.

The library traces the next samples from candidate stream positions (every
candidate: the count pass; or each block's distinct live offsets: the
coalescing search), follows the true path as far as it stays inside the
candidate windows, repeats from there, and renders from the start states it
found (runtime.cpp render_frame_serial).  Cases: the
examples/c_raytracer.rs frame (200x200, 16 spp, depth 8 -- render()'s
settings, lib.rs:51), BASELINE configs[0] (C1), the sphere BVH (RTOW) and the
triangle trees, edge frames, row tiles, a non-default seed, and windows forced
so narrow that every iteration stops short and the next resumes there.
"""
import time

import numpy as np
import pytest

import oracle as O
import raytracer_amd as R
import scenes as S
from conftest import scene_text
from test_gpu_parity import assert_bits_equal

pytestmark = pytest.mark.gpu


def _serial_pair(src, w, h, spp, depth, seed=R.DEFAULT_SEED, **kw):
    img, st, _ = O.Scene(src).render(w, h, spp, depth, mode=O.RNG_SERIAL, seed=seed)
    world = R.World(src)
    t = time.perf_counter()
    out, gst = world.render(w, h, spp, depth, mode=R.RNG_SERIAL, seed=seed, **kw)
    dt = time.perf_counter() - t
    return img, st, out, gst, dt


@pytest.mark.parametrize("scene,w,h,spp,depth", [
    ("c_raytracer_world.txt", 200, 200, 16, 8),  # examples/c_raytracer.rs via render()
    ("three_spheres.txt", 256, 256, 1, 4),       # C1
    ("world.txt", 96, 54, 8, 8),
])
def test_serial_frames_bit_exact(scene, w, h, spp, depth):
    img, st, out, gst, dt = _serial_pair(scene_text(scene), w, h, spp, depth)
    assert_bits_equal(out, img, f"{scene} SERIAL frame")
    assert gst["rays"] == st["rays"]
    print(f"{scene} {w}x{h}x{spp}/{depth}: start states {gst['serial_ms']:.1f} ms, "
          f"replay trace {gst['trace_ms']:.2f} ms, call {dt * 1e3:.1f} ms")


def test_serial_sphere_bvh_and_triangle_trees():
    for src, accel in ((S.rtow(), R.ACCEL_BVH), (S.triangle_soup(7, 300, spheres=40, grid=6), R.ACCEL_BVH),
                       (S.rtow(), R.ACCEL_BRUTE)):
        img, st, out, gst, _ = _serial_pair(src, 64, 36, 4, 8, accel=accel)
        assert_bits_equal(out, img, "SERIAL BVH frame")
        assert gst["rays"] == st["rays"] and gst["accel"] == accel


@pytest.mark.parametrize("w,h,spp,depth,seed", [
    (1, 5, 3, 8, 2547549), (5, 1, 2, 8, 2547549), (6, 4, 0, 8, 2547549), (7, 3, 3, 0, 2547549),
    (9, 7, 5, 1, 7), (33, 17, 3, 6, 123456789),
])
def test_serial_edge_frames(w, h, spp, depth, seed):
    img, st, out, gst, _ = _serial_pair(scene_text("c_raytracer_world.txt"), w, h, spp, depth, seed=seed)
    assert_bits_equal(out, img, "SERIAL edge frame")
    assert gst["rays"] == st["rays"]


def test_serial_narrow_windows_and_short_iterations(monkeypatch):
    """K forced to 24 candidates with 512-sample iterations: paths leave their
    windows after a few samples and each iteration resumes where the last one
    stopped; one-sample iterations; iterations longer than the frame; one K
    for every iteration (no per-iteration windows from the pixel variances);
    states re-walked per block instead of gathered from the recorded paths;
    odd iteration lengths with shallow paths; count-pass chunks and
    partitions of any size."""
    for env, scene, size in [
        (dict(RT_AMD_SERIAL_K="24", RT_AMD_SERIAL_CHUNK="512"), "c_raytracer_world.txt", (80, 60, 16, 8)),
        (dict(RT_AMD_SERIAL_ADAPT="0"), "c_raytracer_world.txt", (40, 30, 16, 8)),
        (dict(RT_AMD_SERIAL_ADAPT="0", RT_AMD_SERIAL_CHUNK="700"), "world.txt", (33, 17, 3, 8)),
        # resolved states re-walked per block instead of gathered from the block
        # paths (the count pass: the coalescing search always gathers)
        (dict(RT_AMD_SERIAL_GATHER="0", RT_AMD_SERIAL_COALESCE="0", RT_AMD_SERIAL_PIXTAB="0"),
         "c_raytracer_world.txt", (40, 30, 16, 8)),
        (dict(RT_AMD_SERIAL_GATHER="0", RT_AMD_SERIAL_COALESCE="0", RT_AMD_SERIAL_PIXTAB="0", RT_AMD_SERIAL_K="24",
              RT_AMD_SERIAL_CHUNK="300"), "world.txt", (29, 13, 4, 8)),
        (dict(RT_AMD_SERIAL_CHUNK="1"), "world.txt", (12, 9, 2, 8)),
        (dict(RT_AMD_SERIAL_CHUNK="100"), "world.txt", (13, 7, 3, 8)),
        (dict(RT_AMD_SERIAL_CHUNK="100000", RT_AMD_SERIAL_Z10="5"), "world.txt", (31, 17, 4, 8)),
        # odd iteration lengths, shallow paths
        (dict(RT_AMD_SERIAL_CHUNK="37"), "world.txt", (15, 9, 3, 1)),
        (dict(RT_AMD_SERIAL_CHUNK="61", RT_AMD_SERIAL_K="4"), "world.txt", (15, 9, 3, 1)),
        # count-pass scheduling: small chunks of any size, many partitions
        (dict(RT_AMD_SERIAL_COALESCE="0", RT_AMD_SERIAL_PIXTAB="0", RT_AMD_SERIAL_CCHUNK="37",
              RT_AMD_SERIAL_PARTS="256"), "c_raytracer_world.txt", (40, 30, 16, 8)),
        # coalescing search: blocks of 1 and 7 samples, narrow windows in long blocks
        (dict(RT_AMD_SERIAL_PIXTAB="0", RT_AMD_SERIAL_R="1", RT_AMD_SERIAL_CHUNK="300"), "c_raytracer_world.txt",
         (20, 15, 4, 8)),
        (dict(RT_AMD_SERIAL_PIXTAB="0", RT_AMD_SERIAL_R="7", RT_AMD_SERIAL_CHUNK="1000"), "world.txt",
         (33, 17, 3, 8)),
        (dict(RT_AMD_SERIAL_PIXTAB="0", RT_AMD_SERIAL_R="200", RT_AMD_SERIAL_K="24", RT_AMD_SERIAL_CHUNK="4000"),
         "world.txt", (40, 30, 4, 8)),
        # pixel table: odd chunks of positions, odd walk blocks, narrow windows,
        # iterations shorter than a pixel, pixels wider than the iteration
        (dict(RT_AMD_SERIAL_PCHUNK="7", RT_AMD_SERIAL_WALKR="5"), "c_raytracer_world.txt", (40, 30, 16, 8)),
        (dict(RT_AMD_SERIAL_K="24", RT_AMD_SERIAL_CHUNK="512", RT_AMD_SERIAL_WALKR="33"), "c_raytracer_world.txt",
         (80, 60, 16, 8)),
        (dict(RT_AMD_SERIAL_CHUNK="9"), "world.txt", (13, 7, 16, 8)),
        (dict(RT_AMD_SERIAL_CHUNK="50", RT_AMD_SERIAL_K="8"), "world.txt", (7, 5, 33, 4)),
        (dict(RT_AMD_SERIAL_PCHUNK="1000"), "world.txt", (33, 17, 5, 8)),
        # LDS-staged rows: blocks of 256 samples over many pixels, a block of one
        # pixel's samples, 1-sample blocks
        (dict(RT_AMD_SERIAL_WALKR="256", RT_AMD_SERIAL_CHUNK="3000"), "world.txt", (33, 17, 4, 8)),
        (dict(RT_AMD_SERIAL_WALKR="16"), "c_raytracer_world.txt", (40, 30, 16, 8)),
        (dict(RT_AMD_SERIAL_WALKR="1", RT_AMD_SERIAL_CHUNK="200"), "world.txt", (13, 7, 4, 8)),
        # pixel table through a gathered count table (the first build's walks)
        (dict(RT_AMD_SERIAL_PGATHER="1", RT_AMD_SERIAL_K="40"), "c_raytracer_world.txt", (40, 30, 16, 8)),
    ]:
        for k, v in env.items():
            monkeypatch.setenv(k, v)
        img, st, out, gst, _ = _serial_pair(scene_text(scene), *size)
        assert_bits_equal(out, img, f"SERIAL frame {env}")
        assert gst["rays"] == st["rays"]
        for k in env:
            monkeypatch.delenv(k)


def test_serial_table_reuse_after_stops(monkeypatch):
    """Windows forced narrow (K = 24 / 30 candidates) so that most pixel-table
    iterations stop short: each next iteration copies the entries of the
    stopped one's table that its own windows cover (serial_reuse_kernel) and
    traces only the rest.  Bit-exact against the oracle's SERIAL frame, and
    the same iterations, stops and frame with the reuse switched off and
    without the per-pixel spans (RT_AMD_SERIAL_SPIX=0: no chunk skipping
    either); odd job chunks (rows padded to 7 and 1000 positions)."""
    for scene, size, env in [
        ("c_raytracer_world.txt", (80, 60, 16, 8), dict(RT_AMD_SERIAL_K="24", RT_AMD_SERIAL_CHUNK="512")),
        ("world.txt", (48, 27, 16, 8), dict(RT_AMD_SERIAL_K="30", RT_AMD_SERIAL_CHUNK="2000")),
        ("world.txt", (40, 30, 8, 8), dict(RT_AMD_SERIAL_K="24", RT_AMD_SERIAL_CHUNK="700",
                                           RT_AMD_SERIAL_PCHUNK="7")),
        ("c_raytracer_world.txt", (40, 30, 16, 8), dict(RT_AMD_SERIAL_K="30", RT_AMD_SERIAL_CHUNK="900",
                                                       RT_AMD_SERIAL_PCHUNK="1000")),
    ]:
        img, st, _ = O.Scene(scene_text(scene)).render(*size, mode=O.RNG_SERIAL)
        runs = {}
        for label, extra in (("reuse", {}), ("off", dict(RT_AMD_SERIAL_REUSE="0")),
                             ("nospix", dict(RT_AMD_SERIAL_SPIX="0"))):
            for k, v in {**env, **extra}.items():
                monkeypatch.setenv(k, v)
            out, gst = R.World(scene_text(scene)).render(*size, mode=R.RNG_SERIAL)
            for k in {**env, **extra}:
                monkeypatch.delenv(k)
            assert_bits_equal(out, img, f"SERIAL frame {scene} {size} {env} {label}")
            assert gst["rays"] == st["rays"]
            runs[label] = (gst["serial_iterations"], gst["serial_retries"])
        assert runs["reuse"] == runs["off"] == runs["nospix"], runs
        assert runs["reuse"][1] > runs["reuse"][0] // 4, runs  # most iterations stop short


SEARCHES = {
    # runtime.cpp serial_find_states: the pixel table (default from 4 spp), the
    # count pass + block walks, the coalescing block search
    "pixtab": dict(RT_AMD_SERIAL_PIXTAB="1"),
    # the pixel table's block walks and state gather reading the table in
    # global memory instead of LDS-staged u8 rows
    "pixtab_global": dict(RT_AMD_SERIAL_PIXTAB="1", RT_AMD_SERIAL_WALK_LDS="0"),
    "count": dict(RT_AMD_SERIAL_PIXTAB="0", RT_AMD_SERIAL_COALESCE="0"),
    "coalesce": dict(RT_AMD_SERIAL_PIXTAB="0", RT_AMD_SERIAL_COALESCE="1"),
}


@pytest.mark.parametrize("search", sorted(SEARCHES))
def test_serial_search_modes(monkeypatch, search):
    """Every start-state search on every scene family: the pixel table, the
    count pass + block walks and the coalescing block search, on small scenes,
    the sphere tree and triangle trees, with wide and narrow windows."""
    for k, v in SEARCHES[search].items():
        monkeypatch.setenv(k, v)
    for src, size, env in [
        (scene_text("c_raytracer_world.txt"), (64, 48, 8, 8), {}),
        (scene_text("world.txt"), (48, 27, 16, 8), dict(RT_AMD_SERIAL_K="30", RT_AMD_SERIAL_CHUNK="2000")),
        (S.rtow(), (48, 27, 4, 8), {}),
        (S.triangle_soup(11, 200, spheres=20, grid=5), (40, 30, 4, 8), dict(RT_AMD_SERIAL_CHUNK="1500")),
    ]:
        for k, v in env.items():
            monkeypatch.setenv(k, v)
        img, st, out, gst, _ = _serial_pair(src, *size)
        assert_bits_equal(out, img, f"SERIAL frame, search={search} {env}")
        assert gst["rays"] == st["rays"]
        for k in env:
            monkeypatch.delenv(k)


def test_serial_tiles_are_rows_of_the_serial_frame():
    src = scene_text("world.txt")
    world = R.World(src)
    full, _ = world.render(40, 30, 4, 8, mode=R.RNG_SERIAL)
    for rank in range(3):
        tile, _ = world.render(40, 30, 4, 8, mode=R.RNG_SERIAL, row_block=4, rank=rank, nranks=3)
        rows = [R.tile_row(k, 4, rank, 3) for k in range(tile.shape[0])]
        assert_bits_equal(tile, full[rows], f"SERIAL tile {rank}")


def test_serial_after_camera_move_and_counter_frames():
    src = scene_text("c_raytracer_world.txt")
    world, ref = R.World(src), O.Scene(src)
    world.render(32, 24, 4, 8)  # a COUNTER frame first (shared scratch)
    world.move_camera(0.3, -0.2, 0.5)
    ref.set_camera(world.camera())
    img, _, _ = ref.render(32, 24, 4, 8, mode=O.RNG_SERIAL)
    out, _ = world.render(32, 24, 4, 8, mode=R.RNG_SERIAL)
    assert_bits_equal(out, img, "moved SERIAL frame")
    cnt, _ = world.render(32, 24, 4, 8)
    img2, _, _ = ref.render(32, 24, 4, 8, mode=O.RNG_COUNTER)
    assert_bits_equal(cnt, img2, "COUNTER frame after SERIAL")
    assert not np.array_equal(cnt, out)


def test_serial_large_frame_bit_exact():
    """render()'s settings (16 spp, depth 8) at 960x540 on the
    examples/c_raytracer.rs world -- 8.3 M samples of the one stream, about
    650 candidate-table iterations -- bit-exact against the oracle's SERIAL
    frame (~3 s of oracle time), with the chain check clean."""
    src = scene_text("c_raytracer_world.txt")
    img, st, out, gst, dt = _serial_pair(src, 960, 540, 16, 8, serial_check=True)
    assert_bits_equal(out, img, "SERIAL 960x540x16 frame")
    assert gst["rays"] == st["rays"]
    assert gst["serial_checked"] == 960 * 540 * 16 and gst["serial_chain_breaks"] == 0
    print(f"960x540x16/8 SERIAL: call {dt * 1e3:.0f} ms, start states {gst['serial_ms']:.0f} ms "
          f"(tables {gst['serial_setup_ms']:.1f} ms, {gst['serial_iterations']} iterations)")


@pytest.mark.parametrize("scene,w,h,spp", [
    ("c_raytracer_world.txt", 1920, 1080, 16),  # render() at 1080p
    ("rtow", 1920, 1080, 64),                   # BASELINE configs[1] (C2) settings
])
def test_serial_chain_full_size(scene, w, h, spp):
    """Sizes the oracle cannot render in a test: the start states found on the
    GPU form the reference's chain (sample 0 at the seed, every sample ending
    where the next one starts, RT_FLAG_SERIAL_CHECK), and the frame is
    deterministic.  With the trace arithmetic pinned bit-exact against the
    oracle above, a closed chain from the seed is the reference's stream."""
    src = S.rtow() if scene == "rtow" else scene_text(scene)
    world = R.World(src)
    t = time.perf_counter()
    out, st = world.render(w, h, spp, 8, mode=R.RNG_SERIAL, serial_check=True)
    dt = time.perf_counter() - t
    assert st["serial_checked"] == w * h * spp
    assert st["serial_chain_breaks"] == 0
    assert (out[..., 3] == 255).all()
    again, st2 = world.render(w, h, spp, 8, mode=R.RNG_SERIAL)
    assert_bits_equal(again, out, "SERIAL frame rendered twice")
    assert st2["rays"] == st["rays"]
    print(f"{scene} {w}x{h}x{spp}/8 SERIAL: call {dt * 1e3:.0f} ms (with the check), start states "
          f"{st2['serial_ms']:.0f} ms, {st2['serial_iterations']} iterations, "
          f"{st2['rays'] / (st2['serial_ms'] + st2['trace_ms']) / 1e3:.1f} Mrays/s")


def test_serial_chain_check_sees_a_corrupted_state(monkeypatch):
    """The check is not vacuous: one corrupted start state breaks the link
    into that sample and the link out of it (sample 0: the seed link).  The
    hook corrupts a scratch copy only the check reads: the frame is still the
    reference's."""
    src = scene_text("world.txt")
    world = R.World(src)
    good, st = world.render(40, 30, 4, 8, mode=R.RNG_SERIAL, serial_check=True)
    assert st["serial_chain_breaks"] == 0
    for j, want in ((777, 2), (0, 2), (40 * 30 * 4 - 1, 2)):
        monkeypatch.setenv("RT_AMD_SERIAL_BREAK", str(j))
        out, st = world.render(40, 30, 4, 8, mode=R.RNG_SERIAL, serial_check=True)
        assert st["serial_chain_breaks"] == want, (j, st["serial_chain_breaks"])
        assert_bits_equal(out, good, "frame under the check's test hook")
