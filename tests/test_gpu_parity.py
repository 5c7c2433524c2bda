"""GPU parity: the HIP render path (through the C-ABI) against the CPU oracle.

Bar: bit-exact.  Every comparison below is on raw bits -- the RGBA8 frame
and, where the frame fits one launch, every sample's float colour.
  * REPLAY mode vs the oracle's SERIAL mode (the reference's semantics, one
    frame-wide xorshift32 stream, common.rs:321): the GPU reproduces the
    reference render bit-for-bit when given each sample's start state.
  * COUNTER mode vs the oracle's COUNTER mode: bit-exact.
  * COUNTER vs SERIAL: different RNG streams by construction -- statistical
    bound only (mean |diff| and PSNR, thresholds in the test).
At BASELINE sizes (1920x1080x64) the tests use size-independent properties:
determinism, tile invariance and oracle parity on sampled rows.
"""
import numpy as np
import pytest

import oracle as O
import raytracer_amd as R
import scenes as S
from conftest import scene_text

pytestmark = pytest.mark.gpu

CWORLD = "c_raytracer_world.txt"


def oracle_samples_to_gpu_order(samples, width, height, spp):
    """Oracle job = (row*W + col)*spp + s (row 0 = bottom); the GPU slab is
    sample-major over image rows (top first): slot = s*(H*W) + ir*W + col."""
    a = samples.reshape(height, width, spp, 4)[::-1].transpose(2, 0, 1, 3)
    return np.ascontiguousarray(a).reshape(-1, 4)


def assert_bits_equal(a, b, what):
    a = np.ascontiguousarray(a)
    b = np.ascontiguousarray(b)
    assert a.shape == b.shape, what
    if a.dtype == np.float32:
        a, b = a.view(np.uint32), b.view(np.uint32)
    bad = np.argwhere(a != b)
    assert bad.size == 0, f"{what}: {len(bad)} mismatches, first at {bad[:5].tolist()}"


def render_kept(world, *args, **kw):
    """Renders three times: by default (pixels resolved inside the trace kernel
    from per-wave sample rings), with keep_samples (every sample to the slab,
    then resolve_kernel), and without stats (the kernel variant whose work
    counters compile away).  The frames must agree bit for bit; afterwards the
    samples are readable (world.read_samples)."""
    out, st = world.render(*args, **kw)
    lean, _ = world.render(*args, stats=False, **kw)  # the kernel without work counters
    assert_bits_equal(lean, out, "kernel without counters")
    kept, st2 = world.render(*args, keep_samples=True, **kw)  # last: leaves the slab readable
    assert_bits_equal(kept, out, "in-kernel resolve vs slab + resolve kernel")
    assert st2["rays"] == st["rays"]
    return out, st


@pytest.mark.parametrize("scene,w,h,spp,depth", [
    (CWORLD, 40, 30, 4, 8),
    ("world.txt", 33, 17, 3, 8),
    ("three_spheres.txt", 64, 64, 1, 4),
])
def test_replay_matches_reference_serial(scene, w, h, spp, depth):
    src = scene_text(scene)
    ref = O.Scene(src)
    img, st, states, smp = ref.render(w, h, spp, depth, mode=O.RNG_SERIAL, record_states=True,
                                      record_samples=True)
    world = R.World(src)
    out, gst = render_kept(world, w, h, spp, depth, mode=R.RNG_REPLAY, replay=states)
    assert_bits_equal(out, img, "frame")
    assert_bits_equal(world.read_samples(w * h * spp)[:, :3],
                      oracle_samples_to_gpu_order(smp, w, h, spp)[:, :3], "samples")
    assert gst["rays"] == st["rays"]
    assert gst["tri_in_range"] == st["tri_in_range"]
    assert gst["sphere_tests"] == st["sphere_tests"]
    assert gst["tri_tests"] == st["tri_tests"]


def test_c1_three_spheres_full_frame_serial():
    """BASELINE configs[0]: 256x256, 1 spp, depth 4, reference serial RNG."""
    src = S.three_spheres()
    img, st, states = O.Scene(src).render(256, 256, 1, 4, record_states=True)
    out, gst = R.World(src).render(256, 256, 1, 4, mode=R.RNG_REPLAY, replay=states)
    assert_bits_equal(out, img, "C1 frame")
    assert gst["rays"] == st["rays"]


def test_c_raytracer_example_frame_serial():
    """examples/c_raytracer.rs: 200x200 via render() settings (16 spp, depth 8)."""
    src = scene_text(CWORLD)
    img, st, states = O.Scene(src).render(200, 200, 16, 8, record_states=True)
    out, gst = R.World(src).render(200, 200, 16, 8, mode=R.RNG_REPLAY, replay=states)
    assert_bits_equal(out, img, "c_raytracer frame")
    assert gst["rays"] == st["rays"] and gst["tri_in_range"] == st["tri_in_range"]


@pytest.mark.parametrize("scene,w,h,spp,depth,seed", [
    (CWORLD, 48, 27, 8, 8, 2547549),
    ("world.txt", 31, 23, 5, 6, 7),
    ("rtow.txt", 64, 36, 4, 8, 2547549),
])
def test_counter_mode_bit_exact(scene, w, h, spp, depth, seed):
    src = scene_text(scene)
    img, st, _, smp = O.Scene(src).render(w, h, spp, depth, mode=O.RNG_COUNTER, seed=seed,
                                          nthreads=8, record_samples=True)
    world = R.World(src)
    out, gst = render_kept(world, w, h, spp, depth, mode=R.RNG_COUNTER, seed=seed)
    assert_bits_equal(out, img, "frame")
    assert_bits_equal(world.read_samples(w * h * spp)[:, :3],
                      oracle_samples_to_gpu_order(smp, w, h, spp)[:, :3], "samples")
    assert gst["rays"] == st["rays"]


def test_render_abi_defaults_match_the_reference(monkeypatch):
    """render() (lib.rs:49-57 -> 16 spp, depth 8) == the reference's frame
    (oracle SERIAL: one xorshift32 stream, common.rs:321), and with
    RT_AMD_RNG=counter == oracle COUNTER at 16/8."""
    src = scene_text(CWORLD)
    img, _, _ = O.Scene(src).render(96, 54, 16, 8, mode=O.RNG_SERIAL)
    out = R.World(src).render_reference(96, 54)
    assert_bits_equal(out, img, "render()")
    monkeypatch.setenv("RT_AMD_RNG", "counter")
    img, _, _ = O.Scene(src).render(96, 54, 16, 8, mode=O.RNG_COUNTER, nthreads=8)
    out = R.World(src).render_reference(96, 54)
    assert_bits_equal(out, img, "render() RT_AMD_RNG=counter")


def test_counter_vs_serial_statistics():
    """Different RNG streams: compare converged images statistically."""
    src = scene_text(CWORLD)
    w, h, spp = 64, 64, 64
    serial, _, _ = O.Scene(src).render(w, h, spp, 8, mode=O.RNG_SERIAL)
    out, _ = R.World(src).render(w, h, spp, 8, mode=R.RNG_COUNTER)
    d = np.abs(out[..., :3].astype(np.float64) - serial[..., :3].astype(np.float64))
    mse = float((d ** 2).mean())
    psnr = 10 * np.log10(255.0 ** 2 / mse)
    assert d.mean() < 4.0, d.mean()          # mean |diff| under 4/255 at 64 spp
    assert psnr > 28.0, psnr                 # Monte-Carlo noise only
    assert (out[..., 3] == serial[..., 3]).all()


@pytest.mark.parametrize("w,h,spp,depth", [
    (1, 5, 2, 8),    # (width-1) == 0: u = inf -> NaN ray -> black pixel
    (5, 1, 2, 8),
    (6, 4, 0, 8),    # spp = 0: sqrt(0 * inf) = NaN -> 0, alpha 255
    (6, 4, -2, 8),   # negative spp: no samples, negative reciprocal
    (6, 4, 3, 0),    # depth 0: every sample is (0, 0, 0)
    (6, 4, 3, -1),
    (7, 3, 65, 3),   # spp > 64
])
def test_edge_cases(w, h, spp, depth):
    src = scene_text(CWORLD)
    img, st, states = O.Scene(src).render(w, h, spp, depth, record_states=True)
    out, gst = R.World(src).render(w, h, spp, depth, mode=R.RNG_REPLAY,
                                   replay=states if states.size else np.zeros(1, np.uint32))
    assert_bits_equal(out, img, "edge frame")
    assert gst["rays"] == st["rays"]


@pytest.mark.parametrize("spp", [1, 3, 4, 12, 20, 64, 255, 257, 1000, 4097])
def test_in_kernel_resolve_chunking(spp):
    """Chunk and ring geometry of the in-kernel resolve: spp below, at and
    above the 256-job chunk (1000: one pixel per 1024-sample ring slot) and
    above 4096 (the slab path); 4, 12, 20, 64, 1000 take the sphere kernel's
    plane-lane fold (spp % 4 == 0, partial 16-sample rounds for 4, 12, 20 and
    1000): bit-exact against the oracle."""
    src = scene_text("rtow.txt")
    w, h = (24, 8) if spp < 1000 else (5, 3)
    img, st, _ = O.Scene(src).render(w, h, spp, 8, mode=O.RNG_COUNTER, nthreads=8)
    world = R.World(src)
    out, gst = world.render(w, h, spp, 8)
    assert_bits_equal(out, img, f"frame spp {spp}")
    assert gst["rays"] == st["rays"]
    assert gst["fused_resolve"] == (1 if spp <= 4096 else 0)


def test_read_samples_needs_keep_samples():
    world = R.World(scene_text(CWORLD))
    world.render(16, 8, 4, 8)
    with pytest.raises(R.RenderError, match="KEEP_SAMPLES"):
        world.read_samples(16 * 8 * 4)


def test_empty_and_triangle_only_scenes():
    for src in ["camera origin 0.0 0.0 0.0 aspect 1.5;",
                "camera origin 0.0 0.5 0.0 aspect 1.0;\nmaterial M : Metal color 0.9 0.2 0.2 fuzz 0.1;\n"
                "triangle v0 -1.0 -1.0 -2.0 v1 1.0 -1.0 -2.0 v2 0.0 1.0 -2.5 material M;\n"
                "triangle v0 -3.0 -0.5 -5.0 v1 3.0 -0.5 -5.0 v2 0.0 -0.5 3.0 material M;\n"]:
        img, st, states = O.Scene(src).render(24, 16, 4, 8, record_states=True)
        out, gst = R.World(src).render(24, 16, 4, 8, mode=R.RNG_REPLAY, replay=states)
        assert_bits_equal(out, img, "frame")
        assert gst["rays"] == st["rays"] and gst["tri_in_range"] == st["tri_in_range"]


def test_mesh_scene_triangle_path():
    """C5 scene (100k triangles + 100 spheres) at a size the oracle finishes."""
    src = S.mesh()
    w, h, spp = 16, 9, 1
    img, st, _, smp = O.Scene(src).render(w, h, spp, 8, mode=O.RNG_COUNTER, nthreads=8,
                                          record_samples=True)
    world = R.World(src)
    assert world.num_triangles == 100000 and world.num_spheres == 100
    out, gst = world.render(w, h, spp, 8, mode=R.RNG_COUNTER, accel=R.ACCEL_BRUTE)
    assert_bits_equal(out, img, "mesh frame (brute force)")
    assert gst["rays"] == st["rays"] and gst["tri_in_range"] == st["tri_in_range"]
    out, gst = render_kept(world, w, h, spp, 8, mode=R.RNG_COUNTER)
    assert gst["tri_bvh"] == 1
    assert_bits_equal(out, img, "mesh frame (BVH)")
    assert_bits_equal(world.read_samples(w * h * spp)[:, :3],
                      oracle_samples_to_gpu_order(smp, w, h, spp)[:, :3], "mesh samples")
    assert gst["rays"] == st["rays"]


def test_move_camera_then_render():
    src = scene_text(CWORLD)
    world = R.World(src)
    ref = O.Scene(src)
    for d in [(0.1, 0.0, 0.0), (0.0, -0.2, 0.5), (-0.3, 0.1, 0.2)]:
        world.move_camera(*d)
        cam = np.zeros(12, np.float32)
        O.lib().ro_camera_move(O.fptr(ref.camera()), d[0], d[1], d[2], O.fptr(cam))
        ref.set_camera(cam)
        assert_bits_equal(world.camera(), ref.camera(), "camera")
        img, _, _ = ref.render(32, 24, 4, 8, mode=O.RNG_COUNTER)
        out, _ = world.render(32, 24, 4, 8, mode=R.RNG_COUNTER)
        assert_bits_equal(out, img, "moved frame")


def test_tiles_assemble_to_full_frame():
    src = scene_text("rtow.txt")
    world = R.World(src)
    w, h, spp = 80, 45, 4
    full, fst = world.render(w, h, spp, 8)
    for nranks, block in [(2, 1), (3, 4), (8, 2)]:
        rays = 0
        asm = np.zeros_like(full)
        for rank in range(nranks):
            tile, st = world.render(w, h, spp, 8, row_block=block, rank=rank, nranks=nranks)
            rays += st["rays"]
            for k in range(tile.shape[0]):
                asm[R.tile_row(k, block, rank, nranks)] = tile[k]
        assert_bits_equal(asm, full, f"tiles {nranks}x{block}")
        assert rays == fst["rays"]


def test_slabs_do_not_change_the_frame(monkeypatch):
    src = scene_text("rtow.txt")
    w, h, spp = 50, 20, 8
    one, _ = R.World(src).render(w, h, spp, 8)
    monkeypatch.setenv("RT_AMD_SLAB_JOBS", str(w * spp * 3))  # 3 rows per launch
    many, st = R.World(src).render(w, h, spp, 8)
    assert st["trace_launches"] == 7
    assert_bits_equal(many, one, "slabbed frame")


@pytest.mark.parametrize("scene", ["rtow", "mesh_soup"])
def test_scheduling_knobs_do_not_change_samples(monkeypatch, scene):
    """Job-queue partitions, chunk size, walk slicing and gating, the tree's
    memory (LDS or global) and the inflation bound only change work, never a
    sample."""
    src = scene_text("rtow.txt") if scene == "rtow" else _triangle_scene(41, 400, spheres=40)
    w, h, spp = 160, 90, 4
    world = R.World(src)
    ref, _ = render_kept(world, w, h, spp, 8)
    ref_s = world.read_samples(w * h * spp)
    for env in [dict(RT_AMD_PARTS="1"), dict(RT_AMD_PARTS="7", RT_AMD_CHUNK="64"),
                dict(RT_AMD_PARTS="1024"), dict(RT_AMD_STEP="1", RT_AMD_STEPS="1"),
                dict(RT_AMD_STEP="1", RT_AMD_STEPS="5"), dict(RT_AMD_STEP="0"),
                dict(RT_AMD_REFILL="17"), dict(RT_AMD_LDS="0"),
                dict(RT_AMD_LDS="0", RT_AMD_STEP="1", RT_AMD_STEPS="3"),
                dict(RT_AMD_LINEAR_E="1"), dict(RT_AMD_PRIMARY_LISTS="0"),
                dict(RT_AMD_SPHERE_LISTS="0"), dict(RT_AMD_FUSED="0"),
                dict(RT_AMD_RESOLVE_PIX="1"), dict(RT_AMD_RESOLVE_PIX="64"),
                # walk gating: every iteration walks / walks once 8 lanes wait
                dict(RT_AMD_WALK_MIN="0"), dict(RT_AMD_WALK_MIN="8", RT_AMD_REFILL="5"),
                dict(RT_AMD_TRI_WALK_MIN="0"), dict(RT_AMD_TRI_WALK_MIN="65"),
                dict(RT_AMD_STEP="1", RT_AMD_STEPS="7", RT_AMD_WALK_MIN="65"),
                # the wide triangle walk's slices and refill rule
                dict(RT_AMD_WSTEPS="1"), dict(RT_AMD_WSTEPS="3", RT_AMD_REFILL="1"),
                dict(RT_AMD_WSTEPS="1000", RT_AMD_TRI_WALK_MIN="0")]:
        for k, v in env.items():
            monkeypatch.setenv(k, v)
        out, _ = render_kept(world, w, h, spp, 8)
        assert_bits_equal(out, ref, f"frame {env}")
        assert_bits_equal(world.read_samples(w * h * spp), ref_s, f"samples {env}")
        for k in env:
            monkeypatch.delenv(k)


@pytest.mark.parametrize("scene", ["rtow", "mesh_soup"])
def test_tree_shape_knobs_do_not_change_samples(monkeypatch, scene):
    """Leaf sizes of the sphere, triangle and camera trees, the SAH's phantom
    scale and bin counts, and the radius above which spheres stay out of the
    tree are load-time knobs: they reshape the trees, never a
    sample (every frame equals the default build's, bit for bit)."""
    src = scene_text("rtow.txt") if scene == "rtow" else _triangle_scene(41, 400, spheres=40)
    w, h, spp = 96, 54, 4
    ref, _ = render_kept(R.World(src), w, h, spp, 8)
    for env in [dict(RT_AMD_LEAF="1"), dict(RT_AMD_LEAF="3"), dict(RT_AMD_LEAF="7"), dict(RT_AMD_TRI_LEAF="2"),
                dict(RT_AMD_TRI_LEAF="7"), dict(RT_AMD_CAM_LEAF="1"), dict(RT_AMD_CAM_LEAF="5"),
                dict(RT_AMD_TRI_PHANTOM="0.5"), dict(RT_AMD_BIG_K="2"),
                dict(RT_AMD_SAH_BINS="2"), dict(RT_AMD_SAH_BINS="16"), dict(RT_AMD_TRI_SAH_BINS="4"),
                dict(RT_AMD_TRI_SAH_BINS="128"),
                dict(RT_AMD_BIG_K="1e9"), dict(RT_AMD_BIG_K="0"),
                # the binary triangle walk instead of the 4-wide image (read at device init)
                dict(RT_AMD_TRI_WIDE="0"), dict(RT_AMD_TRI_WIDE="0", RT_AMD_TRI_LEAF="3")]:
        for k, v in env.items():
            monkeypatch.setenv(k, v)
        out, _ = render_kept(R.World(src), w, h, spp, 8)
        assert_bits_equal(out, ref, f"frame {env}")
        for k in env:
            monkeypatch.delenv(k)


def test_full_size_c2_properties():
    """BASELINE configs[1] at full size: determinism + oracle parity on rows."""
    src = S.rtow()
    world = R.World(src)
    W, H, spp, depth = 1920, 1080, 64, 8
    a, st = world.render(W, H, spp, depth)
    b, st2 = world.render(W, H, spp, depth)
    assert_bits_equal(a, b, "determinism")
    assert st["rays"] == st2["rays"] and st["samples"] == W * H * spp
    assert (a[..., 3] == 255).all()
    c, st3 = world.render(W, H, spp, depth, keep_samples=True)  # 1.6 GB slab + resolve_kernel
    assert_bits_equal(c, a, "in-kernel resolve vs slab + resolve kernel")
    assert st3["rays"] == st["rays"] and st["fused_resolve"] == 1 and st3["fused_resolve"] == 0
    ref = O.Scene(src)
    rows = [0, 333, 700, 1079]  # reference rows (0 = bottom)
    img = np.zeros((H, W, 4), np.uint8)
    for r in rows:
        ref.render(W, H, spp, depth, mode=O.RNG_COUNTER, row_begin=r, row_step=H, nthreads=8,
                   out=img)
        assert_bits_equal(a[H - 1 - r], img[H - 1 - r], f"row {r}")


# ---------------------------------------------------------------- exact BVH
def _random_scene(seed, n, spread, radius, offset=(0.0, 0.0, 0.0), dup=0, big=True,
                  cam=(0.0, 0.0, 0.0)):
    rng = np.random.default_rng(seed)
    kinds = ["Diffuse color 0.7 0.5 0.3", "Metal color 0.9 0.8 0.7 fuzz 0.05",
             "Dielectric ir 1.5", "Metal color 0.6 0.6 0.9 fuzz 0.0"]
    lines = [f"camera origin {cam[0]:.6f} {cam[1]:.6f} {cam[2]:.6f} aspect 1.5;"]
    lines += [f"material K{i} : {k};" for i, k in enumerate(kinds)]
    sph = []
    if big:
        sph.append((offset[0], offset[1] - 1000.0, offset[2], 999.0, 0))
    for _ in range(n):
        c = rng.uniform(-spread, spread, 3) + np.array(offset) + np.array([0, 0, -spread - 2])
        r = radius * rng.uniform(0.3, 1.0)
        sph.append((c[0], c[1], c[2], r, int(rng.integers(0, 4))))
    sph += sph[1:1 + dup]  # exact duplicates: equal t, the lower index must win
    for (x, y, z, r, k) in sph:
        lines.append(f"sphere center {x:.6f} {y:.6f} {z:.6f} radius {r:.6f} material K{k};")
    return "\n".join(lines) + "\n"


def _both_modes(src, w, h, spp, depth=8):
    world = R.World(src)
    a, sa = render_kept(world, w, h, spp, depth, accel=R.ACCEL_BRUTE)
    sma = world.read_samples(w * h * spp)
    b, sb = render_kept(world, w, h, spp, depth, accel=R.ACCEL_BVH)
    smb = world.read_samples(w * h * spp)
    return a, sa, sma, b, sb, smb


@pytest.mark.parametrize("case", [
    dict(seed=1, n=400, spread=6.0, radius=0.3),
    dict(seed=2, n=300, spread=3.0, radius=0.6, dup=40),
    dict(seed=3, n=500, spread=20.0, radius=0.05),
    dict(seed=4, n=200, spread=5.0, radius=0.4, offset=(3000.0, -2000.0, 1500.0),
         cam=(3000.0, -2000.0, 1500.0)),
    dict(seed=5, n=250, spread=2.0, radius=0.5, big=False, cam=(0.0, 0.0, -4.0)),
])
def test_bvh_equals_brute_force(case):
    src = _random_scene(**case)
    a, sa, sma, b, sb, smb = _both_modes(src, 96, 64, 8)
    assert sb["accel"] == R.ACCEL_BVH and sa["accel"] == R.ACCEL_BRUTE
    assert_bits_equal(b, a, "frame")
    assert_bits_equal(smb[:, :3], sma[:, :3], "samples")
    assert sa["rays"] == sb["rays"]
    assert sb["bvh_sphere_tests"] + sb["big_sphere_tests"] < sa["sphere_tests"]


def test_bvh_matches_oracle_rtow():
    src = S.rtow()
    img, st, _, smp = O.Scene(src).render(64, 36, 4, 8, mode=O.RNG_COUNTER, nthreads=8,
                                          record_samples=True)
    world = R.World(src)
    out, gst = render_kept(world, 64, 36, 4, 8, accel=R.ACCEL_BVH)
    assert gst["accel"] == R.ACCEL_BVH
    assert_bits_equal(out, img, "frame")
    assert_bits_equal(world.read_samples(64 * 36 * 4)[:, :3],
                      oracle_samples_to_gpu_order(smp, 64, 36, 4)[:, :3], "samples")
    assert gst["rays"] == st["rays"]


@pytest.mark.parametrize("gpu", ["1", "0"])
def test_primary_sphere_lists_follow_camera_and_size(monkeypatch, gpu):
    """Primary rays test per-pixel candidate lists built for the camera and
    frame size (bvh.h PrimarySphereLists): after camera moves (one into the
    sphere field, one far off, which falls back to the walk) and at several
    sizes every sample equals the tree walk's and brute force.  gpu=1: the
    lists are built on the device, and every list equals the host build's
    (RT_AMD_SPL_CHECK)."""
    monkeypatch.setenv("RT_AMD_GPU_LISTS", gpu)
    monkeypatch.setenv("RT_AMD_SPL_CHECK", gpu)
    monkeypatch.setenv("RT_AMD_SYNC_LISTS", "1")  # (host build) lists built before each frame
    src = S.rtow()
    world = R.World(src)
    for mv, (w, h) in [((0.0, 0.0, 0.0), (96, 54)), ((0.0, 0.0, 0.0), (57, 31)),
                       ((0.5, -1.5, -9.0), (80, 60)), ((3.0, 0.4, -14.0), (64, 36)),
                       ((0.0, 0.0, 2000.0), (48, 27)), ((0.0, 0.0, -2000.0), (40, 30))]:
        world.move_camera(*mv)
        a, _ = render_kept(world, w, h, 4, 8, accel=R.ACCEL_BRUTE)
        sa = world.read_samples(w * h * 4)
        b, sb = render_kept(world, w, h, 4, 8, accel=R.ACCEL_BVH)
        sb_ = world.read_samples(w * h * 4)
        monkeypatch.setenv("RT_AMD_SPHERE_LISTS", "0")
        c, sc = render_kept(world, w, h, 4, 8, accel=R.ACCEL_BVH)
        sc_ = world.read_samples(w * h * 4)
        monkeypatch.delenv("RT_AMD_SPHERE_LISTS")
        assert_bits_equal(b, a, f"frame {mv} {w}x{h}")
        assert_bits_equal(sb_[:, :3], sa[:, :3], f"samples (lists) {mv} {w}x{h}")
        assert_bits_equal(sc_[:, :3], sa[:, :3], f"samples (walk) {mv} {w}x{h}")
        assert sb["rays"] == sc["rays"]
        # (lists exist unless some ball straddles the camera plane or the camera
        # is far out: then every pixel walks)
        assert sc["primary_lists"] == 0 and (sb["primary_lists"] == 1 or mv != (0.0, 0.0, 0.0))


@pytest.mark.parametrize("case,w,h", [
    (dict(seed=71, n=3000, spread=8.0, radius=0.12), 203, 117),
    (dict(seed=72, n=1500, spread=2.0, radius=0.4, dup=300), 160, 90),
    (dict(seed=73, n=800, spread=30.0, radius=0.02, big=False, cam=(0.0, 0.0, 20.0)), 97, 61),
])
def test_device_sphere_lists_many_spheres(monkeypatch, case, w, h):
    """The device list build (render.hip spl_fill_kernel: tiles, spheres culled
    256 at a time, early exit when a tile has overflowed) equals the host build
    list for list on scenes with thousands of spheres, and the frame equals
    brute force."""
    monkeypatch.setenv("RT_AMD_SPL_CHECK", "1")
    src = _random_scene(**case)
    a, sa, sma, b, sb, smb = _both_modes(src, w, h, 4)
    assert sb["primary_lists"] == 1
    assert_bits_equal(b, a, "frame")
    assert_bits_equal(smb[:, :3], sma[:, :3], "samples")


def test_device_sphere_lists_ready_on_the_first_frame():
    """Built on the device, the lists serve the first frame after every camera
    move (no host build to wait for)."""
    world = R.World(S.rtow())
    for mv in [(0.0, 0.0, 0.0), (0.4, -0.3, 1.0), (-1.0, 0.5, 3.0)]:
        world.move_camera(*mv)
        ref, _ = world.render(96, 54, 2, 8, accel=R.ACCEL_BRUTE)
        out, st = world.render(96, 54, 2, 8)
        assert st["primary_lists"] == 1
        assert_bits_equal(out, ref, f"first frame after {mv}")


def test_bvh_full_size_c2_equals_brute_force():
    """Every pixel and every sample colour of a 1920x1080x16 RTOW frame."""
    a, sa, sma, b, sb, smb = _both_modes(S.rtow(), 1920, 1080, 16)
    assert_bits_equal(b, a, "frame")
    assert np.array_equal(smb[:, :3].view(np.uint32), sma[:, :3].view(np.uint32))
    assert sa["rays"] == sb["rays"]


# ------------------------------------------------------- exact triangle BVH
_triangle_scene = S.triangle_soup


@pytest.mark.parametrize("case", [
    dict(seed=11, n=600),
    dict(seed=12, n=400, size=2.0, dup=80, slivers=30),
    dict(seed=13, n=300, spheres=200, grid=12),
    dict(seed=14, n=500, big=6, spread=8.0),
    dict(seed=15, n=400, offset=(2500.0, -1800.0, 900.0), cam=(2500.0, -1800.0, 900.0)),
    dict(seed=16, n=400, cam=(0.0, 0.0, -6.0), size=1.0),   # camera inside the soup
    dict(seed=17, n=200, grid=20, cam=(0.0, 6.0, -4.0)),   # grazing / far phantoms
])
def test_triangle_bvh_equals_brute_force(case):
    src = _triangle_scene(**case)
    a, sa, sma, b, sb, smb = _both_modes(src, 96, 64, 8)
    assert sb["tri_bvh"] == 1 and sa["tri_bvh"] == 0
    assert_bits_equal(b, a, "frame")
    assert_bits_equal(smb[:, :3], sma[:, :3], "samples")
    assert sa["rays"] == sb["rays"]
    assert sb["tri_in_range"] <= sa["tri_in_range"]


@pytest.mark.parametrize("edge", ["1.3", "2.5", "4"])
@pytest.mark.parametrize("case", [
    dict(seed=12, n=400, size=2.0, dup=80, slivers=30),
    dict(seed=13, n=300, spheres=200, grid=12),
    dict(seed=15, n=400, offset=(2500.0, -1800.0, 900.0), cam=(2500.0, -1800.0, 900.0)),
    dict(seed=16, n=400, cam=(0.0, 0.0, -6.0), size=1.0),
])
def test_triangle_cell_trees_equal_brute_force(monkeypatch, case, edge):
    """Per-origin-cell triangle trees (bvh.h TriangleCells; on by default only
    for meshes of >= 64k triangles) forced onto small soups at three cell
    edges: every sample equals brute force, whichever cell tree (or the static
    tree, for origins outside every cell) a ray walks."""
    monkeypatch.setenv("RT_AMD_TRI_CELLS", edge)
    src = _triangle_scene(**case)
    a, sa, sma, b, sb, smb = _both_modes(src, 64, 48, 8)
    assert sb["tri_bvh"] == 1
    assert_bits_equal(b, a, "frame")
    assert_bits_equal(smb[:, :3], sma[:, :3], "samples")
    assert sa["rays"] == sb["rays"]


def test_triangle_bvh_matches_oracle():
    src = _triangle_scene(21, 300, size=1.0, slivers=10, dup=20, spheres=50)
    img, st, _, smp = O.Scene(src).render(48, 32, 4, 8, mode=O.RNG_COUNTER, nthreads=8,
                                          record_samples=True)
    world = R.World(src)
    out, gst = render_kept(world, 48, 32, 4, 8)
    assert gst["tri_bvh"] == 1
    assert_bits_equal(out, img, "frame")
    assert_bits_equal(world.read_samples(48 * 32 * 4)[:, :3],
                      oracle_samples_to_gpu_order(smp, 48, 32, 4)[:, :3], "samples")


def test_triangle_bvh_c5_equals_brute_force():
    """Every sample of a 480x270x4 C5 frame (100k triangles + 100 spheres)."""
    a, sa, sma, b, sb, smb = _both_modes(S.mesh(), 480, 270, 4)
    assert sb["tri_bvh"] == 1
    assert_bits_equal(b, a, "frame")
    assert np.array_equal(smb[:, :3].view(np.uint32), sma[:, :3].view(np.uint32))
    assert sa["rays"] == sb["rays"]


@pytest.mark.parametrize("lists", ["1", "0"])
def test_triangle_camera_tree_follows_camera_moves(monkeypatch, lists):
    """Bounce-0 rays use the phantom records of the camera origin -- through
    the primary strip lists (lists=1: records only, no tree) or the camera
    tree (lists=0); moving the camera must rebuild them (every sample still
    equals brute force)."""
    monkeypatch.setenv("RT_AMD_SYNC_LISTS", "1")  # tree built before each frame
    monkeypatch.setenv("RT_AMD_PRIMARY_LISTS", lists)
    src = _triangle_scene(31, 500, size=1.0, spheres=30, grid=10)
    world = R.World(src)
    for mv in [(0.0, 0.0, 0.0), (0.5, -0.25, 1.0), (-3.0, 2.0, -4.0), (0.0, 0.0, 0.0)]:
        world.move_camera(*mv)
        a, sa = render_kept(world, 64, 48, 4, 8, accel=R.ACCEL_BRUTE)
        sma = world.read_samples(64 * 48 * 4)
        b, sb = render_kept(world, 64, 48, 4, 8, accel=R.ACCEL_BVH)
        smb = world.read_samples(64 * 48 * 4)
        assert sb["tri_bvh"] == 1 and sb["camera_tree"] == 1
        assert_bits_equal(b, a, f"frame after move {mv}")
        assert_bits_equal(smb[:, :3], sma[:, :3], f"samples after move {mv}")


def test_primary_triangle_lists_follow_camera_and_size(monkeypatch):
    """Bounce-0 rays test per-strip candidate lists built for the camera and
    the frame size: after every move and at every size each sample equals
    brute force (includes a camera inside the soup and one looking at the
    soup from behind)."""
    monkeypatch.setenv("RT_AMD_SYNC_LISTS", "1")  # lists built before each frame
    src = _triangle_scene(51, 600, size=0.8, spheres=30, grid=8)
    world = R.World(src)
    for mv, (w, h) in [((0.0, 0.0, 0.0), (128, 72)), ((0.0, 0.0, 0.0), (97, 61)),
                       ((0.3, -0.2, -5.0), (120, 80)), ((0.0, 1.5, -9.0), (64, 150)),
                       ((-2.0, 0.0, 12.0), (80, 45))]:
        world.move_camera(*mv)
        a, _ = render_kept(world, w, h, 4, 8, accel=R.ACCEL_BRUTE)
        sa = world.read_samples(w * h * 4)
        b, sb = render_kept(world, w, h, 4, 8, accel=R.ACCEL_BVH)
        smb = world.read_samples(w * h * 4)
        assert sb["tri_bvh"] == 1 and sb["camera_tree"] == 1 and sb["primary_lists"] == 1
        assert_bits_equal(b, a, f"frame {mv} {w}x{h}")
        assert_bits_equal(smb[:, :3], sa[:, :3], f"samples {mv} {w}x{h}")


@pytest.mark.parametrize("w,h,spp,depth", [(1, 5, 2, 8), (5, 1, 2, 8), (6, 4, 0, 8), (7, 3, 3, 0)])
def test_triangle_bvh_edge_frames(w, h, spp, depth):
    """Degenerate frames (W or H = 1: NaN rays; spp 0; depth 0) through the
    triangle trees: equal to the oracle bit for bit."""
    src = _triangle_scene(61, 300, spheres=20)
    img, st, _ = O.Scene(src).render(w, h, spp, depth, mode=O.RNG_COUNTER)
    out, gst = R.World(src).render(w, h, spp, depth)
    assert_bits_equal(out, img, "edge frame")
    assert gst["rays"] == st["rays"]


def test_sphere_lists_built_in_the_background_after_camera_moves(monkeypatch):
    """RT_AMD_GPU_LISTS=0: after a camera move (or on a new world) the first
    frames of a sphere scene render without the primary candidate lists while a
    host thread builds them (interactive re-render, lib.rs:60-63); the frames
    after the build use them.  Triangle scenes rebuild their camera tree and
    strip lists before the frame (parallel host build).  Every frame equals
    brute force."""
    import time

    monkeypatch.setenv("RT_AMD_GPU_LISTS", "0")

    for scene in ("rtow", "mesh_soup"):
        src = S.rtow() if scene == "rtow" else _triangle_scene(31, 500, size=1.0, spheres=30, grid=10)
        world = R.World(src)
        w, h, spp = 96, 54, 2
        # (moves that keep every sphere in front of the camera: a ball straddling
        # the camera plane sends every pixel to the walk, and the lists are empty)
        for mv in [(0.0, 0.0, 0.0), (0.4, -0.3, 1.0), (-1.0, 0.5, 3.0)]:
            world.move_camera(*mv)
            ref, _ = world.render(w, h, spp, 8, accel=R.ACCEL_BRUTE)
            out, st = world.render(w, h, spp, 8)
            assert_bits_equal(out, ref, f"{scene}: first frame after {mv}")
            if scene == "mesh_soup":
                assert st["camera_tree"] == 1 and st["primary_lists"] == 1
                continue
            assert st["primary_lists"] == 0  # the build has just been started
            deadline = time.time() + 30
            while st["primary_lists"] == 0 and time.time() < deadline:
                time.sleep(0.005)
                out, st = world.render(w, h, spp, 8)
                assert_bits_equal(out, ref, f"frame during the build after {mv}")
            assert st["primary_lists"] == 1, f"lists never adopted after {mv}"
