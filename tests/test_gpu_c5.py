"""GPU parity at BASELINE.json configs[4] (C5: the 100k-triangle mesh scene,
1920x1080, 64 spp, depth 8) at full size.

The path is ray_color's Mesh::hit (common.rs:124-166, 177-224) through the
phantom-aware static tree, the camera tree and the primary strip lists
(DESIGN.md 5.3).  The oracle cannot brute-force a full C5 row in test time
(2.7e10 triangle tests per row), so the full frame is pinned by:
  * determinism: the counting and the lean (timed) kernel give the same bits;
  * alpha 255 everywhere, and every sample traced;
  * two full rows re-rendered by brute force on the GPU (the reference's
    triangle order and t_max, RT_ACCEL_BRUTE, one-row tiles) bit-equal to the
    full frame's rows.
Brute force itself equals the oracle bit for bit on smaller frames
(test_gpu_parity.py test_triangle_bvh_matches_oracle, test_mesh_scene_triangle_path).
"""
import numpy as np
import pytest

import raytracer_amd as R
import scenes as S
from test_gpu_parity import assert_bits_equal

pytestmark = pytest.mark.gpu

C5 = dict(W=1920, H=1080, spp=64, depth=8)


@pytest.fixture(scope="module")
def mesh():
    src = S.mesh()
    return src, R.World(src)


def test_c5_full_size_properties(mesh):
    _, world = mesh
    W, H, spp, depth = C5["W"], C5["H"], C5["spp"], C5["depth"]
    a, st = world.render(W, H, spp, depth)
    assert st["tri_bvh"] == 1 and st["camera_tree"] == 1 and st["primary_lists"] == 1
    assert st["samples"] == W * H * spp
    b, _ = world.render(W, H, spp, depth, stats=False)  # the timed (counter-free) variant
    assert_bits_equal(a, b, "determinism (counting vs lean kernel)")
    assert (a[..., 3] == 255).all()
    for q in (460, 780):  # image rows (0 = top)
        # a one-row tile: row_block 1, rank q of H ranks holds image row q
        t, tst = world.render(W, H, spp, depth, row_block=1, rank=q, nranks=H, accel=R.ACCEL_BRUTE)
        assert tst["tri_bvh"] == 0 and R.tile_row(0, 1, q, H) == q
        assert_bits_equal(a[q], t.reshape(-1, W, 4)[0], f"C5 image row {q} vs brute force")


def test_c5_full_size_row_vs_oracle(mesh):
    """Every 8th pixel of a C5 row at the full settings (64 spp, depth 8)
    of the full-size frame, bit-compared with the oracle's brute-force
    Mesh::hit (common.rs:177-224, every one of the 100k triangles per ray, in
    file order) in COUNTER mode on 16 host threads: the phantom-aware trees,
    camera records and strip lists of the GPU frame against the reference's
    own loop at full size."""
    import oracle as O

    src, world = mesh
    W, H, spp, depth = C5["W"], C5["H"], C5["spp"], C5["depth"]
    a, _ = world.render(W, H, spp, depth, stats=False)
    ref = O.Scene(src)
    img = np.zeros((H, W, 4), np.uint8)
    r = 300  # reference row (0 = bottom): image row 779, across the mesh wall
    cols = slice(3, W, 8)  # every 8th pixel: 240 pixels x 64 samples (~10-20 s on 16 threads)
    ref.render(W, H, spp, depth, mode=O.RNG_COUNTER, row_begin=r, row_step=H, col_begin=3, col_step=8,
               nthreads=16, out=img)
    assert_bits_equal(a[H - 1 - r, cols], img[H - 1 - r, cols], f"C5 reference row {r} vs oracle")
