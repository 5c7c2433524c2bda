"""GPU parity at BASELINE.json configs[2] (C3: 3840x2160, 256 spp, depth 16)
and configs[3] (C4: C3 row-tiled over 8 ranks).

The reference path is ray_trace/ray_color at those settings (common.rs:320-361,
263-285).  C3 runs as ONE trace launch of 2.12 G jobs (uint32 job, partition
and ring-offset arithmetic, ~600 MB of per-wave rings), so these tests pin the
largest-launch path:
  * a small depth-16 / spp-256 frame, bit-exact against the oracle (COUNTER);
  * the full C3 frame: deterministic, alpha 255 everywhere, and four rows
    bit-exact against the oracle (COUNTER);
  * C4 on one GPU: the eight row tiles (blocks of 8 rows, ranks 0-7) of the
    C3 frame reassemble to the one-rank frame bit for bit, and their ray
    counts sum to the one-rank count.
"""
import numpy as np
import pytest

import oracle as O
import raytracer_amd as R
import scenes as S
from test_gpu_parity import assert_bits_equal, oracle_samples_to_gpu_order, render_kept

pytestmark = pytest.mark.gpu

C3 = dict(W=3840, H=2160, spp=256, depth=16)


@pytest.fixture(scope="module")
def rtow():
    src = S.rtow()
    return src, R.World(src)


@pytest.fixture(scope="module")
def c3_frame(rtow):
    _, world = rtow
    return world.render(C3["W"], C3["H"], C3["spp"], C3["depth"])


def test_c3_settings_small_frame_bit_exact(rtow):
    """depth 16, spp 256 (one 256-sample pixel per ring slot) vs oracle COUNTER."""
    src, world = rtow
    w, h, spp, depth = 32, 18, 256, 16
    out, st = render_kept(world, w, h, spp, depth)
    img, ost, _, smp = O.Scene(src).render(w, h, spp, depth, mode=O.RNG_COUNTER, nthreads=8,
                                           record_samples=True)
    assert_bits_equal(out, img, "C3-settings frame")
    assert st["rays"] == ost["rays"] and st["samples"] == w * h * spp
    assert_bits_equal(world.read_samples(w * h * spp)[:, :3],
                      oracle_samples_to_gpu_order(smp, w, h, spp)[:, :3], "samples")


def test_c3_full_size_properties(rtow, c3_frame):
    """configs[2] at full size in one launch: determinism, alpha, oracle rows."""
    src, world = rtow
    W, H, spp, depth = C3["W"], C3["H"], C3["spp"], C3["depth"]
    a, st = c3_frame
    assert st["trace_launches"] == 1 and st["fused_resolve"] == 1
    assert st["samples"] == W * H * spp
    b, st2 = world.render(W, H, spp, depth, stats=False)  # the timed (counter-free) variant
    assert_bits_equal(a, b, "determinism (counting vs lean kernel)")
    assert (a[..., 3] == 255).all()
    ref = O.Scene(src)
    img = np.zeros((H, W, 4), np.uint8)
    for r in (0, 700, 1500, 2159):  # reference rows (0 = bottom)
        ref.render(W, H, spp, depth, mode=O.RNG_COUNTER, row_begin=r, row_step=H, nthreads=16,
                   out=img)
        assert_bits_equal(a[H - 1 - r], img[H - 1 - r], f"C3 row {r}")


def test_c4_eight_tiles_reassemble_to_c3(rtow, c3_frame):
    """configs[3] on one GPU: ranks 0-7, blocks of 8 rows (bench.py ROW_BLOCK)."""
    _, world = rtow
    W, H, spp, depth = C3["W"], C3["H"], C3["spp"], C3["depth"]
    full, fst = c3_frame
    nranks, block = 8, 8
    asm = np.zeros_like(full)
    rays = 0
    for rank in range(nranks):
        tile, st = world.render(W, H, spp, depth, row_block=block, rank=rank, nranks=nranks)
        # 270 blocks of 8 rows over 8 ranks: 34 blocks (272 rows) or 33 (264)
        assert tile.shape == (R.tile_rows(H, block, rank, nranks), W, 4)
        assert tile.shape[0] in (264, 272)
        rays += st["rays"]
        rows = [R.tile_row(k, block, rank, nranks) for k in range(tile.shape[0])]
        asm[rows] = tile
    assert_bits_equal(asm, full, "C4 tiles")
    assert rays == fst["rays"]
