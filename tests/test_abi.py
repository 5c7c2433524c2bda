"""CPU tests of the drop-in C-ABI boundary (no GPU compute calls).

The library must load, export every function include/raytracer.h and
include/raytracer_amd.h declare, keep the reference's struct layouts
(lib.rs:22-33, color.rs:3-10 / raytracer.h:12-34), build the C twin of
examples/c_raytracer.rs against the header, and refuse loudly to render
without a GPU (there is no CPU fallback).
"""
import ctypes as C
import os
import re
import subprocess

import numpy as np
import pytest

import oracle as O
import raytracer_amd as R
from conftest import ROOT, scene_text

INC = os.path.join(ROOT, "include")


def declared_functions(header):
    txt = open(os.path.join(INC, header)).read()
    txt = re.sub(r"/\*.*?\*/", "", txt, flags=re.S)
    names = re.findall(r"\b([A-Za-z_][A-Za-z0-9_]*)\s*\([^;{]*\)\s*;", txt)
    return sorted(set(n for n in names if n not in ("sizeof",)))


@pytest.mark.parametrize("header", ["raytracer.h", "raytracer_amd.h"])
def test_library_exports_every_declared_symbol(header):
    names = declared_functions(header)
    assert names, header
    lib = C.CDLL(R.LIB_PATH)
    missing = [n for n in names if not hasattr(lib, n)]
    assert not missing, missing
    assert set(names) <= set(R.EXPORTS)


def test_reference_entry_points_present():
    assert declared_functions("raytracer.h") == ["load_world", "move_camera_position", "render"]


def test_no_oracle_code_in_the_product():
    out = subprocess.run(["nm", "-D", "--defined-only", R.LIB_PATH], capture_output=True,
                         text=True, check=True).stdout
    assert "ro_" not in " ".join(line.split()[-1] for line in out.splitlines()
                                 if line.split()[-1].startswith("ro_"))
    ldd = subprocess.run(["ldd", R.LIB_PATH], capture_output=True, text=True).stdout
    assert "oracle" not in ldd and "amdhip64" in ldd


def test_struct_layouts_match_reference_abi(tmp_path):
    src = tmp_path / "layout.c"
    src.write_text(r"""
#include <stddef.h>
#include "raytracer.h"
#include "raytracer_amd.h"
_Static_assert(sizeof(Rust_ColorU8) == 4, "ColorU8");
_Static_assert(offsetof(Rust_ColorU8, a) == 3, "ColorU8.a");
_Static_assert(sizeof(Rust_CFramebuffer) == 24, "CFramebuffer");
_Static_assert(offsetof(Rust_CFramebuffer, pixels) == 16, "CFramebuffer.pixels");
_Static_assert(sizeof(Rust_WorldHandle) == 16, "WorldHandle");
_Static_assert(offsetof(Rust_WorldHandle, camera) == 8, "WorldHandle.camera");
_Static_assert(sizeof(Rust_NVec3) == 12, "NVec3");
#include <stdio.h>
int main(void) {
  printf("%zu %zu %zu %zu %zu\n", sizeof(RtRenderOptions), offsetof(RtRenderOptions, ndevices),
         sizeof(RtRenderStats), offsetof(RtRenderStats, fused_resolve),
         offsetof(RtRenderStats, serial_ms));
  return 0;
}
""")
    subprocess.run(["gcc", "-std=c11", "-Wall", "-Werror", f"-I{INC}", "-o",
                    str(tmp_path / "layout"), str(src)], check=True)
    assert C.sizeof(R.CFramebuffer) == 24 and C.sizeof(R.WorldHandle) == 16
    # the ctypes mirrors of the extension structs match the C layouts
    got = subprocess.run([str(tmp_path / "layout")], capture_output=True, text=True,
                         check=True).stdout.split()
    assert [int(x) for x in got] == [C.sizeof(R.RenderOptions), R.RenderOptions.ndevices.offset,
                                     C.sizeof(R.RenderStats), R.RenderStats.fused_resolve.offset,
                                     R.RenderStats.serial_ms.offset]


def test_c_example_links_against_the_header():
    exe = os.path.join(ROOT, "examples", "c_raytracer")
    assert os.path.exists(exe)
    out = subprocess.run(["nm", "-u", exe], capture_output=True, text=True).stdout
    for sym in ("load_world", "render"):
        assert sym in out


def test_default_options_are_the_reference_hard_codes():
    o, _ = R.options()
    assert (o.samples_per_pixel, o.max_ray_bounces) == (16, 8)  # lib.rs:51
    assert o.seed == 2547549 and o.rng_mode == R.RNG_COUNTER and o.nranks == 1
    assert o.ndevices == 0 and o.row_block == 8  # one device unless asked
    raw = R.RenderOptions()
    R.lib().rt_default_options(C.byref(raw))  # the C default: render()'s settings
    assert raw.rng_mode == R.RNG_SERIAL and raw.samples_per_pixel == 16


def test_counter_seed_spec_matches_oracle():
    for j in [0, 1, 2, 17, 1 << 20, (1 << 32) + 5, 132710399, 2123366399]:
        assert R.sample_seed(2547549, j) == O.sample_seed(2547549, j)
        assert R.sample_seed(7, j) == O.sample_seed(7, j)
        assert R.sample_seed(2547549, j) != 0


def test_tile_geometry_helpers():
    assert R.tile_rows(1080, 8, 0, 1) == 1080
    assert sum(R.tile_rows(1080, 8, r, 8) for r in range(8)) == 1080
    assert R.tile_row(0, 8, 3, 8) == 24 and R.tile_row(9, 8, 3, 8) == 64 + 24 + 1
    assert R.tile_rows(10, 8, 9, 8) == 0  # rank out of range


@pytest.mark.skipif(R.device_count() > 0, reason="a GPU is present")
def test_render_fails_loudly_without_gpu():
    w = R.World(scene_text("world.txt"))
    with pytest.raises(R.RenderError, match="no HIP device"):
        w.render(8, 8)
    px = np.zeros((8, 8, 4), np.uint8)
    fb = R.CFramebuffer(8, 8, px.ctypes.data_as(C.POINTER(R.ColorU8)))
    res = R.lib().render(fb, w.handle)
    assert not res.pixels and res.width == 0


@pytest.mark.skipif(R.device_count() > 0, reason="a GPU is present")
def test_multi_device_mode_fails_loudly_without_gpu():
    w = R.World(scene_text("world.txt"))
    for n in (1, 2, 8):
        with pytest.raises(R.RenderError, match="no HIP device"):
            w.render(8, 8, ndevices=n)
        with pytest.raises(R.RenderError, match="no HIP device"):
            R.comm_count(0, n)


def test_load_world_null_and_free():
    assert not R.lib().load_world(None)
    w = R.World(scene_text("c_raytracer_world.txt"))
    assert w.num_spheres == 8 and w.num_triangles == 2
    w.close()
    w.close()


def test_write_ppm(tmp_path):
    img = np.zeros((2, 3, 4), np.uint8)
    img[1, 2] = [7, 8, 9, 255]
    p = tmp_path / "x.ppm"
    R.write_ppm(img, str(p))
    assert p.read_text() == O.ppm(img).decode()


def test_render_null_arguments_return_empty_framebuffer():
    """A caller's bad arguments (NULL handle, NULL pixels) come back as the
    documented {0, 0, NULL} framebuffer, with or without a GPU, and a NULL
    camera is passed through by move_camera_position (lib.rs:49-63)."""
    px = np.zeros((8, 8, 4), np.uint8)
    fb = R.CFramebuffer(8, 8, px.ctypes.data_as(C.POINTER(R.ColorU8)))
    res = R.lib().render(fb, None)
    assert not res.pixels and res.width == 0 and res.height == 0
    w = R.World(scene_text("world.txt"))
    res = R.lib().render(R.CFramebuffer(8, 8, None), w.handle)
    assert not res.pixels and res.width == 0 and res.height == 0
    assert not px.any()
    assert not R.lib().move_camera_position(None, 0.0, 0.0, 1.0)


def test_frame_kernel_hash_covers_the_lean_frame_kernels():
    """bench.py keys roofline.traffic on tools/kernel_hash.py: the gfx950 code
    of the 24 lean frame variants of trace_kernel inside the built library
    (3 sphere searches x 2 walk kinds x 4 mesh kinds), found in the offload
    bundle; the hash is stable across reads."""
    import sys

    sys.path.insert(0, os.path.join(ROOT, "tools"))
    import kernel_hash

    digest, names = kernel_hash.frame_kernel_hash(R.LIB_PATH)
    assert len(names) == 24 and all("trace_kernel" in n for n in names)
    assert re.fullmatch(r"[0-9a-f]{64}", digest)
    assert kernel_hash.frame_kernel_hash(R.LIB_PATH)[0] == digest
