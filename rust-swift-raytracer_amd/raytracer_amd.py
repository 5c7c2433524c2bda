"""Python binding of libraytracer.so (the MI355X render path) over its C-ABI.

Mirrors the reference crate's FFI surface (Naxaes/Rust-Swift-Raytracer
raytracer/src/lib.rs:37-63: load_world / render / move_camera_position) plus
the extensions of include/raytracer_amd.h.  This module only marshals
arguments: every frame is rendered by the HIP kernels inside the library.
There is no CPU fallback -- without a GPU, rendering raises RenderError.
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
# RT_AMD_LIB: another build of the library (A/B timing of build variants)
LIB_PATH = os.environ.get("RT_AMD_LIB") or os.path.join(HERE, "lib", "libraytracer.so")

RNG_COUNTER, RNG_REPLAY, RNG_SERIAL = 1, 2, 3
ACCEL_AUTO, ACCEL_BRUTE, ACCEL_BVH = 0, 1, 2
FLAG_KEEP_SAMPLES = 1
FLAG_SERIAL_CHECK = 2
DEFAULT_SEED = 2547549

# Every symbol declared in include/raytracer.h and include/raytracer_amd.h.
EXPORTS = (
    "load_world", "render", "move_camera_position",
    "rt_default_options", "rt_tile_rows", "rt_tile_row", "rt_sample_seed", "rt_render_ex",
    "rt_render_device", "rt_read_samples", "rt_free_world", "rt_last_error", "rt_world_num_spheres",
    "rt_world_num_triangles", "rt_world_sphere", "rt_world_triangle", "rt_camera_get",
    "rt_last_parse_error", "rt_write_ppm", "rt_device_count", "rt_comm_count",
    "rt_world_set_sphere_material", "rt_world_set_triangle_material", "rt_assemble_tiles",
)


class RenderError(RuntimeError):
    pass


class ColorU8(C.Structure):
    _fields_ = [("r", C.c_uint8), ("g", C.c_uint8), ("b", C.c_uint8), ("a", C.c_uint8)]


class CFramebuffer(C.Structure):  # lib.rs:22-27
    _fields_ = [("width", C.c_size_t), ("height", C.c_size_t), ("pixels", C.POINTER(ColorU8))]


class WorldHandle(C.Structure):  # lib.rs:29-33
    _fields_ = [("world", C.c_void_p), ("camera", C.c_void_p)]


class RenderOptions(C.Structure):
    _fields_ = [("samples_per_pixel", C.c_int32), ("max_ray_bounces", C.c_int32),
                ("rng_mode", C.c_uint32), ("seed", C.c_uint32),
                ("replay_states", C.POINTER(C.c_uint32)), ("row_block", C.c_uint32),
                ("rank", C.c_uint32), ("nranks", C.c_uint32), ("device", C.c_int32),
                ("accel", C.c_int32), ("flags", C.c_uint32), ("ndevices", C.c_int32)]


class RenderStats(C.Structure):
    _fields_ = [("samples", C.c_uint64), ("rays", C.c_uint64), ("sphere_tests", C.c_uint64),
                ("tri_tests", C.c_uint64), ("tri_in_range", C.c_uint64),
                ("trace_ms", C.c_double), ("resolve_ms", C.c_double),
                ("trace_launches", C.c_uint32), ("waves", C.c_uint32), ("accel", C.c_uint32),
                ("bvh_sphere_tests", C.c_uint64), ("bvh_node_tests", C.c_uint64),
                ("big_sphere_tests", C.c_uint64), ("stamp_cycles", C.c_uint64 * 4),
                ("tri_node_tests", C.c_uint64), ("bvh_tri_tests", C.c_uint64),
                ("tri_bvh", C.c_uint32), ("fused_resolve", C.c_uint32), ("serial_ms", C.c_double),
                ("serial_retries", C.c_uint32), ("primary_lists", C.c_uint32),
                ("camera_tree", C.c_uint32), ("serial_iterations", C.c_uint32),
                ("serial_checked", C.c_uint64), ("serial_chain_breaks", C.c_uint64),
                ("serial_setup_ms", C.c_double),
                ("launch_parts", C.c_uint32), ("launch_chunk", C.c_uint32),
                ("launch_refill_min", C.c_uint32), ("launch_walk_min", C.c_uint32),
                ("launch_tri_walk_min", C.c_uint32), ("launch_wsteps", C.c_uint32),
                ("launch_block_threads", C.c_uint32), ("launch_blocks", C.c_uint32)]

    def as_dict(self):
        out = {}
        for k, t in self._fields_:
            v = getattr(self, k)
            out[k] = float(v) if t is C.c_double else list(v) if k == "stamp_cycles" else int(v)
        return out


_libs = {}


def build():
    subprocess.run(["make", "-s", "-C", HERE], check=True)


def lib(path=None):
    """The loaded library (another build can be loaded side by side for A/B runs)."""
    path = path or LIB_PATH
    if path not in _libs:
        # One HIP runtime per process: torch ships its own libamdhip64.so.7 /
        # librccl.so.1 (same sonames as /opt/rocm's).  Whichever loads first
        # serves both, and torch cannot initialise on /opt/rocm's runtime
        # ("No HIP GPUs are available"), so torch is loaded first when present.
        try:
            import torch  # noqa: F401
        except ImportError:
            pass
        if not os.path.exists(path):
            raise RenderError(f"{path} is missing: run `make -C {HERE}` (build())")
        L = C.CDLL(path)
        fp = C.POINTER(C.c_float)
        H = C.POINTER(WorldHandle)
        L.load_world.restype = H
        L.load_world.argtypes = [C.c_char_p]
        L.render.restype = CFramebuffer
        L.render.argtypes = [CFramebuffer, H]
        L.move_camera_position.restype = C.c_void_p
        L.move_camera_position.argtypes = [C.c_void_p, C.c_float, C.c_float, C.c_float]
        L.rt_default_options.argtypes = [C.POINTER(RenderOptions)]
        L.rt_tile_rows.restype = C.c_size_t
        L.rt_tile_rows.argtypes = [C.c_size_t, C.c_uint32, C.c_uint32, C.c_uint32]
        L.rt_tile_row.restype = C.c_size_t
        L.rt_tile_row.argtypes = [C.c_size_t, C.c_uint32, C.c_uint32, C.c_uint32]
        L.rt_sample_seed.restype = C.c_uint32
        L.rt_sample_seed.argtypes = [C.c_uint32, C.c_uint64]
        L.rt_render_ex.restype = C.c_int
        L.rt_render_ex.argtypes = [CFramebuffer, H, C.POINTER(RenderOptions),
                                   C.POINTER(RenderStats)]
        L.rt_render_device.restype = C.c_int
        L.rt_render_device.argtypes = [H, C.c_size_t, C.c_size_t, C.POINTER(RenderOptions),
                                       C.c_void_p, C.c_void_p, C.POINTER(RenderStats)]
        L.rt_read_samples.restype = C.c_long
        L.rt_read_samples.argtypes = [H, C.c_int, C.POINTER(C.c_float), C.c_size_t]
        L.rt_free_world.argtypes = [H]
        L.rt_last_error.restype = C.c_char_p
        L.rt_world_num_spheres.restype = C.c_size_t
        L.rt_world_num_spheres.argtypes = [H]
        L.rt_world_num_triangles.restype = C.c_size_t
        L.rt_world_num_triangles.argtypes = [H]
        L.rt_world_sphere.restype = C.c_int
        L.rt_world_sphere.argtypes = [H, C.c_size_t, fp]
        L.rt_world_triangle.restype = C.c_int
        L.rt_world_triangle.argtypes = [H, C.c_size_t, fp]
        L.rt_camera_get.argtypes = [C.c_void_p, fp]
        for f in (L.rt_world_set_sphere_material, L.rt_world_set_triangle_material):
            f.restype = C.c_int
            f.argtypes = [H, C.c_size_t, fp]
        L.rt_last_parse_error.restype = C.c_int
        L.rt_write_ppm.restype = C.c_int
        L.rt_write_ppm.argtypes = [C.POINTER(CFramebuffer), C.c_char_p]
        L.rt_device_count.restype = C.c_int
        L.rt_comm_count.restype = C.c_int
        L.rt_comm_count.argtypes = [C.c_int, C.c_int]
        L.rt_assemble_tiles.restype = C.c_int
        L.rt_assemble_tiles.argtypes = [C.c_void_p, C.c_void_p, C.c_size_t, C.c_size_t, C.c_uint32,
                                        C.c_uint32, C.c_size_t, C.c_void_p]
        _libs[path] = L
    return _libs[path]


def last_error() -> str:
    return lib().rt_last_error().decode("utf-8", "replace")


def device_count() -> int:
    return int(lib().rt_device_count())


def comm_count(first: int, n: int) -> int:
    """Ranks of the RCCL communicator a multi-device frame over devices
    [first, first + n) uses (created on first use); raises on error."""
    r = int(lib().rt_comm_count(first, n))
    if r < 0:
        raise RenderError(f"rt_comm_count failed ({r}): {last_error()}")
    return r


def assemble_tiles(gathered_ptr: int, out_ptr: int, width, height, row_block, nranks, max_rows,
                   stream_ptr: int = 0):
    """rt_assemble_tiles: the multi-device frame assembly on device buffers."""
    rc = lib().rt_assemble_tiles(C.c_void_p(gathered_ptr), C.c_void_p(out_ptr), width, height, row_block,
                                 nranks, max_rows, C.c_void_p(stream_ptr or None))
    if rc != 0:
        raise RenderError(f"rt_assemble_tiles failed ({rc}): {last_error()}")


def tile_rows(height, row_block, rank, nranks) -> int:
    return int(lib().rt_tile_rows(height, row_block, rank, nranks))


def tile_row(k, row_block, rank, nranks) -> int:
    return int(lib().rt_tile_row(k, row_block, rank, nranks))


def sample_seed(seed: int, job: int) -> int:
    return int(lib().rt_sample_seed(seed, job))


def options(spp=16, depth=8, mode=RNG_COUNTER, seed=DEFAULT_SEED, replay=None, row_block=8,
            rank=0, nranks=1, device=-1, accel=ACCEL_AUTO, keep_samples=False, L=None,
            ndevices=0, serial_check=False):
    o = RenderOptions()
    (L or lib()).rt_default_options(C.byref(o))
    o.samples_per_pixel, o.max_ray_bounces, o.rng_mode, o.seed = spp, depth, mode, seed
    o.row_block, o.rank, o.nranks, o.device = row_block, rank, nranks, device
    o.accel = accel
    o.ndevices = ndevices
    o.flags = (FLAG_KEEP_SAMPLES if keep_samples else 0) | (FLAG_SERIAL_CHECK if serial_check else 0)
    keep = None
    if replay is not None:
        keep = np.ascontiguousarray(replay, dtype=np.uint32)
        o.replay_states = keep.ctypes.data_as(C.POINTER(C.c_uint32))
    return o, keep


class World:
    """A loaded world: load_world (lib.rs:37-46) + camera moves + rendering."""

    def __init__(self, source: str | bytes, lib_path=None):
        self._L = lib(lib_path)
        if isinstance(source, str):
            source = source.encode("utf-8")
        self._h = self._L.load_world(source)
        if not self._h:
            raise ValueError(f"load_world failed: parse error {self._L.rt_last_parse_error()}")

    def close(self):
        if getattr(self, "_h", None):
            self._L.rt_free_world(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    @property
    def handle(self):
        return self._h

    @property
    def num_spheres(self):
        return int(self._L.rt_world_num_spheres(self._h))

    @property
    def num_triangles(self):
        return int(self._L.rt_world_num_triangles(self._h))

    def spheres(self):
        out = np.zeros((self.num_spheres, 10), np.float32)
        for i in range(self.num_spheres):
            self._L.rt_world_sphere(self._h, i, out[i].ctypes.data_as(C.POINTER(C.c_float)))
        return out

    def triangles(self):
        out = np.zeros((self.num_triangles, 18), np.float32)
        for i in range(self.num_triangles):
            self._L.rt_world_triangle(self._h, i, out[i].ctypes.data_as(C.POINTER(C.c_float)))
        return out

    def set_material(self, i, kind, rgb, param=0.0, triangle=False):
        """rt_world_set_{sphere,triangle}_material: kind 0 Diffuse, 1 Metal,
        2 Dielectric, 3 Emission (materials.rs:7-12)."""
        m = np.array([kind, rgb[0], rgb[1], rgb[2], 1.0, param], np.float32)
        f = self._L.rt_world_set_triangle_material if triangle else self._L.rt_world_set_sphere_material
        if f(self._h, i, m.ctypes.data_as(C.POINTER(C.c_float))) != 0:
            raise ValueError(f"set_material failed: {last_error()}")

    def camera(self):
        c = np.zeros(12, np.float32)
        self._L.rt_camera_get(self._h.contents.camera, c.ctypes.data_as(C.POINTER(C.c_float)))
        return c

    def move_camera(self, x, y, z):
        """GameView.swift:200-216: handle.camera = move_camera_position(camera, ...)."""
        self._h.contents.camera = self._L.move_camera_position(self._h.contents.camera, x, y, z)

    def render_reference(self, width, height):
        """The reference ABI call render(fb, handle): 16 spp, depth 8 (lib.rs:49-57)."""
        px = np.zeros((height, width, 4), np.uint8)
        fb = CFramebuffer(width, height, px.ctypes.data_as(C.POINTER(ColorU8)))
        res = self._L.render(fb, self._h)
        if not res.pixels and width * height:
            raise RenderError(self._L.rt_last_error().decode())
        return px

    def render(self, width, height, spp=16, depth=8, mode=RNG_COUNTER, seed=DEFAULT_SEED,
               replay=None, row_block=8, rank=0, nranks=1, device=-1, accel=ACCEL_AUTO,
               keep_samples=False, stats=True, ndevices=0, serial_check=False):
        """rt_render_ex -> (rgba uint8[tile_rows, width, 4], stats dict).
        keep_samples: write every sample to the slab (for read_samples) and
        resolve with the second kernel; the frame is bit-identical.
        stats=False: no counters (the kernel variant without them; stats None).
        ndevices >= 1: the whole frame, row-tiled over that many devices of this
        process and gathered with RCCL (RtRenderOptions.ndevices).
        serial_check: RT_FLAG_SERIAL_CHECK (SERIAL: verify the start-state chain)."""
        o, keep = options(spp, depth, mode, seed, replay, row_block, rank, nranks, device, accel,
                          keep_samples, self._L, ndevices, serial_check)
        rows = int(self._L.rt_tile_rows(height, row_block, rank, nranks)) if nranks > 1 else height
        px = np.zeros((rows, width, 4), np.uint8)
        fb = CFramebuffer(width, height, px.ctypes.data_as(C.POINTER(ColorU8)))
        st = RenderStats()
        rc = self._L.rt_render_ex(fb, self._h, C.byref(o), C.byref(st) if stats else None)
        del keep
        if rc != 0:
            raise RenderError(f"rt_render_ex failed ({rc}): {self._L.rt_last_error().decode()}")
        return px, (st.as_dict() if stats else None)

    def read_samples(self, njobs, device=-1):
        """Per-sample colours of the last trace launch: float32[njobs, 4]."""
        out = np.zeros((njobs, 4), np.float32)
        n = self._L.rt_read_samples(self._h, device, out.ctypes.data_as(C.POINTER(C.c_float)),
                                  out.size)
        if n < 0:
            raise RenderError(f"rt_read_samples failed ({n}): {self._L.rt_last_error().decode()}")
        return out[: n // 4]

    def render_device(self, width, height, out_ptr: int, stream_ptr: int = 0, spp=16, depth=8,
                      mode=RNG_COUNTER, seed=DEFAULT_SEED, row_block=8, rank=0, nranks=1,
                      device=-1, accel=ACCEL_AUTO, stats=True, keep_samples=False, ndevices=0,
                      serial_check=False):
        """rt_render_device into a device buffer (e.g. a torch uint8 tensor).
        stats=False: no counters and no host wait -- the frame is only enqueued
        on the stream (returns None)."""
        o, _ = options(spp, depth, mode, seed, None, row_block, rank, nranks, device, accel,
                       keep_samples, self._L, ndevices, serial_check)
        st = RenderStats()
        rc = self._L.rt_render_device(self._h, width, height, C.byref(o), C.c_void_p(out_ptr),
                                    C.c_void_p(stream_ptr or None), C.byref(st) if stats else None)
        if rc != 0:
            raise RenderError(f"rt_render_device failed ({rc}): {self._L.rt_last_error().decode()}")
        return st.as_dict() if stats else None


def write_ppm(rgba: np.ndarray, path: str):
    h, w = rgba.shape[:2]
    a = np.ascontiguousarray(rgba, dtype=np.uint8)
    fb = CFramebuffer(w, h, a.ctypes.data_as(C.POINTER(ColorU8)))
    if lib().rt_write_ppm(C.byref(fb), path.encode()) != 0:
        raise OSError(f"cannot write {path}")
