"""ctypes binding of the CPU oracle (oracle/rt_oracle.cpp).

TEST INFRASTRUCTURE ONLY: imported by tests/, __graft_entry__.smoke() and
bench.py's cpu_baseline leg -- never by the product package.  See
rt_oracle.h for what the oracle restates and its parity status.
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, "build", "liboracle_rt.so")

RNG_SERIAL, RNG_COUNTER, RNG_REPLAY = 0, 1, 2
DEFAULT_SEED = 2547549  # random.rs:9


class Stats(C.Structure):
    _fields_ = [("samples", C.c_uint64), ("rays", C.c_uint64), ("sphere_tests", C.c_uint64),
                ("tri_tests", C.c_uint64), ("tri_in_range", C.c_uint64)]

    def as_dict(self):
        return {k: int(getattr(self, k)) for k, _ in self._fields_}


_lib = None


def build():
    subprocess.run(["make", "-s", "-C", _HERE], check=True)


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            build()
        L = C.CDLL(LIB_PATH)
        fp = C.POINTER(C.c_float)
        u32p = C.POINTER(C.c_uint32)
        L.ro_parse.restype = C.c_void_p
        L.ro_parse.argtypes = [C.c_char_p]
        L.ro_scene_free.argtypes = [C.c_void_p]
        L.ro_last_parse_error.restype = C.c_int
        L.ro_scene_num_spheres.restype = C.c_size_t
        L.ro_scene_num_spheres.argtypes = [C.c_void_p]
        L.ro_scene_num_triangles.restype = C.c_size_t
        L.ro_scene_num_triangles.argtypes = [C.c_void_p]
        L.ro_scene_camera.argtypes = [C.c_void_p, fp]
        L.ro_scene_set_camera.argtypes = [C.c_void_p, fp]
        L.ro_scene_set_material.restype = C.c_int
        L.ro_scene_set_material.argtypes = [C.c_void_p, C.c_int, C.c_size_t, fp]
        L.ro_scene_sphere.argtypes = [C.c_void_p, C.c_size_t, fp]
        L.ro_scene_triangle.argtypes = [C.c_void_p, C.c_size_t, fp]
        L.ro_camera_new_at.argtypes = [fp, C.c_float, fp]
        L.ro_camera_move.argtypes = [fp, C.c_float, C.c_float, C.c_float, fp]
        L.ro_sample_seed.restype = C.c_uint32
        L.ro_sample_seed.argtypes = [C.c_uint32, C.c_uint64]
        L.ro_render.restype = C.c_int
        L.ro_render.argtypes = [C.c_void_p, C.c_size_t, C.c_size_t, C.c_int, C.c_int, C.c_int,
                                C.c_uint32, u32p, C.c_size_t, C.c_size_t, C.c_int,
                                C.POINTER(C.c_uint8), u32p, fp, C.POINTER(Stats)]
        L.ro_render_cols.restype = C.c_int
        L.ro_render_cols.argtypes = [C.c_void_p, C.c_size_t, C.c_size_t, C.c_int, C.c_int, C.c_int,
                                     C.c_uint32, u32p, C.c_size_t, C.c_size_t, C.c_size_t, C.c_size_t,
                                     C.c_int, C.POINTER(C.c_uint8), u32p, fp, C.POINTER(Stats)]
        L.ro_xorshift32.restype = C.c_uint32
        L.ro_xorshift32.argtypes = [u32p]
        L.ro_random_f32.restype = C.c_float
        L.ro_random_f32.argtypes = [u32p]
        L.ro_reflect.argtypes = [fp, fp, fp]
        L.ro_refract.argtypes = [fp, fp, C.c_float, fp]
        L.ro_normalize.argtypes = [fp, fp]
        L.ro_sphere_hit.restype = C.c_int
        L.ro_sphere_hit.argtypes = [fp, fp, C.c_float, C.c_float, C.c_float, fp]
        L.ro_triangle_intersect.restype = C.c_int
        L.ro_triangle_intersect.argtypes = [fp, fp, C.c_float, C.c_float, fp]
        L.ro_scatter.restype = C.c_int
        L.ro_scatter.argtypes = [fp, fp, fp, u32p, fp, fp]
        L.ro_sky.argtypes = [fp, fp, fp]
        L.ro_cast_ray.argtypes = [fp, C.c_float, C.c_float, fp]
        L.ro_as_u8.restype = C.c_uint8
        L.ro_as_u8.argtypes = [C.c_float]
        L.ro_write_ppm.restype = C.c_long
        L.ro_write_ppm.argtypes = [C.POINTER(C.c_uint8), C.c_size_t, C.c_size_t, C.c_char_p,
                                   C.c_size_t]
        _lib = L
    return _lib


def f32arr(x, n=None):
    a = np.ascontiguousarray(np.asarray(x, dtype=np.float32))
    if n is not None and a.size < n:
        a = np.concatenate([a, np.zeros(n - a.size, np.float32)])
    return a


def fptr(a):
    return a.ctypes.data_as(C.POINTER(C.c_float))


class Scene:
    """A parsed scene (parser.rs restatement)."""

    def __init__(self, source: str | bytes):
        if isinstance(source, str):
            source = source.encode("utf-8")
        self._h = lib().ro_parse(source)
        if not self._h:
            raise ValueError(f"parse error {lib().ro_last_parse_error()}")

    def __del__(self):
        if getattr(self, "_h", None):
            lib().ro_scene_free(self._h)
            self._h = None

    @property
    def num_spheres(self):
        return int(lib().ro_scene_num_spheres(self._h))

    @property
    def num_triangles(self):
        return int(lib().ro_scene_num_triangles(self._h))

    def camera(self):
        c = np.zeros(12, np.float32)
        lib().ro_scene_camera(self._h, fptr(c))
        return c

    def set_material(self, i, kind, rgb, param=0.0, triangle=False):
        m = np.array([kind, rgb[0], rgb[1], rgb[2], 1.0, param], np.float32)
        if lib().ro_scene_set_material(self._h, 1 if triangle else 0, i, fptr(m)) != 0:
            raise IndexError(i)

    def set_camera(self, cam):
        c = f32arr(cam)
        lib().ro_scene_set_camera(self._h, fptr(c))

    def spheres(self):
        out = np.zeros((self.num_spheres, 10), np.float32)
        for i in range(self.num_spheres):
            lib().ro_scene_sphere(self._h, i, fptr(out[i]))
        return out

    def triangles(self):
        out = np.zeros((self.num_triangles, 18), np.float32)
        for i in range(self.num_triangles):
            lib().ro_scene_triangle(self._h, i, fptr(out[i]))
        return out

    def render(self, width, height, spp, depth, mode=RNG_SERIAL, seed=DEFAULT_SEED,
               replay=None, row_begin=0, row_step=1, nthreads=1, record_states=False,
               record_samples=False, out=None, col_begin=0, col_step=1):
        """Returns (rgba[H, W, 4] uint8, stats dict, states or None[, samples]).

        samples (when record_samples): float32[W*H*spp, 4] ray_color results
        indexed by job = (row*W + col)*spp + s (row 0 = bottom)."""
        if out is None:
            out = np.zeros((height, width, 4), np.uint8)
        states = None
        sp = None
        if record_states:
            states = np.zeros(width * height * max(spp, 0), np.uint32)
            sp = states.ctypes.data_as(C.POINTER(C.c_uint32))
        rp = None
        if replay is not None:
            replay = np.ascontiguousarray(replay, dtype=np.uint32)
            rp = replay.ctypes.data_as(C.POINTER(C.c_uint32))
        samples = None
        smp = None
        if record_samples:
            samples = np.zeros((width * height * max(spp, 0), 4), np.float32)
            smp = fptr(samples)
        st = Stats()
        rc = lib().ro_render_cols(self._h, width, height, spp, depth, mode, seed, rp, row_begin,
                                  row_step, col_begin, col_step, nthreads,
                                  out.ctypes.data_as(C.POINTER(C.c_uint8)), sp, smp, C.byref(st))
        if rc != 0:
            raise RuntimeError(f"ro_render failed: {rc}")
        if record_samples:
            return out, st.as_dict(), states, samples
        return out, st.as_dict(), states


def sample_seed(seed: int, job: int) -> int:
    return int(lib().ro_sample_seed(seed, job))


def xorshift_stream(seed: int, n: int):
    s = C.c_uint32(seed)
    return [int(lib().ro_xorshift32(C.byref(s))) for _ in range(n)]


def random_f32_stream(seed: int, n: int):
    s = C.c_uint32(seed)
    return [float(lib().ro_random_f32(C.byref(s))) for _ in range(n)]


def ppm(rgba: np.ndarray) -> bytes:
    h, w = rgba.shape[:2]
    a = np.ascontiguousarray(rgba, dtype=np.uint8)
    n = lib().ro_write_ppm(a.ctypes.data_as(C.POINTER(C.c_uint8)), w, h, None, 0)
    buf = C.create_string_buffer(n)
    lib().ro_write_ppm(a.ctypes.data_as(C.POINTER(C.c_uint8)), w, h, buf, n)
    return buf.raw[:n]
