"""Deterministic synthetic scenes for the BASELINE.json configs, emitted in the
reference's scene DSL (parser.rs:326-335) so that load_world parses them.

  three_spheres()  C1: world.txt camera + GROUND, BALL, METAL_MATERIAL_1, GLASS
                   materials and the ground + 3 ball spheres (world.txt lines
                   1, 6, 7, 9, 13, 15, 17-19).
  rtow(n)          C2/C3: "Ray Tracing in One Weekend" final scene, ~485
                   spheres, generated with xorshift32 (scene seed 0x2547549).
  mesh(...)        C5: 100,000-triangle displaced grid + the first 100 spheres
                   of rtow().
Floats are printed as plain decimals (the DSL has no exponents).
"""
from __future__ import annotations

import hashlib
import math
import os

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SCENES = os.path.join(ROOT, "scenes")


class _XorShift:
    def __init__(self, seed):
        self.s = seed & 0xFFFFFFFF

    def __call__(self):  # uniform in [0, 1)
        x = self.s
        x ^= (x << 13) & 0xFFFFFFFF
        x ^= x >> 17
        x ^= (x << 5) & 0xFFFFFFFF
        self.s = x
        return x / 4294967296.0


def _f(x: float) -> str:
    return f"{x:.6f}"


def read(name: str) -> str:
    with open(os.path.join(SCENES, name)) as fh:
        return fh.read()


def three_spheres() -> str:
    return (
        "camera origin 0.0 0.0 0.0 aspect 1.77778;\n\n"
        "material GROUND_MATERIAL : Diffuse color 0.8 0.8 0.0;\n"
        "material BALL_MATERIAL   : Diffuse color 0.7 0.3 0.3;\n"
        "material METAL_MATERIAL_1 : Metal color 0.8 0.8 0.8 fuzz 0.3;\n"
        "material GLASS  : Dielectric ir 1.5;\n\n"
        "sphere center  0.0 -100.5 -1.0  radius 100.0 material GROUND_MATERIAL;\n"
        "sphere center  0.0  0.0  -1.0  radius 0.5   material BALL_MATERIAL;\n"
        "sphere center -1.0  0.0  -1.0  radius 0.5   material METAL_MATERIAL_1;\n"
        "sphere center  1.0  0.0  -1.0  radius 0.5   material GLASS;\n"
    )


def _rtow_spheres(seed=0x2547549):
    """[(center, radius, material-line-body)] of the RTOW final scene."""
    rnd = _XorShift(seed)
    out = [((0.0, -1000.0, 0.0), 1000.0, "Diffuse color 0.5 0.5 0.5")]
    for a in range(-11, 11):
        for b in range(-11, 11):
            choose = rnd()
            c = (a + 0.9 * rnd(), 0.2, b + 0.9 * rnd())
            if math.dist(c, (4.0, 0.2, 0.0)) <= 0.9:
                continue
            if choose < 0.8:
                alb = [rnd() * rnd() for _ in range(3)]
                mat = "Diffuse color " + " ".join(_f(x) for x in alb)
            elif choose < 0.95:
                alb = [0.5 + 0.5 * rnd() for _ in range(3)]
                mat = ("Metal color " + " ".join(_f(x) for x in alb) +
                       " fuzz " + _f(0.5 * rnd()))
            else:
                mat = "Dielectric ir 1.5"
            out.append((c, 0.2, mat))
    out.append(((0.0, 1.0, 0.0), 1.0, "Dielectric ir 1.5"))
    out.append(((-4.0, 1.0, 0.0), 1.0, "Diffuse color 0.4 0.2 0.1"))
    out.append(((4.0, 1.0, 0.0), 1.0, "Metal color 0.7 0.6 0.5 fuzz 0.0"))
    return out


def _emit(camera, spheres, triangles=(), tri_materials=()):
    lines = [f"camera origin {' '.join(_f(x) for x in camera[0])} aspect {_f(camera[1])};", ""]
    for i, (_, _, m) in enumerate(spheres):
        lines.append(f"material S{i} : {m};")
    for name, m in tri_materials:
        lines.append(f"material {name} : {m};")
    lines.append("")
    for i, (c, r, _) in enumerate(spheres):
        lines.append(f"sphere center {' '.join(_f(x) for x in c)} radius {_f(r)} material S{i};")
    for (v0, v1, v2, name) in triangles:
        lines.append("triangle v0 " + " ".join(_f(x) for x in v0) + " v1 " +
                     " ".join(_f(x) for x in v1) + " v2 " + " ".join(_f(x) for x in v2) +
                     f" material {name};")
    return "\n".join(lines) + "\n"


RTOW_CAMERA = ((0.0, 2.0, 13.0), 1.77778)


def rtow(seed=0x2547549) -> str:
    """C2/C3 scene (BASELINE.json configs[1], [2])."""
    return _emit(RTOW_CAMERA, _rtow_spheres(seed))


def mesh(nx=250, ny=200, nspheres=100, seed=0x2547549) -> str:
    """C5 scene: nx*ny*2 triangles (100,000 by default) of a displaced grid
    spanning x in [-6, 6], y in [-1, 5], z in [-6, -3], plus the first
    `nspheres` spheres of the RTOW scene."""
    tri_mats = [("MESH_A", "Diffuse color 0.6 0.5 0.4"),
                ("MESH_B", "Metal color 0.8 0.8 0.9 fuzz 0.2")]
    pts = {}
    for j in range(ny + 1):
        for i in range(nx + 1):
            x = -6.0 + 12.0 * i / nx
            y = -1.0 + 6.0 * j / ny
            z = -4.5 + 1.2 * math.sin(0.9 * x) * math.cos(1.3 * y) + 0.3 * math.sin(3.1 * x + y)
            pts[i, j] = (x, y, z)
    tris = []
    for j in range(ny):
        for i in range(nx):
            m = "MESH_A" if (i // 10 + j // 10) % 2 == 0 else "MESH_B"
            a, b, c, d = pts[i, j], pts[i + 1, j], pts[i, j + 1], pts[i + 1, j + 1]
            tris.append((a, b, c, m))
            tris.append((c, b, d, m))
    return _emit(((0.0, 1.5, 3.0), 1.77778), _rtow_spheres(seed)[:nspheres], tris, tri_mats)


def triangle_soup(seed, n, spread=4.0, size=0.5, cam=(0.0, 0.0, 0.0), offset=(0.0, 0.0, 0.0),
                    slivers=0, dup=0, spheres=0, big=0, grid=0):
    """Random triangle soup (+ optional spheres) in the scene DSL.  Mixes
    sizes and orientations, near-degenerate slivers, exact duplicates (equal t:
    the lower index must win), huge triangles and a coplanar grid."""
    rng = np.random.default_rng(seed)
    kinds = ["Diffuse color 0.7 0.5 0.3", "Metal color 0.9 0.8 0.7 fuzz 0.05",
             "Dielectric ir 1.5", "Metal color 0.6 0.6 0.9 fuzz 0.0"]
    lines = [f"camera origin {cam[0]:.6f} {cam[1]:.6f} {cam[2]:.6f} aspect 1.5;"]
    lines += [f"material K{i} : {k};" for i, k in enumerate(kinds)]
    off = np.array(offset) + np.array([0.0, 0.0, -spread - 2.0])
    tris = []
    for _ in range(n):
        c = rng.uniform(-spread, spread, 3) + off
        e = rng.normal(size=(2, 3)) * size * rng.uniform(0.1, 1.0)
        tris.append((c, c + e[0], c + e[1], int(rng.integers(0, 4))))
    for _ in range(slivers):
        c = rng.uniform(-spread, spread, 3) + off
        d = rng.normal(size=3)
        tris.append((c, c + d, c + 2.0 * d + rng.normal(size=3) * 1e-4, int(rng.integers(0, 4))))
    for _ in range(big):
        c = rng.uniform(-spread, spread, 3) + off
        e = rng.normal(size=(2, 3)) * 40.0
        tris.append((c, c + e[0], c + e[1], int(rng.integers(0, 4))))
    for j in range(grid):
        for i in range(grid):
            x0, z0 = -3.0 + 6.0 * i / grid, -3.0 + 6.0 * j / grid
            dx = 6.0 / grid
            a = np.array([x0, -1.5, z0]) + off
            b, c2, d = a + [dx, 0, 0], a + [0, 0, dx], a + [dx, 0, dx]
            tris.append((a, c2, b, 0))
            tris.append((b, c2, d, 1))
    tris += tris[:dup]
    for _ in range(spheres):  # the parser takes spheres before triangles only
        c = rng.uniform(-spread, spread, 3) + off
        lines.append(f"sphere center {c[0]:.6f} {c[1]:.6f} {c[2]:.6f} radius "
                     f"{rng.uniform(0.1, 0.6):.6f} material K{int(rng.integers(0, 4))};")
    for (v0, v1, v2, k) in tris:
        lines.append("triangle v0 " + " ".join(f"{x:.6f}" for x in v0) + " v1 " +
                     " ".join(f"{x:.6f}" for x in v1) + " v2 " +
                     " ".join(f"{x:.6f}" for x in v2) + f" material K{k};")
    return "\n".join(lines) + "\n"


def sha256(text: str) -> str:
    return hashlib.sha256(text.encode()).hexdigest()


CONFIGS = {
    # name: (scene fn, width, height, spp, depth)   -- BASELINE.json configs
    "c1": (three_spheres, 256, 256, 1, 4),
    "c2": (rtow, 1920, 1080, 64, 8),
    "c3": (rtow, 3840, 2160, 256, 16),
    # C4 = the C3 frame row-tiled over the GPUs (bench.py --gpus 8 --config c4)
    "c4": (rtow, 3840, 2160, 256, 16),
    "c5": (mesh, 1920, 1080, 64, 8),
}


if __name__ == "__main__":
    os.makedirs(SCENES, exist_ok=True)
    with open(os.path.join(SCENES, "three_spheres.txt"), "w") as fh:
        fh.write(three_spheres())
    with open(os.path.join(SCENES, "rtow.txt"), "w") as fh:
        fh.write(rtow())
    m = mesh()
    with open(os.path.join(SCENES, "mesh_c5.sha256"), "w") as fh:
        fh.write(sha256(m) + "  mesh() of tools/scenes.py (not committed: ~%d bytes)\n" % len(m))
    print("rtow spheres:", rtow().count("sphere center"), "bytes", len(rtow()))
    print("mesh triangles:", m.count("triangle v0"), "bytes", len(m))
