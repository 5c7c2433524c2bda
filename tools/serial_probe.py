"""Times RT_RNG_SERIAL on the examples/c_raytracer.rs frame (render()'s
200x200, 16 spp, depth 8) and C1; run under rocprofv3 for per-kernel times."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "rust-swift-raytracer_amd"), os.path.join(ROOT, "tools")]
import raytracer_amd as R  # noqa: E402
import scenes as S  # noqa: E402

with open(os.path.join(ROOT, "scenes", "c_raytracer_world.txt")) as fh:
    src = fh.read()
cases = [("c_raytracer", src, 200, 200, 16, 8), ("c1", S.three_spheres(), 256, 256, 1, 4),
         ("rtow", S.rtow(), 320, 180, 16, 8)]
for name, s, w, h, spp, depth in cases:
    world = R.World(s)
    world.render(w, h, spp, depth)  # device init
    for k in range(int(os.environ.get("REPS", "2"))):
        t = time.perf_counter()
        _, st = world.render(w, h, spp, depth, mode=R.RNG_SERIAL)
        dt = time.perf_counter() - t
        print(f"{name} {w}x{h}x{spp}/{depth}: call {dt * 1e3:.1f} ms, states {st['serial_ms']:.1f} ms, "
              f"replay {st['trace_ms']:.2f} ms, retries {st['serial_retries']}", flush=True)
