"""Times RT_RNG_SERIAL (render()'s reference-identical mode) on the
examples/c_raytracer.rs world, C1 and RTOW; run under rocprofv3 for per-kernel
times.  CASES="name:WxHxspp/depth,..." picks frames (names: c_raytracer, c1,
rtow, world); default: the round-1 sizes."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "rust-swift-raytracer_amd"), os.path.join(ROOT, "tools")]
import raytracer_amd as R  # noqa: E402
import scenes as S  # noqa: E402


def _scene(name):
    if name == "c1":
        return S.three_spheres()
    if name == "rtow":
        return S.rtow()
    fn = {"c_raytracer": "c_raytracer_world.txt", "world": "world.txt"}[name]
    with open(os.path.join(ROOT, "scenes", fn)) as fh:
        return fh.read()


def _cases():
    spec = os.environ.get("CASES", "c_raytracer:200x200x16/8,c1:256x256x1/4,rtow:320x180x16/8")
    for item in spec.split(","):
        name, geo = item.split(":")
        dims, depth = geo.split("/")
        w, h, spp = (int(v) for v in dims.split("x"))
        yield name, _scene(name), w, h, spp, int(depth)


def main():
    for name, s, w, h, spp, depth in _cases():
        world = R.World(s)
        world.render(w, h, spp, depth)  # device init
        for k in range(int(os.environ.get("REPS", "2"))):
            t = time.perf_counter()
            _, st = world.render(w, h, spp, depth, mode=R.RNG_SERIAL)
            dt = time.perf_counter() - t
            n = w * h * spp
            print(f"{name} {w}x{h}x{spp}/{depth}: call {dt * 1e3:.1f} ms, states {st['serial_ms']:.1f} ms, "
                  f"replay {st['trace_ms']:.2f} ms, retries {st['serial_retries']}, "
                  f"{st['rays'] / dt / 1e6:.1f} Mrays/s, {n / dt / 1e6:.1f} Msamples/s", flush=True)


if __name__ == "__main__":
    main()
