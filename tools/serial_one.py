"""One SERIAL render() frame per case, for rocprofv3 passes over the
start-state search's kernels (tuning tool, not product).
usage: python tools/serial_one.py world:960x540x16 [rtow:1920x1080x64 ...]"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "rust-swift-raytracer_amd"))
sys.path.insert(0, os.path.join(ROOT, "tools"))
import raytracer_amd as R  # noqa: E402
import scenes as S  # noqa: E402

for case in sys.argv[1:]:
    sc, dims = case.split(":")
    W, H, spp = (int(x) for x in dims.split("x"))
    w = R.World(S.read("world.txt") if sc == "world" else S.read("c_raytracer_world.txt") if sc == "c_raytracer" else S.rtow(),
                lib_path=os.environ.get("RT_LIB") or None)
    t = time.perf_counter()
    _, st = w.render(W, H, spp, 8, mode=R.RNG_SERIAL)
    print(case, "wall %.1f ms" % ((time.perf_counter() - t) * 1e3), "search %.1f ms" % st["serial_ms"],
          "iterations", st["serial_iterations"], "stopped", st["serial_retries"], "rays", st["rays"], flush=True)
    w.close()
