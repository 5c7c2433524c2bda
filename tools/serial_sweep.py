"""SERIAL knob sweep in one process (A/B) on the frames of CASES
(tools/serial_probe.py syntax).  SWEEP="VAR=a,b;VAR2=c,d" gives the grid of
environment settings (default: RT_AMD_SERIAL_RUN, the chain-mode run length,
x RT_AMD_SERIAL_CHUNK, the iteration length L; 0 = the library default).
Each setting renders twice and keeps the faster; every frame is checked
against the first setting's bits."""
import itertools
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "rust-swift-raytracer_amd"), os.path.join(ROOT, "tools")]
import raytracer_amd as R  # noqa: E402
from serial_probe import _cases  # noqa: E402


def _grid():
    spec = os.environ.get("SWEEP", "RT_AMD_SERIAL_RUN=1,4,16;RT_AMD_SERIAL_CHUNK=16384,65536")
    axes = []
    for part in spec.split(";"):
        var, vals = part.split("=")
        axes.append([(var, v) for v in vals.split(",")])
    return list(itertools.product(*axes))


def main():
    grid = _grid()
    for name, s, w, h, spp, depth in _cases():
        world = R.World(s)
        world.render(w, h, spp, depth)
        ref = None
        for setting in grid:
            for var, v in setting:
                if v == "0":
                    os.environ.pop(var, None)
                else:
                    os.environ[var] = v
            best = None
            for _ in range(2):
                t = time.perf_counter()
                out, st = world.render(w, h, spp, depth, mode=R.RNG_SERIAL)
                dt = time.perf_counter() - t
                best = dt if best is None else min(best, dt)
            if ref is None:
                ref = out
            label = " ".join(f"{var.replace('RT_AMD_SERIAL_', '')}={v}" for var, v in setting)
            print(f"{name} {w}x{h}x{spp}/{depth} {label}: {best * 1e3:.1f} ms, "
                  f"states {st['serial_ms']:.1f} ms, {st['serial_iterations']} iterations "
                  f"({st['serial_retries']} short), same={np.array_equal(out, ref)}", flush=True)
        for var, _ in grid[0]:
            os.environ.pop(var, None)


if __name__ == "__main__":
    main()
