"""SERIAL knob sweep in one process (A/B): RT_AMD_SERIAL_RUN (chain-mode run
length, 1 = every candidate traced) x RT_AMD_SERIAL_CHUNK (L) on the frames of
CASES (tools/serial_probe.py syntax).  Each setting renders twice and keeps
the faster; every frame is checked against the first setting's bits."""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "rust-swift-raytracer_amd"), os.path.join(ROOT, "tools")]
import raytracer_amd as R  # noqa: E402
from serial_probe import _cases  # noqa: E402

RUNS = [int(v) for v in os.environ.get("RUNS", "1,16,64").split(",")]
CHUNKS = [int(v) for v in os.environ.get("CHUNKS", "16384,65536").split(",")]
for name, s, w, h, spp, depth in _cases():
    world = R.World(s)
    world.render(w, h, spp, depth)
    ref = None
    for chunk in CHUNKS:
        for run in RUNS:
            os.environ["RT_AMD_SERIAL_RUN"] = str(run)
            os.environ["RT_AMD_SERIAL_CHUNK"] = str(chunk)
            best = None
            for _ in range(2):
                t = time.perf_counter()
                out, st = world.render(w, h, spp, depth, mode=R.RNG_SERIAL)
                dt = time.perf_counter() - t
                best = dt if best is None else min(best, dt)
            if ref is None:
                ref = out
            same = np.array_equal(out, ref)
            print(f"{name} {w}x{h}x{spp}/{depth} L={chunk} run={run}: {best * 1e3:.1f} ms, "
                  f"states {st['serial_ms']:.1f} ms, {st['serial_iterations']} iterations "
                  f"({st['serial_retries']} short), same={same}", flush=True)
