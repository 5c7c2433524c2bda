"""Generates the committed golden fixtures in tests/golden/.

The reference (Rust) cannot be built or run in this pipeline (no cargo/rustc),
so every vector here comes from the C++ oracle and is cross-checked, where the
size allows, bit-for-bit against the independent numpy restatement
(tests/pyref.py) before it is written.  Fixtures are data only: inputs and
expected outputs (bit patterns as uint32 for floats).

usage: python tools/make_golden.py
"""
import hashlib
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in ("oracle", "tests", "tools"):
    sys.path.insert(0, os.path.join(ROOT, p))

import oracle as O  # noqa: E402
import pyref as P  # noqa: E402
import scenes as S  # noqa: E402

GOLD = os.path.join(ROOT, "tests", "golden")


def bits(x):
    return int(np.array(x, np.float32).view(np.uint32))


def scene(name):
    return open(os.path.join(ROOT, "scenes", name)).read()


# (name, scene text, W, H, spp, depth, mode, seed, check with pyref)
FRAMES = [
    ("c1_three_spheres_256x256x1x4_serial", S.three_spheres(), 256, 256, 1, 4, O.RNG_SERIAL, 2547549, False),
    ("c_raytracer_200x200x16x8_serial", scene("c_raytracer_world.txt"), 200, 200, 16, 8, O.RNG_SERIAL, 2547549, False),
    ("world_48x27x4x8_serial", scene("world.txt"), 48, 27, 4, 8, O.RNG_SERIAL, 2547549, True),
    ("c_raytracer_24x18x3x8_serial", scene("c_raytracer_world.txt"), 24, 18, 3, 8, O.RNG_SERIAL, 2547549, True),
    ("rtow_64x36x2x8_counter", S.rtow(), 64, 36, 2, 8, O.RNG_COUNTER, 2547549, False),
    ("c_raytracer_1x5x2x8_serial", scene("c_raytracer_world.txt"), 1, 5, 2, 8, O.RNG_SERIAL, 2547549, True),
]


def main():
    os.makedirs(GOLD, exist_ok=True)
    # ---- RNG stream (random.rs:8-30) and counter seeds
    rng = {"seed": 2547549, "xorshift32": O.xorshift_stream(2547549, 32),
           "random_f32_bits": [bits(x) for x in O.random_f32_stream(2547549, 32)],
           "counter_seed": {str(j): O.sample_seed(2547549, j)
                            for j in (0, 1, 2, 63, 64, 12345, 2**32 + 7, 132710399)}}
    pr = P.Random()
    assert [pr.xor_shift_32() for _ in range(32)] == rng["xorshift32"]
    json.dump(rng, open(os.path.join(GOLD, "rng.json"), "w"), indent=1)

    # ---- frames
    meta = {}
    arrays = {}
    for (name, src, w, h, spp, depth, mode, seed, check) in FRAMES:
        img, st, states, smp = O.Scene(src).render(w, h, spp, depth, mode=mode, seed=seed,
                                                   nthreads=1, record_states=True,
                                                   record_samples=True)
        if check:
            cam, world = P.parse(src)
            ps = np.zeros_like(smp)
            a = P.ray_trace(world, cam, w, h, spp, depth, seed=seed, samples=ps)
            assert np.array_equal(a, img), name
            assert np.array_equal(ps.view(np.uint32), smp.view(np.uint32)), name
        arrays[name] = img
        meta[name] = {"width": w, "height": h, "spp": spp, "depth": depth, "mode": int(mode),
                      "seed": seed, "stats": st, "pyref_checked": check,
                      "rgba_sha256": hashlib.sha256(img.tobytes()).hexdigest(),
                      "sample_states_sha256": hashlib.sha256(states.tobytes()).hexdigest(),
                      "sample_bits_sha256": hashlib.sha256(smp.view(np.uint32).tobytes()).hexdigest()}
    np.savez_compressed(os.path.join(GOLD, "frames.npz"), **arrays)
    json.dump(meta, open(os.path.join(GOLD, "frames.json"), "w"), indent=1)
    print("wrote", sorted(os.listdir(GOLD)))


if __name__ == "__main__":
    main()
