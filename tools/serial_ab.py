"""Interleaved A/B of RT_RNG_SERIAL frames (render()'s reference-identical
mode) across library builds / env settings in ONE process.

  python tools/serial_ab.py --variant cur=rust-swift-raytracer_amd/lib/libraytracer.so \
      --variant prev=ab/prev/libraytracer.so[:ENV=V...][:ACCEL=bvh] [--cases world:960x540x16/8,...] [--rounds 3]

Prints one JSON line per (variant, case): median wall ms of the SERIAL frame,
the start-state search ms, iterations and iterations stopped short, and
whether the frame's bytes equal the first variant's.
"""
import argparse
import json
import os
import statistics
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


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--variant", action="append", required=True)
    ap.add_argument("--cases", default="world:960x540x16/8,rtow:1920x1080x64/8")
    ap.add_argument("--rounds", type=int, default=3)
    args = ap.parse_args()
    cases = []
    for item in args.cases.split(","):
        name, geo = item.split(":")
        dims, depth = geo.split("/")
        w, h, spp = (int(v) for v in dims.split("x"))
        cases.append((name, w, h, spp, int(depth)))
    variants = []
    for v in args.variant:
        label, rest = v.split("=", 1)
        parts = rest.split(":")
        path = parts[0] if os.path.isabs(parts[0]) else os.path.join(ROOT, parts[0])
        env = dict(kv.split("=", 1) for kv in parts[1:])
        # ACCEL=brute|bvh|auto: the frame's RtRenderOptions.accel, not an env setting
        accel = {"auto": R.ACCEL_AUTO, "brute": R.ACCEL_BRUTE, "bvh": R.ACCEL_BVH}[env.pop("ACCEL", "auto")]
        variants.append((label, path, env, accel))
    worlds = {}
    for label, path, env, _ in variants:
        for name, *_ in cases:
            worlds[(label, name)] = R.World(_scene(name), lib_path=path)
    res = {}
    ref = {}
    for rnd in range(args.rounds + 1):
        for name, w, h, spp, depth in cases:
            for label, path, env, accel in variants:
                saved = {k: os.environ.get(k) for k in env}
                os.environ.update(env)
                world = worlds[(label, name)]
                t = time.perf_counter()
                img, st = world.render(w, h, spp, depth, mode=R.RNG_SERIAL, accel=accel)
                wall = (time.perf_counter() - t) * 1e3
                for k, v in saved.items():
                    if v is None:
                        os.environ.pop(k, None)
                    else:
                        os.environ[k] = v
                case = f"{name}:{w}x{h}x{spp}/{depth}"
                if rnd == 0:
                    ref.setdefault(case, img)
                    res[(label, case)] = {"same": bool((img == ref[case]).all()), "wall": [], "search": [],
                                          "it": st["serial_iterations"], "short": st["serial_retries"]}
                    continue
                r = res[(label, case)]
                r["wall"].append(wall)
                r["search"].append(st["serial_ms"])
                r["same"] = r["same"] and bool((img == ref[case]).all())
    for (label, case), r in res.items():
        print(json.dumps({"variant": label, "case": case, "wall_ms_median": statistics.median(r["wall"]),
                          "search_ms_median": statistics.median(r["search"]), "iterations": r["it"],
                          "stopped_short": r["short"], "frame_equal_to_first_variant": r["same"]}), flush=True)


if __name__ == "__main__":
    main()
