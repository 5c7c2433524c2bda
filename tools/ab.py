"""Interleaved A/B timing of library builds and env settings in ONE process
(cdna_hip_programming.md §5.4 rule 24: separate invocations add variance).

  python tools/ab.py --variant cur=rust-swift-raytracer_amd/lib/libraytracer.so \
                     --variant prev=ab/prev/libraytracer.so \
                     --variant nolds=rust-swift-raytracer_amd/lib/libraytracer.so:RT_AMD_LDS=0 \
                     [--config c2] [--rounds 7] [--spp N]

Prints one JSON line per variant: median / min trace-kernel ms and frame ms.
"""
import argparse
import json
import os
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "rust-swift-raytracer_amd"))
sys.path.insert(0, os.path.join(ROOT, "tools"))

import torch  # noqa: E402

import raytracer_amd as R  # noqa: E402
import scenes as S  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--variant", action="append", required=True)
    ap.add_argument("--config", default="c2")
    ap.add_argument("--rounds", type=int, default=7)
    ap.add_argument("--spp", type=int, default=0)
    ap.add_argument("--accel", default="auto", choices=["auto", "brute", "bvh"])
    args = ap.parse_args()
    make_scene, W, H, spp, depth = S.CONFIGS[args.config]
    spp = args.spp or spp
    accel = {"auto": R.ACCEL_AUTO, "brute": R.ACCEL_BRUTE, "bvh": R.ACCEL_BVH}[args.accel]
    src = make_scene()
    torch.cuda.set_device(0)
    out = torch.zeros(W * H * 4, dtype=torch.uint8, device="cuda")
    stream = torch.cuda.current_stream()
    variants = []
    for v in args.variant:
        label, rest = v.split("=", 1)
        parts = rest.split(":")
        path = os.path.join(ROOT, parts[0]) if not os.path.isabs(parts[0]) else parts[0]
        env = dict(kv.split("=", 1) for kv in parts[1:])
        saved = {k: os.environ.get(k) for k in env}
        os.environ.update(env)  # load-time knobs (e.g. RT_AMD_LEAF) too
        variants.append((label, R.World(src, lib_path=path), env))
        for k, v in saved.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v
    res = {label: {"trace": [], "frame": [], "lean": [], "rays": 0} for label, _, _ in variants}
    for rnd in range(args.rounds + 1):
        for label, world, env in variants:
            saved = {k: os.environ.get(k) for k in env}
            os.environ.update(env)
            torch.cuda.synchronize()
            t = time.perf_counter()
            st = world.render_device(W, H, out.data_ptr(), stream.cuda_stream, spp=spp,
                                     depth=depth, device=0, accel=accel)
            torch.cuda.synchronize()
            dt = (time.perf_counter() - t) * 1e3
            # frames without stats (the bench's timed path: counters compiled out)
            t = time.perf_counter()
            for _ in range(3):
                world.render_device(W, H, out.data_ptr(), stream.cuda_stream, spp=spp, depth=depth,
                                    device=0, accel=accel, stats=False)
            torch.cuda.synchronize()
            lean = (time.perf_counter() - t) * 1e3 / 3
            for k, v in saved.items():
                if v is None:
                    os.environ.pop(k, None)
                else:
                    os.environ[k] = v
            if rnd == 0:
                continue  # warm-up round
            res[label]["trace"].append(st["trace_ms"])
            res[label]["frame"].append(dt)
            res[label]["lean"].append(lean)
            res[label]["rays"] = st["rays"]
    for label, r in res.items():
        print(json.dumps({"variant": label, "config": args.config, "spp": spp,
                          "trace_ms_median": statistics.median(r["trace"]),
                          "trace_ms_min": min(r["trace"]),
                          "frame_ms_median": statistics.median(r["frame"]),
                          "lean_frame_ms_median": statistics.median(r["lean"]),
                          "grays_per_s": r["rays"] / statistics.median(r["frame"]) / 1e6,
                          "rays": r["rays"]}))


if __name__ == "__main__":
    main()
