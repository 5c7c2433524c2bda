"""One rank's share of a multi-GPU frame on one GPU: renders rank 0's row tile
of config C for N ranks (row blocks of 8, as bench.py) and prints median
trace/frame ms per variant (library / env), interleaved in one process like
tools/ab.py.  Used to size chunks for the small per-rank frames of N = 2..8.

  python tools/rank_probe.py --n 8 --variant cur=rust-swift-raytracer_amd/lib/libraytracer.so \
      --variant p2=rust-swift-raytracer_amd/lib/libraytracer.so:RT_AMD_RESOLVE_PIX=2
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
    ap.add_argument("--n", type=int, default=8)
    ap.add_argument("--rounds", type=int, default=9)
    ap.add_argument("--depth", type=int, default=0, help="override the config's depth")
    ap.add_argument("--rank", type=int, default=0)
    args = ap.parse_args()
    make_scene, W, H, spp, depth = S.CONFIGS[args.config]
    depth = args.depth or depth
    src = make_scene()
    torch.cuda.set_device(0)
    rows = R.tile_rows(H, 8, args.rank, args.n)
    out = torch.zeros(rows * W * 4, dtype=torch.uint8, device="cuda")
    stream = torch.cuda.current_stream()
    variants = []
    for v in args.variant:
        label, rest = v.split("=", 1)
        parts = rest.split(":")
        path = parts[0] if os.path.isabs(parts[0]) else os.path.join(ROOT, parts[0])
        env = dict(kv.split("=", 1) for kv in parts[1:])
        variants.append((label, R.World(src, lib_path=path), env))
    res = {label: {"trace": [], "frame": []} for label, _, _ in variants}
    for rnd in range(args.rounds + 1):
        for label, world, env in variants:
            saved = {k: os.environ.get(k) for k in env}
            os.environ.update(env)
            kw = dict(spp=spp, depth=depth, row_block=8, rank=args.rank, nranks=args.n, device=0)
            world.render_device(W, H, out.data_ptr(), stream.cuda_stream, **kw)  # counters
            torch.cuda.synchronize()
            t = time.perf_counter()
            for _ in range(5):
                world.render_device(W, H, out.data_ptr(), stream.cuda_stream, stats=False, **kw)
            torch.cuda.synchronize()
            dt = (time.perf_counter() - t) * 1e3 / 5
            st = world.render_device(W, H, out.data_ptr(), stream.cuda_stream, **kw)
            for k, v in saved.items():
                if v is None:
                    os.environ.pop(k, None)
                else:
                    os.environ[k] = v
            if rnd:
                res[label]["trace"].append(st["trace_ms"])
                res[label]["frame"].append(dt)
    for label, r in res.items():
        print(json.dumps({"variant": label, "config": args.config, "n": args.n, "rows": rows,
                          "depth": depth, "rank": args.rank,
                          "trace_ms_median": statistics.median(r["trace"]),
                          "frame_ms_median": statistics.median(r["frame"])}))


if __name__ == "__main__":
    main()
