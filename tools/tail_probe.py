"""Per-wave timeline of one rank's tile (diagnostic): renders rank 0's row tile
of config C for N ranks with a -DRT_WAVE_TIMES build (ab/wt/libraytracer.so),
dumps the per-wave records (RT_AMD_WAVE_DUMP) and prints when waves pulled
their last chunk, found the queue empty and exited, on the 100 MHz clock.

  make -C rust-swift-raytracer_amd OBJ=../ab/wt/build LIB=../ab/wt/lib \
      DEFS=-DRT_WAVE_TIMES=1 ../ab/wt/lib/libraytracer.so
  python tools/tail_probe.py --n 8 [--env KEY=VALUE ...]
"""
import argparse
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "rust-swift-raytracer_amd"))
sys.path.insert(0, os.path.join(ROOT, "tools"))
import torch  # noqa: E402

import raytracer_amd as R  # noqa: E402
import scenes as S  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="c2")
    ap.add_argument("--n", type=int, default=8)
    ap.add_argument("--lib", default=os.path.join(ROOT, "ab", "wt", "lib", "libraytracer.so"))
    ap.add_argument("--env", action="append", default=[])
    ap.add_argument("--out", default=os.path.join(ROOT, "gpurun_out", "waves.bin"))
    args = ap.parse_args()
    for kv in args.env:
        k, v = kv.split("=", 1)
        os.environ[k] = v
    make_scene, W, H, spp, depth = S.CONFIGS[args.config]
    torch.cuda.set_device(0)
    rows = R.tile_rows(H, 8, 0, args.n)
    out = torch.zeros(rows * W * 4, dtype=torch.uint8, device="cuda")
    stream = torch.cuda.current_stream()
    world = R.World(make_scene(), lib_path=args.lib)
    kw = dict(spp=spp, depth=depth, row_block=8, rank=0, nranks=args.n, device=0)
    for _ in range(3):
        world.render_device(W, H, out.data_ptr(), stream.cuda_stream, **kw)
    os.environ["RT_AMD_WAVE_DUMP"] = args.out
    st = world.render_device(W, H, out.data_ptr(), stream.cuda_stream, **kw)
    torch.cuda.synchronize()
    del os.environ["RT_AMD_WAVE_DUMP"]
    rec = np.fromfile(args.out, dtype=np.uint64).reshape(-1, 16)
    rec = rec[rec[:, 4] != 0]
    t0 = rec[:, 4].min()
    us = lambda x: (x.astype(np.float64) - t0) / 100.0  # 100 MHz -> us
    start, pull, exh, end = us(rec[:, 4]), us(rec[:, 5]), us(rec[:, 6]), us(rec[:, 7])
    q = lambda a: [round(float(np.percentile(a, p)), 1) for p in (0, 10, 50, 90, 99, 100)]
    print(json.dumps({
        "config": args.config, "n": args.n, "rows": rows, "waves": int(len(rec)),
        "trace_ms": st["trace_ms"], "env": args.env,
        "start_us_pcts": q(start), "last_pull_us_pcts": q(pull), "exhausted_us_pcts": q(exh),
        "end_us_pcts": q(end), "end_minus_pull_us_pcts": q(end - pull),
        "tail_chunk_jobs_pcts": q(rec[:, 14].astype(np.float64)),
        "rays": st["rays"],
    }))


if __name__ == "__main__":
    main()
