"""Segment shares of the trace kernel from a -DRT_STAMPS diagnostic build
(ab/stamps/libraytracer.so): wave cycles per loop segment.  Read the SHARES,
never the run time (stamps fence the schedule).  The library prints the 8 fine
segments to stderr ("stamp segments: ..."): 0 direction normalisation + loop
back, 1 ray setup, 2 walks, 3 shading, 4 sample store, 5 fused resolve,
6 refill, 7 unused.
usage: python tools/stamps.py [config] [lib]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "rust-swift-raytracer_amd"))
sys.path.insert(0, os.path.join(ROOT, "tools"))
import raytracer_amd as R  # noqa: E402
import scenes as S  # noqa: E402

cfg = sys.argv[1] if len(sys.argv) > 1 else "c2"
path = sys.argv[2] if len(sys.argv) > 2 else os.path.join(ROOT, "ab", "stamps", "libraytracer.so")
make, W, H, spp, depth = S.CONFIGS[cfg]
w = R.World(make(), lib_path=path)
w.render(W, H, spp, depth)
_, st = w.render(W, H, spp, depth)
c = st["stamp_cycles"]
tot = sum(c)
print(cfg, "trace_ms %.3f" % st["trace_ms"], "coarse shares:",
      " ".join(f"{n}={x / tot:.3f}" for n, x in zip(["refill+store+resolve+loop", "setup", "walks", "shade"], c)),
      "cycles/ray %.0f" % (tot / st["rays"]), "(fine segments on stderr: renorm setup walks shade store "
      "resolve refill -)", flush=True)
