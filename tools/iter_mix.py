"""Iteration mix of the trace kernel (counting variant): loop iterations per
frame, how many walked the sphere tree, and the active lanes in each kind
(RT_AMD_ITER_DEBUG, printed by the library).  usage: python tools/iter_mix.py [config]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "rust-swift-raytracer_amd"), os.path.join(ROOT, "tools")]
os.environ["RT_AMD_ITER_DEBUG"] = "1"
import raytracer_amd as R  # noqa: E402
import scenes as S  # noqa: E402

cfg = sys.argv[1] if len(sys.argv) > 1 else "c2"
make, W, H, spp, depth = S.CONFIGS[cfg]
w = R.World(make())
w.render(W, H, spp, depth)
_, st = w.render(W, H, spp, depth)
print(cfg, "rays", st["rays"], "trace_ms %.3f" % st["trace_ms"], flush=True)
