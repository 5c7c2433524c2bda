"""Per-stage cost of a C2 frame from timing-only ablations (RT_AMD_ABLATE bits:
1 = skip the tree walk, 2 = skip the fused resolve, 4 = no primary-list load)
at depth 1 and 8.  Counting-variant frames (stats=True), best of 4.

  python tools/probe_walk0.py [ablate ...]      (default: 0 1 2 4)
"""
import os
import sys

sys.path.insert(0, "rust-swift-raytracer_amd")
sys.path.insert(0, "tools")
import raytracer_amd as R  # noqa: E402
import scenes as S  # noqa: E402

make, W, H, spp, depth = S.CONFIGS["c2"]
w = R.World(make())
for ab in (sys.argv[1:] or ["0", "1", "2", "4"]):
    os.environ["RT_AMD_ABLATE"] = ab
    for d in (1, 8):
        best = min((w.render(W, H, spp, d)[1] for _ in range(4)), key=lambda s: s["trace_ms"])
        print(dict(ablate=ab, depth=d, trace_ms=round(best["trace_ms"], 3), rays=best["rays"],
                   node=best["bvh_node_tests"], sph=best["bvh_sphere_tests"]), flush=True)
