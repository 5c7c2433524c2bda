import os, sys
sys.path.insert(0, "rust-swift-raytracer_amd"); sys.path.insert(0, "tools")
import raytracer_amd as R, scenes as S
make, W, H, spp, depth = S.CONFIGS["c2"]
w = R.World(make())
for ab in ["0", "1", "0", "1"]:
    os.environ["RT_AMD_ABLATE"] = ab
    for d in (1, 8):
        best = min((w.render(W, H, spp, d)[1] for _ in range(4)), key=lambda s: s["trace_ms"])
        print(dict(ablate=ab, depth=d, trace_ms=round(best["trace_ms"], 3), rays=best["rays"],
                   node=best["bvh_node_tests"], sph=best["bvh_sphere_tests"]), flush=True)
