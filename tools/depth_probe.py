"""Per-bounce cost probe: renders a config at depth 1..D and prints the
incremental trace time and BVH work of each extra bounce (diagnostic)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "rust-swift-raytracer_amd"))
sys.path.insert(0, os.path.join(ROOT, "tools"))
import raytracer_amd as R  # noqa: E402
import scenes as S  # noqa: E402

cfg = sys.argv[1] if len(sys.argv) > 1 else "c2"
make, W, H, spp, depth = S.CONFIGS[cfg]
w = R.World(make())
prev = None
for d in range(1, depth + 1):
    w.render(W, H, spp, d)
    best = None
    for _ in range(3):
        _, st = w.render(W, H, spp, d)
        best = st if best is None or st["trace_ms"] < best["trace_ms"] else best
    st = best
    row = dict(depth=d, trace_ms=round(st["trace_ms"], 3), rays=st["rays"],
               node=st["bvh_node_tests"], sph=st["bvh_sphere_tests"],
               tnode=st["tri_node_tests"], tri=st["bvh_tri_tests"])
    if prev:
        dr = row["rays"] - prev["rays"]
        row["d_ms"] = round(row["trace_ms"] - prev["trace_ms"], 3)
        row["d_rays"] = dr
        row["d_node_per_ray"] = round((row["node"] - prev["node"]) / max(dr, 1), 2)
        row["d_tnode_per_ray"] = round((row["tnode"] - prev["tnode"]) / max(dr, 1), 2)
    else:
        row["node_per_ray"] = round(row["node"] / row["rays"], 2)
        row["tnode_per_ray"] = round(row["tnode"] / row["rays"], 2)
    print(row, flush=True)
    prev = row
