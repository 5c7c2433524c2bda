"""C5 with per-origin-cell triangle trees (RT_AMD_TRI_CELLS) against the
static tree: load time, lean frame ms (interleaved, one process), triangle
node tests per ray, and the frames' bits (tuning tool, not product).
usage: python tools/c5_cells.py [cell sizes ...]"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "rust-swift-raytracer_amd"))
sys.path.insert(0, os.path.join(ROOT, "tools"))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import raytracer_amd as R  # noqa: E402
import scenes as S  # noqa: E402

make, W, H, spp, depth = S.CONFIGS["c5"]
src = make()
worlds = {}
for cs in ["off"] + sys.argv[1:]:
    # "edge[:sah]": the cell edge and the cell trees' SAH phantom scale
    os.environ.pop("RT_AMD_TRI_CELL_SAH", None)
    if cs == "off":
        os.environ["RT_AMD_TRI_CELLS"] = "0"
    else:
        edge, _, sah = cs.partition(":")
        os.environ["RT_AMD_TRI_CELLS"] = edge
        if sah:
            os.environ["RT_AMD_TRI_CELL_SAH"] = sah
    t = time.perf_counter()
    worlds[cs] = R.World(src)
    print(cs, "load %.1f s" % (time.perf_counter() - t), flush=True)
os.environ.pop("RT_AMD_TRI_CELLS", None)
os.environ.pop("RT_AMD_TRI_CELL_SAH", None)
torch.cuda.set_device(0)
out = torch.zeros(W * H * 4, dtype=torch.uint8, device="cuda")
stream = torch.cuda.current_stream()
ref = None
for cs, w in worlds.items():
    img, st = w.render(W, H, spp, depth)
    same = ref is None or bool(np.array_equal(img, ref))
    ref = img if ref is None else ref
    print(cs, "counted frame: trace %.1f ms, tri node tests/ray %.1f, tri tests/ray %.2f, rays %d, frame == static %s"
          % (st["trace_ms"], st["tri_node_tests"] / st["rays"], st["bvh_tri_tests"] / st["rays"], st["rays"], same),
          flush=True)
times = {cs: [] for cs in worlds}
for rnd in range(5):
    for cs, w in worlds.items():
        torch.cuda.synchronize()
        t = time.perf_counter()
        w.render_device(W, H, out.data_ptr(), stream.cuda_stream, spp=spp, depth=depth, device=0, stats=False)
        torch.cuda.synchronize()
        times[cs].append((time.perf_counter() - t) * 1e3)
for cs, v in times.items():
    print(cs, "lean frame ms median %.1f (all %s)" % (sorted(v)[len(v) // 2], " ".join("%.1f" % x for x in v)),
          flush=True)
