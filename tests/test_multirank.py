"""World-size-2/3 CPU (gloo) tests of the multi-GPU tile path: partition,
all-gather and reassembly (rust-swift-raytracer_amd/tiles.py, used by
bench.py).  The per-rank renderer is the oracle in COUNTER mode: each rank
traces only the image rows the product's row map (rt_tile_row) gives it --
frames are independent of how rows are partitioned, so the assembled frame
must equal the single-process frame bit-for-bit."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

import oracle as O
import raytracer_amd as R
import tiles
from conftest import scene_text

W, H, SPP, DEPTH = 40, 30, 2, 8


def free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, nranks, block, port, q):
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank,
                            world_size=nranks)
    scene = O.Scene(scene_text("c_raytracer_world.txt"))
    rows = R.tile_rows(H, block, rank, nranks)
    mr = tiles.max_tile_rows(H, block, nranks)
    tile = np.zeros((mr, W, 4), np.uint8)
    mine = np.zeros((H, W, 4), np.uint8)
    for k in range(rows):
        # image row r (top = 0) is the reference's row H - 1 - r (common.rs:327-331):
        # render that row alone (row_step = H), into this rank's buffer
        r = R.tile_row(k, block, rank, nranks)
        scene.render(W, H, SPP, DEPTH, mode=O.RNG_COUNTER, row_begin=H - 1 - r, row_step=H, out=mine)
        tile[k] = mine[r]
    rendered = int(np.count_nonzero(mine.reshape(H, -1).any(axis=1)))
    g = tiles.gather_any(torch.from_numpy(tile.reshape(-1)), nranks)
    img = tiles.assemble(g.numpy(), W, H, block, nranks)
    full, _, _ = scene.render(W, H, SPP, DEPTH, mode=O.RNG_COUNTER)
    q.put((rank, bool(np.array_equal(img, full)) and rendered == rows))
    dist.destroy_process_group()


@pytest.mark.parametrize("nranks,block", [(2, 1), (2, 8), (3, 4)])
def test_gloo_tiles_reassemble(nranks, block):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = free_port()
    procs = [ctx.Process(target=_worker, args=(r, nranks, block, port, q)) for r in range(nranks)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=120) for _ in range(nranks))
    for p in procs:
        p.join(timeout=60)
    assert all(res.values()), res


@pytest.mark.parametrize("height,block,nranks", [(1080, 8, 8), (2160, 8, 8), (1080, 8, 3),
                                                 (7, 2, 4), (5, 8, 8), (1, 1, 2)])
def test_partition_covers_every_row_once(height, block, nranks):
    rows = sorted(row for _, _, row in tiles.row_map(height, block, nranks))
    assert rows == list(range(height))
    sizes = [R.tile_rows(height, block, r, nranks) for r in range(nranks)]
    assert sum(sizes) == height and max(sizes) - min(sizes) <= block
