"""Row-tiled multi-GPU frames: partition, RCCL gather and reassembly.

One process per GPU.  Image rows are dealt in blocks of `block` rows,
round-robin over ranks (rank g owns image rows r with (r // block) % n == g),
so cheap sky rows and expensive ground rows spread evenly.  Each rank renders
its tile with rt_render_device (full width, only its rows), the tiles are
all-gathered with torch.distributed (backend "nccl" = RCCL over xGMI on
MI355X, "gloo" in CPU tests) and every rank can rebuild the frame.  Tiles are
padded to the largest tile so the collective moves equal-size buffers.
The reference has no counterpart: its ray_trace is single-threaded
(common.rs:327-358).
"""
from __future__ import annotations

import numpy as np

import raytracer_amd as R


def max_tile_rows(height: int, block: int, nranks: int) -> int:
    return max(R.tile_rows(height, block, r, nranks) for r in range(nranks))


def row_map(height: int, block: int, nranks: int):
    """[(rank, k, image_row)] for every image row."""
    out = []
    for r in range(nranks):
        for k in range(R.tile_rows(height, block, r, nranks)):
            out.append((r, k, R.tile_row(k, block, r, nranks)))
    return out


def assemble(gathered, width: int, height: int, block: int, nranks: int) -> np.ndarray:
    """gathered: [nranks * max_rows * width * 4] uint8 (all-gather output)."""
    g = np.asarray(gathered).reshape(nranks, -1, width, 4)
    img = np.zeros((height, width, 4), np.uint8)
    for r, k, row in row_map(height, block, nranks):
        img[row] = g[r, k]
    return img


def gather(tile, gathered, group=None):
    """All-gather equal-size tiles (torch tensors) over the process group."""
    import torch.distributed as dist

    dist.all_gather_into_tensor(gathered, tile, group=group)
    return gathered


def gather_any(tile, nranks, group=None):
    """Backend-agnostic all-gather (gloo lacks all_gather_into_tensor on CPU)."""
    import torch
    import torch.distributed as dist

    if dist.get_backend(group) == "nccl":
        out = torch.empty(nranks * tile.numel(), dtype=tile.dtype, device=tile.device)
        dist.all_gather_into_tensor(out, tile, group=group)
        return out
    parts = [torch.empty_like(tile) for _ in range(nranks)]
    dist.all_gather(parts, tile, group=group)
    return torch.cat(parts)
