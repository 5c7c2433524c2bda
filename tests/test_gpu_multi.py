"""GPU tests of the multi-GPU paths.

The reference renders serially (common.rs:327-358); the north star row-tiles
the frame over the node's GPUs and gathers the tiles over RCCL.  Two launch
shapes exist and both are exercised here on the one GPU a test box has:
  * one process, N devices (RtRenderOptions.ndevices): tiles + RCCL ncclGather
    (ncclCommInitAll communicator) + assemble kernel, through the C-ABI.  With
    one device the gather is a copy into the frame.  Bit-identical to the
    single-device frame, through rt_render_ex, rt_render_device and render()
    (RT_AMD_DEVICES);
  * one process per GPU (torch.distributed.run, the driver's N>1 launch):
    rehearsed with two ranks sharing device 0 and gloo collectives, HIP tiles,
    the gathered frame checked against a one-rank render (RT_BENCH_VERIFY).
Plus `python bench.py --gpus 1`, which runs the single-process path.
"""
import json
import os
import socket
import subprocess
import sys

import numpy as np
import pytest

import oracle as O
import raytracer_amd as R
from conftest import ROOT, scene_text
from test_gpu_parity import assert_bits_equal

pytestmark = pytest.mark.gpu


def test_comm_count_one_device():
    assert R.comm_count(0, 1) == 1
    with pytest.raises(R.RenderError, match="not all visible"):
        R.comm_count(0, R.device_count() + 1)


@pytest.mark.parametrize("scene,w,h,spp", [("rtow.txt", 160, 90, 4), ("c_raytracer_world.txt", 61, 37, 3)])
def test_ndevices_one_equals_single_device(scene, w, h, spp):
    world = R.World(scene_text(scene))
    ref, st = world.render(w, h, spp, 8)
    out, st1 = world.render(w, h, spp, 8, ndevices=1)
    assert_bits_equal(out, ref, "ndevices=1 frame")
    assert st1["rays"] == st["rays"] and st1["samples"] == st["samples"]
    # the counted multi-device frame reports the schedule its devices ran (the
    # uncounted kernel's launch settings), which a single-device frame shares;
    # its counters are collected after every device's tile was enqueued
    launch = [k for k in st if k.startswith("launch_")]
    assert len(launch) == 8 and all(st1[k] == st[k] for k in launch), (st, st1)
    assert st["launch_blocks"] > 0 and st["launch_parts"] >= 1 and st["launch_chunk"] % spp == 0
    lean, _ = world.render(w, h, spp, 8, ndevices=1, stats=False)
    assert_bits_equal(lean, ref, "ndevices=1 frame without counters")
    with pytest.raises(R.RenderError, match="rank/nranks"):
        world.render(w, h, spp, 8, ndevices=1, rank=1, nranks=2)
    with pytest.raises(R.RenderError, match="not all visible"):
        world.render(w, h, spp, 8, ndevices=R.device_count() + 1)


def test_ndevices_render_device_into_torch_frame():
    import torch

    world = R.World(scene_text("rtow.txt"))
    w, h, spp = 96, 54, 4
    ref, _ = world.render(w, h, spp, 8)
    frame = torch.zeros(h * w * 4, dtype=torch.uint8, device="cuda:0")
    stream = torch.cuda.Stream(device="cuda:0")
    for _ in range(3):  # frames pipelined on the caller's stream, no host wait
        world.render_device(w, h, frame.data_ptr(), stream.cuda_stream, spp=spp, depth=8,
                            device=0, stats=False, ndevices=1)
    torch.cuda.synchronize(0)
    assert_bits_equal(frame.cpu().numpy().reshape(h, w, 4), ref, "device frame")


def test_render_entry_point_with_rt_amd_devices(monkeypatch):
    """render() (lib.rs:49-57, 16 spp / depth 8) spread over RT_AMD_DEVICES."""
    src = scene_text("c_raytracer_world.txt")
    img, _, _ = O.Scene(src).render(40, 30, 16, 8, mode=O.RNG_COUNTER, nthreads=8)
    world = R.World(src)
    monkeypatch.setenv("RT_AMD_RNG", "counter")
    for v in ("1", "0", "junk"):  # 0 / invalid: one device
        monkeypatch.setenv("RT_AMD_DEVICES", v)
        assert_bits_equal(world.render_reference(40, 30), img, f"render() RT_AMD_DEVICES={v}")
    monkeypatch.setenv("RT_AMD_DEVICES", str(R.device_count() + 1))
    with pytest.raises(R.RenderError):
        world.render_reference(40, 30)


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _bench_env():
    env = dict(os.environ)
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK"):
        env.pop(k, None)
    return env


def test_bench_single_process_gpus_1():
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "1", "--config",
                        "c1", "--steps", "3", "--warmup", "1", "--no-cpu-baseline"],
                       env=_bench_env(), capture_output=True, text=True, timeout=110)
    assert r.returncode == 0, r.stderr[-2000:]
    line = json.loads(r.stdout.strip().splitlines()[-1])
    assert line["n_gpus"] == 1 and line["rccl_ranks"] == 1 and line["launch"] == "single process"
    assert line["value"] > 0 and line["rays_per_frame"] > 65536


def test_bench_torchrun_two_ranks_rehearsal():
    """The driver's N>1 launch, two ranks on the one GPU with gloo: HIP tiles,
    all-gather, and the assembled frame equal to a one-rank render."""
    env = _bench_env()
    env.update(RT_BENCH_ONE_DEVICE="1", RT_BENCH_BACKEND="gloo", RT_BENCH_VERIFY="1",
               OMP_NUM_THREADS="2")
    r = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
                        "--nproc-per-node", "2", "--master-addr", "127.0.0.1", "--master-port",
                        str(_free_port()), os.path.join(ROOT, "bench.py"), "--gpus", "2",
                        "--config", "c1", "--steps", "2", "--warmup", "1"],
                       env=env, capture_output=True, text=True, timeout=110)
    assert r.returncode == 0, r.stderr[-3000:]
    assert "verify: assembled frame == single-rank frame" in r.stderr
    # the frame rank 0 assembled inside its timed steps (rt_assemble_tiles on the
    # gathered tiles, as the single-process launch does after its ncclGather)
    assert "verify: timed-step frame == single-rank frame" in r.stderr
    line = json.loads(r.stdout.strip().splitlines()[-1])
    assert line["n_gpus"] == 2 and line["rccl_ranks"] == 2


@pytest.mark.parametrize("n,h", [(2, 90), (3, 91), (8, 90), (8, 37), (3, 5), (5, 8)])
def test_assemble_kernel_n_ranks(n, h):
    """render_frame_multi's last step for n > 1 (which only a multi-GPU node
    runs end to end): every rank's tile rendered on device 0, packed in the
    layout the RCCL gather leaves on the first device (tile g at row g *
    max_rows, short tiles padded), assembled by assemble_kernel through
    rt_assemble_tiles, bit-identical to the single-device frame; also equal
    to the host-side tiles.assemble.  Heights that are not multiples of the
    8-row block, and more ranks than row blocks (3 x 5 rows)."""
    import torch

    import tiles

    world = R.World(scene_text("rtow.txt"))
    w, spp, B = 75, 2, 8
    ref, _ = world.render(w, h, spp, 8)
    max_rows = max(R.tile_rows(h, B, g, n) for g in range(n))
    gathered = torch.full((n * max_rows * w * 4,), 7, dtype=torch.uint8, device="cuda:0")
    for g in range(n):
        rows = R.tile_rows(h, B, g, n)
        if rows == 0:
            continue
        tile, _ = world.render(w, h, spp, 8, row_block=B, rank=g, nranks=n)
        off = g * max_rows * w * 4
        gathered[off:off + rows * w * 4] = torch.from_numpy(tile.reshape(-1)).to("cuda:0")
    frame = torch.zeros(h * w * 4, dtype=torch.uint8, device="cuda:0")
    R.assemble_tiles(gathered.data_ptr(), frame.data_ptr(), w, h, B, n, max_rows)
    torch.cuda.synchronize(0)
    out = frame.cpu().numpy().reshape(h, w, 4)
    assert_bits_equal(out, ref, f"assembled {n}-rank frame")
    host = tiles.assemble(gathered.cpu().numpy(), w, h, B, n)
    assert_bits_equal(host, ref, f"tiles.assemble of the {n}-rank gather")
    with pytest.raises(R.RenderError, match="max_rows"):
        R.assemble_tiles(gathered.data_ptr(), frame.data_ptr(), w, h, B, n, max_rows - 1)


def test_serial_multi_device_path_one_device():
    """SERIAL through the multi-device path (render()'s default RNG with
    RT_AMD_DEVICES): the start states are found once on the first device and
    broadcast, then the tiles render in REPLAY mode -- bit-exact vs the
    oracle's SERIAL frame."""
    src = scene_text("c_raytracer_world.txt")
    img, st, _ = O.Scene(src).render(48, 40, 4, 8, mode=O.RNG_SERIAL)
    world = R.World(src)
    out, gst = world.render(48, 40, 4, 8, mode=R.RNG_SERIAL, ndevices=1, serial_check=True)
    assert_bits_equal(out, img, "ndevices=1 SERIAL frame")
    assert gst["rays"] == st["rays"] and gst["serial_chain_breaks"] == 0 and gst["serial_checked"] == 48 * 40 * 4
    assert gst["serial_ms"] > 0


def test_job_counter_sets_across_streams_serial_and_partitions(monkeypatch):
    """The double-buffered job counters (runtime.cpp: a frame launch takes one
    set, zeroed by the launch before it, and zeroes the other): COUNTER frames
    on a user stream and on the library stream, a SERIAL frame (whose passes
    reset the sets) between them, and the partition count changed from frame
    to frame (RT_AMD_PARTS 1, 1024, 3, default).  Every frame's bits and
    ray / sample counts equal the first frame's."""
    import torch

    src = scene_text("rtow.txt")
    w, h, spp = 120, 68, 8
    world = R.World(src)
    ref, st0 = world.render(w, h, spp, 8)
    frame = torch.zeros(w * h * 4, dtype=torch.uint8, device="cuda:0")
    user = torch.cuda.Stream(device="cuda:0")
    serial_ref, _, _ = O.Scene(src).render(w // 4, h // 4, 4, 8, mode=O.RNG_SERIAL)
    for k, parts in enumerate(["1", "1024", "3", None, "1024", "1"]):
        if parts is None:
            monkeypatch.delenv("RT_AMD_PARTS", raising=False)
        else:
            monkeypatch.setenv("RT_AMD_PARTS", parts)
        if k % 2 == 0:  # a user stream (rt_render_device), counted and uncounted
            st = world.render_device(w, h, frame.data_ptr(), user.cuda_stream, spp=spp, depth=8, device=0)
            world.render_device(w, h, frame.data_ptr(), user.cuda_stream, spp=spp, depth=8, device=0,
                                stats=False)
            user.synchronize()
            out = frame.cpu().numpy().reshape(h, w, 4)
        else:  # the library stream
            out, st = world.render(w, h, spp, 8)
        assert_bits_equal(out, ref, f"frame {k} (RT_AMD_PARTS={parts})")
        assert st["rays"] == st0["rays"] and st["samples"] == st0["samples"], (k, st, st0)
        if k in (1, 3):  # a SERIAL frame between COUNTER frames
            sout, _ = world.render(w // 4, h // 4, 4, 8, mode=R.RNG_SERIAL)
            assert_bits_equal(sout, serial_ref, f"SERIAL frame after frame {k}")
