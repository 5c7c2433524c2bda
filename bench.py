"""Benchmark of the MI355X render path on BASELINE.json's headline config.

metric: Mrays/sec (+ frames/sec) at 1920x1080, spp=64, depth 8, on the ~486-
sphere "Ray Tracing in One Weekend" scene (BASELINE.json configs[1]; scene
from tools/scenes.py, synthetic and deterministic).  A step = one full frame:
every pixel sample traced and resolved to RGBA8 in HBM (and, for N>1 GPUs,
the row tiles gathered over RCCL).  The scene is uploaded before timing.

  python bench.py [--gpus N] [--steps K] [--warmup W] [--config c2|c3|c4|c5]
      one process drives N GPUs through the library (RtRenderOptions.ndevices:
      row tiles + RCCL ncclGather to device 0)
  torchrun --nproc-per-node N bench.py --gpus N ...   (one rank per GPU; the
      launcher's rank count must equal --gpus)

Rank 0 prints one JSON line.  `roofline` prices the trace kernel against the
FP32 vector peak (the path is VALU-bound), `cpu_baseline`
times the CPU oracle (the reference's serial-RNG semantics, 1 thread) on a
bounded row-cyclic sample of the same frame.
"""
from __future__ import annotations

import argparse
import hashlib
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
for _p in ("rust-swift-raytracer_amd", "tools"):
    sys.path.insert(0, os.path.join(ROOT, _p))

import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

import raytracer_amd as R  # noqa: E402
import scenes as S  # noqa: E402
import tiles  # noqa: E402

METRIC = "Mrays/sec + frames/sec at 1920×1080 spp=64; 1/2/4/8 MI355X"
FP32_VECTOR_PEAK_TFLOPS = 157.3  # MI355X_MICROARCH.md, chip-level parameters
HBM_PEAK_GBS = 8000.0
ROW_BLOCK = 8  # multi-GPU: row-cyclic blocks of 8 image rows


# the frame trace launch's scheduling settings (RtRenderStats.launch_*)
LAUNCH_KEYS = ("launch_parts", "launch_chunk", "launch_refill_min", "launch_walk_min",
               "launch_tri_walk_min", "launch_wsteps", "launch_block_threads", "launch_blocks")

NODE_TEST_FLOPS = 26  # slab test: 6 sub, 6 mul, 10 min/max, 4 slack mul/compare
# triangle node: s = n^.o interval (6 mul, 6 min/max, 4 add), phantom offsets
# (3 x [4 mul, 6 min/max, 2 mul, 4 add]), slab test (6 sub, 6 mul, 10 min/max, 3 cmp)
TRI_NODE_TEST_FLOPS = 89


def algorithmic_flops(st):
    """17*sphere_tests + 14*tri_tests + 60*tri_in_range
    + 40*rays + 20*samples (no FMA: every add/mul/div/sqrt/compare is 1),
    with sphere_tests = rays * spheres (the reference's brute force)."""
    return (17 * st["sphere_tests"] + 14 * st["tri_tests"] + 60 * st["tri_in_range"]
            + 40 * st["rays"] + 20 * st["samples"])


def s8d_literal_flops(st):
    """SURVEY.md 8(d)'s price list taken literally on the executed work: no
    price for BVH box tests (the list has none), sphere and triangle tests as
    executed."""
    sph = st["bvh_sphere_tests"] + st["big_sphere_tests"]
    return (17 * sph + 14 * st["bvh_tri_tests"] + 60 * st["tri_in_range"] + 40 * st["rays"]
            + 20 * st["samples"])


def executed_flops(st):
    """The same price list applied to the work the kernel actually executed:
    sphere tests done (BVH leaves + spheres kept out of the tree, or all of
    them in brute force) plus NODE_TEST_FLOPS per BVH box test; triangle
    tests done (leaves + brute-forced ones) plus TRI_NODE_TEST_FLOPS per
    triangle-BVH box test."""
    sph = st["bvh_sphere_tests"] + st["big_sphere_tests"]
    return (17 * sph + NODE_TEST_FLOPS * st["bvh_node_tests"] + 14 * st["bvh_tri_tests"]
            + TRI_NODE_TEST_FLOPS * st["tri_node_tests"]
            + 60 * st["tri_in_range"] + 40 * st["rays"] + 20 * st["samples"])


def _host_cpus():
    """(threads the CPU legs may use, CPUs the host reports).  A GPU box shows
    the whole machine's CPUs but grants this job a share of 16."""
    nproc = os.cpu_count() or 1
    try:
        avail = len(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        avail = nproc
    return max(1, min(16, avail)), nproc


def cpu_baseline(src, W, H, spp, depth, budget_s):
    """Oracle on a bounded row-cyclic sample of the same frame: 1 thread in
    SERIAL RNG mode (the reference's semantics and its single-threaded
    ray_trace, common.rs:320-361), and all usable host cores in COUNTER mode
    (rows dealt over threads)."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle as O

    scene = O.Scene(src)
    img = np.zeros((H, W, 4), np.uint8)
    # calibrate on one mid-frame row at 1 spp, then spread the budget over the
    # frame: rows at the full spp when one fits, else rows at 1 spp (the same
    # rays per sample, so the same per-ray rate; C5 rows cost ~1 s per spp)
    t = time.perf_counter()
    scene.render(W, H, 1, depth, mode=O.RNG_SERIAL, row_begin=H // 3, row_step=H, out=img)
    per_row1 = max(time.perf_counter() - t, 1e-4)
    spp_s = spp if per_row1 * spp <= budget_s / 4 else 1
    nrows = int(max(1, min(H, budget_s / (per_row1 * spp_s))))
    step = max(1, H // nrows)
    t = time.perf_counter()
    _, st, _ = scene.render(W, H, spp_s, depth, mode=O.RNG_SERIAL, row_begin=step // 2,
                            row_step=step, out=img)
    dt = time.perf_counter() - t
    threads, nproc = _host_cpus()
    # all cores (COUNTER mode): threads/4 times the serial leg's rows (~2/3 of its time)
    step_mt = max(1, step // max(1, threads // 4))
    t = time.perf_counter()
    _, st_mt, _ = scene.render(W, H, spp_s, depth, mode=O.RNG_COUNTER, row_begin=step_mt // 2,
                               row_step=step_mt, nthreads=threads, out=img)
    dt_mt = time.perf_counter() - t
    return {"value": st["rays"] / dt / 1e6, "unit": "Mrays/s", "cores": 1, "kind": "port",
            "sample": f"oracle SERIAL RNG, rows {step // 2}::{step} of {W}x{H} at spp {spp_s} "
                      f"({st['samples']} samples, {st['rays']} rays, {dt:.1f} s)",
            "msamples_per_s": st["samples"] / dt / 1e6,
            "host_nproc": nproc,
            "all_cores": {"value": st_mt["rays"] / dt_mt / 1e6, "unit": "Mrays/s",
                          "threads": threads, "mode": "COUNTER",
                          "sample": f"rows {step_mt // 2}::{step_mt} at spp {spp_s} "
                                    f"({st_mt['rays']} rays, {dt_mt:.1f} s)"}}


def _cli_int(tok, key):
    """The reference CLI's `key=N` argument (main.rs:23-45): `parser::starts_with`
    on the key and on "=", then `parser::parse_int` (parser.rs:90-104): the
    leading decimal digits as i32 (none, or an i32 overflow, is an error;
    anything after them is ignored)."""
    rest = tok[len(key) + 1:]
    n = 0
    while n < len(rest) and "0" <= rest[n] <= "9":
        n += 1
    if n == 0 or int(rest[:n]) > 2**31 - 1:
        sys.exit(f"bench.py: cannot parse '{tok}' as {key}=N")
    return rest[:n]


def _translate_reference_args(argv):
    """Mirror of the reference CLI's `samples=N` / `ray_depth=N` arguments
    (raytracer/src/main.rs:23-45): rewritten to --spp / --depth."""
    out = []
    for tok in argv:
        if tok.startswith("samples="):
            out += ["--spp", _cli_int(tok, "samples")]
        elif tok.startswith("ray_depth="):
            out += ["--depth", _cli_int(tok, "ray_depth")]
        else:
            out.append(tok)
    return out


def parse_args(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--config", default="c2", choices=sorted(S.CONFIGS))
    # samples per pixel / max ray bounces of the chosen config, overridden
    # (the reference CLI's samples= / ray_depth=, main.rs:23-45, are accepted too)
    ap.add_argument("--spp", type=int, default=None)
    ap.add_argument("--depth", type=int, default=None)
    ap.add_argument("--cpu-seconds", type=float, default=15.0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--accel", default="auto", choices=["auto", "brute", "bvh"])
    ap.add_argument("--no-serial", action="store_true",
                    help="skip the RT_RNG_SERIAL (reference-identical render()) legs")
    args = ap.parse_args(_translate_reference_args(sys.argv[1:] if argv is None else argv))
    if args.spp is not None and args.spp < 1:
        sys.exit(f"bench.py: --spp must be >= 1 (got {args.spp})")
    return args


def workload(args):
    """(scene maker, W, H, spp, depth) of the config, with --spp / --depth applied."""
    make_scene, W, H, spp, depth = S.CONFIGS[args.config]
    spp = spp if args.spp is None else args.spp
    depth = depth if args.depth is None else args.depth
    return make_scene, W, H, spp, depth


def main():
    args = parse_args()
    launched = "WORLD_SIZE" in os.environ  # torchrun: one process per GPU
    world_size = int(os.environ.get("WORLD_SIZE", "1"))
    if args.gpus < 1:
        sys.exit(f"bench.py: --gpus must be >= 1 (got {args.gpus})")
    if launched and world_size != args.gpus:
        sys.exit(f"bench.py: --gpus {args.gpus} but the launcher started {world_size} ranks")
    if launched:
        multi_process(args, world_size)
    else:
        single_process(args)


def _setup(args):
    make_scene, W, H, spp, depth = workload(args)
    accel = {"auto": R.ACCEL_AUTO, "brute": R.ACCEL_BRUTE, "bvh": R.ACCEL_BVH}[args.accel]
    src = make_scene()
    return src, R.World(src), W, H, spp, depth, accel


def _timed(args, step, stream, sync, barrier):
    """W warmup frames, one counting frame, then K timed frames between
    barrier + synchronize on both sides (HIP events around each frame's render
    on the launch stream), then counting frames like the timed ones."""
    for _ in range(args.warmup):
        step(False)
    st_warm = step(True)  # counters of one frame (the frame is identical every step)
    sync()
    barrier()
    evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
           for _ in range(args.steps)]
    t0 = time.perf_counter()
    for k in range(args.steps):
        step(False, evs[k])
    sync()
    barrier()
    elapsed = time.perf_counter() - t0
    stats = [step(True) for _ in range(max(1, min(args.steps, 3)))]
    assert all(s["rays"] == st_warm["rays"] for s in stats), "frames must be identical"
    # (a timed frame's render is its trace launch(es): each launch zeroes the
    # other job-counter set for the next one, so no fill launch per frame)
    trace_ms = (sum(a.elapsed_time(b) for a, b in evs) / args.steps
                / max(1, stats[-1]["trace_launches"]))
    count_trace_ms = sum(s["trace_ms"] for s in stats) / max(1, sum(s["trace_launches"] for s in stats))
    return st_warm, stats[-1], elapsed, trace_ms, count_trace_ms


def _post_move(world, step, sync, dz=-0.05):
    """Interactive re-render (lib.rs:60-63, GameView.swift:198-219): the frame
    right after move_camera_position, against steady frames of the moved
    camera.  Sphere scenes build the moved camera's primary candidate lists on
    the device before the frame (RT_AMD_GPU_LISTS=0: on a host thread while the
    first frames render without them); triangle scenes rebuild the camera tree
    and strip lists on the host before the frame."""
    sync()
    world.move_camera(0.0, 0.0, dz)
    t0 = time.perf_counter()
    st = step(True)  # (with counters: the flags say what the frame used)
    sync()
    first = (time.perf_counter() - t0) * 1e3
    first_lists = int(st["primary_lists"] or st["camera_tree"])
    t0 = time.perf_counter()
    while not (st["primary_lists"] or st["camera_tree"]) and time.perf_counter() - t0 < 10:
        time.sleep(0.002)
        st = step(True)
    ready = (time.perf_counter() - t0) * 1e3
    sync()
    times = []
    for _ in range(5):
        t = time.perf_counter()
        step(True)
        sync()
        times.append((time.perf_counter() - t) * 1e3)
    steady = sorted(times)[len(times) // 2]
    return {"move": [0.0, 0.0, dz], "first_frame_ms": first, "steady_frame_ms": steady,
            "ratio": first / steady, "lists_ready_ms": ready,
            "first_frame_lists": first_lists,
            "steady_lists": int(st["primary_lists"] or st["camera_tree"])}


SERIAL_CASES = (
    # (label, scene, width, height, spp, depth): render()'s defaults (lib.rs:51)
    # on the Swift app's world.txt at GameView-like window sizes, and the
    # BASELINE C2 settings on the RTOW scene
    ("world.txt 960x540 render()", "world", 960, 540, 16, 8),
    ("world.txt 1920x1080 render()", "world", 1920, 1080, 16, 8),
    ("c2 settings (rtow 1920x1080x64/8)", "rtow", 1920, 1080, 64, 8),
)


def serial_legs(reps=2):
    """The reference-identical mode (RT_RNG_SERIAL, render()'s default: the
    one xorshift32 stream of common.rs:321, resolved on the GPU and rendered
    bit for bit): wall time per frame through the C-ABI, start-state search
    time, iterations, and the frame right after move_camera_position
    (GameView.swift:198-219) against steady frames.  Every frame's chain is
    checked once (RT_FLAG_SERIAL_CHECK) outside the timed calls."""
    out = []
    for label, scene, W, H, spp, depth in SERIAL_CASES:
        src = S.read("world.txt") if scene == "world" else S.rtow()
        world = R.World(src)
        _, chk = world.render(W, H, spp, depth, mode=R.RNG_SERIAL, serial_check=True)
        times, st = [], None
        for _ in range(reps):
            t = time.perf_counter()
            if (spp, depth) == (16, 8):
                world.render_reference(W, H)  # render() itself: host frame, synchronous
            else:
                world.render(W, H, spp, depth, mode=R.RNG_SERIAL, stats=False)
            times.append(time.perf_counter() - t)
        _, st = world.render(W, H, spp, depth, mode=R.RNG_SERIAL)
        wall = min(times)
        leg = {"case": label, "width": W, "height": H, "spp": spp, "depth": depth,
               "samples": W * H * spp, "ms_per_frame": wall * 1e3,
               "mrays_per_s": st["rays"] / wall / 1e6, "msamples_per_s": W * H * spp / wall / 1e6,
               "start_states_ms": st["serial_ms"], "tables_ms": st["serial_setup_ms"],
               "replay_trace_ms": st["trace_ms"], "iterations": st["serial_iterations"],
               "iterations_stopped_short": st["serial_retries"],
               "chain_checked": chk["serial_checked"], "chain_breaks": chk["serial_chain_breaks"],
               "api": "render()" if (spp, depth) == (16, 8) else "rt_render_ex SERIAL"}
        if scene == "world" and W == 960:
            world.move_camera(0.0, 0.0, -0.05)
            t = time.perf_counter()
            world.render_reference(W, H)
            first = time.perf_counter() - t
            steady = []
            for _ in range(reps):
                t = time.perf_counter()
                world.render_reference(W, H)
                steady.append(time.perf_counter() - t)
            leg["post_move"] = {"move": [0.0, 0.0, -0.05], "first_frame_ms": first * 1e3,
                                "steady_frame_ms": min(steady) * 1e3,
                                "ratio": first / min(steady)}
        out.append(leg)
        world.close()
    return out


def single_process(args):
    """N GPUs from this one process through the library's multi-device mode
    (RtRenderOptions.ndevices): every device renders its row blocks, an RCCL
    ncclGather (ncclCommInitAll communicator) collects the tiles on device 0
    and a kernel assembles the frame there.  N = 1 runs the same path (the
    gather is then a copy into the frame)."""
    ngpu = args.gpus
    if R.device_count() < ngpu:
        sys.exit(f"bench.py: --gpus {ngpu} but only {R.device_count()} devices are visible")
    torch.cuda.set_device(0)
    ranks = R.comm_count(0, ngpu)
    assert ranks == ngpu, f"RCCL communicator has {ranks} ranks, --gpus {ngpu}"
    src, world, W, H, spp, depth, accel = _setup(args)
    dev = torch.device("cuda", 0)
    frame = torch.zeros(H * W * 4, dtype=torch.uint8, device=dev)
    stream = torch.cuda.Stream(device=dev)
    torch.cuda.set_stream(stream)

    def step(with_stats, ev=None):
        if ev is not None:
            ev[0].record(stream)
        st = world.render_device(W, H, frame.data_ptr(), stream.cuda_stream, spp=spp, depth=depth,
                                 row_block=ROW_BLOCK, device=0, accel=accel, stats=with_stats,
                                 ndevices=ngpu)
        if ev is not None:
            ev[1].record(stream)
        return st

    def sync():
        for d in range(ngpu):
            torch.cuda.synchronize(d)

    st_warm, st0, elapsed, trace_ms, count_trace_ms = _timed(args, step, stream, sync, lambda: None)
    moved = _post_move(world, step, sync)
    rows = R.tile_rows(H, ROW_BLOCK, 0, ngpu) if ngpu > 1 else H
    if ngpu > 1:
        par = (f"row-tiles x{ngpu} (block {ROW_BLOCK}), one process, RCCL ncclGather "
               f"({ranks} ranks) to device 0 + assemble kernel")
    else:
        par = "one device renders the frame in place (no RCCL call)"
    extra = {"rccl_ranks": ranks, "launch": "single process", "post_move": moved}
    if ngpu == 1 and not args.no_serial:
        torch.cuda.set_stream(torch.cuda.default_stream(dev))
        extra["serial"] = serial_legs()
    _report(args, src, world, W, H, spp, depth, st0, st_warm["rays"] * args.steps, elapsed,
            trace_ms, count_trace_ms, ngpu, rows, par, extra)


def multi_process(args, world_size):
    """One rank per GPU (torch.distributed.run): each rank renders its row
    tile, the tiles are all-gathered over RCCL (torch.distributed "nccl")."""
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    # rehearsal knobs for a 1-GPU box (never set by the driver): all ranks on
    # device 0 and gloo collectives, to exercise the N>1 path end to end
    if os.environ.get("RT_BENCH_ONE_DEVICE") == "1":
        local_rank = 0
    backend = os.environ.get("RT_BENCH_BACKEND", "nccl")
    torch.cuda.set_device(local_rank)
    if world_size > 1:
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", local_rank))
        else:
            dist.init_process_group(backend)
        assert dist.get_world_size() == args.gpus, "process group size != --gpus"

    src, world, W, H, spp, depth, accel = _setup(args)
    nr = world_size
    rows = R.tile_rows(H, ROW_BLOCK, rank, nr) if nr > 1 else H
    max_rows = max(R.tile_rows(H, ROW_BLOCK, r, nr) for r in range(nr)) if nr > 1 else H
    dev = torch.device("cuda", local_rank)
    tile = torch.zeros(max_rows * W * 4, dtype=torch.uint8, device=dev)
    gathered = torch.empty(nr * max_rows * W * 4, dtype=torch.uint8, device=dev) if nr > 1 else None
    # rank 0 assembles the frame from the gathered tiles inside every step (the
    # single-process launch's assemble_kernel after its ncclGather): both launch
    # shapes time the same work
    frame = torch.zeros(H * W * 4, dtype=torch.uint8, device=dev) if nr > 1 and rank == 0 else None
    # one explicit stream for the frames, their HIP events and the RCCL
    # gather (the default stream's handle is 0, which the library would
    # replace with its own stream)
    stream = torch.cuda.Stream(device=dev)
    torch.cuda.set_stream(stream)

    def step(with_stats, ev=None):
        # timed steps run without counters (the kernel variant whose work
        # counters compile away): the frame is only enqueued (no host wait), so
        # frames and the RCCL gather pipeline on the stream
        if ev is not None:
            ev[0].record(stream)
        st = world.render_device(W, H, tile.data_ptr(), stream.cuda_stream, spp=spp, depth=depth,
                                 row_block=ROW_BLOCK, rank=rank, nranks=nr, device=local_rank,
                                 accel=accel, stats=with_stats)
        if ev is not None:
            ev[1].record(stream)
        if nr > 1:
            if backend == "nccl":
                tiles.gather(tile, gathered)  # RCCL all-gather over xGMI
            else:
                gathered.copy_(tiles.gather_any(tile.cpu(), nr))
            if frame is not None:
                R.assemble_tiles(gathered.data_ptr(), frame.data_ptr(), W, H, ROW_BLOCK, nr, max_rows,
                                 stream.cuda_stream)
        return st

    barrier = dist.barrier if nr > 1 else (lambda: None)
    st_warm, st0, elapsed, trace_ms, count_trace_ms = _timed(
        args, step, stream, torch.cuda.synchronize, barrier)
    rays = st_warm["rays"] * args.steps
    if nr > 1:
        tdev = dev if backend == "nccl" else torch.device("cpu")
        t_max = torch.tensor([elapsed], dtype=torch.float64, device=tdev)
        t_sum = torch.tensor([float(rays)], dtype=torch.float64, device=tdev)
        dist.all_reduce(t_max, op=dist.ReduceOp.MAX)
        dist.all_reduce(t_sum, op=dist.ReduceOp.SUM)
        elapsed, rays = float(t_max[0]), int(t_sum[0])
        if os.environ.get("RT_BENCH_VERIFY") == "1":
            # the frame the last timed step assembled on rank 0 (and the host
            # reassembly of the gathered tiles) must equal a one-rank render
            img = tiles.assemble(gathered.cpu().numpy(), W, H, ROW_BLOCK, nr)
            if rank == 0:
                ref, _ = world.render(W, H, spp, depth, device=local_rank)
                assert (img == ref).all(), "assembled multi-rank frame differs"
                timed = frame.cpu().numpy().reshape(H, W, 4)
                assert (timed == ref).all(), "timed-step frame differs from the one-rank frame"
                print("verify: assembled frame == single-rank frame", file=sys.stderr)
                print("verify: timed-step frame == single-rank frame", file=sys.stderr)
    if rank == 0:
        par = (f"row-tiles x{nr} (block {ROW_BLOCK}), one process per GPU, RCCL all-gather "
               "+ assemble kernel on rank 0" if nr > 1 else
               "one device renders the frame in place (no RCCL call)")
        _report(args, src, world, W, H, spp, depth, st0, rays, elapsed, trace_ms, count_trace_ms,
                nr, rows, par, {"rccl_ranks": nr, "launch": "torch.distributed.run"})
    if nr > 1:
        dist.destroy_process_group()


def _report(args, src, world, W, H, spp, depth, st0, rays, elapsed, trace_ms, count_trace_ms,
            nr, rows, parallelism, extra):
    launches = max(1, st0["trace_launches"])
    flops_per_launch = executed_flops(st0) / launches
    achieved_tflops = flops_per_launch / (trace_ms * 1e-3) / 1e12
    alg_tflops = algorithmic_flops(st0) / launches / (trace_ms * 1e-3) / 1e12
    out_bytes = rows * W * 4
    # roofline.traffic: HBM bytes per trace launch from the separate rocprofv3
    # --pmc FETCH_SIZE / WRITE_SIZE passes of tools/profile.sh (counters cannot
    # be read inside this run), keyed on the sha256 of the frame trace kernels'
    # machine code (tools/kernel_hash.py) -- the code those counters describe --
    # next to the same hash of the library this run loaded; the whole-.so
    # hashes are reported too
    # the timed (uncounted) kernel's schedule: profiles record it with their
    # counters, and the traffic below counts only if it is the same
    launch = {k[len("launch_"):]: st0[k] for k in LAUNCH_KEYS}
    traffic, tsrc, ent = None, None, {}
    tfile = os.path.join(ROOT, "profiles", "hbm_traffic.json")
    if os.path.exists(tfile):
        with open(tfile) as fh:
            ent = json.load(fh).get(args.config, {})
        traffic = ent.get("trace_bytes_per_launch")
        with open(R.LIB_PATH, "rb") as fh:
            loaded = hashlib.sha256(fh.read()).hexdigest()
        sys.path.insert(0, os.path.join(ROOT, "tools"))
        import kernel_hash  # noqa: E402
        kloaded, _ = kernel_hash.frame_kernel_hash(R.LIB_PATH)
        tsrc = {"file": "profiles/hbm_traffic.json", "profile": ent.get("from"),
                "profiled_trace_kernel_sha256": ent.get("trace_kernel_sha256"),
                "benched_trace_kernel_sha256": kloaded,
                "same_trace_kernel": ent.get("trace_kernel_sha256") is not None
                and ent.get("trace_kernel_sha256") == kloaded,
                "profiled_launch": ent.get("launch"),
                "same_launch_settings": ent.get("launch") == launch,
                "profiled_lib_sha256": ent.get("lib_sha256"), "benched_lib_sha256": loaded,
                "same_binary": ent.get("lib_sha256") == loaded}
    ms_per_step = elapsed / args.steps * 1e3
    # VALU evidence of the same hash-keyed profile (tools/pmc_summary.py): lanes
    # active per VALU instruction, VALU lane-slots per ray and the issue rate
    # against the v_add_f32 issue rate measured on the box
    # (tools/probe/ubench_enc.hip, profiles/valu_ceiling.json) -- null unless
    # the profiled trace kernel is the one this run loaded
    same = bool(tsrc and tsrc["same_trace_kernel"])
    pv = (ent.get("valu") or {}) if same else {}
    ceiling = None
    cfile = os.path.join(ROOT, "profiles", "valu_ceiling.json")
    if os.path.exists(cfile):
        with open(cfile) as fh:
            ceiling = json.load(fh)
    no_fma = ceiling["v_add_f32_tera_lane_ops_per_s"] if ceiling else None
    s8d_tflops = s8d_literal_flops(st0) / launches / (trace_ms * 1e-3) / 1e12
    valu = {"valu_issue_frac": pv.get("issue_frac_of_v_add_rate"),
            "lanes_active": pv.get("lanes_active"),
            "valu_lane_slots_per_ray": pv.get("lane_slots_per_ray"),
            "wait_frac": pv.get("wait_frac"),
            "valu_from": ent.get("from") if same else None,
            "profile_ms_per_step": ent.get("profile_ms_per_step") if same else None,
            "profile_timed_avg_launch_ms": ent.get("timed_avg_launch_ms") if same else None,
            # the practical ceiling without FMA (parity forbids contraction): one
            # f32 op per lane per v_add_f32 issue slot, measured on the box
            "no_fma_ceiling_tflops": no_fma,
            "frac_of_no_fma_ceiling": achieved_tflops / no_fma if no_fma else None,
            "no_fma_ceiling_from": ceiling.get("from") if ceiling else None,
            # SURVEY 8(d) literally: no price for box tests
            "s8d_literal_tflops": s8d_tflops,
            "s8d_literal_frac": s8d_tflops / FP32_VECTOR_PEAK_TFLOPS}
    result = {
        "metric": METRIC,
        "value": rays / elapsed / 1e6,
        "unit": "Mrays/s",
        "n_gpus": nr,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": ms_per_step,
        "frames_per_sec": 1e3 / ms_per_step,
        "msamples_per_sec": W * H * spp * args.steps / elapsed / 1e6,
        "higher_is_better": True,
        "scaling": "strong",
        "vs_baseline": None,
        "dtype": "f32",
        "data": "synthetic (deterministic RTOW scene, tools/scenes.py)",
        "config": {"workload": f"{args.config}: {W}x{H}, spp {spp}, depth {depth}, "
                               f"{world.num_spheres} spheres, {world.num_triangles} triangles, "
                               "COUNTER RNG", "width": W, "height": H, "spp": spp,
                   "depth": depth, "parallelism": parallelism},
        "roofline": {"bound": "valu", "achieved": achieved_tflops,
                     "peak": FP32_VECTOR_PEAK_TFLOPS, "unit": "TFLOP/s",
                     "frac": achieved_tflops / FP32_VECTOR_PEAK_TFLOPS, "traffic": traffic,
                     "traffic_source": tsrc,
                     "kernel": "trace_kernel", "avg_launch_ms": trace_ms,
                     "counting_variant_ms": count_trace_ms,
                     "flops_per_launch": flops_per_launch, "flops": "executed work",
                     "brute_force_equivalent_tflops": alg_tflops,
                     "algorithmic_hbm_gbs": out_bytes / (trace_ms * 1e-3) / 1e9,
                     "hbm_peak_gbs": HBM_PEAK_GBS, **valu},
        "launch_settings": launch,
        "rays_per_frame": st0["rays"],
        "accel": {1: "brute", 2: "bvh"}.get(st0["accel"], "?"),
        "per_ray": {"sphere_tests": (st0["bvh_sphere_tests"] + st0["big_sphere_tests"]) / st0["rays"],
                    "node_tests": st0["bvh_node_tests"] / st0["rays"],
                    "tri_tests": st0["bvh_tri_tests"] / st0["rays"],
                    "tri_node_tests": st0["tri_node_tests"] / st0["rays"],
                    "tri_in_range": st0["tri_in_range"] / st0["rays"],
                    "brute_force_sphere_tests": st0["sphere_tests"] / st0["rays"]},
    }
    result.update(extra)
    if nr == 1 and not args.no_cpu_baseline:
        result["cpu_baseline"] = cpu_baseline(src, W, H, spp, depth, args.cpu_seconds)
    print(json.dumps(result))


if __name__ == "__main__":
    main()
