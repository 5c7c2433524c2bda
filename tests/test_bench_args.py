"""CPU tests of bench.py's --gpus handling (no GPU needed).

The driver runs `python bench.py --gpus N` (one process drives N GPUs through
the library's multi-device mode) and `torch.distributed.run --nproc-per-node N
bench.py --gpus N` (one rank per GPU).  A rank count that differs from --gpus,
or more GPUs than are visible, must stop the bench before any GPU work instead
of silently timing fewer GPUs.
"""
import os
import subprocess
import sys

from conftest import ROOT

BENCH = os.path.join(ROOT, "bench.py")


def _run(args, env_extra):
    env = dict(os.environ)
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK"):
        env.pop(k, None)
    env.update(env_extra)
    return subprocess.run([sys.executable, BENCH] + args, env=env, capture_output=True, text=True,
                          timeout=300)


def test_launcher_rank_count_must_equal_gpus():
    r = _run(["--gpus", "2", "--steps", "1"], {"WORLD_SIZE": "3", "RANK": "0", "LOCAL_RANK": "0"})
    assert r.returncode != 0
    assert "--gpus 2 but the launcher started 3 ranks" in r.stderr


def test_more_gpus_than_visible_is_refused():
    import raytracer_amd as R

    n = R.device_count() + 1
    r = _run(["--gpus", str(n), "--steps", "1"], {})
    assert r.returncode != 0
    assert f"--gpus {n} but only" in r.stderr


def test_gpus_must_be_positive():
    r = _run(["--gpus", "0"], {})
    assert r.returncode != 0 and "--gpus must be >= 1" in r.stderr


def _bench_module():
    import importlib.util

    spec = importlib.util.spec_from_file_location("bench_under_test", BENCH)
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


def test_spp_and_depth_override_the_config():
    """--spp / --depth (and the reference CLI's samples= / ray_depth=,
    main.rs:23-45) replace the config's spp and depth; the defaults keep the
    config's, so the driver's bench line is unchanged."""
    b = _bench_module()
    _, W, H, spp, depth = b.workload(b.parse_args([]))
    assert (W, H, spp, depth) == (1920, 1080, 64, 8)
    _, W, H, spp, depth = b.workload(b.parse_args(["--spp", "16", "--depth", "4"]))
    assert (W, H, spp, depth) == (1920, 1080, 16, 4)
    _, _, _, spp, depth = b.workload(b.parse_args(["--config", "c3", "--depth", "5"]))
    assert (spp, depth) == (256, 5)
    # the reference's argument syntax: leading digits only (parser.rs:90-104)
    _, _, _, spp, depth = b.workload(b.parse_args(["samples=32", "ray_depth=3x"]))
    assert (spp, depth) == (32, 3)


def test_bad_spp_and_reference_args_are_refused():
    r = _run(["--spp", "0"], {})
    assert r.returncode != 0 and "--spp must be >= 1" in r.stderr
    r = _run(["samples=abc"], {})
    assert r.returncode != 0 and "cannot parse 'samples=abc'" in r.stderr
    r = _run(["ray_depth=99999999999"], {})
    assert r.returncode != 0 and "cannot parse" in r.stderr
