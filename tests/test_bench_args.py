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
