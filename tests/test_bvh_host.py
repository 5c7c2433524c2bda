"""Host-side structural checks of the BVH builders (no GPU): tests/bvh_check.cpp
compiled with g++ against csrc/bvh.cpp + csrc/scene.cpp.  Every primitive in
exactly one leaf, nested boxes (and nested normal boxes), octant links that
walk every node once, quantised kernel nodes that decode to conservative
boxes and round-trip their child/leaf words (bvh.h)."""
import os
import subprocess

import pytest

import scenes as S
from conftest import ROOT

CSRC = os.path.join(ROOT, "rust-swift-raytracer_amd", "csrc")


@pytest.fixture(scope="module")
def checker(tmp_path_factory):
    exe = str(tmp_path_factory.mktemp("bvh") / "bvh_check")
    subprocess.run(["g++", "-O2", "-std=c++17", f"-I{CSRC}", os.path.join(ROOT, "tests", "bvh_check.cpp"),
                    os.path.join(CSRC, "bvh.cpp"), os.path.join(CSRC, "scene.cpp"), "-o", exe], check=True)
    return exe


def run(checker, tmp_path, text, leaf=2):
    path = tmp_path / "scene.txt"
    path.write_text(text)
    r = subprocess.run([checker, str(path), str(leaf)], capture_output=True, text=True)
    assert r.returncode == 0, r.stdout + r.stderr
    return r.stdout


def test_rtow_sphere_tree(checker, tmp_path):
    assert "spheres 486" in run(checker, tmp_path, S.rtow())


@pytest.mark.parametrize("case", [
    dict(seed=11, n=600),
    dict(seed=12, n=400, size=2.0, dup=80, slivers=30),
    dict(seed=13, n=300, spheres=200, grid=12),
    dict(seed=14, n=500, big=6, spread=8.0),
    dict(seed=15, n=400, offset=(2500.0, -1800.0, 900.0), cam=(2500.0, -1800.0, 900.0)),
])
@pytest.mark.parametrize("leaf", [1, 2, 7])
def test_triangle_trees(checker, tmp_path, case, leaf):
    out = run(checker, tmp_path, S.triangle_soup(**case), leaf)
    assert "OK" in out


def test_mesh_c5_trees(checker, tmp_path):
    out = run(checker, tmp_path, S.mesh(nx=100, ny=80))
    assert "triangles 16000 tree 16000" in out
