"""AddressSanitizer + UndefinedBehaviorSanitizer run of the host side
(SURVEY.md 5): the scene parser (csrc/scene.cpp, parser.rs:54-381 grammar with
hand-decoded UTF-8) and the BVH / primary-list builders (csrc/bvh.cpp) under
tests/host_fuzz.cpp -- the committed scenes, ~byte-level mutations of them
(bit flips, insertions, truncations, splices, malformed UTF-8) and random
scenes with degenerate, duplicate, huge and non-finite geometry.  Any
sanitizer report (including float->int casts out of range) fails the test."""
import os
import subprocess

from conftest import ROOT

CSRC = os.path.join(ROOT, "rust-swift-raytracer_amd", "csrc")
SCENES = [os.path.join(ROOT, "scenes", n) for n in
          ("world.txt", "c_raytracer_world.txt", "three_spheres.txt", "rtow.txt")]


def test_parser_and_builders_under_asan_ubsan(tmp_path):
    exe = str(tmp_path / "host_fuzz")
    subprocess.run(["g++", "-O1", "-g", "-std=c++17", "-ffp-contract=off",
                    "-fsanitize=address,undefined,float-cast-overflow", "-fno-sanitize-recover=all",
                    "-fno-omit-frame-pointer", f"-I{CSRC}", os.path.join(ROOT, "tests", "host_fuzz.cpp"),
                    os.path.join(CSRC, "bvh.cpp"), os.path.join(CSRC, "scene.cpp"), "-o", exe],
                   check=True)
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=0",
               UBSAN_OPTIONS="print_stacktrace=1:halt_on_error=1")
    for seed in (1, 2):
        r = subprocess.run([exe, "10", str(seed)] + SCENES, capture_output=True, text=True,
                           timeout=300, env=env)
        assert r.returncode == 0, r.stdout + r.stderr[-4000:]
        assert "runtime error" not in r.stderr and "AddressSanitizer" not in r.stderr
        counts = dict(zip(r.stdout.split()[::2], map(int, r.stdout.split()[1::2])))
        assert counts["parsed"] > 1000 and counts["triangles"] > 1000
