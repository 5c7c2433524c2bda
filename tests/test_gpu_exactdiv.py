"""exactdiv.h on the device: the shared-reciprocal division the kernel uses
for NVec3::new (maths.rs:111-118), the normal's `/ radius` (common.rs:95) and
the camera's `/ (W-1)`, `/ (H-1)` (common.rs:335-336) must give the bits of
IEEE `/`.  tools/exactdiv_check checks every reciprocal in the guarded range
exhaustively and 16384 x 2^23 quotients against HIP's correctly rounded
divide, plus the guard predicates on their boundary values; and xsqrt (v_sqrt_f32
+ two residual checks) against IEEE sqrtf for all 2^32 inputs."""
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
pytestmark = pytest.mark.gpu


def test_exactdiv_matches_ieee_division():
    exe = os.path.join(ROOT, "tools", "exactdiv_check")
    assert os.path.exists(exe), "build with `make -C rust-swift-raytracer_amd`"
    r = subprocess.run([exe, "16384"], capture_output=True, text=True, timeout=240)
    assert r.returncode == 0 and "exactdiv OK" in r.stdout, r.stdout + r.stderr
    assert "0 mismatches" in r.stdout and "sqrt: all 2^32 inputs, 0 mismatches" in r.stdout
