import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "rust-swift-raytracer_amd")  # noqa
for p in (PKG, os.path.join(ROOT, "oracle"), os.path.join(ROOT, "tools"),
          os.path.join(ROOT, "tests")):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through the HIP C-ABI)")


def _make(path):
    subprocess.run(["make", "-s", "-C", path], check=True)


@pytest.fixture(scope="session", autouse=True)
def built():
    """Build the oracle and the product library once (no-ops when up to date)."""
    _make(os.path.join(ROOT, "oracle"))
    _make(PKG)  # (a no-op when the library is newer than its sources)
    return True


def scene_text(name):
    with open(os.path.join(ROOT, "scenes", name)) as fh:
        return fh.read()
