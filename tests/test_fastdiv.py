"""CPU check of the magic-number division the trace kernel uses to map a job
to (pixel, sample) (csrc/fastdiv.h): exact for every 32-bit dividend."""
import os
import subprocess

from conftest import PKG

SRC = r"""
#include <cstdio>
#include <random>
#include "fastdiv.h"
using namespace rtamd;
int main() {
    std::mt19937_64 g(7); long bad = 0;
    const uint32_t ds[] = {1,2,3,5,7,8,16,64,65,100,255,256,1000,1080,1920,2160,3840,123457,
                           1u<<20,(1u<<31)-1,1u<<31,4294967295u};
    for (uint32_t d : ds) { FastDiv f = make_fastdiv(d);
        for (long i = 0; i < 300000; ++i) {
            uint32_t n = i < 1000 ? (uint32_t)i : i < 2000 ? 0xFFFFFFFFu - (uint32_t)(i - 1000) : (uint32_t)g();
            bad += fastdiv_apply(n, f) != n / d; } }
    for (int k = 0; k < 100000; ++k) { uint32_t d = ((uint32_t)g() | 1u) >> (k % 32); if (!d) d = 1;
        FastDiv f = make_fastdiv(d);
        for (int i = 0; i < 10; ++i) { uint32_t n = (uint32_t)g(); bad += fastdiv_apply(n, f) != n / d; } }
    std::printf("%ld\n", bad); return bad != 0;
}
"""


def test_fastdiv_exact(tmp_path):
    src = tmp_path / "fd.cpp"
    src.write_text(SRC)
    exe = tmp_path / "fd"
    subprocess.run(["g++", "-O2", "-std=c++17", f"-I{os.path.join(PKG, 'csrc')}", "-o", str(exe),
                    str(src)], check=True)
    out = subprocess.run([str(exe)], capture_output=True, text=True)
    assert out.returncode == 0 and out.stdout.strip() == "0", out.stdout
