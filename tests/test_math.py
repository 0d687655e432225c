"""The sampler's sin/cos (csrc/fmgi_math.h) against glibc on every reachable input.

photonmap.cl:33,57 draw phi = 6.283184f * rand() with rand() = (float)s * 2^-32 (photonmap.cl:21-25),
so phi takes ~8.4e7 distinct values. The parity contract fixes sin/cos to (float)sin((double)phi); the
exhaustive C checker (tests/tools/check_sincos.c) verifies fmgi_sincosf reproduces glibc bit for bit
on all of them. The GPU twin of this test is in test_gpu_parity.py."""
import os
import subprocess

import numpy as np

import fmgi
from conftest import PKG, REPO


def test_sincos_exhaustive_vs_glibc(tmp_path):
    exe = tmp_path / "check_sincos"
    subprocess.run(
        ["gcc", "-O2", "-ffp-contract=off", "-fopenmp", "-I", os.path.join(PKG, "csrc"),
         os.path.join(REPO, "tests", "tools", "check_sincos.c"), "-o", str(exe), "-lm"],
        check=True,
    )
    out = subprocess.run([str(exe)], capture_output=True, text=True, check=True, timeout=600).stdout.split()
    checked, bad = int(out[-2]), int(out[-1])
    assert checked == 83_886_081
    assert bad == 0


def test_library_sincos_matches_numpy_double_rounding():
    xs = np.float32(6.283184) * (np.arange(0, 2**32, 2**20 + 12345, dtype=np.uint64).astype(np.float32) * np.float32(2.0**-32))
    s, c = fmgi.host_sincosf(xs)
    assert np.array_equal(s, np.sin(xs.astype(np.float64)).astype(np.float32))
    assert np.array_equal(c, np.cos(xs.astype(np.float64)).astype(np.float32))
