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
        ["g++", "-x", "c++", "-O2", "-ffp-contract=off", "-fopenmp", "-I", os.path.join(PKG, "csrc"),
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


def test_roulette_threshold_is_the_double_comparison():
    """k_bake tests photonmap.cl:236's `(double)pos.z > 0.0005` as `pos.z > c` with c the largest float
    below 0.0005: the two agree on every float (checked on the floats around the threshold and signs)."""
    c = np.float32(4.99999965541064739227294921875e-4)
    assert float(c) < 0.0005 < float(np.nextafter(c, np.float32(1)))
    z = c.view(np.uint32) + np.arange(-4096, 4097, dtype=np.int64)
    zf = np.concatenate([z.astype(np.uint32).view(np.float32), [0.0, -0.0, -c, 1.0, 1e-5, np.inf]]).astype(np.float32)
    assert np.array_equal(zf.astype(np.float64) > 0.0005, zf > c)
