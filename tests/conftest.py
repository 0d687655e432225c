"""Test configuration: paths, the `gpu` marker, in-tree builds and shared scene fixtures.

CPU tests (-m "not gpu") check the oracle against the golden fixtures, the host-side logic of the
C ABI (host-only context) and the library's exports. GPU tests (-m gpu) are the parity tests proper:
they call the HIP path through the C ABI and compare with the oracle bit for bit.
"""
import ctypes
import os
import subprocess
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(REPO, "flatmatch-global-illumination_amd")
ORACLE = os.path.join(REPO, "oracle")
GOLDEN = os.path.join(REPO, "tests", "golden")
for p in (PKG, ORACLE, REPO):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (run with -m gpu on the GPU box)")
    config.addinivalue_line("markers", "slow: long-running")


def _make(d):
    subprocess.run(["make", "-s", "-C", d], check=True, stdout=subprocess.DEVNULL)


@pytest.fixture(scope="session", autouse=True)
def built_libs():
    """Build (or confirm up to date) the product library and the oracle."""
    _make(ORACLE)
    _make(PKG)
    yield


@pytest.fixture(scope="session")
def example_scene():
    from fmgi import scene

    return scene.load_geometry(os.path.join(GOLDEN, "example_geometry.bin"), "example")


@pytest.fixture(scope="session")
def box200():
    from fmgi import scene

    return scene.box_scene(200)


@pytest.fixture(scope="session")
def box2000():
    from fmgi import scene

    return scene.box_scene(2000)


@pytest.fixture
def libc():
    lib = ctypes.CDLL(None)
    lib.rand.restype = ctypes.c_int
    lib.srand.argtypes = [ctypes.c_uint]
    lib.srand(1)  # glibc: srand(1) == the unseeded state main.c runs with
    yield lib
    lib.srand(1)


@pytest.fixture(scope="module")
def torch_cuda():
    import torch

    if not torch.cuda.is_available():
        pytest.fail("GPU tests need an MI355X (torch.cuda.is_available() is False)")
    return torch
