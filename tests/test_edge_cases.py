"""Edge cases of the drop-in path on the GPU, each against the oracle and the reference's rand() usage
(global_illumination_cl.c:215-272: one rand() per launch, windows then lights):
  - no walls: every photon escapes at its first scan (photonmap.cl:208-209); texels unchanged, but the
    launches (and their rand() calls) still happen;
  - no windows and no lights: no launches, no rand() call, texels unchanged;
  - lights only, windows only;
  - the virtual work-group size (FMGI_WG, the reference's CL_KERNEL_WORK_GROUP_SIZE) at 64 and 1024;
  - the smallest sample count (spa = 1: n = 0 rounds up to one work group per source, :222)."""
import os

import numpy as np
import pytest

import fm_oracle as O
import fmgi
from conftest import GOLDEN
from fmgi import scene

pytestmark = pytest.mark.gpu


def _golden():
    return np.load(os.path.join(GOLDEN, "glibc_rand_4096.npy"))


def _sub(sc, walls=True, windows=True, lights=True):
    empty = sc.walls[:0]
    return scene.Scene(sc.name, sc.walls if walls else empty, sc.windows if windows else empty,
                       sc.lights if lights else empty, sc.num_texels)


def _check(sc, spa, libc, wg=256):
    golden = _golden()
    L = O.schedule_with_offsets(sc, spa, golden, wg)
    tin = np.random.default_rng(5).random((sc.num_texels, 4), dtype=np.float32)
    libc.srand(1)
    if wg != 256:
        os.environ["FMGI_WG"] = str(wg)
    try:
        out = fmgi.bake_geometry(sc, spa, tin)
    finally:
        os.environ.pop("FMGI_WG", None)
    assert libc.rand() == golden[len(L)], "rand() must be consumed once per reference launch"
    if len(sc.walls):
        olm, _ = O.bake(sc, L)
        exp = O.finalize(olm, tin)
    else:
        exp = tin.copy()
    assert np.array_equal(out.view(np.uint32), exp.view(np.uint32))
    return L


def test_no_walls(torch_cuda, example_scene, libc):
    L = _check(_sub(example_scene, walls=False), 65_000, libc)
    assert len(L) == 10


def test_no_light_sources(torch_cuda, example_scene, libc):
    L = _check(_sub(example_scene, windows=False, lights=False), 65_000, libc)
    assert len(L) == 0


def test_lights_only_and_windows_only(torch_cuda, example_scene, libc):
    _check(_sub(example_scene, windows=False), 200_000, libc)
    _check(_sub(example_scene, lights=False), 65_000, libc)


@pytest.mark.parametrize("wg", [64, 1024])
def test_work_group_size(torch_cuda, example_scene, libc, wg):
    _check(example_scene, 65_000, libc, wg)


def test_smallest_sample_count(torch_cuda, example_scene, box200, libc):
    for sc in (example_scene, box200):
        L = _check(sc, 1, libc)
        assert len(L) == len(sc.windows) + len(sc.lights)
