"""The drop-in entry points across calls (GPU): cached device state, libc rand() state types, and scenes
whose scan image does not fit in LDS.

  - performGlobalIlluminationCl / getGlobalIlluminationCl keep contexts, scene tables and buffers per
    geometry across calls (fmgi_api.cpp DropinShard): repeated, interleaved and uncached
    (FMGI_DROPIN_CACHE=0) calls give exactly the oracle's texels for the rand() values each consumes;
  - the rand() state guard handles glibc's other generator types (initstate with 32-/256-byte arrays):
    the caller's generator continues exactly as after the reference's calls, and nothing outside the
    caller's array is written;
  - a scene of 6,000 shelves (thousands of planes; neither LDS scan image fits) bakes through the exact
    scan with the oracle's lightmap.
"""
import ctypes as C
import os

import numpy as np
import pytest

import fm_oracle as O
import fmgi
from conftest import GOLDEN
from fmgi import scene

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def golden():
    return np.load(os.path.join(GOLDEN, "glibc_rand_4096.npy"))


def _expected(sc, spa, offsets, tin=None):
    L = O.schedule_with_offsets(sc, spa, offsets)
    olm, _ = O.bake(sc, L)
    return O.finalize(olm, sc.texels() if tin is None else tin), len(L)


def test_repeated_and_interleaved_calls_use_the_cache_exactly(torch_cuda, example_scene, box200, libc, golden):
    spa_ex, spa_box = 65_000, 2_000_000
    fmgi.dropin_release()
    libc.srand(1)
    seen = 0
    for sc, spa in ((example_scene, spa_ex), (example_scene, spa_ex), (box200, spa_box), (example_scene, spa_ex)):
        out = fmgi.bake_geometry(sc, spa)
        exp, nl = _expected(sc, spa, golden[seen:])
        assert np.array_equal(out.view(np.uint32), exp.view(np.uint32)), (sc.name, seen)
        seen += nl
    assert libc.rand() == golden[seen]
    os.environ["FMGI_DROPIN_CACHE"] = "0"
    try:
        libc.srand(1)
        out = fmgi.bake_geometry(example_scene, spa_ex)
    finally:
        os.environ.pop("FMGI_DROPIN_CACHE", None)
    exp, _ = _expected(example_scene, spa_ex, golden)
    assert np.array_equal(out.view(np.uint32), exp.view(np.uint32))
    fmgi.dropin_release()


@pytest.mark.parametrize("state_bytes", [32, 64, 256])
def test_rand_state_of_other_glibc_types_is_restored(torch_cuda, example_scene, state_bytes):
    """initstate() with a 32-/64-/256-byte array selects glibc's TYPE_1/2/4 generator; the call consumes
    one rand() per launch from it (global_illumination_cl.c:251) and restores exactly that array."""
    libc = C.CDLL(None)
    libc.rand.restype = C.c_int
    libc.initstate.restype = C.c_void_p
    libc.initstate.argtypes = [C.c_uint, C.c_void_p, C.c_size_t]
    libc.setstate.restype = C.c_void_p
    libc.setstate.argtypes = [C.c_void_p]
    buf = (C.c_char * (state_bytes + 64))()
    canary = b"\xa5" * 64
    C.memmove(C.addressof(buf) + state_bytes, canary, 64)
    prev = libc.initstate(12345, buf, state_bytes)
    try:
        draws = [libc.rand() for _ in range(40)]
        libc.initstate(12345, buf, state_bytes)
        spa = 65_000
        out = fmgi.bake_geometry(example_scene, spa)
        after = libc.rand()
    finally:
        libc.setstate(prev)
    exp, nl = _expected(example_scene, spa, np.array(draws, np.int32))
    assert np.array_equal(out.view(np.uint32), exp.view(np.uint32))
    assert after == draws[nl]
    assert bytes(buf)[state_bytes:] == canary


def test_scene_too_large_for_lds_bakes_exactly(torch_cuda, golden):
    sc = scene.shelves_scene(6000)
    ctx = fmgi.Context(0)
    ctx.set_scene(sc)
    assert ctx.auto_kernel == fmgi.KERNEL_EXACT
    spa = 2_000_000
    ctx.plan(spa, rng_offsets=golden)
    L = O.schedule_with_offsets(sc, spa, golden)
    olm, _ = O.bake(sc, L, 0, 256)
    for kernel in (fmgi.KERNEL_AUTO, fmgi.KERNEL_FAST, fmgi.KERNEL_GRID):  # the LDS scans fall back too
        s = torch_cuda.cuda.Stream()
        with torch_cuda.cuda.stream(s):
            lm = torch_cuda.zeros((sc.num_texels, 4), dtype=torch_cuda.int64, device="cuda")
            ctx.bake_items(0, 256, lm.data_ptr(), kernel, s.cuda_stream)
        s.synchronize()
        assert np.array_equal(lm.cpu().numpy()[:, :3], olm), kernel
    ctx.close()
