"""Radiosity backend: performRadiosityNative (radiosityNative.c:92-268) on the GPU.

  reference (oracle/_ref/rad_ref, tests/golden/rad_ref.json) == oracle/rad_oracle.c          (CPU)
  the jump-matrix rand() skip == libc rand() (any seed, any position)                         (CPU)
  GPU texels == reference fixture; GPU sourceTexelIds == oracle; libc stream left in place   (GPU)

The fixtures hold the reference's texels for small box scenes (tile_size 2 texels/m², 832 level-0
texels: 8.3 M rays) and for the example.png geometry (85,056 level-0 texels: 851 M rays), each with the
rand() value the reference's process draws next. Parity is bit-exact (DESIGN.md §9 bounds the one
source that could break it: device vs glibc double cos/sin, measured exhaustively)."""
import hashlib
import json
import os

import numpy as np
import pytest

import fm_oracle as O
import fmgi
from conftest import GOLDEN
from fmgi import _lib, scene


def _sha(a):
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()


def _fixtures():
    return json.load(open(os.path.join(GOLDEN, "rad_ref.json")))


def _scene(name, example_scene=None):
    if name == "example":
        return example_scene
    return {"box200_t2_lit": lambda: scene.box_scene(200, tile_size=2.0, with_light=True),
            "box200_t2": lambda: scene.box_scene(200, tile_size=2.0)}[name]()


@pytest.mark.parametrize("name", ["box200_t2_lit", "box200_t2"])
def test_oracle_reproduces_reference(name, libc):
    ref = _fixtures()[name]
    sc = _scene(name)
    libc.srand(ref["seed"])
    tex = O.radiosity(sc)
    assert libc.rand() == ref["next_rand"]
    first = [float(tex[int(w["lm"][0]), 0]) for w in sc.walls]
    assert first == ref["first_texel_per_wall"]
    assert _sha(tex) == ref["sha256_f32"]


@pytest.mark.parametrize("seed,pre,n", [(1, 0, 0), (1, 0, 1), (1, 0, 30), (1, 0, 31), (7, 5, 1000),
                                        (3, 12345, 20000 * 832 + 7), (99, 3, 2 ** 33 + 5)])
def test_rand_skip_matches_libc(libc, seed, pre, n):
    """The jump matrices the device replay is built on: skipping n draws == n rand() calls."""
    lib = _lib.load()
    libc.srand(seed)
    for _ in range(pre):
        libc.rand()
    if n < 10 ** 8:
        for _ in range(n):
            libc.rand()
        want = [libc.rand() for _ in range(3)]
        libc.srand(seed)
        for _ in range(pre):
            libc.rand()
        assert lib.fmgi_rand_skip(n) == 0
        assert [libc.rand() for _ in range(3)] == want
    else:  # too long to draw: skip in two different splits and compare
        assert lib.fmgi_rand_skip(n) == 0
        a = [libc.rand() for _ in range(3)]
        libc.srand(seed)
        for _ in range(pre):
            libc.rand()
        assert lib.fmgi_rand_skip(n // 2) == 0 and lib.fmgi_rand_skip(n - n // 2) == 0
        assert [libc.rand() for _ in range(3)] == a


@pytest.mark.gpu
@pytest.mark.parametrize("name", ["box200_t2_lit", "box200_t2", "example"])
def test_gpu_equals_reference(torch_cuda, libc, name, example_scene):
    ref = _fixtures().get(name)
    if ref is None:
        pytest.skip(f"no reference fixture for {name}")
    sc = _scene(name, example_scene)
    libc.srand(ref["seed"])
    tex = fmgi.radiosity(sc)
    assert libc.rand() == ref["next_rand"], "the libc stream must be left where the reference leaves it"
    first = [float(tex[int(w["lm"][0]), 0]) for w in sc.walls]
    bad = [i for i, (a, b) in enumerate(zip(first, ref["first_texel_per_wall"])) if a != b]
    assert not bad, f"walls {bad[:10]} differ"
    assert _sha(tex) == ref["sha256_f32"]
    st = fmgi.radiosity_stats()
    assert st["rays"] == st["jobs"] * 10000


@pytest.mark.gpu
def test_gpu_source_texels_equal_oracle_mid_stream(torch_cuda, libc):
    """sourceTexelIds bit for bit, starting from an arbitrary libc position (seed 5, 777 draws in)."""
    sc = scene.box_scene(200, tile_size=2.0, with_light=True)
    libc.srand(5)
    for _ in range(777):
        libc.rand()
    t_o, s_o = O.radiosity(sc, with_sids=True)
    nxt = libc.rand()
    libc.srand(5)
    for _ in range(777):
        libc.rand()
    t_g, s_g = fmgi.radiosity(sc, with_sids=True)
    assert libc.rand() == nxt
    assert np.array_equal(s_g, s_o), int((s_g != s_o).sum())
    assert (s_g >= 0).all(), "a closed box: every ray lands on a texel"
    assert np.array_equal(t_g.view(np.uint32), t_o.view(np.uint32))


@pytest.mark.gpu
def test_gpu_chunked_rand_replay(torch_cuda, libc, monkeypatch):
    """Jobs split into chunks of 37 for the device rand() replay: same texels."""
    sc = scene.box_scene(200, tile_size=2.0, with_light=True)
    ref = _fixtures()["box200_t2_lit"]
    monkeypatch.setenv("FMGI_RAD_CHUNK", "37")
    libc.srand(ref["seed"])
    tex = fmgi.radiosity(sc)
    assert libc.rand() == ref["next_rand"]
    assert _sha(tex) == ref["sha256_f32"]


@pytest.mark.gpu
def test_gpu_edge_scenes(torch_cuda, libc):
    """No light sources: every texel stays 0 and the rays still draw rand(). No walls: nothing drawn."""
    sc = scene.box_scene(8, tile_size=1.0)
    dark = scene.Scene("dark", sc.walls, sc.windows[:0], sc.lights[:0], sc.num_texels)
    libc.srand(1)
    t_o = O.radiosity(dark)
    nxt = libc.rand()
    libc.srand(1)
    t_g = fmgi.radiosity(dark)
    assert libc.rand() == nxt
    assert not t_g.any() and np.array_equal(t_g.view(np.uint32), t_o.view(np.uint32))
    empty = scene.Scene("empty", sc.walls[:0], sc.windows, sc.lights, 0)
    libc.srand(1)
    first = libc.rand()
    libc.srand(1)
    assert fmgi.radiosity(empty).shape == (0, 4)
    assert libc.rand() == first
