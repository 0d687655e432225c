"""Ambient-occlusion backend: performAmbientOcclusionNative (photonmap.c:435-490)
on the GPU, bit-identical to the reference.

Chain of parity:
  reference (compiled from /root/reference by oracle/build_ref.sh, oracle/_ref/ao_ref)
    == oracle restatement (oracle/ao_oracle.c)     CPU, against tests/golden/ao_ref.json
    == HIP backend (libflatmatch_gi.so)            GPU, against the oracle
and for the direction table: reference geoSphere.c == oracle/geosphere.py (oracle/geosphere_check.py,
tests/golden/geosphere.json) == the product's generator (csrc/fmgi_geosphere.h)."""
import hashlib
import json
import os

import numpy as np
import pytest

import fm_oracle as O
import fmgi
from conftest import GOLDEN
from fmgi import scene

import geosphere


def _scene(name, example_scene, box200):
    return {"box8": scene.box_scene(8), "example": example_scene, "box200": box200}[name]


@pytest.mark.parametrize("level", [3, 4, 5])
def test_direction_tables_match_the_reference(level):
    ref = json.load(open(os.path.join(GOLDEN, "geosphere.json")))[str(level)]
    mine = fmgi.geosphere(level)
    oracle = geosphere.generate(level)
    assert len(mine) == ref["count"]
    assert np.array_equal(mine.view(np.uint32), oracle.view(np.uint32))
    assert hashlib.sha256(mine.tobytes()).hexdigest() == ref["sha256_f32"]


@pytest.mark.parametrize("name", ["box8", "example"])
def test_oracle_reproduces_reference_ao(name, example_scene, box200):
    """The restatement equals the reference's own performAmbientOcclusionNative bit for bit."""
    ref = json.load(open(os.path.join(GOLDEN, "ao_ref.json")))[name]
    sc = _scene(name, example_scene, box200)
    tex = O.ambient_occlusion(sc)
    first = [float(tex[int(w["lm"][0]), 0]) for w in sc.walls]
    assert first == ref["first_texel_per_wall"]
    assert hashlib.sha256(tex.tobytes()).hexdigest() == ref["sha256_f32"]


@pytest.mark.parametrize("name", ["box8", "example", "box200", "box2000"])
def test_product_bsp_equals_oracle_bsp(name, example_scene, box200, box2000):
    sc = {"box8": scene.box_scene(8), "example": example_scene, "box200": box200, "box2000": box2000}[name]
    assert np.array_equal(fmgi.ao_tree(sc), O.ao_tree(sc))


def test_ao_without_device_fails_cleanly(box200):
    """No GPU in this container: the non-mutating entry point reports FMGI_ERR_NO_DEVICE."""
    import torch

    if torch.cuda.is_available():
        pytest.skip("a device is visible")
    with pytest.raises(fmgi.FmgiError):
        fmgi.ambient_occlusion(scene.box_scene(8))


@pytest.mark.gpu
@pytest.mark.parametrize("name", ["box8", "example", "box200"])
def test_gpu_ao_bitwise_equals_oracle(torch_cuda, name, example_scene, box200):
    sc = _scene(name, example_scene, box200)
    got = fmgi.ambient_occlusion(sc)
    exp = O.ambient_occlusion(sc)
    bad = (got.view(np.uint32) != exp.view(np.uint32)).any(axis=1)
    assert not bad.any(), f"{int(bad.sum())} texels differ, first {np.nonzero(bad)[0][:5]}"
    if name in ("box8", "example"):
        ref = json.load(open(os.path.join(GOLDEN, "ao_ref.json")))[name]
        assert hashlib.sha256(got.tobytes()).hexdigest() == ref["sha256_f32"]


@pytest.mark.gpu
def test_gpu_ao_wall_range_and_in_place(torch_cuda, example_scene):
    sc = example_scene
    base = np.random.default_rng(3).random((sc.num_texels, 4), dtype=np.float32)
    part = fmgi.ambient_occlusion(sc, 10, 40, texels=base)
    full = fmgi.ambient_occlusion(sc, texels=base)
    mask = np.zeros(sc.num_texels, bool)
    for w in sc.walls[10:40]:
        mask[w["lm"][0] : w["lm"][0] + w["lm"][1] * w["lm"][2]] = True
    assert np.array_equal(part[mask], full[mask])
    assert np.array_equal(part[~mask], base[~mask])
    # performAmbientOcclusionGpu updates geo->texels in place with the same bits
    tex = base.copy()
    g, keep = fmgi.make_geometry(sc, tex)
    import ctypes as C

    fmgi._lib.load().performAmbientOcclusionGpu(C.byref(g))
    assert np.array_equal(tex.view(np.uint32), full.view(np.uint32))
