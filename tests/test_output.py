"""Output step: main.c:66-79 normalisation + rectangle.c saveAs_core tone map and
floor tint, on the GPU, byte-identical to the reference.

  reference saveAs() (oracle/_ref/out_ref, tests/golden/output_ref.json) == oracle/out_oracle.c   (CPU)
  oracle == fmgi_output_tiles on the GPU                                                         (GPU)
"""
import hashlib
import json
import os

import numpy as np
import pytest

import fm_oracle as O
import fmgi
from conftest import GOLDEN
from fmgi import scene


def _sha(a):
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()


def _gi_input(sc):
    offs = np.load(os.path.join(GOLDEN, "glibc_rand_4096.npy"))
    lm, _ = O.bake(sc, O.schedule_with_offsets(sc, 65_000, offs))
    fx = np.zeros((sc.num_texels, 4), np.int64)
    fx[:, :3] = lm
    return O.finalize(fx, np.zeros((sc.num_texels, 4), np.float32))


def _case(name, example_scene):
    if name == "gi_example":
        return example_scene, _gi_input(example_scene)
    box8 = scene.box_scene(8)
    return box8, O.ambient_occlusion(box8)


@pytest.mark.parametrize("name", ["gi_example", "ao_box8"])
def test_oracle_reproduces_reference_output(name, example_scene):
    ref = json.load(open(os.path.join(GOLDEN, "output_ref.json")))[name]
    sc, tex = _case(name, example_scene)
    assert _sha(tex) == ref["input_sha256"]
    norm, rgb = O.output_tiles(sc, tex, ref["spa"], ref["tint_extra"])
    assert rgb.size == ref["rgb_bytes"]
    assert _sha(rgb) == ref["rgb_sha256"]
    assert _sha(norm) == ref["texels_sha256"]


@pytest.mark.gpu
@pytest.mark.parametrize("name", ["gi_example", "ao_box8"])
def test_gpu_output_equals_reference(torch_cuda, name, example_scene):
    ref = json.load(open(os.path.join(GOLDEN, "output_ref.json")))[name]
    sc, tex = _case(name, example_scene)
    norm, rgb = fmgi.output_tiles(sc, tex, ref["spa"], ref["tint_extra"])
    assert _sha(rgb) == ref["rgb_sha256"]
    assert _sha(norm) == ref["texels_sha256"]


@pytest.mark.gpu
@pytest.mark.parametrize("tint", [0, 1])
def test_gpu_output_random_texels_bytewise(torch_cuda, tint, box200):
    """Random texels over 9 decades (and exact zeros: 0/0 in the tone map) on the box200 walls, which
    include floor walls: GPU bytes == oracle bytes, normalised texels bit for bit."""
    rng = np.random.default_rng(11 + tint)
    tex = (10.0 ** rng.uniform(-6, 3, (box200.num_texels, 4))).astype(np.float32)
    tex[rng.random(box200.num_texels) < 0.01] = 0
    for spa in (0, 172_413_793):
        n_o, rgb_o = O.output_tiles(box200, tex, spa, tint)
        n_g, rgb_g = fmgi.output_tiles(box200, tex, spa, tint)
        assert np.array_equal(rgb_g, rgb_o), int((rgb_g != rgb_o).sum())
        assert np.array_equal(n_g.view(np.uint32), n_o.view(np.uint32))
