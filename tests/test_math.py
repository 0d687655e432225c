"""The samplers' sin/cos (csrc/fmgi_math.h) on every reachable input, and the roulette threshold.

photonmap.cl:33,57 draw phi = 6.283184f * rand() with rand() = (float)s * 2^-32 (photonmap.cl:21-25), so
phi takes 83,886,081 distinct values. On the MI355X the reference's sin/cos come from ROCm's device
library (ocml.bc __ocml_sin_f32 / __ocml_cos_f32, fp32, not correctly rounded); the product and the
oracle restate that algorithm independently. Here (CPU): product restatement == oracle restatement on
every reachable phi, and both equal the device library's own results as recorded on the MI355X
(tests/golden/ocml_sincos.json: SHA-256 of all 2 x 83,886,081 result bits). The GPU twin
(test_gpu_parity.py) checks the device restatement against the device library directly."""
import hashlib
import json
import os

import numpy as np

import fm_oracle as O
import fmgi
from conftest import GOLDEN


def _digest(s, c):
    return hashlib.sha256(s.view(np.uint32).tobytes() + c.view(np.uint32).tobytes()).hexdigest()


def test_sincos_restatements_agree_on_every_reachable_phi_and_match_the_device_library():
    phi = O.reachable_phi()
    assert len(phi) == 83_886_081
    hs, hc = fmgi.host_sincosf(phi)
    os_, oc = O.sincos(phi)
    assert np.array_equal(hs.view(np.uint32), os_.view(np.uint32))
    assert np.array_equal(hc.view(np.uint32), oc.view(np.uint32))
    golden = json.load(open(os.path.join(GOLDEN, "ocml_sincos.json")))
    assert golden["inputs"] == len(phi)
    assert _digest(hs, hc) == golden["sha256_sin_cos_bits"]


def test_device_library_sincos_is_not_correctly_rounded():
    """Why the contract names the library: its fp32 sin/cos differ from the correctly rounded values
    (float)sin((double)phi) on a sizeable share of inputs (~17 % of the reachable phi, mostly by 1 ulp)."""
    phi = O.reachable_phi()[::97]
    s, c = fmgi.host_sincosf(phi)
    es = np.sin(phi.astype(np.float64)).astype(np.float32)
    ec = np.cos(phi.astype(np.float64)).astype(np.float32)
    differ = (s != es) | (c != ec)
    assert 0.05 < differ.mean() < 0.4
    ulps = np.abs(s.view(np.int32).astype(np.int64) - es.view(np.int32).astype(np.int64))
    assert ulps.max() <= 4


def test_roulette_threshold_is_the_double_comparison():
    """k_bake tests photonmap.cl:236's `(double)pos.z > 0.0005` as `pos.z > c` with c the largest float
    below 0.0005: the two agree on every float (checked on the floats around the threshold and signs)."""
    c = np.float32(4.99999965541064739227294921875e-4)
    assert float(c) < 0.0005 < float(np.nextafter(c, np.float32(1)))
    z = c.view(np.uint32) + np.arange(-4096, 4097, dtype=np.int64)
    zf = np.concatenate([z.astype(np.uint32).view(np.float32), [0.0, -0.0, -c, 1.0, 1e-5, np.inf]]).astype(np.float32)
    assert np.array_equal(zf.astype(np.float64) > 0.0005, zf > c)
