"""CPU tests of the oracle (oracle/fm_oracle.c) against golden fixtures and the reference's own
measured facts, plus the oracle's internal consistency."""
import hashlib
import json
import os

import numpy as np
import pytest

import fm_oracle as O
from conftest import GOLDEN

# (scene, spa, launches, photons) measured from the reference host formula (global_illumination_cl.c:220-222,255)
SCHEDULE_FACTS = [
    ("example", 65_000, 10, 1_100_800),
    ("example", 6_500_000, 43, 100_121_600),
    ("box200", 172_413_793, 391, 1_000_012_800),
    ("box200", 1_724_137_931, 3_907, 10_000_025_600),
]


def _scene(name, example_scene, box200):
    return {"example": example_scene, "box200": box200}[name]


@pytest.mark.parametrize("name,spa,nl,photons", SCHEDULE_FACTS)
def test_schedule_matches_reference_counts(name, spa, nl, photons, example_scene, box200, libc):
    sc = _scene(name, example_scene, box200)
    L = O.schedule(sc, spa)
    assert len(L) == nl
    assert int(L["count"].sum()) * 100 == photons
    # launches tile the flattened item list with <= WG*100 items each; window launches come first
    assert np.all(L["count"] <= 25_600)
    assert np.array_equal(np.cumsum(L["count"])[:-1], L["item_begin"][1:])
    isw = L["is_window"].astype(bool)
    assert not np.any(np.diff(isw.astype(int)) > 0)


def test_schedule_consumes_glibc_rand_in_order(example_scene, libc):
    golden = np.load(os.path.join(GOLDEN, "glibc_rand_4096.npy"))
    L = O.schedule(example_scene, 6_500_000)
    assert np.array_equal(L["rng_offset"], golden[: len(L)])
    assert libc.rand() == golden[len(L)]  # exactly one rand() per launch


def test_glibc_rand_prefix_matches_fixture(libc):
    golden = np.load(os.path.join(GOLDEN, "glibc_rand_4096.npy"))
    vals = np.array([libc.rand() for _ in range(len(golden))], np.int32)
    assert np.array_equal(vals, golden)
    assert golden[0] == 1804289383


def test_rand_is_lcg_over_2pow32():
    # photonmap.cl:21-25: s = s*1664525 + 1013904223; return (float)s / (float)0xFFFFFFFF
    s = 12345
    got = O.rand_sequence(s, 8)
    exp = []
    for _ in range(8):
        s = (s * 1664525 + 1013904223) & 0xFFFFFFFF
        exp.append(np.float32(s) / np.float32(4294967296.0))
    assert np.array_equal(got, np.array(exp, np.float32))
    # (float)0xFFFFFFFF rounds to 2^32, so the maximum draw is exactly 1.0
    assert np.float32(0xFFFFFFFF) == np.float32(2**32)


def test_config1_regression(example_scene, libc):
    ref = json.load(open(os.path.join(GOLDEN, "oracle_config1.json")))
    L = O.schedule(example_scene, 65_000)
    assert [list(x) for x in L.tolist()] == ref["launches"]
    lm, st = O.bake(example_scene, L)
    assert st == ref["stats"]
    assert st["inexact"] == 0  # every deposit channel is a multiple of 2^-25
    assert hashlib.sha256(np.ascontiguousarray(lm).tobytes()).hexdigest() == ref["lightmap_sha256"]


def test_bake_is_thread_count_and_split_invariant(box200, libc):
    L = O.schedule(box200, 172_413_793)
    a, sa = O.bake(box200, L, 0, 600, nthreads=1)
    b, sb = O.bake(box200, L, 0, 600, nthreads=8)
    c1, _ = O.bake(box200, L, 0, 250)
    c2, _ = O.bake(box200, L, 250, 600)
    assert np.array_equal(a, b) and sa == sb
    assert np.array_equal(a, c1 + c2)


def test_box_is_closed(box200, libc):
    L = O.schedule(box200, 172_413_793)
    lm, st = O.bake(box200, L, 0, 200)
    # a closed box: photons (almost) never escape and bounce MAX_DEPTH=8 times (photonmap.cl:171)
    assert st["escapes"] <= 2
    assert st["deposits"] >= 8 * st["photons"] - 16
    # deposits land only on level-0 texels (mip levels are written by the caller's mipmap step)
    lvl0 = box200.level0_mask()
    assert not lm[~lvl0].any()


def test_trace_events_sum_to_lightmap(example_scene, libc):
    L = O.schedule(example_scene, 65_000)
    ev, fin = O.trace_item(example_scene, int(L[0]["source"]), 1, int(L[0]["rng_offset"]) + 5)
    lm, _ = O.bake(example_scene, L, 5, 6)
    acc = np.zeros_like(lm)
    for e in ev:
        acc[e["texel"]] += (e["rgb"].astype(np.float64) * 2**25).astype(np.int64)
    assert np.array_equal(acc, lm)
    assert np.all(np.diff(ev["photon"]) >= 0) and ev["photon"].max() <= 99


def test_f32_item_matches_fixed_point_when_no_rounding(example_scene, libc):
    L = O.schedule(example_scene, 65_000)
    st = int(L[0]["rng_offset"]) + 7
    tex = O.trace_item_f32(example_scene, int(L[0]["source"]), 1, st)
    lm, _ = O.bake(example_scene, L, 7, 8)
    # the f32 sequential sum equals the exact sum up to fp32 rounding of the additions
    np.testing.assert_allclose(tex[:, :3], lm / 2**25, rtol=2e-7, atol=0)


def test_port_build_is_bit_identical_to_the_oracle(box200, example_scene, libc):
    """liboracle_port.so (bench.py's CPU baseline: per-rect builtin values hoisted out of the scan, FMA
    instructions) computes exactly the oracle's lightmap and counters."""
    for sc, spa, (b, e) in ((box200, 172_413_793, (0, 700)), (example_scene, 65_000, (9_000, 11_008))):
        L = O.schedule(sc, spa)
        a, sa = O.bake(sc, L, b, e)
        p, sp = O.bake_port(sc, L, b, e)
        assert np.array_equal(a, p) and sa == sp, sc.name
