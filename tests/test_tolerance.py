"""How far the reference's deployed arithmetic moves a whole lightmap from ours (CPU, committed fixtures).

The north star asks for lightmaps "within 1e-4 relative of reference". Ours equal the oracle bit for bit
(tests/test_gpu_*.py), and the oracle equals the reference kernel built strictly (IEEE div/sqrt, no
contraction) item for item (tests/test_reference_pin.py). The reference itself is built with
-cl-fast-relaxed-math (global_illumination_cl.c:196); that build faults on the MI355X, and
-cl-unsafe-math-optimizations ("relaxed") stands for it (tests/golden/make_tolerance_fixtures.py).

tests/golden/ref_launch_<case>.npz hold, for whole reference launch ranges, the race-free sums of the
reference kernel's own per-item fp32 lightmaps (exact, int64 units of 2^-25) minus the oracle's exact sums,
for the strict and the relaxed build. Here the oracle sums are recomputed (their sha256 must match the one
recorded with the fixture), the reference sums rebuilt, and two figures computed per SURVEY §8(c):
  max_rel_ge100  max over level-0 texels with >= 100 deposits of max_c |ref - ours| / ours
  l1_rel         sum |ref - ours| / sum ours over every texel and channel
Strict differs from ours only by the reference's per-item fp32 additions (one work item's deposits on one
texel are added in fp32 before the launch sum); relaxed adds the relaxed math's moved hit points.
"""
import hashlib
import json
import os

import numpy as np
import pytest

import fm_oracle as O
from conftest import GOLDEN

CASES = {"config1": ("example", 65_000), "box200": ("box200", 172_413_793)}
TOL = 1e-4  # BASELINE.json north star: lightmaps within 1e-4 relative of the reference


def _scene(name, example_scene, box200):
    return example_scene if name == "example" else box200


def _metrics(ours, ref, counts, level0):
    a = ours.astype(np.float64)
    d = np.abs(ref.astype(np.float64) - a)
    sel = level0 & (counts >= 100)
    rel = float((d[sel] / np.maximum(a[sel], 1.0)).max()) if sel.any() else 0.0
    return rel, float(d.sum() / max(a.sum(), 1.0)), int(sel.sum())


@pytest.mark.parametrize("case", sorted(CASES))
def test_whole_launch_lightmaps_within_tolerance_of_reference(case, example_scene, box200):
    path = os.path.join(GOLDEN, f"ref_launch_{case}.npz")
    if not os.path.exists(path):
        pytest.skip(f"{path} not generated yet (tests/golden/make_tolerance_fixtures.py on the GPU box)")
    fx = np.load(path)
    scene_name, spa = CASES[case]
    sc = _scene(scene_name, example_scene, box200)
    assert int(fx["spa"]) == spa
    b, e = (int(x) for x in fx["items"])
    offs = np.load(os.path.join(GOLDEN, "glibc_rand_4096.npy"))
    L = O.schedule_with_offsets(sc, spa, offs)
    ours, st, counts = O.bake(sc, L, b, e, counts=True)
    assert hashlib.sha256(ours.tobytes()).hexdigest() == str(fx["oracle_sha256"]), "the oracle changed"
    level0 = sc.level0_mask()
    summary = json.load(open(os.path.join(GOLDEN, "ref_launch_summary.json")))[case]
    mean_dep = ours.astype(np.float64).sum() / (3.0 * st["deposits"])  # one deposit, in 2^-25 units
    for variant in ("strict", "relaxed"):
        ref = ours + fx[f"d_{variant}"]
        assert ref.min() >= 0
        rel, l1, n100 = _metrics(ours, ref, counts, level0)
        rec = summary[variant]
        assert rel == pytest.approx(rec["max_rel_ge100"], rel=1e-9, abs=1e-15), variant
        assert l1 == pytest.approx(rec["l1_rel"], rel=1e-9, abs=1e-15), variant
        assert n100 == rec["texels_ge100"], variant
        d = (ref - ours).astype(np.float64)
        total = abs(d.sum()) / ours.astype(np.float64).sum()  # deposited energy, all texels together
        moved = np.abs(d).sum() / 3.0 / mean_dep / 2.0       # ~ deposits that landed on another texel
        sel = level0 & (counts >= 100)
        texrel = np.abs(d[sel]).max(axis=1) / np.maximum(ours[sel].min(axis=1), 1)
        if variant == "strict":
            # the north star's bound, with five orders of magnitude to spare: only the reference's per-item
            # fp32 additions remain (max 7.6e-9, L1 5.9e-10 on config 1)
            assert rel <= TOL, f"{case}: max relative {rel:.3e} over texels with >= 100 deposits"
            assert l1 <= TOL, f"{case}: L1 relative {l1:.3e}"
            assert moved < 1.0
        else:
            # relaxed math (the deployed build's class) moves a few hit points across texel boundaries and
            # a few bounces onto other walls: the energy total stays (<= 1e-5), < 1e-4 of the deposits land
            # elsewhere (config 1: ~320 of 5.5e6, box200: ~1,800 of 2.0e7), so L1 is 1.2-1.8e-4; the
            # texels that gain or lose one deposit (2-6 % of those with >= 100) move by 1 / their count
            # (<= 1.7e-2), every other texel stays within 1e-4. DESIGN.md §2.
            assert total <= 1e-5, f"{case}: energy total moved by {total:.2e}"
            assert moved <= 1e-4 * st["deposits"], f"{case}: {moved:.0f} deposits moved"
            assert l1 <= 2.5e-4 and rel <= 3e-2, (l1, rel)
            assert (texrel <= 1e-4).mean() >= 0.9
