"""CPU test of FMGI_KERNEL_HYBRID's wall-pair image (host-only context; no device needed).

The hybrid scan tests the walls two records per packed iteration (csrc/fmgi_kernels.hip filter_pairs) over the
pair image fmgi_set_scene builds (fmgi_api.cpp build_filter_pairs). Its keys and candidate tests equal the
one-record filter loop's only if the image holds, for every axis, group and class, records 2g and 2g + 1 of
that class exactly as the filter image does (same floats, same rect index), and never-valid sentinels where
the class has no such record. This replays that mapping for the reference's own layout, the generated
30-room layout and a synthetic box."""
import os

import numpy as np
import pytest

import fmgi
from conftest import GOLDEN
from fmgi import scene


def _images(sc):
    ctx = fmgi.Context(-1)
    ctx.set_scene(sc)
    fimg, pimg = ctx.filter_image(), ctx.pair_image()
    ctx.close()
    return fimg, pimg


@pytest.mark.parametrize("name", ["example", "apartment30", "box200"])
def test_pair_image_holds_the_filter_records(name):
    if name == "box200":
        sc = scene.box_scene(200)
    else:
        sc = scene.load_geometry(os.path.join(GOLDEN, f"{name}_geometry.bin"), name)
    fimg, pimg = _images(sc)
    J, G = fimg["J"], pimg["G"]
    recs, halves = fimg["recs"], pimg["halves"]
    assert halves.shape[0] == 2 * (G[0] + G[1])
    base_f, base_p = 0, 0  # first filter pair / first pair-image half of the axis
    for a in range(2):
        assert G[a] == (J[a] + 1) // 2
        for g in range(G[a]):
            for c in range(2):
                h = halves[base_p + 2 * g + c]
                hidx = h[10:12].view(np.int32)
                for k in range(2):
                    j = 2 * g + k
                    got = (h[0 + k], h[2 + k], h[4 + k], h[6 + k], h[8 + k], int(hidx[k]))
                    if j < J[a]:
                        r = recs[2 * (base_f + j) + c]  # pair j of the axis, class-c half
                        want = (r[0], r[1], r[2], r[3], r[4], int(r[5:6].view(np.int32)[0]))
                        if want[5] >= 0:
                            assert got == want, (name, a, g, c, k)
                            continue
                    # no record: never a candidate (|x| <= -1 is false) and no rect
                    assert got[2] == -1.0 and got[4] == -1.0 and got[5] == -1, (name, a, g, c, k)
        base_f += J[a]
        base_p += 2 * G[a]
    # every axis-aligned x / y wall appears exactly once
    idx = pimg["idx"].ravel()
    idx = idx[idx >= 0]
    assert len(idx) == len(set(idx.tolist()))
    walls = fimg["idx"][: 2 * (J[0] + J[1])]
    assert sorted(idx.tolist()) == sorted(walls[walls >= 0].tolist())
