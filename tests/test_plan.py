"""CPU tests of FMGI_KERNEL_HYBRID's floor plan of the walls (host-only context; no device needed).

The hybrid scan's wall pass (csrc/fmgi_kernels.hip plan_walls) tests only the walls listed in the floor-plan
cells its ray crosses, nearest cell first, and stops once the ray leaves a cell past the 2^-11 band above
its best key. It keeps the filter pass's results only if every wall that passes the filter's test with a
key inside that band is listed in some cell the walk visits (fmgi_api.cpp build_plan). Here the walk is
replayed in float32 with the kernel's operation order, on random rays and on rays aimed at wall ends and
corners, against the filter's brute-force test over every wall."""
import os

import numpy as np
import pytest

import fmgi
from conftest import GOLDEN
from fmgi import scene

F = np.float32
BAND = F(1.00048828125)


def _fma(a, b, c):
    return F(np.float64(a) * np.float64(b) + np.float64(c))


def _tables(sc):
    ctx = fmgi.Context(-1)
    ctx.set_scene(sc)
    plan, fimg = ctx.plan_tables(), ctx.filter_image()
    ctx.close()
    return plan, fimg


def _wall_records(sc, fimg):
    """record index r of the filter image -> (axis, class, plane, cu, hwu, cv, hwv) for every wall record"""
    J0, J1 = fimg["J"][0], fimg["J"][1]
    recs = {}
    for r in range(2 * (J0 + J1)):
        if fimg["idx"][r] < 0:
            continue
        q = fimg["recs"][r]
        recs[r] = (0 if r < 2 * J0 else 1, r & 1) + tuple(F(x) for x in q[:5])
    return recs, J0


def _walk(plan, recs, J0, s, d, L1):
    """the kernel's plan_walls on one ray: the records it tests (faced class only) and the final L1"""
    x0, y0, cs = F(plan["x0"]), F(plan["y0"]), F(plan["cs"])
    ics = F(plan["ics"])
    nx, ny = plan["nx"], plan["ny"]
    st, en = plan["start"], plan["entry"]
    rx = F(1) / d[0] if d[0] != 0 else F(np.inf)
    ry = F(1) / d[1] if d[1] != 0 else F(np.inf)
    cx, cy = (0 if d[0] < 0 else 1), (0 if d[1] < 0 else 1)
    ix = int(min(max(np.floor((s[0] - x0) * ics), F(0)), F(nx - 1)))
    iy = int(min(max(np.floor((s[1] - y0) * ics), F(0)), F(ny - 1)))
    sx, sy = (1 if d[0] > 0 else -1), (1 if d[1] > 0 else -1)
    tested = set()
    for _ in range(nx + ny):
        cell = iy * nx + ix
        for k in range(int(st[cell]), int(st[cell + 1])):
            r = int(en[k])
            a, c = recs[r][0], recs[r][1]
            if c != (cy if a == 1 else cx):
                continue
            tested.add(r)
            ok, f = _test(recs[r], s, d)
            if ok and f < L1:
                L1 = f
        tx = F(np.inf) if d[0] == 0 else (_fma(F(ix + cx), cs, x0) - s[0]) * rx
        ty = F(np.inf) if d[1] == 0 else (_fma(F(iy + cy), cs, y0) - s[1]) * ry
        alongx = tx < ty
        te = tx if alongx else ty
        if not (te <= L1 * BAND):
            break
        if alongx:
            ix += sx
            if not 0 <= ix < nx:
                break
        else:
            iy += sy
            if not 0 <= iy < ny:
                break
    return tested, L1


def _test(rec, s, d):
    """filter_axis's test of one record: (ok, key)"""
    a, c, plane, cu, hwu, cv, hwv = rec
    u = 1 if a == 0 else 0
    rd = F(1) / d[a] if d[a] != 0 else F(np.copysign(np.inf, d[a]))
    with np.errstate(invalid="ignore", over="ignore"):
        f = (plane - s[a]) * rd
        uu = _fma(d[u], f, s[u]) - cu
        vv = _fma(d[2], f, s[2]) - cv
    faced = c == (0 if d[a] < 0 else 1)
    return bool(faced and f >= 0 and abs(uu) <= hwu and abs(vv) <= hwv), f


def _rays(sc, recs, rng, n_random, n_aimed):
    lo = np.min([r[2] for r in recs.values()])
    walls = list(recs.values())
    xs = [r[2] for r in walls if r[0] == 0] + [r[3] - r[4] for r in walls if r[0] == 1] + [r[3] + r[4] for r in walls if r[0] == 1]
    ys = [r[2] for r in walls if r[0] == 1] + [r[3] - r[4] for r in walls if r[0] == 0] + [r[3] + r[4] for r in walls if r[0] == 0]
    box = (min(xs), max(xs), min(ys), max(ys))
    out = []
    for _ in range(n_random):
        s = np.array([rng.uniform(box[0], box[1]), rng.uniform(box[2], box[3]), rng.uniform(0.05, 2.5)], F)
        d = rng.normal(size=3)
        out.append((s, (d / np.linalg.norm(d)).astype(F)))
    for _ in range(n_aimed):  # at a wall's end or corner, from a random point
        r = walls[rng.integers(len(walls))]
        a, plane, cu, hwu, cv, hwv = r[0], r[2], r[3], r[4], r[5], r[6]
        eu = cu + rng.choice([-1, 1]) * hwu * F(rng.choice([1.0, 0.999, 1.001]))
        ev = cv + rng.choice([-1, 1, 0]) * hwv
        t = np.array([plane, eu, ev] if a == 0 else [eu, plane, ev], F)
        s = np.array([rng.uniform(box[0], box[1]), rng.uniform(box[2], box[3]), rng.uniform(0.05, 2.5)], F)
        d = (t - s).astype(np.float64)
        if np.linalg.norm(d) < 1e-3:
            continue
        out.append((s, (d / np.linalg.norm(d)).astype(F)))
    del lo
    return out


@pytest.mark.parametrize("name", ["example", "apartment30"])
def test_plan_walk_finds_every_wall_inside_the_band(name, example_scene):
    sc = example_scene if name == "example" else scene.load_geometry(os.path.join(GOLDEN, "apartment30_geometry.bin"), "a30")
    plan, grid = _tables(sc)
    assert plan is not None, "a layout gets a floor plan"
    recs, J0 = _wall_records(sc, grid)
    assert set(int(r) for r in plan["entry"]) <= set(recs), "an entry that is not a wall record"
    assert len(plan["start"]) == plan["nx"] * plan["ny"] + 1 and int(plan["start"][-1]) == len(plan["entry"])
    rng = np.random.default_rng(3)
    missed = 0
    checked = 0
    for s, d in _rays(sc, recs, rng, 1500, 1500):
        floor_key = F(rng.choice([np.inf, rng.uniform(0.2, 12.0)]))
        res = {r: _test(rec, s, d) for r, rec in recs.items()}
        L1 = min([floor_key] + [f for ok, f in res.values() if ok])
        need = {r for r, (ok, f) in res.items() if ok and f <= L1 * BAND}
        tested, L1w = _walk(plan, recs, J0, s, d, floor_key)
        assert L1w == L1 or not need
        missed += len(need - tested)
        checked += len(need)
    assert checked > 500
    assert missed == 0, f"{missed} of {checked} walls inside the band not visited"


def test_plan_is_small_and_selective(example_scene):
    plan, _ = _tables(example_scene)
    ncells = plan["nx"] * plan["ny"]
    assert ncells <= 4096 and len(plan["entry"]) < 65535
    # a few walls per cell, not the whole layout
    assert len(plan["entry"]) / ncells < 4.0


def test_boxes_have_a_plan_but_use_the_grid(box200):
    """closed boxes run the grid scan (AUTO); their plan, if any, is never walked"""
    ctx = fmgi.Context(-1)
    ctx.set_scene(box200)
    assert ctx.auto_kernel == fmgi.KERNEL_GRID
    ctx.close()
