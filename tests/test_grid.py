"""CPU tests of FMGI_KERNEL_GRID's tables (host-only context; no device needed).

ScanGrid (csrc/fmgi_kernels.hip) is exact only if, for every hit point (u, v) on a plane, the grid
cell the kernel computes for (u, v) lists EVERY record of that plane whose margin-grown extent
contains (u, v) -- the candidate set must stay a superset of photonmap.cl's valid set V. Here the
kernel's cell arithmetic is replayed in float32 (IEEE, same operation order) on random points and on
adversarial points at every record's extent boundaries (and one ulp either side). A cell holds its first
two records as quantized bounds of the cell's 16-bit fixed-point coordinates (GridCell): every point that
passes a record's float test must also pass its quantized test, replayed the same way."""
import numpy as np
import pytest

import fmgi


def _tables(sc, cells_per_record=0):
    ctx = fmgi.Context(-1)
    ctx.set_grid_cells_per_record(cells_per_record)
    ctx.set_scene(sc)
    t = ctx.grid_tables()
    f = ctx.filter_image()["recs"]
    ctx.close()
    # every rect's float record {cu, hwu, cv, hwv} (the filter image holds each axis-aligned rect once)
    ids = f[:, 5].copy().view(np.int32)
    t["rec_of"] = {int(i): f[k, 1:5].astype(np.float32) for k, i in enumerate(ids) if i >= 0}
    return t


def _planes(t):
    """(plane record, entries of every cell) for each non-padding plane."""
    out = []
    for p in t["planes"]:
        if np.isnan(p["plane"]):
            continue
        n = int(p["nu"]) * int(p["nv"])
        cells = t["cells"][p["cell_off"] : p["cell_off"] + n]
        out.append((p, cells))
    return out


def _cell_of(p, u, v):
    """The kernel's cell index for hit point (u, v): fminf(fmaxf((x - o) * inv, 0), n - 1), truncated."""
    f32 = np.float32
    assert p["mu"] == p["nu"] - 1 and p["mv"] == p["nv"] - 1
    tu = np.minimum(np.maximum((u - f32(p["u0"])) * f32(p["iu"]), f32(0)), f32(p["mu"]))
    tv = np.minimum(np.maximum((v - f32(p["v0"])) * f32(p["iv"]), f32(0)), f32(p["mv"]))
    return tv.astype(np.int64) * int(p["nu"]) + tu.astype(np.int64)


def _q(p, u, v):
    """The kernel's 16-bit fixed-point coordinates of (u, v) inside its cell (grid_cell)."""
    f32 = np.float32
    out = []
    for x, o, inv, m in ((u, p["u0"], p["iu"], p["mu"]), (v, p["v0"], p["iv"], p["mv"])):
        r = (x - f32(o)) * f32(inv)
        c = np.floor(np.minimum(np.maximum(r, f32(0)), f32(m)))
        q = np.minimum(np.maximum((r - c) * f32(65536), f32(0)), f32(65535))
        out.append(q.astype(np.uint32))
    return out


def _entries(t, c):
    """(records [n, 4], rect indices [n]) of one cell: the inline first two, then the overflow."""
    n = int(c["count"])
    ids = np.array([c["idx0"], c["idx1"]], np.int32)[: min(n, 2)]
    inline = np.array([t["rec_of"][int(i)] for i in ids], np.float32).reshape(-1, 4)
    rest = slice(int(c["rest"]), int(c["rest"]) + max(n - 2, 0))
    return np.concatenate([inline, t["recs"][rest]]), np.concatenate([ids, t["idx"][rest]]).astype(np.int32)


def _fkey(x):
    b = np.asarray(x, np.float32).view(np.int32).astype(np.int64)
    return np.where(b >= 0, b, -(b & 0x7FFFFFFF) - 1)


def _kfloat(k):
    k = np.asarray(k, np.int64)
    b = np.where(k >= 0, k, (-(k + 1)) | 0x80000000).astype(np.uint32)
    return b.view(np.float32)


def _interval_end(c, hw, hi):
    """per record, the last float from c towards +/-inf with |fl(x - c)| <= hw (binary search on keys)"""
    c, hw = np.asarray(c, np.float32), np.asarray(hw, np.float32)
    inn = _fkey(c)
    out = np.full_like(inn, int(_fkey(np.float32(np.inf if hi else -np.inf))))
    for _ in range(70):
        gap = np.abs(out - inn) > 1
        mid = inn + (out - inn) // 2
        ok = np.abs(_kfloat(mid) - c) <= hw
        inn = np.where(gap & ok, mid, inn)
        out = np.where(gap & ~ok, mid, out)
    return _kfloat(inn)


def _check_plane(t, p, cells, rng):
    per_cell = [_entries(t, c) for c in cells]
    recs = np.concatenate([r for r, _ in per_cell])
    ids = np.concatenate([i for _, i in per_cell])
    # one record per rect of this plane (a rect's entries all carry the same extent)
    uniq, first = np.unique(ids, return_index=True)
    recs, ids = recs[first], uniq
    cu, hwu, cv, hwv = (recs[:, k].astype(np.float32) for k in range(4))
    # candidate points: extent corners/edges +- 1 ulp, centres, and uniform random points
    us, vs = [], []
    for du in (-hwu, hwu):
        for sgn in (-1, 0, 1):
            u = (cu + du).astype(np.float32)
            u = np.nextafter(u, np.float32(np.inf) if sgn > 0 else np.float32(-np.inf)) if sgn else u
            for v in ((cv - hwv).astype(np.float32), cv, (cv + hwv).astype(np.float32)):
                us.append(u)
                vs.append(v)
    for dv in (-hwv, hwv):
        for sgn in (-1, 0, 1):
            v = (cv + dv).astype(np.float32)
            v = np.nextafter(v, np.float32(np.inf) if sgn > 0 else np.float32(-np.inf)) if sgn else v
            us.append(cu)
            vs.append(v)
    # the exact ends of each record's passing interval {x : |fl(x - c)| <= hw} (a binary search over the float
    # bit patterns, independent of the host's), the floats one past them, and c -/+ hw -/+ ulp(c) / 2
    for c, hw, other in ((cu, hwu, cv), (cv, hwv, cu)):
        for hi in (False, True):
            e = _interval_end(c, hw, hi)
            past = np.nextafter(e, np.float32(np.inf) if hi else np.float32(-np.inf))
            half = (c + (hw if hi else -hw) + (1 if hi else -1) * np.spacing(c) / 2).astype(np.float32)
            for x in (e, past, half):
                us.append(x if c is cu else other)
                vs.append(other if c is cu else x)
    lo_u, hi_u = float((cu - hwu).min()), float((cu + hwu).max())
    lo_v, hi_v = float((cv - hwv).min()), float((cv + hwv).max())
    us.append(rng.uniform(lo_u, hi_u, 20000).astype(np.float32))
    vs.append(rng.uniform(lo_v, hi_v, 20000).astype(np.float32))
    U = np.concatenate(us)
    V = np.concatenate(vs)
    cell = _cell_of(p, U, V)
    # every record containing the point must be listed in the point's cell
    inside = (np.abs(U[:, None] - cu[None, :]) <= hwu[None, :]) & (np.abs(V[:, None] - cv[None, :]) <= hwv[None, :])
    lists = [set(i.tolist()) for _, i in per_cell]
    missing = 0
    for k in np.nonzero(inside.any(axis=1))[0]:
        need = set(ids[inside[k]].tolist())
        if not need <= lists[cell[k]]:
            missing += 1
    assert missing == 0, f"{missing} points whose containing records are not in their cell"
    # the cell's inline records: every point that passes a record's float test passes its quantized bounds
    qu, qv = _q(p, U, V)
    col = {int(i): k for k, i in enumerate(ids)}
    bad = 0
    for slot, qname in ((0, "q0"), (1, "q1")):
        ce = cells[cell]
        has = ce["count"] > slot
        rid = ce["idx0"] if slot == 0 else ce["idx1"]
        b = ce[qname]
        for k in np.nonzero(has)[0]:
            j = col[int(rid[k])]
            if inside[k, j]:
                bu, bv = int(b[k, 0]), int(b[k, 1])
                ok = (bu & 0xFFFF) <= qu[k] <= (bu >> 16) and (bv & 0xFFFF) <= qv[k] <= (bv >> 16)
                bad += not ok
    assert bad == 0, f"{bad} points pass a record's float test but not its quantized bounds"
    # the plane's cull box (grid_axis skips the cell when the hit point is outside it): no point outside
    # the box passes any record's float test |x - c| <= hw, so skipping cannot drop a candidate
    f32 = np.float32
    assert p["ulo"] < lo_u and p["uhi"] > hi_u and p["vlo"] < lo_v and p["vhi"] > hi_v
    ob_u = np.concatenate([np.nextafter(f32(p["ulo"]), f32(-np.inf), dtype=np.float32) - rng.uniform(0, 1, 500).astype(f32),
                           np.nextafter(f32(p["uhi"]), f32(np.inf), dtype=np.float32) + rng.uniform(0, 1, 500).astype(f32)])
    ob_v = rng.uniform(lo_v, hi_v, 1000).astype(f32)
    for Uo, Vo in ((ob_u, ob_v), (rng.uniform(lo_u, hi_u, 1000).astype(f32), ob_u - f32(p["ulo"]) + f32(p["vlo"]))):
        ok = (np.abs(Uo[:, None] - cu[None, :]) <= hwu[None, :]) & (np.abs(Vo[:, None] - cv[None, :]) <= hwv[None, :])
        outside = (Uo < f32(p["ulo"])) | (Uo > f32(p["uhi"])) | (Vo < f32(p["vlo"])) | (Vo > f32(p["vhi"]))
        assert not (ok & outside[:, None]).any(), "a point outside the cull box passes a record test"
    # just outside the box edges, at every record's centre line
    for arr_u, arr_v in (([np.nextafter(f32(p["ulo"]), f32(-np.inf), dtype=np.float32)] * len(cv), cv),
                         ([np.nextafter(f32(p["uhi"]), f32(np.inf), dtype=np.float32)] * len(cv), cv),
                         (cu, [np.nextafter(f32(p["vlo"]), f32(-np.inf), dtype=np.float32)] * len(cu)),
                         (cu, [np.nextafter(f32(p["vhi"]), f32(np.inf), dtype=np.float32)] * len(cu))):
        Uo, Vo = np.asarray(arr_u, f32), np.asarray(arr_v, f32)
        ok = (np.abs(Uo[:, None] - cu[None, :]) <= hwu[None, :]) & (np.abs(Vo[:, None] - cv[None, :]) <= hwv[None, :])
        assert not ok.any()
    return len(ids)


@pytest.mark.parametrize("name", ["example", "box200", "box2000", "box8", "apartment30"])
def test_grid_cells_cover_every_containing_record(name, example_scene, box200, box2000):
    import os

    from conftest import GOLDEN
    from fmgi import scene

    sc = {"example": lambda: example_scene, "box200": lambda: box200, "box2000": lambda: box2000,
          "box8": lambda: scene.box_scene(8),
          "apartment30": lambda: scene.load_geometry(os.path.join(GOLDEN, "apartment30_geometry.bin"), "a30")}[name]()
    t = _tables(sc)
    rng = np.random.default_rng(7)
    n = 0
    for p, cells in _planes(t):
        n += _check_plane(t, p, cells, rng)
    # every rect of these scenes is axis-aligned, so every rect is on exactly one grid plane
    assert n == len(sc.walls)


def test_grid_is_small_and_selective(box200, box2000):
    """Expected records per lookup stays near 1 on the synthetic boxes (the point of the grid)."""
    for sc in (box200, box2000):
        t = _tables(sc)
        planes = _planes(t)
        assert len(planes) == 6  # a closed box: six planes
        tot = sum(len(c) for _, c in planes)
        ent = sum(int(c["count"].sum()) for _, c in planes)
        assert tot <= 16 * len(sc.walls) + 16 * 6
        assert ent / tot < 2.0, ent / tot


@pytest.mark.parametrize("cpr", [4, 3, 2])
def test_compact_grids_cover_and_hold_four_records(cpr, box2000):
    """The grids the compact closed-box tables index (fmgi_api.cpp build_compact, BASELINE config 5: 4, 3 or 2
    cells per record, each cell's records as up to four u16 indices): the coverage property of every grid, and
    no box2000 cell of more than four records, so every cell fits its CellC."""
    t = _tables(box2000, cpr)
    rng = np.random.default_rng(11 + cpr)
    n = 0
    planes = _planes(t)
    assert len(planes) == 6
    for p, cells in planes:
        n += _check_plane(t, p, cells, rng)
        assert int(cells["count"].max()) <= 4
    assert n == len(box2000.walls) < 0xFFFF
