"""Scene data for the photon-mapping path: the reference's Rectangle/Geometry layout as numpy
records, the geometry fixture reader, and the synthetic N-rectangle box scenes of BASELINE.json.

Layout (byte-identical to the reference ABI):
  * ``RECT_DTYPE`` == ``Rectangle`` (rectangle.h:19-26): pos, width, height, n as float4 (.w unused)
    and ``lightmapSetup`` int4 = {texel base, tiles along width, tiles along height, 0}; 80 B.
  * texels == ``Vector3`` (cl_float4, vector3_cl.h:14): ``numTexels x 4`` float32.

The box generator restates the reference's rectangle construction so that a synthetic scene looks
exactly like one parseLayout.c would build:
  * ``create_rectangle`` -- rectangle.c:15-57 (``createRectangleV``: normal = normalized(cross(h, w)),
    power-of-two lightmap tiling until >= TILE_SIZE texels per m^2), evaluated in float32 op by op;
  * ``num_mipmap_texels`` -- rectangle.c:166-192;
  * texel bases = running sum of mipmapped texel counts, parseLayout.c:512-517;
  * floor / ceiling / wall orientation conventions of parseLayout.c:43-46 (addHorizontalRect) and
    parseLayout.c:33-36,52-53 (addWall / registerWall).
"""
from __future__ import annotations

import dataclasses
import struct

import numpy as np

RECT_DTYPE = np.dtype(
    [("pos", "<f4", 4), ("width", "<f4", 4), ("height", "<f4", 4), ("n", "<f4", 4), ("lm", "<i4", 4)],
    align=True,
)
assert RECT_DTYPE.itemsize == 80

TILE_SIZE = np.float32(200.0)  # main.c:44: lightmap texels per m^2
HEIGHT = np.float32(2.60)  # parseLayout.c:26

f32 = np.float32


def _len(v):
    # vector3_cl.c:93: sqrtf(x*x + y*y + z*z), evaluated left to right in float32
    return f32(np.sqrt(f32(f32(f32(v[0] * v[0]) + f32(v[1] * v[1])) + f32(v[2] * v[2]))))


def _cross(a, b):
    # vector3_cl.c:79-85
    return (
        f32(f32(a[1] * b[2]) - f32(a[2] * b[1])),
        f32(f32(a[2] * b[0]) - f32(a[0] * b[2])),
        f32(f32(a[0] * b[1]) - f32(a[1] * b[0])),
    )


def _normalized(a):
    # vector3_cl.c:95-101: multiply by the float reciprocal of the length
    fac = f32(f32(1.0) / _len(a))
    return (f32(a[0] * fac), f32(a[1] * fac), f32(a[2] * fac))


def create_rectangle(px, py, pz, wx, wy, wz, hx, hy, hz, tile_size=TILE_SIZE):
    """rectangle.c:15-64 (createRectangle -> createRectangleV) in float32."""
    p = tuple(f32(v) for v in (px, py, pz))
    w = tuple(f32(v) for v in (wx, wy, wz))
    h = tuple(f32(v) for v in (hx, hy, hz))
    n = _normalized(_cross(h, w))
    s1, s2 = 1, 1
    width, height = _len(w), _len(h)
    tile = f32(f32(f32(s1) * f32(s2)) / f32(width * height))
    while tile < f32(tile_size):
        width_res = f32(f32(s1) / width)
        height_res = f32(f32(s2) / height)
        if width_res < height_res:
            s1 *= 2
        else:
            s2 *= 2
        tile = f32(f32(s1 * s2) / f32(width * height))
    r = np.zeros((), RECT_DTYPE)
    r["pos"][:3] = p
    r["width"][:3] = w
    r["height"][:3] = h
    r["n"][:3] = n
    r["lm"][:] = (0, s1, s2, 0)
    return r


def num_mipmap_texels(w: int, h: int) -> int:
    """rectangle.c:166-192."""
    n = w * h
    while w > 1 or h > 1:
        if w > 1:
            w //= 2
        if h > 1:
            h //= 2
        n += w * h
    return n


def assign_texel_bases(walls: np.ndarray) -> int:
    """parseLayout.c:512-517: texel base of each wall = running sum; returns numTexels."""
    total = 0
    for i in range(len(walls)):
        walls[i]["lm"][0] = total
        total += num_mipmap_texels(int(walls[i]["lm"][1]), int(walls[i]["lm"][2]))
    return total


@dataclasses.dataclass
class Scene:
    """The photon-mapping inputs of a reference ``Geometry`` (geometry.h:7-15)."""

    name: str
    walls: np.ndarray  # RECT_DTYPE[numWalls]
    windows: np.ndarray  # RECT_DTYPE[numWindows]
    lights: np.ndarray  # RECT_DTYPE[numLights]
    num_texels: int

    @property
    def sources(self) -> np.ndarray:
        return np.concatenate([self.windows, self.lights])

    def texels(self) -> np.ndarray:
        """A zeroed texel buffer (parseLayout.c:532-533)."""
        return np.zeros((self.num_texels, 4), np.float32)

    def level0_mask(self) -> np.ndarray:
        m = np.zeros(self.num_texels, bool)
        for w in self.walls:
            b, s1, s2 = int(w["lm"][0]), int(w["lm"][1]), int(w["lm"][2])
            m[b : b + s1 * s2] = True
        return m


def load_geometry(path: str, name: str | None = None) -> Scene:
    """Read a FMGIGEO1 fixture (written by oracle/dump_geometry.c from the reference's parseLayout)."""
    with open(path, "rb") as f:
        blob = f.read()
    if blob[:8] != b"FMGIGEO1":
        raise ValueError(f"{path}: not a FMGIGEO1 geometry fixture")
    nw, nl, nwall, ntex = struct.unpack_from("<4i", blob, 8)
    arr = np.frombuffer(blob, RECT_DTYPE, count=nw + nl + nwall, offset=24).copy()
    return Scene(name or path, arr[nw + nl :], arr[:nw], arr[nw : nw + nl], ntex)


def save_geometry(scene: Scene, path: str) -> None:
    with open(path, "wb") as f:
        f.write(b"FMGIGEO1")
        f.write(struct.pack("<4i", len(scene.windows), len(scene.lights), len(scene.walls), scene.num_texels))
        f.write(scene.windows.tobytes())
        f.write(scene.lights.tobytes())
        f.write(scene.walls.tobytes())


def _grid(lo: float, hi: float, k: int):
    return [f32(lo + (hi - lo) * i / k) for i in range(k + 1)]


def box_scene(n_rects: int = 200, room=(10.0, 8.0, 2.6), tile_size: float = TILE_SIZE,
              with_light: bool = False) -> Scene:
    """Synthetic closed box: floor + ceiling tiled g x g, four walls tiled c x r,
    all normals inward, one 4 m x 1.45 m window (not in the rect list) on the y=0 wall.

    n_rects=200: floor 6x6, ceiling 6x6, walls 4 x (8 cols x 4 rows).
    n_rects=2000: floor 20x20, ceiling 20x20, walls 4 x (30 cols x 10 rows).
    tile_size: lightmap texels per m² of the walls (the reference's TILE_SIZE, main.c:44); smaller
    values give small test scenes. with_light adds a 0.5 m x 0.5 m ceiling light (1 x 1 texels, as
    parseLayout.c:278-280 creates lights).
    """
    layouts = {200: (6, 8, 4), 2000: (20, 30, 10), 8: (1, 1, 1)}
    if n_rects not in layouts:
        raise ValueError(f"box_scene supports n_rects in {sorted(layouts)}")
    g, cols, rows = layouts[n_rects]
    X, Y, Z = room
    xs, ys, zs = _grid(0.0, X, g), _grid(0.0, Y, g), _grid(0.0, Z, rows)
    walls = []
    # floor (parseLayout.c:471 convention: pos at x_end, width -dx, height +dy -> n = +z)
    for j in range(g):
        for i in range(g):
            walls.append(create_rectangle(xs[i + 1], ys[j], 0.0, f32(xs[i] - xs[i + 1]), 0, 0, 0, f32(ys[j + 1] - ys[j]), 0,
                                          tile_size))
    # ceiling (parseLayout.c:472: pos at x_start, width +dx, height +dy -> n = -z)
    zc = f32(Z)
    for j in range(g):
        for i in range(g):
            walls.append(create_rectangle(xs[i], ys[j], zc, f32(xs[i + 1] - xs[i]), 0, 0, 0, f32(ys[j + 1] - ys[j]), 0,
                                          tile_size))
    # walls: width (dx, dy, 0), height (0, 0, dz) -> n = normalized(-dy, dx, 0) (parseLayout.c:33-36)
    wx, wy = _grid(0.0, X, cols), _grid(0.0, Y, cols)
    for k in range(rows):
        dz = f32(zs[k + 1] - zs[k])
        for i in range(cols):
            walls.append(create_rectangle(wx[i], 0.0, zs[k], f32(wx[i + 1] - wx[i]), 0, 0, 0, 0, dz, tile_size))  # n=+y
            walls.append(create_rectangle(wx[i + 1], f32(Y), zs[k], f32(wx[i] - wx[i + 1]), 0, 0, 0, 0, dz, tile_size))
            walls.append(create_rectangle(0.0, wy[i + 1], zs[k], 0, f32(wy[i] - wy[i + 1]), 0, 0, 0, dz, tile_size))
            walls.append(create_rectangle(f32(X), wy[i], zs[k], 0, f32(wy[i + 1] - wy[i]), 0, 0, 0, dz, tile_size))
    walls = np.array(walls, RECT_DTYPE)
    ntex = assign_texel_bases(walls)
    window = np.array([create_rectangle(3.0, 0.001, 0.85, 4.0, 0, 0, 0, 0, 1.45)], RECT_DTYPE)
    lights = (np.array([create_rectangle(5.0, 4.0, f32(Z - 0.001), 0.5, 0, 0, 0, 0.5, 0, 0.0)], RECT_DTYPE)
              if with_light else np.zeros(0, RECT_DTYPE))
    name = f"box{n_rects}" + ("" if tile_size == TILE_SIZE else f"_t{tile_size:g}") + ("_lit" if with_light else "")
    return Scene(name, walls, window, lights, ntex)


def shelves_scene(n_panels: int = 6000, tile_size: float = 4.0, seed: int = 7) -> Scene:
    """box200 plus n_panels small horizontal panels, each on its own height (half facing up, half
    down): thousands of distinct planes, so neither scan image (ScanFast's record pairs, ScanGrid's
    plane pairs) fits in LDS and the bake must fall back to the exact scan (fmgi_api.cpp kernel_fits)."""
    box = box_scene(200, tile_size=tile_size)
    rng = np.random.default_rng(seed)
    walls = list(box.walls)
    for i in range(n_panels):
        z = f32(0.2 + 2.2 * (i + 0.5) / n_panels)
        x, y = f32(rng.uniform(0.5, 9.0)), f32(rng.uniform(0.5, 7.0))
        w, h = f32(rng.uniform(0.1, 0.5)), f32(rng.uniform(0.1, 0.5))
        if i % 2:  # normal +z: width along -x from the far corner (parseLayout.c:471 floor convention)
            walls.append(create_rectangle(f32(x + w), y, z, f32(-w), 0, 0, 0, h, 0, tile_size))
        else:      # normal -z (ceiling convention)
            walls.append(create_rectangle(x, y, z, w, 0, 0, 0, h, 0, tile_size))
    walls = np.array(walls, RECT_DTYPE)
    ntex = assign_texel_bases(walls)
    return Scene(f"shelves{n_panels}", walls, box.windows, box.lights, ntex)


def tilted_scene(n_panels: int = 12, tile_size: float = 20.0, seed: int = 11) -> Scene:
    """box200 plus n_panels rects that are not axis-aligned (vertical panels turned about z, and sloped
    ones): every scan's `general` list (ScanFast / ScanGrid test them exactly), as a layout with
    diagonal walls would give (parseLayout.c:48-128 registers a wall along any pixel direction)."""
    box = box_scene(200, tile_size=tile_size)
    rng = np.random.default_rng(seed)
    walls = list(box.walls)
    for i in range(n_panels):
        x, y = f32(rng.uniform(1.5, 8.5)), f32(rng.uniform(1.5, 6.5))
        a = rng.uniform(0.2, 1.4) + (np.pi if i % 2 else 0.0)
        L = f32(rng.uniform(0.5, 1.5))
        wx, wy = f32(L * np.cos(a)), f32(L * np.sin(a))
        if i % 3 == 2:  # sloped: width along the floor, height rising
            walls.append(create_rectangle(x, y, f32(0.3), wx, wy, 0, f32(-0.3 * wy), f32(0.3 * wx), f32(0.8), tile_size))
        else:           # vertical, turned about z
            walls.append(create_rectangle(x, y, f32(0.2), wx, wy, 0, 0, 0, f32(rng.uniform(0.8, 2.0)), tile_size))
    walls = np.array(walls, RECT_DTYPE)
    ntex = assign_texel_bases(walls)
    return Scene(f"tilted{n_panels}", walls, box.windows, box.lights, ntex)


def spa_for_photons(scene: Scene, photons: float) -> int:
    """numSamplesPerArea giving ~`photons` photons over the scene's emitters (main.c:58 semantics)."""
    area = 0.0
    for s in scene.sources:
        area += float(_len(s["width"][:3]) * _len(s["height"][:3]))
    return int(photons / area)
