#!/usr/bin/env python
"""Synthetic layout fixtures: floor-plan PNGs generated here (no reference data file), parsed by the
REFERENCE's own layout parser (parseLayout.c via oracle/_ref/dump_geometry, built by
oracle/build_ref.sh; 30 px/m and TILE_SIZE 200 as main.c:26,44) into FMGIGEO1 geometry fixtures the
GPU box can load without the reference.

  apartment30_geometry.bin  a 6 x 5 grid of ~4 m x 3.3 m rooms: outer windows, doors between most
                            neighbours, ceiling lights in the rooms without windows (the parser's
                            createLights). 654 walls, 22 windows, 12 lights, 731,962 texels: a large
                            layout of the reference's own kind for the acceleration-structure bench.

  python tests/golden/make_layout_fixtures.py
"""
import os
import subprocess
import sys
import tempfile

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))

WALL, EMPTY, OUTSIDE, DOOR, WINDOW = (0, 0, 0), (255, 255, 255), (127, 127, 127), (223, 223, 223), (0, 255, 0)


def apartment_grid(rows=5, cols=6, rw=120, rh=100, t=6, m=12, seed=3):
    """Layout pixels (RGB) of a rows x cols grid of rooms, rw x rh px each, walls t px thick."""
    H, W = 2 * m + rows * rh + (rows + 1) * t, 2 * m + cols * rw + (cols + 1) * t
    img = np.zeros((H, W, 3), np.uint8)
    img[:] = OUTSIDE
    img[m:H - m, m:W - m] = WALL
    rng = np.random.default_rng(seed)
    for r in range(rows):
        for c in range(cols):
            y0, x0 = m + t + r * (rh + t), m + t + c * (rw + t)
            img[y0:y0 + rh, x0:x0 + rw] = EMPTY
            if c < cols - 1 and rng.random() < 0.8:
                img[y0 + 30:y0 + 60, x0 + rw:x0 + rw + t] = DOOR
            if r < rows - 1 and rng.random() < 0.8:
                img[y0 + rh:y0 + rh + t, x0 + 40:x0 + 75] = DOOR
            if r == 0:
                img[m:m + t, x0 + 30:x0 + 80] = WINDOW
            if r == rows - 1:
                img[H - m - t:H - m, x0 + 30:x0 + 80] = WINDOW
            if c == 0:
                img[y0 + 25:y0 + 70, m:m + t] = WINDOW
            if c == cols - 1:
                img[y0 + 25:y0 + 70, W - m - t:W - m] = WINDOW
    return img


def main():
    from PIL import Image

    dump = os.path.join(REPO, "oracle", "_ref", "dump_geometry")
    with tempfile.TemporaryDirectory() as d:
        png = os.path.join(d, "apartment30.png")
        Image.fromarray(apartment_grid(), "RGB").save(png)
        subprocess.run([dump, png, "30", os.path.join(HERE, "apartment30_geometry.bin")], check=True, cwd=d,
                       stdout=subprocess.DEVNULL)
    sys.path.insert(0, os.path.join(REPO, "flatmatch-global-illumination_amd"))
    from fmgi import scene

    sc = scene.load_geometry(os.path.join(HERE, "apartment30_geometry.bin"), "apartment30")
    print("apartment30:", len(sc.walls), "walls,", len(sc.windows), "windows,", len(sc.lights), "lights,",
          sc.num_texels, "texels")


if __name__ == "__main__":
    main()
