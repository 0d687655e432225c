"""End-to-end drop-in: the reference's own command-line program (main.c + parseLayout.c + image.c +
png_helper.c + rectangle.c + ..., compiled from /root/reference by oracle/build_ref.sh) linked against
libflatmatch_gi.so instead of global_illumination_cl.o (oracle/_ref/globalIllumination_fmgi), run on a
synthetic two-room layout PNG made here. It parses the layout, calls our performGlobalIlluminationCl
(main.c:63, 1e8 samples per m²), normalises, tone-maps and writes one PNG per wall (main.c:66-95).

Expected: the same geometry (the reference parser, oracle/_ref/dump_geometry), baked through the
library's non-mutating entry point from the same libc rand() state and run through fmgi_output_tiles
(byte-identical to the reference's saveAs, tests/test_output.py). Every tile PNG must match byte for
byte, and the program's console output carries the reference's per-launch progress lines
(global_illumination_cl.c:248-249, one "\rphoton-mapping window with %d M samples   " per launch with the
samples still to launch for that source, a newline after each source). The layout is generated (no
reference data file is used)."""
import ctypes
import os
import subprocess

import numpy as np
import pytest

import fm_oracle as O
from conftest import REPO

REF = os.path.join(REPO, "oracle", "_ref")
PROG = os.path.join(REF, "globalIllumination_fmgi")
DUMP = os.path.join(REF, "dump_geometry")

pytestmark = pytest.mark.gpu

WALL, EMPTY, OUTSIDE, DOOR, WINDOW = (0, 0, 0), (255, 255, 255), (127, 127, 127), (223, 223, 223), (0, 255, 0)


def _layout(path):
    """Two rooms side by side at 30 px/m: a window in room 1's outer wall, a door between the rooms
    (room 2 has no window, so the reference parser gives it a ceiling light)."""
    from PIL import Image

    img = np.zeros((190, 280, 3), np.uint8)
    img[:] = OUTSIDE
    img[10:180, 10:270] = WALL
    img[16:174, 16:130] = EMPTY
    img[16:174, 136:264] = EMPTY
    img[80:110, 130:136] = DOOR
    img[10:16, 40:100] = WINDOW
    Image.fromarray(img, "RGB").save(path)


@pytest.mark.skipif(not (os.path.exists(PROG) and os.path.exists(DUMP)),
                    reason="oracle/_ref not built (needs /root/reference at build time)")
def test_reference_cli_linked_against_library(torch_cuda, tmp_path):
    from PIL import Image

    import fmgi
    from fmgi import scene

    png = str(tmp_path / "layout.png")
    _layout(png)
    geo_bin = str(tmp_path / "geometry.bin")
    subprocess.run([DUMP, png, "30", geo_bin], check=True, cwd=tmp_path, stdout=subprocess.DEVNULL)
    sc = scene.load_geometry(geo_bin, "layout")
    assert len(sc.walls) > 10 and len(sc.windows) == 1 and len(sc.lights) >= 1

    os.makedirs(tmp_path / "tiles")
    env = {k: v for k, v in os.environ.items() if k != "FMGI_QUIET"}
    run = subprocess.run([PROG, png], cwd=tmp_path, env=env, capture_output=True, timeout=300)
    out = run.stdout.decode(errors="replace")  # bytes: text mode would turn the "\r"s into newlines
    assert run.returncode == 0, out[-2000:] + run.stderr.decode(errors="replace")[-2000:]

    spa = 1000 * 1000 * 100  # main.c:58
    sched = O.schedule_with_offsets(sc, spa, np.zeros(4096, np.int32))
    progress = ""
    for s_idx in range(len(sc.windows) + len(sc.lights)):
        counts = [int(c) for c in sched["count"][sched["source"] == s_idx]]
        left = sum(counts)
        for c in counts:
            progress += "\rphoton-mapping window with %d M samples   " % (left * 100 // 1000000)
            left -= c
        progress += "\n"
    assert "[INF] Selected device '" in out
    assert progress in out, out[-2000:]
    libc = ctypes.CDLL(None)
    libc.srand(1)  # the CLI process starts from glibc's unseeded state
    tex = fmgi.bake_geometry(sc, spa, np.zeros((sc.num_texels, 4), np.float32))
    _, rgb = fmgi.output_tiles(sc, tex, spa, 0)
    off = 0
    for i, w in enumerate(sc.walls):
        n = int(w["lm"][1]) * int(w["lm"][2]) * 3
        got = np.asarray(Image.open(tmp_path / "tiles" / f"tile_{i}.png").convert("RGB")).tobytes()
        assert got == rgb[off:off + n].tobytes(), f"tile {i} differs"
        off += n
    assert off == rgb.size
