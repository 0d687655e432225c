"""CPU tests of the C-ABI boundary: the library loads, exports every symbol include/flatmatch_gi.h
declares and nothing that would clash with the reference objects main.c links, the structure
layouts are the reference's, and the host-side schedule is the reference's (host-only context)."""
import ctypes as C
import os
import re
import subprocess

import numpy as np
import pytest

import fm_oracle as O
import fmgi
from conftest import PKG, REPO
from fmgi import _lib

HEADER = os.path.join(REPO, "include", "flatmatch_gi.h")


def _exports():
    out = subprocess.run(["nm", "-D", "--defined-only", _lib.LIB_PATH], capture_output=True, text=True, check=True)
    syms = set()
    for line in out.stdout.splitlines():
        parts = line.split()
        if len(parts) == 3 and parts[1] in "TDBRW":
            syms.add(parts[2])
    return syms


def _header_functions():
    src = open(HEADER).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    src = re.sub(r"^\s*#.*$", "", src, flags=re.M)
    return set(re.findall(r"\b([A-Za-z_]\w*)\s*\([^;{}]*\)\s*;", src))


def test_library_loads_and_exports_every_declared_symbol():
    lib = _lib.load()
    declared = _header_functions()
    assert "performGlobalIlluminationCl" in declared and "fmgi_bake_items" in declared
    exported = _exports()
    missing = declared - exported
    assert not missing, f"declared but not exported: {missing}"
    assert set(_lib.EXPORTS) <= exported
    for name in declared:
        assert getattr(lib, name) is not None


def test_no_symbol_clashes_with_reference_objects():
    # symbols defined by the reference's own objects that main.c links
    clashing = {"length", "rand", "photonmap", "intersects", "getTileIdAt", "dot", "cross", "normalized",
                "getWidthVector", "getHeightVector", "tracePhoton", "getCosineDistributedRandomRay",
                "getDiffuseSkyRandomRay", "createBase", "add", "sub", "mul"}
    exported = _exports()
    assert not (exported & clashing)
    extra = {s for s in exported if not s.startswith("fmgi_")}
    assert extra == {"performGlobalIlluminationCl", "getGlobalIlluminationCl", "performAmbientOcclusionGpu",
                     "performRadiosityGpu"}


def test_struct_layouts_match_reference_abi():
    from fmgi.scene import RECT_DTYPE

    assert RECT_DTYPE.itemsize == 80 and RECT_DTYPE.fields["lm"][1] == 64
    assert C.sizeof(_lib.Geometry) == 80
    offs = {name: getattr(_lib.Geometry, name).offset for name, _ in _lib.Geometry._fields_}
    # offsetof() values measured on the reference
    assert offs == {"windows": 0, "lights": 8, "walls": 16, "boxWalls": 24, "numWindows": 32, "numLights": 36,
                    "numWalls": 40, "numBoxWalls": 44, "width": 48, "height": 52, "startingPositionX": 56,
                    "startingPositionY": 60, "numTexels": 64, "texels": 72}
    assert fmgi.LAUNCH_DTYPE.itemsize == 24 and fmgi.EVENT_DTYPE.itemsize == 32


def _host_ctx(sc):
    lib = _lib.load()
    h = lib.fmgi_create(-1)
    assert h
    keep = [np.ascontiguousarray(a) for a in (sc.walls, sc.windows, sc.lights)]
    p = [a.ctypes.data_as(C.c_void_p) if len(a) else None for a in keep]
    rc = lib.fmgi_set_scene(h, p[0], len(keep[0]), p[1], len(keep[1]), p[2], len(keep[2]), sc.num_texels)
    assert rc == 0, _lib.last_error()
    return lib, h, keep


@pytest.mark.parametrize("spa", [65_000, 6_500_000, 1_000])
def test_product_plan_equals_oracle_schedule(spa, example_scene, libc):
    lib, h, keep = _host_ctx(example_scene)
    try:
        tot = C.c_uint64()
        libc.srand(1)
        n = lib.fmgi_plan(h, spa, 256, None, 0, C.byref(tot))
        assert n > 0
        after_product = libc.rand()
        plan = np.zeros(n, fmgi.LAUNCH_DTYPE)
        assert lib.fmgi_get_plan(h, plan.ctypes.data_as(C.c_void_p), n) == n
        libc.srand(1)
        ref = O.schedule(example_scene, spa)
        after_oracle = libc.rand()
        assert plan.tobytes() == ref.tobytes()
        assert after_product == after_oracle  # same libc rand() state after the call
        assert fmgi.plan_count(example_scene, spa) == (len(ref), int(ref["count"].sum()))
    finally:
        lib.fmgi_destroy(h)


def test_plan_with_explicit_offsets_and_wg(box200):
    lib, h, keep = _host_ctx(box200)
    try:
        offs = np.arange(1000, 1400, dtype=np.int32)
        tot = C.c_uint64()
        n = lib.fmgi_plan(h, 172_413_793, 1024, offs.ctypes.data_as(C.c_void_p), len(offs), C.byref(tot))
        # NVIDIA-style WG=1024: launches of up to 102,400 items, +1 WG rounding per source
        assert tot.value % 1024 == 0 and tot.value * 100 >= 1_000_000_000
        plan = np.zeros(n, fmgi.LAUNCH_DTYPE)
        lib.fmgi_get_plan(h, plan.ctypes.data_as(C.c_void_p), n)
        assert np.array_equal(plan["rng_offset"], offs[:n])
        assert plan["count"].max() == 102_400
        ref = O.schedule_with_offsets(box200, 172_413_793, offs, wg=1024)
        assert plan.tobytes() == ref.tobytes()
    finally:
        lib.fmgi_destroy(h)


def test_scene_validation_rejects_out_of_range_texels(box200):
    lib = _lib.load()
    h = lib.fmgi_create(-1)
    try:
        walls = np.ascontiguousarray(box200.walls.copy())
        rc = lib.fmgi_set_scene(h, walls.ctypes.data_as(C.c_void_p), len(walls), None, 0, None, 0, 100)
        assert rc == -3 and "outside" in _lib.last_error()
    finally:
        lib.fmgi_destroy(h)


def test_host_only_context_cannot_bake(box200):
    lib, h, keep = _host_ctx(box200)
    try:
        rc = lib.fmgi_bake_items(h, 0, 1, C.c_void_p(16), 0, None)
        assert rc == -1
    finally:
        lib.fmgi_destroy(h)


def test_no_gpu_fails_loudly(tmp_path):
    """Without a device the drop-in entry point prints an error and exits -1 (reference convention)."""
    prog = tmp_path / "nogpu.py"
    prog.write_text(
        "import sys; sys.path.insert(0, %r)\n"
        "import numpy as np, fmgi\n"
        "from fmgi import scene\n"
        "sc = scene.box_scene(8)\n"
        "tex = sc.texels()\n"
        "g, keep = fmgi.make_geometry(sc, tex)\n"
        "import ctypes\n"
        "fmgi._lib.load().performGlobalIlluminationCl(ctypes.byref(g), 1000)\n"
        "print('UNREACHABLE')\n" % PKG
    )
    env = dict(os.environ, HIP_VISIBLE_DEVICES="-1", CUDA_VISIBLE_DEVICES="-1", ROCR_VISIBLE_DEVICES="-1")
    r = subprocess.run(["python", str(prog)], capture_output=True, text=True, env=env, timeout=120)
    assert r.returncode == 255, r.stdout + r.stderr
    assert "[Err] performGlobalIlluminationCl" in r.stdout and "UNREACHABLE" not in r.stdout


@pytest.mark.parametrize("items,ngpu,nshard", [(100_000_256, 8, 8), (10_000_128, 8, 8), (10_000_128, 8, 16),
                                                (1_001_216, 8, 8), (1_001_216, 4, 4), (17, 2, 3), (5, 8, 8),
                                                (391 * 25_600, 3, 7), (0, 2, 2)])
def test_dropin_shard_layout_and_reduction_tree(items, ngpu, nshard):
    """The drop-in's multi-GPU plan (used by bake_geometry_devices): shards partition the work items in
    order, land on devices 0..ngpu-1 (device indices > 0 included), and the reduction tree adds every
    other shard into shard 0 exactly once, each source finished before it is read."""
    dev, b, e = fmgi.dropin_shards(items, ngpu, nshard)
    assert list(dev) == [k % ngpu for k in range(nshard)]
    assert b[0] == 0 and e[-1] == items and np.all(b[1:] == e[:-1]) and np.all(e >= b)
    assert max(e - b) - min(e - b) <= 1
    dst, src = fmgi.dropin_reduce_order(nshard)
    assert len(dst) == nshard - 1
    total = {k: {k} for k in range(nshard)}
    consumed = set()
    for d, s in zip(dst, src):
        assert d < s and s not in consumed and d not in consumed
        total[int(d)] |= total.pop(int(s))
        consumed.add(int(s))
    assert total == {0: set(range(nshard))}


def test_scan_image_too_large_for_lds_falls_back():
    """A scene with thousands of distinct planes: neither ScanFast's record image nor ScanGrid's plane
    image fits the 64-KiB dynamic LDS of a bake launch, so AUTO resolves to the exact scan (same
    results) instead of a launch that would fail; small scenes keep their LDS scans."""
    from fmgi import scene

    big = scene.shelves_scene(6000)
    ctx = fmgi.Context(fmgi.HOST_ONLY)
    ctx.set_scene(big)
    assert ctx.auto_kernel == fmgi.KERNEL_EXACT
    ctx.set_scene(scene.box_scene(200))
    assert ctx.auto_kernel == fmgi.KERNEL_GRID
    ctx.close()
