"""fmgi -- Python mirror of the MI355X photon-mapping lightmap baker's C ABI.

The product is libflatmatch_gi.so (HIP kernels for gfx950 + the C ABI of include/flatmatch_gi.h);
this package only binds it with ctypes for tests, bench.py and Python callers:

  * ``Context``      -- fmgi_create / fmgi_set_scene / fmgi_plan / fmgi_bake_items / fmgi_finalize;
  * ``bake_geometry`` -- getGlobalIlluminationCl on host arrays (the reference's
                         performGlobalIlluminationCl semantics, global_illumination_cl.c:275-321);
  * ``scene``        -- the Rectangle/Geometry layout, fixtures and synthetic box scenes.

Device buffers are passed as plain integer addresses (e.g. ``torch.Tensor.data_ptr()``) and streams as
``hipStream_t`` integers; no torch type crosses the C ABI.
"""
from __future__ import annotations

import ctypes as C

import numpy as np

from . import scene

HOST_ONLY = -1  # FMGI_HOST_ONLY: a context without a device (scene checks and planning only)
from ._lib import (ACCUM_AUTO, ACCUM_FX3, ACCUM_NONE, ACCUM_STATE, ACCUM_STREAM, KERNEL_AUTO, KERNEL_EXACT, KERNEL_FAST, KERNEL_GRID, KERNEL_HYBRID, RadStats, Timing, FmgiError, Geometry, Stats,
                   check, load)
from .scene import RECT_DTYPE, Scene

LAUNCH_DTYPE = np.dtype(
    [("item_begin", "<u8"), ("count", "<u4"), ("rng_offset", "<i4"), ("source", "<i4"), ("is_window", "<i4")]
)
assert LAUNCH_DTYPE.itemsize == 24
EVENT_DTYPE = np.dtype(
    [("photon", "<i4"), ("depth", "<i4"), ("rect", "<i4"), ("texel", "<i4"), ("rgb", "<f4", 3), ("rng", "<u4")]
)
assert EVENT_DTYPE.itemsize == 32
EVENTS_PER_ITEM = 800
FX_SHIFT = 25

__all__ = [
    "Context",
    "bake_geometry",
    "plan_count",
    "scene",
    "Scene",
    "FmgiError",
    "KERNEL_EXACT",
    "KERNEL_FAST",
    "KERNEL_GRID",
    "KERNEL_AUTO",
    "ACCUM_AUTO",
    "ACCUM_FX3",
    "ACCUM_STATE",
    "ACCUM_STREAM",
    "LAUNCH_DTYPE",
    "EVENT_DTYPE",
    "device_count",
    "host_sincosf",
]


UNIT_SQRT = 0       # fmgi_device_unit ops (include/flatmatch_gi.h)
UNIT_TRUNC_DIV = 1
UNIT_TRUNC_DIV_INV = 2


def _ptr(a: np.ndarray | None):
    if a is None or len(a) == 0:
        return None
    assert a.flags["C_CONTIGUOUS"]
    return a.ctypes.data_as(C.c_void_p)


def device_count() -> int:
    return int(load().fmgi_device_count())


def host_sincosf(x):
    """Host fmgi_sincosf over an array (bit-identical to the device sampler's sin/cos)."""
    x = np.ascontiguousarray(np.atleast_1d(x), np.float32)
    s = np.empty_like(x)
    c = np.empty_like(x)
    load().fmgi_host_sincosf(_ptr(x), _ptr(s), _ptr(c), len(x))
    return s, c


def plan_count(sc: Scene, spa: int, wg: int = 256):
    """(launches, work items) of the reference schedule, without consuming rand()."""
    tot = C.c_uint64()
    w = np.ascontiguousarray(sc.windows)
    l = np.ascontiguousarray(sc.lights)
    n = check(load().fmgi_plan_count(_ptr(w), len(w), _ptr(l), len(l), spa, wg, C.byref(tot)), "fmgi_plan_count")
    return int(n), int(tot.value)


class Context:
    """One device's baker state (fmgi_context)."""

    def __init__(self, device: int = 0):
        self.lib = load()
        self.h = self.lib.fmgi_create(device)
        if not self.h:
            raise FmgiError(f"fmgi_create({device}): {self.lib.fmgi_last_error().decode()}")
        self.device = device
        self.scene: Scene | None = None
        self.total_items = 0
        self.nlaunches = 0

    def close(self):
        if self.h:
            self.lib.fmgi_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def set_scene(self, sc: Scene):
        self._keep = [np.ascontiguousarray(a) for a in (sc.walls, sc.windows, sc.lights)]
        w, win, li = self._keep
        check(
            self.lib.fmgi_set_scene(self.h, _ptr(w), len(w), _ptr(win), len(win), _ptr(li), len(li), sc.num_texels),
            "fmgi_set_scene",
        )
        self.scene = sc

    def set_accumulation(self, mode: int):
        """ACCUM_FX3 (3 int64 atomics per deposit), ACCUM_STATE (1 u32 counter per colour state and
        texel) or ACCUM_AUTO. Both modes give identical bits."""
        check(self.lib.fmgi_set_accumulation(self.h, mode), "fmgi_set_accumulation")

    @property
    def accumulation(self) -> int:
        return int(self.lib.fmgi_get_accumulation(self.h))

    def plan(self, spa: int, wg: int = 256, rng_offsets=None) -> int:
        """Reference launch schedule. rng_offsets=None consumes libc rand() like the reference."""
        tot = C.c_uint64()
        offs = None if rng_offsets is None else np.ascontiguousarray(rng_offsets, np.int32)
        n = check(
            self.lib.fmgi_plan(self.h, spa, wg, _ptr(offs), 0 if offs is None else len(offs), C.byref(tot)),
            "fmgi_plan",
        )
        self.total_items = int(tot.value)
        self.nlaunches = int(n)
        return self.total_items

    def get_plan(self) -> np.ndarray:
        out = np.zeros(self.nlaunches, LAUNCH_DTYPE)
        check(self.lib.fmgi_get_plan(self.h, _ptr(out), len(out)), "fmgi_get_plan")
        return out

    def bake_items(self, begin: int, end: int, lm_fx_ptr: int, kernel: int = KERNEL_AUTO, stream: int = 0):
        """Launch on `stream` (a hipStream_t as int; pass the stream that produced lm_fx). 0/None selects
        the context's internal stream, which is NOT ordered with torch's default stream."""
        check(self.lib.fmgi_bake_items(self.h, begin, end, C.c_void_p(lm_fx_ptr), kernel, C.c_void_p(stream or None)),
              "fmgi_bake_items")

    def finalize(self, lm_fx_ptr: int, texels_in_ptr: int, texels_out_ptr: int, stream: int = 0):
        check(
            self.lib.fmgi_finalize(self.h, C.c_void_p(lm_fx_ptr), C.c_void_p(texels_in_ptr), C.c_void_p(texels_out_ptr),
                                   C.c_void_p(stream or None)),
            "fmgi_finalize",
        )

    def stats(self) -> dict:
        st = Stats()
        check(self.lib.fmgi_get_stats(self.h, C.byref(st)), "fmgi_get_stats")
        return st.as_dict()

    def reset_stats(self):
        check(self.lib.fmgi_reset_stats(self.h), "fmgi_reset_stats")

    def trace_items(self, begin: int, end: int, kernel: int = KERNEL_AUTO):
        """Per-photon bounce records of items [begin, end): (events[n, 800], counts[n], rng_final[n])."""
        n = end - begin
        ev = np.zeros(n * EVENTS_PER_ITEM, EVENT_DTYPE)
        cnt = np.zeros(n, np.int32)
        rng = np.zeros(n, np.uint32)
        check(self.lib.fmgi_trace_items(self.h, begin, end, kernel, _ptr(ev), _ptr(cnt), _ptr(rng)), "fmgi_trace_items")
        return ev.reshape(n, EVENTS_PER_ITEM), cnt, rng

    @property
    def auto_kernel(self) -> int:
        return int(self.lib.fmgi_auto_kernel(self.h))

    @property
    def last_bake_kernel(self) -> str:
        """the profiler's name of the k_bake instance(s) the last bake launch ran (fmgi_last_bake_kernel)"""
        if not hasattr(self.lib, "fmgi_last_bake_kernel"):  # (FMGI_LIB=base: an A/B build that predates it)
            return ""
        n = int(self.lib.fmgi_last_bake_kernel(self.h, None, 0))
        buf = C.create_string_buffer(n + 1)
        self.lib.fmgi_last_bake_kernel(self.h, buf, n + 1)
        return buf.value.decode()

    def set_timing(self, on: bool = True):
        check(self.lib.fmgi_set_timing(self.h, 1 if on else 0), "fmgi_set_timing")

    def timing(self) -> dict:
        """Device time of the bake / fold launches since the previous call (needs set_timing(True))."""
        t = Timing()
        check(self.lib.fmgi_get_timing(self.h, C.byref(t)), "fmgi_get_timing")
        return t.as_dict()

    def set_option(self, name: str, value: int):
        """fmgi_set_option: one of _lib.OPTIONS (chunk_items, pool_limit, stream_layout, bucket_fill, wide_tiles,
        coop, no_axes); takes effect at the next bake (no_axes: the next set_scene)."""
        from ._lib import OPTIONS

        check(self.lib.fmgi_set_option(self.h, OPTIONS[name], int(value)), "fmgi_set_option")

    def set_grid_cells_per_record(self, n: int):
        """The grid's cells per record for the next set_scene (0: the product's choice)."""
        check(self.lib.fmgi_set_grid_cells_per_record(self.h, int(n)), "fmgi_set_grid_cells_per_record")

    def grid_tables(self) -> dict:
        """FMGI_KERNEL_GRID's plane/cell/record tables (include/flatmatch_gi.h fmgi_grid_copy)."""
        sz = np.zeros(5, np.int32)
        check(self.lib.fmgi_grid_sizes(self.h, _ptr(sz)), "fmgi_grid_sizes")
        npairs = int(sz[:3].sum())
        planes = np.zeros(2 * max(npairs, 1), GRID_PLANE_DTYPE)
        cells = np.zeros(int(sz[3]), GRID_CELL_DTYPE)
        recs = np.zeros((int(sz[4]), 4), np.float32)
        idx = np.zeros(int(sz[4]), np.int32)
        check(self.lib.fmgi_grid_copy(self.h, _ptr(planes), _ptr(cells), _ptr(recs), _ptr(idx)), "fmgi_grid_copy")
        return {"J": [int(x) for x in sz[:3]], "planes": planes[: 2 * npairs], "cells": cells, "recs": recs,
                "idx": idx}

    def plan_tables(self) -> dict | None:
        """FMGI_KERNEL_HYBRID's floor plan of the walls (include/flatmatch_gi.h fmgi_plan_copy), or None."""
        n = C.c_int32(0)
        check(self.lib.fmgi_plan_copy(self.h, None, C.byref(n)), "fmgi_plan_copy")
        if n.value == 0:
            return None
        blob = np.zeros(n.value, np.uint8)
        check(self.lib.fmgi_plan_copy(self.h, _ptr(blob), C.byref(n)), "fmgi_plan_copy")
        h0 = blob[:16].view(np.float32)
        h1 = blob[16:32].view(np.int32)
        ncells, nent = int(h1[1]), int(h1[2])
        u16 = blob[32:].view(np.uint16)
        return {"x0": h0[0], "y0": h0[1], "ics": h0[2], "cs": h0[3], "nx": int(h1[0]) & 0xFFFF,
                "ny": int(h1[0]) >> 16, "start": u16[: ncells + 1].copy(),
                "entry": u16[ncells + 1 : ncells + 1 + nent].copy()}

    def filter_image(self) -> dict:
        """The filter image (include/flatmatch_gi.h fmgi_filter_copy): records [n, 8] as float32 (idx in
        column 5 as int32 bits) and the pairs per axis."""
        n = C.c_int32(0)
        J = np.zeros(3, np.int32)
        check(self.lib.fmgi_filter_copy(self.h, None, C.byref(n), _ptr(J)), "fmgi_filter_copy")
        img = np.zeros(n.value // 4, np.float32)
        check(self.lib.fmgi_filter_copy(self.h, _ptr(img), C.byref(n), _ptr(J)), "fmgi_filter_copy")
        recs = img.reshape(-1, 8)
        return {"J": [int(x) for x in J], "recs": recs, "idx": recs[:, 5].view(np.int32).copy()}

    def pair_image(self) -> dict:
        """The hybrid scan's wall-pair image (include/flatmatch_gi.h fmgi_pairs_copy): halves [n, 12] as
        float32 (the two rect indices in columns 10, 11 as int32 bits), two halves (+a, -a) per group, and the
        groups per axis (x, y)."""
        n = C.c_int32(0)
        G = np.zeros(2, np.int32)
        check(self.lib.fmgi_pairs_copy(self.h, None, C.byref(n), _ptr(G)), "fmgi_pairs_copy")
        img = np.zeros(n.value // 4, np.float32)
        check(self.lib.fmgi_pairs_copy(self.h, _ptr(img), C.byref(n), _ptr(G)), "fmgi_pairs_copy")
        halves = img.reshape(-1, 12)
        return {"G": [int(x) for x in G], "halves": halves, "idx": halves[:, 10:12].view(np.int32).copy()}

    def device_sincosf(self, x: np.ndarray, library: bool = False):
        """The samplers' sin/cos on the device (the restatement), or with library=True the device
        library's sinf/cosf that it restates."""
        x = np.ascontiguousarray(x, np.float32)
        s = np.empty_like(x)
        c = np.empty_like(x)
        fn = self.lib.fmgi_device_sincosf_library if library else self.lib.fmgi_device_sincosf
        check(fn(self.h, _ptr(x), _ptr(s), _ptr(c), len(x)), "fmgi_device_sincosf")
        return s, c

    def device_unit(self, op: int, a: np.ndarray, b: np.ndarray | None = None) -> np.ndarray:
        """The bake's device arithmetic helpers (include/flatmatch_gi.h fmgi_device_unit): op 0 = the
        sampler's sqrtf (returns float32), op 1 = (int)(a / b) of the tile index (returns int32)."""
        a = np.ascontiguousarray(a, np.float32)
        bb = None if b is None else np.ascontiguousarray(b, np.float32)
        out = np.empty(len(a), np.int32)
        check(self.lib.fmgi_device_unit(self.h, op, _ptr(a), None if bb is None else _ptr(bb), _ptr(out), len(a)),
              "fmgi_device_unit")
        return out.view(np.float32) if op == 0 else out


GRID_PLANE_DTYPE = np.dtype([("plane", "<f4"), ("u0", "<f4"), ("v0", "<f4"), ("iu", "<f4"), ("iv", "<f4"),
                             ("mu", "<f4"), ("mv", "<f4"), ("nu", "<i4"), ("nv", "<i4"), ("cell_off", "<i4"),
                             ("ulo", "<f4"), ("uhi", "<f4"), ("vlo", "<f4"), ("vhi", "<f4"),
                             ("pad0", "<f4"), ("pad1", "<f4")])
assert GRID_PLANE_DTYPE.itemsize == 64
GRID_CELL_DTYPE = np.dtype([("q0", "<u4", (2,)), ("q1", "<u4", (2,)), ("count", "<i4"), ("idx0", "<i4"),
                            ("idx1", "<i4"), ("rest", "<i4")])
assert GRID_CELL_DTYPE.itemsize == 32


def make_geometry(sc: Scene, texels: np.ndarray):
    """A reference Geometry struct pointing at numpy arrays (kept alive by the returned tuple)."""
    keep = [np.ascontiguousarray(a) for a in (sc.windows, sc.lights, sc.walls)]
    g = Geometry()
    g.windows, g.lights, g.walls = (a.ctypes.data if len(a) else None for a in keep)
    g.boxWalls = None
    g.numWindows, g.numLights, g.numWalls = len(keep[0]), len(keep[1]), len(keep[2])
    g.numBoxWalls = 0
    g.numTexels = sc.num_texels
    g.texels = texels.ctypes.data
    return g, keep


def experiments() -> bool:
    """Whether the loaded library is the experiment build (reads the experiment knobs)."""
    return bool(load().fmgi_experiments())


def dropin_release():
    """Free the device state the drop-in entry points cache across calls (fmgi_dropin_release)."""
    load().fmgi_dropin_release()


def dropin_rccl_ranks() -> int:
    """Ranks of the RCCL communicator the last drop-in call reduced over (0: reduced without RCCL)."""
    return int(load().fmgi_dropin_rccl_ranks())


def dropin_shards(items: int, ngpu: int, nshard: int):
    """The drop-in's multi-GPU layout: (device, begin, end) per shard (fmgi_dropin_shards)."""
    dev = np.zeros(nshard, np.int32)
    b = np.zeros(nshard, np.uint64)
    e = np.zeros(nshard, np.uint64)
    check(load().fmgi_dropin_shards(items, ngpu, nshard, _ptr(dev), _ptr(b), _ptr(e)), "fmgi_dropin_shards")
    return dev, b, e


def dropin_reduce_order(nshard: int):
    """The drop-in's shard reduction: (dst, src) pairs in execution order (fmgi_dropin_reduce_order)."""
    dst = np.zeros(max(nshard, 1), np.int32)
    src = np.zeros(max(nshard, 1), np.int32)
    n = check(load().fmgi_dropin_reduce_order(nshard, _ptr(dst), _ptr(src)), "fmgi_dropin_reduce_order")
    return dst[:n], src[:n]


def bake_geometry(sc: Scene, spa: int, texels: np.ndarray | None = None) -> np.ndarray:
    """getGlobalIlluminationCl: bake on host arrays; consumes libc rand() like the reference."""
    tin = sc.texels() if texels is None else np.ascontiguousarray(texels, np.float32)
    out = np.empty_like(tin)
    g, keep = make_geometry(sc, tin)
    check(load().getGlobalIlluminationCl(C.byref(g), spa, out.ctypes.data_as(C.c_void_p)), "getGlobalIlluminationCl")
    del keep
    return out


# ---- ambient occlusion (include/flatmatch_gi.h) ----------------------------------

def ambient_occlusion(sc: Scene, wall_begin: int = 0, wall_end: int | None = None,
                      texels: np.ndarray | None = None) -> np.ndarray:
    """The reference's performAmbientOcclusionNative on the GPU (fmgi_ambient_occlusion): returns
    float32 [numTexels, 4] = `texels` (default zeros) with the level-0 texels of walls
    [wall_begin, wall_end) replaced by (d, d, d, 0)."""
    lib = load()
    tex = np.zeros((sc.num_texels, 4), np.float32) if texels is None else np.ascontiguousarray(texels, np.float32)
    out = np.empty_like(tex)
    g, keep = make_geometry(sc, tex)
    we = len(sc.walls) if wall_end is None else wall_end
    check(lib.fmgi_ambient_occlusion(C.byref(g), wall_begin, we, _ptr(out)), "fmgi_ambient_occlusion")
    return out


def radiosity(sc: Scene, with_sids: bool = False):
    """The reference's performRadiosityNative on the GPU (fmgi_radiosity): returns float32 [numTexels, 4]
    texels, and with with_sids also the int32 [jobs, 10000] sourceTexelIds rows of the level-0 wall
    texels. Consumes the process's libc rand() stream exactly as the reference does."""
    lib = load()
    tex = np.zeros((sc.num_texels, 4), np.float32)
    out = np.empty_like(tex)
    g, keep = make_geometry(sc, tex)
    jobs = int(lib.fmgi_radiosity_jobs(C.byref(g)))
    sids = np.zeros((jobs, 10000), np.int32) if with_sids else None
    check(lib.fmgi_radiosity(C.byref(g), _ptr(out), _ptr(sids) if with_sids else None), "fmgi_radiosity")
    return (out, sids) if with_sids else out


def radiosity_stats() -> dict:
    """fmgi_radiosity_stats: the last radiosity call's sizes and device phase times."""
    lib = load()
    st = RadStats()
    check(lib.fmgi_radiosity_stats(C.byref(st)), "fmgi_radiosity_stats")
    return st.as_dict()


def geosphere(levels: int = 4) -> np.ndarray:
    """The AO direction table (fmgi_geosphere): float32 [n, 3] in the reference's order."""
    lib = load()
    n = lib.fmgi_geosphere(levels, None, 0)
    if n < 0:
        raise FmgiError(lib.fmgi_last_error().decode())
    out = np.zeros((n, 3), np.float32)
    lib.fmgi_geosphere(levels, _ptr(out), n)
    return out


def ao_tree(sc: Scene) -> np.ndarray:
    """The AO BSP tree (fmgi_ao_tree encoding)."""
    lib = load()
    tex = np.zeros((sc.num_texels, 4), np.float32)
    g, keep = make_geometry(sc, tex)
    n = lib.fmgi_ao_tree(C.byref(g), None, 0)
    if n < 0:
        raise FmgiError(lib.fmgi_last_error().decode())
    out = np.zeros(max(n, 1), np.int32)
    lib.fmgi_ao_tree(C.byref(g), _ptr(out), n)
    return out[:n]


def output_tiles(sc: Scene, texels: np.ndarray, spa: int, tint_extra: int = 0):
    """The output step on the GPU (fmgi_output_tiles): (normalised texels, RGB8 bytes of every tile)."""
    lib = load()
    tex = np.ascontiguousarray(texels, np.float32)
    out = np.empty_like(tex)
    g, keep = make_geometry(sc, tex)
    n = lib.fmgi_output_tile_bytes(C.byref(g))
    rgb = np.zeros(max(n, 1), np.uint8)
    check(lib.fmgi_output_tiles(C.byref(g), spa, tint_extra, _ptr(out), _ptr(rgb)), "fmgi_output_tiles")
    return out, rgb[:n]
