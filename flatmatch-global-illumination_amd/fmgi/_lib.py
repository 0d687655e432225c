"""ctypes binding of libflatmatch_gi.so (include/flatmatch_gi.h). No fallback: if the HIP library is
missing or a call fails, an exception is raised -- there is no CPU path in the product."""
from __future__ import annotations

import ctypes as C
import os

PKG_DIR = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
# FMGI_LIB=<name> selects a profiling/experiment build libflatmatch_gi_<name>.so (make -C <pkg> timing,
# make -C <pkg> experiments (FMGI_LIB=exp: the experiment knobs), make -C <pkg> variant VNAME=<name> VFLAGS=...);
# the product and every test use libflatmatch_gi.so
LIB_PATH = os.path.join(PKG_DIR, f"libflatmatch_gi_{os.environ['FMGI_LIB']}.so" if os.environ.get("FMGI_LIB")
                        else "libflatmatch_gi.so")

# Exported symbols of the C ABI (tests check the built library exports exactly these + nothing
# that would clash with the reference objects main.c links against).
EXPORTS = (
    "performGlobalIlluminationCl",
    "getGlobalIlluminationCl",
    "fmgi_dropin_release",
    "fmgi_dropin_shards",
    "fmgi_dropin_reduce_order",
    "fmgi_dropin_rccl_ranks",
    "fmgi_version",
    "fmgi_last_error",
    "fmgi_device_count",
    "fmgi_create",
    "fmgi_destroy",
    "fmgi_set_scene",
    "fmgi_set_accumulation",
    "fmgi_get_accumulation",
    "fmgi_plan",
    "fmgi_get_plan",
    "fmgi_plan_count",
    "fmgi_bake_items",
    "fmgi_finalize",
    "fmgi_get_stats",
    "fmgi_reset_stats",
    "fmgi_trace_items",
    "fmgi_host_sincosf",
    "fmgi_device_sincosf",
    "fmgi_device_sincosf_library",
    "fmgi_device_unit",
    "fmgi_grid_sizes",
    "fmgi_set_grid_cells_per_record",
    "fmgi_experiments",
    "fmgi_set_option",
    "fmgi_grid_copy",
    "fmgi_plan_copy",
    "fmgi_filter_copy",
    "fmgi_pairs_copy",
    "fmgi_get_stage_cycles",
    "fmgi_auto_kernel",
    "fmgi_last_bake_kernel",
    "fmgi_set_timing",
    "fmgi_get_timing",
    "performAmbientOcclusionGpu",
    "fmgi_ambient_occlusion",
    "fmgi_geosphere",
    "fmgi_ao_tree",
    "fmgi_output_tiles",
    "fmgi_output_tile_bytes",
    "performRadiosityGpu",
    "fmgi_radiosity",
    "fmgi_radiosity_jobs",
    "fmgi_radiosity_stats",
    "fmgi_rand_skip",
)

KERNEL_EXACT = 0
KERNEL_FAST = 1
KERNEL_GRID = 2
KERNEL_HYBRID = 4
KERNEL_AUTO = 3
ACCUM_AUTO = 0
ACCUM_FX3 = 1
ACCUM_STATE = 2
ACCUM_NONE = 3  # profiling only: deposits discarded
ACCUM_STREAM = 4
# fmgi_set_option (include/flatmatch_gi.h): tests' handles on product paths a scene would not take
OPTIONS = {"chunk_items": 1, "pool_limit": 2, "stream_layout": 3, "bucket_fill": 4, "wide_tiles": 5, "coop": 6,
           "no_axes": 7}


class FmgiError(RuntimeError):
    pass


class Stats(C.Structure):
    _fields_ = [
        ("photons", C.c_uint64),
        ("scans", C.c_uint64),
        ("deposits", C.c_uint64),
        ("escapes", C.c_uint64),
        ("exact_rescans", C.c_uint64),
        ("tests", C.c_uint64),
        ("rescans_tie", C.c_uint64),
        ("rescans_invalid", C.c_uint64),
        ("stream_overflow", C.c_uint64),
    ]

    def as_dict(self):
        return {k: int(getattr(self, k)) for k, _ in self._fields_}


class Timing(C.Structure):
    _fields_ = [
        ("bake_ms", C.c_double),
        ("fold_ms", C.c_double),
        ("bake_launches", C.c_uint64),
        ("fold_launches", C.c_uint64),
    ]

    def as_dict(self):
        return {k: (float if k.endswith("ms") else int)(getattr(self, k)) for k, _ in self._fields_}


class RadStats(C.Structure):
    """fmgi_rad_stats (include/flatmatch_gi.h)."""

    _fields_ = [
        ("jobs", C.c_int64),
        ("rects", C.c_int64),
        ("texels", C.c_int64),
        ("rays", C.c_int64),
        ("rand_ms", C.c_double),
        ("rays_ms", C.c_double),
        ("bounce_ms", C.c_double),
        ("total_ms", C.c_double),
    ]

    def as_dict(self):
        return {k: (float if k.endswith("ms") else int)(getattr(self, k)) for k, _ in self._fields_}


class Geometry(C.Structure):
    """geometry.h:7-15 (80 B)."""

    _fields_ = [
        ("windows", C.c_void_p),
        ("lights", C.c_void_p),
        ("walls", C.c_void_p),
        ("boxWalls", C.c_void_p),
        ("numWindows", C.c_int32),
        ("numLights", C.c_int32),
        ("numWalls", C.c_int32),
        ("numBoxWalls", C.c_int32),
        ("width", C.c_int32),
        ("height", C.c_int32),
        ("startingPositionX", C.c_float),
        ("startingPositionY", C.c_float),
        ("numTexels", C.c_int32),
        ("texels", C.c_void_p),
    ]


assert C.sizeof(Geometry) == 80

_lib = None


def load() -> C.CDLL:
    """Load the in-tree HIP library (built by __graft_entry__.build() / `make -C <pkg>`)."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise FmgiError(f"{LIB_PATH} is missing: build it with `make -C {PKG_DIR}` (no CPU fallback exists)")
    # One HIP runtime per process: PyTorch-ROCm wheels bundle their own libamdhip64. Loaded first, it
    # satisfies this library's libamdhip64 dependency too; loaded second, a process ends up with two
    # runtimes that enumerate devices independently (observed: one of them then sees no GPU).
    try:
        import torch  # noqa: F401
    except ImportError:
        pass
    lib = C.CDLL(LIB_PATH)
    vp, i32, i64, u64 = C.c_void_p, C.c_int32, C.c_int64, C.c_uint64
    sig = {
        "fmgi_version": (C.c_char_p, []),
        "fmgi_last_error": (C.c_char_p, []),
        "fmgi_device_count": (C.c_int, []),
        "fmgi_create": (vp, [C.c_int]),
        "fmgi_destroy": (None, [vp]),
        "fmgi_set_scene": (C.c_int, [vp, vp, C.c_int, vp, C.c_int, vp, C.c_int, C.c_int]),
        "fmgi_set_accumulation": (C.c_int, [vp, C.c_int]),
        "fmgi_get_accumulation": (C.c_int, [vp]),
        "fmgi_plan": (i64, [vp, C.c_int, C.c_int, vp, i64, C.POINTER(u64)]),
        "fmgi_get_plan": (i64, [vp, vp, i64]),
        "fmgi_plan_count": (i64, [vp, C.c_int, vp, C.c_int, C.c_int, C.c_int, C.POINTER(u64)]),
        "fmgi_bake_items": (C.c_int, [vp, u64, u64, vp, C.c_int, vp]),
        "fmgi_finalize": (C.c_int, [vp, vp, vp, vp, vp]),
        "fmgi_get_stats": (C.c_int, [vp, C.POINTER(Stats)]),
        "fmgi_reset_stats": (C.c_int, [vp]),
        "fmgi_trace_items": (C.c_int, [vp, u64, u64, C.c_int, vp, vp, vp]),
        "fmgi_host_sincosf": (None, [vp, vp, vp, i64]),
        "fmgi_device_sincosf": (C.c_int, [vp, vp, vp, vp, i64]),
        "fmgi_dropin_shards": (C.c_int, [C.c_uint64, C.c_int, C.c_int, vp, vp, vp]),
        "fmgi_dropin_reduce_order": (C.c_int, [C.c_int, vp, vp]),
        "fmgi_dropin_release": (None, []),
        "fmgi_dropin_rccl_ranks": (C.c_int, []),
        "fmgi_device_sincosf_library": (C.c_int, [vp, vp, vp, vp, i64]),
        "fmgi_device_unit": (C.c_int, [vp, C.c_int, vp, vp, vp, i64]),
        "fmgi_grid_sizes": (C.c_int, [vp, vp]),
        "fmgi_set_grid_cells_per_record": (C.c_int, [vp, C.c_int]),
        "fmgi_experiments": (C.c_int, []),
        "fmgi_set_option": (C.c_int, [vp, C.c_int, C.c_int64]),
        "fmgi_get_stage_cycles": (C.c_int, [vp, vp]),
        "fmgi_auto_kernel": (C.c_int, [vp]),
        "fmgi_last_bake_kernel": (C.c_int, [vp, C.c_char_p, C.c_int]),
        "fmgi_set_timing": (C.c_int, [vp, C.c_int]),
        "fmgi_get_timing": (C.c_int, [vp, C.POINTER(Timing)]),
        "performAmbientOcclusionGpu": (None, [vp]),
        "fmgi_ambient_occlusion": (C.c_int, [vp, C.c_int, C.c_int, vp]),
        "fmgi_geosphere": (C.c_int, [C.c_int, vp, C.c_int]),
        "fmgi_ao_tree": (i64, [vp, vp, i64]),
        "fmgi_output_tiles": (C.c_int, [vp, C.c_int, C.c_int, vp, vp]),
        "fmgi_output_tile_bytes": (i64, [vp]),
        "performRadiosityGpu": (None, [vp]),
        "fmgi_radiosity": (C.c_int, [vp, vp, vp]),
        "fmgi_radiosity_jobs": (i64, [vp]),
        "fmgi_radiosity_stats": (C.c_int, [C.POINTER(RadStats)]),
        "fmgi_rand_skip": (C.c_int, [C.c_uint64]),
        "fmgi_grid_copy": (C.c_int, [vp, vp, vp, vp, vp]),
        "fmgi_plan_copy": (C.c_int, [vp, vp, vp]),
        "fmgi_filter_copy": (C.c_int, [vp, vp, vp, vp]),
        "fmgi_pairs_copy": (C.c_int, [vp, vp, vp, vp]),
        "getGlobalIlluminationCl": (C.c_int, [C.POINTER(Geometry), C.c_int, vp]),
        "performGlobalIlluminationCl": (None, [C.POINTER(Geometry), C.c_int]),
    }
    for name, (res, args) in sig.items():
        try:
            f = getattr(lib, name)
        except AttributeError:
            if os.environ.get("FMGI_LIB") == "base":  # an A/B build of an earlier commit may predate a symbol
                continue
            raise
        f.restype = res
        f.argtypes = args
    _ = i32
    _lib = lib
    return lib


def last_error() -> str:
    msg = load().fmgi_last_error()
    return msg.decode() if msg else ""


def check(rc: int, what: str) -> int:
    if rc < 0:
        raise FmgiError(f"{what} failed ({rc}): {last_error()}")
    return rc
