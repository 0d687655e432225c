"""ctypes wrapper of oracle/liboracle.so -- the CPU ORACLE (TEST INFRASTRUCTURE ONLY).

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg import this module, as the
checker / CPU baseline; the product (libflatmatch_gi.so, fmgi) never does. See fm_oracle.h.
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB = os.path.join(HERE, "liboracle.so")

LAUNCH_DTYPE = np.dtype(
    [("item_begin", "<u8"), ("count", "<u4"), ("rng_offset", "<i4"), ("source", "<i4"), ("is_window", "<i4")]
)
EVENT_DTYPE = np.dtype(
    [("photon", "<i4"), ("depth", "<i4"), ("rect", "<i4"), ("texel", "<i4"), ("rgb", "<f4", 3), ("rng", "<u4")]
)


class OracleStats(C.Structure):
    _fields_ = [(k, C.c_uint64) for k in ("photons", "scans", "deposits", "escapes", "inexact")]

    def as_dict(self):
        return {k: int(getattr(self, k)) for k, _ in self._fields_}


_lib = None
_hw_tables = None
HW_TABLES = os.path.join(os.path.dirname(HERE), "tests", "golden", "gfx950_sqrt_rsq.npz")


def hw_tables():
    """gfx950's v_sqrt_f32 / v_rsq_f32 as int8 ulp deltas [2^24] each (recorded on the MI355X by
    tools/hw_sqrt_rsq_table.hip; packed 2 bits per entry in tests/golden/gfx950_sqrt_rsq.npz)."""
    d = np.load(HW_TABLES)
    out = []
    for k in ("sqrt", "rsq"):
        p = d[k]
        v = np.empty(4 * len(p), np.int8)
        for j in range(4):
            v[j::4] = ((p >> (2 * j)) & 3).astype(np.int8) - 1
        out.append(np.ascontiguousarray(v))
    return out


def build():
    subprocess.run(["make", "-s", "-C", HERE], check=True)


def load():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB):
            build()
        lib = C.CDLL(LIB)
        vp, i64, u64 = C.c_void_p, C.c_int64, C.c_uint64
        lib.fmo_schedule_count.restype = i64
        lib.fmo_schedule_count.argtypes = [vp, C.c_int, C.c_int, C.c_int, C.c_int, C.POINTER(u64)]
        lib.fmo_schedule.restype = i64
        lib.fmo_schedule.argtypes = [vp, C.c_int, C.c_int, C.c_int, C.c_int, vp, i64]
        lib.fmo_bake.restype = None
        lib.fmo_bake.argtypes = [vp, C.c_int, vp, vp, i64, u64, u64, vp, i64, C.c_int, C.POINTER(OracleStats)]
        lib.fmo_bake_counts.restype = None
        lib.fmo_bake_counts.argtypes = [vp, C.c_int, vp, vp, i64, u64, u64, vp, vp, i64, C.c_int,
                                        C.POINTER(OracleStats)]
        lib.fmo_trace_item.restype = C.c_int
        lib.fmo_trace_item.argtypes = [vp, C.c_int, vp, C.c_int, C.c_uint32, vp, C.c_int, C.POINTER(C.c_uint32)]
        lib.fmo_trace_item_f32.restype = None
        lib.fmo_trace_item_f32.argtypes = [vp, C.c_int, vp, C.c_int, C.c_uint32, vp]
        lib.fmo_rand.restype = C.c_float
        lib.fmo_rand.argtypes = [C.POINTER(C.c_uint32)]
        lib.fmo_finalize.restype = None
        lib.fmo_finalize.argtypes = [vp, i64, vp, vp]
        lib.ao_oracle.restype = C.c_int
        lib.ao_oracle.argtypes = [vp, C.c_int, C.c_int, C.c_int, vp, C.c_int, vp, C.c_int]
        lib.out_oracle.restype = None
        lib.out_oracle.argtypes = [vp, C.c_int, vp, C.c_int, C.c_int, vp]
        lib.rad_oracle.restype = i64
        lib.rad_oracle.argtypes = [vp, C.c_int, vp, C.c_int, vp, C.c_int, C.c_int, vp, vp, C.c_int]
        lib.ao_oracle_tree.restype = i64
        lib.ao_oracle_tree.argtypes = [vp, C.c_int, vp, i64]
        lib.fmo_sincos_n.restype = None
        lib.fmo_sincos_n.argtypes = [vp, vp, vp, i64]
        lib.fmo_set_hw_tables.restype = None
        lib.fmo_set_hw_tables.argtypes = [vp, vp]
        global _hw_tables
        _hw_tables = hw_tables()
        lib.fmo_set_hw_tables(_p(_hw_tables[0]), _p(_hw_tables[1]))
        _lib = lib
    return _lib


def _p(a):
    return None if a is None or a.size == 0 else a.ctypes.data_as(C.c_void_p)


def schedule(scene, spa: int, wg: int = 256) -> np.ndarray:
    """global_illumination_cl.c:215-272 schedule; calls libc rand() once per launch."""
    lib = load()
    src = np.ascontiguousarray(scene.sources)
    tot = C.c_uint64()
    n = lib.fmo_schedule_count(_p(src), len(scene.windows), len(scene.lights), spa, wg, C.byref(tot))
    out = np.zeros(n, LAUNCH_DTYPE)
    lib.fmo_schedule(_p(src), len(scene.windows), len(scene.lights), spa, wg, _p(out), n)
    return out


def schedule_with_offsets(scene, spa: int, offsets, wg: int = 256) -> np.ndarray:
    """Schedule whose launch k uses offsets[k] instead of rand() (item layout as the reference)."""
    lib = load()
    src = np.ascontiguousarray(scene.sources)
    tot = C.c_uint64()
    n = lib.fmo_schedule_count(_p(src), len(scene.windows), len(scene.lights), spa, wg, C.byref(tot))
    out = np.zeros(n, LAUNCH_DTYPE)
    # build the layout in Python (same arithmetic as fmo_schedule minus rand())
    cap = wg * 100
    item = 0
    k = 0
    f32 = np.float32
    for s_idx, s in enumerate(scene.sources):
        w, h = s["width"][:3], s["height"][:3]
        lw = f32(np.sqrt(f32(f32(f32(w[0] * w[0]) + f32(w[1] * w[1])) + f32(w[2] * w[2]))))
        lh = f32(np.sqrt(f32(f32(f32(h[0] * h[0]) + f32(h[1] * h[1])) + f32(h[2] * h[2]))))
        area = f32(lw * lh)
        nitems = int(f32(f32(f32(spa) * area) / f32(100)))
        nitems = (nitems // wg + 1) * wg
        while nitems:
            ws = min(nitems, cap)
            nitems -= ws
            out[k] = (item, ws, int(offsets[k]), s_idx, int(s_idx < len(scene.windows)))
            item += ws
            k += 1
    assert k == n and item == tot.value
    return out


def bake(scene, launches: np.ndarray, item_begin: int = 0, item_end: int | None = None, nthreads: int = 0,
         counts: bool = False):
    """Exact fixed-point lightmap (int64 [numTexels, 3], units of 2^-25) of items [begin, end);
    counts=True also returns every texel's deposit count (int64 [numTexels])."""
    lib = load()
    if item_end is None:
        item_end = int(launches["item_begin"][-1] + launches["count"][-1]) if len(launches) else 0
    walls = np.ascontiguousarray(scene.walls)
    src = np.ascontiguousarray(scene.sources)
    L = np.ascontiguousarray(launches, LAUNCH_DTYPE)
    lm = np.zeros((scene.num_texels, 3), np.int64)
    st = OracleStats()
    if counts:
        cnt = np.zeros(scene.num_texels, np.int64)
        lib.fmo_bake_counts(_p(walls), len(walls), _p(src), _p(L), len(L), item_begin, item_end, _p(lm), _p(cnt),
                            scene.num_texels, nthreads, C.byref(st))
        return lm, st.as_dict(), cnt
    lib.fmo_bake(_p(walls), len(walls), _p(src), _p(L), len(L), item_begin, item_end, _p(lm), scene.num_texels,
                 nthreads, C.byref(st))
    return lm, st.as_dict()


_port = None


def bake_port(scene, launches: np.ndarray, item_begin: int = 0, item_end: int | None = None, nthreads: int = 0):
    """bake() through liboracle_port.so: the same restatement with the per-rect builtin values hoisted out
    of the scan and FMA instructions (bit-identical, tests/test_oracle.py) -- bench.py's CPU baseline."""
    global _port
    load()
    if _port is None:
        vp, i64, u64 = C.c_void_p, C.c_int64, C.c_uint64
        lib = C.CDLL(os.path.join(HERE, "liboracle_port.so"))
        lib.fmo_bake.restype = None
        lib.fmo_bake.argtypes = [vp, C.c_int, vp, vp, i64, u64, u64, vp, i64, C.c_int, C.POINTER(OracleStats)]
        lib.fmo_set_hw_tables.restype = None
        lib.fmo_set_hw_tables.argtypes = [vp, vp]
        lib.fmo_set_hw_tables(_p(_hw_tables[0]), _p(_hw_tables[1]))
        _port = lib
    if item_end is None:
        item_end = int(launches["item_begin"][-1] + launches["count"][-1]) if len(launches) else 0
    walls = np.ascontiguousarray(scene.walls)
    src = np.ascontiguousarray(scene.sources)
    L = np.ascontiguousarray(launches, LAUNCH_DTYPE)
    lm = np.zeros((scene.num_texels, 3), np.int64)
    st = OracleStats()
    _port.fmo_bake(_p(walls), len(walls), _p(src), _p(L), len(L), item_begin, item_end, _p(lm), scene.num_texels,
                   nthreads, C.byref(st))
    return lm, st.as_dict()


def trace_item(scene, source: int, is_window: int, rng_state: int, cap: int = 800):
    lib = load()
    walls = np.ascontiguousarray(scene.walls)
    src = np.ascontiguousarray(scene.sources[source : source + 1])
    ev = np.zeros(cap, EVENT_DTYPE)
    fin = C.c_uint32()
    n = lib.fmo_trace_item(_p(walls), len(walls), _p(src), is_window, rng_state & 0xFFFFFFFF, _p(ev), cap, C.byref(fin))
    return ev[: min(n, cap)], int(fin.value)


def trace_item_f32(scene, source: int, is_window: int, rng_state: int) -> np.ndarray:
    lib = load()
    walls = np.ascontiguousarray(scene.walls)
    src = np.ascontiguousarray(scene.sources[source : source + 1])
    tex = np.zeros((scene.num_texels, 4), np.float32)
    lib.fmo_trace_item_f32(_p(walls), len(walls), _p(src), is_window, rng_state & 0xFFFFFFFF, _p(tex))
    return tex


def finalize(lm_fx: np.ndarray, texels_in: np.ndarray) -> np.ndarray:
    lib = load()
    lm = np.ascontiguousarray(lm_fx, np.int64)
    tin = np.ascontiguousarray(texels_in, np.float32)
    out = np.empty_like(tin)
    lib.fmo_finalize(_p(lm), len(tin), _p(tin), _p(out))
    return out


def sincos(x: np.ndarray):
    """The oracle's sin/cos of the samplers (ROCm device-library algorithm) over an array."""
    lib = load()
    x = np.ascontiguousarray(x, np.float32)
    s, c = np.empty_like(x), np.empty_like(x)
    lib.fmo_sincos_n(_p(x), _p(s), _p(c), len(x))
    return s, c


def reachable_phi() -> np.ndarray:
    """Every phi = 6.283184f * rand() the samplers can draw (photonmap.cl:33,57; rand() = (float)s * 2^-32
    for a u32 s, photonmap.cl:21-25): 83,886,081 values, in increasing order."""
    parts = [np.arange(0, 2**24, dtype=np.float64)]
    for e in range(24, 32):
        parts.append(np.arange(2.0**e, 2.0 ** (e + 1), 2.0 ** (e - 23)))
    parts.append(np.array([2.0**32]))
    f = np.concatenate(parts).astype(np.float32)
    return np.float32(6.283184) * (f * np.float32(2.0**-32))


def rand_sequence(state: int, n: int) -> np.ndarray:
    lib = load()
    s = C.c_uint32(state)
    return np.array([lib.fmo_rand(C.byref(s)) for _ in range(n)], np.float32)


# ---- the reference kernel itself (GPU only): oracle/_ref/photonmap_*.hsaco via libref_runner.so ----
REF_DIR = os.path.join(HERE, "_ref")
_ref = None


def ref_kernel_available(variant: str = "strict") -> bool:
    return os.path.exists(os.path.join(REF_DIR, f"photonmap_{variant}.hsaco")) and os.path.exists(
        os.path.join(HERE, "libref_runner.so"))


def _ref_open(variant: str):
    if variant not in ("strict", "relaxed"):
        raise ValueError(f"reference variant {variant!r} is not launchable")
    global _ref
    if _ref is None:
        _ref = C.CDLL(os.path.join(HERE, "libref_runner.so"))
        _ref.ref_open.argtypes = [C.c_char_p]
        _ref.ref_last_error.restype = C.c_char_p
        _ref.ref_run_items.argtypes = [C.c_void_p, C.c_void_p, C.c_int, C.c_int, C.c_int, C.c_void_p, C.c_int,
                                       C.c_void_p]
        _ref.ref_run_sum.restype = C.c_longlong
        _ref.ref_run_sum.argtypes = [C.c_void_p, C.c_void_p, C.c_int, C.c_int, C.c_int, C.c_void_p, C.c_int,
                                     C.c_int, C.c_void_p]
    path = os.path.join(REF_DIR, f"photonmap_{variant}.hsaco")
    if _ref.ref_open(path.encode()) != 0:
        raise RuntimeError(_ref.ref_last_error().decode())
    return _ref


def ref_run_sum(scene, launches: np.ndarray, item_begin: int, item_end: int, variant: str = "strict",
                streams: int = 16) -> np.ndarray:
    """The race-free sum of the reference kernel's per-item lightmaps over flattened items [begin, end) of
    a schedule (each item run alone on a zeroed buffer, as ref_run_items), exact in int64 fixed point
    (units of 2^-25, [numTexels, 3]): what the reference computes for those items without its data race,
    with its own per-item fp32 accumulation."""
    ref = _ref_open(variant)
    walls = np.ascontiguousarray(scene.walls)
    srcs = np.ascontiguousarray(scene.sources)
    out = np.zeros((scene.num_texels, 3), np.int64)
    for L in launches:
        lo, hi = max(int(L["item_begin"]), item_begin), min(int(L["item_begin"]) + int(L["count"]), item_end)
        if lo >= hi:
            continue
        gids = np.arange(lo - int(L["item_begin"]), hi - int(L["item_begin"]), dtype=np.int64)
        states = ((gids + int(L["rng_offset"])) & 0xFFFFFFFF).astype(np.uint32)
        win = np.ascontiguousarray(srcs[int(L["source"]) : int(L["source"]) + 1])
        bad = ref.ref_run_sum(_p(win), _p(walls), len(walls), scene.num_texels, int(L["is_window"]), _p(states),
                              len(states), streams, _p(out))
        if bad < 0:
            raise RuntimeError(ref.ref_last_error().decode())
        if bad:
            raise RuntimeError(f"{bad} per-item texel values not multiples of 2^-25")
    return out


def ref_run_items(scene, source: int, is_window: int, rng_states, variant: str = "strict") -> np.ndarray:
    """Run the reference photonmap kernel (photonmap.cl:269) once per work item, each on a zeroed
    lightColors buffer; returns float32 [n, numTexels, 4]. Variant "fast" is refused: built with the
    reference's -cl-fast-relaxed-math it faults on the first escaping photon (see build_ref.sh)."""
    _ref = _ref_open(variant)
    walls = np.ascontiguousarray(scene.walls)
    win = np.ascontiguousarray(scene.sources[source : source + 1])
    rs = np.ascontiguousarray(rng_states, np.uint32)
    out = np.zeros((len(rs), scene.num_texels, 4), np.float32)
    if _ref.ref_run_items(_p(win), _p(walls), len(walls), scene.num_texels, is_window, _p(rs), len(rs), _p(out)) != 0:
        raise RuntimeError(_ref.ref_last_error().decode())
    return out


def ambient_occlusion(scene, wall_begin: int = 0, wall_end: int | None = None, dirs=None, nthreads: int = 0):
    """The reference's performAmbientOcclusionNative restated (ao_oracle.c) on walls [wall_begin,
    wall_end): float32 [numTexels, 4] texels, zero except those walls' level-0 texels. `dirs` is the
    direction table (default: oracle/geosphere.py level 4, the reference's geoSphere4)."""
    import geosphere

    lib = load()
    walls = np.ascontiguousarray(scene.walls)
    we = len(walls) if wall_end is None else wall_end
    d = np.ascontiguousarray(geosphere.generate(4) if dirs is None else dirs, dtype=np.float32)
    tex = np.zeros((scene.num_texels, 4), np.float32)
    threads = nthreads or int(os.environ.get("OMP_NUM_THREADS", "0") or 0) or (os.cpu_count() or 1)
    lib.ao_oracle(_p(walls), len(walls), wall_begin, we, _p(d), len(d), _p(tex), threads)
    return tex


def ao_tree(scene) -> np.ndarray:
    """The oracle's BSP tree in fmgi_ao_tree's encoding."""
    lib = load()
    walls = np.ascontiguousarray(scene.walls)
    n = lib.ao_oracle_tree(_p(walls), len(walls), None, 0)
    out = np.zeros(max(n, 1), np.int32)
    lib.ao_oracle_tree(_p(walls), len(walls), _p(out), n)
    return out[:n]


def output_tiles(scene, texels: np.ndarray, spa: int, tint_extra: int):
    """main.c:66-79 normalisation (spa > 0) + saveAs_core tone map / floor tint (out_oracle.c):
    returns (normalised float32 [numTexels, 4] texels, uint8 RGB bytes of every wall's tile)."""
    lib = load()
    walls = np.ascontiguousarray(scene.walls)
    tex = np.array(texels, dtype=np.float32, copy=True)
    n = int(sum(int(w["lm"][1]) * int(w["lm"][2]) for w in walls))
    rgb = np.zeros(3 * n, np.uint8)
    lib.out_oracle(_p(walls), len(walls), _p(tex), spa, tint_extra, _p(rgb))
    return tex, rgb


RAD_RAYS = 10000  # geoSphereNumVectors, radiosityNative.c:151


def radiosity(scene, nthreads: int = 0, with_sids: bool = False):
    """The reference's performRadiosityNative restated (rad_oracle.c). Consumes libc rand() exactly as
    the reference does (2 x 10000 values per level-0 wall texel), from the process's current state.
    Returns float32 [numTexels, 4] texels, and with with_sids the int32 [jobs, 10000] sourceTexelIds rows
    of the level-0 wall texels (wall/tile order)."""
    lib = load()
    walls, win, lights = (np.ascontiguousarray(a) for a in (scene.walls, scene.windows, scene.lights))
    jobs = int(sum(int(w["lm"][1]) * int(w["lm"][2]) for w in walls))
    tex = np.zeros((scene.num_texels, 4), np.float32)
    sids = np.zeros((jobs, RAD_RAYS), np.int32) if with_sids else None
    threads = nthreads or int(os.environ.get("OMP_NUM_THREADS", "0") or 0) or (os.cpu_count() or 1)
    n = lib.rad_oracle(_p(walls), len(walls), _p(win), len(win), _p(lights), len(lights), scene.num_texels,
                       _p(tex), _p(sids) if with_sids else None, threads)
    if n < 0:
        raise MemoryError("rad_oracle: allocation failed")
    return (tex, sids) if with_sids else tex
