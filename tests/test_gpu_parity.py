"""GPU parity tests: the HIP path (through the C ABI) against the oracle, bit for bit.

Every comparison here is exact: per-photon bounce records (hit rectangle, texel, deposited RGB bits,
RNG state), int64 fixed-point lightmaps, counters, and the finalised float texels. Sizes are the
ones the oracle finishes in seconds; full-size configs are covered by size-independent properties
(split invariance, determinism, photon/deposit accounting).
"""
import ctypes as C
import os

import numpy as np
import pytest

import fm_oracle as O
import fmgi
from conftest import GOLDEN

pytestmark = pytest.mark.gpu

KERNELS = [fmgi.KERNEL_EXACT, fmgi.KERNEL_FAST, fmgi.KERNEL_GRID, fmgi.KERNEL_HYBRID]




@pytest.fixture(scope="module")
def offsets():
    return np.load(os.path.join(GOLDEN, "glibc_rand_4096.npy"))


def _ctx(sc, spa, offsets, accum=fmgi.ACCUM_AUTO):
    ctx = fmgi.Context(0)
    ctx.set_accumulation(accum)
    ctx.set_scene(sc)
    ctx.plan(spa, rng_offsets=offsets)
    return ctx


def _oracle_plan(sc, spa, offsets):
    return O.schedule_with_offsets(sc, spa, offsets)


def _bake_gpu(torch, ctx, b, e, kernel):
    s = torch.cuda.Stream()
    with torch.cuda.stream(s):  # zero-fill and bake ordered on one (non-default) stream
        lm = torch.zeros((ctx.scene.num_texels, 4), dtype=torch.int64, device="cuda")
        ctx.bake_items(b, e, lm.data_ptr(), kernel, s.cuda_stream)
    s.synchronize()
    return lm.cpu().numpy()


def test_device_sincos_bitwise_on_every_reachable_phi(torch_cuda, box200, offsets):
    """The samplers' sin/cos restatement (fmgi_math.h) on the device == the device library's sinf/cosf
    (ROCm ocml: what photonmap.cl's sin/cos execute on MI355X) == the host restatement, on all 83,886,081
    reachable phi."""
    phi = O.reachable_phi()
    assert len(phi) == 83_886_081
    ctx = _ctx(box200, 1000, offsets)
    ds, dc = ctx.device_sincosf(phi)
    ls, lc = ctx.device_sincosf(phi, library=True)
    hs, hc = fmgi.host_sincosf(phi)
    assert np.array_equal(ds.view(np.uint32), ls.view(np.uint32))
    assert np.array_equal(dc.view(np.uint32), lc.view(np.uint32))
    assert np.array_equal(ds.view(np.uint32), hs.view(np.uint32))
    assert np.array_equal(dc.view(np.uint32), hc.view(np.uint32))
    ctx.close()


def _compare_traces(sc, ctx, L, b, e, kernel):
    ev, cnt, rngf = ctx.trace_items(b, e, kernel)
    for w in range(b, e):
        li = int(np.searchsorted(L["item_begin"], w, side="right") - 1)
        gid = w - int(L[li]["item_begin"])
        state = (gid + int(L[li]["rng_offset"])) & 0xFFFFFFFF
        oev, ofin = O.trace_item(sc, int(L[li]["source"]), int(L[li]["is_window"]), state)
        k = w - b
        assert cnt[k] == len(oev), f"item {w}: {cnt[k]} vs {len(oev)} bounces"
        g = ev[k, : cnt[k]]
        assert np.array_equal(g.view(np.uint32), oev.view(np.uint32).reshape(g.view(np.uint32).shape)), f"item {w}"
        assert rngf[k] == ofin, f"item {w}: final RNG"


@pytest.mark.parametrize("kernel", KERNELS)
def test_per_photon_traces_example(torch_cuda, example_scene, offsets, kernel):
    spa = 65_000
    L = _oracle_plan(example_scene, spa, offsets)
    ctx = _ctx(example_scene, spa, offsets)
    assert ctx.get_plan().tobytes() == L.tobytes()
    _compare_traces(example_scene, ctx, L, 0, 256, kernel)  # window 0
    _compare_traces(example_scene, ctx, L, 10_240, 10_304, kernel)  # first light (isWindow = 0)
    ctx.close()


@pytest.mark.parametrize("kernel", KERNELS)
def test_per_photon_traces_boxes(torch_cuda, box200, box2000, offsets, kernel):
    for sc, n in ((box200, 128), (box2000, 16)):
        spa = 172_413_793
        L = _oracle_plan(sc, spa, offsets)
        ctx = _ctx(sc, spa, offsets)
        _compare_traces(sc, ctx, L, 1000, 1000 + n, kernel)
        ctx.close()


def test_box_traces_without_axes_mode(torch_cuda, box200, offsets):
    """The closed boxes use ScanGrid's one-plane-per-class phase 1; FMGI_OPT_NO_AXES routes them through
    the sorted <= 4-slot phase 1 instead, which no other scene here reaches: same traces."""
    spa = 172_413_793
    L = _oracle_plan(box200, spa, offsets)
    ctx = fmgi.Context(0)
    ctx.set_option("no_axes", 1)
    ctx.set_scene(box200)
    ctx.plan(spa, rng_offsets=offsets)
    _compare_traces(box200, ctx, L, 3000, 3128, fmgi.KERNEL_GRID)
    lm = _bake_gpu(torch_cuda, ctx, 5_000, 25_000, fmgi.KERNEL_GRID)
    olm, _ = O.bake(box200, L, 5_000, 25_000)
    assert np.array_equal(lm[:, :3], olm)
    ctx.close()


def test_layout_traces_with_floor_plan(torch_cuda, example_scene, offsets):
    """The hybrid scan's walls through the packed wall-pair filter (default, FMGI_FILTER_PK=1:
    filter_pairs over the pair image) and, in the experiment build, through the floor-plan walk (FMGI_PLAN=1,
    plan_walls): both give the oracle's traces and lightmap."""
    spa = 6_500_000
    L = _oracle_plan(example_scene, spa, offsets)
    ctx = _ctx(example_scene, spa, offsets)
    olm, _ = O.bake(example_scene, L, 40_000, 52_000)
    for env in ("0", "1") if fmgi.experiments() else ("0",):
        os.environ["FMGI_PLAN"] = env
        try:
            _compare_traces(example_scene, ctx, L, 41_000, 41_128, fmgi.KERNEL_HYBRID)
            lm = _bake_gpu(torch_cuda, ctx, 40_000, 52_000, fmgi.KERNEL_HYBRID)
            assert np.array_equal(lm[:, :3], olm), f"FMGI_PLAN={env}"
        finally:
            os.environ.pop("FMGI_PLAN", None)
    ctx.close()


ACCUMS = [fmgi.ACCUM_FX3, fmgi.ACCUM_STATE, fmgi.ACCUM_STREAM]


@pytest.mark.parametrize("accum", ACCUMS)
@pytest.mark.parametrize("kernel", KERNELS)
def test_lightmap_config1_exact(torch_cuda, example_scene, offsets, kernel, accum):
    """BASELINE config 1 (example.png, 1.1e6 photons): GPU int64 lightmap == oracle, bit for bit."""
    spa = 65_000
    L = _oracle_plan(example_scene, spa, offsets)
    ctx = _ctx(example_scene, spa, offsets, accum)
    assert ctx.accumulation == accum
    ctx.reset_stats()
    lm = _bake_gpu(torch_cuda, ctx, 0, ctx.total_items, kernel)
    olm, ost = O.bake(example_scene, L)
    assert np.array_equal(lm[:, :3], olm)
    assert not lm[:, 3].any()
    st = ctx.stats()
    for k in ("photons", "scans", "deposits", "escapes"):
        assert st[k] == ost[k], k
    ctx.close()


@pytest.mark.parametrize("accum", ACCUMS)
@pytest.mark.parametrize("kernel", KERNELS)
def test_lightmap_box_prefix_exact(torch_cuda, box200, box2000, offsets, kernel, accum):
    for sc, items in ((box200, 20_000), (box2000, 1_000)):
        spa = 172_413_793
        L = _oracle_plan(sc, spa, offsets)
        ctx = _ctx(sc, spa, offsets, accum)
        lm = _bake_gpu(torch_cuda, ctx, 5_000, 5_000 + items, kernel)
        olm, _ = O.bake(sc, L, 5_000, 5_000 + items)
        assert np.array_equal(lm[:, :3], olm)
        ctx.close()


# stream layout -> the context options that select it (fmgi_set_option; the product library's layouts)
FOLD_LAYOUTS = {
    "buckets_ring": {"bucket_fill": 0, "wide_tiles": 0},
    "buckets_scatter": {"bucket_fill": 1, "wide_tiles": 0},
    "buckets_scatter_wide": {"bucket_fill": 1, "wide_tiles": 1},
    "buckets_ring_wide": {"bucket_fill": 0, "wide_tiles": 1},
    "sliced": {"stream_layout": 0},
}
# ... and the experiment build's (make experiments, FMGI_LIB=exp: its environment knobs), skipped otherwise
EXP_LAYOUTS = {
    "dense_bin": {"FMGI_PRESORT": "2", "FMGI_DENSE": "1"},
    "dense_bin_wide": {"FMGI_PRESORT": "2", "FMGI_DENSE": "1", "FMGI_WIDE_TILES": "1"},
    # wide bucket tiles folded as 2 or 4 narrower fold tiles that read the same blocks
    "buckets_scatter_wide_split2": {"FMGI_WIDE_TILES": "1", "FMGI_FOLD_SPLIT": "2"},
    "buckets_scatter_w13_split2": {"FMGI_WIDE_TILES": "13", "FMGI_FOLD_SPLIT": "2"},
    "presorted": {"FMGI_PRESORT": "1"},
    "sliced_packed": {"FMGI_PRESORT": "0", "FMGI_PACKED_RUNS": "1"},
    "fold_carry": {"FMGI_FOLD_CARRY": "2", "FMGI_WIDE_TILES": "1"},
}
EXP_ENV = sorted({k for v in EXP_LAYOUTS.values() for k in v})


def _layout_ctx(name, sc, spa, offsets):
    """a STREAM context on layout `name` (FOLD_LAYOUTS options, or EXP_LAYOUTS environment)"""
    for k in EXP_ENV:
        os.environ.pop(k, None)
    if name in EXP_LAYOUTS:
        if not fmgi.experiments():
            pytest.skip("an experiment build's layout (make experiments; FMGI_LIB=exp)")
        os.environ.update(EXP_LAYOUTS[name])
    ctx = _ctx(sc, spa, offsets, fmgi.ACCUM_STREAM)
    for k, v in FOLD_LAYOUTS.get(name, {}).items():
        ctx.set_option(k, v)
    return ctx


@pytest.mark.parametrize("layout", sorted(FOLD_LAYOUTS) + sorted(EXP_LAYOUTS))
def test_stream_fold_orders_exact(torch_cuda, box200, example_scene, offsets, layout):
    """Every STREAM layout gives the oracle's lightmap: per-tile buckets (the default for lightmaps of at most
    63 fold tiles) filled through the bake's per-wave LDS rings (buckets_ring) or lane by lane (buckets_scatter),
    with 2048- or 4096-texel tiles, and the slice-sorted stream (lightmaps of more than 63 tiles); for full-ring
    flushes and the partial rings / blocks at the end of a launch. The experiment build's layouts (the dense
    stream binned by k_bin, split folds, 8192-texel tiles, presorted segments, packed slice runs, the fold's
    carry words) when that build is loaded."""
    try:
        for sc, spa, lo, hi in ((box200, 172_413_793, 7_000, 27_000), (example_scene, 65_000, 0, 300)):
            L = _oracle_plan(sc, spa, offsets)
            ctx = _layout_ctx(layout, sc, spa, offsets)
            lm = _bake_gpu(torch_cuda, ctx, lo, hi, fmgi.KERNEL_AUTO)
            olm, _ = O.bake(sc, L, lo, hi)
            assert np.array_equal(lm[:, :3], olm), sc.name
            assert ctx.stats()["stream_overflow"] == 0
            ctx.close()
    finally:
        for k in EXP_ENV:
            os.environ.pop(k, None)


@pytest.mark.parametrize("layout", ["buckets_ring", "buckets_scatter", "dense_bin"])
def test_bucket_pool_exhaustion_falls_back_exactly(torch_cuda, box200, offsets, layout):
    """A bucket pool that runs out (FMGI_OPT_POOL_LIMIT caps it at 64 blocks, far fewer than the bake needs)
    sends the rest of the codes through device atomics into the int64 lightmap (the bake's bucket_atomic; the
    experiment build's k_bin: bin_atomic), whichever way the buckets are filled: the lightmap still equals the
    oracle's."""
    try:
        spa = 172_413_793
        L = _oracle_plan(box200, spa, offsets)
        ctx = _layout_ctx(layout, box200, spa, offsets)
        ctx.set_option("pool_limit", 64)
        lm = _bake_gpu(torch_cuda, ctx, 2_000, 6_000, fmgi.KERNEL_AUTO)
        olm, _ = O.bake(box200, L, 2_000, 6_000)
        assert np.array_equal(lm[:, :3], olm)
        ctx.close()
    finally:
        for k in EXP_ENV:
            os.environ.pop(k, None)


def test_split_invariance_and_determinism_full_size(torch_cuda, box200, offsets):
    """Config 3 sized work (a 1e8-photon slice): order-free exact accumulation means any split of the
    item range, and any repetition, gives identical bits."""
    spa = 172_413_793
    ctx = _ctx(box200, spa, offsets, fmgi.ACCUM_STATE)
    n = ctx.total_items  # BASELINE config 3 at full size: 1,000,012,800 photons
    a = _bake_gpu(torch_cuda, ctx, 0, n, fmgi.KERNEL_GRID)
    b1 = _bake_gpu(torch_cuda, ctx, 0, n // 3, fmgi.KERNEL_GRID)
    b2 = _bake_gpu(torch_cuda, ctx, n // 3, n, fmgi.KERNEL_GRID)
    ctx.set_accumulation(fmgi.ACCUM_FX3)
    c = _bake_gpu(torch_cuda, ctx, 0, n, fmgi.KERNEL_GRID)
    ctx.set_accumulation(fmgi.ACCUM_STREAM)
    d = _bake_gpu(torch_cuda, ctx, 0, n, fmgi.KERNEL_GRID)  # one memory-sized chunk
    ctx.set_option("chunk_items", 3_000_000)  # four chunks through one buffer set ...
    e = _bake_gpu(torch_cuda, ctx, 0, n, fmgi.KERNEL_GRID)
    f = e
    if fmgi.experiments():  # ... and (experiment build) with each fold beside the next chunk's bake
        os.environ["FMGI_PIPELINE"] = "3"
        try:
            f = _bake_gpu(torch_cuda, ctx, 0, n, fmgi.KERNEL_GRID)
        finally:
            os.environ.pop("FMGI_PIPELINE", None)
    ctx.set_option("chunk_items", 0)
    ctx.set_option("stream_layout", 0)  # the slice-sorted fold (lightmaps of more than 63 fold tiles)
    g = _bake_gpu(torch_cuda, ctx, 0, n, fmgi.KERNEL_GRID)
    ctx.set_option("stream_layout", -1)
    d1 = _bake_gpu(torch_cuda, ctx, 0, 12_345, fmgi.KERNEL_GRID)
    d2 = _bake_gpu(torch_cuda, ctx, 12_345, n, fmgi.KERNEL_GRID)
    assert np.array_equal(a, b1 + b2)
    assert np.array_equal(a, c)  # the accumulation modes agree bit for bit
    assert np.array_equal(a, d)
    assert np.array_equal(a, e)
    assert np.array_equal(a, f)
    assert np.array_equal(a, g)
    assert np.array_equal(a, d1 + d2)
    assert ctx.stats()["stream_overflow"] == 0
    ctx.reset_stats()
    _bake_gpu(torch_cuda, ctx, 0, n, fmgi.KERNEL_GRID)
    st = ctx.stats()
    assert st["photons"] == 100 * n
    assert st["deposits"] + st["escapes"] == st["scans"]
    # the grid's phase 1 in a closed box: ~2 record tests per scan on the coarse grid staged in LDS (5 cells
    # per record), ~1.5 on the 16-per-record grid (FMGI_CELLS_LDS=0)
    assert st["tests"] < 2.5 * st["scans"]
    # energy accounting: the lightmap total equals the sum over deposits (every deposit >= 0.25)
    assert int(a[:, :3].astype(np.float64).sum()) >= st["deposits"] * 3 * (2**25 // 4)
    ctx.close()


def test_finalize_matches_oracle(torch_cuda, example_scene, offsets):
    spa = 65_000
    ctx = _ctx(example_scene, spa, offsets)
    L = _oracle_plan(example_scene, spa, offsets)
    olm, _ = O.bake(example_scene, L, 0, 2000)
    rng = np.random.default_rng(1)
    tin = rng.random((example_scene.num_texels, 4), dtype=np.float32) * 100
    torch = torch_cuda
    lm = torch.zeros((example_scene.num_texels, 4), dtype=torch.int64)
    lm[:, :3] = torch.from_numpy(olm)
    s = torch.cuda.Stream()
    with torch.cuda.stream(s):
        lm = lm.cuda()
        t_in = torch.from_numpy(tin).cuda()
        t_out = torch.empty_like(t_in)
        ctx.finalize(lm.data_ptr(), t_in.data_ptr(), t_out.data_ptr(), s.cuda_stream)
    s.synchronize()
    assert np.array_equal(t_out.cpu().numpy().view(np.uint32), O.finalize(olm, tin).view(np.uint32))
    ctx.close()


def test_drop_in_entry_points(torch_cuda, example_scene, libc):
    """performGlobalIlluminationCl / getGlobalIlluminationCl: same texels as the oracle, and libc rand()
    consumed exactly once per reference launch."""
    spa = 65_000
    golden = np.load(os.path.join(GOLDEN, "glibc_rand_4096.npy"))
    libc.srand(1)
    out = fmgi.bake_geometry(example_scene, spa)
    assert libc.rand() == golden[10]  # 10 launches consumed 10 values
    L = _oracle_plan(example_scene, spa, golden)
    olm, _ = O.bake(example_scene, L)
    exp = O.finalize(olm, example_scene.texels())
    assert np.array_equal(out.view(np.uint32), exp.view(np.uint32))

    # in place, starting from non-zero texels (the callee adds to existing values)
    tex = np.full((example_scene.num_texels, 4), 0.5, np.float32)
    g, keep = fmgi.make_geometry(example_scene, tex)
    libc.srand(1)
    os.environ["FMGI_QUIET"] = "1"
    fmgi._lib.load().performGlobalIlluminationCl(C.byref(g), spa)
    exp2 = O.finalize(olm, np.full_like(tex, 0.5))
    assert np.array_equal(tex.view(np.uint32), exp2.view(np.uint32))


def test_reference_kernel_pins_oracle(torch_cuda, example_scene, offsets):
    """The reference's own photonmap.cl (compiled for gfx950 with ROCm's OpenCL device libraries,
    IEEE div/sqrt, no contraction) run one work item per launch vs the oracle's fp32 per-item sums."""
    if not O.ref_kernel_available("strict"):
        pytest.skip("oracle/_ref not built (needs /root/reference at build time)")
    spa = 65_000
    L = _oracle_plan(example_scene, spa, offsets)
    states = [(g + int(L[0]["rng_offset"])) & 0xFFFFFFFF for g in range(32)]
    ref = O.ref_run_items(example_scene, 0, 1, states, "strict")  # never "fast": it faults (build_ref.sh)
    same = 0
    for k, st in enumerate(states):
        mine = O.trace_item_f32(example_scene, 0, 1, st)
        same += np.array_equal(mine.view(np.uint32), ref[k].view(np.uint32))
    # the strict build is the oracle's arithmetic contract: every item bit for bit (as the committed
    # tests/golden/ref_items_*_strict.npz fixtures record)
    assert same == 32, f"only {same}/32 work items bit-identical to the reference kernel"


def test_multi_shard_drop_in_is_bit_identical(torch_cuda, box200, libc):
    """performGlobalIlluminationCl sharded over FMGI_SHARDS work-item ranges (the multi-GPU path, here
    round-robin on one device) reduces to exactly the single-shard texels."""
    spa = 2_000_000
    outs = []
    for shards in ("1", "3"):
        os.environ["FMGI_SHARDS"] = shards
        try:
            libc.srand(1)
            outs.append(fmgi.bake_geometry(box200, spa))
        finally:
            del os.environ["FMGI_SHARDS"]
    assert np.array_equal(outs[0].view(np.uint32), outs[1].view(np.uint32))
    assert outs[0][:, :3].sum() > 0


def test_rccl_reduce_path_and_cache_modes(torch_cuda, box200, libc):
    """The drop-in's RCCL reduce (FMGI_REDUCE=rccl: ncclCommInitAll over the shard devices, one int64
    ncclReduce into shard 0; on one GPU a one-rank communicator) gives the same texels as the default path;
    shards that share a device refuse it (RCCL allows one rank per GPU) and reduce by peer copies instead.
    FMGI_DROPIN_CACHE=1 (default) frees the stream buffers after the call, 2 keeps them."""
    from fmgi._lib import FmgiError

    spa = 2_000_000
    fmgi.dropin_release()
    libc.srand(1)
    ref = fmgi.bake_geometry(box200, spa)
    assert fmgi.dropin_rccl_ranks() == 0  # one shard, default: nothing to reduce
    os.environ["FMGI_REDUCE"] = "rccl"
    try:
        libc.srand(1)
        out = fmgi.bake_geometry(box200, spa)
        assert fmgi.dropin_rccl_ranks() == 1
        assert np.array_equal(out.view(np.uint32), ref.view(np.uint32))
        os.environ["FMGI_SHARDS"] = "2"
        libc.srand(1)
        with pytest.raises(FmgiError, match="one shard per device"):
            fmgi.bake_geometry(box200, spa)
    finally:
        os.environ.pop("FMGI_REDUCE", None)
        os.environ.pop("FMGI_SHARDS", None)
    fmgi.dropin_release()
    assert fmgi.dropin_rccl_ranks() == 0
    # device memory the call leaves behind: a few MB by default, the stream buffers (GBs) with cache 2
    from fmgi import scene

    example = scene.load_geometry(os.path.join(GOLDEN, "example_geometry.bin"), "example")
    torch_cuda.cuda.synchronize()
    free0 = torch_cuda.cuda.mem_get_info()[0]
    libc.srand(1)
    fmgi.bake_geometry(example, 6_500_000)  # BASELINE config 2: ~3 GB of deposit codes
    free1 = torch_cuda.cuda.mem_get_info()[0]
    assert free0 - free1 < (256 << 20), (free0 - free1) / 2**20
    os.environ["FMGI_DROPIN_CACHE"] = "2"
    try:
        libc.srand(1)
        fmgi.bake_geometry(example, 6_500_000)
        free2 = torch_cuda.cuda.mem_get_info()[0]
        assert free0 - free2 > (1 << 30), (free0 - free2) / 2**20
    finally:
        os.environ.pop("FMGI_DROPIN_CACHE", None)
    fmgi.dropin_release()
