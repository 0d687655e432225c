"""GPU: the bake kernel's arithmetic shortcuts against IEEE references (fmgi_device_unit).

csrc/fmgi_core.h replaces two correctly rounded operations of photonmap.cl by cheaper device sequences
that must give the same bits:
  - sqrt_cr, the samplers' sqrt (photonmap.cl:33,39,57,63): checked on EVERY float the samplers can
    pass it, {0} and [2^-32, 1] (rand() >= 2^-32 when nonzero; 1 - r*r >= 2^-24 when nonzero);
  - trunc_div, the (int)(dx * W / len) of getTileIdAt (photonmap.cl:108-109): checked on quotients next
    to every integer 0..W for many lengths (the band where the fast path must defer) and on random ones.
"""
import numpy as np
import pytest

import fmgi

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def ctx(torch_cuda, box200):
    c = fmgi.Context(0)
    c.set_scene(box200)
    yield c
    c.close()


def test_sampler_sqrt_on_every_reachable_float(ctx):
    lo, hi = np.float32(2.0**-32).view(np.uint32), np.float32(1.0).view(np.uint32)
    step = 1 << 25
    bad = 0
    for b0 in range(int(lo), int(hi) + 1, step):
        bits = np.arange(b0, min(b0 + step, int(hi) + 1), dtype=np.uint32)
        x = bits.view(np.float32)
        got = ctx.device_unit(fmgi.UNIT_SQRT, x)
        bad += int(np.count_nonzero(got.view(np.uint32) != np.sqrt(x).view(np.uint32)))
    zero = ctx.device_unit(fmgi.UNIT_SQRT, np.zeros(1, np.float32))
    assert zero.view(np.uint32)[0] == 0
    assert bad == 0


def test_tile_trunc_div_near_every_integer(ctx):
    rng = np.random.default_rng(7)
    lens = np.concatenate([rng.uniform(0.05, 20.0, 400), [1.0, 0.5, 2.0, 1.6666666, 1.3333334, 0.1, 10.0]])
    xs, ys = [], []
    for W in (1, 2, 8, 64, 256, 1024):
        for y in lens.astype(np.float32):
            k = np.arange(0, W + 1, dtype=np.float32)
            base = (k * y).astype(np.float32)  # x / y lands next to the integer k
            for d in range(-4, 5):
                xs.append(np.nextafter(base, np.float32(np.inf) if d > 0 else np.float32(0)) if d else base)
                if abs(d) > 1:
                    for _ in range(abs(d) - 1):
                        xs[-1] = np.nextafter(xs[-1], np.float32(np.inf) if d > 0 else np.float32(0))
                ys.append(np.full(len(base), y, np.float32))
    x = np.abs(np.concatenate(xs)).astype(np.float32)
    y = np.concatenate(ys)
    xr = (rng.uniform(0, 1, 2_000_000) * 1024).astype(np.float32)
    yr = rng.uniform(0.01, 30, 2_000_000).astype(np.float32)
    x, y = np.concatenate([x, xr]), np.concatenate([y, yr])
    keep = (x / y) < 2.0**30
    x, y = x[keep], y[keep]
    want = np.trunc(x / y).astype(np.int64)  # float32 division: correctly rounded
    for op in (fmgi.UNIT_TRUNC_DIV, fmgi.UNIT_TRUNC_DIV_INV):
        got = ctx.device_unit(op, x, y)
        assert np.array_equal(got.astype(np.int64), want), op
