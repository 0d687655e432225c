/*
 * fmgi_math.h -- the photon samplers' sin/cos, bit-reproducible on host C++ and the HIP device.
 *
 * photonmap.cl:36-37/60-61 evaluate `cos(phi)` and `sin(phi)` on a float phi in [0, 6.283184]. On the
 * MI355X the reference kernel gets them from ROCm's device library (ocml.bc: __ocml_sin_f32 /
 * __ocml_cos_f32); this header restates that fp32 algorithm with explicit FMAs, so host and device
 * produce the library's bits. tests/test_gpu_parity.py checks the device restatement against the device
 * library on EVERY reachable phi (all 6.283184f * rand() values, 83,886,081 inputs), and
 * tests/test_math.py the host restatement against the oracle's on all of them.
 */
#ifndef FMGI_MATH_H
#define FMGI_MATH_H

#include <math.h>

#if defined(__HIPCC__)
#define FMGI_HD __host__ __device__ __forceinline__
#else
#define FMGI_HD static inline
#endif

#if defined(__clang__)
#pragma clang fp contract(off)
#endif

/* sin and cos of a float in [0, 2^17) exactly as ROCm's device library computes them for gfx9+ (the
   fast-FMA reduction path of __ocmlpriv_trigredsmall_f32 and __ocmlpriv_sincosred_f32): k = x * 2/pi
   rounded to the nearest integer, a three-part Cody-Waite reduction with FMAs, minimax polynomials
   (every llvm.fmuladd of the library is an FMA on gfx950), quadrant k & 3. */
FMGI_HD void fmgi_sincosf(float x, float *sf, float *cf) {
    const float k = rintf(x * 0x1.45f306p-1f);
    float r = fmaf(k, -0x1.921fb4p+0f, x);
    r = fmaf(k, -0x1.4442d0p-24f, r);
    r = fmaf(k, -0x1.846988p-48f, r);
    const int q = (int)k & 3;
    const float z = r * r;
    float p = fmaf(z, -0x1.983304p-13f, 0x1.110388p-7f);
    p = fmaf(z, p, -0x1.55553ap-3f);
    p = z * p;
    const float sn = fmaf(r, p, r);
    float cp = fmaf(z, 0x1.aea668p-16f, -0x1.6c9e76p-10f);
    cp = fmaf(z, cp, 0x1.5557eep-5f);
    cp = fmaf(z, cp, -0x1.000008p-1f);
    const float cs = fmaf(z, cp, 1.0f);
    /* quadrant q: (sin, cos) = (s, c), (c, -s), (-s, -c), (-c, s) */
    const float so = (q & 1) ? cs : sn, co = (q & 1) ? -sn : cs;
    *sf = q > 1 ? -so : so;
    *cf = q > 1 ? -co : co;
}

#endif
