/*
 * fmgi_math.h -- bit-reproducible fp32 sin/cos for the photon samplers (host C++ and HIP device).
 *
 * photonmap.cl:36-37/60-61 evaluate `cos(phi)` and `sin(phi)` on a float phi in [0, 6.283184].
 * The parity contract fixes these to (float)sin((double)phi) and
 * (float)cos((double)phi). Device libm results are not bit-specified, so this header evaluates both
 * in IEEE double with a fixed sequence of plain double ops (no FMA contraction, no libm) and rounds
 * once to float: the same bits on x86-64 and on gfx950. tests/test_math.py checks it against glibc on
 * EVERY reachable phi (all 6.283184f * rand() values, ~8.4e7 inputs).
 *
 * Reduction: k = nearest multiple of pi/2 (k <= 4), r = (x - k*P1) - k*P2 with a 33-bit P1 (exact
 * product and difference) and its tail P2. Kernels: fdlibm-style minimax polynomials on |r| <= pi/4.
 */
#ifndef FMGI_MATH_H
#define FMGI_MATH_H

#if defined(__HIPCC__)
#define FMGI_HD __host__ __device__ __forceinline__
#else
#define FMGI_HD static inline
#endif

#if defined(__clang__)
#pragma clang fp contract(off)
#endif

/* The double constants of the evaluation. The device reads them through a pointer (BakeArgs::sincos)
   with scalar loads: a VOP3 double op takes no literal on gfx9, so literals cost two s_mov_b32 each per
   use. The values are the same either way; only where they come from differs. */
struct FmgiSinCosCoef {
    double S1, S2, S3, S4, S5, S6;
    double C1, C2, C3, C4, C5, C6;
    double inv_pio2, p1, p2, pad;
};
#define FMGI_SINCOS_COEF_INIT                                                                                  \
    {-1.66666666666666324348e-01, 8.33333333332248946124e-03, -1.98412698298579493134e-04,                     \
     2.75573137070700676789e-06,  -2.50507602534068634195e-08, 1.58969099521155010221e-10,                     \
     4.16666666666666019037e-02,  -1.38888888888741095749e-03, 2.48015872894767294178e-05,                     \
     -2.75573143513906633035e-07, 2.08757232129817482790e-09,  -1.13596475577881948265e-11,                    \
     6.36619772367581382433e-01,  1.57079632673412561417e+00 /* first 33 bits of pi/2 */,                      \
     6.07710050650619224932e-11 /* pi/2 - P1 */, 0.0}
static const FmgiSinCosCoef kFmgiSinCos = FMGI_SINCOS_COEF_INIT;

template <class K>
FMGI_HD void fmgi_sincos_kernel(double r, const K &k, double *s, double *c) {
    double z = r * r;
    double v = z * r;
    double ps = k->S2 + z * (k->S3 + z * (k->S4 + z * (k->S5 + z * k->S6)));
    *s = r + v * (k->S1 + z * ps);
    double pc = z * (k->C1 + z * (k->C2 + z * (k->C3 + z * (k->C4 + z * (k->C5 + z * k->C6)))));
    double hz = 0.5 * z;
    double w = 1.0 - hz;
    *c = w + (((1.0 - w) - hz) + z * pc);
}

/* sin and cos of a float in [0, 8); result bits == (float)sin((double)x), (float)cos((double)x).
   k points at the FmgiSinCosCoef values (host: &kFmgiSinCos). */
template <class K>
FMGI_HD void fmgi_sincosf_k(float xf, const K &k, float *sf, float *cf) {
    double x = (double)xf;
    int q = (int)(x * k->inv_pio2 + 0.5);
    double dk = (double)q;
    double r = (x - dk * k->p1) - dk * k->p2;
    double s, c;
    fmgi_sincos_kernel(r, k, &s, &c);
    /* quadrant q: (sin, cos) = (s, c), (c, -s), (-s, -c), (-c, s); rounding to float commutes with
       negation, so the swap and the signs are applied after it (selects, no branches) */
    const float s32 = (float)s, c32 = (float)c;
    const float so = (q & 1) ? c32 : s32, co = (q & 1) ? s32 : c32;
    *sf = (q & 2) ? -so : so;
    *cf = ((q + 1) & 2) ? -co : co;
}

FMGI_HD void fmgi_sincosf(float xf, float *sf, float *cf) {
    const FmgiSinCosCoef *k = &kFmgiSinCos;
    fmgi_sincosf_k(xf, k, sf, cf);
}

#endif
