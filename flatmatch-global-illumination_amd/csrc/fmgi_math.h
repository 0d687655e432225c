/*
 * fmgi_math.h -- bit-reproducible fp32 sin/cos for the photon samplers (host C/C++ and HIP device).
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

FMGI_HD void fmgi_sincos_kernel(double r, double *s, double *c) {
    const double S1 = -1.66666666666666324348e-01, S2 = 8.33333333332248946124e-03,
                 S3 = -1.98412698298579493134e-04, S4 = 2.75573137070700676789e-06,
                 S5 = -2.50507602534068634195e-08, S6 = 1.58969099521155010221e-10;
    const double C1 = 4.16666666666666019037e-02, C2 = -1.38888888888741095749e-03,
                 C3 = 2.48015872894767294178e-05, C4 = -2.75573143513906633035e-07,
                 C5 = 2.08757232129817482790e-09, C6 = -1.13596475577881948265e-11;
    double z = r * r;
    double v = z * r;
    double ps = S2 + z * (S3 + z * (S4 + z * (S5 + z * S6)));
    *s = r + v * (S1 + z * ps);
    double pc = z * (C1 + z * (C2 + z * (C3 + z * (C4 + z * (C5 + z * C6)))));
    double hz = 0.5 * z;
    double w = 1.0 - hz;
    *c = w + (((1.0 - w) - hz) + z * pc);
}

/* sin and cos of a float in [0, 8); result bits == (float)sin((double)x), (float)cos((double)x). */
FMGI_HD void fmgi_sincosf(float xf, float *sf, float *cf) {
    const double INV_PIO2 = 6.36619772367581382433e-01;
    const double P1 = 1.57079632673412561417e+00; /* first 33 bits of pi/2 */
    const double P2 = 6.07710050650619224932e-11; /* pi/2 - P1 */
    double x = (double)xf;
    int k = (int)(x * INV_PIO2 + 0.5);
    double dk = (double)k;
    double r = (x - dk * P1) - dk * P2;
    double s, c;
    fmgi_sincos_kernel(r, &s, &c);
    /* quadrant k: (sin, cos) = (s, c), (c, -s), (-s, -c), (-c, s); rounding to float commutes with
       negation, so the swap and the signs are applied after it (selects, no branches) */
    const float s32 = (float)s, c32 = (float)c;
    const float so = (k & 1) ? c32 : s32, co = (k & 1) ? s32 : c32;
    *sf = (k & 2) ? -so : so;
    *cf = ((k + 1) & 2) ? -co : co;
}

#endif
