/*
 * fmgi_core.h -- device-side data layout and the exact photon-step arithmetic.
 *
 * Everything in this header is evaluated with IEEE fp32 ops in the order of photonmap.cl
 * (this translation unit is compiled with -ffp-contract=off and correctly rounded div/sqrt) and the
 * OpenCL builtins as ROCm implements them for gfx950, so the results are bit-identical to the oracle
 * contract (oracle/fm_oracle.h) and to the reference kernel built for MI355X.
 */
#ifndef FMGI_CORE_H
#define FMGI_CORE_H

#include <stdint.h>
#include <math.h>

#include "fmgi_math.h"

#if defined(__clang__)
#pragma clang fp contract(off)
#endif

#define FMGI_FX_SHIFT 25        /* fixed point: one unit = 2^-25 (every deposit channel is a multiple) */
#define FMGI_PHOTONS_PER_ITEM 100 /* photonmap.cl:279 */
#define FMGI_MAX_DEPTH 8          /* photonmap.cl:171 */
#define FMGI_EVENTS_PER_ITEM (FMGI_PHOTONS_PER_ITEM * FMGI_MAX_DEPTH)

struct f3 { float x, y, z; };

FMGI_HD f3 mkf3(float x, float y, float z) { f3 r; r.x = x; r.y = y; r.z = z; return r; }
FMGI_HD f3 add3(f3 a, f3 b) { return mkf3(a.x + b.x, a.y + b.y, a.z + b.z); }
FMGI_HD f3 sub3(f3 a, f3 b) { return mkf3(a.x - b.x, a.y - b.y, a.z - b.z); }
FMGI_HD f3 mul3(f3 a, float s) { return mkf3(a.x * s, a.y * s, a.z * s); }
FMGI_HD f3 div3(f3 a, float s) { return mkf3(a.x / s, a.y / s, a.z / s); }
/* OpenCL dot and cross as ROCm's device library defines them (opencl.bc; its llvm.fmuladd is an FMA on
   gfx950): what the reference kernel computes on MI355X */
FMGI_HD float dot3(f3 a, f3 b) { return fmaf(a.z, b.z, fmaf(a.y, b.y, a.x * b.x)); }
FMGI_HD f3 cross3(f3 a, f3 b) {
    return mkf3(fmaf(a.y, b.z, -(a.z * b.y)), fmaf(a.z, b.x, -(a.x * b.z)), fmaf(a.x, b.y, -(a.y * b.x)));
}
/* the reference HOST's length() (vector3_cl.c:93, gcc without FMA): the launch schedule's source area */
FMGI_HD float host_len3(f3 a) { return sqrtf(a.x * a.x + a.y * a.y + a.z * a.z); }

/*
 * One wall rectangle as the kernels read it: 128 B (two s_load_dwordx16). Exact fields are the
 * reference Rectangle plus values photonmap.cl recomputes per test, hoisted out of the loop and computed
 * once per scene on the device with the same builtins (k_scene_setup, bit-identical): wn =
 * width/length(width) (photonmap.cl:145), wl = length(width) (:144), hn/hl likewise (:149-150), and the
 * sampler basis of the normal (bu, bv; photonmap.cl:65-70).
 * iwl/ihl serve only tile_uv's fast path, which checks its result against a 2^-20 band.
 */
struct __attribute__((aligned(16))) RectDev {
    float px, py, pz;      /* pos                      */
    float nx, ny, nz;      /* n                        */
    float wnx, wny, wnz;   /* width / length(width)     */
    float wl;              /* length(width)            */
    float hnx, hny, hnz;   /* height / length(height)   */
    float hl;              /* length(height)           */
    int32_t base, W, H;    /* lightmapSetup.s0/s1/s2    */
    int32_t axis;          /* filter class: 0..5 = axis-aligned normal (+x,-x,+y,-y,+z,-z), -1 general */
    float bux, buy, buz;   /* sampler basis udir        */
    float bvx, bvy, bvz;   /* sampler basis vdir        */
    float iwl, ihl;        /* 1/wl, 1/hl correctly rounded (tile_uv's quotient estimate) */
    float pad[6];
};
static_assert(sizeof(RectDev) == 128, "RectDev must be 128 B");

/* The fields of a RectDev the scans' phase 2 and the deposit read, as staged in LDS (BakeArgs::rects_off):
   112 B = 28 dwords, so consecutive records start 28 banks apart (a 128-B stride puts every record's
   field k on the same 4 banks: 64 lanes reading their winners' records then conflict up to 32 ways). */
struct __attribute__((aligned(16))) RectLds {
    float px, py, pz, nx;
    float ny, nz, wnx, wny;
    float wnz, wl, hnx, hny;
    float hnz, hl;
    int32_t base, W;
    int32_t H;
    float bux, buy, buz;
    float bvx, bvy, bvz, iwl;
    float ihl, pad0, pad1, pad2;
};
static_assert(sizeof(RectLds) == 112, "RectLds must be 112 B");

/* One emitter (window or light), photonmap.cl:173-181. */
struct __attribute__((aligned(16))) SrcDev {
    float px, py, pz, wx, wy, wz, hx, hy, hz, nx, ny, nz;
    float bux, buy, buz, bvx, bvy, bvz;
    float pad[14];
};
static_assert(sizeof(SrcDev) == 128, "SrcDev must be 128 B");

struct LaunchDev {
    uint64_t item_begin;
    uint32_t count;
    int32_t rng_offset;
    int32_t source;
    int32_t is_window;
};
static_assert(sizeof(LaunchDev) == 24, "LaunchDev must be 24 B");

/* photonmap.cl:21-25 */
FMGI_HD float rng_next(uint32_t &s) {
    s = s * 1664525u + 1013904223u;
    return (float)s * 2.3283064365386963e-10f; /* == (float)s / (float)0xFFFFFFFF, an exact 2^-32 scale */
}

/* Correctly rounded sqrtf (== sqrtf bit for bit) for x == 0 and 2^-96 <= x < inf: v_sqrt_f32 plus one
   residual correction, i.e. LLVM's gfx9 expansion without its rescaling of tiny inputs. The samplers'
   arguments are rand() in {0} u [2^-32, 1] and 1 - r*r in {0} u [2^-24, 1]. */
FMGI_HD float sqrt_cr(float x) {
#if defined(__HIP_DEVICE_COMPILE__)
    const float y = __builtin_amdgcn_sqrtf(x);
    const float ym = __int_as_float(__float_as_int(y) - 1), yp = __int_as_float(__float_as_int(y) + 1);
    const float rm = fmaf(-ym, y, x), rp = fmaf(-yp, y, x);
    float q = rm <= 0.0f ? ym : y;
    q = rp > 0.0f ? yp : q;
    return x == 0.0f ? x : q;
#else
    return sqrtf(x);
#endif
}

/* photonmap.cl:27-74 with the basis precomputed (k_scene_setup): fold=1 is the window ("sky") sampler */
FMGI_HD f3 sample_dir(uint32_t &rng, f3 n, f3 bu, f3 bv, bool fold) {
    float r = sqrt_cr(rng_next(rng));
    float phi = 6.283184f * rng_next(rng);
    float sn, cs;
    fmgi_sincosf(phi, &sn, &cs);
    float u = r * cs;
    float v = r * sn;
    float w = sqrt_cr(1.0f - r * r);
    if (fold && u < 0) u = -u;
    return add3(add3(mul3(bu, u), mul3(bv, v)), mul3(n, w));
}

/* photonmap.cl:123-158; wn/wl/hn/hl are the hoisted, bit-identical per-rect values. */
FMGI_HD float intersect_exact(f3 n, f3 pos, f3 wn, float wl, f3 hn, float hl, f3 src, f3 dir, float closest) {
    float denom = dot3(n, dir);
    if (denom >= 0) return -1;
    float fac = dot3(n, sub3(pos, src)) / denom;
    if (fac < 0) return -1;
    f3 ray = mul3(dir, fac);
    if (closest * closest < dot3(ray, ray)) return -1;
    f3 pDir = sub3(add3(src, ray), pos);
    float dx = dot3(wn, pDir);
    if (dx < 0 || dx > wl) return -1;
    float dy = dot3(hn, pDir);
    if (dy < 0 || dy > hl) return -1;
    return fac;
}

/* intersect_exact with closest = INFINITY (the early-out never fires), also returning the hit point's
   dx = dot(wn, p - pos) and dy = dot(hn, p - pos): the same ops, in the same order, as tile_at's on the
   point p = src + dir * fac that photonmap.cl:216 moves to, so the deposit needs no second evaluation */
FMGI_HD float intersect_exact_uv(f3 n, f3 pos, f3 wn, float wl, f3 hn, float hl, f3 src, f3 dir, float &dx,
                                 float &dy) {
    float denom = dot3(n, dir);
    if (denom >= 0) return -1;
    float fac = dot3(n, sub3(pos, src)) / denom;
    if (fac < 0) return -1;
    f3 pDir = sub3(add3(src, mul3(dir, fac)), pos);
    dx = dot3(wn, pDir);
    if (dx < 0 || dx > wl) return -1;
    dy = dot3(hn, pDir);
    if (dy < 0 || dy > hl) return -1;
    return fac;
}

/* (int)(x / y) for 0 <= x / y < 2^30 (correctly rounded quotient, truncated), given iy ~ 1/y within
   one ulp. On the device: x * iy is within 2^-21 relative of x / y and of its rounding, so when both
   ends of the +-2^-20 band around it truncate to the same integer, that integer is the answer;
   otherwise (a quotient next to an integer) the exact division decides. */
FMGI_HD int trunc_div_inv(float x, float y, float iy) {
#if defined(__HIP_DEVICE_COMPILE__)
    const float q = x * iy;
    const int lo = (int)(q * 0.99999904632568359375f), hi = (int)(q * 1.00000095367431640625f);
    if (lo == hi) return lo;
#endif
    return (int)(x / y);
}

#if defined(__HIP_DEVICE_COMPILE__)
FMGI_HD int trunc_div(float x, float y) { return trunc_div_inv(x, y, __builtin_amdgcn_rcpf(y)); }
#else
FMGI_HD int trunc_div(float x, float y) { return (int)(x / y); }
#endif

/* photonmap.cl:108-119: the tile of in-rect coordinates (dx, dy); iwl, ihl ~ 1/wl, 1/hl (one ulp) */
FMGI_HD int tile_uv(float dx, float dy, float wl, float hl, float iwl, float ihl, int W, int H) {
    int tx = trunc_div_inv(dx * (float)W, wl, iwl);
    int ty = trunc_div_inv(dy * (float)H, hl, ihl);
    tx = tx < 0 ? 0 : (tx > W - 1 ? W - 1 : tx);
    ty = ty < 0 ? 0 : (ty > H - 1 ? H - 1 : ty);
#if defined(__HIP_DEVICE_COMPILE__)
    return (int)__umul24((uint32_t)ty, (uint32_t)W) + tx; /* 0 <= ty < H, W < 2^24: not the quarter-rate v_mul_lo_u32 */
#else
    return ty * W + tx;
#endif
}

/* Warm-up skip-ahead (photonmap.cl:272-275): `r = rand()*40; for (i=0; i<r; i++) rand();` draws
   ceil(r) values; LCG^k(s) = A[k]*s + C[k]. */
struct LcgJump { uint32_t a[41], c[41]; };

inline void lcg_jump_table(LcgJump &t) {
    uint32_t a = 1, c = 0;
    for (int k = 0; k <= 40; k++) {
        t.a[k] = a;
        t.c[k] = c;
        /* compose one more step: s' = 1664525*(a*s + c) + 1013904223 */
        a = 1664525u * a;
        c = 1664525u * c + 1013904223u;
    }
}

#endif
