/*
 * fm_oracle.c -- CPU ORACLE (TEST INFRASTRUCTURE ONLY; see fm_oracle.h for the contract).
 *
 * Restates, function by function, the reference OpenCL kernel /root/reference/photonmap.cl
 * and the launch schedule of /root/reference/global_illumination_cl.c. Each function cites the
 * lines it follows. Build: oracle/Makefile (gcc -O2 -ffp-contract=off -fopenmp, no fast-math).
 */

#include "fm_oracle.h"

#include <math.h>
#include <stdlib.h>
#include <stdio.h>
#include <string.h>
#ifdef _OPENMP
#include <omp.h>
#endif

typedef struct { float x, y, z; } v3;

static inline v3 mk(float x, float y, float z) { v3 r = {x, y, z}; return r; }
static inline v3 ld(const float *p) { return mk(p[0], p[1], p[2]); }
static inline v3 vadd(v3 a, v3 b) { return mk(a.x + b.x, a.y + b.y, a.z + b.z); }
static inline v3 vsub(v3 a, v3 b) { return mk(a.x - b.x, a.y - b.y, a.z - b.z); }
static inline v3 vmul(v3 a, float s) { return mk(a.x * s, a.y * s, a.z * s); }
static inline v3 vdiv(v3 a, float s) { return mk(a.x / s, a.y / s, a.z / s); }
/*
 * OpenCL builtins as ROCm's device libraries implement them for gfx950 -- what the reference kernel
 * executes on MI355X (opencl.bc / ocml.bc; every llvm.fmuladd there is an FMA on gfx950):
 *   dot(a, b)   = fma(a.z, b.z, fma(a.y, b.y, a.x * b.x))                         (_Z3dotDv3_fS_)
 *   cross(a, b) = (fma(a.y, b.z, -(a.z b.y)), fma(a.z, b.x, -(a.x b.z)), fma(a.x, b.y, -(a.y b.x)))
 *   length(v)   = v_sqrt_f32(dot(v, v)) (llvm.sqrt with !fpmath 3.0), rescaled below 2^-126 / at inf
 *   normalize(v)= v * v_rsq_f32(dot(v, v)) (__ocml_rsqrt_f32), rescaled likewise; v if v == 0
 * v_sqrt_f32 and v_rsq_f32 are within 1 ulp, not correctly rounded: hw_sqrt / hw_rsq reproduce them from
 * truth tables recorded on the MI355X (fmo_set_hw_tables; tests/golden/gfx950_sqrt_rsq.npz).
 */
static const int8_t *g_dsqrt, *g_drsq;

void fmo_set_hw_tables(const int8_t *dsqrt, const int8_t *drsq) {
    g_dsqrt = dsqrt;
    g_drsq = drsq;
}

/* base + the recorded ulp delta of x's (exponent parity, mantissa) class; x a positive normal float */
static float hw_adjust(float base, float x, const int8_t *tab) {
    if (!tab) {
        fprintf(stderr, "fm_oracle: gfx950 sqrt/rsq tables not loaded (fmo_set_hw_tables)\n");
        abort();
    }
    uint32_t u, b;
    memcpy(&u, &x, 4);
    memcpy(&b, &base, 4);
    const uint32_t idx = ((((u >> 23) & 0xFFu) - 127u) & 1u) << 23 | (u & 0x7FFFFFu);
    b = (uint32_t)((int32_t)b + tab[idx]);
    memcpy(&base, &b, 4);
    return base;
}

static float hw_sqrt(float x) { /* v_sqrt_f32 */
    if (x == 0.0f || !(x < INFINITY)) return sqrtf(x);
    return hw_adjust((float)sqrt((double)x), x, g_dsqrt);
}

static float hw_rsq(float x) { /* v_rsq_f32 on a positive normal float */
    return hw_adjust((float)(1.0 / sqrt((double)x)), x, g_drsq);
}

static inline float dot3(v3 a, v3 b) { return fmaf(a.z, b.z, fmaf(a.y, b.y, a.x * b.x)); }
static inline v3 cross3(v3 a, v3 b) {
    return mk(fmaf(a.y, b.z, -(a.z * b.y)), fmaf(a.z, b.x, -(a.x * b.z)), fmaf(a.x, b.y, -(a.y * b.x)));
}
static float len3(v3 a) {
    const float d = dot3(a, a);
    if (d < 0x1p-126f) {
        const v3 s = vmul(a, 0x1p+86f);
        return hw_sqrt(dot3(s, s)) * 0x1p-86f;
    }
    if (d == INFINITY) {
        const v3 s = vmul(a, 0x1p-66f);
        return hw_sqrt(dot3(s, s)) * 0x1p+66f;
    }
    return hw_sqrt(d);
}
static float ocml_rsqrt(float x) { /* __ocml_rsqrt_f32 with f32 denormals preserved (gfx950 OpenCL) */
    if (x < 0x1p-126f) return x == 0.0f ? INFINITY : hw_rsq(x * 0x1p+24f) * 4096.0f;
    if (!(x < INFINITY)) return 0.0f;
    return hw_rsq(x);
}
static v3 normalize3(v3 a) {
    if (a.x == 0.0f && a.y == 0.0f && a.z == 0.0f) return a;
    float d = dot3(a, a);
    v3 s = a;
    if (d < 0x1p-126f) {
        s = vmul(a, 0x1p+86f);
        d = dot3(s, s);
    } else if (d == INFINITY) {
        s = vmul(a, 0x1p-66f);
        d = dot3(s, s);
        if (d == INFINITY) {
            s = mk(copysignf(isinf(s.x) ? 1.0f : 0.0f, s.x), copysignf(isinf(s.y) ? 1.0f : 0.0f, s.y),
                   copysignf(isinf(s.z) ? 1.0f : 0.0f, s.z));
            d = dot3(s, s);
        }
    }
    return vmul(s, ocml_rsqrt(d));
}
/*
 * FMO_PORT (oracle/Makefile -> liboracle_port.so; bench.py's CPU baseline only): the same arithmetic, with
 * the per-rect values photonmap.cl recomputes in every intersects() / getTileIdAt() / sampler call
 * (length(width), width / length(width), ..., the sampler basis of the normal) computed once per bake with
 * the same functions -- identical bits, a fraction of the work. The checker build leaves them per call,
 * as the reference source has them.
 */
typedef struct { v3 wn, hn, bu, bv; float wl, hl; } fmo_pre;
#ifdef FMO_PORT
static const fmo_rect *g_pre_rects, *g_pre_srcs;
static int g_pre_nrects, g_pre_nsrcs;
static fmo_pre *g_pre_r, *g_pre_s;
static inline const fmo_pre *pre_of(const fmo_rect *r) {
    if (g_pre_r && r >= g_pre_rects && r < g_pre_rects + g_pre_nrects) return &g_pre_r[r - g_pre_rects];
    if (g_pre_s && r >= g_pre_srcs && r < g_pre_srcs + g_pre_nsrcs) return &g_pre_s[r - g_pre_srcs];
    return NULL;
}
#else
static inline const fmo_pre *pre_of(const fmo_rect *r) { (void)r; return NULL; }
#endif
/* the reference HOST's length() (vector3_cl.c:93: sqrtf(x*x + y*y + z*z), gcc without FMA) */
static float host_len3(v3 a) { return sqrtf(a.x * a.x + a.y * a.y + a.z * a.z); }

/* photonmap.cl:21-25 -- LCG, returns (float)s / (float)0xFFFFFFFF == (float)s * 2^-32 */
float fmo_rand(uint32_t *s) {
    *s = *s * 1664525u + 1013904223u;
    return (float)(*s) / 4294967296.0f;
}

/* sin/cos as ROCm's device library computes them on gfx9+ (ocml.bc __ocml_sin_f32 / __ocml_cos_f32,
   the fast-FMA path) for 0 <= x < 2^17: k = rint(x * 2/pi), a three-part Cody-Waite reduction with FMAs,
   minimax polynomials; quadrant k & 3. Checked bit for bit against the device library on every
   reachable phi (tests/test_gpu_parity.py). */
void fmo_sincos(float x, float *s, float *c) {
    float k = rintf(x * 0x1.45f306p-1f);
    float r = fmaf(k, -0x1.921fb4p+0f, x);
    r = fmaf(k, -0x1.4442d0p-24f, r);
    r = fmaf(k, -0x1.846988p-48f, r);
    int q = (int)k & 3;
    float z = r * r;
    float p = fmaf(z, -0x1.983304p-13f, 0x1.110388p-7f);
    p = fmaf(z, p, -0x1.55553ap-3f);
    p = z * p;
    float sn = fmaf(r, p, r);
    float cp = fmaf(z, 0x1.aea668p-16f, -0x1.6c9e76p-10f);
    cp = fmaf(z, cp, 0x1.5557eep-5f);
    cp = fmaf(z, cp, -0x1.000008p-1f);
    float cs = fmaf(z, cp, 1.0f);
    float so = (q & 1) ? cs : sn, co = (q & 1) ? -sn : cs;
    *s = q > 1 ? -so : so;
    *c = q > 1 ? -co : co;
}

void fmo_sincos_n(const float *x, float *s, float *c, int64_t n) {
    for (int64_t i = 0; i < n; i++) fmo_sincos(x[i], &s[i], &c[i]);
}

/* photonmap.cl:27-52 (sky, fold=1) and :54-74 (cosine, fold=0) */
static v3 sample_hemisphere_b(uint32_t *rng, v3 ndir, const fmo_pre *q, int fold) {
    float r = sqrtf(fmo_rand(rng));
    float phi = 6.283184f * fmo_rand(rng); /* `2 * 3.141592f` folds exactly to 6.283184f */
    float sn, cs;
    fmo_sincos(phi, &sn, &cs);
    float u = r * cs;
    float v = r * sn;
    float n = sqrtf(1.0f - r * r);
    if (fold && u < 0) u = -u;
    v3 udir, vdir;
    if (q) {
        udir = q->bu;
        vdir = q->bv;
    } else {
        udir = mk(0, 0, 1);
        if (fabsf(dot3(udir, ndir)) >= 0.999999f) udir = mk(0, 1, 0);
        vdir = normalize3(cross3(udir, ndir));
        udir = normalize3(cross3(vdir, ndir));
    }
    return vadd(vadd(vmul(udir, u), vmul(vdir, v)), vmul(ndir, n));
}

/* photonmap.cl:43-48 (== :65-70): the sampler basis of a normal, and a rect's hoisted values */
__attribute__((unused)) static void rect_pre(const fmo_rect *r, fmo_pre *q) {
    v3 w = ld(r->width), h = ld(r->height), n = ld(r->n);
    q->wl = len3(w);
    q->hl = len3(h);
    q->wn = vdiv(w, q->wl);
    q->hn = vdiv(h, q->hl);
    v3 udir = mk(0, 0, 1);
    if (fabsf(dot3(udir, n)) >= 0.999999f) udir = mk(0, 1, 0);
    q->bv = normalize3(cross3(udir, n));
    q->bu = normalize3(cross3(q->bv, n));
}

/* photonmap.cl:95-120 */
static int tile_at(const fmo_rect *r, v3 p) {
    v3 pDir = vsub(p, ld(r->pos));
    const fmo_pre *q = pre_of(r);
    float hLength, vLength, dx, dy;
    if (q) {
        hLength = q->wl, vLength = q->hl;
        dx = dot3(q->wn, pDir);
        dy = dot3(q->hn, pDir);
    } else {
        v3 w = ld(r->width), h = ld(r->height);
        hLength = len3(w), vLength = len3(h);
        dx = dot3(vdiv(w, hLength), pDir);
        dy = dot3(vdiv(h, vLength), pDir);
    }
    int W = r->lm[1], H = r->lm[2];
    int tx = (int)(dx * (float)W / hLength);
    int ty = (int)(dy * (float)H / vLength);
    tx = tx < 0 ? 0 : (tx > W - 1 ? W - 1 : tx);
    ty = ty < 0 ? 0 : (ty > H - 1 ? H - 1 : ty);
    return ty * W + tx;
}

/* photonmap.cl:123-158 */
static float intersects(const fmo_rect *r, v3 src, v3 dir, float closest) {
    v3 n = ld(r->n), pos = ld(r->pos);
    float denom = dot3(n, dir);
    if (denom >= 0) return -1;
    float fac = dot3(n, vsub(pos, src)) / denom;
    if (fac < 0) return -1;
    v3 ray = vmul(dir, fac);
    if (closest * closest < dot3(ray, ray)) return -1;
    v3 pDir = vsub(vadd(src, ray), pos);
    const fmo_pre *q = pre_of(r);
    if (q) {
        float dx = dot3(q->wn, pDir);
        if (dx < 0 || dx > q->wl) return -1;
        float dy = dot3(q->hn, pDir);
        if (dy < 0 || dy > q->hl) return -1;
        return fac;
    }
    v3 w = ld(r->width), h = ld(r->height);
    float wl = len3(w);
    float dx = dot3(vdiv(w, wl), pDir);
    if (dx < 0 || dx > wl) return -1;
    float hl = len3(h);
    float dy = dot3(vdiv(h, hl), pDir);
    if (dy < 0 || dy > hl) return -1;
    return fac;
}

/* Deposit sink: either exact fixed point (lm_fx), fp32 (lm_f32) or an event log. */
typedef struct sink {
    int64_t *lm_fx;
    int64_t *counts; /* deposits per texel (fmo_bake_counts), or NULL */
    float *lm_f32;
    fmo_event *ev;
    int nev, cap;
    int photon;
    fmo_stats st;
} sink;

static inline int64_t to_fx(float v, sink *k) {
    double d = ldexp((double)v, FMO_FX_SHIFT);
    int64_t q = (int64_t)d;
    if ((double)q != d) k->st.inexact++;
    return q;
}

/* photonmap.cl:161-265 */
static void trace_photon(uint32_t *rng, const fmo_rect *win, const fmo_rect *rects, int nrects,
                         int isWindow, sink *k) {
    v3 color = isWindow ? mk(18, 18, 18) : mk(16, 16, 18);
    const int MAX_DEPTH = 8;
    float dx = fmo_rand(rng);
    float dy = fmo_rand(rng);
    v3 wn = ld(win->n);
    v3 dir = sample_hemisphere_b(rng, wn, pre_of(win), isWindow);
    v3 pos = vadd(vadd(vadd(ld(win->pos), vmul(ld(win->width), dx)), vmul(ld(win->height), dy)),
                  vmul(dir, 1e-5f));
    k->st.photons++;
    for (int depth = 0; depth < MAX_DEPTH; depth++) {
        int hit = -1;
        float dist_out = INFINITY;
        k->st.scans++;
        for (int i = 0; i < nrects; i++) {
            float dist = intersects(&rects[i], pos, dir, dist_out);
            if (dist < 0) continue;
            if (dist < dist_out) { hit = i; dist_out = dist; }
        }
        if (dist_out == INFINITY) { k->st.escapes++; return; }
        const fmo_rect *h = &rects[hit];
        pos = vadd(pos, vmul(dir, dist_out));
        int tile = tile_at(h, pos);
        int light_idx = h->lm[0] + tile;
        v3 hn = ld(h->n);
        if ((double)pos.z > 0.0005 || fmo_rand(rng) > 0.75f) {
            dir = sample_hemisphere_b(rng, hn, pre_of(h), 0);
            if (pos.z < 1e-5f) {
                color.x *= 1.0f;
                color.y *= 0.85f;
                color.z *= 0.7f;
            }
            color = vmul(color, 0.9f);
        } else {
            float two_d = 2.0f * dot3(hn, dir);
            dir = vsub(dir, vmul(hn, two_d));
        }
        k->st.deposits++;
        if (k->counts) k->counts[light_idx]++;
        if (k->lm_fx) {
            int64_t *t = k->lm_fx + 3 * (int64_t)light_idx;
            t[0] += to_fx(color.x, k);
            t[1] += to_fx(color.y, k);
            t[2] += to_fx(color.z, k);
        }
        if (k->lm_f32) {
            float *t = k->lm_f32 + 4 * (int64_t)light_idx;
            t[0] += color.x;
            t[1] += color.y;
            t[2] += color.z;
        }
        if (k->ev) {
            if (k->nev < k->cap) {
                fmo_event *e = &k->ev[k->nev];
                e->photon = k->photon;
                e->depth = depth;
                e->rect = hit;
                e->texel = light_idx;
                e->rgb[0] = color.x;
                e->rgb[1] = color.y;
                e->rgb[2] = color.z;
                e->rng = *rng;
            }
            k->nev++;
        }
        pos = vadd(pos, vmul(dir, 1e-5f));
    }
}

/* photonmap.cl:269-281 */
static void work_item(uint32_t rng, const fmo_rect *win, const fmo_rect *rects, int nrects, int isWindow,
                      sink *k, uint32_t *rng_final) {
    float r = fmo_rand(&rng) * 40;
    for (int i = 0; i < r; i++) fmo_rand(&rng);
    for (int i = 0; i < 100; i++) {
        k->photon = i;
        trace_photon(&rng, win, rects, nrects, isWindow, k);
    }
    if (rng_final) *rng_final = rng;
}

/* global_illumination_cl.c:217-222: per-source work-item count */
static uint64_t source_items(const fmo_rect *src, float spa, uint64_t wg) {
    float area = host_len3(ld(src->width)) * host_len3(ld(src->height));
    uint64_t n = (uint64_t)((spa * area) / 100);
    return (n / wg + 1) * wg;
}

int64_t fmo_schedule_count(const fmo_rect *sources, int nwindows, int nlights, int spa, int wg,
                           uint64_t *total_items) {
    int64_t nl = 0;
    uint64_t tot = 0, cap = (uint64_t)wg * 100;
    for (int s = 0; s < nwindows + nlights; s++) {
        uint64_t n = source_items(&sources[s], (float)spa, (uint64_t)wg);
        nl += (int64_t)((n + cap - 1) / cap);
        tot += n;
    }
    if (total_items) *total_items = tot;
    return nl;
}

/* global_illumination_cl.c:304-308 (windows, then lights) and :246-267 (launch loop) */
int64_t fmo_schedule(const fmo_rect *sources, int nwindows, int nlights, int spa, int wg,
                     fmo_launch *out, int64_t cap) {
    int64_t nl = 0;
    uint64_t item = 0, wcap = (uint64_t)wg * 100;
    for (int s = 0; s < nwindows + nlights; s++) {
        uint64_t n = source_items(&sources[s], (float)spa, (uint64_t)wg);
        while (n) {
            int32_t off = rand();
            uint64_t ws = n < wcap ? n : wcap;
            n -= ws;
            if (nl < cap) {
                out[nl].item_begin = item;
                out[nl].count = (uint32_t)ws;
                out[nl].rng_offset = off;
                out[nl].source = s;
                out[nl].is_window = s < nwindows;
            }
            nl++;
            item += ws;
        }
    }
    return nl;
}

static int64_t find_launch(const fmo_launch *L, int64_t nl, uint64_t item) {
    int64_t lo = 0, hi = nl - 1;
    while (lo < hi) {
        int64_t mid = (lo + hi + 1) / 2;
        if (L[mid].item_begin <= item) lo = mid; else hi = mid - 1;
    }
    return lo;
}

static void bake_impl(const fmo_rect *rects, int nrects, const fmo_rect *sources, const fmo_launch *launches,
                      int64_t nlaunches, uint64_t item_begin, uint64_t item_end, int64_t *lm_fx,
                      int64_t *counts, int64_t num_texels, int nthreads, fmo_stats *stats) {
    if (item_end <= item_begin || nlaunches <= 0) return;
#ifdef _OPENMP
    int nt = nthreads > 0 ? nthreads : omp_get_max_threads();
#else
    int nt = 1;
    (void)nthreads;
#endif
    int64_t ntot = num_texels * 3;
#ifdef FMO_PORT
    int64_t nsrc = 0;
    for (int64_t l = 0; l < nlaunches; l++) nsrc = launches[l].source + 1 > nsrc ? launches[l].source + 1 : nsrc;
    g_pre_r = (fmo_pre *)malloc(sizeof(fmo_pre) * (size_t)(nrects > 0 ? nrects : 1));
    g_pre_s = (fmo_pre *)malloc(sizeof(fmo_pre) * (size_t)(nsrc > 0 ? nsrc : 1));
    for (int i = 0; i < nrects; i++) rect_pre(&rects[i], &g_pre_r[i]);
    for (int64_t i = 0; i < nsrc; i++) rect_pre(&sources[i], &g_pre_s[i]);
    g_pre_rects = rects, g_pre_nrects = nrects, g_pre_srcs = sources, g_pre_nsrcs = (int)nsrc;
#endif
    fmo_stats tot;
    memset(&tot, 0, sizeof tot);
#pragma omp parallel num_threads(nt)
    {
        int64_t *priv = (int64_t *)calloc((size_t)ntot, sizeof(int64_t));
        int64_t *pcnt = counts ? (int64_t *)calloc((size_t)num_texels, sizeof(int64_t)) : NULL;
        sink k;
        memset(&k, 0, sizeof k);
        k.lm_fx = priv;
        k.counts = pcnt;
#pragma omp for schedule(dynamic, 64)
        for (int64_t w = (int64_t)item_begin; w < (int64_t)item_end; w++) {
            int64_t li = find_launch(launches, nlaunches, (uint64_t)w);
            const fmo_launch *L = &launches[li];
            uint32_t gid = (uint32_t)((uint64_t)w - L->item_begin);
            uint32_t rng = gid + (uint32_t)L->rng_offset;
            work_item(rng, &sources[L->source], rects, nrects, L->is_window, &k, NULL);
        }
#pragma omp critical
        {
            for (int64_t i = 0; i < ntot; i++) lm_fx[i] += priv[i];
            if (pcnt)
                for (int64_t i = 0; i < num_texels; i++) counts[i] += pcnt[i];
            tot.photons += k.st.photons;
            tot.scans += k.st.scans;
            tot.deposits += k.st.deposits;
            tot.escapes += k.st.escapes;
            tot.inexact += k.st.inexact;
        }
        free(priv);
        free(pcnt);
    }
#ifdef FMO_PORT
    free(g_pre_r);
    free(g_pre_s);
    g_pre_r = g_pre_s = NULL;
#endif
    if (stats) {
        stats->photons += tot.photons;
        stats->scans += tot.scans;
        stats->deposits += tot.deposits;
        stats->escapes += tot.escapes;
        stats->inexact += tot.inexact;
    }
}

void fmo_bake(const fmo_rect *rects, int nrects, const fmo_rect *sources, const fmo_launch *launches,
              int64_t nlaunches, uint64_t item_begin, uint64_t item_end, int64_t *lm_fx,
              int64_t num_texels, int nthreads, fmo_stats *stats) {
    bake_impl(rects, nrects, sources, launches, nlaunches, item_begin, item_end, lm_fx, NULL, num_texels, nthreads,
              stats);
}

/* fmo_bake, also adding every texel's deposit count (photonmap.cl:257 executions) into counts[num_texels] */
void fmo_bake_counts(const fmo_rect *rects, int nrects, const fmo_rect *sources, const fmo_launch *launches,
                     int64_t nlaunches, uint64_t item_begin, uint64_t item_end, int64_t *lm_fx, int64_t *counts,
                     int64_t num_texels, int nthreads, fmo_stats *stats) {
    bake_impl(rects, nrects, sources, launches, nlaunches, item_begin, item_end, lm_fx, counts, num_texels, nthreads,
              stats);
}

int fmo_trace_item(const fmo_rect *rects, int nrects, const fmo_rect *source, int is_window,
                   uint32_t rng_state, fmo_event *ev, int cap, uint32_t *rng_final) {
    sink k;
    memset(&k, 0, sizeof k);
    k.ev = ev;
    k.cap = cap;
    work_item(rng_state, source, rects, nrects, is_window, &k, rng_final);
    return k.nev;
}

void fmo_trace_item_f32(const fmo_rect *rects, int nrects, const fmo_rect *source, int is_window,
                        uint32_t rng_state, float *texels4) {
    sink k;
    memset(&k, 0, sizeof k);
    k.lm_f32 = texels4;
    work_item(rng_state, source, rects, nrects, is_window, &k, NULL);
}

void fmo_finalize(const int64_t *lm_fx, int64_t num_texels, const float *in, float *out) {
    for (int64_t i = 0; i < num_texels; i++) {
        for (int c = 0; c < 3; c++)
            out[4 * i + c] = (float)((double)in[4 * i + c] + ldexp((double)lm_fx[3 * i + c], -FMO_FX_SHIFT));
        out[4 * i + 3] = in[4 * i + 3];
    }
}
