/*
 * oracle/rad_oracle.c -- TEST INFRASTRUCTURE ONLY: a CPU restatement of the reference's radiosity
 * backend (performRadiosityNative, radiosityNative.c:92-268) used to check the HIP backend
 * (csrc/fmgi_rad*.{hip,cpp}). It is pinned against the reference itself: tests/test_radiosity.py
 * compares its texels with those the reference's own radiosityNative.o produces (oracle/_ref/rad_ref,
 * tests/golden/rad_ref.json).
 *
 * Restated pieces (file:line of the reference):
 *   rect list + texel bases   radiosityNative.c:108-131 (walls, windows, lights; window/light mipmap
 *                             texels appended after numTexels, getNumMipmapTexels rectangle.c:166-190)
 *   initial radiosity         radiosityNative.c:139-149 (walls 0, windows 30, lights (28,28,32))
 *   candidate lists           radiosityNative.c:25-61 getSortedIntersectableRects: backface and
 *                             isBehindRay (rectangle.c:97-113) culling, getShortestDistanceRectToPoint
 *                             (rectangle.c:442-470) keys, glibc qsort with compareRectInfo (:17-23)
 *   form factors              radiosityNative.c:166-227: 10000 getCosineDistributedRandomRay
 *                             (vector3_cl.c:129-149) rays per level-0 texel, findClosestIntersectionSorted
 *                             (:67-90), intersects (rectangle.c:67-95), getTileIdAt (:205-230),
 *                             getMipmapTexelId (:232-258)
 *   bounces                   radiosityNative.c:230-251 (7 gathers, 0.7/0.3 update, mipmap of every
 *                             rect, rectangle.c:508-575)
 * libc rand() is consumed in the reference's order (two values per ray, texels in wall/tile order);
 * the values are drawn first, then the rays are traced in parallel (OpenMP) -- same values, same rays.
 * Arithmetic: IEEE fp32 in source order, no contraction (-ffp-contract=off), glibc double sqrt/cos/sin,
 * like the reference's gcc -O2 -msse3 build.
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

typedef struct {
    float x, y, z;
} r3;

typedef struct {
    float pos[4], width[4], height[4], n[4];
    int32_t lm[4];
} rrect; /* Rectangle, 80 B */

typedef struct {
    float x, y, z, w;
} r4; /* Vector3 as the texel buffers hold it */

static r3 v_(const float *p) { r3 r = {p[0], p[1], p[2]}; return r; }
static r3 add(r3 a, r3 b) { r3 r = {a.x + b.x, a.y + b.y, a.z + b.z}; return r; }
static r3 add3(r3 a, r3 b, r3 c) { r3 r = {a.x + b.x + c.x, a.y + b.y + c.y, a.z + b.z + c.z}; return r; }
static r3 sub(r3 a, r3 b) { r3 r = {a.x - b.x, a.y - b.y, a.z - b.z}; return r; }
static r3 mul(r3 a, float f) { r3 r = {a.x * f, a.y * f, a.z * f}; return r; }
static float dot(r3 a, r3 b) { return a.x * b.x + a.y * b.y + a.z * b.z; }
static r3 cross(r3 a, r3 b) {
    r3 r = {a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x};
    return r;
}
static float len(r3 a) { return sqrtf(a.x * a.x + a.y * a.y + a.z * a.z); }
static r3 divv(r3 a, float b) { return mul(a, 1.0f / b); }
static r3 unit(r3 a) { return mul(a, 1.0f / len(a)); }

static int num_mip_texels(const rrect *r) { /* rectangle.c:166-190 (asserts compiled out) */
    int w = r->lm[1], h = r->lm[2], n = w * h;
    while (w > 1 || h > 1) {
        if (w > 1) w /= 2;
        if (h > 1) h /= 2;
        n += w * h;
    }
    return n;
}

static r3 tile_center(const rrect *r, int tile) { /* rectangle.c:140-153 */
    if (tile >= r->lm[1] * r->lm[2]) { r3 z = {0, 0, 0}; return z; }
    r3 vw = divv(v_(r->width), (float)r->lm[1]), vh = divv(v_(r->height), (float)r->lm[2]);
    int tx = tile % r->lm[1], ty = tile / r->lm[1];
    return add3(v_(r->pos), mul(vw, (float)(tx + 0.5)), mul(vh, (float)(ty + 0.5)));
}

static int behind_ray(const rrect *r, r3 src, r3 dir) { /* rectangle.c:97-113 */
    r3 p = v_(r->pos), w = v_(r->width), h = v_(r->height);
    r3 d1 = sub(p, src), d2 = sub(add(p, w), src), d3 = sub(add(p, h), src), d4 = sub(add3(p, w, h), src);
    return dot(d1, dir) < 0 && dot(d2, dir) < 0 && dot(d3, dir) < 0 && dot(d4, dir) < 0;
}

static float min_dist(const rrect *r, r3 p) { /* rectangle.c:442-470 */
    r3 pos = v_(r->pos), n = v_(r->n), w = v_(r->width), h = v_(r->height);
    r3 vd = sub(p, pos);
    r3 on_plane = sub(p, mul(n, dot(vd, n)));
    r3 pd = sub(on_plane, pos);
    float u = dot(pd, unit(h)) / len(h);
    float v = dot(pd, unit(w)) / len(w);
    u = (u < 0) ? 0 : ((u > 1) ? 1 : u);
    v = (v < 0) ? 0 : ((v > 1) ? 1 : v);
    return len(sub(p, add3(pos, mul(w, v), mul(h, u))));
}

static float hit(const rrect *r, r3 src, r3 dir, float closest) { /* rectangle.c:67-95, -1: no hit */
    r3 n = v_(r->n), pos = v_(r->pos);
    float denom = dot(n, dir);
    if (denom >= 0) return -1;
    float fac = dot(n, sub(pos, src)) / denom; /* distanceOfIntersectionWithPlane :115-128 */
    if (fac < 0) return -1;
    r3 ray = mul(dir, fac);
    if (closest * closest < dot(ray, ray)) return -1;
    r3 pdir = sub(add(src, ray), pos);
    r3 w = v_(r->width), h = v_(r->height);
    float wl = len(w), hl = len(h);
    float dx = dot(divv(w, wl), pdir), dy = dot(divv(h, hl), pdir);
    if (dx < 0 || dy < 0 || dx > wl || dy > hl) return -1;
    return fac;
}

static int clampi(int v, int lo, int hi) { return v < lo ? lo : (v > hi ? hi : v); }

static int tile_at(const rrect *r, r3 p) { /* rectangle.c:205-230 */
    r3 pd = sub(p, v_(r->pos));
    r3 w = v_(r->width), h = v_(r->height);
    float hl = len(w), vl = len(h);
    float dx = dot(divv(w, hl), pd), dy = dot(divv(h, vl), pd);
    int s1 = r->lm[1], s2 = r->lm[2];
    int tx = clampi((int)(dx * s1 / hl), 0, s1 - 1);
    int ty = clampi((int)(dy * s2 / vl), 0, s2 - 1);
    return ty * s1 + tx;
}

typedef struct {
    int idx;
    float minDistance;
} rinfo;

static int cmp_info(const void *a, const void *b) { /* radiosityNative.c:17-23 */
    float d1 = ((const rinfo *)a)->minDistance, d2 = ((const rinfo *)b)->minDistance;
    return (d1 < d2) ? -1 : ((d1 > d2) ? 1 : 0);
}

static void mip_h(r4 *base, int width) { /* rectangle.c:508-525 */
    if (width == 1) return;
    r4 *dst = base + width;
    int tw = width / 2;
    for (int i = 0; i < tw; i++) {
        r4 a = base[2 * i], b = base[2 * i + 1];
        r4 o = {(a.x + b.x) * 0.5f, (a.y + b.y) * 0.5f, (a.z + b.z) * 0.5f, 0};
        dst[i] = o;
    }
    mip_h(dst, tw);
}

static void mip_2d(r4 *base, int w, int h) { /* rectangle.c:535-569 */
    if (w == 1 && h == 1) return;
    if (h == 1) { mip_h(base, w); return; }
    if (w == 1) { mip_h(base, h); return; }
    r4 *dst = base + w * h;
    int tw = w / 2, th = h / 2;
    for (int i = 0; i < tw; i++)
        for (int j = 0; j < th; j++) {
            r4 a = base[(2 * j) * w + 2 * i], b = base[(2 * j + 1) * w + 2 * i];
            r4 c = base[(2 * j) * w + 2 * i + 1], d = base[(2 * j + 1) * w + 2 * i + 1];
            r4 o = {(a.x + b.x + c.x + d.x) * 0.25f, (a.y + b.y + c.y + d.y) * 0.25f,
                    (a.z + b.z + c.z + d.z) * 0.25f, 0};
            dst[j * tw + i] = o;
        }
    mip_2d(dst, tw, th);
}

#define RAD_RAYS 10000 /* geoSphereNumVectors, radiosityNative.c:151 */

/*
 * texels: float4 x num_texels, overwritten with the reference's result. sids (optional): njobs x
 * RAD_RAYS, the reference's sourceTexelIds rows of the wall level-0 texels, in wall/tile order.
 * Returns the number of level-0 wall texels (jobs), or -1 on allocation failure.
 */
int64_t rad_oracle(const void *walls_v, int nwalls, const void *windows_v, int nwin, const void *lights_v, int nlights,
                   int num_texels, float *texels, int32_t *sids, int nthreads) {
    const int nr = nwalls + nwin + nlights;
    rrect *rects = (rrect *)malloc((size_t)(nr ? nr : 1) * sizeof(rrect));
    if (!rects) return -1;
    memcpy(rects, walls_v, (size_t)nwalls * sizeof(rrect));
    memcpy(rects + nwalls, windows_v, (size_t)nwin * sizeof(rrect));
    memcpy(rects + nwalls + nwin, lights_v, (size_t)nlights * sizeof(rrect));
    int ntex = num_texels;
    for (int i = nwalls; i < nr; i++) { /* :116-131 */
        rects[i].lm[0] = ntex;
        ntex += num_mip_texels(&rects[i]);
    }
    const int first_light = nwalls + nwin < nr ? rects[nwalls + nwin].lm[0] : ntex;
    r4 *src = (r4 *)calloc((size_t)(ntex ? ntex : 1), sizeof(r4));
    r4 *dst = (r4 *)calloc((size_t)(ntex ? ntex : 1), sizeof(r4));
    for (int i = num_texels; i < first_light; i++) src[i] = (r4){30, 30, 30, 0};
    for (int i = first_light; i < ntex; i++) src[i] = (r4){28, 28, 32, 0};

    int64_t njobs = 0;
    for (int i = 0; i < nwalls; i++) njobs += (int64_t)rects[i].lm[1] * rects[i].lm[2];
    int32_t *job_wall = (int32_t *)malloc((size_t)(njobs ? njobs : 1) * 8);
    int32_t *job_tile = job_wall + (njobs ? njobs : 1);
    int32_t *rnd = (int32_t *)malloc((size_t)(njobs ? njobs : 1) * 2 * RAD_RAYS * sizeof(int32_t));
    int32_t *ids = (int32_t *)malloc((size_t)(njobs ? njobs : 1) * RAD_RAYS * sizeof(int32_t));
    if (!src || !dst || !job_wall || !rnd || !ids) return -1;
    {
        int64_t j = 0;
        for (int i = 0; i < nwalls; i++)
            for (int t = 0; t < rects[i].lm[1] * rects[i].lm[2]; t++, j++) job_wall[j] = i, job_tile[j] = t;
    }
    for (int64_t k = 0; k < njobs * 2 * RAD_RAYS; k++) rnd[k] = rand(); /* the reference's draw order */

#pragma omp parallel for schedule(dynamic, 1) num_threads(nthreads > 0 ? nthreads : 1)
    for (int64_t job = 0; job < njobs; job++) {
        const rrect *wall = &rects[job_wall[job]];
        const r3 n = v_(wall->n);
        const r3 cam = tile_center(wall, job_tile[job]);
        rinfo *cand = (rinfo *)malloc((size_t)(nr ? nr : 1) * sizeof(rinfo));
        int nc = 0;
        for (int i = 0; i < nr; i++) { /* getSortedIntersectableRects :25-61 */
            if (dot(v_(rects[i].n), sub(v_(rects[i].pos), cam)) > 0) continue;
            if (behind_ray(&rects[i], cam, n)) continue;
            cand[nc].idx = i;
            cand[nc].minDistance = min_dist(&rects[i], cam);
            nc++;
        }
        qsort(cand, (size_t)nc, sizeof(rinfo), cmp_info);
        /* the ray basis of getCosineDistributedRandomRay (vector3_cl.c:140-145) */
        r3 udir = {0, 0, 1};
        if (fabs(dot(udir, n)) >= 0.999999f) udir = (r3){0, 1, 0};
        const r3 vdir = unit(cross(udir, n));
        udir = unit(cross(vdir, n));
        const int32_t *rj = rnd + job * 2 * RAD_RAYS;
        int32_t *out = ids + job * RAD_RAYS;
        for (int k = 0; k < RAD_RAYS; k++) {
            float r = sqrt(rj[2 * k] / (double)RAND_MAX);
            float phi = 2 * 3.141592f * (rj[2 * k + 1] / (double)RAND_MAX);
            float u = r * cos(phi);
            float v = r * sin(phi);
            float nn = sqrt(1 - r * r);
            const r3 dir = add3(mul(udir, u), mul(vdir, v), mul(n, nn));
            const r3 pos = add(cam, mul(dir, 1E-5));
            float dist = INFINITY;
            int target = -1;
            for (int i = 0; i < nc; i++) { /* findClosestIntersectionSorted :67-90 */
                if (dist < cand[i].minDistance) break;
                float dn = hit(&rects[cand[i].idx], pos, dir, dist);
                if (dn < 0) continue;
                if (dn <= dist) {
                    target = cand[i].idx;
                    dist = dn;
                }
            }
            out[k] = -1;
            if (target < 0) continue;
            const rrect *t = &rects[target];
            const int tile = tile_at(t, add(pos, mul(dir, dist)));
            out[k] = t->lm[0] + (tile / t->lm[1]) * t->lm[1] + tile % t->lm[1]; /* getMipmapTexelId level 0 */
        }
        free(cand);
    }

    const float keep = 1 - 0.3f, gain = 0.3f / RAD_RAYS; /* reflectance, :103 and :244-245 */
    for (int depth = 0; depth < 7; depth++) { /* :230-251 */
        for (int64_t job = 0; job < njobs; job++) {
            const int64_t texel = rects[job_wall[job]].lm[0] + job_tile[job];
            const int32_t *row = ids + job * RAD_RAYS;
            for (int k = 0; k < RAD_RAYS; k++) {
                if (row[k] < 0) continue;
                dst[texel].x += src[row[k]].x;
                dst[texel].y += src[row[k]].y;
                dst[texel].z += src[row[k]].z;
            }
        }
        for (int i = 0; i < ntex; i++) {
            r4 o = {src[i].x * keep + dst[i].x * gain, src[i].y * keep + dst[i].y * gain,
                    src[i].z * keep + dst[i].z * gain, 0};
            src[i] = o;
            dst[i] = (r4){0, 0, 0, 0};
        }
        for (int i = 0; i < nr; i++) mip_2d(src + rects[i].lm[0], rects[i].lm[1], rects[i].lm[2]);
    }
    memcpy(texels, src, (size_t)num_texels * sizeof(r4));
    if (sids) memcpy(sids, ids, (size_t)njobs * RAD_RAYS * sizeof(int32_t));
    free(rects);
    free(src);
    free(dst);
    free(job_wall);
    free(rnd);
    free(ids);
    return njobs;
}
