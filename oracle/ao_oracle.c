/*
 * oracle/ao_oracle.c -- TEST INFRASTRUCTURE ONLY: a CPU restatement of the reference's ambient
 * occlusion (performAmbientOcclusionNative, photonmap.c:435-490) used to check the HIP backend.
 * It is pinned against the reference itself: tests/test_ao.py compares its output with texels
 * produced by the reference's own code (oracle/_ref/ao_ref, tests/golden/ao_ref.json).
 *
 * Restated pieces (file:line of the reference):
 *   BSP build          photonmap.c:278-406 (subdivideNode, getSubdivisionOverhead), getPosition
 *                      rectangle.c:476-505, getDistanceToPlane :436-440
 *   BSP traversal      photonmap.c:54-161 findClosestIntersection (recursive, as in the reference)
 *   ray / rect test    rectangle.c:67-95 intersects, :115-128 distanceOfIntersectionWithPlane
 *   per-texel loop     photonmap.c:435-475, getTileCenter rectangle.c:140-153, createBase
 *                      vector3_cl.c:152-160, transformToOrthoNormalBase photonmap.c:29-44
 * Arithmetic: IEEE fp32 in source order, no contraction (-ffp-contract=off), like the reference's
 * gcc -O2 -msse3 build. The direction table is an input (the caller's geoSphere4 table).
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

typedef struct {
    float x, y, z;
} o3;

typedef struct {
    float pos[4], width[4], height[4], n[4];
    int32_t lm[4];
} orect; /* Rectangle, 80 B */

static o3 o_v(const float *p) { o3 r = {p[0], p[1], p[2]}; return r; }
static o3 o_add(o3 a, o3 b) { o3 r = {a.x + b.x, a.y + b.y, a.z + b.z}; return r; }
static o3 o_sub(o3 a, o3 b) { o3 r = {a.x - b.x, a.y - b.y, a.z - b.z}; return r; }
static o3 o_scale(o3 a, float f) { o3 r = {a.x * f, a.y * f, a.z * f}; return r; }
static float o_dot(o3 a, o3 b) { return a.x * b.x + a.y * b.y + a.z * b.z; }
static o3 o_cross(o3 a, o3 b) {
    o3 r = {a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x};
    return r;
}
static float o_len(o3 a) { return sqrtf(a.x * a.x + a.y * a.y + a.z * a.z); }
static o3 o_divv(o3 a, float b) { return o_scale(a, 1.0f / b); }
static o3 o_unit(o3 a) { return o_scale(a, 1.0f / o_len(a)); }

/* ---- BSP ---- */
typedef struct onode {
    int plane;  /* wall index of the split plane, -1 for a leaf */
    int *items; /* wall indices */
    int count;
    struct onode *lo, *hi;
} onode;

static int o_side(const orect *pl, const orect *r) {
    o3 p = o_v(r->pos), w = o_v(r->width), h = o_v(r->height);
    o3 corner[4];
    corner[0] = p;
    corner[1] = o_add(p, w);
    corner[2] = o_add(p, h);
    corner[3] = o_add(o_add(p, w), h);
    int below = 0, above = 0;
    for (int k = 0; k < 4; k++) {
        double d = o_dot(o_sub(corner[k], o_v(pl->pos)), o_v(pl->n));
        below |= d < 0;
        above |= d > 0;
    }
    return (below && !above) ? -1 : (above && !below) ? 1 : 0;
}

static onode *o_node(int *items, int count) {
    onode *nd = (onode *)calloc(1, sizeof(onode));
    nd->plane = -1;
    nd->items = items;
    nd->count = count;
    return nd;
}

static void o_split(const orect *walls, onode *nd) {
    if (nd->count < 20) return;
    int best = nd->count, pick = 0;
    for (int i = 0; i < nd->count; i++) {
        int lo = 0, hi = 0, mid = 0;
        for (int k = 0; k < nd->count; k++) {
            int s = o_side(&walls[nd->items[i]], &walls[nd->items[k]]);
            if (s < 0) lo++;
            else if (s > 0) hi++;
            else mid++;
        }
        int cost = (lo > hi ? lo : hi) + mid;
        if (cost < best) {
            best = cost;
            pick = i;
        }
    }
    nd->plane = nd->items[pick];
    int *lo = (int *)malloc(sizeof(int) * nd->count), *hi = (int *)malloc(sizeof(int) * nd->count);
    int nlo = 0, nhi = 0, i = 0;
    while (i < nd->count) {
        int s = o_side(&walls[nd->plane], &walls[nd->items[i]]);
        if (s == 0) {
            i++;
            continue;
        }
        if (s < 0) lo[nlo++] = nd->items[i];
        else hi[nhi++] = nd->items[i];
        nd->items[i] = nd->items[--nd->count]; /* the vacated slot takes the last item */
    }
    if (nlo) {
        nd->lo = o_node(lo, nlo);
        o_split(walls, nd->lo);
    } else free(lo);
    if (nhi) {
        nd->hi = o_node(hi, nhi);
        o_split(walls, nd->hi);
    } else free(hi);
}

static void o_free(onode *nd) {
    if (!nd) return;
    o_free(nd->lo);
    o_free(nd->hi);
    free(nd->items);
    free(nd);
}

/* ---- ray queries ---- */
static float o_hit(const orect *r, o3 src, o3 dir, float closest) {
    o3 n = o_v(r->n), pos = o_v(r->pos);
    float denom = o_dot(n, dir);
    if (denom >= 0) return -1;
    float fac = o_dot(n, o_sub(pos, src)) / denom;
    if (fac < 0) return -1;
    o3 ray = o_scale(dir, fac);
    if (closest * closest < o_dot(ray, ray)) return -1;
    o3 rel = o_sub(o_add(src, ray), pos);
    float wl = o_len(o_v(r->width)), hl = o_len(o_v(r->height));
    float dx = o_dot(o_divv(o_v(r->width), wl), rel);
    float dy = o_dot(o_divv(o_v(r->height), hl), rel);
    if (dx < 0 || dy < 0 || dx > wl || dy > hl) return -1;
    return fac;
}

static float o_plane_hit(o3 src, o3 dir, o3 n, o3 p) {
    float denom = o_dot(n, dir);
    if (denom == 0) return -1;
    float fac = o_dot(n, o_sub(p, src)) / denom;
    if (fac < 0) return -1;
    return fac;
}

static int o_find(const orect *walls, const onode *nd, o3 src, o3 dir, float *dist, float shift) {
    int hit = 0;
    for (int i = 0; i < nd->count; i++) {
        float d = o_hit(&walls[nd->items[i]], src, dir, *dist);
        if (d == -1) continue;
        if (d + shift < *dist) {
            *dist = d + shift;
            hit = 1;
        }
    }
    if (!nd->lo && !nd->hi) return hit;
    const orect *pl = &walls[nd->plane];
    o3 facing = o_v(pl->n);
    if (o_dot(o_sub(src, o_v(pl->pos)), facing) < 0) facing = o_scale(facing, -1.0f);
    int away = o_dot(facing, dir) >= 0;
    float side = o_dot(o_sub(src, o_v(pl->pos)), o_v(pl->n));
    const onode *first = side < 0 ? nd->lo : nd->hi, *second = side < 0 ? nd->hi : nd->lo;
    int child = first ? o_find(walls, first, src, dir, dist, shift) : 0;
    if (!child && second && !away) {
        float t = o_plane_hit(src, dir, o_v(pl->n), o_v(pl->pos));
        if (t < 0) t = 0;
        hit |= o_find(walls, second, o_add(src, o_scale(dir, t)), dir, dist, shift + t);
    }
    return hit | child;
}

/* neg(-v) in the reference is a component-wise negation; o_scale by -1 is the same IEEE result. */

/*
 * AO of walls [wb, we): texels (float4 x num_texels) get (d, d, d, 0) on those walls' level-0 texels.
 * dirs: ndirs xyz triples. Returns 0.
 */
int ao_oracle(const void *walls_v, int nwalls, int wb, int we, const float *dirs, int ndirs, float *texels,
              int nthreads) {
    const orect *walls = (const orect *)walls_v;
    int *all = (int *)malloc(sizeof(int) * (nwalls ? nwalls : 1));
    for (int i = 0; i < nwalls; i++) all[i] = i;
    onode *root = o_node(all, nwalls);
    o_split(walls, root);
    float fsum = 0;
    for (int k = 0; k < ndirs; k++) fsum += dirs[3 * k + 2];
    for (int wi = wb; wi < we; wi++) {
        const orect *w = &walls[wi];
        o3 n = o_v(w->n), c1 = {0, 0, 1};
        if (fabs(o_dot(n, c1)) >= 0.999999f) {
            c1.x = 0;
            c1.y = 1;
            c1.z = 0;
        }
        o3 c2 = o_unit(o_cross(c1, n));
        c1 = o_unit(o_cross(c2, n));
        const int tiles = w->lm[1] * w->lm[2];
        o3 vw = o_divv(o_v(w->width), (float)w->lm[1]), vh = o_divv(o_v(w->height), (float)w->lm[2]);
#pragma omp parallel for schedule(dynamic, 16) num_threads(nthreads > 0 ? nthreads : 1)
        for (int j = 0; j < tiles; j++) {
            const int tx = j % w->lm[1], ty = j / w->lm[1];
            o3 centre = o_add(o_add(o_v(w->pos), o_scale(vw, (float)(tx + 0.5))), o_scale(vh, (float)(ty + 0.5)));
            float sum = 0;
            for (int k = 0; k < ndirs; k++) {
                const float gx = dirs[3 * k], gy = dirs[3 * k + 1], gz = dirs[3 * k + 2];
                o3 dir = {gx * c1.x + gy * c2.x + gz * n.x, gx * c1.y + gy * c2.y + gz * n.y,
                          gx * c1.z + gy * c2.z + gz * n.z};
                o3 src = o_add(centre, o_scale(dir, 1E-5f));
                float dist = INFINITY;
                if (!o_find(walls, root, src, dir, &dist, 0)) dist = 10;
                sum += dist * gz;
            }
            sum = (float)((double)sum / ((double)fsum * 1.5));
            float *t = texels + 4 * (size_t)(w->lm[0] + j);
            t[0] = t[1] = t[2] = sum;
            t[3] = 0;
        }
    }
    o_free(root);
    return 0;
}

/* the tree in fmgi_ao_tree's encoding, preorder with the reference's child creation order
   (left subtree fully before the right child): {left, right, plane, n, items...} per node */
static int o_enc(const onode *nd, int32_t *out, int64_t *len, int64_t cap, int *next) {
    const int me = (*next)++;
    int64_t at = *len;
    *len += 4 + nd->count;
    if (*len <= cap) {
        out[at + 2] = nd->plane;
        out[at + 3] = nd->count;
        for (int i = 0; i < nd->count; i++) out[at + 4 + i] = nd->items[i];
    }
    int l = -1, r = -1;
    if (nd->lo) l = o_enc(nd->lo, out, len, cap, next);
    if (nd->hi) r = o_enc(nd->hi, out, len, cap, next);
    if (at + 4 <= cap) {
        out[at] = l;
        out[at + 1] = r;
    }
    return me;
}

int64_t ao_oracle_tree(const void *walls_v, int nwalls, int32_t *out, int64_t cap) {
    const orect *walls = (const orect *)walls_v;
    int *all = (int *)malloc(sizeof(int) * (nwalls ? nwalls : 1));
    for (int i = 0; i < nwalls; i++) all[i] = i;
    onode *root = o_node(all, nwalls);
    o_split(walls, root);
    int64_t len = 0;
    int next = 0;
    o_enc(root, out, &len, cap, &next);
    o_free(root);
    return len;
}
