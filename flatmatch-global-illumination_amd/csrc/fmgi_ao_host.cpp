/*
 * fmgi_ao_host.cpp -- host side of the ambient-occlusion backend: the BSP tree, the per-wall frames,
 * the direction table, and the C ABI (include/flatmatch_gi.h: performAmbientOcclusionGpu,
 * fmgi_ambient_occlusion, fmgi_geosphere, fmgi_ao_tree).
 *
 * The tree is the reference's (photonmap.c:278-406), rebuilt with the same decisions:
 *   - a node with fewer than 20 items is a leaf;
 *   - otherwise the split plane is the first item with the smallest worst-case overhead
 *     max(left, right) + centre (getSubdivisionOverhead :282-305; ties keep the first);
 *   - items wholly on one side move to that child in scan order, and each vacated slot is filled by
 *     the node's last item (the swap-remove of :332-345), which sets the order of the centre items;
 *   - the side of an item is decided by its four corners' signed distances to the plane
 *     (getPosition rectangle.c:476-505).
 * All geometry arithmetic is fp32 in the reference's order (this file is built with
 * -ffp-contract=off; x86-64 SSE, no FMA).
 */
#include <hip/hip_runtime_api.h>

#include <math.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <vector>

#include "../../include/flatmatch_gi.h"
#include "fmgi_ao.h"
#include "fmgi_geosphere.h"
#include "fmgi_output.h"

#define FMGI_API extern "C" __attribute__((visibility("default")))

int internal_set_err(int code, const char *msg);

namespace {

struct F3 {
    float x, y, z;
};
F3 f3of(const fmgi_vec3 &v) { return F3{v.s[0], v.s[1], v.s[2]}; }
F3 add(F3 a, F3 b) { return F3{a.x + b.x, a.y + b.y, a.z + b.z}; }
F3 sub(F3 a, F3 b) { return F3{a.x - b.x, a.y - b.y, a.z - b.z}; }
F3 mul(F3 a, float f) { return F3{a.x * f, a.y * f, a.z * f}; }
float dot(F3 a, F3 b) { return a.x * b.x + a.y * b.y + a.z * b.z; }
F3 cross(F3 a, F3 b) { return F3{a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x}; }
float length(F3 a) { return sqrtf(a.x * a.x + a.y * a.y + a.z * a.z); }
F3 div_vec3(F3 a, float b) { /* vector3_cl.c:53-58: multiply by the reciprocal */
    const float rec = 1.0f / b;
    return mul(a, rec);
}
F3 normalized(F3 a) { /* vector3_cl.c:95-101 */
    const float fac = 1.0f / length(a);
    return mul(a, fac);
}

/* rectangle.c:436-440 getDistanceToPlane */
float plane_dist(const fmgi_rect &plane, F3 p) { return dot(sub(p, f3of(plane.pos)), f3of(plane.n)); }

/* rectangle.c:476-505 getPosition: -1 wholly on the negative side, 1 wholly positive, 0 otherwise */
int side_of(const fmgi_rect &plane, const fmgi_rect &r) {
    const F3 p = f3of(r.pos), w = f3of(r.width), h = f3of(r.height);
    const F3 c[4] = {p, add(p, w), add(p, h), add(add(p, w), h)};
    bool neg = false, pos = false;
    for (const F3 &q : c) {
        const double d = plane_dist(plane, q);
        neg |= d < 0;
        pos |= d > 0;
    }
    if (neg && !pos) return -1;
    if (pos && !neg) return 1;
    return 0;
}

struct Node {
    int plane = -1; /* wall index of the split plane */
    std::vector<int> items;
    int left = -1, right = -1;
};

struct Tree {
    std::vector<Node> nodes;
    int depth = 0;
};

void subdivide(Tree &t, const fmgi_rect *walls, int idx, int depth) {
    t.depth = std::max(t.depth, depth + 1);
    std::vector<int> items = t.nodes[idx].items;
    const int n = (int)items.size();
    if (n < 20) return; /* photonmap.c:312 */
    int lowest = n, split = 0;
    for (int i = 0; i < n; i++) { /* :315-324 */
        int l = 0, r = 0, c = 0;
        for (int k = 0; k < n; k++) {
            const int s = side_of(walls[items[i]], walls[items[k]]);
            l += s < 0;
            r += s > 0;
            c += s == 0;
        }
        const int overhead = std::max(l, r) + c;
        if (overhead < lowest) {
            lowest = overhead;
            split = i;
        }
    }
    const int plane = items[split];
    std::vector<int> left, right;
    int cnt = n;
    for (int i = 0; i < cnt;) { /* :332-345 */
        const int s = side_of(walls[plane], walls[items[i]]);
        if (s < 0) left.push_back(items[i]);
        if (s > 0) right.push_back(items[i]);
        if (s != 0)
            items[i] = items[--cnt];
        else
            i++;
    }
    items.resize(cnt);
    t.nodes[idx].plane = plane;
    t.nodes[idx].items = items;
    if (!left.empty()) {
        const int li = (int)t.nodes.size();
        t.nodes.push_back(Node{});
        t.nodes[li].items = left;
        t.nodes[idx].left = li;
        subdivide(t, walls, li, depth + 1);
    }
    if (!right.empty()) {
        const int ri = (int)t.nodes.size();
        t.nodes.push_back(Node{});
        t.nodes[ri].items = right;
        t.nodes[idx].right = ri;
        subdivide(t, walls, ri, depth + 1);
    }
}

Tree build_tree(const fmgi_rect *walls, int n) {
    Tree t;
    t.nodes.push_back(Node{});
    for (int i = 0; i < n; i++) t.nodes[0].items.push_back(i);
    subdivide(t, walls, 0, 0);
    return t;
}

AoRect ao_rect(const fmgi_rect &r) {
    AoRect a;
    memset(&a, 0, sizeof a);
    a.nx = r.n.s[0], a.ny = r.n.s[1], a.nz = r.n.s[2];
    a.px = r.pos.s[0], a.py = r.pos.s[1], a.pz = r.pos.s[2];
    const F3 w = f3of(r.width), h = f3of(r.height);
    const float wl = length(w), hl = length(h);
    const F3 wn = div_vec3(w, wl), hn = div_vec3(h, hl);
    a.wx = wn.x, a.wy = wn.y, a.wz = wn.z, a.wl = wl;
    a.hx = hn.x, a.hy = hn.y, a.hz = hn.z, a.hl = hl;
    return a;
}

AoWall ao_wall(const fmgi_rect &r) {
    AoWall w;
    memset(&w, 0, sizeof w);
    w.px = r.pos.s[0], w.py = r.pos.s[1], w.pz = r.pos.s[2];
    const F3 vw = div_vec3(f3of(r.width), (float)r.lightmapSetup[1]);
    const F3 vh = div_vec3(f3of(r.height), (float)r.lightmapSetup[2]);
    w.vwx = vw.x, w.vwy = vw.y, w.vwz = vw.z;
    w.vhx = vh.x, w.vhy = vh.y, w.vhz = vh.z;
    /* createBase (vector3_cl.c:152-160) */
    const F3 n = f3of(r.n);
    F3 c1{0, 0, 1};
    if (fabs(dot(n, c1)) >= 0.999999f) c1 = F3{0, 1, 0};
    const F3 c2 = normalized(cross(c1, n));
    c1 = normalized(cross(c2, n));
    w.b1x = c1.x, w.b1y = c1.y, w.b1z = c1.z;
    w.b2x = c2.x, w.b2y = c2.y, w.b2z = c2.z;
    w.nx = n.x, w.ny = n.y, w.nz = n.z;
    w.s0 = r.lightmapSetup[0], w.s1 = r.lightmapSetup[1], w.s2 = r.lightmapSetup[2];
    return w;
}

#define AOCHK(expr)                                                                                    \
    do {                                                                                               \
        hipError_t e_ = (expr);                                                                        \
        if (e_ != hipSuccess) {                                                                        \
            char b_[256];                                                                              \
            snprintf(b_, sizeof b_, "%s: %s", #expr, hipGetErrorString(e_));                           \
            rc = internal_set_err(FMGI_ERR_HIP, b_);                                                   \
            goto done;                                                                                 \
        }                                                                                              \
    } while (0)

int ao_run(const fmgi_geometry *geo, int wb, int we, fmgi_vec3 *texels_out) {
    if (!geo || !texels_out) return internal_set_err(FMGI_ERR_ARG, "fmgi_ambient_occlusion: null argument");
    if (geo->numWalls < 0 || geo->numTexels < 0 || (geo->numWalls && !geo->walls) ||
        (geo->numTexels && !geo->texels))
        return internal_set_err(FMGI_ERR_ARG, "fmgi_ambient_occlusion: bad geometry");
    if (wb < 0 || we > geo->numWalls || wb > we)
        return internal_set_err(FMGI_ERR_ARG, "fmgi_ambient_occlusion: wall range outside the geometry");
    const fmgi_rect *walls = geo->walls;
    if (texels_out != geo->texels) memcpy(texels_out, geo->texels, (size_t)geo->numTexels * sizeof(fmgi_vec3));
    if (wb == we) return FMGI_OK;
    for (int i = wb; i < we; i++) {
        const int32_t *lm = walls[i].lightmapSetup;
        if (lm[1] < 1 || lm[2] < 1 || lm[0] < 0 || (int64_t)lm[0] + (int64_t)lm[1] * lm[2] > geo->numTexels)
            return internal_set_err(FMGI_ERR_ARG, "fmgi_ambient_occlusion: a wall's texels lie outside numTexels");
    }
    int dev_count = 0;
    if (hipGetDeviceCount(&dev_count) != hipSuccess || dev_count <= 0)
        return internal_set_err(FMGI_ERR_NO_DEVICE, "no HIP device visible");

    const Tree tree = build_tree(walls, geo->numWalls);
    if (tree.depth > FMGI_AO_MAX_DEPTH)
        return internal_set_err(FMGI_ERR_ARG, "BSP tree deeper than the device traversal stack");
    std::vector<AoNode> nodes(tree.nodes.size());
    std::vector<AoRect> items;
    for (size_t i = 0; i < tree.nodes.size(); i++) {
        const Node &nd = tree.nodes[i];
        AoNode &o = nodes[i];
        memset(&o, 0, sizeof o);
        if (nd.plane >= 0) {
            const fmgi_rect &p = walls[nd.plane];
            o.px = p.pos.s[0], o.py = p.pos.s[1], o.pz = p.pos.s[2];
            o.nx = p.n.s[0], o.ny = p.n.s[1], o.nz = p.n.s[2];
        }
        o.left = nd.left, o.right = nd.right;
        o.item0 = (int32_t)items.size();
        o.nitems = (int32_t)nd.items.size();
        for (int w : nd.items) items.push_back(ao_rect(walls[w]));
    }
    if (items.empty()) items.push_back(AoRect{});
    std::vector<AoWall> aw;
    std::vector<int32_t> jobs, job_tile;
    for (int i = wb; i < we; i++) {
        const int wi = (int)aw.size();
        aw.push_back(ao_wall(walls[i]));
        const int nt = walls[i].lightmapSetup[1] * walls[i].lightmapSetup[2];
        for (int j = 0; j < nt; j++) {
            jobs.push_back(wi);
            job_tile.push_back(j);
        }
    }
    const std::vector<float> dirs = fmgi_geo::geosphere(4);
    float fac_sum = 0;
    for (size_t k = 0; k < dirs.size() / 3; k++) fac_sum += dirs[3 * k + 2];

    int rc = FMGI_OK;
    AoNode *d_nodes = nullptr;
    AoRect *d_items = nullptr;
    AoWall *d_walls = nullptr;
    int32_t *d_jobs = nullptr, *d_tile = nullptr;
    float *d_dirs = nullptr, *d_tex = nullptr;
    AoArgs a;
    memset(&a, 0, sizeof a);
    {
        const char *dv = getenv("FMGI_DEVICE");
        AOCHK(hipSetDevice(dv ? atoi(dv) : 0));
    }
    AOCHK(hipMalloc(&d_nodes, nodes.size() * sizeof(AoNode)));
    AOCHK(hipMemcpy(d_nodes, nodes.data(), nodes.size() * sizeof(AoNode), hipMemcpyHostToDevice));
    AOCHK(hipMalloc(&d_items, items.size() * sizeof(AoRect)));
    AOCHK(hipMemcpy(d_items, items.data(), items.size() * sizeof(AoRect), hipMemcpyHostToDevice));
    AOCHK(hipMalloc(&d_walls, aw.size() * sizeof(AoWall)));
    AOCHK(hipMemcpy(d_walls, aw.data(), aw.size() * sizeof(AoWall), hipMemcpyHostToDevice));
    AOCHK(hipMalloc(&d_jobs, std::max<size_t>(jobs.size(), 1) * sizeof(int32_t)));
    AOCHK(hipMalloc(&d_tile, std::max<size_t>(jobs.size(), 1) * sizeof(int32_t)));
    if (!jobs.empty()) {
        AOCHK(hipMemcpy(d_jobs, jobs.data(), jobs.size() * sizeof(int32_t), hipMemcpyHostToDevice));
        AOCHK(hipMemcpy(d_tile, job_tile.data(), jobs.size() * sizeof(int32_t), hipMemcpyHostToDevice));
    }
    AOCHK(hipMalloc(&d_dirs, dirs.size() * sizeof(float)));
    AOCHK(hipMemcpy(d_dirs, dirs.data(), dirs.size() * sizeof(float), hipMemcpyHostToDevice));
    AOCHK(hipMalloc(&d_tex, std::max<size_t>((size_t)geo->numTexels, 1) * sizeof(fmgi_vec3)));
    AOCHK(hipMemcpy(d_tex, texels_out, (size_t)geo->numTexels * sizeof(fmgi_vec3), hipMemcpyHostToDevice));
    a.nodes = d_nodes;
    a.items = d_items;
    a.walls = d_walls;
    a.jobs = d_jobs;
    a.job_tile = d_tile;
    a.njobs = (int64_t)jobs.size();
    a.dirs = d_dirs;
    a.ndirs = (int)(dirs.size() / 3);
    a.fac_sum = fac_sum;
    a.texels = d_tex;
    AOCHK(fmgi_launch_ao(a, nullptr));
    AOCHK(hipDeviceSynchronize());
    AOCHK(hipMemcpy(texels_out, d_tex, (size_t)geo->numTexels * sizeof(fmgi_vec3), hipMemcpyDeviceToHost));
done:
    hipFree(d_nodes);
    hipFree(d_items);
    hipFree(d_walls);
    hipFree(d_jobs);
    hipFree(d_tile);
    hipFree(d_dirs);
    hipFree(d_tex);
    return rc;
}

} // namespace

namespace {

int output_run(const fmgi_geometry *geo, int spa, int tint, fmgi_vec3 *texels_out, uint8_t *rgb_out) {
    if (!geo || !texels_out || !rgb_out) return internal_set_err(FMGI_ERR_ARG, "fmgi_output_tiles: null argument");
    if (geo->numWalls < 0 || geo->numTexels < 0 || (geo->numWalls && !geo->walls) ||
        (geo->numTexels && !geo->texels) || spa < 0)
        return internal_set_err(FMGI_ERR_ARG, "fmgi_output_tiles: bad geometry");
    std::vector<OutWall> ow((size_t)std::max(geo->numWalls, 1));
    int64_t tiles = 0;
    for (int i = 0; i < geo->numWalls; i++) {
        const fmgi_rect &r = geo->walls[i];
        const int32_t *lm = r.lightmapSetup;
        if (lm[1] < 1 || lm[2] < 1 || lm[0] < 0 || (int64_t)lm[0] + (int64_t)lm[1] * lm[2] > geo->numTexels)
            return internal_set_err(FMGI_ERR_ARG, "fmgi_output_tiles: a wall's texels lie outside numTexels");
        OutWall &w = ow[i];
        memset(&w, 0, sizeof w);
        w.first_tile = tiles;
        w.s0 = lm[0];
        w.floor = r.pos.s[2] == 0 && r.width.s[2] == 0 && r.height.s[2] == 0;
        const int nt = lm[1] * lm[2];
        /* main.c:71: getNumTiles(obj) / (getArea(obj) * numSamplesPerArea), then 0.35 * that in double */
        const float area = length(f3of(r.width)) * length(f3of(r.height));
        const float per = nt / (area * spa);
        w.norm = (float)(0.35 * per);
        tiles += nt;
    }
    if (texels_out != geo->texels) memcpy(texels_out, geo->texels, (size_t)geo->numTexels * sizeof(fmgi_vec3));
    if (tiles == 0) return FMGI_OK;
    int dev_count = 0;
    if (hipGetDeviceCount(&dev_count) != hipSuccess || dev_count <= 0)
        return internal_set_err(FMGI_ERR_NO_DEVICE, "no HIP device visible");
    int rc = FMGI_OK;
    OutWall *d_walls = nullptr;
    float *d_tex = nullptr;
    uint8_t *d_rgb = nullptr;
    OutArgs a;
    memset(&a, 0, sizeof a);
    {
        const char *dv = getenv("FMGI_DEVICE");
        AOCHK(hipSetDevice(dv ? atoi(dv) : 0));
    }
    AOCHK(hipMalloc(&d_walls, ow.size() * sizeof(OutWall)));
    AOCHK(hipMemcpy(d_walls, ow.data(), ow.size() * sizeof(OutWall), hipMemcpyHostToDevice));
    AOCHK(hipMalloc(&d_tex, (size_t)geo->numTexels * sizeof(fmgi_vec3)));
    AOCHK(hipMemcpy(d_tex, texels_out, (size_t)geo->numTexels * sizeof(fmgi_vec3), hipMemcpyHostToDevice));
    AOCHK(hipMalloc(&d_rgb, (size_t)tiles * 3));
    a.walls = d_walls;
    a.nwalls = geo->numWalls;
    a.ntexels = tiles;
    a.texels = d_tex;
    a.rgb = d_rgb;
    a.normalise = spa > 0;
    a.tint_extra = tint != 0;
    AOCHK(fmgi_launch_output(a, nullptr));
    AOCHK(hipDeviceSynchronize());
    AOCHK(hipMemcpy(texels_out, d_tex, (size_t)geo->numTexels * sizeof(fmgi_vec3), hipMemcpyDeviceToHost));
    AOCHK(hipMemcpy(rgb_out, d_rgb, (size_t)tiles * 3, hipMemcpyDeviceToHost));
done:
    hipFree(d_walls);
    hipFree(d_tex);
    hipFree(d_rgb);
    return rc;
}

} // namespace

FMGI_API int64_t fmgi_output_tile_bytes(const fmgi_geometry *geo) {
    if (!geo || (geo->numWalls && !geo->walls)) return internal_set_err(FMGI_ERR_ARG, "bad geometry");
    int64_t n = 0;
    for (int i = 0; i < geo->numWalls; i++) n += 3 * (int64_t)geo->walls[i].lightmapSetup[1] * geo->walls[i].lightmapSetup[2];
    return n;
}

FMGI_API int fmgi_output_tiles(const fmgi_geometry *geo, int numSamplesPerArea, int tintExtra, fmgi_vec3 *texels_out,
                               uint8_t *rgb_out) {
    return output_run(geo, numSamplesPerArea, tintExtra, texels_out, rgb_out);
}

FMGI_API int fmgi_geosphere(int levels, float *xyz, int cap) {
    if (levels < 1 || levels > 6) return internal_set_err(FMGI_ERR_ARG, "fmgi_geosphere: levels must be 1..6");
    const std::vector<float> t = fmgi_geo::geosphere(levels);
    const int n = (int)(t.size() / 3);
    if (xyz) memcpy(xyz, t.data(), (size_t)std::min(n, std::max(cap, 0)) * 3 * sizeof(float));
    return n;
}

FMGI_API int64_t fmgi_ao_tree(const fmgi_geometry *geo, int32_t *out, int64_t cap) {
    if (!geo || (geo->numWalls && !geo->walls)) return internal_set_err(FMGI_ERR_ARG, "fmgi_ao_tree: bad geometry");
    const Tree t = build_tree(geo->walls, geo->numWalls);
    std::vector<int32_t> enc;
    for (const Node &nd : t.nodes) {
        enc.push_back(nd.left);
        enc.push_back(nd.right);
        enc.push_back(nd.plane);
        enc.push_back((int32_t)nd.items.size());
        for (int w : nd.items) enc.push_back(w);
    }
    if (out) memcpy(out, enc.data(), (size_t)std::min<int64_t>((int64_t)enc.size(), std::max<int64_t>(cap, 0)) * 4);
    return (int64_t)enc.size();
}

FMGI_API int fmgi_ambient_occlusion(const fmgi_geometry *geo, int wall_begin, int wall_end, fmgi_vec3 *texels_out) {
    return ao_run(geo, wall_begin, wall_end, texels_out);
}

FMGI_API void performAmbientOcclusionGpu(fmgi_geometry *geo) {
    const int rc = geo ? ao_run(geo, 0, geo->numWalls, geo->texels) : internal_set_err(FMGI_ERR_ARG, "null geometry");
    if (rc != FMGI_OK) {
        printf("[Err] performAmbientOcclusionGpu: %s\n", fmgi_last_error());
        fflush(stdout);
        exit(-1);
    }
}
