/*
 * fmgi_rad_host.cpp -- host side of the radiosity backend (§8f rank 4) and its C ABI
 * (include/flatmatch_gi.h: performRadiosityGpu, fmgi_radiosity, fmgi_radiosity_jobs,
 * fmgi_radiosity_stats). The reference is performRadiosityNative (radiosityNative.c:92-268).
 *
 * The host
 *   - reads the caller's libc rand() state (glibc TYPE_3: 31 words and a read position), before any HIP
 *     call, since the HIP runtime's first initialisation itself draws a rand() value;
 *   - builds the rectangle list with the window/light texel bases appended after numTexels
 *     (radiosityNative.c:108-131) and one job per level-0 wall texel, in the reference's wall/tile
 *     order, which is also its rand() order;
 *   - builds the jump matrices M^(2500 * 2^b) of the generator's linear recurrence;
 *   - runs the device phases (fmgi_rad.hip) and copies texels [0, numTexels) back;
 *   - leaves the libc generator exactly where 2 x 10000 x jobs rand() calls would have left it.
 * Geometry precomputation is fp32 in the reference's order (built with -ffp-contract=off, no FMA).
 */
#include <hip/hip_runtime_api.h>

#include <math.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <vector>

#include "../../include/flatmatch_gi.h"
#include "fmgi_rad.h"

#define FMGI_API extern "C" __attribute__((visibility("default")))

int internal_set_err(int code, const char *msg);

namespace {

struct F3 {
    float x, y, z;
};
F3 f3of(const fmgi_vec3 &v) { return F3{v.s[0], v.s[1], v.s[2]}; }
F3 add(F3 a, F3 b) { return F3{a.x + b.x, a.y + b.y, a.z + b.z}; }
F3 mul(F3 a, float f) { return F3{a.x * f, a.y * f, a.z * f}; }
float dot(F3 a, F3 b) { return a.x * b.x + a.y * b.y + a.z * b.z; }
F3 cross(F3 a, F3 b) { return F3{a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x}; }
float length(F3 a) { return sqrtf(a.x * a.x + a.y * a.y + a.z * a.z); }
F3 div_vec3(F3 a, float b) { return mul(a, 1.0f / b); } /* vector3_cl.c:53-58 */
F3 normalized(F3 a) { return mul(a, 1.0f / length(a)); } /* vector3_cl.c:95-101 */

constexpr int DEG = FMGI_RAND_DEG;
using Mat = std::vector<uint32_t>; /* 31x31 row-major over Z/2^32 */

/* one step of glibc random_r TYPE_3 on the window (x[n-31] .. x[n-1]): shift, append x[n-31] + x[n-3] */
Mat step_matrix() {
    Mat m((size_t)DEG * DEG, 0);
    for (int i = 0; i + 1 < DEG; i++) m[(size_t)i * DEG + i + 1] = 1;
    m[(size_t)(DEG - 1) * DEG + 0] += 1;
    m[(size_t)(DEG - 1) * DEG + 28] += 1;
    return m;
}

Mat mat_mul(const Mat &a, const Mat &b) {
    Mat c((size_t)DEG * DEG, 0);
    for (int i = 0; i < DEG; i++)
        for (int k = 0; k < DEG; k++) {
            const uint32_t aik = a[(size_t)i * DEG + k];
            if (!aik) continue;
            for (int j = 0; j < DEG; j++) c[(size_t)i * DEG + j] += aik * b[(size_t)k * DEG + j];
        }
    return c;
}

void mat_vec(const Mat &a, const uint32_t *x, uint32_t *y) {
    uint32_t t[DEG];
    for (int i = 0; i < DEG; i++) {
        uint32_t s = 0;
        for (int k = 0; k < DEG; k++) s += a[(size_t)i * DEG + k] * x[k];
        t[i] = s;
    }
    memcpy(y, t, sizeof t);
}

Mat mat_pow(Mat base, uint64_t e) {
    Mat r((size_t)DEG * DEG, 0);
    for (int i = 0; i < DEG; i++) r[(size_t)i * DEG + i] = 1;
    while (e) {
        if (e & 1) r = mat_mul(r, base);
        e >>= 1;
        if (e) base = mat_mul(base, base);
    }
    return r;
}

/*
 * The caller's glibc rand() generator. glibc keeps the TYPE_3 state as an int32 header word followed
 * by 31 words; initstate() on another buffer records the read position in that header (5 * rear + type,
 * random_r.c __initstate_r) and setstate() reloads it (the front index is rear + 3 mod 31).
 */
struct LibcRand {
    int32_t *hdr = nullptr;
    int rear = 0, front = 0;
    bool read(uint32_t v[DEG]) {
#ifdef __GLIBC__
        static char scratch[128];
        hdr = (int32_t *)initstate(1, scratch, sizeof scratch);
        if (!hdr) return false;
        const int32_t h = hdr[0];
        setstate((char *)hdr);
        if (h % 5 != 3) return false; /* TYPE_3 only: the default state and srand() keep it */
        rear = h / 5;
        front = (rear + 3) % DEG;
        const uint32_t *st = (const uint32_t *)(hdr + 1);
        for (int j = 0; j < DEG; j++) v[j] = st[(front + j) % DEG]; /* oldest (the next front) first */
        return true;
#else
        return false;
#endif
    }
    /* install window v as the state after `steps` calls from the one read() saw */
    void write(const uint32_t v[DEG], uint64_t steps) {
#ifdef __GLIBC__
        static char scratch2[128];
        initstate(1, scratch2, sizeof scratch2); /* leave the caller's array (its header is rewritten) */
        const int f = (int)((front + steps) % DEG), r = (int)((rear + steps) % DEG);
        uint32_t *st = (uint32_t *)(hdr + 1);
        for (int j = 0; j < DEG; j++) st[(f + j) % DEG] = v[j];
        hdr[0] = 5 * r + 3;
        setstate((char *)hdr);
#endif
    }
};

int num_mip_texels(const int32_t *lm) { /* rectangle.c:166-190 (asserts compiled out) */
    int w = lm[1], h = lm[2], n = w * h;
    while (w > 1 || h > 1) {
        if (w > 1) w /= 2;
        if (h > 1) h /= 2;
        n += w * h;
    }
    return n;
}

AoRect hit_rect(const fmgi_rect &r) { /* intersects()'s per-call values, rectangle.c:67-95 */
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

fmgi_rad_stats g_stats;

#define RADCHK(expr)                                                                                   \
    do {                                                                                               \
        hipError_t e_ = (expr);                                                                        \
        if (e_ != hipSuccess) {                                                                        \
            char b_[256];                                                                              \
            snprintf(b_, sizeof b_, "%s: %s", #expr, hipGetErrorString(e_));                           \
            rc = internal_set_err(FMGI_ERR_HIP, b_);                                                   \
            goto done;                                                                                 \
        }                                                                                              \
    } while (0)

int64_t count_jobs(const fmgi_geometry *geo) {
    int64_t n = 0;
    for (int i = 0; i < geo->numWalls; i++) n += (int64_t)geo->walls[i].lightmapSetup[1] * geo->walls[i].lightmapSetup[2];
    return n;
}

int check_geometry(const fmgi_geometry *geo) {
    if (!geo) return internal_set_err(FMGI_ERR_ARG, "fmgi_radiosity: null geometry");
    if (geo->numWalls < 0 || geo->numWindows < 0 || geo->numLights < 0 || geo->numTexels < 0 ||
        (geo->numWalls && !geo->walls) || (geo->numWindows && !geo->windows) || (geo->numLights && !geo->lights) ||
        (geo->numTexels && !geo->texels))
        return internal_set_err(FMGI_ERR_ARG, "fmgi_radiosity: bad geometry");
    std::vector<std::pair<int64_t, int64_t>> spans;
    const fmgi_rect *sets[3] = {geo->walls, geo->windows, geo->lights};
    const int counts[3] = {geo->numWalls, geo->numWindows, geo->numLights};
    for (int s = 0; s < 3; s++)
        for (int i = 0; i < counts[s]; i++) {
            const int32_t *lm = sets[s][i].lightmapSetup;
            if (lm[1] < 1 || lm[2] < 1 || (int64_t)lm[1] * lm[2] > (1 << 28))
                return internal_set_err(FMGI_ERR_ARG, "fmgi_radiosity: a rectangle has an empty or huge lightmap");
            if (s == 0) {
                if (lm[0] < 0 || (int64_t)lm[0] + num_mip_texels(lm) > geo->numTexels)
                    return internal_set_err(FMGI_ERR_ARG, "fmgi_radiosity: a wall's texels lie outside numTexels");
                spans.push_back({lm[0], (int64_t)lm[0] + (int64_t)lm[1] * lm[2]});
            }
        }
    std::sort(spans.begin(), spans.end());
    for (size_t i = 1; i < spans.size(); i++)
        if (spans[i].first < spans[i - 1].second)
            return internal_set_err(FMGI_ERR_ARG, "fmgi_radiosity: two walls share level-0 texels");
    const int64_t nr = (int64_t)geo->numWalls + geo->numWindows + geo->numLights;
    if (nr > FMGI_RAD_MAX_SORT)
        return internal_set_err(FMGI_ERR_ARG, "fmgi_radiosity: more rectangles than the candidate sort holds (16384)");
    return FMGI_OK;
}

int rad_run(const fmgi_geometry *geo, fmgi_vec3 *texels_out, int32_t *sids_out) {
    int rc = check_geometry(geo);
    if (rc != FMGI_OK) return rc;
    if (!texels_out && geo->numTexels) return internal_set_err(FMGI_ERR_ARG, "fmgi_radiosity: null texels_out");
    LibcRand libc;
    uint32_t v0[DEG];
    if (!libc.read(v0))
        return internal_set_err(FMGI_ERR_ARG, "fmgi_radiosity: libc rand() is not in glibc's default TYPE_3 state");

    /* the rectangle list, radiosityNative.c:108-131 */
    const int nr = geo->numWalls + geo->numWindows + geo->numLights;
    std::vector<fmgi_rect> all;
    all.reserve((size_t)nr);
    for (int i = 0; i < geo->numWalls; i++) all.push_back(geo->walls[i]);
    for (int i = 0; i < geo->numWindows; i++) all.push_back(geo->windows[i]);
    for (int i = 0; i < geo->numLights; i++) all.push_back(geo->lights[i]);
    int64_t ntex = geo->numTexels;
    for (int i = geo->numWalls; i < nr; i++) {
        if (ntex > INT32_MAX) return internal_set_err(FMGI_ERR_ARG, "fmgi_radiosity: too many texels");
        all[(size_t)i].lightmapSetup[0] = (int32_t)ntex;
        ntex += num_mip_texels(all[(size_t)i].lightmapSetup);
    }
    const int64_t first_light = geo->numLights ? all[(size_t)(geo->numWalls + geo->numWindows)].lightmapSetup[0] : ntex;
    std::vector<RadRect> rects((size_t)std::max(nr, 1));
    std::vector<AoRect> hits((size_t)std::max(nr, 1));
    for (int i = 0; i < nr; i++) {
        const fmgi_rect &r = all[(size_t)i];
        RadRect &o = rects[(size_t)i];
        o.px = r.pos.s[0], o.py = r.pos.s[1], o.pz = r.pos.s[2];
        o.wx = r.width.s[0], o.wy = r.width.s[1], o.wz = r.width.s[2];
        o.hx = r.height.s[0], o.hy = r.height.s[1], o.hz = r.height.s[2];
        o.nx = r.n.s[0], o.ny = r.n.s[1], o.nz = r.n.s[2];
        o.s0 = r.lightmapSetup[0], o.s1 = r.lightmapSetup[1], o.s2 = r.lightmapSetup[2], o.pad = 0;
        hits[(size_t)i] = hit_rect(r);
    }
    int sort_n = 2;
    while (sort_n < nr) sort_n <<= 1;

    /* jobs: every level-0 wall texel, wall/tile order (radiosityNative.c:166-176) */
    const int64_t njobs = count_jobs(geo);
    std::vector<RadJob> jobs((size_t)std::max<int64_t>(njobs, 1));
    {
        int64_t j = 0;
        for (int w = 0; w < geo->numWalls; w++) {
            const fmgi_rect &r = geo->walls[w];
            const int s1 = r.lightmapSetup[1], s2 = r.lightmapSetup[2];
            const F3 vw = div_vec3(f3of(r.width), (float)s1), vh = div_vec3(f3of(r.height), (float)s2);
            const F3 n = f3of(r.n);
            /* getCosineDistributedRandomRay's basis (vector3_cl.c:140-145) */
            F3 ud{0, 0, 1};
            if (fabs(dot(ud, n)) >= 0.999999f) ud = F3{0, 1, 0};
            const F3 vd = normalized(cross(ud, n));
            ud = normalized(cross(vd, n));
            for (int t = 0; t < s1 * s2; t++, j++) {
                RadJob &o = jobs[(size_t)j];
                memset(&o, 0, sizeof o);
                const int tx = t % s1, ty = t / s1; /* getTileCenter (rectangle.c:140-153) */
                const F3 c = add(add(f3of(r.pos), mul(vw, (float)(tx + 0.5))), mul(vh, (float)(ty + 0.5)));
                o.cx = c.x, o.cy = c.y, o.cz = c.z;
                o.nx = n.x, o.ny = n.y, o.nz = n.z;
                o.ux = ud.x, o.uy = ud.y, o.uz = ud.z;
                o.vx = vd.x, o.vy = vd.y, o.vz = vd.z;
                o.texel = r.lightmapSetup[0] + t;
            }
        }
    }

    /* jump matrices and the generator's final window after 20000 draws per job */
    std::vector<uint32_t> jump((size_t)FMGI_RAD_JUMP_BITS * DEG * DEG);
    Mat p = mat_pow(step_matrix(), FMGI_RAD_SUBLEN);
    for (int b = 0; b < FMGI_RAD_JUMP_BITS; b++) {
        memcpy(&jump[(size_t)b * DEG * DEG], p.data(), (size_t)DEG * DEG * 4);
        if (b + 1 < FMGI_RAD_JUMP_BITS) p = mat_mul(p, p);
    }
    const uint64_t qend = (uint64_t)njobs * FMGI_RAD_SUBS;
    if (qend >> FMGI_RAD_JUMP_BITS) return internal_set_err(FMGI_ERR_ARG, "fmgi_radiosity: too many texels");
    uint32_t vend[DEG];
    memcpy(vend, v0, sizeof vend);
    for (int b = 0; b < FMGI_RAD_JUMP_BITS; b++)
        if ((qend >> b) & 1) {
            Mat pb(jump.begin() + (size_t)b * DEG * DEG, jump.begin() + (size_t)(b + 1) * DEG * DEG);
            mat_vec(pb, vend, vend);
        }

    memset(&g_stats, 0, sizeof g_stats);
    g_stats.jobs = njobs;
    g_stats.rects = nr;
    g_stats.texels = ntex;
    g_stats.rays = njobs * FMGI_RAD_RAYS;

    int dev_count = 0;
    RadRect *d_rects = nullptr;
    AoRect *d_hits = nullptr;
    RadJob *d_jobs = nullptr;
    uint32_t *d_jump = nullptr, *d_v0 = nullptr, *d_draws = nullptr;
    int32_t *d_sids = nullptr;
    float4 *d_src = nullptr, *d_dst = nullptr, *d_dest = nullptr;
    hipEvent_t ev[4] = {nullptr, nullptr, nullptr, nullptr};
    std::vector<float4> init((size_t)std::max<int64_t>(ntex, 1));
    int64_t chunk = 1;
    RadArgs a;
    RadBounce bb;
    memset(&a, 0, sizeof a);
    memset(&bb, 0, sizeof bb);
    if (hipGetDeviceCount(&dev_count) != hipSuccess || dev_count <= 0) {
        libc.write(v0, 0);
        return internal_set_err(FMGI_ERR_NO_DEVICE, "no HIP device visible");
    }
    {
        const char *dv = getenv("FMGI_DEVICE");
        RADCHK(hipSetDevice(dv ? atoi(dv) : 0));
    }
    for (auto &e : ev) RADCHK(hipEventCreate(&e));
    RADCHK(hipEventRecord(ev[0], nullptr));
    RADCHK(hipMalloc(&d_rects, rects.size() * sizeof(RadRect)));
    RADCHK(hipMemcpy(d_rects, rects.data(), rects.size() * sizeof(RadRect), hipMemcpyHostToDevice));
    RADCHK(hipMalloc(&d_hits, hits.size() * sizeof(AoRect)));
    RADCHK(hipMemcpy(d_hits, hits.data(), hits.size() * sizeof(AoRect), hipMemcpyHostToDevice));
    RADCHK(hipMalloc(&d_jobs, jobs.size() * sizeof(RadJob)));
    RADCHK(hipMemcpy(d_jobs, jobs.data(), jobs.size() * sizeof(RadJob), hipMemcpyHostToDevice));
    RADCHK(hipMalloc(&d_jump, jump.size() * 4));
    RADCHK(hipMemcpy(d_jump, jump.data(), jump.size() * 4, hipMemcpyHostToDevice));
    RADCHK(hipMalloc(&d_v0, DEG * 4));
    RADCHK(hipMemcpy(d_v0, v0, DEG * 4, hipMemcpyHostToDevice));
    RADCHK(hipMalloc(&d_sids, (size_t)std::max<int64_t>(njobs, 1) * FMGI_RAD_RAYS * 4));
    {
        /* rand() draws of a chunk of jobs: at most 1/8 of free memory, at most 4 GiB */
        size_t fr = 0, tot = 0;
        RADCHK(hipMemGetInfo(&fr, &tot));
        const size_t cap = std::min<size_t>(fr / 8, (size_t)4 << 30);
        chunk = std::max<int64_t>(1, std::min<int64_t>(njobs, (int64_t)(cap / ((size_t)FMGI_RAD_DRAWS * 4))));
        const char *ce = getenv("FMGI_RAD_CHUNK"); /* tests: force several chunks */
        if (ce && atoll(ce) > 0) chunk = std::min<int64_t>(std::max<int64_t>(njobs, 1), atoll(ce));
    }
    RADCHK(hipMalloc(&d_draws, (size_t)chunk * FMGI_RAD_DRAWS * 4));
    a.rects = d_rects;
    a.hits = d_hits;
    a.nrects = nr;
    a.sort_n = sort_n;
    a.jobs = d_jobs;
    a.njobs = njobs;
    a.jump = d_jump;
    a.v0 = d_v0;
    a.draws = d_draws;
    a.sids = d_sids;
    {
        float rand_ms = 0;
        for (int64_t j0 = 0; j0 < njobs; j0 += chunk) {
            a.job0 = j0;
            a.nchunk = std::min(chunk, njobs - j0);
            RADCHK(hipEventRecord(ev[1], nullptr));
            RADCHK(fmgi_rad_launch_rand(a, nullptr));
            RADCHK(hipEventRecord(ev[2], nullptr));
            RADCHK(fmgi_rad_launch_rays(a, nullptr));
            RADCHK(hipEventSynchronize(ev[2]));
            float ms = 0;
            RADCHK(hipEventElapsedTime(&ms, ev[1], ev[2]));
            rand_ms += ms;
        }
        g_stats.rand_ms = rand_ms;
    }
    RADCHK(hipEventRecord(ev[1], nullptr));

    /* radiosity: walls 0, windows 30, lights (28, 28, 32) (radiosityNative.c:139-149) */
    for (int64_t i = 0; i < ntex; i++)
        init[(size_t)i] = i < geo->numTexels ? make_float4(0, 0, 0, 0)
                          : i < first_light  ? make_float4(30, 30, 30, 0)
                                             : make_float4(28, 28, 32, 0);
    RADCHK(hipMalloc(&d_src, init.size() * 16));
    RADCHK(hipMalloc(&d_dst, init.size() * 16));
    RADCHK(hipMalloc(&d_dest, init.size() * 16));
    RADCHK(hipMemcpy(d_src, init.data(), init.size() * 16, hipMemcpyHostToDevice));
    RADCHK(hipMemset(d_dest, 0, init.size() * 16));
    RADCHK(hipEventRecord(ev[2], nullptr));
    bb.sids = d_sids;
    bb.jobs = d_jobs;
    bb.njobs = njobs;
    bb.rects = d_rects;
    bb.nrects = nr;
    bb.ntex = ntex;
    bb.dest = d_dest;
    bb.keep = 1 - 0.3f; /* reflectance = 0.3 (float), radiosityNative.c:103 */
    bb.gain = 0.3f / FMGI_RAD_RAYS;
    for (int it = 0; it < FMGI_RAD_ITERS; it++) {
        bb.src = d_src;
        bb.dst = d_dst;
        RADCHK(fmgi_rad_launch_bounce(bb, nullptr));
        std::swap(d_src, d_dst);
    }
    RADCHK(hipEventRecord(ev[3], nullptr));
    if (geo->numTexels) RADCHK(hipMemcpy(texels_out, d_src, (size_t)geo->numTexels * 16, hipMemcpyDeviceToHost));
    if (sids_out && njobs) {
        std::vector<int32_t> h((size_t)njobs * FMGI_RAD_RAYS);
        RADCHK(hipMemcpy(h.data(), d_sids, h.size() * 4, hipMemcpyDeviceToHost));
        for (int64_t k = 0; k < FMGI_RAD_RAYS; k++) /* device ray-major -> the reference's per-texel rows */
            for (int64_t j = 0; j < njobs; j++) sids_out[j * FMGI_RAD_RAYS + k] = h[(size_t)(k * njobs + j)];
    }
    {
        float ms = 0;
        RADCHK(hipEventSynchronize(ev[3]));
        RADCHK(hipEventElapsedTime(&ms, ev[0], ev[1]));
        g_stats.rays_ms = ms - g_stats.rand_ms; /* rays + uploads */
        RADCHK(hipEventElapsedTime(&ms, ev[2], ev[3]));
        g_stats.bounce_ms = ms;
        RADCHK(hipEventElapsedTime(&ms, ev[0], ev[3]));
        g_stats.total_ms = ms;
    }
    libc.write(vend, 2ull * FMGI_RAD_RAYS * (uint64_t)njobs);
done:
    if (rc != FMGI_OK) libc.write(v0, 0);
    for (auto &e : ev)
        if (e) hipEventDestroy(e);
    hipFree(d_rects);
    hipFree(d_hits);
    hipFree(d_jobs);
    hipFree(d_jump);
    hipFree(d_v0);
    hipFree(d_draws);
    hipFree(d_sids);
    hipFree(d_src);
    hipFree(d_dst);
    hipFree(d_dest);
    return rc;
}

} // namespace

FMGI_API int fmgi_radiosity(const fmgi_geometry *geo, fmgi_vec3 *texels_out, int32_t *sids_out) {
    return rad_run(geo, texels_out, sids_out);
}

FMGI_API int fmgi_rand_skip(uint64_t n) {
    LibcRand libc;
    uint32_t v[DEG];
    if (!libc.read(v)) return internal_set_err(FMGI_ERR_ARG, "fmgi_rand_skip: libc rand() is not in glibc's TYPE_3 state");
    mat_vec(mat_pow(step_matrix(), n), v, v);
    libc.write(v, n);
    return FMGI_OK;
}

FMGI_API int64_t fmgi_radiosity_jobs(const fmgi_geometry *geo) {
    if (!geo || (geo->numWalls && !geo->walls)) return internal_set_err(FMGI_ERR_ARG, "bad geometry");
    return count_jobs(geo);
}

FMGI_API int fmgi_radiosity_stats(fmgi_rad_stats *out) {
    if (!out) return internal_set_err(FMGI_ERR_ARG, "null stats");
    *out = g_stats;
    return FMGI_OK;
}

FMGI_API void performRadiosityGpu(fmgi_geometry *geo) {
    const int rc = rad_run(geo, geo ? geo->texels : nullptr, nullptr);
    if (rc != FMGI_OK) {
        printf("[Err] performRadiosityGpu: %s\n", fmgi_last_error());
        fflush(stdout);
        exit(-1);
    }
}
