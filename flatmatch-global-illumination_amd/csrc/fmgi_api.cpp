/*
 * fmgi_api.cpp -- host side of libflatmatch_gi.so: the C ABI of include/flatmatch_gi.h.
 *
 * Replaces global_illumination_cl.c (the reference's OpenCL host driver):
 *   - device selection / context / runtime compile (global_illumination_cl.c:102-212) become
 *     hipGetDeviceCount/hipSetDevice and a code object linked into this library;
 *   - photonMapLightSource's per-source sample count and launch loop (global_illumination_cl.c:215-272)
 *     become fmgi_plan(): the same float arithmetic, the same `+1` work-group rounding, the same libc
 *     rand() call per launch -- flattened into one work-item list that a single persistent kernel drains;
 *   - performGlobalIlluminationCl (global_illumination_cl.c:275-321) keeps its signature and in-place
 *     texel update; the texel buffer is accumulated exactly in int64 fixed point and added once.
 * Compiled as host C++ with -ffp-contract=off: the per-rectangle precomputation below must produce the
 * same IEEE fp32 bits photonmap.cl computes on the device.
 */
#include <hip/hip_runtime_api.h>
#include <rccl/rccl.h>

#include <dlfcn.h>
#include <math.h>
#include <stdarg.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <map>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "../../include/flatmatch_gi.h"
#include "fmgi_internal.h"

#define FMGI_API extern "C" __attribute__((visibility("default")))

static_assert(sizeof(fmgi_rect) == 80, "Rectangle is 80 B (rectangle.h:19-26)");
static_assert(sizeof(fmgi_geometry) == 80, "Geometry is 80 B (geometry.h:7-15)");
static_assert(sizeof(fmgi_event) == 32, "fmgi_event is 32 B");
static_assert(sizeof(fmgi_launch) == sizeof(LaunchDev), "launch layout");

namespace {

thread_local std::string g_err;

int set_err(int code, const char *fmt, ...) {
    char buf[512];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof buf, fmt, ap);
    va_end(ap);
    g_err = buf;
    return code;
}

#define HIPCHK(expr)                                                                                   \
    do {                                                                                               \
        hipError_t e_ = (expr);                                                                        \
        if (e_ != hipSuccess) return set_err(FMGI_ERR_HIP, "%s: %s", #expr, hipGetErrorString(e_));    \
    } while (0)

} // namespace

/* fmgi_last_error() for the other host translation units (fmgi_ao_host.cpp) */
int internal_set_err(int code, const char *msg) { return set_err(code, "%s", msg); }

namespace {

f3 v3of(const fmgi_vec3 &v) { return mkf3(v.s[0], v.s[1], v.s[2]); }

/* A wall as the kernels read it: the reference Rectangle's fields; the values photonmap.cl derives from
   them with OpenCL builtins (lengths, unit edges, sampler basis) are filled in on the device by
   k_scene_setup, so they carry exactly the builtins' gfx950 bits. */
RectDev make_rect(const fmgi_rect &r) {
    RectDev d;
    memset(&d, 0, sizeof d);
    d.px = r.pos.s[0]; d.py = r.pos.s[1]; d.pz = r.pos.s[2];
    d.nx = r.n.s[0]; d.ny = r.n.s[1]; d.nz = r.n.s[2];
    d.base = r.lightmapSetup[0];
    d.W = r.lightmapSetup[1];
    d.H = r.lightmapSetup[2];
    d.axis = -1;
    return d;
}

/* An emitter (window or light); its sampler basis comes from k_scene_setup as well. */
SrcDev make_src(const fmgi_rect &r) {
    SrcDev s;
    memset(&s, 0, sizeof s);
    s.px = r.pos.s[0]; s.py = r.pos.s[1]; s.pz = r.pos.s[2];
    s.wx = r.width.s[0]; s.wy = r.width.s[1]; s.wz = r.width.s[2];
    s.hx = r.height.s[0]; s.hy = r.height.s[1]; s.hz = r.height.s[2];
    s.nx = r.n.s[0]; s.ny = r.n.s[1]; s.nz = r.n.s[2];
    return s;
}

/* global_illumination_cl.c:217-222: area in float, (float)spa*area/100 -> uint64, then
   (n / wg + 1) * wg (always at least one extra work group, as the reference does). */
uint64_t source_items(const fmgi_rect &src, float spa, uint64_t wg) {
    float area = host_len3(v3of(src.width)) * host_len3(v3of(src.height));
    uint64_t n = (uint64_t)((spa * area) / 100);
    return (n / wg + 1) * wg;
}

/*
 * Filter tables for ScanFast (fmgi_kernels.hip). A rect is "axis-aligned" when its normal, width and
 * height each have exactly one non-zero component, on three different axes: then photonmap.cl's dot
 * products reduce to one product each and the phase-1 value fac' = (plane - src_a) * rcp(dir_a) is within
 * 2^-20 relative of the exact fac. The extent along u/v is grown by a margin M that bounds every other
 * phase-1 vs exact difference for a hit inside the scene's bounding box (distance <= diagonal D,
 * coordinates <= S): |d| * |fac' - fac| <= D * 2^-20 plus a few ulps of S and D from the exact
 * ray/pDir/dot roundings and the phase-1 fma; M = max(S, D) * 2^-17 covers all of it with >= 4x slack.
 */
struct FilterBuild {
    std::vector<FilterRec> img; /* per axis a: J[a] pairs {+a record j, -a record j} */
    int J[3] = {0, 0, 0};
    std::vector<int32_t> general;
    float margin = 0;
    double scale = 1; /* B: scene scale the margin is derived from */
    std::vector<FilterRec> cls[3][2]; /* axis-aligned records by (axis, class), rect order */
    std::vector<int> pos[3][2];       /* cls[a][c][i] is the class-c half of image pair pos[a][c][i] */
};

int nonzero_axis(const float *v) {
    int axis = -1;
    for (int k = 0; k < 3; k++) {
        if (v[k] != 0.0f) {
            if (axis >= 0) return -1;
            axis = k;
        }
    }
    return axis;
}

FilterBuild build_filter(const fmgi_rect *walls, int nw, const fmgi_rect *srcs, int ns) {
    FilterBuild fb;
    double lo[3] = {1e300, 1e300, 1e300}, hi[3] = {-1e300, -1e300, -1e300};
    auto grow = [&](const fmgi_rect &r) {
        for (int cs = 0; cs < 4; cs++) {
            for (int k = 0; k < 3; k++) {
                double x = (double)r.pos.s[k] + ((cs & 1) ? (double)r.width.s[k] : 0.0) +
                           ((cs & 2) ? (double)r.height.s[k] : 0.0);
                lo[k] = std::min(lo[k], x);
                hi[k] = std::max(hi[k], x);
            }
        }
    };
    for (int i = 0; i < nw; i++) grow(walls[i]);
    for (int i = 0; i < ns; i++) grow(srcs[i]);
    double S = 0, D2 = 0;
    for (int k = 0; k < 3; k++) {
        if (nw + ns == 0) break;
        S = std::max(S, std::max(fabs(lo[k]), fabs(hi[k])));
        D2 += (hi[k] - lo[k]) * (hi[k] - lo[k]);
    }
    double B = std::max(std::max(S, sqrt(D2)), 1.0);
    fb.margin = (float)(B * (1.0 / 131072.0));
    fb.scale = B;
    std::vector<FilterRec>(&cls)[3][2] = fb.cls;
    for (int i = 0; i < nw; i++) {
        const fmgi_rect &r = walls[i];
        int a = nonzero_axis(r.n.s), aw = nonzero_axis(r.width.s), ah = nonzero_axis(r.height.s);
        if (a < 0 || aw < 0 || ah < 0 || aw == a || ah == a || aw == ah) {
            fb.general.push_back(i);
            continue;
        }
        int u = (a == 0) ? 1 : 0, v = (a == 2) ? 1 : 2;
        double e_lo[3], e_hi[3];
        for (int k = 0; k < 3; k++) {
            double p0 = r.pos.s[k], p1 = p0 + (double)r.width.s[k] + (double)r.height.s[k];
            e_lo[k] = std::min(p0, p1);
            e_hi[k] = std::max(p0, p1);
        }
        FilterRec f;
        memset(&f, 0, sizeof f);
        f.plane = r.pos.s[a];
        f.cu = (float)((e_lo[u] + e_hi[u]) * 0.5);
        f.hwu = (float)((e_hi[u] - e_lo[u]) * 0.5 + fb.margin);
        f.cv = (float)((e_lo[v] + e_hi[v]) * 0.5);
        f.hwv = (float)((e_hi[v] - e_lo[v]) * 0.5 + fb.margin);
        f.idx = i;
        cls[a][r.n.s[a] > 0 ? 0 : 1].push_back(f);
    }
    FilterRec sentinel;
    memset(&sentinel, 0, sizeof sentinel);
    sentinel.hwu = -1.0f; /* |x| <= -1 is never true: a padding entry is never a candidate */
    sentinel.hwv = -1.0f;
    sentinel.idx = -1;
    /* pair j = {record j of the +a class, record j of the -a class}, rect order. (Measured and dropped,
       profiles/r03/s10-s12: each class nearest-first with a wave-uniform early exit, 22.4 -> 31.6 ms on
       example.png; the two faces of a wall paired, pairs in Morton order, chunks of 4 culled against the
       box of the wave's ray segments, 29.8 ms: 64 random directions span the plan, nothing was culled,
       and both loops lost the filter's 4-deep LDS pipelining) */
    for (int a = 0; a < 3; a++) {
        fb.J[a] = (int)std::max(cls[a][0].size(), cls[a][1].size());
        for (int c = 0; c < 2; c++) {
            fb.pos[a][c].resize(cls[a][c].size());
            for (size_t i = 0; i < cls[a][c].size(); i++) fb.pos[a][c][i] = (int)i;
        }
        for (int j = 0; j < fb.J[a]; j++)
            for (int c = 0; c < 2; c++) fb.img.push_back(j < (int)cls[a][c].size() ? cls[a][c][j] : sentinel);
    }
    /* 8 padding pairs: a cooperative lane group reads up to coop - 1 records past the last class
       (k_bake, filter_axis) and discards them; they stay inside the staged image */
    for (int k = 0; k < 16; k++) fb.img.push_back(sentinel);
    return fb;
}

/* ScanHybrid's wall filter image (FilterPairHalf): for the x and y axes, groups g of records 2g, 2g + 1 of
   each class, in the class order of the filter image (rect order), +a class half first; G[a] groups */
std::vector<FilterPairHalf> build_filter_pairs(const FilterBuild &fb, int G[2]) {
    std::vector<FilterPairHalf> img;
    for (int a = 0; a < 2; a++) {
        G[a] = (fb.J[a] + 1) / 2;
        for (int g = 0; g < G[a]; g++)
            for (int c = 0; c < 2; c++) {
                FilterPairHalf h;
                for (int k = 0; k < 2; k++) {
                    const size_t j = (size_t)(2 * g + k);
                    const bool ok = j < fb.cls[a][c].size();
                    FilterRec r;
                    memset(&r, 0, sizeof r);
                    if (ok) r = fb.cls[a][c][j];
                    h.plane[k] = ok ? r.plane : 0.0f;
                    h.cu[k] = ok ? r.cu : 0.0f;
                    h.hwu[k] = ok ? r.hwu : -1.0f; /* |x| <= -1 never holds: never a candidate */
                    h.cv[k] = ok ? r.cv : 0.0f;
                    h.hwv[k] = ok ? r.hwv : -1.0f;
                    h.idx[k] = ok ? r.idx : -1;
                }
                img.push_back(h);
            }
    }
    return img;
}

template <class T>
hipError_t upload(T **dst, const std::vector<T> &v) {
    hipError_t e = hipMalloc(dst, v.size() * sizeof(T));
    if (e != hipSuccess) return e;
    return hipMemcpy(*dst, v.data(), v.size() * sizeof(T), hipMemcpyHostToDevice);
}

/*
 * Grid tables for ScanGrid (fmgi_kernels.hip). The records of each (axis, class) are grouped by plane
 * (identical float plane coordinate, so identical phase-1 fac'), and each plane's records are bucketed
 * by a uniform nu x nv grid over the bounding box of their grown extents (about 2 cells per record).
 * A record is registered in every cell its grown extent [c - hw, c + hw] overlaps, widened by `slack`
 * cells: the kernel's float cell coordinate t = (x - u0) * iu is within far less than that of the exact
 * value for any x in the scene box, so a hit point inside a record's grown extent always lands in a cell
 * that lists the record. Cell 0 is an empty cell used by the padding planes.
 */
struct GridBuild {
    std::vector<GridPlane> img; /* per axis a: J[a] pairs {+a plane j, -a plane j} */
    int J[3] = {0, 0, 0};
    std::vector<GridCell> cells;
    std::vector<GridCellF> cellsF; /* the same cells with float inline records (general grid walks) */
    std::vector<float> recs; /* overflow records {cu, hwu, cv, hwv} (cell entries 2..count) */
    std::vector<int32_t> idx;
};

/* The quantized inline records of a grid cell (GridCell): the kernel's float ops, replayed in float32 on the
   host (this file is built without FMA contraction). A record passes the float test iff |fl(x - c)| <= hw;
   fl(x - c) is monotone in x, so the passing floats form an interval [a, b] around c. Its ends are found
   exactly by a binary search over the ordered float bit patterns between c and -/+infinity (64 steps at
   most, whatever the ratio of hw to ulp(c)). */
static bool grid_pass(float x, float c, float hw) {
    const float d = x - c;
    return fabsf(d) <= hw;
}
/* a total order of the non-NaN floats as integers (-0 and +0 adjacent), and back */
static int64_t float_key(float x) {
    int32_t b;
    memcpy(&b, &x, 4);
    return b >= 0 ? (int64_t)b : -(int64_t)(b & 0x7FFFFFFF) - 1;
}
static float key_float(int64_t k) {
    const int32_t b = k >= 0 ? (int32_t)k : (int32_t)((-(k + 1)) | 0x80000000ll);
    float x;
    memcpy(&x, &b, 4);
    return x;
}
/* the last float from c towards +/-infinity that passes the record test (c itself passes for hw >= 0) */
static float grid_end(float c, float hw, bool hi) {
    const int64_t kc = float_key(c), kinf = float_key(hi ? INFINITY : -INFINITY);
    int64_t in = kc, out = kinf; /* in passes; out is the first key known to fail (or infinity) */
    if (grid_pass(key_float(out), c, hw)) return key_float(out);
    while (hi ? out - in > 1 : in - out > 1) {
        const int64_t mid = in + (out - in) / 2;
        if (grid_pass(key_float(mid), c, hw)) in = mid;
        else out = mid;
    }
    return key_float(in);
}
/* q of float coordinate x in cell column `cell` of an axis with origin o and inverse cell size inv: the
   kernel's (x - o) * inv, minus the cell, times 2^16, clamped to [0, 65535] and truncated (grid_cell) */
static uint32_t grid_q(float x, float o, float inv, int cell) {
    const float d = x - o;
    const float t = d * inv;
    const float r = t - (float)cell;
    const float m = r * 65536.0f;
    return (uint32_t)std::min(std::max(m, 0.0f), 65535.0f);
}
static uint32_t grid_bounds(float c, float hw, float o, float inv, int cell) {
    if (!(hw >= 0) || !grid_pass(c, c, hw)) return 0xFFFF0000u; /* (a degenerate record) pass-all */
    const float a = grid_end(c, hw, false), b = grid_end(c, hw, true);
    /* the ends pass and the floats just outside them fail (the superset the kernel's bounds rely on) */
    if (!grid_pass(a, c, hw) || !grid_pass(b, c, hw) || (a != -INFINITY && grid_pass(nextafterf(a, -INFINITY), c, hw)) ||
        (b != INFINITY && grid_pass(nextafterf(b, INFINITY), c, hw)))
        return 0xFFFF0000u;
    return grid_q(a, o, inv, cell) | (grid_q(b, o, inv, cell) << 16);
}

/* cells per record the grid's cost model may spend when forced (FMGI_GRID_CPR, experiment builds; 0 if unset);
   fmgi_set_grid_cells_per_record sets it per context (tests of the grids the product builds) */
static int grid_cpr_env() {
    const char *ce = fmgi_exp_env("FMGI_GRID_CPR");
    return ce && atoi(ce) >= 1 && atoi(ce) <= 64 ? atoi(ce) : 0;
}

GridBuild build_grid(const FilterBuild &fb, int cells_per_record) {
    GridBuild gb;
    gb.cells.push_back(GridCell{kGridNoRec, kGridNoRec, kGridNoRec, kGridNoRec, 0, -1, -1, 0}); /* cell 0: empty */
    gb.cellsF.push_back(GridCellF{0.f, -1.f, 0.f, -1.f, 0.f, -1.f, 0.f, -1.f, 0, -1, -1, 0});
    std::vector<GridPlane> planes[3][2];
    for (int a = 0; a < 3; a++) {
        for (int c = 0; c < 2; c++) {
            const std::vector<FilterRec> &L = fb.cls[a][c];
            std::vector<float> keys;
            for (const FilterRec &r : L)
                if (std::find_if(keys.begin(), keys.end(), [&](float k) { return memcmp(&k, &r.plane, 4) == 0; }) ==
                    keys.end())
                    keys.push_back(r.plane);
            for (float pk : keys) {
                std::vector<const FilterRec *> R;
                for (const FilterRec &r : L)
                    if (memcmp(&pk, &r.plane, 4) == 0) R.push_back(&r);
                double ulo = 1e300, uhi = -1e300, vlo = 1e300, vhi = -1e300;
                for (const FilterRec *r : R) {
                    ulo = std::min(ulo, (double)r->cu - r->hwu);
                    uhi = std::max(uhi, (double)r->cu + r->hwu);
                    vlo = std::min(vlo, (double)r->cv - r->hwv);
                    vhi = std::max(vhi, (double)r->cv + r->hwv);
                }
                const double eu = std::max(uhi - ulo, 1e-30), ev = std::max(vhi - vlo, 1e-30);
                auto lo_hi = [](double c, double hw, double o, double inv, double sl, int n, int &i0, int &i1) {
                    i0 = (int)std::floor((c - hw - o) * inv - sl);
                    i1 = (int)std::floor((c + hw - o) * inv + sl);
                    i0 = std::min(std::max(i0, 0), n - 1);
                    i1 = std::min(std::max(i1, 0), n - 1);
                };
                /* one axis of the grid: n cells of size e/m starting half a cell early when `half`
                   (so that rect edges on a regular lattice fall inside cells, not on their borders) */
                struct Axis {
                    float o, inv;
                    int n;
                    double slack;
                    std::vector<int> cnt; /* cells each record is registered in */
                };
                auto make_axis = [&](double lo, double e, int m, bool half, bool is_u) {
                    Axis ax;
                    const double cs = e / m;
                    ax.o = (float)(half ? lo - 0.5 * cs : lo);
                    ax.inv = (float)(1.0 / cs);
                    ax.n = m + (half ? 1 : 0);
                    /* slack in cells: float rounding of (x - o) and of the product, for |x| <= scale */
                    ax.slack = 1.0 / 64 + fb.scale * (double)ax.inv * 0x1p-18;
                    for (const FilterRec *r : R) {
                        int i0, i1;
                        lo_hi(is_u ? r->cu : r->cv, is_u ? r->hwu : r->hwv, ax.o, ax.inv, ax.slack, ax.n, i0, i1);
                        ax.cnt.push_back(i1 - i0 + 1);
                    }
                    return ax;
                };
                /* pick the grid minimising the expected records per lookup (uniform hit points over
                   the plane's box), with at most max(16, 16 x records) cells; ties -> fewer cells */
                const int k = (int)R.size(), cap = std::max(16, cells_per_record * k), mmax = std::min(128, cap);
                std::vector<Axis> us, vs;
                for (int m = 1; m <= mmax; m++)
                    for (int h = 0; h < 2; h++) {
                        us.push_back(make_axis(ulo, eu, m, h, true));
                        vs.push_back(make_axis(vlo, ev, m, h, false));
                    }
                double best_cost = 1e300;
                size_t bu = 0, bv = 0;
                for (size_t x = 0; x < us.size(); x++)
                    for (size_t y = 0; y < vs.size(); y++) {
                        const double cells = (double)us[x].n * vs[y].n;
                        if (cells > cap) continue;
                        double sum = 0;
                        for (int i = 0; i < k; i++) sum += (double)us[x].cnt[i] * vs[y].cnt[i];
                        const double cost = sum / cells + 1e-6 * cells;
                        if (cost < best_cost) {
                            best_cost = cost;
                            bu = x;
                            bv = y;
                        }
                    }
                const Axis &AU = us[bu], &AV = vs[bv];
                const int nu = AU.n, nv = AV.n;
                GridPlane g;
                memset(&g, 0, sizeof g);
                g.plane = pk;
                g.u0 = AU.o;
                g.v0 = AV.o;
                g.iu = AU.inv;
                g.iv = AV.inv;
                g.nu = nu;
                g.nv = nv;
                g.mu = (float)(nu - 1);
                g.mv = (float)(nv - 1);
                g.cell_off = (int32_t)gb.cells.size();
                /* the records' box, widened by far more than the rounding of the kernel's float hit
                   point and of |uh - cu| (so a point outside it fails every record test) */
                const double pad_u = 1e-5 * (fabs(ulo) + fabs(uhi) + 1.0), pad_v = 1e-5 * (fabs(vlo) + fabs(vhi) + 1.0);
                g.ulo = (float)(ulo - pad_u);
                g.uhi = (float)(uhi + pad_u);
                g.vlo = (float)(vlo - pad_v);
                g.vhi = (float)(vhi + pad_v);
                const double su = AU.slack, sv = AV.slack;
                std::vector<std::vector<const FilterRec *>> bucket((size_t)nu * nv);
                for (const FilterRec *r : R) {
                    int u0, u1, v0, v1;
                    lo_hi(r->cu, r->hwu, g.u0, g.iu, su, nu, u0, u1);
                    lo_hi(r->cv, r->hwv, g.v0, g.iv, sv, nv, v0, v1);
                    for (int iv = v0; iv <= v1; iv++)
                        for (int iu = u0; iu <= u1; iu++) bucket[(size_t)iv * nu + iu].push_back(r);
                }
                for (size_t ci = 0; ci < bucket.size(); ci++) {
                    const auto &b = bucket[ci];
                    const int iu = (int)(ci % (size_t)nu), iv = (int)(ci / (size_t)nu);
                    GridCell gc{kGridNoRec, kGridNoRec, kGridNoRec, kGridNoRec, (int32_t)b.size(), -1, -1,
                                (int32_t)gb.idx.size()};
                    if (b.size() > 0) {
                        gc.qu0 = grid_bounds(b[0]->cu, b[0]->hwu, g.u0, g.iu, iu);
                        gc.qv0 = grid_bounds(b[0]->cv, b[0]->hwv, g.v0, g.iv, iv);
                        gc.idx0 = b[0]->idx;
                    }
                    if (b.size() > 1) {
                        gc.qu1 = grid_bounds(b[1]->cu, b[1]->hwu, g.u0, g.iu, iu);
                        gc.qv1 = grid_bounds(b[1]->cv, b[1]->hwv, g.v0, g.iv, iv);
                        gc.idx1 = b[1]->idx;
                    }
                    GridCellF gf{0.f, -1.f, 0.f, -1.f, 0.f, -1.f, 0.f, -1.f, (int32_t)b.size(), -1, -1, gc.rest};
                    if (b.size() > 0) {
                        gf.cu0 = b[0]->cu, gf.hwu0 = b[0]->hwu, gf.cv0 = b[0]->cv, gf.hwv0 = b[0]->hwv;
                        gf.idx0 = b[0]->idx;
                    }
                    if (b.size() > 1) {
                        gf.cu1 = b[1]->cu, gf.hwu1 = b[1]->hwu, gf.cv1 = b[1]->cv, gf.hwv1 = b[1]->hwv;
                        gf.idx1 = b[1]->idx;
                    }
                    for (size_t k = 2; k < b.size(); k++) {
                        gb.recs.insert(gb.recs.end(), {b[k]->cu, b[k]->hwu, b[k]->cv, b[k]->hwv});
                        gb.idx.push_back(b[k]->idx);
                    }
                    gb.cells.push_back(gc);
                    gb.cellsF.push_back(gf);
                }
                planes[a][c].push_back(g);
            }
            /* nearest first along the lanes that face this class: the +a class (c = 0) is faced by rays
               going -a, so its planes run by descending coordinate, the -a class by ascending; fac' is
               then non-decreasing along a lane's walk and ScanGrid can stop early */
            std::stable_sort(planes[a][c].begin(), planes[a][c].end(), [c](const GridPlane &x, const GridPlane &y) {
                return c == 0 ? x.plane > y.plane : x.plane < y.plane;
            });
        }
    }
    GridPlane pad;
    memset(&pad, 0, sizeof pad);
    pad.plane = NAN; /* fac' = NaN: never a candidate */
    pad.nu = pad.nv = 1;
    pad.mu = pad.mv = 0.0f;
    pad.cell_off = 0;
    pad.ulo = pad.vlo = -INFINITY; /* never culled; fac' = NaN keeps it out anyway */
    pad.uhi = pad.vhi = INFINITY;
    for (int a = 0; a < 3; a++) {
        gb.J[a] = (int)std::max(planes[a][0].size(), planes[a][1].size());
        for (int j = 0; j < gb.J[a]; j++)
            for (int c = 0; c < 2; c++) gb.img.push_back(j < (int)planes[a][c].size() ? planes[a][c][j] : pad);
    }
    if (gb.img.empty()) gb.img.push_back(pad);
    if (gb.idx.empty()) { /* keep the device arrays non-empty */
        gb.recs.insert(gb.recs.end(), {0.f, -1.f, 0.f, -1.f});
        gb.idx.push_back(-1);
    }
    return gb;
}

/*
 * Floor plan of the walls for ScanHybrid's wall pass (fmgi_kernels.hip plan_walls). The x- and y-axis
 * records of the filter image are vertical walls: seen from above, a segment x = X, y in
 * [cu - hwu, cu + hwu] (or y = Y, x in [...]). A uniform nx x ny grid of square cells covers the walls and
 * the sources; each cell lists (as u16 indices r of 32-B records in the filter image: byte offset 32 r) every
 * wall whose footprint, grown by `slack`, overlaps it. A lane walks the cells its ray crosses, nearest
 * first, tests the listed walls it faces with the filter's own float ops, and stops once the ray leaves
 * the cell past the 2^-11 band above its best key. Why that finds every wall the filter would find with a
 * key inside the band: a wall that passes its filter test at key f contains the computed hit point, which
 * lies within |d| f 2^-20 + a few ulps of the exact ray point at parameter f; that ray point lies in a cell
 * the walk visits (f <= band < the exit parameter of the last cell, up to the same rounding), and the wall
 * is registered in every cell within `slack` of its footprint, which bounds both roundings and the walk's
 * own cell arithmetic. Walls beyond the band cannot win or change the separation test (grid_phase1_sorted).
 * Layout (LDS, after the plane image): {x0, y0, ics, cs} {nx | ny << 16, ncells, nentries, 0}, then
 * u16 start[ncells + 1] (cell i's entries are entry[start[i] .. start[i + 1])), then u16 entry[].
 */
struct PlanBuild {
    float x0 = 0, y0 = 0, ics = 0, cs = 0;
    int nx = 0, ny = 0;
    std::vector<uint16_t> start, entry;
    bool ok = false;
    std::vector<char> blob() const {
        std::vector<char> b(32 + 2 * (start.size() + entry.size()));
        const float h0[4] = {x0, y0, ics, cs};
        const int32_t h1[4] = {nx | (ny << 16), (int32_t)start.size() - 1, (int32_t)entry.size(), 0};
        memcpy(b.data(), h0, 16);
        memcpy(b.data() + 16, h1, 16);
        memcpy(b.data() + 32, start.data(), 2 * start.size());
        memcpy(b.data() + 32 + 2 * start.size(), entry.data(), 2 * entry.size());
        b.resize((b.size() + 15) & ~(size_t)15);
        return b;
    }
};

PlanBuild build_plan(const FilterBuild &fb, const fmgi_rect *srcs, int ns) {
    PlanBuild pb;
    struct Seg { double a_lo, a_hi, b_lo, b_hi; int r; }; /* footprint box in (x, y) and record index */
    std::vector<Seg> segs;
    for (int a = 0; a < 2; a++)
        for (int c = 0; c < 2; c++)
            for (int j = 0; j < (int)fb.cls[a][c].size(); j++) {
                const FilterRec &f = fb.cls[a][c][j];
                const int r = 2 * ((a == 0 ? 0 : fb.J[0]) + fb.pos[a][c][j]) + c;
                const double lo_u = (double)f.cu - f.hwu, hi_u = (double)f.cu + f.hwu;
                /* x-walls (a = 0): x = plane, y = u; y-walls: y = plane, x = u */
                if (a == 0) segs.push_back({f.plane, f.plane, lo_u, hi_u, r});
                else segs.push_back({lo_u, hi_u, f.plane, f.plane, r});
            }
    if (segs.empty() || fb.J[0] + fb.J[1] > 16000) return pb; /* u16 record indices */
    double xlo = 1e300, xhi = -1e300, ylo = 1e300, yhi = -1e300;
    for (const Seg &s : segs) {
        xlo = std::min(xlo, s.a_lo), xhi = std::max(xhi, s.a_hi);
        ylo = std::min(ylo, s.b_lo), yhi = std::max(yhi, s.b_hi);
    }
    for (int i = 0; i < ns; i++)
        for (int k = 0; k < 4; k++) {
            const double x = (double)srcs[i].pos.s[0] + ((k & 1) ? srcs[i].width.s[0] : 0.f) + ((k & 2) ? srcs[i].height.s[0] : 0.f);
            const double y = (double)srcs[i].pos.s[1] + ((k & 1) ? srcs[i].width.s[1] : 0.f) + ((k & 2) ? srcs[i].height.s[1] : 0.f);
            xlo = std::min(xlo, x), xhi = std::max(xhi, x), ylo = std::min(ylo, y), yhi = std::max(yhi, y);
        }
    const double ex = std::max(xhi - xlo, 1e-6), ey = std::max(yhi - ylo, 1e-6);
    /* the cell size: minimise the expected cost of one walk, (cells visited) x (1 + entries per cell:
       the faced half, doubled for rays that start beside walls), with 1 + 1.27 l / cs cells visited for a horizontal run l of 0.6 x the walls' median height
       (a ray between floor and ceiling; fitted on example.png and the 30-room layout, tests/test_plan.py),
       over cells from 1/4 to 1/64 of the larger extent (FMGI_PLAN_CELLS forces the cells along the larger
       extent, experiments) */
    double run = 1.0;
    {
        std::vector<double> hs;
        for (int a = 0; a < 2; a++)
            for (int c = 0; c < 2; c++)
                for (const FilterRec &f : fb.cls[a][c]) hs.push_back(2.0 * ((double)f.hwv - fb.margin));
        if (!hs.empty()) {
            std::nth_element(hs.begin(), hs.begin() + hs.size() / 2, hs.end());
            run = std::max(0.6 * hs[hs.size() / 2], 1e-3);
        }
    }
    auto regs = [&](double cs, double x0, double y0, double sl, int nx, int ny, std::vector<uint16_t> *st,
                    std::vector<uint16_t> *en) -> size_t {
        std::vector<std::vector<uint16_t>> cell(st ? (size_t)nx * ny : 0);
        size_t n = 0;
        for (const Seg &s : segs) {
            const int i0 = std::max(0, (int)std::floor((s.a_lo - sl - x0) / cs));
            const int i1 = std::min(nx - 1, (int)std::floor((s.a_hi + sl - x0) / cs));
            const int j0 = std::max(0, (int)std::floor((s.b_lo - sl - y0) / cs));
            const int j1 = std::min(ny - 1, (int)std::floor((s.b_hi + sl - y0) / cs));
            for (int jy = j0; jy <= j1; jy++)
                for (int ix = i0; ix <= i1; ix++) {
                    n++;
                    if (st) cell[(size_t)jy * nx + ix].push_back((uint16_t)s.r);
                }
        }
        if (st) {
            st->assign(1, 0);
            en->clear();
            for (const auto &v : cell) {
                en->insert(en->end(), v.begin(), v.end());
                st->push_back((uint16_t)std::min<size_t>(en->size(), 65535));
            }
        }
        return n;
    };
    const double big = std::max(ex, ey);
    int m_lo = 4, m_hi = 64;
    if (const char *pe = fmgi_exp_env("FMGI_PLAN_CELLS"))
        if (atoi(pe) >= 1 && atoi(pe) <= 256) m_lo = m_hi = atoi(pe);
    double best = 1e300;
    for (int m = m_lo; m <= m_hi; m++) {
        const double cs = big / m;
        /* slack: the filter margin (the footprint's own growth already holds it along the wall; across
           the wall it is needed here), plus 1/64 cell for the walk's float cell arithmetic */
        const double sl = (double)fb.margin + cs / 64 + fb.scale * 0x1p-18;
        const double x0 = xlo - cs, y0 = ylo - cs;
        const int nx = (int)std::ceil(ex / cs) + 3, ny = (int)std::ceil(ey / cs) + 3;
        if ((int64_t)nx * ny > 4096 || nx > 255 || ny > 255) continue;
        const size_t n = regs(cs, x0, y0, sl, nx, ny, nullptr, nullptr);
        if (n > 60000) continue;
        const double cost = (1.0 + 1.27 * run / cs) * (1.0 + (double)n / ((double)nx * ny));
        if (cost < best) {
            best = cost;
            pb.cs = (float)cs;
            pb.nx = nx;
            pb.ny = ny;
        }
    }
    if (best == 1e300) return pb;
    const double cs = pb.cs; /* the float cell size the kernel uses */
    pb.ics = (float)(1.0 / cs);
    pb.x0 = (float)(xlo - cs);
    pb.y0 = (float)(ylo - cs);
    const double sl = (double)fb.margin + cs / 64 + fb.scale * 0x1p-18;
    regs(cs, pb.x0, pb.y0, sl, pb.nx, pb.ny, &pb.start, &pb.entry);
    pb.ok = pb.entry.size() < 65535;
    return pb;
}

/* Exact deposit colour of every colour state (kernel: k_bake's `sid`), in fixed point. The float ops
   replay photonmap.cl:167-169,241-249 in the kernel's order, so the values are bit-identical. */
std::vector<long long> colour_table() {
    std::vector<long long> t((size_t)FMGI_COLOUR_STATES * 3, 0);
    for (int sid = 0; sid < FMGI_COLOUR_STATES; sid++) {
        int s = sid & 511;
        if (s == 0) continue;
        f3 c = (sid & 512) ? mkf3(18, 18, 18) : mkf3(16, 16, 18);
        int nb = 0;
        while ((s >> (nb + 1)) != 0) nb++; /* bits below the leading 1 = diffuse bounces */
        for (int b = nb - 1; b >= 0; b--) {
            if ((s >> b) & 1) {
                c.y *= 0.85f;
                c.z *= 0.7f;
            }
            c = mul3(c, 0.9f);
        }
        t[3 * sid + 0] = (long long)ldexp((double)c.x, FMGI_FX_SHIFT);
        t[3 * sid + 1] = (long long)ldexp((double)c.y, FMGI_FX_SHIFT);
        t[3 * sid + 2] = (long long)ldexp((double)c.z, FMGI_FX_SHIFT);
    }
    return t;
}

} // namespace

struct fmgi_context {
    int device = 0;
    int num_cus = 256;
    hipStream_t stream = nullptr;
    RectDev *d_rects = nullptr;
    int nrects = 0;
    SrcDev *d_srcs = nullptr;
    int nsrcs = 0, nwindows = 0, nlights = 0;
    std::vector<fmgi_rect> h_srcs;
    int num_texels = 0;
    std::vector<LaunchDev> h_launches;
    LaunchDev *d_launches = nullptr;
    int64_t d_launch_cap = 0;
    uint64_t total_items = 0;
    uint32_t launch_cap = 0;
    uint64_t *d_src_item_begin = nullptr; /* [nsrc + 1] */
    int32_t *d_src_launch0 = nullptr;     /* [nsrc]     */
    int64_t d_src_cap = 0;
    unsigned long long *d_counter = nullptr;
    unsigned long long *d_stats = nullptr;
    /* ScanFast filter image + non-axis-aligned rect list */
    FilterRec *d_fimg = nullptr;
    int fimg_bytes = 0;
    int32_t *d_general = nullptr;
    int fJ[3] = {0, 0, 0};
    /* ScanGrid tables */
    GridPlane *d_gimg = nullptr;
    int gimg_bytes = 0;
    int gJ[3] = {0, 0, 0};
    GridCell *d_gcells = nullptr;
    GridCellF *d_gcellsF = nullptr;
    bool cells_lds = false;       /* the grid was built coarse to be staged in LDS (closed boxes) */
    char *d_himg = nullptr;       /* ScanHybrid (default instance): the grid's plane image, then the wall pairs */
    int himg_bytes = 0;
    char *d_himg_full = nullptr;  /* ... the floor-plan walk and FMGI_FILTER_PK=0 builds: filter image | plane
                                     image | floor plan | wall pairs */
    int himg_full_bytes = 0;
    int pair_off_full = -1;
    float *d_grecs = nullptr;
    int32_t *d_gidx = nullptr;
    int grid_cells = 0, grid_entries = 0;
    GridBuild h_grid; /* host copy (fmgi_grid_copy) */
    PlanBuild h_plan; /* ScanHybrid's floor plan of the walls (fmgi_plan_copy); h_plan.ok: built */
    std::vector<FilterRec> h_fimg; /* the filter image (fmgi_filter_copy) */
    std::vector<FilterPairHalf> h_pairs; /* the hybrid scan's wall-pair image (fmgi_pairs_copy) */
    int plan_off = -1; /* its byte offset in the full hybrid image */
    int pair_off = -1; /* byte offset of the (default) hybrid image's wall pairs (FilterPairHalf groups) */
    int pG[2] = {0, 0}; /* their groups per axis */
    int auto_kernel = FMGI_KERNEL_FAST;
    /* optional device timing (fmgi_set_timing) */
    bool timing = false;
    std::vector<hipEvent_t> ev_pool;
    std::vector<std::pair<hipEvent_t, hipEvent_t>> ev_bake, ev_fold;
    int ngeneral = 0;
    float margin = 0;
    /* accumulation: FMGI_ACCUM_FX3 or FMGI_ACCUM_STATE (counts[1024][numTexels] + colour table) */
    int accum_req = FMGI_ACCUM_AUTO;
    int accum = FMGI_ACCUM_FX3;
    unsigned long long *d_counts = nullptr;
    long long *d_colfx = nullptr;
    uint32_t *d_colpack = nullptr; /* the same table as u32 {r, g, b, 0} (STREAM fold) */
    /* STREAM: deposit-code stream + fold buffers, grown on demand (fmgi_accum.hip); two sets, so the
       fold of one chunk (on fold_stream) overlaps the bake of the next */
    StreamBufs sb[2]{};
    uint64_t sb_cap_alloc[2] = {0, 0};
    uint64_t sb_entries_alloc[2] = {0, 0};
    hipStream_t fold_stream = nullptr;
    hipEvent_t ev_baked[2] = {nullptr, nullptr}, ev_folded[2] = {nullptr, nullptr};
    /* fetch order (bake_common): per-source item ranges of the plan, scans per item measured on the
       previous bake (device totals -> pinned host copy, ready when ev_cost has completed) */
    std::vector<uint64_t> src_lo, src_hi;
    std::vector<double> src_cost_per_item;
    unsigned long long *d_src_cost = nullptr, *h_src_cost = nullptr;
    int src_cost_n = 0;
    hipEvent_t ev_cost = nullptr;
    bool cost_pending = false;
    uint32_t *d_fetch_tab = nullptr;
    int fetch_tab_cap = 0;
    std::vector<std::vector<uint32_t>> h_fetch_tab; /* the host side of each launch's table, kept for the call */
    std::vector<uint64_t> cost_items;               /* items per source of the measured call */
    /* LDS staging blob of the scans: the scan image, then (optionally) copies of the RectDev and SrcDev
       tables (plan_stage); rebuilt when the scene or the staging choice changes */
    uint64_t scene_gen = 0;
    char *d_blob = nullptr;
    size_t blob_cap = 0;
    uint64_t blob_key = ~0ull;
    std::vector<RectLds> h_rects_lds; /* host staging of the LDS rect copy (kept until the copy is done) */
    bool warned_cells = false;        /* the coarse LDS grid was launched unstaged (said once)          */
    /* the compact closed-box tables (fmgi_internal.h RectC ...; build_compact): set when a closed box's
       RectLds walls and 32-B cells do not fit LDS but these do; the grid is then the one they index */
    /* the launch-tail handoff (bake_common): saved work items (16 B per lane of the saving launch) and
       the counters {idle lanes, states saved, states resumed} */
    uint4 *d_tail = nullptr;
    unsigned *d_tail_ctr = nullptr;
    uint64_t tail_cap = 0;
    std::string last_kernel; /* fmgi_last_bake_kernel: the instance(s) the last bake launch ran */
    int grid_cpr = 0; /* fmgi_set_grid_cells_per_record: the grid's cells per record (0: the product's choice) */
    /* fmgi_set_option: the tests' handles on product paths a given scene would not take (include/flatmatch_gi.h) */
    int64_t opt[FMGI_OPT_COUNT] = {0, 0, 0, -1, -1, -1, 0, 0};
    bool compact = false;
    std::vector<RectC> h_rectc;
    std::vector<ClassC> h_classc;
    std::vector<float> h_recf;     /* {cu, hwu, cv, hwv} by rect index, then the dummy */
    std::vector<uint32_t> h_cellc; /* two u32 per cell: idx0 | idx1 << 16, idx2 | idx3 << 16 */
};

/* the closed-box (one plane per axis and class) instances off: FMGI_OPT_NO_AXES (tests; at fmgi_set_scene) */
static bool no_axes(const fmgi_context *c) { return c->opt[FMGI_OPT_NO_AXES] != 0 || fmgi_exp_env("FMGI_NO_AXES"); }

FMGI_API const char *fmgi_version(void) { return "fmgi 0.1 (gfx950)"; }
FMGI_API const char *fmgi_last_error(void) { return g_err.c_str(); }

FMGI_API int fmgi_device_count(void) {
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess) return 0;
    return n;
}

FMGI_API void fmgi_host_sincosf(const float *x, float *s, float *c, int64_t n) {
    for (int64_t i = 0; i < n; i++) fmgi_sincosf(x[i], &s[i], &c[i]);
}

FMGI_API fmgi_context *fmgi_create(int device) {
    if (device == FMGI_HOST_ONLY) { /* schedule/scene logic only (CPU tests); bakes fail */
        fmgi_context *c = new fmgi_context;
        c->device = FMGI_HOST_ONLY;
        return c;
    }
    int n = fmgi_device_count();
    if (n <= 0) {
        set_err(FMGI_ERR_NO_DEVICE, "no HIP device visible");
        return nullptr;
    }
    if (device < 0 || device >= n) {
        set_err(FMGI_ERR_ARG, "device %d out of range (%d visible)", device, n);
        return nullptr;
    }
    if (hipSetDevice(device) != hipSuccess) {
        set_err(FMGI_ERR_HIP, "hipSetDevice(%d) failed", device);
        return nullptr;
    }
    fmgi_context *c = new fmgi_context;
    c->device = device;
    hipDeviceProp_t prop;
    if (hipGetDeviceProperties(&prop, device) == hipSuccess && prop.multiProcessorCount > 0)
        c->num_cus = prop.multiProcessorCount;
    if (hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking) != hipSuccess ||
        hipMalloc(&c->d_counter, 64) != hipSuccess ||
        hipMalloc(&c->d_stats, KSTAT_ALLOC * sizeof(unsigned long long)) != hipSuccess ||
        hipMemset(c->d_stats, 0, KSTAT_ALLOC * sizeof(unsigned long long)) != hipSuccess) {
        set_err(FMGI_ERR_HIP, "context allocation failed on device %d", device);
        fmgi_destroy(c);
        return nullptr;
    }
    return c;
}

FMGI_API void fmgi_destroy(fmgi_context *c) {
    if (!c) return;
    if (c->device == FMGI_HOST_ONLY) {
        delete c;
        return;
    }
    hipSetDevice(c->device);
    if (c->stream) hipStreamSynchronize(c->stream);
    hipFree(c->d_rects);
    hipFree(c->d_srcs);
    hipFree(c->d_launches);
    hipFree(c->d_fimg);
    hipFree(c->d_general);
    hipFree(c->d_gimg);
    hipFree(c->d_gcells);
    hipFree(c->d_gcellsF);
    hipFree(c->d_himg);
    hipFree(c->d_himg_full);
    hipFree(c->d_blob);
    hipFree(c->d_tail);
    hipFree(c->d_tail_ctr);
    hipFree(c->d_grecs);
    hipFree(c->d_gidx);
    for (hipEvent_t ev : c->ev_pool) hipEventDestroy(ev);
    for (auto &p : c->ev_bake) { hipEventDestroy(p.first); hipEventDestroy(p.second); }
    for (auto &p : c->ev_fold) { hipEventDestroy(p.first); hipEventDestroy(p.second); }
    hipFree(c->d_src_item_begin);
    hipFree(c->d_src_launch0);
    if (c->ev_cost) { hipEventSynchronize(c->ev_cost); hipEventDestroy(c->ev_cost); }
    hipFree(c->d_src_cost);
    if (c->h_src_cost) hipHostFree(c->h_src_cost);
    hipFree(c->d_fetch_tab);
    hipFree(c->d_counts);
    hipFree(c->d_colfx);
    if (c->fold_stream) hipStreamSynchronize(c->fold_stream);
    for (int k = 0; k < 2; k++) {
        hipFree(c->sb[k].stream);
        hipFree(c->sb[k].sorted);
        hipFree(c->sb[k].cursor);
        hipFree(c->sb[k].toff);
        hipFree(c->sb[k].tile_blocks);
        if (c->ev_baked[k]) hipEventDestroy(c->ev_baked[k]);
        if (c->ev_folded[k]) hipEventDestroy(c->ev_folded[k]);
    }
    if (c->fold_stream) hipStreamDestroy(c->fold_stream);
    hipFree(c->d_colpack);
    hipFree(c->d_counter);
    hipFree(c->d_stats);
    if (c->stream) hipStreamDestroy(c->stream);
    delete c;
}

/* AccState needs 8 KiB of u64 counters per texel; above this budget (or on request) AccFx3 is used. */
static const size_t kStateBudget = (size_t)8 << 30;

static const int kStreamMaxTexels = FMGI_MAX_TILES << FMGI_TILE_BITS; /* 4,194,304; also keeps codes != ~0u */

static int ensure_colour_table(fmgi_context *c) {
    if (c->d_colfx) return FMGI_OK;
    std::vector<long long> t = colour_table();
    /* the STREAM fold's table: {R, G - R, B - R} per state (differences as two's complement 32-bit), so
       a grey deposit (R = G = B: a window's photon before any floor bounce) is one LDS add */
    std::vector<uint32_t> p((size_t)FMGI_COLOUR_STATES * 4, 0u);
    for (int sid = 0; sid < FMGI_COLOUR_STATES; sid++) {
        for (int k = 0; k < 3; k++) {
            const long long v = t[3 * sid + k]; /* <= 18 * 2^25 < 2^30 */
            if (v < 0 || v >= (1ll << 30)) return set_err(FMGI_ERR_STATE, "colour table overflow");
        }
        const long long r = t[3 * sid];
        p[4 * sid + 0] = (uint32_t)r;
        p[4 * sid + 1] = (uint32_t)(int32_t)(t[3 * sid + 1] - r);
        p[4 * sid + 2] = (uint32_t)(int32_t)(t[3 * sid + 2] - r);
    }
    HIPCHK(hipMalloc(&c->d_colfx, t.size() * sizeof(long long)));
    HIPCHK(hipMemcpy(c->d_colfx, t.data(), t.size() * sizeof(long long), hipMemcpyHostToDevice));
    HIPCHK(hipMalloc(&c->d_colpack, p.size() * sizeof(uint32_t)));
    HIPCHK(hipMemcpy(c->d_colpack, p.data(), p.size() * sizeof(uint32_t), hipMemcpyHostToDevice));
    return FMGI_OK;
}

static int configure_accum(fmgi_context *c) {
    size_t bytes = (size_t)FMGI_COLOUR_STATES * (size_t)c->num_texels * sizeof(unsigned long long);
    int want = c->accum_req;
    if (want == FMGI_ACCUM_AUTO)
        want = (c->num_texels > 0 && c->num_texels < kStreamMaxTexels) ? FMGI_ACCUM_STREAM : FMGI_ACCUM_FX3;
    if (want == FMGI_ACCUM_STREAM && c->num_texels >= kStreamMaxTexels) want = FMGI_ACCUM_FX3;
    hipFree(c->d_counts);
    c->d_counts = nullptr;
    c->accum = want == FMGI_ACCUM_NONE ? FMGI_ACCUM_NONE : FMGI_ACCUM_FX3;
    HIPCHK(hipSetDevice(c->device));
    if (want == FMGI_ACCUM_STREAM) {
        int rc = ensure_colour_table(c);
        if (rc != FMGI_OK) return rc;
        c->accum = FMGI_ACCUM_STREAM;
        return FMGI_OK;
    }
    if (want != FMGI_ACCUM_STATE || !bytes) return FMGI_OK;
    HIPCHK(hipMalloc(&c->d_counts, bytes));
    HIPCHK(hipMemset(c->d_counts, 0, bytes));
    int rc = ensure_colour_table(c);
    if (rc != FMGI_OK) return rc;
    c->accum = FMGI_ACCUM_STATE;
    return FMGI_OK;
}

/* STREAM buffers for a bake of `items` work items on `grid` blocks of `block` lanes: every item makes at
   most 800 deposits and every wave wastes at most one partly filled block. */
static uint64_t stream_cap_for(uint64_t items, int grid, int block) {
    const uint64_t waves = (uint64_t)grid * (uint64_t)(block / 64);
    return items * FMGI_EVENTS_PER_ITEM + (waves + 1) * FMGI_STREAM_BLOCK;
}

/* STREAM layouts (BakeArgs::presort): 0 = unsorted codes, folded through k_slice_sort's sorted copy;
   1 = ring-sized segments presorted by tile; 2 = per-wave tile buckets (bucket_out / k_bucket_fold) */
enum { kStreamSliced = 0, kStreamSegments = 1, kStreamBuckets = 2, kStreamDense = 3 };

/* the dense stream of a chunk (kStreamDense): one code or sentinel per lane and loop iteration. An item
   scans at most 900 times (8 deposits and one escape per photon); a lane idles (sentinels) at most while
   the other lanes of its wave finish an item each; plus each wave's last partly written block */
static uint64_t dense_cap_for(uint64_t items, int grid, int block) {
    const uint64_t waves = (uint64_t)grid * (uint64_t)(block / 64);
    const uint64_t cap = items * (FMGI_EVENTS_PER_ITEM + FMGI_PHOTONS_PER_ITEM) +
                         waves * (64ull * (FMGI_EVENTS_PER_ITEM + FMGI_PHOTONS_PER_ITEM) + 2 * FMGI_STREAM_BLOCK);
    /* a whole number of blocks: k_bin reads min(cursor, cap) codes in whole 512-code wave batches, so an
       overflowed stream still ends on a block boundary inside the buffer */
    return (cap + FMGI_STREAM_BLOCK - 1) / FMGI_STREAM_BLOCK * FMGI_STREAM_BLOCK;
}

/* the bucketed stream's pool, in blocks: every code of the chunk, plus one partly filled bucket per wave
   and tile */
/* pool blocks for `cap` codes: the codes, the sentinel pads (<= 3 per tile and ring flush: a flush per
   FMGI_RING_CODES codes plus each wave's last), one partly filled block per wave and tile, and the
   blocks a wave holds reserved (< FMGI_BUCKET_ALLOC) */
static uint64_t bucket_pool_blocks(uint64_t cap, int P, int grid, int block) {
    const uint64_t waves = (uint64_t)grid * (uint64_t)(block / 64);
    const uint64_t pads = (cap / FMGI_RING_CODES + waves) * 3u * (uint64_t)P;
    return (cap + pads + FMGI_BUCKET_BLOCK - 1) / FMGI_BUCKET_BLOCK + waves * (uint64_t)(P + FMGI_BUCKET_ALLOC) + 8;
}
static uint64_t stream_alloc_codes(uint64_t cap, int P, int grid, int block, int mode) {
    return mode >= kStreamBuckets ? bucket_pool_blocks(cap, P, grid, block) * FMGI_BUCKET_BLOCK : cap;
}

/* fold tiles of 2^bits texels over the lightmap */
static int tiles_of(const fmgi_context *c, int bits) { return (c->num_texels + (1 << bits) - 1) >> bits; }

/* The fold tile of a STREAM chunk: 2048 texels (FMGI_TILE_BITS), or 4096 (FMGI_WIDE_TILE_BITS) in the bucket
   layouts when the chunk is large. Wide tiles halve the tiles, so each wave-iteration's deposit stores touch
   ~22 instead of ~34 lines (box200 bake 65.7 -> 60.8 ms), while the fold's 96-KB accumulators run one
   workgroup per CU (fold +1.2 ms whatever the chunk: example.png's 1e8 photons lose overall, 22.6 -> 23.2 ms;
   profiles/r05/s16). So: wide from 3e6 work items (3e8 photons) per chunk. FMGI_WIDE_TILES=0/1 forces. */
static int tile_bits(const fmgi_context *c, int mode, uint64_t items) {
    if (mode < kStreamBuckets) return FMGI_TILE_BITS;
    if (c->opt[FMGI_OPT_WIDE_TILES] >= 0) return c->opt[FMGI_OPT_WIDE_TILES] ? FMGI_WIDE_TILE_BITS : FMGI_TILE_BITS;
    if (const char *we = fmgi_exp_env("FMGI_WIDE_TILES")) { /* experiments: 0 / 1 (= 12) or the tile bits, 11-13 */
        const int v = atoi(we);
        return v == 1 ? FMGI_WIDE_TILE_BITS : (v >= 11 && v <= 13 ? v : FMGI_TILE_BITS);
    }
    return items >= 3000000 ? FMGI_WIDE_TILE_BITS : FMGI_TILE_BITS;
}

static bool ensure_stream_needs_growth(const fmgi_context *c, int k, uint64_t items, int grid, int block, int mode) {
    const int P = tiles_of(c, FMGI_TILE_BITS);
    return stream_alloc_codes(stream_cap_for(items, grid, block), P, grid, block, mode) > c->sb_cap_alloc[k] ||
           (mode == kStreamSliced && !c->sb[k].sorted) ||
           (mode == kStreamDense && dense_cap_for(items, grid, block) > c->sb[k].dense_alloc);
}

static int ensure_stream(fmgi_context *c, int k, uint64_t items, int grid, int block, int mode, int tbits) {
    StreamBufs &sb = c->sb[k];
    const uint64_t cap = stream_cap_for(items, grid, block);
    /* (the pool is sized for the narrow tiles' open blocks: enough for either) */
    const int P = tiles_of(c, FMGI_TILE_BITS);
    sb.tile_bits = tbits;
    const uint64_t codes = stream_alloc_codes(cap, P, grid, block, mode);
    if (codes > c->sb_cap_alloc[k] || (mode == kStreamSliced && !sb.sorted)) {
        hipFree(sb.stream);
        hipFree(sb.sorted);
        sb.stream = sb.sorted = nullptr;
        c->sb_cap_alloc[k] = 0;
        HIPCHK(hipMalloc(&sb.stream, codes * sizeof(uint32_t)));
        if (mode == kStreamSliced) HIPCHK(hipMalloc(&sb.sorted, codes * sizeof(uint32_t))); /* the sorted copy */
        c->sb_cap_alloc[k] = codes;
    }
    sb.presort = mode;
    sb.dense_cap = 0;
    if (mode == kStreamDense) { /* the bake's dense stream beside the pool k_bin fills */
        const uint64_t dcap = dense_cap_for(items, grid, block);
        if (dcap > sb.dense_alloc) {
            hipFree(sb.dense);
            sb.dense = nullptr;
            sb.dense_alloc = 0;
            HIPCHK(hipMalloc(&sb.dense, dcap * sizeof(uint32_t)));
            sb.dense_alloc = dcap;
        }
        sb.dense_cap = dcap;
        sb.bin_grid = 2 * std::max(1, c->num_cus);
    }
    /* run tables: per 8192-code slice (sorted by k_slice_sort), or per ring-sized segment (presorted); the
       bucketed stream's per-block tile, length and list instead */
    uint64_t entries = 0;
    if (mode >= kStreamBuckets) {
        sb.pool_blocks = bucket_pool_blocks(cap, P, grid, block);
        /* FMGI_OPT_POOL_LIMIT = n (tests): at most n pool blocks, so the bake runs out of them and takes the
           exact atomic fallback (bucket_atomic) for the rest of its codes */
        if (c->opt[FMGI_OPT_POOL_LIMIT] > 0)
            sb.pool_blocks = std::min<uint64_t>(sb.pool_blocks, (uint64_t)c->opt[FMGI_OPT_POOL_LIMIT]);
        entries = 3 * sb.pool_blocks * 2; /* three u32 arrays, in u16 units */
        if (!sb.tile_blocks) HIPCHK(hipMalloc(&sb.tile_blocks, 2 * (FMGI_PRESORT_MAX_TILES + 1) * sizeof(uint32_t)));
    } else {
        const uint64_t nslices = mode == kStreamSegments ? (cap + FMGI_RING_CODES - 1) / FMGI_RING_CODES
                                                         : (cap + FMGI_STREAM_SLICE - 1) / FMGI_STREAM_SLICE;
        entries = (uint64_t)(P + 1) * nslices;
    }
    if (entries > c->sb_entries_alloc[k]) {
        hipFree(sb.toff);
        sb.toff = nullptr;
        c->sb_entries_alloc[k] = 0;
        HIPCHK(hipMalloc(&sb.toff, entries * sizeof(uint16_t)));
        c->sb_entries_alloc[k] = entries;
    }
    sb.block_tile = mode >= kStreamBuckets ? (uint32_t *)sb.toff : nullptr;
    sb.block_len = mode >= kStreamBuckets ? sb.block_tile + sb.pool_blocks : nullptr;
    sb.block_list = mode >= kStreamBuckets ? sb.block_len + sb.pool_blocks : nullptr;
    if (!sb.cursor) HIPCHK(hipMalloc(&sb.cursor, 64));
    sb.cap = cap;
    sb.colpack = c->d_colpack;
    /* the fold kernels run two 64-KiB workgroups per CU and tiles carry uneven code counts: ~8 (slice-
       sorted) or ~16 (presorted, chained) rounds of P x groups workgroups balance the tail (box200, 46
       tiles, presorted: 19.6 / 18.9 / 17.4 / 16.5 ms at 11 / 22 / 45 / 90 groups) */
    {
        const int ncu = std::max(1, c->num_cus);
        const int Pf = tiles_of(c, mode >= kStreamBuckets ? tbits : FMGI_TILE_BITS); /* the fold's tiles */
        const char *ge = fmgi_exp_env("FMGI_FOLD_GROUPS"); /* experiments */
        /* bucketed: ~36 rounds (box200, 46 tiles: fold 11.22 / 10.86 / 10.92 / 11.19 / 12.70 ms at 96 / 200 /
           300 / 800 / 1600 groups, profiles/r03/s21-s22: finer shares of the largest tiles against the
           per-workgroup set-up and flush) */
        /* slice-sorted (lightmaps of more than 63 tiles): ~48 rounds (30-room layout, 358 tiles: fold 7.49 /
           7.31 / 6.34 / 5.97 ms at 8 / 4 / 16 / 32 groups per tile, profiles/r03/s33) */
        /* (wide bucket tiles: one 96-KB fold workgroup per CU instead of two, so half the rounds; box200 fold
           11.93 / 11.58 / 11.91 ms at ~408 / 200 / 300 groups per tile, profiles/r05/s26-s27) */
        /* (wide tiles, round 6: the balanced share gives every workgroup the same blocks, so a round of them
           ends together and a partly filled last round idles CUs; the groups per tile are rounded DOWN to the
           launch's multiple of 8 so the workgroups fill just under 13 rounds: box200 (23 tiles, 144 groups,
           12.94 rounds) 11.50 -> 11.30 ms, box2000 (26 tiles, 128 groups, 13.0 rounds) 11.57 -> 11.24 ms;
           12.2, 13.7 or 14.4 rounds took 11.45-11.70 ms, profiles/r06/s24-s25) */
        /* (narrow bucket tiles, round 6: only launches of < 3e6 items use them now, whose streams are small; the
           per-workgroup set-up and 2048-texel flush then dominate, and 7 whole rounds of the two workgroups per
           CU beat the 18 the round-3 box200 count gave: example.png fold 1.35 -> 0.85 ms (56 tiles, 64 groups;
           0.86-0.96 ms at 16-48 groups, 1.06 at 128, 1.55 at 192; profiles/r06/s27-s28) */
        const bool wide = mode >= kStreamBuckets && tbits > FMGI_TILE_BITS && fmgi_fold_split(tbits) == 1;
        const bool buckets = mode >= kStreamBuckets && fmgi_fold_split(tbits) == 1;
        const int rounds = mode >= kStreamBuckets ? (wide ? 13 : 14) : (mode == kStreamSegments ? 16 : 48);
        /* (a split bucket tile gets `split` workgroups per group: the same rounds over the fold tiles) */
        const int split = mode >= kStreamBuckets ? fmgi_fold_split(tbits) : 1;
        sb.groups = (ge && atoi(ge) > 0) ? atoi(ge)
                    : buckets ? std::max(8, (rounds * ncu / (Pf * split)) & ~7)
                              : std::max(1, (rounds * ncu + Pf * split - 1) / (Pf * split));
        /* a small stream (config 1: ~8,600 segments at most) would leave most of those workgroups' waves
           without work, and each pays its LDS set-up and tile flush: at least 1024 segments (64 per wave),
           or 16 chain blocks (one per wave), per workgroup */
        if (!(ge && atoi(ge) > 0)) {
            if (mode == kStreamSegments)
                sb.groups = (int)std::min<uint64_t>((uint64_t)sb.groups, std::max<uint64_t>(8, cap / FMGI_RING_CODES / 1024));
            if (mode >= kStreamBuckets) /* at least one 4-KB block per wave of every workgroup */
                sb.groups = (int)std::min<uint64_t>((uint64_t)sb.groups,
                                                    std::max<uint64_t>(8, (cap / FMGI_BUCKET_BLOCK) / ((uint64_t)Pf * 16)));
            if (mode == kStreamSliced) /* at least one big slice's worth of codes per workgroup and tile */
                sb.groups = (int)std::min<uint64_t>((uint64_t)sb.groups,
                                                    std::max<uint64_t>(8, cap / ((uint64_t)P * FMGI_STREAM_SLICE_BIG)));
        }
        const char *be = fmgi_exp_env("FMGI_FOLD_BLOCK"); /* experiments: 256, 512 or 1024 */
        sb.block = (be && (atoi(be) == 256 || atoi(be) == 512 || atoi(be) == 1024)) ? atoi(be) : 1024;
    }
    return FMGI_OK;
}

/* frees the STREAM buffers (codes, slice-sorted copy, run tables); the next bake allocates them again */
static void release_stream_buffers(fmgi_context *c) {
    if (!c || c->device == FMGI_HOST_ONLY || hipSetDevice(c->device) != hipSuccess) return;
    (void)hipStreamSynchronize(c->stream);
    if (c->fold_stream) (void)hipStreamSynchronize(c->fold_stream);
    for (int k = 0; k < 2; k++) {
        (void)hipFree(c->sb[k].stream);
        (void)hipFree(c->sb[k].sorted);
        (void)hipFree(c->sb[k].toff);
        (void)hipFree(c->sb[k].dense);
        c->sb[k].dense = nullptr;
        c->sb[k].dense_alloc = 0;
        c->sb[k].stream = c->sb[k].sorted = nullptr;
        c->sb[k].toff = nullptr;
        c->sb_cap_alloc[k] = 0;
        c->sb_entries_alloc[k] = 0;
    }
}

FMGI_API int fmgi_set_accumulation(fmgi_context *c, int mode) {
    if (!c || mode < FMGI_ACCUM_AUTO || mode > FMGI_ACCUM_STREAM) return set_err(FMGI_ERR_ARG, "bad accumulation mode");
    c->accum_req = mode;
    if (c->device == FMGI_HOST_ONLY || c->num_texels == 0) return FMGI_OK;
    return configure_accum(c);
}

FMGI_API int fmgi_get_accumulation(fmgi_context *c) { return c ? c->accum : set_err(FMGI_ERR_ARG, "null context"); }

/* workgroup size of the bake (FMGI_BLOCK: experiments, 64..1024 lanes) */
static int bake_block() {
    int block = 256;
    if (const char *be = fmgi_exp_env("FMGI_BLOCK"))
        if (atoi(be) >= 64 && atoi(be) <= 1024 && atoi(be) % 64 == 0) block = atoi(be);
    return block;
}

/* dynamic LDS a bake launch may use without raising the kernel's limit: the scan image staged in LDS
   (FAST: 64 B per record pair, GRID: 128 B per plane pair) plus the per-wave code rings must fit, or the
   launch fails; a scene whose image does not fit runs a kernel whose image does, or the exact scan (no
   image, identical results) */
static const size_t kBakeLdsLimit = 65536;
/* ... and with the limit raised (fmgi_launch_bake sets the kernel attribute): what staging may use */
static const size_t kBakeLdsMax = 160 * 1024;

/* whether a hybrid bake reads the full image (the floor-plan walk, FMGI_PLAN=1, or the one-record wall loop
   of FMGI_FILTER_PK=0 builds) rather than the default one (plane image + wall pairs only) */
static bool hybrid_full(const fmgi_context *c) {
    const char *pe = fmgi_exp_env("FMGI_PLAN"), *fe = fmgi_exp_env("FMGI_HYB_FULL"); /* FMGI_HYB_FULL=1: A/B of the image */
    return !fmgi_kernels_filter_pk() || (c->plan_off >= 0 && pe && atoi(pe) == 1) || (fe && atoi(fe) == 1);
}

static int image_bytes(const fmgi_context *c, int kernel) {
    if (kernel == FMGI_KERNEL_HYBRID) return hybrid_full(c) ? c->himg_full_bytes : c->himg_bytes;
    return kernel == FMGI_KERNEL_GRID ? c->gimg_bytes : c->fimg_bytes;
}

static bool kernel_fits(const fmgi_context *c, int kernel, int accum, int block) {
    if (kernel == FMGI_KERNEL_EXACT) return true;
    const int img = image_bytes(c, kernel);
    return fmgi_bake_lds(kernel, accum, block, img, nullptr) <= kBakeLdsLimit;
}

static int fitting_kernel(const fmgi_context *c, int kernel, int accum, int block) {
    if (kernel_fits(c, kernel, accum, block)) return kernel;
    if (kernel == FMGI_KERNEL_HYBRID) kernel = FMGI_KERNEL_FAST;
    if (kernel_fits(c, kernel, accum, block)) return kernel;
    const int other = kernel == FMGI_KERNEL_GRID ? FMGI_KERNEL_FAST : FMGI_KERNEL_GRID;
    if (kernel != FMGI_KERNEL_EXACT && kernel_fits(c, other, accum, block)) return other;
    return FMGI_KERNEL_EXACT;
}

/* LDS a compact closed-box launch holds (one 1024-lane workgroup per CU): the scan image, the emitters, and the
   compact tables, beside the lane-by-lane stores' tile words of its 16 waves */
static size_t compact_bytes(int img_bytes, int nsrcs, size_t nclass, size_t nrects, size_t ncells) {
    size_t off = ((size_t)img_bytes + 15) & ~(size_t)15;
    off += (size_t)nsrcs * sizeof(SrcDev);
    off += nclass * sizeof(ClassC);
    off += (nrects * sizeof(RectC) + 15) & ~(size_t)15;
    off += (nrects + 1) * 16;
    off += ncells * 8;
    return (off + 15) & ~(size_t)15;
}
static const size_t kCompactLds = 160 * 1024 - 16 * FMGI_SCATTER_STRIDE * 4;

/* The compact tables of a closed box (ScanGridT's Compact instance) from the device-computed RectDev table, the
   filter records and grid g: false if some limit does not hold (a cell of more than 4 records, 2^16 walls,
   texel bases of 22 bits, 1024 classes, W or H of 16 bits) or a field does not round-trip bit for bit. */
static bool build_compact(fmgi_context *c, const std::vector<RectDev> &rd, const FilterBuild &fb, const GridBuild &g) {
    const size_t n = rd.size();
    if (n == 0 || n >= 0xFFFF || !fb.general.empty()) return false;
    std::vector<ClassC> cls;
    std::map<std::vector<uint32_t>, uint32_t> key_of;
    std::vector<RectC> rc(n);
    auto bits = [](float x) { uint32_t b; memcpy(&b, &x, 4); return b; };
    for (size_t i = 0; i < n; i++) {
        const RectDev &r = rd[i];
        if (r.base < 0 || r.base >= (1 << kCompactBaseBits) || r.W < 1 || r.W > 0xFFFF || r.H < 1 || r.H > 0xFFFF)
            return false;
        ClassC k;
        memset(&k, 0, sizeof k);
        k.nx = r.nx; k.ny = r.ny; k.nz = r.nz;
        k.wnx = r.wnx; k.wny = r.wny; k.wnz = r.wnz;
        k.hnx = r.hnx; k.hny = r.hny; k.hnz = r.hnz;
        k.bux = r.bux; k.buy = r.buy; k.buz = r.buz;
        k.bvx = r.bvx; k.bvy = r.bvy; k.bvz = r.bvz;
        k.WH = r.W | (r.H << 16);
        std::vector<uint32_t> key((const uint32_t *)&k, (const uint32_t *)&k + 16);
        auto it = key_of.find(key);
        uint32_t id;
        if (it == key_of.end()) {
            id = (uint32_t)cls.size();
            if (id >= (uint32_t)kCompactMaxClasses) return false;
            key_of.emplace(key, id);
            cls.push_back(k);
        } else {
            id = it->second;
        }
        rc[i] = RectC{r.px, r.py, r.pz, r.wl, r.hl, (uint32_t)r.base | (id << kCompactBaseBits)};
        /* the decode the kernel does (exact_hit_compact), compared bit for bit */
        const ClassC &q = cls[rc[i].meta >> kCompactBaseBits];
        const float got[] = {rc[i].px, rc[i].py, rc[i].pz, q.nx, q.ny, q.nz, q.wnx, q.wny, q.wnz, rc[i].wl, q.hnx, q.hny,
                             q.hnz, rc[i].hl, q.bux, q.buy, q.buz, q.bvx, q.bvy, q.bvz};
        const float want[] = {r.px, r.py, r.pz, r.nx, r.ny, r.nz, r.wnx, r.wny, r.wnz, r.wl, r.hnx, r.hny,
                              r.hnz, r.hl, r.bux, r.buy, r.buz, r.bvx, r.bvy, r.bvz};
        for (int f = 0; f < 20; f++)
            if (bits(got[f]) != bits(want[f])) return false;
        if ((int)(rc[i].meta & ((1u << kCompactBaseBits) - 1)) != r.base || (q.WH & 0xFFFF) != r.W ||
            ((uint32_t)q.WH >> 16) != (uint32_t)r.H)
            return false;
    }
    /* filter extents by rect index: every wall is a record of exactly one class list (no general rects) */
    std::vector<float> recf((n + 1) * 4, 0.0f);
    std::vector<char> seen(n, 0);
    for (int a = 0; a < 3; a++)
        for (int cl = 0; cl < 2; cl++)
            for (const FilterRec &r : fb.cls[a][cl]) {
                if (r.idx < 0 || (size_t)r.idx >= n || seen[(size_t)r.idx]) return false;
                seen[(size_t)r.idx] = 1;
                float *q = &recf[(size_t)r.idx * 4];
                q[0] = r.cu; q[1] = r.hwu; q[2] = r.cv; q[3] = r.hwv;
            }
    for (size_t i = 0; i < n; i++)
        if (!seen[i]) return false;
    recf[n * 4 + 1] = -1.0f; /* the dummy: |x - 0| <= -1 never holds */
    recf[n * 4 + 3] = -1.0f;
    /* cells: up to four rect indices (inline two, then the overflow list), absent = the dummy */
    const uint32_t D = (uint32_t)n;
    std::vector<uint32_t> cellc(g.cells.size() * 2);
    for (size_t ci = 0; ci < g.cells.size(); ci++) {
        const GridCell &gc = g.cells[ci];
        if (gc.count < 0 || gc.count > 4) return false;
        uint32_t id[4] = {D, D, D, D};
        for (int k = 0; k < gc.count; k++) {
            const int32_t x = k == 0 ? gc.idx0 : k == 1 ? gc.idx1 : g.idx[(size_t)gc.rest + (size_t)k - 2];
            if (x < 0 || (size_t)x >= n) return false;
            id[k] = (uint32_t)x;
        }
        cellc[2 * ci] = id[0] | (id[1] << 16);
        cellc[2 * ci + 1] = id[2] | (id[3] << 16);
    }
    if (compact_bytes((int)(g.img.size() * sizeof(GridPlane)), c->nsrcs, cls.size(), n, g.cells.size()) > kCompactLds)
        return false;
    c->h_rectc.swap(rc);
    c->h_classc.swap(cls);
    c->h_recf.swap(recf);
    c->h_cellc.swap(cellc);
    return true;
}

FMGI_API int fmgi_set_scene(fmgi_context *c, const fmgi_rect *walls, int num_walls, const fmgi_rect *windows,
                            int num_windows, const fmgi_rect *lights, int num_lights, int num_texels) {
    if (!c || num_walls < 0 || num_windows < 0 || num_lights < 0 || num_texels < 0 ||
        (num_walls && !walls) || (num_windows && !windows) || (num_lights && !lights))
        return set_err(FMGI_ERR_ARG, "fmgi_set_scene: bad arguments");
    /* every texel index a deposit can produce must be inside the texel buffer */
    for (int i = 0; i < num_walls; i++) {
        const int32_t *lm = walls[i].lightmapSetup;
        if (lm[1] < 1 || lm[2] < 1 || lm[0] < 0 || (int64_t)lm[0] + (int64_t)lm[1] * lm[2] > num_texels)
            return set_err(FMGI_ERR_ARG, "wall %d: lightmapSetup {%d,%d,%d} outside %d texels", i, lm[0], lm[1],
                           lm[2], num_texels);
    }
    std::vector<RectDev> rd((size_t)num_walls);
    for (int i = 0; i < num_walls; i++) rd[i] = make_rect(walls[i]);
    std::vector<SrcDev> sd;
    c->h_srcs.clear();
    for (int i = 0; i < num_windows; i++) { sd.push_back(make_src(windows[i])); c->h_srcs.push_back(windows[i]); }
    for (int i = 0; i < num_lights; i++) { sd.push_back(make_src(lights[i])); c->h_srcs.push_back(lights[i]); }
    FilterBuild fb = build_filter(walls, num_walls, c->h_srcs.data(), (int)c->h_srcs.size());
    for (int a = 0; a < 3; a++) c->fJ[a] = fb.J[a];
    c->fimg_bytes = (int)(fb.img.size() * sizeof(FilterRec));
    c->h_fimg = fb.img;
    c->ngeneral = (int)fb.general.size();
    c->margin = fb.margin;
    const int cpr_forced = c->grid_cpr > 0 ? c->grid_cpr : grid_cpr_env();
    GridBuild gb = build_grid(fb, cpr_forced ? cpr_forced : 16);
    /* closed boxes (one plane per class on each axis, the closed-box instance): the coarsest grid of 5 or 4
       cells per record whose cells fit in 32 KB, staged in LDS beside the rings (plan_stage) when that
       keeps the wave count: every cell lookup an LDS read. box200: 951 cells of 32 B, bake 77.4 -> 74.9 ms
       (~2 record tests per scan instead of ~1.5, profiles/r04/s23). FMGI_CELLS_LDS=0 keeps the
       16-per-record grid in global memory. */
    c->cells_lds = false;
    {
        const char *cl = fmgi_exp_env("FMGI_CELLS_LDS");
        if (!cpr_forced && !(cl && atoi(cl) == 0) && gb.J[0] == 1 && gb.J[1] == 1 && gb.J[2] == 1 &&
            !no_axes(c)) {
            for (int cpr : {5, 4}) {
                GridBuild g = build_grid(fb, cpr);
                if (g.cells.size() * sizeof(GridCell) <= 32768) {
                    gb = g;
                    c->cells_lds = true;
                    break;
                }
            }
        }
    }
    /* closed boxes whose coarse cells do not fit either (BASELINE config 5): the finest grid of 4, 3 or 2 cells per
       record with at most 4 records per cell whose compact tables fit (build_compact, after the device has
       computed the walls' builtin-derived fields); FMGI_COMPACT=0 keeps the 16-per-record global grid */
    GridBuild gcomp;
    bool try_compact = false;
    {
        const char *ce = fmgi_exp_env("FMGI_COMPACT");
        if (c->device != FMGI_HOST_ONLY && !c->cells_lds && !cpr_forced && !(ce && atoi(ce) == 0) &&
            gb.J[0] == 1 && gb.J[1] == 1 && gb.J[2] == 1 && !no_axes(c) && fb.general.empty() &&
            num_walls > 0 && num_walls < 0xFFFF) {
            for (int cpr : {4, 3, 2}) {
                GridBuild g = build_grid(fb, cpr);
                bool ok = true;
                for (const GridCell &gc : g.cells) ok = ok && gc.count <= 4;
                /* (classes are at most a few per plane on a box; build_compact checks the real size) */
                if (ok && compact_bytes((int)(g.img.size() * sizeof(GridPlane)), num_windows + num_lights, 64,
                                        (size_t)num_walls, g.cells.size()) <= kCompactLds) {
                    gcomp = g;
                    try_compact = true;
                    break;
                }
            }
        }
    }
    c->compact = false;
    for (int a = 0; a < 3; a++) c->gJ[a] = gb.J[a];
    c->gimg_bytes = (int)(gb.img.size() * sizeof(GridPlane));
    c->grid_cells = (int)gb.cells.size();
    c->grid_entries = (int)gb.idx.size();
    c->h_grid = gb;
    /* ScanHybrid's image is the filter image followed by the plane image and the floor plan: its size must
       be this scene's before the AUTO choice below asks which images fit LDS (also in host-only contexts) */
    c->h_plan = build_plan(fb, c->h_srcs.data(), (int)c->h_srcs.size());
    const std::vector<char> plan_blob = c->h_plan.ok ? c->h_plan.blob() : std::vector<char>();
    c->plan_off = c->h_plan.ok ? c->fimg_bytes + c->gimg_bytes : -1;
    const std::vector<FilterPairHalf> pairs_img = build_filter_pairs(fb, c->pG);
    c->h_pairs = pairs_img;
    const int pairs_bytes = (int)(pairs_img.size() * sizeof(FilterPairHalf));
    c->pair_off_full = (c->fimg_bytes + c->gimg_bytes + (int)plan_blob.size() + 15) & ~15;
    c->himg_full_bytes = c->pair_off_full + pairs_bytes;
    if (const char *pe = fmgi_exp_env("FMGI_PAIRS")) /* experiments: 0 = no pair image (honoured by FMGI_FILTER_PK=0 builds) */
        if (atoi(pe) == 0 && !fmgi_kernels_filter_pk()) c->himg_full_bytes = c->fimg_bytes + c->gimg_bytes + (int)plan_blob.size();
    /* the default instance stages only what it reads: the plane image (a multiple of 64 B) and the pairs */
    c->pair_off = c->gimg_bytes;
    c->himg_bytes = c->pair_off + pairs_bytes;
    {   /* AUTO: phase-1 work per scan ~ 60 VALU per grid plane slot vs ~15 per filter pair (measured on
           the example layout and the synthetic boxes: GRID 1.3-11x faster on boxes, 0.6x on example) */
        const int slots = gb.J[0] + gb.J[1] + gb.J[2], pairs = fb.J[0] + fb.J[1] + fb.J[2];
        c->auto_kernel = (4 * slots < pairs) ? FMGI_KERNEL_GRID : FMGI_KERNEL_FAST;
        /* layouts: floors and ceilings through the grid, walls through the filter (example.png: 3.80e9
           vs 3.65e9 photons/s FAST, 3.02e9 GRID) when the floor/ceiling records share few planes */
        if (c->auto_kernel == FMGI_KERNEL_FAST && 4 * gb.J[2] < fb.J[2]) c->auto_kernel = FMGI_KERNEL_HYBRID;
        /* the largest LDS use (STREAM rings) decides, so the choice holds for every accumulation mode */
        c->auto_kernel = fitting_kernel(c, c->auto_kernel, FMGI_ACCUM_STREAM, bake_block());
    }
    if (c->device != FMGI_HOST_ONLY) {
    HIPCHK(hipSetDevice(c->device));
    hipFree(c->d_rects);
    hipFree(c->d_srcs);
    c->d_rects = nullptr;
    c->d_srcs = nullptr;
    if (num_walls) {
        HIPCHK(hipMalloc(&c->d_rects, rd.size() * sizeof(RectDev)));
        HIPCHK(hipMemcpy(c->d_rects, rd.data(), rd.size() * sizeof(RectDev), hipMemcpyHostToDevice));
    }
    if (!sd.empty()) {
        HIPCHK(hipMalloc(&c->d_srcs, sd.size() * sizeof(SrcDev)));
        HIPCHK(hipMemcpy(c->d_srcs, sd.data(), sd.size() * sizeof(SrcDev), hipMemcpyHostToDevice));
    }
    {   /* the builtin-derived per-rect / per-emitter values, on the device (k_scene_setup) */
        std::vector<fmgi_rect> raw(walls, walls + num_walls);
        raw.insert(raw.end(), c->h_srcs.begin(), c->h_srcs.end());
        if (!raw.empty()) {
            fmgi_rect *d_raw = nullptr;
            HIPCHK(hipMalloc(&d_raw, raw.size() * sizeof(fmgi_rect)));
            hipError_t e = hipMemcpy(d_raw, raw.data(), raw.size() * sizeof(fmgi_rect), hipMemcpyHostToDevice);
            if (e == hipSuccess)
                e = fmgi_launch_scene_setup(d_raw, num_walls, d_raw + num_walls, (int)c->h_srcs.size(), c->d_rects,
                                            c->d_srcs, c->stream);
            if (e == hipSuccess) e = hipStreamSynchronize(c->stream);
            hipFree(d_raw);
            if (e != hipSuccess) return set_err(FMGI_ERR_HIP, "scene setup: %s", hipGetErrorString(e));
        }
    }
    c->nsrcs = num_windows + num_lights; /* (build_compact sizes the staged emitters) */
    if (try_compact) { /* the compact tables need the device-computed fields: the walls back to the host */
        std::vector<RectDev> drd((size_t)num_walls);
        HIPCHK(hipMemcpy(drd.data(), c->d_rects, drd.size() * sizeof(RectDev), hipMemcpyDeviceToHost));
        if (build_compact(c, drd, fb, gcomp)) {
            c->compact = true;
            gb = gcomp;
            c->gimg_bytes = (int)(gb.img.size() * sizeof(GridPlane));
            c->grid_cells = (int)gb.cells.size();
            c->grid_entries = (int)gb.idx.size();
            c->h_grid = gb;
        }
    }
    hipFree(c->d_fimg);
    hipFree(c->d_general);
    c->d_fimg = nullptr;
    c->d_general = nullptr;
    HIPCHK(hipMalloc(&c->d_fimg, fb.img.size() * sizeof(FilterRec)));
    HIPCHK(hipMemcpy(c->d_fimg, fb.img.data(), fb.img.size() * sizeof(FilterRec), hipMemcpyHostToDevice));
    if (!fb.general.empty()) {
        HIPCHK(hipMalloc(&c->d_general, fb.general.size() * sizeof(int32_t)));
        HIPCHK(hipMemcpy(c->d_general, fb.general.data(), fb.general.size() * sizeof(int32_t), hipMemcpyHostToDevice));
    }
    hipFree(c->d_gimg);
    hipFree(c->d_gcells);
    hipFree(c->d_gcellsF);
    hipFree(c->d_grecs);
    hipFree(c->d_gidx);
    c->d_gimg = nullptr;
    c->d_gcells = nullptr;
    c->d_gcellsF = nullptr;
    c->d_grecs = nullptr;
    c->d_gidx = nullptr;
    HIPCHK(upload(&c->d_gimg, gb.img));
    HIPCHK(upload(&c->d_gcells, gb.cells));
    HIPCHK(upload(&c->d_gcellsF, gb.cellsF));
    {   /* ScanHybrid's full image: the filter image (a multiple of 64 B), the plane image, the plan, the pairs */
        std::vector<char> both((size_t)c->himg_full_bytes);
        memcpy(both.data(), fb.img.data(), (size_t)c->fimg_bytes);
        memcpy(both.data() + c->fimg_bytes, gb.img.data(), (size_t)c->gimg_bytes);
        if (!plan_blob.empty()) memcpy(both.data() + c->plan_off, plan_blob.data(), plan_blob.size());
        if (c->pair_off_full + pairs_img.size() * sizeof(FilterPairHalf) <= both.size())
            memcpy(both.data() + c->pair_off_full, pairs_img.data(), pairs_img.size() * sizeof(FilterPairHalf));
        hipFree(c->d_himg_full);
        c->d_himg_full = nullptr;
        HIPCHK(upload(&c->d_himg_full, both));
        /* ... and the default instance's: the plane image, then the pairs */
        std::vector<char> img((size_t)c->himg_bytes);
        memcpy(img.data(), gb.img.data(), (size_t)c->gimg_bytes);
        memcpy(img.data() + c->pair_off, pairs_img.data(), pairs_img.size() * sizeof(FilterPairHalf));
        hipFree(c->d_himg);
        c->d_himg = nullptr;
        HIPCHK(upload(&c->d_himg, img));
    }
    HIPCHK(upload(&c->d_grecs, gb.recs));
    HIPCHK(upload(&c->d_gidx, gb.idx));
    }
    c->num_texels = num_texels;
    if (c->device != FMGI_HOST_ONLY) {
        int rc = configure_accum(c);
        if (rc != FMGI_OK) return rc;
    }
    c->nrects = num_walls;
    c->nsrcs = num_windows + num_lights;
    c->nwindows = num_windows;
    c->nlights = num_lights;
    c->num_texels = num_texels;
    c->h_launches.clear();
    c->total_items = 0;
    c->scene_gen++;
    return FMGI_OK;
}

FMGI_API int fmgi_set_grid_cells_per_record(fmgi_context *c, int cells_per_record) {
    if (!c || cells_per_record < 0 || cells_per_record > 64) return set_err(FMGI_ERR_ARG, "cells per record 0..64");
    c->grid_cpr = cells_per_record;
    return FMGI_OK;
}

FMGI_API int fmgi_experiments(void) { return FMGI_EXPERIMENTS; }

FMGI_API int fmgi_set_option(fmgi_context *c, int option, int64_t value) {
    if (!c || option <= 0 || option >= FMGI_OPT_COUNT) return set_err(FMGI_ERR_ARG, "fmgi_set_option: bad option %d", option);
    c->opt[option] = value;
    return FMGI_OK;
}

FMGI_API int64_t fmgi_plan_count(const fmgi_rect *windows, int num_windows, const fmgi_rect *lights, int num_lights,
                                 int spa, int wg, uint64_t *total_items) {
    if (wg <= 0) return set_err(FMGI_ERR_ARG, "wg must be > 0");
    int64_t nl = 0;
    uint64_t tot = 0, cap = (uint64_t)wg * 100;
    for (int s = 0; s < num_windows + num_lights; s++) {
        const fmgi_rect &r = s < num_windows ? windows[s] : lights[s - num_windows];
        uint64_t n = source_items(r, (float)spa, (uint64_t)wg);
        nl += (int64_t)((n + cap - 1) / cap);
        tot += n;
    }
    if (total_items) *total_items = tot;
    return nl;
}

FMGI_API int64_t fmgi_plan(fmgi_context *c, int spa, int wg, const int32_t *rng_offsets, int64_t n_offsets,
                           uint64_t *total_items) {
    if (!c || wg <= 0) return set_err(FMGI_ERR_ARG, "fmgi_plan: bad arguments");
    std::vector<LaunchDev> L;
    uint64_t item = 0, cap = (uint64_t)wg * 100;
    int64_t k = 0;
    for (int s = 0; s < c->nsrcs; s++) {
        uint64_t n = source_items(c->h_srcs[s], (float)spa, (uint64_t)wg);
        while (n) { /* global_illumination_cl.c:246-256 */
            int32_t off;
            if (rng_offsets) {
                if (k >= n_offsets) return set_err(FMGI_ERR_ARG, "fmgi_plan: %lld rng offsets are not enough", (long long)n_offsets);
                off = rng_offsets[k];
            } else {
                off = rand();
            }
            k++;
            uint64_t ws = n < cap ? n : cap;
            n -= ws;
            LaunchDev d;
            d.item_begin = item;
            d.count = (uint32_t)ws;
            d.rng_offset = off;
            d.source = s;
            d.is_window = s < c->nwindows;
            L.push_back(d);
            item += ws;
        }
    }
    if (c->device != FMGI_HOST_ONLY) {
    HIPCHK(hipSetDevice(c->device));
    if ((int64_t)L.size() > c->d_launch_cap) {
        hipFree(c->d_launches);
        c->d_launches = nullptr;
        c->d_launch_cap = 0;
        HIPCHK(hipMalloc(&c->d_launches, L.size() * sizeof(LaunchDev)));
        c->d_launch_cap = (int64_t)L.size();
    }
    if (!L.empty()) HIPCHK(hipMemcpy(c->d_launches, L.data(), L.size() * sizeof(LaunchDev), hipMemcpyHostToDevice));
    /* per-source lookup tables of the kernel's work-item -> launch mapping */
    std::vector<uint64_t> sib((size_t)c->nsrcs + 1, item);
    std::vector<int32_t> sl0((size_t)std::max(c->nsrcs, 1), (int32_t)L.size());
    for (int64_t k = (int64_t)L.size() - 1; k >= 0; k--) {
        sib[(size_t)L[k].source] = L[k].item_begin;
        sl0[(size_t)L[k].source] = (int32_t)k;
    }
    if ((int64_t)sib.size() > c->d_src_cap) { /* grown only: repeated plans of one scene allocate nothing */
        hipFree(c->d_src_item_begin);
        hipFree(c->d_src_launch0);
        c->d_src_item_begin = nullptr;
        c->d_src_launch0 = nullptr;
        c->d_src_cap = 0;
        HIPCHK(hipMalloc(&c->d_src_item_begin, sib.size() * sizeof(uint64_t)));
        HIPCHK(hipMalloc(&c->d_src_launch0, sib.size() * sizeof(int32_t)));
        c->d_src_cap = (int64_t)sib.size();
    }
    HIPCHK(hipMemcpy(c->d_src_item_begin, sib.data(), sib.size() * sizeof(uint64_t), hipMemcpyHostToDevice));
    HIPCHK(hipMemcpy(c->d_src_launch0, sl0.data(), sl0.size() * sizeof(int32_t), hipMemcpyHostToDevice));
    }
    {   /* per-source item ranges (a source's launches are consecutive in the schedule) */
        const bool same = (int)c->src_lo.size() == c->nsrcs;
        std::vector<uint64_t> lo((size_t)c->nsrcs, UINT64_MAX), hi((size_t)c->nsrcs, 0);
        for (const LaunchDev &l : L) {
            lo[(size_t)l.source] = std::min<uint64_t>(lo[(size_t)l.source], l.item_begin);
            hi[(size_t)l.source] = std::max<uint64_t>(hi[(size_t)l.source], l.item_begin + l.count);
        }
        if (!same || lo != c->src_lo || hi != c->src_hi) c->src_cost_per_item.clear(); /* other schedule */
        c->src_lo.swap(lo);
        c->src_hi.swap(hi);
    }
    c->launch_cap = (uint32_t)cap;
    c->h_launches.swap(L);
    c->total_items = item;
    if (total_items) *total_items = item;
    return (int64_t)c->h_launches.size();
}

FMGI_API int64_t fmgi_get_plan(fmgi_context *c, fmgi_launch *out, int64_t cap) {
    if (!c) return set_err(FMGI_ERR_ARG, "null context");
    int64_t n = (int64_t)c->h_launches.size();
    if (out) memcpy(out, c->h_launches.data(), (size_t)std::min(n, cap) * sizeof(fmgi_launch));
    return n;
}

/*
 * What a bake stages in LDS besides the scan image, and the workgroup size it runs with. Every photon
 * emission reads its emitter's SrcDev and every scan's phase 2 reads the winner's RectDev; from global
 * memory each is a dependent L2 round trip in the loop. A workgroup's LDS copy of the tables (128 B per
 * emitter / wall) replaces them with LDS reads where the copy costs no occupancy: the emitters always
 * (a few KB), the walls when some workgroup size keeps at least the resident waves the bake has without
 * them (box200: 25.6 KB per workgroup; FMGI_RECTS_LDS=0/1 forces, FMGI_SRCS_LDS=0 turns the emitters off,
 * FMGI_BLOCK fixes the workgroup size).
 */
struct StagePlan {
    int block = 256;
    int bytes = 0;                   /* staged blob = image (16-B aligned) | rects | srcs | cells | overflow */
    int rects_off = -1, srcs_off = -1, cells_off = -1, grecs_off = -1, gidx_off = -1;
    int rectc_off = -1, class_off = -1, recf_off = -1, cellc_off = -1; /* the compact closed-box tables */
};

static int stage_bytes(const fmgi_context *c, int kernel, bool rects, bool srcs, bool cells, bool grecs, int *roff,
                       int *soff, int *coff = nullptr, int *groff = nullptr, int *gioff = nullptr) {
    int off = (image_bytes(c, kernel) + 15) & ~15;
    if (roff) *roff = rects ? off : -1;
    if (rects) off += c->nrects * (int)sizeof(RectLds);
    if (soff) *soff = srcs ? off : -1;
    if (srcs) off += c->nsrcs * (int)sizeof(SrcDev);
    off = (off + 15) & ~15;
    if (coff) *coff = cells ? off : -1;
    if (cells) off += c->grid_cells * (int)sizeof(GridCell);
    /* with the cells, the overflow records of cells of more than two (float4) and their rect indices
       (`grecs`): the lane-by-lane stores' instance stages them (then its bake loop reads no global memory at
       all, FMGI_KVAR_STAGED); the rings' instance keeps them in global memory (box200 bake 76.65 -> 77.16 ms
       with them staged at 4 waves/SIMD, profiles/r04/s26). FMGI_GRECS_LDS=0/1 forces (experiments). */
    const char *ge = fmgi_exp_env("FMGI_GRECS_LDS");
    const bool ov = cells && (ge ? atoi(ge) == 1 : grecs);
    if (groff) *groff = ov ? off : -1;
    if (ov) off += c->grid_entries * 16;
    if (gioff) *gioff = ov ? off : -1;
    if (ov) off += c->grid_entries * 4;
    return (off + 15) & ~15;
}

/* the kernel instance a bake of `kernel` launches: the grid scan of a closed box (one plane per axis and
   class) has its own instance (FMGI_KVAR_AXES); FMGI_NO_AXES (experiments) keeps the general one.
   FMGI_PLAN=1 (experiments) walks the hybrid scan's walls over the floor plan: exact, but its per-lane
   walks diverge and wait on dependent LDS reads, and example.png baked 2x slower than with the filter
   pass (profiles/r03/s9) */
static bool grid_axes_scene(const fmgi_context *c) {
    return c->gJ[0] == 1 && c->gJ[1] == 1 && c->gJ[2] == 1 && !no_axes(c);
}
static int kernel_instance(const fmgi_context *c, int kernel) {
    const char *pe = fmgi_exp_env("FMGI_PLAN");
    if (kernel == FMGI_KERNEL_HYBRID && c->plan_off >= 0 && pe && atoi(pe) == 1) return kernel | FMGI_KVAR_PLAN;
    return kernel == FMGI_KERNEL_GRID && grid_axes_scene(c) ? (kernel | FMGI_KVAR_AXES) : kernel;
}

static StagePlan plan_stage(const fmgi_context *c, int kernel, int accum, bool trace) {
    StagePlan p;
    const char *be = fmgi_exp_env("FMGI_BLOCK");
    const int forced_block = (be && atoi(be) >= 64 && atoi(be) <= 1024 && atoi(be) % 64 == 0) ? atoi(be) : 0;
    p.block = forced_block ? forced_block : 256;
    if (kernel == FMGI_KERNEL_EXACT) return p; /* no LDS image: nothing is staged */
    if (c->compact && kernel == FMGI_KERNEL_GRID && accum == kAccScatter && c->nsrcs > 0 && !forced_block) {
        /* the compact closed box: image | emitters | classes | RectC | filter extents | cells, one 1024-lane
           workgroup per CU (the tables take most of its LDS) */
        int off = (c->gimg_bytes + 15) & ~15;
        p.srcs_off = off;
        off += c->nsrcs * (int)sizeof(SrcDev);
        p.class_off = off;
        off += (int)(c->h_classc.size() * sizeof(ClassC));
        p.rectc_off = off;
        off += (int)((c->h_rectc.size() * sizeof(RectC) + 15) & ~(size_t)15);
        p.recf_off = off;
        off += (int)(c->h_recf.size() * sizeof(float));
        p.cellc_off = off;
        off += (int)(c->h_cellc.size() * sizeof(uint32_t));
        p.bytes = (off + 15) & ~15;
        p.block = 1024;
        const int inst = FMGI_KERNEL_GRID | FMGI_KVAR_AXES | FMGI_KVAR_COMPACT;
        if (fmgi_bake_lds(inst, accum, p.block, p.bytes, nullptr) <= kBakeLdsMax &&
            fmgi_bake_resident_blocks(inst, accum, trace, p.block, p.bytes) >= 1)
            return p;
        p = StagePlan{}; /* (does not launch: the general planning below) */
    }
    const char *se = fmgi_exp_env("FMGI_SRCS_LDS"), *re = fmgi_exp_env("FMGI_RECTS_LDS");
    const bool srcs = c->nsrcs > 0 && !(se && atoi(se) == 0);
    const int rects_mode = re ? atoi(re) : -1; /* -1 auto */
    const int kfn = kernel_instance(c, kernel);
    /* resident waves per CU of a (block, staged bytes) choice; 0 if it cannot launch */
    auto waves = [&](int block, int bytes) -> int {
        if (fmgi_bake_lds(kfn, accum, block, bytes, nullptr) > kBakeLdsMax) return 0;
        return fmgi_bake_resident_blocks(kfn, accum, trace, block, bytes) * (block / 64);
    };
    /* multiples of 4 waves only: a workgroup's waves are dealt to the CU's 4 SIMDs, and 10 waves (640
       lanes) left SIMDs unevenly loaded (box200: 149.6 ms against 123.8 ms at 256, profiles/r03/s3) */
    /* (768-lane workgroups measured pathological for every instance built for 4 waves/SIMD: box200 bake
       1.6-2.2 s instead of 0.05-0.08 s, profiles/r04/s7; not offered) */
    /* AccScatter (no rings: ~0.4 KB of LDS per wave) is built for 6 waves/SIMD: 768-lane workgroups, two per
       CU, keep the grid cells staged beside the walls at 24 waves per CU, which 512-lane ones (three per CU)
       cannot */
    const int blocks_ring[] = {256, 512, 1024}, blocks_scatter[] = {256, 512, 768, 1024};
    const bool scat = accum == kAccScatter;
    const int *blocks_all = scat ? blocks_scatter : blocks_ring;
    const int nblocks = scat ? 4 : 3;
    /* the grid cells in LDS: every cell lookup an LDS read instead of an L2 one. The closed boxes' coarse
       grid asks for it (kept only if the wave count holds); FMGI_CELLS_LDS=1 forces it for any grid or
       hybrid scan that fits, 0 turns it off (experiments) */
    const char *ce = fmgi_exp_env("FMGI_CELLS_LDS");
    /* (only the grid scan reads the staged GridCell copy: ScanHybrid's grid walk reads GridCellF from global
       memory, so staging for it would be dead LDS) */
    const bool cells_forced = ce && atoi(ce) == 1 && kernel == FMGI_KERNEL_GRID;
    bool cells = cells_forced || (!ce && c->cells_lds && kernel == FMGI_KERNEL_GRID);
    auto best = [&](bool rects, int &bb, int &bw) {
        const int bytes = stage_bytes(c, kernel, rects, srcs, cells, accum == kAccScatter, nullptr, nullptr);
        bb = p.block;
        bw = waves(p.block, bytes);
        if (forced_block) return;
        for (int k = 0; k < nblocks; k++) {
            const int B = blocks_all[k];
            const int w = waves(B, bytes);
            if (w > bw) { bw = w; bb = B; }
        }
    };
    int b0, w0, b1 = 0, w1 = 0;
    best(false, b0, w0);
    bool rects = false;
    if (rects_mode != 0 && c->nrects > 0) {
        best(true, b1, w1);
        /* the walls in LDS take the winners' records off the vector-memory path, which is what binds the
           bake (TA busy 98 %, profiles/r03/s3): worth a wave per SIMD (box200: 16 waves per CU with the
           walls staged 77.6 ms, 20 waves without 123.8 ms), not two */
        rects = rects_mode == 1 ? w1 > 0 : (w1 > 0 && w1 >= std::min(w0, 16));
    }
    if (cells) { /* staged only if they fit (forced) or keep the wave count of the plan without them */
        const int wc = rects ? w1 : w0;
        cells = false;
        int nb0, nw0, nb1 = 0, nw1 = 0;
        best(false, nb0, nw0);
        if (rects) best(true, nb1, nw1);
        const int wn = rects ? nw1 : nw0;
        if (wc > 0 && (cells_forced || wc >= wn)) {
            cells = true;
        } else {
            b0 = nb0, w0 = nw0, b1 = nb1, w1 = nw1;
        }
    }
    p.block = rects ? b1 : b0;
    p.bytes = stage_bytes(c, kernel, rects, srcs, cells, accum == kAccScatter, &p.rects_off, &p.srcs_off, &p.cells_off,
                          &p.grecs_off,
                          &p.gidx_off);
    return p;
}

static int grid_blocks(const fmgi_context *c, int kernel, int accum, bool trace, int block, int lds, uint64_t items,
                       int inst = -1) {
    /* persistent grid: exactly the blocks that are resident at once (occupancy from the VGPR/SGPR/LDS
       use of the kernel actually launched), so no block starts late and lengthens the tail; never more
       lanes than work items */
    int per_cu = fmgi_bake_resident_blocks(inst >= 0 ? inst : kernel_instance(c, kernel), accum, trace, block, lds);
    if (per_cu <= 0) per_cu = 4;
    if (const char *pe = fmgi_exp_env("FMGI_BAKE_WG_PER_CU")) /* experiments: leave room for concurrent folds */
        if (atoi(pe) > 0) per_cu = std::min(per_cu, atoi(pe));
    uint64_t lanes_max = (uint64_t)c->num_cus * per_cu * block;
    uint64_t lanes = std::min<uint64_t>(items, lanes_max);
    return (int)std::max<uint64_t>(1, (lanes + block - 1) / block);
}

static hipError_t pool_event(fmgi_context *c, hipEvent_t &ev) {
    if (!c->ev_pool.empty()) {
        ev = c->ev_pool.back();
        c->ev_pool.pop_back();
        return hipSuccess;
    }
    return hipEventCreate(&ev);
}

/* with fmgi_set_timing on: an event before a launch ... */
static hipError_t time_begin(fmgi_context *c, hipStream_t s, hipEvent_t &t0) {
    if (!c->timing) return hipSuccess;
    hipError_t e = pool_event(c, t0);
    return e != hipSuccess ? e : hipEventRecord(t0, s);
}

/* ... and one after it, kept for fmgi_get_timing */
static hipError_t time_end(fmgi_context *c, hipStream_t s, hipEvent_t t0, hipEvent_t &t1,
                           std::vector<std::pair<hipEvent_t, hipEvent_t>> &dst) {
    if (!c->timing) return hipSuccess;
    hipError_t e = pool_event(c, t1);
    if (e == hipSuccess) e = hipEventRecord(t1, s);
    if (e == hipSuccess) dst.emplace_back(t0, t1);
    return e;
}

/* work items per STREAM chunk: codes for 800 deposits per item, twice (stream + sorted), for each of the
   `sets` buffer sets in use, in at most half of the device memory that is free or already held by them */
static uint64_t stream_chunk_items(fmgi_context *c, int sets, int mode) {
    size_t fr = 0, tot = 0;
    if (hipMemGetInfo(&fr, &tot) != hipSuccess) fr = (size_t)8 << 30;
    /* the stream, and the slice-sorted copy of the unsorted layout (buckets: the pool is the stream plus its
       pads (<= 3 * 63 per 1024 codes), one partly filled block per wave and tile, and the block tables,
       within the 25 % allowance) */
    const double copies = mode == kStreamSliced ? 2.0 : (mode == kStreamBuckets ? 1.25 : (mode == kStreamDense ? 2.5 : 1.0));
    const double held = 4.0 * (double)(c->sb_cap_alloc[0] + c->sb_cap_alloc[1]) * (c->sb[0].sorted ? 2.0 : 1.0) +
                        4.0 * (double)(c->sb[0].dense_alloc + c->sb[1].dense_alloc);
    const double avail = (double)fr + held;
    uint64_t items = (uint64_t)(avail * 0.5 / ((double)sets * copies * 4.0 * FMGI_EVENTS_PER_ITEM));
    /* slices are indexed in 32 bits by the sort kernel's grid */
    const uint64_t max_items = ((1ull << 31) - 1) / FMGI_EVENTS_PER_ITEM * FMGI_STREAM_SLICE;
    items = std::min(items, max_items);
    return std::max<uint64_t>(items, 65536);
}

/* the stream layout of a STREAM bake: per-wave tile buckets (the bake's ring flush sorts by fold tile and
   appends each tile's run to the wave's bucket of that tile; the fold reads whole blocks) when the tiles
   fit one histogram entry per lane, else unsorted codes + k_slice_sort. FMGI_PRESORT=0/1/2 forces unsorted /
   presorted segments / buckets. */
static int stream_layout(const fmgi_context *c) {
    const int P = (c->num_texels + (1 << FMGI_TILE_BITS) - 1) >> FMGI_TILE_BITS;
    const char *pre_env = fmgi_exp_env("FMGI_PRESORT"); /* experiments: 1 = presorted segments */
    int smode = (P >= 1 && P <= FMGI_PRESORT_MAX_TILES) ? kStreamBuckets : kStreamSliced;
    if (pre_env && P >= 1 && P <= FMGI_PRESORT_MAX_TILES) smode = std::max(0, std::min(2, atoi(pre_env)));
    if (pre_env && atoi(pre_env) == 0) smode = kStreamSliced;
    if (c->opt[FMGI_OPT_STREAM_LAYOUT] == 0) smode = kStreamSliced; /* tests: the slice-sorted layout */
    if (smode == kStreamBuckets) { /* FMGI_DENSE=1: the dense stream and k_bin instead of the bake's rings */
        const char *de = fmgi_exp_env("FMGI_DENSE");
        if (de && atoi(de) == 1) smode = kStreamDense;
    }
    return smode;
}

/* the accumulation of a bake's kernel instance: the bucket layout of the stream through per-wave rings
   (kAccBucket) or through per-workgroup tile lines (kAccLines, FMGI_LINES=1) */
static int exec_accum(const fmgi_context *c) {
    if (c->accum == FMGI_ACCUM_STREAM && stream_layout(c) == kStreamDense) return kAccDense;
    if (c->accum == FMGI_ACCUM_STREAM && stream_layout(c) == kStreamSliced) return kAccSliced;
    if (c->accum != FMGI_ACCUM_STREAM || stream_layout(c) != kStreamBuckets) return c->accum;
    const char *le = fmgi_exp_env("FMGI_LINES");
    if (le && atoi(le) == 1) return kAccLines;
    /* AUTO: the lane-by-lane stores (AccScatter) when the scene's wall table (and the closed box's grid cells)
       fit in LDS beside the image, so the bake loop reads no global memory and the scattered stores' slow
       completions never hold up a load's s_waitcnt (box200: bake 76.7 -> 69.3 ms at 6 instead of 4 waves per
       SIMD; box2000, whose 2000 walls stay in L2: 132 ms with the rings, 160 with scattered stores; profiles/
       r05/s5). FMGI_SCATTER=0/1 forces either (experiments, tests). */
    if (c->opt[FMGI_OPT_BUCKET_FILL] >= 0) return c->opt[FMGI_OPT_BUCKET_FILL] ? kAccScatter : kAccBucket; /* tests */
    if (c->compact) return kAccScatter; /* the compact closed box: every table staged (FMGI_KVAR_COMPACT) */
    const size_t tables = (size_t)c->nrects * sizeof(RectLds) + (c->cells_lds ? (size_t)c->grid_cells * sizeof(GridCell) : 0);
    return tables <= 64 * 1024 ? kAccScatter : kAccBucket;
}

static int bake_common(fmgi_context *c, uint64_t b, uint64_t e, void *lm, int kernel, hipStream_t s, bool trace,
                       void *events, int32_t *counts, uint32_t *rngf) {
    if (!c || !lm) return set_err(FMGI_ERR_ARG, "fmgi_bake_items: bad arguments");
    if (c->device == FMGI_HOST_ONLY) return set_err(FMGI_ERR_NO_DEVICE, "host-only context cannot bake");
    if (e > c->total_items || b > e) return set_err(FMGI_ERR_ARG, "item range [%llu,%llu) outside plan of %llu items",
                                                  (unsigned long long)b, (unsigned long long)e,
                                                  (unsigned long long)c->total_items);
    if (kernel < FMGI_KERNEL_EXACT || kernel > FMGI_KERNEL_HYBRID) return set_err(FMGI_ERR_ARG, "bad kernel %d", kernel);
    const bool was_auto = kernel == FMGI_KERNEL_AUTO;
    /* the kernel instance's accumulation: the bucket layout of the stream has its own (kAccBucket) */
    int kacc = exec_accum(c);
    if (was_auto) kernel = c->auto_kernel;
    /* an image too large for LDS: same results, other scan (checked with the LDS of the instance launched) */
    kernel = fitting_kernel(c, kernel, kacc, bake_block());
    if (b == e) return FMGI_OK;
    /* a launch with at most half as many items as resident lanes runs ScanFast with cooperative lanes
       (below): on such launches that beats the hybrid scan's single lane per item (config 1: 6.6 ms
       hybrid bake vs ~3.5 ms cooperative) */
    if (was_auto && kernel == FMGI_KERNEL_HYBRID && !trace && c->accum == FMGI_ACCUM_STREAM &&
        fitting_kernel(c, FMGI_KERNEL_FAST, kacc, bake_block()) == FMGI_KERNEL_FAST) {
        const StagePlan fp = plan_stage(c, FMGI_KERNEL_FAST, kacc, trace);
        const uint64_t lanes_max =
            (uint64_t)grid_blocks(c, FMGI_KERNEL_FAST, kacc, trace, fp.block, fp.bytes, UINT64_MAX) * fp.block;
        if ((e - b) * 2 <= lanes_max) kernel = FMGI_KERNEL_FAST;
    }
    StagePlan sp = plan_stage(c, kernel, kacc, trace);
    /* the lane-by-lane stores pay only when the loop reads no global table (exec_accum's AUTO choice checks
       the tables' size, the plan whether they were staged): a plan that left the walls, or a closed box's
       cells, in global memory takes the rings instead (box2000 before its compact tables: 160 ms scattered,
       132 ms with the rings) */
    if (kacc == kAccScatter && c->opt[FMGI_OPT_BUCKET_FILL] < 0 && !c->compact &&
        ((c->nrects > 0 && sp.rects_off < 0) || (c->cells_lds && kernel == FMGI_KERNEL_GRID && sp.cells_off < 0)) &&
        fitting_kernel(c, kernel, kAccBucket, bake_block()) == kernel) {
        kacc = kAccBucket;
        sp = plan_stage(c, kernel, kacc, trace);
    }
    const int block = sp.block;
    /* the closed box with every table staged (walls, emitters, grid cells) launches the instance whose
       global-memory paths for them are compiled out (FMGI_KVAR_STAGED); FMGI_NO_STAGED=1 (experiments) keeps
       the general one */
    int inst = kernel_instance(c, kernel);
    /* (the staged and compact instances have no path for rects that are not axis-aligned) */
    if (inst == (FMGI_KERNEL_GRID | FMGI_KVAR_AXES) && sp.rects_off >= 0 && sp.srcs_off >= 0 && sp.cells_off >= 0 &&
        sp.grecs_off >= 0 && c->ngeneral == 0 && !fmgi_exp_env("FMGI_NO_STAGED"))
        inst |= FMGI_KVAR_STAGED;
    if (inst == (FMGI_KERNEL_GRID | FMGI_KVAR_AXES) && sp.rectc_off >= 0) inst |= FMGI_KVAR_COMPACT;
    /* a closed box built with the coarse LDS grid (5 cells per record) but launched without the cells staged
       reads that coarser grid from L2, slower than the 16-per-record grid it replaced: said once per context */
    if (c->cells_lds && kernel == FMGI_KERNEL_GRID && sp.cells_off < 0 && sp.rectc_off < 0 && !c->warned_cells &&
        !getenv("FMGI_QUIET")) {
        fprintf(stderr, "fmgi: the closed-box grid's cells (%d, built for LDS) are not staged at block %d: "
                        "lookups read L2 (FMGI_CELLS_LDS=0 builds the finer global grid)\n", c->grid_cells, block);
        c->warned_cells = true;
    }
    if (c->nsrcs == 0) return set_err(FMGI_ERR_STATE, "no scene");
    /* no walls: every photon escapes at its first scan (photonmap.cl:208), so nothing is deposited */
    if (c->nrects == 0) return FMGI_OK;
    HIPCHK(hipSetDevice(c->device));
    BakeArgs a;
    memset(&a, 0, sizeof a);
    a.rects = c->d_rects;
    a.nrects = c->nrects;
    a.srcs = c->d_srcs;
    a.launches = c->d_launches;
    a.nlaunches = (int)c->h_launches.size();
    a.src_item_begin = c->d_src_item_begin;
    a.src_launch0 = c->d_src_launch0;
    a.nsrc = c->nsrcs;
    a.nwindows = c->nwindows;
    a.launch_cap = c->launch_cap;
    a.item_begin = b;
    a.item_end = e;
    a.counter = c->d_counter;
    a.lm = (unsigned long long *)lm;
    a.stats = c->d_stats;
    if (kernel == FMGI_KERNEL_GRID) {
        a.fimg = c->d_gimg;
        a.fimg_bytes = c->gimg_bytes;
        for (int k = 0; k < 3; k++) a.fJ[k] = c->gJ[k];
        a.gcells = c->d_gcells;
        a.gcellsF = c->d_gcellsF;
        a.grecs = c->d_grecs;
        a.gridx = c->d_gidx;
        a.grid_axes = grid_axes_scene(c) ? 1 : 0;
        a.grid_xy_separate = fmgi_exp_env("FMGI_GRID_SEPARATE") ? 1 : 0;
    } else if (kernel == FMGI_KERNEL_HYBRID) {
        const bool full = hybrid_full(c);
        a.fimg = full ? c->d_himg_full : c->d_himg;
        a.fimg_bytes = full ? c->himg_full_bytes : c->himg_bytes;
        a.hyb_off = full ? c->fimg_bytes : 0;
        for (int k = 0; k < 3; k++) {
            a.fJ[k] = c->fJ[k];
            a.gJ[k] = c->gJ[k];
        }
        a.gcells = c->d_gcells;
        a.gcellsF = c->d_gcellsF;
        a.grecs = c->d_grecs;
        a.gridx = c->d_gidx;
        a.grid_code_or = 0x40000000;
        a.plan_off = full ? c->plan_off : -1;
        a.pair_off = full ? c->pair_off_full : c->pair_off;
        a.pG[0] = c->pG[0];
        a.pG[1] = c->pG[1];
    } else {
        a.fimg = c->d_fimg;
        a.fimg_bytes = c->fimg_bytes;
        for (int k = 0; k < 3; k++) a.fJ[k] = c->fJ[k];
    }
    a.rects_off = a.srcs_off = a.cells_off = a.grecs_off = a.gidx_off = -1;
    a.rectc_off = a.class_off = a.recf_off = a.cellc_off = -1;
    a.cdummy = c->nrects;
    if (sp.rectc_off >= 0) { /* the compact blob: image | srcs | classes | RectC | filter extents | cells */
        const uint64_t key = (c->scene_gen << 9) | 0x1FFu;
        if (c->blob_key != key) {
            if (c->blob_cap < (size_t)sp.bytes) {
                HIPCHK(hipStreamSynchronize(s)); /* no earlier bake may still stage the old blob */
                hipFree(c->d_blob);
                c->d_blob = nullptr;
                c->blob_cap = 0;
                HIPCHK(hipMalloc(&c->d_blob, (size_t)sp.bytes));
                c->blob_cap = (size_t)sp.bytes;
            }
            HIPCHK(hipMemsetAsync(c->d_blob, 0, (size_t)sp.bytes, s));
            if (a.fimg_bytes) HIPCHK(hipMemcpyAsync(c->d_blob, a.fimg, (size_t)a.fimg_bytes, hipMemcpyDeviceToDevice, s));
            HIPCHK(hipMemcpyAsync(c->d_blob + sp.srcs_off, c->d_srcs, (size_t)c->nsrcs * sizeof(SrcDev),
                                  hipMemcpyDeviceToDevice, s));
            HIPCHK(hipMemcpyAsync(c->d_blob + sp.class_off, c->h_classc.data(), c->h_classc.size() * sizeof(ClassC),
                                  hipMemcpyHostToDevice, s));
            HIPCHK(hipMemcpyAsync(c->d_blob + sp.rectc_off, c->h_rectc.data(), c->h_rectc.size() * sizeof(RectC),
                                  hipMemcpyHostToDevice, s));
            HIPCHK(hipMemcpyAsync(c->d_blob + sp.recf_off, c->h_recf.data(), c->h_recf.size() * sizeof(float),
                                  hipMemcpyHostToDevice, s));
            HIPCHK(hipMemcpyAsync(c->d_blob + sp.cellc_off, c->h_cellc.data(), c->h_cellc.size() * sizeof(uint32_t),
                                  hipMemcpyHostToDevice, s));
            HIPCHK(hipStreamSynchronize(s)); /* (the host tables stay; the copies are done before they could change) */
            c->blob_key = key;
        }
        a.fimg = c->d_blob;
        a.fimg_bytes = sp.bytes;
        a.srcs_off = sp.srcs_off;
        a.rectc_off = sp.rectc_off;
        a.class_off = sp.class_off;
        a.recf_off = sp.recf_off;
        a.cellc_off = sp.cellc_off;
    } else if (sp.rects_off >= 0 || sp.srcs_off >= 0 || sp.cells_off >= 0) { /* the blob: image | rects | srcs | cells */
        const uint64_t key = (c->scene_gen << 9) | (sp.grecs_off >= 0 ? 0x100u : 0u) |
                             (kernel == FMGI_KERNEL_HYBRID && hybrid_full(c) ? 0x40u : 0u) |
                             ((uint64_t)(kernel & 0xF) << 2) | (sp.rects_off >= 0 ? 2u : 0u) | (sp.srcs_off >= 0 ? 1u : 0u) |
                             (sp.cells_off >= 0 ? 0x80u : 0u);
        if (c->blob_key != key) {
            if (c->blob_cap < (size_t)sp.bytes) {
                HIPCHK(hipStreamSynchronize(s)); /* no earlier bake may still stage the old blob */
                hipFree(c->d_blob);
                c->d_blob = nullptr;
                c->blob_cap = 0;
                HIPCHK(hipMalloc(&c->d_blob, (size_t)sp.bytes));
                c->blob_cap = (size_t)sp.bytes;
            }
            if (a.fimg_bytes) HIPCHK(hipMemcpyAsync(c->d_blob, a.fimg, (size_t)a.fimg_bytes, hipMemcpyDeviceToDevice, s));
            if (sp.rects_off >= 0) { /* RectDev -> RectLds (the device-computed fields, repacked) */
                std::vector<RectDev> rd((size_t)c->nrects);
                HIPCHK(hipStreamSynchronize(s));
                HIPCHK(hipMemcpy(rd.data(), c->d_rects, rd.size() * sizeof(RectDev), hipMemcpyDeviceToHost));
                c->h_rects_lds.assign((size_t)c->nrects, RectLds{});
                for (size_t i = 0; i < rd.size(); i++) {
                    const RectDev &r = rd[i];
                    RectLds &q = c->h_rects_lds[i];
                    q.px = r.px; q.py = r.py; q.pz = r.pz;
                    q.nx = r.nx; q.ny = r.ny; q.nz = r.nz;
                    q.wnx = r.wnx; q.wny = r.wny; q.wnz = r.wnz; q.wl = r.wl;
                    q.hnx = r.hnx; q.hny = r.hny; q.hnz = r.hnz; q.hl = r.hl;
                    q.base = r.base; q.W = r.W; q.H = r.H;
                    q.bux = r.bux; q.buy = r.buy; q.buz = r.buz;
                    q.bvx = r.bvx; q.bvy = r.bvy; q.bvz = r.bvz;
                    q.iwl = r.iwl; q.ihl = r.ihl;
                }
                HIPCHK(hipMemcpyAsync(c->d_blob + sp.rects_off, c->h_rects_lds.data(),
                                      c->h_rects_lds.size() * sizeof(RectLds), hipMemcpyHostToDevice, s));
            }
            if (sp.srcs_off >= 0)
                HIPCHK(hipMemcpyAsync(c->d_blob + sp.srcs_off, c->d_srcs, (size_t)c->nsrcs * sizeof(SrcDev),
                                      hipMemcpyDeviceToDevice, s));
            if (sp.cells_off >= 0) {
                HIPCHK(hipMemcpyAsync(c->d_blob + sp.cells_off, c->d_gcells, (size_t)c->grid_cells * sizeof(GridCell),
                                      hipMemcpyDeviceToDevice, s));
                if (sp.grecs_off >= 0) {
                    HIPCHK(hipMemcpyAsync(c->d_blob + sp.grecs_off, c->d_grecs, (size_t)c->grid_entries * 16,
                                          hipMemcpyDeviceToDevice, s));
                    HIPCHK(hipMemcpyAsync(c->d_blob + sp.gidx_off, c->d_gidx, (size_t)c->grid_entries * 4,
                                          hipMemcpyDeviceToDevice, s));
                }
            }
            c->blob_key = key;
        }
        a.fimg = c->d_blob;
        a.fimg_bytes = sp.bytes;
        a.rects_off = sp.rects_off;
        a.srcs_off = sp.srcs_off;
        a.cells_off = sp.cells_off;
        a.grecs_off = sp.grecs_off;
        a.gidx_off = sp.gidx_off;
    }
    a.general = c->d_general;
    a.ngeneral = c->ngeneral;
    a.counts = c->accum == FMGI_ACCUM_STATE ? c->d_counts : nullptr;
    a.num_texels = c->num_texels;
    a.events = events;
    a.ev_counts = counts;
    a.rng_final = rngf;
    a.overflow = c->d_stats + KSTAT_OVERFLOW;
    fmgi_bake_lds(kernel, kacc, block, a.fimg_bytes, &a.ring_off);
    /* lanes per work item: a launch with fewer items than resident lanes (BASELINE config 1 has 11,008)
       gives each item a group of up to 8 lanes that split every ScanFast scan's records, so the idle
       lanes shorten the items' serial photon chains (FMGI_COOP forces a group size: tests) */
    a.coop = 1;
    if (kernel == FMGI_KERNEL_FAST && !trace && c->accum == FMGI_ACCUM_STREAM) {
        if (c->opt[FMGI_OPT_COOP] > 0) {
            const int k = (int)c->opt[FMGI_OPT_COOP];
            a.coop = (k == 2 || k == 4 || k == 8) ? k : 1;
        } else {
            const uint64_t lanes_max =
                (uint64_t)grid_blocks(c, kernel, kacc, trace, block, a.fimg_bytes, UINT64_MAX) * block;
            while (a.coop < 8 && (e - b) * (uint64_t)a.coop * 2 <= lanes_max) a.coop *= 2;
        }
        if (a.coop > 1) kernel = FMGI_KERNEL_FAST_COOP;
    }
    /* fetch order: the lanes fetch work items through a table of source ranges, the sources whose items
       took the most scans on this context's previous bake first (longest-processing-time first), so
       the end of a launch with few items per lane is not a run of the longest items (example.png, config
       2, 3 items per lane: the last sources' items are the longest). The lightmap is an order-free exact
       sum, so any order gives the same bits. The first bake of a schedule measures (one atomic per item
       into a per-source total); FMGI_FETCH_ORDER=0 turns it off. */
    constexpr int kMaxTabs = 64;
    const char *fo_env = fmgi_exp_env("FMGI_FETCH_ORDER");
    const bool order_on = !(fo_env && atoi(fo_env) == 0) && c->nsrcs > 0;
    const int ns = c->nsrcs;
    /* only launches of at most 16 items per resident lane reorder (box200's 30 per lane: plain order) */
    const uint64_t order_lanes =
        order_on ? (uint64_t)grid_blocks(c, kernel, kacc, trace, block, a.fimg_bytes, UINT64_MAX) * block /
                       (uint64_t)a.coop
                 : 0;
    if (order_on) {
        if (!c->ev_cost) HIPCHK(hipEventCreateWithFlags(&c->ev_cost, hipEventDisableTiming));
        if (c->cost_pending && hipEventQuery(c->ev_cost) == hipSuccess) { /* the previous measurement */
            c->cost_pending = false;
            if (c->src_cost_per_item.size() != (size_t)ns) c->src_cost_per_item.assign((size_t)ns, 0.0);
            for (int k = 0; k < ns && k < (int)c->cost_items.size(); k++)
                if (c->cost_items[(size_t)k]) c->src_cost_per_item[(size_t)k] = (double)c->h_src_cost[k] / (double)c->cost_items[(size_t)k];
        }
        /* the previous call's kernels (maybe on another stream) are done with the table and the totals */
        HIPCHK(hipStreamWaitEvent(s, c->ev_cost, 0));
        if (c->fetch_tab_cap < kMaxTabs * 2 * ns) {
            hipFree(c->d_fetch_tab);
            c->d_fetch_tab = nullptr;
            c->fetch_tab_cap = 0;
            HIPCHK(hipMalloc(&c->d_fetch_tab, (size_t)kMaxTabs * 2 * ns * sizeof(uint32_t)));
            c->fetch_tab_cap = kMaxTabs * 2 * ns;
        }
        /* measure: the first bake of a schedule whose items could reorder. A call of more than 16 items
           per lane runs in plain order and skips it: its per-item atomics into a few per-source totals
           serialise (box200, one light source: first bake 242 ms instead of 126 ms) */
        if (!c->cost_pending && c->src_cost_per_item.empty() && e - b <= 16 * order_lanes) {
            if (c->src_cost_n < ns) {
                hipFree(c->d_src_cost);
                if (c->h_src_cost) (void)hipHostFree(c->h_src_cost);
                c->d_src_cost = c->h_src_cost = nullptr;
                c->src_cost_n = 0;
                HIPCHK(hipMalloc(&c->d_src_cost, (size_t)ns * 8));
                HIPCHK(hipHostMalloc((void **)&c->h_src_cost, (size_t)ns * 8, hipHostMallocDefault));
                c->src_cost_n = ns;
            }
            HIPCHK(hipMemsetAsync(c->d_src_cost, 0, (size_t)ns * 8, s));
            a.src_cost = c->d_src_cost;
            c->cost_items.assign((size_t)ns, 0);
            for (int k = 0; k < ns && k < (int)c->src_lo.size(); k++) {
                const uint64_t lo = std::max(c->src_lo[(size_t)k], b), hi = std::min(c->src_hi[(size_t)k], e);
                c->cost_items[(size_t)k] = lo < hi ? hi - lo : 0;
            }
        }
        c->h_fetch_tab.resize(kMaxTabs);
    }
    int ntab = 0;
    auto fetch_table = [&](uint64_t cb, uint64_t ce) -> hipError_t { /* a.fetch_tab for items [cb, ce) */
        a.fetch_tab = nullptr;
        a.fetch_nseg = 0;
        if (!order_on || (int)c->src_lo.size() != ns || ntab >= kMaxTabs || ce - cb > 16 * order_lanes ||
            ce > 0xFFFFFFFFull)
            return hipSuccess;
        /* costs per item: measured on this context's previous bake, else the prior "lights, then windows,
           each in reverse schedule order": a light's photons start inside the rooms and rarely escape, so
           its items are the longest (example.png config 2: plain order 24.5 ms, this prior 21.6 ms, the
           measured order 21.3 ms), and a one-shot call (main.c bakes once) gets most of the gain too */
        std::vector<double> prior;
        const std::vector<double> *cost = &c->src_cost_per_item;
        if (c->src_cost_per_item.size() != (size_t)ns) {
            prior.resize((size_t)ns);
            for (int k = 0; k < ns; k++) prior[(size_t)k] = (k >= c->nwindows ? 1e9 : 0.0) + k;
            cost = &prior;
        }
        std::vector<int> ord((size_t)ns);
        for (int k = 0; k < ns; k++) ord[(size_t)k] = k;
        std::stable_sort(ord.begin(), ord.end(), [&](int x, int y) { return (*cost)[(size_t)x] > (*cost)[(size_t)y]; });
        std::vector<uint32_t> &h = c->h_fetch_tab[(size_t)ntab];
        h.clear();
        uint64_t f = 0;
        for (int k : ord) {
            const uint64_t lo = std::max(c->src_lo[(size_t)k], cb), hi = std::min(c->src_hi[(size_t)k], ce);
            if (lo >= hi) continue;
            h.push_back((uint32_t)f);
            h.push_back((uint32_t)lo);
            f += hi - lo;
        }
        if (f != ce - cb || h.empty()) return hipSuccess; /* not covered: plain order */
        uint32_t *d = c->d_fetch_tab + (size_t)ntab * 2 * ns;
        hipError_t err = hipMemcpyAsync(d, h.data(), h.size() * sizeof(uint32_t), hipMemcpyHostToDevice, s);
        if (err != hipSuccess) return err;
        a.fetch_tab = d;
        a.fetch_nseg = (int)(h.size() / 2);
        ntab++;
        return hipSuccess;
    };
    auto finish_call = [&]() -> hipError_t { /* the measured totals to the host, and the call's end marker */
        if (!order_on) return hipSuccess;
        if (a.src_cost) {
            hipError_t err = hipMemcpyAsync(c->h_src_cost, c->d_src_cost, (size_t)ns * 8, hipMemcpyDeviceToHost, s);
            if (err != hipSuccess) return err;
            c->cost_pending = true;
        }
        return hipEventRecord(c->ev_cost, s);
    };
    if (c->accum != FMGI_ACCUM_STREAM) {
        HIPCHK(fetch_table(b, e));
        HIPCHK(hipMemsetAsync(c->d_counter, 0, 8, s));
        hipEvent_t t0 = nullptr, t1 = nullptr;
        HIPCHK(time_begin(c, s, t0));
        c->last_kernel = fmgi_bake_kernel_name(a.coop > 1 ? kernel_instance(c, kernel) : inst, kacc, trace);
        HIPCHK(fmgi_launch_bake(a, a.coop > 1 ? kernel_instance(c, kernel) : inst, kacc, trace,
                                grid_blocks(c, kernel, kacc, trace, block, a.fimg_bytes, (e - b) * (uint64_t)a.coop,
                                            a.coop > 1 ? -1 : inst),
                                block, s));
        HIPCHK(time_end(c, s, t0, t1, c->ev_bake));
        /* AccState: fold the (state, texel) counters into the int64 lightmap and zero them */
        if (a.counts)
            HIPCHK(fmgi_launch_reduce_states(a.counts, c->d_colfx, (unsigned long long *)lm, c->num_texels, s));
        HIPCHK(finish_call());
        return FMGI_OK;
    }
    /* STREAM: the codes of a chunk of work items are held in HBM (2 x 4 B per deposit, worst case 800
       deposits per item); chunks are memory-sized and fold after their bake on s.
       FMGI_PIPELINE=P > 1 (experiment) cuts the items into >= P chunks (every lane still tracing >= 4
       items per chunk) and folds chunk k on the context's fold stream while chunk k + 1 bakes into the
       other buffer set. Measured on box200 (profiles/r01/s36, s37): slower for every P, fold block size
       and bake occupancy tried, because the persistent bake leaves the folds no room to run beside it,
       so the default is 1. */
    const uint64_t n = e - b;
    const int lanes = grid_blocks(c, kernel, kacc, trace, block, a.fimg_bytes, UINT64_MAX) * block;
    int pipeline = 1;
    if (const char *pe = fmgi_exp_env("FMGI_PIPELINE")) pipeline = std::max(1, atoi(pe));
    const int smode = stream_layout(c); /* kStreamBuckets <=> kacc == kAccBucket */
    uint64_t chunk = stream_chunk_items(c, pipeline > 1 ? 2 : 1, smode);
    if (c->opt[FMGI_OPT_CHUNK_ITEMS] > 0) /* tests: force several chunks */
        chunk = std::min<uint64_t>(chunk, (uint64_t)c->opt[FMGI_OPT_CHUNK_ITEMS]);
    if (pipeline > 1) chunk = std::min<uint64_t>(chunk, std::max<uint64_t>((n + pipeline - 1) / pipeline, 4 * (uint64_t)lanes));
    chunk = std::max<uint64_t>(chunk, 1);
    const bool overlap = pipeline > 1 && chunk < n;
    if (overlap) {
        if (!c->fold_stream) HIPCHK(hipStreamCreateWithFlags(&c->fold_stream, hipStreamNonBlocking));
        for (int k = 0; k < 2; k++) {
            if (!c->ev_baked[k]) HIPCHK(hipEventCreateWithFlags(&c->ev_baked[k], hipEventDisableTiming));
            if (!c->ev_folded[k]) HIPCHK(hipEventCreateWithFlags(&c->ev_folded[k], hipEventDisableTiming));
        }
    }
    hipStream_t fs = overlap ? c->fold_stream : s;
    int nchunk = 0;
    /* Experiments (FMGI_TAIL=1 / 2 / 4 in the experiment build; measured and rejected): the
       launch tail of the layouts' hybrid scan handed to a second launch. A saving launch
       (FMGI_KERNEL_HYBRID_TAIL) polls the launch's idle-lane count; once half of its lanes found no item left,
       every lane still in one saves it at its next photon boundary (RNG state, photons left, source: 16 B) and
       leaves; a resuming launch (FMGI_KERNEL_HYBRID_RESUME) finishes the saved items with FMGI_TAIL lanes each
       splitting the wall-pair loop. Exact (the same photons, draws and hits per item), but on example.png half
       of the lanes are idle only once 97.6 % of the scans are done, and the resuming launch (3.5 ms) costs more
       than the tail it replaces (profiles/r06/s12). */
    int tail_coop = 0;
    if (const char *te = fmgi_exp_env("FMGI_TAIL")) tail_coop = atoi(te);
    const bool tail = kernel == FMGI_KERNEL_HYBRID && inst == FMGI_KERNEL_HYBRID && !trace && a.coop == 1 &&
                      (kacc == kAccScatter || kacc == kAccBucket) && (tail_coop == 1 || tail_coop == 2 || tail_coop == 4) &&
                      e - b <= 16 * (uint64_t)lanes;
    const int inst1 = tail ? FMGI_KERNEL_HYBRID_TAIL : inst;
    for (uint64_t cb = b; cb < e; cb += chunk, nchunk++) {
        const uint64_t ce = std::min(e, cb + chunk);
        const int k = overlap ? (nchunk & 1) : 0; /* one buffer set unless the folds run beside the bakes */
        int ring_tail = 0; /* (the saving launch's LDS: the workgroup's idle-count copy before the rings) */
        fmgi_bake_lds(inst1, kacc, block, a.fimg_bytes, &ring_tail);
        const int grid = grid_blocks(c, kernel, kacc, trace, block, a.fimg_bytes, (ce - cb) * (uint64_t)a.coop,
                                     a.coop > 1 ? -1 : inst1);
        const int grid2 = tail ? grid_blocks(c, kernel, kacc, trace, block, a.fimg_bytes, UINT64_MAX, FMGI_KERNEL_HYBRID_RESUME)
                               : 0; /* the resuming launch: every resident lane */
        /* buffer set k is free once the fold of chunk nchunk - 2 has read it (host allocation below
           happens only while growing, after a full wait) */
        if (overlap && nchunk >= 2) HIPCHK(hipStreamWaitEvent(s, c->ev_folded[k], 0));
        /* (the pool holds one partly filled block per wave and tile: the resuming launch's waves too) */
        if (ensure_stream_needs_growth(c, k, ce - cb, grid + grid2, block, smode)) { /* no fold may still read it */
            HIPCHK(hipStreamSynchronize(s));
            if (c->fold_stream) HIPCHK(hipStreamSynchronize(c->fold_stream));
        }
        const int tbits = tile_bits(c, smode, ce - cb);
        int rc = ensure_stream(c, k, ce - cb, grid + grid2, block, smode, tbits);
        if (rc != FMGI_OK) return rc;
        StreamBufs &sb = c->sb[k];
        a.item_begin = cb;
        a.item_end = ce;
        a.stream = sb.stream;
        a.stream_cap = sb.cap;
        a.stream_cursor = sb.cursor;
        a.presort = smode;
        a.ntiles = tiles_of(c, tbits);
        a.tile_shift = 10 + tbits;
        a.toff = sb.toff;
        a.colpack = (const uint4 *)c->d_colpack;
        if (smode == kStreamBuckets) {
            a.block_tile = sb.block_tile;
            a.block_len = sb.block_len;
            a.pool_cursor = sb.cursor;
            a.pool_blocks = sb.pool_blocks;
        }
        if (smode == kStreamDense) { /* the bake writes the dense stream; k_bin fills the pool */
            a.stream = sb.dense;
            a.stream_cap = sb.dense_cap;
            a.stream_cursor = sb.cursor + 1;
        }
        HIPCHK(fetch_table(cb, ce));
        HIPCHK(hipMemsetAsync(c->d_counter, 0, 8, s));
        HIPCHK(hipMemsetAsync(sb.cursor, 0, 16, s)); /* the pool / stream cursor and the dense stream's */
        hipEvent_t t0 = nullptr, t1 = nullptr;
        if (fmgi_exp_env("FMGI_SHOW_LAUNCH")) /* experiments: the launch shape the planner chose */
            fprintf(stderr, "fmgi: bake kernel %d accum %d block %d grid %d lds %zu (staged %d: rects %d srcs %d cells %d)\n",
                    a.coop > 1 ? kernel_instance(c, kernel) : inst, kacc, block, grid, fmgi_bake_lds(kernel_instance(c, kernel), kacc, block, a.fimg_bytes, nullptr),
                    a.fimg_bytes, a.rects_off, a.srcs_off, a.cells_off);
        HIPCHK(time_begin(c, s, t0));
        if (tail) {
            const uint64_t lanes1 = (uint64_t)grid * (uint64_t)block;
            if (c->tail_cap < lanes1) {
                HIPCHK(hipStreamSynchronize(s)); /* (no earlier launch may still use the old buffers) */
                hipFree(c->d_tail);
                c->d_tail = nullptr;
                c->tail_cap = 0;
                HIPCHK(hipMalloc(&c->d_tail, lanes1 * sizeof(uint4)));
                c->tail_cap = lanes1;
            }
            if (!c->d_tail_ctr) HIPCHK(hipMalloc(&c->d_tail_ctr, 4 * sizeof(unsigned)));
            HIPCHK(hipMemsetAsync(c->d_tail_ctr, 0, 4 * sizeof(unsigned), s));
            BakeArgs a1 = a;
            a1.tail_idle = c->d_tail_ctr;
            a1.tail_n = c->d_tail_ctr + 1;
            a1.tail_next = c->d_tail_ctr + 2;
            a1.tail_states = c->d_tail;
            a1.tail_at = (uint32_t)(lanes1 / 2); /* half of the lanes idle */
            if (const char *ta = fmgi_exp_env("FMGI_TAIL_AT")) /* experiments: idle lanes per mille (> 1000: never) */
                a1.tail_at = (uint32_t)std::min<uint64_t>(lanes1 * (uint64_t)atoi(ta) / 1000, 0xFFFFFFFFull);
            a1.ring_off = ring_tail;
            a1.tail_flag_off = ring_tail - 16;
            unsigned long long scans0 = 0, scans1 = 0; /* (experiments: the saving launch's share of the scans) */
            if (fmgi_exp_env("FMGI_SHOW_TAIL")) {
                HIPCHK(hipMemcpyAsync(&scans0, c->d_stats + KSTAT_SCANS, 8, hipMemcpyDeviceToHost, s));
                HIPCHK(hipStreamSynchronize(s));
            }
            HIPCHK(fmgi_launch_bake(a1, FMGI_KERNEL_HYBRID_TAIL, kacc, false, grid, block, s));
            if (fmgi_exp_env("FMGI_SHOW_TAIL")) {
                HIPCHK(hipMemcpyAsync(&scans1, c->d_stats + KSTAT_SCANS, 8, hipMemcpyDeviceToHost, s));
                HIPCHK(hipStreamSynchronize(s));
            }
            BakeArgs a2 = a1;
            a2.tail_at = 0;
            a2.coop = tail_coop;
            a2.fetch_tab = nullptr;
            a2.fetch_nseg = 0;
            fmgi_bake_lds(FMGI_KERNEL_HYBRID_RESUME, kacc, block, a.fimg_bytes, &a2.ring_off);
            HIPCHK(fmgi_launch_bake(a2, FMGI_KERNEL_HYBRID_RESUME, kacc, false, grid2, block, s));
            c->last_kernel = fmgi_bake_kernel_name(FMGI_KERNEL_HYBRID_TAIL, kacc, false) + " + " +
                             fmgi_bake_kernel_name(FMGI_KERNEL_HYBRID_RESUME, kacc, false);
            if (fmgi_exp_env("FMGI_SHOW_TAIL")) { /* experiments: idle lanes, states saved, states resumed */
                unsigned h[4] = {0, 0, 0, 0};
                unsigned long long scans2 = 0;
                HIPCHK(hipMemcpyAsync(h, c->d_tail_ctr, sizeof h, hipMemcpyDeviceToHost, s));
                HIPCHK(hipMemcpyAsync(&scans2, c->d_stats + KSTAT_SCANS, 8, hipMemcpyDeviceToHost, s));
                HIPCHK(hipStreamSynchronize(s));
                fprintf(stderr, "fmgi: tail lanes %llu grid2 %d idle %u saved %u resumed %u scans %llu + %llu\n",
                        (unsigned long long)lanes1, grid2, h[0], h[1], h[2], scans1 - scans0, scans2 - scans1);
            }
        } else {
            c->last_kernel = fmgi_bake_kernel_name(a.coop > 1 ? kernel_instance(c, kernel) : inst, kacc, trace);
            HIPCHK(fmgi_launch_bake(a, a.coop > 1 ? kernel_instance(c, kernel) : inst, kacc, trace, grid, block, s));
        }
        HIPCHK(time_end(c, s, t0, t1, c->ev_bake));
        if (overlap) {
            HIPCHK(hipEventRecord(c->ev_baked[k], s));
            HIPCHK(hipStreamWaitEvent(fs, c->ev_baked[k], 0));
        }
        HIPCHK(time_begin(c, fs, t0));
        HIPCHK(fmgi_stream_fold(sb, c->num_texels, (unsigned long long *)lm, fs));
        HIPCHK(time_end(c, fs, t0, t1, c->ev_fold));
        if (overlap) HIPCHK(hipEventRecord(c->ev_folded[k], fs));
    }
    if (overlap) { /* everything after this call on s sees the complete lightmap */
        HIPCHK(hipStreamWaitEvent(s, c->ev_folded[(nchunk - 1) & 1], 0));
    }
    HIPCHK(finish_call());
    return FMGI_OK;
}

FMGI_API int fmgi_auto_kernel(const fmgi_context *c) { return c ? c->auto_kernel : FMGI_ERR_ARG; }

FMGI_API int fmgi_last_bake_kernel(const fmgi_context *c, char *buf, int cap) {
    if (!c || (cap > 0 && !buf) || cap < 0) return set_err(FMGI_ERR_ARG, "fmgi_last_bake_kernel: bad arguments");
    const int n = (int)c->last_kernel.size();
    if (cap > 0) {
        const int k = n < cap - 1 ? n : cap - 1;
        memcpy(buf, c->last_kernel.data(), (size_t)k);
        buf[k] = 0;
    }
    return n;
}

FMGI_API int fmgi_set_timing(fmgi_context *c, int on) {
    if (!c) return set_err(FMGI_ERR_ARG, "null context");
    c->timing = on != 0;
    return FMGI_OK;
}

FMGI_API int fmgi_get_timing(fmgi_context *c, fmgi_timing *out) {
    if (!c || !out) return set_err(FMGI_ERR_ARG, "fmgi_get_timing: bad arguments");
    memset(out, 0, sizeof *out);
    if (c->device == FMGI_HOST_ONLY) return FMGI_OK;
    HIPCHK(hipSetDevice(c->device));
    auto drain = [&](std::vector<std::pair<hipEvent_t, hipEvent_t>> &v, double &ms, uint64_t &n) -> hipError_t {
        for (auto &p : v) {
            hipError_t e = hipEventSynchronize(p.second);
            if (e != hipSuccess) return e;
            float t = 0;
            e = hipEventElapsedTime(&t, p.first, p.second);
            if (e != hipSuccess) return e;
            ms += t;
            n++;
            c->ev_pool.push_back(p.first);
            c->ev_pool.push_back(p.second);
        }
        v.clear();
        return hipSuccess;
    };
    HIPCHK(drain(c->ev_bake, out->bake_ms, out->bake_launches));
    HIPCHK(drain(c->ev_fold, out->fold_ms, out->fold_launches));
    return FMGI_OK;
}

FMGI_API int fmgi_bake_items(fmgi_context *c, uint64_t item_begin, uint64_t item_end, void *lm_fx_dev, int kernel,
                             void *stream) {
    if (!c) return set_err(FMGI_ERR_ARG, "null context");
    return bake_common(c, item_begin, item_end, lm_fx_dev, kernel, stream ? (hipStream_t)stream : c->stream, false,
                       nullptr, nullptr, nullptr);
}

FMGI_API int fmgi_finalize(fmgi_context *c, const void *lm, const void *tin, void *tout, void *stream) {
    if (!c || !lm || !tin || !tout) return set_err(FMGI_ERR_ARG, "fmgi_finalize: bad arguments");
    if (c->device == FMGI_HOST_ONLY) return set_err(FMGI_ERR_NO_DEVICE, "host-only context");
    HIPCHK(hipSetDevice(c->device));
    HIPCHK(fmgi_launch_finalize((const unsigned long long *)lm, (const float *)tin, (float *)tout, c->num_texels,
                                stream ? (hipStream_t)stream : c->stream));
    return FMGI_OK;
}

FMGI_API int fmgi_get_stage_cycles(fmgi_context *c, uint64_t out[16]) {
    if (!c || !out) return set_err(FMGI_ERR_ARG, "fmgi_get_stage_cycles: bad arguments");
    if (c->device == FMGI_HOST_ONLY) return set_err(FMGI_ERR_NO_DEVICE, "host-only context");
    HIPCHK(hipSetDevice(c->device));
    HIPCHK(hipDeviceSynchronize());
    unsigned long long v[KSTAT_ALLOC];
    HIPCHK(hipMemcpy(v, c->d_stats, sizeof v, hipMemcpyDeviceToHost));
    for (int k = 0; k < 16; k++) out[k] = v[KSTAT_STAGE0 + k];
    return FMGI_OK;
}

FMGI_API int fmgi_grid_sizes(const fmgi_context *c, int32_t sizes[5]) {
    if (!c || !sizes) return set_err(FMGI_ERR_ARG, "fmgi_grid_sizes: bad arguments");
    for (int a = 0; a < 3; a++) sizes[a] = c->h_grid.J[a];
    sizes[3] = (int32_t)c->h_grid.cells.size();
    sizes[4] = (int32_t)c->h_grid.idx.size();
    return FMGI_OK;
}

FMGI_API int fmgi_pairs_copy(const fmgi_context *c, void *img, int32_t *bytes, int32_t groups[2]) {
    if (!c || !bytes || !groups) return set_err(FMGI_ERR_ARG, "fmgi_pairs_copy: bad arguments");
    const int32_t n = (int32_t)(c->h_pairs.size() * sizeof(FilterPairHalf));
    if (img && *bytes < n) return set_err(FMGI_ERR_ARG, "fmgi_pairs_copy: buffer too small");
    if (img && n) memcpy(img, c->h_pairs.data(), (size_t)n);
    *bytes = n;
    groups[0] = c->pG[0];
    groups[1] = c->pG[1];
    return FMGI_OK;
}

FMGI_API int fmgi_filter_copy(const fmgi_context *c, void *img, int32_t *bytes, int32_t pairs[3]) {
    if (!c || !bytes || !pairs) return set_err(FMGI_ERR_ARG, "fmgi_filter_copy: bad arguments");
    const int32_t n = (int32_t)(c->h_fimg.size() * sizeof(FilterRec));
    if (img && *bytes < n) return set_err(FMGI_ERR_ARG, "fmgi_filter_copy: buffer too small");
    if (img && n) memcpy(img, c->h_fimg.data(), (size_t)n);
    *bytes = n;
    for (int a = 0; a < 3; a++) pairs[a] = c->fJ[a];
    return FMGI_OK;
}

FMGI_API int fmgi_plan_copy(const fmgi_context *c, void *blob, int32_t *bytes) {
    if (!c || !bytes) return set_err(FMGI_ERR_ARG, "fmgi_plan_copy: bad arguments");
    const std::vector<char> b = c->h_plan.ok ? c->h_plan.blob() : std::vector<char>();
    if (blob && *bytes < (int32_t)b.size()) return set_err(FMGI_ERR_ARG, "fmgi_plan_copy: buffer too small");
    if (blob && !b.empty()) memcpy(blob, b.data(), b.size());
    *bytes = (int32_t)b.size();
    return FMGI_OK;
}

FMGI_API int fmgi_grid_copy(const fmgi_context *c, void *planes, void *cells, float *recs, int32_t *idx) {
    if (!c) return set_err(FMGI_ERR_ARG, "fmgi_grid_copy: null context");
    const GridBuild &g = c->h_grid;
    if (planes) memcpy(planes, g.img.data(), g.img.size() * sizeof(GridPlane));
    if (cells) memcpy(cells, g.cells.data(), g.cells.size() * sizeof(GridCell));
    if (recs) memcpy(recs, g.recs.data(), g.recs.size() * sizeof(float));
    if (idx) memcpy(idx, g.idx.data(), g.idx.size() * sizeof(int32_t));
    return FMGI_OK;
}

FMGI_API int fmgi_get_stats(fmgi_context *c, fmgi_stats *out) {
    if (!c || !out) return set_err(FMGI_ERR_ARG, "bad arguments");
    if (c->device == FMGI_HOST_ONLY) return set_err(FMGI_ERR_NO_DEVICE, "host-only context");
    HIPCHK(hipSetDevice(c->device));
    HIPCHK(hipDeviceSynchronize());
    unsigned long long v[KSTAT_ALLOC];
    HIPCHK(hipMemcpy(v, c->d_stats, sizeof v, hipMemcpyDeviceToHost));
    memset(out, 0, sizeof *out);
    out->photons = v[KSTAT_PHOTONS];
    out->scans = v[KSTAT_SCANS];
    out->deposits = v[KSTAT_DEPOSITS];
    out->escapes = v[KSTAT_ESCAPES];
    out->exact_rescans = v[KSTAT_RESCANS];
    out->tests = v[KSTAT_TESTS];
    out->rescans_tie = v[KSTAT_TIES];
    out->rescans_invalid = v[KSTAT_INVALID];
    out->stream_overflow = v[KSTAT_OVERFLOW];
    return FMGI_OK;
}

FMGI_API int fmgi_reset_stats(fmgi_context *c) {
    if (!c) return set_err(FMGI_ERR_ARG, "null context");
    if (c->device == FMGI_HOST_ONLY) return set_err(FMGI_ERR_NO_DEVICE, "host-only context");
    HIPCHK(hipSetDevice(c->device));
    HIPCHK(hipDeviceSynchronize());
    HIPCHK(hipMemset(c->d_stats, 0, KSTAT_ALLOC * sizeof(unsigned long long)));
    return FMGI_OK;
}

FMGI_API int fmgi_trace_items(fmgi_context *c, uint64_t b, uint64_t e, int kernel, fmgi_event *events,
                              int32_t *counts, uint32_t *rng_final) {
    if (!c || !events || !counts || !rng_final || e < b || e - b > 4096)
        return set_err(FMGI_ERR_ARG, "fmgi_trace_items: bad arguments");
    if (c->device == FMGI_HOST_ONLY) return set_err(FMGI_ERR_NO_DEVICE, "host-only context");
    uint64_t n = e - b;
    if (!n) return FMGI_OK;
    HIPCHK(hipSetDevice(c->device));
    void *d_ev = nullptr, *d_cnt = nullptr, *d_rng = nullptr, *d_lm = nullptr;
    size_t ev_bytes = (size_t)n * FMGI_EVENTS_PER_ITEM * sizeof(fmgi_event);
    size_t lm_bytes = (size_t)c->num_texels * 4 * sizeof(unsigned long long);
    int rc = FMGI_OK;
    if (hipMalloc(&d_ev, ev_bytes) != hipSuccess || hipMalloc(&d_cnt, n * 4) != hipSuccess ||
        hipMalloc(&d_rng, n * 4) != hipSuccess || hipMalloc(&d_lm, lm_bytes ? lm_bytes : 32) != hipSuccess) {
        rc = set_err(FMGI_ERR_OOM, "trace buffers");
    } else {
        hipMemset(d_lm, 0, lm_bytes ? lm_bytes : 32);
        hipMemset(d_cnt, 0, n * 4);
        rc = bake_common(c, b, e, d_lm, kernel, c->stream, true, d_ev, (int32_t *)d_cnt, (uint32_t *)d_rng);
        if (rc == FMGI_OK) {
            hipError_t err = hipStreamSynchronize(c->stream);
            if (err == hipSuccess) err = hipMemcpy(events, d_ev, ev_bytes, hipMemcpyDeviceToHost);
            if (err == hipSuccess) err = hipMemcpy(counts, d_cnt, n * 4, hipMemcpyDeviceToHost);
            if (err == hipSuccess) err = hipMemcpy(rng_final, d_rng, n * 4, hipMemcpyDeviceToHost);
            if (err != hipSuccess) rc = set_err(FMGI_ERR_HIP, "trace: %s", hipGetErrorString(err));
        }
    }
    hipFree(d_ev);
    hipFree(d_cnt);
    hipFree(d_rng);
    hipFree(d_lm);
    return rc;
}

static int device_sincos(fmgi_context *c, const float *x, float *s, float *co, int64_t n, int lib) {
    if (!c || n < 0) return set_err(FMGI_ERR_ARG, "bad arguments");
    if (c->device == FMGI_HOST_ONLY) return set_err(FMGI_ERR_NO_DEVICE, "host-only context");
    if (!n) return FMGI_OK;
    HIPCHK(hipSetDevice(c->device));
    float *d = nullptr;
    HIPCHK(hipMalloc(&d, (size_t)n * 12));
    hipError_t err = hipMemcpy(d, x, (size_t)n * 4, hipMemcpyHostToDevice);
    if (err == hipSuccess) err = fmgi_launch_sincos(d, d + n, d + 2 * n, n, lib, c->stream);
    if (err == hipSuccess) err = hipStreamSynchronize(c->stream);
    if (err == hipSuccess) err = hipMemcpy(s, d + n, (size_t)n * 4, hipMemcpyDeviceToHost);
    if (err == hipSuccess) err = hipMemcpy(co, d + 2 * n, (size_t)n * 4, hipMemcpyDeviceToHost);
    hipFree(d);
    if (err != hipSuccess) return set_err(FMGI_ERR_HIP, "device sincos: %s", hipGetErrorString(err));
    return FMGI_OK;
}

FMGI_API int fmgi_device_sincosf(fmgi_context *c, const float *x, float *s, float *co, int64_t n) {
    return device_sincos(c, x, s, co, n, 0);
}

FMGI_API int fmgi_device_sincosf_library(fmgi_context *c, const float *x, float *s, float *co, int64_t n) {
    return device_sincos(c, x, s, co, n, 1);
}

FMGI_API int fmgi_device_unit(fmgi_context *c, int op, const float *a, const float *b, int32_t *out, int64_t n) {
    if (!c || n < 0 || !a || !out || (op != FMGI_UNIT_SQRT && !b) ||
        (op != FMGI_UNIT_SQRT && op != FMGI_UNIT_TRUNC_DIV && op != FMGI_UNIT_TRUNC_DIV_INV))
        return set_err(FMGI_ERR_ARG, "bad arguments");
    if (c->device == FMGI_HOST_ONLY) return set_err(FMGI_ERR_NO_DEVICE, "host-only context");
    if (!n) return FMGI_OK;
    HIPCHK(hipSetDevice(c->device));
    float *d = nullptr;
    HIPCHK(hipMalloc(&d, (size_t)n * 12));
    hipError_t err = hipMemcpy(d, a, (size_t)n * 4, hipMemcpyHostToDevice);
    if (err == hipSuccess && b) err = hipMemcpy(d + n, b, (size_t)n * 4, hipMemcpyHostToDevice);
    if (err == hipSuccess) err = fmgi_launch_unit(op, d, d + n, (int32_t *)(d + 2 * n), n, c->stream);
    if (err == hipSuccess) err = hipStreamSynchronize(c->stream);
    if (err == hipSuccess) err = hipMemcpy(out, d + 2 * n, (size_t)n * 4, hipMemcpyDeviceToHost);
    hipFree(d);
    if (err != hipSuccess) return set_err(FMGI_ERR_HIP, "device unit: %s", hipGetErrorString(err));
    return FMGI_OK;
}

/* ---- the drop-in entry points ----------------------------------------------------------------- */

/*
 * libc rand() is part of the drop-in contract (global_illumination_cl.c:251: one call per launch, and
 * the caller sees exactly those calls). The HIP runtime's first device initialisation in a process
 * draws from the same generator (observed on ROCm 7: one call inside the first hipStreamCreate /
 * allocation). So the schedule is built, with its rand() calls, before any HIP call, and the state is
 * snapshotted then and restored after the device work. glibc keeps the state of random_r's TYPE_n
 * generator in the caller's array: a header word (MAX_TYPES * rear + type, just the type for TYPE_0)
 * followed by the degree-n table; setstate() re-reads everything from there. The guard saves and
 * restores exactly that many bytes for the type the header names.
 */
struct RandGuard {
    char *state = nullptr;
    size_t bytes = 0;
    char saved[4 * 64];
    bool ok = false;
    void save() {
#ifdef __GLIBC__
        static char scratch[128];
        state = initstate(1, scratch, sizeof scratch); /* records the position in state[0], switches away */
        if (!state) return;
        int32_t hdr;
        memcpy(&hdr, state, 4);
        static const int kDegree[5] = {0, 7, 15, 31, 63}; /* TYPE_0 .. TYPE_4 (glibc random_r.c) */
        const int type = hdr % 5;
        if (hdr < 0 || type < 0 || type > 4) { /* not a header glibc wrote: leave the state alone */
            setstate(state);
            return;
        }
        bytes = (size_t)4 * (std::max(kDegree[type], 1) + 1); /* header + table (TYPE_0: one LCG word) */
        memcpy(saved, state, bytes);
        setstate(state); /* back to the caller's array and position */
        ok = true;
#endif
    }
    void restore() {
#ifdef __GLIBC__
        if (!ok) return;
        static char scratch2[128];
        initstate(1, scratch2, sizeof scratch2); /* leave the caller's array (its header is rewritten) */
        memcpy(state, saved, bytes);
        setstate(state);
#endif
    }
};

/*
 * The drop-in's device state, cached across calls: per shard a context (scene tables, launch schedule,
 * stream buffers) and its lightmap buffers, keyed by a hash of the geometry, so a repeated call on the
 * same scene uploads nothing but the schedule and the caller's texels (the reference rebuilds its
 * OpenCL context on every call, global_illumination_cl.c:279-286; nothing here requires that).
 * fmgi_dropin_release() frees it; FMGI_DROPIN_CACHE=0 frees it after every call.
 */
struct DropinShard {
    fmgi_context *ctx = nullptr;
    uint64_t scene_hash = 0;
    void *lm = nullptr;    /* int64 [numTexels][4] */
    void *stage = nullptr; /* a peer shard's lightmap during the reduction */
    size_t lm_bytes = 0, stage_bytes = 0;
    hipEvent_t done = nullptr;
};
static std::mutex g_dropin_mu;
static std::vector<DropinShard> g_dropin;
static void *g_dropin_tex = nullptr;
static size_t g_dropin_tex_bytes = 0;
static int g_dropin_tex_dev = -1;
static bool g_peer_on[64][64];

static void dropin_release_shard(DropinShard &S) {
    if (S.ctx && hipSetDevice(S.ctx->device) == hipSuccess) {
        (void)hipStreamSynchronize(S.ctx->stream);
        (void)hipFree(S.lm);
        (void)hipFree(S.stage);
        if (S.done) (void)hipEventDestroy(S.done);
    }
    fmgi_destroy(S.ctx);
    S = DropinShard{};
}

/* the host-only context that plans the reference schedule (its scene set once per geometry) */
static fmgi_context *g_plan_ctx = nullptr;
static uint64_t g_plan_hash = 0;

static void rccl_release();

static void dropin_release_locked() {
    rccl_release();
    fmgi_destroy(g_plan_ctx);
    g_plan_ctx = nullptr;
    g_plan_hash = 0;
    for (DropinShard &S : g_dropin) dropin_release_shard(S);
    g_dropin.clear();
    if (g_dropin_tex && hipSetDevice(g_dropin_tex_dev) == hipSuccess) (void)hipFree(g_dropin_tex);
    g_dropin_tex = nullptr;
    g_dropin_tex_bytes = 0;
    g_dropin_tex_dev = -1;
}

FMGI_API void fmgi_dropin_release(void) {
    std::lock_guard<std::mutex> lk(g_dropin_mu);
    dropin_release_locked();
}

/* FNV-1a over the geometry the bake reads (walls, windows, lights, numTexels) */
static uint64_t geometry_hash(const fmgi_geometry *geo) {
    uint64_t h = 1469598103934665603ull;
    auto mix = [&](const void *p, size_t n) {
        const unsigned char *b = (const unsigned char *)p;
        for (size_t i = 0; i < n; i++) h = (h ^ b[i]) * 1099511628211ull;
    };
    const int32_t counts[4] = {geo->numWalls, geo->numWindows, geo->numLights, geo->numTexels};
    mix(counts, sizeof counts);
    if (geo->numWalls > 0) mix(geo->walls, sizeof(fmgi_rect) * (size_t)geo->numWalls);
    if (geo->numWindows > 0) mix(geo->windows, sizeof(fmgi_rect) * (size_t)geo->numWindows);
    if (geo->numLights > 0) mix(geo->lights, sizeof(fmgi_rect) * (size_t)geo->numLights);
    return h | 1; /* 0 = "no scene" */
}

/* peer access dev -> peer (xGMI), once per pair; false if the pair cannot (copies then stage as HIP does) */
static void enable_peer(int dev, int peer) {
    if (dev == peer || dev >= 64 || peer >= 64 || g_peer_on[dev][peer]) return;
    int can = 0;
    if (hipDeviceCanAccessPeer(&can, dev, peer) == hipSuccess && can && hipSetDevice(dev) == hipSuccess) {
        const hipError_t e = hipDeviceEnablePeerAccess(peer, 0);
        if (e == hipSuccess || e == hipErrorPeerAccessAlreadyEnabled) g_peer_on[dev][peer] = true;
        (void)hipGetLastError(); /* an "already enabled" must not linger as the thread's last error */
    }
}

/*
 * RCCL for the drop-in's one-process multi-GPU reduce (ncclCommInitAll over the shard devices,
 * one ncclReduce of the int64 lightmaps to shard 0 over xGMI). librccl is opened on the first call that
 * reduces through it, so single-GPU callers of the library never load it (releasing with no communicator
 * does not open it either); the communicators are cached with the shards (fmgi_dropin_release destroys
 * them). When librccl cannot be loaded or ncclCommInitAll fails and FMGI_REDUCE=rccl was not set, the call
 * reduces by xGMI peer copies instead (the same integer sums, so the same bits).
 */
struct RcclApi {
    void *h = nullptr;
    decltype(&ncclCommInitAll) comm_init_all = nullptr;
    decltype(&ncclCommDestroy) comm_destroy = nullptr;
    decltype(&ncclCommCount) comm_count = nullptr;
    decltype(&ncclReduce) reduce = nullptr;
    decltype(&ncclGroupStart) group_start = nullptr;
    decltype(&ncclGroupEnd) group_end = nullptr;
    decltype(&ncclGetErrorString) error_string = nullptr;
};

static const RcclApi *rccl_api() {
    static RcclApi api;
    static bool tried = false;
    if (!tried) {
        tried = true;
        void *h = dlopen("librccl.so.1", RTLD_NOW | RTLD_LOCAL);
        if (!h) h = dlopen("librccl.so", RTLD_NOW | RTLD_LOCAL);
        if (h) {
            api.comm_init_all = (decltype(api.comm_init_all))dlsym(h, "ncclCommInitAll");
            api.comm_destroy = (decltype(api.comm_destroy))dlsym(h, "ncclCommDestroy");
            api.comm_count = (decltype(api.comm_count))dlsym(h, "ncclCommCount");
            api.reduce = (decltype(api.reduce))dlsym(h, "ncclReduce");
            api.group_start = (decltype(api.group_start))dlsym(h, "ncclGroupStart");
            api.group_end = (decltype(api.group_end))dlsym(h, "ncclGroupEnd");
            api.error_string = (decltype(api.error_string))dlsym(h, "ncclGetErrorString");
            if (api.comm_init_all && api.comm_destroy && api.comm_count && api.reduce && api.group_start &&
                api.group_end && api.error_string)
                api.h = h;
        }
    }
    return api.h ? &api : nullptr;
}

static std::vector<ncclComm_t> g_rccl_comms; /* one per shard, over the shard devices in shard order */
static std::vector<int> g_rccl_devs;
static bool g_rccl_last = false; /* whether the last drop-in call reduced through RCCL */

static void rccl_release() {
    if (!g_rccl_comms.empty()) { /* comms exist only once librccl was loaded: no dlopen otherwise */
        const RcclApi *R = rccl_api();
        if (R)
            for (ncclComm_t cm : g_rccl_comms) (void)R->comm_destroy(cm);
    }
    g_rccl_comms.clear();
    g_rccl_devs.clear();
    g_rccl_last = false;
}

/* communicators over `devs` (distinct devices; rank k = shard k), created once per device list */
static int rccl_comms(const std::vector<int> &devs) {
    if (g_rccl_devs == devs && g_rccl_comms.size() == devs.size()) return FMGI_OK;
    rccl_release();
    const RcclApi *R = rccl_api();
    if (!R) return set_err(FMGI_ERR_HIP, "librccl could not be loaded (FMGI_REDUCE=peer reduces by xGMI peer copies)");
    std::vector<ncclComm_t> cm(devs.size());
    const ncclResult_t r = R->comm_init_all(cm.data(), (int)devs.size(), devs.data());
    if (r != ncclSuccess) return set_err(FMGI_ERR_HIP, "ncclCommInitAll over %zu devices: %s", devs.size(), R->error_string(r));
    g_rccl_comms = cm;
    g_rccl_devs = devs;
    return FMGI_OK;
}

/* ranks of the communicator the last drop-in call reduced through (ncclCommCount of rank 0's), 0 if that
   call did not reduce through RCCL */
FMGI_API int fmgi_dropin_rccl_ranks(void) {
    if (!g_rccl_last || g_rccl_comms.empty()) return 0;
    const RcclApi *R = rccl_api();
    int n = 0;
    if (!R || R->comm_count(g_rccl_comms[0], &n) != ncclSuccess) return 0;
    return n;
}

/* the stream-accumulation overflow flag of a context's bakes since its reset (never set by sizing; a set
   flag means dropped deposits, so the call fails instead of returning a wrong lightmap) */
static int check_no_overflow(fmgi_context *c) {
    unsigned long long v = 0;
    HIPCHK(hipSetDevice(c->device));
    HIPCHK(hipMemcpy(&v, c->d_stats + KSTAT_OVERFLOW, sizeof v, hipMemcpyDeviceToHost));
    if (v) return set_err(FMGI_ERR_STATE, "stream accumulation overflowed (%llu blocks dropped)", v);
    return FMGI_OK;
}

/* The drop-in's shard layout: shard k runs on device k % ngpu over the contiguous work items
   [items * k / nshard, items * (k + 1) / nshard). */
FMGI_API int fmgi_dropin_shards(uint64_t items, int ngpu, int nshard, int32_t *dev, uint64_t *begin, uint64_t *end) {
    if (ngpu < 1 || nshard < 1 || !dev || !begin || !end) return set_err(FMGI_ERR_ARG, "fmgi_dropin_shards: bad arguments");
    for (int k = 0; k < nshard; k++) {
        dev[k] = k % ngpu;
        begin[k] = items * (uint64_t)k / (uint64_t)nshard;
        end[k] = items * (uint64_t)(k + 1) / (uint64_t)nshard;
    }
    return FMGI_OK;
}

/* ... and its reduction: a binary tree into shard 0; step i adds shard src[i] into shard dst[i], and the
   steps of one round (distance d) are independent. Returns the number of steps (nshard - 1). */
FMGI_API int fmgi_dropin_reduce_order(int nshard, int32_t *dst, int32_t *src) {
    if (nshard < 1 || (nshard > 1 && (!dst || !src))) return set_err(FMGI_ERR_ARG, "fmgi_dropin_reduce_order: bad arguments");
    int n = 0;
    for (int d = 1; d < nshard; d *= 2)
        for (int k = 0; k + d < nshard; k += 2 * d) {
            dst[n] = k;
            src[n] = k + d;
            n++;
        }
    return n;
}

/*
 * One bake of a reference Geometry, sharded over FMGI_GPUS devices of the node (default 1, the
 * reference's one device; at most 8). The reference launch schedule is built once (libc rand() consumed
 * exactly as the reference does, global_illumination_cl.c:251) and its flattened work items are split
 * into equal contiguous shards, one per GPU, prepared and launched concurrently (a host thread per
 * shard); each GPU accumulates its own exact int64 lightmap, and the shards are summed into shard 0 by one
 * RCCL reduce over the shard devices (default with one shard per device) or by a binary tree of xGMI peer
 * copies (FMGI_REDUCE=peer, shards sharing a device, or RCCL unavailable); integer sums are bit-identical
 * for any GPU count and either reduce. FMGI_SHARDS (tests) splits into more shards than GPUs, round-robin,
 * to exercise the reduction on a single device.
 */
static int bake_geometry_devices(const fmgi_geometry *geo, int spa, int wg, int kernel,
                                 const std::vector<int32_t> &offs, uint64_t items, fmgi_vec3 *texels_out,
                                 bool verbose);

/* photonMapLightSource's progress line before each launch, with the samples (work items) still to launch
   for that source, and a newline after each source (global_illumination_cl.c:248-249, :267): the same
   bytes the reference writes, printed once the launches are queued */
static void print_launch_progress(const std::vector<LaunchDev> &launches) {
    for (size_t i = 0; i < launches.size();) {
        size_t j = i;
        uint64_t left = 0;
        while (j < launches.size() && launches[j].source == launches[i].source) left += launches[j++].count;
        for (size_t k = i; k < j; k++) {
            printf("\rphoton-mapping window with %d M samples   ", (int)(left * 100 / 1000000));
            left -= launches[k].count;
        }
        printf("\n");
        i = j;
    }
}

static int bake_geometry(const fmgi_geometry *geo, int spa, fmgi_vec3 *texels_out, bool verbose) {
    if (!geo) return set_err(FMGI_ERR_ARG, "null geometry");
    const char *wg_env = getenv("FMGI_WG");
    int wg = wg_env ? atoi(wg_env) : 256;
    if (wg <= 0) wg = 256;
    const char *k_env = getenv("FMGI_KERNEL");
    int kernel = FMGI_KERNEL_AUTO;
    if (k_env && !strcmp(k_env, "grid")) kernel = FMGI_KERNEL_GRID;
    if (k_env && !strcmp(k_env, "exact")) kernel = FMGI_KERNEL_EXACT;
    if (k_env && !strcmp(k_env, "fast")) kernel = FMGI_KERNEL_FAST;
    if (k_env && !strcmp(k_env, "hybrid")) kernel = FMGI_KERNEL_HYBRID;
    /* the reference schedule and its rand() calls first, before the HIP runtime can draw from rand() */
    std::vector<int32_t> offs;
    uint64_t items = 0;
    int64_t nl = 0;
    std::lock_guard<std::mutex> lk(g_dropin_mu);
    {   /* the planning context and its scene are kept across calls per geometry, like the shards' */
        const uint64_t hash = geometry_hash(geo);
        if (!g_plan_ctx || g_plan_hash != hash) {
            fmgi_destroy(g_plan_ctx);
            g_plan_hash = 0;
            g_plan_ctx = fmgi_create(FMGI_HOST_ONLY);
            if (!g_plan_ctx) return set_err(FMGI_ERR_OOM, "planning context");
            const int rc0 = fmgi_set_scene(g_plan_ctx, geo->walls, geo->numWalls, geo->windows, geo->numWindows,
                                           geo->lights, geo->numLights, geo->numTexels);
            if (rc0 != FMGI_OK) {
                fmgi_destroy(g_plan_ctx);
                g_plan_ctx = nullptr;
                return rc0;
            }
            g_plan_hash = hash;
        }
        nl = fmgi_plan(g_plan_ctx, spa, wg, nullptr, 0, &items);
        if (nl < 0) return (int)nl;
        for (const LaunchDev &L : g_plan_ctx->h_launches) offs.push_back(L.rng_offset);
    }
    RandGuard guard;
    guard.save();
    int rc_all;
    {
        rc_all = bake_geometry_devices(geo, spa, wg, kernel, offs, items, texels_out, verbose);
        /* FMGI_DROPIN_CACHE: 0 = free all device state after the call (the reference's behaviour,
           global_illumination_cl.c:315-320); 1 (default) = keep the per-geometry state (contexts, scene
           tables, lightmaps: a few MB per shard) but free the deposit-code stream buffers, which are
           sized to the call's photon count (tens of GB at 1e9 photons); 2 = keep everything (repeated
           bakes of large photon counts in one process) */
        const char *ce = getenv("FMGI_DROPIN_CACHE");
        const int cache = ce ? atoi(ce) : 1;
        if (rc_all != FMGI_OK || cache <= 0) {
            dropin_release_locked();
        } else if (cache == 1) {
            for (DropinShard &S : g_dropin)
                if (S.ctx) release_stream_buffers(S.ctx);
        }
    }
    guard.restore();
    return rc_all;
}

static int bake_geometry_devices(const fmgi_geometry *geo, int spa, int wg, int kernel, const std::vector<int32_t> &offs,
                                 uint64_t items, fmgi_vec3 *texels_out, bool verbose) {
    int ndev = fmgi_device_count();
    if (ndev <= 0) return set_err(FMGI_ERR_NO_DEVICE, "no HIP device visible");
    const char *g_env = getenv("FMGI_GPUS");
    int ngpu = g_env ? atoi(g_env) : 1;
    ngpu = std::max(1, std::min(std::min(ngpu, ndev), 8));
    const char *s_env = getenv("FMGI_SHARDS");
    const int nshard = s_env ? std::max(1, std::min(atoi(s_env), 64)) : ngpu;
    const uint64_t hash = geometry_hash(geo);
    const size_t tb = (size_t)geo->numTexels * 16, lmb = 2 * tb; /* float4 texels, int64 x 4 lightmap */
    if ((int)g_dropin.size() > nshard) { /* fewer shards than the cached call: drop the extra ones */
        for (size_t k = (size_t)nshard; k < g_dropin.size(); k++) dropin_release_shard(g_dropin[k]);
        g_dropin.resize((size_t)nshard);
    }
    g_dropin.resize((size_t)nshard);

    std::vector<int32_t> sdev((size_t)nshard);
    std::vector<uint64_t> sbeg((size_t)nshard), send((size_t)nshard);
    fmgi_dropin_shards(items, ngpu, nshard, sdev.data(), sbeg.data(), send.data());
    /* per shard: context (cached), scene (if changed), schedule, lightmap buffers, bake launch */
    auto prepare_and_launch = [&](int k, std::string &err) -> int {
        DropinShard &S = g_dropin[(size_t)k];
        const int dev = sdev[(size_t)k];
        if (S.ctx && S.ctx->device != dev) dropin_release_shard(S);
        if (!S.ctx) {
            S.ctx = fmgi_create(dev);
            if (!S.ctx) { err = fmgi_last_error(); return FMGI_ERR_HIP; }
        }
        fmgi_context *c = S.ctx;
        int rc = FMGI_OK;
        if (S.scene_hash != hash) {
            S.scene_hash = 0;
            rc = fmgi_set_scene(c, geo->walls, geo->numWalls, geo->windows, geo->numWindows, geo->lights,
                                geo->numLights, geo->numTexels);
            if (rc != FMGI_OK) { err = fmgi_last_error(); return rc; }
            S.scene_hash = hash;
        }
        /* every shard replays the schedule planned above (the rand() values in offs) */
        const int64_t nl = fmgi_plan(c, spa, wg, offs.data(), (int64_t)offs.size(), nullptr);
        if (nl < 0) { err = fmgi_last_error(); return (int)nl; }
        if (geo->numTexels <= 0) return FMGI_OK;
        hipError_t e = hipSetDevice(dev);
        if (e == hipSuccess && S.lm_bytes < lmb) {
            (void)hipFree(S.lm);
            S.lm = nullptr;
            S.lm_bytes = 0;
            e = hipMalloc(&S.lm, lmb);
            if (e == hipSuccess) S.lm_bytes = lmb;
        }
        if (e == hipSuccess && nshard > 1 && S.stage_bytes < lmb) {
            (void)hipFree(S.stage);
            S.stage = nullptr;
            S.stage_bytes = 0;
            e = hipMalloc(&S.stage, lmb);
            if (e == hipSuccess) S.stage_bytes = lmb;
        }
        if (e == hipSuccess && !S.done) e = hipEventCreateWithFlags(&S.done, hipEventDisableTiming);
        if (e == hipSuccess) e = hipMemsetAsync(S.lm, 0, lmb, c->stream);
        if (e == hipSuccess) e = hipMemsetAsync(c->d_stats + KSTAT_OVERFLOW, 0, sizeof(unsigned long long), c->stream);
        if (e != hipSuccess) {
            err = std::string("shard buffers on device ") + std::to_string(dev) + ": " + hipGetErrorString(e);
            return FMGI_ERR_OOM;
        }
        rc = fmgi_bake_items(c, sbeg[(size_t)k], send[(size_t)k], S.lm, kernel, c->stream);
        if (rc == FMGI_OK && hipEventRecord(S.done, c->stream) != hipSuccess) rc = set_err(FMGI_ERR_HIP, "event");
        if (rc != FMGI_OK) err = fmgi_last_error();
        return rc;
    };
    std::vector<int> rcs((size_t)nshard, FMGI_OK);
    std::vector<std::string> errs((size_t)nshard);
    if (nshard == 1) {
        rcs[0] = prepare_and_launch(0, errs[0]);
    } else { /* shards set up and launch concurrently, one host thread each */
        std::vector<std::thread> th;
        for (int k = 0; k < nshard; k++) th.emplace_back([&, k] { rcs[(size_t)k] = prepare_and_launch(k, errs[(size_t)k]); });
        for (std::thread &t : th) t.join();
    }
    for (int k = 0; k < nshard; k++)
        if (rcs[(size_t)k] != FMGI_OK) return set_err(rcs[(size_t)k], "shard %d: %s", k, errs[(size_t)k].c_str());
    DropinShard &S0 = g_dropin[0];
    if (verbose) { /* the reference's console output (global_illumination_cl.c:59, :248-249, :267) */
        hipDeviceProp_t prop;
        if (hipGetDeviceProperties(&prop, S0.ctx->device) != hipSuccess) prop.name[0] = 0;
        if (ngpu > 1) printf("[INF] Selected device '%s' (x%d)\n\n", prop.name, ngpu);
        else printf("[INF] Selected device '%s'\n\n", prop.name);
        print_launch_progress(S0.ctx->h_launches);
        fflush(stdout);
    }
    if (geo->numTexels <= 0) return FMGI_OK;
    /* the shards' lightmaps summed into shard 0: one RCCL reduce over the shard devices (default when every
       shard has a device of its own), or a binary tree of xGMI peer copies + adds (FMGI_REDUCE=peer, and
       shards sharing a device: RCCL allows one rank per GPU). FMGI_REDUCE=rccl forces RCCL, also for a
       single shard (a one-rank communicator: the in-place reduce leaves the lightmap as it is). */
    const char *r_env = getenv("FMGI_REDUCE");
    bool distinct = true;
    for (int k = 0; k < nshard; k++)
        for (int j = 0; j < k; j++) distinct = distinct && sdev[(size_t)k] != sdev[(size_t)j];
    const bool force_rccl = r_env && !strcmp(r_env, "rccl"), force_peer = r_env && !strcmp(r_env, "peer");
    if (force_rccl && !distinct) return set_err(FMGI_ERR_ARG, "FMGI_REDUCE=rccl needs one shard per device");
    bool use_rccl = force_rccl || (nshard > 1 && distinct && !force_peer);
    g_rccl_last = false;
    if (use_rccl) {
        int rc = rccl_comms(std::vector<int>(sdev.begin(), sdev.end()));
        if (rc != FMGI_OK && force_rccl) return rc;
        if (rc != FMGI_OK) { /* RCCL not loadable or its init failed: the peer-copy tree gives the same sums */
            if (verbose) {
                printf("[INF] RCCL unavailable (%s); shards reduced by xGMI peer copies\n", fmgi_last_error());
                fflush(stdout);
            }
            use_rccl = false;
        }
    }
    if (use_rccl) {
        const RcclApi *R = rccl_api();
        ncclResult_t r = R->group_start();
        for (int k = 0; k < nshard && r == ncclSuccess; k++) {
            DropinShard &S = g_dropin[(size_t)k];
            /* rank k's stream already holds its bake; the reduce follows it there (root: in place) */
            r = R->reduce(S.lm, g_dropin[0].lm, (size_t)geo->numTexels * 4, ncclInt64, ncclSum, 0,
                          g_rccl_comms[(size_t)k], S.ctx->stream);
        }
        const ncclResult_t r2 = R->group_end();
        if (r == ncclSuccess) r = r2;
        if (r != ncclSuccess) return set_err(FMGI_ERR_HIP, "ncclReduce of the shard lightmaps: %s", R->error_string(r));
        g_rccl_last = true;
    }
    /* binary-tree reduction into shard 0 (fmgi_dropin_reduce_order), ordered by events across devices */
    std::vector<int32_t> rdst((size_t)nshard), rsrc((size_t)nshard);
    const int nsteps = use_rccl ? 0 : fmgi_dropin_reduce_order(nshard, rdst.data(), rsrc.data());
    {
        for (int i = 0; i < nsteps; i++) {
            DropinShard &D = g_dropin[(size_t)rdst[(size_t)i]], &Src = g_dropin[(size_t)rsrc[(size_t)i]];
            const int dd = D.ctx->device, sd = Src.ctx->device;
            enable_peer(dd, sd);
            hipError_t e = hipSetDevice(dd);
            if (e == hipSuccess) e = hipStreamWaitEvent(D.ctx->stream, Src.done, 0);
            const void *add_src = Src.lm;
            if (e == hipSuccess && dd != sd) { /* over xGMI into this device's staging buffer */
                e = hipMemcpyPeerAsync(D.stage, dd, Src.lm, sd, lmb, D.ctx->stream);
                add_src = D.stage;
            }
            if (e == hipSuccess)
                e = fmgi_launch_add_u64((unsigned long long *)D.lm, (const unsigned long long *)add_src,
                                        (int64_t)geo->numTexels * 4, D.ctx->stream);
            if (e == hipSuccess) e = hipEventRecord(D.done, D.ctx->stream);
            if (e != hipSuccess) return set_err(FMGI_ERR_HIP, "shard reduction: %s", hipGetErrorString(e));
        }
    }
    /* every shard's bake and the reduction done: a stream overflow fails the call before the caller's
       texels are touched */
    for (int k = 0; k < nshard; k++) {
        fmgi_context *ck = g_dropin[(size_t)k].ctx;
        HIPCHK(hipSetDevice(ck->device));
        HIPCHK(hipStreamSynchronize(ck->stream));
    }
    for (int k = 0; k < nshard; k++) {
        const int rc = check_no_overflow(g_dropin[(size_t)k].ctx);
        if (rc != FMGI_OK) return rc;
    }
    /* texels: the caller's values + the exact sum, rounded once (k_finalize), on shard 0's device */
    fmgi_context *c0 = S0.ctx;
    HIPCHK(hipSetDevice(c0->device));
    if (g_dropin_tex && (g_dropin_tex_dev != c0->device || g_dropin_tex_bytes < tb)) {
        int cur = 0;
        (void)hipGetDevice(&cur);
        (void)hipSetDevice(g_dropin_tex_dev);
        (void)hipFree(g_dropin_tex);
        (void)hipSetDevice(cur);
        g_dropin_tex = nullptr;
        g_dropin_tex_bytes = 0;
    }
    if (!g_dropin_tex) {
        HIPCHK(hipMalloc(&g_dropin_tex, tb));
        g_dropin_tex_bytes = tb;
        g_dropin_tex_dev = c0->device;
    }
    HIPCHK(hipMemcpyAsync(g_dropin_tex, geo->texels, tb, hipMemcpyHostToDevice, c0->stream));
    int rc = fmgi_finalize(c0, S0.lm, g_dropin_tex, g_dropin_tex, c0->stream);
    if (rc != FMGI_OK) return rc;
    HIPCHK(hipMemcpyAsync(texels_out, g_dropin_tex, tb, hipMemcpyDeviceToHost, c0->stream));
    HIPCHK(hipStreamSynchronize(c0->stream));
    return FMGI_OK;
}

FMGI_API int getGlobalIlluminationCl(const fmgi_geometry *geo, int numSamplesPerArea, fmgi_vec3 *texels_out) {
    if (!geo || (geo->numTexels > 0 && (!texels_out || !geo->texels)))
        return set_err(FMGI_ERR_ARG, "getGlobalIlluminationCl: bad arguments");
    return bake_geometry(geo, numSamplesPerArea, texels_out, false);
}

FMGI_API void performGlobalIlluminationCl(fmgi_geometry *geo, int numSamplesPerArea) {
    const char *q = getenv("FMGI_QUIET");
    int rc = bake_geometry(geo, numSamplesPerArea, geo ? geo->texels : nullptr, !(q && atoi(q)));
    if (rc != FMGI_OK) {
        /* the reference's fatal-error convention: message on stdout, exit(-1) (global_illumination_cl.c:263) */
        printf("[Err] performGlobalIlluminationCl: %s\n", fmgi_last_error());
        fflush(stdout);
        exit(-1);
    }
}
