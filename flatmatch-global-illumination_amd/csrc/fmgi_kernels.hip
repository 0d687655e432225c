/*
 * fmgi_kernels.hip -- HIP/CDNA4 (gfx950) kernels of the photon-mapping hot path.
 *
 * Replaces the OpenCL kernel `photonmap` (photonmap.cl:269-281) and its helpers. Design:
 *   - one lane = one reference work item (100 photons from one LCG stream, photonmap.cl:272-280);
 *     lanes fetch work items from a global counter, so a lane that finishes its item starts the next
 *     one at once and the grid is persistent (no per-launch tail, no 25,600-item launches);
 *   - the photon/bounce loops are flattened per lane (a lane whose photon escapes starts its next
 *     photon in the same loop iteration);
 *   - the rectangle list is wave-uniform: every lane tests rect i at the same time, so the rect
 *     record is read with scalar loads into SGPRs (no VGPR/LDS traffic per test);
 *   - deposits go to an int64 fixed-point lightmap with device-scope atomics: exact, race-free and
 *     order-independent (the reference's lightColors[] += is a data race, photonmap.cl:256).
 * Two scan policies share the state machine: ScanExact (photonmap.cl:194-206 literally) and
 * ScanFast (conservative fp32 filter + exact verification; identical results, see below).
 */
#include <hip/hip_runtime.h>

#include "fmgi_internal.h"

#if defined(__clang__)
#pragma clang fp contract(off)
#endif

namespace {

struct LcgJumpC {
    uint32_t a[41], c[41];
};
constexpr LcgJumpC make_jump() {
    LcgJumpC t{};
    uint32_t a = 1, c = 0;
    for (int k = 0; k <= 40; k++) {
        t.a[k] = a;
        t.c[k] = c;
        a = 1664525u * a;
        c = 1664525u * c + 1013904223u;
    }
    return t;
}
__constant__ LcgJumpC c_jump = make_jump();

struct EventDev {
    int32_t photon, depth, rect, texel;
    float rgb[3];
    uint32_t rng;
};

__device__ __forceinline__ int find_launch(const LaunchDev *__restrict__ L, int n, uint64_t item) {
    int lo = 0, hi = n - 1;
    while (lo < hi) {
        int mid = (lo + hi + 1) >> 1;
        if (L[mid].item_begin <= item) lo = mid; else hi = mid - 1;
    }
    return lo;
}

__device__ __forceinline__ unsigned long long fx(float v) {
    /* v >= 0.25 and a float => v * 2^25 is an integer < 2^53: exact */
    return (unsigned long long)((double)v * 33554432.0);
}

__device__ __forceinline__ unsigned long long wave_sum(unsigned long long v) {
    for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off, 64);
    return v;
}

/* ---- scan policies -------------------------------------------------------------------------- */

/* photonmap.cl:189-206, evaluated literally for every rectangle in index order. */
struct ScanExact {
    static __device__ __forceinline__ int scan(const BakeArgs &a, f3 src, f3 dir, float &best,
                                               unsigned long long &tests, unsigned long long &) {
        const RectDev *__restrict__ R = a.rects;
        float bestd = INFINITY;
        int hit = -1;
        for (int i = 0; i < a.nrects; i++) {
            const RectDev &r = R[i];
            float d = intersect_exact(mkf3(r.nx, r.ny, r.nz), mkf3(r.px, r.py, r.pz), mkf3(r.wnx, r.wny, r.wnz),
                                      r.wl, mkf3(r.hnx, r.hny, r.hnz), r.hl, src, dir, bestd);
            if (d < 0) continue;
            if (d < bestd) { bestd = d; hit = i; }
        }
        tests += (unsigned long long)a.nrects;
        best = bestd;
        return hit;
    }
};

/* ---- the per-lane photon state machine ------------------------------------------------------- */

template <class Scan, bool TRACE>
__global__ __launch_bounds__(256) void k_bake(BakeArgs a) {
    uint32_t rng = 0;
    f3 pos = mkf3(0, 0, 0), dir = mkf3(0, 0, 0), col = mkf3(0, 0, 0);
    int depth = 0, left = 0, photon = -1;
    int srci = 0;
    bool win = false, alive = false;
    uint64_t item = 0;
    int nev = 0;
    unsigned long long n_ph = 0, n_scan = 0, n_dep = 0, n_esc = 0, n_tests = 0, n_rescan = 0;

    for (;;) {
        if (!alive) {
            if (left == 0) {
                if (TRACE && photon >= 0) {
                    a.ev_counts[item - a.item_begin] = nev;
                    a.rng_final[item - a.item_begin] = rng;
                }
                uint64_t w = a.item_begin + atomicAdd(a.counter, 1ull);
                if (w >= a.item_end) break;
                item = w;
                const LaunchDev L = a.launches[find_launch(a.launches, a.nlaunches, w)];
                rng = (uint32_t)(w - L.item_begin) + (uint32_t)L.rng_offset;
                /* photonmap.cl:272-275: r = rand()*40; ceil(r) further draws, as one LCG jump */
                float r40 = rng_next(rng) * 40;
                int k = (int)ceilf(r40);
                rng = c_jump.a[k] * rng + c_jump.c[k];
                srci = L.source;
                win = L.is_window != 0;
                left = FMGI_PHOTONS_PER_ITEM;
                photon = -1;
                nev = 0;
            }
            /* photonmap.cl:167-181: emission */
            const SrcDev &S = a.srcs[srci];
            col = win ? mkf3(18, 18, 18) : mkf3(16, 16, 18);
            float dx = rng_next(rng);
            float dy = rng_next(rng);
            dir = sample_dir(rng, mkf3(S.nx, S.ny, S.nz), mkf3(S.bux, S.buy, S.buz), mkf3(S.bvx, S.bvy, S.bvz), win);
            pos = add3(add3(add3(mkf3(S.px, S.py, S.pz), mul3(mkf3(S.wx, S.wy, S.wz), dx)), mul3(mkf3(S.hx, S.hy, S.hz), dy)),
                       mul3(dir, 1e-5f));
            left--;
            photon++;
            depth = 0;
            alive = true;
            n_ph++;
        }

        float best;
        int hit = Scan::scan(a, pos, dir, best, n_tests, n_rescan);
        n_scan++;
        if (best == INFINITY) { /* photonmap.cl:208-209 */
            alive = false;
            n_esc++;
            continue;
        }
        /* photonmap.cl:216-258 */
        const RectDev &h = a.rects[hit];
        pos = add3(pos, mul3(dir, best));
        const f3 hn = mkf3(h.nx, h.ny, h.nz);
        const int texel = h.base + tile_at(mkf3(h.px, h.py, h.pz), mkf3(h.wnx, h.wny, h.wnz), h.wl,
                                           mkf3(h.hnx, h.hny, h.hnz), h.hl, h.W, h.H, pos);
        if ((double)pos.z > 0.0005 || rng_next(rng) > 0.75f) {
            dir = sample_dir(rng, hn, mkf3(h.bux, h.buy, h.buz), mkf3(h.bvx, h.bvy, h.bvz), false);
            if (pos.z < 1e-5f) {
                col.y *= 0.85f;
                col.z *= 0.7f;
            }
            col = mul3(col, 0.9f);
        } else {
            float two = 2.0f * dot3(hn, dir);
            dir = sub3(dir, mul3(hn, two));
        }
        unsigned long long *t = a.lm + 4 * (size_t)texel;
        atomicAdd(t + 0, fx(col.x));
        atomicAdd(t + 1, fx(col.y));
        atomicAdd(t + 2, fx(col.z));
        n_dep++;
        if (TRACE) {
            EventDev e;
            e.photon = photon;
            e.depth = depth;
            e.rect = hit;
            e.texel = texel;
            e.rgb[0] = col.x;
            e.rgb[1] = col.y;
            e.rgb[2] = col.z;
            e.rng = rng;
            ((EventDev *)a.events)[(item - a.item_begin) * FMGI_EVENTS_PER_ITEM + nev] = e;
            nev++;
        }
        pos = add3(pos, mul3(dir, 1e-5f));
        if (++depth == FMGI_MAX_DEPTH) alive = false;
    }
    if (TRACE && photon >= 0) {
        a.ev_counts[item - a.item_begin] = nev;
        a.rng_final[item - a.item_begin] = rng;
    }

    unsigned long long v[6] = {n_ph, n_scan, n_dep, n_esc, n_rescan, n_tests};
#pragma unroll
    for (int i = 0; i < 6; i++) {
        unsigned long long s = wave_sum(v[i]);
        if ((threadIdx.x & 63) == 0 && s) atomicAdd(a.stats + i, s);
    }
}

__global__ void k_finalize(const unsigned long long *__restrict__ lm, const float4 *__restrict__ tin,
                           float4 *__restrict__ tout, int64_t n) {
    int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    float4 t = tin[i];
    const long long *q = (const long long *)lm + 4 * i;
    float4 o;
    o.x = (float)((double)t.x + (double)q[0] * 2.98023223876953125e-08);
    o.y = (float)((double)t.y + (double)q[1] * 2.98023223876953125e-08);
    o.z = (float)((double)t.z + (double)q[2] * 2.98023223876953125e-08);
    o.w = t.w;
    tout[i] = o;
}

__global__ void k_sincos(const float *__restrict__ x, float *__restrict__ s, float *__restrict__ c, int64_t n) {
    int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    float a, b;
    fmgi_sincosf(x[i], &a, &b);
    s[i] = a;
    c[i] = b;
}

} // namespace

int fmgi_block_size() { return 256; }

hipError_t fmgi_launch_bake(const BakeArgs &a, int kernel, bool trace, int grid_blocks, hipStream_t s) {
    (void)kernel;
    dim3 grid(grid_blocks), block(256);
    if (trace)
        hipLaunchKernelGGL((k_bake<ScanExact, true>), grid, block, 0, s, a);
    else
        hipLaunchKernelGGL((k_bake<ScanExact, false>), grid, block, 0, s, a);
    return hipGetLastError();
}

hipError_t fmgi_launch_finalize(const unsigned long long *lm, const float *tin, float *tout, int64_t n,
                                hipStream_t s) {
    if (n <= 0) return hipSuccess;
    int64_t blocks = (n + 255) / 256;
    hipLaunchKernelGGL(k_finalize, dim3((unsigned)blocks), dim3(256), 0, s, lm, (const float4 *)tin, (float4 *)tout, n);
    return hipGetLastError();
}

hipError_t fmgi_launch_sincos(const float *x, float *sn, float *cs, int64_t n, hipStream_t s) {
    if (n <= 0) return hipSuccess;
    int64_t blocks = (n + 255) / 256;
    hipLaunchKernelGGL(k_sincos, dim3((unsigned)blocks), dim3(256), 0, s, x, sn, cs, n);
    return hipGetLastError();
}
