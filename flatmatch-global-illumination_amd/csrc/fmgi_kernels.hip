/*
 * fmgi_kernels.hip -- HIP/CDNA4 (gfx950) kernels of the photon-mapping hot path.
 *
 * Replaces the OpenCL kernel `photonmap` (photonmap.cl:269-281) and its helpers. Design:
 *   - one lane = one reference work item (100 photons from one LCG stream, photonmap.cl:272-280);
 *     lanes fetch work items from a global counter, so a lane that finishes its item starts the next
 *     one at once and the grid is persistent (no per-launch tail, no 25,600-item launches);
 *   - the photon/bounce loops are flattened per lane (a lane whose photon escapes starts its next
 *     photon in the same loop iteration);
 *   - wave-uniform data (rect records of the exact scan) is read through the constant address space,
 *     i.e. scalar loads into SGPRs; the fast scan's filter records are staged in LDS once per
 *     workgroup and read per lane (each lane reads the record of the class it faces);
 *   - deposits are exact and order-free: either three int64 fixed-point atomics per deposit (AccFx3)
 *     or one u32 counter per (colour state, texel) (AccState) folded into int64 by k_reduce_states.
 *     The reference's lightColors[] += is a data race (photonmap.cl:256); these are not.
 * Two scan policies share the state machine: ScanExact (photonmap.cl:194-206 literally) and
 * ScanFast (conservative fp32 filter + exact verification; identical results, see below).
 */
#include <hip/hip_runtime.h>

#include <cxxabi.h>
#include <mutex>
#include <set>
#include <string>
#include <utility>

#include "fmgi_internal.h"
#include "flatmatch_gi.h"

#if defined(__clang__)
#pragma clang fp contract(off)
#endif

namespace {

template <class T>
using cptr = const __attribute__((address_space(4))) T *; /* constant space: scalar loads */
template <class T>
using gptr = const __attribute__((address_space(1))) T *; /* global space: vector loads, never flat */

/* A uniform kernel argument re-read where it is used: the empty volatile asm keeps the compiler from
   hoisting the comparison out of the bake loop as a 64-bit lane mask (one per condition, held across
   the loop: the masks were most of the SGPRs the register allocator spilled to VGPR lanes and read back
   with v_readlane, a VALU instruction, on every use) */
template <class T>
__device__ __forceinline__ T uni(T v) {
    asm volatile("" : "+s"(v));
    return v;
}

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
constexpr LcgJumpC kJump = make_jump();
__constant__ LcgJumpC c_jump = kJump;
static_assert(kJump.a[1] == 1664525u && kJump.c[1] == 1013904223u, "LCG of photonmap.cl:23");

struct EventDev {
    int32_t photon, depth, rect, texel;
    float rgb[3];
    uint32_t rng;
};

__device__ __forceinline__ unsigned long long fx(float v) {
    /* v >= 0.25 and a float => v * 2^25 is an integer < 2^53: exact */
    return (unsigned long long)((double)v * 33554432.0);
}

__device__ __forceinline__ unsigned long long wave_sum(unsigned long long v) {
    for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off, 64);
    return v;
}

__device__ __forceinline__ float exact_on(cptr<RectDev> R, int i, f3 src, f3 dir, float closest) {
    const float nx = R[i].nx, ny = R[i].ny, nz = R[i].nz, px = R[i].px, py = R[i].py, pz = R[i].pz;
    const float wx = R[i].wnx, wy = R[i].wny, wz = R[i].wnz, wl = R[i].wl;
    const float hx = R[i].hnx, hy = R[i].hny, hz = R[i].hnz, hl = R[i].hl;
    return intersect_exact(mkf3(nx, ny, nz), mkf3(px, py, pz), mkf3(wx, wy, wz), wl, mkf3(hx, hy, hz), hl, src,
                           dir, closest);
}

/* exact_on for the rare paths of the fast and grid scans (fallbacks, non-axis-aligned rects): the index
   is made a per-lane (VGPR) value, so the record comes in with vector loads. Scalar loads of a 64-B
   record per test would reserve a block of SGPRs in the whole kernel, whose pressure then spills the
   hot loop's SGPRs into VGPR lanes. */
__device__ __forceinline__ float exact_on_v(const RectDev *R, int i, f3 src, f3 dir, float closest) {
    asm volatile("" : "+v"(i));
    const RectDev &r = R[i];
    return intersect_exact(mkf3(r.nx, r.ny, r.nz), mkf3(r.px, r.py, r.pz), mkf3(r.wnx, r.wny, r.wnz), r.wl,
                           mkf3(r.hnx, r.hny, r.hnz), r.hl, src, dir, closest);
}

/* The scan's result and what the deposit needs of the hit rect, read once (phase 2 of the fast scans
   evaluates the winner exactly; the hit stage reuses its in-rect coordinates, see intersect_exact_uv). */
struct HitRec {
    int idx;             /* hit rect, or -1 (best = INFINITY: the photon escapes)          */
    float best, dx, dy;  /* exact hit distance and in-rect coordinates (photonmap.cl:99-100) */
    float nx, ny, nz, wl, hl, iwl, ihl;
    int base, W, H;
    float bux, buy, buz, bvx, bvy, bvz;
};

/* photonmap.cl:123-158 (closest = INFINITY) on rect r (index idx), filling h's rect fields and dx, dy */
template <class R>
__device__ __forceinline__ float exact_hit_rec(const R &r, int idx, f3 src, f3 dir, HitRec &h) {
    h.idx = idx;
    h.nx = r.nx; h.ny = r.ny; h.nz = r.nz;
    h.wl = r.wl; h.hl = r.hl;
    h.iwl = r.iwl; h.ihl = r.ihl;
    h.base = r.base; h.W = r.W; h.H = r.H;
    h.bux = r.bux; h.buy = r.buy; h.buz = r.buz;
    h.bvx = r.bvx; h.bvy = r.bvy; h.bvz = r.bvz;
    return intersect_exact_uv(mkf3(r.nx, r.ny, r.nz), mkf3(r.px, r.py, r.pz), mkf3(r.wnx, r.wny, r.wnz), r.wl,
                              mkf3(r.hnx, r.hny, r.hnz), r.hl, src, dir, h.dx, h.dy);
}

/* the same on rect idx, read from the workgroup's LDS copy of the table (RectLds records) when the host
   staged it there (BakeArgs::rects_off >= 0), else from global memory; the two reads stay in their own address
   spaces (a pointer that may be either compiles to flat loads, which wait on both counters) */
template <bool Staged = false>
__device__ __forceinline__ float exact_hit(const BakeArgs &a, const char *lds, int idx, f3 src, f3 dir, HitRec &h) {
    if (Staged || uni(a.rects_off) >= 0)
        return exact_hit_rec(*(const __attribute__((address_space(3))) RectLds *)(
                                 (const __attribute__((address_space(3))) char *)lds + a.rects_off +
                                 __umul24((uint32_t)idx, (uint32_t)sizeof(RectLds))), /* not the quarter-rate v_mul_lo_u32 */
                             idx, src, dir, h);
    return exact_hit_rec(((gptr<RectDev>)a.rects)[idx], idx, src, dir, h);
}

/* the global table (rare paths: fallbacks, ScanExact) */
__device__ __forceinline__ float exact_hit(const BakeArgs &a, int idx, f3 src, f3 dir, HitRec &h) {
    return exact_hit_rec(((gptr<RectDev>)a.rects)[idx], idx, src, dir, h);
}

/* phase 2 on the compact closed-box tables (fmgi_internal.h RectC / ClassC, staged in LDS): the same
   intersect_exact_uv on the same bit patterns as exact_hit_rec's RectLds / RectDev fields; 1 / length is
   v_rcp_f32 (tile_uv's quotient estimate needs only one ulp) */
__device__ __forceinline__ float exact_hit_compact(const BakeArgs &a, const char *lds, int idx, f3 src, f3 dir,
                                                   HitRec &h) {
    typedef const __attribute__((address_space(3))) char *lp;
    const __attribute__((address_space(3))) RectC &r =
        *(const __attribute__((address_space(3))) RectC *)((lp)lds + a.rectc_off + __umul24((uint32_t)idx, (uint32_t)sizeof(RectC)));
    const float px = r.px, py = r.py, pz = r.pz, wl = r.wl, hl = r.hl;
    const uint32_t meta = r.meta;
    const __attribute__((address_space(3))) ClassC &k =
        *(const __attribute__((address_space(3))) ClassC *)((lp)lds + a.class_off + ((meta >> kCompactBaseBits) << 6));
    h.idx = idx;
    h.nx = k.nx; h.ny = k.ny; h.nz = k.nz;
    h.wl = wl; h.hl = hl;
    h.iwl = __builtin_amdgcn_rcpf(wl);
    h.ihl = __builtin_amdgcn_rcpf(hl);
    h.base = (int)(meta & ((1u << kCompactBaseBits) - 1));
    const uint32_t wh = (uint32_t)k.WH;
    h.W = (int)(wh & 0xFFFFu); h.H = (int)(wh >> 16);
    h.bux = k.bux; h.buy = k.buy; h.buz = k.buz;
    h.bvx = k.bvx; h.bvy = k.bvy; h.bvz = k.bvz;
    return intersect_exact_uv(mkf3(h.nx, h.ny, h.nz), mkf3(px, py, pz), mkf3(k.wnx, k.wny, k.wnz), wl,
                              mkf3(k.hnx, k.hny, k.hnz), hl, src, dir, h.dx, h.dy);
}

/* the result of a literal scan (hit, best) as a HitRec (rare paths: ScanExact, fallbacks) */
__device__ __forceinline__ void finish_hit(const BakeArgs &a, int hit, float best, f3 src, f3 dir, HitRec &h) {
    h = HitRec{}; /* every field is (re)written here, so none of the caller's phase-2 values stays live */
    h.idx = -1;
    if (hit >= 0 && best != INFINITY)
        exact_hit(a, hit, src, dir, h); /* the same fac again: closest never changes intersects()' fac */
    h.best = best;
    /* (rare path) the record's fields are in registers before the bake loop goes on: none of the
       loop-carried registers (the sample basis) is left pending on a global load, which would make the
       compiler wait vmcnt(0) at the loop's top, i.e. for the scattered deposit store of the iteration before
       (gfx9 counts stores in vmcnt) */
    __builtin_amdgcn_s_waitcnt(0x0F70); /* vmcnt(0) */
}

/* ---- scan policies -------------------------------------------------------------------------- */

/* Stage timing (profiling builds only, -DFMGI_STAGE_TIMING): s_memtime deltas of each bake-loop stage,
   summed per wave into stats[KSTAT_STAGE0 + k]; compiled out otherwise. */
enum { ST_START = 0, ST_SAMPLE, ST_SCAN1, ST_SCAN2, ST_FALLBACK, ST_HIT, ST_APPEND, ST_N };
struct StageClock {
#ifdef FMGI_STAGE_TIMING
    unsigned long long last = 0, acc[ST_N] = {};
    __device__ __forceinline__ void lap(int k) {
        const unsigned long long t = __builtin_amdgcn_s_memtime();
        acc[k] += t - last;
        last = t;
    }
    __device__ __forceinline__ void reset() { last = __builtin_amdgcn_s_memtime(); }
#else
    __device__ __forceinline__ void lap(int) {}
    __device__ __forceinline__ void reset() {}
#endif
};

struct ScanStats {
    StageClock clk;
    /* rectangle tests evaluated (phase-1 records + exact tests) since the lane's last work-item fetch,
       where they are flushed (flush_tests): a work item makes <= 800 scans of <= nrects tests each */
    uint32_t tests = 0;
    /* scans re-done by the literal scan (rescans = ties + invalid; <= the lane's scans, 32 bits) */
    uint32_t ties = 0;    /* the runner-up was within the separation band */
    uint32_t invalid = 0; /* the phase-1 winner failed the exact test     */
};

#ifndef FMGI_LITERAL_LDS /* the fallbacks' literal scan reads the staged walls from LDS (0: the global table) */
#define FMGI_LITERAL_LDS 1
#endif
/* photonmap.cl:189-206, evaluated literally for every rectangle in index order. */
struct ScanExact {
    static constexpr bool kLds = false;
    static constexpr bool kCoop = false;
    static constexpr int kMinWaves = 1; /* k_bake occupancy floor for the register allocator */
    static __device__ __forceinline__ void scan(const BakeArgs &a, const char *lds, f3 src, f3 dir, HitRec &h,
                                                ScanStats &st) {
        float best;
        const int hit = literal<true>(a, lds, src, dir, best, st);
        finish_hit(a, hit, best, src, dir, h);
    }
    /* Scalar: records through scalar loads (the exact kernel's own uniform loop); else vector loads (the
       other scans' rare fallback) */
    template <bool Scalar = false, bool Staged = false>
    static __device__ __forceinline__ int literal(const BakeArgs &a, const char *lds, f3 src, f3 dir, float &best,
                                                  ScanStats &st) {
        cptr<RectDev> R = (cptr<RectDev>)a.rects;
        float bestd = INFINITY;
        int hit = -1;
#if FMGI_LITERAL_LDS
        if (Staged || (!Scalar && uni(a.rects_off) >= 0)) {
            /* the walls staged in LDS (RectLds): every lane of the wave reads the same record (a broadcast),
               where the global table costs a dependent L2 round trip per rect */
            const __attribute__((address_space(3))) char *l = (const __attribute__((address_space(3))) char *)lds;
            for (int i = 0; i < uni(a.nrects); i++) {
                const __attribute__((address_space(3))) RectLds &r =
                    *(const __attribute__((address_space(3))) RectLds *)(l + a.rects_off + i * (int)sizeof(RectLds));
                const float d = intersect_exact(mkf3(r.nx, r.ny, r.nz), mkf3(r.px, r.py, r.pz),
                                                mkf3(r.wnx, r.wny, r.wnz), r.wl, mkf3(r.hnx, r.hny, r.hnz), r.hl, src,
                                                dir, bestd);
                if (d < 0) continue;
                if (d < bestd) { bestd = d; hit = i; }
            }
            st.tests += (uint32_t)a.nrects;
            best = bestd;
            return hit;
        }
#endif
        for (int i = 0; i < uni(a.nrects); i++) {
            const float d = Scalar ? exact_on(R, i, src, dir, bestd) : exact_on_v(a.rects, i, src, dir, bestd);
            if (d < 0) continue;
            if (d < bestd) { bestd = d; hit = i; }
        }
        st.tests += (uint32_t)a.nrects;
        best = bestd;
        return hit;
    }
};

/*
 * ScanFast: same result as ScanExact, bit for bit, at a fraction of the VALU work.
 *
 * Why it is exact (DESIGN.md §Fast scan): let V be the rects passing photonmap.cl's order-independent
 * tests (front face, fac >= 0, hit point inside both extents). The sequential scan returns the rect m
 * with the smallest exact fac whenever every other member of V has fac > fac_m * (1 + 2^-13): m is then
 * accepted whatever was accepted before it (the `closest^2 < |ray|^2` early-out cannot fire for it), and
 * nothing after it can replace it. Phase 1 evaluates, for every rect, a conservative approximation
 * (superset of V, fac' within 2^-20 relative of the exact fac); phase 2 evaluates photonmap.cl's
 * intersects() exactly for the phase-1 winner and checks the separation against the runner-up. Any doubt
 * (runner-up too close, winner not exactly valid) falls back to the literal exact scan.
 *
 * Phase 1 for an axis-aligned rect with normal axis a (all rects of the reference's layouts and of the
 * synthetic boxes): fac' = (plane - src_a) * rcp(dir_a), hit = src + dir*fac' on the two other axes,
 * inside the rect's extent grown by a scene-scale margin (host: fmgi_api.cpp build_filter). The filter
 * image in LDS holds, per axis, pairs {record j of the +a class, record j of the -a class} (64 B); a
 * lane reads the half of the pair whose class it faces (front face <=> n_a * dir_a < 0), so every lane
 * spends iteration j on a front-facing rect and no lane needs a select.
 */
template <int A>
__device__ __forceinline__ float comp(f3 v) { return A == 0 ? v.x : (A == 1 ? v.y : v.z); }

template <int A, bool Coop>
__device__ __forceinline__ void filter_axis(const char *img, int J, int sub, int coop, f3 s, f3 d, float &L1,
                                            float &L2, int &code1) {
    constexpr int U = (A == 0) ? 1 : 0;
    constexpr int V = (A == 2) ? 1 : 2;
    const float sa = comp<A>(s), da = comp<A>(d);
    const float su = comp<U>(s), sv = comp<V>(s), du = comp<U>(d), dv = comp<V>(d);
    const float rd = __builtin_amdgcn_rcpf(da);
    const float4 *p = (const float4 *)__builtin_assume_aligned(img + (da < 0.0f ? 0 : 32), 16);
    /* every record, in a uniform loop (the LDS reads of 4 records in flight at once): measured faster
       than a nearest-first walk with an early exit, whose per-lane trip counts diverge. With coop lanes
       per work item, sub-lane `sub` takes records [sub T, sub T + T) of the class (T uniform; the
       indices past J read LDS beyond the class and are masked) */
    const int T = Coop ? (J + coop - 1) / coop : J, j0 = Coop ? sub * T : 0;
#pragma unroll 4
    for (int t = 0; t < T; t++) {
        const int j = j0 + t;
        const float4 q = p[4 * j];                      /* plane, cu, hwu, cv: ds_read_b128 */
        const float hwv = ((const float *)(p + 4 * j))[4]; /* hwv: ds_read_b32               */
        const float f = (q.x - sa) * rd;
        const float uu = fmaf(du, f, su) - q.y;
        const float vv = fmaf(dv, f, sv) - q.w;
        const int ok = (int)(!Coop || j < J) & (int)(f >= 0.0f) & (int)(fabsf(uu) <= q.z) & (int)(fabsf(vv) <= hwv);
        const float key = ok ? f : INFINITY;
        const bool lt = key < L1;
        L2 = __builtin_amdgcn_fmed3f(L1, key, L2);
        code1 = lt ? ((A << 16) | j) : code1;
        L1 = lt ? key : L1;
    }
}

/*
 * ScanHybrid's wall filter: filter_axis over the pair image (FilterPairHalf, fmgi_internal.h), two records
 * per iteration in packed fp32. A group holds records 2g and 2g + 1 of a class as field pairs, so each
 * pair is a 64-bit register pair straight from ds_read_b128, and fac', the two hit coordinates and their
 * offsets from the records' centres run as v_pk_add_f32 / v_pk_mul_f32 / v_pk_fma_f32: two fp32 ops per
 * lane per instruction, but each occupies the SIMD for 4 cycles, as two v_fma_f32 do (tools/valu_peak.hip,
 * profiles/valu_peak.json: 0.24 v_pk_fma_f32 vs 0.45 v_fma_f32 per SIMD-cycle); the gain is fewer
 * instructions to issue and the 64-bit operand pairs read straight from ds_read_b128. Each element
 * is the same IEEE op on the same operands as filter_axis's, so every key and candidate test is
 * filter_axis's bit for bit; the compares and the (L1, L2, code1) update stay per record, in record
 * order. code1 receives the record's rect index itself (loaded with the fields), not a position.
 */
typedef float pkf2 __attribute__((ext_vector_type(2)));
#ifndef FMGI_FILTER_PK
#define FMGI_FILTER_PK 1
#endif
#ifndef FMGI_PAIR_PREFETCH
#define FMGI_PAIR_PREFETCH 1
#endif

__device__ __forceinline__ void pair_rec(float f, float uu, float vv, float hu, float hv, int idx, float &L1,
                                         float &L2, int &code1) {
    const int ok = (int)(f >= 0.0f) & (int)(fabsf(uu) <= hu) & (int)(fabsf(vv) <= hv);
    const float key = ok ? f : INFINITY;
    const bool lt = key < L1;
    L2 = __builtin_amdgcn_fmed3f(L1, key, L2);
    code1 = lt ? idx : code1;
    L1 = lt ? key : L1;
}

template <int A>
__device__ __forceinline__ void filter_pairs(const char *img, int g0, int G, f3 s, f3 d, float &L1, float &L2,
                                             int &code1) {
    constexpr int U = (A == 0) ? 1 : 0;
    constexpr int V = (A == 2) ? 1 : 2;
    const float sa = comp<A>(s), da = comp<A>(d);
    const float rd = __builtin_amdgcn_rcpf(da);
    const pkf2 sa2 = {sa, sa}, rd2 = {rd, rd};
    const pkf2 su2 = {comp<U>(s), comp<U>(s)}, sv2 = {comp<V>(s), comp<V>(s)};
    const pkf2 du2 = {comp<U>(d), comp<U>(d)}, dv2 = {comp<V>(d), comp<V>(d)};
    const float4 *p = (const float4 *)__builtin_assume_aligned(img + (da < 0.0f ? 0 : 48), 16);
    auto group = [&](float4 q0, float4 q1, float4 q2) {
        const pkf2 pl = {q0.x, q0.y}, cu = {q0.z, q0.w}, cv = {q1.z, q1.w};
        const pkf2 f = (pl - sa2) * rd2;
        const pkf2 uu = __builtin_elementwise_fma(du2, f, su2) - cu;
        const pkf2 vv = __builtin_elementwise_fma(dv2, f, sv2) - cv;
        pair_rec(f.x, uu.x, vv.x, q1.x, q2.x, __float_as_int(q2.z), L1, L2, code1);
        pair_rec(f.y, uu.y, vv.y, q1.y, q2.y, __float_as_int(q2.w), L1, L2, code1);
    };
#if FMGI_PAIR_PREFETCH
    /* two groups per iteration with all six reads issued first (left to itself, the scheduler waits
       for each group's reads right after issuing them, exposing the LDS latency once per group;
       example.png bake 21.07 -> 20.78 ms, profiles/r05/s20) */
    int g = g0;
    for (; g + 1 < G; g += 2) {
        const float4 a0 = p[6 * g], a1 = p[6 * g + 1], a2 = p[6 * g + 2];
        const float4 b0 = p[6 * g + 6], b1 = p[6 * g + 7], b2 = p[6 * g + 8];
        __builtin_amdgcn_sched_group_barrier(0x100, 6, 0);
        __builtin_amdgcn_sched_group_barrier(0x00F, 400, 0);
        group(a0, a1, a2);
        group(b0, b1, b2);
    }
    if (g < G) group(p[6 * g], p[6 * g + 1], p[6 * g + 2]);
#else
#pragma unroll 2
    for (int g = g0; g < G; g++) group(p[6 * g], p[6 * g + 1], p[6 * g + 2]);
#endif
}

/* merges the phase-1 results (L1, L2, code1) of the coop lanes of a group (butterfly over lane ids):
   L1 = the minimum key, L2 = the second smallest of all keys, code1 = the winner (the smaller code on
   equal keys, so every lane of the group ends with the same values; equal keys fail the separation
   test anyway) */
__device__ __forceinline__ void coop_merge(int coop, float &L1, float &L2, int &code1) {
    for (int off = 1; off < coop; off <<= 1) {
        const float oL1 = __shfl_xor(L1, off, 64), oL2 = __shfl_xor(L2, off, 64);
        const int oc = __shfl_xor(code1, off, 64);
        L2 = fminf(fmaxf(L1, oL1), fminf(L2, oL2));
        const bool take = oL1 < L1 || (oL1 == L1 && oc < code1);
        code1 = take ? oc : code1;
        L1 = take ? oL1 : L1;
    }
}

/* Coop = true: the kernel for small launches, whose BakeArgs::coop lanes per work item hold the same
   photon and split every scan's records (the product path for large launches keeps Coop = false) */
template <bool Coop>
struct ScanFastT {
    static constexpr bool kLds = true;
    static constexpr bool kCoop = Coop;
    static constexpr int kMinWaves = 1; /* k_bake occupancy floor for the register allocator */
    static __device__ __forceinline__ void scan(const BakeArgs &a, const char *lds, f3 src, f3 dir, HitRec &h,
                                                ScanStats &st) {
        float L1 = INFINITY, L2 = INFINITY;
        int code1 = -1;
        const int coop = Coop ? a.coop : 1, sub = Coop ? (int)__lane_id() & (coop - 1) : 0;
        filter_axis<0, Coop>(lds, a.fJ[0], sub, coop, src, dir, L1, L2, code1);
        filter_axis<1, Coop>(lds + 64 * a.fJ[0], a.fJ[1], sub, coop, src, dir, L1, L2, code1);
        filter_axis<2, Coop>(lds + 64 * (a.fJ[0] + a.fJ[1]), a.fJ[2], sub, coop, src, dir, L1, L2, code1);
        /* rects that are not axis-aligned: exact order-independent tests (no early-out); coop lanes split
           them like the filter records (each tested by one sub-lane, so coop_merge's L2 is the true
           runner-up and a winning general rect does not look tied with itself) */
        gptr<int32_t> G = (gptr<int32_t>)a.general;
        for (int g = sub; g < a.ngeneral; g += coop) {
            const float f = exact_on_v(a.rects, G[g], src, dir, INFINITY);
            const float key = (f < 0) ? INFINITY : f;
            const bool lt = key < L1;
            L2 = __builtin_amdgcn_fmed3f(L1, key, L2);
            code1 = lt ? ((3 << 16) | g) : code1;
            L1 = lt ? key : L1;
        }
        if (Coop) coop_merge(coop, L1, L2, code1);
        st.tests += (uint32_t)(a.fJ[0] + a.fJ[1] + a.fJ[2] + a.ngeneral);
        if (L1 == INFINITY) { /* V is a subset of the (empty) phase-1 set: the photon escapes */
            h.best = INFINITY;
            h.idx = -1;
            return;
        }
        /* phase 2: exact photonmap.cl intersects() of the winner */
        const int A = code1 >> 16, j = code1 & 0xFFFF;
        int idx;
        if (A == 3) {
            idx = ((gptr<int32_t>)a.general)[j];
        } else {
            const float dA = A == 0 ? dir.x : (A == 1 ? dir.y : dir.z);
            const int off = A == 0 ? 0 : (A == 1 ? 64 * a.fJ[0] : 64 * (a.fJ[0] + a.fJ[1]));
            idx = *(const int32_t *)(lds + off + 64 * j + (dA < 0.0f ? 0 : 32) + 20);
        }
        const float f = exact_hit(a, lds, idx, src, dir, h);
        /* separation: the runner-up's phase-1 value must exceed the exact winner by > 2^-12 relative
           (covers the 2^-20 phase-1 error and the 2^-13 early-out slack); false for f = INF */
        if (!(f < 0) && L2 > f * 1.000244140625f) {
            h.best = f;
            return;
        }
        if (f < 0) st.invalid++; else st.ties++;
        float best;
        const int hit = ScanExact::literal(a, lds, src, dir, best, st);
        finish_hit(a, hit, best, src, dir, h);
    }
};

using ScanFast = ScanFastT<false>;
using ScanFastCoop = ScanFastT<true>;

/*
 * ScanGrid: ScanFast's phase 1 with the rects of each plane bucketed by a 2-D grid.
 *
 * Rects of one class that share a plane share phase 1's fac' = (plane - src_a) * rcp(dir_a) and hit
 * point, so a lane evaluates fac' once per facing plane and tests only the records of the grid cell the
 * hit point falls in. Every rect whose margin-grown extent contains the hit point is registered in that
 * cell (the host registers each rect in every cell its grown extent overlaps, widened by a cell-rounding
 * slack), so the candidate set still contains V and the keys are ScanFast's bit for bit: phase 2 and
 * its separation argument carry over unchanged. A closed box of 200 rects has 6 planes: ~3 cells and a
 * few records per scan instead of ~100 rect tests.
 */
/* The kernel's cell of hit point (uh, vh) on plane record g (64 B, see GridPlane), and the point's
   16-bit fixed-point coordinates (qu, qv) inside that cell, against which the cell's inline records are
   tested (GridCell; the host derives their bounds from these same float ops, fmgi_api.cpp grid_q). */
__device__ __forceinline__ uint32_t grid_cell(const float4 g0, const float4 g1, const float4 g2, float uh, float vh,
                                              uint32_t &qu, uint32_t &qv) {
    /* g0 = {plane, u0, v0, iu}, g1 = {iv, mu, mv, nu}, g2 = {nv, cell_off, -, -} */
    /* clamp to [0, n - 1]: v_med3_f32 (fminf(fmaxf()) adds a canonicalising max); the same cell for
       every non-NaN coordinate */
    const float ru = (uh - g0.y) * g0.w, rv = (vh - g0.z) * g1.x;
    const float cu = __builtin_floorf(__builtin_amdgcn_fmed3f(ru, 0.0f, g1.y));
    const float cv = __builtin_floorf(__builtin_amdgcn_fmed3f(rv, 0.0f, g1.z));
    qu = (uint32_t)__builtin_amdgcn_fmed3f((ru - cu) * 65536.0f, 0.0f, 65535.0f);
    qv = (uint32_t)__builtin_amdgcn_fmed3f((rv - cv) * 65536.0f, 0.0f, 65535.0f);
    return (uint32_t)__float_as_int(g2.y) + __umul24((uint32_t)cv, (uint32_t)__float_as_int(g1.w)) + (uint32_t)cu;
}

/* grid cell ci: from the workgroup's LDS copy of the cell table when the host staged it there
   (BakeArgs::cells_off >= 0), else from global memory (L2-resident). The two reads stay in their own
   address spaces: a pointer that may point into either compiles to flat loads, which count in both
   vmcnt and lgkmcnt and make every LDS wait after them wait for the cell too. */
template <bool Staged = false>
__device__ __forceinline__ GridCell load_cell(const BakeArgs &a, const char *lds, uint32_t ci) {
    typedef uint32_t u4 __attribute__((ext_vector_type(4)));
    u4 q, r;
    if (Staged || uni(a.cells_off) >= 0) {
        const __attribute__((address_space(3))) u4 *l = (const __attribute__((address_space(3))) u4 *)(
            (const __attribute__((address_space(3))) char *)lds + a.cells_off);
        q = l[2 * ci];
        r = l[2 * ci + 1];
    } else {
        q = ((gptr<u4>)a.gcells)[2 * ci];
        r = ((gptr<u4>)a.gcells)[2 * ci + 1];
    }
    GridCell c;
    c.qu0 = q.x; c.qv0 = q.y; c.qu1 = q.z; c.qv1 = q.w;
    c.count = (int)r.x; c.idx0 = (int)r.y; c.idx1 = (int)r.z; c.rest = (int)r.w;
    return c;
}

/* one candidate test of ScanGrid's phase 1: record r against hit point (uh, vh) at fac' f */
__device__ __forceinline__ void grid_rec(float f, float uh, float vh, float4 r, int code, float &L1, float &L2,
                                         int &code1) {
    const bool ok = (int)(fabsf(uh - r.x) <= r.y) & (int)(fabsf(vh - r.z) <= r.w);
    const float key = ok ? f : INFINITY;
    const bool lt = key < L1;
    L2 = __builtin_amdgcn_fmed3f(L1, key, L2);
    code1 = lt ? code : code1;
    L1 = lt ? key : L1;
}

/* one inline record of a cell against the point's fixed-point cell coordinates: {lo | hi << 16} per axis */
__device__ __forceinline__ bool grid_qpass(uint32_t qu, uint32_t qv, uint32_t bu, uint32_t bv) {
    return (int)(qu >= (bu & 0xFFFFu)) & (int)(qu <= (bu >> 16)) & (int)(qv >= (bv & 0xFFFFu)) & (int)(qv <= (bv >> 16));
}
__device__ __forceinline__ void grid_recq(float f, uint32_t qu, uint32_t qv, uint32_t bu, uint32_t bv, int code,
                                          float &L1, float &L2, int &code1) {
    const float key = grid_qpass(qu, qv, bu, bv) ? f : INFINITY;
    const bool lt = key < L1;
    L2 = __builtin_amdgcn_fmed3f(L1, key, L2);
    code1 = lt ? code : code1;
    L1 = lt ? key : L1;
}

/* the candidate tests of one cell: its two inline records (quantized bounds; absent ones are never
   candidates), then its overflow records (float, rare); code1 receives the winner's rect index */
template <bool Staged = false>
__device__ __forceinline__ void grid_cell_tests(const BakeArgs &a, const char *lds, const GridCell &c, float f,
                                                float uh, float vh, uint32_t qu, uint32_t qv, float &L1, float &L2,
                                                int &code1, unsigned &ntest) {
    /* (the closed-box scans' cells: grid_code_or is the hybrid scan's, whose grid walk reads the float cells) */
    ntest += (unsigned)c.count;
    grid_recq(f, qu, qv, c.qu0, c.qv0, c.idx0, L1, L2, code1);
    grid_recq(f, qu, qv, c.qu1, c.qv1, c.idx1, L1, L2, code1);
    if (c.count > 2) {
        if (Staged || uni(a.grecs_off) >= 0) { /* the overflow records staged beside the cells */
            typedef float f4v __attribute__((ext_vector_type(4)));
            const __attribute__((address_space(3))) char *l = (const __attribute__((address_space(3))) char *)lds;
            const __attribute__((address_space(3))) f4v *recs =
                (const __attribute__((address_space(3))) f4v *)(l + a.grecs_off);
            const __attribute__((address_space(3))) int *ix = (const __attribute__((address_space(3))) int *)(l + a.gidx_off);
            for (int k = 2; k < c.count; k++) {
                const f4v r = recs[c.rest + k - 2];
                grid_rec(f, uh, vh, make_float4(r.x, r.y, r.z, r.w), ix[c.rest + k - 2], L1, L2, code1);
            }
        } else {
            const float4 *recs = (const float4 *)a.grecs;
            for (int k = 2; k < c.count; k++)
                grid_rec(f, uh, vh, recs[c.rest + k - 2], a.gridx[c.rest + k - 2], L1, L2, code1);
        }
    }
}

/* The general walks' cell (many planes per scan): the index alone (no 16-bit cell coordinates), and the
   cell's float inline records (GridCellF), as before the 32-B cells: 57 ms against 71 ms on the 30-room
   layout (profiles/r04/s31-s32) */
__device__ __forceinline__ uint32_t grid_cell_idx(const float4 g0, const float4 g1, const float4 g2, float uh, float vh) {
    const float tu = __builtin_amdgcn_fmed3f((uh - g0.y) * g0.w, 0.0f, g1.y);
    const float tv = __builtin_amdgcn_fmed3f((vh - g0.z) * g1.x, 0.0f, g1.z);
    return (uint32_t)__float_as_int(g2.y) + __umul24((uint32_t)tv, (uint32_t)__float_as_int(g1.w)) + (uint32_t)tu;
}
__device__ __forceinline__ void grid_cell_tests_f(const BakeArgs &a, uint32_t ci, float f, float uh, float vh,
                                                  float &L1, float &L2, int &code1, unsigned &ntest) {
    typedef float f4v __attribute__((ext_vector_type(4)));
    const gptr<f4v> cp = (gptr<f4v>)a.gcellsF + 3 * ci;
    const f4v r0 = cp[0], r1 = cp[1], r2 = cp[2];
    const int count = __float_as_int(r2.x), idx0 = __float_as_int(r2.y), idx1 = __float_as_int(r2.z),
              rest = __float_as_int(r2.w);
    ntest += (unsigned)count;
    grid_rec(f, uh, vh, make_float4(r0.x, r0.y, r0.z, r0.w), idx0 | a.grid_code_or, L1, L2, code1);
    grid_rec(f, uh, vh, make_float4(r1.x, r1.y, r1.z, r1.w), idx1 | a.grid_code_or, L1, L2, code1);
    if (count > 2) {
        const float4 *recs = (const float4 *)a.grecs;
        for (int k = 2; k < count; k++)
            grid_rec(f, uh, vh, recs[rest + k - 2], a.gridx[rest + k - 2] | a.grid_code_or, L1, L2, code1);
    }
}

/*
 * Phase 1 of ScanGrid on the planes of axis A: per facing plane, fac' and the hit point once, the cell
 * it falls in, and the records of that cell (the first two loaded together with no wait in between).
 * The LDS image holds, per axis, pairs {+A plane j, -A plane j} of 64-B GridPlane records; a lane reads
 * the one its direction faces. Planes run nearest-first along the lane's direction, so the planes
 * behind it are a prefix (fac' is monotone in the plane coordinate): a binary search skips them. A hit
 * point outside the box of a plane's records passes none of their tests, so that plane's cell is not
 * loaded.
 */
template <int A>
__device__ __forceinline__ void grid_axis(const BakeArgs &a, const char *lds, int off, int J, f3 s, f3 d, float &L1,
                                          float &L2, int &code1, unsigned &ntest) {
    const char *img = lds + off;
    constexpr int U = (A == 0) ? 1 : 0;
    constexpr int V = (A == 2) ? 1 : 2;
    const float sa = comp<A>(s), da = comp<A>(d);
    const float su = comp<U>(s), sv = comp<V>(s), du = comp<U>(d), dv = comp<V>(d);
    const float rd = __builtin_amdgcn_rcpf(da);
    const float4 *p = (const float4 *)__builtin_assume_aligned(img + (da < 0.0f ? 0 : 64), 16);
    int lo = 0, hi = J; /* first plane not behind the photon (padding planes, fac' = NaN, count as not) */
    while (lo < hi) {
        const int mid = (lo + hi) >> 1;
        if ((p[8 * mid].x - sa) * rd < 0.0f) lo = mid + 1;
        else hi = mid;
    }
    for (int j = lo; j < J; j++) {
        const float4 g0 = p[8 * j];
        const float f = (g0.x - sa) * rd;
        if (!(f >= 0.0f)) continue; /* padding plane (NaN) */
        /* the host orders each class nearest-first, so fac' never decreases from here on: past the
           2^-11 band above L1 no later plane can win or decide the separation (grid_phase1_sorted) */
        if (f > L1 * 1.00048828125f) break;
        const float uh = fmaf(du, f, su), vh = fmaf(dv, f, sv);
        const float4 g2 = p[8 * j + 2], g3 = p[8 * j + 3];
        if (uh < g2.z || uh > g2.w || vh < g3.x || vh > g3.y) continue;
        grid_cell_tests_f(a, grid_cell_idx(g0, p[8 * j + 1], g2, uh, vh), f, uh, vh, L1, L2, code1, ntest);
    }
}

/* the first plane of a nearest-first class list that is not behind the photon (binary search; padding
   planes, fac' = NaN, count as not behind), and the fac' of plane j (INFINITY past the list or at padding) */
__device__ __forceinline__ int grid_first_ahead(const float4 *p, int J, float sa, float rd) {
    int lo = 0, hi = J;
    while (lo < hi) {
        const int mid = (lo + hi) >> 1;
        if ((p[8 * mid].x - sa) * rd < 0.0f) lo = mid + 1;
        else hi = mid;
    }
    return lo;
}
__device__ __forceinline__ float grid_plane_fac(const float4 *p, int j, int J, float sa, float rd) {
    const float f = j < J ? (p[8 * j].x - sa) * rd : INFINITY;
    return f >= 0.0f ? f : INFINITY;
}

/*
 * Phase 1 of ScanGrid on the x and y planes of a layout together: the two nearest-first class lists a
 * lane faces are merged by fac', so the walk visits the walls' planes in increasing distance and stops
 * at the first one (of either axis) past the 2^-11 band above L1. Every plane with fac' in the band is
 * visited, which is grid_phase1_sorted's exactness argument; a wall hit lowers L1 early, so the far
 * planes of the other axis are never visited (the per-axis walks visit them until L1 of the floor or
 * ceiling). x planes: u = y, v = z; y planes: u = x, v = z.
 */
__device__ __forceinline__ void grid_xy_merged(const BakeArgs &a, const char *lds, f3 s, f3 d, float &L1, float &L2,
                                               int &code1, unsigned &ntest) {
    const int Jx = a.fJ[0], Jy = a.fJ[1];
    const float rx = __builtin_amdgcn_rcpf(d.x), ry = __builtin_amdgcn_rcpf(d.y);
    const float4 *px = (const float4 *)__builtin_assume_aligned(lds + (d.x < 0.0f ? 0 : 64), 16);
    const float4 *py = (const float4 *)__builtin_assume_aligned(lds + 128 * Jx + (d.y < 0.0f ? 0 : 64), 16);
    int jx = grid_first_ahead(px, Jx, s.x, rx), jy = grid_first_ahead(py, Jy, s.y, ry);
    float fx = grid_plane_fac(px, jx, Jx, s.x, rx), fy = grid_plane_fac(py, jy, Jy, s.y, ry);
    for (;;) {
        const bool ux = fx <= fy;
        const float f = ux ? fx : fy;
        if (!(f < INFINITY) || f > L1 * 1.00048828125f) break; /* both lists done, or past the band */
        const float4 *p = ux ? px + 8 * jx : py + 8 * jy;
        const float uh = fmaf(ux ? d.y : d.x, f, ux ? s.y : s.x), vh = fmaf(d.z, f, s.z);
        const float4 g2 = p[2], g3 = p[3];
        if (!(uh < g2.z || uh > g2.w || vh < g3.x || vh > g3.y)) {
            grid_cell_tests_f(a, grid_cell_idx(p[0], p[1], g2, uh, vh), f, uh, vh, L1, L2, code1, ntest);
        }
        if (ux) {
            jx++;
            fx = grid_plane_fac(px, jx, Jx, s.x, rx);
        } else {
            jy++;
            fy = grid_plane_fac(py, jy, Jy, s.y, ry);
        }
    }
}

/*
 * Phase 1 of ScanGrid for scenes with at most 4 plane slots (the closed boxes: one plane per axis),
 * nearest plane first. A plane contributes keys only at its own fac' f_p (every record on it shares
 * f_p), so the planes are visited in increasing f_p and the visit stops at the first plane with
 * f_p > L1 * (1 + 2^-11). Why that cannot change the scan's result: every skipped key exceeds
 * L1 (1 + 2^-11) > f (1 + 2^-12) for the winner's exact fac f (|f - L1| <= 2^-20 L1), so
 *   - the winner is not among them (L1 only decreases), and
 *   - the separation test `L2 > f (1 + 2^-12)` has the same outcome with or without them.
 * In a box the nearest facing plane holds the hit, so one cell lookup per scan instead of three.
 */
__device__ __forceinline__ void grid_phase1_sorted(const BakeArgs &a, const char *img, f3 s, f3 d, float &L1,
                                                   float &L2, int &code1, unsigned &ntest) {
    const int J0 = a.fJ[0], J01 = a.fJ[0] + a.fJ[1], JT = J01 + a.fJ[2];
    const float rx = __builtin_amdgcn_rcpf(d.x), ry = __builtin_amdgcn_rcpf(d.y), rz = __builtin_amdgcn_rcpf(d.z);
    float fk[4];
    int qk[4];
#pragma unroll
    for (int k = 0; k < 4; k++) { /* fac' of every slot's facing plane: 1 LDS read + 2 VALU */
        const int q = k < JT ? k : 0;
        const bool ax0 = q < J0, ax1 = !ax0 && q < J01;
        const float sa = ax0 ? s.x : (ax1 ? s.y : s.z), da = ax0 ? d.x : (ax1 ? d.y : d.z);
        const float rd = ax0 ? rx : (ax1 ? ry : rz);
        const float plane = *(const float *)(img + 128 * q + (da < 0.0f ? 0 : 64));
        const float f = (plane - sa) * rd;
        fk[k] = (k < JT && f >= 0.0f) ? f : INFINITY; /* behind, NaN or padding: no candidate */
        qk[k] = q;
    }
    /* sort the 4 (f, slot) pairs ascending: 5 compare-exchanges */
#define FMGI_CX(i, j)                                                                                  \
    {                                                                                                  \
        const bool sw = fk[j] < fk[i];                                                                 \
        const float tf = sw ? fk[j] : fk[i];                                                           \
        fk[j] = sw ? fk[i] : fk[j];                                                                    \
        fk[i] = tf;                                                                                    \
        const int tq = sw ? qk[j] : qk[i];                                                             \
        qk[j] = sw ? qk[i] : qk[j];                                                                    \
        qk[i] = tq;                                                                                    \
    }
    FMGI_CX(0, 1) FMGI_CX(2, 3) FMGI_CX(0, 2) FMGI_CX(1, 3) FMGI_CX(1, 2)
#undef FMGI_CX
    for (int k = 0; k < 4; k++) {
        const float f = fk[k];
        if (!(f < INFINITY) || f > L1 * 1.00048828125f) break; /* 1 + 2^-11 */
        const int q = qk[k];
        const bool ax0 = q < J0, ax1 = !ax0 && q < J01;
        const float da = ax0 ? d.x : (ax1 ? d.y : d.z);
        const float su = ax0 ? s.y : s.x, sv = (ax0 || ax1) ? s.z : s.y;
        const float du = ax0 ? d.y : d.x, dv = (ax0 || ax1) ? d.z : d.y;
        const float4 *p = (const float4 *)__builtin_assume_aligned(img + 128 * q + (da < 0.0f ? 0 : 64), 16);
        const float4 g0 = p[0], g1 = p[1], g2 = p[2];
        const float uh = fmaf(du, f, su), vh = fmaf(dv, f, sv);
        grid_cell_tests_f(a, grid_cell_idx(g0, g1, g2, uh, vh), f, uh, vh, L1, L2, code1, ntest);
    }
}

/*
 * Phase 1 of ScanGrid when each axis has exactly one plane per class (the closed boxes): slot a of the
 * image is axis a, so no slot-to-axis selects. The nearest facing plane is visited first; the two others
 * only when their fac' is within the 2^-11 band above the current L1 (rare: a hit next to an edge).
 * Why the visit order cannot change the result: every plane holding a key below L1 (1 + 2^-11) is
 * visited (a skipped plane's f exceeds the current L1 band, and L1 only decreases), so L1 and the winner
 * are the minimum over all planes; a skipped key exceeds L1 (1 + 2^-11) > f (1 + 2^-12) for the
 * winner's exact fac f, so the separation test `L2 > f (1 + 2^-12)` has the same outcome with or
 * without it (grid_phase1_sorted's argument); equal keys fail that test whatever the order.
 */
/* the candidate tests of compact cell ci (CellC: up to four rect indices, absent ones the never-valid dummy):
   every index's float filter extents {cu, hwu, cv, hwv} from the LDS table by rect index, tested as the float
   cells' records are (grid_rec); the four reads are issued together, with no branch */
__device__ __forceinline__ void grid_cell_tests_c(const BakeArgs &a, const char *lds, uint32_t ci, float f, float uh,
                                                  float vh, float &L1, float &L2, int &code1, unsigned &ntest) {
    typedef const __attribute__((address_space(3))) char *lp;
    typedef uint32_t u2v __attribute__((ext_vector_type(2)));
    typedef float f4v __attribute__((ext_vector_type(4)));
    const u2v c = *(const __attribute__((address_space(3))) u2v *)((lp)lds + a.cellc_off + 8u * ci);
    const __attribute__((address_space(3))) f4v *R = (const __attribute__((address_space(3))) f4v *)((lp)lds + a.recf_off);
    const uint32_t i0 = c.x & 0xFFFFu, i1 = c.x >> 16, i2 = c.y & 0xFFFFu, i3 = c.y >> 16;
    const f4v r0 = R[i0], r1 = R[i1], r2 = R[i2], r3 = R[i3];
    const uint32_t D = (uint32_t)uni(a.cdummy);
    ntest += (unsigned)(i0 != D) + (unsigned)(i1 != D) + (unsigned)(i2 != D) + (unsigned)(i3 != D);
    grid_rec(f, uh, vh, make_float4(r0.x, r0.y, r0.z, r0.w), (int)i0, L1, L2, code1);
    grid_rec(f, uh, vh, make_float4(r1.x, r1.y, r1.z, r1.w), (int)i1, L1, L2, code1);
    grid_rec(f, uh, vh, make_float4(r2.x, r2.y, r2.z, r2.w), (int)i2, L1, L2, code1);
    grid_rec(f, uh, vh, make_float4(r3.x, r3.y, r3.z, r3.w), (int)i3, L1, L2, code1);
}

template <int A, bool Staged, bool Compact = false>
__device__ __forceinline__ void grid_axes_visit(const BakeArgs &a, const char *img, f3 s, f3 d, float f, float &L1,
                                                float &L2, int &code1, unsigned &ntest) {
    constexpr int U = (A == 0) ? 1 : 0;
    constexpr int V = (A == 2) ? 1 : 2;
    const float4 *p = (const float4 *)__builtin_assume_aligned(img + 128 * A + (comp<A>(d) < 0.0f ? 0 : 64), 16);
    const float uh = fmaf(comp<U>(d), f, comp<U>(s)), vh = fmaf(comp<V>(d), f, comp<V>(s));
    if (Compact) {
        grid_cell_tests_c(a, img, grid_cell_idx(p[0], p[1], p[2], uh, vh), f, uh, vh, L1, L2, code1, ntest);
        return;
    }
    uint32_t qu, qv;
    const uint32_t ci = grid_cell(p[0], p[1], p[2], uh, vh, qu, qv);
    grid_cell_tests<Staged>(a, img, load_cell<Staged>(a, img, ci), f, uh, vh, qu, qv, L1, L2, code1, ntest);
}

template <bool Staged, bool Compact = false>
__device__ __forceinline__ void grid_phase1_axes(const BakeArgs &a, const char *img, f3 s, f3 d, float &L1,
                                                 float &L2, int &code1, unsigned &ntest) {
    const float fx0 = (*(const float *)(img + (d.x < 0.0f ? 0 : 64)) - s.x) * __builtin_amdgcn_rcpf(d.x);
    const float fy0 = (*(const float *)(img + 128 + (d.y < 0.0f ? 0 : 64)) - s.y) * __builtin_amdgcn_rcpf(d.y);
    const float fz0 = (*(const float *)(img + 256 + (d.z < 0.0f ? 0 : 64)) - s.z) * __builtin_amdgcn_rcpf(d.z);
    const float fx = fx0 >= 0.0f ? fx0 : INFINITY, fy = fy0 >= 0.0f ? fy0 : INFINITY; /* behind or NaN */
    const float fz = fz0 >= 0.0f ? fz0 : INFINITY;
    /* the nearest plane (axis m at fac' fm), with the per-axis values selected once */
    const bool my = fy < fx;
    const float fxy = my ? fy : fx;
    const bool mz = fz < fxy;
    const float fm = mz ? fz : fxy;
    if (!(fm < INFINITY)) return;
    {
        const int m = mz ? 2 : (my ? 1 : 0);
        const float dm = mz ? d.z : (my ? d.y : d.x);
        const float su = (m == 0) ? s.y : s.x, sv = mz ? s.y : s.z;
        const float du = (m == 0) ? d.y : d.x, dv = mz ? d.y : d.z;
        const float4 *p = (const float4 *)__builtin_assume_aligned(img + 128 * m + (dm < 0.0f ? 0 : 64), 16);
        const float uh = fmaf(du, fm, su), vh = fmaf(dv, fm, sv);
        if (Compact) {
            grid_cell_tests_c(a, img, grid_cell_idx(p[0], p[1], p[2], uh, vh), fm, uh, vh, L1, L2, code1, ntest);
        } else {
            uint32_t qu, qv;
            const uint32_t ci = grid_cell(p[0], p[1], p[2], uh, vh, qu, qv);
            grid_cell_tests<Staged>(a, img, load_cell<Staged>(a, img, ci), fm, uh, vh, qu, qv, L1, L2, code1, ntest);
        }
    }
    const int m = mz ? 2 : (my ? 1 : 0); /* the others, within the band above the current L1 (1 + 2^-11) */
    if (m != 0 && fx < INFINITY && fx <= L1 * 1.00048828125f) grid_axes_visit<0, Staged, Compact>(a, img, s, d, fx, L1, L2, code1, ntest);
    if (m != 1 && fy < INFINITY && fy <= L1 * 1.00048828125f) grid_axes_visit<1, Staged, Compact>(a, img, s, d, fy, L1, L2, code1, ntest);
    if (m != 2 && fz < INFINITY && fz <= L1 * 1.00048828125f) grid_axes_visit<2, Staged, Compact>(a, img, s, d, fz, L1, L2, code1, ntest);
}

/* calls fn(idx) for the rect index of every record that passes grid_axis's candidate test */
template <int A, bool FloatCells, class F>
__device__ __forceinline__ void grid_visit(const BakeArgs &a, const char *lds, int off, int J, f3 s, f3 d, F &&fn) {
    const char *img = lds + off;
    constexpr int U = (A == 0) ? 1 : 0;
    constexpr int V = (A == 2) ? 1 : 2;
    const float sa = comp<A>(s), da = comp<A>(d);
    const float su = comp<U>(s), sv = comp<V>(s), du = comp<U>(d), dv = comp<V>(d);
    const float rd = __builtin_amdgcn_rcpf(da);
    const float4 *p = (const float4 *)__builtin_assume_aligned(img + (da < 0.0f ? 0 : 64), 16);
    const float4 *recs = (const float4 *)a.grecs;
    for (int j = 0; j < J; j++) {
        const float4 g0 = p[8 * j], g1 = p[8 * j + 1], g2 = p[8 * j + 2];
        const float f = (g0.x - sa) * rd;
        if (!(f >= 0.0f)) continue;
        const float uh = fmaf(du, f, su), vh = fmaf(dv, f, sv);
        int count, rest;
        if (FloatCells) { /* the general walks' cells (GridCellF): the same float tests as their phase 1 */
            typedef float f4v __attribute__((ext_vector_type(4)));
            const gptr<f4v> cp = (gptr<f4v>)a.gcellsF + 3 * grid_cell_idx(g0, g1, g2, uh, vh);
            const f4v r0 = cp[0], r1 = cp[1], r2 = cp[2];
            count = __float_as_int(r2.x), rest = __float_as_int(r2.w);
            if (count > 0 && (int)(fabsf(uh - r0.x) <= r0.y) & (int)(fabsf(vh - r0.z) <= r0.w)) fn(__float_as_int(r2.y));
            if (count > 1 && (int)(fabsf(uh - r1.x) <= r1.y) & (int)(fabsf(vh - r1.z) <= r1.w)) fn(__float_as_int(r2.z));
        } else {
            uint32_t qu, qv;
            const GridCell c = load_cell(a, lds, grid_cell(g0, g1, g2, uh, vh, qu, qv));
            count = c.count, rest = c.rest;
            if (c.count > 0 && grid_qpass(qu, qv, c.qu0, c.qv0)) fn(c.idx0);
            if (c.count > 1 && grid_qpass(qu, qv, c.qu1, c.qv1)) fn(c.idx1);
        }
        for (int k = 2; k < count; k++) {
            const float4 r = recs[rest + k - 2];
            if ((int)(fabsf(uh - r.x) <= r.y) & (int)(fabsf(vh - r.z) <= r.w)) fn(a.gridx[rest + k - 2]);
        }
    }
}

/* Axes = true: the closed-box specialisation (one plane per axis and class, BakeArgs::grid_axes), whose
   kernel holds grid_phase1_axes alone: the general kernel's register and SGPR budget is set by its layout
   walks, and its spilled SGPRs come back as v_readlane in the box scan too */
template <bool Axes, bool Staged = false, bool Compact = false>
struct ScanGridT {
    static_assert(!Compact || (Axes && Staged), "the compact tables exist for the staged closed-box instance");
    static constexpr bool kLds = true;
    static constexpr bool kCoop = false;
    /* Compact: one 1024-lane workgroup per CU holds the ~150 KB of compact tables, i.e. 4 waves per SIMD, so the
       instance takes the registers of 4 */
    static constexpr int kWaves = Compact ? 4 : 0;
    /* Staged (closed boxes whose walls, emitters, grid cells and the cells' overflow records the plan stages
       in LDS): the global-memory paths of those tables are compiled out, so the bake loop issues no global
       load but its rare fallbacks' and work-item fetches' */
    static constexpr bool kStaged = Staged;
    static constexpr int kMinWaves = 4; /* k_bake occupancy floor for the register allocator */
    static constexpr int kOrderedRounds = 12;

    /*
     * The literal scan (photonmap.cl:189-206) restricted to the phase-1 candidates, in rect-index order.
     * A rect outside V returns -1 from intersects() whatever `closest` is, so skipping it cannot change
     * the result; the candidates are a superset of V, so this equals ScanExact. Each round finds the next
     * candidate index by re-walking the cells (typically 2-3 candidates: a tie on a shared edge).
     */
    static __device__ int ordered_exact(const BakeArgs &a, const char *lds, f3 src, f3 dir, float &best) {
        int prev = -1, hit = -1;
        float closest = INFINITY;
        for (int round = 0; round < kOrderedRounds; round++) {
            int nxt = INT_MAX;
            auto take = [&](int idx) { nxt = (idx > prev && idx < nxt) ? idx : nxt; };
            /* the closed-box instance knows its plane counts ({1, 1, 1}): constants, not uniform masks
               the register allocator would keep live across the bake loop */
            const int J0 = Axes ? 1 : a.fJ[0], J1 = Axes ? 1 : a.fJ[1], J2 = Axes ? 1 : a.fJ[2];
            grid_visit<0, true>(a, lds, 0, J0, src, dir, take);
            grid_visit<1, true>(a, lds, 128 * J0, J1, src, dir, take);
            grid_visit<2, true>(a, lds, 128 * (J0 + J1), J2, src, dir, take);
            for (int g = 0; g < (Staged ? 0 : uni(a.ngeneral)); g++) { /* (the staged instances: none) */
                const int idx = a.general[g];
                if (idx > prev && idx < nxt && exact_on_v(a.rects, idx, src, dir, INFINITY) >= 0) nxt = idx;
            }
            if (nxt == INT_MAX) {
                best = closest;
                return hit;
            }
            const float d = exact_on_v(a.rects, nxt, src, dir, closest);
            if (d >= 0 && d < closest) {
                closest = d;
                hit = nxt;
            }
            prev = nxt;
        }
        return -2; /* more candidates than rounds: caller runs the full literal scan */
    }

    static __device__ __forceinline__ void scan(const BakeArgs &a, const char *lds, f3 src, f3 dir, HitRec &h,
                                                ScanStats &st) {
        float L1 = INFINITY, L2 = INFINITY;
        /* L2 opaque to the compiler: knowing it infinite, it turns the first record tests' v_med3_f32 into
           v_max_f32 with canonicalising v_max_f32 x, x, x of both operands (two VALU more per record) */
        asm volatile("" : "+v"(L2));
        int code1 = -1;
        unsigned ntest = 0;
        if (Axes) {
            grid_phase1_axes<Staged, Compact>(a, lds, src, dir, L1, L2, code1, ntest);
        } else if (a.fJ[0] + a.fJ[1] + a.fJ[2] <= 4) {
            grid_phase1_sorted(a, lds, src, dir, L1, L2, code1, ntest);
        } else {
            /* floors and ceilings first: in a layout they bound almost every ray, and the x / y walks
               stop at the first plane past L1 (the order of the axes changes neither L1 nor L2; an
               exact tie of keys fails the separation test whatever the order) */
            grid_axis<2>(a, lds, 128 * (a.fJ[0] + a.fJ[1]), a.fJ[2], src, dir, L1, L2, code1, ntest);
            if (a.grid_xy_separate) { /* FMGI_GRID_SEPARATE (experiments): one walk per axis */
                grid_axis<0>(a, lds, 0, a.fJ[0], src, dir, L1, L2, code1, ntest);
                grid_axis<1>(a, lds, 128 * a.fJ[0], a.fJ[1], src, dir, L1, L2, code1, ntest);
            } else {
                grid_xy_merged(a, lds, src, dir, L1, L2, code1, ntest);
            }
        }
        /* rects that are not axis-aligned: exact order-independent tests. The staged and compact instances run
           only for scenes without them (bake_common): compiled out there, since the loop's global loads made
           the compiler wait for vmcnt(0) after it, i.e. for the previous iteration's deposit store (gfx9 counts
           stores in vmcnt), on every scan */
        if (!Staged) {
            cptr<int32_t> G = (cptr<int32_t>)a.general;
            for (int g = 0; g < uni(a.ngeneral); g++) {
                const float f = exact_on_v(a.rects, G[g], src, dir, INFINITY);
                const float key = (f < 0) ? INFINITY : f;
                const bool lt = key < L1;
                L2 = __builtin_amdgcn_fmed3f(L1, key, L2);
                code1 = lt ? G[g] : code1;
                L1 = lt ? key : L1;
            }
            ntest += (unsigned)a.ngeneral;
        }
        st.tests += ntest;
        st.clk.lap(ST_SCAN1);
        if (L1 == INFINITY) {
            h.best = INFINITY;
            h.idx = -1;
            return;
        }
        const int idx = code1; /* rect index of the phase-1 winner */
        const float f = Compact ? exact_hit_compact(a, lds, idx, src, dir, h) : exact_hit<Staged>(a, lds, idx, src, dir, h);
        const bool sep = !(f < 0) && L2 > f * 1.000244140625f; /* ScanFast's separation test */
        st.clk.lap(ST_SCAN2);
        if (sep) {
            h.best = f;
            return;
        }
        if (f < 0) st.invalid++; else st.ties++;
        float best;
        int r = ordered_exact(a, lds, src, dir, best);
        if (r == -2) r = ScanExact::literal<false, Staged && !Compact>(a, lds, src, dir, best, st); /* (compact: global) */
        finish_hit(a, r, best, src, dir, h);
        st.clk.lap(ST_FALLBACK);
    }
};

using ScanGrid = ScanGridT<false>;
using ScanGridAxes = ScanGridT<true>;
using ScanGridAxesStaged = ScanGridT<true, true>;
using ScanGridAxesCompact = ScanGridT<true, true, true>;

/*
 * ScanHybrid's wall pass over the floor plan (Plan = true; tables: fmgi_api.cpp build_plan, which holds
 * the argument why it finds every wall the filter pass would find inside the 2^-11 band). The lane walks
 * the cells its ray crosses seen from above, nearest first, and tests the listed walls of the classes it
 * faces with filter_axis's own float ops, so every key is the filter's bit for bit. A wall listed in
 * several cells of the walk is tested once per cell: its repeat key equals the current winner's only
 * when it is the winner itself (code == code1), and is then dropped, since it would pose as a tie;
 * against L2 or beyond, fmed3 leaves L2 unchanged. The walk stops when the ray leaves a cell past the
 * band above L1, or leaves the grid.
 */
__device__ __forceinline__ void plan_walls(const BakeArgs &a, const char *img, f3 s, f3 d, float &L1, float &L2,
                                           int &code1, unsigned &ntest) {
    const char *pl = img + a.plan_off;
    const float4 h0 = *(const float4 *)__builtin_assume_aligned(pl, 16); /* x0, y0, 1 / cs, cs */
    const int4 h1 = *(const int4 *)__builtin_assume_aligned(pl + 16, 16);
    const int nx = h1.x & 0xFFFF, ny = h1.x >> 16;
    const uint16_t *st = (const uint16_t *)(pl + 32), *en = st + h1.y + 1;
    const int r0y = 2 * a.fJ[0]; /* the first y-wall record */
    const float rx = __builtin_amdgcn_rcpf(d.x), ry = __builtin_amdgcn_rcpf(d.y);
    const int cx = d.x < 0.0f ? 0 : 1, cy = d.y < 0.0f ? 0 : 1; /* faced class per axis; next boundary side */
    int ix = (int)fminf(fmaxf(floorf((s.x - h0.x) * h0.z), 0.0f), (float)(nx - 1));
    int iy = (int)fminf(fmaxf(floorf((s.y - h0.y) * h0.z), 0.0f), (float)(ny - 1));
    const int sx = d.x > 0.0f ? 1 : -1, sy = d.y > 0.0f ? 1 : -1;
    for (int step = nx + ny; step > 0; step--) {
        const int cell = iy * nx + ix;
        const int e = st[cell + 1];
        for (int k = st[cell]; k < e; k++) {
            const int r = en[k];
            const bool ay = r >= r0y;
            if ((r & 1) != (ay ? cy : cx)) continue; /* a wall of the class the lane does not face */
            const float *q = (const float *)(img + 32 * r);
            const float4 q4 = *(const float4 *)__builtin_assume_aligned(q, 16); /* plane, cu, hwu, cv */
            const float hwv = q[4];
            const float f = (q4.x - (ay ? s.y : s.x)) * (ay ? ry : rx);
            const float uu = fmaf(ay ? d.x : d.y, f, ay ? s.x : s.y) - q4.y;
            const float vv = fmaf(d.z, f, s.z) - q4.w;
            const int code = ((ay ? 1 : 0) << 16) | ((r >> 1) - (ay ? a.fJ[0] : 0));
            const int ok = (int)(f >= 0.0f) & (int)(fabsf(uu) <= q4.z) & (int)(fabsf(vv) <= hwv) & (int)(code != code1);
            const float key = ok ? f : INFINITY;
            const bool lt = key < L1;
            L2 = __builtin_amdgcn_fmed3f(L1, key, L2);
            code1 = lt ? code : code1;
            L1 = lt ? key : L1;
            ntest++;
        }
        const float tx = d.x == 0.0f ? INFINITY : (fmaf((float)(ix + cx), h0.w, h0.x) - s.x) * rx;
        const float ty = d.y == 0.0f ? INFINITY : (fmaf((float)(iy + cy), h0.w, h0.y) - s.y) * ry;
        const bool alongx = tx < ty;
        if (!((alongx ? tx : ty) <= L1 * 1.00048828125f)) break; /* past the band (or NaN) */
        if (alongx) {
            ix += sx;
            if ((unsigned)ix >= (unsigned)nx) break;
        } else {
            iy += sy;
            if ((unsigned)iy >= (unsigned)ny) break;
        }
    }
}

/*
 * ScanHybrid: the reference's apartment layouts have few floor/ceiling planes holding many records
 * (one floor and one ceiling rect per room) and walls on many planes. Phase 1 takes the floor/ceiling
 * axis through ScanGrid's cells (one cell lookup instead of a filter pass over every room's floor) and
 * the walls through ScanFast's uniform filter loop. The candidate set is the union of the two scans'
 * candidate sets and the keys are theirs, so phase 2, the separation test and the fallback are
 * ScanFast's. Grid candidates carry the rect index with the 0x40000000 flag (BakeArgs::grid_code_or).
 */
/* Tail (the launch-tail handoff, BakeArgs::tail_*): 0 = the plain instance; 1 = the saving launch (k_bake hands
   its lanes' items off once enough lanes are idle); 2 = the resuming launch, whose groups of BakeArgs::coop lanes
   hold the same photon state and split the wall-pair loop (the floors' grid walk on the group's first lane, so
   every record is tested by exactly one lane and coop_merge's L2 stays the true runner-up) */
template <bool Plan, int Tail = 0>
struct ScanHybridT {
    static_assert(!Plan || Tail == 0, "the floor-plan walk has no tail instances");
    static constexpr bool kLds = true;
    static constexpr bool kCoop = Tail == 2;
    static constexpr int kTail = Tail;
    static constexpr int kMinWaves = 1; /* k_bake occupancy floor for the register allocator */
    static __device__ __forceinline__ void scan(const BakeArgs &a, const char *lds, f3 src, f3 dir, HitRec &h,
                                                ScanStats &st) {
        float L1 = INFINITY, L2 = INFINITY;
        int code1 = -1;
        unsigned ntest = 0;
        const int coop = kCoop ? a.coop : 1, sub = kCoop ? (int)__lane_id() & (coop - 1) : 0;
        if (!kCoop || sub == 0)
            grid_axis<2>(a, lds + uni(a.hyb_off), 128 * (uni(a.gJ[0]) + uni(a.gJ[1])), uni(a.gJ[2]), src, dir, L1,
                         L2, code1, ntest);
        if (Plan) { /* the walls the ray's floor-plan cells list, nearest cells first, after the floors */
            plan_walls(a, lds, src, dir, L1, L2, code1, ntest);
        } else {
#if FMGI_FILTER_PK
            /* the walls: the pair image, two records per packed iteration; codes are rect indices (coop lanes:
               sub-lane `sub` takes groups [sub T, sub T + T) of each axis) */
            const int G0 = uni(a.pG[0]), G1 = uni(a.pG[1]);
            const int T0 = kCoop ? (G0 + coop - 1) / coop : G0, T1 = kCoop ? (G1 + coop - 1) / coop : G1;
            const int s0 = sub * T0, s1 = sub * T1;
            filter_pairs<0>(lds + uni(a.pair_off), s0, s0 + T0 < G0 ? s0 + T0 : G0, src, dir, L1, L2, code1);
            filter_pairs<1>(lds + uni(a.pair_off) + 96 * G0, s1, s1 + T1 < G1 ? s1 + T1 : G1, src, dir, L1, L2, code1);
#else       /* experiments (FMGI_FILTER_PK=0 builds): one record per iteration over the filter image */
            filter_axis<0, kCoop>(lds, a.fJ[0], sub, coop, src, dir, L1, L2, code1);
            filter_axis<1, kCoop>(lds + 64 * a.fJ[0], a.fJ[1], sub, coop, src, dir, L1, L2, code1);
#endif
            ntest += (unsigned)(a.fJ[0] + a.fJ[1]);
        }
        cptr<int32_t> G = (cptr<int32_t>)a.general;
        for (int g = sub; g < uni(a.ngeneral); g += coop) { /* not axis-aligned: exact order-independent tests */
            const float f = exact_on_v(a.rects, G[g], src, dir, INFINITY);
            const float key = (f < 0) ? INFINITY : f;
            const bool lt = key < L1;
            L2 = __builtin_amdgcn_fmed3f(L1, key, L2);
            code1 = lt ? (0x20000000 | g) : code1;
            L1 = lt ? key : L1;
        }
        if (kCoop) coop_merge(coop, L1, L2, code1);
        st.tests += ntest + (uint32_t)a.ngeneral;
        if (L1 == INFINITY) {
            h.best = INFINITY;
            h.idx = -1;
            return;
        }
        /* codes: grid records idx | 0x40000000, general rects g | 0x20000000, the pair filter's walls their
           rect index; the floor plan's walls (A << 16) | position in the filter image */
        int idx;
        if (code1 & 0x40000000) {
            idx = code1 & 0x3FFFFFFF;
        } else if (code1 & 0x20000000) {
            idx = ((gptr<int32_t>)a.general)[code1 & 0x1FFFFFFF];
        } else if (!Plan && FMGI_FILTER_PK) {
            idx = code1;
        } else {
            const int A = code1 >> 16, j = code1 & 0xFFFF;
            const float dA = A == 0 ? dir.x : dir.y;
            const int off = A == 0 ? 0 : 64 * a.fJ[0];
            idx = *(const int32_t *)(lds + off + 64 * j + (dA < 0.0f ? 0 : 32) + 20);
        }
        const float f = exact_hit(a, lds, idx, src, dir, h);
        if (!(f < 0) && L2 > f * 1.000244140625f) { /* ScanFast's separation test */
            h.best = f;
            return;
        }
        if (f < 0) st.invalid++; else st.ties++;
        float best;
        const int hit = ScanExact::literal(a, lds, src, dir, best, st);
        finish_hit(a, hit, best, src, dir, h);
    }
};

using ScanHybrid = ScanHybridT<false>;
using ScanHybridPlan = ScanHybridT<true>;
using ScanHybridTail = ScanHybridT<false, 1>;
using ScanHybridResume = ScanHybridT<false, 2>;

/* ---- accumulation policies -------------------------------------------------------------------- */

/* three exact int64 fixed-point atomics per deposit into lm[texel][0..2] */
struct AccFx3 {
    static __device__ __forceinline__ void deposit(const BakeArgs &a, int texel, int, f3 col) {
        unsigned long long *t = a.lm + 4 * (size_t)texel;
        atomicAdd(t + 0, fx(col.x));
        atomicAdd(t + 1, fx(col.y));
        atomicAdd(t + 2, fx(col.z));
    }
};

/* one u64 count per (colour state, texel): the deposited colour is a function of the state
   (source kind + the floor/non-floor sequence of diffuse bounces, see k_reduce_states) */
struct AccState {
    static __device__ __forceinline__ void deposit(const BakeArgs &a, int texel, int sid, f3) {
        atomicAdd(a.counts + (size_t)sid * a.num_texels + texel, 1ull);
    }
};

/* PROFILING ONLY (FMGI_ACCUM_NONE): deposits are discarded, so a bake measures the tracing work alone.
   The lightmap stays zero; never used for results. */
struct AccNone {
    static __device__ __forceinline__ void deposit(const BakeArgs &, int, int, f3) {}
};

/* Deposits become codes (texel << 10 | colour state) appended to a stream (fmgi_accum.hip folds it).
   The append is a wave-level operation at the end of each loop iteration, where every live lane of the
   wave is active: the depositing lanes get consecutive slots (ballot + mbcnt) in the wave's LDS ring
   (FMGI_RING_CODES + 64 codes), and every time the ring holds FMGI_RING_CODES codes the wave copies them
   to its block of the global stream with 16-B stores. A store per iteration would put its completion
   into the next iteration's s_waitcnt vmcnt (gfx9 counts stores there): the ring makes that one flush per
   ~16 iterations. Global blocks are FMGI_STREAM_BLOCK codes (a multiple of the ring), reserved by one
   lane with an atomic, so a flush always fits the block it starts in. `tot` (codes appended by the wave)
   is monotonic: after the loop the lane that left last holds the current state (finish). */
struct WaveStream {
    uint64_t base = 0, end = 0; /* free part of the wave's current global block */
    uint32_t tot = 0;           /* codes appended; the ring holds tot % FMGI_RING_CODES of them */
};

/* Mode: the stream layout, fixed at compile time (2 = per-tile buckets, the default layout: the kernel
   instance then holds no code and no registers for the other layouts' block cursor and copies) or read
   from BakeArgs::presort (-1: unsorted codes or presorted segments) */
template <int Mode>
struct AccStreamT {
    static __device__ __forceinline__ int layout(const BakeArgs &a) { return Mode >= 0 ? Mode : uni(a.presort); }
    static __device__ __forceinline__ void deposit(const BakeArgs &, int, int, f3) {}
    static __device__ __forceinline__ void init(const BakeArgs &a, uint32_t *ring) {
        if (layout(a) == 2) bucket_init(a, ring);
    }

    /* a fresh global block for the wave (every live lane learns it) */
    static __device__ __forceinline__ void reserve(const BakeArgs &a, WaveStream &ws) {
        const uint64_t live = __ballot(true);
        const int leader = __ffsll((long long)live) - 1;
        unsigned long long nb = 0;
        if ((int)__lane_id() == leader) {
            nb = atomicAdd(a.stream_cursor, (unsigned long long)FMGI_STREAM_BLOCK);
            if (nb + FMGI_STREAM_BLOCK > a.stream_cap) atomicAdd(a.overflow, 1ull);
        }
        nb = __shfl(nb, leader, 64);
        ws.base = nb;
        ws.end = nb + FMGI_STREAM_BLOCK;
        if (ws.end > a.stream_cap) ws.end = ws.base; /* (never by sizing) drop instead of writing out of bounds */
    }

    /* copy ring[0, n) (n <= FMGI_RING_CODES, a multiple of 4) to the block, 16 B per live lane per step */
    static __device__ __forceinline__ void copy_out(const BakeArgs &a, WaveStream &ws, const uint32_t *ring,
                                                    uint32_t n) {
        if (ws.end - ws.base < n) reserve(a, ws);
        if (ws.end - ws.base < n) return; /* overflow (counted in reserve) */
        const uint64_t live = __ballot(true);
        const uint32_t nl = (uint32_t)__popcll(live);
        const uint32_t r = __builtin_amdgcn_mbcnt_hi((uint32_t)(live >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)live, 0u));
        uint4 *dst = (uint4 *)(a.stream + ws.base);
        for (uint32_t k = r; k < n / 4; k += nl) dst[k] = ((const uint4 *)ring)[k];
        ws.base += n;
    }

    /* presorted stream: write ring[0, n) (n <= FMGI_RING_CODES) to the next FMGI_RING_CODES-code segment of
       the block sorted by fold tile (counting sort in the wave's LDS histogram), and the segment's P + 1
       run offsets to toff. Called where every live lane of the wave is active. */
    static __device__ __forceinline__ void sorted_out(const BakeArgs &a, WaveStream &ws, uint32_t *ring,
                                                      uint32_t n) {
        if (ws.end - ws.base < FMGI_RING_CODES) reserve(a, ws);
        if (ws.end - ws.base < FMGI_RING_CODES) return; /* overflow (counted in reserve) */
        uint32_t *hist = (uint32_t *)ring + FMGI_RING_HIST;
        const uint64_t live = __ballot(true);
        const uint32_t nl = (uint32_t)__popcll(live);
        const uint32_t r = __builtin_amdgcn_mbcnt_hi((uint32_t)(live >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)live, 0u));
        const int P = uni(a.ntiles);
        const uint32_t shift = (uint32_t)uni(a.tile_shift);
        for (uint32_t k = r; k < 64; k += nl) hist[k] = 0;
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        /* every lane owns 16 consecutive codes (1024-code rings) */
        const bool full = nl == 64 && n == FMGI_RING_CODES && FMGI_RING_CODES == 1024;
        uint32_t cr[16]; /* full: the lane's codes, held while the ring is overwritten in sorted order */
        if (full) {
            const uint4 *rq = (const uint4 *)ring + 4 * r;
#pragma unroll
            for (int h = 0; h < 4; h++) {
                const uint4 c = rq[h];
                cr[4 * h] = c.x, cr[4 * h + 1] = c.y, cr[4 * h + 2] = c.z, cr[4 * h + 3] = c.w;
            }
#pragma unroll
            for (int e = 0; e < 16; e++) atomicAdd(&hist[cr[e] >> shift], 1u);
        } else {
            for (uint32_t k = r; k < n; k += nl) atomicAdd(&hist[ring[k] >> shift], 1u);
        }
        __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
        __builtin_amdgcn_wave_barrier();
        uint16_t *to = a.toff + (ws.base / FMGI_RING_CODES) * (uint64_t)(P + 1);
        if (nl == 64) { /* exclusive scan of the P counts, one per lane */
            const uint32_t lane = r;
            const uint32_t v = (int)lane < P ? hist[lane] : 0u;
            uint32_t incl = v;
            for (int off = 1; off < 64; off <<= 1) {
                const uint32_t o = __shfl_up(incl, off, 64);
                if ((int)lane >= off) incl += o;
            }
            if ((int)lane < P) {
                hist[lane] = incl - v;
                to[lane] = (uint16_t)(incl - v);
            }
            if ((int)lane == P) to[P] = (uint16_t)n;
        } else if (r == 0) { /* the tail of the bake, some lanes done: one lane scans */
            uint32_t run = 0;
            for (int t = 0; t < P; t++) {
                const uint32_t c = hist[t];
                hist[t] = run;
                to[t] = (uint16_t)run;
                run += c;
            }
            to[P] = (uint16_t)n;
        }
        __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
        __builtin_amdgcn_wave_barrier();
        uint32_t *dst = a.stream + ws.base;
        if (full) { /* scatter into the ring itself (LDS), then one coalesced copy to the segment */
#pragma unroll
            for (int h = 0; h < 16; h += 8) {
                uint32_t o[8];
#pragma unroll
                for (int e = 0; e < 8; e++) o[e] = atomicAdd(&hist[cr[h + e] >> shift], 1u);
#pragma unroll
                for (int e = 0; e < 8; e++) ring[o[e]] = cr[h + e];
            }
            __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
            __builtin_amdgcn_wave_barrier();
#pragma unroll
            for (int h = 0; h < 4; h++) ((uint4 *)dst)[r + 64 * h] = ((const uint4 *)ring)[r + 64 * h];
        } else {
            for (uint32_t k = r; k < n; k += nl) {
                const uint32_t c = ring[k];
                dst[atomicAdd(&hist[c >> shift], 1u)] = c;
            }
        }
        ws.base += FMGI_RING_CODES;
    }

    /* ---- bucketed stream (BakeArgs::presort == 2) ----
       Every wave keeps, per fold tile, one open FMGI_BUCKET_BLOCK-code block of the pool (its private
       bucket: no other wave writes it). A ring flush sorts the ring by tile and appends each tile's run to
       the wave's bucket of that tile; a bucket that fills is closed (its length recorded) and a fresh block
       is taken with one atomic on the pool cursor, the block's tile recorded beside it. Runs are padded
       with sentinels to a multiple of 4 codes, so every bucket fill is 16-B aligned and a flush is stored
       as whole 16-B quads. The fold lists the blocks by tile and reads them as whole 4-KB runs. Per-wave
       state, in the wave's LDS info table: info[t] = {open block (kNoBlock: none), codes in it, (flush
       temporaries)}. */
    static constexpr uint32_t kNoBlock = 0xFFFFFFFFu;
    static constexpr uint32_t kSent = 0xFFFFFFFFu;
    static constexpr uint32_t BP = FMGI_BUCKET_BLOCK;
    static_assert(FMGI_RING_PAD >= 3 * FMGI_PRESORT_MAX_TILES, "a padded flush must fit the ring");

    static __device__ __forceinline__ uint4 *bucket_info(uint32_t *ring) { return (uint4 *)(ring + FMGI_RING_INFO); }
    /* at the start of the bake: no wave has an open bucket */
    static __device__ __forceinline__ void bucket_init(const BakeArgs &a, uint32_t *ring) {
        uint4 *info = bucket_info(ring);
        for (int t = (int)__lane_id(); t < 64; t += 64)
            info[t] = t == kFree ? make_uint4(0u, 0u, 0u, 0u) : make_uint4(kNoBlock, BP, 0u, kNoBlock);
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
    }
    /* info[kFree] (no tile: P <= 63): the wave's reserved pool blocks {first, count}. Blocks are reserved
       kAllocBatch at a time, so a flush that fills a bucket rarely waits for the pool cursor's returning
       atomic (one per filled bucket before). Every reserved block gets its tile recorded when handed out;
       the ones still reserved when the bake ends are recorded empty (tile 0, length 0), so the fold's
       block lists see every block below the cursor. */
    static constexpr int kFree = 63;
    static constexpr uint32_t kAllocBatch = FMGI_BUCKET_ALLOC;
    static __device__ __forceinline__ void bucket_release(const BakeArgs &a, uint4 fl) {
        for (uint32_t k = (uint32_t)__lane_id(); k < fl.y; k += 64) {
            a.block_tile[fl.x + k] = 0u;
            a.block_len[fl.x + k] = 0u;
        }
    }
    /* a fresh pool block for tile t on every live lane with `need` (kNoBlock if the pool is exhausted:
       never, by sizing). Called where every live lane of the wave is active. */
    static __device__ __forceinline__ uint32_t bucket_alloc(const BakeArgs &a, uint4 *info, bool need, uint32_t t) {
        const uint64_t m = __ballot(need);
        if (m == 0) return kNoBlock;
        const uint32_t n = (uint32_t)__popcll(m);
        const uint32_t rk = __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
        const uint4 fl = info[kFree];
        uint32_t b = need && rk < fl.y ? fl.x + rk : kNoBlock;
        uint4 nf = make_uint4(fl.x + n, fl.y - n, 0u, 0u);
        if (fl.y < n) { /* (uniform) the rest of the batch, then a new batch */
            const uint32_t more = n - fl.y, want = more > kAllocBatch ? more : kAllocBatch;
            const uint64_t live = __ballot(true);
            const int leader = __ffsll((long long)live) - 1;
            unsigned long long nb = 0;
            if ((int)__lane_id() == leader) nb = atomicAdd(a.pool_cursor, (unsigned long long)want);
            nb = __shfl(nb, leader, 64);
            const uint64_t have64 = nb < a.pool_blocks ? a.pool_blocks - nb : 0ull;
            const uint32_t have = (uint32_t)(have64 < want ? have64 : want);
            if (need && rk >= fl.y && rk - fl.y < have) b = (uint32_t)nb + (rk - fl.y);
            const uint32_t used = more < have ? more : have;
            nf = make_uint4(have ? (uint32_t)nb + used : 0u, have - used, 0u, 0u);
        }
        if (b != kNoBlock) a.block_tile[b] = t;
        __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
        __builtin_amdgcn_wave_barrier();
        if ((int)__lane_id() == __ffsll((long long)__ballot(true)) - 1) info[kFree] = nf;
        __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
        __builtin_amdgcn_wave_barrier();
        return b;
    }
    /* the fallback of an exhausted pool: the code's colour, added to the int64 lightmap with device
       atomics (exact, order-free, as AccFx3) */
    static __device__ __forceinline__ void bucket_atomic(const BakeArgs &a, uint32_t code) {
        if (code == kSent) return;
        const uint4 cc = a.colpack[code & 1023];
        unsigned long long *q = a.lm + 4 * (size_t)(code >> 10);
        const unsigned long long r = cc.x;
        atomicAdd(q + 0, r);
        atomicAdd(q + 1, r + (unsigned long long)(long long)(int32_t)cc.y);
        atomicAdd(q + 2, r + (unsigned long long)(long long)(int32_t)cc.z);
    }

    /* place tile t's padded run of pc codes (pc % 4 == 0; ring run start `start`) in the wave's bucket:
       info[t] becomes {first block, offset in it, run start, second block} (the second only when the
       bucket fills up) */
    /* (on the live lanes with `act`; called where every live lane of the wave is active) */
    static __device__ __forceinline__ void bucket_place(const BakeArgs &a, uint4 *info, int t, bool act,
                                                        uint32_t start, uint32_t pc) {
        const uint4 st = act ? info[t] : make_uint4(kNoBlock, BP, 0u, kNoBlock);
        const uint32_t room = BP - st.y; /* 0 without an open bucket (y = BP); a multiple of 4 */
        const bool spill = act && pc > room;
        if (act && st.x != kNoBlock && (pc == room || (spill && room))) a.block_len[st.x] = BP;
        const uint32_t second = bucket_alloc(a, info, spill, (uint32_t)t);
        if (spill && pc - room == BP && second != kNoBlock) a.block_len[second] = BP;
        if (act) info[t] = make_uint4(st.x, st.y, start, spill ? second : kNoBlock);
    }
    /* the code of rank rk (a quad: rk % 4 == 0) in tile t's run goes to ... (info as bucket_place left it) */
    static __device__ __forceinline__ uint32_t *bucket_slot(const BakeArgs &a, uint4 inf, uint32_t rk) {
        const uint32_t room = BP - inf.y;
        const bool first = rk < room;
        const uint32_t blk = first ? inf.x : inf.w;
        return blk == kNoBlock ? nullptr : a.stream + ((uint64_t)blk * BP + (first ? inf.y + rk : rk - room));
    }
    static __device__ __forceinline__ void bucket_store(const BakeArgs &a, uint4 inf, uint32_t rk, uint32_t code) {
        uint32_t *d = bucket_slot(a, inf, rk);
        if (d) *d = code;
        else bucket_atomic(a, code);
    }
    static __device__ __forceinline__ void bucket_store4(const BakeArgs &a, uint4 inf, uint32_t rk, uint4 q) {
        uint4 *d = (uint4 *)bucket_slot(a, inf, rk);
        if (d) {
            *d = q;
        } else {
            bucket_atomic(a, q.x), bucket_atomic(a, q.y), bucket_atomic(a, q.z), bucket_atomic(a, q.w);
        }
    }
    /* ... and the bucket after the run: the first block while the run fit in it, else the second */
    static __device__ __forceinline__ void bucket_advance(uint4 *info, int t, uint32_t pc) {
        const uint4 inf = info[t];
        const uint32_t room = BP - inf.y;
        info[t] = pc <= room ? make_uint4(inf.x, inf.y + pc, 0u, kNoBlock) : make_uint4(inf.w, pc - room, 0u, kNoBlock);
    }

    /* bucketed stream: append ring[0, n) to the wave's tile buckets. With every lane live (the common
       case), each lane holds 16 codes while an LDS histogram counts them per tile, a scan of the padded
       counts gives each tile's run start, the codes are scattered back into the ring sorted by tile (the
       pads filled with sentinels; the ring's overflow, which the padded runs may cover, is kept in a
       register meanwhile), the lane of tile t places the run in its bucket (bucket_place), and the lanes
       store the sorted ring as 16-B quads, consecutive lanes to consecutive quads of one run. With lanes
       already done (the bake's tail) the ring is not sorted: each code takes its rank in its run from a
       second pass over the histogram and is stored alone. Called where every live lane of the wave is
       active. */
    static __device__ __forceinline__ void bucket_out(const BakeArgs &a, uint32_t *ring, uint32_t n) {
        uint32_t *hist = ring + FMGI_RING_HIST;
        uint4 *info = bucket_info(ring);
        const uint64_t live = __ballot(true);
        const uint32_t nl = (uint32_t)__popcll(live);
        const uint32_t r = __builtin_amdgcn_mbcnt_hi((uint32_t)(live >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)live, 0u));
        const int P = uni(a.ntiles);
        const uint32_t shift = (uint32_t)uni(a.tile_shift);
        for (uint32_t t = r; t < 64; t += nl) hist[t] = 0;
        __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
        __builtin_amdgcn_wave_barrier();
        if (nl == 64) {
            constexpr int CPL = FMGI_RING_CODES / 64; /* codes per lane of a full ring */
            static_assert(CPL % 4 == 0, "rings of a multiple of 256 codes");
            constexpr int SC = CPL < 8 ? CPL : 8;     /* scatter group */
            uint32_t cr[CPL];
            if (n == FMGI_RING_CODES) {
                const uint4 *rq = (const uint4 *)ring + (CPL / 4) * r;
#pragma unroll
                for (int h = 0; h < CPL / 4; h++) {
                    const uint4 c = rq[h];
                    cr[4 * h] = c.x, cr[4 * h + 1] = c.y, cr[4 * h + 2] = c.z, cr[4 * h + 3] = c.w;
                }
            } else {
#pragma unroll
                for (int e = 0; e < CPL; e++) cr[e] = CPL * r + e < n ? ring[CPL * r + e] : kSent;
            }
            const uint32_t ov = ring[FMGI_RING_CODES + r]; /* the overflow (append moves it after the flush) */
            /* counts and ranks in FMGI_SUBHIST histograms, lane mod FMGI_SUBHIST each: the adds of one
               instruction meet on fewer equal addresses (46 tiles under 64 lanes, a same-address LDS
               atomic serialises) */
            constexpr int NS = FMGI_SUBHIST > 1 ? FMGI_SUBHIST : 1;
            uint32_t *sub = NS > 1 ? ring + FMGI_RING_SUB : hist;
            uint32_t *mine = sub + (NS > 1 ? 64 * (r % NS) : 0);
            if (NS > 1) {
#pragma unroll
                for (int g = 0; g < NS; g++) sub[64 * g + r] = 0u;
                __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
                __builtin_amdgcn_wave_barrier();
            }
#pragma unroll
            for (int e = 0; e < CPL; e++)
                if (cr[e] != kSent) atomicAdd(&mine[cr[e] >> shift], 1u);
            __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
            __builtin_amdgcn_wave_barrier();
            uint32_t cg[NS], cnt = 0; /* lane t: tile t's count in each histogram */
#pragma unroll
            for (int g = 0; g < NS; g++) {
                cg[g] = (int)r < P ? sub[64 * g + r] : 0u;
                cnt += cg[g];
            }
            const uint32_t pc = (cnt + 3u) & ~3u;
            uint32_t incl = pc;
            for (int off = 1; off < 64; off <<= 1) {
                const uint32_t o = __shfl_up(incl, off, 64);
                if ((int)r >= off) incl += o;
            }
            const uint32_t start = incl - pc, quads = __shfl(incl, 63, 64) >> 2;
            if ((int)r < P) {
                uint32_t run = start;
#pragma unroll
                for (int g = 0; g < NS; g++) {
                    sub[64 * g + r] = run;
                    run += cg[g];
                }
            }
            __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
            __builtin_amdgcn_wave_barrier();
#pragma unroll
            for (int h = 0; h < CPL; h += SC) {
                uint32_t o[SC];
#pragma unroll
                for (int e = 0; e < SC; e++)
                    o[e] = cr[h + e] != kSent ? atomicAdd(&mine[cr[h + e] >> shift], 1u) : 0u;
#pragma unroll
                for (int e = 0; e < SC; e++)
                    if (cr[h + e] != kSent) ring[o[e]] = cr[h + e];
            }
            for (uint32_t k = cnt; k < pc; k++) ring[start + k] = kSent;
            bucket_place(a, info, (int)r, cnt != 0, start, pc);
            __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
            __builtin_amdgcn_wave_barrier();
            for (uint32_t q = r; q < quads; q += 64) {
                const uint4 v = ((const uint4 *)ring)[q];
                const uint4 inf = info[v.x >> shift]; /* a run starts with a code: v.x is one */
                bucket_store4(a, inf, 4 * q - inf.z, v);
            }
            __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
            __builtin_amdgcn_wave_barrier();
            if (cnt) bucket_advance(info, (int)r, pc);
            ring[FMGI_RING_CODES + r] = ov;
        } else {
            for (uint32_t k = r; k < n; k += nl) atomicAdd(&hist[ring[k] >> shift], 1u);
            __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
            __builtin_amdgcn_wave_barrier();
            for (int t0 = 0; t0 < P; t0 += (int)nl) { /* (uniform trip count: bucket_place is wave-wide) */
                const int t = t0 + (int)r;
                const uint32_t cnt = t < P ? hist[t] : 0u, pc = (cnt + 3u) & ~3u;
                bucket_place(a, info, t, cnt != 0, 0u, pc);
                if (t < P)
                    for (uint32_t k = cnt; k < pc; k++) bucket_store(a, info[t], k, kSent);
            }
            __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
            __builtin_amdgcn_wave_barrier();
            /* ranks: a second count, from the top (hist[t] counts down to 0) */
            for (uint32_t k = r; k < n; k += nl) {
                const uint32_t code = ring[k], t = code >> shift;
                const uint32_t rk = atomicSub(&hist[t], 1u) - 1u;
                bucket_store(a, info[t], rk, code);
            }
            __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
            __builtin_amdgcn_wave_barrier();
            /* the run lengths again (hist is 0 now): from the codes' tiles */
            for (uint32_t k = r; k < n; k += nl) atomicAdd(&hist[ring[k] >> shift], 1u);
            __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
            __builtin_amdgcn_wave_barrier();
            for (int t = (int)r; t < P; t += (int)nl)
                if (hist[t]) bucket_advance(info, t, (hist[t] + 3u) & ~3u);
        }
        __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
        __builtin_amdgcn_wave_barrier();
    }
    /* at the end of the bake: the open buckets' lengths */
    static __device__ __forceinline__ void bucket_close(const BakeArgs &a, uint32_t *ring) {
        const uint4 *info = bucket_info(ring);
        for (int t = (int)__lane_id(); t < a.ntiles; t += 64) {
            const uint4 inf = info[t];
            if (inf.x != kNoBlock && inf.y < BP) a.block_len[inf.x] = inf.y;
        }
        bucket_release(a, info[kFree]);
    }

    static __device__ __forceinline__ void append(const BakeArgs &a, WaveStream &ws, uint32_t *ring, bool dep,
                                                  uint32_t code) {
        const uint64_t m = __ballot(dep);
        if (m == 0) return;
        const uint32_t n = (uint32_t)__popcll(m);
        const uint32_t r = __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
        const uint32_t fill = ws.tot % FMGI_RING_CODES;
        if (dep) ring[fill + r] = code;
        ws.tot += n;
        if (fill + n < FMGI_RING_CODES) return;
        /* the ring is full: write out its first FMGI_RING_CODES codes, keep the (< 64) rest at its start */
        const int presort = layout(a);
#ifdef FMGI_EXP_NOFLUSH /* PROFILING ONLY: the ring wraps without being written out (the lightmap is lost) */
        if (presort < 0)
#endif
        if (presort == 2) bucket_out(a, ring, FMGI_RING_CODES);
        else if (presort) sorted_out(a, ws, ring, FMGI_RING_CODES);
        else copy_out(a, ws, ring, FMGI_RING_CODES);
        const uint32_t rest = fill + n - FMGI_RING_CODES; /* < n <= live lanes: one code per live lane */
        const uint64_t live = __ballot(true);
        const uint32_t k = __builtin_amdgcn_mbcnt_hi((uint32_t)(live >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)live, 0u));
        const uint32_t v = k < rest ? ring[FMGI_RING_CODES + k] : 0u;
        if (k < rest) ring[k] = v;
    }

    /* after the loop (all lanes of the wave reconverged): take the state of the lane that appended last,
       write out the ring's remaining codes (padded to 16 B with sentinels) and fill the rest of the
       block with sentinels */
    static __device__ __forceinline__ void finish(const BakeArgs &a, WaveStream &ws, uint32_t *ring) {
        uint32_t mx = ws.tot;
        for (int off = 32; off > 0; off >>= 1) {
            const uint32_t o = __shfl_xor(mx, off, 64);
            mx = o > mx ? o : mx;
        }
        const int src = __ffsll((long long)__ballot(ws.tot == mx)) - 1;
        ws.tot = __shfl(ws.tot, src, 64);
        ws.base = __shfl(ws.base, src, 64);
        ws.end = __shfl(ws.end, src, 64);
        const uint32_t fill = ws.tot % FMGI_RING_CODES, padded = (fill + 3) & ~3u;
        const uint32_t lane = __lane_id();
        if (layout(a) == 2) { /* the last (partial) ring into the buckets, then close them */
            if (fill) bucket_out(a, ring, fill);
            bucket_close(a, ring);
            return;
        }
        if (a.presort) { /* the last (partial) ring, then empty run tables for the block's unused segments */
            if (fill) sorted_out(a, ws, ring, fill);
            const int P = a.ntiles;
            for (uint64_t sg = ws.base / FMGI_RING_CODES; sg < ws.end / FMGI_RING_CODES; sg++)
                for (int t = (int)lane; t <= P; t += 64) a.toff[sg * (uint64_t)(P + 1) + t] = 0;
            return;
        }
        for (uint32_t k = fill + lane; k < padded; k += 64) ring[k] = 0xFFFFFFFFu;
        if (padded) copy_out(a, ws, ring, padded);
        for (uint64_t k = ws.base + lane; k < ws.end; k += 64) a.stream[k] = 0xFFFFFFFFu;
    }
};

using AccStream = AccStreamT<-1>; /* unsorted codes / presorted segments (BakeArgs::presort 0, 1) */
using AccSliced = AccStreamT<0>;  /* unsorted codes only (lightmaps of more than 63 tiles): the instance
                                     holds none of the presort / bucket code, whose registers and SGPR
                                     spills made the 30-room layout's bake 16 % slower (profiles/r05/s10) */
using AccBucket = AccStreamT<2>;  /* per-tile buckets (BakeArgs::presort 2) */

#if FMGI_EXPERIMENTS
/*
 * The bucket layout written through per-workgroup tile lines (kAccLines). The per-wave rings cost 6 KB of
 * LDS per wave and a register-hungry flush (each lane holds 16 codes while the ring is sorted), which held
 * the bake to 4 waves/SIMD; tracing alone runs 64 ms at 4 waves and 49 ms at 6 (profiles/r04/s3). Here the
 * workgroup's waves share, per fold tile, a small ring of 16-code lines in LDS (FMGI_LINES_PER_TILE lines):
 *   - a depositing lane reserves the next position of its tile (one LDS atomic), waits until the line
 *     slot holding that position is free (the line FMGI_LINES_PER_TILE back has been written out), stores
 *     its code and counts it into the slot's write counter;
 *   - the lane whose count completes a line (16 codes) writes the line to the tile's bucket in HBM as one
 *     64-B run (4 x 16 B) and frees the slot. The workgroup's lines of a tile fill one pool block after
 *     another (FMGI_BUCKET_BLOCK codes = 64 lines; the lane that takes a block's first line allocates it
 *     with one atomic on the pool cursor and publishes it, tagged with its sequence number, to the lanes of
 *     the other lines of that block);
 *   - after the bake loop (a workgroup barrier), one lane per tile pads its partial line with sentinels,
 *     writes it and records the length of the tile's last block.
 * The blocks are the bucket layout k_bucket_fold reads (blocks listed by tile, runs of codes, sentinels
 * skipped), so the fold is unchanged. Progress: a lane waits only for an older line of its tile, and the
 * oldest unwritten line of a tile waits for nothing, so it completes; every wave spends the wait storing
 * the codes of its other lanes. LDS per workgroup: FMGI_LINES_TILES tiles x (68-dword line ring, padded
 * against bank conflicts across tiles, + counters), 21 KB, against 6 KB per wave for the rings.
 */
#define FMGI_LINES_TILES 64        /* tile slots (bucket layouts have P <= 63 tiles)                 */
#ifndef FMGI_LINES_PER_TILE
#define FMGI_LINES_PER_TILE 4      /* 16-code lines per tile ring (a power of 2)                     */
#endif
#define FMGI_LINES_STRIDE (16 * FMGI_LINES_PER_TILE + 4) /* dwords per tile ring (+4: bank spread across tiles) */
#define FMGI_LINES_BLKSLOTS 8      /* published block ids per tile ({sequence, id}; a slot is reused 8 blocks later) */
#define FMGI_LINES_DWORDS (FMGI_LINES_TILES * (FMGI_LINES_STRIDE + 2 + 2 * FMGI_LINES_PER_TILE + 2 * FMGI_LINES_BLKSLOTS))
#define FMGI_LINES_SPIN (1u << 20) /* bound of every wait (s_sleep 1 each, ~30 ms): past it the bake sets the
                                      overflow flag and stops waiting, so the call fails loudly, never hangs */
struct AccLines {
    static constexpr uint32_t NL = FMGI_LINES_PER_TILE, T = FMGI_LINES_TILES, BP = FMGI_BUCKET_BLOCK;
    static constexpr uint32_t kSent = 0xFFFFFFFFu, kNoBlock = 0xFFFFFFFFu;
    static __device__ __forceinline__ int layout(const BakeArgs &) { return 2; }
    static __device__ __forceinline__ void deposit(const BakeArgs &, int, int, f3) {}
    static constexpr uint32_t NB = FMGI_LINES_BLKSLOTS;
    /* the workgroup's region: [T][68] codes, ctr[T], fill[T], wr[T][NL], fl[T][NL], blk[T][NB] x {tag, id} */
    static __device__ __forceinline__ uint32_t *codes(uint32_t *base) { return base; }
    static __device__ __forceinline__ uint32_t *ctr(uint32_t *base) { return base + T * FMGI_LINES_STRIDE; }
    static __device__ __forceinline__ uint32_t *fillc(uint32_t *base) { return ctr(base) + T; }
    static __device__ __forceinline__ uint32_t *wr(uint32_t *base) { return fillc(base) + T; }
    static __device__ __forceinline__ uint32_t *fl(uint32_t *base) { return wr(base) + T * NL; }
    static __device__ __forceinline__ uint2 *blk(uint32_t *base) { return (uint2 *)(fl(base) + T * NL); }

    static __device__ __forceinline__ void init(const BakeArgs &, uint32_t *base) {
        for (uint32_t i = threadIdx.x; i < T; i += blockDim.x) {
            ctr(base)[i] = 0;
            fillc(base)[i] = 0;
#pragma unroll
            for (uint32_t k = 0; k < NL; k++) {
                wr(base)[i * NL + k] = 0;
                fl(base)[i * NL + k] = k; /* line k may use slot k first */
            }
#pragma unroll
            for (uint32_t k = 0; k < NB; k++) blk(base)[i * NB + k] = make_uint2(kNoBlock, kNoBlock);
        }
        __syncthreads();
    }

    /* write line L of tile t (16 codes in its slot) to the tile's bucket and free the slot */
    static __device__ __forceinline__ void write_line(const BakeArgs &a, uint32_t *base, uint32_t t, uint32_t L) {
        const uint32_t sl = L & (NL - 1);
        const uint4 *src = (const uint4 *)(codes(base) + t * FMGI_LINES_STRIDE + 16 * sl);
        const uint4 q0 = src[0], q1 = src[1], q2 = src[2], q3 = src[3];
        const uint32_t u = __hip_atomic_fetch_add(fillc(base) + t, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        /* the codes are in registers: line L + NL may take the slot */
        __hip_atomic_store(fl(base) + t * NL + sl, L + NL, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
        const uint32_t k = u >> 6, pos = u & 63; /* block k of the workgroup's lines of tile t, line pos in it */
        uint2 *slot = blk(base) + t * NB + (k & (NB - 1));
        uint32_t b = kNoBlock;
        /* The lane of a block's first line allocates it and publishes it; the lanes of its other lines wait
           for that. The publisher may be a lane of this same wave (two lines of one tile completed by one
           append), so its step must come first in program order: two sequential ifs with a reconvergence
           point between them, never an if / else the compiler could lay out waiting branch first. */
        if (pos == 0) {
            const unsigned long long nb = atomicAdd(a.pool_cursor, 1ull);
            b = nb < a.pool_blocks ? (uint32_t)nb : kNoBlock;
            if (b != kNoBlock) {
                a.block_tile[b] = t;
                a.block_len[b] = BP; /* every block but the tile's last is filled; finish() sets the last */
            }
            __hip_atomic_store((unsigned long long *)slot, ((unsigned long long)b << 32) | k, __ATOMIC_RELEASE,
                               __HIP_MEMORY_SCOPE_WORKGROUP);
        }
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        if (pos != 0) {
            unsigned long long v = 0;
            for (uint32_t spin = 0;; spin++) { /* published by the lane of the block's first line */
                v = __hip_atomic_load((unsigned long long *)slot, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP);
                if ((uint32_t)v == k) break;
                if (spin >= FMGI_LINES_SPIN) { /* never: fail the call instead of hanging */
                    atomicAdd(a.overflow, 1ull);
                    return;
                }
                __builtin_amdgcn_s_sleep(1);
            }
            b = (uint32_t)(v >> 32);
        }
        if (b != kNoBlock) {
            uint4 *d = (uint4 *)(a.stream + (uint64_t)b * BP + 16 * pos);
            d[0] = q0, d[1] = q1, d[2] = q2, d[3] = q3;
        } else { /* pool exhausted (never, by sizing): exact atomics into the lightmap */
            const uint32_t c[16] = {q0.x, q0.y, q0.z, q0.w, q1.x, q1.y, q1.z, q1.w,
                                    q2.x, q2.y, q2.z, q2.w, q3.x, q3.y, q3.z, q3.w};
            for (int e = 0; e < 16; e++) AccBucket::bucket_atomic(a, c[e]);
        }
    }

    static __device__ __forceinline__ void append(const BakeArgs &a, WaveStream &, uint32_t *base, bool dep,
                                                  uint32_t code) {
        if (__ballot(dep) == 0) return;
        const uint32_t t = code >> uni(a.tile_shift);
        uint32_t old = 0;
        if (dep) old = __hip_atomic_fetch_add(ctr(base) + t, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        bool pend = dep;
        for (uint32_t spin = 0;; spin++) {
            if (pend && spin >= FMGI_LINES_SPIN) { /* never: fail the call instead of hanging */
                atomicAdd(a.overflow, 1ull);
                pend = false;
            }
            if (pend) {
                const uint32_t L = old >> 4, sl = L & (NL - 1);
                const uint32_t f = __hip_atomic_load(fl(base) + t * NL + sl, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP);
                if (f == L) { /* the slot holds line L: store the code and count it */
                    codes(base)[t * FMGI_LINES_STRIDE + 16 * sl + (old & 15)] = code;
                    const uint32_t w = __hip_atomic_fetch_add(wr(base) + t * NL + sl, 1u, __ATOMIC_ACQ_REL,
                                                              __HIP_MEMORY_SCOPE_WORKGROUP);
                    if ((w & 15) == 15) write_line(a, base, t, L); /* this code completed the line */
                    pend = false;
                }
            }
            if (__ballot(pend) == 0) break;
            __builtin_amdgcn_s_sleep(1);
        }
    }

    /* after the loop: every wave of the workgroup has stored its codes; one lane per tile writes the partial
       line (padded with sentinels) and the length of the tile's last block */
    static __device__ __forceinline__ void finish(const BakeArgs &a, WaveStream &, uint32_t *base) {
        __syncthreads();
        for (uint32_t t = threadIdx.x; t < (uint32_t)a.ntiles; t += blockDim.x) {
            const uint32_t n = ctr(base)[t], r = n & 15;
            if (r) {
                const uint32_t L = n >> 4, sl = L & (NL - 1);
                for (uint32_t k = r; k < 16; k++) codes(base)[t * FMGI_LINES_STRIDE + 16 * sl + k] = kSent;
                write_line(a, base, t, L);
            }
            const uint32_t lines = fillc(base)[t];
            if (lines & 63) {
                const uint2 v = blk(base)[t * NB + (((lines - 1) >> 6) & (NB - 1))];
                if (v.y != kNoBlock) a.block_len[v.y] = (lines & 63) * 16;
            }
        }
    }
};

#endif // FMGI_EXPERIMENTS
/*
 * The bucket layout written straight from the lanes (kAccScatter). The rings of AccStreamT cost 6 KB of LDS
 * per wave and a flush that holds 16 codes per lane while it sorts them (115 VGPRs): the bake ran at 4 waves
 * per SIMD, where tracing alone takes 64 ms on box200 against 49 ms at 6 (profiles/r04/s3). Here nothing is
 * staged: a wave keeps, per fold tile t, one open FMGI_BUCKET_BLOCK-code block of the pool and its fill in a
 * 64-bit LDS word tab[t] = {fill, block} (512 B per wave). A depositing lane takes its slot with one
 * ds_add_rtn_u64 on its tile's word (the lanes of one tile get consecutive ranks) and stores its code at
 * pool[block * BP + rank] with a plain dword store. The rank that reaches BP (rare: ~every 16 iterations per
 * wave) closes the block, takes the next one from the wave's reserved batch (one pool-cursor atomic per
 * FMGI_BUCKET_ALLOC blocks) and resets the word to {ranks past BP, new block}; the lanes past BP store into
 * the new block. A bucket's codes are the prefix [0, fill) of each block, so the blocks are exactly the
 * bucketed layout k_bucket_fold reads (no sentinel pads). The stores land 4 B at a time in ~46 open lines
 * per wave; L2 merges them (write-back, byte masks), so HBM sees whole lines in the common case.
 */
struct AccScatter {
    typedef unsigned long long u64;
    static constexpr uint32_t BP = FMGI_BUCKET_BLOCK, kNoBlock = 0xFFFFFFFFu;
    static constexpr int kFree = 63; /* tab[kFree] = the wave's reserved pool blocks {first, count} */
    static constexpr uint32_t kAllocBatch = FMGI_BUCKET_ALLOC;
    static __device__ __forceinline__ int layout(const BakeArgs &) { return 2; }
    static __device__ __forceinline__ void deposit(const BakeArgs &, int, int, f3) {}
    static __device__ __forceinline__ u64 *tab(uint32_t *base) { return (u64 *)base; }

    static __device__ __forceinline__ void init(const BakeArgs &, uint32_t *base) {
        const uint32_t l = __lane_id();
        /* {fill = BP, no block}: a tile's first code opens its first block */
        tab(base)[l] = l == (uint32_t)kFree ? 0ull : (((u64)kNoBlock << 32) | BP);
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
    }

    /* a fresh pool block for tile t on every live lane with `need` (kNoBlock if the pool is exhausted: never,
       by sizing). Called where every live lane of the wave is active. */
    static __device__ __forceinline__ uint32_t alloc(const BakeArgs &a, u64 *T, bool need, uint32_t t) {
        const uint64_t m = __ballot(need);
        const uint32_t n = (uint32_t)__popcll(m);
        const uint32_t rk = __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
        const u64 fl = T[kFree];
        const uint32_t first = (uint32_t)fl, cnt = (uint32_t)(fl >> 32);
        uint32_t b = need && rk < cnt ? first + rk : kNoBlock;
        uint32_t nfirst = first + n, ncnt = cnt - n;
        if (cnt < n) { /* (uniform) the rest of the batch, then a new batch */
            const uint32_t more = n - cnt, want = more > kAllocBatch ? more : kAllocBatch;
            const uint64_t live = __ballot(true);
            const int leader = __ffsll((long long)live) - 1;
            unsigned long long nb = 0;
            if ((int)__lane_id() == leader) nb = atomicAdd(a.pool_cursor, (unsigned long long)want);
            nb = __shfl(nb, leader, 64);
            const uint64_t have64 = nb < a.pool_blocks ? a.pool_blocks - nb : 0ull;
            const uint32_t have = (uint32_t)(have64 < want ? have64 : want);
            if (need && rk >= cnt && rk - cnt < have) b = (uint32_t)nb + (rk - cnt);
            const uint32_t used = more < have ? more : have;
            nfirst = have ? (uint32_t)nb + used : 0u;
            ncnt = have - used;
        }
        if (b != kNoBlock) a.block_tile[b] = t;
        __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
        __builtin_amdgcn_wave_barrier();
        if ((int)__lane_id() == __ffsll((long long)__ballot(true)) - 1) T[kFree] = ((u64)ncnt << 32) | nfirst;
        __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
        __builtin_amdgcn_wave_barrier();
        return b;
    }

    static __device__ __forceinline__ void append(const BakeArgs &a, WaveStream &, uint32_t *base, bool dep,
                                                  uint32_t code) {
        u64 *T = tab(base);
        const uint32_t t = code >> uni(a.tile_shift);
#if defined(FMGI_SCATTER_EXP) && FMGI_SCATTER_EXP == 2 /* PROFILING ONLY: no slot, no store; the codes xor-ed */
        if (dep) T[64 + (threadIdx.x & 63)] ^= code; /* (a per-lane LDS word past the table: keeps the code live) */
        return;
#endif
        u64 old = 0;
        if (dep) old = __hip_atomic_fetch_add(T + t, 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        uint32_t rank = (uint32_t)old, blk = (uint32_t)(old >> 32);
        const bool full = dep && rank >= BP;
        if (__ballot(full)) { /* (uniform, rare) a block of some tile filled up */
            __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
            __builtin_amdgcn_wave_barrier();
            const bool opener = full && rank == BP; /* one lane per filled tile */
            const uint32_t now = opener ? (uint32_t)T[t] : 0u; /* the fill after every lane's add */
            if (opener && blk != kNoBlock) a.block_len[blk] = BP;
            const uint32_t nb = alloc(a, T, opener, t);
            if (opener) T[t] = ((u64)nb << 32) | (now - BP);
            __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
            __builtin_amdgcn_wave_barrier();
            if (full) {
                blk = (uint32_t)(T[t] >> 32);
                rank -= BP;
            }
        }
#ifdef FMGI_SCATTER_EXP /* PROFILING ONLY: 1 = the slot is taken but the code is not stored (lightmap lost);
                           3 = stored coalesced to a fixed per-wave line instead of the slot */
        if (FMGI_SCATTER_EXP == 1 && code != 0xFFFFFFFEu) return;
        if (FMGI_SCATTER_EXP == 3) {
            if (dep) ((__attribute__((address_space(1))) uint32_t *)a.stream)[(uint64_t)(blockIdx.x * 16 + (threadIdx.x >> 6)) * 64 + (threadIdx.x & 63)] = code;
            return;
        }
#endif
        /* Drain the vector-memory counter BEFORE the store (normally only the previous iteration's store is
           still counted, long since written). Loop-carried registers that some rare path fills with global
           loads (the rect and emitter tables' global fallbacks) otherwise make the compiler wait vmcnt(0) at
           the top of the next iteration, and gfx9 counts stores in vmcnt in issue order: every iteration
           would wait for this store's completion (profiles/r05/s8). */
#ifndef FMGI_SCATTER_DRAIN
#define FMGI_SCATTER_DRAIN 0
#endif
        if (FMGI_SCATTER_DRAIN) __builtin_amdgcn_s_waitcnt(0x0F70); /* vmcnt(0), expcnt / lgkmcnt untouched */
        if (dep) {
#ifdef FMGI_SCATTER_NT /* experiments: non-temporal stores */
            if (blk != kNoBlock) __builtin_nontemporal_store(code, ((__attribute__((address_space(1))) uint32_t *)a.stream) + ((uint64_t)blk * BP + rank));
#else
            if (blk != kNoBlock) ((__attribute__((address_space(1))) uint32_t *)a.stream)[(uint64_t)blk * BP + rank] = code;
#endif
            else AccBucket::bucket_atomic(a, code);
        }
    }

    /* after the loop (every lane of the wave reconverged): the open blocks' lengths, and the reserved blocks
       that were never handed out recorded empty */
    static __device__ __forceinline__ void finish(const BakeArgs &a, WaveStream &, uint32_t *base) {
        const u64 *T = tab(base);
        const uint32_t l = __lane_id();
        if ((int)l < a.ntiles) {
            const u64 v = T[l];
            const uint32_t blk = (uint32_t)(v >> 32), fill = (uint32_t)v;
            if (blk != kNoBlock) a.block_len[blk] = fill < BP ? fill : BP;
        }
        const u64 fl = T[kFree];
        const uint32_t first = (uint32_t)fl, cnt = (uint32_t)(fl >> 32);
        for (uint32_t k = l; k < cnt; k += 64) {
            a.block_tile[first + k] = 0u;
            a.block_len[first + k] = 0u;
        }
    }
};

#if FMGI_EXPERIMENTS
/*
 * The dense stream (kAccDense): the bake only writes, the fold's binning pass (k_bin, fmgi_accum.hip) sorts.
 * At the end of every iteration the depositing lanes of a wave take consecutive slots (ballot + mbcnt) after
 * the wave's running count in its current FMGI_STREAM_BLOCK-code block and store their codes there: one
 * coalesced store of <= 256 B per wave and iteration, no LDS, and as state only the block base and the count
 * (both wave-uniform). A full block is followed by the next one (one cursor atomic per 4096 codes); an
 * iteration whose codes straddle the end splits them over the two. After the loop the rest of the wave's last
 * block is filled with sentinels, so every reserved block is entirely written.
 */
struct AccDense {
    static constexpr uint32_t kSent = 0xFFFFFFFFu, BLK = FMGI_STREAM_BLOCK;
    static __device__ __forceinline__ int layout(const BakeArgs &) { return 3; }
    static __device__ __forceinline__ void deposit(const BakeArgs &, int, int, f3) {}
    static __device__ __forceinline__ void init(const BakeArgs &, uint32_t *) {}
    static __device__ __forceinline__ uint32_t sgpr(uint32_t v) { return __builtin_amdgcn_readfirstlane(v); }
    static __device__ __forceinline__ uint64_t sgpr64(uint64_t v) {
        return ((uint64_t)sgpr((uint32_t)(v >> 32)) << 32) | sgpr((uint32_t)v);
    }
    /* ws.base: the wave's current block, ws.tot: the room left in it (0 at the start: no block); uniform
       over the live lanes, kept in SGPRs. Called where every live lane of the wave is active. */
    static __device__ __forceinline__ void append(const BakeArgs &a, WaveStream &ws, uint32_t *, bool dep,
                                                  uint32_t code) {
        const uint64_t m = __ballot(dep);
        if (m == 0) return;
        const uint32_t n = (uint32_t)__popcll(m);
        const uint32_t r = __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
        const uint32_t room = sgpr(ws.tot);
        const uint64_t base = sgpr64(ws.base);
        uint64_t dst = base + (BLK - room) + r;
        if (n > room) { /* (uniform) the block fills: the rest of the codes start the next one */
            unsigned long long nb = 0;
            if (dep && r == 0) { /* the first depositing lane (a lane below it that does not deposit has r == 0 too) */
                nb = atomicAdd(a.stream_cursor, (unsigned long long)BLK);
                if (nb + BLK > a.stream_cap) atomicAdd(a.overflow, 1ull);
            }
            nb = sgpr64(__shfl(nb, __ffsll((long long)m) - 1, 64));
            if (r >= room) dst = nb + (r - room);
            ws.base = nb;
            ws.tot = BLK - (n - room);
        } else {
            ws.tot = room - n;
        }
        /* (a reservation past the end, never by sizing, is counted and its codes dropped: the call fails) */
        if (dep && dst < a.stream_cap) ((__attribute__((address_space(1))) uint32_t *)a.stream)[dst] = code;
    }
    /* after the loop (every lane of the wave reconverged): the state of the lane that appended last (the
       wave's blocks are reserved in increasing order, so it has the largest base + codes in the block), then
       sentinels in the rest of its block */
    static __device__ __forceinline__ void finish(const BakeArgs &a, WaveStream &ws, uint32_t *) {
        const uint64_t key = ws.tot || ws.base ? ws.base + (BLK - ws.tot) + 1 : 0ull;
        uint64_t mx = key;
        for (int off = 32; off > 0; off >>= 1) {
            const uint64_t o = __shfl_xor(mx, off, 64);
            mx = o > mx ? o : mx;
        }
        if (mx == 0) return; /* the wave appended nothing */
        const int src = __ffsll((long long)__ballot(key == mx)) - 1;
        const uint64_t base = __shfl(ws.base, src, 64);
        const uint32_t room = __shfl(ws.tot, src, 64);
        for (uint32_t k = BLK - room + __lane_id(); k < BLK; k += 64)
            if (base + k < a.stream_cap) ((__attribute__((address_space(1))) uint32_t *)a.stream)[base + k] = kSent;
    }
};

#endif // FMGI_EXPERIMENTS
template <class Acc>
struct HasAppend {
    static constexpr bool value = false;
};
#if FMGI_EXPERIMENTS
template <>
struct HasAppend<AccDense> {
    static constexpr bool value = true;
};
#endif

template <>
struct HasAppend<AccScatter> {
    static constexpr bool value = true;
};
template <int Mode>
struct HasAppend<AccStreamT<Mode>> {
    static constexpr bool value = true;
};
#if FMGI_EXPERIMENTS
template <>
struct HasAppend<AccLines> {
    static constexpr bool value = true;
};
#endif
/* the LDS region of an appending accumulation: the wave's ring (AccStreamT), the workgroup's tile lines
   (AccLines) */
template <class Acc>
__device__ __forceinline__ uint32_t *acc_region(char *lds, const BakeArgs &a) {
    return (uint32_t *)(lds + a.ring_off) + (threadIdx.x >> 6) * FMGI_RING_STRIDE;
}
template <>
__device__ __forceinline__ uint32_t *acc_region<AccBucket>(char *lds, const BakeArgs &a) {
    return (uint32_t *)(lds + a.ring_off) + (threadIdx.x >> 6) * FMGI_RING_STRIDE_BUCKET;
}
#if FMGI_EXPERIMENTS
template <>
__device__ __forceinline__ uint32_t *acc_region<AccLines>(char *lds, const BakeArgs &a) {
    return (uint32_t *)(lds + a.ring_off);
}
#endif
template <>
__device__ __forceinline__ uint32_t *acc_region<AccScatter>(char *lds, const BakeArgs &a) {
    return (uint32_t *)(lds + a.ring_off) + (threadIdx.x >> 6) * FMGI_SCATTER_STRIDE;
}

/* ---- the per-lane photon state machine ------------------------------------------------------- */

/* flattened work item w -> (source, launch, gid): launches of one source are consecutive chunks of
   launch_cap = WG*100 items (global_illumination_cl.c:255), so one search over the (few) sources and a
   division replace a search over all launches */
__device__ __forceinline__ void locate_item(const BakeArgs &a, uint64_t w, int &src, int &li, uint32_t &gid) {
    int lo = 0, hi = uni(a.nsrc) - 1;
    while (lo < hi) {
        const int mid = (lo + hi + 1) >> 1;
        if (a.src_item_begin[mid] <= w) lo = mid; else hi = mid - 1;
    }
    const uint64_t off = w - a.src_item_begin[lo];
    src = lo;
    const uint32_t cap = a.launch_cap;
    if ((off >> 32) == 0) { /* every schedule here: a 32-bit division, not the 64-bit expansion */
        const uint32_t o = (uint32_t)off, q = o / cap;
        li = a.src_launch0[lo] + (int)q;
        gid = o - q * cap;
    } else {
        li = a.src_launch0[lo] + (int)(off / cap);
        gid = (uint32_t)(off % cap);
    }
}

/* the emitter fields photon emission reads (photonmap.cl:173-181 and the sampler basis) */
template <class R>
__device__ __forceinline__ SrcDev src_fields(const R &r) {
    SrcDev d;
    d.px = r.px; d.py = r.py; d.pz = r.pz;
    d.wx = r.wx; d.wy = r.wy; d.wz = r.wz;
    d.hx = r.hx; d.hy = r.hy; d.hz = r.hz;
    d.nx = r.nx; d.ny = r.ny; d.nz = r.nz;
    d.bux = r.bux; d.buy = r.buy; d.buz = r.buz;
    d.bvx = r.bvx; d.bvy = r.bvy; d.bvz = r.bvz;
    return d;
}

/* whether a scan's lanes fetch work items with one atomic per wave (wave_ticket64) rather than one per lane:
   the hybrid scan's launches of a few costly items per lane, +1-2 % on example.png (every lane fetches at
   the launch's start); the grid scans' launches of dozens of items per lane lose 0.1-0.3 % (box200) and
   1 % (box2000) with it (profiles/r06/s14) */
template <class Scan, class = void>
struct ScanFetchAgg {
    static constexpr bool value = false;
};
template <class Scan>
struct ScanFetchAgg<Scan, decltype((void)Scan::kTail)> {
    static constexpr bool value = true;
};

/* the launch-tail mode of a scan instance (ScanHybridT::kTail: 1 saving, 2 resuming), else 0 */
template <class Scan, class = void>
struct ScanTail {
    static constexpr int value = 0;
};
template <class Scan>
struct ScanTail<Scan, decltype((void)Scan::kTail)> {
    static constexpr int value = Scan::kTail;
};

/* a work item in flight as the launch-tail handoff saves it, at a photon boundary (16 B): between two photons
   the position, direction, colour, sample basis, depth and colour state are all dead (the next photon's
   emission sets them), so the item's RNG state, its photons left and its source are the whole state.
   (The item's index and photon number serve the trace kernels only, which have no tail launches.) */
__device__ __forceinline__ void tail_save(uint4 *d, uint32_t rng, int left, int srci, uint32_t scans) {
    *d = make_uint4(rng, (uint32_t)left, (uint32_t)srci, scans);
}
__device__ __forceinline__ void tail_load(const uint4 *d, uint32_t &rng, int &left, int &srci, uint32_t &scans) {
    const uint4 q = *d;
    rng = q.x;
    left = (int)q.y;
    srci = (int)q.z;
    scans = q.w;
}

/* wave_ticket on a 64-bit counter (the work-item queue) */
__device__ __forceinline__ uint64_t wave_ticket64(unsigned long long *ctr, bool on) {
    const uint64_t m = __ballot(on);
    const int leader = __ffsll((long long)m) - 1;
    uint64_t base = 0;
    if ((int)__lane_id() == leader) base = atomicAdd(ctr, (unsigned long long)__popcll(m));
    base = __shfl(base, leader, 64);
    return base + __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
}

/* one device-scope atomicAdd for every lane of the wave that has `on` set (they must all be active here):
   returns each such lane's value old + its rank among them. Many lanes reaching a counter at once (the
   launch-tail saves and resumes) otherwise queue on its one word at the L2's rate for a single address
   (MI355X_MICROARCH.md, dequeue: ~88 per us): 190k saves cost the saving launch 2 ms */
__device__ __forceinline__ uint32_t wave_ticket(unsigned *ctr, bool on) {
    const uint64_t m = __ballot(on);
    if (!m) return 0u;
    const int leader = __ffsll((long long)m) - 1;
    uint32_t base = 0;
    if ((int)__lane_id() == leader) base = atomicAdd(ctr, (unsigned)__popcll(m));
    base = __shfl(base, leader, 64);
    return base + __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
}

/* whether a scan's instance compiles the tables' global paths out (ScanGridT::kStaged) */
template <class Scan, class = void>
struct ScanStaged {
    static constexpr bool value = false;
};
template <class Scan>
struct ScanStaged<Scan, decltype((void)Scan::kStaged)> {
    static constexpr bool value = Scan::kStaged;
};

/* emitter srci: from the workgroup's LDS copy of the SrcDev table when staged (BakeArgs::srcs_off >= 0) */
template <bool Staged = false>
__device__ __forceinline__ SrcDev load_src(const BakeArgs &a, const char *lds, int srci) {
    if (Staged || uni(a.srcs_off) >= 0)
        return src_fields(((const __attribute__((address_space(3))) SrcDev *)(
            (const __attribute__((address_space(3))) char *)lds + a.srcs_off))[srci]);
    return src_fields(((gptr<SrcDev>)a.srcs)[srci]);
}

/* LCG^2: the two draws of a direction sample whose result is never used (last bounce) */
__device__ __forceinline__ uint32_t lcg2(uint32_t s) {
    constexpr uint32_t A2 = kJump.a[2], C2 = kJump.c[2];
    return A2 * s + C2;
}

/*
 * One loop iteration = [start a photon and/or sample a direction] -> [scan] -> [hit: deposit].
 * Emission (photonmap.cl:173-181) and the diffuse bounce (:238) share ONE sample_dir call site, so a
 * wave whose lanes are at different points of their photons (escapes, photonmap.cl:208) pays for one
 * sampler per iteration, not two. The direction sampled at the last bounce (depth 8) is never used:
 * its two draws are skipped with one LCG jump. Per lane, RNG draws happen in exactly the reference
 * order: roulette (:236), bounce sample (:238), then the next photon's dx, dy (:173-174) and sample.
 */
#ifdef FMGI_WAVES_PER_EU /* experiment builds: ask the register allocator for this occupancy */
#define FMGI_BAKE_ATTR __attribute__((amdgpu_waves_per_eu(FMGI_WAVES_PER_EU)))
#else /* ScanGrid: 4 waves/SIMD (108 VGPRs, no spills): with the walls staged, LDS holds a CU to 16 waves anyway;
         AccLines leaves the LDS for 6 (768-lane workgroups, two per CU) and asks for the registers of 6 */
#define FMGI_BAKE_ATTR __attribute__((amdgpu_waves_per_eu(ScanWaves<Scan>::value ? ScanWaves<Scan>::value \
    : (acc_min_waves<Acc>() > Scan::kMinWaves ? acc_min_waves<Acc>() : Scan::kMinWaves))))
#endif
/* a scan instance whose occupancy is fixed by its LDS tables (ScanGridT::kWaves), else 0 */
template <class Scan, class = void>
struct ScanWaves {
    static constexpr int value = 0;
};
template <class Scan>
struct ScanWaves<Scan, decltype((void)Scan::kWaves)> {
    static constexpr int value = Scan::kWaves;
};
template <class Acc>
constexpr int acc_min_waves() { return 1; }
#if FMGI_EXPERIMENTS
template <>
constexpr int acc_min_waves<AccLines>() { return 6; }
#endif
#ifndef FMGI_SCATTER_WAVES /* AccScatter: the registers of this many waves per SIMD (experiment builds: 4, 5, 6) */
#define FMGI_SCATTER_WAVES 6
#endif
template <>
constexpr int acc_min_waves<AccScatter>() { return FMGI_SCATTER_WAVES; }
#if FMGI_EXPERIMENTS
template <>
constexpr int acc_min_waves<AccDense>() { return FMGI_SCATTER_WAVES; }
#endif
template <class Scan, class Acc, bool TRACE>
__global__ __launch_bounds__(1024) FMGI_BAKE_ATTR void k_bake(BakeArgs a) {
    extern __shared__ __attribute__((aligned(16))) char s_img[];
    /* AccStream: this wave's ring of deposit codes, after the scan image in LDS (AccLines: the workgroup's
       tile lines) */
    uint32_t *const ring = acc_region<Acc>(s_img, a);
    if (Scan::kLds) { /* stage the filter image once per workgroup */
        const int n16 = a.fimg_bytes >> 4;
        for (int i = threadIdx.x; i < n16; i += blockDim.x) ((uint4 *)s_img)[i] = ((const uint4 *)a.fimg)[i];
        if (ScanTail<Scan>::value == 1 && threadIdx.x == 0) *(uint32_t *)(s_img + a.tail_flag_off) = 0u;
        __syncthreads();
    }
    if constexpr (HasAppend<Acc>::value)
        Acc::init(a, ring);
    uint32_t rng = 0;
    f3 pos = mkf3(0, 0, 0), dir = mkf3(0, 0, 0), col = mkf3(0, 0, 0);
    f3 sn = mkf3(0, 0, 0), sbu = mkf3(0, 0, 0), sbv = mkf3(0, 0, 0); /* pending diffuse sample basis */
    int depth = 0, left = 0, photon = -1, sid = 0, srci = 0;
    bool win = false, start = true, pend = false;
    uint64_t item = 0;
    int nev = 0;
    /* per-lane counts of one launch, in 32 bits: a lane traces a few dozen work items per launch (the
       grid is occupancy-sized, chunks are memory-sized); scans = deposits + escapes */
    uint32_t n_ph = 0, n_dep = 0, n_esc = 0;
#ifdef FMGI_NO_LANE_STATS /* PROFILING ONLY: the deposit / escape counters compiled out (their registers' cost) */
#define FMGI_LANE_COUNT(x) ((void)0)
#else
#define FMGI_LANE_COUNT(x) (x)
#endif
    ScanStats sst;
    WaveStream ws;
    /* BakeArgs::coop lanes per work item (ScanFast splits each scan's records among them; they keep
       identical photon state): the lead lane fetches, deposits and counts for the group */
    const bool lead = !Scan::kCoop || ((int)__lane_id() & (a.coop - 1)) == 0;

    sst.clk.reset();
#ifdef FMGI_CLOCK_STAMP /* diagnostic build: the in-kernel clock (MI355X_MICROARCH.md, DVFS item 6) */
    const unsigned long long ck_t0 = __builtin_amdgcn_s_memtime(), ck_r0 = __builtin_amdgcn_s_memrealtime();
#endif
    constexpr int kTail = ScanTail<Scan>::value;
    bool tail_saving = false; /* (the saving launch) this lane left the loop to hand its item off */
    uint32_t tail_it = 0;      /* (the saving launch) the wave's iterations, for its turn to poll */
    /* (the resuming launch) the items the saving launch saved: final before this launch started */
    const uint32_t tail_saved = kTail == 2 ? *a.tail_n : 0u;
    for (;;) {
        if constexpr (kTail == 2) {
            /* the resuming launch: a group's lanes take the next saved item instead of a new one (the wave's
               groups that need one take consecutive tickets with one atomic) */
            if (start && left == 0) {
                if (uni(a.src_cost) && lead && photon >= 0)
                    atomicAdd(a.src_cost + srci, (unsigned long long)(n_dep + n_esc));
                uint32_t w = wave_ticket(a.tail_next, lead);
                w = __shfl(w, (int)__lane_id() & ~(a.coop - 1), 64);
                if (w >= tail_saved) break;
                uint32_t done = 0; /* the item's scans in the saving launch */
                tail_load(a.tail_states + w, rng, left, srci, done);
                win = srci < a.nwindows;
                photon = 0; /* (an item in flight: >= 0 for the per-source scan totals) */
                if (uni(a.src_cost) && lead)
                    atomicAdd(a.src_cost + srci, (unsigned long long)done - (unsigned long long)(n_dep + n_esc));
            }
        }
        /* ---- stage 1: new photon (and new work item), then the iteration's one direction sample ---- */
        float edx = 0, edy = 0;
        if (start) {
            if (kTail != 2 && left == 0) {
                if (TRACE && photon >= 0) {
                    a.ev_counts[item - a.item_begin] = nev;
                    a.rng_final[item - a.item_begin] = rng;
                }
                /* the finished item's scans, per source (the host orders the next bake's fetches by them):
                   the lane's running scan count is added here and was subtracted at the item's fetch, so
                   no register holds the item's start count */
                if (uni(a.src_cost) && lead && photon >= 0)
                    atomicAdd(a.src_cost + srci, (unsigned long long)(n_dep + n_esc));
                if (sst.tests && lead) { /* flush this lane's rect-test count (see ScanStats) */
                    atomicAdd(a.stats + KSTAT_TESTS, (unsigned long long)sst.tests);
                }
                sst.tests = 0;
                /* one fetch per work item: by the group's lead lane, broadcast to its coop lanes (the hybrid
                   scan: the wave's leads that fetch in the same iteration take consecutive items with one
                   atomic, ScanFetchAgg) */
                uint64_t w = ScanFetchAgg<Scan>::value ? wave_ticket64(a.counter, lead) : (lead ? atomicAdd(a.counter, 1ull) : 0ull);
                if (Scan::kCoop) w = __shfl(w, (int)__lane_id() & ~(a.coop - 1), 64);
                if (w >= a.item_end - a.item_begin) {
                    if constexpr (kTail == 1) { /* more lanes without work: one atomic per wave */
                        const uint64_t m = __ballot(true);
                        if ((int)__lane_id() == __ffsll((long long)m) - 1) atomicAdd(a.tail_idle, (unsigned)__popcll(m));
                    }
                    break;
                }
                if (uni(a.fetch_nseg) > 0) { /* fetch order: segments of source ranges, costliest items first
                                           (32-bit: the host builds a table only below 2^32 items) */
                    const uint32_t f = (uint32_t)w;
                    int lo = 0, hi = a.fetch_nseg - 1;
                    while (lo < hi) {
                        const int mid = (lo + hi + 1) >> 1;
                        if (a.fetch_tab[2 * mid] <= f) lo = mid; else hi = mid - 1;
                    }
                    w = a.fetch_tab[2 * lo + 1] + (f - a.fetch_tab[2 * lo]);
                } else {
                    w += a.item_begin;
                }
                item = w;
                int li;
                uint32_t gid;
                locate_item(a, w, srci, li, gid);
                if (uni(a.src_cost) && lead) atomicAdd(a.src_cost + srci, 0ull - (unsigned long long)(n_dep + n_esc));
                rng = gid + (uint32_t)a.launches[li].rng_offset; /* photonmap.cl:272 */
                /* photonmap.cl:273-275: r = rand()*40; ceil(r) further draws, as one LCG jump */
                const float r40 = rng_next(rng) * 40;
                const int k = (int)ceilf(r40);
                rng = c_jump.a[k] * rng + c_jump.c[k];
                win = srci < a.nwindows;
                left = FMGI_PHOTONS_PER_ITEM;
                photon = -1;
                nev = 0;
            }
            const SrcDev S = load_src<ScanStaged<Scan>::value>(a, s_img, srci);
            col = win ? mkf3(18, 18, 18) : mkf3(16, 16, 18); /* photonmap.cl:167-169 */
            sid = win ? (512 + 1) : 1; /* colour state: source kind, then one bit per diffuse bounce */
            edx = rng_next(rng);
            edy = rng_next(rng);
            sn = mkf3(S.nx, S.ny, S.nz);
            sbu = mkf3(S.bux, S.buy, S.buz);
            sbv = mkf3(S.bvx, S.bvy, S.bvz);
            left--;
            photon++;
            depth = 0;
            n_ph++;
        }
        sst.clk.lap(ST_START);
        if (start || pend) dir = sample_dir(rng, sn, sbu, sbv, start && win);
        if (start) {
            const SrcDev S = load_src<ScanStaged<Scan>::value>(a, s_img, srci);
            pos = add3(add3(add3(mkf3(S.px, S.py, S.pz), mul3(mkf3(S.wx, S.wy, S.wz), edx)),
                            mul3(mkf3(S.hx, S.hy, S.hz), edy)),
                       mul3(dir, 1e-5f));
        } else {
            pos = add3(pos, mul3(dir, 1e-5f)); /* photonmap.cl:261 (after the diffuse sample or the mirror) */
        }
        start = false;
        pend = false;
        sst.clk.lap(ST_SAMPLE);

        /* ---- stage 2: scan ---- */
        HitRec h;
        Scan::scan(a, s_img, pos, dir, h, sst);
        sst.clk.lap(ST_SCAN1); /* scans without an inner split (ScanExact / ScanFast) */
        bool dep = false;
        uint32_t code = 0;
        /* the basis of a diffuse sample at the top of the next iteration (unused unless pend is set; an
           escaped photon's next sample is an emission, whose basis the start block sets) */
        sn = mkf3(h.nx, h.ny, h.nz);
        sbu = mkf3(h.bux, h.buy, h.buz);
        sbv = mkf3(h.bvx, h.bvy, h.bvz);
        if (h.best == INFINITY) { /* photonmap.cl:208-209 */
            start = true;
            FMGI_LANE_COUNT(n_esc++);
        } else {
        /* ---- stage 3: hit (photonmap.cl:216-258) ---- */
        pos = add3(pos, mul3(dir, h.best));
        const f3 hn = mkf3(h.nx, h.ny, h.nz);
        const int texel = h.base + tile_uv(h.dx, h.dy, h.wl, h.hl, h.iwl, h.ihl, h.W, h.H); /* == tile_at(rect, pos) */
        const bool last = depth + 1 == FMGI_MAX_DEPTH;
        /* (double)pos.z > 0.0005 (photonmap.cl:236) <=> pos.z > the largest float below 0.0005 */
        if (pos.z > 4.99999965541064739227294921875e-4f || rng_next(rng) > 0.75f) {
            const bool floor = pos.z < 1e-5f;
            if (floor) {
                col.y *= 0.85f;
                col.z *= 0.7f;
            }
            col = mul3(col, 0.9f);
            sid = (sid & 512) | ((sid & 511) << 1) | (floor ? 1 : 0);
            if (last) {
                rng = lcg2(rng); /* the direction of a photon that ends here is never used */
            } else {
                pend = true; /* sampled at the top of the next iteration */
            }
        } else {
            const float two = 2.0f * dot3(hn, dir);
            dir = sub3(dir, mul3(hn, two));
        }
        if (lead) Acc::deposit(a, texel, sid, col);
        dep = true;
        code = ((uint32_t)texel << 10) | (uint32_t)sid;
        FMGI_LANE_COUNT(n_dep++);
        if (TRACE) {
            EventDev e;
            e.photon = photon;
            e.depth = depth;
            e.rect = h.idx;
            e.texel = texel;
            e.rgb[0] = col.x;
            e.rgb[1] = col.y;
            e.rgb[2] = col.z;
            e.rng = pend ? lcg2(rng) : rng; /* RNG state after this bounce's sample */
            ((EventDev *)a.events)[(item - a.item_begin) * FMGI_EVENTS_PER_ITEM + nev] = e;
            nev++;
        }
        if (last) start = true;
        depth++;
        }
        sst.clk.lap(ST_HIT);
        if constexpr (HasAppend<Acc>::value) Acc::append(a, ws, ring, dep && lead, code);
        sst.clk.lap(ST_APPEND);
        if constexpr (kTail == 1) {
            /* the launch tail: once tail_at lanes of the launch found no work item left, a lane whose photon just
               ended saves its item for the resuming launch and leaves (a lane between items fetches at the next
               iteration: none left, so it goes idle). The workgroup reads the idle count from its LDS copy,
               which each wave refreshes from the global counter once in 64 of its iterations, the waves of a
               workgroup in turn: a poll is a vector load, and its wait on gfx950 also waits for the wave's
               scattered deposit stores (a poll per photon start cost the loop a fifth of its speed) */
            uint32_t *seen = (uint32_t *)(s_img + a.tail_flag_off);
            if (((tail_it++ + 8u * (threadIdx.x >> 6)) & 63u) == 0u)
                *(volatile uint32_t *)seen = __hip_atomic_load(a.tail_idle, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            if (start && left > 0 && *(volatile uint32_t *)seen >= uni(a.tail_at)) {
                tail_saving = true; /* (saved after the loop) */
                break;
            }
        }
    }
#ifdef FMGI_CLOCK_STAMP /* sum over waves of the shader-clock and 100-MHz deltas of the loop: stats[24], [25] */
    {
        const unsigned long long ck_t1 = __builtin_amdgcn_s_memtime(), ck_r1 = __builtin_amdgcn_s_memrealtime();
        if ((threadIdx.x & 63) == 0) {
            atomicAdd(a.stats + KSTAT_STAGE0 + 8, ck_t1 - ck_t0);
            atomicAdd(a.stats + KSTAT_STAGE0 + 9, ck_r1 - ck_r0);
        }
    }
#endif
    if constexpr (kTail == 1) { /* (every lane of the wave is here) the saving lanes' tickets, one atomic per wave */
        const uint32_t k = wave_ticket(a.tail_n, tail_saving);
        if (tail_saving) /* (its scans so far go to the source's total with the resuming launch's atomic) */
            tail_save(a.tail_states + k, rng, left, srci, uni(a.src_cost) && photon >= 0 ? n_dep + n_esc : 0u);
    }
    if constexpr (HasAppend<Acc>::value) Acc::finish(a, ws, ring);
    if (TRACE && photon >= 0) {
        a.ev_counts[item - a.item_begin] = nev;
        a.rng_final[item - a.item_begin] = rng;
    }

    if (!lead) n_ph = n_dep = n_esc = sst.tests = sst.ties = sst.invalid = 0; /* counted once per group */
    const unsigned long long v[8] = {n_ph, (unsigned long long)n_dep + n_esc, n_dep, n_esc, sst.tests,
                                     (unsigned long long)sst.ties + sst.invalid, sst.ties, sst.invalid};
    const int slot[8] = {KSTAT_PHOTONS, KSTAT_SCANS, KSTAT_DEPOSITS, KSTAT_ESCAPES, KSTAT_TESTS, KSTAT_RESCANS,
                         KSTAT_TIES, KSTAT_INVALID};
#pragma unroll
    for (int i = 0; i < 8; i++) {
        unsigned long long s = wave_sum(v[i]);
        if ((threadIdx.x & 63) == 0 && s) atomicAdd(a.stats + slot[i], s);
    }
#ifdef FMGI_STAGE_TIMING
    if ((threadIdx.x & 63) == 0)
        for (int k = 0; k < ST_N; k++) atomicAdd(a.stats + KSTAT_STAGE0 + k, sst.clk.acc[k]);
#endif
}

/* AccState -> int64 fixed point: lm[t][c] += sum_s counts[s][t] * colour_fx[s][c]; counts zeroed.
   One thread per texel; each read of counts[s][*] is coalesced across the block. */
__global__ __launch_bounds__(256) void k_reduce_states(unsigned long long *__restrict__ counts,
                                                       const long long *__restrict__ colfx,
                                                       unsigned long long *__restrict__ lm, int n) {
    const int t = blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= n) return;
    long long r = 0, g = 0, b = 0;
    cptr<long long> C = (cptr<long long>)colfx;
    for (int s = 0; s < FMGI_COLOUR_STATES; s++) {
        unsigned long long *p = counts + (size_t)s * n + t;
        const unsigned long long k = *p;
        if (k) {
            r += (long long)k * C[3 * s + 0];
            g += (long long)k * C[3 * s + 1];
            b += (long long)k * C[3 * s + 2];
            *p = 0;
        }
    }
    unsigned long long *q = lm + 4 * (size_t)t;
    q[0] += (unsigned long long)r;
    q[1] += (unsigned long long)g;
    q[2] += (unsigned long long)b;
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

__global__ void k_add_u64(unsigned long long *__restrict__ dst, const unsigned long long *__restrict__ src,
                          int64_t n) {
    int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) dst[i] += src[i];
}

/* the samplers' sin/cos over n inputs: the restatement (fmgi_math.h) or, lib = 1, the device library's
   sinf/cosf it restates (parity tests) */
__global__ void k_sincos(const float *__restrict__ x, float *__restrict__ s, float *__restrict__ c, int64_t n, int lib) {
    int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    float a, b;
    if (lib) {
        a = sinf(x[i]);
        b = cosf(x[i]);
    } else {
        fmgi_sincosf(x[i], &a, &b);
    }
    s[i] = a;
    c[i] = b;
}

/* ---- per-scene constants: photonmap.cl's OpenCL builtins as ROCm builds them for gfx950 ---------- */

/* length() (opencl.bc _Z6lengthDv3_f): llvm.sqrt with !fpmath 3.0, i.e. v_sqrt_f32 (within 1 ulp, not
   correctly rounded), of dot(v, v), rescaled below 2^-126 and at inf */
__device__ float cl_length(f3 a) {
    const float d = dot3(a, a);
    if (d < 0x1p-126f) {
        const f3 t = mul3(a, 0x1p+86f);
        return __builtin_amdgcn_sqrtf(dot3(t, t)) * 0x1p-86f;
    }
    if (d == INFINITY) {
        const f3 t = mul3(a, 0x1p-66f);
        return __builtin_amdgcn_sqrtf(dot3(t, t)) * 0x1p+66f;
    }
    return __builtin_amdgcn_sqrtf(d);
}

/* __ocml_rsqrt_f32 with f32 denormals preserved: v_rsq_f32, inputs below 2^-126 scaled by 2^24 */
__device__ float cl_rsqrt(float x) {
    const bool tiny = x < 0x1p-126f;
    const float r = __builtin_amdgcn_rsqf(tiny ? x * 0x1p+24f : x);
    return tiny ? r * 4096.0f : r;
}

/* normalize() (opencl.bc _Z9normalizeDv3_f): v * rsqrt(dot(v, v)) with the library's rescaling */
__device__ f3 cl_normalize(f3 a) {
    if (a.x == 0.0f && a.y == 0.0f && a.z == 0.0f) return a;
    float d = dot3(a, a);
    f3 t = a;
    if (d < 0x1p-126f) {
        t = mul3(a, 0x1p+86f);
        d = dot3(t, t);
    } else if (d == INFINITY) {
        t = mul3(a, 0x1p-66f);
        d = dot3(t, t);
        if (d == INFINITY) {
            t = mkf3(copysignf(isinf(t.x) ? 1.0f : 0.0f, t.x), copysignf(isinf(t.y) ? 1.0f : 0.0f, t.y),
                     copysignf(isinf(t.z) ? 1.0f : 0.0f, t.z));
            d = dot3(t, t);
        }
    }
    return mul3(t, cl_rsqrt(d));
}

/* photonmap.cl:43-48 (== :65-70): the sampler basis of a normal */
__device__ void cl_sampler_basis(f3 n, f3 &bu, f3 &bv) {
    f3 udir = mkf3(0, 0, 1);
    if (fabsf(dot3(udir, n)) >= 0.999999f) udir = mkf3(0, 1, 0);
    const f3 vdir = cl_normalize(cross3(udir, n));
    bu = cl_normalize(cross3(vdir, n));
    bv = vdir;
}

__device__ __forceinline__ f3 f3of(const fmgi_vec3 &v) { return mkf3(v.s[0], v.s[1], v.s[2]); }

/* The per-rect values photonmap.cl recomputes in every intersects() / getTileIdAt() call, and every
   emitter's and wall's sampler basis, evaluated once per scene with the kernel's own builtins: wl =
   length(width) (photonmap.cl:144), wn = width / wl (:145), hl, hn (:149-150), bu, bv (:43-48, :65-70).
   One thread per wall, then one per emitter; the other RectDev / SrcDev fields come from the host. */
__global__ void k_scene_setup(const fmgi_rect *__restrict__ walls, int nw, const fmgi_rect *__restrict__ srcs, int ns,
                              RectDev *__restrict__ rd, SrcDev *__restrict__ sd) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    f3 bu, bv;
    if (i < nw) {
        const fmgi_rect &r = walls[i];
        const f3 w = f3of(r.width), h = f3of(r.height);
        const float wl = cl_length(w), hl = cl_length(h);
        const f3 wn = div3(w, wl), hn = div3(h, hl);
        RectDev &d = rd[i];
        d.wnx = wn.x; d.wny = wn.y; d.wnz = wn.z; d.wl = wl;
        d.hnx = hn.x; d.hny = hn.y; d.hnz = hn.z; d.hl = hl;
        d.iwl = 1.0f / wl; /* tile_uv's quotient estimate (checked against a band, fmgi_core.h) */
        d.ihl = 1.0f / hl;
        cl_sampler_basis(f3of(r.n), bu, bv);
        d.bux = bu.x; d.buy = bu.y; d.buz = bu.z;
        d.bvx = bv.x; d.bvy = bv.y; d.bvz = bv.z;
    } else if (i - nw < ns) {
        cl_sampler_basis(f3of(srcs[i - nw].n), bu, bv);
        SrcDev &d = sd[i - nw];
        d.bux = bu.x; d.buy = bu.y; d.buz = bu.z;
        d.bvx = bv.x; d.bvy = bv.y; d.bvz = bv.z;
    }
}

/* the bake's arithmetic helpers, one element per thread (fmgi_device_unit) */
__global__ void k_unit(int op, const float *__restrict__ a, const float *__restrict__ b, int32_t *__restrict__ out,
                       int64_t n) {
    int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    out[i] = op == 0 ? __float_as_int(sqrt_cr(a[i]))
                     : (op == 1 ? trunc_div(a[i], b[i]) : trunc_div_inv(a[i], b[i], 1.0f / b[i]));
}

template <class Scan, class Acc>
void launch3(const BakeArgs &a, bool trace, dim3 grid, dim3 block, size_t lds, hipStream_t s) {
    if (trace)
        hipLaunchKernelGGL((k_bake<Scan, Acc, true>), grid, block, lds, s, a);
    else
        hipLaunchKernelGGL((k_bake<Scan, Acc, false>), grid, block, lds, s, a);
}

template <class Scan, class Acc>
const void *kernel_ptr(bool trace) {
    return trace ? (const void *)&k_bake<Scan, Acc, true> : (const void *)&k_bake<Scan, Acc, false>;
}

/* accumulation codes: FMGI_ACCUM_FX3 1, STATE 2, NONE 3, STREAM 4 (unsorted / presorted layouts) and the
   internal kAccBucket 5 (STREAM in the per-tile bucket layout) */
/* (the experiment build's accumulations: the presorted-segment stream, per-workgroup tile lines, the dense
   stream; the product library has no instance of them and rejects their ids) */
template <class Scan>
const void *kernel_acc(int accum, bool trace) {
    if (accum == 2) return kernel_ptr<Scan, AccState>(trace);
    if (accum == 3) return kernel_ptr<Scan, AccNone>(trace);
    if (accum == kAccSliced) return kernel_ptr<Scan, AccSliced>(trace);
    if (accum == kAccBucket) return kernel_ptr<Scan, AccBucket>(trace);
    if (accum == kAccScatter) return kernel_ptr<Scan, AccScatter>(trace);
#if FMGI_EXPERIMENTS
    if (accum == 4) return kernel_ptr<Scan, AccStream>(trace);
    if (accum == kAccLines) return kernel_ptr<Scan, AccLines>(trace);
    if (accum == kAccDense) return kernel_ptr<Scan, AccDense>(trace);
#else
    if (accum == 4 || accum == kAccLines || accum == kAccDense) return nullptr;
#endif
    return kernel_ptr<Scan, AccFx3>(trace);
}

template <class Scan>
bool launch_acc(const BakeArgs &a, int accum, bool trace, dim3 grid, dim3 block, size_t lds, hipStream_t s) {
    if (accum == 2) launch3<Scan, AccState>(a, trace, grid, block, lds, s);
    else if (accum == 3) launch3<Scan, AccNone>(a, trace, grid, block, lds, s);
    else if (accum == kAccSliced) launch3<Scan, AccSliced>(a, trace, grid, block, lds, s);
    else if (accum == kAccBucket) launch3<Scan, AccBucket>(a, trace, grid, block, lds, s);
    else if (accum == kAccScatter) launch3<Scan, AccScatter>(a, trace, grid, block, lds, s);
#if FMGI_EXPERIMENTS
    else if (accum == 4) launch3<Scan, AccStream>(a, trace, grid, block, lds, s);
    else if (accum == kAccLines) launch3<Scan, AccLines>(a, trace, grid, block, lds, s);
    else if (accum == kAccDense) launch3<Scan, AccDense>(a, trace, grid, block, lds, s);
#else
    else if (accum == 4 || accum == kAccLines || accum == kAccDense) return false;
#endif
    else launch3<Scan, AccFx3>(a, trace, grid, block, lds, s);
    return true;
}

const void *bake_kernel(int kernel, int accum, bool trace) {
    if (kernel == FMGI_KERNEL_FAST_COOP)
        return accum == kAccBucket ? kernel_ptr<ScanFastCoop, AccBucket>(false)
               : accum == kAccScatter ? kernel_ptr<ScanFastCoop, AccScatter>(false)
               : accum == kAccSliced ? kernel_ptr<ScanFastCoop, AccSliced>(false)
#if FMGI_EXPERIMENTS
               : accum == kAccLines ? kernel_ptr<ScanFastCoop, AccLines>(false)
               : accum == kAccDense ? kernel_ptr<ScanFastCoop, AccDense>(false)
               : accum == 4 ? kernel_ptr<ScanFastCoop, AccStream>(false)
#endif
                                    : nullptr;
#if FMGI_EXPERIMENTS
    if (kernel == FMGI_KERNEL_HYBRID_TAIL) /* the launch-tail pair: lane-by-lane stores and the rings */
        return accum == kAccScatter ? kernel_ptr<ScanHybridTail, AccScatter>(false)
               : accum == kAccBucket ? kernel_ptr<ScanHybridTail, AccBucket>(false) : nullptr;
    if (kernel == FMGI_KERNEL_HYBRID_RESUME)
        return accum == kAccScatter ? kernel_ptr<ScanHybridResume, AccScatter>(false)
               : accum == kAccBucket ? kernel_ptr<ScanHybridResume, AccBucket>(false) : nullptr;
#else
    if (kernel == FMGI_KERNEL_HYBRID_TAIL || kernel == FMGI_KERNEL_HYBRID_RESUME) return nullptr;
#endif
    if (kernel == (2 | FMGI_KVAR_AXES | FMGI_KVAR_COMPACT)) /* the lane-by-lane stores only (bake_common) */
        return accum == kAccScatter ? kernel_ptr<ScanGridAxesCompact, AccScatter>(trace) : nullptr;
    if (kernel == (2 | FMGI_KVAR_AXES | FMGI_KVAR_STAGED)) return kernel_acc<ScanGridAxesStaged>(accum, trace);
    if (kernel == (2 | FMGI_KVAR_AXES)) return kernel_acc<ScanGridAxes>(accum, trace);
#if FMGI_EXPERIMENTS
    if (kernel == (4 | FMGI_KVAR_PLAN)) return kernel_acc<ScanHybridPlan>(accum, trace);
#endif
    kernel &= ~(FMGI_KVAR_AXES | FMGI_KVAR_PLAN | FMGI_KVAR_STAGED);
    if (kernel == 2) return kernel_acc<ScanGrid>(accum, trace);
    if (kernel == 4) return kernel_acc<ScanHybrid>(accum, trace);
    if (kernel == 1) return kernel_acc<ScanFast>(accum, trace);
    return kernel_acc<ScanExact>(accum, trace);
}

} // namespace

/* dynamic LDS of a bake launch: the scan image (fast / grid scans), then one ring per wave (AccStream) */
/* 1 when this build's hybrid scan reads the wall-pair image (the default), 0 for FMGI_FILTER_PK=0 builds */
int fmgi_kernels_filter_pk() { return FMGI_FILTER_PK; }

size_t fmgi_bake_lds(int kernel, int accum, int block, int img_bytes, int *ring_off) {
    /* (the launch-tail saving instance: the workgroup's copy of the idle-lane count after the image) */
    const size_t img = kernel != 0 ? (((size_t)img_bytes + 15) & ~(size_t)15) + (kernel == FMGI_KERNEL_HYBRID_TAIL ? 16 : 0) : 0;
    if (ring_off) *ring_off = (int)img;
#if FMGI_EXPERIMENTS
    if (accum == kAccLines) return img + (size_t)FMGI_LINES_DWORDS * 4;
#endif
    if (accum == kAccScatter) return img + (size_t)(block / 64) * FMGI_SCATTER_STRIDE * 4;
    if (accum == kAccBucket) return img + (size_t)(block / 64) * FMGI_RING_STRIDE_BUCKET * 4;
    return img + ((accum == 4 || accum == kAccSliced) ? (size_t)(block / 64) * FMGI_RING_STRIDE * 4 : 0);
}

/* the name a profiler prints for the k_bake instance a launch of (kernel, accum, trace) runs ("void (anonymous
   namespace)::k_bake<...>(BakeArgs)", as in rocprofv3's kernel trace and the committed counter summaries):
   the runtime's symbol name of the instance, demangled; "" if there is none */
std::string fmgi_bake_kernel_name(int kernel, int accum, bool trace) {
    const void *fn = bake_kernel(kernel, accum, trace);
    const char *m = fn ? hipKernelNameRefByPtr(fn, nullptr) : nullptr;
    if (!m) return std::string();
    int st = 0;
    char *d = abi::__cxa_demangle(m, nullptr, nullptr, &st);
    std::string n = st == 0 && d ? std::string(d) : std::string(m);
    free(d);
    return n;
}

/* a bake launch of more than 64 KiB of dynamic LDS (scan image + staged tables + rings, fmgi_api.cpp
   plan_stage) needs the kernel's limit raised, once per (device, kernel instance) */
static hipError_t bake_lds_attr(const void *fn, size_t lds) {
    if (lds <= 65536) return hipSuccess;
    static std::mutex mu;
    static std::set<std::pair<int, const void *>> done;
    int dev = 0;
    hipError_t e = hipGetDevice(&dev);
    if (e != hipSuccess) return e;
    std::lock_guard<std::mutex> lk(mu);
    if (done.count({dev, fn})) return hipSuccess;
    e = hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    if (e == hipSuccess) done.insert({dev, fn});
    return e;
}

int fmgi_bake_resident_blocks(int kernel, int accum, bool trace, int block, int lds_bytes) {
    int n = 0;
    const void *fn = bake_kernel(kernel, accum, trace);
    const size_t lds = fmgi_bake_lds(kernel, accum, block, lds_bytes, nullptr);
    if (bake_lds_attr(fn, lds) != hipSuccess ||
        hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, fn, block, lds) != hipSuccess)
        return 0;
    return n;
}

hipError_t fmgi_launch_bake(const BakeArgs &a, int kernel, int accum, bool trace, int grid_blocks, int block,
                            hipStream_t s) {
    dim3 grid(grid_blocks), blk(block);
    int ring_off = 0;
    const size_t lds = fmgi_bake_lds(kernel, accum, block, a.fimg_bytes, &ring_off);
    if (ring_off != a.ring_off) return hipErrorInvalidValue; /* the caller sets a.ring_off from fmgi_bake_lds */
    {
        const hipError_t e = bake_lds_attr(bake_kernel(kernel, accum, trace), lds);
        if (e != hipSuccess) return e;
    }
    bool ok = true;
    if (kernel == FMGI_KERNEL_FAST_COOP) {
        if (trace || !bake_kernel(kernel, accum, false)) return hipErrorInvalidValue;
        if (accum == kAccBucket) launch3<ScanFastCoop, AccBucket>(a, false, grid, blk, lds, s);
        else if (accum == kAccScatter) launch3<ScanFastCoop, AccScatter>(a, false, grid, blk, lds, s);
        else if (accum == kAccSliced) launch3<ScanFastCoop, AccSliced>(a, false, grid, blk, lds, s);
#if FMGI_EXPERIMENTS
        else if (accum == kAccDense) launch3<ScanFastCoop, AccDense>(a, false, grid, blk, lds, s);
        else if (accum == kAccLines) launch3<ScanFastCoop, AccLines>(a, false, grid, blk, lds, s);
        else launch3<ScanFastCoop, AccStream>(a, false, grid, blk, lds, s);
    } else if (kernel == (4 | FMGI_KVAR_PLAN)) { /* FMGI_KERNEL_HYBRID, walls over the floor plan */
        ok = launch_acc<ScanHybridPlan>(a, accum, trace, grid, blk, lds, s);
#endif
#if FMGI_EXPERIMENTS
    } else if (kernel == FMGI_KERNEL_HYBRID_TAIL || kernel == FMGI_KERNEL_HYBRID_RESUME) { /* the launch tail */
        if (trace || !bake_kernel(kernel, accum, false)) return hipErrorInvalidValue;
        if (kernel == FMGI_KERNEL_HYBRID_TAIL && accum == kAccScatter) launch3<ScanHybridTail, AccScatter>(a, false, grid, blk, lds, s);
        else if (kernel == FMGI_KERNEL_HYBRID_TAIL) launch3<ScanHybridTail, AccBucket>(a, false, grid, blk, lds, s);
        else if (accum == kAccScatter) launch3<ScanHybridResume, AccScatter>(a, false, grid, blk, lds, s);
        else launch3<ScanHybridResume, AccBucket>(a, false, grid, blk, lds, s);
#endif
    } else if (kernel == 4) { /* FMGI_KERNEL_HYBRID */
        ok = launch_acc<ScanHybrid>(a, accum, trace, grid, blk, lds, s);
    } else if (kernel == (2 | FMGI_KVAR_AXES | FMGI_KVAR_COMPACT)) { /* closed box, the compact tables in LDS */
        if (accum != kAccScatter) return hipErrorInvalidValue;
        launch3<ScanGridAxesCompact, AccScatter>(a, trace, grid, blk, lds, s);
    } else if (kernel == (2 | FMGI_KVAR_AXES | FMGI_KVAR_STAGED)) { /* closed box, every table in LDS */
        ok = launch_acc<ScanGridAxesStaged>(a, accum, trace, grid, blk, lds, s);
    } else if (kernel == (2 | FMGI_KVAR_AXES)) { /* FMGI_KERNEL_GRID, closed box */
        ok = launch_acc<ScanGridAxes>(a, accum, trace, grid, blk, lds, s);
    } else if ((kernel & ~FMGI_KVAR_AXES) == 2) { /* FMGI_KERNEL_GRID */
        ok = launch_acc<ScanGrid>(a, accum, trace, grid, blk, lds, s);
    } else if (kernel == 1) { /* FMGI_KERNEL_FAST */
        ok = launch_acc<ScanFast>(a, accum, trace, grid, blk, lds, s);
    } else if ((kernel & 0xF) == 0) {
        ok = launch_acc<ScanExact>(a, accum, trace, grid, blk, lds, s);
    } else {
        ok = false;
    }
    if (!ok) return hipErrorInvalidValue; /* no instance (an experiment build's kernel or accumulation) */
    return hipGetLastError();
}

hipError_t fmgi_launch_reduce_states(unsigned long long *counts, const long long *colfx, unsigned long long *lm, int n,
                                     hipStream_t s) {
    if (n <= 0) return hipSuccess;
    hipLaunchKernelGGL(k_reduce_states, dim3((n + 255) / 256), dim3(256), 0, s, counts, colfx, lm, n);
    return hipGetLastError();
}

hipError_t fmgi_launch_finalize(const unsigned long long *lm, const float *tin, float *tout, int64_t n,
                                hipStream_t s) {
    if (n <= 0) return hipSuccess;
    int64_t blocks = (n + 255) / 256;
    hipLaunchKernelGGL(k_finalize, dim3((unsigned)blocks), dim3(256), 0, s, lm, (const float4 *)tin, (float4 *)tout, n);
    return hipGetLastError();
}

hipError_t fmgi_launch_add_u64(unsigned long long *dst, const unsigned long long *src, int64_t n, hipStream_t s) {
    if (n <= 0) return hipSuccess;
    hipLaunchKernelGGL(k_add_u64, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, dst, src, n);
    return hipGetLastError();
}

hipError_t fmgi_launch_unit(int op, const float *a, const float *b, int32_t *out, int64_t n, hipStream_t s) {
    if (n <= 0) return hipSuccess;
    hipLaunchKernelGGL(k_unit, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, op, a, b, out, n);
    return hipGetLastError();
}

hipError_t fmgi_launch_sincos(const float *x, float *sn, float *cs, int64_t n, int lib, hipStream_t s) {
    if (n <= 0) return hipSuccess;
    int64_t blocks = (n + 255) / 256;
    hipLaunchKernelGGL(k_sincos, dim3((unsigned)blocks), dim3(256), 0, s, x, sn, cs, n, lib);
    return hipGetLastError();
}

hipError_t fmgi_launch_scene_setup(const fmgi_rect *walls, int nw, const fmgi_rect *srcs, int ns, RectDev *rd,
                                   SrcDev *sd, hipStream_t s) {
    const int n = nw + ns;
    if (n <= 0) return hipSuccess;
    hipLaunchKernelGGL(k_scene_setup, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, walls, nw, srcs, ns, rd, sd);
    return hipGetLastError();
}
