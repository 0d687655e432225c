/*
 * fmgi_rad.hip -- the radiosity backend on the GPU, bit-identical to the reference's
 * performRadiosityNative (radiosityNative.c:92-268); see fmgi_rad.h for the kernel plan.
 *
 * Arithmetic: the native C path (radiosityNative.c, rectangle.c, vector3_cl.c; gcc -O2 -msse3, no FMA)
 * is IEEE fp32 in source order, with double sqrt/div/cos/sin in getCosineDistributedRandomRay. Contraction
 * is off here and every operation is written in the reference's order. Double division and sqrt are
 * correctly rounded on gfx950 as on x86; cos/sin come from the device math library (see DESIGN.md §9
 * for how rarely that can differ from glibc in a float result).
 */
#include <hip/hip_runtime.h>

#include "fmgi_lds_attr.h"
#include "fmgi_rad.h"

#pragma clang fp contract(off)

#include "fmgi_rect_dev.h"

namespace {

using namespace fmgi_dev;

constexpr int DEG = FMGI_RAND_DEG;

/* y = A x over Z/2^32 (A row-major 31x31, uniform across the wave: scalar loads) */
__device__ __forceinline__ void jump_apply(const uint32_t *__restrict__ A, const uint32_t (&x)[DEG], uint32_t (&y)[DEG]) {
#pragma unroll
    for (int i = 0; i < DEG; i++) {
        uint32_t s = 0;
#pragma unroll
        for (int k = 0; k < DEG; k++) s += A[i * DEG + k] * x[k];
        y[i] = s;
    }
}

/*
 * One lane per (job, sub-stream): the sub-stream's 31-word window is M^(2500 q) v0, q = job*8 + sub,
 * assembled from the host's M^(2500 * 2^b) matrices; then 2500 steps of glibc random_r TYPE_3
 * (x[n] = x[n-31] + x[n-3], output x[n] >> 1; random_r.c) with the window in registers.
 */
__global__ __launch_bounds__(256) void k_rad_rand(RadArgs a, int qbits) {
    const int64_t g = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (g >= a.nchunk * FMGI_RAD_SUBS) return;
    const int64_t jl = g / FMGI_RAD_SUBS;
    const int sub = (int)(g % FMGI_RAD_SUBS);
    const uint64_t q = (uint64_t)(a.job0 + jl) * FMGI_RAD_SUBS + sub;
    uint32_t x[DEG], y[DEG];
#pragma unroll
    for (int i = 0; i < DEG; i++) x[i] = a.v0[i];
    for (int b = 0; b < qbits; b++) {
        const bool take = (q >> b) & 1;
        if (!__any(take)) continue;
        jump_apply(a.jump + (size_t)b * DEG * DEG, x, y);
#pragma unroll
        for (int i = 0; i < DEG; i++) x[i] = take ? y[i] : x[i];
    }
    uint32_t *out = a.draws + jl * FMGI_RAD_DRAWS + (int64_t)sub * FMGI_RAD_SUBLEN;
    /* x[j] holds x[n-31] for the slot written at step j (mod 31); x[(j+28)%31] is x[n-3] */
    for (int s0 = 0; s0 < FMGI_RAD_SUBLEN; s0 += DEG) {
#pragma unroll
        for (int j = 0; j < DEG; j++) {
            if (s0 + j < FMGI_RAD_SUBLEN) {
                x[j] += x[(j + 28) % DEG];
                out[s0 + j] = x[j] >> 1;
            }
        }
    }
}

/* rectangle.c:97-113 isBehindRay */
__device__ __forceinline__ bool behind_ray(v3 p, v3 w, v3 h, v3 src, v3 dir) {
    const v3 d1 = sub(p, src), d2 = sub(add(p, w), src), d3 = sub(add(p, h), src), d4 = sub(add(add(p, w), h), src);
    return dot(d1, dir) < 0 && dot(d2, dir) < 0 && dot(d3, dir) < 0 && dot(d4, dir) < 0;
}

__device__ __forceinline__ float len3(v3 a) { return sqrtf(a.x * a.x + a.y * a.y + a.z * a.z); }
__device__ __forceinline__ v3 unit(v3 a) { return mul(a, 1.0f / len3(a)); }

/* rectangle.c:442-470 getShortestDistanceRectToPoint */
__device__ __forceinline__ float min_dist(v3 pos, v3 w, v3 h, v3 n, v3 p) {
    const v3 vd = sub(p, pos);
    const v3 on_plane = sub(p, mul(n, dot(vd, n)));
    const v3 pd = sub(on_plane, pos);
    float u = dot(pd, unit(h)) / len3(h);
    float v = dot(pd, unit(w)) / len3(w);
    u = (u < 0) ? 0.0f : ((u > 1) ? 1.0f : u);
    v = (v < 0) ? 0.0f : ((v > 1) ? 1.0f : v);
    return len3(sub(p, add(add(pos, mul(w, v)), mul(h, u))));
}

/* x86-64 cvttss2si, the reference's (int) cast: out of range and NaN give INT_MIN */
__device__ __forceinline__ int cvt_x86(float f) {
    return (f >= -2147483648.0f && f < 2147483648.0f) ? (int)f : (int)0x80000000;
}

__device__ __forceinline__ int clampi(int v, int lo, int hi) { return v < lo ? lo : (v > hi ? hi : v); }

/*
 * One workgroup per job (level-0 wall texel). LDS: sort_n 64-bit keys (distance bits << 32 | rect index;
 * ~0 for culled rectangles). getSortedIntersectableRects (radiosityNative.c:25-61) filters in rect order
 * and glibc 2.35 qsort is a stable merge sort, so the list is ordered by (distance, index).
 */
__global__ __launch_bounds__(256) void k_rad_rays(RadArgs a) {
    extern __shared__ unsigned long long keys[];
    __shared__ int ncand;
    const int tid = threadIdx.x;
    const int64_t jl = blockIdx.x;
    const int64_t job = a.job0 + jl;
    const RadJob J = a.jobs[job];
    const v3 cam = mk(J.cx, J.cy, J.cz), n = mk(J.nx, J.ny, J.nz);
    if (tid == 0) ncand = 0;
    __syncthreads();
    int mine = 0;
    for (int i = tid; i < a.sort_n; i += blockDim.x) {
        unsigned long long key = ~0ull;
        if (i < a.nrects) {
            const RadRect r = a.rects[i];
            const v3 pos = mk(r.px, r.py, r.pz), w = mk(r.wx, r.wy, r.wz), h = mk(r.hx, r.hy, r.hz),
                     rn = mk(r.nx, r.ny, r.nz);
            if (!(dot(rn, sub(pos, cam)) > 0) && !behind_ray(pos, w, h, cam, n)) {
                key = ((unsigned long long)__float_as_uint(min_dist(pos, w, h, rn, cam)) << 32) | (uint32_t)i;
                mine++;
            }
        }
        keys[i] = key;
    }
    if (mine) atomicAdd(&ncand, mine);
    __syncthreads();
    /* bitonic sort, ascending */
    for (int k = 2; k <= a.sort_n; k <<= 1) {
        for (int j = k >> 1; j > 0; j >>= 1) {
            for (int i = tid; i < a.sort_n / 2; i += blockDim.x) {
                const int lo = ((i & ~(j - 1)) << 1) | (i & (j - 1)), hi = lo + j;
                const unsigned long long x = keys[lo], y = keys[hi];
                if ((x > y) == ((lo & k) == 0)) {
                    keys[lo] = y;
                    keys[hi] = x;
                }
            }
            __syncthreads();
        }
    }
    const int C = ncand;
    const uint2 *draws = (const uint2 *)(a.draws + jl * FMGI_RAD_DRAWS);
    const v3 ud = mk(J.ux, J.uy, J.uz), vd = mk(J.vx, J.vy, J.vz);
    for (int k = tid; k < FMGI_RAD_RAYS; k += blockDim.x) {
        /* getCosineDistributedRandomRay (vector3_cl.c:129-149) */
        const uint2 rr = draws[k];
        const float r = (float)sqrt((double)(int)rr.x / (double)2147483647);
        const float phi = (float)((double)(2 * 3.141592f) * ((double)(int)rr.y / (double)2147483647));
        const float u = (float)((double)r * cos((double)phi));
        const float v = (float)((double)r * sin((double)phi));
        const float nn = (float)sqrt((double)(1 - r * r));
        const v3 dir = add(add(mul(ud, u), mul(vd, v)), mul(n, nn));
        const v3 pos = add(cam, mul(dir, 1E-5f));
        /* findClosestIntersectionSorted (radiosityNative.c:67-90) */
        float dist = INFINITY;
        int target = -1;
        for (int i = 0; i < C; i++) {
            const unsigned long long key = keys[i];
            if (dist < __uint_as_float((uint32_t)(key >> 32))) break;
            const int idx = __builtin_amdgcn_readfirstlane((int)(uint32_t)key);
            const float dn = rect_intersects(a.hits[idx], pos, dir, dist);
            if (dn < 0) continue;
            if (dn <= dist) {
                target = idx;
                dist = dn;
            }
        }
        int sid = -1;
        if (target >= 0) {
            /* getTileIdAt (rectangle.c:205-230) + getMipmapTexelId level 0 (:232-258) */
            const AoRect t = a.hits[target];
            const RadRect tr = a.rects[target];
            const v3 pd = sub(add(pos, mul(dir, dist)), mk(t.px, t.py, t.pz));
            const float dx = dot(mk(t.wx, t.wy, t.wz), pd), dy = dot(mk(t.hx, t.hy, t.hz), pd);
            const int tx = clampi(cvt_x86(dx * (float)tr.s1 / t.wl), 0, tr.s1 - 1);
            const int ty = clampi(cvt_x86(dy * (float)tr.s2 / t.hl), 0, tr.s2 - 1);
            const int tile = ty * tr.s1 + tx;
            sid = tr.s0 + (tile / tr.s1) * tr.s1 + tile % tr.s1;
        }
        a.sids[(int64_t)k * a.njobs + job] = sid;
    }
}

/*
 * radiosityNative.c:232-240: one lane per job, the sequential fp32 sum over its rays' source texels
 * (a ray that hit nothing adds nothing). The order of the adds is the reference's; only the loads are
 * batched: GATHER_B source ids per block, the next block's ids in flight while the current block's
 * texels load, so a lane waits one memory round trip per block instead of two per ray.
 * Random 16-B gathers from an L2-resident texel table: bound by cache lines per cycle per CU.
 */
constexpr int GATHER_B = 25;
static_assert(FMGI_RAD_RAYS % GATHER_B == 0, "gather blocks must tile the rays");

__global__ __launch_bounds__(256) void k_rad_gather(RadBounce b) {
    const int64_t job = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (job >= b.njobs) return;
    const int32_t *s = b.sids + job;
    const int64_t stride = b.njobs;
    float x = 0, y = 0, z = 0;
    int32_t nxt[GATHER_B];
#pragma unroll
    for (int i = 0; i < GATHER_B; i++) nxt[i] = __builtin_nontemporal_load(s + (int64_t)i * stride);
    for (int k0 = 0; k0 < FMGI_RAD_RAYS; k0 += GATHER_B) {
        int32_t id[GATHER_B];
#pragma unroll
        for (int i = 0; i < GATHER_B; i++) id[i] = nxt[i];
        if (k0 + GATHER_B < FMGI_RAD_RAYS) {
#pragma unroll
            for (int i = 0; i < GATHER_B; i++)
                nxt[i] = __builtin_nontemporal_load(s + (int64_t)(k0 + GATHER_B + i) * stride);
        }
        float4 t[GATHER_B]; /* one 16-B load per ray: a random gather costs a cache line per lane */
#pragma unroll
        for (int i = 0; i < GATHER_B; i++) t[i] = b.src[id[i] < 0 ? 0 : id[i]];
#pragma unroll
        for (int i = 0; i < GATHER_B; i++) {
            const bool hit = id[i] >= 0;
            x = hit ? x + t[i].x : x;
            y = hit ? y + t[i].y : y;
            z = hit ? z + t[i].z : z;
        }
    }
    b.dest[b.jobs[job].texel] = make_float4(x, y, z, 0.0f);
}

/* radiosityNative.c:242-247 */
__global__ __launch_bounds__(256) void k_rad_update(RadBounce b) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= b.ntex) return;
    const float4 s = b.src[i], d = b.dest[i];
    b.dst[i] = make_float4(s.x * b.keep + d.x * b.gain, s.y * b.keep + d.y * b.gain, s.z * b.keep + d.z * b.gain, 0.0f);
}

/* rectangle.c:508-575 mipmap(): one workgroup per rectangle, one level per step */
__global__ __launch_bounds__(256) void k_rad_mip(RadBounce b) {
    const RadRect r = b.rects[blockIdx.x];
    float4 *t = b.dst;
    int64_t base = r.s0;
    int w = r.s1, h = r.s2;
    while (w > 1 || h > 1) {
        if (w == 1 || h == 1) { /* mipmapInternalHorizontal / Vertical (:508-533) */
            const int m = (h == 1) ? w : h, tm = m / 2;
            for (int i = threadIdx.x; i < tm; i += blockDim.x) {
                const float4 p = t[base + 2 * i], q = t[base + 2 * i + 1];
                t[base + m + i] = make_float4((p.x + q.x) * 0.5f, (p.y + q.y) * 0.5f, (p.z + q.z) * 0.5f, 0.0f);
            }
            base += m;
            if (h == 1) w = tm;
            else h = tm;
        } else { /* mipmapInternal 2-D step (:535-569), add4 order */
            const int tw = w / 2, th = h / 2;
            for (int idx = threadIdx.x; idx < tw * th; idx += blockDim.x) {
                const int i = idx % tw, j = idx / tw;
                const float4 p = t[base + (2 * j) * w + 2 * i], q = t[base + (2 * j + 1) * w + 2 * i];
                const float4 c = t[base + (2 * j) * w + 2 * i + 1], d = t[base + (2 * j + 1) * w + 2 * i + 1];
                t[base + (int64_t)w * h + j * tw + i] =
                    make_float4((p.x + q.x + c.x + d.x) * 0.25f, (p.y + q.y + c.y + d.y) * 0.25f,
                                (p.z + q.z + c.z + d.z) * 0.25f, 0.0f);
            }
            base += (int64_t)w * h;
            w = tw;
            h = th;
        }
        __syncthreads();
    }
}

} // namespace

hipError_t fmgi_rad_launch_rand(const RadArgs &a, hipStream_t s) {
    if (a.nchunk <= 0) return hipSuccess;
    const uint64_t qmax = (uint64_t)(a.job0 + a.nchunk) * FMGI_RAD_SUBS;
    int qbits = 0;
    while (qbits < 64 && (qmax >> qbits)) qbits++;
    if (qbits > FMGI_RAD_JUMP_BITS) return hipErrorInvalidValue;
    const int64_t lanes = a.nchunk * FMGI_RAD_SUBS;
    hipLaunchKernelGGL(k_rad_rand, dim3((unsigned)((lanes + 255) / 256)), dim3(256), 0, s, a, qbits);
    return hipGetLastError();
}

hipError_t fmgi_rad_launch_rays(const RadArgs &a, hipStream_t s) {
    if (a.nchunk <= 0) return hipSuccess;
    if (a.sort_n < 2 || a.sort_n > FMGI_RAD_MAX_SORT || (a.sort_n & (a.sort_n - 1)) || a.nrects > a.sort_n)
        return hipErrorInvalidValue;
    const size_t lds = (size_t)a.sort_n * 8;
    hipError_t e = fmgi_set_lds_attr_once<1>((const void *)k_rad_rays, FMGI_RAD_MAX_SORT * 8);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(k_rad_rays, dim3((unsigned)a.nchunk), dim3(256), lds, s, a);
    return hipGetLastError();
}

hipError_t fmgi_rad_launch_bounce(const RadBounce &b, hipStream_t s) {
    if (b.njobs > 0) hipLaunchKernelGGL(k_rad_gather, dim3((unsigned)((b.njobs + 255) / 256)), dim3(256), 0, s, b);
    if (b.ntex > 0) hipLaunchKernelGGL(k_rad_update, dim3((unsigned)((b.ntex + 255) / 256)), dim3(256), 0, s, b);
    if (b.nrects > 0) hipLaunchKernelGGL(k_rad_mip, dim3((unsigned)b.nrects), dim3(256), 0, s, b);
    return hipGetLastError();
}
