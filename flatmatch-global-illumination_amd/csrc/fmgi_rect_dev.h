/*
 * fmgi_rect_dev.h -- device-side fp32 vector helpers and the ray/rectangle test of the native C
 * backends (vector3_cl.c, rectangle.c:67-95 intersects), shared by the ambient-occlusion (fmgi_ao.hip)
 * and radiosity (fmgi_rad.hip) kernels. Every operation is IEEE fp32 in the reference's source order;
 * the including file turns contraction off (#pragma clang fp contract(off)) before including this.
 */
#ifndef FMGI_RECT_DEV_H
#define FMGI_RECT_DEV_H

#include <hip/hip_runtime.h>

#include "fmgi_ao.h"

namespace fmgi_dev {

struct v3 {
    float x, y, z;
};
__device__ __forceinline__ v3 mk(float x, float y, float z) { return v3{x, y, z}; }
__device__ __forceinline__ v3 add(v3 a, v3 b) { return mk(a.x + b.x, a.y + b.y, a.z + b.z); }
__device__ __forceinline__ v3 sub(v3 a, v3 b) { return mk(a.x - b.x, a.y - b.y, a.z - b.z); }
__device__ __forceinline__ v3 mul(v3 a, float f) { return mk(a.x * f, a.y * f, a.z * f); }
__device__ __forceinline__ float dot(v3 a, v3 b) { return a.x * b.x + a.y * b.y + a.z * b.z; }

/* rectangle.c:67-95 intersects() on an AoRect (normalised edges and lengths precomputed with the same
   IEEE ops as the per-call div_vec3/length): the hit distance, or -1 for no hit */
__device__ __forceinline__ float rect_intersects(const AoRect &r, v3 src, v3 dir, float closest) {
    const v3 n = mk(r.nx, r.ny, r.nz), pos = mk(r.px, r.py, r.pz);
    const float denom = dot(n, dir);
    if (denom >= 0) return -1;
    const float fac = dot(n, sub(pos, src)) / denom;
    if (fac < 0) return -1;
    const v3 ray = mul(dir, fac);
    if (closest * closest < dot(ray, ray)) return -1; /* squaredLength */
    const v3 pdir = sub(add(src, ray), pos);
    const float dx = dot(mk(r.wx, r.wy, r.wz), pdir);
    const float dy = dot(mk(r.hx, r.hy, r.hz), pdir);
    if (dx < 0 || dy < 0 || dx > r.wl || dy > r.hl) return -1;
    return fac;
}

} // namespace fmgi_dev

#endif
