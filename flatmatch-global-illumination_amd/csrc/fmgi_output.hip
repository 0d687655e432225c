/*
 * fmgi_output.hip -- the output step after a bake, on the GPU, byte-identical to
 * the reference's host code:
 *   normalisation   main.c:66-79 (photon modes): level-0 texels *= (float)(0.35 * tilesPerSample)
 *   tone map        rectangle.c:263-286 convert/convert2: luminance in double, 1 - exp(-2 L) in double
 *   RGB8 + tint     rectangle.c:288-331 saveAs_core: clamp + truncation, floor walls G*0.95, B*0.9
 *                   (doubles), and again in float with tintExtra
 * One thread per level-0 texel; the wall is found by a binary search over the tile prefix sums, and
 * the bytes land at the wall's offset in the concatenation of the reference's per-wall tile buffers.
 */
#include <hip/hip_runtime.h>

#include "fmgi_output.h"

#pragma clang fp contract(off)

namespace {

__device__ __forceinline__ uint8_t to_byte(float d) { /* clamp() rectangle.c:288-293, then (uint8_t) */
    if (d != d) return 0; /* what x86's cvttss2si low byte gives for NaN (0/0 on a black texel) */
    if (d < 0) d = 0;
    if (d > 255) d = 255;
    return (uint8_t)(int)d;
}

__global__ __launch_bounds__(256) void k_output(OutArgs a) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= a.ntexels) return;
    int lo = 0, hi = a.nwalls - 1; /* last wall with first_tile <= i */
    while (lo < hi) {
        const int mid = (lo + hi + 1) >> 1;
        if (a.walls[mid].first_tile <= i) lo = mid; else hi = mid - 1;
    }
    const OutWall w = a.walls[lo];
    const int64_t j = i - w.first_tile;
    float4 *t = (float4 *)a.texels + w.s0 + j;
    float4 c = *t;
    if (a.normalise) {
        c = make_float4(c.x * w.norm, c.y * w.norm, c.z * w.norm, 0.0f);
        *t = c;
    }
    const float lum = (float)(0.2126 * (double)c.x + 0.7152 * (double)c.y + 0.0722 * (double)c.z);
    const float per = (float)(1 - exp((double)(-2 * lum)));
    const float r = c.x * (per / lum), g = c.y * (per / lum), b = c.z * (per / lum);
    uint8_t px0 = to_byte(r * 255), px1 = to_byte(g * 255), px2 = to_byte(b * 255);
    if (w.floor) {
        px1 = (uint8_t)(int)(px1 * 0.95);
        px2 = (uint8_t)(int)(px2 * 0.9);
        if (a.tint_extra) {
            px0 = (uint8_t)(int)(px0 * 1.0f);
            px1 = (uint8_t)(int)(px1 * 0.95f);
            px2 = (uint8_t)(int)(px2 * 0.9f);
        }
    }
    uint8_t *o = a.rgb + 3 * i;
    o[0] = px0;
    o[1] = px1;
    o[2] = px2;
}

} // namespace

hipError_t fmgi_launch_output(const OutArgs &a, hipStream_t s) {
    if (a.ntexels <= 0) return hipSuccess;
    hipLaunchKernelGGL(k_output, dim3((unsigned)((a.ntexels + 255) / 256)), dim3(256), 0, s, a);
    return hipGetLastError();
}
