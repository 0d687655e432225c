/* fmgi_output.h -- the output step's device arguments (fmgi_output.hip, fmgi_ao_host.cpp). */
#ifndef FMGI_OUTPUT_H
#define FMGI_OUTPUT_H

#include <stdint.h>

#include <hip/hip_runtime_api.h>

struct OutWall {
    int64_t first_tile; /* prefix sum of level-0 tiles = this wall's offset in the RGB tile stream */
    int32_t s0;         /* texel base */
    int32_t floor;      /* rectangle.c:313: pos.z == width.z == height.z == 0 */
    float norm;         /* (float)(0.35 * tiles / (area * spa)), main.c:71-76 */
    int32_t pad;
};
static_assert(sizeof(OutWall) == 24, "OutWall must be 24 B");

struct OutArgs {
    const OutWall *walls;
    int nwalls;
    int64_t ntexels; /* level-0 texels of all walls */
    float *texels;   /* float4 per texel, normalised in place when `normalise` */
    uint8_t *rgb;    /* 3 B per level-0 texel */
    int normalise, tint_extra;
};

hipError_t fmgi_launch_output(const OutArgs &a, hipStream_t s);

#endif
