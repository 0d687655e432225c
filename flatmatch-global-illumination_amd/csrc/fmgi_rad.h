/*
 * fmgi_rad.h -- shared host/device structures of the radiosity backend (§8f rank 4): the reference's
 * performRadiosityNative (radiosityNative.c:92-268) on the GPU.
 *
 * The reference (1) gives every level-0 wall texel 10000 cosine-distributed rays drawn from libc
 * rand(), each traced against that texel's sorted candidate list, and records the level-0 texel each
 * ray lands on (the "form factors", :166-227); (2) runs 7 gather/update/mipmap bounces over those
 * texel ids (:230-251). Here:
 *   k_rad_rand   replays the caller's glibc TYPE_3 rand() stream on the device: every job (texel)
 *                owns 20000 consecutive values, split into RAD_SUBS sub-streams whose 31-word starting
 *                windows come from host-built jump matrices (x_n = x_{n-31} + x_{n-3} mod 2^32 is
 *                linear, so a window N steps ahead is M^N times the current one);
 *   k_rad_rays   one workgroup per job: the candidate list (backface / isBehindRay culling, the
 *                getShortestDistanceRectToPoint keys, glibc 2.35's stable merge-sort order reproduced
 *                by a bitonic sort on (distance, index)) in LDS, then one lane per ray;
 *   k_rad_gather one lane per job: the sequential fp32 sum over its 10000 source texels;
 *   k_rad_update src = src*0.7f + dest*(0.3f/10000) on every texel;
 *   k_rad_mip    one workgroup per rectangle: rectangle.c:508-575 mipmap, level by level.
 */
#ifndef FMGI_RAD_H
#define FMGI_RAD_H

#include <stdint.h>

#include <hip/hip_runtime_api.h>

#include "fmgi_ao.h"

#define FMGI_RAD_RAYS 10000   /* geoSphereNumVectors, radiosityNative.c:151 */
#define FMGI_RAD_DRAWS 20000  /* rand() values per job: two per ray (vector3_cl.c:131-132) */
#define FMGI_RAD_SUBS 8       /* rand sub-streams per job */
#define FMGI_RAD_SUBLEN 2500  /* FMGI_RAD_DRAWS / FMGI_RAD_SUBS */
#define FMGI_RAD_ITERS 7      /* bounce iterations, radiosityNative.c:230 */
#define FMGI_RAD_MAX_SORT 16384 /* candidate sort capacity (LDS keys of 8 B) */
#define FMGI_RAD_JUMP_BITS 40 /* jump matrices M^(2500 * 2^b), b < 40 */

/* glibc random_r TYPE_3 window: 31 words, oldest first */
#define FMGI_RAND_DEG 31

/* a rectangle as the candidate tests see it (rectangle.c:97-113, :442-470): pos, width, height, n */
struct RadRect {
    float px, py, pz, wx, wy, wz, hx, hy, hz, nx, ny, nz;
    int32_t s0, s1, s2, pad;
};
static_assert(sizeof(RadRect) == 64, "RadRect must be 64 B");

/* one level-0 wall texel (a job): the ray origin frame and basis of its wall */
struct RadJob {
    float cx, cy, cz;    /* getTileCenter (rectangle.c:140-153) */
    float nx, ny, nz;    /* wall normal */
    float ux, uy, uz;    /* getCosineDistributedRandomRay's udir (vector3_cl.c:140-145) */
    float vx, vy, vz;    /* ... and vdir */
    int32_t texel;       /* wall s0 + tile */
    int32_t pad[3];
};
static_assert(sizeof(RadJob) == 64, "RadJob must be 64 B");

struct RadArgs {
    const RadRect *rects; /* walls, windows, lights (window/light s0 appended after numTexels) */
    const AoRect *hits;   /* the same rectangles as intersects() sees them */
    int nrects;
    int sort_n;           /* power of two >= nrects */
    const RadJob *jobs;
    int64_t njobs;        /* all jobs */
    int64_t job0, nchunk; /* this launch: jobs [job0, job0 + nchunk) */
    const uint32_t *jump; /* FMGI_RAD_JUMP_BITS matrices of 31x31 words, row-major */
    const uint32_t *v0;   /* the caller's rand window (31 words, oldest first) */
    uint32_t *draws;      /* nchunk x FMGI_RAD_DRAWS rand() values of this chunk */
    int32_t *sids;        /* FMGI_RAD_RAYS x njobs (ray-major): the source texel of every ray, -1 none */
};

struct RadBounce {
    const int32_t *sids;
    const RadJob *jobs;
    int64_t njobs;
    const RadRect *rects;
    int nrects;
    int64_t ntex;        /* texels incl. the window/light texels */
    const float4 *src;
    float4 *dst;         /* next src */
    float4 *dest;        /* the gather sums (zero except job texels) */
    float keep, gain;    /* 1 - reflectance, reflectance / 10000 */
};

hipError_t fmgi_rad_launch_rand(const RadArgs &a, hipStream_t s);
hipError_t fmgi_rad_launch_rays(const RadArgs &a, hipStream_t s);
hipError_t fmgi_rad_launch_bounce(const RadBounce &b, hipStream_t s);

#endif
