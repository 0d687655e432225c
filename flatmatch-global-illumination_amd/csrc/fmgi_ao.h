/*
 * fmgi_ao.h -- shared host/device structures of the ambient-occlusion backend (§8f rank 2):
 * the reference's performAmbientOcclusionNative (photonmap.c:478-490, per wall :435-475) on the GPU.
 *
 * The reference traces, for every level-0 texel of every wall, 481 rays (the geoSphere4 directions,
 * fmgi_geosphere.h) through its BSP tree (buildBspTree/subdivideNode photonmap.c:278-406, traversal
 * findClosestIntersection :54-161) and stores the cosine-weighted mean hit distance. The host rebuilds
 * the same tree (same split choice, same item order); the device replays the traversal, including its
 * shifted ray origins and its pruning, so every texel is bit-identical.
 */
#ifndef FMGI_AO_H
#define FMGI_AO_H

#include <stdint.h>

#include <hip/hip_runtime_api.h>

/* a wall as rectangle.c:67 intersects() sees it: n, pos, width*(1/|width|), |width|, height*(1/|height|),
   |height| (the per-call div_vec3/length values, computed once with the same IEEE ops) */
struct AoRect {
    float nx, ny, nz, px, py, pz;
    float wx, wy, wz, wl;
    float hx, hy, hz, hl;
    float pad0, pad1;
};
static_assert(sizeof(AoRect) == 64, "AoRect must be 64 B");

/* a BSP node: its split plane (a wall's pos and n), children (-1: none), and its items[] */
struct AoNode {
    float px, py, pz, nx, ny, nz;
    int32_t left, right;
    int32_t item0, nitems;
    int32_t pad0, pad1;
};
static_assert(sizeof(AoNode) == 48, "AoNode must be 48 B");

/* one wall's texel-centre frame (getTileCenter rectangle.c:140-153) and its direction basis
   (createBase vector3_cl.c:152-160) */
struct AoWall {
    float px, py, pz;
    float vwx, vwy, vwz; /* width  * (1/s1) */
    float vhx, vhy, vhz; /* height * (1/s2) */
    float b1x, b1y, b1z, b2x, b2y, b2z;
    float nx, ny, nz;
    int32_t s0, s1, s2, pad;
};
static_assert(sizeof(AoWall) == 88, "AoWall must be 88 B");

#define FMGI_AO_MAX_DEPTH 48 /* BSP depth bound of the device traversal stack (checked on the host) */
#define FMGI_AO_DIRS_MAX 512

struct AoArgs {
    const AoNode *nodes;
    const AoRect *items;
    const AoWall *walls;
    const int32_t *jobs; /* per texel job: wall index; the tile index is the job's offset in its wall */
    const int32_t *job_tile;
    int64_t njobs;
    const float *dirs; /* ndirs xyz triples, the geoSphere4 order */
    int ndirs;
    float fac_sum; /* sequential fp32 sum of the directions' z */
    float *texels; /* float4 per texel */
};

hipError_t fmgi_launch_ao(const AoArgs &a, hipStream_t s);

#endif
