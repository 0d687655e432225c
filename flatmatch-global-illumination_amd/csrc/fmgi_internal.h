/*
 * fmgi_internal.h -- interface between the host C ABI (fmgi_api.cpp) and the HIP kernels
 * (fmgi_kernels.hip). Not installed; not part of the C ABI.
 */
#ifndef FMGI_INTERNAL_H
#define FMGI_INTERNAL_H

#include <hip/hip_runtime_api.h>
#include <stdint.h>

#include "fmgi_core.h"

struct BakeArgs {
    const RectDev *rects;
    int nrects;
    const SrcDev *srcs;
    const LaunchDev *launches;
    int nlaunches;
    uint64_t item_begin, item_end;
    unsigned long long *counter;   /* work-item fetch counter, zeroed before each bake */
    unsigned long long *lm;        /* int64 fixed point [numTexels][4]                   */
    unsigned long long *stats;     /* fmgi_stats words                                   */
    /* fast-kernel filter parameters (fmgi_kernels.hip, "conservative filter") */
    int axis_begin[7];             /* rects sorted by axis class: [axis_begin[c], axis_begin[c+1]) */
    float eps_abs;                 /* absolute slack of the filter (scene-scale dependent)          */
    /* debug trace (TRACE kernels only) */
    void *events;                  /* fmgi_event[(item - item_begin) * 800 + k]                     */
    int32_t *ev_counts;
    uint32_t *rng_final;
};

enum { KSTAT_PHOTONS = 0, KSTAT_SCANS, KSTAT_DEPOSITS, KSTAT_ESCAPES, KSTAT_RESCANS, KSTAT_TESTS, KSTAT_N = 8 };

hipError_t fmgi_launch_bake(const BakeArgs &a, int kernel, bool trace, int grid_blocks, hipStream_t s);
hipError_t fmgi_launch_finalize(const unsigned long long *lm, const float *tin, float *tout, int64_t n,
                                hipStream_t s);
hipError_t fmgi_launch_sincos(const float *x, float *sn, float *cs, int64_t n, hipStream_t s);
int fmgi_block_size();

#endif
