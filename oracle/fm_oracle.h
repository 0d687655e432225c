/*
 * fm_oracle.h -- CPU ORACLE for the photon-mapping hot path (TEST INFRASTRUCTURE ONLY).
 *
 * This is a plain-C restatement of the reference kernel `photonmap.cl` and of the
 * host launch schedule in `global_illumination_cl.c`. Only tests/, __graft_entry__.smoke()
 * and bench.py's cpu_baseline leg may load it, and only as the checker / CPU baseline.
 * The product path (libflatmatch_gi.so) never links, loads or calls anything in oracle/.
 *
 * Arithmetic contract (the "oracle semantics"): photonmap.cl as ROCm's
 * OpenCL compiler builds it for gfx950 with IEEE division/sqrt and no contraction (the reference
 * kernel on MI355X, oracle/build_ref.sh "strict"):
 *   - IEEE-754 binary32 for every float op written in photonmap.cl, in source order, no FMA
 *     contraction, correctly rounded `/` and sqrt();
 *   - the OpenCL builtins as ROCm's device libraries define them: dot and cross as FMA chains,
 *     length(v) = v_sqrt_f32(dot(v,v)), normalize(v) = v * v_rsq_f32(dot(v,v)) (the hardware ops
 *     are reproduced from truth tables recorded on the MI355X, fmo_set_hw_tables), sin/cos = the
 *     device library's fp32 algorithm (OCML __ocml_sin_f32 / __ocml_cos_f32);
 *   - `pos.s2 > 0.0005` compares in double (the literal is a double, photonmap.cl:236);
 *   - host-side code (the launch schedule's area, global_illumination_cl.c:217) keeps the host's
 *     own length() (vector3_cl.c:93);
 *   - texel accumulation is the race-free sum: each deposit channel (always a multiple of
 *     2^-25) is added EXACTLY into an int64 fixed-point accumulator.
 *
 * Parity pinning: the restatement is checked against the reference kernel itself
 * (photonmap.cl compiled for gfx950 by oracle/build_ref.sh and run one work item at a
 * time on the GPU, tests/golden/ref_items_*.npz) -- see DESIGN.md.
 */
#ifndef FM_ORACLE_H
#define FM_ORACLE_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* Byte-identical to the reference `Rectangle` (rectangle.h:19-26): 4 x float4 + int4. */
typedef struct __attribute__((aligned(16))) fmo_rect {
    float pos[4], width[4], height[4], n[4];
    int32_t lm[4]; /* lightmapSetup: [0] texel base, [1] tiles along width, [2] tiles along height */
} fmo_rect;

/* One reference kernel launch (global_illumination_cl.c:246-267), flattened. */
typedef struct fmo_launch {
    uint64_t item_begin; /* index of this launch's gid 0 in the flattened work-item list */
    uint32_t count;      /* workSize (number of work items = gids 0..count-1)            */
    int32_t rng_offset;  /* libc rand() value passed as kernel arg 4                     */
    int32_t source;      /* index into the source list (windows first, then lights)      */
    int32_t is_window;   /* kernel arg 5                                                 */
} fmo_launch;

typedef struct fmo_stats {
    uint64_t photons;  /* tracePhoton calls                          */
    uint64_t scans;    /* rect-list scans (photonmap.cl:194 loop)     */
    uint64_t deposits; /* lightColors[] updates (photonmap.cl:257)   */
    uint64_t escapes;  /* scans that hit nothing (photonmap.cl:208)   */
    uint64_t inexact;  /* deposits whose channels were not multiples of 2^-25 (must stay 0) */
} fmo_stats;

/* One bounce of one photon (for per-photon trace parity). */
typedef struct fmo_event {
    int32_t photon;   /* 0..99 within the work item */
    int32_t depth;    /* 0..7                        */
    int32_t rect;     /* index of the hit rectangle  */
    int32_t texel;    /* lightmapSetup.s0 + tile id  */
    float rgb[3];     /* deposited colour            */
    uint32_t rng;     /* RNG state after the bounce  */
} fmo_event;

#define FMO_FX_SHIFT 25 /* fixed point: 1 unit = 2^-25 */

/* Host schedule (global_illumination_cl.c:215-222,246-256). Does NOT call rand(). Returns the
   number of launches and the total number of work items in *total_items. */
int64_t fmo_schedule_count(const fmo_rect *sources, int nwindows, int nlights, int spa, int wg,
                           uint64_t *total_items);
/* Same, filling `out` and calling libc rand() exactly once per launch, in reference order. */
int64_t fmo_schedule(const fmo_rect *sources, int nwindows, int nlights, int spa, int wg,
                     fmo_launch *out, int64_t cap);

/* Trace flattened work items [item_begin, item_end) of the schedule; adds exact fixed-point
   deposits into lm_fx[numTexels*3]. nthreads<=0 -> OpenMP default. */
void fmo_bake(const fmo_rect *rects, int nrects, const fmo_rect *sources, const fmo_launch *launches,
              int64_t nlaunches, uint64_t item_begin, uint64_t item_end, int64_t *lm_fx,
              int64_t num_texels, int nthreads, fmo_stats *stats);

/* Trace one work item (100 photons) starting from rng_state = gid + rng_offset, recording
   every bounce. Returns the number of events (<= cap are written). */
/* fmo_bake, also adding each texel's deposit count into counts[num_texels] */
void fmo_bake_counts(const fmo_rect *rects, int nrects, const fmo_rect *sources, const fmo_launch *launches,
                     int64_t nlaunches, uint64_t item_begin, uint64_t item_end, int64_t *lm_fx, int64_t *counts,
                     int64_t num_texels, int nthreads, fmo_stats *stats);
int fmo_trace_item(const fmo_rect *rects, int nrects, const fmo_rect *source, int is_window,
                   uint32_t rng_state, fmo_event *ev, int cap, uint32_t *rng_final);

/* Trace one work item and add its deposits into a float4 lightmap in fp32, sequentially in
   deposit order -- exactly what the reference kernel does for a single work item. */
void fmo_trace_item_f32(const fmo_rect *rects, int nrects, const fmo_rect *source, int is_window,
                        uint32_t rng_state, float *texels4);

/* The reference's float RNG and sampler pieces, exposed for unit tests. */
float fmo_rand(uint32_t *state);
void fmo_sincos(float x, float *s, float *c);
void fmo_sincos_n(const float *x, float *s, float *c, int64_t n);
/* gfx950 v_sqrt_f32 / v_rsq_f32 truth tables: int8 ulp deltas from the once-rounded double value for
   x in [1, 4) (index = exponent parity << 23 | mantissa); must be set before any trace. */
void fmo_set_hw_tables(const int8_t *dsqrt, const int8_t *drsq);

/* Convert the fixed-point sums to float texels the way the product does:
   out = (float)((double)in + (double)sum * 2^-25). texels4 has 4 floats per texel. */
void fmo_finalize(const int64_t *lm_fx, int64_t num_texels, const float *texels_in, float *texels_out);

#ifdef __cplusplus
}
#endif
#endif
