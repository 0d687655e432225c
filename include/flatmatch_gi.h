/*
 * flatmatch_gi.h -- C ABI of libflatmatch_gi.so, the MI355X-native drop-in for the reference's
 * OpenCL photon-mapping path (rbuch703/flatmatch-global-illumination).
 *
 * Drop-in entry point (replaces global_illumination_cl.c:275-321, declared at
 * global_illumination_cl.h:10):
 *
 *     void performGlobalIlluminationCl(Geometry *geo, int numSamplesPerArea);
 *
 * The reference's main.c (main.c:63) links against this library unchanged: it includes its own
 * global_illumination_cl.h; the symbol name, argument meaning, in-place texel update and fatal-error
 * behaviour (message on stdout + exit(-1), global_illumination_cl.c:254,263) are the reference's.
 * libc rand() is consumed once per kernel launch of the reference schedule
 * (global_illumination_cl.c:251), so RNG seeds and post-call libc state match the reference.
 *
 * Everything else here is build-defined (prefix fmgi_) and exists so tests and bench.py can drive
 * the device-resident path with plain pointers: no torch or HIP types cross this boundary
 * (streams are passed as void* hipStream_t, device buffers as void*).
 *
 * Environment knobs the reference ABI cannot carry (read by performGlobalIlluminationCl):
 *   FMGI_WG        virtual OpenCL work-group size of the launch schedule (default 256, the value
 *                  ROCm's OpenCL reports for CL_KERNEL_WORK_GROUP_SIZE; global_illumination_cl.c:300)
 *   FMGI_GPUS      number of GPUs one drop-in call shards over (default 1, like the reference; max 8)
 *   FMGI_REDUCE    how a multi-GPU call sums the shard lightmaps: "rccl" (default: one ncclReduce over
 *                  the shard devices) or "peer" (binary tree of xGMI peer copies + adds)
 *   FMGI_KERNEL    "auto" (default), "grid", "fast", "hybrid" or "exact" -- all produce identical bits
 *   FMGI_DROPIN_CACHE  0, 1 (default) or 2: device state kept between calls (fmgi_dropin_release)
 *   FMGI_QUIET     1 = suppress the reference's progress line
 */
#ifndef FLATMATCH_GI_H
#define FLATMATCH_GI_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ---- Layout-identical equivalents of the reference ABI types (no CL headers needed). ---------- */
/* Vector3 == cl_float4 (vector3_cl.h:14): 16 B, 16-B aligned; .s[3] unused.                      */
typedef struct __attribute__((aligned(16))) fmgi_vec3 { float s[4]; } fmgi_vec3;
/* Rectangle (rectangle.h:19-26): 80 B, 16-B aligned. lightmapSetup = {texel base, tiles along
   width, tiles along height, 0}. Windows/lights have lightmapSetup.s0 == 0.                       */
typedef struct __attribute__((aligned(16))) fmgi_rect {
    fmgi_vec3 pos, width, height, n;
    int32_t lightmapSetup[4];
} fmgi_rect;
/* Geometry (geometry.h:7-15): 80 B. boxWalls are not used by the photon-mapping path.             */
typedef struct fmgi_geometry {
    fmgi_rect *windows, *lights, *walls, *boxWalls;
    int32_t numWindows, numLights, numWalls, numBoxWalls;
    int32_t width, height;
    float startingPositionX, startingPositionY;
    int32_t numTexels;
    fmgi_vec3 *texels;
} fmgi_geometry;

/* ---- Drop-in entry points ----------------------------------------------------------------------- */
#ifndef GLOBAL_ILLUMINATION_CL /* the reference header declares it with its own Geometry type */
void performGlobalIlluminationCl(fmgi_geometry *geo, int numSamplesPerArea);
#endif
/* North-star name, build-defined (the reference has no such symbol): same bake, but the result is
   written to texels_out[numTexels] (initial values taken from geo->texels, which is not modified).
   Returns 0 on success, a negative fmgi error code otherwise (no exit()). */
int getGlobalIlluminationCl(const fmgi_geometry *geo, int numSamplesPerArea, fmgi_vec3 *texels_out);
/* The drop-in entry points keep their per-geometry device state (contexts, scene tables, lightmaps; a
   few MB per shard) across calls and free the deposit-code stream buffers at the end of every call
   (FMGI_DROPIN_CACHE=1, the default); FMGI_DROPIN_CACHE=0 frees everything after every call, as the
   reference does (global_illumination_cl.c:315-320); FMGI_DROPIN_CACHE=2 keeps the stream buffers too.
   This frees all of it, and the RCCL communicators of a multi-GPU call. */
void fmgi_dropin_release(void);
/* Ranks of the RCCL communicator the last multi-GPU drop-in call reduced over (ncclCommCount; one rank
   per shard device), 0 if that call reduced without RCCL. */
int fmgi_dropin_rccl_ranks(void);
/* The drop-in's multi-GPU layout (host only; for tests): shard k -> device dev[k], work items
   [begin[k], end[k]); and its binary-tree reduction into shard 0 (returns the step count, nshard - 1). */
int fmgi_dropin_shards(uint64_t items, int ngpu, int nshard, int32_t *dev, uint64_t *begin, uint64_t *end);
int fmgi_dropin_reduce_order(int nshard, int32_t *dst, int32_t *src);

/* ---- Ambient occlusion ------------------------------------------------------ */
/* The reference's performAmbientOcclusionNative (global_illumination_native.h:16, photonmap.c:478-490)
   on the GPU, bit-identical: every level-0 texel of every wall becomes (d, d, d, 0), d the
   cosine-weighted mean distance over the 481 geoSphere4 directions (misses count 10), traced through
   the reference's BSP tree. Same argument meaning and in-place update; a different name, because the
   reference's photonmap.o (which main.c also needs for performPhotonMappingNative) already defines
   performAmbientOcclusionNative. Fatal errors print "[Err] ..." and exit(-1). */
void performAmbientOcclusionGpu(fmgi_geometry *geo);
/* Non-mutating form for walls [wall_begin, wall_end) (the BSP always spans every wall):
   texels_out = geo->texels with those walls' level-0 texels replaced. Returns 0 or FMGI_ERR_*. */
int fmgi_ambient_occlusion(const fmgi_geometry *geo, int wall_begin, int wall_end, fmgi_vec3 *texels_out);
/* The direction table of `levels` subdivisions (4 = the AO table, 481 directions) in the reference's
   order, as xyz float triples; returns the count and copies at most `cap` directions. */
int fmgi_geosphere(int levels, float *xyz, int cap);
/* The AO BSP tree, encoded per node as {left, right, plane wall, n, n wall indices}; returns the
   encoding's length and copies at most `cap` ints. */
int64_t fmgi_ao_tree(const fmgi_geometry *geo, int32_t *out, int64_t cap);

/* ---- Output step: what main.c:66-95 does after the bake, minus the PNG encoding */
/* Normalisation for the photon modes (main.c:66-79; numSamplesPerArea = 0 skips it, as the reference
   does for AO/radiosity), then every wall's RGB8 tile as the reference's saveAs()/saveAs_core
   (rectangle.c:295-345) builds it before write_png_file: tone map 1 - exp(-2 L), clamp, floor tint
   (tintExtra: the second tint of the AO/native modes). texels_out = geo->texels normalised;
   rgb_out = the walls' tiles concatenated in wall order, fmgi_output_tile_bytes(geo) bytes.
   Byte-identical to the reference. Returns 0 or FMGI_ERR_*. */
int fmgi_output_tiles(const fmgi_geometry *geo, int numSamplesPerArea, int tintExtra, fmgi_vec3 *texels_out,
                      uint8_t *rgb_out);
int64_t fmgi_output_tile_bytes(const fmgi_geometry *geo);

/* ---- Radiosity --------------------------------------------------------------- */
/* The reference's performRadiosityNative (radiosityNative.h:10, radiosityNative.c:92-268) on the GPU:
   10000 libc-rand() cosine rays per level-0 wall texel against its sorted candidate list, then 7
   gather/update/mipmap bounces; geo->texels[0, numTexels) receive the result (w = 0). The caller's
   libc rand() stream (glibc's default TYPE_3 generator) is replayed on the device and left where the
   reference leaves it (2 x 10000 draws per level-0 wall texel). Same argument meaning and in-place
   update; a different name so that the reference's radiosityNative.o can stay linked. Fatal errors
   print "[Err] ..." and exit(-1). */
void performRadiosityGpu(fmgi_geometry *geo);
/* Non-mutating form: texels_out[numTexels] = the result; sids_out (NULL or jobs x 10000 int32) = the
   reference's sourceTexelIds rows of the level-0 wall texels, wall/tile order (-1: the ray hit
   nothing). Returns 0 or FMGI_ERR_*. */
int fmgi_radiosity(const fmgi_geometry *geo, fmgi_vec3 *texels_out, int32_t *sids_out);
/* number of level-0 wall texels (jobs); the rand() draws of a call are 20000 x this */
int64_t fmgi_radiosity_jobs(const fmgi_geometry *geo);
typedef struct fmgi_rad_stats {
    int64_t jobs, rects, texels, rays; /* texels includes the window/light texels */
    double rand_ms;                    /* device rand() replay */
    double rays_ms;                    /* candidate lists + ray casts (+ uploads) */
    double bounce_ms;                  /* 7 x (gather, update, mipmap) */
    double total_ms;                   /* first upload .. last bounce */
} fmgi_rad_stats;
/* statistics of the last fmgi_radiosity / performRadiosityGpu call */
int fmgi_radiosity_stats(fmgi_rad_stats *out);
/* Host only: advance the caller's libc rand() generator by n draws with the jump matrices the
   radiosity backend uses (as n rand() calls would). Returns 0 or FMGI_ERR_ARG (not glibc TYPE_3). */
int fmgi_rand_skip(uint64_t n);

/* ---- Build-defined device-resident API ---------------------------------------------------------- */
enum {
    FMGI_OK = 0,
    FMGI_ERR_NO_DEVICE = -1,
    FMGI_ERR_HIP = -2,
    FMGI_ERR_ARG = -3,
    FMGI_ERR_STATE = -4,
    FMGI_ERR_OOM = -5
};

/* Scan kernels (identical bits): EXACT = photonmap.cl's scan over every rect; FAST = conservative fp32
   filter over every rect + exact verification; GRID = FAST's filter over per-plane grid cells only;
   HYBRID = GRID's cells for the floor/ceiling planes and FAST's filter for the walls. */
enum { FMGI_KERNEL_EXACT = 0, FMGI_KERNEL_FAST = 1, FMGI_KERNEL_GRID = 2, FMGI_KERNEL_AUTO = 3, FMGI_KERNEL_HYBRID = 4 };
/* AUTO = GRID when the scene has few planes for its rect count (closed boxes), HYBRID when only the
   floor/ceiling records share few planes (apartment layouts), else FAST; a scan whose image does not
   fit LDS falls back to one that does (EXACT needs none). */
/* Deposit accumulation (both exact and order-free; results are identical):
   FX3   three int64 fixed-point atomics per deposit into the lightmap;
   STATE one u64 atomic per deposit into counts[colour state][texel] (8 KiB per texel of device memory),
         folded into the int64 lightmap at the end of every fmgi_bake_items;
   STREAM no atomics per deposit: 32-bit codes (texel << 10 | colour state) collected in each wave's LDS
         ring and written with 16-B stores (when the lightmap has at most 63 fold tiles of 2048 texels,
         sorted by tile into per-wave, per-tile 4-KB buckets; else into plain blocks that a second pass
         sorts per 8192-code slice), then summed per tile exactly in LDS (needs < 4,194,304 texels; the
         codes of a chunk of work items stay in HBM, 3.2 KB per work item at most, chunks sized to half
         of the free device memory: one 1e9-photon chunk on an MI355X);
   AUTO  STREAM when the texel count allows it, else FX3;
   NONE  PROFILING ONLY: deposits are discarded (measures the tracing work alone; wrong lightmap). */
enum { FMGI_ACCUM_AUTO = 0, FMGI_ACCUM_FX3 = 1, FMGI_ACCUM_STATE = 2, FMGI_ACCUM_NONE = 3, FMGI_ACCUM_STREAM = 4 };

/* Per-bake counters, accumulated on the device (one atomic per wave). */
typedef struct fmgi_stats {
    uint64_t photons;   /* tracePhoton calls                                     */
    uint64_t scans;     /* rectangle-list scans (photonmap.cl:194)                */
    uint64_t deposits;  /* lightmap deposits (photonmap.cl:257)                   */
    uint64_t escapes;   /* scans that hit nothing (photonmap.cl:208)              */
    uint64_t exact_rescans; /* fast kernel: scans re-done by the exact scan          */
    uint64_t tests;     /* rectangle tests actually evaluated                      */
    uint64_t rescans_tie;     /* exact_rescans caused by a runner-up within the separation band */
    uint64_t rescans_invalid; /* exact_rescans caused by a phase-1 winner that is not exactly valid */
    uint64_t stream_overflow; /* STREAM: reservations past the stream capacity (must stay 0) */
} fmgi_stats;

/* One work item of the flattened reference launch schedule (global_illumination_cl.c:246-267). */
typedef struct fmgi_launch {
    uint64_t item_begin; /* flattened index of this launch's gid 0 */
    uint32_t count;      /* workSize                               */
    int32_t rng_offset;  /* rand() value (kernel arg 4)             */
    int32_t source;      /* windows first, then lights              */
    int32_t is_window;   /* kernel arg 5                            */
} fmgi_launch;

/* One recorded bounce (debug trace mode, for per-photon parity tests). */
typedef struct fmgi_event {
    int32_t photon, depth, rect, texel;
    float rgb[3];
    uint32_t rng;
} fmgi_event;

typedef struct fmgi_context fmgi_context;

const char *fmgi_version(void);
const char *fmgi_last_error(void);
int fmgi_device_count(void);

/* Create a context on HIP device `device` (hipSetDevice is called). NULL on failure.
   device == FMGI_HOST_ONLY gives a context without a device: scene checks and fmgi_plan work, every
   device operation returns FMGI_ERR_NO_DEVICE (used by the CPU test-suite). */
#define FMGI_HOST_ONLY (-1)
fmgi_context *fmgi_create(int device);
void fmgi_destroy(fmgi_context *ctx);

/* Upload the scene: wall rectangles (the rect list scanned by every photon) and the emitters
   (windows first, then lights). The per-rectangle values photonmap.cl derives with OpenCL builtins
   (edge lengths, unit edges, sampler bases) are computed on the device by k_scene_setup with the
   builtins' gfx950 instructions, so they carry the reference kernel's bits; the scan tables (filter
   image, grid) are built on the host. */
int fmgi_set_scene(fmgi_context *ctx, const fmgi_rect *walls, int num_walls, const fmgi_rect *windows,
                   int num_windows, const fmgi_rect *lights, int num_lights, int num_texels);

/* Select the accumulation mode (FMGI_ACCUM_*); takes effect for the current and later scenes. */
int fmgi_set_accumulation(fmgi_context *ctx, int mode);
/* The mode in effect (FMGI_ACCUM_FX3, FMGI_ACCUM_STATE, FMGI_ACCUM_STREAM or FMGI_ACCUM_NONE). */
int fmgi_get_accumulation(fmgi_context *ctx);

/* Reference launch schedule for spa / wg. If rng_offsets is NULL, libc rand() is called once per
   launch in reference order; otherwise offsets are taken from rng_offsets[0..n_offsets).
   Returns the number of launches (>=0) or an error code; *total_items receives the work-item count
   (photons = 100 * items). The schedule is kept in the context for fmgi_bake_items. */
int64_t fmgi_plan(fmgi_context *ctx, int spa, int wg, const int32_t *rng_offsets, int64_t n_offsets,
                  uint64_t *total_items);
/* Copy the current schedule out (cap entries). Returns the number of launches. */
int64_t fmgi_get_plan(fmgi_context *ctx, fmgi_launch *out, int64_t cap);
/* Schedule helpers that do not call rand(). */
int64_t fmgi_plan_count(const fmgi_rect *windows, int num_windows, const fmgi_rect *lights, int num_lights,
                        int spa, int wg, uint64_t *total_items);

/* Trace flattened work items [item_begin, item_end) of the planned schedule on `stream`, adding
   exact fixed-point deposits (int64, units of 2^-25, layout [numTexels][4], .s[3] unused) into the
   device buffer lm_fx. Asynchronous; the buffer must be zeroed (or hold a previous partial sum). */
int fmgi_bake_items(fmgi_context *ctx, uint64_t item_begin, uint64_t item_end, void *lm_fx_dev,
                    int kernel, void *stream);
/* Device-side finalisation: texels_out[i].c = (float)((double)texels_in[i].c + lm_fx[i].c * 2^-25),
   .s[3] copied. Either texel pointer may alias. */
int fmgi_finalize(fmgi_context *ctx, const void *lm_fx_dev, const void *texels_in_dev, void *texels_out_dev,
                  void *stream);
/* The kernel FMGI_KERNEL_AUTO resolves to for the current scene. */
int fmgi_auto_kernel(const fmgi_context *ctx);
/* The profiler's name of the k_bake instance the last bake launch ran ("void (anonymous namespace)::k_bake<...>
   (BakeArgs)"; two names joined by " + " for the launch-tail pair), written NUL-terminated into buf (truncated
   to cap - 1 characters); returns its full length, 0 before the first bake. No reference counterpart: the
   measurement's handle on which instance the committed counter summaries must name. */
int fmgi_last_bake_kernel(const fmgi_context *ctx, char *buf, int cap);
/* Device-side timing of the bake's kernels (HIP events around each launch, on the bake's stream), off
   by default. fmgi_get_timing synchronises, returns the sums since the previous call and resets them. */
typedef struct {
    double bake_ms;         /* k_bake launches                                   */
    double fold_ms;         /* STREAM fold (k_bucket_count/list/fold, k_tile_runs_pre, or k_slice_sort +
                               k_tile_runs / k_tile_runs_pre over slices) */
    uint64_t bake_launches;
    uint64_t fold_launches;
} fmgi_timing;
int fmgi_set_timing(fmgi_context *ctx, int on);
int fmgi_get_timing(fmgi_context *ctx, fmgi_timing *out);
/* Counters of all bakes since the last reset (synchronises the context's device). */
int fmgi_get_stats(fmgi_context *ctx, fmgi_stats *out);
int fmgi_reset_stats(fmgi_context *ctx);
/* Debug trace: runs items [item_begin, item_end) (<= 4096 items) with the chosen kernel and returns
   every bounce in events[(item - item_begin) * 800 + k] (800 = 100 photons x 8 bounces), the number
   of events per item in counts[], and the final per-item RNG state in rng_final[]. Synchronous. */
int fmgi_trace_items(fmgi_context *ctx, uint64_t item_begin, uint64_t item_end, int kernel,
                     fmgi_event *events, int32_t *counts, uint32_t *rng_final);

/* Grid tables of FMGI_KERNEL_GRID (built by fmgi_set_scene; host-only contexts too), for tests and
   tooling. sizes[0..2] = plane pairs per axis (x, y, z), sizes[3] = cells, sizes[4] = overflow entries.
   fmgi_grid_copy fills (any pointer may be NULL):
     planes[2 * (sizes[0] + sizes[1] + sizes[2])]: per axis, pairs {plane of the +n class, plane of the
       -n class}, each {float plane, u0, v0, iu, iv, mu, mv; int32 nu, nv, cell_off; float ulo, uhi,
       vlo, vhi (the records' box, rounded outward), pad[2]} (64 B; mu = nu - 1, mv = nv - 1; NaN
       plane = padding);
     cells[sizes[3]] (32 B each): the cell's first two records as quantized bounds {uint32 qu, qv} each
       ({lo | hi << 16} of the cell's 16-bit fixed-point coordinates that the record's margin-grown
       extent can reach; {0xFFFF, 0xFFFF} when absent), then {int32 count, rect index of record 0, of
       record 1, first overflow entry};
     recs[4 * sizes[4]], idx[sizes[4]]: the overflow records (entries 3..count of every cell) and their
       rect indices. */
int fmgi_grid_sizes(const fmgi_context *ctx, int32_t sizes[5]);
/* The grid's cells per record for the next fmgi_set_scene of ctx (0, the default: the product's choice, 16,
   or the coarse LDS grids of the closed boxes); tests use it to check the grids those choices build. */
int fmgi_set_grid_cells_per_record(fmgi_context *ctx, int cells_per_record);
/* 1 in the experiment build (make experiments -> libflatmatch_gi_exp.so), whose experiment knobs
   (environment variables of measured-and-rejected paths) it reads; 0 in the product library. */
int fmgi_experiments(void);
/* Per-context handles on product paths that a given scene or launch size would not take, for tests (each
   takes effect at the next bake; FMGI_OPT_NO_AXES at the next fmgi_set_scene):
     FMGI_OPT_CHUNK_ITEMS   > 0: at most this many work items per STREAM chunk (several chunks per call)
     FMGI_OPT_POOL_LIMIT    > 0: at most this many bucket-pool blocks (the exact atomic fallback takes the rest)
     FMGI_OPT_STREAM_LAYOUT 0: the slice-sorted stream (lightmaps of more than 63 tiles); -1: by the scene
     FMGI_OPT_BUCKET_FILL   0: per-wave LDS rings, 1: lane-by-lane stores; -1: by the tables' LDS fit
     FMGI_OPT_WIDE_TILES    0 / 1: 2048- / 4096-texel bucket tiles; -1: by the launch size
     FMGI_OPT_COOP          2, 4, 8: lanes per work item of ScanFast's small launches; 0: by the launch size
     FMGI_OPT_NO_AXES       1: closed boxes through the general grid instance (its sorted <= 4-slot phase 1) */
#define FMGI_OPT_CHUNK_ITEMS 1
#define FMGI_OPT_POOL_LIMIT 2
#define FMGI_OPT_STREAM_LAYOUT 3
#define FMGI_OPT_BUCKET_FILL 4
#define FMGI_OPT_WIDE_TILES 5
#define FMGI_OPT_COOP 6
#define FMGI_OPT_NO_AXES 7
#define FMGI_OPT_COUNT 8
int fmgi_set_option(fmgi_context *ctx, int option, int64_t value);
/* Profiling builds only (make timing -> libflatmatch_gi_timing.so, -DFMGI_STAGE_TIMING): shader-clock
   cycles summed over waves per bake-loop stage {start, sample, scan phase 1, phase 2, fallback, hit,
   append}, since the last fmgi_reset_stats; all zero in the normal library. */
int fmgi_get_stage_cycles(fmgi_context *ctx, uint64_t out[16]);
int fmgi_grid_copy(const fmgi_context *ctx, void *planes, void *cells, float *recs, int32_t *idx);
/* FMGI_KERNEL_HYBRID's floor plan of the walls (built by fmgi_set_scene; host-only contexts too; the
   hybrid scan walks it with FMGI_PLAN=1): *bytes = its size (0: no plan for this scene); with
   blob != NULL and *bytes >= that size, copies it: {float x0, y0, 1 / cs, cs}, {int32 nx | ny << 16,
   ncells, nentries, 0}, u16 start[ncells + 1], u16 entry[nentries] (cell (ix, iy) = iy * nx + ix lists
   entry[start[i] .. start[i + 1]]: 32-B records of the filter image, record r at byte 32 r; x walls
   first, r & 1 = the class, +n = 0). */
int fmgi_plan_copy(const fmgi_context *ctx, void *blob, int32_t *bytes);
/* The filter image of FMGI_KERNEL_FAST / HYBRID (built by fmgi_set_scene; host-only contexts too): pairs[a]
   = its pairs on axis a; *bytes = its size; with img != NULL and *bytes >= that size, copies it: per axis,
   pairs[a] pairs {record of the +n class, record of the -n class}, then 16 padding records; a record is
   {float plane, cu, hwu, cv, hwv; int32 rect index (-1: padding); pad[2]} (32 B; extents grown by the
   filter margin). Pair j holds record j of each class, rect order. */
int fmgi_filter_copy(const fmgi_context *ctx, void *img, int32_t *bytes, int32_t pairs[3]);
/* FMGI_KERNEL_HYBRID's wall-pair image (built by fmgi_set_scene; host-only contexts too): for the x and then
   the y axis, groups[a] groups of two 48-B halves (the +a class, then the -a class), each half
   {float plane[2], cu[2], hwu[2], cv[2], hwv[2]; int32 rect index[2]} = records 2g and 2g + 1 of its class as
   the filter image holds them (a missing record: hwu = hwv = -1, index -1). Same size protocol. */
int fmgi_pairs_copy(const fmgi_context *ctx, void *img, int32_t *bytes, int32_t groups[2]);

/* Host helpers exported for tests (no device needed). */
void fmgi_host_sincosf(const float *x, float *s, float *c, int64_t n);
/* Device-side twin of fmgi_host_sincosf over n inputs (synchronous; for parity tests). */
int fmgi_device_sincosf(fmgi_context *ctx, const float *x, float *s, float *c, int64_t n);
/* The device library's own sinf/cosf (ROCm ocml, what photonmap.cl's sin/cos run on MI355X) over n
   inputs, for checking the restatement (synchronous; parity tests). */
int fmgi_device_sincosf_library(fmgi_context *ctx, const float *x, float *s, float *c, int64_t n);
/* Device arithmetic helpers of the bake kernel over n inputs (synchronous; for parity tests):
   op FMGI_UNIT_SQRT: out[i] = bits of the sampler's correctly rounded sqrtf(a[i]) (b unused);
   op FMGI_UNIT_TRUNC_DIV: out[i] = (int)(a[i] / b[i]), the tile index step of photonmap.cl:108-109
   (through v_rcp_f32); op FMGI_UNIT_TRUNC_DIV_INV: the same through the host-rounded 1.0f / b[i]. */
#define FMGI_UNIT_SQRT 0
#define FMGI_UNIT_TRUNC_DIV 1
#define FMGI_UNIT_TRUNC_DIV_INV 2
int fmgi_device_unit(fmgi_context *ctx, int op, const float *a, const float *b, int32_t *out, int64_t n);

#ifdef __cplusplus
}
#endif
#endif
