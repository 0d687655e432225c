/*
 * fmgi_internal.h -- interface between the host C ABI (fmgi_api.cpp) and the HIP kernels
 * (fmgi_kernels.hip). Not installed; not part of the C ABI.
 */
#ifndef FMGI_INTERNAL_H
#define FMGI_INTERNAL_H

#include <hip/hip_runtime_api.h>
#include <stdint.h>

#include <string>

#include "fmgi_lds_attr.h"

#include "fmgi_core.h"

/* One axis-aligned rectangle as the conservative filter sees it (32 B = one s_load_dwordx8):
   the plane coordinate along its normal's axis a, and centre / half-extent (+ margin) along the two
   other axes u < v. idx = index in the rect list (the exact data is in RectDev[idx]). */
/* Experiment knobs: FMGI_EXPERIMENTS builds (make experiments -> libflatmatch_gi_exp.so, FMGI_LIB=exp) read the
   environment variables of the measured-and-rejected paths (dense stream + k_bin, presorted segments, split
   folds, 8192-texel tiles, per-workgroup tile lines, the floor-plan walk, staging and launch-shape overrides);
   the product library reads none of them and does not contain those kernel instances. */
#ifndef FMGI_EXPERIMENTS
#define FMGI_EXPERIMENTS 0
#endif
#include <stdlib.h>
static inline const char *fmgi_exp_env(const char *name) {
#if FMGI_EXPERIMENTS
    return getenv(name);
#else
    (void)name;
    return nullptr;
#endif
}

struct FilterRec {
    float plane, cu, hwu, cv, hwv;
    int32_t idx;
    float pad0, pad1;
};
static_assert(sizeof(FilterRec) == 32, "FilterRec must be 32 B");

/* ScanHybrid's wall filter, two records per group (FilterPairs, 96 B): for each class c of the axis (+a
   class first, then -a), records 2g and 2g + 1 of the class as field pairs, so each pair loads into a
   64-bit register pair for packed fp32 ops: {plane0, plane1, cu0, cu1}, {hwu0, hwu1, cv0, cv1},
   {hwv0, hwv1, idx0, idx1} (idx = rect index; a missing record is a never-valid sentinel, hwu = hwv = -1). */
struct FilterPairHalf {
    float plane[2], cu[2], hwu[2], cv[2], hwv[2];
    int32_t idx[2];
};
static_assert(sizeof(FilterPairHalf) == 48, "FilterPairHalf must be 48 B");

/* One plane of the grid kernel (ScanGrid): all axis-aligned rects of one class (axis a, normal sign)
   that lie in the plane x_a = plane, bucketed by a nu x nv grid over the plane's (u, v) bounding box of
   their margin-grown extents. Cell (iu, iv) = cells[cell_off + iv*nu + iu] = {first record, count}. */
struct GridPlane {
    float plane, u0, v0, iu; /* iu, iv = cells per unit length */
    float iv, mu, mv;        /* mu = nu - 1, mv = nv - 1 (the clamp bounds of the cell coordinates) */
    int32_t nu, nv, cell_off;
    float ulo, uhi, vlo, vhi; /* box of the plane's grown record extents, rounded outward: a hit point
                                 outside it passes no record test, so its cell need not be loaded */
    float pad0, pad1;
};
static_assert(sizeof(GridPlane) == 64, "GridPlane must be 64 B");

/* One grid cell (32 B: two 16-B loads per lookup). Its first two records are inline as quantized bounds
   with their rect indices; records 3..count live in the overflow arrays at [rest, rest + count - 2) as
   float records. The kernel maps a hit point to the cell's 16-bit fixed-point coordinates
   q = clamp(floor((t - cell) * 65536), 0, 65535), t its float cell coordinate (grid_cell); a record's
   bounds {lo | hi << 16} per axis are q at the smallest and largest float that pass the record's float
   test |x - c| <= hw, so every point that passes the float test passes lo <= q <= hi (q is monotone in x):
   a superset, as the exactness argument needs. An absent record is {0xFFFF, 0} (never a candidate). */
struct GridCell {
    uint32_t qu0, qv0, qu1, qv1;
    int32_t count, idx0, idx1, rest;
};
static_assert(sizeof(GridCell) == 32, "GridCell must be 32 B");
constexpr uint32_t kGridNoRec = 0xFFFFu; /* lo 0xFFFF, hi 0: no q passes */
/* the same cell with float records (centre, half-extent; absent: half-extent -1), read by the general
   grid walks (many planes per scan), where the 16-bit cell coordinates cost more per visited plane than
   the 16 B they save */
struct GridCellF {
    float cu0, hwu0, cv0, hwv0;
    float cu1, hwu1, cv1, hwv1;
    int32_t count, idx0, idx1, rest;
};
static_assert(sizeof(GridCellF) == 48, "GridCellF must be 48 B");

/* The compact closed-box tables (ScanGridT's Compact instance, FMGI_KVAR_COMPACT): closed boxes whose RectLds
   walls (112 B each) and 32-B grid cells do not fit LDS (BASELINE config 5: 2000 walls) stage instead
     - RectC: phase 2's per-wall fields, 24 B (2000 walls: 48 KB): pos, length(width), length(height), and
       meta = texel base (22 bits) | class (10 bits);
     - ClassC: what walls share, 64 B per distinct bit pattern of {n, width / length(width), height /
       length(height), sampler basis bu, bv, W, H} (a closed box has a few per plane);
     - the walls' float filter extents {cu, hwu, cv, hwv} by rect index (16 B; one never-valid dummy after
       the last wall);
     - CellC: a grid cell as up to four u16 rect indices (8 B; absent = the dummy), no inline bounds.
   The host builds RectC / ClassC from the device-computed RectDev and checks that every field round-trips bit
   for bit (fmgi_api.cpp build_compact); 1 / length, which only the tile index's quotient estimate uses (any
   value within one ulp gives the same tile, fmgi_core.h trunc_div_inv), is v_rcp_f32 of the length. */
struct RectC {
    float px, py, pz, wl;
    float hl;
    uint32_t meta; /* texel base | class << 22 */
};
static_assert(sizeof(RectC) == 24, "RectC must be 24 B");
struct __attribute__((aligned(16))) ClassC {
    float nx, ny, nz, wnx;
    float wny, wnz, hnx, hny;
    float hnz, bux, buy, buz;
    float bvx, bvy, bvz;
    int32_t WH; /* W | H << 16 */
};
static_assert(sizeof(ClassC) == 64, "ClassC must be 64 B");
constexpr int kCompactBaseBits = 22;
constexpr int kCompactMaxClasses = 1 << (32 - kCompactBaseBits);

struct BakeArgs {
    const RectDev *rects;
    int nrects;
    const SrcDev *srcs;
    const LaunchDev *launches;
    int nlaunches;
    /* work item -> launch: per source, its first flattened item (nsrc + 1 entries) and first launch */
    const uint64_t *src_item_begin;
    const int32_t *src_launch0;
    int nsrc, nwindows;
    uint32_t launch_cap; /* WG * 100 items per reference launch */
    uint64_t item_begin, item_end;
    unsigned long long *counter;   /* work-item fetch counter, zeroed before each bake */
    unsigned long long *lm;        /* int64 fixed point [numTexels][4]                   */
    unsigned long long *stats;     /* fmgi_stats words                                   */
    /* fast-kernel filter (fmgi_kernels.hip, ScanFast): the LDS image = for each axis a, fJ[a] pairs of
       FilterRec {+a class record j, -a class record j} (64 B per pair; the shorter class is padded with
       never-valid sentinels). Rects that are not axis-aligned are listed in `general`. */
    const void *fimg;
    int fimg_bytes;
    int fJ[3];
    const int32_t *general;
    int ngeneral;
    /* grid kernel (ScanGrid): fimg/fJ then hold GridPlane pairs {+a plane j, -a plane j}; the cells
       (GridCell), the overflow records (float4 {cu, hwu, cv, hwv}) and their rect indices live in
       global memory */
    const void *gcells;
    const void *gcellsF;  /* GridCellF, same indices */
    const float *grecs;
    const int32_t *gridx;
    int grid_axes; /* fJ == {1, 1, 1}: slot a of the image is axis a (ScanGrid's grid_phase1_axes) */
    int grid_xy_separate; /* layouts: walk the x and y planes one axis after the other (else merged) */
    /* >= 0: byte offsets in the staged LDS blob (fimg) of a copy of the RectDev table (the phase-2 reads of
       the scans' winners) and of the SrcDev table (every photon's emission); -1: read from global memory */
    int rects_off, srcs_off;
    int cells_off;        /* >= 0: byte offset of a copy of the grid cells (GridCell) in the staged blob */
    int grecs_off;        /* >= 0 (with cells_off): byte offsets of copies of the grid's overflow records */
    int gidx_off;         /*   (float4) and their rect indices (int32) in the staged blob             */
    int gJ[3];            /* ScanHybrid: the grid's plane pairs per axis; its plane image is at LDS  */
    int hyb_off;          /* offset hyb_off after the filter image (fimg = filter image || plane image) */
    int plan_off;         /* ScanHybridPlan: byte offset of the floor plan in the image (-1: none)      */
    int pair_off;         /* ScanHybrid: byte offset of the wall-pair image (FilterPairs) in the image  */
    int pG[2];            /* ScanHybrid: FilterPairs groups per axis (x, y)                            */
    const uint32_t *fetch_tab;    /* fetch_nseg > 0: [f_begin, item_begin] pairs, f_begin ascending from 0:
                                     fetch f maps into the segment holding it (sums are order-free) */
    int fetch_nseg;
    unsigned long long *src_cost; /* non-null: per-source scan totals of the finished items */
    int grid_code_or;     /* ScanHybrid: flag or-ed into the codes of grid records (rect indices)    */
    /* the compact closed-box instance (FMGI_KVAR_COMPACT): byte offsets in the staged blob of the RectC,
       ClassC, filter-extent (float4 by rect index) and CellC tables, and the dummy record's index */
    int rectc_off, class_off, recf_off, cellc_off, cdummy;
    /* the launch tail of layouts with few work items per lane (ScanHybridT's Tail modes, fmgi_api.cpp
       bake_common): the saving launch counts its lanes that found no item left in *tail_idle and, once
       tail_at of them are idle, every lane still in an item saves it at its next photon boundary (tail_states[*tail_n++], 16 B)
       and leaves; the resuming launch's groups of `coop` lanes take the saved states through *tail_next and
       finish those items with the wall loop split among them */
    unsigned *tail_idle, *tail_n, *tail_next;
    uint32_t tail_at;
    int tail_flag_off;    /* the saving launch: LDS byte offset of the workgroup's copy of *tail_idle */
    uint4 *tail_states;
    int coop;             /* lanes per work item (1, 2, 4, 8; ScanFast only): small launches split each
                             scan's records over several lanes instead of leaving the GPU mostly idle */
    /* AccState accumulation: u64 counts[FMGI_COLOUR_STATES][num_texels] */
    unsigned long long *counts;
    /* AccStream accumulation: deposit codes (texel << 10 | colour state) appended to stream[0..cap) in
       blocks of FMGI_STREAM_BLOCK codes reserved through stream_cursor (fmgi_accum.hip) */
    uint32_t *stream;
    uint64_t stream_cap;
    unsigned long long *stream_cursor;
    unsigned long long *overflow; /* set if a reservation would pass stream_cap (never, by sizing) */
    /* presorted stream (P <= FMGI_PRESORT_MAX_TILES tiles): each wave writes its rings of
       FMGI_RING_CODES codes sorted by fold tile, with the P + 1 run offsets of every ring-sized segment
       in toff[segment * (P + 1) + t]; the fold then needs no sort pass */
    int presort, ntiles;
    uint16_t *toff;
    /* bucketed stream (presort == 2, P <= FMGI_PRESORT_MAX_TILES): every wave appends each tile's codes
       to its own open FMGI_BUCKET_BLOCK-code block of the pool (`stream`); blocks are taken with one atomic
       on pool_cursor, their tile recorded in block_tile[] and their length in block_len[] when they close */
    uint32_t *block_tile, *block_len;
    unsigned long long *pool_cursor;
    uint64_t pool_blocks;
    const uint4 *colpack; /* {R, G - R, B - R, 0} per colour state (the bucketed stream's atomic fallback) */
    int tile_shift;       /* a code's fold tile is code >> tile_shift (10 + tile bits: 11, or 12 for wide tiles) */
    int ring_off;                 /* byte offset of the per-wave code rings in dynamic LDS (fmgi_bake_lds) */
    int num_texels;
    /* debug trace (TRACE kernels only) */
    void *events;                  /* fmgi_event[(item - item_begin) * 800 + k]                     */
    int32_t *ev_counts;
    uint32_t *rng_final;
};

enum { KSTAT_PHOTONS = 0, KSTAT_SCANS, KSTAT_DEPOSITS, KSTAT_ESCAPES, KSTAT_RESCANS, KSTAT_TESTS, KSTAT_TIES,
       KSTAT_INVALID, KSTAT_N, KSTAT_OVERFLOW = KSTAT_N, KSTAT_STAGE0 = 16, KSTAT_ALLOC = 32 };

/* stream accumulation geometry (fmgi_accum.hip) */
#define FMGI_STREAM_BLOCK 4096 /* codes reserved per wave at a time                         */
#ifndef FMGI_RING_CODES        /* (experiment builds: make fullvariant)                     */
#define FMGI_RING_CODES 1024   /* codes a wave collects in LDS before writing them out       */
#endif
static_assert(FMGI_STREAM_BLOCK % FMGI_RING_CODES == 0, "ring flushes must tile the stream blocks");
#define FMGI_STREAM_SLICE 8192 /* codes per histogram / scatter block                        */
#define FMGI_STREAM_SLICE_BIG 32768 /* ... for lightmaps of more than 128 fold tiles                */
static_assert(FMGI_STREAM_SLICE_BIG % FMGI_STREAM_SLICE == 0, "run tables are sized for the small slices");
#define FMGI_RING_PAD 192 /* the ring's overflow (< 64 codes) lies in the first 64 of these; the bucketed
                             stream sorts a flush into ring[0, RING + 3 * 63) (runs padded to 4 codes)   */
#define FMGI_RING_HIST (FMGI_RING_CODES + FMGI_RING_PAD)      /* tile histogram (64)                     */
#define FMGI_RING_INFO (FMGI_RING_HIST + 64)                  /* bucketed stream's per-tile info (64 x 16 B) */
#define FMGI_RING_STRIDE (FMGI_RING_INFO + 256)               /* per-wave LDS dwords                     */
#ifndef FMGI_SUBHIST  /* bucketed stream (experiment builds): the flush counts and ranks codes in k tile */
#define FMGI_SUBHIST 1 /* histograms, one per lane mod k, after the info table. k = 2 or 4: box200 bake */
#endif                 /* 77.33 / 77.46 ms against 77.32 with the one (profiles/r04/s21)              */
#define FMGI_RING_SUB FMGI_RING_STRIDE                         /* FMGI_SUBHIST x 64 counters            */
#define FMGI_RING_STRIDE_BUCKET (FMGI_RING_STRIDE + (FMGI_SUBHIST > 1 ? FMGI_SUBHIST * 64 : 0))
#define FMGI_PRESORT_MAX_TILES 63 /* presorted stream: a tile histogram of one entry per lane        */
#define FMGI_BUCKET_BLOCK 1024 /* codes per block of the bucketed stream (4 KB; >= a ring, so a ring's run of
                                  one tile spans at most two blocks)                              */
#ifndef FMGI_BUCKET_ALLOC         /* pool blocks a wave reserves at a time (experiment builds)   */
#define FMGI_BUCKET_ALLOC 8
#endif
#ifndef FMGI_TILE_BITS          /* (experiment builds: make fullvariant VFLAGS=-DFMGI_TILE_BITS=12) */
#define FMGI_TILE_BITS 11      /* 2048-texel tiles summed in LDS (64 KB: two sum workgroups per
                                  CU; measured 25 ms per 1e9 photons vs 28 ms with 4096, 31 ms with 1024) */
#endif
#define FMGI_MAX_TILES (1 << (22 - FMGI_TILE_BITS)) /* => at most 4M texels (texel < 2^22 keeps codes != ~0u) */
#define FMGI_WIDE_TILE_BITS 12 /* the bucket layouts' wide tiles (4096 texels): half the tiles, so a wave's
                                  deposit stores touch fewer lines (fmgi_api.cpp tile_bits) */
#ifndef FMGI_FOLD_SPLIT_DEFAULT  /* fold tiles per wide bucket tile (fmgi_fold_split): 1 = one
                                    4096-texel fold (96 KB of accumulators, one workgroup per CU), 2 = two
                                    2048-texel folds reading the same blocks */
#define FMGI_FOLD_SPLIT_DEFAULT 1
#endif

struct StreamBufs {
    uint32_t *stream;           /* deposit codes, cap entries                                   */
    uint64_t cap;
    unsigned long long *cursor; /* reserved codes (device)                                      */
    uint32_t *sorted;           /* per 8192-code slice: its codes sorted by tile, cap entries    */
    uint16_t *toff;             /* per slice: P + 1 run offsets (the last = valid codes)        */
    const uint32_t *colpack;    /* colour table {R, G - R, B - R, 0} per state (fixed point, the
                                   differences two's complement)                                */
    int groups;                 /* slice groups per tile in the sum kernel                      */
    int presort;                /* codes were written presorted per FMGI_RING_CODES segment (toff per
                                   segment); the fold skips k_slice_sort                         */
    int block;                  /* threads per sum workgroup (256, 512 or 1024)                  */
    /* bucketed stream (presort == 2): the pool is `stream` (pool_blocks x FMGI_BUCKET_BLOCK codes) */
    uint32_t *block_tile, *block_len; /* [pool_blocks] per block: its tile, its length              */
    uint32_t *block_list;             /* [pool_blocks] block ids grouped by tile (the fold's list)     */
    uint32_t *tile_blocks;            /* [2 * (FMGI_PRESORT_MAX_TILES + 1)] counts, then list cursors  */
    uint64_t pool_blocks;
    /* dense stream (presort == 3): the bake's codes in iteration order (dense_cap entries, reserved through
       cursor[1]); k_bin moves them into the bucket pool (`stream`, pool cursor = cursor[0]) */
    uint32_t *dense;
    uint64_t dense_cap, dense_alloc;
    int bin_grid;                     /* k_bin workgroups (persistent: two per CU)                     */
    int tile_bits;                    /* bucket tile = 2^tile_bits texels: FMGI_TILE_BITS, or 12-13 (wide
                                         tiles, bucket layouts only; fold tiles per fold_split)         */
};
hipError_t fmgi_stream_fold(const StreamBufs &sb, int num_texels, unsigned long long *lm, hipStream_t s);
int fmgi_fold_split(int tile_bits); /* fold tiles per bucket tile of 2^tile_bits texels */

#define FMGI_COLOUR_STATES 1024 /* bit 9: window (18,18,18) vs light (16,16,18); bits 0-8: 1 + diffuse-bounce floor bits */

/* internal kernel id (not in the C ABI): ScanFast with BakeArgs::coop lanes per work item */
#define FMGI_KERNEL_FAST_COOP 101
/* internal kernel ids of the launch-tail handoff (FMGI_KERNEL_HYBRID): the saving and the resuming launch */
#define FMGI_KERNEL_HYBRID_TAIL 102
#define FMGI_KERNEL_HYBRID_RESUME 103

/* accum: 1 = AccFx3, 2 = AccState, 3 = AccNone (profiling only), 4 = AccStream (unsorted / presorted
   stream layouts), kAccBucket = AccBucket (the stream in the per-tile bucket layout, BakeArgs::presort 2:
   its own kernel instance) */
constexpr int kAccBucket = 5;
constexpr int kAccLines = 6; /* the bucket layout through per-workgroup tile lines (AccLines) */
constexpr int kAccScatter = 7; /* the bucket layout stored lane by lane into per-wave tile blocks (AccScatter) */
#ifndef FMGI_SCATTER_STRIDE
#define FMGI_SCATTER_STRIDE 128 /* AccScatter: LDS dwords per wave (64 x {fill, block} words) */
#endif
constexpr int kAccDense = 8; /* a dense code stream (one code or sentinel per lane and iteration), binned by k_bin */
constexpr int kAccSliced = 9; /* the STREAM's unsorted layout alone (BakeArgs::presort 0, AccStreamT<0>) */
/* `kernel` of the bake launch helpers below: the public FMGI_KERNEL_* id, or FMGI_KERNEL_GRID |
   FMGI_KVAR_AXES for the closed-box instance of the grid scan (BakeArgs::grid_axes set) */
#define FMGI_KVAR_AXES 0x100
#define FMGI_KVAR_PLAN 0x200 /* FMGI_KERNEL_HYBRID | this: the walls over the floor plan (BakeArgs::plan_off) */
#define FMGI_KVAR_STAGED 0x400 /* FMGI_KERNEL_GRID | FMGI_KVAR_AXES | this: walls, emitters and cells all in LDS */
#define FMGI_KVAR_COMPACT 0x800 /* FMGI_KERNEL_GRID | FMGI_KVAR_AXES | this: the compact tables (RectC ...) in LDS */
hipError_t fmgi_launch_bake(const BakeArgs &a, int kernel, int accum, bool trace, int grid_blocks, int block,
                            hipStream_t s);
int fmgi_bake_resident_blocks(int kernel, int accum, bool trace, int block, int lds_bytes);
size_t fmgi_bake_lds(int kernel, int accum, int block, int img_bytes, int *ring_off);
/* the profiler's name of the k_bake instance (kernel, accum, trace) runs (fmgi_last_bake_kernel) */
std::string fmgi_bake_kernel_name(int kernel, int accum, bool trace);
int fmgi_kernels_filter_pk(); /* the kernels' FMGI_FILTER_PK (whether the hybrid scan reads the pair image) */
hipError_t fmgi_launch_reduce_states(unsigned long long *counts, const long long *colfx, unsigned long long *lm,
                                     int n, hipStream_t s);
hipError_t fmgi_launch_add_u64(unsigned long long *dst, const unsigned long long *src, int64_t n, hipStream_t s);
hipError_t fmgi_launch_finalize(const unsigned long long *lm, const float *tin, float *tout, int64_t n,
                                hipStream_t s);
hipError_t fmgi_launch_sincos(const float *x, float *sn, float *cs, int64_t n, int lib, hipStream_t s);
struct fmgi_rect;
hipError_t fmgi_launch_scene_setup(const fmgi_rect *walls, int nw, const fmgi_rect *srcs, int ns, RectDev *rd,
                                   SrcDev *sd, hipStream_t s);
hipError_t fmgi_launch_unit(int op, const float *a, const float *b, int32_t *out, int64_t n, hipStream_t s);

#endif
