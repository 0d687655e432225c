/*
 * fmgi_accum.hip -- "stream" accumulation of the lightmap deposits (FMGI_ACCUM_STREAM).
 *
 * The reference adds every deposit straight into lightColors[] (photonmap.cl:256-258, a data race).
 * Device-scope atomics make that exact but cost one memory-side transaction per deposit, and MI355X
 * executes ~2e10 of those per second (MI355X_MICROARCH.md §Global float atomics): the bake then runs at
 * the atomic rate instead of the tracing rate. This path replaces the atomics with bandwidth:
 *
 *   bake : each deposit appends a 32-bit code (texel << 10 | colour state) to a stream with plain,
 *          wave-coalesced stores (k_bake, AccStream; one reservation atomic per 4096 codes per wave)
 *   sort : per 8192-code slice, a counting sort by 2048-texel tile in LDS, written back contiguously,
 *          plus the slice's tile offsets (u16)                                         k_slice_sort
 *   sum  : one workgroup per (tile, group of slices) reads that tile's run of every slice of its group
 *          and sums it exactly in LDS (int64 R, G - R, B - R per texel, ds_add_u64: a grey deposit
 *          is one add), then adds the tile to the lightmap with one coalesced atomic per channel
 *                                                                                      k_tile_runs
 *
 * HBM traffic per deposit: 4 B written by the bake, 4 B read + 4 B written by the sort, 4 B read by the
 * sum. Every step is exact integer arithmetic, so the lightmap is bit-identical to the atomic paths.
 * Both kernels read the stream length from the device (no host round trip between bake and fold).
 */
#include <hip/hip_runtime.h>
#include <stdlib.h>
#include <stdio.h>

#include <algorithm>

#include "fmgi_internal.h"

namespace {

constexpr int kSlice = FMGI_STREAM_SLICE; /* codes per sort block */
constexpr int kTileTexels = 1 << FMGI_TILE_BITS;
constexpr uint32_t kSentinel = 0xFFFFFFFFu;

__device__ __forceinline__ int tile_of(uint32_t code) { return (int)(code >> (10 + FMGI_TILE_BITS)); }

/* exclusive scan of cnt[0..P) into loc[0..P) by the first 256 threads of a block of NT >= 256 (P <=
   FMGI_MAX_TILES); every thread of the block takes part in its barriers */
template <int NT>
__device__ void block_exclusive_scan(const uint32_t *cnt, uint32_t *loc, int P) {
    __shared__ uint32_t part[256];
    constexpr int per = FMGI_MAX_TILES / 256;
    const bool in = NT == 256 || threadIdx.x < 256;
    const int t0 = threadIdx.x * per;
    uint32_t s = 0;
    if (in) {
        for (int k = 0; k < per; k++) s += (t0 + k < P) ? cnt[t0 + k] : 0u;
        part[threadIdx.x] = s;
    }
    __syncthreads();
    for (int off = 1; off < 256; off <<= 1) { /* Hillis-Steele over the 256 partial sums */
        const uint32_t v = in && threadIdx.x >= (unsigned)off ? part[threadIdx.x - off] : 0u;
        __syncthreads();
        if (in) part[threadIdx.x] += v;
        __syncthreads();
    }
    if (in) {
        uint32_t run = part[threadIdx.x] - s;
        for (int k = 0; k < per; k++) {
            if (t0 + k < P) {
                loc[t0 + k] = run;
                run += cnt[t0 + k];
            }
        }
    }
    __syncthreads();
}

/* one block of NT threads per SL-code slice; the slice is staged in dynamic LDS (SL x 4 B) */
template <int SL, int NT>
__global__ __launch_bounds__(NT) void k_slice_sort(const uint32_t *__restrict__ stream,
                                                  const unsigned long long *__restrict__ n_ptr, uint64_t cap,
                                                  int P, uint32_t *__restrict__ sorted,
                                                  uint16_t *__restrict__ toff) {
    extern __shared__ uint32_t buf[];
    __shared__ uint32_t cnt[FMGI_MAX_TILES], loc[FMGI_MAX_TILES];
    constexpr int per = SL / NT;
    const uint64_t n = *n_ptr < cap ? *n_ptr : cap;
    const uint64_t b0 = (uint64_t)blockIdx.x * SL;
    if (b0 >= n) return; /* uniform: the whole slice is past the end of the stream */
    for (int i = threadIdx.x; i < P; i += blockDim.x) cnt[i] = 0;
    __syncthreads();
    uint32_t c[per];
#pragma unroll
    for (int k = 0; k < per; k++) { /* all loads in flight before the first LDS atomic */
        const uint64_t i = b0 + (uint64_t)k * NT + threadIdx.x;
        c[k] = i < n ? stream[i] : kSentinel;
        /* a code of a tile >= P is never written by the bake; only the unwritten part of a block whose
           reservation failed (stream overflow, reported by the call) can hold one: dropped */
        if (c[k] != kSentinel && tile_of(c[k]) >= P) c[k] = kSentinel;
    }
#pragma unroll
    for (int k = 0; k < per; k++)
        if (c[k] != kSentinel) atomicAdd(&cnt[tile_of(c[k])], 1u);
    __syncthreads();
    block_exclusive_scan<NT>(cnt, loc, P);
    uint16_t *to = toff + (size_t)blockIdx.x * (P + 1);
    for (int i = threadIdx.x; i < P; i += blockDim.x) {
        to[i] = (uint16_t)loc[i];
        cnt[i] = loc[i]; /* running cursor of each tile */
    }
    __syncthreads();
#pragma unroll
    for (int k = 0; k < per; k++)
        if (c[k] != kSentinel) buf[atomicAdd(&cnt[tile_of(c[k])], 1u)] = c[k];
    __syncthreads();
    const int total = (int)cnt[P - 1]; /* end of the last tile's run = valid codes in the slice */
    if (threadIdx.x == 0) to[P] = (uint16_t)total;
    for (int k = threadIdx.x; k < total; k += blockDim.x) sorted[b0 + k] = buf[k];
}

/* k_bucket_fold's CARRY channels: value v (a u32 two's complement int32) added to lo[tx]; hi[tx] (at lo + T)
   takes the carry or borrow of the 64-bit sum */
__device__ __forceinline__ void carry_add(uint32_t *lo, int T, int tx, uint32_t v) {
    const uint32_t old = atomicAdd(&lo[tx], v); /* ds_add_rtn_u32 */
    const uint32_t nw = old + v;
    const int delta = (int)(nw < old) - (int)((int32_t)v < 0);
    if (delta) atomicAdd(&lo[T + tx], (uint32_t)delta);
}
__device__ __forceinline__ unsigned long long carry_val(const uint32_t *lo, int T, int i) {
    return ((unsigned long long)lo[T + i] << 32) | lo[i];
}
/* k_bucket_fold's split colour table (CARRY >= 4): state i's {R | (G != R) << 31, B - R} as 8 B at slot
   colour_slot(i), its G - R as 4 B at the same slot of a second array read only by the lanes whose flag is
   set. The slot XORs the low five bits with the high bits times 3, so the powers of two (a photon's
   untinted states, the most frequent) take distinct bank pairs (CARRY 5: no swizzle) */
template <int CARRY>
__device__ __forceinline__ uint32_t colour_slot(uint32_t i) {
    return CARRY == 4 ? i ^ (((i >> 5) * 3u) & 31u) : i;
}
/* the split colour table in LDS (k_bucket_fold's CARRY 5 and the slice-sorted folds): colour state i's
   {R | (G != R) << 31, B - R} at col2[i], its G - R at colg[i] */
__device__ __forceinline__ void stage_split_colours(const uint4 *colpack, uint2 *col2, uint32_t *colg) {
    for (int i = threadIdx.x; i < FMGI_COLOUR_STATES; i += blockDim.x) {
        const uint4 v = colpack[i];
        col2[i] = make_uint2(v.x | (v.y ? 0x80000000u : 0u), v.z); /* R < 2^30 */
        colg[i] = v.y;
    }
}
/* one code's exact sums into the carry-word channels of a T-texel tile (acc: R, G - R, B - R, each as
   lo[T] | hi[T]): an 8-B colour read, the R add, B - R where nonzero, G - R only for the tinted states */
__device__ __forceinline__ void sum_code_split(unsigned long long *acc, int T, int tx, const uint2 *col2,
                                               const uint32_t *colg, uint32_t c) {
    uint32_t *lo = (uint32_t *)acc;
    const uint2 rb = col2[c & 1023];
    carry_add(lo, T, tx, rb.x & 0x7FFFFFFFu);
    if (rb.y) carry_add(lo + 4 * T, T, tx, rb.y);
    if ((int32_t)rb.x < 0) carry_add(lo + 2 * T, T, tx, colg[c & 1023]);
}

__global__ __launch_bounds__(1024) void k_tile_runs(const uint32_t *__restrict__ sorted,
                                                   const uint16_t *__restrict__ toff,
                                                   const unsigned long long *__restrict__ n_ptr, uint64_t cap,
                                                   int P, int G, const uint4 *__restrict__ colpack,
                                                   unsigned long long *__restrict__ lm, int num_texels) {
    /* per texel of the tile: sum R, sum (G - R), sum (B - R) (modulo 2^64 as carry-word channels; the true
       sums of G and B are non-negative) with the split colour table (sum_code_split), as k_bucket_fold */
    extern __shared__ __attribute__((aligned(16))) unsigned long long s_acc[]; /* 3 x [2048] + colours */
    uint2 *col2 = (uint2 *)(s_acc + 3 * kTileTexels);
    uint32_t *colg = (uint32_t *)(col2 + FMGI_COLOUR_STATES);
    /* XCD-aware order: the dispatcher deals workgroups to the 8 XCDs round-robin (workgroup i -> XCD
       i % 8), so XCD x gets groups g = x, x + 8, ... and, within a group, consecutive tiles back to
       back: the runs of neighbouring tiles share the cache lines at their boundaries, and those reads
       now meet in one L2. G is a multiple of 8 (fmgi_stream_fold). */
    const int xcd = blockIdx.x & 7, j = blockIdx.x >> 3;
    const int t = j % P, g = xcd + 8 * (j / P);
    const uint64_t n = *n_ptr < cap ? *n_ptr : cap;
    const uint64_t ns = (n + kSlice - 1) / kSlice;
    const uint64_t b_lo = ns * g / G, b_hi = ns * (g + 1) / G;
    if (b_lo >= b_hi) return; /* uniform */
    for (int i = threadIdx.x; i < 3 * kTileTexels; i += blockDim.x) s_acc[i] = 0;
    stage_split_colours(colpack, col2, colg);
    __syncthreads();
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63;
    const int waves = blockDim.x >> 6;
    for (uint64_t b = b_lo + wave; b < b_hi; b += waves) {
        const uint16_t *to = toff + b * (P + 1);
        const int r0 = to[t], r1 = to[t + 1]; /* to[P] = the slice's total */
        const uint32_t *run = sorted + b * kSlice;
        for (int k0 = r0; k0 < r1; k0 += 256) { /* up to 4 loads in flight per lane */
            uint32_t v[4];
#pragma unroll
            for (int u = 0; u < 4; u++) {
                const int k = k0 + 64 * u + lane;
                v[u] = k < r1 ? run[k] : kSentinel;
            }
#pragma unroll
            for (int u = 0; u < 4; u++) {
                if (v[u] == kSentinel) continue;
                const int tx = (int)((v[u] >> 10) & (kTileTexels - 1));
                sum_code_split(s_acc, kTileTexels, tx, col2, colg, v[u]);
            }
        }
    }
    __syncthreads();
    for (int i = threadIdx.x; i < kTileTexels; i += blockDim.x) {
        const int texel = t * kTileTexels + i;
        if (texel >= num_texels) break;
        const uint32_t *lo = (const uint32_t *)s_acc;
        const unsigned long long r = carry_val(lo, kTileTexels, i);
        const unsigned long long gg = r + carry_val(lo + 2 * kTileTexels, kTileTexels, i);
        const unsigned long long bb = r + carry_val(lo + 4 * kTileTexels, kTileTexels, i);
        unsigned long long *q = lm + 4 * (size_t)texel;
        if (r) atomicAdd(q + 0, r);
        if (gg) atomicAdd(q + 1, gg);
        if (bb) atomicAdd(q + 2, bb);
    }
}

/* The fold of a presorted stream (BakeArgs::presort): every SEG-code segment already holds its codes
   sorted by tile with the run offsets in toff, so one workgroup per (tile, group of segments) reads its
   tile's run of every segment directly. A wave takes kW segments at a time and packs their runs onto its
   lanes (runs average SEG / P codes: kW = 16 for the bake's 1024-code segments, 4 for 32768-code slices,
   whose runs are 4x longer and whose packed index costs kW - 1 compares per code); the sums are
   k_tile_runs' (R, G - R, B - R as carry-word channels in LDS). */
template <int SEG, int kW>
__global__ __launch_bounds__(1024) void k_tile_runs_pre(const uint32_t *__restrict__ stream,
                                                       const uint16_t *__restrict__ toff,
                                                       const unsigned long long *__restrict__ n_ptr, uint64_t cap,
                                                       int P, int G, const uint4 *__restrict__ colpack,
                                                       unsigned long long *__restrict__ lm, int num_texels) {
    extern __shared__ __attribute__((aligned(16))) unsigned long long s_acc[]; /* 3 x [2048] + colours */
    uint2 *col2 = (uint2 *)(s_acc + 3 * kTileTexels);
    uint32_t *colg = (uint32_t *)(col2 + FMGI_COLOUR_STATES);
    const int xcd = blockIdx.x & 7, j = blockIdx.x >> 3; /* XCD-aware order, as k_tile_runs */
    const int t = j % P, g = xcd + 8 * (j / P);
    const uint64_t n = *n_ptr < cap ? *n_ptr : cap;
    /* presorted: reserved blocks are whole numbers of segments; slice-sorted: the last slice is partial */
    const uint64_t ns = SEG == FMGI_RING_CODES ? n / SEG : (n + SEG - 1) / SEG;
    const uint64_t s_lo = ns * g / G, s_hi = ns * (g + 1) / G;
    if (s_lo >= s_hi) return; /* uniform */
    for (int i = threadIdx.x; i < 3 * kTileTexels; i += blockDim.x) s_acc[i] = 0;
    stage_split_colours(colpack, col2, colg);
    __syncthreads();
    /* a wave takes kW segments at a time and packs their runs for tile t onto its 64 lanes: lane L < kW
       reads segment L's run bounds, a wave prefix sum gives each run's first packed index, and packed
       index i maps back to its code with kW - 1 uniform compares (runs average n / (segments * P) codes,
       far fewer than 64, so one lane per run would leave most lanes idle on the LDS atomics). The next
       group's run bounds are loaded before this group's codes are folded. */
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63;
    const int waves = blockDim.x >> 6;
    auto bounds = [&](uint64_t s0, int &r0, int &len) {
        r0 = 0, len = 0;
        if (lane < kW && s0 + lane < s_hi) {
            const uint16_t *to = toff + (s0 + lane) * (uint64_t)(P + 1);
            /* clamped to the segment: a block whose reservation failed (stream overflow, never by sizing;
               the call then reports the error) has no run table written, and its stale offsets must not
               send a read past the segment */
            r0 = min((int)to[t], SEG);
            len = max(0, min((int)to[t + 1], SEG) - r0);
        }
    };
    int nr0, nlen;
    bounds(s_lo + kW * (uint64_t)wave, nr0, nlen);
    for (uint64_t s0 = s_lo + kW * (uint64_t)wave; s0 < s_hi; s0 += kW * (uint64_t)waves) {
        const int r0 = nr0, len = nlen;
        bounds(s0 + kW * (uint64_t)waves, nr0, nlen);
        int pre = len; /* inclusive prefix over lanes 0..kW-1 */
#pragma unroll
        for (int d = 1; d < kW; d <<= 1) {
            const int o = __shfl_up(pre, d, 64);
            if (lane >= d) pre += o;
        }
        const int total = __builtin_amdgcn_readlane(pre, kW - 1);
        /* packed index i of run j (i in [start_j, start_j + len_j)) reads run_base + j*SEG + r0_j + i - start_j */
        const int shift_l = lane * SEG + r0 - (pre - len);
        int start[kW], shift[kW];
#pragma unroll
        for (int j = 0; j < kW; j++) {
            start[j] = __builtin_amdgcn_readlane(pre - len, j);
            shift[j] = __builtin_amdgcn_readlane(shift_l, j);
        }
        const uint32_t *run = stream + s0 * SEG;
        for (int i0 = lane; i0 < total; i0 += 4 * 64) {
            uint32_t v[4];
#pragma unroll
            for (int u = 0; u < 4; u++) {
                const int i = i0 + 64 * u;
                int sh = shift[0];
#pragma unroll
                for (int j = 1; j < kW; j++) sh = i >= start[j] ? shift[j] : sh;
                v[u] = i < total ? run[i + sh] : kSentinel;
            }
#pragma unroll
            for (int u = 0; u < 4; u++) {
                if (v[u] == kSentinel) continue;
                const int tx = (int)((v[u] >> 10) & (kTileTexels - 1));
                sum_code_split(s_acc, kTileTexels, tx, col2, colg, v[u]);
            }
        }
    }
    __syncthreads();
    for (int i = threadIdx.x; i < kTileTexels; i += blockDim.x) {
        const int texel = t * kTileTexels + i;
        if (texel >= num_texels) break;
        const uint32_t *lo = (const uint32_t *)s_acc;
        const unsigned long long r = carry_val(lo, kTileTexels, i);
        const unsigned long long gg = r + carry_val(lo + 2 * kTileTexels, kTileTexels, i);
        const unsigned long long bb = r + carry_val(lo + 4 * kTileTexels, kTileTexels, i);
        unsigned long long *qq = lm + 4 * (size_t)texel;
        if (r) atomicAdd(qq + 0, r);
        if (gg) atomicAdd(qq + 1, gg);
        if (bb) atomicAdd(qq + 2, bb);
    }
}

/* The fold of a bucketed stream (BakeArgs::presort == 2). k_bucket_count / k_bucket_list group the pool's
   blocks by tile (block_tile[] -> block_list[], each tile's blocks contiguous; one global atomic per tile
   and workgroup), and k_bucket_fold gives each (tile, group of blocks) one workgroup: a wave takes a
   whole 4-KB block (16 codes per lane, four 16-B loads, all in flight before the first add) and sums it
   exactly in LDS as k_tile_runs does. */
constexpr int kListThreads = 1024;

constexpr int kListPerThread = 8;

__global__ __launch_bounds__(kListThreads) void k_bucket_count(const uint32_t *__restrict__ block_tile,
                                                               const unsigned long long *__restrict__ cursor,
                                                               uint64_t pool_blocks, int P,
                                                               uint32_t *__restrict__ counts) {
    __shared__ uint32_t h[64];
    const uint64_t nb = min(*cursor, pool_blocks);
    const uint64_t b0 = (uint64_t)blockIdx.x * kListThreads * kListPerThread;
    if (b0 >= nb) return; /* uniform */
    if (threadIdx.x < 64) h[threadIdx.x] = 0;
    __syncthreads();
    for (int k = 0; k < kListPerThread; k++) {
        const uint64_t b = b0 + (uint64_t)k * kListThreads + threadIdx.x;
        if (b < nb) atomicAdd(&h[block_tile[b]], 1u);
    }
    __syncthreads();
    if ((int)threadIdx.x < P && h[threadIdx.x]) atomicAdd(&counts[threadIdx.x], h[threadIdx.x]);
}

__global__ __launch_bounds__(kListThreads) void k_bucket_list(const uint32_t *__restrict__ block_tile,
                                                              const unsigned long long *__restrict__ cursor,
                                                              uint64_t pool_blocks, int P,
                                                              const uint32_t *__restrict__ counts,
                                                              uint32_t *__restrict__ cursors,
                                                              uint32_t *__restrict__ list) {
    __shared__ uint32_t h[64], base[64];
    const uint64_t nb = min(*cursor, pool_blocks);
    const uint64_t b0 = (uint64_t)blockIdx.x * kListThreads * kListPerThread;
    if (b0 >= nb) return; /* uniform */
    if (threadIdx.x < 64) h[threadIdx.x] = 0;
    __syncthreads();
    uint32_t t[kListPerThread], rk[kListPerThread];
    for (int k = 0; k < kListPerThread; k++) {
        const uint64_t b = b0 + (uint64_t)k * kListThreads + threadIdx.x;
        t[k] = b < nb ? block_tile[b] : 0xFFFFFFFFu;
        rk[k] = t[k] != 0xFFFFFFFFu ? atomicAdd(&h[t[k]], 1u) : 0u;
    }
    __syncthreads();
    if ((int)threadIdx.x < P) { /* this workgroup's range in tile t's part of the list */
        uint32_t off = 0;
        for (int u = 0; u < (int)threadIdx.x; u++) off += counts[u];
        base[threadIdx.x] = h[threadIdx.x] ? off + atomicAdd(&cursors[threadIdx.x], h[threadIdx.x]) : 0u;
    }
    __syncthreads();
    for (int k = 0; k < kListPerThread; k++)
        if (t[k] != 0xFFFFFFFFu) list[base[t[k]] + rk[k]] = (uint32_t)(b0 + (uint64_t)k * kListThreads + threadIdx.x);
}

/* EXP (experiments, FMGI_EXP_FOLD; PROFILING, results wrong): 1 = the codes read and discarded (the
   read alone), 2 = one LDS add per code and no colour lookup, 3 = the colour lookup and the R add only,
   4 = the three adds of a colour computed from the code (no lookup). box200, 1e9 photons (profiles/r04/
   s13-s17): the fold 10.9 ms; 1 = 5.8 ms, 2 = 6.3 ms: the adds, not the reads, bind it. Issuing a quad's
   four colour reads before its adds (12.2 ms) or adding the tinted differences unconditionally (13.8 ms)
   was slower. */
/* 8 waves per SIMD (<= 64 VGPRs): two 1024-lane workgroups per CU, as their 64 KB of LDS allow (at 66
   VGPRs only one fitted, and the fold took 13.7 ms instead of 11) */
/* SPLIT > 1: the buckets' tiles are SPLIT fold tiles wide (bucket tile bits = TB + log2 SPLIT); each
   (tile, group of blocks) gets SPLIT workgroups, one per fold tile, that read the same blocks and sum only
   their own texels' codes. The SPLIT workgroups of one block range are dispatched 8 apart, i.e. on one XCD
   at about the same time, so the blocks' second and later reads are meant to hit its L2 (or the Infinity
   Cache) rather than HBM. The bake's per-lane bucket stores touch fewer lines per store the wider its
   tiles (§4.1), while the fold keeps 64-KB workgroups, two per CU. */
/* CARRY: channels summed as a u32 low word with a returning ds_add_rtn_u32 plus a u32 carry
   word that takes +-1 only when the low word wraps (old + v < old for v >= 0; a negative difference borrows
   when old + v >= old): 0 = every channel as one ds_add_u64, 1 = G - R and B - R with carries (their adds
   wrap ~1/64 of the time), 2 = R as well (the default: fewer bank dwords per add, -2 % on box200's fold). The sum mod 2^64 is the same either way: a channel is
   hi * 2^32 + lo, and only hi mod 2^32 matters mod 2^64. The carry channels reuse the u64 array's 8 B per texel
   as lo[T] | hi[T]. 4 and 5 = 2 with the split colour table (colour_slot): the fold's LDS work is counted in
   dwords, and the 16-B colour read was two thirds of a box200 code's; 5 (the default since profiles/r06/s31)
   reads 8 B per code plus 4 B for the tinted ones: box200 11.30 -> 9.89 ms, example 0.87 -> 0.74 ms, bit-identical;
   4's swizzled slots measured 10.07 ms. */
/* NB: blocks a wave has in flight, as whole-block register buffers (2: the block being summed and the next;
   more need the registers of fewer waves: NB > 2 instances are launched where the tile's LDS already holds
   a CU to one 1024-lane workgroup, i.e. 4 waves per SIMD and 128 VGPRs) */
template <int EXP, int TB = FMGI_TILE_BITS, int SPLIT = 1, int CARRY = 0, int NB = 2>
__global__ __launch_bounds__(1024, NB > 2 ? 1 : 8) void k_bucket_fold(const uint32_t *__restrict__ pool,
                                                     const uint32_t *__restrict__ list,
                                                     const uint32_t *__restrict__ block_len,
                                                     const uint32_t *__restrict__ counts, int P, int G,
                                                     int balanced, const uint4 *__restrict__ colpack,
                                                     unsigned long long *__restrict__ lm, int num_texels) {
    constexpr uint32_t BP = FMGI_BUCKET_BLOCK;
    constexpr int kTileTexels = 1 << TB; /* this instance's fold tile */
    constexpr int kSplitBits = SPLIT == 4 ? 2 : (SPLIT == 2 ? 1 : 0);
    static_assert(SPLIT == 1 << kSplitBits, "SPLIT must be 1, 2 or 4");
    constexpr uint32_t kBucketMask = (1u << (TB + kSplitBits)) - 1; /* texel bits of a bucket tile */
    const uint32_t n = blockIdx.x;
    const uint32_t part = SPLIT > 1 ? (n >> 3) & (SPLIT - 1) : 0u;                   /* fold tile in the bucket */
    const uint32_t wid = SPLIT > 1 ? ((n >> (3 + kSplitBits)) << 3) | (n & 7) : n; /* the block-range workgroup */
    extern __shared__ __attribute__((aligned(16))) unsigned long long s_acc[]; /* 3 x [2048] + colours */
    unsigned long long *acc_r = s_acc, *acc_g = s_acc + kTileTexels, *acc_b = s_acc + 2 * kTileTexels;
    uint4 *col = (uint4 *)(s_acc + 3 * kTileTexels);
    uint32_t t = 0, off = 0, nt = 0, j_lo = 0, j_hi = 0;
    if (balanced) {
        /* the P * G workgroups shared out in proportion to the tiles' block counts (at least one each):
           tile t owns workgroups [c(t), c(t + 1)) with c(t) = t + floor((W - P) * blocks before t / all),
           so every workgroup folds about the same number of blocks whatever the tiles' sizes */
        const uint32_t W = (uint32_t)(P * G), w = wid;
        uint64_t total = 0;
        for (int u = 0; u < P; u++) total += counts[u];
        if (total == 0) return;
        uint64_t cum = 0;
        uint32_t c0 = 0, c1 = 0;
        for (int u = 0; u < P; u++) {
            c0 = (uint32_t)u + (uint32_t)((uint64_t)(W - P) * cum / total);
            c1 = (uint32_t)u + 1 + (uint32_t)((uint64_t)(W - P) * (cum + counts[u]) / total);
            if (w < c1 || u == P - 1) {
                t = (uint32_t)u;
                break;
            }
            cum += counts[u];
        }
        off = (uint32_t)cum;
        nt = counts[t];
        const uint32_t wt = c1 - c0, g = w - c0;
        if (w >= c1) return; /* uniform */
        j_lo = (uint32_t)((uint64_t)nt * g / wt);
        j_hi = (uint32_t)((uint64_t)nt * (g + 1) / wt);
    } else {
        const int xcd = (int)(wid & 7), j = (int)(wid >> 3); /* XCD-aware order, as k_tile_runs */
        t = (uint32_t)(j % P);
        const uint32_t g = (uint32_t)(xcd + 8 * (j / P));
        for (uint32_t u = 0; u < t; u++) off += counts[u];
        nt = counts[t];
        j_lo = (uint32_t)((uint64_t)nt * g / G);
        j_hi = (uint32_t)((uint64_t)nt * (g + 1) / G);
    }
    if (j_lo >= j_hi) return; /* uniform */
    for (int i = threadIdx.x; i < 3 * kTileTexels; i += blockDim.x) s_acc[i] = 0;
    uint2 *col2 = (uint2 *)col;                         /* CARRY >= 4: {R | G-flag, B - R} per slot */
    uint32_t *colg = (uint32_t *)(col2 + FMGI_COLOUR_STATES); /* CARRY >= 4: G - R per slot */
    for (int i = threadIdx.x; i < FMGI_COLOUR_STATES; i += blockDim.x) {
        const uint4 v = colpack[i];
        if (CARRY == 6) {
            col2[i] = make_uint2(v.y, v.z); /* {G - R, B - R}: read by the tinted codes only */
        } else if (CARRY >= 4) {
            const uint32_t p = colour_slot<CARRY>((uint32_t)i);
            col2[p] = make_uint2(v.x | (v.y ? 0x80000000u : 0u), v.z); /* R < 2^30 */
            colg[p] = v.y;
        } else {
            col[i] = v;
        }
    }
    __syncthreads();
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63;
    const int waves = blockDim.x >> 6;
    /* the wave's blocks are j_lo + wave + k * waves: lane k holds block k's pool index and length (one
       load each for up to 64 blocks at a time), so the loop reads them with readlane instead of two
       dependent loads per block, and the next block's four 16-B loads are in flight while this block's
       codes are summed */
    const uint32_t span = j_hi - j_lo;
    const uint32_t nb = span > (uint32_t)wave ? (span - (uint32_t)wave + waves - 1) / waves : 0u;
    typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
    for (uint32_t k0 = 0; k0 < nb; k0 += 64) {
        const uint32_t kn = min(nb - k0, 64u);
        uint32_t lb = 0, ll = 0;
        if ((uint32_t)lane < kn) {
            lb = list[off + j_lo + wave + (k0 + lane) * waves];
            ll = min(block_len[lb], BP);
        }
        u32x4 q[NB][4];
        uint32_t len[NB];
        /* the whole 4-KB block, unconditionally (codes past the block's length are skipped when summed):
           four 16-B loads per lane with no branch around them, so the wait before a block's sums leaves
           the next blocks' loads in flight (loads under a lane condition compiled to 16 dword loads each,
           and the wait at the branch's join waited for the prefetch too) */
        auto fetch = [&](uint32_t k, u32x4 (&qq)[4], uint32_t &ln) {
            const uint32_t b = (uint32_t)__builtin_amdgcn_readlane((int)lb, (int)k);
            ln = (uint32_t)__builtin_amdgcn_readlane((int)ll, (int)k);
            const __attribute__((address_space(1))) u32x4 *blk =
                (const __attribute__((address_space(1))) u32x4 *)(pool + (uint64_t)b * BP);
#pragma unroll
            for (int u = 0; u < 4; u++) qq[u] = blk[64 * u + lane]; /* codes 4 i4 .. 4 i4 + 3, i4 = 64 u + lane */
        };
        auto sum = [&](const u32x4 (&qq)[4], uint32_t ln) {
#pragma unroll
            for (int u = 0; u < 4; u++) {
                const uint32_t i0 = 4 * (64 * u + lane);
                const uint32_t cs[4] = {qq[u].x, qq[u].y, qq[u].z, qq[u].w};
#pragma unroll
                for (int m = 0; m < 4; m++) {
                    const uint32_t c = cs[m];
                    if (i0 + m >= ln || c == kSentinel) continue; /* runs are padded to 4 codes */
                    if (SPLIT > 1 && (((c >> 10) & kBucketMask) >> TB) != part) continue; /* another fold tile's */
                    const int tx = (int)((c >> 10) & (kTileTexels - 1));
                    if (EXP == 1) {
                        if (c == 0x7FFFFFFFu) acc_r[tx] = 1; /* never: keeps the loads */
                        continue;
                    }
                    if (EXP == 2) {
                        atomicAdd(&acc_r[tx], 1ull);
                        continue;
                    }
                    if (CARRY == 6) {
                        /* R from the state's bounce count (a tint scales G and B only): the float replay of
                           colour_table()'s x channel; an untinted state's B - R the same way; an 8-B {G - R,
                           B - R} read only for the tinted states */
                        const uint32_t st = c & 511;
                        if (st == 0) continue; /* colour 0 */
                        const int nbn = 31 - __clz((int)st);
                        float x = (c & 512) ? 18.0f : 16.0f, z = 18.0f;
#pragma unroll
                        for (int k = 0; k < 8; k++) {
                            const bool m = k < nbn;
                            x = m ? x * 0.9f : x;
                            z = m ? z * 0.9f : z;
                        }
                        const uint32_t R = (uint32_t)(x * 33554432.0f); /* 2^FMGI_FX_SHIFT */
                        carry_add((uint32_t *)acc_r, kTileTexels, tx, R);
                        if (st == (1u << nbn)) {
                            const uint32_t d = (uint32_t)(z * 33554432.0f) - R;
                            if (d) carry_add((uint32_t *)acc_b, kTileTexels, tx, d);
                        } else {
                            const uint2 gb = col2[c & 1023];
                            if (gb.y) carry_add((uint32_t *)acc_b, kTileTexels, tx, gb.y);
                            if (gb.x) carry_add((uint32_t *)acc_g, kTileTexels, tx, gb.x);
                        }
                        continue;
                    }
                    if (CARRY >= 4) { /* an 8-B colour read per code, the 4-B G - R only where G != R */
                        const uint32_t p = colour_slot<CARRY>(c & 1023);
                        const uint2 rb = col2[p];
                        carry_add((uint32_t *)acc_r, kTileTexels, tx, rb.x & 0x7FFFFFFFu);
                        if (rb.y) carry_add((uint32_t *)acc_b, kTileTexels, tx, rb.y);
                        if ((int32_t)rb.x < 0) carry_add((uint32_t *)acc_g, kTileTexels, tx, colg[p]);
                        continue;
                    }
                    const uint4 cc = EXP == 4 ? make_uint4(c & 1023, (c & 3) ? c & 511 : 0u, (c & 3) ? c & 255 : 0u, 0u)
                                              : col[c & 1023];
                    if (CARRY == 3) {
                        /* R and B - R in one 64-bit word per texel, {B - R : R}: one returning ds_add_rtn_u64 per
                           code; R's wraps (the hardware carries them into the high half) are counted in cR and
                           the high half's own wraps in cD, both from the returned old value */
                        uint32_t *cR = (uint32_t *)acc_g, *cD = cR + kTileTexels;
                        const uint32_t R = cc.x, D = cc.z;
                        const unsigned long long old = atomicAdd(&acc_r[tx], ((unsigned long long)D << 32) | R);
                        const uint32_t lo = (uint32_t)old, cin = (uint32_t)(lo + R < lo);
                        const unsigned long long hs = (old >> 32) + (unsigned long long)D + cin;
                        const int dD = (int)(hs >> 32) - (int)((int32_t)D < 0);
                        if (cin) atomicAdd(&cR[tx], 1u);
                        if (dD) atomicAdd(&cD[tx], (uint32_t)dD);
                        if (cc.y) carry_add((uint32_t *)acc_b, kTileTexels, tx, cc.y);
                        continue;
                    }
                    if (CARRY >= 2) carry_add((uint32_t *)acc_r, kTileTexels, tx, cc.x);
                    else atomicAdd(&acc_r[tx], (unsigned long long)cc.x);
                    if (EXP == 3) continue;
                    if (CARRY >= 1) {
                        if (cc.y) carry_add((uint32_t *)acc_g, kTileTexels, tx, cc.y);
                        if (cc.z) carry_add((uint32_t *)acc_b, kTileTexels, tx, cc.z);
                        continue;
                    }
                    if (cc.y) atomicAdd(&acc_g[tx], (unsigned long long)(long long)(int32_t)cc.y);
                    if (cc.z) atomicAdd(&acc_b[tx], (unsigned long long)(long long)(int32_t)cc.z);
                }
            }
        };
        /* a ring of NB blocks: block k is summed from buffer k % NB once block k + NB - 1's loads are issued
           into the buffer block k - 1 left (the unrolled steps keep every buffer index static) */
#pragma unroll
        for (int s0 = 0; s0 < NB - 1; s0++) fetch(s0 < (int)kn ? (uint32_t)s0 : kn - 1, q[s0], len[s0]);
        for (uint32_t kb = 0; kb < kn; kb += NB) {
#pragma unroll
            for (int s0 = 0; s0 < NB; s0++) {
                const uint32_t k = kb + (uint32_t)s0;
                if (k >= kn) break; /* uniform */
                const uint32_t kf = k + NB - 1 < kn ? k + NB - 1 : kn - 1; /* (past the end: re-reads, unused) */
                fetch(kf, q[(s0 + NB - 1) % NB], len[(s0 + NB - 1) % NB]);
                sum(q[s0], len[s0]);
            }
        }
    }
    __syncthreads();
    for (int i = threadIdx.x; i < kTileTexels; i += blockDim.x) {
        const int texel = (int)((t << (TB + kSplitBits)) + part * kTileTexels) + i;
        if (texel >= num_texels) break;
        unsigned long long r = CARRY >= 2 ? carry_val((const uint32_t *)acc_r, kTileTexels, i) : acc_r[i];
        unsigned long long ag = CARRY >= 1 ? carry_val((const uint32_t *)acc_g, kTileTexels, i) : acc_g[i];
        unsigned long long ab = CARRY >= 1 ? carry_val((const uint32_t *)acc_b, kTileTexels, i) : acc_b[i];
        if (CARRY == 3) { /* R = cR * 2^32 + the low half; B - R = {cD : high half} - cR; G - R from acc_b */
            const uint32_t *cR = (const uint32_t *)acc_g, *cD = cR + kTileTexels;
            const unsigned long long w = acc_r[i];
            r = ((unsigned long long)cR[i] << 32) | (uint32_t)w;
            ab = ((((unsigned long long)cD[i] << 32) | (w >> 32)) - cR[i]);
            ag = carry_val((const uint32_t *)acc_b, kTileTexels, i);
        }
        const unsigned long long gg = r + ag, bb = r + ab;
        unsigned long long *qq = lm + 4 * (size_t)texel;
        if (r) atomicAdd(qq + 0, r);
        if (gg) atomicAdd(qq + 1, gg);
        if (bb) atomicAdd(qq + 2, bb);
    }
}

#if FMGI_EXPERIMENTS
/* The binning pass of the dense stream (kAccDense, BakeArgs::presort == 3): the bake wrote one code or
   sentinel per lane and iteration, in no order; k_bin groups them into the bucket layout k_bucket_fold reads
   (pool blocks of FMGI_BUCKET_BLOCK codes, each holding one fold tile's codes, its tile and length recorded).
   Persistent workgroups of 1024 lanes take 8192-code batches in turn. Per batch: each wave counts its 512
   codes per tile in its own LDS histogram; a scan over (tile, wave) gives every wave's range in the batch
   sorted by tile; the codes are scattered into that order in LDS (32 KB); one lane per tile appends the
   tile's run to the workgroup's open block of that tile, taking new blocks (one pool-cursor atomic per tile
   and batch when the run overflows); then all lanes copy the sorted batch out, consecutive lanes to
   consecutive codes of one run. Runs average 8192 / P codes (~178 on box200), so the stores are whole
   lines. HBM traffic per code: 4 B read, 4 B written. A pool too small (never, by sizing) sends the codes
   through exact int64 atomics into the lightmap, as the bake's bucket fallback. */
constexpr int kBinThreads = 1024, kBinPer = 8, kBinBatch = kBinThreads * kBinPer;
constexpr uint32_t kNoBlk = 0xFFFFFFFFu;

__device__ __forceinline__ void bin_atomic(const uint4 *colpack, unsigned long long *lm, uint32_t code) {
    const uint4 cc = colpack[code & 1023];
    unsigned long long *q = lm + 4 * (size_t)(code >> 10);
    const unsigned long long r = cc.x;
    atomicAdd(q + 0, r);
    atomicAdd(q + 1, r + (unsigned long long)(long long)(int32_t)cc.y);
    atomicAdd(q + 2, r + (unsigned long long)(long long)(int32_t)cc.z);
}

__global__ __launch_bounds__(kBinThreads, 8) void k_bin(const uint32_t *__restrict__ dense,
                                                     const unsigned long long *__restrict__ n_ptr, uint64_t cap,
                                                     int P, uint32_t *__restrict__ pool,
                                                     uint32_t *__restrict__ block_tile, uint32_t *__restrict__ block_len,
                                                     unsigned long long *__restrict__ pool_cursor, uint64_t pool_blocks,
                                                     const uint4 *__restrict__ colpack, unsigned long long *__restrict__ lm,
                                                     uint32_t shift) {
    constexpr uint32_t BP = FMGI_BUCKET_BLOCK;
    extern __shared__ __attribute__((aligned(16))) uint32_t stage[]; /* kBinBatch codes */
    __shared__ uint32_t hist[16][64];
    __shared__ uint32_t ttot[64], tstart[64];
    __shared__ uint2 info[64];  /* per tile: the workgroup's open block {block, fill} */
    __shared__ uint4 tab[64];   /* per tile, this batch: {run start, codes into the open block, the open block, first new block} */
    __shared__ uint32_t tfill[64]; /* ... and the open block's fill before the batch */
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63;
    const uint64_t n = *n_ptr < cap ? *n_ptr : cap;
    const uint64_t nbatch = (n + kBinBatch - 1) / kBinBatch;
    if (threadIdx.x < 64) info[threadIdx.x] = make_uint2(kNoBlk, BP);
    typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
    for (uint64_t b = blockIdx.x; b < nbatch; b += gridDim.x) {
        /* the wave's kBinPer * 64 codes (n is a multiple of FMGI_STREAM_BLOCK: a wave's part is all in or out) */
        const uint64_t w0 = b * kBinBatch + (uint64_t)wave * (kBinPer * 64);
        uint32_t c[kBinPer];
        if (w0 < n) {
            const __attribute__((address_space(1))) u32x4 *src = (const __attribute__((address_space(1))) u32x4 *)(dense + w0);
#pragma unroll
            for (int u = 0; u < kBinPer / 4; u++) {
                const u32x4 q = src[64 * u + lane];
                c[4 * u] = q.x, c[4 * u + 1] = q.y, c[4 * u + 2] = q.z, c[4 * u + 3] = q.w;
            }
        } else {
#pragma unroll
            for (int e = 0; e < kBinPer; e++) c[e] = kSentinel;
        }
#pragma unroll
        for (int e = 0; e < kBinPer; e++) /* a tile past P is never written by the bake: treated as a sentinel */
            if (c[e] != kSentinel && (c[e] >> shift) >= (uint32_t)P) c[e] = kSentinel;
        hist[wave][lane] = 0;
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
#pragma unroll
        for (int e = 0; e < kBinPer; e++)
            if (c[e] != kSentinel) atomicAdd(&hist[wave][c[e] >> shift], 1u);
        __syncthreads();
        /* lane group (tile t = tid / 16, wave w = tid % 16): exclusive prefix over the waves of tile t */
        const int st = threadIdx.x >> 4, sw = threadIdx.x & 15;
        const uint32_t v = hist[sw][st];
        uint32_t incl = v;
#pragma unroll
        for (int off = 1; off < 16; off <<= 1) {
            const uint32_t o = __shfl_up(incl, off, 16);
            if (sw >= off) incl += o;
        }
        if (sw == 15) ttot[st] = incl;
        __syncthreads();
        if (wave == 0) { /* tiles' run starts: an exclusive scan of the 64 tile totals */
            const uint32_t x = lane < P ? ttot[lane] : 0u;
            uint32_t in2 = x;
#pragma unroll
            for (int off = 1; off < 64; off <<= 1) {
                const uint32_t o = __shfl_up(in2, off, 64);
                if (lane >= off) in2 += o;
            }
            tstart[lane] = in2 - x;
        }
        __syncthreads();
        hist[sw][st] = tstart[st] + incl - v; /* the wave's cursor in tile st's run */
        __syncthreads();
#pragma unroll
        for (int e = 0; e < kBinPer; e += 4) {
            uint32_t o[4];
#pragma unroll
            for (int k = 0; k < 4; k++) o[k] = c[e + k] != kSentinel ? atomicAdd(&hist[wave][c[e + k] >> shift], 1u) : 0u;
#pragma unroll
            for (int k = 0; k < 4; k++)
                if (c[e + k] != kSentinel) stage[o[k]] = c[e + k];
        }
        __syncthreads();
        if (wave == 0) { /* (after the scatter: no code is held in registers) */
            const uint32_t x = lane < P ? ttot[lane] : 0u;
            if (lane < P && x) { /* the tile's run into its open block, then whole new blocks */
                const uint2 inf = info[lane];
                const uint32_t room = inf.x == kNoBlk ? 0u : BP - inf.y;
                const uint32_t first = x < room ? x : room, rest = x - first;
                const uint32_t nnew = (rest + BP - 1) / BP;
                uint32_t b0 = kNoBlk;
                if (nnew) {
                    const unsigned long long nb = atomicAdd(pool_cursor, (unsigned long long)nnew);
                    if (nb + nnew <= pool_blocks) {
                        b0 = (uint32_t)nb;
                        for (uint32_t j = 0; j < nnew; j++) {
                            block_tile[b0 + j] = (uint32_t)lane;
                            block_len[b0 + j] = BP; /* every block but the tile's last is full; the last is set
                                                      when the workgroup closes it */
                        }
                    } else { /* (never, by sizing) blocks past the pool: recorded empty, codes sent to atomics */
                        for (uint64_t j = nb; j < pool_blocks && j < nb + nnew; j++) {
                            block_tile[j] = 0u;
                            block_len[j] = 0u;
                        }
                    }
                }
                tab[lane] = make_uint4(tstart[lane], first, inf.x, b0);
                tfill[lane] = inf.y;
                if (nnew) info[lane] = b0 == kNoBlk ? make_uint2(kNoBlk, 0u) : make_uint2(b0 + nnew - 1, rest - (nnew - 1) * BP);
                else info[lane] = make_uint2(inf.x, inf.y + x);
            }
        }
        __syncthreads();
        const uint32_t total = tstart[63]; /* (P <= 63: tile 63 is empty) */
        for (uint32_t i = threadIdx.x; i < total; i += kBinThreads) {
            const uint32_t code = stage[i];
            const uint4 tb = tab[code >> shift];
            const uint32_t k = i - tb.x;
            if (k < tb.y) {
                pool[(uint64_t)tb.z * BP + tfill[code >> shift] + k] = code;
            } else if (tb.w != kNoBlk) {
                const uint32_t r = k - tb.y;
                pool[(uint64_t)(tb.w + r / BP) * BP + (r % BP)] = code;
            } else {
                bin_atomic(colpack, lm, code);
            }
        }
        __syncthreads();
    }
    /* the workgroup's open blocks: their lengths (a full one was recorded when it was taken) */
    if (threadIdx.x < 64 && (int)threadIdx.x < P) {
        const uint2 inf = info[threadIdx.x];
        if (inf.x != kNoBlk) block_len[inf.x] = inf.y;
    }
}

#endif // FMGI_EXPERIMENTS

} // namespace

/* fold tiles per bucket tile for a bucket layout of 2^tb-texel tiles: FMGI_FOLD_SPLIT (1, 2 or 4) if set and
   an instance exists, else 1 */
int fmgi_fold_split(int tb) {
    if (!FMGI_EXPERIMENTS) return 1;
    const char *e = fmgi_exp_env("FMGI_FOLD_SPLIT");
    const int env = e ? atoi(e) : 0;
    const int want = env > 0 ? env : FMGI_FOLD_SPLIT_DEFAULT;
    int got = 1;
    if (tb == 12 && (want == 1 || want == 2)) got = want;
    else if (tb == 13) got = want == 4 ? 4 : 2; /* 8192-texel fold tiles do not fit LDS */
    if (env > 0 && got != env) { /* an A/B would otherwise measure another split than the one it names */
        static bool said = false;
        if (!said) fprintf(stderr, "fmgi: FMGI_FOLD_SPLIT=%d has no fold instance for %d-texel buckets: split %d\n",
                           env, 1 << tb, got);
        said = true;
    }
    return got;
}

hipError_t fmgi_stream_fold(const StreamBufs &sb, int num_texels, unsigned long long *lm, hipStream_t s) {
    /* the bucket layouts' tiles may be wide (sb.tile_bits); the others are FMGI_TILE_BITS */
    const int tb = sb.presort >= 2 && sb.tile_bits > 0 ? sb.tile_bits : FMGI_TILE_BITS;
    const int P = (num_texels + (1 << tb) - 1) >> tb;
    /* the bucket layouts' fold tiles: a bucket tile split in `split` fold tiles (fmgi_fold_split) */
    const int split = sb.presort >= 2 ? fmgi_fold_split(tb) : 1;
    const int fb = tb - (split == 4 ? 2 : split == 2 ? 1 : 0);
    const size_t plds = (size_t)3 * ((size_t)1 << fb) * 8 + (size_t)FMGI_COLOUR_STATES * 16;
#if FMGI_EXPERIMENTS
    if (sb.presort == 3) { /* the dense stream: binned into the pool, then folded as the bucket layout */
        hipError_t e = fmgi_set_lds_attr_once<6>((const void *)k_bin, kBinBatch * 4);
        if (e != hipSuccess) return e;
        hipLaunchKernelGGL(k_bin, dim3((unsigned)std::max(1, sb.bin_grid)), dim3(kBinThreads), (size_t)kBinBatch * 4, s,
                           sb.dense, sb.cursor + 1, sb.dense_cap, P, sb.stream, sb.block_tile, sb.block_len, sb.cursor,
                           sb.pool_blocks, (const uint4 *)sb.colpack, lm, (uint32_t)(10 + tb));
        e = hipGetLastError();
        if (e != hipSuccess) return e;
    }
#else
    if (sb.presort == 3 || sb.presort == 1) return hipErrorInvalidValue; /* (experiment builds' layouts) */
#endif
    if (sb.presort >= 2) {
        /* the blocks listed by tile (counts, then each workgroup's range in its tiles' parts), then the sums */
        const unsigned lg = (unsigned)((sb.pool_blocks + (uint64_t)kListThreads * kListPerThread - 1) /
                                       ((uint64_t)kListThreads * kListPerThread));
        hipError_t e = hipMemsetAsync(sb.tile_blocks, 0, 2 * (FMGI_PRESORT_MAX_TILES + 1) * sizeof(uint32_t), s);
        if (e != hipSuccess) return e;
        hipLaunchKernelGGL(k_bucket_count, dim3(lg), dim3(kListThreads), 0, s, sb.block_tile, sb.cursor, sb.pool_blocks,
                           P, sb.tile_blocks);
        hipLaunchKernelGGL(k_bucket_list, dim3(lg), dim3(kListThreads), 0, s, sb.block_tile, sb.cursor, sb.pool_blocks, P,
                           sb.tile_blocks, sb.tile_blocks + FMGI_PRESORT_MAX_TILES + 1, sb.block_list);
        typedef void (*FoldFn)(const uint32_t *, const uint32_t *, const uint32_t *, const uint32_t *, int, int, int,
                               const uint4 *, unsigned long long *, int);
        /* the channels summed as u32 low words with carry words (CARRY >= 2): box200's wide fold 11.76 -> 11.54 ms,
           bit-identical (profiles/r06/s5 ab_carry.log); with the split colour table (CARRY = 5: an 8-B colour read
           per code, G - R only for the tinted states) 11.30 -> 9.89 ms (profiles/r06/s31); the experiment build's
           FMGI_FOLD_CARRY=0 keeps the int64 adds, =2 the 16-B colour reads */
        FoldFn fn = nullptr;
        if (split == 1 && tb == FMGI_TILE_BITS) fn = k_bucket_fold<0, FMGI_TILE_BITS, 1, 5>;
        else if (split == 1 && tb == 12) fn = k_bucket_fold<0, 12, 1, 5>;
#if FMGI_EXPERIMENTS
        {   /* FMGI_EXP_FOLD (profiling variants), FMGI_FOLD_SPLIT (split folds), FMGI_FOLD_CARRY (carry words) */
            const char *xe = fmgi_exp_env("FMGI_EXP_FOLD"), *ce = fmgi_exp_env("FMGI_FOLD_CARRY");
            const int exp = xe ? atoi(xe) : 0, carry = ce ? atoi(ce) : 0;
            static const FoldFn folds[] = {k_bucket_fold<0>, k_bucket_fold<1>, k_bucket_fold<2>, k_bucket_fold<3>,
                                           k_bucket_fold<4>};
            if (split == 1 && tb == FMGI_TILE_BITS && exp >= 1 && exp <= 4) fn = folds[exp];
            if (tb == 12 && split == 2) fn = k_bucket_fold<0, 11, 2>;
            if (tb == 13 && split == 2) fn = k_bucket_fold<0, 12, 2>;
            if (tb == 13 && split == 4) fn = k_bucket_fold<0, 11, 4>;
            const bool plain = split == 1 && (tb == 12 || exp == 0);
            if (plain && ce && carry == 0) fn = tb == 12 ? (FoldFn)k_bucket_fold<0, 12, 1> : (FoldFn)k_bucket_fold<0>;
            if (plain && carry == 1) fn = tb == 12 ? (FoldFn)k_bucket_fold<0, 12, 1, 1> : (FoldFn)k_bucket_fold<0, FMGI_TILE_BITS, 1, 1>;
            if (plain && carry == 2) fn = tb == 12 ? (FoldFn)k_bucket_fold<0, 12, 1, 2> : (FoldFn)k_bucket_fold<0, FMGI_TILE_BITS, 1, 2>;
            if (plain && carry == 3) fn = tb == 12 ? (FoldFn)k_bucket_fold<0, 12, 1, 3> : (FoldFn)k_bucket_fold<0, FMGI_TILE_BITS, 1, 3>;
            if (plain && carry == 4) fn = tb == 12 ? (FoldFn)k_bucket_fold<0, 12, 1, 4> : (FoldFn)k_bucket_fold<0, FMGI_TILE_BITS, 1, 4>;
            if (plain && carry == 6) fn = tb == 12 ? (FoldFn)k_bucket_fold<0, 12, 1, 6> : (FoldFn)k_bucket_fold<0, FMGI_TILE_BITS, 1, 6>;
            if (plain && carry == 5) fn = tb == 12 ? (FoldFn)k_bucket_fold<0, 12, 1, 5> : (FoldFn)k_bucket_fold<0, FMGI_TILE_BITS, 1, 5>;
            if (const char *nbe = fmgi_exp_env("FMGI_FOLD_NB")) { /* blocks in flight per wave, wide tiles */
                const int nbv = atoi(nbe);
                if (split == 1 && tb == 12 && nbv == 3) fn = k_bucket_fold<0, 12, 1, 2, 3>;
                if (split == 1 && tb == 12 && nbv == 4) fn = k_bucket_fold<0, 12, 1, 2, 4>;
            }
        }
#endif
        if (!fn) return hipErrorInvalidValue; /* no instance for this tile width and split */
        e = fmgi_set_lds_attr_fn((const void *)fn, (int)plds);
        if (e != hipSuccess) return e;
        const int G = (sb.groups + 7) & ~7;
        const char *be = fmgi_exp_env("FMGI_FOLD_BALANCE"); /* experiments: 0 = equal groups per tile */
        const int balanced = be ? atoi(be) != 0 : 1;
        const dim3 grid((unsigned)(P * G * split)), blk(sb.block > 0 ? sb.block : 1024);
        hipLaunchKernelGGL(fn, grid, blk, plds, s, sb.stream, sb.block_list, sb.block_len, sb.tile_blocks, P, G,
                           balanced, (const uint4 *)sb.colpack, lm, num_texels);
        return hipGetLastError();
    }
#if FMGI_EXPERIMENTS
    if (sb.presort) {
        hipError_t e = fmgi_set_lds_attr_once<2>((const void *)k_tile_runs_pre<FMGI_RING_CODES, 16>, (int)plds);
        if (e != hipSuccess) return e;
        const int G = (sb.groups + 7) & ~7;
        hipLaunchKernelGGL((k_tile_runs_pre<FMGI_RING_CODES, 16>), dim3((unsigned)(P * G)), dim3(sb.block > 0 ? sb.block : 1024), plds, s,
                           sb.stream, sb.toff, sb.cursor, sb.cap, P, G, (const uint4 *)sb.colpack, lm, num_texels);
        return hipGetLastError();
    }
#endif
    const size_t lds = (size_t)3 * kTileTexels * 8 + (size_t)FMGI_COLOUR_STATES * 16; /* 64 KiB: two workgroups per CU */
    const int G = (sb.groups + 7) & ~7; /* a multiple of 8 for the XCD-aware order */
    /* a slice's run of one tile averages slice / P codes: past 128 tiles the slices are 32768 codes (runs
       of ~90 at 358 tiles instead of ~23: the fold's per-run work and run-table reads shrink 4x; the sort
       stays HBM-bound) and a wave packs 16 slices' runs onto its lanes (k_tile_runs_pre over slices);
       below, 8192-code slices and one run at a time (FMGI_PACKED_RUNS=0/1 forces either, experiments) */
    bool packed = P > 128;
    if (const char *pe = fmgi_exp_env("FMGI_PACKED_RUNS")) packed = atoi(pe) != 0;
    if (packed) {
        constexpr int kBig = FMGI_STREAM_SLICE_BIG;
        const uint64_t nslices = (sb.cap + kBig - 1) / kBig;
        hipError_t e = fmgi_set_lds_attr_once<5>((const void *)k_slice_sort<kBig, 1024>, kBig * 4);
        if (e != hipSuccess) return e;
        hipLaunchKernelGGL((k_slice_sort<kBig, 1024>), dim3((unsigned)nslices), dim3(1024), (size_t)kBig * 4, s,
                           sb.stream, sb.cursor, sb.cap, P, sb.sorted, sb.toff);
        e = fmgi_set_lds_attr_once<4>((const void *)k_tile_runs_pre<kBig, 4>, (int)lds);
        if (e != hipSuccess) return e;
        hipLaunchKernelGGL((k_tile_runs_pre<kBig, 4>), dim3((unsigned)(P * G)), dim3(sb.block > 0 ? sb.block : 1024), lds,
                           s, sb.sorted, sb.toff, sb.cursor, sb.cap, P, G, (const uint4 *)sb.colpack, lm, num_texels);
        return hipGetLastError();
    }
    const uint64_t nslices = (sb.cap + kSlice - 1) / kSlice;
    hipLaunchKernelGGL((k_slice_sort<kSlice, 256>), dim3((unsigned)nslices), dim3(256), (size_t)kSlice * 4, s, sb.stream,
                       sb.cursor, sb.cap, P, sb.sorted, sb.toff);
    hipError_t e = fmgi_set_lds_attr_once<0>((const void *)k_tile_runs, (int)lds);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(k_tile_runs, dim3((unsigned)(P * G)), dim3(sb.block > 0 ? sb.block : 1024), lds, s, sb.sorted, sb.toff,
                       sb.cursor, sb.cap, P, G, (const uint4 *)sb.colpack, lm, num_texels);
    return hipGetLastError();
}
