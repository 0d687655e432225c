/*
 * fmgi_accum.hip -- "stream" accumulation of the lightmap deposits (FMGI_ACCUM_STREAM).
 *
 * The reference adds every deposit straight into lightColors[] (photonmap.cl:256-258, a data race).
 * Device-scope atomics make that exact but cost one memory-side transaction per deposit, and MI355X
 * executes ~2e10 of those per second (MI355X_MICROARCH.md §Global float atomics): the bake then runs at
 * the atomic rate instead of the tracing rate. This path replaces the atomics with bandwidth:
 *
 *   bake   : each deposit appends a 32-bit code (texel << 10 | colour state) to a stream with plain,
 *            wave-coalesced stores (k_bake, AccStream; one reservation atomic per 4096 codes per wave)
 *   hist   : per 8192-code slice, a histogram of 4096-texel tiles (LDS)                 k_tile_hist
 *   scan   : exclusive scan of the tile-major histogram (hipCUB) -> each (tile, slice) run's offset
 *   scatter: per slice, a counting sort by tile in LDS, written out as contiguous runs   k_tile_scatter
 *   accum  : per chunk of the tile-sorted stream, exact int64 RGB sums of one tile at a time in LDS
 *            (ds_add_u64), flushed once per tile and chunk into the lightmap           k_tile_accum
 *
 * Every step is exact integer arithmetic, so the lightmap is bit-identical to the atomic paths.
 */
#include <hip/hip_runtime.h>
#include <hipcub/hipcub.hpp>

#include "fmgi_internal.h"

namespace {

constexpr int kSlice = FMGI_STREAM_SLICE;     /* codes per hist/scatter block */
constexpr int kTileTexels = 1 << FMGI_TILE_BITS;
constexpr uint32_t kSentinel = 0xFFFFFFFFu;

__device__ __forceinline__ int tile_of(uint32_t code) { return (int)(code >> (10 + FMGI_TILE_BITS)); }

__global__ __launch_bounds__(256) void k_tile_hist(const uint32_t *__restrict__ stream,
                                                  const unsigned long long *__restrict__ n_ptr, uint64_t cap, int P,
                                                  int nslices, unsigned long long *__restrict__ hist) {
    __shared__ uint32_t h[FMGI_MAX_TILES];
    for (int i = threadIdx.x; i < P; i += blockDim.x) h[i] = 0;
    __syncthreads();
    const uint64_t n = *n_ptr < cap ? *n_ptr : cap;
    const uint64_t b0 = (uint64_t)blockIdx.x * kSlice;
    if (b0 >= n) return; /* uniform; hist was zeroed */
    constexpr int per = kSlice / 256;
    uint32_t c[per];
#pragma unroll
    for (int k = 0; k < per; k++) { /* all loads in flight before the first LDS atomic */
        const uint64_t i = b0 + (uint64_t)k * 256 + threadIdx.x;
        c[k] = i < n ? stream[i] : kSentinel;
    }
#pragma unroll
    for (int k = 0; k < per; k++)
        if (c[k] != kSentinel) atomicAdd(&h[tile_of(c[k])], 1u);
    __syncthreads();
    for (int t = threadIdx.x; t < P; t += blockDim.x) hist[(size_t)t * nslices + blockIdx.x] = h[t];
}

/* exclusive scan of cnt[0..P) into loc[0..P) by one block (P <= FMGI_MAX_TILES) */
__device__ void block_exclusive_scan(const uint32_t *cnt, uint32_t *loc, int P) {
    __shared__ uint32_t part[256];
    constexpr int per = FMGI_MAX_TILES / 256;
    const int t0 = threadIdx.x * per;
    uint32_t s = 0;
    for (int k = 0; k < per; k++) s += (t0 + k < P) ? cnt[t0 + k] : 0u;
    part[threadIdx.x] = s;
    __syncthreads();
    for (int off = 1; off < 256; off <<= 1) { /* Hillis-Steele over the 256 partial sums */
        const uint32_t v = threadIdx.x >= (unsigned)off ? part[threadIdx.x - off] : 0u;
        __syncthreads();
        part[threadIdx.x] += v;
        __syncthreads();
    }
    uint32_t run = part[threadIdx.x] - s;
    for (int k = 0; k < per; k++) {
        if (t0 + k < P) {
            loc[t0 + k] = run;
            run += cnt[t0 + k];
        }
    }
    __syncthreads();
}

__global__ __launch_bounds__(256) void k_tile_scatter(const uint32_t *__restrict__ stream,
                                                     const unsigned long long *__restrict__ n_ptr, uint64_t cap, int P,
                                                     int nslices, const unsigned long long *__restrict__ offs,
                                                     uint32_t *__restrict__ sorted) {
    __shared__ uint32_t buf[kSlice];
    __shared__ uint32_t cnt[FMGI_MAX_TILES], loc[FMGI_MAX_TILES];
    __shared__ unsigned long long dst[FMGI_MAX_TILES]; /* this slice's run start of each tile */
    constexpr int per = kSlice / 256;
    const uint64_t n = *n_ptr < cap ? *n_ptr : cap;
    const uint64_t b0 = (uint64_t)blockIdx.x * kSlice;
    if (b0 >= n) return; /* uniform: the whole block is past the end */
    for (int i = threadIdx.x; i < P; i += blockDim.x) {
        cnt[i] = 0;
        dst[i] = offs[(size_t)i * nslices + blockIdx.x];
    }
    __syncthreads();
    uint32_t c[per];
#pragma unroll
    for (int k = 0; k < per; k++) {
        const uint64_t i = b0 + (uint64_t)k * 256 + threadIdx.x;
        c[k] = i < n ? stream[i] : kSentinel;
    }
#pragma unroll
    for (int k = 0; k < per; k++)
        if (c[k] != kSentinel) atomicAdd(&cnt[tile_of(c[k])], 1u);
    __syncthreads();
    block_exclusive_scan(cnt, loc, P);
    /* counting sort into LDS: cnt becomes the running cursor of each tile */
    for (int i = threadIdx.x; i < P; i += blockDim.x) cnt[i] = loc[i];
    __syncthreads();
#pragma unroll
    for (int k = 0; k < per; k++)
        if (c[k] != kSentinel) buf[atomicAdd(&cnt[tile_of(c[k])], 1u)] = c[k];
    __syncthreads();
    const int total = (int)(cnt[P - 1]); /* end of the last tile = number of valid codes */
    for (int k = threadIdx.x; k < total; k += blockDim.x) {
        const uint32_t v = buf[k];
        const int t = tile_of(v);
        sorted[dst[t] + (uint64_t)(k - (int)loc[t])] = v;
    }
}

__global__ __launch_bounds__(1024) void k_tile_accum(const uint32_t *__restrict__ sorted,
                                                    const unsigned long long *__restrict__ offs, int P,
                                                    int nslices, const long long *__restrict__ colfx,
                                                    unsigned long long *__restrict__ lm, int num_texels) {
    extern __shared__ __attribute__((aligned(16))) unsigned long long s_acc[]; /* [4096][3] + colour table */
    unsigned long long *acc = s_acc;
    long long *col = (long long *)(s_acc + 3 * kTileTexels);
    for (int i = threadIdx.x; i < 3 * FMGI_COLOUR_STATES; i += blockDim.x) col[i] = colfx[i];
    const uint64_t total = offs[(size_t)P * nslices];
    const uint64_t per_block = (total + gridDim.x - 1) / gridDim.x;
    const uint64_t c0 = (uint64_t)blockIdx.x * per_block;
    const uint64_t c1 = c0 + per_block < total ? c0 + per_block : total;
    if (c0 >= c1) return; /* uniform */
    /* first tile overlapping [c0, c1): tile t spans [offs[t*nslices], offs[(t+1)*nslices]) */
    int lo = 0, hi = P - 1;
    while (lo < hi) {
        const int mid = (lo + hi + 1) >> 1;
        if (offs[(size_t)mid * nslices] <= c0) lo = mid; else hi = mid - 1;
    }
    for (int t = lo; t < P; t++) {
        const uint64_t ts = offs[(size_t)t * nslices], te = offs[(size_t)(t + 1) * nslices];
        const uint64_t s0 = ts > c0 ? ts : c0, s1 = te < c1 ? te : c1;
        if (s0 >= c1) break;
        if (s0 >= s1) continue;
        for (int i = threadIdx.x; i < 3 * kTileTexels; i += blockDim.x) acc[i] = 0;
        __syncthreads();
        constexpr int U = 4; /* loads in flight per thread */
        for (uint64_t i0 = s0 + threadIdx.x; i0 < s1; i0 += (uint64_t)U * blockDim.x) {
            uint32_t v[U];
#pragma unroll
            for (int u = 0; u < U; u++) {
                const uint64_t i = i0 + (uint64_t)u * blockDim.x;
                v[u] = i < s1 ? sorted[i] : kSentinel;
            }
#pragma unroll
            for (int u = 0; u < U; u++) {
                if (v[u] == kSentinel) continue;
                const int tx = (int)((v[u] >> 10) & (kTileTexels - 1));
                const int sid = (int)(v[u] & 1023);
                atomicAdd(&acc[3 * tx + 0], (unsigned long long)col[3 * sid + 0]);
                atomicAdd(&acc[3 * tx + 1], (unsigned long long)col[3 * sid + 1]);
                atomicAdd(&acc[3 * tx + 2], (unsigned long long)col[3 * sid + 2]);
            }
        }
        __syncthreads();
        for (int i = threadIdx.x; i < 3 * kTileTexels; i += blockDim.x) {
            const unsigned long long v = acc[i];
            const int texel = t * kTileTexels + i / 3;
            if (v && texel < num_texels) atomicAdd(lm + 4 * (size_t)texel + (i % 3), v);
        }
        __syncthreads();
    }
}

} // namespace

size_t fmgi_stream_scan_bytes(int entries) {
    size_t b = 0;
    (void)hipcub::DeviceScan::ExclusiveSum(nullptr, b, (const unsigned long long *)nullptr,
                                           (unsigned long long *)nullptr, entries, (hipStream_t)0);
    return b;
}

hipError_t fmgi_stream_fold(const StreamBufs &sb, int num_texels, const long long *colfx, unsigned long long *lm,
                            hipStream_t s) {
    const int P = (num_texels + kTileTexels - 1) / kTileTexels;
    const int nslices = (int)((sb.cap + kSlice - 1) / kSlice);
    const int entries = P * nslices + 1;
    hipError_t e = hipMemsetAsync(sb.hist, 0, (size_t)entries * sizeof(unsigned long long), s);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(k_tile_hist, dim3(nslices), dim3(256), 0, s, sb.stream, sb.cursor, sb.cap, P, nslices, sb.hist);
    size_t tb = sb.scan_tmp_bytes;
    e = hipcub::DeviceScan::ExclusiveSum(sb.scan_tmp, tb, sb.hist, sb.offs, entries, s); /* u64 in, u64 out */
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(k_tile_scatter, dim3(nslices), dim3(256), 0, s, sb.stream, sb.cursor, sb.cap, P, nslices, sb.offs,
                       sb.sorted);
    const size_t lds = (size_t)(3 * kTileTexels + 3 * FMGI_COLOUR_STATES) * 8; /* 120 KiB of the 160 */
    static bool lds_set = false;
    if (!lds_set) {
        e = hipFuncSetAttribute((const void *)k_tile_accum, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
        if (e != hipSuccess) return e;
        lds_set = true;
    }
    hipLaunchKernelGGL(k_tile_accum, dim3(sb.accum_blocks), dim3(1024), lds, s, sb.sorted, sb.offs, P, nslices,
                       colfx, lm, num_texels);
    return hipGetLastError();
}
