/*
 * ref_runner.cpp -- runs the REFERENCE kernel (TEST INFRASTRUCTURE ONLY).
 *
 * Loads oracle/_ref/photonmap_{strict,fast}.hsaco -- /root/reference/photonmap.cl compiled for gfx950
 * by oracle/build_ref.sh with ROCm's own OpenCL device libraries -- and launches its `photonmap`
 * kernel (photonmap.cl:269) the way global_illumination_cl.c:233-258 does, but with ONE work item per
 * launch and a fresh zeroed lightColors buffer per item. One work item per launch removes the
 * kernel's lightColors[] += data race (photonmap.cl:256), and since the kernel only uses
 * get_global_id(0) through `gid + rng_offset` (photonmap.cl:272), running gid 0 with
 * rng_offset = gid + offset reproduces work item `gid` of a real launch exactly.
 *
 * Exposed to Python (tests/golden/make_ref_fixtures.py) through a tiny C interface.
 */
#include <hip/hip_runtime.h>

#include <stdint.h>
#include <stdio.h>
#include <string.h>

#include <algorithm>
#include <vector>

#define API extern "C" __attribute__((visibility("default")))

static hipModule_t g_mod = nullptr;
static hipFunction_t g_fn = nullptr;
static char g_err[512];

API const char *ref_last_error(void) { return g_err; }

#define CHK(x)                                                                              \
    do {                                                                                    \
        hipError_t e_ = (x);                                                                \
        if (e_ != hipSuccess) {                                                             \
            snprintf(g_err, sizeof g_err, "%s: %s", #x, hipGetErrorString(e_));             \
            return -1;                                                                      \
        }                                                                                   \
    } while (0)

API int ref_open(const char *hsaco) {
    if (g_mod) {
        (void)hipModuleUnload(g_mod);
        g_mod = nullptr;
    }
    CHK(hipSetDevice(0));
    CHK(hipModuleLoad(&g_mod, hsaco));
    CHK(hipModuleGetFunction(&g_fn, g_mod, "photonmap"));
    return 0;
}

/* Run n work items; item k uses rng_state = rng_states[k] (= gid + rng_offset of the real launch).
   texels_out receives n consecutive float4[num_texels] lightmaps (each from zero). */
/* exact fixed-point sum (units of 2^-25, int64 [num_texels][3]) of n per-item float4 lightmaps; every
   per-item value is a sum of deposits >= 0.25 (photonmap.cl:167-169,241-249), i.e. a multiple of 2^-25,
   so the conversion is exact (inexact conversions are counted, and must stay 0) */
__global__ void k_sum_fx(const float4 *__restrict__ tex, int n, int64_t num_texels, long long *__restrict__ sum,
                         unsigned long long *__restrict__ inexact) {
    const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= num_texels) return;
    long long r = 0, g = 0, b = 0;
    unsigned long long bad = 0;
    for (int k = 0; k < n; k++) { /* item order: deterministic */
        const float4 v = tex[(int64_t)k * num_texels + t];
        const double x = (double)v.x * 33554432.0, y = (double)v.y * 33554432.0, z = (double)v.z * 33554432.0;
        bad += (x != (double)(long long)x) + (y != (double)(long long)y) + (z != (double)(long long)z);
        r += (long long)x;
        g += (long long)y;
        b += (long long)z;
    }
    sum[3 * t] += r;
    sum[3 * t + 1] += g;
    sum[3 * t + 2] += b;
    if (bad) atomicAdd(inexact, bad);
}

/* Run n work items (item k: rng_state = rng_states[k]), each on its own zeroed lightColors buffer, in
   batches on `streams` concurrent streams, and add their lightmaps exactly into sum_fx[num_texels][3]
   (the launch's race-free sum; host array, accumulated into). Returns the inexact-conversion count
   (0 expected) or -1. */
API long long ref_run_sum(const void *window80, const void *rects80, int nrects, int num_texels, int is_window,
                          const uint32_t *rng_states, int n, int streams, long long *sum_fx) {
    if (!g_fn) {
        snprintf(g_err, sizeof g_err, "ref_open() first");
        return -1;
    }
    const int NS = streams < 1 ? 1 : (streams > 32 ? 32 : streams);
    std::vector<hipStream_t> st(NS);
    for (int i = 0; i < NS; i++) CHK(hipStreamCreateWithFlags(&st[i], hipStreamNonBlocking));
    const size_t tb = (size_t)num_texels * 16;
    int B = (int)std::max<size_t>(1, std::min<size_t>((size_t)1 << 30, tb * 1024) / tb); /* <= 1 GiB per batch */
    if (B > n) B = n;
    void *d_win = nullptr, *d_rects = nullptr, *d_tex = nullptr;
    long long *d_sum = nullptr;
    unsigned long long *d_bad = nullptr;
    CHK(hipMalloc(&d_win, 80));
    CHK(hipMalloc(&d_rects, (size_t)nrects * 80 + 80));
    CHK(hipMalloc(&d_tex, tb * (size_t)B));
    CHK(hipMalloc(&d_sum, (size_t)num_texels * 24));
    CHK(hipMalloc(&d_bad, 8));
    CHK(hipMemcpy(d_win, window80, 80, hipMemcpyHostToDevice));
    if (nrects) CHK(hipMemcpy(d_rects, rects80, (size_t)nrects * 80, hipMemcpyHostToDevice));
    CHK(hipMemcpy(d_sum, sum_fx, (size_t)num_texels * 24, hipMemcpyHostToDevice));
    CHK(hipMemset(d_bad, 0, 8));
    for (int b0 = 0; b0 < n; b0 += B) {
        const int nb = std::min(B, n - b0);
        CHK(hipMemset(d_tex, 0, tb * (size_t)nb));
        for (int k = 0; k < nb; k++) {
            void *tex = (char *)d_tex + tb * (size_t)k;
            int32_t off = (int32_t)rng_states[b0 + k];
            int32_t nr = nrects, isw = is_window;
            void *args[] = {&d_win, &d_rects, &nr, &tex, &off, &isw};
            CHK(hipModuleLaunchKernel(g_fn, 1, 1, 1, 1, 1, 1, 0, st[k % NS], args, nullptr));
        }
        CHK(hipDeviceSynchronize());
        hipLaunchKernelGGL(k_sum_fx, dim3((unsigned)((num_texels + 255) / 256)), dim3(256), 0, 0, (const float4 *)d_tex,
                           nb, (int64_t)num_texels, d_sum, d_bad);
        CHK(hipGetLastError());
        CHK(hipDeviceSynchronize());
    }
    unsigned long long bad = 0;
    CHK(hipMemcpy(sum_fx, d_sum, (size_t)num_texels * 24, hipMemcpyDeviceToHost));
    CHK(hipMemcpy(&bad, d_bad, 8, hipMemcpyDeviceToHost));
    (void)hipFree(d_win);
    (void)hipFree(d_rects);
    (void)hipFree(d_tex);
    (void)hipFree(d_sum);
    (void)hipFree(d_bad);
    for (int i = 0; i < NS; i++) (void)hipStreamDestroy(st[i]);
    return (long long)bad;
}

API int ref_run_items(const void *window80, const void *rects80, int nrects, int num_texels, int is_window,
                      const uint32_t *rng_states, int n, float *texels_out) {
    if (!g_fn) {
        snprintf(g_err, sizeof g_err, "ref_open() first");
        return -1;
    }
    const int NS = 4;
    hipStream_t st[NS];
    for (int i = 0; i < NS; i++) CHK(hipStreamCreateWithFlags(&st[i], hipStreamNonBlocking));
    void *d_win = nullptr, *d_rects = nullptr, *d_tex = nullptr;
    size_t tb = (size_t)num_texels * 16;
    CHK(hipMalloc(&d_win, 80));
    CHK(hipMalloc(&d_rects, (size_t)nrects * 80));
    CHK(hipMalloc(&d_tex, tb * (size_t)n));
    CHK(hipMemcpy(d_win, window80, 80, hipMemcpyHostToDevice));
    CHK(hipMemcpy(d_rects, rects80, (size_t)nrects * 80, hipMemcpyHostToDevice));
    CHK(hipMemset(d_tex, 0, tb * (size_t)n));
    for (int k = 0; k < n; k++) {
        void *tex = (char *)d_tex + tb * (size_t)k;
        int32_t off = (int32_t)rng_states[k];
        int32_t nr = nrects, isw = is_window;
        void *args[] = {&d_win, &d_rects, &nr, &tex, &off, &isw};
        CHK(hipModuleLaunchKernel(g_fn, 1, 1, 1, 1, 1, 1, 0, st[k % NS], args, nullptr));
    }
    CHK(hipDeviceSynchronize());
    CHK(hipMemcpy(texels_out, d_tex, tb * (size_t)n, hipMemcpyDeviceToHost));
    (void)hipFree(d_win);
    (void)hipFree(d_rects);
    (void)hipFree(d_tex);
    for (int i = 0; i < NS; i++) (void)hipStreamDestroy(st[i]);
    return 0;
}
