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
