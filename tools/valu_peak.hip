// tools/valu_peak.hip -- measured instruction-issue ceilings of one MI355X: wave64 VALU instructions per
// second for dependency-free v_fma_f32 streams (three VGPR sources, as compiled code reads them, and one
// VGPR source with inline constants: no operand-bank conflicts) and v_fma_f64, at 1-8 waves per SIMD, on
// launches of >= 50 ms (the chip's clock under sustained load, not a 0.3-ms burst), with the in-kernel
// clock of every case measured per MI355X_MICROARCH.md "DVFS give-back" item 6: delta s_memtime / delta
// s_memrealtime x 100 MHz, stamped by each wave around its loop (median over waves). Each lane runs 8
// independent FMA chains so dependency latency never stalls issue. Prints one JSON line per case.
//   build: hipcc --offload-arch=gfx950 -O3 tools/valu_peak.hip -o tools/valu_peak
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>

#include <algorithm>
#include <vector>

template <int MODE>
__global__ __launch_bounds__(256) void k_issue(float *out, unsigned long long *stamps, float seed, int iters) {
    float a0 = seed + threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6,
          a7 = a0 + 7;
    double d0 = a0, d1 = a1, d2 = a2, d3 = a3, d4 = a4, d5 = a5, d6 = a6, d7 = a7;
    const float m = 0.999f, c = 0.001f;
    const unsigned long long t0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
    for (int i = 0; i < iters; i++) {
        if (MODE == 0) { // 8 x v_fma_f32
            asm volatile("v_fma_f32 %0, %0, %8, %9\n v_fma_f32 %1, %1, %8, %9\n v_fma_f32 %2, %2, %8, %9\n"
                         " v_fma_f32 %3, %3, %8, %9\n v_fma_f32 %4, %4, %8, %9\n v_fma_f32 %5, %5, %8, %9\n"
                         " v_fma_f32 %6, %6, %8, %9\n v_fma_f32 %7, %7, %8, %9"
                         : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7)
                         : "v"(m), "v"(c));
        } else if (MODE == 2) { // 8 x v_fma_f32 with one VGPR source (inline constants: no operand-bank conflicts)
            asm volatile("v_fma_f32 %0, %0, 0.5, 1.0\n v_fma_f32 %1, %1, 0.5, 1.0\n v_fma_f32 %2, %2, 0.5, 1.0\n"
                         " v_fma_f32 %3, %3, 0.5, 1.0\n v_fma_f32 %4, %4, 0.5, 1.0\n v_fma_f32 %5, %5, 0.5, 1.0\n"
                         " v_fma_f32 %6, %6, 0.5, 1.0\n v_fma_f32 %7, %7, 0.5, 1.0"
                         : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7));
        } else { // 8 x v_fma_f64
            asm volatile("v_fma_f64 %0, %0, %8, %9\n v_fma_f64 %1, %1, %8, %9\n v_fma_f64 %2, %2, %8, %9\n"
                         " v_fma_f64 %3, %3, %8, %9\n v_fma_f64 %4, %4, %8, %9\n v_fma_f64 %5, %5, %8, %9\n"
                         " v_fma_f64 %6, %6, %8, %9\n v_fma_f64 %7, %7, %8, %9"
                         : "+v"(d0), "+v"(d1), "+v"(d2), "+v"(d3), "+v"(d4), "+v"(d5), "+v"(d6), "+v"(d7)
                         : "v"((double)m), "v"((double)c));
        }
    }
    const unsigned long long t1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
    const unsigned w = blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
    if ((threadIdx.x & 63) == 0) { // vector stores of the stamps (a buffer of their own)
        stamps[2 * w] = t1 - t0;
        stamps[2 * w + 1] = r1 - r0;
    }
    out[blockIdx.x * blockDim.x + threadIdx.x] =
        a0 + a1 + a2 + a3 + a4 + a5 + a6 + a7 + (float)(d0 + d1 + d2 + d3 + d4 + d5 + d6 + d7);
}

template <int MODE>
float launch(int blocks, float *d_out, unsigned long long *d_st, int iters, int reps) {
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    hipEventRecord(e0);
    for (int r = 0; r < reps; r++) hipLaunchKernelGGL(k_issue<MODE>, dim3(blocks), dim3(256), 0, 0, d_out, d_st, 1.0f, iters);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms = 0;
    hipEventElapsedTime(&ms, e0, e1);
    hipEventDestroy(e0);
    hipEventDestroy(e1);
    return ms / reps;
}

template <int MODE>
void run(const char *name, int cus, int waves_per_simd, float *d_out, unsigned long long *d_st) {
    const int blocks = cus * waves_per_simd; // 256-lane blocks = 4 waves = one wave per SIMD each
    // calibrate: one short launch, then iterations for >= 60 ms per launch
    int iters = 4096;
    launch<MODE>(blocks, d_out, d_st, iters, 1);
    const float ms0 = launch<MODE>(blocks, d_out, d_st, iters, 1);
    iters = (int)std::min(2.0e9, iters * (60.0 / std::max(ms0, 1e-3f)));
    launch<MODE>(blocks, d_out, d_st, iters, 2); // >= 2 s of back-to-back load before the measured launches
    for (int k = 0; k < 30; k++) launch<MODE>(blocks, d_out, d_st, iters, 1);
    const int reps = 3;
    const float ms = launch<MODE>(blocks, d_out, d_st, iters, reps);
    const int nw = blocks * 4;
    std::vector<unsigned long long> st(2 * (size_t)nw);
    hipMemcpy(st.data(), d_st, st.size() * 8, hipMemcpyDeviceToHost);
    std::vector<double> clk(nw);
    for (int w = 0; w < nw; w++) clk[w] = st[2 * w + 1] ? 0.1 * (double)st[2 * w] / (double)st[2 * w + 1] : 0.0;
    std::sort(clk.begin(), clk.end());
    const double ghz = clk[nw / 2];
    const double insts = (double)nw * iters * 8; // VALU instructions per launch
    const double per_s = insts / (ms * 1e-3);
    printf("{\"case\": \"%s\", \"waves_per_simd\": %d, \"launch_ms\": %.2f, \"wave_valu_insts_per_s\": %.4e, "
           "\"in_kernel_clock_ghz\": %.3f, \"per_simd_per_clk_at_measured_clock\": %.4f, "
           "\"per_simd_per_clk_at_2.4GHz\": %.4f}\n",
           name, waves_per_simd, ms, per_s, ghz, per_s / (cus * 4.0) / (ghz * 1e9), per_s / (cus * 4.0) / 2.4e9);
    fflush(stdout);
}

int main() {
    hipDeviceProp_t p;
    hipGetDeviceProperties(&p, 0);
    const int cus = p.multiProcessorCount;
    float *d_out;
    unsigned long long *d_st;
    hipMalloc(&d_out, (size_t)cus * 8 * 256 * sizeof(float));
    hipMalloc(&d_st, (size_t)cus * 8 * 4 * 2 * sizeof(unsigned long long));
    for (int w : {1, 2, 4, 5, 8}) run<0>("v_fma_f32", cus, w, d_out, d_st);
    for (int w : {1, 2, 4, 5, 8}) run<2>("v_fma_f32_1vgpr", cus, w, d_out, d_st);
    for (int w : {1, 5, 8}) run<1>("v_fma_f64", cus, w, d_out, d_st);
    printf("{\"cus\": %d, \"clock_khz\": %d}\n", cus, p.clockRate);
    return 0;
}
