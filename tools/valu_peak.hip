// tools/valu_peak.hip -- measured instruction-issue ceilings of one MI355X: wave64
// VALU instructions per second for dependency-free v_fma_f32 and v_fma_f64 streams
// at occupancies of 1, 2, 6 and 8 waves per SIMD. Each lane runs 8 independent FMA
// chains so dependency latency never stalls issue. Prints one JSON line per case.
//   build: hipcc --offload-arch=gfx950 -O3 tools/valu_peak.hip -o tools/valu_peak
#include <hip/hip_runtime.h>
#include <stdio.h>

constexpr int kIters = 4096;

template <int MODE>
__global__ __launch_bounds__(256) void k_issue(float *out, float seed) {
    float a0 = seed + threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6,
          a7 = a0 + 7;
    double d0 = a0, d1 = a1, d2 = a2, d3 = a3, d4 = a4, d5 = a5, d6 = a6, d7 = a7;
    const float m = 0.999f, c = 0.001f;
    for (int i = 0; i < kIters; i++) {
        if (MODE == 0) { // 8 x v_fma_f32
            asm volatile("v_fma_f32 %0, %0, %8, %9\n v_fma_f32 %1, %1, %8, %9\n v_fma_f32 %2, %2, %8, %9\n"
                         " v_fma_f32 %3, %3, %8, %9\n v_fma_f32 %4, %4, %8, %9\n v_fma_f32 %5, %5, %8, %9\n"
                         " v_fma_f32 %6, %6, %8, %9\n v_fma_f32 %7, %7, %8, %9"
                         : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7)
                         : "v"(m), "v"(c));
        } else if (MODE == 1) { // 8 x v_fma_f64
            asm volatile("v_fma_f64 %0, %0, %8, %9\n v_fma_f64 %1, %1, %8, %9\n v_fma_f64 %2, %2, %8, %9\n"
                         " v_fma_f64 %3, %3, %8, %9\n v_fma_f64 %4, %4, %8, %9\n v_fma_f64 %5, %5, %8, %9\n"
                         " v_fma_f64 %6, %6, %8, %9\n v_fma_f64 %7, %7, %8, %9"
                         : "+v"(d0), "+v"(d1), "+v"(d2), "+v"(d3), "+v"(d4), "+v"(d5), "+v"(d6), "+v"(d7)
                         : "v"((double)m), "v"((double)c));
        }
    }
    out[blockIdx.x * blockDim.x + threadIdx.x] =
        a0 + a1 + a2 + a3 + a4 + a5 + a6 + a7 + (float)(d0 + d1 + d2 + d3 + d4 + d5 + d6 + d7);
}

template <int MODE>
void run(const char *name, int cus, int waves_per_simd, float *d_out) {
    const int blocks = cus * waves_per_simd; // 256-lane blocks = 4 waves = one wave per SIMD each
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    hipLaunchKernelGGL(k_issue<MODE>, dim3(blocks), dim3(256), 0, 0, d_out, 1.0f); // warm-up
    hipEventRecord(e0);
    const int reps = 5;
    for (int r = 0; r < reps; r++) hipLaunchKernelGGL(k_issue<MODE>, dim3(blocks), dim3(256), 0, 0, d_out, 1.0f);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms = 0;
    hipEventElapsedTime(&ms, e0, e1);
    const double waves = (double)blocks * 4 * reps, insts = waves * kIters * 8; // VALU instructions counted
    printf("{\"case\": \"%s\", \"waves_per_simd\": %d, \"wave_valu_insts_per_s\": %.4e, \"per_simd_per_clk_at_2.4GHz\": %.3f}\n",
           name, waves_per_simd, insts / (ms * 1e-3), insts / (ms * 1e-3) / (cus * 4.0) / 2.4e9);
}

int main() {
    hipDeviceProp_t p;
    hipGetDeviceProperties(&p, 0);
    const int cus = p.multiProcessorCount;
    float *d_out;
    hipMalloc(&d_out, (size_t)cus * 8 * 256 * sizeof(float));
    for (int w : {1, 2, 6, 8}) {
        run<0>("v_fma_f32", cus, w, d_out);
        run<1>("v_fma_f64", cus, w, d_out);
    }
    printf("{\"cus\": %d, \"clock_khz\": %d}\n", cus, p.clockRate);
    return 0;
}
