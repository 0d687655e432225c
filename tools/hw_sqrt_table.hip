// tools/hw_sqrt_table.hip -- experiment: v_sqrt_f32 / v_rsq_f32 (the hardware ops behind ROCm's OpenCL
// length() / normalize() builtins on gfx950) of the float32 inputs in argv[1]; writes {in, sqrt, rsq}
// float32 triples to argv[2] and checks whether v_sqrt_f32 depends only on (mantissa, exponent parity).
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <vector>

__global__ void k_eval(const float *x, float *out, int n) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    out[3 * i] = x[i];
    out[3 * i + 1] = __builtin_amdgcn_sqrtf(x[i]);
    out[3 * i + 2] = __builtin_amdgcn_rsqf(x[i]);
}

// v_sqrt_f32(4x) == 2 v_sqrt_f32(x) for every x in [2^-20, 2^20)?
__global__ void k_period(unsigned long long *bad) {
    const unsigned i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= (40u << 23)) return;
    const float x = __uint_as_float(0x35800000u + i); // 2^-20 ...
    const float a = __builtin_amdgcn_sqrtf(4.0f * x), b = 2.0f * __builtin_amdgcn_sqrtf(x);
    const float c = __builtin_amdgcn_rsqf(4.0f * x), d = 0.5f * __builtin_amdgcn_rsqf(x);
    if (__float_as_uint(a) != __float_as_uint(b)) atomicAdd(bad, 1ull);
    if (__float_as_uint(c) != __float_as_uint(d)) atomicAdd(bad + 1, 1ull);
}

int main(int argc, char **argv) {
    FILE *f = fopen(argv[1], "rb");
    std::vector<float> x(1 << 20);
    const int n = (int)fread(x.data(), 4, x.size(), f);
    fclose(f);
    float *dx, *dout;
    unsigned long long *dbad;
    if (hipMalloc(&dx, 4 * n) || hipMalloc(&dout, 12 * n) || hipMalloc(&dbad, 16) || hipMemset(dbad, 0, 16) ||
        hipMemcpy(dx, x.data(), 4 * n, hipMemcpyHostToDevice))
        return 1;
    hipLaunchKernelGGL(k_eval, dim3((n + 255) / 256), dim3(256), 0, 0, dx, dout, n);
    hipLaunchKernelGGL(k_period, dim3((40u << 23) / 256), dim3(256), 0, 0, dbad);
    std::vector<float> out(3 * n);
    unsigned long long bad[2];
    if (hipMemcpy(out.data(), dout, 12 * n, hipMemcpyDeviceToHost) || hipMemcpy(bad, dbad, 16, hipMemcpyDeviceToHost))
        return 1;
    FILE *g = fopen(argv[2], "wb");
    fwrite(out.data(), 4, 3 * n, g);
    fclose(g);
    printf("{\"inputs\": %d, \"sqrt_not_periodic\": %llu, \"rsq_not_periodic\": %llu}\n", n, bad[0], bad[1]);
    return 0;
}
