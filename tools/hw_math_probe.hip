// tools/hw_math_probe.hip -- experiment: the arithmetic ROCm's OpenCL builtins execute on gfx950 (what the
// reference photonmap.cl runs on MI355X) against exact restatements:
//   1. OCML __ocml_sin_f32/__ocml_cos_f32 (HIP sinf/cosf) vs the C restatement in fmgi_math.h
//      (fmgi_sincosf_ocml) on every reachable sampler phi;
//   2. v_sqrt_f32 (the length() builtin: llvm.sqrt with !fpmath 3.0) vs a correctly rounded sqrt, every
//      float in [2^-2, 2^2);
//   3. v_rsq_f32 (normalize() via __ocml_rsqrt_f32) vs 1/sqrt rounded once, every float in [2^-2, 2^2).
// Prints one JSON line of mismatch counts and the first examples.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

#include "fmgi_math.h"

#pragma clang fp contract(off)

constexpr uint32_t kReach = 83886081u;

__device__ __forceinline__ float reachable_phi(uint32_t i) {
    float f;
    if (i < (1u << 24)) f = (float)i;
    else if (i == kReach - 1) f = 4294967296.0f;
    else {
        const uint32_t j = i - (1u << 24), e = 24 + j / (1u << 23), m = j % (1u << 23);
        f = ldexpf((float)((1u << 23) + m), (int)e - 23);
    }
    return 6.283184f * (f * 2.3283064365386963e-10f);
}

struct Ex { uint32_t in, got, want, kind; };

__global__ void k_sincos(unsigned long long *cnt, Ex *ex) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= kReach) return;
    const float phi = reachable_phi(i);
    float s, c;
    fmgi_sincosf(phi, &s, &c);
    const float os = sinf(phi), oc = cosf(phi);
    if (__float_as_uint(s) != __float_as_uint(os) || __float_as_uint(c) != __float_as_uint(oc)) {
        const unsigned long long k = atomicAdd(cnt + 0, 1ull);
        if (k < 4) ex[k] = Ex{__float_as_uint(phi), __float_as_uint(s), __float_as_uint(os), 0};
    }
}

__global__ void k_sqrt(unsigned long long *cnt, Ex *ex) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; // 4 binades from 2^-2
    if (i >= (4u << 23)) return;
    const float x = __uint_as_float(0x3E800000u + i);
    const float hs = __builtin_amdgcn_sqrtf(x), cs = (float)__dsqrt_rn((double)x);
    if (__float_as_uint(hs) != __float_as_uint(cs)) {
        const unsigned long long k = atomicAdd(cnt + 1, 1ull);
        if (k < 4) ex[4 + k] = Ex{__float_as_uint(x), __float_as_uint(hs), __float_as_uint(cs), 1};
    }
    const float hr = __builtin_amdgcn_rsqf(x), cr = (float)(1.0 / __dsqrt_rn((double)x));
    if (__float_as_uint(hr) != __float_as_uint(cr)) {
        const unsigned long long k = atomicAdd(cnt + 2, 1ull);
        if (k < 4) ex[8 + k] = Ex{__float_as_uint(x), __float_as_uint(hr), __float_as_uint(cr), 2};
    }
}

int main() {
    unsigned long long *d_cnt;
    Ex *d_ex;
    if (hipMalloc(&d_cnt, 64) || hipMalloc(&d_ex, sizeof(Ex) * 12) || hipMemset(d_cnt, 0, 64) ||
        hipMemset(d_ex, 0, sizeof(Ex) * 12))
        return 1;
    hipLaunchKernelGGL(k_sincos, dim3((kReach + 255) / 256), dim3(256), 0, 0, d_cnt, d_ex);
    hipLaunchKernelGGL(k_sqrt, dim3((4u << 23) / 256), dim3(256), 0, 0, d_cnt, d_ex);
    unsigned long long cnt[8];
    Ex ex[12];
    if (hipMemcpy(cnt, d_cnt, 64, hipMemcpyDeviceToHost) || hipMemcpy(ex, d_ex, sizeof ex, hipMemcpyDeviceToHost))
        return 1;
    printf("{\"sincos_restatement_vs_ocml\": %llu, \"v_sqrt_f32_vs_rn\": %llu, \"v_rsq_f32_vs_rn\": %llu, "
           "\"inputs\": [%u, %u]}\n", cnt[0], cnt[1], cnt[2], kReach, 4u << 23);
    for (int k = 0; k < 12; k++)
        if (ex[k].in) printf("kind %u in %08x got %08x want %08x\n", ex[k].kind, ex[k].in, ex[k].got, ex[k].want);
    return 0;
}
