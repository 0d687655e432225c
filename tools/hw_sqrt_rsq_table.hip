// tools/hw_sqrt_rsq_table.hip -- records gfx950's v_sqrt_f32 and v_rsq_f32 (the hardware ops behind ROCm's
// OpenCL length() and normalize() builtins, which the reference photonmap.cl calls) as truth tables for the
// CPU oracle. Both ops depend only on the input's mantissa and exponent parity (checked over 40 binades by
// tools/hw_sqrt_table.hip), so the inputs x in [1, 4) -- index i = parity << 23 | mantissa -- describe them
// for every normal input. Output (argv[1]): int8 delta_sqrt[2^24] then int8 delta_rsq[2^24], each the
// difference in ulps (float bit patterns) from the once-rounded double value (float)sqrt((double)x) and
// (float)(1.0 / sqrt((double)x)). tests/golden/make_hw_tables.py compresses it into
// tests/golden/gfx950_sqrt_rsq.npz.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>

__global__ void k_table(signed char *ds, signed char *dr, unsigned long long *big) {
    const unsigned i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= (1u << 24)) return;
    const float x = __uint_as_float(((127u + (i >> 23)) << 23) | (i & 0x7FFFFFu));
    const float bs = (float)__dsqrt_rn((double)x), br = (float)(1.0 / __dsqrt_rn((double)x));
    const int s = (int)__float_as_uint(__builtin_amdgcn_sqrtf(x)) - (int)__float_as_uint(bs);
    const int r = (int)__float_as_uint(__builtin_amdgcn_rsqf(x)) - (int)__float_as_uint(br);
    if (s < -1 || s > 1) atomicAdd(big, 1ull);
    if (r < -1 || r > 1) atomicAdd(big + 1, 1ull);
    ds[i] = (signed char)s;
    dr[i] = (signed char)r;
}

int main(int argc, char **argv) {
    const size_t n = 1u << 24;
    signed char *d;
    unsigned long long *db;
    if (argc < 2 || hipMalloc(&d, 2 * n) || hipMalloc(&db, 16) || hipMemset(db, 0, 16)) return 1;
    hipLaunchKernelGGL(k_table, dim3(n / 256), dim3(256), 0, 0, d, d + n, db);
    signed char *h = (signed char *)malloc(2 * n);
    unsigned long long big[2];
    if (hipMemcpy(h, d, 2 * n, hipMemcpyDeviceToHost) || hipMemcpy(big, db, 16, hipMemcpyDeviceToHost)) return 1;
    FILE *f = fopen(argv[1], "wb");
    if (!f || fwrite(h, 1, 2 * n, f) != 2 * n) return 1;
    fclose(f);
    long long ns = 0, nr = 0;
    for (size_t i = 0; i < n; i++) { ns += h[i] != 0; nr += h[n + i] != 0; }
    printf("{\"entries\": %zu, \"sqrt_differs\": %lld, \"rsq_differs\": %lld, \"beyond_1ulp\": [%llu, %llu]}\n", n, ns,
           nr, big[0], big[1]);
    return big[0] || big[1];
}
