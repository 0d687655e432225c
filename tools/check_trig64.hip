// Exhaustive check (experiment): device double cos/sin vs the host's glibc cos/sin on every float x in
// [0, 6.283184f], as (double)x. Prints the mismatch counts. Build: hipcc -O3 --offload-arch=gfx950.
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdio.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#include <algorithm>
#include <thread>
#include <vector>

__global__ void k_trig(uint32_t first, uint32_t n, double *c, double *s) {
    uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    uint32_t bits = first + i;
    float x = __uint_as_float(bits);
    c[i] = cos((double)x);
    s[i] = sin((double)x);
}

int main() {
    float hi = 2 * 3.141592f;
    uint32_t lastbits;
    memcpy(&lastbits, &hi, 4);
    const uint32_t total = lastbits + 1;  // bit patterns 0 .. bits(6.283184f)
    const uint32_t chunk = 1u << 26;
    double *dc, *ds;
    hipMalloc(&dc, chunk * 8ull);
    hipMalloc(&ds, chunk * 8ull);
    std::vector<double> hc(chunk), hs(chunk);
    unsigned long long badc = 0, bads = 0;
    for (uint32_t first = 0; first < total; first += chunk) {
        uint32_t n = std::min(chunk, total - first);
        hipLaunchKernelGGL(k_trig, dim3((n + 255) / 256), dim3(256), 0, 0, first, n, dc, ds);
        hipMemcpy(hc.data(), dc, n * 8ull, hipMemcpyDeviceToHost);
        hipMemcpy(hs.data(), ds, n * 8ull, hipMemcpyDeviceToHost);
        const int T = 16;
        std::vector<unsigned long long> bc(T, 0), bs(T, 0);
        std::vector<std::thread> th;
        for (int t = 0; t < T; t++)
            th.emplace_back([&, t] {
                for (uint32_t i = t; i < n; i += T) {
                    uint32_t bits = first + i;
                    float x;
                    memcpy(&x, &bits, 4);
                    double c = cos((double)x), s = sin((double)x);
                    if (memcmp(&c, &hc[i], 8)) bc[t]++;
                    if (memcmp(&s, &hs[i], 8)) bs[t]++;
                }
            });
        for (auto &t : th) t.join();
        for (int t = 0; t < T; t++) { badc += bc[t]; bads += bs[t]; }
    }
    printf("floats checked %u, cos mismatches %llu, sin mismatches %llu\n", total, badc, bads);
    return 0;
}
