// tools/valu_peak.hip -- the vector-instruction issue ceiling of one MI355X SIMD, measured per SIMD.
//
// Each case is a loop whose body is 64 (or, for the round-3 form, 8) independent instructions in one asm
// block over 16 accumulator chains, so that neither dependency latency nor the loop's own s_add / s_cmp /
// s_cbranch (3 scalar instructions per iteration) sets the rate unless the case asks for it. Every wave
// stamps s_memtime (shader clock) and s_memrealtime (100 MHz) around its loop and records HW_REG_HW_ID and
// HW_REG_XCC_ID, so the host knows which SIMD each wave ran on. The rate of a SIMD is
//     (instructions of the waves that ran on it) / (last stamp out - first stamp in), in shader cycles,
// which does not depend on how the dispatcher spread the workgroups. Placement is reported beside it
// (how many SIMDs held exactly the requested number of waves). The launch is >= 50 ms, so the clock is the
// one the chip holds under sustained load (MI355X_MICROARCH.md "DVFS give-back").
//
// Cases (per loop iteration):
//   fma8        8 x v_fma_f32 (three VGPR sources), the round-3 form: 3 scalar loop instructions per 8 VALU
//   fma64       64 x v_fma_f32, three VGPR sources
//   fma64_k     64 x v_fma_f32, one VGPR source + inline constants
//   pk_fma64    64 x v_pk_fma_f32 (two fp32 FMAs per lane each)
//   add64_u32   64 x v_add_u32
//   mul24_64    64 x v_mul_u32_u24
//   fma64_salu16 64 x v_fma_f32 interleaved with 16 x s_mul_i32 (4 VALU : 1 SALU; no SCC write)
//   fma64_salu64 64 x v_fma_f32 interleaved with 64 x s_mul_i32 (1 : 1)
//   fma64_f64   64 x v_fma_f64
//
//   build: hipcc --offload-arch=gfx950 -O3 tools/valu_peak.hip -o tools/valu_peak
//   run:   ./tools/valu_peak [case|all] [waves,waves,...] [--ms MS]     (one JSON line per case and wave count)
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <map>
#include <string>
#include <vector>

#define CHK(x)                                                                                     \
    do {                                                                                           \
        hipError_t e_ = (x);                                                                       \
        if (e_ != hipSuccess) {                                                                    \
            fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_));      \
            exit(1);                                                                               \
        }                                                                                          \
    } while (0)

enum Case { FMA8, FMA64, FMA64_K, PK_FMA64, ADD64_U32, MUL24_64, FMA64_SALU16, FMA64_SALU64, FMA64_F64, NCASES };
static const char *kNames[NCASES] = {"fma8",     "fma64",        "fma64_k",      "pk_fma64", "add64_u32",
                                     "mul24_64", "fma64_salu16", "fma64_salu64", "fma64_f64"};
static const int kValuPerIter[NCASES] = {8, 64, 64, 64, 64, 64, 64, 64, 64};
static const int kSaluPerIter[NCASES] = {0, 0, 0, 0, 0, 0, 16, 64, 0};

// 16 instructions over the 16 chains %0..%15; X(i) is one instruction on chain i
#define R16(X) X(0) X(1) X(2) X(3) X(4) X(5) X(6) X(7) X(8) X(9) X(10) X(11) X(12) X(13) X(14) X(15)
#define FMA3(i) "v_fma_f32 %" #i ", %" #i ", %16, %17\n"
#define FMAK(i) "v_fma_f32 %" #i ", %" #i ", 0.5, 1.0\n"
#define PKFMA(i) "v_pk_fma_f32 %" #i ", %" #i ", %16, %17\n"
#define ADDU(i) "v_add_u32 %" #i ", %" #i ", %16\n"
#define MUL24(i) "v_mul_u32_u24 %" #i ", %" #i ", %16\n"
#define FMA_S(i) "v_fma_f32 %" #i ", %" #i ", %17, %18\n s_mul_i32 %16, %16, %19\n"
#define FMA_T(i) "v_fma_f32 %" #i ", %" #i ", %17, %18\n"
#define R16Q(X, Y) X(0) X(1) X(2) Y(3) X(4) X(5) X(6) Y(7) X(8) X(9) X(10) Y(11) X(12) X(13) X(14) Y(15)
#define FMAD(i) "v_fma_f64 %" #i ", %" #i ", %16, %17\n"

#define OUT16(T, a) "+v"(a[0]), "+v"(a[1]), "+v"(a[2]), "+v"(a[3]), "+v"(a[4]), "+v"(a[5]), "+v"(a[6]), \
    "+v"(a[7]), "+v"(a[8]), "+v"(a[9]), "+v"(a[10]), "+v"(a[11]), "+v"(a[12]), "+v"(a[13]), "+v"(a[14]), "+v"(a[15])

struct WaveRec {
    uint32_t hw_id, xcc_id, iters, pad;
    uint64_t t0, t1, r0, r1;
};

template <int C>
__global__ __launch_bounds__(256) void k_issue(float *out, WaveRec *rec, float seed, int iters) {
    float a[16];
    double d[16];
    uint32_t u[16];
    for (int i = 0; i < 16; i++) {
        a[i] = seed + threadIdx.x + i;
        d[i] = a[i];
        u[i] = threadIdx.x * 3u + i;
    }
    const float m = 0.999f, c = 0.001f;
    const double dm = 0.999, dc = 0.001;
    uint32_t s = blockIdx.x, sk = 3;
    uint32_t hw, xcc;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(hw));
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
    const uint64_t t0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
    for (int it = 0; it < iters; it++) {
        if (C == FMA8) {
            asm volatile("v_fma_f32 %0, %0, %8, %9\n v_fma_f32 %1, %1, %8, %9\n v_fma_f32 %2, %2, %8, %9\n"
                         " v_fma_f32 %3, %3, %8, %9\n v_fma_f32 %4, %4, %8, %9\n v_fma_f32 %5, %5, %8, %9\n"
                         " v_fma_f32 %6, %6, %8, %9\n v_fma_f32 %7, %7, %8, %9"
                         : "+v"(a[0]), "+v"(a[1]), "+v"(a[2]), "+v"(a[3]), "+v"(a[4]), "+v"(a[5]), "+v"(a[6]),
                           "+v"(a[7])
                         : "v"(m), "v"(c));
        } else if (C == FMA64) {
            asm volatile(R16(FMA3) R16(FMA3) R16(FMA3) R16(FMA3) : OUT16(float, a) : "v"(m), "v"(c));
        } else if (C == FMA64_K) {
            asm volatile(R16(FMAK) R16(FMAK) R16(FMAK) R16(FMAK) : OUT16(float, a));
        } else if (C == PK_FMA64) {
            // the 16 double registers hold fp32 pairs (two lanes of work per VGPR pair)
            asm volatile(R16(PKFMA) R16(PKFMA) R16(PKFMA) R16(PKFMA) : OUT16(double, d) : "v"(dm), "v"(dc));
        } else if (C == ADD64_U32) {
            asm volatile(R16(ADDU) R16(ADDU) R16(ADDU) R16(ADDU) : OUT16(uint32_t, u) : "v"(sk));
        } else if (C == MUL24_64) {
            asm volatile(R16(MUL24) R16(MUL24) R16(MUL24) R16(MUL24) : OUT16(uint32_t, u) : "v"(sk));
        } else if (C == FMA64_SALU16) { // one s_mul_i32 (no SCC) after every 4th v_fma_f32
            asm volatile(R16Q(FMA_T, FMA_S) R16Q(FMA_T, FMA_S) R16Q(FMA_T, FMA_S) R16Q(FMA_T, FMA_S)
                         : OUT16(float, a), "+s"(s)
                         : "v"(m), "v"(c), "s"(sk));
        } else if (C == FMA64_SALU64) {
            asm volatile(R16(FMA_S) R16(FMA_S) R16(FMA_S) R16(FMA_S) : OUT16(float, a), "+s"(s)
                         : "v"(m), "v"(c), "s"(sk));
        } else {
            asm volatile(R16(FMAD) R16(FMAD) R16(FMAD) R16(FMAD) : OUT16(double, d) : "v"(dm), "v"(dc));
        }
    }
    const uint64_t t1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
    const unsigned w = blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
    if ((threadIdx.x & 63) == 0) { // vector stores of the record (a buffer of its own)
        WaveRec r;
        r.hw_id = hw;
        r.xcc_id = xcc;
        r.iters = iters;
        r.pad = s;
        r.t0 = t0;
        r.t1 = t1;
        r.r0 = r0;
        r.r1 = r1;
        rec[w] = r;
    }
    float acc = 0;
    for (int i = 0; i < 16; i++) acc += a[i] + (float)d[i] + (float)u[i];
    out[blockIdx.x * blockDim.x + threadIdx.x] = acc;
}

typedef void (*KernelFn)(float *, WaveRec *, float, int);
static KernelFn kernel_of(int c) {
    switch (c) {
    case FMA8: return k_issue<FMA8>;
    case FMA64: return k_issue<FMA64>;
    case FMA64_K: return k_issue<FMA64_K>;
    case PK_FMA64: return k_issue<PK_FMA64>;
    case ADD64_U32: return k_issue<ADD64_U32>;
    case MUL24_64: return k_issue<MUL24_64>;
    case FMA64_SALU16: return k_issue<FMA64_SALU16>;
    case FMA64_SALU64: return k_issue<FMA64_SALU64>;
    default: return k_issue<FMA64_F64>;
    }
}

static float launch(int c, int blocks, float *d_out, WaveRec *d_rec, int iters, int reps) {
    hipEvent_t e0, e1;
    CHK(hipEventCreate(&e0));
    CHK(hipEventCreate(&e1));
    CHK(hipEventRecord(e0));
    for (int r = 0; r < reps; r++)
        hipLaunchKernelGGL(kernel_of(c), dim3(blocks), dim3(256), 0, 0, d_out, d_rec, 1.0f, iters);
    CHK(hipGetLastError());
    CHK(hipEventRecord(e1));
    CHK(hipEventSynchronize(e1));
    float ms = 0;
    CHK(hipEventElapsedTime(&ms, e0, e1));
    CHK(hipEventDestroy(e0));
    CHK(hipEventDestroy(e1));
    return ms / reps;
}

static double median(std::vector<double> v) {
    if (v.empty()) return 0;
    std::sort(v.begin(), v.end());
    return v[v.size() / 2];
}

static void run(int c, int cus, int waves_per_simd, double target_ms, float *d_out, WaveRec *d_rec) {
    const int blocks = cus * waves_per_simd; // 256-lane blocks = 4 waves
    int iters = 256;
    launch(c, blocks, d_out, d_rec, iters, 1);
    const float ms0 = launch(c, blocks, d_out, d_rec, iters, 1);
    iters = (int)std::min(1.0e9, iters * (target_ms / std::max(ms0, 1e-3f)));
    launch(c, blocks, d_out, d_rec, iters, 2); // sustained load before the measured launch
    const float ms = launch(c, blocks, d_out, d_rec, iters, 1);
    const int nw = blocks * 4;
    std::vector<WaveRec> rec(nw);
    CHK(hipMemcpy(rec.data(), d_rec, nw * sizeof(WaveRec), hipMemcpyDeviceToHost));
    // group the waves by SIMD: (xcc, se, sh, cu, simd) from HW_ID (gfx9 layout) and XCC_ID
    struct Simd {
        int waves = 0;
        uint64_t t0 = ~0ull, t1 = 0;
    };
    std::map<uint64_t, Simd> simds;
    std::vector<double> clk;
    for (const WaveRec &r : rec) {
        const uint32_t simd = (r.hw_id >> 4) & 3, cu = (r.hw_id >> 8) & 15, sh = (r.hw_id >> 12) & 1,
                       se = (r.hw_id >> 13) & 7, xcc = r.xcc_id & 15;
        const uint64_t key = ((uint64_t)xcc << 16) | (se << 8) | (sh << 6) | (cu << 2) | simd;
        Simd &s = simds[key];
        s.waves++;
        s.t0 = std::min(s.t0, r.t0);
        s.t1 = std::max(s.t1, r.t1);
        if (r.r1 > r.r0) clk.push_back(0.1 * (double)(r.t1 - r.t0) / (double)(r.r1 - r.r0));
    }
    const double per_wave = (double)iters * kValuPerIter[c];
    std::vector<double> rate_all, rate_exact;
    std::map<int, int> hist;
    for (auto &kv : simds) {
        const Simd &s = kv.second;
        const double r = s.waves * per_wave / (double)(s.t1 - s.t0);
        rate_all.push_back(r);
        if (s.waves == waves_per_simd) rate_exact.push_back(r);
        hist[s.waves]++;
    }
    const double ghz = median(clk);
    const double chip = (double)nw * per_wave / (ms * 1e-3) / (cus * 4.0) / (ghz * 1e9);
    std::string h;
    for (auto &kv : hist) h += (h.empty() ? "" : ", ") + std::string("\"") + std::to_string(kv.first) + "\": " + std::to_string(kv.second);
    printf("{\"case\": \"%s\", \"waves_per_simd\": %d, \"valu_per_iter\": %d, \"salu_per_iter\": %d, "
           "\"launch_ms\": %.2f, \"in_kernel_clock_ghz\": %.3f, \"simds_seen\": %zu, "
           "\"simds_by_resident_waves\": {%s}, "
           "\"per_simd_cycle_median\": %.4f, \"per_simd_cycle_median_exact_w\": %.4f, "
           "\"per_simd_cycle_chip\": %.4f, \"cycles_per_inst_per_wave\": %.3f}\n",
           kNames[c], waves_per_simd, kValuPerIter[c], kSaluPerIter[c], ms, ghz, simds.size(), h.c_str(),
           median(rate_all), median(rate_exact), chip,
           rate_exact.empty() ? 0.0 : waves_per_simd / median(rate_exact));
    fflush(stdout);
}

int main(int argc, char **argv) {
    std::vector<int> cases, waves = {1, 2, 3, 4, 5, 6, 8};
    double target_ms = 60;
    for (int i = 1; i < argc; i++) {
        if (!strcmp(argv[i], "--ms") && i + 1 < argc) {
            target_ms = atof(argv[++i]);
        } else if (argv[i][0] >= '0' && argv[i][0] <= '9') {
            waves.clear();
            for (char *p = strtok(argv[i], ","); p; p = strtok(nullptr, ",")) waves.push_back(atoi(p));
        } else if (strcmp(argv[i], "all")) {
            for (int c = 0; c < NCASES; c++)
                if (!strcmp(argv[i], kNames[c])) cases.push_back(c);
        }
    }
    if (cases.empty())
        for (int c = 0; c < NCASES; c++) cases.push_back(c);
    hipDeviceProp_t p;
    CHK(hipGetDeviceProperties(&p, 0));
    const int cus = p.multiProcessorCount;
    float *d_out;
    WaveRec *d_rec;
    CHK(hipMalloc(&d_out, (size_t)cus * 8 * 256 * sizeof(float)));
    CHK(hipMalloc(&d_rec, (size_t)cus * 8 * 4 * sizeof(WaveRec)));
    for (int c : cases)
        for (int w : waves) run(c, cus, w, target_ms, d_out, d_rec);
    printf("{\"cus\": %d, \"clock_khz\": %d}\n", cus, p.clockRate);
    return 0;
}
