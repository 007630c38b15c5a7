// exec_half.hip -- measurement tool (not product code): does a gfx950 wave64 VALU instruction cost less when
// EXEC leaves a 32-lane half empty?  GICP's lane-0 LM arithmetic (the 6x6 LDLT, se3_exp, the LM decisions) runs
// as uniform code on all 64 lanes; if an empty half is skipped, running it on lanes 0-31 (or lane 0) frees
// issue cycles for the other waves of the SIMD.
// Each kernel runs INDEP independent FMA chains (f32 or f64) per active lane, 8 workgroups of 256 threads per CU,
// with the chains executed under `lane < ACTIVE`.  Output: wave-instructions per SIMD per cycle.
//   hipcc --offload-arch=gfx950 -O3 -o tools/bin/exec_half tools/exec_half.hip && tools/bin/exec_half
#include <hip/hip_runtime.h>

#include <cstdio>

#define CHECK(x)                                                                                   \
    do {                                                                                           \
        hipError_t e_ = (x);                                                                       \
        if (e_ != hipSuccess) {                                                                    \
            fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_));      \
            return 1;                                                                              \
        }                                                                                          \
    } while (0)

constexpr int ITERS = 2048;
constexpr int INDEP = 8;

__device__ unsigned long long g_clk[2];

__device__ __forceinline__ float fma_t(float x, float a, float b) { return __builtin_fmaf(x, a, b); }
__device__ __forceinline__ double fma_t(double x, double a, double b) { return __builtin_fma(x, a, b); }

template <typename T, int ACTIVE>
__global__ void __launch_bounds__(256) chains(T* out, T a, T b) {
    const int lane = threadIdx.x & 63;
    T x[INDEP];
#pragma unroll
    for (int i = 0; i < INDEP; i++) x[i] = (T)(threadIdx.x + i) * (T)1e-3 + (T)1;
    unsigned long long t0 = 0, r0 = 0;
    if (blockIdx.x == 0 && threadIdx.x == 0) {
        t0 = __builtin_amdgcn_s_memtime();
        r0 = __builtin_amdgcn_s_memrealtime();
    }
    if (lane < ACTIVE) {
        for (int it = 0; it < ITERS; it++) {
#pragma unroll
            for (int i = 0; i < INDEP; i++) x[i] = fma_t(x[i], a, b);
        }
    }
    if (blockIdx.x == 0 && threadIdx.x == 0) {
        g_clk[0] = __builtin_amdgcn_s_memtime() - t0;
        g_clk[1] = __builtin_amdgcn_s_memrealtime() - r0;
    }
    T s = 0;
#pragma unroll
    for (int i = 0; i < INDEP; i++) s += x[i];
    if (s == (T)12345.678) out[threadIdx.x] = s;  // keep the chains alive
}

template <typename T, int ACTIVE>
int run(const char* name, T* out, int cus) {
    hipEvent_t e0, e1;
    CHECK(hipEventCreate(&e0));
    CHECK(hipEventCreate(&e1));
    const int wgs = cus * 8;
    hipLaunchKernelGGL((chains<T, ACTIVE>), dim3(wgs), dim3(256), 0, 0, out, (T)1.0001, (T)0.5);  // warm-up
    CHECK(hipDeviceSynchronize());
    CHECK(hipEventRecord(e0));
    const int reps = 5;
    for (int r = 0; r < reps; r++)
        hipLaunchKernelGGL((chains<T, ACTIVE>), dim3(wgs), dim3(256), 0, 0, out, (T)1.0001, (T)0.5);
    CHECK(hipEventRecord(e1));
    CHECK(hipEventSynchronize(e1));
    float ms = 0.0f;
    CHECK(hipEventElapsedTime(&ms, e0, e1));
    unsigned long long clk[2];
    CHECK(hipMemcpyFromSymbol(clk, HIP_SYMBOL(g_clk), sizeof(clk)));
    const double ghz = (double)clk[0] / (double)clk[1] * 0.1;  // s_memrealtime runs at 100 MHz
    const double waves = (double)wgs * 4 * reps;
    const double per_simd = waves * ITERS * INDEP / (cus * 4.0);
    const double secs = ms * 1e-3;
    printf("{\"kind\": \"%s\", \"active_lanes\": %d, \"ms\": %.3f, \"clock_ghz\": %.3f, "
           "\"wave_instr_per_simd_cycle\": %.4f, \"cycles_per_wave_instr\": %.2f}\n",
           name, ACTIVE, ms / reps, ghz, per_simd / (secs * ghz * 1e9), (secs * ghz * 1e9) / per_simd);
    return 0;
}

int main() {
    hipDeviceProp_t p;
    CHECK(hipGetDeviceProperties(&p, 0));
    void* out;
    CHECK(hipMalloc(&out, 1024 * sizeof(double)));
    const int cus = p.multiProcessorCount;
    if (run<float, 64>("v_fma_f32", (float*)out, cus)) return 1;
    if (run<float, 32>("v_fma_f32", (float*)out, cus)) return 1;
    if (run<float, 1>("v_fma_f32", (float*)out, cus)) return 1;
    if (run<double, 64>("v_fma_f64", (double*)out, cus)) return 1;
    if (run<double, 32>("v_fma_f64", (double*)out, cus)) return 1;
    if (run<double, 1>("v_fma_f64", (double*)out, cus)) return 1;
    CHECK(hipFree(out));
    return 0;
}
