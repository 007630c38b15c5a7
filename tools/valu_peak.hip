// valu_peak.hip -- measurement tool (not product code): the sustained VALU issue rate of gfx950 for the
// instruction kinds the fused COST kernel is made of, so that roofline.frac ("valu") has a measured peak
// next to the 2-cycles-per-wave64-instruction figure of MI355X_MICROARCH.md.
//
// Each kernel runs INDEP independent dependency chains per lane of one instruction kind, on every SIMD
// (grid = 8 workgroups of 256 threads per CU), for ITERS iterations.  Output per kernel: wave-instructions
// per SIMD per cycle at the in-kernel clock (s_memtime / s_memrealtime), and at 2.4 GHz wall.
//   hipcc --offload-arch=gfx950 -O3 -o valu_peak tools/valu_peak.hip && ./valu_peak
#include <hip/hip_runtime.h>

#include <cstdio>
#include <vector>

#define CHECK(x)                                                                        \
    do {                                                                                \
        hipError_t e_ = (x);                                                            \
        if (e_ != hipSuccess) {                                                         \
            fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
            return 1;                                                                   \
        }                                                                               \
    } while (0)

constexpr int ITERS = 4096;
constexpr int INDEP = 8;

__device__ unsigned long long g_clk[2];

template <int KIND>
__global__ void __launch_bounds__(256) chains(float* out, float a, float b) {
    float x[INDEP];
    float2 y[INDEP];
#pragma unroll
    for (int i = 0; i < INDEP; i++) {
        x[i] = (float)(threadIdx.x + i) * 1e-3f + 1.0f;
        y[i] = make_float2(x[i], x[i] + 0.5f);
    }
    unsigned long long t0 = 0, r0 = 0;
    if (blockIdx.x == 0 && threadIdx.x == 0) {
        t0 = __builtin_amdgcn_s_memtime();
        r0 = __builtin_amdgcn_s_memrealtime();
    }
    for (int it = 0; it < ITERS; it++) {
#pragma unroll
        for (int i = 0; i < INDEP; i++) {
            if constexpr (KIND == 0) {  // v_fma_f32
                x[i] = __builtin_fmaf(x[i], a, b);
            } else if constexpr (KIND == 1) {  // v_pk_fma_f32
                typedef float f2 __attribute__((ext_vector_type(2)));
                f2 v = {y[i].x, y[i].y};
                const f2 va = {a, a}, vb = {b, b};
                v = __builtin_elementwise_fma(v, va, vb);
                y[i] = make_float2(v.x, v.y);
            } else if constexpr (KIND == 2) {  // v_rcp_f32 (transcendental)
                x[i] = __builtin_amdgcn_rcpf(x[i]);
            } else if constexpr (KIND == 3) {  // v_add_u32 / integer
                unsigned v = __float_as_uint(x[i]);
                v = (v >> 1) + threadIdx.x;  // one v_lshr_add_u32
                x[i] = __int_as_float(v);
            } else if constexpr (KIND == 4) {  // IEEE division (the compiler's 10-11 instruction sequence)
                x[i] = x[i] / a + b;
            } else if constexpr (KIND == 5) {  // v_pk_mul_f32
                typedef float f2 __attribute__((ext_vector_type(2)));
                f2 v = {y[i].x, y[i].y};
                const f2 va = {a, b};
                v = v * va;
                y[i] = make_float2(v.x, v.y);
            } else if constexpr (KIND == 6) {  // v_lshl_add_u64 (64-bit address arithmetic)
                unsigned long long v = ((unsigned long long)__float_as_uint(y[i].x) << 32) | __float_as_uint(y[i].y);
                v = (v << 2) + (unsigned long long)(threadIdx.x + it);
                y[i] = make_float2(__uint_as_float((unsigned)(v >> 32)), __uint_as_float((unsigned)v));
            } else if constexpr (KIND == 7) {  // v_cvt_i32_f32 + v_cvt_f32_i32
                int v;
                asm volatile("v_cvt_i32_f32 %0, %1" : "=v"(v) : "v"(x[i]));
                x[i] = (float)v + a;
            } else if constexpr (KIND == 8) {  // v_pk_min_i16
                typedef short s2 __attribute__((ext_vector_type(2)));
                s2 v = __builtin_bit_cast(s2, __float_as_uint(x[i]));
                const s2 w = {(short)it, (short)(it + 1)};
                v = __builtin_elementwise_min(v, w);
                x[i] = __uint_as_float(__builtin_bit_cast(unsigned, v));
            } else if constexpr (KIND == 9) {  // v_cmp + v_cndmask
                x[i] = x[i] > a ? x[i] * b : x[i] + b;
            }
        }
    }
    if (blockIdx.x == 0 && threadIdx.x == 0) {
        g_clk[0] = __builtin_amdgcn_s_memtime() - t0;
        g_clk[1] = __builtin_amdgcn_s_memrealtime() - r0;
    }
    float s = 0.0f;
#pragma unroll
    for (int i = 0; i < INDEP; i++) s += x[i] + y[i].x + y[i].y;
    if (s == 12345.678f) out[threadIdx.x] = s;  // keep the chains alive
}

template <int KIND>
int run(const char* name, double instr_per_op, float* out, int cus) {
    hipEvent_t e0, e1;
    CHECK(hipEventCreate(&e0));
    CHECK(hipEventCreate(&e1));
    const int wgs = cus * 8;
    hipLaunchKernelGGL(chains<KIND>, dim3(wgs), dim3(256), 0, 0, out, 1.0001f, 0.5f);  // warm-up
    CHECK(hipDeviceSynchronize());
    CHECK(hipEventRecord(e0));
    const int reps = 5;
    for (int r = 0; r < reps; r++) hipLaunchKernelGGL(chains<KIND>, dim3(wgs), dim3(256), 0, 0, out, 1.0001f, 0.5f);
    CHECK(hipEventRecord(e1));
    CHECK(hipEventSynchronize(e1));
    float ms = 0.0f;
    CHECK(hipEventElapsedTime(&ms, e0, e1));
    unsigned long long clk[2];
    CHECK(hipMemcpyFromSymbol(clk, HIP_SYMBOL(g_clk), sizeof(clk)));
    const double ghz = (double)clk[0] / (double)clk[1] * 0.1;  // s_memrealtime runs at 100 MHz
    const double waves = (double)wgs * 4 * reps;
    const double instrs = waves * ITERS * INDEP * instr_per_op;
    const double per_simd = instrs / (cus * 4.0);
    const double secs = ms * 1e-3;
    printf("{\"kind\": \"%s\", \"ms\": %.3f, \"clock_ghz\": %.3f, \"instr_per_simd_cycle\": %.4f, "
           "\"instr_per_simd_cycle_at_2p4\": %.4f}\n",
           name, ms / reps, ghz, per_simd / (secs * ghz * 1e9), per_simd / (secs * 2.4e9));
    return 0;
}

int main() {
    hipDeviceProp_t p;
    CHECK(hipGetDeviceProperties(&p, 0));
    float* out;
    CHECK(hipMalloc(&out, 1024 * sizeof(float)));
    const int cus = p.multiProcessorCount;
    if (run<0>("v_fma_f32", 1, out, cus)) return 1;
    if (run<1>("v_pk_fma_f32", 1, out, cus)) return 1;
    if (run<2>("v_rcp_f32", 1, out, cus)) return 1;
    if (run<3>("v_lshrrev_b32 + v_add_u32", 2, out, cus)) return 1;
    if (run<4>("fdiv_ieee_plus_add (11.5 instr)", 11.5, out, cus)) return 1;
    if (run<5>("v_pk_mul_f32", 1, out, cus)) return 1;
    if (run<6>("v_lshl_add_u64 (+ v_add_co 2)", 3, out, cus)) return 1;
    if (run<7>("v_cvt_i32_f32 + v_cvt_f32_i32 + v_add", 3, out, cus)) return 1;
    if (run<8>("v_pk_min_i16", 1, out, cus)) return 1;
    if (run<9>("v_cmp + v_mul + v_add + v_cndmask", 4, out, cus)) return 1;
    CHECK(hipFree(out));
    return 0;
}
