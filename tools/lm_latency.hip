// lm_latency.hip -- measurement tool (not product code): shader clocks of the uniform pieces of one GICP LM step on
// gfx950, one wave per call chain, at 1 wave per CU (no contention) and at 3 waves per SIMD (gicp_kernel's occupancy).
// Pieces: gicpm::lm_solve_schur (the block / adjugate solve), gicpm::se3_exp + compose, and a chain of six dependent
// IEEE f64 divisions.  Every call's inputs come from LDS (as the 28 reduced sums do in gicp_kernel) and its result
// feeds the next call's damping, so calls do not overlap.  Round 5, the same box (profiles/r05c/lm_latency.txt), clocks
// per call at 1 / 12 waves per CU: the row-per-lane pivoted LDLT it replaced 4270 / 6141, lm_solve_schur 1198 / 1853;
// se3_exp + compose 1358 / 2071 unfused, 1305 / 1954 fused; six divisions 461 / 656.
//   hipcc --offload-arch=gfx950 -O2 -std=c++17 -ffp-contract=off -o tools/bin/lm_latency tools/lm_latency.hip
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "../perception_amd/csrc/pcore_gicp_math.h"

#pragma clang fp contract(off)

#define CHECK(x)                                                                              \
    do {                                                                                      \
        hipError_t e_ = (x);                                                                  \
        if (e_ != hipSuccess) {                                                               \
            fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
            return 1;                                                                         \
        }                                                                                     \
    } while (0)

using namespace pcore;

constexpr int kReps = 64;

__device__ __forceinline__ void wave_sync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

#define TD(v, dep)                                                                         \
    unsigned long long v;                                                                  \
    asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(v) : "v"(dep) : "memory")

template <int V>
__global__ void __launch_bounds__(64) lm_bench(const double* systems, int nsys, double* out,
                                               unsigned long long* clk) {
    __shared__ double s[gicpm::kTerms];
    __shared__ double sSe3[4 * gicpm::kSe3Terms];
    const int lane = threadIdx.x;
    if (lane < 4 * gicpm::kSe3Terms) sSe3[lane] = gicpm::kSe3Coef[lane];
    double acc = 0.0, lam_bias = 0.0;
    unsigned long long t = 0;
    for (int r = 0; r < kReps; r++) {
        const int k = (blockIdx.x * 7 + r) % nsys;
        wave_sync();
        if (lane < gicpm::kTerms) s[lane] = systems[(size_t)gicpm::kTerms * k + lane];
        wave_sync();
        const double lambda = 1e-9 * fabs(s[0]) + lam_bias;
        const double l0 = s[0] + lambda;
        TD(t0, l0);
        double d[6];
        if constexpr (V == 1) {
            gicpm::lm_solve_schur(s, lambda, d);
        } else if constexpr (V == 4) {
            double a6[6];
            for (int i = 0; i < 6; i++) a6[i] = s[21 + i] * 1e-3 + lambda;
            double Rd[3][3], td[3], R[3][3], tt[3], Ro[3][3], to[3];
            gicpm::se3_exp(a6, Rd, td, (__attribute__((address_space(3))) const double*)sSe3);
            for (int i = 0; i < 3; i++) {
                for (int j = 0; j < 3; j++) R[i][j] = i == j ? 1.0 : 1e-3;
                tt[i] = 0.1;
            }
            gicpm::compose(Rd, td, R, tt, Ro, to);
            for (int i = 0; i < 3; i++) d[i] = Ro[i][i];
            for (int i = 0; i < 3; i++) d[3 + i] = to[i];
        } else {
            double x = s[1] + l0;  // an LDS read after the first mark: the chain cannot start before it
            for (int i = 0; i < 6; i++) {
                x = 1.0 / x + 0.5;
                d[i] = x;
            }
        }
        TD(t1, d[5]);
        t += t1 - t0;
        acc += d[0] + d[5];
        lam_bias = d[5] * 1e-300;
    }
    if (lane == 0) {
        out[blockIdx.x] = acc;
        clk[blockIdx.x] = t;
    }
}

template <int V>
int run(const char* name, const double* d_sys, int nsys, double* d_out, unsigned long long* d_clk, int cus) {
    for (int per_cu : {1, 12}) {
        const int blocks = cus * per_cu;
        hipLaunchKernelGGL(lm_bench<V>, dim3(blocks), dim3(64), 0, 0, d_sys, nsys, d_out, d_clk);
        CHECK(hipGetLastError());
        CHECK(hipDeviceSynchronize());
        std::vector<unsigned long long> c(blocks);
        CHECK(hipMemcpy(c.data(), d_clk, sizeof(unsigned long long) * blocks, hipMemcpyDeviceToHost));
        double m = 0;
        for (auto v : c) m += (double)v;
        printf("%-28s waves/CU %2d: %8.0f clk per call\n", name, per_cu, m / blocks / kReps);
    }
    return 0;
}

int main() {
    int dev = 0, cus = 0;
    CHECK(hipGetDevice(&dev));
    CHECK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev));
    const int nsys = 512;
    std::vector<double> sys((size_t)nsys * gicpm::kTerms);
    srand(7);
    for (int k = 0; k < nsys; k++) {
        double A[6][6], H[6][6];
        for (int i = 0; i < 6; i++)
            for (int j = 0; j < 6; j++) A[i][j] = (rand() / (double)RAND_MAX - 0.5) * (i < 3 ? 10.0 : 1000.0);
        for (int i = 0; i < 6; i++)
            for (int j = 0; j < 6; j++) {
                H[i][j] = 0;
                for (int q = 0; q < 6; q++) H[i][j] += A[i][q] * A[j][q];
            }
        int h = 0;
        for (int i = 0; i < 6; i++)
            for (int j = i; j < 6; j++) sys[(size_t)gicpm::kTerms * k + h++] = H[i][j];
        for (int i = 0; i < 6; i++) sys[(size_t)gicpm::kTerms * k + 21 + i] = rand() / (double)RAND_MAX - 0.5;
        sys[(size_t)gicpm::kTerms * k + 27] = 1.0;
    }
    double *d_sys, *d_out;
    unsigned long long* d_clk;
    CHECK(hipMalloc(&d_sys, sizeof(double) * sys.size()));
    CHECK(hipMalloc(&d_out, sizeof(double) * cus * 12));
    CHECK(hipMalloc(&d_clk, sizeof(unsigned long long) * cus * 12));
    CHECK(hipMemcpy(d_sys, sys.data(), sizeof(double) * sys.size(), hipMemcpyHostToDevice));
    if (run<3>("6 dependent f64 divisions", d_sys, nsys, d_out, d_clk, cus)) return 1;
    if (run<1>("lm_solve_schur", d_sys, nsys, d_out, d_clk, cus)) return 1;
    if (run<4>("se3_exp + compose", d_sys, nsys, d_out, d_clk, cus)) return 1;
    return 0;
}
