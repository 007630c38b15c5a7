// fdiv_check.hip -- checker (test infrastructure, not product code): pcore::fdiv2_exact (pcore_fdiv.h)
// against the compiler's IEEE f32 division `a / b`, bit for bit, on the GPU.
//
// Inputs: 2^26 pairs per launch from a counter-based hash, with exponents drawn over the whole f32 range
// (zeros, denormals, infinities and NaNs included) and a dense band around the [2^-40, 2^41) fast-path
// bounds, plus structured pairs (exact quotients, quotients near rounding ties: a = b * (1 + k ulp)).
// Also pcore::cvt_i32_rz_sat (one v_cvt_i32_f32) against the branchy NVIDIA-semantics conversion on special
// values and random bit patterns.
// And pcore::frag_depth_certified (the fused kernel's fragment depth through reciprocal estimates with an error
// certificate) against frag_depth_ieee on barycentrics that pass the reference's inside test and vertex depths
// over typical, tiny, huge, negative, zero, infinite and NaN values, including depths a few ulps from x.5.
// Prints one JSON line {"pairs": N, "mismatches": M, "fast_frac": F, "cvt_values": C, "cvt_mismatches": K,
// "frag_values": V, "frag_mismatches": X, "frag_certified_frac": G}; exit status 1 on any mismatch.
//   hipcc --offload-arch=gfx950 -O3 -ffp-contract=off -o tools/bin/fdiv_check tools/fdiv_check.hip
#include <hip/hip_runtime.h>

#include <cstdio>

#include "../perception_amd/csrc/pcore_fdiv.h"

#pragma clang fp contract(off)

__device__ __forceinline__ uint32_t mix(uint32_t x) {
    x ^= x >> 16; x *= 0x7feb352du; x ^= x >> 15; x *= 0x846ca68bu; x ^= x >> 16;
    return x;
}

__device__ __forceinline__ float draw(uint32_t h, uint32_t h2) {
    const uint32_t kind = h2 & 15u;
    uint32_t e;
    if (kind < 6) e = (h2 >> 4) & 0xffu;               // any exponent incl. 0 (denormal / zero) and 255
    else if (kind < 12) e = 80u + ((h2 >> 4) % 96u);   // dense band around the fast-path bounds 87..167
    else e = 120u + ((h2 >> 4) % 16u);                 // typical magnitudes (0.002 .. 500)
    uint32_t m = h & 0x7fffffu;
    if ((h2 >> 20) % 64u == 0) m = 0;                  // exact powers of two
    const uint32_t s = (h2 >> 31) << 31;
    return __uint_as_float(s | (e << 23) | m);
}

__global__ void check(uint32_t seed, unsigned long long* bad, unsigned long long* fast) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    const uint32_t h0 = mix(i * 4u + seed), h1 = mix(i * 4u + 1u + seed * 7u), h2 = mix(i * 4u + 2u + seed * 13u),
                   h3 = mix(i * 4u + 3u + seed * 31u);
    float a0 = draw(h0, h1), b = draw(h2, h3), a1 = draw(h1 ^ h3, h0 ^ h2);
    if ((h3 >> 8) % 8u == 0) {  // quotients near rounding ties: a = b * (1 + k ulp) and exact multiples
        const float q = draw(h1, h0 | 0xc00u);
        a0 = b * q;
        a1 = __uint_as_float(__float_as_uint(a0) + ((h3 >> 12) & 3u) - 1u);
    }
    float q0, q1;
    pcore::fdiv2_exact(a0, a1, b, q0, q1);
    const float r0 = a0 / b, r1 = a1 / b;
    const bool ok0 = __float_as_uint(q0) == __float_as_uint(r0) || (q0 != q0 && r0 != r0);
    const bool ok1 = __float_as_uint(q1) == __float_as_uint(r1) || (q1 != q1 && r1 != r1);
    if (!ok0 || !ok1) atomicAdd(bad, 1ull);
    const uint32_t e0 = pcore::fexp_bits(a0), e1 = pcore::fexp_bits(a1), eb = pcore::fexp_bits(b);
    if (pcore::fdiv_range_ok(min(min(e0, e1), eb), max(max(e0, e1), eb))) atomicAdd(fast, 1ull);
}

// reference semantics of cvt_i32_rz_sat (NVIDIA cvt.rzi.s32.f32), written out with branches
__device__ __forceinline__ int32_t cvt_ref(float f) {
    if (!(f == f)) return 0;
    if (f >= 2147483648.0f) return 2147483647;
    if (f <= -2147483648.0f) return (int32_t)0x80000000u;
    return (int32_t)f;
}

__global__ void check_cvt(uint32_t seed, unsigned long long* bad) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    const uint32_t h0 = mix(i * 2u + seed), h1 = mix(i * 2u + 1u + seed * 5u);
    float f = draw(h0, h1);
    if ((h1 >> 24) % 4u == 0) f = (float)(int32_t)h0 + (float)((h1 >> 8) & 3u) * 0.25f;  // near integers
    if (i < 8) {
        const float sp[8] = {__int_as_float(0x7fc00000), __int_as_float(0xffc00001), __int_as_float(0x7f800000),
                             __int_as_float(0xff800000), 2147483648.0f, -2147483648.0f, 2147483520.0f, -0.0f};
        f = sp[i];
    }
    if (pcore::cvt_i32_rz_sat(f) != cvt_ref(f)) atomicAdd(bad, 1ull);
}

__device__ __forceinline__ float depth_draw(uint32_t h, uint32_t h2) {
    const uint32_t kind = h2 % 32u;
    const float u = (float)(h >> 8) * 0x1p-24f;
    if (kind < 20) return 20.0f + 480.0f * u;                                      // typical cm depths
    if (kind < 24) return (float)(int)(20.0f + 480.0f * u) + 0.5f;                 // half-integers
    if (kind < 26) return -(20.0f + 480.0f * u);                                   // behind the camera
    if (kind < 28) return draw(h, h2 >> 5);                                        // any bit pattern
    const float sp[4] = {0.0f, __int_as_float(0x7f800000), 0x1p-110f, 0x1p110f};
    return sp[kind - 28];
}

__global__ void check_frag(uint32_t seed, unsigned long long* bad, unsigned long long* tested,
                           unsigned long long* certified) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    const uint32_t h0 = mix(i * 6u + seed), h1 = mix(i * 6u + 1u + seed * 3u), h2 = mix(i * 6u + 2u + seed * 5u),
                   h3 = mix(i * 6u + 3u + seed * 7u), h4 = mix(i * 6u + 4u + seed * 11u), h5 = mix(i * 6u + 5u + seed * 13u);
    // barycentrics as the fragment test forms them: beta, gamma, then alpha = 1 - beta - gamma
    float beta = (float)(h0 >> 8) * 0x1p-24f, gamma = (float)(h1 >> 8) * 0x1p-24f;
    const uint32_t bk = h5 % 64u;
    if (bk == 0) beta = 0.0f;
    else if (bk == 1) beta = -0.0f;
    else if (bk == 2) gamma = 0.0f;
    else if (bk == 3) beta = __int_as_float(0x7fc00000);  // a degenerate triangle's NaN
    else if (bk == 4) gamma = (float)(h1 >> 8) * 0x1p-60f;
    const float alpha = 1.0f - beta - gamma;
    if (alpha < -0.0f || beta < -0.0f || gamma < -0.0f || alpha > 1.0f || beta > 1.0f || gamma > 1.0f) return;
    float z0 = depth_draw(h2, h3), z1 = depth_draw(h3 ^ h4, h2 >> 3), z2 = depth_draw(h4, h2 ^ h3);
    if ((h5 >> 8) % 4u == 0) {  // one depth for all three vertices: Q = z, placed a few ulps from a half-integer
        const float half = (float)(int)(20.0f + 480.0f * ((float)(h4 >> 8) * 0x1p-24f)) + 0.5f;
        z0 = z1 = z2 = __uint_as_float(__float_as_uint(half) + ((h5 >> 12) & 7u) - 3u);
    }
    atomicAdd(tested, 1ull);
    const int32_t a = pcore::frag_depth_certified(alpha, beta, gamma, z0, z1, z2);
    const int32_t r = pcore::frag_depth_ieee(alpha, beta, gamma, z0, z1, z2);
    if (a != r) atomicAdd(bad, 1ull);
    // the certificate alone (no IEEE branch): typical depths, no NaN
    const float zmin = fminf(fminf(z0, z1), z2), zmax = fmaxf(fmaxf(z0, z1), z2);
    if (zmin >= 0x1p-100f && zmax <= 0x1p100f && beta == beta) {
        const float num = alpha + beta + gamma;
        const float f = num * __builtin_amdgcn_rcpf(alpha * __builtin_amdgcn_rcpf(z0) + beta * __builtin_amdgcn_rcpf(z1) +
                                                    gamma * __builtin_amdgcn_rcpf(z2));
        const float e = fabsf(f) * 0x1p-19f;
        if (pcore::cvt_i32_rz_sat((f - e) + 0.5f) == pcore::cvt_i32_rz_sat((f + e) + 0.5f)) atomicAdd(certified, 1ull);
    }
}

int main() {
    unsigned long long *d, h[6] = {0, 0, 0, 0, 0, 0};
    if (hipMalloc(&d, 48) != hipSuccess) return 2;
    if (hipMemset(d, 0, 48) != hipSuccess) return 2;
    const int launches = 16, blocks = 1 << 18, threads = 256;
    for (int l = 0; l < launches; l++) hipLaunchKernelGGL(check, dim3(blocks), dim3(threads), 0, 0, (uint32_t)l * 0x9e3779b9u, d, d + 1);
    for (int l = 0; l < 4; l++) hipLaunchKernelGGL(check_cvt, dim3(blocks), dim3(threads), 0, 0, (uint32_t)l * 0x85ebca6bu, d + 2);
    for (int l = 0; l < 16; l++)
        hipLaunchKernelGGL(check_frag, dim3(blocks), dim3(threads), 0, 0, (uint32_t)l * 0xc2b2ae35u, d + 3, d + 4, d + 5);
    if (hipDeviceSynchronize() != hipSuccess) return 2;
    if (hipMemcpy(h, d, 48, hipMemcpyDeviceToHost) != hipSuccess) return 2;
    const double pairs = 2.0 * launches * (double)blocks * threads;
    const double cvts = 4.0 * (double)blocks * threads;
    printf("{\"pairs\": %.0f, \"mismatches\": %llu, \"fast_frac\": %.4f, \"cvt_values\": %.0f, \"cvt_mismatches\": %llu, "
           "\"frag_values\": %llu, \"frag_mismatches\": %llu, \"frag_certified_frac\": %.4f}\n",
           pairs, h[0], 2.0 * h[1] / pairs, cvts, h[2], h[4], h[3], h[4] ? (double)h[5] / (double)h[4] : 0.0);
    return h[0] == 0 && h[2] == 0 && h[3] == 0 ? 0 : 1;
}
