// pcore_fdiv.h -- IEEE-exact f32 division for the fused COST kernel without the range-scaling steps, and the
// reference GPU's float -> int32 conversion as one instruction.
//
// hipcc expands every f32 `a / b` (no fast-math) into 11 instructions:
//   v_div_scale(b), v_rcp, fma, fma        -> r1, a refined reciprocal of b
//   v_div_scale(a), mul, fma, fma, fma     -> q1, e2
//   v_div_fmas(e2, r1, q1)                 -> fma, times 2^+-64 when div_scale scaled an operand
//   v_div_fixup(q, b, a)                   -> special cases (0, inf, NaN, over/underflow), sign
// On gfx950 that sequence costs ~44 SIMD cycles (tools/valu_peak.hip: 0.25 instr/SIMD-cycle against 0.47
// for plain FMAs; v_rcp alone is quarter rate), against ~2 per FMA.
//
// When the biased exponents of a and b lie in [87, 167] (|x| in [2^-40, 2^41)), v_div_scale returns both
// operands unchanged with VCC = 0 (exponent difference < 96, no denormal operand / reciprocal / quotient,
// numerator exponent > 23), v_div_fmas is then a plain fma, and v_div_fixup returns the fma result with
// its own (correct) sign.  The steps below are therefore the compiler's sequence minus the no-op steps, and
// the quotient is bit-identical to `a / b`, i.e. the correctly rounded IEEE quotient the CPU oracle
// computes.  Lanes outside that range take `a / b` itself in an exec-masked branch (skipped by the wave
// when no lane needs it), so every input -- zeros, denormals, infinities, NaNs -- keeps IEEE semantics.
// Two quotients with one denominator (the vertex stage's px / z and py / z) share r1.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace pcore {

__device__ __forceinline__ float recip_refined(float b) {
    const float r = __builtin_amdgcn_rcpf(b);
    const float e = __builtin_fmaf(-b, r, 1.0f);
    return __builtin_fmaf(e, r, r);
}

__device__ __forceinline__ float quot_refined(float a, float b, float r1) {
    const float q0 = a * r1;
    const float e1 = __builtin_fmaf(-b, q0, a);
    const float q1 = __builtin_fmaf(e1, r1, q0);
    const float e2 = __builtin_fmaf(-b, q1, a);
    return __builtin_fmaf(e2, r1, q1);
}

// biased exponent of x (8 bits)
__device__ __forceinline__ uint32_t fexp_bits(float x) { return (__float_as_uint(x) >> 23) & 0xffu; }

// every biased exponent in [87, 167]: the unscaled steps equal the IEEE expansion
__device__ __forceinline__ bool fdiv_range_ok(uint32_t emin, uint32_t emax) { return emin >= 87u && emax <= 167u; }

// a / b, IEEE-exact
__device__ __forceinline__ float fdiv_exact(float a, float b) {
    const uint32_t ea = fexp_bits(a), eb = fexp_bits(b);
    float q = quot_refined(a, b, recip_refined(b));
    if (!fdiv_range_ok(min(ea, eb), max(ea, eb))) {
        asm volatile("");
        q = a / b;
    }
    return q;
}

// int32_t(f) with NVIDIA cvt.rzi.s32.f32 semantics (image_renderer.cuh:129 on the reference's GPU): round toward
// zero, saturate to INT_MIN / INT_MAX, NaN -> 0.  v_cvt_i32_f32 implements exactly that (checked against the
// branchy restatement over special values and random bit patterns by tools/fdiv_check.hip), so the fragment
// test needs none of the compiler's range branches around a C++ conversion (undefined out of range).
__device__ __forceinline__ int32_t cvt_i32_rz_sat(float f) {
    int32_t r;
    asm("v_cvt_i32_f32 %0, %1" : "=v"(r) : "v"(f));
    return r;
}

// |x| as bits, with 0 mapped to 1.0f: a zero numerator is exact in the unscaled steps except for the sign of a
// zero quotient (-0 / b can come out +0), which only matters where noted
__device__ __forceinline__ uint32_t absbits_zero_as_one(float x) {
    const uint32_t u = __float_as_uint(x) & 0x7fffffffu;
    return u == 0u ? 0x3f800000u : u;
}
// every |x| (as bits, non-negative floats order like their bit patterns) in [2^-40, 2^41): the exponent range
// of fdiv_range_ok
__device__ __forceinline__ bool absbits_range_ok(uint32_t umin, uint32_t umax) {
    return umin >= (87u << 23) && umax < (168u << 23);
}

// The fragment depth of the reference (image_renderer.cuh:123-129) from its barycentrics and vertex depths, with IEEE
// divisions in the reference's order: int32_t((alpha + beta + gamma) / (alpha/z0 + beta/z1 + gamma/z2) + 0.5f).
__device__ __forceinline__ int32_t frag_depth_ieee(float alpha, float beta, float gamma, float z0, float z1, float z2) {
    const float ox = alpha / z0, oy = beta / z1, oz = gamma / z2;
    return cvt_i32_rz_sat((alpha + beta + gamma) / (ox + oy + oz) + 0.5f);
}

// frag_depth_ieee, bit for bit, mostly without divisions.  Precondition (what passes the reference's inside
// test): each of alpha, beta, gamma is in [-0, 1] or NaN.  The depth d(Q) = int(Q + 0.5) is monotone in the
// quotient Q of the IEEE chain.  With every z_i in [2^-100, 2^100] and no NaN, every term of the denominator is
// non-negative, so the chain through v_rcp_f32 (<= 1 ulp) and products has a relative error below 2^-20 against
// Q: 2^-22 per term (reciprocal, product and the IEEE quotient's own rounding), no cancellation in the two sums,
// then 2^-21 + 2^-23 + 2 * 2^-24 for the last quotient.  Q therefore lies in [f - e, f + e] with e = 2^-19 |f| (a
// factor-2 margin that also covers the rounding of f -/+ e), and where d(f - e) == d(f + e) that value is d(Q).
// Anywhere else -- a half-integer within e, depths out of range, a NaN -- the lane takes the IEEE divisions in an
// exec-masked branch.
// z_known_ok: the caller guarantees every z_i in [1, 2^41] (the fused kernel's pose-level bound), so only the
// NaN barycentric and the bracket are tested.
// active = false: the caller discards the result (a pixel outside the triangle), so the fallback is not taken.
__device__ __forceinline__ int32_t frag_depth_certified(float alpha, float beta, float gamma, float z0, float z1,
                                                        float z2, bool z_known_ok = false, bool active = true) {
    const float num = alpha + beta + gamma;
    const float oxa = alpha * __builtin_amdgcn_rcpf(z0), oya = beta * __builtin_amdgcn_rcpf(z1),
                oza = gamma * __builtin_amdgcn_rcpf(z2);
    const float f = num * __builtin_amdgcn_rcpf(oxa + oya + oza);
    const float e = fabsf(f) * 0x1p-19f;
    int32_t d = cvt_i32_rz_sat((f - e) + 0.5f);
    const int32_t dh = cvt_i32_rz_sat((f + e) + 0.5f);
    // fminf / fmaxf skip a NaN operand; a NaN depth makes zs NaN, a NaN barycentric makes num NaN
    bool z_ok = z_known_ok;
    if (!z_known_ok) {
        const float zmin = fminf(fminf(z0, z1), z2), zmax = fmaxf(fmaxf(z0, z1), z2), zs = z0 + z1 + z2;
        z_ok = zmin >= 0x1p-100f && zmax <= 0x1p100f && zs == zs;
    }
    if (active && (!z_ok || num != num || d != dh)) {
        asm volatile("");
        d = frag_depth_ieee(alpha, beta, gamma, z0, z1, z2);
    }
    return d;
}

// q0 = a0 / b, q1 = a1 / b, IEEE-exact
__device__ __forceinline__ void fdiv2_exact(float a0, float a1, float b, float& q0, float& q1) {
    const uint32_t e0 = fexp_bits(a0), e1 = fexp_bits(a1), eb = fexp_bits(b);
    const uint32_t emin = min(min(e0, e1), eb), emax = max(max(e0, e1), eb);
    const float r1 = recip_refined(b);
    q0 = quot_refined(a0, b, r1);
    q1 = quot_refined(a1, b, r1);
    if (!fdiv_range_ok(emin, emax)) {  // rare: zeros, tiny / huge values, inf, NaN
        asm volatile("");  // a side effect: keeps the compiler from speculating the division into every lane
        q0 = a0 / b;
        q1 = a1 / b;
    }
}

}  // namespace pcore
