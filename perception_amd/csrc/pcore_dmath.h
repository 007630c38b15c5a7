// pcore_dmath.h -- double-precision sin / cos with one fixed operation sequence, for the GICP step's
// SE(3) exponential (fast_gicp so3.hpp so3_exp / se3_exp; DESIGN.md "GICP spec").
//
// The GPU kernel and the CPU oracle must produce the same bits, and ROCm's ocml and glibc evaluate sin / cos
// differently, so the build owns its own: a three-part Cody-Waite reduction by pi/2 and the fdlibm kernel
// polynomials (__kernel_sin / __kernel_cos coefficients, as in musl's __sin.c / __cos.c), no tail word.  Within
// 1 ulp of numpy's sin / cos for |x| < 1e4 and 2 ulp up to 1e6, and within 1e-29 |x| absolute next to the
// functions' zeros (tests/test_gicp_spec.py); every finite input has a defined result, which is all the step needs
// from a huge argument.  Compiled with -ffp-contract=off on both sides.
#pragma once

#ifdef __HIPCC__
#define PCORE_DMH __host__ __device__ __forceinline__
#else
#include <math.h>
#define PCORE_DMH inline
#endif

namespace pcore {
namespace dmath {

// pi/2 in three pieces of 33 significant bits: n * kPio2_k is exact for |n| < 2^20
constexpr double kPio2_1 = 1.57079632673412561417e+00;
constexpr double kPio2_2 = 6.07710050630396597660e-11;
constexpr double kPio2_3 = 2.02226624871116645580e-21;
constexpr double kInvPio2 = 6.36619772367581382433e-01;

PCORE_DMH double ksin(double x) {  // |x| <= ~pi/4
    const double S1 = -1.66666666666666324348e-01, S2 = 8.33333333332248946124e-03,
                 S3 = -1.98412698298579493134e-04, S4 = 2.75573137070700676789e-06,
                 S5 = -2.50507602534068634195e-08, S6 = 1.58969099521155010221e-10;
    const double z = x * x;
    const double w = z * z;
    const double r = S2 + z * (S3 + z * S4) + z * w * (S5 + z * S6);
    const double v = z * x;
    return x + v * (S1 + z * r);
}

PCORE_DMH double kcos(double x) {  // |x| <= ~pi/4
    const double C1 = 4.16666666666666019037e-02, C2 = -1.38888888888741095749e-03,
                 C3 = 2.48015872894767294178e-05, C4 = -2.75573143513906633035e-07,
                 C5 = 2.08757232129817482790e-09, C6 = -1.13596475577881948265e-11;
    const double z = x * x;
    const double w = z * z;
    const double r = z * (C1 + z * (C2 + z * C3)) + w * w * (C4 + z * (C5 + z * C6));
    const double hz = 0.5 * z;
    const double u = 1.0 - hz;
    return u + (((1.0 - u) - hz) + z * r);
}

// sin (want_cos false) or cos of x
PCORE_DMH double sincos_d(double x, bool want_cos) {
    if (!(x - x == 0.0)) return x - x;  // NaN / inf -> NaN
    const double n = __builtin_rint(x * kInvPio2);
    const double r = ((x - n * kPio2_1) - n * kPio2_2) - n * kPio2_3;
    const double an = n < 0.0 ? -n : n;
    // quadrant n mod 4 (0 beyond 2^62, where the reduction means nothing anyway)
    long long q = an < 4.6116860184273879e18 ? (long long)an : 0;
    q &= 3;
    if (n < 0.0) q = (4 - q) & 3;
    if (want_cos) q = (q + 1) & 3;
    switch (q) {
        case 0: return ksin(r);
        case 1: return kcos(r);
        case 2: return -ksin(r);
        default: return -kcos(r);
    }
}

PCORE_DMH double sin_d(double x) { return sincos_d(x, false); }
PCORE_DMH double cos_d(double x) { return sincos_d(x, true); }

}  // namespace dmath
}  // namespace pcore
