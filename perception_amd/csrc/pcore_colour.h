// pcore_colour.h -- colour cost of cost_type 1: RGB -> CIE Lab and the CIEDE2000
// colour distance of compute_costs.cuh:57-159, as host + device code with one fixed arithmetic.
//
// The reference mixes float and double and calls the CUDA float transcendentals sqrtf / atan2f / fmodf
// / sinf / cosf / expf on double arguments (converted to float).  Those library functions are not
// bit-identical across CUDA, ROCm and glibc, so this build fixes its own: sqrtf / fmodf are the exact
// IEEE operations, and sin / cos / atan2 / exp are evaluated in double (Cody-Waite reduction +
// polynomial) and rounded to float -- the same operation sequence on the GPU and in the oracle
// (oracle/colour_spec.h), so the gate decisions match bit for bit.  Every float / double conversion of
// the reference expression is kept (see the comments in pc_colour_distance).
#pragma once

#include <math.h>
#include <stdint.h>

#ifdef __HIPCC__
#define PCORE_HD __host__ __device__ __forceinline__
#else
#define PCORE_HD inline
#endif

namespace pcore {
namespace colour {

constexpr double kPi = 3.14159265358979323846;
constexpr double kPio2Hi = 1.57079632673412561417e+00;  // pi/2 split: 33 significant bits + rest
constexpr double kPio2Lo = 6.07710050650619224932e-11;
constexpr double kLn2Hi = 6.93147180369123816490e-01;
constexpr double kLn2Lo = 1.90821492927058770002e-10;

PCORE_HD double poly_sin(double r) {  // |r| <= pi/4
    const double r2 = r * r;
    double p = -7.6471637318198164759e-13;
    p = p * r2 + 1.6059043836821614599e-10;
    p = p * r2 - 2.5052108385441718775e-08;
    p = p * r2 + 2.7557319223985890653e-06;
    p = p * r2 - 1.9841269841269841270e-04;
    p = p * r2 + 8.3333333333333333333e-03;
    p = p * r2 - 1.6666666666666666667e-01;
    return r + r * (r2 * p);
}

PCORE_HD double poly_cos(double r) {  // |r| <= pi/4
    const double r2 = r * r;
    double p = 4.7794773323873852974e-14;
    p = p * r2 - 1.1470745597729724714e-11;
    p = p * r2 + 2.0876756987868098979e-09;
    p = p * r2 - 2.7557319223985890653e-07;
    p = p * r2 + 2.4801587301587301587e-05;
    p = p * r2 - 1.3888888888888888889e-03;
    p = p * r2 + 4.1666666666666666667e-02;
    return 1.0 - 0.5 * r2 + r2 * (r2 * p);
}

// sin (want_cos = false) or cos of a float argument, |x| < 2^20
PCORE_HD float sincos_f(float xf, bool want_cos) {
    const double x = (double)xf;
    if (!(x == x) || x - x != 0.0) return (float)(x - x);  // NaN / inf -> NaN
    const double k = floor(x * 6.36619772367581382433e-01 + 0.5);
    const double r = (x - k * kPio2Hi) - k * kPio2Lo;
    int q = (int)(k - 4.0 * floor(k * 0.25));  // k mod 4 in [0, 4)
    if (want_cos) q = (q + 1) & 3;
    double v;
    switch (q) {
        case 0: v = poly_sin(r); break;
        case 1: v = poly_cos(r); break;
        case 2: v = -poly_sin(r); break;
        default: v = -poly_cos(r); break;
    }
    return (float)v;
}

PCORE_HD float sin_f(float x) { return sincos_f(x, false); }
PCORE_HD float cos_f(float x) { return sincos_f(x, true); }

PCORE_HD float exp_f(float xf) {
    const double x = (double)xf;
    if (!(x == x)) return xf;
    if (x > 89.0) return (float)INFINITY;
    if (x < -104.0) return 0.0f;
    const double k = floor(x * 1.44269504088896340736e+00 + 0.5);
    const double r = (x - k * kLn2Hi) - k * kLn2Lo;  // |r| <= 0.35
    double p = 1.0 / 479001600.0;                     // Taylor to r^12
    p = p * r + 1.0 / 39916800.0;
    p = p * r + 1.0 / 3628800.0;
    p = p * r + 1.0 / 362880.0;
    p = p * r + 1.0 / 40320.0;
    p = p * r + 1.0 / 5040.0;
    p = p * r + 1.0 / 720.0;
    p = p * r + 1.0 / 120.0;
    p = p * r + 1.0 / 24.0;
    p = p * r + 1.0 / 6.0;
    p = p * r + 0.5;
    p = p * r + 1.0;
    p = p * r + 1.0;
    return (float)ldexp(p, (int)k);
}

PCORE_HD double atan_01(double t) {  // 0 <= t <= 1
    // atan(t) = pi/6 + atan((sqrt(3) t - 1) / (t + sqrt(3))) above tan(pi/12)
    double base = 0.0;
    if (t > 2.67949192431122706473e-01) {
        t = (1.73205080756887729353 * t - 1.0) / (t + 1.73205080756887729353);
        base = kPi / 6.0;
    }
    const double t2 = t * t;  // |t| <= tan(pi/12): odd Taylor series to t^27
    double p = 1.0 / 27.0;
    p = -p * t2 + 1.0 / 25.0;
    p = -p * t2 + 1.0 / 23.0;
    p = -p * t2 + 1.0 / 21.0;
    p = -p * t2 + 1.0 / 19.0;
    p = -p * t2 + 1.0 / 17.0;
    p = -p * t2 + 1.0 / 15.0;
    p = -p * t2 + 1.0 / 13.0;
    p = -p * t2 + 1.0 / 11.0;
    p = -p * t2 + 1.0 / 9.0;
    p = -p * t2 + 1.0 / 7.0;
    p = -p * t2 + 1.0 / 5.0;
    p = -p * t2 + 1.0 / 3.0;
    p = -p * t2 + 1.0;
    return base + t * p;
}

// atan2 of float arguments with the IEEE special cases for zeros; finite inputs only (Lab values)
PCORE_HD float atan2_f(float yf, float xf) {
    const double y = (double)yf, x = (double)xf;
    if (!(y == y) || !(x == x)) return (float)(x + y);
    const bool yneg = signbit(yf), xneg = signbit(xf);
    if (y == 0.0) {
        const double a = xneg ? kPi : 0.0;
        return (float)(yneg ? -a : a);
    }
    if (x == 0.0) return (float)(yneg ? -kPi / 2.0 : kPi / 2.0);
    const double ay = fabs(y), ax = fabs(x);
    double a = ay <= ax ? atan_01(ay / ax) : kPi / 2.0 - atan_01(ax / ay);
    if (xneg) a = kPi - a;
    return (float)(yneg ? -a : a);
}

// fmodf of the reference's hue: x in [0, 4 pi), y = (float)(2 pi); exact (Sterbenz)
PCORE_HD float fmod_f(float x, float y) {
    float r = x;
    while (r >= y) r = r - y;
    return r;
}

PCORE_HD float sqrt_f(float x) { return sqrtf(x); }

// compute_costs.cuh:90-158, term by term with the reference's conversions
PCORE_HD double colour_distance(float l1, float a1, float b1, float l2, float a2, float b2) {
    const double eps = 1e-5;
    double c1 = sqrt_f(a1 * a1 + b1 * b1);
    double c2 = sqrt_f(a2 * a2 + b2 * b2);
    double meanC = (c1 + c2) / 2.0;
    double meanC7 = meanC * meanC * meanC * (meanC * meanC * meanC) * meanC;
    const double g = 0.5 * (1 - (double)sqrt_f((float)(meanC7 / (meanC7 + 6103515625.))));
    const double a1p = a1 * (1 + g);
    const double a2p = a2 * (1 + g);
    c1 = sqrt_f((float)(a1p * a1p + (double)(b1 * b1)));
    c2 = sqrt_f((float)(a2p * a2p + (double)(b2 * b2)));
    const float two_pi_f = (float)(2 * kPi);
    const double h1 = fmod_f((float)((double)atan2_f(b1, (float)a1p) + 2 * kPi), two_pi_f);
    const double h2 = fmod_f((float)((double)atan2_f(b2, (float)a2p) + 2 * kPi), two_pi_f);
    const double deltaL = (double)(l2 - l1);
    const double deltaC = c2 - c1;
    double deltah;
    if (fabs(h2 - h1) <= kPi) deltah = h2 - h1;
    else if (h2 > h1) deltah = h2 - h1 - 2 * kPi;
    else deltah = h2 - h1 + 2 * kPi;
    const double deltaH = (double)(2.0f * sqrt_f((float)(c1 * c2)) * sin_f((float)(deltah / 2)));
    const double meanL = (double)((l1 + l2) / 2);
    meanC = (c1 + c2) / 2.0;
    meanC7 = meanC * meanC * meanC * (meanC * meanC * meanC) * meanC;
    double meanH;
    if (fabs(h1 - h2) <= kPi + eps) meanH = (h1 + h2) / 2;
    else if (h1 + h2 < 2 * kPi) meanH = (h1 + h2 + 2 * kPi) / 2;
    else meanH = (h1 + h2 - 2 * kPi) / 2;
    const double T = 1 - 0.17 * (double)cos_f((float)(meanH - 30 * kPi / 180)) +
                     0.24 * (double)cos_f((float)(2 * meanH)) +
                     0.32 * (double)cos_f((float)(3 * meanH + 6 * kPi / 180)) -
                     0.2 * (double)cos_f((float)(4 * meanH - 63 * kPi / 180));
    const double dl = meanL - 50;
    const double sl = 1 + (0.015 * (dl * dl)) / (double)sqrt_f((float)(20 + dl * dl));
    const double sc = 1 + 0.045 * meanC;
    const double sh = 1 + 0.015 * meanC * T;
    const double rc = (double)(2.0f * sqrt_f((float)(meanC7 / (meanC7 + 6103515625.))));
    const double e = (meanH / kPi * 180 - 275) / 25;
    const float ex = exp_f((float)(-(e * e)));
    const double rt = (double)(-sin_f((float)((double)(60.0f * ex) * kPi / 180))) * rc;
    const double q1 = deltaL / sl, q2 = deltaC / sc, q3 = deltaH / sh;
    return (double)sqrt_f((float)(q1 * q1 + q2 * q2 + q3 * q3 + rt * deltaC / sc * deltaH / sh));
}

}  // namespace colour
}  // namespace pcore
