// pcore_gicp_math.h -- the arithmetic of the GICP spec (DESIGN.md "GICP spec"): fast_gicp's published
// FastGICP / LsqRegistration algorithm with Levenberg-Marquardt step control, at the settings of the reference's
// call site (renderer.cu:1693-1720).  One set of functions compiled into both the HIP kernels (pcore_gicp.hip)
// and the CPU oracle's bit-exact GICP (oracle/pcore_oracle.cpp, orc_gicp), so the two evaluate the same
// double-precision expression trees bit for bit (both are built with -ffp-contract=off).  The oracle also holds an
// independent textbook restatement of the per-point step (4x4 homogeneous form, orc_gicp_linearize_textbook) that
// the tests hold this one to (tests/test_gicp_spec.py).
//
// Per source point (fast_gicp FastGICP::update_correspondences / linearize):
//   correspondence  the nearest target of q_f = T_f s (float transform, float arithmetic)
//   residual        e = t_j - q with q = T s in double
//   Mahalanobis     M = (C_t + R C_s R^T)^-1 (adjugate / determinant; RCR(3,3) = 1 and M(3,3) = 0 of the 4x4 form)
//   Jacobian        J = [skew(q) | -I]  =  [[0, -q2, q1, -1, 0, 0], [q2, 0, -q0, 0, -1, 0], [-q1, q0, 0, 0, 0, -1]]
//   terms           H += J^T M J (upper triangle), b += J^T M e, y += e^T M e
// The products with J's structural zeros and -1 entries are not evaluated: J^T v for a 3-vector v is
//   (q2 v1 - q1 v2, q0 v2 - q2 v0, q1 v0 - q0 v1, -v0, -v1, -v2).
// Per iteration (LsqRegistration::step_lm, so3.hpp se3_exp, Quaternion::toRotationMatrix):
//   lambda <- 1e-9 max|diag H| on the first iteration; up to 10 trials of d = (H + lambda I)^-1 (-b) (lm_solve_schur:
//   fast_gicp solves with Eigen's LDLT; the spec eliminates the translation block with 3x3 adjugates),
//   delta = se3_exp(d), x_i = delta x, y_i = sum e^T M e at x_i with the iteration's correspondences and M,
//   rho = (y - y_i) / d.(lambda d - b); rho < 0 rejects (stop if delta is converged, else lambda *= nu, nu *= 2),
//   otherwise x <- x_i and lambda *= max(1/3, 1 - (2 rho - 1)^3).  The search stops when a step is converged
//   (max(|dR - I| / rot_eps, |dt| / trans_eps) < 1), when ten trials are rejected, or after max_iter iterations.
#pragma once

#include "pcore_dmath.h"

#ifdef __HIPCC__
#define PCORE_GHD __host__ __device__ __forceinline__
#define PCORE_UNROLL _Pragma("unroll")
#else
#define PCORE_GHD inline
#define PCORE_UNROLL
#endif

namespace pcore {
namespace gicpm {

// Correspondence key (segments of at most kKeyScanMax targets; larger ones use the plain float squared distance
// and the exact grid search).  With the segment's origin c (float midpoint of its finite targets' bounding box),
// q' = q - c and t' = t - c, a target is stored as (-2 t'x, -2 t'y, -2 t'z, |t'|^2) and scored by
//   key = fma(-2 t'x, q'x, fma(-2 t'y, q'y, fma(-2 t'z, q'z, |t'|^2)))  =  |q' - t'|^2 - |q'|^2  (+ rounding),
// three FMAs instead of three subtractions, three products and two sums; |q'|^2 is the same for every target,
// so the nearest target is the first strict minimum of the key.  Centring keeps |q'|^2 small (objects are
// ~0.1 m across), so the cancellation costs ~1e-9 m^2 (tests/test_gicp_spec.py bounds the distance lost against
// the exact squared-distance argmin).  Non-finite targets never win (key +inf); a non-finite query has no
// correspondence.
constexpr int kKeyScanMax = 2048;

struct NNTarget {
    float m2x, m2y, m2z, tt;
};

PCORE_GHD NNTarget nn_target(float x, float y, float z, float cx, float cy, float cz) {
    if (!(__builtin_isfinite(x) && __builtin_isfinite(y) && __builtin_isfinite(z))) return {0.0f, 0.0f, 0.0f, __builtin_inff()};
    const float dx = x - cx, dy = y - cy, dz = z - cz;
    return {-2.0f * dx, -2.0f * dy, -2.0f * dz, __builtin_fmaf(dx, dx, __builtin_fmaf(dy, dy, dz * dz))};
}

PCORE_GHD float nn_key(float m2x, float m2y, float m2z, float tt, float qx, float qy, float qz) {
    return __builtin_fmaf(m2x, qx, __builtin_fmaf(m2y, qy, __builtin_fmaf(m2z, qz, tt)));
}

// the origin c of a segment: float midpoint of the bounding box of its finite targets (0 when there are none);
// get(i, p) fills p[3] with target i
template <class Get>
inline void nn_origin(int n, Get get, float (&c)[3]) {
    float lo[3] = {__builtin_inff(), __builtin_inff(), __builtin_inff()};
    float hi[3] = {-__builtin_inff(), -__builtin_inff(), -__builtin_inff()};
    bool any = false;
    for (int i = 0; i < n; i++) {
        float p[3];
        get(i, p);
        if (!(__builtin_isfinite(p[0]) && __builtin_isfinite(p[1]) && __builtin_isfinite(p[2]))) continue;
        any = true;
        for (int a = 0; a < 3; a++) {
            lo[a] = p[a] < lo[a] ? p[a] : lo[a];
            hi[a] = p[a] > hi[a] ? p[a] : hi[a];
        }
    }
    for (int a = 0; a < 3; a++) c[a] = any ? (lo[a] + hi[a]) * 0.5f : 0.0f;
}

// The correspondence query q_f = T_f s: the float transform (Rf, tf) = float(R, t) applied in float, row by row
// left to right (fast_gicp update_correspondences: trans.cast<float>() * point)
PCORE_GHD void query_f(const float (&Rf)[3][3], const float (&tf)[3], float sx, float sy, float sz, float (&qf)[3]) {
PCORE_UNROLL
    for (int r = 0; r < 3; r++) qf[r] = Rf[r][0] * sx + Rf[r][1] * sy + Rf[r][2] * sz + tf[r];
}

// Terms of the normal equations a point adds: acc[0..20] upper(J^T M J) row-major, acc[21..26] J^T M e,
// acc[27] e^T M e (the error y of step_lm).
constexpr int kTerms = 28;
constexpr int kErr = 27;
// index of H[a][a] in the upper triangle
PCORE_GHD constexpr int hdiag(int a) { return a * 6 - (a * (a - 1)) / 2; }

// Fused products (spec round 5): fma is correctly rounded on the GPU (v_fma_f64) and on the host (glibc fma), so the
// kernels and the oracle evaluate every expression built from these bit for bit.  The linearisation, the trials'
// errors, the damped solve, se3_exp and compose all use them: about 40 % fewer f64 instructions than separate
// products and sums, which is what the GICP kernel's VALU time is made of (f64: 57 % of its VALU cycles in round 4).
PCORE_GHD double fma_d(double a, double b, double c) { return __builtin_fma(a, b, c); }
// a0 b0 + a1 b1 + a2 b2 as fma(a0, b0, fma(a1, b1, a2 b2))
PCORE_GHD double dot3f(double a0, double a1, double a2, double b0, double b1, double b2) {
    return fma_d(a0, b0, fma_d(a1, b1, a2 * b2));
}

// Adjugate (upper: 00 01 02 11 12 22) and determinant of a symmetric 3x3 given by its upper triangle (same order)
PCORE_GHD void adj_sym3(const double (&m)[6], double (&a)[6], double& det) {
    a[0] = fma_d(m[3], m[5], -(m[4] * m[4]));
    a[1] = fma_d(m[2], m[4], -(m[1] * m[5]));
    a[2] = fma_d(m[1], m[4], -(m[2] * m[3]));
    a[3] = fma_d(m[0], m[5], -(m[2] * m[2]));
    a[4] = fma_d(m[1], m[2], -(m[0] * m[4]));
    a[5] = fma_d(m[0], m[3], -(m[1] * m[1]));
    det = dot3f(m[0], m[1], m[2], a[0], a[1], a[2]);
}


// Lane-parallel evaluation of a few uniform operations (device only).  The LM step is uniform work that every
// lane of the wave repeats; where it holds several independent IEEE divisions (se3_exp's three quotients) or
// several sin / cos, lane i evaluates the i-th one in a single
// instruction sequence and the results return through v_readlane.  Every lane still performs the same IEEE
// operation on the same operands as the scalar code, so the results are bit-identical to the host's (the oracle
// runs the scalar path).
#ifndef PCORE_SE3_LANE_SERIES
#define PCORE_SE3_LANE_SERIES 1  // se3_exp's four series on lanes 0..3: gicp_kernel -0.8..-1.7 % in 4 of 4 pairs (profiles/r06se/)
#endif
#if defined(__HIP_DEVICE_COMPILE__)
#define PCORE_LANE_PAR 1
__device__ __forceinline__ int lane_index() {
    return (int)__builtin_amdgcn_mbcnt_hi(~0u, __builtin_amdgcn_mbcnt_lo(~0u, 0u));
}
template <int LANE>
__device__ __forceinline__ double read_lane_d(double v) {
    const unsigned long long u = __builtin_bit_cast(unsigned long long, v);
    const unsigned lo = (unsigned)__builtin_amdgcn_readlane((int)(unsigned)u, LANE);
    const unsigned hi = (unsigned)__builtin_amdgcn_readlane((int)(unsigned)(u >> 32), LANE);
    return __builtin_bit_cast(double, ((unsigned long long)hi << 32) | lo);
}
// q[i] = num[i] / den[i] for i < N, one division sequence across lanes 0..N-1
template <int N>
__device__ __forceinline__ void lane_div(const double (&num)[N], const double (&den)[N], double (&q)[N]) {
    const int l = lane_index();
    double a = num[0], b = den[0];
PCORE_UNROLL
    for (int i = 1; i < N; i++) {
        a = l == i ? num[i] : a;
        b = l == i ? den[i] : b;
    }
    const double r = a / b;
    if constexpr (N > 0) q[0] = read_lane_d<0>(r);
    if constexpr (N > 1) q[1] = read_lane_d<1>(r);
    if constexpr (N > 2) q[2] = read_lane_d<2>(r);
    if constexpr (N > 3) q[3] = read_lane_d<3>(r);
    if constexpr (N > 4) q[4] = read_lane_d<4>(r);
    if constexpr (N > 5) q[5] = read_lane_d<5>(r);
}
#else
#define PCORE_LANE_PAR 0
#endif

// q = R s + t row by row, fused: the transformed source point of the linearisation and of the trials' errors
PCORE_GHD void transform_point(const double (&R)[3][3], const double (&t)[3], double s0, double s1, double s2,
                               double (&q)[3]) {
PCORE_UNROLL
    for (int r = 0; r < 3; r++) q[r] = fma_d(R[r][0], s0, fma_d(R[r][1], s1, fma_d(R[r][2], s2, t[r])));
}

// y + e^T M e with M given by its upper triangle (xx, xy, xz, yy, yz, zz): Me row by row (dot3f), then
// fma(e0, Me0, fma(e1, Me1, fma(e2, Me2, y))).  The linearisation's error term (contrib) and the trials' errors use
// this one expression, so a trial at the linearisation point reproduces its error bit for bit.
PCORE_GHD double mahal_err_add(const double (&M6)[6], const double (&e)[3], double y) {
    const double me0 = dot3f(M6[0], M6[1], M6[2], e[0], e[1], e[2]);
    const double me1 = dot3f(M6[1], M6[3], M6[4], e[0], e[1], e[2]);
    const double me2 = dot3f(M6[2], M6[4], M6[5], e[0], e[1], e[2]);
    return fma_d(e[0], me0, fma_d(e[1], me1, fma_d(e[2], me2, y)));
}

// M = (C_t + R C_s R^T)^-1 of one point (xx, xy, xz, yy, yz, zz), contrib's first half: row r of R C_s, then row r
// of A = C_t + (R C_s) R^T with C_t as the innermost addend (only one row of R C_s is live at a time); the adjugate
// and determinant of the symmetric A (adj_sym3) and M = adj(A) * (1 / det)
PCORE_GHD void mahal_matrix(const double (&R)[3][3], const double (&cs)[6], const double (&ct)[6], double (&M6)[6]) {
    constexpr int S3[3][3] = {{0, 1, 2}, {1, 3, 4}, {2, 4, 5}};
    double A[6];
PCORE_UNROLL
    for (int r = 0; r < 3; r++) {
        double RC[3];
PCORE_UNROLL
        for (int c = 0; c < 3; c++) RC[c] = dot3f(R[r][0], R[r][1], R[r][2], cs[S3[0][c]], cs[S3[1][c]], cs[S3[2][c]]);
PCORE_UNROLL
        for (int c = r; c < 3; c++)
            A[S3[r][c]] = fma_d(RC[0], R[c][0], fma_d(RC[1], R[c][1], fma_d(RC[2], R[c][2], ct[S3[r][c]])));
    }
    double adj[6], det;
    adj_sym3(A, adj, det);
    const double inv = 1.0 / det;
PCORE_UNROLL
    for (int k = 0; k < 6; k++) M6[k] = adj[k] * inv;
}

// One point's contribution for the transformed point q (double), its correspondence tj and both covariances
// (xx, xy, xz, yy, yz, zz); M6 receives the point's Mahalanobis matrix (kept for the trials' errors).
// H[a][b] (a <= b) column by column: column b of M J as a 3-vector cb (b < 3: the skew part, one fma and one product
// per entry; b >= 3: -M's column), then for every a <= b the J^T row a against cb fused into the sum:
// acc = fma(q2, cb1, fma(-q1, cb2, acc)) for a = 0 (and the cyclic forms for a = 1, 2), acc - cb[a - 3] for a >= 3.
// Each sum takes one term per point, so the column order of the updates changes no sum, and only one column is live
// at a time.  b += J^T M e the same way, y by mahal_err_add.
PCORE_GHD void contrib(const double (&R)[3][3], const double (&q)[3], const double (&cs)[6], const double (&tj)[3],
                       const double (&ct)[6], double (&acc)[kTerms], double (&M6)[6]) {
    mahal_matrix(R, cs, ct, M6);
    const double M[3][3] = {{M6[0], M6[1], M6[2]}, {M6[1], M6[3], M6[4]}, {M6[2], M6[4], M6[5]}};
    const double e[3] = {tj[0] - q[0], tj[1] - q[1], tj[2] - q[2]};
    // J^T row a (a < 3) against v, fused into the sum s
    auto jt_add = [&](int a, const double (&v)[3], double sum) {
        return a == 0 ? fma_d(q[2], v[1], fma_d(-q[1], v[2], sum))
             : a == 1 ? fma_d(q[0], v[2], fma_d(-q[2], v[0], sum))
                      : fma_d(q[1], v[0], fma_d(-q[0], v[1], sum));
    };
PCORE_UNROLL
    for (int b = 0; b < 6; b++) {
        double cb[3];
PCORE_UNROLL
        for (int r = 0; r < 3; r++) {
            if (b == 0) cb[r] = fma_d(M[r][1], q[2], -(M[r][2] * q[1]));
            else if (b == 1) cb[r] = fma_d(M[r][2], q[0], -(M[r][0] * q[2]));
            else if (b == 2) cb[r] = fma_d(M[r][0], q[1], -(M[r][1] * q[0]));
            else cb[r] = -M[r][b - 3];
        }
PCORE_UNROLL
        for (int a = 0; a <= b; a++) {
            double& h = acc[hdiag(a) + b - a];
            h = a < 3 ? jt_add(a, cb, h) : h - cb[a - 3];
        }
    }
    double Me[3];
PCORE_UNROLL
    for (int r = 0; r < 3; r++) Me[r] = dot3f(M[r][0], M[r][1], M[r][2], e[0], e[1], e[2]);
PCORE_UNROLL
    for (int a = 0; a < 3; a++) acc[21 + a] = jt_add(a, Me, acc[21 + a]);
PCORE_UNROLL
    for (int a = 3; a < 6; a++) acc[21 + a] = acc[21 + a] - Me[a - 3];
    acc[kErr] = mahal_err_add(M6, e, acc[kErr]);
}

// ---- the step (uniform per pose) ----------------------------------------------------------------------------

constexpr int kLmMaxTrials = 10;          // LsqRegistration lm_max_iterations_
constexpr double kLmInitFactor = 1e-9;    // LsqRegistration lm_init_lambda_factor_

// initial damping: 1e-9 * max |H_aa| (maxCoeff: the first strict maximum in index order)
PCORE_GHD double lm_init_lambda(const double* sys) {
    double m = __builtin_fabs(sys[hdiag(0)]);
PCORE_UNROLL
    for (int a = 1; a < 6; a++) {
        const double v = __builtin_fabs(sys[hdiag(a)]);
        m = v > m ? v : m;
    }
    return kLmInitFactor * m;
}

// d = (H + lambda I)^-1 (-b) by the 3x3 block elimination of the translation block: with
// H = [[A, B], [B^T, C]] (A rotation, C translation, both + lambda I) and r = -b,
//   adj(C), det(C) = dC;  P = B adj(C);  S~ = dC A - P B^T (= dC times the Schur complement, upper triangle);
//   u~ = dC r_rot - P r_trans;  x_rot = adj(S~) u~ / det(S~);  x_trans = adj(C) (r_trans - B^T x_rot) / dC,
// the 3-term sums as fma chains (dot3f).  H + lambda I is positive definite whenever it is not zero (H is a sum of
// J^T M J with M positive definite, lambda = 1e-9 max|H_aa| > 0 unless H = 0): a zero diagonal gives d = 0 (Eigen's
// LDLT of the zero matrix); a non-finite system gives a non-finite d, which stops the pose (lm_iteration's guard).
// The dependent chain is two adjugates, two 3-term products and two divisions deep, against the LDLT's six pivot steps.
// On the device the wave holds one system (every lane the same), so each group of three quotients runs as one division
// sequence on lanes 0..2 (lane_div): the same IEEE divisions as the host's.
PCORE_GHD void lm_solve_schur(const double* sys, double lambda, double (&d)[6]) {
    // upper triangles (00 01 02 11 12 22) of the rotation block A and the translation block C, + lambda on the diagonal
    const double A[6] = {sys[0] + lambda, sys[1], sys[2], sys[6] + lambda, sys[7], sys[11] + lambda};
    const double C[6] = {sys[15] + lambda, sys[16], sys[17], sys[18] + lambda, sys[19], sys[20] + lambda};
    // B[i][j] = H[i][3 + j]
    const double B00 = sys[3], B01 = sys[4], B02 = sys[5];
    const double B10 = sys[8], B11 = sys[9], B12 = sys[10];
    const double B20 = sys[12], B21 = sys[13], B22 = sys[14];
    const double r0 = -sys[21], r1 = -sys[22], r2 = -sys[23], r3 = -sys[24], r4 = -sys[25], r5 = -sys[26];
    if (A[0] == 0.0 && A[3] == 0.0 && A[5] == 0.0 && C[0] == 0.0 && C[3] == 0.0 && C[5] == 0.0) {
PCORE_UNROLL
        for (int i = 0; i < 6; i++) d[i] = 0.0;  // the zero system
        return;
    }
    double aC[6], dC;
    adj_sym3(C, aC, dC);
    // P = B adj(C) (adj(C) symmetric: column j = (aC[j0], aC[j1], aC[j2]))
    const double P00 = dot3f(B00, B01, B02, aC[0], aC[1], aC[2]);
    const double P01 = dot3f(B00, B01, B02, aC[1], aC[3], aC[4]);
    const double P02 = dot3f(B00, B01, B02, aC[2], aC[4], aC[5]);
    const double P10 = dot3f(B10, B11, B12, aC[0], aC[1], aC[2]);
    const double P11 = dot3f(B10, B11, B12, aC[1], aC[3], aC[4]);
    const double P12 = dot3f(B10, B11, B12, aC[2], aC[4], aC[5]);
    const double P20 = dot3f(B20, B21, B22, aC[0], aC[1], aC[2]);
    const double P21 = dot3f(B20, B21, B22, aC[1], aC[3], aC[4]);
    const double P22 = dot3f(B20, B21, B22, aC[2], aC[4], aC[5]);
    // S~ = dC A - P B^T (upper), u~ = dC r_rot - P r_trans
    const double St[6] = {fma_d(dC, A[0], -dot3f(P00, P01, P02, B00, B01, B02)),
                          fma_d(dC, A[1], -dot3f(P00, P01, P02, B10, B11, B12)),
                          fma_d(dC, A[2], -dot3f(P00, P01, P02, B20, B21, B22)),
                          fma_d(dC, A[3], -dot3f(P10, P11, P12, B10, B11, B12)),
                          fma_d(dC, A[4], -dot3f(P10, P11, P12, B20, B21, B22)),
                          fma_d(dC, A[5], -dot3f(P20, P21, P22, B20, B21, B22))};
    const double u0 = fma_d(dC, r0, -dot3f(P00, P01, P02, r3, r4, r5));
    const double u1 = fma_d(dC, r1, -dot3f(P10, P11, P12, r3, r4, r5));
    const double u2 = fma_d(dC, r2, -dot3f(P20, P21, P22, r3, r4, r5));
    double aS[6], dS;
    adj_sym3(St, aS, dS);
    const double nx[3] = {dot3f(aS[0], aS[1], aS[2], u0, u1, u2), dot3f(aS[1], aS[3], aS[4], u0, u1, u2),
                          dot3f(aS[2], aS[4], aS[5], u0, u1, u2)};
    double x[3];
#if PCORE_LANE_PAR
    // the wave holds one system: the three quotients on lanes 0..2 in one division sequence (the same IEEE divisions)
    const double dSv[3] = {dS, dS, dS};
    lane_div<3>(nx, dSv, x);
#else
    for (int i = 0; i < 3; i++) x[i] = nx[i] / dS;
#endif
    // w = r_trans - B^T x_rot
    const double w0 = r3 - dot3f(B00, B10, B20, x[0], x[1], x[2]);
    const double w1 = r4 - dot3f(B01, B11, B21, x[0], x[1], x[2]);
    const double w2 = r5 - dot3f(B02, B12, B22, x[0], x[1], x[2]);
    d[0] = x[0];
    d[1] = x[1];
    d[2] = x[2];
    const double nt[3] = {dot3f(aC[0], aC[1], aC[2], w0, w1, w2), dot3f(aC[1], aC[3], aC[4], w0, w1, w2),
                          dot3f(aC[2], aC[4], aC[5], w0, w1, w2)};
#if PCORE_LANE_PAR
    const double dCv[3] = {dC, dC, dC};
    double y[3];
    lane_div<3>(nt, dCv, y);
    d[3] = y[0];
    d[4] = y[1];
    d[5] = y[2];
#else
    for (int i = 0; i < 3; i++) d[3 + i] = nt[i] / dC;
#endif
}

// se3_exp's four functions of theta as even power series in u = theta^2 (Horner, fused), used below theta^2 = 1/4:
//   imag = sin(theta / 2) / theta = sum (-1)^k u^k / (2^(2k+1) (2k+1)!)     real = cos(theta / 2) = sum (-1)^k u^k / (2^(2k) (2k)!)
//   c1 = (1 - cos theta) / theta^2 = sum (-1)^k u^k / (2k+2)!               c2 = (theta - sin theta) / theta^3 = sum (-1)^k u^k / (2k+3)!
// Eight terms: below u = 1/4 the first omitted one is < 1e-17 of the sum.  The coefficients are the doubles nearest
// the exact rationals.  (so3_exp's own Taylor branch below theta^2 = 1e-10 is the first two terms of imag / real.)
constexpr int kSe3Terms = 8;
constexpr double kSe3SeriesMax = 0.25;
// The coefficients interleaved by power: kSe3Coef[4 k + f] is the coefficient of u^k of imag, real, c1, c2 (f = 0..3)
constexpr double kSe3Coef[4 * kSe3Terms] = {
    0.5, 1.0, 0.5, 0.16666666666666666,
    -0.020833333333333332, -0.125, -0.041666666666666664, -0.008333333333333333,
    0.00026041666666666666, 0.0026041666666666665, 0.001388888888888889, 0.0001984126984126984,
    -1.5500992063492063e-06, -2.170138888888889e-05, -2.48015873015873e-05, -2.7557319223985893e-06,
    5.382288910934745e-09, 9.68812003968254e-08, 2.755731922398589e-07, 2.505210838544172e-08,
    -1.2232474797578965e-11, -2.691144455467372e-10, -2.08767569878681e-09, -1.6059043836821613e-10,
    1.9603324996120133e-14, 5.096864498991235e-13, 1.1470745597729725e-11, 7.647163731819816e-13,
    -2.333729166204778e-17, -7.001187498614334e-16, -4.779477332387385e-14, -2.8114572543455206e-15};
// The four series by Horner in u, one power at a time for all four (four independent chains; the kernels' LDS copy
// is then read as two 16-byte loads per power, all issued ahead of the chain).  The kernels pass a pointer into an
// LDS copy of kSe3Coef whose address they make opaque inside the iteration loop (as 32 literal doubles the constants
// were hoisted out of it into 64 VGPRs for the whole kernel; read through a volatile pointer each load waited on
// its own before the next, 32 LDS round trips in a row); the host passes kSe3Coef.
template <typename P>
PCORE_GHD void se3_series(P c, double u, double (&out)[4]) {
#if PCORE_LANE_PAR && PCORE_SE3_LANE_SERIES
    // the wave holds one step: series f on lane f & 3 (its coefficients read per lane), the four results by v_readlane
    const int f = lane_index() & 3;
    double v = c[4 * (kSe3Terms - 1) + f];
PCORE_UNROLL
    for (int k = kSe3Terms - 2; k >= 0; k--) v = fma_d(v, u, c[4 * k + f]);
    out[0] = read_lane_d<0>(v);
    out[1] = read_lane_d<1>(v);
    out[2] = read_lane_d<2>(v);
    out[3] = read_lane_d<3>(v);
#else
PCORE_UNROLL
    for (int f = 0; f < 4; f++) out[f] = c[4 * (kSe3Terms - 1) + f];
PCORE_UNROLL
    for (int k = kSe3Terms - 2; k >= 0; k--)
PCORE_UNROLL
        for (int f = 0; f < 4; f++) out[f] = fma_d(out[f], u, c[4 * k + f]);
#endif
}

// se3_exp (fast_gicp so3.hpp): so3_exp's quaternion (imag = sin(theta/2)/theta, real = cos(theta/2)), Eigen's
// Quaternion::toRotationMatrix, translation V rho with V = I + c1 Omega + c2 Omega^2, c1 = (1 - cos theta)/theta^2,
// c2 = (theta - sin theta)/theta^3 (V = the rotation below theta = 1e-10, as published: here theta^2 < 1e-20), formed
// without V as rho + c1 (omega x rho) + c2 (omega x (omega x rho)) (Omega v = omega x v); products and sums fused
// (fma_d / dot3f).  Below theta^2 = 1/4 -- nearly every LM step -- imag, real, c1 and c2 are the power series above:
// no square root, no sin / cos, no division, and no cancellation in 1 - cos theta or theta - sin theta (the published
// quotients lose ~eps / theta^2 of relative accuracy there).  Larger steps take the published quotients; WAVE: every
// lane holds the same step, so their four sin / cos and three divisions run lane-parallel (lane_div).
template <bool WAVE = (PCORE_LANE_PAR != 0), typename P = const double*>
PCORE_GHD void se3_exp(const double (&a)[6], double (&Rd)[3][3], double (&td)[3], P coef) {
    const double w0 = a[0], w1 = a[1], w2 = a[2];
    const double theta_sq = dot3f(w0, w1, w2, w0, w1, w2);
    double imag, real, c1, c2;
    if (theta_sq < kSe3SeriesMax) {
        double fs[4];
        se3_series(coef, theta_sq, fs);
        imag = fs[0];
        real = fs[1];
        c1 = fs[2];
        c2 = fs[3];
    } else {
        const double theta = __builtin_sqrt(theta_sq);
        const double half_theta = 0.5 * theta;
        const double th2 = theta * theta;
#if PCORE_LANE_PAR
        if constexpr (WAVE) {
            // the four sin / cos on lanes 0..3 and the three quotients on lanes 0..2, one sequence each (same values)
            const int l = lane_index();
            const double tv = dmath::sincos_d(l < 2 ? half_theta : theta, (l & 1) != 0);
            const double sin_h = read_lane_d<0>(tv), cos_h = read_lane_d<1>(tv);
            const double sin_t = read_lane_d<2>(tv), cos_t = read_lane_d<3>(tv);
            const double num[3] = {sin_h, 1.0 - cos_t, theta - sin_t}, den[3] = {theta, th2, th2 * theta};
            double quo[3];
            lane_div<3>(num, den, quo);
            imag = quo[0];
            real = cos_h;
            c1 = quo[1];
            c2 = quo[2];
        } else
#endif
        {
            imag = dmath::sin_d(half_theta) / theta;
            real = dmath::cos_d(half_theta);
            c1 = (1.0 - dmath::cos_d(theta)) / th2;
            c2 = (theta - dmath::sin_d(theta)) / (th2 * theta);
        }
    }
    const double qw = real, qx = imag * w0, qy = imag * w1, qz = imag * w2;
    const double tx = 2.0 * qx, ty = 2.0 * qy, tz = 2.0 * qz;
    Rd[0][0] = 1.0 - fma_d(ty, qy, tz * qz);
    Rd[0][1] = fma_d(ty, qx, -(tz * qw));
    Rd[0][2] = fma_d(tz, qx, ty * qw);
    Rd[1][0] = fma_d(ty, qx, tz * qw);
    Rd[1][1] = 1.0 - fma_d(tx, qx, tz * qz);
    Rd[1][2] = fma_d(tz, qy, -(tx * qw));
    Rd[2][0] = fma_d(tz, qx, -(ty * qw));
    Rd[2][1] = fma_d(tz, qy, tx * qw);
    Rd[2][2] = 1.0 - fma_d(tx, qx, ty * qy);
    const double r0 = a[3], r1 = a[4], r2 = a[5];
    if (theta_sq < 1e-20) {
PCORE_UNROLL
        for (int r = 0; r < 3; r++) td[r] = dot3f(Rd[r][0], Rd[r][1], Rd[r][2], r0, r1, r2);
    } else {
        const double a0 = fma_d(w1, r2, -(w2 * r1)), a1 = fma_d(w2, r0, -(w0 * r2)), a2 = fma_d(w0, r1, -(w1 * r0));
        const double b0 = fma_d(w1, a2, -(w2 * a1)), b1 = fma_d(w2, a0, -(w0 * a2)), b2 = fma_d(w0, a1, -(w1 * a0));
        td[0] = fma_d(c2, b0, fma_d(c1, a0, r0));
        td[1] = fma_d(c2, b1, fma_d(c1, a1, r1));
        td[2] = fma_d(c2, b2, fma_d(c1, a2, r2));
    }
}

// x_i = delta * x (Isometry3d product): R_i = R_d R, t_i = R_d t + t_d, fused
PCORE_GHD void compose(const double (&Rd)[3][3], const double (&td)[3], const double (&R)[3][3], const double (&t)[3],
                       double (&Ro)[3][3], double (&to)[3]) {
PCORE_UNROLL
    for (int r = 0; r < 3; r++) {
PCORE_UNROLL
        for (int c = 0; c < 3; c++) Ro[r][c] = dot3f(Rd[r][0], Rd[r][1], Rd[r][2], R[0][c], R[1][c], R[2][c]);
        to[r] = fma_d(Rd[r][0], t[0], fma_d(Rd[r][1], t[1], fma_d(Rd[r][2], t[2], td[r])));
    }
}

// LsqRegistration::is_converged: max(max|R_d - I| / rot_eps, max|t_d| / trans_eps) < 1, the quotients as
// (1 / eps) * |x| and the maxima in Eigen's column-major coefficient order (first strict maximum)
PCORE_GHD bool is_converged(const double (&Rd)[3][3], const double (&td)[3], double rot_eps, double trans_eps) {
    const double ir = 1.0 / rot_eps, it = 1.0 / trans_eps;
    double mr = ir * __builtin_fabs(Rd[0][0] - 1.0);
PCORE_UNROLL
    for (int c = 0; c < 3; c++)
PCORE_UNROLL
        for (int r = 0; r < 3; r++) {
            if (r == 0 && c == 0) continue;
            const double v = ir * __builtin_fabs(Rd[r][c] - (r == c ? 1.0 : 0.0));
            mr = v > mr ? v : mr;
        }
    double mt = it * __builtin_fabs(td[0]);
PCORE_UNROLL
    for (int r = 1; r < 3; r++) {
        const double v = it * __builtin_fabs(td[r]);
        mt = v > mt ? v : mt;
    }
    const double m = mr < mt ? mt : mr;  // std::max(a, b) = a < b ? b : a
    return m < 1.0;
}

// rho = (y0 - yi) / d.(lambda d - b), the dot product in index order
PCORE_GHD double lm_rho(const double* sys, double lambda, const double (&d)[6], double y0, double yi) {
    double den = d[0] * (lambda * d[0] - sys[21]);
PCORE_UNROLL
    for (int a = 1; a < 6; a++) den = den + d[a] * (lambda * d[a] - sys[21 + a]);
    return (y0 - yi) / den;
}

// u^3 rounded once, as fast_gicp's std::pow(2 rho - 1, 3) (glibc's pow is correctly rounded up to its < 0.52 ulp
// worst cases; the two-rounding (u u) u differs from it by an ulp for ~1 in 4 inputs): u u = p + e and p u = c + e2
// exactly (fma), so u^3 = c + e2 + e u and c + (e2 + e u) is the correctly rounded cube unless u^3 lies within
// ~2^-104 |u^3| of a rounding boundary (tests/test_gicp_spec.py checks it against exact rationals and against pow)
PCORE_GHD double cube_rn(double u) {
    const double p = u * u;
    const double e = fma(u, u, -p);
    const double c = p * u;
    const double e2 = fma(p, u, -c);
    return c + (e2 + e * u);
}

// accepted step: lambda <- lambda * max(1/3, 1 - (2 rho - 1)^3); lm_gain is the factor
PCORE_GHD double lm_gain(double rho) {
    const double u = 2.0 * rho - 1.0;
    const double f = 1.0 - cube_rn(u);
    const double third = 1.0 / 3.0;
    return third < f ? f : third;  // std::max(1/3, f)
}
PCORE_GHD double lm_accept_lambda(double lambda, double rho) { return lambda * lm_gain(rho); }

// The damping is inert on this system: adding lambda changes no diagonal entry of H, so the damped solve is the
// undamped one bit for bit (the GICP cycle exit's condition).
PCORE_GHD bool lm_lambda_inert(const double* sys, double lambda) {
    bool ok = true;
PCORE_UNROLL
    for (int a = 0; a < 6; a++) ok = ok && (sys[hdiag(a)] + lambda == sys[hdiag(a)]);
    return ok;
}

// ---- the cycle exit -------------------------------------------------------------------
// A capped pose is an LM 2-cycle (or a longer one): its float transforms T_f(j) = float(x_{j-1}), and so its
// correspondences, recur with a period p while the doubles drift in their last bits.  After every accepted step of
// iteration k < max_iter that is not converged, p_k = the smallest lag q <= kCycleLags with T_f(k+1) == T_f(k+1-q)
// bit for bit (0: none), and the step is "inert" when it was accepted at its first trial with rho >= 1/2 (lambda
// does not grow) and lambda changed no diagonal entry of H (lm_lambda_inert).  When the last W lags are the same
// p > 0 and the last W steps are inert, the pose stops: it reports max_iter iterations and the transform T_f(j') of
// the cycle member j' = max_iter + 1 (mod p) among its last p iterations -- the float transform the remaining
// iterations would end on while the cycle holds.  W = 0 runs the iterations out (fast_gicp).
constexpr int kCycleLags = 32;
constexpr int kCycleWindow = 8;  // the spec's W (tools/cycle_exit_sim.py: 2,000 C3 candidates, 766 of 810 capped exit)

struct CycleRun {
    int lag, run, okrun;
};

PCORE_GHD bool cycle_update(CycleRun& c, int p, bool inert, int window) {
    c.run = p > 0 ? (p == c.lag ? c.run + 1 : 1) : 0;
    c.lag = p;
    c.okrun = inert ? c.okrun + 1 : 0;
    return window > 0 && p > 0 && c.run >= window && c.okrun >= window;
}

// j' in (cur - p, cur] with j' = max_iter + 1 (mod p), cur = k + 1 <= max_iter
PCORE_GHD int cycle_member(int cur, int p, int max_iter) {
    const int d = (max_iter + 1 - cur) % p;
    return d == 0 ? cur : cur - (p - d);
}

PCORE_GHD bool all_finite6(const double (&d)[6]) {
    bool ok = true;
PCORE_UNROLL
    for (int a = 0; a < 6; a++) ok = ok && (d[a] - d[a] == 0.0);
    return ok;
}

// outcome of one LM iteration
enum LmStatus { kLmAccepted = 0, kLmConverged = 1, kLmFailed = 2 };

}  // namespace gicpm
}  // namespace pcore
