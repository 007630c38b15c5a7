// pcore_gicp_math.h -- the per-point Gauss-Newton contribution of the GICP spec (DESIGN.md "GICP spec"),
// one function compiled into both the HIP kernel (pcore_gicp.hip) and the CPU oracle
// (oracle/pcore_oracle.cpp), so the two evaluate the same double-precision expression tree bit for bit
// (both are built with -ffp-contract=off).
//
// Residual e = t_j - q with q = R s + t, Mahalanobis M = (C_t + R C_s R^T)^-1 (adjugate / determinant),
// Jacobian J = [skew(q) | -I] (fast_gicp's left perturbation):
//   J = [[0, -q2, q1, -1, 0, 0], [q2, 0, -q0, 0, -1, 0], [-q1, q0, 0, 0, 0, -1]].
// The products with J's structural zeros and -1 entries are not evaluated: J^T v for a 3-vector v is
//   (q2 v1 - q1 v2, q0 v2 - q2 v0, q1 v0 - q0 v1, -v0, -v1, -v2),
// MJ = M J column by column likewise, and acc += (upper(J^T M J), J^T M e, e^T M e).
#pragma once

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
// ~0.1 m across), so the cancellation costs ~1e-9 m^2.  Non-finite targets never win (key +inf); a non-finite
// query has no correspondence.
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

// J^T v (the 6-vector above)
PCORE_GHD void jt_mul(const double (&q)[3], const double (&v)[3], double (&o)[6]) {
    o[0] = q[2] * v[1] - q[1] * v[2];
    o[1] = q[0] * v[2] - q[2] * v[0];
    o[2] = q[1] * v[0] - q[0] * v[1];
    o[3] = -v[0];
    o[4] = -v[1];
    o[5] = -v[2];
}

// Terms of the normal equations a point adds: the upper triangle of J^T M J and J^T M e.  (fast_gicp also
// sums the error e^T M e; nothing in the step or the convergence test reads it, so it is not accumulated.)
constexpr int kTerms = 27;

// acc[0..20] += upper(J^T M J) row-major, acc[21..26] += J^T M e, for the point q with correspondence tj,
// source covariance cs and target covariance ct (xx, xy, xz, yy, yz, zz).
PCORE_GHD void contrib(const double (&R)[3][3], const double (&q)[3], const double (&cs)[6], const double (&tj)[3],
                       const double (&ct)[6], double (&acc)[kTerms]) {
    const double Cs[3][3] = {{cs[0], cs[1], cs[2]}, {cs[1], cs[3], cs[4]}, {cs[2], cs[4], cs[5]}};
    const double Ct[3][3] = {{ct[0], ct[1], ct[2]}, {ct[1], ct[3], ct[4]}, {ct[2], ct[4], ct[5]}};
    double RC[3][3], A[3][3];
PCORE_UNROLL
    for (int r = 0; r < 3; r++)
PCORE_UNROLL
        for (int c = 0; c < 3; c++) RC[r][c] = R[r][0] * Cs[0][c] + R[r][1] * Cs[1][c] + R[r][2] * Cs[2][c];
PCORE_UNROLL
    for (int r = 0; r < 3; r++)
PCORE_UNROLL
        for (int c = r; c < 3; c++)
            A[r][c] = Ct[r][c] + (RC[r][0] * R[c][0] + RC[r][1] * R[c][1] + RC[r][2] * R[c][2]);
    A[1][0] = A[0][1];
    A[2][0] = A[0][2];
    A[2][1] = A[1][2];
    // adjugate of the symmetric A (symmetric too) and the determinant
    double m[3][3];
    m[0][0] = A[1][1] * A[2][2] - A[1][2] * A[2][1];
    m[0][1] = A[0][2] * A[2][1] - A[0][1] * A[2][2];
    m[0][2] = A[0][1] * A[1][2] - A[0][2] * A[1][1];
    m[1][1] = A[0][0] * A[2][2] - A[0][2] * A[2][0];
    m[1][2] = A[0][2] * A[1][0] - A[0][0] * A[1][2];
    m[2][2] = A[0][0] * A[1][1] - A[0][1] * A[1][0];
    m[1][0] = m[0][1];
    m[2][0] = m[0][2];
    m[2][1] = m[1][2];
    const double det = A[0][0] * m[0][0] + A[0][1] * m[1][0] + A[0][2] * m[2][0];
    const double inv = 1.0 / det;
    double M[3][3];
PCORE_UNROLL
    for (int r = 0; r < 3; r++)
PCORE_UNROLL
        for (int c = 0; c < 3; c++) M[r][c] = m[r][c] * inv;
    const double e[3] = {tj[0] - q[0], tj[1] - q[1], tj[2] - q[2]};
    // MJ columns 0..2 (skew part); columns 3..5 are -M's columns
    double MJ[3][3];
PCORE_UNROLL
    for (int r = 0; r < 3; r++) {
        MJ[r][0] = M[r][1] * q[2] - M[r][2] * q[1];
        MJ[r][1] = M[r][2] * q[0] - M[r][0] * q[2];
        MJ[r][2] = M[r][0] * q[1] - M[r][1] * q[0];
    }
    // column b of M J as a 3-vector, then its J^T product gives H[a][b] for every a
    int h = 0;
PCORE_UNROLL
    for (int a = 0; a < 6; a++)
PCORE_UNROLL
        for (int b = a; b < 6; b++) {
            const double cb[3] = {b < 3 ? MJ[0][b] : -M[0][b - 3], b < 3 ? MJ[1][b] : -M[1][b - 3],
                                  b < 3 ? MJ[2][b] : -M[2][b - 3]};
            double v;
            if (a == 0) v = q[2] * cb[1] - q[1] * cb[2];
            else if (a == 1) v = q[0] * cb[2] - q[2] * cb[0];
            else if (a == 2) v = q[1] * cb[0] - q[0] * cb[1];
            else v = -cb[a - 3];
            acc[h] += v;
            h++;
        }
    double Me[3];
PCORE_UNROLL
    for (int r = 0; r < 3; r++) Me[r] = M[r][0] * e[0] + M[r][1] * e[1] + M[r][2] * e[2];
    double g[6];
    jt_mul(q, Me, g);
PCORE_UNROLL
    for (int a = 0; a < 6; a++) acc[21 + a] += g[a];
}

}  // namespace gicpm
}  // namespace pcore
