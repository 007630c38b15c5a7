// pcore_cov.h -- the GICP covariances of a point segment (fast_gicp's k-NN covariances with PLANE regularisation;
// DESIGN.md section 5): one wave per round of 64 query points, brute-force k-NN over the segment with candidates
// staged through a 64-point LDS tile, double mean / covariance in list order, Jacobi (<= 6 thresholded sweeps), PLANE regularisation.
// Shared by covariance_kernel (pcore_gicp.hip: one wave per segment) and render_cloud_kernel (pcore_kernels.hip: the
// rendered clouds' covariances in the launch that produced them, its four waves taking the query rounds in turn).
// Bit-identical to the oracle's covariance_one (tests/test_gpu_covariances.py, the GICP parity tests).
#pragma once

#include <hip/hip_runtime.h>

#include <climits>
#include <type_traits>

#ifndef PCORE_COV_SKIP
#define PCORE_COV_SKIP 0  // ablation timing builds only: bit 0 skips the PLANE regularisation, bit 1 the k-NN search
#endif

namespace pcore {
namespace {

constexpr double kPlaneScale = 1.0 - 1e-3;
constexpr double kJacobiEps2 = 4.440892098500626e-16;    // 2 eps (double)
constexpr double kJacobiTiny = 2.2250738585072014e-308;  // the smallest normal double (Eigen's considerAsZero)

// LDS writes by some lanes of a wave visible to all its lanes (no block barrier: waves are independent)
__device__ __forceinline__ void wave_lds_sync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

__device__ __forceinline__ float sqdist3(float ax, float ay, float az, float bx, float by, float bz) {
    const float dx = ax - bx, dy = ay - by, dz = az - bz;
    return dx * dx + dy * dy + dz * dz;
}

// Jacobi (at most 6 cyclic sweeps) + PLANE regularisation, same operation order as orc plane_regularize.  A rotation
// is skipped when its off-diagonal entry is at most 2 eps times the largest diagonal magnitude (Eigen JacobiSVD's
// convergence threshold, which fast_gicp's PLANE regularisation runs), and a sweep without a rotation ends the loop.
__device__ void plane_regularize(const double c[6], double out[6]) {
    double A[3][3] = {{c[0], c[1], c[2]}, {c[1], c[3], c[4]}, {c[2], c[4], c[5]}};
    double V[3][3] = {{1.0, 0.0, 0.0}, {0.0, 1.0, 0.0}, {0.0, 0.0, 1.0}};
#pragma unroll 1
    for (int sweep = 0; sweep < 6; sweep++) {
        bool rotated = false;
#pragma unroll
        for (int r = 0; r < 3; r++) {
            const int p = r < 2 ? 0 : 1, q = r == 0 ? 1 : 2, o = 3 - p - q;
            const double apq = A[p][q];
            const double d0 = fabs(A[0][0]), d1 = fabs(A[1][1]), d2 = fabs(A[2][2]);
            double dm = d0 > d1 ? d0 : d1;
            dm = dm > d2 ? dm : d2;
            double thr = kJacobiEps2 * dm;
            thr = thr > kJacobiTiny ? thr : kJacobiTiny;
            if (fabs(apq) <= thr) continue;
            rotated = true;
            const double theta = (A[q][q] - A[p][p]) / (2.0 * apq);
            double t = 1.0 / (fabs(theta) + sqrt(theta * theta + 1.0));
            if (theta < 0.0) t = -t;
            const double cc = 1.0 / sqrt(t * t + 1.0);
            const double ss = t * cc;
            const double app = A[p][p], aqq = A[q][q];
            A[p][p] = app - t * apq;
            A[q][q] = aqq + t * apq;
            A[p][q] = 0.0;
            A[q][p] = 0.0;
            const double aop = A[o][p], aoq = A[o][q];
            A[o][p] = cc * aop - ss * aoq;
            A[p][o] = A[o][p];
            A[o][q] = ss * aop + cc * aoq;
            A[q][o] = A[o][q];
#pragma unroll
            for (int k = 0; k < 3; k++) {
                const double vkp = V[k][p], vkq = V[k][q];
                V[k][p] = cc * vkp - ss * vkq;
                V[k][q] = ss * vkp + cc * vkq;
            }
        }
        if (!rotated) break;
    }
    // smallest eigenvalue's column, first on ties (selects, not a dynamic register index)
    int m = 0;
    double am = A[0][0];
    if (A[1][1] < am) { m = 1; am = A[1][1]; }
    if (A[2][2] < am) m = 2;
    const double n0 = m == 0 ? V[0][0] : (m == 1 ? V[0][1] : V[0][2]);
    const double n1 = m == 0 ? V[1][0] : (m == 1 ? V[1][1] : V[1][2]);
    const double n2 = m == 0 ? V[2][0] : (m == 1 ? V[2][1] : V[2][2]);
    out[0] = 1.0 - kPlaneScale * (n0 * n0);
    out[1] = 0.0 - kPlaneScale * (n0 * n1);
    out[2] = 0.0 - kPlaneScale * (n0 * n2);
    out[3] = 1.0 - kPlaneScale * (n1 * n1);
    out[4] = 0.0 - kPlaneScale * (n1 * n2);
    out[5] = 1.0 - kPlaneScale * (n2 * n2);
}


// mean / covariance (double, list order) of the listed neighbours and PLANE regularisation (orc covariance_one)
template <int KMAX, class Pts>
__device__ __forceinline__ void cov_from_list(const Pts& P, const int (&nb)[KMAX], int cnt, double* out6) {
    double mx = 0.0, my = 0.0, mz = 0.0;
#pragma unroll
    for (int q = 0; q < KMAX; q++)
        if (q < cnt) {
            const float4 p = P[nb[q]];
            mx += (double)p.x; my += (double)p.y; mz += (double)p.z;
        }
    const double kd = (double)cnt;
    mx = mx / kd; my = my / kd; mz = mz / kd;
    double c6[6] = {0.0, 0.0, 0.0, 0.0, 0.0, 0.0};
#pragma unroll
    for (int q = 0; q < KMAX; q++)
        if (q < cnt) {
            const float4 p = P[nb[q]];
            const double dx = (double)p.x - mx, dy = (double)p.y - my, dz = (double)p.z - mz;
            c6[0] += dx * dx; c6[1] += dx * dy; c6[2] += dx * dz;
            c6[3] += dy * dy; c6[4] += dy * dz; c6[5] += dz * dz;
        }
#pragma unroll
    for (int e = 0; e < 6; e++) c6[e] = c6[e] / kd;
    double r6[6];
#if PCORE_COV_SKIP & 1  // ablation timing only (wrong results): no eigen-decomposition / PLANE regularisation
#pragma unroll
    for (int e = 0; e < 6; e++) r6[e] = c6[e];
#else
    plane_regularize(c6, r6);
#endif
#pragma unroll
    for (int e = 0; e < 6; e++) out6[e] = r6[e];
}

constexpr int kCovLanes = 64;

// the threshold k-NN's point sources: the cloud in global memory, or its copy in the wave's LDS (x, y, z floats)
struct GlobalPts {
    const float4* p;
    __device__ __forceinline__ float4 operator[](int j) const { return p[j]; }
};
struct LdsPts {
    const float* p;
    __device__ __forceinline__ float4 operator[](int j) const {
        return make_float4(p[3 * j], p[3 * j + 1], p[3 * j + 2], 0.0f);
    }
};

// One round of 64 queries i0 + lane of the segment P[0, n): k nearest (distance, index) in the scan's order, their
// covariance into C[6 i].  `tile`: this wave's kCovLanes points of LDS.
// KFIXED: k == KMAX known at compile time (GICP's k = 10): the list's last entry and every `q < k` test are static,
// so the insertion is straight-line code; with a run-time k the compiler indexed nd[k - 1] through s_set_gpr_idx and
// branched once per list entry.
template <int KMAX, bool KFIXED>
__device__ __forceinline__ void cov_knn_round(const float4* P, int n, int k_arg, int i0, int lane, float4* tile,
                                              double* C) {
    const int k = KFIXED ? KMAX : k_arg;
    const int i = i0 + lane;
    const float4 xi = i < n ? P[i] : make_float4(0.0f, 0.0f, 0.0f, 0.0f);
    float nd[KMAX];
    int nb[KMAX];
#pragma unroll
    for (int q = 0; q < KMAX; q++) { nd[q] = 0.0f; nb[q] = 0; }
    int cnt = 0;
    // the list holds a NaN distance (a non-finite point among the first k candidates): it is no longer sorted,
    // and only the counting insertion below reproduces orc knn_self's placement
    bool nan_list = false;
    // insertion identical to orc knn_self: the new element starts at pos and bubbles down past entries with a
    // strictly larger distance
    auto insert_counting = [&](float d, int j) {
        int pos;
        if (cnt < k) pos = cnt;
        else if (d < nd[k - 1]) pos = k - 1;
        else return;
        int c = 0;
#pragma unroll
        for (int q = 0; q < KMAX; q++) c += (q < pos && nd[q] > d) ? 1 : 0;
        const int fin = pos - c;
#pragma unroll
        for (int q = KMAX - 1; q >= 1; q--)
            if (q > fin && q <= pos) { nd[q] = nd[q - 1]; nb[q] = nb[q - 1]; }
#pragma unroll
        for (int q = 0; q < KMAX; q++)
            if (q == fin) { nd[q] = d; nb[q] = j; }
        if (cnt < k) cnt++;
        nan_list = nan_list || d != d;
    };
#if PCORE_COV_SKIP & 2  // ablation timing only (wrong results): the first k points instead of the k-NN search
    for (int q = 0; q < KMAX; q++)
        if (q < k && q < n) { nb[q] = q; cnt = q + 1; }
    for (int j0 = n; j0 < n; j0 += kCovLanes) {
#else
    for (int j0 = 0; j0 < n; j0 += kCovLanes) {
#endif
        wave_lds_sync();  // the previous tile is read
        if (j0 + lane < n) tile[lane] = P[j0 + lane];
        wave_lds_sync();
        const int jn = min(kCovLanes, n - j0);
        float4 xn = tile[0];  // (jn >= 1 here) the next candidate's read is issued before this one's insertion
        for (int jj = 0; jj < jn; jj++) {
            const float4 xj = xn;
            xn = tile[jj + 1 < jn ? jj + 1 : jj];
            const float d = sqdist3(xi.x, xi.y, xi.z, xj.x, xj.y, xj.z);
            const int j = j0 + jj;
            if (cnt < k || nan_list) {  // the first k candidates (every lane at once), or a NaN list
                insert_counting(d, j);
            } else if (d < nd[k - 1]) {
                // a full, sorted list (no NaN: one could only enter among the first k): the counting insertion's
                // result in one pass -- the entries greater than d (a suffix, the list being sorted) move right by
                // one and d takes the first of their slots (d < nd[k - 1], so there is one).  Written from the
                // end, each entry reads its left neighbour before that one is overwritten: no temporaries.
                bool g[KMAX];
#pragma unroll
                for (int q = 0; q < KMAX; q++) g[q] = q < k && nd[q] > d;
#pragma unroll
                for (int q = KMAX - 1; q >= 1; q--) {
                    if (q < k) {
                        // the same value as g[q - 1] ? nd[q - 1] : (g[q] ? d : nd[q]) on a sorted list without NaN
                        nd[q] = __builtin_amdgcn_fmed3f(nd[q - 1], nd[q], d);
                        nb[q] = g[q - 1] ? nb[q - 1] : (g[q] ? j : nb[q]);
                    }
                }
                nd[0] = fminf(nd[0], d);
                nb[0] = g[0] ? j : nb[0];
            }
        }
    }
    if (i < n) cov_from_list<KMAX>(GlobalPts{P}, nb, cnt, C + (size_t)6 * i);
}

}  // namespace
}  // namespace pcore

namespace pcore {
namespace {

// ---- the threshold k-NN of a rendered cloud (round 6) ----------------------------------------------------------
// A cloud unprojected from a stride-s sample grid keeps each point's grid cell: (kx, ky) = rint((x / z fx + cx) / s),
// rint((y / z fy + cy) / s).  The k nearest (distance, index) of a point are the first k of all candidates in that
// order; any tau at or above the k-th smallest distance keeps them all.  So:
//   1. tau = the k-th smallest distance to the points of the 7 x 7 grid cells around the query (an LDS map of the
//      cloud's window gives them; fewer than k there: tau = +inf),
//   2. one pass over all candidates (the brute-force scan's order and arithmetic) collects the j with d <= tau,
//   3. the collected ones, in index order, go through the brute-force's insertion: the list is the brute force's,
//      bit for bit, whatever tau is (tau only bounds what is collected).
// The brute-force scan runs its insertion block whenever any lane of the wave inserts -- nearly every candidate of a
// ~100-point cloud; here the insertions are the 49 neighbourhood steps and the ~10-14 collected per lane (tools/
// knn_threshold_estimate.py), and the full pass is a compare and a predicated LDS store.  A lane collecting more than
// kThrCap candidates, a cloud whose window exceeds kThrMap cells or holding a non-finite point take the brute force.
struct CovGrid {
    float fx, fy, cx, cy;
    int stride;
};

// The launch's LDS per wave (map + lists + points) sets its occupancy: 6 granules (a 1,536-cell map, 24-entry lists,
// 128 points) gave 5 waves per SIMD and 1.61-1.65 ms per C3 call; 5 granules (1,024 / 20 / 96) 1.50-1.53 ms;
// 4 granules (768 / 20 / 64) 1.48-1.50 ms, and with 8 waves per SIMD (64 VGPRs, 7 spilled; PCORE_COV_WAVES_PER_EU)
// 1.45-1.46 ms (profiles/r06m2..4/).  Clouds whose window exceeds the map, or lanes collecting more than the list
// holds, take the brute force (the same results).
#ifndef PCORE_THR_MAP
#define PCORE_THR_MAP 768
#endif
#ifndef PCORE_THR_CAP
#define PCORE_THR_CAP 20
#endif
constexpr int kThrMap = PCORE_THR_MAP;  // window cells of the map (ushort point index each; 0xffff = empty)
constexpr int kThrCap = PCORE_THR_CAP;  // collected candidates per lane
static_assert(kThrMap % 8 == 0 && kThrCap % 4 == 0, "the LDS regions stay 16-byte aligned");
constexpr int kThrR = 3;       // the neighbourhood: (2 kThrR + 1)^2 cells
#ifndef PCORE_THR_UNROLL
#define PCORE_THR_UNROLL 7  // a neighbourhood row per loop trip: its map reads and point loads issue together
#endif
// clouds of at most kThrLdsPts points are copied into the wave's LDS (12 B a point) for the neighbourhood, collecting
// and insertion reads; larger ones are read from global memory through a 64-point tile (the same results).  With the
// 1,536-cell map: 128 points (6 LDS granules per wave) 1.63 / 1.66 ms per C3 call against 1.70 / 1.70 without the
// copy; 232 points (a seventh granule) 1.73 / 1.75 ms (profiles/r06n/).
#ifndef PCORE_THR_LDS_PTS
#define PCORE_THR_LDS_PTS 64
#endif
constexpr int kThrLdsPts = PCORE_THR_LDS_PTS;
constexpr size_t kThrPtsBytes = (size_t)kThrLdsPts * 12 > kCovLanes * 16 ? (size_t)kThrLdsPts * 12 : kCovLanes * 16;
constexpr size_t kThrLdsBytes = kThrMap * 2 + (size_t)kThrCap * kCovLanes * 2 + kThrPtsBytes;

__device__ __forceinline__ void cov_cell(const float4& p, const CovGrid& cg, int& kx, int& ky) {
    kx = (int)rintf((p.x / p.z * cg.fx + cg.cx) / (float)cg.stride);
    ky = (int)rintf((p.y / p.z * cg.fy + cg.cy) / (float)cg.stride);
}

__device__ __forceinline__ int wave_min_i(int v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v = min(v, __shfl_xor(v, o));
    return v;
}
__device__ __forceinline__ int wave_max_i(int v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v = max(v, __shfl_xor(v, o));
    return v;
}

// the cloud's window and its cell map (ushort point index per cell); false: the brute force serves this segment
__device__ __forceinline__ bool cov_thr_map(const float4* P, int n, const CovGrid& cg, int lane, unsigned short* map,
                                            int& kx0, int& ky0, int& wx, int& wy) {
    if (n > 0xfffe) return false;
    int x0 = INT_MAX, x1 = INT_MIN, y0 = INT_MAX, y1 = INT_MIN;
    bool ok = true;
    for (int i = lane; i < n; i += kCovLanes) {
        const float4 p = P[i];
        const bool fin = __builtin_isfinite(p.x) && __builtin_isfinite(p.y) && __builtin_isfinite(p.z) && p.z > 0.0f;
        ok = ok && fin;
        if (fin) {
            int kx, ky;
            cov_cell(p, cg, kx, ky);
            x0 = min(x0, kx); x1 = max(x1, kx); y0 = min(y0, ky); y1 = max(y1, ky);
        }
    }
    if (__ballot(!ok) != 0ull) return false;
    x0 = wave_min_i(x0); x1 = wave_max_i(x1); y0 = wave_min_i(y0); y1 = wave_max_i(y1);
    if (n == 0 || x1 < x0 || y1 < y0) return false;
    const long long cells = (long long)(x1 - x0 + 1) * (long long)(y1 - y0 + 1);
    if (cells > kThrMap) return false;
    kx0 = x0; ky0 = y0; wx = x1 - x0 + 1; wy = y1 - y0 + 1;
    for (int c = lane; c < (int)cells; c += kCovLanes) map[c] = 0xffff;
    wave_lds_sync();
    for (int i = lane; i < n; i += kCovLanes) {
        int kx, ky;
        cov_cell(P[i], cg, kx, ky);
        map[(ky - y0) * wx + (kx - x0)] = (unsigned short)i;  // a shared cell keeps one of its points: any subset bounds
    }
    wave_lds_sync();
    return true;
}

// One round of 64 queries by the threshold k-NN (k = 10).  Returns false (nothing written) when a lane collects more
// than kThrCap candidates: the caller runs cov_knn_round for this round.
template <bool LDS_PTS>
__device__ __forceinline__ bool cov_knn_round_thr(const float4* Pg, const float* lds_pts, int n, int i0, int lane,
                                                  const CovGrid& cg, const unsigned short* map, int kx0, int ky0, int wx,
                                                  int wy, unsigned short* list, float4* tile, double* C) {
    constexpr int K = 10;
    const int i = i0 + lane;
    const bool act = i < n;
    typedef typename std::conditional<LDS_PTS, LdsPts, GlobalPts>::type PtsT;
    PtsT P;
    if constexpr (LDS_PTS) P.p = lds_pts;
    else P.p = Pg;
    const float4 xi = act ? P[i] : make_float4(0.0f, 0.0f, 1.0f, 0.0f);
    // 1. tau: the K-th smallest distance over the neighbourhood cells (sorted values, one-pass insertion)
    float t[K];
#pragma unroll
    for (int q = 0; q < K; q++) t[q] = INFINITY;
    int kx, ky;
    cov_cell(xi, cg, kx, ky);
    for (int dv = -kThrR; dv <= kThrR; dv++) {
        const int cy = ky + dv - ky0;
#pragma unroll PCORE_THR_UNROLL
        for (int du = -kThrR; du <= kThrR; du++) {
            const int cx = kx + du - kx0;
            const bool in = act && cx >= 0 && cx < wx && cy >= 0 && cy < wy;
            const int j = in ? (int)map[cy * wx + cx] : 0xffff;
            if (j != 0xffff) {
                const float4 p = P[j];
                const float d = sqdist3(xi.x, xi.y, xi.z, p.x, p.y, p.z);
                // t stays sorted: entry q becomes the median of (t[q - 1], t[q], d) -- one v_med3_f32 each (no NaN:
                // the points are finite) where the selects took a compare and two v_cndmask
#pragma unroll
                for (int q = K - 1; q >= 1; q--) t[q] = __builtin_amdgcn_fmed3f(t[q - 1], t[q], d);
                t[0] = fminf(t[0], d);
            }
        }
    }
    const float tau = t[K - 1];
    // 2. every candidate in scan order; the ones at or below tau are collected (index order)
    int cnt = 0;
    if constexpr (LDS_PTS) {
        for (int j = 0; j < n; j++) {
            const float4 xj = P[j];
            const float d = sqdist3(xi.x, xi.y, xi.z, xj.x, xj.y, xj.z);
            if (act && d <= tau) {
                if (cnt < kThrCap) list[cnt * kCovLanes + lane] = (unsigned short)j;
                cnt++;
            }
        }
    } else {
        for (int j0 = 0; j0 < n; j0 += kCovLanes) {
            wave_lds_sync();  // the previous tile is read
            if (j0 + lane < n) tile[lane] = Pg[j0 + lane];
            wave_lds_sync();
            const int jn = min(kCovLanes, n - j0);
            for (int jj = 0; jj < jn; jj++) {
                const float4 xj = tile[jj];
                const float d = sqdist3(xi.x, xi.y, xi.z, xj.x, xj.y, xj.z);
                if (act && d <= tau) {
                    if (cnt < kThrCap) list[cnt * kCovLanes + lane] = (unsigned short)(j0 + jj);
                    cnt++;
                }
            }
        }
    }
    if (__ballot(cnt > kThrCap) != 0ull) return false;
    // 3. the collected candidates through the brute force's insertion (stable: entries strictly greater move right)
    // The list's unfilled entries hold +inf, so one form serves the filling and the full list: the entries strictly
    // greater than d (a suffix of the sorted list, +inf included) move right by one and d takes the first of their
    // slots -- the counting insertion's placement, since d is finite (the points are) and each j exceeds the listed
    // ones.  Values by one v_med3_f32 per entry, indices by the same compares.
    float nd[K];
    int nb[K];
#pragma unroll
    for (int q = 0; q < K; q++) { nd[q] = INFINITY; nb[q] = 0; }
    int len = 0;
    const int cmax = wave_max_i(cnt);
    for (int c = 0; c < cmax; c++) {
        if (c < cnt) {
            const int j = list[c * kCovLanes + lane];
            const float4 p = P[j];
            const float d = sqdist3(xi.x, xi.y, xi.z, p.x, p.y, p.z);
            if (d < nd[K - 1]) {
                bool g[K];
#pragma unroll
                for (int q = 0; q < K; q++) g[q] = nd[q] > d;
#pragma unroll
                for (int q = K - 1; q >= 1; q--) {
                    nd[q] = __builtin_amdgcn_fmed3f(nd[q - 1], nd[q], d);
                    nb[q] = g[q - 1] ? nb[q - 1] : (g[q] ? j : nb[q]);
                }
                nd[0] = fminf(nd[0], d);
                nb[0] = g[0] ? j : nb[0];
                len = len < K ? len + 1 : K;
            }
        }
    }
    if (act) cov_from_list<K>(P, nb, len, C + (size_t)6 * i);
    return true;
}

}  // namespace
}  // namespace pcore
