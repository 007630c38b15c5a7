// pcore_gicp.hip -- per-pose GICP refinement on gfx950.
//
// Build-owned spec (fast_gicp is an un-vendored fork; see DESIGN.md "GICP spec"): fast_gicp's published
// FastGICP + LsqRegistration algorithm at the reference's settings (renderer.cu:1693-1720): k = 10 covariance
// neighbours with PLANE regularisation, nearest-neighbour correspondences inside the pose's label segment,
// Mahalanobis (C_t + R C_s R^T)^-1, Levenberg-Marquardt steps on SE(3) through the exact se3_exp, <= 150
// iterations, rotation / translation epsilons 2e-3 / 5e-4.  The arithmetic lives in pcore_gicp_math.h; its
// order -- including the reduction tree of the normal equations and of the trial errors -- is fixed, and the
// CPU oracle (oracle/pcore_oracle.cpp, orc_gicp) follows the same order, so the refined transforms are
// reproducible bit for bit.
//
//   covariance_kernel  one wave per segment (a pose's rendered cloud or an observed label): brute-force
//                      k-NN of every point inside its segment (candidates staged through LDS), double
//                      mean / covariance, Jacobi (<= 6 sweeps, thresholded), PLANE regularisation.
//   gicp_kernel        one wave per pose: per-lane sequential partial sums of J^T M J / J^T M e / e^T M e,
//                      the shuffle-down tree in registers (wave_tree_sums), the LM iteration (uniform: the
//                      damped solve by 3x3 block elimination, se3_exp, the trial), the correspondence history, then
//                      concatenate_transforms (renderer.cu:1412-1429).
//   gicp_wide_kernel   small batches: eight waves search a pose's correspondences, wave 0 as gicp_kernel.
#include "pcore_internal.h"

#include <hipcub/hipcub.hpp>
#include "pcore_cov.h"
#include "pcore_gicp_math.h"

#include <algorithm>
#include <cstdlib>
#include <cfloat>
#include <climits>

#pragma clang fp contract(off)

namespace pcore {

namespace {

constexpr int kGThreads = 256;
constexpr int kMaxK = 16;
// Build with -DPCORE_GICP_PROFILE to accumulate per-phase shader clocks of gicp_kernel (tools only):
// [0] correspondence search, [1] contributions (+ M stores), [2] wave reduction, [3] LM iteration, which splits into [4] damped
// solves, [5] se3_exp + compose, [6] the trials' error sums and their reduction, [7] the decisions; [8] counts the
// iterations that reused a set of the correspondence history instead of searching.
// Each wave sums its clocks in registers and adds them once at exit (no atomics inside the loop); each
// clock read is ordered after its phase's last result by an asm input dependency.
#ifdef PCORE_GICP_PROFILE
constexpr int kGprof = 10;  // [9]: the pose-iterations the sums cover (poses of >= PCORE_GICP_PROF_MIN_NS points)
#ifndef PCORE_GICP_PROF_MIN_NS
#define PCORE_GICP_PROF_MIN_NS 0
#endif
__device__ unsigned long long g_gicp_prof[kGprof];
#define GPROF_DECL unsigned long long gp_acc[kGprof] = {}
#define GPROF_T(v) const unsigned long long v = __builtin_readcyclecounter()
#define GPROF_TD(v, dep)                                                                   \
    unsigned long long v;                                                                  \
    asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(v) : "v"(dep) : "memory")
#define GPROF_ADD(k, a, b) gp_acc[k] += (unsigned long long)((b) - (a))
#define GPROF_FLUSH \
    if (lane == 0)  \
        for (int k_ = 0; k_ < kGprof; k_++) atomicAdd(&g_gicp_prof[k_], gp_acc[k_])
#define GPROF_PARAM , unsigned long long (&gp_acc)[kGprof]
#define GPROF_ARG , gp_acc
#else
#define GPROF_DECL
#define GPROF_T(v)
#define GPROF_TD(v, dep)
#define GPROF_ADD(k, a, b)
#define GPROF_FLUSH
#define GPROF_PARAM
#define GPROF_ARG
#endif
// Build with -DPCORE_GICP_TIMELINE (tools only, tools/gicp_timeline.py): gicp_kernel records, per pose, the real-time
// clock (100 MHz) when a wave dequeues it and when it writes the refined pose, and per wave its start and exit.
#ifdef PCORE_GICP_TIMELINE
constexpr int kTlPoses = 1 << 17, kTlWaves = 1 << 14;
__device__ unsigned long long g_tl_pose[2 * kTlPoses];
__device__ unsigned long long g_tl_wave[2 * kTlWaves];
__device__ unsigned int g_tl_nwaves;
__device__ int g_tl_run[kTlPoses];  // iterations each pose executed (fewer than it reports after a cycle exit)
extern "C" int pcore_debug_gicp_timeline_run(int* run) {
    return hipMemcpyFromSymbol(run, HIP_SYMBOL(g_tl_run), sizeof(g_tl_run)) == hipSuccess ? 0 : 1;
}
extern "C" int pcore_debug_gicp_timeline(unsigned long long* poses, unsigned long long* waves, unsigned int* nwaves) {
    hipError_t e = hipMemcpyFromSymbol(poses, HIP_SYMBOL(g_tl_pose), sizeof(g_tl_pose));
    if (e == hipSuccess) e = hipMemcpyFromSymbol(waves, HIP_SYMBOL(g_tl_wave), sizeof(g_tl_wave));
    if (e == hipSuccess) e = hipMemcpyFromSymbol(nwaves, HIP_SYMBOL(g_tl_nwaves), sizeof(unsigned int));
    const unsigned int z = 0;
    if (e == hipSuccess) e = hipMemcpyToSymbol(HIP_SYMBOL(g_tl_nwaves), &z, sizeof(z));
    return e == hipSuccess ? 0 : 1;
}
#endif

typedef float f2v __attribute__((ext_vector_type(2)));
typedef float f4v __attribute__((ext_vector_type(4)));

// se3_exp's series coefficients as the kernels read them: an LDS copy through an address-space-3 pointer offset by an
// opaque zero produced inside the iteration loop, so the loads cannot be hoisted out of it (as literal constants they
// were hoisted into 64 VGPRs for the whole kernel; a generic pointer made them flat loads) but can be issued together
// ahead of the series (a volatile pointer serialised them: one LDS round trip per coefficient, 32 in a row)
typedef __attribute__((address_space(3))) const double lds_cvd;
__device__ __forceinline__ int opaque_zero() {
    int z;
    asm volatile("s_mov_b32 %0, 0" : "=s"(z));
    return z;
}

}  // namespace

// ------------------------------------------------------------------------------------------------
// Exact neighbour search over a segment's grid (segments above kGridNNMin points)
// ------------------------------------------------------------------------------------------------
//
// Cells are visited in shells of growing Chebyshev radius r around the query's cell.  A point binned in
// cell i has its float cell coordinate fp in [i, i + 1) (the grid spans the points' own bounds, so no
// clamping), so along each axis |fp - fq| is at least the gap between fq and that interval, and the true
// distance at least (gap - eps) * cell; a cell whose bound exceeds the caller's limit (the best distance,
// or the k-th best once k are held) is skipped without loading it, and the search stops once the limit is
// below the bound of the nearest face of the visited box that still has cells beyond it.  Every skipped
// point is strictly farther than the limit, so the result equals the brute-force scan's lexicographic
// minimum of (float distance, index).
// Returns false when the cell budget runs out first (or the query is far outside the grid): the caller
// then scans the whole segment.  Non-finite queries are the caller's business.
// Cell budget of one search: a visited cell costs about as much as two points of the in-order scan (its lower-bound
// test, the CSR range loads, the loop), so the shells may visit up to half the segment's point count before the scan
// would have been cheaper, and at least 343 cells (r <= 3 around an in-grid query).  C1 (a 19.2 k-point whole-scene
// target, `tools/c1_gicp_stats.py`): a fixed 343-cell budget sent the queries of poses that GICP walks away from the
// scene into the 19.2 k-point scan, 64.7 ms per GICP call; budgets of 2,197 / 9,261 / 35,937 cells gave 18.6 / 18.4 /
// 18.2 ms, and this rule 19.7 ms (profiles/r03x/).  Measured and dropped: the 343-cell shells followed by an exact
// search over the grid's list of non-empty cells (an upper bound from the least farthest-corner distance, then the
// cells whose lower bound is within it) instead of the in-order scan, 37.1 ms.
__device__ __forceinline__ int shell_budget(int n) { return max(343, n >> 1); }

template <typename Visit, typename Limit>
__device__ __forceinline__ bool grid_shells(const LabelGrid& g, const int32_t* cell_start, float qx, float qy,
                                            float qz, int budget, Visit&& visit, Limit&& limit) {
    const float fx = (qx - g.ox) * g.inv_c, fy = (qy - g.oy) * g.inv_c, fz = (qz - g.oz) * g.inv_c;
    const float fm = fmaxf(fabsf(fx), fmaxf(fabsf(fy), fabsf(fz)));
    if (!(fm < 65536.0f)) return false;
    const int cx = (int)floorf(fx), cy = (int)floorf(fy), cz = (int)floorf(fz);
    const float e = 0.01f + 1e-6f * fm;  // cell-unit slack for the rounding of fp, fq and inv_c
    const float c2 = g.cell * g.cell * 0.99999f;
    // lower bound of the float squared distance from q to any point binned in cell (ix, iy, iz): a point's
    // cell coordinate fp lies in [i, i + 1), so |fp - fq| >= gap along each axis
    auto cell_lb = [&](int ix, int iy, int iz) {
        const float gx = fmaxf(fmaxf((float)ix - fx, fx - (float)(ix + 1)) - e, 0.0f);
        const float gy = fmaxf(fmaxf((float)iy - fy, fy - (float)(iy + 1)) - e, 0.0f);
        const float gz = fmaxf(fmaxf((float)iz - fz, fz - (float)(iz + 1)) - e, 0.0f);
        return (gx * gx + gy * gy + gz * gz) * c2;
    };
    auto try_cell = [&](int row, int ix, int iy, int iz) {
        if (cell_lb(ix, iy, iz) > limit()) return;  // every point of the cell is strictly farther
        visit(cell_start[row + ix], cell_start[row + ix + 1]);
    };
    int visited = 0;
    for (int r = 0;; r++) {
        const int z0 = max(0, cz - r), z1 = min(g.nz - 1, cz + r);
        const int y0 = max(0, cy - r), y1 = min(g.ny - 1, cy + r);
        const int x0 = max(0, cx - r), x1 = min(g.nx - 1, cx + r);
        for (int iz = z0; iz <= z1; iz++)
            for (int iy = y0; iy <= y1; iy++) {
                const int row = g.cell_base + (iz * g.ny + iy) * g.nx;
                const bool face = iz == cz - r || iz == cz + r || iy == cy - r || iy == cy + r;
                if (face) {
                    for (int ix = x0; ix <= x1; ix++) try_cell(row, ix, iy, iz);
                    visited += x1 >= x0 ? x1 - x0 + 1 : 0;
                } else {
                    if (cx - r >= 0 && cx - r < g.nx) {
                        try_cell(row, cx - r, iy, iz);
                        visited++;
                    }
                    if (r > 0 && cx + r >= 0 && cx + r < g.nx) {
                        try_cell(row, cx + r, iy, iz);
                        visited++;
                    }
                }
            }
        // unvisited cells lie beyond the faces of the box [c - r, c + r + 1) that are inside the grid; the
        // distance from fq to the nearest such face bounds every unvisited point
        float B = INFINITY;
        if (cx - r > 0) B = fminf(B, fx - (float)(cx - r));
        if (cx + r < g.nx - 1) B = fminf(B, (float)(cx + r + 1) - fx);
        if (cy - r > 0) B = fminf(B, fy - (float)(cy - r));
        if (cy + r < g.ny - 1) B = fminf(B, (float)(cy + r + 1) - fy);
        if (cz - r > 0) B = fminf(B, fz - (float)(cz - r));
        if (cz + r < g.nz - 1) B = fminf(B, (float)(cz + r + 1) - fz);
        if (B == INFINITY) return true;  // every cell visited
        B -= e;
        if (B > 0.0f && limit() < B * B * c2) return true;
        if (visited >= budget) return false;
    }
}

// k best (distance, index) pairs in lexicographic order, as the brute-force insertion keeps them
template <int KMAX>
__device__ __forceinline__ void knn_insert_lex(float (&nd)[KMAX], int (&nb)[KMAX], int& cnt, int k, float d, int j) {
    if (cnt == k && !(d < nd[k - 1] || (d == nd[k - 1] && j < nb[k - 1]))) return;
    const int pos = cnt < k ? cnt : k - 1;
    int c = 0;
#pragma unroll
    for (int q = 0; q < KMAX; q++) c += (q < pos && (nd[q] > d || (nd[q] == d && nb[q] > j))) ? 1 : 0;
    const int fin = pos - c;
#pragma unroll
    for (int q = KMAX - 1; q >= 1; q--)
        if (q > fin && q <= pos) { nd[q] = nd[q - 1]; nb[q] = nb[q - 1]; }
#pragma unroll
    for (int q = 0; q < KMAX; q++)
        if (q == fin) { nd[q] = d; nb[q] = j; }
    if (cnt < k) cnt++;
}

// ------------------------------------------------------------------------------------------------
// covariances
// ------------------------------------------------------------------------------------------------
// One wave per segment (a pose's rendered cloud or an observed label), one lane per point in rounds of 64 (pcore_cov.h
// cov_knn_round); a 256-thread workgroup per segment left two of its four waves idle on C3's ~111-point clouds.
// C3: 2.65 -> 2.61 ms per 50 k clouds -- the time is the insertion block, which the wave runs whenever any lane
// inserts (k ln(n / k) + k insertions per point), not the candidate loads.
template <int KMAX, bool KFIXED = false>
__global__ void __launch_bounds__(kCovLanes) covariance_kernel(const float4* pts, const int32_t* seg_off,
                                                               const int32_t* seg_cnt, int seg_stride, int k_arg,
                                                               double* cov_out, int max_n) {
    __shared__ float4 tile[kCovLanes];
    const int sg = blockIdx.x;
    const int off = seg_off ? seg_off[sg] : sg * seg_stride;
    const int n = seg_cnt[sg];
    if (n > max_n) return;  // covariance_grid_kernel's segment
    const int lane = threadIdx.x;
    for (int i0 = 0; i0 < n; i0 += kCovLanes)
        cov_knn_round<KMAX, KFIXED>(pts + off, n, k_arg, i0, lane, tile, cov_out + (size_t)6 * off);
}

// The rendered clouds' covariances (k = 10): the threshold k-NN where the cloud's sample grid allows it, else the brute
// force, round by round (pcore_cov.h); bit-identical either way.  Dynamic LDS: kThrLdsBytes.
#ifndef PCORE_COV_WAVES_PER_EU
#define PCORE_COV_WAVES_PER_EU 8  // 64 VGPRs (7 spilled): 8 waves per SIMD, which the 4-granule LDS allows (pcore_cov.h)
#endif
// One rendered cloud's covariances by one wave: P[0, n) -> C[6 i], thr_lds = kThrLdsBytes of the wave's LDS.  Used by
// covariance_cloud_kernel (one wave per cloud) and by gicp_kernel's pose prologue (GicpArgs::cov_fold).
__device__ __forceinline__ void cov_cloud_segment(const float4* P, int n, const CovGrid& cg, int lane,
                                                  unsigned char* thr_lds, double* C) {
    float4* tile = reinterpret_cast<float4*>(thr_lds);  // the global path's tile, or the cloud's points (LDS path)
    float* lpts = reinterpret_cast<float*>(thr_lds);
    unsigned short* map = reinterpret_cast<unsigned short*>(thr_lds + kThrPtsBytes);
    unsigned short* list = map + kThrMap;
    int kx0 = 0, ky0 = 0, wx = 0, wy = 0;
    const bool thr = cov_thr_map(P, n, cg, lane, map, kx0, ky0, wx, wy);
    bool in_lds = thr && n <= kThrLdsPts;
    if (in_lds) {
        for (int j = lane; j < n; j += kCovLanes) {
            const float4 p = P[j];
            lpts[3 * j] = p.x;
            lpts[3 * j + 1] = p.y;
            lpts[3 * j + 2] = p.z;
        }
        wave_lds_sync();
    }
    for (int i0 = 0; i0 < n; i0 += kCovLanes) {
        if (in_lds) {
            if (cov_knn_round_thr<true>(P, lpts, n, i0, lane, cg, map, kx0, ky0, wx, wy, list, tile, C)) continue;
            wave_lds_sync();  // the brute force's tile overwrites the points: every lane is done with them
            in_lds = false;   // the later rounds read the cloud from global memory
        } else if (thr && cov_knn_round_thr<false>(P, lpts, n, i0, lane, cg, map, kx0, ky0, wx, wy, list, tile, C)) {
            continue;
        }
        cov_knn_round<10, true>(P, n, 10, i0, lane, tile, C);
    }
}

// gicp_kernel's call of it: not inlined, so the k-NN's registers do not add to those of the iteration loop
__device__ __attribute__((noinline)) void cov_cloud_segment_call(const float4* P, int n, CovGrid cg, int lane,
                                                                 unsigned char* thr_lds, double* C) {
    cov_cloud_segment(P, n, cg, lane, thr_lds, C);
}

__global__ void __launch_bounds__(kCovLanes) __attribute__((amdgpu_waves_per_eu(PCORE_COV_WAVES_PER_EU)))
covariance_cloud_kernel(const float4* pts, const int32_t* seg_cnt, int seg_stride, CovGrid cg, double* cov_out) {
    extern __shared__ __attribute__((aligned(16))) unsigned char thr_lds[];
    const int off = blockIdx.x * seg_stride;
    cov_cloud_segment(pts + off, seg_cnt[blockIdx.x], cg, threadIdx.x, thr_lds, cov_out + (size_t)6 * off);
}

hipError_t launch_covariances_cloud(const float4* pts, const int32_t* seg_cnt, int seg_stride, int num_segs,
                                    float fx, float fy, float cx, float cy, int stride, double* cov_out, hipStream_t s) {
    if (num_segs <= 0) return hipSuccess;
    const CovGrid cg{fx, fy, cx, cy, stride};
    hipLaunchKernelGGL(covariance_cloud_kernel, dim3(num_segs), dim3(kCovLanes), kThrLdsBytes, s, pts, seg_cnt,
                       seg_stride, cg, cov_out);
    return hipGetLastError();
}

// Segments above kGridNNMin points: one thread per point, k-NN by the exact grid shell search
template <int KMAX>
__global__ void __launch_bounds__(kGThreads) covariance_grid_kernel(const float4* pts, int off, int n,
                                                                    const LabelGrid* grid, const int32_t* cell_start,
                                                                    const float4* gpts, int k, double* cov_out) {
    const int i = blockIdx.x * kGThreads + threadIdx.x;
    if (i >= n) return;
    const LabelGrid g = *grid;
    const float4* P = pts + off;
    const float4 xi = P[i];
    float nd[KMAX];
    int nb[KMAX];
#pragma unroll
    for (int q = 0; q < KMAX; q++) { nd[q] = 0.0f; nb[q] = 0; }
    int cnt = 0;
    auto visit = [&](int b, int e) {
        for (int pi = b; pi < e; pi++) {
            const float4 o = gpts[pi];
            knn_insert_lex<KMAX>(nd, nb, cnt, k, sqdist3(xi.x, xi.y, xi.z, o.x, o.y, o.z), __float_as_int(o.w));
        }
    };
    const bool ok = isfinite(xi.x) && isfinite(xi.y) && isfinite(xi.z) &&
                    grid_shells(g, cell_start, xi.x, xi.y, xi.z, shell_budget(n), visit,
                                [&] { return cnt == k ? nd[k - 1] : INFINITY; });
    if (!ok) {
        cnt = 0;
        for (int j = 0; j < n; j++) {
            const float4 xj = P[j];
            knn_insert_lex<KMAX>(nd, nb, cnt, k, sqdist3(xi.x, xi.y, xi.z, xj.x, xj.y, xj.z), j);
        }
    }
    cov_from_list<KMAX>(P, nb, cnt, cov_out + (size_t)6 * (off + i));
}

hipError_t launch_covariances(const float4* pts, const int32_t* seg_off, const int32_t* seg_cnt, int seg_stride,
                              int num_segs, int k, double* cov_out, hipStream_t s, int max_n) {
    if (num_segs <= 0) return hipSuccess;
    if (k <= 0 || k > kMaxK) return hipErrorInvalidValue;
    if (k == 10)
        hipLaunchKernelGGL((covariance_kernel<10, true>), dim3(num_segs), dim3(kCovLanes), 0, s, pts, seg_off, seg_cnt,
                           seg_stride, k, cov_out, max_n);
    else if (k < 10)
        hipLaunchKernelGGL(covariance_kernel<10>, dim3(num_segs), dim3(kCovLanes), 0, s, pts, seg_off, seg_cnt,
                           seg_stride, k, cov_out, max_n);
    else
        hipLaunchKernelGGL(covariance_kernel<kMaxK>, dim3(num_segs), dim3(kCovLanes), 0, s, pts, seg_off, seg_cnt,
                           seg_stride, k, cov_out, max_n);
    return hipGetLastError();
}

hipError_t launch_covariances_grid(const float4* pts, const int32_t* seg_off_host, const int32_t* seg_cnt_host,
                                   int num_segs, int first_grid, const LabelGrid* grids, const int32_t* cell_start,
                                   const float4* grid_pts, int k, double* cov_out, hipStream_t s) {
    if (k <= 0 || k > kMaxK) return hipErrorInvalidValue;
    for (int sg = 0; sg < num_segs; sg++) {
        const int n = seg_cnt_host[sg];
        if (n <= kGridNNMin) continue;
        const dim3 blocks((n + kGThreads - 1) / kGThreads);
        if (k <= 10)
            hipLaunchKernelGGL(covariance_grid_kernel<10>, blocks, dim3(kGThreads), 0, s, pts, seg_off_host[sg], n,
                               grids + first_grid + sg, cell_start, grid_pts, k, cov_out);
        else
            hipLaunchKernelGGL(covariance_grid_kernel<kMaxK>, blocks, dim3(kGThreads), 0, s, pts, seg_off_host[sg], n,
                               grids + first_grid + sg, cell_start, grid_pts, k, cov_out);
        const hipError_t e = hipGetLastError();
        if (e != hipSuccess) return e;
    }
    return hipSuccess;
}

// ------------------------------------------------------------------------------------------------
// GICP
// ------------------------------------------------------------------------------------------------

// Nearest target by the segment's grid (segments above kGridNNMin): the lexicographic minimum of (float
// squared distance, index) -- the brute-force scan's first strict minimum -- or j = -1 when no distance is
// below +inf (a non-finite query).  Falls back to an in-order scan of the segment.
__device__ __forceinline__ void grid_nn(const LabelGrid& G, const int32_t* cell_start, const float4* gpts,
                                        const float4* tgt, int nt, float qx, float qy, float qz, float& best, int& j) {
    best = INFINITY;
    j = -1;
    if (!(isfinite(qx) && isfinite(qy) && isfinite(qz))) return;
    auto visit = [&](int b, int e) {
        for (int pi = b; pi < e; pi++) {
            const float4 o = gpts[pi];
            const float d = sqdist3(qx, qy, qz, o.x, o.y, o.z);
            const int oi = __float_as_int(o.w);
            if (d < best || (d == best && j >= 0 && oi < j)) { best = d; j = oi; }
        }
    };
    if (grid_shells(G, cell_start, qx, qy, qz, shell_budget(nt), visit, [&] { return best; })) return;
    best = INFINITY;
    j = -1;
    for (int i = 0; i < nt; i++) {
        const float4 o = tgt[i];
        const float d = sqdist3(qx, qy, qz, o.x, o.y, o.z);
        if (d < best) { best = d; j = i; }
    }
}

// Nearest of a segment's targets read through the scalar cache: every lane scans the same quads of four targets
// stored as correspondence keys (pcore_gicp_math.h: -2 t'x [4], -2 t'y [4], -2 t'z [4], |t'|^2 [4] about the
// segment's origin, which the header quad before them holds), so the loads are wave-uniform s_loads and the
// targets reach the VALU as SGPR operands -- no LDS traffic (an LDS broadcast read still moves 64 lanes x 16 B
// through the LDS pipe).  A pair of targets costs three packed FMAs.  The index work stays out of the per-quad
// loop: alternate quads feed two chains that keep only their smallest quad minimum and the first quad reaching it
// (strict <); the chains merge by (key, quad), and the winning quad's element is found once at the end by
// recomputing its four keys (the same FMAs, so one of them equals the minimum bit for bit) and taking the first
// equal one -- the lexicographic minimum of (key, index), i.e. the oracle's first strict minimum.  Measured on
// C3's GICP call: a per-quad (distance, index) tournament over x / y / z quads 21.9 ms, the index-free scan of
// float squared distances 21.2 ms.  Keys of finite targets and a finite query are finite, so minNum's NaN
// handling never decides a comparison.
typedef __attribute__((address_space(4))) const f4v cf4v;
#ifndef PCORE_SCAN_UNROLL
#define PCORE_SCAN_UNROLL 4  // quad pairs per loop trip (C3: 2 -> 4: 20.60 -> 20.45 ms per step; 1: 21.25)
#endif
#ifndef PCORE_GICP_PAIR_SCAN
#define PCORE_GICP_PAIR_SCAN 1  // 0: scan a round pair's queries one after the other (A/B)
#endif
#ifndef PCORE_SCAN2_UNROLL
#define PCORE_SCAN2_UNROLL 2  // scan_quads2: quad pairs per loop trip
#endif
#ifndef PCORE_SCAN_PAIRQ
#define PCORE_SCAN_PAIRQ 0  // scan_quads2: one compare per pair of quads per chain (A/B)
#endif

__device__ __forceinline__ void scan_quads(const float* seg_quads, int nt, float qx, float qy, float qz, float& best,
                                           int& j) {
    const int nq = (nt + 3) >> 2;
    const cf4v* hq = (const cf4v*)seg_quads;
    const f4v org = hq[0];
    qx = qx - org.x;
    qy = qy - org.y;
    qz = qz - org.z;
    if (!(__builtin_isfinite(qx) && __builtin_isfinite(qy) && __builtin_isfinite(qz))) return;  // no correspondence
    const cf4v* tq = hq + 4;
    const f2v qx2 = {qx, qx}, qy2 = {qy, qy}, qz2 = {qz, qz};
    float bA = INFINITY, bB = INFINITY;
    int oA = -1, oB = -1;
    auto qmin = [&](const cf4v* q) {
        const f4v X = q[0], Y = q[1], Z = q[2], T = q[3];
        const f2v ka = __builtin_elementwise_fma(X.xy, qx2, __builtin_elementwise_fma(Y.xy, qy2,
                                                  __builtin_elementwise_fma(Z.xy, qz2, T.xy)));
        const f2v kb = __builtin_elementwise_fma(X.zw, qx2, __builtin_elementwise_fma(Y.zw, qy2,
                                                  __builtin_elementwise_fma(Z.zw, qz2, T.zw)));
        return fminf(fminf(fminf(ka.x, ka.y), kb.x), kb.y);
    };
    int o = 0;
    const cf4v* q = tq;  // wave-uniform: the quads' addresses stay scalar
#pragma unroll PCORE_SCAN_UNROLL
    for (; o + 2 <= nq; o += 2, q += 8) {
        const float ma = qmin(q);
        if (ma < bA) { bA = ma; oA = o; }
        const float mb = qmin(q + 4);
        if (mb < bB) { bB = mb; oB = o + 1; }
    }
    if (o < nq) {
        const float ma = qmin(q);
        if (ma < bA) { bA = ma; oA = o; }
    }
    if (bB < bA || (bB == bA && oB >= 0 && oB < oA)) { bA = bB; oA = oB; }
    if (bA < best) {
        // the winning quad, per lane (a vector load), its first element at the minimum
        const float* Q = seg_quads + 16 + 16 * oA;
        const float4 X = *reinterpret_cast<const float4*>(Q), Y = *reinterpret_cast<const float4*>(Q + 4);
        const float4 Z = *reinterpret_cast<const float4*>(Q + 8), T = *reinterpret_cast<const float4*>(Q + 12);
        const int k = gicpm::nn_key(X.x, Y.x, Z.x, T.x, qx, qy, qz) == bA ? 0
                    : gicpm::nn_key(X.y, Y.y, Z.y, T.y, qx, qy, qz) == bA ? 1
                    : gicpm::nn_key(X.z, Y.z, Z.z, T.z, qx, qy, qz) == bA ? 2 : 3;
        best = bA;
        // one of the four recomputed keys equals bA (same FMAs); the clamp only keeps a broken match (which would
        // pick slot 3, padding in a segment's last quad) inside the segment
        j = min(4 * oA + k, nt - 1);
    }
}

// scan_quads for two queries per lane (the pose's source points i and i + 64): every scalar load of a quad feeds both,
// so a pair of rounds reads the segment's key quads once.  Each query keeps its own two chains (alternate quads) and
// its own winner recovery, so (best, j) of each is scan_quads' bit for bit.
__device__ __forceinline__ void scan_quads2(const float* seg_quads, int nt, float ax, float ay, float az, float bx,
                                            float by, float bz, int& ja, int& jb) {
    const int nq = (nt + 3) >> 2;
    const cf4v* hq = (const cf4v*)seg_quads;
    const f4v org = hq[0];
    ax = ax - org.x; ay = ay - org.y; az = az - org.z;
    bx = bx - org.x; by = by - org.y; bz = bz - org.z;
    const bool fa = __builtin_isfinite(ax) && __builtin_isfinite(ay) && __builtin_isfinite(az);
    const bool fb = __builtin_isfinite(bx) && __builtin_isfinite(by) && __builtin_isfinite(bz);
    const cf4v* tq = hq + 4;
    const f2v ax2 = {ax, ax}, ay2 = {ay, ay}, az2 = {az, az};
    const f2v bx2 = {bx, bx}, by2 = {by, by}, bz2 = {bz, bz};
    float aA = INFINITY, aB = INFINITY, bA = INFINITY, bB = INFINITY;
    int oaA = -1, oaB = -1, obA = -1, obB = -1;
    auto qmin2 = [&](const cf4v* q, float& ma, float& mb) {
        const f4v X = q[0], Y = q[1], Z = q[2], T = q[3];
        const f2v ka = __builtin_elementwise_fma(X.xy, ax2, __builtin_elementwise_fma(Y.xy, ay2,
                                                  __builtin_elementwise_fma(Z.xy, az2, T.xy)));
        const f2v kb = __builtin_elementwise_fma(X.zw, ax2, __builtin_elementwise_fma(Y.zw, ay2,
                                                  __builtin_elementwise_fma(Z.zw, az2, T.zw)));
        ma = fminf(fminf(fminf(ka.x, ka.y), kb.x), kb.y);
        const f2v la = __builtin_elementwise_fma(X.xy, bx2, __builtin_elementwise_fma(Y.xy, by2,
                                                  __builtin_elementwise_fma(Z.xy, bz2, T.xy)));
        const f2v lb = __builtin_elementwise_fma(X.zw, bx2, __builtin_elementwise_fma(Y.zw, by2,
                                                  __builtin_elementwise_fma(Z.zw, bz2, T.zw)));
        mb = fminf(fminf(fminf(la.x, la.y), lb.x), lb.y);
    };
    int o = 0;
    const cf4v* q = tq;
#if PCORE_SCAN_PAIRQ
    // each chain compares once per PAIR of quads (8 keys): chain A takes quads o, o + 1 and chain B o + 2, o + 3 of
    // every four; a chain's index is the pair's first quad (a pair past the segment's last quad is that quad alone).
    // The first strict minimum per chain, the lower pair on a tie between chains, then the first of the pair's 8 keys
    // equal to the minimum: the same (key, index) minimum as the per-quad chains.
#pragma unroll PCORE_SCAN2_UNROLL
    for (; o + 4 <= nq; o += 4, q += 16) {
        float ma0, mb0, ma1, mb1;
        qmin2(q, ma0, mb0);
        qmin2(q + 4, ma1, mb1);
        const float pa = fminf(ma0, ma1), pb = fminf(mb0, mb1);
        if (pa < aA) { aA = pa; oaA = o; }
        if (pb < bA) { bA = pb; obA = o; }
        qmin2(q + 8, ma0, mb0);
        qmin2(q + 12, ma1, mb1);
        const float ra = fminf(ma0, ma1), rb = fminf(mb0, mb1);
        if (ra < aB) { aB = ra; oaB = o + 2; }
        if (rb < bB) { bB = rb; obB = o + 2; }
    }
    for (; o < nq; o += 2, q += 8) {  // the last one to three quads: pairs (or a lone quad) into chain A
        float ma, mb;
        qmin2(q, ma, mb);
        if (o + 1 < nq) {
            float ma1, mb1;
            qmin2(q + 4, ma1, mb1);
            ma = fminf(ma, ma1);
            mb = fminf(mb, mb1);
        }
        if (ma < aA) { aA = ma; oaA = o; }
        if (mb < bA) { bA = mb; obA = o; }
    }
#else
#pragma unroll PCORE_SCAN2_UNROLL
    for (; o + 2 <= nq; o += 2, q += 8) {
        float ma, mb;
        qmin2(q, ma, mb);
        if (ma < aA) { aA = ma; oaA = o; }
        if (mb < bA) { bA = mb; obA = o; }
        qmin2(q + 4, ma, mb);
        if (ma < aB) { aB = ma; oaB = o + 1; }
        if (mb < bB) { bB = mb; obB = o + 1; }
    }
    if (o < nq) {
        float ma, mb;
        qmin2(q, ma, mb);
        if (ma < aA) { aA = ma; oaA = o; }
        if (mb < bA) { bA = mb; obA = o; }
    }
#endif
    if (aB < aA || (aB == aA && oaB >= 0 && oaB < oaA)) { aA = aB; oaA = oaB; }
    if (bB < bA || (bB == bA && obB >= 0 && obB < obA)) { bA = bB; obA = obB; }
    auto element1 = [&](int oq, float m, float qx, float qy, float qz, int& k) {  // first key == m in quad oq, or 4
        const float* Q = seg_quads + 16 + 16 * oq;
        const float4 X = *reinterpret_cast<const float4*>(Q), Y = *reinterpret_cast<const float4*>(Q + 4);
        const float4 Z = *reinterpret_cast<const float4*>(Q + 8), T = *reinterpret_cast<const float4*>(Q + 12);
        k = gicpm::nn_key(X.x, Y.x, Z.x, T.x, qx, qy, qz) == m ? 0
          : gicpm::nn_key(X.y, Y.y, Z.y, T.y, qx, qy, qz) == m ? 1
          : gicpm::nn_key(X.z, Y.z, Z.z, T.z, qx, qy, qz) == m ? 2
          : gicpm::nn_key(X.w, Y.w, Z.w, T.w, qx, qy, qz) == m ? 3 : 4;
    };
    auto element = [&](int oq, float m, float qx, float qy, float qz) {
        int k;
        element1(oq, m, qx, qy, qz, k);
#if PCORE_SCAN_PAIRQ
        if (k == 4 && oq + 1 < nq) {  // the pair's second quad
            element1(oq + 1, m, qx, qy, qz, k);
            k += 4;
        }
#endif
        // one of the keys equals m (same FMAs); the clamp only keeps a broken match inside the segment
        return min(4 * oq + min(k, PCORE_SCAN_PAIRQ ? 7 : 3), nt - 1);
    };
    ja = fa && aA < INFINITY ? element(oaA, aA, ax, ay, az) : -1;
    jb = fb && bA < INFINITY ? element(obA, bA, bx, by, bz) : -1;
}

__device__ __forceinline__ void load_cov(const double* cov, int i, double (&c)[6]) {
    const double2* c2 = reinterpret_cast<const double2*>(cov + (size_t)6 * i);
    const double2 a = c2[0], b = c2[1], d = c2[2];
    c[0] = a.x; c[1] = a.y; c[2] = b.x; c[3] = b.y; c[4] = d.x; c[5] = d.y;
}

// a wave-uniform double moved to SGPRs (R, t of the pose being refined, the LM scalars)
__device__ __forceinline__ double uniform_d(double x) {
    const unsigned long long u = __builtin_bit_cast(unsigned long long, x);
    const unsigned lo = __builtin_amdgcn_readfirstlane((unsigned)u);
    const unsigned hi = __builtin_amdgcn_readfirstlane((unsigned)(u >> 32));
    return __builtin_bit_cast(double, ((unsigned long long)hi << 32) | lo);
}
__device__ __forceinline__ float uniform_f(float x) {
    return __builtin_bit_cast(float, __builtin_amdgcn_readfirstlane(__builtin_bit_cast(unsigned, x)));
}

// The wave shuffle-down tree of the 28 normal-equation sums (the oracle's order: node(l, off) = node(l, 2 off) +
// node(l + off, 2 off) for off = 32 ... 1, node(l, 64) = lane l's entry, so lane 0's sums ((x0 + x32) + (x16 + x48))
// + ... ), computed in registers with the values split between the halves at every level: at offset o the lanes of
// each 2o-block pair two registers A, B; the lower half adds its partner's A and keeps value A, the upper half adds
// its partner's B and keeps value B.  Lane l then holds node(l mod o, o) of half as many values, so the wave does
// 16 + 8 + 4 + 2 + 1 + 1 adds instead of 28 x 6.  The sums are the tree's own (IEEE addition commutes), whichever lane
// forms them: value v ends on lane 2 v.  Offsets 32 and 16 swap halves with v_permlane32_swap / v_permlane16_swap,
// 8 and 4 use DPP row shifts written bank by bank, 2 and 1 quad permutations.  (Round 3 transposed the partial sums
// through 7.4 KB of LDS per wave and summed them on 14 lanes: 5.6 k of ~36 k clocks per pose-iteration.)
template <int CTRL, int ROWS, int BANKS>
__device__ __forceinline__ double dpp_d(double old, double src) {
    const unsigned long long o = __builtin_bit_cast(unsigned long long, old);
    const unsigned long long v = __builtin_bit_cast(unsigned long long, src);
    const unsigned lo = __builtin_amdgcn_update_dpp((unsigned)o, (unsigned)v, CTRL, ROWS, BANKS, false);
    const unsigned hi = __builtin_amdgcn_update_dpp((unsigned)(o >> 32), (unsigned)(v >> 32), CTRL, ROWS, BANKS, false);
    return __builtin_bit_cast(double, ((unsigned long long)hi << 32) | lo);
}
template <bool ROWS16>
__device__ __forceinline__ double swap_add(double a, double b) {  // offsets 32 (ROWS16 false) and 16
    const unsigned long long ua = __builtin_bit_cast(unsigned long long, a);
    const unsigned long long ub = __builtin_bit_cast(unsigned long long, b);
    unsigned alo = (unsigned)ua, ahi = (unsigned)(ua >> 32), blo = (unsigned)ub, bhi = (unsigned)(ub >> 32);
    if constexpr (ROWS16) {
        const auto l = __builtin_amdgcn_permlane16_swap(alo, blo, false, false);
        const auto h = __builtin_amdgcn_permlane16_swap(ahi, bhi, false, false);
        alo = l[0]; blo = l[1]; ahi = h[0]; bhi = h[1];
    } else {
        const auto l = __builtin_amdgcn_permlane32_swap(alo, blo, false, false);
        const auto h = __builtin_amdgcn_permlane32_swap(ahi, bhi, false, false);
        alo = l[0]; blo = l[1]; ahi = h[0]; bhi = h[1];
    }
    return __builtin_bit_cast(double, ((unsigned long long)ahi << 32) | alo) +
           __builtin_bit_cast(double, ((unsigned long long)bhi << 32) | blo);
}
template <int OFF>
__device__ __forceinline__ double bank_add(double a, double b) {  // offsets 8 (banks 0-1 | 2-3) and 4 (0, 2 | 1, 3)
    constexpr int LOW = OFF == 8 ? 0x3 : 0x5;
    const double t = dpp_d<0x110 + OFF, 0xf, 0xf ^ LOW>(dpp_d<0x100 + OFF, 0xf, LOW>(0.0, a), b);  // row_shl / row_shr
    const double u = dpp_d<0xE4, 0xf, 0xf ^ LOW>(a, b);                                            // own value
    return u + t;
}
__device__ __forceinline__ const double* wave_tree_sums(const double (&acc)[gicpm::kTerms], double* out, int lane) {
    constexpr int K = gicpm::kTerms;
    static_assert(K > 16 && K <= 32, "28 sums: 16 register pairs at offset 32");
    double r[16];
#pragma unroll
    for (int k = 0; k < 16; k++) r[k] = swap_add<false>(acc[k], k + 16 < K ? acc[k + 16] : 0.0);
#pragma unroll
    for (int k = 0; k < 8; k++) r[k] = swap_add<true>(r[k], r[k + 8]);
#pragma unroll
    for (int k = 0; k < 4; k++) r[k] = bank_add<8>(r[k], r[k + 4]);
#pragma unroll
    for (int k = 0; k < 2; k++) r[k] = bank_add<4>(r[k], r[k + 2]);
    {  // offset 2: lanes 0-1 of a quad keep r0, lanes 2-3 r1
        const bool up = lane & 2;
        const double sel = up ? r[0] : r[1], own = up ? r[1] : r[0];
        r[0] = own + dpp_d<0x4E, 0xf, 0xf>(0.0, sel);  // quad_perm [2, 3, 0, 1]
    }
    r[0] = r[0] + dpp_d<0xB1, 0xf, 0xf>(0.0, r[0]);    // offset 1: quad_perm [1, 0, 3, 2]
    // (the slot's address formed here, not hoisted out of the iteration loop into a register that gets spilled)
    if (!(lane & 1) && (lane >> 1) < K) out[(lane >> 1) + opaque_zero()] = r[0];
    wave_lds_sync();
    return out;
}

// Lane 0's value of the wave shuffle-down tree x <- x + shfl_down(x, off), off = 32 ... 1 (the oracle's reduction
// order: ((x0 + x32) + (x16 + x48)) + ...), without the LDS pipe: the 32- and 16-lane levels through
// v_permlane32_swap / v_permlane16_swap (lane l < 32 receives lane l + 32, lane l of an even row lane l + 16), the
// 8 ... 1 levels through DPP row_shl (lane l of a row receives lane l + off).  Other lanes end with partial sums
// (read lane 0).
__device__ __forceinline__ double wave_sum_lane0(double x) {
    auto halves = [](double v, unsigned& lo, unsigned& hi) {
        const unsigned long long u = __builtin_bit_cast(unsigned long long, v);
        lo = (unsigned)u;
        hi = (unsigned)(u >> 32);
    };
    auto join = [](unsigned lo, unsigned hi) {
        return __builtin_bit_cast(double, ((unsigned long long)hi << 32) | lo);
    };
    unsigned lo, hi;
    halves(x, lo, hi);
    x = x + join(__builtin_amdgcn_permlane32_swap(lo, lo, false, false)[1],
                 __builtin_amdgcn_permlane32_swap(hi, hi, false, false)[1]);
    halves(x, lo, hi);
    x = x + join(__builtin_amdgcn_permlane16_swap(lo, lo, false, false)[1],
                 __builtin_amdgcn_permlane16_swap(hi, hi, false, false)[1]);
    halves(x, lo, hi);
    x = x + join(__builtin_amdgcn_update_dpp(0u, lo, 0x108, 0xf, 0xf, false),   // row_shl:8
                 __builtin_amdgcn_update_dpp(0u, hi, 0x108, 0xf, 0xf, false));
    halves(x, lo, hi);
    x = x + join(__builtin_amdgcn_update_dpp(0u, lo, 0x104, 0xf, 0xf, false),   // row_shl:4
                 __builtin_amdgcn_update_dpp(0u, hi, 0x104, 0xf, 0xf, false));
    halves(x, lo, hi);
    x = x + join(__builtin_amdgcn_update_dpp(0u, lo, 0x102, 0xf, 0xf, false),   // row_shl:2
                 __builtin_amdgcn_update_dpp(0u, hi, 0x102, 0xf, 0xf, false));
    halves(x, lo, hi);
    x = x + join(__builtin_amdgcn_update_dpp(0u, lo, 0x101, 0xf, 0xf, false),   // row_shl:1
                 __builtin_amdgcn_update_dpp(0u, hi, 0x101, 0xf, 0xf, false));
    return x;
}

// the pose's state in double: rotation and translation of the GICP transform (source -> target, metres)
struct Xform {
    double R[3][3];
    double t[3];
};

__device__ __forceinline__ void xform_identity(Xform& x) {
#pragma unroll
    for (int r = 0; r < 3; r++) {
#pragma unroll
        for (int c = 0; c < 3; c++) x.R[r][c] = r == c ? 1.0 : 0.0;
        x.t[r] = 0.0;
    }
}

// The first kLdsRounds rounds of source points' inputs to the trials' errors, kept in the wave's LDS (SoA,
// conflict-free): M as three double2 per point, the source point and the correspondence's target (w = 1 when the
// point has one).  Later rounds go through the per-pose scratch slots in HBM / L2.  5 KB per round and wave: two
// rounds cover C3's clouds (111 source points on average), so their trials read no HBM scratch; 10.4 KB per wave at
// 12 waves per CU is 125 KB of the CU's 160 KB.
#ifndef PCORE_GICP_LDS_ROUNDS
#define PCORE_GICP_LDS_ROUNDS 2
#endif
constexpr int kLdsPts = 64 * PCORE_GICP_LDS_ROUNDS;
// the first rounds' source points in LDS as three floats (12 B: the cycle exit's 32-slot ring fits the wave's LDS
// in the same 1,280-byte granules)
struct Pt3 {
    float x, y, z;
};

struct Round0 {
    double2 (*m)[kLdsPts];
    Pt3* s;
    float4* t;
};

// Linearisation of one round of 64 source points (point i on lane i % 64), fast_gicp linearize /
// update_correspondences: the correspondence of the float query, then -- for points with one -- the shared
// contribution into acc; the correspondence and M go to the iteration's scratch (corr[i], mah[6 i ..]) for the
// trials' errors.
template <bool STORE_CORR>
__device__ __forceinline__ void linearize_round(const Xform& x, const float (&Rf)[3][3], const float (&tf)[3],
                                                const float4* src, const double* scov, const float4* tgt,
                                                const double* tcov, int ns, int i, bool use_grid, const LabelGrid& G,
                                                const GicpArgs& g, const float* tquads, int nt, int j_in,
                                                int32_t* corr, double* mah, const Round0& r0,
                                                double (&acc)[gicpm::kTerms], bool search GPROF_PARAM) {
    GPROF_T(t_s0);
    const bool act = i < ns;
    const float4 sp = act ? src[i] : make_float4(0.0f, 0.0f, 0.0f, 0.0f);
    int j = j_in;
    if (STORE_CORR && !search) {
        j = act ? corr[i] : -1;  // the iteration's set from the correspondence history (gicp_kernel)
    } else if (STORE_CORR) {
        float qf[3];
        gicpm::query_f(Rf, tf, sp.x, sp.y, sp.z, qf);
        // correspondence: first strict minimum of the key (segments <= kKeyScanMax) or of the float squared
        // distance (grid search of larger segments), as orc_gicp
        float best = INFINITY;
        j = -1;
        if (use_grid) {
            if (act) grid_nn(G, g.cell_start, g.grid_pts, tgt, nt, qf[0], qf[1], qf[2], best, j);
        } else {
            scan_quads(tquads, nt, qf[0], qf[1], qf[2], best, j);
        }
        if (act) corr[i] = j;
    }
    GPROF_TD(t_s1, j);
    GPROF_ADD(0, t_s0, t_s1);
    const bool first = i < kLdsPts;  // a point of the rounds kept in LDS
    if (first && !(act && j >= 0)) r0.t[i] = make_float4(0.0f, 0.0f, 0.0f, 0.0f);
    if (act && j >= 0) {
        double q[3];
        gicpm::transform_point(x.R, x.t, (double)sp.x, (double)sp.y, (double)sp.z, q);
        double cs[6], ct[6], M6[6];
        load_cov(scov, i, cs);
        load_cov(tcov, j, ct);
        const float4 tj = tgt[j];
        const double t3[3] = {(double)tj.x, (double)tj.y, (double)tj.z};
        gicpm::contrib(x.R, q, cs, t3, ct, acc, M6);
        if (first) {
            r0.m[0][i] = make_double2(M6[0], M6[1]);
            r0.m[1][i] = make_double2(M6[2], M6[3]);
            r0.m[2][i] = make_double2(M6[4], M6[5]);
            r0.s[i] = Pt3{sp.x, sp.y, sp.z};
            r0.t[i] = make_float4(tj.x, tj.y, tj.z, 1.0f);
        } else {
            double2* m2 = reinterpret_cast<double2*>(mah + (size_t)6 * i);
            m2[0] = make_double2(M6[0], M6[1]);
            m2[1] = make_double2(M6[2], M6[3]);
            m2[2] = make_double2(M6[4], M6[5]);
        }
    }
    GPROF_TD(t_s2, acc[gicpm::kErr]);
    GPROF_ADD(1, t_s1, t_s2);
}


// One Levenberg-Marquardt iteration of one wave (LsqRegistration::step_lm) on the reduced system `sys` (28 sums in
// LDS: upper H, b, the error y0 at x): up to kLmMaxTrials solves of (H + lambda I) d = -b, each scored by the error
// at delta * x with the iteration's correspondences and M (point i on lane i % 64, summed by the shuffle-down tree).
// Every lane runs the same uniform arithmetic; the scalars that steer it are moved to SGPRs.
template <typename CorrPtr>
__device__ __forceinline__ int lm_iteration(const double* sys, Xform& x, double& lambda, const float4* src,
                                            CorrPtr corr, const double* mah, const float4* tgt, int ns, int lane,
                                            const Round0& r0, const lds_cvd* se3c, double rot_eps,
                                            double trans_eps, bool& inert GPROF_PARAM) {
    const double y0 = uniform_d(sys[gicpm::kErr]);
    if (lambda < 0.0) lambda = uniform_d(gicpm::lm_init_lambda(sys));
    inert = false;
    double nu = 2.0;
    for (int trial = 0; trial < gicpm::kLmMaxTrials; trial++) {
        GPROF_T(p0);
        double d[6];
        gicpm::lm_solve_schur(sys, lambda, d);
#pragma unroll
        for (int a = 0; a < 6; a++) d[a] = uniform_d(d[a]);
        GPROF_TD(p1, d[5]);
        GPROF_ADD(4, p0, p1);
        if (!gicpm::all_finite6(d)) return gicpm::kLmFailed;  // guard: a non-finite system
        double Rd[3][3], td[3];
        gicpm::se3_exp(d, Rd, td, se3c + opaque_zero());
        Xform xi;
        gicpm::compose(Rd, td, x.R, x.t, xi.R, xi.t);
#pragma unroll
        for (int r = 0; r < 3; r++) {
#pragma unroll
            for (int c = 0; c < 3; c++) xi.R[r][c] = uniform_d(xi.R[r][c]);
            xi.t[r] = uniform_d(xi.t[r]);
        }
        GPROF_TD(p2, xi.t[2]);
        GPROF_ADD(5, p1, p2);
        // the error at x_i (FastGICP::compute_error: this iteration's correspondences and Mahalanobis matrices)
        auto err_add = [&](const auto& sp, const float4& tj, const double (&M6)[6], double y) {
            double q[3];
            gicpm::transform_point(xi.R, xi.t, (double)sp.x, (double)sp.y, (double)sp.z, q);
            const double e[3] = {(double)tj.x - q[0], (double)tj.y - q[1], (double)tj.z - q[2]};
            return gicpm::mahal_err_add(M6, e, y);
        };
        double ea = 0.0;
        // the first rounds from the wave's LDS copy (written by the linearisation; a round past ns is not read), the
        // later rounds from the scratch slots
#pragma unroll
        for (int i0 = 0; i0 < kLdsPts; i0 += 64) {
            if (i0 > 0 && i0 >= ns) break;
            const int i = i0 + lane;
            const float4 t0 = r0.t[i];
            if (t0.w != 0.0f) {
                const double2 a = r0.m[0][i], b = r0.m[1][i], c = r0.m[2][i];
                const double M6[6] = {a.x, a.y, b.x, b.y, c.x, c.y};
                ea = err_add(r0.s[i], t0, M6, ea);
            }
        }
        for (int i0 = kLdsPts; i0 < ns; i0 += 64) {
            const int i = i0 + lane + opaque_zero();  // per-lane addresses formed here (hoisted, they were spilled)
            const int j = i < ns ? corr[i] : -1;
            if (j >= 0) {
                const double2* m2 = reinterpret_cast<const double2*>(mah + (size_t)6 * i);
                const double2 a = m2[0], b = m2[1], c = m2[2];
                const double M6[6] = {a.x, a.y, b.x, b.y, c.x, c.y};
                ea = err_add(src[i], tgt[j], M6, ea);
            }
        }
        const double yi = uniform_d(wave_sum_lane0(ea));  // lane 0: the tree's sum
        GPROF_TD(p3, yi);
        GPROF_ADD(6, p2, p3);
        const double rho = uniform_d(gicpm::lm_rho(sys, lambda, d, y0, yi));
        GPROF_TD(p4, rho);
        GPROF_ADD(7, p3, p4);
        if (rho < 0.0) {
            if (gicpm::is_converged(Rd, td, rot_eps, trans_eps)) return gicpm::kLmConverged;
            lambda = nu * lambda;
            nu = 2.0 * nu;
            continue;
        }
        x = xi;
        // the cycle exit's condition: accepted at the first trial, lambda not growing and inert on this system
        inert = trial == 0 && rho >= 0.5 && gicpm::lm_lambda_inert(sys, lambda);
        lambda = uniform_d(gicpm::lm_accept_lambda(lambda, rho));
        return gicpm::is_converged(Rd, td, rot_eps, trans_eps) ? gicpm::kLmConverged : gicpm::kLmAccepted;
    }
    return gicpm::kLmFailed;  // LsqRegistration: "lm not converged"
}

// concatenate_transforms (renderer.cu:1412-1429): float(T) * to_eigen(pose, 100), init_from_eigen(., 100)
__device__ __forceinline__ void write_pose(const GicpArgs& g, int gp, const Xform& x, int iters) {
    const float* pin = g.poses_in + (size_t)16 * gp;
    float A[4][4], Tf[4][4];
    for (int r = 0; r < 4; r++)
        for (int c = 0; c < 4; c++) {
            A[r][c] = r < 3 ? pin[4 * r + c] / 100.0f : pin[4 * r + c];
            Tf[r][c] = r < 3 ? (float)(c < 3 ? x.R[r][c] : x.t[r]) : (c == 3 ? 1.0f : 0.0f);
        }
    float* pout = g.poses_out + (size_t)16 * gp;
    for (int r = 0; r < 4; r++)
        for (int c = 0; c < 4; c++) {
            const float p = Tf[r][0] * A[0][c] + Tf[r][1] * A[1][c] + Tf[r][2] * A[2][c] + Tf[r][3] * A[3][c];
            pout[4 * r + c] = r < 3 ? (float)((double)p * 100) : p;
        }
    if (g.iters_out) g.iters_out[gp] = iters;
}

__device__ __forceinline__ void xform_float(const Xform& x, float (&Rf)[3][3], float (&tf)[3]) {
#pragma unroll
    for (int r = 0; r < 3; r++) {
#pragma unroll
        for (int c = 0; c < 3; c++) Rf[r][c] = uniform_f((float)x.R[r][c]);
        tf[r] = uniform_f((float)x.t[r]);
    }
}

// A 16-slot ring of float transforms in LDS (the correspondence history and the cycle exit): lane l holds components
// 3 (l & 3) + v (v = 0, 1, 2) of slot l >> 2 in word v (R rows 0..2, then t), as bit patterns (-0 != +0, NaN == NaN).
__device__ __forceinline__ void xf_lane_words(const float (&Rf)[3][3], const float (&tf)[3], int sub, unsigned& b0,
                                              unsigned& b1, unsigned& b2) {
    const float c0 = sub == 0 ? Rf[0][0] : sub == 1 ? Rf[1][0] : sub == 2 ? Rf[2][0] : tf[0];
    const float c1 = sub == 0 ? Rf[0][1] : sub == 1 ? Rf[1][1] : sub == 2 ? Rf[2][1] : tf[1];
    const float c2 = sub == 0 ? Rf[0][2] : sub == 1 ? Rf[1][2] : sub == 2 ? Rf[2][2] : tf[2];
    b0 = __builtin_bit_cast(unsigned, c0);
    b1 = __builtin_bit_cast(unsigned, c1);
    b2 = __builtin_bit_cast(unsigned, c2);
}

// bit s set: all four lanes of slot s hold (b0, b1, b2) (the lanes' current words hv0..hv2)
__device__ __forceinline__ unsigned ring_match16(unsigned b0, unsigned b1, unsigned b2, unsigned hv0, unsigned hv1,
                                                 unsigned hv2) {
    unsigned long long eq = __ballot(b0 == hv0 && b1 == hv1 && b2 == hv2);
    eq = eq & (eq >> 1) & (eq >> 2) & (eq >> 3) & 0x1111111111111111ull;  // bit 4s: slot s
    eq = (eq | (eq >> 3)) & 0x0303030303030303ull;                         // gather bit 4s to bit s
    eq = (eq | (eq >> 6)) & 0x000f000f000f000full;
    eq = (eq | (eq >> 12)) & 0x000000ff000000ffull;
    eq = (eq | (eq >> 24)) & 0xffffull;
    return (unsigned)eq;
}

// The cycle exit (pcore_gicp_math.h cycle_update) of one wave: the last 32 float transforms T_f(j) in slot
// (j - 1) % 32 of an LDS ring of two 16-slot banks (words 0..2: slots 0..15, words 3..5: slots 16..31, each bank laid out
// as xf_lane_words), the slots written so far and the run counters.
static_assert(gicpm::kCycleLags == 32, "CycleExit holds 32 slots");
constexpr int kCycleRingWords = 6 * 64;

struct CycleExit {
    unsigned* ring;  // kCycleRingWords, this wave's
    unsigned written;
    gicpm::CycleRun run;

    __device__ __forceinline__ void start(int lane) {  // T_f(1) = float(identity) in slot 0
        // lane l < 4 writes row l of I (t = 0 for l = 3): word v is 1.0f where v == l; formed here from an opaque lane
        // index, or the compiler hoists the words and addresses out of the persistent pose loop and holds 4 VGPRs
        const int l = lane + opaque_zero();
        if (l < 4) {  // every lane reads back only the words it wrote itself
            ring[l] = l == 0 ? 0x3f800000u : 0u;
            ring[64 + l] = l == 1 ? 0x3f800000u : 0u;
            ring[128 + l] = l == 2 ? 0x3f800000u : 0u;
        }
        written = 1u;
        run = {0, 0, 0};
    }

    // after iteration `iters`' accepted step (iters < max_iter): T_f(iters + 1) = float(x).  Returns -1, or the ring slot
    // of the cycle member the pose stops with (read by `member` once the loop has ended).
    __device__ __forceinline__ int step(const Xform& x, int iters, int max_iter, int window, bool inert, int lane_) {
        const int lane = lane_ + opaque_zero();  // per-lane values formed here, not hoisted out of the iteration loop
        float Rf[3][3], tf[3];
        xform_float(x, Rf, tf);
        unsigned b0, b1, b2;
        xf_lane_words(Rf, tf, lane & 3, b0, b1, b2);
        const int cur = iters + 1, c0 = (cur - 1) & 31, bank = c0 >> 4;
        const unsigned m0 = ring_match16(b0, b1, b2, ring[lane], ring[64 + lane], ring[128 + lane]);
        const unsigned m1 = ring_match16(b0, b1, b2, ring[192 + lane], ring[256 + lane], ring[320 + lane]);
        const unsigned m = (m0 | (m1 << 16)) & written;
        // lag q lives in slot (c0 - q) % 32: in the doubled mask at c0 + 32 - q, so the smallest lag is the highest bit
        const unsigned long long mm = (unsigned long long)m | ((unsigned long long)m << 32);
        const unsigned t = (unsigned)(mm >> c0);
        const int p = t ? 32 - (31 - __builtin_clz(t)) : 0;
        if ((lane >> 2) == (c0 & 15)) {
            unsigned* w = ring + 192 * bank + lane;
            w[0] = b0;
            w[64] = b1;
            w[128] = b2;
        }
        written |= 1u << c0;
        if (!gicpm::cycle_update(run, p, inert, window)) return -1;
        return (gicpm::cycle_member(cur, p, max_iter) - 1) & 31;
    }

    // the float transform of ring slot s as the pose's result (after the loop: x is written back, not iterated on; the
    // ring was written by the whole wave, read here by every lane)
    __device__ __forceinline__ void member(int s, Xform& x) {
        wave_lds_sync();
        const unsigned* w = ring + 192 * (s >> 4) + 4 * (s & 15);
#pragma unroll
        for (int r = 0; r < 4; r++)
#pragma unroll
            for (int v = 0; v < 3; v++) {
                const double f = (double)__builtin_bit_cast(float, w[64 * v + r]);
                if (r < 3) x.R[r][v] = f;
                else x.t[v] = f;
            }
    }
};

// the launch's iteration counters (GicpArgs::iter_stats): no-return atomics, one lane per pose
__device__ __forceinline__ void count_iterations(const GicpArgs& g, int reported, int run, bool exited) {
    if (!g.iter_stats) return;
    __hip_atomic_fetch_add(g.iter_stats + 0, (unsigned long long)reported, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __hip_atomic_fetch_add(g.iter_stats + 1, (unsigned long long)run, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (exited) __hip_atomic_fetch_add(g.iter_stats + 2, 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// the pose a GICP workgroup works on next and its target segment
struct GicpPose {
    int pose, gp, ns, nt, seg;
    const float4* src;
    const double* scov;
    const double* tcov;
    const float4* tgt;
    const float* tquads;
    int32_t* corr;
    double* mah;
    bool use_grid;
};

__device__ __forceinline__ GicpPose gicp_pose(const GicpArgs& g, int pose) {
    GicpPose p;
    p.pose = pose;
    p.gp = g.pose_base + pose;
    p.ns = g.src_count[pose];
    p.src = g.src + (size_t)pose * g.src_cap;
    p.scov = g.src_cov + (size_t)6 * pose * g.src_cap;
    p.corr = g.corr + (size_t)pose * g.src_cap;
    p.mah = g.mahal + (size_t)6 * pose * g.src_cap;
    int seg = g.whole_seg;
    if (g.pose_label) {
        const int pl = g.pose_label[p.gp];
        seg = (pl >= 0 && pl < g.num_segs) ? pl : -1;
    }
    seg = __builtin_amdgcn_readfirstlane(seg);
    p.seg = seg;
    const int lo = seg >= 0 ? g.seg_lo[seg] : 0;
    p.nt = seg >= 0 ? g.seg_hi[seg] - lo : 0;
    p.tcov = g.tgt_cov + (size_t)6 * lo;
    p.tgt = g.tgt + lo;
    p.tquads = g.tgt_quads + (seg >= 0 ? (size_t)16 * g.seg_qoff[seg] : 0);
    p.use_grid = seg >= 0 && segment_uses_grid(p.nt, g.grids != nullptr);  // exact grid shell search
    return p;
}

constexpr int kCycleExited = 3;  // coop_pose's flag: wave 0's cycle exit stopped the pose (LmStatus + 1)

// One pose by the NW waves of a workgroup (gicp_wide_kernel's poses; gicp_kernel's heavy poses): every wave searches
// the iteration's correspondences of rounds r = wave (mod NW) into `corr`, then wave 0 adds the contributions and runs
// the LM iteration exactly as the one-wave path does -- point i on lane i % 64, in point order -- so the refined pose
// is bit-identical; x and the iteration's outcome reach the other waves through LDS (sX, sFlag).  `r0`, `sRed`, `ring`:
// wave 0's LDS.  Every thread of the workgroup calls this; thread 0 writes the pose.
template <bool GRID, int NW, typename Corr>
__device__ __forceinline__ void coop_pose(const GicpArgs& g, const GicpPose& P, int wave, int lane, Corr corr,
                                          double* sRed, const Round0& r0, const lds_cvd* se3c, unsigned* ring,
                                          double* sX, int* sFlag GPROF_PARAM) {
    constexpr int NT = 64 * NW;
    const int tid = wave * 64 + lane;
#ifdef PCORE_GICP_TIMELINE
    const unsigned long long tl_p0 = __builtin_amdgcn_s_memrealtime();
#endif
    LabelGrid G{};
    if (GRID && P.use_grid) G = g.grids[P.seg];
    Xform x;
    xform_identity(x);
    double lambda = -1.0;  // wave 0's
    int iters = 0, iters_run = 0;
    CycleExit cyc;  // wave 0's
    cyc.ring = ring;
    if (wave == 0) cyc.start(lane);
    const bool run = P.ns > 0 && P.nt > 0;
    for (int it = 0; run && it < g.max_iter; it++) {
        iters++;
        float Rf[3][3], tf[3];
        xform_float(x, Rf, tf);
        GPROF_T(t_w0);
        // correspondences, all waves
        for (int i0 = wave * 64; i0 < P.ns; i0 += NT) {
            const int i = i0 + lane;
            const bool act = i < P.ns;
            const float4 sp = act ? P.src[i] : make_float4(0.0f, 0.0f, 0.0f, 0.0f);
            float qf[3];
            gicpm::query_f(Rf, tf, sp.x, sp.y, sp.z, qf);
            int j = -1;
            float best = INFINITY;
            if (GRID && P.use_grid) {
                if (act) grid_nn(G, g.cell_start, g.grid_pts, P.tgt, P.nt, qf[0], qf[1], qf[2], best, j);
            } else {
                scan_quads(P.tquads, P.nt, qf[0], qf[1], qf[2], best, j);
            }
            if (act) corr[i] = j;
        }
        __syncthreads();
        GPROF_TD(t_w1, Rf[0][0]);
        GPROF_ADD(0, t_w0, t_w1);
        if (wave == 0) {
            double acc[gicpm::kTerms];
#pragma unroll
            for (int v = 0; v < gicpm::kTerms; v++) acc[v] = 0.0;
            for (int i0 = 0; i0 < P.ns; i0 += 64) {
                const int i = i0 + lane;
                linearize_round<false>(x, Rf, tf, P.src, P.scov, P.tgt, P.tcov, P.ns, i, P.use_grid, G, g, P.tquads,
                                       P.nt, i < P.ns ? corr[i] : -1, nullptr, P.mah, r0, acc, false GPROF_ARG);
            }
            GPROF_TD(t_w2, acc[0]);
            const double* sys = wave_tree_sums(acc, sRed, lane);
            GPROF_TD(t_w3, sys[0]);
            bool inert;
            int st = lm_iteration(sys, x, lambda, P.src, corr, P.mah, P.tgt, P.ns, lane, r0, se3c, g.rot_eps,
                                  g.trans_eps, inert GPROF_ARG);
            GPROF_TD(t_w4, st);
            GPROF_ADD(2, t_w2, t_w3);  // [1]: linearize_round's own marks
            GPROF_ADD(3, t_w3, t_w4);
            if (st == gicpm::kLmAccepted && g.cycle_window > 0 && iters < g.max_iter) {
                const int s2 = cyc.step(x, iters, g.max_iter, g.cycle_window, inert, lane);
                if (s2 >= 0) {
                    cyc.member(s2, x);
                    st = kCycleExited;
                }
            }
            if (lane == 0) {
                *sFlag = st;
#pragma unroll
                for (int r = 0; r < 3; r++) {
#pragma unroll
                    for (int c = 0; c < 3; c++) sX[3 * r + c] = x.R[r][c];
                    sX[9 + r] = x.t[r];
                }
            }
        }
        __syncthreads();
        const int flag = __builtin_amdgcn_readfirstlane(*sFlag);
#pragma unroll
        for (int r = 0; r < 3; r++) {
#pragma unroll
            for (int c = 0; c < 3; c++) x.R[r][c] = uniform_d(sX[3 * r + c]);
            x.t[r] = uniform_d(sX[9 + r]);
        }
        if (flag == kCycleExited) {
            iters_run = iters;
            iters = g.max_iter;
        }
        if (flag != gicpm::kLmAccepted) break;
    }
    __syncthreads();
    if (tid == 0) {
        write_pose(g, P.gp, x, iters);
        count_iterations(g, iters, iters_run ? iters_run : iters, iters_run != 0);
#ifdef PCORE_GICP_TIMELINE
        if (P.gp < kTlPoses) {
            g_tl_pose[2 * P.gp] = tl_p0;
            g_tl_pose[2 * P.gp + 1] = __builtin_amdgcn_s_memrealtime();
            g_tl_run[P.gp] = iters_run ? iters_run : iters;
        }
#endif
    }
}

// ------------------------------------------------------------------------------------------------
// The help board (GicpArgs::help_*; VERDICT r05 next #5, the launch's queue-dry tail).  Once the pose queue has run
// dry, the waves that find it empty become helpers, and the waves still refining a pose of kHelpMinRounds or more
// rounds of 64 source points (each looks at the board's dry word every iteration: one load, read an iteration later)
// list themselves on the board.  The first helper to enlist a listed pose zeroes its slot's granules and raises the
// slot's flag; from the next iteration on the owner shares each searching iteration's correspondence search with up to
// rounds - 1 helpers, by rounds of 64 points (help_search, help_attached).  A wave's slot is its workgroup index.
// Hand-offs between workgroups take the R2 form of cdna_hip_programming.md section 6, guideline 16: every shared value
// travels in an 8-byte granule {tag, value} written by one agent-scope atomic store and polled by agent-scope atomic
// loads until its tag matches, so no fence is needed.  A tag is the launch's tag (GicpArgs::help_tag) and the epoch: a
// wave that has seen the queue dry takes no further pose, so a slot is helped for one pose at most, and the epoch of
// the pose's iteration `it` is it + 1, so epochs only grow.  The results are the owner's own search's bit for bit: a
// helper runs the same float queries (the published bits) through the same scan.  Every wait is bounded
// (kHelpTimeoutTicks of the 100 MHz clock): an owner whose helper is late searches that round itself, a helper whose
// owner has moved on gives up, and every helper leaves once all of the launch's poses are written (or after
// kHelpLifeTicks).  Measured: owners that registered from every fourth iteration with a zeroing loop of their own cost
// the iteration loop 8 VGPRs; helpers that scanned every wave's posted pose instead of a list slowed the launch.
typedef __attribute__((address_space(1))) unsigned gu32;
typedef __attribute__((address_space(1))) unsigned long long gu64;
constexpr unsigned long long kHelpTimeoutTicks = 200000;   // 2 ms
constexpr unsigned long long kHelpLifeTicks = 100000000;  // 1 s
#ifndef PCORE_HELP_MIN_ROUNDS
#define PCORE_HELP_MIN_ROUNDS 3
#endif
constexpr int kHelpMinRounds = PCORE_HELP_MIN_ROUNDS;  // two rounds: one helper saves about what the hand-offs cost


__device__ __forceinline__ unsigned hb_load(const unsigned* p) {
    return __hip_atomic_load((gu32*)p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ unsigned long long hb_load64(const unsigned long long* p) {
    return __hip_atomic_load((gu64*)p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void hb_store(unsigned* p, unsigned v) {
    __hip_atomic_store((gu32*)p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void hb_store64(unsigned long long* p, unsigned long long v) {
    __hip_atomic_store((gu64*)p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ unsigned hb_add(unsigned* p, unsigned v) {
    return __hip_atomic_fetch_add((gu32*)p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
// The board's arguments, read from the kernarg segment where they are used (behind an opaque offset): as kernel
// arguments held in registers they were live through the whole persistent loop, for code that runs in the tail only.
struct HelpRef {
    unsigned* ctl;
    unsigned long long* gran;
    unsigned long long* stats;
    int slots, cap;
    unsigned tag;  // the launch's tag (GicpArgs::help_tag, 1..0xFFFF)
};
__device__ __forceinline__ HelpRef help_ref() {
    typedef __attribute__((address_space(4))) const GicpArgs kargs_t;
    typedef __attribute__((address_space(4))) const char kbytes_t;
    kargs_t* a = (kargs_t*)((kbytes_t*)__builtin_amdgcn_kernarg_segment_ptr() + opaque_zero());  // gicp_kernel's g
    return {a->help_ctl, a->help_gran, a->help_stats, a->help_slots, a->src_cap, a->help_tag};
}
// The covariance prologue's arguments (GicpArgs::cov_fold), read from the kernarg segment at each pose in the same way:
// as registers they were live through the iteration loop (146 -> 167 VGPRs, 96 -> 149 SGPRs spilled)
struct CovFoldRef {
    double* out;
    CovGrid cg;
};
__device__ __forceinline__ CovFoldRef cov_fold_ref() {
    typedef __attribute__((address_space(4))) const GicpArgs kargs_t;
    typedef __attribute__((address_space(4))) const char kbytes_t;
    kargs_t* a = (kargs_t*)((kbytes_t*)__builtin_amdgcn_kernarg_segment_ptr() + opaque_zero());  // gicp_kernel's g
    return {a->cov_fold, {a->cov_fx, a->cov_fy, a->cov_cx, a->cov_cy, a->cov_stride}};
}
__device__ __forceinline__ void hb_count(const HelpRef& h, int k) {
    if (h.stats) __hip_atomic_fetch_add((gu64*)(h.stats + k), 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
// control words after [0] dry, [1] poses finished, [2] poses listed, [3] unused: per list entry the listed slot
// ((rounds << 24) | (slot + 1)) and its helpers (kHelpFull once its pose is done); per slot its claim word and flag
constexpr unsigned kHelpFull = 0xFFFFu;
__device__ __forceinline__ int hb_stride(const HelpRef& h) { return (h.slots + 3) & ~3; }
__device__ __forceinline__ unsigned* hb_list(const HelpRef& h) { return h.ctl + 4; }
__device__ __forceinline__ unsigned* hb_helpers(const HelpRef& h) { return h.ctl + 4 + hb_stride(h); }
__device__ __forceinline__ unsigned* hb_claim(const HelpRef& h) { return h.ctl + 4 + 2 * hb_stride(h); }
__device__ __forceinline__ unsigned* hb_flag(const HelpRef& h) { return h.ctl + 4 + 3 * hb_stride(h); }
__device__ __forceinline__ unsigned long long* hb_gran(const HelpRef& h, int slot) {
    return h.gran + (size_t)slot * (kHelpXfGranules + h.cap);
}
__device__ __forceinline__ unsigned long long hb_now() { return __builtin_amdgcn_s_memrealtime(); }
// a granule's tag: the launch's tag and the epoch (a granule left by an earlier launch never matches)
__device__ __forceinline__ unsigned hb_tag(const HelpRef& h, unsigned e) { return (h.tag << 16) | e; }

// round r's correspondences (point 64 r + lane), exactly as the iteration's own search finds them
__device__ __forceinline__ int help_round_scan(const GicpPose& P, int r, const float (&Rf)[3][3], const float (&tf)[3],
                                               int lane) {
    const int i = 64 * r + lane;
    int j = -1;
    if (i < P.ns) {
        const float4 sp = P.src[i];
        float q[3];
        gicpm::query_f(Rf, tf, sp.x, sp.y, sp.z, q);
        float best = INFINITY;
        scan_quads(P.tquads, P.nt, q[0], q[1], q[2], best, j);
    }
    return j;
}

// The owner's side before its pose is shared, once an iteration (hstate: -1 = watching the dry word, -3 = listed,
// watching its flag; >= 0 = the slot, shared).  `hv` is the word loaded at the previous iteration (read here, so its
// latency hides behind an iteration), reloaded for the next one.
__device__ __forceinline__ void help_watch(int& hstate, unsigned& hv, int np, int lane) {
    const HelpRef g = help_ref();
    const int w = blockIdx.x;
    if (__builtin_amdgcn_readfirstlane(hv)) {
        if (hstate == -3) {  // enlisted: the slot's granules are zeroed
            hstate = w;
            return;
        }
        if (w >= g.slots) {  // no slot of its own (a board smaller than the launch)
            hstate = -2;
            return;
        }
        unsigned k = 0;  // the queue ran dry: list the pose
        if (lane == 0) k = hb_add(g.ctl + 2, 1u);
        k = __builtin_amdgcn_readfirstlane(k);
        if ((int)k >= g.slots) {
            hstate = -2;
            return;
        }
        if (lane == 0) hb_store(hb_list(g) + k, ((unsigned)np << 24) | (unsigned)(w + 1));
        hstate = -3;
        hv = 0u;
    }
    if (lane == 0) hv = hb_load(hstate == -3 ? hb_flag(g) + w : g.ctl);
}

// An enlisted pose's search of one iteration (epoch e) into cset: the transform published in the slot's granules,
// round 0 searched by the owner, every further round claimed from the slot's counter by whoever asks first (the
// owner included); the rounds helpers took are read from their granules.
__device__ __forceinline__ void help_search(const GicpPose& P, int s, unsigned e, const float (&Rf)[3][3],
                                            const float (&tf)[3], int32_t* cset, int lane) {
    const HelpRef g = help_ref();
    const int npass = (P.ns + 63) >> 6;
    unsigned long long* gr = hb_gran(g, s);
    unsigned* claim = hb_claim(g) + s;
    const unsigned long long T = (unsigned long long)hb_tag(g, e) << 32;
    if (lane < 4) {  // granule 3 r + c: row r of R (r = 3: t), as xf_lane_words lays them out (no indexed selects)
        unsigned b0, b1, b2;
        xf_lane_words(Rf, tf, lane, b0, b1, b2);
        hb_store64(gr + 3 * lane, T | b0);
        hb_store64(gr + 3 * lane + 1, T | b1);
        hb_store64(gr + 3 * lane + 2, T | b2);
    } else if (lane < 6) {  // granules 12, 13: the pose and its rounds
        hb_store64(gr + 8 + lane, T | (lane == 4 ? (unsigned)P.pose + 1u : (unsigned)npass));
    }
    if (lane == 0) hb_store(claim, (e << 16) | 1u);  // round 0 is the owner's
    unsigned long long mine0 = 0ull, mine1 = 0ull;
    int c = 0;
    for (;;) {
        const int j = help_round_scan(P, c, Rf, tf, lane);
        if (64 * c + lane < P.ns) cset[64 * c + lane] = j;
        if (c < 64) mine0 |= 1ull << c;
        else mine1 |= 1ull << (c - 64);
        unsigned old = 0;
        if (lane == 0) old = hb_add(claim, 1u);
        old = __builtin_amdgcn_readfirstlane(old);
        if ((old >> 16) != e || (int)(old & 0xffffu) >= npass) break;
        c = (int)(old & 0xffffu);
    }
    for (int r = 1; r < npass; r++) {
        if (((r < 64 ? mine0 >> r : mine1 >> (r - 64)) & 1ull) != 0ull) continue;
        const int i = 64 * r + lane;
        const bool act = i < P.ns;
        const unsigned long long t0 = hb_now();
        unsigned long long v = 0ull;
        bool got = false;
        for (;;) {
            if (act) v = hb_load64(gr + kHelpXfGranules + i);
            if (__ballot(act && (v >> 32) != (T >> 32)) == 0ull) {
                got = true;
                break;
            }
            if (hb_now() - t0 > kHelpTimeoutTicks) break;
            __builtin_amdgcn_s_sleep(1);
        }
        if (got) {
            if (act) cset[i] = (int32_t)(unsigned)v;
        } else {  // the helper is late: the owner searches the round (the same correspondences)
            const int j = help_round_scan(P, r, Rf, tf, lane);
            if (act) cset[i] = j;
            if (lane == 0) hb_count(g, 1);
        }
    }
}

// A helper attached to slot s: claims rounds of the published epochs until the pose is done.
__device__ __forceinline__ void help_attached(const GicpArgs& ga, const HelpRef& g, int s, int np, int lane,
                                              unsigned long long born) {
    unsigned long long* gr = hb_gran(g, s);
    unsigned* claim = hb_claim(g) + s;
    for (;;) {
        unsigned w = 0;
        if (lane == 0) w = hb_load(claim);
        w = __builtin_amdgcn_readfirstlane(w);
        if ((w >> 16) == 0xFFFFu || hb_now() - born > kHelpLifeTicks) return;
        if ((w >> 16) == 0u || (int)(w & 0xffffu) >= np) {
            __builtin_amdgcn_s_sleep(2);
            continue;
        }
        if (lane == 0) w = hb_add(claim, 1u);
        w = __builtin_amdgcn_readfirstlane(w);
        const unsigned e = w >> 16;
        const int c = (int)(w & 0xffffu);
        if (e == 0u || e == 0xFFFFu || c >= np) continue;
        // the transform and pose of epoch e (their granules may land after the claim word)
        const unsigned T = hb_tag(g, e);
        const unsigned long long t0 = hb_now();
        unsigned bits = 0;
        bool ok = false;
        for (;;) {
            unsigned long long v = 0ull;
            if (lane < 14) v = hb_load64(gr + lane);
            const unsigned tag = (unsigned)(v >> 32);
            // the owner has moved on (this launch's tag, a later epoch)
            if (__ballot(lane < 14 && (tag >> 16) == g.tag && (tag & 0xffffu) > e) != 0ull) break;
            if (__ballot(lane < 14 && tag != T) == 0ull) {
                bits = (unsigned)v;
                ok = true;
                break;
            }
            if (hb_now() - t0 > kHelpTimeoutTicks) break;
            __builtin_amdgcn_s_sleep(1);
        }
        if (!ok) {
            if (lane == 0) hb_count(g, 2);
            continue;
        }
        float Rf[3][3], tf[3];
#pragma unroll
        for (int a = 0; a < 3; a++) {
#pragma unroll
            for (int b = 0; b < 3; b++) Rf[a][b] = __builtin_bit_cast(float, __builtin_amdgcn_readlane(bits, 3 * a + b));
            tf[a] = __builtin_bit_cast(float, __builtin_amdgcn_readlane(bits, 9 + a));
        }
        const GicpPose P = gicp_pose(ga, (int)__builtin_amdgcn_readlane(bits, 12) - 1);
        const int j = help_round_scan(P, c, Rf, tf, lane);
        if (64 * c + lane < P.ns)
            hb_store64(gr + kHelpXfGranules + 64 * c + lane, ((unsigned long long)T << 32) | (unsigned)j);
        if (lane == 0) hb_count(g, 0);
    }
}

// A wave whose queue ran dry: marks the queue dry, then helps listed poses (a pose of np rounds takes np - 1 helpers;
// the first to enlist zeroes the slot's granules, drains the stores, then raises the flag) until every pose of the
// launch is written.
__device__ __forceinline__ void help_loop(const GicpArgs& ga, int num_poses, int lane) {
    const HelpRef g = help_ref();
    if (lane == 0) hb_store(g.ctl, 1u);
    const unsigned long long born = hb_now();
    const unsigned* list = hb_list(g);
    unsigned* helpers = hb_helpers(g);
    for (;;) {
        unsigned fin = 0, nl = 0;
        if (lane == 0) {
            fin = hb_load(g.ctl + 1);
            nl = hb_load(g.ctl + 2);
        }
        fin = __builtin_amdgcn_readfirstlane(fin);
        const int n = min((int)__builtin_amdgcn_readfirstlane(nl), g.slots);
        if ((int)fin >= num_poses || hb_now() - born > kHelpLifeTicks) return;
        int slot = -1, np = 0;
        for (int b = 0; b < n && slot < 0; b += 64) {
            const int k = b + lane;
            unsigned e = 0, h = kHelpFull;
            if (k < n) {
                e = hb_load(list + k);
                h = hb_load(helpers + k);
            }
            const int npk = (int)(e >> 24);
            unsigned long long m = __ballot(e != 0u && h != kHelpFull && (int)h < npk - 1);
            while (m != 0ull) {
                const int l = __builtin_ctzll(m);
                m &= m - 1ull;
                const unsigned el = __builtin_amdgcn_readlane(e, l);
                const int npl = (int)(el >> 24), sl = (int)(el & 0xFFFFFFu) - 1;
                unsigned cw = 0;  // a pose that is done: its entry marked full for everyone
                if (lane == 0) cw = hb_load(hb_claim(g) + sl);
                if ((__builtin_amdgcn_readfirstlane(cw) >> 16) == 0xFFFFu) {
                    if (lane == 0) hb_store(helpers + b + l, kHelpFull);
                    continue;
                }
                unsigned got = 0;
                if (lane == 0) got = hb_add(helpers + b + l, 1u);
                got = __builtin_amdgcn_readfirstlane(got);
                if ((int)got < npl - 1) {
                    slot = sl;
                    np = npl;
                    if (got == 0u) {  // the first helper: the slot's granules zeroed and drained, then the flag
                        unsigned long long* gr = hb_gran(g, slot);
                        if (lane < kHelpXfGranules) hb_store64(gr + lane, 0ull);
                        for (int i = lane; i < 64 * np; i += 64) hb_store64(gr + kHelpXfGranules + i, 0ull);
                        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
                        if (lane == 0) {
                            hb_store(hb_flag(g) + slot, 1u);
                            hb_count(g, 3);
                        }
                    }
                    break;
                }
            }
        }
        if (slot < 0) {
            __builtin_amdgcn_s_sleep(127);
            continue;
        }
        help_attached(ga, g, slot, np, lane, born);
    }
}

// One wave per pose; persistent waves pull poses from a counter.  Each iteration linearises in rounds of 64
// source points (point i -> lane i % 64, contributions added in point order), reduces the 28 terms by the
// shuffle-down tree in registers and runs the LM iteration on the wave.  The per-pose iteration chain is
// latency-bound, so the slowest pose sets a chunk's tail (the queue is ordered longest first).
#ifndef PCORE_GICP_WAVES_PER_EU
#define PCORE_GICP_WAVES_PER_EU 3
#endif
#ifndef PCORE_GICP_NO_COOP
#define PCORE_GICP_NO_COOP 0  // register-budget experiments: the kernel without the heavy-pose phase
#endif

// GRID: the kernel holds the exact grid search of large segments (> kGridNNMin targets).  launch_gicp picks the
// instance without it when no segment of the observation is that large (every C2-C5 label): the search's registers
// then weigh on no pose (gicp_kernel 12.1 -> 11.9 ms per C3 call).
// NW: waves per workgroup.  The heaviest poses of the queue (GicpArgs::heavy_count, the first entries of the cost
// order) are refined first, each by a whole workgroup (coop_pose: the NW waves split the correspondence search, the
// part that grows with points x targets); then every wave pulls the remaining poses one at a time.  A heavy chain that
// runs all its iterations alone outlasted the rest of the launch (the queue-dry tail).
template <bool GRID, int NW>
__global__ void __launch_bounds__(64 * NW) __attribute__((amdgpu_waves_per_eu(PCORE_GICP_WAVES_PER_EU)))
gicp_kernel(GicpArgs g, int num_poses) {
    __shared__ double sRedA[NW][gicpm::kTerms];
    __shared__ double2 sM0A[NW][3][kLdsPts];
    __shared__ Pt3 sS0A[NW][kLdsPts];
    __shared__ float4 sT0A[NW][kLdsPts];
    __shared__ int sPoseA[NW];
    __shared__ double sSe3[4 * gicpm::kSe3Terms];  // se3_exp's series coefficients, read at their use
    __shared__ unsigned sHistA[NW][3 * 64];          // the correspondence history's float transforms (below)
    __shared__ unsigned sCycA[NW][kCycleRingWords];  // the cycle exit's last 32 float transforms (CycleExit)
    __shared__ double sX[12];                         // coop_pose's broadcast of x and the iteration's outcome
    __shared__ int sFlag, sCoop;
    const int wave = NW > 1 ? __builtin_amdgcn_readfirstlane(threadIdx.x >> 6) : 0;
    const int lane = threadIdx.x & 63;
    double* const sRed = sRedA[wave];
    int* const pPose = &sPoseA[wave];
    unsigned* const sHist = sHistA[wave];
    unsigned* const sCyc = sCycA[wave];
    const Round0 r0{sM0A[wave], sS0A[wave], sT0A[wave]};
    if (threadIdx.x < 4 * gicpm::kSe3Terms) sSe3[threadIdx.x] = gicpm::kSe3Coef[threadIdx.x];
    GPROF_DECL;
#ifdef PCORE_GICP_TIMELINE
    const unsigned long long tl_w0 = __builtin_amdgcn_s_memrealtime();
#endif
    int nheavy = 0;
    if constexpr (NW > 1 && !PCORE_GICP_NO_COOP) {
        __syncthreads();  // sSe3 written by the first waves' lanes
        if (g.heavy_count && g.pose_order)
            nheavy = __builtin_amdgcn_readfirstlane(min(min(*g.heavy_count, g.heavy_max), num_poses));
        for (;;) {
            __syncthreads();  // the previous heavy pose is written and sCoop read
            if (threadIdx.x == 0) {
                const int q = atomicAdd(g.heavy_counter, 1);
                sCoop = q < nheavy ? g.pose_order[q] : -1;
            }
            __syncthreads();
            const int pose = __builtin_amdgcn_readfirstlane(sCoop);
            if (pose < 0) break;
            const GicpPose P = gicp_pose(g, pose);
            if (!GRID && P.use_grid && threadIdx.x == 0 && g.iter_stats)
                __hip_atomic_fetch_add(g.iter_stats + 3, 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            coop_pose<GRID, NW>(g, P, wave, lane, P.corr, sRedA[0], Round0{sM0A[0], sS0A[0], sT0A[0]},
                                (const lds_cvd*)sSe3, sCycA[0], sX, &sFlag GPROF_ARG);
        }
    }
    for (;;) {
        wave_lds_sync();  // the previous pose's reads of sPose are done
        if (lane == 0) {
            // the poses after the heavy ones, in the cost order
            const int q = atomicAdd(g.work_counter, 1) + nheavy;
            *pPose = (g.pose_order && q < num_poses) ? g.pose_order[q] : q;
        }
        wave_lds_sync();
        const int pose = __builtin_amdgcn_readfirstlane(*pPose);  // chunk-local, uniform
        if (pose >= num_poses) break;
        const GicpPose P = gicp_pose(g, pose);
        if (!GRID && P.use_grid && lane == 0 && g.iter_stats)  // the host picked the instance without the search
            __hip_atomic_fetch_add(g.iter_stats + 3, 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (const CovFoldRef cf = cov_fold_ref(); cf.out) {
            // the pose's source covariances first, in the LDS of its first rounds' trial inputs (written only by the
            // linearisation below): covariance_cloud_kernel's code, so bit-identical; point i's covariance is
            // written and later read by lane i % 64
            static_assert(kThrLdsBytes <= sizeof(sM0A[0]), "the covariance scratch fits the wave's trial-input LDS");
            cov_cloud_segment_call(P.src, P.ns, cf.cg, lane, reinterpret_cast<unsigned char*>(&sM0A[wave][0][0]),
                              cf.out + (size_t)6 * pose * g.src_cap);
            wave_lds_sync();
        }
#ifdef PCORE_GICP_TIMELINE
        const unsigned long long tl_p0 = __builtin_amdgcn_s_memrealtime();
#endif
#ifdef PCORE_GICP_PROFILE
        unsigned long long gp_snap[kGprof];  // the sums before this pose (restored if the pose is below the size filter)
        for (int k_ = 0; k_ < kGprof; k_++) gp_snap[k_] = gp_acc[k_];
#endif
        const LabelGrid G{};  // linearize_round's grid argument, unused here: the searches below load the grid
        Xform x;
        xform_identity(x);
        double lambda = -1.0;
        int iters = 0, iters_run = 0, exit_slot = -1;
        CycleExit cyc;
        cyc.ring = sCyc;
        cyc.start(lane);
        // correspondence history: sHist[64 v + l] holds component 3 (l & 3) + v (v = 0, 1, 2) of set l >> 2's float
        // transform (R rows 0..2, then t); `kept` has bit 4e set for every filled set e (the words of unfilled sets
        // are never compared).  In LDS rather than in three VGPRs per lane: the kernel is at its register budget,
        // and a history word held in a VGPR was spilled to scratch and reloaded behind a vmcnt(0) every iteration.
        const bool hist = g.corr_hist != nullptr && P.ns <= g.corr_hist_cap;
        int32_t* const hbase = hist ? g.corr_hist + (size_t)pose * kCorrHist * g.corr_hist_cap : nullptr;
        unsigned long long kept = 0ull;
        int ring = 0;
        const int sub = lane & 3;
        // the help board (one-wave workgroups; help_watch): -2 = no help, -1 / -3 = watching, else the slot
        int hslot = -2;
        unsigned hv = 0u;  // the board word loaded at an iteration's top, read at the next one's
        if constexpr (kGicpHelpBoard && NW == 1 && !GRID)  // the grid instance keeps its registers for the search
            if (P.ns > 64 * (kHelpMinRounds - 1) && P.ns <= 64 * kHelpMaxRounds && !P.use_grid && g.max_iter < 0xFFFF &&
                help_ref().ctl)
                hslot = -1;
        if (P.ns > 0 && P.nt > 0) {
            for (int it = 0; it < g.max_iter; it++) {
                iters++;
                float Rf[3][3], tf[3];
                xform_float(x, Rf, tf);
                int32_t* cset = P.corr;
                bool reuse = false;
                if (hist) {
                    unsigned b0, b1, b2;
                    xf_lane_words(Rf, tf, sub, b0, b1, b2);
                    // bitwise equality (-0 != +0, NaN == NaN): the float queries, and so the correspondences, are
                    // functions of these bits
                    const unsigned hv0 = sHist[lane], hv1 = sHist[64 + lane], hv2 = sHist[128 + lane];
                    const unsigned long long eq = __ballot(b0 == hv0 && b1 == hv1 && b2 == hv2);
                    const unsigned long long full = eq & (eq >> 1) & (eq >> 2) & (eq >> 3) & kept;
                    int e;
                    if (full != 0ull) {
                        e = __builtin_ctzll(full) >> 2;
                        reuse = true;
                    } else {
                        e = ring;
                        ring = ring + 1 == kCorrHist ? 0 : ring + 1;
                        kept |= 1ull << (4 * e);
                        if ((lane >> 2) == e) {  // every lane reads back only the words it wrote itself
                            sHist[lane] = b0;
                            sHist[64 + lane] = b1;
                            sHist[128 + lane] = b2;
                        }
                    }
                    cset = hbase + (size_t)__builtin_amdgcn_readfirstlane(e) * g.corr_hist_cap;
                }
                if (hslot == -1 || hslot == -3) help_watch(hslot, hv, (P.ns + 63) >> 6, lane);
                if (hslot >= 0 && !reuse) {  // the search shared with the helpers; the contributions read cset
                    help_search(P, hslot, (unsigned)it + 1u, Rf, tf, cset, lane);
                    reuse = true;
                }
#ifdef PCORE_GICP_PROFILE
                gp_acc[8] += reuse ? 1ull : 0ull;
#endif
                double acc[gicpm::kTerms];
#pragma unroll
                for (int v = 0; v < gicpm::kTerms; v++) acc[v] = 0.0;
                // rounds in pairs: both rounds' correspondences first (one pass over the key quads serves both:
                // scan_quads2), then their contributions in point order -- the sums are those of round-by-round
                // linearisation, bit for bit
                for (int i0 = 0; i0 < P.ns; i0 += 128) {
                    const int ia = i0 + lane, ib = ia + 64;
                    const bool two = i0 + 64 < P.ns;  // uniform
                    GPROF_T(t_s0);
                    int ja = -1, jb = -1;
                    if (reuse) {
                        if (ia < P.ns) ja = cset[ia];
                        if (two && ib < P.ns) jb = cset[ib];
                    } else {
                        const float4 sa = ia < P.ns ? P.src[ia] : make_float4(0.0f, 0.0f, 0.0f, 0.0f);
                        const float4 sb = two && ib < P.ns ? P.src[ib] : make_float4(0.0f, 0.0f, 0.0f, 0.0f);
                        float qa[3], qb[3];
                        gicpm::query_f(Rf, tf, sa.x, sa.y, sa.z, qa);
                        gicpm::query_f(Rf, tf, sb.x, sb.y, sb.z, qb);
                        if (GRID && P.use_grid) {  // segments above kGridNNMin (the grid is read here, not per pose)
                            const LabelGrid Gs = g.grids[P.seg];
                            float best;
                            if (ia < P.ns) grid_nn(Gs, g.cell_start, g.grid_pts, P.tgt, P.nt, qa[0], qa[1], qa[2], best, ja);
                            if (two && ib < P.ns)
                                grid_nn(Gs, g.cell_start, g.grid_pts, P.tgt, P.nt, qb[0], qb[1], qb[2], best, jb);
                        } else if (two && PCORE_GICP_PAIR_SCAN) {
                            scan_quads2(P.tquads, P.nt, qa[0], qa[1], qa[2], qb[0], qb[1], qb[2], ja, jb);
                        } else if (two) {  // A/B: the pair's queries scanned one after the other
                            float best = INFINITY;
                            scan_quads(P.tquads, P.nt, qa[0], qa[1], qa[2], best, ja);
                            best = INFINITY;
                            scan_quads(P.tquads, P.nt, qb[0], qb[1], qb[2], best, jb);
                        } else {
                            float best = INFINITY;
                            scan_quads(P.tquads, P.nt, qa[0], qa[1], qa[2], best, ja);
                        }
                        if (ia < P.ns) cset[ia] = ja;
                        if (two && ib < P.ns) cset[ib] = jb;
                    }
                    GPROF_TD(t_s1, ja + jb);
                    GPROF_ADD(0, t_s0, t_s1);
                    linearize_round<false>(x, Rf, tf, P.src, P.scov, P.tgt, P.tcov, P.ns, ia, P.use_grid, G, g,
                                           P.tquads, P.nt, ia < P.ns ? ja : -1, nullptr, P.mah, r0, acc, false GPROF_ARG);
                    if (two)
                        linearize_round<false>(x, Rf, tf, P.src, P.scov, P.tgt, P.tcov, P.ns, ib, P.use_grid, G, g,
                                               P.tquads, P.nt, ib < P.ns ? jb : -1, nullptr, P.mah, r0, acc,
                                               false GPROF_ARG);
                }
                GPROF_T(t_b);
                const double* sys = wave_tree_sums(acc, sRed, lane);
                GPROF_TD(t_c, sys[0]);
                bool inert;
                const int st = lm_iteration(sys, x, lambda, P.src, cset, P.mah, P.tgt, P.ns, lane, r0, (const lds_cvd*)sSe3,
                                            g.rot_eps, g.trans_eps, inert GPROF_ARG);
                GPROF_TD(t_d, st);
                GPROF_ADD(2, t_b, t_c);
                GPROF_ADD(3, t_c, t_d);
                if (st != gicpm::kLmAccepted) break;
                if (g.cycle_window > 0 && iters < g.max_iter) {
                    exit_slot = cyc.step(x, iters, g.max_iter, g.cycle_window, inert, lane);
                    if (exit_slot >= 0) {
                        iters_run = iters;
                        iters = g.max_iter;
                        break;
                    }
                }
            }
        }
        if (exit_slot >= 0) cyc.member(exit_slot, x);
#ifdef PCORE_GICP_PROFILE
        gp_acc[9] += iters_run ? iters_run : iters;
        if (P.ns < PCORE_GICP_PROF_MIN_NS)
            for (int k_ = 0; k_ < kGprof; k_++) gp_acc[k_] = gp_snap[k_];
#endif
        if (lane == 0) {
            write_pose(g, P.gp, x, iters);
            count_iterations(g, iters, iters_run ? iters_run : iters, iters_run != 0);
            if (kGicpHelpBoard && NW == 1 && !GRID) {
                const HelpRef h = help_ref();
                if (h.ctl) {
                    if (hslot >= 0 || hslot == -3) hb_store(hb_claim(h) + blockIdx.x, kHelpClosed);
                    hb_add(h.ctl + 1, 1u);  // poses finished (the helpers leave at num_poses)
                }
            }
        }
#ifdef PCORE_GICP_TIMELINE
        if (lane == 0 && P.gp < kTlPoses) {
            g_tl_pose[2 * P.gp] = tl_p0;
            g_tl_pose[2 * P.gp + 1] = __builtin_amdgcn_s_memrealtime();
            g_tl_run[P.gp] = iters_run ? iters_run : iters;
        }
#endif
    }
    if constexpr (kGicpHelpBoard && NW == 1 && !GRID)
        if (help_ref().ctl) help_loop(g, num_poses, lane);
    GPROF_FLUSH;
#ifdef PCORE_GICP_TIMELINE
    if (lane == 0) {
        const unsigned int w = atomicAdd(&g_tl_nwaves, 1u);
        if (w < (unsigned)kTlWaves) {
            g_tl_wave[2 * w] = tl_w0;
            g_tl_wave[2 * w + 1] = __builtin_amdgcn_s_memrealtime();
        }
    }
#endif
}


// Small batches (C1: 128 poses fill 128 of 1024 SIMDs) with large target segments: WPP waves per pose.
// All waves search the correspondences of the iteration's source points (round r -> wave r % WPP), the
// indices go to LDS, and wave 0 then adds the contributions and runs the LM iteration exactly as gicp_kernel
// does -- point i on lane i % 64, in point order -- so the refined poses are bit-identical; only the
// nearest-target searches, the expensive part against a whole-scene target, run in parallel.
template <int WPP>
__global__ void __launch_bounds__(64 * WPP) gicp_wide_kernel(GicpArgs g, int num_poses) {
    extern __shared__ __attribute__((aligned(16))) int32_t jbuf[];  // src_cap correspondences
    __shared__ double sRed[gicpm::kTerms];
    __shared__ double2 sM0[3][kLdsPts];
    __shared__ Pt3 sS0[kLdsPts];
    __shared__ float4 sT0[kLdsPts];
    __shared__ double sX[12];
    __shared__ int sPose, sFlag;
    __shared__ double sSe3[4 * gicpm::kSe3Terms];
    __shared__ unsigned sCyc[kCycleRingWords];  // wave 0's cycle exit ring
    const int tid = threadIdx.x, wave = __builtin_amdgcn_readfirstlane(tid >> 6), lane = tid & 63;
    const Round0 r0{sM0, sS0, sT0};  // wave 0's
    if (tid < 4 * gicpm::kSe3Terms) sSe3[tid] = gicpm::kSe3Coef[tid];
    GPROF_DECL;  // wave 0's phases: [0] the searches of all waves (to the barrier), [1] contributions, [2] tree, [3] LM
    for (;;) {
        __syncthreads();
        if (tid == 0) {
            const int q = atomicAdd(g.work_counter, 1);
            sPose = (g.pose_order && q < num_poses) ? g.pose_order[q] : q;
        }
        __syncthreads();
        const int pose = __builtin_amdgcn_readfirstlane(sPose);
        if (pose >= num_poses) break;
        coop_pose<true, WPP>(g, gicp_pose(g, pose), wave, lane, jbuf, sRed, r0, (const lds_cvd*)sSe3, sCyc, sX,
                             &sFlag GPROF_ARG);
    }
    if (wave == 0) GPROF_FLUSH;
}

constexpr int kGicpWideWpp = 8;
constexpr size_t kGicpWideMaxLds = 96 * 1024;  // correspondence buffer: src_cap <= 24576

#ifdef PCORE_GICP_PROFILE
extern "C" int pcore_debug_gicp_profile(unsigned long long* out, int reset) {
    hipError_t e = hipMemcpyFromSymbol(out, HIP_SYMBOL(g_gicp_prof), sizeof(unsigned long long) * kGprof);
    if (e == hipSuccess && reset) {
        const unsigned long long z[kGprof] = {};
        e = hipMemcpyToSymbol(HIP_SYMBOL(g_gicp_prof), z, sizeof(z));
    }
    return e == hipSuccess ? 0 : 1;
}
#endif

// Test hook of the kernels' damped solve (gicpm::lm_solve_schur): one wave per 28-term system.
__global__ void __launch_bounds__(64) lm_solve_test_kernel(const double* sys, const double* lambda, double* out, int n) {
    const int i = blockIdx.x;
    if (i >= n) return;
    double d[6];
    gicpm::lm_solve_schur(sys + (size_t)gicpm::kTerms * i, lambda[i], d);
    if (threadIdx.x == 0)
        for (int a = 0; a < 6; a++) out[(size_t)6 * i + a] = d[a];
}

hipError_t launch_lm_solve_test(const double* sys, const double* lambda, double* out, int n, hipStream_t s) {
    if (n <= 0) return hipSuccess;
    hipLaunchKernelGGL(lm_solve_test_kernel, dim3(n), dim3(64), 0, s, sys, lambda, out, n);
    return hipGetLastError();
}

// predicted cost of one GICP iteration of a pose: source points x targets of its segment (the scan); the poses at
// or above g.heavy_cost are counted into *g.heavy_count (the cost order puts them first: gicp_kernel's heavy poses)
__global__ void gicp_cost_key_kernel(GicpArgs g, int n, uint32_t* keys, int32_t* idx) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    int seg = g.whole_seg;
    if (g.pose_label) {
        const int pl = g.pose_label[g.pose_base + i];
        seg = (pl >= 0 && pl < g.num_segs) ? pl : -1;
    }
    const unsigned long long nt = seg >= 0 ? (unsigned long long)(g.seg_hi[seg] - g.seg_lo[seg]) : 0ull;
    const unsigned long long c = (unsigned long long)max(g.src_count[i], 0) * nt;
    keys[i] = (uint32_t)min(c >> 4, 0xffffffffull);
    idx[i] = i;
    if (g.heavy_count && g.heavy_cost > 0 && c >= (unsigned long long)g.heavy_cost) atomicAdd(g.heavy_count, 1);
}

size_t gicp_order_temp_bytes(int n) {
    size_t bytes = 0;
    (void)hipcub::DeviceRadixSort::SortPairsDescending(nullptr, bytes, (const uint32_t*)nullptr, (uint32_t*)nullptr,
                                                       (const int32_t*)nullptr, (int32_t*)nullptr, n);
    return bytes;
}

hipError_t launch_gicp_order(const GicpArgs& g, int n, uint32_t* keys_in, uint32_t* keys_out, int32_t* idx_in,
                             int32_t* order_out, void* temp, size_t temp_bytes, hipStream_t s) {
    if (n <= 0) return hipSuccess;
    hipLaunchKernelGGL(gicp_cost_key_kernel, dim3((n + 255) / 256), dim3(256), 0, s, g, n, keys_in, idx_in);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
    return hipcub::DeviceRadixSort::SortPairsDescending(temp, temp_bytes, keys_in, keys_out, idx_in, order_out, n, 0,
                                                        32, s);
}

#ifndef PCORE_GICP_WG_WAVES
#define PCORE_GICP_WG_WAVES 1  // 4: the heavy poses by 4-wave workgroups -- measured, no faster
#endif
constexpr int kGicpWgWaves = PCORE_GICP_WG_WAVES;  // gicp_kernel's waves per workgroup (the heavy poses' team)

hipError_t gicp_occupancy_per_cu(int* per_cu) {
    *per_cu = 0;
    int other = 0;
    hipError_t e = hipOccupancyMaxActiveBlocksPerMultiprocessor(per_cu, gicp_kernel<true, kGicpWgWaves>,
                                                                64 * kGicpWgWaves, 0);
    if (e == hipSuccess)
        e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&other, gicp_kernel<false, kGicpWgWaves>, 64 * kGicpWgWaves, 0);
    if (e == hipSuccess) *per_cu = std::min(*per_cu, other);
    return e;
}

hipError_t launch_gicp(const GicpArgs& g, int num_poses, const DeviceInfo& d, hipStream_t s, bool grid) {
    if (num_poses <= 0) return hipSuccess;
    const int resident_wgs = std::max(1, d.gicp_resident_wgs), num_cus = std::max(1, d.num_cus);
    // the one-wave queue's and the heavy queue's counters (heavy_count was set by the cost-key kernel)
    hipError_t e = hipMemsetAsync(g.work_counter, 0, 2 * sizeof(int32_t), s);
    if (e != hipSuccess) return e;
    // a batch too small to give every SIMD a pose: spread each pose's searches over kGicpWideWpp waves
    const size_t wide_lds = (size_t)g.src_cap * sizeof(int32_t);
    bool wide = num_poses <= num_cus * 2 && wide_lds <= kGicpWideMaxLds;
    if (const char* e = getenv("PCORE_GICP_KERNEL")) {  // tests pin either kernel (same results)
        if (e[0] == 'n') wide = false;
        else if (e[0] == 'w' && wide_lds <= kGicpWideMaxLds) wide = true;
    }
    GicpArgs ga = g;
    if (ga.cov_fold && (wide || kGicpWgWaves != 1)) {  // only the one-wave gicp_kernel has the covariance prologue
        e = launch_covariances_cloud(g.src, g.src_count, g.src_cap, num_poses, g.cov_fx, g.cov_fy, g.cov_cx, g.cov_cy,
                                     g.cov_stride, ga.cov_fold, s);
        if (e != hipSuccess) return e;
        ga.cov_fold = nullptr;
    }
    if (wide) {
        const int wgs = std::min(num_poses, num_cus * 2);
        hipLaunchKernelGGL(gicp_wide_kernel<kGicpWideWpp>, dim3(wgs), dim3(64 * kGicpWideWpp), wide_lds, s, ga,
                           num_poses);
        return hipGetLastError();
    }
    const dim3 wgs(std::min(resident_wgs, (num_poses + kGicpWgWaves - 1) / kGicpWgWaves)), block(64 * kGicpWgWaves);
    if (!kGicpHelpBoard || kGicpWgWaves != 1 || grid) ga.help_ctl = nullptr;  // the one-wave grid-free instance only
    if (ga.help_ctl && (e = hipMemsetAsync(ga.help_ctl, 0, help_ctl_words(ga.help_slots) * sizeof(unsigned), s)) != hipSuccess)
        return e;
    if (grid)
        hipLaunchKernelGGL((gicp_kernel<true, kGicpWgWaves>), wgs, block, 0, s, ga, num_poses);
    else
        hipLaunchKernelGGL((gicp_kernel<false, kGicpWgWaves>), wgs, block, 0, s, ga, num_poses);
    return hipGetLastError();
}

}  // namespace pcore
