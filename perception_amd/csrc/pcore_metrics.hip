// pcore_metrics.hip -- ADD / ADD-S pose distances on gfx950.
//
// The YCB harness scores every detected pose against ground truth with
//   ADD   = mean_i |T_gt p_i - T_est p_i|                 (fat_pose_image.py:2116-2121, pose_error.py:72-86)
//   ADD-S = mean_i min_j |T_gt p_i - T_est p_j|           (fat_pose_image.py:2123-2136, pose_error.py:89-108)
// over the model's points (tens of thousands for a YCB textured.ply), which is O(n^2) per pose for
// ADD-S -- sklearn's pairwise_distances_argmin_min on the CPU in the reference.
//
//   pose_dist_kernel      grid (ceil(n/256), pairs): one thread per ground-truth point.  The estimated
//                         cloud is transformed tile by tile into LDS (SoA doubles) and scanned with a
//                         running f64 minimum of the squared distance; per-block partial sums of the two
//                         distances in a fixed LDS tree.
//   pose_dist_finalize    one thread per pair: partials summed in block order, divided by n.
// Arithmetic is f64 throughout (the reference works in float64 on float32 model points).
#include "pcore_internal.h"

namespace pcore {

namespace {

constexpr int kMThreads = 256;
constexpr int kMTile = 1024;  // estimated points per LDS tile (24 KiB of doubles)

__device__ __forceinline__ void xform(const double* T, double px, double py, double pz, double& x, double& y,
                                      double& z) {
    x = T[0] * px + T[1] * py + T[2] * pz + T[3];
    y = T[4] * px + T[5] * py + T[6] * pz + T[7];
    z = T[8] * px + T[9] * py + T[10] * pz + T[11];
}

}  // namespace

__global__ void __launch_bounds__(kMThreads) pose_dist_kernel(const float* pts, int n, const double* T_gt,
                                                              const double* T_est, int want_adds, double* part) {
    __shared__ double sx[kMTile], sy[kMTile], sz[kMTile];
    __shared__ double red[2][kMThreads];
    const int m = blockIdx.y;
    const double* G = T_gt + (size_t)16 * m;
    const double* E = T_est + (size_t)16 * m;
    const int i = blockIdx.x * kMThreads + threadIdx.x;
    const bool act = i < n;
    double ax = 0.0, ay = 0.0, az = 0.0, add = 0.0, adds = 0.0;
    if (act) {
        const double px = pts[3 * i], py = pts[3 * i + 1], pz = pts[3 * i + 2];
        double bx, by, bz;
        xform(G, px, py, pz, ax, ay, az);
        xform(E, px, py, pz, bx, by, bz);
        const double dx = ax - bx, dy = ay - by, dz = az - bz;
        add = sqrt(dx * dx + dy * dy + dz * dz);
    }
    if (want_adds) {
        double best = INFINITY;
        for (int t0 = 0; t0 < n; t0 += kMTile) {
            const int tn = min(kMTile, n - t0);
            __syncthreads();
            for (int o = threadIdx.x; o < tn; o += kMThreads) {
                const int q = t0 + o;
                xform(E, (double)pts[3 * q], (double)pts[3 * q + 1], (double)pts[3 * q + 2], sx[o], sy[o], sz[o]);
            }
            __syncthreads();
#pragma unroll 4
            for (int o = 0; o < tn; o++) {
                const double dx = ax - sx[o], dy = ay - sy[o], dz = az - sz[o];
                const double d = __builtin_fma(dz, dz, __builtin_fma(dy, dy, dx * dx));
                best = fmin(best, d);
            }
        }
        if (act) adds = sqrt(best);
    }
    red[0][threadIdx.x] = add;
    red[1][threadIdx.x] = adds;
    __syncthreads();
    for (int s = kMThreads / 2; s > 0; s >>= 1) {
        if ((int)threadIdx.x < s) {
            red[0][threadIdx.x] += red[0][threadIdx.x + s];
            red[1][threadIdx.x] += red[1][threadIdx.x + s];
        }
        __syncthreads();
    }
    if (threadIdx.x == 0) {
        double* p = part + 2 * ((size_t)m * gridDim.x + blockIdx.x);
        p[0] = red[0][0];
        p[1] = red[1][0];
    }
}

__global__ void pose_dist_finalize(const double* part, int nblk, int n, int pairs, double* out_add, double* out_adds) {
    const int m = blockIdx.x * blockDim.x + threadIdx.x;
    if (m >= pairs) return;
    double s0 = 0.0, s1 = 0.0;
    for (int b = 0; b < nblk; b++) {
        s0 += part[2 * ((size_t)m * nblk + b)];
        s1 += part[2 * ((size_t)m * nblk + b) + 1];
    }
    if (out_add) out_add[m] = s0 / (double)n;
    if (out_adds) out_adds[m] = s1 / (double)n;
}

int pose_dist_blocks(int n) { return (n + kMThreads - 1) / kMThreads; }

hipError_t launch_pose_distances(const float* pts, int n, const double* T_gt, const double* T_est, int pairs,
                                 double* part, double* out_add, double* out_adds, hipStream_t s) {
    if (pairs <= 0 || n <= 0) return hipSuccess;
    const int nblk = pose_dist_blocks(n);
    hipLaunchKernelGGL(pose_dist_kernel, dim3(nblk, pairs), dim3(kMThreads), 0, s, pts, n, T_gt, T_est,
                       out_adds ? 1 : 0, part);
    hipLaunchKernelGGL(pose_dist_finalize, dim3((pairs + 63) / 64), dim3(64), 0, s, part, nblk, n, pairs, out_add,
                       out_adds);
    return hipGetLastError();
}

}  // namespace pcore
