// pcore_states.hip -- the per-state host work of the greedy search moved next to the GPU search
// (the callers of render_cuda_multi_unified on the pose path):
//
//   state_pose_kernel    GetStateImagesUnifiedGPU's pose building (search_env.cpp:1535-1576): for every state
//                        (x y z qx qy qz qw), inv(cam_z_front) * (ContPose::GetTransform * preprocess[model]), then
//                        mat4x4::init_from_eigen(., 100) (model.h:89-107) -- one thread per state, double.
//   count_within_kernel  IsValidPose's neighbour count (search_env.cpp:359-396): points of the query's label
//                        segment strictly within the radius, PCL KdTreeFLANN radiusSearch semantics (float query
//                        and points, squared radius as float, ((0 + dx^2) + dy^2) + dz^2 < r^2).
//
// Both evaluate the host restatements' exact IEEE operations in their order (perception_amd/model.py
// quat_xyzw_to_matrix_batch, pose_matrix_batch, chain_matmul_batch, init_from_eigen_batch; recognizer.py
// radius_counts), built with -ffp-contract=off, so the results are bit-identical to the host's
// (tests/test_gpu_states.py).
#include "pcore_internal.h"

#pragma clang fp contract(off)

namespace pcore {

namespace {

struct StatePoseArgs {
    const double* states;     // n x 7
    const int32_t* model;     // n
    const double* preprocess; // num_models x 16, row-major
    double cam[16];           // inv(cam_z_front), row-major
    int32_t num_models;
    int32_t n;
    float* out;               // n x 16
};

// (((x0 y0 + x1 y1) + x2 y2) + x3 y3): one entry of a 4x4 product, model.py chain_matmul_batch
__device__ __forceinline__ double dot4(double a0, double a1, double a2, double a3, double b0, double b1, double b2,
                                       double b3) {
    return ((a0 * b0 + a1 * b1) + a2 * b2) + a3 * b3;
}

__global__ void __launch_bounds__(256) state_pose_kernel(StatePoseArgs a) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= a.n) return;
    const double* s = a.states + (size_t)7 * i;
    // quat_xyzw_to_matrix: normalised quaternion -> rotation (Eigen::Quaterniond::toRotationMatrix)
    double x = s[3], y = s[4], z = s[5], w = s[6];
    // Eigen's squaredNorm of the 4 coefficients (x, y, z, w) in 2-wide SSE2 packets: (x^2 + z^2) + (y^2 + w^2)
    const double nrm = sqrt((x * x + z * z) + (y * y + w * w));
    x = x / nrm;
    y = y / nrm;
    z = z / nrm;
    w = w / nrm;
    double T[4][4];
    T[0][0] = 1.0 - 2.0 * (y * y + z * z);
    T[0][1] = 2.0 * (x * y - z * w);
    T[0][2] = 2.0 * (x * z + y * w);
    T[1][0] = 2.0 * (x * y + z * w);
    T[1][1] = 1.0 - 2.0 * (x * x + z * z);
    T[1][2] = 2.0 * (y * z - x * w);
    T[2][0] = 2.0 * (x * z - y * w);
    T[2][1] = 2.0 * (y * z + x * w);
    T[2][2] = 1.0 - 2.0 * (x * x + y * y);
    T[0][3] = s[0];
    T[1][3] = s[1];
    T[2][3] = s[2];
    T[3][0] = 0.0;
    T[3][1] = 0.0;
    T[3][2] = 0.0;
    T[3][3] = 1.0;
    int m = a.model[i];
    m = m < 0 ? 0 : (m >= a.num_models ? a.num_models - 1 : m);  // the caller checks the ids
    const double* B = a.preprocess + (size_t)16 * m;
    // search_env.cpp:1567-1571: transform = T * preprocess first, then pose_in_cam = cam_matrix * transform
    double M1[4][4];
#pragma unroll
    for (int r = 0; r < 4; r++)
#pragma unroll
        for (int c = 0; c < 4; c++)
            M1[r][c] = dot4(T[r][0], T[r][1], T[r][2], T[r][3], B[c], B[4 + c], B[8 + c], B[12 + c]);
    float* o = a.out + (size_t)16 * i;
#pragma unroll
    for (int r = 0; r < 4; r++)
#pragma unroll
        for (int c = 0; c < 4; c++) {
            const double v = dot4(a.cam[4 * r], a.cam[4 * r + 1], a.cam[4 * r + 2], a.cam[4 * r + 3], M1[0][c],
                                  M1[1][c], M1[2][c], M1[3][c]);
            o[4 * r + c] = r < 3 ? (float)(v * 100.0) : (float)v;
        }
}

// one thread per query, the segment's points in order
__global__ void __launch_bounds__(256) count_within_kernel(const float* q, const int32_t* labels, const float* r2,
                                                           int n, const float4* pts, const int32_t* seg_lo,
                                                           const int32_t* seg_hi, int num_segs, int32_t* out) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const int l = labels[i];
    int cnt = 0;
    if (l >= 0 && l < num_segs) {
        const float qx = q[3 * (size_t)i], qy = q[3 * (size_t)i + 1], qz = q[3 * (size_t)i + 2], rr = r2[i];
        const int lo = seg_lo[l], hi = seg_hi[l];
        for (int j = lo; j < hi; j++) {
            const float4 p = pts[j];
            const float dx = qx - p.x, dy = qy - p.y, dz = qz - p.z;
            float d = dx * dx;
            d = d + dy * dy;
            d = d + dz * dz;
            cnt += d < rr ? 1 : 0;
        }
    }
    out[i] = cnt;
}

}  // namespace

hipError_t launch_state_poses(const double* states, const int32_t* model, const double* preprocess,
                              const double cam[16], int num_models, int n, float* out, hipStream_t s) {
    if (n <= 0) return hipSuccess;
    StatePoseArgs a{};
    a.states = states;
    a.model = model;
    a.preprocess = preprocess;
    for (int k = 0; k < 16; k++) a.cam[k] = cam[k];
    a.num_models = num_models;
    a.n = n;
    a.out = out;
    hipLaunchKernelGGL(state_pose_kernel, dim3((n + 255) / 256), dim3(256), 0, s, a);
    return hipGetLastError();
}

hipError_t launch_count_within(const float* q, const int32_t* labels, const float* r2, int n, const float4* pts,
                               const int32_t* seg_lo, const int32_t* seg_hi, int num_segs, int32_t* out,
                               hipStream_t s) {
    if (n <= 0) return hipSuccess;
    hipLaunchKernelGGL(count_within_kernel, dim3((n + 255) / 256), dim3(256), 0, s, q, labels, r2, n, pts, seg_lo,
                       seg_hi, num_segs, out);
    return hipGetLastError();
}

}  // namespace pcore
