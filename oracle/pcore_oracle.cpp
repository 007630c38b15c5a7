// pcore_oracle.cpp -- CPU restatement of the reference hot path.  TEST INFRASTRUCTURE ONLY.
// See pcore_oracle.h for the parity status ("parity unpinned" vs the reference binary).
// Build: oracle/Makefile (g++ -O2 -ffp-contract=off -fno-fast-math -fopenmp).
#include "pcore_oracle.h"

// The colour spec (deterministic sin / cos / atan2 / exp, CIEDE2000 term order) is shared with the GPU
// build: it defines the arithmetic, like the GICP spec; tests/test_colour_spec.py pins it against numpy.
#include "../perception_amd/csrc/pcore_colour.h"
#include "../perception_amd/csrc/pcore_gicp_math.h"

#include <climits>
#include <cfloat>
#include <cmath>
#include <cstring>
#include <vector>
#include <omp.h>



namespace {

// NVIDIA cvt.rzi.s32.f32 (what `int32_t(float)` compiles to in image_renderer.cuh:129):
// truncate toward zero, NaN -> 0, saturate.
inline int32_t cvt_i32_gpu(float f) {
    if (!(f == f)) return 0;
    if (f >= 2147483648.0f) return INT_MAX;
    if (f <= -2147483648.0f) return INT_MIN;
    return (int32_t)f;
}
// NVIDIA cvt.rzi.u64.f32 (`size_t(bboxmin+0.5f)`, image_renderer.cuh:110-111): NaN/neg -> 0, saturate.
inline uint64_t cvt_u64_gpu(float f) {
    if (!(f == f) || f <= 0.0f) return 0;
    if (f >= 18446744073709551616.0f) return UINT64_MAX;
    return (uint64_t)f;
}
// x86 cvttss2si (host `(int) float` in search_env.cpp:2022-2048): NaN / out of range -> INT_MIN.
inline int32_t cvt_i32_x86(float f) {
    if (!(f == f) || f >= 2147483648.0f || f < -2147483648.0f) return INT_MIN;
    return (int32_t)f;
}
// CUDA int abs() on a wrapped int32 difference (image_renderer.cuh:163-165).
inline int32_t iabs_wrap(int32_t a, int32_t b) {
    int32_t d = (int32_t)((uint32_t)a - (uint32_t)b);
    return d < 0 ? (int32_t)(0u - (uint32_t)d) : d;
}

struct F3 { float x, y, z; };

// image_renderer.cuh:14-18
inline float std_max(float a, float b) { return (a > b) ? a : b; }
inline float std_min(float a, float b) { return (a < b) ? a : b; }

// image_renderer.cuh:20-27 mat_mul_v: ((a0*x + a1*y) + a2*z) + a3
inline F3 mat_mul_v(const float* m, const F3& v) {
    F3 r;
    r.x = m[0] * v.x + m[1] * v.y + m[2] * v.z + m[3];
    r.y = m[4] * v.x + m[5] * v.y + m[6] * v.z + m[7];
    r.z = m[8] * v.x + m[9] * v.y + m[10] * v.z + m[11];
    return r;
}

// image_renderer.cuh:39-42
inline float signed_area(const float* A, const float* B, const float* C) {
    return 0.5f * ((C[0] - A[0]) * (B[1] - A[1]) - (B[0] - A[0]) * (C[1] - A[1]));
}

// image_renderer.cuh:44-57
inline F3 barycentric(const float* A, const float* B, const float* C, const uint64_t* P) {
    float fP[2] = {(float)P[0], (float)P[1]};
    float base_inv = 1.0f / signed_area(A, B, C);
    float beta = signed_area(A, fP, C) * base_inv;
    float gamma = signed_area(A, B, fP) * base_inv;
    return {1.0f - beta - gamma, beta, gamma};
}

// image_renderer.cuh:59-210, executed for one triangle of one pose, serially.
void rasterize_with_source(const F3 tri[3], F3 last_row, int32_t* depth, int width, int height,
                           const int32_t* src_depth, const uint8_t* src_mask, bool use_seg,
                           int32_t pose_label, float occlusion_threshold, int32_t* dmin = nullptr,
                           int32_t* tri_id = nullptr, int32_t t = 0) {
    const float W = (float)width, H = (float)height;
    float pts2[3][2];
    const float lr[3] = {last_row.x, last_row.y, last_row.z};
    for (int i = 0; i < 3; i++) {
        pts2[i][0] = tri[i].x / lr[i] * W / 2.0f + W / 2.0f;
        pts2[i][1] = tri[i].y / lr[i] * H / 2.0f + H / 2.0f;
    }
    float bboxmin[2] = {FLT_MAX, FLT_MAX};
    float bboxmax[2] = {-FLT_MAX, -FLT_MAX};
    const float clamp_max[2] = {(float)(width - 1), (float)(height - 1)};
    const float clamp_min[2] = {0.0f, 0.0f};
    for (int i = 0; i < 3; i++)
        for (int j = 0; j < 2; j++) {
            bboxmin[j] = std_max(clamp_min[j], std_min(bboxmin[j], pts2[i][j]));
            bboxmax[j] = std_min(clamp_max[j], std_max(bboxmax[j], pts2[i][j]));
        }
    uint64_t P[2];
    for (P[1] = cvt_u64_gpu(bboxmin[1] + 0.5f); (float)P[1] <= bboxmax[1]; P[1] += 1) {
        for (P[0] = cvt_u64_gpu(bboxmin[0] + 0.5f); (float)P[0] <= bboxmax[0]; P[0] += 1) {
            F3 bc = barycentric(pts2[0], pts2[1], pts2[2], P);
            if (bc.x < -0.0f || bc.y < -0.0f || bc.z < -0.0f || bc.x > 1.0f || bc.y > 1.0f || bc.z > 1.0f)
                continue;
            F3 boz = {bc.x / last_row.x, bc.y / last_row.y, bc.z / last_row.z};
            float frag_depth = (bc.x + bc.y + bc.z) / (boz.x + boz.y + boz.z);
            const size_t x = (size_t)P[0];
            const size_t y = (size_t)height - 1 - (size_t)P[1];
            const size_t idx = x + y * (size_t)width;
            const int32_t curr = cvt_i32_gpu(frag_depth + 0.5f);
            // colour of the pixel: the first triangle (serial order) reaching the minimum fragment depth
            if (dmin != nullptr && curr < dmin[idx]) {
                dmin[idx] = curr;
                tri_id[idx] = t;
            }
            // z-test (image_renderer.cuh:146-159), serial order
            if (curr < depth[idx]) depth[idx] = curr;
            const int32_t nd = depth[idx];
            const int32_t src = src_depth[idx];
            const int lab = use_seg ? (int)src_mask[idx] : 0;
            // source occlusion black-out (image_renderer.cuh:160-196)
            if ((!use_seg && (float)iabs_wrap(nd, src) > occlusion_threshold) ||
                (use_seg && pose_label != lab - 1 && (float)iabs_wrap(nd, src) > 0.5f)) {
                if (nd > src && src > 0) depth[idx] = INT_MAX;
            }
        }
    }
}

void render_one_pose(const float* tris, int lo, int hi, const float* pose, int width, int height,
                     const float* proj, const int32_t* src_depth, const uint8_t* src_mask, bool use_seg,
                     int32_t pose_label, float occlusion_threshold, int32_t* depth, int32_t* dmin = nullptr,
                     int32_t* tri_id = nullptr) {
    const size_t npx = (size_t)width * height;
    for (size_t i = 0; i < npx; i++) depth[i] = INT_MAX;
    if (dmin != nullptr)
        for (size_t i = 0; i < npx; i++) {
            dmin[i] = INT_MAX;
            tri_id[i] = -1;
        }
    for (int t = lo; t < hi; t++) {
        const float* tp = tris + (size_t)9 * t;
        F3 v[3] = {{tp[0], tp[1], tp[2]}, {tp[3], tp[4], tp[5]}, {tp[6], tp[7], tp[8]}};
        // image_renderer.cuh:296-305: model transform, keep camera z, projection transform
        F3 local[3], projd[3];
        for (int k = 0; k < 3; k++) local[k] = mat_mul_v(pose, v[k]);
        F3 last_row = {local[0].z, local[1].z, local[2].z};
        for (int k = 0; k < 3; k++) projd[k] = mat_mul_v(proj, local[k]);
        rasterize_with_source(projd, last_row, depth, width, height, src_depth, src_mask, use_seg, pose_label,
                              occlusion_threshold, dmin, tri_id, t);
    }
    // max2zero (image_renderer.cuh:324-333, 465-466)
    for (size_t i = 0; i < npx; i++)
        if (depth[i] == INT_MAX) depth[i] = 0;
}

void model_ranges(const int32_t* tris_model_count, int num_models, std::vector<int>& lo, std::vector<int>& hi) {
    lo.assign(num_models, 0);
    hi.assign(num_models, 0);
    int acc = 0;
    for (int m = 0; m < num_models; m++) {  // exclusive / inclusive scans, image_renderer.cuh:371-380
        lo[m] = acc;
        acc += tris_model_count[m];
        hi[m] = acc;
    }
}

// compute_point_clouds.cuh:14-35 transform_point (camera_transform == NULL)
inline void transform_point(int x, int y, int32_t d, float cx, float cy, float fx, float fy, float df,
                            float& xp, float& yp, float& zp) {
    zp = (float)d / df;
    xp = ((float)x - cx) / fx * zp;
    yp = ((float)y - cy) / fy * zp;
}

inline float sqdist(const float* a, const float* b) {
    float dx = a[0] - b[0], dy = a[1] - b[1], dz = a[2] - b[2];
    return dx * dx + dy * dy + dz * dz;
}

void knn1_range(const float* q, const float* o_xyz, int lo, int hi, float& best_d2, int32_t& best_i) {
    best_d2 = INFINITY;
    best_i = -1;
    for (int o = lo; o < hi; o++) {
        float d = sqdist(q, o_xyz + (size_t)3 * o);
        if (d < best_d2) {  // strict: ties keep the lowest index
            best_d2 = d;
            best_i = o;
        }
    }
}

}  // namespace

extern "C" {

void orc_compute_proj(float fx, float fy, float cx, float cy, int width, int height, float near_plane,
                      float far_plane, float out[16]) {
    // renderer.cu:1386-1410 (K(0,1) = 0 for a pinhole camera)
    const float k01 = 0.0f;
    float a0 = 2 * fx / width;
    float a1 = -2 * k01 / width; a1 = -a1;
    float a2 = -2 * cx / width + 1; a2 = -a2;
    float b1 = 2 * fy / height; b1 = -b1;
    float b2 = 2 * cy / height - 1; b2 = -b2;
    float c2 = -(far_plane + near_plane) / (far_plane - near_plane); c2 = -c2;
    float c3 = -2 * far_plane * near_plane / (far_plane - near_plane);
    float d2 = -1; d2 = -d2;
    const float m[16] = {a0, a1, a2, 0, 0, b1, b2, 0, 0, 0, c2, c3, 0, 0, d2, 0};
    std::memcpy(out, m, sizeof(m));
}

void orc_render_depth(const float* tris, int num_tris, const int32_t* tris_model_count, int num_models,
                      const float* poses, const int32_t* pose_model, const int32_t* pose_label, int num_poses,
                      int width, int height, const float* proj, const int32_t* src_depth, const uint8_t* src_mask,
                      float occlusion_threshold, int32_t* out, int nthreads) {
    (void)num_tris;
    std::vector<int> lo, hi;
    model_ranges(tris_model_count, num_models, lo, hi);
    const bool use_seg = pose_label != nullptr;
    const size_t npx = (size_t)width * height;
    if (nthreads > 0) omp_set_num_threads(nthreads);
#pragma omp parallel for schedule(dynamic, 1)
    for (int n = 0; n < num_poses; n++) {
        const int m = pose_model[n];
        render_one_pose(tris, lo[m], hi[m], poses + (size_t)16 * n, width, height, proj, src_depth, src_mask,
                        use_seg, use_seg ? pose_label[n] : 0, occlusion_threshold, out + npx * n);
    }
}

int orc_depth_to_cloud(const int32_t* depth, int num_poses, int width, int height, int stride, float cx, float cy,
                       float fx, float fy, float depth_factor, const uint8_t* label_mask, const int32_t* pose_label,
                       float* out_xyz, int32_t* out_pose, int32_t* out_label, int cap) {
    int count = 0;
    const size_t npx = (size_t)width * height;
    for (int n = 0; n < num_poses; n++)
        for (int y = 0; y < height; y += stride)
            for (int x = 0; x < width; x += stride) {
                const size_t idx = npx * n + (size_t)x + (size_t)y * width;
                if (depth[idx] <= 0) continue;                              // depth_to_mask, :64
                if (label_mask != nullptr && label_mask[idx] <= 0) continue;  // :71-77, :125-128
                if (count < cap) {
                    float xp, yp, zp;
                    transform_point(x, y, depth[idx], cx, cy, fx, fy, depth_factor, xp, yp, zp);
                    out_xyz[3 * (size_t)count + 0] = xp;
                    out_xyz[3 * (size_t)count + 1] = yp;
                    out_xyz[3 * (size_t)count + 2] = zp;
                    if (out_pose) out_pose[count] = n;
                    if (out_label) {
                        if (label_mask != nullptr) out_label[count] = (int32_t)label_mask[idx] - 1;  // :172
                        else if (pose_label != nullptr) out_label[count] = pose_label[n];           // :177
                        else out_label[count] = 0;
                    }
                }
                count++;
            }
    return count;
}

// depth2cloud_global with camera_transform + observed_cloud_bounds (3-DoF; compute_point_clouds.cuh:14-35,
// 79-91, 125-157): keep a pixel when its world point (R p left to right, then + t, in float) is inside the
// bounds (x_max, x_min, y_max, y_min, z_max, z_min as floats); emit the CAMERA-frame point and its colour.
int orc_depth_to_cloud_bounded(const int32_t* depth, int width, int height, int stride, float cx, float cy, float fx,
                               float fy, float depth_factor, const float* cam_to_world, const double* bounds,
                               const uint8_t* rgb, float* out_xyz, uint8_t* out_rgb, int cap) {
    int count = 0;
    float b[6];
    for (int i = 0; i < 6; i++) b[i] = bounds ? (float)bounds[i] : 0.0f;
    for (int y = 0; y < height; y += stride)
        for (int x = 0; x < width; x += stride) {
            const size_t idx = (size_t)x + (size_t)y * width;
            if (depth[idx] <= 0) continue;
            float xp, yp, zp;
            transform_point(x, y, depth[idx], cx, cy, fx, fy, depth_factor, xp, yp, zp);
            if (cam_to_world != nullptr) {
                const float* m = cam_to_world;
                const float wx = (m[0] * xp + m[1] * yp + m[2] * zp) + m[3];
                const float wy = (m[4] * xp + m[5] * yp + m[6] * zp) + m[7];
                const float wz = (m[8] * xp + m[9] * yp + m[10] * zp) + m[11];
                if (wx > b[0] || wx < b[1]) continue;
                if (wy > b[2] || wy < b[3]) continue;
                if (wz > b[4] || wz < b[5]) continue;
            }
            if (count < cap) {
                out_xyz[3 * (size_t)count + 0] = xp;
                out_xyz[3 * (size_t)count + 1] = yp;
                out_xyz[3 * (size_t)count + 2] = zp;
                if (out_rgb != nullptr && rgb != nullptr)
                    for (int ch = 0; ch < 3; ch++) out_rgb[3 * (size_t)count + ch] = rgb[3 * idx + ch];
            }
            count++;
        }
    return count;
}

void orc_knn1(const float* r_xyz, const int32_t* r_label, int num_r, const float* o_xyz, int num_o,
              const int32_t* label_start, const int32_t* label_end, int num_labels, float* out_d2, int32_t* out_idx) {
#pragma omp parallel for schedule(static)
    for (int i = 0; i < num_r; i++) {
        int lo = 0, hi = num_o;
        if (label_start != nullptr) {
            const int L = r_label[i];
            if (L < 0 || L >= num_labels) { lo = 0; hi = 0; }
            else { lo = label_start[L]; hi = label_end[L]; }
        }
        knn1_range(r_xyz + (size_t)3 * i, o_xyz, lo, hi, out_d2[i], out_idx[i]);
    }
}

void orc_costs(int num_poses, int cost_type, int calc_obs, float sensor_resolution, const float* d2,
               const int32_t* idx, const int32_t* r_pose, int num_r, int num_o, const float* pose_obs_total,
               float* out_rc, float* out_oc, float* out_diff) {
    (void)cost_type;  // types 0 and 2 mark explained identically (compute_costs.cuh:241-270)
    const float r2 = sensor_resolution * sensor_resolution;  // renderer.cu:1877
    std::vector<float> num(num_poses, 0.0f), bad(num_poses, 0.0f);
    std::vector<uint8_t> explained((size_t)num_poses * (num_o > 0 ? num_o : 1), 0);
    for (int i = 0; i < num_r; i++) {  // compute_render_cost, compute_costs.cuh:161-273
        const int p = r_pose[i];
        num[p] += 1.0f;
        if (d2[i] > r2) bad[p] += 1.0f;
        else if (idx[i] >= 0) explained[(size_t)p * num_o + idx[i]] = 1;
    }
    for (int p = 0; p < num_poses; p++) {
        const float rendered_explained = num[p] - bad[p];           // :364-368
        float rc = (num[p] == 0) ? -1.0f : bad[p] / num[p];        // cost_percentage_functor
        rc = (rc == -1.0f) ? -1.0f : rc * 100.0f;                  // cost_multiplier_functor
        out_rc[p] = rc;
        if (calc_obs) {
            float expl = 0.0f;                                       // compute_observed_cost :274-290
            for (int o = 0; o < num_o; o++) expl += (float)explained[(size_t)p * num_o + o];
            out_diff[p] = rendered_explained - expl;                 // :407-411
            float oc = pose_obs_total[p] - expl;                     // :422-426
            oc = oc / pose_obs_total[p];                             // :435-439
            out_oc[p] = oc * 100.0f;                                 // :442-446
        } else {
            out_oc[p] = 0.0f;
            out_diff[p] = 0.0f;
        }
    }
}

void orc_select(int num_poses, const float* rc, const float* oc, const int32_t* pose_model, int num_models,
                int64_t index_base, int32_t* out_best_cost, int64_t* out_best_index) {
    for (int m = 0; m < num_models; m++) {
        out_best_cost[m] = INT_MAX;
        out_best_index[m] = -1;
    }
    for (int i = 0; i < num_poses; i++) {
        int32_t cost, target, source;
        if (cvt_i32_x86(rc[i]) < 0) {  // search_env.cpp:2022-2027
            cost = -1;
        } else {
            cost = cvt_i32_x86(rc[i] + oc[i]);  // :2035
        }
        target = cvt_i32_x86(rc[i]);  // :2043-2044
        source = cvt_i32_x86(oc[i]);
        if (cost == -1 || cost == -2) continue;  // :2554-2556
        const int m = pose_model[i];
        const int32_t diff = (int32_t)((uint32_t)target - (uint32_t)source);
        const int32_t adiff = diff < 0 ? (int32_t)(0u - (uint32_t)diff) : diff;
        if (cost < out_best_cost[m] && adiff < 30) {  // :2560-2566, strict '<' keeps the first index
            out_best_cost[m] = cost;
            out_best_index[m] = index_base + i;
        }
    }
}

void orc_evaluate(const float* tris, int num_tris, const int32_t* tris_model_count, int num_models,
                  const float* poses, const int32_t* pose_model, const int32_t* pose_label, int num_poses,
                  int width, int height, const float* proj, const int32_t* src_depth, const uint8_t* src_mask,
                  float occlusion_threshold, int stride, float cx, float cy, float fx, float fy, float depth_factor,
                  const float* o_xyz, int num_o, const int32_t* label_start, const int32_t* label_end,
                  int num_labels, const float* pose_obs_total, int cost_type, int calc_obs,
                  float sensor_resolution, float* out_rc, float* out_oc, float* out_diff, int nthreads) {
    (void)num_tris;
    std::vector<int> lo, hi;
    model_ranges(tris_model_count, num_models, lo, hi);
    const bool use_seg = pose_label != nullptr;
    const size_t npx = (size_t)width * height;
    const int ws = (width + stride - 1) / stride, hs = (height + stride - 1) / stride;
    if (nthreads > 0) omp_set_num_threads(nthreads);
#pragma omp parallel
    {
        std::vector<int32_t> depth(npx);
        std::vector<float> xyz((size_t)3 * ws * hs);
        std::vector<float> d2((size_t)ws * hs);
        std::vector<int32_t> nn((size_t)ws * hs), rpose((size_t)ws * hs, 0), rlab((size_t)ws * hs);
#pragma omp for schedule(dynamic, 1)
        for (int n = 0; n < num_poses; n++) {
            const int m = pose_model[n];
            const int32_t pl = use_seg ? pose_label[n] : 0;
            render_one_pose(tris, lo[m], hi[m], poses + (size_t)16 * n, width, height, proj, src_depth, src_mask,
                            use_seg, pl, occlusion_threshold, depth.data());
            const int nr = orc_depth_to_cloud(depth.data(), 1, width, height, stride, cx, cy, fx, fy, depth_factor,
                                              nullptr, nullptr, xyz.data(), nullptr, nullptr, ws * hs);
            for (int i = 0; i < nr; i++) {
                int l0 = 0, l1 = num_o;
                if (use_seg && label_start != nullptr) {
                    if (pl < 0 || pl >= num_labels) { l0 = 0; l1 = 0; }
                    else { l0 = label_start[pl]; l1 = label_end[pl]; }
                }
                knn1_range(xyz.data() + (size_t)3 * i, o_xyz, l0, l1, d2[i], nn[i]);
            }
            float rc, oc, df;
            const float tot = pose_obs_total ? pose_obs_total[n] : 0.0f;
            orc_costs(1, cost_type, calc_obs, sensor_resolution, d2.data(), nn.data(), rpose.data(), nr, num_o,
                      &tot, &rc, &oc, &df);
            out_rc[n] = rc;
            out_oc[n] = oc;
            out_diff[n] = df;
        }
    }
}

}  // extern "C"

// ==================================================================================================
// GICP (build-owned spec; see pcore_oracle.h and DESIGN.md "GICP spec")
// ==================================================================================================
namespace {

constexpr int kGicpThreads = 64;  // one GPU wave per pose: its reduction order is mirrored here
constexpr int kMaxK = 16;
constexpr double kPlaneScale = 1.0 - 1e-3;  // I - (1 - 1e-3) n n^T == U diag(1, 1, 1e-3) U^T

// k nearest points of the same cloud, ordered by (distance, index).
int knn_self(const float* xyz, int n, int i, int k, int* nb) {
    float nd[kMaxK];
    int cnt = 0;
    const float* xi = xyz + (size_t)3 * i;
    for (int j = 0; j < n; j++) {
        const float d = sqdist(xi, xyz + (size_t)3 * j);
        int pos;
        if (cnt < k) pos = cnt++;
        else if (d < nd[k - 1]) pos = k - 1;
        else continue;
        while (pos > 0 && nd[pos - 1] > d) {
            nd[pos] = nd[pos - 1];
            nb[pos] = nb[pos - 1];
            pos--;
        }
        nd[pos] = d;
        nb[pos] = j;
    }
    return cnt;
}

void plane_regularize(const double c[6], double out[6]) {
    double A[3][3] = {{c[0], c[1], c[2]}, {c[1], c[3], c[4]}, {c[2], c[4], c[5]}};
    double V[3][3] = {{1.0, 0.0, 0.0}, {0.0, 1.0, 0.0}, {0.0, 0.0, 1.0}};
    static const int PQ[3][2] = {{0, 1}, {0, 2}, {1, 2}};
    for (int sweep = 0; sweep < 6; sweep++)
        for (int r = 0; r < 3; r++) {
            const int p = PQ[r][0], q = PQ[r][1], o = 3 - p - q;
            const double apq = A[p][q];
            if (apq == 0.0) continue;
            const double theta = (A[q][q] - A[p][p]) / (2.0 * apq);
            double t = 1.0 / (std::fabs(theta) + std::sqrt(theta * theta + 1.0));
            if (theta < 0.0) t = -t;
            const double cc = 1.0 / std::sqrt(t * t + 1.0);
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
            for (int k = 0; k < 3; k++) {
                const double vkp = V[k][p], vkq = V[k][q];
                V[k][p] = cc * vkp - ss * vkq;
                V[k][q] = ss * vkp + cc * vkq;
            }
        }
    int m = 0;
    if (A[1][1] < A[m][m]) m = 1;
    if (A[2][2] < A[m][m]) m = 2;
    const double n0 = V[0][m], n1 = V[1][m], n2 = V[2][m];
    out[0] = 1.0 - kPlaneScale * (n0 * n0);
    out[1] = 0.0 - kPlaneScale * (n0 * n1);
    out[2] = 0.0 - kPlaneScale * (n0 * n2);
    out[3] = 1.0 - kPlaneScale * (n1 * n1);
    out[4] = 0.0 - kPlaneScale * (n1 * n2);
    out[5] = 1.0 - kPlaneScale * (n2 * n2);
}

void covariance_one(const float* xyz, int n, int i, int k, double* out6) {
    int nb[kMaxK];
    const int ke = knn_self(xyz, n, i, k, nb);
    double mx = 0.0, my = 0.0, mz = 0.0;
    for (int q = 0; q < ke; q++) {
        mx += (double)xyz[3 * (size_t)nb[q] + 0];
        my += (double)xyz[3 * (size_t)nb[q] + 1];
        mz += (double)xyz[3 * (size_t)nb[q] + 2];
    }
    const double kd = (double)ke;
    mx = mx / kd; my = my / kd; mz = mz / kd;
    double c[6] = {0.0, 0.0, 0.0, 0.0, 0.0, 0.0};
    for (int q = 0; q < ke; q++) {
        const double dx = (double)xyz[3 * (size_t)nb[q] + 0] - mx;
        const double dy = (double)xyz[3 * (size_t)nb[q] + 1] - my;
        const double dz = (double)xyz[3 * (size_t)nb[q] + 2] - mz;
        c[0] += dx * dx; c[1] += dx * dy; c[2] += dx * dz;
        c[3] += dy * dy; c[4] += dy * dz; c[5] += dz * dz;
    }
    for (int e = 0; e < 6; e++) c[e] = c[e] / kd;
    plane_regularize(c, out6);
}

// per-point Gauss-Newton contribution: acc[0..20] = upper(H) row-major, [21..26] = b, [27] = error
// Correspondence: the first strict minimum of the key of pcore_gicp_math.h over the segment (keys / org non-null:
// segments of <= kKeyScanMax targets), else of the float squared distance (larger segments; the GPU's exact
// grid search reproduces it).
bool gicp_contrib(const double R[3][3], const double t[3], const float* s, const double* cs, const float* tgt,
                  const double* tcov, int nt, const pcore::gicpm::NNTarget* keys, const float* org,
                  double acc[pcore::gicpm::kTerms]) {
    const double s0 = (double)s[0], s1 = (double)s[1], s2 = (double)s[2];
    double q[3];
    for (int r = 0; r < 3; r++) q[r] = R[r][0] * s0 + R[r][1] * s1 + R[r][2] * s2 + t[r];
    const float qf[3] = {(float)q[0], (float)q[1], (float)q[2]};
    int j = -1;
    float best = INFINITY;
    if (keys) {
        const float qx = qf[0] - org[0], qy = qf[1] - org[1], qz = qf[2] - org[2];
        if (std::isfinite(qx) && std::isfinite(qy) && std::isfinite(qz))
            for (int o = 0; o < nt; o++) {
                const pcore::gicpm::NNTarget& k = keys[o];
                const float d = pcore::gicpm::nn_key(k.m2x, k.m2y, k.m2z, k.tt, qx, qy, qz);
                if (d < best) { best = d; j = o; }
            }
    } else {
        for (int o = 0; o < nt; o++) {
            const float d = sqdist(qf, tgt + (size_t)3 * o);
            if (d < best) { best = d; j = o; }
        }
    }
    if (j < 0) return false;
    const double* ctp = tcov + (size_t)6 * j;
    const double ct[6] = {ctp[0], ctp[1], ctp[2], ctp[3], ctp[4], ctp[5]};
    const double csa[6] = {cs[0], cs[1], cs[2], cs[3], cs[4], cs[5]};
    const double Rm[3][3] = {{R[0][0], R[0][1], R[0][2]}, {R[1][0], R[1][1], R[1][2]}, {R[2][0], R[2][1], R[2][2]}};
    const double qa[3] = {q[0], q[1], q[2]};
    const double tj[3] = {(double)tgt[3 * (size_t)j + 0], (double)tgt[3 * (size_t)j + 1], (double)tgt[3 * (size_t)j + 2]};
    double a27[pcore::gicpm::kTerms];
    for (int v = 0; v < pcore::gicpm::kTerms; v++) a27[v] = acc[v];
    pcore::gicpm::contrib(Rm, qa, csa, tj, ct, a27);
    for (int v = 0; v < pcore::gicpm::kTerms; v++) acc[v] = a27[v];
    return true;
}

// 6x6 LDLT without pivoting; returns false if not positive definite.
bool ldlt_solve6(const double Hu[21], const double b[6], double d[6]) {
    double H[6][6];
    int h = 0;
    for (int a = 0; a < 6; a++)
        for (int c = a; c < 6; c++) { H[a][c] = Hu[h]; H[c][a] = Hu[h]; h++; }
    double L[6][6] = {}, D[6], iD[6];
    for (int j = 0; j < 6; j++) {
        double v = H[j][j];
        for (int k = 0; k < j; k++) v = v - L[j][k] * L[j][k] * D[k];
        if (!(v > 0.0) || !std::isfinite(v)) return false;
        D[j] = v;
        iD[j] = 1.0 / v;  // one division per column; the column and the back substitution multiply by it
        for (int i = j + 1; i < 6; i++) {
            double w = H[i][j];
            for (int k = 0; k < j; k++) w = w - L[i][k] * L[j][k] * D[k];
            L[i][j] = w * iD[j];
        }
    }
    double y[6];
    for (int i = 0; i < 6; i++) {
        double v = -b[i];
        for (int k = 0; k < i; k++) v = v - L[i][k] * y[k];
        y[i] = v;
    }
    for (int i = 5; i >= 0; i--) {
        double v = y[i] * iD[i];
        for (int k = i + 1; k < 6; k++) v = v - L[k][i] * d[k];
        d[i] = v;
    }
    for (int i = 0; i < 6; i++)
        if (!std::isfinite(d[i])) return false;
    return true;
}

}  // namespace

extern "C" {

void orc_covariances(const float* xyz, int n, int k, double* out_cov6) {
    if (k > kMaxK) k = kMaxK;
#pragma omp parallel for schedule(static)
    for (int i = 0; i < n; i++) covariance_one(xyz, n, i, k, out_cov6 + (size_t)6 * i);
}

int orc_gicp(const float* src_xyz, const double* src_cov, int ns, const float* tgt_xyz, const double* tgt_cov, int nt,
             int max_iter, double rot_eps, double trans_eps, double* out_T) {
    double R[3][3] = {{1.0, 0.0, 0.0}, {0.0, 1.0, 0.0}, {0.0, 0.0, 1.0}};
    double t[3] = {0.0, 0.0, 0.0};
    int it = 0;
    if (ns > 0 && nt > 0) {
        std::vector<double> part((size_t)kGicpThreads * pcore::gicpm::kTerms);
        std::vector<pcore::gicpm::NNTarget> keys;
        float org[3] = {0.0f, 0.0f, 0.0f};
        if (nt <= pcore::gicpm::kKeyScanMax) {
            pcore::gicpm::nn_origin(nt, [&](int i, float* p) {
                for (int a = 0; a < 3; a++) p[a] = tgt_xyz[(size_t)3 * i + a];
            }, org);
            keys.resize(nt);
            for (int i = 0; i < nt; i++)
                keys[i] = pcore::gicpm::nn_target(tgt_xyz[3 * (size_t)i], tgt_xyz[3 * (size_t)i + 1],
                                                  tgt_xyz[3 * (size_t)i + 2], org[0], org[1], org[2]);
        }
        for (it = 0; it < max_iter;) {
            std::fill(part.begin(), part.end(), 0.0);
            for (int i = 0; i < ns; i++)
                gicp_contrib(R, t, src_xyz + (size_t)3 * i, src_cov + (size_t)6 * i, tgt_xyz, tgt_cov, nt,
                             keys.empty() ? nullptr : keys.data(), org,
                             part.data() + (size_t)pcore::gicpm::kTerms * (i % kGicpThreads));
            // fixed reduction: per wave shuffle-down tree to lane 0, then the 4 waves in order
            double tot[pcore::gicpm::kTerms];
            for (int v = 0; v < pcore::gicpm::kTerms; v++) {
                double wsum[kGicpThreads / 64];
                for (int w = 0; w < kGicpThreads / 64; w++) {
                    double lane[64];
                    for (int l = 0; l < 64; l++) lane[l] = part[(size_t)pcore::gicpm::kTerms * (w * 64 + l) + v];
                    for (int off = 32; off > 0; off >>= 1)
                        for (int l = 0; l < off; l++) lane[l] = lane[l] + lane[l + off];
                    wsum[w] = lane[0];
                }
                double s = wsum[0];
                for (int w = 1; w < kGicpThreads / 64; w++) s = s + wsum[w];
                tot[v] = s;
            }
            double d[6];
            if (!ldlt_solve6(tot, tot + 21, d)) break;
            it++;
            double qw = 1.0, qx = d[0] * 0.5, qy = d[1] * 0.5, qz = d[2] * 0.5;
            const double nrm = std::sqrt(qw * qw + qx * qx + qy * qy + qz * qz);
            const double inv = 1.0 / nrm;
            qw = qw * inv; qx = qx * inv; qy = qy * inv; qz = qz * inv;
            const double xx = qx * qx, yy = qy * qy, zz = qz * qz, xy = qx * qy, xz = qx * qz, yz = qy * qz;
            const double wx = qw * qx, wy = qw * qy, wz = qw * qz;
            const double Rd[3][3] = {{1.0 - 2.0 * (yy + zz), 2.0 * (xy - wz), 2.0 * (xz + wy)},
                                     {2.0 * (xy + wz), 1.0 - 2.0 * (xx + zz), 2.0 * (yz - wx)},
                                     {2.0 * (xz - wy), 2.0 * (yz + wx), 1.0 - 2.0 * (xx + yy)}};
            double Rn[3][3], tn[3];
            for (int r = 0; r < 3; r++) {
                for (int c = 0; c < 3; c++) Rn[r][c] = Rd[r][0] * R[0][c] + Rd[r][1] * R[1][c] + Rd[r][2] * R[2][c];
                tn[r] = Rd[r][0] * t[0] + Rd[r][1] * t[1] + Rd[r][2] * t[2] + d[3 + r];
            }
            double dr = 0.0, dt = 0.0;
            for (int r = 0; r < 3; r++) {
                for (int c = 0; c < 3; c++) {
                    const double v = std::fabs(Rd[r][c] - (r == c ? 1.0 : 0.0));
                    dr = v > dr ? v : dr;
                }
                const double v = std::fabs(d[3 + r]);
                dt = v > dt ? v : dt;
            }
            std::memcpy(R, Rn, sizeof(R));
            std::memcpy(t, tn, sizeof(t));
            if (dr < rot_eps && dt < trans_eps) break;
        }
    }
    for (int r = 0; r < 3; r++) {
        for (int c = 0; c < 3; c++) out_T[4 * r + c] = R[r][c];
        out_T[4 * r + 3] = t[r];
    }
    out_T[12] = 0.0; out_T[13] = 0.0; out_T[14] = 0.0; out_T[15] = 1.0;
    return it;
}

void orc_concat_pose(const double* T, const float* pose, float* out_pose) {
    float A[4][4], Tf[4][4], P[4][4];
    for (int r = 0; r < 4; r++)
        for (int c = 0; c < 4; c++) {
            A[r][c] = r < 3 ? pose[4 * r + c] / 100.0f : pose[4 * r + c];  // to_eigen(100)
            Tf[r][c] = (float)T[4 * r + c];                                // Isometry3f
        }
    for (int r = 0; r < 4; r++)
        for (int c = 0; c < 4; c++) P[r][c] = Tf[r][0] * A[0][c] + Tf[r][1] * A[1][c] + Tf[r][2] * A[2][c] + Tf[r][3] * A[3][c];
    for (int r = 0; r < 4; r++)
        for (int c = 0; c < 4; c++) out_pose[4 * r + c] = r < 3 ? (float)((double)P[r][c] * 100) : P[r][c];
}

void orc_evaluate_icp(const float* tris, int num_tris, const int32_t* tris_model_count, int num_models,
                      const float* poses, const int32_t* pose_model, const int32_t* pose_label, int num_poses,
                      int width, int height, const float* proj, const int32_t* src_depth, const uint8_t* src_mask,
                      float occlusion_threshold, int stride, float cx, float cy, float fx, float fy,
                      float depth_factor, const float* o_xyz, const double* o_cov, int num_o,
                      const int32_t* label_start, const int32_t* label_end, int num_labels,
                      const float* pose_obs_total, int cost_type, int calc_obs, float sensor_resolution, int k_corr,
                      int max_iter, double rot_eps, double trans_eps, float* out_adj, int32_t* out_iters,
                      float* out_rc, float* out_oc, float* out_diff, int nthreads) {
    (void)num_tris;
    std::vector<int> lo, hi;
    model_ranges(tris_model_count, num_models, lo, hi);
    const bool use_seg = pose_label != nullptr;
    const size_t npx = (size_t)width * height;
    const int ws = (width + stride - 1) / stride, hs = (height + stride - 1) / stride;
    if (nthreads > 0) omp_set_num_threads(nthreads);
#pragma omp parallel
    {
        std::vector<int32_t> depth(npx);
        std::vector<float> xyz((size_t)3 * ws * hs);
        std::vector<double> cov((size_t)6 * ws * hs);
        std::vector<float> d2((size_t)ws * hs);
        std::vector<int32_t> nn((size_t)ws * hs), rpose((size_t)ws * hs, 0);
#pragma omp for schedule(dynamic, 1)
        for (int n = 0; n < num_poses; n++) {
            const int m = pose_model[n];
            const int32_t pl = use_seg ? pose_label[n] : 0;
            int l0 = 0, l1 = num_o;
            if (use_seg && label_start != nullptr) {
                if (pl < 0 || pl >= num_labels) { l0 = 0; l1 = 0; }
                else { l0 = label_start[pl]; l1 = label_end[pl]; }
            }
            const float* pose = poses + (size_t)16 * n;
            render_one_pose(tris, lo[m], hi[m], pose, width, height, proj, src_depth, src_mask, use_seg, pl,
                            occlusion_threshold, depth.data());
            int nr = orc_depth_to_cloud(depth.data(), 1, width, height, stride, cx, cy, fx, fy, depth_factor, nullptr,
                                        nullptr, xyz.data(), nullptr, nullptr, ws * hs);
            int k = k_corr > kMaxK ? kMaxK : k_corr;
            for (int i = 0; i < nr; i++) covariance_one(xyz.data(), nr, i, k, cov.data() + (size_t)6 * i);
            double T[16];
            const int iters = orc_gicp(xyz.data(), cov.data(), nr, o_xyz + (size_t)3 * l0, o_cov + (size_t)6 * l0,
                                       l1 - l0, max_iter, rot_eps, trans_eps, T);
            if (out_iters) out_iters[n] = iters;
            float* adj = out_adj + (size_t)16 * n;
            orc_concat_pose(T, pose, adj);
            render_one_pose(tris, lo[m], hi[m], adj, width, height, proj, src_depth, src_mask, use_seg, pl,
                            occlusion_threshold, depth.data());
            nr = orc_depth_to_cloud(depth.data(), 1, width, height, stride, cx, cy, fx, fy, depth_factor, nullptr,
                                    nullptr, xyz.data(), nullptr, nullptr, ws * hs);
            for (int i = 0; i < nr; i++) knn1_range(xyz.data() + (size_t)3 * i, o_xyz, l0, l1, d2[i], nn[i]);
            float rc, oc, df;
            const float tot = pose_obs_total ? pose_obs_total[n] : 0.0f;
            orc_costs(1, cost_type, calc_obs, sensor_resolution, d2.data(), nn.data(), rpose.data(), nr, num_o, &tot,
                      &rc, &oc, &df);
            out_rc[n] = rc;
            out_oc[n] = oc;
            out_diff[n] = df;
        }
    }
}


// rgb2lab (compute_costs.cuh:57-88) in double, with the cost's channel order rgb2lab(c2, c1, c0)
// (compute_costs.cuh:214-220).
void orc_rgb2lab(const uint8_t c[3], float lab[3]) {
    double r = c[2] / 255.0, g = c[1] / 255.0, b = c[0] / 255.0;
    r = ((r > 0.04045) ? std::pow((r + 0.055) / 1.055, 2.4) : (r / 12.92)) * 100.0;
    g = ((g > 0.04045) ? std::pow((g + 0.055) / 1.055, 2.4) : (g / 12.92)) * 100.0;
    b = ((b > 0.04045) ? std::pow((b + 0.055) / 1.055, 2.4) : (b / 12.92)) * 100.0;
    double x = r * 0.4124564 + g * 0.3575761 + b * 0.1804375;
    double y = r * 0.2126729 + g * 0.7151522 + b * 0.0721750;
    double z = r * 0.0193339 + g * 0.1191920 + b * 0.9503041;
    x = x / 95.047;
    y = y / 100.00;
    z = z / 108.883;
    x = (x > 0.008856) ? std::cbrt(x) : (7.787 * x + 16.0 / 116.0);
    y = (y > 0.008856) ? std::cbrt(y) : (7.787 * y + 16.0 / 116.0);
    z = (z > 0.008856) ? std::cbrt(z) : (7.787 * z + 16.0 / 116.0);
    lab[0] = (float)((116.0 * y) - 16);
    lab[1] = (float)(500 * (x - y));
    lab[2] = (float)(200 * (y - z));
}

double orc_colour_distance(const float* lab1, const float* lab2) {
    return pcore::colour::colour_distance(lab1[0], lab1[1], lab1[2], lab2[0], lab2[1], lab2[2]);
}

float orc_sin_f(float x) { return pcore::colour::sin_f(x); }
float orc_cos_f(float x) { return pcore::colour::cos_f(x); }
float orc_exp_f(float x) { return pcore::colour::exp_f(x); }
float orc_atan2_f(float y, float x) { return pcore::colour::atan2_f(y, x); }

// Cost type 1 (3-DoF RGB-D): as orc_evaluate without labels, plus the colour gate of
// compute_render_cost (compute_costs.cuh:201-240): a point within the sensor radius of its nearest
// observed point is explained only if CIEDE2000(observed, rendered) <= colour_thr, else it is bad.
// Rendered colour = tri_rgb of the first triangle (serial order) reaching the pixel's minimum depth.
void orc_evaluate_colour(const float* tris, int num_tris, const uint8_t* tri_rgb, const int32_t* tris_model_count,
                         int num_models, const float* poses, const int32_t* pose_model, int num_poses, int width,
                         int height, const float* proj, const int32_t* src_depth, float occlusion_threshold,
                         int stride, float cx, float cy, float fx, float fy, float depth_factor, const float* o_xyz,
                         const uint8_t* o_rgb, int num_o, const float* pose_obs_total, int calc_obs,
                         float sensor_resolution, float colour_thr, float* out_rc, float* out_oc, float* out_diff,
                         int nthreads) {
    std::vector<int> lo, hi;
    model_ranges(tris_model_count, num_models, lo, hi);
    const size_t npx = (size_t)width * height;
    std::vector<float> tri_lab((size_t)3 * num_tris), o_lab((size_t)3 * (num_o > 0 ? num_o : 1));
    for (int t = 0; t < num_tris; t++) orc_rgb2lab(tri_rgb + (size_t)3 * t, &tri_lab[(size_t)3 * t]);
    for (int o = 0; o < num_o; o++) orc_rgb2lab(o_rgb + (size_t)3 * o, &o_lab[(size_t)3 * o]);
    const float r2 = sensor_resolution * sensor_resolution;
    if (nthreads > 0) omp_set_num_threads(nthreads);
#pragma omp parallel
    {
        std::vector<int32_t> depth(npx), dmin(npx), tid(npx);
        std::vector<uint8_t> explained(num_o > 0 ? num_o : 1);
#pragma omp for schedule(dynamic, 1)
        for (int n = 0; n < num_poses; n++) {
            const int m = pose_model[n];
            render_one_pose(tris, lo[m], hi[m], poses + (size_t)16 * n, width, height, proj, src_depth, nullptr,
                            false, 0, occlusion_threshold, depth.data(), dmin.data(), tid.data());
            std::fill(explained.begin(), explained.end(), 0);
            float num = 0.0f, bad = 0.0f;
            for (int y = 0; y < height; y += stride)
                for (int x = 0; x < width; x += stride) {
                    const size_t idx = (size_t)x + (size_t)y * width;
                    if (depth[idx] <= 0) continue;
                    float q[3];
                    transform_point(x, y, depth[idx], cx, cy, fx, fy, depth_factor, q[0], q[1], q[2]);
                    float d2;
                    int32_t nn;
                    knn1_range(q, o_xyz, 0, num_o, d2, nn);
                    num += 1.0f;
                    if (d2 > r2) { bad += 1.0f; continue; }
                    if (nn < 0) continue;
                    const int t = tid[idx];
                    const double cd = orc_colour_distance(&o_lab[(size_t)3 * nn], &tri_lab[(size_t)3 * t]);
                    if (cd > (double)colour_thr) bad += 1.0f;
                    else explained[nn] = 1;
                }
            const float rendered_explained = num - bad;
            float rc = (num == 0) ? -1.0f : bad / num;
            rc = (rc == -1.0f) ? -1.0f : rc * 100.0f;
            out_rc[n] = rc;
            if (calc_obs) {
                float expl = 0.0f;
                for (int o = 0; o < num_o; o++) expl += (float)explained[o];
                out_diff[n] = rendered_explained - expl;
                float oc = pose_obs_total[n] - expl;
                oc = oc / pose_obs_total[n];
                out_oc[n] = oc * 100.0f;
            } else {
                out_oc[n] = 0.0f;
                out_diff[n] = 0.0f;
            }
        }
    }
}

}  // extern "C"
