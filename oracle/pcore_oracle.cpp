// pcore_oracle.cpp -- CPU restatement of the reference hot path.  TEST INFRASTRUCTURE ONLY.
// See pcore_oracle.h for the parity status ("parity unpinned" vs the reference binary).
// Build: oracle/Makefile (g++ -O2 -ffp-contract=off -fno-fast-math -fopenmp).
#include "pcore_oracle.h"

// The colour spec (deterministic sin / cos / atan2 / exp, CIEDE2000 term order) is shared with the GPU
// build: it defines the arithmetic, like the GICP spec; tests/test_colour_spec.py pins it against numpy.
#include "../perception_amd/csrc/pcore_colour.h"
#include "../perception_amd/csrc/pcore_gicp_math.h"

#include <array>
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
                           int32_t* tri_id = nullptr, int32_t t = 0, const uint8_t* rgb = nullptr,
                           uint8_t* col = nullptr) {
    const size_t npx = (size_t)width * height;
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
            // z-test (image_renderer.cuh:146-159), serial order; the colour planes with the depth
            if (curr < depth[idx]) {
                depth[idx] = curr;
                if (col) {
                    col[idx] = rgb[0];
                    col[npx + idx] = rgb[1];
                    col[2 * npx + idx] = rgb[2];
                }
            }
            const int32_t nd = depth[idx];
            const int32_t src = src_depth[idx];
            const int lab = use_seg ? (int)src_mask[idx] : 0;
            // source occlusion black-out (image_renderer.cuh:160-196)
            if ((!use_seg && (float)iabs_wrap(nd, src) > occlusion_threshold) ||
                (use_seg && pose_label != lab - 1 && (float)iabs_wrap(nd, src) > 0.5f)) {
                if (nd > src && src > 0) {
                    if (col) col[idx] = col[npx + idx] = col[2 * npx + idx] = 0;
                    depth[idx] = INT_MAX;
                }
            }
        }
    }
}

void render_one_pose(const float* tris, int lo, int hi, const float* pose, int width, int height,
                     const float* proj, const int32_t* src_depth, const uint8_t* src_mask, bool use_seg,
                     int32_t pose_label, float occlusion_threshold, int32_t* depth, int32_t* dmin = nullptr,
                     int32_t* tri_id = nullptr, const uint8_t* tri_rgb = nullptr, uint8_t* col = nullptr) {
    const size_t npx = (size_t)width * height;
    for (size_t i = 0; i < npx; i++) depth[i] = INT_MAX;
    if (col != nullptr) std::memset(col, 0, 3 * npx);
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
        static const uint8_t grey[3] = {128, 128, 128};  // model.cpp:97-101
        rasterize_with_source(projd, last_row, depth, width, height, src_depth, src_mask, use_seg, pose_label,
                              occlusion_threshold, dmin, tri_id, t,
                              col ? (tri_rgb ? tri_rgb + (size_t)3 * t : grey) : nullptr, col);
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

// Stage RENDER with the colour planes: out_col = 3 planes (red, green, blue) per pose, pose-major (3 x H x W each);
// tri_rgb nullable (grey 128).
void orc_render_depth_color(const float* tris, int num_tris, const uint8_t* tri_rgb, const int32_t* tris_model_count,
                            int num_models, const float* poses, const int32_t* pose_model, const int32_t* pose_label,
                            int num_poses, int width, int height, const float* proj, const int32_t* src_depth,
                            const uint8_t* src_mask, float occlusion_threshold, int32_t* out, uint8_t* out_col,
                            int nthreads) {
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
                        use_seg, use_seg ? pose_label[n] : 0, occlusion_threshold, out + npx * n, nullptr, nullptr,
                        tri_rgb, out_col + 3 * npx * n);
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
    // at most 6 cyclic sweeps; a rotation is skipped when |A_pq| <= max(2 eps max_i |A_ii|, the smallest normal double)
    // (Eigen JacobiSVD's threshold), and a sweep without a rotation ends the loop
    for (int sweep = 0; sweep < 6; sweep++) {
        bool rotated = false;
        for (int r = 0; r < 3; r++) {
            const int p = PQ[r][0], q = PQ[r][1], o = 3 - p - q;
            const double apq = A[p][q];
            const double d0 = std::fabs(A[0][0]), d1 = std::fabs(A[1][1]), d2 = std::fabs(A[2][2]);
            double dm = d0 > d1 ? d0 : d1;
            dm = dm > d2 ? dm : d2;
            double thr = 4.440892098500626e-16 * dm;
            thr = thr > 2.2250738585072014e-308 ? thr : 2.2250738585072014e-308;
            if (std::fabs(apq) <= thr) continue;
            rotated = true;
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
        if (!rotated) break;
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

// Correspondence of the float query qf (fast_gicp update_correspondences): the first strict minimum of the key of
// pcore_gicp_math.h over the segment (keys / org non-null: segments of <= kKeyScanMax targets), else of the float
// squared distance (larger segments; the GPU's exact grid search reproduces it).  -1: no correspondence.
int gicp_nn(const float qf[3], const float* tgt, int nt, const pcore::gicpm::NNTarget* keys, const float* org) {
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
    return j;
}

// The segment's correspondence keys (empty for segments above kKeyScanMax)
void gicp_keys(const float* tgt_xyz, int nt, std::vector<pcore::gicpm::NNTarget>& keys, float org[3]) {
    keys.clear();
    org[0] = org[1] = org[2] = 0.0f;
    if (nt > pcore::gicpm::kKeyScanMax) return;
    float o3[3];
    pcore::gicpm::nn_origin(nt, [&](int i, float* p) {
        for (int a = 0; a < 3; a++) p[a] = tgt_xyz[(size_t)3 * i + a];
    }, o3);
    for (int a = 0; a < 3; a++) org[a] = o3[a];
    keys.resize(nt);
    for (int i = 0; i < nt; i++)
        keys[i] = pcore::gicpm::nn_target(tgt_xyz[3 * (size_t)i], tgt_xyz[3 * (size_t)i + 1], tgt_xyz[3 * (size_t)i + 2],
                                          org[0], org[1], org[2]);
}

struct OXform {
    double R[3][3];
    double t[3];
};

// the GPU's reduction: 64 per-lane sequential partials (point i -> lane i % 64), then the wave shuffle-down tree
double lane_tree(const double* part, int stride, int v) {
    double lane[64];
    for (int l = 0; l < 64; l++) lane[l] = part[(size_t)stride * l + v];
    for (int off = 32; off > 0; off >>= 1)
        for (int l = 0; l < off; l++) lane[l] = lane[l] + lane[l + off];
    return lane[0];
}

// Linearisation at x (fast_gicp linearize): correspondences, per-point Mahalanobis matrices and the 28 reduced
// terms (upper H, b, error), in the GPU's order.
void gicp_linearize_spec(const OXform& x, const float* src_xyz, const double* src_cov, int ns, const float* tgt_xyz,
                         const double* tgt_cov, int nt, const pcore::gicpm::NNTarget* keys, const float* org,
                         int32_t* corr, double* mah, double sys[pcore::gicpm::kTerms]) {
    constexpr int NT = pcore::gicpm::kTerms;
    std::vector<double> part((size_t)64 * NT, 0.0);
    float Rf[3][3], tf[3];
    for (int r = 0; r < 3; r++) {
        for (int c = 0; c < 3; c++) Rf[r][c] = (float)x.R[r][c];
        tf[r] = (float)x.t[r];
    }
    for (int i = 0; i < ns; i++) {
        const float* s = src_xyz + (size_t)3 * i;
        float qf[3];
        pcore::gicpm::query_f(Rf, tf, s[0], s[1], s[2], qf);
        const int j = gicp_nn(qf, tgt_xyz, nt, keys, org);
        corr[i] = j;
        if (j < 0) continue;
        double q[3];
        pcore::gicpm::transform_point(x.R, x.t, (double)s[0], (double)s[1], (double)s[2], q);
        double cs[6], ct[6], M6[6], acc[NT];
        for (int e = 0; e < 6; e++) { cs[e] = src_cov[(size_t)6 * i + e]; ct[e] = tgt_cov[(size_t)6 * j + e]; }
        const double tj[3] = {(double)tgt_xyz[3 * (size_t)j + 0], (double)tgt_xyz[3 * (size_t)j + 1],
                              (double)tgt_xyz[3 * (size_t)j + 2]};
        double* pl = part.data() + (size_t)NT * (i % 64);
        for (int v = 0; v < NT; v++) acc[v] = pl[v];
        pcore::gicpm::contrib(x.R, q, cs, tj, ct, acc, M6);
        for (int v = 0; v < NT; v++) pl[v] = acc[v];
        for (int e = 0; e < 6; e++) mah[(size_t)6 * i + e] = M6[e];
    }
    for (int v = 0; v < NT; v++) sys[v] = lane_tree(part.data(), NT, v);
}

// Test reference only: the damped solve as fast_gicp performs it, Eigen's LDLT with diagonal pivoting
// (Eigen 3 LDLT::compute -> ldlt_inplace<Lower>::unblocked, left-looking: the pivot is the largest |diagonal| of the
// not yet factored part, swapped in place; D's pseudo-inverse zeroes pivots below the smallest normal), then
// P^T L^-T D^+ L^-1 P (-b).  The spec solves by block elimination (lm_solve_schur); orc_gicp_trace(solver = 1)
// runs whole chains on this one so tests can measure where the two solves change an LM decision.
void ldlt_solve_ref(const double* sys, double lambda, double (&d)[6]) {
    double A[6][6];
    int h = 0;
    for (int a = 0; a < 6; a++)
        for (int c = a; c < 6; c++) {
            A[c][a] = a == c ? sys[h] + lambda : sys[h];  // the lower triangle of H + lambda I
            h++;
        }
    int tr[6];
    bool zero = false;
    for (int k = 0; k < 6; k++) {
        int p = k;
        double big = std::fabs(A[k][k]);
        for (int i = k + 1; i < 6; i++)
            if (std::fabs(A[i][i]) > big) { big = std::fabs(A[i][i]); p = i; }
        tr[k] = p;
        if (p != k) {  // symmetric swap of rows / columns k and p in the lower triangle
            for (int j = 0; j < k; j++) std::swap(A[k][j], A[p][j]);
            for (int i = p + 1; i < 6; i++) std::swap(A[i][k], A[i][p]);
            std::swap(A[k][k], A[p][p]);
            for (int i = k + 1; i < p; i++) std::swap(A[i][k], A[p][i]);
        }
        if (k > 0) {
            double temp[6];
            for (int j = 0; j < k; j++) temp[j] = A[j][j] * A[k][j];
            double s = A[k][0] * temp[0];
            for (int j = 1; j < k; j++) s = s + A[k][j] * temp[j];
            A[k][k] = A[k][k] - s;
            for (int i = k + 1; i < 6; i++) {
                double w = A[i][0] * temp[0];
                for (int j = 1; j < k; j++) w = w + A[i][j] * temp[j];
                A[i][k] = A[i][k] - w;
            }
        }
        const double akk = A[k][k];
        if (k == 0 && !(std::fabs(akk) > 0.0)) {  // the whole diagonal is zero
            zero = true;
            break;
        }
        if (std::fabs(akk) > 0.0)
            for (int i = k + 1; i < 6; i++) A[i][k] = A[i][k] / akk;
    }
    double x[6];
    for (int i = 0; i < 6; i++) x[i] = -sys[21 + i];
    if (zero) {
        for (int i = 0; i < 6; i++) d[i] = 0.0;
        return;
    }
    for (int k = 0; k < 6; k++) std::swap(x[k], x[tr[k]]);
    for (int j = 0; j < 6; j++)
        for (int i = j + 1; i < 6; i++) x[i] = x[i] - x[j] * A[i][j];
    for (int i = 0; i < 6; i++) {
        const double Di = A[i][i];
        x[i] = std::fabs(Di) > 2.2250738585072014e-308 ? x[i] / Di : 0.0;
    }
    for (int i = 4; i >= 0; i--) {
        double s = A[i + 1][i] * x[i + 1];
        for (int j = i + 2; j < 6; j++) s = s + A[j][i] * x[j];
        x[i] = x[i] - s;
    }
    for (int k = 5; k >= 0; k--) std::swap(x[k], x[tr[k]]);
    for (int i = 0; i < 6; i++) d[i] = x[i];
}

// One LM iteration (LsqRegistration::step_lm) on the reduced system, as the GPU's lm_iteration
int gicp_lm_iteration(const double sys[pcore::gicpm::kTerms], OXform& x, double& lambda, const float* src_xyz, int ns,
                      const float* tgt_xyz, const int32_t* corr, const double* mah, double rot_eps, double trans_eps,
                      double* lambda_used, int* trials = nullptr, int* flags = nullptr, int solver = 0) {
    namespace gm = pcore::gicpm;
    const double y0 = sys[gm::kErr];
    if (lambda < 0.0) lambda = gm::lm_init_lambda(sys);
    double nu = 2.0;
    std::vector<double> part(64);
    *lambda_used = lambda;
    if (flags) *flags = gm::lm_lambda_inert(sys, lambda) ? 1 : 0;
    for (int trial = 0; trial < gm::kLmMaxTrials; trial++) {
        if (trials) *trials = trial + 1;
        double d[6];
        if (solver == 1) ldlt_solve_ref(sys, lambda, d);
        else gm::lm_solve_schur(sys, lambda, d);
        if (!gm::all_finite6(d)) return gm::kLmFailed;
        double Rd[3][3], td[3];
        gm::se3_exp(d, Rd, td, gm::kSe3Coef);
        OXform xi;
        gm::compose(Rd, td, x.R, x.t, xi.R, xi.t);
        std::fill(part.begin(), part.end(), 0.0);
        for (int i = 0; i < ns; i++) {
            const int j = corr[i];
            if (j < 0) continue;
            double q[3];
            gm::transform_point(xi.R, xi.t, (double)src_xyz[3 * (size_t)i], (double)src_xyz[3 * (size_t)i + 1],
                                (double)src_xyz[3 * (size_t)i + 2], q);
            double e[3];
            for (int r = 0; r < 3; r++) e[r] = (double)tgt_xyz[3 * (size_t)j + r] - q[r];
            double M6[6];
            for (int k = 0; k < 6; k++) M6[k] = mah[(size_t)6 * i + k];
            part[i % 64] = gm::mahal_err_add(M6, e, part[i % 64]);
        }
        const double yi = lane_tree(part.data(), 1, 0);
        const double rho = gm::lm_rho(sys, lambda, d, y0, yi);
        if (rho < 0.0) {
            if (gm::is_converged(Rd, td, rot_eps, trans_eps)) return gm::kLmConverged;
            lambda = nu * lambda;
            nu = 2.0 * nu;
            continue;
        }
        x = xi;
        if (flags && rho >= 0.5) *flags |= 2;
        lambda = gm::lm_accept_lambda(lambda, rho);
        return gm::is_converged(Rd, td, rot_eps, trans_eps) ? gm::kLmConverged : gm::kLmAccepted;
    }
    return gm::kLmFailed;
}

// ---- independent textbook restatement of one point's linearisation (test reference; shares nothing with
// pcore_gicp_math.h): fast_gicp's 4x4 homogeneous form in long double,
//   RCR = C_B + T C_A T^T, RCR(3,3) = 1, M = RCR^-1 (Gauss-Jordan, partial pivoting), M(3,3) = 0,
//   e = mean_B - T mean_A, J = [[skew(T mean_A), -I], [0, 0]] (4 x 6), H += J^T M J, b += J^T M e, y += e^T M e.
typedef long double ld;

void inverse4(const ld A[4][4], ld out[4][4]) {
    ld M[4][8];
    for (int r = 0; r < 4; r++)
        for (int c = 0; c < 8; c++) M[r][c] = c < 4 ? A[r][c] : (c - 4 == r ? 1.0L : 0.0L);
    for (int k = 0; k < 4; k++) {
        int p = k;
        for (int r = k + 1; r < 4; r++)
            if (std::fabs(M[r][k]) > std::fabs(M[p][k])) p = r;
        if (p != k)
            for (int c = 0; c < 8; c++) std::swap(M[k][c], M[p][c]);
        const ld piv = M[k][k];
        for (int c = 0; c < 8; c++) M[k][c] /= piv;
        for (int r = 0; r < 4; r++) {
            if (r == k) continue;
            const ld f = M[r][k];
            for (int c = 0; c < 8; c++) M[r][c] -= f * M[k][c];
        }
    }
    for (int r = 0; r < 4; r++)
        for (int c = 0; c < 4; c++) out[r][c] = M[r][c + 4];
}

void textbook_point(const ld T[4][4], const float* s, const double* cs6, const float* tj, const double* ct6, ld H[6][6],
                    ld b[6], ld& err) {
    const ld mA[4] = {(ld)s[0], (ld)s[1], (ld)s[2], 1.0L};
    const ld mB[4] = {(ld)tj[0], (ld)tj[1], (ld)tj[2], 1.0L};
    ld CA[4][4] = {}, CB[4][4] = {};
    const int sym[3][3] = {{0, 1, 2}, {1, 3, 4}, {2, 4, 5}};
    for (int r = 0; r < 3; r++)
        for (int c = 0; c < 3; c++) {
            CA[r][c] = (ld)cs6[sym[r][c]];
            CB[r][c] = (ld)ct6[sym[r][c]];
        }
    ld tA[4];
    for (int r = 0; r < 4; r++) {
        tA[r] = 0.0L;
        for (int k = 0; k < 4; k++) tA[r] += T[r][k] * mA[k];
    }
    ld TC[4][4], RCR[4][4];
    for (int r = 0; r < 4; r++)
        for (int c = 0; c < 4; c++) {
            TC[r][c] = 0.0L;
            for (int k = 0; k < 4; k++) TC[r][c] += T[r][k] * CA[k][c];
        }
    for (int r = 0; r < 4; r++)
        for (int c = 0; c < 4; c++) {
            ld v = 0.0L;
            for (int k = 0; k < 4; k++) v += TC[r][k] * T[c][k];
            RCR[r][c] = CB[r][c] + v;
        }
    RCR[3][3] = 1.0L;
    ld M[4][4];
    inverse4(RCR, M);
    M[3][3] = 0.0L;
    ld e[4];
    for (int r = 0; r < 4; r++) e[r] = mB[r] - tA[r];
    ld J[4][6] = {};
    J[0][1] = -tA[2]; J[0][2] = tA[1];
    J[1][0] = tA[2];  J[1][2] = -tA[0];
    J[2][0] = -tA[1]; J[2][1] = tA[0];
    J[0][3] = -1.0L; J[1][4] = -1.0L; J[2][5] = -1.0L;
    ld MJ[4][6], Me[4];
    for (int r = 0; r < 4; r++) {
        for (int c = 0; c < 6; c++) {
            MJ[r][c] = 0.0L;
            for (int k = 0; k < 4; k++) MJ[r][c] += M[r][k] * J[k][c];
        }
        Me[r] = 0.0L;
        for (int k = 0; k < 4; k++) Me[r] += M[r][k] * e[k];
    }
    for (int a = 0; a < 6; a++) {
        for (int c = 0; c < 6; c++) {
            ld v = 0.0L;
            for (int k = 0; k < 4; k++) v += J[k][a] * MJ[k][c];
            H[a][c] += v;
        }
        ld v = 0.0L;
        for (int k = 0; k < 4; k++) v += J[k][a] * Me[k];
        b[a] += v;
    }
    ld y = 0.0L;
    for (int k = 0; k < 4; k++) y += e[k] * Me[k];
    err += y;
}

}  // namespace

extern "C" {

void orc_covariances(const float* xyz, int n, int k, double* out_cov6) {
    if (k > kMaxK) k = kMaxK;
#pragma omp parallel for schedule(static)
    for (int i = 0; i < n; i++) covariance_one(xyz, n, i, k, out_cov6 + (size_t)6 * i);
}

// The spec's GICP with an optional per-iteration trace (max_iter x 16: R, t after the iteration, the lambda of its
// first trial, its number of trials, flags (1: lambda inert on its system, 2: accepted with rho >= 1/2), the LM
// status) and the cycle exit of window cycle_window (0: off; pcore_gicp_math.h cycle_update).  Returns the iterations
// reported (max_iter after a cycle exit); *executed (nullable) the iterations run.
int orc_gicp_trace(const float* src_xyz, const double* src_cov, int ns, const float* tgt_xyz, const double* tgt_cov,
                   int nt, int max_iter, double rot_eps, double trans_eps, int cycle_window, double* out_T,
                   double* trace, int* executed, int solver) {
    namespace gm = pcore::gicpm;
    OXform x;
    for (int r = 0; r < 3; r++) {
        for (int c = 0; c < 3; c++) x.R[r][c] = r == c ? 1.0 : 0.0;
        x.t[r] = 0.0;
    }
    int it = 0, reported = 0;
    if (ns > 0 && nt > 0) {
        std::vector<gm::NNTarget> keys;
        float org[3];
        gicp_keys(tgt_xyz, nt, keys, org);
        std::vector<int32_t> corr(ns);
        std::vector<double> mah((size_t)6 * ns);
        // T_f(j), j = 1.. (float(x_{j-1}), bit patterns): the cycle exit's record
        std::vector<std::array<uint32_t, 12>> tf;
        auto float_bits = [](const OXform& v) {
            std::array<uint32_t, 12> b;
            for (int r = 0; r < 3; r++) {
                for (int c = 0; c < 3; c++) {
                    const float f = (float)v.R[r][c];
                    std::memcpy(&b[3 * r + c], &f, 4);
                }
                const float f = (float)v.t[r];
                std::memcpy(&b[9 + r], &f, 4);
            }
            return b;
        };
        tf.push_back(float_bits(x));
        gm::CycleRun cyc{0, 0, 0};
        double lambda = -1.0;
        for (it = 0; it < max_iter;) {
            const int k = it;
            it++;
            double sys[gm::kTerms];
            gicp_linearize_spec(x, src_xyz, src_cov, ns, tgt_xyz, tgt_cov, nt, keys.empty() ? nullptr : keys.data(),
                                org, corr.data(), mah.data(), sys);
            double lam_used;
            int trials = 0, flags = 0;
            const int st = gicp_lm_iteration(sys, x, lambda, src_xyz, ns, tgt_xyz, corr.data(), mah.data(), rot_eps,
                                             trans_eps, &lam_used, &trials, &flags, solver);
            if (trace) {
                double* tr = trace + (size_t)16 * k;
                for (int r = 0; r < 3; r++) {
                    for (int c = 0; c < 3; c++) tr[3 * r + c] = x.R[r][c];
                    tr[9 + r] = x.t[r];
                }
                tr[12] = lam_used; tr[13] = trials; tr[14] = flags; tr[15] = st;
            }
            if (st != gm::kLmAccepted) break;
            if (it >= max_iter) break;
            // the cycle exit after iteration it's accepted step: T_f(it + 1) against the last kCycleLags
            const int cur = it + 1;
            tf.push_back(float_bits(x));
            int p = 0;
            for (int q = 1; q <= gm::kCycleLags && cur - q >= 1; q++)
                if (tf[cur - 1] == tf[cur - 1 - q]) { p = q; break; }
            const bool inert = trials == 1 && flags == 3;
            if (gm::cycle_update(cyc, p, inert, cycle_window)) {
                const auto& m = tf[gm::cycle_member(cur, p, max_iter) - 1];
                for (int r = 0; r < 3; r++) {
                    for (int c = 0; c < 3; c++) {
                        float f;
                        std::memcpy(&f, &m[3 * r + c], 4);
                        x.R[r][c] = f;
                    }
                    float f;
                    std::memcpy(&f, &m[9 + r], 4);
                    x.t[r] = f;
                }
                reported = max_iter;
                break;
            }
        }
    }
    for (int r = 0; r < 3; r++) {
        for (int c = 0; c < 3; c++) out_T[4 * r + c] = x.R[r][c];
        out_T[4 * r + 3] = x.t[r];
    }
    out_T[12] = 0.0; out_T[13] = 0.0; out_T[14] = 0.0; out_T[15] = 1.0;
    if (executed) *executed = it;
    return reported ? reported : it;
}

int orc_gicp(const float* src_xyz, const double* src_cov, int ns, const float* tgt_xyz, const double* tgt_cov, int nt,
             int max_iter, double rot_eps, double trans_eps, int cycle_window, double* out_T) {
    return orc_gicp_trace(src_xyz, src_cov, ns, tgt_xyz, tgt_cov, nt, max_iter, rot_eps, trans_eps, cycle_window, out_T,
                          nullptr, nullptr, 0);
}

// The linearisation at T (double 4x4 row-major) two ways, on the spec's correspondences (out_corr, ns):
// textbook = 0: the spec's (pcore_gicp_math.h contrib, the GPU's reduction order); textbook = 1: the independent
// long-double 4x4 restatement summed in point order.  out_sys: 28 terms (upper H row-major, b, error).
void orc_gicp_linearize(const float* src_xyz, const double* src_cov, int ns, const float* tgt_xyz,
                        const double* tgt_cov, int nt, const double* T, int textbook, int32_t* out_corr,
                        double* out_sys) {
    OXform x;
    for (int r = 0; r < 3; r++) {
        for (int c = 0; c < 3; c++) x.R[r][c] = T[4 * r + c];
        x.t[r] = T[4 * r + 3];
    }
    std::vector<pcore::gicpm::NNTarget> keys;
    float org[3];
    gicp_keys(tgt_xyz, nt, keys, org);
    std::vector<double> mah((size_t)6 * (ns > 0 ? ns : 1));
    double sys[pcore::gicpm::kTerms];
    gicp_linearize_spec(x, src_xyz, src_cov, ns, tgt_xyz, tgt_cov, nt, keys.empty() ? nullptr : keys.data(), org,
                        out_corr, mah.data(), sys);
    if (!textbook) {
        for (int v = 0; v < pcore::gicpm::kTerms; v++) out_sys[v] = sys[v];
        return;
    }
    ld TT[4][4];
    for (int r = 0; r < 4; r++)
        for (int c = 0; c < 4; c++) TT[r][c] = (ld)T[4 * r + c];
    ld H[6][6] = {}, b[6] = {}, err = 0.0L;
    for (int i = 0; i < ns; i++) {
        const int j = out_corr[i];
        if (j < 0) continue;
        textbook_point(TT, src_xyz + (size_t)3 * i, src_cov + (size_t)6 * i, tgt_xyz + (size_t)3 * j,
                       tgt_cov + (size_t)6 * j, H, b, err);
    }
    int h = 0;
    for (int a = 0; a < 6; a++)
        for (int c = a; c < 6; c++) out_sys[h++] = (double)H[a][c];
    for (int a = 0; a < 6; a++) out_sys[21 + a] = (double)b[a];
    out_sys[27] = (double)err;
}

// The step's pieces, for the CPU tests of the spec: se3_exp -> 4x4 row-major; the damped solve of a 28-term system
// (lm_solve_schur); the double sin / cos.
void orc_gicp_se3_exp(const double* a6, double* out_T) {
    const double a[6] = {a6[0], a6[1], a6[2], a6[3], a6[4], a6[5]};
    double Rd[3][3], td[3];
    pcore::gicpm::se3_exp(a, Rd, td, pcore::gicpm::kSe3Coef);
    for (int r = 0; r < 3; r++) {
        for (int c = 0; c < 3; c++) out_T[4 * r + c] = Rd[r][c];
        out_T[4 * r + 3] = td[r];
    }
    out_T[12] = 0.0; out_T[13] = 0.0; out_T[14] = 0.0; out_T[15] = 1.0;
}

void orc_gicp_lm_solve_ldlt(const double* sys, double lambda, double* out_d) {
    double d[6];
    ldlt_solve_ref(sys, lambda, d);
    for (int a = 0; a < 6; a++) out_d[a] = d[a];
}

void orc_gicp_lm_solve(const double* sys, double lambda, double* out_d) {
    double d[6];
    pcore::gicpm::lm_solve_schur(sys, lambda, d);
    for (int a = 0; a < 6; a++) out_d[a] = d[a];
}

double orc_sin_d(double x) { return pcore::dmath::sin_d(x); }
double orc_cos_d(double x) { return pcore::dmath::cos_d(x); }
double orc_cube_rn(double u) { return pcore::gicpm::cube_rn(u); }
double orc_lm_gain(double rho) { return pcore::gicpm::lm_gain(rho); }

// The spec's correspondence of float queries (n x 3) in a target segment: key scan (segments <= kKeyScanMax) or
// plain float squared distance; out_j: -1 for none.
void orc_gicp_nn(const float* q, int n, const float* tgt_xyz, int nt, int32_t* out_j) {
    std::vector<pcore::gicpm::NNTarget> keys;
    float org[3];
    gicp_keys(tgt_xyz, nt, keys, org);
    for (int i = 0; i < n; i++) out_j[i] = gicp_nn(q + (size_t)3 * i, tgt_xyz, nt, keys.empty() ? nullptr : keys.data(), org);
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
                      int max_iter, double rot_eps, double trans_eps, int cycle_window, float* out_adj,
                      int32_t* out_iters, float* out_rc, float* out_oc, float* out_diff, int nthreads) {
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
                                       l1 - l0, max_iter, rot_eps, trans_eps, cycle_window, T);
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
