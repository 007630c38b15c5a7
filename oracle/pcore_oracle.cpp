// pcore_oracle.cpp -- CPU restatement of the reference hot path.  TEST INFRASTRUCTURE ONLY.
// See pcore_oracle.h for the parity status ("parity unpinned" vs the reference binary).
// Build: oracle/Makefile (g++ -O2 -ffp-contract=off -fno-fast-math -fopenmp).
#include "pcore_oracle.h"

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
                           int32_t pose_label, float occlusion_threshold) {
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
                     int32_t pose_label, float occlusion_threshold, int32_t* depth) {
    const size_t npx = (size_t)width * height;
    for (size_t i = 0; i < npx; i++) depth[i] = INT_MAX;
    for (int t = lo; t < hi; t++) {
        const float* tp = tris + (size_t)9 * t;
        F3 v[3] = {{tp[0], tp[1], tp[2]}, {tp[3], tp[4], tp[5]}, {tp[6], tp[7], tp[8]}};
        // image_renderer.cuh:296-305: model transform, keep camera z, projection transform
        F3 local[3], projd[3];
        for (int k = 0; k < 3; k++) local[k] = mat_mul_v(pose, v[k]);
        F3 last_row = {local[0].z, local[1].z, local[2].z};
        for (int k = 0; k < 3; k++) projd[k] = mat_mul_v(proj, local[k]);
        rasterize_with_source(projd, last_row, depth, width, height, src_depth, src_mask, use_seg, pose_label,
                              occlusion_threshold);
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
