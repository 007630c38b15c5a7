/*
 * pcore_oracle.h -- CPU restatement of the reference render-and-compare hot path.
 *
 * TEST INFRASTRUCTURE ONLY.  Nothing in perception_amd/ links, loads or calls this
 * library: only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg use it,
 * and only as the checker / the reported CPU baseline.
 *
 * Parity status (see DESIGN.md "Oracle"):
 *   - The reference's own path (CUDA + Thrust + Eigen + assimp + OpenCV + fast_gicp) cannot be
 *     built in this image (no nvcc, no Eigen/OpenCV/assimp headers, fast_gicp not vendored), and
 *     the reference holds no golden vectors for this path.  The raster,
 *     unprojection, cost and selection restatements are therefore pinned only by analytic
 *     known-answer tests: "parity unpinned" against the reference binary.
 *   - KNN tie-break and GICP arithmetic live in the un-vendored fast_gicp fork: build-owned spec,
 *     parity unpinned.
 *
 * Float semantics: compiled with -ffp-contract=off -fno-fast-math, IEEE f32 (SSE) division, no FMA.
 * The GPU kernels follow the same explicit operation order; the reference's NVIDIA conversions
 * (cvt.rzi.s32.f32 / cvt.rzi.u64.f32: NaN -> 0, saturating) are spelled out as helpers.
 */
#pragma once
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* renderer.cu:1386-1410 compute_proj (near/far defaults renderer.h:87). out: mat4x4 a0..d3 row-major. */
void orc_compute_proj(float fx, float fy, float cx, float cy, int width, int height,
                      float near_plane, float far_plane, float out[16]);

/* image_renderer.cuh:212-321 render_triangle_multi + 59-210 rasterization_with_source + 465-472
 * max2zero, executed serially (triangle order) per pose.  tris: T x 9 floats (v0,v1,v2 xyz).
 * tris_model_count: triangles per model (image_renderer.cuh:371-380 scans).  pose_label NULL = 3-DoF
 * (no segmentation label, image_renderer.cuh:426-432).  src_mask used only when pose_label != NULL.
 * out: N x H x W int32 (cm). */
void orc_render_depth(const float* tris, int num_tris, const int32_t* tris_model_count, int num_models,
                      const float* poses, const int32_t* pose_model, const int32_t* pose_label, int num_poses,
                      int width, int height, const float* proj,
                      const int32_t* src_depth, const uint8_t* src_mask, float occlusion_threshold,
                      int32_t* out, int nthreads);

/* orc_render_depth plus the colour planes the serial z-test writes (image_renderer.cuh:146-196: a strictly nearer
 * fragment writes its triangle's colour, the black-out writes 0): out_col = per pose 3 planes (red, green, blue) of
 * H x W uint8, pose-major.  tri_rgb: T x 3 (nullable: grey 128). */
void orc_render_depth_color(const float* tris, int num_tris, const uint8_t* tri_rgb, const int32_t* tris_model_count,
                            int num_models, const float* poses, const int32_t* pose_model, const int32_t* pose_label,
                            int num_poses, int width, int height, const float* proj, const int32_t* src_depth,
                            const uint8_t* src_mask, float occlusion_threshold, int32_t* out, uint8_t* out_col,
                            int nthreads);

/* compute_point_clouds.cuh:37-184 + 265-346: stride mask, exclusive scan (pose-major, row, col),
 * unprojection.  label_mask (H x W, only valid for num_poses == 1) -> observed cloud, label = mask-1;
 * else pose_label (nullable) -> rendered cloud label.  Writes at most `cap` points; returns the
 * total count.  xyz: AoS cap x 3. */
int orc_depth_to_cloud(const int32_t* depth, int num_poses, int width, int height, int stride,
                       float cx, float cy, float fx, float fy, float depth_factor,
                       const uint8_t* label_mask, const int32_t* pose_label,
                       float* out_xyz, int32_t* out_pose, int32_t* out_label, int cap);
/* depth2cloud_global with camera_transform + observed_cloud_bounds (3-DoF): camera-frame points of the
 * pixels whose world point lies inside bounds; colours copied from rgb (H x W x 3, nullable). */
int orc_depth_to_cloud_bounded(const int32_t* depth, int width, int height, int stride, float cx, float cy, float fx,
                               float fy, float depth_factor, const float* cam_to_world, const double* bounds,
                               const uint8_t* rgb, float* out_xyz, uint8_t* out_rgb, int cap);

/* fast_gicp::brute_force_knn_search(k=1) as called at renderer.cu:1852-1871 (label-restricted
 * via observed_label_indices).  Build-owned spec: squared distance ((dx*dx + dy*dy) + dz*dz),
 * dx = r - o; minimum, ties -> lowest observed index; empty range -> (+inf, -1).
 * label_start/label_end == NULL: search the whole observed cloud (3-DoF). */
void orc_knn1(const float* r_xyz, const int32_t* r_label, int num_r,
              const float* o_xyz, int num_o, const int32_t* label_start, const int32_t* label_end,
              int num_labels, float* out_d2, int32_t* out_idx);

/* compute_costs.cuh:293-457 for cost_type 0 / 2 (depth only).  sensor_resolution is squared here,
 * as renderer.cu:1877 does before calling compute_costs. */
void orc_costs(int num_poses, int cost_type, int calc_obs, float sensor_resolution,
               const float* d2, const int32_t* idx, const int32_t* r_pose, int num_r, int num_o,
               const float* pose_obs_total, float* out_rc, float* out_oc, float* out_diff);

/* search_env.cpp:1987-2051 (int cost) + 2542-2583 (per-model argmin, strict '<', |t-s| < 30).
 * Host int conversions follow x86 cvttss2si (NaN / out of range -> INT_MIN).
 * out_best_cost[m] = INT_MAX and out_best_index[m] = -1 when no pose qualifies. */
void orc_select(int num_poses, const float* rc, const float* oc, const int32_t* pose_model,
                int num_models, int64_t index_base, int32_t* out_best_cost, int64_t* out_best_index);

/* Fused per-pose CPU pipeline (render full frame -> stride cloud -> 1-NN -> costs), OpenMP over
 * poses.  Used as the timed CPU baseline and as the large-N checker.  o_xyz is label-sorted AoS. */
void orc_evaluate(const float* tris, int num_tris, const int32_t* tris_model_count, int num_models,
                  const float* poses, const int32_t* pose_model, const int32_t* pose_label, int num_poses,
                  int width, int height, const float* proj,
                  const int32_t* src_depth, const uint8_t* src_mask, float occlusion_threshold,
                  int stride, float cx, float cy, float fx, float fy, float depth_factor,
                  const float* o_xyz, int num_o, const int32_t* label_start, const int32_t* label_end,
                  int num_labels, const float* pose_obs_total, int cost_type, int calc_obs,
                  float sensor_resolution, float* out_rc, float* out_oc, float* out_diff, int nthreads);



/* ---- GICP (a9/a10): build-owned spec, parity unpinned vs fast_gicp (un-vendored fork) --------------
 * fast_gicp's published FastGICP + LsqRegistration algorithm at the settings of renderer.cu:1693-1720, with a
 * deterministic arithmetic order that the GPU kernels follow exactly (DESIGN.md "GICP spec"; the arithmetic is
 * pcore_gicp_math.h, shared with the kernels, and held to the independent textbook restatement below):
 *  - covariance: k nearest points of the same cloud (float squared distance, ties -> lower index,
 *    list ordered by (distance, index)), double mean / covariance over k_eff = min(k, n), PLANE
 *    regularisation C = U diag(1, 1, 1e-3) U^T from at most 6 cyclic Jacobi sweeps with a 2-eps rotation threshold (double, sqrt/div only);
 *  - per iteration: correspondence of the float query float(T) s = the first strict minimum over the target
 *    segment of the three-FMA key (|q'-t'|^2 - |q'|^2 about the segment's origin; segments of <= 2048 targets) or
 *    of the float squared distance (larger segments); Mahalanobis (C_t + R C_s R^T)^-1, J = [skew(q) | -I];
 *    H, b and the error e^T M e reduced in the GPU's fixed order (64 per-lane sequential partials, then the wave
 *    shuffle-down tree);
 *  - Levenberg-Marquardt (LsqRegistration::step_lm): lambda0 = 1e-9 max|diag H|, <= 10 trials of the damped solve
 *    of H + lambda I (3x3 block elimination of the translation block, lm_solve_schur; fast_gicp uses Eigen's LDLT),
 *    se3_exp (exact so3_exp + V rho), errors of the trials with the iteration's
 *    correspondences, accept / reject by rho, lambda update; stop on a converged step
 *    (max(|dR - I| / rot_eps, |dt| / trans_eps) < 1), ten rejections or max_iter iterations.
 * Covariances: double[6] (xx, xy, xz, yy, yz, zz) per point. */
void orc_covariances(const float* xyz, int n, int k, double* out_cov6);

/* Returns iterations (linearisations; max_iter after a cycle exit); out_T: double 4x4 row-major (source -> target,
 * metres).  cycle_window: the cycle exit's W (pcore_gicp_math.h cycle_update; 0 runs the iterations out). */
int orc_gicp(const float* src_xyz, const double* src_cov, int ns, const float* tgt_xyz, const double* tgt_cov,
             int nt, int max_iter, double rot_eps, double trans_eps, int cycle_window, double* out_T);

/* orc_gicp with a per-iteration trace (nullable; max_iter x 16 doubles: R (9) and t (3) after the iteration, the
 * lambda of its first trial, its trials, flags (1 lambda inert, 2 rho >= 1/2), the LM status 0 accepted /
 * 1 converged / 2 failed); *executed (nullable): the iterations run (rows of the trace); solver 0 the spec's block
 * elimination, 1 Eigen's LDLT (orc_gicp_lm_solve_ldlt, a test reference). */
int orc_gicp_trace(const float* src_xyz, const double* src_cov, int ns, const float* tgt_xyz, const double* tgt_cov,
                   int nt, int max_iter, double rot_eps, double trans_eps, int cycle_window, double* out_T,
                   double* trace, int* executed, int solver);

/* The linearisation at T (4x4 row-major double) on the spec's correspondences (out_corr: ns, -1 = none):
 * textbook = 0 the spec's arithmetic and reduction order, textbook = 1 an independent long-double restatement of
 * fast_gicp's 4x4 homogeneous form (RCR = C_B + T C_A T^T, RCR(3,3) = 1, M = RCR^-1 by Gauss-Jordan, M(3,3) = 0,
 * dense J^T M J / J^T M e / e^T M e).  out_sys: 28 doubles (upper H row-major, b, error). */
void orc_gicp_linearize(const float* src_xyz, const double* src_cov, int ns, const float* tgt_xyz,
                        const double* tgt_cov, int nt, const double* T, int textbook, int32_t* out_corr,
                        double* out_sys);
/* Pieces of the step for the CPU spec tests: se3_exp(a6) -> 4x4; d = (H + lambda I)^-1 (-b) of a 28-term system
 * (lm_solve_schur); the double sin / cos of pcore_dmath.h; the spec's correspondences of n float queries. */
void orc_gicp_se3_exp(const double* a6, double* out_T);
void orc_gicp_lm_solve(const double* sys, double lambda, double* out_d);
/* Test reference: the damped solve by Eigen's pivoted LDLT (what fast_gicp uses; orc_gicp_trace solver = 1). */
void orc_gicp_lm_solve_ldlt(const double* sys, double lambda, double* out_d);
double orc_sin_d(double x);
double orc_cos_d(double x);
double orc_cube_rn(double u);   // step_lm's std::pow(u, 3), rounded once
double orc_lm_gain(double rho); // max(1/3, 1 - (2 rho - 1)^3)
void orc_gicp_nn(const float* q, int n, const float* tgt_xyz, int nt, int32_t* out_j);

/* concatenate_transforms (renderer.cu:1412-1429): pose' = init_from_eigen((float(T) * to_eigen(pose,100)), 100). */
void orc_concat_pose(const double* T, const float* pose, float* out_pose);

/* do_icp = true flow of render_cuda_multi_unified (renderer.cu:1688-1817) per pose: render, stride cloud,
 * covariances, GICP against the pose's label segment (tgt_cov = label-sorted target covariances),
 * concatenate, re-render, re-score.  out_adj: N x 16 adjusted poses; out_iters: N (nullable). */
void orc_evaluate_icp(const float* tris, int num_tris, const int32_t* tris_model_count, int num_models,
                      const float* poses, const int32_t* pose_model, const int32_t* pose_label, int num_poses,
                      int width, int height, const float* proj,
                      const int32_t* src_depth, const uint8_t* src_mask, float occlusion_threshold,
                      int stride, float cx, float cy, float fx, float fy, float depth_factor,
                      const float* o_xyz, const double* o_cov, int num_o, const int32_t* label_start,
                      const int32_t* label_end, int num_labels, const float* pose_obs_total, int cost_type,
                      int calc_obs, float sensor_resolution, int k_corr, int max_iter, double rot_eps,
                      double trans_eps, int cycle_window, float* out_adj, int32_t* out_iters, float* out_rc,
                      float* out_oc, float* out_diff, int nthreads);

/* Colour cost (cost_type 1, f4): rgb2lab with the cost's channel order, the CIEDE2000 distance of the
 * shared colour spec, its float transcendentals, and the 3-DoF RGB-D evaluation (serial raster keeping
 * the first triangle that reaches each pixel's minimum depth). */
void orc_rgb2lab(const uint8_t c[3], float lab[3]);
double orc_colour_distance(const float* lab1, const float* lab2);
float orc_sin_f(float x);
float orc_cos_f(float x);
float orc_exp_f(float x);
float orc_atan2_f(float y, float x);
void orc_evaluate_colour(const float* tris, int num_tris, const uint8_t* tri_rgb, const int32_t* tris_model_count,
                         int num_models, const float* poses, const int32_t* pose_model, int num_poses, int width,
                         int height, const float* proj, const int32_t* src_depth, float occlusion_threshold,
                         int stride, float cx, float cy, float fx, float fy, float depth_factor, const float* o_xyz,
                         const uint8_t* o_rgb, int num_o, const float* pose_obs_total, int calc_obs,
                         float sensor_resolution, float colour_thr, float* out_rc, float* out_oc, float* out_diff,
                         int nthreads);

/* ---- a14: the reference's CPU/OMP path (ref_cpu_path.cpp) -------------------------------------------
 * render_cpu (renderer.cpp:228-330: full frame, no source occlusion) -> depth2cloud_cpu at stride 1
 * (icp.cpp:64-108) -> ICP_Point2Plane_cpu against Scene_projective of the observed depth (icp.cpp:116-179,
 * depth_scene.h:25-48, get_normal common.cpp:17-107), host float semantics (x86 conversions).
 * out_T: the ICP transform (metres, row-major 4x4) per pose. */
void orc_ref_render_cpu(const float* tris, int num_tris, const float* poses, int num_poses, int width, int height,
                        const float* proj, int32_t* out, int nthreads);
int orc_ref_depth2cloud(const int32_t* depth, int width, int height, float fx, float fy, float cx, float cy,
                        float* out_xyz, int cap);
void orc_ref_scene(const int32_t* depth, int width, int height, float fx, float fy, float cx, float cy,
                   float* out_pcd, float* out_normal);
int orc_ref_icp(float* model_xyz, int n, const float* scene_pcd, const float* scene_normal, int width, int height,
                float fx, float fy, float cx, float cy, float max_dist_diff, float rel_fitness, float rel_rmse,
                int max_iter, float* out_T, float* out_fitness, float* out_rmse);
void orc_ref_solver666(const float* A, const float* b, float* out_T);
void orc_ref_cpu_pipeline(const float* tris, int num_tris, const float* poses, int num_poses, int width, int height,
                          const float* proj, float fx, float fy, float cx, float cy, const int32_t* scene_depth,
                          float max_dist_diff, float rel_fitness, float rel_rmse, int max_iter, float* out_T,
                          float* out_fitness, float* out_rmse, int32_t* out_iters, int32_t* out_points,
                          int nthreads);

#ifdef __cplusplus
}
#endif
