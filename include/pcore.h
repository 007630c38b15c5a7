/*
 * pcore.h -- C ABI of the MI355X render-and-compare pose-search core (libpcore.so).
 *
 * Drop-in boundary for the reference's GPU seam
 *   cuda_renderer::render_cuda_multi_unified(...)   (cuda_renderer/include/cuda_renderer/renderer.h:221-268,
 *                                                     cuda_renderer/src/cuda/renderer.cu:1431-1934)
 *   cuda_renderer::depth2cloud_global(...)          (renderer.h:131-153, renderer.cu:1936-2069)
 * and for the host selection it feeds
 *   EnvObjectRecognition::ComputeGreedyCostsInParallelGPU / ComputeGreedyRenderPoses
 *                                                    (sbpl_perception/src/search_env.cpp:1987-2051, 2542-2636).
 *
 * Conventions (differences from the reference are deliberate and listed in INTEGRATION.md):
 *   - Plain C types only.  Large per-batch arrays are DEVICE pointers (e.g. tensor.data_ptr() of a
 *     PyTorch-ROCm tensor); mesh and camera setup take HOST pointers (copied once).
 *   - Every call is asynchronous on the caller's stream (`stream` may be NULL = default stream); the
 *     caller synchronises.  One context per (host thread, device); calls on a context are not re-entrant,
 *     and its calls must all go to one stream (the context's device scratch -- GICP slots, the fused
 *     kernel's overflow list and window histogram -- is reused by the next call in stream order).
 *   - Caller-allocated outputs.  The context owns persistent device scratch and never frees caller memory.
 *   - Return value: PCORE_OK or an error code; pcore_last_error() describes the last failure.
 *     The reference's in-band "invalid pose" convention (rendered cost -1, compute_costs.cuh:28-31) is kept.
 *   - Poses are the reference's Model::mat4x4 (model.h:76-107): 16 floats a0..d3, row-major, rotation AND
 *     translation scaled by 100 (mat4x4::init_from_eigen(pose_in_cam, 100)), so vertices land in cm.
 */
#ifndef PCORE_H_
#define PCORE_H_

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define PCORE_ABI_VERSION 7

enum pcore_status {
    PCORE_OK = 0,
    PCORE_E_INVALID_ARG = 1, /* bad size / pointer / parameter */
    PCORE_E_HIP = 2,         /* a HIP runtime call failed */
    PCORE_E_OOM = 3,         /* device allocation failed */
    PCORE_E_STATE = 4        /* required setup call missing (meshes / camera / observation) */
};

/* Cost types of render_cuda_multi_unified (renderer.cu:1498): 0 = 3-DoF depth, 1 = 3-DoF RGB-D (a
 * matched point also needs CIEDE2000 <= color_distance_threshold, compute_costs.cuh:57-159, 222-240;
 * needs pcore_set_observation_colors), 2 = 6-DoF depth + labels. */
enum pcore_cost_type { PCORE_COST_DEPTH_3DOF = 0, PCORE_COST_RGBD_3DOF = 1, PCORE_COST_DEPTH_6DOF = 2 };

typedef struct pcore_ctx pcore_ctx;
typedef void* pcore_stream; /* hipStream_t */

/* Image geometry + intrinsics.  `proj` replaces the reference's proj_mat argument (renderer.h:225,
 * built by compute_proj, renderer.cu:1386-1410); fx/fy/cx/cy are kCameraFX.. (renderer.h:231-234). */
typedef struct pcore_camera {
    int32_t width, height;
    float fx, fy, cx, cy;
    float proj[16];
} pcore_camera;

/* Per-batch parameters of render_cuda_multi_unified that are not arrays (renderer.h:228-252). */
typedef struct pcore_eval_params {
    int32_t cost_type;           /* enum pcore_cost_type */
    int32_t calc_obs_cost;       /* calculate_observed_cost */
    int32_t stride;              /* gpu_stride; width % stride == 0 (compute_point_clouds.cuh:271) */
    float depth_factor;          /* rendered cm -> metres (the reference passes 100) */
    float sensor_resolution;     /* metres; squared internally like renderer.cu:1877 */
    float occlusion_threshold;   /* 3-DoF source-occlusion threshold in cm (gpu_occlusion_threshold) */
    float color_distance_threshold; /* cost_type 1: CIEDE2000 gate (renderer.h:247) */
} pcore_eval_params;

/* ---- lifetime ---------------------------------------------------------------------------------- */
int pcore_create(int device, pcore_ctx** out_ctx);
void pcore_destroy(pcore_ctx* ctx);
const char* pcore_last_error(const pcore_ctx* ctx);
int pcore_abi_version(void);

/* Generation of the context's device state.  A captured HIP graph of pcore_evaluate bakes in the kernel
 * arguments and the scratch pointers of the call it captured (sampled source, neighbour grids, overflow
 * list, colour scratch, tile size); the counter changes whenever any of them may have changed:
 * pcore_upload_meshes, pcore_set_camera, pcore_set_observation, pcore_set_observation_colors, a new
 * sampling stride, and every reallocation of per-batch scratch.  A replay is valid only while the
 * generation equals the one read right after the capture (no reference counterpart: the reference
 * re-uploads everything per call, renderer.cu:1532-1544).  0 for a NULL context.  A C caller that captures
 * pcore_evaluate into a graph compares pcore_generation before every replay, and orders its setup calls
 * after any replay still in flight on its stream (the check runs when the replay is enqueued). */
uint64_t pcore_generation(const pcore_ctx* ctx);

/* ---- static inputs ----------------------------------------------------------------------------- */
/* Triangles of all models concatenated + triangles per model: the `tris` and `tris_model_count`
 * arguments (renderer.h:223-226; filled by LoadObjFiles, search_env.cpp:253-307 / Model::LoadModel,
 * model.cpp:16-135).  tri_xyz: num_tris x 9 floats (v0,v1,v2) in metres, HOST.  tri_rgb: num_tris x 3
 * (vertex-0 colour, model.cpp:81-97), HOST, may be NULL (colour 128).  The context deduplicates
 * vertices and builds meshlets once here. */
int pcore_upload_meshes(pcore_ctx* ctx, const float* tri_xyz, const uint8_t* tri_rgb, int32_t num_tris,
                        const int32_t* tris_model_count, int32_t num_models);

int pcore_set_camera(pcore_ctx* ctx, const pcore_camera* cam);

/* ---- per-scene inputs -------------------------------------------------------------------------- */
/* depth2cloud_global (renderer.h:131-153; used by SetInput, search_env.cpp:5993-6017): unproject the
 * observed depth image (raw sensor units, e.g. YCB uint16 widened to int32) at `stride`, keeping pixels
 * with depth > 0 and (if label_mask != NULL) label > 0.  Writes xyz (cap x 3, metres) and label
 * (mask - 1) in the reference's compaction order; *out_count (HOST) receives the point count (the call
 * synchronises `stream` to return it).  Device pointers. */
int pcore_observed_cloud(pcore_ctx* ctx, const int32_t* d_depth, const uint8_t* d_label_mask, int32_t width,
                         int32_t height, int32_t stride, float depth_factor, float* d_out_xyz,
                         int32_t* d_out_label, int32_t cap, int32_t* out_count, pcore_stream stream);

/* depth2cloud_global for 3-DoF table-top scenes (renderer.cu:1936-2069 with camera_transform and
 * observed_cloud_bounds; compute_point_clouds.cuh:14-35, 79-91, 125-157): as pcore_observed_cloud
 * without a label mask, keeping only pixels whose point, moved to the world frame by `cam_to_world`
 * (HOST, 4 x 4 row-major float, R p + t evaluated left to right in float), lies inside `bounds` (HOST,
 * 6 doubles: x_max, x_min, y_max, y_min, z_max, z_min, compared as floats).  The output points stay in
 * the CAMERA frame, as in the reference.  cam_to_world and bounds are both given or both NULL.
 * d_rgb (nullable): H x W x 3 uint8 image; d_out_rgb (nullable, needs d_rgb) receives each kept
 * pixel's 3 bytes in the input's channel order. */
int pcore_observed_cloud_bounded(pcore_ctx* ctx, const int32_t* d_depth, const uint8_t* d_rgb, int32_t width,
                                 int32_t height, int32_t stride, float depth_factor, const float* cam_to_world,
                                 const double* bounds, float* d_out_xyz, uint8_t* d_out_rgb, int32_t cap,
                                 int32_t* out_count, pcore_stream stream);

/* Observation used by every evaluate call until replaced: the source depth in cm (H x W int32; the
 * reference's source_depth after search_env.cpp:2487-2498), the source mask label (H x W uint8, the
 * reference's source_mask_label; NULL for 3-DoF) and the observed cloud with its labels (the
 * observed_depth_eigen / result_observed_cloud_label pair, renderer.h:236-242).  The context sorts the
 * cloud by label (stable, renderer.cu:1674-1686) and builds its fixed-radius neighbour grids for
 * `sensor_resolution` metres.  Device pointers; the call synchronises `stream`. */
int pcore_set_observation(pcore_ctx* ctx, const int32_t* d_src_depth_cm, const uint8_t* d_src_mask,
                          const float* d_obs_xyz, const int32_t* d_obs_label, int32_t num_obs,
                          float sensor_resolution, pcore_stream stream);

/* Colours of the observed points for cost_type 1 (the observed_color argument, renderer.h:236-238):
 * n x 3 uint8 (DEVICE) in the order of the d_obs_xyz given to pcore_set_observation, channels as the
 * image (the reference's result_observed_cloud_color planes).  The context converts them to CIE Lab with
 * the reference's channel order (rgb2lab(c2, c1, c0), compute_costs.cuh:57-88, 214-220).  Valid until the
 * next pcore_set_observation.  Triangle colours come from pcore_upload_meshes (tri_rgb; 128 grey when
 * NULL, model.cpp:97-101). */
int pcore_set_observation_colors(pcore_ctx* ctx, const uint8_t* d_obs_rgb, int32_t num_obs, pcore_stream stream);

/* ---- per-batch hot path ------------------------------------------------------------------------ */
/* Stage "COST" of render_cuda_multi_unified with do_icp = false: render every pose, unproject at
 * stride, 1-NN against the same-label observed points, and the rendered / observed / points-diff
 * costs (compute_costs.cuh:293-457).  d_pose_label NULL selects 3-DoF (all observed points, occlusion
 * by threshold).  d_pose_obs_total: pose_observed_points_total (renderer.h:240).  Outputs N floats each
 * (d_out_oc / d_out_diff are written as 0 when calc_obs_cost == 0).  d_dbg_zs (nullable): the sampled
 * z-buffer after source occlusion, N x ceil(H/stride) x (W/stride) int32 (parity / debugging). */
int pcore_evaluate(pcore_ctx* ctx, const float* d_poses, const int32_t* d_pose_model,
                   const int32_t* d_pose_label, const float* d_pose_obs_total, int32_t num_poses,
                   const pcore_eval_params* params, float* d_out_rc, float* d_out_oc, float* d_out_diff,
                   int32_t* d_dbg_zs, pcore_stream stream);

/* GICP settings; the reference hard-codes the first four at renderer.cu:1696-1705.  cycle_exit_window (no
 * reference counterpart): a pose whose float transforms have recurred with the same period for
 * this many iterations, each step accepted at its first trial with an inert damping, stops and reports
 * max_iterations and the cycle member the remaining iterations end on; 0 runs every iteration out, as fast_gicp
 * does; the spec's value is 8 (PCORE_GICP_CYCLE_WINDOW). */
#define PCORE_GICP_CYCLE_WINDOW 8
typedef struct pcore_icp_params {
    int32_t k_correspondences;      /* covariance neighbours, 10 (<= 16) */
    int32_t max_iterations;         /* 150 */
    double rotation_epsilon;        /* 2e-3 */
    double transformation_epsilon;  /* 5e-4 */
    int32_t cycle_exit_window;      /* 8 (0 = off) */
} pcore_icp_params;

/* pcore_evaluate followed by pcore_select in one launch: every pose's argmin key (pcore_select's, global index
 * index_base + i) is folded into d_keys[model] (atomic MIN) by the workgroup that scores the pose, so the batch
 * needs no separate selection pass.  The costs are written as by pcore_evaluate (d_out_oc may not be null); the
 * keys equal pcore_evaluate + pcore_select's. */
int pcore_evaluate_select(pcore_ctx* ctx, const float* d_poses, const int32_t* d_pose_model,
                          const int32_t* d_pose_label, const float* d_pose_obs_total, int32_t num_poses,
                          const pcore_eval_params* params, float* d_out_rc, float* d_out_oc, float* d_out_diff,
                          int64_t index_base, int32_t num_models, int64_t* d_keys, pcore_stream stream);

/* Stage "COST" with do_icp = true (renderer.cu:1688-1817): render, unproject at stride, per-pose GICP of
 * the rendered cloud onto the pose's observed label segment (FastGICPCudaCore::optimize_multi), compose
 * T * pose (concatenate_transforms, renderer.cu:1412-1429), re-render and re-score.  d_out_poses: N x 16
 * adjusted mat4x4 (the reference's adjusted_poses); d_out_iters (nullable): GICP iterations per pose.
 * Costs as pcore_evaluate, for the adjusted poses.  Device pointers; needs per-context scratch that
 * grows on first use (64 B per pose and stride sample; a batch is split into equal chunks that fit a
 * budget of min(32 GiB, 40 % of the free device memory)). */
int pcore_evaluate_icp(pcore_ctx* ctx, const float* d_poses, const int32_t* d_pose_model,
                       const int32_t* d_pose_label, const float* d_pose_obs_total, int32_t num_poses,
                       const pcore_eval_params* params, const pcore_icp_params* icp, float* d_out_poses,
                       int32_t* d_out_iters, float* d_out_rc, float* d_out_oc, float* d_out_diff,
                       pcore_stream stream);

/* Stage "RENDER" / "DEBUG" images (renderer.cu:1594-1615): full-resolution int32 z-buffers (cm) with source
 * occlusion and INT_MAX -> 0 (image_render, image_renderer.cuh:336-496).  d_out_depth: N x H x W.
 * d_out_color (nullable): the reference's result_color -- three planes red, green, blue of N x H x W uint8 each,
 * concatenated -- holding each pixel's nearest triangle colour (the first triangle reaching the minimum depth,
 * as the serial z-test of image_renderer.cuh:146-159 keeps it; the tri_rgb of pcore_upload_meshes), black where
 * nothing is rendered or the source occludes the render (image_renderer.cuh:160-196). */
int pcore_render(pcore_ctx* ctx, const float* d_poses, const int32_t* d_pose_model, const int32_t* d_pose_label,
                 int32_t num_poses, float occlusion_threshold, int32_t* d_out_depth, uint8_t* d_out_color,
                 pcore_stream stream);

/* gpu_stats of render_cuda_multi_unified (model.h:24-27, filled at renderer.cu:1707 and 1739) for the last
 * pcore_evaluate_icp: icp_runtime = seconds of its GICP stage (source covariances + GICP launches, HIP events on
 * the call's stream -- this call waits for them); peak_memory_usage = the most device memory in use (MB,
 * hipMemGetInfo like print_cuda_memory_usage, cuda/utils.cuh:6-24) at a GICP stage since the last reset;
 * gicp_ms = the GICP launches alone; icp_chunks = chunks the batch ran in; gicp_iterations = the iterations the
 * poses report (d_out_iters summed), gicp_iterations_run = the iterations executed (fewer by the cycle exits),
 * gicp_cycle_exits = poses that left by the cycle exit.  reset != 0 restarts the peak. */
typedef struct pcore_gpu_stats {
    float icp_runtime;
    double peak_memory_usage;
    float gicp_ms;
    int32_t icp_chunks;
    int64_t gicp_iterations;
    int64_t gicp_iterations_run;
    int64_t gicp_cycle_exits;
} pcore_gpu_stats;
int pcore_get_stats(pcore_ctx* ctx, pcore_gpu_stats* out, int32_t reset);

/* LDS tile of the fused window launch (no reference counterpart: the reference renders whole frames; DESIGN.md
 * "Pose windows").  tier = the tier the next call starts from (wgs_per_cu[tier] workgroups per CU, a tile of
 * edge[tier] samples), tcap = the tile of the last launch; hist[b] = the poses of launch seq whose window held
 * more than edge[b-1] and at most edge[b] samples (hist[num_tiers]: more than edge[num_tiers-1]); chunked = its
 * poses scored in chunks of the tile.  seq numbers the context's launches from 1 (each launch publishes the counts
 * of the one before it); seq < 1: no counts yet.  Diagnostics only: the results never depend on the tile. */
#define PCORE_MAX_TILE_TIERS 8
typedef struct pcore_tile_info {
    int32_t num_tiers;
    int32_t tier;
    int32_t tcap;
    int32_t seq;
    int32_t edge[PCORE_MAX_TILE_TIERS];
    int32_t wgs_per_cu[PCORE_MAX_TILE_TIERS];
    int32_t hist[PCORE_MAX_TILE_TIERS + 1];
    int32_t chunked;
} pcore_tile_info;
int pcore_get_tile_info(pcore_ctx* ctx, pcore_tile_info* out);

/* Test hook (no reference counterpart): the GICP kernels' damped LM solve (H + lambda I) d = -b of n raw 28-term
 * systems (upper H row-major, b, error; d_sys n x 28, d_lambda n, d_out n x 6 doubles), one wave each, for the
 * parity test against the oracle's restatement of Eigen's pivoted LDLT. */
int pcore_debug_lm_solve(const double* d_sys, const double* d_lambda, double* d_out, int32_t n, pcore_stream stream);

/* Test hook (no reference counterpart): the GICP covariances of point segments by covariance_kernel (fast_gicp's
 * k-nearest-neighbour covariance with PLANE regularisation): d_xyzw = points as x, y, z, w floats;
 * segment s is points d_seg_off[s] .. + d_seg_cnt[s] (its own neighbour set); d_out_cov6 gets 6 doubles per point
 * (upper triangle, row-major).  1 <= k <= 16. */
int pcore_debug_covariances(const float* d_xyzw, const int32_t* d_seg_off, const int32_t* d_seg_cnt, int32_t num_segs,
                            int32_t k, double* d_out_cov6, pcore_stream stream);
/* Test hook (no reference counterpart): the k = 10 covariances of rendered-cloud slots (segment i: d_xyzw + 4 i
 * seg_stride, d_seg_cnt[i] points) by the threshold k-NN over each cloud's stride-s sample grid (camera fx, fy, cx, cy;
 * pcore_cov.h), falling back to the brute force where the grid does not allow it: bit-identical to
 * pcore_debug_covariances for any points. */
int pcore_debug_covariances_cloud(const float* d_xyzw, const int32_t* d_seg_cnt, int32_t seg_stride, int32_t num_segs,
                                  float fx, float fy, float cx, float cy, int32_t stride, double* d_out_cov6,
                                  pcore_stream stream);
/* Test hook (no reference counterpart): the last pcore_evaluate_icp call's GICP help board counters (DESIGN.md
 * section 4, the queue-dry tail): out4 = rounds of 64 correspondences searched by helper waves, owner timeouts
 * (rounds a late helper left to the owner), helper give-ups, poses registered for help.  Waits for the call's last
 * GICP launch. */
int pcore_debug_gicp_help_stats(pcore_ctx* c, int64_t* out4);

/* GenerateSuccessorStates / GetStateImagesUnifiedGPU host work on the device (search_env.cpp:7056-7254,
 * 1535-1576), for the drop-in recognizer's states:
 *
 * pcore_count_within: IsValidPose's neighbour count (search_env.cpp:359-396, pcl::search::KdTree radiusSearch):
 * for every query i, the points of observed label segment d_labels[i] (as set by pcore_set_observation; a label
 * outside the segments counts 0) strictly within the radius -- float query and points, d_radius_sq[i] = float(r *
 * r), ((0 + dx^2) + dy^2) + dz^2 < r^2 in float.  d_queries: n x 3 float; d_out_counts: n int32.
 *
 * pcore_state_poses: the states' poses for the GPU search: for state i (x y z qx qy qz qw, double), cam_from_world
 * (HOST, 16 doubles row-major: inv(camera_pose * cam_to_body)) * ContPose::GetTransform (normalised quaternion,
 * object_state.cpp:83-97) * d_preprocess[d_model[i]] (16 doubles row-major per model, PreprocessModel), every
 * product summed in index order in double, then mat4x4::init_from_eigen(., 100) (model.h:89-107) into
 * d_out_poses (n x 16 float).  Model ids must lie in [0, num_models). */
int pcore_count_within(pcore_ctx* ctx, const float* d_queries, const int32_t* d_labels, const float* d_radius_sq,
                       int32_t n, int32_t* d_out_counts, pcore_stream stream);
int pcore_state_poses(pcore_ctx* ctx, const double* d_states, const int32_t* d_model, const double* cam_from_world,
                      const double* d_preprocess, int32_t num_models, int32_t n, float* d_out_poses,
                      pcore_stream stream);

/* Stage "CLOUD": compute_point_clouds (compute_point_clouds.cuh:188-367) over N z-buffers: stride mask,
 * pose-major / row / column compaction, unprojection.  xyz AoS (cap x 3).  d_label_mask (H x W) only
 * for num_poses == 1; d_pose_label gives the rendered-cloud label.  *out_count (HOST) = total points
 * (the call synchronises `stream`). */
int pcore_depth_to_cloud(pcore_ctx* ctx, const int32_t* d_depth, int32_t num_poses, int32_t width, int32_t height,
                         int32_t stride, float depth_factor, const uint8_t* d_label_mask,
                         const int32_t* d_pose_label, float* d_out_xyz, int32_t* d_out_pose, int32_t* d_out_label,
                         int32_t cap, int32_t* out_count, pcore_stream stream);

/* Stage "CLOUD" with the reference's two debug outputs as well (renderer.cu:1821-1847): d_color_planes = the
 * rendered colour planes (red, green, blue planes of N x H x W uint8 each -- pcore_render's d_out_color) and
 * d_out_color = each point's colour from them as three planes of `cap` bytes (depth_to_2d_cloud,
 * compute_point_clouds.cuh:163-165; the reference's plane stride is its point count, the same when cap equals it);
 * d_out_dc_index = result_dc_index (N x H x W int32): for every pixel the number of cloud points before it in pose /
 * row / column order, the reference's exclusive scan of the stride mask (compute_point_clouds.cuh:267-292).  Both
 * outputs are nullable; the rest is pcore_depth_to_cloud's. */
int pcore_depth_to_cloud_ex(pcore_ctx* ctx, const int32_t* d_depth, int32_t num_poses, int32_t width, int32_t height,
                            int32_t stride, float depth_factor, const uint8_t* d_label_mask, const int32_t* d_pose_label,
                            const uint8_t* d_color_planes, float* d_out_xyz, int32_t* d_out_pose, int32_t* d_out_label,
                            uint8_t* d_out_color, int32_t* d_out_dc_index, int32_t cap, int32_t* out_count,
                            pcore_stream stream);

/* Host selection of the reference moved on device: cost = (int)(rc + oc) (x86 conversion semantics),
 * skip invalid (-1/-2), keep |(int)rc - (int)oc| < 30, per-model minimum with strict '<' (lowest global
 * index wins ties) -- search_env.cpp:2022-2048, 2554-2566.  Result is folded into d_keys[num_models]
 * (int64, atomic min) as key = ((uint32)(cost ^ 0x80000000) << 31) | (index_base + i); initialise
 * d_keys to PCORE_KEY_NONE.  Keys from several batches / ranks combine with a MIN reduction
 * (RCCL all-reduce). */
#define PCORE_KEY_NONE ((int64_t)0x7fffffffffffffffLL)
int pcore_select(pcore_ctx* ctx, const float* d_rc, const float* d_oc, const int32_t* d_pose_model,
                 int32_t num_poses, int64_t index_base, int32_t num_models, int64_t* d_keys, pcore_stream stream);

/* ADD / ADD-S of estimated against ground-truth poses over one model's points -- the YCB harness
 * metric: compare_clouds (sbpl_perception/src/scripts/tools/fat_dataset/
 * fat_pose_image.py:2020-2139) and pose_error.add / adi (fat_dataset/lib/utils/pose_error.py:72-108).
 *   d_pts      n x 3 float model points (model frame, metres), device
 *   d_T_gt,    num_pairs x 16 double, row-major 4x4 object-to-camera transforms, device
 *   d_T_est
 *   d_add      num_pairs doubles: mean_i |T_gt p_i - T_est p_i|           (nullable)
 *   d_adds     num_pairs doubles: mean_i min_j |T_gt p_i - T_est p_j|     (nullable)
 * f64 arithmetic; the minimum is exact (no kd-tree approximation).  Needs only a context (no meshes /
 * camera / observation). */
int pcore_pose_distances(pcore_ctx* ctx, const float* d_pts, int32_t n, const double* d_T_gt, const double* d_T_est,
                         int32_t num_pairs, double* d_add, double* d_adds, pcore_stream stream);

#ifdef __cplusplus
}
#endif
#endif /* PCORE_H_ */
