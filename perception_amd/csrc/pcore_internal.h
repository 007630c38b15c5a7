// pcore_internal.h -- data layouts shared by the host API (pcore_api.hip) and the kernels
// (pcore_kernels.hip).  Not part of the ABI.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "pcore_gicp_math.h"

namespace pcore {

// Vertex-ring streams ("Vertex-ring streams").  A model's triangles are cut into streams, one
// per wave of the fused workgroup.  A stream is a sequence of steps; a step is an optional vertex pass (<= 64
// new vertices, transformed by one lane each into the wave's LDS vertex ring) followed by one batch of <= 64
// triangles (one lane each).  The ring holds the last kVRing passes: pass p of a stream lives in ring buffer
// p mod kVRing, and a triangle names its three vertices by ring slot (buffer * 64 + lane), 9 bits each.  The
// builder guarantees that a batch issued after pass h references only passes h - 1 and h (kRefPasses = 2),
// so a vertex is transformed once for every ~2 triangles (the 64-vertex meshlets of round 1 transformed one
// per ~1.1), and a queued triangle record needs only its three slot numbers: before pass P overwrites the
// buffer of pass P - kVRing, the kernel flushes the records that may still reference it.
//   sverts: 64 float4 slots per vertex pass (x, y, z, w), stream-major; w = 1 for a vertex, 0 for padding
//   stris:  64 uint32 slots per step, i0 | i1 << 9 | i2 << 18 (ring slots) | vpass << 30 (the step begins with a
//           vertex pass; the same in all 64 slots, read with readfirstlane); padding slots have bit 31 set
//   streams: int4 (first step, end step, first vertex pass, end vertex pass) per stream
// All loads of a step are unconditional (the next step's triangle slots and the next unconsumed vertex pass
// are prefetched while the current step runs), so the compiler counts them in vmcnt.
constexpr int kStepSlots = 64;
// Per-vertex sample-window bounds (packed int16, computed once per vertex in the vertex pass; pcore_kernels.hip,
// vertex_bounds).  A batch reads the bounds of the last kRefPasses passes only, so they live in two ring buffers of
// their own: pass p in buffer p mod 2, which equals (p mod kVRing) mod 2 because kVRing is even.
#ifndef PCORE_VRING
#define PCORE_VRING 4
#endif
constexpr int kVRing = PCORE_VRING;    // vertex passes resident per wave
constexpr int kRefPasses = 2;          // a batch references the last kRefPasses passes
constexpr int kRingSlotBits = 9;       // kVRing * 64 <= 512
static_assert(PCORE_VRING % 2 == 0, "per-vertex bounds index their two buffers by ring slot parity");
constexpr int kStreamChunks = 1;       // chunks per stream (pcore_streams.h, build_model)
#ifndef PCORE_FUSED_WAVES
#define PCORE_FUSED_WAVES 4
#endif
constexpr int kFusedWaves = PCORE_FUSED_WAVES;  // waves per fused / cloud workgroup = streams per model

// Fixed-radius neighbour grid over the observed points of one label (6-DoF) or of the whole cloud
// (3-DoF).  Cells are >= 2 * sensor_resolution wide, so every point within the radius of a query lies
// in the <= 2 x 2 x 2 cells its radius box touches.  Points are stored cell-sorted as float4
// (x, y, z, bitcast(label-local index)).
struct LabelGrid {
    float ox, oy, oz, inv_c;
    int32_t nx, ny, nz;
    int32_t cell_base;  // offset of this grid's CSR row pointer in cell_start (nx*ny*nz + 1 entries)
    int32_t pt_count;   // points of this label (bitmap size)
    float cell;         // cell edge (inv_c = 1 / cell, rounded)
    int32_t pad1, pad2;
};

// tile tiers of the fused window launch: workgroups per CU PCORE_TIER_MAX, ..., 3, 2 (the LDS tile that
// leaves room for that many workgroups); the host picks the tier from the previous call's window histogram
#ifndef PCORE_DEBUG_SKIP_RT
#define PCORE_DEBUG_SKIP_RT 0  // 1: the fused kernels honour PCORE_DEBUG_SKIP (ablation builds, tools/ablate_sq.sh)
#endif
#ifndef PCORE_TIER_MAX
#define PCORE_TIER_MAX 6
#endif
constexpr int kTileTiers = PCORE_TIER_MAX - 1;
constexpr int tier_wgs(int t) { return PCORE_TIER_MAX - t; }
constexpr int kDefaultTier = 0;  // the most workgroups per CU until a histogram is known

struct FusedArgs {
    // batch
    const float* poses;
    const int32_t* pose_model;
    const int32_t* pose_label;  // nullptr: 3-DoF
    const float* pose_obs_total;
    int32_t num_poses;
    // mesh: vertex-ring streams (see kVRing above)
    const float4* sverts;
    const uint32_t* stris;
    const int4* streams;
    const int32_t* model_st_lo;
    const int32_t* model_st_hi;
    const float4* model_box;  // 2 per model: (min x, y, z, 1 if every vertex is finite), (max x, y, z, 0)
    int32_t num_models;
    // camera
    float p00, p01, p02, p03, p10, p11, p12, p13;  // rows 0 and 1 of proj
    int32_t proj_sparse;  // p01, p03, p10, p13 are zeros (compute_proj's layout, renderer.cu:1386-1410)
    int32_t width, height, stride, ws, hs;
    float cx, cy, fx, fy, depth_factor;
    // observation (sampled source depth / mask at the stride grid)
    const int32_t* src_s;
    const uint8_t* lab_s;  // nullptr when 3-DoF
    const LabelGrid* grids;
    const int32_t* cell_start;
    const float4* grid_pts;
    int32_t num_grids;  // labels; the 3-DoF grid is grids[num_grids]
    int32_t bitmap_words;
    // cost
    float r2;
    float occlusion_threshold;
    int32_t calc_obs;
    float* out_rc;
    float* out_oc;
    float* out_diff;
    int32_t* dbg_zs;
    // stage CLOUD-into-scratch (GICP input): per-pose slots of `cloud_cap` points
    float4* cloud_out;
    int32_t* cloud_count;
    int32_t cloud_cap;
    // the clouds' GICP covariances (k = 10) in the same launch, same slots (6 doubles per point); nullable
    double* cloud_cov;
    // colour gate of cost_type 1 (compute_costs.cuh:201-240); null / 0 otherwise
    const uint32_t* stri_orig;  // original triangle index of every stream triangle slot
    const float4* tri_lab;      // Lab of every original triangle's colour (reference channel order)
    const float4* obs_lab;      // Lab of every observed point, label-sorted order
    int32_t* cid;               // N x nsamp scratch: original triangle of each sample's nearest fragment
    float colour_thr;           // color_distance_threshold
    // sample windows ("Pose windows"): the z-sample tile in LDS holds `tcap` samples; a pose whose window
    // is larger is processed in chunks of the tile.  fb_ctr[par] counts those poses (two buffers by launch parity)
    int32_t tcap;
    int32_t* fb_ctr;
    // window-size histogram (bin b: windows of at most hist_edge[b] samples, the last bin the rest), two sets by
    // launch parity fb_par: each launch counts into its own and its workgroup 0 publishes the other (the previous
    // launch's) to fb_host (mapped host memory, nullable: not in a captured graph) and clears it
    int32_t hist_edge[kTileTiers];
    int32_t* win_hist;  // 2 x (kTileTiers + 1) bins
    int32_t* fb_host;   // kTileTiers + 1 bins + 1 chunked-pose count + 1 sequence number
    int32_t fb_par;
    int32_t fb_seq;
    // ablation knob for profiling (PCORE_DEBUG_SKIP): bit0 skip sample raster, bit1 skip triangle stage,
    // bit2 skip phase 2 (cloud/NN), bit3 skip vertex stage.  0 in production.
    int32_t dbg_skip;  // PCORE_DEBUG_SKIP, read by the kernels only in a -DPCORE_DEBUG_SKIP_RT=1 build
    // pcore_evaluate_select: each pose's argmin key (select_kernel's) folded into sel_keys[model] by the launch
    // that scores it (nullptr: plain pcore_evaluate)
    int64_t* sel_keys;
    int64_t sel_base;
    int32_t sel_models;
};

// GICP over a chunk of poses (pcore_kernels.hip, gicp_kernel)
struct GicpArgs {
    const float4* src;        // chunk-local per-pose slots: src + pose * src_cap
    const int32_t* src_count;
    const double* src_cov;    // 6 per source point, same slots
    int32_t src_cap;
    // per-iteration scratch, same slots: each source point's correspondence (-1: none) and Mahalanobis matrix
    // (xx, xy, xz, yy, yz, zz), written by the linearisation and read by the LM trials' error sums
    int32_t* corr;
    double* mahal;
    const float4* tgt;        // observed points, label-sorted
    const double* tgt_cov;    // 6 per target point (covariances within the segment)
    const int32_t* seg_lo;    // num_segs entries
    const int32_t* seg_hi;
    int32_t num_segs;
    int32_t whole_seg;        // segment used when pose_label == nullptr (3-DoF)
    const int32_t* pose_label;  // batch-global, nullable
    const float* poses_in;    // batch-global N x 16
    float* poses_out;         // batch-global N x 16
    int32_t* iters_out;       // batch-global, nullable
    int32_t pose_base;        // first batch index of this chunk
    int32_t max_iter;
    double rot_eps, trans_eps;
    int32_t* work_counter;    // device int, zeroed by launch_gicp (persistent-wave pose queue)
    // queue order (chunk-local pose indices, nullable = index order): longest first, by the predicted cost of
    // an iteration (source points x segment targets), so the long serial chains start early
    const int32_t* pose_order;
    // neighbour grids of the segments (grids[seg], same indices as seg_lo / seg_hi): segments larger than
    // kGridNNMin targets take the exact grid search instead of the LDS scan
    const LabelGrid* grids;
    const int32_t* cell_start;
    const float4* grid_pts;
    // the segments as quads of 16 floats for the scalar-cache nearest-target scan, from quad seg_qoff[s]: a header
    // quad (the key origin in [0..2]), then four targets per quad as correspondence keys (-2 t'x [4], -2 t'y [4],
    // -2 t'z [4], |t'|^2 [4]; padding 0, 0, 0, +inf; pcore_gicp_math.h)
    const float* tgt_quads;
    const int32_t* seg_qoff;
    // correspondence history (gicp_kernel): per pose kCorrHist sets of corr_hist_cap correspondences, the sets of the
    // last searched iterations, keyed by the float transform T_f each was searched at.  An iteration whose T_f equals
    // a kept one bit for bit has the same float queries and so the same correspondences: it reuses the set instead
    // of searching.  Poses with more than corr_hist_cap source points search every iteration (into corr).
    int32_t* corr_hist;       // nullable: no history
    int32_t corr_hist_cap;
    // the cycle exit's window W (pcore_gicp_math.h cycle_update; 0 = off) and the launch's iteration counters
    // (nullable; [0] iterations reported, [1] iterations run, [2] cycle exits: one no-return atomic each per pose;
    // [3] poses that needed the grid search in the instance without it -- a host / kernel rule mismatch, an error)
    int32_t cycle_window;
    unsigned long long* iter_stats;
    // heavy poses (gicp_kernel: one workgroup each, its waves splitting the correspondence search): the poses whose
    // source points x segment targets reach heavy_cost (counted into *heavy_count by the cost-key kernel), at most
    // heavy_max, dequeued through *heavy_counter before the one-wave queue; heavy_count nullable (none)
    int32_t* heavy_counter;
    int32_t* heavy_count;
    long long heavy_cost;
    int32_t heavy_max;
    // the help board (gicp_kernel, one-wave workgroups; pcore_gicp.hip): once the pose queue runs dry, the waves that
    // find it empty help the waves still refining large poses with their correspondence searches.  help_ctl (zeroed per
    // launch, help_ctl_words): [0] queue dry, [1] poses finished, [2] poses listed, [3] unused, then help_slots
    // entries each of the list, its helpers, the claim words and the flags.  help_gran per slot (= workgroup): 16
    // granules {tag, value} of the transform (12), the pose (+ 1) and its rounds, then src_cap granules {tag,
    // correspondence}.  help_stats (zeroed per call, nullable): [0] rounds searched by helpers, [1] owner timeouts,
    // [2] helper give-ups, [3] poses enlisted.  help_ctl nullptr: no help.
    unsigned* help_ctl;
    unsigned long long* help_gran;
    unsigned long long* help_stats;
    int32_t help_slots;
    uint32_t help_tag;  // 1..0xFFFF, a different one for every launch: the granules' tags are (help_tag << 16) | epoch
    // the source covariances computed by gicp_kernel itself, in each pose's prologue (nullptr: a launch of their own
    // wrote src_cov first): cov_fold = src_cov, and the rendered clouds' sample grid of the threshold k-NN (pcore_cov.h)
    double* cov_fold;
    float cov_fx, cov_fy, cov_cx, cov_cy;
    int32_t cov_stride;
};

// The help board is built, bit-identical and measured, but off: the launch's tail is the
// 150-iteration chains of the smallest poses (one round of 64 points, nothing to share), and the board's code in the
// iteration loop (the dry-word load; 16 more VGPRs, 93 more SGPR spills) cost 3 % with the board idle.
// -DPCORE_GICP_HELP_BOARD=1 builds it (PCORE_GICP_HELP=0 then turns it off per call).
#ifndef PCORE_GICP_HELP_BOARD
#define PCORE_GICP_HELP_BOARD 0
#endif
constexpr bool kGicpHelpBoard = PCORE_GICP_HELP_BOARD;
constexpr unsigned kHelpClosed = 0xFFFF0000u;  // a help slot's claim word once its pose is done (epoch 0xFFFF)
constexpr int kHelpMaxRounds = 128;            // poses of at most 128 rounds (8,192 points) are helped
constexpr int kHelpXfGranules = 16;            // per slot, ahead of its src_cap correspondence granules
// the help board's zeroed control words for `slots` slots (a multiple of 16 bytes)
inline size_t help_ctl_words(int slots) { return 4 + 4 * (size_t)((slots + 3) & ~3); }

#if defined(PCORE_GICP_WG_WAVES) && PCORE_GICP_WG_WAVES > 1
constexpr bool kGicpHeavyBuild = true;
#else
constexpr bool kGicpHeavyBuild = false;
#endif

constexpr int kCorrHist = 16;      // history sets per pose: lanes 4e .. 4e + 3 of three VGPRs hold set e's 12 floats
constexpr int kCorrHistCap = 512;  // source points per history set (poses with more search every iteration)

// segments above this many points use the exact shell search of their neighbour grid (GICP
// correspondences and target covariances); smaller ones the brute-force scans
constexpr int kGridNNMin = 2048;

// The one rule for the exact grid search of a GICP target segment, shared by the host (which launches the
// gicp_kernel instance holding the search only when some segment needs it) and the kernels (gicp_pose's use_grid)
__host__ __device__ inline bool segment_uses_grid(int nt, bool grids_present) {
    return grids_present && nt > kGridNNMin;
}
static_assert(kGridNNMin == gicpm::kKeyScanMax, "the key scan covers exactly the segments without the grid search");

// gfx950 allocates a workgroup's LDS in 1,280-byte granules (160 KiB = 128 of them), not the 512 bytes of
// earlier CDNA parts: a census of resident fused_cost_kernel workgroups (tools/wg_timeline.py,
// tools/lds_census.sh) found 27,136-byte tiles at 5 per CU and 32,768-byte ones at 4, but 26,880 and 32,000
// bytes at 6 and 5.  PCORE_LDS_GRANULE overrides it (A/B only).
constexpr size_t kLdsGranule = 1280;

// Launch constants of one device, computed once per context (pcore_create) and passed to the launchers.
struct DeviceInfo {
    int num_cus = 0;
    int gicp_resident_wgs = 0;  // gicp_kernel workgroups the whole device holds at once (occupancy x CUs)
    size_t lds_per_cu = 0;
    size_t lds_granule = kLdsGranule;
};
// resident gicp_kernel workgroups per CU (occupancy query of the persistent launch)
hipError_t gicp_occupancy_per_cu(int* per_cu);

// launchers (pcore_kernels.hip)
hipError_t launch_render_cloud(const FusedArgs& a, hipStream_t s);
// brute-force k-NN covariances, one workgroup per segment; segments above max_n points are skipped
hipError_t launch_covariances(const float4* pts, const int32_t* seg_off, const int32_t* seg_cnt, int seg_stride,
                              int num_segs, int k, double* cov_out, hipStream_t s, int max_n = 0x7fffffff);
// the rendered ICP clouds' covariances, k = 10, by pcore_cov.h's threshold k-NN (seg i at pts + i * seg_stride)
hipError_t launch_covariances_cloud(const float4* pts, const int32_t* seg_cnt, int seg_stride, int num_segs,
                                    float fx, float fy, float cx, float cy, int stride, double* cov_out, hipStream_t s);
// covariances of the segments above kGridNNMin points via their grids (grids[first_grid + seg]), one
// thread per point; seg_off_host / seg_cnt_host: host copies of the segment table
hipError_t launch_covariances_grid(const float4* pts, const int32_t* seg_off_host, const int32_t* seg_cnt_host,
                                   int num_segs, int first_grid, const LabelGrid* grids, const int32_t* cell_start,
                                   const float4* grid_pts, int k, double* cov_out, hipStream_t s);
// grid: some segment the poses may use has more than kGridNNMin targets (the kernel instance with the grid search)
hipError_t launch_gicp(const GicpArgs& g, int num_poses, const DeviceInfo& d, hipStream_t s, bool grid = true);
// scratch of launch_gicp_order: 4 arrays of n 32-bit words + the radix sort's temporary storage
size_t gicp_order_temp_bytes(int n);
// g.pose_order for a chunk of n poses whose clouds are rendered (g.src_count): chunk-local indices sorted by
// descending src_count x segment size
hipError_t launch_gicp_order(const GicpArgs& g, int n, uint32_t* keys_in, uint32_t* keys_out, int32_t* idx_in,
                             int32_t* order_out, void* temp, size_t temp_bytes, hipStream_t s);
// pcore_states.hip: the recognizer's per-state pose building and IsValidPose neighbour counts
hipError_t launch_state_poses(const double* states, const int32_t* model, const double* preprocess,
                              const double cam[16], int num_models, int n, float* out, hipStream_t s);
hipError_t launch_count_within(const float* q, const int32_t* labels, const float* r2, int n, const float4* pts,
                               const int32_t* seg_lo, const int32_t* seg_hi, int num_segs, int32_t* out,
                               hipStream_t s);
// pcore_metrics.hip
int pose_dist_blocks(int n);
hipError_t launch_pose_distances(const float* pts, int n, const double* T_gt, const double* T_est, int pairs,
                                 double* part, double* out_add, double* out_adds, hipStream_t s);
hipError_t launch_fused_cost(const FusedArgs& a, hipStream_t s);
// LDS of one fused / cloud workgroup whose z-sample tile holds `tile_samples` samples
size_t fused_lds_bytes(int tile_samples, int bitmap_words, bool colour = false);
// tile capacity (samples) of tier t: the largest tile that leaves room for tier_wgs(t) workgroups per CU
// (capped at the whole sampled image)
int fused_tier_samples(int t, int ws, int hs, int bitmap_words, bool colour, const DeviceInfo& d);
// the tier histogram (a.hist_edge) of a batch's pose windows into hist[0..kTileTiers] (added to)
hipError_t launch_window_probe(const FusedArgs& a, int32_t* hist, hipStream_t s);
// test hook: gicpm::lm_solve_rows of n raw 28-term systems, one wave each (pcore_debug_lm_solve)
hipError_t launch_lm_solve_test(const double* sys, const double* lambda, double* out, int n, hipStream_t s);
hipError_t launch_render_full(const float* tris, int num_tris, const int32_t* tri_lo, const int32_t* tri_hi,
                              const float* poses, const int32_t* pose_model, int num_poses, int width, int height,
                              const float* proj, int32_t* depth, hipStream_t s);
// colour of stage RENDER: tri_min (N x H x W, filled with INT_MAX) receives the lowest triangle whose fragment
// depth equals the z-buffer's minimum (depth before launch_render_finalize)
hipError_t launch_render_full_tri(const float* tris, int num_tris, const int32_t* tri_lo, const int32_t* tri_hi,
                                  const float* poses, const int32_t* pose_model, int num_poses, int width, int height,
                                  const float* proj, const int32_t* depth, int32_t* tri_min, hipStream_t s);
// tri_min / rgb / color nullable (no colour): rgb packed r | g << 8 | b << 16 per triangle, color 3 planes N x H x W
hipError_t launch_render_finalize(int32_t* depth, const int32_t* src_depth, const uint8_t* src_mask,
                                  const int32_t* pose_label, int num_poses, int width, int height,
                                  float occlusion_threshold, hipStream_t s, const int32_t* tri_min = nullptr,
                                  const uint32_t* rgb = nullptr, uint8_t* color = nullptr);
hipError_t launch_fill_i32(int32_t* p, int32_t v, size_t n, hipStream_t s);
// 3-DoF world-frame bounds of depth2cloud_global (compute_point_clouds.cuh:79-91, 125-133): a pixel is
// kept when its camera-frame point, moved to the world by m (3 x 4 row-major, camera_transform), lies
// inside [b1, b0] x [b3, b2] x [b5, b4] (the reference's xmax, xmin, ymax, ymin, zmax, zmin, as floats).
struct CloudBounds {
    int32_t on;
    float m[12];
    float b[6];
    float cx, cy, fx, fy, depth_factor;
};
hipError_t launch_cloud_count(const int32_t* depth, int num_poses, int width, int height, int stride,
                              const uint8_t* label_mask, const CloudBounds& cb, int32_t* counts, hipStream_t s);
hipError_t launch_exclusive_scan(const int32_t* in, int32_t* out, int n, int32_t* total, hipStream_t s);
hipError_t launch_cloud_write(const int32_t* depth, int num_poses, int width, int height, int stride, float cx,
                              float cy, float fx, float fy, float depth_factor, const uint8_t* label_mask,
                              const int32_t* pose_label, const int32_t* offsets, float* xyz, int32_t* pose,
                              int32_t* label, int cap, const CloudBounds& cb, const uint8_t* rgb_in,
                              uint8_t* rgb_out, hipStream_t s, const uint8_t* planes_in = nullptr,
                              uint8_t* planes_out = nullptr);
// result_dc_index of stage CLOUD into dc (N x H x W int32); pre: N x (samples + 1) int32 scratch
hipError_t launch_cloud_dc_index(const int32_t* depth, int num_poses, int width, int height, int stride,
                                 const uint8_t* label_mask, const int32_t* offsets, int32_t* pre, int32_t* dc,
                                 hipStream_t s);
hipError_t launch_sample_source(const int32_t* src_depth, const uint8_t* src_mask, int width, int height,
                                int stride, int32_t* src_s, uint8_t* lab_s, hipStream_t s);
hipError_t launch_select(const float* rc, const float* oc, const int32_t* pose_model, int num_poses,
                         int64_t index_base, int num_models, int64_t* keys, hipStream_t s);

}  // namespace pcore
