// pcore_kernels.hip -- CDNA4 (gfx950) kernels of the render-and-compare hot path.
//
// Float semantics: every kernel here is compiled with -ffp-contract=off (plus the pragma below), IEEE
// f32 division and no fast-math, so each expression is evaluated in the explicit order of the
// reference CUDA code it restates (file:line cited per function).  Integer z-buffers are therefore
// bit-identical to the CPU oracle (oracle/pcore_oracle.cpp), which follows the same order.
//
// Kernels
//   fused_cost_kernel      stage COST: one workgroup per candidate pose; z-buffer of the stride-sampled
//                          pixels kept in LDS, vertex-ring stream transform, per-wave compaction of the
//                          (triangle, sample) work, source occlusion, unprojection, fixed-radius 1-NN and
//                          the three per-pose costs.  No per-pose HBM traffic except 64 B of pose in and
//                          12 B of costs out.
//   render_full_kernel     stage RENDER (parity): full-resolution z-buffer in HBM via atomicMin.
//   render_full_tri_kernel stage RENDER colour: the lowest triangle reaching each pixel's minimum depth.
//   render_finalize_kernel source occlusion + INT_MAX -> 0 on the full z-buffer (+ the colour planes).
//   cloud_count / cloud_write  stage CLOUD and depth2cloud_global: stride mask, ordered compaction, unprojection.
//   select_kernel          host selection of the reference (int cost, filter, per-model argmin key).
#include "pcore_internal.h"
#include "pcore_colour.h"
#include "pcore_cov.h"
#include "pcore_fdiv.h"

#include <algorithm>
#include <climits>
#include <cfloat>
#include <cstdlib>

#pragma clang fp contract(off)

// fragment depth quotients: 0 IEEE divisions, 3 reciprocal estimates with an error certificate and IEEE fallback
// (pcore_fdiv.h, frag_depth_certified); unscaled exact divisions for all five quotients measured slower
#ifndef PCORE_FRAG_FDIV
#define PCORE_FRAG_FDIV 3
#endif
#ifndef PCORE_STEP_UNROLL
#define PCORE_STEP_UNROLL 1
#endif

namespace pcore {

constexpr int kWave = 64;
constexpr int kWaves = kFusedWaves;  // waves per fused / cloud workgroup (one pose)
constexpr int kThreads = kWaves * kWave;
// per-wave circular ring of queued triangle records, flushed 64 at a time: after every full flush fewer than
// 64 remain and a batch appends at most 64, so 128 never overflows; phase 2 reuses it as a point queue of
// up to 127 (tile index, kx | ky << 16) pairs
constexpr int kRecCap = 128;
// per-wave record ring stride: kRecCap records + a discard record (lanes with nothing to queue write there, so the
// queue store needs no branch) + one for 16-byte alignment
constexpr int kRecStride = kRecCap + 2;
constexpr int64_t PCORE_KEY_NONE_DEV = 0x7fffffffffffffffLL;
constexpr int kSmallK = 4;    // triangles touching <= kSmallK samples are queued; larger ones are
                              // processed cooperatively by the whole wave

// ------------------------------------------------------------------------------------------------
// Exact-semantics helpers (shared by every kernel)
// ------------------------------------------------------------------------------------------------

// x86 cvttss2si semantics of the host `(int) float` casts (search_env.cpp:2022-2048).
__device__ __forceinline__ int32_t cvt_i32_x86(float f) {
    if (!(f == f) || f >= 2147483648.0f || f < -2147483648.0f) return INT_MIN;
    return (int32_t)f;
}

// CUDA abs() of a wrapped int32 difference (image_renderer.cuh:163-165).
__device__ __forceinline__ int32_t iabs_wrap(int32_t a, int32_t b) {
    int32_t d = (int32_t)((uint32_t)a - (uint32_t)b);
    return d < 0 ? (int32_t)(0u - (uint32_t)d) : d;
}

__device__ __forceinline__ float ref_max(float a, float b) { return (a > b) ? a : b; }  // image_renderer.cuh:14-15
__device__ __forceinline__ float ref_min(float a, float b) { return (a < b) ? a : b; }  // image_renderer.cuh:17-18

// mat_mul_v row (image_renderer.cuh:20-27): ((m0*x + m1*y) + m2*z) + m3
__device__ __forceinline__ float row4(float m0, float m1, float m2, float m3, float x, float y, float z) {
    return m0 * x + m1 * y + m2 * z + m3;
}

// Source-occlusion rule applied to the per-pixel minimum fragment depth.  Equals the reference's
// serial z-test + black-out sequence (image_renderer.cuh:146-196) for every fragment order because the
// black-out predicate is monotone in the stored depth ("Deterministic raster contract").
__device__ __forceinline__ int32_t occlusion_rule(int32_t z, int32_t src, int lab, bool use_seg, int32_t pl,
                                                  float occlusion_threshold) {
    if (z == INT_MAX) return 0;  // no fragment: max2zero (image_renderer.cuh:465-466)
    bool cond;
    if (use_seg) cond = (pl != lab - 1) && ((float)iabs_wrap(z, src) > 0.5f);
    else cond = (float)iabs_wrap(z, src) > occlusion_threshold;
    if (cond && z > src && src > 0) return 0;  // blacked out -> INT_MAX -> max2zero
    return z;
}

// Reference bounding box (image_renderer.cuh:86-107) with its exact NaN behaviour.
__device__ __forceinline__ void bbox_ref(const float (&p)[3][2], float cmax0, float cmax1, float (&bmin)[2],
                                         float (&bmax)[2]) {
    bmin[0] = FLT_MAX; bmin[1] = FLT_MAX;
    bmax[0] = -FLT_MAX; bmax[1] = -FLT_MAX;
    const float cmax[2] = {cmax0, cmax1};
#pragma unroll
    for (int i = 0; i < 3; i++)
#pragma unroll
        for (int j = 0; j < 2; j++) {
            bmin[j] = ref_max(0.0f, ref_min(bmin[j], p[i][j]));
            bmax[j] = ref_min(cmax[j], ref_max(bmax[j], p[i][j]));
        }
}

// Loop bounds of `for (P = size_t(bmin + 0.5f); P <= bmax; ++P)` (image_renderer.cuh:110-111) with
// NVIDIA float->u64 conversion (NaN/negative -> 0, saturating).  Returns false if the loop is empty.
__device__ __forceinline__ bool loop_bounds(float bmin, float bmax, int& lo, int& hi) {
    if (!(bmax >= 0.0f)) return false;  // NaN or negative upper bound: P (>= 0) <= bmax never holds
    const float st = bmin + 0.5f;
    int start;
    if (!(st > 0.0f)) start = 0;
    else if (st >= 1.0e9f) return false;  // bmax <= width-1, so a start this large never iterates
    else start = (int)st;
    hi = (int)floorf(bmax);
    lo = start;
    return lo <= hi;
}

// One fragment test at raster pixel (P0, P1) (image_renderer.cuh:44-57, 112-129).  Returns true and the
// int depth if the pixel is inside the triangle (NaN barycentrics count as inside, as in the reference).
// Returns whether the pixel is inside (NaN barycentrics count as inside, as in the reference) and sets the depth
// for inside pixels; every lane runs the same instructions (no branch on the inside test), so a batch of
// fragment tests is one straight-line block plus the depth's rare IEEE fallback.
__device__ __forceinline__ bool fragment(float A0, float A1, float B0, float B1, float C0, float C1, float z0,
                                         float z1, float z2, float P0, float P1, int32_t& depth, bool z_ok = false) {
    const float area = 0.5f * ((C0 - A0) * (B1 - A1) - (B0 - A0) * (C1 - A1));
    const float base_inv = 1.0f / area;
    const float beta = 0.5f * ((C0 - A0) * (P1 - A1) - (P0 - A0) * (C1 - A1)) * base_inv;
    const float gamma = 0.5f * ((P0 - A0) * (B1 - A1) - (B0 - A0) * (P1 - A1)) * base_inv;
    const float alpha = 1.0f - beta - gamma;
    // !(alpha < -0 || beta < -0 || gamma < -0 || alpha > 1 || beta > 1 || gamma > 1) as one v_min3 / v_max3 each:
    // the three are arithmetic results (quiet NaNs at most), on which v_min3 / v_max3 follow IEEE minNum / maxNum
    // -- a NaN operand is skipped, as in the comparisons, and an all-NaN triple gives NaN (inside, as in the
    // reference) -- so the compiler's canonicalising v_max per operand (it cannot know there is no sNaN) is not needed
    float mn, mx;
    asm("v_min3_f32 %0, %1, %2, %3" : "=v"(mn) : "v"(alpha), "v"(beta), "v"(gamma));
    asm("v_max3_f32 %0, %1, %2, %3" : "=v"(mx) : "v"(alpha), "v"(beta), "v"(gamma));
    const bool inside = !(mn < -0.0f) && !(mx > 1.0f);
#if PCORE_FRAG_FDIV == 3
    // the depth quotient chain through reciprocal estimates with an error certificate, the IEEE divisions only
    // where the certificate fails (pcore_fdiv.h, frag_depth_certified); outside lanes never take the fallback
    depth = frag_depth_certified(alpha, beta, gamma, z0, z1, z2, z_ok, inside);
#else
    (void)z_ok;
    depth = 0;
    if (inside) {
        const float ox = alpha / z0, oy = beta / z1, oz = gamma / z2;
        depth = cvt_i32_rz_sat((alpha + beta + gamma) / (ox + oy + oz) + 0.5f);
    }
#endif
    return inside;
}

__device__ __forceinline__ void wave_sync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

__device__ __forceinline__ int lane_id() { return __builtin_amdgcn_mbcnt_hi(~0u, __builtin_amdgcn_mbcnt_lo(~0u, 0)); }

__device__ __forceinline__ int mbcnt64(uint64_t mask) {
    return __builtin_amdgcn_mbcnt_hi((uint32_t)(mask >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)mask, 0));
}

// ------------------------------------------------------------------------------------------------
// Stage COST: fused sampled render + unproject + 1-NN + cost
// ------------------------------------------------------------------------------------------------

struct TriRec {  // a triangle in registers: screen-space vertices, camera z
    float a0, a1, b0, b1, c0, c1, z0, z1, z2;
};
// A queued triangle in the LDS record ring (8 bytes): x = its three vertex-ring slots i0 | i1 << 9 | i2 << 18,
// y = its sample window kx0 | ky0 << 12 | (nx-1) << 24 | (ny-1) << 28 (nx * ny <= kSmallK).

template <int STRIDE>
__device__ __forceinline__ int sdiv(int v, int s) {
    if constexpr (STRIDE > 0) return v / STRIDE;
    else return v / s;
}

// Sample window of a triangle with exact reference bbox (bmin, bmax): kx in [kx0, kx0+nx),
// ky in [ky0, ky0+ny) where the sampled output pixel is (kx*s, ky*s) and raster row P1 = H-1-ky*s.
template <int STRIDE>
__device__ __forceinline__ int sample_window(const float (&bmin)[2], const float (&bmax)[2], int s, int H, int& kx0,
                                             int& ky0, int& nx, int& ny) {
    int lo0, hi0, lo1, hi1;
    if (!loop_bounds(bmin[0], bmax[0], lo0, hi0)) return 0;
    if (!loop_bounds(bmin[1], bmax[1], lo1, hi1)) return 0;
    const int ss = STRIDE > 0 ? STRIDE : s;
    kx0 = sdiv<STRIDE>(lo0 + ss - 1, s);
    const int kx1 = sdiv<STRIDE>(hi0, s);
    // output rows y = H-1-P1 for P1 in [lo1, hi1]
    ky0 = sdiv<STRIDE>(H - 1 - hi1 + ss - 1, s);
    const int ky1 = sdiv<STRIDE>(H - 1 - lo1, s);
    nx = kx1 - kx0 + 1;
    ny = ky1 - ky0 + 1;
    if (nx <= 0 || ny <= 0) return 0;
    return nx * ny;
}

struct FusedSmem {
    int32_t* zbuf;  // tile samples
    float2* vxy;    // kWaves * kVRing * 64: screen (x, y) of the wave's vertex ring
    float* vz;      // kWaves * kVRing * 64: camera z (cm)
    uint2* vbd;     // kWaves * 2 * 64: packed int16 sample-window bounds of the last two passes
    uint2* ring;    // kWaves * kRecStride queued triangle records (phase 1); int32 point queues in phase 2
    uint32_t* ring_id;  // kWaves * kRecStride original triangle ids (colour id pass only)
    uint32_t* bitmap;
    int32_t* counters;  // [0] bad, [1] explained, [2] points; [4..8] the pose window (x0, y0, nx, ny, fastdiv)
};
constexpr int kRingSlots = kVRing * kWave;
static_assert(kRingSlots <= (1 << kRingSlotBits), "vertex ring slots must fit the 9-bit triangle indices");
static_assert(kVRing > kRefPasses, "the ring must hold the referenced passes and the one being written");
static_assert(kRecCap >= 128 && (kRecCap & (kRecCap - 1)) == 0, "record ring: >= 128 records, a power of two");

// IDPASS = false: depth pass (atomicMin of the fragment depth).  IDPASS = true: colour id pass over the
// final depths: the fragments whose depth equals the sample's minimum leave the lowest original triangle
// index -- the colour the reference's serial z-test (strict <) keeps.
// Sample window of a pose: samples kx in [x0, x0 + nx), ky in [y0, y0 + ny); the LDS z-sample tile stores
// them row-major, sample (kx, ky) at (ky - y0) * nx + (kx - x0).
struct SampleWin {
    int x0, y0, nx, ny;
    // every vertex of the pose has 1 <= z < 2^41 and |x|, |y| < 2^41 after the projection (pose_window's bounds),
    // so the vertex pass needs no per-vertex range check of its unscaled division (see the vertex pass)
    int fastdiv;
};

template <bool IDPASS = false>
__device__ __forceinline__ void raster_sample(const TriRec& r, int kx, int ky, int s, int H, const SampleWin& w,
                                              int32_t* zbuf, int32_t* cid = nullptr, uint32_t id = 0) {
    const float P0 = (float)(kx * s);
    const float P1 = (float)(H - 1 - ky * s);
    int32_t d;
    const bool in = fragment(r.a0, r.a1, r.b0, r.b1, r.c0, r.c1, r.z0, r.z1, r.z2, P0, P1, d, w.fastdiv != 0);
    const int k = (int)__umul24((uint32_t)(ky - w.y0), (uint32_t)w.nx) + (kx - w.x0);  // inside the window
    if constexpr (IDPASS) {
        if (in && d == zbuf[k]) atomicMin(&cid[k], (int32_t)id);
    } else {
        // only inside lanes take part: an outside lane's INT_MAX min changed nothing but still collided with the
        // inside lanes on the same bank (C2: SQ_LDS_BANK_CONFLICT 15.1 M -> 11.0 M per launch, time unchanged)
        if (in) atomicMin(&zbuf[k], d);
    }
}

size_t fused_lds_bytes(int tile_samples, int bitmap_words, bool colour) {
    auto al = [](size_t b) { return (b + 15) & ~size_t(15); };
    size_t b = al((size_t)tile_samples * 4);
    b += al((size_t)kWaves * kRingSlots * 8);
    b += al((size_t)kWaves * kRingSlots * 4);
    b += al((size_t)kWaves * 2 * kWave * 8);
    b += al((size_t)kWaves * kRecStride * 8);
    if (colour) b += al((size_t)kWaves * kRecStride * 4);
    b += al((size_t)bitmap_words * 4);
    b += 48;  // counters: [0] bad, [1] explained, [2] points; [4..8] the pose window (fused_cost_kernel)
    return b;
}

__device__ __forceinline__ FusedSmem carve_smem(unsigned char* smem_raw, int nsamp, int bitmap_words,
                                                bool colour = false) {
    auto al = [](size_t b) { return (b + 15) & ~size_t(15); };
    FusedSmem sm;
    unsigned char* p = smem_raw;
    sm.zbuf = (int32_t*)p; p += al((size_t)nsamp * 4);
    sm.vxy = (float2*)p; p += al((size_t)kWaves * kRingSlots * 8);
    sm.vz = (float*)p; p += al((size_t)kWaves * kRingSlots * 4);
    sm.vbd = (uint2*)p; p += al((size_t)kWaves * 2 * kWave * 8);
    sm.ring = (uint2*)p; p += al((size_t)kWaves * kRecStride * 8);
    sm.ring_id = nullptr;
    if (colour) { sm.ring_id = (uint32_t*)p; p += al((size_t)kWaves * kRecStride * 4); }
    sm.bitmap = (uint32_t*)p; p += al((size_t)bitmap_words * 4);
    sm.counters = (int32_t*)p;
    return sm;
}

template <int STRIDE>
__device__ __forceinline__ int floor_div(int v, int s) {
    if constexpr (STRIDE == 8) return v >> 3;  // arithmetic shift == floor division by 8
    else {
        const int q = v / s;
        return (v % s != 0 && v < 0) ? q - 1 : q;
    }
}

// Sample window of a triangle whose screen coordinates are not NaN (finite or infinite), from the reference's
// bounding box and loop bounds (image_renderer.cuh:86-111): bmin = max(0, min p), first pixel trunc(bmin + 0.5);
// bmax = min(W-1, max p), last pixel floor(bmax) -- for non-NaN inputs the ternary chains of bbox_ref() are exactly
// these min / max.  Clamping to [0, 65536] / [-65536, W-1] first changes no window of a <= 16384-pixel image and
// keeps the conversions in range.  Sample kx covers raster column kx * s, sample row ky raster row H-1-ky*s:
//   a0 = ceil(trunc(max(0, min x) + 0.5) / s)      a1 = floor(floor(min(W-1, max x)) / s)
//   b0 = ceil((H-1 - floor(min(H-1, max y))) / s)  b1 = floor((H-1 - trunc(max(0, min y) + 0.5)) / s)
// Each bound is a monotone function of the triangle's min or max coordinate, so it equals the min or max of that
// function over the three vertices: a0 = min A0(x_i), a1 = max A1(x_i), b0 = min B0(y_i), b1 = max B1(y_i), and
// clipping to the pose window commutes as well.  The vertex pass stores (A0, B0) and (A1, B1) as int16 pairs;
// the triangle stage takes two packed minima and two packed maxima.  At stride 8 every bound fits int16
// (|bound| <= (16384 + 65536) / 8); the generic stride clamps them to +-32767, which leaves a window of a
// <= 16384-sample image empty exactly when it was.  A NaN screen coordinate marks the vertex with -32768 lower
// bounds (a real lower bound is >= 0), and its triangles take the reference's NaN-propagating bbox instead.
// floor(v + 0.5) and floor(v) of a finite float of magnitude < 2^23 (exact), one instruction each
__device__ __forceinline__ int cvt_rpi(float v) {
    int r;
    asm("v_cvt_rpi_i32_f32 %0, %1" : "=v"(r) : "v"(v));
    return r;
}
__device__ __forceinline__ int cvt_flr(float v) {
    int r;
    asm("v_cvt_flr_i32_f32 %0, %1" : "=v"(r) : "v"(v));
    return r;
}

typedef short short2v __attribute__((ext_vector_type(2)));
__device__ __forceinline__ short2v as_s2(uint32_t v) { return __builtin_bit_cast(short2v, v); }
constexpr uint32_t kNanBounds = 0x80008000u;

template <int STRIDE>
__device__ __forceinline__ uint2 vertex_bounds(float sx, float sy, int s, float cmax0, float cmax1, int H,
                                              bool finite = false) {
    if (!finite && __builtin_isunordered(sx, sy)) return make_uint2(kNanBounds, 0u);
    const int ss = STRIDE > 0 ? STRIDE : s;
    // sx, sy are not NaN here, so each clamp is one v_med3_f32, and the clamped values are small enough
    // (|v| <= 65536 < 2^23) that v + 0.5 is exact: trunc(v + 0.5) = floor(v + 0.5) for v >= 0 is one
    // v_cvt_rpi_i32_f32, floor(v) one v_cvt_flr_i32_f32 (cvt_rpi / cvt_flr below)
    const int lo0 = cvt_rpi(__builtin_amdgcn_fmed3f(sx, 0.0f, 65536.0f));
    const int lo1 = cvt_rpi(__builtin_amdgcn_fmed3f(sy, 0.0f, 65536.0f));
    const int hi0 = cvt_flr(__builtin_amdgcn_fmed3f(sx, -65536.0f, cmax0));
    const int hi1 = cvt_flr(__builtin_amdgcn_fmed3f(sy, -65536.0f, cmax1));
    int A0 = floor_div<STRIDE>(lo0 + ss - 1, s), A1 = floor_div<STRIDE>(hi0, s);
    int B0 = floor_div<STRIDE>(H - 1 - hi1 + ss - 1, s), B1 = floor_div<STRIDE>(H - 1 - lo1, s);
    if constexpr (STRIDE == 0) {
        A0 = min(A0, 32767);
        B0 = min(B0, 32767);
        A1 = max(A1, -32767);
        B1 = max(B1, -32767);
    }
    return make_uint2(((uint32_t)A0 & 0xffffu) | ((uint32_t)B0 << 16), ((uint32_t)A1 & 0xffffu) | ((uint32_t)B1 << 16));
}

// Measurement build only (-DPCORE_FUSED_PROFILE, tools/fused_phase_prof.py): per-wave shader clocks of the
// fused kernel's phases -- [0] setup, [1] vertex stage, [2] triangle windows + queueing, [3] fragment
// batches, [4] wait at the end-of-raster barrier, [5] phase 2 (occlusion, unprojection, 1-NN, counts),
// [6] phase 3 + barriers.  Each wave sums in registers and adds once at exit.
#ifdef PCORE_FUSED_PROFILE
__device__ unsigned long long g_fprof[8];
extern "C" int pcore_debug_fused_profile(unsigned long long* out, int reset) {
    hipError_t e = hipMemcpyFromSymbol(out, HIP_SYMBOL(g_fprof), sizeof(unsigned long long) * 8);
    if (e == hipSuccess && reset) {
        const unsigned long long z[8] = {0, 0, 0, 0, 0, 0, 0, 0};
        e = hipMemcpyToSymbol(HIP_SYMBOL(g_fprof), z, sizeof(z));
    }
    return e == hipSuccess ? 0 : 1;
}
struct FProf {
    unsigned long long acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    unsigned long long last = __builtin_amdgcn_s_memtime();
    __device__ __forceinline__ void mark(int k) {
        const unsigned long long t = __builtin_amdgcn_s_memtime();
        acc[k] += t - last;
        last = t;
    }
    __device__ __forceinline__ void flush() {
        if ((threadIdx.x & 63) == 0)
            for (int k = 0; k < 8; k++) atomicAdd(&g_fprof[k], acc[k]);
    }
};
#else
struct FProf {
    __device__ __forceinline__ void mark(int) {}
    __device__ __forceinline__ void flush() {}
};
#endif

#ifdef PCORE_FLUSH_STATS
// measurement build only: small-triangle flush batches, records, fragment tests, loop trips
__device__ unsigned long long pcore_flush_stats[9];
extern "C" int pcore_debug_flush_stats(unsigned long long* host) {
    return (int)hipMemcpyFromSymbol(host, HIP_SYMBOL(pcore_flush_stats), sizeof(unsigned long long) * 9);
}
#endif

// FD: the pose's fastdiv flag known at compile time (0 / 1; the depth pass instantiates both and picks one per pose, so
// a fastdiv pose's steps carry no NaN-triangle test or range checks at all), or -1 to read it from the window
template <int STRIDE, bool IDPASS = false, int FD = -1>
__device__ __forceinline__ void raster_phase(const FusedArgs& a, const FusedSmem& sm, int pose, const SampleWin& sw_in,
                                             int32_t* cid, FProf& fp) {
    SampleWin sw = sw_in;
    if constexpr (FD >= 0) sw.fastdiv = FD;
    const int tid = threadIdx.x;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);  // wave-uniform: scalar loads of stream headers
    const int lane = tid & 63;
    const int s = STRIDE > 0 ? STRIDE : a.stride;
    const int W = a.width, H = a.height;
    // pose (wave-uniform -> scalar loads)
    const float* P = a.poses + (size_t)16 * pose;
    const float m00 = P[0], m01 = P[1], m02 = P[2], m03 = P[3];
    const float m10 = P[4], m11 = P[5], m12 = P[6], m13 = P[7];
    const float m20 = P[8], m21 = P[9], m22 = P[10], m23 = P[11];
    const int model = a.pose_model[pose];
    // Projection with compute_proj's zeros skipped: the reference's ((p00 x + p01 y) + p02 z) + p03 with
    // p01 = p03 = 0 differs from p00 x + p02 z only in the sign of a zero result -- which x / z * W/2 + W/2
    // does not see (both give W/2 exactly) -- as long as the skipped products 0 * y are zeros, i.e. the camera
    // point is finite.  It is when every model vertex is finite (model_box flag) and the bound of |row . v|
    // over the model's box (B below, as in pose_window) stays far from FLT_MAX; NaN entries fail the test.
    bool proj_sparse = false;
    if (a.proj_sparse && model >= 0 && model < a.num_models) {
        const float4 lo = a.model_box[2 * model], hi = a.model_box[2 * model + 1];
        const float ax = fmaxf(fabsf(lo.x), fabsf(hi.x)), ay = fmaxf(fabsf(lo.y), fabsf(hi.y));
        const float az = fmaxf(fabsf(lo.z), fabsf(hi.z));
        const float Bx = fabsf(m00) * ax + fabsf(m01) * ay + fabsf(m02) * az + fabsf(m03);
        const float By = fabsf(m10) * ax + fabsf(m11) * ay + fabsf(m12) * az + fabsf(m13);
        proj_sparse = lo.w != 0.0f && Bx < 1.0e30f && By < 1.0e30f;
    }
    __syncthreads();

    // ---------------- phase 1: raster of the sampled pixels ----------------
    const float Wf = (float)W, Hf = (float)H;
    const float hw = Wf / 2.0f, hh = Hf / 2.0f;
    const float cmax0 = (float)(W - 1), cmax1 = (float)(H - 1);
    float2* vxy = sm.vxy + wave * kRingSlots;
    float* vz = sm.vz + wave * kRingSlots;
    uint2* vbd = sm.vbd + wave * 2 * kWave;
    // the pose window as int16 pairs (first sample, last sample); an empty window has last < first
    const short2v wfirst = {(short)sw.x0, (short)sw.y0};
    const short2v wlast = {(short)(sw.x0 + sw.nx - 1), (short)(sw.y0 + sw.ny - 1)};
    uint2* ring = sm.ring + wave * kRecStride;
    uint32_t* ring_id = IDPASS ? sm.ring_id + wave * kRecStride : nullptr;
    // record ring: wave-uniform monotone counters of appended and flushed records; record i lives in slot
    // i mod kRecCap.  Full 64-record batches are flushed as soon as they exist; a partial batch only when a
    // vertex pass would overwrite vertices a pending record may reference, at a stream switch and at the end.
    int rec_total = 0, rec_done = 0;

    // PCORE_DEBUG_SKIP ablations only in a -DPCORE_DEBUG_SKIP_RT=1 build (tools/ablate_sq.sh): a run-time flag kept as a
    // lane-mask boolean across the step loop cost two VALU per test per step
#if PCORE_DEBUG_SKIP_RT
    const int dbg = a.dbg_skip;
#else
    constexpr int dbg = 0;
#endif
    auto flush = [&](int count) {  // the `count` oldest pending records
        fp.mark(2);
        wave_sync();
        if (!(dbg & 1)) {
            for (int base = 0; base < count; base += kWave) {
#ifdef PCORE_FLUSH_STATS
                if (lane == 0) {
                    atomicAdd(&pcore_flush_stats[0], 1ull);
                    atomicAdd(&pcore_flush_stats[1], (unsigned long long)min(count - base, kWave));
                }
#endif
                if (base + lane < count) {
                    const int j = (rec_done + base + lane) & (kRecCap - 1);
                    const uint2 rec = ring[j];
                    const uint32_t id = IDPASS ? ring_id[j] : 0u;
                    const int i0 = rec.x & 511, i1 = (rec.x >> 9) & 511, i2 = (rec.x >> 18) & 511;
                    const float2 q0 = vxy[i0], q1 = vxy[i1], q2 = vxy[i2];
                    TriRec r;
                    r.a0 = q0.x; r.a1 = q0.y;
                    r.b0 = q1.x; r.b1 = q1.y;
                    r.c0 = q2.x; r.c1 = q2.y;
                    r.z0 = vz[i0]; r.z1 = vz[i1]; r.z2 = vz[i2];
                    // the depths are needed only past the inside test, but reading them with the screen
                    // coordinates puts all six reads in one LDS round trip instead of two
                    asm volatile("" : "+v"(r.z0), "+v"(r.z1), "+v"(r.z2));
                    // one record per (triangle, sample): the sample is rec.y = kx | ky << 16
#ifdef PCORE_FLUSH_STATS
                    atomicAdd(&pcore_flush_stats[2], 1ull);
#endif
                    raster_sample<IDPASS>(r, (int)(rec.y & 0xffffu), (int)(rec.y >> 16), s, H, sw, sm.zbuf, cid, id);
                }
            }
        }
        rec_done += count;
        wave_sync();
        fp.mark(3);
    };

    if (model < 0 || model >= a.num_models) return;
    const int st_lo = a.model_st_lo[model], st_hi = a.model_st_hi[model];
    fp.mark(0);
    for (int st = st_lo + wave; st < st_hi; st += kWaves) {
        const int4 sd = a.streams[st];  // first step, end step, first vertex pass, end vertex pass
        if (rec_total > rec_done) {      // a new stream numbers its ring slots from buffer 0
#ifdef PCORE_FLUSH_STATS
            if (lane == 0) atomicAdd(&pcore_flush_stats[3], 1ull);
#endif
            flush(rec_total - rec_done);
        }
        // hist[k]: rec_total when pass P-1-k was written (P = the next pass).  A batch issued after pass h
        // references passes >= h - kRefPasses + 1, so before pass P overwrites the buffer of pass P - kVRing every
        // record appended before pass P - (kVRing - kRefPasses) was written must be flushed.
        int hist[kVRing - kRefPasses];
#pragma unroll
        for (int k = 0; k < kVRing - kRefPasses; k++) hist[k] = rec_total;
        int buf = 0;                 // ring buffer of the next vertex pass
        // wave-uniform stream pointers (SGPRs): the current step's triangle slots and the next unconsumed vertex pass
        const uint32_t* tp = a.stris + (size_t)sd.x * kStepSlots;
        const uint32_t* op = IDPASS ? a.stri_orig + (size_t)sd.x * kStepSlots : nullptr;
        const float4* vq = a.sverts + (size_t)sd.z * kStepSlots;
        // one step: the current step's triangle slots / vertex pass in (cv, ct, cidt); prefetches the next step's
        // triangle slots and the next unconsumed vertex pass into (ncv, nct, ncid) -- unconditional loads (after a
        // stream's last step they read the next stream's first, or the padding step and pass the upload appends).
        // The loop below alternates two register sets, so no copy of a prefetched register makes the wave wait
        // for the load at the end of its step.
        auto run_step = [&](int step, const float4& cv, const uint32_t ct, const uint32_t cidt, float4& ncv,
                            uint32_t& nct, uint32_t& ncid) {
            (void)step;
            tp += kStepSlots;
            nct = tp[lane];
            if constexpr (IDPASS) {
                op += kStepSlots;
                ncid = op[lane];
            } else {
                ncid = 0u;
            }
            // the step's "vertex pass first" flag is in every triangle slot (pcore_internal.h)
            const bool vpass = (__builtin_amdgcn_readfirstlane((int)ct) >> 30) & 1;
            if (vpass) vq += kStepSlots;
            ncv = vq[lane];
            if (vpass) {
                if (rec_done < hist[kVRing - kRefPasses - 1]) {
#ifdef PCORE_FLUSH_STATS
                    if (lane == 0) atomicAdd(&pcore_flush_stats[3], 1ull);
#endif
                    flush(rec_total - rec_done);
                }
                // vertex stage: model transform, keep camera z, projection rows 0/1, viewport
                // (image_renderer.cuh:296-305, 82-84)
                // every lane transforms its slot: a padding lane (cv.w == 0) writes a slot no triangle names
                if (!(dbg & 8)) {
                    const float lx = row4(m00, m01, m02, m03, cv.x, cv.y, cv.z);
                    const float ly = row4(m10, m11, m12, m13, cv.x, cv.y, cv.z);
                    const float lz = row4(m20, m21, m22, m23, cv.x, cv.y, cv.z);
                    float px, py;
                    if (proj_sparse) {
                        px = a.p00 * lx + a.p02 * lz;
                        py = a.p11 * ly + a.p12 * lz;
                    } else {
                        px = row4(a.p00, a.p01, a.p02, a.p03, lx, ly, lz);
                        py = row4(a.p10, a.p11, a.p12, a.p13, lx, ly, lz);
                    }
                    // px / lz and py / lz sharing one refined reciprocal of lz, IEEE-exact where every exponent is
                    // in range (pcore_fdiv.h); there |q| < 2^81, so (q * W) / 2 is q * (W / 2) exactly (a power-of-
                    // two scaling, no overflow or underflow).  Elsewhere the reference's expressions.  With the pose's
                    // fastdiv bound (1 <= lz < 2^41, |px|, |py| < 2^41) the only operand out of range is a numerator
                    // below 2^-40, whose quotient (IEEE or unscaled) is below 2^-40: q * W/2 + W/2 rounds to W/2 either
                    // way, so no per-vertex check is needed.
                    const float r1 = recip_refined(lz);
                    float qx = quot_refined(px, lz, r1), qy = quot_refined(py, lz, r1);
                    float sx = qx * hw + hw, sy = qy * hh + hh;
                    if (!sw.fastdiv) {
                        const uint32_t ex = fexp_bits(px), ey = fexp_bits(py), ez = fexp_bits(lz);
                        if (!fdiv_range_ok(min(min(ex, ey), ez), max(max(ex, ey), ez))) {
                            asm volatile("");
                            qx = px / lz;
                            qy = py / lz;
                            sx = qx * Wf / 2.0f + Wf / 2.0f;
                            sy = qy * Hf / 2.0f + Hf / 2.0f;
                        }
                    }
                    vxy[buf * kWave + lane] = make_float2(sx, sy);
                    vz[buf * kWave + lane] = lz;
                    // a wave-uniform branch, so a fastdiv pose's pass carries no NaN test, default bounds or exec
                    // masking (the screen coordinates are finite there)
                    uint2 vb;
                    if (sw.fastdiv) vb = vertex_bounds<STRIDE>(sx, sy, s, cmax0, cmax1, H, true);
                    else vb = vertex_bounds<STRIDE>(sx, sy, s, cmax0, cmax1, H, false);
                    vbd[(buf & 1) * kWave + lane] = vb;
                }
#pragma unroll
                for (int k = kVRing - kRefPasses - 1; k > 0; k--) hist[k] = hist[k - 1];
                hist[0] = rec_total;
                buf = buf + 1 == kVRing ? 0 : buf + 1;
#ifdef PCORE_FLUSH_STATS
                if (lane == 0) atomicAdd(&pcore_flush_stats[8], 1ull);
#endif
                wave_sync();
            }
            fp.mark(1);
            if (!(dbg & 2)) {
                // the triangle's clipped window, packed: pos = first sample (kx0 | ky0 << 16), nxy = its size
                // (nx | ny << 16), nk = nx * ny samples (0: none)
                uint32_t pos = 0u, nxy = 0u;
                int nk = 0;
                // the vertices' ring slots (9 bits each) and, for the bounds, their pass parity + lane (7 bits);
                // the slots proper are decoded only where a rare path needs the screen coordinates
                auto slot_of = [ct](int k) { return (int)((ct >> (9 * k)) & 511u); };
                // a padding slot names slot 0 three times: its bounds are read (harmless) and nk forced to 0
                const bool pad = ct >> 31;
                {
                    // bit-field extracts as v_bfe (asm: the compiler turns them back into shift / mask / add, three
                    // instructions per address instead of v_bfe + v_lshl_add)
                    uint32_t i1, i2;
                    asm("v_bfe_u32 %0, %1, 9, 7" : "=v"(i1) : "v"(ct));
                    asm("v_bfe_u32 %0, %1, 18, 7" : "=v"(i2) : "v"(ct));
                    const uint2 w0 = vbd[ct & 127u], w1 = vbd[i1], w2 = vbd[i2];
                    short2v lo = __builtin_elementwise_min(__builtin_elementwise_min(as_s2(w0.x), as_s2(w1.x)), as_s2(w2.x));
                    short2v hi = __builtin_elementwise_max(__builtin_elementwise_max(as_s2(w0.y), as_s2(w1.y)), as_s2(w2.y));
                    // (fastdiv poses have finite screen coordinates: no NaN vertex)
                    const bool nan_tri = !sw.fastdiv && lo.x < 0 && !pad;
                    lo = __builtin_elementwise_max(lo, wfirst);
                    hi = __builtin_elementwise_min(hi, wlast);
                    const short2v d = hi - lo;  // (nx - 1, ny - 1), negative where the window is empty
                    const short2v one = {1, 1};
                    pos = __builtin_bit_cast(uint32_t, lo);
                    nxy = __builtin_bit_cast(uint32_t, d + one);
                    const bool nonempty = (__builtin_bit_cast(uint32_t, d) & 0x80008000u) == 0u && !pad;
                    nk = nonempty ? (int)__umul24(nxy & 0xffffu, nxy >> 16) : 0;
                    if (nan_tri) {
                        // NaN screen coordinates: the reference's exact bbox with its NaN-propagating clamps
                        const float2 q0 = vxy[slot_of(0)], q1 = vxy[slot_of(1)], q2 = vxy[slot_of(2)];
                        const float p[3][2] = {{q0.x, q0.y}, {q1.x, q1.y}, {q2.x, q2.y}};
                        float bmin[2], bmax[2];
                        bbox_ref(p, cmax0, cmax1, bmin, bmax);
                        int kx0 = 0, ky0 = 0, nx = 0, ny = 0;
                        nk = sample_window<STRIDE>(bmin, bmax, s, H, kx0, ky0, nx, ny);
                        if (nk > 0) {  // clip to the pose window
                            const int kx1 = min(kx0 + nx, sw.x0 + sw.nx), ky1 = min(ky0 + ny, sw.y0 + sw.ny);
                            kx0 = max(kx0, sw.x0);
                            ky0 = max(ky0, sw.y0);
                            nx = kx1 - kx0;
                            ny = ky1 - ky0;
                            nk = (nx > 0 && ny > 0) ? nx * ny : 0;
                        }
                        pos = (uint32_t)kx0 | ((uint32_t)ky0 << 16);
                        nxy = (uint32_t)nx | ((uint32_t)ny << 16);
                    }
                }
                // large triangles: whole-wave cooperative
                uint64_t big = __ballot(nk > kSmallK);
#ifdef PCORE_FLUSH_STATS
                {
                    const uint64_t btouch = __ballot(nk > 0), blanes = __ballot(!(ct >> 31));
                    if (lane == 0) {
                        atomicAdd(&pcore_flush_stats[4], (unsigned long long)__popcll(big));
                        atomicAdd(&pcore_flush_stats[5], (unsigned long long)__popcll(btouch));
                        atomicAdd(&pcore_flush_stats[6], (unsigned long long)__popcll(blanes));
                        atomicAdd(&pcore_flush_stats[7], 1ull);
                    }
                }
#endif
                if (big) {
                    // the big triangles' screen vertices, read again (rare: not kept in registers through the step)
                    float2 q0 = make_float2(0.f, 0.f), q1 = q0, q2 = q0;
                    float z0 = 0.0f, z1 = 0.0f, z2 = 0.0f;
                    if (nk > kSmallK) {
                        const int i0 = slot_of(0), i1 = slot_of(1), i2 = slot_of(2);
                        q0 = vxy[i0];
                        q1 = vxy[i1];
                        q2 = vxy[i2];
                        z0 = vz[i0];
                        z1 = vz[i1];
                        z2 = vz[i2];
                    }
                    do {
                        const int j = __ffsll((unsigned long long)big) - 1;
                        big &= big - 1;
                        // j is wave-uniform: v_readlane into SGPRs (no LDS round trip)
                        auto rl = [&](float x) { return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(x), j)); };
                        TriRec rb;
                        rb.a0 = rl(q0.x); rb.a1 = rl(q0.y);
                        rb.b0 = rl(q1.x); rb.b1 = rl(q1.y);
                        rb.c0 = rl(q2.x); rb.c1 = rl(q2.y);
                        rb.z0 = rl(z0); rb.z1 = rl(z1); rb.z2 = rl(z2);
                        const uint32_t bpos = (uint32_t)__builtin_amdgcn_readlane((int)pos, j);
                        const int bkx0 = (int)(bpos & 0xffffu), bky0 = (int)(bpos >> 16);
                        const int bnx = (int)((uint32_t)__builtin_amdgcn_readlane((int)nxy, j) & 0xffffu);
                        const int bnk = __builtin_amdgcn_readlane(nk, j);
                        const uint32_t bid = IDPASS ? (uint32_t)__builtin_amdgcn_readlane((int)cidt, j) : 0u;
                        // q / bnx without an integer division: the float quotient is within 1e-3 of q / bnx (q / bnx
                        // is at most the sample rows), so one correction step gives the exact row
                        const float inv_nx = 1.0f / (float)bnx;
                        for (int q = lane; q < bnk; q += kWave) {
                            int iy = (int)(((float)q + 0.5f) * inv_nx), ix = q - iy * bnx;
                            if (ix < 0) { iy--; ix += bnx; } else if (ix >= bnx) { iy++; ix -= bnx; }
                            raster_sample<IDPASS>(rb, bkx0 + ix, bky0 + iy, s, H, sw, sm.zbuf, cid, bid);
                        }
                    } while (big);
                }
                // small triangles: one record per (triangle, sample) into the wave's record ring -- the first
                // sample of every queued triangle, then (rare) the second to fourth of those touching more, one
                // ballot round each; full 64-record batches are flushed after every round (<= 127 pending)
                const bool qd = nk > 0 && nk <= kSmallK;
                const uint64_t bq = __ballot(qd);
#if PCORE_RING_DISCARD
                {  // the record keeps the whole triangle slot word (the flush reads its 27 slot bits); lanes with
                   // nothing to queue write the discard record instead of branching around the store
                    const int slot = qd ? (rec_total + mbcnt64(bq)) & (kRecCap - 1) : kRecCap;
                    ring[slot] = make_uint2(ct, pos);
                    if (IDPASS) ring_id[slot] = cidt;
                }
#else
                if (qd) {  // the record keeps the whole triangle slot word (the flush reads its 27 slot bits)
                    const int slot = (rec_total + mbcnt64(bq)) & (kRecCap - 1);
                    ring[slot] = make_uint2(ct, pos);
                    if (IDPASS) ring_id[slot] = cidt;
                }
#endif
                rec_total += __popcll(bq);
                while (rec_total - rec_done >= kWave) flush(kWave);  // full batches only
                if (__ballot(qd && nk > 1)) {
                    for (int q = 1; q < kSmallK; q++) {
                        const bool qr = qd && nk > q;
                        const uint64_t br = __ballot(qr);
                        if (!br) break;
                        if (qr) {  // sample q of the window, row-major (nx * ny <= 4)
                            const int nx = (int)(nxy & 0xffffu);
                            const int iy = nx == 1 ? q : (nx == 2 ? q >> 1 : 0), ix = q - iy * nx;
                            const int slot = (rec_total + mbcnt64(br)) & (kRecCap - 1);
                            ring[slot] = make_uint2(ct, pos + (uint32_t)ix + ((uint32_t)iy << 16));
                            if (IDPASS) ring_id[slot] = cidt;
                        }
                        rec_total += __popcll(br);
                        while (rec_total - rec_done >= kWave) flush(kWave);
                    }
                }
            }
            fp.mark(2);
        };
        float4 cvA = vq[lane], cvB;
        uint32_t ctA = tp[lane], ctB, cidA, cidB;
        cidA = IDPASS ? op[lane] : 0u;
#if PCORE_STEP_UNROLL
        for (int step = sd.x; step < sd.y; step += 2) {
            run_step(step, cvA, ctA, cidA, cvB, ctB, cidB);
            if (step + 1 < sd.y) run_step(step + 1, cvB, ctB, cidB, cvA, ctA, cidA);
        }
#else
        for (int step = sd.x; step < sd.y; step++) {
            run_step(step, cvA, ctA, cidA, cvB, ctB, cidB);
            cvA = cvB; ctA = ctB; cidA = cidB;
        }
#endif
    }
    if (rec_total > rec_done) flush(rec_total - rec_done);
}

// Conservative sample window of a pose ("Pose windows").  Lanes 0-7 of every wave project the
// corners of the model's bounding box with the vertex stage's own arithmetic; the window is their screen
// box widened by a bound on the float error of any vertex's projection, mapped to samples through the
// bounds of vertex_window (every triangle window lies inside).  The whole sampled image when the box is
// not finite or comes within 5 % of its depth magnitude of the camera plane.  Wave-uniform; every wave of
// the workgroup computes the same window.
__device__ SampleWin pose_window(const FusedArgs& a, int model, const float (&m)[12], int s) {
    const SampleWin whole = {0, 0, a.ws, a.hs, 0};
    const float4 lo = a.model_box[2 * model], hi = a.model_box[2 * model + 1];
    const int c = lane_id() & 7;
    const float x = (c & 1) ? hi.x : lo.x, y = (c & 2) ? hi.y : lo.y, z = (c & 4) ? hi.z : lo.z;
    const float Wf = (float)a.width, Hf = (float)a.height;
    const float lx = row4(m[0], m[1], m[2], m[3], x, y, z);
    const float ly = row4(m[4], m[5], m[6], m[7], x, y, z);
    const float lz = row4(m[8], m[9], m[10], m[11], x, y, z);
    const float px = row4(a.p00, a.p01, a.p02, a.p03, lx, ly, lz);
    const float py = row4(a.p10, a.p11, a.p12, a.p13, lx, ly, lz);
    const float sx = px / lz * Wf / 2.0f + Wf / 2.0f;
    const float sy = py / lz * Hf / 2.0f + Hf / 2.0f;
    const bool bad = !(fabsf(sx) < 1.0e7f) || !(fabsf(sy) < 1.0e7f) || !(lz > 0.0f);  // also NaN
    float lzmin = lz, sx0 = sx, sx1 = sx, sy0 = sy, sy1 = sy;
#pragma unroll
    for (int off = 1; off < 8; off <<= 1) {
        lzmin = fminf(lzmin, __shfl_xor(lzmin, off));
        sx0 = fminf(sx0, __shfl_xor(sx0, off));
        sx1 = fmaxf(sx1, __shfl_xor(sx1, off));
        sy0 = fminf(sy0, __shfl_xor(sy0, off));
        sy1 = fmaxf(sy1, __shfl_xor(sy1, off));
    }
    auto uni = [](float v) { return __int_as_float(__builtin_amdgcn_readfirstlane(__float_as_int(v))); };
    lzmin = uni(lzmin); sx0 = uni(sx0); sx1 = uni(sx1); sy0 = uni(sy0); sy1 = uni(sy1);
    if ((__ballot(bad) & 0xffull) || lo.w == 0.0f) return whole;
    // magnitude of the terms of each camera row over the box (bounds the rounding of any vertex's row)
    const float ax = fmaxf(fabsf(lo.x), fabsf(hi.x)), ay = fmaxf(fabsf(lo.y), fabsf(hi.y));
    const float az = fmaxf(fabsf(lo.z), fabsf(hi.z));
    const float Bx = fabsf(m[0]) * ax + fabsf(m[1]) * ay + fabsf(m[2]) * az + fabsf(m[3]);
    const float By = fabsf(m[4]) * ax + fabsf(m[5]) * ay + fabsf(m[6]) * az + fabsf(m[7]);
    const float Bz = fabsf(m[8]) * ax + fabsf(m[9]) * ay + fabsf(m[10]) * az + fabsf(m[11]);
    if (!(lzmin > 0.05f * Bz)) return whole;
    // |error of sx| <= (W/2) (Pbx / lzmin) eps (8 + 4 Bz / lzmin) + 4 eps (|sx| + W), Bz / lzmin <= 20
    const float eps = 5.9604645e-8f;
    const float Pbx = fabsf(a.p00) * Bx + fabsf(a.p01) * By + fabsf(a.p02) * Bz + fabsf(a.p03);
    const float Pby = fabsf(a.p10) * Bx + fabsf(a.p11) * By + fabsf(a.p12) * Bz + fabsf(a.p13);
    const float mgx = 2.0f + 256.0f * eps * (0.5f * Wf) * Pbx / lzmin + 8.0f * eps * (fmaxf(fabsf(sx0), fabsf(sx1)) + Wf);
    const float mgy = 2.0f + 256.0f * eps * (0.5f * Hf) * Pby / lzmin + 8.0f * eps * (fmaxf(fabsf(sy0), fabsf(sy1)) + Hf);
    if (!(mgx < 1.0e6f) || !(mgy < 1.0e6f)) return whole;
    const float xlo = sx0 - mgx, xhi = sx1 + mgx, ylo = sy0 - mgy, yhi = sy1 + mgy;
    // vertex_window: lo.x >= (sx - 0.5) / s, hi.x <= sx / s; lo.y >= (H - 1 - sy) / s, hi.y <= (H - 0.5 - sy) / s
    const float sf = (float)s;
    const int X0 = max(0, (int)floorf((xlo - 1.0f) / sf)), X1 = min(a.ws - 1, (int)floorf(xhi / sf));
    const int Y0 = max(0, (int)floorf((Hf - 1.0f - yhi) / sf)), Y1 = min(a.hs - 1, (int)floorf((Hf - ylo) / sf));
    // Every vertex's computed z is at least the corners' minimum less the rounding of two dot products
    // (<= 6 eps Bz); the margin 1e-5 Bz covers that.  |x|, |y| after the projection are below Pbx, Pby.
    const bool fastdiv = lzmin - 1.0e-5f * Bz >= 1.0f && Bz < 0x1p40f && Pbx < 0x1p40f && Pby < 0x1p40f;
    return SampleWin{X0, Y0, max(0, X1 - X0 + 1), max(0, Y1 - Y0 + 1), fastdiv ? 1 : 0};
}

// One pose of stage COST on the workgroup's LDS tile (sw.nx * sw.ny <= tile capacity).
// select_kernel's per-pose key (search_env.cpp:1987-2051: int conversion, the |target - source| < 30 filter, cost
// -1 / -2 / INT_MAX excluded): ((cost ^ 0x80000000) << 31) | global index, or PCORE_KEY_NONE_DEV
__device__ __forceinline__ int64_t select_key(float rc, float oc, int m, int num_models, int64_t gidx) {
    const int32_t target = cvt_i32_x86(rc);
    const int32_t source = cvt_i32_x86(oc);
    const int32_t cost = (target < 0) ? -1 : cvt_i32_x86(rc + oc);
    const int32_t adiff = iabs_wrap(target, source);
    const bool ok = !(cost == -1 || cost == -2) && adiff < 30 && cost != INT_MAX && m >= 0 && m < num_models;
    if (!ok) return PCORE_KEY_NONE_DEV;
    const uint64_t hi = (uint64_t)((uint32_t)cost ^ 0x80000000u);
    return (int64_t)((hi << 31) | ((uint64_t)gidx & 0x7fffffffull));
}

// The window is processed in chunks of at most `cap` samples (the LDS tile): one chunk -- the window -- for every
// pose the tile holds; otherwise row bands of whole window rows (blocks of columns when one row exceeds the tile),
// each rasterised over the full stream walk with triangle windows clipped to the chunk.  The costs are functions of
// the chunks' integer counts and of the explained bitmap, which accumulate across chunks, so they do not depend on
// the chunking (the overflow launch that scored such poses before round 4 took a whole-image tile instead).
template <int STRIDE, bool COLOUR>
__device__ __forceinline__ void fused_pose(const FusedArgs& a, const FusedSmem& sm, int pose, const SampleWin& pw,
                                           int cap) {
    const int tid = threadIdx.x;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int lane = tid & 63;
    const int s = STRIDE > 0 ? STRIDE : a.stride;
    const int ws = a.ws, nsamp = a.ws * a.hs;

    for (int i = tid; i < a.bitmap_words; i += kThreads) sm.bitmap[i] = 0u;
    if (tid < 4) sm.counters[tid] = 0;
    if (a.dbg_zs)  // debug z-samples: the samples outside the window stay 0
        for (int i = tid; i < nsamp; i += kThreads) a.dbg_zs[(size_t)pose * nsamp + i] = 0;

    const bool use_seg = a.pose_label != nullptr;
    const int32_t pl = use_seg ? a.pose_label[pose] : 0;
    FProf fp;
    // counts accumulated over the chunks (wave-uniform)
    int wave_bad = 0, wave_pts = 0;
    int32_t* cid = nullptr;
    if constexpr (COLOUR) cid = a.cid + (size_t)pose * nsamp;
    auto chunk = [&](const SampleWin& sw) __attribute__((always_inline)) {
    const int tn = sw.nx * sw.ny;  // samples of the chunk (tile)
    for (int i = tid; i < tn; i += kThreads) sm.zbuf[i] = INT_MAX;
    if (sw.fastdiv) raster_phase<STRIDE, false, 1>(a, sm, pose, sw, nullptr, fp);
    else raster_phase<STRIDE, false, 0>(a, sm, pose, sw, nullptr, fp);
    fp.mark(2);
    __syncthreads();
    fp.mark(4);
    if constexpr (COLOUR) {
        // colour id pass (cost_type 1): which triangle left each sample's minimum depth (tile-local index)
        for (int i = tid; i < tn; i += kThreads) cid[i] = INT_MAX;
        __syncthreads();
        raster_phase<STRIDE, true>(a, sm, pose, sw, cid, fp);
        __syncthreads();
    }

    // ---------------- phase 2: occlusion, unprojection, 1-NN, counts ----------------
    // per-wave point queue in the (now free) triangle ring: (tile index, kx | ky << 16) pairs
    int32_t* queue = reinterpret_cast<int32_t*>(sm.ring + wave * kRecStride);  // <= 127 pairs (kRecCap >= 128)
    int qcount = 0;
    const int grid_id = use_seg ? pl : a.num_grids;
    const bool grid_ok = use_seg ? (pl >= 0 && pl < a.num_grids) : true;
    LabelGrid g;
    if (grid_ok) g = a.grids[grid_id];
    const float r_eff = sqrtf(a.r2) * 1.0001f + 1e-7f;
    int my_bad = 0;

    auto process_points = [&](int count) {
        wave_sync();
        for (int base = 0; base < count; base += kWave) {
            const int j = base + lane;
            bool is_bad = false;
            if (j < count) {
                const int k = queue[2 * j];
                const int kxy = queue[2 * j + 1];
                const int32_t Z = sm.zbuf[k];
                const int kx = kxy & 0xffff, ky = kxy >> 16;
                // compute_point_clouds.cuh:14-22 with depth_factor (cm -> m)
                const float zp = (float)Z / a.depth_factor;
                const float xp = ((float)(kx * s) - a.cx) / a.fx * zp;
                const float yp = ((float)(ky * s) - a.cy) / a.fy * zp;
                float best = INFINITY;
                int bidx = 0x7fffffff;
                if (grid_ok) {
                    const float rc = r_eff * g.inv_c;
                    const float fx0 = (xp - g.ox) * g.inv_c, fy0 = (yp - g.oy) * g.inv_c, fz0 = (zp - g.oz) * g.inv_c;
                    const float lx = fx0 - rc, hx = fx0 + rc, ly = fy0 - rc, hy = fy0 + rc, lz = fz0 - rc, hz = fz0 + rc;
                    if (hx >= 0.0f && lx < (float)g.nx && hy >= 0.0f && ly < (float)g.ny && hz >= 0.0f && lz < (float)g.nz) {
                        const int ix0 = (int)floorf(fmaxf(lx, 0.0f)), ix1 = min(g.nx - 1, (int)floorf(hx));
                        const int iy0 = (int)floorf(fmaxf(ly, 0.0f)), iy1 = min(g.ny - 1, (int)floorf(hy));
                        const int iz0 = (int)floorf(fmaxf(lz, 0.0f)), iz1 = min(g.nz - 1, (int)floorf(hz));
                        // the radius box spans <= 2 cells per axis (cell >= 2.02 r): the <= 2 cells along x of one
                        // (y, z) row are adjacent in the CSR order, so their points form ONE range -- <= 4 ranges,
                        // fetched with independent loads, then their points as one flattened sequence four at a time
                        // (clamped loads issued together); the (distance, index) minimum does not depend on the order
                        int cb[4], ce[4];
#pragma unroll
                        for (int q = 0; q < 4; q++) {
                            const int iy = iy0 + (q & 1), iz = iz0 + (q >> 1);
                            const bool ok = iy <= iy1 && iz <= iz1;
                            const int c = g.cell_base + (iz * g.ny + iy) * g.nx + ix0;
                            cb[q] = ok ? a.cell_start[c] : 0;
                            ce[q] = ok ? a.cell_start[c + 1 + (ix1 - ix0)] : 0;
                        }
                        // the <= 4 ranges as one flattened candidate sequence, four at a time: the wave loops over its
                        // lanes' largest total instead of the sum of the per-range maxima
                        const int l0 = ce[0] - cb[0], l1 = l0 + (ce[1] - cb[1]), l2 = l1 + (ce[2] - cb[2]);
                        const int ltot = l2 + (ce[3] - cb[3]);
                        for (int k0 = 0; k0 < ltot; k0 += 4) {
                            float4 o[4];
#pragma unroll
                            for (int u = 0; u < 4; u++) {
                                const int k = min(k0 + u, ltot - 1);
                                const int pi = k < l0 ? cb[0] + k : k < l1 ? cb[1] + (k - l0)
                                             : k < l2 ? cb[2] + (k - l1) : cb[3] + (k - l2);
                                o[u] = a.grid_pts[pi];
                            }
#pragma unroll
                            for (int u = 0; u < 4; u++) {
                                const float dx = xp - o[u].x, dy = yp - o[u].y, dz = zp - o[u].z;
                                const float d = dx * dx + dy * dy + dz * dz;
                                const int oi = __float_as_int(o[u].w);
                                const bool take = k0 + u < ltot && (d < best || (d == best && oi < bidx));
                                best = take ? d : best;
                                bidx = take ? oi : bidx;
                            }
                        }
                    }
                }
                // compute_costs.cuh:201-270 (cost types 0 / 2: explained marking; type 1: colour gate first)
                if (best > a.r2) {
                    is_bad = true;
                } else if (bidx != 0x7fffffff) {
                    bool expl = true;
                    if constexpr (COLOUR) {
                        const int id = cid[k];
                        const float4 lr = a.tri_lab[id == INT_MAX ? 0 : id];  // a valid sample has an id
                        const float4 lo = a.obs_lab[bidx];
                        const double cd = colour::colour_distance(lo.x, lo.y, lo.z, lr.x, lr.y, lr.z);
                        expl = !(cd > (double)a.colour_thr);
                    }
                    if (expl) atomicOr(&sm.bitmap[bidx >> 5], 1u << (bidx & 31));
                    else is_bad = true;
                }
            }
            my_bad += is_bad ? 1 : 0;
        }
        wave_sync();
    };

    // tile index k -> (ix, iy) without an integer division: (k + 0.5) / nx in float is within 1e-3 of the
    // quotient (k < 2^14), so one correction step gives the exact row
    const float inv_nx = tn > 0 ? 1.0f / (float)sw.nx : 0.0f;
    for (int base = wave * kWave; base < tn; base += kThreads) {
        const int k = base + lane;
        bool valid = false;
        int kx = 0, ky = 0;
#if PCORE_DEBUG_SKIP_RT
        if (k < tn && !(a.dbg_skip & 4)) {
#else
        if (k < tn) {
#endif
            int iy = (int)(((float)k + 0.5f) * inv_nx), ix = k - iy * sw.nx;
            if (ix < 0) { iy--; ix += sw.nx; } else if (ix >= sw.nx) { iy++; ix -= sw.nx; }
            kx = sw.x0 + ix;
            ky = sw.y0 + iy;
            const int gk = ky * ws + kx;
            const int32_t z = sm.zbuf[k];
            // no fragment: Z = 0 whatever the source (the sampled source is read only under a fragment)
            const int32_t zf = z == INT_MAX ? 0
                                            : occlusion_rule(z, a.src_s[gk], use_seg ? (int)a.lab_s[gk] : 0, use_seg,
                                                             pl, a.occlusion_threshold);
            if (zf != z) sm.zbuf[k] = zf;
            if (a.dbg_zs) a.dbg_zs[(size_t)pose * nsamp + gk] = zf;
            valid = zf > 0;  // depth_to_mask, compute_point_clouds.cuh:64
        }
        const uint64_t bv = __ballot(valid);
        if (valid) {
            const int q = qcount + mbcnt64(bv);
            queue[2 * q] = k;
            queue[2 * q + 1] = kx | (ky << 16);
        }
        qcount += __popcll(bv);
        wave_pts += __popcll(bv);
        if (qcount >= kWave) {
            process_points(qcount);
            qcount = 0;
        }
    }
    if (qcount > 0) process_points(qcount);
    fp.mark(5);
    for (int off = 32; off > 0; off >>= 1) my_bad += __shfl_xor(my_bad, off);
    wave_bad += __builtin_amdgcn_readfirstlane(my_bad);
    };
    if (pw.nx * pw.ny <= cap) {
        chunk(pw);  // the window fits the tile (the common case: its own copy of the code, no loop state)
    } else {
        const int cw = min(pw.nx, cap), ch = max(1, cap / max(cw, 1));  // chunk columns / rows
        for (int r0 = 0; r0 < pw.ny; r0 += ch)
            for (int c0 = 0; c0 < pw.nx; c0 += cw) {
                if (r0 > 0 || c0 > 0) __syncthreads();  // the previous chunk's points are processed
                chunk(SampleWin{pw.x0 + c0, pw.y0 + r0, min(cw, pw.nx - c0), min(ch, pw.ny - r0), pw.fastdiv});
            }
    }
    // per-wave totals
    __syncthreads();  // all points counted / marked
    if (lane == 0) atomicAdd(&sm.counters[0], wave_bad);
    // number of points = number of valid samples (counted per wave above)
    int my_expl = 0;
    for (int w = tid; w < a.bitmap_words; w += kThreads) my_expl += __popc(sm.bitmap[w]);
    for (int off = 32; off > 0; off >>= 1) my_expl += __shfl_xor(my_expl, off);
    if (lane == 0) {
        atomicAdd(&sm.counters[1], my_expl);
        atomicAdd(&sm.counters[2], wave_pts);
    }
    __syncthreads();

    // ---------------- phase 3: costs (compute_costs.cuh:362-446), exact float order ----------------
    if (tid == 0) {
        const float num = (float)sm.counters[2];
        const float badf = (float)sm.counters[0];
        const float rendered_explained = num - badf;
        float rc = (num == 0.0f) ? -1.0f : badf / num;
        rc = (rc == -1.0f) ? -1.0f : rc * 100.0f;
        a.out_rc[pose] = rc;
        float ocw = 0.0f;  // the observed cost as stored
        if (a.calc_obs) {
            const float expl = (float)sm.counters[1];
            const float tot = a.pose_obs_total[pose];
            a.out_diff[pose] = rendered_explained - expl;
            float oc = tot - expl;
            oc = oc / tot;
            ocw = oc * 100.0f;
            a.out_oc[pose] = ocw;
        } else {
            if (a.out_oc) a.out_oc[pose] = 0.0f;
            if (a.out_diff) a.out_diff[pose] = 0.0f;
        }
        if (a.sel_keys) {
            const int m = a.pose_model[pose];
            const int64_t key = select_key(rc, ocw, m, a.sel_models, a.sel_base + pose);
            if (key != PCORE_KEY_NONE_DEV) atomicMin((unsigned long long*)&a.sel_keys[m], (unsigned long long)key);
        }
    }
    fp.mark(6);
    fp.flush();
}

__device__ __forceinline__ void load_pose_rows(const float* poses, int pose, float (&m)[12]) {
    const float* P = poses + (size_t)16 * pose;
#pragma unroll
    for (int i = 0; i < 12; i++) m[i] = P[i];
}

// Window launch: one workgroup per pose, LDS tile of a.tcap samples.  A pose whose window exceeds the tile is
// processed in chunks of the tile (fused_pose).
#ifdef PCORE_WG_TIMING
// measurement build only (tools/wg_timeline.py): wall clock (100 MHz) at the start and end of every
// fused_cost_kernel workgroup, indexed by pose
__device__ unsigned long long pcore_wg_clock[2 * 1048576];
extern "C" int pcore_debug_wg_clock(unsigned long long* host, int n) {
    return (int)hipMemcpyFromSymbol(host, HIP_SYMBOL(pcore_wg_clock), sizeof(unsigned long long) * 2 * (size_t)n);
}
#endif

// register budget of the fused kernel: as many waves per SIMD as the most-occupied tile tier has workgroups per CU
// (6: <= 80 VGPRs; without the bound the certified fragment depth takes 82 and the kernel drops to 5 waves).  The
// colour-cost kernel (two raster passes, CIEDE2000) is left unbounded: under 80 VGPRs it spills.
#ifndef PCORE_FUSED_WAVES_PER_EU
#define PCORE_FUSED_WAVES_PER_EU PCORE_TIER_MAX
#endif
template <int STRIDE, bool COLOUR = false>
__global__ void __launch_bounds__(kThreads) __attribute__((amdgpu_waves_per_eu(COLOUR ? 1 : PCORE_FUSED_WAVES_PER_EU)))
fused_cost_kernel(FusedArgs a) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem_raw[];
    const int pose = blockIdx.x;
#ifdef PCORE_WG_TIMING
    if (threadIdx.x == 0) pcore_wg_clock[2 * pose] = wall_clock64();
    struct End {
        int pose;
        __device__ ~End() {
            __syncthreads();
            if (threadIdx.x == 0) pcore_wg_clock[2 * pose + 1] = wall_clock64();
        }
    } end_clock{pose};
#endif
    const FusedSmem sm = carve_smem(smem_raw, a.tcap, a.bitmap_words, COLOUR);
    // the pose window, by wave 0 only (every wave would compute the same one), shared through LDS
    if (threadIdx.x < kWave) {
        const int model = a.pose_model[pose];
        SampleWin w = {0, 0, 0, 0, 0};  // invalid model: nothing is rendered
        if (model >= 0 && model < a.num_models) {
            float m[12];
            load_pose_rows(a.poses, pose, m);
            w = pose_window(a, model, m, STRIDE > 0 ? STRIDE : a.stride);
        }
        if (threadIdx.x == 0) {
            sm.counters[4] = w.x0;
            sm.counters[5] = w.y0;
            sm.counters[6] = w.nx;
            sm.counters[7] = w.ny;
            sm.counters[8] = w.fastdiv;
        }
    }
    __syncthreads();
    const SampleWin sw = {__builtin_amdgcn_readfirstlane(sm.counters[4]), __builtin_amdgcn_readfirstlane(sm.counters[5]),
                          __builtin_amdgcn_readfirstlane(sm.counters[6]), __builtin_amdgcn_readfirstlane(sm.counters[7]),
                          __builtin_amdgcn_readfirstlane(sm.counters[8])};
    const int tn = sw.nx * sw.ny;
    // Tile feedback, double-buffered by launch parity: every workgroup counts its window into this launch's
    // histogram (and, when chunked, the chunked-pose count) with atomics whose result it does not wait for;
    // workgroup 0 publishes the previous launch's counts -- complete, since launches on a stream run in order -- to
    // mapped host memory for the next call's tile choice and clears them for the launch after this one.  (A
    // last-workgroup-done publish instead made every workgroup wait on a returning atomic at exit: C2 -6 %.)
    if (threadIdx.x == 0) {
        const int par = a.fb_par;
        int b = 0;
#pragma unroll
        for (int t = 0; t < kTileTiers; t++) b += tn > a.hist_edge[t] ? 1 : 0;
        atomicAdd(&a.win_hist[par * (kTileTiers + 1) + b], 1);
        if (tn > a.tcap) atomicAdd(&a.fb_ctr[par], 1);
        if (blockIdx.x == 0 && a.fb_host) {
            const int o = (1 - par) * (kTileTiers + 1);
            for (int k = 0; k <= kTileTiers; k++) a.fb_host[k] = atomicExch(&a.win_hist[o + k], 0);
            a.fb_host[kTileTiers + 1] = atomicExch(&a.fb_ctr[1 - par], 0);
            // no system fence: the host may read a torn set, which only steers a later tile choice
            a.fb_host[kTileTiers + 2] = a.fb_seq - 1;  // the launch these counts belong to
        }
    }
    fused_pose<STRIDE, COLOUR>(a, sm, pose, sw, a.tcap);
}

// Window probe: the tier histogram of a batch's pose windows, for the tile choice of a context that has no
// published feedback yet (set_fused_tiles).  One wave per pose at a time (pose_window's corner lanes), poses strided
// over a bounded grid; waves count in registers, workgroups in LDS, and each workgroup adds its bins once (one
// address per bin: a per-pose atomic serialised, 270 us for 50 k poses).
constexpr int kProbeBlocks = 2048;
__global__ void __launch_bounds__(kThreads) window_probe_kernel(FusedArgs a, int32_t* hist) {
    constexpr int kWaves = kThreads / kWave;
    int cnt[kTileTiers + 1] = {};
    for (int pose = blockIdx.x * kWaves + (int)(threadIdx.x / kWave); pose < a.num_poses;
         pose += gridDim.x * kWaves) {  // wave-uniform
        const int model = a.pose_model[pose];
        int tn = 0;
        if (model >= 0 && model < a.num_models) {
            float m[12];
            load_pose_rows(a.poses, pose, m);
            const SampleWin w = pose_window(a, model, m, a.stride);
            tn = w.nx * w.ny;
        }
        int b = 0;
#pragma unroll
        for (int t = 0; t < kTileTiers; t++) b += tn > a.hist_edge[t] ? 1 : 0;
#pragma unroll
        for (int k = 0; k <= kTileTiers; k++) cnt[k] += b == k ? 1 : 0;
    }
    __shared__ int32_t wg_cnt[kTileTiers + 1];
    if (threadIdx.x <= kTileTiers) wg_cnt[threadIdx.x] = 0;
    __syncthreads();
    if (lane_id() == 0) {
#pragma unroll
        for (int k = 0; k <= kTileTiers; k++)
            if (cnt[k]) atomicAdd(&wg_cnt[k], cnt[k]);
    }
    __syncthreads();
    if (threadIdx.x <= kTileTiers && wg_cnt[threadIdx.x]) atomicAdd(&hist[threadIdx.x], wg_cnt[threadIdx.x]);
}

hipError_t launch_window_probe(const FusedArgs& a, int32_t* hist, hipStream_t s) {
    if (a.num_poses <= 0) return hipSuccess;
    const int per_wg = kThreads / kWave;
    const int blocks = std::min(kProbeBlocks, (a.num_poses + per_wg - 1) / per_wg);
    hipLaunchKernelGGL(window_probe_kernel, dim3(blocks), dim3(kThreads), 0, s, a, hist);
    return hipGetLastError();
}

// Stage CLOUD into per-pose scratch slots (the GICP source clouds): sampled raster, source occlusion,
// then the reference's compaction order (row-major samples, compute_point_clouds.cuh:290-346).
template <int STRIDE>
__global__ void __launch_bounds__(kThreads) render_cloud_kernel(FusedArgs a) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem_raw[];
    __shared__ int wsum[kWaves];
    __shared__ int carry_s;
    const int pose = blockIdx.x;
    const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
    const int s = STRIDE > 0 ? STRIDE : a.stride;
    const int ws = a.ws, nsamp = a.ws * a.hs;
    const int cap = a.tcap > 0 && a.tcap < nsamp ? a.tcap : nsamp;  // the LDS tile (samples)
    const FusedSmem sm = carve_smem(smem_raw, cap, 0);
    const int model = a.pose_model[pose];
    SampleWin sw = {0, 0, 0, 0, 0};
    if (model >= 0 && model < a.num_models) {
        float m[12];
        load_pose_rows(a.poses, pose, m);
        sw = pose_window(a, model, m, s);
    }
    if (tid == 0) carry_s = 0;
    const bool use_seg = a.pose_label != nullptr;
    const int32_t pl = use_seg ? a.pose_label[pose] : 0;
    FProf fp;
    float4* out = a.cloud_out + (size_t)pose * a.cloud_cap;
    // one chunk of the window (fused_pose's chunking): raster into the tile, then the chunk's valid samples appended
    // in row-major order -- row bands of whole window rows (column blocks when a row exceeds the tile) keep the
    // reference's row-major compaction order (no valid sample lies outside the window)
    auto chunk = [&](const SampleWin& cw) __attribute__((always_inline)) {
        const int tn = cw.nx * cw.ny;
        for (int i = tid; i < tn; i += kThreads) sm.zbuf[i] = INT_MAX;
        if (cw.fastdiv) raster_phase<STRIDE, false, 1>(a, sm, pose, cw, nullptr, fp);
        else raster_phase<STRIDE, false, 0>(a, sm, pose, cw, nullptr, fp);
        __syncthreads();
        const float inv_nx = tn > 0 ? 1.0f / (float)cw.nx : 0.0f;
        for (int base = 0; base < tn; base += kThreads) {
            const int k = base + tid;
            int32_t zf = 0;
            int kx = 0, ky = 0;
            if (k < tn) {
                int iy = (int)(((float)k + 0.5f) * inv_nx), ix = k - iy * cw.nx;
                if (ix < 0) { iy--; ix += cw.nx; } else if (ix >= cw.nx) { iy++; ix -= cw.nx; }
                kx = cw.x0 + ix;
                ky = cw.y0 + iy;
                const int gk = ky * ws + kx;
                zf = occlusion_rule(sm.zbuf[k], a.src_s[gk], use_seg ? (int)a.lab_s[gk] : 0, use_seg, pl,
                                    a.occlusion_threshold);
            }
            const bool valid = zf > 0;
            const uint64_t b = __ballot(valid);
            if (lane == 0) wsum[wave] = __popcll(b);
            __syncthreads();
            int woff = 0, tot = 0;
            for (int w = 0; w < kWaves; w++) {
                if (w < wave) woff += wsum[w];
                tot += wsum[w];
            }
            const int carry = carry_s;
            if (valid) {
                const int o = carry + woff + mbcnt64(b);
                const float zp = (float)zf / a.depth_factor;
                const float xp = ((float)(kx * s) - a.cx) / a.fx * zp;
                const float yp = ((float)(ky * s) - a.cy) / a.fy * zp;
                if (o < a.cloud_cap) out[o] = make_float4(xp, yp, zp, 0.0f);
            }
            __syncthreads();
            if (tid == 0) carry_s = carry + tot;
            __syncthreads();
        }
    };
    if (sw.nx * sw.ny <= cap) {
        chunk(sw);
    } else {
        const int cw = min(sw.nx, cap), ch = max(1, cap / max(cw, 1));
        for (int r0 = 0; r0 < sw.ny; r0 += ch)
            for (int c0 = 0; c0 < sw.nx; c0 += cw)
                chunk(SampleWin{sw.x0 + c0, sw.y0 + r0, min(cw, sw.nx - c0), min(ch, sw.ny - r0), sw.fastdiv});
    }
    if (tid == 0) a.cloud_count[pose] = carry_s < a.cloud_cap ? carry_s : a.cloud_cap;
    // the source covariances of the cloud this workgroup has just written: pcore_cov.h's rounds of
    // 64 queries, round r on wave r % 4, each wave staging candidates through its own 64-point tile in the vertex ring's
    // LDS (free once the raster is done); the points are read back from the slot (L2, written before the barrier)
    if (a.cloud_cov) {
        __syncthreads();  // every chunk's points are written and carry_s is final
        const int n = carry_s < a.cloud_cap ? carry_s : a.cloud_cap;
        float4* tile = reinterpret_cast<float4*>(sm.vxy) + wave * kCovLanes;
        double* C = a.cloud_cov + (size_t)6 * pose * a.cloud_cap;
        for (int i0 = wave * kCovLanes; i0 < n; i0 += kThreads)
            cov_knn_round<10, true>(out, n, 10, i0, lane, tile, C);
    }
}

hipError_t launch_render_cloud(const FusedArgs& a, hipStream_t s) {
    const int nsamp = a.ws * a.hs;
    const size_t lds = fused_lds_bytes(a.tcap > 0 && a.tcap < nsamp ? a.tcap : nsamp, 0);
    if (a.num_poses <= 0) return hipSuccess;
    if (a.stride == 8)
        hipLaunchKernelGGL(render_cloud_kernel<8>, dim3(a.num_poses), dim3(kThreads), lds, s, a);
    else
        hipLaunchKernelGGL(render_cloud_kernel<0>, dim3(a.num_poses), dim3(kThreads), lds, s, a);
    return hipGetLastError();
}

// The LDS granule (kLdsGranule, pcore_internal.h) comes from the context's DeviceInfo.
int fused_tier_samples(int t, int ws, int hs, int bitmap_words, bool colour, const DeviceInfo& d) {
    const int nsamp = ws * hs;
    const size_t granule = d.lds_granule;
    const size_t per_wg = (d.lds_per_cu / tier_wgs(t)) / granule * granule;
    const size_t fixed = fused_lds_bytes(0, bitmap_words, colour);
    if (per_wg <= fixed + 64) return 0;
    const int cap = (int)((per_wg - fixed) / 4) & ~3;
    return cap >= nsamp ? nsamp : cap;
}

hipError_t launch_fused_cost(const FusedArgs& a0, hipStream_t s) {
    if (a0.num_poses <= 0) return hipSuccess;
    const bool colour = a0.cid != nullptr;
    const int nsamp = a0.ws * a0.hs;
    FusedArgs a = a0;
    if (a.tcap <= 0 || a.tcap > nsamp) a.tcap = nsamp;
    const size_t lds = fused_lds_bytes(a.tcap, a.bitmap_words, colour);
    if (colour)
        hipLaunchKernelGGL((fused_cost_kernel<0, true>), dim3(a.num_poses), dim3(kThreads), lds, s, a);
    else if (a.stride == 8)
        hipLaunchKernelGGL(fused_cost_kernel<8>, dim3(a.num_poses), dim3(kThreads), lds, s, a);
    else
        hipLaunchKernelGGL(fused_cost_kernel<0>, dim3(a.num_poses), dim3(kThreads), lds, s, a);
    return hipGetLastError();
}

// ------------------------------------------------------------------------------------------------
// Stage RENDER (parity): full-resolution z-buffer
// ------------------------------------------------------------------------------------------------

// One thread per (triangle, pose), as render_triangle_multi (image_renderer.cuh:212-321); the per-pixel
// spin-lock is replaced by atomicMin and the black-out by render_finalize_kernel.
__global__ void __launch_bounds__(256) render_full_kernel(const float* tris, int num_tris, const int32_t* tri_lo,
                                                          const int32_t* tri_hi, const float* poses,
                                                          const int32_t* pose_model, int width, int height,
                                                          const float* proj, int32_t* depth) {
    const int pose = blockIdx.y;
    const int t = blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= num_tris) return;
    const int m = pose_model[pose];
    if (!(t >= tri_lo[m] && t < tri_hi[m])) return;
    const float* M = poses + (size_t)16 * pose;
    const float* tp = tris + (size_t)9 * t;
    const float Wf = (float)width, Hf = (float)height;
    float p[3][2], z[3];
#pragma unroll
    for (int k = 0; k < 3; k++) {
        const float x = tp[3 * k], y = tp[3 * k + 1], zz = tp[3 * k + 2];
        const float lx = row4(M[0], M[1], M[2], M[3], x, y, zz);
        const float ly = row4(M[4], M[5], M[6], M[7], x, y, zz);
        const float lz = row4(M[8], M[9], M[10], M[11], x, y, zz);
        const float px = row4(proj[0], proj[1], proj[2], proj[3], lx, ly, lz);
        const float py = row4(proj[4], proj[5], proj[6], proj[7], lx, ly, lz);
        p[k][0] = px / lz * Wf / 2.0f + Wf / 2.0f;
        p[k][1] = py / lz * Hf / 2.0f + Hf / 2.0f;
        z[k] = lz;
    }
    float bmin[2], bmax[2];
    bbox_ref(p, (float)(width - 1), (float)(height - 1), bmin, bmax);
    int lo0, hi0, lo1, hi1;
    if (!loop_bounds(bmin[0], bmax[0], lo0, hi0) || !loop_bounds(bmin[1], bmax[1], lo1, hi1)) return;
    int32_t* img = depth + (size_t)pose * width * height;
    for (int P1 = lo1; P1 <= hi1; P1++)
        for (int P0 = lo0; P0 <= hi0; P0++) {
            int32_t d;
            if (fragment(p[0][0], p[0][1], p[1][0], p[1][1], p[2][0], p[2][1], z[0], z[1], z[2], (float)P0, (float)P1, d))
                atomicMin(&img[P0 + (size_t)(height - 1 - P1) * width], d);
        }
}

// The colour of stage RENDER (render_triangle_multi's red / green / blue planes, image_renderer.cuh:146-196): the
// serial z-test writes a triangle's colour whenever its fragment is strictly nearer, so the pixel keeps the colour
// of the first triangle (lowest index) whose fragment reaches the minimum depth.  A second pass over the same
// fragments keeps, per pixel, the lowest triangle index whose depth equals the z-buffer's minimum.
__global__ void __launch_bounds__(256) render_full_tri_kernel(const float* tris, int num_tris, const int32_t* tri_lo,
                                                              const int32_t* tri_hi, const float* poses,
                                                              const int32_t* pose_model, int width, int height,
                                                              const float* proj, const int32_t* depth,
                                                              int32_t* tri_min) {
    const int pose = blockIdx.y;
    const int t = blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= num_tris) return;
    const int m = pose_model[pose];
    if (!(t >= tri_lo[m] && t < tri_hi[m])) return;
    const float* M = poses + (size_t)16 * pose;
    const float* tp = tris + (size_t)9 * t;
    const float Wf = (float)width, Hf = (float)height;
    float p[3][2], z[3];
#pragma unroll
    for (int k = 0; k < 3; k++) {
        const float x = tp[3 * k], y = tp[3 * k + 1], zz = tp[3 * k + 2];
        const float lx = row4(M[0], M[1], M[2], M[3], x, y, zz);
        const float ly = row4(M[4], M[5], M[6], M[7], x, y, zz);
        const float lz = row4(M[8], M[9], M[10], M[11], x, y, zz);
        const float px = row4(proj[0], proj[1], proj[2], proj[3], lx, ly, lz);
        const float py = row4(proj[4], proj[5], proj[6], proj[7], lx, ly, lz);
        p[k][0] = px / lz * Wf / 2.0f + Wf / 2.0f;
        p[k][1] = py / lz * Hf / 2.0f + Hf / 2.0f;
        z[k] = lz;
    }
    float bmin[2], bmax[2];
    bbox_ref(p, (float)(width - 1), (float)(height - 1), bmin, bmax);
    int lo0, hi0, lo1, hi1;
    if (!loop_bounds(bmin[0], bmax[0], lo0, hi0) || !loop_bounds(bmin[1], bmax[1], lo1, hi1)) return;
    const size_t base = (size_t)pose * width * height;
    for (int P1 = lo1; P1 <= hi1; P1++)
        for (int P0 = lo0; P0 <= hi0; P0++) {
            int32_t d;
            if (fragment(p[0][0], p[0][1], p[1][0], p[1][1], p[2][0], p[2][1], z[0], z[1], z[2], (float)P0, (float)P1, d)) {
                const size_t i = base + P0 + (size_t)(height - 1 - P1) * width;
                if (d == depth[i]) atomicMin(&tri_min[i], t);
            }
        }
}

// Source occlusion + max2zero on the full z-buffer (the a6' rule); with `rgb` (packed r | g << 8
// | b << 16 per triangle) also the colour planes (red, green, blue planes of N x H x W each, the reference's
// result_color): the nearest triangle's colour, black where no fragment landed or the source occludes the render.
__global__ void render_finalize_kernel(int32_t* depth, const int32_t* src_depth, const uint8_t* src_mask,
                                       const int32_t* pose_label, int width, int height, float occlusion_threshold,
                                       const int32_t* tri_min, const uint32_t* rgb, uint8_t* color, int num_poses) {
    const int pose = blockIdx.y;
    const size_t npx = (size_t)width * height;
    const bool use_seg = pose_label != nullptr;
    const int32_t pl = use_seg ? pose_label[pose] : 0;
    int32_t* img = depth + npx * pose;
    const size_t plane = npx * (size_t)num_poses;
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < npx; i += (size_t)gridDim.x * blockDim.x) {
        const int32_t dmin = img[i];
        const int32_t z = occlusion_rule(dmin, src_depth[i], use_seg ? (int)src_mask[i] : 0, use_seg, pl, occlusion_threshold);
        img[i] = z;
        if (color) {
            // blocked fragments end at INT_MAX (0 after max2zero) and a blocked dmin is > src > 0, so z != dmin
            const bool shown = dmin != INT_MAX && z == dmin;
            const uint32_t c = shown ? rgb[tri_min[npx * pose + i]] : 0u;
            uint8_t* px = color + npx * pose + i;
            px[0] = (uint8_t)(c & 0xff);
            px[plane] = (uint8_t)((c >> 8) & 0xff);
            px[2 * plane] = (uint8_t)((c >> 16) & 0xff);
        }
    }
}

__global__ void fill_i32_kernel(int32_t* p, int32_t v, size_t n) {
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) p[i] = v;
}

hipError_t launch_fill_i32(int32_t* p, int32_t v, size_t n, hipStream_t s) {
    if (n == 0) return hipSuccess;
    size_t blocks = (n + 255) / 256;
    if (blocks > 4096) blocks = 4096;
    hipLaunchKernelGGL(fill_i32_kernel, dim3((unsigned)blocks), dim3(256), 0, s, p, v, n);
    return hipGetLastError();
}

hipError_t launch_render_full(const float* tris, int num_tris, const int32_t* tri_lo, const int32_t* tri_hi,
                              const float* poses, const int32_t* pose_model, int num_poses, int width, int height,
                              const float* proj, int32_t* depth, hipStream_t s) {
    if (num_poses <= 0 || num_tris <= 0) return hipSuccess;
    dim3 grid((num_tris + 255) / 256, num_poses);
    hipLaunchKernelGGL(render_full_kernel, grid, dim3(256), 0, s, tris, num_tris, tri_lo, tri_hi, poses, pose_model,
                       width, height, proj, depth);
    return hipGetLastError();
}

hipError_t launch_render_full_tri(const float* tris, int num_tris, const int32_t* tri_lo, const int32_t* tri_hi,
                                  const float* poses, const int32_t* pose_model, int num_poses, int width, int height,
                                  const float* proj, const int32_t* depth, int32_t* tri_min, hipStream_t s) {
    if (num_poses <= 0 || num_tris <= 0) return hipSuccess;
    dim3 grid((num_tris + 255) / 256, num_poses);
    hipLaunchKernelGGL(render_full_tri_kernel, grid, dim3(256), 0, s, tris, num_tris, tri_lo, tri_hi, poses,
                       pose_model, width, height, proj, depth, tri_min);
    return hipGetLastError();
}

hipError_t launch_render_finalize(int32_t* depth, const int32_t* src_depth, const uint8_t* src_mask,
                                  const int32_t* pose_label, int num_poses, int width, int height,
                                  float occlusion_threshold, hipStream_t s, const int32_t* tri_min,
                                  const uint32_t* rgb, uint8_t* color) {
    if (num_poses <= 0) return hipSuccess;
    const size_t npx = (size_t)width * height;
    unsigned bx = (unsigned)((npx + 255) / 256);
    if (bx > 256) bx = 256;
    hipLaunchKernelGGL(render_finalize_kernel, dim3(bx, num_poses), dim3(256), 0, s, depth, src_depth, src_mask,
                       pose_label, width, height, occlusion_threshold, tri_min, rgb, color, num_poses);
    return hipGetLastError();
}

// ------------------------------------------------------------------------------------------------
// Stage CLOUD / depth2cloud_global (compute_point_clouds.cuh:37-184, 265-346)
// ------------------------------------------------------------------------------------------------

__device__ __forceinline__ bool cloud_valid(const int32_t* depth, const uint8_t* label_mask, size_t idx, int x, int y,
                                            const CloudBounds& cb) {
    if (depth[idx] <= 0) return false;                                 // :64, :123
    if (label_mask != nullptr && label_mask[idx] <= 0) return false;  // :74, :127
    if (cb.on) {
        // transform_point with camera_transform (:14-35): camera point, then R p (left to right) + t
        const float zc = (float)depth[idx] / cb.depth_factor;
        const float xc = ((float)x - cb.cx) / cb.fx * zc;
        const float yc = ((float)y - cb.cy) / cb.fy * zc;
        float w[3];
#pragma unroll
        for (int r = 0; r < 3; r++) {
            w[r] = cb.m[4 * r] * xc + cb.m[4 * r + 1] * yc + cb.m[4 * r + 2] * zc;
            w[r] = w[r] + cb.m[4 * r + 3];
        }
        if (w[0] > cb.b[0] || w[0] < cb.b[1]) return false;  // :86-88, :130-132
        if (w[1] > cb.b[2] || w[1] < cb.b[3]) return false;
        if (w[2] > cb.b[4] || w[2] < cb.b[5]) return false;
    }
    return true;
}

// one block per image: number of valid stride samples
__global__ void cloud_count_kernel(const int32_t* depth, int width, int height, int stride, const uint8_t* label_mask,
                                   CloudBounds cb, int32_t* counts) {
    const int n = blockIdx.x;
    const int ws = (width + stride - 1) / stride, hs = (height + stride - 1) / stride;
    const size_t npx = (size_t)width * height;
    int c = 0;
    for (int k = threadIdx.x; k < ws * hs; k += blockDim.x) {
        const int ky = k / ws, kx = k - ky * ws;
        c += cloud_valid(depth, label_mask, npx * n + (size_t)(kx * stride) + (size_t)(ky * stride) * width,
                         kx * stride, ky * stride, cb) ? 1 : 0;
    }
    for (int off = 32; off > 0; off >>= 1) c += __shfl_xor(c, off);
    __shared__ int part[16];
    if ((threadIdx.x & 63) == 0) part[threadIdx.x >> 6] = c;
    __syncthreads();
    if (threadIdx.x == 0) {
        int t = 0;
        for (int w = 0; w < (int)(blockDim.x >> 6); w++) t += part[w];
        counts[n] = t;
    }
}

// single-block exclusive scan (n up to millions: chunked)
__global__ void exclusive_scan_kernel(const int32_t* in, int32_t* out, int n, int32_t* total) {
    __shared__ int wsum[16];
    __shared__ int carry_s;
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, nw = blockDim.x >> 6;
    if (threadIdx.x == 0) carry_s = 0;
    __syncthreads();
    for (int base = 0; base < n; base += blockDim.x) {
        const int i = base + threadIdx.x;
        const int v = i < n ? in[i] : 0;
        int incl = v;
        for (int off = 1; off < 64; off <<= 1) {
            const int y = __shfl_up(incl, off);
            if (lane >= off) incl += y;
        }
        if (lane == 63) wsum[wave] = incl;
        __syncthreads();
        int woff = 0;
        for (int w = 0; w < wave; w++) woff += wsum[w];
        int chunk_total = 0;
        for (int w = 0; w < nw; w++) chunk_total += wsum[w];
        const int carry = carry_s;
        if (i < n) out[i] = carry + woff + incl - v;
        __syncthreads();
        if (threadIdx.x == 0) carry_s = carry + chunk_total;
        __syncthreads();
    }
    if (threadIdx.x == 0 && total) *total = carry_s;
}

__global__ void cloud_write_kernel(const int32_t* depth, int width, int height, int stride, float cx, float cy,
                                   float fx, float fy, float depth_factor, const uint8_t* label_mask,
                                   const int32_t* pose_label, const int32_t* offsets, float* xyz, int32_t* pose_out,
                                   int32_t* label_out, int cap, CloudBounds cb, const uint8_t* rgb_in,
                                   uint8_t* rgb_out, const uint8_t* planes_in, uint8_t* planes_out, int num_poses) {
    __shared__ int wsum[16];
    __shared__ int carry_s;
    const int n = blockIdx.x;
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, nw = blockDim.x >> 6;
    const int ws = (width + stride - 1) / stride, hs = (height + stride - 1) / stride;
    const size_t npx = (size_t)width * height;
    if (threadIdx.x == 0) carry_s = offsets[n];
    __syncthreads();
    for (int base = 0; base < ws * hs; base += blockDim.x) {
        const int k = base + threadIdx.x;
        bool v = false;
        int kx = 0, ky = 0;
        size_t idx = 0;
        if (k < ws * hs) {
            ky = k / ws; kx = k - ky * ws;
            idx = npx * n + (size_t)(kx * stride) + (size_t)(ky * stride) * width;
            v = cloud_valid(depth, label_mask, idx, kx * stride, ky * stride, cb);
        }
        const uint64_t b = __ballot(v);
        if (lane == 0) wsum[wave] = __popcll(b);
        __syncthreads();
        int woff = 0, tot = 0;
        for (int w = 0; w < nw; w++) {
            if (w < wave) woff += wsum[w];
            tot += wsum[w];
        }
        const int carry = carry_s;
        if (v) {
            const int o = carry + woff + mbcnt64(b);
            if (o < cap) {
                const int32_t d = depth[idx];
                const float zp = (float)d / depth_factor;
                const float xp = ((float)(kx * stride) - cx) / fx * zp;
                const float yp = ((float)(ky * stride) - cy) / fy * zp;
                xyz[3 * (size_t)o + 0] = xp;
                xyz[3 * (size_t)o + 1] = yp;
                xyz[3 * (size_t)o + 2] = zp;
                if (pose_out) pose_out[o] = n;
                if (rgb_out) {  // depth_to_2d_cloud :155-157, the input image's channels in order
                    rgb_out[3 * (size_t)o + 0] = rgb_in[3 * idx + 0];
                    rgb_out[3 * (size_t)o + 1] = rgb_in[3 * idx + 1];
                    rgb_out[3 * (size_t)o + 2] = rgb_in[3 * idx + 2];
                }
                if (planes_out) {  // depth_to_2d_cloud :163-165: the rendered colour planes into point planes
                    const size_t plane = npx * (size_t)num_poses;
                    planes_out[o] = planes_in[idx];
                    planes_out[(size_t)cap + o] = planes_in[plane + idx];
                    planes_out[2 * (size_t)cap + o] = planes_in[2 * plane + idx];
                }
                if (label_out) {
                    if (label_mask) label_out[o] = (int32_t)label_mask[idx] - 1;
                    else if (pose_label) label_out[o] = pose_label[n];
                    else label_out[o] = 0;
                }
            }
        }
        __syncthreads();
        if (threadIdx.x == 0) carry_s = carry + tot;
        __syncthreads();
    }
}

hipError_t launch_cloud_count(const int32_t* depth, int num_poses, int width, int height, int stride,
                              const uint8_t* label_mask, const CloudBounds& cb, int32_t* counts, hipStream_t s) {
    if (num_poses <= 0) return hipSuccess;
    hipLaunchKernelGGL(cloud_count_kernel, dim3(num_poses), dim3(256), 0, s, depth, width, height, stride, label_mask,
                       cb, counts);
    return hipGetLastError();
}

hipError_t launch_exclusive_scan(const int32_t* in, int32_t* out, int n, int32_t* total, hipStream_t s) {
    hipLaunchKernelGGL(exclusive_scan_kernel, dim3(1), dim3(1024), 0, s, in, out, n, total);
    return hipGetLastError();
}

hipError_t launch_cloud_write(const int32_t* depth, int num_poses, int width, int height, int stride, float cx,
                              float cy, float fx, float fy, float depth_factor, const uint8_t* label_mask,
                              const int32_t* pose_label, const int32_t* offsets, float* xyz, int32_t* pose,
                              int32_t* label, int cap, const CloudBounds& cb, const uint8_t* rgb_in,
                              uint8_t* rgb_out, hipStream_t s, const uint8_t* planes_in, uint8_t* planes_out) {
    if (num_poses <= 0) return hipSuccess;
    hipLaunchKernelGGL(cloud_write_kernel, dim3(num_poses), dim3(256), 0, s, depth, width, height, stride, cx, cy, fx,
                       fy, depth_factor, label_mask, pose_label, offsets, xyz, pose, label, cap, cb, rgb_in,
                       rgb_out, planes_in, planes_out, num_poses);
    return hipGetLastError();
}

// result_dc_index (compute_point_clouds.cuh:267-292): the reference scans a 0/1 mask over every pixel of the N
// z-buffers, so a pixel's entry is the number of cloud points (valid stride samples) before it in pose / row / column
// order.  Per pose, the exclusive count at every stride sample and at the pose's end (one block per pose) ...
__global__ void cloud_sample_prefix_kernel(const int32_t* depth, int width, int height, int stride,
                                           const uint8_t* label_mask, const int32_t* offsets, int32_t* pre) {
    __shared__ int wsum[16];
    __shared__ int carry_s;
    const int n = blockIdx.x;
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, nw = blockDim.x >> 6;
    const int ws = (width + stride - 1) / stride, hs = (height + stride - 1) / stride;
    const size_t npx = (size_t)width * height;
    int32_t* P = pre + (size_t)n * (ws * hs + 1);
    const CloudBounds cb{};
    if (threadIdx.x == 0) carry_s = offsets[n];
    __syncthreads();
    for (int base = 0; base < ws * hs; base += blockDim.x) {
        const int k = base + threadIdx.x;
        bool v = false;
        if (k < ws * hs) {
            const int ky = k / ws, kx = k - ky * ws;
            v = cloud_valid(depth, label_mask, npx * n + (size_t)(kx * stride) + (size_t)(ky * stride) * width,
                            kx * stride, ky * stride, cb);
        }
        const uint64_t b = __ballot(v);
        if (lane == 0) wsum[wave] = __popcll(b);
        __syncthreads();
        int woff = 0, tot = 0;
        for (int w = 0; w < nw; w++) {
            if (w < wave) woff += wsum[w];
            tot += wsum[w];
        }
        const int carry = carry_s;
        if (k < ws * hs) P[k] = carry + woff + mbcnt64(b);
        __syncthreads();
        if (threadIdx.x == 0) carry_s = carry + tot;
        __syncthreads();
    }
    if (threadIdx.x == 0) P[ws * hs] = carry_s;
}

// ... then every pixel: the samples before pixel (x, y) are the rows of samples above it and, on a sample row, the
// samples left of it
__global__ void cloud_dc_index_kernel(int num_poses, int width, int height, int stride, const int32_t* pre,
                                      int32_t* dc) {
    const int ws = (width + stride - 1) / stride, hs = (height + stride - 1) / stride;
    const size_t npx = (size_t)width * height, total = npx * num_poses;
    for (size_t p = (size_t)blockIdx.x * blockDim.x + threadIdx.x; p < total; p += (size_t)gridDim.x * blockDim.x) {
        const size_t n = p / npx, r = p - n * npx;
        const int y = (int)(r / width), x = (int)(r - (size_t)y * width);
        const int ry = y % stride == 0 ? y / stride : y / stride + 1;
        const int cx = y % stride == 0 ? (x + stride - 1) / stride : 0;
        const int k = min(ry * ws + cx, ws * hs);
        dc[p] = pre[n * (size_t)(ws * hs + 1) + k];
    }
}

hipError_t launch_cloud_dc_index(const int32_t* depth, int num_poses, int width, int height, int stride,
                                 const uint8_t* label_mask, const int32_t* offsets, int32_t* pre, int32_t* dc,
                                 hipStream_t s) {
    if (num_poses <= 0) return hipSuccess;
    hipLaunchKernelGGL(cloud_sample_prefix_kernel, dim3(num_poses), dim3(256), 0, s, depth, width, height, stride,
                       label_mask, offsets, pre);
    const size_t total = (size_t)width * height * num_poses;
    const int blocks = (int)std::min<size_t>((total + 255) / 256, 65535);
    hipLaunchKernelGGL(cloud_dc_index_kernel, dim3(blocks), dim3(256), 0, s, num_poses, width, height, stride, pre, dc);
    return hipGetLastError();
}

// sampled copy of the source depth / mask at the stride grid (used by the fused kernel)
__global__ void sample_source_kernel(const int32_t* src_depth, const uint8_t* src_mask, int width, int height,
                                     int stride, int32_t* src_s, uint8_t* lab_s) {
    const int ws = (width + stride - 1) / stride, hs = (height + stride - 1) / stride;
    for (int k = blockIdx.x * blockDim.x + threadIdx.x; k < ws * hs; k += gridDim.x * blockDim.x) {
        const int ky = k / ws, kx = k - ky * ws;
        const size_t idx = (size_t)(kx * stride) + (size_t)(ky * stride) * width;
        src_s[k] = src_depth[idx];
        if (lab_s) lab_s[k] = src_mask ? src_mask[idx] : 0;
    }
}

hipError_t launch_sample_source(const int32_t* src_depth, const uint8_t* src_mask, int width, int height, int stride,
                                int32_t* src_s, uint8_t* lab_s, hipStream_t s) {
    hipLaunchKernelGGL(sample_source_kernel, dim3(64), dim3(256), 0, s, src_depth, src_mask, width, height, stride,
                       src_s, lab_s);
    return hipGetLastError();
}

// ------------------------------------------------------------------------------------------------
// Selection (search_env.cpp:1987-2051, 2542-2583) as per-model int64 argmin keys
// ------------------------------------------------------------------------------------------------

__global__ void select_kernel(const float* rc, const float* oc, const int32_t* pose_model, int num_poses,
                              int64_t index_base, int num_models, int64_t* keys) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    int64_t key = PCORE_KEY_NONE_DEV;
    int m = -1;
    if (i < num_poses) {
        m = pose_model[i];
        key = select_key(rc[i], oc[i], m, num_models, index_base + i);
    }
    // wave-level minimum when the wave's poses share one model (the common case)
    const int m0 = __shfl(m, 0);
    const bool uniform = __all(m == m0 || m < 0);
    if (uniform) {
        int64_t k = key;
        for (int off = 32; off > 0; off >>= 1) {
            const int64_t o = __shfl_xor(k, off);
            k = o < k ? o : k;
        }
        if ((threadIdx.x & 63) == 0 && k != PCORE_KEY_NONE_DEV && m0 >= 0 && m0 < num_models)
            atomicMin((unsigned long long*)&keys[m0], (unsigned long long)k);
    } else if (key != PCORE_KEY_NONE_DEV) {
        atomicMin((unsigned long long*)&keys[m], (unsigned long long)key);
    }
}

hipError_t launch_select(const float* rc, const float* oc, const int32_t* pose_model, int num_poses,
                         int64_t index_base, int num_models, int64_t* keys, hipStream_t s) {
    if (num_poses <= 0) return hipSuccess;
    hipLaunchKernelGGL(select_kernel, dim3((num_poses + 255) / 256), dim3(256), 0, s, rc, oc, pose_model, num_poses,
                       index_base, num_models, keys);
    return hipGetLastError();
}

}  // namespace pcore
