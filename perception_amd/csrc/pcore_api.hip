// pcore_api.hip -- C ABI (include/pcore.h) of the MI355X pose-search core: context, static inputs
// (mesh dedupe + vertex-ring streams, camera), per-scene observation (label sort + neighbour grids) and dispatch of
// the kernels in pcore_kernels.hip.  Host code; no hidden allocations on the per-batch path (evaluate /
// select), scratch for the parity stages grows monotonically.
#include "../../include/pcore.h"
#include "pcore_internal.h"
#include "pcore_streams.h"
#include "pcore_gicp_math.h"

#include <algorithm>
#include <climits>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <unordered_map>
#include <vector>

using namespace pcore;

namespace {

template <typename T>
struct DevBuf {
    T* p = nullptr;
    size_t n = 0;
};

}  // namespace

struct pcore_ctx {
    int device = 0;
    std::string err;
    hipDeviceProp_t prop{};
    DeviceInfo dinfo{};       // per-device launch constants, filled once in pcore_create
    uint64_t generation = 1;  // pcore_generation: bumped whenever captured state may change
    // mesh
    int num_models = 0;
    int num_tris = 0;
    DevBuf<float> tris;          // original triangle soup (parity render)
    DevBuf<int32_t> tri_lo, tri_hi;
    DevBuf<float4> sverts;       // vertex-ring streams (pcore_internal.h, kVRing)
    DevBuf<uint32_t> stris;
    DevBuf<int4> streams;
    DevBuf<int32_t> model_st_lo, model_st_hi;
    DevBuf<float4> model_box;  // FusedArgs::model_box
    DevBuf<uint32_t> tri_rgb;  // per original triangle: r | g << 8 | b << 16 (stage RENDER colour planes)
    bool have_mesh = false;
    // camera
    pcore_camera cam{};
    DevBuf<float> proj;
    bool have_cam = false;
    // observation
    DevBuf<int32_t> src_depth;
    DevBuf<uint8_t> src_mask;
    bool obs_has_mask = false;
    int sampled_stride = 0;
    DevBuf<int32_t> src_s;
    DevBuf<uint8_t> lab_s;
    DevBuf<LabelGrid> grids;
    DevBuf<int32_t> cell_start;
    DevBuf<float4> grid_pts;
    int num_grids = 0;
    int bitmap_words = 1;
    bool have_obs = false;
    // GICP targets: label-sorted observed points, segments [lo, hi) per label + the whole cloud
    int num_obs = 0;
    int max_seg = 0;
    DevBuf<float4> tgt;
    DevBuf<int32_t> seg_lo, seg_hi, seg_cnt;
    std::vector<int32_t> seg_lo_h, seg_cnt_h;  // host copies (grid covariance launches)
    DevBuf<float> tgt_quads;                   // GicpArgs::tgt_quads
    DevBuf<int32_t> seg_qoff;
    DevBuf<double> tgt_cov_label, tgt_cov_all;
    int cov_k_label = 0, cov_k_all = 0;
    // GICP scratch
    DevBuf<float4> icp_cloud;
    DevBuf<int32_t> icp_count;
    DevBuf<double> icp_cov;
    DevBuf<int32_t> icp_corr;   // GicpArgs::corr
    DevBuf<int32_t> scratch_dc_pre;  // stage CLOUD result_dc_index: per-pose sample prefixes
    DevBuf<int32_t> icp_corr_hist;  // GicpArgs::corr_hist
    DevBuf<double> icp_mahal;   // GicpArgs::mahal
    DevBuf<int32_t> icp_counter;
    DevBuf<unsigned long long> icp_iter_stats;  // GicpArgs::iter_stats ([0..3]) and help_stats ([4..7]), zeroed per call
    DevBuf<unsigned> icp_help_ctl;              // GicpArgs::help_ctl (zeroed per launch by launch_gicp)
    DevBuf<unsigned long long> icp_help_gran;   // GicpArgs::help_gran
    uint32_t icp_help_tag = 0;                  // GicpArgs::help_tag of the last launch (1..0xFFFF, cycling)
    // their copy in pinned host memory, made on the call's stream before each chunk's end event (pcore_get_stats reads
    // it after that event: no synchronous copy, which would wait for every blocking stream of the device)
    unsigned long long* icp_iter_stats_host = nullptr;
    DevBuf<uint32_t> icp_order_keys;  // 2 x chunk keys (in, out)
    DevBuf<int32_t> icp_order_idx;    // 2 x chunk indices (in, out = GicpArgs::pose_order)
    DevBuf<unsigned char> icp_order_temp;
    // colour gate (cost_type 1)
    DevBuf<uint32_t> stri_orig;   // original triangle of every stream triangle slot
    DevBuf<float4> tri_lab;       // Lab per original triangle
    DevBuf<float4> obs_lab;       // Lab per observed point, label-sorted
    DevBuf<int32_t> colour_id;    // N x nsamp scratch of the fused kernel's colour id pass
    DevBuf<int32_t> fb_ctr;       // FusedArgs::fb_ctr
    DevBuf<int32_t> win_hist;     // FusedArgs::win_hist
    DevBuf<int32_t> fb_ctr_cap;   // the same for captured launches: counted into, never published or read
    DevBuf<int32_t> win_hist_cap;
    int32_t* fb_host = nullptr;   // mapped host memory (FusedArgs::fb_host), host view
    int32_t* fb_dev = nullptr;    // the same, device view
    int32_t fb_seq = 0;           // sequence number of the last fused launch
    int32_t tile_key_seq = 0;     // first sequence number launched with the current tile configuration
    long long tile_key = -1;      // ws, hs, bitmap words, colour of the current tile configuration
    int tile_tier = kDefaultTier;
    int32_t tile_tcap = 0;        // tile (samples) of the last window launch
    bool tile_probed = false;     // the window probe has chosen a tier for the current tile key
    DevBuf<int32_t> win_probe;    // its histogram
    int32_t tile_edge[kTileTiers] = {};
    std::vector<int> obs_order;   // label-sorted position -> caller's observed index
    bool have_obs_colours = false;
    DevBuf<double> metric_part;  // ADD / ADD-S per-block partial sums
    // scratch (parity stages)
    DevBuf<int32_t> scratch_counts, scratch_offsets, scratch_total;
    DevBuf<int32_t> render_tri;  // stage RENDER colour: nearest triangle per pixel
    // gpu_stats of the last pcore_evaluate_icp (pcore_get_stats): per chunk, events at the source covariances,
    // the GICP launch and its end on the call's stream; the peak device memory in use at a GICP stage
    std::vector<hipEvent_t> icp_ev;
    int icp_ev_used = 0;
    double peak_mem_mb = 0.0;
};

namespace {

int fail(pcore_ctx* c, int code, const std::string& msg) {
    if (c) c->err = msg;
    return code;
}

#define HIPC(ctx, call)                                                                         \
    do {                                                                                        \
        hipError_t e_ = (call);                                                                 \
        if (e_ != hipSuccess)                                                                   \
            return fail(ctx, e_ == hipErrorOutOfMemory ? PCORE_E_OOM : PCORE_E_HIP,             \
                        std::string(#call) + ": " + hipGetErrorString(e_));                     \
    } while (0)

template <typename T>
hipError_t dev_free(DevBuf<T>& b) {
    hipError_t e = hipSuccess;
    if (b.p) e = hipFree(b.p);
    b.p = nullptr;
    b.n = 0;
    return e;
}

template <typename T>
hipError_t dev_reserve(DevBuf<T>& b, size_t n) {
    if (b.n >= n && b.p) return hipSuccess;
    hipError_t e = dev_free(b);
    if (e != hipSuccess) return e;
    e = hipMalloc(&b.p, std::max<size_t>(n, 1) * sizeof(T));
    if (e == hipSuccess) b.n = n;
    return e;
}

// dev_reserve for scratch a captured evaluate graph points into: a reallocation invalidates such graphs
template <typename T>
hipError_t reserve_gen(pcore_ctx* c, DevBuf<T>& b, size_t n) {
    if (b.n >= n && b.p) return hipSuccess;
    c->generation++;
    return dev_reserve(b, n);
}

template <typename T>
hipError_t dev_upload(DevBuf<T>& b, const std::vector<T>& v) {
    hipError_t e = dev_reserve(b, v.size());
    if (e != hipSuccess) return e;
    if (!v.empty()) e = hipMemcpy(b.p, v.data(), v.size() * sizeof(T), hipMemcpyHostToDevice);
    return e;
}

struct VKey {
    uint32_t x, y, z;
    bool operator==(const VKey& o) const { return x == o.x && y == o.y && z == o.z; }
};
struct VKeyHash {
    size_t operator()(const VKey& k) const {
        uint64_t h = k.x * 0x9E3779B97F4A7C15ull;
        h ^= (k.y + 0x632BE59BD9B4E019ull) + (h << 6) + (h >> 2);
        h ^= (k.z + 0x85EBCA77C2B2AE63ull) + (h << 6) + (h >> 2);
        return (size_t)h;
    }
};

// rgb2lab (compute_costs.cuh:57-88) in double with glibc pow / cbrt, stored as float.  The cost reads
// its "red" from colour plane 2 and "blue" from plane 0 (compute_costs.cuh:214-220): rgb2lab(c2, c1, c0).
float4 lab_of(const uint8_t c[3]) {
    const uint8_t rr = c[2], gg = c[1], bbb = c[0];
    double r = rr / 255.0, g = gg / 255.0, b = bbb / 255.0;
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
    const float l = (float)((116.0 * y) - 16), a = (float)(500 * (x - y)), bb = (float)(200 * (y - z));
    return make_float4(l, a, bb, 0.0f);
}

// Neighbour grid over one point set.  `pts` are (x,y,z, local index) in label-sorted order.
void build_grid(const std::vector<float4>& pts, float radius, LabelGrid& g, std::vector<int32_t>& cell_start,
                std::vector<float4>& grid_pts) {
    g = LabelGrid{};
    g.pt_count = (int)pts.size();
    g.cell_base = (int)cell_start.size();
    if (pts.empty()) {
        g.ox = g.oy = g.oz = 0.0f;
        g.inv_c = 1.0f;
        g.cell = 1.0f;
        g.nx = g.ny = g.nz = 1;
        cell_start.push_back((int32_t)grid_pts.size());
        cell_start.push_back((int32_t)grid_pts.size());
        return;
    }
    float lo[3] = {INFINITY, INFINITY, INFINITY}, hi[3] = {-INFINITY, -INFINITY, -INFINITY};
    for (const float4& p : pts) {
        const float c[3] = {p.x, p.y, p.z};
        for (int k = 0; k < 3; k++) {
            if (!std::isfinite(c[k])) continue;
            lo[k] = std::min(lo[k], c[k]);
            hi[k] = std::max(hi[k], c[k]);
        }
    }
    for (int k = 0; k < 3; k++)
        if (!(lo[k] <= hi[k])) { lo[k] = 0.0f; hi[k] = 0.0f; }
    // cell >= 2r so a query's radius box touches <= 2 cells per axis; at most 64 cells per axis
    const float ext = std::max({hi[0] - lo[0], hi[1] - lo[1], hi[2] - lo[2]});
    float cell = std::max(2.0f * radius * 1.01f, ext / 64.0f);
    if (!(cell > 0.0f)) cell = 1.0f;
    g.ox = lo[0];
    g.oy = lo[1];
    g.oz = lo[2];
    g.inv_c = 1.0f / cell;
    g.cell = cell;
    g.nx = std::max(1, (int)std::floor((hi[0] - lo[0]) * g.inv_c) + 1);
    g.ny = std::max(1, (int)std::floor((hi[1] - lo[1]) * g.inv_c) + 1);
    g.nz = std::max(1, (int)std::floor((hi[2] - lo[2]) * g.inv_c) + 1);
    const int ncell = g.nx * g.ny * g.nz;
    std::vector<int> cell_of(pts.size());
    std::vector<int> cnt(ncell + 1, 0);
    for (size_t i = 0; i < pts.size(); i++) {
        // same float formula as the device query (pcore_kernels.hip, process_points)
        const float fx = (pts[i].x - g.ox) * g.inv_c, fy = (pts[i].y - g.oy) * g.inv_c, fz = (pts[i].z - g.oz) * g.inv_c;
        int ix = (int)std::floor(std::max(fx, 0.0f)), iy = (int)std::floor(std::max(fy, 0.0f)),
            iz = (int)std::floor(std::max(fz, 0.0f));
        if (!std::isfinite(fx) || !std::isfinite(fy) || !std::isfinite(fz)) {
            cell_of[i] = -1;  // non-finite points can never be within the radius of a finite query
            continue;
        }
        ix = std::min(ix, g.nx - 1);
        iy = std::min(iy, g.ny - 1);
        iz = std::min(iz, g.nz - 1);
        cell_of[i] = (iz * g.ny + iy) * g.nx + ix;
        cnt[cell_of[i] + 1]++;
    }
    for (int c = 0; c < ncell; c++) cnt[c + 1] += cnt[c];
    const int base = (int)grid_pts.size();
    grid_pts.resize(base + cnt[ncell]);
    std::vector<int> fillp(cnt.begin(), cnt.end() - 1);
    for (size_t i = 0; i < pts.size(); i++)
        if (cell_of[i] >= 0) grid_pts[base + fillp[cell_of[i]]++] = pts[i];
    for (int c = 0; c <= ncell; c++) cell_start.push_back(base + cnt[c]);
}

}  // namespace

extern "C" {

int pcore_abi_version(void) { return PCORE_ABI_VERSION; }

int pcore_create(int device, pcore_ctx** out_ctx) {
    if (!out_ctx) return PCORE_E_INVALID_ARG;
    *out_ctx = nullptr;
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || device < 0 || device >= ndev) return PCORE_E_INVALID_ARG;
    pcore_ctx* c = new pcore_ctx();
    c->device = device;
    if (hipSetDevice(device) != hipSuccess || hipGetDeviceProperties(&c->prop, device) != hipSuccess) {
        delete c;
        return PCORE_E_HIP;
    }
    // per-context (not function-static) launch constants: contexts on other devices or threads never share
    // or race on them
    DeviceInfo& d = c->dinfo;
    d.num_cus = std::max(1, c->prop.multiProcessorCount);
    d.lds_per_cu = c->prop.maxSharedMemoryPerMultiProcessor ? (size_t)c->prop.maxSharedMemoryPerMultiProcessor
                                                            : (size_t)160 * 1024;
    d.lds_granule = kLdsGranule;
    if (const char* e = getenv("PCORE_LDS_GRANULE")) d.lds_granule = (size_t)std::max(atoi(e), 4);  // A/B only
    int per_cu = 0;
    if (gicp_occupancy_per_cu(&per_cu) != hipSuccess) {
        delete c;
        return PCORE_E_HIP;
    }
    d.gicp_resident_wgs = std::max(1, per_cu) * d.num_cus;
    *out_ctx = c;
    return PCORE_OK;
}

uint64_t pcore_generation(const pcore_ctx* c) { return c ? c->generation : 0; }

void pcore_destroy(pcore_ctx* c) {
    if (!c) return;
    (void)hipSetDevice(c->device);
    (void)dev_free(c->tris); (void)dev_free(c->tri_lo); (void)dev_free(c->tri_hi);
    (void)dev_free(c->sverts); (void)dev_free(c->stris); (void)dev_free(c->streams);
    (void)dev_free(c->model_st_lo); (void)dev_free(c->model_st_hi); (void)dev_free(c->model_box); (void)dev_free(c->proj);
    (void)dev_free(c->fb_ctr); (void)dev_free(c->win_hist);
    if (c->fb_host) (void)hipHostFree(c->fb_host);
    if (c->icp_iter_stats_host) (void)hipHostFree(c->icp_iter_stats_host);
    (void)dev_free(c->src_depth); (void)dev_free(c->src_mask); (void)dev_free(c->src_s); (void)dev_free(c->lab_s);
    (void)dev_free(c->grids); (void)dev_free(c->cell_start); (void)dev_free(c->grid_pts);
    (void)dev_free(c->scratch_counts); (void)dev_free(c->scratch_offsets); (void)dev_free(c->scratch_total);
    (void)dev_free(c->tgt); (void)dev_free(c->seg_lo); (void)dev_free(c->seg_hi); (void)dev_free(c->seg_cnt); (void)dev_free(c->tgt_quads); (void)dev_free(c->seg_qoff);
    (void)dev_free(c->tgt_cov_label); (void)dev_free(c->tgt_cov_all);
    (void)dev_free(c->icp_cloud); (void)dev_free(c->icp_count); (void)dev_free(c->icp_cov); (void)dev_free(c->icp_corr); (void)dev_free(c->icp_corr_hist); (void)dev_free(c->scratch_dc_pre); (void)dev_free(c->icp_mahal); (void)dev_free(c->icp_counter); (void)dev_free(c->icp_iter_stats); (void)dev_free(c->icp_help_ctl); (void)dev_free(c->icp_help_gran); (void)dev_free(c->icp_order_keys); (void)dev_free(c->icp_order_idx); (void)dev_free(c->icp_order_temp);
    (void)dev_free(c->stri_orig); (void)dev_free(c->tri_lab); (void)dev_free(c->obs_lab); (void)dev_free(c->colour_id);
    (void)dev_free(c->metric_part); (void)dev_free(c->tri_rgb); (void)dev_free(c->render_tri);
    for (hipEvent_t e : c->icp_ev) (void)hipEventDestroy(e);
    delete c;
}

const char* pcore_last_error(const pcore_ctx* c) { return c ? c->err.c_str() : "null context"; }

int pcore_upload_meshes(pcore_ctx* c, const float* tri_xyz, const uint8_t* tri_rgb, int32_t num_tris,
                        const int32_t* tris_model_count, int32_t num_models) {
    if (!c) return PCORE_E_INVALID_ARG;
    if (!tri_xyz || num_tris <= 0 || !tris_model_count || num_models <= 0)
        return fail(c, PCORE_E_INVALID_ARG, "upload_meshes: empty mesh");
    long long acc = 0;
    for (int m = 0; m < num_models; m++) {
        if (tris_model_count[m] < 0) return fail(c, PCORE_E_INVALID_ARG, "upload_meshes: negative count");
        acc += tris_model_count[m];
    }
    if (acc != num_tris) return fail(c, PCORE_E_INVALID_ARG, "upload_meshes: sum(tris_model_count) != num_tris");
    HIPC(c, hipSetDevice(c->device));
    c->generation++;

    streams::Built sb;
    int chunks = kStreamChunks;
    if (const char* e = getenv("PCORE_STREAM_CHUNKS")) chunks = std::max(1, atoi(e));  // A/B knob
    int model_streams = kFusedWaves;
    if (const char* e = getenv("PCORE_MODEL_STREAMS")) model_streams = std::max(1, atoi(e));  // A/B knob
    std::vector<float4> box;
    std::vector<int32_t> slo(num_models), shi(num_models), tlo(num_models), thi(num_models);
    int t0 = 0;
    for (int m = 0; m < num_models; m++) {
        const int T = tris_model_count[m];
        tlo[m] = t0;
        thi[m] = t0 + T;
        // exact-bit vertex dedupe within the model
        std::unordered_map<VKey, int, VKeyHash> idx;
        idx.reserve((size_t)T * 2);
        std::vector<int> tv((size_t)T * 3);
        std::vector<float> vxyz;
        for (int t = 0; t < T; t++)
            for (int k = 0; k < 3; k++) {
                const float* p = tri_xyz + (size_t)9 * (t0 + t) + 3 * k;
                VKey key;
                std::memcpy(&key.x, &p[0], 4);
                std::memcpy(&key.y, &p[1], 4);
                std::memcpy(&key.z, &p[2], 4);
                auto it = idx.find(key);
                int id;
                if (it == idx.end()) {
                    id = (int)(vxyz.size() / 3);
                    idx.emplace(key, id);
                    vxyz.push_back(p[0]);
                    vxyz.push_back(p[1]);
                    vxyz.push_back(p[2]);
                } else {
                    id = it->second;
                }
                tv[(size_t)3 * t + k] = id;
            }
        // bounding box of the model's vertices (pose windows); w = 1 when every coordinate is finite
        float4 bmin = make_float4(INFINITY, INFINITY, INFINITY, 1.0f), bmax = make_float4(-INFINITY, -INFINITY, -INFINITY, 0.0f);
        for (size_t i = 0; i < vxyz.size(); i += 3) {
            if (!std::isfinite(vxyz[i]) || !std::isfinite(vxyz[i + 1]) || !std::isfinite(vxyz[i + 2])) bmin.w = 0.0f;
            bmin.x = std::min(bmin.x, vxyz[i]); bmax.x = std::max(bmax.x, vxyz[i]);
            bmin.y = std::min(bmin.y, vxyz[i + 1]); bmax.y = std::max(bmax.y, vxyz[i + 1]);
            bmin.z = std::min(bmin.z, vxyz[i + 2]); bmax.z = std::max(bmax.z, vxyz[i + 2]);
        }
        if (vxyz.empty()) bmin = bmax = make_float4(0.0f, 0.0f, 0.0f, 0.0f);
        box.push_back(bmin);
        box.push_back(bmax);
        slo[m] = (int)sb.streams.size();
        streams::build_model(tv, vxyz, t0, model_streams, kVRing, kRefPasses, sb, chunks);
        shi[m] = (int)sb.streams.size();
        t0 += T;
    }
    // one padding step and one padding vertex pass after the last stream: the fused kernel prefetches the step and
    // the pass after the current ones unconditionally (within a model that is the next stream's first one)
    sb.stris.insert(sb.stris.end(), kStepSlots, streams::kSlotPadding);
    sb.sorig.insert(sb.sorig.end(), kStepSlots, 0u);
    sb.sverts.insert(sb.sverts.end(), kStepSlots, streams::F4{0.0f, 0.0f, 0.0f, 0.0f});
    std::vector<float> soup(tri_xyz, tri_xyz + (size_t)9 * num_tris);
    HIPC(c, dev_upload(c->tris, soup));
    HIPC(c, dev_upload(c->tri_lo, tlo));
    HIPC(c, dev_upload(c->tri_hi, thi));
    static_assert(sizeof(streams::F4) == sizeof(float4) && sizeof(streams::I4) == sizeof(int4), "stream layouts");
    std::vector<float4> sv(sb.sverts.size());
    if (!sv.empty()) std::memcpy(sv.data(), sb.sverts.data(), sv.size() * sizeof(float4));
    std::vector<int4> sd(sb.streams.size());
    if (!sd.empty()) std::memcpy(sd.data(), sb.streams.data(), sd.size() * sizeof(int4));
    HIPC(c, dev_upload(c->sverts, sv));
    HIPC(c, dev_upload(c->stris, sb.stris));
    HIPC(c, dev_upload(c->streams, sd));
    HIPC(c, dev_upload(c->stri_orig, sb.sorig));
    std::vector<float4> tl((size_t)num_tris);
    for (int t = 0; t < num_tris; t++) {
        uint8_t col[3] = {128, 128, 128};
        if (tri_rgb) for (int k = 0; k < 3; k++) col[k] = tri_rgb[3 * (size_t)t + k];
        tl[t] = lab_of(col);
    }
    HIPC(c, dev_upload(c->tri_lab, tl));
    std::vector<uint32_t> packed((size_t)num_tris);
    for (int t = 0; t < num_tris; t++) {
        uint32_t v = 128u | 128u << 8 | 128u << 16;  // model.cpp:97-101: grey without vertex colours
        if (tri_rgb)
            v = (uint32_t)tri_rgb[3 * (size_t)t] | (uint32_t)tri_rgb[3 * (size_t)t + 1] << 8 |
                (uint32_t)tri_rgb[3 * (size_t)t + 2] << 16;
        packed[t] = v;
    }
    HIPC(c, dev_upload(c->tri_rgb, packed));
    HIPC(c, dev_upload(c->model_st_lo, slo));
    HIPC(c, dev_upload(c->model_st_hi, shi));
    HIPC(c, dev_upload(c->model_box, box));
    c->num_models = num_models;
    c->num_tris = num_tris;
    c->have_mesh = true;
    return PCORE_OK;
}

int pcore_set_camera(pcore_ctx* c, const pcore_camera* cam) {
    if (!c || !cam) return PCORE_E_INVALID_ARG;
    if (cam->width <= 0 || cam->height <= 0 || cam->width > 16384 || cam->height > 16384)
        return fail(c, PCORE_E_INVALID_ARG, "set_camera: bad image size");
    HIPC(c, hipSetDevice(c->device));
    c->generation++;
    c->cam = *cam;
    std::vector<float> pj(cam->proj, cam->proj + 16);
    HIPC(c, dev_upload(c->proj, pj));
    c->have_cam = true;
    c->have_obs = false;  // observation is tied to the image size
    c->sampled_stride = 0;
    return PCORE_OK;
}

int pcore_observed_cloud(pcore_ctx* c, const int32_t* d_depth, const uint8_t* d_label_mask, int32_t width,
                         int32_t height, int32_t stride, float depth_factor, float* d_out_xyz, int32_t* d_out_label,
                         int32_t cap, int32_t* out_count, pcore_stream stream) {
    if (!c) return PCORE_E_INVALID_ARG;
    if (!c->have_cam) return fail(c, PCORE_E_STATE, "observed_cloud: camera not set");
    return pcore_depth_to_cloud(c, d_depth, 1, width, height, stride, depth_factor, d_label_mask, nullptr, d_out_xyz,
                                nullptr, d_out_label, cap, out_count, stream);
}

int pcore_observed_cloud_bounded(pcore_ctx* c, const int32_t* d_depth, const uint8_t* d_rgb, int32_t width,
                                 int32_t height, int32_t stride, float depth_factor, const float* cam_to_world,
                                 const double* bounds, float* d_out_xyz, uint8_t* d_out_rgb, int32_t cap,
                                 int32_t* out_count, pcore_stream stream) {
    if (!c) return PCORE_E_INVALID_ARG;
    if (!c->have_cam) return fail(c, PCORE_E_STATE, "observed_cloud_bounded: camera not set");
    if (width <= 0 || height <= 0 || stride <= 0 || !d_depth || cap < 0 || (cap > 0 && !d_out_xyz) || !out_count ||
        (!cam_to_world) != (!bounds) || (d_out_rgb && !d_rgb))
        return fail(c, PCORE_E_INVALID_ARG, "observed_cloud_bounded: bad arguments");
    if (width % stride != 0) return fail(c, PCORE_E_INVALID_ARG, "observed_cloud_bounded: width % stride != 0");
    CloudBounds cb{};
    if (cam_to_world) {
        cb.on = 1;
        for (int i = 0; i < 12; i++) cb.m[i] = cam_to_world[i];
        for (int i = 0; i < 6; i++) cb.b[i] = (float)bounds[i];
        cb.cx = c->cam.cx;
        cb.cy = c->cam.cy;
        cb.fx = c->cam.fx;
        cb.fy = c->cam.fy;
        cb.depth_factor = depth_factor;
    }
    *out_count = 0;
    HIPC(c, hipSetDevice(c->device));
    hipStream_t s = (hipStream_t)stream;
    HIPC(c, dev_reserve(c->scratch_counts, 1));
    HIPC(c, dev_reserve(c->scratch_offsets, 1));
    HIPC(c, dev_reserve(c->scratch_total, 1));
    HIPC(c, launch_cloud_count(d_depth, 1, width, height, stride, nullptr, cb, c->scratch_counts.p, s));
    HIPC(c, launch_exclusive_scan(c->scratch_counts.p, c->scratch_offsets.p, 1, c->scratch_total.p, s));
    HIPC(c, launch_cloud_write(d_depth, 1, width, height, stride, c->cam.cx, c->cam.cy, c->cam.fx, c->cam.fy,
                               depth_factor, nullptr, nullptr, c->scratch_offsets.p, d_out_xyz, nullptr, nullptr, cap,
                               cb, d_rgb, d_out_rgb, s));
    int32_t total = 0;
    HIPC(c, hipMemcpyAsync(&total, c->scratch_total.p, 4, hipMemcpyDeviceToHost, s));
    HIPC(c, hipStreamSynchronize(s));
    *out_count = total;
    return PCORE_OK;
}

int pcore_set_observation_colors(pcore_ctx* c, const uint8_t* d_obs_rgb, int32_t num_obs, pcore_stream stream) {
    if (!c) return PCORE_E_INVALID_ARG;
    if (!c->have_obs) return fail(c, PCORE_E_STATE, "set_observation_colors: call pcore_set_observation first");
    if (num_obs != (int)c->obs_order.size() || (num_obs > 0 && !d_obs_rgb))
        return fail(c, PCORE_E_INVALID_ARG, "set_observation_colors: num_obs differs from the observation");
    HIPC(c, hipSetDevice(c->device));
    c->generation++;
    hipStream_t s = (hipStream_t)stream;
    std::vector<uint8_t> rgb((size_t)num_obs * 3);
    if (num_obs > 0) HIPC(c, hipMemcpyAsync(rgb.data(), d_obs_rgb, rgb.size(), hipMemcpyDeviceToHost, s));
    HIPC(c, hipStreamSynchronize(s));
    std::vector<float4> labv(std::max(num_obs, 1), make_float4(0.0f, 0.0f, 0.0f, 0.0f));
    for (int k = 0; k < num_obs; k++) labv[k] = lab_of(&rgb[3 * (size_t)c->obs_order[k]]);
    HIPC(c, dev_upload(c->obs_lab, labv));
    c->have_obs_colours = true;
    return PCORE_OK;
}

int pcore_set_observation(pcore_ctx* c, const int32_t* d_src_depth_cm, const uint8_t* d_src_mask,
                          const float* d_obs_xyz, const int32_t* d_obs_label, int32_t num_obs,
                          float sensor_resolution, pcore_stream stream) {
    if (!c) return PCORE_E_INVALID_ARG;
    if (!c->have_cam) return fail(c, PCORE_E_STATE, "set_observation: camera not set");
    if (!d_src_depth_cm || num_obs < 0 || (num_obs > 0 && !d_obs_xyz))
        return fail(c, PCORE_E_INVALID_ARG, "set_observation: bad arguments");
    if (!(sensor_resolution >= 0.0f)) return fail(c, PCORE_E_INVALID_ARG, "set_observation: bad sensor_resolution");
    HIPC(c, hipSetDevice(c->device));
    c->generation++;
    hipStream_t s = (hipStream_t)stream;
    const size_t npx = (size_t)c->cam.width * c->cam.height;
    HIPC(c, dev_reserve(c->src_depth, npx));
    HIPC(c, hipMemcpyAsync(c->src_depth.p, d_src_depth_cm, npx * 4, hipMemcpyDeviceToDevice, s));
    c->obs_has_mask = d_src_mask != nullptr;
    HIPC(c, dev_reserve(c->src_mask, npx));
    if (d_src_mask) HIPC(c, hipMemcpyAsync(c->src_mask.p, d_src_mask, npx, hipMemcpyDeviceToDevice, s));
    else HIPC(c, hipMemsetAsync(c->src_mask.p, 0, npx, s));

    // observed cloud -> host: stable label sort (renderer.cu:1674-1686) + neighbour grids
    std::vector<float> xyz((size_t)num_obs * 3);
    std::vector<int32_t> lab(num_obs, 0);
    if (num_obs > 0) {
        HIPC(c, hipMemcpyAsync(xyz.data(), d_obs_xyz, xyz.size() * 4, hipMemcpyDeviceToHost, s));
        if (d_obs_label) HIPC(c, hipMemcpyAsync(lab.data(), d_obs_label, lab.size() * 4, hipMemcpyDeviceToHost, s));
    }
    HIPC(c, hipStreamSynchronize(s));
    int max_label = -1;
    for (int i = 0; i < num_obs; i++) max_label = std::max(max_label, lab[i]);
    const int num_labels = std::max(0, max_label + 1);
    std::vector<int> order(num_obs);
    for (int i = 0; i < num_obs; i++) order[i] = i;
    std::stable_sort(order.begin(), order.end(), [&](int a, int b) { return lab[a] < lab[b]; });
    c->obs_order = order;
    c->have_obs_colours = false;
    std::vector<LabelGrid> grids(num_labels + 1);
    std::vector<int32_t> cell_start;
    std::vector<float4> gpts;
    int max_cnt = 0;
    // per-label grids (6-DoF): points with negative labels are never matched (no rendered label < 0)
    for (int L = 0; L < num_labels; L++) {
        std::vector<float4> pts;
        int local = 0;
        for (int i : order)
            if (lab[i] == L) {
                float4 p = make_float4(xyz[3 * i], xyz[3 * i + 1], xyz[3 * i + 2], 0.0f);
                int li = local++;
                std::memcpy(&p.w, &li, 4);
                pts.push_back(p);
            }
        max_cnt = std::max(max_cnt, (int)pts.size());
        build_grid(pts, sensor_resolution, grids[L], cell_start, gpts);
    }
    // 3-DoF grid over the whole cloud, in label-sorted order
    {
        std::vector<float4> pts;
        for (int k = 0; k < num_obs; k++) {
            const int i = order[k];
            float4 p = make_float4(xyz[3 * i], xyz[3 * i + 1], xyz[3 * i + 2], 0.0f);
            std::memcpy(&p.w, &k, 4);
            pts.push_back(p);
        }
        max_cnt = std::max(max_cnt, (int)pts.size());
        build_grid(pts, sensor_resolution, grids[num_labels], cell_start, gpts);
    }
    // GICP targets (label-sorted) and their segments; covariances are computed lazily per k
    {
        std::vector<float4> tp(std::max(num_obs, 1));
        for (int k2 = 0; k2 < num_obs; k2++) {
            const int i = order[k2];
            tp[k2] = make_float4(xyz[3 * i], xyz[3 * i + 1], xyz[3 * i + 2], 0.0f);
        }
        std::vector<int32_t> slo(num_labels + 1), shi(num_labels + 1), scnt(num_labels + 1);
        int pos = 0, mx = num_obs;
        for (int L = 0; L < num_labels; L++) {
            while (pos < num_obs && lab[order[pos]] < L) pos++;
            slo[L] = pos;
            int e = pos;
            while (e < num_obs && lab[order[e]] == L) e++;
            shi[L] = e;
            scnt[L] = e - pos;
            mx = std::max(mx, e - pos);
        }
        slo[num_labels] = 0;
        shi[num_labels] = num_obs;
        scnt[num_labels] = num_obs;
        HIPC(c, dev_upload(c->tgt, tp));
        HIPC(c, dev_upload(c->seg_lo, slo));
        HIPC(c, dev_upload(c->seg_hi, shi));
        HIPC(c, dev_upload(c->seg_cnt, scnt));
        c->seg_lo_h = slo;
        c->seg_cnt_h = scnt;
        // quad-SoA copy of every segment (labels, then the whole cloud) for the scalar-cache scan: a header quad
        // (the segment's key origin c in [0..2]), then quads of four targets as correspondence keys
        // (-2 t'x [4], -2 t'y [4], -2 t'z [4], |t'|^2 [4]; padding: 0, 0, 0, +inf), pcore_gicp_math.h
        std::vector<int32_t> qoff(num_labels + 1);
        std::vector<float> quads;
        for (int L = 0; L <= num_labels; L++) {
            qoff[L] = (int32_t)(quads.size() / 16);
            const int n = scnt[L], nq = (n + 3) / 4;
            float org[3];
            gicpm::nn_origin(n, [&](int i, float* p) {
                const float4 v = tp[slo[L] + i];
                p[0] = v.x; p[1] = v.y; p[2] = v.z;
            }, org);
            const size_t q0 = quads.size();
            quads.resize(q0 + (size_t)16 * (nq + 1), 0.0f);
            quads[q0] = org[0]; quads[q0 + 1] = org[1]; quads[q0 + 2] = org[2];
            for (int i = n; i < 4 * nq; i++) quads[q0 + 16 + (size_t)16 * (i / 4) + 12 + i % 4] = INFINITY;
            for (int i = 0; i < n; i++) {
                const float4 p = tp[slo[L] + i];
                const gicpm::NNTarget t = gicpm::nn_target(p.x, p.y, p.z, org[0], org[1], org[2]);
                float* Q = &quads[q0 + 16 + (size_t)16 * (i / 4)];
                Q[i % 4] = t.m2x;
                Q[4 + i % 4] = t.m2y;
                Q[8 + i % 4] = t.m2z;
                Q[12 + i % 4] = t.tt;
            }
        }
        HIPC(c, dev_upload(c->tgt_quads, quads));
        HIPC(c, dev_upload(c->seg_qoff, qoff));
        c->num_obs = num_obs;
        c->max_seg = mx;
        c->cov_k_label = 0;
        c->cov_k_all = 0;
    }
    HIPC(c, dev_upload(c->grids, grids));
    HIPC(c, dev_upload(c->cell_start, cell_start));
    HIPC(c, dev_upload(c->grid_pts, gpts));
    c->num_grids = num_labels;
    c->bitmap_words = std::max(1, (max_cnt + 31) / 32);
    c->sampled_stride = 0;
    c->have_obs = true;
    return PCORE_OK;
}

// the tier with the most workgroups per CU whose tile holds the windows of >= 99 % of the histogram's poses
static int choose_tier(const int32_t* h, const int* edge, int fallback) {
    long long tot = 0;
    for (int b = 0; b <= kTileTiers; b++) tot += h[b];
    if (tot <= 0) return fallback;
    long long over = tot;  // windows above edge[t]
    for (int t = 0; t < kTileTiers; t++) {
        over -= h[t];
        if (edge[t] > 0 && over * 100 <= tot) return t;
    }
    return kTileTiers - 1;
}

// Tile of the fused window launch ("Pose windows"): choose_tier over the window histogram of the
// last launch that has published one with the same sampled image.  Until one has (the first call with a new
// image, or every call of a host that runs ahead of the GPU), the tier comes from a window probe of the
// first such batch: one small launch and a wait, once per sampled image.  Only the speed depends on the choice,
// never the results.
static hipError_t set_fused_tiles(pcore_ctx* c, int num_poses, FusedArgs& a, hipStream_t s) {
    const bool colour = a.cid != nullptr;
    const int nsamp = a.ws * a.hs;
    hipError_t e;
    if (!c->fb_host) {
        if ((e = hipHostMalloc((void**)&c->fb_host, 16 * sizeof(int32_t), hipHostMallocMapped)) != hipSuccess) return e;
        std::memset(c->fb_host, 0, 16 * sizeof(int32_t));
        c->fb_host[kTileTiers + 2] = -1;
        if ((e = hipHostGetDevicePointer((void**)&c->fb_dev, c->fb_host, 0)) != hipSuccess) return e;
        if ((e = dev_reserve(c->fb_ctr, 2)) != hipSuccess) return e;
        if ((e = dev_reserve(c->win_hist, 2 * (kTileTiers + 1))) != hipSuccess) return e;
        // captured launches' own counters, allocated here: no allocation may happen while a stream captures
        if ((e = dev_reserve(c->fb_ctr_cap, 2)) != hipSuccess) return e;
        if ((e = dev_reserve(c->win_hist_cap, 2 * (kTileTiers + 1))) != hipSuccess) return e;
        if ((e = hipMemset(c->fb_ctr.p, 0, 2 * sizeof(int32_t))) != hipSuccess) return e;
        if ((e = hipMemset(c->win_hist.p, 0, 2 * (kTileTiers + 1) * sizeof(int32_t))) != hipSuccess) return e;
    }
    // A captured launch counts into buffers of its own that nothing publishes or reads: its replays can
    // never add to the parity histograms the eager launches publish.  A stream whose capture state cannot be queried
    // (hipStreamIsCapturing fails, e.g. on the legacy stream while another stream captures in global mode) is treated
    // as capturing: no window probe, no feedback.
    hipStreamCaptureStatus cap = hipStreamCaptureStatusNone;
    if (hipStreamIsCapturing(s, &cap) != hipSuccess) {
        (void)hipGetLastError();
        cap = hipStreamCaptureStatusActive;
    }
    const bool capturing = cap != hipStreamCaptureStatusNone;
    int edge[kTileTiers];
    for (int t = 0; t < kTileTiers; t++) edge[t] = fused_tier_samples(t, a.ws, a.hs, a.bitmap_words, colour, c->dinfo);
    const long long key = (((long long)a.ws * 4096 + a.hs) * 65536 + a.bitmap_words) * 2 + (colour ? 1 : 0);
    bool published = false;
    if (key != c->tile_key) {
        c->tile_key = key;
        c->tile_key_seq = c->fb_seq + 1;
        c->tile_tier = kDefaultTier;
        c->tile_probed = false;
    } else {
        volatile int32_t* fb = c->fb_host;
        const int32_t seq = fb[kTileTiers + 2];
        if (seq >= c->tile_key_seq && seq <= c->fb_seq) {
            int32_t h[kTileTiers + 1];
            for (int b = 0; b <= kTileTiers; b++) h[b] = fb[b];
            c->tile_tier = choose_tier(h, edge, c->tile_tier);
            published = true;
        }
    }
    const char* env_tier = getenv("PCORE_FUSED_TIER");  // A/B + test knob; >= kTileTiers: whole image
    if (!published && !c->tile_probed && !capturing && !env_tier && !getenv("PCORE_NO_WINDOW_PROBE")) {
        if ((e = dev_reserve(c->win_probe, kTileTiers + 1)) != hipSuccess) return e;
        if ((e = hipMemsetAsync(c->win_probe.p, 0, (kTileTiers + 1) * sizeof(int32_t), s)) != hipSuccess) return e;
        for (int t = 0; t < kTileTiers; t++) a.hist_edge[t] = edge[t];
        if ((e = launch_window_probe(a, c->win_probe.p, s)) != hipSuccess) return e;
        int32_t h[kTileTiers + 1];
        if ((e = hipMemcpyAsync(h, c->win_probe.p, sizeof(h), hipMemcpyDeviceToHost, s)) != hipSuccess) return e;
        if ((e = hipStreamSynchronize(s)) != hipSuccess) return e;
        c->tile_tier = choose_tier(h, edge, c->tile_tier);
        c->tile_probed = true;
    }
    if (env_tier) c->tile_tier = std::min(std::max(atoi(env_tier), 0), kTileTiers);
    // tier kTileTiers (A/B knob only): the whole image
    a.tcap = c->tile_tier < kTileTiers && edge[c->tile_tier] > 0 ? edge[c->tile_tier] : nsamp;
    if (const char* env = getenv("PCORE_FUSED_TCAP"))  // test knob: a tile of this many samples (most poses overflow)
        a.tcap = std::min(std::max(atoi(env), 1), nsamp);
    for (int t = 0; t < kTileTiers; t++) a.hist_edge[t] = c->tile_edge[t] = edge[t];
    c->tile_tcap = a.tcap;
    a.fb_ctr = capturing ? c->fb_ctr_cap.p : c->fb_ctr.p;
    a.win_hist = capturing ? c->win_hist_cap.p : c->win_hist.p;
    a.fb_host = capturing ? nullptr : c->fb_dev;
    a.fb_seq = ++c->fb_seq;
    a.fb_par = a.fb_seq & 1;
    return hipSuccess;
}

static int ensure_sampled(pcore_ctx* c, int stride, hipStream_t s) {
    if (c->sampled_stride == stride) return PCORE_OK;
    c->generation++;  // a captured graph would read a source sampled at another stride
    const int ws = (c->cam.width + stride - 1) / stride, hs = (c->cam.height + stride - 1) / stride;
    HIPC(c, dev_reserve(c->src_s, (size_t)ws * hs));
    HIPC(c, dev_reserve(c->lab_s, (size_t)ws * hs));
    HIPC(c, launch_sample_source(c->src_depth.p, c->src_mask.p, c->cam.width, c->cam.height, stride, c->src_s.p,
                                 c->lab_s.p, s));
    c->sampled_stride = stride;
    return PCORE_OK;
}

// Every check pcore_evaluate makes before it launches anything.  pcore_evaluate_icp runs the same checks up
// front, so an invalid call fails before it writes any output.
static int validate_eval(pcore_ctx* c, const char* who, const float* d_poses, const int32_t* d_pose_model,
                         const int32_t* d_pose_label, const float* d_pose_obs_total, int32_t num_poses,
                         const pcore_eval_params* p, const float* d_out_rc, const float* d_out_oc,
                         const float* d_out_diff) {
    const std::string w(who);
    if (!c->have_mesh || !c->have_cam || !c->have_obs)
        return fail(c, PCORE_E_STATE, w + ": meshes, camera and observation must be set first");
    if (num_poses < 0 || (num_poses > 0 && (!d_poses || !d_pose_model || !d_out_rc)))
        return fail(c, PCORE_E_INVALID_ARG, w + ": null pose / output pointer");
    if (p->cost_type != PCORE_COST_DEPTH_3DOF && p->cost_type != PCORE_COST_DEPTH_6DOF &&
        p->cost_type != PCORE_COST_RGBD_3DOF)
        return fail(c, PCORE_E_INVALID_ARG, w + ": unknown cost_type");
    if (p->cost_type == PCORE_COST_RGBD_3DOF && (d_pose_label || !c->have_obs_colours))
        return fail(c, PCORE_E_INVALID_ARG,
                    w + ": cost_type 1 is 3-DoF (no pose labels) and needs pcore_set_observation_colors");
    if (num_poses == 0) return PCORE_OK;
    if (p->cost_type == PCORE_COST_DEPTH_6DOF && (!d_pose_label || !c->obs_has_mask))
        return fail(c, PCORE_E_INVALID_ARG, w + ": cost_type 2 needs pose labels and a source mask");
    if (p->calc_obs_cost && (!d_pose_obs_total || !d_out_oc || !d_out_diff))
        return fail(c, PCORE_E_INVALID_ARG, w + ": calc_obs_cost needs pose_obs_total and oc/diff outputs");
    const int W = c->cam.width, H = c->cam.height;
    if (p->stride <= 0 || W % p->stride != 0)
        return fail(c, PCORE_E_INVALID_ARG, w + ": width must be a multiple of stride");
    const int ws = W / p->stride, hs = (H + p->stride - 1) / p->stride;
    if (ws > 4095 || hs > 4095) return fail(c, PCORE_E_INVALID_ARG, w + ": sampled image too large");
    // the overflow launch holds the whole sampled image in LDS (the GICP cloud launch needs less: no bitmap)
    const size_t lds = fused_lds_bytes(ws * hs, c->bitmap_words, p->cost_type == PCORE_COST_RGBD_3DOF);
    if (lds > (size_t)c->prop.sharedMemPerBlock)
        return fail(c, PCORE_E_INVALID_ARG,
                    w + ": sampled z-buffer does not fit in LDS (use a larger stride); need " + std::to_string(lds) +
                        " B");
    return PCORE_OK;
}

static int evaluate_impl(pcore_ctx* c, const float* d_poses, const int32_t* d_pose_model, const int32_t* d_pose_label,
                         const float* d_pose_obs_total, int32_t num_poses, const pcore_eval_params* p, float* d_out_rc,
                         float* d_out_oc, float* d_out_diff, int32_t* d_dbg_zs, int64_t* d_keys, int64_t index_base,
                         int32_t num_models, pcore_stream stream) {
    if (!c || !p) return PCORE_E_INVALID_ARG;
    const int vr = validate_eval(c, "evaluate", d_poses, d_pose_model, d_pose_label, d_pose_obs_total, num_poses, p,
                                 d_out_rc, d_out_oc, d_out_diff);
    if (vr != PCORE_OK || num_poses == 0) return vr;
    const int W = c->cam.width, H = c->cam.height;
    const int ws = W / p->stride, hs = (H + p->stride - 1) / p->stride;
    HIPC(c, hipSetDevice(c->device));
    hipStream_t s = (hipStream_t)stream;
    int rc = ensure_sampled(c, p->stride, s);
    if (rc != PCORE_OK) return rc;

    FusedArgs a{};
    a.poses = d_poses;
    a.pose_model = d_pose_model;
    a.pose_label = (p->cost_type == PCORE_COST_DEPTH_6DOF) ? d_pose_label : nullptr;
    a.pose_obs_total = d_pose_obs_total;
    a.num_poses = num_poses;
    a.sverts = c->sverts.p;
    a.stris = c->stris.p;
    a.streams = c->streams.p;
    a.model_st_lo = c->model_st_lo.p;
    a.model_st_hi = c->model_st_hi.p;
    a.model_box = c->model_box.p;
    a.num_models = c->num_models;
    const float* pj = c->cam.proj;
    a.p00 = pj[0]; a.p01 = pj[1]; a.p02 = pj[2]; a.p03 = pj[3];
    a.p10 = pj[4]; a.p11 = pj[5]; a.p12 = pj[6]; a.p13 = pj[7];
    a.proj_sparse = (pj[1] == 0.0f && pj[3] == 0.0f && pj[4] == 0.0f && pj[7] == 0.0f) ? 1 : 0;
    a.width = W;
    a.height = H;
    a.stride = p->stride;
    a.ws = ws;
    a.hs = hs;
    a.cx = c->cam.cx; a.cy = c->cam.cy; a.fx = c->cam.fx; a.fy = c->cam.fy;
    a.depth_factor = p->depth_factor;
    a.src_s = c->src_s.p;
    a.lab_s = c->lab_s.p;
    a.grids = c->grids.p;
    a.cell_start = c->cell_start.p;
    a.grid_pts = c->grid_pts.p;
    a.num_grids = c->num_grids;
    a.bitmap_words = c->bitmap_words;
    a.r2 = p->sensor_resolution * p->sensor_resolution;  // renderer.cu:1877
    a.occlusion_threshold = p->occlusion_threshold;
    a.calc_obs = p->calc_obs_cost;
    a.out_rc = d_out_rc;
    a.out_oc = d_out_oc;
    a.out_diff = d_out_diff;
    a.dbg_zs = d_dbg_zs;
    if (p->cost_type == PCORE_COST_RGBD_3DOF) {
        a.stri_orig = c->stri_orig.p;
        a.tri_lab = c->tri_lab.p;
        a.obs_lab = c->obs_lab.p;
        a.colour_thr = p->color_distance_threshold;
        HIPC(c, reserve_gen(c, c->colour_id, (size_t)num_poses * ws * hs));
        a.cid = c->colour_id.p;
    }
    if (const char* e = getenv("PCORE_DEBUG_SKIP")) a.dbg_skip = atoi(e);
    a.sel_keys = d_keys;
    a.sel_base = index_base;
    a.sel_models = num_models;
    HIPC(c, set_fused_tiles(c, num_poses, a, s));
    HIPC(c, launch_fused_cost(a, s));
    return PCORE_OK;
}

int pcore_evaluate(pcore_ctx* c, const float* d_poses, const int32_t* d_pose_model, const int32_t* d_pose_label,
                   const float* d_pose_obs_total, int32_t num_poses, const pcore_eval_params* p, float* d_out_rc,
                   float* d_out_oc, float* d_out_diff, int32_t* d_dbg_zs, pcore_stream stream) {
    return evaluate_impl(c, d_poses, d_pose_model, d_pose_label, d_pose_obs_total, num_poses, p, d_out_rc, d_out_oc,
                         d_out_diff, d_dbg_zs, nullptr, 0, 0, stream);
}

int pcore_evaluate_select(pcore_ctx* c, const float* d_poses, const int32_t* d_pose_model,
                          const int32_t* d_pose_label, const float* d_pose_obs_total, int32_t num_poses,
                          const pcore_eval_params* p, float* d_out_rc, float* d_out_oc, float* d_out_diff,
                          int64_t index_base, int32_t num_models, int64_t* d_keys, pcore_stream stream) {
    if (!c) return PCORE_E_INVALID_ARG;
    if (num_models <= 0 || index_base < 0 || index_base + num_poses > 0x7fffffffLL || (num_poses > 0 && !d_keys))
        return fail(c, PCORE_E_INVALID_ARG, "evaluate_select: bad selection arguments");
    return evaluate_impl(c, d_poses, d_pose_model, d_pose_label, d_pose_obs_total, num_poses, p, d_out_rc, d_out_oc,
                         d_out_diff, nullptr, d_keys, index_base, num_models, stream);
}

static int fill_fused_args(pcore_ctx* c, const pcore_eval_params* p, FusedArgs& a) {
    const int W = c->cam.width, H = c->cam.height;
    const int ws = W / p->stride, hs = (H + p->stride - 1) / p->stride;
    a = FusedArgs{};
    a.sverts = c->sverts.p;
    a.stris = c->stris.p;
    a.streams = c->streams.p;
    a.model_st_lo = c->model_st_lo.p;
    a.model_st_hi = c->model_st_hi.p;
    a.model_box = c->model_box.p;
    a.num_models = c->num_models;
    const float* pj = c->cam.proj;
    a.p00 = pj[0]; a.p01 = pj[1]; a.p02 = pj[2]; a.p03 = pj[3];
    a.p10 = pj[4]; a.p11 = pj[5]; a.p12 = pj[6]; a.p13 = pj[7];
    a.proj_sparse = (pj[1] == 0.0f && pj[3] == 0.0f && pj[4] == 0.0f && pj[7] == 0.0f) ? 1 : 0;
    a.width = W;
    a.height = H;
    a.stride = p->stride;
    a.ws = ws;
    a.hs = hs;
    a.cx = c->cam.cx; a.cy = c->cam.cy; a.fx = c->cam.fx; a.fy = c->cam.fy;
    a.depth_factor = p->depth_factor;
    a.src_s = c->src_s.p;
    a.lab_s = c->lab_s.p;
    a.grids = c->grids.p;
    a.cell_start = c->cell_start.p;
    a.grid_pts = c->grid_pts.p;
    a.num_grids = c->num_grids;
    a.bitmap_words = c->bitmap_words;
    a.r2 = p->sensor_resolution * p->sensor_resolution;  // renderer.cu:1877
    a.occlusion_threshold = p->occlusion_threshold;
    a.calc_obs = p->calc_obs_cost;
    return PCORE_OK;
}

int pcore_evaluate_icp(pcore_ctx* c, const float* d_poses, const int32_t* d_pose_model, const int32_t* d_pose_label,
                       const float* d_pose_obs_total, int32_t num_poses, const pcore_eval_params* p,
                       const pcore_icp_params* ip, float* d_out_poses, int32_t* d_out_iters, float* d_out_rc,
                       float* d_out_oc, float* d_out_diff, pcore_stream stream) {
    if (!c || !p || !ip) return PCORE_E_INVALID_ARG;
    if (ip->k_correspondences <= 0 || ip->k_correspondences > 16 || ip->max_iterations < 0)
        return fail(c, PCORE_E_INVALID_ARG, "evaluate_icp: k_correspondences must be in [1, 16]");
    if (ip->cycle_exit_window < 0)
        return fail(c, PCORE_E_INVALID_ARG, "evaluate_icp: cycle_exit_window must be >= 0");
    if (num_poses > 0 && !d_out_poses) return fail(c, PCORE_E_INVALID_ARG, "evaluate_icp: null d_out_poses");
    if (p->cost_type != PCORE_COST_DEPTH_3DOF && p->cost_type != PCORE_COST_DEPTH_6DOF)
        return fail(c, PCORE_E_INVALID_ARG, "evaluate_icp: cost_type must be 0 or 2");
    // everything the final pcore_evaluate (the re-score) checks, before any chunk writes an output
    const int vr = validate_eval(c, "evaluate_icp", d_poses, d_pose_model, d_pose_label, d_pose_obs_total, num_poses,
                                 p, d_out_rc, d_out_oc, d_out_diff);
    if (vr != PCORE_OK || num_poses == 0) return vr;
    const bool six = p->cost_type == PCORE_COST_DEPTH_6DOF;
    const int W = c->cam.width;
    const int ws = W / p->stride, hs = (c->cam.height + p->stride - 1) / p->stride;
    HIPC(c, hipSetDevice(c->device));
    hipStream_t s = (hipStream_t)stream;
    int rc = ensure_sampled(c, p->stride, s);
    if (rc != PCORE_OK) return rc;
    const int k = ip->k_correspondences;
    // target covariances, once per (observation, k)
    const int nl = c->num_grids;
    if (six && c->cov_k_label != k) {
        HIPC(c, dev_reserve(c->tgt_cov_label, (size_t)6 * std::max(c->num_obs, 1)));
        HIPC(c, launch_covariances(c->tgt.p, c->seg_lo.p, c->seg_cnt.p, 0, nl, k, c->tgt_cov_label.p, s, kGridNNMin));
        HIPC(c, launch_covariances_grid(c->tgt.p, c->seg_lo_h.data(), c->seg_cnt_h.data(), nl, 0, c->grids.p,
                                        c->cell_start.p, c->grid_pts.p, k, c->tgt_cov_label.p, s));
        c->cov_k_label = k;
    }
    if (!six && c->cov_k_all != k) {
        HIPC(c, dev_reserve(c->tgt_cov_all, (size_t)6 * std::max(c->num_obs, 1)));
        HIPC(c, launch_covariances(c->tgt.p, c->seg_lo.p + nl, c->seg_cnt.p + nl, 0, 1, k, c->tgt_cov_all.p, s,
                                   kGridNNMin));
        HIPC(c, launch_covariances_grid(c->tgt.p, c->seg_lo_h.data() + nl, c->seg_cnt_h.data() + nl, 1, nl, c->grids.p,
                                        c->cell_start.p, c->grid_pts.p, k, c->tgt_cov_all.p, s));
        c->cov_k_all = k;
    }
    const int nsamp = ws * hs;
    // GICP scratch per pose: nsamp cloud slots (16 B) + covariances (48 B) + the iteration's correspondences (4 B)
    // and Mahalanobis matrices (48 B).  Chunks are as large as the budget below allows and equal in size: every
    // chunk ends with the tail of its slowest pose, so fewer chunks mean fewer tails.
    const size_t per_pose = (size_t)nsamp * 116 + (size_t)kCorrHist * std::min(nsamp, kCorrHistCap) * 4;
    // Up to 32 GiB (and at most 40 % of the free HBM): one chunk for 100k poses at 640x480 / stride 8.
    // Each chunk ends with the tail of its slowest pose, so on C3 (50k poses) one chunk instead of two
    // saves ~5 ms of a 37 ms step.
    size_t budget = (size_t)32 << 30;
    {
        size_t free_b = 0, total_b = 0;
        if (hipMemGetInfo(&free_b, &total_b) == hipSuccess && free_b > 0)
            budget = std::min(budget, std::max<size_t>((size_t)1 << 30, free_b / 5 * 2));
    }
    if (const char* e = getenv("PCORE_ICP_SCRATCH_GIB")) budget = (size_t)std::max(1, atoi(e)) << 30;  // A/B knob
    const int max_chunk = (int)std::max<size_t>(1, budget / per_pose);
    const int nchunks = (num_poses + max_chunk - 1) / max_chunk;
    const int chunk = (num_poses + nchunks - 1) / nchunks;
    HIPC(c, dev_reserve(c->icp_cloud, (size_t)chunk * nsamp));
    HIPC(c, dev_reserve(c->icp_count, (size_t)chunk));
    HIPC(c, dev_reserve(c->icp_cov, (size_t)6 * chunk * nsamp));
    HIPC(c, dev_reserve(c->icp_corr, (size_t)chunk * nsamp));
    // gicp_kernel's correspondence history: kCorrHist sets per pose of up to hist_cap points (C3's rendered clouds
    // hold <= 467 of 4,800 samples; larger clouds search every iteration)
    const int hist_cap = std::min(nsamp, kCorrHistCap);
    const bool use_hist = !getenv("PCORE_GICP_NO_HIST");  // A/B knob (same results)
    if (use_hist) HIPC(c, dev_reserve(c->icp_corr_hist, (size_t)chunk * kCorrHist * hist_cap));
    HIPC(c, dev_reserve(c->icp_mahal, (size_t)6 * chunk * nsamp));
    HIPC(c, dev_reserve(c->icp_counter, 4));  // [0] one-wave queue, [1] heavy queue, [2] heavy poses
    HIPC(c, dev_reserve(c->icp_iter_stats, 8));
    if (!c->icp_iter_stats_host)
        HIPC(c, hipHostMalloc((void**)&c->icp_iter_stats_host, 8 * sizeof(unsigned long long), hipHostMallocDefault));
    // the GICP help board (a -DPCORE_GICP_HELP_BOARD=1 build): a slot per resident wave, at most 512 MiB of granules
    // (PCORE_GICP_HELP=0: no help, A/B)
    int help_slots = 0;
    if (kGicpHelpBoard && !(getenv("PCORE_GICP_HELP") && atoi(getenv("PCORE_GICP_HELP")) == 0)) {
        const size_t per_slot = (size_t)(kHelpXfGranules + nsamp) * sizeof(unsigned long long);
        help_slots = (int)std::min<size_t>((size_t)std::max(1, c->dinfo.gicp_resident_wgs), ((size_t)512 << 20) / per_slot);
        HIPC(c, dev_reserve(c->icp_help_ctl, help_ctl_words(help_slots)));
        HIPC(c, dev_reserve(c->icp_help_gran, (size_t)help_slots * (kHelpXfGranules + nsamp)));
    }
    HIPC(c, dev_reserve(c->icp_order_keys, (size_t)2 * chunk));
    HIPC(c, dev_reserve(c->icp_order_idx, (size_t)2 * chunk));
    const size_t order_temp = gicp_order_temp_bytes(chunk);
    HIPC(c, dev_reserve(c->icp_order_temp, order_temp));
    FusedArgs a{};
    fill_fused_args(c, p, a);
    // gpu_stats (renderer.cu:1707, 1739): device memory in use at the GICP stage, events around it per chunk
    {
        size_t free_b = 0, total_b = 0;
        if (hipMemGetInfo(&free_b, &total_b) == hipSuccess)
            c->peak_mem_mb = std::max(c->peak_mem_mb, (double)(total_b - free_b) / 1024.0 / 1024.0);
    }
    hipStreamCaptureStatus cap_status = hipStreamCaptureStatusNone;
    HIPC(c, hipStreamIsCapturing(s, &cap_status));
    const bool timed = cap_status == hipStreamCaptureStatusNone;
    c->icp_ev_used = 0;
    HIPC(c, hipMemsetAsync(c->icp_iter_stats.p, 0, 8 * sizeof(unsigned long long), s));
    while (timed && c->icp_ev.size() < (size_t)3 * nchunks) {
        hipEvent_t e;
        HIPC(c, hipEventCreate(&e));
        c->icp_ev.push_back(e);
    }
    GicpArgs g{};
    g.src = c->icp_cloud.p;
    g.src_count = c->icp_count.p;
    g.src_cov = c->icp_cov.p;
    g.corr = c->icp_corr.p;
    g.mahal = c->icp_mahal.p;
    g.corr_hist = use_hist ? c->icp_corr_hist.p : nullptr;
    g.corr_hist_cap = hist_cap;
    g.src_cap = nsamp;
    g.tgt = c->tgt.p;
    g.tgt_cov = six ? c->tgt_cov_label.p : c->tgt_cov_all.p;
    g.seg_lo = c->seg_lo.p;
    g.seg_hi = c->seg_hi.p;
    g.num_segs = nl;
    g.whole_seg = nl;
    g.pose_label = six ? d_pose_label : nullptr;
    g.poses_in = d_poses;
    g.poses_out = d_out_poses;
    g.iters_out = d_out_iters;
    g.max_iter = ip->max_iterations;
    g.rot_eps = ip->rotation_epsilon;
    g.trans_eps = ip->transformation_epsilon;
    g.work_counter = c->icp_counter.p;
    g.heavy_counter = c->icp_counter.p + 1;
    g.heavy_count = c->icp_counter.p + 2;
    // heavy poses (a -DPCORE_GICP_WG_WAVES=4 build only): source points x targets >= 60,000 (e.g. 211 points on a
    // 285-target segment), at most 2 per CU; PCORE_GICP_HEAVY_COST / PCORE_GICP_HEAVY_MAX for A/B (0: none)
    g.heavy_cost = kGicpHeavyBuild ? 60000 : 0;
    g.heavy_max = 2 * std::max(1, c->dinfo.num_cus);
    if (const char* e = getenv("PCORE_GICP_HEAVY_COST")) g.heavy_cost = atoll(e);
    if (const char* e = getenv("PCORE_GICP_HEAVY_MAX")) g.heavy_max = atoi(e);
    g.cycle_window = ip->cycle_exit_window;
    g.iter_stats = c->icp_iter_stats.p;
    g.help_ctl = help_slots > 0 ? c->icp_help_ctl.p : nullptr;
    g.help_gran = help_slots > 0 ? c->icp_help_gran.p : nullptr;
    g.help_stats = c->icp_iter_stats.p + 4;
    g.help_slots = help_slots;
    g.tgt_quads = c->tgt_quads.p;
    g.seg_qoff = c->seg_qoff.p;
    g.grids = c->grids.p;
    g.cell_start = c->cell_start.p;
    g.grid_pts = c->grid_pts.p;
    // the GICP kernel instance with the grid search only when some segment the poses can use is large (gicp_pose:
    // use_grid = nt > kGridNNMin with grids present); 6-DoF poses use their label's segment, 3-DoF the whole cloud
    bool grid_needed = false;
    if (c->grids.p) {
        if (six) {
            for (int L = 0; L < nl; L++) grid_needed = grid_needed || segment_uses_grid(c->seg_cnt_h[L], true);
        } else {
            grid_needed = segment_uses_grid(c->seg_cnt_h[nl], true);
        }
    }
    for (int base = 0; base < num_poses; base += chunk) {
        const int n = std::min(chunk, num_poses - base);
        a.poses = d_poses + (size_t)16 * base;
        a.pose_model = d_pose_model + base;
        a.pose_label = six ? d_pose_label + base : nullptr;
        a.num_poses = n;
        a.cloud_out = c->icp_cloud.p;
        a.cloud_count = c->icp_count.p;
        a.cloud_cap = nsamp;
        // the fused launch's most-occupied tile (6 workgroups per CU); larger windows are rastered in chunks of it
        a.tcap = fused_tier_samples(0, a.ws, a.hs, 0, false, c->dinfo);
        if (const char* e = getenv("PCORE_FUSED_TCAP")) a.tcap = std::min(std::max(atoi(e), 1), a.ws * a.hs);
        if (a.tcap <= 0) a.tcap = a.ws * a.hs;
        // the source covariances in a launch of their own, or (PCORE_COV_FOLD=1, A/B) in render_cloud's launch; either
        // way bit-identical (pcore_cov.h).  Folded, the C3 step took 13.70 / 13.75 ms against 12.74 / 12.95 ms
        // (profiles/r06g/): render_cloud's workgroups hold their raster LDS (6 per CU) through the k-NN rounds, where
        // the covariance launch runs 32 one-wave workgroups per CU.
        const bool fold = k == 10 && getenv("PCORE_COV_FOLD") && atoi(getenv("PCORE_COV_FOLD")) == 1;
        a.cloud_cov = fold ? c->icp_cov.p : nullptr;
        // PCORE_COV_GICP=1: the covariances in gicp_kernel's pose prologue instead (launch_gicp runs the covariance
        // launch itself when it picks a kernel without the prologue); bit-identical
        const bool gfold = !fold && k == 10 && !getenv("PCORE_COV_BRUTE") && getenv("PCORE_COV_GICP") &&
                           atoi(getenv("PCORE_COV_GICP")) == 1;
        g.cov_fold = gfold ? c->icp_cov.p : nullptr;
        g.cov_fx = a.fx;
        g.cov_fy = a.fy;
        g.cov_cx = a.cx;
        g.cov_cy = a.cy;
        g.cov_stride = p->stride;
        hipEvent_t* ev = timed ? c->icp_ev.data() + 3 * c->icp_ev_used : nullptr;
        if (ev && fold) HIPC(c, hipEventRecord(ev[0], s));  // icp_runtime then spans the cloud + covariance launch
        HIPC(c, launch_render_cloud(a, s));
        if (ev && !fold) HIPC(c, hipEventRecord(ev[0], s));
        // the clouds' covariances: k = 10 by the threshold k-NN over each cloud's sample grid (pcore_cov.h;
        // PCORE_COV_BRUTE=1 restores the brute-force kernel for A/B), other k by the brute force; bit-identical
        if (!fold && !gfold && k == 10 && !getenv("PCORE_COV_BRUTE"))
            HIPC(c, launch_covariances_cloud(c->icp_cloud.p, c->icp_count.p, nsamp, n, a.fx, a.fy, a.cx, a.cy, p->stride,
                                             c->icp_cov.p, s));
        else if (!fold && !gfold)
            HIPC(c, launch_covariances(c->icp_cloud.p, nullptr, c->icp_count.p, nsamp, n, k, c->icp_cov.p, s));
        g.pose_base = base;
        g.pose_order = nullptr;
        HIPC(c, hipMemsetAsync(g.heavy_count, 0, sizeof(int32_t), s));
        if (!getenv("PCORE_GICP_INDEX_ORDER")) {  // A/B knob: the queue in index order
            HIPC(c, launch_gicp_order(g, n, c->icp_order_keys.p, c->icp_order_keys.p + chunk, c->icp_order_idx.p,
                                      c->icp_order_idx.p + chunk, c->icp_order_temp.p, order_temp, s));
            g.pose_order = c->icp_order_idx.p + chunk;
        }
        c->icp_help_tag = c->icp_help_tag % 0xFFFFu + 1u;  // a new tag for every launch on this context's board
        g.help_tag = c->icp_help_tag;
        if (ev) HIPC(c, hipEventRecord(ev[1], s));
        HIPC(c, launch_gicp(g, n, c->dinfo, s, grid_needed));
        if (ev)  // the counters so far (the last chunk's copy holds the call's totals)
            HIPC(c, hipMemcpyAsync(c->icp_iter_stats_host, c->icp_iter_stats.p, 8 * sizeof(unsigned long long),
                                   hipMemcpyDeviceToHost, s));
        if (ev) {
            HIPC(c, hipEventRecord(ev[2], s));
            c->icp_ev_used++;
        }
    }
    // re-render and re-score the adjusted poses (renderer.cu:1757-1907)
    return pcore_evaluate(c, d_out_poses, d_pose_model, d_pose_label, d_pose_obs_total, num_poses, p, d_out_rc,
                          d_out_oc, d_out_diff, nullptr, stream);
}

int pcore_render(pcore_ctx* c, const float* d_poses, const int32_t* d_pose_model, const int32_t* d_pose_label,
                 int32_t num_poses, float occlusion_threshold, int32_t* d_out_depth, uint8_t* d_out_color,
                 pcore_stream stream) {
    if (!c) return PCORE_E_INVALID_ARG;
    if (!c->have_mesh || !c->have_cam || !c->have_obs)
        return fail(c, PCORE_E_STATE, "render: meshes, camera and observation must be set first");
    if (num_poses < 0 || (num_poses > 0 && (!d_poses || !d_pose_model || !d_out_depth)))
        return fail(c, PCORE_E_INVALID_ARG, "render: null pointer");
    if (d_pose_label && !c->obs_has_mask)
        return fail(c, PCORE_E_INVALID_ARG, "render: pose labels need a source mask");
    if (num_poses == 0) return PCORE_OK;
    HIPC(c, hipSetDevice(c->device));
    hipStream_t s = (hipStream_t)stream;
    const int W = c->cam.width, H = c->cam.height;
    HIPC(c, launch_fill_i32(d_out_depth, INT_MAX, (size_t)num_poses * W * H, s));
    HIPC(c, launch_render_full(c->tris.p, c->num_tris, c->tri_lo.p, c->tri_hi.p, d_poses, d_pose_model, num_poses, W,
                               H, c->proj.p, d_out_depth, s));
    int32_t* tri_min = nullptr;
    if (d_out_color) {  // stage RENDER / DEBUG colour planes: the nearest triangle per pixel, second pass
        const size_t npx = (size_t)num_poses * W * H;
        HIPC(c, dev_reserve(c->render_tri, npx));
        tri_min = c->render_tri.p;
        HIPC(c, launch_fill_i32(tri_min, INT_MAX, npx, s));
        HIPC(c, launch_render_full_tri(c->tris.p, c->num_tris, c->tri_lo.p, c->tri_hi.p, d_poses, d_pose_model,
                                       num_poses, W, H, c->proj.p, d_out_depth, tri_min, s));
    }
    HIPC(c, launch_render_finalize(d_out_depth, c->src_depth.p, c->src_mask.p, d_pose_label, num_poses, W, H,
                                   occlusion_threshold, s, tri_min, d_out_color ? c->tri_rgb.p : nullptr, d_out_color));
    return PCORE_OK;
}

int pcore_get_stats(pcore_ctx* c, pcore_gpu_stats* out, int32_t reset) {
    if (!c || !out) return PCORE_E_INVALID_ARG;
    HIPC(c, hipSetDevice(c->device));
    double icp_ms = 0.0, gicp_ms = 0.0;
    for (int i = 0; i < c->icp_ev_used; i++) {
        hipEvent_t* ev = c->icp_ev.data() + 3 * i;
        HIPC(c, hipEventSynchronize(ev[2]));
        float a = 0.0f, b = 0.0f;
        HIPC(c, hipEventElapsedTime(&a, ev[0], ev[2]));
        HIPC(c, hipEventElapsedTime(&b, ev[1], ev[2]));
        icp_ms += a;
        gicp_ms += b;
    }
    out->icp_runtime = (float)(icp_ms * 1e-3);
    out->peak_memory_usage = c->peak_mem_mb;
    out->gicp_ms = (float)gicp_ms;
    out->icp_chunks = c->icp_ev_used;
    unsigned long long it[4] = {0ull, 0ull, 0ull, 0ull};
    if (c->icp_ev_used > 0 && c->icp_iter_stats_host)  // the last chunk's end event (after its copy) has completed
        for (int i = 0; i < 4; i++) it[i] = c->icp_iter_stats_host[i];
    if (it[3] != 0)
        return fail(c, PCORE_E_HIP, "evaluate_icp: " + std::to_string(it[3]) +
                                        " poses needed the grid search in the GICP instance without it");
    out->gicp_iterations = (int64_t)it[0];
    out->gicp_iterations_run = (int64_t)it[1];
    out->gicp_cycle_exits = (int64_t)it[2];
    if (reset) c->peak_mem_mb = 0.0;
    return PCORE_OK;
}

int pcore_debug_gicp_help_stats(pcore_ctx* c, int64_t* out4) {
    if (!c || !out4) return PCORE_E_INVALID_ARG;
    HIPC(c, hipSetDevice(c->device));
    for (int i = 0; i < 4; i++) out4[i] = 0;
    if (c->icp_ev_used <= 0 || !c->icp_iter_stats_host) return PCORE_OK;
    HIPC(c, hipEventSynchronize(c->icp_ev[3 * (c->icp_ev_used - 1) + 2]));  // after the last chunk's copy
    for (int i = 0; i < 4; i++) out4[i] = (int64_t)c->icp_iter_stats_host[4 + i];
    return PCORE_OK;
}

int pcore_get_tile_info(pcore_ctx* c, pcore_tile_info* out) {
    if (!c || !out) return PCORE_E_INVALID_ARG;
    static_assert(kTileTiers <= PCORE_MAX_TILE_TIERS, "pcore_tile_info holds the tiers");
    std::memset(out, 0, sizeof(*out));
    out->num_tiers = kTileTiers;
    out->tier = c->tile_tier;
    out->tcap = c->tile_tcap;
    out->seq = -1;
    for (int t = 0; t < kTileTiers; t++) {
        out->edge[t] = c->tile_edge[t];
        out->wgs_per_cu[t] = tier_wgs(t);
    }
    if (c->fb_host) {
        const volatile int32_t* fb = c->fb_host;
        for (int b = 0; b <= kTileTiers; b++) out->hist[b] = fb[b];
        out->chunked = fb[kTileTiers + 1];
        out->seq = fb[kTileTiers + 2];
    }
    return PCORE_OK;
}

int pcore_debug_lm_solve(const double* d_sys, const double* d_lambda, double* d_out, int32_t n, pcore_stream stream) {
    if (n < 0 || (n > 0 && (!d_sys || !d_lambda || !d_out))) return PCORE_E_INVALID_ARG;
    return launch_lm_solve_test(d_sys, d_lambda, d_out, n, (hipStream_t)stream) == hipSuccess ? PCORE_OK : PCORE_E_HIP;
}

int pcore_debug_covariances(const float* d_xyzw, const int32_t* d_seg_off, const int32_t* d_seg_cnt, int32_t num_segs,
                            int32_t k, double* d_out_cov6, pcore_stream stream) {
    if (num_segs < 0 || k <= 0 || k > 16 || (num_segs > 0 && (!d_xyzw || !d_seg_off || !d_seg_cnt || !d_out_cov6)))
        return PCORE_E_INVALID_ARG;
    return launch_covariances(reinterpret_cast<const float4*>(d_xyzw), d_seg_off, d_seg_cnt, 0, num_segs, k, d_out_cov6,
                              (hipStream_t)stream, INT_MAX) == hipSuccess ? PCORE_OK : PCORE_E_HIP;
}

int pcore_debug_covariances_cloud(const float* d_xyzw, const int32_t* d_seg_cnt, int32_t seg_stride, int32_t num_segs,
                                  float fx, float fy, float cx, float cy, int32_t stride, double* d_out_cov6,
                                  pcore_stream stream) {
    if (num_segs < 0 || seg_stride < 0 || stride <= 0 || (num_segs > 0 && (!d_xyzw || !d_seg_cnt || !d_out_cov6)))
        return PCORE_E_INVALID_ARG;
    return launch_covariances_cloud(reinterpret_cast<const float4*>(d_xyzw), d_seg_cnt, seg_stride, num_segs, fx, fy, cx,
                                    cy, stride, d_out_cov6, (hipStream_t)stream) == hipSuccess ? PCORE_OK : PCORE_E_HIP;
}

int pcore_depth_to_cloud(pcore_ctx* c, const int32_t* d_depth, int32_t num_poses, int32_t width, int32_t height,
                         int32_t stride, float depth_factor, const uint8_t* d_label_mask, const int32_t* d_pose_label,
                         float* d_out_xyz, int32_t* d_out_pose, int32_t* d_out_label, int32_t cap, int32_t* out_count,
                         pcore_stream stream) {
    return pcore_depth_to_cloud_ex(c, d_depth, num_poses, width, height, stride, depth_factor, d_label_mask,
                                   d_pose_label, nullptr, d_out_xyz, d_out_pose, d_out_label, nullptr, nullptr, cap,
                                   out_count, stream);
}

int pcore_depth_to_cloud_ex(pcore_ctx* c, const int32_t* d_depth, int32_t num_poses, int32_t width, int32_t height,
                            int32_t stride, float depth_factor, const uint8_t* d_label_mask, const int32_t* d_pose_label,
                            const uint8_t* d_color_planes, float* d_out_xyz, int32_t* d_out_pose, int32_t* d_out_label,
                            uint8_t* d_out_color, int32_t* d_out_dc_index, int32_t cap, int32_t* out_count,
                            pcore_stream stream) {
    if (!c) return PCORE_E_INVALID_ARG;
    if (!c->have_cam) return fail(c, PCORE_E_STATE, "depth_to_cloud: camera not set");
    if (num_poses < 0 || width <= 0 || height <= 0 || stride <= 0 || !d_depth || cap < 0 ||
        (cap > 0 && !d_out_xyz) || !out_count || (d_out_color && !d_color_planes))
        return fail(c, PCORE_E_INVALID_ARG, "depth_to_cloud: bad arguments");
    if (width % stride != 0) return fail(c, PCORE_E_INVALID_ARG, "depth_to_cloud: width % stride != 0");
    if (d_label_mask && num_poses != 1)
        return fail(c, PCORE_E_INVALID_ARG, "depth_to_cloud: label mask needs num_poses == 1");
    *out_count = 0;
    if (num_poses == 0) return PCORE_OK;
    HIPC(c, hipSetDevice(c->device));
    hipStream_t s = (hipStream_t)stream;
    HIPC(c, dev_reserve(c->scratch_counts, num_poses));
    HIPC(c, dev_reserve(c->scratch_offsets, num_poses));
    HIPC(c, dev_reserve(c->scratch_total, 1));
    const CloudBounds no_bounds{};
    HIPC(c, launch_cloud_count(d_depth, num_poses, width, height, stride, d_label_mask, no_bounds,
                               c->scratch_counts.p, s));
    HIPC(c, launch_exclusive_scan(c->scratch_counts.p, c->scratch_offsets.p, num_poses, c->scratch_total.p, s));
    HIPC(c, launch_cloud_write(d_depth, num_poses, width, height, stride, c->cam.cx, c->cam.cy, c->cam.fx, c->cam.fy,
                               depth_factor, d_label_mask, d_pose_label, c->scratch_offsets.p, d_out_xyz, d_out_pose,
                               d_out_label, cap, no_bounds, nullptr, nullptr, s, d_out_color ? d_color_planes : nullptr,
                               d_out_color));
    if (d_out_dc_index) {
        const size_t samples = (size_t)((width + stride - 1) / stride) * ((height + stride - 1) / stride);
        HIPC(c, dev_reserve(c->scratch_dc_pre, (size_t)num_poses * (samples + 1)));
        HIPC(c, launch_cloud_dc_index(d_depth, num_poses, width, height, stride, d_label_mask, c->scratch_offsets.p,
                                      c->scratch_dc_pre.p, d_out_dc_index, s));
    }
    int32_t total = 0;
    HIPC(c, hipMemcpyAsync(&total, c->scratch_total.p, 4, hipMemcpyDeviceToHost, s));
    HIPC(c, hipStreamSynchronize(s));
    *out_count = total;
    return PCORE_OK;
}

int pcore_select(pcore_ctx* c, const float* d_rc, const float* d_oc, const int32_t* d_pose_model, int32_t num_poses,
                 int64_t index_base, int32_t num_models, int64_t* d_keys, pcore_stream stream) {
    if (!c) return PCORE_E_INVALID_ARG;
    if (num_poses < 0 || num_models <= 0 || index_base < 0 || index_base + num_poses > 0x7fffffffLL ||
        (num_poses > 0 && (!d_rc || !d_oc || !d_pose_model || !d_keys)))
        return fail(c, PCORE_E_INVALID_ARG, "select: bad arguments");
    if (num_poses == 0) return PCORE_OK;
    HIPC(c, hipSetDevice(c->device));
    HIPC(c, launch_select(d_rc, d_oc, d_pose_model, num_poses, index_base, num_models, d_keys, (hipStream_t)stream));
    return PCORE_OK;
}

int pcore_count_within(pcore_ctx* c, const float* d_queries, const int32_t* d_labels, const float* d_radius_sq,
                       int32_t n, int32_t* d_out_counts, pcore_stream stream) {
    if (!c) return PCORE_E_INVALID_ARG;
    if (n < 0 || (n > 0 && (!d_queries || !d_labels || !d_radius_sq || !d_out_counts)))
        return fail(c, PCORE_E_INVALID_ARG, "count_within: null pointer");
    if (!c->have_obs) return fail(c, PCORE_E_STATE, "count_within: the observation must be set first");
    if (n == 0) return PCORE_OK;
    HIPC(c, hipSetDevice(c->device));
    HIPC(c, launch_count_within(d_queries, d_labels, d_radius_sq, n, c->tgt.p, c->seg_lo.p, c->seg_hi.p,
                                c->num_obs > 0 ? c->num_grids : 0, d_out_counts, (hipStream_t)stream));
    return PCORE_OK;
}

int pcore_state_poses(pcore_ctx* c, const double* d_states, const int32_t* d_model, const double* cam_from_world,
                      const double* d_preprocess, int32_t num_models, int32_t n, float* d_out_poses,
                      pcore_stream stream) {
    if (!c) return PCORE_E_INVALID_ARG;
    if (n < 0 || !cam_from_world || num_models <= 0 ||
        (n > 0 && (!d_states || !d_model || !d_preprocess || !d_out_poses)))
        return fail(c, PCORE_E_INVALID_ARG, "state_poses: bad arguments");
    if (n == 0) return PCORE_OK;
    HIPC(c, hipSetDevice(c->device));
    HIPC(c, launch_state_poses(d_states, d_model, d_preprocess, cam_from_world, num_models, n, d_out_poses,
                               (hipStream_t)stream));
    return PCORE_OK;
}

int pcore_pose_distances(pcore_ctx* c, const float* d_pts, int32_t n, const double* d_T_gt, const double* d_T_est,
                         int32_t num_pairs, double* d_add, double* d_adds, pcore_stream stream) {
    if (!c) return PCORE_E_INVALID_ARG;
    if (n <= 0 || num_pairs < 0 || (num_pairs > 0 && (!d_pts || !d_T_gt || !d_T_est)))
        return fail(c, PCORE_E_INVALID_ARG, "pose_distances: need n > 0 points and pose pointers");
    if (num_pairs == 0 || (!d_add && !d_adds)) return PCORE_OK;
    if (num_pairs > 65535) return fail(c, PCORE_E_INVALID_ARG, "pose_distances: at most 65535 pairs per call");
    HIPC(c, hipSetDevice(c->device));
    HIPC(c, dev_reserve(c->metric_part, (size_t)2 * num_pairs * pose_dist_blocks(n)));
    HIPC(c, launch_pose_distances(d_pts, n, d_T_gt, d_T_est, num_pairs, c->metric_part.p, d_add, d_adds,
                                  (hipStream_t)stream));
    return PCORE_OK;
}

}  // extern "C"
