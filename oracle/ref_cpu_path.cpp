// ref_cpu_path.cpp -- SURVEY.md 8(a) row a14: the reference's CPU/OMP path, restated.
//
// TEST INFRASTRUCTURE ONLY (the reported CPU baseline of bench.py and the checker of tests/).  Nothing in
// perception_amd/ links, loads or calls it.
//
// What it restates (all under /root/reference):
//   render_cpu + rasterization      cuda_renderer/src/renderer.cpp:228-330 (OMP over poses, full frame,
//                                   no source occlusion, plain `<` z-test on an INT_MAX buffer, INT_MAX -> 0)
//   depth2cloud_cpu                 cuda_icp/icp.cpp:64-108 (stride 1 only: the mask index x + y*width of
//                                   icp.cpp:73/96 overruns the W*H/s^2 mask for s > 1)
//   Scene_projective                cuda_icp/include/cuda_icp/depth_scene.h:7-50 (query),
//                                   cuda_icp/scene/depth_scene/depth_scene.cpp:3-35 (init: dep2pcd per pixel)
//   dep2pcd / pcd2dep               cuda_icp/include/cuda_icp/common.h (float order kept)
//   get_normal                      cuda_icp/scene/common.cpp:17-107 (linemod bilateral normals, r = 5)
//   thrust__pcd2Ab                  cuda_icp/include/cuda_icp/icp.h:135-209 (29-float row per point)
//   ICP_Point2Plane_cpu             cuda_icp/icp.cpp:116-179, ICPConvergenceCriteria(1e-5, 1e-5, 30) (icp.h:39-51)
//   eigen_slover_666                cuda_icp/icp.cpp:29-36: Eigen LDLT (diagonal pivoting) in double, then
//                                   TransformVector6dToMatrix4d (icp.cpp:7-17): R = AngleAxis(z) AngleAxis(y)
//                                   AngleAxis(x) evaluated as the quaternion product Eigen performs
//   Mat4x4f product                 cuda_icp/include/cuda_icp/geometry.h:292-298 (dot products summed from the
//                                   last index down, as `for (size_t i=DIM; i--; ret+=lhs[i]*rhs[i])`)
//
// Deterministic choices (the reference leaves them open): the OpenMP `reduction(+: reducer)` over points
// (icp.cpp:128-133) has no fixed order; here every pose runs on one thread and its points are summed in
// index order.  Poses run in parallel instead (the reference runs render_cpu over poses and ICP over
// points).  Eigen is not vendored (no headers in this image): LDLT and the AngleAxis products follow
// Eigen 3.3's published unblocked algorithms; parity of this row is therefore unpinned against the
// reference binary, like every other row.
#include "pcore_oracle.h"

#include <climits>
#include <cfloat>
#include <cmath>
#include <cstdint>
#include <cstdlib>
#include <vector>

#ifdef _OPENMP
#include <omp.h>
#endif

namespace {

struct V3 {
    float x, y, z;
};

// float -> int32 as the host compiles `int32_t(float)` / `int(float)` (x86 cvttss2si: NaN and out of
// range -> INT_MIN)
inline int32_t cvt_i32_host(float f) {
    if (!(f == f) || f >= 2147483648.0f || f < -2147483648.0f) return INT_MIN;
    return (int32_t)f;
}

// float -> size_t as g++ compiles it on x86-64 (values >= 2^63 through the subtract-and-xor branch,
// NaN -> 0 through that branch; negatives wrap through cvttss2si64)
inline uint64_t cvt_u64_host(float f) {
    if (f < 9223372036854775808.0f) {
        if (!(f == f)) return 0;
        return (uint64_t)(int64_t)f;
    }
    const float g = f - 9223372036854775808.0f;
    if (!(g == g) || g >= 9223372036854775808.0f) return 0;  // cvttss2si64 -> 2^63, xor 2^63 -> 0
    return ((uint64_t)(int64_t)g) ^ 0x8000000000000000ull;
}

inline float fmax_ref(float a, float b) { return (a > b) ? a : b; }  // std__max (renderer.h)
inline float fmin_ref(float a, float b) { return (a < b) ? a : b; }  // std__min

// mat_mul_v (renderer.h): ((m0 x + m1 y) + m2 z) + m3 per row of the 4x4 row-major matrix
inline V3 mat_mul_v(const float* m, const V3& v) {
    return {m[0] * v.x + m[1] * v.y + m[2] * v.z + m[3], m[4] * v.x + m[5] * v.y + m[6] * v.z + m[7],
            m[8] * v.x + m[9] * v.y + m[10] * v.z + m[11]};
}

inline float signed_area(const float* A, const float* B, const float* C) {
    return 0.5f * ((C[0] - A[0]) * (B[1] - A[1]) - (B[0] - A[0]) * (C[1] - A[1]));
}

// renderer.cpp:228-289 rasterization (ROI off): viewport, clamped bbox, barycentric test, perspective
// depth, `if (depth < depth_to_write) depth_to_write = depth`
void rasterize_cpu(const V3 tri[3], V3 last_row, int32_t* depth, int width, int height) {
    const float W = (float)width, H = (float)height;
    float pts2[3][2];
    const float lr[3] = {last_row.x, last_row.y, last_row.z};
    for (int i = 0; i < 3; i++) {
        pts2[i][0] = tri[i].x / lr[i] * W / 2.0f + W / 2.0f;
        pts2[i][1] = tri[i].y / lr[i] * H / 2.0f + H / 2.0f;
    }
    float bmin[2] = {FLT_MAX, FLT_MAX}, bmax[2] = {-FLT_MAX, -FLT_MAX};
    const float cmax[2] = {(float)(width - 1), (float)(height - 1)}, cmin[2] = {0.0f, 0.0f};
    for (int i = 0; i < 3; i++)
        for (int j = 0; j < 2; j++) {
            bmin[j] = fmax_ref(cmin[j], fmin_ref(bmin[j], pts2[i][j]));
            bmax[j] = fmin_ref(cmax[j], fmax_ref(bmax[j], pts2[i][j]));
        }
    for (uint64_t P1 = cvt_u64_host(bmin[1] + 0.5f); (float)P1 <= bmax[1]; P1 += 1) {
        for (uint64_t P0 = cvt_u64_host(bmin[0] + 0.5f); (float)P0 <= bmax[0]; P0 += 1) {
            const float fp[2] = {(float)P0, (float)P1};
            const float base_inv = 1 / signed_area(pts2[0], pts2[1], pts2[2]);
            const float beta = signed_area(pts2[0], fp, pts2[2]) * base_inv;
            const float gamma = signed_area(pts2[0], pts2[1], fp) * base_inv;
            const float bx = 1.0f - beta - gamma, by = beta, bz = gamma;
            if (bx < -0.0f || by < -0.0f || bz < -0.0f || bx > 1.0f || by > 1.0f || bz > 1.0f) continue;
            const float ox = bx / lr[0], oy = by / lr[1], oz = bz / lr[2];
            const float frag = (bx + by + bz) / (ox + oy + oz);
            const uint64_t xw = P0, yw = (uint64_t)(height - 1) - P1;
            const int32_t d = cvt_i32_host(frag + 0.5f);
            int32_t& dst = depth[xw + yw * (uint64_t)width];
            if (d < dst) dst = d;
        }
    }
}

void render_one(const float* tris, int num_tris, const float* pose, int width, int height, const float* proj,
                int32_t* depth) {
    const size_t npx = (size_t)width * height;
    for (size_t i = 0; i < npx; i++) depth[i] = INT_MAX;
    for (int t = 0; t < num_tris; t++) {
        const float* tr = tris + (size_t)9 * t;
        V3 local[3];
        for (int k = 0; k < 3; k++) local[k] = mat_mul_v(pose, V3{tr[3 * k], tr[3 * k + 1], tr[3 * k + 2]});
        const V3 last_row = {local[0].z, local[1].z, local[2].z};
        V3 scr[3];
        for (int k = 0; k < 3; k++) scr[k] = mat_mul_v(proj, local[k]);
        rasterize_cpu(scr, last_row, depth, width, height);
    }
    for (size_t i = 0; i < npx; i++)
        if (depth[i] == INT_MAX) depth[i] = 0;
}

// K as Mat3x3f rows: K[0][0] = fx, K[0][2] = cx, K[1][1] = fy, K[1][2] = cy
struct Intr {
    float fx, fy, cx, cy;
};

// depth2cloud_cpu, stride 1 (icp.cpp:64-108): row-major compaction of depth > 0 pixels, z = d / 100
int depth2cloud(const int32_t* depth, int width, int height, const Intr& K, V3* out, int cap) {
    int n = 0;
    for (int y = 0; y < height; y++)
        for (int x = 0; x < width; x++) {
            const int32_t d = depth[(size_t)x + (size_t)y * width];
            if (d <= 0) continue;
            const float z = (float)d / 100.0f;
            const float xp = ((float)(uint32_t)x - K.cx) / K.fx * z;
            const float yp = ((float)(uint32_t)y - K.cy) / K.fy * z;
            if (n < cap) out[n] = {xp, yp, z};
            n++;
        }
    return n;
}

// dep2pcd (common.h): dep == 0 -> (0, 0, 0)
inline V3 dep2pcd(size_t x, size_t y, uint32_t dep, const Intr& K) {
    if (dep == 0) return {0.0f, 0.0f, 0.0f};
    const float z = (float)dep / 100.0f;
    return {((float)x - K.cx) / K.fx * z, ((float)y - K.cy) / K.fy * z, z};
}

// accumBilateral (common.cpp:3-15)
inline void accum_bilateral(long delta, long i, long j, long* A, long* b, int threshold) {
    const long f = std::labs(delta) < threshold ? 1 : 0;
    const long fi = f * i, fj = f * j;
    A[0] += fi * i;
    A[1] += fi * j;
    A[3] += fj * j;
    b[0] += fi * delta;
    b[1] += fj * delta;
}

struct Mat4 {
    float m[4][4];
};

inline Mat4 mat4_identity() {
    Mat4 r;
    for (int i = 0; i < 4; i++)
        for (int j = 0; j < 4; j++) r.m[i][j] = (i == j) ? 1.0f : 0.0f;
    return r;
}

// geometry.h:292-298: result[i][j] = lhs[i] . rhs.col(j), the dot summed from index 3 down to 0
inline Mat4 mat4_mul(const Mat4& a, const Mat4& b) {
    Mat4 r;
    for (int i = 0; i < 4; i++)
        for (int j = 0; j < 4; j++) {
            float acc = 0.0f;
            for (int k = 4; k--;) acc += a.m[i][k] * b.m[k][j];
            r.m[i][j] = acc;
        }
    return r;
}

// Eigen 3.3 LDLT<Matrix<double,6,6>, Lower>: unblocked in-place factorisation with diagonal pivoting
// (largest |diagonal| of the trailing corner), then solve P^T L^-T D^+ L^-1 P b (LDLT.h).
void ldlt_solve6(const double A_in[36] /*column-major*/, const double b_in[6], double x[6]) {
    double m[6][6];
    for (int i = 0; i < 6; i++)
        for (int j = 0; j < 6; j++) m[i][j] = A_in[i + 6 * j];
    int trans[6];
    double temp[6];
    const int n = 6;
    for (int k = 0; k < n; k++) {
        int big = k;
        double bigv = std::fabs(m[k][k]);
        for (int i = k + 1; i < n; i++)
            if (std::fabs(m[i][i]) > bigv) { bigv = std::fabs(m[i][i]); big = i; }
        trans[k] = big;
        if (k != big) {
            for (int j = 0; j < k; j++) std::swap(m[k][j], m[big][j]);
            for (int i = big + 1; i < n; i++) std::swap(m[i][k], m[i][big]);
            std::swap(m[k][k], m[big][big]);
            for (int i = k + 1; i < big; i++) {
                const double t = m[i][k];
                m[i][k] = m[big][i];
                m[big][i] = t;
            }
        }
        const int rs = n - k - 1;
        if (k > 0) {
            for (int j = 0; j < k; j++) temp[j] = m[j][j] * m[k][j];
            double dot = 0.0;
            for (int j = 0; j < k; j++) dot += m[k][j] * temp[j];
            m[k][k] -= dot;
            for (int i = k + 1; i < n; i++) {
                double s = 0.0;
                for (int j = 0; j < k; j++) s += m[i][j] * temp[j];
                m[i][k] -= s;
            }
        }
        const double akk = m[k][k];
        if (rs > 0 && std::fabs(akk) > 0.0)
            for (int i = k + 1; i < n; i++) m[i][k] /= akk;
    }
    double d[6];
    for (int i = 0; i < n; i++) d[i] = b_in[i];
    for (int k = 0; k < n; k++)
        if (trans[k] != k) std::swap(d[k], d[trans[k]]);
    for (int i = 0; i < n; i++)  // L (unit lower) forward substitution
        for (int j = 0; j < i; j++) d[i] -= m[i][j] * d[j];
    const double tol = DBL_MIN;
    for (int i = 0; i < n; i++) d[i] = (std::fabs(m[i][i]) > tol) ? d[i] / m[i][i] : 0.0;
    for (int i = n - 1; i >= 0; i--)  // L^T back substitution
        for (int j = i + 1; j < n; j++) d[i] -= m[j][i] * d[j];
    for (int k = n - 1; k >= 0; k--)
        if (trans[k] != k) std::swap(d[k], d[trans[k]]);
    for (int i = 0; i < n; i++) x[i] = d[i];
}

struct Quat {
    double w, x, y, z;
};

inline Quat quat_mul(const Quat& a, const Quat& b) {  // Eigen quat_product
    return {a.w * b.w - a.x * b.x - a.y * b.y - a.z * b.z, a.w * b.x + a.x * b.w + a.y * b.z - a.z * b.y,
            a.w * b.y + a.y * b.w + a.z * b.x - a.x * b.z, a.w * b.z + a.z * b.w + a.x * b.y - a.y * b.x};
}

// TransformVector6dToMatrix4d (icp.cpp:7-17) -> .cast<float>() (icp.cpp:35)
Mat4 vec6_to_mat4(const double u[6]) {
    const Quat qz = {std::cos(u[2] / 2), 0.0, 0.0, std::sin(u[2] / 2)};
    const Quat qy = {std::cos(u[1] / 2), 0.0, std::sin(u[1] / 2), 0.0};
    const Quat qx = {std::cos(u[0] / 2), std::sin(u[0] / 2), 0.0, 0.0};
    const Quat q = quat_mul(quat_mul(qz, qy), qx);
    const double tx = 2.0 * q.x, ty = 2.0 * q.y, tz = 2.0 * q.z;
    const double twx = tx * q.w, twy = ty * q.w, twz = tz * q.w;
    const double txx = tx * q.x, txy = ty * q.x, txz = tz * q.x;
    const double tyy = ty * q.y, tyz = tz * q.y, tzz = tz * q.z;
    const double R[3][3] = {{1.0 - (tyy + tzz), txy - twz, txz + twy},
                            {txy + twz, 1.0 - (txx + tzz), tyz - twx},
                            {txz - twy, tyz + twx, 1.0 - (txx + tyy)}};
    Mat4 r = mat4_identity();
    for (int i = 0; i < 3; i++) {
        for (int j = 0; j < 3; j++) r.m[i][j] = (float)R[i][j];
        r.m[i][3] = (float)u[3 + i];
    }
    return r;
}

struct SceneProj {
    int width, height;
    float max_dist_diff;
    Intr K;
    const float* pcd;     // W*H*3
    const float* normal;  // W*H*3
};

// Scene_projective::query (depth_scene.h:25-48) with pcd2dep (common.h)
inline bool scene_query(const SceneProj& sc, const V3& s, V3& dst, V3& nrm) {
    const int x = cvt_i32_host(s.x / s.z * sc.K.fx + sc.K.cx - 0.0f + 0.5f);
    const int y = cvt_i32_host(s.y / s.z * sc.K.fy + sc.K.cy - 0.0f + 0.5f);
    if ((size_t)(int64_t)x >= (size_t)sc.width || (size_t)(int64_t)y >= (size_t)sc.height || x < 0 || y < 0)
        return false;
    const size_t idx = (size_t)x + (size_t)y * sc.width;
    dst = {sc.pcd[3 * idx], sc.pcd[3 * idx + 1], sc.pcd[3 * idx + 2]};
    const float dz = s.z - dst.z;
    const float adz = (dz > 0) ? dz : -dz;  // std__abs
    if (dst.z <= 0 || adz > sc.max_dist_diff) return false;
    nrm = {sc.normal[3 * idx], sc.normal[3 * idx + 1], sc.normal[3 * idx + 2]};
    return true;
}

// thrust__pcd2Ab (icp.h:135-209) accumulated in index order into a float[29]
inline void pcd2ab_accum(const SceneProj& sc, const V3& s, float acc[29]) {
    V3 d, n;
    if (!scene_query(sc, s, d, n)) return;
    float r[29];
    r[28] = 1;
    const float ex = d.x - s.x, ey = d.y - s.y, ez = d.z - s.z;
    const float b = ex * n.x + ey * n.y + ez * n.z;
    r[27] = b * b;
    float A[6];
    A[0] = n.z * s.y - n.y * s.z;
    A[1] = n.x * s.z - n.z * s.x;
    A[2] = n.y * s.x - n.x * s.y;
    A[3] = n.x;
    A[4] = n.y;
    A[5] = n.z;
    int sh = 0;
    for (int i = 0; i < 6; i++)
        for (int j = i; j < 6; j++) r[sh++] = A[i] * A[j];
    for (int i = 0; i < 6; i++) r[21 + i] = A[i] * b;
    for (int i = 0; i < 29; i++) acc[i] += r[i];
}

// ICP_Point2Plane_cpu (icp.cpp:116-179).  Returns the iteration at which it returned.
int icp_point2plane(std::vector<V3>& pcd, const SceneProj& sc, float rel_fitness, float rel_rmse, int max_iter,
                    Mat4& T, float& fitness, float& rmse) {
    T = mat4_identity();
    fitness = 0.0f;
    rmse = 0.0f;
    for (int iter = 0; iter <= max_iter; iter++) {
        float acc[29] = {0};
        for (size_t i = 0; i < pcd.size(); i++) pcd2ab_accum(sc, pcd[i], acc);
        const float prev_fit = fitness, prev_rmse = rmse;
        const float count = acc[28], total = acc[27];
        if (count == 0) return iter;
        fitness = float(count) / (float)pcd.size();
        rmse = std::sqrt(total / count);
        if (iter == max_iter) return iter;
        const float df = fitness - prev_fit, dr = rmse - prev_rmse;
        if (std::fabs(df) < rel_fitness && std::fabs(dr) < rel_rmse) return iter;
        double A[36], b[6], u[6];
        for (int i = 0; i < 6; i++) b[i] = (double)acc[21 + i];
        int sh = 0;
        for (int y = 0; y < 6; y++)
            for (int x = y; x < 6; x++) {
                A[x + y * 6] = (double)acc[sh];
                A[y + x * 6] = (double)acc[sh];
                sh++;
            }
        ldlt_solve6(A, b, u);
        const Mat4 E = vec6_to_mat4(u);
        for (auto& p : pcd) {  // transform_pcd (icp.cpp:38-51)
            const float nx = E.m[0][0] * p.x + E.m[0][1] * p.y + E.m[0][2] * p.z + E.m[0][3];
            const float ny = E.m[1][0] * p.x + E.m[1][1] * p.y + E.m[1][2] * p.z + E.m[1][3];
            const float nz = E.m[2][0] * p.x + E.m[2][1] * p.y + E.m[2][2] * p.z + E.m[2][3];
            p = {nx, ny, nz};
        }
        T = mat4_mul(E, T);
    }
    return max_iter;
}

}  // namespace

extern "C" {

void orc_ref_render_cpu(const float* tris, int num_tris, const float* poses, int num_poses, int width, int height,
                        const float* proj, int32_t* out, int nthreads) {
#ifdef _OPENMP
    if (nthreads > 0) omp_set_num_threads(nthreads);
#pragma omp parallel for schedule(dynamic, 1)
#endif
    for (int i = 0; i < num_poses; i++)
        render_one(tris, num_tris, poses + (size_t)16 * i, width, height, proj, out + (size_t)i * width * height);
}

int orc_ref_depth2cloud(const int32_t* depth, int width, int height, float fx, float fy, float cx, float cy,
                        float* out_xyz, int cap) {
    std::vector<V3> tmp((size_t)width * height);
    const int n = depth2cloud(depth, width, height, Intr{fx, fy, cx, cy}, tmp.data(), (int)tmp.size());
    for (int i = 0; i < n && i < cap; i++) {
        out_xyz[3 * i] = tmp[i].x;
        out_xyz[3 * i + 1] = tmp[i].y;
        out_xyz[3 * i + 2] = tmp[i].z;
    }
    return n;
}

void orc_ref_scene(const int32_t* depth, int width, int height, float fx, float fy, float cx, float cy,
                   float* out_pcd, float* out_normal) {
    const Intr K{fx, fy, cx, cy};
    // depth_scene.cpp:24-29 (CV_32S read as uint32)
    for (int r = 0; r < height; r++)
        for (int c = 0; c < width; c++) {
            const V3 p = dep2pcd(c, r, (uint32_t)depth[(size_t)c + (size_t)r * width], K);
            const size_t i = (size_t)c + (size_t)r * width;
            out_pcd[3 * i] = p.x;
            out_pcd[3 * i + 1] = p.y;
            out_pcd[3 * i + 2] = p.z;
        }
    // get_normal (common.cpp:17-107): CV_32S -> CV_16U (saturate), linemod normals, zero elsewhere
    std::vector<uint16_t> d16((size_t)width * height);
    for (size_t i = 0; i < d16.size(); i++) {
        const int32_t v = depth[i];
        d16[i] = (uint16_t)(v < 0 ? 0 : (v > 65535 ? 65535 : v));
    }
    for (size_t i = 0; i < (size_t)width * height * 3; i++) out_normal[i] = 0.0f;
    const int distance_threshold = 2000, difference_threshold = 50, l_r = 5;
    const int W = width, H = height;
    const int off[8] = {-l_r - l_r * W, 0 - l_r * W, +l_r - l_r * W, -l_r, +l_r, -l_r + l_r * W, 0 + l_r * W,
                        +l_r + l_r * W};
    const int di[8] = {-l_r, 0, +l_r, -l_r, +l_r, -l_r, 0, +l_r};
    const int dj[8] = {-l_r, -l_r, -l_r, 0, 0, +l_r, +l_r, +l_r};
    for (int y = l_r; y < H - l_r - 1; ++y)
        for (int x = l_r; x < W - l_r - 1; ++x) {
            const uint16_t* line = d16.data() + (size_t)y * W + x;
            const long d = line[0];
            if (!(d < distance_threshold)) continue;
            long A[4] = {0, 0, 0, 0}, b[2] = {0, 0};
            for (int k = 0; k < 8; k++) accum_bilateral((long)line[off[k]] - d, di[k], dj[k], A, b, difference_threshold);
            const long det = A[0] * A[3] - A[1] * A[1];
            const long ddx = A[3] * b[0] - A[1] * b[1];
            const long ddy = -A[1] * b[0] + A[0] * b[1];
            float nx = (float)(K.fx * (float)ddx);
            float ny = (float)(K.fy * (float)ddy);
            float nz = (float)(-det * d);
            const float sq = std::sqrt(nx * nx + ny * ny + nz * nz);
            if (sq > 0) {
                const float inv = 1.0f / sq;
                nx *= inv;
                ny *= inv;
                nz *= inv;
                const size_t i = (size_t)y * W + x;
                out_normal[3 * i] = nx;
                out_normal[3 * i + 1] = ny;
                out_normal[3 * i + 2] = nz;
            }
        }
}

int orc_ref_icp(float* model_xyz, int n, const float* scene_pcd, const float* scene_normal, int width, int height,
                float fx, float fy, float cx, float cy, float max_dist_diff, float rel_fitness, float rel_rmse,
                int max_iter, float* out_T, float* out_fitness, float* out_rmse) {
    std::vector<V3> pcd(n);
    for (int i = 0; i < n; i++) pcd[i] = {model_xyz[3 * i], model_xyz[3 * i + 1], model_xyz[3 * i + 2]};
    const SceneProj sc{width, height, max_dist_diff, Intr{fx, fy, cx, cy}, scene_pcd, scene_normal};
    Mat4 T;
    float fit, rmse;
    const int it = icp_point2plane(pcd, sc, rel_fitness, rel_rmse, max_iter, T, fit, rmse);
    for (int i = 0; i < 4; i++)
        for (int j = 0; j < 4; j++) out_T[4 * i + j] = T.m[i][j];
    for (int i = 0; i < n; i++) {
        model_xyz[3 * i] = pcd[i].x;
        model_xyz[3 * i + 1] = pcd[i].y;
        model_xyz[3 * i + 2] = pcd[i].z;
    }
    *out_fitness = fit;
    *out_rmse = rmse;
    return it;
}

// eigen_slover_666 (icp.cpp:29-36): A (column-major 6x6 float), b (6 float) -> float 4x4 row-major
void orc_ref_solver666(const float* A, const float* b, float* out_T) {
    double Ad[36], bd[6], u[6];
    for (int i = 0; i < 36; i++) Ad[i] = (double)A[i];
    for (int i = 0; i < 6; i++) bd[i] = (double)b[i];
    ldlt_solve6(Ad, bd, u);
    const Mat4 E = vec6_to_mat4(u);
    for (int i = 0; i < 4; i++)
        for (int j = 0; j < 4; j++) out_T[4 * i + j] = E.m[i][j];
}

// The whole a14 path per pose: render_cpu -> depth2cloud_cpu (stride 1) -> ICP_Point2Plane_cpu against the
// projective scene of `scene_depth` (int32 cm).  Poses run in parallel, one per thread.
void orc_ref_cpu_pipeline(const float* tris, int num_tris, const float* poses, int num_poses, int width, int height,
                          const float* proj, float fx, float fy, float cx, float cy, const int32_t* scene_depth,
                          float max_dist_diff, float rel_fitness, float rel_rmse, int max_iter, float* out_T,
                          float* out_fitness, float* out_rmse, int32_t* out_iters, int32_t* out_points,
                          int nthreads) {
    const size_t npx = (size_t)width * height;
    std::vector<float> spcd(npx * 3), snrm(npx * 3);
    orc_ref_scene(scene_depth, width, height, fx, fy, cx, cy, spcd.data(), snrm.data());
    const SceneProj sc{width, height, max_dist_diff, Intr{fx, fy, cx, cy}, spcd.data(), snrm.data()};
#ifdef _OPENMP
    if (nthreads > 0) omp_set_num_threads(nthreads);
#pragma omp parallel
#endif
    {
        std::vector<int32_t> depth(npx);
        std::vector<V3> cloud(npx);
#ifdef _OPENMP
#pragma omp for schedule(dynamic, 1)
#endif
        for (int i = 0; i < num_poses; i++) {
            render_one(tris, num_tris, poses + (size_t)16 * i, width, height, proj, depth.data());
            const int n = depth2cloud(depth.data(), width, height, sc.K, cloud.data(), (int)npx);
            std::vector<V3> pcd(cloud.begin(), cloud.begin() + n);
            Mat4 T;
            float fit, rmse;
            const int it = icp_point2plane(pcd, sc, rel_fitness, rel_rmse, max_iter, T, fit, rmse);
            for (int r = 0; r < 4; r++)
                for (int c = 0; c < 4; c++) out_T[(size_t)16 * i + 4 * r + c] = T.m[r][c];
            out_fitness[i] = fit;
            out_rmse[i] = rmse;
            if (out_iters) out_iters[i] = it;
            if (out_points) out_points[i] = n;
        }
    }
}

}  // extern "C"
