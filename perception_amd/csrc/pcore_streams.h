// pcore_streams.h -- host-side builder of the fused kernel's vertex-ring streams (pcore_internal.h, kVRing;
// DESIGN.md, "Vertex-ring streams").  Plain C++ (no HIP): also compiled into tools/stream_stats for builder
// experiments on the CPU.
//
// Input: one model's triangles as unique-vertex ids (tv, 3 per triangle) and the vertex positions.  The
// triangles are put in a locality order (greedy adjacency growth, or a sweep of normal-binned surface patches when
// that needs fewer vertex passes), cut into `num_streams` contiguous streams
// of near-equal length, and every stream is turned into steps by simulating the kernel's vertex ring:
//   - a vertex pass loads the vertices the next triangles miss -- those not loaded by the previous pass --
//     in order of first use, up to 64;
//   - the following batches take triangles in order while all three vertices were loaded by the last two
//     passes (kRefPasses), 64 per step; a partial batch left when the next triangle needs a new pass is
//     carried past that pass (reloading its vertices the pass would age out), so batches stay full.
// Layout (no per-step header, so the kernel never waits on a separate uniform load): every triangle slot of a
// step carries the step's "vertex pass first" flag in bit 30, padding slots have bit 31 set, and a vertex
// slot's w is 1 for a vertex, 0 for padding.
// A triangle names each vertex by the ring slot of its latest load: (pass mod kVRing) * 64 + lane.
#pragma once
#include <algorithm>
#include <cmath>
#include <cstdint>
#include <cstring>
#include <vector>

namespace pcore {
namespace streams {

struct F4 {
    float x, y, z, w;
};
struct I4 {
    int32_t x, y, z, w;
};

struct Built {
    std::vector<F4> sverts;         // 64 per vertex pass
    std::vector<uint32_t> stris;    // 64 per step: i0 | i1 << 9 | i2 << 18 | vpass << 30, padding bit 31
    std::vector<uint32_t> sorig;    // 64 per step: original triangle index
    std::vector<I4> streams;        // (first step, end step, first pass, end pass)
    long long passes = 0, steps = 0, filled = 0;
};

// Greedy adjacency-growth order: grow a patch from the lowest unassigned triangle, always adding the
// unassigned neighbour that shares the most vertices with the last `window` vertices loaded (ties: lowest
// index), so consecutive triangles reuse recently loaded vertices.
inline std::vector<int> locality_order(const std::vector<int>& tv, int num_verts) {
    const int T = (int)tv.size() / 3;
    std::vector<std::vector<int>> adj(num_verts);
    for (int t = 0; t < T; t++)
        for (int k = 0; k < 3; k++) adj[tv[3 * t + k]].push_back(t);
    std::vector<char> done(T, 0);
    std::vector<int> order;
    order.reserve(T);
    std::vector<int> stamp(num_verts, -1);  // order position of the vertex's latest use
    int next_seed = 0;
    const int window = 96;  // "recent" = used by the last ~window/1.5 triangles
    std::vector<int> cand;
    while ((int)order.size() < T) {
        while (next_seed < T && done[next_seed]) next_seed++;
        int cur = next_seed;
        while (cur >= 0) {
            done[cur] = 1;
            const int pos = (int)order.size();
            order.push_back(cur);
            for (int k = 0; k < 3; k++) stamp[tv[3 * cur + k]] = pos;
            // candidates: unassigned triangles around the vertices of the last few triangles
            int best = -1, best_score = -1;
            const int lo = std::max(0, pos - 8);
            for (int q = pos; q >= lo; q--) {
                const int t = order[q];
                for (int k = 0; k < 3; k++)
                    for (int u : adj[tv[3 * t + k]]) {
                        if (done[u]) continue;
                        int score = 0;
                        for (int kk = 0; kk < 3; kk++) {
                            const int sv = stamp[tv[3 * u + kk]];
                            score += (sv >= 0 && pos - sv <= window) ? 1 : 0;
                        }
                        if (score > best_score || (score == best_score && u < best)) {
                            best_score = score;
                            best = u;
                        }
                    }
                if (best_score == 3) break;
            }
            cur = best;
        }
    }
    return order;
}

// Sweep order: triangles binned by the dominant axis (and sign) of their normal, each bin swept along the principal
// axis of its triangle centroids (stable for equal keys), so a bin is traversed in rows across its short extent.
// On the tessellated cylinders of the YCB proxies this halves the vertex reloads of the greedy growth order (the
// side's rows wrap around the axis and outgrow the two-pass window); on the boxes the greedy order stays ahead, so
// build_model keeps whichever order needs fewer vertex passes.
inline std::vector<int> sweep_order(const std::vector<int>& tv, const std::vector<float>& vxyz) {
    const int T = (int)tv.size() / 3;
    std::vector<int> bin(T);
    std::vector<float> cx(T), cy(T), cz(T);
    for (int t = 0; t < T; t++) {
        const float* a = &vxyz[3 * tv[3 * t]];
        const float* b = &vxyz[3 * tv[3 * t + 1]];
        const float* c = &vxyz[3 * tv[3 * t + 2]];
        const double ux = b[0] - a[0], uy = b[1] - a[1], uz = b[2] - a[2];
        const double vx = c[0] - a[0], vy = c[1] - a[1], vz = c[2] - a[2];
        const double nx = uy * vz - uz * vy, ny = uz * vx - ux * vz, nz = ux * vy - uy * vx;
        const double ax = std::fabs(nx), ay = std::fabs(ny), az = std::fabs(nz);
        int bb;
        if (!(ax == ax && ay == ay && az == az)) bb = 6;
        else if (ax >= ay && ax >= az) bb = nx >= 0 ? 0 : 1;
        else if (ay >= az) bb = ny >= 0 ? 2 : 3;
        else bb = nz >= 0 ? 4 : 5;
        bin[t] = bb;
        cx[t] = (a[0] + b[0] + c[0]) / 3.0f; cy[t] = (a[1] + b[1] + c[1]) / 3.0f; cz[t] = (a[2] + b[2] + c[2]) / 3.0f;
        if (!(cx[t] == cx[t] && cy[t] == cy[t] && cz[t] == cz[t])) { cx[t] = cy[t] = cz[t] = 0.0f; bin[t] = 6; }
    }
    std::vector<int> order;
    order.reserve(T);
    for (int bb = 0; bb < 7; bb++) {
        std::vector<int> ts;
        for (int t = 0; t < T; t++) if (bin[t] == bb) ts.push_back(t);
        if (ts.empty()) continue;
        // principal axis of the centroids (power iteration on the covariance)
        double m[3] = {0, 0, 0};
        for (int t : ts) { m[0] += cx[t]; m[1] += cy[t]; m[2] += cz[t]; }
        for (double& v : m) v /= ts.size();
        double C[3][3] = {{0}};
        for (int t : ts) {
            const double d[3] = {cx[t] - m[0], cy[t] - m[1], cz[t] - m[2]};
            for (int i = 0; i < 3; i++) for (int j = 0; j < 3; j++) C[i][j] += d[i] * d[j];
        }
        double e[3] = {1.0, 0.7, 0.4};
        for (int it = 0; it < 50; it++) {
            double f[3] = {0, 0, 0};
            for (int i = 0; i < 3; i++) for (int j = 0; j < 3; j++) f[i] += C[i][j] * e[j];
            const double n = std::sqrt(f[0] * f[0] + f[1] * f[1] + f[2] * f[2]);
            if (!(n > 0)) break;
            for (int i = 0; i < 3; i++) e[i] = f[i] / n;
        }
        std::vector<std::pair<double, int>> key;
        for (int t : ts) key.push_back({cx[t] * e[0] + cy[t] * e[1] + cz[t] * e[2], t});
        std::stable_sort(key.begin(), key.end(),
                         [](const std::pair<double, int>& p, const std::pair<double, int>& q) { return p.first < q.first; });
        for (auto& k : key) order.push_back(k.second);
    }
    return order;
}

constexpr int kNever = -(1 << 20);              // "latest pass" of a vertex no pass of the stream has loaded
constexpr uint32_t kStepVertexPass = 1u << 30;  // every triangle slot of a step that begins with a vertex pass
constexpr uint32_t kSlotPadding = 1u << 31;     // a triangle slot past the batch

// Append the streams of one model in the triangle order order0.  tri_base: index of the model's first triangle in the
// upload.  The order is cut into num_streams * chunks chunks and stream s concatenates chunks s, s + num_streams,
// ...: every wave's triangles are spread over the whole model, so the waves of a pose see similar numbers of
// visible (fragment-producing) triangles and meet at the end-of-raster barrier at similar times.  A chunk
// boundary only costs the reuse of one vertex pass.
inline void build_model_order(const std::vector<int>& tv, const std::vector<float>& vxyz, const std::vector<int>& order0,
                              int tri_base, int num_streams, int vring, int ref_passes, Built& out, int chunks) {
    const int T = (int)tv.size() / 3;
    if (T == 0) return;
    const int num_verts = (int)vxyz.size() / 3;
    const int S = std::max(1, std::min(num_streams, (T + 63) / 64));
    const int C = std::max(1, std::min(S * std::max(chunks, 1), (T + 255) / 256));  // chunks of >= ~256 triangles
    std::vector<int> order;
    order.reserve(T);
    std::vector<int> stream_end;
    for (int sidx = 0; sidx < S; sidx++) {
        for (int c = sidx; c < C; c += S) {
            const int c0 = (int)((long long)T * c / C), c1 = (int)((long long)T * (c + 1) / C);
            order.insert(order.end(), order0.begin() + c0, order0.begin() + c1);
        }
        stream_end.push_back((int)order.size());
    }
    std::vector<int> latest(num_verts, kNever), slot(num_verts, 0);
    std::vector<char> in_new(num_verts, 0);
    std::vector<int> newv, batch;
    for (int sidx = 0; sidx < S; sidx++) {
        const int b0 = sidx == 0 ? 0 : stream_end[sidx - 1], b1 = stream_end[sidx];
        I4 sd;
        sd.x = (int)(out.stris.size() / 64);
        sd.z = (int)(out.sverts.size() / 64);
        // fresh ring per stream
        for (int i = b0; i < b1; i++)
            for (int k = 0; k < 3; k++) latest[tv[3 * order[i] + k]] = kNever;
        int P = -1, i = b0;
        bool attached = true;  // the last vertex pass is announced by an emitted step
        batch.clear();
        auto emit = [&]() {  // one step: the pending batch (padded to 64), flagged if it follows a new pass
            const uint32_t vflag = attached ? 0u : kStepVertexPass;
            for (int t : batch) {
                const int v0 = tv[3 * t], v1 = tv[3 * t + 1], v2 = tv[3 * t + 2];
                out.stris.push_back((uint32_t)slot[v0] | ((uint32_t)slot[v1] << 9) | ((uint32_t)slot[v2] << 18) | vflag);
                out.sorig.push_back((uint32_t)(tri_base + t));
            }
            for (int k = (int)batch.size(); k < 64; k++) {
                out.stris.push_back(kSlotPadding | vflag);
                out.sorig.push_back(0u);
            }
            out.filled += (long long)batch.size();
            out.steps++;
            attached = true;
            batch.clear();
        };
        auto usable_after = [&](int t, int head) {  // all vertices loaded by passes > head - ref_passes
            for (int k = 0; k < 3; k++)
                if (latest[tv[3 * t + k]] <= head - ref_passes) return false;
            return true;
        };
        while (true) {
            // batches: triangles whose vertices were all loaded by the last ref_passes passes, 64 per step
            while (i < b1 && usable_after(order[i], P)) {
                batch.push_back(order[i++]);
                if ((int)batch.size() == 64) emit();
            }
            if (i >= b1) {
                if (!batch.empty() || !attached) emit();
                break;
            }
            // a new vertex pass P + 1.  A pending partial batch is carried into the next step when its vertices
            // stay referenceable after the pass -- reloading the few that would not -- unless the last pass has
            // no step yet (every pass is announced by the step after it) or the reloads would crowd the pass.
            newv.clear();
            if (!batch.empty()) {
                bool carry = attached;
                for (int t : batch)
                    for (int k = 0; k < 3 && carry; k++) {
                        const int v = tv[3 * t + k];
                        if (latest[v] > P + 1 - ref_passes || in_new[v]) continue;
                        in_new[v] = 1;
                        newv.push_back(v);
                        carry = (int)newv.size() <= 32;
                    }
                if (!carry) {
                    for (int v : newv) in_new[v] = 0;
                    newv.clear();
                    emit();
                }
            } else if (!attached) {
                emit();  // an empty step announces the last pass (never happens: a pass always enables a triangle)
            }
            // then the vertices the next triangles miss (not loaded by pass P), first use first
            for (int j = i; j < b1; j++) {
                int miss[3], nm = 0;
                for (int k = 0; k < 3; k++) {
                    const int v = tv[3 * order[j] + k];
                    if (latest[v] > P + 1 - ref_passes || in_new[v]) continue;
                    bool dup = false;
                    for (int q = 0; q < nm; q++) dup |= miss[q] == v;
                    if (!dup) miss[nm++] = v;
                }
                if ((int)newv.size() + nm > 64) break;
                for (int q = 0; q < nm; q++) {
                    in_new[miss[q]] = 1;
                    newv.push_back(miss[q]);
                }
            }
            P++;
            for (int k = 0; k < (int)newv.size(); k++) {
                const int v = newv[k];
                in_new[v] = 0;
                latest[v] = P;
                slot[v] = (P % vring) * 64 + k;
                out.sverts.push_back(F4{vxyz[3 * v], vxyz[3 * v + 1], vxyz[3 * v + 2], 1.0f});
            }
            for (int k = (int)newv.size(); k < 64; k++) out.sverts.push_back(F4{0.0f, 0.0f, 0.0f, 0.0f});  // w 0: padding
            out.passes++;
            attached = false;
        }
        sd.y = (int)(out.stris.size() / 64);
        sd.w = (int)(out.sverts.size() / 64);
        out.streams.push_back(sd);
    }
}

// Append the streams of one model, from the greedy growth order or the sweep order, whichever needs fewer vertex
// passes (then fewer steps; ties: the growth order).
inline void build_model(const std::vector<int>& tv, const std::vector<float>& vxyz, int tri_base, int num_streams,
                        int vring, int ref_passes, Built& out, int chunks = 4) {
    if (tv.empty()) return;
    Built a, b;
    build_model_order(tv, vxyz, locality_order(tv, (int)vxyz.size() / 3), tri_base, num_streams, vring, ref_passes, a,
                      chunks);
    build_model_order(tv, vxyz, sweep_order(tv, vxyz), tri_base, num_streams, vring, ref_passes, b, chunks);
    const Built& w = (b.passes < a.passes || (b.passes == a.passes && b.steps < a.steps)) ? b : a;
    const int step0 = (int)(out.stris.size() / 64), pass0 = (int)(out.sverts.size() / 64);
    out.sverts.insert(out.sverts.end(), w.sverts.begin(), w.sverts.end());
    out.stris.insert(out.stris.end(), w.stris.begin(), w.stris.end());
    out.sorig.insert(out.sorig.end(), w.sorig.begin(), w.sorig.end());
    for (I4 sd : w.streams) {
        sd.x += step0;
        sd.y += step0;
        sd.z += pass0;
        sd.w += pass0;
        out.streams.push_back(sd);
    }
    out.passes += w.passes;
    out.steps += w.steps;
    out.filled += w.filled;
}

}  // namespace streams
}  // namespace pcore
