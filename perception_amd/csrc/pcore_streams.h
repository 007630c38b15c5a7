// pcore_streams.h -- host-side builder of the fused kernel's vertex-ring streams (pcore_internal.h, kVRing;
// DESIGN.md, "Vertex-ring streams").  Plain C++ (no HIP): also compiled into tools/stream_stats for builder
// experiments on the CPU.
//
// Input: one model's triangles as unique-vertex ids (tv, 3 per triangle) and the vertex positions.  The
// triangles are put in a locality order (greedy adjacency growth), cut into `num_streams` contiguous streams
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

constexpr int kNever = -(1 << 20);
constexpr uint32_t kStepVertexPass = 1u << 30;  // every triangle slot of a step that begins with a vertex pass
constexpr uint32_t kSlotPadding = 1u << 31;     // a triangle slot past the batch  // "latest pass" of a vertex no pass of the stream has loaded

// Append the streams of one model.  tri_base: index of the model's first triangle in the upload.  The
// locality order is cut into num_streams * chunks chunks and stream s concatenates chunks s, s + num_streams,
// ...: every wave's triangles are spread over the whole model, so the waves of a pose see similar numbers of
// visible (fragment-producing) triangles and meet at the end-of-raster barrier at similar times.  A chunk
// boundary only costs the reuse of one vertex pass.
inline void build_model(const std::vector<int>& tv, const std::vector<float>& vxyz, int tri_base, int num_streams,
                        int vring, int ref_passes, Built& out, int chunks = 4) {
    const int T = (int)tv.size() / 3;
    if (T == 0) return;
    const int num_verts = (int)vxyz.size() / 3;
    const std::vector<int> order0 = locality_order(tv, num_verts);
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

}  // namespace streams
}  // namespace pcore
