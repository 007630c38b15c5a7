// Builder statistics of the fused kernel's vertex-ring streams (perception_amd/csrc/pcore_streams.h) for one
// mesh, on the CPU: g++ -O2 -shared -fPIC tools/stream_stats.cpp -o tools/bin/libstreamstats.so
#include <cstring>
#include <unordered_map>

#include "../perception_amd/csrc/pcore_streams.h"

extern "C" int stream_stats(const float* tri_xyz, int T, int num_streams, int vring, int ref_passes, int chunks,
                            long long* out) {
    struct K { uint32_t x, y, z; bool operator==(const K& o) const { return x == o.x && y == o.y && z == o.z; } };
    struct H { size_t operator()(const K& k) const { return (size_t)k.x * 73856093u ^ (size_t)k.y * 19349663u ^ (size_t)k.z * 83492791u; } };
    std::unordered_map<K, int, H> idx;
    std::vector<int> tv(3 * (size_t)T);
    std::vector<float> vxyz;
    for (int t = 0; t < T; t++)
        for (int k = 0; k < 3; k++) {
            const float* p = tri_xyz + 9 * (size_t)t + 3 * k;
            K key;
            std::memcpy(&key.x, p, 4); std::memcpy(&key.y, p + 1, 4); std::memcpy(&key.z, p + 2, 4);
            auto it = idx.find(key);
            int id;
            if (it == idx.end()) { id = (int)vxyz.size() / 3; idx.emplace(key, id); vxyz.insert(vxyz.end(), p, p + 3); }
            else id = it->second;
            tv[3 * (size_t)t + k] = id;
        }
    pcore::streams::Built b;
    pcore::streams::build_model(tv, vxyz, 0, num_streams, vring, ref_passes, b, chunks);
    out[0] = b.passes; out[1] = b.steps; out[2] = (long long)vxyz.size() / 3; out[3] = T;
    out[4] = b.filled;
    long long vfill = 0;
    for (const auto& v : b.sverts) vfill += v.w != 0.0f ? 1 : 0;
    out[5] = vfill;
    return 0;
}

// Invariants of the builder's output that the fused kernel relies on (tests/test_streams.py): every triangle in
// exactly one slot; all 64 slots of a step carry the same "vertex pass first" flag and each flagged step consumes
// the stream's next pass; a triangle slot names, for each of its vertices in the triangle's own order, a ring slot
// that holds that vertex's exact position and was written by one of the last ref_passes passes; padding slots have
// bit 31; stream descriptors tile the step / pass arrays.  Returns 0, or the negative number of the first broken
// invariant; info: passes, steps, unique vertices, streams.
extern "C" int stream_check(const float* tri_xyz, int T, int num_streams, int vring, int ref_passes, int chunks,
                            long long* info) {
    struct K { uint32_t x, y, z; bool operator==(const K& o) const { return x == o.x && y == o.y && z == o.z; } };
    struct H { size_t operator()(const K& k) const { return (size_t)k.x * 73856093u ^ (size_t)k.y * 19349663u ^ (size_t)k.z * 83492791u; } };
    std::unordered_map<K, int, H> idx;
    std::vector<int> tv(3 * (size_t)T);
    std::vector<float> vxyz;
    for (int t = 0; t < T; t++)
        for (int k = 0; k < 3; k++) {
            const float* p = tri_xyz + 9 * (size_t)t + 3 * k;
            K key;
            std::memcpy(&key.x, p, 4); std::memcpy(&key.y, p + 1, 4); std::memcpy(&key.z, p + 2, 4);
            auto it = idx.find(key);
            int id;
            if (it == idx.end()) { id = (int)vxyz.size() / 3; idx.emplace(key, id); vxyz.insert(vxyz.end(), p, p + 3); }
            else id = it->second;
            tv[3 * (size_t)t + k] = id;
        }
    pcore::streams::Built b;
    pcore::streams::build_model(tv, vxyz, 0, num_streams, vring, ref_passes, b, chunks);
    using pcore::streams::kSlotPadding;
    using pcore::streams::kStepVertexPass;
    if (b.stris.size() % 64 || b.sverts.size() % 64 || b.sorig.size() != b.stris.size()) return -1;
    std::vector<int> seen(T, 0);
    int next_step = 0, next_pass = 0;
    for (const auto& sd : b.streams) {
        if (sd.x != next_step || sd.y < sd.x || sd.z != next_pass || sd.w < sd.z) return -2;  // descriptors tile the arrays
        next_step = sd.y;
        next_pass = sd.w;
        std::vector<pcore::streams::F4> ring((size_t)vring * 64);
        std::vector<int> ring_pass((size_t)vring * 64, -1000000);
        int P = -1;
        for (int st = sd.x; st < sd.y; st++) {
            const uint32_t* sl = &b.stris[(size_t)st * 64];
            const uint32_t vflag = sl[0] & kStepVertexPass;
            for (int l = 0; l < 64; l++)
                if ((sl[l] & kStepVertexPass) != vflag) return -3;  // one flag per step
            if (vflag) {  // the step consumes the stream's next pass into ring buffer P mod vring
                P++;
                if (sd.z + P >= sd.w) return -4;
                for (int l = 0; l < 64; l++) {
                    ring[(size_t)(P % vring) * 64 + l] = b.sverts[(size_t)(sd.z + P) * 64 + l];
                    ring_pass[(size_t)(P % vring) * 64 + l] = P;
                }
            }
            for (int l = 0; l < 64; l++) {
                const uint32_t s = sl[l];
                if (s & kSlotPadding) continue;
                const uint32_t t = b.sorig[(size_t)st * 64 + l];
                if (t >= (uint32_t)T) return -5;
                seen[t]++;
                for (int k = 0; k < 3; k++) {
                    const int slot = (int)((s >> (9 * k)) & 511u);
                    if (slot >= vring * 64) return -6;
                    if (ring_pass[slot] <= P - ref_passes || ring_pass[slot] > P) return -7;  // the last ref_passes passes
                    const auto& v = ring[slot];
                    if (v.w != 1.0f) return -8;  // a vertex, not padding
                    if (std::memcmp(&v.x, tri_xyz + 9 * (size_t)t + 3 * k, 12) != 0) return -9;  // the exact position
                }
            }
        }
        if (sd.z + P + 1 != sd.w) return -10;  // every pass of the stream is consumed
    }
    if (next_step != (int)(b.stris.size() / 64) || next_pass != (int)(b.sverts.size() / 64)) return -11;
    for (int t = 0; t < T; t++)
        if (seen[t] != 1) return -12;  // every triangle exactly once
    info[0] = b.passes; info[1] = b.steps; info[2] = (long long)vxyz.size() / 3; info[3] = (long long)b.streams.size();
    return 0;
}

// LDS bank conflicts of the fused kernel's triangle stage (its three ds_read_b64 gathers of vertex bounds per step,
// vbd[(slot & 127)], which every step issues for all 64 lanes whatever the pose) under a placement of the ring slots:
// physical lane of (buffer b, lane l) = mode 0: l; 1: l ^ 16 (b odd); 2: l ^ (8 b); 3: (l + 16 b) mod 64; 4: l ^ (16 b).
// ds_read_b64 serves two 32-lane groups; a 8-byte entry at index i sits on bank pair i mod 32, and each extra
// distinct address on a bank pair costs one cycle.  out: [0] extra cycles, [1] group-reads, [2] steps.
extern "C" int stream_bank_sim(const float* tri_xyz, int T, int num_streams, int vring, int ref_passes, int chunks,
                               int mode, long long* out) {
    struct K { uint32_t x, y, z; bool operator==(const K& o) const { return x == o.x && y == o.y && z == o.z; } };
    struct H { size_t operator()(const K& k) const { return (size_t)k.x * 73856093u ^ (size_t)k.y * 19349663u ^ (size_t)k.z * 83492791u; } };
    std::unordered_map<K, int, H> idx;
    std::vector<int> tv(3 * (size_t)T);
    std::vector<float> vxyz;
    for (int t = 0; t < T; t++)
        for (int k = 0; k < 3; k++) {
            const float* p = tri_xyz + 9 * (size_t)t + 3 * k;
            K key;
            std::memcpy(&key.x, p, 4); std::memcpy(&key.y, p + 1, 4); std::memcpy(&key.z, p + 2, 4);
            auto it = idx.find(key);
            int id;
            if (it == idx.end()) { id = (int)vxyz.size() / 3; idx.emplace(key, id); vxyz.insert(vxyz.end(), p, p + 3); }
            else id = it->second;
            tv[3 * (size_t)t + k] = id;
        }
    pcore::streams::Built b;
    pcore::streams::build_model(tv, vxyz, 0, num_streams, vring, ref_passes, b, chunks);
    auto place = [mode](int buf, int l) {
        switch (mode) {
            case 1: return (buf & 1) ? (l ^ 16) : l;
            case 2: return l ^ ((8 * buf) & 63);
            case 3: return (l + 16 * buf) & 63;
            case 4: return l ^ ((16 * buf) & 63);
            default:
                if (mode >= 100) return (l >= 32) ? (l ^ (mode - 100)) : l;  // upper half XOR m (m < 32)
                return l;
        }
    };
    long long extra = 0, reads = 0;
    const long long steps = (long long)b.stris.size() / 64;
    for (long long s = 0; s < steps; s++) {
        for (int k = 0; k < 3; k++)
            for (int g = 0; g < 2; g++) {
                int cnt[32] = {0};
                int seen[32][32];
                for (int l = 0; l < 32; l++) {
                    const uint32_t ct = b.stris[64 * s + 32 * g + l];
                    const int slot = (int)((ct >> (9 * k)) & 511u);
                    const int buf = slot >> 6, ln = slot & 63;
                    const int vi = (buf & 1) * 64 + place(buf, ln);  // vbd entry
                    const int bank = vi & 31;
                    bool dup = false;
                    for (int q = 0; q < cnt[bank]; q++) dup = dup || seen[bank][q] == vi;
                    if (!dup) seen[bank][cnt[bank]++] = vi;
                }
                int mx = 0;
                for (int q = 0; q < 32; q++) mx = cnt[q] > mx ? cnt[q] : mx;
                extra += mx > 0 ? mx - 1 : 0;
                reads++;
            }
    }
    out[0] = extra; out[1] = reads; out[2] = steps;
    return 0;
}

// The builder's steps for one mesh: out_orig[64 * step + slot] = the original triangle index of the slot, or -1 for
// padding (at most max_steps steps); returns the number of steps (tools/step_skip_estimate.py).
extern "C" int stream_steps(const float* tri_xyz, int T, int num_streams, int vring, int ref_passes, int chunks,
                            int32_t* out_orig, int max_steps) {
    struct K { uint32_t x, y, z; bool operator==(const K& o) const { return x == o.x && y == o.y && z == o.z; } };
    struct H { size_t operator()(const K& k) const { return (size_t)k.x * 73856093u ^ (size_t)k.y * 19349663u ^ (size_t)k.z * 83492791u; } };
    std::unordered_map<K, int, H> idx;
    std::vector<int> tv(3 * (size_t)T);
    std::vector<float> vxyz;
    for (int t = 0; t < T; t++)
        for (int k = 0; k < 3; k++) {
            const float* p = tri_xyz + 9 * (size_t)t + 3 * k;
            K key;
            std::memcpy(&key.x, p, 4); std::memcpy(&key.y, p + 1, 4); std::memcpy(&key.z, p + 2, 4);
            auto it = idx.find(key);
            int id;
            if (it == idx.end()) { id = (int)vxyz.size() / 3; idx.emplace(key, id); vxyz.insert(vxyz.end(), p, p + 3); }
            else id = it->second;
            tv[3 * (size_t)t + k] = id;
        }
    pcore::streams::Built b;
    pcore::streams::build_model(tv, vxyz, 0, num_streams, vring, ref_passes, b, chunks);
    const int steps = (int)b.steps;
    for (int s = 0; s < steps && s < max_steps; s++)
        for (int l = 0; l < 64; l++) {
            const uint32_t w = b.stris[(size_t)64 * s + l];
            out_orig[(size_t)64 * s + l] = (w >> 31) ? -1 : (int32_t)b.sorig[(size_t)64 * s + l];
        }
    return steps;
}
