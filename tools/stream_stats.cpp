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
