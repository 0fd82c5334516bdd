// Host cost of building a scene (rt_scene_create / rt_scene_update minus the
// upload): make -C openglraytracer_amd/csrc scene-build-time. Prints the
// median build time of the benchmark scenes (masks, BVH, blob) and a hash of
// each blob (builder changes that must not change the scene compare it).
#include <algorithm>
#include <chrono>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <vector>

#include "../../openglraytracer_amd/csrc/rt_internal.h"

namespace rtamd {
int build_scene(const rt_object *objs, int n_objs, const rt_material *mats, int n_mats, const rt_light *lights,
                int n_lights, std::vector<float4> &blob, DeviceScene &ds, bool with_origin_lists);
int build_origin_lists_for(const std::vector<float4> &host, const DeviceScene &ds, std::vector<uint8_t> &olist);
}

int main() {
    rt_material mats[RT_REFERENCE_MATERIALS];
    rt_light lights[RT_REFERENCE_LIGHTS];
    rt_reference_materials(mats);
    rt_reference_lights(lights);
    for (int n : {16, 33, 64, 100, 256}) {
        std::vector<rt_object> objs(n + 1);
        rt_bench_objects(n, 0, objs.data());
        std::vector<double> ms;
        uint64_t hash = 1469598103934665603ull;  // FNV-1a over the blob bytes
        for (int rep = 0; rep < 7; ++rep) {
            std::vector<float4> blob;
            rtamd::DeviceScene ds;
            const auto t0 = std::chrono::steady_clock::now();
            rtamd::build_scene(objs.data(), n + 1, mats, RT_REFERENCE_MATERIALS, lights, RT_REFERENCE_LIGHTS, blob, ds, false);
            ms.push_back(std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count());
            if (rep == 0) {
                const unsigned char *b = reinterpret_cast<const unsigned char *>(blob.data());
                for (size_t i = 0; i < blob.size() * sizeof(float4); ++i) hash = (hash ^ b[i]) * 1099511628211ull;
            }
        }
        std::sort(ms.begin(), ms.end());
        std::vector<float4> blob;
        rtamd::DeviceScene ds;
        rtamd::build_scene(objs.data(), n + 1, mats, RT_REFERENCE_MATERIALS, lights, RT_REFERENCE_LIGHTS, blob, ds, false);
        if (ds.off_glist >= 0) {  // candidate-list lengths of the wide masks (rt_internal.h kGListMax)
            const unsigned char *g = reinterpret_cast<const unsigned char *>(blob.data()) + 16L * ds.off_glist;
            const long texels = (static_cast<long>(blob.size()) - ds.off_glist);
            long over = 0, hist[4] = {0, 0, 0, 0};
            double sum = 0;
            for (long t = 0; t < texels; ++t) {
                const int c = g[16 * t];
                if (c == 255) { ++over; continue; }
                sum += c;
                ++hist[c == 0 ? 0 : (c <= 2 ? 1 : (c <= 7 ? 2 : 3))];
            }
            std::printf("room + %3d spheres: %ld texel lists, mean length %.2f, 0: %ld, 1-2: %ld, 3-7: %ld, 8-15: %ld, "
                        "overflow (> 15): %ld\n", n, texels, sum / (texels - over), hist[0], hist[1], hist[2], hist[3], over);
        }
        // LDS per work-group: the staged blob + per-sphere camera terms and footprints + per-box camera terms
        const long lds = 16L * (ds.blob_units + 2L * n + 1);
        std::printf("room + %3d spheres: scene build %.3f ms (median of 7), blob %016llx, LDS %ld B (masks %d B)\n", n,
                    ms[3], static_cast<unsigned long long>(hash), lds,
                    ds.off_dmask >= 0 ? 16 * (ds.blob_units - ds.off_dmask) : 0);
        if (ds.olist_eligible) {  // the origin-sphere lists, built on a scene's first deep render
            std::vector<double> ol;
            std::vector<uint8_t> olist;
            for (int rep = 0; rep < 3; ++rep) {
                const auto t0 = std::chrono::steady_clock::now();
                rtamd::build_origin_lists_for(blob, ds, olist);
                ol.push_back(std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count());
            }
            std::sort(ol.begin(), ol.end());
            std::printf("room + %3d spheres: origin lists %.3f ms (median of 3), %zu B\n", n, ol[1], olist.size());
        }
    }
    return 0;
}
