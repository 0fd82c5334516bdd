// Host-only sanitizer driver (make -C openglraytracer_amd/csrc asan): runs
// the host C++ of the product — scene description parser, scene builder
// (masks, BVH, blob layout), per-frame constants, reference scene / camera,
// image dump — under AddressSanitizer + UndefinedBehaviorSanitizer, on the
// shipped scene descriptions, the benchmark scenes and a malformed-JSON
// corpus (every truncation of every scene file, seeded byte mutations, and
// hand-written edge cases). No GPU: nothing here launches a kernel.
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <sstream>
#include <string>
#include <vector>

#include "../../openglraytracer_amd/csrc/rt_internal.h"

namespace rtamd {
int build_scene(const rt_object *objs, int n_objs, const rt_material *mats, int n_mats, const rt_light *lights,
                int n_lights, std::vector<float4> &blob, DeviceScene &ds, bool with_origin_lists);
int build_origin_lists_for(const std::vector<float4> &host, const DeviceScene &ds, std::vector<uint8_t> &olist);
}  // namespace rtamd

namespace {

int g_parsed = 0, g_rejected = 0, g_built = 0;

void parse_and_build(const std::string &text, float t) {
    std::vector<rt_object> objs(RT_MAX_OBJECTS);
    std::vector<rt_material> mats(RT_MAX_MATERIALS);
    std::vector<rt_light> lights(RT_MAX_LIGHTS);
    rt_camera cam;
    int no = 0, nm = 0, nl = 0, hc = 0;
    if (rt_scene_desc_parse(text.c_str(), t, objs.data(), RT_MAX_OBJECTS, &no, mats.data(), RT_MAX_MATERIALS, &nm,
                            lights.data(), RT_MAX_LIGHTS, &nl, &cam, &hc) != RT_OK) {
        ++g_rejected;
        (void)rt_last_error();
        return;
    }
    ++g_parsed;
    std::vector<float4> blob;
    rtamd::DeviceScene ds;
    if (rtamd::build_scene(objs.data(), no, mats.data(), nm, lights.data(), nl, blob, ds, true) == RT_OK) {
        ++g_built;
        rt_view view;
        rt_make_view(hc ? &cam : nullptr, t, &view);
        rtamd::LaunchParams p{};
        p.n_views = 1;
        std::memcpy(p.view[0].unproj, view.unprojection, sizeof view.unprojection);
        std::memcpy(p.view[0].origin, view.origin, sizeof view.origin);
        p.view[0].cull = 1;
        p.width = 320;
        p.height = 180;
        p.n_spheres = ds.n_spheres;
        p.n_boxes = ds.n_boxes;
        p.off_spheres = ds.off_spheres;
        p.off_smeta = ds.off_smeta;
        p.off_boxes = ds.off_boxes;
        const float4 *blobs[1] = {blob.data()};
        rtamd::host_frame_setup(p, blobs);
    }
}

std::string slurp(const char *path) {
    std::ifstream f(path);
    std::stringstream ss;
    ss << f.rdbuf();
    return ss.str();
}

}  // namespace

int main(int argc, char **argv) {
    // reference tables, benchmark scenes up to the object limit, cameras
    rt_material mats[RT_REFERENCE_MATERIALS];
    rt_light lights[RT_REFERENCE_LIGHTS];
    rt_reference_materials(mats);
    rt_reference_lights(lights);
    for (float t : {0.0f, 3.7f, -100.0f, 1e4f}) {
        rt_object ref[RT_REFERENCE_OBJECTS];
        rt_reference_objects(t, ref);
        std::vector<float4> blob;
        rtamd::DeviceScene ds;
        if (rtamd::build_scene(ref, RT_REFERENCE_OBJECTS, mats, RT_REFERENCE_MATERIALS, lights, RT_REFERENCE_LIGHTS,
                               blob, ds, true) != RT_OK)
            return 1;
        rt_view v;
        rt_make_view(nullptr, t, &v);
    }
    for (int n : {0, 1, 16, 17, 33, 64, 65, 256, 257, RT_MAX_OBJECTS - 1}) {
        std::vector<rt_object> objs(n + 1);
        if (rt_bench_objects(n, 7, objs.data()) != RT_OK) return 1;
        std::vector<float4> blob;
        rtamd::DeviceScene ds;
        if (rtamd::build_scene(objs.data(), n + 1, mats, RT_REFERENCE_MATERIALS, lights, RT_REFERENCE_LIGHTS, blob,
                               ds, true) != RT_OK)
            return 1;
        ++g_built;
    }
    // image dump and RGBA8 packing (NaN / inf / negative values)
    std::vector<float> img(37 * 11 * 4);
    for (size_t i = 0; i < img.size(); ++i) img[i] = (i % 7 == 0) ? NAN : (i % 5 == 0 ? INFINITY : -0.5f + i * 0.01f);
    std::vector<uint8_t> rgba8(img.size());
    rt_pack_rgba8(img.data(), 37 * 11, rgba8.data());
    rt_write_ppm("/tmp/rt_asan.ppm", img.data(), 37, 11);
    rt_write_pfm("/tmp/rt_asan.pfm", img.data(), 37, 11);
    // scene descriptions: as shipped, every truncation, seeded mutations
    std::vector<std::string> files;
    for (int i = 1; i < argc; ++i) files.push_back(slurp(argv[i]));
    uint64_t st = 0x1234567;
    for (const std::string &text : files) {
        parse_and_build(text, 0.0f);
        parse_and_build(text, 2.5f);
        for (size_t cut = 0; cut < text.size(); ++cut) parse_and_build(text.substr(0, cut), 0.0f);
        for (int k = 0; k < 3000; ++k) {
            std::string m = text;
            for (int j = 0; j < 1 + k % 4; ++j) {
                st = st * 6364136223846793005ULL + 1442695040888963407ULL;
                const size_t at = (st >> 33) % (m.size() ? m.size() : 1);
                const char pool[] = "{}[]\":,-+.eE0123456789 \\nutlfa\x01\xff";
                const char c = pool[(st >> 20) % (sizeof pool - 1)];
                switch ((st >> 50) % 3) {
                    case 0: if (!m.empty()) m[at] = c; break;
                    case 1: m.insert(m.begin() + static_cast<long>(at), c); break;
                    default: if (!m.empty()) m.erase(at, 1 + (st >> 40) % 8); break;
                }
            }
            parse_and_build(m, 0.0f);
        }
    }
    const char *edge[] = {
        "", "{", "}", "[]", "null", "{\"objects\": [", "{\"objects\": [{}]}",
        "{\"objects\": [{\"sphere\": {\"position\": [1e400, 0, 0], \"radius\": 1, \"material\": 0}}]}",
        "{\"objects\": [{\"sphere\": {\"position\": [0, 0], \"radius\": 1}}]}",
        "{\"materials\": [], \"objects\": []}", "{\"lights\": [{\"position\": \"x\"}]}",
        "{\"camera\": {\"position\": [0,0,0], \"angles\": [0,0,0], \"v_fov\": -1e38}}",
        "{\"objects\": {\"bench\": {\"spheres\": 2147483647}}}", "{\"objects\": {\"bench\": {\"spheres\": -5}}}",
        "\"\\u12", "{\"a\": \"\\ud800\"}", "{\"objects\": [1, 2, 3]}",
    };
    for (const char *e : edge) parse_and_build(e, 0.0f);
    std::string deep(100000, '[');
    parse_and_build(deep, 0.0f);
    std::printf("asan driver: %d parsed, %d rejected, %d scenes built — clean\n", g_parsed, g_rejected, g_built);
    return 0;
}
