// rt_cli — headless frame driver: the counterpart of the reference's
// main()/draw() loop (OpenGLRaytracer/main.cpp:47-93, :210-261) without a
// window. Renders the shipped scene (or a benchmark scene) at `time`, K frames
// apart by `dt` (the orbiting camera and animated boxes, :334-364, :261-321),
// and writes each frame as PPM (what the RGBA8 surface shows) and/or PFM.
//
//   rt_cli [--width 1280] [--height 720] [--depth 0] [--time 0] [--frames 1]
//          [--dt 0.016] [--scene shipped|spheres:N[:seed]|FILE.json] [--ppm out_%04d.ppm]
//          [--pfm out_%04d.pfm] [--device 0] [--gpus N [--transport rccl|copy] [--block-rows 8]]
//
// --gpus N renders every frame on devices device..device+N-1 with
// rt_render_multi (row blocks per GPU, RCCL gather to the first GPU).
#include <chrono>
#include <fstream>
#include <sstream>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "../../include/rt.h"

namespace {

int fail(const char *what) {
    std::fprintf(stderr, "rt_cli: %s: %s\n", what, rt_last_error());
    return 1;
}

std::string frame_name(const std::string &pattern, int k) {
    if (pattern.find('%') == std::string::npos) return pattern;
    char buf[4096];
    std::snprintf(buf, sizeof buf, pattern.c_str(), k);
    return buf;
}

}  // namespace

int main(int argc, char **argv) {
    int width = 1280, height = 720, depth = 0, frames = 1, device = 0;  // main.cpp:17-19
    int gpus = 1, block_rows = 8, transport = RT_MULTI_RCCL;
    float time0 = 0.0f, dt = 1.0f / 60.0f;
    std::string scene = "shipped", ppm, pfm;
    for (int i = 1; i < argc; ++i) {
        std::string a = argv[i];
        auto next = [&]() -> const char * {
            if (i + 1 >= argc) { std::fprintf(stderr, "rt_cli: %s needs a value\n", a.c_str()); std::exit(2); }
            return argv[++i];
        };
        if (a == "--width") width = std::atoi(next());
        else if (a == "--height") height = std::atoi(next());
        else if (a == "--depth") depth = std::atoi(next());
        else if (a == "--time") time0 = std::strtof(next(), nullptr);
        else if (a == "--frames") frames = std::atoi(next());
        else if (a == "--dt") dt = std::strtof(next(), nullptr);
        else if (a == "--scene") scene = next();
        else if (a == "--ppm") ppm = next();
        else if (a == "--pfm") pfm = next();
        else if (a == "--device") device = std::atoi(next());
        else if (a == "--gpus") gpus = std::atoi(next());
        else if (a == "--block-rows") block_rows = std::atoi(next());
        else if (a == "--transport") transport = std::strcmp(next(), "copy") == 0 ? RT_MULTI_COPY : RT_MULTI_RCCL;
        else {
            std::fprintf(stderr, "usage: rt_cli [--width W] [--height H] [--depth D] [--time T] [--frames K] "
                                 "[--dt S] [--scene shipped|spheres:N[:seed]|FILE.json] [--ppm PAT] [--pfm PAT] "
                                 "[--device I] [--gpus N] [--transport rccl|copy] [--block-rows B]\n");
            return 2;
        }
    }
    if (gpus < 1) { std::fprintf(stderr, "rt_cli: --gpus must be >= 1\n"); return 2; }
    std::vector<rt_context *> ctxs(gpus, nullptr);
    for (int g = 0; g < gpus; ++g)
        if (rt_create(device + g, &ctxs[g]) != RT_OK) return fail("rt_create");
    rt_context *ctx = ctxs[0];
    rt_multi *group = nullptr;
    if (gpus > 1 && rt_multi_create(gpus, ctxs.data(), transport, &group) != RT_OK) return fail("rt_multi_create");
    std::vector<rt_scene *> scs(gpus, nullptr);
    std::vector<rt_material> mats(RT_REFERENCE_MATERIALS);
    std::vector<rt_light> lights(RT_REFERENCE_LIGHTS);
    rt_reference_materials(mats.data());
    rt_reference_lights(lights.data());
    std::string json;  // a scene description file (rt_scene_desc_parse), re-read at every frame's time
    if (scene.size() > 5 && scene.compare(scene.size() - 5, 5, ".json") == 0) {
        std::ifstream f(scene);
        if (!f) { std::fprintf(stderr, "rt_cli: cannot read %s\n", scene.c_str()); return 2; }
        std::stringstream ss;
        ss << f.rdbuf();
        json = ss.str();
    }
    std::vector<float> frame(static_cast<size_t>(width) * height * 4);
    for (int k = 0; k < frames; ++k) {
        const float t = time0 + k * dt;
        std::vector<rt_object> objs;
        rt_camera cam;
        int has_cam = 0;
        if (!json.empty()) {
            int no = 0, nm = 0, nl = 0;
            objs.resize(RT_MAX_OBJECTS);
            mats.resize(RT_MAX_MATERIALS);
            lights.resize(RT_MAX_LIGHTS);
            if (rt_scene_desc_parse(json.c_str(), t, objs.data(), RT_MAX_OBJECTS, &no, mats.data(), RT_MAX_MATERIALS,
                                    &nm, lights.data(), RT_MAX_LIGHTS, &nl, &cam, &has_cam) != RT_OK)
                return fail("rt_scene_desc_parse");
            objs.resize(no);
            mats.resize(nm);
            lights.resize(nl);
        } else if (scene == "shipped") {
            objs.resize(RT_REFERENCE_OBJECTS);
            rt_reference_objects(t, objs.data());
        } else if (scene.rfind("spheres:", 0) == 0) {
            int n = 0;
            unsigned long long seed = 0;
            std::sscanf(scene.c_str() + 8, "%d:%llu", &n, &seed);
            objs.resize(static_cast<size_t>(n) + 1);
            if (rt_bench_objects(n, seed, objs.data()) != RT_OK) return fail("rt_bench_objects");
        } else {
            std::fprintf(stderr, "rt_cli: unknown scene %s\n", scene.c_str());
            return 2;
        }
        for (int g = 0; g < gpus; ++g) {  // the frame's scene on every GPU
            if (!scs[g]) {
                if (rt_scene_create(ctxs[g], objs.data(), static_cast<int>(objs.size()), mats.data(),
                                    static_cast<int>(mats.size()), lights.data(), static_cast<int>(lights.size()),
                                    &scs[g]) != RT_OK)
                    return fail("rt_scene_create");
            } else if (rt_scene_update(ctxs[g], scs[g], objs.data(), static_cast<int>(objs.size()), mats.data(),
                                       static_cast<int>(mats.size()), lights.data(),
                                       static_cast<int>(lights.size())) != RT_OK) {
                return fail("rt_scene_update");
            }
        }
        const auto t0 = std::chrono::steady_clock::now();
        if (group) {
            if (rt_render_multi(group, scs.data(), has_cam ? &cam : nullptr, t, width, height, depth, block_rows,
                                frame.data(), 0) != RT_OK)
                return fail("rt_render_multi");
        } else if (rt_render(ctx, scs[0], has_cam ? &cam : nullptr, t, width, height, depth, 0, height, frame.data(),
                             0, nullptr) != RT_OK) {
            return fail("rt_render");
        }
        const double wall = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
        if (group) {
            std::vector<float> kms(gpus, 0.0f);
            float gms = 0.0f, ams = 0.0f;
            rt_multi_last_ms(group, kms.data(), &gms, &ams);
            std::printf("frame %d t=%.4f  kernels", k, t);
            for (float v : kms) std::printf(" %.3f", v);
            std::printf(" ms  gather %.3f ms  assembly %.3f ms  call %.3f ms (incl. device->host copy)\n", gms, ams,
                        wall * 1e3);
        } else {
            float kms = 0.0f;
            rt_last_kernel_ms(ctx, &kms);
            std::printf("frame %d t=%.4f  kernel %.3f ms  call %.3f ms (incl. device->host copy)\n", k, t, kms,
                        wall * 1e3);
        }
        if (!ppm.empty() && rt_write_ppm(frame_name(ppm, k).c_str(), frame.data(), width, height) != RT_OK)
            return fail("rt_write_ppm");
        if (!pfm.empty() && rt_write_pfm(frame_name(pfm, k).c_str(), frame.data(), width, height) != RT_OK)
            return fail("rt_write_pfm");
    }
    rt_multi_destroy(group);
    for (int g = 0; g < gpus; ++g) {
        rt_scene_destroy(scs[g]);
        rt_destroy(ctxs[g]);
    }
    return 0;
}
