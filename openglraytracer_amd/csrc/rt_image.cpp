// rt_image.cpp — headless image output (the reference displays the texture
// with a full-screen quad instead: draw_screen_vert/frag.glsl, main.cpp:240-260).
#include <cstdio>
#include <string>
#include <vector>

#include "rt_internal.h"

using rtamd::set_error;

extern "C" {

int rt_write_ppm(const char *path, const float *rgba, int width, int height) {
    if (!path || !rgba || width <= 0 || height <= 0) {
        set_error("rt_write_ppm: bad arguments");
        return RT_ERR_INVALID;
    }
    const size_t n = static_cast<size_t>(width) * height;
    std::vector<uint8_t> px(n * 4);
    rt_pack_rgba8(rgba, n, px.data());
    FILE *f = std::fopen(path, "wb");
    if (!f) {
        set_error(std::string("rt_write_ppm: cannot open ") + path);
        return RT_ERR_INVALID;
    }
    std::fprintf(f, "P6\n%d %d\n255\n", width, height);
    std::vector<uint8_t> row(static_cast<size_t>(width) * 3);
    bool ok = true;
    for (int y = height - 1; y >= 0 && ok; --y) {  // GL row 0 is the bottom row
        const uint8_t *src = px.data() + static_cast<size_t>(y) * width * 4;
        for (int x = 0; x < width; ++x)
            for (int c = 0; c < 3; ++c) row[x * 3 + c] = src[x * 4 + c];
        ok = std::fwrite(row.data(), 1, row.size(), f) == row.size();
    }
    ok = (std::fclose(f) == 0) && ok;
    if (!ok) {
        set_error(std::string("rt_write_ppm: write failed: ") + path);
        return RT_ERR_INVALID;
    }
    return RT_OK;
}

int rt_write_pfm(const char *path, const float *rgba, int width, int height) {
    if (!path || !rgba || width <= 0 || height <= 0) {
        set_error("rt_write_pfm: bad arguments");
        return RT_ERR_INVALID;
    }
    FILE *f = std::fopen(path, "wb");
    if (!f) {
        set_error(std::string("rt_write_pfm: cannot open ") + path);
        return RT_ERR_INVALID;
    }
    std::fprintf(f, "PF\n%d %d\n-1.0\n", width, height);  // negative scale: little-endian
    std::vector<float> row(static_cast<size_t>(width) * 3);
    bool ok = true;
    for (int y = 0; y < height && ok; ++y) {  // PFM stores rows bottom-up, as GL does
        const float *src = rgba + static_cast<size_t>(y) * width * 4;
        for (int x = 0; x < width; ++x)
            for (int c = 0; c < 3; ++c) row[x * 3 + c] = src[x * 4 + c];
        ok = std::fwrite(row.data(), sizeof(float), row.size(), f) == row.size();
    }
    ok = (std::fclose(f) == 0) && ok;
    if (!ok) {
        set_error(std::string("rt_write_pfm: write failed: ") + path);
        return RT_ERR_INVALID;
    }
    return RT_OK;
}

}  // extern "C"
