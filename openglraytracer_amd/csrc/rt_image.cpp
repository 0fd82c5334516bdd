// rt_image.cpp — headless image output (the reference displays the texture
// with a full-screen quad instead: draw_screen_vert/frag.glsl, main.cpp:240-260).
#include <algorithm>
#include <cmath>
#include <cstdio>
#include <string>
#include <vector>

#include "rt_internal.h"

using rtamd::set_error;

extern "C" {

// GL_RGBA8 unorm store of a float colour (main.cpp:152-159, :223): NaN -> 0,
// clamp to [0, 1], v * 255 rounded to nearest even — the conversion the
// reference's GL applies (probed: tests/golden/make_rgba8_golden.py); alpha
// stored as written, 0 (:404).
int rt_pack_rgba8(const float *in, size_t n_pixels, uint8_t *out) {
    if ((!in || !out) && n_pixels) {
        set_error("rt_pack_rgba8: null buffer");
        return RT_ERR_INVALID;
    }
    for (size_t i = 0; i < n_pixels * 4; ++i) {
        float v = in[i];
        v = v != v ? 0.0f : std::min(std::max(v, 0.0f), 1.0f);
        out[i] = static_cast<uint8_t>(std::nearbyint(v * 255.0f));  // default rounding: to nearest even
    }
    return RT_OK;
}

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
