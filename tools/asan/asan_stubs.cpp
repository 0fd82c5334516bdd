// The error channel of the C-ABI (rt_api.cpp) for the host-only sanitizer
// build, which leaves out the device code and its launch API.
#include <string>

#include "../../openglraytracer_amd/csrc/rt_internal.h"

namespace {
thread_local std::string g_error;
}
namespace rtamd {
void set_error(const std::string &msg) { g_error = msg; }
}  // namespace rtamd
extern "C" const char *rt_last_error(void) { return g_error.c_str(); }
extern "C" int rt_pack_rgba8(const float *in, size_t n_pixels, uint8_t *out) {
    for (size_t i = 0; i < n_pixels * 4; ++i) {
        float v = in[i];
        v = v != v ? 0.0f : (v < 0.0f ? 0.0f : (v > 1.0f ? 1.0f : v));
        out[i] = static_cast<uint8_t>(v * 255.0f + 0.5f);
    }
    return 0;
}
