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
