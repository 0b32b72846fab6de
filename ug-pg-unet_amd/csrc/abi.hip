// C-ABI plumbing for libugpg.so: version string and thread-local error message.
#include "common.h"

namespace ugpg {
namespace {
thread_local char g_err[512] = "";
}

void set_error(const char* fmt, ...) {
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(g_err, sizeof(g_err), fmt, ap);
    va_end(ap);
}
}  // namespace ugpg

extern "C" const char* ugpg_version(void) { return "ugpg 0.1.0 gfx950"; }

extern "C" const char* ugpg_last_error(void) { return ugpg::g_err; }
