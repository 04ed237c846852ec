// errors.cpp -- see errors.h.  Host-only, so the host sources (plan
// building, frame parsing) report errors the same way as the GPU runtime.
#include "errors.h"

#include <cstdarg>
#include <cstdio>

#include "hdfs_crc32c.h"

namespace hdfs_crc {

namespace {
thread_local char g_err[512] = "";
}  // namespace

int fail(int code, const char *fmt, ...) {
    va_list ap;
    va_start(ap, fmt);
    std::vsnprintf(g_err, sizeof g_err, fmt, ap);
    va_end(ap);
    return code;
}

}  // namespace hdfs_crc

extern "C" const char *crc32c_last_error(void) { return hdfs_crc::g_err; }
