// Error reporting shared by every entry point of liblincheck.
#include <cstdarg>

#include "common.hpp"

namespace lc {

static thread_local std::string g_last_error;

void set_error(const std::string &msg) { g_last_error = msg; }

int fail(int code, const char *fmt, ...) {
    char buf[1024];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof buf, fmt, ap);
    va_end(ap);
    g_last_error = buf;
    return code;
}

}  // namespace lc

extern "C" const char *lc_last_error(void) { return lc::g_last_error.c_str(); }
extern "C" int lc_abi_version(void) { return LC_ABI_VERSION; }
