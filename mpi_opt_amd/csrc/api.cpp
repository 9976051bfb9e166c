// api.cpp -- error plumbing and version of the libmpo.so C ABI.
#include "mpo_internal.h"

namespace mpo {

static thread_local std::string g_last_error;

void set_error(const char* fmt, ...) {
    char buf[1024];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof(buf), fmt, ap);
    va_end(ap);
    g_last_error = buf;
}

void clear_error() { g_last_error.clear(); }

}  // namespace mpo

extern "C" {

const char* mpo_last_error(void) { return mpo::g_last_error.c_str(); }

const char* mpo_version(void) { return "mpo 0.1 gfx950"; }

}
