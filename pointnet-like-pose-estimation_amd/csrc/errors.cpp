// errors.cpp -- thread-local error reporting of the pn2 C ABI (the library's only state).
#include <stdarg.h>
#include <stdio.h>

#include "pn2.h"

namespace pn2 {
static thread_local char g_msg[512] = "";

int set_error(int code, const char *fmt, ...) {
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(g_msg, sizeof(g_msg), fmt, ap);
    va_end(ap);
    return code;
}
}  // namespace pn2

extern "C" const char *pn2_last_error(void) { return pn2::g_msg; }
extern "C" int pn2_abi_version(void) { return PN2_ABI_VERSION; }
