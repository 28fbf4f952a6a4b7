// errors.cpp -- the pn2 C ABI's library state: the thread-local error message and the
// kernel-selection tuning (pn2_internal.h PN2_TUNING_KEYS): process-wide, or a thread's own
// copy between pn2_tuning_local(1) and pn2_tuning_local(0).
#include <stdarg.h>
#include <stdio.h>
#include <string.h>

#include "pn2_internal.h"

namespace pn2 {
static thread_local char g_msg[512] = "";

int set_error(int code, const char *fmt, ...) {
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(g_msg, sizeof(g_msg), fmt, ap);
    va_end(ap);
    return code;
}

static Tuning g_tuning;
// pn2_tuning_local: this thread's own copy of the keys while depth > 0
static thread_local Tuning t_tuning;
static thread_local int t_depth = 0;
static Tuning &active() { return t_depth > 0 ? t_tuning : g_tuning; }
const Tuning &tuning() { return t_depth > 0 ? t_tuning : g_tuning; }
}  // namespace pn2

extern "C" int pn2_tuning_local(int enter) {
    if (enter) {
        if (pn2::t_depth++ == 0) pn2::t_tuning = pn2::g_tuning;
        return PN2_OK;
    }
    PN2_REQUIRE(pn2::t_depth > 0, "pn2_tuning_local: leave without enter");
    --pn2::t_depth;
    return PN2_OK;
}

extern "C" const char *pn2_last_error(void) { return pn2::g_msg; }
extern "C" int pn2_abi_version(void) { return PN2_ABI_VERSION; }

extern "C" int pn2_device_errors(int clear, uint32_t *bits) {
    PN2_REQUIRE(bits, "pn2_device_errors: null pointer");
    unsigned a = 0, b = 0;
    if (pn2::read_bq_errors(&a, clear) != 0 || pn2::read_group_errors(&b, clear) != 0)
        return pn2::set_error(PN2_EHIP, "pn2_device_errors: %s", hipGetErrorString(hipGetLastError()));
    *bits = a | b;
    return PN2_OK;
}

extern "C" int pn2_tuning_get(const char *key, int64_t *value) {
    PN2_REQUIRE(key && value, "pn2_tuning_get: null pointer");
#define PN2_TUNING_GET(name, dflt)                 \
    if (strcmp(key, #name) == 0) {                 \
        *value = pn2::active().name;               \
        return PN2_OK;                             \
    }
    PN2_TUNING_KEYS(PN2_TUNING_GET)
#undef PN2_TUNING_GET
    return pn2::set_error(PN2_EINVAL, "pn2_tuning_get: unknown key '%s'", key);
}

extern "C" int pn2_tuning_set(const char *key, int64_t value) {
    PN2_REQUIRE(key, "pn2_tuning_set: null pointer");
#define PN2_TUNING_SET(name, dflt)                 \
    if (strcmp(key, #name) == 0) {                 \
        pn2::active().name = value;                \
        return PN2_OK;                             \
    }
    PN2_TUNING_KEYS(PN2_TUNING_SET)
#undef PN2_TUNING_SET
    return pn2::set_error(PN2_EINVAL, "pn2_tuning_set: unknown key '%s'", key);
}

extern "C" const char *pn2_tuning_keys(void) {
    static const char keys[] =
#define PN2_TUNING_NAME(name, dflt) #name " "
        PN2_TUNING_KEYS(PN2_TUNING_NAME)
#undef PN2_TUNING_NAME
        ;
    return keys;
}
