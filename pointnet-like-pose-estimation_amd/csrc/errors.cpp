// errors.cpp -- the pn2 C ABI's library state, all of it safe under concurrent host threads
// (the reference's /root/reference/mutilthreading/predict_test.py:44-63 runs four heads from four
// threads on one device):
//   - the error message of the last failure: thread-local;
//   - the kernel-selection tuning (pn2_internal.h PN2_TUNING_KEYS): one atomic word per key
//     process-wide (a launch reads a consistent snapshot of each key, never a torn value), or a
//     thread's own copy between pn2_tuning_local(1) and pn2_tuning_local(0);
//   - the device error slots: each thread's own slot per device (pn2_error_slot_set), or the
//     process-wide default slot, whose reads are serialised by a host mutex.
#include <stdarg.h>
#include <stdio.h>
#include <string.h>

#include <atomic>
#include <mutex>

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

// process-wide keys: relaxed atomics (a key is one independent value; no ordering between keys
// is promised -- change them while no launch depends on two of them changing together)
struct SharedTuning {
#define PN2_TUNING_ATOMIC(name, dflt) std::atomic<int64_t> name{dflt};
    PN2_TUNING_KEYS(PN2_TUNING_ATOMIC)
#undef PN2_TUNING_ATOMIC
};
static SharedTuning g_tuning;
// pn2_tuning_local: this thread's own copy of the keys while depth > 0
static thread_local Tuning t_tuning;
static thread_local int t_depth = 0;

static Tuning shared_snapshot() {
    Tuning t;
#define PN2_TUNING_LOAD(name, dflt) t.name = g_tuning.name.load(std::memory_order_relaxed);
    PN2_TUNING_KEYS(PN2_TUNING_LOAD)
#undef PN2_TUNING_LOAD
    return t;
}

Tuning tuning() { return t_depth > 0 ? t_tuning : shared_snapshot(); }

// ---- device error slots
static thread_local unsigned *t_slots[kMaxDevices] = {};
static std::mutex g_default_read;

static int current_device(int *dev) {
    const hipError_t e = hipGetDevice(dev);
    if (e != hipSuccess) return set_error(PN2_EHIP, "hipGetDevice: %s", hipGetErrorString(e));
    if (*dev < 0 || *dev >= kMaxDevices) return set_error(PN2_EUNSUPPORTED, "device %d >= %d", *dev, kMaxDevices);
    return PN2_OK;
}

// the device a launch on `st` runs on: the stream's own device (a model on cuda:1 may be
// launched while the thread's current device is cuda:0), the current one for the null stream
int stream_device(hipStream_t st) {
    int d = -1;
    if (st) {
        hipDevice_t sd = -1;
        if (hipStreamGetDevice(st, &sd) == hipSuccess) d = (int)sd;
    }
    if (d < 0 && hipGetDevice(&d) != hipSuccess) return -1;
    return d >= 0 && d < kMaxDevices ? d : -1;
}

unsigned *error_word(hipStream_t st) {
    const int d = stream_device(st);
    if (d < 0) return nullptr;
    if (t_slots[d]) return t_slots[d];
    return default_error_slot(d);
}

// take (and with clear, reset) `slot`, stream-ordered on st, then wait for st
static int take(unsigned *slot, int clear, uint32_t *bits, hipStream_t st, bool sync_device) {
    unsigned v = 0;
    hipError_t e = hipSuccess;
    const char *what = "";
    auto run = [&]() -> bool {
        // every stream's work first (pn2_device_errors): kernels still in flight on other
        // streams may raise bits
        if (sync_device && (e = hipDeviceSynchronize()) != hipSuccess) { what = "hipDeviceSynchronize"; return false; }
        if ((e = take_errors(slot, clear, &v, st)) != hipSuccess) { what = "take"; return false; }
        return true;
    };
    bool ok;
    if (is_default_error_slot(slot)) {  // shared with other threads: one reader at a time
        std::lock_guard<std::mutex> g(g_default_read);
        ok = run();
    } else {
        ok = run();
    }
    if (!ok) return set_error(PN2_EHIP, "pn2 device errors (%s): %s", what, hipGetErrorString(e));
    *bits = v;
    return PN2_OK;
}
}  // namespace pn2

extern "C" int pn2_tuning_local(int enter) {
    if (enter) {
        if (pn2::t_depth++ == 0) pn2::t_tuning = pn2::shared_snapshot();
        return PN2_OK;
    }
    PN2_REQUIRE(pn2::t_depth > 0, "pn2_tuning_local: leave without enter");
    --pn2::t_depth;
    return PN2_OK;
}

extern "C" const char *pn2_last_error(void) { return pn2::g_msg; }
extern "C" int pn2_abi_version(void) { return PN2_ABI_VERSION; }

extern "C" int pn2_error_slot_set(uint32_t *slot) {
    int d = 0;
    if (const int rc = pn2::current_device(&d)) return rc;
    pn2::t_slots[d] = slot;
    return PN2_OK;
}

extern "C" int pn2_error_slot_take(int clear, uint32_t *bits, void *stream) {
    PN2_REQUIRE(bits, "pn2_error_slot_take: null pointer");
    unsigned *slot = pn2::error_word(pn2::as_stream(stream));
    if (!slot) return pn2::set_error(PN2_EHIP, "pn2_error_slot_take: no device error slot");
    return pn2::take(slot, clear, bits, pn2::as_stream(stream), false);
}

extern "C" int pn2_device_errors(int clear, uint32_t *bits) {
    PN2_REQUIRE(bits, "pn2_device_errors: null pointer");
    unsigned *slot = pn2::error_word(nullptr);
    if (!slot) return pn2::set_error(PN2_EHIP, "pn2_device_errors: no device error slot");
    return pn2::take(slot, clear, bits, nullptr, true);
}

extern "C" int pn2_tuning_get(const char *key, int64_t *value) {
    PN2_REQUIRE(key && value, "pn2_tuning_get: null pointer");
#define PN2_TUNING_GET(name, dflt)                                                           \
    if (strcmp(key, #name) == 0) {                                                           \
        *value = pn2::t_depth > 0 ? pn2::t_tuning.name                                       \
                                  : pn2::g_tuning.name.load(std::memory_order_relaxed);      \
        return PN2_OK;                                                                       \
    }
    PN2_TUNING_KEYS(PN2_TUNING_GET)
#undef PN2_TUNING_GET
    return pn2::set_error(PN2_EINVAL, "pn2_tuning_get: unknown key '%s'", key);
}

extern "C" int pn2_tuning_set(const char *key, int64_t value) {
    PN2_REQUIRE(key, "pn2_tuning_set: null pointer");
#define PN2_TUNING_SET(name, dflt)                                                           \
    if (strcmp(key, #name) == 0) {                                                           \
        if (pn2::t_depth > 0) pn2::t_tuning.name = value;                                    \
        else pn2::g_tuning.name.store(value, std::memory_order_relaxed);                     \
        return PN2_OK;                                                                       \
    }
    PN2_TUNING_KEYS(PN2_TUNING_SET)
#undef PN2_TUNING_SET
    return pn2::set_error(PN2_EINVAL, "pn2_tuning_set: unknown key '%s'", key);
}

extern "C" int pn2_tuning_default(const char *key, int64_t *value) {
    PN2_REQUIRE(key && value, "pn2_tuning_default: null pointer");
#define PN2_TUNING_DFLT(name, dflt)                \
    if (strcmp(key, #name) == 0) {                 \
        *value = dflt;                             \
        return PN2_OK;                             \
    }
    PN2_TUNING_KEYS(PN2_TUNING_DFLT)
#undef PN2_TUNING_DFLT
    return pn2::set_error(PN2_EINVAL, "pn2_tuning_default: unknown key '%s'", key);
}

extern "C" const char *pn2_tuning_keys(void) {
    static const char keys[] =
#define PN2_TUNING_NAME(name, dflt) #name " "
        PN2_TUNING_KEYS(PN2_TUNING_NAME)
#undef PN2_TUNING_NAME
        ;
    return keys;
}
