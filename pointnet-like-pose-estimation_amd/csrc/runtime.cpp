// runtime.cpp -- host-side runtime helpers of libpn2: CU-partitioned HIP streams.
//
// The pipelined forward (pn2/pipeline.py) runs the latency-bound FPS chain of the next batch on
// a few dedicated CUs while the current batch's MLPs run on the rest; MI355X queues accept a CU
// mask (hipExtStreamCreateWithCUMask), so the two streams partition the chip instead of
// time-sharing CUs (an FPS workgroup sharing a CU with MFMA work runs its serial loop ~2.7x
// slower, measured).
#include "pn2_internal.h"

#include <vector>

extern "C" int pn2_device_cu_count(int device, int *count) {
    PN2_REQUIRE(count, "pn2_device_cu_count: null pointer");
    int n = 0;
    hipError_t e = hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, device);
    if (e != hipSuccess) return pn2::set_error(PN2_EHIP, "pn2_device_cu_count: %s", hipGetErrorString(e));
    *count = n;
    return PN2_OK;
}

extern "C" int pn2_stream_create_cu_masked(int device, const uint32_t *mask, int mask_words,
                                           void **stream) {
    PN2_REQUIRE(mask && stream && mask_words > 0, "pn2_stream_create_cu_masked: bad arguments");
    int any = 0;
    for (int i = 0; i < mask_words; ++i) any |= mask[i] != 0;
    PN2_REQUIRE(any, "pn2_stream_create_cu_masked: empty CU mask");
    int prev = 0;
    hipError_t e = hipGetDevice(&prev);
    if (e == hipSuccess && prev != device) e = hipSetDevice(device);
    hipStream_t s = nullptr;
    if (e == hipSuccess) e = hipExtStreamCreateWithCUMask(&s, (uint32_t)mask_words, mask);
    if (prev != device) (void)hipSetDevice(prev);
    if (e != hipSuccess)
        return pn2::set_error(PN2_EHIP, "pn2_stream_create_cu_masked: %s", hipGetErrorString(e));
    *stream = s;
    return PN2_OK;
}

extern "C" int pn2_stream_destroy(void *stream) {
    if (!stream) return PN2_OK;
    hipError_t e = hipStreamDestroy(reinterpret_cast<hipStream_t>(stream));
    if (e != hipSuccess) return pn2::set_error(PN2_EHIP, "pn2_stream_destroy: %s", hipGetErrorString(e));
    return PN2_OK;
}
