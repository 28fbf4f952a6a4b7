// group.hip -- index_points and the neighbourhood grouping, for the public op API.
//
// index_points:        /root/reference/model/pointnet2_utils.py:28-45
// sample_and_group:    pointnet2_utils.py:107-116  ([xyz - centroid, feature], xyz first)
// SA-MSG grouping:     pointnet2_utils.py:204-209  ([feature, xyz - centroid], feature first)
// The fused SA path (sa_mlp.hip) gathers straight into LDS and never materialises these
// tensors; these kernels serve the standalone functions of the drop-in module.
// One thread per output element (contiguous output => coalesced stores); the subtraction is a
// single correctly rounded float32 op, bit-identical to the reference.
//
// Indices follow torch's advanced indexing: -N <= n < 0 counts from the end.  Outside [-N, N)
// the reference raises IndexError; a kernel cannot, so the element is NaN (never an
// out-of-bounds read) and PN2_DEVERR_INDEX is raised in the launching thread's device error slot
// (pn2_error_slot_set / pn2_device_errors; pn2.check_device_errors() raises IndexError).
#include <atomic>

#include "pn2_internal.h"

namespace pn2 {

// the process-wide default error slot (pn2_internal.h): [0] bits, [1] the take's snapshot
__device__ unsigned g_default_errors[2];

static std::atomic<unsigned *> g_default_cache[kMaxDevices];

// device d's copy of g_default_errors (the symbol's address is per device: resolved with d
// current, once)
unsigned *default_error_slot(int d) {
    if (d < 0 || d >= kMaxDevices) return nullptr;
    unsigned *p = g_default_cache[d].load(std::memory_order_acquire);
    if (!p) {
        int cur = -1;
        if (hipGetDevice(&cur) != hipSuccess) return nullptr;
        if (cur != d && hipSetDevice(d) != hipSuccess) return nullptr;
        void *a = nullptr;
        const hipError_t e = hipGetSymbolAddress(&a, HIP_SYMBOL(g_default_errors));
        if (cur != d) (void)hipSetDevice(cur);
        if (e != hipSuccess) return nullptr;
        p = static_cast<unsigned *>(a);
        g_default_cache[d].store(p, std::memory_order_release);
    }
    return p;
}

bool is_default_error_slot(const unsigned *slot) {
    for (int d = 0; d < kMaxDevices; ++d)
        if (slot && g_default_cache[d].load(std::memory_order_acquire) == slot) return true;
    return false;
}

// the slot's value (and, with clear, its reset) in ONE device atomic: a bit that a kernel ORs in
// between cannot be lost (a read followed by a separate clear could drop it)
__global__ void errors_take_kernel(unsigned *slot, int clear) {
    slot[1] = clear ? atomicExch(&slot[0], 0u) : atomicOr(&slot[0], 0u);
}

hipError_t take_errors(unsigned *slot, int clear, unsigned *bits, hipStream_t st) {
    hipLaunchKernelGGL(errors_take_kernel, dim3(1), dim3(1), 0, st, slot, clear);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
    unsigned v = 0;
    if ((e = hipMemcpyAsync(&v, slot + 1, sizeof(v), hipMemcpyDeviceToHost, st)) != hipSuccess) return e;
    if ((e = hipStreamSynchronize(st)) != hipSuccess) return e;
    *bits = v;
    return hipSuccess;
}

// torch's index rule; -1 when out of range (and the error bit raised in the launch's slot)
__device__ __forceinline__ int64_t torch_index(int64_t n, int64_t N, unsigned *err) {
    if (n < 0) n += N;
    if (n < 0 || n >= N) {
        atomicOr(err, (unsigned)PN2_DEVERR_INDEX);
        return -1;
    }
    return n;
}

__global__ __launch_bounds__(256) void index_points_kernel(const float *__restrict__ pts,
                                                           int64_t B, int64_t N, int64_t C,
                                                           int64_t sb, int64_t sn, int64_t sc,
                                                           const int64_t *__restrict__ idx,
                                                           int64_t M, float *__restrict__ out,
                                                           unsigned *err) {
    const int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (e >= B * M * C) return;
    const int64_t c = e % C;
    const int64_t bm = e / C;
    const int64_t b = bm / M;
    const int64_t n = torch_index(idx[bm], N, err);
    out[e] = n < 0 ? __builtin_nanf("") : pts[b * sb + n * sn + c * sc];
}

__global__ __launch_bounds__(256) void group_kernel(const float *__restrict__ pts, int64_t N,
                                                    int64_t C, int64_t sb, int64_t sn, int64_t sc,
                                                    const float *__restrict__ feat, int64_t D,
                                                    int64_t fb, int64_t fn, int64_t fd,
                                                    const float *__restrict__ ctr, int64_t S,
                                                    const int64_t *__restrict__ idx, int64_t K,
                                                    int feature_first, int64_t total,
                                                    float *__restrict__ out, unsigned *err) {
    const int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (e >= total) return;
    const int64_t W = C + D;
    const int64_t ch = e % W;
    const int64_t row = e / W;  // (b*S + s)*K + k
    const int64_t g = row / K;
    const int64_t b = g / S;
    const int64_t n = torch_index(idx[row], N, err);
    const int64_t xc = feature_first ? ch - D : ch;  // xyz channel, if any
    float v;
    if (n < 0)
        v = __builtin_nanf("");
    else if (xc >= 0 && xc < C)
        v = __fsub_rn(pts[b * sb + n * sn + xc * sc], ctr[g * C + xc]);
    else {
        const int64_t d = feature_first ? ch : ch - C;
        v = feat[b * fb + n * fn + d * fd];
    }
    out[e] = v;
}

}  // namespace pn2

using namespace pn2;

extern "C" int pn2_index_points_f32(const float *pts, int64_t B, int64_t N, int64_t C,
                                    int64_t sb, int64_t sn, int64_t sc, const int64_t *idx,
                                    int64_t M, float *out, void *stream) {
    PN2_REQUIRE(pts && idx && out, "pn2_index_points_f32: null pointer");
    PN2_REQUIRE(B >= 0 && N >= 1 && C >= 1 && M >= 0, "pn2_index_points_f32: bad shape");
    const int64_t tot = B * M * C;
    if (tot == 0) return PN2_OK;
    unsigned *err = error_word(as_stream(stream));
    PN2_REQUIRE(err, "pn2_index_points_f32: no device error slot");
    hipLaunchKernelGGL(index_points_kernel, dim3((unsigned)((tot + 255) / 256)), dim3(256), 0,
                       as_stream(stream), pts, B, N, C, sb, sn, sc, idx, M, out, err);
    PN2_LAUNCH_CHECK("index_points_kernel");
    return PN2_OK;
}

extern "C" int pn2_group_f32(const float *pts, int64_t B, int64_t N, int64_t C, int64_t sb,
                             int64_t sn, int64_t sc, const float *feat, int64_t D, int64_t fb,
                             int64_t fn, int64_t fd, const float *ctr, int64_t S,
                             const int64_t *idx, int64_t K, int feature_first, float *out,
                             void *stream) {
    PN2_REQUIRE(pts && ctr && idx && out, "pn2_group_f32: null pointer");
    PN2_REQUIRE(D == 0 || feat, "pn2_group_f32: D > 0 but feat is null");
    PN2_REQUIRE(B >= 0 && N >= 1 && C >= 1 && D >= 0 && S >= 0 && K >= 1,
                "pn2_group_f32: bad shape");
    const int64_t tot = B * S * K * (C + D);
    if (tot == 0) return PN2_OK;
    unsigned *err = error_word(as_stream(stream));
    PN2_REQUIRE(err, "pn2_group_f32: no device error slot");
    hipLaunchKernelGGL(group_kernel, dim3((unsigned)((tot + 255) / 256)), dim3(256), 0,
                       as_stream(stream), pts, N, C, sb, sn, sc, feat, D, fb, fn, fd, ctr, S, idx,
                       K, feature_first, tot, out, err);
    PN2_LAUNCH_CHECK("group_kernel");
    return PN2_OK;
}
