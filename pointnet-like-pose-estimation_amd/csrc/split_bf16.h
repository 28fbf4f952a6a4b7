// split_bf16.h -- fp32-accurate products on the bf16 matrix cores (gfx950), shared by the
// register-resident chain kernel (sa_chain.hip) and the dense layer kernel (sa_dense.hip).
//
// An fp32 operand x is split into three bf16 planes x = h + m + l (round-to-nearest; the
// residuals are exact in fp32, so the planes hold x to 2^-24 relative).  A product is taken as
// hh + hm + mh + mm + hl + lh -- each an exact bf16 x bf16 product accumulated in fp32 by
// v_mfma_f32_32x32x16_bf16 -- and the three dropped terms are <= 2^-23 of it: fp32-GEMM
// accuracy at 6/16 of the fp32 MFMA cost.
#pragma once
#include <hip/hip_runtime.h>

namespace pn2 {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float cfloatx16 __attribute__((ext_vector_type(16)));
typedef float cfloatx4 __attribute__((ext_vector_type(4)));

struct Split {
    bf16x8 h, m, l;
};

__device__ __forceinline__ float chain_relu(float t) { return t > 0.f ? t : 0.f; }  // never -0

__device__ __forceinline__ Split split8(const float (&x)[8]) {
    Split s;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
        const __bf16 a = (__bf16)x[j];
        const float r = x[j] - (float)a;
        const __bf16 b = (__bf16)r;
        const float r2 = r - (float)b;
        s.h[j] = a;
        s.m[j] = b;
        s.l[j] = (__bf16)r2;
    }
    return s;
}

#define PN2_MFMA16 __builtin_amdgcn_mfma_f32_32x32x16_bf16
// acc += a * b with both operands split (6 bf16 products).  The weight operand's planes are
// consumed in the order they are read from the ring (hi, mid, lo), so the first products can
// start while the later planes are still in flight.
__device__ __forceinline__ cfloatx16 mma6_wa(const Split &w, const Split &x, cfloatx16 acc) {
    acc = PN2_MFMA16(w.h, x.h, acc, 0, 0, 0);
    acc = PN2_MFMA16(w.h, x.m, acc, 0, 0, 0);
    acc = PN2_MFMA16(w.h, x.l, acc, 0, 0, 0);
    acc = PN2_MFMA16(w.m, x.h, acc, 0, 0, 0);
    acc = PN2_MFMA16(w.m, x.m, acc, 0, 0, 0);
    acc = PN2_MFMA16(w.l, x.h, acc, 0, 0, 0);
    return acc;
}
__device__ __forceinline__ cfloatx16 mma6_wb(const Split &x, const Split &w, cfloatx16 acc) {
    acc = PN2_MFMA16(x.h, w.h, acc, 0, 0, 0);
    acc = PN2_MFMA16(x.m, w.h, acc, 0, 0, 0);
    acc = PN2_MFMA16(x.l, w.h, acc, 0, 0, 0);
    acc = PN2_MFMA16(x.h, w.m, acc, 0, 0, 0);
    acc = PN2_MFMA16(x.m, w.m, acc, 0, 0, 0);
    acc = PN2_MFMA16(x.h, w.l, acc, 0, 0, 0);
    return acc;
}

__device__ __forceinline__ Split ring_read(const char *slot, int lane) {
    const bf16x8 *q = reinterpret_cast<const bf16x8 *>(slot) + lane;
    Split w;
    w.h = q[0];
    w.m = q[64];
    w.l = q[128];
    return w;
}

// ---- plane count NP: 3 = the fp32-accurate split above; 1 = plain bf16 arithmetic (operands
// rounded to bf16 -- the hi plane -- products exact, fp32 accumulation), one MFMA per product.
// NP == 1 leaves m / l as copies of h; nothing reads them, so they cost nothing.
template <int NP>
__device__ __forceinline__ Split splitN(const float (&x)[8]) {
    if constexpr (NP == 3) {
        return split8(x);
    } else {
        static_assert(NP == 1, "plane count");
        Split s;
#pragma unroll
        for (int j = 0; j < 8; ++j) s.h[j] = (__bf16)x[j];
        s.m = s.h;
        s.l = s.h;
        return s;
    }
}
template <int NP>
__device__ __forceinline__ cfloatx16 mma_wa(const Split &w, const Split &x, cfloatx16 acc) {
    if constexpr (NP == 3) return mma6_wa(w, x, acc);
    else return PN2_MFMA16(w.h, x.h, acc, 0, 0, 0);
}
template <int NP>
__device__ __forceinline__ cfloatx16 mma_wb(const Split &x, const Split &w, cfloatx16 acc) {
    if constexpr (NP == 3) return mma6_wb(x, w, acc);
    else return PN2_MFMA16(x.h, w.h, acc, 0, 0, 0);
}
// a step's NP plane fragments stored back to back (1 KB each) in LDS
template <int NP>
__device__ __forceinline__ Split ring_readN(const char *slot, int lane) {
    if constexpr (NP == 3) {
        return ring_read(slot, lane);
    } else {
        Split w;
        w.h = reinterpret_cast<const bf16x8 *>(slot)[lane];
        w.m = w.h;
        w.l = w.h;
        return w;
    }
}

// max / min of x over lanes l and l^32 (the two halves of a 32x32 tile column): one
// v_permlane32_swap (a VALU lane exchange) in place of a ds_bpermute LDS round trip.  The swap
// leaves lane l < 32 with (x[l], x[l+32]) and lane l >= 32 with (x[l-32], x[l]).
__device__ __forceinline__ float max_halves(float x) {
    const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(x), __float_as_uint(x), false, false);
    return fmaxf(__uint_as_float(r[0]), __uint_as_float(r[1]));
}
__device__ __forceinline__ float min_halves(float x) {
    const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(x), __float_as_uint(x), false, false);
    return fminf(__uint_as_float(r[0]), __uint_as_float(r[1]));
}

typedef __attribute__((address_space(3))) void lds_void;

}  // namespace pn2
