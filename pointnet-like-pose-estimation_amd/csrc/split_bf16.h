// split_bf16.h -- fp32-accurate products on the 16-bit matrix cores (gfx950), shared by the
// register-resident chain kernel (sa_chain.hip) and the dense layer kernel (sa_dense.hip).
//
// NP = 3 (split bf16): an fp32 operand x is split into three bf16 planes x = h + m + l
// (round-to-nearest; the residuals are exact in fp32, so the planes hold x to 2^-24 relative).
// A product is taken as hh + hm + mh + mm + hl + lh -- each an exact bf16 x bf16 product
// accumulated in fp32 by v_mfma_f32_32x32x16_bf16 -- and the three dropped terms are <= 2^-23 of
// it: fp32-GEMM accuracy at 6/16 of the fp32 MFMA cost.
//
// NP = 2 (split fp16): x = h + m in two fp16 planes (h = f16(x), m = f16(x - h), round-to-
// nearest: 22 significant bits, x to 2^-22 relative while m stays a normal fp16), and a product
// is hh + hm + mh by v_mfma_f32_32x32x16_f16 (the dropped mm <= 2^-22): 3 MFMAs instead of 6,
// two 1 KB weight planes per step instead of three.  fp16's exponent range is narrow, so both
// operands are scaled by powers of two first (exact): each weight row (output channel) so that
// its largest |w| lies in [2^14, 2^15) (pack_split_kernel; the inverse scale is folded into the
// BN scale), each wave's 32 activation rows by one wave-uniform factor that puts their largest
// |x| in [2^14, 2^15) (act_scale; folded into the consuming layer's BN scale likewise).  Scaling
// by 2^k commutes with fp32 rounding, so the result is that of an unbounded-exponent split;
// values more than 2^17 below their wave's / row's maximum lose relative precision, but their
// absolute error stays below 2^-39 of that maximum.
#pragma once
#include <hip/hip_runtime.h>

namespace pn2 {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
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

// NP = 2: fp16 planes h, m of x (held in bf16x8 containers: Split's registers are 16-bit data)
__device__ __forceinline__ Split split8_f16(const float (&x)[8]) {
    Split s;
    f16x8 a, b;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
        a[j] = (_Float16)x[j];
        b[j] = (_Float16)(x[j] - (float)a[j]);
    }
    s.h = __builtin_bit_cast(bf16x8, a);
    s.m = __builtin_bit_cast(bf16x8, b);
    s.l = s.h;  // unused
    return s;
}

#define PN2_MFMA16 __builtin_amdgcn_mfma_f32_32x32x16_bf16
#define PN2_MFMA16H(a, b, c) \
    __builtin_amdgcn_mfma_f32_32x32x16_f16(__builtin_bit_cast(f16x8, a), __builtin_bit_cast(f16x8, b), c, 0, 0, 0)
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

// ---- plane count NP: 3 = the fp32-accurate bf16 split above; 2 = the fp32-accurate fp16 split
// (operands pre-scaled, see the header); 1 = plain bf16 arithmetic (operands rounded to bf16 --
// the hi plane -- products exact, fp32 accumulation), one MFMA per product.
// Unused planes are copies of h; nothing reads them, so they cost nothing.
template <int NP>
__device__ __forceinline__ Split splitN(const float (&x)[8]) {
    if constexpr (NP == 3) {
        return split8(x);
    } else if constexpr (NP == 2) {
        return split8_f16(x);
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
    if constexpr (NP == 3) {
        return mma6_wa(w, x, acc);
    } else if constexpr (NP == 2) {
        acc = PN2_MFMA16H(w.h, x.h, acc);
        acc = PN2_MFMA16H(w.h, x.m, acc);
        return PN2_MFMA16H(w.m, x.h, acc);
    } else {
        return PN2_MFMA16(w.h, x.h, acc, 0, 0, 0);
    }
}
template <int NP>
__device__ __forceinline__ cfloatx16 mma_wb(const Split &x, const Split &w, cfloatx16 acc) {
    if constexpr (NP == 3) {
        return mma6_wb(x, w, acc);
    } else if constexpr (NP == 2) {
        acc = PN2_MFMA16H(x.h, w.h, acc);
        acc = PN2_MFMA16H(x.m, w.h, acc);
        return PN2_MFMA16H(x.h, w.m, acc);
    } else {
        return PN2_MFMA16(x.h, w.h, acc, 0, 0, 0);
    }
}
// a step's NP plane fragments stored back to back (1 KB each) in LDS
template <int NP>
__device__ __forceinline__ Split ring_readN(const char *slot, int lane) {
    if constexpr (NP == 3) {
        return ring_read(slot, lane);
    } else if constexpr (NP == 2) {
        const bf16x8 *q = reinterpret_cast<const bf16x8 *>(slot) + lane;
        Split w;
        w.h = q[0];
        w.m = q[64];
        w.l = w.h;
        return w;
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

// NP = 2 activation scaling: the factor 2^k that puts m (the largest |x| of the wave's rows, a
// wave-uniform value >= 0) in [2^14, 2^15), and its inverse; 1 for m = 0.  k is clamped so both
// factors stay normal floats.
struct ActScale {
    float up, down;
};
__device__ __forceinline__ ActScale act_scale(float m) {
    int k = 0;
    if (m > 0.f) k = 15 - __builtin_amdgcn_frexp_expf(m);  // m in [2^(e-1), 2^e)
    k = k < -100 ? -100 : (k > 100 ? 100 : k);
    ActScale a;
    a.up = __uint_as_float((unsigned)(127 + k) << 23);
    a.down = __uint_as_float((unsigned)(127 - k) << 23);
    return a;
}

// the NP = 2 planes (3-4) and the row scales inside a pn2_pack_layer_split_bf16 image of a layer
// with `cout` outputs and `kbs` input k-blocks (include/pn2.h)
__host__ __device__ inline const bf16x8 *split_f16_planes(const void *img, int64_t cout, int64_t kbs) {
    return reinterpret_cast<const bf16x8 *>(static_cast<const char *>(img) + 3 * cout * kbs * 32);
}
__host__ __device__ inline const float *split_f16_inv_scale(const void *img, int64_t cout, int64_t kbs) {
    return reinterpret_cast<const float *>(static_cast<const char *>(img) + 5 * cout * kbs * 32);
}

// NP = 2 dense layers (sa_dense.hip): the producing layer leaves, per 32-row block and 32-column
// output tile, the largest |value| it wrote (uint bits, >= 0: order-preserving), so the consuming
// layer's wave knows its 32 rows' scale before it splits its first k-block (pn2_internal.h's
// wave_max_u32 reduces a lane's maxima; lane 0 stores the entry).
typedef __attribute__((address_space(3))) void lds_void;

}  // namespace pn2
