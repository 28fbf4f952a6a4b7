// pn2_internal.h -- shared host/device helpers for libpn2.so (gfx950 only).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdarg.h>
#include <stdio.h>

#include "pn2.h"

namespace pn2 {

// ---------------------------------------------------------------- host-side error plumbing
int set_error(int code, const char *fmt, ...);

#define PN2_REQUIRE(cond, ...)                                   \
    do {                                                         \
        if (!(cond)) return ::pn2::set_error(PN2_EINVAL, __VA_ARGS__); \
    } while (0)

// the launch's own error (hipGetLastError returns, and resets, the first error since the last
// call; its value is the one reported -- not a second call's hipSuccess)
#define PN2_LAUNCH_CHECK(what)                                                        \
    do {                                                                              \
        const hipError_t e_ = hipGetLastError();                                      \
        if (e_ != hipSuccess)                                                         \
            return ::pn2::set_error(PN2_EHIP, "%s: %s", what, hipGetErrorString(e_)); \
    } while (0)

static inline hipStream_t as_stream(void *s) { return reinterpret_cast<hipStream_t>(s); }

// ------------------------------------------------------------------ kernel-selection tuning
// Parameters of the launch choices (defaults = the measured best): process-wide (one atomic word
// per key, errors.cpp) or a thread's own copy (pn2_tuning_local).  Nothing reads
// the environment: tests and A/B tools set them through pn2_tuning_set (pn2/tuning.py parses
// the one PN2_TUNING variable).  X(name, default)
#define PN2_TUNING_KEYS(X)                                                                     \
    X(mlp_f32, 0)          /* 1: fp32 MFMA kernels instead of the split-bf16 ones          */ \
    X(chain_f16, 1)        /* 1: fp32-accurate chains as split fp16 (3 MFMAs per product)   */ \
    X(dense_frag, 1)       /* 1: dense hidden rows in MFMA-fragment order (register kernel) */ \
    X(dense_pair, 1)       /* 1: group_all's first two dense layers as one launch          */ \
    X(dense_f16, 1)        /* split fp16 dense layers: 1 after the first, 2 also the first  */ \
                           /* where eligible; 0: split bf16 (6)                             */ \
    X(chain_prepass, 1)    /* 0: no layer-0 pre-pass (wide first layers of a chain)        */ \
    X(compact, 1)          /* 0: no compact neighbourhoods (every padded row computed)     */ \
    X(compact_pool, 16)     /* LDS pool rows of compact chain launches (0: automatic)       */ \
    X(fps_prio, 1)         /* 1: FPS waves at raised issue priority (s_setprio 3)            */ \
    X(fps_side, 1)         /* 0: FPS side jobs as their own launches, not in the chain's    */ \
    X(compact_stages, 2)   /* weight-ring stages of compact chain launches (2 or 3)        */ \
    X(bq_waves, 16)        /* ball query waves per workgroup (8 or 16; 0: 16 for xyz clouds  */ \
                           /* of >= 2048 points, else 8 -- the pipelines' choice)           */ \
    X(bq_rowbuf_kb, 96)    /* largest LDS row buffer of the ball query (KB); bigger rows   */ \
                           /* are written straight to HBM (0: always)                      */ \
    X(fps_threads, 0)      /* FPS block shape threads x points per thread (0: automatic)   */ \
    X(fps_ppt, 0)                                                                              \
    X(fps_mid, 512)        /* automatic FPS block for 256 < N <= 1024: 512 threads x 2      */ \
                           /* points (fastest alone: the eager forward) or 256 x 4 (the     */ \
                           /* pipelines' geometry, beside the chains)                       */ \
    X(dense_maxntc, 2)     /* widest 32-column tile count of the 4-wave dense layer         */ \
    X(dense_minwg, 256)    /* workgroups a wider dense tile must still leave                 */ \
    X(dense_wide_minwg, 512) /* workgroups the 256 x 128 dense tile must leave              */ \
    X(dense_lds, 1)        /* 1: LDS-staged dense kernel for layers of >= dense_lds_mincin   */ \
                           /* (2: only first layers over points, group_all / pre-pass)      */ \
                           /* input channels (faster alone: the eager forward; the          */ \
                           /* pipelines run with 0, pn2/tuning.py PIPELINE_PROFILE)         */ \
    X(dense_lds_mincin, 0)                                                                     \
    X(dense_lds_stages, 3) /* ring stages of the LDS-staged dense kernel (3 or 4)            */ \
    X(dense_lds_xcd2d, 0)  /* 1: XCD rectangles of row blocks x column tiles                */ \
    X(dense_lds_tile, 0)   /* LDS-staged dense tile WR*10+NTW (82, 44, 42, 22; 0: auto)      */

struct Tuning {
#define PN2_TUNING_FIELD(name, dflt) int64_t name = dflt;
    PN2_TUNING_KEYS(PN2_TUNING_FIELD)
#undef PN2_TUNING_FIELD
};
// a snapshot of the calling thread's keys (its pn2_tuning_local copy, else the process-wide ones)
Tuning tuning();

// ---- device error slots (pn2_error_slot_set): two device words, [0] the PN2_DEVERR_* bits the
// kernels OR in, [1] the take kernel's snapshot.  error_word(st): the launching thread's slot on
// the device of the launch stream st (the current device for the null stream), else that
// device's process-wide default slot (a __device__ array, group.hip).
constexpr int kMaxDevices = 64;
int stream_device(hipStream_t st);  // -1 on a HIP error
unsigned *error_word(hipStream_t st);
unsigned *default_error_slot(int device);  // nullptr on a HIP error
bool is_default_error_slot(const unsigned *slot);
// one device atomic takes slot[0] (and with clear resets it: a bit raised meanwhile is never
// lost) into slot[1], copied to *bits; stream-ordered on st, which it then waits for
hipError_t take_errors(unsigned *slot, int clear, unsigned *bits, hipStream_t st);

constexpr int kMaxC = 16;      // point dims (xyz + one-hot) of the register-resident kernels
constexpr int kMaxCWide = 64;  // point dims of the streamed FPS / wide ball query (16 < C <= 64)

// np: bf16 planes per operand -- 3 = fp32-accurate split products, 1 = plain bf16 products
// sa_chain.hip: 1 launched, 0 not eligible, <0 error
int try_launch_chain(const pn2_sa_src &s, const pn2_mlp_layer *layers, int nlayers, int pool,
                     float *out, int64_t ostride, int64_t M, int64_t K, int np, float *ws,
                     int64_t ws_bytes, hipStream_t st);
// planes per operand of this thread's last chain launch (3 split bf16, 2 split fp16, 1 bf16)
int chain_last_planes();
// sa_dense.hip: split-bf16 layer-by-layer path for group_all / dense-row chains
int64_t dense_split_width(const pn2_sa_src &s, const pn2_mlp_layer *layers, int nlayers, int np);
int64_t dense_split_ws_bytes(int64_t M, int64_t w);
// FPS side jobs of SA MLP calls (pn2_fps_side, csrc/fps.hip): argument check, the separate
// launch (when no chain launch took the job), and the calling thread's "taken" flag that
// try_launch_chain sets when its launch runs the job
int fps_side_check(const pn2_fps_side &f);
int fps_side_launch(const pn2_fps_side &f, hipStream_t st);
bool &fps_side_taken();
// planes per operand carrying most of the flops of the calling thread's last dense-layer call
int dense_last_planes();
int try_launch_dense_split(const pn2_sa_src &s, const pn2_mlp_layer *layers, int nlayers, int pool,
                           float *out, int64_t ostride, float *ws, int64_t ws_bytes, int64_t M,
                           int64_t K, int np, hipStream_t st);
int launch_layer0_prepass(const pn2_sa_src &s, const pn2_mlp_layer &L0, float *z, hipStream_t st);
// bytes of workspace the chain kernel's layer-0 pre-pass needs for this chain (0: not used)
int64_t chain_prepass_bytes(const pn2_sa_src &s, const pn2_mlp_layer *layers, int nlayers, int np);

// --------------------------------------------------------------- device: reference sum orders
// torch.sum(x**2, -1) over the channel axis, reproduced bit-for-bit (torch 2.10 CPU, AVX512);
// pinned in oracle/pn2_oracle.c and tests/test_oracle_golden.py.
//  contig  (stride_c == 1):  C<8 -> row_sum with 4 accumulators; C>=8 -> 8 lane partials
//                            (8-channel vectors: whole 32-channel blocks into 4 vector
//                            accumulators, the leftover vectors into the first, then
//                            ((a0+a1)+a2)+a3 per lane), scalar tail first, then tail+v0+...+v7.
//  strided (stride_n == 1):  n < strided_body_points(N) (32*floor(N/32); 4 for N = 4..7) ->
//                            sequential within 16-channel chunks, the chunk sums added in
//                            order; the other points -> row_sum order.
// (C > 16 pinned to C = 64 by tools/probe/sum_orders_past_16.py and the r24/r40/r64 goldens;
// for C <= 16 both reduce to the plain forms.)
// `a` is a register array; C is runtime (<= CM).
// Element-wise adds in round-to-nearest.  The vector overload (two points per packed
// v_pk_add_f32) is a plain add under `fp contract(off)` (no product may be fused into it).
typedef float pn2_f2 __attribute__((ext_vector_type(2)));
// (__fadd_rn / __fmul_rn are plain operators in the HIP headers: contractible in a unit built
// with contraction on, e.g. the SA chain unit that runs the FPS side job)
__device__ __forceinline__ float add_rn(float a, float b) {
#pragma clang fp contract(off)
    return a + b;
}
__device__ __forceinline__ float mul_rn(float a, float b) {
#pragma clang fp contract(off)
    return a * b;
}
__device__ __forceinline__ pn2_f2 add_rn(pn2_f2 a, pn2_f2 b) {
#pragma clang fp contract(off)
    return a + b;
}

template <int CM, typename T>
__device__ __forceinline__ T seq_sum(const T (&a)[CM], int C) {
    T r = T(0.f);
#pragma unroll
    for (int k = 0; k < CM; ++k)
        if (k < C) r = add_rn(r, a[k]);
    return r;
}

template <int CM, typename T>
__device__ __forceinline__ T rowsum4(const T (&a)[CM], int C) {
    T acc[4] = {T(0.f), T(0.f), T(0.f), T(0.f)};
    const int n4 = (C / 4) * 4;
#pragma unroll
    for (int k = 0; k < CM; ++k) {
        if (k < n4) acc[k & 3] = add_rn(acc[k & 3], a[k]);
        else if (k < C) acc[0] = add_rn(acc[0], a[k]);
    }
    return add_rn(add_rn(add_rn(acc[0], acc[1]), acc[2]), acc[3]);
}

template <int CM, typename T>
__device__ __forceinline__ T contig_sum(const T (&a)[CM], int C) {
    if (C < 8) return rowsum4<CM>(a, C);
    const int nv8 = (C / 8) * 8;
    T v[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) v[k] = T(0.f);
    if constexpr (CM < 40) {
#pragma unroll
        for (int k = 0; k < CM; ++k)
            if (k < nv8) v[k & 7] = add_rn(v[k & 7], a[k]);
    } else {
        // 4 vector accumulators over whole 32-channel blocks, leftover vectors into the first
        const int nb32 = (C / 32) * 32;
        T u[3][8];
#pragma unroll
        for (int j = 0; j < 3; ++j)
#pragma unroll
            for (int l = 0; l < 8; ++l) u[j][l] = T(0.f);
#pragma unroll
        for (int k = 0; k < CM; ++k) {
            const int j = (k / 8) & 3;
            if (k < nb32 && j > 0) u[j - 1][k & 7] = add_rn(u[j - 1][k & 7], a[k]);
            else if (k < nv8) v[k & 7] = add_rn(v[k & 7], a[k]);
        }
        if (nb32 > 0) {
#pragma unroll
            for (int l = 0; l < 8; ++l) v[l] = add_rn(add_rn(add_rn(v[l], u[0][l]), u[1][l]), u[2][l]);
        }
    }
    T r = T(0.f);
#pragma unroll
    for (int k = 0; k < CM; ++k)
        if (k >= nv8 && k < C) r = add_rn(r, a[k]);
#pragma unroll
    for (int k = 0; k < 8; ++k) r = add_rn(r, v[k]);
    return r;
}

// strided rows' body points: sequential within 16-channel chunks, chunk sums in order
template <int CM, typename T>
__device__ __forceinline__ T chunk16_sum(const T (&a)[CM], int C) {
    if constexpr (CM <= 16) {
        return seq_sum<CM>(a, C);
    } else {
        T r = T(0.f), s = T(0.f);
#pragma unroll
        for (int k = 0; k < CM; ++k) {
            if (k < C) s = add_rn(s, a[k]);
            if (k % 16 == 15 || k == CM - 1) {
                if (k < 16) r = s;
                else if (k - k % 16 < C) r = add_rn(r, s);
                s = T(0.f);
            }
        }
        return r;
    }
}

// sum of squares of one row in the order ATen uses for its layout/position (rule: 0 contiguous,
// 1 strided body, 2 strided tail)
template <int CM, typename T>
__device__ __forceinline__ T layout_sum(const T (&a)[CM], int C, int rule) {
    if (rule == 0) return contig_sum<CM>(a, C);
    if (rule == 1) return chunk16_sum<CM>(a, C);
    return rowsum4<CM>(a, C);
}

// neighbour index i of a group-mode source (int64 lists, or the int32 ones of pn2_ball_query_i32)
__device__ __forceinline__ int src_index(const pn2_sa_src &s, int64_t i) {
    return s.idx32 ? s.idx32[i] : (int)s.idx[i];
}

__host__ __device__ __forceinline__ int layout_kind(int64_t sn, int64_t sc) {
    return (sc != 1 && sn == 1) ? 1 : 0;  // 1: point-contiguous ("strided") rows
}

// the strided rows summed by ATen's vectorised body: whole blocks of 32 points, or the first 4
// of a 4..7-point cloud (measured round 6 over N = 2..2064, C = 5..64; C <= 4 every order agrees)
__host__ __device__ __forceinline__ int64_t strided_body_points(int64_t N) {
    return N >= 32 ? (N / 32) * 32 : (N >= 4 && N < 8) ? 4 : 0;
}

__device__ __forceinline__ int point_rule(int kind, int64_t n, int64_t N) {
    if (kind == 0) return 0;
    return (n < strided_body_points(N)) ? 1 : 2;
}

// ----------------------------------------------------------------- device: wave reductions
// DPP row reductions: after these four steps every lane of a 16-lane row holds the row result.
// (quad_perm xor1 = 0xB1, xor2 = 0x4E, row_half_mirror = 0x141, row_mirror = 0x140)
#define PN2_DPP(v, ctrl) \
    static_cast<unsigned>(__builtin_amdgcn_update_dpp(0, static_cast<int>(v), ctrl, 0xF, 0xF, false))

__device__ __forceinline__ unsigned wave_max_u32(unsigned v) {
    v = max(v, PN2_DPP(v, 0xB1));
    v = max(v, PN2_DPP(v, 0x4E));
    v = max(v, PN2_DPP(v, 0x141));
    v = max(v, PN2_DPP(v, 0x140));
    unsigned a = __builtin_amdgcn_readlane(v, 0), b = __builtin_amdgcn_readlane(v, 16);
    unsigned c = __builtin_amdgcn_readlane(v, 32), d = __builtin_amdgcn_readlane(v, 48);
    return max(max(a, b), max(c, d));
}

__device__ __forceinline__ unsigned wave_min_u32(unsigned v) {
    // min via bitwise-not max (update_dpp's `old`=0 only matters for masked lanes; none here)
    return ~wave_max_u32(~v);
}

// Logical workgroup id under which every XCD runs a contiguous range of ids (dispatch places
// workgroup i on XCD i % 8, each XCD with its own L2): consecutive logical ids -- a cloud's
// row blocks, or the groups of one cloud -- share an L2.  Identity unless n % 8 == 0.
__device__ __forceinline__ unsigned xcd_contiguous(unsigned id, unsigned n) {
    return (n & 7u) ? id : (id & 7u) * (n >> 3) + (id >> 3);
}

__device__ __forceinline__ int lane_id() { return __builtin_amdgcn_mbcnt_hi(~0u, __builtin_amdgcn_mbcnt_lo(~0u, 0u)); }

}  // namespace pn2
