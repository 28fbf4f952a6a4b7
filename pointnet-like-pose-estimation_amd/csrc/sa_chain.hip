// sa_chain.hip -- register-resident SA layer chain for gfx950: gather -> 3 x (1x1 conv + BN +
// ReLU) -> max over the neighbourhood, with fp32-accurate products on the bf16 matrix cores.
//
// Same job as sa_mlp.hip's fused kernel (PointNetSetAbstraction.forward :163-172,
// PointNetSetAbstractionMsg.forward :211-221 of /root/reference/model/pointnet2_utils.py) for
// the chains every reference head uses (3 layers, hidden widths <= 128, grouped rows).
//
// Arithmetic.  Every fp32 operand x is split into three bf16 planes, x = h + m + l exactly up to
// 2^-24 |x| (h = bf16(x), m = bf16(x - h), l = bf16(x - h - m), round-to-nearest, the residuals
// are exact in fp32).  A product x*w is taken as hh + hm + mh + mm + hl + lh (the dropped terms
// are <= 2^-23 |xw|), each an exact bf16 x bf16 product accumulated in fp32 by
// v_mfma_f32_32x32x16_bf16.  The result has fp32-GEMM accuracy (tests hold it to the same
// 1e-5 bar as the fp32 path) at 6/16 of the fp32 MFMA cost.
//
// Data flow.  One wave owns a slab of 32 consecutive rows (a row = one (group, neighbour) pair)
// and carries it through the whole chain in registers -- no LDS for activations:
//   layer 0   (hidden, transposed: acc[cout tile] += W . X^T) streams 16-channel blocks of the
//             gathered rows from HBM (two 16-byte loads per lane per block: channel-last
//             features, then xyz - centroid), splits them and accumulates every output tile.
//   layer 1   (hidden, transposed) reads its input from registers: the transposed output tile
//             of the previous layer holds, in lane (row r, half h), channels
//             32t + (q&3) + 8(q>>2) + 4h of row r in register q -- exactly the B fragment of the
//             next layer's k-blocks 2t, 2t+1 when the weights are packed with that channel
//             order (pn2_pack_layer_split_bf16).  BN + ReLU + split happen in the epilogue.
//   layer 2   (last, standard orientation: acc[row][col] += X . W^T) takes the same registers
//             as its A operand, so each lane ends with one output column and the tile's rows in
//             registers: the max over the neighbourhood is a register reduction (+ one lane
//             exchange), merged across slabs in LDS (ds_max_u32) or HBM (atomicMax) when a
//             group spans several slabs (ReLU output >= +0: uint order == float order).
// Weights stream from L2 (1 KB per fragment and plane, shared by every wave on the chip).
#include "pn2_internal.h"

#include <cstdlib>
#include <cstring>

namespace pn2 {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float cfloatx16 __attribute__((ext_vector_type(16)));
typedef float cfloatx4 __attribute__((ext_vector_type(4)));

constexpr int kChainWaves = 4;
constexpr int kChainRows = 32 * kChainWaves;

struct ChainLayer {
    const bf16x8 *w;  // [3][tiles][kb][64] fragments
    const float *alpha;
    const float *beta;
    int kb;     // 16-deep k blocks of the input
    int tiles;  // 32-wide output tiles
};

struct ChainArgs {
    pn2_sa_src src;
    ChainLayer L[3];
    int M, K, S, C, D;
    int pool_mode;  // 0: registers, 1: LDS (groups inside a workgroup), 2: HBM atomics
    int vec_feat;
    float *out;
    int64_t ostride;
};

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
// acc += a * b with both operands split (6 bf16 products)
__device__ __forceinline__ cfloatx16 mma6(const Split &a, const Split &b, cfloatx16 acc) {
    acc = PN2_MFMA16(a.l, b.h, acc, 0, 0, 0);
    acc = PN2_MFMA16(a.h, b.l, acc, 0, 0, 0);
    acc = PN2_MFMA16(a.m, b.m, acc, 0, 0, 0);
    acc = PN2_MFMA16(a.m, b.h, acc, 0, 0, 0);
    acc = PN2_MFMA16(a.h, b.m, acc, 0, 0, 0);
    acc = PN2_MFMA16(a.h, b.h, acc, 0, 0, 0);
    return acc;
}

__device__ __forceinline__ Split load_w(const ChainLayer &L, int t, int kb, int lane) {
    const int64_t plane = (int64_t)L.tiles * L.kb * 64;
    const bf16x8 *p = L.w + ((int64_t)t * L.kb + kb) * 64 + lane;
    Split s;
    s.h = p[0];
    s.m = p[plane];
    s.l = p[2 * plane];
    return s;
}

// BN + ReLU of a transposed hidden tile, split into the next layer's k-blocks 2t, 2t+1
__device__ __forceinline__ void hidden_epilogue(const cfloatx16 &acc, const ChainLayer &L, int t,
                                                int h, Split &lo, Split &hi) {
    cfloatx4 a4[4], b4[4];
#pragma unroll
    for (int m = 0; m < 4; ++m) {
        a4[m] = *reinterpret_cast<const cfloatx4 *>(L.alpha + 32 * t + 8 * m + 4 * h);
        b4[m] = *reinterpret_cast<const cfloatx4 *>(L.beta + 32 * t + 8 * m + 4 * h);
    }
    float y0[8], y1[8];
#pragma unroll
    for (int q = 0; q < 8; ++q) {
        y0[q] = chain_relu(__builtin_fmaf(acc[q], a4[q >> 2][q & 3], b4[q >> 2][q & 3]));
        y1[q] = chain_relu(__builtin_fmaf(acc[q + 8], a4[2 + (q >> 2)][q & 3], b4[2 + (q >> 2)][q & 3]));
    }
    lo = split8(y0);
    hi = split8(y1);
}

template <int T0, int T1>
__global__ __launch_bounds__(64 * kChainWaves) void sa_chain_kernel(const ChainArgs A) {
    extern __shared__ __attribute__((aligned(16))) unsigned cpool[];
    const int tid = threadIdx.x;
    const int lane = tid & 63;
    const int r = lane & 31, h = lane >> 5;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int slab = blockIdx.x * kChainWaves + wave;
    const pn2_sa_src &s = A.src;
    const ChainLayer &L0 = A.L[0], &L1 = A.L[1], &L2 = A.L[2];
    const int coutL = 32 * L2.tiles;
    const int gpb = kChainRows / A.K;  // groups per workgroup (pool_mode 1)

    if (A.pool_mode == 1) {
        for (int e = tid; e < gpb * coutL; e += 64 * kChainWaves) cpool[e] = 0u;
        __syncthreads();
    }

    // ---- this lane's row: (group g, batch b, point n)
    const unsigned R = (unsigned)slab * 32u + (unsigned)r;
    const bool valid = R < (unsigned)A.M;
    const unsigned g = valid ? R / (unsigned)A.K : 0u;
    const unsigned b = g / (unsigned)A.S;
    const int n = valid ? (int)s.idx[R] : 0;
    const float *frow = s.feat ? s.feat + (int64_t)b * s.fb + (int64_t)n * s.fn : nullptr;
    const float *prow = s.pts + (int64_t)b * s.pb + (int64_t)n * s.pn;
    const float *crow = s.ctr + (int64_t)g * A.C;
    const int D = A.D, C = A.C;

    // 4 channels [c, c+4) of the row layout [feature | xyz - centroid | 0]
    auto load_run = [&](int c, float *v) {
        if (!valid) {
#pragma unroll
            for (int i = 0; i < 4; ++i) v[i] = 0.f;
        } else if (A.vec_feat && c + 4 <= D) {
            const cfloatx4 q = *reinterpret_cast<const cfloatx4 *>(frow + c);
#pragma unroll
            for (int i = 0; i < 4; ++i) v[i] = q[i];
        } else {
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                const int ch = c + i;
                v[i] = ch < D ? frow[ch]
                     : ch < D + C ? __fsub_rn(prow[(int64_t)(ch - D) * s.pc], crow[ch - D])
                     : 0.f;
            }
        }
    };
    // lane (r, h) holds channels 16kb + (j&3) + 8(j>>2) + 4h of its row in element j
    auto load_x = [&](int kb, float (&x)[8]) {
        load_run(16 * kb + 4 * h, x);
        load_run(16 * kb + 8 + 4 * h, x + 4);
    };

    // ---- layer 0: stream the gathered input, accumulate every output tile (transposed)
    Split X1[2 * T0];
    {
        cfloatx16 acc[T0];
#pragma unroll
        for (int t = 0; t < T0; ++t)
#pragma unroll
            for (int q = 0; q < 16; ++q) acc[t][q] = 0.f;
        float xn[8];
        load_x(0, xn);
        for (int kb = 0; kb < L0.kb; ++kb) {
            float x[8];
#pragma unroll
            for (int j = 0; j < 8; ++j) x[j] = xn[j];
            if (kb + 1 < L0.kb) load_x(kb + 1, xn);
            const Split xs = split8(x);
#pragma unroll
            for (int t = 0; t < T0; ++t) acc[t] = mma6(load_w(L0, t, kb, lane), xs, acc[t]);
        }
#pragma unroll
        for (int t = 0; t < T0; ++t) hidden_epilogue(acc[t], L0, t, h, X1[2 * t], X1[2 * t + 1]);
    }

    // ---- layer 1: input in registers, one output tile at a time (transposed)
    Split X2[2 * T1];
#pragma unroll
    for (int t = 0; t < T1; ++t) {
        cfloatx16 acc;
#pragma unroll
        for (int q = 0; q < 16; ++q) acc[q] = 0.f;
#pragma unroll
        for (int kb = 0; kb < 2 * T0; ++kb) acc = mma6(load_w(L1, t, kb, lane), X1[kb], acc);
        hidden_epilogue(acc, L1, t, h, X2[2 * t], X2[2 * t + 1]);
    }

    // ---- layer 2: standard orientation, pooled over the neighbourhood
    const unsigned G = (unsigned)A.M / (unsigned)A.K;
    for (int t = 0; t < L2.tiles; ++t) {
        cfloatx16 acc;
#pragma unroll
        for (int q = 0; q < 16; ++q) acc[q] = 0.f;
#pragma unroll
        for (int kb = 0; kb < 2 * T1; ++kb) acc = mma6(X2[kb], load_w(L2, t, kb, lane), acc);
        const int col = 32 * t + r;
        const float al = L2.alpha[col], be = L2.beta[col];
        float v[16];
#pragma unroll
        for (int q = 0; q < 16; ++q) v[q] = chain_relu(__builtin_fmaf(acc[q], al, be));
        // register q of lane half h is row (q&3) + 8(q>>2) + 4h of the slab
        if (A.K == 8 || A.K == 16) {
            constexpr int kParts = 4;
            float m[kParts];
#pragma unroll
            for (int k = 0; k < kParts; ++k)
                m[k] = fmaxf(fmaxf(v[4 * k], v[4 * k + 1]), fmaxf(v[4 * k + 2], v[4 * k + 3]));
#pragma unroll
            for (int k = 0; k < kParts; ++k) m[k] = fmaxf(m[k], __shfl_xor(m[k], 32));
            // rows 8k..8k+7 of the slab are register group k (both halves)
            if (h == 0) {
                if (A.K == 8) {
#pragma unroll
                    for (int k = 0; k < kParts; ++k) {
                        const unsigned gg = (unsigned)slab * 4u + k;
                        if (gg < G) A.out[(int64_t)gg * A.ostride + col] = m[k];
                    }
                } else {
#pragma unroll
                    for (int k = 0; k < 2; ++k) {
                        const unsigned gg = (unsigned)slab * 2u + k;
                        if (gg < G) A.out[(int64_t)gg * A.ostride + col] = fmaxf(m[2 * k], m[2 * k + 1]);
                    }
                }
            }
        } else {
            float m = 0.f;
#pragma unroll
            for (int q = 0; q < 16; ++q) m = fmaxf(m, v[q]);
            m = fmaxf(m, __shfl_xor(m, 32));
            const unsigned gg = ((unsigned)slab * 32u) / (unsigned)A.K;
            if (h == 0 && (unsigned)slab * 32u < (unsigned)A.M) {
                if (A.pool_mode == 0) A.out[(int64_t)gg * A.ostride + col] = m;
                else if (A.pool_mode == 1)
                    atomicMax(&cpool[(int)(gg - (unsigned)blockIdx.x * gpb) * coutL + col], __float_as_uint(m));
                else
                    atomicMax(reinterpret_cast<unsigned *>(A.out + (int64_t)gg * A.ostride + col), __float_as_uint(m));
            }
        }
    }
    if (A.pool_mode == 1) {
        __syncthreads();
        for (int e = tid; e < gpb * coutL; e += 64 * kChainWaves) {
            const int gl = e / coutL, c = e - gl * coutL;
            const unsigned gg = (unsigned)blockIdx.x * gpb + gl;
            if (gg < G) A.out[(int64_t)gg * A.ostride + c] = __uint_as_float(cpool[e]);
        }
    }
}

// hidden-width signatures (output tiles of layers 0 and 1) compiled; the reference heads use
// SSG [64,64,128] [128,128,256], MSG [32,32,64] [64,64,128] [64,96,128] [128,128,256]
#define PN2_CHAIN_SIGS(X) X(1, 1) X(2, 2) X(2, 3) X(4, 4)

}  // namespace pn2

using namespace pn2;

// ------------------------------------------------------------------ weight packing
// plane p, tile t, block kb, lane l = 32h + r, element j:
//   W[32t + r][(k + rot) % cin] with k = 16kb + (j&3) + 8(j>>2) + 4h  (0 for k >= cin)
__global__ __launch_bounds__(256) void pack_split_kernel(const float *__restrict__ W, int cout,
                                                          int cin, int kbs, int rot,
                                                          __bf16 *__restrict__ out) {
    const int64_t per_plane = (int64_t)cout * kbs * 16;
    const int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (e >= per_plane) return;
    const int j = (int)(e & 7);
    const int l = (int)((e >> 3) & 63);
    const int64_t f = e >> 9;  // fragment = t * kbs + kb
    const int kb = (int)(f % kbs), t = (int)(f / kbs);
    const int r = l & 31, h = l >> 5;
    const int k = 16 * kb + (j & 3) + 8 * (j >> 2) + 4 * h;
    const float w = k < cin ? W[(int64_t)(32 * t + r) * cin + (k + rot) % cin] : 0.f;
    const __bf16 a = (__bf16)w;
    const float r1 = w - (float)a;
    const __bf16 m = (__bf16)r1;
    const __bf16 lo = (__bf16)(r1 - (float)m);
    out[e] = a;
    out[per_plane + e] = m;
    out[2 * per_plane + e] = lo;
}

extern "C" int64_t pn2_layer_split_bytes(int64_t cout, int64_t cin) {
    if (cout < 32 || cout % 32 != 0 || cin < 1) return -1;
    return 3 * cout * ((cin + 15) / 16) * 16 * 2;
}

extern "C" int pn2_pack_layer_split_bf16(const float *W, int64_t cout, int64_t cin, int64_t rot,
                                         void *out, void *stream) {
    PN2_REQUIRE(W && out, "pn2_pack_layer_split_bf16: null pointer");
    PN2_REQUIRE(cout >= 32 && cout % 32 == 0 && cin >= 1 && rot >= 0 && rot < cin,
                "pn2_pack_layer_split_bf16: bad shape cout=%lld cin=%lld rot=%lld", (long long)cout,
                (long long)cin, (long long)rot);
    PN2_REQUIRE(((uintptr_t)out & 15) == 0, "pn2_pack_layer_split_bf16: output not 16-byte aligned");
    const int kbs = (int)((cin + 15) / 16);
    const int64_t per_plane = cout * kbs * 16;
    hipLaunchKernelGGL(pack_split_kernel, dim3((unsigned)((per_plane + 255) / 256)), dim3(256), 0,
                       as_stream(stream), W, (int)cout, (int)cin, kbs, (int)rot,
                       reinterpret_cast<__bf16 *>(out));
    PN2_LAUNCH_CHECK("pack_split_kernel");
    return PN2_OK;
}

// ------------------------------------------------------------------ host: dispatch
namespace pn2 {

template <int T0, int T1>
static int launch_chain_sig(const ChainArgs &A, unsigned grid, size_t lds, hipStream_t st) {
    hipLaunchKernelGGL((sa_chain_kernel<T0, T1>), dim3(grid), dim3(64 * kChainWaves), lds, st, A);
    PN2_LAUNCH_CHECK("sa_chain_kernel");
    return PN2_OK;
}

static bool chain_sig_compiled(int T0, int T1) {
#define PN2_CHAIN_HAS(a, b) \
    if (T0 == a && T1 == b) return true;
    PN2_CHAIN_SIGS(PN2_CHAIN_HAS)
#undef PN2_CHAIN_HAS
    return false;
}

// 1: launched, 0: this chain is not eligible (caller uses the fp32 kernels), <0: error
int try_launch_chain(const pn2_sa_src &s, const pn2_mlp_layer *layers, int nlayers, int pool,
                     float *out, int64_t ostride, int64_t M, int64_t K, hipStream_t st) {
    if (const char *e = getenv("PN2_MLP_PATH"))
        if (strcmp(e, "f32") == 0) return 0;
    if (nlayers != 3 || !pool) return 0;
    if (s.mode != PN2_SRC_GROUP_XYZ_FIRST && s.mode != PN2_SRC_GROUP_FEAT_FIRST) return 0;
    if (s.C > kMaxC) return 0;
    for (int l = 0; l < 3; ++l)
        if (!layers[l].wt_split || ((uintptr_t)layers[l].wt_split & 15)) return 0;
    const int T0 = (int)(layers[0].cout / 32), T1 = (int)(layers[1].cout / 32);
    if (!chain_sig_compiled(T0, T1)) return 0;
    if (!(K == 8 || K == 16 || K % 32 == 0)) return 0;

    ChainArgs A;
    memset(&A, 0, sizeof(A));
    A.src = s;
    for (int l = 0; l < 3; ++l) {
        A.L[l].w = reinterpret_cast<const bf16x8 *>(layers[l].wt_split);
        A.L[l].alpha = layers[l].alpha;
        A.L[l].beta = layers[l].beta;
        A.L[l].kb = (int)((layers[l].cin + 15) / 16);
        A.L[l].tiles = (int)(layers[l].cout / 32);
    }
    A.M = (int)M;
    A.K = (int)K;
    A.S = (int)s.S;
    A.C = (int)s.C;
    A.D = (int)s.D;
    A.out = out;
    A.ostride = ostride;
    A.vec_feat = (s.D > 0 && s.D % 4 == 0 && ((uintptr_t)s.feat & 15) == 0 && s.fn % 4 == 0 &&
                  s.fb % 4 == 0) ? 1 : 0;
    const int64_t coutL = layers[2].cout;
    size_t lds = 0;
    if (K == 8 || K == 16 || K == 32) {
        A.pool_mode = 0;
    } else if (kChainRows % K == 0) {
        A.pool_mode = 1;
        lds = (size_t)(kChainRows / K) * coutL * 4;
    } else {
        A.pool_mode = 2;
    }
    if (lds > 64 * 1024) A.pool_mode = 2, lds = 0;
    if (A.pool_mode == 2) {
        const int64_t G = M / K;
        hipError_t e = (ostride == coutL)
                           ? hipMemsetAsync(out, 0, (size_t)G * coutL * 4, st)
                           : hipMemset2DAsync(out, (size_t)ostride * 4, 0, (size_t)coutL * 4, (size_t)G, st);
        if (e != hipSuccess) return set_error(PN2_EHIP, "sa_chain: memset: %s", hipGetErrorString(e));
    }
    const unsigned grid = (unsigned)((M + kChainRows - 1) / kChainRows);
    int rc = PN2_EUNSUPPORTED;
#define PN2_CHAIN_GO(a, b) \
    if (T0 == a && T1 == b) rc = launch_chain_sig<a, b>(A, grid, lds, st);
    PN2_CHAIN_SIGS(PN2_CHAIN_GO)
#undef PN2_CHAIN_GO
    return rc == PN2_OK ? 1 : rc;
}

}  // namespace pn2
