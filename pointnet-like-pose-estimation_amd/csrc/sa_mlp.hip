// sa_mlp.hip -- fused set-abstraction MLP for gfx950: gather -> (1x1 conv + BN + ReLU)* -> max.
//
// Replaces, for eval-mode inference, the SA feature path of
//   PointNetSetAbstraction.forward     /root/reference/model/pointnet2_utils.py:158-174
//   PointNetSetAbstractionMsg.forward  /root/reference/model/pointnet2_utils.py:195-223
// i.e. index_points of the neighbourhoods (:109-116, :205-209; :137-139 for group_all),
// permute to [B,C,K,S] (:167, :211), the Conv2d-1x1 / BatchNorm2d / ReLU stack (:168-170,
// :213-216) and torch.max over the neighbourhood axis (:172, :218).
//
// Rows are (group, neighbour) pairs: M = B*S*K.  A workgroup owns BM consecutive rows
// (BM/32 row tiles x 2 column halves = BM/16 waves) and runs the whole layer chain on them:
//   1. gather: each row's [xyz - centroid | feature] (or MSG / group_all order) is read from
//      HBM (features channels-last, so one row is one contiguous run) into an LDS activation
//      tile act[BM][ld] (ld odd -> the column-of-rows A-fragment reads are bank-conflict free);
//   2. per layer: W^T is streamed through a double-buffered 16 KB LDS chunk (register-staged
//      prefetch of chunk c+1 overlaps the MFMAs of chunk c), each wave accumulates up to 4
//      32x32 output tiles with v_mfma_f32_32x32x2_f32 (exact fp32 products, fma-chain
//      accumulation) and applies the folded BN scale/shift + ReLU in the epilogue, writing the
//      hidden activations back into the same LDS tile -- hidden layers never touch HBM;
//   3. last layer: max over each group's K rows in registers (16 accumulators + one cross-half
//      exchange when K % 32 == 0), merged across waves with LDS ds_max_u32 on the float bits
//      (ReLU output is >= +0, so uint order == float order), one coalesced store per group;
//      groups that straddle workgroups are merged with global atomicMax into a zeroed output.
#include "pn2_internal.h"

#include <algorithm>
#include <cstring>

namespace pn2 {

typedef float floatx16 __attribute__((ext_vector_type(16)));
typedef float floatx4 __attribute__((ext_vector_type(4)));

constexpr int kWch = 4096;     // floats per staged W chunk (16 KB)
constexpr int kMaxLayers = 4;
constexpr int kMaxSlice = 256; // output columns per pass

struct LayerDev {
    const float *wt;
    const float *alpha;
    const float *beta;
    int cin, cin_pad, cout;
};

struct MlpArgs {
    pn2_sa_src src;
    LayerDev L[kMaxLayers];
    int nlayers;
    int64_t M;        // rows
    int ld;           // LDS activation stride (floats, odd)
    int ycols;        // last-layer columns per grid.y block
    int pool;         // 1: pooled output
    int pool_lds;     // 1: merge groups in LDS first; 0: global atomics straight from registers
    int k32;          // group size is a multiple of 32 (tile-aligned groups)
    int64_t K;        // rows per group (pool)
    float *out;
    int64_t ostride;
};

__device__ __forceinline__ float relu_pos(float t) { return t > 0.f ? t : 0.f; }  // never -0

// ------------------------------------------------------------------ gather of one row element
__device__ __forceinline__ float fetch(const pn2_sa_src &s, int64_t R, int64_t M, int c, int cin) {
    if (R >= M || c >= cin) return 0.f;
    const int C = (int)s.C;
    switch (s.mode) {
    case PN2_SRC_GROUP_XYZ_FIRST:
    case PN2_SRC_GROUP_FEAT_FIRST: {
        const int64_t g = R / s.K;
        const int64_t b = g / s.S;
        const int64_t n = s.idx[R];
        const int xc = (s.mode == PN2_SRC_GROUP_XYZ_FIRST) ? c : c - (int)s.D;
        if (xc >= 0 && xc < C)
            return s.pts[b * s.pb + n * s.pn + (int64_t)xc * s.pc] - s.ctr[g * C + xc];
        const int d = (s.mode == PN2_SRC_GROUP_XYZ_FIRST) ? c - C : c;
        return s.feat[b * s.fb + n * s.fn + d];
    }
    case PN2_SRC_GROUP_ALL: {
        const int64_t b = R / s.N;
        const int64_t n = R - b * s.N;
        if (c < C) return s.pts[b * s.pb + n * s.pn + (int64_t)c * s.pc];
        return s.feat[b * s.fb + n * s.fn + (c - C)];
    }
    default:
        return s.rows[R * s.rs + c];
    }
}

// ------------------------------------------------------------------ W chunk staging
template <int NT>
struct Stage {
    static constexpr int ST = kWch / 4 / NT;  // float4 per thread
    floatx4 r[ST];
    __device__ __forceinline__ void load(const float *wt, int cout, int cb, int cw, int k0, int kc,
                                         int tid) {
        const int c4 = cw >> 2;
        const int tot = kc * c4;
#pragma unroll
        for (int i = 0; i < ST; ++i) {
            // unconditional (clamped) loads keep r[] in registers and the prefetch in flight
            const int e0 = tid + i * NT;
            const int e = e0 < tot ? e0 : 0;
            const int kr = e / c4;
            const int cc = e - kr * c4;
            r[i] = *reinterpret_cast<const floatx4 *>(wt + (int64_t)(k0 + kr) * cout + cb + cc * 4);
        }
    }
    __device__ __forceinline__ void store(float *buf, int cw, int kc, int tid) const {
        const int tot = kc * (cw >> 2);
#pragma unroll
        for (int i = 0; i < ST; ++i) {
            const int e = tid + i * NT;
            if (e < tot) reinterpret_cast<floatx4 *>(buf)[e] = r[i];
        }
    }
};

// ------------------------------------------------------------------ one GEMM pass
// acc[j] (+)= act[rows of row-tile rt][0:cin_pad] x W^T[0:cin_pad][cb + ct_j*32 .. +32]
template <int NT, int NTILE>
__device__ __forceinline__ void gemm_pass(floatx16 (&acc)[NTILE], const float *act, int ld,
                                          float *wbuf, const LayerDev &L, int cb, int cw, int rt,
                                          int ct0, int ctstep, int tid, int lane) {
#pragma unroll
    for (int j = 0; j < NTILE; ++j)
#pragma unroll
        for (int r = 0; r < 16; ++r) acc[j][r] = 0.f;

    const int kcf = (kWch / cw) & ~15;  // k-depth of a staged chunk: multiple of 16 (cw <= 256)
    const int nch = (L.cin_pad + kcf - 1) / kcf;
    const int CT = cw >> 5;
    Stage<NT> st;
    st.load(L.wt, L.cout, cb, cw, 0, min(kcf, L.cin_pad), tid);
    st.store(wbuf, cw, min(kcf, L.cin_pad), tid);
    __syncthreads();

    const float *arow = act + (rt * 32 + (lane & 31)) * ld + (lane >> 5);
    for (int ch = 0; ch < nch; ++ch) {
        const int k0 = ch * kcf;
        const int kc = min(kcf, L.cin_pad - k0);
        float *cur = wbuf + (ch & 1) * kWch;
        float *nxt = wbuf + ((ch + 1) & 1) * kWch;
        const bool more = ch + 1 < nch;
        if (more) st.load(L.wt, L.cout, cb, cw, k0 + kcf, min(kcf, L.cin_pad - k0 - kcf), tid);

        if (ct0 < CT) {
            const float *bcol = cur + (lane >> 5) * cw + (lane & 31);
            const float *ap = arow + k0;
            for (int kk = 0; kk < kc; kk += 8) {
                float a[4], bv[4][NTILE];
#pragma unroll
                for (int u = 0; u < 4; ++u) {
                    a[u] = ap[kk + 2 * u];
#pragma unroll
                    for (int j = 0; j < NTILE; ++j)  // odd CT: the spare tile repeats a valid one
                        bv[u][j] = bcol[(kk + 2 * u) * cw + min(ct0 + j * ctstep, CT - 1) * 32];
                }
#pragma unroll
                for (int u = 0; u < 4; ++u)
#pragma unroll
                    for (int j = 0; j < NTILE; ++j)
                        acc[j] = __builtin_amdgcn_mfma_f32_32x32x2f32(a[u], bv[u][j], acc[j], 0, 0, 0);
            }
        }
        if (more) st.store(nxt, cw, min(kcf, L.cin_pad - k0 - kcf), tid);
        __syncthreads();
    }
}

// ------------------------------------------------------------------ one layer of the chain
// LAST: the layer's output is pooled / stored to HBM; otherwise it overwrites the LDS tile.
template <int BM, int NTILE, bool LAST>
__device__ __forceinline__ void run_layer(const MlpArgs &A, const LayerDev &L, float *act,
                                          float *wbuf, unsigned *pool, int64_t row0, int tid,
                                          int lane, int wave) {
    constexpr int NT = BM * 4;
    constexpr int RT = BM / 32;
    const int rt = wave % RT;
    const int ct0 = wave / RT;  // column half: 0 or 1
    constexpr int ctstep = 2;

    if constexpr (!LAST) {
        floatx16 acc[NTILE];
        gemm_pass<NT, NTILE>(acc, act, A.ld, wbuf, L, 0, L.cout, rt, ct0, ctstep, tid, lane);
        // every wave is past its last read of act for this layer -> overwrite in place
        const int CT = L.cout >> 5;
#pragma unroll
        for (int j = 0; j < NTILE; ++j) {
            const int ct = ct0 + j * ctstep;
            if (ct < CT) {
                const int col = ct * 32 + (lane & 31);
                const float al = L.alpha[col], be = L.beta[col];
#pragma unroll
                for (int r = 0; r < 16; ++r) {
                    const int row = rt * 32 + (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5);
                    act[row * A.ld + col] = relu_pos(__builtin_fmaf(acc[j][r], al, be));
                }
            }
        }
        // the next layer's first staging barrier orders these writes before its reads
    } else {
        const int64_t M = A.M;
        const int64_t K = A.K;
        const int64_t G = A.pool ? M / K : 0;
        const int ybase = blockIdx.y * A.ycols;
        for (int s0 = 0; s0 < A.ycols; s0 += kMaxSlice) {
            const int cw = min(kMaxSlice, A.ycols - s0);
            const int cb = ybase + s0;
            const int CT = cw >> 5;
            const int64_t g0 = A.pool ? row0 / K : 0;
            const int64_t rend = min(row0 + BM, M);
            const int ngl = A.pool ? (int)((rend - 1) / K - g0 + 1) : 0;
            if (A.pool_lds)
                for (int e = tid; e < ngl * cw; e += NT) pool[e] = 0u;

            floatx16 acc[NTILE];
            gemm_pass<NT, NTILE>(acc, act, A.ld, wbuf, L, cb, cw, rt, ct0, ctstep, tid, lane);

            const int64_t rb = row0 + rt * 32;
#pragma unroll
            for (int j = 0; j < NTILE; ++j) {
                const int ct = ct0 + j * ctstep;
                if (ct >= CT || rb >= M) continue;
                const int col = ct * 32 + (lane & 31);
                const float al = L.alpha[cb + col], be = L.beta[cb + col];
                if (!A.pool) {
#pragma unroll
                    for (int r = 0; r < 16; ++r) {
                        const int64_t row = rb + (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5);
                        if (row < M)
                            A.out[row * A.ostride + cb + col] =
                                relu_pos(__builtin_fmaf(acc[j][r], al, be));
                    }
                } else if (A.k32) {
                    // all 32 rows of the tile belong to one group: reduce in registers
                    float m = relu_pos(__builtin_fmaf(acc[j][0], al, be));
#pragma unroll
                    for (int r = 1; r < 16; ++r) m = fmaxf(m, relu_pos(__builtin_fmaf(acc[j][r], al, be)));
                    m = fmaxf(m, __shfl_xor(m, 32));
                    const int64_t g = rb / K;
                    if (lane < 32) {
                        if (A.pool_lds) atomicMax(&pool[(g - g0) * cw + col], __float_as_uint(m));
                        else atomicMax(reinterpret_cast<unsigned *>(A.out + g * A.ostride + cb + col),
                                       __float_as_uint(m));
                    }
                } else {
#pragma unroll
                    for (int r = 0; r < 16; ++r) {
                        const int64_t row = rb + (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5);
                        if (row < M) {
                            const unsigned u = __float_as_uint(relu_pos(__builtin_fmaf(acc[j][r], al, be)));
                            const int64_t g = row / K;
                            if (A.pool_lds) atomicMax(&pool[(g - g0) * cw + col], u);
                            else atomicMax(reinterpret_cast<unsigned *>(A.out + g * A.ostride + cb + col), u);
                        }
                    }
                }
            }
            if (A.pool_lds) {
                __syncthreads();
                for (int e = tid; e < ngl * cw; e += NT) {
                    const int gl = e / cw;
                    const int c = e - gl * cw;
                    const int64_t g = g0 + gl;
                    if (g >= G) continue;
                    const unsigned val = pool[e];
                    float *dst = A.out + g * A.ostride + cb + c;
                    if (g * K >= row0 && (g + 1) * K <= row0 + BM) *dst = __uint_as_float(val);
                    else atomicMax(reinterpret_cast<unsigned *>(dst), val);
                }
                __syncthreads();  // the pool is reused by the next slice
            }
        }
    }
}

// ------------------------------------------------------------------ the kernel
// T0..T3: 32x32 column tiles per wave for each layer (0 = no such layer).  The chain is
// straight-line code, so every layer's parameters are static kernel-argument loads.
template <int BM, int T0, int T1, int T2, int T3>
__global__ __launch_bounds__(BM * 4) void sa_mlp_kernel(const MlpArgs A) {
    constexpr int NW = BM / 16;
    extern __shared__ __attribute__((aligned(16))) float smem[];
    float *act = smem;
    float *wbuf = smem + ((BM * A.ld + 3) & ~3);
    unsigned *pool = reinterpret_cast<unsigned *>(wbuf + 2 * kWch);

    const int tid = threadIdx.x;
    const int lane = tid & 63;
    const int wave = tid >> 6;
    const int64_t row0 = (int64_t)blockIdx.x * BM;

    // ---- gather the BM input rows into act[BM][ld]; G lanes per row, rows spread over waves
    {
        const int cinp = A.L[0].cin_pad;
        const int cin = A.L[0].cin;
        const int G = cinp <= 8 ? 8 : cinp <= 16 ? 16 : cinp <= 32 ? 32 : 64;
        const int rpw = 64 / G;
        const int sub = lane / G, cl = lane % G;
        for (int r0 = wave * rpw; r0 < BM; r0 += NW * rpw) {
            const int r = r0 + sub;
            const int64_t R = row0 + r;
            for (int c = cl; c < cinp; c += G) act[r * A.ld + c] = fetch(A.src, R, A.M, c, cin);
        }
    }
    // (the first barrier is inside the first gemm_pass, after its W chunk is staged)
    run_layer<BM, T0, T1 == 0>(A, A.L[0], act, wbuf, pool, row0, tid, lane, wave);
    if constexpr (T1 != 0) run_layer<BM, T1, T2 == 0>(A, A.L[1], act, wbuf, pool, row0, tid, lane, wave);
    if constexpr (T2 != 0) run_layer<BM, T2, T3 == 0>(A, A.L[2], act, wbuf, pool, row0, tid, lane, wave);
    if constexpr (T3 != 0) run_layer<BM, T3, true>(A, A.L[3], act, wbuf, pool, row0, tid, lane, wave);
}

// Layer-tile signatures compiled as fused chains (covers every head of the reference:
// SSG [64,64,128] [128,128,256], MSG [32,32,64] [64,64,128] [64,96,128] [32,64,128]
// [64,128,256] [96,128,256], group_all [256,512|...]); other chains run layer by layer.
#define PN2_MLP_SIGS(X)                                                                    \
    X(1, 0, 0, 0) X(2, 0, 0, 0) X(3, 0, 0, 0) X(4, 0, 0, 0) X(4, 4, 0, 0) X(2, 4, 0, 0)   \
    X(1, 1, 1, 0) X(1, 1, 2, 0) X(1, 2, 2, 0) X(2, 2, 4, 0) X(1, 2, 4, 0) X(2, 2, 2, 0)
// 32-row tiles (very wide inputs, e.g. a 512-channel layer) exist for single layers only
#define PN2_MLP_SIGS32(X) X(1, 0, 0, 0) X(2, 0, 0, 0) X(3, 0, 0, 0) X(4, 0, 0, 0)

// ------------------------------------------------------------------ BN/conv packing
__global__ __launch_bounds__(256) void pack_layer_kernel(
    const float *__restrict__ W, const float *__restrict__ bias, const float *__restrict__ gamma,
    const float *__restrict__ beta, const float *__restrict__ mean, const float *__restrict__ var,
    float eps, int cout, int cin, int cin_pad, float *__restrict__ wt, float *__restrict__ alpha,
    float *__restrict__ beta_out) {
    const int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (e < (int64_t)cin_pad * cout) {
        const int k = (int)(e / cout), o = (int)(e - (int64_t)k * cout);
        wt[e] = k < cin ? W[(int64_t)o * cin + k] : 0.f;
    }
    if (e < cout) {
        const int o = (int)e;
        // ATen eval BN: invstd = 1/sqrt(var+eps); alpha = invstd*gamma; beta' = beta - mean*alpha
        const float inv = var ? 1.0f / sqrtf(var[o] + eps) : 1.0f;
        const float a = gamma ? inv * gamma[o] : inv;
        const float sh = (beta ? beta[o] : 0.f) - (mean ? mean[o] * a : 0.f);
        alpha[o] = a;
        beta_out[o] = __builtin_fmaf(bias ? bias[o] : 0.f, a, sh);
    }
}

}  // namespace pn2

using namespace pn2;

extern "C" int64_t pn2_layer_cin_pad(int64_t cin) { return ((cin + 7) / 8) * 8; }

extern "C" int pn2_pack_layer_f32(const float *W, const float *bias, const float *gamma,
                                  const float *beta, const float *mean, const float *var,
                                  double eps, int64_t cout, int64_t cin, float *wt, float *alpha,
                                  float *beta_out, void *stream) {
    PN2_REQUIRE(W && wt && alpha && beta_out, "pn2_pack_layer_f32: null pointer");
    PN2_REQUIRE(cout >= 1 && cin >= 1, "pn2_pack_layer_f32: bad shape");
    const int64_t cinp = pn2_layer_cin_pad(cin);
    const int64_t tot = std::max(cinp * cout, cout);
    hipLaunchKernelGGL(pack_layer_kernel, dim3((unsigned)((tot + 255) / 256)), dim3(256), 0,
                       as_stream(stream), W, bias, gamma, beta, mean, var, (float)eps, (int)cout,
                       (int)cin, (int)cinp, wt, alpha, beta_out);
    PN2_LAUNCH_CHECK("pack_layer_kernel");
    return PN2_OK;
}

// ------------------------------------------------------------------ host side
struct Plan {
    MlpArgs A;
    int BM;
    int64_t tiles;
    int ysplit;
    size_t lds;
    int T[kMaxLayers];
};

static size_t lds_bytes(int BM, int ld, int cw, int groups) {
    return (size_t)(((BM * ld + 3) & ~3) + 2 * kWch) * 4 + (size_t)groups * cw * 4;
}

// Plan one fused launch of layers[0..n) reading `s` (rows M, group size K).
static int make_plan(Plan &P, const pn2_sa_src &s, const pn2_mlp_layer *layers, int n, int pool,
                     float *out, int64_t ostride, int64_t M, int64_t K) {
    MlpArgs &A = P.A;
    memset(&A, 0, sizeof(A));
    A.src = s;
    A.nlayers = n;
    A.M = M;
    A.K = pool ? K : 1;
    A.k32 = (pool && K % 32 == 0) ? 1 : 0;
    int maxw = 0;
    for (int l = 0; l < n; ++l) {
        const pn2_mlp_layer &q = layers[l];
        A.L[l].wt = q.wt; A.L[l].alpha = q.alpha; A.L[l].beta = q.beta;
        A.L[l].cin = (int)q.cin; A.L[l].cin_pad = (int)pn2_layer_cin_pad(q.cin);
        A.L[l].cout = (int)q.cout;
        if (l == 0) maxw = A.L[0].cin_pad;
        if (l < n - 1) maxw = std::max(maxw, (int)q.cout);
    }
    A.ld = maxw | 1;
    A.pool = pool ? 1 : 0;
    A.out = out;
    A.ostride = ostride;
    const int64_t coutL = layers[n - 1].cout;
    // rows per workgroup: 128 when the activation tile leaves room for 2 workgroups' worth of
    // other state, else 64, else 32 (single-layer launches only)
    P.BM = 128;
    if (lds_bytes(128, A.ld, 0, 0) > 112 * 1024) P.BM = 64;
    if (lds_bytes(64, A.ld, 0, 0) > 144 * 1024) P.BM = 32;
    P.tiles = (M + P.BM - 1) / P.BM;
    // a single-layer launch can also split its columns over grid.y (nothing is recomputed)
    P.ysplit = 1;
    if (n == 1)
        while (P.tiles * P.ysplit < 1024 && coutL / (P.ysplit * 2) >= 64 &&
               (coutL / (P.ysplit * 2)) % 32 == 0)
            P.ysplit *= 2;
    A.ycols = (int)(coutL / P.ysplit);
    const int cwmax = std::min(A.ycols, kMaxSlice);
    int groups = 0;
    if (pool) {
        groups = (int)(P.BM / K + 2);
        A.pool_lds = (size_t)groups * cwmax * 4 <= 32 * 1024 ? 1 : 0;
    }
    P.lds = lds_bytes(P.BM, A.ld, cwmax, A.pool_lds ? groups : 0);
    for (int l = 0; l < kMaxLayers; ++l) P.T[l] = 0;
    for (int l = 0; l < n; ++l) {
        const int cw = (l == n - 1) ? cwmax : (int)layers[l].cout;
        P.T[l] = ((cw >> 5) + 1) >> 1;
    }
    if (P.lds > 160 * 1024)
        return set_error(PN2_EUNSUPPORTED, "pn2_sa_mlp_max_f32: LDS %zu > 160 KiB (ld=%d)", P.lds, A.ld);
    if (P.BM == 32 && n > 1)
        return set_error(PN2_EUNSUPPORTED, "pn2_sa_mlp_max_f32: 32-row tiles are single-layer only");
    return PN2_OK;
}

template <int BM, int T0, int T1, int T2, int T3>
static int launch_sig(const Plan &P, hipStream_t st) {
    // one-time, idempotent kernel attribute (C++11 thread-safe static init)
    static const hipError_t attr = hipFuncSetAttribute(
        reinterpret_cast<const void *>(&sa_mlp_kernel<BM, T0, T1, T2, T3>),
        hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    (void)attr;
    hipLaunchKernelGGL((sa_mlp_kernel<BM, T0, T1, T2, T3>), dim3((unsigned)P.tiles, (unsigned)P.ysplit),
                       dim3(BM * 4), P.lds, st, P.A);
    PN2_LAUNCH_CHECK("sa_mlp_kernel");
    return PN2_OK;
}

// returns 1 when launched, 0 when the signature is not compiled, <0 on error
static int try_launch(const Plan &P, hipStream_t st) {
    if (P.A.pool && (P.BM % P.A.K != 0 || !P.A.pool_lds)) {
        // groups straddle workgroups (or bypass LDS): merged with atomicMax into a zeroed output
        const int64_t coutL = (int64_t)P.A.ycols * P.ysplit;
        const int64_t G = P.A.M / P.A.K;
        hipError_t e = (P.A.ostride == coutL)
                           ? hipMemsetAsync(P.A.out, 0, (size_t)G * coutL * 4, st)
                           : hipMemset2DAsync(P.A.out, (size_t)P.A.ostride * 4, 0, (size_t)coutL * 4,
                                              (size_t)G, st);
        if (e != hipSuccess)
            return set_error(PN2_EHIP, "pn2_sa_mlp_max_f32: memset: %s", hipGetErrorString(e));
    }
#define PN2_TRY(t0, t1, t2, t3)                                                          \
    if (P.BM != 32 && P.T[0] == t0 && P.T[1] == t1 && P.T[2] == t2 && P.T[3] == t3) {  \
        const int rc = P.BM == 128 ? launch_sig<128, t0, t1, t2, t3>(P, st)              \
                                   : launch_sig<64, t0, t1, t2, t3>(P, st);              \
        return rc == PN2_OK ? 1 : rc;                                                    \
    }
    PN2_MLP_SIGS(PN2_TRY)
#undef PN2_TRY
#define PN2_TRY32(t0, t1, t2, t3)                                                        \
    if (P.BM == 32 && P.T[0] == t0 && P.T[1] == t1 && P.T[2] == t2 && P.T[3] == t3) {  \
        const int rc = launch_sig<32, t0, t1, t2, t3>(P, st);                            \
        return rc == PN2_OK ? 1 : rc;                                                    \
    }
    PN2_MLP_SIGS32(PN2_TRY32)
#undef PN2_TRY32
    return 0;
}

static int validate(const pn2_sa_src *src, const pn2_mlp_layer *layers, int nlayers,
                    int64_t &M, int64_t &K) {
    PN2_REQUIRE(src && layers, "pn2_sa_mlp_max_f32: null pointer");
    PN2_REQUIRE(nlayers >= 1 && nlayers <= kMaxLayers, "pn2_sa_mlp_max_f32: nlayers=%d", nlayers);
    const pn2_sa_src &s = *src;
    int64_t cin0 = 0;
    switch (s.mode) {
    case PN2_SRC_GROUP_XYZ_FIRST:
    case PN2_SRC_GROUP_FEAT_FIRST:
        PN2_REQUIRE(s.pts && s.ctr && s.idx && (s.D == 0 || s.feat), "pn2_sa_mlp_max_f32: group source");
        PN2_REQUIRE(s.B >= 0 && s.N >= 1 && s.S >= 1 && s.K >= 1 && s.C >= 1 && s.D >= 0,
                    "pn2_sa_mlp_max_f32: bad group shape");
        M = s.B * s.S * s.K; cin0 = s.C + s.D; K = s.K;
        break;
    case PN2_SRC_GROUP_ALL:
        PN2_REQUIRE(s.pts && (s.D == 0 || s.feat), "pn2_sa_mlp_max_f32: group_all source");
        PN2_REQUIRE(s.B >= 0 && s.N >= 1 && s.C >= 1 && s.D >= 0, "pn2_sa_mlp_max_f32: bad group_all shape");
        M = s.B * s.N; cin0 = s.C + s.D; K = s.N;
        break;
    case PN2_SRC_ROWS:
        PN2_REQUIRE(s.rows && s.rs >= layers[0].cin, "pn2_sa_mlp_max_f32: rows source");
        PN2_REQUIRE(s.B >= 0 && s.S >= 1 && s.K >= 1, "pn2_sa_mlp_max_f32: bad rows shape");
        M = s.B * s.S * s.K; cin0 = layers[0].cin; K = s.K;
        break;
    default:
        return set_error(PN2_EINVAL, "pn2_sa_mlp_max_f32: mode %d", s.mode);
    }
    PN2_REQUIRE(layers[0].cin == cin0, "pn2_sa_mlp_max_f32: layer0 cin %lld != source width %lld",
                (long long)layers[0].cin, (long long)cin0);
    for (int l = 0; l < nlayers; ++l) {
        const pn2_mlp_layer &q = layers[l];
        PN2_REQUIRE(q.wt && q.alpha && q.beta, "pn2_sa_mlp_max_f32: layer %d null", l);
        PN2_REQUIRE(q.cout % 32 == 0 && q.cout >= 32,
                    "pn2_sa_mlp_max_f32: layer %d cout=%lld not a multiple of 32", l, (long long)q.cout);
        if (l > 0)
            PN2_REQUIRE(q.cin == layers[l - 1].cout, "pn2_sa_mlp_max_f32: layer %d cin mismatch", l);
    }
    return PN2_OK;
}

// A chain runs as consecutive fused segments; a segment ends after a layer wider than one
// column slice (its output cannot stay in LDS) or at the end of the chain.  Segment outputs
// go to two ping-pong [M][w] workspace buffers.  A segment with no compiled signature (or too
// wide for LDS) runs layer by layer through the same workspace.
static int seg_end(const pn2_mlp_layer *layers, int nlayers, int l0) {
    int l = l0;
    while (l < nlayers - 1 && layers[l].cout <= kMaxSlice) ++l;
    return l;  // inclusive
}

static bool segment_fused(const pn2_sa_src &s, const pn2_mlp_layer *layers, int l0, int l1,
                          int64_t M, int64_t K, int pool) {
    Plan P;
    if (make_plan(P, s, layers + l0, l1 - l0 + 1, pool, nullptr, layers[l1].cout, M, K) != PN2_OK)
        return false;
    bool found = false;
#define PN2_HAS(t0, t1, t2, t3) \
    if (P.BM != 32 && P.T[0] == t0 && P.T[1] == t1 && P.T[2] == t2 && P.T[3] == t3) found = true;
    PN2_MLP_SIGS(PN2_HAS)
#undef PN2_HAS
#define PN2_HAS32(t0, t1, t2, t3) \
    if (P.BM == 32 && P.T[0] == t0 && P.T[1] == t1 && P.T[2] == t2 && P.T[3] == t3) found = true;
    PN2_MLP_SIGS32(PN2_HAS32)
#undef PN2_HAS32
    return found;
}

static pn2_sa_src rows_src(const float *rows, int64_t w, int64_t M, int64_t K) {
    pn2_sa_src nx;
    memset(&nx, 0, sizeof(nx));
    nx.mode = PN2_SRC_ROWS;
    nx.rows = rows;
    nx.rs = w;
    nx.B = 1; nx.S = M / K; nx.K = K;
    return nx;
}

// workspace width needed: the widest layer output that has to round-trip through HBM
static int64_t workspace_width(const pn2_sa_src &s, const pn2_mlp_layer *layers, int nlayers,
                               int64_t M, int64_t K) {
    int64_t w = 0;
    for (int l0 = 0; l0 < nlayers;) {
        const int l1 = seg_end(layers, nlayers, l0);
        const bool last_seg = l1 == nlayers - 1;
        pn2_sa_src src = l0 == 0 ? s : rows_src(nullptr, 0, M, K);
        if (l0 > 0) src.rows = reinterpret_cast<const float *>(16);
        if (!segment_fused(src, layers, l0, l1, M, K, last_seg ? 1 : 0))
            for (int l = l0; l < l1; ++l) w = std::max(w, layers[l].cout);
        if (!last_seg) w = std::max(w, layers[l1].cout);
        l0 = l1 + 1;
    }
    return w;
}

extern "C" int64_t pn2_sa_mlp_workspace_bytes(const pn2_sa_src *src, const pn2_mlp_layer *layers,
                                              int nlayers) {
    int64_t M = 0, K = 1;
    if (validate(src, layers, nlayers, M, K) != PN2_OK) return -1;
    return 2 * M * workspace_width(*src, layers, nlayers, M, K) * 4;
}

static int run_single(const pn2_sa_src &cur, const pn2_mlp_layer *layers, int l0, int l1,
                      int pool, float *dst, int64_t ostride, int64_t M, int64_t K, hipStream_t st) {
    Plan P;
    int rc = make_plan(P, cur, layers + l0, l1 - l0 + 1, pool, dst, ostride, M, K);
    if (rc != PN2_OK) return rc;
    rc = try_launch(P, st);
    if (rc < 0) return rc;
    if (rc == 0) return set_error(PN2_EUNSUPPORTED, "pn2_sa_mlp_max_f32: no kernel for layers %d..%d", l0, l1);
    return PN2_OK;
}

extern "C" int pn2_sa_mlp_max_f32(const pn2_sa_src *src, const pn2_mlp_layer *layers,
                                  int nlayers, int pool, float *out, int64_t ostride,
                                  float *workspace, int64_t workspace_bytes, void *stream) {
    int64_t M = 0, K = 1;
    int rc = validate(src, layers, nlayers, M, K);
    if (rc != PN2_OK) return rc;
    PN2_REQUIRE(out, "pn2_sa_mlp_max_f32: null out");
    PN2_REQUIRE(ostride >= layers[nlayers - 1].cout, "pn2_sa_mlp_max_f32: ostride");
    if (M == 0) return PN2_OK;
    if (pool) PN2_REQUIRE(M % K == 0, "pn2_sa_mlp_max_f32: rows not a multiple of the group size");
    hipStream_t st = as_stream(stream);
    const int64_t w = workspace_width(*src, layers, nlayers, M, K);
    if (w > 0)
        PN2_REQUIRE(workspace && workspace_bytes >= 2 * M * w * 4,
                    "pn2_sa_mlp_max_f32: this layer chain needs a %lld-byte workspace",
                    (long long)(2 * M * w * 4));
    pn2_sa_src cur = *src;
    int buf = 0;
    for (int l0 = 0; l0 < nlayers;) {
        const int l1 = seg_end(layers, nlayers, l0);
        const bool last_seg = l1 == nlayers - 1;
        if (segment_fused(cur, layers, l0, l1, M, K, last_seg ? pool : 0)) {
            float *dst = last_seg ? out : workspace + buf * M * w;
            rc = run_single(cur, layers, l0, l1, last_seg ? pool : 0, dst, last_seg ? ostride : w,
                            M, K, st);
            if (rc != PN2_OK) return rc;
            if (!last_seg) { cur = rows_src(dst, w, M, K); buf ^= 1; }
        } else {
            for (int l = l0; l <= l1; ++l) {
                const bool last = l == nlayers - 1;
                float *dst = last ? out : workspace + buf * M * w;
                rc = run_single(cur, layers, l, l, last ? pool : 0, dst, last ? ostride : w, M, K, st);
                if (rc != PN2_OK) return rc;
                if (!last) { cur = rows_src(dst, w, M, K); buf ^= 1; }
            }
        }
        l0 = l1 + 1;
    }
    return PN2_OK;
}
