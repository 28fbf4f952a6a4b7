// sa_mlp.hip -- fused set-abstraction MLP for gfx950: gather -> (1x1 conv + BN + ReLU)* -> max.
//
// Replaces, for eval-mode inference, the SA feature path of
//   PointNetSetAbstraction.forward     /root/reference/model/pointnet2_utils.py:158-174
//   PointNetSetAbstractionMsg.forward  /root/reference/model/pointnet2_utils.py:195-223
// i.e. index_points of the neighbourhoods (:109-116, :205-209; :137-139 for group_all), the
// permute to [B,C,K,S] (:167, :211), the Conv2d-1x1 / BatchNorm2d / ReLU stack (:168-170,
// :213-216) and torch.max over the neighbourhood axis (:172, :218).
//
// Rows are (group, neighbour) pairs, M = B*S*K.  A workgroup (8 waves) owns BM consecutive rows
// and runs the whole layer chain on them ("fused" kernel):
//   gather   row indices are resolved first (one LDS table), then every lane issues all of its
//            16-byte feature loads before writing any, so a tile costs ~2 dependent memory
//            round trips; features are channels-last so each row is one contiguous run.
//            LDS row layout is [feature | xyz | 0-pad]; the packed weights are rotated to match.
//   layer    acc(32x32 tiles) += A x W^T with v_mfma_f32_32x32x2_f32 (exact fp32 products,
//            fma-chain accumulation).  A (activations) comes from LDS by ds_read_b64 -- row
//            stride ld = 2 (mod 4), conflict-free -- and feeds two MFMAs; B (weights) comes
//            straight from L2 into registers (pair-interleaved [k/2][cout][2] packing: one 8-byte
//            load per lane per 2 MFMAs), prefetched one 8-deep k block ahead.  No weight staging,
//            no per-chunk barrier: two barriers per layer.  Epilogue: folded BN scale/shift +
//            ReLU, written back into the LDS tile (hidden activations never touch HBM).
//   pool     the last layer's wave owns whole neighbourhoods (contiguous row blocks), so the max
//            over K rows is a register reduction + one cross-half exchange and one coalesced
//            store per group; other shapes merge through LDS (ds_max_u32 on the float bits --
//            ReLU output is >= +0, so uint order == float order), and groups straddling
//            workgroups through global atomicMax into a zeroed output.
// Single layers too wide for an LDS-resident tile (e.g. 512 -> 1024 of group_all) use the
// "dense" kernel: the same wave tiling with A streamed through LDS in 32-deep k chunks.
#include "pn2_internal.h"

#include <algorithm>
#include <cstring>

namespace pn2 {

typedef float floatx16 __attribute__((ext_vector_type(16)));
typedef float floatx4 __attribute__((ext_vector_type(4)));
typedef float floatx2 __attribute__((ext_vector_type(2)));

constexpr int kMaxLayers = 4;
constexpr int kNW = 8;           // waves per workgroup
constexpr int kNT = kNW * 64;    // threads per workgroup
constexpr int kMaxSlice = 256;   // output columns per pass (8 col tiles x 32)

struct LayerDev {
    const float *wt;    // pair-interleaved W^T: [cin_pad/2][cout][2]
    const float *alpha;
    const float *beta;
    int cin, cin_pad, cout;
};

struct MlpArgs {
    pn2_sa_src src;
    LayerDev L[kMaxLayers];
    int nlayers;
    int64_t M;        // rows
    int ld;           // LDS activation stride (floats), = 2 (mod 4)
    int ycols;        // last-layer columns per grid.y block
    int pool;         // 1: pooled output
    int pool_mode;    // 0: registers, 1: LDS ds_max, 2: global atomics
    int64_t K;        // rows per group (pool)
    int vec_feat;     // feature rows are 16-byte aligned with D % 4 == 0
    float *out;
    int64_t ostride;
};

__device__ __forceinline__ float relu_pos(float t) { return t > 0.f ? t : 0.f; }  // never -0

// ------------------------------------------------------------------ gather
// act[r][0:D] = features of row r's point, act[r][D:D+C] = xyz (- centroid), 0-pad to cin_pad.
// ROWS source: act[r][0:cin] = rows[R][0:cin].
__device__ __forceinline__ void gather_rows(const MlpArgs &A, float *act, int *rn, int *rb,
                                            int64_t row0, int BM, int tid) {
    const pn2_sa_src &s = A.src;
    const int cinp = A.L[0].cin_pad;
    const int ld = A.ld;
    const unsigned M = (unsigned)A.M;
    // 1. row -> (point n, batch b)   (32-bit index math: M < 2^31 is checked on the host)
    for (int r = tid; r < BM; r += kNT) {
        const unsigned R = (unsigned)row0 + r;
        int n = -1, b = 0;
        if (R < M) {
            if (s.mode == PN2_SRC_GROUP_XYZ_FIRST || s.mode == PN2_SRC_GROUP_FEAT_FIRST) {
                const unsigned g = R / (unsigned)s.K;
                b = (int)(g / (unsigned)s.S);
                n = src_index(s, R);
                if ((unsigned)n >= (unsigned)s.N) n = 0;  // no-neighbour pad (PN2_DEVERR_NO_NEIGHBOUR)
            } else if (s.mode == PN2_SRC_GROUP_ALL) {
                b = (int)(R / (unsigned)s.N);
                n = (int)(R - (unsigned)b * (unsigned)s.N);
            } else {
                n = 0;
            }
        }
        rn[r] = n;
        rb[r] = b;
    }
    __syncthreads();
    const int D = (s.mode == PN2_SRC_ROWS) ? A.L[0].cin : (int)s.D;
    // 2. feature (or dense row) part: 16-byte loads all issued before the LDS writes
    if (A.vec_feat && D > 0) {
        const int D4 = D >> 2;
        const int tot = BM * D4;
        constexpr int U = 8;
        for (int e0 = tid; e0 < tot; e0 += U * kNT) {
            floatx4 v[U];
#pragma unroll
            for (int u = 0; u < U; ++u) {
                const int e = e0 + u * kNT;
                const int r = e / D4, q = e - r * D4;
                v[u] = floatx4{0.f, 0.f, 0.f, 0.f};
                if (e < tot && rn[r] >= 0) {
                    const float *src = (s.mode == PN2_SRC_ROWS)
                                           ? s.rows + (row0 + r) * s.rs
                                           : s.feat + (int64_t)rb[r] * s.fb + (int64_t)rn[r] * s.fn;
                    v[u] = *reinterpret_cast<const floatx4 *>(src + 4 * q);
                }
            }
#pragma unroll
            for (int u = 0; u < U; ++u) {
                const int e = e0 + u * kNT;
                if (e < tot) {
                    const int r = e / D4, q = e - r * D4;
                    floatx2 *dst = reinterpret_cast<floatx2 *>(act + r * ld + 4 * q);
                    dst[0] = floatx2{v[u][0], v[u][1]};
                    dst[1] = floatx2{v[u][2], v[u][3]};
                }
            }
        }
    } else if (D > 0) {
        const int tot = BM * D;
        for (int e = tid; e < tot; e += kNT) {
            const int r = e / D, c = e - r * D;
            float v = 0.f;
            if (rn[r] >= 0)
                v = (s.mode == PN2_SRC_ROWS) ? s.rows[(row0 + r) * s.rs + c]
                                             : s.feat[(int64_t)rb[r] * s.fb + (int64_t)rn[r] * s.fn + c];
            act[r * ld + c] = v;
        }
    }
    // 3. xyz part (centred for grouping modes) and zero padding
    const int C = (s.mode == PN2_SRC_ROWS) ? 0 : (int)s.C;
    const int tail = cinp - D;  // xyz + pad columns
    const bool centre = s.mode == PN2_SRC_GROUP_XYZ_FIRST || s.mode == PN2_SRC_GROUP_FEAT_FIRST;
    for (int e = tid; e < BM * tail; e += kNT) {
        const int r = e / tail, c = e - r * tail;
        float v = 0.f;
        if (c < C && rn[r] >= 0) {
            const float p = s.pts[(int64_t)rb[r] * s.pb + (int64_t)rn[r] * s.pn + (int64_t)c * s.pc];
            v = centre ? __fsub_rn(p, s.ctr[(int64_t)(((unsigned)row0 + r) / (unsigned)s.K) * C + c]) : p;
        }
        act[r * ld + D + c] = v;
    }
}

// ------------------------------------------------------------------ tile geometry
// Per layer: NTR row tiles (contiguous block) x NTC column tiles per wave.
//   NWr = (BM/32)/NTR wave rows, NWc = 8/NWr wave columns; col tile i of wave = wc + i*NWc.
template <int BM, int NTR, int NTC>
struct Geo {
    static constexpr int RT = BM / 32;
    static constexpr int NWr = RT / NTR;
    static constexpr int NWc = kNW / NWr;
    static_assert(NWr >= 1 && NWr * NTR == RT && NWc * NWr == kNW, "bad tile geometry");
};

// acc[i][j] += A[32 rows of tile j][blocks 0..nblk) x B[..][col tile i], 8-deep k blocks.
// ap[j]: lane's A row at k = 0 of the range (+2h); bp[i]: lane's B pair column at pair 0.
// B is prefetched one block ahead into ping-pong register buffers (no register copies).
template <int NTR, int NTC>
__device__ __forceinline__ void mma_blocks(floatx16 (&acc)[NTC][NTR], const float *const (&ap)[NTR],
                                           const floatx2 *const (&bp)[NTC], int pstride, int nblk) {
    floatx2 b0[2][NTC], b1[2][NTC];
    auto loadb = [&](floatx2 (&bb)[2][NTC], int kb) {
#pragma unroll
        for (int i = 0; i < NTC; ++i) {
            bb[0][i] = bp[i][(2 * kb) * pstride];
            bb[1][i] = bp[i][(2 * kb + 1) * pstride];
        }
    };
    auto block = [&](const floatx2 (&bb)[2][NTC], int kb) {
#pragma unroll
        for (int p = 0; p < 2; ++p) {
            floatx2 a[NTR];
#pragma unroll
            for (int j = 0; j < NTR; ++j) a[j] = *reinterpret_cast<const floatx2 *>(ap[j] + kb * 8 + p * 4);
#pragma unroll
            for (int j = 0; j < NTR; ++j)
#pragma unroll
                for (int i = 0; i < NTC; ++i) {
                    acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(a[j][0], bb[p][i][0], acc[i][j], 0, 0, 0);
                    acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(a[j][1], bb[p][i][1], acc[i][j], 0, 0, 0);
                }
        }
    };
    loadb(b0, 0);
    for (int kb = 0; kb < nblk; kb += 2) {
        const bool has1 = kb + 1 < nblk;
        if (has1) loadb(b1, kb + 1);
        block(b0, kb);
        if (has1) {
            if (kb + 2 < nblk) loadb(b0, kb + 2);
            block(b1, kb + 1);
        }
    }
}

template <int NTR, int NTC>
__device__ __forceinline__ void zero_acc(floatx16 (&acc)[NTC][NTR]) {
#pragma unroll
    for (int i = 0; i < NTC; ++i)
#pragma unroll
        for (int j = 0; j < NTR; ++j)
#pragma unroll
            for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;
}

// lane's B pointers: element (k, n) of the pair-packed W^T at ((k>>1)*cout + n)*2 + (k&1); pair
// p (k = 4p..4p+3) of lane half h is kp = 2p + h.  Invalid (odd-CT) tiles read tile CT-1.
template <int NTC>
__device__ __forceinline__ void b_ptrs(const floatx2 *(&bp)[NTC], const LayerDev &L, int cb,
                                       const int (&ct)[NTC], int CT, int lane) {
#pragma unroll
    for (int i = 0; i < NTC; ++i)
        bp[i] = reinterpret_cast<const floatx2 *>(L.wt) + (int64_t)(lane >> 5) * L.cout + cb +
                min(ct[i], CT - 1) * 32 + (lane & 31);
}

// acc[i][j] = act[row tile rt0+j][0:cin_pad] x W^T[0:cin_pad][col tile ct_i]
template <int NTR, int NTC>
__device__ __forceinline__ void mma_layer(floatx16 (&acc)[NTC][NTR], const float *act, int ld,
                                          const LayerDev &L, int cb, const int (&ct)[NTC], int CT,
                                          int rt0, int lane) {
    zero_acc<NTR, NTC>(acc);
    const floatx2 *bp[NTC];
    b_ptrs<NTC>(bp, L, cb, ct, CT, lane);
    const float *ap[NTR];
#pragma unroll
    for (int j = 0; j < NTR; ++j) ap[j] = act + ((rt0 + j) * 32 + (lane & 31)) * ld + 2 * (lane >> 5);
    mma_blocks<NTR, NTC>(acc, ap, bp, 2 * L.cout, L.cin_pad >> 3);
}

// Pool / store the last layer's tiles.  Rows of tile j: rbase + 32*j + (r&3) + 8*(r>>2) + 4*h.
// relu(alpha*acc+beta) is applied per element (alpha may be negative, so it does not commute
// with the max) on the fly, without a second register copy of the tile.
template <int NTR, int NTC, bool LDS_POOL>
__device__ __forceinline__ void last_epilogue(const MlpArgs &A, const floatx16 (&acc)[NTC][NTR],
                                              const LayerDev &L, int cb, const int (&ct)[NTC], int CT,
                                              int rbase, unsigned *pool, int g0, int cw,
                                              int lane) {
    const int h = lane >> 5;
    const int x = lane & 31;
    const unsigned M = (unsigned)A.M, K = (unsigned)A.K;
    const unsigned G = A.pool ? M / K : 0u;
#pragma unroll
    for (int i = 0; i < NTC; ++i) {
        if (ct[i] >= CT) continue;
        const int col = ct[i] * 32 + x;
        const float al = L.alpha[cb + col], be = L.beta[cb + col];
        if (!A.pool) {
#pragma unroll
            for (int j = 0; j < NTR; ++j) {
                float *o = A.out + (int64_t)(rbase + 32 * j + 4 * h) * A.ostride + cb + col;
                const int rem = (int)M - (rbase + 32 * j + 4 * h);
#pragma unroll
                for (int r = 0; r < 16; ++r) {
                    const int dr = (r & 3) + 8 * (r >> 2);
                    if (dr < rem) o[(int64_t)dr * A.ostride] = relu_pos(__builtin_fmaf(acc[i][j][r], al, be));
                }
            }
        } else if (K % 32 == 0) {
            // every 32-row tile lies in one group: reduce the tile in registers first
            const int tpg = (int)(K >> 5);
            float m = 0.f;
#pragma unroll
            for (int j = 0; j < NTR; ++j) {
                if ((unsigned)(rbase + 32 * j) >= M) break;
                float t = 0.f;
#pragma unroll
                for (int r = 0; r < 16; ++r) t = fmaxf(t, relu_pos(__builtin_fmaf(acc[i][j][r], al, be)));
                t = fmaxf(t, __shfl_xor(t, 32));
                const unsigned g = (unsigned)(rbase + 32 * j) / K;
                if (A.pool_mode == 0) {  // whole group inside this wave's row block
                    m = fmaxf(m, t);
                    if ((j + 1) % tpg == 0) {
                        if (h == 0 && g < G) A.out[(int64_t)g * A.ostride + cb + col] = m;
                        m = 0.f;
                    }
                } else if (h == 0) {
                    if (LDS_POOL && A.pool_mode == 1) atomicMax(&pool[((int)g - g0) * cw + col], __float_as_uint(t));
                    else atomicMax(reinterpret_cast<unsigned *>(A.out + (int64_t)g * A.ostride + cb + col), __float_as_uint(t));
                }
            }
        } else if (A.pool_mode == 0) {
            // K in {8, 16}: 32/K groups in every tile, 16/(32/K) consecutive registers each
            const int rpg = 16 / (int)(32 / K);
#pragma unroll
            for (int j = 0; j < NTR; ++j) {
                float m = 0.f;
#pragma unroll
                for (int r = 0; r < 16; ++r) {
                    m = fmaxf(m, relu_pos(__builtin_fmaf(acc[i][j][r], al, be)));
                    if ((r + 1) % rpg == 0) {
                        m = fmaxf(m, __shfl_xor(m, 32));
                        const unsigned g = (unsigned)(rbase + 32 * j) / K + r / rpg;
                        if (h == 0 && g < G) A.out[(int64_t)g * A.ostride + cb + col] = m;
                        m = 0.f;
                    }
                }
            }
        } else {
            // general group size: per element
#pragma unroll
            for (int j = 0; j < NTR; ++j)
#pragma unroll
                for (int r = 0; r < 16; ++r) {
                    const unsigned row = rbase + 32 * j + (r & 3) + 8 * (r >> 2) + 4 * h;
                    if (row < M) {
                        const unsigned g = row / K;
                        const unsigned u = __float_as_uint(relu_pos(__builtin_fmaf(acc[i][j][r], al, be)));
                        if (LDS_POOL && A.pool_mode == 1) atomicMax(&pool[((int)g - g0) * cw + col], u);
                        else atomicMax(reinterpret_cast<unsigned *>(A.out + (int64_t)g * A.ostride + cb + col), u);
                    }
                }
        }
    }
}

// flush the LDS pool (pool_mode 1) of one column slice
__device__ __forceinline__ void flush_pool(const MlpArgs &A, const unsigned *pool, int row0,
                                           int BM, int g0, int ngl, int cb, int cw, int tid) {
    const unsigned K = (unsigned)A.K, G = (unsigned)A.M / K;
    for (int e = tid; e < ngl * cw; e += kNT) {
        const int gl = e / cw;
        const int c = e - gl * cw;
        const unsigned g = g0 + gl;
        if (g >= G) continue;
        const unsigned val = pool[e];
        float *dst = A.out + (int64_t)g * A.ostride + cb + c;
        if (g * K >= (unsigned)row0 && (g + 1) * K <= (unsigned)(row0 + BM)) *dst = __uint_as_float(val);
        else atomicMax(reinterpret_cast<unsigned *>(dst), val);
    }
}

template <int BM, int NTR, int NTC, bool LAST>
__device__ __forceinline__ void run_layer(const MlpArgs &A, const LayerDev &L, float *act,
                                          unsigned *pool, int64_t row0, int tid, int lane,
                                          int wave) {
    using Gm = Geo<BM, NTR, NTC>;
    const int wr = wave / Gm::NWc, wc = wave % Gm::NWc;
    const int rt0 = wr * NTR;
    if constexpr (!LAST) {
        const int CT = L.cout >> 5;
        int ct[NTC];
#pragma unroll
        for (int i = 0; i < NTC; ++i) ct[i] = wc + i * Gm::NWc;
        floatx16 acc[NTC][NTR];
        mma_layer<NTR, NTC>(acc, act, A.ld, L, 0, ct, CT, rt0, lane);
        __syncthreads();  // every wave is done reading act for this layer
        const int h = lane >> 5, x = lane & 31;
#pragma unroll
        for (int i = 0; i < NTC; ++i) {
            if (ct[i] >= CT) continue;
            const int col = ct[i] * 32 + x;
            const float al = L.alpha[col], be = L.beta[col];
#pragma unroll
            for (int j = 0; j < NTR; ++j)
#pragma unroll
                for (int r = 0; r < 16; ++r) {
                    const int row = (rt0 + j) * 32 + (r & 3) + 8 * (r >> 2) + 4 * h;
                    act[row * A.ld + col] = relu_pos(__builtin_fmaf(acc[i][j][r], al, be));
                }
        }
        __syncthreads();
    } else {
        // one column slice (<= 256) per workgroup: the planner splits wider layers over grid.y
        const int cw = A.ycols;
        const int cb = blockIdx.y * A.ycols;
        const int CT = cw >> 5;
        int ct[NTC];
#pragma unroll
        for (int i = 0; i < NTC; ++i) ct[i] = wc + i * Gm::NWc;
        int g0 = 0;
        int ngl = 0;
        if (A.pool_mode == 1) {
            const unsigned K = (unsigned)A.K;
            g0 = (int)((unsigned)row0 / K);
            ngl = (int)((min((unsigned)row0 + BM, (unsigned)A.M) - 1) / K) - g0 + 1;
            for (int e = tid; e < ngl * cw; e += kNT) pool[e] = 0u;
            __syncthreads();
        }
        floatx16 acc[NTC][NTR];
        mma_layer<NTR, NTC>(acc, act, A.ld, L, cb, ct, CT, rt0, lane);
        last_epilogue<NTR, NTC, true>(A, acc, L, cb, ct, CT, (int)row0 + rt0 * 32, pool, g0, cw, lane);
        if (A.pool_mode == 1) {
            __syncthreads();
            flush_pool(A, pool, (int)row0, BM, g0, ngl, cb, cw, tid);
        }
    }
}

// shape code of a layer = NTR*4 + NTC (0: no layer)
#define PN2_NTR(code) ((code) >> 2)
#define PN2_NTC(code) ((code) & 3)

template <int BM, int S0, int S1, int S2, int S3>
__global__ __launch_bounds__(kNT, 4) void sa_mlp_kernel(const MlpArgs A) {
    extern __shared__ __attribute__((aligned(16))) float smem[];
    int *rn = reinterpret_cast<int *>(smem);
    int *rb = rn + BM;
    float *act = smem + 2 * BM;
    unsigned *pool = reinterpret_cast<unsigned *>(act + BM * A.ld);

    const int tid = threadIdx.x;
    const int lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int64_t row0 = (int64_t)blockIdx.x * BM;

    gather_rows(A, act, rn, rb, row0, BM, tid);
    __syncthreads();
    run_layer<BM, PN2_NTR(S0), PN2_NTC(S0), S1 == 0>(A, A.L[0], act, pool, row0, tid, lane, wave);
    if constexpr (S1 != 0)
        run_layer<BM, PN2_NTR(S1), PN2_NTC(S1), S2 == 0>(A, A.L[1], act, pool, row0, tid, lane, wave);
    if constexpr (S2 != 0)
        run_layer<BM, PN2_NTR(S2), PN2_NTC(S2), S3 == 0>(A, A.L[2], act, pool, row0, tid, lane, wave);
    if constexpr (S3 != 0)
        run_layer<BM, PN2_NTR(S3), PN2_NTC(S3), true>(A, A.L[3], act, pool, row0, tid, lane, wave);
}

// ------------------------------------------------------------------ dense single layer
// out = relu(alpha * (A x W^T) + beta) for a single layer whose input is too wide to keep an
// LDS-resident tile: 128 rows x one <=256-column slice per workgroup, A streamed through LDS in
// double-buffered 64-deep k chunks (row stride 66 = 2 mod 4), B from L2 as in the fused kernel.
constexpr int kDenseBM = 128, kDenseKC = 64, kDenseLd = kDenseKC + 2;
constexpr int kDenseLoads = kDenseBM * kDenseKC / 4 / kNT;  // float4 per thread per chunk

template <int NTR, int NTC>
__global__ __launch_bounds__(kNT, 4) void dense_layer_kernel(const MlpArgs A) {
    __shared__ __attribute__((aligned(16))) float abuf[2][kDenseBM * kDenseLd];
    const int tid = threadIdx.x;
    const int lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const LayerDev &L = A.L[0];
    const pn2_sa_src &s = A.src;
    const int64_t row0 = (int64_t)blockIdx.x * kDenseBM;
    const int cb = blockIdx.y * A.ycols;
    using Gm = Geo<kDenseBM, NTR, NTC>;
    const int wr = wave / Gm::NWc, wc = wave % Gm::NWc;
    const int rt0 = wr * NTR;
    const int CT = A.ycols >> 5;
    int ct[NTC];
#pragma unroll
    for (int i = 0; i < NTC; ++i) ct[i] = wc + i * Gm::NWc;

    // chunk loader: columns [k0, k0+64) of 128 rows.
    // ROWS: rows[R][k]; GROUP_ALL: [feat(b,n) | xyz(b,n) | 0] with R = b*N + n.
    floatx4 st[kDenseLoads];
    auto load = [&](int k0) {
#pragma unroll
        for (int u = 0; u < kDenseLoads; ++u) {
            const int e = tid + u * kNT;  // 128 rows x 16 float4
            const int r = e >> 4, q = e & 15;
            const int64_t R = row0 + r;
            const int k = k0 + 4 * q;
            floatx4 v = floatx4{0.f, 0.f, 0.f, 0.f};
            if (R < A.M && k < L.cin) {
                if (s.mode == PN2_SRC_ROWS) {
                    const float *fr = s.rows + R * s.rs;
                    if (A.vec_feat && k + 3 < L.cin) {
                        v = *reinterpret_cast<const floatx4 *>(fr + k);
                    } else {
#pragma unroll
                        for (int j = 0; j < 4; ++j) {
                            const float t = (k + j < L.cin) ? fr[k + j] : 0.f;
                            v[j] = t;
                        }
                    }
                } else {
                    const unsigned b = (unsigned)R / (unsigned)s.N, n = (unsigned)R - b * (unsigned)s.N;
                    const int D = (int)s.D;
                    const float *fr = s.feat + (int64_t)b * s.fb + (int64_t)n * s.fn;
                    if (A.vec_feat && k + 3 < D) {
                        v = *reinterpret_cast<const floatx4 *>(fr + k);
                    } else {
#pragma unroll
                        for (int j = 0; j < 4; ++j) {
                            const int kk = k + j;
                            v[j] = kk < D ? fr[kk]
                                 : kk < L.cin ? s.pts[(int64_t)b * s.pb + (int64_t)n * s.pn + (int64_t)(kk - D) * s.pc] : 0.f;
                        }
                    }
                }
            }
            st[u] = v;
        }
    };
    auto store = [&](float *buf) {
#pragma unroll
        for (int u = 0; u < kDenseLoads; ++u) {
            const int e = tid + u * kNT;
            const int r = e >> 4, q = e & 15;
            floatx2 *dst = reinterpret_cast<floatx2 *>(buf + r * kDenseLd + 4 * q);
            dst[0] = floatx2{st[u][0], st[u][1]};
            dst[1] = floatx2{st[u][2], st[u][3]};
        }
    };

    floatx16 acc[NTC][NTR];
    zero_acc<NTR, NTC>(acc);
    const floatx2 *bp0[NTC];
    b_ptrs<NTC>(bp0, L, cb, ct, CT, lane);
    const int pstride = 2 * L.cout;
    const int nch = (L.cin_pad + kDenseKC - 1) / kDenseKC;
    load(0);
    store(abuf[0]);
    __syncthreads();
    for (int c = 0; c < nch; ++c) {
        if (c + 1 < nch) load((c + 1) * kDenseKC);
        const float *ap[NTR];
#pragma unroll
        for (int j = 0; j < NTR; ++j)
            ap[j] = abuf[c & 1] + ((rt0 + j) * 32 + (lane & 31)) * kDenseLd + 2 * (lane >> 5);
        const floatx2 *bp[NTC];
#pragma unroll
        for (int i = 0; i < NTC; ++i) bp[i] = bp0[i] + (int64_t)(c * (kDenseKC / 4)) * pstride;
        mma_blocks<NTR, NTC>(acc, ap, bp, pstride, min(kDenseKC, L.cin_pad - c * kDenseKC) >> 3);
        if (c + 1 < nch) store(abuf[(c + 1) & 1]);
        __syncthreads();
    }
    last_epilogue<NTR, NTC, false>(A, acc, L, cb, ct, CT, (int)row0 + rt0 * 32, nullptr, 0, A.ycols, lane);
}

// Fused-chain signatures compiled (layer shape codes NTR*4+NTC; the reference's heads use
// SSG [64,64,128] [128,128,256], MSG [32,32,64] [64,64,128] [64,96,128] [32,64,128]
// [64,128,256] [96,128,256], group_all [256 | ...]).  BM=128: NTR in {1,2,4}; BM=64: {1,2}.
#define PN2_SIGS128(X)                                                                     \
    X(5, 0, 0, 0) X(6, 0, 0, 0) X(9, 0, 0, 0) X(17, 0, 0, 0)                               \
    X(5, 5, 9, 0) X(9, 9, 17, 0) X(5, 5, 5, 0) X(5, 6, 9, 0) X(5, 9, 17, 0) X(6, 9, 17, 0) \
    X(17, 17, 0, 0)
#define PN2_SIGS64(X)                                                                      \
    X(5, 0, 0, 0) X(9, 0, 0, 0) X(5, 5, 5, 0) X(5, 5, 9, 0) X(9, 9, 0, 0)
#define PN2_DENSE_SIGS(X) X(5) X(6) X(9)

}  // namespace pn2

using namespace pn2;

// ------------------------------------------------------------------ BN/conv packing
__global__ __launch_bounds__(256) void pack_layer_kernel(
    const float *__restrict__ W, const float *__restrict__ bias, const float *__restrict__ gamma,
    const float *__restrict__ beta, const float *__restrict__ mean, const float *__restrict__ var,
    float eps, int cout, int cin, int cin_pad, int rot, float *__restrict__ wt,
    float *__restrict__ alpha, float *__restrict__ beta_out) {
    const int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (e < (int64_t)cin_pad * cout) {
        // pair-interleaved W^T: element (k, o) at ((k>>1)*cout + o)*2 + (k&1); input channel of
        // LDS column k is (k + rot) % cin (rot moves the leading xyz channels behind the features)
        const int k = (int)(e / cout), o = (int)(e - (int64_t)k * cout);
        const float w = k < cin ? W[(int64_t)o * cin + (k + rot) % cin] : 0.f;
        wt[((int64_t)(k >> 1) * cout + o) * 2 + (k & 1)] = w;
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

extern "C" int64_t pn2_layer_cin_pad(int64_t cin) { return ((cin + 7) / 8) * 8; }

extern "C" int pn2_pack_layer_f32(const float *W, const float *bias, const float *gamma,
                                  const float *beta, const float *mean, const float *var,
                                  double eps, int64_t cout, int64_t cin, int64_t rot, float *wt,
                                  float *alpha, float *beta_out, void *stream) {
    PN2_REQUIRE(W && wt && alpha && beta_out, "pn2_pack_layer_f32: null pointer");
    PN2_REQUIRE(cout >= 1 && cin >= 1 && rot >= 0 && rot < cin, "pn2_pack_layer_f32: bad shape");
    const int64_t cinp = pn2_layer_cin_pad(cin);
    const int64_t tot = std::max(cinp * cout, cout);
    hipLaunchKernelGGL(pack_layer_kernel, dim3((unsigned)((tot + 255) / 256)), dim3(256), 0,
                       as_stream(stream), W, bias, gamma, beta, mean, var, (float)eps, (int)cout,
                       (int)cin, (int)cinp, (int)rot, wt, alpha, beta_out);
    PN2_LAUNCH_CHECK("pack_layer_kernel");
    return PN2_OK;
}

// ------------------------------------------------------------------ host side
struct Plan {
    MlpArgs A;
    int BM;      // rows per workgroup; 0 = dense kernel
    int64_t tiles;
    int ysplit;
    size_t lds;
    int S[kMaxLayers];
};

static int shape_code(int cw, int RT) {
    // column tiles of this layer (<= 8 per slice) -> NTR row tiles x NTC column tiles per wave:
    // the largest NTR (B-fragment reuse) that leaves no wave column without a column tile.
    const int CT = cw >> 5;
    int ntr = 1;
    while (ntr * 2 <= RT && kNW * (ntr * 2) / RT <= CT) ntr *= 2;
    const int nwc = kNW * ntr / RT;
    const int ntc = (CT + nwc - 1) / nwc;
    return ntr * 4 + ntc;
}

static size_t fused_lds(int BM, int ld, int pool_groups, int cw) {
    return (size_t)(2 * BM + BM * ld) * 4 + (size_t)pool_groups * cw * 4;
}

static int pool_mode_for(int64_t K, int BM, int ntr_last, int pool, size_t *groups) {
    *groups = 0;
    if (!pool) return 0;
    const int span = 32 * ntr_last;  // rows per wave row block
    if ((K % 32 == 0 && K <= span && span % K == 0) || K == 8 || K == 16) return 0;
    if (K <= BM) {
        *groups = (size_t)(BM / K + 2);
        return 1;
    }
    return 2;
}

static int make_plan(Plan &P, const pn2_sa_src &s, const pn2_mlp_layer *layers, int n, int pool,
                     float *out, int64_t ostride, int64_t M, int64_t K) {
    MlpArgs &A = P.A;
    memset(&A, 0, sizeof(A));
    memset(P.S, 0, sizeof(P.S));
    A.src = s;
    A.nlayers = n;
    A.M = M;
    A.K = pool ? K : 1;
    A.pool = pool ? 1 : 0;
    A.out = out;
    A.ostride = ostride;
    int maxw = 0;
    for (int l = 0; l < n; ++l) {
        const pn2_mlp_layer &q = layers[l];
        A.L[l].wt = q.wt; A.L[l].alpha = q.alpha; A.L[l].beta = q.beta;
        A.L[l].cin = (int)q.cin; A.L[l].cin_pad = (int)pn2_layer_cin_pad(q.cin);
        A.L[l].cout = (int)q.cout;
        if (l == 0) maxw = A.L[0].cin_pad;
        if (l < n - 1) maxw = std::max(maxw, (int)q.cout);
    }
    A.ld = maxw + 2;  // = 2 (mod 4): conflict-free ds_read_b64 of 32 rows
    const int64_t coutL = layers[n - 1].cout;
    const int D = s.mode == PN2_SRC_ROWS ? (int)layers[0].cin : (int)s.D;
    const float *fp = s.mode == PN2_SRC_ROWS ? s.rows : s.feat;
    const int64_t fr = s.mode == PN2_SRC_ROWS ? s.rs : s.fn;
    const int64_t fb = s.mode == PN2_SRC_ROWS ? 0 : s.fb;
    A.vec_feat = (D > 0 && D % 4 == 0 && ((uintptr_t)fp & 15) == 0 && fr % 4 == 0 && fb % 4 == 0) ? 1 : 0;

    // dense kernel: a single layer over dense rows / group_all whose input is wide (no gather
    // tables needed, A streams through LDS in k chunks)
    const bool wide = A.L[0].cin_pad >= 256 || fused_lds(128, A.ld, 0, 0) > 80 * 1024;
    const bool dense = n == 1 && (s.mode == PN2_SRC_ROWS || s.mode == PN2_SRC_GROUP_ALL) && wide;
    P.BM = dense ? 0 : 128;
    if (!dense && fused_lds(128, A.ld, 0, 0) > 80 * 1024) {
        if (n > 1 && (s.mode == PN2_SRC_ROWS || s.mode == PN2_SRC_GROUP_ALL))
            return set_error(PN2_EUNSUPPORTED, "pn2_sa_mlp_max_f32: wide dense chain runs per layer");
        P.BM = 64;
    }
    const int BMr = dense ? kDenseBM : P.BM;
    P.tiles = (M + BMr - 1) / BMr;
    P.ysplit = 1;
    // at most one 256-column slice per workgroup (128 for the dense kernel: its A staging
    // registers + 64 accumulators would not fit the 4-waves/SIMD budget)
    while (coutL / P.ysplit > (dense ? kMaxSlice / 2 : kMaxSlice)) P.ysplit *= 2;
    if (n > 1 && P.ysplit > 1)
        return set_error(PN2_EUNSUPPORTED, "pn2_sa_mlp_max_f32: chained layer wider than %d", kMaxSlice);
    if (n == 1)  // a single layer can split its columns over grid.y (nothing is recomputed)
        while (P.tiles * P.ysplit < 512 && coutL / (P.ysplit * 2) >= 64 &&
               (coutL / (P.ysplit * 2)) % 32 == 0)
            P.ysplit *= 2;
    A.ycols = (int)(coutL / P.ysplit);
    const int RT = BMr / 32;
    for (int l = 0; l < n; ++l) {
        const int cw = (l == n - 1) ? std::min(A.ycols, kMaxSlice) : (int)layers[l].cout;
        P.S[l] = shape_code(cw, RT);
    }
    size_t groups = 0;
    A.pool_mode = pool_mode_for(pool ? K : 1, BMr, P.S[n - 1] >> 2, pool, &groups);
    if (dense && A.pool_mode == 1) A.pool_mode = 2;  // the dense kernel has no LDS pool
    P.lds = dense ? 0 : fused_lds(P.BM, A.ld, (int)groups, std::min(A.ycols, kMaxSlice));
    if (P.lds > 160 * 1024)
        return set_error(PN2_EUNSUPPORTED, "pn2_sa_mlp_max_f32: LDS %zu > 160 KiB (ld=%d)", P.lds, A.ld);
    return PN2_OK;
}

template <int BM, int S0, int S1, int S2, int S3>
static int launch_sig(const Plan &P, hipStream_t st) {
    static const hipError_t attr = hipFuncSetAttribute(  // one-time, idempotent
        reinterpret_cast<const void *>(&sa_mlp_kernel<BM, S0, S1, S2, S3>),
        hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    (void)attr;
    hipLaunchKernelGGL((sa_mlp_kernel<BM, S0, S1, S2, S3>), dim3((unsigned)P.tiles, (unsigned)P.ysplit),
                       dim3(kNT), P.lds, st, P.A);
    PN2_LAUNCH_CHECK("sa_mlp_kernel");
    return PN2_OK;
}

template <int S0>
static int launch_dense(const Plan &P, hipStream_t st) {
    hipLaunchKernelGGL((dense_layer_kernel<PN2_NTR(S0), PN2_NTC(S0)>),
                       dim3((unsigned)P.tiles, (unsigned)P.ysplit), dim3(kNT), 0, st, P.A);
    PN2_LAUNCH_CHECK("dense_layer_kernel");
    return PN2_OK;
}

static bool has_kernel(const Plan &P) {
    bool found = false;
#define PN2_HAS128(a, b, c, d) \
    if (P.BM == 128 && P.S[0] == a && P.S[1] == b && P.S[2] == c && P.S[3] == d) found = true;
#define PN2_HAS64(a, b, c, d) \
    if (P.BM == 64 && P.S[0] == a && P.S[1] == b && P.S[2] == c && P.S[3] == d) found = true;
#define PN2_HASD(a) \
    if (P.BM == 0 && P.S[0] == a) found = true;
    PN2_SIGS128(PN2_HAS128) PN2_SIGS64(PN2_HAS64) PN2_DENSE_SIGS(PN2_HASD)
#undef PN2_HAS128
#undef PN2_HAS64
#undef PN2_HASD
    return found;
}

// returns 1 when launched, 0 when no kernel is compiled for the plan, <0 on error
static int try_launch(const Plan &P, hipStream_t st) {
    if (!has_kernel(P)) return 0;
    if (P.A.pool && P.A.pool_mode != 0 && (P.A.pool_mode == 2 || (P.BM && P.BM % P.A.K != 0))) {
        // groups straddle workgroups: merged with atomicMax into a zeroed output
        const int64_t coutL = (int64_t)P.A.ycols * P.ysplit;
        const int64_t G = P.A.M / P.A.K;
        hipError_t e = (P.A.ostride == coutL)
                           ? hipMemsetAsync(P.A.out, 0, (size_t)G * coutL * 4, st)
                           : hipMemset2DAsync(P.A.out, (size_t)P.A.ostride * 4, 0, (size_t)coutL * 4,
                                              (size_t)G, st);
        if (e != hipSuccess)
            return set_error(PN2_EHIP, "pn2_sa_mlp_max_f32: memset: %s", hipGetErrorString(e));
    }
    int rc = PN2_EUNSUPPORTED;
#define PN2_GO128(a, b, c, d) \
    if (P.BM == 128 && P.S[0] == a && P.S[1] == b && P.S[2] == c && P.S[3] == d) rc = launch_sig<128, a, b, c, d>(P, st);
#define PN2_GO64(a, b, c, d) \
    if (P.BM == 64 && P.S[0] == a && P.S[1] == b && P.S[2] == c && P.S[3] == d) rc = launch_sig<64, a, b, c, d>(P, st);
#define PN2_GOD(a) \
    if (P.BM == 0 && P.S[0] == a) rc = launch_dense<a>(P, st);
    PN2_SIGS128(PN2_GO128) PN2_SIGS64(PN2_GO64) PN2_DENSE_SIGS(PN2_GOD)
#undef PN2_GO128
#undef PN2_GO64
#undef PN2_GOD
    return rc == PN2_OK ? 1 : rc;
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
        PN2_REQUIRE(s.pts && s.ctr && (s.idx || s.idx32) && (s.D == 0 || s.feat), "pn2_sa_mlp_max_f32: group source");
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
    PN2_REQUIRE(M < (int64_t(1) << 31), "pn2_sa_mlp_max_f32: %lld rows exceed 2^31", (long long)M);
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
// go to two ping-pong [M][w] workspace buffers.  A segment with no compiled kernel runs layer
// by layer through the same workspace.
static int seg_end(const pn2_mlp_layer *layers, int nlayers, int l0) {
    // a layer wider than one column slice runs alone (its columns split over grid.y)
    if (layers[l0].cout > kMaxSlice) return l0;
    int l = l0;
    while (l < nlayers - 1 && layers[l + 1].cout <= kMaxSlice) ++l;
    return l;  // inclusive
}

static bool segment_ok(const pn2_sa_src &s, const pn2_mlp_layer *layers, int l0, int l1,
                       int64_t M, int64_t K, int pool) {
    Plan P;
    if (make_plan(P, s, layers + l0, l1 - l0 + 1, pool, nullptr, layers[l1].cout, M, K) != PN2_OK)
        return false;
    return has_kernel(P);
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

// workspace row width: the widest layer output that has to round-trip through HBM (rounded
// to 4 floats so every workspace row is 16-byte aligned)
static int64_t workspace_width(const pn2_sa_src &s, const pn2_mlp_layer *layers, int nlayers,
                               int64_t M, int64_t K) {
    int64_t w = 0;
    for (int l0 = 0; l0 < nlayers;) {
        const int l1 = seg_end(layers, nlayers, l0);
        const bool last_seg = l1 == nlayers - 1;
        pn2_sa_src src = s;
        if (l0 > 0) src = rows_src(reinterpret_cast<const float *>(256), 1024, M, K);
        if (!segment_ok(src, layers, l0, l1, M, K, last_seg ? 1 : 0))
            for (int l = l0; l < l1; ++l) w = std::max(w, layers[l].cout);
        if (!last_seg) w = std::max(w, layers[l1].cout);
        l0 = l1 + 1;
    }
    return (w + 3) / 4 * 4;
}

extern "C" int64_t pn2_sa_mlp_workspace_bytes(const pn2_sa_src *src, const pn2_mlp_layer *layers,
                                              int nlayers) {
    int64_t M = 0, K = 1;
    if (validate(src, layers, nlayers, M, K) != PN2_OK) return -1;
    const int64_t ds = nlayers > 1 ? dense_split_width(*src, layers, nlayers, 3) : 0;
    return std::max({dense_split_ws_bytes(M, ds), 2 * M * workspace_width(*src, layers, nlayers, M, K) * 4,
                     chain_prepass_bytes(*src, layers, nlayers, 3)});
}

static int run_plan(const pn2_sa_src &cur, const pn2_mlp_layer *layers, int l0, int l1, int pool,
                    float *dst, int64_t ostride, int64_t M, int64_t K, hipStream_t st) {
    Plan P;
    int rc = make_plan(P, cur, layers + l0, l1 - l0 + 1, pool, dst, ostride, M, K);
    if (rc != PN2_OK) return rc;
    rc = try_launch(P, st);
    if (rc < 0) return rc;
    if (rc == 0)
        return set_error(PN2_EUNSUPPORTED, "pn2_sa_mlp_max_f32: no kernel for layers %d..%d (shape %d,%d,%d,%d BM=%d)",
                         l0, l1, P.S[0], P.S[1], P.S[2], P.S[3], P.BM);
    return PN2_OK;
}

static thread_local int g_last_path = 0;
static thread_local int g_last_planes = 0;  // planes per operand of the call's MLP kernels
extern "C" int pn2_sa_mlp_last_path(void) { return g_last_path; }
extern "C" int pn2_sa_mlp_last_planes(void) { return g_last_planes; }
static thread_local int g_last_side = -1;  // pn2_sa_mlp_last_fps_side
extern "C" int pn2_sa_mlp_last_fps_side(void) { return g_last_side; }

// the src's zero side job on the paths whose kernels do not take it (the dense-layer path's
// last layer does)
static int zero_side_job(const pn2_sa_src &s, hipStream_t st) {
    if (!s.zero_out || s.zero_count <= 0) return PN2_OK;
    const hipError_t e = hipMemsetAsync(s.zero_out, 0, (size_t)s.zero_count * 4, st);
    return e == hipSuccess ? PN2_OK : set_error(PN2_EHIP, "pn2_sa_mlp_max: zero_out: %s", hipGetErrorString(e));
}

static int mlp_max_f32(const pn2_sa_src *src, const pn2_mlp_layer *layers,
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
    rc = try_launch_chain(*src, layers, nlayers, pool, out, ostride, M, K, 3, workspace,
                          workspace_bytes, st);
    if (rc != 0) {
        if (rc > 0) g_last_path = PN2_PATH_SPLIT_BF16, g_last_planes = chain_last_planes();
        return rc < 0 ? rc : zero_side_job(*src, st);
    }
    rc = try_launch_dense_split(*src, layers, nlayers, pool, out, ostride, workspace, workspace_bytes,
                                M, K, 3, st);
    if (rc != 0) {
        if (rc > 0) g_last_path = PN2_PATH_SPLIT_BF16, g_last_planes = dense_last_planes();
        return rc < 0 ? rc : PN2_OK;
    }
    if ((rc = zero_side_job(*src, st)) != PN2_OK) return rc;
    for (int l = 0; l < nlayers; ++l)
        if (layers[l].flags & PN2_LAYER_NO_RELU)
            return set_error(PN2_EUNSUPPORTED, "pn2_sa_mlp_max_f32: layer %d without ReLU needs the split "
                             "dense-layer path (group_all / rows source, split weight images)", l);
    g_last_path = PN2_PATH_F32;
    g_last_planes = 0;
    const int64_t w = workspace_width(*src, layers, nlayers, M, K);
    if (w > 0)
        PN2_REQUIRE(workspace && workspace_bytes >= 2 * M * w * 4 && ((uintptr_t)workspace & 15) == 0,
                    "pn2_sa_mlp_max_f32: this layer chain needs a 16-byte aligned %lld-byte workspace",
                    (long long)(2 * M * w * 4));
    pn2_sa_src cur = *src;
    int buf = 0;
    for (int l0 = 0; l0 < nlayers;) {
        const int l1 = seg_end(layers, nlayers, l0);
        const bool last_seg = l1 == nlayers - 1;
        if (segment_ok(cur, layers, l0, l1, M, K, last_seg ? pool : 0)) {
            float *dst = last_seg ? out : workspace + buf * M * w;
            rc = run_plan(cur, layers, l0, l1, last_seg ? pool : 0, dst, last_seg ? ostride : w, M, K, st);
            if (rc != PN2_OK) return rc;
            if (!last_seg) { cur = rows_src(dst, w, M, K); buf ^= 1; }
        } else {
            for (int l = l0; l <= l1; ++l) {
                const bool last = l == nlayers - 1;
                float *dst = last ? out : workspace + buf * M * w;
                rc = run_plan(cur, layers, l, l, last ? pool : 0, dst, last ? ostride : w, M, K, st);
                if (rc != PN2_OK) return rc;
                if (!last) { cur = rows_src(dst, w, M, K); buf ^= 1; }
            }
        }
        l0 = l1 + 1;
    }
    return PN2_OK;
}

// bf16 arithmetic (BASELINE config 5, the large-N stress run): the same fused kernels with one
// bf16 plane per operand -- activations rounded to bf16 (round-to-nearest-even) where a layer
// reads them, weights = the hi plane of the split image, products exact, fp32 accumulation,
// BN / ReLU / max in fp32, fp32 output.  No fp32 fallback: a chain neither the chain kernel nor
// the dense-layer kernel covers is PN2_EUNSUPPORTED.
extern "C" int64_t pn2_sa_mlp_workspace_bytes_bf16(const pn2_sa_src *src,
                                                   const pn2_mlp_layer *layers, int nlayers) {
    int64_t M = 0, K = 1;
    if (validate(src, layers, nlayers, M, K) != PN2_OK) return -1;
    const int64_t ds = nlayers > 1 ? dense_split_width(*src, layers, nlayers, 1) : 0;
    return std::max(ds ? dense_split_ws_bytes(M, ds) : 0, chain_prepass_bytes(*src, layers, nlayers, 1));
}

static int mlp_max_bf16(const pn2_sa_src *src, const pn2_mlp_layer *layers,
                        int nlayers, int pool, float *out, int64_t ostride,
                        float *workspace, int64_t workspace_bytes, void *stream) {
    int64_t M = 0, K = 1;
    int rc = validate(src, layers, nlayers, M, K);
    if (rc != PN2_OK) return rc;
    PN2_REQUIRE(out, "pn2_sa_mlp_max_bf16: null out");
    PN2_REQUIRE(ostride >= layers[nlayers - 1].cout, "pn2_sa_mlp_max_bf16: ostride");
    for (int l = 0; l < nlayers; ++l)
        PN2_REQUIRE(layers[l].wt_split && ((uintptr_t)layers[l].wt_split & 15) == 0,
                    "pn2_sa_mlp_max_bf16: layer %d needs its 16-byte aligned split weight image", l);
    if (M == 0) return PN2_OK;
    if (pool) PN2_REQUIRE(M % K == 0, "pn2_sa_mlp_max_bf16: rows not a multiple of the group size");
    hipStream_t st = as_stream(stream);
    rc = try_launch_chain(*src, layers, nlayers, pool, out, ostride, M, K, 1, workspace,
                          workspace_bytes, st);
    if (rc > 0 && (rc = zero_side_job(*src, st)) == PN2_OK) rc = 1;
    if (rc == 0)
        rc = try_launch_dense_split(*src, layers, nlayers, pool, out, ostride, workspace,
                                    workspace_bytes, M, K, 1, st);
    if (rc < 0) return rc;
    if (rc == 0)
        return set_error(PN2_EUNSUPPORTED,
                         "pn2_sa_mlp_max_bf16: no bf16 kernel for this chain (%d layers, mode %d) "
                         "or workspace too small", nlayers, src->mode);
    g_last_path = PN2_PATH_BF16;
    g_last_planes = 1;
    return PN2_OK;
}

// The entry points: the MLP, and the caller's FPS side job (pn2_fps_side) -- inside the chain
// launch when try_launch_chain took it, else as its own launch after the MLP's
template <typename F>
static int with_fps_side(const pn2_sa_src *src, void *stream, F &&mlp) {
    const pn2_fps_side *side = src ? src->fps_side : nullptr;
    if (side) {
        const int rc = fps_side_check(*side);
        if (rc != PN2_OK) return rc;
    }
    fps_side_taken() = false;
    const int rc = mlp();
    const bool taken = fps_side_taken();
    fps_side_taken() = false;
    if (rc != PN2_OK) return rc;
    g_last_side = !side ? -1 : taken ? 1 : 0;
    if (!side || taken) return rc;
    return fps_side_launch(*side, as_stream(stream));
}

extern "C" int pn2_sa_mlp_max_f32(const pn2_sa_src *src, const pn2_mlp_layer *layers,
                                  int nlayers, int pool, float *out, int64_t ostride,
                                  float *workspace, int64_t workspace_bytes, void *stream) {
    return with_fps_side(src, stream, [&] {
        return mlp_max_f32(src, layers, nlayers, pool, out, ostride, workspace, workspace_bytes, stream);
    });
}

extern "C" int pn2_sa_mlp_max_bf16(const pn2_sa_src *src, const pn2_mlp_layer *layers,
                                   int nlayers, int pool, float *out, int64_t ostride,
                                   float *workspace, int64_t workspace_bytes, void *stream) {
    return with_fps_side(src, stream, [&] {
        return mlp_max_bf16(src, layers, nlayers, pool, out, ostride, workspace, workspace_bytes, stream);
    });
}
