// sa_dense.hip -- one wide shared-MLP layer as a split-bf16 GEMM on gfx950: the group_all SA
// layer (PointNetSetAbstraction with group_all=True, /root/reference/model/pointnet2_utils.py
// :163-172 over sample_and_group_all :122-141) and any chain too wide for the register-resident
// kernel run layer by layer through an HBM workspace with it.
//
//   out = relu(alpha * (A . W^T) + beta)            (optionally max-pooled over K-row groups)
//
// Workgroup: 4 waves, 128 rows x NTC 32-column tiles; wave w owns rows 32w..32w+31 (standard
// MFMA orientation: A = activations, lane = row; B = weights, lane = output column).
//   A   each lane loads its row's 16-channel k-block (two 16-byte runs) straight from HBM/L2 --
//       the previous layer's fp32 rows, or for group_all's first layer the [xyz | features] of
//       the point (split layout: block 0 = xyz, blocks >= 1 = features) -- splits it once and
//       feeds all NTC column tiles with it.  A for the next stage is loaded before the stage's
//       weight DMA is issued, so waiting for it never waits for the DMA.
//   B   the workgroup's weight fragments (3 planes x NTC tiles x kKC k-blocks = one stage) are
//       copied to LDS once by global_load_lds, double-buffered, one barrier per stage.
//   out dense rows (row-major, coalesced per row), or the max over each group of K rows: in
//       registers, then across the workgroup's waves in LDS (K | 128), or by atomicMax on the
//       float bits into a zeroed output (ReLU output >= +0: uint order == float order).
#include "pn2_internal.h"
#include "split_bf16.h"

#include <algorithm>
#include <cstdlib>
#include <cstring>

namespace pn2 {

// Timeline stamps (diagnostic builds only: -DPN2_DENSE_STAMPS, tools/debug/dense_stamps.py):
// s_memrealtime (100 MHz, chip-wide) of every workgroup of the last launch, wave 0 lane 0:
// [0] entry, [1 + c] past stage c's barrier (c < 12), [14] main loop done, [15] exit; [16] /
// [17] s_memtime (shader clock) at entry / exit.
#ifdef PN2_DENSE_STAMPS
constexpr int kDStampWG = 4096, kDStamps = 18;
__device__ unsigned long long g_dense_stamps[kDStampWG * kDStamps];
// launches stamped: every one (-1, the last one wins) or those with mode * 1000 + tiles == sel
__device__ int g_dense_sel = -1;
extern "C" int pn2_debug_dense_select(int sel) {
    return hipMemcpyToSymbol(HIP_SYMBOL(g_dense_sel), &sel, sizeof(int)) == hipSuccess ? 0 : -1;
}
#define PN2_DSEL (g_dense_sel < 0 || g_dense_sel == A.mode * 1000 + A.tiles)
#define PN2_DSTAMP(i)                                                                           \
    do {                                                                                        \
        const unsigned b_ = blockIdx.x + blockIdx.y * gridDim.x;                                \
        if (threadIdx.x == 0 && b_ < kDStampWG && PN2_DSEL)                                     \
            g_dense_stamps[b_ * kDStamps + (i)] = __builtin_amdgcn_s_memrealtime();             \
    } while (0)
extern "C" int pn2_debug_dense_stamps(unsigned long long *dst, int64_t n) {
    const int64_t m = n < (int64_t)kDStampWG * kDStamps ? n : (int64_t)kDStampWG * kDStamps;
    return hipMemcpyFromSymbol(dst, HIP_SYMBOL(g_dense_stamps), m * 8) == hipSuccess ? 0 : -1;
}
#define PN2_DCLOCK(i)                                                                           \
    do {                                                                                        \
        const unsigned b_ = blockIdx.x + blockIdx.y * gridDim.x;                                \
        if (threadIdx.x == 0 && b_ < kDStampWG && PN2_DSEL)                                     \
            g_dense_stamps[b_ * kDStamps + (i)] = __builtin_amdgcn_s_memtime();                 \
    } while (0)
#else
#define PN2_DSTAMP(i) do {} while (0)
#define PN2_DCLOCK(i) do {} while (0)
#endif

constexpr int kDW = 4;            // waves per workgroup
constexpr int kDRows = 32 * kDW;  // rows per workgroup
constexpr int kKC = 4;            // k-blocks per weight stage

struct DenseSplitArgs {
    int mode;  // 0: rows [M][rs] fp32; 1: group_all points (row R = point R % N of cloud R / N)
    const float *rows;
    int64_t rs;
    const float *pts;
    int64_t pb, pn, pc;
    const float *feat;
    int64_t fb, fn;
    int N, C, D;  // group_all: points per cloud, xyz channels, feature channels
    int cin;      // rows mode: valid input channels
    int vec;      // 16-byte loads of feature / row runs are allowed
    const bf16x8 *w;
    const float *alpha, *beta;
    int kb, tiles;  // k-blocks of the input, 32-column tiles of the output
    int M;
    int pool;       // 0: out[row][col]; 1: out[group][col] = max over K rows
    int K;
    int pool_mode;  // 0: registers (K = 8, 16), 1: LDS (K | kDRows), 2: HBM atomics
    float *out;
    int64_t ostride;
    int raw;        // 1: out = A . W^T as accumulated (no BN / ReLU; the chain's layer-0 pre-pass)
    int norelu;     // 1: out = alpha * (A . W^T) + beta, no ReLU (signed values: pooled as keys)
    // side job: zero [zrows][zcols] floats at `zero` (row stride zstride) -- the NEXT layer's
    // atomicMax pool, so that layer needs no memset launch of its own
    float *zero;
    int64_t zrows, zcols, zstride;
    // dense_lds_kernel: XCD x runs a (row blocks / (8 / xcx)) x (column tiles / xcx) rectangle of
    // the output (0: XCD-contiguous logical ids, whole row blocks per XCD)
    int xcx;
    // split fp16 (NP = 2, rows mode): w = the image's fp16 planes, wscale the weight rows' inverse
    // scales, in_max [M/32][in_tiles] the producing layer's per-(32-row block, 32-column tile)
    // max |value| bits (split_bf16.h): each wave's activation scale
    const float *wscale;
    const unsigned *in_max;
    int in_tiles;
    // out_max [M/32][tiles] (or null): this layer's own per-(row block, tile) max |value| bits of
    // the rows it writes (pool == 0), for an NP = 2 layer after it
    unsigned *out_max;
    // fragment-ordered hidden rows (frag_off): the producing layer writes them (frag_out), the
    // register-staged consumer reads each lane's k-block as 32 contiguous bytes (frag_in, rows
    // mode: `rows` is the block array, rs unused) -- a wave's A operand one 2 KB run per k-block
    // instead of 16-byte pieces of 32 rows
    int frag_in, frag_out;
};

// Fragment order of a [M][16*kbw] row matrix: block (32-row block, 16-channel k-block) = 512
// floats, lane (r, h) = (row & 31) + 32h holding channels (j&3) + 8(j>>2) + 4h of its row in
// element j -- the A-fragment order of split_bf16.h, so a lane's 8 values are contiguous
__host__ __device__ __forceinline__ int64_t frag_off(int64_t row, int col, int kbw) {
    return (((row >> 5) * kbw + (col >> 4)) * 64 + (row & 31) + 32 * ((col >> 2) & 1)) * 8 + (col & 3) +
           4 * ((col >> 3) & 1);
}

// NP = 2: this wave's activation scale, from the max |value| of its 32 rows (rb*32 ..): the
// producing layer's per-(row block, tile) maxima (in_max, rows mode), or -- a first layer over
// points (mode 1: group_all, the pre-pass) -- the rows themselves, read once more before the
// main loop ([xyz | features], L2-resident; lane (r, h) takes every other channel of row r)
__device__ __forceinline__ unsigned abs_bits(float x) { return __float_as_uint(x) & 0x7FFFFFFFu; }
template <int NP>
__device__ __forceinline__ ActScale dense_act_scale(const DenseSplitArgs &A, int rb, int lane) {
    if constexpr (NP != 2) {
        return ActScale{1.f, 1.f};
    } else {
        unsigned m = 0;
        if (A.in_max) {
            if (32 * rb < A.M)
                for (int t = lane; t < A.in_tiles; t += 64) m = max(m, A.in_max[(int64_t)rb * A.in_tiles + t]);
        } else {
            const int h = lane >> 5, R = 32 * rb + (lane & 31);
            if (R < A.M) {
                const int b = R / A.N, n = R - b * A.N;
                const float *p = A.pts + (int64_t)b * A.pb + (int64_t)n * A.pn;
                for (int c = h; c < A.C; c += 2) m = max(m, abs_bits(p[(int64_t)c * A.pc]));
                if (A.feat) {
                    const float *f = A.feat + (int64_t)b * A.fb + (int64_t)n * A.fn;
                    if (A.vec) {
                        for (int c = 4 * h; c < A.D; c += 8) {
                            const cfloatx4 q = *reinterpret_cast<const cfloatx4 *>(f + c);
                            m = max(max(m, max(abs_bits(q[0]), abs_bits(q[1]))), max(abs_bits(q[2]), abs_bits(q[3])));
                        }
                    } else {
                        for (int c = h; c < A.D; c += 2) m = max(m, abs_bits(f[c]));
                    }
                }
            }
        }
        return act_scale(__uint_as_float(wave_max_u32(m)));
    }
}
// a k-block of the A operand split, scaled first for NP = 2
template <int NP>
__device__ __forceinline__ Split split_scaled(const float (&x)[8], float up) {
    if constexpr (NP == 2) {
        float y[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) y[j] = x[j] * up;
        return splitN<NP>(y);
    } else {
        return splitN<NP>(x);
    }
}
// the BN scale of output column col (NP = 2: times the weight row's inverse scale and the
// wave's activation down-scale)
template <int NP>
__device__ __forceinline__ float dense_alpha(const DenseSplitArgs &A, int col, float down) {
    if constexpr (NP == 2) return (A.raw ? 1.f : A.alpha[col]) * A.wscale[col] * down;
    else return A.raw ? 1.f : A.alpha[col];
}

// Signed max through unsigned atomics: key() is monotone from float order to uint order (and
// key(anything) > 0, so a zeroed pool is below every value); unkey() inverts it.
__device__ __forceinline__ unsigned fkey(float f) {
    const unsigned u = __float_as_uint(f);
    return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
}
__device__ __forceinline__ float funkey(unsigned k) {
    return __uint_as_float((k & 0x80000000u) ? (k & 0x7fffffffu) : ~k);
}

__global__ void unkey_kernel(float *out, int64_t ostride, int64_t G, int cols) {
    const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (e >= G * cols) return;
    const int64_t g = e / cols;
    float *p = out + g * ostride + (e - g * cols);
    *p = funkey(__float_as_uint(*p));
}

// one lane-linear 16-byte-per-lane copy HBM/L2 -> LDS (global_load_lds, no VGPR destination)
__device__ __forceinline__ void dma16(const char *src, char *dst) {
    __builtin_amdgcn_global_load_lds(src, (lds_void *)dst, 16, 0, 0);
}

// raw s_barrier (__syncthreads' fence would wait vmcnt(0) and drain the DMA ring)
__device__ __forceinline__ void stage_barrier() {
    asm volatile("" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
}

template <int NTC, int NP, bool FAST, int NW>
__global__ __launch_bounds__(64 * NW) __attribute__((amdgpu_waves_per_eu(NW == 4 ? (NTC == 1 ? 4 : NTC == 2 ? 3 : 1) : 1)))
void dense_split_kernel(const DenseSplitArgs A) {
    constexpr int kDW = NW, kDRows = 32 * NW;  // waves, rows per workgroup
    extern __shared__ __attribute__((aligned(16))) char dsm[];
    PN2_DSTAMP(0);
    constexpr int kFrag = NP * NTC;                  // fragments per k-block
    constexpr int kStage = kKC * kFrag * 1024;       // bytes per weight stage
    const int tid = threadIdx.x;
    const int lane = tid & 63;
    const int r = lane & 31, h = lane >> 5;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    // logical (row block, column tiles) with the row blocks in contiguous ranges per XCD: the
    // next layer's row block runs on the XCD whose L2 holds its rows (and the SA chain's
    // workgroups of a cloud on the one whose L2 holds the cloud's pre-pass rows)
    const unsigned lid = xcd_contiguous(blockIdx.x + blockIdx.y * gridDim.x, gridDim.x * gridDim.y);
    const int row0 = (int)(lid / gridDim.y) * kDRows;
    const int ct0 = (int)(lid % gridDim.y) * NTC;  // first output tile
    const int ncols = 32 * NTC;
    char *stages = dsm;
    float *opool = reinterpret_cast<float *>(dsm + 2 * kStage);  // [groups][ncols]
    const int gpb = A.pool_mode == 1 ? kDRows / A.K : 0;
    if (A.pool_mode == 1)
        for (int e = tid; e < gpb * ncols; e += 64 * kDW) opool[e] = 0.f;
    if (A.zero) {  // this workgroup's share of the next layer's pool (stream order publishes it)
        const int64_t tot = A.zrows * A.zcols, nwg = (int64_t)gridDim.x * gridDim.y;
        const int64_t per = (tot + nwg - 1) / nwg, e0 = (int64_t)(blockIdx.x + blockIdx.y * gridDim.x) * per;
        const int64_t e1 = e0 + per < tot ? e0 + per : tot;
        for (int64_t e = e0 + tid; e < e1; e += 64 * kDW) {
            const int64_t g = e / A.zcols;
            A.zero[g * A.zstride + (e - g * A.zcols)] = 0.f;
        }
    }

    // ---- this lane's row (A operand)
    const int R = row0 + 32 * wave + r;
    const bool valid = R < A.M;
    const ActScale asc = dense_act_scale<NP>(A, (row0 >> 5) + wave, lane);
    const float *arow = nullptr, *frow = nullptr, *prow = nullptr;
    if (A.mode == 0) {
        if (A.frag_in) {  // this lane's 8 values of k-block 0 (rows past M: the last row's)
            const int fr = valid ? R : A.M - 1;
            arow = A.rows + ((int64_t)(fr >> 5) * A.kb * 64 + (fr & 31) + 32 * h) * 8;
        } else {
            arow = A.rows + (int64_t)(valid ? R : 0) * A.rs;
        }
    } else {
        const int b = (valid ? R : 0) / A.N, n = (valid ? R : 0) - b * A.N;
        prow = A.pts + (int64_t)b * A.pb + (int64_t)n * A.pn;
        if (A.feat) frow = A.feat + (int64_t)b * A.fb + (int64_t)n * A.fn;
    }
    // lane (r, h) holds channels 16kb + (j&3) + 8(j>>2) + 4h of its row in element j
    auto load_a = [&](int kb, float (&x)[8]) {
        if (!valid || kb >= A.kb) {
#pragma unroll
            for (int j = 0; j < 8; ++j) x[j] = 0.f;
            return;
        }
        if (A.mode == 1 && kb == 0) {  // raw xyz (sample_and_group_all does not centre)
#pragma unroll
            for (int j = 0; j < 8; ++j) {
                const int ch = (j & 3) + 8 * (j >> 2) + 4 * h;
                x[j] = ch < A.C ? prow[(int64_t)ch * A.pc] : 0.f;
            }
            return;
        }
        if (A.mode == 0 && A.frag_in) {
            const float *p = arow + 512 * (int64_t)kb;
#pragma unroll
            for (int run = 0; run < 2; ++run) {
                const cfloatx4 q = *reinterpret_cast<const cfloatx4 *>(p + 4 * run);
#pragma unroll
                for (int i = 0; i < 4; ++i) x[4 * run + i] = q[i];
            }
            return;
        }
        const float *src = A.mode == 0 ? arow : frow;
        const int lim = A.mode == 0 ? A.cin : A.D;
        const int base = A.mode == 0 ? 16 * kb : 16 * (kb - 1);
#pragma unroll
        for (int run = 0; run < 2; ++run) {
            const int f = base + 8 * run + 4 * h;
            if (A.vec) {
                cfloatx4 q = {0.f, 0.f, 0.f, 0.f};
                if (f < lim) q = *reinterpret_cast<const cfloatx4 *>(src + f);
#pragma unroll
                for (int i = 0; i < 4; ++i) x[4 * run + i] = q[i];
            } else {
#pragma unroll
                for (int i = 0; i < 4; ++i) x[4 * run + i] = f + i < lim ? src[f + i] : 0.f;
            }
        }
    };

    // FAST: every k-block past the first stage is 16 contiguous channels of one row run, at
    // lrow + 16 kb (rows mode: the row; group_all: the features, blocks >= 1) -- two 16-byte
    // loads at immediate offsets from one pointer per stage, no per-element branches
    const float *lrow = A.mode == 0 ? arow : frow - 16;
    if (!(A.mode == 0 && A.frag_in)) lrow += 4 * h;
    auto load_fast = [&](int c, float (&x)[kKC][8]) {
        const int kb0 = c * kKC;
        if (A.mode == 0 && A.frag_in) {  // k-block kb: 8 contiguous floats at lrow + 512 kb
#pragma unroll
            for (int k = 0; k < kKC; ++k) {
                const float *p = lrow + 512 * (int64_t)min(kb0 + k, A.kb - 1);
#pragma unroll
                for (int run = 0; run < 2; ++run) {
                    const cfloatx4 q = *reinterpret_cast<const cfloatx4 *>(p + 4 * run);
#pragma unroll
                    for (int i = 0; i < 4; ++i) x[k][4 * run + i] = q[i];
                }
            }
            return;
        }
        if (kb0 + kKC <= A.kb) {
            const float *p = lrow + 16 * kb0;
            constexpr int ks = 16, rs_ = 8;
#pragma unroll
            for (int k = 0; k < kKC; ++k)
#pragma unroll
                for (int run = 0; run < 2; ++run) {
                    const cfloatx4 q = *reinterpret_cast<const cfloatx4 *>(p + ks * k + rs_ * run);
#pragma unroll
                    for (int i = 0; i < 4; ++i) x[k][4 * run + i] = q[i];
                }
        } else {  // the last, partial stage: blocks past the input are never multiplied
#pragma unroll
            for (int k = 0; k < kKC; ++k) {
                const float *p = lrow + 16 * min(kb0 + k, A.kb - 1);
#pragma unroll
                for (int run = 0; run < 2; ++run) {
                    const cfloatx4 q = *reinterpret_cast<const cfloatx4 *>(p + 8 * run);
#pragma unroll
                    for (int i = 0; i < 4; ++i) x[k][4 * run + i] = q[i];
                }
            }
        }
    };

    // ---- weight stages: stage c = k-blocks [c*kKC, c*kKC + kKC) of this workgroup's NTC tiles,
    // fragment (kbl, i, p) at ((kbl * NTC + i) * NP + p) KB.  Wave w copies fragments w, w + kDW,
    // ...; their source bases are wave-uniform and computed once, so a stage's copies cost a few
    // scalar adds (the lane's 16-byte offset is the copy's only vector operand).
    constexpr int kPer = kKC * kFrag / kDW;
    static_assert(kKC * kFrag % kDW == 0, "fragments per wave");
    const int nst = (A.kb + kKC - 1) / kKC;
    const int64_t plane = (int64_t)A.tiles * A.kb * 64;
    const unsigned loff = (unsigned)lane * 16u;
    const char *fsrc[kPer];
    int fkbl[kPer];
#pragma unroll
    for (int j = 0; j < kPer; ++j) {
        const int f = wave + kDW * j;
        const int kbl = f / kFrag, rem = f - kbl * kFrag;
        const int i = rem / NP, p = rem - NP * i;
        fsrc[j] = reinterpret_cast<const char *>(A.w + p * plane + (int64_t)(ct0 + i) * A.kb * 64);
        fkbl[j] = kbl;
    }
    auto issue_stage = [&](int c) {
        char *buf = stages + (c & 1) * kStage;
#pragma unroll
        for (int j = 0; j < kPer; ++j) {
            const int kb = min(c * kKC + fkbl[j], A.kb - 1);
            dma16(fsrc[j] + (int64_t)kb * 1024 + loff, buf + (wave + kDW * j) * 1024);
        }
    };

    cfloatx16 acc[NTC];
#pragma unroll
    for (int i = 0; i < NTC; ++i)
#pragma unroll
        for (int q = 0; q < 16; ++q) acc[i][q] = 0.f;
    // one stage: wait for stage c, prefetch stage c + 1 (rows into xn, weights by DMA), then
    // the MFMAs of stage c from xc.  Stages alternate between two register sets (no copies).
    auto step = [&](int c, float (&xc)[kKC][8], float (&xn)[kKC][8]) {
        // this wave's rows and weight copies of stage c have landed (issued one stage ago; a
        // real s_waitcnt the compiler's own wait insertion sees), then the barrier: stage c is
        // whole in LDS and buffer (c+1)&1 is free again
        __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0)
        __syncthreads();
        if (c < 12) PN2_DSTAMP(1 + c);
        if (c + 1 < nst) {
            if constexpr (FAST) {
                load_fast(c + 1, xn);
            } else {
#pragma unroll
                for (int k = 0; k < kKC; ++k) load_a((c + 1) * kKC + k, xn[k]);
            }
            issue_stage(c + 1);
        }
        const char *buf = stages + (c & 1) * kStage;
        if (c * kKC + kKC <= A.kb) {
            // a whole stage, branch-free (one basic block for the scheduler).  Reading block
            // k+1's fragments and splitting its rows under block k's MFMAs by hand
            // (sched_group_barrier) measured no faster, and cost registers.
#pragma unroll
            for (int k = 0; k < kKC; ++k) {
                const Split xs = split_scaled<NP>(xc[k], asc.up);
#pragma unroll
                for (int i = 0; i < NTC; ++i)
                    acc[i] = mma_wb<NP>(xs, ring_readN<NP>(buf + (k * kFrag + NP * i) * 1024, lane), acc[i]);
            }
        } else {
#pragma unroll
            for (int k = 0; k < kKC; ++k) {
                if (c * kKC + k < A.kb) {
                    const Split xs = split_scaled<NP>(xc[k], asc.up);
#pragma unroll
                    for (int i = 0; i < NTC; ++i)
                        acc[i] = mma_wb<NP>(xs, ring_readN<NP>(buf + (k * kFrag + NP * i) * 1024, lane), acc[i]);
                }
            }
        }
    };
    float xa[kKC][8], xb[kKC][8];
#pragma unroll
    for (int k = 0; k < kKC; ++k) load_a(k, xa[k]);
    issue_stage(0);
    for (int c = 0; c < nst; c += 2) {
        step(c, xa, xb);
        if (c + 1 < nst) step(c + 1, xb, xa);
    }
    PN2_DSTAMP(14);

    // ---- epilogue: lane = output column, register q = row (q&3) + 8(q>>2) + 4h of the slab
    const int slab_row = row0 + 32 * wave;
    const unsigned G = A.pool ? (unsigned)A.M / (unsigned)A.K : 0u;
#pragma unroll
    for (int i = 0; i < NTC; ++i) {
        const int col = 32 * (ct0 + i) + r;
        const float al = dense_alpha<NP>(A, col, asc.down), be = A.raw ? 0.f : A.beta[col];
        if (!A.pool) {
            unsigned tmax = 0;  // max |value| written (A.out_max)
#pragma unroll
            for (int q = 0; q < 16; ++q) {
                const int row = slab_row + (q & 3) + 8 * (q >> 2) + 4 * h;
                if (row < A.M) {
                    const float y = __builtin_fmaf(acc[i][q], al, be);
                    const float v = A.raw ? acc[i][q] * al : (A.norelu ? y : chain_relu(y));
                    A.out[A.frag_out ? frag_off(row, col, 2 * A.tiles) : (int64_t)row * A.ostride + col] = v;
                    tmax = max(tmax, __float_as_uint(v) & 0x7FFFFFFFu);
                }
            }
            if (A.out_max) {
                const unsigned m = wave_max_u32(tmax);
                if (lane == 0 && slab_row < A.M) A.out_max[(int64_t)(slab_row >> 5) * A.tiles + ct0 + i] = m;
            }
            continue;
        }
        // max over rows of relu(fma(acc, al, be)) = relu(fma(row max (al >= 0) or min, al, be))
        const bool up = al >= 0.f;
        auto fin = [&](float mx, float mn) {
            const float y = __builtin_fmaf(up ? mx : mn, al, be);
            return A.norelu ? y : chain_relu(y);
        };
        if (A.pool_mode == 0) {  // K = 8 or 16: rows 8k..8k+7 are registers 4k..4k+3
            float mx[4], mn[4];
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                mx[k] = fmaxf(fmaxf(acc[i][4 * k], acc[i][4 * k + 1]), fmaxf(acc[i][4 * k + 2], acc[i][4 * k + 3]));
                mn[k] = fminf(fminf(acc[i][4 * k], acc[i][4 * k + 1]), fminf(acc[i][4 * k + 2], acc[i][4 * k + 3]));
                mx[k] = max_halves(mx[k]);
                mn[k] = min_halves(mn[k]);
            }
            if (h == 0) {
                const int per = A.K / 8;  // register groups per output group
#pragma unroll
                for (int k = 0; k < 4; k += 1) {
                    if (k % per) continue;
                    float a = mx[k], z = mn[k];
                    if (per == 2) a = fmaxf(a, mx[k + 1]), z = fminf(z, mn[k + 1]);
                    const unsigned gg = (unsigned)(slab_row + 8 * k) / (unsigned)A.K;
                    if (gg < G) A.out[(int64_t)gg * A.ostride + col] = fin(a, z);
                }
            }
            continue;
        }
        if (A.pool_mode == 2 && (slab_row + 31 >= A.M || (unsigned)slab_row / (unsigned)A.K !=
                                                             (unsigned)(slab_row + 31) / (unsigned)A.K)) {
            // K % 32 != 0: this slab straddles a group boundary or the end of the rows (whose
            // zero-filled rows must not pool) -- one atomic per valid row
#pragma unroll
            for (int q = 0; q < 16; ++q) {
                const int row = slab_row + (q & 3) + 8 * (q >> 2) + 4 * h;
                if (row < A.M) {
                    const float m = fin(acc[i][q], acc[i][q]);
                    atomicMax(reinterpret_cast<unsigned *>(A.out + (int64_t)((unsigned)row / (unsigned)A.K) * A.ostride + col),
                              A.norelu ? fkey(m) : __float_as_uint(m));
                }
            }
            continue;
        }
        float mx = acc[i][0], mn = acc[i][0];
#pragma unroll
        for (int q = 1; q < 16; ++q) {
            mx = fmaxf(mx, acc[i][q]);
            mn = fminf(mn, acc[i][q]);
        }
        const float m = fin(max_halves(mx), min_halves(mn));
        // ReLU output >= +0: its bits order as uints; signed (norelu) values go through fkey
        const unsigned mk = A.norelu ? fkey(m) : __float_as_uint(m);
        if (h == 0 && slab_row < A.M) {
            const unsigned gg = (unsigned)slab_row / (unsigned)A.K;
            if (A.pool_mode == 1)
                atomicMax(reinterpret_cast<unsigned *>(opool) + ((int)gg - row0 / A.K) * ncols + 32 * i + r, mk);
            else
                atomicMax(reinterpret_cast<unsigned *>(A.out + (int64_t)gg * A.ostride + col), mk);
        }
    }
    if (A.pool && A.pool_mode == 1) {
        __syncthreads();
        for (int e = tid; e < gpb * ncols; e += 64 * kDW) {
            const int gl = e / ncols, c = e - gl * ncols;
            const unsigned gg = (unsigned)(row0 / A.K + gl);
            if (gg < G)
                A.out[(int64_t)gg * A.ostride + 32 * ct0 + c] =
                    A.norelu ? funkey(__float_as_uint(opool[e])) : opool[e];
        }
    }
    PN2_DSTAMP(15);
}

template <int NTC, int NP, int NW = 4>
static int launch_dense_split(const DenseSplitArgs &A, hipStream_t st) {
    constexpr int kDW = NW, kDRows = 32 * NW;
    // every k-block after the first stage is one contiguous 16-channel run of the row
    const bool fast = A.vec && (A.mode == 0 ? A.cin % 16 == 0 && A.kb * 16 == A.cin
                                            : A.feat && A.D > 0 && A.D % 16 == 0 && A.kb == 1 + A.D / 16);
    const size_t lds = (size_t)2 * kKC * NP * NTC * 1024 +
                       (A.pool_mode == 1 ? (size_t)(kDRows / A.K) * 32 * NTC * 4 : 0);
    dim3 grid((unsigned)((A.M + kDRows - 1) / kDRows), (unsigned)(A.tiles / NTC));
    if (lds > 64 * 1024) {  // NTC = 4: two 48 KB weight stages (one-time, idempotent)
        static const hipError_t a1 = hipFuncSetAttribute(
            reinterpret_cast<const void *>(&dense_split_kernel<NTC, NP, true, NW>),
            hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
        static const hipError_t a2 = hipFuncSetAttribute(
            reinterpret_cast<const void *>(&dense_split_kernel<NTC, NP, false, NW>),
            hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
        (void)a1;
        (void)a2;
    }
    if (fast) hipLaunchKernelGGL((dense_split_kernel<NTC, NP, true, NW>), grid, dim3(64 * kDW), lds, st, A);
    else hipLaunchKernelGGL((dense_split_kernel<NTC, NP, false, NW>), grid, dim3(64 * kDW), lds, st, A);
    PN2_LAUNCH_CHECK("dense_split_kernel");
    return PN2_OK;
}

// ------------------------------------------------------------------ LDS-staged dense layer
// The same layer with BOTH operands staged in LDS by global_load_lds: the A rows as whole
// 128-byte lines (32 fp32 channels per row and stage) instead of two 16-byte pieces per lane
// from 32 different rows (the pattern that bounded dense_split_kernel's stages: its load stage
// alone took 1.7 of its ~2.5 us, tools/micro/row_loads.hip), and the B fragments as before.
// Tiles are TR x TC = 32*WR x 32*NTW with WR waves; wave w computes rows 32w.. x every column
// of the tile (NTW 32-column MFMA tiles), so each A element is split into its bf16 planes once
// per workgroup -- the split is the VALU cost that competes with the MFMAs for issue slots.
// An NS-stage ring (stage = 32 input channels) keeps NS-2 stages' DMA in flight: a counted
// vmcnt and a raw s_barrier per stage, never vmcnt(0) inside the loop.
//
// A's LDS image is [TR rows][8 chunks of 16 B]; chunk c of row r is stored at c ^ ((r>>1) & 7)
// (DMA writes lane-linearly, so the swizzle is on the source address): the two ds_read_b128 of
// an A fragment (chunks 4kb+h and 4kb+2+h of 32 consecutive rows) then cover all 64 banks in
// every 16-lane group of the b128 read (conflict-free for gfx950's lane grouping; SQ counters:
// no bank conflicts).
//
// Sources: rows mode (dense fp32 rows, row stride rs, cin % 32 == 0, 16-byte aligned) and
// group_all (block 0 = xyz of the point, read straight into registers before the loop; then
// the features, D % 32 == 0).  Epilogue as dense_split_kernel (raw / BN + ReLU / no-ReLU, and
// pools over K rows when K % 32 == 0 and K divides TR or TR divides K).  Every product and
// accumulation is the one dense_split_kernel computes, in the same k order: the same bits.
// (LDS keeps one workgroup of 8 waves, or 2-4 waves, per CU: the register file allows up to 256
// VGPRs per wave, and the scheduler may use them to issue a stage's fragment reads early)
template <int WR, int NTW, int NP, int NS>
__global__ __launch_bounds__(64 * WR) __attribute__((amdgpu_waves_per_eu(WR == 8 ? 2 : 1, WR == 8 ? 2 : 1)))
void dense_lds_kernel(const DenseSplitArgs A) {
    constexpr int NW = WR;
    constexpr int TR = 32 * WR, TC = 32 * NTW, NT = NTW;
    constexpr int kAStage = TR * 128;             // TR rows x 32 channels x 4 B
    constexpr int kBStage = 2 * NT * NP * 1024;   // 2 k-blocks x NT tiles x NP planes
    constexpr int kStage = kAStage + kBStage;
    constexpr int kAIns = kAStage / 1024, kIns = kAIns + kBStage / 1024;  // DMA per stage
    constexpr int kMaxPer = (kIns + NW - 1) / NW;
    extern __shared__ __attribute__((aligned(16))) char lsm[];
    PN2_DSTAMP(0);
    PN2_DCLOCK(16);
    const int tid = threadIdx.x;
    const int lane = tid & 63;
    const int r = lane & 31, h = lane >> 5;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    // this wave's DMA instructions per stage: i = wave + NW j < kIns (the first kIns % NW
    // waves issue one more)
    const bool more = kIns % NW != 0 && wave < kIns % NW;
    const unsigned ntile = (unsigned)(A.tiles / NT);
    unsigned rbi, cti;  // row block, column tile
    if (A.xcx > 0) {
        // dispatch deals workgroup i to XCD i % 8: XCD x gets a rectangle of row blocks x column
        // tiles, so its L2 holds a share of both operands
        const unsigned x = blockIdx.x & 7u, i = blockIdx.x >> 3;
        const unsigned cx = (unsigned)A.xcx, nr = gridDim.x / ntile;
        const unsigned rpx = nr / (8u / cx), cpx = ntile / cx;
        rbi = (x / cx) * rpx + i / cpx;
        cti = (x % cx) * cpx + i % cpx;
    } else {
        const unsigned lid = xcd_contiguous(blockIdx.x, gridDim.x);
        rbi = lid / ntile;
        cti = lid % ntile;
    }
    const int row0 = (int)rbi * TR;
    const int ct0 = (int)cti * NT;  // first 32-column tile of the workgroup
    if (A.zero) {  // a side job: the next layer's pool, or the caller's zero_out
        const int64_t tot = A.zrows * A.zcols, nwg = gridDim.x;
        const int64_t per = (tot + nwg - 1) / nwg, e0 = (int64_t)blockIdx.x * per;
        const int64_t e1 = e0 + per < tot ? e0 + per : tot;
        for (int64_t e = e0 + tid; e < e1; e += 64 * NW) {
            const int64_t g = e / A.zcols;
            A.zero[g * A.zstride + (e - g * A.zcols)] = 0.f;
        }
    }
    const int kb0 = A.mode == 1 ? 1 : 0;        // group_all: block 0 = xyz (registers)
    const int nst = (A.kb - kb0) / 2;           // 32-channel stages

    // ---- this lane's DMA sources.  A instruction i < kAIns covers tile rows 8i .. 8i+7: lane l
    // -> row + (l >> 3), LDS chunk l & 7, source chunk (l & 7) ^ ((row >> 1) & 7).  B
    // instruction i >= kAIns is fragment f = i - kAIns = (kbl * NT + t) * NP + p of the stage.
    const int64_t plane = (int64_t)A.tiles * A.kb * 64;
    const unsigned loff = (unsigned)lane * 16u;
    const char *src[kMaxPer];
    int64_t step[kMaxPer];  // source bytes per stage
#pragma unroll
    for (int j = 0; j < kMaxPer; ++j) {
        const int i = min(wave + NW * j, kIns - 1);
        if (i < kAIns) {
            const int tr = 8 * i + (lane >> 3);
            const int R = min(row0 + tr, A.M - 1);  // rows past M: any valid row, never stored
            const int chunk = (lane & 7) ^ ((tr >> 1) & 7);
            const float *base;
            if (A.mode == 0) {
                base = A.rows + (int64_t)R * A.rs;
            } else {
                const int b = R / A.N, n = R - b * A.N;
                base = A.feat + (int64_t)b * A.fb + (int64_t)n * A.fn;
            }
            src[j] = reinterpret_cast<const char *>(base + 4 * chunk);
            step[j] = 32 * 4;
        } else {
            const int f = i - kAIns;
            const int p = f % NP, t = (f / NP) % NT, kbl = f / (NP * NT);
            src[j] = reinterpret_cast<const char *>(A.w + p * plane + ((int64_t)(ct0 + t) * A.kb + kb0 + kbl) * 64) + loff;
            step[j] = 2 * 1024;
        }
    }
    auto issue = [&](int st) {
        char *buf = lsm + (st % NS) * kStage;
#pragma unroll
        for (int j = 0; j < kMaxPer; ++j) {
            const int i = wave + NW * j;
            if (j < kMaxPer - 1 || kIns % NW == 0 || more)
                dma16(src[j] + st * step[j], buf + i * 1024);
        }
    };

    cfloatx16 acc[NT];
#pragma unroll
    for (int i = 0; i < NT; ++i)
#pragma unroll
        for (int q = 0; q < 16; ++q) acc[i][q] = 0.f;

#pragma unroll
    for (int s = 0; s < NS - 1; ++s)
        if (s < nst) issue(s);
    const int trow = 32 * wave + r;  // this lane's tile row (A fragment)
    const ActScale asc = dense_act_scale<NP>(A, (row0 >> 5) + wave, lane);
    if (A.mode == 1) {
        // block 0: raw xyz of the point (sample_and_group_all does not centre), and its
        // fragments straight from L2
        const int R = min(row0 + trow, A.M - 1);
        const int b = R / A.N, n = R - b * A.N;
        const float *prow = A.pts + (int64_t)b * A.pb + (int64_t)n * A.pn;
        float x[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            const int ch = (j & 3) + 8 * (j >> 2) + 4 * h;
            x[j] = ch < A.C ? prow[(int64_t)ch * A.pc] : 0.f;
        }
        const Split xs = split_scaled<NP>(x, asc.up);
#pragma unroll
        for (int i = 0; i < NT; ++i) {
            const bf16x8 *wq = A.w + (int64_t)(ct0 + i) * A.kb * 64 + lane;
            Split w;
            w.h = wq[0];
            w.m = NP >= 2 ? wq[plane] : w.h;
            w.l = NP == 3 ? wq[2 * plane] : w.h;
            acc[i] = mma_wb<NP>(xs, w, acc[i]);
        }
    }
    const int swz = (trow >> 1) & 7;
    constexpr int kLo = kIns / NW, kHi = kLo + (kIns % NW ? 1 : 0);
    // the epilogue's BN scale / shift, loaded now (their latency hides under the main loop)
    float eal[NT], ebe[NT];
#pragma unroll
    for (int i = 0; i < NT; ++i) {
        const int col = 32 * (ct0 + i) + r;
        eal[i] = dense_alpha<NP>(A, col, asc.down);
        ebe[i] = A.raw ? 0.f : A.beta[col];
    }
    // ---- main loop, software-pipelined across stages.  Without it both waves of a SIMD left
    // each barrier together and split their A fragments together, with the matrix pipe idle
    // (the stage's arithmetic alone ran at ~55 % of its MFMA time, tools/debug/dense_stamps.py
    // on a no-DMA build).  Now stage st's k-block 0 MFMAs are issued first; behind them the
    // wave passes the barrier of stage st+1, issues its reads and splits its A fragments
    // under stage st's k-block 1 MFMAs.  Stage st+NS overwrites stage st's buffer: every wave's
    // reads of it returned before it reached the barrier of stage st+1.
    // this wave's DMA of stage s has landed, `y` younger stages may stay in flight
    auto wait_dma = [&](int y) {
        if (y >= 2) {
            if (more) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(2 * kHi) : "memory");
            else asm volatile("s_waitcnt vmcnt(%0)" ::"n"(2 * kLo) : "memory");
        } else if (y == 1) {
            if (more) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(kHi) : "memory");
            else asm volatile("s_waitcnt vmcnt(%0)" ::"n"(kLo) : "memory");
        } else {
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        }
    };
    struct Frags {
        cfloatx4 a[2][2];
        Split b[2][NT];
    };
    // the stage's fragments, all reads issued together (A first: its split is the first use)
    auto read_stage = [&](int st, Frags &f) {
        const char *buf = lsm + (st % NS) * kStage;
        const char *arow = buf + trow * 128;
#pragma unroll
        for (int kbl = 0; kbl < 2; ++kbl) {
            f.a[kbl][0] = *reinterpret_cast<const cfloatx4 *>(arow + (((4 * kbl + h) ^ swz) << 4));
            f.a[kbl][1] = *reinterpret_cast<const cfloatx4 *>(arow + (((4 * kbl + 2 + h) ^ swz) << 4));
        }
#pragma unroll
        for (int kbl = 0; kbl < 2; ++kbl)
#pragma unroll
            for (int i = 0; i < NT; ++i) f.b[kbl][i] = ring_readN<NP>(buf + kAStage + ((kbl * NT + i) * NP) * 1024, lane);
    };
    auto split_stage = [&](const Frags &f, Split (&xs)[2]) {
#pragma unroll
        for (int kbl = 0; kbl < 2; ++kbl) {
            float x[8];
#pragma unroll
            for (int i = 0; i < 4; ++i) x[i] = f.a[kbl][0][i], x[4 + i] = f.a[kbl][1][i];
            xs[kbl] = split_scaled<NP>(x, asc.up);
        }
    };
    auto mfma_kb = [&](const Split &xs, const Frags &f, int kbl) {
#pragma unroll
        for (int i = 0; i < NT; ++i) acc[i] = mma_wb<NP>(xs, f.b[kbl][i], acc[i]);
    };
    // barrier of stage s (its DMA landed everywhere, stage s-1's buffer is free) + the DMA of
    // stage s+NS-1 into it
    auto enter_stage = [&](int s) {
        wait_dma(min(NS - 2, nst - 1 - s));
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        stage_barrier();
        if (s < 12) PN2_DSTAMP(1 + s);
        if (s + NS - 1 < nst) issue(s + NS - 1);
    };
    // one stage with the next one's entry, reads and split behind its MFMAs
    auto stage_step = [&](int st, const Frags &cur, const Split (&xc)[2], Frags &nxt, Split (&xn)[2]) {
        mfma_kb(xc[0], cur, 0);
        enter_stage(st + 1);
        read_stage(st + 1, nxt);
        mfma_kb(xc[1], cur, 1);
        split_stage(nxt, xn);
    };
    if (nst > 0) {
        Frags fa, fb;
        Split xa[2], xb[2];
        enter_stage(0);
        read_stage(0, fa);
        split_stage(fa, xa);
        int st = 0;
        for (; st + 2 < nst; st += 2) {
            stage_step(st, fa, xa, fb, xb);
            stage_step(st + 1, fb, xb, fa, xa);
        }
        if (st + 1 < nst) {
            stage_step(st, fa, xa, fb, xb);
            mfma_kb(xb[0], fb, 0);
            mfma_kb(xb[1], fb, 1);
        } else {
            mfma_kb(xa[0], fa, 0);
            mfma_kb(xa[1], fa, 1);
        }
    }
    __syncthreads();  // the stage buffers are free again (the pool below reuses them)
    PN2_DSTAMP(14);

    // ---- epilogue: lane = output column, register q = row (q&3) + 8(q>>2) + 4h of the slab
    const int slab_row = row0 + 32 * wave;
    const unsigned G = A.pool ? (unsigned)A.M / (unsigned)A.K : 0u;
    const bool lds_pool = A.pool && TR % A.K == 0;
    const int gpb = lds_pool ? TR / A.K : 0;
    unsigned *opool = reinterpret_cast<unsigned *>(lsm);  // [gpb][TC]
    if (lds_pool) {
        for (int e = tid; e < gpb * TC; e += 64 * NW) opool[e] = 0u;
        __syncthreads();
    }
#pragma unroll
    for (int i = 0; i < NT; ++i) {
        const int lcol = 32 * i + r;
        const int col = 32 * ct0 + lcol;
        const float al = eal[i], be = ebe[i];
        if (!A.pool) {
            unsigned tmax = 0;  // max |value| written (A.out_max)
#pragma unroll
            for (int q = 0; q < 16; ++q) {
                const int row = slab_row + (q & 3) + 8 * (q >> 2) + 4 * h;
                if (row < A.M) {
                    const float y = __builtin_fmaf(acc[i][q], al, be);
                    const float v = A.raw ? acc[i][q] * al : (A.norelu ? y : chain_relu(y));
                    A.out[A.frag_out ? frag_off(row, col, 2 * A.tiles) : (int64_t)row * A.ostride + col] = v;
                    tmax = max(tmax, __float_as_uint(v) & 0x7FFFFFFFu);
                }
            }
            if (A.out_max) {
                const unsigned m = wave_max_u32(tmax);
                if (lane == 0 && slab_row < A.M) A.out_max[(int64_t)(slab_row >> 5) * A.tiles + ct0 + i] = m;
            }
            continue;
        }
        // max over rows of relu(fma(acc, al, be)) = relu(fma(row max (al >= 0) or min, al, be))
        float mx = acc[i][0], mn = acc[i][0];
#pragma unroll
        for (int q = 1; q < 16; ++q) {
            mx = fmaxf(mx, acc[i][q]);
            mn = fminf(mn, acc[i][q]);
        }
        mx = max_halves(mx);
        mn = min_halves(mn);
        const float y = __builtin_fmaf(al >= 0.f ? mx : mn, al, be);
        const float m = A.norelu ? y : chain_relu(y);
        // ReLU output >= +0: its bits order as uints; signed (norelu) values go through fkey
        const unsigned mk = A.norelu ? fkey(m) : __float_as_uint(m);
        if (h == 0 && slab_row < A.M) {
            const unsigned gg = (unsigned)slab_row / (unsigned)A.K;
            if (lds_pool)
                atomicMax(opool + ((int)gg - row0 / A.K) * TC + lcol, mk);
            else
                atomicMax(reinterpret_cast<unsigned *>(A.out + (int64_t)gg * A.ostride + col), mk);
        }
    }
    if (lds_pool) {
        __syncthreads();
        for (int e = tid; e < gpb * TC; e += 64 * NW) {
            const int gl = e / TC, c = e - gl * TC;
            const unsigned gg = (unsigned)(row0 / A.K + gl);
            if (gg < G)
                A.out[(int64_t)gg * A.ostride + 32 * ct0 + c] =
                    A.norelu ? funkey(opool[e]) : __uint_as_float(opool[e]);
        }
    }
    PN2_DSTAMP(15);
    PN2_DCLOCK(17);
}

// Tiles of the LDS-staged kernel, as WR * 10 + NTW (rows 32 WR, columns 32 NTW): the first that
// leaves a workgroup per CU -- 256 x 64 (8 waves, 2 per SIMD), 128 x 128 (4 waves), 128 x 64,
// 64 x 64 -- and pools (0: not eligible).  Tuning dense_lds_tile forces one.
static const int kLdsTiles[] = {82, 44, 42, 22};

static int dense_lds_tile(const DenseSplitArgs &A) {
    if (!tuning().dense_lds || !A.vec) return 0;
    if (tuning().dense_lds == 2 && A.mode == 0) return 0;  // 2: group_all / pre-pass layers only
    // tuning dense_lds_mincin keeps narrower layers on the register-staged kernel (default 0:
    // none -- SSG eager 67.6k at 0 or 128 vs 66.6k at 256, PointNet-v1 equal or faster,
    // tools/gpu_r04af.sh)
    if ((A.mode == 0 ? A.cin : A.D) < tuning().dense_lds_mincin) return 0;
    const bool ok = A.mode == 0 ? (A.cin % 32 == 0 && A.kb * 16 == A.cin && A.rs % 4 == 0 &&
                                   ((uintptr_t)A.rows & 15) == 0)
                                : (A.feat && A.D > 0 && A.D % 32 == 0 && A.kb == 1 + A.D / 16 &&
                                   A.fn % 4 == 0 && A.fb % 4 == 0 && ((uintptr_t)A.feat & 15) == 0);
    if (!ok) return 0;
    auto fits = [&](int t) {
        const int tr = 32 * (t / 10), ntw = t % 10;
        return A.tiles % ntw == 0 && (!A.pool || (A.K % 32 == 0 && (tr % A.K == 0 || A.K % tr == 0)));
    };
    if (const int64_t f = tuning().dense_lds_tile) return fits((int)f) ? (int)f : 0;
    for (int t : kLdsTiles) {
        const int tr = 32 * (t / 10), ntw = t % 10;
        if (fits(t) && (A.M + tr - 1) / tr * (A.tiles / ntw) >= 256) return t;
    }
    return fits(22) ? 22 : 0;
}

template <int WR, int NTW, int NP, int NS>
static int launch_dense_lds_ns(DenseSplitArgs A, hipStream_t st) {
    constexpr int TR = 32 * WR, NT = NTW;
    const size_t stage = (size_t)TR * 128 + (size_t)2 * NT * NP * 1024;
    const size_t pool = A.pool && TR % A.K == 0 ? (size_t)(TR / A.K) * 32 * NT * 4 : 0;
    const size_t lds = std::max((size_t)NS * stage, pool);
    static const hipError_t attr = hipFuncSetAttribute(
        reinterpret_cast<const void *>(&dense_lds_kernel<WR, NTW, NP, NS>),
        hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    (void)attr;
    const int64_t nr = (A.M + TR - 1) / TR, nc = A.tiles / NT;
    // XCD rectangles: the column split cx (1, 2, 4, 8) that holds the fewest operand bytes per
    // XCD, when the grid divides evenly (tuning dense_lds_xcd2d = 0: whole row blocks per XCD)
    A.xcx = 0;
    if (tuning().dense_lds_xcd2d && (nr * nc) % 8 == 0) {
        const int64_t abytes = (int64_t)TR * A.kb * 64, bbytes = (int64_t)32 * NT * A.kb * 16 * 2 * NP;
        int64_t best = -1;
        for (int cx = 1; cx <= 8; cx *= 2) {
            if (nc % cx || nr % (8 / cx)) continue;
            const int64_t b = nr / (8 / cx) * abytes + nc / cx * bbytes;
            if (best < 0 || b < best) best = b, A.xcx = cx;
        }
    }
    hipLaunchKernelGGL((dense_lds_kernel<WR, NTW, NP, NS>), dim3((unsigned)(nr * nc)), dim3(64 * WR), lds, st, A);
    PN2_LAUNCH_CHECK("dense_lds_kernel");
    return PN2_OK;
}

// ring depth: tuning dense_lds_stages (2, 3 or 4; 4 only where four stages fit the CU's LDS)
template <int WR, int NTW, int NP>
static int launch_dense_lds(const DenseSplitArgs &A, hipStream_t st) {
    constexpr size_t stage = (size_t)32 * WR * 128 + (size_t)2 * NTW * NP * 1024;
    if constexpr (4 * stage <= 160 * 1024)
        if (tuning().dense_lds_stages >= 4) return launch_dense_lds_ns<WR, NTW, NP, 4>(A, st);
    if (tuning().dense_lds_stages <= 2) return launch_dense_lds_ns<WR, NTW, NP, 2>(A, st);
    return launch_dense_lds_ns<WR, NTW, NP, 3>(A, st);
}

static int launch_dense_lds_tile(int tile, const DenseSplitArgs &A, int np, hipStream_t st) {
#define PN2_LDS_NP(WR, NTW) \
    (np == 3 ? launch_dense_lds<WR, NTW, 3>(A, st) : np == 2 ? launch_dense_lds<WR, NTW, 2>(A, st) \
             : launch_dense_lds<WR, NTW, 1>(A, st))
    switch (tile) {
        case 82: return PN2_LDS_NP(8, 2);
        case 44: return PN2_LDS_NP(4, 4);
        case 42: return PN2_LDS_NP(4, 2);
        default: return PN2_LDS_NP(2, 2);
    }
#undef PN2_LDS_NP
}

// ------------------------------------------------------------------ fused group_all layer pair
// The first two layers of a group_all MLP (sa3: [xyz | 256 features] -> 256 -> 512) in one
// launch, the 256-wide intermediate never leaving the CU.  Taken one per launch, those two
// layers are each ~6 us of fixed cost (the first DMA's latency, the store drain at the end)
// around 5-7 us of stages (tools/debug/dense_stamps.py SEL=1008 / 16).
// Workgroup = one 32-row block x one of `cs` column slices of the second layer, 8 waves:
//   1. the block's layer-0 A operand split once into LDS planes [kb][NP0][64 lanes][16 B]
//      (wave w loads all of its k-blocks w, w + 8, ... at once, then splits them; NP0 = 2, the
//      split-fp16 first layer of dense_f16 = 2: after the block's scale is reduced over the
//      waves through LDS);
//   2. wave w: layer-0 column tile w over every k-block, its weight fragments streamed straight
//      into registers RD k-blocks ahead (nothing else to share: each wave has its own tile);
//   3. BN + ReLU in registers; the block's max |value| (the maxima the unfused layer 0 would
//      leave for layer 1) through LDS; every value split (elementwise, scaled for NP1 = 2) and
//      written into layer 1's A planes, which replace layer 0's;
//   4. wave w: layer-1 column tile (slice * 8 + w), weights streamed the same way (its first
//      k-blocks already requested behind step 2), epilogue as dense_lds_kernel's (rows or
//      fragment order, out_max for layer 2).
// Layer 0 is computed once per slice (cs = 2 for 512 outputs: 256 workgroups at SSG's 4096
// rows).  Products, accumulation order, scales and epilogues are the unfused layers': the same
// bits (tests/test_gpu_mlp.py).
template <int NP>
__device__ __forceinline__ Split load_wfrag(const bf16x8 *wq, int64_t plane) {
    Split w;
    w.h = wq[0];
    w.m = NP >= 2 ? wq[plane] : w.h;
    w.l = NP == 3 ? wq[2 * plane] : w.h;
    return w;
}

#ifndef PN2_PAIR_RD
#define PN2_PAIR_RD 4
#endif
constexpr int kPairWaves = 8, kPairRD = PN2_PAIR_RD;  // k-blocks of weights in flight per wave

template <int NP0, int NP1, int KB0>
__global__ __launch_bounds__(64 * kPairWaves) void dense_pair_kernel(const DenseSplitArgs A0, const DenseSplitArgs A1,
                                                                     int cs) {
    // k-block counts are compile-time (layer 1's input is layer 0's 8 tiles): fully unrolled,
    // branch-free weight streams whose vmcnt waits the compiler counts exactly
    constexpr int NW = kPairWaves, RD = kPairRD, KB1 = 2 * kPairWaves;
    const DenseSplitArgs &A = A0;  // the stamps' launch selection (diagnostic builds)
    (void)A;
    PN2_DSTAMP(0);
    extern __shared__ __attribute__((aligned(16))) char psm[];
    unsigned *smax = reinterpret_cast<unsigned *>(psm);  // [NW] layer-0 tile maxima, [NW] A maxima
    char *planes = psm + 64;
    const int tid = threadIdx.x;
    const int lane = tid & 63;
    const int r = lane & 31, h = lane >> 5;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const unsigned lid = xcd_contiguous(blockIdx.x, gridDim.x);
    const int rb = (int)(lid / (unsigned)cs), slice = (int)(lid % (unsigned)cs);
    const int row0 = 32 * rb;
    const int M = A0.M;
    if (A1.zero) {  // side job: the next layer's pool
        const int64_t tot = A1.zrows * A1.zcols, nwg = gridDim.x;
        const int64_t per = (tot + nwg - 1) / nwg, e0 = (int64_t)blockIdx.x * per;
        const int64_t e1 = e0 + per < tot ? e0 + per : tot;
        for (int64_t e = e0 + tid; e < e1; e += 64 * NW) {
            const int64_t g = e / A1.zcols;
            A1.zero[g * A1.zstride + (e - g * A1.zcols)] = 0.f;
        }
    }
    constexpr int kb0n = KB0, kb1n = KB1;
    const int64_t plane0 = (int64_t)A0.tiles * kb0n * 64, plane1 = (int64_t)A1.tiles * kb1n * 64;
    const bf16x8 *w0 = A0.w + (int64_t)wave * kb0n * 64 + lane;
    const int t1 = slice * NW + wave;
    const bf16x8 *w1 = A1.w + (int64_t)t1 * kb1n * 64 + lane;
    // both epilogues' BN scale / shift, loaded first (a load behind the weight stream would wait
    // for all of it); layer 1's scale still lacks the activation down-scale (dense_alpha's last
    // factor)
    const int col0 = 32 * wave + r, col1 = 32 * t1 + r;
    const float pa0 = NP0 == 2 ? (A0.raw ? 1.f : A0.alpha[col0]) * A0.wscale[col0] : dense_alpha<NP0>(A0, col0, 1.f);
    const float be0 = A0.raw ? 0.f : A0.beta[col0];
    const float pa1 = NP1 == 2 ? (A1.raw ? 1.f : A1.alpha[col1]) * A1.wscale[col1] : dense_alpha<NP1>(A1, col1, 1.f);
    const float be1 = A1.raw ? 0.f : A1.beta[col1];

    // ---- 1. layer-0 A planes: this wave's k-blocks w, w + 8, ... all requested at once, then
    // the layer-0 weights' first RD k-blocks behind them, then the splits
    constexpr int PER = (KB0 + NW - 1) / NW;
    float xa[PER][8];
    {
        const int R = min(row0 + r, M - 1);  // rows past M: any valid row, never stored
        const int b = R / A0.N, n = R - b * A0.N;
#pragma unroll
        for (int i = 0; i < PER; ++i) {
            const int kb = wave + NW * i;
            if (kb == 0) {  // raw xyz (sample_and_group_all does not centre)
                const float *prow = A0.pts + (int64_t)b * A0.pb + (int64_t)n * A0.pn;
#pragma unroll
                for (int j = 0; j < 8; ++j) {
                    const int ch = (j & 3) + 8 * (j >> 2) + 4 * h;
                    xa[i][j] = ch < A0.C ? prow[(int64_t)ch * A0.pc] : 0.f;
                }
            } else if (kb < kb0n) {
                const float *f = A0.feat + (int64_t)b * A0.fb + (int64_t)n * A0.fn + 16 * (kb - 1) + 4 * h;
                const cfloatx4 q0 = *reinterpret_cast<const cfloatx4 *>(f);
                const cfloatx4 q1 = *reinterpret_cast<const cfloatx4 *>(f + 8);
#pragma unroll
                for (int j = 0; j < 4; ++j) xa[i][j] = q0[j], xa[i][4 + j] = q1[j];
            }
        }
    }
    Split wb[RD];
#pragma unroll
    for (int i = 0; i < RD; ++i)
        if (i < kb0n) wb[i] = load_wfrag<NP0>(w0 + i * 64, plane0);
    // NP0 = 2 (split fp16 first layer): the block's scale from the max |value| of its 32 rows'
    // [xyz | features] -- the unfused layer's dense_act_scale, reduced here over the waves'
    // k-blocks through LDS (rows past M are copies of row M - 1, which is in the block)
    ActScale asc0{1.f, 1.f};
    if constexpr (NP0 == 2) {
        unsigned m = 0;
#pragma unroll
        for (int i = 0; i < PER; ++i)
            if (wave + NW * i < kb0n)
#pragma unroll
                for (int j = 0; j < 8; ++j) m = max(m, abs_bits(xa[i][j]));
        m = wave_max_u32(m);
        unsigned *amax = smax + NW;
        if (lane == 0) amax[wave] = m;
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        stage_barrier();
        m = 0;
#pragma unroll
        for (int i = 0; i < NW; ++i) m = max(m, amax[i]);
        asc0 = act_scale(__uint_as_float(m));
    }
    const float al0 = NP0 == 2 ? pa0 * asc0.down : pa0;
#pragma unroll
    for (int i = 0; i < PER; ++i) {
        const int kb = wave + NW * i;
        if (kb < kb0n) {
            const Split sp = split_scaled<NP0>(xa[i], asc0.up);
            bf16x8 *dst = reinterpret_cast<bf16x8 *>(planes + kb * NP0 * 1024) + lane;
            dst[0] = sp.h;
            if (NP0 >= 2) dst[64] = sp.m;
            if (NP0 == 3) dst[128] = sp.l;
        }
    }
    // barriers without __syncthreads' vmcnt(0): the weight prefetches stay in flight
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    stage_barrier();
    PN2_DSTAMP(1);

    // ---- 2. layer 0, tile `wave`
    cfloatx16 acc;
#pragma unroll
    for (int q = 0; q < 16; ++q) acc[q] = 0.f;
    // per k-block, in this order (sched_barrier: the scheduler would sink the weight requests
    // under the MFMAs and leave one or two in flight): the next k-block's A planes from LDS,
    // this k-block's MFMAs, the request RD k-blocks ahead into the register just consumed
    Split xb[2];  // A planes double-buffered in registers (static indices: the loop is unrolled)
    xb[0] = ring_readN<NP0>(planes, lane);
#pragma unroll
    for (int kb = 0; kb < kb0n; ++kb) {
        if (kb + 1 < kb0n) xb[(kb + 1) & 1] = ring_readN<NP0>(planes + (kb + 1) * NP0 * 1024, lane);
        __builtin_amdgcn_sched_barrier(0);  // the reads first: a full k-block of MFMAs to land
        acc = mma_wb<NP0>(xb[kb & 1], wb[kb % RD], acc);
        if (kb + RD < kb0n) wb[kb % RD] = load_wfrag<NP0>(w0 + (int64_t)(kb + RD) * 64, plane0);
        __builtin_amdgcn_sched_barrier(0);
    }
    PN2_DSTAMP(2);
    // layer-1 weights: the first RD k-blocks requested behind layer 0's MFMAs
    Split wc[RD];
#pragma unroll
    for (int i = 0; i < RD; ++i) wc[i] = load_wfrag<NP1>(w1 + i * 64, plane1);

    // ---- 3. layer-0 epilogue -> layer-1 A planes
    float v[16];
    unsigned tmax = 0;
#pragma unroll
    for (int q = 0; q < 16; ++q) {
        const int row = row0 + (q & 3) + 8 * (q >> 2) + 4 * h;
        const float y = __builtin_fmaf(acc[q], al0, be0);
        v[q] = A0.raw ? acc[q] * al0 : (A0.norelu ? y : chain_relu(y));
        if (row < M) tmax = max(tmax, __float_as_uint(v[q]) & 0x7FFFFFFFu);
    }
    tmax = wave_max_u32(tmax);
    if (lane == 0) smax[wave] = tmax;
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    stage_barrier();  // the maxima are in; every wave's layer-0 plane reads returned
    PN2_DSTAMP(3);
    ActScale asc{1.f, 1.f};
    if constexpr (NP1 == 2) {
        unsigned m = 0;
#pragma unroll
        for (int i = 0; i < NW; ++i) m = max(m, smax[i]);
        asc = act_scale(__uint_as_float(m));
    }
    {
        // element (row, col) of the block -> layer-1 k-block col / 16, lane (row & 31) + 32 h',
        // element j of that lane's 8 (channel c = col % 16 = (j & 3) + 8 (j >> 2) + 4 h')
        const int kb = col0 >> 4, c = col0 & 15;
        const int hh = (c >> 2) & 1, j = (c & 3) + 4 * (c >> 3);
        char *base = planes + kb * NP1 * 1024 + 32 * hh * 16 + j * 2;
#pragma unroll
        for (int q = 0; q < 16; ++q) {
            const int rr = (q & 3) + 8 * (q >> 2) + 4 * h;
            char *p = base + rr * 16;
            if constexpr (NP1 == 2) {
                const float y = v[q] * asc.up;
                const _Float16 a = (_Float16)y;
                const _Float16 b2 = (_Float16)(y - (float)a);
                *reinterpret_cast<_Float16 *>(p) = a;
                *reinterpret_cast<_Float16 *>(p + 1024) = b2;
            } else if constexpr (NP1 == 3) {
                const __bf16 a = (__bf16)v[q];
                const float r1 = v[q] - (float)a;
                const __bf16 b2 = (__bf16)r1;
                const float r2 = r1 - (float)b2;
                *reinterpret_cast<__bf16 *>(p) = a;
                *reinterpret_cast<__bf16 *>(p + 1024) = b2;
                *reinterpret_cast<__bf16 *>(p + 2048) = (__bf16)r2;
            } else {
                *reinterpret_cast<__bf16 *>(p) = (__bf16)v[q];
            }
        }
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    stage_barrier();
    PN2_DSTAMP(4);

    // ---- 4. layer 1, tile t1
#pragma unroll
    for (int q = 0; q < 16; ++q) acc[q] = 0.f;
    Split yb[2];
    yb[0] = ring_readN<NP1>(planes, lane);
#pragma unroll
    for (int kb = 0; kb < kb1n; ++kb) {
        if (kb + 1 < kb1n) yb[(kb + 1) & 1] = ring_readN<NP1>(planes + (kb + 1) * NP1 * 1024, lane);
        __builtin_amdgcn_sched_barrier(0);
        acc = mma_wb<NP1>(yb[kb & 1], wc[kb % RD], acc);
        if (kb + RD < kb1n) wc[kb % RD] = load_wfrag<NP1>(w1 + (int64_t)(kb + RD) * 64, plane1);
        __builtin_amdgcn_sched_barrier(0);
    }
    PN2_DSTAMP(5);
    PN2_DSTAMP(14);
    const float al1 = NP1 == 2 ? pa1 * asc.down : pa1;
    unsigned omax = 0;
#pragma unroll
    for (int q = 0; q < 16; ++q) {
        const int row = row0 + (q & 3) + 8 * (q >> 2) + 4 * h;
        if (row < M) {
            const float y = __builtin_fmaf(acc[q], al1, be1);
            const float o = A1.raw ? acc[q] * al1 : (A1.norelu ? y : chain_relu(y));
            A1.out[A1.frag_out ? frag_off(row, col1, 2 * A1.tiles) : (int64_t)row * A1.ostride + col1] = o;
            omax = max(omax, __float_as_uint(o) & 0x7FFFFFFFu);
        }
    }
    if (A1.out_max) {
        const unsigned m = wave_max_u32(omax);
        if (lane == 0 && row0 < M) A1.out_max[(int64_t)rb * A1.tiles + t1] = m;
    }
    PN2_DSTAMP(15);
}

// The pair's LDS: the maxima + the larger layer's A planes
static size_t dense_pair_lds(const DenseSplitArgs &A0, const DenseSplitArgs &A1, int np0, int np1) {
    return 64 + (size_t)std::max(A0.kb * np0, A1.kb * np1) * 1024;
}

// Whether layers A0 (group_all, first) and A1 (its consumer) run as one dense_pair_kernel
// launch: layer 0 = 8 column tiles (256 outputs: one per wave), layer 1 reads all of them and
// has a multiple of 8 tiles, neither pools, rows of 16-byte feature runs.
static bool dense_pair_ok(const DenseSplitArgs &A0, const DenseSplitArgs &A1, int np0, int np1) {
    if (!tuning().dense_pair || A0.mode != 1 || A1.mode != 0 || A0.pool || A1.pool) return false;
    if (A0.tiles != kPairWaves || A1.tiles % kPairWaves != 0 || A1.cin != 32 * A0.tiles || A1.kb != 2 * A0.tiles)
        return false;
    if (!A0.vec || !A0.feat || A0.D <= 0 || A0.D % 16 != 0 || A0.kb != 1 + A0.D / 16 || A0.C > 16) return false;
    if (A0.fn % 4 || A0.fb % 4 || ((uintptr_t)A0.feat & 15)) return false;
    if ((np0 != 3 && np0 != 2) || (np1 != 2 && np1 != 3) || (np0 == 2 && np1 != 2)) return false;
    if (np0 == 2 && !A0.wscale) return false;
    if (A0.kb != 17 && A0.kb != 41) return false;  // the instantiated k-block counts (D = 256, 640)
    if (np1 == 2 && !A1.wscale) return false;
    if (A1.frag_in) return false;
    return dense_pair_lds(A0, A1, np0, np1) <= 160 * 1024;
}

template <int NP0, int NP1, int KB0>
static void launch_pair(const DenseSplitArgs &A0, const DenseSplitArgs &A1, int cs, dim3 grid, dim3 block, size_t lds,
                        hipStream_t st) {
    static const hipError_t attr = hipFuncSetAttribute(reinterpret_cast<const void *>(&dense_pair_kernel<NP0, NP1, KB0>),
                                                       hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    (void)attr;
    hipLaunchKernelGGL((dense_pair_kernel<NP0, NP1, KB0>), grid, block, lds, st, A0, A1, cs);
}

static int launch_dense_pair(const DenseSplitArgs &A0, const DenseSplitArgs &A1, int np0, int np1, hipStream_t st) {
    const int cs = A1.tiles / kPairWaves;
    const int64_t nrb = (A0.M + 31) / 32;
    const size_t lds = dense_pair_lds(A0, A1, np0, np1);
    const dim3 grid((unsigned)(nrb * cs)), block(64 * kPairWaves);
    if (np0 == 2) {
        if (A0.kb == 17) launch_pair<2, 2, 17>(A0, A1, cs, grid, block, lds, st);
        else launch_pair<2, 2, 41>(A0, A1, cs, grid, block, lds, st);
    } else if (np1 == 2) {
        if (A0.kb == 17) launch_pair<3, 2, 17>(A0, A1, cs, grid, block, lds, st);
        else launch_pair<3, 2, 41>(A0, A1, cs, grid, block, lds, st);
    } else {
        if (A0.kb == 17) launch_pair<3, 3, 17>(A0, A1, cs, grid, block, lds, st);
        else launch_pair<3, 3, 41>(A0, A1, cs, grid, block, lds, st);
    }
    PN2_LAUNCH_CHECK("dense_pair_kernel");
    return PN2_OK;
}

// Large split (fp32-accurate) layers take 256 x 128 tiles (see dense_split_layer); the rows a
// launch's workgroup covers decide which pools fit in LDS.  bf16 layers keep the 128-row tiles:
// with one MFMA per product instead of six the big tile's one workgroup per CU (8 waves, 221
// VGPRs) is load-latency bound -- STRESS (sa3 512 -> 1024 over 16384 rows, pipelined) 129.3-132.5k
// with it, 134.1-135.6k without (interleaved A/B x3).
static bool dense_wide(const DenseSplitArgs &A, int np) {
    const int64_t wide_min = tuning().dense_wide_minwg;
    return np >= 2 && A.tiles % 4 == 0 && (A.M + 255) / 256 * (A.tiles / 4) >= wide_min;
}
// the 4-wave tile's column tiles per wave: the widest that still leaves dense_minwg workgroups
static int dense_ntc(const DenseSplitArgs &A) {
    const int64_t rowblocks = (A.M + kDRows - 1) / kDRows;
    const int64_t min_wg = tuning().dense_minwg;
    for (int t = (int)tuning().dense_maxntc; t > 1; t /= 2)
        if (A.tiles % t == 0 && rowblocks * (A.tiles / t) >= min_wg) return t;
    return 1;
}
static int dense_pool_mode(const DenseSplitArgs &A, int np) {
    const int64_t kRowsSel = dense_wide(A, np) ? 256 : kDRows;
    if (A.K == 8 || A.K == 16) return 0;
    if (A.K % 32 == 0 && kRowsSel % A.K == 0) return 1;
    return 2;
}

// whether the layer, as it will be launched, pools through HBM atomics into a zeroed output
static bool dense_needs_zero(const DenseSplitArgs &A, int np) {
    if (!A.pool) return false;
    const int tile = dense_lds_tile(A);
    if (tile) return (32 * (tile / 10)) % A.K != 0;
    return dense_pool_mode(A, np) == 2;
}

static int dense_split_layer(DenseSplitArgs &A, int np, hipStream_t st, bool prezeroed = false) {
    if (const int tile = dense_lds_tile(A)) {
        const bool hbm = dense_needs_zero(A, np);
        const int64_t G = A.pool ? A.M / A.K : 0, cols = 32 * (int64_t)A.tiles;
        if (hbm && !prezeroed) {
            hipError_t e = A.ostride == cols
                               ? hipMemsetAsync(A.out, 0, (size_t)G * cols * 4, st)
                               : hipMemset2DAsync(A.out, (size_t)A.ostride * 4, 0, (size_t)cols * 4, (size_t)G, st);
            if (e != hipSuccess) return set_error(PN2_EHIP, "dense_lds: memset: %s", hipGetErrorString(e));
        }
        const int rc = launch_dense_lds_tile(tile, A, np, st);
        if (rc == PN2_OK && hbm && A.norelu) {  // keys -> floats
            hipLaunchKernelGGL(unkey_kernel, dim3((unsigned)((G * cols + 255) / 256)), dim3(256), 0, st,
                               A.out, A.ostride, G, (int)cols);
            PN2_LAUNCH_CHECK("unkey_kernel");
        }
        return rc;
    }
    // Large layers (e.g. translation_ssg's group_all over B*512 rows) take 256 x 128 tiles (8
    // waves of 32 rows x 4 column tiles): the 128 x 64 tile re-reads its A rows once per 64
    // output columns and its weights once per 128 rows, and at these sizes that L2 -> CU
    // stream, not the MFMA, was the bound.  Only when they still leave wide_min workgroups.
    const bool wide = dense_wide(A, np);
    // otherwise the widest tile (NTC 32-column tiles per wave) that still leaves min_wg workgroups
    const int ntc = dense_ntc(A);
    if (A.pool) {
        A.pool_mode = dense_pool_mode(A, np);
        if (A.pool_mode == 2 && !prezeroed) {
            const int64_t G = A.M / A.K, cols = 32 * (int64_t)A.tiles;
            hipError_t e = A.ostride == cols
                               ? hipMemsetAsync(A.out, 0, (size_t)G * cols * 4, st)
                               : hipMemset2DAsync(A.out, (size_t)A.ostride * 4, 0, (size_t)cols * 4, (size_t)G, st);
            if (e != hipSuccess) return set_error(PN2_EHIP, "dense_split: memset: %s", hipGetErrorString(e));
        }
    }
    int rc;
    if (wide) rc = np == 1 ? launch_dense_split<4, 1, 8>(A, st) : np == 2 ? launch_dense_split<4, 2, 8>(A, st)
                                                                         : launch_dense_split<4, 3, 8>(A, st);
    else if (np == 1) rc = ntc == 4 ? launch_dense_split<4, 1>(A, st) : ntc == 2 ? launch_dense_split<2, 1>(A, st)
                                                                      : launch_dense_split<1, 1>(A, st);
    else if (np == 2) rc = ntc == 4 ? launch_dense_split<4, 2>(A, st) : ntc == 2 ? launch_dense_split<2, 2>(A, st)
                                                                      : launch_dense_split<1, 2>(A, st);
    else rc = ntc == 4 ? launch_dense_split<4, 3>(A, st) : ntc == 2 ? launch_dense_split<2, 3>(A, st)
                                                           : launch_dense_split<1, 3>(A, st);
    if (rc == PN2_OK && A.pool && A.pool_mode == 2 && A.norelu) {  // keys -> floats
        const int64_t G = A.M / A.K, cols = 32 * (int64_t)A.tiles;
        hipLaunchKernelGGL(unkey_kernel, dim3((unsigned)((G * cols + 255) / 256)), dim3(256), 0, st,
                           A.out, A.ostride, G, (int)cols);
        PN2_LAUNCH_CHECK("unkey_kernel");
    }
    return rc;
}

// The chain kernel's layer-0 pre-pass (sa_chain.hip, KB0M < 0): z[b*N + n][c] = sum_k W0[c][k] *
// x_k(b, n) over the raw [xyz | features] row of every source point (no bias / BN / ReLU), with
// the fp32-accurate split products.  z is [B*N][cout0] fp32 at `z` (16-byte aligned).
int launch_layer0_prepass(const pn2_sa_src &s, const pn2_mlp_layer &L0, float *z, hipStream_t st) {
    DenseSplitArgs A;
    memset(&A, 0, sizeof(A));
    A.mode = 1;
    A.pts = s.pts; A.pb = s.pb; A.pn = s.pn; A.pc = s.pc;
    A.feat = s.feat; A.fb = s.fb; A.fn = s.fn;
    A.N = (int)s.N; A.C = (int)s.C; A.D = (int)s.D;
    A.vec = (s.D == 0 || (s.D % 4 == 0 && ((uintptr_t)s.feat & 15) == 0 && s.fn % 4 == 0 &&
                          s.fb % 4 == 0)) ? 1 : 0;
    A.kb = (int)pn2_layer_split_kblocks(L0.cin, s.C);
    A.w = reinterpret_cast<const bf16x8 *>(L0.wt_split);
    A.tiles = (int)(L0.cout / 32);
    A.M = (int)(s.B * s.N);
    A.out = z;
    A.ostride = L0.cout;
    A.raw = 1;
    // split fp16 with the scale from each 32-point block's own [xyz | features] (a cloud's points
    // fill whole blocks); tuning dense_f16 = 0: split bf16
    if (tuning().dense_f16 >= 2 && s.N % 32 == 0) {
        A.w = split_f16_planes(L0.wt_split, L0.cout, A.kb);
        A.wscale = split_f16_inv_scale(L0.wt_split, L0.cout, A.kb);
        return dense_split_layer(A, 2, st);
    }
    return dense_split_layer(A, 3, st);
}

static thread_local int g_dense_planes = 3;
int dense_last_planes() { return g_dense_planes; }

// Workspace of the layer-by-layer path: two [M][w] fp32 halves, then two [ceil(M/32)][w/32]
// uint max tables (the split-fp16 layers' activation scales, split_bf16.h)
int64_t dense_split_ws_bytes(int64_t M, int64_t w) {
    const int64_t Mp = (M + 31) / 32 * 32;  // fragment-ordered halves cover whole row blocks
    return 2 * Mp * w * 4 + 2 * (Mp / 32) * ((w + 31) / 32) * 4;
}

// Widest hidden layer of a chain the split dense path runs layer by layer (0: not eligible).
int64_t dense_split_width(const pn2_sa_src &s, const pn2_mlp_layer *layers, int nlayers, int np) {
    if (np == 3 && tuning().mlp_f32) return 0;
    if (s.mode != PN2_SRC_GROUP_ALL && s.mode != PN2_SRC_ROWS) return 0;
    if (s.mode == PN2_SRC_GROUP_ALL && s.C > 16) return 0;
    int64_t w = 0;
    for (int l = 0; l < nlayers; ++l) {
        if (!layers[l].wt_split || ((uintptr_t)layers[l].wt_split & 15)) return 0;
        if (l < nlayers - 1) w = std::max(w, layers[l].cout);
    }
    return nlayers > 1 ? (w + 3) / 4 * 4 : 1;
}

// 1: launched, 0: not eligible, <0: error.  Layers run one by one; hidden outputs ping-pong
// through the two [M][w] halves of the workspace.
int try_launch_dense_split(const pn2_sa_src &s, const pn2_mlp_layer *layers, int nlayers, int pool,
                           float *out, int64_t ostride, float *ws, int64_t ws_bytes, int64_t M,
                           int64_t K, int np, hipStream_t st) {
    const int64_t w = dense_split_width(s, layers, nlayers, np);
    if (w == 0) return 0;
    if (nlayers > 1 && (!ws || ws_bytes < dense_split_ws_bytes(M, w) || ((uintptr_t)ws & 15))) return 0;
    // The fp32-accurate hidden layers after the first (their rows are the workspace rows the
    // layer before wrote, with its per-block maxima) run split fp16 (3 MFMAs per product);
    // the first layer keeps split bf16 (its input comes from outside: no maxima).  A cloud's rows
    // must start at a 32-row block (K % 32 == 0) so its scale never depends on other clouds.
    // Tuning dense_f16 = 0: split bf16 everywhere.
    const bool f16 = np == 3 && tuning().dense_f16 && K % 32 == 0;
    const int64_t tw = (w + 31) / 32, nrb = (M + 31) / 32, Mp = nrb * 32;
    unsigned *maxtab = nlayers > 1 ? reinterpret_cast<unsigned *>(ws + 2 * Mp * w) : nullptr;
    // the first layer over points (group_all) takes its scale from its own rows when a cloud's
    // points fill whole 32-row blocks
    const bool f16_first = f16 && tuning().dense_f16 >= 2 && s.mode == PN2_SRC_GROUP_ALL && s.N % 32 == 0;
    auto layer_np = [&](int l) { return (f16 && l >= 1) || (f16_first && l == 0) ? 2 : np; };
    auto make = [&](int l) {
        const bool last = l == nlayers - 1;
        DenseSplitArgs A;
        memset(&A, 0, sizeof(A));
        if (l == 0 && s.mode == PN2_SRC_GROUP_ALL) {
            A.mode = 1;
            A.pts = s.pts; A.pb = s.pb; A.pn = s.pn; A.pc = s.pc;
            A.feat = s.feat; A.fb = s.fb; A.fn = s.fn;
            A.N = (int)s.N; A.C = (int)s.C; A.D = (int)s.D;
            A.vec = (s.D == 0 || (s.D % 4 == 0 && ((uintptr_t)s.feat & 15) == 0 && s.fn % 4 == 0 &&
                                  s.fb % 4 == 0)) ? 1 : 0;
            A.kb = (int)pn2_layer_split_kblocks(layers[0].cin, s.C);
        } else {
            A.mode = 0;
            if (l == 0) {
                A.rows = s.rows;
                A.rs = s.rs;
            } else {
                A.rows = ws + ((l - 1) & 1) * Mp * w;
                A.rs = w;
            }
            A.cin = (int)layers[l].cin;
            A.vec = (((uintptr_t)A.rows & 15) == 0 && A.rs % 4 == 0) ? 1 : 0;
            A.kb = (int)((layers[l].cin + 15) / 16);
        }
        A.w = reinterpret_cast<const bf16x8 *>(layers[l].wt_split);
        A.alpha = layers[l].alpha;
        A.beta = layers[l].beta;
        A.tiles = (int)(layers[l].cout / 32);
        A.M = (int)M;
        if (layer_np(l) == 2) {
            A.w = split_f16_planes(layers[l].wt_split, layers[l].cout, A.kb);
            A.wscale = split_f16_inv_scale(layers[l].wt_split, layers[l].cout, A.kb);
            if (l > 0) {
                A.in_max = maxtab + ((l - 1) & 1) * nrb * tw;
                A.in_tiles = (int)(layers[l - 1].cout / 32);
            }
        }
        if (l < nlayers - 1 && layer_np(l + 1) == 2) A.out_max = maxtab + (l & 1) * nrb * tw;
        A.pool = last ? pool : 0;
        A.norelu = (layers[l].flags & PN2_LAYER_NO_RELU) ? 1 : 0;
        A.K = (int)K;
        A.out = last ? out : ws + (l & 1) * Mp * w;
        A.ostride = last ? ostride : w;
        return A;
    };
    // hidden rows in fragment order where their consumer is the register-staged kernel (the
    // LDS-staged one DMAs whole row lines); tuning dense_frag = 0: row-major everywhere
    bool frag[5] = {false, false, false, false, false};
    for (int l = 1; l < nlayers && l < 5; ++l) frag[l] = tuning().dense_frag && dense_lds_tile(make(l)) == 0;
    auto make_f = [&](int l) {
        DenseSplitArgs A = make(l);
        if (l >= 1 && frag[l]) A.frag_in = 1, A.vec = 1;
        if (l + 1 < nlayers && l + 1 < 5 && frag[l + 1]) A.frag_out = 1;
        return A;
    };
    // a last layer that pools by HBM atomics gets its output zeroed by the layer before it
    // (one launch fewer than a memset: PointNet-v1's max over N points, group_all over K > 256)
    DenseSplitArgs last = make_f(nlayers - 1);
    const bool fold_zero = nlayers > 1 && last.pool && dense_needs_zero(last, layer_np(nlayers - 1));
    if (s.zero_out && s.zero_count > 0) {  // the caller's side job rides on the last layer
        last.zero = s.zero_out;
        last.zrows = 1;
        last.zcols = s.zero_count;
        last.zstride = s.zero_count;
    }
    auto args_of = [&](int l) {
        DenseSplitArgs A = l == nlayers - 1 ? last : make_f(l);
        if (fold_zero && l == nlayers - 2) {
            A.zero = last.out;
            A.zrows = last.M / last.K;
            A.zcols = 32 * (int64_t)last.tiles;
            A.zstride = last.ostride;
        }
        return A;
    };
    int64_t flops[4] = {0, 0, 0, 0};
    for (int l = 0; l < nlayers; ++l) {
        flops[layer_np(l)] += layers[l].cin * layers[l].cout;
        DenseSplitArgs A = args_of(l);
        if (l == 0 && nlayers > 1) {  // group_all's first two layers as one launch
            DenseSplitArgs B = args_of(1);
            B.frag_in = 0;  // its input never leaves the CU
            if (dense_pair_ok(A, B, layer_np(0), layer_np(1))) {
                const int rc = launch_dense_pair(A, B, layer_np(0), layer_np(1), st);
                if (rc != PN2_OK) return rc;
                flops[layer_np(1)] += layers[1].cin * layers[1].cout;
                l = 1;
                continue;
            }
        }
        const int rc = dense_split_layer(A, layer_np(l), st, fold_zero && l == nlayers - 1);
        if (rc != PN2_OK) return rc;
    }
    g_dense_planes = flops[2] > flops[np] ? 2 : np;
    return 1;
}

}  // namespace pn2
