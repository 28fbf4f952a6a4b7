// train.hip -- training-mode (batch-statistics) BatchNorm + ReLU + max over the neighbourhood,
// forward and backward, for the SA layers' shared MLP.
//
// Reference: PointNetSetAbstraction.forward in train mode, /root/reference/model/
// pointnet2_utils.py:167-172 (Conv2d 1x1 -> BatchNorm2d -> ReLU per layer, torch.max over the
// K neighbours), the same for the MSG scales (:211-221); the loop train_rotation.py:99-133 runs
// it under autograd.  BatchNorm2d in training normalises with the batch statistics over all
// B*S*K rows (biased variance), updates running_mean / running_var (unbiased) with momentum, and
// its backward couples every row of the batch through the two column sums below.
//
// The matmuls (Y = X W^T + b, dW = dY^T X, dX = dY W) are plain GEMMs and go to the library
// (hipBLASLt via torch.mm, pn2/train.py); what is here is everything around them, fused so each
// pass reads the [M, C] activations once:
//   pn2_bn_train_stats_f32    column sum / sum of squares of Y (float64 partials per row chunk),
//                             then mean, invstd, running-stat update
//   pn2_bn_relu_apply_f32     A = relu((Y - mean) * invstd * gamma + beta)  (no ReLU with
//                             PN2_LAYER_NO_RELU: PointNet-v1's conv3 + bn3 before its max)
//   pn2_group_max_f32         out[g][c] = max_k A[g*K + k][c] and its first argmax
//   pn2_bn_relu_backward_f32  dXn = dA * [A > 0] (unmasked with PN2_LAYER_NO_RELU; dA from the
//                             next layer, or scattered from the max: arg[g][c] == k ?
//                             dOut[g][c] : 0), its column sums
//                             S1 = sum dXn and S2 = sum dXn * xhat (= dbeta, dgamma), then
//                             dY = gamma * invstd * (dXn - S1/M - xhat * S2/M)
// Layout: channels-last rows [M][C] with row stride ld (the SA path's layout), so every pass is
// a coalesced column-tiled sweep: a 256-thread block covers 64 columns x 4 row lanes of one row
// chunk and reduces through LDS; chunk partials are merged in float64 by a per-column pass.
#include "pn2_internal.h"

namespace pn2 {

constexpr int kTrCols = 64;     // columns per block
constexpr int kTrLanes = 4;     // row lanes per block
constexpr int kTrChunk = 1024;  // rows per chunk (partials per chunk), at most
constexpr int kTrChunkMin = 64;
constexpr int kTrMinBlocks = 2048;  // column sweeps: enough blocks to fill 256 CUs several times
constexpr int kTrUnroll = 8;    // rows in flight per thread in the column sweeps

__device__ __forceinline__ float tr_xhat(float y, float mean, float invstd) { return (y - mean) * invstd; }

// partial column sums of Y and Y^2 over row chunk blockIdx.y -> part[chunk][2][C] (double)
__global__ __launch_bounds__(256) void bn_stats_partial_kernel(const float *__restrict__ Y, int64_t M,
                                                               int64_t C, int64_t ld, int64_t chunk,
                                                               double *__restrict__ part) {
    __shared__ double red[2][kTrLanes][kTrCols];
    const int tx = threadIdx.x & (kTrCols - 1), ty = threadIdx.x / kTrCols;
    const int64_t c = (int64_t)blockIdx.x * kTrCols + tx;
    const int64_t r0 = (int64_t)blockIdx.y * chunk;
    const int64_t r1 = r0 + chunk < M ? r0 + chunk : M;
    double s = 0.0, q = 0.0;
    if (c < C) {
        // kTrUnroll rows in flight per thread: the loop is load-latency bound otherwise
        int64_t r = r0 + ty;
        for (; r + (kTrUnroll - 1) * kTrLanes < r1; r += kTrUnroll * kTrLanes) {
            float v[kTrUnroll];
#pragma unroll
            for (int u = 0; u < kTrUnroll; ++u) v[u] = Y[(r + u * kTrLanes) * ld + c];
#pragma unroll
            for (int u = 0; u < kTrUnroll; ++u) s += (double)v[u], q += (double)v[u] * (double)v[u];
        }
        for (; r < r1; r += kTrLanes) {
            const double y = (double)Y[r * ld + c];
            s += y;
            q += y * y;
        }
    }
    red[0][ty][tx] = s;
    red[1][ty][tx] = q;
    __syncthreads();
    if (ty == 0 && c < C) {
        for (int l = 1; l < kTrLanes; ++l) s += red[0][l][tx], q += red[1][l][tx];
        part[((int64_t)blockIdx.y * 2 + 0) * C + c] = s;
        part[((int64_t)blockIdx.y * 2 + 1) * C + c] = q;
    }
}

// merge the chunk partials of column c; mean, invstd; running-stat update (torch's BatchNorm
// train-mode rule: biased variance normalises, unbiased variance enters running_var)
// sum of the nch chunk partials of column c (pair p of the [chunk][2][C] layout), one wave per
// column: each lane takes every 64th chunk, then a shuffle tree
__device__ __forceinline__ double wave_col_sum(const double *__restrict__ part, int64_t nch, int64_t C,
                                               int64_t c, int p) {
    const int lane = threadIdx.x;
    double s = 0.0;
    for (int64_t k = lane; k < nch; k += 64) s += part[(k * 2 + p) * C + c];
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) s += __shfl_xor(s, off);
    return s;
}

__global__ __launch_bounds__(64) void bn_stats_final_kernel(const double *__restrict__ part, int64_t nch,
                                                            int64_t M, int64_t C, double eps,
                                                            double momentum, float *running_mean,
                                                            float *running_var,
                                                            float *__restrict__ mean_out,
                                                            float *__restrict__ invstd_out,
                                                            double *__restrict__ sxhat) {
    const int64_t c = blockIdx.x;
    const double s = wave_col_sum(part, nch, C, c, 0), q = wave_col_sum(part, nch, C, c, 1);
    if (threadIdx.x != 0) return;
    const double mean = s / (double)M;
    double var = q / (double)M - mean * mean;
    if (var < 0.0) var = 0.0;
    mean_out[c] = (float)mean;
    invstd_out[c] = (float)(1.0 / sqrt(var + eps));
    // sum over rows of xhat = (y - mean_f32) * invstd_f32 with the rounded statistics the other
    // kernels use: the conv bias gradient (sum of dY) is -gamma*invstd*dgamma/M times this
    sxhat[c] = (s - (double)M * (double)mean_out[c]) * (double)invstd_out[c];
    if (running_mean && momentum > 0.0) {
        const double unb = M > 1 ? var * (double)M / (double)(M - 1) : var;
        running_mean[c] = (float)((1.0 - momentum) * (double)running_mean[c] + momentum * mean);
        running_var[c] = (float)((1.0 - momentum) * (double)running_var[c] + momentum * unb);
    }
}

// elementwise sweeps: block (64 columns x 4 row lanes) walks kTrEwRows rows of its column tile
constexpr int kTrEwRows = 64;

__global__ __launch_bounds__(256) void bn_relu_apply_kernel(const float *__restrict__ Y, int64_t M,
                                                            int64_t C, int64_t ld,
                                                            const float *__restrict__ mean,
                                                            const float *__restrict__ invstd,
                                                            const float *__restrict__ gamma,
                                                            const float *__restrict__ beta,
                                                            float *__restrict__ A, int64_t lda,
                                                            int relu) {
    const int tx = threadIdx.x & (kTrCols - 1), ty = threadIdx.x / kTrCols;
    const int64_t c = (int64_t)blockIdx.x * kTrCols + tx;
    if (c >= C) return;
    const float mu = mean[c], is = invstd[c], ga = gamma[c], be = beta[c];
    const int64_t r0 = (int64_t)blockIdx.y * kTrEwRows;
    const int64_t r1 = r0 + kTrEwRows < M ? r0 + kTrEwRows : M;
#pragma unroll 4
    for (int64_t r = r0 + ty; r < r1; r += kTrLanes) {
        const float x = tr_xhat(Y[r * ld + c], mu, is) * ga + be;
        A[r * lda + c] = relu ? (x > 0.f ? x : 0.f) : x;  // relu is uniform: no divergence
    }
}

// one thread per (group, column): max over the group's K rows, first index of the max
__global__ __launch_bounds__(256) void group_max_kernel(const float *__restrict__ A, int64_t G,
                                                        int64_t K, int64_t C, int64_t lda,
                                                        float *__restrict__ out, int64_t ldo,
                                                        int32_t *__restrict__ arg) {
    const int tx = threadIdx.x & (kTrCols - 1), ty = threadIdx.x / kTrCols;
    const int64_t c = (int64_t)blockIdx.x * kTrCols + tx;
    const int64_t g = (int64_t)blockIdx.y * kTrLanes + ty;
    if (c >= C || g >= G) return;
    const float *p = A + g * K * lda + c;
    float m = p[0];
    int32_t a = 0;
    int64_t k = 1;
    for (; k + 8 <= K; k += 8) {  // 8 rows in flight
        float v[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) v[u] = p[(k + u) * lda];
#pragma unroll
        for (int u = 0; u < 8; ++u)
            if (v[u] > m || (v[u] != v[u] && m == m)) m = v[u], a = (int32_t)(k + u);  // NaN wins
    }
    for (; k < K; ++k) {
        const float v = p[k * lda];
        if (v > m || (v != v && m == m)) m = v, a = (int32_t)k;  // NaN wins, as torch.max
    }
    out[g * ldo + c] = m;
    arg[g * C + c] = a;
}

// (v, a) beats (m, b) in the max's order: NaN above every number, then value, then the first
// index (torch.max's first argmax)
__device__ __forceinline__ bool tr_better(float v, int32_t a, float m, int32_t b) {
    if (v != v) return m == m || a < b;
    if (m != m) return false;
    return v > m || (v == m && a < b);
}

// Large K (a PointNet-v1 max over a cloud's N points): one block per (group, 64 columns), the K
// rows split over kTrWideLanes row lanes (8 rows in flight each), lanes merged through LDS.
// One thread per (group, column) walking all K rows would serialise K/8 dependent load rounds.
constexpr int kTrWideLanes = 16;
constexpr int kTrWideK = 256;  // K from which the wide kernel is used

__global__ __launch_bounds__(kTrCols * kTrWideLanes) void group_max_wide_kernel(
    const float *__restrict__ A, int64_t K, int64_t C, int64_t lda, float *__restrict__ out, int64_t ldo,
    int32_t *__restrict__ arg) {
    __shared__ float sv[kTrWideLanes][kTrCols];
    __shared__ int32_t sa[kTrWideLanes][kTrCols];
    const int tx = threadIdx.x & (kTrCols - 1), ty = threadIdx.x / kTrCols;
    const int64_t c = (int64_t)blockIdx.x * kTrCols + tx;
    const int64_t g = blockIdx.y;
    float m = -__builtin_inff();
    int32_t a = 0x7fffffff;
    if (c < C) {
        const float *p = A + g * K * lda + c;
        int64_t k = ty;
        for (; k + 7 * kTrWideLanes < K; k += 8 * kTrWideLanes) {
            float v[8];
#pragma unroll
            for (int u = 0; u < 8; ++u) v[u] = p[(k + u * kTrWideLanes) * lda];
#pragma unroll
            for (int u = 0; u < 8; ++u)  // increasing row order within the lane: strict > keeps the first
                if (v[u] > m || (v[u] != v[u] && m == m) || a == 0x7fffffff)
                    m = v[u], a = (int32_t)(k + u * kTrWideLanes);
        }
        for (; k < K; k += kTrWideLanes) {
            const float v = p[k * lda];
            if (v > m || (v != v && m == m) || a == 0x7fffffff) m = v, a = (int32_t)k;
        }
    }
    sv[ty][tx] = m;
    sa[ty][tx] = a;
    __syncthreads();
    if (ty == 0 && c < C) {
        for (int l = 1; l < kTrWideLanes; ++l)
            if (sa[l][tx] != 0x7fffffff && tr_better(sv[l][tx], sa[l][tx], m, a)) m = sv[l][tx], a = sa[l][tx];
        out[g * ldo + c] = m;
        arg[g * C + c] = a;
    }
}

// dXn of row r, column c (see header); dA dense [M][C] (ldd) or scattered from the max
__device__ __forceinline__ float tr_dxn(const float *__restrict__ Y, int64_t ld, int64_t r, int64_t c,
                                        float mean, float invstd, float gamma, float beta,
                                        const float *__restrict__ dA, int64_t ldd,
                                        const float *__restrict__ dOut, int64_t ldo,
                                        const int32_t *__restrict__ arg, int64_t K, int64_t C,
                                        int relu, float &xhat) {
    // branch-free: every load is issued whatever the ReLU mask, so unrolled rows stay in flight
    xhat = tr_xhat(Y[r * ld + c], mean, invstd);
    float d;
    if (dA) {
        d = dA[r * ldd + c];
    } else {
        // 32-bit division (the host checks M < 2^31): the 64-bit one is a long call sequence
        const uint32_t g = (uint32_t)r / (uint32_t)K;
        const float o = dOut[(int64_t)g * ldo + c];
        d = arg[(int64_t)g * C + c] == (int32_t)((uint32_t)r - g * (uint32_t)K) ? o : 0.f;
    }
    return !relu || xhat * gamma + beta > 0.f ? d : 0.f;
}

__global__ __launch_bounds__(256) void bn_bwd_partial_kernel(
    const float *__restrict__ Y, int64_t M, int64_t C, int64_t ld, const float *__restrict__ mean,
    const float *__restrict__ invstd, const float *__restrict__ gamma, const float *__restrict__ beta,
    const float *__restrict__ dA, int64_t ldd, const float *__restrict__ dOut, int64_t ldo,
    const int32_t *__restrict__ arg, int64_t K, int relu, int64_t chunk, double *__restrict__ part) {
    __shared__ double red[2][kTrLanes][kTrCols];
    const int tx = threadIdx.x & (kTrCols - 1), ty = threadIdx.x / kTrCols;
    const int64_t c = (int64_t)blockIdx.x * kTrCols + tx;
    const int64_t r0 = (int64_t)blockIdx.y * chunk;
    const int64_t r1 = r0 + chunk < M ? r0 + chunk : M;
    double s1 = 0.0, s2 = 0.0;
    if (c < C) {
        const float mu = mean[c], is = invstd[c], ga = gamma[c], be = beta[c];
        int64_t r = r0 + ty;
        for (; r + (kTrUnroll - 1) * kTrLanes < r1; r += kTrUnroll * kTrLanes) {
            float d[kTrUnroll], xh[kTrUnroll];
#pragma unroll
            for (int u = 0; u < kTrUnroll; ++u)
                d[u] = tr_dxn(Y, ld, r + u * kTrLanes, c, mu, is, ga, be, dA, ldd, dOut, ldo, arg, K, C, relu, xh[u]);
#pragma unroll
            for (int u = 0; u < kTrUnroll; ++u) s1 += (double)d[u], s2 += (double)d[u] * (double)xh[u];
        }
        for (; r < r1; r += kTrLanes) {
            float xh;
            const float d = tr_dxn(Y, ld, r, c, mu, is, ga, be, dA, ldd, dOut, ldo, arg, K, C, relu, xh);
            s1 += (double)d;
            s2 += (double)d * (double)xh;
        }
    }
    red[0][ty][tx] = s1;
    red[1][ty][tx] = s2;
    __syncthreads();
    if (ty == 0 && c < C) {
        for (int l = 1; l < kTrLanes; ++l) s1 += red[0][l][tx], s2 += red[1][l][tx];
        part[((int64_t)blockIdx.y * 2 + 0) * C + c] = s1;
        part[((int64_t)blockIdx.y * 2 + 1) * C + c] = s2;
    }
}

// The same column sums when dA is scattered from the max (the last layer): dXn is nonzero only
// on each group's argmax row, so S1 = sum_g mask * dOut[g][c] and S2 = sum_g mask * dOut[g][c] *
// xhat(Y[g*K + arg[g][c]][c]) read G = M/K gathered rows instead of sweeping all M (K = 32-64 x
// fewer bytes: the SA layers' widest Y, 268 MB at SSG, is the largest term of a training step).
// Chunk blockIdx.y covers groups [y*chunk, y*chunk + chunk); partials as above.
__global__ __launch_bounds__(256) void bn_bwd_partial_gather_kernel(
    const float *__restrict__ Y, int64_t G, int64_t C, int64_t ld, const float *__restrict__ mean,
    const float *__restrict__ invstd, const float *__restrict__ gamma, const float *__restrict__ beta,
    const float *__restrict__ dOut, int64_t ldo, const int32_t *__restrict__ arg, int64_t K, int relu,
    int64_t chunk, double *__restrict__ part) {
    __shared__ double red[2][kTrLanes][kTrCols];
    const int tx = threadIdx.x & (kTrCols - 1), ty = threadIdx.x / kTrCols;
    const int64_t c = (int64_t)blockIdx.x * kTrCols + tx;
    const int64_t g0 = (int64_t)blockIdx.y * chunk;
    const int64_t g1 = g0 + chunk < G ? g0 + chunk : G;
    double s1 = 0.0, s2 = 0.0;
    if (c < C) {
        const float mu = mean[c], is = invstd[c], ga = gamma[c], be = beta[c];
        for (int64_t g = g0 + ty; g < g1; g += kTrLanes) {
            const int64_t r = g * K + arg[g * C + c];
            const float xh = tr_xhat(Y[r * ld + c], mu, is);
            const float d = !relu || xh * ga + be > 0.f ? dOut[g * ldo + c] : 0.f;
            s1 += (double)d;
            s2 += (double)d * (double)xh;
        }
    }
    red[0][ty][tx] = s1;
    red[1][ty][tx] = s2;
    __syncthreads();
    if (ty == 0 && c < C) {
        for (int l = 1; l < kTrLanes; ++l) s1 += red[0][l][tx], s2 += red[1][l][tx];
        part[((int64_t)blockIdx.y * 2 + 0) * C + c] = s1;
        part[((int64_t)blockIdx.y * 2 + 1) * C + c] = s2;
    }
}

__global__ __launch_bounds__(64) void bn_bwd_final_kernel(const double *__restrict__ part, int64_t nch,
                                                          int64_t M, int64_t C, const float *__restrict__ gamma,
                                                          const float *__restrict__ invstd,
                                                          const double *__restrict__ sxhat,
                                                          float *__restrict__ dbeta, float *__restrict__ dgamma,
                                                          float *__restrict__ dbias, double *__restrict__ sums) {
    const int64_t c = blockIdx.x;
    const double s1 = wave_col_sum(part, nch, C, c, 0), s2 = wave_col_sum(part, nch, C, c, 1);
    if (threadIdx.x != 0) return;
    dbeta[c] = (float)s1;
    dgamma[c] = (float)s2;
    sums[c] = s1;
    sums[C + c] = s2;
    // sum_r dY = gamma*invstd*(s1 - M*(s1/M) - (s2/M)*sum_r xhat): the conv bias gradient
    if (dbias) dbias[c] = (float)(-(double)gamma[c] * (double)invstd[c] * (s2 / (double)M) * sxhat[c]);
}

__global__ __launch_bounds__(256) void bn_bwd_apply_kernel(
    const float *__restrict__ Y, int64_t M, int64_t C, int64_t ld, const float *__restrict__ mean,
    const float *__restrict__ invstd, const float *__restrict__ gamma, const float *__restrict__ beta,
    const float *__restrict__ dA, int64_t ldd, const float *__restrict__ dOut, int64_t ldo,
    const int32_t *__restrict__ arg, int64_t K, int relu, const double *__restrict__ sums,
    float *__restrict__ dY, int64_t ldy) {
    const int tx = threadIdx.x & (kTrCols - 1), ty = threadIdx.x / kTrCols;
    const int64_t c = (int64_t)blockIdx.x * kTrCols + tx;
    if (c >= C) return;
    const float mu = mean[c], is = invstd[c], ga = gamma[c], be = beta[c];
    const float m1 = (float)(sums[c] / (double)M), m2 = (float)(sums[C + c] / (double)M);
    const int64_t r0 = (int64_t)blockIdx.y * kTrEwRows;
    const int64_t r1 = r0 + kTrEwRows < M ? r0 + kTrEwRows : M;
#pragma unroll 4
    for (int64_t r = r0 + ty; r < r1; r += kTrLanes) {
        float xh;
        const float d = tr_dxn(Y, ld, r, c, mu, is, ga, be, dA, ldd, dOut, ldo, arg, K, C, relu, xh);
        dY[r * ldy + c] = ga * is * (d - m1 - xh * m2);
    }
}

// ---- 16-byte variants (C, ld, ldd, ldy multiples of 4, 16-byte aligned bases: every SA / v1
// layer): a thread covers 4 adjacent columns with one dwordx4 load or store per row, a block 64
// columns x 16 row lanes.  The scalar sweeps issued 4-byte loads and reached 2.9 (partial) and
// 3.9 TB/s (apply) at SSG training sizes.
constexpr int kTrVecLanes = 16;

__device__ __forceinline__ float4 ld4(const float *p) { return *reinterpret_cast<const float4 *>(p); }

// partial column sums of dXn and dXn * xhat, dA dense (the non-max layers)
__global__ __launch_bounds__(256) void bn_bwd_partial_vec_kernel(
    const float *__restrict__ Y, int64_t M, int64_t C, int64_t ld, const float *__restrict__ mean,
    const float *__restrict__ invstd, const float *__restrict__ gamma, const float *__restrict__ beta,
    const float *__restrict__ dA, int64_t ldd, int relu, int64_t chunk, double *__restrict__ part) {
    __shared__ double red[2][kTrVecLanes][kTrCols];
    const int cq = threadIdx.x & 15, rl = threadIdx.x >> 4;
    const int64_t c = (int64_t)blockIdx.x * kTrCols + cq * 4;
    const int64_t r0 = (int64_t)blockIdx.y * chunk;
    const int64_t r1 = r0 + chunk < M ? r0 + chunk : M;
    double s1[4] = {0.0, 0.0, 0.0, 0.0}, s2[4] = {0.0, 0.0, 0.0, 0.0};
    if (c < C) {
        const float4 mu = ld4(mean + c), is = ld4(invstd + c), ga = ld4(gamma + c), be = ld4(beta + c);
        const float mus[4] = {mu.x, mu.y, mu.z, mu.w}, iss[4] = {is.x, is.y, is.z, is.w};
        const float gas[4] = {ga.x, ga.y, ga.z, ga.w}, bes[4] = {be.x, be.y, be.z, be.w};
        int64_t r = r0 + rl;
        constexpr int U = 4;  // rows in flight per thread (2 x 16-byte loads each)
        for (; r + (U - 1) * kTrVecLanes < r1; r += U * kTrVecLanes) {
            float4 y[U], d[U];
#pragma unroll
            for (int u = 0; u < U; ++u) y[u] = ld4(Y + (r + u * kTrVecLanes) * ld + c);
#pragma unroll
            for (int u = 0; u < U; ++u) d[u] = ld4(dA + (r + u * kTrVecLanes) * ldd + c);
#pragma unroll
            for (int u = 0; u < U; ++u) {
                const float yv[4] = {y[u].x, y[u].y, y[u].z, y[u].w}, dv[4] = {d[u].x, d[u].y, d[u].z, d[u].w};
#pragma unroll
                for (int j = 0; j < 4; ++j) {
                    const float xh = tr_xhat(yv[j], mus[j], iss[j]);
                    const float dd = !relu || xh * gas[j] + bes[j] > 0.f ? dv[j] : 0.f;
                    s1[j] += (double)dd;
                    s2[j] += (double)dd * (double)xh;
                }
            }
        }
        for (; r < r1; r += kTrVecLanes) {
            const float4 y = ld4(Y + r * ld + c), d = ld4(dA + r * ldd + c);
            const float yv[4] = {y.x, y.y, y.z, y.w}, dv[4] = {d.x, d.y, d.z, d.w};
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                const float xh = tr_xhat(yv[j], mus[j], iss[j]);
                const float dd = !relu || xh * gas[j] + bes[j] > 0.f ? dv[j] : 0.f;
                s1[j] += (double)dd;
                s2[j] += (double)dd * (double)xh;
            }
        }
    }
#pragma unroll
    for (int j = 0; j < 4; ++j) red[0][rl][cq * 4 + j] = s1[j], red[1][rl][cq * 4 + j] = s2[j];
    __syncthreads();
    // 128 threads finish: (sum p, column) over the 16 row lanes
    if (threadIdx.x < 2 * kTrCols) {
        const int pp = threadIdx.x / kTrCols, col = threadIdx.x % kTrCols;
        const int64_t cc = (int64_t)blockIdx.x * kTrCols + col;
        if (cc < C) {
            double t = 0.0;
            for (int l = 0; l < kTrVecLanes; ++l) t += red[pp][l][col];
            part[((int64_t)blockIdx.y * 2 + pp) * C + cc] = t;
        }
    }
}

// dY = gamma * invstd * (dXn - S1/M - xhat * S2/M), dA dense or scattered from the max
__global__ __launch_bounds__(256) void bn_bwd_apply_vec_kernel(
    const float *__restrict__ Y, int64_t M, int64_t C, int64_t ld, const float *__restrict__ mean,
    const float *__restrict__ invstd, const float *__restrict__ gamma, const float *__restrict__ beta,
    const float *__restrict__ dA, int64_t ldd, const float *__restrict__ dOut, int64_t ldo,
    const int32_t *__restrict__ arg, int64_t K, int relu, const double *__restrict__ sums,
    float *__restrict__ dY, int64_t ldy) {
    const int cq = threadIdx.x & 15, rl = threadIdx.x >> 4;
    const int64_t c = (int64_t)blockIdx.x * kTrCols + cq * 4;
    if (c >= C) return;
    float mus[4], iss[4], gas[4], bes[4], m1[4], m2[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        mus[j] = mean[c + j], iss[j] = invstd[c + j], gas[j] = gamma[c + j], bes[j] = beta[c + j];
        m1[j] = (float)(sums[c + j] / (double)M), m2[j] = (float)(sums[C + c + j] / (double)M);
    }
    const int64_t r0 = (int64_t)blockIdx.y * kTrEwRows;
    constexpr int U = kTrEwRows / kTrVecLanes;  // 4 rows per thread, all in flight
    float4 y[U], d[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
        const int64_t r = r0 + rl + u * kTrVecLanes;
        const int64_t rr = r < M ? r : M - 1;  // clamped: loads stay branch-free
        y[u] = ld4(Y + rr * ld + c);
        if (dA) {
            d[u] = ld4(dA + rr * ldd + c);
        } else {
            const uint32_t g = (uint32_t)rr / (uint32_t)K, k = (uint32_t)rr - g * (uint32_t)K;
            const float4 o = ld4(dOut + (int64_t)g * ldo + c);
            const int4 a = *reinterpret_cast<const int4 *>(arg + (int64_t)g * C + c);
            d[u] = make_float4(a.x == (int32_t)k ? o.x : 0.f, a.y == (int32_t)k ? o.y : 0.f,
                               a.z == (int32_t)k ? o.z : 0.f, a.w == (int32_t)k ? o.w : 0.f);
        }
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
        const int64_t r = r0 + rl + u * kTrVecLanes;
        if (r >= M) break;
        const float yv[4] = {y[u].x, y[u].y, y[u].z, y[u].w}, dv[4] = {d[u].x, d[u].y, d[u].z, d[u].w};
        float o[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const float xh = tr_xhat(yv[j], mus[j], iss[j]);
            const float dd = !relu || xh * gas[j] + bes[j] > 0.f ? dv[j] : 0.f;
            o[j] = gas[j] * iss[j] * (dd - m1[j] - xh * m2[j]);
        }
        *reinterpret_cast<float4 *>(dY + r * ldy + c) = make_float4(o[0], o[1], o[2], o[3]);
    }
}

// rows per partial chunk of the column sweeps: kTrChunk, halved while the grid (column tiles x
// chunks) would have fewer than kTrMinBlocks blocks -- PointNet-v1 layers have M = B*N = 32k
// rows (32 chunks of 1024: a 64-column layer would run on 32 workgroups), SA layers 500k
inline int64_t chunk_rows(int64_t M, int64_t C) {
    const int64_t tiles = (C + kTrCols - 1) / kTrCols;
    int64_t ch = kTrChunk;
    while (ch > kTrChunkMin && tiles * ((M + ch - 1) / ch) < kTrMinBlocks) ch >>= 1;
    return ch;
}
inline int64_t chunks(int64_t M, int64_t C) { const int64_t ch = chunk_rows(M, C); return (M + ch - 1) / ch; }

}  // namespace pn2

using namespace pn2;

extern "C" int64_t pn2_bn_train_workspace_bytes(int64_t M, int64_t C) {
    if (M <= 0 || C <= 0) return 0;
    return chunks(M, C) * 2 * C * (int64_t)sizeof(double) + 3 * C * (int64_t)sizeof(double);
}

extern "C" int pn2_bn_train_stats_f32(const float *Y, int64_t M, int64_t C, int64_t ld, double eps,
                                      double momentum, float *running_mean, float *running_var,
                                      float *mean, float *invstd, double *sxhat, void *ws,
                                      int64_t ws_bytes, void *stream) {
    PN2_REQUIRE(Y && mean && invstd && sxhat && ws, "pn2_bn_train_stats_f32: null pointer");
    PN2_REQUIRE(M >= 1 && C >= 1 && ld >= C, "pn2_bn_train_stats_f32: bad shape");
    PN2_REQUIRE(ws_bytes >= pn2_bn_train_workspace_bytes(M, C), "pn2_bn_train_stats_f32: workspace too small");
    PN2_REQUIRE(momentum <= 0.0 || (running_mean && running_var), "pn2_bn_train_stats_f32: running stats");
    hipStream_t st = as_stream(stream);
    double *part = static_cast<double *>(ws);
    hipLaunchKernelGGL(bn_stats_partial_kernel, dim3((unsigned)((C + kTrCols - 1) / kTrCols), (unsigned)chunks(M, C)),
                       dim3(256), 0, st, Y, M, C, ld, chunk_rows(M, C), part);
    PN2_LAUNCH_CHECK("bn_stats_partial_kernel");
    hipLaunchKernelGGL(bn_stats_final_kernel, dim3((unsigned)C), dim3(64), 0, st, part, chunks(M, C), M, C,
                       eps, momentum, running_mean, running_var, mean, invstd, sxhat);
    PN2_LAUNCH_CHECK("bn_stats_final_kernel");
    return PN2_OK;
}

extern "C" int pn2_bn_relu_apply_f32(const float *Y, int64_t M, int64_t C, int64_t ld, const float *mean,
                                     const float *invstd, const float *gamma, const float *beta, float *A,
                                     int64_t lda, int flags, void *stream) {
    PN2_REQUIRE(Y && mean && invstd && gamma && beta && A, "pn2_bn_relu_apply_f32: null pointer");
    PN2_REQUIRE(M >= 0 && C >= 1 && ld >= C && lda >= C, "pn2_bn_relu_apply_f32: bad shape");
    PN2_REQUIRE((flags & ~PN2_LAYER_NO_RELU) == 0, "pn2_bn_relu_apply_f32: unknown flags");
    if (M == 0) return PN2_OK;
    hipLaunchKernelGGL(bn_relu_apply_kernel,
                       dim3((unsigned)((C + kTrCols - 1) / kTrCols), (unsigned)((M + kTrEwRows - 1) / kTrEwRows)),
                       dim3(256), 0, as_stream(stream), Y, M, C, ld, mean, invstd, gamma, beta, A, lda,
                       (flags & PN2_LAYER_NO_RELU) ? 0 : 1);
    PN2_LAUNCH_CHECK("bn_relu_apply_kernel");
    return PN2_OK;
}

extern "C" int pn2_bn_train_forward_f32(const float *Y, int64_t M, int64_t C, int64_t ld, double eps,
                                        double momentum, float *running_mean, float *running_var,
                                        const float *gamma, const float *beta, float *A, int64_t lda,
                                        int flags, float *stats, double *sxhat, void *ws, int64_t ws_bytes,
                                        void *stream) {
    PN2_REQUIRE(stats, "pn2_bn_train_forward_f32: null pointer");
    const int rc = pn2_bn_train_stats_f32(Y, M, C, ld, eps, momentum, running_mean, running_var, stats,
                                          stats + C, sxhat, ws, ws_bytes, stream);
    if (rc != PN2_OK) return rc;
    return pn2_bn_relu_apply_f32(Y, M, C, ld, stats, stats + C, gamma, beta, A, lda, flags, stream);
}

extern "C" int pn2_group_max_f32(const float *A, int64_t G, int64_t K, int64_t C, int64_t lda, float *out,
                                 int64_t ldo, int32_t *arg, void *stream) {
    PN2_REQUIRE(A && out && arg, "pn2_group_max_f32: null pointer");
    PN2_REQUIRE(G >= 0 && K >= 1 && K < ((int64_t)1 << 31) && C >= 1 && lda >= C && ldo >= C,
                "pn2_group_max_f32: bad shape");
    if (G == 0) return PN2_OK;
    if (K >= kTrWideK && G < 65536) {
        hipLaunchKernelGGL(group_max_wide_kernel, dim3((unsigned)((C + kTrCols - 1) / kTrCols), (unsigned)G),
                           dim3(kTrCols * kTrWideLanes), 0, as_stream(stream), A, K, C, lda, out, ldo, arg);
        PN2_LAUNCH_CHECK("group_max_wide_kernel");
        return PN2_OK;
    }
    hipLaunchKernelGGL(group_max_kernel, dim3((unsigned)((C + kTrCols - 1) / kTrCols), (unsigned)((G + kTrLanes - 1) / kTrLanes)),
                       dim3(256), 0, as_stream(stream), A, G, K, C, lda, out, ldo, arg);
    PN2_LAUNCH_CHECK("group_max_kernel");
    return PN2_OK;
}

extern "C" int pn2_bn_relu_backward_f32(const float *Y, int64_t M, int64_t C, int64_t ld, const float *mean,
                                        const float *invstd, const float *gamma, const float *beta,
                                        const float *dA, int64_t ldd, const float *dOut, int64_t ldo,
                                        const int32_t *arg, int64_t K, const double *sxhat,
                                        float *dY, int64_t ldy, float *dgamma, float *dbeta,
                                        float *dbias, void *ws, int64_t ws_bytes, int flags, void *stream) {
    PN2_REQUIRE(Y && mean && invstd && gamma && beta && dY && dgamma && dbeta && ws && (!dbias || sxhat),
                "pn2_bn_relu_backward_f32: null pointer");
    PN2_REQUIRE(dA || (dOut && arg && K >= 1 && M % K == 0), "pn2_bn_relu_backward_f32: need dA or (dOut, arg, K)");
    PN2_REQUIRE(M >= 1 && M < ((int64_t)1 << 31) && C >= 1 && ld >= C && ldy >= C && (!dA || ldd >= C) &&
                    (dA || ldo >= C),
                "pn2_bn_relu_backward_f32: bad shape");
    PN2_REQUIRE(ws_bytes >= pn2_bn_train_workspace_bytes(M, C), "pn2_bn_relu_backward_f32: workspace too small");
    PN2_REQUIRE((flags & ~PN2_LAYER_NO_RELU) == 0, "pn2_bn_relu_backward_f32: unknown flags");
    const int relu = (flags & PN2_LAYER_NO_RELU) ? 0 : 1;
    hipStream_t st = as_stream(stream);
    double *part = static_cast<double *>(ws);
    double *sums = part + chunks(M, C) * 2 * C;
    int64_t nch;
    const bool vec4 = (C % 4) == 0 && (ld % 4) == 0 && (ldy % 4) == 0 && (!dA || (ldd % 4) == 0) &&
                      (dA || (ldo % 4) == 0) &&
                      (((uintptr_t)Y | (uintptr_t)dY | (uintptr_t)(dA ? (const void *)dA : (const void *)dOut) |
                        (uintptr_t)(dA ? nullptr : (const void *)arg) | (uintptr_t)mean | (uintptr_t)invstd |
                        (uintptr_t)gamma | (uintptr_t)beta) & 15) == 0;
    if (dA && vec4) {
        nch = chunks(M, C);
        hipLaunchKernelGGL(bn_bwd_partial_vec_kernel, dim3((unsigned)((C + kTrCols - 1) / kTrCols), (unsigned)nch),
                           dim3(256), 0, st, Y, M, C, ld, mean, invstd, gamma, beta, dA, ldd, relu,
                           chunk_rows(M, C), part);
        PN2_LAUNCH_CHECK("bn_bwd_partial_vec_kernel");
    } else if (dA) {
        nch = chunks(M, C);
        hipLaunchKernelGGL(bn_bwd_partial_kernel, dim3((unsigned)((C + kTrCols - 1) / kTrCols), (unsigned)nch),
                           dim3(256), 0, st, Y, M, C, ld, mean, invstd, gamma, beta, dA, ldd, dOut, ldo, arg, K,
                           relu, chunk_rows(M, C), part);
        PN2_LAUNCH_CHECK("bn_bwd_partial_kernel");
    } else {  // scattered from the max: only the G argmax rows contribute
        const int64_t G = M / K, gch = chunk_rows(G, C);
        nch = (G + gch - 1) / gch;
        PN2_REQUIRE(nch <= chunks(M, C), "pn2_bn_relu_backward_f32: gather partials exceed the workspace");
        hipLaunchKernelGGL(bn_bwd_partial_gather_kernel, dim3((unsigned)((C + kTrCols - 1) / kTrCols), (unsigned)nch),
                           dim3(256), 0, st, Y, G, C, ld, mean, invstd, gamma, beta, dOut, ldo, arg, K, relu, gch,
                           part);
        PN2_LAUNCH_CHECK("bn_bwd_partial_gather_kernel");
    }
    hipLaunchKernelGGL(bn_bwd_final_kernel, dim3((unsigned)C), dim3(64), 0, st, part, nch, M, C, gamma,
                       invstd, sxhat, dbeta, dgamma, dbias, sums);
    PN2_LAUNCH_CHECK("bn_bwd_final_kernel");
    const dim3 egrid((unsigned)((C + kTrCols - 1) / kTrCols), (unsigned)((M + kTrEwRows - 1) / kTrEwRows));
    if (vec4) {
        hipLaunchKernelGGL(bn_bwd_apply_vec_kernel, egrid, dim3(256), 0, st, Y, M, C, ld, mean, invstd, gamma,
                           beta, dA, ldd, dOut, ldo, arg, K, relu, sums, dY, ldy);
        PN2_LAUNCH_CHECK("bn_bwd_apply_vec_kernel");
    } else {
        hipLaunchKernelGGL(bn_bwd_apply_kernel, egrid, dim3(256), 0, st, Y, M, C, ld, mean, invstd, gamma, beta,
                           dA, ldd, dOut, ldo, arg, K, relu, sums, dY, ldy);
        PN2_LAUNCH_CHECK("bn_bwd_apply_kernel");
    }
    return PN2_OK;
}
