// linear.hip -- small-batch fully connected layer: out = act(x W^T + bias), rows in blocks of
// 16.
//
// Reference: the FC tails of the PointNet-v1 networks, /root/reference/model/pointnet_utils.py:
// 36-40 (T-Net fc1-fc3 + bn4/bn5), pointnet_cls.py:26-28 and the v1 heads' fc / bn_fc stacks
// (rotation.py:45-49), with each eval BatchNorm1d folded into W and bias on the host
// (pn2/pointnet_utils.py linear_bn).  At a few rows these are matrix-vector products:
// the weight (up to 1024 x 4096 floats) is read once, so the bound is HBM bytes of W -- and in
// practice the launch: the library GEMMs chosen for these shapes run 5-13 us each, several
// times the weight's read time.
//
// Layout: one workgroup of 4 waves per kLinRows (4 or 2 by the row count) consecutive output
// features; the four waves split K (256-float chunk c goes to wave c % 4), each lane walking its
// chunks with 16-byte loads of the W rows (coalesced: a wave reads 1 KB of a row per chunk) and
// of the x rows (L2 resident: x is at most 16 x K floats), accumulating kLinRows x B partial
// dot products in registers; then a transpose-reduce across each wave (32 shuffles for the 32
// sums) and the four waves' sums added in LDS in wave order.  With K split over the waves
// every load of a layer is in flight at once (one wave walking all of K waited for its loads
// chunk by chunk: 9.8 us for 1024->512 at B=32, latency-bound).  Float32 FMA throughout (the
// library GEMM's arithmetic; the summation order differs, as between any two GEMM kernels).
// More rows run as blocks of 16 (grid.y).
#include "pn2_internal.h"

namespace pn2 {

constexpr int kLinWaves = 4;   // waves per workgroup (they split K)

// output features per wave: kLinRows x BT accumulators stay within ~128 VGPRs
template <int BT>
constexpr int lin_rows() { return BT <= 8 ? 4 : 2; }

// one transpose-reduce step over lane bit 2H: keep H of the 2H values, add the partner's copy
// (H is a template parameter so every register index is static)
template <int H>
__device__ __forceinline__ void lin_reduce_step(float *a, int lane) {
    const bool up = (lane & (2 * H)) != 0;
#pragma unroll
    for (int i = 0; i < H; ++i) {
        const float send = up ? a[i] : a[i + H];
        const float keep = up ? a[i + H] : a[i];
        a[i] = keep + __shfl_xor(send, 2 * H);
    }
}

// one workgroup's block: output features blockIdx.x * kLinRows.., rows blockIdx.y * BT..
template <int BT>
__device__ __forceinline__ void linear_rows_block(const float *__restrict__ x, int64_t ldx, int B, int64_t K,
                                                  const float *__restrict__ W,
                                                  const float *__restrict__ bias,
                                                  float *__restrict__ out, int64_t ldo, int64_t N,
                                                  int relu, int vec) {
    constexpr int kLinRows = lin_rows<BT>();
    const int lane = threadIdx.x & 63;
    // row block blockIdx.y: every output element is computed the same way whatever B is (the
    // per-lane FMA order depends on k only, the reduction tree on the lane only), so a batch
    // split into shards gives bit-identical rows
    x += (int64_t)blockIdx.y * BT * ldx;
    out += (int64_t)blockIdx.y * BT * ldo;
    B = B - (int)blockIdx.y * BT < BT ? B - (int)blockIdx.y * BT : BT;
    const int wave = threadIdx.x / 64;
    const int64_t o0 = (int64_t)blockIdx.x * kLinRows;
    float acc[kLinRows][BT];
#pragma unroll
    for (int r = 0; r < kLinRows; ++r)
#pragma unroll
        for (int b = 0; b < BT; ++b) acc[r][b] = 0.f;
    // row pointers clamped into range instead of guarded: every load of an iteration issues
    // back to back (a branch per row made each wait for the previous one); the rows past B or N
    // accumulate duplicates that are never stored
    const float *wr[kLinRows];
#pragma unroll
    for (int r = 0; r < kLinRows; ++r) wr[r] = W + (o0 + r < N ? o0 + r : N - 1) * K;
    const float *xr[BT];
#pragma unroll
    for (int b = 0; b < BT; ++b) xr[b] = x + (int64_t)(b < B ? b : B - 1) * ldx;
    if (vec) {  // 16-byte aligned rows (host-checked)
        for (int64_t k = (int64_t)wave * 256 + lane * 4; k < K; k += 256 * kLinWaves) {
            float4 w[kLinRows], v[BT];
#pragma unroll
            for (int r = 0; r < kLinRows; ++r) w[r] = *reinterpret_cast<const float4 *>(wr[r] + k);
#pragma unroll
            for (int b = 0; b < BT; ++b) v[b] = *reinterpret_cast<const float4 *>(xr[b] + k);
#pragma unroll
            for (int b = 0; b < BT; ++b) {
#pragma unroll
                for (int r = 0; r < kLinRows; ++r) {
                    float a = acc[r][b];
                    a = fmaf(w[r].x, v[b].x, a);
                    a = fmaf(w[r].y, v[b].y, a);
                    a = fmaf(w[r].z, v[b].z, a);
                    a = fmaf(w[r].w, v[b].w, a);
                    acc[r][b] = a;
                }
            }
        }
    } else {
        for (int64_t k = (int64_t)wave * 64 + lane; k < K; k += 64 * kLinWaves) {
            float w[kLinRows], v[BT];
#pragma unroll
            for (int r = 0; r < kLinRows; ++r) w[r] = wr[r][k];
#pragma unroll
            for (int b = 0; b < BT; ++b) v[b] = xr[b][k];
#pragma unroll
            for (int b = 0; b < BT; ++b)
#pragma unroll
                for (int r = 0; r < kLinRows; ++r) acc[r][b] = fmaf(w[r], v[b], acc[r][b]);
        }
    }
    // transpose-reduce: kLinRows x BT = 32 partial sums per lane.  Each xor step keeps half
    // of the values and adds the partner lane's copy of that half (one shuffle per kept value:
    // 16 + 8 + 4 + 2 + 1 + 1 = 32 shuffles, not 32 x 6); lane L ends with value (L >> 1) & 31
    static_assert(kLinRows * BT == 32, "32 values per lane");
    float a[32];
#pragma unroll
    for (int r = 0; r < kLinRows; ++r)
#pragma unroll
        for (int b = 0; b < BT; ++b) a[r * BT + b] = acc[r][b];
    lin_reduce_step<16>(a, lane);
    lin_reduce_step<8>(a, lane);
    lin_reduce_step<4>(a, lane);
    lin_reduce_step<2>(a, lane);
    lin_reduce_step<1>(a, lane);
    a[0] += __shfl_xor(a[0], 1);
    const int v = (lane >> 1) & 31, r = v / BT, b = v % BT;
    // the waves' sums, added in wave order (the same order for every row count)
    __shared__ float red[kLinWaves][32];
    if ((lane & 1) == 0) red[wave][v] = a[0];
    __syncthreads();
    if (wave == 0 && (lane & 1) == 0 && b < B && o0 + r < N) {
        float y = red[0][v];
#pragma unroll
        for (int w = 1; w < kLinWaves; ++w) y += red[w][v];
        y += bias ? bias[o0 + r] : 0.f;
        out[b * ldo + o0 + r] = relu ? (y > 0.f ? y : 0.f) : y;
    }
}

template <int BT>
__global__ __launch_bounds__(64 * kLinWaves) void linear_rows_kernel(const float *__restrict__ x, int64_t ldx,
                                                                     int B, int64_t K,
                                                                     const float *__restrict__ W,
                                                                     const float *__restrict__ bias,
                                                                     float *__restrict__ out, int64_t ldo,
                                                                     int64_t N, int relu, int vec) {
    linear_rows_block<BT>(x, ldx, B, K, W, bias, out, ldo, N, relu, vec);
}

// ---- the heads' FC tail, last layer: fc3 for kTailRows rows per workgroup and, with
// PN2_TAIL_LOGSOFTMAX, log_softmax and the first argmax of each row (pointnet2_cls_ssg.py:36-38:
// F.log_softmax(x, -1) and x.data.max(1)[1]) -- one launch, after fc1 and fc2 as
// linear_rows_kernel launches.  (An in-launch fc2 -> fc3 seam, an arrival ticket with the last
// workgroup computing fc3, cost 10-15 us over the separate launches: the fan-in of the ~128
// arrivals and their skew; MI355X_MICROARCH.md's splitk-seam / fanin rows.)
// fc3 element (b, n) is the in-order sum of kTailKS partial fma chains over consecutive
// segments of k: one thread per (n, segment) holds the workgroup's kTailRows rows, its weight
// segment read once.  The order depends on the shape only, never on the row count (sharded
// batches stay bit-identical).
constexpr int kTailKS = 4, kTailRows = 4;
constexpr int kTailT = 256;

template <bool VEC>
__global__ __launch_bounds__(kTailT) void fc3_tail_kernel(const float *__restrict__ y2, int B, int64_t N2,
                                                          const float *__restrict__ W3,
                                                          const float *__restrict__ b3, int N3, int flags,
                                                          float *__restrict__ out, int64_t ldo,
                                                          int64_t *__restrict__ amax) {
    extern __shared__ __attribute__((aligned(16))) float tsm[];
    float *logits = tsm;                          // [kTailRows][N3]
    float *part = tsm + kTailRows * N3;           // [kTailKS][kTailRows][N3]
    float *sy = part + kTailKS * kTailRows * N3;  // VEC: [kTailRows][N2], 16-byte aligned
    const int r0 = (int)blockIdx.x * kTailRows;
    const int R = B - r0 < kTailRows ? B - r0 : kTailRows;
    y2 += (int64_t)r0 * N2;
    out += (int64_t)r0 * ldo;
    const int64_t kl = VEC ? N2 / kTailKS : (N2 + kTailKS - 1) / kTailKS;
    const int items = N3 * kTailKS;
    if constexpr (VEC) {
        // one round trip: the thread's first weight chunk (kC float4 of its row segment) in
        // flight together with the rows' y2 staging into LDS; lanes then read y2 from LDS at one
        // address per k (a broadcast)
        constexpr int kC = 16;
        float4 w[kC];
        auto load_w = [&](int it, int64_t kb) {
            const int n = it % N3, q = it / N3;
            const int64_t k1 = q * kl + kl;
            const float *wr = W3 + (int64_t)n * N2;
#pragma unroll
            for (int u = 0; u < kC; ++u) {
                const int64_t k = kb + 4 * u < k1 ? kb + 4 * u : k1 - 4;  // clamped, not used
                w[u] = *reinterpret_cast<const float4 *>(wr + k);
            }
        };
        if ((int)threadIdx.x < items) load_w(threadIdx.x, (threadIdx.x / N3) * kl);
        const float4 *y4 = reinterpret_cast<const float4 *>(y2);
        for (int64_t e = threadIdx.x; e < (int64_t)R * N2 / 4; e += kTailT) reinterpret_cast<float4 *>(sy)[e] = y4[e];
        __syncthreads();
        for (int it = threadIdx.x; it < items; it += kTailT) {
            const int n = it % N3, q = it / N3;
            const int64_t k0 = q * kl, k1 = k0 + kl;
            float acc[kTailRows];
#pragma unroll
            for (int i = 0; i < kTailRows; ++i) acc[i] = 0.f;
            for (int64_t kb = k0; kb < k1; kb += 4 * kC) {
                if (it != (int)threadIdx.x || kb != k0) load_w(it, kb);
#pragma unroll
                for (int u = 0; u < kC; ++u)
                    if (kb + 4 * u < k1)
#pragma unroll
                        for (int i = 0; i < kTailRows; ++i) {
                            const float4 y =
                                *reinterpret_cast<const float4 *>(sy + (int64_t)(i < R ? i : R - 1) * N2 + kb + 4 * u);
                            float a = acc[i];
                            a = fmaf(w[u].x, y.x, a);
                            a = fmaf(w[u].y, y.y, a);
                            a = fmaf(w[u].z, y.z, a);
                            a = fmaf(w[u].w, y.w, a);
                            acc[i] = a;
                        }
            }
#pragma unroll
            for (int i = 0; i < kTailRows; ++i) part[(q * kTailRows + i) * N3 + n] = acc[i];
        }
    } else {
        const float *yr[kTailRows];
#pragma unroll
        for (int i = 0; i < kTailRows; ++i) yr[i] = y2 + (int64_t)(i < R ? i : R - 1) * N2;
        for (int it = threadIdx.x; it < items; it += kTailT) {
            const int n = it % N3, q = it / N3;
            const int64_t k0 = q * kl, k1 = k0 + kl < N2 ? k0 + kl : N2;
            const float *wr = W3 + (int64_t)n * N2;
            float acc[kTailRows];
#pragma unroll
            for (int i = 0; i < kTailRows; ++i) acc[i] = 0.f;
            for (int64_t k = k0; k < k1; ++k) {
                const float w = wr[k];
#pragma unroll
                for (int i = 0; i < kTailRows; ++i) acc[i] = fmaf(w, yr[i][k], acc[i]);
            }
#pragma unroll
            for (int i = 0; i < kTailRows; ++i) part[(q * kTailRows + i) * N3 + n] = acc[i];
        }
    }
    __syncthreads();
    for (int e = threadIdx.x; e < R * N3; e += kTailT) {
        const int b = e / N3, n = e - b * N3;
        float a = part[e];
#pragma unroll
        for (int q = 1; q < kTailKS; ++q) a += part[q * kTailRows * N3 + e];
        a += b3 ? b3[n] : 0.f;
        if (flags & PN2_TAIL_LOGSOFTMAX) logits[e] = a;
        else out[(int64_t)b * ldo + n] = a;
    }
    if (flags & PN2_TAIL_LOGSOFTMAX) {
        __syncthreads();
        // one wave per row: max, sum of exp and the first argmax as wave reductions
        const int lane = threadIdx.x & 63, wave = threadIdx.x / 64;
        for (int b = wave; b < R; b += kTailT / 64) {
            const float *v = logits + b * N3;
            float m = -INFINITY;
            for (int n = lane; n < N3; n += 64) m = fmaxf(m, v[n]);
#pragma unroll
            for (int o = 32; o >= 1; o >>= 1) m = fmaxf(m, __shfl_xor(m, o));
            float sum = 0.f;
            for (int n = lane; n < N3; n += 64) sum += expf(v[n] - m);
#pragma unroll
            for (int o = 32; o >= 1; o >>= 1) sum += __shfl_xor(sum, o);
            const float ls = logf(sum);
            float best = -INFINITY;
            int bi = N3;
            for (int n = lane; n < N3; n += 64) {
                const float o = (v[n] - m) - ls;
                out[(int64_t)b * ldo + n] = o;
                if (o > best) best = o, bi = n;  // the lane's first maximum
            }
#pragma unroll
            for (int o = 32; o >= 1; o >>= 1) {  // the first index among equal maxima
                const float ob = __shfl_xor(best, o);
                const int oi = __shfl_xor(bi, o);
                if (ob > best || (ob == best && oi < bi)) best = ob, bi = oi;
            }
            if (amax && lane == 0) amax[r0 + b] = bi < N3 ? bi : 0;
        }
    }
}

}  // namespace pn2

using namespace pn2;

extern "C" int pn2_linear_rows_f32(const float *x, int64_t ldx, int64_t B, int64_t K, const float *W,
                                   const float *bias, float *out, int64_t ldo, int64_t N, int flags,
                                   void *stream) {
    PN2_REQUIRE(x && W && out, "pn2_linear_rows_f32: null pointer");
    PN2_REQUIRE(B >= 1 && (B + 15) / 16 <= 65535 && K >= 1 && N >= 1 && ldx >= K && ldo >= N,
                "pn2_linear_rows_f32: bad shape");
    PN2_REQUIRE((flags & ~PN2_LINEAR_RELU) == 0, "pn2_linear_rows_f32: unknown flags");
    // 16-byte loads when every row start is 16-byte aligned, else the scalar path
    const int vec = ((reinterpret_cast<uintptr_t>(x) | reinterpret_cast<uintptr_t>(W)) & 15) == 0 &&
                    (K & 3) == 0 && (ldx & 3) == 0;
    const int relu = (flags & PN2_LINEAR_RELU) ? 1 : 0;
    hipStream_t st = as_stream(stream);
    auto grid = [N, B](int rows, int bt) {
        return dim3((unsigned)((N + rows - 1) / rows), (unsigned)((B + bt - 1) / bt));
    };
    const dim3 block(64 * kLinWaves);
    if (B <= 8)
        hipLaunchKernelGGL(linear_rows_kernel<8>, grid(lin_rows<8>(), 8), block, 0, st, x, ldx, (int)B, K, W, bias,
                           out, ldo, N, relu, vec);
    else
        hipLaunchKernelGGL(linear_rows_kernel<16>, grid(lin_rows<16>(), 16), block, 0, st, x, ldx, (int)B, K, W, bias,
                           out, ldo, N, relu, vec);
    PN2_LAUNCH_CHECK("linear_rows_kernel");
    return PN2_OK;
}

static int64_t tail_ws_floats(int64_t B, int64_t N1, int64_t N2) {
    return (B * N1 + 3) / 4 * 4 + (B * N2 + 3) / 4 * 4;
}

extern "C" int64_t pn2_fc_tail_workspace_bytes(int64_t B, int64_t N1, int64_t N2) {
    if (B < 1 || N1 < 1 || N2 < 1) return -1;
    return tail_ws_floats(B, N1, N2) * 4;
}

extern "C" int pn2_fc_tail_f32(const float *x, int64_t ldx, int64_t B, int64_t K, const float *W1,
                               const float *b1, int64_t N1, const float *W2, const float *b2, int64_t N2,
                               const float *W3, const float *b3, int64_t N3, int flags, float *out,
                               int64_t ldo, int64_t *argmax, void *workspace, int64_t workspace_bytes,
                               void *stream) {
    PN2_REQUIRE(x && W1 && W2 && W3 && out && workspace, "pn2_fc_tail_f32: null pointer");
    PN2_REQUIRE(B >= 1 && (B + 15) / 16 <= 65535 && K >= 1 && N1 >= 1 && N2 >= 1 && N3 >= 1 &&
                    ldx >= K && ldo >= N3, "pn2_fc_tail_f32: bad shape");
    PN2_REQUIRE((flags & ~PN2_TAIL_LOGSOFTMAX) == 0, "pn2_fc_tail_f32: unknown flags");
    const size_t lds = (size_t)(1 + kTailKS) * kTailRows * N3 * 4;
    PN2_REQUIRE(lds <= 64 * 1024, "pn2_fc_tail_f32: N3 = %lld exceeds %d", (long long)N3,
                64 * 1024 / (4 * (1 + kTailKS) * kTailRows));
    const size_t lds_vec = (lds + 15) / 16 * 16 + (size_t)kTailRows * N2 * 4;  // + the y2 rows
    PN2_REQUIRE(workspace_bytes >= pn2_fc_tail_workspace_bytes(B, N1, N2) && ((uintptr_t)workspace & 15) == 0,
                "pn2_fc_tail_f32: workspace too small or not 16-byte aligned");
    float *y1 = reinterpret_cast<float *>(workspace);
    float *y2 = y1 + (B * N1 + 3) / 4 * 4;
    if (const int rc = pn2_linear_rows_f32(x, ldx, B, K, W1, b1, y1, N1, N1, PN2_LINEAR_RELU, stream)) return rc;
    if (const int rc = pn2_linear_rows_f32(y1, N1, B, N1, W2, b2, y2, N2, N2, PN2_LINEAR_RELU, stream)) return rc;
    // 16-byte loads when the weight rows and the y2 rows are 16-byte aligned and k splits into
    // kTailKS segments of whole float4s (a shape-only choice: the summation order with it)
    const bool vec = (reinterpret_cast<uintptr_t>(W3) & 15) == 0 && N2 % (4 * kTailKS) == 0 &&
                     lds_vec <= 64 * 1024;
    const dim3 grid((unsigned)((B + kTailRows - 1) / kTailRows)), block(kTailT);
    hipStream_t st = as_stream(stream);
    if (vec)
        hipLaunchKernelGGL(fc3_tail_kernel<true>, grid, block, lds_vec, st, y2, (int)B, N2, W3, b3, (int)N3, flags, out,
                           ldo, argmax);
    else
        hipLaunchKernelGGL(fc3_tail_kernel<false>, grid, block, lds, st, y2, (int)B, N2, W3, b3, (int)N3, flags, out,
                           ldo, argmax);
    PN2_LAUNCH_CHECK("fc3_tail_kernel");
    return PN2_OK;
}
