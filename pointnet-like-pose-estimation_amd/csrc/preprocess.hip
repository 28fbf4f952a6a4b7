// preprocess.hip -- the input preparation the reference's scripts run on the host before every
// forward, as one kernel writing the model's input in HBM.
//
// Reference sequence (test_translation.py:72-79, test_rotation.py:71-77, train_*.py:113-118
// without the augmentations; /root/reference/provider.py):
//   points = points.data.numpy()                 float64 [B,N,C] (np.loadtxt rows)
//   mean   = np.mean(points[:, :3, :], axis=1)   translation heads only: the first 3 POINTS
//   points[:, :, 0:3] = provider.normalization(points[:, :, 0:3])        provider.py:5-21
//   points = torch.Tensor(points)                float32 (round to nearest even)
//   points = provider.splice_torch(points, label)                        provider.py:166-180
//   points = points.transpose(2, 1)              [B, C+K, N] view of [B, N, C+K] storage
//
// normalization() per cloud, in float64 with numpy's operation order (measured here,
// tests/test_preprocess.py): centroid = np.mean(pc, axis=0) -- an axis-0 reduction adds the
// rows sequentially, starting from row 0, then divides by N; pc - centroid; pc ** 2 is x*x;
// np.sum(axis=1) over 3 columns is ((x2 + y2) + z2); sqrt is correctly rounded; the max is
// exact (NaN propagates); pc / m is a correctly rounded division.  The unit is built without
// FMA contraction (Makefile GEOFLAGS), so every op rounds separately as numpy's do.
//
// One workgroup per cloud.  The two sequential sums (centroid over N points, mean over the
// first 3) are inherently serial in numpy's rounding order: a few lanes of wave 0 run them
// (the centroid from LDS chunks the other waves stage ahead); everything else is per point.
#include "pn2_internal.h"

namespace pn2 {

constexpr int kPrepThreads = 256;
constexpr int kPrepChunk = 1024;  // points per LDS chunk of the centroid sum (2 x 24 KB)

__device__ __forceinline__ double nan_max(double a, double b) {
    return (a > b || a != a) ? a : b;  // np.max: NaN wins
}

__global__ __launch_bounds__(kPrepThreads) void prepare_kernel(
    const double *__restrict__ pts, int64_t N, int C, int64_t sb, int64_t sn, int64_t sc,
    const int64_t *__restrict__ labels, int K, int normalize, float *__restrict__ out,
    float *__restrict__ mean_out) {
    __shared__ double cen[3];
    __shared__ double chunk[2][kPrepChunk * 3];
    __shared__ double wmax[kPrepThreads / 64];
    const int tid = threadIdx.x;
    const int64_t b = blockIdx.x;
    const double *P = pts + b * sb;

    // mean of the first min(3, N) points, every channel (before normalising)
    if (mean_out && tid < C) {
        const int64_t cnt = N < 3 ? N : 3;
        double s = P[(int64_t)tid * sc];
        for (int64_t n = 1; n < cnt; ++n) s = __dadd_rn(s, P[n * sn + (int64_t)tid * sc]);
        mean_out[b * C + tid] = (float)__ddiv_rn(s, (double)cnt);
    }
    if (!normalize) {
        for (int64_t n = tid; n < N; n += kPrepThreads) {
            float *o = out + (b * N + n) * (C + K);
            for (int c = 0; c < C; ++c) o[c] = (float)P[n * sn + (int64_t)c * sc];
            for (int k = 0; k < K; ++k) o[C + k] = (labels[b] == k) ? 1.f : 0.f;
        }
        return;
    }
    // centroid: sequential sum from row 0 by lanes 0..2 of wave 0, reading the cloud from LDS
    // in chunks that waves 1..3 stage one chunk ahead (double-buffered): the dependent add
    // chain, not global-load latency, sets the time
    {
        const int64_t nch = (N + kPrepChunk - 1) / kPrepChunk;
        auto stage = [&](int64_t k) {
            double *dst = chunk[k & 1];
            const int64_t n0 = k * kPrepChunk;
            const int64_t cnt = (N - n0 < kPrepChunk ? N - n0 : kPrepChunk) * 3;
            for (int64_t e = tid - 64; e < cnt; e += kPrepThreads - 64) {
                const int64_t n = n0 + e / 3;
                dst[e] = P[n * sn + (e % 3) * sc];
            }
        };
        if (tid >= 64) stage(0);
        __syncthreads();
        double s = 0.0;
        for (int64_t k = 0; k < nch; ++k) {
            if (tid >= 64) {
                if (k + 1 < nch) stage(k + 1);
            } else if (tid < 3) {
                const double *src = chunk[k & 1] + tid;
                const int cnt = (int)(N - k * kPrepChunk < kPrepChunk ? N - k * kPrepChunk : kPrepChunk);
                int j = 0;
                if (k == 0) s = src[0], j = 1;  // numpy starts from row 0
                for (; j + 8 <= cnt; j += 8) {
                    double v[8];
#pragma unroll
                    for (int u = 0; u < 8; ++u) v[u] = src[3 * (j + u)];
#pragma unroll
                    for (int u = 0; u < 8; ++u) s = __dadd_rn(s, v[u]);
                }
                for (; j < cnt; ++j) s = __dadd_rn(s, src[3 * j]);
            }
            __syncthreads();
        }
        if (tid < 3) cen[tid] = __ddiv_rn(s, (double)N);
    }
    __syncthreads();
    const double c0 = cen[0], c1 = cen[1], c2 = cen[2];
    // m = max_n sqrt((x^2 + y^2) + z^2) of the centred points
    double m = -__builtin_inf();
    for (int64_t n = tid; n < N; n += kPrepThreads) {
        const double *p = P + n * sn;
        const double x = __dsub_rn(p[0], c0), y = __dsub_rn(p[sc], c1), z = __dsub_rn(p[2 * sc], c2);
        const double d = __dsqrt_rn(__dadd_rn(__dadd_rn(__dmul_rn(x, x), __dmul_rn(y, y)), __dmul_rn(z, z)));
        m = nan_max(m, d);
    }
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) m = nan_max(m, __shfl_xor(m, off));
    if ((tid & 63) == 0) wmax[tid >> 6] = m;
    __syncthreads();
#pragma unroll
    for (int w = 0; w < kPrepThreads / 64; ++w) m = nan_max(m, wmax[w]);
    // out row: normalised xyz, other channels as they are, one-hot of the label
    for (int64_t n = tid; n < N; n += kPrepThreads) {
        const double *p = P + n * sn;
        float *o = out + (b * N + n) * (C + K);
        o[0] = (float)__ddiv_rn(__dsub_rn(p[0], c0), m);
        o[1] = (float)__ddiv_rn(__dsub_rn(p[sc], c1), m);
        o[2] = (float)__ddiv_rn(__dsub_rn(p[2 * sc], c2), m);
        for (int c = 3; c < C; ++c) o[c] = (float)p[(int64_t)c * sc];
        for (int k = 0; k < K; ++k) o[C + k] = (labels[b] == k) ? 1.f : 0.f;
    }
}

}  // namespace pn2

using namespace pn2;

extern "C" int pn2_prepare_points_f64(const double *pts, int64_t B, int64_t N, int64_t C,
                                      int64_t sb, int64_t sn, int64_t sc, int normalize,
                                      const int64_t *labels, int64_t num_category, float *out,
                                      float *mean_out, void *stream) {
    PN2_REQUIRE(pts && out, "pn2_prepare_points_f64: null pointer");
    PN2_REQUIRE(B >= 0 && N >= 1 && C >= (normalize ? 3 : 1) && C <= 64,
                "pn2_prepare_points_f64: bad shape (B=%lld N=%lld C=%lld)", (long long)B,
                (long long)N, (long long)C);
    PN2_REQUIRE(num_category >= 0 && num_category <= 1024 && (num_category == 0 || labels),
                "pn2_prepare_points_f64: bad num_category / labels");
    if (B == 0) return PN2_OK;
    hipLaunchKernelGGL(prepare_kernel, dim3((unsigned)B), dim3(kPrepThreads), 0,
                       as_stream(stream), pts, N, (int)C, sb, sn, sc, labels, (int)num_category,
                       normalize ? 1 : 0, out, mean_out);
    PN2_LAUNCH_CHECK("prepare_kernel");
    return PN2_OK;
}
