// ball_query.hip -- query_ball_point for gfx950.
//
// Replaces query_ball_point (/root/reference/model/pointnet2_utils.py:70-90) including the
// square_distance it calls (pointnet2_utils.py:5-26).  The reference materialises the full
// [B,S,N] distance matrix, masks it and SORTS every row to find the first K in-radius indices;
// here one wave owns one centroid and streams the cloud in index order, 64 points per step:
//   d = ((-2 * fma-chain(ctr . p)) + ssq(ctr)) + ssq(p)     (MKL sgemm + ATen sum order;
//       unfused mul/add chain when S*N*C < 400: ATen's naive small-bmm kernel)
//   hit = !(d > (float)(r*r))                                (the reference's masking test)
//   ballot -> popcount prefix -> ordered compaction, early exit once K hits are found.
// No [B,S,N] tensor exists.  Points come from the packed [B][N][cp] records
// (coords, ssq, pad) so one lane's point is one or three 16-byte loads.
#include "pn2_internal.h"

namespace pn2 {

template <int CP, int WPB>
__global__ __launch_bounds__(64 * WPB) void ball_query_kernel(const float *__restrict__ pts,
                                                              const float *__restrict__ ctr,
                                                              int64_t B, int N, int S, int C,
                                                              float r2, int K, int small,
                                                              int64_t *__restrict__ out,
                                                              int *__restrict__ out_cnt) {
    const int lane = threadIdx.x & 63;
    const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int64_t q = (int64_t)blockIdx.x * WPB + w;  // centroid (b*S + s)
    if (q >= B * S) return;
    const int64_t b = q / S;

    // centroid record (wave-uniform)
    float cq[CP];
    const float4 *cptr = reinterpret_cast<const float4 *>(ctr + q * CP);
#pragma unroll
    for (int v = 0; v < CP / 4; ++v) {
        const float4 t = cptr[v];
        cq[4 * v + 0] = t.x; cq[4 * v + 1] = t.y; cq[4 * v + 2] = t.z; cq[4 * v + 3] = t.w;
    }
    const float ssq_c = cq[C];

    const float4 *P = reinterpret_cast<const float4 *>(pts + b * (int64_t)N * CP);
    int64_t *o = out + q * K;
    int cnt = 0;
    int first = N;
    const unsigned long long below = (lane == 0) ? 0ull : (~0ull >> (64 - lane));

    for (int n0 = 0; n0 < N; n0 += 64) {
        const int n = n0 + lane;
        bool hit = false;
        if (n < N) {
            float pp[CP];
#pragma unroll
            for (int v = 0; v < CP / 4; ++v) {
                const float4 t = P[(int64_t)n * (CP / 4) + v];
                pp[4 * v + 0] = t.x; pp[4 * v + 1] = t.y; pp[4 * v + 2] = t.z; pp[4 * v + 3] = t.w;
            }
            float mm = __fmul_rn(cq[0], pp[0]);
            if (small) {
#pragma unroll
                for (int k = 1; k < CP - 1; ++k)
                    if (k < C) mm = __fadd_rn(mm, __fmul_rn(cq[k], pp[k]));
            } else {
#pragma unroll
                for (int k = 1; k < CP - 1; ++k)
                    if (k < C) mm = __builtin_fmaf(cq[k], pp[k], mm);
            }
            const float d = __fadd_rn(__fadd_rn(__fmul_rn(-2.0f, mm), ssq_c), pp[C]);
            hit = !(d > r2);
        }
        const unsigned long long m = __ballot(hit);
        if (m) {
            if (cnt == 0) first = n0 + (int)__builtin_ctzll(m);
            const int pos = cnt + __builtin_popcountll(m & below);
            if (hit && pos < K) o[pos] = n;
            cnt += __builtin_popcountll(m);
            if (cnt >= K) break;
        }
    }
    for (int k = cnt + lane; k < K; k += 64) o[k] = first;
    // distinct neighbours: entries past them repeat entry 0 (the SA chain computes only these)
    if (out_cnt && lane == 0) out_cnt[q] = min(cnt, K);
}

}  // namespace pn2

using namespace pn2;

template <int CP>
static int launch_bq(const float *pp, const float *cp_, int64_t B, int64_t N, int64_t S,
                     int64_t C, float r2, int64_t K, int64_t *out, int *cnt, hipStream_t st) {
    constexpr int WPB = 4;
    const int64_t nq = B * S;
    hipLaunchKernelGGL((ball_query_kernel<CP, WPB>), dim3((unsigned)((nq + WPB - 1) / WPB)),
                       dim3(64 * WPB), 0, st, pp, cp_, B, (int)N, (int)S, (int)C, r2, (int)K,
                       (int)(S * N * C < 400), out, cnt);
    PN2_LAUNCH_CHECK("ball_query_kernel");
    return PN2_OK;
}

extern "C" int pn2_ball_query_f32(const float *pts_packed, const float *ctr_packed, int64_t B,
                                  int64_t N, int64_t S, int64_t C, double radius, int64_t K,
                                  int64_t *out_idx, void *stream) {
    return pn2_ball_query_cnt_f32(pts_packed, ctr_packed, B, N, S, C, radius, K, out_idx, nullptr,
                                  stream);
}

extern "C" int pn2_ball_query_cnt_f32(const float *pts_packed, const float *ctr_packed, int64_t B,
                                      int64_t N, int64_t S, int64_t C, double radius, int64_t K,
                                      int64_t *out_idx, int32_t *out_cnt, void *stream) {
    PN2_REQUIRE(pts_packed && ctr_packed && out_idx, "pn2_ball_query_f32: null pointer");
    PN2_REQUIRE(B >= 0 && N >= 1 && S >= 0 && C >= 1 && C <= kMaxC && K >= 1,
                "pn2_ball_query_f32: bad shape B=%lld N=%lld S=%lld C=%lld K=%lld", (long long)B,
                (long long)N, (long long)S, (long long)C, (long long)K);
    PN2_REQUIRE(K <= N, "pn2_ball_query_f32: sample_number %lld > N %lld", (long long)K,
                (long long)N);
    if (B == 0 || S == 0) return PN2_OK;
    // radius ** 2 in double (Python float), compared in float32 like torch's wrapped scalar
    const float r2 = (float)(radius * radius);
    hipStream_t st = as_stream(stream);
    const int64_t cp = pn2_packed_stride(C);
    if (cp == 4) return launch_bq<4>(pts_packed, ctr_packed, B, N, S, C, r2, K, out_idx, out_cnt, st);
    if (cp == 8) return launch_bq<8>(pts_packed, ctr_packed, B, N, S, C, r2, K, out_idx, out_cnt, st);
    if (cp == 12) return launch_bq<12>(pts_packed, ctr_packed, B, N, S, C, r2, K, out_idx, out_cnt, st);
    if (cp == 16) return launch_bq<16>(pts_packed, ctr_packed, B, N, S, C, r2, K, out_idx, out_cnt, st);
    if (cp == 20) return launch_bq<20>(pts_packed, ctr_packed, B, N, S, C, r2, K, out_idx, out_cnt, st);
    return set_error(PN2_EUNSUPPORTED, "pn2_ball_query_f32: C=%lld", (long long)C);
}

// ------------------------------------------------------------------ square_distance
// The full [B,S,N] matrix of square_distance (pointnet2_utils.py:5-26), for the public
// function of the same name; the SA path never materialises it.
namespace pn2 {
__global__ __launch_bounds__(256) void square_distance_kernel(const float *__restrict__ src,
                                                              const float *__restrict__ dst,
                                                              int64_t B, int64_t S, int64_t N,
                                                              int C, int cp, int small,
                                                              float *__restrict__ out) {
    const int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (e >= B * S * N) return;
    const int64_t n = e % N;
    const int64_t bs = e / N;
    const int64_t b = bs / S;
    const float *q = src + bs * cp;
    const float *p = dst + (b * N + n) * cp;
    float mm = __fmul_rn(q[0], p[0]);
    if (small)
        for (int k = 1; k < C; ++k) mm = __fadd_rn(mm, __fmul_rn(q[k], p[k]));
    else
        for (int k = 1; k < C; ++k) mm = __builtin_fmaf(q[k], p[k], mm);
    out[e] = __fadd_rn(__fadd_rn(__fmul_rn(-2.0f, mm), q[C]), p[C]);
}
}  // namespace pn2

extern "C" int pn2_square_distance_f32(const float *src_packed, const float *dst_packed,
                                       int64_t B, int64_t S, int64_t N, int64_t C, float *out,
                                       void *stream) {
    PN2_REQUIRE(src_packed && dst_packed && out, "pn2_square_distance_f32: null pointer");
    PN2_REQUIRE(B >= 0 && S >= 0 && N >= 0 && C >= 1 && C <= kMaxC, "pn2_square_distance_f32: bad shape");
    const int64_t tot = B * S * N;
    if (tot == 0) return PN2_OK;
    hipLaunchKernelGGL(square_distance_kernel, dim3((unsigned)((tot + 255) / 256)), dim3(256), 0,
                       as_stream(stream), src_packed, dst_packed, B, S, N, (int)C,
                       (int)pn2_packed_stride(C), (int)(S * N * C < 400), out);
    PN2_LAUNCH_CHECK("square_distance_kernel");
    return PN2_OK;
}
