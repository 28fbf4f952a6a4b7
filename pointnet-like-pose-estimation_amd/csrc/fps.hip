// fps.hip -- farthest point sampling for gfx950.
//
// Replaces farthest_point_sample (/root/reference/model/pointnet2_utils.py:47-68) and the
// index_points(points, fps_idx) that follows it (pointnet2_utils.py:106, 201).
//
// One workgroup per cloud.  The cloud lives in registers for the whole run (PPT points per
// lane, point n = j*NT + lane-in-block so the loads coalesce for the reference's [B,C,N]
// input), the running min-distance too (as the uint bits of a non-negative float, so every
// compare/max is an integer op).  One iteration =
//   distance of every point to the current centroid in the reference's exact float32 order
//   (differences, exact squares, layout-dependent channel sum, no FMA contraction) ->
//   strict-< min update -> per-lane argmax -> wave argmax by DPP (max value, then min index:
//   torch.max returns the FIRST maximum) -> [NW > 1] one LDS slot per wave + ONE barrier
//   (slots double-buffered by iteration parity) -> every wave re-reduces the NW slots itself,
//   so the new centroid's coordinates arrive by v_readlane / LDS broadcast with no second
//   barrier.
// The sampled indices are kept in LDS and written, with the gathered centroids and the packed
// (coords, ssq) records the ball query reads, after the serial loop.
#include "pn2_internal.h"

namespace pn2 {

constexpr int kFpsMaxS = 8192;

template <int NT, int PPT, int CM, bool FIXED>
__global__ __launch_bounds__(NT) void fps_kernel(const float *__restrict__ pts, int N, int Crt,
                                                 int64_t sb, int64_t sn, int64_t sc, int kind,
                                                 const int64_t *__restrict__ start, int S,
                                                 int64_t *__restrict__ out_idx,
                                                 float *__restrict__ out_pts,
                                                 float *__restrict__ out_packed,
                                                 float *__restrict__ pts_packed, int cp) {
    constexpr int NW = NT / 64;
    constexpr int SLOT = CM + 2;
    const int C = FIXED ? CM : Crt;
    const int tid = threadIdx.x;
    const int lane = tid & 63;
    const int wave = tid >> 6;
    const int b = blockIdx.x;
    const float *P = pts + (int64_t)b * sb;

    __shared__ int sidx[kFpsMaxS];
    __shared__ float slots[2][NW][SLOT];

    // ---- load the cloud into registers (and emit the packed copy for the ball query)
    float p[PPT][CM];
    unsigned dist[PPT];
#pragma unroll
    for (int j = 0; j < PPT; ++j) {
        const int n = j * NT + tid;
        const bool valid = n < N;
#pragma unroll
        for (int k = 0; k < CM; ++k)
            p[j][k] = (valid && k < C) ? P[(int64_t)n * sn + (int64_t)k * sc] : 0.f;
        dist[j] = valid ? __float_as_uint(1e10f) : 0u;
        if (valid && pts_packed) {
            float sq[CM];
#pragma unroll
            for (int k = 0; k < CM; ++k) sq[k] = __fmul_rn(p[j][k], p[j][k]);
            float *dst = pts_packed + ((int64_t)b * N + n) * cp;
#pragma unroll
            for (int k = 0; k < CM; ++k)
                if (k < C) dst[k] = p[j][k];
            dst[C] = layout_sum<CM>(sq, C, point_rule(kind, n, N));
            for (int k = C + 1; k < cp; ++k) dst[k] = 0.f;
        }
    }

    // ---- serial loop
    int far = (int)start[b];
    float c[CM];
#pragma unroll
    for (int k = 0; k < CM; ++k) c[k] = (k < C) ? P[(int64_t)far * sn + (int64_t)k * sc] : 0.f;

    for (int i = 0; i < S; ++i) {
        if (tid == 0) sidx[i] = far;
        if (i == S - 1) break;

        unsigned bv = 0u, bi = 0xFFFFFFFFu;
        float bc[CM];
#pragma unroll
        for (int k = 0; k < CM; ++k) bc[k] = 0.f;
#pragma unroll
        for (int j = 0; j < PPT; ++j) {
            const int n = j * NT + tid;
            if (n < N) {
                float sq[CM];
#pragma unroll
                for (int k = 0; k < CM; ++k) {
                    const float d = __fsub_rn(p[j][k], c[k]);
                    sq[k] = __fmul_rn(d, d);
                }
                const float dd = layout_sum<CM>(sq, C, point_rule(kind, n, N));
                const unsigned db = __float_as_uint(dd);
                if (db < dist[j]) dist[j] = db;
                if (j == 0 || dist[j] > bv) {
                    bv = dist[j];
                    bi = (unsigned)n;
#pragma unroll
                    for (int k = 0; k < CM; ++k) bc[k] = p[j][k];
                }
            }
        }
        // wave argmax (first index among maxima)
        const unsigned wv = wave_max_u32(bv);
        const unsigned wi = wave_min_u32(bv == wv ? bi : 0xFFFFFFFFu);
        const unsigned long long own = __ballot(bi == wi);
        const int owner = own ? (int)__builtin_ctzll(own) : 0;
        if (NW == 1) {
#pragma unroll
            for (int k = 0; k < CM; ++k)
                c[k] = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(bc[k]), owner));
            far = (int)wi;
        } else {
            const int par = i & 1;
            if (lane == owner) {
                slots[par][wave][0] = __uint_as_float(wv);
                slots[par][wave][1] = __uint_as_float(wi);
#pragma unroll
                for (int k = 0; k < CM; ++k) slots[par][wave][2 + k] = bc[k];
            }
            __syncthreads();
            unsigned rv = 0u, ri = 0xFFFFFFFFu;
            if (lane < NW) {
                rv = __float_as_uint(slots[par][lane][0]);
                ri = __float_as_uint(slots[par][lane][1]);
            }
            const unsigned gv = wave_max_u32(rv);
            const unsigned gi = wave_min_u32(rv == gv ? ri : 0xFFFFFFFFu);
            const unsigned long long gown = __ballot(lane < NW && ri == gi);
            const int ow = (int)__builtin_ctzll(gown);
#pragma unroll
            for (int k = 0; k < CM; ++k) c[k] = slots[par][ow][2 + k];
            far = (int)gi;
        }
    }
    __syncthreads();

    // ---- outputs: indices, gathered centroids (index_points), packed centroids
    for (int i = tid; i < S; i += NT) {
        const int n = sidx[i];
        out_idx[(int64_t)b * S + i] = n;
        if (out_pts || out_packed) {
            float q[CM], sq[CM];
#pragma unroll
            for (int k = 0; k < CM; ++k) {
                q[k] = (k < C) ? P[(int64_t)n * sn + (int64_t)k * sc] : 0.f;
                sq[k] = __fmul_rn(q[k], q[k]);
            }
            if (out_pts) {
                float *o = out_pts + ((int64_t)b * S + i) * C;
#pragma unroll
                for (int k = 0; k < CM; ++k)
                    if (k < C) o[k] = q[k];
            }
            if (out_packed) {
                // index_points returns a contiguous tensor: contiguous-layout ssq
                float *o = out_packed + ((int64_t)b * S + i) * cp;
#pragma unroll
                for (int k = 0; k < CM; ++k)
                    if (k < C) o[k] = q[k];
                o[C] = contig_sum<CM>(sq, C);
                for (int k = C + 1; k < cp; ++k) o[k] = 0.f;
            }
        }
    }
}

// ------------------------------------------------------------------------- pack kernel
template <int CM>
__global__ __launch_bounds__(256) void pack_points_kernel(const float *__restrict__ pts, int64_t B,
                                                          int N, int C, int64_t sb, int64_t sn,
                                                          int64_t sc, int kind,
                                                          float *__restrict__ packed, int cp) {
    const int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (e >= B * N) return;
    const int64_t b = e / N;
    const int n = (int)(e - b * N);
    const float *q = pts + b * sb + (int64_t)n * sn;
    float a[CM], sq[CM];
#pragma unroll
    for (int k = 0; k < CM; ++k) {
        a[k] = (k < C) ? q[(int64_t)k * sc] : 0.f;
        sq[k] = __fmul_rn(a[k], a[k]);
    }
    float *o = packed + e * cp;
#pragma unroll
    for (int k = 0; k < CM; ++k)
        if (k < C) o[k] = a[k];
    o[C] = layout_sum<CM>(sq, C, point_rule(kind, n, N));
    for (int k = C + 1; k < cp; ++k) o[k] = 0.f;
}

}  // namespace pn2

using namespace pn2;

extern "C" int64_t pn2_packed_stride(int64_t C) { return ((C + 1 + 3) / 4) * 4; }

template <int NT, int PPT, int CM, bool FIXED>
static int launch_fps(const float *pts, int64_t B, int64_t N, int64_t C, int64_t sb, int64_t sn,
                      int64_t sc, const int64_t *start, int64_t S, int64_t *out_idx,
                      float *out_pts, float *out_packed, float *pts_packed, hipStream_t st) {
    const int kind = layout_kind(sn, sc);
    hipLaunchKernelGGL((fps_kernel<NT, PPT, CM, FIXED>), dim3((unsigned)B), dim3(NT), 0, st, pts,
                       (int)N, (int)C, sb, sn, sc, kind, start, (int)S, out_idx, out_pts,
                       out_packed, pts_packed, (int)pn2_packed_stride(C));
    PN2_LAUNCH_CHECK("fps_kernel");
    return PN2_OK;
}

// Block shape per cloud size: one wave (no barrier at all) for small clouds, a few waves for
// mid-size ones, 1024 lanes for large ones.  CAP bounds the register-resident cloud size.
template <int CM, bool FIXED, int CAP>
static int dispatch_fps(const float *pts, int64_t B, int64_t N, int64_t C, int64_t sb, int64_t sn,
                        int64_t sc, const int64_t *start, int64_t S, int64_t *out_idx,
                        float *out_pts, float *out_packed, float *pts_packed, hipStream_t st) {
#define A pts, B, N, C, sb, sn, sc, start, S, out_idx, out_pts, out_packed, pts_packed, st
    if (N <= 256) return launch_fps<64, 4, CM, FIXED>(A);
    if (N <= 512) return launch_fps<64, 8, CM, FIXED>(A);
    if (N <= 1024) return launch_fps<256, 4, CM, FIXED>(A);
    if (N <= 2048) return launch_fps<256, 8, CM, FIXED>(A);
    if (N <= 4096) return launch_fps<1024, 4, CM, FIXED>(A);
    if constexpr (CAP >= 8192)
        if (N <= 8192) return launch_fps<1024, 8, CM, FIXED>(A);
    if constexpr (CAP >= 16384)
        if (N <= 16384) return launch_fps<1024, 16, CM, FIXED>(A);
#undef A
    return set_error(PN2_EUNSUPPORTED, "pn2_fps_f32: N=%lld exceeds the register-resident cap %d for C=%lld",
                     (long long)N, CAP, (long long)C);
}

extern "C" int pn2_fps_f32(const float *pts, int64_t B, int64_t N, int64_t C, int64_t sb,
                           int64_t sn, int64_t sc, const int64_t *start, int64_t S,
                           int64_t *out_idx, float *out_pts, float *out_packed, float *pts_packed,
                           void *stream) {
    PN2_REQUIRE(pts && start && out_idx, "pn2_fps_f32: null pointer");
    PN2_REQUIRE(B >= 0 && N >= 1 && C >= 1 && S >= 1, "pn2_fps_f32: bad shape B=%lld N=%lld C=%lld S=%lld",
                (long long)B, (long long)N, (long long)C, (long long)S);
    PN2_REQUIRE(S <= kFpsMaxS, "pn2_fps_f32: S=%lld exceeds %d", (long long)S, kFpsMaxS);
    if (B == 0) return PN2_OK;
    hipStream_t st = as_stream(stream);
#define A pts, B, N, C, sb, sn, sc, start, S, out_idx, out_pts, out_packed, pts_packed, st
    if (C == 3) return dispatch_fps<3, true, 16384>(A);
    if (C == 10) return dispatch_fps<10, true, 8192>(A);
    if (C <= kMaxC) return dispatch_fps<kMaxC, false, 4096>(A);
#undef A
    return set_error(PN2_EUNSUPPORTED, "pn2_fps_f32: unsupported C=%lld (max %d)", (long long)C,
                     kMaxC);
}

extern "C" int pn2_pack_points_f32(const float *pts, int64_t B, int64_t N, int64_t C, int64_t sb,
                                   int64_t sn, int64_t sc, float *packed, void *stream) {
    PN2_REQUIRE(pts && packed, "pn2_pack_points_f32: null pointer");
    PN2_REQUIRE(B >= 0 && N >= 1 && C >= 1 && C <= kMaxC, "pn2_pack_points_f32: bad shape");
    if (B == 0) return PN2_OK;
    const int kind = layout_kind(sn, sc);
    const int64_t tot = B * N;
    const dim3 grid((unsigned)((tot + 255) / 256));
    const int cp = (int)pn2_packed_stride(C);
    if (C == 3)
        hipLaunchKernelGGL(pack_points_kernel<3>, grid, dim3(256), 0, as_stream(stream), pts, B,
                           (int)N, 3, sb, sn, sc, kind, packed, cp);
    else
        hipLaunchKernelGGL(pack_points_kernel<kMaxC>, grid, dim3(256), 0, as_stream(stream), pts,
                           B, (int)N, (int)C, sb, sn, sc, kind, packed, cp);
    PN2_LAUNCH_CHECK("pack_points_kernel");
    return PN2_OK;
}
