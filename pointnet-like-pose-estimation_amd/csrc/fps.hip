// fps.hip -- farthest point sampling for gfx950.
//
// Replaces farthest_point_sample (/root/reference/model/pointnet2_utils.py:47-68) and the
// index_points(points, fps_idx) that follows it (pointnet2_utils.py:106, 201).
//
// One workgroup per cloud.  Lane t of the block owns the CONTIGUOUS points t*PPT .. t*PPT+PPT-1
// and keeps them in registers for the whole run, together with their running min-distance (the
// uint bits of a non-negative float, so compares/maxima are integer ops).  Because ownership is
// contiguous and in lane/wave order, "the first index among the maxima" (torch.max's tie rule)
// is simply the first lane -- then the first wave -- that holds the maximum: one DPP max per
// level plus a ballot, no second (index) reduction.  One iteration:
//   branchless distance of every owned point to the centroid in the reference's exact float32
//   order (differences, exact squares, layout-dependent channel sum, no FMA contraction) ->
//   strict-< min update -> per-lane max -> wave max by DPP + ballot/ctz for the owner lane -> the
//   owner's first point at the max by one ballot per point (wave-uniform index, SALU scan) and its
//   coordinates by one indexed register move each -> [NW > 1] the owner writes {max, index,
//   coordinates} to its wave's LDS slot (double-buffered by iteration parity), ONE barrier,
//   every wave reads all NW
//   slots (one lane each), DPP max over a 16-lane row + ballot picks the winning wave and
//   v_readlane broadcasts its index/coordinates.  No second barrier, no global memory in the loop.
// The sampled indices are kept in LDS and written, with the gathered centroids and the packed
// (coords, ssq) records the ball query reads, after the serial loop.
#include "fps_body.h"

#include <stdlib.h>

#include <algorithm>

namespace pn2 {

template <int NT, int PPT, int CM, bool FIXED, bool LDSC, int CR = CM>
__global__ __launch_bounds__(NT) void fps_kernel(const FpsArgs F) {
    extern __shared__ __attribute__((aligned(16))) float fsm[];
    fps_block<NT, PPT, CM, FIXED, LDSC, CR>(F, (int)blockIdx.x, fsm);
}

// ------------------------------------------------------------------------- streamed FPS
// Any N and S: nothing of the cloud is register-resident.  Each iteration every thread walks
// the points n = tid, tid + NT, ... (coalesced reads of the input for either layout), computes
// the distance in the reference's order, updates the running minimum -- held in LDS when the
// cloud's N words fit (DL), else in the caller's workspace (one word per point) -- and keeps
// the 64-bit key (distance bits : ~index), whose maximum is torch.max's first index among the
// maxima.  Wave max by shuffles, one LDS slot per wave (double-buffered by parity), ONE
// barrier, every thread reduces the NW slots.  The centroid's coordinates are re-read from
// the input (one broadcast load).  Indices go straight to out_idx; the output pass reads them
// back with sc1 loads (stores of other waves of this workgroup).
// Point dimensions past the register-resident kMaxC (16 < C <= kMaxCWide) always take this
// kernel, with 256 threads: a point's channels, squares and the centroid are register arrays
// of kMaxCWide entries (predicated on C), too many for 1024-thread workgroups.
constexpr int kFpsStreamT = 1024;
template <int CM>
constexpr int fps_stream_threads() { return CM > kMaxC ? 256 : kFpsStreamT; }

__device__ __forceinline__ unsigned long long wave_max_u64(unsigned long long v) {
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) {
        const unsigned long long w = __shfl_xor(v, o);
        v = w > v ? w : v;
    }
    return v;
}

template <int CM, bool FIXED, bool DL>
__global__ __launch_bounds__(fps_stream_threads<CM>()) void fps_stream_kernel(
    const float *__restrict__ pts, int N, int Crt, int64_t sb, int64_t sn, int64_t sc, int kind,
    const FpsStart start, int S, int64_t *__restrict__ out_idx, float *__restrict__ out_pts,
    float *__restrict__ out_packed, float *__restrict__ pts_packed, int cp, unsigned *__restrict__ dist_ws) {
    constexpr int NT = fps_stream_threads<CM>(), NW = NT / 64;
    __builtin_amdgcn_s_setprio(PN2_FPS_PRIO);
    const int C = FIXED ? CM : Crt;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int b = blockIdx.x;
    const float *P = pts + (int64_t)b * sb;
    extern __shared__ __attribute__((aligned(16))) unsigned long long ssm[];
    unsigned long long *slots = ssm;                               // [2][NW]
    unsigned *dist = DL ? reinterpret_cast<unsigned *>(ssm + 2 * NW)  // [N]
                        : dist_ws + (int64_t)b * N;
    auto point = [&](int64_t n, float (&q)[CM]) {
#pragma unroll
        for (int k = 0; k < CM; ++k) q[k] = (k < C) ? P[n * sn + (int64_t)k * sc] : 0.f;
    };
    for (int n = tid; n < N; n += NT) {
        dist[n] = __float_as_uint(1e10f);
        if (pts_packed) {
            float q[CM], sq[CM];
            point(n, q);
#pragma unroll
            for (int k = 0; k < CM; ++k) sq[k] = __fmul_rn(q[k], q[k]);
            float *dst = pts_packed + ((int64_t)b * N + n) * cp;
#pragma unroll
            for (int k = 0; k < CM; ++k)
                if (k < C) dst[k] = q[k];
            dst[C] = layout_sum<CM>(sq, C, point_rule(kind, n, N));
            for (int k = C + 1; k < cp; ++k) dst[k] = 0.f;
        }
    }
    int far = fps_start(start, b);
    float c[CM];
    point(far, c);
    __syncthreads();
    int64_t *oi = out_idx + (int64_t)b * S;
    for (int i = 0;; ++i) {
        if (tid == 0) oi[i] = far;
        if (i == S - 1) break;
        unsigned long long best = 0ull;
        for (int n = tid; n < N; n += NT) {
            float q[CM], sq[CM];
            point(n, q);
#pragma unroll
            for (int k = 0; k < CM; ++k) {
                const float d = q[k] - c[k];
                sq[k] = __fmul_rn(d, d);
            }
            float dd;
            if constexpr (FIXED && CM == 3) dd = seq_sum<CM>(sq, C);  // every rule agrees for C=3
            else dd = layout_sum<CM>(sq, C, point_rule(kind, n, N));
            const unsigned v = min(dist[n], __float_as_uint(dd));  // strict '<' update
            dist[n] = v;
            const unsigned long long key = ((unsigned long long)v << 32) | (0xFFFFFFFFu - (unsigned)n);
            best = key > best ? key : best;
        }
        best = wave_max_u64(best);
        const int par = i & 1;
        if (lane == 0) slots[par * NW + wave] = best;
        __syncthreads();  // the other parity's slots were last read before this barrier
        unsigned long long g = slots[par * NW];
#pragma unroll
        for (int w = 1; w < NW; ++w) {
            const unsigned long long v = slots[par * NW + w];
            g = v > g ? v : g;
        }
        far = (int)(0xFFFFFFFFu - (unsigned)g);
        point(far, c);
    }
    __syncthreads();
    for (int i = tid; i < S; i += NT) {
        const int64_t n = __hip_atomic_load(oi + i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (out_pts || out_packed) {
            float q[CM], sq[CM];
            point(n, q);
#pragma unroll
            for (int k = 0; k < CM; ++k) sq[k] = __fmul_rn(q[k], q[k]);
            if (out_pts) {
                float *o = out_pts + ((int64_t)b * S + i) * C;
#pragma unroll
                for (int k = 0; k < CM; ++k)
                    if (k < C) o[k] = q[k];
            }
            if (out_packed) {
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

// the FpsArgs of a launch (or side job) over points pts[b*sb + n*sn + c*sc]
FpsArgs pn2::fps_args(const float *pts, int64_t N, int64_t C, int64_t sb, int64_t sn, int64_t sc,
                 const FpsStart &start, int64_t S, int64_t *out_idx, float *out_pts, float *out_packed,
                 float *pts_packed) {
    FpsArgs F;
    F.pts = pts;
    F.N = (int)N;
    F.C = (int)C;
    F.sb = sb;
    F.sn = sn;
    F.sc = sc;
    F.kind = layout_kind(sn, sc);
    F.S = (int)S;
    F.out_idx = out_idx;
    F.out_pts = out_pts;
    F.out_packed = out_packed;
    F.pts_packed = pts_packed;
    F.cp = (int)pn2_packed_stride(C);
    F.prio = tuning().fps_prio ? 1 : 0;
    F.start = start;
    return F;
}

template <int NT, int PPT, int CM, bool FIXED, int CR = CM>
static int launch_fps(const float *pts, int64_t B, int64_t N, int64_t C, int64_t sb, int64_t sn,
                      int64_t sc, const FpsStart &start, int64_t S, int64_t *out_idx,
                      float *out_pts, float *out_packed, float *pts_packed, hipStream_t st) {
    const FpsArgs F = fps_args(pts, N, C, sb, sn, sc, start, S, out_idx, out_pts, out_packed, pts_packed);
    const size_t head = fps_block_lds(NT, CM, true, 0, S);
    const size_t cloud = fps_block_lds(NT, CM, true, N, S) - head;
    const bool ldsc = CR == CM && cloud <= (size_t)kFpsLdsCloud && head + cloud <= (size_t)160 * 1024;
    const size_t lds = fps_block_lds(NT, CM, ldsc, N, S);
    if constexpr (CR != CM) {
        hipLaunchKernelGGL((fps_kernel<NT, PPT, CM, FIXED, false, CR>), dim3((unsigned)B), dim3(NT), lds, st, F);
    } else if (ldsc) {
        static const hipError_t attr = hipFuncSetAttribute(
            reinterpret_cast<const void *>(&fps_kernel<NT, PPT, CM, FIXED, true>),
            hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
        (void)attr;
        hipLaunchKernelGGL((fps_kernel<NT, PPT, CM, FIXED, true>), dim3((unsigned)B), dim3(NT), lds, st, F);
    } else {
        hipLaunchKernelGGL((fps_kernel<NT, PPT, CM, FIXED, false>), dim3((unsigned)B), dim3(NT), lds, st, F);
    }
    PN2_LAUNCH_CHECK("fps_kernel");
    return PN2_OK;
}

// Block shape per cloud size.  Tuning fps_threads / fps_ppt force one of the compiled shapes
// (tuning experiments only).
template <int CM, bool FIXED, int CAP>
static int dispatch_fps(const float *pts, int64_t B, int64_t N, int64_t C, int64_t sb, int64_t sn,
                        int64_t sc, const FpsStart &start, int64_t S, int64_t *out_idx,
                        float *out_pts, float *out_packed, float *pts_packed, hipStream_t st) {
#define A pts, B, N, C, sb, sn, sc, start, S, out_idx, out_pts, out_packed, pts_packed, st
    const int64_t fnt = tuning().fps_threads, fppt = tuning().fps_ppt;
#define PN2_FPS_TRY(nt, ppt) \
    if (fnt == nt && fppt == ppt && N <= (int64_t)nt * ppt) return launch_fps<nt, ppt, CM, FIXED>(A);
    PN2_FPS_TRY(64, 8) PN2_FPS_TRY(64, 16) PN2_FPS_TRY(128, 4) PN2_FPS_TRY(128, 8) PN2_FPS_TRY(256, 2)
    PN2_FPS_TRY(256, 4) PN2_FPS_TRY(512, 2) PN2_FPS_TRY(1024, 1) PN2_FPS_TRY(512, 4) PN2_FPS_TRY(1024, 2)
    if constexpr (CM == 3) {
        PN2_FPS_TRY(512, 16) PN2_FPS_TRY(512, 32) PN2_FPS_TRY(256, 32) PN2_FPS_TRY(1024, 8)
    }
#undef PN2_FPS_TRY
    if (N <= 256) return launch_fps<64, 4, CM, FIXED>(A);
    // measured on MI355X (tools/bench_fps.py): two points per lane and 4-16 waves win until
    // the per-wave register set grows; past 2048 points the block is capped at 1024 threads.
    // Up to 1024 points (tuning fps_mid): alone on the chip 8 waves of 2 points are fastest
    // (r04, interleaved x3: SSG sa1 154 vs 178 us at 256 x 4, sa2 43.0 vs 49.4; the eager
    // forward +6.5 %); in the pipelines, beside the chains on the same SIMDs, 4 waves of 4
    // points read ~2 % better (K = 100, tools/gpu_r04ab.sh), so pn2/pipeline.py selects that
    // for its geometry
    if (N <= 1024) {
        if (tuning().fps_mid == 256) return launch_fps<256, 4, CM, FIXED>(A);
        return launch_fps<512, 2, CM, FIXED>(A);
    }
    if (N <= 2048) return launch_fps<1024, 2, CM, FIXED>(A);
    if (N <= 4096) return launch_fps<1024, 4, CM, FIXED>(A);
    if constexpr (CAP >= 8192)
        if (N <= 8192) return launch_fps<1024, 8, CM, FIXED>(A);
    if constexpr (CAP >= 16384)
        if (N <= 16384) return launch_fps<1024, 16, CM, FIXED>(A);
    // past the register-resident caps: xyz in registers, the other channels re-read from the
    // input each iteration when they are not constant (the pose heads' one-hot clouds -- e.g.
    // the 10000-point camera scans -- never read them)
    if constexpr (CM > 3)
        if (N <= 16384) return launch_fps<1024, 16, CM, FIXED, 3>(A);
#undef A
    return set_error(PN2_EUNSUPPORTED, "pn2_fps_f32: N=%lld: no register-resident shape", (long long)N);
}

// the register-resident kernels' limits (dispatch_fps); past them the streamed kernel
static bool fps_resident(int64_t N, int64_t S) { return N <= 16384 && S <= kFpsMaxS; }
static size_t fps_stream_lds(int64_t N, int nt = kFpsStreamT) { return (size_t)2 * (nt / 64) * 8 + (size_t)N * 4; }
static bool fps_stream_dl(int64_t N, int nt = kFpsStreamT) { return fps_stream_lds(N, nt) <= (size_t)160 * 1024; }

template <int CM, bool FIXED>
static int launch_fps_stream(const float *pts, int64_t B, int64_t N, int64_t C, int64_t sb, int64_t sn,
                             int64_t sc, const FpsStart &start, int64_t S, int64_t *out_idx, float *out_pts,
                             float *out_packed, float *pts_packed, unsigned *ws, hipStream_t st) {
    const int kind = layout_kind(sn, sc);
    const int cp = (int)pn2_packed_stride(C);
    constexpr int NT = fps_stream_threads<CM>();
    if (fps_stream_dl(N, NT)) {
        static const hipError_t attr = hipFuncSetAttribute(
            reinterpret_cast<const void *>(&fps_stream_kernel<CM, FIXED, true>),
            hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
        PN2_REQUIRE(attr == hipSuccess, "pn2_fps_f32: LDS attribute: %s", hipGetErrorString(attr));
        hipLaunchKernelGGL((fps_stream_kernel<CM, FIXED, true>), dim3((unsigned)B), dim3(NT),
                           fps_stream_lds(N, NT), st, pts, (int)N, (int)C, sb, sn, sc, kind, start, (int)S, out_idx,
                           out_pts, out_packed, pts_packed, cp, nullptr);
    } else {
        hipLaunchKernelGGL((fps_stream_kernel<CM, FIXED, false>), dim3((unsigned)B), dim3(NT),
                           fps_stream_lds(0, NT), st, pts, (int)N, (int)C, sb, sn, sc, kind, start, (int)S, out_idx,
                           out_pts, out_packed, pts_packed, cp, ws);
    }
    PN2_LAUNCH_CHECK("fps_stream_kernel");
    return PN2_OK;
}

extern "C" int64_t pn2_fps_workspace_bytes(int64_t B, int64_t N, int64_t C, int64_t S) {
    if (B < 0 || N < 1 || C < 1 || S < 1) return -1;
    if (C > kMaxC) return fps_stream_dl(N, fps_stream_threads<kMaxCWide>()) ? 0 : B * N * 4;
    return (fps_resident(N, S) || fps_stream_dl(N)) ? 0 : B * N * 4;
}

static int fps_check(const float *pts, const int64_t *start, int64_t *out_idx, int64_t B, int64_t N,
                     int64_t C, int64_t S, void *workspace, int64_t workspace_bytes) {
    PN2_REQUIRE(pts && start && out_idx, "pn2_fps_f32: null pointer");
    PN2_REQUIRE(B >= 0 && N >= 1 && C >= 1 && S >= 1 && N < INT32_MAX && S < INT32_MAX,
                "pn2_fps_f32: bad shape B=%lld N=%lld C=%lld S=%lld", (long long)B, (long long)N, (long long)C,
                (long long)S);
    if (C > kMaxCWide)
        return set_error(PN2_EUNSUPPORTED, "pn2_fps_f32: unsupported C=%lld (max %d)", (long long)C, kMaxCWide);
    const int64_t need = pn2_fps_workspace_bytes(B, N, C, S);
    PN2_REQUIRE(workspace_bytes >= need && (need == 0 || workspace),
                "pn2_fps_f32: N=%lld needs pn2_fps_workspace_bytes = %lld bytes of workspace", (long long)N,
                (long long)need);
    return PN2_OK;
}

static int fps_run(const float *pts, int64_t B, int64_t N, int64_t C, int64_t sb, int64_t sn, int64_t sc,
                   const FpsStart &start, int64_t S, int64_t *out_idx, float *out_pts, float *out_packed,
                   float *pts_packed, void *workspace, hipStream_t st) {
#define A pts, B, N, C, sb, sn, sc, start, S, out_idx, out_pts, out_packed, pts_packed
    if (C > kMaxC) return launch_fps_stream<kMaxCWide, false>(A, static_cast<unsigned *>(workspace), st);
    if (!fps_resident(N, S)) {
        unsigned *ws = static_cast<unsigned *>(workspace);
        if (C == 3) return launch_fps_stream<3, true>(A, ws, st);
        if (C == 10) return launch_fps_stream<10, true>(A, ws, st);
        return launch_fps_stream<kMaxC, false>(A, ws, st);
    }
    if (C == 3) return dispatch_fps<3, true, 16384>(A, st);
    if (C == 10) return dispatch_fps<10, true, 8192>(A, st);
    return dispatch_fps<kMaxC, false, 4096>(A, st);
#undef A
}

extern "C" int pn2_fps_ws_f32(const float *pts, int64_t B, int64_t N, int64_t C, int64_t sb, int64_t sn,
                              int64_t sc, const int64_t *start, int64_t S, int64_t *out_idx, float *out_pts,
                              float *out_packed, float *pts_packed, void *workspace, int64_t workspace_bytes,
                              void *stream) {
    const int rc = fps_check(pts, start, out_idx, B, N, C, S, workspace, workspace_bytes);
    if (rc != PN2_OK || B == 0) return rc;
    FpsStart fs;
    fs.dev = start;
    return fps_run(pts, B, N, C, sb, sn, sc, fs, S, out_idx, out_pts, out_packed, pts_packed, workspace,
                   as_stream(stream));
}

// start in host memory, read during the call (the caller may reuse it on return): carried in
// the kernel arguments, kFpsArgStarts clouds per launch (a launch of that many clouds already
// covers the chip's 256 CUs, so the split costs no concurrency)
extern "C" int pn2_fps_host_ws_f32(const float *pts, int64_t B, int64_t N, int64_t C, int64_t sb, int64_t sn,
                                   int64_t sc, const int64_t *start_host, int64_t S, int64_t *out_idx,
                                   float *out_pts, float *out_packed, float *pts_packed, void *workspace,
                                   int64_t workspace_bytes, void *stream) {
    int rc = fps_check(pts, start_host, out_idx, B, N, C, S, workspace, workspace_bytes);
    if (rc != PN2_OK || B == 0) return rc;
    for (int64_t b = 0; b < B; ++b)
        PN2_REQUIRE(start_host[b] >= 0 && start_host[b] < N, "pn2_fps_f32: start[%lld] = %lld outside [0, %lld)",
                    (long long)b, (long long)start_host[b], (long long)N);
    const int cp = (int)pn2_packed_stride(C);
    hipStream_t st = as_stream(stream);
    FpsStart fs;
    fs.dev = nullptr;
    for (int64_t b0 = 0; b0 < B; b0 += kFpsArgStarts) {
        const int64_t nb = std::min<int64_t>(kFpsArgStarts, B - b0);
        for (int64_t j = 0; j < nb; ++j) fs.v[j] = (int)start_host[b0 + j];
        rc = fps_run(pts + b0 * sb, nb, N, C, sb, sn, sc, fs, S, out_idx + b0 * S, out_pts ? out_pts + b0 * S * C : nullptr,
                     out_packed ? out_packed + b0 * S * cp : nullptr, pts_packed ? pts_packed + b0 * N * cp : nullptr,
                     workspace ? static_cast<unsigned *>(workspace) + b0 * N : nullptr, st);
        if (rc != PN2_OK) return rc;
    }
    return PN2_OK;
}

extern "C" int pn2_fps_f32(const float *pts, int64_t B, int64_t N, int64_t C, int64_t sb,
                           int64_t sn, int64_t sc, const int64_t *start, int64_t S,
                           int64_t *out_idx, float *out_pts, float *out_packed, float *pts_packed,
                           void *stream) {
    return pn2_fps_ws_f32(pts, B, N, C, sb, sn, sc, start, S, out_idx, out_pts, out_packed, pts_packed, nullptr, 0,
                          stream);
}

#ifdef PN2_FPS_STAMPS
extern "C" int pn2_debug_fps_stamps(unsigned long long *out) {
    if (hipDeviceSynchronize() != hipSuccess) return -1;
    return hipMemcpyFromSymbol(out, HIP_SYMBOL(g_fps_stamps), sizeof(g_fps_stamps)) == hipSuccess ? 0 : -1;
}
#endif

// ------------------------------------------------------------------------- FPS side jobs
bool &pn2::fps_side_taken() {
    static thread_local bool taken = false;
    return taken;
}

int pn2::fps_side_check(const pn2_fps_side &f) {
    PN2_REQUIRE(f.start_host, "pn2_fps_side: null start_host");
    const int rc = fps_check(f.pts, f.start_host, f.out_idx, f.B, f.N, f.C, f.S, nullptr, 0);
    if (rc != PN2_OK) return rc;
    for (int64_t b = 0; b < f.B; ++b)
        PN2_REQUIRE(f.start_host[b] >= 0 && f.start_host[b] < f.N,
                    "pn2_fps_side: start[%lld] = %lld outside [0, %lld)", (long long)b,
                    (long long)f.start_host[b], (long long)f.N);
    return PN2_OK;
}

int pn2::fps_side_launch(const pn2_fps_side &f, hipStream_t st) {
    return pn2_fps_host_ws_f32(f.pts, f.B, f.N, f.C, f.sb, f.sn, f.sc, f.start_host, f.S, f.out_idx, f.out_pts,
                               f.out_packed, f.pts_packed, nullptr, 0, st);
}

// The side job as workgroups of a chain launch (sa_chain_kernel<., ., 1, ., .>: fps_block<256, 2,
// C, true, true>, one workgroup per cloud): false when its shape does not fit that instance or
// its LDS exceeds the chain's
bool pn2::fps_side_block_args(const pn2_fps_side &f, size_t lds_avail, FpsArgs &F) {
    if (f.B < 1 || f.B > kFpsArgStarts || f.N > 512 || f.S > kFpsMaxS || (f.C != 3 && f.C != 10)) return false;
    if (fps_block_lds(256, (int)f.C, true, f.N, f.S) > lds_avail) return false;
    FpsStart fs;
    fs.dev = nullptr;
    for (int64_t b = 0; b < f.B; ++b) fs.v[b] = (int)f.start_host[b];
    F = fps_args(f.pts, f.N, f.C, f.sb, f.sn, f.sc, fs, f.S, f.out_idx, f.out_pts, f.out_packed, f.pts_packed);
    return true;
}

extern "C" int pn2_pack_points_f32(const float *pts, int64_t B, int64_t N, int64_t C, int64_t sb,
                                   int64_t sn, int64_t sc, float *packed, void *stream) {
    PN2_REQUIRE(pts && packed, "pn2_pack_points_f32: null pointer");
    PN2_REQUIRE(B >= 0 && N >= 1 && C >= 1, "pn2_pack_points_f32: bad shape");
    if (C > kMaxCWide)
        return set_error(PN2_EUNSUPPORTED, "pn2_pack_points_f32: unsupported C=%lld (max %d)", (long long)C, kMaxCWide);
    if (B == 0) return PN2_OK;
    const int kind = layout_kind(sn, sc);
    const int64_t tot = B * N;
    const dim3 grid((unsigned)((tot + 255) / 256));
    const int cp = (int)pn2_packed_stride(C);
    if (C == 3)
        hipLaunchKernelGGL(pack_points_kernel<3>, grid, dim3(256), 0, as_stream(stream), pts, B,
                           (int)N, 3, sb, sn, sc, kind, packed, cp);
    else if (C <= kMaxC)
        hipLaunchKernelGGL(pack_points_kernel<kMaxC>, grid, dim3(256), 0, as_stream(stream), pts,
                           B, (int)N, (int)C, sb, sn, sc, kind, packed, cp);
    else
        hipLaunchKernelGGL(pack_points_kernel<kMaxCWide>, grid, dim3(256), 0, as_stream(stream), pts,
                           B, (int)N, (int)C, sb, sn, sc, kind, packed, cp);
    PN2_LAUNCH_CHECK("pack_points_kernel");
    return PN2_OK;
}
