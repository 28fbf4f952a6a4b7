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
#include "pn2_internal.h"

#include <stdlib.h>

#include <algorithm>

namespace pn2 {

constexpr int kFpsMaxS = 8192;

// The start indices of a launch: a device array (dev), or -- pn2_fps_host_ws_f32 -- up to
// kFpsArgStarts values carried in the kernel arguments (the reference draws them on the host,
// pointnet2_utils.py:59; as arguments they need no host->device copy, and the kernel after that
// copy no longer waits for it: ~10 us per FPS call of the eager forward)
constexpr int kFpsArgStarts = 256;
struct FpsStart {
    const int64_t *dev;
    int v[kFpsArgStarts];
};
__device__ __forceinline__ int fps_start(const FpsStart &s, int b) { return s.dev ? (int)s.dev[b] : s.v[b]; }
constexpr int kFpsLdsCloud = 128 * 1024;  // bytes of LDS a cloud copy may take

// max over the first 16 lanes (row 0), result valid in every lane of row 0
__device__ __forceinline__ unsigned row_max_u32(unsigned v) {
    v = max(v, PN2_DPP(v, 0xB1));
    v = max(v, PN2_DPP(v, 0x4E));
    v = max(v, PN2_DPP(v, 0x141));
    v = max(v, PN2_DPP(v, 0x140));
    return v;
}

// LDSC: keep a copy of the cloud in LDS (N*CM floats) so the winner's coordinates are one
// broadcast ds_read; otherwise they travel with the per-wave slots.
#ifndef PN2_FPS_PRIO
#define PN2_FPS_PRIO 3
#endif
//
// CR: channels held in registers (CR = CM normally).  Large clouds whose points do not fit the
// register file with every channel keep only xyz (CR = 3) or nothing (CR = 0) there and re-read
// the other channels of their points from the input each iteration (slow, but any N up to
// NT*PPT); a cloud whose extra channels are constant (the one-hot class) never reads them.
#ifdef PN2_FPS_WGSTAMPS
// Diagnostic builds only (tools/debug/fps_wg.py): s_memrealtime (100 MHz) at entry and exit of
// every fps_kernel workgroup, in dispatch-counter order (65536 slots, wrapping)
__device__ unsigned g_fps_wgctr;
__device__ unsigned long long g_fps_wg[65536 * 2];
extern "C" int pn2_debug_fps_wg(unsigned long long *out, unsigned *count) {
    if (hipDeviceSynchronize() != hipSuccess) return -1;
    if (hipMemcpyFromSymbol(count, HIP_SYMBOL(g_fps_wgctr), sizeof(unsigned)) != hipSuccess) return -1;
    return hipMemcpyFromSymbol(out, HIP_SYMBOL(g_fps_wg), sizeof(g_fps_wg)) == hipSuccess ? 0 : -1;
}
#endif

template <int NT, int PPT, int CM, bool FIXED, bool LDSC, int CR = CM>
__global__ __launch_bounds__(NT) void fps_kernel(const float *__restrict__ pts, int N, int Crt,
                                                 int64_t sb, int64_t sn, int64_t sc, int kind,
                                                 const FpsStart start, int S,
                                                 int64_t *__restrict__ out_idx,
                                                 float *__restrict__ out_pts,
                                                 float *__restrict__ out_packed,
                                                 float *__restrict__ pts_packed, int cp) {
    constexpr int NW = NT / 64;
    static_assert(NW <= 16, "one 16-lane row reduces the wave slots");
    // In the pipelined launch FPS shares every SIMD with the MLP kernels' waves, and its
    // dependent chain (one short VALU burst, a reduction and a barrier per iteration) is the
    // pipeline's critical path: its waves take issue priority over co-resident waves.
    __builtin_amdgcn_s_setprio(PN2_FPS_PRIO);
#ifdef PN2_FPS_WGSTAMPS
    unsigned wg_slot = 0;
    if (threadIdx.x == 0) {
        wg_slot = atomicAdd(&g_fps_wgctr, 1u) & 65535u;
        g_fps_wg[2 * wg_slot] = __builtin_amdgcn_s_memrealtime();
    }
#endif
    constexpr int SLOT = (CM + 2 + 3) & ~3;  // {max, index, coords...} padded to 16 bytes
    const int C = FIXED ? CM : Crt;
    const int tid = threadIdx.x;
    const int lane = tid & 63;
    const int wave = tid >> 6;
    const int b = blockIdx.x;
    const float *P = pts + (int64_t)b * sb;

    extern __shared__ __attribute__((aligned(16))) float fsm[];
    int *sidx = reinterpret_cast<int *>(fsm);                          // [S]
    unsigned long long *key = reinterpret_cast<unsigned long long *>(  // [3] (LDSC)
        fsm + ((S + 3) & ~3));
    float *slots = fsm + ((S + 3) & ~3) + 8;                            // [2][NW][SLOT] (!LDSC)
    constexpr int CS = CM == 3 ? 4 : CM;  // cloud row stride (16-byte rows for xyz)
    float *cloud = slots + (LDSC ? 0 : 2 * NW * SLOT);                  // [N][CS] (LDSC)

    // ---- load the owned points into registers (and emit the packed copy for the ball query).
    // Points are held in pairs (one packed v_pk_* op computes two distances).  Lanes past the
    // end own padding points: coordinates 0, distance 0 -- they never beat a real point (real
    // points precede them and ties go to the first index).
    constexpr int PH = (PPT + 1) / 2;
    static_assert(CR == CM || (CR <= 3 && !LDSC), "partial register residency: xyz or nothing");
    constexpr int CQ = CR > 0 ? CR : 1;
    // per channel, the owned points' coordinates as one register vector: pairs feed the packed
    // distance ops, and a wave-uniform index selects one element with a single indexed move
    // (s_set_gpr_idx) instead of a select chain
    typedef float VQ __attribute__((ext_vector_type(2 * PH)));
    VQ q[CQ];
    unsigned dist[PPT];
    // channel k of owned point j: registers, or the input (through `base`, which the serial
    // loop launders every iteration so the compiler cannot hoist the re-reads out of it into
    // registers the kernel does not have)
    auto coord = [&](const float *base, int j, int k) -> float {
        if (k < CR) return q[k < CQ ? k : 0][j];
        const int n = tid * PPT + j;
        return (j < PPT && n < N && k < C) ? base[(int64_t)n * sn + (int64_t)k * sc] : 0.f;
    };
    // the packed copy first, point n on thread n % NT: each store instruction writes one
    // contiguous run of records (a 16-byte record per lane for xyz), where the owned-points
    // order below would scatter 4-byte stores 16*PPT bytes apart over a line per lane -- partial
    // lines the L2 writes back, and re-reads, several times over.  The register loads after it
    // hit the lines this pass brought into the L2.
    if (pts_packed) {
        for (int n = tid; n < N; n += NT) {
            float pj[CM], sq[CM];
#pragma unroll
            for (int k = 0; k < CM; ++k) {
                pj[k] = k < C ? P[(int64_t)n * sn + (int64_t)k * sc] : 0.f;
                sq[k] = __fmul_rn(pj[k], pj[k]);
            }
            const float s = layout_sum<CM>(sq, C, point_rule(kind, n, N));
            float *dst = pts_packed + ((int64_t)b * N + n) * cp;
            if (CM == 3 && cp == 4) {
                *reinterpret_cast<float4 *>(dst) = make_float4(pj[0], pj[1], pj[2], s);
            } else {
#pragma unroll
                for (int k = 0; k < CM; ++k)
                    if (k < C) dst[k] = pj[k];
                dst[C] = s;
                for (int k = C + 1; k < cp; ++k) dst[k] = 0.f;
            }
        }
    }
    int rule[PH];  // a pair shares its rule: the strided tail starts at an even index
#pragma unroll
    for (int j = 0; j < 2 * PH; ++j) {
        const int n = tid * PPT + j;
        const bool valid = j < PPT && n < N;
        float pj[CM];
#pragma unroll
        for (int k = 0; k < CM; ++k) {
            pj[k] = (valid && k < C) ? P[(int64_t)n * sn + (int64_t)k * sc] : 0.f;
            if (k < CR) q[k < CQ ? k : 0][j] = pj[k];
        }
        if (j < PPT) dist[j] = valid ? __float_as_uint(1e10f) : 0u;
        if ((j & 1) == 0) rule[j >> 1] = point_rule(kind, n, N);
        if (LDSC && valid) {
#pragma unroll
            for (int k = 0; k < CS; ++k) cloud[n * CS + k] = k < CM ? pj[k] : 0.f;
        }
    }
    if (LDSC && tid < 3) key[tid] = 0ull;

    // ---- channels past xyz that are constant over the cloud (the pose heads' one-hot class:
    // one label per cloud) contribute (v - v)^2 = +0 to every distance, and adding +0 leaves
    // each of the reference's channel-sum orders equal to ((dx^2 + dy^2) + dz^2) -- so such a
    // cloud runs the 3-channel loop, bit-identically.  Non-finite constants keep the full
    // loop (inf - inf is NaN).
    bool cst = true;
    if constexpr (FIXED && CM > 3) {
#pragma unroll
        for (int k = 3; k < CM; ++k) {
            const float v0 = P[(int64_t)k * sc];
            cst = cst && __builtin_isfinite(v0);
#pragma unroll
            for (int j = 0; j < 2 * PH; ++j)
                if (j < PPT && tid * PPT + j < N) cst = cst && (coord(P, j, k) == v0);
        }
    }
    // block AND through a spare LDS word behind the key words (no static LDS: the cloud copy
    // may use the whole 160 KB dynamically)
    bool xyz_only = false;
    if constexpr (FIXED && CM > 3) {
        int *flag = reinterpret_cast<int *>(fsm + ((S + 3) & ~3) + 6);
        if (tid == 0) *flag = 1;
        __syncthreads();
        if (!cst) *flag = 0;  // every writer stores 0: a benign race
        __syncthreads();
        xyz_only = *flag != 0;
    }

    // ---- serial loop
    int far = fps_start(start, b);
    float c[CM];
#pragma unroll
    for (int k = 0; k < CM; ++k) c[k] = (k < C) ? P[(int64_t)far * sn + (int64_t)k * sc] : 0.f;
    __syncthreads();

    for (int i = 0;; ++i) {
        if (tid == 0) sidx[i] = far;
        if (i == S - 1) break;
        const float *Pl = P;
        if constexpr (CR < CM) asm volatile("" : "+s"(Pl));

        // distances (two points per packed op) and the running min -- branchless
#pragma unroll
        for (int h = 0; h < PH; ++h) {
            pn2_f2 dd;
            if (xyz_only) {
                pn2_f2 s3[3];
#pragma unroll
                for (int k = 0; k < 3; ++k) {
                    const pn2_f2 qk = k < CR ? pn2_f2{q[k < CQ ? k : 0][2 * h], q[k < CQ ? k : 0][2 * h + 1]}
                                             : pn2_f2{coord(Pl, 2 * h, k), coord(Pl, 2 * h + 1, k)};
                    const pn2_f2 d = qk - c[k];
                    s3[k] = d * d;
                }
                dd = (s3[0] + s3[1]) + s3[2];
            } else {
                pn2_f2 sq[CM];
#pragma unroll
                for (int k = 0; k < CM; ++k) {
                    const pn2_f2 qk = k < CR ? pn2_f2{q[k < CQ ? k : 0][2 * h], q[k < CQ ? k : 0][2 * h + 1]}
                                             : pn2_f2{coord(Pl, 2 * h, k), coord(Pl, 2 * h + 1, k)};
                    const pn2_f2 d = qk - c[k];
                    sq[k] = d * d;
                }
                if constexpr (FIXED && CM == 3) dd = seq_sum<CM>(sq, C);  // every rule agrees for C=3
                else dd = layout_sum<CM>(sq, C, rule[h]);
            }
            // strict '<' update == min on the (non-negative) float bits; padding stays 0
            dist[2 * h] = min(dist[2 * h], __float_as_uint(dd.x));
            if (2 * h + 1 < PPT) dist[2 * h + 1] = min(dist[2 * h + 1], __float_as_uint(dd.y));
        }
        unsigned bv = dist[0];
#pragma unroll
        for (int j = 1; j < PPT; ++j) bv = max(bv, dist[j]);
        // wave: max value, then its first lane (contiguous ownership -> smallest index)
        const unsigned wv = wave_max_u32(bv);
        const int ol = (int)__builtin_ctzll(__ballot(bv == wv));
        // the owner lane's first point holding the max, wave-uniform: one compare per point
        // writes its lane mask straight to an SGPR pair, the scan over the owner's bit is SALU
        int bj = PPT - 1;
#pragma unroll
        for (int j = PPT - 2; j >= 0; --j)
            if ((__ballot(dist[j] == wv) >> ol) & 1ull) bj = j;
        if constexpr (LDSC) {
            if constexpr (NW == 1) {
                far = ol * PPT + bj;
            } else {
                // one 64-bit LDS max per wave: key = dist bits : ~index (max dist, then first
                // index).  key[i%3] is reset one iteration ahead; its last reader passed the
                // previous barrier.
                if (lane == ol) {
                    const unsigned idx = (unsigned)(tid * PPT + bj);
                    atomicMax(&key[i % 3], ((unsigned long long)wv << 32) | (0xFFFFFFFFu - idx));
                }
                if (tid == 64) key[(i + 1) % 3] = 0ull;
                __syncthreads();
                far = __builtin_amdgcn_readfirstlane((int)(0xFFFFFFFFu - (unsigned)key[i % 3]));
            }
#pragma unroll
            for (int k = 0; k < CM; ++k) c[k] = cloud[far * CS + k];
        } else {
            float bc[CM];
#pragma unroll
            for (int k = 0; k < CM; ++k) {
                if (k < CR) {
                    bc[k] = q[k < CQ ? k : 0][bj];  // meaningful in the owner lane
                } else if (k < 3 || !xyz_only) {  // the owner lane reads its point's other channels
                    const int n = tid * PPT + bj;
                    bc[k] = (lane == ol && n < N && k < C) ? Pl[(int64_t)n * sn + (int64_t)k * sc] : 0.f;
                } else {
                    bc[k] = 0.f;  // a constant channel: its difference is +0 whatever c[k] is
                }
            }
            if constexpr (NW == 1) {
                far = ol * PPT + bj;
#pragma unroll
                for (int k = 0; k < CM; ++k)
                    c[k] = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(bc[k]), ol));
                continue;
            }
            const int par = i & 1;
            if (lane == ol) {
                float *sl = slots + (par * NW + wave) * SLOT;
                sl[0] = __uint_as_float(wv);
                sl[1] = __int_as_float(tid * PPT + bj);
#pragma unroll
                for (int k = 0; k < CM; ++k) sl[2 + k] = bc[k];
            }
            __syncthreads();
            unsigned rv = 0u;
            int ri = 0x7FFFFFFF;
            float rc[CM];
#pragma unroll
            for (int k = 0; k < CM; ++k) rc[k] = 0.f;
            if (lane < NW) {
                const float *sl = slots + (par * NW + lane) * SLOT;
                rv = __float_as_uint(sl[0]);
                ri = __float_as_int(sl[1]);
#pragma unroll
                for (int k = 0; k < CM; ++k) rc[k] = sl[2 + k];
            }
            const unsigned gv = __builtin_amdgcn_readlane(row_max_u32(rv), 0);
            const int gw = (int)__builtin_ctzll(__ballot(lane < NW && rv == gv));
            far = __builtin_amdgcn_readlane(ri, gw);
#pragma unroll
            for (int k = 0; k < CM; ++k)
                c[k] = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(rc[k]), gw));
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
#ifdef PN2_FPS_WGSTAMPS
    if (threadIdx.x == 0) g_fps_wg[2 * wg_slot + 1] = __builtin_amdgcn_s_memrealtime();
#endif
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
constexpr int kFpsStreamT = 1024;

__device__ __forceinline__ unsigned long long wave_max_u64(unsigned long long v) {
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) {
        const unsigned long long w = __shfl_xor(v, o);
        v = w > v ? w : v;
    }
    return v;
}

template <int CM, bool FIXED, bool DL>
__global__ __launch_bounds__(kFpsStreamT) void fps_stream_kernel(
    const float *__restrict__ pts, int N, int Crt, int64_t sb, int64_t sn, int64_t sc, int kind,
    const FpsStart start, int S, int64_t *__restrict__ out_idx, float *__restrict__ out_pts,
    float *__restrict__ out_packed, float *__restrict__ pts_packed, int cp, unsigned *__restrict__ dist_ws) {
    constexpr int NT = kFpsStreamT, NW = NT / 64;
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

template <int NT, int PPT, int CM, bool FIXED, int CR = CM>
static int launch_fps(const float *pts, int64_t B, int64_t N, int64_t C, int64_t sb, int64_t sn,
                      int64_t sc, const FpsStart &start, int64_t S, int64_t *out_idx,
                      float *out_pts, float *out_packed, float *pts_packed, hipStream_t st) {
    const int kind = layout_kind(sn, sc);
    constexpr int NW = NT / 64;
    constexpr int SLOT = (CM + 2 + 3) & ~3;
    const size_t head = (size_t)((S + 3) & ~3) * 4 + 32;
    const size_t cloud = (size_t)N * (CM == 3 ? 4 : CM) * 4;
    const bool ldsc = CR == CM && cloud <= (size_t)kFpsLdsCloud && head + cloud <= (size_t)160 * 1024;
    const size_t lds = head + (ldsc ? cloud : (size_t)2 * NW * SLOT * 4);
    if constexpr (CR != CM) {
        hipLaunchKernelGGL((fps_kernel<NT, PPT, CM, FIXED, false, CR>), dim3((unsigned)B), dim3(NT), lds, st,
                           pts, (int)N, (int)C, sb, sn, sc, kind, start, (int)S, out_idx, out_pts,
                           out_packed, pts_packed, (int)pn2_packed_stride(C));
    } else if (ldsc) {
        static const hipError_t attr = hipFuncSetAttribute(
            reinterpret_cast<const void *>(&fps_kernel<NT, PPT, CM, FIXED, true>),
            hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
        (void)attr;
        hipLaunchKernelGGL((fps_kernel<NT, PPT, CM, FIXED, true>), dim3((unsigned)B), dim3(NT), lds, st, pts,
                           (int)N, (int)C, sb, sn, sc, kind, start, (int)S, out_idx, out_pts,
                           out_packed, pts_packed, (int)pn2_packed_stride(C));
    } else {
        hipLaunchKernelGGL((fps_kernel<NT, PPT, CM, FIXED, false>), dim3((unsigned)B), dim3(NT), lds, st, pts,
                           (int)N, (int)C, sb, sn, sc, kind, start, (int)S, out_idx, out_pts,
                           out_packed, pts_packed, (int)pn2_packed_stride(C));
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
static size_t fps_stream_lds(int64_t N) { return (size_t)2 * (kFpsStreamT / 64) * 8 + (size_t)N * 4; }
static bool fps_stream_dl(int64_t N) { return fps_stream_lds(N) <= (size_t)160 * 1024; }

template <int CM, bool FIXED>
static int launch_fps_stream(const float *pts, int64_t B, int64_t N, int64_t C, int64_t sb, int64_t sn,
                             int64_t sc, const FpsStart &start, int64_t S, int64_t *out_idx, float *out_pts,
                             float *out_packed, float *pts_packed, unsigned *ws, hipStream_t st) {
    const int kind = layout_kind(sn, sc);
    const int cp = (int)pn2_packed_stride(C);
    if (fps_stream_dl(N)) {
        static const hipError_t attr = hipFuncSetAttribute(
            reinterpret_cast<const void *>(&fps_stream_kernel<CM, FIXED, true>),
            hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
        PN2_REQUIRE(attr == hipSuccess, "pn2_fps_f32: LDS attribute: %s", hipGetErrorString(attr));
        hipLaunchKernelGGL((fps_stream_kernel<CM, FIXED, true>), dim3((unsigned)B), dim3(kFpsStreamT),
                           fps_stream_lds(N), st, pts, (int)N, (int)C, sb, sn, sc, kind, start, (int)S, out_idx,
                           out_pts, out_packed, pts_packed, cp, nullptr);
    } else {
        hipLaunchKernelGGL((fps_stream_kernel<CM, FIXED, false>), dim3((unsigned)B), dim3(kFpsStreamT),
                           fps_stream_lds(0), st, pts, (int)N, (int)C, sb, sn, sc, kind, start, (int)S, out_idx,
                           out_pts, out_packed, pts_packed, cp, ws);
    }
    PN2_LAUNCH_CHECK("fps_stream_kernel");
    return PN2_OK;
}

extern "C" int64_t pn2_fps_workspace_bytes(int64_t B, int64_t N, int64_t C, int64_t S) {
    if (B < 0 || N < 1 || C < 1 || S < 1) return -1;
    return (fps_resident(N, S) || fps_stream_dl(N)) ? 0 : B * N * 4;
}

static int fps_check(const float *pts, const int64_t *start, int64_t *out_idx, int64_t B, int64_t N,
                     int64_t C, int64_t S, void *workspace, int64_t workspace_bytes) {
    PN2_REQUIRE(pts && start && out_idx, "pn2_fps_f32: null pointer");
    PN2_REQUIRE(B >= 0 && N >= 1 && C >= 1 && S >= 1 && N < INT32_MAX && S < INT32_MAX,
                "pn2_fps_f32: bad shape B=%lld N=%lld C=%lld S=%lld", (long long)B, (long long)N, (long long)C,
                (long long)S);
    if (C > kMaxC) return set_error(PN2_EUNSUPPORTED, "pn2_fps_f32: unsupported C=%lld (max %d)", (long long)C, kMaxC);
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
