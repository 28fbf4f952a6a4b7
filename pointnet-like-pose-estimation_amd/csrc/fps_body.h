// fps_body.h -- the register-resident farthest point sampling of one cloud by one workgroup,
// shared by fps_kernel (csrc/fps.hip: one workgroup per cloud) and the SA chain kernel's side
// job (csrc/sa_chain.hip: the next SA layer's FPS run by extra workgroups of this layer's MLP
// launch).  Replaces farthest_point_sample (/root/reference/model/pointnet2_utils.py:47-68)
// and the index_points(points, fps_idx) after it (:106, :201); see fps.hip for the algorithm.
#pragma once
#include "pn2_internal.h"

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
// b is wave-uniform (the workgroup's cloud): the argument array is read at constant offsets and
// selected by compares -- a dynamic index into a by-value kernel argument made the compiler copy
// the whole argument block to scratch in some kernels (1.5 KB per lane)
__device__ __forceinline__ int fps_start(const FpsStart &s, int b) {
    if (s.dev) return (int)s.dev[b];
    int v = 0;
#pragma unroll
    for (int j = 0; j < kFpsArgStarts; ++j) v = j == b ? s.v[j] : v;
    return v;
}
constexpr int kFpsLdsCloud = 128 * 1024;  // bytes of LDS a cloud copy may take
// bytes of the cross-wave key words ([3] u64, triple-buffered) + the block flag, 16-aligned
constexpr int kFpsKeyRegion = (3 * 8 + 4 + 15) / 16 * 16;


// One launch's (or side job's) FPS arguments: points[b, n, c] = pts[b*sb + n*sn + c*sc]
struct FpsArgs {
    const float *pts;
    int N, C;
    int64_t sb, sn, sc;
    int kind;  // layout_kind(sn, sc)
    int S;
    int64_t *out_idx;
    float *out_pts, *out_packed, *pts_packed;
    int cp;    // pn2_packed_stride(C)
    int prio;  // raise the waves' issue priority (tuning fps_prio)
    FpsStart start;
};

FpsArgs fps_args(const float *pts, int64_t N, int64_t C, int64_t sb, int64_t sn, int64_t sc,
                 const FpsStart &start, int64_t S, int64_t *out_idx, float *out_pts, float *out_packed,
                 float *pts_packed);
bool fps_side_block_args(const pn2_fps_side &f, size_t lds_avail, FpsArgs &F);

// Per-link cycle breakdown of the serial loop (diagnostic builds only, -DPN2_FPS_STAMPS:
// tools/debug/fps_stamps.py).  Every wave of workgroups 0-3 accumulates s_memtime deltas per
// link, each stamp first waiting for its LDS operations (so a link's cost includes the latency
// of its own LDS traffic): 0 loop top, 1 distances + running min, 2 lane max + wave max, 3
// owner lane + point (ballots), 4 key atomic + reset, 5 barrier, 6 key read, 7 centroid read.
#ifdef PN2_FPS_STAMPS
static __device__ unsigned long long g_fps_stamps[4 * 16 * 8];
#define PN2_FPS_T(i)                                                 \
    do {                                                             \
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");           \
        const unsigned long long t_ = __builtin_amdgcn_s_memtime();  \
        st_acc[i] += t_ - st_last;                                   \
        st_last = t_;                                                \
    } while (0)
#else
#define PN2_FPS_T(i) do {} while (0)
#endif

// LDS bytes of fps_block<NT, PPT, CM, FIXED, LDSC> for N points and S samples
__host__ __device__ inline size_t fps_block_lds(int NT, int CM, bool ldsc, int64_t N, int64_t S) {
    const int NW = NT / 64, SLOT = (CM + 2 + 3) & ~3;
    const size_t head = (size_t)((S + 3) & ~3) * 4 + kFpsKeyRegion;
    const size_t cloud = (size_t)N * (CM == 3 ? 4 : CM) * 4;
    return head + (ldsc ? cloud : (size_t)2 * NW * SLOT * 4);
}

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

template <int NT, int PPT, int CM, bool FIXED, bool LDSC, int CR = CM>
__device__ __forceinline__ void fps_block(const FpsArgs &F, const int b, float *fsm) {
    // the reference's separately rounded ops whatever the including unit's -ffp-contract (the
    // SA chain unit that runs the side job contracts its own arithmetic)
#pragma clang fp contract(off)
    const float *__restrict__ pts = F.pts;
    const int N = F.N, Crt = F.C, kind = F.kind, S = F.S, cp = F.cp;
    const int64_t sb = F.sb, sn = F.sn, sc = F.sc;
    const FpsStart &start = F.start;
    int64_t *__restrict__ out_idx = F.out_idx;
    float *__restrict__ out_pts = F.out_pts;
    float *__restrict__ out_packed = F.out_packed;
    float *__restrict__ pts_packed = F.pts_packed;
    constexpr int NW = NT / 64;
    static_assert(NW <= 16, "one 16-lane row reduces the wave slots");
    // In the pipelined launch FPS shares every SIMD with the MLP kernels' waves, and its
    // dependent chain (one short VALU burst, a reduction and a barrier per iteration) is the
    // pipeline's critical path: its waves take issue priority over co-resident waves.
    if (F.prio) __builtin_amdgcn_s_setprio(PN2_FPS_PRIO);
    constexpr int SLOT = (CM + 2 + 3) & ~3;  // {max, index, coords...} padded to 16 bytes
    const int C = FIXED ? CM : Crt;
    const int tid = threadIdx.x;
    const int lane = tid & 63;
    const int wave = tid >> 6;
    const float *P = pts + (int64_t)b * sb;

    int *sidx = reinterpret_cast<int *>(fsm);                          // [S]
    unsigned long long *key = reinterpret_cast<unsigned long long *>(  // [3] (LDSC)
        fsm + ((S + 3) & ~3));
    float *slots = fsm + ((S + 3) & ~3) + kFpsKeyRegion / 4;            // [2][NW][SLOT] (!LDSC)
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
                sq[k] = mul_rn(pj[k], pj[k]);
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
        int *flag = reinterpret_cast<int *>(key + 3);
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

#ifdef PN2_FPS_STAMPS
    unsigned long long st_acc[8] = {0, 0, 0, 0, 0, 0, 0, 0}, st_last = __builtin_amdgcn_s_memtime();
#endif
    for (int i = 0;; ++i) {
        PN2_FPS_T(0);
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
        PN2_FPS_T(1);
        unsigned bv = dist[0];
#pragma unroll
        for (int j = 1; j < PPT; ++j) bv = max(bv, dist[j]);
        // wave: max value, then its first lane (contiguous ownership -> smallest index)
        const unsigned wv = wave_max_u32(bv);
        PN2_FPS_T(2);
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
                PN2_FPS_T(3);
                if (lane == ol) {
                    const unsigned idx = (unsigned)(tid * PPT + bj);
                    atomicMax(&key[i % 3], ((unsigned long long)wv << 32) | (0xFFFFFFFFu - idx));
                }
                if (tid == 64) key[(i + 1) % 3] = 0ull;
                PN2_FPS_T(4);
                __syncthreads();
                PN2_FPS_T(5);
                far = __builtin_amdgcn_readfirstlane((int)(0xFFFFFFFFu - (unsigned)key[i % 3]));
                PN2_FPS_T(6);
            }
#pragma unroll
            for (int k = 0; k < CM; ++k) c[k] = cloud[far * CS + k];
            PN2_FPS_T(7);
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
#ifdef PN2_FPS_STAMPS
    if (b < 4 && lane == 0)
        for (int k = 0; k < 8; ++k) g_fps_stamps[(b * 16 + wave) * 8 + k] = st_acc[k];
#endif

    // ---- outputs: indices, gathered centroids (index_points), packed centroids
    for (int i = tid; i < S; i += NT) {
        const int n = sidx[i];
        out_idx[(int64_t)b * S + i] = n;
        if (out_pts || out_packed) {
            float q[CM], sq[CM];
#pragma unroll
            for (int k = 0; k < CM; ++k) {
                q[k] = (k < C) ? P[(int64_t)n * sn + (int64_t)k * sc] : 0.f;
                sq[k] = mul_rn(q[k], q[k]);
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

}  // namespace pn2
