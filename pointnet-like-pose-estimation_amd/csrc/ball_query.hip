// ball_query.hip -- query_ball_point for gfx950.
//
// Replaces query_ball_point (/root/reference/model/pointnet2_utils.py:70-90) including the
// square_distance it calls (pointnet2_utils.py:5-26).  The reference materialises the full
// [B,S,N] distance matrix, masks it and SORTS every row to find the first K in-radius indices.
// Here no [B,S,N] tensor exists.
//
// Mapping: the 64 lanes of a wave are 64 consecutive centroids of one cloud (a centroid's
// record lives in the lane's registers); the P waves of a workgroup share those centroids and
// split the cloud into consecutive segments of TS points.  The cloud is scanned in rounds of
// P*TS points: the workgroup stages the round's packed records (coords, ssq, pad) in LDS with
// coalesced 16-byte loads, then every wave reads its segment back at wave-uniform addresses
// (one broadcast ds_read_b128 per xyz point, 8 in flight) and tests each point against its
// 64 centroids:
//     d = ((-2 * fma-chain(ctr . p)) + ssq(ctr)) + ssq(p)   (MKL sgemm + ATen sum order;
//         unfused mul/add chain when S*N*C < 400: ATen's naive small-bmm kernel)
//     hit = !(d > (float)(r*r))                              (the reference's masking test)
// A lane accumulates its hits as one bitmask word per 32 points (shift + or, no branch).
// After the scan the per-(segment, centroid) hit counts go through LDS; a lane's prefix over
// the earlier segments and rounds is the output slot of its first hit in the segment, so the
// hits are written in index order ("first K in index order") with no sort.  The workgroup
// stops after the round in which every one of its centroids reached K hits.  Padding (the
// first hit repeated) and the per-centroid distinct-neighbour count (out_cnt, optional: the
// SA chain computes only those rows) are written per centroid row, coalesced.  Workgroups are
// mapped so that all groups of a cloud run on one XCD (one L2 holds the cloud).
//
// Why this shape (profiles/r02_bq/): with lanes = points and one or a few centroids per wave
// (round 1's design, and a multi-centroid LDS-tiled variant of it), every 64 point-centroid
// pairs cost ~28 scalar instructions of ballot / popcount / exec bookkeeping: the SQ counters
// showed 2x more SALU than VALU instructions, and SALU issue bounded the kernel (19-21 us at
// SSG sa1).  Here the bookkeeping is per lane, ~9 vector instructions per point per 64
// centroids and almost no scalar work (9 us).  Points by scalar loads instead of LDS
// (uniform s_load_dwordx16, no staging) measured slower (11-13 us): SMEM returns out of order,
// so every use waits for all loads in flight and their latency is exposed.
#include <stdlib.h>
#include <string.h>

#include "pn2_internal.h"

namespace pn2 {

// CC > 0: the channel count is known at compile time (C = 3 xyz, C = 10 pose) and the shape is
// not ATen's naive-bmm size; CC = 0: runtime C and the `small` flag.  NW bitmask words per
// segment (TS = 32*NW points per wave per round).
// one point record against one centroid: the reference's distance, then its masking test
template <int CP>
__device__ __forceinline__ float bq_dist(const float (&c)[CP], float ssq_c, const float *p, int C, bool small) {
    float mm = __fmul_rn(c[0], p[0]);
#pragma unroll
    for (int k = 1; k < CP - 1; ++k)
        if (k < C) mm = small ? __fadd_rn(mm, __fmul_rn(c[k], p[k])) : __builtin_fmaf(c[k], p[k], mm);
    float sp = p[CP - 1];
#pragma unroll
    for (int k = 1; k < CP - 1; ++k)
        if (k == C) sp = p[k];  // static register indices (no scratch)
    // (-2 * mm) is exact, so one fma rounds (-2 * mm) + ssq_c exactly as the separate ops do
    return __fadd_rn(__builtin_fmaf(-2.0f, mm, ssq_c), sp);
}

template <int CP>
__device__ __forceinline__ unsigned bq_near(const float (&c)[CP], float ssq_c, const float *p, int C,
                                            bool small, float r2) {
    return !(bq_dist<CP>(c, ssq_c, p, C, small) > r2);
}

// wd = 2 wd + hit, hit = !(d > r2) = !(r2 < d): the compare into VCC and one add with carry-in
// (the compiler's select + shift + or is three instructions)
__device__ __forceinline__ void bq_insert(unsigned &wd, float d, float r2) {
    asm volatile("v_cmp_nlt_f32 vcc, %1, %2\n\tv_addc_co_u32 %0, vcc, %0, %0, vcc" : "+v"(wd) : "s"(r2), "v"(d) : "vcc");
}

// OT: the index type written (int64: the reference's query_ball_point; int32: the SA path's
// lists, half the bytes).  ROWBUF: each lane's hits go to its centroid's row of an LDS buffer
// (64 rows of K + 1 entries per radius, dynamic LDS); after the scan every row is written out
// whole, padding included, one coalesced row per wave step.  !ROWBUF (rows too long for LDS, any
// K <= N as the reference's slice [:, :, :nsample] allows, pointnet2_utils.py:87): a hit goes
// straight to its slot of the output row (the slot is known from the prefix), the row's first
// hit is kept in LDS for the padding, and only the padding is written in the coalesced pass.
// NR radii (the MSG layers' scales, pointnet2_utils.py:197-203): one distance per (centroid,
// point) pair, compared with each radius -- NR independent queries, each exactly the
// one-radius query's result (hits past a radius' K are dropped; the scan stops once every
// radius of every centroid has its K).
constexpr int kBqMaxR = 3;
template <typename OT>
struct BqOut {
    float r2[kBqMaxR];
    int K[kBqMaxR];
    int obase[kBqMaxR];  // ROWBUF: element offset of radius r's [64][K + 1] rows in the LDS buffer
    OT *out[kBqMaxR];
    int *cnt[kBqMaxR];
};

template <int CP, int CC, int NW, int P, typename OT, bool ROWBUF, int NR>
__global__ __launch_bounds__(64 * P) void ball_query_kernel(
    const float *__restrict__ pts, const float *__restrict__ ctr, int N, int S, int C_, int small_,
    const BqOut<OT> O, unsigned *__restrict__ err) {
    constexpr int TS = 32 * NW;
    constexpr int TV = P * TS * CP / 4;  // float4 per staged round
    __shared__ float4 tile[TV];
    const int C = CC > 0 ? CC : C_;
    const bool small = CC > 0 ? false : small_;  // the specialised instances never see tiny shapes
    __shared__ int cnts[2][NR][P][64];
    __shared__ int first[NR][64];  // !ROWBUF: each row's first hit (slot 0)
    extern __shared__ __attribute__((aligned(16))) char bq_dyn[];
    OT *obuf = reinterpret_cast<OT *>(bq_dyn);  // [NR][64][K + 1]

    const int lane = threadIdx.x & 63;
    const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int gpc = (S + 63) >> 6;  // 64-centroid groups per cloud
    int bid = blockIdx.x;
    const int nb = gridDim.x;
    if ((nb & 7) == 0) bid = (bid & 7) * (nb >> 3) + (bid >> 3);  // a cloud's groups on one XCD
    const int b = bid / gpc;
    const int g0 = (bid - b * gpc) * 64;
    const int s = g0 + lane;
    const bool valid = s < S;
    const int64_t q = (int64_t)b * S + (valid ? s : g0);

    float c[CP];
    {
        const float4 *cp = reinterpret_cast<const float4 *>(ctr + q * CP);
#pragma unroll
        for (int v = 0; v < CP / 4; ++v) {
            const float4 t = cp[v];
            c[4 * v + 0] = t.x; c[4 * v + 1] = t.y; c[4 * v + 2] = t.z; c[4 * v + 3] = t.w;
        }
    }
    float ssq_c = c[CP - 1];
#pragma unroll
    for (int k = 1; k < CP - 1; ++k)
        if (k == C) ssq_c = c[k];  // static register indices (no scratch)

    // point i of the staged round as a record
    auto point_rec = [&](int i, float (&pv)[CP]) {
        const float4 *tp = tile + i * (CP / 4);
#pragma unroll
        for (int v = 0; v < CP / 4; ++v) {
            const float4 q4 = tp[v];
            pv[4 * v] = q4.x; pv[4 * v + 1] = q4.y; pv[4 * v + 2] = q4.z; pv[4 * v + 3] = q4.w;
        }
    };

    int total[NR];  // hits so far per radius (invalid lanes count as done)
#pragma unroll
    for (int rr = 0; rr < NR; ++rr) total[rr] = valid ? 0 : O.K[rr];
    int r = 0;
    for (int R0 = 0; R0 < N; R0 += P * TS, ++r) {
        const int seg0 = R0 + w * TS;
        unsigned bits[NR][NW];
        int mine[NR];
#pragma unroll
        for (int rr = 0; rr < NR; ++rr) mine[rr] = 0;
        {  // stage the round's P*TS records (coalesced 16-byte loads by the whole workgroup)
            if (R0 > 0) __syncthreads();  // every wave is done with the previous round's tile
            const int npt = min(P * TS, N - R0);
            const float4 *src = reinterpret_cast<const float4 *>(pts + ((int64_t)b * N + R0) * CP);
            const int nv = npt * (CP / 4);
            for (int x = threadIdx.x; x < nv; x += 64 * P) tile[x] = src[x];
            __syncthreads();
        }
#pragma unroll
        for (int t = 0; t < NW; ++t) {
            const int base = seg0 + 32 * t;
            const int np = min(32, N - base);  // points in this word (<= 0: none)
            unsigned wd[NR];
#pragma unroll
            for (int rr = 0; rr < NR; ++rr) wd[rr] = 0;
            if (np == 32 && CC == 0) {  // runtime C (small shapes): one record at a time
#pragma unroll 8
                for (int i = 0; i < 32; ++i) {
                    float pv[CP];
                    point_rec(w * TS + 32 * t + i, pv);
                    const float d = bq_dist<CP>(c, ssq_c, pv, C, small);
#pragma unroll
                    for (int rr = 0; rr < NR; ++rr) bq_insert(wd[rr], d, O.r2[rr]);
                }
            } else if (np == 32) {
                // records in chunks of U points, the next chunk's reads issued before this
                // chunk's arithmetic (bq_insert's asm keeps the compiler from hoisting them
                // itself: one read in flight, its full LDS latency per point)
                constexpr int U = CP == 4 ? 8 : 4;
                const float4 *tw = tile + (w * TS + 32 * t) * (CP / 4);  // uniform addresses
                float pv[2][U][CP];
                auto read_chunk = [&](int k, float (&dst)[U][CP]) {
#pragma unroll
                    for (int u = 0; u < U; ++u)
#pragma unroll
                        for (int v = 0; v < CP / 4; ++v) {
                            const float4 q4 = tw[(k * U + u) * (CP / 4) + v];
                            dst[u][4 * v] = q4.x; dst[u][4 * v + 1] = q4.y; dst[u][4 * v + 2] = q4.z; dst[u][4 * v + 3] = q4.w;
                        }
                };
                read_chunk(0, pv[0]);
#pragma unroll
                for (int k = 0; k < 32 / U; ++k) {
                    if (k + 1 < 32 / U) read_chunk(k + 1, pv[(k + 1) & 1]);
#pragma unroll
                    for (int u = 0; u < U; ++u) {
                        const float d = bq_dist<CP>(c, ssq_c, pv[k & 1][u], C, small);
#pragma unroll
                        for (int rr = 0; rr < NR; ++rr) bq_insert(wd[rr], d, O.r2[rr]);  // point base+i -> bit 31-i
                    }
                }
            } else if (np > 0) {
                for (int i = 0; i < 32; ++i) {
                    float d = 0.f;
                    if (i < np) {
                        float pv[CP];
                        point_rec(w * TS + 32 * t + i, pv);
                        d = bq_dist<CP>(c, ssq_c, pv, C, small);
                    }
#pragma unroll
                    for (int rr = 0; rr < NR; ++rr) wd[rr] = (wd[rr] << 1) | (i < np ? (unsigned)!(d > O.r2[rr]) : 0u);
                }
            }
#pragma unroll
            for (int rr = 0; rr < NR; ++rr) {
                bits[rr][t] = wd[rr];
                mine[rr] += __builtin_popcount(wd[rr]);
            }
        }
#pragma unroll
        for (int rr = 0; rr < NR; ++rr) cnts[r & 1][rr][w][lane] = mine[rr];
        __syncthreads();
        bool more = false;
#pragma unroll
        for (int rr = 0; rr < NR; ++rr) {
            const int K = O.K[rr];
            int off = total[rr], round = 0;
#pragma unroll
            for (int v = 0; v < P; ++v) {
                const int x = cnts[r & 1][rr][v][lane];
                if (v < w) off += x;
                round += x;
            }
            // this segment's hits, in index order, into the slots [off, K)
            OT *orow = O.out[rr] + q * K;  // !ROWBUF (invalid lanes start at total = K: no writes)
#pragma unroll
            for (int t = 0; t < NW; ++t) {
                unsigned wd = bits[rr][t];
                while (wd != 0 && off < K) {
                    const int i = __builtin_clz(wd);
                    const int n = seg0 + 32 * t + i;
                    if constexpr (ROWBUF) {
                        obuf[O.obase[rr] + lane * (K + 1) + off] = (OT)n;
                    } else {
                        orow[off] = (OT)n;
                        if (off == 0) first[rr][lane] = n;
                    }
                    ++off;
                    wd ^= 0x80000000u >> i;
                }
            }
            total[rr] += round;
            more = more || total[rr] < K;
        }
        if (__builtin_amdgcn_ballot_w64(more) == 0) break;  // same in every wave
    }
    __syncthreads();  // every row's hits are in obuf

    // rows out, hits then padding (the first hit; N when there is none: the reference's
    // pad), one centroid row per step, coalesced over the K slots; and the counts
#pragma unroll
    for (int rr = 0; rr < NR; ++rr) {
        const int K = O.K[rr], KP = K + 1;
        for (int j = w; j < 64; j += P) {
            if (g0 + j >= S) break;
            const int cj = min(__builtin_amdgcn_readlane(total[rr], j), K);
            const OT fj = cj > 0 ? (ROWBUF ? obuf[O.obase[rr] + j * KP] : (OT)first[rr][j]) : (OT)N;
            // no point within the radius: the row is padded with index N (the reference's
            // out-of-range pad, pointnet2_utils.py:85-89, which makes its index_points raise
            // IndexError); the SA kernels clamp such indices instead of reading past the cloud
            if (cj == 0 && lane == 0) atomicOr(err, (unsigned)PN2_DEVERR_NO_NEIGHBOUR);
            OT *o = O.out[rr] + ((int64_t)b * S + g0 + j) * K;
            if constexpr (ROWBUF) {
                for (int k = lane; k < K; k += 64) o[k] = k < cj ? obuf[O.obase[rr] + j * KP + k] : fj;
            } else {
                for (int k = cj + lane; k < K; k += 64) o[k] = fj;  // the hits are already out
            }
            if (O.cnt[rr] && lane == 0) O.cnt[rr][(int64_t)b * S + g0 + j] = cj;
        }
    }
}

// Point dimensions 16 < C <= kMaxCWide: lanes = 64 centroids of one cloud as above; every lane
// walks the cloud's packed records in index order (wave-uniform addresses: broadcast loads that
// stay in L1/L2) and writes its first K hits straight into its output row.  Same distance,
// test, hit order, padding, counts and error flag as ball_query_kernel, without the LDS
// staging and segment prefix -- at these widths the scan is a few MFLOP per cloud, and a
// register tile of 64+ channels per record would not leave room for one.
constexpr int kBqWideCP = ((kMaxCWide + 1 + 3) / 4) * 4;

template <typename OT>
__global__ __launch_bounds__(64) void ball_query_wide_kernel(const float *__restrict__ pts,
                                                             const float *__restrict__ ctr, int N, int S,
                                                             int C, int cp, int small, int nr,
                                                             const BqOut<OT> O, unsigned *__restrict__ err) {
    const int gpc = (S + 63) >> 6;
    const int b = blockIdx.x / gpc;
    const int g0 = (blockIdx.x - b * gpc) * 64;
    const int s = g0 + (int)threadIdx.x;
    const bool valid = s < S;
    const int64_t q = (int64_t)b * S + (valid ? s : g0);
    float c[kBqWideCP];
#pragma unroll
    for (int k = 0; k < kBqWideCP; ++k) c[k] = k < cp ? ctr[q * cp + k] : 0.f;
    float ssq_c = 0.f;
#pragma unroll
    for (int k = 1; k < kBqWideCP; ++k)
        if (k == C) ssq_c = c[k];  // static register indices (no scratch)
    int total[kBqMaxR], first[kBqMaxR];
#pragma unroll
    for (int rr = 0; rr < kBqMaxR; ++rr) {
        total[rr] = (valid && rr < nr) ? 0 : O.K[rr];
        first[rr] = N;
    }
    const float *P = pts + (int64_t)b * N * cp;
    for (int n = 0; n < N; ++n) {
        if ((n & 31) == 0) {  // the wave stops once all its centroids have every K
            bool more = false;
#pragma unroll
            for (int rr = 0; rr < kBqMaxR; ++rr) more = more || (rr < nr && total[rr] < O.K[rr]);
            if (__builtin_amdgcn_ballot_w64(more) == 0) break;
        }
        const float *p = P + (int64_t)n * cp;
        float mm = __fmul_rn(c[0], p[0]);
#pragma unroll
        for (int k = 1; k < kBqWideCP - 1; ++k)
            if (k < C) mm = small ? __fadd_rn(mm, __fmul_rn(c[k], p[k])) : __builtin_fmaf(c[k], p[k], mm);
        const float d = __fadd_rn(__builtin_fmaf(-2.0f, mm, ssq_c), p[C]);
#pragma unroll
        for (int rr = 0; rr < kBqMaxR; ++rr) {
            if (rr < nr && !(d > O.r2[rr]) && total[rr] < O.K[rr]) {
                if (total[rr] == 0) first[rr] = n;
                O.out[rr][q * O.K[rr] + total[rr]] = (OT)n;
                ++total[rr];
            }
        }
    }
    if (!valid) return;
#pragma unroll
    for (int rr = 0; rr < kBqMaxR; ++rr) {
        if (rr >= nr) break;
        const int K = O.K[rr], cj = total[rr];
        // no point within the radius: padded with index N, the reference's out-of-range pad
        // (see ball_query_kernel)
        if (cj == 0) atomicOr(err, (unsigned)PN2_DEVERR_NO_NEIGHBOUR);
        OT *o = O.out[rr] + q * K;
        for (int k = cj; k < K; ++k) o[k] = (OT)first[rr];
        if (O.cnt[rr]) O.cnt[rr][q] = cj;
    }
}

}  // namespace pn2

using namespace pn2;

template <typename OT>
static int launch_bq_wide(const float *pp, const float *cp_, int64_t B, int64_t N, int64_t S, int64_t C, int nr,
                          const BqOut<OT> &O, hipStream_t st) {
    const int64_t nblk = B * ((S + 63) / 64);
    PN2_REQUIRE(nblk < (int64_t)1 << 31, "pn2_ball_query_f32: too many centroids");
    unsigned *err = error_word(st);
    PN2_REQUIRE(err, "pn2_ball_query_f32: no device error slot");
    hipLaunchKernelGGL(ball_query_wide_kernel<OT>, dim3((unsigned)nblk), dim3(64), 0, st, pp, cp_, (int)N, (int)S,
                       (int)C, (int)pn2_packed_stride(C), (int)(S * N * C < 400), nr, O, err);
    PN2_LAUNCH_CHECK("ball_query_wide_kernel");
    return PN2_OK;
}

template <int CP, int CC, typename OT, int NR>
static int launch_bq(const float *pp, const float *cp_, int64_t B, int64_t N, int64_t S,
                     int64_t C, BqOut<OT> O, hipStream_t st) {
    const int64_t nblk = B * ((S + 63) / 64);
    PN2_REQUIRE(nblk < (int64_t)1 << 31, "pn2_ball_query_f32: too many centroids");
    // waves per workgroup: bq_waves = 16 (the default: alone on the chip more segments in
    // flight win, SSG eager +1 %, r04) or 8; 0 = the pipelines' choice, 16 for long xyz clouds
    // only (profiles/r02_bq/bq_modes.txt).  Clouds with extra channels keep 8 (LDS budget)
    int P = (CP == 4 && N >= 2048) ? 16 : 8;
    if (tuning().bq_waves) P = (tuning().bq_waves == 16 && CP == 4) ? 16 : 8;
    // words per segment: a round stages up to P*32*nw records (<= 64 per wave beyond xyz)
    const int64_t per_wave = (N + P - 1) / P;
    int nw = per_wave <= 32 ? 1 : per_wave <= 64 ? 2 : 4;
    if (CP > 4 && nw > 2) nw = 2;
    const int sm = (int)(S * N * C < 400);
    // rows in an LDS buffer while they stay within bq_rowbuf_kb (<= 96 KB: with the tile and
    // the counts that still fits a CU), else hits straight to HBM
    size_t obytes = 0;
    for (int r = 0; r < NR; ++r) {
        O.obase[r] = (int)(obytes / sizeof(OT));
        obytes += (size_t)64 * (O.K[r] + 1) * sizeof(OT);
    }
    const int64_t rb_kb = tuning().bq_rowbuf_kb < 96 ? tuning().bq_rowbuf_kb : 96;
    // the kernel's static LDS for this shape (tile + per-segment counts + first hits): the row
    // buffer gets what is left of the CU's 160 KB, else the rows go straight to HBM (an MSG
    // layer's multi-radius launch with long rows would otherwise fail to launch)
    const int nwe = nw == 1 ? 1 : nw == 2 ? 2 : (CP > 4 ? 2 : 4);
    const size_t lds_static = (size_t)P * 32 * nwe * CP * 4 + (size_t)2 * NR * P * 64 * 4 + (size_t)NR * 64 * 4;
    const size_t lds_left = lds_static < (size_t)160 * 1024 ? (size_t)160 * 1024 - lds_static : 0;
    const bool rowbuf = obytes <= (size_t)rb_kb * 1024 && obytes <= lds_left;
    unsigned *err = error_word(st);
    PN2_REQUIRE(err, "pn2_ball_query_f32: no device error slot");
#define PN2_BQ_L2(NW, PP, RB)                                                                          \
    do {                                                                                               \
        static const hipError_t attr = hipFuncSetAttribute(                                           \
            reinterpret_cast<const void *>(&ball_query_kernel<CP, CC, NW, PP, OT, RB, NR>),           \
            hipFuncAttributeMaxDynamicSharedMemorySize, 96 * 1024);                                   \
        PN2_REQUIRE(attr == hipSuccess, "pn2_ball_query_f32: LDS attribute");                         \
        hipLaunchKernelGGL((ball_query_kernel<CP, CC, NW, PP, OT, RB, NR>), dim3((unsigned)nblk),    \
                           dim3(64 * PP), RB ? obytes : 0, st, pp, cp_, (int)N, (int)S, (int)C, sm,   \
                           O, err);                                                                    \
    } while (0)
#define PN2_BQ_L(NW, PP)                    \
    do {                                    \
        if (rowbuf) PN2_BQ_L2(NW, PP, true); \
        else PN2_BQ_L2(NW, PP, false);       \
    } while (0)
    if (P == 8) {
        if (nw == 1) PN2_BQ_L(1, 8);
        else if (nw == 2) PN2_BQ_L(2, 8);
        else PN2_BQ_L((CP > 4 ? 2 : 4), 8);
    } else {
        if (nw == 1) PN2_BQ_L(1, 16);
        else if (nw == 2) PN2_BQ_L(2, 16);
        else PN2_BQ_L((CP > 4 ? 2 : 4), 16);
    }
#undef PN2_BQ_L
#undef PN2_BQ_L2
    PN2_LAUNCH_CHECK("ball_query_kernel");
    return PN2_OK;
}

extern "C" int pn2_ball_query_f32(const float *pts_packed, const float *ctr_packed, int64_t B,
                                  int64_t N, int64_t S, int64_t C, double radius, int64_t K,
                                  int64_t *out_idx, void *stream) {
    return pn2_ball_query_cnt_f32(pts_packed, ctr_packed, B, N, S, C, radius, K, out_idx, nullptr,
                                  stream);
}

// nr radii over the same points and centroids (one launch; nr = 1: query_ball_point)
template <typename OT>
static int ball_query_impl(const float *pts_packed, const float *ctr_packed, int64_t B, int64_t N, int64_t S,
                           int64_t C, int nr, const double *radius, const int64_t *Ks, OT *const *out_idx,
                           int32_t *const *out_cnt, void *stream) {
    PN2_REQUIRE(pts_packed && ctr_packed && out_idx && radius && Ks, "pn2_ball_query_f32: null pointer");
    PN2_REQUIRE(nr >= 1 && nr <= kBqMaxR, "pn2_ball_query_multi: 1..%d radii (got %d)", kBqMaxR, nr);
    PN2_REQUIRE(B >= 0 && N >= 1 && S >= 0 && C >= 1,
                "pn2_ball_query_f32: bad shape B=%lld N=%lld S=%lld C=%lld", (long long)B,
                (long long)N, (long long)S, (long long)C);
    if (C > kMaxCWide)
        return set_error(PN2_EUNSUPPORTED, "pn2_ball_query_f32: unsupported C=%lld (max %d)", (long long)C, kMaxCWide);
    BqOut<OT> O;
    memset(&O, 0, sizeof(O));
    for (int r = 0; r < nr; ++r) {
        const int64_t K = Ks[r];
        PN2_REQUIRE(out_idx[r], "pn2_ball_query_f32: null pointer");
        PN2_REQUIRE(K >= 1, "pn2_ball_query_f32: bad shape K=%lld", (long long)K);
        PN2_REQUIRE(K <= N, "pn2_ball_query_f32: sample_number %lld > N %lld", (long long)K, (long long)N);
        // radius ** 2 in double (Python float), compared in float32 like torch's wrapped scalar
        O.r2[r] = (float)(radius[r] * radius[r]);
        O.K[r] = (int)K;
        O.out[r] = out_idx[r];
        O.cnt[r] = out_cnt ? out_cnt[r] : nullptr;
    }
    PN2_REQUIRE(N < (int64_t)1 << 30 && S < (int64_t)1 << 30, "pn2_ball_query_f32: N or S too large");
    if (B == 0 || S == 0) return PN2_OK;
    hipStream_t st = as_stream(stream);
    const int64_t cp = pn2_packed_stride(C);
    if (C > kMaxC) return launch_bq_wide<OT>(pts_packed, ctr_packed, B, N, S, C, nr, O, st);
#define PN2_BQ(CPV, CC)                                                                               \
    if (cp == CPV && (CC == 0 || (C == CC && S * N * C >= 400)))                                      \
        return nr == 1 ? launch_bq<CPV, CC, OT, 1>(pts_packed, ctr_packed, B, N, S, C, O, st)         \
             : nr == 2 ? launch_bq<CPV, CC, OT, 2>(pts_packed, ctr_packed, B, N, S, C, O, st)         \
                       : launch_bq<CPV, CC, OT, 3>(pts_packed, ctr_packed, B, N, S, C, O, st);
    PN2_BQ(4, 3) PN2_BQ(12, 10)
    PN2_BQ(4, 0) PN2_BQ(8, 0) PN2_BQ(12, 0) PN2_BQ(16, 0) PN2_BQ(20, 0)
#undef PN2_BQ
    return set_error(PN2_EUNSUPPORTED, "pn2_ball_query_f32: C=%lld", (long long)C);
}

extern "C" int pn2_ball_query_cnt_f32(const float *pts_packed, const float *ctr_packed, int64_t B,
                                      int64_t N, int64_t S, int64_t C, double radius, int64_t K,
                                      int64_t *out_idx, int32_t *out_cnt, void *stream) {
    return ball_query_impl<int64_t>(pts_packed, ctr_packed, B, N, S, C, 1, &radius, &K, &out_idx,
                                    out_cnt ? &out_cnt : nullptr, stream);
}

extern "C" int pn2_ball_query_i32(const float *pts_packed, const float *ctr_packed, int64_t B, int64_t N,
                                  int64_t S, int64_t C, double radius, int64_t K, int32_t *out_idx,
                                  int32_t *out_cnt, void *stream) {
    return ball_query_impl<int32_t>(pts_packed, ctr_packed, B, N, S, C, 1, &radius, &K, &out_idx,
                                    out_cnt ? &out_cnt : nullptr, stream);
}

extern "C" int pn2_ball_query_multi_i32(const float *pts_packed, const float *ctr_packed, int64_t B,
                                        int64_t N, int64_t S, int64_t C, int nr, const double *radii,
                                        const int64_t *K, int32_t *const *out_idx, int32_t *const *out_cnt,
                                        void *stream) {
    return ball_query_impl<int32_t>(pts_packed, ctr_packed, B, N, S, C, nr, radii, K, out_idx, out_cnt,
                                    stream);
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
    PN2_REQUIRE(B >= 0 && S >= 0 && N >= 0 && C >= 1, "pn2_square_distance_f32: bad shape");
    if (C > kMaxCWide)
        return set_error(PN2_EUNSUPPORTED, "pn2_square_distance_f32: unsupported C=%lld (max %d)", (long long)C,
                         kMaxCWide);
    const int64_t tot = B * S * N;
    if (tot == 0) return PN2_OK;
    hipLaunchKernelGGL(square_distance_kernel, dim3((unsigned)((tot + 255) / 256)), dim3(256), 0,
                       as_stream(stream), src_packed, dst_packed, B, S, N, (int)C,
                       (int)pn2_packed_stride(C), (int)(S * N * C < 400), out);
    PN2_LAUNCH_CHECK("square_distance_kernel");
    return PN2_OK;
}
