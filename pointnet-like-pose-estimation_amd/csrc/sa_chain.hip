// sa_chain.hip -- register-resident SA layer chain for gfx950: gather -> 3 x (1x1 conv + BN +
// ReLU) -> max over the neighbourhood, with fp32-accurate products on the bf16 matrix cores.
//
// Same job as sa_mlp.hip's fused kernel (PointNetSetAbstraction.forward :163-172,
// PointNetSetAbstractionMsg.forward :211-221 of /root/reference/model/pointnet2_utils.py) for
// the chains every reference head uses (3 layers, hidden widths <= 128, grouped rows).
//
// Arithmetic.  Every fp32 operand x is split into three bf16 planes, x = h + m + l exactly up to
// 2^-24 |x| (h = bf16(x), m = bf16(x - h), l = bf16(x - h - m), round-to-nearest, the residuals
// are exact in fp32).  A product x*w is taken as hh + hm + mh + mm + hl + lh (the dropped terms
// are <= 2^-23 |xw|), each an exact bf16 x bf16 product accumulated in fp32 by
// v_mfma_f32_32x32x16_bf16.  The result has fp32-GEMM accuracy (tests hold it to the same
// 1e-5 bar as the fp32 path) at 6/16 of the fp32 MFMA cost.
//
// Data flow.  One wave owns a slab of 32 consecutive rows (a row = one (group, neighbour) pair)
// and carries it through the whole chain in registers -- no LDS for activations:
//   layer 0   (hidden, transposed: acc[cout tile] += W . X^T) streams 16-channel blocks of the
//             gathered rows from HBM (two 16-byte loads per lane per block: channel-last
//             features, then xyz - centroid), splits them and accumulates every output tile.
//   layer 1   (hidden, transposed) reads its input from registers: the transposed output tile
//             of the previous layer holds, in lane (row r, half h), channels
//             32t + (q&3) + 8(q>>2) + 4h of row r in register q -- exactly the B fragment of the
//             next layer's k-blocks 2t, 2t+1 when the weights are packed with that channel
//             order (pn2_pack_layer_split_bf16).  BN + ReLU + split happen in the epilogue.
//   layer 2   (last, standard orientation: acc[row][col] += X . W^T) takes the same registers
//             as its A operand, so each lane ends with one output column and the tile's rows in
//             registers: the max over the neighbourhood is a register reduction (+ one lane
//             exchange), merged across slabs in LDS (ds_max_u32) or HBM (atomicMax) when a
//             group spans several slabs (ReLU output >= +0: uint order == float order).
// Weights (3 KB per (tile, k-block) step: 1 KB fragment x 3 planes, L2-resident, shared by every
// wave on the chip) are copied by global_load_lds into a small per-wave LDS ring a few steps
// ahead of use (see ring_issue below); BN scale/shift are staged in LDS once per workgroup.
#include "pn2_internal.h"
#include "fps_body.h"
#include "split_bf16.h"

#include <algorithm>

#include <cstdlib>
#include <cstring>

namespace pn2 {

constexpr int kChainWaves = 4;
constexpr int kChainRows = 32 * kChainWaves;

struct ChainLayer {
    const bf16x8 *w;  // [NP][tiles][kb][64] fragments
    const float *alpha;
    const float *beta;
    const float *wscale;  // NP = 2: per output channel, the inverse of the weight row's scale
    int kb;     // 16-deep k blocks of the input
    int tiles;  // 32-wide output tiles
};

struct ChainArgs {
    pn2_sa_src src;
    ChainLayer L[3];
    int M, K, S, C, D;
    int pool_mode;  // 0: registers, 1: LDS (groups inside a workgroup), 2: HBM atomics
    int vec_feat;
    float *out;
    int64_t ostride;
    int lds_bn;    // byte offset of the staged BN scale/shift
    int lds_ring;  // byte offset of the workgroup weight ring (kStages stage buffers)
    // KB0M < 0 (layer 0 pre-transformed): z [B*N][32*T0] = W0 . [xyz | features] of every source
    // point (launch_layer0_prepass); u [B*S][32*T0] = W0_xyz . centroid of every group
    // (u_table_kernel, or compact_scan_kernel's extra workgroups)
    const float *z;
    const float *u;
    // compact neighbourhoods (pool_mode 3, given the ball query's distinct-neighbour counts): a
    // group's rows past its distinct neighbours repeat its first neighbour
    // (pointnet2_utils.py:87-89), and the max over the group is the same without them -- so
    // only each group's distinct rows are computed, in 8-row units laid out in group order, 4
    // per wave (compact_scan_kernel).  cdesc[wg].x = the workgroup's first group within its
    // cloud (y < 0: an unused workgroup); cunits[wg*16 + i] = (group - first) << 8 | unit of
    // the group << 4 | last unit of the group << 3 | (rows of the unit - 1), or -1 (unused).
    const int *cunits;
    const int2 *cdesc;
    int wpc;  // workgroups per cloud
    // compact: LDS pool rows (groups of a workgroup pooled in LDS; a group past them is merged
    // straight into its output row by atomicMax -- compact_scan_kernel zeroed that row) and the
    // weight ring's stage count (2 or 3)
    int pool_rows;
    int ks;
    // side job (pn2_fps_side): workgroups 0 .. fps_blocks-1 of the launch run the next SA
    // layer's FPS, one cloud each (fps_nb clouds; fps_blocks rounded up to a multiple of 8 so the
    // chain's own workgroups keep their XCD placement), the rest the chain (KB0M == 1 instances)
    FpsArgs fps;
    int fps_blocks, fps_nb;
};

// Timeline stamps (diagnostic builds only: -DPN2_CHAIN_STAMPS, tools/debug/chain_stamps.py):
// s_memrealtime (100 MHz, chip-wide) at fixed points of every workgroup, wave 0 lane 0.
#ifdef PN2_CHAIN_STAMPS
constexpr int kStampWG = 16384, kStamps = 6;
__device__ unsigned long long g_chain_stamps[kStampWG * kStamps];
#define PN2_STAMP(i)                                                                          \
    do {                                                                                      \
        if (threadIdx.x == 0 && blockIdx.x < kStampWG)                                        \
            g_chain_stamps[blockIdx.x * kStamps + (i)] = __builtin_amdgcn_s_memrealtime();    \
    } while (0)
#else
#define PN2_STAMP(i) do {} while (0)
#endif

constexpr int kUnitRows = 8;
constexpr int kUnitsPerWG = kChainRows / kUnitRows;  // 16

// Pool merges.  HBM: a global_atomic_umax through a global (not generic) pointer -- a flat
// atomic counts in both vmcnt and lgkmcnt and the compiler drained vmcnt(0) (the weight ring's
// copies in flight) before each one.  LDS: ds_max_u32 as inline asm -- as a C++ atomic the
// compiler waited for every LDS-DMA copy in flight (vmcnt(0)) first, since the ring's copies
// write the same dynamic LDS array; the pool never overlaps the ring, and its readers sit
// behind a barrier with lgkmcnt(0).
__device__ __forceinline__ void hbm_max_u32(float *p, unsigned v) {
    __hip_atomic_fetch_max(reinterpret_cast<__attribute__((address_space(1))) unsigned *>(
                               reinterpret_cast<uintptr_t>(p)),
                           v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void lds_max_u32(unsigned *p, unsigned v) {
    const unsigned a = (unsigned)(size_t)(__attribute__((address_space(3))) unsigned *)p;
    asm volatile("ds_max_u32 %0, %1" ::"v"(a), "v"(v) : "memory");
}

template <int NP>
__device__ __forceinline__ Split load_w(const ChainLayer &L, int t, int kb, int lane) {
    const int64_t plane = (int64_t)L.tiles * L.kb * 64;
    const bf16x8 *p = L.w + ((int64_t)t * L.kb + kb) * 64 + lane;
    Split s;
    s.h = p[0];
    s.m = NP >= 2 ? p[plane] : s.h;
    s.l = NP == 3 ? p[2 * plane] : s.h;
    return s;
}

// BN + ReLU of a transposed hidden tile, split into the next layer's k-blocks 2t, 2t+1
// al/be: this layer's BN scale/shift staged in LDS
// asc: NP = 2, the down-scale of the layer's input activations (act_scale), else 1
template <int NP>
__device__ __forceinline__ void hidden_epilogue(const cfloatx16 &acc, const float *al,
                                                const float *be, int t, int h, Split &lo,
                                                Split &hi, float asc = 1.f) {
    cfloatx4 a4[4], b4[4];
#pragma unroll
    for (int m = 0; m < 4; ++m) {
        a4[m] = *reinterpret_cast<const cfloatx4 *>(al + 32 * t + 8 * m + 4 * h);
        b4[m] = *reinterpret_cast<const cfloatx4 *>(be + 32 * t + 8 * m + 4 * h);
        if constexpr (NP == 2) a4[m] *= asc;
    }
    float y0[8], y1[8];
#pragma unroll
    for (int q = 0; q < 8; ++q) {
        y0[q] = chain_relu(__builtin_fmaf(acc[q], a4[q >> 2][q & 3], b4[q >> 2][q & 3]));
        y1[q] = chain_relu(__builtin_fmaf(acc[q + 8], a4[2 + (q >> 2)][q & 3], b4[2 + (q >> 2)][q & 3]));
    }
    lo = splitN<NP>(y0);
    hi = splitN<NP>(y1);
}


// Layer 0's output blocks (layer 1's input) are held as fp32 when the arithmetic is split
// (NP = 3: 8 VGPRs per block instead of 12 for the three bf16 planes) and split as layer 1
// consumes them -- layer 1 runs k-outer, so each block is still split exactly once.  At the
// start of layer 1 the whole input and every accumulator of the layer are live: for the (4, 4)
// chains that is 96 + 64 VGPRs split, 64 + 64 as fp32.
struct F8 {
    float v[8];
};
template <int NP> struct HidT { using type = Split; };
template <> struct HidT<3> { using type = F8; };
template <> struct HidT<2> { using type = F8; };  // (split after the wave's scale is known)

template <int NP>
__device__ __forceinline__ void hidden_epilogue_h(const cfloatx16 &acc, const float *al,
                                                  const float *be, int t, int h,
                                                  typename HidT<NP>::type &lo,
                                                  typename HidT<NP>::type &hi, float asc = 1.f) {
    if constexpr (NP >= 2) {
        cfloatx4 a4[4], b4[4];
#pragma unroll
        for (int m = 0; m < 4; ++m) {
            a4[m] = *reinterpret_cast<const cfloatx4 *>(al + 32 * t + 8 * m + 4 * h);
            b4[m] = *reinterpret_cast<const cfloatx4 *>(be + 32 * t + 8 * m + 4 * h);
            if constexpr (NP == 2) a4[m] *= asc;
        }
#pragma unroll
        for (int q = 0; q < 8; ++q) {
            lo.v[q] = chain_relu(__builtin_fmaf(acc[q], a4[q >> 2][q & 3], b4[q >> 2][q & 3]));
            hi.v[q] = chain_relu(__builtin_fmaf(acc[q + 8], a4[2 + (q >> 2)][q & 3], b4[2 + (q >> 2)][q & 3]));
        }
    } else {
        hidden_epilogue<NP>(acc, al, be, t, h, lo, hi);
    }
}
template <int NP>
__device__ __forceinline__ Split hid_split(const Split &x, float = 1.f) { return x; }
template <int NP>
__device__ __forceinline__ Split hid_split(const F8 &x, float up = 1.f) {
    if constexpr (NP == 2) {
        float y[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) y[j] = x.v[j] * up;
        return splitN<NP>(y);
    } else {
        return splitN<NP>(x.v);
    }
}
// NP = 2: the wave-uniform scale of a set of activations from the lane's running max of their
// magnitudes (as uint bits: order-preserving for values >= +0)
__device__ __forceinline__ ActScale wave_act_scale(unsigned lane_max_bits) {
    return act_scale(__uint_as_float(wave_max_u32(lane_max_bits)));
}
__device__ __forceinline__ unsigned mag_bits(float x) { return __float_as_uint(x) & 0x7fffffffu; }
__device__ __forceinline__ unsigned hid_dep(const Split &x) {
    return __builtin_bit_cast(unsigned, __builtin_shufflevector(x.h, x.h, 0, 1));
}
__device__ __forceinline__ unsigned hid_dep(const F8 &x) { return __float_as_uint(x.v[0]); }

// Materialise a split pair in registers at this point (see the layer-0 pre-pass loop): keeps
// the compiler from sinking an epilogue to the pair's last use and holding its inputs live.
template <int NP>
__device__ __forceinline__ void pin_pair(Split &a, Split &b) {
    if constexpr (NP == 3)
        asm volatile("" : "+v"(a.h), "+v"(a.m), "+v"(a.l), "+v"(b.h), "+v"(b.m), "+v"(b.l));
    else if constexpr (NP == 2)
        asm volatile("" : "+v"(a.h), "+v"(a.m), "+v"(b.h), "+v"(b.m));
    else
        asm volatile("" : "+v"(a.h), "+v"(b.h));
}
template <int NP>
__device__ __forceinline__ void pin_pair(F8 &a, F8 &b) {
    asm volatile("" : "+v"(a.v[0]), "+v"(a.v[1]), "+v"(a.v[2]), "+v"(a.v[3]), "+v"(a.v[4]),
                      "+v"(a.v[5]), "+v"(a.v[6]), "+v"(a.v[7]));
    asm volatile("" : "+v"(b.v[0]), "+v"(b.v[1]), "+v"(b.v[2]), "+v"(b.v[3]), "+v"(b.v[4]),
                      "+v"(b.v[5]), "+v"(b.v[6]), "+v"(b.v[7]));
}

// ---- workgroup weight ring.  A step = one (tile, k-block) of a layer = its three 1 KB plane
// fragments; every wave of the workgroup consumes the same steps in the same order (its own 32
// rows), so one LDS copy of a step feeds all four waves' MFMAs (128 rows per 3 KB of weights --
// per-wave copies made the L2 -> LDS weight stream, not the MFMA, the bound).  Steps are copied
// HBM/L2 -> LDS by global_load_lds (lane-linear, no VGPRs) in stages of kChainWaves steps: wave
// w copies step kChainWaves*st + w of stage st into stage buffer st % kStages.  At the first
// step of stage st every wave
//   1. waits for its own earlier LDS reads (lgkmcnt(0): stage st-1 is no longer read by it),
//   2. waits for its own copy of stage st (counted vmcnt: stages st+1 .. st+kStages-2 stay in
//      flight),
//   3. s_barrier (raw: __syncthreads' fence would wait vmcnt(0) and drain the ring) -- now
//      stage st is whole in LDS and no wave reads stage st-1 any more,
//   4. copies its step of stage st+kStages-1 into stage st-1's buffer.
// Past the last step the copies repeat the last step (same counts, never read).
constexpr int kStages = 3;
template <int NP> constexpr int step_bytes() { return NP * 1024; }  // one step: NP planes
template <int NP> constexpr int stage_bytes() { return kChainWaves * step_bytes<NP>(); }

// frag: the step's plane-0 fragment (wave-uniform); loff = lane * 16 -- the uniform-base +
// lane-offset form lets the copy use a scalar base address (no per-copy vector address math)
template <int NP>
__device__ __forceinline__ void ring_issue(const bf16x8 *frag, int64_t plane, char *slot,
                                           unsigned loff) {
#pragma unroll
    for (int p = 0; p < NP; ++p)
        __builtin_amdgcn_global_load_lds(reinterpret_cast<const char *>(frag + p * plane) + loff,
                                         (lds_void *)(slot + p * 1024), 16, 0, 0);
}

// step 2 above: this wave's copies of the kStages-2 younger stages (NP each) may stay in flight
// (KS == 2, the compact launches' shallower ring: nothing younger is in flight)
template <int NP, int KS>
__device__ __forceinline__ void stage_wait() {
    static_assert(KS == 2 || KS == 3, "stage_wait count");
    if constexpr (KS == 2) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    else if constexpr (NP == 3) asm volatile("s_waitcnt vmcnt(3)" ::: "memory");
    else if constexpr (NP == 2) asm volatile("s_waitcnt vmcnt(2)" ::: "memory");
    else asm volatile("s_waitcnt vmcnt(1)" ::: "memory");
}

// Before a buffer is refilled, this wave's reads of it must have returned.  The compiler does
// not see that global_load_lds (addressed through M0) writes that buffer, so the memory clobber
// also keeps those reads from being scheduled after the refill.
__device__ __forceinline__ void ring_fence() { asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory"); }

__device__ __forceinline__ void stage_barrier() {
    asm volatile("" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
}

// KB0M > 0: the layer-0 input (<= KB0M k-blocks) is gathered once into registers and layer 0 runs
// tile by tile from the ring like layers 1 and 2; KB0M == 0: layer 0 streams its input blocks
// (k-outer, every output tile accumulating) with ordinary loads and the ring starts at layer 1.
// KS: weight-ring stages (3; 2 for compact launches, whose LDS group pool needs the room)
template <int T0, int T1, int KB0M, int NP, int KS>
__global__ __launch_bounds__(64 * kChainWaves) __attribute__((amdgpu_waves_per_eu(3))) void sa_chain_kernel(
    const ChainArgs A) {
    constexpr int kStepBytes = step_bytes<NP>(), kStageBytes = stage_bytes<NP>();
    extern __shared__ __attribute__((aligned(16))) char csm[];
    constexpr int KB1 = 2 * T0, KB2 = 2 * T1;
    unsigned *cpool = reinterpret_cast<unsigned *>(csm);
    const int tid = threadIdx.x;
    const int lane = tid & 63;
    const int r = lane & 31, h = lane >> 5;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    // a cloud's workgroups on one XCD: its rows gather the same points (and the pre-pass wrote
    // that cloud's z rows from the same XCD, see sa_dense.hip)
    PN2_STAMP(0);
    if constexpr (KB0M == 1) {
        // the FPS side job: dispatched first (lowest ids), at issue priority 3 (fps_block) beside
        // the chain's waves on its CUs; no barrier of the chain is reached by these workgroups
        if ((int)blockIdx.x < A.fps_blocks) {
            if ((int)blockIdx.x < A.fps_nb) {
                if (A.fps.C == 3) fps_block<256, 2, 3, true, true>(A.fps, (int)blockIdx.x, reinterpret_cast<float *>(csm));
                else fps_block<256, 2, 10, true, true>(A.fps, (int)blockIdx.x, reinterpret_cast<float *>(csm));
            }
            return;
        }
    }
    const int bid = (int)xcd_contiguous(blockIdx.x - (unsigned)A.fps_blocks, gridDim.x - (unsigned)A.fps_blocks);
    const int slab = bid * kChainWaves + wave;
    const pn2_sa_src &s = A.src;
    const ChainLayer &L0 = A.L[0], &L1 = A.L[1], &L2 = A.L[2];
    const int coutL = 32 * L2.tiles;
    const bool compact = A.pool_mode == 3;
    unsigned c_g0 = 0;
    int c_ng = 0, c_flags = 0;
    if (compact) {
        const int2 d = A.cdesc[bid];
        if (d.y < 0) {  // no rows left for this workgroup (uniform: before any barrier)
            PN2_STAMP(5);
            return;
        }
        c_g0 = (unsigned)(bid / A.wpc) * (unsigned)A.S + (unsigned)d.x;
        c_ng = d.y & 255;
        c_flags = d.y >> 8;
    }
    // groups per workgroup of the LDS pool (pool_mode 1; compact: up to one per unit)
    const int gpb = compact ? A.pool_rows : kChainRows / A.K;

    // ---- prologue.  vmcnt counts in issue order (a wait for one load waits for every older
    // one), so the independent loads go out oldest-first in the order they are needed: the BN
    // operands (registers, written to LDS below), the first weight-ring stages (they land while
    // the dependent row gather runs, instead of after the setup barrier), then the gather.
    float *bn = reinterpret_cast<float *>(csm + A.lds_bn);
    float *al0 = bn, *be0 = al0 + 32 * T0, *al1 = be0 + 32 * T0, *be1 = al1 + 32 * T1;
    float *al2 = be1 + 32 * T1, *be2 = al2 + coutL;
    const bool bnreg = coutL <= 2 * 64 * kChainWaves;  // every thread's share fits 8 registers
    float bnv[8];
    // NP = 2: the BN scale of a layer whose products run on the chain's MFMAs takes the inverse
    // of the weight rows' scale (split_bf16.h); a pre-transformed layer 0 has none (wscale null)
    auto alpha_of = [&](const ChainLayer &L, int c) {
        if constexpr (NP == 2) return L.wscale ? L.alpha[c] * L.wscale[c] : L.alpha[c];
        else return L.alpha[c];
    };
    if (bnreg) {
        const int e2 = tid + 64 * kChainWaves;
        bnv[0] = tid < 32 * T0 ? alpha_of(L0, tid) : 0.f;
        bnv[1] = tid < 32 * T0 ? L0.beta[tid] : 0.f;
        bnv[2] = tid < 32 * T1 ? alpha_of(L1, tid) : 0.f;
        bnv[3] = tid < 32 * T1 ? L1.beta[tid] : 0.f;
        bnv[4] = tid < coutL ? alpha_of(L2, tid) : 0.f;
        bnv[5] = tid < coutL ? L2.beta[tid] : 0.f;
        bnv[6] = e2 < coutL ? alpha_of(L2, e2) : 0.f;
        bnv[7] = e2 < coutL ? L2.beta[e2] : 0.f;
    }

    char *ring = csm + A.lds_ring;
    const unsigned loff = (unsigned)lane * 16u;
    // Ring steps in consumption order: layers 0 (resident input only) and 1 block-major, layer 2
    // tile-major; source addresses come from scalar arithmetic on the layer's base.
    auto issue_l = [&](const ChainLayer &L, int t, int kb, char *dst) {
        ring_issue<NP>(L.w + ((int64_t)t * L.kb + kb) * 64, (int64_t)L.tiles * L.kb * 64, dst, loff);
    };
    auto issue2 = [&](int z, char *dst) {  // layer-2 step z
        z = min(z, L2.tiles * KB2 - 1);
        issue_l(L2, z / KB2, z % KB2, dst);
    };
    auto issue1 = [&](int y, char *dst) {  // layer-1 step y (block-major)
        if (y < T1 * KB1) issue_l(L1, y % T1, y / T1, dst);
        else issue2(y - T1 * KB1, dst);
    };
    const int n0 = T0 * L0.kb;
    auto issue_stage = [&](int st) {  // this wave's step of stage st
        const int x = st * kChainWaves + wave;
        char *dst = ring + (st % KS) * kStageBytes + wave * kStepBytes;
        if constexpr (KB0M > 0) {
            if (x < n0) issue_l(L0, x % T0, x / T0, dst);
            else issue1(x - n0, dst);
        } else {
            issue1(x, dst);
        }
    };
    int nread = 0;
    auto read_w = [&]() {
        if ((nread & (kChainWaves - 1)) == 0) {  // first step of a stage
            const int st = nread / kChainWaves;
            ring_fence();
            stage_wait<NP, KS>();
            stage_barrier();
            issue_stage(st + KS - 1);
        }
        const Split w = ring_readN<NP>(ring + ((nread / kChainWaves) % KS) * kStageBytes +
                                      (nread & (kChainWaves - 1)) * kStepBytes, lane);
        ++nread;
        return w;
    };
    // One step of lookahead: the next step's weight planes are read before this step's MFMAs
    // (the compiler kept two fragments in flight and waited lgkmcnt(0) every 2-3 MFMAs: an LDS
    // round trip exposed per step, ISA of sa_chain_kernel<4,4,-1>).  The last step reads one
    // step past the end, unconditionally: a branch there made every step's MFMAs a control-flow
    // merge, where the compiler waited for the lookahead reads as well (lgkmcnt(0)).  The ring
    // repeats its last step past the end, so that read is in bounds; it is never used.
    Split wpre;
    bool primed = false;
    auto next_w = [&]() {
        if (!primed) {
            wpre = read_w();
            primed = true;
        }
        const Split w = wpre;
        wpre = read_w();
        return w;
    };
    // ASMR (split chains with a register-resident or pre-transformed layer 0): the weight
    // planes are read by inline-asm ds_read_b128 into two register sets used alternately, the
    // next step's reads issued before this step's MFMAs, and each step waits for its own reads
    // only (lgkmcnt(3): the next step's three reads may stay in flight).  The compiler's own
    // schedule kept one or two fragments in flight and waited lgkmcnt(0) before most MFMAs
    // (register pressure, and the stage-sync branch merges).  Pending asm reads never cross a
    // control-flow merge: the runtime tile loop of layer 2 waits lgkmcnt(0) before its back-edge.
#ifndef PN2_CHAIN_ASMR
#define PN2_CHAIN_ASMR 1
#endif
    constexpr bool ASMR = PN2_CHAIN_ASMR && NP >= 2 && (KB0M == 1 || KB0M < 0);
    Split WB[2];
    int nr = 0;  // ASMR: the next step to read
    const unsigned ring3 = (unsigned)(size_t)(__attribute__((address_space(3))) char *)ring;
    auto rd = [&](Split &w) {
        if ((nr & (kChainWaves - 1)) == 0) {  // first step of a stage: see read_w
            ring_fence();
            stage_wait<NP, KS>();
            stage_barrier();
            issue_stage(nr / kChainWaves + KS - 1);
        }
        const unsigned a = ring3 + (unsigned)(((nr / kChainWaves) % KS) * kStageBytes +
                                              (nr & (kChainWaves - 1)) * kStepBytes) + loff;
        if constexpr (NP == 3)
            asm volatile("ds_read_b128 %0, %3\n\tds_read_b128 %1, %3 offset:1024\n\tds_read_b128 %2, %3 offset:2048"
                         : "=&v"(w.h), "=&v"(w.m), "=&v"(w.l)
                         : "v"(a));
        else
            asm volatile("ds_read_b128 %0, %2\n\tds_read_b128 %1, %2 offset:1024"
                         : "=&v"(w.h), "=&v"(w.m)
                         : "v"(a));
        ++nr;
    };
    // wait for this step's reads; the next step's NP reads (issued after them) may stay in flight
    auto wt3 = [&](Split &w) {
        if constexpr (NP == 3) asm volatile("s_waitcnt lgkmcnt(3)" : "+v"(w.h), "+v"(w.m), "+v"(w.l));
        else asm volatile("s_waitcnt lgkmcnt(2)" : "+v"(w.h), "+v"(w.m));
    };
    auto wt0 = [&](Split &w) {
        if constexpr (NP == 3) asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(w.h), "+v"(w.m), "+v"(w.l));
        else asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(w.h), "+v"(w.m));
    };
    constexpr int P0 = KB0M > 0 ? T0 * KB0M : 0;  // ASMR layer-0 steps (L0.kb == KB0M == 1)
    constexpr int P1 = P0 + T1 * KB1;              // steps before layer 2

    if constexpr (KB0M != 0) {  // KB0M == 0: the ring starts after layer 0's streamed loads
#pragma unroll
        for (int st = 0; st < KS - 1; ++st) issue_stage(st);
    }


    // ---- this lane's row: (group g, batch b, point n)
    unsigned g;
    bool valid;
    int n, urow_e = -1;
    if (compact) {
        // unit i of the workgroup = rows 8(i%4).. of wave i/4; a row past the unit's distinct
        // neighbours takes the unit's first (a distinct neighbour of the same group)
        urow_e = A.cunits[bid * kUnitsPerWG + wave * 4 + (r >> 3)];
        valid = urow_e >= 0;
        const int k = (urow_e >> 4) & 15, nv = (urow_e & 7) + 1;
        g = valid ? c_g0 + (unsigned)(urow_e >> 8) : c_g0;
        const int j = kUnitRows * k + ((r & 7) < nv ? (r & 7) : 0);
        n = valid ? src_index(s, (int64_t)g * A.K + j) : 0;
    } else {
        const unsigned R = (unsigned)slab * 32u + (unsigned)r;
        valid = R < (unsigned)A.M;
        g = valid ? R / (unsigned)A.K : 0u;
        n = valid ? src_index(s, R) : 0;
    }
    // a centroid with no neighbour in its radius is padded with N (the ball query raises
    // PN2_DEVERR_NO_NEIGHBOUR): read point 0 there, never past the cloud
    if ((unsigned)n >= (unsigned)s.N) n = 0;
    const unsigned b = g / (unsigned)A.S;
    const float *frow = s.feat ? s.feat + (int64_t)b * s.fb + (int64_t)n * s.fn : nullptr;
    const float *prow = s.pts + (int64_t)b * s.pb + (int64_t)n * s.pn;
    const float *crow = s.ctr + (int64_t)g * A.C;
    const int D = A.D, C = A.C;

    // Row layout: block 0 = [xyz - centroid | 0], blocks >= 1 = features (16 per block).  Lane
    // (r, h) holds channels 16kb + (j&3) + 8(j>>2) + 4h of its row in element j.
    auto load_x = [&](int kb, float (&x)[8]) {
        if (kb == 0) {
#pragma unroll
            for (int j = 0; j < 8; ++j) {
                const int ch = (j & 3) + 8 * (j >> 2) + 4 * h;
                x[j] = (valid && ch < C) ? __fsub_rn(prow[(int64_t)ch * s.pc], crow[ch]) : 0.f;
            }
            return;
        }
#pragma unroll
        for (int run = 0; run < 2; ++run) {
            const int f = 16 * (kb - 1) + 8 * run + 4 * h;
            if (A.vec_feat) {
                cfloatx4 q = {0.f, 0.f, 0.f, 0.f};
                if (valid && f < D) q = *reinterpret_cast<const cfloatx4 *>(frow + f);
#pragma unroll
                for (int i = 0; i < 4; ++i) x[4 * run + i] = q[i];
            } else {
#pragma unroll
                for (int i = 0; i < 4; ++i) x[4 * run + i] = (valid && f + i < D) ? frow[f + i] : 0.f;
            }
        }
    };

    // The row gather (unit table -> neighbour index -> point / feature / pre-pass row: a chain
    // of dependent loads) is issued here, before the BN staging and its barrier, so its latency
    // overlaps the setup instead of following it (tools/debug/chain_stamps.py: the gather was
    // ~28 % of a workgroup's life at SSG sa1).
    float x0[KB0M > 0 ? KB0M : 1][8];  // KB0M > 0: the whole layer-0 input
    float xs0[8];                       // KB0M == 0: its first block
    cfloatx4 zc[4], uc[4];              // KB0M < 0: tile 0 of the row's z and its group's u
    if constexpr (KB0M > 0) {
#pragma unroll
        for (int kb = 0; kb < KB0M; ++kb) {
            if (kb < L0.kb) {
                load_x(kb, x0[kb]);
            } else {
#pragma unroll
                for (int j = 0; j < 8; ++j) x0[kb][j] = 0.f;
            }
        }
    } else if constexpr (KB0M == 0) {
        load_x(0, xs0);
    } else {
        const float *zrow0 = A.z + ((int64_t)b * s.N + n) * (32 * T0);
        const float *urow0 = A.u + (int64_t)g * (32 * T0);
#pragma unroll
        for (int m = 0; m < 4; ++m) {
            zc[m] = *reinterpret_cast<const cfloatx4 *>(zrow0 + 4 * h + 8 * m);
            uc[m] = *reinterpret_cast<const cfloatx4 *>(urow0 + 4 * h + 8 * m);
        }
    }

    // BN operands to LDS, the pool zeroed; no vmcnt drain at the barrier: the gather and the
    // ring's first stages stay in flight (their consumers wait for them)
    if (bnreg) {
        const int e2 = tid + 64 * kChainWaves;
        if (tid < 32 * T0) { al0[tid] = bnv[0]; be0[tid] = bnv[1]; }
        if (tid < 32 * T1) { al1[tid] = bnv[2]; be1[tid] = bnv[3]; }
        if (tid < coutL) { al2[tid] = bnv[4]; be2[tid] = bnv[5]; }
        if (e2 < coutL) { al2[e2] = bnv[6]; be2[e2] = bnv[7]; }
    } else {
        for (int e = tid; e < coutL; e += 64 * kChainWaves) { al2[e] = alpha_of(L2, e); be2[e] = L2.beta[e]; }
        for (int e = tid; e < 32 * T0; e += 64 * kChainWaves) { al0[e] = alpha_of(L0, e); be0[e] = L0.beta[e]; }
        for (int e = tid; e < 32 * T1; e += 64 * kChainWaves) { al1[e] = alpha_of(L1, e); be1[e] = L1.beta[e]; }
    }
    if (A.pool_mode == 1 || compact)
        for (int e = tid; e < gpb * coutL; e += 64 * kChainWaves) cpool[e] = 0u;
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    stage_barrier();
    PN2_STAMP(1);
    typename HidT<NP>::type X1[2 * T0];
    if constexpr (KB0M < 0) {
        // ---- layer 0 pre-transformed: acc = z[point] - u[group], already in the transposed
        // accumulator layout (register 4m + i of lane (r, h) = channel 32t + 8m + 4h + i)
        const float *zrow = A.z + ((int64_t)b * s.N + n) * (32 * T0);
        const float *urow = A.u + (int64_t)g * (32 * T0);
        // Tile t+1's z / u loads are issued while tile t is split (one tile of lookahead).  The
        // loads are read-only, so the compiler would hoist every tile's loads to the top and
        // spill at 2 waves/SIMD: the address of tile t+1 is tied (opaque asm) to tile t-1's
        // result, which bounds the loads in flight to two tiles.
        auto load_tile = [&](int o, cfloatx4 (&zq)[4], cfloatx4 (&uq)[4]) {
#pragma unroll
            for (int m = 0; m < 4; ++m) {
                zq[m] = *reinterpret_cast<const cfloatx4 *>(zrow + o + 8 * m);
                uq[m] = *reinterpret_cast<const cfloatx4 *>(urow + o + 8 * m);
            }
        };
        unsigned dep = 0;
#pragma unroll
        for (int t = 0; t < T0; ++t) {
            cfloatx4 zn[4], un[4];
            if (t + 1 < T0) {
                int o = 32 * (t + 1) + 4 * h;
                asm volatile("" : "+v"(o) : "v"(dep));
                load_tile(o, zn, un);
            }
            cfloatx16 acc;
#pragma unroll
            for (int m = 0; m < 4; ++m)
#pragma unroll
                for (int i = 0; i < 4; ++i) acc[4 * m + i] = zc[m][i] - uc[m][i];
            int zero = 0;  // the BN scale / shift reads of tile t wait for tile t-1 likewise
            asm volatile("" : "+v"(zero) : "v"(dep));
            hidden_epilogue_h<NP>(acc, al0 + zero, be0 + zero, t, h, X1[2 * t], X1[2 * t + 1]);
            dep = hid_dep(X1[2 * t]);
#pragma unroll
            for (int m = 0; m < 4; ++m) zc[m] = zn[m], uc[m] = un[m];
            // Materialise tile t's split planes here: otherwise the epilogue of the last tile is
            // sunk to its use at the end of layer 1, keeping its raw inputs (accumulator, BN
            // scale / shift) live across layer 1 -- 24 VGPRs of spill at 2 waves/SIMD.
            pin_pair<NP>(X1[2 * t], X1[2 * t + 1]);
        }
    } else if constexpr (KB0M > 0) {
        // ---- layer 0 from registers: the whole input gathered once (raw fp32), then k-outer
        // (each block split once, every output tile accumulating) with weights from the ring
        auto &x = x0;  // gathered before the setup; the ring's first stages are in flight
        cfloatx16 acc[T0];
#pragma unroll
        for (int t = 0; t < T0; ++t)
#pragma unroll
            for (int q = 0; q < 16; ++q) acc[t][q] = 0.f;
        float asc0 = 1.f;  // NP = 2: the down-scale of layer 0's input
        if constexpr (NP == 2) {
            unsigned mb = 0;
#pragma unroll
            for (int kb = 0; kb < KB0M; ++kb)
#pragma unroll
                for (int j = 0; j < 8; ++j) mb = max(mb, mag_bits(x[kb][j]));
            const ActScale sc = wave_act_scale(mb);
#pragma unroll
            for (int kb = 0; kb < KB0M; ++kb)
#pragma unroll
                for (int j = 0; j < 8; ++j) x[kb][j] *= sc.up;
            asc0 = sc.down;
        }
        if constexpr (ASMR) {  // KB0M == 1: one block, T0 steps
            rd(WB[0]);
            const Split xs = splitN<NP>(x[0]);
#pragma unroll
            for (int t = 0; t < T0; ++t) {
                rd(WB[(t + 1) & 1]);
                wt3(WB[t & 1]);
                acc[t] = mma_wa<NP>(WB[t & 1], xs, acc[t]);
            }
        } else {
#pragma unroll
            for (int kb = 0; kb < KB0M; ++kb) {
                if (kb < L0.kb) {
                    const Split xs = splitN<NP>(x[kb]);
#pragma unroll
                    for (int t = 0; t < T0; ++t) acc[t] = mma_wa<NP>(next_w(), xs, acc[t]);
                }
            }
        }
#pragma unroll
        for (int t = 0; t < T0; ++t) {
            hidden_epilogue_h<NP>(acc[t], al0, be0, t, h, X1[2 * t], X1[2 * t + 1], asc0);
            pin_pair<NP>(X1[2 * t], X1[2 * t + 1]);
        }
    } else {
        // ---- layer 0 streamed: k-outer, every output tile accumulating (transposed)
        cfloatx16 acc[T0];
#pragma unroll
        for (int t = 0; t < T0; ++t)
#pragma unroll
            for (int q = 0; q < 16; ++q) acc[t][q] = 0.f;
        float xn[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) xn[j] = xs0[j];  // block 0, gathered before the setup
        for (int kb = 0; kb < L0.kb; ++kb) {
            float x[8];
#pragma unroll
            for (int j = 0; j < 8; ++j) x[j] = xn[j];
            if (kb + 1 < L0.kb) load_x(kb + 1, xn);
            const Split xs = splitN<NP>(x);
#pragma unroll
            for (int t = 0; t < T0; ++t) acc[t] = mma_wa<NP>(load_w<NP>(L0, t, kb, lane), xs, acc[t]);
        }
        // layer 0's loads are all consumed: start the ring, then the epilogue hides its latency
#pragma unroll
        for (int st = 0; st < KS - 1; ++st) issue_stage(st);
#pragma unroll
        for (int t = 0; t < T0; ++t) {
            hidden_epilogue_h<NP>(acc[t], al0, be0, t, h, X1[2 * t], X1[2 * t + 1]);
            pin_pair<NP>(X1[2 * t], X1[2 * t + 1]);
        }
    }

    PN2_STAMP(2);
    // ---- layer 1: input in registers, k-outer (each input block dies after its use, so X1 and
    // X2 are never both whole in registers), every output tile accumulating (transposed)
    Split X2[2 * T1];
    float asc2 = 1.f;  // NP = 2: the down-scale of layer 2's input
    {
        cfloatx16 acc[T1];
#pragma unroll
        for (int t = 0; t < T1; ++t)
#pragma unroll
            for (int q = 0; q < 16; ++q) acc[t][q] = 0.f;
        // NP = 2: one scale for the wave's layer-1 input (ReLU outputs, >= +0)
        float up1 = 1.f, asc1 = 1.f;
        if constexpr (NP == 2) {
            unsigned mb = 0;
#pragma unroll
            for (int kb = 0; kb < KB1; ++kb)
#pragma unroll
                for (int j = 0; j < 8; ++j) mb = max(mb, __float_as_uint(X1[kb].v[j]));
            const ActScale sc = wave_act_scale(mb);
            up1 = sc.up;
            asc1 = sc.down;
        }
        if constexpr (ASMR) {
            if constexpr (KB0M < 0) rd(WB[0]);  // (KB0M == 1: layer 0 read this step ahead)
#pragma unroll
            for (int kb = 0; kb < KB1; ++kb) {
                const Split xs = hid_split<NP>(X1[kb], up1);
#pragma unroll
                for (int t = 0; t < T1; ++t) {
                    constexpr int dummy = 0;
                    (void)dummy;
                    const int g = P0 + kb * T1 + t;  // compile-time after unrolling
                    rd(WB[(g + 1) & 1]);
                    wt3(WB[g & 1]);
                    acc[t] = mma_wa<NP>(WB[g & 1], xs, acc[t]);
                }
            }
        } else {
#pragma unroll
            for (int kb = 0; kb < KB1; ++kb) {
                const Split xs = hid_split<NP>(X1[kb], up1);
#pragma unroll
                for (int t = 0; t < T1; ++t) acc[t] = mma_wa<NP>(next_w(), xs, acc[t]);
            }
        }
        if constexpr (NP == 2) {
            // BN + ReLU of every tile in place (fp32), then one scale for the wave's layer-2
            // input, then the split
            F8 y[2 * T1];
            unsigned mb = 0;
#pragma unroll
            for (int t = 0; t < T1; ++t) {
                hidden_epilogue_h<NP>(acc[t], al1, be1, t, h, y[2 * t], y[2 * t + 1], asc1);
#pragma unroll
                for (int j = 0; j < 8; ++j)
                    mb = max(mb, max(__float_as_uint(y[2 * t].v[j]), __float_as_uint(y[2 * t + 1].v[j])));
            }
            const ActScale sc = wave_act_scale(mb);
            asc2 = sc.down;
#pragma unroll
            for (int kb = 0; kb < KB2; ++kb) X2[kb] = hid_split<NP>(y[kb], sc.up);
        } else {
#pragma unroll
            for (int t = 0; t < T1; ++t) hidden_epilogue<NP>(acc[t], al1, be1, t, h, X2[2 * t], X2[2 * t + 1]);
        }
    }

    PN2_STAMP(3);
    // ---- layer 2: standard orientation, pooled over the neighbourhood
    const unsigned G = (unsigned)A.M / (unsigned)A.K;
    for (int t = 0; t < L2.tiles; ++t) {
        cfloatx16 acc;
#pragma unroll
        for (int q = 0; q < 16; ++q) acc[q] = 0.f;
        if constexpr (ASMR) {
#pragma unroll
            for (int kb = 0; kb < KB2; ++kb) {
                const int b = (P1 + kb) & 1;  // KB2 is even: the same parity in every tile
                rd(WB[b ^ 1]);                // kb = KB2 - 1: the next tile's first step
                wt3(WB[b]);
                acc = mma_wb<NP>(X2[kb], WB[b], acc);
            }
        } else {
#pragma unroll
            for (int kb = 0; kb < KB2; ++kb) acc = mma_wb<NP>(X2[kb], next_w(), acc);
        }
        // max over rows of relu(fma(acc, al, be)) = relu(fma(extreme, al, be)) exactly: fma with
        // a fixed al is monotone in acc (non-decreasing for al >= 0, else non-increasing) and
        // so is relu -- only the row max (al >= 0) or min of the accumulator is needed.
        // Register q of lane half h is row (q&3) + 8(q>>2) + 4h of the slab.
        const int col = 32 * t + r;
        const float al = NP == 2 ? al2[col] * asc2 : al2[col], be = be2[col];
        const bool up = al >= 0.f;
        auto fin = [&](float mx, float mn) { return chain_relu(__builtin_fmaf(up ? mx : mn, al, be)); };
        if (compact) {
            // one max per 8-row unit (registers 4k..4k+3 of both halves); consecutive units of a
            // group merged in registers, then into the workgroup's LDS pool (ds_max_u32; ReLU
            // outputs >= +0: uint order == float order).  No global write inside the ring's
            // loop: its counted vmcnt waits would also wait for them.
            float smx = 0.f, smn = 0.f;
            int sg = -1;
            auto flush = [&]() {
                if (sg >= 0 && h == 0) {
                    if (sg < gpb)
                        lds_max_u32(&cpool[sg * coutL + col], __float_as_uint(fin(smx, smn)));
                    else  // past the pool (rare): the row was zeroed by the scan
                        hbm_max_u32(A.out + (int64_t)(c_g0 + (unsigned)sg) * A.ostride + col,
                                    __float_as_uint(fin(smx, smn)));
                }
            };
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                const int ue = __builtin_amdgcn_readlane(urow_e, 8 * k);  // uniform
                if (ue < 0) break;  // units are used in order: the rest of the slab is unused
                float mx = fmaxf(fmaxf(acc[4 * k], acc[4 * k + 1]), fmaxf(acc[4 * k + 2], acc[4 * k + 3]));
                float mn = fminf(fminf(acc[4 * k], acc[4 * k + 1]), fminf(acc[4 * k + 2], acc[4 * k + 3]));
                mx = max_halves(mx);
                mn = min_halves(mn);
                if ((ue >> 8) != sg) {
                    flush();
                    sg = ue >> 8;
                    smx = mx;
                    smn = mn;
                } else {
                    smx = fmaxf(smx, mx);
                    smn = fminf(smn, mn);
                }
            }
            flush();
        } else if (A.K == 8 || A.K == 16) {
            float mx[4], mn[4];
#pragma unroll
            for (int k = 0; k < 4; ++k) {  // rows 8k..8k+7 of the slab: registers 4k..4k+3, both halves
                mx[k] = fmaxf(fmaxf(acc[4 * k], acc[4 * k + 1]), fmaxf(acc[4 * k + 2], acc[4 * k + 3]));
                mn[k] = fminf(fminf(acc[4 * k], acc[4 * k + 1]), fminf(acc[4 * k + 2], acc[4 * k + 3]));
                mx[k] = max_halves(mx[k]);
                mn[k] = min_halves(mn[k]);
            }
            if (h == 0) {
                if (A.K == 8) {
#pragma unroll
                    for (int k = 0; k < 4; ++k) {
                        const unsigned gg = (unsigned)slab * 4u + k;
                        if (gg < G) A.out[(int64_t)gg * A.ostride + col] = fin(mx[k], mn[k]);
                    }
                } else {
#pragma unroll
                    for (int k = 0; k < 2; ++k) {
                        const unsigned gg = (unsigned)slab * 2u + k;
                        if (gg < G)
                            A.out[(int64_t)gg * A.ostride + col] =
                                fin(fmaxf(mx[2 * k], mx[2 * k + 1]), fminf(mn[2 * k], mn[2 * k + 1]));
                    }
                }
            }
        } else {
            float mx = acc[0], mn = acc[0];
#pragma unroll
            for (int q = 1; q < 16; ++q) {
                mx = fmaxf(mx, acc[q]);
                mn = fminf(mn, acc[q]);
            }
            const float m = fin(max_halves(mx), min_halves(mn));
            const unsigned gg = ((unsigned)slab * 32u) / (unsigned)A.K;
            if (h == 0 && (unsigned)slab * 32u < (unsigned)A.M) {
                if (A.pool_mode == 0) A.out[(int64_t)gg * A.ostride + col] = m;
                else if (A.pool_mode == 1)
                    lds_max_u32(&cpool[(int)(gg - (unsigned)bid * gpb) * coutL + col], __float_as_uint(m));
                else
                    hbm_max_u32(A.out + (int64_t)gg * A.ostride + col, __float_as_uint(m));
            }
        }
        // ASMR: the next tile's first weights (read under this tile's last MFMAs and its
        // epilogue) have landed before the loop's back-edge
        if constexpr (ASMR) wt0(WB[P1 & 1]);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the ring's trailing (repeat) copies
    PN2_STAMP(4);
    if (compact) {
        __syncthreads();
        // a group shared with the neighbouring workgroup is merged by atomicMax into its row
        // (zeroed by compact_scan_kernel); the others are stored
        for (int e = tid; e < min(c_ng, gpb) * coutL; e += 64 * kChainWaves) {
            const int gl = e / coutL, c = e - gl * coutL;
            float *o = A.out + (int64_t)(c_g0 + (unsigned)gl) * A.ostride + c;
            if ((gl == 0 && (c_flags & 1)) || (gl == c_ng - 1 && (c_flags & 2)))
                hbm_max_u32(o, cpool[e]);
            else
                *o = __uint_as_float(cpool[e]);
        }
    } else if (A.pool_mode == 1) {
        __syncthreads();
        for (int e = tid; e < gpb * coutL; e += 64 * kChainWaves) {
            const int gl = e / coutL, c = e - gl * coutL;
            const unsigned gg = (unsigned)bid * gpb + gl;
            if (gg < G) A.out[(int64_t)gg * A.ostride + c] = __uint_as_float(cpool[e]);
        }
    }
    PN2_STAMP(5);
}

// hidden-width signatures (output tiles of layers 0 and 1) compiled; the reference heads use
// SSG [64,64,128] [128,128,256], MSG [32,32,64] [64,64,128] [64,96,128] [128,128,256]
// (T0, T1, KB0M): KB0M = 1 for xyz-only inputs (sa1 layers), 9 for 131/138-channel inputs
// (SSG/pose sa2), 0 = streamed layer-0 input (any width)
// -1 = layer 0 pre-transformed per source point (wide first layers, see chain_use_prepass)
#define PN2_CHAIN_SIGS(X) \
    X(1, 1, 1) X(2, 2, 1) X(2, 3, 1) X(4, 4, 9) X(1, 1, 0) X(2, 2, 0) X(2, 3, 0) X(4, 4, 0) \
    X(2, 2, -1) X(4, 4, -1)

}  // namespace pn2

using namespace pn2;

// ------------------------------------------------------------------ weight packing
// Kernel input channel k of a layer (k-block kb = k / 16) -> input channel of W:
//   xyz == 0 (hidden layers)  k (0 past cin)
//   xyz  > 0 (first layer: rows [xyz | features], D = cin - xyz)
//             block 0 holds xyz - centroid (k < xyz), blocks >= 1 the features (k - 16 < D);
//             W's order is [xyz, features] when xyz_first (sample_and_group, :114), else
//             [features, xyz] (PointNetSetAbstractionMsg, :209).
// Fragment element: plane p, tile t, block kb, lane l = 32h + r, element j holds
//   W[32t + r][in(16kb + (j&3) + 8(j>>2) + 4h)]  split into bf16 planes hi / mid / lo
// (planes 0-2), then the same fragments of W[o][.] * 2^e_o split into fp16 planes hi / lo
// (planes 3-4, the NP = 2 chains: e_o puts the row's largest |w| in [2^14, 2^15)), then the
// per-row inverse scales 2^-e_o as float [cout] (split_bf16.h).
__device__ __forceinline__ int split_in_channel(int k, int cin, int xyz, int xyz_first) {
    if (xyz == 0) return k < cin ? k : -1;
    const int D = cin - xyz;
    if (k < 16) return k < xyz ? (xyz_first ? k : D + k) : -1;
    const int f = k - 16;
    return f < D ? (xyz_first ? xyz + f : f) : -1;
}

// the fp16 image's row scales: 2^e_o with the row's largest |w| * 2^e_o in [2^14, 2^15) (1 for
// an all-zero row); the image keeps the inverse
__device__ __forceinline__ float row_scale_exp2(const float *__restrict__ Wrow, int cin, bool inverse) {
    float m = 0.f;
    for (int k = 0; k < cin; ++k) m = fmaxf(m, fabsf(Wrow[k]));
    int e = 0;
    if (m > 0.f) e = 15 - __builtin_amdgcn_frexp_expf(m);
    e = e < -100 ? -100 : (e > 100 ? 100 : e);
    return __uint_as_float((unsigned)(127 + (inverse ? -e : e)) << 23);
}

__global__ __launch_bounds__(256) void pack_scale_kernel(const float *__restrict__ W, int cout, int cin,
                                                          float *__restrict__ inv) {
    const int o = blockIdx.x * 256 + threadIdx.x;
    if (o < cout) inv[o] = row_scale_exp2(W + (int64_t)o * cin, cin, true);
}

__global__ __launch_bounds__(256) void pack_split_kernel(const float *__restrict__ W, int cout,
                                                          int cin, int kbs, int xyz, int xyz_first,
                                                          __bf16 *__restrict__ out,
                                                          const float *__restrict__ inv) {
    const int64_t per_plane = (int64_t)cout * kbs * 16;
    const int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (e >= per_plane) return;
    const int j = (int)(e & 7);
    const int l = (int)((e >> 3) & 63);
    const int64_t f = e >> 9;  // fragment = t * kbs + kb
    const int kb = (int)(f % kbs), t = (int)(f / kbs);
    const int r = l & 31, h = l >> 5;
    const int ci = split_in_channel(16 * kb + (j & 3) + 8 * (j >> 2) + 4 * h, cin, xyz, xyz_first);
    const float w = ci >= 0 ? W[(int64_t)(32 * t + r) * cin + ci] : 0.f;
    const __bf16 a = (__bf16)w;
    const float r1 = w - (float)a;
    const __bf16 m = (__bf16)r1;
    const __bf16 lo = (__bf16)(r1 - (float)m);
    out[e] = a;
    out[per_plane + e] = m;
    out[2 * per_plane + e] = lo;
    // fp16 planes of the scaled row (inv[] was written by pack_scale_kernel before this launch)
    const float ws = w * (1.f / inv[32 * t + r]);  // exact: a power of two
    const _Float16 fh = (_Float16)ws;
    const _Float16 fl = (_Float16)(ws - (float)fh);
    _Float16 *o16 = reinterpret_cast<_Float16 *>(out + 3 * per_plane);
    o16[e] = fh;
    o16[per_plane + e] = fl;
}

extern "C" int64_t pn2_layer_split_kblocks(int64_t cin, int64_t xyz) {
    if (cin < 1 || xyz < 0 || xyz > 16 || xyz > cin) return -1;
    return xyz > 0 ? 1 + (cin - xyz + 15) / 16 : (cin + 15) / 16;
}

extern "C" int64_t pn2_layer_split_bytes(int64_t cout, int64_t cin, int64_t xyz) {
    const int64_t kbs = pn2_layer_split_kblocks(cin, xyz);
    if (cout < 32 || cout % 32 != 0 || kbs < 0) return -1;
    return 5 * cout * kbs * 16 * 2 + (cout * 4 + 15) / 16 * 16;
}


extern "C" int pn2_pack_layer_split_bf16(const float *W, int64_t cout, int64_t cin, int64_t xyz,
                                         int xyz_first, void *out, void *stream) {
    PN2_REQUIRE(W && out, "pn2_pack_layer_split_bf16: null pointer");
    const int64_t kbs = pn2_layer_split_kblocks(cin, xyz);
    PN2_REQUIRE(cout >= 32 && cout % 32 == 0 && kbs > 0,
                "pn2_pack_layer_split_bf16: bad shape cout=%lld cin=%lld xyz=%lld", (long long)cout,
                (long long)cin, (long long)xyz);
    PN2_REQUIRE(((uintptr_t)out & 15) == 0, "pn2_pack_layer_split_bf16: output not 16-byte aligned");
    const int64_t per_plane = cout * kbs * 16;
    float *inv = const_cast<float *>(split_f16_inv_scale(out, cout, kbs));
    hipLaunchKernelGGL(pack_scale_kernel, dim3((unsigned)((cout + 255) / 256)), dim3(256), 0,
                       as_stream(stream), W, (int)cout, (int)cin, inv);
    PN2_LAUNCH_CHECK("pack_scale_kernel");
    hipLaunchKernelGGL(pack_split_kernel, dim3((unsigned)((per_plane + 255) / 256)), dim3(256), 0,
                       as_stream(stream), W, (int)cout, (int)cin, (int)kbs, (int)xyz, xyz_first ? 1 : 0,
                       reinterpret_cast<__bf16 *>(out), inv);
    PN2_LAUNCH_CHECK("pack_split_kernel");
    return PN2_OK;
}

// ------------------------------------------------------------------ compact neighbourhoods
namespace pn2 {

// One workgroup per cloud: every group's 8-row units (its distinct-neighbour count from the
// ball query, pn2_ball_query_cnt_f32, rounded up to whole units) laid out in group order (an
// exclusive scan), 16 units per chain workgroup; the workgroup descriptors and unit table the
// chain kernel reads; and a zeroed output row for every group whose units span two workgroups
// (merged there by atomicMax).
// 512 threads: in the pipeline the scan's workgroups wait for CU room beside the chains; 8-wave
// workgroups get it sooner than 16-wave ones (SSG, interleaved A/B x3: 130.3-132.5k vs
// 128.6-129.8k clouds/s with 1024, 128.7-130.9k with 256)
#ifndef PN2_SCAN_THREADS
#define PN2_SCAN_THREADS 512
#endif
constexpr int kScanThreads = PN2_SCAN_THREADS;

// Pre-pass chains: workgroups B .. B + gridDim.x - 1 of the same launch compute the centroid
// term u [g][c] = sum_k W0[c][xyz k] * centroid[g][k] (k ascending, one fma chain from 0), the
// centroid's share of layer 0 that the per-point z cannot subtract (W0's fp32 image is
// pair-interleaved [cin_pad/2][cout0][2], its xyz rows from w0x_row).  One launch fewer on the
// compute stream than a u kernel of its own (4.8 us); as a job of the B scan workgroups it made
// the launch 6 -> 22 us (SSG sa2, eager), on the chain's critical path.
__global__ __launch_bounds__(kScanThreads) void compact_scan_kernel(
    const int *__restrict__ cnt, int B, int S, int K, int wpc, int *__restrict__ units,
    int2 *__restrict__ desc, float *__restrict__ out, int64_t ostride, int cout, int prow,
    const float *__restrict__ w0x, int w0x_row, int cout0, const float *__restrict__ ctr, int C,
    float *__restrict__ u) {
    if ((int)blockIdx.x >= B) {
        // a contiguous range of groups per workgroup; thread t keeps output column t % cout0
        // (its W0 xyz weights in registers) over groups t / cout0, + kScanThreads / cout0, ...
        const int G = B * S, nwg = gridDim.x - B;
        const int gper = (G + nwg - 1) / nwg, g0 = ((int)blockIdx.x - B) * gper;
        const int g1 = min(G, g0 + gper);
        const int tid = threadIdx.x;
        if (kScanThreads % cout0 == 0 && C <= kMaxC) {
            const int c = tid % cout0, gstep = kScanThreads / cout0;
            float w[kMaxC];
#pragma unroll
            for (int k = 0; k < kMaxC; ++k) {
                const int row = w0x_row + k;
                w[k] = k < C ? w0x[((int64_t)(row >> 1) * cout0 + c) * 2 + (row & 1)] : 0.f;
            }
            for (int g = g0 + tid / cout0; g < g1; g += gstep) {
                const float *cg = ctr + (int64_t)g * C;
                float acc = 0.f;
#pragma unroll
                for (int k = 0; k < kMaxC; ++k)
                    if (k < C) acc = __builtin_fmaf(w[k], cg[k], acc);
                u[(int64_t)g * cout0 + c] = acc;
            }
        } else {
            for (int e = tid; e < (g1 - g0) * cout0; e += kScanThreads) {
                const int g = g0 + e / cout0, c = e % cout0;
                float acc = 0.f;
                for (int k = 0; k < C; ++k) {
                    const int row = w0x_row + k;
                    acc = __builtin_fmaf(w0x[((int64_t)(row >> 1) * cout0 + c) * 2 + (row & 1)],
                                         ctr[(int64_t)g * C + k], acc);
                }
                u[(int64_t)g * cout0 + c] = acc;
            }
        }
        return;
    }
    extern __shared__ int ssm[];
    int *st = ssm;            // [S] units of group s, then its first unit
    int *strad = st + S;      // [S] groups to zero
    int *glo = strad + S;     // [wpc] first group of each workgroup
    int *wsum = glo + wpc;    // [16] wave totals, [16] straddler count
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int b = blockIdx.x;
    const int *cb = cnt + (int64_t)b * S;
    const int per = (S + kScanThreads - 1) / kScanThreads;
    const int lo = min(S, tid * per), hi = min(S, lo + per);
    int sum = 0;
    for (int i = lo; i < hi; ++i) {
        const int u = max(1, (cb[i] + kUnitRows - 1) / kUnitRows);
        st[i] = u;
        sum += u;
    }
    if (tid == 0) wsum[16] = 0;
    // exclusive scan of the per-thread sums: within each wave, then over the 16 wave totals
    int inc = sum;
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) {
        const int v = __shfl_up(inc, off);
        if (lane >= off) inc += v;
    }
    if (lane == 63) wsum[wave] = inc;
    __syncthreads();
    int wpre = 0, total = 0;
    for (int w = 0; w < kScanThreads / 64; ++w) {
        const int t = wsum[w];
        if (w < wave) wpre += t;
        total += t;
    }
    int run = wpre + inc - sum;
    for (int i = lo; i < hi; ++i) {
        const int u = st[i];
        st[i] = (run << 8) | u;
        run += u;
    }
    __syncthreads();
    // the first group of every workgroup (the one holding unit 16w)
    for (int i = tid; i < S; i += kScanThreads) {
        const int s0 = st[i] >> 8, en = s0 + (st[i] & 255) - 1;
        for (int w = (s0 + kUnitsPerWG - 1) / kUnitsPerWG; w * kUnitsPerWG <= en; ++w) glo[w] = i;
    }
    __syncthreads();
    // rows to zero: groups that span two workgroups, and groups past the pool rows of the
    // workgroup holding their first unit (both merged by atomicMax)
    for (int i = tid; i < S; i += kScanThreads) {
        const int s0 = st[i] >> 8, en = s0 + (st[i] & 255) - 1;
        if (s0 / kUnitsPerWG != en / kUnitsPerWG || i - glo[s0 / kUnitsPerWG] >= prow)
            strad[atomicAdd(&wsum[16], 1)] = i;
    }
    __syncthreads();
    for (int w = tid; w < wpc; w += kScanThreads) {
        int2 d = make_int2(0, -1);
        if (w * kUnitsPerWG < total) {
            const int g = glo[w];
            // last group: the one holding the workgroup's last used unit
            const int lu = min((w + 1) * kUnitsPerWG, total) - 1;
            int l = g;
            while (l + 1 < S && (st[l + 1] >> 8) <= lu) ++l;
            const int first = (st[g] >> 8) < w * kUnitsPerWG ? 1 : 0;
            const int last = (st[l] >> 8) + (st[l] & 255) > (w + 1) * kUnitsPerWG ? 2 : 0;
            d = make_int2(g, (l - g + 1) | ((first | last) << 8));
        }
        desc[(int64_t)b * wpc + w] = d;
    }
    int *ub = units + (int64_t)b * wpc * kUnitsPerWG;
    for (int u = total + tid; u < wpc * kUnitsPerWG; u += kScanThreads) ub[u] = -1;
    for (int i = tid; i < S; i += kScanThreads) {
        const int s0 = st[i] >> 8, nu = st[i] & 255;
        for (int k = 0; k < nu; ++k) {
            // rows past the distinct ones inside a unit are the group's padding (repeats of its
            // first neighbour); only rows past K (K % 8 != 0) are cut
            const int u = s0 + k, nv = min(kUnitRows, K - kUnitRows * k);
            ub[u] = ((i - glo[u / kUnitsPerWG]) << 8) | (k << 4) | ((k == nu - 1) << 3) | (nv - 1);
        }
    }
    const int ns = wsum[16];
    for (int e = tid; e < ns * cout; e += kScanThreads) {
        const int j = e / cout, c = e - j * cout;
        out[((int64_t)b * S + strad[j]) * ostride + c] = 0.f;
    }
}

// u without compaction: the same fma chain as compact_scan_kernel's u workgroups
__global__ __launch_bounds__(256) void u_table_kernel(const float *__restrict__ w0x, int w0x_row,
                                                      int cout, const float *__restrict__ ctr,
                                                      int C, int64_t G, float *__restrict__ u) {
    const int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (e >= G * cout) return;
    const int64_t g = e / cout;
    const int c = (int)(e - g * cout);
    float acc = 0.f;
    for (int k = 0; k < C; ++k) {
        const int row = w0x_row + k;
        acc = __builtin_fmaf(w0x[((int64_t)(row >> 1) * cout + c) * 2 + (row & 1)], ctr[g * C + k], acc);
    }
    u[e] = acc;
}

// ------------------------------------------------------------------ host: dispatch

#ifdef PN2_CHAIN_STAMPS
// copy the stamps of the last chain launch out (diagnostic builds only)
extern "C" int pn2_debug_chain_stamps(unsigned long long *dst, int64_t n) {
    const int64_t m = n < (int64_t)kStampWG * kStamps ? n : (int64_t)kStampWG * kStamps;
    return hipMemcpyFromSymbol(dst, HIP_SYMBOL(g_chain_stamps), m * 8) == hipSuccess ? 0 : -1;
}
#endif

template <int T0, int T1, int KB0M, int NP>
static int launch_chain_sig(const ChainArgs &A, unsigned grid, size_t lds, hipStream_t st) {
    if constexpr (NP == 2 && KB0M != 1 && KB0M != -1) {
        return set_error(PN2_EUNSUPPORTED, "sa_chain: no split-fp16 instance");  // (not reached)
    } else {
        if (A.pool_mode == 3 && A.ks == 2)
            hipLaunchKernelGGL((sa_chain_kernel<T0, T1, KB0M, NP, 2>), dim3(grid), dim3(64 * kChainWaves), lds, st, A);
        else
            hipLaunchKernelGGL((sa_chain_kernel<T0, T1, KB0M, NP, kStages>), dim3(grid), dim3(64 * kChainWaves), lds, st, A);
        PN2_LAUNCH_CHECK("sa_chain_kernel");
        return PN2_OK;
    }
}

// planes of the last chain launch on this thread (pn2_sa_mlp_last_planes)
static thread_local int g_last_planes = 0;

// the compiled KB0M for this chain: the smallest resident bound >= kb0, else 0 (streamed);
// -1 when (T0, T1) has no instance
static int chain_kb0m(int T0, int T1, int kb0) {
    int best = -1;
#define PN2_CHAIN_HAS(a, b, c) \
    if (c >= 0 && T0 == a && T1 == b && (c == 0 ? best < 0 : (kb0 <= c && (best <= 0 || c < best)))) best = c;
    PN2_CHAIN_SIGS(PN2_CHAIN_HAS)
#undef PN2_CHAIN_HAS
    return best;
}

// Layer-0 pre-pass (KB0M = -1).  Layer 0 is linear in [xyz - centroid | features], so
// W0 . row = W0 . [xyz | features](point) - W0_xyz . centroid: the first term depends only on
// the source point and is computed once per point (launch_layer0_prepass) instead of once per
// (group, neighbour) row -- K*S/N times fewer products (16x at SSG sa2) -- and the chain gathers
// it in place of the raw row.  Used for wide first layers (>= 5 k-blocks) of fp32 chains with
// a compiled (T0, T1, -1) instance when the rows outnumber the points 4:1, given workspace.
static bool chain_use_prepass(const pn2_sa_src &s, const pn2_mlp_layer *layers, int T0, int T1,
                              int kb0, int64_t M, int np) {
    if (np != 3 || kb0 < 5 || s.C < 1 || s.C > kMaxC || !layers[0].wt) return false;
    if (!tuning().chain_prepass) return false;
    if (4 * s.B * s.N > M) return false;
    bool has = false;
#define PN2_CHAIN_HAS(a, b, c) \
    if (c < 0 && T0 == a && T1 == b) has = true;
    PN2_CHAIN_SIGS(PN2_CHAIN_HAS)
#undef PN2_CHAIN_HAS
    return has;
}

static bool chain_shape(const pn2_sa_src &s, const pn2_mlp_layer *layers, int nlayers, int pool,
                        int &T0, int &T1, int (&kbs)[3]) {
    if (nlayers != 3 || !pool) return false;
    if (s.mode != PN2_SRC_GROUP_XYZ_FIRST && s.mode != PN2_SRC_GROUP_FEAT_FIRST) return false;
    if (s.C > kMaxC) return false;
    for (int l = 0; l < 3; ++l)
        if (!layers[l].wt_split || ((uintptr_t)layers[l].wt_split & 15) ||
            (layers[l].flags & PN2_LAYER_NO_RELU))
            return false;
    T0 = (int)(layers[0].cout / 32);
    T1 = (int)(layers[1].cout / 32);
    kbs[0] = (int)pn2_layer_split_kblocks(layers[0].cin, s.C);
    kbs[1] = (int)((layers[1].cin + 15) / 16);
    kbs[2] = (int)((layers[2].cin + 15) / 16);
    return kbs[0] >= 1;
}

// compact neighbourhoods (pool_mode 3): groups of K in [9, 128] (K <= 8 is one unit anyway),
// given the ball query's counts, the scan kernel's LDS within one CU's 160 KB.  Tuning
// compact = 0 disables (A/B); compact_stages = 3 keeps the 3-stage ring.
static int64_t compact_wpc(const pn2_sa_src &s) {
    return (s.S * ((s.K + kUnitRows - 1) / kUnitRows) + kUnitsPerWG - 1) / kUnitsPerWG;
}
static size_t compact_scan_lds(const pn2_sa_src &s) {
    return (size_t)(2 * s.S + compact_wpc(s) + 32) * 4;
}
static bool chain_use_compact(const pn2_sa_src &s) {
    if (!s.cnt || s.K <= kUnitRows || s.K > 128 || s.S < 1) return false;
    if (compact_scan_lds(s) > (size_t)160 * 1024) return false;
    if (!tuning().compact) return false;
    return true;
}
static int64_t compact_table_bytes(const pn2_sa_src &s) {
    return s.B * compact_wpc(s) * (kUnitsPerWG * 4 + 8);
}

// the pre-pass tables: z [B*N][cout0] and u [B*S][cout0], 16-byte aligned each
static int64_t prepass_z_bytes(const pn2_sa_src &s, const pn2_mlp_layer &L0) {
    return (s.B * s.N * L0.cout * 4 + 15) / 16 * 16;
}
static int64_t prepass_bytes(const pn2_sa_src &s, const pn2_mlp_layer &L0) {
    return prepass_z_bytes(s, L0) + (s.B * s.S * L0.cout * 4 + 15) / 16 * 16;
}

// workspace of a chain launch: [pre-pass z | pre-pass u | compact unit table | descriptors]
int64_t chain_prepass_bytes(const pn2_sa_src &s, const pn2_mlp_layer *layers, int nlayers, int np) {
    int T0, T1, kbs[3];
    if (!chain_shape(s, layers, nlayers, 1, T0, T1, kbs)) return 0;
    if (chain_kb0m(T0, T1, kbs[0]) < 0) return 0;
    const int64_t M = s.B * s.S * s.K;
    int64_t bytes = 0;
    if (chain_use_prepass(s, layers, T0, T1, kbs[0], M, np))
        bytes += prepass_bytes(s, layers[0]);
    if (chain_use_compact(s)) bytes += compact_table_bytes(s);
    return bytes;
}

// 1: launched, 0: this chain is not eligible (caller uses the fp32 kernels), <0: error
int try_launch_chain(const pn2_sa_src &s, const pn2_mlp_layer *layers, int nlayers, int pool,
                     float *out, int64_t ostride, int64_t M, int64_t K, int np, float *ws,
                     int64_t ws_bytes, hipStream_t st) {
    if (np == 3 && tuning().mlp_f32) return 0;
    // k-blocks per layer (the first layer's rows are [xyz | features], see split_in_channel)
    int T0, T1, kbs[3];
    if (!chain_shape(s, layers, nlayers, pool, T0, T1, kbs)) return 0;
    int KB0M = chain_kb0m(T0, T1, kbs[0]);
    if (KB0M < 0) return 0;
    // bf16 chains stream a multi-block layer-0 input rather than hold it resident: the
    // resident block takes the VGPRs of a wave per SIMD (STRESS sa2 (4,4): 144 -> 112 VGPRs,
    // 3 -> 4 waves/SIMD; eager 265 -> 193 us, pipelined STRESS 124.6k -> 130.1k clouds/s).  The
    // split (fp32) chains gain nothing: (4,4,9) 158, (4,4,0) 151 VGPRs, both 3 waves/SIMD.
    if (np == 1 && KB0M > 1 && chain_kb0m(T0, T1, 1 << 20) == 0) KB0M = 0;
    // without compaction a 32-row slab must hold rows of one group (K = 8, 16: several whole
    // groups; K % 32 == 0: part of one)
    if (!(pool && chain_use_compact(s)) && !(K == 8 || K == 16 || K % 32 == 0)) return 0;
    const int64_t pbytes = prepass_bytes(s, layers[0]);
    const bool pre = chain_use_prepass(s, layers, T0, T1, kbs[0], M, np) && ws &&
                     ws_bytes >= pbytes && ((uintptr_t)ws & 15) == 0;
    const int64_t zb = pre ? pbytes : 0;
    bool compact = pool && chain_use_compact(s) && ws && ((uintptr_t)ws & 15) == 0 &&
                   ws_bytes >= zb + compact_table_bytes(s);
    // With the layer-0 pre-pass (wide first layers: SSG / pose sa2) compaction paid only once
    // the centroid term u came from a global table instead of being computed
    // per workgroup for its 16 groups (setup 8.8 us of a 49 us workgroup life,
    // tools/debug/chain_stamps.py): SSG sa2 115 us vs 130 us computing the padding rows.
    float *utab = pre ? reinterpret_cast<float *>(reinterpret_cast<char *>(ws) + prepass_z_bytes(s, layers[0]))
                      : nullptr;
    if (pre) {
        const int rc = launch_layer0_prepass(s, layers[0], ws, st);
        if (rc != PN2_OK) return rc;
        if (!compact) {  // with compaction the scan launch's extra workgroups compute u
            const int64_t G = s.B * s.S, cout0 = layers[0].cout;
            hipLaunchKernelGGL(u_table_kernel, dim3((unsigned)((G * cout0 + 255) / 256)), dim3(256), 0, st,
                               layers[0].wt, (int)(layers[0].cin - s.C), (int)cout0, s.ctr, (int)s.C, G,
                               utab);  // the fp32 image's rows are [features | xyz]
            PN2_LAUNCH_CHECK("u_table_kernel");
        }
        KB0M = -1;
    }
    // the fp32-accurate chains run split fp16 (3 MFMAs per product, split_bf16.h) where a whole
    // layer-0 input is in registers or pre-transformed (the activation scale needs the wave's
    // whole input); tuning chain_f16 = 0 keeps split bf16 (6 MFMAs)
    // The activation scale is per wave (32 rows): a cloud's rows must start at a wave boundary
    // (compact launches: a workgroup per cloud; else S*K a multiple of 32), so a cloud's results
    // never depend on which other clouds share its batch.
    const bool f16_ok = compact || (s.S * K) % 32 == 0;
    const int npk = (np == 3 && tuning().chain_f16 && f16_ok && (KB0M == 1 || KB0M == -1)) ? 2 : np;
    const size_t stage_b = npk == 3 ? stage_bytes<3>() : npk == 2 ? stage_bytes<2>() : stage_bytes<1>();
    const int wpc = compact ? (int)compact_wpc(s) : 0;
    // Compact launches: the weight ring's depth against the LDS group pool.  With the full
    // 16-row pool a 3-stage ring cost a workgroup per CU (SSG sa2: 3 -> 2 live per CU, 114 ->
    // 130 us, although each workgroup lived 36 us instead of 45: tools/debug/chain_stamps.py).
    // An 8-row pool (groups past it merge through HBM atomics into rows the scan zeroed) keeps
    // 3 per CU with 3 stages: eager (each kernel alone) 117.8 vs 114.2 us, but in the pipeline,
    // where the chains share CUs with the heads and the scans, the deeper ring wins.  Defaults
    // (r03, interleaved A/B x4, SSG K = 100): tuning compact_pool = 16 (the full pool, one
    // workgroup per CU fewer at sa1: 5 -> 4) and compact_stages = 3 (the 3-stage ring with the
    // 8-row pool wherever it keeps the workgroups per CU, i.e. sa2): 132.2-133.2k vs
    // 119.5-129.7k clouds/s; MSG / POSE / STRESS within noise.  r05, split fp16 (rings a third
    // smaller): compact_stages = 2 -- the 3-stage sa2 instance spilled 16 B per lane (168-VGPR
    // cap at 3 waves per SIMD; PMC write 7.9 vs 5.4 MB per call), eager sa1 49.0 -> 46.0 us, sa2
    // 82.5 -> 81.6 us; pipelined SSG K = 20 166.3-167.2k -> 170.3-172.3k, K = 100 190.6-191.1k
    // -> 190.3-194.7k, MSG / POSE / STRESS +1-2 % (tools/pmc_ab.sh, tools/args_ab.sh).
    int cks = 2, cprow = kUnitsPerWG;
    if (compact) {
        const int64_t cL = layers[2].cout;
        const size_t bnb = (size_t)2 * 4 * (layers[0].cout + layers[1].cout + cL) + 32;
        const size_t sb = stage_b;
        const int occ_v = T1 >= 4 ? 3 : T1 == 3 ? 4 : 5;  // workgroups per CU the VGPRs allow
        auto wgs = [&](int ks, int prow) {
            return std::min<int64_t>(occ_v, (int64_t)(160 * 1024) / (int64_t)(prow * cL * 4 + bnb + ks * sb));
        };
        // an 8-row pool when it buys a workgroup per CU (SSG sa1 eager: 4 -> 5 per CU, 62.4 ->
        // 59.9 us; its many small groups past the 8th of a workgroup merge through HBM atomics)
        // -- unless tuning compact_pool sets the pool rows (default 16: in the pipeline the
        // full pool measured faster, see above)
        if (wgs(2, 8) > wgs(2, kUnitsPerWG)) cprow = 8;
        if (tuning().compact_pool > 0)
            cprow = (int)std::max<int64_t>(1, std::min<int64_t>(kUnitsPerWG, tuning().compact_pool));
        // the 3-stage ring where it keeps the workgroups per CU: with the whole pool when that
        // fits too (split-fp16 rings are a third smaller: SSG sa2 then needs no HBM merges),
        // else with the 8-row pool
        if (tuning().compact_stages == 3) {
            if (wgs(3, cprow) >= wgs(2, kUnitsPerWG)) cks = 3;
            else if (wgs(3, 8) >= wgs(2, kUnitsPerWG)) cks = 3, cprow = 8;
        }
    }
    int *cunits = nullptr;
    int2 *cdesc = nullptr;
    if (compact) {
        cunits = reinterpret_cast<int *>(reinterpret_cast<char *>(ws) + zb);
        cdesc = reinterpret_cast<int2 *>(cunits + s.B * wpc * kUnitsPerWG);
        const size_t slds = compact_scan_lds(s);
        // u's workgroups (pre-pass chains): ~4 outputs per thread
        const int64_t ut = utab ? s.B * s.S * layers[0].cout : 0;
        const unsigned nu = (unsigned)std::min<int64_t>(std::min<int64_t>(1024, s.B * s.S),
                                                        (ut + 4 * kScanThreads - 1) / (4 * kScanThreads));
        static const hipError_t attr = hipFuncSetAttribute(
            reinterpret_cast<const void *>(&compact_scan_kernel),
            hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
        (void)attr;
        hipLaunchKernelGGL(compact_scan_kernel, dim3((unsigned)s.B + nu), dim3(kScanThreads), slds, st,
                           s.cnt, (int)s.B, (int)s.S, (int)s.K, wpc, cunits, cdesc, out, ostride,
                           (int)layers[2].cout, cprow, layers[0].wt, (int)(layers[0].cin - s.C),
                           (int)layers[0].cout, s.ctr, (int)s.C, utab);
        PN2_LAUNCH_CHECK("compact_scan_kernel");
    }
    ChainArgs A;
    memset(&A, 0, sizeof(A));
    A.src = s;
    for (int l = 0; l < 3; ++l) {
        A.L[l].w = reinterpret_cast<const bf16x8 *>(layers[l].wt_split);
        A.L[l].alpha = layers[l].alpha;
        A.L[l].beta = layers[l].beta;
        A.L[l].kb = kbs[l];
        A.L[l].tiles = (int)(layers[l].cout / 32);
        if (npk == 2 && !(l == 0 && pre)) {  // (a pre-transformed layer 0 runs no MFMA here)
            A.L[l].w = split_f16_planes(layers[l].wt_split, layers[l].cout, kbs[l]);
            A.L[l].wscale = split_f16_inv_scale(layers[l].wt_split, layers[l].cout, kbs[l]);
        }
    }
    A.M = (int)M;
    A.K = (int)K;
    A.S = (int)s.S;
    A.C = (int)s.C;
    A.D = (int)s.D;
    A.out = out;
    A.ostride = ostride;
    A.vec_feat = (s.D > 0 && s.D % 4 == 0 && ((uintptr_t)s.feat & 15) == 0 && s.fn % 4 == 0 &&
                  s.fb % 4 == 0) ? 1 : 0;
    A.cunits = cunits;
    A.cdesc = cdesc;
    A.wpc = wpc;
    if (pre) {
        A.z = ws;
        A.u = utab;
    }
    const int64_t coutL = layers[2].cout;
    size_t lds = 0;
    if (compact) {
        A.pool_mode = 3;
        A.pool_rows = cprow;
        A.ks = cks;
        lds = (size_t)cprow * coutL * 4;
    } else if (K == 8 || K == 16 || K == 32) {
        A.pool_mode = 0;
    } else if (kChainRows % K == 0) {
        A.pool_mode = 1;
        lds = (size_t)(kChainRows / K) * coutL * 4;
    } else {
        A.pool_mode = 2;
    }
    if (lds > 32 * 1024 && !compact) A.pool_mode = 2, lds = 0;
    if (A.pool_mode == 2) {
        const int64_t G = M / K;
        hipError_t e = (ostride == coutL)
                           ? hipMemsetAsync(out, 0, (size_t)G * coutL * 4, st)
                           : hipMemset2DAsync(out, (size_t)ostride * 4, 0, (size_t)coutL * 4, (size_t)G, st);
        if (e != hipSuccess) return set_error(PN2_EHIP, "sa_chain: memset: %s", hipGetErrorString(e));
    }
    const unsigned grid = compact ? (unsigned)(s.B * wpc) : (unsigned)((M + kChainRows - 1) / kChainRows);
    // LDS: [pool][BN scale/shift][per-wave rings]
    A.lds_bn = (int)((lds + 15) / 16 * 16);
    const size_t bn_bytes = (size_t)2 * 4 * (layers[0].cout + layers[1].cout + coutL);
    A.lds_ring = (int)((A.lds_bn + bn_bytes + 15) / 16 * 16);
    lds = (size_t)A.lds_ring + (size_t)(compact ? cks : kStages) * stage_b;
    // the caller's FPS side job rides on this launch when the instance has it (KB0M == 1: the
    // xyz-only first layers, i.e. sa1) and it fits the chain's LDS
    unsigned lgrid = grid;
    if (s.fps_side && KB0M == 1 && tuning().fps_side && fps_side_block_args(*s.fps_side, lds, A.fps)) {
        A.fps_nb = (int)s.fps_side->B;
        A.fps_blocks = (A.fps_nb + 7) / 8 * 8;
        lgrid += (unsigned)A.fps_blocks;
    }
    int rc = PN2_EUNSUPPORTED;
#define PN2_CHAIN_GO(a, b, c)                                                             \
    if (T0 == a && T1 == b && KB0M == c)                                                  \
        rc = npk == 3 ? launch_chain_sig<a, b, c, 3>(A, lgrid, lds, st)                   \
           : npk == 2 ? launch_chain_sig<a, b, c, 2>(A, lgrid, lds, st)                   \
                      : launch_chain_sig<a, b, c, 1>(A, lgrid, lds, st);
    PN2_CHAIN_SIGS(PN2_CHAIN_GO)
#undef PN2_CHAIN_GO
    if (rc == PN2_OK) {
        g_last_planes = npk;
        if (A.fps_blocks) fps_side_taken() = true;
    }
    return rc == PN2_OK ? 1 : rc;
}

}  // namespace pn2

int pn2::chain_last_planes() { return pn2::g_last_planes; }
