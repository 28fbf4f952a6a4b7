// Microbenchmark of the LDS-staged dense kernel's stage body (sa_dense.hip dense_lds_kernel):
// per wave and iteration 2 k-blocks x 2 column tiles x 6 split-bf16 MFMAs (24
// v_mfma_f32_32x32x16_bf16), optionally with the stage's 16 ds_read_b128 fragment reads, the
// A split (16 floats -> 3 bf16 planes) and an s_barrier.  Cycles per iteration (s_memtime) at
// 1 and 2 waves per SIMD: hipcc -O3 --offload-arch=gfx950 tools/micro/mfma_split.hip -o mfma_split
#include <hip/hip_runtime.h>
#include <cstdio>

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float floatx16 __attribute__((ext_vector_type(16)));
typedef float floatx4 __attribute__((ext_vector_type(4)));
#define MF __builtin_amdgcn_mfma_f32_32x32x16_bf16

struct Split {
    bf16x8 h, m, l;
};
__device__ __forceinline__ Split split8(const float (&x)[8]) {
    Split s;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
        const __bf16 a = (__bf16)x[j];
        const float r = x[j] - (float)a;
        const __bf16 b = (__bf16)r;
        s.h[j] = a;
        s.m[j] = b;
        s.l[j] = (__bf16)(r - (float)b);
    }
    return s;
}
__device__ __forceinline__ floatx16 mma6(const Split &x, const Split &w, floatx16 acc) {
    acc = MF(x.h, w.h, acc, 0, 0, 0);
    acc = MF(x.m, w.h, acc, 0, 0, 0);
    acc = MF(x.l, w.h, acc, 0, 0, 0);
    acc = MF(x.h, w.m, acc, 0, 0, 0);
    acc = MF(x.m, w.m, acc, 0, 0, 0);
    acc = MF(x.h, w.l, acc, 0, 0, 0);
    return acc;
}

// MODE 0: MFMAs only (operands fixed in registers); 1: + LDS reads and split per iteration;
// 2: + s_barrier per iteration
template <int MODE>
__global__ __launch_bounds__(1024) void k(const float *in, floatx16 *out, long long *cyc, int iters) {
    __shared__ __attribute__((aligned(16))) char lds[65536];
    const int lane = threadIdx.x & 63;
    for (int i = threadIdx.x; i < 65536 / 4; i += blockDim.x) reinterpret_cast<float *>(lds)[i] = in[i & 1023];
    __syncthreads();
    float x0[8];
    for (int j = 0; j < 8; ++j) x0[j] = in[lane * 8 + j];
    Split xs0 = split8(x0), xs1 = xs0;
    Split w[2][2];
    for (int a = 0; a < 2; ++a)
        for (int b = 0; b < 2; ++b) w[a][b] = split8(x0);
    floatx16 acc[2];
    for (int c = 0; c < 2; ++c)
        for (int q = 0; q < 16; ++q) acc[c][q] = 0.f;
    const long long t0 = __builtin_amdgcn_s_memtime();
    for (int it = 0; it < iters; ++it) {
        if (MODE >= 2) __builtin_amdgcn_s_barrier();
        if (MODE >= 1) {
            const char *base = lds + ((it & 7) * 8192) + lane * 16;
            floatx4 a[4];
            for (int j = 0; j < 4; ++j) a[j] = *reinterpret_cast<const floatx4 *>(base + j * 1024);
            for (int kb = 0; kb < 2; ++kb)
                for (int t = 0; t < 2; ++t) {
                    const bf16x8 *q = reinterpret_cast<const bf16x8 *>(base + 4096 + (kb * 2 + t) * 3072);
                    w[kb][t].h = q[0];
                    w[kb][t].m = q[64];
                    w[kb][t].l = q[128];
                }
            float xa[8], xb[8];
            for (int j = 0; j < 4; ++j) xa[j] = a[0][j], xa[4 + j] = a[1][j], xb[j] = a[2][j], xb[4 + j] = a[3][j];
            xs0 = split8(xa);
            xs1 = split8(xb);
        }
        for (int t = 0; t < 2; ++t) acc[t] = mma6(xs0, w[0][t], acc[t]);
        for (int t = 0; t < 2; ++t) acc[t] = mma6(xs1, w[1][t], acc[t]);
    }
    const long long t1 = __builtin_amdgcn_s_memtime();
    out[blockIdx.x * blockDim.x + threadIdx.x] = acc[0] + acc[1];
    if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
}

int main() {
    float *in;
    floatx16 *out;
    long long *cyc;
    hipMalloc(&in, 4096 * 4);
    float hin[4096];
    for (int i = 0; i < 4096; ++i) hin[i] = (float)((i * 2654435761u) % 1000) / 997.f - 0.5f;
    hipMemcpy(in, hin, sizeof(hin), hipMemcpyHostToDevice);
    hipMalloc(&out, (size_t)256 * 1024 * 64);  // up to 1024 threads per block, one floatx16 each
    hipMalloc(&cyc, 256 * 8);
    const int iters = 4000;
    long long h[256];
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    for (int mode = 0; mode < 3; ++mode)
        for (int waves = 4; waves <= (mode == 0 ? 16 : 8); waves += 4) {
            float ms = 0.f;
            for (int rep = 0; rep < 2; ++rep) {
                hipEventRecord(e0, 0);
                if (mode == 0) hipLaunchKernelGGL(k<0>, dim3(256), dim3(64 * waves), 0, 0, in, out, cyc, iters);
                if (mode == 1) hipLaunchKernelGGL(k<1>, dim3(256), dim3(64 * waves), 0, 0, in, out, cyc, iters);
                if (mode == 2) hipLaunchKernelGGL(k<2>, dim3(256), dim3(64 * waves), 0, 0, in, out, cyc, iters);
                hipEventRecord(e1, 0);
                hipDeviceSynchronize();
                hipEventElapsedTime(&ms, e0, e1);
            }
            hipMemcpy(h, cyc, sizeof(h), hipMemcpyDeviceToHost);
            double s = 0;
            for (int i = 0; i < 256; ++i) s += h[i];
            const double per_it = s / 256 / iters;
            // MFMA cycles per SIMD and iteration: waves/4 waves x 24 MFMAs x 32 cycles
            const double flops = 256.0 * waves * iters * 24 * 32768.0;
            printf("mode %d waves/SIMD %d: %.0f cycles/iteration, 32-cycle floor %d (%.0f%%); %.3f ms = %.0f TFLOP/s bf16\n",
                   mode, waves / 4, per_it, waves / 4 * 24 * 32, 100.0 * waves / 4 * 24 * 32 / per_it, ms,
                   flops / (ms * 1e-3) / 1e12);
        }
    return 0;
}
