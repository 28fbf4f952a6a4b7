// Microbenchmark: cycles per v_mfma_f32_32x32x16_bf16 for one dependent accumulator chain vs
// two interleaved chains, one wave per SIMD (grid = 4 waves per CU x 256 CUs).
#include <hip/hip_runtime.h>
#include <cstdio>
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float floatx16 __attribute__((ext_vector_type(16)));
template <int CHAINS>
__global__ __launch_bounds__(256) void k(const bf16x8 *in, floatx16 *out, long long *cyc, int iters) {
    bf16x8 a = in[threadIdx.x & 63], b = in[64 + (threadIdx.x & 63)];
    floatx16 acc[CHAINS];
    for (int c = 0; c < CHAINS; ++c) for (int q = 0; q < 16; ++q) acc[c][q] = 0.f;
    long long t0 = clock64();
    for (int i = 0; i < iters; ++i) {
#pragma unroll
        for (int s = 0; s < 12 / CHAINS; ++s)
#pragma unroll
            for (int c = 0; c < CHAINS; ++c) acc[c] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, acc[c], 0, 0, 0);
    }
    long long t1 = clock64();
    floatx16 r = acc[0];
    for (int c = 1; c < CHAINS; ++c) r += acc[c];
    out[blockIdx.x * 256 + threadIdx.x] = r;
    if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
}
int main() {
    bf16x8 *in; floatx16 *out; long long *cyc;
    hipMalloc(&in, 128 * 16); hipMemset(in, 0, 128 * 16);
    hipMalloc(&out, 256 * 256 * 64); hipMalloc(&cyc, 256 * 8);
    const int iters = 2000;
    long long h[256];
    for (int v = 0; v < 2; ++v) {
        for (int rep = 0; rep < 2; ++rep) {
            if (v == 0) hipLaunchKernelGGL(k<1>, dim3(256), dim3(256), 0, 0, in, out, cyc, iters);
            else hipLaunchKernelGGL(k<2>, dim3(256), dim3(256), 0, 0, in, out, cyc, iters);
            hipDeviceSynchronize();
        }
        hipMemcpy(h, cyc, sizeof(h), hipMemcpyDeviceToHost);
        double s = 0; for (int i = 0; i < 256; ++i) s += h[i];
        printf("chains=%d cycles/mfma=%.2f (clock64 units)\n", v + 1, s / 256 / (iters * 12.0));
    }
    return 0;
}
