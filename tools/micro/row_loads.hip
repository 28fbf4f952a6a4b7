// Microbenchmark: the dense layer's load stage in isolation (no MFMAs).  512 workgroups of 4
// waves (2 per CU, as sa3's 512 -> 1024 layer runs), each looping over "stages": issue one
// stage's loads, wait for them (vmcnt(0)), barrier.  Patterns per stage and wave:
//   rows  8 x 16-byte loads per lane, lane (r, h) reading row r at 32 k + 16 h (the A operand:
//         32 rows x 32 bytes per instruction), rows of 2 KB
//   lines 8 x 16-byte loads per lane, each instruction 1 KB contiguous (whole lines)
//   dma   6 x global_load_lds (1 KB per instruction, lane-linear), the weight copies
//   both  rows + dma (a full dense stage)
//   lnd   lines + dma (the same stage with the rows in fragment order)
// The source (8 MB of rows, 3 MB of "weights") stays L2/MALL-resident across the launches.
// Prints us per stage and GB/s per CU.   hipcc --offload-arch=gfx950 -O3 row_loads.hip
#include <hip/hip_runtime.h>
#include <cstdio>

typedef float f4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) void lds_void;

template <int MODE>  // 0 rows, 1 lines, 2 dma, 3 rows + dma, 4 lines + dma
__global__ __launch_bounds__(256) void k(const float *rows, const char *w, float *out, int stages) {
    __shared__ __attribute__((aligned(16))) char lds[2 * 24 * 1024];
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, r = lane & 31, h = lane >> 5;
    const int rb = (blockIdx.x >> 4) & 31;  // row block of 128 rows (32 row blocks x 16 col groups)
    const float *arow = rows + (size_t)(rb * 128 + wave * 32 + r) * 512 + 4 * h;
    const float *aline = rows + (size_t)(rb * 128 + wave * 32) * 512 + lane * 4;
    const char *wsrc = w + (size_t)(blockIdx.x & 15) * 192 * 1024 + wave * 1024 + lane * 16;
    f4 acc = {0.f, 0.f, 0.f, 0.f};
    for (int c = 0; c < stages; ++c) {
        const int s = c & 7;  // 8 stages of 64 floats per 512-float row
        f4 q[8];
        if (MODE == 0 || MODE == 3) {
#pragma unroll
            for (int j = 0; j < 8; ++j) q[j] = *reinterpret_cast<const f4 *>(arow + s * 64 + 8 * j);
        } else if (MODE == 1 || MODE == 4) {
#pragma unroll
            for (int j = 0; j < 8; ++j) q[j] = *reinterpret_cast<const f4 *>(aline + s * 64 * 32 + j * 256);
        }
        if (MODE >= 2) {
#pragma unroll
            for (int j = 0; j < 6; ++j)
                __builtin_amdgcn_global_load_lds(wsrc + (size_t)(s * 24 + j * 4) * 1024,
                                                 (lds_void *)(lds + (c & 1) * 24 * 1024 + (j * 4 + wave) * 1024), 16, 0, 0);
        }
        __builtin_amdgcn_s_waitcnt(0x0F70);
        __syncthreads();
        if (MODE != 2)
#pragma unroll
            for (int j = 0; j < 8; ++j) acc += q[j];
    }
    if (MODE >= 2) acc[0] += *reinterpret_cast<const float *>(lds + threadIdx.x * 4);
    out[blockIdx.x * 256 + threadIdx.x] = acc[0] + acc[1] + acc[2] + acc[3];
}

template <int MODE>
static void run(const char *name, const float *rows, const char *w, float *out, double bytes_stage_wg) {
    const int stages = 800;
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    for (int i = 0; i < 3; ++i) hipLaunchKernelGGL(k<MODE>, dim3(512), dim3(256), 0, 0, rows, w, out, stages);
    hipEventRecord(e0);
    const int reps = 10;
    for (int i = 0; i < reps; ++i) hipLaunchKernelGGL(k<MODE>, dim3(512), dim3(256), 0, 0, rows, w, out, stages);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms = 0.f;
    hipEventElapsedTime(&ms, e0, e1);
    const double us_stage = ms * 1e3 / reps / stages;
    printf("%-6s %6.3f us per stage  %7.1f GB/s per CU (2 workgroups)  %6.2f TB/s chip\n", name, us_stage,
           2 * bytes_stage_wg / (us_stage * 1e-6) / 1e9, 512 * bytes_stage_wg / (us_stage * 1e-6) / 1e12);
}

int main() {
    float *rows, *out;
    char *w;
    hipMalloc(&rows, (size_t)4096 * 512 * 4);
    hipMalloc(&w, (size_t)16 * 192 * 1024);
    hipMalloc(&out, (size_t)512 * 256 * 4);
    hipMemset(rows, 0, (size_t)4096 * 512 * 4);
    hipMemset(w, 0, (size_t)16 * 192 * 1024);
    run<0>("rows", rows, w, out, 32.0 * 1024);
    run<1>("lines", rows, w, out, 32.0 * 1024);
    run<2>("dma", rows, w, out, 24.0 * 1024);
    run<3>("both", rows, w, out, 56.0 * 1024);
    run<4>("lnd", rows, w, out, 56.0 * 1024);
    return 0;
}
