// Which XCD / shader engine / CU does bit i of a hipExtStreamCreateWithCUMask mask select?
// One single-bit stream per CU; a one-wave kernel records HW_REG_XCC_ID and HW_REG_HW_ID.
#include <hip/hip_runtime.h>
#include <cstdio>
__global__ void where(unsigned *out) {
    if (threadIdx.x == 0) {
        out[0] = __builtin_amdgcn_s_getreg((20) | (0 << 6) | (31 << 11));  // HW_REG_XCC_ID
        out[1] = __builtin_amdgcn_s_getreg((4) | (0 << 6) | (31 << 11));   // HW_REG_HW_ID
    }
}
int main() {
    int ncu = 0;
    hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, 0);
    unsigned *d;
    hipMalloc(&d, 8);
    printf("ncu %d\n", ncu);
    for (int c = 0; c < ncu; ++c) {
        unsigned mask[16] = {0};
        mask[c / 32] = 1u << (c % 32);
        hipStream_t s;
        if (hipExtStreamCreateWithCUMask(&s, (ncu + 31) / 32, mask) != hipSuccess) { printf("bit %d: create failed\n", c); continue; }
        hipLaunchKernelGGL(where, dim3(1), dim3(64), 0, s, d);
        unsigned h[2] = {0, 0};
        hipStreamSynchronize(s);
        hipMemcpy(h, d, 8, hipMemcpyDeviceToHost);
        // gfx9 HW_ID: wave[3:0] simd[5:4] pipe[7:6] cu[11:8] sh[12] se[15:13] tg[19:16] vm[23:20] queue[26:24] state[29:27] me[31:30]
        printf("bit %3d xcc %u se %u sh %u cu %u\n", c, h[0] & 0xF, (h[1] >> 13) & 7, (h[1] >> 12) & 1, (h[1] >> 8) & 15);
        hipStreamDestroy(s);
    }
    return 0;
}
