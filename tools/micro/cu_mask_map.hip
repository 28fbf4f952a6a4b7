// Which CUs does a hipExtStreamCreateWithCUMask stream really use?  A 4096-workgroup kernel on
// the masked stream records every (XCC, SE, SH, CU) its workgroups ran on; printed per mask:
// distinct CUs used, per XCC.  Masks: the ones pn2.pipeline builds (GEO CUs spread with stride
// ncu/GEO, and the complement) plus contiguous bit ranges.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstring>
#include <vector>

__global__ void where(unsigned *bitmap) {
    if (threadIdx.x == 0) {
        const unsigned xcc = __builtin_amdgcn_s_getreg((20) | (0 << 6) | (31 << 11)) & 0xF;
        const unsigned hw = __builtin_amdgcn_s_getreg((4) | (0 << 6) | (31 << 11));
        const unsigned se = (hw >> 13) & 7, sh = (hw >> 12) & 1, cu = (hw >> 8) & 15;
        const unsigned idx = ((xcc * 8 + se) * 2 + sh) * 16 + cu;
        atomicOr(&bitmap[idx / 32], 1u << (idx % 32));
        // keep the CU busy briefly so the dispatcher spreads the workgroups
        for (int i = 0; i < 2000; ++i) __builtin_amdgcn_s_sleep(1);
    }
}

static void run(const char *name, const std::vector<int> &bits, int ncu, unsigned *d) {
    std::vector<unsigned> mask((ncu + 31) / 32, 0u);
    for (int b : bits) mask[b / 32] |= 1u << (b % 32);
    hipStream_t s;
    if (hipExtStreamCreateWithCUMask(&s, (uint32_t)mask.size(), mask.data()) != hipSuccess) {
        printf("%s: create failed\n", name);
        return;
    }
    hipMemsetAsync(d, 0, 2048 / 8, s);
    hipLaunchKernelGGL(where, dim3(4096), dim3(64), 0, s, d);
    unsigned h[64];
    hipStreamSynchronize(s);
    hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost);
    int total = 0, per[8] = {0};
    for (int i = 0; i < 2048; ++i)
        if (h[i / 32] >> (i % 32) & 1) { ++total; ++per[i / 256]; }
    printf("%-26s bits %3zu -> CUs used %3d  per XCC:", name, bits.size(), total);
    for (int x = 0; x < 8; ++x) printf(" %2d", per[x]);
    printf("\n");
    hipStreamDestroy(s);
}

int main() {
    int ncu = 0;
    hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, 0);
    unsigned *d;
    hipMalloc(&d, 2048 / 8);
    printf("ncu %d\n", ncu);
    std::vector<int> all;
    for (int c = 0; c < ncu; ++c) all.push_back(c);
    run("all", all, ncu, d);
    for (int g : {8, 16, 32, 64}) {
        std::vector<int> geo, rest;
        const double stride = (double)ncu / g;
        std::vector<char> in(ncu, 0);
        for (int i = 0; i < g; ++i) in[(int)(i * stride)] = 1;
        for (int c = 0; c < ncu; ++c) (in[c] ? geo : rest).push_back(c);
        char n1[64], n2[64];
        snprintf(n1, 64, "spread %d", g);
        snprintf(n2, 64, "spread %d complement", g);
        run(n1, geo, ncu, d);
        run(n2, rest, ncu, d);
        std::vector<int> blk, blkc;
        for (int c = 0; c < ncu; ++c) (c < g ? blk : blkc).push_back(c);
        snprintf(n1, 64, "block [0,%d)", g);
        snprintf(n2, 64, "block [%d,%d)", g, ncu);
        run(n1, blk, ncu, d);
        run(n2, blkc, ncu, d);
    }
    for (int b : {0, 1, 7, 8, 31, 32, 33, 255}) {
        char n[64];
        snprintf(n, 64, "bit %d", b);
        run(n, std::vector<int>{b}, ncu, d);
    }
    return 0;
}
