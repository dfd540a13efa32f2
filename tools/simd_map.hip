// Which SIMD does each wave of an 8-wave workgroup run on?  (HW_ID register)
// build: hipcc -O3 --offload-arch=gfx950 tools/simd_map.hip -o tools/simd_map
#include <hip/hip_runtime.h>

#include <cstdio>

__global__ __launch_bounds__(512, 1) void k(unsigned* out) {
    unsigned id;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(id));
    if ((threadIdx.x & 63) == 0) out[blockIdx.x * 8 + (threadIdx.x >> 6)] = id;
}

int main() {
    unsigned* d;
    (void)hipMalloc(&d, 64 * 8 * 4);
    hipLaunchKernelGGL(k, dim3(64), dim3(512), 0, 0, d);
    unsigned h[64 * 8];
    (void)hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost);
    for (int b = 0; b < 6; ++b) {
        printf("block %d: ", b);
        for (int w = 0; w < 8; ++w) {
            const unsigned id = h[b * 8 + w];
            // HW_ID: WAVE_ID[3:0] SIMD_ID[5:4] PIPE_ID[7:6] CU_ID[11:8] SH_ID[12] SE_ID[15:13]
            printf("w%d:simd%u(cu%u) ", w, (id >> 4) & 3, (id >> 8) & 15);
        }
        printf("\n");
    }
    return 0;
}
