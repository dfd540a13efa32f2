// ubench_split_mix.hip -- check (tools only): the fp16 residual pair of
// nfk_fused_impl.h f16_residual_pair (v_fma_mix{lo,hi}_f16 inline asm) is bitwise
// (_Float16)(v - (float)(_Float16)v) for both halves, over activations in the
// kernels' range (|v| <= 2^14: tanh outputs x 2^14), subnormal-sized residuals,
// ties, +-0, and the layer-1 inputs' range (|v| < 2^15).
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>

#include "nfk_spline.h"
int nfk_set_error(const char*);
#include "nfk_fused_impl.h"

__device__ __forceinline__ uint32_t hash32(uint32_t v) {
    v ^= v >> 16; v *= 0x7feb352dU; v ^= v >> 15; v *= 0x846ca68bU; v ^= v >> 16;
    return v;
}

__global__ void k_check(int* bad, int iters) {
    const uint32_t g = blockIdx.x * blockDim.x + threadIdx.x;
    int nb = 0;
    for (int it = 0; it < iters; ++it) {
        const uint32_t r0 = hash32(g * 2654435761u + it * 97u), r1 = hash32(r0 + 1);
        // mix of magnitudes: uniform in +-2^14, tiny, and random bit patterns of finite floats
        float v0, v1;
        switch (it & 3) {
            case 0: v0 = ((int)(r0 >> 8) - (1 << 23)) * (16384.0f / 8388608.0f); v1 = ((int)(r1 >> 8) - (1 << 23)) * (16384.0f / 8388608.0f); break;
            case 1: v0 = ((int)(r0 >> 8) - (1 << 23)) * 1e-9f; v1 = ((int)(r1 >> 8) - (1 << 23)) * 3e-7f; break;
            case 2: v0 = __uint_as_float((r0 & 0x807FFFFFu) | (((r0 >> 23) % 30 + 100) << 23)); v1 = __uint_as_float((r1 & 0x807FFFFFu) | (((r1 >> 23) % 30 + 100) << 23)); break;
            default: v0 = (r0 & 1) ? 0.0f : -0.0f; v1 = (float)(int)(r1 % 65536) * 0.25f; break;
        }
        const _Float16 h0 = (_Float16)v0, h1 = (_Float16)v1;
        const uint32_t hp = (uint32_t)__builtin_bit_cast(uint16_t, h0) | ((uint32_t)__builtin_bit_cast(uint16_t, h1) << 16);
        const uint32_t got = nfk_fused::f16_residual_pair(v0, v1, hp);
        const _Float16 l0 = (_Float16)(v0 - (float)h0), l1 = (_Float16)(v1 - (float)h1);
        const uint32_t want = (uint32_t)__builtin_bit_cast(uint16_t, l0) | ((uint32_t)__builtin_bit_cast(uint16_t, l1) << 16);
        nb += got != want;
    }
    if (nb) atomicAdd(bad, nb);
}

int main() {
    int* bad;
    (void)hipMalloc(&bad, sizeof(int));
    (void)hipMemset(bad, 0, sizeof(int));
    const int blocks = 4096, iters = 256;
    hipLaunchKernelGGL(k_check, dim3(blocks), dim3(256), 0, 0, bad, iters);
    int h = -1;
    hipError_t e = hipMemcpy(&h, bad, sizeof(int), hipMemcpyDeviceToHost);
    printf("f16_residual_pair vs (_Float16)(v - (float)h): %d mismatching pairs of %lld%s\n", h,
           (long long)blocks * 256 * iters, e == hipSuccess ? "" : " (error)");
    return h == 0 && e == hipSuccess ? 0 : 1;
}
