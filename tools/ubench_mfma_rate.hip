// Issue rate of the f16 MFMA shapes on gfx950: back-to-back MFMAs, one wave
// per SIMD, 4 independent accumulators.
// build: hipcc -O3 --offload-arch=gfx950 tools/ubench_mfma_rate.hip -o tools/ubench_mfma_rate
#include <hip/hip_runtime.h>

#include <cstdio>

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef _Float16 h8 __attribute__((ext_vector_type(8)));
typedef _Float16 h4 __attribute__((ext_vector_type(4)));

template <int SHAPE>
__global__ __launch_bounds__(256, 1) void k(float* out, int iters, float seed) {
    f32x4 acc[4] = {};
    h8 a8, b8;
    h4 a4, b4;
    for (int i = 0; i < 8; ++i) {
        a8[i] = (_Float16)(seed + threadIdx.x + i);
        b8[i] = (_Float16)(seed - i);
    }
    for (int i = 0; i < 4; ++i) {
        a4[i] = a8[i];
        b4[i] = b8[i];
    }
    for (int it = 0; it < iters; ++it) {
        // inline asm pins the accumulators (no compiler register shuffles)
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            if constexpr (SHAPE == 32)
                asm volatile("v_mfma_f32_16x16x32_f16 %0, %1, %2, %0" : "+v"(acc[j]) : "v"(a8), "v"(b8));
            else
                asm volatile("v_mfma_f32_16x16x16_f16 %0, %1, %2, %0" : "+v"(acc[j]) : "v"(a4), "v"(b4));
        }
    }
    float s = 0.f;
    for (int j = 0; j < 4; ++j) s += acc[j][0] + acc[j][1] + acc[j][2] + acc[j][3];
    if (s == 12345.678f) out[threadIdx.x] = s;
}

template <int SHAPE>
float run(int iters) {
    float* out;
    (void)hipMalloc(&out, 4096);
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    hipLaunchKernelGGL(k<SHAPE>, dim3(256), dim3(256), 0, 0, out, iters, 1.0f);
    (void)hipEventRecord(e0);
    for (int r = 0; r < 5; ++r) hipLaunchKernelGGL(k<SHAPE>, dim3(256), dim3(256), 0, 0, out, iters, 1.0f);
    (void)hipEventRecord(e1);
    (void)hipEventSynchronize(e1);
    float ms;
    (void)hipEventElapsedTime(&ms, e0, e1);
    (void)hipFree(out);
    return ms / 5;
}

int main() {
    const int iters = 20000;
    const float t32 = run<32>(iters), t16 = run<16>(iters);
    auto cyc = [&](float ms) { return ms * 1e-3 * 2.4e9 / (iters * 4.0); };
    printf("v_mfma_f32_16x16x32_f16  %.3f ms  %.1f cyc/MFMA (at 2.4 GHz)\n", t32, cyc(t32));
    printf("v_mfma_f32_16x16x16_f16  %.3f ms  %.1f cyc/MFMA (at 2.4 GHz)\n", t16, cyc(t16));
    return 0;
}
