// Microbenchmark: do fp32 MFMA (v_mfma_f32_16x16x4_f32) and VALU work from two
// different waves on the same SIMD execute concurrently on gfx950?
// 256 workgroups x 8 waves (two per SIMD: wave w and w+4 share a SIMD).
// mode 0: waves 0-3 MFMA only      mode 1: waves 4-7 VALU only
// mode 2: both (partners)          mode 3: every wave does MFMA then VALU
// mode 4: every wave interleaves MFMA and VALU in one stream
// build: hipcc -O3 --offload-arch=gfx950 tools/ubench_coexec.hip -o /tmp/ubench
#include <hip/hip_runtime.h>

#include <cstdio>

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));

// BF=true: the MFMA is v_mfma_f32_16x16x32_bf16 (16x the flops of the f32 one)
template <bool BF>
__device__ __forceinline__ f32x4 mm(float a, float b, bf16x8 ab, bf16x8 bb, f32x4 c) {
    if constexpr (BF)
        return __builtin_amdgcn_mfma_f32_16x16x32_bf16(ab, bb, c, 0, 0, 0);
    else
        return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
}

template <int MODE, bool BF>
__global__ __launch_bounds__(512, 1) void k(float* out, int iters, float seed) {
    const int wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const bool mfma_wave = (MODE == 0 || MODE == 2) ? wid < 4 : (MODE == 1 ? false : true);
    const bool valu_wave = (MODE == 1 || MODE == 2) ? wid >= 4 : (MODE == 0 ? false : true);
    f32x4 acc[4] = {};
    float v[8];
    for (int i = 0; i < 8; ++i) v[i] = seed + threadIdx.x * 1e-3f + i;
    const float a = seed + threadIdx.x, b = seed * 0.5f;
    bf16x8 ab, bb;
    for (int i = 0; i < 8; ++i) {
        ab[i] = (__bf16)(a + i);
        bb[i] = (__bf16)(b - i);
    }
    if (MODE == 4) {
        for (int it = 0; it < iters; ++it) {
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                acc[j] = mm<BF>(a, b, ab, bb, acc[j]);
#pragma unroll
                for (int i = 0; i < 8; ++i) v[i] = fmaf(v[i], 0.999f, 0.001f);
            }
        }
    } else {
        if (mfma_wave) {
            for (int it = 0; it < iters; ++it) {
#pragma unroll
                for (int j = 0; j < 4; ++j) acc[j] = mm<BF>(a, b, ab, bb, acc[j]);
            }
        }
        if (valu_wave) {
            for (int it = 0; it < iters; ++it) {
#pragma unroll
                for (int j = 0; j < 4; ++j)
#pragma unroll
                    for (int i = 0; i < 8; ++i) v[i] = fmaf(v[i], 0.999f, 0.001f);
            }
        }
    }
    float s = 0.f;
    for (int j = 0; j < 4; ++j) s += acc[j][0] + acc[j][1] + acc[j][2] + acc[j][3];
    for (int i = 0; i < 8; ++i) s += v[i];
    if (s == 12345.678f) out[threadIdx.x] = s;
}

template <int MODE, bool BF>
float run(int iters) {
    float* out;
    hipMalloc(&out, 4096);
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    hipLaunchKernelGGL((k<MODE, BF>), dim3(256), dim3(512), 0, 0, out, iters, 1.0f);
    hipEventRecord(e0);
    for (int r = 0; r < 5; ++r) hipLaunchKernelGGL((k<MODE, BF>), dim3(256), dim3(512), 0, 0, out, iters, 1.0f);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms;
    hipEventElapsedTime(&ms, e0, e1);
    hipFree(out);
    return ms / 5;
}

template <bool BF>
void suite(const char* tag) {
    const int iters = 20000;
    const float t0 = run<0, BF>(iters), t1 = run<1, BF>(iters), t2 = run<2, BF>(iters),
                t3 = run<3, BF>(iters), t4 = run<4, BF>(iters);
    // cycles per wave per iteration at 2.4 GHz: an iteration = 4 MFMA and/or 32 FMA
    auto cyc = [&](float ms) { return ms * 1e-3 * 2.4e9 / iters; };
    printf("[%s] mode0 MFMA waves only        %.3f ms  %.1f cyc/iter\n", tag, t0, cyc(t0));
    printf("[%s] mode1 VALU waves only        %.3f ms  %.1f cyc/iter\n", tag, t1, cyc(t1));
    printf("[%s] mode2 MFMA || VALU partners  %.3f ms  %.1f cyc/iter\n", tag, t2, cyc(t2));
    printf("[%s] mode3 all waves MFMA;VALU    %.3f ms  %.1f cyc/iter\n", tag, t3, cyc(t3));
    printf("[%s] mode4 all waves interleaved  %.3f ms  %.1f cyc/iter\n", tag, t4, cyc(t4));
}

int main() {
    suite<false>("f32 16x16x4 ");
    suite<true>("bf16 16x16x32");
    return 0;
}
