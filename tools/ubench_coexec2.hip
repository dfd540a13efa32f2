// Co-execution of v_mfma_f32_16x16x32_f16 with fp32 VALU on gfx950, with the
// MFMAs pinned by inline asm (no compiler accumulator shuffles).
// One workgroup of 8 waves per CU (waves w and w+4 share a SIMD).
//   mode 0: waves 0-3 MFMA only            (MFMA reference)
//   mode 1: waves 4-7 VALU only            (VALU reference)
//   mode 2: waves 0-3 MFMA, waves 4-7 VALU (partner overlap)
//   mode 3: waves 0-3: each MFMA followed by NV independent VALU FMAs (same-wave fill)
//   mode 4: as mode 0 but the 4 MFMAs form one dependent chain (same accumulator)
//   mode 5: mode 4's dependent chain || VALU partner waves
//   mode 6: two interleaved chains (a0 a1 a0 a1) || VALU partner waves
//   mode 7: two interleaved chains alone
//   mode 8: two chains || partner doing v_exp_f32 (transcendental) instead of FMA
//   mode 9: partner v_exp_f32 only
//   mode 10: two chains + 2 ds_read_b128 per 3 MFMAs || partner FMA
//   mode 11: mode 10's MFMA+LDS wave alone
// build: hipcc -O3 --offload-arch=gfx950 tools/ubench_coexec2.hip -o tools/ubench_coexec2
#include <hip/hip_runtime.h>

#include <cstdio>

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef _Float16 h8 __attribute__((ext_vector_type(8)));

#define MFMA(acc) asm volatile("v_mfma_f32_16x16x32_f16 %0, %1, %2, %0" : "+v"(acc) : "v"(a8), "v"(b8))
#define FMA(x) asm volatile("v_fma_f32 %0, %0, %1, %2" : "+v"(x) : "v"(c1), "v"(c2))
#define EXP(x) asm volatile("v_exp_f32 %0, %0" : "+v"(x))
#define DSR(r, addr, off) asm volatile("ds_read_b128 %0, %1 offset:" #off : "=v"(r) : "v"(addr))

template <int MODE, int NV>
__global__ __launch_bounds__(512, 1) void k(float* out, int iters, float seed) {
    const int wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    f32x4 a0 = {}, a1 = {}, a2 = {}, a3 = {};
    h8 a8, b8;
    for (int i = 0; i < 8; ++i) {
        a8[i] = (_Float16)(seed + i);
        b8[i] = (_Float16)(seed - i);
    }
    float v0 = seed, v1 = seed + 1, v2 = seed + 2, v3 = seed + 3, v4 = seed + 4, v5 = seed + 5, v6 = seed + 6,
          v7 = seed + 7;
    const float c1 = 0.999f, c2 = 0.001f;
    const bool mf = (MODE == 0 || MODE == 2 || MODE == 3) && wid < 4;
    const bool va = (MODE == 1 || MODE == 2 || MODE == 5 || MODE == 6 || MODE == 10) && wid >= 4;
    if ((MODE == 8 || MODE == 9) && wid >= 4) {
        for (int it = 0; it < iters; ++it) {
            EXP(v0); EXP(v1); EXP(v2); EXP(v3); EXP(v4); EXP(v5); EXP(v6); EXP(v7);
        }
    }
    if (MODE == 8 && wid < 4) {
        for (int it = 0; it < iters; ++it) {
            MFMA(a0);
            MFMA(a1);
            MFMA(a0);
            MFMA(a1);
        }
    }
    if ((MODE == 10 || MODE == 11) && wid < 4) {
        extern __shared__ float4 sh[];
        const unsigned addr = (unsigned)(uintptr_t)(__attribute__((address_space(3))) float4*)(sh + (threadIdx.x & 63));
        f32x4 r0, r1;
        for (int it = 0; it < iters; ++it) {
            DSR(r0, addr, 0);
            MFMA(a0);
            DSR(r1, addr, 1024);
            MFMA(a1);
            MFMA(a0);
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
            MFMA(a1);
            a2 += r0;
            a3 += r1;
        }
    }
    if ((MODE == 6 || MODE == 7) && wid < 4) {
        for (int it = 0; it < iters; ++it) {
            MFMA(a0);
            MFMA(a1);
            MFMA(a0);
            MFMA(a1);
        }
    }
    if ((MODE == 4 || MODE == 5) && wid < 4) {
        for (int it = 0; it < iters; ++it) {
            MFMA(a0);
            MFMA(a0);
            MFMA(a0);
            MFMA(a0);
        }
    }
    if (mf) {
        for (int it = 0; it < iters; ++it) {
            MFMA(a0);
            if (MODE == 3) {
                if (NV > 0) FMA(v0);
                if (NV > 1) FMA(v1);
                if (NV > 2) FMA(v2);
                if (NV > 3) FMA(v3);
            }
            MFMA(a1);
            if (MODE == 3) {
                if (NV > 0) FMA(v4);
                if (NV > 1) FMA(v5);
                if (NV > 2) FMA(v6);
                if (NV > 3) FMA(v7);
            }
            MFMA(a2);
            if (MODE == 3) {
                if (NV > 0) FMA(v0);
                if (NV > 1) FMA(v1);
                if (NV > 2) FMA(v2);
                if (NV > 3) FMA(v3);
            }
            MFMA(a3);
            if (MODE == 3) {
                if (NV > 0) FMA(v4);
                if (NV > 1) FMA(v5);
                if (NV > 2) FMA(v6);
                if (NV > 3) FMA(v7);
            }
        }
    }
    if (va) {
        // 4 "MFMA slots" worth of VALU per iteration: 16 independent FMAs
        for (int it = 0; it < iters; ++it) {
            FMA(v0); FMA(v1); FMA(v2); FMA(v3); FMA(v4); FMA(v5); FMA(v6); FMA(v7);
            FMA(v0); FMA(v1); FMA(v2); FMA(v3); FMA(v4); FMA(v5); FMA(v6); FMA(v7);
        }
    }
    float s = a0[0] + a1[1] + a2[2] + a3[3] + v0 + v1 + v2 + v3 + v4 + v5 + v6 + v7;
    if (s == 12345.678f) out[threadIdx.x] = s;
}

template <int MODE, int NV>
float run(int iters) {
    float* out;
    (void)hipMalloc(&out, 4096);
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    hipLaunchKernelGGL((k<MODE, NV>), dim3(256), dim3(512), 8192, 0, out, iters, 1.0f);
    (void)hipEventRecord(e0);
    for (int r = 0; r < 5; ++r) hipLaunchKernelGGL((k<MODE, NV>), dim3(256), dim3(512), 8192, 0, out, iters, 1.0f);
    (void)hipEventRecord(e1);
    (void)hipEventSynchronize(e1);
    float ms;
    (void)hipEventElapsedTime(&ms, e0, e1);
    (void)hipFree(out);
    return ms / 5;
}

int main() {
    const int iters = 20000;
    // cycles per iteration (4 MFMAs and/or 16 FMAs) at 2.4 GHz
    auto cyc = [&](float ms) { return ms * 1e-3 * 2.4e9 / iters; };
    const float t0 = run<0, 0>(iters), t1 = run<1, 0>(iters), t2 = run<2, 0>(iters);
    printf("mode0 MFMA only (4 MFMA/iter)          %.1f cyc/iter\n", cyc(t0));
    printf("mode1 VALU only (16 FMA/iter)          %.1f cyc/iter\n", cyc(t1));
    printf("mode2 MFMA wave || VALU partner wave   %.1f cyc/iter\n", cyc(t2));
    printf("mode3 same wave, 1 FMA per MFMA        %.1f cyc/iter\n", cyc(run<3, 1>(iters)));
    printf("mode3 same wave, 2 FMA per MFMA        %.1f cyc/iter\n", cyc(run<3, 2>(iters)));
    printf("mode3 same wave, 4 FMA per MFMA        %.1f cyc/iter\n", cyc(run<3, 4>(iters)));
    printf("mode4 dependent MFMA chain only        %.1f cyc/iter\n", cyc(run<4, 0>(iters)));
    printf("mode5 dependent chain || VALU partner  %.1f cyc/iter\n", cyc(run<5, 0>(iters)));
    printf("mode7 two interleaved chains only      %.1f cyc/iter\n", cyc(run<7, 0>(iters)));
    printf("mode6 two chains || VALU partner       %.1f cyc/iter\n", cyc(run<6, 0>(iters)));
    printf("mode9 partner v_exp only (8 exp/iter)  %.1f cyc/iter\n", cyc(run<9, 0>(iters)));
    printf("mode8 two chains || v_exp partner      %.1f cyc/iter\n", cyc(run<8, 0>(iters)));
    printf("mode11 chains + ds_read_b128 alone     %.1f cyc/iter\n", cyc(run<11, 0>(iters)));
    printf("mode10 chains + ds_read || FMA partner %.1f cyc/iter\n", cyc(run<10, 0>(iters)));
    return 0;
}
