// ubench_mfma_dep.hip -- diagnostic (tools only): does a v_mfma_f32_16x16x32_f16
// read as SrcC what the same-shape MFMA wrote NACC instructions earlier, when
// NACC - 1 independent MFMAs sit between them?  Each wave runs STEPS rounds of
// acc[j] = mfma(A, B, acc[j]) for j = 0 .. NACC-1 (one dependent chain per
// accumulator, the chains interleaved round robin: dependency distance NACC),
// with A = B = all ones (every product step adds exactly 32 to every element),
// optionally NOPS wait states after each MFMA.  Any element that is not
// exactly 32 STEPS at the end lost a step: a stale SrcC read.
// Also the cross-shape case of nfk_fused_impl.h's tail step: a 16x16x16 f16
// MFMA reading what a 16x16x32 MFMA wrote one instruction earlier (TAIL = 1).
// Built by tools/gpu_r4m.sh; run as ./ubench_mfma_dep.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

typedef _Float16 h8 __attribute__((ext_vector_type(8)));
typedef _Float16 h4 __attribute__((ext_vector_type(4)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

template <int NACC, int NOPS, int TAIL>
__global__ __launch_bounds__(256) void k_dep(float* out, int steps, int* bad) {
    h8 a, b;
    for (int j = 0; j < 8; ++j) a[j] = b[j] = (_Float16)1.0f;
    h4 a4, b4;
    for (int j = 0; j < 4; ++j) a4[j] = b4[j] = (_Float16)1.0f;
    f32x4 acc[NACC];
    for (int j = 0; j < NACC; ++j) acc[j] = f32x4{0.0f, 0.0f, 0.0f, 0.0f};
    for (int s = 0; s < steps; ++s) {  // steps: a multiple of 8, rounds back to back
#pragma unroll
      for (int u = 0; u < 8; ++u, ++s) {
#pragma unroll
        for (int j = 0; j < NACC; ++j) {
            acc[j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(a, b, acc[j], 0, 0, 0);
            __builtin_amdgcn_sched_barrier(0);
            if constexpr (NOPS > 0) asm volatile("s_nop %0" ::"i"(NOPS - 1));
            __builtin_amdgcn_sched_barrier(0);
        }
        if constexpr (TAIL) {
            // 16x16x16 f16 on the chain 0 accumulator right after its 16x16x32 (adds 16)
            acc[NACC - 1] = __builtin_amdgcn_mfma_f32_16x16x16f16(a4, b4, acc[NACC - 1], 0, 0, 0);
            __builtin_amdgcn_sched_barrier(0);
        }
      }
      --s;
    }
    const float want = 32.0f * steps;
    int nb = 0;
    for (int j = 0; j < NACC; ++j) {
        const float w = want + ((TAIL && j == NACC - 1) ? 16.0f * steps : 0.0f);
        for (int r = 0; r < 4; ++r) nb += acc[j][r] != w ? 1 : 0;
    }
    if (nb) atomicAdd(bad, nb);
    out[blockIdx.x * blockDim.x + threadIdx.x] = acc[0][0];
}

template <int NACC, int NOPS, int TAIL>
static void run(int waves_per_simd, int steps, int reps) {
    const int cus = 256, blocks = cus * waves_per_simd;  // 4 waves per block, one per SIMD
    float* out;
    int* bad;
    (void)hipMalloc(&out, sizeof(float) * blocks * 256);
    (void)hipMalloc(&bad, sizeof(int));
    long long total = 0;
    for (int r = 0; r < reps; ++r) {
        (void)hipMemset(bad, 0, sizeof(int));
        hipLaunchKernelGGL((k_dep<NACC, NOPS, TAIL>), dim3(blocks), dim3(256), 0, 0, out, steps, bad);
        int h = 0;
        (void)hipMemcpy(&h, bad, sizeof(int), hipMemcpyDeviceToHost);
        total += h;
    }
    const long long elems = (long long)reps * blocks * 256 * NACC * 4;
    printf("NACC %d NOPS %2d TAIL %d waves/SIMD %d: stale elements %lld of %lld\n", NACC, NOPS, TAIL,
           waves_per_simd, total, elems);
    fflush(stdout);
    (void)hipFree(out);
    (void)hipFree(bad);
}

int main() {
    const int steps = 64, reps = 20;
    for (int w = 1; w <= 2; ++w) {
        run<1, 0, 0>(w, steps, reps);
        run<2, 0, 0>(w, steps, reps);
        run<3, 0, 0>(w, steps, reps);
        run<4, 0, 0>(w, steps, reps);
        run<2, 4, 0>(w, steps, reps);
        run<2, 8, 0>(w, steps, reps);
        run<2, 0, 1>(w, steps, reps);
        run<4, 0, 1>(w, steps, reps);
    }
    return 0;
}
