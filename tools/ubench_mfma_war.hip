// ubench_mfma_war.hip -- diagnostic (tools only): when does v_mfma_f32_16x16x32_f16
// read its A / B operands?  One asm block per step: fill v[40:47] with fp16
// ones (A = v[40:43], B = v[44:47]), issue the MFMA (acc += 32 per element),
// then after N wait states overwrite one source register with fp16 twos -- the
// write-after-read the compiler emits when it reuses an MFMA source register
// right after the MFMA (seen in the wide fused NSF_AR's ISA: a v_accvgpr_read
// into the MFMA's SrcA register one instruction later).  If the MFMA had not
// read that register yet, the step adds more than 32: counted as a late read.
// Accumulator in AGPRs ("+a") or VGPRs ("+v").  Run: ./ubench_mfma_war
#include <hip/hip_runtime.h>

#include <cstdio>

typedef float f32x4 __attribute__((ext_vector_type(4)));

#define WAR_KERNEL(NAME, NOPTXT, REG, CONS)                                                            \
    __global__ __launch_bounds__(256) void NAME(int steps, int* bad) {                                 \
        const unsigned ones = 0x3C003C00u, twos = 0x40004000u;                                         \
        f32x4 acc = {0.0f, 0.0f, 0.0f, 0.0f};                                                          \
        for (int s = 0; s < steps; ++s) {                                                              \
            asm volatile(                                                                              \
                "v_mov_b32 v40, %1\n\tv_mov_b32 v41, %1\n\tv_mov_b32 v42, %1\n\tv_mov_b32 v43, %1\n\t" \
                "v_mov_b32 v44, %1\n\tv_mov_b32 v45, %1\n\tv_mov_b32 v46, %1\n\tv_mov_b32 v47, %1\n\t" \
                "s_nop 4\n\t"                                                                          \
                "v_mfma_f32_16x16x32_f16 %0, v[40:43], v[44:47], %0\n\t" NOPTXT                        \
                "v_mov_b32 " REG ", %2\n\t"                                                            \
                "s_nop 7\n\ts_nop 7\n\ts_nop 7\n\ts_nop 7"                                             \
                : CONS(acc)                                                                            \
                : "v"(ones), "v"(twos)                                                                 \
                : "v40", "v41", "v42", "v43", "v44", "v45", "v46", "v47");                             \
        }                                                                                              \
        int nb = 0;                                                                                    \
        for (int r = 0; r < 4; ++r) nb += acc[r] != 32.0f * steps ? 1 : 0;                             \
        if (nb) atomicAdd(bad, nb);                                                                    \
    }

#define LIST(X)                                       \
    X(k_a3_n0_agpr, "", "v43", "+a")                  \
    X(k_a3_n1_agpr, "s_nop 0\n\t", "v43", "+a")       \
    X(k_a3_n2_agpr, "s_nop 1\n\t", "v43", "+a")       \
    X(k_a3_n4_agpr, "s_nop 3\n\t", "v43", "+a")       \
    X(k_a3_n8_agpr, "s_nop 7\n\t", "v43", "+a")       \
    X(k_a0_n0_agpr, "", "v40", "+a")                  \
    X(k_b3_n0_agpr, "", "v47", "+a")                  \
    X(k_b0_n0_agpr, "", "v44", "+a")                  \
    X(k_a3_n0_vgpr, "", "v43", "+v")                  \
    X(k_b3_n0_vgpr, "", "v47", "+v")                  \
    X(k_a3_n2_vgpr, "s_nop 1\n\t", "v43", "+v")

LIST(WAR_KERNEL)

static void run(const char* name, void (*k)(int, int*), int waves_per_simd) {
    const int blocks = 256 * waves_per_simd, steps = 256, reps = 10;
    int* bad;
    (void)hipMalloc(&bad, sizeof(int));
    long long total = 0;
    for (int r = 0; r < reps; ++r) {
        (void)hipMemset(bad, 0, sizeof(int));
        hipLaunchKernelGGL(k, dim3(blocks), dim3(256), 0, 0, steps, bad);
        int h = 0;
        (void)hipMemcpy(&h, bad, sizeof(int), hipMemcpyDeviceToHost);
        total += h;
    }
    printf("%-14s waves/SIMD %d: wrong elements %lld of %lld\n", name, waves_per_simd, total,
           (long long)reps * blocks * 256 * 4);
    fflush(stdout);
    (void)hipFree(bad);
}

int main() {
#define RUN(NAME, A, B, C) run(#NAME, NAME, w);
    for (int w = 1; w <= 2; ++w) { LIST(RUN) }
    return 0;
}
