// ubench_mfma_raw.hip -- diagnostic (tools only): how many wait states must
// separate the last v_mfma_f32_16x16x32_f16 of a chain from a v_accvgpr_read of
// its result?  One asm block: zero a[0:7], run S rounds of two interleaved
// chains (a[0:3], a[4:7]; A = B = fp16 ones, +32 per MFMA per element), then
// after N wait states read a0 and a3 (rows written first / last) of the last
// MFMA's accumulator.  A value below 32 S is a stale read.  Run: ./ubench_mfma_raw
#include <hip/hip_runtime.h>

#include <cstdio>

#define RAW_KERNEL(NAME, NOPTXT)                                                                      \
    __global__ __launch_bounds__(256) void NAME(int* bad, float* sink) {                            \
        const unsigned ones = 0x3C003C00u;                                                            \
        float r0, r3, q3;                                                                              \
        asm volatile(                                                                                  \
            "v_mov_b32 v40, %3\n\tv_mov_b32 v41, %3\n\tv_mov_b32 v42, %3\n\tv_mov_b32 v43, %3\n\t"    \
            "v_accvgpr_write_b32 a0, 0\n\tv_accvgpr_write_b32 a1, 0\n\tv_accvgpr_write_b32 a2, 0\n\t" \
            "v_accvgpr_write_b32 a3, 0\n\tv_accvgpr_write_b32 a4, 0\n\tv_accvgpr_write_b32 a5, 0\n\t" \
            "v_accvgpr_write_b32 a6, 0\n\tv_accvgpr_write_b32 a7, 0\n\ts_nop 4\n\t"                  \
            "v_mfma_f32_16x16x32_f16 a[0:3], v[40:43], v[40:43], a[0:3]\n\t"                           \
            "v_mfma_f32_16x16x32_f16 a[4:7], v[40:43], v[40:43], a[4:7]\n\t"                           \
            "v_mfma_f32_16x16x32_f16 a[0:3], v[40:43], v[40:43], a[0:3]\n\t"                           \
            "v_mfma_f32_16x16x32_f16 a[4:7], v[40:43], v[40:43], a[4:7]\n\t"                           \
            "v_mfma_f32_16x16x32_f16 a[0:3], v[40:43], v[40:43], a[0:3]\n\t"                           \
            "v_mfma_f32_16x16x32_f16 a[4:7], v[40:43], v[40:43], a[4:7]\n\t" NOPTXT                    \
            "v_accvgpr_read_b32 %0, a4\n\t"                                                            \
            "v_accvgpr_read_b32 %1, a7\n\t"                                                            \
            "v_accvgpr_read_b32 %2, a3\n\t"                                                            \
            "s_nop 7\n\ts_nop 7\n\ts_nop 7\n\ts_nop 7"                                                 \
            : "=&v"(r0), "=&v"(r3), "=&v"(q3)                                                          \
            : "v"(ones)                                                                                \
            : "v40", "v41", "v42", "v43", "a0", "a1", "a2", "a3", "a4", "a5", "a6", "a7");             \
        const int nb = (r0 != 96.0f) + (r3 != 96.0f) * 2 + (q3 != 96.0f) * 4;                       \
        if (nb) atomicOr(bad, nb);                                                                     \
        if (nb) atomicAdd(bad + 1, 1);                                                                 \
        sink[blockIdx.x * 256 + threadIdx.x] = r0 + r3 + q3;                                          \
    }

#define LIST(X)                                              \
    X(k_n0, "")                                              \
    X(k_n2, "s_nop 1\n\t")                                   \
    X(k_n4, "s_nop 3\n\t")                                   \
    X(k_n8, "s_nop 7\n\t")                                   \
    X(k_n10, "s_nop 7\n\ts_nop 1\n\t")                       \
    X(k_n12, "s_nop 7\n\ts_nop 3\n\t")                       \
    X(k_n16, "s_nop 7\n\ts_nop 7\n\t")                       \
    X(k_n20, "s_nop 7\n\ts_nop 7\n\ts_nop 3\n\t")            \
    X(k_n32, "s_nop 7\n\ts_nop 7\n\ts_nop 7\n\ts_nop 7\n\t")

LIST(RAW_KERNEL)

static void run(const char* name, void (*k)(int*, float*), int waves_per_simd) {
    const int blocks = 256 * waves_per_simd, reps = 50;
    int* bad;
    float* sink;
    (void)hipMalloc(&bad, 2 * sizeof(int));
    (void)hipMalloc(&sink, sizeof(float) * blocks * 256);
    int mask = 0;
    long long lanes = 0;
    for (int r = 0; r < reps; ++r) {
        (void)hipMemset(bad, 0, 2 * sizeof(int));
        hipLaunchKernelGGL(k, dim3(blocks), dim3(256), 0, 0, bad, sink);
        int h[2] = {0, 0};
        (void)hipMemcpy(h, bad, 2 * sizeof(int), hipMemcpyDeviceToHost);
        mask |= h[0];
        lanes += h[1];
    }
    printf("%-6s waves/SIMD %d: stale lanes %lld of %lld (mask: 1 = last MFMA row 0, 2 = its row 3, 4 = the chain "
           "before it, row 3): %d\n", name, waves_per_simd, lanes, (long long)reps * blocks * 256, mask);
    fflush(stdout);
    (void)hipFree(bad);
    (void)hipFree(sink);
}

int main() {
#define RUN(NAME, A) run(#NAME, NAME, w);
    for (int w = 1; w <= 2; ++w) { LIST(RUN) }
    return 0;
}
