// ubench_mfma_dnec.hip -- diagnostic (tools only): an accumulate chain whose
// MFMA writes a DIFFERENT register than its SrcC (v_mfma v[D] ... v[C], D != C:
// the renamed accumulator hipcc emits in the fused VJP kernel) -- is the
// previous MFMA's result forwarded, or read stale from the register file?
// Chain of 6 v_mfma_f32_16x16x32_f16 (A = B = fp16 ones, +32 each) through
// v[48:51] -> v[52:55] -> v[48:51] -> ..., back to back or with N wait states
// between; control: the same chain with D == C.  Expected final value 192.
#include <hip/hip_runtime.h>

#include <cstdio>

#define DNEC_KERNEL(NAME, GAP, DST_ALT)                                                                 \
    __global__ __launch_bounds__(256) void NAME(int* bad, float* sink) {                              \
        const unsigned ones = 0x3C003C00u;                                                              \
        float r0, r3;                                                                                   \
        asm volatile(                                                                                   \
            "v_mov_b32 v40, %2\n\tv_mov_b32 v41, %2\n\tv_mov_b32 v42, %2\n\tv_mov_b32 v43, %2\n\t"      \
            "v_mov_b32 v48, 0\n\tv_mov_b32 v49, 0\n\tv_mov_b32 v50, 0\n\tv_mov_b32 v51, 0\n\ts_nop 4\n\t" \
            "v_mfma_f32_16x16x32_f16 " DST_ALT(1) ", v[40:43], v[40:43], v[48:51]\n\t" GAP              \
            "v_mfma_f32_16x16x32_f16 v[48:51], v[40:43], v[40:43], " DST_ALT(1) "\n\t" GAP              \
            "v_mfma_f32_16x16x32_f16 " DST_ALT(1) ", v[40:43], v[40:43], v[48:51]\n\t" GAP              \
            "v_mfma_f32_16x16x32_f16 v[48:51], v[40:43], v[40:43], " DST_ALT(1) "\n\t" GAP              \
            "v_mfma_f32_16x16x32_f16 " DST_ALT(1) ", v[40:43], v[40:43], v[48:51]\n\t" GAP              \
            "v_mfma_f32_16x16x32_f16 v[48:51], v[40:43], v[40:43], " DST_ALT(1) "\n\t"                  \
            "s_nop 7\n\ts_nop 7\n\t"                                                                    \
            "v_mov_b32 %0, v48\n\tv_mov_b32 %1, v51\n\ts_nop 7"                                         \
            : "=&v"(r0), "=&v"(r3)                                                                      \
            : "v"(ones)                                                                                 \
            : "v40", "v41", "v42", "v43", "v48", "v49", "v50", "v51", "v52", "v53", "v54", "v55");      \
        const int nb = (r0 != 192.0f) + (r3 != 192.0f) * 2;                                           \
        if (nb) atomicOr(bad, nb);                                                                      \
        if (nb) atomicAdd(bad + 1, 1);                                                                  \
        sink[blockIdx.x * 256 + threadIdx.x] = r0 + r3;                                                \
    }
#define ALT(x) "v[52:55]"
#define SAME(x) "v[48:51]"

#define LIST(X)                                            \
    X(k_dnec_g0, "", ALT)                                  \
    X(k_dnec_g1, "s_nop 0\n\t", ALT)                       \
    X(k_dnec_g2, "s_nop 1\n\t", ALT)                       \
    X(k_dnec_g4, "s_nop 3\n\t", ALT)                       \
    X(k_dnec_g8, "s_nop 7\n\t", ALT)                       \
    X(k_dnec_g10, "s_nop 7\n\ts_nop 1\n\t", ALT)           \
    X(k_same_g0, "", SAME)

LIST(DNEC_KERNEL)

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
    printf("%-11s waves/SIMD %d: wrong lanes %lld of %lld (mask 1 = row 0, 2 = row 3): %d\n", name, waves_per_simd,
           lanes, (long long)reps * blocks * 256, mask);
    fflush(stdout);
    (void)hipFree(bad);
    (void)hipFree(sink);
}

int main() {
#define RUN(NAME, A, B) run(#NAME, NAME, w);
    for (int w = 1; w <= 2; ++w) { LIST(RUN) }
    return 0;
}
