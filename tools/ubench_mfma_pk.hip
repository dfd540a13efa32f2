// ubench_mfma_pk.hip -- diagnostic (tools only): a 16x16x32 f16 MFMA writes its
// result to VGPRs v[48:51] (the fused VJP keeps accumulators in VGPRs); after N
// wait states a packed-FP32 VALU op (v_pk_mul_f32 by 1.0) reads the pair
// v[50:51] (rows written last), a scalar v_mul_f32 reads v51, and a second
// v_pk_mul_f32 reads v[48:49].  Any result below the chain's 96 is stale.
// Also what hipcc itself emits between an MFMA and a packed read (k_cc).
#include <hip/hip_runtime.h>

#include <cstdio>

typedef _Float16 h8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x2 __attribute__((ext_vector_type(2)));

#define PK_KERNEL(NAME, NOPTXT)                                                                        \
    __global__ __launch_bounds__(256) void NAME(int* bad, float* sink) {                             \
        const unsigned ones = 0x3C003C00u;                                                             \
        const float one = 1.0f;                                                                        \
        const f32x2 one2 = {1.0f, 1.0f};                                                               \
        float p2, p3, s3, p0;                                                                          \
        asm volatile(                                                                                  \
            "v_mov_b32 v40, %4\n\tv_mov_b32 v41, %4\n\tv_mov_b32 v42, %4\n\tv_mov_b32 v43, %4\n\t"     \
            "v_mov_b32 v48, 0\n\tv_mov_b32 v49, 0\n\tv_mov_b32 v50, 0\n\tv_mov_b32 v51, 0\n\t"         \
            "v_mov_b32 v44, 0\n\tv_mov_b32 v45, 0\n\tv_mov_b32 v46, 0\n\tv_mov_b32 v47, 0\n\ts_nop 4\n\t" \
            "v_mfma_f32_16x16x32_f16 v[48:51], v[40:43], v[40:43], v[48:51]\n\t"                       \
            "v_mfma_f32_16x16x32_f16 v[44:47], v[40:43], v[40:43], v[44:47]\n\t"                       \
            "v_mfma_f32_16x16x32_f16 v[48:51], v[40:43], v[40:43], v[48:51]\n\t"                       \
            "v_mfma_f32_16x16x32_f16 v[44:47], v[40:43], v[40:43], v[44:47]\n\t"                       \
            "v_mfma_f32_16x16x32_f16 v[48:51], v[40:43], v[40:43], v[48:51]\n\t" NOPTXT                \
            "v_pk_mul_f32 v[52:53], v[50:51], %6\n\t"                                  \
            "v_mul_f32 v54, v51, %5\n\t"                                                               \
            "v_pk_mul_f32 v[56:57], v[48:49], %6\n\t"                                  \
            "s_nop 7\n\ts_nop 7\n\t"                                                                   \
            "v_mov_b32 %0, v52\n\tv_mov_b32 %1, v53\n\tv_mov_b32 %2, v54\n\tv_mov_b32 %3, v56\n\t"     \
            "s_nop 7\n\ts_nop 7"                                                                       \
            : "=&v"(p2), "=&v"(p3), "=&v"(s3), "=&v"(p0)                                               \
            : "v"(ones), "v"(one), "v"(one2)                                                           \
            : "v40", "v41", "v42", "v43", "v44", "v45", "v46", "v47", "v48", "v49", "v50", "v51",      \
              "v52", "v53", "v54", "v55", "v56", "v57");                                               \
        const int nb = (p2 != 96.0f) + (p3 != 96.0f) * 2 + (s3 != 96.0f) * 4 + (p0 != 96.0f) * 8;   \
        if (nb) atomicOr(bad, nb);                                                                     \
        if (nb) atomicAdd(bad + 1, 1);                                                                 \
        sink[blockIdx.x * 256 + threadIdx.x] = p2 + p3 + s3 + p0;                                     \
    }

#define LIST(X)                                     \
    X(k_n0, "")                                     \
    X(k_n2, "s_nop 1\n\t")                          \
    X(k_n4, "s_nop 3\n\t")                          \
    X(k_n6, "s_nop 5\n\t")                          \
    X(k_n8, "s_nop 7\n\t")                          \
    X(k_n10, "s_nop 7\n\ts_nop 1\n\t")              \
    X(k_n12, "s_nop 7\n\ts_nop 3\n\t")              \
    X(k_n16, "s_nop 7\n\ts_nop 7\n\t")

LIST(PK_KERNEL)

// what hipcc emits between an MFMA with a VGPR result and packed-FP32 consumers
__global__ __launch_bounds__(256) void k_cc(const float* in, float* out, float s) {
    h8 a;
    for (int j = 0; j < 8; ++j) a[j] = (_Float16)in[threadIdx.x * 8 + j];
    f32x4 acc = {in[0], in[1], in[2], in[3]};
    acc = __builtin_amdgcn_mfma_f32_16x16x32_f16(a, a, acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_16x16x32_f16(a, a, acc, 0, 0, 0);
    out[threadIdx.x * 4 + 0] = acc[0] * s;
    out[threadIdx.x * 4 + 1] = acc[1] * s;
    out[threadIdx.x * 4 + 2] = acc[2] * s;
    out[threadIdx.x * 4 + 3] = acc[3] * s;
}

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
    printf("%-6s waves/SIMD %d: stale lanes %lld of %lld (mask: 1/2 = pk read of rows 2/3, 4 = scalar read of row 3, "
           "8 = pk read of row 0): %d\n", name, waves_per_simd, lanes, (long long)reps * blocks * 256, mask);
    fflush(stdout);
    (void)hipFree(bad);
    (void)hipFree(sink);
}

int main() {
#define RUN(NAME, A) run(#NAME, NAME, w);
    for (int w = 1; w <= 2; ++w) { LIST(RUN) }
    return 0;
}
