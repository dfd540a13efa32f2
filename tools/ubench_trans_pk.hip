// ubench_trans_pk.hip -- diagnostic (tools only): a transcendental VALU op
// (v_exp_f32 / v_rcp_f32) writes one register of a pair that a packed-FP32
// op (v_pk_mul_f32 by 1.0) reads after N wait states -- as the pair's low
// (v50) or high (v51) half.  A stale read returns the pair's old value (-1).
// Run: ./ubench_trans_pk
#include <hip/hip_runtime.h>

#include <cstdio>

typedef float f32x2 __attribute__((ext_vector_type(2)));

#define TP_KERNEL(NAME, TRANS, DSTREG, NOPTXT, RESREG)                                                \
    __global__ __launch_bounds__(256) void NAME(int* bad, float* sink, float xin) {                  \
        const f32x2 one2 = {1.0f, 1.0f};                                                               \
        float r;                                                                                       \
        asm volatile(                                                                                  \
            "v_mov_b32 v50, -1.0\n\tv_mov_b32 v51, -1.0\n\ts_nop 4\n\t"                                \
            TRANS " " DSTREG ", %1\n\t" NOPTXT                                                         \
            "v_pk_mul_f32 v[52:53], v[50:51], %2\n\t"                                                  \
            "s_nop 7\n\ts_nop 7\n\t"                                                                   \
            "v_mov_b32 %0, " RESREG "\n\ts_nop 3"                                                      \
            : "=&v"(r)                                                                                 \
            : "v"(xin), "v"(one2)                                                                      \
            : "v50", "v51", "v52", "v53");                                                             \
        sink[blockIdx.x * 256 + threadIdx.x] = r;                                                     \
        if (r < 0.0f) atomicAdd(bad, 1);                                                               \
    }

#define LIST(X)                                                    \
    X(exp_hi_n0, "v_exp_f32", "v51", "", "v53")                    \
    X(exp_hi_n1, "v_exp_f32", "v51", "s_nop 0\n\t", "v53")         \
    X(exp_hi_n2, "v_exp_f32", "v51", "s_nop 1\n\t", "v53")         \
    X(exp_hi_n4, "v_exp_f32", "v51", "s_nop 3\n\t", "v53")         \
    X(exp_lo_n0, "v_exp_f32", "v50", "", "v52")                    \
    X(exp_lo_n1, "v_exp_f32", "v50", "s_nop 0\n\t", "v52")         \
    X(rcp_hi_n0, "v_rcp_f32", "v51", "", "v53")                    \
    X(rcp_hi_n1, "v_rcp_f32", "v51", "s_nop 0\n\t", "v53")         \
    X(rcp_lo_n0, "v_rcp_f32", "v50", "", "v52")                    \
    X(log_hi_n0, "v_log_f32", "v51", "", "v53")

LIST(TP_KERNEL)

static void run(const char* name, void (*k)(int*, float*, float), int waves_per_simd) {
    const int blocks = 256 * waves_per_simd, reps = 50;
    int* bad;
    float* sink;
    (void)hipMalloc(&bad, sizeof(int));
    (void)hipMalloc(&sink, sizeof(float) * blocks * 256);
    long long n = 0;
    for (int r = 0; r < reps; ++r) {
        (void)hipMemset(bad, 0, sizeof(int));
        hipLaunchKernelGGL(k, dim3(blocks), dim3(256), 0, 0, bad, sink, 1.5f);
        int h = 0;
        (void)hipMemcpy(&h, bad, sizeof(int), hipMemcpyDeviceToHost);
        n += h;
    }
    printf("%-10s waves/SIMD %d: stale lanes %lld of %lld\n", name, waves_per_simd, n,
           (long long)reps * blocks * 256);
    fflush(stdout);
    (void)hipFree(bad);
    (void)hipFree(sink);
}

int main() {
#define RUN(NAME, A, B, C, D) run(#NAME, NAME, w);
    for (int w = 1; w <= 2; ++w) { LIST(RUN) }
    return 0;
}
