// ubench_trans_pk2.hip -- diagnostic (tools only): a transcendental's result
// read by a packed-FP32 op N instructions later (N-1 independent VALU ops
// between), with the SIMD's other waves idle, issuing transcendentals, or
// issuing MFMAs.  The fused VJP's element backward (profiles/r5/*) computes
// different results in lanes 48-63 -- the last quarter of a wave64 pass
// through the quarter-rate transcendental unit -- only when other waves share
// the SIMD and only in builds with packed-FP32 code; its gaps between a
// transcendental and a packed consumer are 2-9 instructions (hipcc pads 1).
// Every step: v20 = exp2(v20 - v20) = 1 (trans), independent fillers, then
// v[20:21] = v[20:21] * v[24:25] (packed, 1.0) -- a stale read of v20 shows
// as the value before the exp (x0 + 7 != 1).
#include <hip/hip_runtime.h>

#include <cstdio>

#define FILL1 ""
#define FILL2 "v_add_f32 v30, 1.0, v30\n\t"
#define FILL3 FILL2 "v_add_f32 v31, 1.0, v31\n\t"
#define FILL5 FILL3 "v_add_f32 v32, 1.0, v32\n\tv_add_f32 v33, 1.0, v33\n\t"
#define STEP(F) "v_mov_b32 v20, v29\n\ts_nop 4\n\tv_exp_f32 v20, v28\n\t" F "v_pk_mul_f32 v[22:23], v[20:21], v[24:25]\n\ts_nop 4\n\tv_add_f32 v26, v26, v22\n\t"
#define X8(s) s s s s s s s s

#define LIST(X) X(g1, FILL1) X(g2, FILL2) X(g3, FILL3) X(g5, FILL5)

// partner: 0 none, 1 transcendentals, 2 MFMAs, 3 both
#define TP_KERNEL(NAME, F)                                                                            \
    template <int PARTNER>                                                                            \
    __global__ __launch_bounds__(512) void NAME(int* bad, float* sink, int iters) {                  \
        const int wave = threadIdx.x >> 6;                                                            \
        if (wave >= 4) {                                                                              \
            if (PARTNER == 0) return;                                                                 \
            float r = 0.0f;                                                                           \
            if (PARTNER & 1) {                                                                        \
                asm volatile("v_mov_b32 v60, 0x3f000000\n\ts_mov_b32 s7, %1\n"                        \
                             "3:\n\t" X8("v_exp_f32 v61, v60\n\tv_rcp_f32 v62, v60\n\tv_log_f32 v63, v60\n\t") \
                             "s_sub_u32 s7, s7, 1\n\ts_cmp_lg_u32 s7, 0\n\ts_cbranch_scc1 3b\n\t"          \
                             "s_nop 4\n\tv_add_f32 %0, v61, v62"                                      \
                             : "=v"(r) : "s"(iters * 2) : "v60", "v61", "v62", "v63", "s7", "scc");    \
            }                                                                                         \
            if (PARTNER & 2) {                                                                        \
                float q;                                                                              \
                asm volatile(                                                                         \
                    "v_mov_b32 v40, 0x3c003c00\n\tv_mov_b32 v41, 0x3c003c00\n\tv_mov_b32 v42, 0x3c003c00\n\t" \
                    "v_mov_b32 v43, 0x3c003c00\n\tv_mov_b32 v48, 0\n\tv_mov_b32 v49, 0\n\tv_mov_b32 v50, 0\n\t" \
                    "v_mov_b32 v51, 0\n\ts_mov_b32 s6, %1\n\ts_nop 4\n"                                \
                    "2:\n\t"                                                                          \
                    "v_mfma_f32_16x16x32_f16 v[48:51], v[40:43], v[40:43], v[48:51]\n\t"              \
                    "v_mfma_f32_16x16x32_f16 v[48:51], v[40:43], v[40:43], v[48:51]\n\t"              \
                    "s_sub_u32 s6, s6, 1\n\ts_cmp_lg_u32 s6, 0\n\ts_cbranch_scc1 2b\n\t"              \
                    "s_nop 15\n\tv_mov_b32 %0, v48"                                                   \
                    : "=v"(q) : "s"(iters * 4) : "v40", "v41", "v42", "v43", "v48", "v49", "v50", "v51", "s6", "scc"); \
                r += q;                                                                               \
            }                                                                                         \
            sink[blockIdx.x * 512 + threadIdx.x] = r;                                                 \
            return;                                                                                   \
        }                                                                                             \
        const float x0 = 5.0f + (float)(threadIdx.x & 63);                                            \
        float acc;                                                                                    \
        asm volatile(                                                                                 \
            "v_mov_b32 v29, %1\n\tv_mov_b32 v28, 0\n\tv_mov_b32 v21, 1.0\n\tv_mov_b32 v24, 1.0\n\t"   \
            "v_mov_b32 v25, 1.0\n\tv_mov_b32 v26, 0\n\ts_mov_b32 s5, %2\n\ts_nop 4\n"                 \
            "1:\n\t" X8(STEP(F)) "s_sub_u32 s5, s5, 1\n\ts_cmp_lg_u32 s5, 0\n\ts_cbranch_scc1 1b\n\t" \
            "s_nop 4\n\tv_mov_b32 %0, v26"                                                            \
            : "=v"(acc)                                                                               \
            : "v"(x0), "s"(iters)                                                                     \
            : "v20", "v21", "v22", "v23", "v24", "v25", "v26", "v28", "v29", "v30", "v31", "v32",    \
              "v33", "s5", "scc");                                                                    \
        const int l = threadIdx.x & 63;                                                               \
        if (acc != 8.0f * (float)iters) atomicAdd(bad + 1 + (l >> 4), 1);                             \
        sink[blockIdx.x * 512 + threadIdx.x] = acc;                                                   \
    }
LIST(TP_KERNEL)

static const char* pname[4] = {"alone        ", "trans partner", "MFMA partner ", "trans + MFMA "};

static void run(const char* name, void (*k)(int*, float*, int), int wgs_per_cu, int partner) {
    const int blocks = 256 * wgs_per_cu, reps = 20, iters = 64;
    int* bad;
    float* sink;
    (void)hipMalloc(&bad, 5 * sizeof(int));
    (void)hipMalloc(&sink, sizeof(float) * blocks * 512);
    (void)hipMemset(bad, 0, 5 * sizeof(int));
    for (int r = 0; r < reps; ++r) hipLaunchKernelGGL(k, dim3(blocks), dim3(512), 0, 0, bad, sink, iters);
    int h[5] = {0};
    (void)hipMemcpy(h, bad, sizeof(h), hipMemcpyDeviceToHost);
    printf("trans->pk %-3s %s, %d workgroups/CU: wrong lanes %d of %lld; by lane quarter 0-15 %d, 16-31 %d, "
           "32-47 %d, 48-63 %d\n", name, pname[partner], wgs_per_cu, h[1] + h[2] + h[3] + h[4],
           (long long)reps * blocks * 256, h[1], h[2], h[3], h[4]);
    fflush(stdout);
    (void)hipFree(bad);
    (void)hipFree(sink);
}

int main() {
#define RUN(NAME, F) run(#NAME, NAME<0>, w, 0); run(#NAME, NAME<1>, w, 1); run(#NAME, NAME<2>, w, 2); run(#NAME, NAME<3>, w, 3);
    for (int w = 1; w <= 2; ++w) { LIST(RUN) }
    return 0;
}
