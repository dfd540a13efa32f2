// ubench_pk_raw.hip -- diagnostic (tools only): read-after-write between
// back-to-back packed-FP32 VALU instructions on gfx950.
//
// The fused VJP's divergence (profiles/r5_vjp_capture.txt) is confined to
// lanes 48-63 of the element backward, whose inputs were bitwise equal across
// runs; the only instruction pattern that separates the diverging builds from
// the reproducible ones is a v_pk_fma_f32 reading the result of the
// v_pk_fma_f32 right before it (2 sites in the fast forward instance, 8 in
// each exact instance, 0 in the fast inverse).  Here: chains of dependent
// packed ops at gap 1 (back to back) and gap 2 (s_nop 0 between), plus the
// kernel's own sequence, alone and beside MFMA chains on the same SIMD.  Each
// step adds a known amount to each half, so a stale read shows as a short
// count; wrong lanes are counted per lane quarter.
#include <hip/hip_runtime.h>

#include <cstdio>

#define STEP_G1 "v_pk_fma_f32 v[22:23], v[24:25], v[20:21], v[24:25]\n\tv_pk_fma_f32 v[20:21], v[24:25], v[22:23], v[24:25]\n\t"
#define STEP_G2 \
    "v_pk_fma_f32 v[22:23], v[24:25], v[20:21], v[24:25]\n\ts_nop 0\n\tv_pk_fma_f32 v[20:21], v[24:25], v[22:23], v[24:25]\n\ts_nop 0\n\t"
// the element backward's own shape: pk_mul, a SALU op, pk_fma (D1), pk_fma reading D1
#define STEP_KS                                                    \
    "v_pk_mul_f32 v[26:27], v[24:25], v[20:21]\n\t"                \
    "s_mov_b32 s4, 1.0\n\t"                                        \
    "v_pk_fma_f32 v[22:23], v[24:25], v[26:27], v[24:25]\n\t"      \
    "v_pk_fma_f32 v[20:21], v[24:25], v[22:23], v[28:29]\n\t"
// a 32-bit VALU write of the pair's high register, then a packed read at gap 1
#define STEP_HI32 "v_add_f32 v21, 1.0, v21\n\tv_pk_fma_f32 v[20:21], v[24:25], v[20:21], v[24:25]\n\t"
#define STEP_LO32 "v_add_f32 v20, 1.0, v20\n\tv_pk_fma_f32 v[20:21], v[24:25], v[20:21], v[24:25]\n\t"
#define X8(s) s s s s s s s s
#define X32(s) X8(s) X8(s) X8(s) X8(s)

// per step of each chain: how much it adds to the low and the high half
#define LIST(X)                       \
    X(pkpk_g1, STEP_G1, 2.0f, 2.0f)   \
    X(pkpk_g2, STEP_G2, 2.0f, 2.0f)   \
    X(pk_kseq, STEP_KS, 1.0f, 1.0f)   \
    X(hi32_pk, STEP_HI32, 1.0f, 2.0f) \
    X(lo32_pk, STEP_LO32, 2.0f, 1.0f)

// 512-thread workgroups: waves 0-3 run the packed chain; with PARTNER, waves
// 4-7 (which share SIMDs with waves 0-3, tools/simd_map.hip) run dependent
// 16x16x32 f16 MFMA chains meanwhile, so VALU and MFMA co-execute on a SIMD
#define PK_KERNEL(NAME, STEP, PLO, PHI)                                                               \
    template <bool PARTNER>                                                                           \
    __global__ __launch_bounds__(512) void NAME(int* bad, float* sink, int iters) {                  \
        const int wave = threadIdx.x >> 6;                                                            \
        if (wave >= 4) {                                                                              \
            if (!PARTNER) return;                                                                     \
            float r;                                                                                  \
            asm volatile(                                                                             \
                "v_mov_b32 v40, 0x3c003c00\n\tv_mov_b32 v41, 0x3c003c00\n\tv_mov_b32 v42, 0x3c003c00\n\t" \
                "v_mov_b32 v43, 0x3c003c00\n\t"                                                      \
                "v_mov_b32 v48, 0\n\tv_mov_b32 v49, 0\n\tv_mov_b32 v50, 0\n\tv_mov_b32 v51, 0\n\t"   \
                "v_mov_b32 v52, 0\n\tv_mov_b32 v53, 0\n\tv_mov_b32 v54, 0\n\tv_mov_b32 v55, 0\n\t"   \
                "s_mov_b32 s6, %1\n\ts_nop 4\n"                                                       \
                "2:\n\t"                                                                              \
                "v_mfma_f32_16x16x32_f16 v[48:51], v[40:43], v[40:43], v[48:51]\n\t"                  \
                "v_mfma_f32_16x16x32_f16 v[52:55], v[40:43], v[40:43], v[52:55]\n\t"                  \
                "v_mfma_f32_16x16x32_f16 v[48:51], v[40:43], v[40:43], v[48:51]\n\t"                  \
                "v_mfma_f32_16x16x32_f16 v[52:55], v[40:43], v[40:43], v[52:55]\n\t"                  \
                "s_sub_u32 s6, s6, 1\n\ts_cmp_lg_u32 s6, 0\n\ts_cbranch_scc1 2b\n\t"                  \
                "s_nop 15\n\tv_add_f32 %0, v48, v52"                                                  \
                : "=v"(r)                                                                             \
                : "s"(iters * 4)                                                                      \
                : "v40", "v41", "v42", "v43", "v48", "v49", "v50", "v51", "v52", "v53", "v54", "v55", \
                  "s6", "scc");                                                                       \
            sink[blockIdx.x * 512 + threadIdx.x] = r;                                                 \
            return;                                                                                   \
        }                                                                                             \
        const float x0 = (float)(threadIdx.x & 63) * 4.0f;                                            \
        float lo, hi;                                                                                 \
        asm volatile(                                                                                 \
            "v_mov_b32 v20, %2\n\tv_mov_b32 v21, %2\n\tv_mov_b32 v24, 1.0\n\tv_mov_b32 v25, 1.0\n\t"  \
            "v_mov_b32 v28, 0\n\tv_mov_b32 v29, 0\n\ts_mov_b32 s5, %3\n\ts_nop 4\n"                   \
            "1:\n\t" X8(STEP) "s_sub_u32 s5, s5, 1\n\ts_cmp_lg_u32 s5, 0\n\ts_cbranch_scc1 1b\n\t"   \
            "s_nop 4\n\tv_mov_b32 %0, v20\n\tv_mov_b32 %1, v21\n\ts_nop 4"                            \
            : "=v"(lo), "=v"(hi)                                                                      \
            : "v"(x0), "s"(iters)                                                                     \
            : "v20", "v21", "v22", "v23", "v24", "v25", "v26", "v27", "v28", "v29", "s4", "s5",     \
              "scc");                                                                                 \
        const int l = threadIdx.x & 63;                                                               \
        const float n = 8.0f * (float)iters;                                                          \
        if (lo != x0 + n * (PLO) || hi != x0 + n * (PHI)) atomicAdd(bad + 1 + (l >> 4), 1);           \
        sink[blockIdx.x * 512 + threadIdx.x] = lo + hi;                                               \
    }
LIST(PK_KERNEL)

static void run(const char* name, void (*k)(int*, float*, int), int wgs_per_cu, bool partner) {
    const int blocks = 256 * wgs_per_cu, reps = 20, iters = 64;
    int* bad;
    float* sink;
    (void)hipMalloc(&bad, 5 * sizeof(int));
    (void)hipMalloc(&sink, sizeof(float) * blocks * 512);
    (void)hipMemset(bad, 0, 5 * sizeof(int));
    for (int r = 0; r < reps; ++r) hipLaunchKernelGGL(k, dim3(blocks), dim3(512), 0, 0, bad, sink, iters);
    int h[5] = {0};
    (void)hipMemcpy(h, bad, sizeof(h), hipMemcpyDeviceToHost);
    printf("%-9s %s, %d workgroups/CU: wrong lanes %d of %lld; by lane quarter 0-15 %d, 16-31 %d, 32-47 %d, "
           "48-63 %d\n", name, partner ? "MFMA partner" : "alone       ", wgs_per_cu, h[1] + h[2] + h[3] + h[4],
           (long long)reps * blocks * 256, h[1], h[2], h[3], h[4]);
    fflush(stdout);
    (void)hipFree(bad);
    (void)hipFree(sink);
}

int main() {
#define RUN(NAME, STEP, PLO, PHI) run(#NAME, NAME<false>, w, false); run(#NAME, NAME<true>, w, true);
    for (int w = 1; w <= 2; ++w) { LIST(RUN) }
    return 0;
}
