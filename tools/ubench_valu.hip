// Aggregate VALU issue rate of one SIMD with 1..4 resident waves (gfx950).
// Each wave runs ILP independent dependency chains of one instruction kind;
// the per-wave cycle count (s_memtime) and the kernel wall time give cycles
// per wave-instruction per SIMD.  Used to set the VALU-issue floor in
// bench.py (what one VALU / transcendental instruction costs the SIMD when
// several waves share it).
//   hipcc -O3 --offload-arch=gfx950 -fno-slp-vectorize -w tools/ubench_valu.hip -o tools/ubench_valu
#include <hip/hip_runtime.h>
#include <cstdio>

constexpr int ILP = 8;
constexpr int UNROLL = 16;

template <int KIND>
__global__ __launch_bounds__(256) void k_valu(float* out, long long* cyc, int iters, float b, float c) {
    float a[ILP];
#pragma unroll
    for (int i = 0; i < ILP; ++i) a[i] = threadIdx.x * 1e-3f + i;
    const long long t0 = __builtin_readcyclecounter();
    for (int it = 0; it < iters; ++it) {
#pragma unroll
        for (int u = 0; u < UNROLL; ++u)
#pragma unroll
            for (int i = 0; i < ILP; ++i) {
                if (KIND == 0) a[i] = __builtin_fmaf(a[i], b, c);
                if (KIND == 1) a[i] = __builtin_amdgcn_exp2f(a[i]);
                if (KIND == 2) a[i] = a[i] + c;
                if (KIND == 3 && (i & 1) == 0) {  // packed fp32 FMA on the pair (i, i+1)
                    typedef float f2 __attribute__((ext_vector_type(2)));
                    const f2 r = __builtin_elementwise_fma(f2{a[i], a[i + 1]}, f2{b, b}, f2{c, c});
                    a[i] = r.x;
                    a[i + 1] = r.y;
                }
            }
    }
    const long long t1 = __builtin_readcyclecounter();
    float s = 0.0f;
#pragma unroll
    for (int i = 0; i < ILP; ++i) s += a[i];
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
    if ((threadIdx.x & 63) == 0) cyc[(blockIdx.x * blockDim.x + threadIdx.x) >> 6] = t1 - t0;
}

template <int KIND>
void run(const char* name, int waves_per_simd) {
    const int blocks = 256 * waves_per_simd;  // 256 threads = 4 waves, one per SIMD
    const int iters = 2000;
    float* out;
    long long* cyc;
    hipMalloc(&out, blocks * 256 * sizeof(float));
    hipMalloc(&cyc, blocks * 4 * sizeof(long long));
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    k_valu<KIND><<<blocks, 256>>>(out, cyc, 10, 0.999f, 1e-4f);
    hipEventRecord(e0);
    k_valu<KIND><<<blocks, 256>>>(out, cyc, iters, 0.999f, 1e-4f);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms;
    hipEventElapsedTime(&ms, e0, e1);
    long long* h = new long long[blocks * 4];
    hipMemcpy(h, cyc, blocks * 4 * sizeof(long long), hipMemcpyDeviceToHost);
    double mean = 0;
    for (int i = 0; i < blocks * 4; ++i) mean += h[i];
    mean /= blocks * 4;
    const double inst_per_wave = (double)iters * UNROLL * ILP;
    // wall: every SIMD ran waves_per_simd waves of inst_per_wave instructions
    const double ghz_nominal = 2.4;
    printf("%-6s waves/SIMD %d: per-wave %.2f cyc/inst (s_memtime), wall %.3f ms -> %.2f ns per "
           "wave-inst per SIMD (%.2f cyc at %.1f GHz)\n",
           name, waves_per_simd, mean / inst_per_wave, ms, ms * 1e6 / (inst_per_wave * waves_per_simd),
           ms * 1e6 / (inst_per_wave * waves_per_simd) * ghz_nominal, ghz_nominal);
    delete[] h;
    hipFree(out);
    hipFree(cyc);
}

int main() {
    for (int w = 1; w <= 4; ++w) run<0>("v_fma", w);
    for (int w = 1; w <= 4; ++w) run<2>("v_add", w);
    for (int w = 1; w <= 4; ++w) run<1>("v_exp", w);
    for (int w = 1; w <= 4; ++w) run<3>("pk_fma", w);  // ILP/2 instructions per unrolled step
    return 0;
}
