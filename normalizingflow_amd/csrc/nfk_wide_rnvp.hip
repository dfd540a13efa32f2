// nfk_wide_rnvp.hip -- RealNVP layers with wide conditioners at small batches:
// applications/input/Polymer_rnvp.yaml's flow (RealNVP(2048, hidden 4000) x 10,
// batch 40; the driver, applications/examples/polymer.py:29,37-41, samples 100
// rows and evaluates them), nf/flows.py:44-76 over FCNN conditioners (20-35).
//
// At 40-128 rows a layer is its weights: 4 FCNN(1024, 1024, 4000) = 96.8 M
// parameters (387 MB) against 40 x 2048 x 4 B of x.  Every weight is read once
// per layer launch sequence, so the floor is the HBM stream (48 us per layer
// at 8 TB/s).  Per half-coupling (s and t conditioners of one input run side
// by side as the two "groups" of every stage):
//
//   k_wl_rows   x half -> fp16 hi/lo B fragments of the input, per-row 2^e scale
//   k_wl_gemm   L1: [M, half] x W1^T for s and t     -> split-K partial sums
//   k_wl_act    sum the partials, unscale, + b1, tanh -> hi/lo fragments (2^14)
//   k_wl_gemm   L2: [M, H] x W2^T (s, t)              -> partials
//   k_wl_act    + b2, tanh                             -> fragments
//   (up to 64 rows each GEMM + act pair is ONE k_wl_gemm_act launch: 9
//   launches per layer instead of 13)
//   k_wl_gemm   L3: [M, H] x W3^T (s, t)              -> partials
//   k_wl_rows   s, t = partials + b3; the affine coupling (flows.py:56, 59 /
//               69, 72), log|det| += (-)sum s per row (fixed order), and the
//               fragments of the output half: the next half-coupling's input
//
// GEMM (k_wl_gemm): weights packed once (nfk_wlin_pack) as the A operand of
// v_mfma_f32_16x16x32_f16 in the two-way fp16 split of the fused kernels
// (hi = f16(2^s w), lo = f16(2^s w - hi); products lo.hi + hi.lo + hi.hi in
// fp32 accumulators; 2^s puts max|W| just under 2^15), 16 output features x 32
// k per 2-KiB (hi, lo) block, the blocks of one 16-feature tile contiguous over
// k.  A workgroup = 4 waves (one per SIMD) owns 4 NTW output tiles of one group
// and a chunk of KC k-blocks: the chunk's input fragments (MT sample tiles)
// are copied into LDS once (LDS-DMA) and shared by the 4 waves; each wave
// streams its NTW tiles' weights from HBM straight into registers, kWlPF
// k-blocks ahead, and writes fp32 partial sums [group][split][row][feature].
// The split count is chosen so the grid covers every CU (>= 256 workgroups)
// with as few partial sums as that allows; they are summed in split order by
// the next stage (deterministic, bitwise reproducible).
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdint>
#include <cstdlib>

#include "../../include/nfk.h"

int nfk_set_error(const char* msg);  // nfk_kernels.hip

namespace {

typedef _Float16 h8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

// GEMM workgroup shapes (waves NW, output tiles per wave NTW, k-blocks of
// weights in flight per wave PF; 8 output tiles per workgroup either way): see
// wl_cfg
constexpr int kWlTilesPerWG = 8;
constexpr int kWlMaxMT = 8;                    // sample tiles per pass: 128 rows
constexpr int kWlHdr = 64;                     // pack header floats ([0] = 2^-s)
constexpr float kWlAct = 16384.0f;             // tanh outputs split at 2^14
constexpr int kWlTarget = 256;                 // GEMM workgroups: at least one per CU
// the weight stream's loads non-temporal (every weight is read once per layer)
#ifndef NFK_WL_NT
#define NFK_WL_NT 1
#endif

int wl_status(const char* what) {
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) {
        nfk_set_error(what);
        return (int)e;
    }
    return 0;
}

__device__ __forceinline__ f32x4 mfma16(h8 a, h8 b, f32x4 c) {
    return __builtin_amdgcn_mfma_f32_16x16x32_f16(a, b, c, 0, 0, 0);
}

__device__ __forceinline__ uint32_t lds_addr(const void* p) {
    return (uint32_t)(uintptr_t)(const __attribute__((address_space(3))) void*)p;
}

// one 16-byte LDS-DMA per lane (global_load_lds_dwordx4; m0 = the LDS base of
// the wave's 1-KiB block, restored after: the compiler reserves m0)
__device__ __forceinline__ void dma16(const float4* gsrc, uint32_t lds) {
    uint32_t saved;
    asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %1\n\ts_nop 0\n\t"
                 "global_load_lds_dwordx4 %2, off\n\ts_mov_b32 m0, %0"
                 : "=&s"(saved)
                 : "s"(__builtin_amdgcn_readfirstlane(lds)), "v"(gsrc)
                 : "memory");
}

// ---------------------------------------------------------------------------
// pack: float[0] = 2^-s (exact), float[1] = max|W| (bits, atomicMax), body
// from float kWlHdr: halfs [nt][kb][part][lane][8] = part of 2^s W[16 nt +
// (lane & 15)][32 kb + 8 (lane >> 4) + j] (zero outside N x K), then one
// all-zero 2-KiB block
__global__ __launch_bounds__(256) void k_wl_max(const float* __restrict__ W, int64_t n, float* pack) {
    float mx = 0.0f;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
        mx = fmaxf(mx, fabsf(W[i]));
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) mx = fmaxf(mx, __shfl_xor(mx, off, 64));
    if ((threadIdx.x & 63) == 0 && mx > 0.0f)
        atomicMax(reinterpret_cast<int*>(pack) + 1, __float_as_int(fminf(mx, 3.0e38f)));
}

__global__ __launch_bounds__(256) void k_wl_pack(const float* __restrict__ W, int N, int K, int KB, int64_t units,
                                                 float* pack) {
    const float mx = __int_as_float(reinterpret_cast<const int*>(pack)[1]);
    int ex = 0;
    if (mx > 0.0f) frexpf(mx, &ex);  // mx < 2^ex
    const float s = ldexpf(1.0f, 15 - ex);
    if (blockIdx.x == 0 && threadIdx.x == 0) pack[0] = ldexpf(1.0f, ex - 15);
    h8* body = reinterpret_cast<h8*>(pack + kWlHdr);
    for (int64_t u = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; u < units; u += (int64_t)gridDim.x * blockDim.x) {
        const int lane = (int)(u & 63), part = (int)((u >> 6) & 1);
        const int64_t blk = u >> 7;  // nt KB + kb
        const int kb = (int)(blk % KB), nt = (int)(blk / KB);
        const int n = 16 * nt + (lane & 15), k0 = 32 * kb + 8 * (lane >> 4);
        h8 v;
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            const float w = (n < N && k0 + j < K) ? W[(int64_t)n * K + k0 + j] * s : 0.0f;
            const _Float16 hi = (_Float16)w;
            v[j] = part == 0 ? hi : (_Float16)(w - (float)hi);
        }
        body[u] = v;
    }
}

// ---------------------------------------------------------------------------
struct WlGemm {
    const float* pack[2];  // the two groups' packs (s, t)
    const float* xf[2];    // their input fragments: halfs [mt][kb][part][lane][8]
    float* part;           // fp32 partial sums [group][split][row][feature]
    int N, NT, KB;         // features per group, their 16-tiles, k-blocks
    int KS, KC, M, nblk;   // splits, k-blocks per split, rows, feature blocks per group
};

template <int MT, int NTW, int NW, int PF>
__global__ __launch_bounds__(64 * NW, 1) void k_wl_gemm(WlGemm a) {
    constexpr int kWlWaves = NW, kWlPF = PF, kWlRing = PF + 1;
    // the input fragments of k-block kk of the chunk: 2 MT 1-KiB blocks in
    // ring slot kk % kWlRing, copied by LDS-DMA kWlPF k-blocks ahead together
    // with the weights (every wave copies D blocks per step; a wave with fewer
    // distinct blocks re-copies the last one, so every wave's vmcnt is the same)
    constexpr int XB = 2 * MT, D = (XB + kWlWaves - 1) / kWlWaves;
    constexpr int PER = D + 2 * NTW;  // vector-memory operations per wave and step
    extern __shared__ __attribute__((aligned(16))) float4 xs[];  // [kWlRing][XB][64]
    const int lane = threadIdx.x & 63;
    const int wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    int b = blockIdx.x;
    const int ks = b % a.KS;
    b /= a.KS;
    const int nb = b % a.nblk, g = b / a.nblk;
    const int kb0 = ks * a.KC;
    const int nkc = a.KB - kb0 < a.KC ? a.KB - kb0 : a.KC;
    const float4* xg = reinterpret_cast<const float4*>(a.xf[g]);
    const f32x4* wg = reinterpret_cast<const f32x4*>(a.pack[g] + kWlHdr);
    const uint32_t xb = lds_addr(xs);
    const int nt0 = (nb * kWlWaves + wid) * NTW;
    int ntc[NTW];
#pragma unroll
    for (int t = 0; t < NTW; ++t) ntc[t] = nt0 + t < a.NT ? nt0 + t : a.NT - 1;
    // steps past the chunk read the pack's zero block (L2-resident) and re-copy
    // the chunk's last input block: they add zeros, and keep the loop free of
    // branches, so the ring's loads stay in a fixed order the waits count
    const int64_t zoff = (int64_t)a.NT * a.KB * 2 * 64;  // the zero block (f32x4 units)
    f32x4 w[kWlPF][NTW][2];
    auto issue = [&](int kk, f32x4 (&dst)[NTW][2]) {
        const int kx = kk < nkc ? kk : nkc - 1;
        const uint32_t slot = xb + (uint32_t)((kk % kWlRing) * XB * 1024);
#pragma unroll
        for (int d = 0; d < D; ++d) {
            const int blk = wid + kWlWaves * d < XB ? wid + kWlWaves * d : XB - 1;  // (wave-uniform)
            const int s = blk >> 1, part = blk & 1;
            dma16(xg + ((int64_t)(s * a.KB + kb0 + kx) * 2 + part) * 64 + lane, slot + (uint32_t)(blk * 1024));
        }
        // (a wave-uniform offset select, not a branch)
        const int64_t live = kk < nkc ? 1 : 0;
#pragma unroll
        for (int t = 0; t < NTW; ++t) {
            const int64_t off = ((int64_t)ntc[t] * a.KB + kb0 + kk) * 2 * 64;
            const f32x4* p = wg + (zoff + live * (off - zoff)) + lane;
#if NFK_WL_NT
            dst[t][0] = __builtin_nontemporal_load(p);
            dst[t][1] = __builtin_nontemporal_load(p + 64);
#else
            dst[t][0] = p[0];
            dst[t][1] = p[64];
#endif
        }
    };
#pragma unroll
    for (int j = 0; j < kWlPF; ++j) issue(j, w[j]);

    f32x4 acc[NTW][MT];
#pragma unroll
    for (int t = 0; t < NTW; ++t)
#pragma unroll
        for (int s = 0; s < MT; ++s) acc[t][s] = f32x4{0.0f, 0.0f, 0.0f, 0.0f};
    const int nkr = (nkc + kWlPF - 1) / kWlPF * kWlPF;
    for (int k0 = 0; k0 < nkr; k0 += kWlPF) {
#pragma unroll
        for (int j = 0; j < kWlPF; ++j) {
            const int kk = k0 + j;
            // this step's copies and weights landed (the kWlPF - 1 later steps'
            // operations may still be in flight), then every wave's copies
            asm volatile("s_waitcnt vmcnt(%0)" ::"n"((kWlPF - 1) * PER) : "memory");
            __builtin_amdgcn_s_barrier();
            asm volatile("" ::: "memory");
            const float4* f = xs + (kk % kWlRing) * XB * 64 + lane;
            h8 xh[MT], xl[MT];
#pragma unroll
            for (int s = 0; s < MT; ++s) {
                xh[s] = __builtin_bit_cast(h8, f[(2 * s) * 64]);
                xl[s] = __builtin_bit_cast(h8, f[(2 * s + 1) * 64]);
            }
#pragma unroll
            for (int t = 0; t < NTW; ++t) {
                const h8 ah = __builtin_bit_cast(h8, w[j][t][0]), al = __builtin_bit_cast(h8, w[j][t][1]);
#pragma unroll
                for (int s = 0; s < MT; ++s) {
                    acc[t][s] = mfma16(al, xh[s], acc[t][s]);
                    acc[t][s] = mfma16(ah, xl[s], acc[t][s]);
                    acc[t][s] = mfma16(ah, xh[s], acc[t][s]);
                }
            }
            // the slot refilled below was read one step ago: every wave has
            // passed this step's barrier, so its reads of it have returned
            issue(kk + kWlPF, w[j]);
            // (keep the refill here: the scheduler otherwise sinks the ring's
            // loads to the end of the unrolled body and the prefetch depth collapses)
            __builtin_amdgcn_sched_barrier(0);
        }
    }

    // partial sums: lane (q, n) of tile (t, s) holds row 16 s + n, features
    // 16 nt + 4 q .. + 3
    const int q = lane >> 4, n = lane & 15;
    float* P = a.part + (int64_t)(g * a.KS + ks) * a.M * a.N;
#pragma unroll
    for (int t = 0; t < NTW; ++t) {
        if (nt0 + t >= a.NT) continue;
        const int f0 = 16 * (nt0 + t) + 4 * q;
        if (f0 >= a.N) continue;
#pragma unroll
        for (int s = 0; s < MT; ++s) {
            const int m = 16 * s + n;
            if (m < a.M)
                *reinterpret_cast<float4*>(P + (int64_t)m * a.N + f0) =
                    make_float4(acc[t][s][0], acc[t][s][1], acc[t][s][2], acc[t][s][3]);
        }
    }
}

// ---------------------------------------------------------------------------
// GEMM + activation in one launch (hidden layers 1 and 2 at <= 64 rows): a
// workgroup owns TWO output tiles of one group over the WHOLE contraction, its
// 4 waves each a quarter of the k-blocks.  Each wave streams its weights AND
// its input fragments (L2-resident) straight into a register ring PF k-blocks
// deep -- no LDS and no barrier per step -- then the four waves' sums meet in
// LDS, are added in wave order (fixed: deterministic), unscaled, + bias, tanh,
// and written as the next GEMM's fp16 hi/lo fragments.  No split-K partial
// sums and no k_wl_act launch (whose ~6 us, plus a kernel boundary, per stage
// were a sixth of a layer).
struct WlGemmAct {
    const float* pack[2];  // the two groups' packs
    const float* xf[2];    // their input fragments: halfs [mt][kb][part][lane][8]
    const float* bias[2];
    const float* xun;      // per-row input unscale (nullptr: 2^-14, a hidden layer's input)
    float* out[2];         // output fragments [MT][KBo][part][64][8] halfs
    int N, NT, KB, M, KBo, npair;
};

template <int MT, int PF>
__global__ __launch_bounds__(256, 1) void k_wl_gemm_act(WlGemmAct a) {
    constexpr int PER = 4 + 2 * MT;  // vector-memory operations per wave and step
    extern __shared__ __attribute__((aligned(16))) float4 red4[];  // [4 waves][2 tiles][MT][64]
    const int lane = threadIdx.x & 63;
    const int wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int tp = blockIdx.x % a.npair, g = blockIdx.x / a.npair;
    const float4* xg = reinterpret_cast<const float4*>(a.xf[g]);
    const f32x4* wg = reinterpret_cast<const f32x4*>(a.pack[g] + kWlHdr);
    int ntc[2];
#pragma unroll
    for (int t = 0; t < 2; ++t) ntc[t] = 2 * tp + t < a.NT ? 2 * tp + t : a.NT - 1;
    // this wave's k-blocks [kb0, kb0 + nk)
    const int KW = (a.KB + 3) >> 2;
    const int kb0 = wid * KW < a.KB ? wid * KW : a.KB;
    const int nk = a.KB - kb0 < KW ? a.KB - kb0 : KW;
    const int64_t zoff = (int64_t)a.NT * a.KB * 2 * 64;  // the pack's zero block (f32x4 units)
    f32x4 w[PF][2][2];
    float4 x[PF][MT][2];
    auto issue = [&](int kk, f32x4 (&dw)[2][2], float4 (&dx)[MT][2]) {
        // steps past the wave's range: zero weights (the zero block) times a
        // valid input block -- branch-free, so the counted waits stay exact
        const int64_t live = kk < nk ? 1 : 0;
        const int kx = kb0 + (kk < nk ? kk : 0);
#pragma unroll
        for (int t = 0; t < 2; ++t) {
            const int64_t off = ((int64_t)ntc[t] * a.KB + kb0 + kk) * 2 * 64;
            const f32x4* p = wg + (zoff + live * (off - zoff)) + lane;
#if NFK_WL_NT
            dw[t][0] = __builtin_nontemporal_load(p);
            dw[t][1] = __builtin_nontemporal_load(p + 64);
#else
            dw[t][0] = p[0];
            dw[t][1] = p[64];
#endif
        }
#pragma unroll
        for (int s = 0; s < MT; ++s) {
            const float4* f = xg + ((int64_t)(s * a.KB + (kx < a.KB ? kx : a.KB - 1)) * 2) * 64 + lane;
            dx[s][0] = f[0];
            dx[s][1] = f[64];
        }
    };
#pragma unroll
    for (int j = 0; j < PF; ++j) issue(j, w[j], x[j]);
    f32x4 acc[2][MT];
#pragma unroll
    for (int t = 0; t < 2; ++t)
#pragma unroll
        for (int s = 0; s < MT; ++s) acc[t][s] = f32x4{0.0f, 0.0f, 0.0f, 0.0f};
    const int nkr = (KW + PF - 1) / PF * PF;  // (uniform over the workgroup's waves)
    for (int k0 = 0; k0 < nkr; k0 += PF) {
#pragma unroll
        for (int j = 0; j < PF; ++j) {
            asm volatile("s_waitcnt vmcnt(%0)" ::"n"((PF - 1) * PER) : "memory");
            h8 xh[MT], xl[MT];
#pragma unroll
            for (int s = 0; s < MT; ++s) {
                xh[s] = __builtin_bit_cast(h8, x[j][s][0]);
                xl[s] = __builtin_bit_cast(h8, x[j][s][1]);
            }
#pragma unroll
            for (int t = 0; t < 2; ++t) {
                const h8 ah = __builtin_bit_cast(h8, w[j][t][0]), al = __builtin_bit_cast(h8, w[j][t][1]);
#pragma unroll
                for (int s = 0; s < MT; ++s) {
                    acc[t][s] = mfma16(al, xh[s], acc[t][s]);
                    acc[t][s] = mfma16(ah, xl[s], acc[t][s]);
                    acc[t][s] = mfma16(ah, xh[s], acc[t][s]);
                }
            }
            issue(k0 + j + PF, w[j], x[j]);
            __builtin_amdgcn_sched_barrier(0);
        }
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    // the waves' sums through LDS; wave v then finishes the (tile, sample
    // tile) pairs p = v, v + 4, ...: sum over waves 0..3 in order, activation
#pragma unroll
    for (int t = 0; t < 2; ++t)
#pragma unroll
        for (int s = 0; s < MT; ++s)
            red4[((wid * 2 + t) * MT + s) * 64 + lane] = make_float4(acc[t][s][0], acc[t][s][1], acc[t][s][2], acc[t][s][3]);
    __syncthreads();
    const int q = lane >> 4, n = lane & 15;
    for (int pr = wid; pr < 2 * MT; pr += 4) {
        const int t = pr / MT, sm = pr - t * MT, nt = 2 * tp + t;
        if (nt >= 2 * a.KBo) continue;  // (wave-uniform) past the fragments' features
        float4 v = red4[((0 * 2 + t) * MT + sm) * 64 + lane];
#pragma unroll
        for (int wv = 1; wv < 4; ++wv) {
            const float4 o = red4[((wv * 2 + t) * MT + sm) * 64 + lane];
            v.x += o.x, v.y += o.y, v.z += o.z, v.w += o.w;
        }
        const int m = 16 * sm + n, f0 = 16 * nt + 4 * q;
        const float u = a.pack[g][0] * (a.xun != nullptr ? a.xun[m < a.M ? m : 0] : 1.0f / kWlAct);
        const float* bz = a.bias[g];
        const float vv[4] = {v.x, v.y, v.z, v.w};
        _Float16 hi[4], lo[4];
#pragma unroll
        for (int e = 0; e < 4; ++e) {
            float h = 0.0f;
            if (m < a.M && nt < a.NT && f0 + e < a.N) h = tanhf(vv[e] * u + bz[f0 + e]) * kWlAct;
            hi[e] = (_Float16)h;
            lo[e] = (_Float16)(h - (float)hi[e]);
        }
        // feature f0 + e of row m: k-block nt / 2, lane 16 (2 (nt & 1) + q / 2) + n, element 4 (q & 1) + e
        _Float16* o = reinterpret_cast<_Float16*>(a.out[g]) +
                      ((((int64_t)sm * a.KBo + (nt >> 1)) * 2) * 64 + 16 * (2 * (nt & 1) + (q >> 1)) + n) * 8 +
                      4 * (q & 1);
        typedef _Float16 h4v __attribute__((ext_vector_type(4)));
        *reinterpret_cast<h4v*>(o) = h4v{hi[0], hi[1], hi[2], hi[3]};
        *reinterpret_cast<h4v*>(o + 64 * 8) = h4v{lo[0], lo[1], lo[2], lo[3]};
    }
}

// ---------------------------------------------------------------------------
// hidden activations: h = tanh(sum_split P * 2^-s * u_row + b), split at 2^14
// into the next GEMM's fragments.  One thread per (group, row, 8 features)
struct WlAct {
    const float* part;    // [2][KS][M][N]
    const float* pack[2];
    const float* bias[2];
    const float* xun;     // per-row input unscale of the GEMM (nullptr: 2^-14, a hidden layer)
    float* out[2];        // fragments [MT][KBo][part][64][8] halfs
    int N, KS, M, MT, KBo;
};

__global__ __launch_bounds__(256) void k_wl_act(WlAct a) {
    // thread i: group g, row m (padded to 16 MT), features 8 n8 .. + 7, n8
    // fastest: a wave reads 64 consecutive 32-B runs of one partial-sum row
    const int N8 = 4 * a.KBo, RM = 16 * a.MT;
    int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (i >= 2LL * RM * N8) return;
    const int n8 = (int)(i % N8);
    i /= N8;
    const int m = (int)(i % RM), g = (int)(i / RM);
    const int kb = n8 >> 2, q = n8 & 3, f0 = 8 * n8;
    h8 hi, lo;
#pragma unroll
    for (int j = 0; j < 8; ++j) hi[j] = lo[j] = (_Float16)0.0f;
    if (m < a.M) {
        const float u = a.pack[g][0] * (a.xun != nullptr ? a.xun[m] : 1.0f / kWlAct);
        float v[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) v[j] = 0.0f;
        const float* P = a.part + ((int64_t)g * a.KS * a.M + m) * a.N + f0;
        const int64_t st = (int64_t)a.M * a.N;
        if (f0 + 8 <= a.N) {
            // four splits' loads in flight at a time, added in split order
            int ks = 0;
            for (; ks + 4 <= a.KS; ks += 4) {
                float4 u[4][2];
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    u[r][0] = *reinterpret_cast<const float4*>(P + (ks + r) * st);
                    u[r][1] = *reinterpret_cast<const float4*>(P + (ks + r) * st + 4);
                }
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    v[0] += u[r][0].x, v[1] += u[r][0].y, v[2] += u[r][0].z, v[3] += u[r][0].w;
                    v[4] += u[r][1].x, v[5] += u[r][1].y, v[6] += u[r][1].z, v[7] += u[r][1].w;
                }
            }
            for (; ks < a.KS; ++ks) {
                const float4 x0 = *reinterpret_cast<const float4*>(P + ks * st);
                const float4 x1 = *reinterpret_cast<const float4*>(P + ks * st + 4);
                v[0] += x0.x, v[1] += x0.y, v[2] += x0.z, v[3] += x0.w;
                v[4] += x1.x, v[5] += x1.y, v[6] += x1.z, v[7] += x1.w;
            }
        } else {
            for (int ks = 0; ks < a.KS; ++ks)
#pragma unroll
                for (int j = 0; j < 8; ++j)
                    if (f0 + j < a.N) v[j] += P[ks * st + j];
        }
        const float* bz = a.bias[g];
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            if (f0 + j < a.N) {
                const float h = tanhf(v[j] * u + bz[f0 + j]) * kWlAct;
                const _Float16 hh = (_Float16)h;
                hi[j] = hh;
                lo[j] = (_Float16)(h - (float)hh);
            }
        }
    }
    h8* o = reinterpret_cast<h8*>(a.out[g]) + ((int64_t)((m >> 4) * a.KBo + kb) * 2) * 64 + 16 * q + (m & 15);
    o[0] = hi;
    o[64] = lo;
}

// ---------------------------------------------------------------------------
// one workgroup per row: (a) part == nullptr: the row of x as fragments (the
// first half-coupling's input); (b) the affine half-coupling of the row from
// the L3 partial sums (s = group 0, t = group 1), its log|det|, and optionally
// the fragments of the output half (the next half-coupling's input)
struct WlRows {
    const float* part;    // [2][KS][M][h] or nullptr
    const float* pack[2];
    const float* bias[2];
    const float* xin;     // the half being transformed (or split)
    int64_t ldin;
    float* out;           // the transformed half (coupling only)
    int64_t ldo;
    float* logdet;
    int mode, inverse;
    float* frag;          // fragments of the row's values [MT][KBf][part][64][8], or nullptr
    float* frag_un;       // their per-row unscale 2^(e - 14)
    int h, KS, M, MT, KBf;
};

constexpr int kRowThreads = 1024;  // one thread per column at Polymer_rnvp's half of 1024

__global__ __launch_bounds__(kRowThreads) void k_wl_rows(WlRows a) {
    extern __shared__ float rowv[];  // the row's values (h floats) when fragments are written
    __shared__ float red[kRowThreads / 64];
    const int m = blockIdx.x;
    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    const bool live = m < a.M;
    float amax = 0.0f, lsum = 0.0f;
    if (live) {
        const float* xr = a.xin + (int64_t)m * a.ldin;
        if (a.part == nullptr) {
            for (int c = tid; c < a.h; c += kRowThreads) {
                const float v = xr[c];
                rowv[c] = v;
                amax = fmaxf(amax, fabsf(v));
            }
        } else {
            const float us = a.pack[0][0] * (1.0f / kWlAct), ut = a.pack[1][0] * (1.0f / kWlAct);
            const float* Ps = a.part + (int64_t)m * a.h;
            const float* Pt = a.part + ((int64_t)a.KS * a.M + m) * a.h;
            const int64_t st = (int64_t)a.M * a.h;
            float* orow = a.out + (int64_t)m * a.ldo;
            for (int c = tid; c < a.h; c += kRowThreads) {
                float s = 0.0f, t = 0.0f;
                int ks = 0;
                for (; ks + 4 <= a.KS; ks += 4) {  // four splits' loads in flight, added in order
                    float us4[4], ut4[4];
#pragma unroll
                    for (int r = 0; r < 4; ++r) {
                        us4[r] = Ps[(ks + r) * st + c];
                        ut4[r] = Pt[(ks + r) * st + c];
                    }
#pragma unroll
                    for (int r = 0; r < 4; ++r) {
                        s += us4[r];
                        t += ut4[r];
                    }
                }
                for (; ks < a.KS; ++ks) {
                    s += Ps[ks * st + c];
                    t += Pt[ks * st + c];
                }
                s = s * us + a.bias[0][c];
                t = t * ut + a.bias[1][c];
                const float x = xr[c];
                // flows.py:56, 59 (t + x exp(s)) and 69, 72 ((x - t) exp(-s)),
                // each operation rounded (no contraction: -ffp-contract=off)
                const float o = a.inverse ? (x - t) * expf(-s) : t + x * expf(s);
                orow[c] = o;
                lsum += s;
                if (a.frag != nullptr) rowv[c] = o;
                amax = fmaxf(amax, fabsf(o));
            }
        }
    }
    if (a.part != nullptr && a.mode != 0) {
        // sum s over the row: each thread its columns in order, then a fixed tree
#pragma unroll
        for (int off = 32; off > 0; off >>= 1) lsum += __shfl_xor(lsum, off, 64);
        if (lane == 0) red[wid] = lsum;
        __syncthreads();
        if (tid == 0 && live) {
            float tot = 0.0f;
            for (int w = 0; w < kRowThreads / 64; ++w) tot += red[w];
            const float ld = a.inverse ? -tot : tot;
            a.logdet[m] = a.mode == 2 ? a.logdet[m] + ld : ld;
        }
        __syncthreads();
    }
    if (a.frag == nullptr) return;
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) amax = fmaxf(amax, __shfl_xor(amax, off, 64));
    if (lane == 0) red[wid] = amax;
    __syncthreads();
    float mx = 0.0f;
    for (int w = 0; w < kRowThreads / 64; ++w) mx = fmaxf(mx, red[w]);
    int ex = 0;
    if (mx > 0.0f && mx < 3.0e38f) frexpf(mx, &ex);  // mx < 2^ex
    ex = ex < -64 ? -64 : ex;
    const float sc = ldexpf(1.0f, 14 - ex);
    if (tid == 0) a.frag_un[m] = live ? ldexpf(1.0f, ex - 14) : 0.0f;
    const int mt = m >> 4;
    h8* base = reinterpret_cast<h8*>(a.frag);
    for (int u = tid; u < a.KBf * 4; u += kRowThreads) {
        const int kb = u >> 2, q = u & 3, f0 = 32 * kb + 8 * q;
        h8 hi, lo;
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            const float v = (live && f0 + j < a.h) ? rowv[f0 + j] * sc : 0.0f;
            const _Float16 hh = (_Float16)v;
            hi[j] = hh;
            lo[j] = (_Float16)(v - (float)hh);
        }
        const int ln = 16 * q + (m & 15);
        h8* o = base + ((int64_t)(mt * a.KBf + kb) * 2) * 64 + ln;
        o[0] = hi;
        o[64] = lo;
    }
}

// ---------------------------------------------------------------------------
// host: the GEMM stage plan
struct WlPlan {
    int NTW, KS, KC, nblk;
    size_t lds;
};

// GEMM workgroup shape: 0 = 4 waves x 2 tiles x 8 k-blocks in flight (the
// default: 11 / 28 / 12 us for Polymer_rnvp's three stages at 40 rows,
// profiles/r6/), 1 = 8 waves x 1 tile x 16 (16 / 30 / 16 us: slower),
// 2 = 4 x 2 x 10; NFK_WL_CFG selects one for A/B runs (1 and 2 up to 64 rows)
int wl_cfg(int MT) {
    static const int env = [] {
        const char* e = std::getenv("NFK_WL_CFG");
        return e != nullptr ? std::atoi(e) : 0;
    }();
    return MT <= 4 ? env : 0;
}

WlPlan wl_plan(int N, int KB, int MT) {
    // one round of workgroups over the CUs (one workgroup each), as few k
    // splits (partial sums) as that allows
    WlPlan p{};
    const int NT = (N + 15) / 16;
    const int cfg = wl_cfg(MT);
    p.NTW = cfg == 1 ? 1 : 2;
    const int pf = cfg == 1 ? 16 : (cfg == 2 ? 10 : 8);
    p.nblk = (NT + kWlTilesPerWG - 1) / kWlTilesPerWG;
    int ks = kWlTarget / (2 * p.nblk);
    ks = ks < 1 ? 1 : (ks > KB ? KB : ks);
    p.KC = (KB + ks - 1) / ks;
    p.KS = (KB + p.KC - 1) / p.KC;
    // (at least 84 KiB: one workgroup per CU, so the round spreads over every CU)
    p.lds = (size_t)(pf + 1) * 2 * MT * 1024;
    p.lds = p.lds > (size_t)84 * 1024 ? p.lds : (size_t)84 * 1024;
    return p;
}

template <int MT, int NTW, int NW, int PF>
int wl_gemm_launch(const WlGemm& a, const WlPlan& p, hipStream_t st) {
    static bool attr = false;  // (every instance sets its dynamic-LDS cap once)
    if (!attr) {
        (void)hipFuncSetAttribute(reinterpret_cast<const void*>(&k_wl_gemm<MT, NTW, NW, PF>),
                                  hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
        attr = true;
    }
    hipLaunchKernelGGL((k_wl_gemm<MT, NTW, NW, PF>), dim3((unsigned)(2 * p.nblk * p.KS)), dim3(64 * NW), p.lds, st,
                       a);
    return wl_status("nfk_wide_rnvp: GEMM launch");
}

int wl_gemm(const float* const pk[2], const float* const xf[2], float* part, int N, int K, int M, int MT,
            hipStream_t st) {
    const int KB = (K + 31) / 32;
    const WlPlan p = wl_plan(N, KB, MT);
    WlGemm a;
    a.pack[0] = pk[0], a.pack[1] = pk[1];
    a.xf[0] = xf[0], a.xf[1] = xf[1];
    a.part = part;
    a.N = N, a.NT = (N + 15) / 16, a.KB = KB, a.KS = p.KS, a.KC = p.KC, a.M = M, a.nblk = p.nblk;
    const int cfg = wl_cfg(MT);
#define NFK_WL_SMALL(mt)                                                      \
    case mt:                                                                  \
        if (cfg == 1) return wl_gemm_launch<mt, 1, 8, 16>(a, p, st);          \
        if (cfg == 2) return wl_gemm_launch<mt, 2, 4, 10>(a, p, st);          \
        return wl_gemm_launch<mt, 2, 4, 8>(a, p, st);
    switch (MT) {
        NFK_WL_SMALL(1) NFK_WL_SMALL(2) NFK_WL_SMALL(3) NFK_WL_SMALL(4)
#undef NFK_WL_SMALL
        case 5: return wl_gemm_launch<5, 2, 4, 8>(a, p, st);
        case 6: return wl_gemm_launch<6, 2, 4, 8>(a, p, st);
        case 7: return wl_gemm_launch<7, 2, 4, 8>(a, p, st);
        case 8: return wl_gemm_launch<8, 2, 4, 8>(a, p, st);
        default: return nfk_set_error("nfk_wide_rnvp: bad row tile count");
    }
}

// hidden layers' GEMM + activation in one launch (k_wl_gemm_act) up to 64
// rows; NFK_WL_FUSED=0 selects the split-K GEMM + k_wl_act pair (A/B)
bool wl_fused(int MT) {
    static const bool env = [] {
        const char* e = std::getenv("NFK_WL_FUSED");
        return !(e != nullptr && e[0] == '0');
    }();
    return env && MT <= 4;
}

template <int MT, int PF>
int wl_gemm_act_launch(const WlGemmAct& a, hipStream_t st) {
    static bool attr = false;
    if (!attr) {
        (void)hipFuncSetAttribute(reinterpret_cast<const void*>(&k_wl_gemm_act<MT, PF>),
                                  hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
        attr = true;
    }
    // (at least 84 KiB: one workgroup per CU, so the grid spreads over every CU)
    size_t lds = (size_t)4 * 2 * MT * 1024;
    lds = lds > (size_t)84 * 1024 ? lds : (size_t)84 * 1024;
    hipLaunchKernelGGL((k_wl_gemm_act<MT, PF>), dim3((unsigned)(2 * a.npair)), dim3(256), lds, st, a);
    return wl_status("nfk_wide_rnvp: GEMM + activation launch");
}

int wl_gemm_act(const float* const pk[2], const float* const xf[2], const float* const bias[2], const float* xun,
                float* const out[2], int N, int K, int M, int MT, hipStream_t st) {
    WlGemmAct a;
    for (int g = 0; g < 2; ++g) a.pack[g] = pk[g], a.xf[g] = xf[g], a.bias[g] = bias[g], a.out[g] = out[g];
    a.xun = xun;
    a.N = N, a.NT = (N + 15) / 16, a.KB = (K + 31) / 32, a.M = M, a.KBo = (N + 31) / 32;
    a.npair = (a.NT + 1) / 2;
    switch (MT) {
        case 1: return wl_gemm_act_launch<1, 8>(a, st);
        case 2: return wl_gemm_act_launch<2, 8>(a, st);
        case 3: return wl_gemm_act_launch<3, 6>(a, st);
        case 4: return wl_gemm_act_launch<4, 6>(a, st);
        default: return nfk_set_error("nfk_wide_rnvp: bad row tile count for the fused stage");
    }
}

int64_t frag_floats(int MT, int K) { return (int64_t)MT * ((K + 31) / 32) * 512; }

// workspace of one pass of MT sample tiles (floats, each region 16-byte aligned)
struct WlWs {
    float *fx[2], *fun[2], *fh[2][2], *part;
    int64_t total;
};

WlWs wl_ws(float* base, int half, int hidden, int MT) {
    WlWs w{};
    const int M = 16 * MT;
    int64_t off = 0;
    auto take = [&](int64_t n) {
        float* p = base == nullptr ? nullptr : base + off;
        off += (n + 3) / 4 * 4;
        return p;
    };
    for (int i = 0; i < 2; ++i) w.fx[i] = take(frag_floats(MT, half));
    for (int i = 0; i < 2; ++i) w.fun[i] = take(M);
    for (int l = 0; l < 2; ++l)
        for (int g = 0; g < 2; ++g) w.fh[l][g] = take(frag_floats(MT, hidden));
    int64_t pmax = 0;
    const int shapes[3][2] = {{hidden, half}, {hidden, hidden}, {half, hidden}};  // (N, K) per stage
    for (auto& s : shapes) {
        const WlPlan p = wl_plan(s[0], (s[1] + 31) / 32, MT);
        const int64_t n = 2LL * p.KS * M * s[0];
        pmax = n > pmax ? n : pmax;
    }
    w.part = take(pmax);
    w.total = off;
    return w;
}

}  // namespace

extern "C" int64_t nfk_wlin_pack_floats(int32_t N, int32_t K) {
    if (N <= 0 || K <= 0) return 0;
    // header, the fragment blocks, one zero block (the GEMM's steps past a chunk)
    return kWlHdr + (int64_t)((N + 15) / 16) * ((K + 31) / 32) * 512 + 512;
}

extern "C" int nfk_wlin_pack(const float* W, int32_t N, int32_t K, float* pack, nfk_stream_t stream) {
    if (nfk_wlin_pack_floats(N, K) == 0) return nfk_set_error("nfk_wlin_pack: bad shape");
    if (!W || !pack) return nfk_set_error("nfk_wlin_pack: null pointer");
    hipStream_t st = (hipStream_t)stream;
    const int64_t body = (int64_t)((N + 15) / 16) * ((K + 31) / 32) * 512;
    if (hipMemsetAsync(pack, 0, kWlHdr * sizeof(float), st) != hipSuccess ||
        hipMemsetAsync(pack + kWlHdr + body, 0, 512 * sizeof(float), st) != hipSuccess)
        return nfk_set_error("nfk_wlin_pack: memset failed");
    const int64_t n = (int64_t)N * K;
    const int64_t gm = (n + 4095) / 4096;
    hipLaunchKernelGGL(k_wl_max, dim3((unsigned)(gm < 1024 ? gm : 1024)), dim3(256), 0, st, W, n, pack);
    const int KB = (K + 31) / 32;
    const int64_t units = (int64_t)((N + 15) / 16) * KB * 128;
    const int64_t gp = (units + 255) / 256;
    hipLaunchKernelGGL(k_wl_pack, dim3((unsigned)(gp < 8192 ? gp : 8192)), dim3(256), 0, st, W, N, K, KB, units, pack);
    return wl_status("nfk_wlin_pack");
}

extern "C" int nfk_wide_rnvp_supported(int32_t half, int32_t hidden) {
    return (half >= 4 && half % 4 == 0 && half <= 16384 && hidden >= 16 && hidden % 4 == 0 && hidden <= 16384) ? 1 : 0;
}

extern "C" int64_t nfk_wide_rnvp_workspace(int32_t half, int32_t hidden, int64_t batch) {
    if (!nfk_wide_rnvp_supported(half, hidden) || batch <= 0) return 0;
    const int64_t mt = (batch + 15) / 16;
    return wl_ws(nullptr, half, hidden, (int)(mt < kWlMaxMT ? mt : kWlMaxMT)).total;
}

namespace {

// nl layers in execution order (packs / biases: 12 per layer), each layer's
// half-couplings in its direction.  Within a row block the layers run back to
// back: layer l reads the previous layer's output rows (ping-ponged through
// tmp, the last layer writing z), and the last coupling of every layer but
// the last also writes the fragments of its output half -- the next layer's
// first conditioner input -- so only the first layer converts x (no per-layer
// k_wl_rows prep launch).
int wl_layers(const float* x, int64_t ldx, const float* const* packs, const float* const* biases, int nl, int h,
              int H, float* z, int64_t ldz, float* logdet, int logdet_mode, int64_t batch, bool inverse,
              float* workspace, float* tmp, hipStream_t st) {
    for (int64_t r0 = 0; r0 < batch; r0 += 16 * kWlMaxMT) {
        const int M = (int)(batch - r0 < 16 * kWlMaxMT ? batch - r0 : 16 * kWlMaxMT);
        const int MT = (M + 15) / 16;
        const WlWs w = wl_ws(workspace, h, H, MT);
        float* ldr = logdet_mode != 0 ? logdet + r0 : nullptr;
        const int first = inverse ? 1 : 0;
        for (int l = 0; l < nl; ++l) {
            // layer l's input and output rows of this block
            const float* xr;
            int64_t ldxr;
            if (l == 0) {
                xr = x + r0 * ldx, ldxr = ldx;
            } else {
                const bool prev_z = ((nl - 1 - (l - 1)) & 1) == 0;
                xr = prev_z ? z + r0 * ldz : tmp, ldxr = prev_z ? ldz : 2 * h;
            }
            const bool out_z = ((nl - 1 - l) & 1) == 0;
            float* zr = out_z ? z + r0 * ldz : tmp;
            const int64_t ldzr = out_z ? ldz : 2 * h;
            const float* const* lp = packs + 12 * l;
            const float* const* lb = biases + 12 * l;
            if (l == 0) {
                // the first conditioner's input: x's lower half (forward) or upper (inverse)
                WlRows a{};
                a.xin = xr + (first == 0 ? 0 : h);
                a.ldin = ldxr;
                a.frag = w.fx[0];
                a.frag_un = w.fun[0];
                a.h = h, a.M = M, a.MT = MT, a.KBf = (h + 31) / 32;
                hipLaunchKernelGGL(k_wl_rows, dim3(16 * MT), dim3(kRowThreads), (size_t)h * sizeof(float), st, a);
                if (int e = wl_status("nfk_wide_rnvp: rows launch")) return e;
            }
            for (int step = 0; step < 2; ++step) {
                const int c = inverse ? 1 - step : step;
                const float* const* pk = lp + 6 * c;
                const float* const* bs = lb + 6 * c;
                const int fi = step;  // this coupling's input fragments
                // L1: [M, h] -> [M, H] (s and t), + b1, tanh
                if (wl_fused(MT)) {
                    const float* p2[2] = {pk[0], pk[1]};
                    const float* x2[2] = {w.fx[fi], w.fx[fi]};
                    const float* b2[2] = {bs[0], bs[1]};
                    float* o2[2] = {w.fh[0][0], w.fh[0][1]};
                    if (int e = wl_gemm_act(p2, x2, b2, w.fun[fi], o2, H, h, M, MT, st)) return e;
                } else {
                    const float* p2[2] = {pk[0], pk[1]};
                    const float* x2[2] = {w.fx[fi], w.fx[fi]};
                    if (int e = wl_gemm(p2, x2, w.part, H, h, M, MT, st)) return e;
                    const WlPlan p = wl_plan(H, (h + 31) / 32, MT);
                    WlAct a{};
                    a.part = w.part, a.pack[0] = pk[0], a.pack[1] = pk[1], a.bias[0] = bs[0], a.bias[1] = bs[1];
                    a.xun = w.fun[fi], a.out[0] = w.fh[0][0], a.out[1] = w.fh[0][1];
                    a.N = H, a.KS = p.KS, a.M = M, a.MT = MT, a.KBo = (H + 31) / 32;
                    const int64_t n = 2LL * MT * a.KBo * 64;
                    hipLaunchKernelGGL(k_wl_act, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, a);
                    if (int e = wl_status("nfk_wide_rnvp: act launch")) return e;
                }
                // L2: [M, H] -> [M, H], + b2, tanh
                if (wl_fused(MT)) {
                    const float* p2[2] = {pk[2], pk[3]};
                    const float* x2[2] = {w.fh[0][0], w.fh[0][1]};
                    const float* b2[2] = {bs[2], bs[3]};
                    float* o2[2] = {w.fh[1][0], w.fh[1][1]};
                    if (int e = wl_gemm_act(p2, x2, b2, nullptr, o2, H, H, M, MT, st)) return e;
                } else {
                    const float* p2[2] = {pk[2], pk[3]};
                    const float* x2[2] = {w.fh[0][0], w.fh[0][1]};
                    if (int e = wl_gemm(p2, x2, w.part, H, H, M, MT, st)) return e;
                    const WlPlan p = wl_plan(H, (H + 31) / 32, MT);
                    WlAct a{};
                    a.part = w.part, a.pack[0] = pk[2], a.pack[1] = pk[3], a.bias[0] = bs[2], a.bias[1] = bs[3];
                    a.xun = nullptr, a.out[0] = w.fh[1][0], a.out[1] = w.fh[1][1];
                    a.N = H, a.KS = p.KS, a.M = M, a.MT = MT, a.KBo = (H + 31) / 32;
                    const int64_t n = 2LL * MT * a.KBo * 64;
                    hipLaunchKernelGGL(k_wl_act, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, a);
                    if (int e = wl_status("nfk_wide_rnvp: act launch")) return e;
                }
                // L3: [M, H] -> [M, h] (s, t), + b3; the coupling of the other half
                {
                    const float* p2[2] = {pk[4], pk[5]};
                    const float* x2[2] = {w.fh[1][0], w.fh[1][1]};
                    if (int e = wl_gemm(p2, x2, w.part, h, H, M, MT, st)) return e;
                    const WlPlan p = wl_plan(h, (H + 31) / 32, MT);
                    const int col = c == 0 ? h : 0;  // the half this coupling changes
                    WlRows a{};
                    a.part = w.part, a.pack[0] = pk[4], a.pack[1] = pk[5], a.bias[0] = bs[4], a.bias[1] = bs[5];
                    a.xin = xr + col, a.ldin = ldxr, a.out = zr + col, a.ldo = ldzr;
                    a.logdet = ldr;
                    a.mode = ldr == nullptr ? 0 : (step == 0 && l == 0 ? logdet_mode : 2);
                    a.inverse = inverse ? 1 : 0;
                    // the first coupling's output is the second one's input; the
                    // second's, the next layer's first input
                    const bool fr = step == 0 || l + 1 < nl;
                    a.frag = step == 0 ? w.fx[1] : (fr ? w.fx[0] : nullptr);
                    a.frag_un = step == 0 ? w.fun[1] : (fr ? w.fun[0] : nullptr);
                    a.h = h, a.KS = p.KS, a.M = M, a.MT = MT, a.KBf = (h + 31) / 32;
                    hipLaunchKernelGGL(k_wl_rows, dim3(16 * MT), dim3(kRowThreads), fr ? (size_t)h * sizeof(float) : 0,
                                       st, a);
                    if (int e = wl_status("nfk_wide_rnvp: coupling launch")) return e;
                }
            }
        }
    }
    return 0;
}

int wl_check(int32_t half, int32_t hidden, int64_t batch, const float* x, const float* const* packs,
             const float* const* biases, int nl, float* z, float* logdet, int32_t logdet_mode, int64_t ldx,
             int64_t ldz, const float* workspace) {
    if (!nfk_wide_rnvp_supported(half, hidden)) return nfk_set_error("nfk_wide_rnvp: shape not supported");
    if (batch < 0 || nl < 1) return nfk_set_error("nfk_wide_rnvp: bad batch or layer count");
    if (!x || !packs || !biases || !z || !workspace) return nfk_set_error("nfk_wide_rnvp: null pointer");
    if (logdet_mode != 0 && !logdet) return nfk_set_error("nfk_wide_rnvp: null logdet");
    if (ldx < 2 * half || ldz < 2 * half) return nfk_set_error("nfk_wide_rnvp: bad leading dimension");
    for (int i = 0; i < 12 * nl; ++i)
        if (!packs[i] || !biases[i]) return nfk_set_error("nfk_wide_rnvp: null pack or bias");
    return 0;
}

}  // namespace

extern "C" int nfk_wide_rnvp(const float* x, int64_t ldx, const float* const* packs, const float* const* biases,
                             int32_t half, int32_t hidden, float* z, int64_t ldz, float* logdet, int32_t logdet_mode,
                             int64_t batch, int32_t inverse, float* workspace, int64_t workspace_floats,
                             nfk_stream_t stream) {
    if (int e = wl_check(half, hidden, batch, x, packs, biases, 1, z, logdet, logdet_mode, ldx, ldz, workspace))
        return e;
    if (batch == 0) return 0;
    if (workspace_floats < nfk_wide_rnvp_workspace(half, hidden, batch))
        return nfk_set_error("nfk_wide_rnvp: workspace too small (nfk_wide_rnvp_workspace)");
    return wl_layers(x, ldx, packs, biases, 1, half, hidden, z, ldz, logdet, logdet_mode, batch, inverse != 0,
                     workspace, nullptr, (hipStream_t)stream);
}

extern "C" int64_t nfk_wide_rnvp_chain_workspace(int32_t half, int32_t hidden, int64_t batch) {
    const int64_t w = nfk_wide_rnvp_workspace(half, hidden, batch);
    return w == 0 ? 0 : w + (int64_t)16 * kWlMaxMT * 2 * half;  // + one row block's ping-pong rows
}

extern "C" int nfk_wide_rnvp_chain(const float* x, int64_t ldx, const float* const* packs, const float* const* biases,
                                   int32_t nlayers, int32_t half, int32_t hidden, float* z, int64_t ldz, float* logdet,
                                   int32_t logdet_mode, int64_t batch, int32_t inverse, float* workspace,
                                   int64_t workspace_floats, nfk_stream_t stream) {
    if (int e = wl_check(half, hidden, batch, x, packs, biases, nlayers, z, logdet, logdet_mode, ldx, ldz, workspace))
        return e;
    if (batch == 0) return 0;
    if (workspace_floats < nfk_wide_rnvp_chain_workspace(half, hidden, batch))
        return nfk_set_error("nfk_wide_rnvp_chain: workspace too small (nfk_wide_rnvp_chain_workspace)");
    float* tmp = workspace + nfk_wide_rnvp_workspace(half, hidden, batch);
    return wl_layers(x, ldx, packs, biases, nlayers, half, hidden, z, ldz, logdet, logdet_mode, batch, inverse != 0,
                     workspace, tmp, (hipStream_t)stream);
}
