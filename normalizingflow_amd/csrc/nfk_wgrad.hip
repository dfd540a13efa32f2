// nfk_wgrad.hip -- weight-gradient GEMMs of the FCNN conditioner's backward
// (nf/flows.py:20-35 differentiated, applications/src/train.py:26): for an
// nn.Linear with input activations h [B, N] (with the bias column of ones,
// [h | 1]) and output gradient g [B, M],
//
//   dW[i, j] = sum_b g[b, i] h[b, j]            (the reduction runs over the batch)
//
// split over the batch into slices whose partial products the host sums in a
// fixed order (deterministic).  At c3 the largest is the output Linear's
// M = 736 (32 coordinates x 23 spline logits), N = 101 at B = 2^20.
//
// Arithmetic: bf16 three-way split on v_mfma_f32_16x16x32_bf16 with fp32
// accumulation.  x = hi + mid + lo (bf16 each, the two subtractions exact in
// fp32), and the six products hi.hi, hi.mid, mid.hi, mid.mid, hi.lo, lo.hi
// leave out terms of relative size <= 2^-24: fp32-level products with
// bf16's 8-bit exponent, so no scaling of the (often tiny) gradients.
//
// Layout: the contraction index is the batch row, which every MFMA operand
// holds 8 consecutive of per lane (A[i][k = 8 (l >> 4) + e], B[k][j]), so the
// fragments are gathered by 4-byte loads (one row per load, 16 consecutive
// columns per lane group: 64-B segments).  A wave owns TM = 4 M-tiles and
// every N-tile (NT <= 8) of one batch slice; a 4-wave workgroup 16 M-tiles.
// The workgroups of one slice are placed on one XCD (blockIdx mod 8), so h's
// rows, read by each of them, come from that XCD's L2.
#include <hip/hip_runtime.h>

#include <cstdio>

#include "../../include/nfk.h"

int nfk_set_error(const char* msg);

namespace {

typedef __bf16 bf8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

constexpr int kTM = 4;       // M-tiles per wave
constexpr int kWaves = 4;    // waves per workgroup
constexpr int kMaxNT = 8;    // N <= 128
constexpr int kXcds = 8;

__device__ __forceinline__ f32x4 mfma_bf(bf8 a, bf8 b, f32x4 c) {
    return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
}

// v (8 fp32) -> three bf16 fragments with v = hi + mid + lo to 24 bits
__device__ __forceinline__ void split3(const float (&v)[8], bf8& hi, bf8& mid, bf8& lo) {
#pragma unroll
    for (int e = 0; e < 8; ++e) {
        const __bf16 a = (__bf16)v[e];
        const float r1 = v[e] - (float)a;
        const __bf16 b = (__bf16)r1;
        const float r2 = r1 - (float)b;
        hi[e] = a;
        mid[e] = b;
        lo[e] = (__bf16)r2;
    }
}

template <int NT>
__global__ __launch_bounds__(64 * kWaves, 2) void k_wgrad(const float* __restrict__ g, int64_t ldg,
                                                         const float* __restrict__ h, int64_t ldh, int64_t batch,
                                                         int M, int N, int64_t rows_per_slice, int nslices,
                                                         int mblocks, float* __restrict__ part) {
    // XCD-aware placement: workgroup b runs on XCD b % 8; the mblocks
    // workgroups of one slice take the same residue
    const int b = blockIdx.x;
    const int xcd = b % kXcds, r = b / kXcds;
    const int slice = (r / mblocks) * kXcds + xcd;
    const int mb = r % mblocks;
    if (slice >= nslices) return;
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    const int q = lane >> 4, c16 = lane & 15;
    const int tile0 = (mb * kWaves + wid) * kTM;  // first M-tile of this wave
    const int64_t r0 = (int64_t)slice * rows_per_slice;
    const int64_t r1 = r0 + rows_per_slice < batch ? r0 + rows_per_slice : batch;

    f32x4 acc[kTM][NT];
#pragma unroll
    for (int t = 0; t < kTM; ++t)
#pragma unroll
        for (int n = 0; n < NT; ++n) acc[t][n] = f32x4{0.f, 0.f, 0.f, 0.f};

    bool mok[kTM];
#pragma unroll
    for (int t = 0; t < kTM; ++t) mok[t] = 16 * (tile0 + t) + c16 < M;
    bool nok[NT];
#pragma unroll
    for (int n = 0; n < NT; ++n) nok[n] = 16 * n + c16 < N;

    for (int64_t k0 = r0; k0 < r1; k0 += 32) {
        const int64_t kr = k0 + 8 * q;  // this lane's first row of the k-step
        // A fragments: g[kr + e][16 (tile0 + t) + c16]
        bf8 ah[kTM], am[kTM], al[kTM];
#pragma unroll
        for (int t = 0; t < kTM; ++t) {
            float v[8];
            const float* src = g + kr * ldg + 16 * (tile0 + t) + c16;
#pragma unroll
            for (int e = 0; e < 8; ++e) v[e] = (mok[t] && kr + e < r1) ? src[e * ldg] : 0.0f;
            split3(v, ah[t], am[t], al[t]);
        }
#pragma unroll
        for (int n = 0; n < NT; ++n) {
            float v[8];
            const float* src = h + kr * ldh + 16 * n + c16;
#pragma unroll
            for (int e = 0; e < 8; ++e) v[e] = (nok[n] && kr + e < r1) ? src[e * ldh] : 0.0f;
            bf8 bh, bm, bl;
            split3(v, bh, bm, bl);
#pragma unroll
            for (int t = 0; t < kTM; ++t) {
                // small terms first
                acc[t][n] = mfma_bf(al[t], bh, acc[t][n]);
                acc[t][n] = mfma_bf(ah[t], bl, acc[t][n]);
                acc[t][n] = mfma_bf(am[t], bm, acc[t][n]);
                acc[t][n] = mfma_bf(am[t], bh, acc[t][n]);
                acc[t][n] = mfma_bf(ah[t], bm, acc[t][n]);
                acc[t][n] = mfma_bf(ah[t], bh, acc[t][n]);
            }
        }
    }
    // C/D: column (n) = lane & 15, row (m) = 4 (lane >> 4) + e
    float* out = part + (int64_t)slice * M * N;
#pragma unroll
    for (int t = 0; t < kTM; ++t) {
#pragma unroll
        for (int n = 0; n < NT; ++n) {
            const int j = 16 * n + c16;
            if (j >= N) continue;
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                const int i = 16 * (tile0 + t) + 4 * q + e;
                if (i < M) out[(int64_t)i * N + j] = acc[t][n][e];
            }
        }
    }
}

int launch_status(const char* what) {
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) {
        char buf[200];
        std::snprintf(buf, sizeof(buf), "%s: %s", what, hipGetErrorString(e));
        nfk_set_error(buf);
        return (int)e;
    }
    return 0;
}

}  // namespace

extern "C" int nfk_wgrad_supported(int32_t M, int32_t N) {
    return (M >= 1 && M <= 4096 && N >= 1 && N <= 16 * kMaxNT) ? 1 : 0;
}

extern "C" int nfk_wgrad(const float* g, int64_t ldg, const float* h, int64_t ldh, int64_t batch, int32_t M,
                         int32_t N, int64_t rows_per_slice, int32_t nslices, float* partial,
                         nfk_stream_t stream) {
    if (!nfk_wgrad_supported(M, N)) return nfk_set_error("nfk_wgrad: shape not supported (M <= 4096, N <= 128)");
    if (batch < 0 || nslices < 1 || rows_per_slice < 32 || rows_per_slice % 32 != 0 ||
        (int64_t)nslices * rows_per_slice < batch)
        return nfk_set_error("nfk_wgrad: slices must cover the batch in multiples of 32 rows");
    if (!g || !h || !partial) return nfk_set_error("nfk_wgrad: null pointer");
    if (ldg < M || ldh < N) return nfk_set_error("nfk_wgrad: leading dimension smaller than the row");
    const int mtiles = (M + 15) / 16;
    const int mblocks = (mtiles + kWaves * kTM - 1) / (kWaves * kTM);
    // slices rounded up to a multiple of the XCD count so every residue class
    // holds whole slices; the extra workgroups return at once
    const int sgroups = (nslices + kXcds - 1) / kXcds;
    const dim3 grid((unsigned)(sgroups * mblocks * kXcds)), block(64 * kWaves);
    hipStream_t st = (hipStream_t)stream;
    const int NT = (N + 15) / 16;
    switch (NT) {
#define NFK_WG_CASE(n)                                                                                     \
    case n:                                                                                                \
        k_wgrad<n><<<grid, block, 0, st>>>(g, ldg, h, ldh, batch, M, N, rows_per_slice, nslices, mblocks, \
                                           partial);                                                       \
        break;
        NFK_WG_CASE(1) NFK_WG_CASE(2) NFK_WG_CASE(3) NFK_WG_CASE(4)
        NFK_WG_CASE(5) NFK_WG_CASE(6) NFK_WG_CASE(7) NFK_WG_CASE(8)
#undef NFK_WG_CASE
        default:
            return nfk_set_error("nfk_wgrad: N out of range");
    }
    return launch_status("nfk_wgrad");
}
