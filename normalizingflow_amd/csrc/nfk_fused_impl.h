// nfk_fused_impl.h -- fused NSF coupling-layer kernel; design notes in nfk_fused.hip.
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>

#include "../../include/nfk.h"
#include "nfk_spline.h"

typedef float f32x4 __attribute__((ext_vector_type(4)));

namespace nfk_fused {

constexpr int kWaves = 4;  // waves per workgroup (one per SIMD; two workgroups per CU)
constexpr int kMaxD = 256; // n_lo + n_up staged in LDS (4 waves x 16 rows x (2D+1) floats)
constexpr int kPF = 2;             // weight prefetch distance (k-steps)

struct Layout {  // packed-weight layout, all offsets in floats
    int n_lo, n_up, H, K, P, HT, KS1, KSH, NCH, TGH, TGK, TGD;
    int64_t o_w1, o_b1, o_w2, o_b2, o_w3, o_b3, total, w3_chunk, b3_chunk;
};

// W1 [KS1][TGH][64][4] | b1 [HT*16] | W2 [KSH][TGH][64][4] | b2 [HT*16] |
// W3 [NCH][phase W,H,D][KSH][groups][64][4] | b3 [NCH][P][64][4]
inline Layout make_layout(int n_lo, int n_up, int H, int K) {
    Layout L;
    L.n_lo = n_lo;
    L.n_up = n_up;
    L.H = H;
    L.K = K;
    L.P = 3 * K - 1;
    L.HT = (H + 15) / 16;
    L.KS1 = (n_lo + 3) / 4;
    L.KSH = (H + 3) / 4;
    L.NCH = (n_up + 15) / 16;
    L.TGH = (L.HT + 3) / 4;
    L.TGK = (K + 3) / 4;
    L.TGD = (K - 1 + 3) / 4;
    int64_t o = 0;
    L.o_w1 = o;
    o += (int64_t)L.KS1 * L.TGH * 256;
    L.o_b1 = o;
    o += L.HT * 16;
    L.o_w2 = o;
    o += (int64_t)L.KSH * L.TGH * 256;
    L.o_b2 = o;
    o += L.HT * 16;
    L.w3_chunk = (int64_t)L.KSH * (2 * L.TGK + L.TGD) * 256;
    L.o_w3 = o;
    o += L.NCH * L.w3_chunk;
    L.b3_chunk = (int64_t)L.P * 256;
    L.o_b3 = o;
    o += L.NCH * L.b3_chunk;
    L.total = o;
    return L;
}

// hidden feature held by MFMA row i (0..15) of tile t
__host__ __device__ inline int hid_row(int t, int i) { return 16 * t + 4 * (i & 3) + (i >> 2); }

struct FusedArgs {
    const float* x;
    const float *w1, *b1, *w2, *b2, *w3, *b3;
    const int32_t *up_in, *up_out, *lo_in, *lo_out;
    float* z;
    float* logdet;
    int32_t* status;
    int64_t ldx, ldz, batch;
    int32_t w3_chunk, b3_chunk;  // floats per coordinate chunk
    int32_t n_lo, n_up, KS1, NCH, mode;
    NfkSplineConst c;
};

__device__ __forceinline__ f32x4 mfma(float a, float b, f32x4 c) {
    return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
}

__device__ __forceinline__ float pick4(const float4& w, int e) {
    return e == 0 ? w.x : e == 1 ? w.y : e == 2 ? w.z : w.w;
}

// ---------------------------------------------------------------------------
// weight streaming: A fragments of KS k-steps (NG float4 groups = 4 tiles
// each per k-step) flow through a register ring kPF k-steps deep.
// ring_fill issues the first k-steps (called one segment ahead, so the loads
// land while the wave runs VALU work); gemm_ring consumes the ring and keeps
// it topped up.  B fragment of k-step ks = act[ks>>2][ks&3].
template <int KS, int NG, int NGR>
__device__ __forceinline__ void ring_fill(const float4* __restrict__ wp, int lane,
                                          float4 (&ring)[kPF][NGR]) {
    constexpr int PF = KS < kPF ? KS : kPF;
#pragma unroll
    for (int p = 0; p < PF; ++p)
#pragma unroll
        for (int g = 0; g < NG; ++g) ring[p][g] = wp[(p * NG + g) * 64 + lane];
}

template <int KS, int NT, int NG, int NGR, int HTA>
__device__ __forceinline__ void gemm_ring(const f32x4 (&act)[HTA], const float4* __restrict__ wp,
                                          int lane, float4 (&ring)[kPF][NGR], f32x4 (&acc)[NT]) {
    constexpr int PF = KS < kPF ? KS : kPF;
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) {
        float4 cur[NG];
#pragma unroll
        for (int g = 0; g < NG; ++g) cur[g] = ring[ks % PF][g];
        if (ks + PF < KS) {
#pragma unroll
            for (int g = 0; g < NG; ++g) ring[ks % PF][g] = wp[((ks + PF) * NG + g) * 64 + lane];
        }
        // keep the refill of k-step ks+PF ahead of k-step ks's MFMAs (the
        // scheduler otherwise sinks the loads next to their use)
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int g = 0; g < NG; ++g) {
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                const int t = 4 * g + e;
                if (t < NT) acc[t] = mfma(pick4(cur[g], e), act[ks >> 2][ks & 3], acc[t]);
            }
        }
    }
}

template <int NT>
__device__ __forceinline__ void zero_acc(f32x4 (&acc)[NT]) {
#pragma unroll
    for (int t = 0; t < NT; ++t) acc[t] = f32x4{0.0f, 0.0f, 0.0f, 0.0f};
}

// acc += packed bias (one float4 per tile and lane), at the start of a VALU segment
template <int NT>
__device__ __forceinline__ void add_bias(const float4* __restrict__ bp, int lane, f32x4 (&acc)[NT]) {
    float4 b[NT];
#pragma unroll
    for (int t = 0; t < NT; ++t) b[t] = bp[t * 64 + lane];
#pragma unroll
    for (int t = 0; t < NT; ++t) {
        acc[t][0] = acc[t][0] + b[t].x;
        acc[t][1] = acc[t][1] + b[t].y;
        acc[t][2] = acc[t][2] + b[t].z;
        acc[t][3] = acc[t][3] + b[t].w;
    }
}

// Knot phase epilogue: for the 4 coordinates of this lane, normalise the K
// logits of register r (NSF_CL's 2B*softmax, then RQS's own softmax + floor +
// cumsum), optionally search the bin of x, and keep (edge_k, size_k).
template <int K, bool SEARCH, bool Y>
__device__ __forceinline__ void knot_phase(const f32x4 (&acc)[K], const float (&xv)[4],
                                           const NfkSplineConst& c, int (&kb)[4], float (&ek)[4],
                                           float (&sk)[4]) {
#pragma unroll
    for (int r = 0; r < 4; ++r) {
        float u[K], edge[K + 1];
#pragma unroll
        for (int t = 0; t < K; ++t) u[t] = acc[t][r];
        nfk_softmax<K, true>(u);
#pragma unroll
        for (int t = 0; t < K; ++t) u[t] = c.scale2b * u[t];
        if (Y)
            nfk_knots<K, true>(u, c.ylo, c.yhi, c.yspan, c.min_h, c.fh, edge);
        else
            nfk_knots<K, true>(u, c.lo, c.hi, c.span, c.min_w, c.fw, edge);
        if (SEARCH) kb[r] = nfk_bin<K>(edge, xv[r], c.knot_eps);
        const int k = kb[r];
        float e = edge[0], w = edge[1] - edge[0];
#pragma unroll
        for (int jj = 1; jj < K; ++jj)
            if (k == jj) {
                e = edge[jj];
                w = edge[jj + 1] - edge[jj];
            }
        ek[r] = e;
        sk[r] = w;
#ifdef NFK_PAIR_FENCE
        __builtin_amdgcn_sched_barrier(0);  // one pair at a time: bounds live registers
#endif
    }
}

// One wave = 16 samples, free-running (no inter-wave synchronisation after
// the x tile is staged).  Measured on gfx950 (tools/ubench_coexec.hip): fp32
// MFMA and VALU instructions of two waves on one SIMD do NOT co-execute (the
// f32 MFMA runs at the vector datapath's rate), so layer time ~ MFMA cycles +
// epilogue VALU cycles; the epilogue therefore uses the short-sequence
// transcendentals of nfk_spline.h.
template <int KSH, int K, bool INV>
__global__ __launch_bounds__(64 * kWaves, 2) void k_fused_nsf(FusedArgs a) {
    constexpr int HT = (KSH + 3) / 4;
    constexpr int TGH = (HT + 3) / 4;
    constexpr int TGK = (K + 3) / 4;
    constexpr int TGD = (K - 1 + 3) / 4;
    constexpr int DN = K - 1 > 0 ? K - 1 : 1;
    const int lane = threadIdx.x & 63;
    const int wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int q = lane >> 4, sl = lane & 15;
    const int D = a.n_lo + a.n_up;
    const int XS = D + 1;
    extern __shared__ __attribute__((aligned(16))) float lds[];
    float* xt = lds + wid * 16 * (XS + D);
    float* zt = xt + 16 * XS;
    const int64_t b0 = ((int64_t)blockIdx.x * kWaves + wid) * 16;
    const int64_t rem = a.batch - b0;
    const int nrows = rem <= 0 ? 0 : (rem < 16 ? (int)rem : 16);
    const NfkSplineConst& c = a.c;

    // ---- stage this wave's x rows (full-row coalesced loads)
    for (int r = 0; r < 16; ++r)
        for (int cc = lane; cc < D; cc += 64) xt[r * XS + cc] = (r < nrows) ? a.x[(b0 + r) * a.ldx + cc] : 0.0f;
    __syncthreads();

    // ---- hidden layers
    f32x4 h1[HT];
#pragma unroll
    for (int t = 0; t < HT; ++t) {
#pragma unroll
        for (int r = 0; r < 4; ++r) h1[t][r] = a.b1[16 * t + 4 * r + q];
    }
    {
        const float4* wp = reinterpret_cast<const float4*>(a.w1);
        for (int ks = 0; ks < a.KS1; ++ks) {
            const int k = 4 * ks + q;
            const int col = (k < a.n_lo) ? a.lo_in[k] : -1;
            const float bf = (col >= 0) ? xt[sl * XS + col] : 0.0f;
#pragma unroll
            for (int g = 0; g < TGH; ++g) {
                const float4 w = wp[(ks * TGH + g) * 64 + lane];
#pragma unroll
                for (int e = 0; e < 4; ++e) {
                    const int t = 4 * g + e;
                    if (t < HT) h1[t] = mfma(pick4(w, e), bf, h1[t]);
                }
            }
        }
    }
#pragma unroll
    for (int t = 0; t < HT; ++t)
#pragma unroll
        for (int r = 0; r < 4; ++r) h1[t][r] = tanhf(h1[t][r]);
    f32x4 h2[HT];
#pragma unroll
    for (int t = 0; t < HT; ++t) {
#pragma unroll
        for (int r = 0; r < 4; ++r) h2[t][r] = a.b2[16 * t + 4 * r + q];
    }
    {
        float4 ring2[kPF][TGH];
        ring_fill<KSH, TGH, TGH>(reinterpret_cast<const float4*>(a.w2), lane, ring2);
        gemm_ring<KSH, HT, TGH, TGH, HT>(h1, reinterpret_cast<const float4*>(a.w2), lane, ring2, h2);
    }
#pragma unroll
    for (int t = 0; t < HT; ++t)
#pragma unroll
        for (int r = 0; r < 4; ++r) h2[t][r] = tanhf(h2[t][r]);

    const int w3_phase = KSH * TGK * 64;  // float4s per W/H phase
    float4 ring[kPF][TGK];
    {
        const float4* w3 = reinterpret_cast<const float4*>(a.w3);
        ring_fill<KSH, TGK, TGK>(INV ? w3 + w3_phase : w3, lane, ring);
    }

    float ldsum = 0.0f;
    bool any_in = false, any_nd = false;
    for (int ch = 0; ch < a.NCH; ++ch) {
        const int jbase = 16 * ch;
        const float4* w3 = reinterpret_cast<const float4*>(a.w3 + (int64_t)ch * a.w3_chunk);
        const float4* wW = w3;
        const float4* wH = w3 + w3_phase;
        const float4* wD = w3 + 2 * w3_phase;
        const float4* b3 = reinterpret_cast<const float4*>(a.b3 + (int64_t)ch * a.b3_chunk);
        int jj4[4];
        float xv[4];
        int kb[4];
        float cw_k[4], w_k[4], ch_k[4], h_k[4];

        // ---- searched knots' GEMM (widths forward / heights inverse)
        f32x4 acc[K];
        zero_acc<K>(acc);
        gemm_ring<KSH, K, TGK, TGK, HT>(h2, INV ? wH : wW, lane, ring, acc);
        ring_fill<KSH, TGK, TGK>(INV ? wW : wH, lane, ring);
        __builtin_amdgcn_sched_barrier(0);  // phase fence: keeps register pressure per phase
        // ---- bin search
        add_bias<K>(b3 + (INV ? K : 0) * 64, lane, acc);
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const int j = jbase + 4 * q + r;
            jj4[r] = j;
            xv[r] = (j < a.n_up) ? xt[sl * XS + a.up_in[j]] : 0.0f;
        }
        if (INV)
            knot_phase<K, true, true>(acc, xv, c, kb, ch_k, h_k);
        else
            knot_phase<K, true, false>(acc, xv, c, kb, cw_k, w_k);
        __builtin_amdgcn_sched_barrier(0);

        // ---- the other knots' GEMM
        zero_acc<K>(acc);
        gemm_ring<KSH, K, TGK, TGK, HT>(h2, INV ? wW : wH, lane, ring, acc);
        ring_fill<KSH, TGD, TGK>(wD, lane, ring);
        __builtin_amdgcn_sched_barrier(0);
        // ---- select the other knots at the bin
        add_bias<K>(b3 + (INV ? 0 : K) * 64, lane, acc);
        if (INV)
            knot_phase<K, false, false>(acc, xv, c, kb, cw_k, w_k);
        else
            knot_phase<K, false, true>(acc, xv, c, kb, ch_k, h_k);
        __builtin_amdgcn_sched_barrier(0);

        // ---- derivative logits' GEMM
        f32x4 accd[DN];
        zero_acc<DN>(accd);
        gemm_ring<KSH, DN, TGD, TGK, HT>(h2, wD, lane, ring, accd);
        if (ch + 1 < a.NCH) {
            const float4* nx = reinterpret_cast<const float4*>(a.w3 + (int64_t)(ch + 1) * a.w3_chunk);
            ring_fill<KSH, TGK, TGK>(INV ? nx + w3_phase : nx, lane, ring);
        }
        __builtin_amdgcn_sched_barrier(0);
        // ---- derivatives of the bin, evaluate the spline, log|det|
        add_bias<DN>(b3 + 2 * K * 64, lane, accd);
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const int k = kb[r];
            float raw_k = 0.0f, raw_k1 = 0.0f;
#pragma unroll
            for (int t = 0; t < K - 1; ++t) {
                if (k == t + 1) raw_k = accd[t][r];
                if (k == t) raw_k1 = accd[t][r];
            }
            raw_k = nfk_splus<true>(raw_k);  // NSF_CL's D <- softplus(D)
            raw_k1 = nfk_splus<true>(raw_k1);
            raw_k = (k == 0) ? c.dpad : raw_k;
            raw_k1 = (k == K - 1) ? c.dpad : raw_k1;
            const float d_k = c.min_d + nfk_splus<true>(raw_k);
            const float d_k1 = c.min_d + nfk_splus<true>(raw_k1);
            const float x = xv[r];
            const float delta = nfk_div<true>(h_k[r], w_k[r]);
            const float gap = (d_k + d_k1) - 2.0f * delta;
            float out, th;
            bool nd = false;
            if (INV) {
                const float y = x - ch_k[r];
                const float qa = y * gap + h_k[r] * (delta - d_k);
                const float qb = h_k[r] * d_k - y * gap;
                const float qc = (-delta) * y;
                const float disc = qb * qb - (4.0f * qa) * qc;
                nd = !(disc >= 0.0f);
                const float root = nfk_div<true>(2.0f * qc, -qb - sqrtf(disc));
                out = root * w_k[r] + cw_k[r];
                th = root;
            } else {
                th = nfk_div<true>(x - cw_k[r], w_k[r]);
            }
            const float t1mt = th * (1.0f - th);
            const float den = delta + gap * t1mt;
            if (!INV) {
                const float num = h_k[r] * (delta * (th * th) + d_k * t1mt);
                out = ch_k[r] + nfk_div<true>(num, den);
            }
            const float omt = 1.0f - th;
            const float dnum = (delta * delta) * ((d_k1 * (th * th) + (2.0f * delta) * t1mt) + d_k * (omt * omt));
            float lad = nfk_log<true>(dnum) - 2.0f * nfk_log<true>(den);
            lad = INV ? -lad : lad;
            const bool inside = (x >= c.lo) && (x <= c.hi);
            const bool valid = jj4[r] < a.n_up;
            out = inside ? out : x;
            lad = (inside && valid && sl < nrows) ? lad : 0.0f;
            if (valid) zt[sl * D + a.up_out[jj4[r]]] = out;
            ldsum += lad;
            any_in |= inside && valid && sl < nrows;
            any_nd |= nd && inside && valid && sl < nrows;
#ifdef NFK_PAIR_FENCE
            __builtin_amdgcn_sched_barrier(0);
#endif
        }
    }

    // ---- identity-copied coordinates, per-sample log|det|, full-row stores of z
    for (int i = lane; i < 16 * a.n_lo; i += 64) {
        const int row = i / a.n_lo, qq = i - row * a.n_lo;
        zt[row * D + a.lo_out[qq]] = xt[row * XS + a.lo_in[qq]];
    }
    {
        float v = ldsum;
        v += __shfl_xor(v, 16, 64);
        v += __shfl_xor(v, 32, 64);
        if (q == 0 && sl < nrows && a.mode != 0) {
            float* dst = a.logdet + b0 + sl;
            *dst = (a.mode == 2) ? (*dst + v) : v;
        }
    }
    for (int r = 0; r < nrows; ++r)
        for (int cc = lane; cc < D; cc += 64) a.z[(b0 + r) * a.ldz + cc] = zt[r * D + cc];

    if (a.status != nullptr) {
        const int bits = (__any(any_in) ? NFK_ST_INSIDE_SEEN : 0) | (__any(any_nd) ? NFK_ST_NEG_DISC : 0);
        if (lane == 0 && bits != 0) {
            if ((__hip_atomic_load(a.status, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) & bits) != bits)
                atomicOr(a.status, bits);
        }
    }
}

template <int KSH, int K>
int launch_fused(const FusedArgs& a, bool inv, hipStream_t st) {
    const int D = a.n_lo + a.n_up;
    const size_t lds = (size_t)kWaves * 16 * (2 * D + 1) * sizeof(float);
    const int64_t per_block = (int64_t)kWaves * 16;
    const int64_t blocks = (a.batch + per_block - 1) / per_block;
    if (blocks == 0) return 0;
    if (inv)
        hipLaunchKernelGGL((k_fused_nsf<KSH, K, true>), dim3((unsigned)blocks), dim3(64 * kWaves), lds,
                           st, a);
    else
        hipLaunchKernelGGL((k_fused_nsf<KSH, K, false>), dim3((unsigned)blocks), dim3(64 * kWaves),
                           lds, st, a);
    hipError_t e = hipGetLastError();
    return e == hipSuccess ? 0 : (int)e;
}

// explicit instantiation: definitions live in nfk_fused_ksh<KSH>.hip (one TU
// per hidden k-step count so make -j compiles them in parallel); nfk_fused.hip
// sees only the extern declarations.
#define NFK_FUSED_INSTANCE(KSH, K) \
    template int launch_fused<KSH, K>(const FusedArgs& a, bool inv, hipStream_t st);
#define NFK_FUSED_EXTERN(KSH, K) \
    extern template int launch_fused<KSH, K>(const FusedArgs& a, bool inv, hipStream_t st);

// supported hidden sizes: KSH = ceil(H/4) k-steps of 4 (H = 12, 16, 32, 64, 100, 128)
#define NFK_FUSED_KSH(X) X(3) X(4) X(8) X(16) X(25) X(32)
#define NFK_FUSED_K(X, KSH) X(KSH, 4) X(KSH, 5) X(KSH, 6) X(KSH, 8) X(KSH, 10)

}  // namespace nfk_fused
