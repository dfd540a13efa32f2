// nfk_fused_impl.h -- fused NSF coupling-layer kernel; design notes in nfk_fused.hip.
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>

#include "../../include/nfk.h"
#include "nfk_spline.h"

typedef float f32x4 __attribute__((ext_vector_type(4)));

namespace nfk_fused {

constexpr int kWaves = 4;  // waves per workgroup
#ifndef NFK_FUSED_ST
#define NFK_FUSED_ST 1
#endif
constexpr int kST = NFK_FUSED_ST;  // 16-sample tiles per wave
constexpr int kMaxD = 256;         // n_lo + n_up staged in LDS
constexpr int kPF = 4;             // weight prefetch distance (k-steps)

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

// acc[st][t] += W[tile t] . act^T over KS k-steps; A fragments streamed from
// the packed weights (4 tiles per float4, NG groups per k-step) with a
// register ring kPF k-steps deep; B fragment of k-step ks = act[st][ks>>2][ks&3].
template <int KS, int NT, int NG, int ST, int HTA>
__device__ __forceinline__ void gemm_stream(const f32x4 (&act)[ST][HTA], const float4* __restrict__ wp,
                                            int lane, f32x4 (&acc)[ST][NT]) {
    constexpr int PF = KS < kPF ? KS : kPF;
    float4 ring[PF][NG];
#pragma unroll
    for (int p = 0; p < PF; ++p)
#pragma unroll
        for (int g = 0; g < NG; ++g) ring[p][g] = wp[(p * NG + g) * 64 + lane];
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) {
        float4 cur[NG];
#pragma unroll
        for (int g = 0; g < NG; ++g) cur[g] = ring[ks % PF][g];
        if (ks + PF < KS) {
#pragma unroll
            for (int g = 0; g < NG; ++g) ring[ks % PF][g] = wp[((ks + PF) * NG + g) * 64 + lane];
        }
        // keep the prefetch of k-step ks+PF ahead of k-step ks's MFMAs (the
        // scheduler otherwise sinks the loads next to their use)
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int g = 0; g < NG; ++g) {
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                const int t = 4 * g + e;
                if (t < NT) {
                    const float av = pick4(cur[g], e);
#pragma unroll
                    for (int st = 0; st < ST; ++st) acc[st][t] = mfma(av, act[st][ks >> 2][ks & 3], acc[st][t]);
                }
            }
        }
    }
}

// bias-initialised accumulators of NT parameter tiles (packed b3: one float4 per tile)
template <int NT, int ST>
__device__ __forceinline__ void bias_init(const float4* __restrict__ bp, int lane, f32x4 (&acc)[ST][NT]) {
#pragma unroll
    for (int t = 0; t < NT; ++t) {
        const float4 b = bp[t * 64 + lane];
        f32x4 v;
        v[0] = b.x;
        v[1] = b.y;
        v[2] = b.z;
        v[3] = b.w;
#pragma unroll
        for (int st = 0; st < ST; ++st) acc[st][t] = v;
    }
}

template <int KSH, int K, bool INV, int ST>
__global__ __launch_bounds__(256, 2) void k_fused_nsf(FusedArgs a) {
    constexpr int HT = (KSH + 3) / 4;
    constexpr int TGH = (HT + 3) / 4;
    constexpr int TGK = (K + 3) / 4;
    constexpr int TGD = (K - 1 + 3) / 4;
    constexpr int DN = K - 1 > 0 ? K - 1 : 1;
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    const int q = lane >> 4, sl = lane & 15;
    const int D = a.n_lo + a.n_up;
    const int XS = D + 1;
    extern __shared__ __attribute__((aligned(16))) float lds[];
    float* xt = lds + wid * (ST * 16) * (XS + D);
    float* zt = xt + (ST * 16) * XS;
    const int64_t b0 = ((int64_t)blockIdx.x * kWaves + wid) * (16 * ST);
    const int64_t rem = a.batch - b0;
    const int nrows = rem <= 0 ? 0 : (rem < 16 * ST ? (int)rem : 16 * ST);

    // ---- stage this wave's x rows (full-row coalesced loads)
    for (int r = 0; r < 16 * ST; ++r)
        for (int c = lane; c < D; c += 64)
            xt[r * XS + c] = (r < nrows) ? a.x[(b0 + r) * a.ldx + c] : 0.0f;
    __syncthreads();

    // ---- layer 1: h1^T = tanh(W1 . lower^T + b1)
    f32x4 h1[ST][HT];
#pragma unroll
    for (int t = 0; t < HT; ++t) {
        f32x4 bv;
#pragma unroll
        for (int r = 0; r < 4; ++r) bv[r] = a.b1[16 * t + 4 * r + q];
#pragma unroll
        for (int st = 0; st < ST; ++st) h1[st][t] = bv;
    }
    {
        const float4* wp = reinterpret_cast<const float4*>(a.w1);
        for (int ks = 0; ks < a.KS1; ++ks) {
            const int k = 4 * ks + q;
            const int col = (k < a.n_lo) ? a.lo_in[k] : -1;
            float bf[ST];
#pragma unroll
            for (int st = 0; st < ST; ++st) bf[st] = (col >= 0) ? xt[(st * 16 + sl) * XS + col] : 0.0f;
#pragma unroll
            for (int g = 0; g < TGH; ++g) {
                const float4 w = wp[(ks * TGH + g) * 64 + lane];
#pragma unroll
                for (int e = 0; e < 4; ++e) {
                    const int t = 4 * g + e;
                    if (t < HT) {
#pragma unroll
                        for (int st = 0; st < ST; ++st) h1[st][t] = mfma(pick4(w, e), bf[st], h1[st][t]);
                    }
                }
            }
        }
    }
#pragma unroll
    for (int st = 0; st < ST; ++st)
#pragma unroll
        for (int t = 0; t < HT; ++t)
#pragma unroll
            for (int r = 0; r < 4; ++r) h1[st][t][r] = tanhf(h1[st][t][r]);

    // ---- layer 2: h2^T = tanh(W2 . h1^T + b2); register r of tile t = k-step 4t+r
    f32x4 h2[ST][HT];
#pragma unroll
    for (int t = 0; t < HT; ++t) {
        f32x4 bv;
#pragma unroll
        for (int r = 0; r < 4; ++r) bv[r] = a.b2[16 * t + 4 * r + q];
#pragma unroll
        for (int st = 0; st < ST; ++st) h2[st][t] = bv;
    }
    gemm_stream<KSH, HT, TGH, ST, HT>(h1, reinterpret_cast<const float4*>(a.w2), lane, h2);
#pragma unroll
    for (int st = 0; st < ST; ++st)
#pragma unroll
        for (int t = 0; t < HT; ++t)
#pragma unroll
            for (int r = 0; r < 4; ++r) h2[st][t][r] = tanhf(h2[st][t][r]);

    // ---- output layer + spline, chunk by chunk of 16 coordinates
    const NfkSplineConst& c = a.c;
    float ldsum[ST];
#pragma unroll
    for (int st = 0; st < ST; ++st) ldsum[st] = 0.0f;
    bool any_in = false, any_nd = false;

    for (int ch = 0; ch < a.NCH; ++ch) {
        const int jbase = 16 * ch;
        const float4* w3 = reinterpret_cast<const float4*>(a.w3 + (int64_t)ch * a.w3_chunk);
        const float4* wW = w3;
        const float4* wH = w3 + KSH * TGK * 64;
        const float4* wD = w3 + 2 * KSH * TGK * 64;
        const float4* b3 = reinterpret_cast<const float4*>(a.b3 + (int64_t)ch * a.b3_chunk);
        int kb[ST][4];
        float e0[ST][4], e1[ST][4], e2[ST][4], e3[ST][4];  // (cw_k, w_k, ch_k, h_k)

        // phase 1: the searched knots (widths forward, heights inverse)
        {
            f32x4 acc[ST][K];
            bias_init<K, ST>(b3 + (INV ? K : 0) * 64, lane, acc);
            gemm_stream<KSH, K, TGK, ST, HT>(h2, INV ? wH : wW, lane, acc);
#pragma unroll
            for (int st = 0; st < ST; ++st) {
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    const int j = jbase + 4 * q + r;
                    const float xv = (j < a.n_up) ? xt[(st * 16 + sl) * XS + a.up_in[j]] : 0.0f;
                    float u[K], edge[K + 1];
#pragma unroll
                    for (int t = 0; t < K; ++t) u[t] = acc[st][t][r];
                    nfk_softmax<K>(u);
#pragma unroll
                    for (int t = 0; t < K; ++t) u[t] = c.scale2b * u[t];
                    if (INV)
                        nfk_knots<K>(u, c.ylo, c.yhi, c.yspan, c.min_h, c.fh, edge);
                    else
                        nfk_knots<K>(u, c.lo, c.hi, c.span, c.min_w, c.fw, edge);
                    const int k = nfk_bin<K>(edge, xv, c.knot_eps);
                    float ek = edge[0], sk = edge[1] - edge[0];
#pragma unroll
                    for (int jj = 1; jj < K; ++jj)
                        if (k == jj) {
                            ek = edge[jj];
                            sk = edge[jj + 1] - edge[jj];
                        }
                    kb[st][r] = k;
                    if (INV) {
                        e2[st][r] = ek;
                        e3[st][r] = sk;
                    } else {
                        e0[st][r] = ek;
                        e1[st][r] = sk;
                    }
                }
            }
        }
        // phase 2: the other knots, selected at the bin found above
        {
            f32x4 acc[ST][K];
            bias_init<K, ST>(b3 + (INV ? 0 : K) * 64, lane, acc);
            gemm_stream<KSH, K, TGK, ST, HT>(h2, INV ? wW : wH, lane, acc);
#pragma unroll
            for (int st = 0; st < ST; ++st) {
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    float u[K], edge[K + 1];
#pragma unroll
                    for (int t = 0; t < K; ++t) u[t] = acc[st][t][r];
                    nfk_softmax<K>(u);
#pragma unroll
                    for (int t = 0; t < K; ++t) u[t] = c.scale2b * u[t];
                    if (INV)
                        nfk_knots<K>(u, c.lo, c.hi, c.span, c.min_w, c.fw, edge);
                    else
                        nfk_knots<K>(u, c.ylo, c.yhi, c.yspan, c.min_h, c.fh, edge);
                    const int k = kb[st][r];
                    float ek = edge[0], sk = edge[1] - edge[0];
#pragma unroll
                    for (int jj = 1; jj < K; ++jj)
                        if (k == jj) {
                            ek = edge[jj];
                            sk = edge[jj + 1] - edge[jj];
                        }
                    if (INV) {
                        e0[st][r] = ek;
                        e1[st][r] = sk;
                    } else {
                        e2[st][r] = ek;
                        e3[st][r] = sk;
                    }
                }
            }
        }
        // phase 3: derivative logits -> the two derivatives of the bin -> evaluate
        {
            f32x4 acc[ST][DN];
            bias_init<DN, ST>(b3 + 2 * K * 64, lane, acc);
            gemm_stream<KSH, DN, TGD, ST, HT>(h2, wD, lane, acc);
#pragma unroll
            for (int st = 0; st < ST; ++st) {
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    const int j = jbase + 4 * q + r;
                    const bool valid = j < a.n_up;
                    const int row = st * 16 + sl;
                    const float xv = valid ? xt[row * XS + a.up_in[j]] : 0.0f;
                    const int k = kb[st][r];
                    float raw_k = 0.0f, raw_k1 = 0.0f;
#pragma unroll
                    for (int t = 0; t < K - 1; ++t) {
                        if (k == t + 1) raw_k = acc[st][t][r];
                        if (k == t) raw_k1 = acc[st][t][r];
                    }
                    raw_k = nfk_softplus(raw_k);  // NSF_CL's D <- softplus(D)
                    raw_k1 = nfk_softplus(raw_k1);
                    raw_k = (k == 0) ? c.dpad : raw_k;
                    raw_k1 = (k == K - 1) ? c.dpad : raw_k1;
                    const float d_k = c.min_d + nfk_softplus(raw_k);
                    const float d_k1 = c.min_d + nfk_softplus(raw_k1);
                    const float cw_k = e0[st][r], w_k = e1[st][r];
                    const float ch_k = e2[st][r], h_k = e3[st][r];
                    const float delta = h_k / w_k;
                    const float gap = (d_k + d_k1) - 2.0f * delta;
                    float out, th;
                    bool nd = false;
                    if (INV) {
                        const float y = xv - ch_k;
                        const float qa = y * gap + h_k * (delta - d_k);
                        const float qb = h_k * d_k - y * gap;
                        const float qc = (-delta) * y;
                        const float disc = qb * qb - (4.0f * qa) * qc;
                        nd = !(disc >= 0.0f);
                        const float root = (2.0f * qc) / (-qb - sqrtf(disc));
                        out = root * w_k + cw_k;
                        th = root;
                    } else {
                        th = (xv - cw_k) / w_k;
                    }
                    const float t1mt = th * (1.0f - th);
                    const float den = delta + gap * t1mt;
                    if (!INV) {
                        const float num = h_k * (delta * (th * th) + d_k * t1mt);
                        out = ch_k + num / den;
                    }
                    const float omt = 1.0f - th;
                    const float dnum = (delta * delta) *
                                       ((d_k1 * (th * th) + (2.0f * delta) * t1mt) + d_k * (omt * omt));
                    float lad = logf(dnum) - 2.0f * logf(den);
                    lad = INV ? -lad : lad;
                    const bool inside = (xv >= c.lo) && (xv <= c.hi);
                    if (!inside) {
                        out = xv;
                        lad = 0.0f;
                        nd = false;
                    }
                    if (valid) {
                        zt[row * D + a.up_out[j]] = out;
                        if (row < nrows) {
                            ldsum[st] += lad;
                            any_in |= inside;
                            any_nd |= nd;
                        }
                    }
                }
            }
        }
    }

    // ---- identity-copied coordinates, then full-row stores of z
    for (int i = lane; i < 16 * ST * a.n_lo; i += 64) {
        const int row = i / a.n_lo, qq = i - row * a.n_lo;
        zt[row * D + a.lo_out[qq]] = xt[row * XS + a.lo_in[qq]];
    }
#pragma unroll
    for (int st = 0; st < ST; ++st) {
        float v = ldsum[st];
        v += __shfl_xor(v, 16, 64);
        v += __shfl_xor(v, 32, 64);
        const int row = st * 16 + sl;
        if (q == 0 && row < nrows && a.mode != 0) {
            float* dst = a.logdet + b0 + row;
            *dst = (a.mode == 2) ? (*dst + v) : v;
        }
    }
    __syncthreads();
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
    const size_t lds = (size_t)kWaves * (kST * 16) * (2 * D + 1) * sizeof(float);
    const int64_t per_block = (int64_t)kWaves * 16 * kST;
    const int64_t blocks = (a.batch + per_block - 1) / per_block;
    if (blocks == 0) return 0;
    if (inv)
        hipLaunchKernelGGL((k_fused_nsf<KSH, K, true, kST>), dim3((unsigned)blocks), dim3(64 * kWaves),
                           lds, st, a);
    else
        hipLaunchKernelGGL((k_fused_nsf<KSH, K, false, kST>), dim3((unsigned)blocks),
                           dim3(64 * kWaves), lds, st, a);
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
