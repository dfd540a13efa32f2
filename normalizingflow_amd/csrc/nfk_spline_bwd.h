// nfk_spline_bwd.h -- backward of one rational-quadratic spline element
// (derivation in nfk_backward.hip), shared by the streaming VJP kernel
// (k_rqs_coupling_bwd) and the fused recompute + VJP kernel (nfk_fused_vjp.hip).
#pragma once
#include <hip/hip_runtime.h>

#include "nfk_spline.h"

namespace nfk_bwd {

// Diagnostic probes (NFK_BWD_PROBE builds only: tools/dbg_vjp_save.py's
// "probe" variant): rqs_element_bwd stores its intermediates at fixed slots of
// a caller array so two evaluations can be compared stage by stage.
#ifdef NFK_BWD_PROBE
#define NFK_PROBE_PARAM , float* nfk_probe
#define NFK_PROBE(i, v) (nfk_probe[(i)] = (float)(v))
#else
#define NFK_PROBE_PARAM
#define NFK_PROBE(i, v) ((void)0)
#endif
constexpr int kProbeSlots = 80;

// d softplus(v) / dv as torch's softplus_backward (beta 1, threshold 20)
template <bool FAST = false>
__device__ __forceinline__ float softplus_grad(float v) {
    if (v > 20.0f) return 1.0f;
    const float e = nfk_exp<FAST>(v);
    return nfk_div<FAST>(e, e + 1.0f);
}

// softmax backward in place: g <- s * (g - sum(g * s))
template <int K>
__device__ __forceinline__ void softmax_bwd(const float (&s)[K], float (&g)[K]) {
    float dot = 0.0f;
#pragma unroll
    for (int i = 0; i < K; ++i) dot += g[i] * s[i];
#pragma unroll
    for (int i = 0; i < K; ++i) g[i] = s[i] * (g[i] - dot);
}

// softmax forward, reference summation order (shared with the forward kernels)
template <int K, bool FAST = false>
__device__ __forceinline__ void softmax_fwd(const float (&u)[K], float (&s)[K]) {
#pragma unroll
    for (int i = 0; i < K; ++i) s[i] = u[i];
    nfk_softmax<K, FAST>(s);
}

// One side (widths or heights): logits -> (s0 if PRE) -> s1 -> edges.
// FAST: hardware exp / reciprocal and an fp32 cumulative sum (the fused VJP
// kernel, whose forward recompute is itself the lean arithmetic); otherwise
// the reference's op order with the double-accumulated cumsum.
template <int K, bool PRE, bool FAST = false>
struct KnotSide {
    float s0[K];  // first softmax (PRE only)
    float s1[K];  // second softmax
    float edge[K + 1];

    __device__ __forceinline__ void build(const float (&u)[K], float scale2b, float lo, float hi,
                                          float span, float min_b, float fb) {
        if (PRE) {
            softmax_fwd<K, FAST>(u, s0);
#pragma unroll
            for (int i = 0; i < K; ++i) s1[i] = scale2b * s0[i];
        } else {
#pragma unroll
            for (int i = 0; i < K; ++i) s1[i] = u[i];
        }
        nfk_softmax<K, FAST>(s1);
        edge[0] = lo;
        if constexpr (FAST) {
            float acc = 0.0f;
#pragma unroll
            for (int i = 0; i < K; ++i) {
                acc += min_b + fb * s1[i];
                edge[i + 1] = span * acc + lo;
            }
        } else {
            double acc = 0.0;
#pragma unroll
            for (int i = 0; i < K; ++i) {
                acc += (double)(min_b + fb * s1[i]);
                edge[i + 1] = span * (float)acc + lo;
            }
        }
        edge[K] = hi;
    }

    // gradient w.r.t. the logits from the adjoints of (edge_k, size_k = edge_k+1 - edge_k)
    __device__ __forceinline__ void backward(int k, float g_pos, float g_size, float span, float fb,
                                             float scale2b, float (&g)[K]) const {
        // adjoint of edge_k and edge_k+1 (the pinned ends 0 and K carry none)
        const float ga = (k >= 1) ? (g_pos - g_size) : 0.0f;
        const float gb = (k + 1 <= K - 1) ? g_size : 0.0f;
#pragma unroll
        for (int j = 0; j < K; ++j) {
            float v = 0.0f;
            if (j < k) v += ga;
            if (j <= k) v += gb;
            g[j] = span * fb * v;  // d edge_e / d s1_j = span * fb for j < e
        }
        softmax_bwd<K>(s1, g);
        if (PRE) {
#pragma unroll
            for (int j = 0; j < K; ++j) g[j] *= scale2b;
            softmax_bwd<K>(s0, g);
        }
    }
};

template <int K>
__device__ __forceinline__ float sel(const float (&a)[K], int k) { return nfk_sel<K>(a, k); }

// Backward of one spline element.  wr/hr/dr in: logits; out: their gradients.
// FAST: hardware exp / log / reciprocal throughout (see KnotSide).
template <int K, bool INV, bool PRE, bool DFULL, bool FAST = false>
__device__ __forceinline__ float rqs_element_bwd(float x, float (&wr)[K], float (&hr)[K],
                                                 float (&dr)[NfkDN<K, DFULL>::n],
                                                 const NfkSplineConst& c, float gout, float gl NFK_PROBE_PARAM) {
    constexpr int DN = NfkDN<K, DFULL>::n;
    const bool inside = !c.tails || ((x >= c.lo) && (x <= c.hi));
    if (!inside) {
#pragma unroll
        for (int i = 0; i < K; ++i) wr[i] = hr[i] = 0.0f;
#pragma unroll
        for (int i = 0; i < DN; ++i) dr[i] = 0.0f;
        return gout;
    }
    KnotSide<K, PRE, FAST> W, H;
    W.build(wr, c.scale2b, c.lo, c.hi, c.span, c.min_w, c.fw);
    H.build(hr, c.scale2b, c.ylo, c.yhi, c.yspan, c.min_h, c.fh);
    const int k = nfk_bin<K>(INV ? H.edge : W.edge, x, c.knot_eps);
#pragma unroll
    for (int j = 0; j < K && j < 8; ++j) {
        NFK_PROBE(j, W.s1[j]);
        NFK_PROBE(17 + j, H.s1[j]);
    }
#pragma unroll
    for (int j = 0; j <= K && j < 9; ++j) {
        NFK_PROBE(8 + j, W.edge[j]);
        NFK_PROBE(25 + j, H.edge[j]);
    }
    NFK_PROBE(34, k);
    float cw_k = W.edge[0], w_k = W.edge[1] - W.edge[0], ch_k = H.edge[0], h_k = H.edge[1] - H.edge[0];
#pragma unroll
    for (int j = 1; j < K; ++j) {
        if (k == j) {
            cw_k = W.edge[j];
            w_k = W.edge[j + 1] - W.edge[j];
            ch_k = H.edge[j];
            h_k = H.edge[j + 1] - H.edge[j];
        }
    }
    // derivative logits used by bin k: v0 -> d_k, v1 -> d_k1 (pre-RQS-softplus
    // values), with their source index (-1: the constant boundary pad)
    int i0 = -1, i1 = -1;
    float v0 = c.dpad, v1 = c.dpad, r0 = 0.0f, r1 = 0.0f;  // r: NSF_CL raw logit (PRE)
    if (DFULL) {
        i0 = k;
        i1 = k + 1;
#pragma unroll
        for (int j = 0; j < DN; ++j) {
            if (j == i0) v0 = dr[j];
            if (j == i1) v1 = dr[j];
        }
    } else {
        i0 = k - 1;  // padded index k holds logit k-1
        i1 = (k + 1 <= K - 1) ? k : -1;
#pragma unroll
        for (int j = 0; j < DN; ++j) {
            if (j == i0) r0 = dr[j];
            if (j == i1) r1 = dr[j];
        }
        if (i0 >= 0) v0 = PRE ? nfk_splus<FAST>(r0) : r0;
        if (i1 >= 0) v1 = PRE ? nfk_splus<FAST>(r1) : r1;
    }
    const float d0 = c.min_d + nfk_splus<FAST>(v0);
    const float d1 = c.min_d + nfk_splus<FAST>(v1);
    const float delta = nfk_div<FAST>(h_k, w_k);
    const float gap = (d0 + d1) - 2.0f * delta;
    NFK_PROBE(35, d0);
    NFK_PROBE(36, d1);
    NFK_PROBE(37, delta);

    float th;
    if (INV) {
        const float y = x - ch_k;
        const float qa = y * gap + h_k * (delta - d0);
        const float qb = h_k * d0 - y * gap;
        const float qc = (-delta) * y;
        const float disc = qb * qb - (4.0f * qa) * qc;
        th = nfk_div<FAST>(2.0f * qc, -qb - sqrtf(fmaxf(disc, 0.0f)));
    } else {
        th = nfk_div<FAST>(x - cw_k, w_k);
    }
    const float s = th * (1.0f - th);
    const float omt = 1.0f - th;
    const float Dn = delta + gap * s;
    const float N = h_k * (delta * th * th + d0 * s);
    const float R = nfk_div<FAST>(N, Dn);
    const float M = delta * delta * (d1 * th * th + 2.0f * delta * s + d0 * omt * omt);
    const float iDn = nfk_div<FAST>(1.0f, Dn), iM = nfk_div<FAST>(1.0f, M);
    const float one_m2t = 1.0f - 2.0f * th;
    // partials of Dn, N, M over the base variables
    const float Dn_t = gap * one_m2t, Dn_dl = 1.0f - 2.0f * s, Dn_d0 = s, Dn_d1 = s;
    const float N_t = h_k * (2.0f * delta * th + d0 * one_m2t), N_dl = h_k * th * th;
    const float N_h = delta * th * th + d0 * s, N_d0 = h_k * s;
    const float M_t = delta * delta * (2.0f * d1 * th + 2.0f * delta * one_m2t - 2.0f * d0 * omt);
    const float M_dl = 2.0f * delta * (d1 * th * th + 2.0f * delta * s + d0 * omt * omt) +
                       2.0f * delta * delta * s;
    const float M_d0 = delta * delta * omt * omt, M_d1 = delta * delta * th * th;
    // f and lad partials over (theta, delta, h explicit, d0, d1)
    const float f_t = (N_t - R * Dn_t) * iDn, f_dl = (N_dl - R * Dn_dl) * iDn;
    const float f_h = N_h * iDn, f_d0 = (N_d0 - R * Dn_d0) * iDn, f_d1 = (-R * Dn_d1) * iDn;
    const float l_t = M_t * iM - 2.0f * Dn_t * iDn, l_dl = M_dl * iM - 2.0f * Dn_dl * iDn;
    const float l_d0 = M_d0 * iM - 2.0f * Dn_d0 * iDn, l_d1 = M_d1 * iM - 2.0f * Dn_d1 * iDn;
    const float iw = nfk_div<FAST>(1.0f, w_k);
    NFK_PROBE(38, th);
    NFK_PROBE(39, Dn);
    NFK_PROBE(40, N);
    NFK_PROBE(41, M);
    NFK_PROBE(42, iDn);
    NFK_PROBE(43, iM);
    NFK_PROBE(44, iw);

    float a, b, gx;  // g_bin = a * f_bin + b * lad_bin
    if (INV) {
        const float fprime = f_t * iw;
        const float gbar = gout - gl * (l_t * iw);
        gx = nfk_div<FAST>(gbar, fprime);
        a = -gx;
        b = -gl;
    } else {
        a = gout;
        b = gl;
        gx = a * f_t * iw + b * l_t * iw;
    }
    const float G_t = a * f_t + b * l_t, G_dl = a * f_dl + b * l_dl;
    const float g_cw = -G_t * iw;
    const float g_w = -(G_t * th + G_dl * delta) * iw;
    const float g_ch = a;
    const float g_h = a * f_h + G_dl * iw;
    const float g_d0 = a * f_d0 + b * l_d0;
    const float g_d1 = a * f_d1 + b * l_d1;
    NFK_PROBE(45, G_t);
    NFK_PROBE(46, G_dl);
    NFK_PROBE(47, g_w);
    NFK_PROBE(48, g_h);

    W.backward(k, g_cw, g_w, c.span, c.fw, c.scale2b, wr);
    H.backward(k, g_ch, g_h, c.yspan, c.fh, c.scale2b, hr);
    // derivative logits: d = min_d + softplus(v); v = softplus(r) under PRE
    float gv0 = g_d0 * softplus_grad<FAST>(v0), gv1 = g_d1 * softplus_grad<FAST>(v1);
    if (PRE && !DFULL) {
        gv0 *= softplus_grad<FAST>(r0);
        gv1 *= softplus_grad<FAST>(r1);
    }
#pragma unroll
    for (int j = 0; j < DN; ++j) {
        float g = 0.0f;
        if (j == i0) g += gv0;
        if (j == i1) g += gv1;
        dr[j] = g;
    }
#pragma unroll
    for (int j = 0; j < K && j < 8; ++j) {
        NFK_PROBE(49 + j, wr[j]);
        NFK_PROBE(57 + j, hr[j]);
    }
#pragma unroll
    for (int j = 0; j < DN && j < 7; ++j) NFK_PROBE(65 + j, dr[j]);
    NFK_PROBE(72, gx);
    return gx;
}

}  // namespace nfk_bwd
