// nfk_backward.hip -- vector-Jacobian product of the spline coupling
// (the backward of nfk_rqs_coupling / the spline half of nfk_fused_nsf).
//
// Given the layer input x, the conditioner's raw output `params` and the
// upstream gradients gz = dL/dz, gld = dL/dlog|det| (per sample), one lane per
// (sample, transformed coordinate) element computes
//     g_params = dL/dparams   (same [batch, n_up, P] layout as params)
//     gx[:, up_in[j]] = dL/dx_up
// and the lower (identity-copied) coordinates pass gz through:
//     gx[:, lo_in[q]] = gz[:, lo_out[q]].
// The conditioner's own backward (GEMMs) runs outside, fed by g_params.
//
// Derivation (reference math nf/utils.py:58-152, nf/flows.py:233-235):
//   forward map at bin k, theta = (x - cw_k)/w_k, delta = h_k/w_k, s = theta(1-theta):
//     f   = ch_k + h_k (delta theta^2 + d_k s) / Dn,  Dn = delta + (d_k + d_k1 - 2 delta) s
//     lad = log(delta^2 (d_k1 theta^2 + 2 delta s + d_k (1-theta)^2)) - 2 log Dn
//   Partials of f and lad with respect to (theta, delta, h_k explicit, d_k, d_k1)
//   are chained to the bin quantities (cw_k, w_k, ch_k, h_k, d_k, d_k1).
//   The inverse, o = f^-1(x), L = -lad(o), uses implicit differentiation:
//     go' = gz - gld * dlad/do;  gx = go' / f'(o);
//     g_bin = -(go'/f') df/dbin - gld dlad/dbin   (partials at fixed o).
//   Bin quantities -> knots: cw_k = edge_k, w_k = edge_k+1 - edge_k with the
//   two end edges pinned; edge_e = lo + span * sum_{j<e} (min_w + fw softmax(W)_j);
//   then softmax backward (twice for NSF_CL's 2B*softmax pre-normalisation)
//   and softplus backward (twice: NSF_CL's softplus, then RQS's) for the two
//   derivatives the bin uses.  Outside [-B, B]: identity, gx = gz, g = 0.
// The bin is located exactly as in the forward kernels (same knot arithmetic).
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdio>

#include "../../include/nfk.h"
#include "nfk_spline.h"

int nfk_set_error(const char* msg);
NfkSplineConst nfk_make_const(int K, double left, double right, double bottom, double top,
                              int tails, double min_w, double min_h, double min_d);

namespace {

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

// d softplus(v) / dv as torch's softplus_backward (beta 1, threshold 20)
__device__ __forceinline__ float softplus_grad(float v) {
    if (v > 20.0f) return 1.0f;
    const float e = expf(v);
    return e / (e + 1.0f);
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
template <int K>
__device__ __forceinline__ void softmax_fwd(const float (&u)[K], float (&s)[K]) {
#pragma unroll
    for (int i = 0; i < K; ++i) s[i] = u[i];
    nfk_softmax<K>(s);
}

// One side (widths or heights): logits -> (s0 if PRE) -> s1 -> edges.
template <int K, bool PRE>
struct KnotSide {
    float s0[K];  // first softmax (PRE only)
    float s1[K];  // second softmax
    float edge[K + 1];

    __device__ __forceinline__ void build(const float (&u)[K], float scale2b, float lo, float hi,
                                          float span, float min_b, float fb) {
        if (PRE) {
            softmax_fwd<K>(u, s0);
#pragma unroll
            for (int i = 0; i < K; ++i) s1[i] = scale2b * s0[i];
        } else {
#pragma unroll
            for (int i = 0; i < K; ++i) s1[i] = u[i];
        }
        nfk_softmax<K>(s1);
        double acc = 0.0;
        edge[0] = lo;
#pragma unroll
        for (int i = 0; i < K; ++i) {
            acc += (double)(min_b + fb * s1[i]);
            edge[i + 1] = span * (float)acc + lo;
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
template <int K, bool INV, bool PRE, bool DFULL>
__device__ __forceinline__ float rqs_element_bwd(float x, float (&wr)[K], float (&hr)[K],
                                                 float (&dr)[NfkDN<K, DFULL>::n],
                                                 const NfkSplineConst& c, float gout, float gl) {
    constexpr int DN = NfkDN<K, DFULL>::n;
    const bool inside = !c.tails || ((x >= c.lo) && (x <= c.hi));
    if (!inside) {
#pragma unroll
        for (int i = 0; i < K; ++i) wr[i] = hr[i] = 0.0f;
#pragma unroll
        for (int i = 0; i < DN; ++i) dr[i] = 0.0f;
        return gout;
    }
    KnotSide<K, PRE> W, H;
    W.build(wr, c.scale2b, c.lo, c.hi, c.span, c.min_w, c.fw);
    H.build(hr, c.scale2b, c.ylo, c.yhi, c.yspan, c.min_h, c.fh);
    const int k = nfk_bin<K>(INV ? H.edge : W.edge, x, c.knot_eps);
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
        if (i0 >= 0) v0 = PRE ? nfk_softplus(r0) : r0;
        if (i1 >= 0) v1 = PRE ? nfk_softplus(r1) : r1;
    }
    const float d0 = c.min_d + nfk_softplus(v0);
    const float d1 = c.min_d + nfk_softplus(v1);
    const float delta = h_k / w_k;
    const float gap = (d0 + d1) - 2.0f * delta;

    float th;
    if (INV) {
        const float y = x - ch_k;
        const float qa = y * gap + h_k * (delta - d0);
        const float qb = h_k * d0 - y * gap;
        const float qc = (-delta) * y;
        const float disc = qb * qb - (4.0f * qa) * qc;
        th = (2.0f * qc) / (-qb - sqrtf(fmaxf(disc, 0.0f)));
    } else {
        th = (x - cw_k) / w_k;
    }
    const float s = th * (1.0f - th);
    const float omt = 1.0f - th;
    const float Dn = delta + gap * s;
    const float N = h_k * (delta * th * th + d0 * s);
    const float R = N / Dn;
    const float M = delta * delta * (d1 * th * th + 2.0f * delta * s + d0 * omt * omt);
    const float iDn = 1.0f / Dn, iM = 1.0f / M;
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
    const float iw = 1.0f / w_k;

    float a, b, gx;  // g_bin = a * f_bin + b * lad_bin
    if (INV) {
        const float fprime = f_t * iw;
        const float gbar = gout - gl * (l_t * iw);
        gx = gbar / fprime;
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

    W.backward(k, g_cw, g_w, c.span, c.fw, c.scale2b, wr);
    H.backward(k, g_ch, g_h, c.yspan, c.fh, c.scale2b, hr);
    // derivative logits: d = min_d + softplus(v); v = softplus(r) under PRE
    float gv0 = g_d0 * softplus_grad(v0), gv1 = g_d1 * softplus_grad(v1);
    if (PRE && !DFULL) {
        gv0 *= softplus_grad(r0);
        gv1 *= softplus_grad(r1);
    }
#pragma unroll
    for (int j = 0; j < DN; ++j) {
        float g = 0.0f;
        if (j == i0) g += gv0;
        if (j == i1) g += gv1;
        dr[j] = g;
    }
    return gx;
}

struct RqsBwdArgs {
    const float* x;
    int64_t ldx;
    const float* params;
    const int32_t* up_in;
    const int32_t* up_out;
    int32_t n_up;
    const int32_t* lo_in;
    const int32_t* lo_out;
    int32_t n_lo;
    const float* gz;
    int64_t ldgz;
    const float* gld;
    float* gparams;
    float* gx;
    int64_t ldgx;
    int64_t batch;
    int32_t spb;
    NfkSplineConst c;
};

// Block layout as the forward (k_rqs_coupling): S whole samples per block,
// the [elements, P] parameter slab streamed through LDS with 16-B accesses in
// both directions; each lane overwrites its own LDS row with its gradients.
template <int K, bool INV, bool PRE, bool DFULL, int EPB>
__global__ __launch_bounds__(EPB) void k_rqs_coupling_bwd(RqsBwdArgs a) {
    constexpr int DN = NfkDN<K, DFULL>::n;
    constexpr int P = DFULL ? 3 * K + 1 : 3 * K - 1;
    extern __shared__ __attribute__((aligned(16))) float smem[];
    float* sp = smem;  // [EPB][P]
    const int tid = threadIdx.x;
    const int64_t b0 = (int64_t)blockIdx.x * a.spb;
    if (b0 >= a.batch) return;
    const int nb = (int)((a.batch - b0) < a.spb ? (a.batch - b0) : a.spb);
    const int64_t e_begin = b0 * a.n_up, e_end = (b0 + nb) * a.n_up;

    for (int i = tid; i < nb * a.n_lo; i += EPB) {
        const int s = i / a.n_lo, q = i - s * a.n_lo;
        a.gx[(b0 + s) * a.ldgx + a.lo_in[q]] =
            a.gz != nullptr ? a.gz[(b0 + s) * a.ldgz + a.lo_out[q]] : 0.0f;
    }

    for (int64_t e0 = e_begin; e0 < e_end; e0 += EPB) {
        const int cnt = (int)((e_end - e0) < EPB ? (e_end - e0) : EPB);
        const int n = cnt * P;
        __syncthreads();
        {
            const float* src = a.params + e0 * P;
            if ((((uintptr_t)src) & 15) == 0) {
                const int n4 = n >> 2;
                const float4* s4 = reinterpret_cast<const float4*>(src);
                for (int i = tid; i < n4; i += EPB) reinterpret_cast<float4*>(sp)[i] = s4[i];
                for (int i = (n4 << 2) + tid; i < n; i += EPB) sp[i] = src[i];
            } else {
                for (int i = tid; i < n; i += EPB) sp[i] = src[i];
            }
        }
        __syncthreads();
        if (tid < cnt) {
            const int64_t e = e0 + tid;
            const int64_t b = e / a.n_up;
            const int j = (int)(e - b * a.n_up);
            const float xv = a.x[b * a.ldx + a.up_in[j]];
            const float go = a.gz != nullptr ? a.gz[b * a.ldgz + a.up_out[j]] : 0.0f;
            const float gl = a.gld != nullptr ? a.gld[b] : 0.0f;
            float wr[K], hr[K], dr[DN];
            float* p = sp + tid * P;
#pragma unroll
            for (int i = 0; i < K; ++i) wr[i] = p[i];
#pragma unroll
            for (int i = 0; i < K; ++i) hr[i] = p[K + i];
#pragma unroll
            for (int i = 0; i < P - 2 * K; ++i) dr[i] = p[2 * K + i];
            const float gxv = rqs_element_bwd<K, INV, PRE, DFULL>(xv, wr, hr, dr, a.c, go, gl);
            a.gx[b * a.ldgx + a.up_in[j]] = gxv;
#pragma unroll
            for (int i = 0; i < K; ++i) p[i] = wr[i];
#pragma unroll
            for (int i = 0; i < K; ++i) p[K + i] = hr[i];
#pragma unroll
            for (int i = 0; i < P - 2 * K; ++i) p[2 * K + i] = dr[i];
        }
        __syncthreads();
        {
            float* dst = a.gparams + e0 * P;
            if ((((uintptr_t)dst) & 15) == 0) {
                const int n4 = n >> 2;
                float4* d4 = reinterpret_cast<float4*>(dst);
                for (int i = tid; i < n4; i += EPB) d4[i] = reinterpret_cast<const float4*>(sp)[i];
                for (int i = (n4 << 2) + tid; i < n; i += EPB) dst[i] = sp[i];
            } else {
                for (int i = tid; i < n; i += EPB) dst[i] = sp[i];
            }
        }
    }
}

template <int K, bool INV, bool PRE, bool DFULL>
int launch_bwd_k(RqsBwdArgs a, hipStream_t st) {
    constexpr int P = DFULL ? 3 * K + 1 : 3 * K - 1;
    constexpr int EPB = (P <= 49) ? 256 : (P <= 97 ? 128 : 64);
    a.spb = a.n_up <= EPB ? EPB / a.n_up : 1;
    const int64_t blocks = (a.batch + a.spb - 1) / a.spb;
    if (blocks == 0) return 0;
    const size_t lds = (size_t)EPB * P * sizeof(float);
    hipLaunchKernelGGL((k_rqs_coupling_bwd<K, INV, PRE, DFULL, EPB>), dim3((unsigned)blocks),
                       dim3(EPB), lds, st, a);
    return launch_status("nfk_rqs_coupling_bwd");
}

template <int K>
int launch_bwd_modes(RqsBwdArgs a, bool inv, int mode, hipStream_t st) {
    if (inv) {
        if (mode == 0) return launch_bwd_k<K, true, true, false>(a, st);
        if (mode == 1) return launch_bwd_k<K, true, false, false>(a, st);
        return launch_bwd_k<K, true, false, true>(a, st);
    }
    if (mode == 0) return launch_bwd_k<K, false, true, false>(a, st);
    if (mode == 1) return launch_bwd_k<K, false, false, false>(a, st);
    return launch_bwd_k<K, false, false, true>(a, st);
}

}  // namespace

#define NFK_BWD_KLIST(X) \
    X(2) X(3) X(4) X(5) X(6) X(7) X(8) X(9) X(10) X(11) X(12) X(16) X(20) X(24) X(32)

extern "C" int nfk_rqs_coupling_bwd(const float* x, int64_t ldx, const float* params,
                                    const int32_t* up_in, const int32_t* up_out, int32_t n_up,
                                    const int32_t* lo_in, const int32_t* lo_out, int32_t n_lo,
                                    const float* gz, int64_t ldgz, const float* glogdet,
                                    float* gparams, float* gx, int64_t ldgx, int64_t batch,
                                    int32_t K, double left, double right, double bottom,
                                    double top, int32_t tails, double min_bin_width,
                                    double min_bin_height, double min_derivative,
                                    int32_t param_mode, int32_t inverse, nfk_stream_t stream) {
    if (batch < 0 || n_up <= 0 || n_lo < 0) return nfk_set_error("nfk_rqs_coupling_bwd: bad sizes");
    if (batch == 0) return 0;
    if (x == nullptr || params == nullptr || gparams == nullptr || gx == nullptr ||
        up_in == nullptr || up_out == nullptr)
        return nfk_set_error("nfk_rqs_coupling_bwd: null pointer");
    if (n_lo > 0 && (lo_in == nullptr || lo_out == nullptr))
        return nfk_set_error("nfk_rqs_coupling_bwd: null lower index map");
    if (param_mode < 0 || param_mode > 2) return nfk_set_error("nfk_rqs_coupling_bwd: bad param_mode");
    RqsBwdArgs a{x, ldx, params, up_in, up_out, n_up, lo_in, lo_out, n_lo, gz, ldgz, glogdet,
                 gparams, gx, ldgx, batch, 1,
                 nfk_make_const(K, left, right, bottom, top, tails, min_bin_width, min_bin_height,
                                min_derivative)};
    hipStream_t st = (hipStream_t)stream;
    const bool inv = inverse != 0;
    switch (K) {
#define NFK_CASE(k) \
    case k: return launch_bwd_modes<k>(a, inv, param_mode, st);
        NFK_BWD_KLIST(NFK_CASE)
#undef NFK_CASE
        default: break;
    }
    return nfk_set_error("nfk_rqs_coupling_bwd: unsupported K (supported: 2-12, 16, 20, 24, 32)");
}
