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
#include "nfk_spline_bwd.h"

int nfk_set_error(const char* msg);
NfkSplineConst nfk_make_const(int K, double left, double right, double bottom, double top,
                              int tails, double min_w, double min_h, double min_d);

namespace {

using namespace nfk_bwd;

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
