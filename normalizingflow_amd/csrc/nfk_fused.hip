// nfk_fused.hip -- one launch per NSF coupling layer: conditioner MLP
// (FCNN, nf/flows.py:20-35) on fp32 MFMA + rational-quadratic spline epilogue
// (nf/flows.py:227-253, nf/utils.py:27-152).  The [B, n_up, 3K-1] conditioner
// output never leaves registers.
//
// Work decomposition: one wave owns ST tiles of 16 samples.  All products
// are computed transposed, h^T[feature][sample] = W . act^T, with
// v_mfma_f32_16x16x4_f32 (exact fp32: a k-ordered fmaf chain):
//   A operand = weights   (lane l: W[row l&15][k l>>4]),
//   B operand = activations (lane l: act[k l>>4][sample l&15]),
//   D: lane l, register r = output row 4*(l>>4)+r of sample l&15.
// Hidden feature f of tile t sits in row 4*r+q... precisely: row i = 4q + r of
// tile t holds feature 16t + 4r + q, so register r of tile t IS the B
// fragment of k-step 4t + r (features 4ks + q) of the next product -- no LDS
// transpose between layers.
//
// Output layer: per chunk of 16 coordinates the 3K-1 parameter tiles are
// produced in three phases (W logits, H logits, D logits; H first when
// inverting).  Row i of a parameter tile is coordinate jbase + i, so lane l
// holds, for sample l&15, all K logits of coordinates jbase + 4q + r in
// registers and evaluates the spline there (same fp32 op order as
// nfk_spline.h).  Per-sample log|det| is reduced across the four lane groups
// with xor-16/32 shuffles.
//
// Weights are packed once per weight version (nfk_fused_nsf_pack) in MFMA
// fragment order, 4 tiles per float4, so every A fragment is one coalesced
// 16-B load that feeds 4 x ST MFMAs; a register ring keeps kPF k-steps of
// weights in flight.  The hidden k-step count is a template parameter, so the
// whole chain is branch-free straight-line code the scheduler can pipeline.  The x tile and the output z tile are
// staged through a per-wave LDS region so HBM sees only full-row accesses.
#include <hip/hip_runtime.h>

#include <cstdint>

#include "../../include/nfk.h"
#include "nfk_spline.h"

int nfk_set_error(const char* msg);
NfkSplineConst nfk_make_const(int K, double left, double right, double bottom, double top,
                              int tails, double min_w, double min_h, double min_d);

#include "nfk_fused_impl.h"

using namespace nfk_fused;

namespace nfk_fused {
#define NFK_X(h) NFK_FUSED_K(NFK_FUSED_EXTERN, h)
NFK_FUSED_KSH(NFK_X)
#undef NFK_X
}  // namespace nfk_fused

namespace {

struct PackArgs {
    const float *w0, *b0, *w2, *b2, *w4, *b4;
    float* out;
    Layout L;
};

// One thread per packed float (layout described at make_layout()).
__device__ float pack_hidden(const float* W, const float* bias, int KS, int kin, int H, int TGH, int HT,
                             int blk, int lane, int e) {
    if (blk < KS * TGH) {
        const int ks = blk / TGH, g = blk - ks * TGH, t = 4 * g + e;
        const int f = hid_row(t, lane & 15), k = 4 * ks + (lane >> 4);
        return (t < HT && f < H && k < kin) ? W[(int64_t)f * kin + k] : 0.0f;
    }
    const int t = blk - KS * TGH, f = 16 * t + 4 * e + (lane >> 4);  // bias: register e of tile t
    return f < H ? bias[f] : 0.0f;
}

__global__ __launch_bounds__(256) void k_pack(PackArgs a) {
    const Layout& L = a.L;
    for (int64_t g = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; g < L.total;
         g += (int64_t)gridDim.x * blockDim.x) {
        const int e = (int)(g & 3), lane = (int)((g >> 2) & 63);
        float v;
        if (g < L.o_h2) {
            v = pack_hidden(a.w0, a.b0, L.KS1, L.n_lo, L.H, L.TGH, L.HT, (int)(g >> 8), lane, e);
        } else if (g < L.o_w3) {
            v = pack_hidden(a.w2, a.b2, L.KSH, L.H, L.H, L.TGH, L.HT, (int)((g - L.o_h2) >> 8), lane, e);
        } else {
            const int64_t bl = (g - L.o_w3) >> 8;
            const int c = (int)(bl / L.blk_chunk);
            int b = (int)(bl - (int64_t)c * L.blk_chunk);
            int ng = L.TGK, nt = L.K, pbase = 0;
            if (b >= L.blk_w) {
                b -= L.blk_w;
                pbase = L.K;
                if (b >= L.blk_w) {
                    b -= L.blk_w;
                    pbase = 2 * L.K;
                    ng = L.TGD;
                    nt = L.K - 1;
                }
            }
            v = 0.0f;
            if (b < L.KSH * ng) {
                const int ks = b / ng, gg = b - ks * ng, t = 4 * gg + e;
                const int j = 16 * c + (lane & 15), k = 4 * ks + (lane >> 4);
                if (t < nt && j < L.n_up && k < L.H) v = a.w4[((int64_t)j * L.P + pbase + t) * L.H + k];
            } else {
                const int t = b - L.KSH * ng, j = 16 * c + 4 * (lane >> 4) + e;
                if (t < nt && j < L.n_up) v = a.b4[(int64_t)j * L.P + pbase + t];
            }
        }
        a.out[g] = v;
    }
}

bool shape_ok(int n_lo, int n_up, int H, int K) {
    if (n_lo < 1 || n_up < 1 || n_lo + n_up > kMaxD || H < 1 || K < 2) return false;
    if (lds_bytes(make_layout(n_lo, n_up, H, K)) > (size_t)kLdsBytes) return false;
    const int KSH = (H + 3) / 4;
    bool ks = false, kk = false;
#define CHK_KSH(h) ks |= (KSH == h);
    NFK_FUSED_KSH(CHK_KSH)
#undef CHK_KSH
#define CHK_K(h, k) kk |= (K == k);
    NFK_FUSED_K(CHK_K, 0)
#undef CHK_K
    return ks && kk;
}

}  // namespace

extern "C" int nfk_fused_nsf_supported(int32_t n_lo, int32_t n_up, int32_t hidden, int32_t K) {
    return shape_ok(n_lo, n_up, hidden, K) ? 1 : 0;
}

extern "C" int64_t nfk_fused_nsf_pack_elems(int32_t n_lo, int32_t n_up, int32_t hidden, int32_t K) {
    if (!shape_ok(n_lo, n_up, hidden, K)) return 0;
    return make_layout(n_lo, n_up, hidden, K).total;
}

extern "C" int nfk_fused_nsf_pack(const float* w0, const float* b0, const float* w2, const float* b2,
                                  const float* w4, const float* b4, int32_t n_lo, int32_t n_up,
                                  int32_t hidden, int32_t K, float* wpack, nfk_stream_t stream) {
    if (!shape_ok(n_lo, n_up, hidden, K)) return nfk_set_error("nfk_fused_nsf_pack: shape not supported");
    if (!w0 || !b0 || !w2 || !b2 || !w4 || !b4 || !wpack)
        return nfk_set_error("nfk_fused_nsf_pack: null pointer");
    PackArgs a{w0, b0, w2, b2, w4, b4, wpack, make_layout(n_lo, n_up, hidden, K)};
    int64_t g = (a.L.total + 255) / 256;
    if (g > 8192) g = 8192;
    hipLaunchKernelGGL(k_pack, dim3((unsigned)g), dim3(256), 0, (hipStream_t)stream, a);
    hipError_t e = hipGetLastError();
    return e == hipSuccess ? 0 : (int)e;
}

extern "C" int nfk_fused_nsf(const float* x, int64_t ldx, const float* wpack, const int32_t* up_in,
                             const int32_t* up_out, int32_t n_up, const int32_t* lo_in,
                             const int32_t* lo_out, int32_t n_lo, int32_t hidden, float* z,
                             int64_t ldz, float* logdet, int32_t logdet_mode, int64_t batch,
                             int32_t K, double tail_bound, int32_t inverse, int32_t* status,
                             nfk_stream_t stream) {
    if (!shape_ok(n_lo, n_up, hidden, K)) return nfk_set_error("nfk_fused_nsf: shape not supported");
    if (batch < 0) return nfk_set_error("nfk_fused_nsf: bad batch");
    if (batch == 0) return 0;
    if (!x || !wpack || !up_in || !up_out || !lo_in || !lo_out || !z)
        return nfk_set_error("nfk_fused_nsf: null pointer");
    if (logdet_mode != 0 && !logdet) return nfk_set_error("nfk_fused_nsf: null logdet");
    const Layout L = make_layout(n_lo, n_up, hidden, K);
    FusedArgs a;
    a.x = x;
    a.pack = wpack;
    a.up_in = up_in;
    a.up_out = up_out;
    a.lo_in = lo_in;
    a.lo_out = lo_out;
    a.z = z;
    a.logdet = logdet;
    a.status = status;
    a.ldx = ldx;
    a.ldz = ldz;
    a.batch = batch;
    a.n_lo = n_lo;
    a.n_up = n_up;
    a.KS1 = L.KS1;
    a.NCH = L.NCH;
    a.mode = logdet_mode;
    a.slot_blocks = L.slot_blocks;
    a.blk_h1 = L.blk_h1;
    a.blk_h2 = L.blk_h2;
    a.blk_w = L.blk_w;
    a.blk_d = L.blk_d;
    a.blk_chunk = L.blk_chunk;
    a.o_h2 = (int32_t)L.o_h2;
    a.o_w3 = (int32_t)L.o_w3;
    a.c = nfk_make_const(K, -tail_bound, tail_bound, -tail_bound, tail_bound, 1, 1e-3, 1e-3, 1e-3);
    const size_t lds = lds_bytes(L);
    hipStream_t st = (hipStream_t)stream;
    const bool inv = inverse != 0;
    const int KSH = L.KSH;
#define DISPATCH(h, k) \
    if (KSH == h && K == k) return launch_fused<h, k>(a, lds, inv, st);
#define DISPATCH_KSH(h) NFK_FUSED_K(DISPATCH, h)
    NFK_FUSED_KSH(DISPATCH_KSH)
#undef DISPATCH_KSH
#undef DISPATCH
    return nfk_set_error("nfk_fused_nsf: no kernel instance");
}
