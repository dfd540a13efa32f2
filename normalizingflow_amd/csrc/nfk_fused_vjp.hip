// nfk_fused_vjp.hip -- training backward of one NSF_CL layer, recompute and
// spline VJP fused (nf/flows.py:227-253 differentiated, nf/utils.py:58-152):
// per 16-sample wave the conditioner FCNN (flows.py:20-35) is recomputed on
// the matrix cores exactly as the forward kernel computes it (same pack
// arithmetic, so the same logits), and the rational-quadratic spline's
// vector-Jacobian product (nfk_spline_bwd.h) is evaluated on the logits while
// they are in registers.  Written: dL/dparams [B, n_up, 3K-1] (the input of
// the conditioner's own backward GEMMs), dL/dx (upper coordinates through the
// spline, lower ones the identity part gz), and the two tanh activations
// [h | 1] that the weight-gradient GEMMs consume.  What it replaces per layer:
// the recompute GEMMs + elementwise tanh, and the [B, n_up, 3K-1] logits' HBM
// round trip into nfk_rqs_coupling_bwd.
//
// Layout: the output layer in 8-coordinate chunks (the wide record layout,
// nfk_fused_impl.h: lane group q holds coordinates 8c + 2q, 8c + 2q + 1 with
// ALL their parameters in registers 2h, 2h + 1 of the W, H and D tiles), so
// one lane has every logit of its two coordinates at once for the element
// backward.  The records are re-cut into kVNS-tile sub-records of SB blocks
// (the pack's VJP stream) and double-buffered through two LDS slots with one
// barrier per sub-record (the RealNVP chain's schedule, nfk_fused_rnvp.hip).
#ifndef NFK_VJP_FAST
#define NFK_VJP_FAST 1  // hardware exp / rcp and an fp32 knot cumsum in the element backward
#endif
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdint>

#include "../../include/nfk.h"
#include "nfk_spline.h"

int nfk_set_error(const char* msg);
NfkSplineConst nfk_make_const(int K, double left, double right, double bottom, double top,
                              int tails, double min_w, double min_h, double min_d);

#include "nfk_fused_impl.h"
#include "nfk_spline_bwd.h"

namespace nfk_fused {

struct VjpArgs {
    const float* x;
    const float* stream;  // the pack's VJP stream (sub-records in execution order)
    const float* hdr;     // the pack's header block (unscale factors)
    const int32_t *up_in, *up_out, *lo_in, *lo_out;
    const float* gz;      // nullable: dL/dz [B, D]
    const float* gld;     // nullable: dL/dlog|det| [B]
    float* gp;            // [B, n_up * (3K - 1)]
    float* gx;            // [B, D]
    float *h1, *h2;       // [B, ldh]: tanh activations in columns [0, H), 1 at column H
    int64_t ldx, ldgz, ldgx, ldh, batch;
    int32_t n_lo, n_up, H, NCH, nsub;  // NCH: 8-coordinate chunks; nsub: sub-records per launch
    NfkSplineConst c;
};

// parts J.. of a kVNS-tile record GEMM in the alternating slots (cur: slot of
// the next part, flipped by each step)
template <int KBH, bool T1, int NT, int J, class Step>
__device__ __forceinline__ void vjp_parts(const h8 (&bh)[KBH], const h8 (&bl)[KBH], h4 bt, float4* s0, float4* s1,
                                          int& cur, int lane, f32x4 (&acc)[NT], Step&& step) {
    constexpr int T0 = J * kVNS;
    constexpr int N = (NT - T0) < kVNS ? (NT - T0) : kVNS;
    float4* const sl = cur ? s1 : s0;
    gemm_h<KBH, T1, N, kVNS, T0, NT>(bh, bl, bt, sl, lane, acc);
    step(sl);
    cur ^= 1;
    if constexpr (T0 + kVNS < NT) vjp_parts<KBH, T1, NT, J + 1>(bh, bl, bt, s0, s1, cur, lane, acc, step);
}

// hidden activations (scaled tanh in h[][], see act_operands) -> row b of out:
// tile t < 2 KBH holds features 32 (t >> 1) + 8 q + 4 (t & 1) + r; the tail tile
// features 32 KBH + r (r < H - 32 KBH, from lane group 0); 1 at column H
template <int KBH, bool T1, int HT>
__device__ __forceinline__ void store_act(const f32x4 (&h)[HT], float* row, int q, int H) {
    constexpr float un = 1.0f / kActScale;
#pragma unroll
    for (int t = 0; t < 2 * KBH; ++t)
        *reinterpret_cast<float4*>(row + 32 * (t >> 1) + 8 * q + 4 * (t & 1)) =
            make_float4(h[t][0] * un, h[t][1] * un, h[t][2] * un, h[t][3] * un);
    if constexpr (T1) {
        if (q == 0)
#pragma unroll
            for (int r = 0; r < 4; ++r)
                if (32 * KBH + r < H) row[32 * KBH + r] = h[HT - 1][r] * un;
    }
    if (q == 1) row[H] = 1.0f;
}

#ifdef NFK_VJP_DIAG_SAVE  // diagnostic: every element backward's inputs, [B][n_up][3K + 2] floats
__device__ float* g_vjp_dbg;
extern "C" int nfk_vjp_diag_set(float* p) {
    return (int)hipMemcpyToSymbol(HIP_SYMBOL(g_vjp_dbg), &p, sizeof(p), 0, hipMemcpyHostToDevice);
}
#endif
#ifdef NFK_VJP_DIAG_TWICE  // diagnostic: per-lane counts of elements whose two evaluations differed
__device__ int g_vjp_cnt[64 + 80];  // per-lane mismatches, then per first-differing probe slot
extern "C" int nfk_vjp_diag_counts(int* host, int reset) {
    int rc = (int)hipMemcpyFromSymbol(host, HIP_SYMBOL(g_vjp_cnt), sizeof(g_vjp_cnt), 0, hipMemcpyDeviceToHost);
    if (reset) {
        static const int zero[64 + 80] = {0};
        rc |= (int)hipMemcpyToSymbol(HIP_SYMBOL(g_vjp_cnt), zero, sizeof(zero), 0, hipMemcpyHostToDevice);
    }
    return rc;
}
#endif

template <int KBH, bool T1, int K, bool INV>
__global__ __launch_bounds__(64 * kNsfWaves, 3) void k_nsf_vjp(VjpArgs a) {
    constexpr VjpDims d = vjp_dims(KBH, T1 ? 1 : 0, K);
    constexpr int HT = d.HT, SB = d.SB, KW = d.KW, KD = d.KD, P = 3 * K - 1;
    const int lane = threadIdx.x & 63;
    const int wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int q = lane >> 4, sl = lane & 15;
    const int n_lo = a.n_lo, n_up = a.n_up, D = n_lo + n_up, XS = D + 1;
    extern __shared__ __attribute__((aligned(16))) float4 lds4[];
    float4* const slot0 = lds4;
    float4* const slot1 = lds4 + SB * 64;
    int32_t* const m_up_in = reinterpret_cast<int32_t*>(lds4 + 2 * SB * 64);
    int32_t* const m_up_out = m_up_in + n_up;
    int32_t* const m_lo_in = m_up_out + n_up;
    int32_t* const m_lo_out = m_lo_in + n_lo;
    float* const tile = reinterpret_cast<float*>(lds4 + 2 * SB * 64 + (2 * D + 3) / 4) + wid * 16 * XS;
    const int64_t b0 = ((int64_t)blockIdx.x * kNsfWaves + wid) * 16;
    const int64_t rem = a.batch - b0;
    const int nrows = rem <= 0 ? 0 : (rem < 16 ? (int)rem : 16);
    const bool row_ok = sl < nrows;
    // rows past the batch compute on the wave's first row (as the forward
    // kernel, so the input scale and hence the logits match it) and
    // store nothing
    const int64_t brow0 = nrows > 0 ? b0 : 0;
    const int64_t b = row_ok ? b0 + sl : brow0;

    int nsub = 0;  // next sub-record to copy
    auto stage_next = [&](float4* slot) {
        if (nsub >= a.nsub) return;
        const float* src = a.stream + (int64_t)nsub * SB * 256;
#ifdef NFK_VJP_DIAG_PLAIN  // diagnostic: plain loads + ds_write instead of LDS-DMA
#pragma unroll
        for (int i = 0; i < SB / 4; ++i)
            slot[(wid + 4 * i) * 64 + lane] = *reinterpret_cast<const float4*>(src + (int64_t)(wid + 4 * i) * 256 + lane * 4);
#else
        const uint32_t base = lds_addr(slot);
#pragma unroll
        for (int i = 0; i < SB / 4; ++i)
            dma16(src + (int64_t)(wid + 4 * i) * 256 + lane * 4, base + (wid + 4 * i) * 1024);
#endif
        ++nsub;
    };
    auto step = [&](float4* freed) {
#ifndef NFK_VJP_NO_FENCE
        gemm_fence();
#endif
        asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_barrier();
        asm volatile("" ::: "memory");
        stage_next(freed);
    };

    // ---- prologue: maps and the wave's x rows (plain loads), the first two
    // sub-records by LDS-DMA, one wait
    for (int i = threadIdx.x; i < n_up; i += 64 * kNsfWaves) {
        m_up_in[i] = a.up_in[i];
        m_up_out[i] = a.up_out[i];
    }
    for (int i = threadIdx.x; i < n_lo; i += 64 * kNsfWaves) {
        m_lo_in[i] = a.lo_in[i];
        m_lo_out[i] = a.lo_out[i];
    }
    for (int i = lane; i < 16 * D; i += 64) {
        const int r = i / D, c = i - r * D;
        tile[r * XS + c] = a.x[(r < nrows ? b0 + r : brow0) * a.ldx + c];
    }
    stage_next(slot0);
    stage_next(slot1);
    asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    int cur = 0;
    const float un1 = a.hdr[3], un2 = a.hdr[4], un3 = a.hdr[5];

    // ---- layer 1 (one k-block: n_lo <= 32), per-sample power-of-two scaled x (each row its own exponent: rows stay independent)
    h8 bh[KBH], bl[KBH];
    h4 bt;
    {
        float e[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            const int k = 8 * q + j;
            e[j] = k < n_lo ? tile[sl * XS + m_lo_in[k]] : 0.0f;
        }
        float mx = 0.0f;
#pragma unroll
        for (int j = 0; j < 8; ++j) mx = fmaxf(mx, fabsf(e[j]));
#pragma unroll
        for (int off = 16; off < 64; off <<= 1) mx = fmaxf(mx, __shfl_xor(mx, off, 64));  // per sample: the 4 lanes of column sl
        int ex = 0;
        if (mx > 0.0f && mx < 3.0e38f) frexpf(mx, &ex);
        ex = ex < -64 ? -64 : ex;  // a tiny sample: its scale 2^(14 - ex) and bias scale stay finite
        const float sx = ldexpf(1.0f, 14 - ex);
        h8 xh[1], xl[1];
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            const float v = e[j] * sx;
            const _Float16 hh = (_Float16)v;
            xh[0][j] = hh;
            xl[0][j] = (_Float16)(v - (float)hh);
        }
        const float unx = ldexpf(un1, ex - 14);
        f32x4 h1[HT];
        input_gemm<1, HT>(xh, xl, slot0, 1.0f / unx, lane, h1);
        step(slot0);
        cur = 1;
        act_operands<KBH, T1, HT>(h1, -2.0f * kL2E * unx, bh, bl, bt);
        if (row_ok) store_act<KBH, T1, HT>(h1, a.h1 + b * a.ldh, q, a.H);
    }
    // ---- layer 2
    {
        f32x4 h2[HT];
        vjp_parts<KBH, T1, HT, 0>(bh, bl, bt, slot0, slot1, cur, lane, h2, step);
        act_operands<KBH, T1, HT>(h2, -2.0f * kL2E * un2, bh, bl, bt);
        if (row_ok) store_act<KBH, T1, HT>(h2, a.h2 + b * a.ldh, q, a.H);
    }
    const float gl = (a.gld != nullptr) ? a.gld[b] : 0.0f;
#ifdef NFK_VJP_DIAG_VGPRC  // diagnostic: the spline constants in VGPRs (no SGPR pressure from them)
    NfkSplineConst cc = a.c;
    asm volatile("" : "+v"(cc.scale2b), "+v"(cc.lo), "+v"(cc.hi), "+v"(cc.span), "+v"(cc.ylo), "+v"(cc.yhi),
                 "+v"(cc.yspan), "+v"(cc.min_w), "+v"(cc.fw), "+v"(cc.min_h), "+v"(cc.fh));
    asm volatile("" : "+v"(cc.min_d), "+v"(cc.dpad), "+v"(cc.knot_eps), "+v"(cc.m2b), "+v"(cc.d_edge));
#else
    const NfkSplineConst& cc = a.c;
#endif
#ifdef NFK_VJP_DIAG_NOP
#define NFK_VJP_NOPS() do { __builtin_amdgcn_sched_barrier(0); \
        asm volatile("s_nop 7\n\ts_nop 7\n\ts_nop 7\n\ts_nop 7\n\ts_nop 7\n\ts_nop 7"); \
        __builtin_amdgcn_sched_barrier(0); } while (0)
#else
#define NFK_VJP_NOPS() do { } while (0)
#endif
    // ---- output layer in 8-coordinate chunks: W, H, D logits of the lane's two
    // coordinates in registers, then the spline VJP of each
    for (int ch = 0; ch < a.NCH; ++ch) {
        f32x4 aw[KW], ah[KW], ad[KD];
        vjp_parts<KBH, T1, KW, 0>(bh, bl, bt, slot0, slot1, cur, lane, aw, step);
        vjp_parts<KBH, T1, KW, 0>(bh, bl, bt, slot0, slot1, cur, lane, ah, step);
        vjp_parts<KBH, T1, KD, 0>(bh, bl, bt, slot0, slot1, cur, lane, ad, step);
        NFK_VJP_NOPS();
#pragma unroll
        for (int cb = 0; cb < 2; ++cb) {
            const int j = 8 * ch + 2 * q + cb;
            if (j >= n_up) continue;
            // register 2 cb + p of tile t = parameter 2 t + p of this coordinate
            float wr[K], hr[K], dr[K - 1];
#pragma unroll
            for (int i = 0; i < K; ++i) {
                wr[i] = aw[i >> 1][2 * cb + (i & 1)] * un3;
                hr[i] = ah[i >> 1][2 * cb + (i & 1)] * un3;
                if (i < K - 1) dr[i] = ad[i >> 1][2 * cb + (i & 1)] * un3;
            }
            const float xv = tile[sl * XS + m_up_in[j]];
            const float go = (a.gz != nullptr) ? a.gz[b * a.ldgz + m_up_out[j]] : 0.0f;
#ifdef NFK_VJP_DIAG_SAVE
            if (row_ok) {
                float* sv = g_vjp_dbg + (b * n_up + j) * (3 * K + 2);
#pragma unroll
                for (int i = 0; i < K; ++i) sv[i] = wr[i];
#pragma unroll
                for (int i = 0; i < K; ++i) sv[K + i] = hr[i];
#pragma unroll
                for (int i = 0; i < K - 1; ++i) sv[2 * K + i] = dr[i];
                sv[3 * K - 1] = xv;
                sv[3 * K] = go;
                sv[3 * K + 1] = gl;
            }
#ifdef NFK_VJP_DIAG_RELOAD  // diagnostic: the element backward runs on the values just stored, re-read
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            {
                volatile const float* rv = g_vjp_dbg + (b * n_up + j) * (3 * K + 2);
#pragma unroll
                for (int i = 0; i < K; ++i) wr[i] = rv[i];
#pragma unroll
                for (int i = 0; i < K; ++i) hr[i] = rv[K + i];
#pragma unroll
                for (int i = 0; i < K - 1; ++i) dr[i] = rv[2 * K + i];
            }
#endif
#endif
#ifdef NFK_VJP_DUMP  // diagnostic: the element backward's inputs instead of its outputs
            const float gxv = xv + 1000.0f * go + 1.0e6f * gl;
#else
#ifdef NFK_VJP_DIAG_TWICE  // diagnostic: the element backward twice on the same registers; mismatches counted
            float w2[K], h2[K], d2[K - 1];
#pragma unroll
            for (int i = 0; i < K; ++i) w2[i] = wr[i], h2[i] = hr[i];
#pragma unroll
            for (int i = 0; i < K - 1; ++i) d2[i] = dr[i];
#ifdef NFK_BWD_PROBE
            float pr1[nfk_bwd::kProbeSlots], pr2[nfk_bwd::kProbeSlots];
#pragma unroll
            for (int i = 0; i < nfk_bwd::kProbeSlots; ++i) pr1[i] = pr2[i] = 0.0f;
#define NFK_PA1 , pr1
#define NFK_PA2 , pr2
#else
#define NFK_PA1
#define NFK_PA2
#endif
            const float gx2 = nfk_bwd::rqs_element_bwd<K, INV, true, false, NFK_VJP_FAST>(xv, w2, h2, d2, cc, go, gl NFK_PA2);
            asm volatile("" ::: "memory");
#endif
#ifndef NFK_PA1
#define NFK_PA1
#endif
            const float gxv = nfk_bwd::rqs_element_bwd<K, INV, true, false, NFK_VJP_FAST>(xv, wr, hr, dr, cc, go, gl NFK_PA1);
#ifdef NFK_VJP_DIAG_TWICE
            {
                bool same = __float_as_uint(gx2) == __float_as_uint(gxv);
#pragma unroll
                for (int i = 0; i < K; ++i) same = same && __float_as_uint(w2[i]) == __float_as_uint(wr[i]);
                if (!same && row_ok) atomicAdd(g_vjp_cnt + lane, 1);
#ifdef NFK_BWD_PROBE
                // the first intermediate (in computation order) where the two evaluations part
                int first = -1;
#pragma unroll
                for (int i = nfk_bwd::kProbeSlots - 1; i >= 0; --i)
                    first = __float_as_uint(pr1[i]) != __float_as_uint(pr2[i]) ? i : first;
                if (first >= 0 && row_ok) atomicAdd(g_vjp_cnt + 64 + first, 1);
#endif
            }
#endif
#endif
            if (row_ok) {
                a.gx[b * a.ldgx + m_up_in[j]] = gxv;
                float* g = a.gp + (b * n_up + j) * P;
#pragma unroll
                for (int i = 0; i < K; ++i) g[i] = wr[i];
#pragma unroll
                for (int i = 0; i < K; ++i) g[K + i] = hr[i];
#pragma unroll
                for (int i = 0; i < K - 1; ++i) g[2 * K + i] = dr[i];
            }
        }
        NFK_VJP_NOPS();
    }
    // ---- lower coordinates: the identity part of dL/dx (flows.py:239)
    for (int i = lane; i < 16 * n_lo; i += 64) {
        const int r = i / n_lo, k = i - r * n_lo;
        if (r < nrows)
            a.gx[(b0 + r) * a.ldgx + m_lo_in[k]] = a.gz != nullptr ? a.gz[(b0 + r) * a.ldgz + m_lo_out[k]] : 0.0f;
    }
}

template <int KBH, int T1, int K>
int launch_vjp(const VjpArgs& a, bool inv, hipStream_t st) {
    const int64_t blocks = (a.batch + kNsfWaves * 16 - 1) / (kNsfWaves * 16);
    if (blocks == 0) return 0;
#ifdef NFK_VJP_DIAG_ONEWG  // diagnostic: LDS padded so that one workgroup runs per CU
    const size_t lds = 96 * 1024;
    hipFuncSetAttribute(reinterpret_cast<const void*>(&k_nsf_vjp<KBH, T1 != 0, K, false>),
                        hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    hipFuncSetAttribute(reinterpret_cast<const void*>(&k_nsf_vjp<KBH, T1 != 0, K, true>),
                        hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
#else
    const size_t lds = vjp_lds_bytes(vjp_dims(KBH, T1, K), a.n_lo + a.n_up);
#endif
    if (inv)
        hipLaunchKernelGGL((k_nsf_vjp<KBH, T1 != 0, K, true>), dim3((unsigned)blocks), dim3(64 * kNsfWaves), lds,
                           st, a);
    else
        hipLaunchKernelGGL((k_nsf_vjp<KBH, T1 != 0, K, false>), dim3((unsigned)blocks), dim3(64 * kNsfWaves), lds,
                           st, a);
    const hipError_t e = hipGetLastError();
    return e == hipSuccess ? 0 : (int)e;
}

}  // namespace nfk_fused

using namespace nfk_fused;

extern "C" int nfk_fused_nsf_vjp(const float* x, int64_t ldx, const float* vpack, const int32_t* up_in,
                                 const int32_t* up_out, int32_t n_up, const int32_t* lo_in, const int32_t* lo_out,
                                 int32_t n_lo, int32_t hidden, const float* gz, int64_t ldgz, const float* glogdet,
                                 float* gparams, float* gx, int64_t ldgx, float* h1, float* h2, int64_t ldh,
                                 int64_t batch, int32_t K, double tail_bound, int32_t inverse, nfk_stream_t stream) {
    if (!vjp_ok(n_lo, n_up, hidden, K)) return nfk_set_error("nfk_fused_nsf_vjp: shape not supported");
    if (batch < 0) return nfk_set_error("nfk_fused_nsf_vjp: bad batch");
    if (batch == 0) return 0;
    if (!x || !vpack || !up_in || !up_out || !lo_in || !lo_out || !gparams || !gx || !h1 || !h2)
        return nfk_set_error("nfk_fused_nsf_vjp: null pointer");
    if (ldh < hidden + 1 || ldh % 4 != 0 || ((uintptr_t)h1 % 16) != 0 || ((uintptr_t)h2 % 16) != 0)
        return nfk_set_error("nfk_fused_nsf_vjp: h1/h2 rows must hold hidden + 1 floats, 16-byte aligned");
    const Layout L = make_layout(n_lo, n_up, hidden, K, 1);
    const VjpDims dd = vjp_dims(L.KBH, L.T1, K);
    VjpArgs a;
    a.x = x;
    a.stream = vpack + L.total;
    a.hdr = vpack;
    a.up_in = up_in;
    a.up_out = up_out;
    a.lo_in = lo_in;
    a.lo_out = lo_out;
    a.gz = gz;
    a.gld = glogdet;
    a.gp = gparams;
    a.gx = gx;
    a.h1 = h1;
    a.h2 = h2;
    a.ldx = ldx;
    a.ldgz = ldgz;
    a.ldgx = ldgx;
    a.ldh = ldh;
    a.batch = batch;
    a.n_lo = n_lo;
    a.n_up = n_up;
    a.H = hidden;
    a.NCH = L.NCH;
    a.nsub = vjp_nsub(dd, L.NCH);
    a.c = nfk_make_const(K, -tail_bound, tail_bound, -tail_bound, tail_bound, 1, 1e-3, 1e-3, 1e-3);
    hipStream_t st = (hipStream_t)stream;
    const bool inv = inverse != 0;
#define VDISPATCH(h, t, k) \
    if (L.KBH == h && L.T1 == t && K == k) return launch_vjp<h, t, k>(a, inv, st);
    NFK_VJP_SHAPES(VDISPATCH)
#undef VDISPATCH
    return nfk_set_error("nfk_fused_nsf_vjp: no kernel instance");
}
