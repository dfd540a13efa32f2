// nfk_fused_impl.h -- fused NSF coupling-layer kernel; design notes in nfk_fused.hip.
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>

#include "../../include/nfk.h"
#include "nfk_spline.h"

typedef float f32x4 __attribute__((ext_vector_type(4)));

namespace nfk_fused {

constexpr int kWaves = 8;         // waves per workgroup (two per SIMD), 16 samples each
constexpr int kMaxD = 128;        // n_lo + n_up staged in LDS
constexpr int kLdsBytes = 160 * 1024;

// Packed weights: a stream of "phase records", each a run of 1-KiB blocks
// (64 lanes x float4) in MFMA fragment order: the weight blocks of the
// phase's KS k-steps x NG tile groups ([ks][g], 4 tiles per float4), then NT
// bias blocks (lane l, register r of tile t = bias of the row that lane holds).
//   hidden 1: KS1*TGH + HT blocks      hidden 2: KSH*TGH + HT blocks
//   per 16-coordinate chunk: W logits KSH*TGK + K, H logits KSH*TGK + K,
//                            D logits KSH*TGD + (K-1)
// The workgroup copies one record at a time into an LDS slot with
// global_load_lds (one wave-instruction per block), double-buffered.
struct Layout {
    int n_lo, n_up, H, K, P, HT, KS1, KSH, NCH, TGH, TGK, TGD;
    int blk_h1, blk_h2, blk_w, blk_d, blk_chunk, slot_blocks;
    int64_t o_h1, o_h2, o_w3, total;  // offsets / size in floats
};

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
    L.blk_h1 = L.KS1 * L.TGH + L.HT;
    L.blk_h2 = L.KSH * L.TGH + L.HT;
    L.blk_w = L.KSH * L.TGK + K;
    L.blk_d = L.KSH * L.TGD + (K - 1);
    L.blk_chunk = 2 * L.blk_w + L.blk_d;
    L.slot_blocks = L.blk_h1;
    if (L.blk_h2 > L.slot_blocks) L.slot_blocks = L.blk_h2;
    if (L.blk_w > L.slot_blocks) L.slot_blocks = L.blk_w;
    if (L.blk_d > L.slot_blocks) L.slot_blocks = L.blk_d;
    L.o_h1 = 0;
    L.o_h2 = (int64_t)L.blk_h1 * 256;
    L.o_w3 = L.o_h2 + (int64_t)L.blk_h2 * 256;
    L.total = L.o_w3 + (int64_t)L.NCH * L.blk_chunk * 256;
    return L;
}

// dynamic LDS bytes: two weight slots, the index maps, one x tile per wave
inline size_t lds_bytes(const Layout& L) {
    const int D = L.n_lo + L.n_up;
    const size_t maps = ((size_t)(2 * D) * sizeof(int32_t) + 15) & ~(size_t)15;
    return 2 * (size_t)L.slot_blocks * 1024 + maps + (size_t)kWaves * 16 * (D + 1) * sizeof(float);
}

// hidden feature held by MFMA row i (0..15) of tile t
__host__ __device__ inline int hid_row(int t, int i) { return 16 * t + 4 * (i & 3) + (i >> 2); }

struct FusedArgs {
    const float* x;
    const float* pack;
    const int32_t *up_in, *up_out, *lo_in, *lo_out;
    float* z;
    float* logdet;
    int32_t* status;
    int64_t ldx, ldz, batch;
    int32_t n_lo, n_up, KS1, NCH, mode, slot_blocks;
    int32_t blk_h1, blk_h2, blk_w, blk_d, blk_chunk;
    int32_t o_h2, o_w3;  // float offsets into pack (< 2^31 by shape limits)
    NfkSplineConst c;
};

__device__ __forceinline__ f32x4 mfma(float a, float b, f32x4 c) {
    return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
}

__device__ __forceinline__ float pick4(const float4& w, int e) {
    return e == 0 ? w.x : e == 1 ? w.y : e == 2 ? w.z : w.w;
}

__device__ __forceinline__ f32x4 as_f32x4(const float4& v) {
    f32x4 r;
    r[0] = v.x;
    r[1] = v.y;
    r[2] = v.z;
    r[3] = v.w;
    return r;
}

// Copy one phase record (nblk 1-KiB blocks at src) into an LDS slot: block i
// goes by wave i % kWaves as one global_load_lds_dwordx4 (LDS destination =
// wave-uniform base + 16 B x lane).  Completion is waited for by the
// workgroup barrier that precedes the slot's first read (vmcnt(0) + s_barrier).
__device__ __forceinline__ void stage_record(const float* __restrict__ src, int nblk, float4* slot,
                                             int wid, int lane) {
    for (int i = wid; i < nblk; i += kWaves)
        __builtin_amdgcn_global_load_lds(
            (const __attribute__((address_space(1))) void*)(src + (int64_t)i * 256 + lane * 4),
            (__attribute__((address_space(3))) void*)(slot + i * 64), 16, 0, 0);
}

// acc[t] = bias + W[tile t] . act^T over KS k-steps, A fragments and bias from
// an LDS slot; B fragment of k-step ks = act[ks>>2][ks&3].
template <int KS, int NT, int NG, int HTA>
__device__ __forceinline__ void gemm_lds(const f32x4 (&act)[HTA], const float4* slot, int lane,
                                         f32x4 (&acc)[NT]) {
    float4 cur[NG], nxt[NG];
#pragma unroll
    for (int g = 0; g < NG; ++g) cur[g] = slot[g * 64 + lane];
#pragma unroll
    for (int t = 0; t < NT; ++t) acc[t] = as_f32x4(slot[(KS * NG + t) * 64 + lane]);
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) {
        // A fragments of k-step ks+1 are read while k-step ks's MFMAs run
        if (ks + 1 < KS) {
#pragma unroll
            for (int g = 0; g < NG; ++g) nxt[g] = slot[((ks + 1) * NG + g) * 64 + lane];
        }
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int g = 0; g < NG; ++g) {
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                const int t = 4 * g + e;
                if (t < NT) acc[t] = mfma(pick4(cur[g], e), act[ks >> 2][ks & 3], acc[t]);
            }
        }
        if (ks + 1 < KS) {
#pragma unroll
            for (int g = 0; g < NG; ++g) cur[g] = nxt[g];
        }
    }
}

// Knot phase epilogue: for the 4 coordinates of this lane, turn the K logits
// of register r into knots (NSF_CL's 2B softmax, then RQS's softmax, floor and
// cumsum: nfk_knots_nsf_lean) and keep (edge_k, size_k) of the bin.  The
// searched phase finds the bin by a running select over the interior edges
// (edges are strictly increasing, so the last edge <= x is the bin of
// utils.py:20-25 for every x inside the tails); the other phase selects by k.
template <int K, bool SEARCH, bool Y>
__device__ __forceinline__ void knot_phase(const f32x4 (&acc)[K], const float (&xv)[4],
                                           const NfkSplineConst& c, int (&kb)[4], float (&ek)[4],
                                           float (&sk)[4]) {
#pragma unroll
    for (int r = 0; r < 4; ++r) {
        float u[K], edge[K + 1];
#pragma unroll
        for (int t = 0; t < K; ++t) u[t] = acc[t][r];
        if (Y)
            nfk_knots_nsf_lean<K>(u, c.ylo, c.yhi, c.yspan, c.min_h, c.fh, c.m2b, edge);
        else
            nfk_knots_nsf_lean<K>(u, c.lo, c.hi, c.span, c.min_w, c.fw, c.m2b, edge);
        float e = edge[0], e1 = edge[1];
        int k = 0;
#pragma unroll
        for (int j = 1; j < K; ++j) {
            const bool ge = SEARCH ? (xv[r] >= edge[j]) : (kb[r] >= j);
            e = ge ? edge[j] : e;
            e1 = ge ? edge[j + 1] : e1;
            if (SEARCH) k += ge ? 1 : 0;
        }
        if (SEARCH) kb[r] = k;
        ek[r] = e;
        sk[r] = e1 - e;
    }
}

// One workgroup = kWaves waves x 16 samples.  Phase records stream through
// two LDS slots: while phase p computes from slot p&1, the record of phase
// p+1 is already in the other slot and phase p+2's copy is issued right after
// the barrier that ends phase p.  One barrier per phase; everything else is
// wave-local.  (fp32 MFMA and VALU share the vector datapath on gfx950 --
// tools/ubench_coexec.hip -- so the epilogue uses the short-sequence
// transcendentals of nfk_spline.h.)
template <int KSH, int K, bool INV>
__global__ __launch_bounds__(64 * kWaves, 1) void k_fused_nsf(FusedArgs a) {
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
    extern __shared__ __attribute__((aligned(16))) float4 lds4[];
    float4* slot0 = lds4;
    float4* slot1 = lds4 + a.slot_blocks * 64;
    int32_t* m_up_in = reinterpret_cast<int32_t*>(lds4 + 2 * a.slot_blocks * 64);
    int32_t* m_up_out = m_up_in + a.n_up;
    int32_t* m_lo_in = m_up_out + a.n_up;
    int32_t* m_lo_out = m_lo_in + a.n_lo;
    float* xt = reinterpret_cast<float*>(lds4 + 2 * a.slot_blocks * 64 + ((2 * D + 3) / 4)) +
                wid * 16 * XS;
    const int64_t b0 = ((int64_t)blockIdx.x * kWaves + wid) * 16;
    const int64_t rem = a.batch - b0;
    const int nrows = rem <= 0 ? 0 : (rem < 16 ? (int)rem : 16);
    const NfkSplineConst& c = a.c;
    const float* pk = a.pack;

    // ---- prologue: x rows, index maps, first two phase records
    for (int r = 0; r < 16; ++r)
        for (int cc = lane; cc < D; cc += 64) xt[r * XS + cc] = (r < nrows) ? a.x[(b0 + r) * a.ldx + cc] : 0.0f;
    for (int i = threadIdx.x; i < a.n_up; i += 64 * kWaves) {
        m_up_in[i] = a.up_in[i];
        m_up_out[i] = a.up_out[i];
    }
    for (int i = threadIdx.x; i < a.n_lo; i += 64 * kWaves) {
        m_lo_in[i] = a.lo_in[i];
        m_lo_out[i] = a.lo_out[i];
    }
    stage_record(pk, a.blk_h1, slot0, wid, lane);
    __syncthreads();
    stage_record(pk + a.o_h2, a.blk_h2, slot1, wid, lane);

    // ---- layer 1 (slot 0): h1^T = tanh(W1 . lower^T + b1)
    f32x4 h1[HT];
    {
        const float4* s = slot0;
#pragma unroll
        for (int t = 0; t < HT; ++t) h1[t] = as_f32x4(s[(a.KS1 * TGH + t) * 64 + lane]);
        for (int ks = 0; ks < a.KS1; ++ks) {
            const int k = 4 * ks + q;
            const int col = (k < a.n_lo) ? m_lo_in[k] : -1;
            const float bf = (col >= 0) ? xt[sl * XS + col] : 0.0f;
#pragma unroll
            for (int g = 0; g < TGH; ++g) {
                const float4 w = s[(ks * TGH + g) * 64 + lane];
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
        for (int r = 0; r < 4; ++r) h1[t][r] = nfk_tanh_lean(h1[t][r]);
    __syncthreads();  // slot 0 free, hidden-2 record landed
    const float* w3 = pk + a.o_w3;
    // execution order of the three records of a chunk: searched knots, other knots, derivatives
    const int offA = INV ? a.blk_w : 0, offB = INV ? 0 : a.blk_w, offC = 2 * a.blk_w;
    stage_record(w3 + offA * 256, a.blk_w, slot0, wid, lane);

    // ---- layer 2 (slot 1): h2^T = tanh(W2 . h1^T + b2); register r of tile t = k-step 4t+r
    f32x4 h2[HT];
    gemm_lds<KSH, HT, TGH, HT>(h1, slot1, lane, h2);
#pragma unroll
    for (int t = 0; t < HT; ++t)
#pragma unroll
        for (int r = 0; r < 4; ++r) h2[t][r] = nfk_tanh_lean(h2[t][r]);
    __syncthreads();  // slot 1 free, chunk-0 record A landed
    stage_record(w3 + offB * 256, a.blk_w, slot1, wid, lane);

    float ldsum = 0.0f;
    bool any_in = false, any_nd = false;
    float* zrow = a.z + (b0 + sl) * a.ldz;
    // record A and C of a chunk use slot sA, record B slot sB; the next chunk's
    // A is staged into sB once B is consumed, so the roles swap every chunk
    float4* sA = slot0;
    float4* sB = slot1;
    const bool row_ok = sl < nrows;
    for (int ch = 0; ch < a.NCH; ++ch) {
        const int jbase = 16 * ch;
        const float* wc = w3 + (int64_t)ch * a.blk_chunk * 256;
        const float* wn = wc + (int64_t)a.blk_chunk * 256;  // next chunk
        int jj4[4];
        float xv[4];
        int kb[4];
        float cw_k[4], w_k[4], ch_k[4], h_k[4];
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const int j = jbase + 4 * q + r;
            jj4[r] = j;
            xv[r] = (j < a.n_up) ? xt[sl * XS + m_up_in[j]] : 0.0f;
        }

        // ---- record A (slot sA): searched knots (widths forward / heights inverse)
        {
            f32x4 acc[K];
            gemm_lds<KSH, K, TGK, HT>(h2, sA, lane, acc);
            if (INV)
                knot_phase<K, true, true>(acc, xv, c, kb, ch_k, h_k);
            else
                knot_phase<K, true, false>(acc, xv, c, kb, cw_k, w_k);
        }
        __syncthreads();
        stage_record(wc + offC * 256, a.blk_d, sA, wid, lane);

        // ---- record B (slot sB): the other knots, selected at the bin
        {
            f32x4 acc[K];
            gemm_lds<KSH, K, TGK, HT>(h2, sB, lane, acc);
            if (INV)
                knot_phase<K, false, false>(acc, xv, c, kb, cw_k, w_k);
            else
                knot_phase<K, false, true>(acc, xv, c, kb, ch_k, h_k);
        }
        __syncthreads();
        if (ch + 1 < a.NCH) stage_record(wn + offA * 256, a.blk_w, sB, wid, lane);

        // ---- record C (slot sA): derivatives of the bin, evaluate, log|det|
        {
            f32x4 accd[DN];
            gemm_lds<KSH, DN, TGD, HT>(h2, sA, lane, accd);
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                // padded derivative index j+1 holds logit j (utils.py:36-39):
                // raw_k = logit k-1, raw_k1 = logit k, by running select on k >= j
                const int k = kb[r];
                float raw_k = accd[0][r], raw_k1 = accd[0][r];
#pragma unroll
                for (int j = 1; j < K - 1; ++j) {
                    const bool ge = k >= j;
                    raw_k = (k >= j + 1) ? accd[j][r] : raw_k;
                    raw_k1 = ge ? accd[j][r] : raw_k1;
                }
                raw_k = nfk_softplus_lean(raw_k);  // NSF_CL's D <- softplus(D) (flows.py:235)
                raw_k1 = nfk_softplus_lean(raw_k1);
                raw_k = (k == 0) ? c.dpad : raw_k;
                raw_k1 = (k == K - 1) ? c.dpad : raw_k1;
                const float d_k = c.min_d + nfk_softplus_lean(raw_k);
                const float d_k1 = c.min_d + nfk_softplus_lean(raw_k1);
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
                const float dnum =
                    (delta * delta) * ((d_k1 * (th * th) + (2.0f * delta) * t1mt) + d_k * (omt * omt));
                float lad = (__builtin_amdgcn_logf(dnum) - 2.0f * __builtin_amdgcn_logf(den)) * kLN2;
                lad = INV ? -lad : lad;
                const bool inside = (x >= c.lo) && (x <= c.hi);
                const bool live = jj4[r] < a.n_up && row_ok;
                out = inside ? out : x;
                if (live) zrow[m_up_out[jj4[r]]] = out;
                ldsum += (inside && live) ? lad : 0.0f;
                any_in |= inside && live;
                any_nd |= nd && inside && live;
            }
        }
        __syncthreads();
        if (ch + 1 < a.NCH) stage_record(wn + offB * 256, a.blk_w, sA, wid, lane);
        float4* t = sA;
        sA = sB;
        sB = t;
    }

    // ---- identity-copied coordinates, per-sample log|det|
    for (int i = lane; i < 16 * a.n_lo; i += 64) {
        const int row = i / a.n_lo, qq = i - row * a.n_lo;
        if (row < nrows) a.z[(b0 + row) * a.ldz + m_lo_out[qq]] = xt[row * XS + m_lo_in[qq]];
    }
    {
        float v = ldsum;
        v += __shfl_xor(v, 16, 64);
        v += __shfl_xor(v, 32, 64);
        if (q == 0 && row_ok && a.mode != 0) {
            float* dst = a.logdet + b0 + sl;
            *dst = (a.mode == 2) ? (*dst + v) : v;
        }
    }
    if (a.status != nullptr) {
        const int bits = (__any(any_in) ? NFK_ST_INSIDE_SEEN : 0) | (__any(any_nd) ? NFK_ST_NEG_DISC : 0);
        if (lane == 0 && bits != 0) {
            if ((__hip_atomic_load(a.status, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) & bits) != bits)
                atomicOr(a.status, bits);
        }
    }
}

template <int KSH, int K>
int launch_fused(const FusedArgs& a, size_t lds, bool inv, hipStream_t st) {
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
    template int launch_fused<KSH, K>(const FusedArgs& a, size_t lds, bool inv, hipStream_t st);
#define NFK_FUSED_EXTERN(KSH, K) \
    extern template int launch_fused<KSH, K>(const FusedArgs& a, size_t lds, bool inv, hipStream_t st);

// supported hidden sizes: KSH = ceil(H/4) k-steps of 4 (H = 12, 16, 32, 64, 100, 128)
#define NFK_FUSED_KSH(X) X(3) X(4) X(8) X(16) X(25) X(32)
#define NFK_FUSED_K(X, KSH) X(KSH, 4) X(KSH, 5) X(KSH, 6) X(KSH, 8) X(KSH, 10)

}  // namespace nfk_fused
