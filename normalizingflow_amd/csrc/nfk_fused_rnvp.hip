// nfk_fused_rnvp.hip -- one launch per RealNVP layer (nf/flows.py:38-76):
// both affine half-couplings, each with its s- and t-conditioner FCNN
// (flows.py:20-35: Linear -> tanh -> Linear -> tanh -> Linear), on MFMA, with
// the [B, D/2] conditioner outputs never leaving registers.
//
//   forward:  up <- t1(lo) + up * exp(s1(lo));  lo <- t2(up) + lo * exp(s2(up))
//   inverse:  lo <- (lo - t2(up)) * exp(-s2(up));  up <- (up - t1(lo)) * exp(-s1(lo))
//   log|det| (+)= sum s1 + sum s2   (inverse: minus)
//
// The machinery is the NSF_CL kernel's (nfk_fused_impl.h): one wave = 16
// samples, products transposed (A = weights from an LDS record slot, B =
// activations in registers), fp16 two-way split MFMAs with power-of-two
// pre-scaling, hidden features permuted so accumulators are the next B
// fragments, records streamed by asm LDS-DMA with one barrier per phase.
// Additionally the INPUT coordinates of every layer-1 weight are permuted by
//   pi(32 kb + 8 q + j) = 32 kb + 16 (j >> 2) + 4 q + (j & 3),
// so the accumulators of a half's output layer (lane q, register r of tile t
// = coordinate 16 t + 4 q + r) are, element for element, the B fragment the
// other half's layer 1 needs: the halves chain in registers too.
//
// Phases of a layer (record p, slot p & 1), per net pair (s1,t1) then (s2,t2)
// in the pack, executed in that order forward and reversed when inverting:
//   4 pr + 0: layer 1 of the pair's s and t nets (two sub-records)
//   4 pr + 1: layer 2 of s;   4 pr + 2: layer 2 of t
//   4 pr + 3: layer 3 of s and t (two sub-records) + the affine update
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdint>
#include <type_traits>

#include "../../include/nfk.h"
#include "nfk_spline.h"

int nfk_set_error(const char* msg);

#include "nfk_fused_impl.h"

namespace nfk_rnvp {

using namespace nfk_fused;

struct RLayout {
    int n, H, NO, KBI, KBH, T1, HT;
    int blk_l1, blk_l2, blk_l3;  // one net's layer-1 / 2 / 3 record
    int rec[4];                  // blocks of the four phase records of a pair
    int pair_blocks, slot_blocks;
    int64_t total;               // floats (header block + 2 pairs)
};

inline RLayout make_rlayout(int n, int H) {
    RLayout L;
    const Layout h = make_layout(1, 16, H, 4);  // hidden-width split (KBH, T1, HT)
    L.n = n;
    L.H = H;
    L.NO = n / 16;
    L.KBI = (L.NO + 1) / 2;
    L.KBH = h.KBH;
    L.T1 = h.T1;
    L.HT = h.HT;
    L.blk_l1 = L.KBI * L.HT * 2 + 1;
    L.blk_l2 = rec_blocks(L.KBH, L.T1, L.HT);
    L.blk_l3 = rec_blocks(L.KBH, L.T1, L.NO);
    L.rec[0] = 2 * L.blk_l1;
    L.rec[1] = L.blk_l2;
    L.rec[2] = L.blk_l2;
    L.rec[3] = 2 * L.blk_l3;
    L.pair_blocks = L.rec[0] + L.rec[1] + L.rec[2] + L.rec[3];
    L.slot_blocks = 0;
    for (int i = 0; i < 4; ++i) L.slot_blocks = L.rec[i] > L.slot_blocks ? L.rec[i] : L.slot_blocks;
    L.total = 256 + (int64_t)2 * L.pair_blocks * 256;
    return L;
}

// x/z tile of one wave: 16 rows x [lower | upper], each half padded to 32 KBI
inline int tile_row(const RLayout& L) { return 2 * 32 * L.KBI; }
inline size_t lds_bytes(const RLayout& L) {
    return 2 * (size_t)L.slot_blocks * 1024 + (size_t)kWaves * 16 * tile_row(L) * sizeof(float);
}

// input coordinate of k-slot 32 kb + 8 q + j of a layer-1 B fragment
__host__ __device__ inline int in_perm(int k) {
    const int kb = k >> 5, q = (k >> 3) & 3, j = k & 7;
    return 32 * kb + 16 * (j >> 2) + 4 * q + (j & 3);
}

struct RArgs {
    const float* x;
    const float* pack;
    float* z;
    float* logdet;
    int64_t ldx, ldz, batch;
    int32_t n, mode, slot_blocks;
    int32_t blk_l1, blk_l3, pair_blocks;
    int32_t rec_off[4];  // block offsets of the phase records inside a pair
    int32_t rec_len[4];
};

__device__ __forceinline__ void stage_rphase(const RArgs& a, int p, bool inv, float4* slot0, float4* slot1,
                                             int wid, int lane) {
    // kernel phase p -> pack record: pair order reversed when inverting
    const int pr = (p >> 2) ^ (inv ? 1 : 0), ph = p & 3;
    const float* src = a.pack + 256 + ((int64_t)pr * a.pair_blocks + a.rec_off[ph]) * 256;
    stage_record(src, a.rec_len[ph], (p & 1) ? slot1 : slot0, wid, lane);
}

__device__ __forceinline__ void rblock_end(int b, const RArgs& a, bool inv, float4* slot0, float4* slot1,
                                           int wid, int lane) {
    asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    if (b + 2 < 8) stage_rphase(a, b + 2, inv, slot0, slot1, wid, lane);
}

template <int KBH, bool T1, int NO, bool INV>
__global__ __launch_bounds__(64 * kWaves, 1) void k_fused_rnvp(RArgs a) {
    constexpr int HT = 2 * KBH + (T1 ? 1 : 0);
    constexpr int KBI = (NO + 1) / 2;
    constexpr int XI = 32 * KBI;  // tile columns per half
    const int lane = threadIdx.x & 63;
    const int wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int q = lane >> 4, sl = lane & 15;
    extern __shared__ __attribute__((aligned(16))) float4 lds4[];
    float4* slot0 = lds4;
    float4* slot1 = lds4 + a.slot_blocks * 64;
    float* tile = reinterpret_cast<float*>(lds4 + 2 * a.slot_blocks * 64) + wid * 16 * 2 * XI;
    const int64_t b0 = ((int64_t)blockIdx.x * kWaves + wid) * 16;
    const int64_t rem = a.batch - b0;
    const int nrows = rem <= 0 ? 0 : (rem < 16 ? (int)rem : 16);
    const int n = a.n;
    const float* hdr = a.pack;

    // ---- prologue: this wave's 16 x rows into its tile (plain loads, no DMA in
    // flight yet), padding zero; then the first two records
    for (int i = lane; i < 16 * 2 * XI; i += 64) {
        const int r = i / (2 * XI), cc = i - r * 2 * XI, hf = cc >= XI ? 1 : 0, c = cc - hf * XI;
        tile[i] = (r < nrows && c < n) ? a.x[(b0 + r) * a.ldx + hf * n + c] : 0.0f;
    }
    stage_rphase(a, 0, INV, slot0, slot1, wid, lane);
    stage_rphase(a, 1, INV, slot0, slot1, wid, lane);
    dma_barrier();

    float ldsum = 0.0f;
    float* trow = tile + sl * 2 * XI;
#pragma unroll 1
    for (int hk = 0; hk < 2; ++hk) {
        const int pr = INV ? 1 - hk : hk;        // net pair of this half: 0 = (s1,t1), 1 = (s2,t2)
        const int in_off = pr == 0 ? 0 : XI;     // pair 0 reads the lower half, updates the upper
        const int tg_off = pr == 0 ? XI : 0;
        const int b = 4 * hk;
        const float4* s_l1 = ((b & 1) ? slot1 : slot0);
        // header: per (pair, net, layer) unscale factors at hdr[16 + (2 pr + net) 3 + layer]
        const float* un = hdr + 16 + pr * 6;

        // ---- phase 0: layer 1 of s and t from the (per-sample scaled) input half
        h8 bsh[KBH], bsl[KBH], bth[KBH], btl[KBH];
        h4 bst, btt;
        {
            float mx = 0.0f;
#pragma unroll
            for (int kb = 0; kb < KBI; ++kb) {
                const float4 u = *reinterpret_cast<const float4*>(trow + in_off + 32 * kb + 4 * q);
                const float4 v = *reinterpret_cast<const float4*>(trow + in_off + 32 * kb + 16 + 4 * q);
                mx = fmaxf(mx, fmaxf(fmaxf(fmaxf(fabsf(u.x), fabsf(u.y)), fmaxf(fabsf(u.z), fabsf(u.w))),
                                     fmaxf(fmaxf(fabsf(v.x), fabsf(v.y)), fmaxf(fabsf(v.z), fabsf(v.w)))));
            }
#pragma unroll
            for (int off = 16; off < 64; off <<= 1) mx = fmaxf(mx, __shfl_xor(mx, off, 64));  // per sample: the 4 lanes of column sl
            int ex = 0;
            if (mx > 0.0f && mx < 3.0e38f) frexpf(mx, &ex);  // mx < 2^ex
            ex = ex < -64 ? -64 : ex;  // a tiny sample: its scale 2^(14 - ex) and bias scale stay finite
            const float sx = ldexpf(1.0f, 14 - ex);
            h8 xh[KBI], xl[KBI];
#pragma unroll
            for (int kb = 0; kb < KBI; ++kb) {
                const float4 u = *reinterpret_cast<const float4*>(trow + in_off + 32 * kb + 4 * q);
                const float4 v = *reinterpret_cast<const float4*>(trow + in_off + 32 * kb + 16 + 4 * q);
                const float x8[8] = {u.x * sx, u.y * sx, u.z * sx, u.w * sx, v.x * sx, v.y * sx, v.z * sx, v.w * sx};
#pragma unroll
                for (int j = 0; j < 8; ++j) {
                    const _Float16 hh = (_Float16)x8[j];
                    xh[kb][j] = hh;
                    xl[kb][j] = (_Float16)(x8[j] - (float)hh);
                }
            }
            f32x4 h1[HT];
            // s net (sub-record 0), then t net (sub-record 1)
            const float us = ldexpf(un[0], ex - 14), ut = ldexpf(un[3], ex - 14);
            input_gemm<KBI, HT>(xh, xl, s_l1, 1.0f / us, lane, h1);
            act_operands<KBH, T1, HT>(h1, -2.0f * kL2E * us, bsh, bsl, bst);
            input_gemm<KBI, HT>(xh, xl, s_l1 + a.blk_l1 * 64, 1.0f / ut, lane, h1);
            act_operands<KBH, T1, HT>(h1, -2.0f * kL2E * ut, bth, btl, btt);
        }
        rblock_end(b, a, INV, slot0, slot1, wid, lane);

        // ---- phases 1, 2: layer 2 of s, of t
        {
            f32x4 h2[HT];
            gemm_h<KBH, T1, HT>(bsh, bsl, bst, ((b + 1) & 1) ? slot1 : slot0, lane, h2);
            act_operands<KBH, T1, HT>(h2, -2.0f * kL2E * un[1], bsh, bsl, bst);
        }
        rblock_end(b + 1, a, INV, slot0, slot1, wid, lane);
        {
            f32x4 h2[HT];
            gemm_h<KBH, T1, HT>(bth, btl, btt, ((b + 2) & 1) ? slot1 : slot0, lane, h2);
            act_operands<KBH, T1, HT>(h2, -2.0f * kL2E * un[4], bth, btl, btt);
        }
        rblock_end(b + 2, a, INV, slot0, slot1, wid, lane);

        // ---- phase 3: s and t outputs, affine update of the target half (flows.py:56-76)
        {
            const float4* s3 = ((b + 3) & 1) ? slot1 : slot0;
            f32x4 so[NO], to[NO];
            gemm_h<KBH, T1, NO>(bsh, bsl, bst, s3, lane, so);
            gemm_h<KBH, T1, NO>(bth, btl, btt, s3 + a.blk_l3 * 64, lane, to);
            const float u3s = un[2], u3t = un[5];
#pragma unroll
            for (int t = 0; t < NO; ++t) {
                float4 xv = *reinterpret_cast<const float4*>(trow + tg_off + 16 * t + 4 * q);
                float o[4];
                const float xr[4] = {xv.x, xv.y, xv.z, xv.w};
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    const float sv = so[t][r] * u3s, tv = to[t][r] * u3t;
                    if (INV) {
                        o[r] = (xr[r] - tv) * expf(-sv);
                        ldsum += -sv;
                    } else {
                        o[r] = tv + xr[r] * expf(sv);
                        ldsum += sv;
                    }
                }
                *reinterpret_cast<float4*>(trow + tg_off + 16 * t + 4 * q) = make_float4(o[0], o[1], o[2], o[3]);
            }
        }
        rblock_end(b + 3, a, INV, slot0, slot1, wid, lane);
    }

    // ---- z rows (lower | upper), per-sample log|det|
    for (int i = lane; i < 16 * 2 * XI; i += 64) {
        const int r = i / (2 * XI), cc = i - r * 2 * XI, hf = cc >= XI ? 1 : 0, c = cc - hf * XI;
        if (r < nrows && c < n) a.z[(b0 + r) * a.ldz + hf * n + c] = tile[i];
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
}

// ---------------------------------------------------------------- packing
struct RPackArgs {
    const float* w[24];  // nets s1, t1, s2, t2 (pairs (s1,t1), (s2,t2)); per net W0 b0 W2 b2 W4 b4
    float* out;
    RLayout L;
};

__global__ __launch_bounds__(256) void k_rnvp_max(RPackArgs a) {
    // hdr[(2 pr + net) 3 + layer] = max |W| of that net layer (uint bits)
    const RLayout& L = a.L;
    const int64_t sz[3] = {(int64_t)L.H * L.n, (int64_t)L.H * L.H, (int64_t)L.n * L.H};
    for (int m = 0; m < 12; ++m) {
        const float* w = a.w[(m / 3) * 6 + 2 * (m % 3)];
        const int64_t cnt = sz[m % 3];
        float mx = 0.0f;
        for (int64_t g = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; g < cnt;
             g += (int64_t)gridDim.x * blockDim.x)
            mx = fmaxf(mx, fabsf(w[g]));
#pragma unroll
        for (int off = 32; off > 0; off >>= 1) mx = fmaxf(mx, __shfl_xor(mx, off, 64));
        if ((threadIdx.x & 63) == 0) atomicMax(reinterpret_cast<unsigned int*>(a.out) + m, __float_as_uint(mx));
    }
}

__device__ inline int rscale_exp(float maxw) {
    if (!(maxw > 0.0f) || !(maxw < 3.0e38f)) return 0;
    int e;
    frexpf(maxw, &e);
    return 15 - e;
}

__device__ inline uint32_t f16_pair(float v0, float v1, int part) {
    const _Float16 h0 = (_Float16)v0, h1 = (_Float16)v1;
    const _Float16 r0 = part ? (_Float16)(v0 - (float)h0) : h0;
    const _Float16 r1 = part ? (_Float16)(v1 - (float)h1) : h1;
    return (uint32_t)__builtin_bit_cast(uint16_t, r0) | ((uint32_t)__builtin_bit_cast(uint16_t, r1) << 16);
}

// word wl of block blk of a gemm_h-form record (f16 blocks, tail blocks, bias)
// with nt tiles; rows: weight row pointer (or null) per (tile, row)
template <class RowF, class BiasF>
__device__ uint32_t rec_word(int blk, int wl, const RLayout& L, int nt, float sc, float bsc, RowF row_of,
                             BiasF bias_of) {
    const int nf = L.KBH * nt * 2, ntg = L.T1 ? (nt + 1) / 2 : 0;
    if (blk < nf) {
        const int part = blk & 1, idx = blk >> 1, kb = idx / nt, t = idx - kb * nt;
        const int lane = wl >> 2, j = 2 * (wl & 3), k0 = 32 * kb + 8 * (lane >> 4) + j;
        const float* w = row_of(t, lane & 15);
        const int klim = L.T1 ? 32 * L.KBH : L.H;
        float v0 = 0.0f, v1 = 0.0f;
        if (w != nullptr) {
            if (k0 < klim && k0 < L.H) v0 = w[k0] * sc;
            if (k0 + 1 < klim && k0 + 1 < L.H) v1 = w[k0 + 1] * sc;
        }
        return f16_pair(v0, v1, part);
    }
    if (blk < nf + ntg) return tail_word(blk - nf, wl, nt, 32 * L.KBH, L.H, sc, row_of);
    const int t = wl >> 4, i = wl & 15;
    return __float_as_uint(t < nt ? bias_of(t, i) * bsc : 0.0f);
}

__global__ __launch_bounds__(256) void k_rnvp_pack(RPackArgs a) {
    const RLayout& L = a.L;
    const unsigned int* hmax = reinterpret_cast<const unsigned int*>(a.out);
    uint32_t* out = reinterpret_cast<uint32_t*>(a.out);
    for (int64_t g = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; g < L.total;
         g += (int64_t)gridDim.x * blockDim.x) {
        if (g < 256) {  // header: words 16 + m = unscale of net layer m
            if (g >= 16 && g < 28) {
                const int m = (int)g - 16, s = rscale_exp(__uint_as_float(hmax[m]));
                out[g] = __float_as_uint(ldexpf(1.0f, (m % 3 == 0) ? -s : -(s + 14)));
            } else if (g >= 12) {
                out[g] = 0;
            }
            continue;
        }
        const int64_t w = g - 256;
        const int pr = (int)(w / ((int64_t)L.pair_blocks * 256));
        int blk = (int)((w >> 8) - (int64_t)pr * L.pair_blocks);
        const int wl = (int)(w & 255);
        int ph = 0;
        while (blk >= L.rec[ph]) blk -= L.rec[ph++];
        // phase -> (net, layer, block inside the net's sub-record)
        int net, layer;
        if (ph == 0) {
            net = blk >= L.blk_l1 ? 1 : 0;
            blk -= net * L.blk_l1;
            layer = 0;
        } else if (ph == 3) {
            net = blk >= L.blk_l3 ? 1 : 0;
            blk -= net * L.blk_l3;
            layer = 2;
        } else {
            net = ph - 1;
            layer = 1;
        }
        const int m = (2 * pr + net) * 3 + layer;
        const float* const* W = a.w + (2 * pr + net) * 6;
        const int s = rscale_exp(__uint_as_float(hmax[m]));
        const float sc = ldexpf(1.0f, s);
        const int kbh = L.KBH;
        if (layer == 0) {  // input GEMM: f16 blocks over the permuted input coordinates + unscaled bias
            if (blk < L.KBI * L.HT * 2) {
                const int part = blk & 1, idx = blk >> 1, kb = idx / L.HT, t = idx - kb * L.HT;
                const int lane = wl >> 2, j = 2 * (wl & 3);
                const int f = hid_feature(t, lane & 15, kbh), k0 = 32 * kb + 8 * (lane >> 4) + j;
                const int c0 = in_perm(k0), c1 = in_perm(k0 + 1);
                float v0 = 0.0f, v1 = 0.0f;
                if (f < L.H) {
                    if (c0 < L.n) v0 = W[0][(int64_t)f * L.n + c0] * sc;
                    if (c1 < L.n) v1 = W[0][(int64_t)f * L.n + c1] * sc;
                }
                out[g] = f16_pair(v0, v1, part);
            } else {
                const int t = wl >> 4, f = hid_feature(t, wl & 15, kbh);
                out[g] = __float_as_uint((t < L.HT && f < L.H) ? W[1][f] : 0.0f);
            }
        } else if (layer == 1) {
            out[g] = rec_word(
                blk, wl, L, L.HT, sc, ldexpf(1.0f, s + 14),
                [&](int t, int i) -> const float* {
                    const int f = hid_feature(t, i, kbh);
                    return f < L.H ? W[2] + (int64_t)f * L.H : nullptr;
                },
                [&](int t, int i) -> float {
                    const int f = hid_feature(t, i, kbh);
                    return f < L.H ? W[3][f] : 0.0f;
                });
        } else {
            out[g] = rec_word(
                blk, wl, L, L.NO, sc, ldexpf(1.0f, s + 14),
                [&](int t, int i) -> const float* {
                    const int c = 16 * t + i;
                    return c < L.n ? W[4] + (int64_t)c * L.H : nullptr;
                },
                [&](int t, int i) -> float {
                    const int c = 16 * t + i;
                    return c < L.n ? W[5][c] : 0.0f;
                });
        }
    }
}

bool rshape_ok(int n, int H) {
    if (n < 16 || n % 16 != 0 || n > 64 || H < 1) return false;
    const RLayout L = make_rlayout(n, H);
    if (lds_bytes(L) > (size_t)kLdsBytes || L.HT > 16) return false;
    bool kb = false;
#define CHK_KB(h, t) kb |= (L.KBH == h && L.T1 == t);
    NFK_FUSED_KB(CHK_KB)
#undef CHK_KB
    return kb;
}

// ---------------------------------------------------------------- chain form
// k_rnvp_chain: every layer of a run of RealNVP layers in ONE launch.  Each
// wave keeps its 16 x rows in an LDS tile from the first layer to the last
// (lower half at columns [0, XI), upper at [XI, 2 XI); the layers read and
// overwrite it in place) and writes z -- or only log p, with the isotropic
// Normal prior as the epilogue -- at the end.
// Work split as the split-form NSF kernel (nfk_fused_impl.h): 4-wave
// workgroups, one wave per SIMD, three workgroups per CU.  The conditioner
// weights stream through TWO LDS slots as a sequence of equal sub-records
// (the pack's chain stream, built by k_rnvp_stream): per net, the layer-1
// record, then layer 2 and layer 3 in sub-records of kRNS output tiles.  At
// the barrier that ends the GEMM of sub-record k every wave has read slot
// k & 1 and (vmcnt(0) before it) has landed its part of sub-record k + 1 in
// the other slot, so the copy of k + 2 goes into slot k & 1 and overlaps the
// GEMM of k + 1: one barrier per sub-record, no copy latency exposed (the
// RealNVP epilogues are too short to cover a copy, unlike the spline's).
// Per half-coupling the s net runs first (its output tiles kept in
// registers), then the t net on the same input operands, then the affine
// update of the target half (flows.py:56-63, inverse 68-75).  The
// arithmetic and its order are those of k_fused_rnvp, so z and log|det| are
// bitwise those of one k_fused_rnvp launch per layer.
constexpr int kRNS = 2;  // output tiles per layer-2 / layer-3 sub-record

struct RChainDims {
    int HT, KBI, XI, RS, NP2, NP3, NSUB, NTB, B1, BP, SB;
    size_t lds;
};

__host__ __device__ constexpr RChainDims rchain_dims(int KBH, int T1, int NO) {
    RChainDims d{};
    d.HT = 2 * KBH + (T1 ? 1 : 0);
    d.KBI = (NO + 1) / 2;
    d.XI = 32 * d.KBI;
    d.RS = 2 * d.XI + 4;  // tile row stride (floats): rows 4 banks apart, 16-B reads conflict-free
    d.NP2 = (d.HT + kRNS - 1) / kRNS;
    d.NP3 = (NO + kRNS - 1) / kRNS;
    d.NSUB = 1 + d.NP2 + d.NP3;  // sub-records per net
    d.NTB = T1 ? (kRNS + 1) / 2 : 0;
    d.B1 = d.KBI * d.HT * 2 + 1;          // layer-1 record (input_gemm form)
    d.BP = KBH * kRNS * 2 + d.NTB + 1;    // a layer-2/3 sub-record (stage_tiles form)
    d.SB = (((d.B1 > d.BP ? d.B1 : d.BP) + 3) / 4) * 4;  // slot blocks: a multiple of the 4 waves
    d.lds = (size_t)2 * d.SB * 1024 + (size_t)4 * 16 * d.RS * sizeof(float);
    return d;
}

// floats of one layer's chain stream: 2 pairs x 2 nets x NSUB sub-records of SB blocks
__host__ __device__ inline int64_t rchain_stream_floats(const RLayout& L) {
    const RChainDims d = rchain_dims(L.KBH, L.T1, L.NO);
    return (int64_t)4 * d.NSUB * d.SB * 256;
}

// the chain form applies where three workgroups share a CU (LDS counted in
// the 1280-B allocation granule of nfk_fused_impl.h)
inline bool rchain_ok(const RLayout& L) {
    const RChainDims d = rchain_dims(L.KBH, L.T1, L.NO);
    return 3 * lds_alloc(d.lds) <= (size_t)kLdsBytes;
}

// The chain stream of a pack (after k_rnvp_pack wrote its records): sub-record
// u = (2 pr + net) NSUB + j, j = 0: the net's layer-1 record; 1..NP2: its
// layer-2 tiles [(j-1) kRNS, ..); then its layer-3 tiles; zero padding to SB.
__global__ __launch_bounds__(256) void k_rnvp_stream(float* pack, RLayout L, int64_t o_stream) {
    const RChainDims d = rchain_dims(L.KBH, L.T1, L.NO);
    const int64_t total = rchain_stream_floats(L);
    int off[4];
    off[0] = 0;
    for (int i = 1; i < 4; ++i) off[i] = off[i - 1] + L.rec[i - 1];
    for (int64_t g = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; g < total;
         g += (int64_t)gridDim.x * blockDim.x) {
        const int wl = (int)(g & 255);
        const int64_t blk = g >> 8;
        const int u = (int)(blk / d.SB), b = (int)(blk - (int64_t)u * d.SB);
        const int pr = u / (2 * d.NSUB), rem = u - pr * 2 * d.NSUB, net = rem / d.NSUB, j = rem - net * d.NSUB;
        const int base = pr * L.pair_blocks;
        int src = -1;
        if (j == 0) {
            if (b < d.B1) src = base + off[0] + net * L.blk_l1 + b;
        } else if (j <= d.NP2) {
            const int r = subrec_tile_src(b, L.KBH, L.T1, kRNS, d.HT, (j - 1) * kRNS);
            if (r >= 0) src = base + off[1 + net] + r;
        } else {
            const int r = subrec_tile_src(b, L.KBH, L.T1, kRNS, L.NO, (j - 1 - d.NP2) * kRNS);
            if (r >= 0) src = base + off[3] + net * L.blk_l3 + r;
        }
        pack[o_stream + g] = src >= 0 ? pack[256 + (int64_t)src * 256 + wl] : 0.0f;
    }
}

struct RChainArgs {
    const float* x;
    const float* const* packs;  // device array: the layers' packs, in execution order
    float* z;
    float* logdet;
    float* log_prob;  // optional prior epilogue: log N(z; 0, s^2 I) + log|det| (z may be null)
    int32_t* status;  // NFK_ST_NAN_Z of the prior epilogue (nullable)
    int64_t ldx, ldz, batch;
    int32_t n, mode, nlayers, o_stream;
    float prior_inv_scale, prior_c2pi, prior_hld;
};

// layer-2 / layer-3 GEMM over its kRNS-tile sub-records J, J + 1, ... in
// alternating slots (part J in slot (P + J) & 1), each followed by
// step(that slot)
template <int KBH, bool T1, int NT, int J, int P, class Step>
__device__ __forceinline__ void rchain_parts(const h8 (&bh)[KBH], const h8 (&bl)[KBH], h4 bt, float4* s0,
                                             float4* s1, int lane, f32x4 (&acc)[NT], Step&& step) {
    constexpr int T0 = J * kRNS;
    constexpr int N = (NT - T0) < kRNS ? (NT - T0) : kRNS;
    float4* const sl = ((P + J) & 1) ? s1 : s0;
    gemm_h<KBH, T1, N, kRNS, T0, NT>(bh, bl, bt, sl, lane, acc);
    step(sl);
    if constexpr (T0 + kRNS < NT) rchain_parts<KBH, T1, NT, J + 1, P>(bh, bl, bt, s0, s1, lane, acc, step);
}

template <int KBH, bool T1, int NO, bool INV>
__global__ __launch_bounds__(64 * kNsfWaves, 3) void k_rnvp_chain(RChainArgs a) {
    constexpr RChainDims d = rchain_dims(KBH, T1 ? 1 : 0, NO);
    constexpr int HT = d.HT, KBI = d.KBI, XI = d.XI, RS = d.RS, NSUB = d.NSUB, SB = d.SB;
    constexpr int NPL = 4 * NSUB;  // sub-records per layer (even: the slot parity repeats per layer)
    // the arguments through the kernarg-segment pointer, re-derived opaquely
    // per layer (as k_fused_nsf's chain form: values loaded from them are not
    // kept live across the layer loop)
    using ArgsK = const __attribute__((address_space(4))) RChainArgs;
    ArgsK* A = (ArgsK*)__builtin_amdgcn_kernarg_segment_ptr();
    (void)a;
    const int lane = threadIdx.x & 63;
    const int wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int q = lane >> 4, sl = lane & 15;
    extern __shared__ __attribute__((aligned(16))) float4 lds4[];
    float4* const slot0 = lds4;
    float4* const slot1 = lds4 + SB * 64;
    float* const tile = reinterpret_cast<float*>(lds4 + 2 * SB * 64) + wid * 16 * RS;
    const int64_t b0 = ((int64_t)blockIdx.x * kNsfWaves + wid) * 16;
    const int64_t rem = A->batch - b0;
    const int nrows = rem <= 0 ? 0 : (rem < 16 ? (int)rem : 16);
    const int n = A->n, NL = A->nlayers;

    // ---- sub-record staging: (nl, nj) is the next sub-record to copy, in
    // execution order; its pack position swaps the two pairs when inverting
    int nl = 0, nj = 0;
    const float* nbase = A->packs[0] + A->o_stream;
    auto stage_next = [&](float4* slot) {
        if (nl >= NL) return;
        const int pos = INV ? (nj < 2 * NSUB ? nj + 2 * NSUB : nj - 2 * NSUB) : nj;
        const float* src = nbase + (int64_t)pos * SB * 256;
        const uint32_t base = lds_addr(slot);
#pragma unroll
        for (int i = 0; i < SB / 4; ++i)
            dma16(src + (int64_t)(wid + 4 * i) * 256 + lane * 4, base + (wid + 4 * i) * 1024);
        if (++nj == NPL) {
            nj = 0;
            if (++nl < NL) nbase = A->packs[nl] + A->o_stream;
        }
    };
    // end of the GEMM of sub-record k (slot k & 1 = freed): this wave's reads
    // of it and its copy of k + 1 done, barrier, then the copy of k + 2 into it
    auto step = [&](float4* freed) {
        asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_barrier();
        asm volatile("" ::: "memory");
        stage_next(freed);
    };

    // ---- prologue: the wave's x rows into its tile (plain loads, padding
    // columns zero), then the first two sub-records, one wait
    {
        const float* x = A->x;
        const int64_t ldx = A->ldx;
        constexpr int R4 = 2 * XI / 4;  // float4 per tile row
        for (int i = lane; i < 16 * R4; i += 64) {
            const int r = i / R4, c = 4 * (i - r * R4);
            const int hf = c >= XI ? 1 : 0, cc = c - hf * XI;
            float4 v = make_float4(0.0f, 0.0f, 0.0f, 0.0f);
            if (r < nrows && cc < n) {
                const float4* src = reinterpret_cast<const float4*>(x + (b0 + r) * ldx + hf * n + cc);
#if NFK_X_NT
                // read once: the nt policy (see dma4_nt)
                const f32x4 t = __builtin_nontemporal_load(reinterpret_cast<const f32x4*>(src));
                v = make_float4(t[0], t[1], t[2], t[3]);
#else
                v = *src;
#endif
            }
            *reinterpret_cast<float4*>(tile + r * RS + c) = v;
        }
    }
    stage_next(slot0);
    stage_next(slot1);
    asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");

    const bool row_ok = sl < nrows;
    float ld_acc = (q == 0 && row_ok && A->mode == 2) ? A->logdet[b0 + sl] : 0.0f;
    float* const trow = tile + sl * RS;
    for (int l = 0; l < NL; ++l) {
        asm volatile("" : "+s"(A));
        const float* hdr = A->packs[l];
        float ldsum = 0.0f;
#pragma unroll
        for (int hk = 0; hk < 2; ++hk) {
            const int pr = INV ? 1 - hk : hk;     // net pair of this half: 0 = (s1, t1), 1 = (s2, t2)
            const int in_off = pr == 0 ? 0 : XI;  // pair 0 reads the lower half, updates the upper
            const int tg_off = pr == 0 ? XI : 0;
            const float* un = hdr + 16 + pr * 6;  // unscale factors of (net, layer) in the pair
            // layer-1 operands of the input half, per-sample power-of-two scaled (as k_fused_rnvp)
            h8 xh[KBI], xl[KBI];
            int ex = 0;
            {
                float mx = 0.0f;
#pragma unroll
                for (int kb = 0; kb < KBI; ++kb) {
                    const float4 u = *reinterpret_cast<const float4*>(trow + in_off + 32 * kb + 4 * q);
                    const float4 v = *reinterpret_cast<const float4*>(trow + in_off + 32 * kb + 16 + 4 * q);
                    mx = fmaxf(mx, fmaxf(fmaxf(fmaxf(fabsf(u.x), fabsf(u.y)), fmaxf(fabsf(u.z), fabsf(u.w))),
                                         fmaxf(fmaxf(fabsf(v.x), fabsf(v.y)), fmaxf(fabsf(v.z), fabsf(v.w)))));
                }
#pragma unroll
                for (int off = 16; off < 64; off <<= 1) mx = fmaxf(mx, __shfl_xor(mx, off, 64));  // per sample: the 4 lanes of column sl
                if (mx > 0.0f && mx < 3.0e38f) frexpf(mx, &ex);
                ex = ex < -64 ? -64 : ex;  // a tiny sample: its scale 2^(14 - ex) and bias scale stay finite
                const float sx = ldexpf(1.0f, 14 - ex);
#pragma unroll
                for (int kb = 0; kb < KBI; ++kb) {
                    const float4 u = *reinterpret_cast<const float4*>(trow + in_off + 32 * kb + 4 * q);
                    const float4 v = *reinterpret_cast<const float4*>(trow + in_off + 32 * kb + 16 + 4 * q);
                    const float x8[8] = {u.x * sx, u.y * sx, u.z * sx, u.w * sx,
                                         v.x * sx, v.y * sx, v.z * sx, v.w * sx};
#pragma unroll
                    for (int j = 0; j < 8; ++j) {
                        const _Float16 hh = (_Float16)x8[j];
                        xh[kb][j] = hh;
                        xl[kb][j] = (_Float16)(x8[j] - (float)hh);
                    }
                }
            }
            // one net (c = 0: s, 1: t): layer 1 (sub-record 0), layer 2 (NP2
            // sub-records), layer 3 (NP3) into out, unscaled.  A half starts at
            // an even sub-record, so net c's sub-record j sits in slot (c NSUB + j) & 1.
            auto run_net = [&](auto netc, f32x4 (&out)[NO]) {
                constexpr int C = decltype(netc)::value;
                constexpr int P0 = (C * NSUB) & 1, P2 = (C * NSUB + 1) & 1, P3 = (C * NSUB + 1 + d.NP2) & 1;
                const float u1 = ldexpf(un[3 * C], ex - 14);
                h8 bh[KBH], bl[KBH];
                h4 bt;
                {
                    f32x4 h1[HT];
                    input_gemm<KBI, HT>(xh, xl, P0 ? slot1 : slot0, 1.0f / u1, lane, h1);
                    step(P0 ? slot1 : slot0);
                    act_operands<KBH, T1, HT>(h1, -2.0f * kL2E * u1, bh, bl, bt);
                }
                {
                    f32x4 h2[HT];
                    rchain_parts<KBH, T1, HT, 0, P2>(bh, bl, bt, slot0, slot1, lane, h2, step);
                    act_operands<KBH, T1, HT>(h2, -2.0f * kL2E * un[3 * C + 1], bh, bl, bt);
                }
                rchain_parts<KBH, T1, NO, 0, P3>(bh, bl, bt, slot0, slot1, lane, out, step);
            };
            f32x4 so[NO], to[NO];
            run_net(std::integral_constant<int, 0>{}, so);
            run_net(std::integral_constant<int, 1>{}, to);
            // affine update of the target half (flows.py:56-63; inverse 68-75)
            const float u3s = un[2], u3t = un[5];
#pragma unroll
            for (int t = 0; t < NO; ++t) {
                float* p = trow + tg_off + 16 * t + 4 * q;
                const float4 xv = *reinterpret_cast<const float4*>(p);
                const float xr[4] = {xv.x, xv.y, xv.z, xv.w};
                float o[4];
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    const float sv = so[t][r] * u3s, tv = to[t][r] * u3t;
                    if (INV) {
                        o[r] = (xr[r] - tv) * expf(-sv);
                        ldsum += -sv;
                    } else {
                        o[r] = tv + xr[r] * expf(sv);
                        ldsum += sv;
                    }
                }
                *reinterpret_cast<float4*>(p) = make_float4(o[0], o[1], o[2], o[3]);
            }
        }
        // the layer's log|det| added to the running sum, in the order of one
        // k_fused_rnvp launch per layer
        float v = ldsum;
        v += __shfl_xor(v, 16, 64);
        v += __shfl_xor(v, 32, 64);
        ld_acc = ld_acc + v;
    }

    // ---- tail: z rows (lower | upper), log|det|, or the prior epilogue
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    if (A->z != nullptr) {
        float* z = A->z;
        const int64_t ldz = A->ldz;
        const int N4 = n / 2;  // float4 per z row (2 n floats)
        for (int i = lane; i < 16 * N4; i += 64) {
            const int r = i / N4, c = 4 * (i - r * N4);
            const int hf = c >= n ? 1 : 0;
            if (r < nrows)
                *reinterpret_cast<float4*>(z + (b0 + r) * ldz + c) =
                    *reinterpret_cast<const float4*>(tile + r * RS + hf * XI + c - hf * n);
        }
    }
    if (q == 0 && row_ok && A->mode != 0) A->logdet[b0 + sl] = ld_acc;
    if (A->log_prob != nullptr) {
        // log N(z; 0, s^2 I) + log|det| from the tile row: the four lanes of sample
        // sl sum output columns 4 (q + 4 i) .. + 3 as k_normal_lp4 (y = z / s)
        const float il = A->prior_inv_scale;
        float m = 0.0f;
        for (int g = q; g < (n >> 1); g += 4) {
            const int o = 4 * g, c = o < n ? o : XI + o - n;
            const float4 zv = *reinterpret_cast<const float4*>(trow + c);
            const float y0 = zv.x * il, y1 = zv.y * il, y2 = zv.z * il, y3 = zv.w * il;
            m += (y0 * y0 + y1 * y1) + (y2 * y2 + y3 * y3);
        }
        m += __shfl_xor(m, 16, 64);
        m += __shfl_xor(m, 32, 64);
        const float lp = -0.5f * (A->prior_c2pi + m) - A->prior_hld;
        if (q == 0 && row_ok) A->log_prob[b0 + sl] = lp + ld_acc;
        // a NaN in z: the prior's argument validation raises (NFK_ST_NAN_Z)
        if (__any(row_ok && m != m) && lane == 0 && A->status != nullptr) atomicOr(A->status, NFK_ST_NAN_Z);
    }
}

template <int KBH, int T1, int NO>
int launch_chain(const RChainArgs& a, bool inv, hipStream_t st) {
    const int64_t blocks = (a.batch + kNsfWaves * 16 - 1) / (kNsfWaves * 16);
    if (blocks == 0) return 0;
    const size_t lds = rchain_dims(KBH, T1, NO).lds;
    if (inv)
        hipLaunchKernelGGL((k_rnvp_chain<KBH, T1 != 0, NO, true>), dim3((unsigned)blocks), dim3(64 * kNsfWaves),
                           lds, st, a);
    else
        hipLaunchKernelGGL((k_rnvp_chain<KBH, T1 != 0, NO, false>), dim3((unsigned)blocks), dim3(64 * kNsfWaves),
                           lds, st, a);
    const hipError_t e = hipGetLastError();
    return e == hipSuccess ? 0 : (int)e;
}

template <int KBH, int T1, int NO>
int launch(const RArgs& a, size_t lds, bool inv, hipStream_t st) {
    const int64_t blocks = (a.batch + kWaves * 16 - 1) / (kWaves * 16);
    if (blocks == 0) return 0;
    if (inv)
        hipLaunchKernelGGL((k_fused_rnvp<KBH, T1 != 0, NO, true>), dim3((unsigned)blocks), dim3(64 * kWaves),
                           lds, st, a);
    else
        hipLaunchKernelGGL((k_fused_rnvp<KBH, T1 != 0, NO, false>), dim3((unsigned)blocks), dim3(64 * kWaves),
                           lds, st, a);
    const hipError_t e = hipGetLastError();
    return e == hipSuccess ? 0 : (int)e;
}

}  // namespace nfk_rnvp

using namespace nfk_rnvp;

extern "C" int nfk_fused_realnvp_supported(int32_t half_dim, int32_t hidden) {
    return rshape_ok(half_dim, hidden) ? 1 : 0;
}

// floats of a pack: the per-layer kernel's records, then (where the chain form
// applies) the chain stream
static int64_t rpack_floats(int32_t half_dim, int32_t hidden) {
    const RLayout L = make_rlayout(half_dim, hidden);
    return L.total + (rchain_ok(L) ? rchain_stream_floats(L) : 0);
}

extern "C" int64_t nfk_fused_realnvp_pack_elems(int32_t half_dim, int32_t hidden) {
    return rshape_ok(half_dim, hidden) ? rpack_floats(half_dim, hidden) : 0;
}

extern "C" int nfk_fused_realnvp_pack(const float* const* nets, int32_t half_dim, int32_t hidden, float* wpack,
                                      nfk_stream_t stream) {
    if (!rshape_ok(half_dim, hidden)) return nfk_set_error("nfk_fused_realnvp_pack: shape not supported");
    if (!nets || !wpack) return nfk_set_error("nfk_fused_realnvp_pack: null pointer");
    RPackArgs a;
    for (int i = 0; i < 24; ++i) {
        if (!nets[i]) return nfk_set_error("nfk_fused_realnvp_pack: null weight pointer");
        a.w[i] = nets[i];
    }
    a.out = wpack;
    a.L = make_rlayout(half_dim, hidden);
    hipStream_t st = (hipStream_t)stream;
    hipError_t e = hipMemsetAsync(wpack, 0, 12 * sizeof(float), st);
    if (e != hipSuccess) return (int)e;
    hipLaunchKernelGGL(k_rnvp_max, dim3(32), dim3(256), 0, st, a);
    int64_t g = (a.L.total + 255) / 256;
    if (g > 8192) g = 8192;
    hipLaunchKernelGGL(k_rnvp_pack, dim3((unsigned)g), dim3(256), 0, st, a);
    if (rchain_ok(a.L)) {  // the chain stream, re-cut from the records just written
        int64_t gs = (rchain_stream_floats(a.L) + 255) / 256;
        if (gs > 8192) gs = 8192;
        hipLaunchKernelGGL(k_rnvp_stream, dim3((unsigned)gs), dim3(256), 0, st, wpack, a.L, a.L.total);
    }
    e = hipGetLastError();
    return e == hipSuccess ? 0 : (int)e;
}

extern "C" int nfk_fused_realnvp(const float* x, int64_t ldx, const float* wpack, int32_t half_dim,
                                 int32_t hidden, float* z, int64_t ldz, float* logdet, int32_t logdet_mode,
                                 int64_t batch, int32_t inverse, nfk_stream_t stream) {
    if (!rshape_ok(half_dim, hidden)) return nfk_set_error("nfk_fused_realnvp: shape not supported");
    if (batch < 0) return nfk_set_error("nfk_fused_realnvp: bad batch");
    if (batch == 0) return 0;
    if (!x || !wpack || !z) return nfk_set_error("nfk_fused_realnvp: null pointer");
    if (logdet_mode != 0 && !logdet) return nfk_set_error("nfk_fused_realnvp: null logdet");
    const RLayout L = make_rlayout(half_dim, hidden);
    RArgs a;
    a.x = x;
    a.pack = wpack;
    a.z = z;
    a.logdet = logdet;
    a.ldx = ldx;
    a.ldz = ldz;
    a.batch = batch;
    a.n = half_dim;
    a.mode = logdet_mode;
    a.slot_blocks = L.slot_blocks;
    a.blk_l1 = L.blk_l1;
    a.blk_l3 = L.blk_l3;
    a.pair_blocks = L.pair_blocks;
    int off = 0;
    for (int i = 0; i < 4; ++i) {
        a.rec_off[i] = off;
        a.rec_len[i] = L.rec[i];
        off += L.rec[i];
    }
    const size_t lds = lds_bytes(L);
    hipStream_t st = (hipStream_t)stream;
    const bool inv = inverse != 0;
#define RDISPATCH(h, t, no) \
    if (L.KBH == h && L.T1 == t && L.NO == no) return launch<h, t, no>(a, lds, inv, st);
#define RDISPATCH_KB(h, t) RDISPATCH(h, t, 1) RDISPATCH(h, t, 2) RDISPATCH(h, t, 3) RDISPATCH(h, t, 4)
    NFK_FUSED_KB(RDISPATCH_KB)
#undef RDISPATCH_KB
#undef RDISPATCH
    return nfk_set_error("nfk_fused_realnvp: no kernel instance");
}

extern "C" int nfk_fused_realnvp_chain_max(int32_t half_dim, int32_t hidden) {
    if (!rshape_ok(half_dim, hidden) || !rchain_ok(make_rlayout(half_dim, hidden))) return 0;
    return 1 << 16;  // no per-layer state in LDS: any run length
}

extern "C" int nfk_fused_realnvp_chain(const float* x, int64_t ldx, const float* const* wpacks, int32_t nlayers,
                                       int32_t half_dim, int32_t hidden, float* z, int64_t ldz, float* logdet,
                                       int32_t logdet_mode, int64_t batch, int32_t inverse, int32_t* status,
                                       float* log_prob, float prior_scale, float prior_half_log_det,
                                       nfk_stream_t stream) {
    if (nfk_fused_realnvp_chain_max(half_dim, hidden) == 0)
        return nfk_set_error("nfk_fused_realnvp_chain: shape not supported");
    if (nlayers < 1 || nlayers > (1 << 16)) return nfk_set_error("nfk_fused_realnvp_chain: bad layer count");
    if (batch < 0) return nfk_set_error("nfk_fused_realnvp_chain: bad batch");
    if (batch == 0) return 0;
    if (!x || !wpacks || (!z && !log_prob)) return nfk_set_error("nfk_fused_realnvp_chain: null pointer");
    if (logdet_mode != 0 && !logdet) return nfk_set_error("nfk_fused_realnvp_chain: null logdet");
    if (log_prob && !(prior_scale > 0.0f)) return nfk_set_error("nfk_fused_realnvp_chain: bad prior scale");
    if (((uintptr_t)x % 16) != 0 || ((uintptr_t)z % 16) != 0 || ldx % 4 != 0 || (z && ldz % 4 != 0))
        return nfk_set_error("nfk_fused_realnvp_chain: x and z rows must be 16-byte aligned");
    const RLayout L = make_rlayout(half_dim, hidden);
    RChainArgs a;
    a.x = x;
    a.packs = wpacks;
    a.z = z;
    a.logdet = logdet;
    a.log_prob = log_prob;
    a.status = status;
    a.ldx = ldx;
    a.ldz = ldz;
    a.batch = batch;
    a.n = half_dim;
    a.mode = logdet_mode;
    a.nlayers = nlayers;
    a.o_stream = (int32_t)L.total;
    a.prior_inv_scale = log_prob ? 1.0f / prior_scale : 0.0f;
    a.prior_c2pi = (float)(2 * half_dim * std::log(2.0 * M_PI));
    a.prior_hld = prior_half_log_det;
    hipStream_t st = (hipStream_t)stream;
    const bool inv = inverse != 0;
#define RDISPATCH(h, t, no) \
    if (L.KBH == h && L.T1 == t && L.NO == no) return launch_chain<h, t, no>(a, inv, st);
#define RDISPATCH_KB(h, t) RDISPATCH(h, t, 1) RDISPATCH(h, t, 2) RDISPATCH(h, t, 3) RDISPATCH(h, t, 4)
    NFK_FUSED_KB(RDISPATCH_KB)
#undef RDISPATCH_KB
#undef RDISPATCH
    return nfk_set_error("nfk_fused_realnvp_chain: no kernel instance");
}
