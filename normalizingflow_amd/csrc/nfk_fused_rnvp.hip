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

#include <cstdint>

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

// layer 1 of one net: acc = b 2^(s1+sx) + 2^s1 W1 . (2^sx in)^T (fp16 split)
template <int KBI, int HT>
__device__ __forceinline__ void input_gemm(const h8 (&xh)[KBI], const h8 (&xl)[KBI], const float4* rec,
                                           float bsc, int lane, f32x4 (&acc)[HT]) {
    const int q = lane >> 4;
    const float4* bias = rec + KBI * HT * 2 * 64;
#pragma unroll
    for (int t = 0; t < HT; ++t) {
        const float4 bv = bias[t * 4 + q];
        acc[t] = f32x4{bv.x * bsc, bv.y * bsc, bv.z * bsc, bv.w * bsc};
    }
#pragma unroll
    for (int kb = 0; kb < KBI; ++kb)
#pragma unroll
        for (int t = 0; t < HT; ++t) {
            const h8 ahi = __builtin_bit_cast(h8, rec[((kb * HT + t) * 2) * 64 + lane]);
            const h8 alo = __builtin_bit_cast(h8, rec[((kb * HT + t) * 2 + 1) * 64 + lane]);
            acc[t] = mfma16(alo, xh[kb], acc[t]);
            acc[t] = mfma16(ahi, xl[kb], acc[t]);
            acc[t] = mfma16(ahi, xh[kb], acc[t]);
        }
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

        // ---- phase 0: layer 1 of s and t from the (per-wave scaled) input half
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
            for (int off = 32; off > 0; off >>= 1) mx = fmaxf(mx, __shfl_xor(mx, off, 64));
            int ex = 0;
            if (mx > 0.0f && mx < 3.0e38f) frexpf(mx, &ex);  // mx < 2^ex
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

extern "C" int64_t nfk_fused_realnvp_pack_elems(int32_t half_dim, int32_t hidden) {
    return rshape_ok(half_dim, hidden) ? make_rlayout(half_dim, hidden).total : 0;
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
