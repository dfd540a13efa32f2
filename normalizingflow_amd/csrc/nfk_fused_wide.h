// nfk_fused_wide.h -- fused NSF coupling-layer kernel for wide layers (BASELINE
// config c5: D = 256, H = 256, K = 16, NSF_CL of nf/flows.py:216-253).
//
// Same arithmetic as k_fused_nsf (nfk_fused_impl.h: transposed products on
// v_mfma_f32_16x16x32_f16 as a two-way fp16 split, permuted hidden features so
// accumulators are the next layer's B fragments, knot prefixes in 2^-30 fixed
// point, spline evaluated in registers) and the same packed weights
// (make_layout / k_pack).  What changes is the staging, because a c5 layer
// streams 6.4 MB of packed weights (one 16-coordinate chunk's W-logit record
// alone is 257 KiB) and its activations are 1 KiB per sample:
//   * 8-coordinate chunks (Layout.wide): a lane group holds 2 coordinates x
//     all their parameters (registers 2h, 2h+1 of K/2 tiles), half the
//     accumulators of the 16-coordinate form -- H = 256 needs 64 VGPRs of
//     resident fp16 operands, and the 16-coordinate form spilled;
//   * sub-records: every record is consumed G = min(KBH, 32/NT) k-blocks at
//     a time (2 G NT <= 64 one-KiB blocks, plus the record's bias block with
//     the first); a sub-step is the GEMM over one sub-record, ended by the
//     workgroup barrier that recycles its LDS slot; a phase's epilogue runs
//     after its last sub-step, so the copy of sub-record s+2 (issued right
//     after the barrier ending s) overlaps the epilogue and the GEMM of s+1;
//   * layer-1 operands (x at the lower coordinates) are read once per wave
//     into registers by plain loads in the prologue, before any copy is
//     waited on, and split there (per-sample power-of-two scale);
//   * per chunk pair, each wave stages the 32 coordinates (16 upper, 16
//     lower) of its 16 rows by LDS-DMA gathers into a 16 x 32 tile; the
//     spline reads x there, writes z back in place (the lower coordinates
//     pass through, flows.py:239), and the tile is stored after the pair as
//     whole 128-B row segments.  Writing the lower half of z from the
//     prologue registers instead (x's lower half read once) was measured
//     worse: the two halves of every z line then reach HBM as separate
//     partial-line writes, 2.15 GB written and 4.56 GB read per c5 launch
//     against 1.2 / 3.7 GB (profiles/r3e_pmc_c5.txt);
//   * LDS: two 65-KiB slots + 2 KiB x tile per wave + index maps (152 KiB at
//     c5), one 8-wave workgroup (128 samples) per CU.
// Copies follow the invariant of nfk_fused_impl.h: a copy is waited for
// (vmcnt(0)) at the barrier ending the sub-step after the one it was issued
// in, and the loop issues no VGPR-destination global load.
#pragma once
#include <type_traits>

#include "nfk_fused_impl.h"

namespace nfk_fused {

// Frame size and workgroup shape.  Default: one 8-wave workgroup per CU,
// 65-block frames.  NFK_WIDE_FB=32 NFK_WIDE_NW=4 builds two 4-wave workgroups
// per CU with 33-block frames (measured 4-5 % slower at c5: twice the
// sub-steps, and the two workgroups do not desynchronise usefully).
#ifndef NFK_WIDE_FB
#define NFK_WIDE_FB 64
#endif
#ifndef NFK_WIDE_NW
#define NFK_WIDE_NW 8
#endif
#ifndef NFK_WIDE_PK
#define NFK_WIDE_PK 1
#endif
#ifndef NFK_WIDE_PIN
#define NFK_WIDE_PIN 1
#endif
constexpr int kWideFB = NFK_WIDE_FB;             // f16 blocks of a frame
constexpr int kWideSlotBlocks = kWideFB + 1;     // + the record's bias block
constexpr int kWideWaves = NFK_WIDE_NW;          // waves per workgroup
constexpr int kWideWGs = kWideWaves == 4 ? 2 : 1;  // workgroups per CU
constexpr int kWideTile = 16 * 32;               // floats of a wave's chunk-pair tile
static_assert(kWideFB == 32 || kWideFB == 64, "frame of 32 or 64 blocks");
static_assert(kWideWaves == 4 || kWideWaves == 8 || kWideWaves == 12, "4-, 8- or 12-wave workgroups");

// k-blocks per sub-record of a record with nt tiles
__host__ __device__ constexpr int wide_g(int nt, int kbh) {
    return (kWideFB / 2 / nt) < kbh ? (kWideFB / 2 / nt) : kbh;
}

struct WideArgs {
    const float* x;
    const float* pack;  // header block + frame stream (k_pack_frames)
    const int32_t *up_in, *up_out, *lo_in, *lo_out;
    float* z;
    float* logdet;
    int32_t* status;
    int64_t ldx, ldz, batch;
    int32_t n_lo, n_up, KB1, NCH, mode;
    int32_t S1, NS;  // layer-1 sub-steps, sub-steps per layer
    FusedConst c;
    uint32_t* trace;  // diagnostic timeline buffer (NFK_TRACE builds), else unused
};

inline size_t wide_lds_bytes(int n_lo, int n_up) {
    return 2 * (size_t)kWideSlotBlocks * 1024 + (size_t)((2 * (n_lo + n_up) + 3) / 4) * 16 +
           (size_t)kWideWaves * kWideTile * sizeof(float);
}

// sub-steps of one layer: layer 1, layer 2, then per 8-coordinate chunk the
// searched knots, the other knots and the derivatives
inline int wide_substeps(int kb1, int kbh, int K, int nch, int* s1) {
    const int g1 = wide_g(2 * kbh, kbh), gc = wide_g(K / 2, kbh);
    *s1 = (kb1 + g1 - 1) / g1;
    return *s1 + kbh / g1 + 3 * nch * (kbh / gc);
}

// Copy the frame of sub-step s (if any) into slot s & 1.  The pack holds one
// frame per sub-step in forward order (W, H, D records per chunk); the
// inverse searches the heights, so it takes each chunk's H frames first.
template <int KBH, int K, bool INV>
__device__ __forceinline__ void wide_stage(const WideArgs& a, int s, float4* slot0, float4* slot1, int wid,
                                           int lane) {
    if (s >= a.NS) return;
    constexpr int S2 = KBH / wide_g(2 * KBH, KBH), SC = KBH / wide_g(K / 2, KBH);
    int f = s;
    if (INV && s >= a.S1 + S2) {
        const int v = (s - a.S1 - S2) % (3 * SC);
        if (v < 2 * SC) f = v < SC ? s + SC : s - SC;
    }
#ifdef NFK_WABL_L2HOT
    f &= 1;  // diagnostic: two frames only (every weight read hits L2)
#endif
#ifdef NFK_WABL_NOSTAGE
    if (s >= 2) return;  // diagnostic: no copies after the prologue
#endif
    float4* slot = (s & 1) ? slot1 : slot0;
    stage_record<kWideWaves>(a.pack + 256 + (int64_t)f * (kWideSlotBlocks * 256), kWideSlotBlocks, slot, wid,
                             lane);
}

// GEMM over sub-record J (k-blocks G J .. G J + G - 1, those below nkb) of a
// record with NT tiles; J == 0 starts the accumulators at bias * bscale.
template <int KBH, int NT, int J>
__device__ __forceinline__ void gemm_sub(const h8 (&bh)[KBH], const h8 (&bl)[KBH], const float4* slot, int lane,
                                         f32x4 (&acc)[NT], int nkb, float bscale) {
    constexpr int G = wide_g(NT, KBH);
    constexpr int NPR = (NT + 1) / 2;
    constexpr int N = G * NPR;
    static_assert(G * (J + 1) <= KBH, "sub-record beyond the k-blocks");
    const int q = lane >> 4;
    if constexpr (J == 0) {
        const float4* bias = slot + kWideFB * 64;
#pragma unroll
        for (int t = 0; t < NT; ++t) {
            const float4 b = bias[t * 4 + q];
            acc[t] = f32x4{b.x * bscale, b.y * bscale, b.z * bscale, b.w * bscale};
        }
    }
    auto blk = [](int i, int j) {  // block j (0..3) of step i: tile pair pr of local k-block kl
        const int kl = i / NPR, pr = i - kl * NPR;
        return (kl * NT + 2 * pr) * 2 + j;
    };
    float4 ring[2][4];
#pragma unroll
    for (int j = 0; j < 4; ++j)
        if ((j >> 1) < NT) ring[0][j] = slot[blk(0, j) * 64 + lane];
#pragma unroll
    for (int i = 0; i < N; ++i) {
        const int kl = i / NPR, pr = i - kl * NPR, t0 = 2 * pr;
        const int kb = G * J + kl;
        const bool two = t0 + 1 < NT;
        if (i + 1 < N) {
            const int pn = (i + 1) % NPR;
#pragma unroll
            for (int j = 0; j < 4; ++j)
                if (2 * pn + (j >> 1) < NT) ring[(i + 1) & 1][j] = slot[blk(i + 1, j) * 64 + lane];
        }
        __builtin_amdgcn_sched_barrier(0);
        if (kl > 0 && kb >= nkb) continue;
        const float4* r = ring[i & 1];
        const h8 ahi0 = __builtin_bit_cast(h8, r[0]), alo0 = __builtin_bit_cast(h8, r[1]);
        if (two) {
            const h8 ahi1 = __builtin_bit_cast(h8, r[2]), alo1 = __builtin_bit_cast(h8, r[3]);
            acc[t0] = mfma16(alo0, bh[kb], acc[t0]);
            acc[t0 + 1] = mfma16(alo1, bh[kb], acc[t0 + 1]);
            acc[t0] = mfma16(ahi0, bl[kb], acc[t0]);
            acc[t0 + 1] = mfma16(ahi1, bl[kb], acc[t0 + 1]);
            acc[t0] = mfma16(ahi0, bh[kb], acc[t0]);
            acc[t0 + 1] = mfma16(ahi1, bh[kb], acc[t0 + 1]);
        } else {
            acc[t0] = mfma16(alo0, bh[kb], acc[t0]);
            acc[t0] = mfma16(ahi0, bl[kb], acc[t0]);
            acc[t0] = mfma16(ahi0, bh[kb], acc[t0]);
        }
    }
}

// A whole phase: the GEMM of each of its sub-records (nsub of them, at most
// KBH/G), each ended by the barrier that recycles its slot and issues the
// copy of sub-record s + 2.
template <int KBH, int K, bool INV, int NT>
__device__ __forceinline__ void wide_phase(const WideArgs& a, int& s, int nsub, int nkb, const h8 (&bh)[KBH],
                                           const h8 (&bl)[KBH], f32x4 (&acc)[NT], float bscale, float4* slot0,
                                           float4* slot1, int wid, int lane, NfkTrace& tr) {
    constexpr int NS = KBH / wide_g(NT, KBH);
    static_assert(NS <= 8, "at most 8 sub-records per phase");
    auto one = [&](auto Jc) {
        constexpr int J = decltype(Jc)::value;
        if (J < nsub) {
            gemm_sub<KBH, NT, J>(bh, bl, (s & 1) ? slot1 : slot0, lane, acc, nkb, bscale);
            NFK_MARK(tr);  // GEMM issued
            asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
            __builtin_amdgcn_s_barrier();
            asm volatile("" ::: "memory");
            NFK_MARK(tr);  // barrier passed
            wide_stage<KBH, K, INV>(a, s + 2, slot0, slot1, wid, lane);
            ++s;
        }
    };
    one(std::integral_constant<int, 0>{});
    if constexpr (NS > 1) one(std::integral_constant<int, 1>{});
    if constexpr (NS > 2) one(std::integral_constant<int, 2>{});
    if constexpr (NS > 3) one(std::integral_constant<int, 3>{});
    if constexpr (NS > 4) one(std::integral_constant<int, 4>{});
    if constexpr (NS > 5) one(std::integral_constant<int, 5>{});
    if constexpr (NS > 6) one(std::integral_constant<int, 6>{});
    if constexpr (NS > 7) one(std::integral_constant<int, 7>{});
}

// Knot epilogue of the wide form: coordinate h (0, 1) of this lane group has
// logit p in register 2h + (p & 1) of tile p >> 1 (see knot_phase).
template <int K, bool SEARCH>
__device__ __forceinline__ void knot_phase_w(const f32x4 (&acc)[K / 2], const float (&xv)[2], const FusedConst& c,
                                             float l2e, int (&kb)[2], float (&ek)[2], float (&sk)[2]) {
#ifdef NFK_WABL_NOEPI
#pragma unroll
    for (int h = 0; h < 2; ++h) {
        float v = 0.0f;
#pragma unroll
        for (int p = 0; p < K; ++p) v += acc[p >> 1][2 * h + (p & 1)];
        if (SEARCH) kb[h] = 0;
        ek[h] = v;
        sk[h] = xv[h];
    }
    return;
#endif
#if NFK_WIDE_PK
    // both coordinates' prefixes as packed pairs (bitwise those of the scalar
    // form, nfk_spline.h), then the selects one coordinate at a time
    int pre2[2][K];
    nfk_f2 s22;
    {
        float u0[K], u1[K];
#pragma unroll
        for (int p = 0; p < K; ++p) {
            u0[p] = acc[p >> 1][p & 1];
            u1[p] = acc[p >> 1][2 + (p & 1)];
        }
        s22 = nfk_prefix_nsf_lean2<K>(u0, u1, l2e, c.m2b, c.fb30, c.mb30, pre2[0], pre2[1]);
    }
#endif
#pragma unroll
    for (int h = 0; h < 2; ++h) {
#if NFK_WIDE_PK
        const int(&pre)[K] = pre2[h];
        const float s2 = h ? s22.y : s22.x;
#else
        float u[K];
        int pre[K];
#pragma unroll
        for (int p = 0; p < K; ++p) u[p] = acc[p >> 1][2 * h + (p & 1)];
        const float s2 = nfk_prefix_nsf_lean<K>(u, l2e, c.m2b, c.fb30, c.mb30, pre);
#endif
        const float lo = __builtin_fmaf(s2, 0.0f, c.lo);  // NaN iff the logits were (knot_phase)
        int p0 = 0, p1 = pre[1 < K ? 1 : 0], k = 0;
        const int xi = __float2int_rd(__builtin_fmaf(xv[h], c.inv30, -c.lo * c.inv30));
#pragma unroll
        for (int j = 1; j < K; ++j) {
            const bool ge = SEARCH ? (xi >= pre[j]) : (kb[h] >= j);
            p0 = ge ? pre[j] : p0;
            if (j + 1 < K) p1 = ge ? pre[j + 1] : p1;
            if (SEARCH) k += ge ? 1 : 0;
        }
        if (SEARCH) kb[h] = k;
        const int kk = kb[h];
        const float e = __builtin_fmaf(c.sp30, (float)p0, lo);
        const float e1 = (kk == K - 1) ? c.hi : __builtin_fmaf(c.sp30, (float)p1, lo);
        ek[h] = e;
        sk[h] = e1 - e;
        if constexpr (K > 8 && !NFK_WIDE_PK) __builtin_amdgcn_sched_barrier(0);  // one coordinate at a time
    }
}

// Pin a knot epilogue's results at its place in the schedule: without it
// the compiler sinks the searched-knot and other-knot epilogues below the
// derivative record's GEMMs (only register dependences order them), so the
// logits of three records stay live at once (256 VGPRs and scratch spills
// whose reloads wait on the frame copies in flight) and every epilogue of a
// chunk runs back to back.
__device__ __forceinline__ void wide_pin(int (&kb)[2], float (&e)[2], float (&s)[2]) {
#if NFK_WIDE_PIN
#pragma unroll
    for (int h = 0; h < 2; ++h) asm volatile("" : "+v"(kb[h]), "+v"(e[h]), "+v"(s[h]));
#endif
}

// Column of a chunk-pair tile: even t = lower coordinate 16 g + t/2, odd t = upper.
__device__ __forceinline__ int wide_col(const int32_t* m_lo, const int32_t* m_up, int n_lo, int n_up, int g, int t,
                                        bool& valid) {
    const int j = 16 * g + (t >> 1);
    if (t & 1) {
        valid = j < n_up;
        return m_up[valid ? j : 0];
    }
    valid = j < n_lo;
    return m_lo[valid ? j : 0];
}

// LDS-DMA gather of pair g's x tile: element e = 64 i + lane is (e >> 5, e & 31)
__device__ __forceinline__ void wide_gather(const WideArgs& a, const int32_t* m_lo_in, const int32_t* m_up_in,
                                            int64_t b0, int g, float* tile, int lane) {
    const uint32_t base = lds_addr(tile);
#pragma unroll
    for (int i = 0; i < 8; ++i) {
        const int e = 64 * i + lane, r = e >> 5, t = e & 31;
        bool ok;
        const int col = wide_col(m_lo_in, m_up_in, a.n_lo, a.n_up, g, t, ok);
        int64_t row = b0 + r;
        if (row >= a.batch) row = a.batch - 1;
        dma4(a.x + row * a.ldx + col, base + i * 256);
    }
}

// z of pair g from the tile (upper coordinates transformed, lower ones passed through)
__device__ __forceinline__ void wide_store(const WideArgs& a, const int32_t* m_lo_out, const int32_t* m_up_out,
                                           int64_t b0, int nrows, int g, const float* tile, int lane) {
    float v[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) v[i] = tile[64 * i + lane];
#pragma unroll
    for (int i = 0; i < 8; ++i) {
        const int e = 64 * i + lane, r = e >> 5, t = e & 31;
        bool ok;
        const int col = wide_col(m_lo_out, m_up_out, a.n_lo, a.n_up, g, t, ok);
        if (ok && r < nrows) a.z[(b0 + r) * a.ldz + col] = v[i];
    }
}

template <int KBH, int K, bool INV>
__global__ __launch_bounds__(64 * kWideWaves, kWideWGs) void k_fused_nsf_wide(WideArgs a) {
    constexpr int HT = 2 * KBH;
    constexpr int NTC = K / 2;  // tiles of a chunk's W, H or D record
    constexpr int S2 = KBH / wide_g(HT, KBH);
    constexpr int SC = KBH / wide_g(NTC, KBH);
    static_assert(K % 2 == 0, "wide form needs even K");
    const int lane = threadIdx.x & 63;
    const int wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int q = lane >> 4, sl = lane & 15;
    extern __shared__ __attribute__((aligned(16))) float4 lds4[];
    float4* slot0 = lds4;
    float4* slot1 = lds4 + kWideSlotBlocks * 64;
    int32_t* m_up_in = reinterpret_cast<int32_t*>(lds4 + 2 * kWideSlotBlocks * 64);
    int32_t* m_up_out = m_up_in + a.n_up;
    int32_t* m_lo_in = m_up_out + a.n_up;
    int32_t* m_lo_out = m_lo_in + a.n_lo;
    float* tile = reinterpret_cast<float*>(lds4 + 2 * kWideSlotBlocks * 64 + (2 * (a.n_lo + a.n_up) + 3) / 4) +
                  wid * kWideTile;
    const int64_t b0 = ((int64_t)blockIdx.x * kWideWaves + wid) * 16;
    const int64_t rem = a.batch - b0;
    const int nrows = rem <= 0 ? 0 : (rem < 16 ? (int)rem : 16);
    const bool row_ok = sl < nrows;
    const FusedConst c = a.c;  // by value: SGPRs
    const float* pk = a.pack;
    NfkTrace tr;
    NFK_MARK(tr);  // start

    // ---- prologue: index maps (plain loads, no copy in flight yet)
    for (int i = threadIdx.x; i < a.n_up; i += 64 * kWideWaves) {
        m_up_in[i] = a.up_in[i];
        m_up_out[i] = a.up_out[i];
    }
    for (int i = threadIdx.x; i < a.n_lo; i += 64 * kWideWaves) {
        m_lo_in[i] = a.lo_in[i];
        m_lo_out[i] = a.lo_out[i];
    }
    const float un1 = pk[3], un2 = pk[4], un3 = pk[5];
    __syncthreads();
    int s = 0;
    wide_stage<KBH, K, INV>(a, 0, slot0, slot1, wid, lane);
    wide_stage<KBH, K, INV>(a, 1, slot0, slot1, wid, lane);
    wide_gather(a, m_lo_in, m_up_in, b0, 0, tile, lane);

    // layer-1 operands: x at the lower coordinates of sample sl, k = 32 kb + 8 q + j
    h8 bh[KBH], bl[KBH];
    float unx, bsc;
    {
        int64_t row = b0 + sl;
        if (row >= a.batch) row = a.batch - 1;
        const float* xr = a.x + row * a.ldx;
        float xv[KBH][8];
        float mx = 0.0f;
#pragma unroll
        for (int kb = 0; kb < KBH; ++kb)
#pragma unroll
            for (int j = 0; j < 8; ++j) {
                const int k = 32 * kb + 8 * q + j;
                xv[kb][j] = (kb < a.KB1 && k < a.n_lo) ? xr[m_lo_in[k]] : 0.0f;
                mx = fmaxf(mx, fabsf(xv[kb][j]));
            }
#pragma unroll
        for (int off = 16; off < 64; off <<= 1) mx = fmaxf(mx, __shfl_xor(mx, off, 64));  // per sample: the 4 lanes of column sl
        int ex = 0;
        if (mx > 0.0f && mx < 3.0e38f) frexpf(mx, &ex);  // mx < 2^ex
        ex = ex < -64 ? -64 : ex;  // a tiny sample: its scale 2^(14 - ex) and bias scale stay finite
        const float sx = ldexpf(1.0f, 14 - ex);
        unx = ldexpf(un1, ex - 14);
        bsc = sx / un1;  // bias b1 2^(s1 + sx): the epilogue only multiplies by 2^-(s1 + sx)
#pragma unroll
        for (int kb = 0; kb < KBH; ++kb)
#pragma unroll
            for (int j = 0; j < 8; ++j) {
                const float v = xv[kb][j] * sx;
                const _Float16 hh = (_Float16)v;
                bh[kb][j] = hh;
                bl[kb][j] = (_Float16)(v - (float)hh);
            }
    }
    dma_barrier();  // sub-records 0, 1 and the first x tile landed
    NFK_MARK(tr);  // prologue done

    // ---- layer 1 (S1 sub-steps) and layer 2 (S2 sub-steps)
    h4 btail;
    {
        f32x4 h[HT];
        wide_phase<KBH, K, INV, HT>(a, s, a.S1, a.KB1, bh, bl, h, bsc, slot0, slot1, wid, lane, tr);
        act_operands<KBH, false, HT>(h, -2.0f * kL2E * unx, bh, bl, btail);
        wide_phase<KBH, K, INV, HT>(a, s, S2, KBH, bh, bl, h, 1.0f, slot0, slot1, wid, lane, tr);
        act_operands<KBH, false, HT>(h, -2.0f * kL2E * un2, bh, bl, btail);
    }

    const float l2e3 = kL2E * un3;
    float ldsum = 0.0f;
    bool any_in = false, any_nd = false;
    for (int ch = 0; ch < a.NCH; ++ch) {
        const int g = ch >> 1;
        // this lane group's coordinates 8 ch + 2 q + h; tile column of upper coordinate
        const int tcol = 2 * (8 * (ch & 1) + 2 * q) + 1;
        int jj[2];
        float xv[2];
        int kb[2];
        float cw_k[2], w_k[2], ch_k[2], h_k[2];

        // ---- searched knots (widths forward / heights inverse)
        {
            f32x4 acc[NTC];
            wide_phase<KBH, K, INV, NTC>(a, s, SC, KBH, bh, bl, acc, 1.0f, slot0, slot1, wid, lane, tr);
            const float4 u = *reinterpret_cast<const float4*>(tile + sl * 32 + tcol - 1);
            xv[0] = u.y;
            xv[1] = u.w;
#pragma unroll
            for (int h = 0; h < 2; ++h) {
                jj[h] = 8 * ch + 2 * q + h;
                if (jj[h] >= a.n_up) xv[h] = 0.0f;
            }
            knot_phase_w<K, true>(acc, xv, c, l2e3, kb, INV ? ch_k : cw_k, INV ? h_k : w_k);
            wide_pin(kb, INV ? ch_k : cw_k, INV ? h_k : w_k);
            NFK_MARK(tr);  // epilogue A
        }
        // ---- the other knots, selected at the bin
        {
            f32x4 acc[NTC];
            wide_phase<KBH, K, INV, NTC>(a, s, SC, KBH, bh, bl, acc, 1.0f, slot0, slot1, wid, lane, tr);
            knot_phase_w<K, false>(acc, xv, c, l2e3, kb, INV ? cw_k : ch_k, INV ? w_k : h_k);
            wide_pin(kb, INV ? cw_k : ch_k, INV ? w_k : h_k);
            NFK_MARK(tr);  // epilogue B
        }
        // ---- derivatives of the bin, evaluate, log|det|
        {
            f32x4 accd[NTC];
            wide_phase<KBH, K, INV, NTC>(a, s, SC, KBH, bh, bl, accd, 1.0f, slot0, slot1, wid, lane, tr);
            float outv[2];
#ifdef NFK_WABL_NOEPI
#pragma unroll
            for (int h = 0; h < 2; ++h) {
                float v = cw_k[h] + w_k[h] + ch_k[h] + h_k[h];
#pragma unroll
                for (int t = 0; t < NTC; ++t) v += accd[t][2 * h] + accd[t][2 * h + 1];
                outv[h] = v;
                ldsum += v;
                any_in = true;
            }
            if (false)
#endif
#pragma unroll
            for (int h = 0; h < 2; ++h) {
                // derivative logit j in register 2h + (j & 1) of tile j >> 1;
                // padded index j+1 holds logit j (utils.py:36-39): raw_k = logit k-1, raw_k1 = logit k
                const int k = kb[h];
                float raw_k = accd[0][2 * h], raw_k1 = accd[0][2 * h];
#pragma unroll
                for (int j = 1; j < K - 1; ++j) {
                    const float v = accd[j >> 1][2 * h + (j & 1)];
                    raw_k = (k >= j + 1) ? v : raw_k;
                    raw_k1 = (k >= j) ? v : raw_k1;
                }
                const float d_k = (k == 0) ? c.d_edge : nfk_deriv_lean_s(raw_k, l2e3, c.min_d);
                const float d_k1 = (k == K - 1) ? c.d_edge : nfk_deriv_lean_s(raw_k1, l2e3, c.min_d);
                const float x = xv[h];
                const float rw = nfk_rcp_fast(w_k[h]);
                const float delta = h_k[h] * rw;
                const float gap = (d_k + d_k1) - 2.0f * delta;
                float out, th;
                bool nd = false;
                if (INV) {
                    const float y = x - ch_k[h];
                    const float qa = y * gap + h_k[h] * (delta - d_k);
                    const float qb = h_k[h] * d_k - y * gap;
                    const float qc = (-delta) * y;
                    const float disc = qb * qb - (4.0f * qa) * qc;
                    nd = !(disc >= 0.0f);
                    const float root = nfk_div<true>(2.0f * qc, -qb - sqrtf(disc));
                    out = root * w_k[h] + cw_k[h];
                    th = root;
                } else {
                    th = (x - cw_k[h]) * rw;
                }
                const float t1mt = th * (1.0f - th);
                const float den = delta + gap * t1mt;
                if (!INV) {
                    const float num = h_k[h] * (delta * (th * th) + d_k * t1mt);
                    out = ch_k[h] + nfk_div<true>(num, den);
                }
                const float omt = 1.0f - th;
                const float dnum =
                    (delta * delta) * ((d_k1 * (th * th) + (2.0f * delta) * t1mt) + d_k * (omt * omt));
                float lad = (__builtin_amdgcn_logf(dnum) - 2.0f * __builtin_amdgcn_logf(den)) * kLN2;
                lad = INV ? -lad : lad;
                const bool inside = (x >= c.lo) && (x <= c.hi);
                const bool live = jj[h] < a.n_up && row_ok;
                outv[h] = inside ? out : x;
                ldsum += (inside && live) ? lad : 0.0f;
                any_in |= inside && live;
                any_nd |= nd && inside && live;
            }
            float* tw = tile + sl * 32 + tcol;
            tw[0] = outv[0];  // z back into the upper columns
            tw[2] = outv[1];
            NFK_MARK(tr);  // epilogue C
        }
        // after a chunk pair: its z, then the next pair's x into the same tile
        // (the stores' data left the tile before the copy is issued)
        if ((ch & 1) || ch + 1 == a.NCH) {
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
            wide_store(a, m_lo_out, m_up_out, b0, nrows, g, tile, lane);
            if (ch + 1 < a.NCH) {
                asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
                wide_gather(a, m_lo_in, m_up_in, b0, g + 1, tile, lane);
            }
        }
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
#ifdef NFK_TRACE
    NFK_MARK(tr);  // end
    nfk_trace_flush(tr, a.trace, wid, lane);
#endif
}

template <int KBH, int K>
int launch_fused_wide(const WideArgs& a, size_t lds, bool inv, hipStream_t st) {
    const int64_t per_block = (int64_t)kWideWaves * 16;
    const int64_t blocks = (a.batch + per_block - 1) / per_block;
    if (blocks == 0) return 0;
    if (inv)
        hipLaunchKernelGGL((k_fused_nsf_wide<KBH, K, true>), dim3((unsigned)blocks), dim3(64 * kWideWaves), lds, st, a);
    else
        hipLaunchKernelGGL((k_fused_nsf_wide<KBH, K, false>), dim3((unsigned)blocks), dim3(64 * kWideWaves), lds, st, a);
    hipError_t e = hipGetLastError();
    return e == hipSuccess ? 0 : (int)e;
}

#define NFK_WIDE_INSTANCE(KBH, K) \
    template int launch_fused_wide<KBH, K>(const WideArgs& a, size_t lds, bool inv, hipStream_t st);
#define NFK_WIDE_EXTERN(KBH, K) \
    extern template int launch_fused_wide<KBH, K>(const WideArgs& a, size_t lds, bool inv, hipStream_t st);

// hidden widths H = 32 KBH (no f32 tail), bins K
#define NFK_WIDE_KB(X) X(4) X(8)
#define NFK_WIDE_K(X, KBH) X(KBH, 8) X(KBH, 16)

}  // namespace nfk_fused
