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
//     waited on, and split there (per-wave power-of-two scale as before);
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
#ifndef NFK_WIDE_PIPE
#define NFK_WIDE_PIPE 1  // two-tile form: pipelined chunk schedule
#endif
#ifndef NFK_WIDE_BAGPR
#define NFK_WIDE_BAGPR 1
#endif
#ifndef NFK_WIDE_SGB
#define NFK_WIDE_SGB 0  // pipelined schedule: sched_group_barrier pattern (measured: defeats interleaving)
#endif
#ifndef NFK_WIDE_FV
#define NFK_WIDE_FV 2  // pipelined schedule: filler VALU instructions per MFMA
#endif
constexpr int kWideFB = NFK_WIDE_FB;             // f16 blocks of a frame
constexpr int kWideSlotBlocks = kWideFB + 1;     // + the record's bias block
constexpr int kWideWaves = NFK_WIDE_NW;          // waves per workgroup
constexpr int kWideWGs = kWideWaves == 4 ? 2 : 1;  // workgroups per CU
constexpr int kWideTile = 16 * 32;               // floats of a wave's chunk-pair tile
static_assert(kWideFB == 32 || kWideFB == 64, "frame of 32 or 64 blocks");
static_assert(kWideWaves == 4 || kWideWaves == 8 || kWideWaves == 12, "4-, 8- or 12-wave workgroups");
// Two-tile form (NU = 2): every wave owns two 16-row sample tiles, so each A
// fragment read from the slot feeds the MFMAs of both (half the ds_read_b128
// bytes per MFMA: the one-tile form's GEMMs ran the LDS array at its 256
// B/clk/CU peak); one 4-wave workgroup per CU, 512 registers per lane.  The
// rows of tile u of wave w are those of wave 2w + u of the one-tile form, so
// both forms are bitwise equal.
template <int NU>
__host__ __device__ constexpr int wide_nw() {
    return NU == 2 ? 4 : kWideWaves;
}
template <int NU>
__host__ __device__ constexpr int wide_wgs() {
    return NU == 2 ? 1 : kWideWGs;
}

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

// LDS of a workgroup of the form with nu sample tiles per wave (one x tile each)
// (two-tile form: plus a 16 x 16 buffer of the pair's upper x per tile, the
// pipelined schedule's spline inputs)
inline size_t wide_lds_bytes(int n_lo, int n_up, int nu = 1) {
    const int tiles = nu == 2 ? 2 * wide_nw<2>() : kWideWaves;
    return 2 * (size_t)kWideSlotBlocks * 1024 + (size_t)((2 * (n_lo + n_up) + 3) / 4) * 16 +
           (size_t)tiles * kWideTile * sizeof(float) + (nu == 2 ? (size_t)tiles * 256 * sizeof(float) : 0);
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
template <int KBH, int K, bool INV, int NW>
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
    stage_record<NW>(a.pack + 256 + (int64_t)f * (kWideSlotBlocks * 256), kWideSlotBlocks, slot, wid,
                             lane);
}

// GEMM over sub-record J (k-blocks G J .. G J + G - 1, those below nkb) of a
// record with NT tiles, for the NU sample tiles of this wave (each A fragment
// feeds all of them); J == 0 starts the accumulators at bias * bscale[u].
// Per accumulator the products run in the one-tile order (lo hi, hi lo, hi hi).
template <int KBH, int NT, int J, int NU, bool SB = true, class Mid = int>
__device__ __forceinline__ void gemm_sub(const h8 (&bh)[NU][KBH], const h8 (&bl)[NU][KBH], const float4* slot,
                                         int lane, f32x4 (&acc)[NU][NT], int nkb, const float (&bscale)[NU],
                                         Mid mid = 0) {
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
#pragma unroll
            for (int u = 0; u < NU; ++u)
                acc[u][t] = f32x4{b.x * bscale[u], b.y * bscale[u], b.z * bscale[u], b.w * bscale[u]};
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
        if constexpr (SB) __builtin_amdgcn_sched_barrier(0);
        if constexpr (!std::is_same<Mid, int>::value) {
            // the filler's second half, in the GEMM's second half (its own
            // scheduling region: half the epilogue's live values per region)
            if (i == N / 2) {
                __builtin_amdgcn_sched_barrier(0);
                mid();
            }
        }
        if (kl > 0 && kb >= nkb) continue;
        const float4* r = ring[i & 1];
        const h8 ahi0 = __builtin_bit_cast(h8, r[0]), alo0 = __builtin_bit_cast(h8, r[1]);
        if (two) {
            const h8 ahi1 = __builtin_bit_cast(h8, r[2]), alo1 = __builtin_bit_cast(h8, r[3]);
#pragma unroll
            for (int u = 0; u < NU; ++u) {
                acc[u][t0] = mfma16(alo0, bh[u][kb], acc[u][t0]);
                acc[u][t0 + 1] = mfma16(alo1, bh[u][kb], acc[u][t0 + 1]);
            }
#pragma unroll
            for (int u = 0; u < NU; ++u) {
                acc[u][t0] = mfma16(ahi0, bl[u][kb], acc[u][t0]);
                acc[u][t0 + 1] = mfma16(ahi1, bl[u][kb], acc[u][t0 + 1]);
            }
#pragma unroll
            for (int u = 0; u < NU; ++u) {
                acc[u][t0] = mfma16(ahi0, bh[u][kb], acc[u][t0]);
                acc[u][t0 + 1] = mfma16(ahi1, bh[u][kb], acc[u][t0 + 1]);
            }
        } else {
#pragma unroll
            for (int u = 0; u < NU; ++u) acc[u][t0] = mfma16(alo0, bh[u][kb], acc[u][t0]);
#pragma unroll
            for (int u = 0; u < NU; ++u) acc[u][t0] = mfma16(ahi0, bl[u][kb], acc[u][t0]);
#pragma unroll
            for (int u = 0; u < NU; ++u) acc[u][t0] = mfma16(ahi0, bh[u][kb], acc[u][t0]);
        }
    }
}

// A whole phase: the GEMM of each of its sub-records (nsub of them, at most
// KBH/G), each ended by the barrier that recycles its slot and issues the
// copy of sub-record s + 2.
struct NoFill {
    __device__ void operator()(int, int) const {}
};

// fill(J, part): independent work placed in sub-step J's basic block beside
// its MFMAs (the pipelined chunk schedule: the previous record's epilogue):
// part 0 with the GEMM's first half, part 1 with its second half (a
// scheduling fence between), part 2 after it (result pins, LDS stores: what
// orders against the GEMM's LDS reads); with a filler the GEMM steps carry
// no other scheduling barriers, so the scheduler can interleave each half
template <int KBH, int K, bool INV, int NT, int NU, class Fill = NoFill>
__device__ __forceinline__ void wide_phase(const WideArgs& a, int& s, int nsub, int nkb, const h8 (&bh)[NU][KBH],
                                           const h8 (&bl)[NU][KBH], f32x4 (&acc)[NU][NT],
                                           const float (&bscale)[NU], float4* slot0, float4* slot1, int wid,
                                           int lane, NfkTrace& tr, Fill fill = Fill{}) {
    constexpr int NS = KBH / wide_g(NT, KBH);
    constexpr bool FILL = !std::is_same<Fill, NoFill>::value;
    static_assert(NS <= 8, "at most 8 sub-records per phase");
    auto one = [&](auto Jc) {
        constexpr int J = decltype(Jc)::value;
        if (J < nsub) {
            if constexpr (FILL) {
                fill(J, 0);
                gemm_sub<KBH, NT, J, NU, false>(bh, bl, (s & 1) ? slot1 : slot0, lane, acc, nkb, bscale,
                                                [&] { fill(J, 1); });
            } else {
                gemm_sub<KBH, NT, J, NU>(bh, bl, (s & 1) ? slot1 : slot0, lane, acc, nkb, bscale);
            }
            if constexpr (FILL && NFK_WIDE_SGB) {
                // interleave: per GEMM step its A-fragment reads, then each
                // MFMA followed by NFK_WIDE_FV filler VALU instructions
                constexpr int G = wide_g(NT, KBH), NPR = (NT + 1) / 2;
#pragma unroll
                for (int i = 0; i < G * NPR; ++i) {
                    __builtin_amdgcn_sched_group_barrier(0x100, 4, 0);
#pragma unroll
                    for (int m = 0; m < 6 * NU; ++m) {
                        __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
                        __builtin_amdgcn_sched_group_barrier(0x002, NFK_WIDE_FV, 0);
                    }
                }
            }
            if constexpr (FILL) fill(J, 2);
            NFK_MARK(tr);  // GEMM issued
            asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
            __builtin_amdgcn_s_barrier();
            asm volatile("" ::: "memory");
            NFK_MARK(tr);  // barrier passed
            wide_stage<KBH, K, INV, wide_nw<NU>()>(a, s + 2, slot0, slot1, wid, lane);
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

// knot_phase_w for coordinate h of this lane group alone (scalar prefixes:
// bitwise the packed pair form), the pipelined schedule's half-epilogue
template <int K, bool SEARCH>
__device__ __forceinline__ void knot_one_w(const f32x4 (&acc)[K / 2], int h, float xv, const FusedConst& c, float l2e,
                                           int& kb, float& ek, float& sk) {
    float u[K];
    int pre[K];
#pragma unroll
    for (int p = 0; p < K; ++p) u[p] = acc[p >> 1][2 * h + (p & 1)];
    const float s2 = nfk_prefix_nsf_lean<K>(u, l2e, c.m2b, c.fb30, c.mb30, pre);
    const float lo = __builtin_fmaf(s2, 0.0f, c.lo);  // NaN iff the logits were (knot_phase)
    int p0 = 0, p1 = pre[1 < K ? 1 : 0], k = 0;
    const int xi = __float2int_rd(__builtin_fmaf(xv, c.inv30, -c.lo * c.inv30));
#pragma unroll
    for (int j = 1; j < K; ++j) {
        const bool ge = SEARCH ? (xi >= pre[j]) : (kb >= j);
        p0 = ge ? pre[j] : p0;
        if (j + 1 < K) p1 = ge ? pre[j + 1] : p1;
        if (SEARCH) k += ge ? 1 : 0;
    }
    if (SEARCH) kb = k;
    const float e = __builtin_fmaf(c.sp30, (float)p0, lo);
    const float e1 = (kb == K - 1) ? c.hi : __builtin_fmaf(c.sp30, (float)p1, lo);
    ek = e;
    sk = e1 - e;
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

// LDS-DMA gather of the upper x of pair g (16 rows x upper coordinates
// 16 g .. 16 g + 15) into a 16 x 16 buffer: element e = 64 i + lane is (e >> 4, e & 15)
__device__ __forceinline__ void wide_gather_up(const WideArgs& a, const int32_t* m_up_in, int64_t b0, int g,
                                               float* xb, int lane) {
    const uint32_t base = lds_addr(xb);
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const int e = 64 * i + lane, r = e >> 4, j = 16 * g + (e & 15);
        const int col = m_up_in[j < a.n_up ? j : 0];
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

template <int KBH, int K, bool INV, int NU>
__global__ __launch_bounds__(64 * wide_nw<NU>(), wide_wgs<NU>()) void k_fused_nsf_wide(WideArgs a) {
    constexpr int NW = wide_nw<NU>();
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
    float* tiles0 = reinterpret_cast<float*>(lds4 + 2 * kWideSlotBlocks * 64 + (2 * (a.n_lo + a.n_up) + 3) / 4);
    float* tiles = tiles0 + wid * NU * kWideTile;  // x tile of sample tile u: tiles + u * kWideTile
    // two-tile form: upper x of the current pair, 16 x 16 per tile
    float* xbuf = tiles0 + NW * NU * kWideTile + wid * NU * 256;
    int64_t b0[NU];
    int nrows[NU];
    bool row_ok[NU];
#pragma unroll
    for (int u = 0; u < NU; ++u) {
        b0[u] = (((int64_t)blockIdx.x * NW + wid) * NU + u) * 16;
        const int64_t rem = a.batch - b0[u];
        nrows[u] = rem <= 0 ? 0 : (rem < 16 ? (int)rem : 16);
        row_ok[u] = sl < nrows[u];
    }
    const FusedConst c = a.c;  // by value: SGPRs
    const float* pk = a.pack;
    NfkTrace tr;
    NFK_MARK(tr);  // start

    // ---- prologue: index maps (plain loads, no copy in flight yet)
    for (int i = threadIdx.x; i < a.n_up; i += 64 * NW) {
        m_up_in[i] = a.up_in[i];
        m_up_out[i] = a.up_out[i];
    }
    for (int i = threadIdx.x; i < a.n_lo; i += 64 * NW) {
        m_lo_in[i] = a.lo_in[i];
        m_lo_out[i] = a.lo_out[i];
    }
    const float un1 = pk[3], un2 = pk[4], un3 = pk[5];
    __syncthreads();
    int s = 0;
    wide_stage<KBH, K, INV, NW>(a, 0, slot0, slot1, wid, lane);
    wide_stage<KBH, K, INV, NW>(a, 1, slot0, slot1, wid, lane);
#pragma unroll
    for (int u = 0; u < NU; ++u) wide_gather(a, m_lo_in, m_up_in, b0[u], 0, tiles + u * kWideTile, lane);
    if constexpr (NU == 2 && NFK_WIDE_PIPE)
#pragma unroll
        for (int u = 0; u < NU; ++u) wide_gather_up(a, m_up_in, b0[u], 0, xbuf + u * 256, lane);

    // layer-1 operands: x at the lower coordinates of sample sl, k = 32 kb + 8 q + j
    // (per sample tile: its own power-of-two scale, as one wave of the one-tile form)
    h8 bh[NU][KBH], bl[NU][KBH];
    float unx[NU], bsc[NU], ones[NU];
#pragma unroll
    for (int u = 0; u < NU; ++u) {
        ones[u] = 1.0f;
        int64_t row = b0[u] + sl;
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
        for (int off = 32; off > 0; off >>= 1) mx = fmaxf(mx, __shfl_xor(mx, off, 64));
        int ex = 0;
        if (mx > 0.0f && mx < 3.0e38f) frexpf(mx, &ex);  // mx < 2^ex
        const float sx = ldexpf(1.0f, 14 - ex);
        unx[u] = ldexpf(un1, ex - 14);
        bsc[u] = sx / un1;  // bias b1 2^(s1 + sx): the epilogue only multiplies by 2^-(s1 + sx)
#pragma unroll
        for (int kb = 0; kb < KBH; ++kb)
#pragma unroll
            for (int j = 0; j < 8; ++j) {
                const float v = xv[kb][j] * sx;
                const _Float16 hh = (_Float16)v;
                bh[u][kb][j] = hh;
                bl[u][kb][j] = (_Float16)(v - (float)hh);
            }
    }
    dma_barrier();  // sub-records 0, 1 and the first x tiles landed
    NFK_MARK(tr);  // prologue done

    // ---- layer 1 (S1 sub-steps) and layer 2 (S2 sub-steps)
    {
        h4 btail;
        f32x4 h[NU][HT];
        wide_phase<KBH, K, INV, HT, NU>(a, s, a.S1, a.KB1, bh, bl, h, bsc, slot0, slot1, wid, lane, tr);
#pragma unroll
        for (int u = 0; u < NU; ++u) act_operands<KBH, false, HT>(h[u], -2.0f * kL2E * unx[u], bh[u], bl[u], btail);
        wide_phase<KBH, K, INV, HT, NU>(a, s, S2, KBH, bh, bl, h, ones, slot0, slot1, wid, lane, tr);
#pragma unroll
        for (int u = 0; u < NU; ++u) act_operands<KBH, false, HT>(h[u], -2.0f * kL2E * un2, bh[u], bl[u], btail);
#if NFK_WIDE_BAGPR
        // two-tile pipelined form: the output layer's B operands live in
        // AGPRs (MFMA sources may be AGPRs), leaving the VGPRs to the
        // epilogue the schedule interleaves with the GEMM
        if constexpr (NU == 2 && NFK_WIDE_PIPE)
#pragma unroll
            for (int u = 0; u < NU; ++u)
#pragma unroll
                for (int kb = 0; kb < KBH; ++kb) asm volatile("" : "+a"(bh[u][kb]), "+a"(bl[u][kb]));
#endif
    }

    const float l2e3 = kL2E * un3;
    float ldsum[NU];
#pragma unroll
    for (int u = 0; u < NU; ++u) ldsum[u] = 0.0f;
    bool any_in = false, any_nd = false;
    if constexpr (NU == 2 && NFK_WIDE_PIPE) {
        // Pipelined chunk schedule: a record's spline epilogue runs beside the
        // NEXT record's GEMM (fill), tile u's in sub-step u (both in sub-step
        // 0 of one-sub-step records): A(ch) GEMM | C(ch-1) epilogue, B(ch) |
        // A(ch), C(ch) | B(ch).  Same arithmetic, so bitwise the other forms.
        // The searched phase reads x from xbuf (the pair's upper x, gathered a
        // phase ahead), so the z tile of a pair can be stored and refilled
        // while the next pair's first epilogues run.
        int kb[NU][2];
        float xv[NU][2], cw_k[NU][2], w_k[NU][2], ch_k[NU][2], h_k[NU][2];
        f32x4 accA[NU][NTC], accB[NU][NTC], accC[NU][NTC];
        float zout[NU][2];
        // pins: the epilogue's inputs and results pass through empty volatile
        // asm at the start and end of its pieces, so the optimiser cannot move
        // the (side-effect free) epilogue out of the GEMM's regions
        auto pin_in = [](f32x4 (&v)[NTC], int h) {
#pragma unroll
            for (int t = 0; t < NTC; ++t)
#pragma unroll
                for (int r = 0; r < 2; ++r) {
                    float e = v[t][2 * h + r];
                    asm volatile("" : "+v"(e));
                    v[t][2 * h + r] = e;
                }
        };
        // the pieces of sub-step J's filler: part 0 (beside the GEMM's first
        // half) and part 1 (its second half) are (tile, coordinate) pieces,
        // part 2 the closing pins/stores per tile.  Two-sub-step records
        // (K = 16): tile J, coordinate = part; one-sub-step records: tile =
        // part, both coordinates.
        auto pieces = [&](int J, int part, auto&& f) {
            if (SC == 1) {
                if (part < 2) {
                    f(part, 0, false);
                    f(part, 1, false);
                } else {
                    f(0, 0, true);
                    f(1, 0, true);
                }
            } else if (J < 2) {
                f(J, part < 2 ? part : 0, part == 2);
            }
        };
        auto epi_a = [&](int u, int h, bool fin) {
            if (fin) {
                wide_pin(kb[u], INV ? ch_k[u] : cw_k[u], INV ? h_k[u] : w_k[u]);
                return;
            }
            pin_in(accA[u], h);
            knot_one_w<K, true>(accA[u], h, xv[u][h], c, l2e3, kb[u][h], INV ? ch_k[u][h] : cw_k[u][h],
                                INV ? h_k[u][h] : w_k[u][h]);
        };
        // chunk ch's spline inputs from xbuf, read at the end of its searched
        // record's GEMM (the epilogue that needs them runs in the next phase)
        auto read_xv = [&](int ch, int u) {
            const float2 v = *reinterpret_cast<const float2*>(xbuf + u * 256 + sl * 16 + 8 * (ch & 1) + 2 * q);
            xv[u][0] = 8 * ch + 2 * q < a.n_up ? v.x : 0.0f;
            xv[u][1] = 8 * ch + 2 * q + 1 < a.n_up ? v.y : 0.0f;
            asm volatile("" : "+v"(xv[u][0]), "+v"(xv[u][1]));
        };
        auto epi_b = [&](int u, int h, bool fin) {
            if (fin) {
                wide_pin(kb[u], INV ? cw_k[u] : ch_k[u], INV ? w_k[u] : h_k[u]);
                return;
            }
            pin_in(accB[u], h);
            knot_one_w<K, false>(accB[u], h, xv[u][h], c, l2e3, kb[u][h], INV ? cw_k[u][h] : ch_k[u][h],
                                 INV ? w_k[u][h] : h_k[u][h]);
        };
        auto epi_c = [&](int ch, int u, int h, bool fin) {
            if (fin) {
                asm volatile("" : "+v"(ldsum[u]), "+v"(zout[u][0]), "+v"(zout[u][1]));
                float* tw = tiles + u * kWideTile + sl * 32 + 2 * (8 * (ch & 1) + 2 * q) + 1;
                tw[0] = zout[u][0];  // z back into the upper columns
                tw[2] = zout[u][1];
                return;
            }
            pin_in(accC[u], h);
            const int k = kb[u][h];
            float raw_k = accC[u][0][2 * h], raw_k1 = accC[u][0][2 * h];
#pragma unroll
            for (int j = 1; j < K - 1; ++j) {
                const float v = accC[u][j >> 1][2 * h + (j & 1)];
                raw_k = (k >= j + 1) ? v : raw_k;
                raw_k1 = (k >= j) ? v : raw_k1;
            }
            const float d_k = (k == 0) ? c.d_edge : nfk_deriv_lean(raw_k * un3, c.min_d);
            const float d_k1 = (k == K - 1) ? c.d_edge : nfk_deriv_lean(raw_k1 * un3, c.min_d);
            const float x = xv[u][h];
            const float wk = w_k[u][h], hk = h_k[u][h], cwk = cw_k[u][h], chk = ch_k[u][h];
            const float rw = nfk_rcp_fast(wk);
            const float delta = hk * rw;
            const float gap = (d_k + d_k1) - 2.0f * delta;
            float out, th;
            bool nd = false;
            if (INV) {
                const float y = x - chk;
                const float qa = y * gap + hk * (delta - d_k);
                const float qb = hk * d_k - y * gap;
                const float qc = (-delta) * y;
                const float disc = qb * qb - (4.0f * qa) * qc;
                nd = !(disc >= 0.0f);
                const float root = nfk_div<true>(2.0f * qc, -qb - sqrtf(disc));
                out = root * wk + cwk;
                th = root;
            } else {
                th = (x - cwk) * rw;
            }
            const float t1mt = th * (1.0f - th);
            const float den = delta + gap * t1mt;
            if (!INV) {
                const float num = hk * (delta * (th * th) + d_k * t1mt);
                out = chk + nfk_div<true>(num, den);
            }
            const float omt = 1.0f - th;
            const float dnum = (delta * delta) * ((d_k1 * (th * th) + (2.0f * delta) * t1mt) + d_k * (omt * omt));
            float lad = (__builtin_amdgcn_logf(dnum) - 2.0f * __builtin_amdgcn_logf(den)) * kLN2;
            lad = INV ? -lad : lad;
            const bool inside = (x >= c.lo) && (x <= c.hi);
            const bool live = 8 * ch + 2 * q + h < a.n_up && row_ok[u];
            zout[u][h] = inside ? out : x;
            ldsum[u] += (inside && live) ? lad : 0.0f;  // coordinate order: h = 0 first, as the other forms
            any_in |= inside && live;
            any_nd |= nd && inside && live;
        };
        for (int ch = 0; ch < a.NCH; ++ch) {
            const int g = ch >> 1;
            if (ch == 0) {
                wide_phase<KBH, K, INV, NTC, NU>(a, s, SC, KBH, bh, bl, accA, ones, slot0, slot1, wid, lane, tr,
                                                 [&](int J, int part) {
                                                     pieces(J, part, [&](int u, int, bool f) {
                                                         if (f) read_xv(0, u);
                                                     });
                                                 });
            } else {
                wide_phase<KBH, K, INV, NTC, NU>(a, s, SC, KBH, bh, bl, accA, ones, slot0, slot1, wid, lane, tr,
                                                 [&](int J, int part) {
                                                     pieces(J, part, [&](int u, int h, bool f) {
                                                         epi_c(ch - 1, u, h, f);
                                                         if (f) read_xv(ch, u);
                                                     });
                                                 });
                if (!(ch & 1)) {
                    // pair g - 1 complete: its z out, pair g's x into the tile
                    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#pragma unroll
                    for (int u = 0; u < NU; ++u)
                        wide_store(a, m_lo_out, m_up_out, b0[u], nrows[u], g - 1, tiles + u * kWideTile, lane);
                    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#pragma unroll
                    for (int u = 0; u < NU; ++u)
                        wide_gather(a, m_lo_in, m_up_in, b0[u], g, tiles + u * kWideTile, lane);
                }
            }
            wide_phase<KBH, K, INV, NTC, NU>(a, s, SC, KBH, bh, bl, accB, ones, slot0, slot1, wid, lane, tr,
                                             [&](int J, int part) { pieces(J, part, [&](int u, int h, bool f) { epi_a(u, h, f); }); });
            if ((ch & 1) && ch + 1 < a.NCH) {
                // xbuf's last reader (the searched epilogue of ch) is done: pair g + 1's upper x
#pragma unroll
                for (int u = 0; u < NU; ++u) wide_gather_up(a, m_up_in, b0[u], g + 1, xbuf + u * 256, lane);
            }
            wide_phase<KBH, K, INV, NTC, NU>(a, s, SC, KBH, bh, bl, accC, ones, slot0, slot1, wid, lane, tr,
                                             [&](int J, int part) { pieces(J, part, [&](int u, int h, bool f) { epi_b(u, h, f); }); });
        }
        // the last chunk's derivative epilogue, then the last pair's z
#pragma unroll
        for (int u = 0; u < NU; ++u) {
            epi_c(a.NCH - 1, u, 0, false);
            epi_c(a.NCH - 1, u, 1, false);
            epi_c(a.NCH - 1, u, 0, true);
        }
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#pragma unroll
        for (int u = 0; u < NU; ++u)
            wide_store(a, m_lo_out, m_up_out, b0[u], nrows[u], (a.NCH - 1) >> 1, tiles + u * kWideTile, lane);
    } else
    for (int ch = 0; ch < a.NCH; ++ch) {
        const int g = ch >> 1;
        // this lane group's coordinates 8 ch + 2 q + h; tile column of upper coordinate
        const int tcol = 2 * (8 * (ch & 1) + 2 * q) + 1;
        int jj[2];
#pragma unroll
        for (int h = 0; h < 2; ++h) jj[h] = 8 * ch + 2 * q + h;
        float xv[NU][2];
        int kb[NU][2];
        float cw_k[NU][2], w_k[NU][2], ch_k[NU][2], h_k[NU][2];

        // ---- searched knots (widths forward / heights inverse)
        {
            f32x4 acc[NU][NTC];
            wide_phase<KBH, K, INV, NTC, NU>(a, s, SC, KBH, bh, bl, acc, ones, slot0, slot1, wid, lane, tr);
#pragma unroll
            for (int u = 0; u < NU; ++u) {
                const float4 v = *reinterpret_cast<const float4*>(tiles + u * kWideTile + sl * 32 + tcol - 1);
                xv[u][0] = jj[0] < a.n_up ? v.y : 0.0f;
                xv[u][1] = jj[1] < a.n_up ? v.w : 0.0f;
                knot_phase_w<K, true>(acc[u], xv[u], c, l2e3, kb[u], INV ? ch_k[u] : cw_k[u], INV ? h_k[u] : w_k[u]);
                wide_pin(kb[u], INV ? ch_k[u] : cw_k[u], INV ? h_k[u] : w_k[u]);
            }
            NFK_MARK(tr);  // epilogue A
        }
        // ---- the other knots, selected at the bin
        {
            f32x4 acc[NU][NTC];
            wide_phase<KBH, K, INV, NTC, NU>(a, s, SC, KBH, bh, bl, acc, ones, slot0, slot1, wid, lane, tr);
#pragma unroll
            for (int u = 0; u < NU; ++u) {
                knot_phase_w<K, false>(acc[u], xv[u], c, l2e3, kb[u], INV ? cw_k[u] : ch_k[u], INV ? w_k[u] : h_k[u]);
                wide_pin(kb[u], INV ? cw_k[u] : ch_k[u], INV ? w_k[u] : h_k[u]);
            }
            NFK_MARK(tr);  // epilogue B
        }
        // ---- derivatives of the bin, evaluate, log|det|
        {
            f32x4 accd[NU][NTC];
            wide_phase<KBH, K, INV, NTC, NU>(a, s, SC, KBH, bh, bl, accd, ones, slot0, slot1, wid, lane, tr);
#pragma unroll
            for (int u = 0; u < NU; ++u) {
                float outv[2];
#ifdef NFK_WABL_NOEPI
#pragma unroll
                for (int h = 0; h < 2; ++h) {
                    float v = cw_k[u][h] + w_k[u][h] + ch_k[u][h] + h_k[u][h];
#pragma unroll
                    for (int t = 0; t < NTC; ++t) v += accd[u][t][2 * h] + accd[u][t][2 * h + 1];
                    outv[h] = v;
                    ldsum[u] += v;
                    any_in = true;
                }
                if (false)
#endif
#pragma unroll
                for (int h = 0; h < 2; ++h) {
                    // derivative logit j in register 2h + (j & 1) of tile j >> 1;
                    // padded index j+1 holds logit j (utils.py:36-39): raw_k = logit k-1, raw_k1 = logit k
                    const int k = kb[u][h];
                    float raw_k = accd[u][0][2 * h], raw_k1 = accd[u][0][2 * h];
#pragma unroll
                    for (int j = 1; j < K - 1; ++j) {
                        const float v = accd[u][j >> 1][2 * h + (j & 1)];
                        raw_k = (k >= j + 1) ? v : raw_k;
                        raw_k1 = (k >= j) ? v : raw_k1;
                    }
                    const float d_k = (k == 0) ? c.d_edge : nfk_deriv_lean(raw_k * un3, c.min_d);
                    const float d_k1 = (k == K - 1) ? c.d_edge : nfk_deriv_lean(raw_k1 * un3, c.min_d);
                    const float x = xv[u][h];
                    const float wk = w_k[u][h], hk = h_k[u][h], cwk = cw_k[u][h], chk = ch_k[u][h];
                    const float rw = nfk_rcp_fast(wk);
                    const float delta = hk * rw;
                    const float gap = (d_k + d_k1) - 2.0f * delta;
                    float out, th;
                    bool nd = false;
                    if (INV) {
                        const float y = x - chk;
                        const float qa = y * gap + hk * (delta - d_k);
                        const float qb = hk * d_k - y * gap;
                        const float qc = (-delta) * y;
                        const float disc = qb * qb - (4.0f * qa) * qc;
                        nd = !(disc >= 0.0f);
                        const float root = nfk_div<true>(2.0f * qc, -qb - sqrtf(disc));
                        out = root * wk + cwk;
                        th = root;
                    } else {
                        th = (x - cwk) * rw;
                    }
                    const float t1mt = th * (1.0f - th);
                    const float den = delta + gap * t1mt;
                    if (!INV) {
                        const float num = hk * (delta * (th * th) + d_k * t1mt);
                        out = chk + nfk_div<true>(num, den);
                    }
                    const float omt = 1.0f - th;
                    const float dnum =
                        (delta * delta) * ((d_k1 * (th * th) + (2.0f * delta) * t1mt) + d_k * (omt * omt));
                    float lad = (__builtin_amdgcn_logf(dnum) - 2.0f * __builtin_amdgcn_logf(den)) * kLN2;
                    lad = INV ? -lad : lad;
                    const bool inside = (x >= c.lo) && (x <= c.hi);
                    const bool live = jj[h] < a.n_up && row_ok[u];
                    outv[h] = inside ? out : x;
                    ldsum[u] += (inside && live) ? lad : 0.0f;
                    any_in |= inside && live;
                    any_nd |= nd && inside && live;
                }
                float* tw = tiles + u * kWideTile + sl * 32 + tcol;
                tw[0] = outv[0];  // z back into the upper columns
                tw[2] = outv[1];
            }
            NFK_MARK(tr);  // epilogue C
        }
        // after a chunk pair: its z, then the next pair's x into the same tile
        // (the stores' data left the tile before the copy is issued)
        if ((ch & 1) || ch + 1 == a.NCH) {
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#pragma unroll
            for (int u = 0; u < NU; ++u)
                wide_store(a, m_lo_out, m_up_out, b0[u], nrows[u], g, tiles + u * kWideTile, lane);
            if (ch + 1 < a.NCH) {
                asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#pragma unroll
                for (int u = 0; u < NU; ++u)
                    wide_gather(a, m_lo_in, m_up_in, b0[u], g + 1, tiles + u * kWideTile, lane);
            }
        }
    }

#pragma unroll
    for (int u = 0; u < NU; ++u) {
        float v = ldsum[u];
        v += __shfl_xor(v, 16, 64);
        v += __shfl_xor(v, 32, 64);
        if (q == 0 && row_ok[u] && a.mode != 0) {
            float* dst = a.logdet + b0[u] + sl;
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

// form: 1 = one sample tile per wave (kWideWaves-wave workgroups), 2 = two
template <int KBH, int K>
int launch_fused_wide(const WideArgs& a, size_t lds, bool inv, int form, hipStream_t st) {
    const int nw = form == 2 ? wide_nw<2>() : wide_nw<1>();
    const int64_t per_block = (int64_t)nw * 16 * (form == 2 ? 2 : 1);
    const int64_t blocks = (a.batch + per_block - 1) / per_block;
    if (blocks == 0) return 0;
    const dim3 grid((unsigned)blocks), block(64 * nw);
    if (form == 2) {
        if (inv)
            hipLaunchKernelGGL((k_fused_nsf_wide<KBH, K, true, 2>), grid, block, lds, st, a);
        else
            hipLaunchKernelGGL((k_fused_nsf_wide<KBH, K, false, 2>), grid, block, lds, st, a);
    } else {
        if (inv)
            hipLaunchKernelGGL((k_fused_nsf_wide<KBH, K, true, 1>), grid, block, lds, st, a);
        else
            hipLaunchKernelGGL((k_fused_nsf_wide<KBH, K, false, 1>), grid, block, lds, st, a);
    }
    hipError_t e = hipGetLastError();
    return e == hipSuccess ? 0 : (int)e;
}

#define NFK_WIDE_INSTANCE(KBH, K) \
    template int launch_fused_wide<KBH, K>(const WideArgs& a, size_t lds, bool inv, int form, hipStream_t st);
#define NFK_WIDE_EXTERN(KBH, K) \
    extern template int launch_fused_wide<KBH, K>(const WideArgs& a, size_t lds, bool inv, int form, hipStream_t st);

// hidden widths H = 32 KBH (no f32 tail), bins K
#define NFK_WIDE_KB(X) X(4) X(8)
#define NFK_WIDE_K(X, KBH) X(KBH, 8) X(KBH, 16)

}  // namespace nfk_fused
